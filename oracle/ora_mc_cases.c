/* ora_mc_cases.c -- TEST INFRASTRUCTURE (part of the CPU oracle, liboracle_tsdf.so): the
 * marching-cubes case table, derived here from the cube's geometry instead of being included from
 * the product (disinfect-slam_amd/csrc/tsdf_mc_tables.h, made by scripts/gen_mc_tables.py).
 * tests/test_mc_table.py checks that the two tables are equal entry for entry, so a wrong entry in
 * either shows up as a mismatch.
 *
 * The reference meshes with KrisLibrary's SparseTSDFReconstruction (examples/ros_camera_driver/
 * ros_offline.cc:279-287), whose table is not vendored: the case table is defined by these rules
 * (parity against KrisLibrary unpinned):
 *  - corner i at (i & 1, i >> 1 & 1, i >> 2 & 1), inside when its value is < 0; edges numbered
 *    x edges (0,1) (2,3) (4,5) (6,7), y edges (0,2) (1,3) (4,6) (5,7), z edges (0,4) (1,5) (2,6) (3,7);
 *  - on each face, walking its corners counter-clockwise seen from outside, every run of inside
 *    corners contributes one iso-segment from the edge that ends the run to the edge that starts it
 *    (the diagonal pattern separates the inside corners); the segments chain into loops, listed by
 *    their smallest edge, each starting there;
 *  - each loop is triangulated by the candidate (all triangulations of the polygon, enumerated by
 *    the triangle on the edge first-last, apex ascending) whose worst triangle is best oriented:
 *    score = n . (centroid - mean of the triangle's inside edge endpoints) / |n|, compared exactly;
 *    the first candidate wins exact ties; triangles are oriented so normals point to the outside
 *    (>= 0) corners. */
#include <stdint.h>
#include <string.h>

#define MC_MAX_TRI 5
#define MC_MAX_LOOP 12
#define MC_MAX_CAND 512

static const int kCornerEdges[12][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3},
                                        {4, 6}, {5, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};

static int edge_of(int a, int b) {
  for (int k = 0; k < 12; ++k)
    if ((kCornerEdges[k][0] == a && kCornerEdges[k][1] == b) || (kCornerEdges[k][0] == b && kCornerEdges[k][1] == a))
      return k;
  return -1;
}

/* corner index of the point with coordinate `side` on axis a and (u, v) on axes a+1, a+2 */
static int corner_at(int a, int side, int u, int v) {
  int c[3];
  c[a] = side;
  c[(a + 1) % 3] = u;
  c[(a + 2) % 3] = v;
  return c[0] | c[1] << 1 | c[2] << 2;
}

/* the 6 faces, corners counter-clockwise seen from outside: on the +a face (normal +e_a) the
 * (e_{a+1}, e_{a+2}) plane is seen as is; the -a face is seen mirrored, so its cycle reverses */
static void face_cycles(int faces[6][4]) {
  static const int uv[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
  for (int a = 0; a < 3; ++a)
    for (int side = 0; side < 2; ++side)
      for (int k = 0; k < 4; ++k) {
        const int j = side ? k : 3 - k;
        faces[2 * a + side][k] = corner_at(a, side, uv[j][0], uv[j][1]);
      }
}

/* loops of case c: returns their count; lens[i] edges of loop i in loops[i] */
static int case_loops(int c, int loops[4][MC_MAX_LOOP], int lens[4]) {
  int faces[6][4];
  face_cycles(faces);
  int next[12];
  for (int k = 0; k < 12; ++k) next[k] = -1;
  for (int f = 0; f < 6; ++f) {
    const int* cy = faces[f];
    for (int k = 0; k < 4; ++k) {
      const int ck = cy[k], cn = cy[(k + 1) & 3];
      if (!((c >> ck) & 1) || ((c >> cn) & 1)) continue; /* not the last corner of an inside run */
      int j = k;
      while ((c >> cy[(j + 3) & 3]) & 1) j = (j + 3) & 3; /* back to the run's first corner */
      const int entry = edge_of(cy[(j + 3) & 3], cy[j]);
      const int exit_ = edge_of(ck, cn);
      next[exit_] = entry;
    }
  }
  int seen[12] = {0}, n = 0;
  for (int s = 0; s < 12; ++s) {
    if (next[s] < 0 || seen[s]) continue;
    int len = 0, e = s;
    while (!seen[e]) {
      seen[e] = 1;
      loops[n][len++] = e;
      e = next[e];
    }
    lens[n++] = len;
  }
  return n;
}

/* all triangulations of poly[0..m), in the enumeration order of the rules above; each candidate
 * is m - 2 triangles (vertex triples) appended to out; returns the number of candidates */
typedef struct {
  int tri[MC_MAX_LOOP][3];
} cand_t;

static int triangulate(const int* poly, int m, cand_t* out, int cap) {
  if (m < 3) {
    if (cap < 1) return 0;
    return 1; /* one empty triangulation */
  }
  int n = 0;
  for (int k = 1; k <= m - 2; ++k) {
    cand_t left[MC_MAX_CAND / 8], right[MC_MAX_CAND / 8];
    const int nl = triangulate(poly, k + 1, left, MC_MAX_CAND / 8);
    const int nr = triangulate(poly + k, m - k, right, MC_MAX_CAND / 8);
    const int tl = k + 1 - 2 > 0 ? k + 1 - 2 : 0, tr = m - k - 2 > 0 ? m - k - 2 : 0;
    for (int a = 0; a < nl; ++a)
      for (int b = 0; b < nr; ++b) {
        if (n >= cap) return n;
        cand_t* o = &out[n++];
        int t = 0;
        for (int i = 0; i < tl; ++i, ++t) memcpy(o->tri[t], left[a].tri[i], sizeof(o->tri[t]));
        o->tri[t][0] = poly[0];
        o->tri[t][1] = poly[k];
        o->tri[t][2] = poly[m - 1];
        ++t;
        for (int i = 0; i < tr; ++i, ++t) memcpy(o->tri[t], right[b].tri[i], sizeof(o->tri[t]));
      }
  }
  return n;
}

/* doubled integer coordinates: corner i -> 2 * (its coordinates); edge midpoint -> sum of corners */
static void corner2(int i, int p[3]) {
  p[0] = 2 * (i & 1);
  p[1] = 2 * ((i >> 1) & 1);
  p[2] = 2 * ((i >> 2) & 1);
}
static void mid2(int e, int p[3]) {
  int a[3], b[3];
  corner2(kCornerEdges[e][0], a);
  corner2(kCornerEdges[e][1], b);
  for (int j = 0; j < 3; ++j) p[j] = (a[j] + b[j]) / 2;
}

typedef struct {
  int64_t n, d, q; /* score = n / (d sqrt(q)); q == 0 reads as 0 */
} score_t;

static score_t tri_score(int c, const int t[3]) {
  int a[3], b[3], d[3];
  mid2(t[0], a);
  mid2(t[1], b);
  mid2(t[2], d);
  const int64_t u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, v[3] = {d[0] - a[0], d[1] - a[1], d[2] - a[2]};
  const int64_t nrm[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
  int64_t sum_in[3] = {0, 0, 0}, k = 0;
  for (int i = 0; i < 3; ++i)
    for (int s = 0; s < 2; ++s) {
      const int corner = kCornerEdges[t[i]][s];
      if ((c >> corner) & 1) {
        int p[3];
        corner2(corner, p);
        for (int j = 0; j < 3; ++j) sum_in[j] += p[j];
        ++k;
      }
    }
  score_t r;
  r.n = 0;
  for (int j = 0; j < 3; ++j) r.n += nrm[j] * (k * (a[j] + b[j] + d[j]) - 3 * sum_in[j]);
  r.d = 3 * k;
  r.q = nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2];
  if (r.q == 0) {
    r.n = 0;
    r.d = 1;
    r.q = 1;
  }
  return r;
}

static int score_less(score_t s, score_t t) {
  const int64_t A = s.n * t.d, B = t.n * s.d; /* compare A sqrt(t.q) with B sqrt(s.q) */
  if ((A >= 0) != (B >= 0)) return A < 0;
  if (A >= 0) return A * A * t.q < B * B * s.q;
  return A * A * t.q > B * B * s.q;
}

static int8_t g_tri[256][3 * MC_MAX_TRI];
static uint8_t g_ntri[256];
static int g_built = 0;

static void build(void) {
  /* orientation: case 1 (corner 0 inside), plain fan of its loop; flip when its normal does not
   * point away from corner 0 */
  int loops[4][MC_MAX_LOOP], lens[4];
  (void)case_loops(1, loops, lens);
  int flip;
  {
    int a[3], b[3], d[3];
    mid2(loops[0][0], a);
    mid2(loops[0][1], b);
    mid2(loops[0][2], d);
    const int u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, v[3] = {d[0] - a[0], d[1] - a[1], d[2] - a[2]};
    const int n[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
    int cen = 0; /* n . (3 * centroid - 3 * corner0), corner 0 at the origin */
    for (int j = 0; j < 3; ++j) cen += n[j] * (a[j] + b[j] + d[j]);
    flip = !(cen > 0);
  }
  static cand_t cands[MC_MAX_CAND];
  for (int c = 0; c < 256; ++c) {
    const int nl = case_loops(c, loops, lens);
    int nt = 0;
    memset(g_tri[c], -1, sizeof(g_tri[c]));
    for (int l = 0; l < nl; ++l) {
      const int m = lens[l];
      const int nc = triangulate(loops[l], m, cands, MC_MAX_CAND);
      int best = -1;
      score_t best_s = {0, 1, 1};
      for (int i = 0; i < nc; ++i) {
        if (flip)
          for (int t = 0; t < m - 2; ++t) {
            const int x = cands[i].tri[t][1];
            cands[i].tri[t][1] = cands[i].tri[t][2];
            cands[i].tri[t][2] = x;
          }
        score_t mn = tri_score(c, cands[i].tri[0]);
        for (int t = 1; t < m - 2; ++t) {
          const score_t s = tri_score(c, cands[i].tri[t]);
          if (score_less(s, mn)) mn = s;
        }
        if (best < 0 || score_less(best_s, mn)) {
          best = i;
          best_s = mn;
        }
      }
      for (int t = 0; t < m - 2 && nt < MC_MAX_TRI; ++t, ++nt)
        for (int j = 0; j < 3; ++j) g_tri[c][3 * nt + j] = (int8_t)cands[best].tri[t][j];
    }
    g_ntri[c] = (uint8_t)nt;
  }
  g_built = 1;
}

/* the oracle's table (built on first use) */
const int8_t* ora_mc_tri(void) {
  if (!g_built) build();
  return &g_tri[0][0];
}
const uint8_t* ora_mc_ntri(void) {
  if (!g_built) build();
  return g_ntri;
}
int ora_mc_edge(int e, int s) { return kCornerEdges[e][s]; }

/* exported for tests/test_mc_table.py: edges 12 x 2, triangle counts 256, triangles 256 x 15 */
int ora_mc_table(int8_t* edges, uint8_t* ntri, int8_t* tri) {
  if (!g_built) build();
  for (int e = 0; e < 12; ++e) {
    edges[2 * e] = (int8_t)kCornerEdges[e][0];
    edges[2 * e + 1] = (int8_t)kCornerEdges[e][1];
  }
  memcpy(ntri, g_ntri, sizeof(g_ntri));
  memcpy(tri, g_tri, sizeof(g_tri));
  return MC_MAX_TRI;
}
