#!/usr/bin/env python3
"""Generate the marching-cubes case table (disinfect-slam_amd/csrc/tsdf_mc_tables.h).

The reference meshes with KrisLibrary's SparseTSDFReconstruction::ExtractMesh
(examples/ros_camera_driver/ros_offline.cc:279-287), which is not vendored and not in this image,
so its exact table cannot be reproduced (parity unpinned). This generator derives a
crack-free table from first principles instead of transcribing one:

  corner i of a cube sits at (i & 1, i >> 1 & 1, i >> 2 & 1); edge k joins the two corners in
  EDGES[k]. A corner is INSIDE when its value is < 0 (iso level 0, the TSDF zero crossing).
  On every face, the iso-line segments join crossing edges; the one ambiguous face pattern
  (diagonal corners inside) always separates the inside corners. The decision depends on the
  face's 4 corners only, so two cubes sharing a face agree and the mesh has no cracks.
  Segments are oriented "exit -> entry" while walking each face counter-clockwise as seen from
  outside the cube, which chains them into consistently oriented loops; each loop is fanned
  into triangles, and the whole table is flipped once so triangle normals (right-hand rule)
  point from inside (< 0) to outside (>= 0), i.e. toward free space.

Usage: python3 scripts/gen_mc_tables.py  (rewrites the header; the output is committed)
"""
import itertools
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "disinfect-slam_amd", "csrc", "tsdf_mc_tables.h")

P = np.array([[(i >> 0) & 1, (i >> 1) & 1, (i >> 2) & 1] for i in range(8)], float)
EDGES = [(0, 1), (2, 3), (4, 5), (6, 7),   # x edges
         (0, 2), (1, 3), (4, 6), (5, 7),   # y edges
         (0, 4), (1, 5), (2, 6), (3, 7)]   # z edges
EDGE_OF = {frozenset(e): k for k, e in enumerate(EDGES)}


def faces():
    out = []
    for axis in range(3):
        for side in (0, 1):
            cs = [i for i in range(8) if ((i >> axis) & 1) == side]
            n = np.zeros(3)
            n[axis] = 1 if side else -1
            c = P[cs].mean(0)
            # order the 4 corners counter-clockwise seen from outside (looking along -n)
            u = np.zeros(3); u[(axis + 1) % 3] = 1
            v = np.cross(n, u)
            ang = [np.arctan2(np.dot(P[i] - c, v), np.dot(P[i] - c, u)) for i in cs]
            cyc = [cs[k] for k in np.argsort(ang)]
            a, b, d = P[cyc[0]], P[cyc[1]], P[cyc[2]]
            assert np.dot(np.cross(b - a, d - b), n) > 0
            out.append(cyc)
    return out


FACES = faces()


def loops_for(case):
    inside = [(case >> i) & 1 for i in range(8)]
    nxt = {}
    for cyc in FACES:
        for k in range(4):
            c = cyc[k]
            if not inside[c]:
                continue
            # inside corner c: its entry edge (from the previous corner) and its exit edge
            # (to the next corner); walking CCW, an inside run ends at an exit edge and the
            # iso-line goes from that exit back to the entry edge that started the run
            # (for the diagonal pattern each run is a single corner: inside corners separated)
            if inside[cyc[(k + 1) % 4]]:
                continue  # not the end of the run
            j = k
            while inside[cyc[(j - 1) % 4]]:
                j -= 1
            entry = EDGE_OF[frozenset((cyc[(j - 1) % 4], cyc[j % 4]))]
            exit_ = EDGE_OF[frozenset((c, cyc[(k + 1) % 4]))]
            assert exit_ not in nxt
            nxt[exit_] = entry
    loops, seen = [], set()
    for s in sorted(nxt):
        if s in seen:
            continue
        loop, e = [], s
        while e not in seen:
            seen.add(e)
            loop.append(e)
            e = nxt[e]
        assert e == s
        loops.append(loop)
    return loops


def edge_mid(k):
    a, b = EDGES[k]
    return (P[a] + P[b]) / 2


P2 = [tuple(2 * int(v) for v in P[i]) for i in range(8)]  # corners in doubled integer coordinates


def edge_mid2(k):
    a, b = EDGES[k]
    return tuple(P2[a][j] // 2 + P2[b][j] // 2 for j in range(3))


def sub(u, v):
    return tuple(u[j] - v[j] for j in range(3))


def cross(u, v):
    return (u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0])


def triangulations(poly):
    """All triangulations of a polygon (vertex list, boundary order kept), recursive on the
    triangle that contains the edge poly[0]-poly[-1]."""
    if len(poly) < 3:
        return [[]]
    out = []
    a, b = poly[0], poly[-1]
    for k in range(1, len(poly) - 1):
        for left in triangulations(poly[:k + 1]):
            for right in triangulations(poly[k:]):
                out.append(left + [(a, poly[k], b)] + right)
    return out


def tri_score(case, t):
    """How well triangle t (edge indices) faces away from the inside endpoints of its edges: the
    cosine-like n . (centroid - mean of the inside corners) / |n|, kept exact as (N, D, Q) with
    score = N / (D sqrt(Q)) in doubled integer coordinates (edge midpoints are on the half grid)."""
    a, b, d = (edge_mid2(k) for k in t)
    n = cross(sub(b, a), sub(d, a))
    ins = [P2[i] for k in t for i in EDGES[k] if (case >> i) & 1]
    k = len(ins)
    c = [k * (a[j] + b[j] + d[j]) - 3 * sum(p[j] for p in ins) for j in range(3)]
    return (sum(n[j] * c[j] for j in range(3)), 3 * k, sum(v * v for v in n))


def score_less(s, t):
    """s < t for exact scores (N, D, Q): N1 / (D1 sqrt Q1) < N2 / (D2 sqrt Q2); Q = 0 reads 0."""
    (n1, d1, q1), (n2, d2, q2) = s, t
    if q1 == 0:
        n1, d1, q1 = 0, 1, 1
    if q2 == 0:
        n2, d2, q2 = 0, 1, 1
    A, B = n1 * d2, n2 * d1            # compare A sqrt(q2) with B sqrt(q1)
    if (A >= 0) != (B >= 0):
        return A < 0
    if A >= 0:
        return A * A * q2 < B * B * q1
    return A * A * q2 > B * B * q1


def min_score(case, ts):
    m = None
    for t in ts:
        v = tri_score(case, t)
        if m is None or score_less(v, m):
            m = v
    return m


def tris_for(case, flip):
    tris = []
    for loop in loops_for(case):
        cands = []
        for tri_set in triangulations(loop):
            ts = [((t[0], t[2], t[1]) if flip else t) for t in tri_set]
            cands.append(ts)
        if flip is None:  # orientation probe: plain fan
            tris += [(loop[0], loop[i], loop[i + 1]) for i in range(1, len(loop) - 1)]
            continue
        # the triangulation whose worst triangle is best oriented (the first one on exact ties)
        best, best_s = None, None
        for ts in cands:
            m = min_score(case, ts)
            if best is None or score_less(best_s, m):
                best, best_s = ts, m
        tris += best
    return tris


def orientation_sign():
    # single inside corner 0: the outward (toward >= 0) normal points away from corner 0
    t = tris_for(1, None)[0]
    a, b, c = (edge_mid(k) for k in t)
    n = np.cross(b - a, c - a)
    return np.dot(n, (a + b + c) / 3 - P[0]) > 0


def main():
    flip = not orientation_sign()
    table = [tris_for(c, flip) for c in range(256)]
    # sanity: every crossing edge is used, every case's loops are closed, complement symmetry
    for c in range(256):
        used = {k for t in table[c] for k in t}
        cross = {k for k, (a, b) in enumerate(EDGES) if ((c >> a) & 1) != ((c >> b) & 1)}
        assert used == cross, c
        for t in table[c]:  # normal points away from the inside endpoints of its 3 edges
            a, b, d = (edge_mid(k) for k in t)
            n = np.cross(b - a, d - a)
            ins = [P[i] for k in t for i in EDGES[k] if (c >> i) & 1]
            assert np.dot(n, (a + b + d) / 3 - np.mean(ins, 0)) > 0, (c, t)
    maxt = max(len(t) for t in table)
    lines = [
        "// tsdf_mc_tables.h -- GENERATED by scripts/gen_mc_tables.py (do not edit).",
        "// Marching-cubes case table: corner i at (i&1, i>>1&1, i>>2&1); a corner is inside when its",
        "// value is < 0. Edge k joins corners TSDF_MC_EDGE_INIT[k]; case c has TSDF_MC_NUM_TRI_INIT[c]",
        "// triangles, TSDF_MC_TRI_INIT[c] lists them as edge-index triples (-1 padded), normals",
        "// toward the outside (>= 0) corners. Initialisers, so C (oracle) and HIP (__constant__)",
        "// instantiate the same data.",
        "#pragma once",
        f"#define TSDF_MC_MAX_TRI {maxt}",
        "#define TSDF_MC_EDGE_INIT {" + ", ".join(f"{{{a}, {b}}}" for a, b in EDGES) + "}",
        "#define TSDF_MC_NUM_TRI_INIT {" + ", ".join(str(len(t)) for t in table) + "}",
        "#define TSDF_MC_TRI_INIT { \\",
    ]
    for c, t in enumerate(table):
        flat = [k for tri in t for k in tri] + [-1] * (3 * maxt - 3 * len(t))
        lines.append("    {" + ", ".join(map(str, flat)) + "}, \\")
    lines.append("}")
    open(OUT, "w").write("\n".join(lines) + "\n")
    print("wrote", OUT, "max triangles per case", maxt,
          "total", sum(len(t) for t in table))


if __name__ == "__main__":
    main()
