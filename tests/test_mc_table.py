"""The generated marching-cubes table (disinfect-slam_amd/csrc/tsdf_mc_tables.h) equals the one the
oracle derives on its own (oracle/ora_mc_cases.c), and yields closed,
consistently oriented surfaces: on random scalar fields whose border is outside, every mesh edge
(a pair of grid-edge vertices) is shared by exactly two triangles with opposite directions, and
on a sphere every normal points outward. This is what "crack free" means for the table the
oracle and the HIP kernel both use (KrisLibrary's own table is not available: parity unpinned)."""
import os
import re

import numpy as np
import pytest

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "disinfect-slam_amd",
                   "csrc", "tsdf_mc_tables.h")


def load_table():
    txt = open(HDR).read().replace("\\\n", "")
    get = lambda name: eval(re.search(rf"#define {name} (.*)", txt).group(1).replace("{", "[").replace("}", "]"))
    return get("TSDF_MC_EDGE_INIT"), get("TSDF_MC_NUM_TRI_INIT"), get("TSDF_MC_TRI_INIT")


EDGE, NTRI, TRI = load_table()
CORNER = [((i >> 0) & 1, (i >> 1) & 1, (i >> 2) & 1) for i in range(8)]


def mesh(field):
    """Triangles as triples of global edge ids ((x, y, z) of the lower corner, axis)."""
    n = field.shape
    tris = []
    for x in range(n[0] - 1):
        for y in range(n[1] - 1):
            for z in range(n[2] - 1):
                cube = 0
                for i, (dx, dy, dz) in enumerate(CORNER):
                    if field[x + dx, y + dy, z + dz] < 0:
                        cube |= 1 << i
                for t in range(NTRI[cube]):
                    tri = []
                    for k in TRI[cube][3 * t:3 * t + 3]:
                        a, b = EDGE[k]
                        ca, cb = CORNER[a], CORNER[b]
                        axis = [i for i in range(3) if ca[i] != cb[i]][0]
                        lo = tuple(int(v) for v in np.minimum(ca, cb))
                        tri.append(((x + lo[0], y + lo[1], z + lo[2]), axis))
                    tris.append(tri)
    return tris


def check_closed(tris):
    directed = {}
    for t in tris:
        for i in range(3):
            e = (t[i], t[(i + 1) % 3])
            directed[e] = directed.get(e, 0) + 1
    for (a, b), c in directed.items():
        assert c == 1, "directed edge used twice (orientation flip)"
        assert directed.get((b, a), 0) == 1, "boundary edge: mesh not closed"


@pytest.mark.parametrize("seed", range(6))
def test_random_fields_are_closed_and_oriented(seed):
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((9, 9, 9))
    f[0, :, :] = f[-1, :, :] = f[:, 0, :] = f[:, -1, :] = f[:, :, 0] = f[:, :, -1] = 1.0
    tris = mesh(f)
    assert len(tris) > 50
    check_closed(tris)


def test_sphere_normals_point_outward():
    g = np.arange(12) - 5.5
    X, Y, Z = np.meshgrid(g, g, g, indexing="ij")
    f = np.sqrt(X ** 2 + Y ** 2 + Z ** 2) - 4.2
    tris = mesh(f)
    check_closed(tris)
    for t in tris:
        p = [np.array(v[0], float) + 0.5 * np.eye(3)[v[1]] - 5.5 for v in t]
        n = np.cross(p[1] - p[0], p[2] - p[0])
        assert np.dot(n, (p[0] + p[1] + p[2]) / 3) > 0


def test_every_case_uses_exactly_its_crossing_edges():
    for c in range(256):
        used = {k for k in TRI[c][:3 * NTRI[c]]}
        cross = {k for k, (a, b) in enumerate(EDGE) if ((c >> a) & 1) != ((c >> b) & 1)}
        assert used == cross
        assert all(k == -1 for k in TRI[c][3 * NTRI[c]:])


def test_oracle_derives_the_same_table():
    """The oracle's case table (oracle/ora_mc_cases.c, derived from the cube's geometry in C) and
    the product's (csrc/tsdf_mc_tables.h, scripts/gen_mc_tables.py in Python) are equal entry for
    entry: the oracle no longer includes the product's table, so a wrong entry in either shows up
    here and in the GPU-vs-oracle mesh parity."""
    import ctypes as C

    from _oracle import LIB_PATH as ORACLE_LIB
    L = C.CDLL(ORACLE_LIB)
    e = np.zeros(24, np.int8)
    n = np.zeros(256, np.uint8)
    t = np.zeros(256 * 15, np.int8)
    assert L.ora_mc_table(e.ctypes.data_as(C.c_void_p), n.ctypes.data_as(C.c_void_p),
                          t.ctypes.data_as(C.c_void_p)) == 5
    np.testing.assert_array_equal(e.reshape(12, 2), np.asarray(EDGE))
    np.testing.assert_array_equal(n, np.asarray(NTRI))
    np.testing.assert_array_equal(t.reshape(256, 15), np.asarray(TRI))
