"""The HIP engine against the committed golden stream (tests/golden/integrate_48x36.npz): no oracle
call at run time -- entries, pool indices, free stack, tsdf / rgbw bit-exact, probability within
1e-4, raycast alpha exact and colours within 1 LSB, Query positions / tsdf exact."""
import numpy as np
import pytest

from test_golden import load_stream

pytestmark = pytest.mark.gpu


def test_engine_reproduces_golden_stream():
    import tsdf_amd
    G = load_stream()
    W, H = int(G["W"]), int(G["H"])
    eng = tsdf_amd.Engine(float(G["voxel"]), float(G["trunc"]), max_width=W, max_height=H,
                          num_block_bits=int(G["num_block_bits"]))
    try:
        for f in range(G["depth"].shape[0]):
            eng.integrate(G["rgb"][f], G["depth"][f], G["ht"][f], G["lt"][f], G["K"],
                          tsdf_amd.SE3(G["q"][f], G["t"][f]), float(G["max_depth"]))
            s = eng.stats()
            assert s["status"] == 0
            assert [s["last_num_visible"], s["last_num_updated"], s["last_num_deleted"],
                    s["active_blocks"]] == G["stats"][f].tolist(), f
        d = eng.dump()
        live = np.flatnonzero(d["entry_idx"] >= 0)
        np.testing.assert_array_equal(live, G["live_entry"])
        np.testing.assert_array_equal(d["entry_pos"][live], G["live_pos"])
        idx = d["entry_idx"][live]
        np.testing.assert_array_equal(idx, G["live_idx"])
        np.testing.assert_array_equal(d["heap"], G["heap"])
        assert d["free"] == int(G["free"])
        blk = lambda a: a.reshape(-1, 512, *a.shape[1:])[idx]
        np.testing.assert_array_equal(blk(d["tsdf"]).view(np.uint32), G["tsdf"].view(np.uint32))
        np.testing.assert_array_equal(blk(d["rgbw"]), G["rgbw"])
        assert np.abs(blk(d["prob"]) - G["prob"]).max() <= 1e-4
        rgba, normal = eng.raycast(G["K"], W, H, tsdf_amd.SE3(G["q"][-1], G["t"][-1]),
                                   float(G["max_depth"]))
        np.testing.assert_array_equal(rgba[..., 3], G["rgba"][..., 3])
        assert np.abs(rgba.astype(int) - G["rgba"]).max() <= 1
        assert np.abs(normal.astype(int) - G["normal"]).max() <= 1
        q = eng.query(None)
        assert q.shape[0] == int(G["query_count"])
        head = G["query_head"]
        np.testing.assert_array_equal(np.stack([q[k] for k in "xyz"], 1)[:head.shape[0]], head[:, :3])
        np.testing.assert_array_equal(q["tsdf"][:head.shape[0]].view(np.uint32),
                                      head[:, 3].copy().view(np.uint32))
    finally:
        eng.close()
