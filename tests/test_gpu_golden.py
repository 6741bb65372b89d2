"""The HIP engine against the committed golden streams (tests/golden/integrate_48x36*.npz): no oracle
call at run time -- entries, pool indices, free stack, tsdf / rgbw / probability bit-exact (NaN ==
NaN), raycast images bit-exact, Query positions / tsdf exact. The streams: the complement ht / lt
field (6 frames) and, over 40 frames into the weight cap, the segmentation-shaped inputs of VERDICT r5
-- independent ht / lt channels over (0, 1] with the extremes 1e-6 / 1 - 1e-6 / 1, uint16 / 65535
maps with exact zeros in lt (p exactly 1), and in both channels (the reference's 0 / 0 NaN)."""
import numpy as np
import pytest

from test_golden import STREAMS, load_stream, prob_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", STREAMS)
def test_engine_reproduces_golden_stream(name):
    import tsdf_amd
    G = load_stream(name)
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
        assert prob_same(blk(d["prob"]), G["prob"])
        rgba, normal = eng.raycast(G["K"], W, H, tsdf_amd.SE3(G["q"][-1], G["t"][-1]),
                                   float(G["max_depth"]))
        np.testing.assert_array_equal(rgba, G["rgba"])
        np.testing.assert_array_equal(normal, G["normal"])
        q = eng.query(None)
        assert q.shape[0] == int(G["query_count"])
        head = G["query_head"]
        np.testing.assert_array_equal(np.stack([q[k] for k in "xyz"], 1)[:head.shape[0]], head[:, :3])
        np.testing.assert_array_equal(q["tsdf"][:head.shape[0]].view(np.uint32),
                                      head[:, 3].copy().view(np.uint32))
    finally:
        eng.close()
