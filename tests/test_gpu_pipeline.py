"""Pipelined frames: tsdf_integrate of frame c launches one k_frame that carves frame
c - 2, allocates and updates frame c - 1 (its listed blocks before that carving) and runs frame c's
ingest; every other entry point completes the pending frames first. Every observable result must be that of the frames in order: the
oracle decides at the small sizes, the unpipelined engine (TSDF_PIPELINE=0, the two-launch frame the
other GPU tests pin to the oracle frame by frame) at full size, with frames integrated back to back
so that the fused launch and the probe-only ingest actually run (a read between frames would flush)."""
import os

import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _engine(pipeline, *args, **kw):
    import tsdf_amd
    old = os.environ.get("TSDF_PIPELINE")
    os.environ["TSDF_PIPELINE"] = "1" if pipeline else "0"
    try:
        return tsdf_amd.Engine(*args, **kw)
    finally:
        if old is None:
            del os.environ["TSDF_PIPELINE"]
        else:
            os.environ["TSDF_PIPELINE"] = old


def _same(a, b, tag):
    da, db = a.dump(), b.dump()
    for k in ("entry_pos", "entry_idx", "heap"):
        assert np.array_equal(da[k], db[k]), f"{tag}: {k}"
    assert da["free"] == db["free"], tag
    for k in ("tsdf", "prob"):
        assert np.array_equal(da[k].view(np.uint32), db[k].view(np.uint32)), f"{tag}: {k}"
    assert np.array_equal(da["rgbw"], db["rgbw"]), f"{tag}: rgbw"
    sa, sb = a.stats(), b.stats()
    for k in ("frames", "total_visible", "total_updated", "total_alloc", "total_deleted", "active_blocks",
              "status"):
        assert sa[k] == sb[k], (tag, k, sa[k], sb[k])


def test_pipelined_stream_equals_oracle_heavy_carving():
    """2 cm voxels at 96x72: many allocations and carvings per frame; 16 frames back to back, the
    oracle compared at frames 8 and 16 (the dumps flush the deferred update)."""
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    cam = synth.camera(96, 72)
    eng = _engine(True, 0.02, 0.08, max_width=96, max_height=72, num_block_bits=13)
    ora = OracleGrid(0.02, 0.08, 13)
    try:
        eng.profile_begin()
        tot = dict(total_visible=0, total_updated=0, total_alloc=0, total_deleted=0)
        for f in range(16):
            fr = synth.render(cam, f)
            eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
            so = ora.stats()  # (the oracle keeps per-frame counts: summed here)
            for k in tot:
                tot[k] += so["last_num_" + k[len("total_"):]]
            if f in (7, 15):
                compare(eng, ora, tag=f"frame {f}")
                s = eng.stats()
                for k in tot:
                    assert s[k] == tot[k], (f, k, s[k], tot[k])
                assert s["active_blocks"] == so["active_blocks"] and s["status"] == 0, (s, so)
        prof = eng.profile_end()
        assert prof["pipelined"] >= 13, prof  # every frame but the two after a dump and the first
        assert tot["total_deleted"] > 0
    finally:
        eng.close()
        ora.close()


def test_pipelined_equals_unpipelined_bench_stream():
    """The bench's 640x480 stream, 60 frames back to back into a pipelined and an unpipelined engine:
    the whole state bit for bit."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    cam = synth.camera(640, 480)
    K = tsdf_amd.CameraIntrinsics(*[float(v) for v in cam.K])
    n = 60
    fr = synth.render_torch(cam, list(range(n)), device="cuda")
    engs = [_engine(p, 0.005, 0.03, max_width=640, max_height=480, num_block_bits=18) for p in (True, False)]
    try:
        for e in engs:
            e.profile_begin()
            for i in range(n):
                e.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], K,
                            tsdf_amd.SE3(fr["q"][i], fr["t"][i]), 4.0)
            e.flush()
            torch.cuda.synchronize()
        p0, p1 = engs[0].profile_end(), engs[1].profile_end()
        assert p0["pipelined"] == n - 1 and p1["pipelined"] == 0, (p0, p1)
        assert p0["sum_visible"] == p1["sum_visible"] and p0["sum_updated"] == p1["sum_updated"]
        _same(engs[0], engs[1], "bench stream")
    finally:
        for e in engs:
            e.close()


def test_pipelined_frame_sizes_and_host_frames_change_between_frames():
    """Consecutive frames of different sizes (the fused launch updates one size and prepares the
    other), host and device frames mixed, with and without the semantic maps."""
    import torch

    import tsdf_amd
    from tsdf_amd import synth
    cams = [synth.camera(640, 480), synth.camera(320, 240), synth.camera(160, 120)]
    engs = [_engine(p, 0.01, 0.04, max_width=640, max_height=480, num_block_bits=16) for p in (True, False)]
    try:
        for f in range(18):
            cam = cams[f % 3]
            fr = synth.render(cam, f)
            ht, lt = (fr["ht"], fr["lt"]) if f % 4 else (None, None)
            args = [fr["rgb"], fr["depth"], ht, lt]
            if f % 2:  # device frames on odd frames
                args = [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in args]
            for e in engs:
                e.integrate(*args, cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
        torch.cuda.synchronize()
        _same(engs[0], engs[1], "mixed sizes")
    finally:
        for e in engs:
            e.close()


def test_reads_between_pipelined_frames_see_every_frame():
    """A raycast, a query and the statistics after each frame (each enqueues the deferred update
    first) give what the unpipelined engine gives; the stream continues pipelined afterwards."""
    import tsdf_amd
    from tsdf_amd import synth
    cam = synth.camera(160, 120)
    engs = [_engine(p, 0.01, 0.04, max_width=160, max_height=120, num_block_bits=14) for p in (True, False)]
    try:
        for f in range(12):
            fr = synth.render(cam, f)
            pose = tsdf_amd.SE3(fr["q"], fr["t"])
            for e in engs:
                e.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, pose, 4.0)
            if f % 3 == 2:
                ra, rb = (e.raycast(cam.K, 160, 120, pose, 4.0) for e in engs)
                assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1]), f
                qa, qb = (e.query() for e in engs)
                assert np.array_equal(qa, qb), f
                sa, sb = (e.stats() for e in engs)
                assert sa == sb, (f, sa, sb)
        _same(engs[0], engs[1], "reads between frames")
    finally:
        for e in engs:
            e.close()
