"""Snapshot / restore (tsdf_snapshot_save / _load, SURVEY.md 5 checkpoint / resume): an engine
restored from a snapshot continues a frame stream exactly as the engine that wrote it -- entries,
pool indices, free stack and every voxel bit-identical -- and both still equal the CPU oracle run
over the whole stream. A snapshot of another configuration is refused.
"""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

W, H, VOXEL, TRUNC, NB = 128, 96, 0.01, 0.04, 14


def _same(a, b, tag):
    da, db = a.dump(pool=True), b.dump(pool=True)
    for k in ("entry_pos", "entry_idx", "heap", "tsdf", "rgbw", "prob"):
        x, y = np.asarray(da[k]), np.asarray(db[k])
        if x.dtype.kind == "f":
            x, y = x.view(np.uint32), y.view(np.uint32)
        assert np.array_equal(x, y), f"{tag}: {k} differs"
    assert da["free"] == db["free"], tag


def _feed(eng, cam, frames):
    import tsdf_amd
    from tsdf_amd import synth
    for f in frames:
        fr = synth.render(cam, f)
        eng.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], cam.K, tsdf_amd.SE3(fr["q"], fr["t"]), 4.0)
        assert eng.stats()["status"] == 0


def test_restore_continues_stream_bit_exact(tmp_path):
    import tsdf_amd
    from tsdf_amd import synth
    from _oracle import OracleGrid
    cam = synth.camera(W, H, synth.TUM_FR1)
    a = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=NB)
    b = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=NB)
    ora = OracleGrid(VOXEL, TRUNC, NB)
    try:
        _feed(a, cam, range(0, 12, 2))
        snap = a.snapshot()
        path = tmp_path / "vol.snap"
        snap.tofile(path)
        b.restore(np.fromfile(path, dtype=np.uint8))
        _same(a, b, "right after restore")
        assert b.stats()["active_blocks"] == a.stats()["active_blocks"] > 0
        # both continue with frames that carve (the camera moves on) and allocate
        _feed(a, cam, range(12, 40, 2))
        _feed(b, cam, range(12, 40, 2))
        _same(a, b, "after resuming")
        for f in range(0, 40, 2):
            fr = synth.render(cam, f)
            ora.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
        compare(b, ora, tag="restored engine vs oracle")
        # rewinding an engine onto its own earlier snapshot replays identically
        a.restore(snap)
        _feed(a, cam, range(12, 40, 2))
        _same(a, b, "rewound engine")
    finally:
        a.close()
        b.close()
        ora.close()


def test_restore_rejects_other_configurations():
    import tsdf_amd
    a = tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=12)
    snap = a.snapshot()
    others = [tsdf_amd.Engine(VOXEL, TRUNC, max_width=W, max_height=H, num_block_bits=13),
              tsdf_amd.Engine(0.02, TRUNC, max_width=W, max_height=H, num_block_bits=12)]
    try:
        for o in others:
            with pytest.raises(tsdf_amd.TSDFError):
                o.restore(snap)
        with pytest.raises(tsdf_amd.TSDFError):
            a.restore(snap[:-1])  # truncated
        bad = snap.copy()
        bad[0] ^= 0xFF
        with pytest.raises(tsdf_amd.TSDFError):
            a.restore(bad)
        a.restore(snap)  # its own snapshot is fine
    finally:
        a.close()
        for o in others:
            o.close()
