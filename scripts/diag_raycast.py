#!/usr/bin/env python3
"""Step statistics of k_raycast on the C5 bench stream, from the DIAG=1 library (diagnostic only).

Usage (GPU box): TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so python scripts/diag_raycast.py
Per frame: exact-march iterations summed over lanes / rays, iterations where the lane (or any lane of
its wave) looked a block up or read a voxel, and the wave-level maxima.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disinfect-slam_amd"))
NK, NWG, NS = 9, 4096, 8


def main():
    import ctypes as C
    import torch
    import tsdf_amd
    from tsdf_amd import _lib, synth

    L = _lib.load()
    dev = torch.device("cuda", 0)
    cam = synth.camera(640, 480, synth.TUM_FR1)
    nwarm = 60
    fr = synth.render_torch(cam, list(range(nwarm + 5)), device=dev)
    torch.cuda.synchronize()
    eng = tsdf_amd.Engine(0.005, 0.03, max_width=640, max_height=480, num_block_bits=18,
                          device=0, stream=torch.cuda.current_stream().cuda_stream)
    en = C.c_int(0)
    L.tsdf_debug_stamps(eng._h, None, 0, C.byref(en))
    if not en.value:
        raise SystemExit("library built without TSDF_DIAG_STAMPS")
    buf = np.zeros(NK * NWG * NS, np.uint64)
    rgba = torch.zeros((480, 640, 4), dtype=torch.uint8, device=dev)
    normal = torch.zeros_like(rgba)
    for i in range(nwarm):
        eng.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], cam.K,
                      tsdf_amd.SE3(fr["q"][i], fr["t"][i]), 4.0)
    for i in range(nwarm, nwarm + 3):
        pose = tsdf_amd.SE3(fr["q"][i], fr["t"][i])
        torch.cuda.synchronize()
        L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
        eng.raycast(cam.K, 640, 480, pose, 4.0, rgba=rgba, normal=normal)
        torch.cuda.synchronize()
        L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
        q = buf.reshape(NK, NWG, NS)[5].astype(np.int64).sum(axis=0)
        rays, waves = 640 * 480, int(q[7])
        print(f"frame {i}: waves {waves} hits {q[6]} / {rays}")
        print(f"  per ray : iterations {q[0] / rays:7.1f}  block lookups {q[1] / rays:6.1f}  voxel reads {q[2] / rays:6.1f}")
        print(f"  per wave: iterations {q[3] / waves:7.1f}")
        # per-wave lifetimes (kernel 6 stamps: wave w of workgroup wg at 2w / 2w + 1)
        S6 = buf.reshape(NK, NWG, NS)[6].astype(np.int64)
        nwg = 40 * 30
        st, en = S6[:nwg, 0::2], S6[:nwg, 1::2]
        ok = (st > 0) & (en > 0)
        if ok.any():
            t0 = st[ok].min()
            dur = (en - st)[ok] * 10e-3
            endt = (en[ok] - t0) * 10e-3
            stt = (st[ok] - t0) * 10e-3
            print(f"  wave lifetime us: p10 {np.percentile(dur, 10):6.1f} p50 {np.median(dur):6.1f} "
                  f"p90 {np.percentile(dur, 90):6.1f} max {dur.max():6.1f}; start p50 {np.median(stt):5.1f} "
                  f"max {stt.max():5.1f}; end p50 {np.median(endt):6.1f} p90 {np.percentile(endt, 90):6.1f} max {endt.max():6.1f}")
            # where the slowest waves are: their tiles' rows / columns (XCD-aware tile map of k_raycast)
            wg = np.repeat(np.arange(nwg)[:, None], 4, axis=1)[ok]
            g = wg & 7
            tile = g * (nwg >> 3) + np.minimum(g, nwg & 7) + (wg >> 3)
            ty, tx = tile // 40, tile % 40
            slow = dur >= np.percentile(dur, 95)
            print(f"  slowest 5% of waves: tile rows {np.bincount(ty[slow], minlength=30).tolist()}")
            print(f"                       tile cols {np.bincount(tx[slow], minlength=40).tolist()}")
    eng.close()


if __name__ == "__main__":
    main()
