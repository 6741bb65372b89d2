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
NK, NWG, NS = 8, 4096, 8


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
        print(f"  per wave: iterations {q[3] / waves:7.1f}  with a lookup {q[4] / waves:6.1f}  with a read {q[5] / waves:6.1f}")
    eng.close()


if __name__ == "__main__":
    main()
