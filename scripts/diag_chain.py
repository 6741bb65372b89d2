#!/usr/bin/env python3
"""Where the one-launch frame's time goes after the carving is published (DIAG=1 library, GPU box).

k_integrate_pre stamps (kernel slot 5): per chained workgroup w -- start, before its wait, after its
wait, done -- and in slot kDiagMaxWg - 1 the tail: carving published (t_pub), flags stored, every
chained workgroup counted, allocation resolver done. All times in us relative to t_pub; the tiles
(w < tiles: the shipped order, tiles first) and the sweep workgroups reported apart (--sweep-first
for a TSDF_PRE_SWEEP_FIRST build). Frames are integrated in pairs (the second is a
pipelined launch) and the stamps read after each pair (the read flushes the pending update).
Usage: make -C disinfect-slam_amd diag && \
    TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so python scripts/diag_chain.py
Diagnostic only: nothing here is part of the product or the bench.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disinfect-slam_amd"))
NK, NWG, NS, NVIS = 8, 4096, 8, 256


def main():
    import ctypes as C
    import torch
    import tsdf_amd
    from tsdf_amd import _lib, synth

    L = _lib.load()
    torch.cuda.set_device(0)
    cam = synth.camera(640, 480, synth.TUM_FR1)
    nwarm, npairs = 60, 20
    n = nwarm + 2 * npairs
    fr = synth.render_torch(cam, list(range(n)), device="cuda")
    torch.cuda.synchronize()
    eng = tsdf_amd.Engine(0.005, 0.03, max_width=640, max_height=480, num_block_bits=18, device=0,
                          stream=torch.cuda.current_stream().cuda_stream)
    en = C.c_int(0)
    L.tsdf_debug_stamps(eng._h, None, 0, C.byref(en))
    if not en.value:
        raise SystemExit("library built without TSDF_DIAG_STAMPS (make diag; set TSDF_AMD_LIB)")
    buf = np.zeros(NK * NWG * NS, np.uint64)
    tiles = 40 * 30

    def step(i):
        eng.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], cam.K,
                      tsdf_amd.SE3(fr["q"][i], fr["t"][i]), 4.0)

    for i in range(nwarm):
        step(i)
    torch.cuda.synchronize()
    L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
    acc = {}

    def put(k, v):
        acc.setdefault(k, []).append(v)

    for p in range(npairs):
        step(nwarm + 2 * p)
        step(nwarm + 2 * p + 1)
        torch.cuda.synchronize()
        buf[:] = 0
        L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
        S = buf.reshape(NK, NWG, NS)[5].astype(np.int64)
        tail = S[NWG - 1]
        if tail[0] == 0:
            continue
        rel = lambda a: (a - tail[0]) * 10e-3
        put("tail: flags stored", rel(tail[1]))
        put("tail: all chained counted", rel(tail[2]))
        put("tail: allocation done", rel(tail[3]))
        sweep_first = "--sweep-first" in sys.argv
        groups = ((("sweep", slice(0, NVIS)), ("tiles", slice(NVIS, NVIS + tiles))) if sweep_first else
                  (("tiles", slice(0, tiles)), ("sweep", slice(tiles, tiles + NVIS))))
        for name, sl in groups:
            rows = S[sl]
            rows = rows[rows[:, 0] > 0]
            for j, ph in enumerate(("start", "pre-wait", "wait end", "done")):
                r = rel(rows[:, j])
                put(f"{name}: {ph} p50", np.median(r))
                put(f"{name}: {ph} p90", np.percentile(r, 90))
                put(f"{name}: {ph} max", r.max())
            put(f"{name}: wait->done p50", np.median((rows[:, 3] - rows[:, 2]) * 10e-3))
            put(f"{name}: wait->done max", ((rows[:, 3] - rows[:, 2]) * 10e-3).max())
            put(f"{name}: n", len(rows))
    print(f"median over {npairs} pipelined launches; us relative to the carving published")
    for k, v in acc.items():
        print(f"   {k:32s} {np.median(v):9.2f}")
    eng.close()


if __name__ == "__main__":
    main()
