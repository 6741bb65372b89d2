#!/usr/bin/env python3
"""Per-part timeline of the pipelined frame kernel k_frame from the DIAG=1 library (diagnostic only).

Usage (GPU box): TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so python scripts/diag_frame.py
The driver's workload (bench.py C3: 640x480, frames 0-24, the first five warm-up): after each
tsdf_integrate (one k_frame) the stamps of every workgroup -- part, start, end (D.dbg kernel 8) --
relative to the launch's first workgroup start, in microseconds, as medians over the launches.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disinfect-slam_amd"))
NK, NWG, NS = 9, 4096, 8
PARTS = {1: "head", 2: "fresh update", 3: "listed update", 4: "tiles", 5: "sweep"}


def main():
    import ctypes as C
    import torch
    import tsdf_amd
    from tsdf_amd import _lib, synth

    L = _lib.load()
    dev = torch.device("cuda", 0)
    cam = synth.camera(640, 480, synth.TUM_FR1)
    nfr = 25
    fr = synth.render_torch(cam, list(range(nfr)), device=dev)
    torch.cuda.synchronize()
    eng = tsdf_amd.Engine(0.005, 0.03, max_width=640, max_height=480, num_block_bits=18,
                          device=0, stream=torch.cuda.current_stream().cuda_stream)
    en = C.c_int(0)
    L.tsdf_debug_stamps(eng._h, None, 0, C.byref(en))
    if not en.value:
        raise SystemExit("library built without TSDF_DIAG_STAMPS")
    buf = np.zeros(NK * NWG * NS, np.uint64)
    rows = {k: [] for k in PARTS}
    head = []
    coll = []
    tiles = []
    phases = []
    for i in range(nfr):
        torch.cuda.synchronize()
        L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)  # (clears)
        eng.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], cam.K,
                      tsdf_amd.SE3(fr["q"][i], fr["t"][i]), 4.0)
        torch.cuda.synchronize()
        L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
        if i < 6:
            continue
        S = buf.reshape(NK, NWG, NS)[8].astype(np.int64)
        ok = S[:, 0] > 0
        if not ok.any():
            continue
        t0 = S[ok, 1].min()
        for k in PARTS:
            m = S[:, 0] == k
            if m.any():
                st, en_ = (S[m, 1] - t0) * 1e-2, (S[m, 2] - t0) * 1e-2
                rows[k].append((m.sum(), np.median(st), st.max(), np.median(en_), np.percentile(en_, 90),
                                en_.max(), np.median(en_ - st)))
        T = buf.reshape(NK, NWG, NS)[0].astype(np.int64)  # tile stamps (tsdf_ingest.h ingest_tile)
        mt = (S[:, 0] == 4) & (T[:, 0] > 0) & (T[:, 5] > 0)
        if mt.any():
            st = T[mt, 0]
            tiles.append([np.median((T[mt, k] - st) * 1e-2) for k in (1, 2, 3, 6, 7, 5)] +
                         [np.median((T[mt, 7] - T[mt, 6]) * 1e-2)])
        m = S[:, 0] == 3
        if m.any() and (S[m, 5] > 0).any():  # listed update: collect phases (first / last end), records
            st = S[m, 1]
            coll.append((np.median((S[m, 3] - st) * 1e-2), np.percentile((S[m, 3] - st) * 1e-2, 90),
                         np.median((S[m, 4] - st) * 1e-2), np.median(S[m, 5] & 0xFFFF)))
        A1 = buf.reshape(NK, NWG, NS)[1, 0].astype(np.int64)  # head: allocation resolver stamps
        D4 = buf.reshape(NK, NWG, NS)[4, 0].astype(np.int64)  # head: carving resolver stamps
        rel = lambda v: (v - t0) * 1e-2 if v else np.nan
        phases.append((rel(D4[0]), rel(D4[3]), rel(D4[4]), rel(S[0, 3]), rel(A1[0]), rel(A1[7]), rel(A1[3]),
                       rel(A1[4]), rel(A1[5]), rel(S[0, 4])))
        h = S[0]
        if h[0] == 1:
            head.append(((h[3] - t0) * 1e-2 if h[3] else np.nan, (h[4] - t0) * 1e-2 if h[4] else np.nan,
                         (h[2] - t0) * 1e-2))
    print("k_frame part timeline, us from the launch's first workgroup start (medians over launches)")
    print(f"{'part':>14} {'WGs':>5} {'start p50':>9} {'start max':>9} {'end p50':>8} {'end p90':>8} "
          f"{'end max':>8} {'dur p50':>8}")
    for k, name in PARTS.items():
        if rows[k]:
            a = np.median(np.array(rows[k], dtype=float), axis=0)
            print(f"{name:>14} {a[0]:5.0f} {a[1]:9.1f} {a[2]:9.1f} {a[3]:8.1f} {a[4]:8.1f} {a[5]:8.1f} {a[6]:8.1f}")
    if tiles:
        a = np.median(np.array(tiles), axis=0)
        print("tile phases (us from the tile's start, medians): LDS init %.1f, pixel records %.1f, DDA %.1f, "
              "corner tests %.1f, allocation flag seen %.1f, probes + inserts done %.1f; waiting %.1f" % tuple(a))
    if coll:
        a = np.median(np.array(coll), axis=0)
        print(f"listed update: first collect done {a[0]:.1f} (p90 {a[1]:.1f}), last collect done {a[2]:.1f} us "
              f"after the workgroup start; records + collections {a[3]:.0f}")
    if phases:
        a = np.nanmedian(np.array(phases), axis=0)
        print("head phases (us from the launch start): carving start %.1f, buckets loaded %.1f, deletes issued "
              "%.1f, published %.1f | allocation start %.1f, counters+keys %.1f, orders+buckets+heap %.1f, "
              "barrier %.1f, commits issued %.1f, published %.1f" % tuple(a))
    if head:
        a = np.nanmedian(np.array(head), axis=0)
        print(f"head: carving published {a[0]:.1f}, allocation published {a[1]:.1f}, head end {a[2]:.1f}")
    eng.close()


if __name__ == "__main__":
    main()
