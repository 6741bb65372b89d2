#!/usr/bin/env python3
"""Per-workgroup phase timing of the frame kernels from the DIAG=1 library (s_memrealtime, 100 MHz).

Usage (GPU box): make -C disinfect-slam_amd diag && \
    TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so python scripts/diag_stamps.py
Diagnostic only: nothing here is part of the product or the bench.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disinfect-slam_amd"))

KERNELS = {0: ("ingest", ["lds_init", "pix_write", "dda", "barrier", "sweep"]),
           1: ("resolve_alloc", ["prepare", "sort", "claim", "dirty", "commit", "rest"]),
           2: ("vis (in ingest)", ["all"]),
           3: ("integrate", ["all"]),
           4: ("resolve_delete", ["sum+prepare", "rounds"]),
           6: ("ingest_tail", ["resolve", "ticks"]),
           7: ("integrate_tail", ["carve", "stats"])}
NK, NWG, NS = 9, 4096, 8
ORDER = [2, 0, 1, 6, 3, 4, 7]  # dispatch / execution order of the stamped phases


def main():
    import ctypes as C
    import torch
    import tsdf_amd
    from tsdf_amd import _lib, synth

    L = _lib.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    W, H = int(os.environ.get("DIAG_W", 640)), int(os.environ.get("DIAG_H", 480))
    cam = synth.camera(W, H, synth.TUM_FR1)
    nwarm, nmeas = 60, 20
    fr = synth.render_torch(cam, list(range(nwarm + nmeas)), device=dev)
    torch.cuda.synchronize()
    eng = tsdf_amd.Engine(0.005, 0.03, max_width=W, max_height=H, num_block_bits=18,
                          device=0, stream=torch.cuda.current_stream().cuda_stream)
    en = C.c_int(0)
    L.tsdf_debug_stamps(eng._h, None, 0, C.byref(en))
    if not en.value:
        raise SystemExit("library built without TSDF_DIAG_STAMPS (make diag; set TSDF_AMD_LIB)")
    buf = np.zeros(NK * NWG * NS, np.uint64)

    def step(i):
        eng.integrate(fr["rgb"][i], fr["depth"][i], fr["ht"][i], fr["lt"][i], cam.K,
                      tsdf_amd.SE3(fr["q"][i], fr["t"][i]), 4.0)

    for i in range(nwarm):
        step(i)
    torch.cuda.synchronize()
    L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
    acc = {}
    for i in range(nwarm, nwarm + nmeas):
        step(i)
        torch.cuda.synchronize()
        L.tsdf_debug_stamps(eng._h, buf.ctypes.data, buf.size, None)
        S = buf.reshape(NK, NWG, NS).astype(np.int64)
        t0 = None
        bounds = []
        for k, (name, phases) in sorted(KERNELS.items(), key=lambda kv: ORDER.index(kv[0])):
            s = S[k]
            valid = s[:, 0] > 0
            if not valid.any():
                continue
            s = s[valid]
            last = len(phases)
            start, end = s[:, 0].min(), s[:, last].max()
            if t0 is None:
                t0 = start
            bounds.append((name, start, end))
            d = acc.setdefault(name, {"n_wg": [], "span": [], "start_skew_p50": [],
                                      "start_skew_max": [], **{p: [] for p in phases},
                                      **{p + "_max": [] for p in phases}})
            d["n_wg"].append(len(s))
            d["span"].append((end - start) * 10e-3)
            sk = (s[:, 0] - start) * 10e-3
            d["start_skew_p50"].append(np.median(sk))
            d["start_skew_max"].append(sk.max())
            for q in (10, 90, 99):
                d.setdefault(f"start_skew_p{q}", []).append(np.percentile(sk, q))
            ek = (s[:, last] - start) * 10e-3
            for q in (10, 50, 90, 99):
                d.setdefault(f"end_p{q}", []).append(np.percentile(ek, q))
            late = s[sk > 5.0]
            d.setdefault("n_start_after_5us", []).append(len(late))
            for j, p in enumerate(phases):
                dur = (s[:, j + 1] - s[:, j]) * 10e-3
                d[p].append(np.median(dur))
                d[p + "_max"].append(dur.max())
            if k == 0 and (s[:, 6] > 0).all():  # the tile's tail: corner tests (4 -> 6), probes + inserts (6 -> 5)
                for p, a, b in (("corners", 4, 6), ("probe_insert", 6, 5)):
                    dur = (s[:, b] - s[:, a]) * 10e-3
                    d.setdefault(p, []).append(np.median(dur))
                    d.setdefault(p + "_max", []).append(dur.max())
        if S[1, 0, 7] > 0:  # TSDF_EXP & 16 diag build: the resolver's sort repeated (warm)
            acc.setdefault("resolve_alloc sort repeated", {}).setdefault("sort2", []).append(
                (S[1, 0, 7] - S[1, 0, 2]) * 10e-3)
        # k_integrate placement (diag build): per CU (xcc, se, cu) the pairs of its workgroups and
        # the latest end; per pair count the workgroups' end times
        s3 = S[3]
        ok3 = s3[:, 0] > 0
        if ok3.any() and (s3[ok3, 5] >= 0).all():
            t3 = s3[ok3, 0].min()
            hw = s3[ok3, 4].astype(np.int64)
            cu = (s3[ok3, 5] << 9) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
            pairs = np.maximum(s3[ok3, 6], 0)
            end = (s3[ok3, 1] - t3) * 10e-3
            d = acc.setdefault("integrate per CU", {})
            ucu = np.unique(cu)
            per_pairs = np.array([pairs[cu == c].sum() for c in ucu])
            per_end = np.array([end[cu == c].max() for c in ucu])
            per_nwg = np.array([(cu == c).sum() for c in ucu])
            d.setdefault("n_cu", []).append(len(ucu))
            d.setdefault("wg_per_cu_min", []).append(per_nwg.min())
            d.setdefault("wg_per_cu_max", []).append(per_nwg.max())
            d.setdefault("pairs_per_cu_min", []).append(per_pairs.min())
            d.setdefault("pairs_per_cu_mean", []).append(per_pairs.mean())
            d.setdefault("pairs_per_cu_max", []).append(per_pairs.max())
            d.setdefault("cu_end_min", []).append(per_end.min())
            d.setdefault("cu_end_p50", []).append(np.median(per_end))
            d.setdefault("cu_end_max", []).append(per_end.max())
            d.setdefault("corr_pairs_end", []).append(np.corrcoef(per_pairs, per_end)[0, 1] if per_pairs.std() > 0 else 0)
            for npair in (0, 1, 2, 3):
                m = pairs == npair
                if m.any():
                    d.setdefault(f"wg_end_p50_{npair}pairs", []).append(np.median(end[m]))
                    d.setdefault(f"wg_end_max_{npair}pairs", []).append(end[m].max())
                    d.setdefault(f"n_wg_{npair}pairs", []).append(m.sum())
        for (n1, _, e1), (n2, s2, _) in zip(bounds, bounds[1:]):
            acc.setdefault("gaps", {}).setdefault(f"{n1}->{n2}", []).append((s2 - e1) * 10e-3)
        acc.setdefault("frame", {}).setdefault("first_start_to_last_end", []).append(
            (bounds[-1][2] - bounds[0][1]) * 10e-3)
    print("median over", nmeas, "frames; microseconds (per-WG medians / maxima)")
    for name, d in acc.items():
        print(f"[{name}]")
        for key, v in d.items():
            print(f"   {key:24s} {np.median(v):9.2f}")
    eng.close()


if __name__ == "__main__":
    main()
