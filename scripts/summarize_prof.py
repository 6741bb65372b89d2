#!/usr/bin/env python3
"""Summarise a scripts/profile_integrate.sh run: per-kernel trace stats + PMC HBM bytes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled.
Writes <out>/summary.json and prints a table.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def find(pattern):
    m = glob.glob(pattern, recursive=True)
    return m[0] if m else None


def bench_line(path):
    try:
        for line in open(path):
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    except OSError:
        pass
    return None


def kname(full):
    """Short kernel name: 'tsdf::k_x(args)' / 'void tsdf::k_integrate_t<false>(args)' -> 'k_x' /
    'k_integrate' (the eager instantiation; the graph one is 'k_integrate_graph')."""
    n = full.split("(")[0].replace("tsdf::", "")
    n = re.sub(r"^void ", "", n)
    return re.sub(r"k_integrate_t<true(, false)?>", "k_integrate_graph", re.sub(r"k_integrate_t<false(, false)?>", "k_integrate", n))


def main(out):
    res = {"kernels": {}, "pmc": {}}
    st = find(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    if st:
        for r in csv.DictReader(open(st)):
            if not re.search(r"tsdf::", r["Name"]):
                continue
            name = kname(r["Name"])
            res["kernels"][name] = {
                "calls": int(r["Calls"]),
                "avg_us": float(r["AverageNs"]) / 1e3,
                "min_us": float(r["MinNs"]) / 1e3,
                "max_us": float(r["MaxNs"]) / 1e3,
                "total_ms": float(r["TotalDurationNs"]) / 1e6,
            }
    # per-dispatch trace: k_integrate durations inside the bench's timed window (launches
    # [warmup, warmup + steps) of the kernel), the same launches the bench's HIP events bracket
    tr = find(os.path.join(out, "trace", "**", "*kernel_trace.csv"))
    b0 = bench_line(os.path.join(out, "trace_bench.log"))
    if tr and b0:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tr))
                if kname(r["Kernel_Name"]) == "k_integrate"]
        w, k = b0["warmup"], b0["steps"]
        win = durs[w:w + k]
        if win:
            res["integrate_timed_window"] = {"launches": len(win), "avg_us": statistics.mean(win) / 1e3,
                                             "event_avg_us": b0["roofline"]["us_per_launch"]}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = find(os.path.join(out, f"pmc_{c}", "**", "*counter_collection.csv"))
        if not f:
            continue
        vals = {}
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if "tsdf::" not in kn or r.get("Counter_Name") != c:
                continue
            name = kname(kn)
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
        for name, v in vals.items():
            kib = statistics.mean(v)
            corr = 2.0 if c == "FETCH_SIZE" else 1.0
            res["pmc"].setdefault(name, {})[c] = {"mean_kib_raw": kib, "bytes_per_launch": kib * 1024 * corr,
                                                   "dispatches": len(v)}
    b = bench_line(os.path.join(out, "trace_bench.log")) or bench_line(os.path.join(out, "pmc_FETCH_SIZE_bench.log"))
    if b:
        res["bench"] = b
    ki = res["pmc"].get("k_integrate", {})
    if "FETCH_SIZE" in ki and "WRITE_SIZE" in ki:
        res["integrate_hbm_bytes_per_launch"] = ki["FETCH_SIZE"]["bytes_per_launch"] + ki["WRITE_SIZE"]["bytes_per_launch"]
        if b:
            res["integrate_alg_bytes_per_launch"] = b["roofline"]["alg_bytes_per_launch"]
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
    if "integrate_hbm_bytes_per_launch" in res and b:
        # the file bench.py reads for roofline.traffic (same workload only)
        json.dump({"width": b["config"]["width"], "height": b["config"]["height"],
                   "hbm_bytes_per_launch": res["integrate_hbm_bytes_per_launch"],
                   "fetch_bytes_per_launch": ki["FETCH_SIZE"]["bytes_per_launch"],
                   "write_bytes_per_launch": ki["WRITE_SIZE"]["bytes_per_launch"],
                   "note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, separate passes, "
                           "mean over all k_integrate dispatches of the bench command"},
                  open(os.path.join(out, "pmc_integrate_latest.json"), "w"), indent=1)
    if "integrate_timed_window" in res:
        t = res["integrate_timed_window"]
        print(f"k_integrate timed window: {t['launches']} launches avg {t['avg_us']:.2f}us "
              f"(bench HIP events {t['event_avg_us']:.2f}us)")
    for k, v in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["total_ms"]):
        p = res["pmc"].get(k, {})
        fb = p.get("FETCH_SIZE", {}).get("bytes_per_launch")
        wb = p.get("WRITE_SIZE", {}).get("bytes_per_launch")
        fs = "n/a" if fb is None else f"{fb / 1e6:.3f}MB"
        ws = "n/a" if wb is None else f"{wb / 1e6:.3f}MB"
        print(f"{k:22s} calls={v['calls']:6d} avg={v['avg_us']:9.2f}us min={v['min_us']:8.2f} "
              f"max={v['max_us']:9.2f} fetch={fs} write={ws}")


if __name__ == "__main__":
    main(sys.argv[1])
