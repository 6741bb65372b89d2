#!/usr/bin/env python3
"""Summarise a scripts/profile_integrate.sh run: per-kernel trace stats + PMC HBM bytes.

  summarize_prof.py <out_dir>            -> <out_dir>/summary.json, <out_dir>/pmc_entry.json, table
  summarize_prof.py --merge <entry.json> <profiles/pmc_integrate_r2.json>

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled.
The PMC means are over the k_integrate dispatches of the bench's timed window only (launches
[warmup, warmup + steps) in dispatch order), and the entry carries the bench's pmc_key and the
N_vis / N_upd sums of that window, which bench.py matches before it reports roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def find(pattern):
    m = sorted(glob.glob(pattern, recursive=True))
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
    n = re.sub(r"k_integrate_t<false(, false)?>", "k_integrate", n)
    return re.sub(r"k_integrate_t<true(, false)?>", "k_integrate_graph", n)


def window(rows, b, name=""):
    """rows (dispatch id, value) of one kernel -> the bench's timed-window launches. Pipelined frames
    (k_frame): the timed window is one k_ingest_dda (the first frame after the warmup's flush), then
    steps - 1 k_frame launches of one frame each, then the flush's two k_frame launches (the last
    frame's allocation + update, then its carving alone): the window's per-frame launches are the
    last steps + 1 but two."""
    rows = sorted(rows)
    w, k = b["warmup"], b["steps"]
    if name in ("k_frame", "k_frame_g"):
        return [v for _, v in rows[-(k + 1):-2]]
    return [v for _, v in rows[w:w + k]]


def main(out):
    res = {"kernels": {}, "pmc": {}}
    st = find(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    b0 = bench_line(os.path.join(out, "trace_bench.log"))
    if st:
        for r in csv.DictReader(open(st)):
            if "tsdf::" not in r["Name"]:
                continue
            res["kernels"][kname(r["Name"])] = {
                "calls": int(r["Calls"]),
                "avg_us": float(r["AverageNs"]) / 1e3,
                "min_us": float(r["MinNs"]) / 1e3,
                "max_us": float(r["MaxNs"]) / 1e3,
                "total_ms": float(r["TotalDurationNs"]) / 1e6,
            }
    tr = find(os.path.join(out, "trace", "**", "*kernel_trace.csv"))
    if tr and b0:
        per = {}
        for r in csv.DictReader(open(tr)):
            per.setdefault(kname(r["Kernel_Name"]), []).append(
                (int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        res["timed_window"] = {}
        for name, rows in per.items():
            if not name.startswith("k_") or len(rows) < b0["steps"] - 1 or (name in ("k_frame", "k_frame_g") and len(rows) < b0["steps"] + 1):
                continue
            win = window(rows, b0, name)
            res["timed_window"][name] = {"launches": len(win), "avg_us": statistics.mean(win) / 1e3,
                                         "min_us": min(win) / 1e3, "max_us": max(win) / 1e3}
        res["bench_event_us_per_launch"] = b0["roofline"]["us_per_launch"]
    pmc_lines = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = find(os.path.join(out, f"pmc_{c}", "**", "*counter_collection.csv"))
        b = bench_line(os.path.join(out, f"pmc_{c}_bench.log"))
        if not f or not b:
            continue
        pmc_lines[c] = b
        per = {}
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if "tsdf::" not in kn or r.get("Counter_Name") != c:
                continue
            per.setdefault(kname(kn), []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        corr = 2.0 if c == "FETCH_SIZE" else 1.0
        for name, rows in per.items():
            full = len(rows) >= b["warmup"] + b["steps"] or (name in ("k_frame", "k_frame_g") and len(rows) >= b["steps"] + 1)
            win = window(rows, b, name) if full else [v for _, v in sorted(rows)]
            res["pmc"].setdefault(name, {})[c] = {
                "bytes_per_launch": statistics.mean(win) * 1024 * corr, "dispatches": len(win),
                "timed_window": full}
    if b0:
        res["bench"] = b0
    # the frame launch of the line: k_frame for pipelined frames, else k_integrate
    kn = next((k for k in ("k_frame", "k_frame_g", "k_integrate_vg", "k_integrate", "k_integrate_graph") if k in res["pmc"]), None)
    ki = res["pmc"].get(kn, {}) if kn else {}
    if "FETCH_SIZE" in ki and "WRITE_SIZE" in ki:
        bf, bw = pmc_lines["FETCH_SIZE"], pmc_lines["WRITE_SIZE"]
        same = (bf["sum_visible"], bf["sum_updated"]) == (bw["sum_visible"], bw["sum_updated"])
        if b0:
            same = same and (b0["sum_visible"], b0["sum_updated"]) == (bf["sum_visible"], bf["sum_updated"])
        fetch, write = ki["FETCH_SIZE"]["bytes_per_launch"], ki["WRITE_SIZE"]["bytes_per_launch"]
        entry = {"key": bf["pmc_key"], "sum_visible": bf["sum_visible"], "sum_updated": bf["sum_updated"],
                 "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                 "hbm_bytes_per_launch": fetch + write,
                 "alg_bytes_per_launch": bf["roofline"]["alg_bytes_per_launch"],
                 "alg_read_bytes_per_launch": bf["roofline"]["alg_read_bytes_per_launch"],
                 "launches": ki["FETCH_SIZE"]["dispatches"], "passes_saw_same_frames": same,
                 # the frame kernel's timed-window mean from the kernel trace of the same command: bench.py
                 # takes it as the launch duration where no dispatch events exist (graph frames)
                 "trace_kernel": kn,
                 "trace_kernel_avg_us": res.get("timed_window", {}).get(kn, {}).get("avg_us"),
                 "note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE, separate passes of "
                         "the bench command; mean over the timed-window k_integrate dispatches"}
        res["integrate_pmc_entry"] = entry
        json.dump(entry, open(os.path.join(out, "pmc_entry.json"), "w"), indent=1)
        if not same:
            print("WARNING: the passes integrated different frames (N_vis/N_upd sums differ)")
        print(f"{kn} PMC (timed window, {entry['launches']} launches): fetch {fetch / 1e6:.3f} MB, "
              f"write {write / 1e6:.3f} MB, total {(fetch + write) / 1e6:.3f} MB vs algorithmic "
              f"{entry['alg_bytes_per_launch'] / 1e6:.3f} MB (read {entry['alg_read_bytes_per_launch'] / 1e6:.3f})")
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
    if b0:
        d = b0.get("device_us_per_frame", {})
        print("bench: %.1f frames/s, %.4f ms/step; device us/frame: %s" % (
            b0["value"], b0["ms_per_step"], {k: v for k, v in d.items() if k != "note"}))
    for name, t in sorted(res.get("timed_window", {}).items()):
        print(f"{name} timed window: {t['launches']} launches avg {t['avg_us']:.2f}us "
              f"(min {t['min_us']:.2f}, max {t['max_us']:.2f})")
    if "bench_event_us_per_launch" in res:
        print(f"bench HIP events (frame kernel): {res['bench_event_us_per_launch']}us")
    for k, v in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["total_ms"]):
        p = res["pmc"].get(k, {})
        fb = p.get("FETCH_SIZE", {}).get("bytes_per_launch")
        wb = p.get("WRITE_SIZE", {}).get("bytes_per_launch")
        fs = "n/a" if fb is None else f"{fb / 1e6:.3f}MB"
        ws = "n/a" if wb is None else f"{wb / 1e6:.3f}MB"
        print(f"{k:22s} calls={v['calls']:6d} avg={v['avg_us']:9.2f}us min={v['min_us']:8.2f} "
              f"max={v['max_us']:9.2f} fetch={fs} write={ws}")


def merge(entry_path, table_path):
    e = json.load(open(entry_path))
    try:
        t = json.load(open(table_path))
    except (OSError, ValueError):
        t = {"runs": []}
    t["runs"] = [r for r in t["runs"] if r.get("key") != e["key"]] + [e]
    json.dump(t, open(table_path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--merge":
        merge(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1])
