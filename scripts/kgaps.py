#!/usr/bin/env python3
"""Durations of, and idle gaps between, consecutive dispatches of the frame kernel in a rocprofv3
kernel trace (diagnostic). Usage: kgaps.py <rocprofv3 output dir> [kernel regex]"""
import csv
import glob
import re
import statistics as st
import sys

d = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_frame")
f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
names = {}
for s, e, n in rows:
    names[n.split("(")[0][:60]] = names.get(n.split("(")[0][:60], 0) + 1
print("kernels:", names)
fr = [r for r in rows if pat.search(r[2])]
fr = fr[len(fr) // 4:]  # (past the warmup)
dur = [(e - s) / 1e3 for s, e, _ in fr]
gap = [(b[0] - a[1]) / 1e3 for a, b in zip(fr, fr[1:])]
allgap = [(b[0] - a[1]) / 1e3 for a, b in zip(rows, rows[1:])]
print(f"{len(fr)} dispatches: duration p50 {st.median(dur):.2f} us, gap to next p50 {st.median(gap):.2f} "
      f"p10 {sorted(gap)[len(gap) // 10]:.2f} p90 {sorted(gap)[9 * len(gap) // 10]:.2f} us; "
      f"period {st.median([(b[0] - a[0]) / 1e3 for a, b in zip(fr, fr[1:])]):.2f} us")
print("gaps (first 24):", " ".join(f"{g:.1f}" for g in gap[:24]))
