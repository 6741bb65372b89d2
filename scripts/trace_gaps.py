#!/usr/bin/env python3
"""Per-frame kernel timeline of a `rocprofv3 --kernel-trace` run of bench.py:
   scripts/trace_gaps.py <trace dir> [frames] [first]
Takes `frames` occurrences from frame index `first` (default: the last `frames`) of the per-frame kernel sequence (the bench's timed window)
and prints each kernel's average duration and the average idle gap before it, plus the frame
period -- where the frame time goes beyond the kernels themselves (launch gaps)."""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def main(d, frames=200, first=None):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "tsdf::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("tsdf::", "").replace("void ", "").split("<")[0].replace(
        "k_integrate_t", "k_integrate")
    # the frame starts with k_ingest_dda
    starts = [i for i, r in enumerate(rows) if name(r) == "k_ingest_dda"]
    starts = starts[-(frames + 1):] if first is None else starts[first:first + frames + 1]
    dur, gap = defaultdict(list), defaultdict(list)
    periods = []
    for a, b in zip(starts, starts[1:]):
        periods.append(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]))
        prev_end = None
        for r in rows[a:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            dur[name(r)].append(e - s)
            if prev_end is not None:
                gap[name(r)].append(s - prev_end)
            prev_end = e
        gap["(next frame)"].append(int(rows[b]["Start_Timestamp"]) - prev_end)
    print(f"frames {len(periods)}  period avg {statistics.mean(periods)/1e3:.2f} us  "
          f"median {statistics.median(periods)/1e3:.2f} us")
    for k in dur:
        g = statistics.mean(gap[k]) / 1e3 if gap[k] else float("nan")
        print(f"  {k:20s} dur avg {statistics.mean(dur[k])/1e3:7.2f} us  med {statistics.median(dur[k])/1e3:7.2f}"
              f"  gap before {g:6.2f} us")
    print(f"  {'(next frame)':20s} gap before {statistics.mean(gap['(next frame)'])/1e3:6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 200,
         int(sys.argv[3]) if len(sys.argv) > 3 else None)
