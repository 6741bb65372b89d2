#!/usr/bin/env python3
"""Per-frame kernel chain of a rocprofv3 kernel trace (diagnostic): for every kernel name its mean
duration and the mean idle gap before it (the previous dispatch's end -> its start), over the last
half of the trace (the timed frames), plus the total busy / idle time per frame.
Usage: chain_timeline.py <rocprofv3 output dir> [frame-kernel regex]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_ingest_dda|k_frame")
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[len(rows) // 2:]
    short = lambda n: re.sub(r"\(.*", "", n).replace("tsdf::", "").replace("void ", "")
    dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
    nfr = sum(1 for r in rows if first.search(r[2]))
    prev = None
    busy = idle = 0
    for s, e, n in rows:
        k = short(n)
        dur[k] += (e - s) / 1e3
        cnt[k] += 1
        if prev is not None:
            g = max(0, s - prev) / 1e3
            gap[k] += g
            idle += g
        busy += (e - s) / 1e3 if prev is None or s >= prev else max(0, e - prev) / 1e3
        prev = max(prev or 0, e)
    print(f"{f}\n{len(rows)} dispatches, {nfr} frames (first kernel /{first.pattern}/)")
    print(f"{'kernel':>40} {'per frame':>9} {'mean us':>8} {'gap us':>7} {'us/frame':>9}")
    for k in sorted(dur, key=lambda k: -dur[k]):
        print(f"{k[:40]:>40} {cnt[k] / max(nfr, 1):9.2f} {dur[k] / cnt[k]:8.2f} {gap[k] / cnt[k]:7.2f} "
              f"{dur[k] / max(nfr, 1):9.2f}")
    print(f"per frame: busy {busy / max(nfr, 1):.1f} us, idle {idle / max(nfr, 1):.1f} us")


if __name__ == "__main__":
    main()
