#!/usr/bin/env python3
"""Per-frame kernel chain of a rocprofv3 kernel trace of a frame loop (diagnostic).

A frame starts at each dispatch of its first kernel (regex, default k_ingest_dda /
k_render_ingest / k_frame / k_copy_words); frames holding only engine kernels (k_* and the runtime's copies) are kept. Prints
the frame period (median over the plain frames, and each marching-cubes frame's period with its
kernels) and, per kernel, the median duration in the plain frames.
Usage: chain_timeline.py <rocprofv3 output dir> [first-kernel regex]"""
import csv
import glob
import re
import statistics as st
import sys
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*", "", n).replace("tsdf::", "").replace("void ", "")


def main():
    d = sys.argv[1]
    first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_ingest_dda|k_render_ingest|k_frame|k_copy_words")
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                  for r in csv.DictReader(open(f)))
    idx = [i for i, r in enumerate(rows) if first.match(r[2])]
    engine = lambda n: n.startswith("k_") or n.startswith("__amd_rocclr_copy")
    segs = [rows[a:b] for a, b in zip(idx, idx[1:]) if all(engine(r[2]) for r in rows[a:b])]
    plain_len = st.mode(len(s) for s in segs)
    plain = [s for s in segs if len(s) == plain_len]
    print(f"{f}: {len(idx)} frames, {len(plain)} plain frames of {plain_len} dispatches")
    per = [(s[-1][1] - s[0][0]) / 1e3 for s in plain]
    print(f"plain frame, first start -> last end: median {st.median(per):.1f} us")
    gaps = [sum(max(0, s[k + 1][0] - s[k][1]) for k in range(len(s) - 1)) / 1e3 for s in plain]
    print(f"plain frame, idle gaps between its kernels: median {st.median(gaps):.1f} us")
    dur = defaultdict(list)
    for s in plain:
        for a, b, n in s:
            dur[n].append((b - a) / 1e3)
    for n, v in dur.items():
        print(f"  {n[:40]:>40}  {st.median(v):7.1f} us")
    for a, b in zip(idx, idx[1:]):
        s = rows[a:b]
        if len(s) > plain_len and all(engine(r[2]) for r in s):
            extra = "  ".join(f"{n[:14]}={(e - t) / 1e3:.1f}" for t, e, n in s[plain_len:])
            print(f"mesh frame: period {(rows[b][0] - rows[a][0]) / 1e3:.0f} us; {extra}")


if __name__ == "__main__":
    main()
