#!/usr/bin/env python3
"""The counter passes of scripts/profile_kernel_sq.sh for one kernel as the JSON bench.py reads
(profiles/<round>_raycast_sq.json): mean counter value per dispatch and per-wave derived values.
usage: sq_json.py <profile_kernel_sq out dir> <kernel substring> "<command>" <width> <height> > out.json"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main(out, kernel, command, width, height):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {"kernel": kernel, "width": int(width), "height": int(height), "command": command,
         "source": "rocprofv3 --pmc passes (scripts/profile_kernel_sq.sh), mean over the run's dispatches",
         "n_dispatches": max(len(v) for v in acc.values())}
    for c, v in sorted(acc.items()):
        d[c] = round(statistics.mean(v), 1)
    w = d.get("SQ_WAVES") or 1.0
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
        if c in d:
            d[c + "_per_wave"] = round(d[c] / w, 1)
    if "SQ_WAVE_CYCLES" in d:
        d["SQ_WAVE_CYCLES_per_wave_quad"] = round(d["SQ_WAVE_CYCLES"] / w, 1)
    json.dump(d, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:6])
