#!/usr/bin/env python3
"""Summarise the SQ counter passes of scripts/profile_sq.sh: per-kernel mean counter value per
dispatch, plus derived VALU instructions per wave and busy fractions. Prints a table and writes
<out>/sq_summary.json."""
import csv
import glob
import json
import os
import re
import statistics
import sys


def main(out):
    vals = {}
    for f in sorted(glob.glob(os.path.join(out, "sq*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if "tsdf::" not in kn:
                continue
            name = re.sub(r"^void ", "", kn.split("(")[0].replace("tsdf::", "")).replace("k_integrate_t<false, false>", "k_integrate").replace("k_integrate_t<false>", "k_integrate")
            vals.setdefault(name, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res = {k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in vals.items()}
    for k, c in res.items():
        w = c.get("SQ_WAVES")
        if w:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
                if n in c:
                    c[n + "_per_wave"] = c[n] / w
        if c.get("SQ_WAVE_CYCLES"):
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    c[n + "_frac"] = c[n] / c["SQ_WAVE_CYCLES"]
    json.dump(res, open(os.path.join(out, "sq_summary.json"), "w"), indent=1)
    for k in sorted(res):
        c = res[k]
        keys = [x for x in ("SQ_WAVES", "SQ_INSTS_VALU_per_wave", "SQ_INSTS_VMEM_per_wave",
                            "SQ_INSTS_LDS_per_wave", "SQ_WAIT_ANY_frac", "SQ_ACTIVE_INST_VALU_frac",
                            "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE") if x in c]
        print(f"{k:20s} " + " ".join(f"{x}={c[x]:.3g}" for x in keys))


if __name__ == "__main__":
    main(sys.argv[1])
