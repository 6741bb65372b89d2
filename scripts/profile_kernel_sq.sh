#!/bin/bash
# SQ / memory counters of one kernel under one bench command, one pass per counter group:
#   scripts/profile_kernel_sq.sh <out_dir> <kernel regex> [bench args...]
set -euo pipefail
OUT=${1:?out dir}
RX=${2:?kernel regex}
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for GROUP in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $GROUP --kernel-include-regex "$RX" --output-format csv \
    -d "$OUT/pmc$i" -o run -- python3 bench.py --no-cpu "$@" > "$OUT/pmc${i}_bench.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tsdf::", "")
        acc[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:30s} {c:22s} mean {statistics.mean(v):16.1f} n={len(v)}")
PY
