#!/bin/bash
# Raycast iteration loop on the GPU box: parity tests, the C5 bench line, kernel trace and SQ counters.
#   scripts/raycast_check.sh <out_dir>
set -euo pipefail
OUT=${1:?out}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > "$OUT/tests.log" 2>&1
timeout -k 10 200 python3 bench.py --loop c5 --no-cpu > "$OUT/c5.log" 2>&1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run -- python3 bench.py --loop c5 --no-cpu --steps 100 > "$OUT/c5_prof.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  --kernel-include-regex k_raycast --output-format csv -d "$OUT/pmc" -o run -- python3 bench.py --loop c5 --no-cpu --steps 40 --warmup 5 > "$OUT/pmc.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics, collections, json
out = sys.argv[1]
for l in open(out + "/c5.log"):
    if l.startswith("{"):
        d = json.loads(l); print("C5", d["value"], "fps", d["ms_per_step"], "ms/step")
for r in csv.DictReader(open(glob.glob(out + "/prof_c5/*kernel_stats.csv")[0])):
    if "tsdf::" in r["Name"]:
        print(f'{r["Name"].split("(")[0]:40s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:9.2f} us')
acc = collections.defaultdict(list)
for f in glob.glob(out + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = statistics.mean(acc["SQ_WAVES"]) if acc.get("SQ_WAVES") else 1
for k, v in sorted(acc.items()):
    print(f"{k:22s} mean {statistics.mean(v):14.1f}  per wave {statistics.mean(v) / w:10.1f}")
PY
