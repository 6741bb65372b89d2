#!/bin/bash
# r3 final lines: default bench (CPU baseline + PMC traffic), unpipelined default, C4 unsharded,
# 8-shard C4 rehearsal, per-phase stamps (diagnostic library, frames synchronised one by one)
set -uo pipefail
OUT=gpurun_out/r3final2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
head -c 200 $OUT/bench_default.json; echo
TSDF_PIPELINE=0 timeout -k 10 200 python3 bench.py --no-cpu > $OUT/bench_unpipelined.json 2>/dev/null || exit 1
timeout -k 10 200 python3 bench.py --no-cpu --width 1280 --height 720 > $OUT/bench_c4.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --width 1280 --height 720 --shard 8 > $OUT/rehearsal_c4_8shards.json 2>/dev/null || exit 1
TSDF_PIPELINE=0 TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_stamps.py > $OUT/stamps_unpipelined.txt 2>&1 || exit 1
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], d["value"], d.get("ms_per_step"), d.get("device_us_per_frame", {}).get("ingest_dda") if isinstance(d.get("device_us_per_frame"), dict) else "")
PY
