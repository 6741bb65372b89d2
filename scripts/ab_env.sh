#!/bin/bash
# A/B timing of one engine library under different environment settings (GPU box):
#   scripts/ab_env.sh <steps> <lib.so> "VAR=a" "VAR=b" ...
set -uo pipefail
STEPS=$1; LIB=$2; shift 2
OUT=gpurun_out/ab
mkdir -p $OUT
for rep in 1 2; do
  for kv in "$@"; do
    n=$(echo "$kv" | tr '=' '_')
    env "$kv" TSDF_AMD_LIB=$LIB timeout -k 10 120 python3 bench.py --no-cpu --steps $STEPS > $OUT/${n}_$rep.log 2>&1 || { echo "$kv failed"; tail -5 $OUT/${n}_$rep.log; exit 1; }
    python3 - "$OUT/${n}_$rep.log" "$kv" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
r = d['roofline']
print(f"{sys.argv[2]:>28} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} integ_evt={r['us_per_launch']:.2f}us dev={r.get('us_per_launch_device_clock')}us frac={r['frac']:.3f}")
PY
  done
done
