#!/bin/bash
# A/B timing of bench.py argument sets on one library (GPU box), each run twice, interleaved:
#   scripts/ab_args.sh <steps> "<args A>" "<args B>" ...
set -uo pipefail
STEPS=$1; shift
OUT=gpurun_out/ab
mkdir -p $OUT
for rep in 1 2; do
  i=0
  for args in "$@"; do
    i=$((i+1))
    timeout -k 10 120 python3 bench.py --no-cpu --steps $STEPS $args > $OUT/args${i}_$rep.log 2>&1 || { echo "[$args] failed"; tail -5 $OUT/args${i}_$rep.log; exit 1; }
    python3 - "$OUT/args${i}_$rep.log" "$args" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
r = d['roofline']; dv = d['device_us_per_frame']
print(f"{sys.argv[2]:>24} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} integ_evt={r['us_per_launch']:.2f}us "
      f"ingest={dv['ingest_dda']} alloc={dv['resolve_alloc']} integ={dv['integrate']} carve={dv['resolve_delete']}")
PY
  done
done
