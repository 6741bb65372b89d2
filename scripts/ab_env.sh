#!/bin/bash
# A/B of engine environment settings on the driver's bench command (GPU box, repo root):
#   scripts/ab_env.sh "<ENV=a ENV2=b>" "<ENV=c>" ...   (each setting run twice, interleaved)
set -uo pipefail
OUT=gpurun_out/ab_env
mkdir -p $OUT
for rep in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    env $setting timeout -k 10 120 python3 bench.py --no-cpu --gpus 1 --steps 20 --warmup 5 ${AB_ARGS:-} > $OUT/s${i}_$rep.log 2>&1 || { echo "$setting failed"; tail -5 $OUT/s${i}_$rep.log; exit 1; }
    python3 - "$OUT/s${i}_$rep.log" "$setting" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
r = d['roofline']
dv = {k: v for k, v in d['device_us_per_frame'].items() if k != 'note'}
print(f"{sys.argv[2]:>36} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} launch={r['us_per_launch']:.2f}us dev={dv}")
PY
  done
done
