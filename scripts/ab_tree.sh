#!/bin/bash
# A/B of whole trees (an older round's bench.py + package + built library staged under abtree/<name>,
# git-ignored) against this tree, on the driver's bench command, interleaved, each run twice:
#   scripts/ab_tree.sh "<label>:<dir>:<ENV=a ...>[:<extra bench args>]" ...      (dir "." = this tree)
set -uo pipefail
OUT=gpurun_out/ab_tree
mkdir -p $OUT
for rep in 1 2; do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    IFS=: read -r label dir envs extra <<< "$spec"
    log=$PWD/$OUT/t${i}_$rep.log
    (cd "$dir" && env $envs timeout -k 10 120 python3 bench.py --no-cpu --gpus 1 --steps 20 --warmup 5 $extra > "$log" 2>&1) || { echo "$label failed"; tail -5 "$log"; exit 1; }
    python3 - "$log" "$label" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
dv = {k: v for k, v in d.get('device_us_per_frame', {}).items() if k != 'note'}
print(f"{sys.argv[2]:>14} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} dev={dv}")
PY
  done
done
