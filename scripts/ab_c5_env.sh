#!/bin/bash
# GPU box: C5 loop A/B of environment settings (interleaved, twice).  scripts/ab_c5_env.sh <steps> VAR=a VAR=b ...
set -uo pipefail
STEPS=$1; shift
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for kv in "$@"; do
    env "$kv" timeout -k 10 200 python3 bench.py --no-cpu --loop c5 --steps $STEPS 2>&1 | grep '^{' > gpurun_out/ab/c5_${kv}_$rep.json || { echo "$kv failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab/c5_${kv}_$rep.json')); print('$kv', 'fps', d['value'], 'ms', d['ms_per_step'], 'integ_dev', d['device_us_per_frame']['integrate'])"
  done
done
