#!/bin/bash
# GPU box: sharded-volume rehearsals (G shard engines on one GPU) next to the unsharded frame.
#   scripts/gpu_shard_rehearsal.sh <tag> [G]  -> gpurun_out/<tag>/
set -uo pipefail
TAG=${1:?tag}; G=${2:-8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { timeout -k 10 300 python3 bench.py --no-cpu "$@" 2>&1 | grep '^{' ; }
run --steps 100 --width 1280 --height 720 > $OUT/c4_unsharded.json || exit 1
run --steps 100 --width 1280 --height 720 --shard $G > $OUT/c4_shard$G.json || exit 1
run --steps 100 --shard $G > $OUT/c3_shard$G.json || exit 1
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read())
    print(f.split("/")[-1], d["value"], d["unit"], d.get("ms_per_step"), d.get("max_shard_device_us_per_frame"),
          d.get("device_us_per_frame") or [ {k: v for k, v in s.items()} for s in d.get("per_shard_device_us", [])][:2])
PY
