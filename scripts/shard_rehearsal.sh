#!/bin/bash
# Single-GPU rehearsal of --mode sharded (GPU box): the unsharded rate and each shard of G alone,
# at the given resolution. The G-GPU sharded rate is bounded by the slowest shard.
#   scripts/shard_rehearsal.sh <G> <width> <height> [steps]
set -uo pipefail
G=$1; W=$2; H=$3; STEPS=${4:-300}
OUT=gpurun_out/shard_${W}x${H}
mkdir -p $OUT
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
r = d['roofline']
print(f"{sys.argv[2]:>8} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} integ={r['us_per_launch']:.2f}us "
      f"vis={d['avg_visible_blocks']:.0f} upd={d['avg_updated_voxels']:.0f} active={d['active_blocks']} phases={d['phases_ms_per_frame']}")
PY
}
timeout -k 10 150 python3 bench.py --no-cpu --width $W --height $H --steps $STEPS > $OUT/full.log 2>&1 || exit 1
summ $OUT/full.log full
for ((i = 0; i < G; i++)); do
  timeout -k 10 150 python3 bench.py --no-cpu --width $W --height $H --steps $STEPS --mode sharded --shard $i/$G > $OUT/shard$i.log 2>&1 || { tail -5 $OUT/shard$i.log; exit 1; }
  summ $OUT/shard$i.log "$i/$G"
done
