#!/bin/bash
# GPU box: k_integrate grid (workgroups per CU) against the frame time, unsharded C3 and the C4 8-shard
# rehearsal.  scripts/exp_wgpercu.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
for n in 8 4 2 1; do
  TSDF_INTEGRATE_WG_PER_CU=$n timeout -k 10 120 python3 bench.py --no-cpu --steps 200 2>&1 | grep '^{' > $OUT/c3_wg$n.json
  TSDF_INTEGRATE_WG_PER_CU=$n timeout -k 10 200 python3 bench.py --no-cpu --steps 100 --width 1280 --height 720 --shard 8 2>&1 | grep '^{' > $OUT/c4s8_wg$n.json
  python3 - $OUT $n <<'PY'
import json, sys
o, n = sys.argv[1], sys.argv[2]
a = json.load(open(f"{o}/c3_wg{n}.json")); b = json.load(open(f"{o}/c4s8_wg{n}.json"))
print(f"wg/cu={n} c3 fps={a['value']} integ={a['device_us_per_frame']['integrate']} evt={a['roofline']['us_per_launch']} | c4s8 per-shard={b['value']} ms maxdev={b['max_shard_device_us_per_frame']} integ={b['per_shard_device_us'][0]['integrate']}")
PY
done
