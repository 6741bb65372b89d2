#!/bin/bash
set -uo pipefail
bash scripts/ab.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_arr64/libdisinfect_tsdf.so || exit 1
for lib in disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_arr64/libdisinfect_tsdf.so; do
  TSDF_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 100 --width 1280 --height 720 --shard 8 2>&1 | grep '^{' | python3 -c "
import json,sys; b=json.loads(sys.stdin.read()); print('$lib'.split('/')[-2], 'c4s8 per-shard', b['value'], 'maxdev', b['max_shard_device_us_per_frame'], b['per_shard_device_us'][0])"
done
bash scripts/exp_wgpercu.sh r3f
