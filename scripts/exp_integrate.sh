#!/bin/bash
# Timing study of the integrate kernel variants (disinfect-slam_amd/Makefile exp targets).
set -uo pipefail
OUT=gpurun_out/exp
mkdir -p $OUT
for v in base 1 2 4 7; do
  if [ $v = base ]; then lib=disinfect-slam_amd/libdisinfect_tsdf.so; else lib=disinfect-slam_amd/libdisinfect_tsdf_exp$v.so; fi
  TSDF_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --steps 150 > $OUT/exp_$v.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/exp_$v.log') if l.startswith('{')][0]); print('$v', d['roofline']['us_per_launch'], d['avg_visible_blocks'], d['avg_updated_voxels'], d['device_us_per_frame'])"
done
