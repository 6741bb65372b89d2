#!/bin/bash
# r3: update grid of the one-launch frame (WGs per CU left to the chained work) x chained order; chain stamps
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3grid; mkdir -p $OUT
scripts/ab_env.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so TSDF_INTEGRATE_WG_PER_CU=7 TSDF_INTEGRATE_WG_PER_CU=6 TSDF_INTEGRATE_WG_PER_CU=5 || exit 1
scripts/ab_env.sh 300 disinfect-slam_amd/build/var_tf/libdisinfect_tsdf.so TSDF_INTEGRATE_WG_PER_CU=7 TSDF_INTEGRATE_WG_PER_CU=6 TSDF_INTEGRATE_WG_PER_CU=5 || exit 1
for g in 7 6; do
TSDF_INTEGRATE_WG_PER_CU=$g TSDF_AMD_LIB=disinfect-slam_amd/build/var_cdiag/libdisinfect_tsdf.so timeout -k 10 120 python3 bench.py --no-cpu > $OUT/cdiag_$g.json 2>/dev/null || exit 1
python3 -c "
import json,sys; d=json.loads([l for l in open('$OUT/cdiag_$g.json') if l.startswith('{')][-1]); print('cdiag $g', d['value'], {k:v for k,v in d['device_us_per_frame'].items() if k!='note'})"
done
