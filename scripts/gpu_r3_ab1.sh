#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r3ab1; mkdir -p $OUT
bash scripts/gpu_tests.sh r3ab1 tests || exit 1
bash scripts/ab.sh 300 disinfect-slam_amd/build/var_base/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so > $OUT/ab.txt 2>&1 || exit 1
bash scripts/ab_env.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so TSDF_INTEGRATE_WG_PER_CU=8 TSDF_INTEGRATE_WG_PER_CU=7 TSDF_INTEGRATE_WG_PER_CU=6 TSDF_INTEGRATE_WG_PER_CU=4 > $OUT/wgpercu.txt 2>&1 || exit 1
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_stamps.py > $OUT/stamps.txt 2>&1 || exit 1
TSDF_AMD_LIB=disinfect-slam_amd/build/diag16/libdisinfect_tsdf.so timeout -k 10 120 python3 scripts/diag_stamps.py > $OUT/stamps16.txt 2>&1 || exit 1
echo done
