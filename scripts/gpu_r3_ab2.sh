#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r3ab2; mkdir -p $OUT
bash scripts/gpu_tests.sh r3ab2 tests || exit 1
bash scripts/ab.sh 300 disinfect-slam_amd/build/var_base/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so > $OUT/ab.txt 2>&1 || exit 1
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_stamps.py > $OUT/stamps.txt 2>&1 || exit 1
echo done
