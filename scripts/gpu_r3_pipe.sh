#!/bin/bash
# r3: parity of the fast resolvers (default) and of pipelined frames (TSDF_PIPELINE=1), then A/B
set -uo pipefail
OUT=gpurun_out/r3pipe; mkdir -p $OUT
export TMPDIR=/tmp
B=disinfect-slam_amd/build
L=disinfect-slam_amd/libdisinfect_tsdf.so
scripts/ab.sh 300 $B/var_nofast/libdisinfect_tsdf.so $L || exit 1
scripts/ab_env.sh 300 $L TSDF_PIPELINE=1 || exit 1
scripts/ab_env.sh 300 $B/var_w7/libdisinfect_tsdf.so TSDF_PIPELINE=1 || exit 1
scripts/ab_env.sh 300 $B/var_w6/libdisinfect_tsdf.so TSDF_PIPELINE=1 || exit 1
