#!/bin/bash
# r3: chained order (sweep first / tiles first) and update grid, with the pre-carving sweep
set -uo pipefail
export TMPDIR=/tmp
scripts/ab.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_tf/libdisinfect_tsdf.so || exit 1
scripts/ab_env.sh 300 disinfect-slam_amd/build/var_tf/libdisinfect_tsdf.so TSDF_INTEGRATE_WG_PER_CU=6 || exit 1
scripts/ab_env.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so TSDF_INTEGRATE_WG_PER_CU=6 || exit 1
