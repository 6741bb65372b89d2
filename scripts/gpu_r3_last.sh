#!/bin/bash
# r3: poll interval of the chained waiters (s_sleep 2 vs 16) and chained order (tiles first) on the
# shipped build
set -uo pipefail
export TMPDIR=/tmp
scripts/ab.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_s2/libdisinfect_tsdf.so disinfect-slam_amd/build/var_tf2/libdisinfect_tsdf.so || exit 1
