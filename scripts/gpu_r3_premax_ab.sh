#!/bin/bash
# r3: A/B of the pre-carving sweep (main), its fallback forced on most workgroups (kPreMax 16) and
# the committed one-launch build before the pre-carving sweep
set -uo pipefail
export TMPDIR=/tmp
scripts/ab.sh 300 disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_premax16/libdisinfect_tsdf.so disinfect-slam_amd/build/var_head/libdisinfect_tsdf.so || exit 1
