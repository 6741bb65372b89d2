#!/bin/bash
# r3: nofast without the ingest cap (full-ingest regression), integrate / pre kernel occupancy, pipelining
set -uo pipefail
export TMPDIR=/tmp
B=disinfect-slam_amd/build
L=disinfect-slam_amd/libdisinfect_tsdf.so
scripts/ab.sh 300 $B/var_nfa0/libdisinfect_tsdf.so $L $B/var_w7/libdisinfect_tsdf.so || exit 1
for lib in $L $B/var_w7/libdisinfect_tsdf.so $B/var_p7/libdisinfect_tsdf.so $B/var_p6/libdisinfect_tsdf.so; do
  echo "== $lib"
  scripts/ab_env.sh 300 $lib TSDF_PIPELINE=1 || exit 1
done
