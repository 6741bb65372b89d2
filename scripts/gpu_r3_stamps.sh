#!/bin/bash
# r3: per-phase stamps of the round-2 tree (build/wt_base) and the current tree, C3 stream, frames synchronised
set -uo pipefail
OUT=gpurun_out/r3stamps; mkdir -p $OUT
export TMPDIR=/tmp
ROOTD=$PWD
(cd disinfect-slam_amd/build/wt_base && TSDF_AMD_LIB=$ROOTD/disinfect-slam_amd/build/wt_base/disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_stamps.py > $ROOTD/$OUT/base.txt 2>&1) || { echo base failed; tail $OUT/base.txt; exit 1; }
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_stamps.py > $OUT/cur.txt 2>&1 || { echo cur failed; tail $OUT/cur.txt; exit 1; }
echo done
