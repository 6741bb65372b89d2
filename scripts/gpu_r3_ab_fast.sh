#!/bin/bash
# r3 A/B: commit-all fast resolvers (allocation + carving), ingest occupancy cap, integrate at 7 waves;
# parity of the new build first
set -uo pipefail
OUT=gpurun_out/r3abfast; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
B=disinfect-slam_amd/build
scripts/ab.sh 300 $B/var_base/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so $B/var_nofast/libdisinfect_tsdf.so $B/var_w7/libdisinfect_tsdf.so
