#!/bin/bash
# r3: one-launch frame (sweep first): full GPU suite, unpipelined parity files, A/B vs the tiles-only pipeline
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3one7; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_all.log 2>&1
rc=$?; tail -2 $OUT/pytest_all.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_all.log | head -30; exit $rc; }
TSDF_PIPELINE=0 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_unpipelined.log 2>&1
rc=$?; tail -2 $OUT/pytest_unpipelined.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_unpipelined.log | head -30; exit $rc; }
scripts/ab.sh 300 disinfect-slam_amd/build/var_tiles/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so || exit 1
