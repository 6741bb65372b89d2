#!/bin/bash
# r3: chained-phase stamps of the one-launch frame; pipeline + snapshot tests after the counter change
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3chain; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_snapshot.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_chain.py > $OUT/chain.txt 2>&1; rc=$?
cat $OUT/chain.txt; exit $rc
