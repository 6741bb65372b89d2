#!/bin/bash
# r3: 64 copies of the carving-published flag vs 8: pipelining tests, chain stamps, A/B
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3flags; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_chain.py > $OUT/chain.txt 2>&1 || { tail $OUT/chain.txt; exit 1; }
head -5 $OUT/chain.txt
scripts/ab.sh 300 disinfect-slam_amd/build/var_f8/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so || exit 1
