#!/bin/bash
# r3: chained sweep tested before the carving is published (vis_sweep_chained): pipeline + parity
# tests, chain stamps, A/B against the sweep after the wait
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3pre; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_snapshot.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_chain.py > $OUT/chain.txt 2>&1 || { tail $OUT/chain.txt; exit 1; }
cat $OUT/chain.txt
scripts/ab.sh 300 disinfect-slam_amd/build/var_head/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so || exit 1
