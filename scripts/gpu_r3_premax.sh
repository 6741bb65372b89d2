#!/bin/bash
# r3: the chained sweep's fallback (a wave with more than kPreMax live entries waits and sweeps at
# agent scope) exercised by a build with kPreMax = 16: the pipelining and parity tests on it
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3premax; mkdir -p $OUT
TSDF_AMD_LIB=disinfect-slam_amd/build/var_premax16/libdisinfect_tsdf.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_AMD_LIB=disinfect-slam_amd/build/var_premax16/libdisinfect_tsdf.so timeout -k 10 120 python3 bench.py --no-cpu --steps 200 > $OUT/bench.json 2>/dev/null || exit 1
head -c 150 $OUT/bench.json; echo
