#!/bin/bash
# r3: pipelining tests, whole GPU suite, unpipelined parity subset, A/B of the prepared sweep
# (current) against the tiles-only pipeline (var_tiles), then the default bench line and C5
set -uo pipefail
OUT=gpurun_out/r3sweep; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_pipeline.log 2>&1
rc=$?; tail -2 $OUT/pytest_pipeline.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_pipeline.log | head -30; exit $rc; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_PIPELINE=0 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_nopipe.log 2>&1
rc=$?; tail -2 $OUT/pytest_nopipe.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_nopipe.log | head -30; exit $rc; }
scripts/ab.sh 300 disinfect-slam_amd/build/var_tiles/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
head -c 300 $OUT/bench_default.json; echo
timeout -k 10 200 python3 bench.py --no-cpu --loop c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 1; }
head -c 300 $OUT/bench_c5.json; echo
