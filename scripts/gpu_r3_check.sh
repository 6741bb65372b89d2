#!/bin/bash
# r3: GPU suite with pipelined frames (default) + the unpipelined parity subset, then the default bench
# and the C5 line
set -uo pipefail
OUT=gpurun_out/r3check; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_PIPELINE=0 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_nopipe.log 2>&1
rc=$?; tail -2 $OUT/pytest_nopipe.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_nopipe.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
head -c 400 $OUT/bench_default.json; echo
timeout -k 10 200 python3 bench.py --no-cpu --loop c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 1; }
head -c 300 $OUT/bench_c5.json; echo
