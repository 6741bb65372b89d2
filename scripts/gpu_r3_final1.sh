#!/bin/bash
# r3 evidence of the pipelined build: GPU suite (+ unpipelined parity subset), kernel trace + PMC
# passes of the default bench command, SQ counters of k_integrate_pre, C5 line
set -uo pipefail
OUT=gpurun_out/r3final; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TSDF_PIPELINE=0 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_nopipe.log 2>&1
rc=$?; tail -2 $OUT/pytest_nopipe.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_nopipe.log | head -30; exit $rc; }
bash scripts/profile_integrate.sh $OUT/prof || { echo profile failed; exit 1; }
tail -12 $OUT/prof/summary.txt
bash scripts/profile_kernel_sq.sh $OUT/sq k_integrate_pre > $OUT/sq.txt 2>&1 || { echo sq failed; tail $OUT/sq.txt; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu --loop c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 1; }
echo done
