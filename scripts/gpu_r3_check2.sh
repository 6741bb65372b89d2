#!/bin/bash
# r3: the pipelining tests first, then the rest of scripts/gpu_r3_check.sh
set -uo pipefail
OUT=gpurun_out/r3check; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_pipeline.log 2>&1
rc=$?; tail -2 $OUT/pytest_pipeline.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_pipeline.log | head -30; exit $rc; }
exec_check() { bash scripts/gpu_r3_check.sh; }
exec_check
