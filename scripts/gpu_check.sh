#!/bin/bash
# GPU box: the GPU test suite, then an interleaved A/B of engine builds on the default bench.
#   scripts/gpu_check.sh <tag> [lib.so ...]   -> gpurun_out/<tag>/
set -uo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; exit $rc; }
[ $# -gt 0 ] && bash scripts/ab.sh 300 "$@" 2>&1 | tee $OUT/ab.txt
exit 0
