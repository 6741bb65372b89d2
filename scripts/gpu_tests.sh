#!/bin/bash
# GPU box: selected GPU tests.  scripts/gpu_tests.sh <tag> <pytest args...>  -> gpurun_out/<tag>/
set -uo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || grep -E "^E |FAILED" $OUT/pytest.log | head -30
exit $rc
