#!/bin/bash
# r3 state check: the whole GPU suite, then the default bench line
set -uo pipefail
OUT=gpurun_out/r3state; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
head -c 600 $OUT/bench_default.json
