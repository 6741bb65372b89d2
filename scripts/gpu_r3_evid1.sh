#!/bin/bash
# r3 evidence: default bench line, C5 line (raycast entry), kernel traces (csv) of both
set -uo pipefail
OUT=gpurun_out/r3evid1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 200 python3 bench.py --no-cpu --loop c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o run -- python3 bench.py --no-cpu --loop c5 > $OUT/trace_c5.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/trace_c3.log 2>&1 || exit 1
echo done
