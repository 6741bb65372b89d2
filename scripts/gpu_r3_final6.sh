#!/bin/bash
# r3 evidence of the one-launch frame with the pre-carving sweep: GPU suite (+ unpipelined parity), kernel trace + PMC passes of the default bench command, SQ
# counters of k_integrate_pre, default line with the CPU baseline, unpipelined line, C5, C4 unsharded,
# 8-shard C4 rehearsal, chained-phase stamps (diagnostic library)
set -uo pipefail
OUT=gpurun_out/r3final6; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_all.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_all.log | head -30; exit 1; }
tail -1 $OUT/pytest_all.log
TSDF_PIPELINE=0 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_unpipelined.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_unpipelined.log | head -30; exit 1; }
tail -1 $OUT/pytest_unpipelined.log
bash scripts/profile_integrate.sh $OUT/prof || { echo profile failed; exit 1; }
tail -12 $OUT/prof/summary.txt
bash scripts/profile_kernel_sq.sh $OUT/sq k_integrate_pre > $OUT/sq.txt 2>&1 || { echo sq failed; tail $OUT/sq.txt; exit 1; }
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
TSDF_PIPELINE=0 timeout -k 10 200 python3 bench.py --no-cpu > $OUT/bench_unpipelined.json 2>/dev/null || exit 1
timeout -k 10 200 python3 bench.py --no-cpu --loop c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu --width 1280 --height 720 > $OUT/bench_c4.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --width 1280 --height 720 --shard 8 > $OUT/rehearsal_c4_8shards.json 2>/dev/null || exit 1
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_chain.py > $OUT/chain_stamps.txt 2>&1 || exit 1
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], d["value"], d.get("ms_per_step"), d.get("roofline", {}).get("frac"))
PY
