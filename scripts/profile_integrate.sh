#!/bin/bash
# Kernel-trace + PMC passes of the default bench workload (run on the GPU box from the repo root).
#   scripts/profile_integrate.sh <out_dir> [steps]
# Pass 1: --kernel-trace --stats (per-kernel durations). Passes 2/3: one --pmc counter each
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), filtered to the integrate kernel.
set -euo pipefail
OUT=${1:?out dir}
STEPS=${2:-300}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps "$STEPS" > "$OUT/trace_bench.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc "$C" --kernel-include-regex "k_integrate|k_ingest_dda|k_vis|k_resolve" \
    --output-format csv -d "$OUT/pmc_$C" -o run \
    -- python3 bench.py --no-cpu --steps "$STEPS" > "$OUT/pmc_${C}_bench.log" 2>&1
done
python3 scripts/summarize_prof.py "$OUT"
