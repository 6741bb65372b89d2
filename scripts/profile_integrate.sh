#!/bin/bash
# Kernel-trace + PMC passes of one bench command (run on the GPU box from the repo root):
#   scripts/profile_integrate.sh <out_dir> [bench args...]     (default: the bench defaults)
# Pass 1: --kernel-trace --stats. Passes 2/3: one --pmc counter each (FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950), restricted to the frame kernels (k_integrate, k_frame). Every pass runs the same command, so the
# same frames; summarize_prof.py checks that from the bench lines' N_vis / N_upd sums.
set -euo pipefail
OUT=${1:?out dir}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --no-cpu "$@" > "$OUT/trace_bench.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc "$C" --kernel-include-regex "k_integrate|k_frame" \
    --output-format csv -d "$OUT/pmc_$C" -o run \
    -- python3 bench.py --no-cpu "$@" > "$OUT/pmc_${C}_bench.log" 2>&1
done
python3 scripts/summarize_prof.py "$OUT" > "$OUT/summary.txt"
# keep the per-kernel stats, drop the raw per-dispatch CSVs (the whole output must stay small enough to
# come back from the GPU box); KEEP_RAW=1 keeps them
if [ "${KEEP_RAW:-0}" != 1 ]; then
  st=$(find "$OUT/trace" -name '*kernel_stats.csv' -print -quit)
  [ -n "$st" ] && cp "$st" "$OUT/kernel_stats.csv"
  rm -rf "$OUT/trace" "$OUT"/pmc_FETCH_SIZE "$OUT"/pmc_WRITE_SIZE
fi
