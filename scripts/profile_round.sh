#!/bin/bash
# One round's profile set (run on the GPU box from the repo root):
#   scripts/profile_round.sh <tag>   -> gpurun_out/prof_<tag>/ (trace + FETCH/WRITE + SQ passes)
set -euo pipefail
TAG=${1:?tag}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 200 python3 bench.py > "$OUT/bench_plain.log" 2>&1
bash scripts/profile_integrate.sh "$OUT"
bash scripts/profile_sq.sh "$OUT" 60
python3 scripts/summarize_prof.py "$OUT" > "$OUT/summary.txt"
python3 scripts/summarize_sq.py "$OUT" >> "$OUT/summary.txt" || true
