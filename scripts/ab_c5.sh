#!/bin/bash
# A/B of the C5 raycast between the in-tree library and variants (same box, alternating):
#   scripts/ab_c5.sh <out> <variant lib>...
set -euo pipefail
OUT=${1:?out}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for L in disinfect-slam_amd/libdisinfect_tsdf.so "$@"; do
    tag=$(echo "$L" | tr '/' '_')
    TSDF_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p_${tag}_$rep" -o run \
      -- python3 bench.py --loop c5 --no-cpu --steps 100 > "$OUT/b_${tag}_$rep.log" 2>&1
    echo "$L rep $rep: $(grep -h 'k_raycast' $OUT/p_${tag}_$rep/*kernel_stats.csv | cut -d, -f4)" 
  done
done
