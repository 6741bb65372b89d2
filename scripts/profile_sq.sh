#!/bin/bash
# SQ (shader sequencer) counters of the engine kernels, one pass per counter group.
#   scripts/profile_sq.sh <out_dir> [steps]
set -euo pipefail
OUT=${1:?out dir}
STEPS=${2:-60}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for GROUP in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $GROUP --kernel-include-regex "tsdf::" --output-format csv \
    -d "$OUT/sq$i" -o run -- python3 bench.py --no-cpu --steps "$STEPS" > "$OUT/sq${i}_bench.log" 2>&1 || echo "group $i failed"
done
