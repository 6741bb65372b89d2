#!/bin/bash
# r3 probes (GPU box): tail stamps of the C3 frame, raycast SQ counters and the C5 kernel trace.
set -uo pipefail
OUT=gpurun_out/r3probe
mkdir -p $OUT
export TMPDIR=/tmp
TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_stamps.py > $OUT/stamps.txt 2>&1 || { echo stamps failed; tail $OUT/stamps.txt; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c5trace -o run -- python3 bench.py --no-cpu --loop c5 --steps 100 > $OUT/c5trace.log 2>&1 || { echo c5 trace failed; exit 1; }
bash scripts/profile_kernel_sq.sh $OUT/sq_raycast k_raycast --loop c5 --steps 60 > $OUT/sq_raycast.txt 2>&1 || { echo sq failed; exit 1; }
echo done
