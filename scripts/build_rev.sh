#!/bin/bash
# Build the engine library of an earlier revision for same-box A/B runs (CPU container):
#   scripts/build_rev.sh <git-rev> <name> ["<extra flags>"]  ->  disinfect-slam_amd/build/var_<name>/libdisinfect_tsdf.so
# (the C ABI must match the current Python mirror's; the sources come from `git archive`)
set -euo pipefail
REV=$1; NAME=$2; FLAGS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" disinfect-slam_amd/csrc include | tar -x -C "$TMP"
OUT=$ROOT/disinfect-slam_amd/build/var_$NAME
mkdir -p "$OUT"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-function -I$TMP/include -I$TMP/disinfect-slam_amd/csrc $FLAGS"
pids=()
for f in tsdf_alloc tsdf_fuse tsdf_extract tsdf_mesh tsdf_frontend tsdf_engine; do
  /opt/rocm/bin/hipcc $HIPFLAGS -c "$TMP/disinfect-slam_amd/csrc/$f.hip" -o "$OUT/$f.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libdisinfect_tsdf.so" "$OUT"/*.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx
rm -rf "$TMP" "$OUT"/*.o
echo "$OUT/libdisinfect_tsdf.so"
