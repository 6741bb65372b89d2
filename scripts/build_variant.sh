#!/bin/bash
# Build an experiment variant of the engine library with extra compile flags (CPU container):
#   scripts/build_variant.sh <name> "<flags>"  ->  disinfect-slam_amd/build/var_<name>/libdisinfect_tsdf.so
set -euo pipefail
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../disinfect-slam_amd"
OUT=build/var_$NAME
mkdir -p $OUT
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function ${NOPK--Xclang -target-feature -Xclang -packed-fp32-ops} -I../include -Icsrc $FLAGS"
pids=()
for f in csrc/tsdf_alloc.hip csrc/tsdf_fuse.hip csrc/tsdf_extract.hip csrc/tsdf_mesh.hip csrc/tsdf_frontend.hip csrc/tsdf_engine.hip csrc/tsdf_group.hip; do
  /opt/rocm/bin/hipcc $HIPFLAGS -c $f -o $OUT/$(basename $f .hip).o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libdisinfect_tsdf.so $OUT/*.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx
echo $OUT/libdisinfect_tsdf.so
