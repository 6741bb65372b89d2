cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A=disinfect-slam_amd/build/var_pk/libdisinfect_tsdf.so
B=disinfect-slam_amd/libdisinfect_tsdf.so
AB_REPS=2 bash scripts/ab.sh lib $A $B || exit 1
for args in "--loop c5" "--width 1280 --height 720" "--depth-only"; do
  echo "== $args"; AB_REPS=2 AB_ARGS="$args" bash scripts/ab.sh lib $A $B || exit 1
done
AB_REPS=1 bash scripts/ab.sh c5 $A $B && rm -rf gpurun_out/ab_c5/p*
