cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A=disinfect-slam_amd/build/var_pk/libdisinfect_tsdf.so
B=disinfect-slam_amd/libdisinfect_tsdf.so
C=disinfect-slam_amd/build/var_raypk/libdisinfect_tsdf.so
AB_REPS=3 AB_ARGS="--loop c5" bash scripts/ab.sh lib $A $B $C || exit 1
AB_REPS=1 bash scripts/ab.sh c5 $A $B $C && rm -rf gpurun_out/ab_c5/p*
