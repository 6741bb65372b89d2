cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_semantic.py -k "160 or golden" > gpurun_out/r6_t2.log 2>&1
rc=$?
tail -3 gpurun_out/r6_t2.log
[ $rc -eq 0 ] || exit $rc
AB_REPS=2 timeout -k 10 600 scripts/ab.sh lib disinfect-slam_amd/build/var_head/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_w6/libdisinfect_tsdf.so > gpurun_out/r6_ab2.log 2>&1
cat gpurun_out/r6_ab2.log
