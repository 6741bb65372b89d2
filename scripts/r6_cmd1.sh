cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_numerics.py tests/test_gpu_golden.py tests/test_gpu_semantic.py tests/test_gpu_parity.py > gpurun_out/r6_t1.log 2>&1
rc=$?
tail -5 gpurun_out/r6_t1.log
[ $rc -eq 0 ] || exit $rc
AB_REPS=2 timeout -k 10 900 scripts/ab.sh lib disinfect-slam_amd/build/var_head/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so disinfect-slam_amd/build/var_w6/libdisinfect_tsdf.so disinfect-slam_amd/build/var_w5/libdisinfect_tsdf.so > gpurun_out/r6_ab1.log 2>&1
cat gpurun_out/r6_ab1.log
