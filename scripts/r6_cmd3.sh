cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_semantic.py -k "160 or golden" > gpurun_out/r6_t3.log 2>&1
rc=$?
tail -2 gpurun_out/r6_t3.log
[ $rc -eq 0 ] || exit $rc
B=disinfect-slam_amd/build
AB_REPS=2 timeout -k 10 900 scripts/ab.sh lib $B/var_head/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so $B/var_w6/libdisinfect_tsdf.so $B/var_w5/libdisinfect_tsdf.so $B/var_nochain/libdisinfect_tsdf.so $B/var_nochain6/libdisinfect_tsdf.so > gpurun_out/r6_ab3.log 2>&1
cat gpurun_out/r6_ab3.log
