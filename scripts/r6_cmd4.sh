cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=disinfect-slam_amd/build
TSDF_AMD_LIB=$B/var_f6/libdisinfect_tsdf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_semantic.py -k "160 or golden" > gpurun_out/r6_t4.log 2>&1
rc=$?
tail -2 gpurun_out/r6_t4.log
[ $rc -eq 0 ] || exit $rc
AB_REPS=2 timeout -k 10 900 scripts/ab.sh lib $B/var_f7/libdisinfect_tsdf.so $B/var_f6/libdisinfect_tsdf.so $B/var_f5/libdisinfect_tsdf.so > gpurun_out/r6_ab4.log 2>&1
cat gpurun_out/r6_ab4.log
AB_REPS=1 TSDF_AMD_LIB=$B/var_f6/libdisinfect_tsdf.so timeout -k 10 900 scripts/ab.sh env "TSDF_FRAME_UPD_WGS=512" "TSDF_FRAME_UPD_WGS=768" "TSDF_FRAME_UPD_WGS=896" "TSDF_FRAME_UPD_WGS=1024" "TSDF_FRAME_UPD_WGS=1280" > gpurun_out/r6_ab4b.log 2>&1
cat gpurun_out/r6_ab4b.log
