cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_render.py tests/test_gpu_parity.py tests/test_gpu_graph.py -m gpu > gpurun_out/r6_t13.log 2>&1 || { tail -30 gpurun_out/r6_t13.log; exit 1; }
tail -1 gpurun_out/r6_t13.log
AB_REPS=2 bash scripts/ab.sh c5 disinfect-slam_amd/build/var_nojump/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so && rm -rf gpurun_out/ab_c5/p*
AB_REPS=2 AB_ARGS="--loop c5" bash scripts/ab.sh lib disinfect-slam_amd/build/var_nojump/libdisinfect_tsdf.so disinfect-slam_amd/libdisinfect_tsdf.so
