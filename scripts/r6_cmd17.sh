cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_graph.py tests/test_gpu_render.py -m gpu > gpurun_out/r6_t17.log 2>&1 || { tail -30 gpurun_out/r6_t17.log; exit 1; }
tail -1 gpurun_out/r6_t17.log
AB_REPS=3 AB_ARGS="--loop c5 --graph" bash scripts/ab.sh env "TSDF_FUSE_VIEW_GRID=0" "TSDF_FUSE_VIEW_GRID=1"
