cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_facade.py tests/test_gpu_c5.py tests/test_gpu_graph.py tests/test_gpu_sharded.py > gpurun_out/r6_t6.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|Error|error" gpurun_out/r6_t6.log | tail -50
exit $rc
