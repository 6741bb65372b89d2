# full GPU suite + driver bench + smoke on the current tree (round 6)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.json 2> gpurun_out/${TAG}_bench_driver.err || exit 1
tail -c 600 gpurun_out/${TAG}_bench_driver.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/${TAG}_smoke.log
