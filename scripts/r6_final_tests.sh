cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6f
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=15 tests -m gpu > gpurun_out/r6f/pytest.log 2>&1 || { tail -40 gpurun_out/r6f/pytest.log; exit 1; }
tail -20 gpurun_out/r6f/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6f/smoke.log 2>&1 || { tail -20 gpurun_out/r6f/smoke.log; exit 1; }
tail -2 gpurun_out/r6f/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6f/bench_driver.json 2> gpurun_out/r6f/bench_driver.err || { tail -20 gpurun_out/r6f/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r6f/bench_driver.json') if l.startswith('{')][0])
print('driver', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['roofline']['frac'], d['roofline']['us_per_launch'], d.get('cpp_loop',{}).get('frames_per_s'), d['cpu_baseline'])"
