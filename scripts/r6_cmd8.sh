cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_facade.py tests/test_gpu_graph.py tests/test_gpu_c5.py tests/test_gpu_sharded.py > gpurun_out/r6_t8.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|Error" gpurun_out/r6_t8.log | tail -70
[ $rc -eq 0 ] || exit $rc
for args in "" "--graph" "--graph --graph-batch 8" "--loop c5" "--loop c5 --graph" "--loop c5 --graph --graph-batch 8"; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu $args > gpurun_out/r6_b8.json 2> gpurun_out/r6_b8.err || { tail -5 gpurun_out/r6_b8.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/r6_b8.json') if l.startswith('{')][0])
print('$args', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('cpp_loop'))"
done
