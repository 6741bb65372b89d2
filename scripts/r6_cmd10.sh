cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_group.py > gpurun_out/r6_t10.log 2>&1 || { tail -30 gpurun_out/r6_t10.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r6_t10.log
for args in "--shard 1 --mode sharded --native-group" "--shard 4 --mode sharded --native-group"; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 5 --no-cpu $args > gpurun_out/r6_b10.json 2> gpurun_out/r6_b10.err || { tail -20 gpurun_out/r6_b10.err; exit 1; }
  echo "== $args"; grep '^{' gpurun_out/r6_b10.json >> gpurun_out/r6_rehearsal.jsonl
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r6_b10.json') if l.startswith('{')][0]); print(d['group_ms_per_frame'], d['value'], d['max_shard_device_us_per_frame'])"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/r6_b10d.json 2> gpurun_out/r6_b10d.err || { tail -20 gpurun_out/r6_b10d.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r6_b10d.json') if l.startswith('{')][0])
print('driver', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('cpp_loop'))"
