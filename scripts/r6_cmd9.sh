cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for args in "--shard 8 --mode sharded --native-group" "--shard 8 --mode sharded" "--shard 2 --mode sharded --native-group" "--shard 1 --mode sharded --native-group"; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 5 --no-cpu $args > gpurun_out/r6_b9.json 2> gpurun_out/r6_b9.err || { tail -20 gpurun_out/r6_b9.err; exit 1; }
  echo "== $args"; grep '^{' gpurun_out/r6_b9.json | tee -a gpurun_out/r6_rehearsal.jsonl
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/r6_b9d.json 2> gpurun_out/r6_b9d.err || { tail -20 gpurun_out/r6_b9d.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r6_b9d.json') if l.startswith('{')][0])
print('driver', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('cpp_loop'))"
