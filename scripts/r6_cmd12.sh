cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kg4 -o kg -- python3 bench.py --gpus 1 --steps 64 --warmup 5 --no-cpu --no-cpp-loop --graph --graph-batch 32 > gpurun_out/kg4.json 2> gpurun_out/kg4.err || { tail -20 gpurun_out/kg4.err; exit 1; }
echo "== trace batch 32"; python3 scripts/kgaps.py gpurun_out/kg4 && rm -rf gpurun_out/kg4
for env in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
for args in "--graph --graph-batch 8" "--graph --graph-batch 16" "--graph --graph-batch 32" "" "--loop c5 --graph --graph-batch 32" "--loop c5"; do
  env $env timeout -k 10 300 python bench.py --gpus 1 --steps 64 --warmup 5 --no-cpu --no-cpp-loop $args > gpurun_out/r6_b12.json 2> gpurun_out/r6_b12.err || { tail -5 gpurun_out/r6_b12.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/r6_b12.json') if l.startswith('{')][0])
print('$env', '$args', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
done
done
