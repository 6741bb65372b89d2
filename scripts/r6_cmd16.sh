cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for args in "--loop c5 --graph --graph-batch 1" "--loop c5 --graph --graph-batch 16" "--loop c5"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kc$i -o kc -- python3 bench.py --gpus 1 --steps 60 --warmup 5 --no-cpu --no-cpp-loop $args > gpurun_out/kc$i.json 2> gpurun_out/kc$i.err || { tail -20 gpurun_out/kc$i.err; exit 1; }
  echo "== $args"; python3 scripts/kgaps.py gpurun_out/kc$i "k_render_ingest" && python3 scripts/chain_timeline.py gpurun_out/kc$i "k_render_ingest" | tail -12 && rm -rf gpurun_out/kc$i
done
