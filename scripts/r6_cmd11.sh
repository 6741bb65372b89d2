cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for args in "" "--graph" "--graph --graph-batch 8"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kg$i -o kg -- python3 bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu --no-cpp-loop $args > gpurun_out/kg$i.json 2> gpurun_out/kg$i.err || { tail -20 gpurun_out/kg$i.err; exit 1; }
  echo "== $args"; python3 scripts/kgaps.py gpurun_out/kg$i && rm -rf gpurun_out/kg$i
done
