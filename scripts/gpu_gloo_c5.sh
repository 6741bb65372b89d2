#!/bin/bash
# GPU box: 2-rank gloo rehearsals of the sharded C5 loop (both ranks on this GPU), eager and graph.
set -uo pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p $OUT
for g in "" "--graph"; do
  n=c5_gloo2${g:+_graph}
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --backend gloo --loop c5 $g --steps 30 --warmup 5 --secondary none \
    > $OUT/$n.log 2>&1
  rc=$?
  grep '^{' $OUT/$n.log > $OUT/$n.json
  echo "$n rc=$rc $(cut -c1-300 $OUT/$n.json)"
  [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }
done
