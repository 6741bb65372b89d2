set -uo pipefail
OUT=gpurun_out/r4c; mkdir -p $OUT
bash scripts/gpu.sh r4c tests:test_gpu_pipeline.py tests:test_gpu_graph.py || exit 1
for K in 4 2; do
  TSDF_RAYCAST_SEGS=$K timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_render.py -m gpu > $OUT/pytest_c5_K$K.log 2>&1 || { echo "K=$K tests failed"; tail -30 $OUT/pytest_c5_K$K.log; exit 1; }
  tail -1 $OUT/pytest_c5_K$K.log
done
for K in 1 2 4; do
  TSDF_RAYCAST_SEGS=$K timeout -k 10 300 python3 bench.py --no-cpu --loop c5 --steps 100 --warmup 10 > $OUT/c5_K$K.json 2> $OUT/c5_K$K.err || { tail $OUT/c5_K$K.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/c5_K$K.json').read().splitlines()[-1]); print('K=$K', d['value'], d['raycast']['us_per_call'])"
done
bash scripts/ab_env.sh "TSDF_FRAME_ORDER=0 TSDF_FRAME_WG_PER_CU=7" "TSDF_FRAME_ORDER=0 TSDF_FRAME_WG_PER_CU=4" "TSDF_FRAME_ORDER=1 TSDF_FRAME_WG_PER_CU=7" "TSDF_FRAME_ORDER=1 TSDF_FRAME_WG_PER_CU=4" "TSDF_FRAME_ORDER=2 TSDF_FRAME_WG_PER_CU=5" "TSDF_FRAME_ORDER=0 TSDF_FRAME_WG_PER_CU=5" "TSDF_PIPELINE=0"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_render.py -m gpu -k "eight" > $OUT/pytest_eight.log 2>&1 || { tail -30 $OUT/pytest_eight.log; exit 1; }
tail -1 $OUT/pytest_eight.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py -m gpu -k "pipe" > $OUT/pytest_shardpipe.log 2>&1 || { tail -30 $OUT/pytest_shardpipe.log; exit 1; }
tail -1 $OUT/pytest_shardpipe.log
timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --width 1280 --height 720 --shard 8 --mode sharded > $OUT/shard8_c4_pipe.json 2> $OUT/shard8_c4_pipe.err || { tail $OUT/shard8_c4_pipe.err; exit 1; }
tail -c 600 $OUT/shard8_c4_pipe.json
