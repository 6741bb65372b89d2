#!/bin/bash
# GPU-box evidence runs -- ONE parametrised script (run through gpurun from the repo root):
#   scripts/gpu.sh <tag> <stage> [<stage> ...]        -> gpurun_out/<tag>/
# Stages (each under its own time limit; the first failure ends the run):
#   tests             the whole GPU suite (pytest -m gpu)
#   tests:<file.py>   one GPU test file
#   unpiped           tests/test_gpu_parity.py with TSDF_PIPELINE=0
#   driver            the driver's bench command: bench.py --gpus 1 --steps 20 --warmup 5
#   profile-driver    kernel trace + FETCH_SIZE / WRITE_SIZE PMC passes of the driver command
#                     (scripts/profile_integrate.sh; summary + pmc_entry.json under <tag>/prof_driver)
#   profile-c3|c4|c5|c5graph|c2  the same for those bench lines (default steps) -> <tag>/prof_<name>
#   default           bench.py (300 timed frames, CPU baseline)
#   c5 | c5graph | c4 | c2 | graph   bench.py --loop c5 [--graph] / 1280x720 / --depth-only / --graph
#   c5tests           the raycast / render / C5 GPU tests
#   host-pinned|host-pageable  bench.py --host-frames (C3 frames from host memory through TSDF_MEM_HOST)
#   group8            bench.py --shard 8 --mode sharded --native-group (C3, 8 shards of one tsdf_group on one GPU)
#   shard8            bench.py --width 1280 --height 720 --shard 8 (single-GPU 8-shard rehearsal)
#   sq:<kernel>       SQ counter passes of one kernel on the default command (profile_kernel_sq.sh)
#   c5trace|c5gtrace  kernel trace (eager / graph) of the C5 loop -> per-frame kernel chain and gaps (scripts/chain_timeline.py)
#   raysq             SQ / FETCH / WRITE passes of k_raycast on the C5 loop -> <tag>/r5_raycast_sq.json
#   raydiag           raycast step statistics and wave lifetimes (diagnostic library, scripts/diag_raycast.py)
#   framediag[:A=1,B=2]  k_frame per-part timeline (diagnostic library, scripts/diag_frame.py), optional env
#   abargs:<a1>,<a2>  interleaved A/B of bench arguments (scripts/ab.sh args; spaces as '+', e.g. --loop+c5)
#   ab:<lib1>,<lib2>  interleaved A/B of engine builds on the driver command (scripts/ab.sh lib; the other
#                     A/B forms -- env, tree, c5 -- are run directly; variants: scripts/build_variant.sh)
set -uo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
DRIVER="--gpus 1 --steps 20 --warmup 5"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
fail() { echo "stage $1 failed"; tail -20 "$2"; exit 1; }
line() { python3 - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d.get("roofline", {})
print(sys.argv[1].split("/")[-1], d["value"], d.get("unit"), "ms/step", d.get("ms_per_step"),
      "frac", r.get("frac"), "frame.frac_read", r.get("frame", {}).get("frac_read"), "traffic", r.get("traffic"))
PY
}
for st in "$@"; do
  case $st in
    tests) timeout -k 10 900 $PYT tests -m gpu > $OUT/pytest.log 2>&1 || fail $st $OUT/pytest.log
           tail -1 $OUT/pytest.log ;;
    tests:*) f=${st#tests:}; timeout -k 10 600 $PYT tests/$f -m gpu -v > $OUT/pytest_${f%.py}.log 2>&1 || fail $st $OUT/pytest_${f%.py}.log
           tail -1 $OUT/pytest_${f%.py}.log ;;
    unpiped) TSDF_PIPELINE=0 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu > $OUT/pytest_unpiped.log 2>&1 || fail $st $OUT/pytest_unpiped.log
           tail -1 $OUT/pytest_unpiped.log ;;
    driver) timeout -k 10 300 python3 bench.py $DRIVER > $OUT/bench_driver.json 2> $OUT/bench_driver.err || fail $st $OUT/bench_driver.err
           line $OUT/bench_driver.json ;;
    profile-driver) bash scripts/profile_integrate.sh $OUT/prof_driver $DRIVER || fail $st $OUT/prof_driver/trace_bench.log
           tail -14 $OUT/prof_driver/summary.txt ;;
    profile-c3|profile-c4|profile-c5|profile-c5graph|profile-c2)
           case $st in profile-c3) A="";; profile-c4) A="--width 1280 --height 720";; profile-c5) A="--loop c5";;
                       profile-c5graph) A="--loop c5 --graph";; profile-c2) A="--depth-only";; esac
           bash scripts/profile_integrate.sh $OUT/prof_${st#profile-} $A || fail $st $OUT/prof_${st#profile-}/trace_bench.log
           tail -14 $OUT/prof_${st#profile-}/summary.txt ;;
    default) timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || fail $st $OUT/bench_default.err
           line $OUT/bench_default.json ;;
    c5) timeout -k 10 300 python3 bench.py --no-cpu --loop c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || fail $st $OUT/bench_c5.err
           line $OUT/bench_c5.json ;;
    c5graph) timeout -k 10 300 python3 bench.py --no-cpu --loop c5 --graph > $OUT/bench_c5graph.json 2> $OUT/bench_c5graph.err || fail $st $OUT/bench_c5graph.err
           line $OUT/bench_c5graph.json ;;
    graph) timeout -k 10 300 python3 bench.py --no-cpu --graph > $OUT/bench_graph.json 2> $OUT/bench_graph.err || fail $st $OUT/bench_graph.err
           line $OUT/bench_graph.json ;;
    c4) timeout -k 10 300 python3 bench.py --no-cpu --width 1280 --height 720 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || fail $st $OUT/bench_c4.err
           line $OUT/bench_c4.json ;;
    c2) timeout -k 10 300 python3 bench.py --no-cpu --depth-only > $OUT/bench_c2.json 2> $OUT/bench_c2.err || fail $st $OUT/bench_c2.err
           line $OUT/bench_c2.json ;;
    host-pinned|host-pageable) k=${st#host-}
           timeout -k 10 300 python3 bench.py --no-cpu --host-frames $k > $OUT/bench_host_$k.json 2> $OUT/bench_host_$k.err || fail $st $OUT/bench_host_$k.err
           line $OUT/bench_host_$k.json; grep -o '"host_frames": {[^}]*}' $OUT/bench_host_$k.json ;;
    c5tests) timeout -k 10 600 $PYT tests/test_gpu_c5.py tests/test_gpu_render.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_graph.py -m gpu > $OUT/pytest_c5.log 2>&1 || fail $st $OUT/pytest_c5.log
           tail -1 $OUT/pytest_c5.log ;;
    group8) timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --shard 8 --mode sharded --native-group > $OUT/group8_c3.json 2> $OUT/group8_c3.err || fail $st $OUT/group8_c3.err
           line $OUT/group8_c3.json ;;
    shard8) timeout -k 10 300 python3 bench.py --no-cpu --steps 100 --width 1280 --height 720 --shard 8 > $OUT/shard8_c4.json 2> $OUT/shard8_c4.err || fail $st $OUT/shard8_c4.err
           line $OUT/shard8_c4.json ;;
    c5trace|c5gtrace) g=; [ $st = c5gtrace ] && g=--graph
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$st -o run -- python3 bench.py --no-cpu --loop c5 --steps 120 $g > $OUT/$st.log 2>&1 || fail $st $OUT/$st.log
           python3 scripts/chain_timeline.py $OUT/$st > $OUT/${st}_chain.txt && tail -30 $OUT/${st}_chain.txt ;;
    raysq) bash scripts/profile_kernel_sq.sh $OUT/sq_ray k_raycast --loop c5 --steps 30 > $OUT/sq_ray.txt 2>&1 || fail $st $OUT/sq_ray.txt
           python3 scripts/sq_json.py $OUT/sq_ray k_raycast "python3 bench.py --no-cpu --loop c5 --steps 30" 640 480 > $OUT/r5_raycast_sq.json
           grep -E "VALU_per_wave|SALU_per_wave" $OUT/r5_raycast_sq.json ;;
    sq:*) k=${st#sq:}; bash scripts/profile_kernel_sq.sh $OUT/sq_$k $k > $OUT/sq_$k.txt 2>&1 || fail $st $OUT/sq_$k.txt
           tail -8 $OUT/sq_$k.txt ;;
    raydiag) TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 180 python3 scripts/diag_raycast.py > $OUT/raycast_diag.txt 2>&1 || fail $st $OUT/raycast_diag.txt
           tail -12 $OUT/raycast_diag.txt ;;
    framediag*) e=${st#framediag}; e=${e#:}; f=$OUT/frame_diag${e:+_$e}.txt; env ${e//,/ } TSDF_AMD_LIB=disinfect-slam_amd/libdisinfect_tsdf_diag.so timeout -k 10 120 python3 scripts/diag_frame.py > $f 2>&1 || fail $st $f
           tail -9 $f ;;
    abargs:*) IFS=, read -ra SP <<< "${st#abargs:}"; SP=("${SP[@]//+/ }"); bash scripts/ab.sh args "${SP[@]}" || exit 1 ;;
    ab:*) IFS=, read -ra LIBS <<< "${st#ab:}"; bash scripts/ab.sh lib "${LIBS[@]}" || exit 1 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
