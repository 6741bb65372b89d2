#!/bin/bash
# Same-box interleaved A/B runs (GPU box, repo root; every setting run twice, alternating):
#   scripts/ab.sh env  "<ENV=a ENV2=b>" ...        engine environment settings on the driver's command
#                                                  (AB_ARGS: extra bench arguments, e.g. "--width 1280 --height 720")
#   scripts/ab.sh lib  <lib.so> ...                engine builds (scripts/build_variant.sh) on the driver's command
#   scripts/ab.sh tree "<label>:<dir>:<ENV=a ...>[:<extra args>]" ...
#                                                  whole trees (an older round's bench.py + package + library
#                                                  staged under abtree/<name>, git-ignored; dir "." = this tree)
#   scripts/ab.sh args "<bench args>" ...          bench arguments on the driver's command (e.g. "--loop c5 --no-defer")
#   scripts/ab.sh c5   <lib.so> ...                k_raycast kernel time (kernel trace) on the C5 loop
#                                                  (pass disinfect-slam_amd/libdisinfect_tsdf.so for this tree's)
set -uo pipefail
MODE=${1:?mode}; shift
OUT=gpurun_out/ab_$MODE
mkdir -p $OUT
export TMPDIR=/tmp
DRIVER="--no-cpu --gpus 1 --steps 20 --warmup 5"
show() {  # <log> <label>
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
dv = {k: v for k, v in d.get('device_us_per_frame', {}).items() if k != 'note'}
r = d.get('roofline', {})
print(f"{sys.argv[2]:>40} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} launch={r.get('us_per_launch')}us dev={dv}")
PY
}
for rep in $(seq 1 ${AB_REPS:-2}); do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    log=$PWD/$OUT/r${i}_$rep.log
    case $MODE in
      env) env $spec timeout -k 10 120 python3 bench.py $DRIVER ${AB_ARGS:-} > $log 2>&1 || { echo "$spec failed"; tail -5 $log; exit 1; }
           show $log "$spec" ;;
      args) timeout -k 10 120 python3 bench.py $DRIVER $spec > $log 2>&1 || { echo "$spec failed"; tail -5 $log; exit 1; }
           show $log "$spec" ;;
      lib) TSDF_AMD_LIB=$spec timeout -k 10 120 python3 bench.py $DRIVER ${AB_ARGS:-} > $log 2>&1 || { echo "$spec failed"; tail -5 $log; exit 1; }
           show $log "$spec" ;;
      tree) IFS=: read -r label dir envs extra <<< "$spec"
            (cd "$dir" && env $envs timeout -k 10 120 python3 bench.py $DRIVER $extra > "$log" 2>&1) || { echo "$label failed"; tail -5 "$log"; exit 1; }
            show $log "$label" ;;
      c5) L=$spec
          TSDF_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p${i}_$rep" -o run \
            -- python3 bench.py --loop c5 --no-cpu --steps 100 > "$log" 2>&1 || { echo "$L failed"; tail -5 $log; exit 1; }
          python3 - "$OUT/p${i}_$rep" "$L" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_raycast" in r["Name"][:40]:
        print(f"{sys.argv[2]:>60} k_raycast avg {float(r['AverageNs']) / 1e3:.1f} us over {r['Calls']} calls")
PY
          ;;
      *) echo "unknown mode $MODE"; exit 2 ;;
    esac
  done
done
