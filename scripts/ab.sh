#!/bin/bash
# A/B timing of engine library builds on the default bench workload (run on the GPU box):
#   scripts/ab.sh <steps> lib1.so lib2.so ...   (each run twice, interleaved)
set -uo pipefail
STEPS=$1; shift
OUT=gpurun_out/ab
mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    n=$(echo "${lib%.so}" | tr "/" "_")
    TSDF_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --steps $STEPS > $OUT/${n}_$rep.log 2>&1 || { echo "$n failed"; tail -5 $OUT/${n}_$rep.log; exit 1; }
    python3 - "$OUT/${n}_$rep.log" "$n" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
r = d['roofline']
print(f"{sys.argv[2]:>10} fps={d['value']:9.1f} ms/step={d['ms_per_step']:.4f} integ_evt={r['us_per_launch']:.2f}us dev={r.get('us_per_launch_device_clock')}us frac={r['frac']:.3f} dev={d['device_us_per_frame']}")
PY
  done
done
