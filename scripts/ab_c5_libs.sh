#!/bin/bash
# C5 A/B of engine library builds (GPU box), each run twice, interleaved:
#   scripts/ab_c5_libs.sh <steps> lib1.so lib2.so ...
set -uo pipefail
STEPS=$1; shift
OUT=gpurun_out/ab_c5
mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    n=$(echo "${lib%.so}" | tr "/" "_")
    TSDF_AMD_LIB=$lib timeout -k 10 150 python3 bench.py --no-cpu --loop c5 --steps $STEPS > $OUT/${n}_$rep.log 2>&1 || { echo "$n failed"; tail -5 $OUT/${n}_$rep.log; exit 1; }
    python3 - "$OUT/${n}_$rep.log" "$n" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
r = d.get('raycast', {})
print(f"{sys.argv[2][-40:]:>40} fps={d['value']:8.1f} ms/step={d['ms_per_step']:.4f} raycast_call={r.get('us_per_call')}us")
PY
  done
done
