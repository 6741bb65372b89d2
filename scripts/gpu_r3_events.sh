#!/bin/bash
# r3: HIP-event kernel timing vs the kernel trace for the pipelined launch (event cadence 1 / 8 / none)
set -uo pipefail
OUT=gpurun_out/r3events; mkdir -p $OUT
export TMPDIR=/tmp
for ev in 1 8 0; do
  if [ $ev = 0 ]; then A="--no-events"; else A="--event-every $ev"; fi
  timeout -k 10 200 python3 bench.py --no-cpu $A > $OUT/bench_$ev.json 2>/dev/null || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$ev -o run -- python3 bench.py --no-cpu $A > $OUT/trace_$ev.log 2>&1 || exit 1
  python3 - $OUT $ev <<'PY'
import json, sys, glob, csv, statistics
out, ev = sys.argv[1], sys.argv[2]
b = json.loads(open(f"{out}/bench_{ev}.json").read().strip().splitlines()[-1])
t = glob.glob(f"{out}/trace_{ev}/**/*kernel_trace.csv", recursive=True)[0]
d = sorted((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(t)) if "k_integrate_pre" in r["Kernel_Name"])
w = [x for _, x in d[-299:]]
print(f"event_every={ev}: {b['value']:.0f} fps, bench us_per_launch {b['roofline']['us_per_launch']}, trace k_integrate_pre window avg {statistics.mean(w)/1e3:.2f} us; every 8th {statistics.mean(w[7::8])/1e3:.2f}")
PY
done
