set -uo pipefail
mkdir -p gpurun_out/spg
for k in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --no-cpu --streams-per-gpu $k > gpurun_out/spg/k$k.log 2>&1 || { echo "k=$k failed"; tail -5 gpurun_out/spg/k$k.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/spg/k$k.log') if l.startswith('{')][0]); r=d['roofline']
print('k=$k', d['value'], d['ms_per_step'], r['us_per_launch'], r['frac'], d['status'])"
done
