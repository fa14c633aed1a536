#!/bin/bash
# Round-5 GPU session: sustained headline -- the default bench line's workload timed over 50,
# 200 and 1000 steps (~1, 4 and 20 s of back-to-back launches) on one box.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 50 200 1000; do
  timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu-baseline --extras 0 > gpurun_out/soak_$k.json 2> gpurun_out/soak.err || { tail -5 gpurun_out/soak.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/soak_$k.json')); r=d['roofline']
print('steps $k', round(d['value']/1e6,2), 'M proofs/s, ms/step', round(d['ms_per_step'],3), 'frac', round(r['frac'],4), 'kernel clock', r.get('peak_clock_ghz'))" | tee -a gpurun_out/soak.txt
done
