#!/bin/bash
# Round-5 GPU session T: the GPU suite with the latency kernel off (CPZ_WIDE_MAX=0: every small
# launch on k_verify_small) and with the copies back (CPZ_ZERO_COPY=0), then three default
# bench runs without extras for the headline's spread.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
CPZ_WIDE_MAX=0 CPZ_ZERO_COPY=0 timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_t.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_t.log | head -20; tail -30 gpurun_out/gpu_all_t.log; exit 1; }
tail -1 gpurun_out/gpu_all_t.log
for k in 1 2 3; do
  timeout -k 10 600 python bench.py --extras 0 > gpurun_out/bench_t$k.json 2> gpurun_out/bench_t.err || { tail -20 gpurun_out/bench_t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_t$k.json'))
print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'], 'cpu', d['cpu_baseline']['value'])"
done
