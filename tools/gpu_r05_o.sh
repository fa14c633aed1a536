#!/bin/bash
# Round-5 GPU session O: where a one-proof synchronous call's time goes outside the kernel --
# rocprofv3 kernel + HIP runtime trace of repeated n = 1 cpz_verify_each calls (no counters) --
# and two longer default bench runs (100 steps) for the line's spread.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out/trace_o
N=1 MODE=each timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/trace_o -o sb -- python3 tools/sb_trace.py > gpurun_out/trace_o.log 2>&1 || { tail -20 gpurun_out/trace_o.log; exit 1; }
tail -2 gpurun_out/trace_o.log
find gpurun_out/trace_o -name "*.csv" | head
for k in 1 2; do
  timeout -k 10 900 python bench.py --steps 100 --warmup 5 --extras 0 > gpurun_out/bench_o$k.json 2> gpurun_out/bench_o.err || { tail -20 gpurun_out/bench_o.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_o$k.json'))
print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'])"
done
