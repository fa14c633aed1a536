#!/bin/bash
# Round-5 GPU session N: Keccak-f spread over wave 4's lanes (keccak_wave.h) and the
# variable-base waves on four 64-bit windows -- the permutation's equality with the register
# form and timing (w4_parts), the latency-path tests on the variant library, phases (default
# and custom generators) and small_batch against HEAD.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
timeout -k 10 60 tools/ubench/w4_parts > gpurun_out/w4_parts_n.json 2>&1 || { cat gpurun_out/w4_parts_n.json; exit 1; }
cat gpurun_out/w4_parts_n.json
CPZ_LIB=$V/wavekeccak.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_n.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_n.log | head -20; tail -30 gpurun_out/gpu_n.log; exit 1; }
tail -1 gpurun_out/gpu_n.log
for lib in $V/probe_wavekeccak.so $PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_n.jsonl || exit 1
done
for lib in $V/probe_wavekeccak.so $PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so; do
  N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_n.jsonl || exit 1
done
cat gpurun_out/wide_phases_n.jsonl
for lib in wavekeccak libcpz wavekeccak libcpz; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_n.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_n.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_n.txt
done
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
