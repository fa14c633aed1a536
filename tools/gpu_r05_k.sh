#!/bin/bash
# Round-5 GPU session K: k_verify_wide with the 31-bit-window split in wave 4 and the branch-free
# row-pair decode product -- the latency-path tests, micro-benchmarks, phases (pair A/B), the
# small_batch table.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py tests/test_gpu_parity.py > gpurun_out/gpu_k.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_k.log | head -20; tail -30 gpurun_out/gpu_k.log; exit 1; }
tail -1 gpurun_out/gpu_k.log
timeout -k 10 120 tools/ubench/wide_mul gpurun_out/wide_mul_k.bin > gpurun_out/wide_mul_k.txt 2>&1 || { cat gpurun_out/wide_mul_k.txt; exit 1; }
cat gpurun_out/wide_mul_k.txt
timeout -k 10 60 tools/ubench/w4_parts > gpurun_out/w4_parts_k.json 2>&1 || { cat gpurun_out/w4_parts_k.json; exit 1; }
cat gpurun_out/w4_parts_k.json
for lib in $V/probe_nopair.so $P $V/probe_nopair.so $P; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_k.jsonl || exit 1
done
for n in 8 64; do
  N=$n CALLS=40 CUSTOM=1 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"clock_probe.so\", #" >> gpurun_out/wide_phases_k.jsonl || exit 1
done
cat gpurun_out/wide_phases_k.jsonl
for rep in 1 2; do
  timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_k$rep.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_k$rep.json'))
print([(r['n'], round(r['verify_each_ms'],4), round(r['verify_batch_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_k.txt
done
