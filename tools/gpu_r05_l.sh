#!/bin/bash
# Round-5 GPU session L: the branch-free 31-bit split in k_verify_wide's wave 4 -- latency-path
# tests, the wave-4 micro-benchmark, phases, small_batch.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_l.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_l.log | head -20; tail -30 gpurun_out/gpu_l.log; exit 1; }
tail -1 gpurun_out/gpu_l.log
timeout -k 10 60 tools/ubench/w4_parts > gpurun_out/w4_parts_l.json 2>&1 || { cat gpurun_out/w4_parts_l.json; exit 1; }
cat gpurun_out/w4_parts_l.json
for n in 1 1 8; do
  N=$n CALLS=40 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_l.jsonl || exit 1
done
N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_l.jsonl || exit 1
cat gpurun_out/wide_phases_l.jsonl
for rep in 1 2; do
  timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_l$rep.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_l$rep.json'))
print([(r['n'], round(r['verify_each_ms'],4), round(r['verify_batch_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_l.txt
done
