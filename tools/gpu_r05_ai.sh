#!/bin/bash
# Round-5 GPU session AI: k_verify_wide's tables with their 2 d T products batched (two
# products per table instead of seven in the chain) -- latency tests, phases, small_batch.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_ai.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_ai.log | head -20; tail -30 gpurun_out/gpu_ai.log; exit 1; }
tail -1 gpurun_out/gpu_ai.log
for n in 1 8; do
  N=$n CALLS=40 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_ai.jsonl || exit 1
done
N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_ai.jsonl || exit 1
cat gpurun_out/wide_phases_ai.jsonl
for rep in 1 2; do
  timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_ai.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_ai.json'))
print('libcpz', [(r['n'], round(r['verify_each_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_ai.txt
done
