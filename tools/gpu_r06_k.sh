#!/bin/bash
# Round-6 GPU session K: the prepare pipelined with the overlapped MSM spans (span j's prepare
# chunk, then its MSM on its set's stream) -- the scale / RLC / distributed tests on it, then
# A/B against the whole prepare first (CPZ_RLC_PIPELINE=0, same library) on configs[3] at N = 1.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_rlc.py tests/test_gpu_distributed.py tests/test_gpu_msm.py > gpurun_out/gpu_k.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_k.log | head -20; tail -30 gpurun_out/gpu_k.log; exit 1; }
tail -1 gpurun_out/gpu_k.log
for rep in 1 2 3; do
  for pl in 1 0; do
    CPZ_RLC_PIPELINE=$pl timeout -k 10 300 python bench.py --steps 3 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 5 > gpurun_out/k_c4.json 2> gpurun_out/k_c4.err || { tail -10 gpurun_out/k_c4.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/k_c4.json')); c=d['c4']
print('pipeline=$pl configs[3] %.4g proofs/s  %.1f ms/step  ok %s  forged %.0f ms' % (c['proofs_per_s'], c['ms_per_step'], c['ok'], c['forged']['ms']))" | tee -a gpurun_out/k_ab.txt
  done
done
