#!/bin/bash
# Round-5 GPU session W: k_verify_wide with two decodes per wave (CPZ_WIDE_DUAL, the challenge
# and split on a SIMD of their own) -- latency-path tests, phases and small_batch A/B against
# the one-decode-per-wave layout.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_w.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_w.log | head -20; tail -30 gpurun_out/gpu_w.log; exit 1; }
tail -1 gpurun_out/gpu_w.log
for rep in 1 2; do
for lib in $V/probe_nodual.so $P $V/probe_dualp0.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_w.jsonl || exit 1
  [ $rep = 1 ] && { N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_w.jsonl || exit 1; }
done
done
cat gpurun_out/wide_phases_w.jsonl
for lib in nodual libcpz dualp0 nodual libcpz dualp0; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_w.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_w.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_w.txt
done
SIZES="1 256 384 512 640" STEPS=15 timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross_w.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
cat gpurun_out/wide_cross_w.json
