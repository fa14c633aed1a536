#!/bin/bash
# Round-5 GPU session AB: custom-pair [s'] g, [s'] h on four waves (two per equation, four
# 32-bit parts each) against two (CPZ_WIDE_VB_WAVES=2) -- variable-base and latency tests,
# phases with a custom pair, alternating.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_varbase.py tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py > gpurun_out/gpu_ab.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_ab.log | head -20; tail -30 gpurun_out/gpu_ab.log; exit 1; }
tail -1 gpurun_out/gpu_ab.log
for rep in 1 2; do
for lib in $V/probe_vbw2.so $P; do
  for n in 1 8 100; do
    N=$n CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_ab.jsonl || exit 1
  done
done
done
N=1 CALLS=40 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"clock_probe.so\", #" >> gpurun_out/wide_phases_ab.jsonl || exit 1
cat gpurun_out/wide_phases_ab.jsonl
