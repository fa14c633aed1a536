#!/bin/bash
# Round-5 GPU session U: issue priority (s_setprio) on k_verify_wide's critical waves --
# latency tests on the new default, phases and small_batch A/B against CPZ_WIDE_PRIO=0.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_u.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_u.log | head -20; tail -30 gpurun_out/gpu_u.log; exit 1; }
tail -1 gpurun_out/gpu_u.log
for lib in $P $V/probe_noprio.so $P $V/probe_noprio.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_u.jsonl || exit 1
  N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_u.jsonl || exit 1
done
cat gpurun_out/wide_phases_u.jsonl
for lib in libcpz noprio libcpz noprio; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_u.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_u.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_u.txt
done
SIZES="1 256 384 512 640" STEPS=15 timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross_u.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
cat gpurun_out/wide_cross_u.json
