#!/bin/bash
# Round-5 GPU session AG: the wave Keccak with chi's neighbours read straight from pi's sources
# (three dependent exchange levels a round instead of four) -- wave-vs-register equality and
# cycles (w4_parts), latency tests, phases and small_batch against CPZ_KECCAK_FUSED_PI=0.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 60 tools/ubench/w4_parts > gpurun_out/w4_parts_ag.json 2>&1 || { cat gpurun_out/w4_parts_ag.json; exit 1; }
cat gpurun_out/w4_parts_ag.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_ag.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_ag.log | head -20; tail -30 gpurun_out/gpu_ag.log; exit 1; }
tail -1 gpurun_out/gpu_ag.log
for rep in 1 2; do
for lib in $P $V/probe_unfused.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_ag.jsonl || exit 1
done
done
cat gpurun_out/wide_phases_ag.jsonl
for lib in libcpz unfused libcpz unfused; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_ag.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_ag.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_ag.txt
done
