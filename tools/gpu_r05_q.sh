#!/bin/bash
# Round-5 GPU session Q: the split's batch rows on four lanes (sc_half_split32<true>) -- the
# wave-4 micro-benchmark, latency tests on the variant, phases and small_batch A/B.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
timeout -k 10 60 tools/ubench/w4_parts > gpurun_out/w4_parts_q.json 2>&1 || { cat gpurun_out/w4_parts_q.json; exit 1; }
cat gpurun_out/w4_parts_q.json
CPZ_LIB=$V/lanes.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_q.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_q.log | head -20; tail -30 gpurun_out/gpu_q.log; exit 1; }
tail -1 gpurun_out/gpu_q.log
for lib in $V/probe_lanes.so $PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so $V/probe_lanes.so $PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_q.jsonl || exit 1
done
cat gpurun_out/wide_phases_q.jsonl
for lib in lanes libcpz lanes libcpz; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_q.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_q.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_q.txt
done
