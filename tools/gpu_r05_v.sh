#!/bin/bash
# Round-5 GPU session V: k_verify_wide issue-priority modes (CPZ_WIDE_PRIO 0..3) -- phases
# (with wave 1's uncontended decode / Straus beside wave 0's) and small_batch A/B.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py -k wide > gpurun_out/gpu_v.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_v.log | head -20; tail -30 gpurun_out/gpu_v.log; exit 1; }
tail -1 gpurun_out/gpu_v.log
for rep in 1 2; do
for lib in $V/probe_prio0.so $P $V/probe_prio2.so $V/probe_prio3.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_v.jsonl || exit 1
  [ $rep = 1 ] && { N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_v.jsonl || exit 1; }
done
done
cat gpurun_out/wide_phases_v.jsonl
for lib in prio0 libcpz prio2 prio3 prio0 libcpz prio2 prio3; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_v.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_v.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_v.txt
done
