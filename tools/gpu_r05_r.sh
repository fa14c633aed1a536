#!/bin/bash
# Round-5 GPU session R: the row product's shifted operand as one v_mul_i32_i24 through DPP
# (fe16.h shifted) on top of the four-lane split rows -- latency tests on the variant, phases,
# small_batch A/B against HEAD.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
CPZ_LIB=$V/shift1.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_varbase.py > gpurun_out/gpu_r.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_r.log | head -20; tail -30 gpurun_out/gpu_r.log; exit 1; }
tail -1 gpurun_out/gpu_r.log
for lib in $V/probe_shift1.so $PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so $V/probe_shift1.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_r.jsonl || exit 1
done
N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$V/probe_shift1.so timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"probe_shift1.so\", #" >> gpurun_out/wide_phases_r.jsonl || exit 1
cat gpurun_out/wide_phases_r.jsonl
for lib in shift1 libcpz shift1 libcpz; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_r.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_r.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_r.txt
done
SIZES="1 128 256 384 512 640 768" STEPS=15 CPZ_LIB=$V/shift1.so timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross_r.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
cat gpurun_out/wide_cross_r.json
