#!/bin/bash
# Round-5 GPU session J: k_verify_wide with the scalar split and its variable-base waves
# (custom Parameters) -- full suite, smoke, wave-4 micro-benchmark, phases (A/B of the split
# on the scalar unit), small_batch A/B, then the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_j.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_j.log | head -20; tail -30 gpurun_out/gpu_all_j.log; exit 1; }
tail -1 gpurun_out/gpu_all_j.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_j.log 2>&1 || { tail -20 gpurun_out/smoke_j.log; exit 1; }
tail -1 gpurun_out/smoke_j.log
timeout -k 10 120 tools/ubench/wide_mul gpurun_out/wide_mul_j.bin > gpurun_out/wide_mul_j.txt 2>&1 || { cat gpurun_out/wide_mul_j.txt; exit 1; }
python3 tools/ubench/wide_mul_check.py gpurun_out/wide_mul_j.bin >> gpurun_out/wide_mul_j.txt; cat gpurun_out/wide_mul_j.txt
timeout -k 10 60 tools/ubench/w4_parts > gpurun_out/w4_parts.json 2>&1 || { cat gpurun_out/w4_parts.json; exit 1; }
cat gpurun_out/w4_parts.json
for lib in $V/probe_split_vector.so $P; do
  for n in 1 8; do
    N=$n CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_j.jsonl || exit 1
  done
done
for n in 1 8 64; do
  N=$n CALLS=40 CUSTOM=1 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"clock_probe.so\", #" >> gpurun_out/wide_phases_j.jsonl || exit 1
done
cat gpurun_out/wide_phases_j.jsonl
for lib in libcpz split_vector libcpz split_vector; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_$lib.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_$lib.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_j.txt
done
timeout -k 10 900 python bench.py > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err || { tail -20 gpurun_out/bench_j.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_j.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('at_omp_threads'))
print('small', [(r['n'], round(r['verify_each_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', [(r['pairs'], round(r['cold_ms'],2), round(r['warm_ms'],2), round(r['varbase_build_ms'],2)) for r in d['custom_pairs']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5']['roofline']['k_part_acc']['frac'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
