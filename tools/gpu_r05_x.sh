#!/bin/bash
# Round-5 GPU session X: HEAD with k_verify_wide decoding two points per wave (challenge and split on
# a SIMD of their own) -- full GPU suite, smoke, phases, crossover, the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_x.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_x.log | head -20; tail -30 gpurun_out/gpu_all_x.log; exit 1; }
tail -1 gpurun_out/gpu_all_x.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_x.log 2>&1 || { tail -20 gpurun_out/smoke_x.log; exit 1; }
tail -1 gpurun_out/smoke_x.log
for n in 1 8 100; do
  RAW=1 N=$n CALLS=40 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_x.jsonl || exit 1
done
for n in 1 8; do
  N=$n CALLS=40 CUSTOM=1 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_x.jsonl || exit 1
done
cat gpurun_out/wide_phases_x.jsonl
SIZES="1 2 8 32 128 256 384 512 640 768 1024" STEPS=15 timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross_x.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
cat gpurun_out/wide_cross_x.json
timeout -k 10 900 python bench.py > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err || { tail -20 gpurun_out/bench_x.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_x.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('at_omp_threads'))
print('small', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', [(r['pairs'], round(r['cold_ms'],2), round(r['warm_ms'],2), round(r['varbase_build_ms'],2)) for r in d['custom_pairs']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5']['roofline']['k_part_acc']['frac'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
