#!/bin/bash
# Round-5 GPU session AD: k_verify_wide in its own unit (wide.hip, -falign-loops=64) with the
# comb's [s'] B split over waves 4 and 5 -- full GPU suite, smoke, phases and small_batch
# against the same code without aligned loops, then the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_ad.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_ad.log | head -20; tail -30 gpurun_out/gpu_all_ad.log; exit 1; }
tail -1 gpurun_out/gpu_all_ad.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ad.log 2>&1 || { tail -20 gpurun_out/smoke_ad.log; exit 1; }
tail -1 gpurun_out/smoke_ad.log
for rep in 1 2; do
for lib in $P $V/probe_noalign.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_ad.jsonl || exit 1
  N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_ad.jsonl || exit 1
done
done
cat gpurun_out/wide_phases_ad.jsonl
for lib in libcpz noalign libcpz noalign; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_ad.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_ad.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_ad.txt
done
SIZES="1 8 128 256 384 512 640" STEPS=15 timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross_ad.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
cat gpurun_out/wide_cross_ad.json
timeout -k 10 900 python bench.py > gpurun_out/bench_ad.json 2> gpurun_out/bench_ad.err || { tail -20 gpurun_out/bench_ad.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_ad.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('at_omp_threads'))
print('small', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', [(r['pairs'], round(r['cold_ms'],2), round(r['warm_ms'],2), round(r['varbase_build_ms'],2)) for r in d['custom_pairs']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5']['roofline']['k_part_acc']['frac'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
