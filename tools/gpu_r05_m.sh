#!/bin/bash
# Round-5 GPU session M: the full GPU suite and the smoke on HEAD, the spin-wait A/B of small
# synchronous calls, then the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_m.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_m.log | head -20; tail -30 gpurun_out/gpu_all_m.log; exit 1; }
tail -1 gpurun_out/gpu_all_m.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_m.log 2>&1 || { tail -20 gpurun_out/smoke_m.log; exit 1; }
tail -1 gpurun_out/smoke_m.log
for sp in 1 0 1 0; do
  CPZ_SPIN_SYNC=$sp timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_m$sp.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_m$sp.json'))
print('spin=$sp', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_m.txt
done
timeout -k 10 900 python bench.py > gpurun_out/bench_m.json 2> gpurun_out/bench_m.err || { tail -20 gpurun_out/bench_m.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_m.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('at_omp_threads'))
print('small', [(r['n'], round(r['verify_each_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', [(r['pairs'], round(r['cold_ms'],2), round(r['warm_ms'],2), round(r['varbase_build_ms'],2)) for r in d['custom_pairs']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5']['roofline']['k_part_acc']['frac'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
