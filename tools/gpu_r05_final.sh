#!/bin/bash
# Round-5 closing check at HEAD, in the driver's order: full GPU suite, smoke, default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_final.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_final.log | head -20; tail -30 gpurun_out/gpu_all_final.log; exit 1; }
tail -1 gpurun_out/gpu_all_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 900 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_final.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('at_omp_threads'))
print('small', [(r['n'], round(r['verify_each_ms'],4), round(r['cpu_batch_verifier_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', [(r['pairs'], round(r['cold_ms'],2), round(r['warm_ms'],2)) for r in d['custom_pairs']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
