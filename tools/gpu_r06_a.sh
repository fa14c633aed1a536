#!/bin/bash
# Round-6 GPU session A: the new tests (light-set bound at 110 CUs, the world-4 rehearsal's c4
# object), the default bench line with configs[3] measured at N = 1, then the f64-limb
# microbenchmark (tools/ubench/fe_f64.hip).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_varbase.py "tests/test_gpu_distributed.py::test_bench_rlc_four_rank_rehearsal" > gpurun_out/gpu_a.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_a.log | head -20; tail -30 gpurun_out/gpu_a.log; exit 1; }
tail -1 gpurun_out/gpu_a.log
timeout -k 10 900 python bench.py > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { tail -20 gpurun_out/bench_a.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_a.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline'].get('cores_basis'))
c=d['c4']; print('c4', c['proofs_per_s'], c['ms_per_step'], c['identity'], c['forged'])
print('c5', d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
# f64 limbs against radix 2^25.5 (ISA VALU counts per call from profiles/r06_fe_f64_isa.txt)
timeout -k 10 120 tools/ubench/fe_f64 20 149 214 118 175 > gpurun_out/fe_f64_a.jsonl 2>&1; rc=$?
cat gpurun_out/fe_f64_a.jsonl
exit $rc
