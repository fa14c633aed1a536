#!/bin/bash
# Round-6 closing check at HEAD (k_rlc_final16, lane-parallel combine, the final-knob test), in the driver's order.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_t.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_t.log | head -20; tail -30 gpurun_out/gpu_all_t.log; exit 1; }
tail -1 gpurun_out/gpu_all_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_t.log 2>&1 || { tail -20 gpurun_out/smoke_t.log; exit 1; }
tail -1 gpurun_out/smoke_t.log
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err || { tail -20 gpurun_out/bench_t.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_t.json'))
print('value %.4g frac %.3f cpu %.4g/%d  c4 %.4g ok %s forged %.0f ms  rlc %.4g  c5 %.3f / %.3f  small n=1 %.4f ms batch n=1 %.3f ms' % (d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['c4']['proofs_per_s'], d['c4']['ok'], d['c4']['forged']['ms'], d['rlc']['proofs_per_s'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], d['small_batch']['rows'][0]['verify_each_ms'], d['small_batch']['rows'][0]['verify_batch_ms']))"
