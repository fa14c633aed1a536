#!/bin/bash
# Round-6 GPU session H, HEAD in the driver's order: the full GPU suite, the smoke, the default
# bench line twice, then the headline held over 200 and 1000 back-to-back steps.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_h.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_h.log | head -20; tail -30 gpurun_out/gpu_all_h.log; exit 1; }
tail -1 gpurun_out/gpu_all_h.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_h.log 2>&1 || { tail -20 gpurun_out/smoke_h.log; exit 1; }
tail -1 gpurun_out/smoke_h.log
for k in 1 2; do
  timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_h$k.json 2> gpurun_out/bench_h$k.err || { tail -20 gpurun_out/bench_h$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_h$k.json'))
print('value %.4g frac %.3f cpu %.4g/%d  c4 %.4g ok %s forged %.0f ms  rlc %.4g  c5 %.3f / %.3f  small n=1 %.4f ms' % (d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['c4']['proofs_per_s'], d['c4']['ok'], d['c4']['forged']['ms'], d['rlc']['proofs_per_s'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], d['small_batch']['rows'][0]['verify_each_ms']))"
done
for s in 200 1000; do
  timeout -k 10 300 python bench.py --steps $s --warmup 5 --extras 0 --no-cpu-baseline --c4-n 0 > gpurun_out/soak_$s.json 2> gpurun_out/soak.err || { tail -10 gpurun_out/soak.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/soak_$s.json')); print('soak %d steps: %.4g proofs/s, %.3f ms/step' % ($s, d['value'], d['ms_per_step']))"
done
