#!/bin/bash
# NOTE: CPZ_RLC_SPAN_SETS existed only in the measured build (not kept; DESIGN.md "Three MSM sets").
# Three MSM sets / streams for configs[3]'s overlapped spans (CPZ_RLC_SPAN_SETS=3) against two:
# the spans' parity tests with three sets first, then an alternating A/B of the same library on
# configs[3] (c4 line, forged variant included) and the RLC extra.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
CPZ_RLC_SPAN_SETS=3 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_rlc.py > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --extras 0 --rlc-extra 1 --rlc-inflight 0 --c4-steps 5"
for rep in 1 2 3; do
  for ns in 2 3; do
    CPZ_RLC_SPAN_SETS=$ns timeout -k 10 300 python bench.py $ARGS > gpurun_out/q_ab_${ns}_${rep}.json 2> gpurun_out/q_ab_${ns}_${rep}.err || { tail -20 gpurun_out/q_ab_${ns}_${rep}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/q_ab_${ns}_${rep}.json')); c=d['c4']
print('sets=$ns rep $rep: c4 %.4g (%.1f ms/step) ok %s forged %.0f ms total %s  rlc %.4g  head %.4g' % (c['proofs_per_s'], c['ms_per_step'], c['ok'], c['forged']['ms'], c['forged']['combined_total'][:16], d['rlc']['proofs_per_s'], d['value']))" | tee -a gpurun_out/q_ab.txt
  done
done
