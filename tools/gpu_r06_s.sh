#!/bin/bash
# NOTE: CPZ_RLC_SPAN_PIPE existed only in the measured build (not kept; DESIGN.md "Sort-first / sort-ahead spans").
# Sort-ahead span pipeline (CPZ_RLC_SPAN_PIPE=1: the sorts one span ahead on the second stream, every
# accumulation + reduction in order on the caller's stream) against the default interleaved spans:
# spans / RLC parity with the knob on, an alternating A/B on configs[3] and the RLC extra, a trace.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
CPZ_RLC_SPAN_PIPE=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_rlc.py > gpurun_out/s_tests.log 2>&1 || { tail -30 gpurun_out/s_tests.log; exit 1; }
tail -1 gpurun_out/s_tests.log
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --extras 0 --rlc-extra 1 --rlc-inflight 0 --c4-steps 5"
for rep in 1 2 3; do
  for sf in 0 1; do
    CPZ_RLC_SPAN_PIPE=$sf timeout -k 10 300 python bench.py $ARGS > gpurun_out/s_ab_${sf}_${rep}.json 2> gpurun_out/s_ab_${sf}_${rep}.err || { tail -20 gpurun_out/s_ab_${sf}_${rep}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/s_ab_${sf}_${rep}.json')); c=d['c4']
print('pipe=$sf rep $rep: c4 %.4g (%.1f ms/step) ok %s forged %.0f ms total %s  rlc %.4g  head %.4g' % (c['proofs_per_s'], c['ms_per_step'], c['ok'], c['forged']['ms'], c['forged']['combined_total'][:16], d['rlc']['proofs_per_s'], d['value']))" | tee -a gpurun_out/s_ab.txt
  done
done
CPZ_RLC_SPAN_PIPE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s_trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --extras 0 --rlc-extra 0 --c4-steps 2 > gpurun_out/s_trace.json 2> gpurun_out/s_trace.err
