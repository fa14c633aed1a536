#!/bin/bash
# k_rlc_final16 (Horner on 16-lane rows) against the quad tree k_rlc_final: parity tests of the
# RLC path on the new default, then an alternating A/B of the same library (CPZ_RLC_FINAL16=0/1):
# configs[2] (rlc), configs[3] (c4 + forged), the batch-check latency (small_batch), then a
# kernel trace of the new final.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rlc.py tests/test_gpu_scale.py tests/test_gpu_distributed.py > $OUT/n_tests.log 2>&1 || { tail -30 $OUT/n_tests.log; exit 1; }
tail -1 $OUT/n_tests.log
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --extras 0 --rlc-extra 1 --rlc-inflight 0 --small-batch 1"
for rep in 1 2; do
  for f in 0 1; do
    CPZ_RLC_FINAL16=$f timeout -k 10 300 python bench.py $ARGS > $OUT/n_ab_${f}_${rep}.json 2> $OUT/n_ab_${f}_${rep}.err || { tail -20 $OUT/n_ab_${f}_${rep}.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$OUT/n_ab_${f}_${rep}.json'))
sb=d['small_batch']['rows']
print('final16=$f rep $rep: head %.4g rlc %.4g c4 %.4g forged %.0f ms  batch_ms n=1 %.3f n=10 %.3f n=100 %.3f n=1000 %.3f' % (d['value'], d['rlc']['proofs_per_s'], d['c4']['proofs_per_s'], d['c4']['forged']['ms'], sb[0]['verify_batch_ms'], sb[3]['verify_batch_ms'], sb[6]['verify_batch_ms'], sb[7]['verify_batch_ms']), 'c4ok', d['c4']['ok'], d['c4']['forged']['combined_total'][:16])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/n_trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras 0 --rlc-extra 1 --rlc-inflight 0 --small-batch 1 --c4-n 0 > $OUT/n_trace.json 2> $OUT/n_trace.err
rc=$?
grep -h "k_rlc_final" $OUT/n_trace/run_kernel_stats.csv
exit $rc
