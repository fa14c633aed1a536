#!/bin/bash
# Round-6 session P at HEAD (k_rlc_final16, lane-parallel combine): configs[3] at full size through
# the driver's plain multi-rank form as gloo rehearsals (every rank on the box's one GPU, no rate),
# N = 2, 4, 8; then three back-to-back default bench lines on the same box (spread).
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for n in 2 4 8; do
  timeout -k 10 400 python bench.py --gpus $n --same-device --backend gloo --steps 1 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 1 > gpurun_out/p_reh$n.json 2> gpurun_out/p_reh$n.err || { tail -20 gpurun_out/p_reh$n.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/p_reh$n.json') if l.startswith('{\"metric\"')][0]; c=d['c4']
print('N=%d n_gpus=%d c4 ok %s identity %s per_rank_forged %s exact %s not_identity %s total %s' % ($n, d['n_gpus'], c['ok'], c['identity'], c['forged']['per_rank_forged'], c['forged']['statuses_exact_every_rank'], c['forged']['combined_total_not_identity'], c['forged']['combined_total'][:16]))" | tee -a gpurun_out/p_reh.txt
done
for rep in 1 2 3; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/p_bench$rep.json 2> gpurun_out/p_bench$rep.err || { tail -20 gpurun_out/p_bench$rep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/p_bench$rep.json'))
print('rep $rep: value %.4g frac %.3f cpu %.4g/%d  c4 %.4g ok %s forged %.0f ms  rlc %.4g  c5 %.3f / %.3f  small n=1 %.4f ms batch n=1 %.3f ms' % (d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['c4']['proofs_per_s'], d['c4']['ok'], d['c4']['forged']['ms'], d['rlc']['proofs_per_s'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], d['small_batch']['rows'][0]['verify_each_ms'], d['small_batch']['rows'][0]['verify_batch_ms']))" | tee -a gpurun_out/p_bench.txt
done
