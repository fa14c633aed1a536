#!/bin/bash
# Round-6 GPU session E: configs[3] at full size through the driver's multi-rank form, as gloo
# rehearsals with every rank on the box's one GPU (no rate: ranks share the device) -- plain
# `bench.py --gpus N` for N = 2, 4, 8: 2^26 proofs split over the ranks, per-rank partials,
# all-gather, combine, the forged variant in two ranks' shards -- then the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4 8; do
  timeout -k 10 400 python bench.py --gpus $n --same-device --backend gloo --steps 1 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 1 > gpurun_out/e_reh$n.json 2> gpurun_out/e_reh$n.err || { tail -20 gpurun_out/e_reh$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/e_reh$n.json')); c=d['c4']
print('N=%d n_gpus=%d c4 ok %s identity %s per_rank_forged %s exact %s not_identity %s total %s' % ($n, d['n_gpus'], c['ok'], c['identity'], c['forged']['per_rank_forged'], c['forged']['statuses_exact_every_rank'], c['forged']['combined_total_not_identity'], c['forged']['combined_total'][:16]))" | tee -a gpurun_out/e_reh.txt
done
timeout -k 10 900 python bench.py > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err || { tail -20 gpurun_out/bench_e.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_e.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
c=d['c4']; print('c4', c['proofs_per_s'], c['ok'], 'c5', d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
