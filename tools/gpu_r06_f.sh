#!/bin/bash
# Round-6 GPU session F: span-local batch-fail fallback -- the scale / RLC / distributed GPU
# tests on it, configs[3] at full size through the driver's multi-rank form as gloo rehearsals
# (plain `bench.py --gpus N --same-device`, N = 2 and 8: 2^26 proofs over the ranks, forged
# variant in two ranks' shards), then the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_rlc.py tests/test_gpu_distributed.py > gpurun_out/gpu_f.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_f.log | head -20; tail -30 gpurun_out/gpu_f.log; exit 1; }
tail -1 gpurun_out/gpu_f.log
for n in 2 8; do
  timeout -k 10 400 python bench.py --gpus $n --same-device --backend gloo --steps 1 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 1 > gpurun_out/f_reh$n.json 2> gpurun_out/f_reh$n.err || { tail -20 gpurun_out/f_reh$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/f_reh$n.json')); c=d['c4']
print('N=%d n_gpus=%d c4 ok %s identity %s per_rank_forged %s exact %s not_identity %s fallback %s' % ($n, d['n_gpus'], c['ok'], c['identity'], c['forged']['per_rank_forged'], c['forged']['statuses_exact_every_rank'], c['forged']['combined_total_not_identity'], c['forged']['rank0_fallback']))" | tee -a gpurun_out/f_reh.txt
done
timeout -k 10 900 python bench.py > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err || { tail -20 gpurun_out/bench_f.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_f.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
c=d['c4']; print('c4', c['proofs_per_s'], c['ok'], 'forged ms', c['forged']['ms'], c['forged']['rank0_fallback'])
print('c5', d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
