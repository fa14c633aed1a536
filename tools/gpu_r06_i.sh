#!/bin/bash
# Round-6 GPU session I: k_part_combine with one lane per block (C5's first pass) -- the
# partitioned-check tests on it, then C5 A/B against the quad-cooperative combine
# (lib/var/lane0.so), alternating, one box, with per-kernel stage times.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py > gpurun_out/gpu_i.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_i.log | head -20; tail -30 gpurun_out/gpu_i.log; exit 1; }
tail -1 gpurun_out/gpu_i.log
for rep in 1 2 3; do
  for lib in libcpz var/lane0; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/$lib.so timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c4-n 0 --rlc-extra 0 --host-e2e 0 --small-batch 0 > gpurun_out/i_c5.json 2> gpurun_out/i_c5.err || { tail -10 gpurun_out/i_c5.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/i_c5.json'))
print('%-10s C5 %.1f ms (%.3fx)  ctx %.1f ms (%.3fx)  per-proof %.1f ms  msm %.2f  part_acc %.2f' % ('$lib', d['c5']['ms'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ms'], d['c5_ctx']['ratio_to_per_proof'], d['c5']['per_proof_only_ms'], d['c5']['phase_ms']['rlc_msm'], d['c5']['phase_ms']['part_acc']))" | tee -a gpurun_out/i_ab.txt
  done
done
