#!/bin/bash
# Round-6 GPU session J: C5 tuning around the one-lane combine -- HEAD against the one-lane
# combine for the locate pass too (lib/var/lanemin8k.so) and 256-proof blocks (lib/var/part256.so),
# alternating, one box.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in libcpz var/lanemin8k var/part256; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/$lib.so timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c4-n 0 --rlc-extra 0 --host-e2e 0 --small-batch 0 > gpurun_out/j_c5.json 2> gpurun_out/j_c5.err || { tail -10 gpurun_out/j_c5.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/j_c5.json'))
print('%-14s C5 %.1f ms (%.3fx)  ctx %.1f ms (%.3fx)  per-proof %.1f ms  msm %.2f  part_acc %.2f  locate %.2f' % ('$lib', d['c5']['ms'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ms'], d['c5_ctx']['ratio_to_per_proof'], d['c5']['per_proof_only_ms'], d['c5']['phase_ms']['rlc_msm'], d['c5']['phase_ms']['part_acc'], d['c5']['phase_ms']['part_acc_locate']))" | tee -a gpurun_out/j_ab.txt
  done
done
