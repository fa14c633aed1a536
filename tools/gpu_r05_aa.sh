#!/bin/bash
# Round-5 GPU session AA: does the two-decode k_verify_wide beat k_verify_small above 512 proofs?
# quad_crossover with CPZ_WIDE_MAX raised (every launch <= 4096 on k_verify_wide) against the
# default (512), alternating.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for wm in 512 4096; do
    CPZ_WIDE_MAX=$wm SIZES="384 512 640 768 896 1000 1024 1536 2048" STEPS=15 timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/xo_aa_$wm.json 2> gpurun_out/xo_aa.err || { tail -5 gpurun_out/xo_aa.err; exit 1; }
    echo "wide_max=$wm $(cat gpurun_out/xo_aa_$wm.json)" | tee -a gpurun_out/xo_aa.txt
  done
done
