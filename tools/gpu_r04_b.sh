#!/bin/bash
# Round-4 GPU session B: small-batch kernels (dynamic bucket chunk, four-lane prepare) --
# their tests, the small-batch table, and an A/B of the four-lane prepare at 2^20 proofs.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_rlc.py tests/test_gpu_msm.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_b.log 2>&1; rc=$?
tail -5 gpurun_out/t_b.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_b.log | head -30; exit $rc; }
timeout -k 10 300 python tools/small_batch.py > gpurun_out/small_batch_r04c.json 2> gpurun_out/small_batch_r04c.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu -k "partitioned" --timeout 300 --timeout-method thread > gpurun_out/t_b2.log 2>&1; rc=$?
tail -5 gpurun_out/t_b2.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_b2.log | head -30; exit $rc; }
VARIANTS="base wide" ROUNDS=2 STEPS=10 BENCH_ARGS="--mode rlc" bash tools/gpu_ab.sh
