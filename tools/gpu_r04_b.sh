#!/bin/bash
# Round-4 GPU session B: small-batch kernels (dynamic bucket chunk, four-lane prepare) and the
# partitioned check's block size -- tests, the small-batch table, A/Bs (prepare at 2^20 in the
# RLC step; C5 with 256- vs 128-proof blocks).  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_rlc.py tests/test_gpu_msm.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_b.log 2>&1; rc=$?
tail -3 gpurun_out/t_b.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_b.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu -k "partitioned" --timeout 300 --timeout-method thread > gpurun_out/t_b2.log 2>&1; rc=$?
tail -3 gpurun_out/t_b2.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_b2.log | head -30; exit $rc; }
CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/p128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu -k "partitioned" --timeout 300 --timeout-method thread > gpurun_out/t_b3.log 2>&1; rc=$?
tail -3 gpurun_out/t_b3.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_b3.log | head -30; exit $rc; }
timeout -k 10 300 python tools/small_batch.py > gpurun_out/small_batch_r04c.json 2> gpurun_out/small_batch_r04c.err || exit $?
VARIANTS="base wide" ROUNDS=2 STEPS=10 BENCH_ARGS="--mode rlc" bash tools/gpu_ab.sh || exit $?
VARIANTS="base p128" ROUNDS=2 STEPS=1 bash tools/c5_ab.sh
