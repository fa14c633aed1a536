#!/bin/bash
# Round-5 GPU session G: the world-1 RCCL gather test and the lane-layout micro-benchmark
# for the drop-in's latency (tools/ubench/wide_mul.hip).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_distributed.py -k rccl > gpurun_out/rccl.log 2>&1 || { tail -40 gpurun_out/rccl.log; exit 1; }
tail -1 gpurun_out/rccl.log
timeout -k 10 120 tools/ubench/wide_mul gpurun_out/wide_mul.bin > gpurun_out/wide_mul.txt 2>&1 || { cat gpurun_out/wide_mul.txt; exit 1; }
cat gpurun_out/wide_mul.txt
python3 tools/ubench/wide_mul_check.py gpurun_out/wide_mul.bin
