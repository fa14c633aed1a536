#!/bin/bash
# The fallback switches still verify exactly: the RLC / scale / distributed GPU tests with the spans
# in order (CPZ_RLC_SPAN_OVERLAP=0, the path taken when the second MSM set does not fit) and with
# the quad-tree window combine (CPZ_RLC_FINAL16=0).
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
CPZ_RLC_SPAN_OVERLAP=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rlc.py tests/test_gpu_scale.py tests/test_gpu_distributed.py > gpurun_out/u_overlap0.log 2>&1 || { tail -30 gpurun_out/u_overlap0.log; exit 1; }
echo "CPZ_RLC_SPAN_OVERLAP=0: $(tail -1 gpurun_out/u_overlap0.log)"
CPZ_RLC_FINAL16=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rlc.py tests/test_gpu_scale.py tests/test_gpu_distributed.py > gpurun_out/u_final0.log 2>&1 || { tail -30 gpurun_out/u_final0.log; exit 1; }
echo "CPZ_RLC_FINAL16=0: $(tail -1 gpurun_out/u_final0.log)"
