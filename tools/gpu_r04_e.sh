#!/bin/bash
# Round-4 GPU session E: the partitioned check's locate pass -- its GPU tests, then an
# alternating C5 A/B of the library without (loc0) and with (loc1) the pass.
set -o pipefail
export TMPDIR=/tmp
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_scale.py \
  -k "partitioned" > gpurun_out/t_loc.log 2>&1 || { tail -40 gpurun_out/t_loc.log; exit 1; }
tail -3 gpurun_out/t_loc.log
VARIANTS="loc0 locj16" ROUNDS=2 bash tools/c5_ab.sh
