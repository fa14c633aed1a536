#!/bin/bash
# Round-6 GPU session G: the full GPU suite and the smoke at HEAD, then the round's profiles
# (tools/gpu_r06_c.sh: rocprofv3 passes of the bench workload, configs[3] kernel trace, clock
# probes).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_g.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_g.log | head -20; tail -30 gpurun_out/gpu_all_g.log; exit 1; }
tail -1 gpurun_out/gpu_all_g.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_g.log 2>&1 || { tail -20 gpurun_out/smoke_g.log; exit 1; }
tail -1 gpurun_out/smoke_g.log
bash tools/gpu_r06_c.sh
