#!/bin/bash
# Round-5 GPU session Z: rocprofv3 evidence for k_verify_wide at HEAD -- kernel trace + stats of
# one-proof synchronous calls (tools/sb_trace.py N=1 MODE=each) and two SQ counter passes.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
export N=1 MODE=each
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide -o run -- python3 tools/sb_trace.py > gpurun_out/prof_wide.log 2>&1 || { tail -20 gpurun_out/prof_wide.log; exit 1; }
grep "ms per call" gpurun_out/prof_wide.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/prof_wide_sq -o run -- python3 tools/sb_trace.py > gpurun_out/prof_wide_sq.log 2>&1 || { tail -20 gpurun_out/prof_wide_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/prof_wide_sq2 -o run -- python3 tools/sb_trace.py > gpurun_out/prof_wide_sq2.log 2>&1 || { tail -20 gpurun_out/prof_wide_sq2.log; exit 1; }
find gpurun_out/prof_wide gpurun_out/prof_wide_sq gpurun_out/prof_wide_sq2 -name "*.csv" | head -20
