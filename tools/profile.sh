#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root): the
# headline per-proof steps plus the RLC extra, so both paths' kernels are in every pass.
#   A: kernel trace + stats (per-kernel durations)      -> gpurun_out/prof_trace
#   B/C: HBM traffic counters, one per pass (FETCH_SIZE, WRITE_SIZE)
#   D: SQ instruction / wave counters
#   E: L2 hit / miss and the GUI-active cycles (effective clock)
# Each GPU step has its own time limit; steps are chained with && so a failure stops the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --extras 0 --rlc-extra 1 --rlc-inflight 0 ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- python3 bench.py $ARGS > $OUT/prof_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o run -- python3 bench.py $ARGS > $OUT/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o run -- python3 bench.py $ARGS > $OUT/prof_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/prof_sq -o run -- python3 bench.py $ARGS > $OUT/prof_sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS --output-format csv -d $OUT/prof_l2 -o run -- python3 bench.py $ARGS > $OUT/prof_l2.log 2>&1
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" | head -50
exit $rc
