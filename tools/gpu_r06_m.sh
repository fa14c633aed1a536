#!/bin/bash
# Round-6 final library under the profiler: kernel trace + stats of the bench with configs[3] (c4),
# C5 (single-lane combine) and the RLC extra, then the HBM fetch / write passes of the same command.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --extras 1 --rlc-inflight 0 --host-e2e 0 --small-batch 0 --c4-steps 3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/m_trace -o run -- python3 bench.py $ARGS > $OUT/m_trace.json 2> $OUT/m_trace.err &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/m_fetch -o run -- python3 bench.py $ARGS > $OUT/m_fetch.json 2> $OUT/m_fetch.err &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/m_write -o run -- python3 bench.py $ARGS > $OUT/m_write.json 2> $OUT/m_write.err
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" -path "*m_*" | head -20
exit $rc
