#!/bin/bash
# Round artefacts on the GPU box (repo root): headline bench with CPU baseline, RLC-mode
# bench, rocprofv3 kernel stats of the RLC mode.  Outputs under gpurun_out/; copy the
# ones to keep into profiles/<round>_*.  Each GPU step has its own limit, chained with &&.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --mode rlc --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_rlc.json 2> $OUT/bench_rlc.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rlc -o run -- python3 bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_rlc.log 2>&1
rc=$?
cat $OUT/bench.json $OUT/bench_rlc.json
exit $rc
