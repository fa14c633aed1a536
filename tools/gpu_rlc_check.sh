#!/bin/bash
# RLC / MSM GPU tests, RLC-mode bench and its rocprofv3 kernel stats (GPU box, repo root).
# Each GPU step has its own time limit; steps are chained so a failure stops the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rlc.py tests/test_gpu_msm.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $OUT/t.log 2>&1
rc=$?
tail -5 $OUT/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode rlc --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rlc -o run -- \
  python3 bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_rlc.log 2>&1
rc=$?
cat $OUT/b.json
python3 - <<'EOF'
import csv
for r in csv.DictReader(open("gpurun_out/prof_rlc/run_kernel_stats.csv")):
    if "rlc" in r["Name"] or "challenge" in r["Name"]:
        print("%-32s calls %3s avg_us %9.1f" % (r["Name"].split("(")[0][:32], r["Calls"], float(r["AverageNs"]) / 1e3))
EOF
exit $rc
