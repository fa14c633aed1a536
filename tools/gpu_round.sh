#!/bin/bash
# One GPU session: tests, smoke, bench (with CPU baseline), profiles.  Stops at the first failure.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then echo "== profile"; bash tools/profile.sh; fi
