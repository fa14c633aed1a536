#!/bin/bash
# One GPU session for a round's checks: the GPU tests, smoke, the VALU clock microbenchmark,
# the in-kernel clock probe of k_verify_each (timing-only build), then the bench.  Stops at the
# first failure; every step has its own time limit.  STEPS selects a subset (default: all).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
steps=${STEPS:-"quick tests smoke clock probe sq bench"}
for s in $steps; do
  case $s in
    tests) echo "== pytest -m gpu ${TESTS:-tests}"
      timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
      grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -80; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    quick) echo "== quick: ${QUICK:-tests/test_gpu_scale.py::test_partitioned_fallback_at_c5_density}"
      timeout -k 10 600 python -u -m pytest ${QUICK:-tests/test_gpu_scale.py::test_partitioned_fallback_at_c5_density} -x -v --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1; rc=$?
      grep -E "PASSED|FAILED|ERROR|assert|Error" gpurun_out/quick.log | tail -30; [ $rc -eq 0 ] || exit $rc ;;
    sq) echo "== sq_radix"
      timeout -k 10 120 tools/ubench/sq_radix > gpurun_out/sq_radix.json 2> gpurun_out/sq_radix.err; rc=$?; cat gpurun_out/sq_radix.json; [ $rc -eq 0 ] || exit $rc ;;
    smoke) echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    clock) echo "== clock_rates"
      timeout -k 10 120 tools/ubench/clock_rates > gpurun_out/clock_rates.json 2> gpurun_out/clock_rates.err; rc=$?; cat gpurun_out/clock_rates.json; [ $rc -eq 0 ] || exit $rc ;;
    probe) echo "== clock probe"
      CLOCK=1 CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 240 python tools/time_verify.py > gpurun_out/clock_probe.log 2>&1; rc=$?; cat gpurun_out/clock_probe.log; [ $rc -eq 0 ] || exit $rc ;;
    bench) echo "== bench"
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
