#!/bin/bash
# Round-4 GPU session: new tests, the small-batch table, the full GPU suite, the RLC clock probe.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_api.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_new.log | tail -40
[ $rc -eq 0 ] || { tail -60 gpurun_out/t_new.log; exit $rc; }
timeout -k 10 300 python tools/small_batch.py > gpurun_out/small_batch_r04b.json 2> gpurun_out/small_batch_r04b.err || exit $?
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -15 gpurun_out/t_all.log
[ $rc -eq 0 ] || exit $rc
MODE=rlc CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 240 python tools/time_verify.py > gpurun_out/rlc_clock_probe.json 2> gpurun_out/rlc_clock_probe.err || exit $?
cat gpurun_out/rlc_clock_probe.json
