#!/bin/bash
# Round-4 GPU session D: the profiles of the bench workload (tools/profile.sh: kernel trace +
# stats, FETCH / WRITE / SQ / L2 counter passes), a kernel trace of configs[4] on its own, the
# in-kernel clock probe of k_verify_each and the v_mad issue-rate microbenchmark.
set -o pipefail
export TMPDIR=/tmp
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
bash tools/profile.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 tools/c5_probe.py > gpurun_out/prof_c5.log 2>&1 || exit $?
CLOCK=1 CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 240 python tools/time_verify.py > gpurun_out/verify_clock_probe.log 2>&1 || exit $?
cat gpurun_out/verify_clock_probe.log
timeout -k 10 120 tools/ubench/clock_rates > gpurun_out/clock_rates.json 2> gpurun_out/clock_rates.err || exit $?
head -c 600 gpurun_out/clock_rates.json
