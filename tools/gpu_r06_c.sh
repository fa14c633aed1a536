#!/bin/bash
# Round-6 GPU session C: the round's profiles at HEAD -- rocprofv3 passes of the bench workload
# (tools/profile.sh, configs[3] object off so the passes match r05's), a kernel trace of
# configs[3] at N = 1 (2^26 proofs, overlapped spans), and the in-kernel clock probes of
# k_verify_each and the RLC kernels (clock-probe build).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_ARGS="--c4-n 0" bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; exit 1; }
tail -3 gpurun_out/profile.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 bench.py --steps 1 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 3 > gpurun_out/prof_c4.log 2>&1 || { tail -20 gpurun_out/prof_c4.log; exit 1; }
grep '^{"metric"' gpurun_out/prof_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 under profiler', d['c4']['proofs_per_s'], d['c4']['ok'])"
CLOCK=1 CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 200 python tools/time_verify.py > gpurun_out/verify_clock.txt 2> gpurun_out/verify_clock.err || { tail -5 gpurun_out/verify_clock.err; exit 1; }
cat gpurun_out/verify_clock.txt
MODE=rlc CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 200 python tools/time_verify.py > gpurun_out/rlc_clock.json 2> gpurun_out/rlc_clock.err || { tail -5 gpurun_out/rlc_clock.err; exit 1; }
head -c 600 gpurun_out/rlc_clock.json
