#!/bin/bash
# Round-5 GPU session B: the box's CPU share; the variable-base tests first, then the full GPU
# suite, the smoke, and the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
{ echo "nproc=$(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; echo "OMP=$OMP_NUM_THREADS"; cat /sys/fs/cgroup/pids.max 2>/dev/null; } > gpurun_out/box_cpu.txt 2>&1
cat gpurun_out/box_cpu.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_varbase.py tests/test_gpu_dropin.py > gpurun_out/gpu_varbase.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_varbase.log | head -20; tail -60 gpurun_out/gpu_varbase.log; exit 1; }
tail -1 gpurun_out/gpu_varbase.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', {k: d['cpu_baseline'].get(k) for k in ('value','cores','affinity_cpus','cgroup_cpu_quota','at_omp_threads')})
print('small', [(r['n'], round(r['verify_each_ms'],3), round(r['cpu_batch_verifier_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', d.get('custom_pairs'))
print('c5', d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
export TMPDIR=/tmp
CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so MODE=c5 STEPS=2 timeout -k 10 300 python tools/time_verify.py > gpurun_out/c5_clock.json 2> gpurun_out/c5_clock.err || { tail -20 gpurun_out/c5_clock.err; exit 1; }
cat gpurun_out/c5_clock.json
STEPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 tools/c5_probe.py > gpurun_out/prof_c5.log 2>&1 || { tail -20 gpurun_out/prof_c5.log; exit 1; }
tail -1 gpurun_out/prof_c5.log | cut -c1-600
