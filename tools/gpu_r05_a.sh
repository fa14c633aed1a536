#!/bin/bash
# Round-5 GPU session A: the box's CPU share, the full GPU suite (incl. the launcher-less
# `bench.py --gpus 4` rehearsal), then the default bench line.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
{ echo "nproc=$(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; echo "OMP=$OMP_NUM_THREADS"; cat /sys/fs/cgroup/pids.max 2>/dev/null; } > gpurun_out/box_cpu.txt 2>&1
cat gpurun_out/box_cpu.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', {k: d['cpu_baseline'].get(k) for k in ('value','cores','affinity_cpus','cgroup_cpu_quota','at_omp_threads')})
print('small', [(r['n'], round(r['verify_each_ms'],3), round(r['cpu_batch_verifier_ms'],3)) for r in d['small_batch']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
