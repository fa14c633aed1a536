#!/bin/bash
# Round-5 GPU session F: the full suite and the smoke on HEAD, the default bench line, the
# rocprofv3 passes of the bench workload (tools/profile.sh), and the in-kernel clock probes of
# k_verify_each and the RLC kernels (clock-probe build).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('at_omp_threads'))
print('small', [(r['n'], round(r['verify_each_ms'],3)) for r in d['small_batch']['rows']])
print('pairs', [(r['pairs'], round(r['cold_ms'],2), round(r['warm_ms'],2), round(r['varbase_build_ms'],2)) for r in d['custom_pairs']['rows']])
print('c5', d['c5']['ratio_to_per_proof'], d['c5']['roofline']['k_part_acc']['frac'], d['c5_ctx']['ratio_to_per_proof'], 'rlc', d['rlc']['proofs_per_s'])"
bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; exit 1; }
tail -3 gpurun_out/profile.log
CLOCK=1 CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 200 python tools/time_verify.py > gpurun_out/verify_clock.txt 2> gpurun_out/verify_clock.err || { tail -5 gpurun_out/verify_clock.err; exit 1; }
cat gpurun_out/verify_clock.txt
MODE=rlc CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 200 python tools/time_verify.py > gpurun_out/rlc_clock.json 2> gpurun_out/rlc_clock.err || { tail -5 gpurun_out/rlc_clock.err; exit 1; }
head -c 400 gpurun_out/rlc_clock.json
