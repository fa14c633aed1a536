#!/bin/bash
# Round-5 GPU session H: k_verify_wide (one proof per five-wave workgroup, field products on
# 16-lane rows) -- parity on the small-launch tests (product library; then the row-pair
# decode variant), its phases, and the latency crossover against k_verify_small.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "small_kernel" tests/test_gpu_dropin.py tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_varbase.py > gpurun_out/wide_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/wide_tests.log | head -20; tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -1 gpurun_out/wide_tests.log
CPZ_LIB=$V/wide_pair.so timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "small_kernel" > gpurun_out/wide_pair_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/wide_pair_tests.log | head -20; tail -30 gpurun_out/wide_pair_tests.log; exit 1; }
tail -1 gpurun_out/wide_pair_tests.log
for lib in $V/probe_nopair.so $PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so; do
  for n in 1 8 32; do
    N=$n CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases.jsonl 2> gpurun_out/wide_phases.err || { tail -5 gpurun_out/wide_phases.err; exit 1; }
  done
done
N=1 CALLS=40 CPZ_WIDE_MAX=0 CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases.jsonl 2> gpurun_out/wide_phases.err || { tail -5 gpurun_out/wide_phases.err; exit 1; }
cat gpurun_out/wide_phases.jsonl
for cfg in "0 $V/wide_pair.so" "4096 $V/wide_nopair.so" "4096 $V/wide_pair.so" "0 $V/wide_pair.so" "4096 $V/wide_nopair.so" "4096 $V/wide_pair.so"; do
  set -- $cfg
  SIZES="1 2 4 8 16 32 64 128 256 512 1024" STEPS=15 CPZ_WIDE_MAX=$1 CPZ_LIB=$2 timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
  echo "wide_max=$1 lib=$(basename $2) $(cat gpurun_out/wide_cross.json)" | tee -a gpurun_out/wide_crossover.txt
done
CPZ_LIB=$V/wide_pair.so timeout -k 10 300 python tools/small_batch.py > gpurun_out/wide_small_batch.json 2> gpurun_out/wide_small_batch.err || { tail -5 gpurun_out/wide_small_batch.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/wide_small_batch.json'))
print([(r['n'], round(r['verify_each_ms'],3), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])"
