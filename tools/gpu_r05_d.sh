#!/bin/bash
# Round-5 GPU session D: k_verify_small (three waves per 8 proofs) -- its boundary tests and the
# drop-in / variable-base tests, the full suite, then the per-call latency table A/B against the
# same library without it (small0), and the affine-table bound (head / niels / inv).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "small_kernel" tests/test_gpu_dropin.py tests/test_gpu_varbase.py > gpurun_out/gpu_small.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_small.log | head -20; tail -50 gpurun_out/gpu_small.log; exit 1; }
tail -1 gpurun_out/gpu_small.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
for r in 1 2; do
  for v in head small0; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_${v}_$r.json 2> gpurun_out/sb_${v}_$r.err || { tail -5 gpurun_out/sb_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sb_${v}_$r.json'))
print('$v $r', [(r['n'], round(r['verify_each_ms'],3), round(r['verify_batch_ms'],3), round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])"
  done
done
for r in 1 2; do
  for v in head niels inv; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so STEPS=10 timeout -k 10 200 python tools/time_verify.py > gpurun_out/aff_${v}_$r.txt 2> gpurun_out/aff_${v}_$r.err || { tail -5 gpurun_out/aff_${v}_$r.err; exit 1; }
    cat gpurun_out/aff_${v}_$r.txt
  done
done
