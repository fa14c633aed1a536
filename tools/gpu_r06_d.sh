#!/bin/bash
# Round-6 GPU session D: split prepare (k_rlc_decode4 at 4 waves/SIMD with the low-register
# decode + k_rlc_scalars) -- the RLC / scale / distributed GPU tests on it, then A/B against
# the one-kernel prepare (lib/var/nosplit.so) and a 3-wave decode (lib/var/split3.so): the RLC
# step at 2^20 (configs[2]), configs[3] at N = 1, and C5 (configs[4]), alternating, one box;
# and the per-proof decode split (lib/var/vsplit.so: k_verify_decode4 + k_verify_prepared) on
# the headline.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rlc.py tests/test_gpu_scale.py tests/test_gpu_msm.py tests/test_gpu_distributed.py > gpurun_out/gpu_d.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_d.log | head -20; tail -30 gpurun_out/gpu_d.log; exit 1; }
tail -1 gpurun_out/gpu_d.log
for rep in 1 2; do
  for lib in libcpz var/nosplit var/split3; do
    L=$PWD/chaum-pedersen-zkp_amd/lib/$lib.so
    CPZ_LIB=$L timeout -k 10 300 python bench.py --mode rlc --steps 10 --warmup 2 --extras 0 --no-cpu-baseline --c4-n 0 > gpurun_out/d_rlc.json 2> gpurun_out/d_rlc.err || { tail -10 gpurun_out/d_rlc.err; exit 1; }
    CPZ_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 5 > gpurun_out/d_c4.json 2> gpurun_out/d_c4.err || { tail -10 gpurun_out/d_c4.err; exit 1; }
    python3 -c "
import json; r=json.load(open('gpurun_out/d_rlc.json')); c=json.load(open('gpurun_out/d_c4.json'))
ms=(r['roofline'].get('rlc') or {}).get('kernel_ms_per_step',{})
print('%-12s configs[2] %.4g proofs/s (prepare %.3f ms/step)  configs[3] %.4g proofs/s ok %s' % ('$lib', r['value'], ms.get('rlc_prepare',0), c['c4']['proofs_per_s'], c['c4']['ok']))" | tee -a gpurun_out/d_ab.txt
  done
done
for rep in 1 2 3; do
  for lib in libcpz var/vsplit; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/$lib.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --extras 0 --no-cpu-baseline --c4-n 0 > gpurun_out/d_each.json 2> gpurun_out/d_each.err || { tail -10 gpurun_out/d_each.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/d_each.json')); r=d['roofline']
print('%-12s configs[1] %.4g proofs/s  verify kernel %.3f ms  challenge(+decode) %.3f ms  span %.3f ms' % ('$lib', d['value'], r['kernel_ms'], r['challenge_kernel_ms'], r['verify_span_ms_per_step']))" | tee -a gpurun_out/d_ab.txt
  done
done
for rep in 1 2; do
  for lib in libcpz var/nosplit; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/$lib.so timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c4-n 0 --rlc-extra 0 --host-e2e 0 --small-batch 0 > gpurun_out/d_c5.json 2> gpurun_out/d_c5.err || { tail -10 gpurun_out/d_c5.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/d_c5.json'))
print('%-12s C5 %.1f ms (%.3fx)  ctx %.1f ms (%.3fx)  prepare %.2f ms' % ('$lib', d['c5']['ms'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ms'], d['c5_ctx']['ratio_to_per_proof'], d['c5']['phase_ms']['rlc_prepare']))" | tee -a gpurun_out/d_ab.txt
  done
done
# the per-proof split's parity: the headline-scale tests through vsplit.so
CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/vsplit.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py > gpurun_out/gpu_d_vsplit.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_d_vsplit.log | head -20; tail -30 gpurun_out/gpu_d_vsplit.log; exit 1; }
tail -1 gpurun_out/gpu_d_vsplit.log
