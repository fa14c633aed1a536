#!/bin/bash
# Round-4 GPU session H: eight-lanes-per-proof verification of small batches (k_verify_quad) --
# the GPU suite, then the small-batch table without (quad0) and with it (product).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
for r in 1 2; do
  for v in quad0 head; do
    lib=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so; [ $v = head ] && lib=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so
    CPZ_LIB=$lib timeout -k 10 300 python tools/small_batch.py > gpurun_out/sbq_${v}_$r.json 2> gpurun_out/sbq_${v}_$r.err || { tail -5 gpurun_out/sbq_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sbq_${v}_$r.json'))
print('%-6s' % '$v', ' '.join('%d:%.3f/%.3f/%.3f' % (x['n'], x['verify_each_ms'], x['verify_batch_ms'], x.get('verify_batch_one_forged_ms', 0)) for x in d['rows']))"
  done
done
