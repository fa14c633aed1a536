#!/bin/bash
# Round-4 GPU session I: the eight-lane kernel on the partitioned check's listed blocks -- GPU
# suite, then C5 and the sparse-forgery probe with it off (quad0) and on (product).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
cp chaum-pedersen-zkp_amd/lib/libcpz.so chaum-pedersen-zkp_amd/lib/var/head.so
VARIANTS="quad0 head" ROUNDS=2 bash tools/c5_ab.sh || exit 1
for v in quad0 head; do
  CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so FORGED="1 3 24" timeout -k 10 300 python tools/sparse_probe.py > gpurun_out/spq_$v.json 2> gpurun_out/spq_$v.err || { tail -3 gpurun_out/spq_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/spq_$v.json'))
print('$v', [(r['forged'], r['ms'], r['exact']) for r in d['runs']])"
done
