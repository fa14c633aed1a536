#!/bin/bash
# Round-4 GPU session F: sparse forgeries (tools/sparse_probe.py) with bisection (sp0) and with the
# partitioned check after a failed MSM (product), at 2^19 and 2^20 proofs.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for N in 524288 1048576; do
  for v in sp0 head; do
    lib=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so; [ $v = head ] && lib=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so
    CPZ_LIB=$lib N=$N timeout -k 10 300 python tools/sparse_probe.py > gpurun_out/sparse_${v}_$N.json 2> gpurun_out/sparse_${v}_$N.err || { tail -5 gpurun_out/sparse_${v}_$N.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sparse_${v}_$N.json'))
print('$v', d['n'], [(r['forged'], r['ms'], r['exact'], r['fallback']['path']) for r in d['runs']])"
  done
done
