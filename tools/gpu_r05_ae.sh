#!/bin/bash
# Round-5 GPU session AE: where the kernel arguments live (HIP_FORCE_DEV_KERNARG unset / 1 / 0)
# for the drop-in's synchronous calls -- k_verify_wide's arguments are 1,336 bytes.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for kv in unset 1 0; do
    if [ $kv = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$kv; fi
    timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_ae.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sb_ae.json'))
print('HIP_FORCE_DEV_KERNARG=$kv', [(r['n'], round(r['verify_each_ms'],4), round(r['verify_batch_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_ae.txt
  done
done
