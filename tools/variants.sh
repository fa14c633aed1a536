#!/bin/bash
# Side-by-side bench of library variants built by build_native.build_libcpz(out=..., defines=...)
# under chaum-pedersen-zkp_amd/lib/var/*.so (run on the GPU box from the repo root).
set -o pipefail
mkdir -p gpurun_out
for so in chaum-pedersen-zkp_amd/lib/var/*.so; do
  name=$(basename $so .so)
  CPZ_LIB=$PWD/$so timeout -k 10 240 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --extras 0 --rlc-extra ${RLC:-0} ${BENCH_ARGS} > gpurun_out/var_$name.json 2> gpurun_out/var_$name.err || { echo "$name failed"; tail -5 gpurun_out/var_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/var_$name.json')); r=d.get('roofline') or {}; rl=d.get('rlc') or {}; print('%-12s %10.0f proofs/s  kernel %s ms  challenge %s ms' % ('$name', d['value'], r.get('kernel_ms'), r.get('challenge_kernel_ms')), ' rlc %s ms/step %s' % (rl.get('ms_per_step'), (rl.get('roofline') or {}).get('kernel_ms_per_step','')))"
done
