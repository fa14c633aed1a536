#!/bin/bash
# Alternating A/B of library variants (chaum-pedersen-zkp_amd/lib/var/<name>.so) on the headline
# bench, in one GPU session: ROUNDS x (each variant once), then optional extra steps.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for name in ${VARIANTS:-r02 r03}; do
    so=chaum-pedersen-zkp_amd/lib/var/$name.so
    CPZ_LIB=$PWD/$so timeout -k 10 240 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --extras 0 ${BENCH_ARGS} > gpurun_out/ab${TAG}_${name}_$r.json 2> gpurun_out/ab${TAG}_${name}_$r.err || { echo "$name failed"; tail -5 gpurun_out/ab${TAG}_${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab${TAG}_${name}_$r.json')); r=d.get('roofline') or {}; print('%-6s round $r %10.0f proofs/s  kernel %.4f ms' % ('$name', d['value'], r.get('kernel_ms') or 0))"
  done
done
