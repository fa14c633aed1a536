#!/bin/bash
# Alternating A/B of library variants (chaum-pedersen-zkp_amd/lib/var/<name>.so) on configs[4]
# (tools/c5_probe.py), in one GPU session: ROUNDS x (each variant once).  Run from the repo root.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for name in ${VARIANTS:-p1 p2}; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$name.so STEPS=${STEPS:-1} timeout -k 10 200 python tools/c5_probe.py > gpurun_out/c5_${name}_$r.json 2> gpurun_out/c5_${name}_$r.err || { echo "$name failed"; tail -5 gpurun_out/c5_${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c5_${name}_$r.json')); c=d['calls'][-1]; print('%-6s round $r  %8.2f ms  msm %8.2f  per-proof-only %8.2f  exact %s' % ('$name', c['ms'], c['stages_ms'].get('rlc_msm', 0), d['per_proof_only_ms'], c['exact']))"
  done
done
