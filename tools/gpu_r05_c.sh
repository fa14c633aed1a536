#!/bin/bash
# Round-5 GPU session C: (1) affine per-proof tables, bounded by two timing-only builds against
# HEAD in alternating rounds (k_verify_each per launch: head / niels = entries added as affine
# Niels points, no normalisation / inv = one extra inversion per equation); (2) where a small
# synchronous call spends its time (k_verify_quad phase stamps, clock-probe build).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for args in "N=1" "N=10" "N=1000" "N=1 CUSTOM=1" "N=1000 CUSTOM=1"; do
  env $args CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so CALLS=40 timeout -k 10 200 python tools/quad_phases.py >> gpurun_out/quad_phases.jsonl 2> gpurun_out/quad_phases.err || { tail -5 gpurun_out/quad_phases.err; exit 1; }
done
cat gpurun_out/quad_phases.jsonl
AMD_LOG_LEVEL=1 CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/niels.so STEPS=2 timeout -k 10 200 python tools/time_verify.py > gpurun_out/aff_niels_dbg.txt 2> gpurun_out/aff_niels_dbg.err
echo "niels rc=$?"; grep -v "^$" gpurun_out/aff_niels_dbg.err | tail -12
for r in 1 2 3; do
  for v in head inv; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so STEPS=10 timeout -k 10 200 python tools/time_verify.py > gpurun_out/aff_${v}_$r.txt 2> gpurun_out/aff_${v}_$r.err || { tail -5 gpurun_out/aff_${v}_$r.err; exit 1; }
    cat gpurun_out/aff_${v}_$r.txt
  done
done
