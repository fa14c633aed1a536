#!/bin/bash
# Round-5 GPU session E: full suite on HEAD (quad-doubling Niels build, small-kernel stamps);
# k_verify_small's phases (clock-probe build); the small / quad crossover (smallmax16k: the
# small kernel up to 16384 proofs); C5 with blocks of 256 proofs against 128 (part256).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
rm -f gpurun_out/small_phases.jsonl
for args in "N=1" "N=8" "N=1000" "N=1 CUSTOM=1" "N=1000 CUSTOM=1"; do
  env $args CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so CALLS=40 timeout -k 10 200 python tools/quad_phases.py >> gpurun_out/small_phases.jsonl 2> gpurun_out/small_phases.err || { tail -5 gpurun_out/small_phases.err; exit 1; }
done
cat gpurun_out/small_phases.jsonl
for r in 1 2; do
  for v in head smallmax16k; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so SIZES="256 1024 2048 4096 8192 16384" timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/xo_${v}_$r.json 2> gpurun_out/xo_${v}_$r.err || { tail -5 gpurun_out/xo_${v}_$r.err; exit 1; }
    echo "$v $r $(cat gpurun_out/xo_${v}_$r.json)"
  done
done
for r in 1 2; do
  for v in head part256; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so STEPS=2 timeout -k 10 300 python tools/c5_probe.py > gpurun_out/c5ab_${v}_$r.json 2> gpurun_out/c5ab_${v}_$r.err || { tail -5 gpurun_out/c5ab_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/c5ab_${v}_$r.json'))
print('$v $r', [c['ms'] for c in d['calls']], [c['exact'] for c in d['calls']], d['per_proof_only_ms'], d['calls'][-1]['stages_ms'])"
  done
done
