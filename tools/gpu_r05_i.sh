#!/bin/bash
# Round-5 GPU session I: k_verify_wide with the row-pair decode and the small-quotient split,
# zero-copy small calls -- the full GPU suite, smoke, phases, crossover, small_batch A/B.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_i.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_i.log | head -20; tail -30 gpurun_out/gpu_all_i.log; exit 1; }
tail -1 gpurun_out/gpu_all_i.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_i.log 2>&1 || { tail -20 gpurun_out/smoke_i.log; exit 1; }
tail -1 gpurun_out/smoke_i.log
for n in 1 8 512; do
  N=$n CALLS=40 CPZ_LIB=$P timeout -k 10 120 python tools/quad_phases.py >> gpurun_out/wide_phases_i.jsonl 2> gpurun_out/wide_phases.err || { tail -5 gpurun_out/wide_phases.err; exit 1; }
done
cat gpurun_out/wide_phases_i.jsonl
for cfg in "0 libcpz" "512 libcpz" "512 nopair" "0 libcpz" "512 libcpz" "512 nopair"; do
  set -- $cfg
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $2 = nopair ] && L=$V/wide_nopair.so
  SIZES="1 2 8 32 128 256 384 512 768 1024" STEPS=15 CPZ_WIDE_MAX=$1 CPZ_LIB=$L timeout -k 10 200 python tools/quad_crossover.py > gpurun_out/wide_cross.json 2> gpurun_out/wide_cross.err || { tail -5 gpurun_out/wide_cross.err; exit 1; }
  echo "wide_max=$1 lib=$2 $(cat gpurun_out/wide_cross.json)" | tee -a gpurun_out/wide_crossover_i.txt
done
for zc in 1 0 1 0; do
  CPZ_ZERO_COPY=$zc timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_zc$zc.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_zc$zc.json'))
print('zero_copy=$zc', [(r['n'], round(r['verify_each_ms'],4), round(r['verify_batch_ms'],4) if r.get('verify_batch_ms') else None, round(r['cpu_batch_verifier_ms'],3)) for r in d['rows']])" | tee -a gpurun_out/sb_zc.txt
done
