#!/bin/bash
# Round-6 GPU session B: the full GPU suite at HEAD (RLC spans now overlap), smoke, then A/B of
# the span overlap (CPZ_RLC_SPAN_OVERLAP=0/1, same library) on configs[3] at N = 1, and of the
# span size (lib/var/span19.so, span20.so against HEAD's 2^21) on configs[2] / configs[3].
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_b.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gpu_all_b.log | head -20; tail -30 gpurun_out/gpu_all_b.log; exit 1; }
tail -1 gpurun_out/gpu_all_b.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_b.log 2>&1 || { tail -20 gpurun_out/smoke_b.log; exit 1; }
tail -1 gpurun_out/smoke_b.log
summ() {
  python3 -c "
import json,sys; d=json.load(open('$1')); c=d.get('c4') or {}; r=d.get('roofline') or {}
print('%-28s value %.4g  c4 %s  c4_ms %s  ok %s' % ('$2', d['value'] or 0, c.get('proofs_per_s'), c.get('ms_per_step'), c.get('ok')))" | tee -a gpurun_out/ab_b.txt
}
for rep in 1 2; do
  for ov in 1 0; do
    CPZ_RLC_SPAN_OVERLAP=$ov timeout -k 10 300 python bench.py --steps 5 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 5 > gpurun_out/ab_ov$ov.json 2> gpurun_out/ab_ov$ov.err || { tail -10 gpurun_out/ab_ov$ov.err; exit 1; }
    summ gpurun_out/ab_ov$ov.json "overlap=$ov (span 2^21)"
  done
  for sp in 19 20; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/span$sp.so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --extras 0 --no-cpu-baseline --c4-steps 5 > gpurun_out/ab_sp$sp.json 2> gpurun_out/ab_sp$sp.err || { tail -10 gpurun_out/ab_sp$sp.err; exit 1; }
    summ gpurun_out/ab_sp$sp.json "span 2^$sp overlap=1"
  done
  for lib in libcpz var/span19; do
    CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/$lib.so timeout -k 10 300 python bench.py --mode rlc --steps 10 --warmup 2 --extras 0 --no-cpu-baseline --c4-n 0 > gpurun_out/ab_rlc.json 2> gpurun_out/ab_rlc.err || { tail -10 gpurun_out/ab_rlc.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_rlc.json')); print('configs[2] 2^20 RLC %-12s %.4g proofs/s' % ('$lib', d['value']))" | tee -a gpurun_out/ab_b.txt
  done
done
