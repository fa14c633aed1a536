#!/bin/bash
# Round-5 GPU session AC: code placement of the row kernels -- -falign-loops=64 / 256 builds
# against the default (the Straus phase moved 46.8 <-> 53.2 us between builds whose loop code
# is identical): phases, small_batch and the headline per variant, alternating.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/chaum-pedersen-zkp_amd/lib/var
P=$PWD/chaum-pedersen-zkp_amd/lib/timing/clock_probe.so
for rep in 1 2; do
for lib in $P $V/probe_a64.so $V/probe_256.so; do
  N=1 CALLS=40 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_ac.jsonl || exit 1
  [ $rep = 1 ] && { N=8 CALLS=40 CUSTOM=1 CPZ_LIB=$lib timeout -k 10 120 python tools/quad_phases.py | sed "s#^{#{\"lib\": \"$(basename $lib)\", #" >> gpurun_out/wide_phases_ac.jsonl || exit 1; }
done
done
cat gpurun_out/wide_phases_ac.jsonl
for lib in libcpz al_a64 al_256 libcpz al_a64 al_256; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 300 python tools/small_batch.py > gpurun_out/sb_ac.json 2> gpurun_out/sb.err || { tail -5 gpurun_out/sb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sb_ac.json'))
print('$lib', [(r['n'], round(r['verify_each_ms'],4)) for r in d['rows']])" | tee -a gpurun_out/sb_ac.txt
done
for lib in libcpz al_a64 al_256 libcpz al_a64 al_256; do
  L=$PWD/chaum-pedersen-zkp_amd/lib/libcpz.so; [ $lib != libcpz ] && L=$V/$lib.so
  CPZ_LIB=$L timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --extras 0 > gpurun_out/b_ac.json 2> gpurun_out/b_ac.err || { tail -5 gpurun_out/b_ac.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b_ac.json')); print('$lib headline', round(d['value']/1e6,2), 'M/s frac', round(d['roofline']['frac'],4))" | tee -a gpurun_out/sb_ac.txt
done
