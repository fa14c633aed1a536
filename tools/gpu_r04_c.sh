#!/bin/bash
# Round-4 GPU session C: the full GPU suite at HEAD, a same-box A/B of HEAD against the round-3
# library (headline and RLC step), then the default bench line.  Each step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/t_c.log 2>&1; rc=$?
tail -3 gpurun_out/t_c.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_c.log | head -30; exit $rc; }
VARIANTS="r03 head" ROUNDS=3 STEPS=20 bash tools/gpu_ab.sh || exit $?
VARIANTS="r03 head" ROUNDS=2 STEPS=10 BENCH_ARGS="--mode rlc" bash tools/gpu_ab.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err || { tail -5 gpurun_out/bench_r04a.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r04a.json')); print(d['value'], d['roofline']['frac'], d['rlc']['proofs_per_s'], d['c5']['ratio_to_per_proof'], d['c5_ctx']['ratio_to_per_proof'])"
