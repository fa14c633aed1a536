#!/bin/bash
# Round-4 GPU session J: the tree combine for few partition blocks (k_part_combine_tree) -- the GPU
# suite, then C5 with it off (tree0), for few blocks (product) and for every size (treebig), and
# the sparse-forgery probe at 2^20 off / on.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gpu_all.log | head; tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
cp chaum-pedersen-zkp_amd/lib/libcpz.so chaum-pedersen-zkp_amd/lib/var/head.so
VARIANTS="tree0 head treebig" ROUNDS=2 bash tools/c5_ab.sh || exit 1
for v in tree0 head; do
  CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so FORGED="0 1 3 24" timeout -k 10 300 python tools/sparse_probe.py > gpurun_out/spt_$v.json 2> gpurun_out/spt_$v.err || { tail -3 gpurun_out/spt_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/spt_$v.json'))
print('$v', [(r['forged'], r['ms'], r['exact']) for r in d['runs']])"
done
