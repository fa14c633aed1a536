export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out
for r in 1 2; do for v in q0 q1; do
  CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so STEPS=10 timeout -k 10 200 python tools/rlc_inflight.py > gpurun_out/infl_${v}_$r.json 2> gpurun_out/infl_${v}_$r.err || { echo "$v failed"; tail -3 gpurun_out/infl_${v}_$r.err; exit 1; }
  echo "$v $r $(cat gpurun_out/infl_${v}_$r.json)"
done; done
ROUNDS=2 STEPS=20 VARIANTS="q0 q1" bash tools/gpu_ab.sh || exit 1
CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/q1.so STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_infl_q1 -o run -- python3 tools/rlc_inflight.py > gpurun_out/prof_infl_q1.log 2>&1
echo trace rc=$?
for r in 1 2; do RLC=1 STEPS=10 VARS="q0 q1 p1 p2 p4" bash -c 'for v in $VARS; do CPZ_LIB=$PWD/chaum-pedersen-zkp_amd/lib/var/$v.so timeout -k 10 240 python bench.py --steps 10 --warmup 1 --no-cpu-baseline --extras 0 --rlc-extra 1 > gpurun_out/rlcab_${v}.json 2> gpurun_out/rlcab_${v}.err || exit 1; python3 -c "import json; d=json.load(open(\"gpurun_out/rlcab_$v.json\")); print(\"$v\", round(d[\"rlc\"][\"ms_per_step\"],3), round(d[\"rlc\"][\"proofs_per_s\"]/1e6,1))"; done' || exit 1; done
