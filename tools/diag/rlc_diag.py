import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
import chaum_pedersen as cp
g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
case = g["rlc"][1]
ps = case["proofs"]
A = lambda ps, k: np.frombuffer(b"".join(bytes.fromhex(p[k]) for p in ps), np.uint8).reshape(-1, 32)
args = [A(ps, k) for k in ("y1", "y2", "r1", "r2", "s")]
seed = bytes.fromhex(case["seed"])
sh = case["shards"]
def run(gpu, lo, hi, fi, st=False):
    p, ok, s = gpu.verify_batch(*[a[lo:hi] for a in args], seed=seed, first_index=fi, statuses=st)
    return p.hex()
with cp.Gpu(0) as gpu:
    print("fresh shard0", run(gpu, 0, 6, 5) == sh[0]["partial"])
    print("then shard1", run(gpu, 6, 12, 11) == sh[1]["partial"])
    print("then full", run(gpu, 0, 12, 5) == case["partial"])
    print("then shard0", run(gpu, 0, 6, 5) == sh[0]["partial"])
with cp.Gpu(0) as gpu:
    print("fresh full+st", run(gpu, 0, 12, 5, True) == case["partial"])
    print("then shard0", run(gpu, 0, 6, 5) == sh[0]["partial"])
with cp.Gpu(0) as gpu:
    for lo, hi in [(0, 1), (0, 2), (0, 3), (0, 4), (0, 5), (0, 6), (3, 4)]:
        import pyoracle as O
        recs = [O.ProofRecord(*(bytes.fromhex(p[k]) for k in ("y1","y2","r1","r2","s"))) for p in ps[lo:hi]]
        exp = O.ristretto_encode(O.rlc_partial(recs, seed, 5 + lo)).hex()
        print("range", lo, hi, run(gpu, lo, hi, 5 + lo) == exp)
