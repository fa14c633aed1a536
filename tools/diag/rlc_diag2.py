import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import chaum_pedersen as cp
import pyoracle as O
g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
ps = g["rlc"][1]["proofs"]
seed = bytes.fromhex(g["rlc"][1]["seed"])
A = lambda ps, k: np.frombuffer(b"".join(bytes.fromhex(p[k]) for p in ps), np.uint8).reshape(-1, 32)
with cp.Gpu(0) as gpu:
    for lo, fi in [(3, 8), (3, 5), (3, 0), (0, 8), (0, 11)]:
        sub = ps[lo:lo + 1]
        p, ok, s = gpu.verify_batch(*[A(sub, k) for k in ("y1", "y2", "r1", "r2", "s")], seed=seed, first_index=fi, statuses=False)
        rec = [O.ProofRecord(*(bytes.fromhex(q[k]) for k in ("y1","y2","r1","r2","s"))) for q in sub]
        match = [b for b in range(16) if O.ristretto_encode(O.rlc_partial(rec, seed, b)) == p]
        # also: which component?  try only-G/H or only points
        print("lo", lo, "fi", fi, "gpu matches oracle base", match, "identity" if p == bytes(32) else "")
