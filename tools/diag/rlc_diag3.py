import os, sys, hashlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch
import chaum_pedersen as cp
import pyoracle as O
sx = hashlib.sha256(b"cpz-bench-x").digest(); sk = hashlib.sha256(b"cpz-bench-k").digest()
seed = hashlib.sha256(b"cpz-weights-v1").digest()
def synth(gpu, n, first):
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device="cuda:0") for k in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_synthetic_device(n, sx, sk, t["y1"], t["y2"], t["r1"], t["r2"], t["s"], first_index=first)
    return t
def bump(t, i):
    s = t["s"].cpu().numpy().copy()
    v = (int.from_bytes(s[i].tobytes(), "little") + 1) % O.L
    s[i] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
    t["s"].copy_(torch.from_numpy(s))
with cp.Gpu(0) as gpu:
    for n, first, bad in [(1 << 10, 0, 5), (1 << 10, 1 << 20, 5), (1 << 16, 0, 40000), (1 << 17, 0, 100000), (1 << 18, 0, 200003), (1 << 18, 1 << 20, 200003), (1 << 18, 1 << 20, 3)]:
        t = synth(gpu, n, first)
        bump(t, bad)
        st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], st)
        torch.cuda.synchronize()
        each_bad = np.nonzero(st.cpu().numpy())[0].tolist()
        p, ok = gpu.verify_batch_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], st, seed, first_index=0)
        # oracle expectation: partial = [a]g + [b]h for weights at index `bad`
        a = O.batch_weight(seed, bad); b = O.batch_weight2(seed, bad)
        exp = O.ristretto_encode(O.pt_add(O.pt_mul(O.BASEPOINT, a), O.pt_mul(O.generator_h(), b)))
        print(n, first, bad, "each:", each_bad, "rlc ok:", ok, "partial==exp:", p == exp, "partial zero:", p == bytes(32), flush=True)
