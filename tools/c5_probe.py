"""configs[4] on its own (for rocprofv3 --kernel-trace --stats and A/B runs): 2^24 synthetic proofs,
0.1 % forged (half s + 1, half wrong y1, bench.py's set), one warm-up and STEPS timed calls of the
batch check with its fallback; prints the phase times, the fallback's path and the exact-set check."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    import chaum_pedersen as cp
    n = int(os.environ.get("N", 1 << 24))
    nf = max(1, n // 1000)
    dev = torch.device("cuda", 0)
    gpu = cp.Gpu(0)
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_synthetic_device(n, bench.SEED_X, bench.SEED_K, t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    idx = np.sort(np.random.default_rng(2024).choice(n, size=nf, replace=False))
    bump, swap = idx[0::2], idx[1::2]
    bench._bump_s(torch, t, bump)
    dst = torch.from_numpy(swap.astype(np.int64)).to(dev)
    src = torch.from_numpy(((swap + 7) % n).astype(np.int64)).to(dev)
    t["y1"].index_copy_(0, dst, t["y1"].index_select(0, src).clone())
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    rows = [t[k] for k in ("y1", "y2", "r1", "r2", "s")]
    gpu.verify_batch_device(*rows, st, bench.WEIGHT_SEED, fallback=True)
    torch.cuda.synchronize()
    out = []
    for _ in range(int(os.environ.get("STEPS", "2"))):
        gpu.set_timing(True)
        gpu.stage_times()
        t0 = time.perf_counter()
        p, ok = gpu.verify_batch_device(*rows, st, bench.WEIGHT_SEED, fallback=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        stages = {k: round(v[0], 3) for k, v in gpu.stage_times().items()}
        got = st.cpu().numpy()
        exact = (not ok) and np.array_equal(np.nonzero(got)[0], idx)
        out.append({"ms": round(el * 1e3, 2), "stages_ms": stages, "fallback": gpu.fallback_stats(), "exact": bool(exact)})
    t0 = time.perf_counter()
    gpu.verify_each_device(*rows, st)
    torch.cuda.synchronize()
    print(json.dumps({"n": n, "forged": nf, "calls": out, "per_proof_only_ms": round((time.perf_counter() - t0) * 1e3, 2)}))


if __name__ == "__main__":
    main()
