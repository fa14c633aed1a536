"""The batch check with its fallback on 2^20 synthetic proofs holding k forged entries (s + 1),
k in FORGED (default 0 1 2 3 8 24): milliseconds per call (median of STEPS), the fallback's path and
stats, and the exact-set check -- the sparse branch (one MSM, then bisection) of verify_batch_impl."""
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
    n = int(os.environ.get("N", 1 << 20))
    steps = int(os.environ.get("STEPS", "3"))
    dev = torch.device("cuda", 0)
    gpu = cp.Gpu(0)
    base = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_synthetic_device(n, bench.SEED_X, bench.SEED_K, base["y1"], base["y2"], base["r1"], base["r2"], base["s"])
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    out = []
    for k in [int(x) for x in os.environ.get("FORGED", "0 1 2 3 8 24").split()]:
        t = {key: v.clone() for key, v in base.items()}
        idx = np.sort(np.random.default_rng(1000 + k).choice(n, size=k, replace=False)) if k else np.zeros(0, np.int64)
        if k:
            bench._bump_s(torch, t, idx)
        rows = [t[key] for key in ("y1", "y2", "r1", "r2", "s")]
        gpu.verify_batch_device(*rows, st, bench.WEIGHT_SEED, fallback=True)
        torch.cuda.synchronize()
        ms = []
        for _ in range(steps):
            t0 = time.perf_counter()
            gpu.verify_batch_device(*rows, st, bench.WEIGHT_SEED, fallback=True)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
        got = st.cpu().numpy()
        exact = np.array_equal(np.nonzero(got)[0], idx)
        out.append({"forged": k, "ms": round(float(np.median(ms)), 3), "fallback": gpu.fallback_stats(), "exact": bool(exact)})
        del t, rows
    print(json.dumps({"n": n, "runs": out}))


if __name__ == "__main__":
    main()
