"""cpz_verify_each_device latency per call at several batch sizes (device buffers, median of
STEPS calls): run once per library (CPZ_LIB) to place the limit between k_verify_quad (eight
lanes per proof) and k_verify_each (one lane per proof)."""
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
    gpu = cp.Gpu(0)
    sizes = [int(x) for x in os.environ.get("SIZES", "1024 2048 4096 8192 16384 32768").split()]
    nmax = max(sizes)
    dev = torch.device("cuda", 0)
    t = {k: torch.empty((nmax, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_synthetic_device(nmax, bench.SEED_X, bench.SEED_K, t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    st = torch.empty(nmax, dtype=torch.uint8, device=dev)
    out = []
    for n in sizes:
        rows = [t[k][:n] for k in ("y1", "y2", "r1", "r2", "s")]
        for _ in range(3):
            gpu.verify_each_device(*rows, st[:n])
        torch.cuda.synchronize()
        ms = []
        for _ in range(int(os.environ.get("STEPS", "7"))):
            t0 = time.perf_counter()
            gpu.verify_each_device(*rows, st[:n])
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
        assert not st[:n].any().item()
        out.append({"n": n, "ms": round(float(np.median(ms)), 4)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
