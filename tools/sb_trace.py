"""One small synchronous call repeated (N proofs; MODE=batch: cpz_verify_batch, MODE=each:
cpz_verify_each), for a kernel / copy trace of the drop-in's regime under rocprofv3."""
import os, sys, time
sys.path.insert(0, "/root/repo/chaum-pedersen-zkp_amd"); sys.path.insert(0, "/root/repo")
import numpy as np
import bench
import chaum_pedersen as cp
gpu = cp.Gpu(0)
n = int(os.environ.get("N", "10"))
rows = gpu.prove_synthetic(n, bench.SEED_X, bench.SEED_K)
args = [np.ascontiguousarray(rows[k]) for k in ("y1", "y2", "r1", "r2", "s")]
if os.environ.get("MODE", "batch") == "each":
    call = lambda: gpu.verify_each(*args, equations_only=True)
else:
    call = lambda: gpu.verify_batch(*args, seed=bench.WEIGHT_SEED, equations_only=True)
for _ in range(30):
    call()
t0 = time.perf_counter()
for _ in range(50):
    call()
print("ms per call", (time.perf_counter() - t0) * 1e3 / 50)
