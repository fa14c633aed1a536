"""Probe: RLC stage times (HIP-event marks) of verify_batch_device over 2^20 proofs, for
A/B of library variants built with build_native.build_libcpz(out=..., defines=...):

    CPZ_LIB=/path/libcpz_variant.so python3 tools/rlc_stage_probe.py

Prints per-step stage ms and a digest of a forged batch's partial (must agree across
variants: same weights, same forged entries)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))


def main():
    import torch
    import chaum_pedersen as cp
    n, steps = 1 << 20, 10
    keys = ("y1", "y2", "r1", "r2", "s")
    dev = torch.device("cuda", 0)
    gpu = cp.Gpu(0)
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in keys}
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    gpu.prove_synthetic_device(n, bytes(32), bytes(range(32)), *(t[k] for k in keys))
    seed = hashlib.sha256(b"probe").digest()
    p, ok = gpu.verify_batch_device(*(t[k] for k in keys), st, seed)
    assert ok and p == bytes(32)
    torch.cuda.synchronize()
    gpu.set_timing(True)
    gpu.stage_times()
    for _ in range(steps):
        gpu.verify_batch_device(*(t[k] for k in keys), st, seed)
    torch.cuda.synchronize()
    times = gpu.stage_times()
    gpu.set_timing(False)
    for name in ("rlc_prepare", "rlc_sort", "rlc_bucket", "rlc_bucket_fix", "rlc_reduce", "rlc_final", "rlc_msm"):
        if name in times:
            print("%-15s %.4f ms" % (name, times[name][0] / steps), flush=True)
    # forged: s + 1 on 37 entries (one byte bump keeps s canonical for these synthetic rows
    # with overwhelming probability; the digest only has to agree across variants)
    idx = torch.arange(1000, n, n // 37, device=dev)[:37]
    t["s"][idx, 0] ^= 1
    p, ok = gpu.verify_batch_device(*(t[k] for k in keys), st, seed)
    print("forged partial digest", hashlib.sha256(p).hexdigest()[:16], "ok", ok, flush=True)


if __name__ == "__main__":
    main()
