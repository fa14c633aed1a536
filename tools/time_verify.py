"""Kernel-timing harness for experiments (variant libraries via CPZ_LIB): times
k_verify_each on 2^20 synthetic proofs with the runtime's HIP-event stage timers and does
NOT check verdicts -- for timing variants that deliberately compute wrong answers.  The
reported bench number always comes from bench.py, which refuses invalid verdicts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))


def main():
    import torch
    import chaum_pedersen as cp
    n, steps = 1 << 20, int(os.environ.get("STEPS", "10"))
    dev = torch.device("cuda", 0)
    gpu = cp.Gpu(0)
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    gpu.prove_synthetic_device(n, bytes(32), bytes(range(32)), t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    for _ in range(2):
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status)
    torch.cuda.synchronize()
    gpu.set_timing(True)
    gpu.stage_times()
    for _ in range(steps):
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status)
    torch.cuda.synchronize()
    st = gpu.stage_times()
    v_ms, v_cnt = st.get("verify_each", (0.0, 1))
    print("%-14s verify_each %.3f ms  rejected %d" % (os.path.basename(os.environ.get("CPZ_LIB", "default")),
                                                     v_ms / v_cnt, int((status != 0).sum().item())))


if __name__ == "__main__":
    main()
