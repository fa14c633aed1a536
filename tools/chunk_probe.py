"""Probe: k_verify_each over 2^20 proofs as one call vs calls on 2^k-proof slices (device
tensors).  Prints per-variant kernel ms (HIP-event stage timers).  The launch-size numbers in
DESIGN.md were taken with a single-stream, one-launch-per-call runtime (today's equivalent:
a library built with -DCPZ_VERIFY_STREAMS=1 -DCPZ_VERIFY_CHUNK_DIV=1 and a very large chunk);
with the default runtime every call is itself cut into two-stream launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))


def main():
    import torch
    import chaum_pedersen as cp
    n, steps = 1 << 20, 5
    dev = torch.device("cuda", 0)
    gpu = cp.Gpu(0)
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    gpu.prove_synthetic_device(n, bytes(32), bytes(range(32)), t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    for lg in (20, 19, 18, 17, 16, 15):
        c = 1 << lg

        def run():
            for off in range(0, n, c):
                gpu.verify_each_device(*(t[k][off:off + c] for k in ("y1", "y2", "r1", "r2", "s")),
                                       status[off:off + c])
        run()
        torch.cuda.synchronize()
        gpu.set_timing(True)
        gpu.stage_times()
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        st = gpu.stage_times()
        gpu.set_timing(False)
        assert int(status.sum().item()) == 0
        v = st["verify_each"][0] / steps
        ch = st["challenge"][0] / steps
        print("chunk 2^%d: verify %.3f ms, challenge %.3f ms per 2^20" % (lg, v, ch), flush=True)


if __name__ == "__main__":
    main()
