"""RLC batch checks of configs[2] (2^20 proofs) with one or two batches in flight on one GPU.

One in flight: STEPS calls of cpz_verify_batch_device on one context, back to back (what the
bench's `rlc` line times).  K in flight (env K, default 2): K contexts, each driven by its own host thread on
its own stream (the context's own, on its own hardware queue), STEPS calls each -- independent
batches, as a verifier service would run them -- so that one batch's latency-bound tails (bucket
fix-up, reductions, the 240-doubling final) and memory-bound sort can run beside the other
batch's VALU-bound prepare and buckets.  Prints one
JSON line: proofs/s of each mode over all the batches it checked (every batch must pass)."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import chaum_pedersen as cp

    n = int(os.environ.get("N", 1 << 20))
    steps = int(os.environ.get("STEPS", "10"))
    dev = torch.device("cuda", 0)
    k_ctx = int(os.environ.get("K", "2"))
    gpus = [cp.Gpu(0) for _ in range(k_ctx)]
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    gpus[0].prove_synthetic_device(n, bench.SEED_X, bench.SEED_K, t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    torch.cuda.synchronize(dev)
    rows = [t[k] for k in ("y1", "y2", "r1", "r2", "s")]
    # each context on its own stream (the context's, unless TORCH_STREAMS=1 asks for torch streams)
    streams = ([torch.cuda.Stream(dev) for _ in range(k_ctx)] if os.environ.get("TORCH_STREAMS") == "1"
               else [None] * k_ctx)
    status = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(k_ctx)]
    bad = []

    def run(k, count):
        for _ in range(count):
            st = streams[k].cuda_stream if streams[k] is not None else None
            _, ok = gpus[k].verify_batch_device(*rows, status[k], bench.WEIGHT_SEED, stream=st)
            if not ok:
                bad.append(k)

    for k in range(k_ctx):  # warm-up: tables, buffers
        run(k, 2)
    torch.cuda.synchronize(dev)
    out = {"n": n, "steps_per_context": steps}
    t0 = time.perf_counter()
    run(0, steps)
    torch.cuda.synchronize(dev)
    el1 = time.perf_counter() - t0
    out["one_in_flight"] = {"batches": steps, "ms_per_batch": el1 * 1e3 / steps, "proofs_per_s": n * steps / el1}
    th = [threading.Thread(target=run, args=(k, steps)) for k in range(k_ctx)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize(dev)
    el2 = time.perf_counter() - t0
    out["k_in_flight"] = {"k": k_ctx, "batches": k_ctx * steps, "ms_per_batch": el2 * 1e3 / (k_ctx * steps),
                          "proofs_per_s": k_ctx * n * steps / el2}
    out["ratio"] = out["k_in_flight"]["proofs_per_s"] / out["one_in_flight"]["proofs_per_s"]
    out["all_passed"] = not bad and all(int((s != 0).sum().item()) == 0 for s in status)
    print(json.dumps(out))
    if not out["all_passed"]:
        raise SystemExit("a valid batch was rejected")


if __name__ == "__main__":
    main()
