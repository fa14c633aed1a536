"""The multi-GPU RLC path with HIP partials: two ranks (gloo process group; both on cuda:0,
the only device of the test box) each reduce their shard of a forged batch to a 32-byte
partial on the GPU (weights keyed by the global index), all-gather them with
chaum_pedersen.shard.all_gather_partials (bench.py's code path) and combine them on the
device; the result equals the single-process whole-batch partial, and the per-proof
shards' statuses concatenate to the whole batch's.  (RCCL's "nccl" backend cannot put two
ranks on one GPU; the driver's 8-GPU run exercises it.)"""
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = (1 << 16) + 300
FORGED = [17, 30000, 40001, N - 1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(gpu):
    import hashlib
    import numpy as np
    rows = gpu.prove_synthetic(N, hashlib.sha256(b"dist-x").digest(), hashlib.sha256(b"dist-k").digest())
    rows = {k: np.ascontiguousarray(v) for k, v in rows.items()}
    L = 2**252 + 27742317777372353535851937790883648493
    for i in FORGED:
        v = (int.from_bytes(rows["s"][i].tobytes(), "little") + 1) % L
        rows["s"][i] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
    return rows


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import chaum_pedersen as cp
    from chaum_pedersen.shard import all_gather_partials, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        gpu = cp.Gpu(0)
        rows = _rows(gpu)
        lo, hi = shard_range(N, world, rank)
        d = {k: torch.from_numpy(v[lo:hi].copy()).cuda() for k, v in rows.items()}
        st = torch.empty(hi - lo, dtype=torch.uint8, device="cuda:0")
        seed = bytes(range(32))
        partial, ok = gpu.verify_batch_device(d["y1"], d["y2"], d["r1"], d["r2"], d["s"], st, seed, first_index=lo,
                                              fallback=True)
        parts = all_gather_partials(partial)
        total, ident = gpu.combine_partials(parts)
        bad = [lo + int(i) for i in torch.nonzero(st).flatten().cpu().tolist()]
        q.put((rank, parts, total, ident, ok, bad))
        gpu.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_hip_partials_gather_and_combine(gpu):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    rows = _rows(gpu)
    whole, ok, st = gpu.verify_batch(*(rows[k] for k in ("y1", "y2", "r1", "r2", "s")), seed=bytes(range(32)))
    assert not ok and sorted(i for i in range(N) if st[i]) == FORGED
    (r0, parts0, total0, id0, ok0, bad0), (r1, parts1, total1, id1, ok1, bad1) = res
    assert parts0 == parts1 and len(parts0) == 2          # every rank gathered both partials
    assert total0 == total1 == whole and not id0 and not id1
    assert not ok0 and not ok1                           # each shard holds a forgery
    assert sorted(bad0 + bad1) == FORGED
