"""The multi-GPU RLC path with HIP partials: two ranks (gloo process group; both on cuda:0,
the only device of the test box) each reduce their shard of a forged batch to a 32-byte
partial on the GPU (weights keyed by the global index), all-gather them with
chaum_pedersen.shard.all_gather_partials (bench.py's code path) and combine them on the
device; the result equals the single-process whole-batch partial, and the per-proof
shards' statuses concatenate to the whole batch's.  RCCL's "nccl" backend cannot put two
ranks on one GPU: a world of one runs all_gather_partials' RCCL branch here, and the driver's
8-GPU run exercises the exchange itself."""
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


def _dense_worker(rank, world, port, q):
    """Rank 0's shard is 2^21 proofs with 1 % forged (its fallback's density probe skips the
    MSM and reports the no-partial marker 32 x 0xff); rank 1's shard is clean."""
    sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import hashlib
    import numpy as np
    import torch
    import torch.distributed as dist
    import chaum_pedersen as cp
    from chaum_pedersen.shard import all_gather_partials, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        gpu = cp.Gpu(0)
        n = 1 << 22
        lo, hi = shard_range(n, world, rank)
        d = {k: torch.empty((hi - lo, 32), dtype=torch.uint8, device="cuda:0") for k in ("y1", "y2", "r1", "r2", "s")}
        gpu.prove_synthetic_device(hi - lo, hashlib.sha256(b"dense-x").digest(), hashlib.sha256(b"dense-k").digest(),
                                   d["y1"], d["y2"], d["r1"], d["r2"], d["s"], first_index=lo)
        forged = []
        if rank == 0:
            forged = np.sort(np.random.default_rng(5).choice(hi - lo, (hi - lo) // 100, replace=False))
            dst = torch.from_numpy(forged.astype(np.int64)).cuda()
            src = torch.from_numpy(((forged + 7) % (hi - lo)).astype(np.int64)).cuda()
            d["y1"].index_copy_(0, dst, d["y1"].index_select(0, src).clone())
        st = torch.empty(hi - lo, dtype=torch.uint8, device="cuda:0")
        partial, ok = gpu.verify_batch_device(d["y1"], d["y2"], d["r1"], d["r2"], d["s"], st, bytes(range(32)),
                                              first_index=lo, fallback=True)
        parts = all_gather_partials(partial)
        total, ident = gpu.combine_partials(parts)
        bad = torch.nonzero(st).flatten().cpu().numpy()
        q.put((rank, parts, total, ident, ok, bool(np.array_equal(bad, np.asarray(forged, dtype=bad.dtype)))))
        gpu.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_dense_shard_marker_combines(gpu):
    """A dense shard's no-partial marker through the torch.distributed flow
    (all_gather_partials -> combine_partials): the combine reports the marker and "not
    identity" instead of failing on an undecodable partial, on every rank; each rank's
    statuses are exact."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (_, parts0, total0, id0, ok0, exact0), (_, parts1, total1, id1, ok1, exact1) = res
    marker = b"\xff" * 32
    assert parts0 == parts1 and parts0[0] == marker and parts0[1] == bytes(32)
    assert total0 == total1 == marker and not id0 and not id1
    assert not ok0 and ok1 and exact0 and exact1


def _rccl_worker(port, q):
    """World 1 over the "nccl" backend (RCCL): the collective bench.py's N > 1 RLC path runs,
    on the one GPU of the box (RCCL cannot put two ranks on one device)."""
    sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import chaum_pedersen as cp
    from chaum_pedersen.shard import all_gather_partials
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        gpu = cp.Gpu(0)
        rows = _rows(gpu)
        d = {k: torch.from_numpy(v.copy()).cuda() for k, v in rows.items()}
        st = torch.empty(N, dtype=torch.uint8, device="cuda:0")
        partial, ok = gpu.verify_batch_device(d["y1"], d["y2"], d["r1"], d["r2"], d["s"], st, bytes(range(32)),
                                              fallback=True)
        parts = all_gather_partials(partial)
        total, ident = gpu.combine_partials(parts)
        q.put((dist.get_backend(), parts, partial, total, ident, ok))
        gpu.close()
    finally:
        dist.destroy_process_group()


def test_rccl_all_gather_of_partials_world_one(gpu):
    """all_gather_partials' RCCL branch (device tensors, "nccl" backend) -- the exchange of
    configs[3]'s per-GPU partials -- in a world of one rank: the gathered list is the rank's own
    HIP partial, and combining it gives it back."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    backend, parts, partial, total, ident, ok = q.get(timeout=240)
    p.join(timeout=60)
    assert backend == "nccl"
    assert parts == [partial] and total == partial and not ident and not ok


@pytest.mark.parametrize("launcher", ["torchrun", "none"])
def test_bench_rlc_four_rank_rehearsal(launcher):
    """bench.py's multi-rank RLC path (configs[3]'s flow: per-rank shard partials keyed by the
    global index, all-gather, combine) as a world-4 gloo rehearsal on the box's one GPU: the
    combined total of a valid set is the identity, and the line reports no rate.  launcher =
    "none" is the driver's own form, plain `python3 bench.py --gpus 4`: bench.py starts the four
    ranks itself (torch.distributed.run as a child process) and relays rank 0's line."""
    import json
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    args = ["--gpus", "4", "--mode", "rlc", "--n-total", str(1 << 20), "--same-device", "--backend", "gloo",
            "--steps", "1", "--warmup", "1", "--extras", "0", "--no-cpu-baseline", "--c4-n", str(1 << 21),
            "--c4-steps", "1"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=360, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] is None and d["ms_per_step"] is None and d["n_gpus"] == 4
    assert d["rehearsal"]["combined_total_identity"] is True
    assert d["rehearsal"]["combined_total"] == "00" * 32
    # configs[3]'s object at this world size: shards of 2^21 proofs over 4 ranks, identity on the
    # valid set; the forged variant lands in two ranks' shards (ranks 0 and 2), every rank's
    # statuses are exactly its forged entries, and the combined total is not the identity
    c4 = d["c4"]
    assert c4["ok"] is True and c4["identity"] is True and c4["combined_total_valid"] == "00" * 32
    assert c4["proofs_total"] == 1 << 21 and c4["proofs_per_gpu_max"] == 1 << 19
    f = c4["forged"]
    assert f["per_rank_forged"] == [2, 0, 2, 0]
    assert f["statuses_exact_every_rank"] is True and f["combined_total_not_identity"] is True
    assert f["combined_total"] != "00" * 32
    assert c4["proofs_per_s"] is None   # ranks sharing one GPU: no rate
    # the scaling invariant: the four shard partials of the forged variant sum to the partial
    # one process computes over the whole 2^21 proofs (weights keyed by the global index)
    if launcher == "none":
        one = [sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "rlc", "--n-total", str(1 << 20),
               "--steps", "1", "--warmup", "1", "--extras", "0", "--no-cpu-baseline", "--c4-n", str(1 << 21),
               "--c4-steps", "1"]
        r1 = subprocess.run(one, capture_output=True, text=True, timeout=360, env=env, cwd=ROOT)
        assert r1.returncode == 0, r1.stderr[-3000:]
        d1 = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][0])
        assert d1["n_gpus"] == 1 and d1["c4"]["ok"] is True and d1["c4"]["forged"]["per_rank_forged"] == [4]
        assert d1["c4"]["forged"]["combined_total"] == f["combined_total"]
