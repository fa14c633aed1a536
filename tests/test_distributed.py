"""The multi-GPU data path on CPU: world_size-2 `gloo` process group, shard ranges,
all-gather of 32-byte partials, and the sharding invariant -- partials of shards keyed
by global index sum to the whole-batch partial (computed here by the CPU oracle)."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_ranges_cover_and_align():
    from chaum_pedersen.shard import shard_range
    for n in (1, 255, 256, 1000, 1 << 20, (1 << 26) + 3):
        for world in (1, 2, 3, 4, 8):
            rs = [shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and a <= b
            for a, _ in rs:
                assert a % 256 == 0 or a == n


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import pyoracle as O
    from chaum_pedersen.shard import all_gather_partials, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = [O.prove(O.bench_scalar(b"x", 300 + i), O.bench_scalar(b"k", 300 + i)) for i in range(6)]
        bad = recs[4]
        recs[4] = O.ProofRecord(bad.y1, bad.y2, bad.r1, bad.r2, O.scalar_bytes(int.from_bytes(bad.s, "little") + 1))
        seed = b"\x05" * 32
        lo, hi = shard_range(len(recs), world, rank, align=1)
        mine = O.ristretto_encode(O.rlc_partial(recs[lo:hi], seed, base_index=lo))
        parts = all_gather_partials(mine)
        total = O.IDENTITY
        for p in parts:
            total = O.pt_add(total, O.ristretto_decode(p))
        whole = O.rlc_partial(recs, seed, base_index=0)
        q.put((rank, O.ristretto_encode(total) == O.ristretto_encode(whole), len(parts)))
    finally:
        dist.destroy_process_group()


def test_gloo_partial_gather_matches_whole_batch():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True, 2), (1, True, 2)]
