"""Parity at the configs' full sizes against the C oracle (oracle/cpz_oracle.c, the at-scale
checker; test infrastructure only):

* C2 (configs[1]): 2^20 proofs, a quarter with 32-byte transcript contexts (the service's
  challenge ids), a 2^16-entry sample carrying every forgery / malformation kind -- s + 1,
  wrong y1, wrong context, undecodable point, non-canonical s, zero s, identity commitment.
  Statuses AND challenges of the whole sample equal the oracle's (batch.rs:185-231,
  transcript.rs:29-71, gadgets.rs:364-489); every entry outside it is valid.
* C3 (configs[2]) shaped like the reference service's batches (service.rs:512-517: every entry
  carries its 32-byte challenge id as transcript context): 2^20 proofs, s + 1 and wrong-context
  forgeries; the batch partial equals the oracle's partial of the forged entries alone and the
  fallback (the failed MSM, then the partitioned check with its locate pass) returns exactly the
  forged set.
* C5 (configs[4]) and C4 (configs[3]): the RLC partial of a forged batch -- whole batch and
  every shard, weights keyed by the global index -- equals, byte for byte, the oracle's
  partial computed from the forged entries ALONE (valid entries contribute the identity, so
  the CPU needs only those), for 2^24 proofs with 16,777 forged and 2^26 proofs as 8 shards.
"""
import hashlib
import os

import numpy as np
import pytest

import coracle as C
import pyoracle as O

pytestmark = pytest.mark.gpu

SX = hashlib.sha256(b"cpz-bench-x").digest()
SK = hashlib.sha256(b"cpz-bench-k").digest()
WSEED = hashlib.sha256(b"cpz-weights-v1").digest()
KEYS = ("y1", "y2", "r1", "r2", "s")


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


def _le(b):
    return int.from_bytes(bytes(b), "little")


def test_c2_sample_every_forgery_kind(gpu, golden):
    _every_forgery_kind(gpu, golden, 1 << 20, 1 << 16, 20)


@pytest.mark.parametrize("n", [16383, 16384, 16385])
def test_small_batch_eight_lanes_every_forgery_kind(gpu, golden, n):
    """Launches of at most 16384 proofs are verified on eight lanes per proof (k_verify_quad,
    a quad per equation), larger ones on one lane per proof (k_verify_each): on both sides of
    the limit every entry's status and challenge equal the C oracle's, with a quarter of the
    entries carrying one of the seven forgery / malformation kinds."""
    _every_forgery_kind(gpu, golden, n, n, 7 + n)


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 100, 2047, 2048, 2049])
def test_small_kernel_every_forgery_kind_and_context_shape(gpu, golden, n):
    """Launches of at most 2048 proofs compute the transcript challenge inside the verify
    kernel (fixed schedules for no context and 32-byte contexts, the byte-wise sponge for
    Some(b"") and other lengths): up to 512 proofs k_verify_wide (a six-wave workgroup per
    proof), then k_verify_small (three waves per 8 proofs).  On both sides of the 2048 limit
    and at the 8-proof workgroup edges every status and challenge equals the C oracle's."""
    _every_forgery_kind(gpu, golden, n, n, 31 + n, ctx_shapes=True)


@pytest.mark.parametrize("n", [3, 511, 512, 513])
def test_wide_kernel_boundary_every_forgery_kind(gpu, golden, n):
    """k_verify_wide (field products on 16-lane rows, csrc/fe16.h) takes launches of at most
    512 proofs, k_verify_small the next: on both sides of the limit, every forgery kind and
    context shape, every status and challenge equals the C oracle's."""
    _every_forgery_kind(gpu, golden, n, n, 57 + n, ctx_shapes=True)


def _every_forgery_kind(gpu, golden, n, nsample, seed, ctx_shapes=False):
    rng = np.random.default_rng(seed)
    if ctx_shapes:   # none, 32 bytes (fixed schedules), Some(b"") and 1..80 bytes (the sponge)
        ctxs = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() if i % 4 == 0 else
                (b"" if i % 4 == 1 else (rng.integers(0, 256, int(rng.integers(1, 81)), dtype=np.uint8).tobytes()
                                         if i % 4 == 2 else None)) for i in range(n)]
    else:
        ctxs = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() if i % 4 == 0 else None for i in range(n)]
    rows = gpu.prove_synthetic(n, SX, SK, contexts=ctxs)
    rows = {k: np.ascontiguousarray(rows[k]) for k in KEYS}
    sample = np.sort(rng.choice(n, size=nsample, replace=False))
    forged = sample[rng.random(sample.size) < 0.25]
    kinds = ("s_plus_1", "wrong_y1", "wrong_context", "bad_point", "s_plus_l", "zero_s", "identity_r")
    bad_pts = [bytes.fromhex(e) for e in golden["rfc9496_bad"]]
    expect_kind = {}
    y1_orig = rows["y1"].copy()
    for j, i in enumerate(forged):
        kind = kinds[j % len(kinds)]
        expect_kind[int(i)] = kind
        if kind == "s_plus_1":
            rows["s"][i] = np.frombuffer(((_le(rows["s"][i]) + 1) % O.L).to_bytes(32, "little"), np.uint8)
        elif kind == "wrong_y1":
            rows["y1"][i] = y1_orig[(i + 1) % n]
        elif kind == "wrong_context":
            ctxs[i] = b"replayed-" + bytes(8) if ctxs[i] is None else bytes(32)
        elif kind == "bad_point":
            rows[("y1", "y2", "r1", "r2")[j % 4]][i] = np.frombuffer(bad_pts[j % len(bad_pts)], np.uint8)
        elif kind == "s_plus_l":
            rows["s"][i] = np.frombuffer((_le(rows["s"][i]) + O.L).to_bytes(32, "little"), np.uint8)
        elif kind == "zero_s":
            rows["s"][i] = 0
        else:
            rows["r2" if j % 2 else "r1"][i] = 0
    st = gpu.verify_each(*(rows[k] for k in KEYS), contexts=ctxs)
    c = gpu.challenges(*(rows[k] for k in KEYS[:4]), contexts=ctxs)
    sub = {k: rows[k][sample] for k in KEYS}
    sub_ctx = [ctxs[i] for i in sample]
    t = _threads()
    st_o = C.verify_many_ctx(sub, sub_ctx, threads=t)
    c_o = C.challenge_many(sub, sub_ctx, threads=t)
    mism = np.nonzero(st[sample] != st_o)[0]
    assert mism.size == 0, [(int(sample[m]), expect_kind.get(int(sample[m])), int(st[sample[m]]), int(st_o[m]))
                            for m in mism[:10]]
    assert np.array_equal(c[sample], c_o)
    outside = np.setdiff1d(np.arange(n), sample)
    assert not st[outside].any()
    # every kind occurred and produced its reference status
    want = {"s_plus_1": {1}, "wrong_y1": {1}, "wrong_context": {1}, "bad_point": {2}, "s_plus_l": {3},
            "zero_s": {5}, "identity_r": {4}}
    seen = {}
    for i, kind in expect_kind.items():
        seen.setdefault(kind, set()).add(int(st[i]))
    if len(forged) >= 2 * len(kinds):
        assert seen == want, seen
    else:
        assert all(seen[k] == want[k] for k in seen), seen
    assert np.array_equal(np.nonzero(st)[0], np.sort(forged))


def _synthetic_device(gpu, torch, n):
    dev = torch.device("cuda:0")
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in KEYS}
    gpu.prove_synthetic_device(n, SX, SK, t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    return t


def _forge(t, torch, idx):
    """Half s := s + 1, half y1 := another proof's y1 (device rows, in place); returns the
    forged rows as host arrays (what the CPU checker needs)."""
    n = t["s"].shape[0]
    bump, swap = idx[0::2], idx[1::2]
    sel = torch.from_numpy(bump.astype(np.int64)).to("cuda:0")
    rows = t["s"].index_select(0, sel).cpu().numpy()
    for r in range(rows.shape[0]):
        rows[r] = np.frombuffer(((_le(rows[r]) + 1) % O.L).to_bytes(32, "little"), np.uint8)
    t["s"].index_copy_(0, sel, torch.from_numpy(rows).to("cuda:0"))
    dst = torch.from_numpy(swap.astype(np.int64)).to("cuda:0")
    src = torch.from_numpy(((swap + 7) % n).astype(np.int64)).to("cuda:0")
    t["y1"].index_copy_(0, dst, t["y1"].index_select(0, src).clone())
    allsel = torch.from_numpy(idx.astype(np.int64)).to("cuda:0")
    return {k: t[k].index_select(0, allsel).cpu().numpy() for k in KEYS}


def _oracle_partial(host, gidx, lo=None, hi=None):
    m = np.ones(len(gidx), bool) if lo is None else (gidx >= lo) & (gidx < hi)
    if not m.any():
        return bytes(32)
    enc, live = C.rlc_partial({k: host[k][m] for k in KEYS}, gidx[m], WSEED, threads=_threads())
    assert live == int(m.sum())
    return enc


def test_c3_service_contexts_partial_and_located_set(gpu):
    n = 1 << 20
    rng = np.random.default_rng(33)
    ctxs = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(n)]
    rows = gpu.prove_synthetic(n, SX, SK, contexts=ctxs)
    rows = {k: np.ascontiguousarray(rows[k]) for k in KEYS}
    # few forgeries, spread out: the density probe (with contexts) sees at most one, so the
    # batch MSM runs first; it fails, and the fallback is the partitioned check (every block's
    # partial over the points just prepared, each failing block's one forgery located)
    forged = np.sort(rng.choice(n, size=24, replace=False))
    for j, i in enumerate(forged):
        if j % 2:
            ctxs[i] = bytes(32)  # replayed under another challenge id
        else:
            rows["s"][i] = np.frombuffer(((_le(rows["s"][i]) + 1) % O.L).to_bytes(32, "little"), np.uint8)
    partial, ok, st = gpu.verify_batch(*(rows[k] for k in KEYS), seed=WSEED, contexts=ctxs)
    stats = gpu.fallback_stats()
    assert not ok
    assert np.array_equal(np.nonzero(st)[0], forged) and set(st[forged].tolist()) == {1}
    assert stats["path"] == "partitioned" and stats["probe_invalid"] <= 1, stats
    blk = _part_block(n, stats)
    nfail, one, want_pp = _locate_expect(forged, blk, n)
    assert stats["blocks_failing"] == nfail and stats["blocks_located"] == one and stats["per_proof"] == want_pp
    sub = {k: rows[k][forged] for k in KEYS}
    want, live = C.rlc_partial(sub, forged, WSEED, contexts=[ctxs[i] for i in forged], threads=_threads())
    assert live == forged.size
    assert partial == want


def test_c5_partial_from_forged_entries_alone(gpu):
    torch = pytest.importorskip("torch")
    n, nf = 1 << 24, 16_777
    t = _synthetic_device(gpu, torch, n)
    idx = np.sort(np.random.default_rng(2024).choice(n, size=nf, replace=False))
    host = _forge(t, torch, idx)
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    whole, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED)
    assert not ok
    assert whole == _oracle_partial(host, idx)
    shards = 8
    per = n // shards
    for k in range(shards):
        lo, hi = k * per, (k + 1) * per
        p, _ = gpu.verify_batch_device(*(t[q][lo:hi] for q in KEYS), st[lo:hi], WSEED, first_index=lo)
        assert p == _oracle_partial(host, idx, lo, hi), k


def test_c4_shard_partials_from_forged_entries_alone(gpu):
    torch = pytest.importorskip("torch")
    n, shards = 1 << 26, 8
    per = n // shards
    t = _synthetic_device(gpu, torch, n)
    rng = np.random.default_rng(26)
    idx = np.sort(np.concatenate([rng.choice(np.arange(2 * per, 3 * per), 300, replace=False),
                                  rng.choice(np.arange(5 * per, 6 * per), 200, replace=False),
                                  np.array([n - 1])]))
    host = _forge(t, torch, idx)
    st = torch.empty(per, dtype=torch.uint8, device="cuda:0")
    parts = []
    for k in range(shards):
        lo, hi = k * per, (k + 1) * per
        p, ok = gpu.verify_batch_device(*(t[q][lo:hi] for q in KEYS), st, WSEED, first_index=lo)
        assert p == _oracle_partial(host, idx, lo, hi), k
        assert ok == (p == bytes(32))
        parts.append(p)
    total, ident = gpu.combine_partials(parts)
    assert not ident and total == _oracle_partial(host, idx)


def test_fallback_probe_sparse_and_dense(gpu):
    """Fallback-enabled batch checks of 2^21 proofs: three forgeries (the density probe sees
    none -> MSM, which fails, then the partitioned check with the locate pass: exact set, and
    the partial equals the oracle's partial of the three), then 1 % forged (the probe sees
    several -> MSM skipped: exact set, partial_out 0xff...ff, batch not ok)."""
    torch = pytest.importorskip("torch")
    n = 1 << 21
    t = _synthetic_device(gpu, torch, n)
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    sparse = np.array([12345, 1_000_001, n - 2])
    host = _forge(t, torch, sparse)
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    stats = gpu.fallback_stats()
    assert not ok and p == _oracle_partial(host, sparse)
    got = st.cpu().numpy()
    assert np.array_equal(np.nonzero(got)[0], sparse) and set(got[sparse].tolist()) == {1}
    assert stats["path"] == "partitioned" and stats["blocks_located"] == 3 and stats["per_proof"] == 3, stats
    dense = np.sort(np.random.default_rng(7).choice(np.setdiff1d(np.arange(n), sparse), n // 100, replace=False))
    _forge(t, torch, dense)
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    assert not ok and p == b"\xff" * 32
    got = st.cpu().numpy()
    want = np.sort(np.concatenate([sparse, dense]))
    assert np.array_equal(np.nonzero(got)[0], want) and set(got[want].tolist()) == {1}
    # without a fallback the partial is always computed
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED)
    assert not ok and p != b"\xff" * 32 and p != bytes(32)


def test_spans_forged_only_in_a_later_span(gpu):
    """A 2^23-proof batch is checked as four MSMs of 2^21-proof spans (rlc_range), each
    span's P added on the device.  Forgeries ONLY in span 2: the batch partial must be the
    oracle's partial of those entries (an identity partial here would accept a forged batch),
    the batch must fail, and the fallback must return exactly the forged set.  Also checked
    for the same span as a batch of its own (first_index = its global start) and for spans
    0..1 alone (valid: identity, batch ok).  The fallback is span-local: each span's final
    records whether its own P is the identity, and only the failing span is searched."""
    torch = pytest.importorskip("torch")
    n, span = 1 << 23, 1 << 21
    t = _synthetic_device(gpu, torch, n)
    rng = np.random.default_rng(232)
    idx = np.sort(rng.choice(np.arange(2 * span, 3 * span), 40, replace=False))
    host = _forge(t, torch, idx)
    want = _oracle_partial(host, idx)
    assert want != bytes(32)
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED)
    assert not ok and p == want
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    assert not ok and p == want
    got = st.cpu().numpy()
    assert np.array_equal(np.nonzero(got)[0], idx) and set(got[idx].tolist()) == {1}
    # span-local fallback: only span 2's own P failed, so only span 2 is searched (no
    # partitioned pass over the whole batch's blocks)
    fb = gpu.fallback_stats()
    assert fb["path"] == "bisection" and fb["blocks_checked"] == 0, fb
    assert fb["per_proof"] <= span, fb
    lo, hi = 2 * span, 3 * span
    p, ok = gpu.verify_batch_device(*(t[k][lo:hi] for k in KEYS), st[lo:hi], WSEED, first_index=lo)
    assert not ok and p == want
    p, ok = gpu.verify_batch_device(*(t[k][:lo] for k in KEYS), st[:lo], WSEED)
    assert ok and p == bytes(32)


def _part_block(n, stats):
    """The partitioned check's block size (128 or 256 proofs), from the blocks it checked."""
    b = 1
    while b * stats["blocks_checked"] < n:
        b <<= 1
    assert b in (128, 256) and -(-n // b) == stats["blocks_checked"], (n, stats)
    return b


def _blocks_with(idx, b):
    return np.unique(np.asarray(idx) // b)


def _locate_expect(idx, b, n):
    """(failing blocks, blocks the locate pass finds, entries verified per proof): a failing
    block with exactly one forged entry is located and that entry alone verified per proof;
    a block with more is verified whole (rlc.h, the index-weighted partial)."""
    blocks, counts = np.unique(np.asarray(idx) // b, return_counts=True)
    one = int((counts == 1).sum())
    whole = sum(min(b, n - b * int(k)) for k, c in zip(blocks, counts) if c > 1)
    return blocks.size, one, one + whole


@pytest.mark.parametrize("n", [1 << 22, (1 << 20) + 77])
def test_partitioned_fallback_at_c5_density(gpu, n):
    """configs[4]'s density (0.1 % forged, half s + 1, half wrong y1) through the batch check
    with its fallback: the density probe sees a few invalid samples, so the fallback is the
    partitioned check -- every block's RLC partial (128 or 256 proofs), then per-proof verification of
    the failing blocks ONLY.  Checked: the exact forged set (statuses 1 there, 0 elsewhere);
    the batch partial equals the C oracle's partial of the forged entries alone; the path
    taken; the failing blocks are exactly the blocks holding a forgery; and no entry of a
    clean block is verified per proof: a failing block holding one forgery is located by its
    index-weighted partial and only that entry is verified per proof, a block holding more is
    verified whole.  The ragged size puts a forgery in the partial last block."""
    torch = pytest.importorskip("torch")
    t = _synthetic_device(gpu, torch, n)
    rng = np.random.default_rng(4242 + n)
    idx = np.sort(rng.choice(n - 1, size=max(8, n // 1000) - 1, replace=False))
    idx = np.union1d(idx, [n - 1])
    host = _forge(t, torch, idx)
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    stats = gpu.fallback_stats()
    got = st.cpu().numpy()
    assert not ok
    assert np.array_equal(np.nonzero(got)[0], idx) and set(got[idx].tolist()) == {1}
    assert stats["path"] == "partitioned", stats
    B = _part_block(n, stats)
    dirty = _blocks_with(idx, B)
    assert stats["blocks_failing"] == dirty.size, (stats, dirty.size)
    nfail, one, want_pp = _locate_expect(idx, B, n)
    assert stats["blocks_indexed"] == nfail and stats["blocks_located"] == one, stats
    assert stats["per_proof"] == want_pp, stats
    assert p == _oracle_partial(host, idx)


def test_two_contexts_in_flight_on_one_gpu(gpu):
    """Two contexts on one GPU, each driven by its own host thread on its own stream (the
    contexts' streams have hardware queues of their own, so their kernels run concurrently):
    batch checks of two different batches -- one valid, one with forgeries -- issued back to back
    from both threads give every call its own batch's result: the valid batch passes with the
    identity partial, the forged one fails with the oracle's partial of its forged entries and
    (with the fallback) exactly its forged set.  Guards the per-context buffers and ordering
    when the two contexts' work overlaps on the device."""
    import threading

    import chaum_pedersen as cp
    torch = pytest.importorskip("torch")
    n = 1 << 18
    good = _synthetic_device(gpu, torch, n)
    bad = {k: v.clone() for k, v in good.items()}
    idx = np.sort(np.random.default_rng(77).choice(n, size=10, replace=False))
    host = _forge(bad, torch, idx)
    want = _oracle_partial(host, idx)
    other = cp.Gpu(0)
    out = {0: [], 1: []}

    def run(k, g, rows):
        st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        for _ in range(4):
            p, ok = g.verify_batch_device(*(rows[key] for key in KEYS), st, WSEED, fallback=(k == 1), stream=0)
            out[k].append((p, ok, st.cpu().numpy().copy()))

    try:
        th = [threading.Thread(target=run, args=(0, gpu, good)), threading.Thread(target=run, args=(1, other, bad))]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        other.close()
    assert len(out[0]) == 4 and len(out[1]) == 4
    for p, ok, st in out[0]:
        assert ok and p == bytes(32) and not st.any()
    for p, ok, st in out[1]:
        assert not ok and p == want
        assert np.array_equal(np.nonzero(st)[0], idx) and set(st[idx].tolist()) == {1}


def test_partitioned_fallback_with_service_contexts(gpu):
    """configs[4]'s density on batches shaped like the service's (every entry with a 32-byte
    challenge id as transcript context, service.rs:512-517; batch.rs:262-268): 2^22 proofs,
    0.1 % forged -- half s + 1, half a replayed context (the proof verified under another
    challenge id).  The density probe samples the batch WITH its contexts (k_probe_gather), so
    the fallback is the partitioned check: exact forged set, the C oracle's partial of the
    forged entries (with their contexts), and no clean block verified per proof."""
    torch = pytest.importorskip("torch")
    n = 1 << 22
    dev = "cuda:0"
    gen = torch.Generator(device=dev)
    gen.manual_seed(5151)
    cb = torch.randint(0, 256, (32 * n,), dtype=torch.int32, device=dev, generator=gen).to(torch.uint8)
    co = torch.arange(n + 1, dtype=torch.int64, device=dev) * 32
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in KEYS}
    gpu.prove_synthetic_device(n, SX, SK, t["y1"], t["y2"], t["r1"], t["r2"], t["s"], ctx_bytes=cb, ctx_off=co)
    rng = np.random.default_rng(2222)
    idx = np.sort(rng.choice(n, size=n // 1000, replace=False))
    bump, replay = idx[0::2], idx[1::2]
    sel = torch.from_numpy(bump.astype(np.int64)).to(dev)
    rows = t["s"].index_select(0, sel).cpu().numpy()
    for r in range(rows.shape[0]):
        rows[r] = np.frombuffer(((_le(rows[r]) + 1) % O.L).to_bytes(32, "little"), np.uint8)
    t["s"].index_copy_(0, sel, torch.from_numpy(rows).to(dev))
    cbv = cb.view(n, 32)
    rsel = torch.from_numpy(replay.astype(np.int64)).to(dev)
    cbv.index_copy_(0, rsel, cbv.index_select(0, (rsel + 1) % n).clone())   # another entry's challenge id
    allsel = torch.from_numpy(idx.astype(np.int64)).to(dev)
    host = {k: t[k].index_select(0, allsel).cpu().numpy() for k in KEYS}
    hctx = [bytes(r) for r in cbv.index_select(0, allsel).cpu().numpy()]
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True, ctx_bytes=cb, ctx_off=co)
    stats = gpu.fallback_stats()
    got = st.cpu().numpy()
    assert not ok
    assert np.array_equal(np.nonzero(got)[0], idx) and set(got[idx].tolist()) == {1}
    assert stats["path"] == "partitioned", stats
    B = _part_block(n, stats)
    dirty = _blocks_with(idx, B)
    nfail, one, want_pp = _locate_expect(idx, B, n)
    assert stats["blocks_failing"] == dirty.size == nfail, stats
    assert stats["blocks_located"] == one and stats["per_proof"] == want_pp, stats
    want, live = C.rlc_partial(host, idx, WSEED, contexts=hctx, threads=_threads())
    assert live == idx.size and p == want


def test_partitioned_locate_edges(gpu):
    """The locate pass at its edges (2^20 + 77 proofs, 0.1 % s + 1 / wrong-y1 forgeries plus
    placed ones): a block whose one forgery is its first entry (j = 1) and one whose forgery is
    its last (j = 128 or 256), a block with two and one with three forgeries (no j matches:
    verified whole), and the batch's last entry, in the partial last block.  Exact set, the
    oracle's partial, and the stats' located / whole split."""
    torch = pytest.importorskip("torch")
    n = (1 << 20) + 77
    t = _synthetic_device(gpu, torch, n)
    rng = np.random.default_rng(6060)
    idx = rng.choice(n, size=n // 1000, replace=False)
    B = 256   # placed so that they hold for 128- and 256-proof blocks alike
    free = [b for b in range(64, n // B - 64, 37) if not np.any(idx // B == b)]
    b1, b2, b3, b4 = free[:4]
    placed = [B * b1, B * b2 + B - 1, B * b3 + 5, B * b3 + 9, B * b4 + 100, B * b4 + 101, B * b4 + 200, n - 1]
    idx = np.union1d(idx, placed)
    host = _forge(t, torch, idx)
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    stats = gpu.fallback_stats()
    got = st.cpu().numpy()
    assert not ok and stats["path"] == "partitioned", stats
    assert np.array_equal(np.nonzero(got)[0], idx) and set(got[idx].tolist()) == {1}
    blk = _part_block(n, stats)
    nfail, one, want_pp = _locate_expect(idx, blk, n)
    assert stats["blocks_failing"] == stats["blocks_indexed"] == nfail, stats
    assert stats["blocks_located"] == one and stats["per_proof"] == want_pp, stats
    assert p == _oracle_partial(host, idx)


def test_partitioned_related_forgeries_in_one_block(gpu):
    """Blocks whose forgeries are related: a forged proof copied byte for byte into
    another slot of its block (the same error point, differently weighted), s + 1 and s + 2 on
    two slots (scaled errors), s + 1 and s - 1 on two copies of one proof (opposite errors), and
    three copies of one forged proof.  For a secret seed no index-weighted candidate matches, so
    each such block is verified whole: the exact set, the oracle's partial, and the located /
    whole split of the stats as for independent forgeries."""
    torch = pytest.importorskip("torch")
    n = (1 << 20) + 77
    t = _synthetic_device(gpu, torch, n)
    rng = np.random.default_rng(7171)
    idx = rng.choice(n, size=n // 1000, replace=False)
    B = 256   # placed inside one 128-proof block, whatever the block size
    free = [b for b in range(64, n // B - 64, 41) if not np.any(idx // B == b)]
    b1, b2, b3, b4 = free[:4]
    host = _forge(t, torch, np.sort(idx))

    def copy_row(dst, src):
        for k in KEYS:
            t[k][dst] = t[k][src].clone()

    def add_s(e, delta):
        v = (_le(t["s"][e].cpu().numpy()) + delta) % O.L
        t["s"][e] = torch.from_numpy(np.frombuffer(v.to_bytes(32, "little"), np.uint8).copy()).to("cuda:0")

    related = []
    e = B * b1 + 10                      # the same forged proof in two slots
    add_s(e, 1)
    copy_row(e + 3, e)
    related += [e, e + 3]
    e = B * b2 + 20                      # scaled: s + 1 and s + 2
    add_s(e, 1)
    add_s(e + 7, 2)
    related += [e, e + 7]
    e = B * b3 + 30                      # opposite: s + 1 and s - 1 on two copies of one proof
    copy_row(e + 1, e)
    add_s(e, 1)
    add_s(e + 1, -1)
    related += [e, e + 1]
    e = B * b4 + 40                      # three copies of one forged proof
    add_s(e, 1)
    copy_row(e + 2, e)
    copy_row(e + 5, e)
    related += [e, e + 2, e + 5]
    allf = np.union1d(idx, related)
    sel = torch.from_numpy(allf.astype(np.int64)).to("cuda:0")
    host = {k: t[k].index_select(0, sel).cpu().numpy() for k in KEYS}
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    stats = gpu.fallback_stats()
    got = st.cpu().numpy()
    assert not ok and stats["path"] == "partitioned", stats
    assert np.array_equal(np.nonzero(got)[0], allf) and set(got[allf].tolist()) == {1}
    blk = _part_block(n, stats)
    nfail, one, want_pp = _locate_expect(allf, blk, n)
    assert stats["blocks_failing"] == stats["blocks_indexed"] == nfail, stats
    assert stats["blocks_located"] == one and stats["per_proof"] == want_pp, stats
    assert p == _oracle_partial(host, allf)


def test_partitioned_fallback_decode_failures_and_equations_only(gpu, golden):
    """The partitioned check with entries whose decode-level status is non-zero:
    an undecodable r1, s + l (non-canonical), zero s and an identity r1, placed in blocks that
    are otherwise clean, in failing blocks and in the partial last block, beside 0.1 % s + 1 /
    wrong-y1 forgeries.  Those entries carry zero weight and keep their decode-level status
    (2, 3, 5, 4); the partial is the oracle's over the live forged entries.  Then the same batch
    with commitment checks off: identity r1 and zero s are judged by the equations (status 1,
    and they keep their weight), the others are unchanged."""
    torch = pytest.importorskip("torch")
    n = (1 << 21) + 77
    t = _synthetic_device(gpu, torch, n)
    rng = np.random.default_rng(9191)
    idx = np.sort(rng.choice(n, size=n // 1000, replace=False))
    host = _forge(t, torch, idx)
    B = 128   # spots placed per 128 proofs: inside one block whether blocks are 128 or 256 proofs
    dirty256 = set(int(b) for b in _blocks_with(idx, 256))
    dirty = set(int(b) for b in _blocks_with(idx, B))
    clean = [b for b in range(0, (n + B - 1) // B, 97) if b // 2 not in dirty256][:8]
    last = (n - 1) // B
    spots = []   # (entry, kind): a few per kind in clean blocks, failing blocks and the last block
    for j, b in enumerate(clean + sorted(dirty)[:8] + [last]):
        e = min(n - 1, B * b + 17 + j) if b != last else n - 3
        if e in set(idx.tolist()):
            e = e - 1
        spots.append((e, ("bad_point", "s_plus_l", "zero_s", "identity_r")[j % 4]))
    bad_pt = np.frombuffer(bytes.fromhex(golden["rfc9496_bad"][0]), np.uint8)
    for e, kind in spots:
        if kind == "bad_point":
            t["r1"][e] = torch.from_numpy(bad_pt.copy()).to("cuda:0")
        elif kind == "identity_r":
            t["r1"][e] = 0
        elif kind == "zero_s":
            t["s"][e] = 0
        else:
            v = _le(t["s"][e].cpu().numpy()) + O.L
            t["s"][e] = torch.from_numpy(np.frombuffer(v.to_bytes(32, "little"), np.uint8).copy()).to("cuda:0")
    code = {"bad_point": 2, "s_plus_l": 3, "zero_s": 5, "identity_r": 4}
    st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    p, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
    assert gpu.fallback_stats()["path"] == "partitioned"
    got = st.cpu().numpy()
    want = np.zeros(n, np.uint8)
    want[idx] = 1
    for e, kind in spots:
        want[e] = code[kind]
    assert not ok and np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert p == _oracle_partial(host, idx)
    gpu.set_commitment_checks(False)
    try:
        p2, ok = gpu.verify_batch_device(*(t[k] for k in KEYS), st, WSEED, fallback=True)
        stats = gpu.fallback_stats()
    finally:
        gpu.set_commitment_checks(True)
    for e, kind in spots:
        if kind in ("zero_s", "identity_r"):
            want[e] = 1
    got = st.cpu().numpy()
    assert stats["path"] == "partitioned" and not ok
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert p2 != p   # the two equation-judged entries are weighted now
