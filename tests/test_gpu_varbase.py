"""Custom `Parameters` without the fixed-base combs: every BatchVerifier entry
carries its own (g, h) (batch.rs:52, gadgets.rs:77-103), and a per-proof call of at most
var_base_max proofs (the eight-lane bound: 16384 on MI355X) on a pair whose combs are not cached
verifies [s'] g and [s'] h from the pair's 128-entry Niels tables -- k_verify_wide's
variable-base waves up to 512 proofs, k_verify_small up to 2048, k_verify_quad<kVar> above --
instead of building 128 MiB of combs.  Every status is compared with the oracle's verify_one
under the entry's own generators; the context's stage 13 counts the light table builds and
stage 7 (the comb builds) stays at zero."""
import hashlib

import numpy as np
import pytest

import chaum_pedersen as cp
import pyoracle as O

pytestmark = pytest.mark.gpu

VARBASE_MAX = 16384


def _pairs(k, tag=b"pair"):
    """k distinct custom generator pairs (g_i = [a_i] B, h_i = [b_i] B)."""
    out = []
    for i in range(k):
        a = O.scalar_wide(hashlib.sha512(tag + b"-g-%d" % i).digest())
        b = O.scalar_wide(hashlib.sha512(tag + b"-h-%d" % i).digest())
        out.append(cp.Parameters(O.ristretto_encode(O.pt_mul(O.BASEPOINT, a)),
                                 O.ristretto_encode(O.pt_mul(O.BASEPOINT, b))))
    return out


def _prove_grouped(gpu, pairs, groups, ctxs, seed=b"vb"):
    n = len(groups)
    rows = {q: np.zeros((n, 32), np.uint8) for q in ("y1", "y2", "r1", "r2", "s")}
    for p in range(len(pairs)):
        idx = np.nonzero(groups == p)[0]
        if len(idx) == 0:
            continue
        x = [O.bench_scalar(seed + b"x", int(i)) for i in idx]
        k = [O.bench_scalar(seed + b"k", int(i)) for i in idx]
        out = gpu.prove(x, k, contexts=[ctxs[i] for i in idx], params=pairs[p])
        for q in rows:
            rows[q][idx] = out[q]
    return rows


def _forge(rows, ctxs, n, every=13):
    """s + 1, a replayed context and another entry's statement, spread over the batch."""
    kinds = {}
    for j, i in enumerate(range(3, n, every)):
        kind = ("s+1", "ctx", "stmt")[j % 3]
        if kind == "s+1":
            v = (int.from_bytes(rows["s"][i].tobytes(), "little") + 1) % O.L
            rows["s"][i] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
        elif kind == "ctx":
            ctxs[i] = b"replayed-" + (ctxs[i] or b"")
        else:
            j2 = (i + 1) % n
            rows["y1"][i], rows["y2"][i] = rows["y1"][j2].copy(), rows["y2"][j2].copy()
        kinds[i] = kind
    return kinds


def _oracle(pairs, groups, rows, ctxs):
    import coracle
    return np.array([coracle.verify_one(pairs[int(groups[i])].g, pairs[int(groups[i])].h,
                                        *(rows[q][i].tobytes() for q in ("y1", "y2", "r1", "r2", "s")), ctx=ctxs[i])
                     for i in range(len(groups))], np.uint8)


@pytest.mark.parametrize("npairs", [1, 8, 64])
def test_batch_verifier_over_many_pairs_builds_no_comb(gpu, npairs):
    """1000 BatchVerifier entries over npairs distinct (g, h): each Parameters group is one
    per-proof call (gpu.rs), served from variable-base tables; statuses equal the oracle's."""
    n = 1000
    pairs = _pairs(npairs)
    rng = np.random.default_rng(npairs)
    groups = rng.integers(0, npairs, n)
    ctxs = [None if i % 3 == 0 else b"user-%d-session" % i for i in range(n)]
    rows = _prove_grouped(gpu, pairs, groups, ctxs)
    kinds = _forge(rows, ctxs, n)
    exp = _oracle(pairs, groups, rows, ctxs)
    assert set(exp[list(kinds)].tolist()) == {1} and (exp == 0).sum() == n - len(kinds)
    with cp.Gpu(0) as fresh:   # no comb of these pairs cached
        fresh.set_timing(True)
        fresh.stage_times()
        b = cp.BatchVerifier(fresh)
        for i in range(n):
            p = pairs[int(groups[i])]
            b.add_with_context(p, cp.Statement(rows["y1"][i].tobytes(), rows["y2"][i].tobytes()),
                               cp.Proof(rows["r1"][i].tobytes(), rows["r2"][i].tobytes(), rows["s"][i].tobytes()),
                               ctxs[i])
        res = b.verify()
        st = fresh.stage_times()
        got = np.array([r.status for r in res], np.uint8)
        assert np.array_equal(got, exp), (np.nonzero(got != exp)[0][:8], got[got != exp][:8])
        assert st.get("generators", (0.0, 0))[1] == 0, st             # no 128 MiB comb built
        assert st.get("generators_varbase", (0.0, 0))[1] == len(set(groups.tolist())), st
        # a second pass reuses the cached light sets: nothing is built
        assert [r.status for r in b.verify()] == got.tolist()
        assert "generators_varbase" not in fresh.stage_times()


def test_varbase_statuses_equal_comb_path_on_malformed_entries(gpu, golden):
    """The same custom-pair batch through the variable-base path (fresh context) and through
    the comb path (a context that built the pair's combs for the prover): every decode-level
    status (undecodable point, s >= l, zero s, identity commitment), challenge-bound forgery and
    caller-challenge result agrees, and agrees with the oracle."""
    cg = golden["custom_generators"]
    params = cp.Parameters(bytes.fromhex(cg["g"]), bytes.fromhex(cg["h"]))
    n = 300
    ctxs = [None if i % 2 else bytes([i % 251]) * 32 for i in range(n)]
    rows = _prove_grouped(gpu, [params], np.zeros(n, np.int64), ctxs, seed=b"vbm")
    kinds = _forge(rows, ctxs, n, every=17)
    bad = bytes.fromhex(golden["rfc9496_bad"][0])
    rows["r1"][10] = np.frombuffer(bad, np.uint8)                        # undecodable r1
    rows["y2"][11] = np.frombuffer(bad, np.uint8)                        # undecodable y2
    v = int.from_bytes(rows["s"][12].tobytes(), "little") + O.L          # s + l: not canonical
    rows["s"][12] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
    rows["s"][13] = 0                                                    # zero s
    rows["r2"][14] = 0                                                   # identity commitment
    cols = [rows[q] for q in ("y1", "y2", "r1", "r2", "s")]
    comb = gpu.verify_each(*cols, contexts=ctxs, params=params)          # gpu built the combs (prove)
    with cp.Gpu(0) as fresh:
        fresh.set_timing(True)
        fresh.stage_times()
        light = fresh.verify_each(*cols, contexts=ctxs, params=params)
        light_eq = fresh.verify_each(*cols, contexts=ctxs, params=params, equations_only=True)
        c = fresh.challenges(*cols[:4], contexts=ctxs, params=params)
        resp = fresh.verify_response(*cols, c, params=params)
        st = fresh.stage_times()
    assert np.array_equal(light, comb)
    assert st.get("generators", (0.0, 0))[1] == 0 and st.get("generators_varbase", (0.0, 0))[1] == 1
    exp = np.array([O.verify_one(O.ProofRecord(*(rows[q][i].tobytes() for q in ("y1", "y2", "r1", "r2", "s")),
                                                ctx=ctxs[i]), g_bytes=params.g, h_bytes=params.h)
                    if i in (10, 11, 12, 13, 14) else 0 for i in range(n)], np.uint8)
    for i in kinds:
        exp[i] = 1
    assert np.array_equal(light, exp), (np.nonzero(light != exp)[0], light[light != exp], exp[light != exp])
    assert light[10] == cp.STATUS_BAD_POINT and light[11] == cp.STATUS_BAD_POINT
    assert light[12] == cp.STATUS_BAD_SCALAR and light[13] == cp.STATUS_ZERO_S and light[14] == cp.STATUS_IDENTITY
    # equations only (Proof::new values): zero s and the identity commitment are judged by the equations
    assert light_eq[13] == 1 and light_eq[14] == 1 and light_eq[12] == cp.STATUS_BAD_SCALAR
    # caller challenges = the transcript's own (Verifier::verify_response): the same statuses
    assert np.array_equal(resp, light)


def test_light_set_bound_follows_the_devices_slab(gpu, monkeypatch):
    """the light-set threshold is the runtime's eight-lane bound (verify_quad_max:
    kQuadVerifyMax capped by one verify slab's tables, full * 128 proofs), not the constant
    16384.  A context sized as on a 110-CU part (CPZ_CUS=110: bound 14080) verifies a custom
    pair's call of 14080 proofs from the light set and one of 14081 .. 16384 proofs (which
    used to fail with hipErrorInvalidValue) by building the pair's combs; every status equals
    the forged set."""
    pair = _pairs(1, tag=b"cus110")[0]
    n = 15000
    rng = np.random.default_rng(110)
    x = rng.integers(0, 256, (n, 32), dtype=np.uint8)   # taken mod l by cpz_prove
    k = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    rows = gpu.prove(x, k, params=pair)
    forged = list(range(5, n, 997))
    for i in forged:
        v = (int.from_bytes(rows["s"][i].tobytes(), "little") + 1) % O.L
        rows["s"][i] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
    monkeypatch.setenv("CPZ_CUS", "110")
    for m, light in ((14080, True), (14081, False), (n, False)):
        cols = [np.ascontiguousarray(rows[q][:m]) for q in ("y1", "y2", "r1", "r2", "s")]
        with cp.Gpu(0) as small:
            small.set_timing(True)
            small.stage_times()
            st = small.verify_each(*cols, params=pair)
            stg = small.stage_times()
        exp = np.zeros(m, np.uint8)
        exp[[i for i in forged if i < m]] = 1
        assert np.array_equal(st, exp), (m, np.nonzero(st != exp)[0][:8])
        assert stg.get("generators_varbase", (0.0, 0))[1] == (1 if light else 0), (m, stg)
        assert stg.get("generators", (0.0, 0))[1] == (0 if light else 1), (m, stg)
