"""The drop-in's own regime: BatchVerifier batches of n <= 1000 (batch.rs:48) served through
the call sequence rust/reference-patch/gpu.rs issues, exercised through its C++ mirror
(include/cpz_batch.hpp, tests/cpp/dropin_test.cpp):

  * entries grouped by Parameters in order of first appearance (two interleaved groups here:
    the default generators and the golden custom pair);
  * a one-entry batch (verify_one, batch.rs:178-180) leaves the rng untouched: its RLC check
    is keyed by a seed from the OS entropy source;
  * otherwise the rng is drawn as the reference draws it, one 64-byte random_scalar per entry
    (batch.rs:239-240), whatever entry point each group takes; the first draw's first 32
    bytes key every group's RLC check,
    groups take consecutive weight indices (first_index = entries of the earlier groups),
    groups of >= rlc_min_group entries run cpz_verify_batch_ex, smaller ones
    cpz_verify_each_ex; every call passes CPZ_CALL_EQUATIONS_ONLY (Proof values).

Every entry's result is compared with the oracle's verify_one (commitment checks off, as the
reference's verify_one judges a Proof value: a nonce-0 proof with identity commitments is
valid), and every RLC group's partial with the C oracle's partial of that group at the same
seed and global indices (valid entries contribute the identity, so it is the partial of the
group's forgeries)."""
import os
import struct
import subprocess

import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu

SEED = bytes((7 * i + 3) % 256 for i in range(32))


def _entries(gpu, golden, n, rng):
    """n entries over two interleaved Parameters groups with forgeries in both: s + 1, a
    replayed context, a wrong statement, and a nonce-0 proof (identity commitments, valid)."""
    import chaum_pedersen as cp
    cg = golden["custom_generators"]
    params = [cp.Parameters(), cp.Parameters(bytes.fromhex(cg["g"]), bytes.fromhex(cg["h"]))]
    groups = rng.integers(0, 2, n)
    if n >= 2:
        groups[0], groups[1] = 1, 0          # group order != params order: first appearance wins
    ctxs = []
    for i in range(n):
        r = rng.integers(0, 4)
        ctxs.append(None if r == 0 else (b"" if r == 1 else rng.integers(0, 256, 32, dtype=np.uint8).tobytes()))
    x = [int(v) for v in rng.integers(1, 2**62, n)]
    k = [int(v) for v in rng.integers(1, 2**62, n)]
    # forgeries: the first entry of each group plus ~1/12 of the rest; one nonce-0 proof (n >= 10)
    pick = {int(np.nonzero(groups == g)[0][0]) for g in (0, 1) if (groups == g).any()}
    pick |= {int(i) for i in rng.choice(n, size=min(n, n // 12), replace=False)}
    kinds = ["s+1", "ctx", "stmt"]
    forged = {i: kinds[j % 3] for j, i in enumerate(sorted(pick))}
    if n >= 10:
        k0 = next(i for i in range(n) if i not in forged)
        forged[k0] = "k0"
        k[k0] = 0
    rows = {q: np.zeros((n, 32), np.uint8) for q in ("y1", "y2", "r1", "r2", "s")}
    for gsel in (0, 1):
        idx = np.nonzero(groups == gsel)[0]
        if len(idx) == 0:
            continue
        out = gpu.prove([x[i] for i in idx], [k[i] for i in idx], contexts=[ctxs[i] for i in idx],
                        params=params[gsel])
        for q in rows:
            rows[q][idx] = out[q]
    for i, kind in forged.items():
        if kind == "s+1":
            v = (int.from_bytes(rows["s"][i].tobytes(), "little") + 1) % O.L
            rows["s"][i] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
        elif kind == "ctx":
            ctxs[i] = b"replayed-" + (ctxs[i] or b"")
        elif kind == "stmt":  # another entry's statement (n >= 2 here)
            j = (i + 1) % n
            rows["y1"][i], rows["y2"][i] = rows["y1"][j].copy(), rows["y2"][j].copy()
    return params, groups, rows, ctxs, forged


def _run_mirror(tmp_path, params, groups, rows, ctxs, rlc_min):
    import build_native
    exe = build_native.build_dropin_test()
    n = len(groups)
    blob = bytearray(b"CPZD" + struct.pack("<II", n, rlc_min) + SEED)
    for p in params:
        blob += p.g + p.h
    for i in range(n):
        blob += bytes([int(groups[i])])
        for q in ("y1", "y2", "r1", "r2", "s"):
            blob += rows[q][i].tobytes()
        c = ctxs[i]
        blob += bytes([0 if c is None else 1]) + struct.pack("<I", 0 if c is None else len(c)) + (c or b"")
    inp, outp = tmp_path / "in.bin", tmp_path / "out.txt"
    inp.write_bytes(bytes(blob))
    r = subprocess.run([exe, str(inp), str(outp)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    st, disp, draws = {}, [], (None, None)
    for line in outp.read_text().splitlines():
        f = line.split()
        if f[0] == "status":
            st[int(f[1])] = int(f[2])
        elif f[0] == "dispatch":
            disp.append({"rlc": f[1] == "1", "entries": int(f[2]), "first_index": int(f[3]), "batch_ok": f[4] == "1",
                         "seed": bytes.fromhex(f[5]), "partial": bytes.fromhex(f[6])})
        elif f[0] == "rng_draws":
            draws = (int(f[1]), int(f[2]))
    return np.array([st[i] for i in range(n)], np.uint8), disp, draws


def _expected(params, groups, rows, ctxs, forged):
    import coracle
    exp = np.zeros(len(groups), np.uint8)
    for i in range(len(groups)):
        p = params[int(groups[i])]
        args = [rows[q][i].tobytes() for q in ("y1", "y2", "r1", "r2", "s")]
        if forged.get(i) == "k0":
            rec = O.ProofRecord(*args, ctx=ctxs[i])
            exp[i] = O.verify_one(rec, commitment_checks=False, g_bytes=p.g, h_bytes=p.h)
        else:
            exp[i] = coracle.verify_one(p.g, p.h, *args, ctx=ctxs[i])
    return exp


@pytest.mark.parametrize("n", [1, 2, 10, 100, 1000])
@pytest.mark.parametrize("rlc_min", [1, 2, 1 << 30])
def test_dropin_call_sequence_matches_verify_one(gpu, golden, tmp_path, n, rlc_min):
    import coracle
    rng = np.random.default_rng(1000 * n + (rlc_min & 0xff))
    params, groups, rows, ctxs, forged = _entries(gpu, golden, n, rng)
    st, disp, draws = _run_mirror(tmp_path, params, groups, rows, ctxs, rlc_min)
    exp = _expected(params, groups, rows, ctxs, forged)
    assert np.array_equal(st, exp), (np.nonzero(st != exp)[0], st[st != exp], exp[st != exp])
    # the forgeries are rejected in both groups, the nonce-0 proofs accepted
    for i, kind in forged.items():
        assert (st[i] == 0) == (kind == "k0"), (i, kind)
    # the call sequence: groups in order of first appearance, consecutive weight indices
    order = []
    for g in groups:
        if int(g) not in order:
            order.append(int(g))
    assert [d["entries"] for d in disp] == [int((groups == g).sum()) for g in order]
    fi = 0
    for g, d in zip(order, disp):
        assert d["first_index"] == fi
        idx = np.nonzero(groups == g)[0]
        want_rlc = len(idx) >= rlc_min
        assert d["rlc"] == want_rlc
        if want_rlc:
            if n > 1:
                assert d["seed"] == SEED
            else:   # the OS's seed, not the caller's rng
                assert d["seed"] != SEED
            p = params[g]
            sub = {q: rows[q][idx] for q in rows}
            part, _ = coracle.rlc_partial(sub, np.arange(fi, fi + len(idx)), d["seed"],
                                          contexts=[ctxs[i] for i in idx], g=p.g, h=p.h)
            assert d["partial"] == part, (g, len(idx))
            assert d["batch_ok"] == all(exp[i] == 0 for i in idx)
        fi += len(idx)
    # the reference's consumption of rng: n calls of 64 bytes for n >= 2, nothing for n == 1
    assert draws == ((n, 64 * n) if n > 1 else (0, 0))
