"""The C oracle (oracle/cpz_oracle.c: CPU baseline + at-scale checker) against the golden
fixtures and the reference's BatchVerifier semantics."""
import numpy as np

import coracle as C


def _f(p):
    return {k: bytes.fromhex(p[k]) for k in ("y1", "y2", "r1", "r2", "s")}


def test_golden_statuses_and_challenges(golden):
    g, h = bytes.fromhex(golden["g"]), bytes.fromhex(golden["h"])
    for p in golden["proofs"]:
        f = _f(p)
        ctx = None if p["ctx"] is None else bytes.fromhex(p["ctx"])
        assert C.verify_one(g, h, f["y1"], f["y2"], f["r1"], f["r2"], f["s"], ctx) == p["status"], p["kind"]
        if "c" in p:
            assert C.challenge(g, h, f["y1"], f["y2"], f["r1"], f["r2"], ctx).hex() == p["c"]
    cg = golden["custom_generators"]
    g2, h2 = bytes.fromhex(cg["g"]), bytes.fromhex(cg["h"])
    for p in cg["proofs"]:
        f = _f(p)
        ctx = bytes.fromhex(p["ctx"])
        assert C.verify_one(g2, h2, f["y1"], f["y2"], f["r1"], f["r2"], f["s"], ctx) == 0


def test_decode_encode_and_scalar_mul(golden):
    import ctypes
    lib = C.load()
    out = ctypes.create_string_buffer(32)
    for enc in golden["rfc9496_multiples"]:
        assert lib.cpzo_decode_encode(out, bytes.fromhex(enc)) == 1 and out.raw.hex() == enc
    for enc in golden["rfc9496_bad"]:
        assert lib.cpzo_decode_encode(out, bytes.fromhex(enc)) == 0
    B = bytes.fromhex(golden["rfc9496_multiples"][1])
    for k in range(16):
        assert lib.cpzo_scalar_mul(out, B, k.to_bytes(32, "little")) == 1
        assert out.raw.hex() == golden["rfc9496_multiples"][k]


def test_reference_batch_semantics(golden):
    valid = [p for p in golden["proofs"] if p["ctx"] is None and p["kind"] == "valid"][:6]
    rows = {k: np.frombuffer(b"".join(bytes.fromhex(p[k]) for p in valid), np.uint8).reshape(-1, 32)
            for k in ("y1", "y2", "r1", "r2", "s")}
    held, st = C.reference_batch_verify(rows, 0, 6)
    assert held == 0 and not st.any()          # defective equation fails, fallback accepts all
    held, st = C.reference_batch_verify(rows, 0, 1)
    assert held == 0 and not st.any()          # n == 1 -> verify_one
    bad = {k: v.copy() for k, v in rows.items()}
    bad["y1"][3] = rows["y1"][4]
    held, st = C.reference_batch_verify(bad, 0, 6)
    assert list(st) == [0, 0, 0, 1, 0, 0]
    assert list(C.verify_many(bad, threads=2)) == [0, 0, 0, 1, 0, 0]


def _rows(ps):
    return {k: np.frombuffer(b"".join(bytes.fromhex(p[k]) for p in ps), np.uint8).reshape(-1, 32)
            for k in ("y1", "y2", "r1", "r2", "s")}


def _ctxs(ps):
    return [None if p["ctx"] is None else bytes.fromhex(p["ctx"]) for p in ps]


def test_bulk_checkers_against_golden(golden):
    """The at-scale checkers (statuses and challenges with contexts, multithreaded) agree
    with every golden proof."""
    ps = golden["proofs"]
    st = C.verify_many_ctx(_rows(ps), _ctxs(ps), threads=3)
    assert [int(v) for v in st] == [p["status"] for p in ps]
    with_c = [p for p in ps if "c" in p]
    c = C.challenge_many(_rows(with_c), _ctxs(with_c), threads=2)
    assert [bytes(r).hex() for r in c] == [p["c"] for p in with_c]


def test_rlc_partial_against_golden(golden):
    """cpzo_rlc_partial (an independent C restatement: weights reduced word by word, the
    constant-time ladder) reproduces the golden RLC partials, whole batches and shards,
    and the partial of a forged batch equals the partial of its forged entries alone."""
    for case in golden["rlc"]:
        ps = case["proofs"]
        seed = bytes.fromhex(case["seed"])
        n = len(ps)
        gidx = np.arange(case["first_index"], case["first_index"] + n, dtype=np.uint64)
        enc, live = C.rlc_partial(_rows(ps), gidx, seed, threads=2)
        assert enc.hex() == case["partial"], case["name"]
        for sh in case.get("shards", []):
            sub = ps[sh["lo"]:sh["hi"]]
            enc, _ = C.rlc_partial(_rows(sub), np.arange(sh["first_index"], sh["first_index"] + len(sub)), seed)
            assert enc.hex() == sh["partial"]
        if "statuses" in case:
            bad = [i for i, s in enumerate(case["statuses"]) if s == 1]
            enc, _ = C.rlc_partial(_rows([ps[i] for i in bad]), gidx[bad], seed)
            assert enc.hex() == case["partial"]
