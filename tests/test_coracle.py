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
