"""Generate tests/golden/golden.json from the CPU oracle (oracle/pyoracle.py).

Run in the build container:  python tests/golden/make_golden.py
The fixtures are data only (inputs + expected outputs); the GPU tests and the C-oracle
tests compare against them.  Independent pins checked while generating (and again by
tests/test_oracle_pins.py when libsodium is importable): libsodium's ristretto255 for
every encoding, the merlin KAT, RFC 9496 vectors.

Reference semantics being pinned (no fixed vectors exist in the reference's own tests,
which all draw from OsRng -- SURVEY 4, 8c):
  challenge:        src/primitives/transcript.rs:29-71, batch.rs:188-206
  per-proof status: batch.rs:185-231, gadgets.rs:364-489, verifier/mod.rs:144-171
"""
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as O  # noqa: E402

# RFC 9496 Appendix A.1: encodings of k * B, k = 0..15.
RFC_MULTIPLES = """0000000000000000000000000000000000000000000000000000000000000000
e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76
6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919
94741f5d5d52755ece4f23f044ee27d5d1ea1e2bd196b462166b16152a9d0259
da80862773358b466ffadfe0b3293ab3d9fd53c5ea6c955358f568322daf6a57
e882b131016b52c1d3337080187cf768423efccbb517bb495ab812c4160ff44e
f64746d3c92b13050ed8d80236a7f0007c3b3f962f5ba793d19a601ebb1df403
44f53520926ec81fbd5a387845beb7df85a96a24ece18738bdcfa6a7822a176d
903293d8f2287ebe10e2374dc1a53e0bc887e592699f02d077d5263cdd55601c
02622ace8f7303a31cafc63f8fc48fdc16e1c8c8d234b2f0d6685282a9076031
20706fd788b2720a1ed2a5dad4952b01f413bcf0e7564de8cdc816689e2db95f
bce83f8ba5dd2fa572864c24ba1810f9522bc6004afe95877ac73241cafdab42
e4549ee16b9aa03099ca208c67adafcafa4c3f3e4e5303de6026e3ca8ff84460
aa52e000df2e16f55fb1032fc33bc42742dad6bd5a8fc0be0167436c5948501f
46376b80f409b29dc2b5f6f0c52591990896e5716f41477cd30085ab7f10301e
e0c418f7c8d9c4cdd7395b93ea124f3ad99021bb681dfc3302a9d99a2e53e64e""".split()

# RFC 9496 Appendix A.2: encodings that must fail to decode (non-canonical, negative,
# non-square x^2, negative xy, s = -1).
RFC_BAD = """00ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff
ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f
f3ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f
edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f
0100000000000000000000000000000000000000000000000000000000000000
01ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f
ed57ffd8c914fb201471d1c3d245ce3c746fcbe63a3679d51b6a516ebebe0e20
c34c4e1826e5d403b78e246e88aa051c36ccf0aafebffe137d148a2bf9104562
c940e5a4404157cfb1628b108db051a8d439e1a421394ec4ebccb9ec92a8ac78
47cfc5497c53dc8e61c91d17fd626ffb1c49e2bca94eed052281b510b1117a24
f1c6165d33367351b0da8f6e4511010c68174a03b6581212c71c0e1d026c3c72
87260f7a2f12495118360f02c26a470f450dadf34a413d21042b43b9d93e1309
26948d35ca62e643e26a83177332e6b6afeb9d08e4268b650f1f5bbd8d81d371
4eac077a713c57b4f4397629a4145982c661f48044dd3f96427d40b147d9742f
de6a7b00deadc788eb6b6c8d20c0ae96c2f2019078fa604fee5b87d6e989ad7b
bcab477be20861e01e4a0e295284146a510150d9817763caf1a6f4b422d67042
2a292df7e32cababbd9de088d1d1abec9fc0440f637ed2fba145094dc14bea08
f4a9e534fc0d216c44b218fa0c42d99635a0127ee2e53c712f70609649fdff22
8268436f8c4126196cf64b3c7ddbda90746a378625f9813dd9b8457077256731
2810e5cbc2cc4d4eece54f61c6f69758e289aa7ab440b3cbeaa21995c2f4232b
3eb858e78f5a7254d8c9731174a94f76755fd3941c0ac93735c07ba14579630e
a45fdc55c76448c049a1ab33f17023edfb2be3581e9c7aade8a6125215e04220
d483fe813c6ba647ebbfd3ec41adca1c6130c2beeee9d9bf065c8d151c5f396e
8a2e1d30050198c65a54483123960ccc38aef6848e1ec8f5f780e8523769ba32
32888462f8b486c68ad7dd9610be5192bbeaf3b443951ac1a8118419d9fa097b
227142501b9d4355ccba290404bde41575b037693cef1f438c47f8fbf35d1165
5c37cc491da847cfeb9281d407efc41e15144c876e0170b499a96a22ed31e01e
445425117cb8c90edcbc7c1cc0e74f747f2c1efa5630a967c64f287792a48a4b
ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f""".split()

SEED_X = hashlib.sha256(b"cpz-bench-x").digest()
SEED_K = hashlib.sha256(b"cpz-bench-k").digest()


def chacha_scalar(seed: bytes, i: int) -> int:
    return O.scalar_wide(O.chacha20_block(seed, i))


def rec_json(rec, status, c=None, kind="valid"):
    d = {"y1": rec.y1.hex(), "y2": rec.y2.hex(), "r1": rec.r1.hex(), "r2": rec.r2.hex(), "s": rec.s.hex(),
         "ctx": None if rec.ctx is None else rec.ctx.hex(), "status": status, "kind": kind}
    if c is not None:
        d["c"] = O.scalar_bytes(c).hex()
    return d


def main():
    out = {
        "generator": "tests/golden/make_golden.py (oracle/pyoracle.py)",
        "g": O.G_BYTES.hex(),
        "h": O.H_BYTES.hex(),
        "merlin_kat": {"protocol": "test protocol", "label": "some label", "message": "some data",
                       "challenge_label": "challenge", "n": 32,
                       "out": "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"},
        "rfc9496_multiples": RFC_MULTIPLES,
        "rfc9496_bad": RFC_BAD,
        "seed_x": SEED_X.hex(),
        "seed_k": SEED_K.hex(),
    }
    for k, enc in enumerate(RFC_MULTIPLES):
        assert O.ristretto_encode(O.pt_mul(O.BASEPOINT, k)).hex() == enc
    for enc in RFC_BAD:
        assert O.ristretto_decode(bytes.fromhex(enc)) is None

    # 1. Valid proofs, deterministic witnesses (SHA-512 derivation), three context modes.
    proofs = []
    recs = []
    for i in range(48):
        mode = i % 3
        ctx = None if mode == 0 else (b"user-%d-session" % i if mode == 1 else b"")
        x, k = O.bench_scalar(b"x", i), O.bench_scalar(b"k", i)
        rec = O.prove(x, k, ctx)
        c = O.challenge(O.G_BYTES, O.H_BYTES, rec.y1, rec.y2, rec.r1, rec.r2, ctx)
        assert O.verify_one(rec) == O.ST_OK
        recs.append(rec)
        proofs.append(rec_json(rec, O.ST_OK, c))

    # 2. Forgeries (status 1): s + 1, wrong statement, wrong / missing / extra context,
    #    swapped commitments.
    L = O.L
    def forged(rec, kind, **kw):
        d = dict(y1=rec.y1, y2=rec.y2, r1=rec.r1, r2=rec.r2, s=rec.s, ctx=rec.ctx)
        d.update(kw)
        r = O.ProofRecord(**d)
        st = O.verify_one(r)
        c = O.challenge(O.G_BYTES, O.H_BYTES, r.y1, r.y2, r.r1, r.r2, r.ctx)
        proofs.append(rec_json(r, st, c, kind))
        return st

    for i in range(8):
        rec = recs[i]
        s1 = O.scalar_bytes(int.from_bytes(rec.s, "little") + 1)
        assert forged(rec, "s_plus_1", s=s1) == O.ST_EQ_FAIL
        assert forged(rec, "wrong_statement", y1=recs[i + 8].y1, y2=recs[i + 8].y2) == O.ST_EQ_FAIL
        assert forged(rec, "wrong_y2_only", y2=recs[i + 9].y2) == O.ST_EQ_FAIL
        assert forged(rec, "wrong_context", ctx=b"session-2" if rec.ctx != b"session-2" else b"x") == O.ST_EQ_FAIL
        assert forged(rec, "swapped_commitment", r1=rec.r2, r2=rec.r1) == O.ST_EQ_FAIL
    # context None vs Some(b"") are different transcripts
    rec = recs[0]  # mode 0: ctx None
    assert forged(rec, "none_vs_empty_context", ctx=b"") == O.ST_EQ_FAIL
    rec = recs[2]  # mode 2: ctx b""
    assert forged(rec, "empty_vs_none_context", ctx=None) == O.ST_EQ_FAIL

    # 3. Malformed encodings (status 2/3/4), in the reference's rejection order.
    base = recs[3]
    ident = bytes(32)
    s_int = int.from_bytes(base.s, "little")
    cases = [
        ("s_plus_l", dict(s=(s_int + L).to_bytes(32, "little")), O.ST_BAD_SCALAR),
        ("s_high_bit", dict(s=(s_int | (1 << 255)).to_bytes(32, "little")), O.ST_BAD_SCALAR),
        ("s_eq_l", dict(s=L.to_bytes(32, "little")), O.ST_BAD_SCALAR),
        ("s_all_ff", dict(s=b"\xff" * 32), O.ST_BAD_SCALAR),
        ("s_zero", dict(s=ident), O.ST_ZERO_S),
        ("r1_identity", dict(r1=ident), O.ST_IDENTITY),
        ("r2_identity", dict(r2=ident), O.ST_IDENTITY),
        ("identity_statement", dict(y1=ident, y2=ident), O.ST_EQ_FAIL),
        ("bad_point_and_bad_scalar", dict(r1=bytes.fromhex(RFC_BAD[5]), s=b"\xff" * 32), O.ST_BAD_POINT),
        ("bad_scalar_and_identity", dict(r1=ident, s=b"\xff" * 32), O.ST_BAD_SCALAR),
        ("zero_s_and_identity", dict(r1=ident, s=ident), O.ST_IDENTITY),
    ]
    for j, enc in enumerate(RFC_BAD):
        field = ("y1", "y2", "r1", "r2")[j % 4]
        cases.append(("bad_%s_rfc%d" % (field, j), {field: bytes.fromhex(enc)}, O.ST_BAD_POINT))
    for kind, kw, expect in cases:
        d = dict(y1=base.y1, y2=base.y2, r1=base.r1, r2=base.r2, s=base.s, ctx=base.ctx)
        d.update(kw)
        r = O.ProofRecord(**d)
        st = O.verify_one(r)
        assert st == expect, (kind, st, expect)
        proofs.append(rec_json(r, st, None, kind))

    # A proof that verifies with identity statement y1 = y2 = O, x = 0 (reference allows
    # identity statements, security_tests.rs:136-149): s = k, r = k g.
    x0 = 0
    rec0 = O.prove(x0, O.bench_scalar(b"k", 99), None)
    assert rec0.y1 == ident and O.verify_one(rec0) == O.ST_OK
    proofs.append(rec_json(rec0, O.ST_OK, O.challenge(O.G_BYTES, O.H_BYTES, rec0.y1, rec0.y2, rec0.r1, rec0.r2),
                           "identity_statement_valid"))
    out["proofs"] = proofs

    # 4. Custom generators (Parameters::with_generators): g' = 5B, h' = 7 H.
    g2 = O.pt_mul(O.BASEPOINT, 5)
    h2 = O.pt_mul(O.generator_h(), 7)
    g2b, h2b = O.ristretto_encode(g2), O.ristretto_encode(h2)
    cust = []
    for i in range(4):
        rec = O.prove(O.bench_scalar(b"x", 200 + i), O.bench_scalar(b"k", 200 + i), b"ctx-%d" % i, g2, h2)
        assert O.verify_one(rec, g2b, h2b) == O.ST_OK
        assert O.verify_one(rec) == O.ST_EQ_FAIL  # under the default generators
        cust.append(rec_json(rec, O.ST_OK, O.challenge(g2b, h2b, rec.y1, rec.y2, rec.r1, rec.r2, rec.ctx)))
    out["custom_generators"] = {"g": g2b.hex(), "h": h2b.hex(), "proofs": cust}

    # 5. The synthetic generator's proofs (GPU prover, cpz_prove_synthetic): x_i, k_i =
    #    wide(ChaCha20(SEED_X / SEED_K, block i)), no context.
    synth = []
    for i in list(range(8)) + [1000, 2**20 - 1]:
        rec = O.prove(chacha_scalar(SEED_X, i), chacha_scalar(SEED_K, i), None)
        d = rec_json(rec, O.ST_OK)
        d["index"] = i
        synth.append(d)
    out["synthetic"] = synth

    # 6. ChaCha20 keystream blocks for the weight seed (batch weights alpha_i, gamma_i).
    wseed = hashlib.sha256(b"cpz-weights-v1").digest()
    out["weight_seed"] = wseed.hex()
    out["weights"] = [{"index": i, "alpha": O.scalar_bytes(O.batch_weight(wseed, i)).hex(),
                       "gamma": O.scalar_bytes(O.batch_weight2(wseed, i)).hex()} for i in (0, 1, 2, 63, 1 << 20)]
    # RLC weights (a_i, b_i) of the corrected batch check (pyoracle.rlc_weights).
    out["rlc_weights"] = [{"index": i, "a": O.scalar_bytes(O.rlc_weights(wseed, i)[0]).hex(),
                           "b": O.scalar_bytes(O.rlc_weights(wseed, i)[1]).hex()} for i in (0, 1, 2, 63, 1 << 20)]

    # 7. RLC partials (corrected batch equation, the MSM the GPU runs) for fixed seeds:
    #    all-valid batches are the identity; forged / malformed entries make a specific point;
    #    shards keyed by global index sum to the whole.
    rseed = hashlib.sha256(b"cpz-rlc-golden").digest()
    valid = [r for r, p in zip(recs, proofs[:48]) if r.ctx is None][:12]
    def prs(rs):
        return [rec_json(r, 0) for r in rs]
    rlc = []
    P = O.rlc_partial(valid, rseed)
    assert O.pt_is_identity(P)
    rlc.append({"name": "valid12", "seed": rseed.hex(), "first_index": 0, "proofs": prs(valid),
                "partial": O.ristretto_encode(P).hex(), "identity": True})
    forged_set = list(valid)
    forged_set[3] = O.ProofRecord(valid[3].y1, valid[3].y2, valid[3].r1, valid[3].r2,
                                  O.scalar_bytes(int.from_bytes(valid[3].s, "little") + 1))
    forged_set[7] = O.ProofRecord(valid[8].y1, valid[8].y2, valid[7].r1, valid[7].r2, valid[7].s)
    forged_set[9] = O.ProofRecord(valid[9].y1, valid[9].y2, bytes.fromhex(RFC_BAD[5]), valid[9].r2, valid[9].s)
    P = O.rlc_partial(forged_set, rseed, 5)
    P0 = O.rlc_partial(forged_set[:6], rseed, 5)
    P1 = O.rlc_partial(forged_set[6:], rseed, 11)
    assert O.pt_eq(O.pt_add(P0, P1), P) and not O.pt_is_identity(P)
    rlc.append({"name": "forged12", "seed": rseed.hex(), "first_index": 5, "proofs": prs(forged_set),
                "partial": O.ristretto_encode(P).hex(), "identity": False,
                "shards": [{"lo": 0, "hi": 6, "first_index": 5, "partial": O.ristretto_encode(P0).hex()},
                           {"lo": 6, "hi": 12, "first_index": 11, "partial": O.ristretto_encode(P1).hex()}],
                "statuses": [O.verify_one(r) for r in forged_set]})
    out["rlc"] = rlc

    # 7. Wire format (Proof::from_bytes, gadgets.rs:364-489): valid blobs, every truncation,
    #    bad versions / lengths / points / scalars, trailing bytes, identity / zero, and
    #    doubly-malformed blobs where the reference's order of checks decides the error.
    import struct
    def blob(r1, r2, s, ver=1, l1=None, l2=None, l3=None, tail=b""):
        return (bytes([ver]) + struct.pack(">I", len(r1) if l1 is None else l1) + r1 +
                struct.pack(">I", len(r2) if l2 is None else l2) + r2 +
                struct.pack(">I", len(s) if l3 is None else l3) + s + tail)
    good = recs[0]
    gb = blob(good.r1, good.r2, good.s)
    assert len(gb) == 109 and gb == O.proof_to_bytes(good.r1, good.r2, good.s)
    bad_pt = bytes.fromhex(RFC_BAD[3])
    big_s = L.to_bytes(32, "little")
    wire = [gb, blob(recs[1].r1, recs[1].r2, recs[1].s)]
    wire += [gb[:k] for k in range(0, 109)]                      # every truncation
    wire += [bytes([v]) + gb[1:] for v in (0, 2, 255)]           # versions
    wire += [gb + b"\x00", gb + b"\x01\x02\x03\x04\x05"]       # trailing
    wire += [blob(good.r1, good.r2, good.s, l1=0), blob(good.r1, good.r2, good.s, l1=4097),
             blob(good.r1, good.r2, good.s, l2=0), blob(good.r1, good.r2, good.s, l2=5000),
             blob(good.r1, good.r2, good.s, l3=0), blob(good.r1, good.r2, good.s, l3=513),
             blob(good.r1 + b"\x00", good.r2, good.s), blob(good.r1[:31], good.r2, good.s),
             blob(good.r1, good.r2 + b"\x07", good.s), blob(good.r1, good.r2[:30], good.s),
             blob(good.r1, good.r2, good.s + b"\x00"), blob(good.r1, good.r2, good.s[:31]),
             blob(good.r1, good.r2, good.s, l1=4096)]
    wire += [blob(bad_pt, good.r2, good.s), blob(good.r1, bad_pt, good.s), blob(good.r1, good.r2, big_s),
             blob(bytes(32), good.r2, good.s), blob(good.r1, bytes(32), good.s), blob(good.r1, good.r2, bytes(32))]
    # precedence: r1 decode before r2 structure; r2 decode before s; s before trailing;
    # trailing before identity; identity before zero s
    wire += [blob(bad_pt, good.r2, good.s)[:50], blob(bad_pt, good.r2, good.s, l2=0),
             blob(good.r1, bad_pt, good.s)[:90], blob(good.r1, bad_pt, good.s, l3=600),
             blob(good.r1, good.r2, big_s, tail=b"\x00"), blob(bytes(32), good.r2, good.s, tail=b"\x00"),
             blob(bytes(32), good.r2, bytes(32)), blob(bad_pt, bad_pt, big_s, tail=b"zz")]
    for rb in RFC_BAD[:12]:
        wire.append(blob(good.r1, bytes.fromhex(rb), good.s))
    out["wire"] = [{"blob": w.hex(), "code": O.proof_from_bytes_code(w)[0], "aux": O.proof_from_bytes_code(w)[1]}
                   for w in wire]
    for w, e in zip(wire, out["wire"]):  # the coarse oracle (error kind) agrees
        kind = O.proof_from_bytes(w)
        assert (kind[0] == "ok") == (e["code"] == 0)

    # 8. verify_response (verifier/mod.rs:144-171) with caller-supplied challenges: the
    #    transcript's challenge (with or without a context: the caller's c replaces the
    #    transcript), c + 1, c + l (non-canonical), and decode-level failures first.
    resp = []
    for i in range(6):
        rec = recs[i]
        c = O.challenge(O.G_BYTES, O.H_BYTES, rec.y1, rec.y2, rec.r1, rec.r2, rec.ctx)
        cases = [("transcript_c", O.scalar_bytes(c)), ("c_plus_1", O.scalar_bytes((c + 1) % L)),
                 ("c_plus_l", (c + L).to_bytes(32, "little")), ("c_zero", bytes(32))]
        for kind, cb in cases:
            st = O.verify_response(rec, cb)
            d = rec_json(rec, st, None, kind)
            d["c"] = cb.hex()
            resp.append(d)
    # c = 0 verifies exactly when s is the nonce: g^k == r1 (a proof made with x = 0 or c = 0)
    rec0c = O.prove(O.bench_scalar(b"x", 77), O.bench_scalar(b"k", 77), None)
    k77 = O.bench_scalar(b"k", 77)
    zero_c = O.ProofRecord(rec0c.y1, rec0c.y2, rec0c.r1, rec0c.r2, O.scalar_bytes(k77))
    d = rec_json(zero_c, O.verify_response(zero_c, bytes(32)), None, "s_eq_k_with_c_zero")
    d["c"] = bytes(32).hex()
    assert d["status"] == O.ST_OK
    resp.append(d)
    for p in proofs[48:]:
        if p["kind"] in ("s_zero", "r1_identity", "s_plus_l", "bad_r1_rfc2", "identity_statement"):
            r = O.ProofRecord(*(bytes.fromhex(p[k]) for k in ("y1", "y2", "r1", "r2", "s")))
            cb = (L + 5).to_bytes(32, "little")  # non-canonical c: decode-level statuses come first
            d = rec_json(r, O.verify_response(r, cb), None, "resp_" + p["kind"])
            d["c"] = cb.hex()
            resp.append(d)
    out["response"] = resp

    # 9. Prover (Prover::prove_with_transcript / commit / respond, prover/mod.rs:86-131, and
    #    the statement y = x g, x h, gadgets.rs:217-221) from caller witnesses and nonces.
    prv = []
    for i in range(10):
        x = O.bench_scalar(b"px", i) if i != 3 else 0
        k = O.bench_scalar(b"pk", i)
        ctx = [None, b"", b"user-%d-session" % i, bytes(range(32))][i % 4]
        rec = O.prove(x, k, ctx)
        assert O.verify_one(rec) == (O.ST_OK if True else None) or x == 0
        d = rec_json(rec, O.verify_one(rec))
        d["x"] = O.scalar_bytes(x).hex()
        d["k"] = O.scalar_bytes(k).hex()
        prv.append(d)
    out["prove"] = prv

    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, "proofs:", len(proofs))


if __name__ == "__main__":
    main()
