"""GPU tests of the reference interface beyond BatchVerifier: Proof::from_bytes through the
device parser (gadgets.rs:364-489), Verifier::verify_response with caller challenges
(verifier/mod.rs:144-171), the prover from caller witnesses (prover/mod.rs:86-131,
gadgets.rs:217-221), bulk element_from_bytes / element_to_bytes (ristretto.rs:120-143), the
service's registration checks (service.rs:61-97), and call ordering across streams."""
import hashlib

import numpy as np
import pytest

import chaum_pedersen as cp
import pyoracle as O

pytestmark = pytest.mark.gpu


def _rows(ps, k):
    return np.frombuffer(b"".join(bytes.fromhex(p[k]) for p in ps), np.uint8).reshape(-1, 32)


def test_from_bytes_golden_wire(gpu, golden):
    """Every golden blob: Proof.from_bytes returns the proof or raises the reference's error
    type with its exact message (the oracle's code / value for that blob)."""
    for w in golden["wire"]:
        b = bytes.fromhex(w["blob"])
        want = cp.parse_error(w["code"], w["aux"])
        if want is None:
            p = cp.Proof.from_bytes(b, gpu)
            assert (p.r1, p.r2, p.s) == (b[5:37], b[41:73], b[77:109])
            assert p.to_bytes() == b
        else:
            with pytest.raises(cp.Error) as exc:
                cp.Proof.from_bytes(b, gpu)
            assert type(exc.value) is type(want) and str(exc.value) == str(want), w
    many = cp.Proof.from_bytes_many([bytes.fromhex(w["blob"]) for w in golden["wire"]], gpu)
    assert [isinstance(m, cp.Proof) for m in many] == [w["code"] == 0 for w in golden["wire"]]


def test_verify_response_golden(gpu, golden):
    rs = golden["response"]
    st = gpu.verify_response(*(_rows(rs, k) for k in ("y1", "y2", "r1", "r2", "s", "c")))
    assert [int(v) for v in st] == [r["status"] for r in rs], [(r["kind"], int(v)) for r, v in zip(rs, st)]
    # the transcript's challenge as the caller's c gives verify_one's answer on the golden proofs
    ps = [p for p in golden["proofs"] if "c" in p]
    st = gpu.verify_response(*(_rows(ps, k) for k in ("y1", "y2", "r1", "r2", "s", "c")))
    assert [int(v) for v in st] == [p["status"] for p in ps]


def test_prove_golden_and_roundtrip(gpu, golden):
    pv = golden["prove"]
    ctxs = [None if p["ctx"] is None else bytes.fromhex(p["ctx"]) for p in pv]
    out = gpu.prove(_rows(pv, "x"), _rows(pv, "k"), contexts=ctxs)
    for i, p in enumerate(pv):
        for k in ("y1", "y2", "r1", "r2", "s"):
            assert out[k][i].tobytes().hex() == p[k], (i, k)
    st = gpu.verify_each(out["y1"], out["y2"], out["r1"], out["r2"], out["s"], contexts=ctxs)
    assert [int(v) for v in st] == [p["status"] for p in pv]


def test_prove_device_matches_host_and_verifies(gpu):
    """2^16 random witnesses / nonces (>= l included, taken mod l): the device-buffer prover
    equals the host-buffer one byte for byte, every proof verifies, a sample equals the oracle."""
    torch = pytest.importorskip("torch")
    n = 1 << 16
    rng = np.random.default_rng(3)
    x = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    k = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    x[5] = 0xFF                      # >= l: taken mod l
    host = gpu.prove(x, k)
    dev = torch.device("cuda:0")
    t = {q: torch.empty((n, 32), dtype=torch.uint8, device=dev) for q in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_device(torch.from_numpy(x).to(dev), torch.from_numpy(k).to(dev), t["y1"], t["y2"], t["r1"], t["r2"],
                     t["s"])
    torch.cuda.synchronize()
    for q in t:
        assert np.array_equal(t[q].cpu().numpy(), host[q]), q
    st = gpu.verify_each(host["y1"], host["y2"], host["r1"], host["r2"], host["s"])
    assert not st.any()
    for i in (0, 5, 1234, n - 1):
        rec = O.prove(int.from_bytes(x[i].tobytes(), "little") % O.L, int.from_bytes(k[i].tobytes(), "little") % O.L)
        assert (host["y1"][i].tobytes(), host["r2"][i].tobytes(), host["s"][i].tobytes()) == (rec.y1, rec.r2, rec.s)


def test_verifier_and_prover_mirrors(gpu):
    """verifier/mod.rs:174-229 and prover/mod.rs:154-197 through the Python mirrors."""
    params = cp.Parameters()
    pv = cp.Prover(params, O.bench_scalar(b"x", 5), gpu)
    st = pv.statement()
    rec = O.prove(O.bench_scalar(b"x", 5), 9)
    assert (st.y1, st.y2) == (rec.y1, rec.y2)
    v = cp.Verifier(params, st, gpu)
    proof = pv.prove_with_transcript(None, cp.Transcript.new(), nonce=9)
    assert (proof.r1, proof.r2, proof.s) == (rec.r1, rec.r2, rec.s)
    v.verify(proof)
    # proofs are randomised (security_tests.rs:166-209): two calls, two different proofs, both valid
    p1, p2 = pv.prove(), pv.prove()
    assert p1.s != p2.s and p1.r1 != p2.r1
    v.verify(p1)
    v.verify(p2)
    # wrong statement (verifier/mod.rs tests): InvalidParams("Proof verification failed")
    other = cp.Prover(params, 12345, gpu).statement()
    with pytest.raises(cp.InvalidParams) as e:
        cp.Verifier(params, other, gpu).verify(proof)
    assert str(e.value) == "Proof verification failed"
    # transcript context binds the proof (security_tests.rs:6-39)
    t = cp.Transcript.new()
    t.append_context(b"challenge-12345")
    bound = pv.prove_with_transcript(None, t)
    v.verify_with_transcript(bound, t)
    with pytest.raises(cp.InvalidParams):
        v.verify(bound)
    # interactive: commit, caller challenge, respond, verify_response
    (r1, r2), k = pv.commit()
    c = 0xC0FFEE
    s = pv.respond(k, c)
    v.verify_response(c, cp.Proof(r1, r2, s))
    with pytest.raises(cp.InvalidParams):
        v.verify_response(c + 1, cp.Proof(r1, r2, s))
    with pytest.raises(cp.InvalidScalar):
        v.verify_response((O.L + 1).to_bytes(32, "little"), cp.Proof(r1, r2, s))


def test_decode_points_rfc9496(gpu, golden):
    """element_from_bytes / element_to_bytes: RFC 9496 A.1 multiples decode and re-encode to
    themselves; every A.2 invalid encoding is rejected."""
    good = [bytes.fromhex(e) for e in golden["rfc9496_multiples"]]
    bad = [bytes.fromhex(e) for e in golden["rfc9496_bad"]]
    ok, enc = gpu.decode_points(good + bad)
    assert list(ok) == [1] * len(good) + [0] * len(bad)
    assert [enc[i].tobytes() for i in range(len(good))] == good
    assert not enc[len(good):].any()
    # statements and commitments of the golden proofs: decode <=> the oracle decodes
    pts = [bytes.fromhex(p[k]) for p in golden["proofs"] for k in ("y1", "r1")]
    ok, enc = gpu.decode_points(pts)
    for i, p in enumerate(pts):
        dec = O.ristretto_decode(p)
        assert bool(ok[i]) == (dec is not None)
        if dec is not None:
            assert enc[i].tobytes() == O.ristretto_encode(dec)


def test_register_handler_checks(gpu):
    """service.rs:61-97: sizes, element_from_bytes of y1 / y2, identity statements refused."""
    from chaum_pedersen.service import AlreadyExists, InvalidArgument, MemoryState, register
    st = MemoryState()
    rec = O.prove(O.bench_scalar(b"x", 1), 3)
    register(st, "alice", rec.y1, rec.y2, gpu)
    assert st.get_user("alice") == (rec.y1, rec.y2)
    cases = [("bob", b"", rec.y2, "Empty y1 or y2 values"),
             ("bob", rec.y1, b"\x01" * 4097, "y1 or y2 values too large"),
             ("bob", rec.y1[:31], rec.y2, "Invalid y1: Invalid group element: Expected 32 bytes, got 31"),
             ("bob", rec.y1, bytes.fromhex("01" + "00" * 31),
              "Invalid y2: Invalid group element: Bytes do not represent a valid Ristretto point"),
             ("bob", bytes(32), rec.y2, "Statement contains identity elements"),
             ("bad id!", rec.y1, rec.y2, "User ID contains invalid characters")]
    for uid, y1, y2, msg in cases:
        with pytest.raises(InvalidArgument) as e:
            register(st, uid, y1, y2, gpu)
        assert str(e.value) == msg
    assert st.get_user("bob") is None
    # a taken id is Status::already_exists, not invalid_argument (service.rs:108-112)
    with pytest.raises(AlreadyExists) as e:
        register(st, "alice", rec.y1, rec.y2, gpu)
    assert str(e.value) == "Registration failed: Invalid group parameters: User 'alice' already registered"
    assert e.value.code == "ALREADY_EXISTS"


def test_calls_ordered_across_streams(gpu, golden):
    """A device-path verify enqueued on a side stream, then -- without any synchronisation --
    a host-path call and a call with other generators (which rebuilds the context's tables):
    every call still sees its own inputs (each call is ordered after the previous one)."""
    torch = pytest.importorskip("torch")
    n = 1 << 18
    dev = torch.device("cuda:0")
    sx, sk = hashlib.sha256(b"cpz-bench-x").digest(), hashlib.sha256(b"cpz-bench-k").digest()
    t = {q: torch.empty((n, 32), dtype=torch.uint8, device=dev) for q in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_synthetic_device(n, sx, sk, t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    torch.cuda.synchronize()
    status = torch.full((n,), 0xFF, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status)
    # host path on the context's own stream, other data (golden proofs, some invalid)
    ps = golden["proofs"]
    st = gpu.verify_each(*(_rows(ps, k) for k in ("y1", "y2", "r1", "r2", "s")),
                         contexts=[None if p["ctx"] is None else bytes.fromhex(p["ctx"]) for p in ps])
    assert [int(v) for v in st] == [p["status"] for p in ps]
    # other generators: the comb / prefix tables are rebuilt
    cg = golden["custom_generators"]
    params = cp.Parameters.with_generators(bytes.fromhex(cg["g"]), bytes.fromhex(cg["h"]))
    cps = cg["proofs"]
    st = gpu.verify_each(*(_rows(cps, k) for k in ("y1", "y2", "r1", "r2", "s")),
                         contexts=[bytes.fromhex(p["ctx"]) for p in cps], params=params)
    assert not st.any()
    side.synchronize()
    assert int((status != 0).sum().item()) == 0


def test_security_tests_mirror(gpu):
    """tests/security_tests.rs:136-163, 212-237 through the GPU path: an identity statement
    (x = 0) is allowed and its proof verifies; malformed blobs are rejected by
    Proof.from_bytes; a serialised proof is between 32 bytes and 1 KB."""
    x = np.zeros((1, 32), np.uint8)
    k = np.frombuffer(O.bench_scalar(b"k", 77).to_bytes(32, "little"), np.uint8).reshape(1, 32)
    out = gpu.prove(x, k)
    assert out["y1"][0].tobytes() == bytes(32) and out["y2"][0].tobytes() == bytes(32)
    st = gpu.verify_each(out["y1"], out["y2"], out["r1"], out["r2"], out["s"])
    assert list(st) == [0]
    for blob in (b"", b"\x00", b"\xff" * 10, b"\x01" * 1000):
        with pytest.raises(cp.Error):
            cp.Proof.from_bytes(blob, gpu)
    p = cp.Proof(out["r1"][0].tobytes(), out["r2"][0].tobytes(), out["s"][0].tobytes())
    assert 32 < len(p.to_bytes()) < 1024 and cp.Proof.from_bytes(p.to_bytes(), gpu).to_bytes() == p.to_bytes()


def _cons_rows(recs):
    return [np.frombuffer(b"".join(getattr(r, k) for r in recs), np.uint8).reshape(-1, 32)
            for k in ("y1", "y2", "r1", "r2", "s")]


def test_commitment_checks_off_equals_verify_one_on_constructed_proofs(gpu):
    """Proofs built with Proof::new(Commitment::new(..), Response::new(..)) (gadgets.rs:252, 278,
    317) skip from_bytes' identity / zero-s checks, and the reference's verify_one
    (batch.rs:185-231) judges them by the equations alone.  With commitment checks off
    (cpz_ctx_set_commitment_checks) the GPU does the same -- per proof, through the RLC
    batch check and its fallback, with caller challenges, and through the mirrors:
      nonce k = 0            -> r1 = r2 = identity, s = c x: valid (default mode: status 4)
      x = 0, k = 0           -> identity statement and commitment, s = 0: valid (default: 4)
      valid proof with s = 0 -> equation failure (default: 5)."""
    x = O.bench_scalar(b"x", 4242)
    k0 = O.prove(x, 0)
    assert k0.r1 == bytes(32) and k0.r2 == bytes(32)
    zz = O.prove(0, 0)
    assert zz.s == bytes(32) and zz.y1 == bytes(32)
    s0 = O.prove(x, 99)
    s0.s = bytes(32)
    ok = O.prove(x, 7)
    recs = [ok, k0, zz, s0]
    rows = _cons_rows(recs)
    default = [O.verify_one(r) for r in recs]
    eq_only = [O.verify_one(r, commitment_checks=False) for r in recs]
    assert default == [0, 4, 4, 5] and eq_only == [0, 0, 0, 1]
    assert list(gpu.verify_each(*rows)) == default
    # per call (CPZ_CALL_EQUATIONS_ONLY): the context's mode is untouched
    assert list(gpu.verify_each(*rows, equations_only=True)) == eq_only
    _, bok, st = gpu.verify_batch(*rows, seed=bytes(range(32)), equations_only=True)
    assert not bok and list(st) == eq_only
    # the RLC weights the identity-commitment entries (they are valid): the partial is the
    # oracle's with the same checks off, i.e. the s = 0 entry's alone
    part, _, _ = gpu.verify_batch(*rows, seed=bytes(range(32)), statuses=False, equations_only=True)
    want = O.rlc_partial(recs, bytes(range(32)), commitment_checks=False)
    assert part == O.ristretto_encode(want)
    assert part == O.ristretto_encode(O.rlc_partial([s0], bytes(range(32)), base_index=3,
                                                    commitment_checks=False))
    _, bok, st = gpu.verify_batch(*[r[:3] for r in rows], seed=bytes(range(32)), equations_only=True)
    assert bok and not st.any()
    c = gpu.challenges(*rows[:4])
    assert list(gpu.verify_response(*rows, c, equations_only=True)) == eq_only
    assert list(gpu.verify_each(*rows)) == default
    # the context's mode (cpz_ctx_set_commitment_checks): every call until it is switched back
    gpu.set_commitment_checks(False)
    try:
        assert list(gpu.verify_each(*rows)) == eq_only
        _, bok, st = gpu.verify_batch(*rows, seed=bytes(range(32)))
        assert not bok and list(st) == eq_only
        assert list(gpu.verify_response(*rows, c)) == eq_only
    finally:
        gpu.set_commitment_checks(True)
    # back to the default mode
    assert list(gpu.verify_each(*rows)) == default
    _, bok, st = gpu.verify_batch(*rows, seed=bytes(range(32)))
    assert not bok and list(st) == default
    # the mirrors hold Proof values (Proof::new): equations only, as the reference
    b = cp.BatchVerifier(gpu)
    params = cp.Parameters()
    for r in recs:
        b.add(params, cp.Statement(r.y1, r.y2), cp.Proof(r.r1, r.r2, r.s))
    res = b.verify()
    assert [v.status for v in res] == eq_only
    cp.Verifier(params, cp.Statement(k0.y1, k0.y2), gpu).verify(cp.Proof(k0.r1, k0.r2, k0.s))
    cp.Verifier(params, cp.Statement(zz.y1, zz.y2), gpu).verify(cp.Proof(zz.r1, zz.r2, zz.s))
    with pytest.raises(cp.InvalidParams):
        cp.Verifier(params, cp.Statement(s0.y1, s0.y2), gpu).verify(cp.Proof(s0.r1, s0.r2, s0.s))
    # but Proof.from_bytes (the wire) still rejects them, with the reference's messages
    with pytest.raises(cp.InvalidParams, match="Commitment contains identity element"):
        cp.Proof.from_bytes(cp.Proof(k0.r1, k0.r2, k0.s).to_bytes(), gpu)
    with pytest.raises(cp.InvalidParams, match="Response scalar is zero"):
        cp.Proof.from_bytes(cp.Proof(s0.r1, s0.r2, s0.s).to_bytes(), gpu)


def test_batch_verifier_rng_consumption_and_csprng(gpu):
    """The mirror draws `rng` as the reference does (batch.rs:178-180, 239-240): nothing for
    one entry, one 64-byte random_scalar per entry otherwise, whatever entry point runs; a
    predictable random.Random is refused when the RLC check would be keyed by it."""
    import random
    import secrets

    class Counting:
        def __init__(self):
            self.calls = []
            self._r = secrets.SystemRandom()

        def randbytes(self, k):
            self.calls.append(k)
            return self._r.randbytes(k)

    params = cp.Parameters()
    recs = [O.prove(O.bench_scalar(b"x", i), 11 + i) for i in range(5)]
    for n in (1, 2, 5):
        for rlc_min in (1, cp.RLC_MIN_GROUP):
            b = cp.BatchVerifier(gpu)
            for r in recs[:n]:
                b.add(params, cp.Statement(r.y1, r.y2), cp.Proof(r.r1, r.r2, r.s))
            rng = Counting()
            res = b.verify(rng, rlc_min_group=rlc_min)
            assert all(v.is_ok() for v in res)
            assert rng.calls == ([64] * n if n > 1 else [])
    b = cp.BatchVerifier(gpu)
    for r in recs[:3]:
        b.add(params, cp.Statement(r.y1, r.y2), cp.Proof(r.r1, r.r2, r.s))
    with pytest.raises(cp.InvalidParams, match="cryptographic rng"):
        b.verify(random.Random(5), rlc_min_group=1)
    # the per-proof path does not key anything by the rng: a seeded rng is accepted there
    assert all(v.is_ok() for v in b.verify(random.Random(5)))
    assert all(v.is_ok() for v in b.verify(secrets.SystemRandom(), rlc_min_group=1))


def test_add_time_statement_validation_and_capacity(gpu, golden):
    """batch.rs:158 (statement.validate() in add_with_context) and batch.rs:113-118."""
    b = cp.BatchVerifier.with_capacity(5000, gpu)
    assert b.capacity == cp.MAX_BATCH_SIZE
    rec = O.prove(O.bench_scalar(b"x", 1), 3)
    bad = bytes.fromhex(golden["rfc9496_bad"][0])
    with pytest.raises(cp.InvalidGroupElement):
        b.add(cp.Parameters(), cp.Statement(bad, rec.y2), cp.Proof(rec.r1, rec.r2, rec.s))
    assert b.is_empty()
    b.add(cp.Parameters(), cp.Statement(rec.y1, rec.y2), cp.Proof(rec.r1, rec.r2, rec.s))
    assert b.len() == 1 and b.verify()[0].is_ok()


def test_equations_only_is_per_call_across_threads(gpu):
    """CPZ_CALL_EQUATIONS_ONLY applies to its own call only: one thread verifies
    with the flag while another, on the same context, verifies in the context's default mode;
    neither ever sees the other's mode."""
    import threading
    x = O.bench_scalar(b"x", 5151)
    recs = [O.prove(x, 7), O.prove(x, 0)]          # valid; nonce 0: identity commitments
    rows = _cons_rows(recs)
    bad = []

    def run(eq, want):
        for _ in range(25):
            got = list(gpu.verify_each(*rows, equations_only=eq))
            if got != want:
                bad.append((eq, got))
            _, _, st = gpu.verify_batch(*rows, seed=bytes(32), equations_only=eq)
            if list(st) != want:
                bad.append((eq, "batch", list(st)))

    th = [threading.Thread(target=run, args=(True, [0, 0])), threading.Thread(target=run, args=(False, [0, 4]))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not bad, bad[:4]


def test_generator_cache_two_pairs_two_contexts(golden):
    """A context keeps the tables of several (g, h) pairs: two host threads, each on its own
    context, alternate the default and the golden custom generators -- each context builds
    each pair's tables once (stage 7 counts the builds) and every status is right."""
    import threading
    cg = golden["custom_generators"]
    pa = cp.Parameters()
    pb = cp.Parameters(bytes.fromhex(cg["g"]), bytes.fromhex(cg["h"]))
    rows = {}
    with cp.Gpu(0) as g0:
        for key, p in (("a", pa), ("b", pb)):
            out = g0.prove([O.bench_scalar(b"x", i) for i in range(40)],
                           [O.bench_scalar(b"k", i) for i in range(40)], params=p)
            rows[key] = [out[q] for q in ("y1", "y2", "r1", "r2", "s")]
    gpus = [cp.Gpu(0), cp.Gpu(0)]
    builds, bad = [0, 0], []

    def run(k):
        g = gpus[k]
        g.set_timing(True)
        g.stage_times()
        for it in range(8):
            key, p, other = ("a", pa, pb) if (it + k) % 2 == 0 else ("b", pb, pa)
            if list(g.verify_each(*rows[key], params=p)) != [0] * 40:
                bad.append((k, it, "own"))
            if list(g.verify_each(*rows[key], params=other)) != [1] * 40:   # wrong generators
                bad.append((k, it, "other"))
            _, ok, st = g.verify_batch(*rows[key], seed=bytes(range(32)), params=p)
            if not ok or st.any():
                bad.append((k, it, "batch"))
        builds[k] = g.stage_times().get("generators", (0.0, 0))[1]
        g.set_timing(False)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for g in gpus:
        g.close()
    assert not bad, bad[:4]
    assert builds == [2, 2], builds
