"""Pins for the CPU oracle itself (oracle/pyoracle.py) before it is trusted:
RFC 9496 vectors, the public merlin KAT, hashlib's SHA3 (Keccak-f), and -- when the
container's libsodium 1.0.18 is present -- an independent ristretto255 / ChaCha20.
The reference's own tests hold no fixed vectors."""
import ctypes
import hashlib
import os
import random

import pytest

import pyoracle as O

SODIUM = "/opt/conda/lib/libsodium.so"


def test_rfc9496_vectors(golden):
    for k, enc in enumerate(golden["rfc9496_multiples"]):
        assert O.ristretto_encode(O.pt_mul(O.BASEPOINT, k)).hex() == enc
        p = O.ristretto_decode(bytes.fromhex(enc))
        assert p is not None and O.ristretto_encode(p).hex() == enc
    for enc in golden["rfc9496_bad"]:
        assert O.ristretto_decode(bytes.fromhex(enc)) is None


def test_generators(golden):
    assert O.G_BYTES.hex() == golden["g"] == "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76"
    assert O.H_BYTES.hex() == golden["h"]


def test_keccak_vs_sha3():
    for msg in (b"", b"abc", bytes(range(256)) * 3):
        assert O.sha3_256(msg) == hashlib.sha3_256(msg).digest()


def test_merlin_kat(golden):
    k = golden["merlin_kat"]
    t = O.MerlinTranscript(k["protocol"].encode())
    t.append_message(k["label"].encode(), k["message"].encode())
    assert t.challenge_bytes(k["challenge_label"].encode(), k["n"]).hex() == k["out"]


def test_chacha20_rfc8439_block():
    # RFC 8439 section 2.3.2 test vector (block function; 32-bit counter 1, nonce 000000090000004a00000000)
    key = bytes(range(32))
    init = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    init += [int.from_bytes(key[4 * i:4 * i + 4], "little") for i in range(8)]
    init += [1, 0x09000000, 0x4A000000, 0x00000000]
    out = O.chacha20_block_words(init)
    assert out.hex().startswith("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e")


def test_golden_self_consistency(golden):
    for p in golden["proofs"]:
        rec = O.ProofRecord(*(bytes.fromhex(p[k]) for k in ("y1", "y2", "r1", "r2", "s")),
                            ctx=None if p["ctx"] is None else bytes.fromhex(p["ctx"]))
        assert O.verify_one(rec) == p["status"], p["kind"]


def test_reference_batch_equation_is_defective():
    """for >= 2 valid proofs the reference's batch equation (batch.rs:271-312)
    fails, so verify() falls back to per-entry verification; the corrected RLC holds."""
    recs = [O.prove(O.bench_scalar(b"x", i), O.bench_scalar(b"k", i)) for i in range(2)]
    alphas = [O.batch_weight(b"\x07" * 32, i) for i in range(2)]
    assert not O.reference_batch_equation(recs, alphas)
    assert O.reference_verify(recs, alphas) == [O.ST_OK, O.ST_OK]
    assert O.pt_is_identity(O.rlc_partial(recs, b"\x07" * 32))


@pytest.mark.skipif(not os.path.exists(SODIUM), reason="libsodium not present")
def test_against_libsodium():
    so = ctypes.CDLL(SODIUM)
    assert so.sodium_init() >= 0
    rnd = random.Random(11)
    out = ctypes.create_string_buffer(32)
    for _ in range(20):
        k = rnd.randrange(1, O.L)
        so.crypto_scalarmult_ristretto255_base(out, k.to_bytes(32, "little"))
        assert out.raw == O.ristretto_encode(O.pt_mul(O.BASEPOINT, k))
    so.crypto_core_ristretto255_from_hash(out, hashlib.sha512(O.GENERATOR_H_DST).digest())
    assert out.raw == O.H_BYTES
    for _ in range(200):
        b = bytes(rnd.getrandbits(8) for _ in range(32))
        b = bytes([b[0] & 0xFE]) + b[1:31] + bytes([b[31] & 0x7F])
        assert (O.ristretto_decode(b) is not None) == (so.crypto_core_ristretto255_is_valid_point(b) == 1 or b == bytes(32))
    key = bytes(range(32))
    ks = ctypes.create_string_buffer(192)
    so.crypto_stream_chacha20(ks, ctypes.c_ulonglong(192), bytes(8), key)
    assert ks.raw == O.chacha20_block(key, 0) + O.chacha20_block(key, 1) + O.chacha20_block(key, 2)
