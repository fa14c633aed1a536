"""CPU oracle (pure Python, small cases) for the Chaum-Pedersen batch-verify hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP kernels, the
C-ABI library, the host runtime) may import or call this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker.

It restates, in plain Python integers, what the reference computes on the
verify path.  The reference (Rust, kobby-pentangeli/chaum-pedersen-zkp) keeps
all arithmetic in third-party crates that are not vendored under
/root/reference and cannot be built here (no cargo/rustc); their published
algorithms are restated instead:

* curve25519-dalek 4.1.3 (Cargo.lock:607-619) -> ristretto255 per RFC 9496
  (decode, encode, equality, hash-to-group), F_p = GF(2^255-19), scalars mod l.
* merlin 3.0.0 (Cargo.lock:1182-1191) -> STROBE-128 v1.0.2 over Keccak-f[1600]
  with Merlin v1.0 framing.
* sha2 0.10.9 (Cargo.lock:1954) -> hashlib.sha512.
* rand_chacha 0.3.1 (Cargo.lock:1603-1606) -> ChaCha20 block function; the
  batch weights are alpha_i = wide_reduce(ChaCha20(seed) block i), i.e.
  ``random_scalar(&mut ChaCha20Rng::from_seed(seed))`` drawn in entry order.

Parity pins (see tests/test_oracle_pins.py): libsodium 1.0.18's independent
ristretto255 / ChaCha20 (this container only), hashlib.sha3_256 for
Keccak-f, the public merlin known-answer test, and RFC 9496's published
basepoint-multiple encodings.

Reference call sites restated here:
  src/primitives/transcript.rs:10-71   (labels, message order, challenge_scalar)
  src/primitives/ristretto.rs:79-221   (generators, (de)serialisation, scalar ops)
  src/primitives/gadgets.rs:343-489    (109-byte proof wire format, rejections)
  src/verifier/batch.rs:171-318        (verify / verify_one / verify_batch / fallback)
  src/verifier/mod.rs:120-171          (verify_with_transcript / verify_response)
  src/prover/mod.rs:86-131             (prove_with_transcript / commit / respond)
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

# ----------------------------------------------------------------------------
# F_p, p = 2^255 - 19
# ----------------------------------------------------------------------------
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493  # group order (scalars)

D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)


def fe_is_negative(x: int) -> bool:
    return (x % P) & 1 == 1


def fe_abs(x: int) -> int:
    x %= P
    return (P - x) % P if fe_is_negative(x) else x


def sqrt_ratio_m1(u: int, v: int) -> Tuple[bool, int]:
    """RFC 9496 section 4.2 SQRT_RATIO_M1."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (P - u) % P
    flipped_i = check == (P - u) * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    r = fe_abs(r)
    return (correct or flipped), r


# RFC 9496 section 4.1 constants.  SQRT_AD_MINUS_ONE is the odd ("negative") root there.
SQRT_AD_MINUS_ONE = 25063068953384623474111414158702152701244531502492656460079210482610430750235
assert SQRT_AD_MINUS_ONE * SQRT_AD_MINUS_ONE % P == (-D - 1) % P
INVSQRT_A_MINUS_D = sqrt_ratio_m1(1, (-1 - D) % P)[1]
assert INVSQRT_A_MINUS_D == 54469307008909316920995813868745141605393597292927456921205312896311721017578
ONE_MINUS_D_SQ = (1 - D * D) % P
D_MINUS_ONE_SQ = (D - 1) * (D - 1) % P

# ----------------------------------------------------------------------------
# Edwards points, extended coordinates (X:Y:Z:T), a = -1
# ----------------------------------------------------------------------------
Point = Tuple[int, int, int, int]
IDENTITY: Point = (0, 1, 1, 0)


def pt_add(p1: Point, p2: Point) -> Point:
    x1, y1, z1, t1 = p1
    x2, y2, z2, t2 = p2
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = t1 * D2 % P * t2 % P
    d = z1 * 2 * z2 % P
    e, f, g, h = (b - a) % P, (d - c) % P, (d + c) % P, (b + a) % P
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def pt_neg(p1: Point) -> Point:
    x, y, z, t = p1
    return ((-x) % P, y, z, (-t) % P)


def pt_mul(p1: Point, k: int) -> Point:
    """Scalar multiplication (value semantics of dalek `RistrettoPoint * Scalar`)."""
    k %= L
    acc = IDENTITY
    base = p1
    while k:
        if k & 1:
            acc = pt_add(acc, base)
        base = pt_add(base, base)
        k >>= 1
    return acc


def pt_eq(p1: Point, p2: Point) -> bool:
    """Ristretto equality, RFC 9496 section 4.3.3 (dalek `RistrettoPoint::eq`)."""
    x1, y1, _, _ = p1
    x2, y2, _, _ = p2
    return (x1 * y2 - y1 * x2) % P == 0 or (y1 * y2 - x1 * x2) % P == 0


def pt_is_identity(p1: Point) -> bool:
    return pt_eq(p1, IDENTITY)


# ----------------------------------------------------------------------------
# Ristretto255 encode / decode / hash-to-group (RFC 9496 section 4.3)
# ----------------------------------------------------------------------------

def ristretto_decode(b: bytes) -> Optional[Point]:
    """`CompressedRistretto::decompress` (ristretto.rs:120-138 -> dalek)."""
    if len(b) != 32:
        return None
    s = int.from_bytes(b, "little")
    if s >= P or (s & 1):
        return None
    ss = s * s % P
    u1 = (1 - ss) % P
    u2 = (1 + ss) % P
    u2_sqr = u2 * u2 % P
    v = (-(D * u1 % P * u1) - u2_sqr) % P
    was_square, invsqrt = sqrt_ratio_m1(1, v * u2_sqr)
    den_x = invsqrt * u2 % P
    den_y = invsqrt * den_x % P * v % P
    x = fe_abs(2 * s * den_x)
    y = u1 * den_y % P
    t = x * y % P
    if not was_square or fe_is_negative(t) or y == 0:
        return None
    return (x, y, 1, t)


def ristretto_encode(pt: Point) -> bytes:
    """`RistrettoPoint::compress` (ristretto.rs:141-143 -> dalek)."""
    x0, y0, z0, t0 = pt
    u1 = (z0 + y0) * (z0 - y0) % P
    u2 = x0 * y0 % P
    _, invsqrt = sqrt_ratio_m1(1, u1 * u2 % P * u2)
    den1 = invsqrt * u1 % P
    den2 = invsqrt * u2 % P
    z_inv = den1 * den2 % P * t0 % P
    ix0 = x0 * SQRT_M1 % P
    iy0 = y0 * SQRT_M1 % P
    enchanted = den1 * INVSQRT_A_MINUS_D % P
    rotate = fe_is_negative(t0 * z_inv)
    x, y = (iy0, ix0) if rotate else (x0, y0)
    den_inv = enchanted if rotate else den2
    if fe_is_negative(x * z_inv):
        y = (-y) % P
    s = fe_abs(den_inv * (z0 - y))
    return s.to_bytes(32, "little")


def _elligator_map(t: int) -> Point:
    r = SQRT_M1 * t % P * t % P
    u = (r + 1) * ONE_MINUS_D_SQ % P
    v = (-1 - r * D) * (r + D) % P
    was_square, s = sqrt_ratio_m1(u, v)
    s_prime = (-fe_abs(s * t)) % P
    if not was_square:
        s = s_prime
    c = (P - 1) if was_square else r
    n = (c * (r - 1) % P * D_MINUS_ONE_SQ - v) % P
    w0 = 2 * s * v % P
    w1 = n * SQRT_AD_MINUS_ONE % P
    w2 = (1 - s * s) % P
    w3 = (1 + s * s) % P
    return (w0 * w3 % P, w2 * w1 % P, w1 * w3 % P, w0 * w2 % P)


def ristretto_from_uniform_bytes(b: bytes) -> Point:
    """`RistrettoPoint::from_uniform_bytes` (ristretto.rs:90 -> dalek)."""
    assert len(b) == 64
    r0 = int.from_bytes(b[:32], "little") & ((1 << 255) - 1)
    r1 = int.from_bytes(b[32:], "little") & ((1 << 255) - 1)
    return pt_add(_elligator_map(r0 % P), _elligator_map(r1 % P))


# ----------------------------------------------------------------------------
# Scalars mod l (ristretto.rs:94-112, 146-150, 198-221)
# ----------------------------------------------------------------------------

def scalar_from_canonical(b: bytes) -> Optional[int]:
    """`Scalar::from_canonical_bytes`: None unless the 32 bytes encode a value < l."""
    if len(b) != 32:
        return None
    v = int.from_bytes(b, "little")
    return v if v < L else None


def scalar_wide(b: bytes) -> int:
    """`Scalar::from_bytes_mod_order_wide` (64 bytes LE mod l)."""
    assert len(b) == 64
    return int.from_bytes(b, "little") % L


def scalar_bytes(k: int) -> bytes:
    return (k % L).to_bytes(32, "little")


# ----------------------------------------------------------------------------
# Generators (ristretto.rs:27, 79-91)
# ----------------------------------------------------------------------------
GENERATOR_H_DST = b"chaum-pedersen-zkp-v1.0.0-generator-h"
# RISTRETTO_BASEPOINT: the Ed25519 basepoint, y = 4/5, x positive (even).
_BY = 4 * pow(5, P - 2, P) % P
_BX2 = (_BY * _BY - 1) * pow(D * _BY * _BY + 1, P - 2, P) % P
_BX = pow(_BX2, (P + 3) // 8, P)
if (_BX * _BX - _BX2) % P != 0:
    _BX = _BX * SQRT_M1 % P
if _BX & 1:
    _BX = P - _BX
BASEPOINT: Point = (_BX, _BY, 1, _BX * _BY % P)


def generator_g() -> Point:
    return BASEPOINT


def generator_h() -> Point:
    return ristretto_from_uniform_bytes(hashlib.sha512(GENERATOR_H_DST).digest())


G_BYTES = ristretto_encode(BASEPOINT)
H_BYTES = ristretto_encode(generator_h())

# ----------------------------------------------------------------------------
# Keccak-f[1600], STROBE-128 (v1.0.2), Merlin v1.0   (merlin 3.0.0)
# ----------------------------------------------------------------------------
_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_ROT = [
    [0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56], [27, 20, 39, 8, 14],
]
_M64 = (1 << 64) - 1


def _rol(v: int, n: int) -> int:
    return ((v << n) | (v >> (64 - n))) & _M64 if n else v


def keccak_f1600(state: bytearray) -> None:
    """In-place Keccak-f[1600] on 200 bytes (lanes little-endian, A[x][y] = lane x+5y)."""
    a = [[int.from_bytes(state[8 * (x + 5 * y): 8 * (x + 5 * y) + 8], "little") for y in range(5)]
         for x in range(5)]
    for rnd in range(24):
        c = [a[x][0] ^ a[x][1] ^ a[x][2] ^ a[x][3] ^ a[x][4] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        a = [[a[x][y] ^ d[x] for y in range(5)] for x in range(5)]
        b = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                b[y][(2 * x + 3 * y) % 5] = _rol(a[x][y], _ROT[x][y])
        a = [[b[x][y] ^ ((~b[(x + 1) % 5][y]) & b[(x + 2) % 5][y]) for y in range(5)] for x in range(5)]
        a[0][0] ^= _RC[rnd]
    for x in range(5):
        for y in range(5):
            state[8 * (x + 5 * y): 8 * (x + 5 * y) + 8] = a[x][y].to_bytes(8, "little")


def sha3_256(msg: bytes) -> bytes:
    """SHA3-256 built on keccak_f1600 (used only to pin the permutation vs hashlib)."""
    rate = 136
    st = bytearray(200)
    m = bytearray(msg) + b"\x06"
    while len(m) % rate:
        m.append(0)
    m[-1] |= 0x80
    for off in range(0, len(m), rate):
        for i in range(rate):
            st[i] ^= m[off + i]
        keccak_f1600(st)
    return bytes(st[:32])


STROBE_R = 166
_FLAG_I, _FLAG_A, _FLAG_C, _FLAG_T, _FLAG_M, _FLAG_K = 1, 2, 4, 8, 16, 32


class Strobe128:
    """STROBE-128 as used by merlin 3.0.0 (meta_ad / ad / prf only)."""

    def __init__(self, protocol_label: bytes):
        st = bytearray(200)
        st[0:6] = bytes([1, STROBE_R + 2, 1, 0, 1, 96])
        st[6:18] = b"STROBEv1.0.2"
        keccak_f1600(st)
        self.state = st
        self.pos = 0
        self.pos_begin = 0
        self.cur_flags = 0
        self.permutations = 0
        self.meta_ad(protocol_label, False)

    def clone(self) -> "Strobe128":
        c = Strobe128.__new__(Strobe128)
        c.state = bytearray(self.state)
        c.pos, c.pos_begin, c.cur_flags = self.pos, self.pos_begin, self.cur_flags
        c.permutations = self.permutations
        return c

    def _run_f(self) -> None:
        self.state[self.pos] ^= self.pos_begin
        self.state[self.pos + 1] ^= 0x04
        self.state[STROBE_R + 1] ^= 0x80
        keccak_f1600(self.state)
        self.permutations += 1
        self.pos = 0
        self.pos_begin = 0

    def _absorb(self, data: bytes) -> None:
        for byte in data:
            self.state[self.pos] ^= byte
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()

    def _squeeze(self, n: int) -> bytes:
        out = bytearray(n)
        for i in range(n):
            out[i] = self.state[self.pos]
            self.state[self.pos] = 0
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()
        return bytes(out)

    def _begin_op(self, flags: int, more: bool) -> None:
        if more:
            assert self.cur_flags == flags
            return
        assert flags & _FLAG_T == 0
        old_begin = self.pos_begin
        self.pos_begin = self.pos + 1
        self.cur_flags = flags
        self._absorb(bytes([old_begin, flags]))
        if (flags & (_FLAG_C | _FLAG_K)) and self.pos != 0:
            self._run_f()

    def meta_ad(self, data: bytes, more: bool) -> None:
        self._begin_op(_FLAG_M | _FLAG_A, more)
        self._absorb(data)

    def ad(self, data: bytes, more: bool) -> None:
        self._begin_op(_FLAG_A, more)
        self._absorb(data)

    def prf(self, n: int, more: bool) -> bytes:
        self._begin_op(_FLAG_I | _FLAG_A | _FLAG_C, more)
        return self._squeeze(n)


class MerlinTranscript:
    """merlin 3.0.0 `Transcript`."""

    def __init__(self, label: bytes):
        self.strobe = Strobe128(b"Merlin v1.0")
        self.append_message(b"dom-sep", label)

    def append_message(self, label: bytes, message: bytes) -> None:
        self.strobe.meta_ad(label, False)
        self.strobe.meta_ad(struct.pack("<I", len(message)), True)
        self.strobe.ad(message, False)

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        self.strobe.meta_ad(label, False)
        self.strobe.meta_ad(struct.pack("<I", n), True)
        return self.strobe.prf(n, False)


# The protocol transcript (src/primitives/transcript.rs:10-71).
PROTOCOL_LABEL = b"Chaum-Pedersen ZKP v1.0.0"
PROTOCOL_DST = b"chaum-pedersen-ristretto255"
CHALLENGE_DST = b"challenge"


class Transcript:
    def __init__(self):  # transcript.rs:29-33
        self.t = MerlinTranscript(PROTOCOL_LABEL)
        self.t.append_message(b"protocol", PROTOCOL_DST)

    def append_context(self, ctx: bytes) -> None:  # transcript.rs:42-44
        self.t.append_message(b"context", ctx)

    def append_parameters(self, g: bytes, h: bytes) -> None:  # transcript.rs:47-50
        self.t.append_message(b"generator-g", g)
        self.t.append_message(b"generator-h", h)

    def append_statement(self, y1: bytes, y2: bytes) -> None:  # transcript.rs:53-56
        self.t.append_message(b"y1", y1)
        self.t.append_message(b"y2", y2)

    def append_commitment(self, r1: bytes, r2: bytes) -> None:  # transcript.rs:59-62
        self.t.append_message(b"r1", r1)
        self.t.append_message(b"r2", r2)

    def challenge_scalar(self) -> int:  # transcript.rs:67-71
        return scalar_wide(self.t.challenge_bytes(CHALLENGE_DST, 64))


def challenge(g: bytes, h: bytes, y1: bytes, y2: bytes, r1: bytes, r2: bytes,
              ctx: Optional[bytes] = None) -> int:
    """Fiat-Shamir challenge exactly as batch.rs:188-206 / verifier/mod.rs:123-136 build it."""
    t = Transcript()
    if ctx is not None:
        t.append_context(ctx)
    t.append_parameters(g, h)
    t.append_statement(y1, y2)
    t.append_commitment(r1, r2)
    return t.challenge_scalar()


# ----------------------------------------------------------------------------
# ChaCha20 (rand_chacha 0.3.1 ChaCha20Rng block function, 64-bit counter)
# ----------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _qr(s, a, b, c, d):
    s[a] = (s[a] + s[b]) & _M32; s[d] ^= s[a]; s[d] = ((s[d] << 16) | (s[d] >> 16)) & _M32
    s[c] = (s[c] + s[d]) & _M32; s[b] ^= s[c]; s[b] = ((s[b] << 12) | (s[b] >> 20)) & _M32
    s[a] = (s[a] + s[b]) & _M32; s[d] ^= s[a]; s[d] = ((s[d] << 8) | (s[d] >> 24)) & _M32
    s[c] = (s[c] + s[d]) & _M32; s[b] ^= s[c]; s[b] = ((s[b] << 7) | (s[b] >> 25)) & _M32


def chacha20_block_words(init: Sequence[int]) -> bytes:
    s = list(init)
    for _ in range(10):
        _qr(s, 0, 4, 8, 12); _qr(s, 1, 5, 9, 13); _qr(s, 2, 6, 10, 14); _qr(s, 3, 7, 11, 15)
        _qr(s, 0, 5, 10, 15); _qr(s, 1, 6, 11, 12); _qr(s, 2, 7, 8, 13); _qr(s, 3, 4, 9, 14)
    return b"".join(struct.pack("<I", (s[i] + init[i]) & _M32) for i in range(16))


def chacha20_block(key: bytes, counter: int, stream: int = 0) -> bytes:
    """djb ChaCha20 block: words 12-13 = 64-bit block counter, 14-15 = 64-bit stream id."""
    init = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    init += list(struct.unpack("<8I", key))
    init += [counter & _M32, (counter >> 32) & _M32, stream & _M32, (stream >> 32) & _M32]
    return chacha20_block_words(init)


def batch_weight(seed: bytes, index: int) -> int:
    """alpha_i: the i-th `random_scalar` drawn from ChaCha20Rng::from_seed(seed) (batch.rs:240)."""
    return scalar_wide(chacha20_block(seed, index))


def batch_weight2(seed: bytes, index: int) -> int:
    """gamma_i: independent weight for the second (h-) equation, ChaCha20 stream 1."""
    return scalar_wide(chacha20_block(seed, index, 1))


def rlc_weights(seed: bytes, index: int):
    """(a_i, b_i) of the corrected RLC batch check: 128-bit weights drawn as signed
    radix-2^16 digit vectors.  ChaCha20 block `index` (stream 0) read as 32 little-endian
    int16 words: a_i = sum_k w_k 2^(16k) over words 0..7, b_i over words 8..15 (mod l).
    Each weight is uniform over a set of 2^128 values (error 2^-128 per forged entry, the
    standard batch-verification bound), and its MSM digits are the words themselves: 8
    radix-2^16 windows, no carry -- half the bucket work of a full 253-bit weight."""
    w = struct.unpack("<32h", chacha20_block(seed, index))
    a = sum(w[k] << (16 * k) for k in range(8)) % L
    b = sum(w[8 + k] << (16 * k) for k in range(8)) % L
    return a, b


# ----------------------------------------------------------------------------
# Protocol: prover (input generator) and per-proof verification
# ----------------------------------------------------------------------------
ST_OK, ST_EQ_FAIL, ST_BAD_POINT, ST_BAD_SCALAR, ST_IDENTITY, ST_ZERO_S = 0, 1, 2, 3, 4, 5


@dataclass
class ProofRecord:
    y1: bytes
    y2: bytes
    r1: bytes
    r2: bytes
    s: bytes
    ctx: Optional[bytes] = None


def bench_scalar(tag: bytes, i: int, domain: bytes = b"cpz-bench-v1") -> int:
    """Deterministic witness / nonce derivation used for synthetic inputs."""
    return scalar_wide(hashlib.sha512(domain + tag + struct.pack("<Q", i)).digest())


def prove(x: int, k: int, ctx: Optional[bytes] = None, g: Point = BASEPOINT,
          h: Optional[Point] = None) -> ProofRecord:
    """`Prover::prove_with_transcript` (prover/mod.rs:86-131) with a given nonce k."""
    if h is None:
        h = generator_h()
    gb, hb = ristretto_encode(g), ristretto_encode(h)
    y1, y2 = ristretto_encode(pt_mul(g, x)), ristretto_encode(pt_mul(h, x))
    r1, r2 = ristretto_encode(pt_mul(g, k)), ristretto_encode(pt_mul(h, k))
    c = challenge(gb, hb, y1, y2, r1, r2, ctx)
    s = (k + c * x) % L
    return ProofRecord(y1, y2, r1, r2, scalar_bytes(s), ctx)


def decode_status(rec: ProofRecord, commitment_checks: bool = True):
    """Decode-time rejections, in the order the reference meets them.

    Statement points are decoded when the Statement is built (service.rs:82-86);
    then `Proof::from_bytes` (gadgets.rs:364-489): r1, r2 decode -> InvalidGroupElement,
    s non-canonical -> InvalidScalar, identity r1/r2 -> InvalidParams, zero s -> InvalidParams.
    commitment_checks=False: a Proof built with Proof::new(Commitment::new, Response::new)
    (gadgets.rs:252, 278, 317), which has no identity / zero-s checks -- verify_one judges it
    by the equations alone (cpz_ctx_set_commitment_checks(ctx, 0)).
    Returns (status, points or None, s or None).
    """
    y1 = ristretto_decode(rec.y1)
    y2 = ristretto_decode(rec.y2)
    if y1 is None or y2 is None:
        return ST_BAD_POINT, None, None
    r1 = ristretto_decode(rec.r1)
    r2 = ristretto_decode(rec.r2)
    if r1 is None or r2 is None:
        return ST_BAD_POINT, None, None
    s = scalar_from_canonical(rec.s)
    if s is None:
        return ST_BAD_SCALAR, None, None
    if commitment_checks and (pt_is_identity(r1) or pt_is_identity(r2)):
        return ST_IDENTITY, None, None      # gadgets.rs:474-478
    if commitment_checks and s == 0:
        return ST_ZERO_S, None, None        # gadgets.rs:480-482
    return ST_OK, (y1, y2, r1, r2), s


def verify_one(rec: ProofRecord, g_bytes: bytes = G_BYTES, h_bytes: bytes = H_BYTES,
               commitment_checks: bool = True) -> int:
    """`BatchVerifier::verify_one` (batch.rs:185-231) preceded by decode_status."""
    st, pts, s = decode_status(rec, commitment_checks)
    if st != ST_OK:
        return st
    y1, y2, r1, r2 = pts
    g = ristretto_decode(g_bytes)
    h = ristretto_decode(h_bytes)
    c = challenge(g_bytes, h_bytes, rec.y1, rec.y2, rec.r1, rec.r2, rec.ctx)
    lhs1 = pt_mul(g, s)
    rhs1 = pt_add(r1, pt_mul(y1, c))
    lhs2 = pt_mul(h, s)
    rhs2 = pt_add(r2, pt_mul(y2, c))
    return ST_OK if (pt_eq(lhs1, rhs1) and pt_eq(lhs2, rhs2)) else ST_EQ_FAIL


def verify_response(rec: ProofRecord, c_bytes: bytes, g_bytes: bytes = G_BYTES, h_bytes: bytes = H_BYTES,
                    commitment_checks: bool = True) -> int:
    """`Verifier::verify_response` (verifier/mod.rs:144-171) with a caller-supplied challenge,
    preceded by decode_status (the Proof / Statement were decoded before the call).  The
    challenge arrives as 32 bytes here: non-canonical bytes (scalar_from_bytes would fail,
    ristretto.rs:94-112) give ST_BAD_SCALAR, after the entry's own decode-level checks."""
    st, pts, s = decode_status(rec, commitment_checks)
    if st != ST_OK:
        return st
    c = scalar_from_canonical(c_bytes)
    if c is None:
        return ST_BAD_SCALAR
    y1, y2, r1, r2 = pts
    g = ristretto_decode(g_bytes)
    h = ristretto_decode(h_bytes)
    ok1 = pt_eq(pt_mul(g, s), pt_add(r1, pt_mul(y1, c)))
    ok2 = pt_eq(pt_mul(h, s), pt_add(r2, pt_mul(y2, c)))
    return ST_OK if (ok1 and ok2) else ST_EQ_FAIL


def reference_batch_equation(recs: Sequence[ProofRecord], alphas: Sequence[int],
                             g_bytes: bytes = G_BYTES, h_bytes: bytes = H_BYTES) -> bool:
    """`verify_batch_equations` (batch.rs:271-312) AS WRITTEN (rhs omits alpha on y*c)."""
    g = ristretto_decode(g_bytes)
    h = ristretto_decode(h_bytes)
    lhs1 = rhs1 = lhs2 = rhs2 = IDENTITY
    for rec, alpha in zip(recs, alphas):
        _, (y1, y2, r1, r2), s = decode_status(rec)
        c = challenge(g_bytes, h_bytes, rec.y1, rec.y2, rec.r1, rec.r2, rec.ctx)
        alpha_s = alpha * s % L
        lhs1 = pt_add(lhs1, pt_mul(g, alpha_s))
        rhs1 = pt_add(rhs1, pt_add(pt_mul(r1, alpha), pt_mul(y1, c)))
        lhs2 = pt_add(lhs2, pt_mul(h, alpha_s))
        rhs2 = pt_add(rhs2, pt_add(pt_mul(r2, alpha), pt_mul(y2, c)))
    return pt_eq(lhs1, rhs1) and pt_eq(lhs2, rhs2)


def reference_verify(recs: Sequence[ProofRecord], alphas: Optional[Sequence[int]] = None,
                     g_bytes: bytes = G_BYTES, h_bytes: bytes = H_BYTES) -> List[int]:
    """`BatchVerifier::verify` (batch.rs:171-183, 233-269, 314-318) per-entry outcome.

    Empty -> ValueError (batch.rs:172-176).  n == 1 -> verify_one.  n >= 2 -> defective
    batch equation, which fails for any n >= 2 valid batch with overwhelming probability,
    then per-entry fallback: so the result equals verify_one per entry.
    """
    if len(recs) == 0:
        raise ValueError("Cannot verify empty batch")
    if len(recs) == 1:
        return [verify_one(recs[0], g_bytes, h_bytes)]
    if alphas is not None and all(decode_status(r)[0] == ST_OK for r in recs):
        if reference_batch_equation(recs, alphas, g_bytes, h_bytes):
            return [ST_OK] * len(recs)
    return [verify_one(r, g_bytes, h_bytes) for r in recs]


# ----------------------------------------------------------------------------
# Corrected random-linear-combination (RLC) batch check (the MSM the GPU runs)
# ----------------------------------------------------------------------------

def rlc_partial(recs: Sequence[ProofRecord], seed: bytes, base_index: int = 0,
                g_bytes: bytes = G_BYTES, h_bytes: bytes = H_BYTES, commitment_checks: bool = True) -> Point:
    """Sum over valid-decoding entries i of

        [a_i s_i] G - [a_i] R1_i - [a_i c_i] Y1_i  +  [b_i s_i] H - [b_i] R2_i - [b_i c_i] Y2_i

    with (a_i, b_i) = rlc_weights(seed, base_index+i).
    Entries whose decode status is non-zero carry zero weight.  Identity iff every
    weighted entry satisfies both verification equations (w.o.p.).
    """
    g = ristretto_decode(g_bytes)
    h = ristretto_decode(h_bytes)
    acc = IDENTITY
    sg = sh = 0
    for j, rec in enumerate(recs):
        st, pts, s = decode_status(rec, commitment_checks)
        if st != ST_OK:
            continue
        y1, y2, r1, r2 = pts
        c = challenge(g_bytes, h_bytes, rec.y1, rec.y2, rec.r1, rec.r2, rec.ctx)
        a, b = rlc_weights(seed, base_index + j)
        sg = (sg + a * s) % L
        sh = (sh + b * s) % L
        acc = pt_add(acc, pt_mul(r1, (L - a) % L))
        acc = pt_add(acc, pt_mul(y1, (L - a * c % L) % L))
        acc = pt_add(acc, pt_mul(r2, (L - b) % L))
        acc = pt_add(acc, pt_mul(y2, (L - b * c % L) % L))
    acc = pt_add(acc, pt_mul(g, sg))
    acc = pt_add(acc, pt_mul(h, sh))
    return acc


# ----------------------------------------------------------------------------
# 109-byte proof wire format (gadgets.rs:343-489)
# ----------------------------------------------------------------------------
PROTOCOL_VERSION = 1


def proof_to_bytes(r1: bytes, r2: bytes, s: bytes) -> bytes:
    out = bytearray([PROTOCOL_VERSION])
    for part in (r1, r2, s):
        out += struct.pack(">I", len(part)) + part
    return bytes(out)


def proof_from_bytes(b: bytes):
    """Returns ('ok', (r1, r2, s)) or ('err', kind) following gadgets.rs:364-489."""
    if len(b) < 1 + 4 + 1 + 4 + 1 + 4 + 1:
        return "err", "InvalidParams"
    if b[0] != PROTOCOL_VERSION:
        return "err", "InvalidParams"
    pos = 1
    parts = []
    for idx, (kind, maxlen) in enumerate((("point", 4096), ("point", 4096), ("scalar", 512))):
        if pos + 4 > len(b):
            return "err", "InvalidParams"
        ln = struct.unpack(">I", b[pos:pos + 4])[0]
        pos += 4
        if ln == 0 or ln > maxlen:
            return "err", "InvalidParams"
        if pos + ln > len(b):
            return "err", "InvalidParams"
        field = b[pos:pos + ln]
        pos += ln
        if kind == "point":
            if ln != 32 or ristretto_decode(field) is None:
                return "err", "InvalidGroupElement"
        else:
            if ln != 32 or scalar_from_canonical(field) is None:
                return "err", "InvalidScalar"
        parts.append(field)
    if pos != len(b):
        return "err", "InvalidParams"
    r1, r2, s = parts
    if pt_is_identity(ristretto_decode(r1)) or pt_is_identity(ristretto_decode(r2)):
        return "err", "InvalidParams"
    if int.from_bytes(s, "little") == 0:
        return "err", "InvalidParams"
    return "ok", (r1, r2, s)


def proof_from_bytes_code(b: bytes):
    """(code, aux) of Proof::from_bytes (gadgets.rs:364-489) with the bulk parser's numbering
    (include/cpz.h CPZ_PARSE_*): the first check the reference fails, in its order; aux is
    the value its message prints (length, version, trailing count) or 0."""
    if len(b) < 1 + 4 + 1 + 4 + 1 + 4 + 1:
        return 1, len(b)
    if b[0] != PROTOCOL_VERSION:
        return 2, b[0]
    pos = 1
    parts = []
    for q, maxlen in enumerate((4096, 4096, 512)):
        base = 3 + 5 * q
        if pos + 4 > len(b):
            return base, 0
        ln = struct.unpack(">I", b[pos:pos + 4])[0]
        pos += 4
        if ln == 0 or ln > maxlen:
            return base + 1, ln
        if pos + ln > len(b):
            return base + 2, 0
        if ln != 32:                       # element_from_bytes / scalar_from_bytes size check
            return base + 3, ln
        field = b[pos:pos + 32]
        pos += 32
        ok = (ristretto_decode(field) is not None) if q < 2 else (scalar_from_canonical(field) is not None)
        if not ok:
            return base + 4, 0
        parts.append(field)
    if pos != len(b):
        return 18, len(b) - pos
    r1, r2, s = parts
    if pt_is_identity(ristretto_decode(r1)) or pt_is_identity(ristretto_decode(r2)):
        return 19, 0
    if int.from_bytes(s, "little") == 0:
        return 20, 0
    return 0, 0
