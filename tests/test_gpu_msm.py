"""The Pippenger MSM kernels alone (cpz_msm) against the oracle's sum of scalar
multiples, including adversarial digit patterns: windows equal to 0x8000 (digit -2^15,
the top bucket), all-0xffff chunks (carry chains), collisions (the same point several
times, P and -P), zero scalars and single points."""
import random

import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu


def _pts(k, seed):
    rnd = random.Random(seed)
    return [O.pt_mul(O.BASEPOINT, rnd.randrange(1, O.L)) for _ in range(k)]


def _check(gpu, pts, scal):
    want = O.IDENTITY
    for P, k in zip(pts, scal):
        want = O.pt_add(want, O.pt_mul(P, k))
    got = gpu.msm([O.ristretto_encode(P) for P in pts], scal)
    assert got == O.ristretto_encode(want)


def test_msm_random(gpu):
    rnd = random.Random(1)
    for n in (1, 2, 5, 64):
        pts = _pts(n, n)
        _check(gpu, pts, [rnd.randrange(O.L) for _ in range(n)])


def test_msm_adversarial_digits(gpu):
    pts = _pts(6, 7)
    specials = [
        int("8000" * 15 + "0fff", 16) % (1 << 253),                  # every window 0x8000
        sum(0x8000 << (16 * w) for w in range(15)),                      # digit -2^15 everywhere
        (1 << 253) - 1,                                                  # all ones -> carries
        O.L - 1, 1, 0,
    ]
    _check(gpu, pts, specials)
    _check(gpu, pts[:1], [specials[1]])
    _check(gpu, [pts[0]] * 4, [5, 5, 5, 5])                             # same bucket, same point
    P = pts[1]
    _check(gpu, [P, O.pt_neg(P)], [12345, 12345])                        # P + (-P)
    _check(gpu, [P, P], [O.L - 3, 3])


def test_msm_buckets_spanning_chunks(gpu):
    """Buckets far larger than one accumulation chunk (64 sorted entries per thread): the
    owner / head partials of every chunk a bucket spans must all be summed."""
    B = O.BASEPOINT
    pts, P = [], B
    for _ in range(300):
        pts.append(P)                       # (i + 1) B
        P = O.pt_add(P, B)
    rnd = random.Random(5)
    small = [5, 0x00030001, (7 << 240) | (9 << 16) | 2]                # a few distinct digit patterns
    scal = [small[rnd.randrange(3)] for _ in range(300)]
    want = O.pt_mul(B, sum((i + 1) * k for i, k in enumerate(scal)) % O.L)
    assert gpu.msm([O.ristretto_encode(Q) for Q in pts], scal) == O.ristretto_encode(want)
    # one bucket per window holding all 300 entries (5 chunks), same point repeated
    assert gpu.msm([O.ristretto_encode(B)] * 300, [0x8000_0003] * 300) == \
        O.ristretto_encode(O.pt_mul(B, 300 * 0x8000_0003 % O.L))


def test_msm_single_weights_from_failing_case(gpu, golden):
    """The single-proof RLC partial (golden forged proof #3) at several first indices."""
    case = golden["rlc"][1]
    p = case["proofs"][3]
    rec = O.ProofRecord(*(bytes.fromhex(p[k]) for k in ("y1", "y2", "r1", "r2", "s")))
    seed = bytes.fromhex(case["seed"])
    import numpy as np
    arr = lambda k: np.frombuffer(bytes.fromhex(p[k]), np.uint8).reshape(1, 32)
    for fi in range(0, 16):
        part, ok, st = gpu.verify_batch(*[arr(k) for k in ("y1", "y2", "r1", "r2", "s")], seed=seed,
                                        first_index=fi, statuses=False)
        assert part == O.ristretto_encode(O.rlc_partial([rec], seed, fi)), fi
