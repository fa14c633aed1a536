"""The partitioned batch check's digit bounds (csrc/part.hip, part_width; csrc/rlc.h,
kPartTopBuckets), checked on the host against the prepare's recoding (rlc_dev.h recode16):
every MSM scalar of a block -- a c and b c (reduced mod l), the block sums of a s and b s
(reduced mod l), the 128-bit weights (windows 0..7 only) -- splits into signed 8-bit digits
d = lo + 2^8 hi with |lo| <= 128, |hi| <= 128, and the top window's high halves are <= 16, so
the four lanes of the top window cover buckets 1..16 (4 each) and k_part_sort never has to
mark a block for an out-of-range digit.  Pure arithmetic, no GPU."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as O  # noqa: E402

TOP_BUCKETS = 16  # kPartTopBuckets


def recode16(s):
    """rlc_dev.h recode16: 16 signed radix-2^16 digits of s < 2^253."""
    d, carry = [], 0
    for w in range(16):
        chunk = ((s >> (16 * w)) & 0xFFFF) + carry
        carry = (chunk + 0x8000) >> 16
        d.append(chunk - (carry << 16))
    assert carry == 0
    return d


def split8(d):
    """part.hip split8."""
    lo = ((d + 128) & 255) - 128
    return lo, (d - lo) >> 8


def test_top_window_high_halves_at_most_16():
    rng = random.Random(20261017)
    extremes = [0, 1, O.L - 1, O.L - 2, (1 << 252) - 1, 1 << 252, O.L - (1 << 239), (1 << 240) * 4096 - 1]
    samples = extremes + [rng.randrange(O.L) for _ in range(20000)]
    worst = 0
    for s in samples:
        d = recode16(s)
        assert all(-(1 << 15) <= x < (1 << 15) for x in d)
        assert 0 <= d[15] <= 4097
        for x in d:
            lo, hi = split8(x)
            assert -128 <= lo < 128 and -128 <= hi <= 128 and lo + 256 * hi == x
        worst = max(worst, abs(split8(d[15])[1]))
    assert worst <= TOP_BUCKETS
    # the bound is tight: scalars just below l reach it
    assert abs(split8(recode16(O.L - 1)[15])[1]) == TOP_BUCKETS
