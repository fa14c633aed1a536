"""Expected work of one partitioned-check block (k_part_sort / k_part_acc, csrc/part.hip) for
bench/opcount.json's "part" entry: the number of non-zero signed radix-2^8 digits (walk
entries) over a block's kPartProofs = 128 proofs, simulated with the prepare's own scalars --
the r-points' 128-bit weights as their eight int16 words, the y-points' a c and b c mod l and
the block sums of a s, b s mod l recoded to signed radix-2^16 digits (rlc_dev.h recode16) and
each digit split into two signed bytes (part.hip split8) -- with uniform weights, challenges
and responses.  Boundaries (bucket ends the walk visits) are fixed: 31 windows x 128 buckets
+ the top window's 16."""
import json
import random

L = 2**252 + 27742317777372353535851937790883648493


def recode16(s):
    d, carry = [], 0
    for w in range(16):
        chunk = ((s >> (16 * w)) & 0xffff) + carry
        carry = (chunk + 0x8000) >> 16
        d.append(chunk - (carry << 16))
    return d


def split8(d):
    lo = ((d + 128) & 255) - 128
    return lo, (d - lo) >> 8


def nonzero_bytes(digits):
    n = 0
    for d in digits:
        lo, hi = split8(d)
        n += (lo != 0) + (hi != 0)
    return n


def block_entries(rng, proofs=128):
    n, sa, sb = 0, 0, 0
    for _ in range(proofs):
        words = [rng.getrandbits(16) for _ in range(16)]
        signed = [w - 65536 if w >= 32768 else w for w in words]
        a = sum(signed[k] << (16 * k) for k in range(8)) % L
        b = sum(signed[8 + k] << (16 * k) for k in range(8)) % L
        c, s = rng.randrange(L), rng.randrange(1, L)
        n += nonzero_bytes(signed[:8]) + nonzero_bytes(signed[8:])          # -r1, -r2: the weights
        n += nonzero_bytes(recode16(a * c % L)) + nonzero_bytes(recode16(b * c % L))  # -y1, -y2
        sa, sb = (sa + a * s) % L, (sb + b * s) % L
    return n + nonzero_bytes(recode16(sa)) + nonzero_bytes(recode16(sb))      # g, h


def main(blocks=64, seed=5):
    rng = random.Random(seed)
    e = [block_entries(rng) for _ in range(blocks)]
    mean = sum(e) / len(e)
    print(json.dumps({"blocks_simulated": blocks, "entries_per_block": round(mean, 1),
                      "min": min(e), "max": max(e), "boundaries_per_block": 31 * 128 + 16}))


if __name__ == "__main__":
    main()
