"""csrc/fe16.h (k_verify_wide's row arithmetic) carries the curve constants as 16-bit limbs; they
must equal d = -121665/121666, 2d and sqrt(-1) mod p (RFC 7748 / RFC 9496), the values the
radix-2^25.5 constants of fe25519.h hold.  CPU only: reads the header text."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**255 - 19


def _limbs(name):
    src = open(os.path.join(ROOT, "chaum-pedersen-zkp_amd", "csrc", "fe16.h")).read()
    m = re.search(r"int %s\(const Lane& L\) \{\s*constexpr uint16_t c\[16\] = \{([^}]*)\}" % name, src)
    assert m, name
    vals = [int(v, 16) for v in m.group(1).replace("\n", " ").split(",")]
    assert len(vals) == 16 and all(0 <= v < 1 << 16 for v in vals)
    return sum(v << (16 * k) for k, v in enumerate(vals))


def test_row_constants():
    d = (-121665 * pow(121666, P - 2, P)) % P
    assert _limbs("K_D") == d
    assert _limbs("K_D2") == 2 * d % P
    i = _limbs("K_SQRT_M1")
    assert i * i % P == P - 1
    # the same square root as fe25519.h's FE_SQRT_M1 (radix 2^25.5 limbs)
    src = open(os.path.join(ROOT, "chaum-pedersen-zkp_amd", "csrc", "fe25519.h")).read()
    m = re.search(r"FE_SQRT_M1\(\) \{ return fe_const\(([^)]*)\)", src)
    off = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    v = [int(x) for x in m.group(1).split(",")]
    assert sum(a << o for a, o in zip(v, off)) % P == i
