"""Checks tools/ubench/wide_mul's outputs: every element squared `chain` times, in both
layouts, against Python's pow(x, 2^chain, p)."""
import sys

import numpy as np

P = 2**255 - 19


def main(path):
    raw = open(path, "rb").read()
    nelem, n16, chain = np.frombuffer(raw[:12], np.int32)
    off = 12
    words = np.frombuffer(raw[off:off + nelem * 32], np.uint32).reshape(nelem, 8)
    off += nelem * 32
    o25 = np.frombuffer(raw[off:off + nelem * 32], np.uint32).reshape(nelem, 8)
    off += nelem * 32
    o16 = np.frombuffer(raw[off:off + n16 * 64], np.int32).reshape(n16, 16)       # r16b
    off += n16 * 64
    o16a = np.frombuffer(raw[off:off + n16 * 64], np.int32).reshape(n16, 16)      # r16
    off += n16 * 64
    o16c = np.frombuffer(raw[off:off + n16 * 64], np.int32).reshape(n16, 16)      # r16c
    e = pow(2, int(chain), P - 1)
    bad25 = bad16 = 0
    for i in range(nelem):
        x = sum(int(w) << (32 * j) for j, w in enumerate(words[i]))
        want = pow(x, e, P)
        got = sum(int(w) << (32 * j) for j, w in enumerate(o25[i]))
        bad25 += got != want
        if i < n16:
            for o in (o16, o16a, o16c):
                g16 = sum(int(l) << (16 * k) for k, l in enumerate(o[i])) % P
                bad16 += g16 != want
    lim = int(max(np.abs(o16).max(), np.abs(o16a).max(), np.abs(o16c).max()))
    print('{"elements_r25": %d, "bad_r25": %d, "elements_r16": %d, "bad_r16": %d, "max_abs_limb_r16": %d}'
          % (nelem, bad25, n16, bad16, lim))
    return 1 if bad25 or bad16 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
