"""Stand-alone cost of the no-context challenge kernel: cpz_challenges over N proofs (env N,
default 2^20, one launch of k_challenge_noctx), REPS times; run under
`rocprofv3 --kernel-trace --stats` for the kernel's own duration with nothing beside it."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))


def main():
    import chaum_pedersen as cp

    n = int(os.environ.get("N", 1 << 20))
    reps = int(os.environ.get("REPS", "5"))
    gpu = cp.Gpu(0)
    rng = np.random.default_rng(1)
    # any 32-byte strings: the transcript absorbs them as bytes (no decode on this path)
    rows = [rng.integers(0, 256, size=(n, 32), dtype=np.uint8) for _ in range(4)]
    gpu.challenges(*rows)
    t0 = time.perf_counter()
    for _ in range(reps):
        gpu.challenges(*rows)
    el = (time.perf_counter() - t0) / reps
    print('{"n": %d, "reps": %d, "host_ms_per_call": %.3f}' % (n, reps, el * 1e3))


if __name__ == "__main__":
    main()
