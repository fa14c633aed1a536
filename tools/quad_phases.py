"""Where a small synchronous per-proof call spends its time: with the CPZ_CLOCK_PROBE timing
build (CPZ_LIB=lib/timing/clock_probe.so), k_verify_quad stamps the shader clock at its phase
boundaries for block 0's first proof (kernels.hip) -- challenge split and digits, the decode,
the two tables, the Straus loop, the comb, the verdict -- and the 100 MHz clock around it, so
the phases come out in microseconds at the kernel's own clock.  N proofs per call (default 1),
CALLS calls, median per phase; the wall time of the synchronous call beside it."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
sys.path.insert(0, ROOT)

NAMES = ("split_digits", "decode", "tables", "straus", "comb", "verdict")


def main():
    import numpy as np
    import bench
    import chaum_pedersen as cp
    n = int(os.environ.get("N", "1"))
    calls = int(os.environ.get("CALLS", "50"))
    lib = cp._native.load()
    gpu = cp.Gpu(0, timing_only=hasattr(lib, "cpz_ctx_create_timing_only"))
    params = None
    if os.environ.get("CUSTOM"):   # a custom pair: the variable-base form
        o = gpu.prove([5, 7], [5, 7])
        params = cp.Parameters(o["y1"][0].tobytes(), o["y1"][1].tobytes())
    rows = gpu.prove_synthetic(n, bench.SEED_X, bench.SEED_K, params=params)
    cols = [np.ascontiguousarray(rows[k]) for k in ("y1", "y2", "r1", "r2", "s")]
    fn = lib.cpz_ctx_clock_probe
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    per, wall, clk = {k: [] for k in NAMES}, [], []
    for it in range(calls + 3):
        t0 = time.perf_counter()
        gpu.verify_each(*cols, params=params, equations_only=True)
        el = (time.perf_counter() - t0) * 1e6
        buf = np.zeros(10, np.uint64)
        got = ctypes.c_size_t(0)
        cp._native.check(fn(gpu._h, 3, buf.ctypes.data, 2, ctypes.byref(got)))
        if it < 3:
            continue
        st = buf[:9].astype(np.int64)
        real_us = (st[8] - st[7]) / 100.0
        ticks = st[6] - st[0]
        ghz = ticks / (real_us * 1e3) if real_us > 0 else float("nan")
        clk.append(ghz)
        for k, name in enumerate(NAMES):
            per[name].append((st[k + 1] - st[k]) / (ghz * 1e3))
        wall.append(el)
    out = {"n": n, "calls": calls, "custom_pair": bool(params), "kernel_clock_ghz": statistics.median(clk),
           "phase_us": {k: round(statistics.median(v), 1) for k, v in per.items()},
           "kernel_us": round(sum(statistics.median(v) for v in per.values()), 1),
           "call_wall_us": round(statistics.median(wall), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
