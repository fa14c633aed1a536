"""Where a small synchronous per-proof call spends its time: with the CPZ_CLOCK_PROBE timing
build (CPZ_LIB=lib/timing/clock_probe.so) the per-proof kernel stamps the shader clock at its
phase boundaries for block 0 (kernels.hip) and the 100 MHz clock around it, so the phases come
out in microseconds at the kernel's own clock.  k_verify_wide (launches of <= CPZ_WIDE_MAX
proofs, default 512): wave 0's decode, table, wait for wave 4's digits, Straus, wait, combine,
verdict, wave 4's challenge + split and [s'] B, and wave 1's decode, table and Straus (the
wave 0 / wave 4 SIMD sharing shows against it).  k_verify_small (launches of <= 2048 proofs):
wave 0's decode, table, wait for wave 2's digits, Straus, wait for the partial sums, verdict,
and wave 2's challenge + split and [s'] B; k_verify_quad (larger launches, or a library built
with CPZ_VERIFY_SMALL=0; KERNEL=quad): split, decode, tables, Straus, comb, verdict.  N proofs
per call (default 1), CALLS calls, median per phase; the synchronous call's wall time beside."""
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
WIDE = (("decode", 0, 1), ("table", 1, 2), ("wait_digits", 2, 3), ("straus", 3, 4), ("wait_partials", 4, 5),
        ("combine", 5, 6), ("verdict", 6, 7), ("w4_challenge", 0, 12), ("w4_split_digits", 12, 8),
        ("w4_s_B", 8, 9), ("w1_decode", 0, 13), ("w1_table", 13, 14), ("w1_straus", 3, 15))
SMALL = (("decode", 0, 1), ("table", 1, 2), ("wait_digits", 2, 3), ("straus", 3, 4), ("wait_partials", 4, 5),
         ("verdict", 5, 6), ("w2_challenge_split", 11, 7), ("w2_s_B", 7, 8))


def main():
    import numpy as np
    import bench
    import chaum_pedersen as cp
    n = int(os.environ.get("N", "1"))
    calls = int(os.environ.get("CALLS", "50"))
    lib = cp._native.load()
    gpu = cp.Gpu(0, timing_only=hasattr(lib, "cpz_ctx_create_timing_only"))
    params = None
    pg = gpu
    if os.environ.get("CUSTOM"):   # a custom pair proved on another context: variable bases here
        pg = cp.Gpu(0, timing_only=hasattr(lib, "cpz_ctx_create_timing_only"))
        o = pg.prove([5, 7], [5, 7])
        params = cp.Parameters(o["y1"][0].tobytes(), o["y1"][1].tobytes())
    rows = pg.prove_synthetic(n, bench.SEED_X, bench.SEED_K, params=params)
    cols = [np.ascontiguousarray(rows[k]) for k in ("y1", "y2", "r1", "r2", "s")]
    fn = lib.cpz_ctx_clock_probe
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    wide_max = int(os.environ.get("CPZ_WIDE_MAX", "512"))
    kern = os.environ.get("KERNEL", "wide" if n <= wide_max else ("small" if n <= 2048 else "quad"))
    small = kern in ("small", "wide")
    table = WIDE if kern == "wide" else SMALL
    names = [x[0] for x in table] if small else list(NAMES)
    per, wall, clk = {k: [] for k in names}, [], []
    for it in range(calls + 3):
        t0 = time.perf_counter()
        gpu.verify_each(*cols, params=params, equations_only=True)
        el = (time.perf_counter() - t0) * 1e6
        buf = np.zeros(16, np.uint64)
        got = ctypes.c_size_t(0)
        cp._native.check(fn(gpu._h, 3, buf.ctypes.data, 3, ctypes.byref(got)))
        if it < 3:
            continue
        st = buf[:16].astype(np.int64)
        if kern == "wide":
            real_us, ticks = (st[11] - st[10]) / 100.0, st[7] - st[0]
        elif small:
            real_us, ticks = (st[10] - st[9]) / 100.0, st[6] - st[0]
        else:
            real_us, ticks = (st[8] - st[7]) / 100.0, st[6] - st[0]
        ghz = ticks / (real_us * 1e3) if real_us > 0 else float("nan")
        clk.append(ghz)
        if small:
            for name, a, b in table:
                per[name].append((st[b] - st[a]) / (ghz * 1e3))
        else:
            for k, name in enumerate(NAMES):
                per[name].append((st[k + 1] - st[k]) / (ghz * 1e3))
        wall.append(el)
    if os.environ.get("RAW"):  # the last call's stamps, relative to wave 0's start
        print(json.dumps({"raw_stamps_minus_start": [int(x - st[0]) if x else 0 for x in st]}))
    med = {k: round(statistics.median(v), 1) for k, v in per.items()}
    out = {"n": n, "calls": calls, "kernel": "k_verify_" + kern,
           "custom_pair": bool(params), "kernel_clock_ghz": statistics.median(clk), "phase_us": med,
           "kernel_us": round(sum(med[k] for k in names if not k.startswith(("w1_", "w2_", "w4_"))), 1),
           "call_wall_us": round(statistics.median(wall), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
