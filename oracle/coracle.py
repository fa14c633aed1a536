"""ctypes wrapper of the C oracle (oracle/cpz_oracle.c -> oracle/liboracle_cpz.so).

TEST / MEASUREMENT INFRASTRUCTURE ONLY: used by tests/ as the at-scale checker and by
bench.py's cpu_baseline leg.  The product path never imports this module.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_cpz.so")
_lib = None
_p = ctypes.c_void_p

DEFAULT_G = bytes.fromhex("e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76")
DEFAULT_H = bytes.fromhex("c8db6f46e1b91e7e93ace69eab46976efebe07deaf5b9a2a7442fd0236401623")
WEIGHT_SEED = hashlib.sha256(b"cpz-weights-v1").digest()


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "cpz_oracle.c")):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        lib = ctypes.CDLL(LIB)
        lib.cpzo_verify_one.restype = ctypes.c_int
        lib.cpzo_verify_one.argtypes = [_p] * 7 + [_p, ctypes.c_uint64, ctypes.c_int]
        lib.cpzo_verify_many.restype = None
        lib.cpzo_verify_many.argtypes = [_p, _p, ctypes.c_size_t] + [_p] * 6
        lib.cpzo_reference_batch_verify.restype = ctypes.c_int
        lib.cpzo_reference_batch_verify.argtypes = [_p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, ctypes.c_uint64, _p]
        lib.cpzo_challenge.restype = None
        lib.cpzo_challenge.argtypes = [_p] * 7 + [_p, ctypes.c_uint64, ctypes.c_int]
        lib.cpzo_decode_encode.restype = ctypes.c_int
        lib.cpzo_decode_encode.argtypes = [_p, _p]
        lib.cpzo_scalar_mul.restype = ctypes.c_int
        lib.cpzo_scalar_mul.argtypes = [_p, _p, _p]
        lib.cpzo_point_sum.restype = ctypes.c_int
        lib.cpzo_point_sum.argtypes = [_p, ctypes.c_size_t, _p]
        lib.cpzo_sc_reduce_wide.argtypes = [_p, _p]
        lib.cpzo_sc_mul.argtypes = [_p, _p, _p]
        lib.cpzo_chacha_block.argtypes = [_p, _p, ctypes.c_uint64, ctypes.c_uint64]
        lib.cpzo_verify_many_ctx.restype = None
        lib.cpzo_verify_many_ctx.argtypes = [_p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p]
        lib.cpzo_challenge_many.restype = None
        lib.cpzo_challenge_many.argtypes = [_p, _p, ctypes.c_size_t] + [_p] * 4 + [_p, _p, _p, _p]
        lib.cpzo_rlc_partial.restype = ctypes.c_long
        lib.cpzo_rlc_partial.argtypes = [_p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p, _p, _p]
        _lib = lib
    return _lib


def _c(b):
    return ctypes.c_char_p(bytes(b)) if b is not None else None


def verify_one(g, h, y1, y2, r1, r2, s, ctx=None) -> int:
    lib = load()
    cb = b"" if ctx is None else bytes(ctx)
    return lib.cpzo_verify_one(g, h, bytes(y1), bytes(y2), bytes(r1), bytes(r2), bytes(s), cb, len(cb),
                               0 if ctx is None else 1)


def challenge(g, h, y1, y2, r1, r2, ctx=None) -> bytes:
    lib = load()
    out = ctypes.create_string_buffer(32)
    cb = b"" if ctx is None else bytes(ctx)
    lib.cpzo_challenge(out, g, h, bytes(y1), bytes(y2), bytes(r1), bytes(r2), cb, len(cb), 0 if ctx is None else 1)
    return out.raw


def _rows(rows, k, lo, hi):
    a = np.ascontiguousarray(rows[k][lo:hi], dtype=np.uint8)
    return a, a.ctypes.data


def verify_many(rows, lo=0, hi=None, g=DEFAULT_G, h=DEFAULT_H, threads=1) -> np.ndarray:
    """Per-proof statuses for rows[k][lo:hi] (k in y1,y2,r1,r2,s), on `threads` threads
    (ctypes releases the GIL during each call)."""
    lib = load()
    hi = len(rows["y1"]) if hi is None else hi
    out = np.zeros(hi - lo, np.uint8)
    chunks = np.array_split(np.arange(lo, hi), max(1, threads))
    keep = []

    def work(idx):
        if len(idx) == 0:
            return
        a, b = int(idx[0]), int(idx[-1]) + 1
        arrs = [_rows(rows, k, a, b) for k in ("y1", "y2", "r1", "r2", "s")]
        keep.append(arrs)
        sub = np.zeros(b - a, np.uint8)
        lib.cpzo_verify_many(g, h, b - a, *[p for _, p in arrs], sub.ctypes.data)
        out[a - lo:b - lo] = sub

    ts = [threading.Thread(target=work, args=(c,)) for c in chunks]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def _ctx_arrays(contexts, n):
    """None -> (None, None, None); else (blob, absolute offsets[n + 1], present[n])."""
    if contexts is None:
        return None, None, None
    present = np.array([0 if c is None else 1 for c in contexts], np.uint8)
    lens = np.array([0 if c is None else len(c) for c in contexts], np.uint64)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(c for c in contexts if c is not None) + b"\0", np.uint8).copy()
    return blob, off, present


def _pp(a):
    return None if a is None else a.ctypes.data


def _parallel(n, threads, fn):
    """fn(lo, hi) on `threads` threads over [0, n) (ctypes releases the GIL)."""
    bounds = [(n * t) // threads for t in range(threads + 1)]
    ts = [threading.Thread(target=fn, args=(bounds[t], bounds[t + 1])) for t in range(threads) if bounds[t + 1] > bounds[t]]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def verify_many_ctx(rows, contexts=None, g=DEFAULT_G, h=DEFAULT_H, threads=1) -> np.ndarray:
    """Per-proof statuses (decode + verify_one) for rows (dict of (n, 32) arrays) with an
    optional context per entry (None / bytes), on `threads` threads."""
    lib = load()
    n = len(rows["y1"])
    arr = [np.ascontiguousarray(rows[k], dtype=np.uint8) for k in ("y1", "y2", "r1", "r2", "s")]
    blob, off, present = _ctx_arrays(contexts, n)
    out = np.zeros(n, np.uint8)

    def work(lo, hi):
        lib.cpzo_verify_many_ctx(g, h, hi - lo, *[a[lo:].ctypes.data for a in arr], _pp(blob),
                                 None if off is None else off[lo:].ctypes.data,
                                 None if present is None else present[lo:].ctypes.data, out[lo:].ctypes.data)
    _parallel(n, max(1, threads), work)
    return out


def challenge_many(rows, contexts=None, g=DEFAULT_G, h=DEFAULT_H, threads=1) -> np.ndarray:
    """Transcript challenges (n, 32) for rows with optional contexts."""
    lib = load()
    n = len(rows["y1"])
    arr = [np.ascontiguousarray(rows[k], dtype=np.uint8) for k in ("y1", "y2", "r1", "r2")]
    blob, off, present = _ctx_arrays(contexts, n)
    out = np.zeros((n, 32), np.uint8)

    def work(lo, hi):
        lib.cpzo_challenge_many(g, h, hi - lo, *[a[lo:].ctypes.data for a in arr], _pp(blob),
                                None if off is None else off[lo:].ctypes.data,
                                None if present is None else present[lo:].ctypes.data, out[lo:].ctypes.data)
    _parallel(n, max(1, threads), work)
    return out


def rlc_partial(rows, gidx, seed, contexts=None, g=DEFAULT_G, h=DEFAULT_H, threads=1):
    """(encoding, live count) of the corrected RLC partial over the given entries, whose
    global batch indices are gidx (weights keyed by them).  Threads sum disjoint slices
    (partials combined by cpzo_point_sum)."""
    lib = load()
    n = len(rows["y1"])
    arr = [np.ascontiguousarray(rows[k], dtype=np.uint8) for k in ("y1", "y2", "r1", "r2", "s")]
    gi = np.ascontiguousarray(np.asarray(gidx, dtype=np.uint64))
    blob, off, present = _ctx_arrays(contexts, n)
    parts, lives = {}, {}

    def work(lo, hi):
        out = ctypes.create_string_buffer(32)
        live = lib.cpzo_rlc_partial(g, h, hi - lo, *[a[lo:].ctypes.data for a in arr], _pp(blob),
                                    None if off is None else off[lo:].ctypes.data,
                                    None if present is None else present[lo:].ctypes.data, gi[lo:].ctypes.data,
                                    bytes(seed), out)
        parts[lo], lives[lo] = out.raw, live
    _parallel(n, max(1, threads), work)
    if len(parts) == 1:
        return parts[min(parts)], sum(lives.values())
    out = ctypes.create_string_buffer(32)
    blob_p = b"".join(parts[k] for k in sorted(parts))
    assert lib.cpzo_point_sum(out, len(parts), blob_p) == 1
    return out.raw, sum(lives.values())


def reference_batch_verify(rows, lo, hi, g=DEFAULT_G, h=DEFAULT_H, seed=WEIGHT_SEED):
    """BatchVerifier::verify semantics on rows[lo:hi] (<= 1000 entries)."""
    lib = load()
    arrs = [_rows(rows, k, lo, hi) for k in ("y1", "y2", "r1", "r2", "s")]
    out = np.zeros(hi - lo, np.uint8)
    ok = lib.cpzo_reference_batch_verify(g, h, hi - lo, *[p for _, p in arrs], seed, lo, out.ctypes.data)
    return ok, out


def time_verify(rows, seconds: float = 12.0, threads: int = 1, batch: int = 1000):
    """CPU baseline: the reference's BatchVerifier::verify (batches of <= 1000, defective
    batch equation + per-entry fallback) on `threads` threads over a bounded sample of
    `rows`, stopping after ~`seconds`; plus verify_one (per-proof loop) on the same
    threads.  Proofs/s, aggregated over threads."""
    load()
    n = len(rows["y1"])
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass

    def run(mode, budget, threads=threads):
        done = [0] * threads
        stop = time.perf_counter() + budget

        def work(tid):
            lo = (tid * n) // threads
            hi = ((tid + 1) * n) // threads
            pos = lo
            while time.perf_counter() < stop:
                if mode == "batch":
                    e = min(pos + batch, hi)
                    ok, st = reference_batch_verify(rows, pos, e)
                    assert not st.any(), "CPU baseline rejected a valid proof"
                    done[tid] += e - pos
                    pos = e if e < hi else lo
                else:
                    e = min(pos + 64, hi)
                    st = verify_many(rows, pos, e, threads=1)
                    assert not st.any(), "CPU baseline rejected a valid proof"
                    done[tid] += e - pos
                    pos = e if e < hi else lo

        t0 = time.perf_counter()
        ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        el = time.perf_counter() - t0
        return sum(done) / el, sum(done), el

    b_rate, b_n, b_t = run("batch", seconds * 0.6)
    o_rate, o_n, o_t = run("one", seconds * 0.3)
    # the reference itself is single-threaded: the same batch loop on one core
    s_rate, s_n, _ = run("batch", seconds * 0.1, threads=1) if threads > 1 else (b_rate, b_n, b_t)
    return {
        "value": b_rate, "unit": "proofs/s", "cores": threads, "kind": "port",
        "sample": "%d proofs: the first %d of the same synthetic set (verified until the time budget ran out, "
                  "wrapping); BatchVerifier::verify semantics in batches of %d (batch.rs:171-318, defective "
                  "equation then per-entry fallback), from 32-byte encodings (decode included)"
                  % (b_n, n, batch),
        "seconds": b_t,
        "verify_one_value": o_rate,
        "verify_one_sample": "%d proofs, per-proof verify_one loop (batch.rs:185-231) incl. decode" % o_n,
        "single_thread_value": s_rate,
        "single_thread_sample": "%d proofs, the BatchVerifier::verify loop above on 1 thread" % s_n,
        "cpu_model": cpu_model,
        "implementation": "oracle/cpz_oracle.c (C restatement of dalek's u64 backend + merlin; gcc -O3)",
    }
