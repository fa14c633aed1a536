"""Kernel-timing harness for experiments (variant libraries via CPZ_LIB): times
k_verify_each on 2^20 synthetic proofs with the runtime's HIP-event stage timers and does
NOT check verdicts -- for timing variants that deliberately compute wrong answers.  The
reported bench number always comes from bench.py, which refuses invalid verdicts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))


def _clock_summary(w):
    """Per-wave clock records (rows of 5 int64: shader ticks, 100 MHz ticks, 100 MHz start /
    end, hw id) -> mean / p10 / p90 shader clock in GHz and the wave time in us."""
    import numpy as np
    w = w[w[:, 1] > 0]
    ghz = w[:, 0] / (w[:, 1] / 100e6) / 1e9
    us = w[:, 1] / 100.0
    return {"waves": int(len(w)), "shader_clock_ghz": {"mean": round(float(ghz.mean()), 4),
                                                        "p10": round(float(np.percentile(ghz, 10)), 4),
                                                        "p90": round(float(np.percentile(ghz, 90)), 4)},
            "wave_time_us": {"mean": round(float(us.mean()), 1), "p10": round(float(np.percentile(us, 10)), 1),
                             "p90": round(float(np.percentile(us, 90)), 1)}}


def rlc_probe(cp, gpu, t, status, steps):
    """MODE=rlc: the RLC batch check of the same proofs; the last step's k_rlc_prepare and
    k_rlc_bucket clock stamps (cpz_ctx_clock_probe, CPZ_CLOCK_PROBE builds) and their
    HIP-event times per step."""
    import ctypes
    import json

    import numpy as np
    import torch
    seed = bytes(range(32))
    for _ in range(2):
        gpu.verify_batch_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status, seed)
    torch.cuda.synchronize()
    gpu.set_timing(True)
    gpu.stage_times()
    for _ in range(steps):
        _, ok = gpu.verify_batch_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status, seed)
    torch.cuda.synchronize()
    st = gpu.stage_times()
    lib = cp._native.load()
    fn = lib.cpz_ctx_clock_probe
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    out = {"what": "k_rlc_prepare / k_rlc_bucket built with -DCPZ_CLOCK_PROBE -DCPZ_TIMING_ONLY (rlc_dev.h "
                   "ClockStamp): per wave, s_memtime / s_memrealtime around its work; the last of %d RLC steps "
                   "over 2^20 proofs (tools/time_verify.py MODE=rlc)" % steps, "batch_ok": bool(ok)}
    for k, name, stage in ((0, "k_rlc_prepare", "rlc_prepare"), (1, "k_rlc_bucket", "rlc_bucket")):
        got = ctypes.c_size_t(0)
        buf = np.zeros((1 << 22) * 5, np.uint64)
        cp._native.check(fn(gpu._h, k, buf.ctypes.data, 1 << 22, ctypes.byref(got)))
        w = buf[:5 * min(got.value, 1 << 22)].reshape(-1, 5).astype(np.int64)
        rec = _clock_summary(w)
        ms, cnt = st.get(stage, (0.0, 1))
        rec["kernel_ms_per_step"] = ms / max(cnt, 1)
        out[name] = rec
    print(json.dumps(out))


def c5_probe(cp, gpu, steps):
    """MODE=c5: a configs[4]-shaped batch (N proofs, default 2^22, 0.1 % s + 1 forgeries) through
    the batch check's partitioned fallback; the first pass's k_part_acc clock stamps (kernel 2 of
    cpz_ctx_clock_probe: one record per wave = per 128-proof block, of the last walk launch)
    and its HIP-event time (stage 14) per call.  Verdicts are not checked (timing-only build)."""
    import ctypes
    import json

    import numpy as np
    import torch
    n = int(os.environ.get("N", 1 << 22))
    dev = torch.device("cuda", 0)
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    gpu.prove_synthetic_device(n, bytes(32), bytes(range(32)), t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    idx = np.sort(np.random.default_rng(2024).choice(n, size=max(1, n // 1000), replace=False))
    sys.path.insert(0, ROOT)
    import bench
    bench._bump_s(torch, t, idx)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    rows = [t[k] for k in ("y1", "y2", "r1", "r2", "s")]
    seed = bytes(range(32))
    gpu.verify_batch_device(*rows, status, seed, fallback=True)
    torch.cuda.synchronize()
    gpu.set_timing(True)
    gpu.stage_times()
    for _ in range(steps):
        gpu.verify_batch_device(*rows, status, seed, fallback=True)
    torch.cuda.synchronize()
    st = gpu.stage_times()
    lib = cp._native.load()
    fn = lib.cpz_ctx_clock_probe
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    got = ctypes.c_size_t(0)
    buf = np.zeros((1 << 20) * 5, np.uint64)
    cp._native.check(fn(gpu._h, 2, buf.ctypes.data, 1 << 20, ctypes.byref(got)))
    w = buf[:5 * min(got.value, 1 << 20)].reshape(-1, 5).astype(np.int64)
    rec = _clock_summary(w)
    ms, cnt = st.get("part_acc", (0.0, 1))
    rec["kernel_ms_per_call"] = ms / max(steps, 1)
    rec["launches_per_call"] = cnt / max(steps, 1)
    print(json.dumps({"what": "k_part_acc built with -DCPZ_CLOCK_PROBE -DCPZ_TIMING_ONLY (rlc_dev.h ClockStamp): per "
                              "wave (one 128-proof block), s_memtime / s_memrealtime around its walk; the partitioned "
                              "check's first pass over %d proofs with 0.1 %% forged, last of %d calls "
                              "(tools/time_verify.py MODE=c5)" % (n, steps),
                      "fallback": gpu.fallback_stats(), "k_part_acc": rec}))


def main():
    import torch
    import chaum_pedersen as cp
    n, steps = 1 << 20, int(os.environ.get("STEPS", "10"))
    dev = torch.device("cuda", 0)
    # a timing-only build (csrc/timing_only.h) opens its context through the timing entry
    gpu = cp.Gpu(0, timing_only=hasattr(cp._native.load(), "cpz_ctx_create_timing_only"))
    if os.environ.get("MODE") == "c5":
        return c5_probe(cp, gpu, steps)
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    gpu.prove_synthetic_device(n, bytes(32), bytes(range(32)), t["y1"], t["y2"], t["r1"], t["r2"], t["s"])
    if os.environ.get("MODE") == "rlc":
        return rlc_probe(cp, gpu, t, status, steps)
    for _ in range(2):
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status)
    torch.cuda.synchronize()
    gpu.set_timing(True)
    gpu.stage_times()
    for _ in range(steps):
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status)
    torch.cuda.synchronize()
    st = gpu.stage_times()
    v_ms, v_cnt = st.get("verify_each", (0.0, 1))
    print("%-14s verify_each %.3f ms  rejected %d" % (os.path.basename(os.environ.get("CPZ_LIB", "default")),
                                                     v_ms / v_cnt, int((status != 0).sum().item())))
    if os.environ.get("CLOCK"):
        # a CPZ_CLOCK_PROBE build (last step's launches): per wave, shader-clock and 100 MHz
        # ticks of its work, its absolute 100 MHz start / end and its SIMD
        import numpy as np
        w = status.cpu().numpy().view("uint64").reshape(-1, 8)[:, :5].astype("int64")
        ghz = w[:, 0] / (w[:, 1] / 100e6) / 1e9
        us = w[:, 1] / 100.0
        print("clock probe: %d waves, shader clock %.3f GHz (p10 %.3f, p90 %.3f), wave time %.0f us (p10 %.0f, p90 %.0f)"
              % (len(ghz), ghz.mean(), np.percentile(ghz, 10), np.percentile(ghz, 90), us.mean(),
                 np.percentile(us, 10), np.percentile(us, 90)))
        hw = w[:, 4]
        # HW_REG_HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13]; XCC id in the high word
        simd = ((hw >> 32) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) | (((hw >> 8) & 15) << 3) | \
            ((hw >> 4) & 3)
        t0, t1 = w[:, 2], w[:, 3]
        lo, hi = t0.min(), t1.max()
        span_us = (hi - lo) / 100.0
        busy = 0.0
        occ = np.zeros(4)
        for sid in np.unique(simd):
            m = simd == sid
            ev = sorted([(x, 1) for x in t0[m]] + [(x, -1) for x in t1[m]])
            cur, last = 0, lo
            for x, d in ev:
                occ[min(cur, 3)] += x - last
                last, cur = x, cur + d
            occ[0] += hi - last
            busy += (t1[m] - t0[m]).sum()
        nsimd = len(np.unique(simd))
        occ /= occ.sum()
        print("timeline: %d SIMDs, span %.0f us (first wave start .. last wave end), mean waves/SIMD %.3f; "
              "time share with 0/1/2/3+ waves resident: %s" % (nsimd, span_us, busy / nsimd / (hi - lo),
                                                               " / ".join("%.3f" % x for x in occ)))


if __name__ == "__main__":
    main()
