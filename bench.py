#!/usr/bin/env python3
"""Headline benchmark: verified Chaum-Pedersen proofs per second on MI355X.

Workload (BASELINE.json configs[1]): 2^20 ristretto255 Chaum-Pedersen proofs, per-proof
(non-batched) verification -- the reference's BatchVerifier::verify outcome per entry
(batch.rs:171-231) -- with inputs resident in HBM.  One step = one pass of the verify path
over the whole batch: k_challenge (Merlin/STROBE Fiat-Shamir challenges + response checks)
and k_verify_each (4 ristretto decodes + 2 half-size Straus equations per proof).  Inputs are
synthetic: valid proofs from the GPU prover (ChaCha20-derived witnesses, distinct per rank).

--mode rlc makes the step the random-linear-combination batch check (configs[2]; with
--n-total 67108864 on 8 ranks, configs[3]): each rank reduces its shard to a 32-byte partial
(weights keyed by the global index), the partials are all-gathered (RCCL over xGMI with the
"nccl" backend) and combined.

Multi-GPU (torchrun, one process per GPU): contiguous shards, no data-path collective in
'each' mode.  --n sets the proofs per GPU (weak scaling, the default); --n-total sets the
proofs of the whole job, split over the ranks (strong scaling, configs[3]).  value = all
ranks' proofs / max-over-ranks time.

Every line, at every N, carries a "c4" object: configs[3] at this world size -- 2^26 proofs split
over the ranks, per-rank RLC partial keyed by the global index, all-gather of the 32-byte
partials (RCCL over xGMI at N > 1), combine, barrier-timed and max over ranks; the valid set
must combine to the identity, and a forged variant (s + 1 in two ranks' shards) must give every
rank exactly its forged statuses and a non-identity total.  Fewer visible GPUs than ranks is
refused before the process group is set up.

At N = 1 the same run also measures (reported beside value, never as value): the RLC batch
check of the same proofs with per-kernel roofline fractions (configs[2]), the 2^24-proof
batch with 0.1 % forged proofs through the batch check + fallback (configs[4]), the prover
(proof generation, published ~144 us/proof, lib.rs:55), the host-buffer entry point (PCIe
included), the per-call latency of BatchVerifier-sized batches (n = 1 .. 1000, both entry
points, beside the CPU's BatchVerifier::verify), and the CPU baseline.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))

SEED_X = hashlib.sha256(b"cpz-bench-x").digest()
SEED_K = hashlib.sha256(b"cpz-bench-k").digest()
WEIGHT_SEED = hashlib.sha256(b"cpz-weights-v1").digest()
L = 2**252 + 27742317777372353535851937790883648493
METRIC = "verified proofs/sec (1/2/4/8 MI355X) + % int-VALU roofline vs host-CPU"


def _load_json(rel):
    p = os.path.join(ROOT, rel)
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def _profile(name):
    """The newest committed PMC summary of that name (profiles/rNN_<name>.json)."""
    cands = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_" + name + ".json"))
    return (_load_json(os.path.join("profiles", cands[-1])) or {}) if cands else {}


def _newest_profile(suffix):
    pdir = os.path.join(ROOT, "profiles")
    cands = sorted(f for f in os.listdir(pdir) if f.endswith(suffix))
    return (cands[-1], _load_json(os.path.join("profiles", cands[-1])) or {}) if cands else (None, {})


def mad_peak_at_kernel_clock(oc, kernel="k_verify_each"):
    """The v_mad_i64_i32 issue ceiling at the clock `kernel` itself runs at: the best measured
    lane rate per SIMD cycle (tools/ubench/clock_rates.hip, profiles/rNN_clock_rates.json:
    event-timed launch cycles at the measured shader clock) x 1024 SIMDs x the kernel's own
    shader clock from the in-kernel s_memtime / s_memrealtime probe of a timing-only build
    (profiles/rNN_verify_clock_probe.json for k_verify_each, profiles/rNN_rlc_clock_probe.json
    for k_rlc_prepare / k_rlc_bucket).  None when either file is missing."""
    cr_name, cr = _newest_profile("_clock_rates.json")
    if kernel == "k_verify_each":
        pr_name, pr = _newest_profile("_verify_clock_probe.json")
    elif kernel == "k_part_acc":
        pr_name, pr = _newest_profile("_c5_clock_probe.json")
        pr = pr.get(kernel) or {}
    else:
        pr_name, pr = _newest_profile("_rlc_clock_probe.json")
        pr = pr.get(kernel) or {}
    rows = [r for r in cr.get("rows", []) if r.get("op") == "v_mad_i64_i32"]
    clk = (pr.get("shader_clock_ghz") or {}).get("mean")
    if not rows or not clk:
        return None
    simds = 4 * cr.get("cus", 256)
    best = max(rows, key=lambda r: r.get("gops", 0.0))
    lanes = best.get("lanes_per_simd_cycle") or best["gops"] * 1e9 / (simds * best["clock_ghz"] * 1e9)
    return {"peak": lanes * simds * clk * 1e9, "lanes_per_simd_cycle": lanes, "clock_ghz": clk,
            "best_waves_per_simd": best.get("waves_per_simd"), "ubench_clock_ghz": best.get("clock_ghz"),
            "sources": ["profiles/" + cr_name, "profiles/" + pr_name]}


def _cgroup_cpu_quota():
    """CPUs' worth of the cgroup v2 CPU quota (cpu.max 'quota period'), or None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        return None


def cpu_threads(requested: int) -> dict:
    """Threads for the CPU baseline: the cores the job can actually use -- the CPUs this process
    may run on (sched_getaffinity), capped at the whole CPUs of the cgroup quota (cpu.max; the
    GPU box gives a job 16 of its 256 affinity CPUs, profiles/r05_box_cpu.txt).  Running one
    thread per affinity CPU past the quota only oversubscribes the share (r05: 23 K proofs/s on
    256 threads against 33 K on 16)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    quota = _cgroup_cpu_quota()
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    t = requested or usable
    return {"threads": max(1, t), "affinity_cpus": aff, "omp_num_threads": omp,
            "cgroup_cpu_quota": quota, "usable_cpus": usable}


def cpu_baseline(host_rows, seconds: float, threads: int):
    """Time the C oracle (reference-semantics per-proof verify, oracle/cpz_oracle.c) on a
    bounded sample of the same synthetic proofs.  Test/measurement infrastructure only."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle  # noqa: WPS433
    except Exception as exc:  # pragma: no cover - reported, not fatal
        return {"value": None, "error": "C oracle unavailable: %s" % exc}
    return coracle.time_verify(host_rows, seconds=seconds, threads=threads)


def _bump_s(torch, t, idx):
    """s := s + 1 (mod l) on the given rows (host round trip of those rows only)."""
    import numpy as np
    sel = torch.from_numpy(np.asarray(idx, dtype=np.int64)).to(t["s"].device)
    rows = t["s"].index_select(0, sel).cpu().numpy()
    for r in range(rows.shape[0]):
        v = (int.from_bytes(rows[r].tobytes(), "little") + 1) % L
        rows[r] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
    t["s"].index_copy_(0, sel, torch.from_numpy(rows).to(t["s"].device))


def rlc_roofline(stages, n, steps, oc):
    """Per-kernel fractions of the RLC step from the runtime's HIP-event stage times, each
    MAD-bound kernel priced on the headline's basis: the v_mad issue rate x 1024 SIMDs x that
    kernel's own shader clock (in-kernel probe, mad_peak_at_kernel_clock)."""
    r = oc.get("rlc", {})
    hbm = oc["peaks"]["hbm_bytes_per_s"]
    ms = {k: (v[0] / steps) for k, v in stages.items()}
    out = {"unit_mad": "Tmad/s", "unit_hbm": "GB/s", "peak_hbm": hbm / 1e9, "kernel_ms_per_step": ms}

    def priced(kernel, achieved):
        kc = mad_peak_at_kernel_clock(oc, kernel)
        if not kc:
            return {"achieved": achieved, "frac": None, "peak": None,
                    "peak_basis": "unpriced: no in-kernel clock probe of %s under profiles/" % kernel}
        pk = kc["peak"] / 1e12
        return {"achieved": achieved, "peak": pk, "frac": achieved / pk, "peak_clock_ghz": kc["clock_ghz"],
                "peak_basis": "v_mad_i64_i32 %.2f lanes / SIMD cycle x 1024 SIMDs x %s's own shader clock %.3f GHz "
                              "(in-kernel probe)" % (kc["lanes_per_simd_cycle"], kernel, kc["clock_ghz"]),
                "peak_sources": kc["sources"]}

    prep = r.get("prepare_per_proof", {}).get("mads")
    if prep and ms.get("rlc_prepare"):
        a = prep * n / (ms["rlc_prepare"] * 1e-3) / 1e12
        out["k_rlc_prepare"] = dict(bound="valu-int", mads_per_proof=prep, **priced("k_rlc_prepare", a))
    ent = r.get("bucket_entries_per_proof")
    bk = r.get("bucket_per_entry", {})
    if ent and ms.get("rlc_bucket"):
        t = ms["rlc_bucket"] * 1e-3
        a = bk["mads"] * ent * n / t / 1e12
        gbs = bk["bytes"] * ent * n / t / 1e9
        pmc = _profile("rlc_bucket_pmc")
        out["k_rlc_bucket"] = dict(bound="valu-int", mads_per_entry=bk["mads"], entries_per_proof=ent,
                                   **priced("k_rlc_bucket", a),
                                   algorithmic_bytes_per_entry=bk["bytes"], achieved_gbs=gbs,
                                   hbm_frac=gbs / (hbm / 1e9), traffic_bytes_per_2p20=pmc.get("hbm_bytes_per_2p20"),
                                   traffic_source=pmc.get("source"))
    tails = sum(ms.get(k, 0.0) for k in ("rlc_sort", "rlc_bucket_fix", "rlc_reduce", "rlc_final"))
    out["sort_plus_tails_ms"] = tails
    return out


def rlc_two_in_flight(cp, gpu, t, n, steps, device, first_index):
    """Service-style throughput of the batch check: two contexts on one GPU, each driven by its
    own host thread on its own stream (each context's stream has a hardware queue of its own),
    `steps` independent batch checks each.  One batch's latency-bound tails and memory-bound
    sort then run beside the other's VALU-bound prepare and buckets.  Every batch must pass."""
    import threading

    import torch
    gpus = [gpu, cp.Gpu(device)]
    status = [torch.empty(n, dtype=torch.uint8, device=t["s"].device) for _ in range(2)]
    bad = []

    def run(k, count):
        for _ in range(count):
            _, ok = gpus[k].verify_batch_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status[k], WEIGHT_SEED,
                                                first_index=first_index, stream=0)
            if not ok:
                bad.append(k)

    run(1, 2)  # the second context's tables and buffers
    torch.cuda.synchronize()
    th = [threading.Thread(target=run, args=(k, steps)) for k in range(2)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gpus[1].close()
    if bad or any(int((st != 0).sum().item()) for st in status):
        raise SystemExit("bench: a batch check in flight rejected a valid batch")
    return {"batches": 2 * steps, "proofs_per_s": 2 * n * steps / el, "ms_per_batch": el * 1e3 / (2 * steps),
            "how": "two contexts, two host threads, each context on its own stream / hardware queue "
                   "(tools/rlc_inflight.py); not the line's value"}


SMALL_SIZES = (1, 2, 5, 10, 20, 50, 100, 1000)


def _median_call_ms(fn, budget_s=0.25, min_calls=5, max_calls=200):
    """Median wall time of synchronous calls of fn (ms), after one untimed call."""
    fn()
    times = []
    stop = time.perf_counter() + budget_s
    while len(times) < min_calls or (time.perf_counter() < stop and len(times) < max_calls):
        t0 = time.perf_counter()
        fn()
        times.append((time.perf_counter() - t0) * 1e3)
    times.sort()
    return times[len(times) // 2], len(times)


def small_batch_table(gpu=None, sizes=SMALL_SIZES, stages=False, cpu=True):
    """The drop-in's own regime: one synchronous BatchVerifier-sized call from pageable host
    buffers per n (the reference bench's sizes, benches/batch_verification.rs:12-35, plus the
    cap 1000, batch.rs:48), median wall ms per call, through
      verify_each   cpz_verify_each (per-proof equations; what gpu.rs runs for n == 1)
      verify_batch  cpz_verify_batch with statuses (RLC + exact fallback; gpu.rs for n >= 2)
    beside the C oracle's BatchVerifier::verify on one thread (cpzo_reference_batch_verify: the
    reference's defective batch equation then per-entry verify_one, oracle/cpz_oracle.c).
    Valid proofs; a second verify_batch row has one forged entry (its fallback included)."""
    import numpy as np

    import chaum_pedersen as cp
    own = gpu is None
    gpu = gpu or cp.Gpu(0)
    nmax = max(sizes)
    rows = gpu.prove_synthetic(nmax, SEED_X, SEED_K)
    forged = {k: v.copy() for k, v in rows.items()}
    s0 = (int.from_bytes(forged["s"][0].tobytes(), "little") + 1) % L
    forged["s"][0] = np.frombuffer(s0.to_bytes(32, "little"), np.uint8)
    keys = ("y1", "y2", "r1", "r2", "s")
    out = {"sizes": list(sizes), "unit": "ms per call (median, synchronous, host buffers)", "rows": []}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle  # CPU baseline only (test infrastructure)
    for n in sizes:
        sub = [rows[k][:n] for k in keys]
        subf = [forged[k][:n] for k in keys]
        r = {"n": n}
        # equations-only per call, as the drop-in issues them (gpu.rs, cpz_batch.hpp)
        r["verify_each_ms"], _ = _median_call_ms(lambda: gpu.verify_each(*sub, equations_only=True))
        st = gpu.verify_each(*sub, equations_only=True)
        assert not st.any(), "small_batch: valid proofs rejected"
        r["verify_batch_ms"], _ = _median_call_ms(lambda: gpu.verify_batch(*sub, WEIGHT_SEED, equations_only=True))
        _, ok, st = gpu.verify_batch(*sub, WEIGHT_SEED, equations_only=True)
        assert ok and not st.any(), "small_batch: valid batch rejected"
        if n >= 2:
            r["verify_batch_one_forged_ms"], _ = _median_call_ms(
                lambda: gpu.verify_batch(*subf, WEIGHT_SEED, equations_only=True))
            _, ok, st = gpu.verify_batch(*subf, WEIGHT_SEED, equations_only=True)
            assert (not ok) and st[0] == 1 and not st[1:].any(), "small_batch: forged entry not located"
        if stages:
            gpu.set_timing(True)
            gpu.stage_times()
            gpu.verify_each(*sub)
            r["verify_each_stages"] = {k: v[0] for k, v in gpu.stage_times().items()}
            gpu.verify_batch(*sub, WEIGHT_SEED)
            r["verify_batch_stages"] = {k: v[0] for k, v in gpu.stage_times().items()}
            gpu.set_timing(False)
        if cpu:
            hr = {k: rows[k] for k in keys}
            r["cpu_batch_verifier_ms"], _ = _median_call_ms(lambda: coracle.reference_batch_verify(hr, 0, n),
                                                            budget_s=0.5, min_calls=3)
        best = min(("verify_each", r["verify_each_ms"]), ("verify_batch", r["verify_batch_ms"]), key=lambda x: x[1])
        r["faster_gpu_entry"] = best[0]
        if cpu:
            r["gpu_over_cpu_speedup"] = r["cpu_batch_verifier_ms"] / best[1]
        out["rows"].append(r)
    if cpu:
        out["cpu"] = {"cores": 1, "kind": "port", "what": "cpzo_reference_batch_verify (BatchVerifier::verify "
                      "semantics: defective equation + per-entry fallback, batch.rs:171-318), one thread"}
    if own:
        gpu.close()
    return out


PAIR_COUNTS = (1, 8, 64)


def custom_pairs_table(gpu, n=1000, counts=PAIR_COUNTS, cpu=True):
    """BatchVerifier batches whose entries carry their own Parameters (batch.rs:52,
    gadgets.rs:77-103): n entries spread over k distinct (g, h) pairs, verified through the
    drop-in's call sequence (the Python mirror of gpu.rs: one per-proof call per Parameters
    group, equations only).  A pair without cached combs is verified from its Niels tables
    (variable bases, stage 13) instead of building 128 MiB of combs per pair.  cold: a fresh
    context (every pair's tables built inside the call); warm: the same batch again (tables
    cached, a service reusing its pairs).  CPU: the C oracle's BatchVerifier::verify per group
    under that group's generators, one thread."""
    import hashlib

    import numpy as np

    import chaum_pedersen as cp
    out = {"n": n, "unit": "ms per BatchVerifier::verify (median of synchronous calls)", "rows": []}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle  # CPU baseline only (test infrastructure)
    base = gpu.prove_synthetic(n, SEED_X, SEED_K)   # x, k: reuse the synthetic witnesses per pair below
    for k in counts:
        pairs = []
        for j in range(k):
            # [a] B, [b] B as encodings: prove with x = a gives y1 = [a] g (default g = B)
            a = hashlib.sha512(b"bench-pair-g-%d" % j).digest()[:31] + b"\0"
            b2 = hashlib.sha512(b"bench-pair-h-%d" % j).digest()[:31] + b"\0"
            o = gpu.prove([a, b2], [a, b2])
            pairs.append(cp.Parameters(o["y1"][0].tobytes(), o["y1"][1].tobytes()))
        groups = np.arange(n) % k
        rows = {q: np.zeros((n, 32), np.uint8) for q in ("y1", "y2", "r1", "r2", "s")}
        for j in range(k):
            idx = np.nonzero(groups == j)[0]
            xs = [hashlib.sha256(b"bx%d" % i).digest() for i in idx]
            ks = [hashlib.sha256(b"bk%d" % i).digest() for i in idx]
            o = gpu.prove(xs, ks, params=pairs[j])
            for q in rows:
                rows[q][idx] = o[q]
        fresh = cp.Gpu(gpu.device if hasattr(gpu, "device") else 0)
        b = cp.BatchVerifier(fresh)
        for i in range(n):
            b.add(pairs[int(groups[i])], cp.Statement(rows["y1"][i].tobytes(), rows["y2"][i].tobytes()),
                  cp.Proof(rows["r1"][i].tobytes(), rows["r2"][i].tobytes(), rows["s"][i].tobytes()))
        fresh.set_timing(True)
        fresh.stage_times()
        t0 = time.perf_counter()
        res = b.verify()
        cold = (time.perf_counter() - t0) * 1e3
        st = fresh.stage_times()
        fresh.set_timing(False)
        if any(not r.is_ok() for r in res):
            raise SystemExit("bench: custom-pair batch rejected a valid proof")
        warm, calls = _median_call_ms(lambda: b.verify(), budget_s=0.5, min_calls=3)
        r = {"pairs": k, "cold_ms": cold, "warm_ms": warm, "calls": calls,
             "varbase_table_builds": st.get("generators_varbase", (0.0, 0))[1],
             "comb_builds": st.get("generators", (0.0, 0))[1],
             "varbase_build_ms": st.get("generators_varbase", (0.0, 0))[0]}
        fresh.close()
        if cpu:
            def cpu_run():
                for j in range(k):
                    idx = np.nonzero(groups == j)[0]
                    sub = {q: np.ascontiguousarray(rows[q][idx]) for q in rows}
                    coracle.reference_batch_verify(sub, 0, len(idx), g=pairs[j].g, h=pairs[j].h)
            r["cpu_batch_verifier_ms"], _ = _median_call_ms(cpu_run, budget_s=0.5, min_calls=2)
            r["gpu_over_cpu_speedup_cold"] = r["cpu_batch_verifier_ms"] / cold
            r["gpu_over_cpu_speedup_warm"] = r["cpu_batch_verifier_ms"] / warm
        out["rows"].append(r)
    return out


def c5_roofline(ms, n5, oc):
    """configs[4]'s dominant kernels on the headline's basis: k_part_acc (every 128-proof
    block's bucket walk, stage 14) by its algorithmic MADs per block -- entries x 7 M + bucket
    boundaries x 9 M (bench/opcount.json "part": host-counted step costs, entries simulated by
    tools/part_entries.py) -- and k_rlc_prepare by its MADs per proof, each against the v_mad
    issue rate x 1024 SIMDs x that kernel's own probed shader clock."""
    part = oc.get("part", {})
    out = {"unit": "Tmad/s"}

    def priced(kernel, achieved, **extra):
        kc = mad_peak_at_kernel_clock(oc, kernel)
        r = dict(extra, achieved=achieved)
        if kc:
            pk = kc["peak"] / 1e12
            r.update(peak=pk, frac=achieved / pk, peak_clock_ghz=kc["clock_ghz"], peak_sources=kc["sources"],
                     peak_basis="v_mad_i64_i32 %.2f lanes / SIMD cycle x 1024 SIMDs x %s's own shader clock %.3f GHz"
                                % (kc["lanes_per_simd_cycle"], kernel, kc["clock_ghz"]))
        else:
            r.update(peak=None, frac=None, peak_basis="unpriced: no in-kernel clock probe of %s under profiles/" % kernel)
        return r

    blocks = (n5 + 127) // 128
    t = ms.get("part_acc")
    if t and part:
        a = part["algorithmic_mads_per_block"] * blocks / (t * 1e-3) / 1e12
        out["k_part_acc"] = priced(
            "k_part_acc", a, blocks=blocks, kernel_ms=t, algorithmic_mads_per_block=part["algorithmic_mads_per_block"],
            executed_mads_per_block=part["executed_mads_per_block"],
            executed_tmad_s=part["executed_mads_per_block"] * blocks / (t * 1e-3) / 1e12,
            non_algorithmic_share=part["non_algorithmic_share"],
            basis="%d entries x 7 M + %d boundaries x 9 M per block (the kernel executes 9 M per step)"
                  % (part["entries_per_block"], part["boundaries_per_block"]))
    prep = oc.get("rlc", {}).get("prepare_per_proof", {}).get("mads")
    t = ms.get("rlc_prepare")
    if t and prep:
        out["k_rlc_prepare"] = priced("k_rlc_prepare", prep * n5 / (t * 1e-3) / 1e12, kernel_ms=t, mads_per_proof=prep)
    if ms.get("part_acc_locate"):
        out["k_part_acc_locate_ms"] = ms["part_acc_locate"]
    return out


def c5_extra(gpu, torch, dev, stream, n5, ctx_len):
    """configs[4]: n5 proofs, 0.1 % forged, through the batch check + fallback -> the exact
    invalid set, timed against cpz_verify_each of the same batch.  ctx_len = 32: every proof
    carries a 32-byte transcript context (the service's challenge ids, service.rs:512-517) and
    half the forgeries are a replayed context instead of a wrong y1."""
    import numpy as np
    nf = max(1, n5 // 1000)
    t5 = {k: torch.empty((n5, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    cx = {}
    if ctx_len:
        gen = torch.Generator(device=dev)
        gen.manual_seed(555)
        cx["ctx_bytes"] = torch.randint(0, 256, (n5 * ctx_len,), dtype=torch.int32, device=dev,
                                        generator=gen).to(torch.uint8)
        cx["ctx_off"] = torch.arange(n5 + 1, dtype=torch.int64, device=dev) * ctx_len
    gpu.prove_synthetic_device(n5, SEED_X, SEED_K, t5["y1"], t5["y2"], t5["r1"], t5["r2"], t5["s"], stream=stream, **cx)
    idx = np.sort(np.random.default_rng(2024).choice(n5, size=nf, replace=False))
    bump, swap = idx[0::2], idx[1::2]
    _bump_s(torch, t5, bump)
    dst = torch.from_numpy(swap.astype(np.int64)).to(dev)
    if ctx_len:   # the proof presented under another entry's context (a replayed challenge id)
        cv = cx["ctx_bytes"].view(n5, ctx_len)
        cv.index_copy_(0, dst, cv.index_select(0, (dst + 1) % n5).clone())
    else:
        src = torch.from_numpy(((swap + 7) % n5).astype(np.int64)).to(dev)
        t5["y1"].index_copy_(0, dst, t5["y1"].index_select(0, src).clone())
    rows = [t5[k] for k in ("y1", "y2", "r1", "r2", "s")]
    st5 = torch.empty(n5, dtype=torch.uint8, device=dev)
    gpu.verify_batch_device(*rows, st5, WEIGHT_SEED, fallback=True, stream=stream, **cx)  # warm-up (allocations)
    st5.fill_(0xFF)
    gpu.set_timing(True)
    gpu.stage_times()
    torch.cuda.synchronize(dev)
    c0 = time.perf_counter()
    partial, ok = gpu.verify_batch_device(*rows, st5, WEIGHT_SEED, fallback=True, stream=stream, **cx)
    torch.cuda.synchronize(dev)
    c_el = time.perf_counter() - c0
    c_st = gpu.stage_times()
    c_fb = gpu.fallback_stats()
    got = st5.cpu().numpy()
    exact = (not ok) and np.array_equal(np.nonzero(got)[0], idx) and set(got[idx].tolist()) == {1}
    if not exact:
        raise SystemExit("bench: C5 fallback did not return exactly the forged set")
    st5.fill_(0xFF)
    torch.cuda.synchronize(dev)
    p0 = time.perf_counter()
    gpu.verify_each_device(*rows, st5, stream=stream, **cx)
    torch.cuda.synchronize(dev)
    p_el = time.perf_counter() - p0
    gpu.set_timing(False)
    pp = st5.cpu().numpy()
    if not np.array_equal(pp, got):
        raise SystemExit("bench: C5 per-proof statuses differ from the fallback's")
    ms = {k: v[0] for k, v in c_st.items()}
    roof = c5_roofline(ms, n5, oc=_load_json("bench/opcount.json") or {})
    out = {"workload": "configs[4]: %d proofs%s, %d forged (half s+1, half %s), RLC batch check + fallback "
                       "(density probe beside the challenges; at this density the partitioned check: every "
                       "128-proof block's RLC partial, the failing blocks' index-weighted partials locating a "
                       "single forgery, per-proof verification of the located entries and of the blocks holding "
                       "more) -> exact invalid set" % (n5, (" with %d-byte contexts" % ctx_len) if ctx_len else "", nf,
                                              "a replayed context" if ctx_len else "wrong y1"),
           "proofs": n5, "forged": nf, "ms": c_el * 1e3, "proofs_per_s": n5 / c_el, "exact_set": True,
           "phase_ms": {"challenge": ms.get("challenge", 0.0), "rlc_prepare": ms.get("rlc_prepare", 0.0),
                        "rlc_msm": ms.get("rlc_msm", 0.0), "part_acc": ms.get("part_acc", 0.0),
                        "part_acc_locate": ms.get("part_acc_locate", 0.0),
                        "fallback_per_proof": ms.get("fallback", 0.0)},
           "fallback": c_fb,
           "roofline": roof,
           "per_proof_only_ms": p_el * 1e3,
           "ratio_to_per_proof": c_el / p_el,
           "partial": partial.hex(),
           "note": "per_proof_only_ms: cpz_verify_each of the same batch (same statuses); rlc_msm is the "
                   "partitioned MSMs (k_part_*: every block's partial, then the failing blocks' index-weighted "
                   "partials and the locate step), fallback_per_proof the per-proof pass"}
    del t5, st5, cx
    torch.cuda.empty_cache()
    return out


def c4_forged_indices(n_total: int):
    """Global indices forged (s + 1) in configs[3]'s forged variant: two pairs, one pair in the
    second eighth of the index space and one in the sixth, so at 2, 4 and 8 ranks they land in
    exactly two ranks' shards (ranks 0 / 1, 0 / 2, 1 / 5), and at N = 1 all in rank 0's."""
    e = n_total // 8
    return sorted({e + 5, e + 4099, 5 * e + 101, 5 * e + 77777} if e > 77777 else
                  {e + 5, e + 9, 5 * e + 1, 5 * e + 3})


def c4_run(gpu, torch, dist, dev, stream, world, rank, n_total, steps, warmup, backend):
    """configs[3] at this world size: n_total proofs split over the ranks (contiguous shards,
    shard_range), each rank reducing its shard to one 32-byte RLC partial whose weights are
    keyed by the GLOBAL index (cpz_verify_batch_device, first_index = shard start), an
    all-gather of the partials (RCCL over xGMI with the "nccl" backend) and cpz_combine_partials
    on every rank.  One step = the whole exchange; barrier + synchronize on both sides of the
    timed steps, max over ranks.  A valid set must combine to the identity.  Then the forged
    variant: s + 1 at c4_forged_indices, the batch check with fallback -- every rank's statuses
    must be exactly its own forged entries (status 1) and the combined total must not be the
    identity.  This replaces the reference's sequential loops (batch.rs:239-260, 279-309)."""
    import numpy as np

    from chaum_pedersen.shard import all_gather_partials, shard_range
    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    t4 = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    rows = [t4[k] for k in ("y1", "y2", "r1", "r2", "s")]
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    gpu.prove_synthetic_device(n, SEED_X, SEED_K, *rows, first_index=lo, stream=stream)
    torch.cuda.synchronize(dev)
    state = {}

    def step(fallback=False):
        partial, ok = gpu.verify_batch_device(*rows, st, WEIGHT_SEED, first_index=lo, fallback=fallback,
                                              stream=stream)
        parts = all_gather_partials(partial) if world > 1 else [partial]
        total, ident = gpu.combine_partials(parts)
        state.update(partial=partial, ok=ok, parts=parts, total=total, ident=ident)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(warmup):
        step()
    st.fill_(0xFF)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    el = time.perf_counter() - t0
    local_el = el
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    valid_ok = bool(state["ident"] and state["total"] == bytes(32) and state["ok"]
                    and not int((st != 0).sum().item()))
    clean = {"total": state["total"].hex(), "identity": bool(state["ident"])}

    # forged variant: s + 1 on the forged entries of this shard, batch check + fallback
    forged = c4_forged_indices(n_total)
    mine = [i - lo for i in forged if lo <= i < hi]
    if mine:
        _bump_s(torch, t4, mine)
    st.fill_(0xFF)
    barrier()
    torch.cuda.synchronize(dev)
    f0 = time.perf_counter()
    step(fallback=True)
    torch.cuda.synchronize(dev)
    barrier()
    f_el = time.perf_counter() - f0
    fb = gpu.fallback_stats()
    got = st.cpu().numpy()
    bad = np.nonzero(got)[0]
    exact_local = bool(np.array_equal(bad, np.asarray(mine, dtype=bad.dtype)) and (got[bad] == 1).all())
    forged_ok = bool((not state["ident"]) and state["total"] != bytes(32) and state["ok"] == (not mine))
    checks = torch.tensor([int(valid_ok), int(exact_local), int(forged_ok), len(mine)], dtype=torch.int64,
                          device=dev if backend == "nccl" else "cpu")
    if world > 1:
        gathered = [torch.empty_like(checks) for _ in range(world)]
        dist.all_gather(gathered, checks)
        per_rank = [g.cpu().tolist() for g in gathered]
    else:
        per_rank = [checks.cpu().tolist()]
    del t4, rows, st
    torch.cuda.empty_cache()
    out = {"workload": "configs[3]: %d proofs split over %d GPU%s (contiguous shards), per-rank RLC partial keyed "
                       "by the global index, all-gather of the 32-B partials (%s), combine on every rank"
                       % (n_total, world, "s" if world > 1 else "", backend if world > 1 else "world of one"),
           "proofs_total": n_total, "proofs_per_gpu_max": max(shard_range(n_total, world, r)[1] -
                                                                shard_range(n_total, world, r)[0]
                                                                for r in range(world)),
           "steps": steps, "warmup": warmup, "ms_per_step": el * 1e3 / steps,
           "proofs_per_s": n_total * steps / el, "scaling": "strong",
           "identity": valid_ok and all(r[0] for r in per_rank),
           "combined_total_valid": clean["total"],
           "forged": {"indices": forged, "per_rank_forged": [r[3] for r in per_rank],
                      "statuses_exact_every_rank": all(r[1] for r in per_rank),
                      "combined_total_not_identity": all(r[2] for r in per_rank),
                      "combined_total": state["total"].hex(), "ms": f_el * 1e3,
                      "rank0_fallback": fb,
                      "how": "s + 1 at the forged global indices; cpz_verify_batch_device with fallback on every "
                             "rank, all-gather, combine"},
           "local_ms_per_step_rank0": local_el * 1e3 / steps}
    out["ok"] = bool(out["identity"] and out["forged"]["statuses_exact_every_rank"]
                     and out["forged"]["combined_total_not_identity"])
    return out


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n: int) -> int:
    """Run this same command as n ranks under torch.distributed.run (one process per GPU,
    rendezvous on 127.0.0.1) in a child process and return its exit code.  Only rank 0 prints
    the JSON line; the children's stdout/stderr are inherited, so the line reaches our stdout
    unchanged.  The parent imports neither torch nor HIP: the GPU is touched only by the
    ranks."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        rc = subprocess.run(cmd, env=env).returncode
    except KeyboardInterrupt:
        return 130
    return 128 - rc if rc < 0 else rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1 << 20, help="proofs per GPU (weak scaling)")
    ap.add_argument("--n-total", type=int, default=0,
                    help="proofs of the whole job, split over the ranks (strong scaling; configs[3] = 67108864)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: the usable cores, min(affinity CPUs, cgroup quota))")
    ap.add_argument("--cpu-oversubscribed", type=int, default=0,
                    help="also time one thread per affinity CPU past the quota (reported as a note only)")
    ap.add_argument("--c4-n", type=int, default=1 << 26,
                    help="configs[3]: proofs of the whole job split over the ranks, per-rank RLC partial + "
                         "all-gather + combine, measured at every N (0: skip)")
    ap.add_argument("--c4-steps", type=int, default=None, help="timed configs[3] steps (default: --steps)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=("each", "rlc"), default="each",
                    help="each: per-proof verification (configs[1], the headline); rlc: random-linear-"
                         "combination batch check via Pippenger MSM (configs[2]/[3]: per-rank partials, "
                         "all-gather of 32-B partials, combine)")
    ap.add_argument("--ctx-len", type=int, default=0,
                    help="per-proof transcript context of this many random bytes (0: none, the configs' default; "
                         "32: the reference service's challenge ids, service.rs:294-295)")
    ap.add_argument("--extras", type=int, default=1,
                    help="at N=1 in 'each' mode also measure the RLC check, C5, the prover and the host path")
    ap.add_argument("--rlc-extra", type=int, default=None, help="override --extras for the RLC extra")
    ap.add_argument("--rlc-inflight", type=int, default=1,
                    help="add the two-batches-in-flight figure to the RLC extra (0: one batch at a time only, "
                         "e.g. under a profiler whose per-kernel averages should not mix the two)")
    ap.add_argument("--host-e2e", type=int, default=None, help="override --extras for the host-buffer extra")
    ap.add_argument("--small-batch", type=int, default=None,
                    help="override --extras for the small-batch latency table (the drop-in's n <= 1000 regime)")
    ap.add_argument("--c5-n", type=int, default=1 << 24, help="configs[4] batch size (0.1 %% forged)")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N > 1 ('nccl' = RCCL over xGMI; 'gloo' only for rehearsals)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 (with --backend gloo); not a measurement")
    args = ap.parse_args()
    extra = lambda v: args.extras if v is None else v

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: start one rank per GPU as a CHILD process
        # group (torch.distributed.run), before anything here imports torch or touches HIP,
        # relay its output and exit with its code.  Never exec.
        sys.exit(_launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit("bench: --gpus %d but WORLD_SIZE=%s; refusing to report a line for the wrong N"
                 % (args.gpus, env_world))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    if args.same_device:
        local_rank = 0
    else:
        # one rank per GPU: refuse before any collective is set up when the node shows fewer
        # devices than ranks (device_count does not initialise HIP on this image)
        ndev = torch.cuda.device_count()
        if ndev < world or local_rank >= ndev:
            sys.exit("bench: %d rank(s) (LOCAL_RANK %d) but %d visible GPU(s); one process per GPU is required "
                     "(--same-device only for rehearsals)" % (world, local_rank, ndev))
    torch.cuda.set_device(local_rank)  # before the process group, so RCCL binds each rank to its own GPU
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group(args.backend, init_method="env://")

    import chaum_pedersen as cp
    from chaum_pedersen.shard import all_gather_partials, shard_range

    gpu = cp.Gpu(local_rank)
    if args.n_total:
        lo, hi = shard_range(args.n_total, world, rank)
        scaling = "strong"
    else:
        lo, hi = rank * args.n, (rank + 1) * args.n
        scaling = "weak"
    n = hi - lo
    total_proofs = args.n_total if args.n_total else world * args.n
    t = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("y1", "y2", "r1", "r2", "s")}
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    cx = {}
    if args.ctx_len:
        gen = torch.Generator(device=dev)
        gen.manual_seed(1000 + rank)
        cx["ctx_bytes"] = torch.randint(0, 256, (n * args.ctx_len,), dtype=torch.int32, device=dev,
                                        generator=gen).to(torch.uint8)
        cx["ctx_off"] = torch.arange(n + 1, dtype=torch.int64, device=dev) * args.ctx_len
    gpu.prove_synthetic_device(n, SEED_X, SEED_K, t["y1"], t["y2"], t["r1"], t["r2"], t["s"], first_index=lo,
                               stream=stream, **cx)
    torch.cuda.synchronize(dev)

    def step_each():
        gpu.verify_each_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status, stream=stream, **cx)

    rlc_state = {"ok": True, "total": None}

    def step_rlc():
        partial, ok = gpu.verify_batch_device(t["y1"], t["y2"], t["r1"], t["r2"], t["s"], status, WEIGHT_SEED,
                                              first_index=lo, stream=stream, **cx)
        if world > 1:
            parts = all_gather_partials(partial)
            total, ident = gpu.combine_partials(parts)
            ok = ok and ident and total == bytes(32)
            rlc_state["total"] = total.hex()
        rlc_state["ok"] = rlc_state["ok"] and ok

    step = step_each if args.mode == "each" else step_rlc

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    n_bad = int((status != 0).sum().item())
    if n_bad or not rlc_state["ok"]:
        raise SystemExit("bench: %d of %d valid synthetic proofs rejected -- refusing to report" % (n_bad, n))

    status.fill_(0xFF)  # the timed steps must write every entry (checked below)
    gpu.set_timing(True)
    gpu.stage_times()  # reset
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = gpu.stage_times()
    gpu.set_timing(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    n_bad = int((status != 0).sum().item())
    if n_bad or not rlc_state["ok"]:
        raise SystemExit("bench: %d proofs rejected (or not written) in the timed region" % n_bad)

    oc = _load_json("bench/opcount.json") or {}
    peak_mad = oc.get("peaks", {}).get("v_mad_i64_i32_lane_ops_per_s", 28.32e12)
    solo = world == 1

    # -- configs[3] at this N (every rank; N = 1 included) ---------------------------------
    c4 = None
    if args.c4_n:
        c4 = c4_run(gpu, torch, dist, dev, stream, world, rank, args.c4_n,
                    args.c4_steps if args.c4_steps is not None else args.steps, 1, args.backend)
        if not c4["ok"]:
            raise SystemExit("bench: configs[3] check failed: %s" % json.dumps(c4))

    # -- extras at N = 1 ------------------------------------------------------------------
    rlc_extra = None
    if args.mode == "each" and solo and extra(args.rlc_extra):
        for _ in range(2):
            step_rlc()
        status.fill_(0xFF)
        gpu.set_timing(True)
        gpu.stage_times()
        torch.cuda.synchronize(dev)
        r0 = time.perf_counter()
        for _ in range(args.steps):
            step_rlc()
        torch.cuda.synchronize(dev)
        r_el = time.perf_counter() - r0
        r_st = gpu.stage_times()
        gpu.set_timing(False)
        if not rlc_state["ok"] or int((status != 0).sum().item()):
            raise SystemExit("bench: RLC batch check rejected a valid batch")
        rlc_extra = {"workload": "configs[2]: RLC batch check of the same 2^20 proofs (Pippenger, 16-bit windows)",
                     "proofs_per_s": n * args.steps / r_el, "ms_per_step": r_el * 1e3 / args.steps,
                     "roofline": rlc_roofline(r_st, n, args.steps, oc),
                     "two_in_flight": (rlc_two_in_flight(cp, gpu, t, n, args.steps, local_rank, lo)
                                       if args.rlc_inflight else None)}

    c5 = c5_ctx = None
    if args.mode == "each" and solo and args.extras and args.c5_n:
        c5 = c5_extra(gpu, torch, dev, stream, args.c5_n, 0)
        c5_ctx = c5_extra(gpu, torch, dev, stream, args.c5_n, 32)

    prove = None
    if args.mode == "each" and solo and args.extras:
        gen = torch.Generator(device=dev)
        gen.manual_seed(77)
        xk = [torch.randint(0, 256, (n, 32), dtype=torch.int32, device=dev, generator=gen).to(torch.uint8)
              for _ in range(2)]
        outs = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in t}
        gpu.prove_device(xk[0], xk[1], *(outs[k] for k in ("y1", "y2", "r1", "r2", "s")), stream=stream)
        torch.cuda.synchronize(dev)
        psteps = max(1, min(args.steps, 5))
        q0 = time.perf_counter()
        for _ in range(psteps):
            gpu.prove_device(xk[0], xk[1], *(outs[k] for k in ("y1", "y2", "r1", "r2", "s")), stream=stream)
        torch.cuda.synchronize(dev)
        q_el = time.perf_counter() - q0
        status.fill_(0xFF)
        gpu.verify_each_device(*(outs[k] for k in ("y1", "y2", "r1", "r2", "s")), status, stream=stream)
        torch.cuda.synchronize(dev)
        if int((status != 0).sum().item()):
            raise SystemExit("bench: generated proofs do not verify")
        rate = n * psteps / q_el
        prove = {"workload": "cpz_prove_device: %d proofs from random caller witnesses / nonces (prover/mod.rs:86-131)"
                             % n, "proofs_per_s": rate, "us_per_proof": 1e6 / rate,
                 "published_us_per_proof": 144.0, "published_source": "src/lib.rs:55 (M-series Mac, one core)",
                 "all_verified": True}
        del outs, xk

    host_e2e = None
    if args.mode == "each" and solo and extra(args.host_e2e):
        hrows = {k: t[k].cpu().numpy() for k in t}
        hst = gpu.verify_each(hrows["y1"], hrows["y2"], hrows["r1"], hrows["r2"], hrows["s"])
        steps_h = max(1, min(args.steps, 5))
        h0 = time.perf_counter()
        for _ in range(steps_h):
            hst = gpu.verify_each(hrows["y1"], hrows["y2"], hrows["r1"], hrows["r2"], hrows["s"])
        h_el = time.perf_counter() - h0
        if int((hst != 0).sum()):
            raise SystemExit("bench: host-buffer path rejected valid proofs")
        host_e2e = {"workload": "cpz_verify_each from pageable host arrays (H2D of 5 x 32 B/proof + D2H of statuses)",
                    "proofs_per_s": n * steps_h / h_el, "ms_per_call": h_el * 1e3 / steps_h, "calls": steps_h}
        del hrows

    small = pairs_tab = None
    if args.mode == "each" and solo and extra(args.small_batch):
        small = small_batch_table(gpu, cpu=not args.no_cpu_baseline)
        pairs_tab = custom_pairs_table(gpu, cpu=not args.no_cpu_baseline)

    value = total_proofs * args.steps / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    mads = oc.get("verify_each", {}).get("mads_per_proof", 342380)
    v_ms, v_cnt = stages.get("verify_each", (0.0, 0))
    c_ms, c_cnt = stages.get("challenge", (0.0, 0))
    # The runtime cuts a batch into launches of half the occupancy grid (2^16 proofs) on two
    # streams, so two launches are always in flight and their durations overlap: achieved =
    # algorithmic MADs of the step's verify work / the verify span (first launch start to last
    # launch end, HIP events on the launch stream).
    per_launch = (n * args.steps / v_cnt) if v_cnt else None
    sp_ms, sp_cnt = stages.get("verify_span", (0.0, 0))
    span_s = (sp_ms / args.steps) * 1e-3 if sp_cnt else None
    pmc = _profile("verify_each_pmc")
    if args.mode == "each":
        achieved = (mads * n / span_s) / 1e12 if span_s else None
        kc = mad_peak_at_kernel_clock(oc)
        peak_k = kc["peak"] if kc else peak_mad
        roofline = {
            "kernel": "k_verify_each",
            "bound": "valu-int",
            "achieved": achieved,
            "peak": peak_k / 1e12,
            "unit": "Tmad/s",
            "frac": (achieved / (peak_k / 1e12)) if achieved else None,
            "peak_clock_ghz": kc["clock_ghz"] if kc else None,
            "peak_basis": ("v_mad_i64_i32 issue rate %.2f lanes / SIMD cycle (best of the clock_rates sweep, %s "
                           "waves/SIMD) x 1024 SIMDs x the kernel's own shader clock %.3f GHz (in-kernel probe)"
                           % (kc["lanes_per_simd_cycle"], kc["best_waves_per_simd"], kc["clock_ghz"])) if kc else
                          "v_mad_i64_i32 rate measured by the clock_rates sweep",
            "peak_sources": kc["sources"] if kc else None,
            "peak_at_ubench_clock": peak_mad / 1e12,
            "frac_vs_peak_at_ubench_clock": (achieved / (peak_mad / 1e12)) if achieved else None,
            "traffic": pmc.get("hbm_bytes_per_launch"),
            "traffic_per_proof": pmc.get("hbm_bytes_per_proof"),
            "traffic_source": pmc.get("source"),
            "peak_source": oc.get("peaks", {}).get("source"),
            "frac_vs_2p4ghz_spec": (achieved / (oc["peaks"]["v_mad_spec_lane_ops_per_s_at_2p4ghz"] / 1e12))
            if achieved and "v_mad_spec_lane_ops_per_s_at_2p4ghz" in oc.get("peaks", {}) else None,
            "algorithmic_mads_per_proof": mads,
            "kernel_ms": v_ms / v_cnt if v_cnt else None,
            "proofs_per_launch": per_launch,
            "launches_in_flight": 2,
            "verify_span_ms_per_step": sp_ms / args.steps if sp_cnt else None,
            "span_covers": "all k_verify_each launches of a step and the per-chunk challenge launches between them",
            "challenge_kernel_ms": c_ms / c_cnt if c_cnt else None,
            "hbm_frac": ((194 * n / span_s) / 8.0e12) if span_s else None,
        }
    else:
        rr = rlc_roofline(stages, n, args.steps, oc)
        pk = rr.get("k_rlc_prepare", {})
        roofline = {"kernel": "k_rlc_prepare (the RLC step's largest kernel; k_rlc_bucket below)",
                    "bound": "valu-int", "achieved": pk.get("achieved"), "peak": pk.get("peak"), "unit": "Tmad/s",
                    "frac": pk.get("frac"), "peak_clock_ghz": pk.get("peak_clock_ghz"),
                    "peak_basis": pk.get("peak_basis"), "traffic": None, "rlc": rr}

    cpu = None
    if rank == 0 and solo and not args.no_cpu_baseline:
        th = cpu_threads(args.cpu_threads)
        sample = 1 << 14
        rows = {k: t[k][:sample].cpu().numpy() for k in t}
        cpu = cpu_baseline(rows, args.cpu_seconds, th["threads"])
        if cpu:
            cpu["affinity_cpus"] = th["affinity_cpus"]
            cpu["omp_num_threads"] = th["omp_num_threads"]
            cpu["cgroup_cpu_quota"] = th["cgroup_cpu_quota"]
            cpu["cores_basis"] = ("min(affinity CPUs %d, whole CPUs of the cgroup quota %s) = %d threads, one per "
                                  "usable core" % (th["affinity_cpus"], th["cgroup_cpu_quota"], th["usable_cpus"])
                                  if not args.cpu_threads else "--cpu-threads %d" % args.cpu_threads)
            if cpu.get("value") and th["affinity_cpus"] > th["threads"] and args.cpu_oversubscribed:
                # note only: one thread per affinity CPU, past the quota (r05's mislabelled figure)
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                import coracle  # CPU baseline only (test infrastructure)
                sub = coracle.time_verify(rows, seconds=max(2.0, args.cpu_seconds / 4), threads=th["affinity_cpus"])
                cpu["note_oversubscribed"] = {"threads": th["affinity_cpus"], "value": sub.get("value"),
                                              "what": "one thread per affinity CPU, past the cgroup quota: "
                                                      "a note, not the baseline"}

    if rank == 0:
        if args.mode == "each":
            workload = ("configs[1]: per-proof verification (challenge + 2 equations), %d proofs per GPU" % n
                        if scaling == "weak" else
                        "per-proof verification of %d proofs split over %d GPUs" % (total_proofs, world))
        else:
            workload = ("configs[2]/[3]: RLC batch check via Pippenger MSM, %d proofs %s, per-rank 32-B partial + "
                        "all-gather + combine" % (total_proofs if scaling == "strong" else n,
                                                  "split over the GPUs" if scaling == "strong" else "per GPU"))
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "proofs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "int32/int64 limbs (GF(2^255-19), radix 2^25.5)",
            "data": "synthetic (GPU prover, ChaCha20-derived witnesses; all proofs valid, checked)",
            "config": {"workload": workload,
                       "proofs_total": total_proofs,
                       "proofs_per_gpu": n,
                       "contexts": ("%d random bytes per proof" % args.ctx_len) if args.ctx_len else "none",
                       "generators": "default (g, h)",
                       "parallelism": "dp%d (contiguous shards%s)" % (
                           world, ", no collective" if args.mode == "each" else ", all-gather of 32-B partials")},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if c4:
            if args.same_device:   # ranks sharing one GPU: correctness only, no rate
                c4.update(proofs_per_s=None, ms_per_step=None, local_ms_per_step_rank0=None)
                c4["forged"]["ms"] = None
            line["c4"] = c4
        if rlc_extra:
            line["rlc"] = rlc_extra
        if c5:
            line["c5"] = c5
        if c5_ctx:
            line["c5_ctx"] = c5_ctx
        if prove:
            line["prove"] = prove
        if host_e2e:
            line["host_e2e"] = host_e2e
        if small:
            line["small_batch"] = small
        if pairs_tab:
            line["custom_pairs"] = pairs_tab
        if args.same_device:
            # several ranks on one GPU: a correctness rehearsal of the multi-rank path, not a
            # measurement -- no rate is reported
            line["value"] = None
            line["ms_per_step"] = None
            line["roofline"] = None
            line["rehearsal"] = {"ranks_on_one_gpu": world, "backend": args.backend,
                                 "combined_total": rlc_state["total"],
                                 "combined_total_identity": rlc_state["total"] == bytes(32).hex() if world > 1 else None,
                                 "all_statuses_valid": True}
        print(json.dumps(line), flush=True)
    gpu.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
