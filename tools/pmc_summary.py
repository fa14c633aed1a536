#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/profile.sh into profiles/<round>_*.json / .csv.

  python tools/pmc_summary.py r01 [gpurun_out]

Per kernel: average duration (kernel trace), FETCH_SIZE / WRITE_SIZE (kB per launch, one
counter per pass; FETCH doubled per MI355X_MICROARCH.md's gfx950 correction for wide
coalesced reads) and the SQ counters.  k_verify_each also gets its per-proof figures
(2^16 proofs per launch in the bench workload: the runtime cuts 2^20 into 16 launches of
half the occupancy grid, two in flight on two streams).
"""
import csv
import collections
import json
import os
import shutil
import sys

rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("cpz::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def mean(v):
    return sum(v) / len(v)


out = {}
for tag in ("prof_fetch", "prof_write", "prof_sq", "prof_l2"):
    for k, d in counters(os.path.join(src, tag, "run_counter_collection.csv")).items():
        if not k.startswith("k_"):
            continue
        for c, v in d.items():
            out.setdefault(k, {})[c] = mean(v)
stats = os.path.join(src, "prof_trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(prof, "%s_kernel_stats.csv" % rnd))
    for r in csv.DictReader(open(stats)):
        k = r["Name"].split("(")[0].replace("cpz::", "")
        if k in out or k.startswith("k_"):
            out.setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            out[k]["calls"] = int(r["Calls"])
for k, d in out.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes_per_launch"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
        d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in d and d.get("avg_ns"):
        # MI355X_MICROARCH.md DVFS: effective clock ~ GRBM_GUI_ACTIVE / 8 XCDs / wall time
        d["effective_clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8.0 / d["avg_ns"]
ve = out.get("k_verify_each", {})
if ve:
    n = int(os.environ.get("PROOFS_PER_LAUNCH", 1 << 16))
    if "SQ_INSTS_VALU" in ve:
        ve["valu_instructions_per_proof"] = ve["SQ_INSTS_VALU"] * 64 / n
    ve["workload"] = ("%d proofs per launch (bench.py default 2^20 per step = 16 launches), rocprofv3 --pmc, "
                      "one counter group per pass" % n)
    ve["correction"] = ("gfx950: FETCH_SIZE reports 64 B per 128-B L2 line miss, for coalesced streams and "
                        "random 128/160-B gathers alike (MI355X_MICROARCH.md HBM; profiles/r02_gather_calibration.json) "
                        "-> doubled; WRITE_SIZE as reported; units kB")
    ve["algorithmic_bytes_per_launch"] = 194 * n
    # two launches overlap on two streams, so GRBM_GUI_ACTIVE / duration is not its clock; the
    # in-kernel probe (s_memtime against s_memrealtime per wave) is
    ve.pop("effective_clock_ghz", None)
    ve["clock"] = "in-kernel probe: profiles/%s_verify_clock_probe.json (CPZ_CLOCK_PROBE, tools/time_verify.py)" % rnd
    if "hbm_bytes_per_launch" in ve:
        ve["hbm_bytes_per_proof"] = ve["hbm_bytes_per_launch"] / n
    ve["source"] = "profiles/%s_verify_each_pmc.json (tools/profile.sh + tools/pmc_summary.py)" % rnd
# Verify span from the kernel trace: k_verify_each launches overlap (two streams), so the
# per-step time is the union of their intervals; a "step" is 2^20 proofs = 2^20 / n launches.
trace = os.path.join(src, "prof_trace", "run_kernel_trace.csv")
if ve and os.path.exists(trace):
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace))
                if r["Kernel_Name"].startswith("cpz::k_verify_each"))
    union, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                union += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        union += cur[1] - cur[0]
    steps = len(iv) * n / float(1 << 20)
    ve["trace_launches"] = len(iv)
    ve["trace_span_ns_per_2p20"] = union / steps if steps else None
# The bench line printed by the kernel-trace pass itself: its HIP-event kernel time for
# k_verify_each must agree with rocprof's average for the same launches.
bench_line = None
log = os.path.join(src, "prof_trace.log")
if os.path.exists(log):
    for line in open(log):
        if line.startswith('{"metric"'):
            bench_line = json.loads(line)
if bench_line:
    with open(os.path.join(prof, "%s_bench_under_profiler.json" % rnd), "w") as f:
        json.dump(bench_line, f, indent=1, sort_keys=True)
    ev = (bench_line.get("roofline") or {}).get("kernel_ms")
    if ve and ev and ve.get("avg_ns"):
        ve["bench_event_kernel_ms_same_run"] = ev
        ve["rocprof_avg_kernel_ms"] = ve["avg_ns"] / 1e6
        ve["event_vs_rocprof"] = ev / (ve["avg_ns"] / 1e6)
summary = {"round": rnd, "source": "tools/profile.sh + tools/pmc_summary.py", "kernels": out}
with open(os.path.join(prof, "%s_pmc.json" % rnd), "w") as f:
    json.dump(summary, f, indent=1, sort_keys=True)
if ve:
    with open(os.path.join(prof, "%s_verify_each_pmc.json" % rnd), "w") as f:
        json.dump(dict(ve, kernel="cpz::k_verify_each"), f, indent=1, sort_keys=True)
# k_rlc_bucket: one launch per RLC step of 2^20 proofs (the bench's RLC extra)
bk = out.get("k_rlc_bucket", {})
if bk:
    bk = dict(bk, kernel="cpz::k_rlc_bucket", workload="2^20 proofs per launch (bench.py RLC extra)",
              source="profiles/%s_rlc_bucket_pmc.json (tools/profile.sh + tools/pmc_summary.py)" % rnd)
    if "hbm_bytes_per_launch" in bk:
        bk["hbm_bytes_per_2p20"] = bk["hbm_bytes_per_launch"]
    bk["algorithmic_bytes_per_2p20"] = 48 * 132 * (1 << 20)
    with open(os.path.join(prof, "%s_rlc_bucket_pmc.json" % rnd), "w") as f:
        json.dump(bk, f, indent=1, sort_keys=True)
print(json.dumps({k: {c: round(v, 1) if isinstance(v, float) else v for c, v in d.items()}
                  for k, d in out.items() if k in ("k_verify_each", "k_challenge", "k_rlc_bucket", "k_rlc_prepare")},
                 indent=1))
