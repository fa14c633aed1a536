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
for tag in ("prof_fetch", "prof_write", "prof_sq"):
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
ve = out.get("k_verify_each", {})
if ve:
    n = int(os.environ.get("PROOFS_PER_LAUNCH", 1 << 16))
    if "SQ_INSTS_VALU" in ve:
        ve["valu_instructions_per_proof"] = ve["SQ_INSTS_VALU"] * 64 / n
    ve["workload"] = ("%d proofs per launch (bench.py default 2^20 per step = 16 launches), rocprofv3 --pmc, "
                      "one counter group per pass" % n)
    ve["correction"] = ("gfx950: FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads "
                        "(MI355X_MICROARCH.md HBM) -> doubled; WRITE_SIZE as reported; units kB")
    ve["algorithmic_bytes_per_launch"] = 194 * n
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
summary = {"round": rnd, "source": "tools/profile.sh + tools/pmc_summary.py", "kernels": out}
with open(os.path.join(prof, "%s_pmc.json" % rnd), "w") as f:
    json.dump(summary, f, indent=1, sort_keys=True)
if ve:
    with open(os.path.join(prof, "%s_verify_each_pmc.json" % rnd), "w") as f:
        json.dump(dict(ve, kernel="cpz::k_verify_each"), f, indent=1, sort_keys=True)
print(json.dumps({k: {c: round(v, 1) if isinstance(v, float) else v for c, v in d.items()}
                  for k, d in out.items() if k in ("k_verify_each", "k_challenge")}, indent=1))
