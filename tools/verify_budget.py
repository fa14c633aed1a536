"""Instruction and cycle budget of k_verify_each's inner loops, by instruction class.

    python3 tools/verify_budget.py [k.s] [profiles/rNN_clock_rates.json] > profiles/rNN_verify_budget.json

k.s is the device assembly of kernels.hip (built here with the product flags when omitted).  The
loops are found by their MAD counts, which follow from the formulas (tools/isa_hist.py prints every
loop): the Straus step's additions (2 cached additions, each p1p1->p3 + add: 16 products x 110
MADs = 1760), one doubling of the 4 per window (p1p1->p2 + 4 squarings: 3 x 110 + 4 x 65 = 590,
one MAD of which is address arithmetic), the comb's mixed addition (7 x 110 = 770) and one squaring
of the decode chains (55).  Each class is priced at the issue cost the clock_rates sweep measured for
its representative instruction at 2 waves/SIMD (the kernel's occupancy), in SIMD cycles per wave64
instruction; scalar instructions issue on the scalar unit and are priced at 0.
"""
import collections
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_hist  # noqa: E402

KERNEL = "_ZN3cpz13k_verify_eachENS_10VerifyArgsE"
CLASSES = [  # (class, mnemonic prefixes, clock_rates op that prices it)
    ("mad: v_mad_i64_i32 (products + the high-word carry)", ("v_mad_i64_i32",), "v_mad_i64_i32"),
    ("carry: v_and / v_lshrrev / v_add3 (32-bit limb split)", ("v_and_b32", "v_lshrrev_b32", "v_add3_u32"),
     "v_and_b32"),
    ("carry (squaring chains): v_ashrrev_i64 / v_lshl_add_u64", ("v_ashrrev_i64", "v_lshl_add_u64"),
     "v_lshl_add_u64"),
    ("19 g operands: v_mul_lo_u32", ("v_mul_lo_u32",), "v_mul_lo_u32"),
    ("field add / sub: v_add_u32 / v_sub_u32", ("v_add_u32", "v_sub_u32", "v_subrev"), "v_add_u32"),
    ("2 f operands, digits, addresses: shifts, u24 mads, alignbit, or, bfe",
     ("v_lshlrev", "v_lshl_add_u32", "v_mad_u32_u24", "v_mad_i32_i24", "v_alignbit", "v_or_b32", "v_bfe",
      "v_mad_u64_u32", "v_mov_b32", "v_cmp"), "v_add_u32"),
    ("table sign select: v_cndmask", ("v_cndmask",), "v_and_b32"),
    ("memory: global / ds loads", ("global_", "ds_", "scratch_", "buffer_"), None),
    ("scalar + control (s_*)", ("s_",), None),
]
LOOPS = [("straus_additions", 1760), ("doubling", 589), ("comb_mixed_addition", 770), ("decode_squaring", 55)]


def classify(mn):
    for name, prefixes, op in CLASSES:
        if mn.startswith(prefixes):
            return name, op
    return "other", "v_add_u32"


def main():
    asm = sys.argv[1] if len(sys.argv) > 1 else None
    rates = sys.argv[2] if len(sys.argv) > 2 else None
    if asm is None:
        asm = "/tmp/cpz_kernels_budget.s"
        csrc = os.path.join(ROOT, "chaum-pedersen-zkp_amd", "csrc")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", csrc,
                               "-I", os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                               os.path.join(csrc, "kernels.hip"), "-o", asm], stderr=subprocess.DEVNULL)
    if rates is None:
        pdir = os.path.join(ROOT, "profiles")
        rates = os.path.join(pdir, sorted(f for f in os.listdir(pdir) if f.endswith("_clock_rates.json"))[-1])
    cyc = {r["op"]: r["cycles_per_instr"] for r in json.load(open(rates))["rows"] if r["waves_per_simd"] == 2}
    bodies = isa_hist.loop_bodies(asm, KERNEL)
    out = {"kernel": "k_verify_each", "asm": "kernels.hip, hipcc --offload-arch=gfx950 -O3 (product flags)",
           "cycle_costs": {"source": os.path.relpath(rates, ROOT), "waves_per_simd": 2, "cycles": cyc},
           "loops": {}}
    for name, mads in LOOPS:
        hit = [c for _, c in bodies if c.get("v_mad_i64_i32", 0) == mads]
        if not hit:
            out["loops"][name] = None
            continue
        body = hit[0]
        per = collections.OrderedDict()
        for mn, k in body.items():
            cls, op = classify(mn)
            e = per.setdefault(cls, {"instructions": 0, "cycles": 0.0})
            e["instructions"] += k
            e["cycles"] += k * (cyc.get(op, 0.0) if op else 0.0)
        tot_i = sum(e["instructions"] for e in per.values())
        tot_c = sum(e["cycles"] for e in per.values())
        for e in per.values():
            e["share_instructions"] = round(e["instructions"] / tot_i, 4)
            e["share_cycles"] = round(e["cycles"] / tot_c, 4) if tot_c else 0.0
            e["cycles"] = round(e["cycles"], 1)
        out["loops"][name] = {"instructions": tot_i, "cycles": round(tot_c, 1),
                              "classes": dict(sorted(per.items(), key=lambda kv: -kv[1]["cycles"]))}
    win = [out["loops"].get("straus_additions"), out["loops"].get("doubling")]
    if all(win):
        agg = collections.defaultdict(lambda: {"instructions": 0, "cycles": 0.0})
        for mult, lp in ((1, win[0]), (4, win[1])):
            for cls, e in lp["classes"].items():
                agg[cls]["instructions"] += mult * e["instructions"]
                agg[cls]["cycles"] += mult * e["cycles"]
        ti = sum(e["instructions"] for e in agg.values())
        tc = sum(e["cycles"] for e in agg.values())
        out["straus_window"] = {
            "what": "one radix-16 window of the two-point Straus loop: 4 doublings + 2 cached additions",
            "instructions": ti, "cycles": round(tc, 1),
            "classes": {k: {"instructions": v["instructions"], "share_instructions": round(v["instructions"] / ti, 4),
                            "cycles": round(v["cycles"], 1), "share_cycles": round(v["cycles"] / tc, 4)}
                        for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["cycles"])}}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
