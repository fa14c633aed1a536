"""bench/opcount.json (the algorithmic work the roofline divides by) must match what the
device code actually executes per proof, counted on the host build of csrc/verify.h."""
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_verify_each_opcount(golden):
    import build_native
    lib = ctypes.CDLL(build_native.build_hosttest())
    oc = json.load(open(os.path.join(ROOT, "bench", "opcount.json")))["verify_each"]
    g, h = bytes.fromhex(golden["g"]), bytes.fromhex(golden["h"])
    for p in [q for q in golden["proofs"] if "c" in q][:5]:
        f = {k: bytes.fromhex(p[k]) for k in ("y1", "y2", "r1", "r2", "s", "c")}
        m, s = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        lib.cpzt_verify_opcount(ctypes.byref(m), ctypes.byref(s), g, h, f["y1"], f["y2"], f["r1"], f["r2"], f["s"],
                                f["c"])
        # fixed windows: the work does not depend on the data
        assert (m.value, s.value) == (oc["fe_mul"], oc["fe_sq"])
    assert oc["mads_per_proof"] == oc["fe_mul"] * oc["mads_per_fe_mul"] + oc["fe_sq"] * oc["mads_per_fe_sq"]


def test_rlc_opcounts(golden):
    """The RLC roofline's per-unit work (bench/opcount.json "rlc") is what the host build of
    the same device code executes; the prepared-point fallback verify gives verify_one's
    statuses on the golden proofs."""
    import build_native
    lib = ctypes.CDLL(build_native.build_hosttest())
    oc = json.load(open(os.path.join(ROOT, "bench", "opcount.json")))["rlc"]
    g, h = bytes.fromhex(golden["g"]), bytes.fromhex(golden["h"])
    keys = {0: "prepare_per_proof", 1: "bucket_per_entry", 2: "verify_prepared_per_proof"}
    part = json.load(open(os.path.join(ROOT, "bench", "opcount.json")))["part"]
    for p in [q for q in golden["proofs"] if "c" in q and q["status"] in (0, 1)]:
        f = {k: bytes.fromhex(p[k]) for k in ("y1", "y2", "r1", "r2", "s", "c")}
        for which, key in keys.items():
            m, s = ctypes.c_ulonglong(), ctypes.c_ulonglong()
            st = lib.cpzt_rlc_opcount(which, ctypes.byref(m), ctypes.byref(s), g, h, f["y1"], f["y2"], f["r1"],
                                      f["r2"], f["s"], f["c"])
            assert (m.value, s.value) == (oc[key]["fe_mul"], oc[key]["fe_sq"]), key
            assert oc[key]["mads"] == 100 * m.value + 55 * s.value
            if which == 2:
                assert st == p["status"], p["kind"]
        # the partitioned check's walk (k_part_acc): executed step, algorithmic entry step
        for which, key in ((3, "walk_step_executed"), (4, "walk_entry_step")):
            m, s = ctypes.c_ulonglong(), ctypes.c_ulonglong()
            assert lib.cpzt_rlc_opcount(which, ctypes.byref(m), ctypes.byref(s), g, h, f["y1"], f["y2"], f["r1"],
                                        f["r2"], f["s"], f["c"]) == 0
            assert (m.value, s.value) == (part[key]["fe_mul"], part[key]["fe_sq"]), key
    assert part["walk_boundary_step"]["fe_mul"] == part["walk_step_executed"]["fe_mul"]
    e, b = part["entries_per_block"], part["boundaries_per_block"]
    assert part["algorithmic_mads_per_block"] == e * part["walk_entry_step"]["mads"] + b * part["walk_boundary_step"]["mads"]
    assert part["executed_mads_per_block"] == (e + b) * part["walk_step_executed"]["mads"]
