"""The timing experiments that compile wrong verdicts into the kernels (csrc/timing_only.h:
CPZ_EXP_SLAB_MOD, CPZ_EXP_NOSPLIT, CPZ_CLOCK_PROBE) cannot reach the product ABI: without
CPZ_TIMING_ONLY a translation unit that sees one does not compile; with it, cpz_ctx_create
refuses (CPZ_EINVAL, naming the flag) and only cpz_ctx_create_timing_only -- exported by such
builds alone -- opens a context.  Checked by preprocessing each unit for the host (no GPU,
no full compile), plus the product library's symbol table and ABI version."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "chaum-pedersen-zkp_amd", "csrc")
LIB = os.path.join(ROOT, "chaum-pedersen-zkp_amd", "lib", "libcpz.so")
FLAGS = ("CPZ_EXP_SLAB_MOD=4096", "CPZ_EXP_NOSPLIT", "CPZ_CLOCK_PROBE")
UNITS = ("kernels.hip", "wide.hip", "rlc.hip", "runtime.hip")


def _hipcc():
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        pytest.skip("hipcc not available")
    return h


def _pre(unit, defines, out=os.devnull):
    cmd = [_hipcc(), "--offload-arch=gfx950", "-std=c++17", "-E", "--cuda-host-only", "-I", CSRC,
           "-I", os.path.join(ROOT, "include")] + ["-D" + d for d in defines] + [os.path.join(CSRC, unit), "-o", out]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.parametrize("flag", FLAGS)
@pytest.mark.parametrize("unit", UNITS)
def test_wrong_verdict_flag_needs_timing_only(flag, unit):
    r = _pre(unit, [flag])
    assert r.returncode != 0
    assert "build them with -DCPZ_TIMING_ONLY" in r.stdout + r.stderr


@pytest.mark.parametrize("flag", FLAGS)
def test_timing_only_build_refuses_the_product_create(flag, tmp_path):
    out = str(tmp_path / "rt.i")
    r = _pre("runtime.hip", [flag, "CPZ_TIMING_ONLY"], out)
    assert r.returncode == 0, r.stderr[-2000:]
    src = open(out).read()
    body = src[src.index("int cpz_ctx_create(int device_ordinal, cpz_ctx** out) {"):]
    body = body[:body.index("\n}\n")]
    # the product entry point returns the error naming the flag, and never creates a context
    assert "CPZ_EINVAL" in body or "(-1)" in body
    assert '"' + flag.split("=")[0] + '"' in body and "ctx_create(" not in body.replace("cpz_ctx_create(", "")
    assert "int cpz_ctx_create_timing_only(int device_ordinal" in src


def test_product_build_has_no_timing_entry_and_reports_abi():
    if not os.path.exists(LIB):
        pytest.skip("libcpz.so not built")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    assert "cpz_ctx_create_timing_only" not in out
    import chaum_pedersen._native as nat
    lib = nat.load()
    hdr = open(os.path.join(ROOT, "include", "cpz.h")).read()
    assert int(re.search(r"#define CPZ_ABI_VERSION (\d+)", hdr).group(1)) == lib.cpz_abi_version() == nat.ABI_VERSION
    for unit in UNITS:  # and the product units preprocess cleanly with no experiment flag
        assert _pre(unit, []).returncode == 0
