"""Build recipes for the in-tree native artefacts (no cmake/ninja needed).

* ``lib/libcpz.so``      -- the product: gfx950 HIP kernels + host runtime + C ABI
                           (hipcc --offload-arch=gfx950).
* ``tests/native/libcpz_hosttest.so`` -- CPU build of the device-library headers with
                           limb-bound assertions, for unit tests only.
* ``oracle/``            -- delegated to oracle/Makefile (the C oracle: CPU baseline and
                           at-scale checker; test infrastructure only).

Each target is rebuilt only when one of its sources is newer than the output.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIBCPZ = os.path.join(LIBDIR, "libcpz.so")
HOSTTEST = os.path.join(ROOT, "tests", "native", "libcpz_hosttest.so")
ARCH = os.environ.get("CPZ_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the gfx950 build needs ROCm")


def _newer(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _headers():
    hdr = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hdr + [os.path.join(ROOT, "include", "cpz.h")]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed: %s\n%s" % (" ".join(cmd), r.stdout[-4000:]))
    return r.stdout


# Per-unit flags: k_verify_wide's single-wave row loops ran 12 % apart with their placement
# (Straus 46.6 against 52.7 us for identical loop code, profiles/r05_wide_align_ab.txt);
# aligned loop heads make that independent of the code before them.
UNIT_FLAGS = {"wide.hip": ["-falign-loops=64"]}


def build_libcpz(force: bool = False, verbose: bool = False, out: str = LIBCPZ, defines=()) -> str:
    """Build the product library.  `out` / `defines` build a tuning variant (e.g.
    CPZ_VERIFY_WAVES=3) elsewhere, for side-by-side measurement with CPZ_LIB=<out>."""
    units = ["kernels.hip", "wide.hip", "rlc.hip", "part.hip", "runtime.hip"]
    srcs = [os.path.join(CSRC, u) for u in units] + _headers()
    if not force and not defines and not _newer(out, srcs):
        return out
    objdir = os.path.join(os.path.dirname(out), "obj" if not defines else "obj_" + "_".join(defines).replace("=", ""))
    os.makedirs(objdir, exist_ok=True)
    hipcc = _hipcc()
    common = [hipcc, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I", CSRC,
              "-I", os.path.join(ROOT, "include")] + ["-D" + d for d in defines]
    if defines and os.environ.get("CPZ_EXTRA_FLAGS"):  # tuning variants only, never the product build
        common += os.environ["CPZ_EXTRA_FLAGS"].split()

    def compile_one(u):
        obj = os.path.join(objdir, u.replace(".hip", ".o"))
        if force or defines or _newer(obj, [os.path.join(CSRC, u)] + _headers()):
            uf = [] if defines and os.environ.get("CPZ_NO_UNIT_FLAGS") else UNIT_FLAGS.get(u, [])  # variants only
            _run(common + uf + ["-c", os.path.join(CSRC, u), "-o", obj])
        return obj

    with ThreadPoolExecutor(max_workers=len(units)) as ex:
        objs = list(ex.map(compile_one, units))
    tmp = out + ".tmp"
    _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, out)
    if verbose:
        print("built", out)
    return out


CLOCK_PROBE_LIB = os.path.join(LIBDIR, "timing", "clock_probe.so")


def build_clock_probe(force: bool = False) -> str:
    """Timing-only build with the in-kernel clock probes (csrc/timing_only.h): k_verify_each,
    k_rlc_prepare, k_rlc_bucket stamp their shader clock; tools/time_verify.py reads them.
    Not part of build_all: only the measurement runs load it (CPZ_LIB)."""
    os.makedirs(os.path.dirname(CLOCK_PROBE_LIB), exist_ok=True)
    return build_libcpz(force, out=CLOCK_PROBE_LIB, defines=("CPZ_CLOCK_PROBE", "CPZ_TIMING_ONLY"))


def build_hosttest(force: bool = False) -> str:
    src = os.path.join(ROOT, "tests", "native", "hostlib.cpp")
    if not force and not _newer(HOSTTEST, [src] + _headers()):
        return HOSTTEST
    cxx = shutil.which("g++") or "g++"
    tmp = HOSTTEST + ".tmp"
    # CPZ_HOST_DEFINES: extra -D flags to check a tuning variant of the device library on the CPU
    extra = ["-D" + d for d in os.environ.get("CPZ_HOST_DEFINES", "").split()]
    _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-DCPZ_BOUNDS_CHECK", "-DCPZ_COUNT_OPS"] + extra +
         ["-I", CSRC, src, "-o", tmp])
    os.replace(tmp, HOSTTEST)
    return HOSTTEST


CPP_TEST = os.path.join(ROOT, "tests", "cpp", "batch_verifier_test")


def build_cpp_test(force: bool = False) -> str:
    """C++ mirror of batch.rs's unit tests over include/cpz_batch.hpp (links libcpz.so)."""
    src = os.path.join(ROOT, "tests", "cpp", "batch_verifier_test.cpp")
    hdrs = [os.path.join(ROOT, "include", "cpz.h"), os.path.join(ROOT, "include", "cpz_batch.hpp")]
    # libcpz.so is linked dynamically: only the sources and headers make the binary stale (a rebuild
    # inside a GPU test run is what the in-tree build is there to avoid)
    if not force and not _newer(CPP_TEST, [src] + hdrs):
        return CPP_TEST
    cxx = shutil.which("g++") or "g++"
    _run([cxx, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-o", CPP_TEST + ".tmp",
          "-L", LIBDIR, "-lcpz", "-Wl,-rpath,$ORIGIN/../../chaum-pedersen-zkp_amd/lib"])
    os.replace(CPP_TEST + ".tmp", CPP_TEST)
    return CPP_TEST


DROPIN_TEST = os.path.join(ROOT, "tests", "cpp", "dropin_test")


def build_dropin_test(force: bool = False) -> str:
    """The drop-in's call sequence through the C++ mirror (tests/test_gpu_dropin.py)."""
    src = os.path.join(ROOT, "tests", "cpp", "dropin_test.cpp")
    hdrs = [os.path.join(ROOT, "include", "cpz.h"), os.path.join(ROOT, "include", "cpz_batch.hpp")]
    if not force and not _newer(DROPIN_TEST, [src] + hdrs):  # libcpz.so: linked dynamically
        return DROPIN_TEST
    cxx = shutil.which("g++") or "g++"
    _run([cxx, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-o", DROPIN_TEST + ".tmp",
          "-L", LIBDIR, "-lcpz", "-Wl,-rpath,$ORIGIN/../../chaum-pedersen-zkp_amd/lib"])
    os.replace(DROPIN_TEST + ".tmp", DROPIN_TEST)
    return DROPIN_TEST


def build_oracle(force: bool = False) -> None:
    mk = os.path.join(ROOT, "oracle", "Makefile")
    if os.path.exists(mk):
        _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")] + (["-B"] if force else []))


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_hosttest(force)
    build_oracle(force)
    build_libcpz(force, verbose)
    build_cpp_test(force)
    build_dropin_test(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
