"""The drop-in boundary without a GPU: the C-ABI library loads, exports every function
include/cpz.h declares, the headers compile as C and C++, and calls fail loudly (no CPU
fallback) when no device is visible."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "cpz.h")


def _declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cpz_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import chaum_pedersen._native as nat
    return nat.load()


def test_every_declared_symbol_is_exported(lib):
    names = _declared()
    assert len(names) >= 12
    for name in names:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "chaum-pedersen-zkp_amd", "lib", "libcpz.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (cpz_\w+)", out))
    assert set(names) <= exported
    import chaum_pedersen._native as nat
    assert set(nat.EXPORTED) <= set(names)


def test_headers_compile_as_c_and_cpp(tmp_path):
    c = tmp_path / "t.c"
    c.write_text('#include "cpz.h"\nint main(void){ uint8_t g[32], h[32]; cpz_default_generators(g, h); return 0; }\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(c)],
                   check=True)
    cc = tmp_path / "t.cpp"
    cc.write_text('#include "cpz_batch.hpp"\nint main(){ return (int)chaum_pedersen::MAX_BATCH_SIZE - 1000; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                    str(cc)], check=True)


def test_default_generators_without_device(lib, golden):
    g = ctypes.create_string_buffer(32)
    h = ctypes.create_string_buffer(32)
    lib.cpz_default_generators(g, h)
    assert g.raw.hex() == golden["g"] and h.raw.hex() == golden["h"]


def test_no_device_fails_loudly(lib):
    if lib.cpz_device_count() > 0:
        pytest.skip("a GPU is visible")
    import chaum_pedersen as cp
    with pytest.raises(cp.CpzError):
        cp.Gpu(0)
    h = ctypes.c_void_p()
    assert lib.cpz_ctx_create(0, ctypes.byref(h)) != 0
    assert lib.cpz_verify_each(None, None, None, 1, *([None] * 9)) == -1


def test_missing_library_raises(tmp_path):
    import chaum_pedersen._native as nat
    with pytest.raises(nat.CpzError):
        nat._lib_backup = nat._lib
        try:
            nat._lib = None
            nat.load(str(tmp_path / "nope.so"))
        finally:
            nat._lib = nat._lib_backup
