"""ctypes binding of the C ABI in include/cpz.h (lib/libcpz.so, built in-tree).

The product path is the HIP library: there is no CPU fallback.  If the shared library
is missing or no GPU is visible, every verifying call raises CpzError.
"""
from __future__ import annotations

import ctypes
import os
import threading

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("CPZ_LIB") or os.path.join(_PKG_ROOT, "lib", "libcpz.so")

CPZ_OK = 0
CPZ_EINVAL = -1
CPZ_EHIP = -2
CPZ_ENOMEM = -3
CPZ_EGENERATOR = -4
CPZ_EEMPTY = -5

STATUS_OK = 0
STATUS_EQ_FAIL = 1
STATUS_BAD_POINT = 2
STATUS_BAD_SCALAR = 3
STATUS_IDENTITY = 4
STATUS_ZERO_S = 5

EXPORTED = (
    "cpz_device_count", "cpz_ctx_create", "cpz_ctx_destroy", "cpz_last_error",
    "cpz_default_generators", "cpz_verify_each", "cpz_verify_each_device", "cpz_challenges",
    "cpz_prove_synthetic", "cpz_prove_synthetic_device", "cpz_ctx_set_timing", "cpz_ctx_stage_times",
    "cpz_verify_batch", "cpz_verify_batch_device", "cpz_combine_partials", "cpz_msm",
    "cpz_parse_proofs", "cpz_parse_proofs_device", "cpz_verify_each_multi", "cpz_verify_batch_multi",
    "cpz_verify_response", "cpz_verify_response_device", "cpz_prove", "cpz_prove_device", "cpz_decode_points",
    "cpz_abi_version", "cpz_ctx_set_commitment_checks", "cpz_ctx_stage_times_n", "cpz_ctx_fallback_stats",
    "cpz_verify_each_ex", "cpz_verify_batch_ex", "cpz_verify_response_ex",
)
CALL_EQUATIONS_ONLY = 1   # CPZ_CALL_EQUATIONS_ONLY: commitment checks off for one call
NUM_STAGES = 16
FALLBACK_STATS = 8
FALLBACK_PATHS = {0: "none", 1: "bisection", 2: "partitioned", 3: "per_proof"}
ABI_VERSION = 5     # CPZ_ABI_VERSION of the cpz.h these declarations follow


class CpzError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("cpz error %d: %s" % (code, msg))
        self.code = code


_lock = threading.Lock()
_lib = None

_p = ctypes.c_void_p
_u8p = ctypes.c_char_p


def _declare(lib):
    lib.cpz_device_count.restype = ctypes.c_int
    lib.cpz_device_count.argtypes = []
    lib.cpz_ctx_create.restype = ctypes.c_int
    lib.cpz_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(_p)]
    lib.cpz_ctx_destroy.restype = None
    lib.cpz_ctx_destroy.argtypes = [_p]
    lib.cpz_last_error.restype = ctypes.c_char_p
    lib.cpz_last_error.argtypes = []
    lib.cpz_default_generators.restype = None
    lib.cpz_default_generators.argtypes = [_p, _p]
    lib.cpz_verify_each.restype = ctypes.c_int
    lib.cpz_verify_each.argtypes = [_p, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p]
    lib.cpz_verify_each_ex.restype = ctypes.c_int
    lib.cpz_verify_each_ex.argtypes = [_p, ctypes.c_uint32, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p]
    lib.cpz_verify_each_device.restype = ctypes.c_int
    lib.cpz_verify_each_device.argtypes = [_p, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p, _p]
    lib.cpz_challenges.restype = ctypes.c_int
    lib.cpz_challenges.argtypes = [_p, _p, _p, ctypes.c_size_t] + [_p] * 4 + [_p, _p, _p, _p]
    lib.cpz_prove_synthetic.restype = ctypes.c_int
    lib.cpz_prove_synthetic.argtypes = ([_p, _p, _p, ctypes.c_size_t, ctypes.c_uint64, _p, _p, _p, _p, _p]
                                        + [_p] * 5)
    lib.cpz_ctx_set_timing.restype = ctypes.c_int
    lib.cpz_ctx_set_timing.argtypes = [_p, ctypes.c_int]
    lib.cpz_ctx_stage_times.restype = ctypes.c_int
    lib.cpz_ctx_stage_times.argtypes = [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    lib.cpz_verify_batch.restype = ctypes.c_int
    lib.cpz_verify_batch.argtypes = ([_p, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p, ctypes.c_uint64,
                                     _p, ctypes.POINTER(ctypes.c_int), _p])
    lib.cpz_verify_batch_ex.restype = ctypes.c_int
    lib.cpz_verify_batch_ex.argtypes = ([_p, ctypes.c_uint32, _p, _p, ctypes.c_size_t] + [_p] * 5 +
                                        [_p, _p, _p, _p, ctypes.c_uint64, _p, ctypes.POINTER(ctypes.c_int), _p])
    lib.cpz_verify_each_multi.restype = ctypes.c_int
    lib.cpz_verify_each_multi.argtypes = [_p, ctypes.c_int, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p]
    lib.cpz_verify_batch_multi.restype = ctypes.c_int
    lib.cpz_verify_batch_multi.argtypes = ([_p, ctypes.c_int, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p,
                                           _p, _p, ctypes.POINTER(ctypes.c_int), _p])
    lib.cpz_verify_batch_device.restype = ctypes.c_int
    lib.cpz_verify_batch_device.argtypes = ([_p, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p, _p,
                                            ctypes.c_uint64, _p, ctypes.POINTER(ctypes.c_int), _p, ctypes.c_int, _p])
    lib.cpz_msm.restype = ctypes.c_int
    lib.cpz_msm.argtypes = [_p, ctypes.c_size_t, _p, _p, _p]
    lib.cpz_parse_proofs.restype = ctypes.c_int
    lib.cpz_parse_proofs.argtypes = [_p, ctypes.c_size_t, _p, _p, _p, _p, _p, _p, _p]
    lib.cpz_parse_proofs_device.restype = ctypes.c_int
    lib.cpz_parse_proofs_device.argtypes = [_p, ctypes.c_size_t, _p, _p, _p, _p, _p, _p, _p, _p]
    lib.cpz_combine_partials.restype = ctypes.c_int
    lib.cpz_combine_partials.argtypes = [_p, ctypes.c_size_t, _p, _p, ctypes.POINTER(ctypes.c_int)]
    lib.cpz_verify_response.restype = ctypes.c_int
    lib.cpz_verify_response.argtypes = [_p, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p]
    lib.cpz_verify_response_ex.restype = ctypes.c_int
    lib.cpz_verify_response_ex.argtypes = [_p, ctypes.c_uint32, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p]
    lib.cpz_verify_response_device.restype = ctypes.c_int
    lib.cpz_verify_response_device.argtypes = [_p, _p, _p, ctypes.c_size_t] + [_p] * 5 + [_p, _p, _p]
    lib.cpz_prove.restype = ctypes.c_int
    lib.cpz_prove.argtypes = [_p, _p, _p, ctypes.c_size_t, _p, _p, _p, _p, _p] + [_p] * 5
    lib.cpz_prove_device.restype = ctypes.c_int
    lib.cpz_prove_device.argtypes = [_p, _p, _p, ctypes.c_size_t, _p, _p, _p, _p, _p] + [_p] * 5 + [_p]
    lib.cpz_decode_points.restype = ctypes.c_int
    lib.cpz_decode_points.argtypes = [_p, ctypes.c_size_t, _p, _p, _p]
    lib.cpz_abi_version.restype = ctypes.c_int
    lib.cpz_abi_version.argtypes = []
    lib.cpz_ctx_set_commitment_checks.restype = ctypes.c_int
    lib.cpz_ctx_set_commitment_checks.argtypes = [_p, ctypes.c_int]
    lib.cpz_ctx_stage_times_n.restype = ctypes.c_int
    lib.cpz_ctx_stage_times_n.argtypes = [_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_int)]
    lib.cpz_ctx_fallback_stats.restype = ctypes.c_int
    lib.cpz_ctx_fallback_stats.argtypes = [_p, ctypes.POINTER(ctypes.c_uint64)]
    lib.cpz_ctx_create_timing_only.restype = ctypes.c_int
    lib.cpz_ctx_create_timing_only.argtypes = [ctypes.c_int, ctypes.POINTER(_p)]
    lib.cpz_prove_synthetic_device.restype = ctypes.c_int
    lib.cpz_prove_synthetic_device.argtypes = ([_p, _p, _p, ctypes.c_size_t, ctypes.c_uint64, _p, _p, _p, _p,
                                                _p] + [_p] * 5 + [_p])


class _Tolerant:
    """Attribute proxy for _declare on an older library: missing functions are skipped."""

    class _Sink:
        pass

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        try:
            return getattr(self._lib, name)
        except AttributeError:
            return _Tolerant._Sink()


def load(path: str = LIB_PATH):
    """Load (once) and return the native library; raises CpzError if it is absent."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise CpzError(CPZ_EHIP, "native library %s is missing: run __graft_entry__.build()" % path)
            # PyTorch-ROCm ships its own libamdhip64 (same SONAME as /opt/rocm's).  Load it
            # first so libcpz binds to the already-loaded runtime: one HIP runtime per
            # process, and device pointers / streams can be shared with torch tensors.
            try:
                import torch  # noqa: F401
            except Exception:
                pass
            lib = ctypes.CDLL(path)
            # every library declares what it exports: cpz_ctx_create_timing_only exists only in
            # timing-only builds, and a tuning variant (tools/variants.sh) may predate newer
            # entry points; the product library must export all of EXPORTED (test_abi)
            _declare(_Tolerant(lib))
            if not os.environ.get("CPZ_LIB"):
                got = lib.cpz_abi_version()
                if got != ABI_VERSION:
                    raise CpzError(CPZ_EINVAL, "%s has ABI version %d, these bindings follow %d: rebuild it"
                                   % (path, got, ABI_VERSION))
            _lib = lib
        return _lib


def check(rc: int) -> None:
    if rc != CPZ_OK:
        msg = load().cpz_last_error()
        raise CpzError(rc, msg.decode() if msg else "")


def default_generators():
    g = ctypes.create_string_buffer(32)
    h = ctypes.create_string_buffer(32)
    load().cpz_default_generators(g, h)
    return g.raw, h.raw
