"""chaum_pedersen -- MI355X-native drop-in for the reference's verify path.

Mirrors the reference crate's public surface for the batch-verification path
(kobby-pentangeli/chaum-pedersen-zkp: src/verifier/batch.rs, src/primitives/gadgets.rs)
on top of the C ABI in include/cpz.h:

    Parameters, Statement, Proof       gadgets.rs:25-489 (encodings kept as 32-byte strings;
                                       Proof.from_bytes runs the device parser, k_parse_proofs)
    Transcript                         transcript.rs:25-72 (the optional context only)
    Verifier                           verifier/mod.rs:42-172 (verify, verify_with_transcript,
                                       verify_response)
    Prover                             prover/mod.rs:25-132 (prove, prove_with_transcript,
                                       commit, respond)
    BatchVerifier                      batch.rs:82-324 (same names, cap, errors, ordering)
    Gpu                                bulk / device-resident entry points (no 1000 cap)

Every verification runs the gfx950 kernels in lib/libcpz.so; nothing here computes a
verification result on the CPU.
"""
from __future__ import annotations

import ctypes
import struct
from typing import List, Optional, Sequence

import numpy as np

from . import _native
from ._native import (CpzError, STATUS_BAD_POINT, STATUS_BAD_SCALAR, STATUS_EQ_FAIL,
                      STATUS_IDENTITY, STATUS_OK, STATUS_ZERO_S)

__all__ = [
    "Error", "InvalidParams", "InvalidScalar", "InvalidGroupElement", "CpzError",
    "Parameters", "Statement", "Proof", "BatchVerifier", "Gpu", "VerifyResult", "Transcript", "Verifier", "Prover",
    "MAX_BATCH_SIZE", "RLC_MIN_GROUP", "PROTOCOL_VERSION", "STATUS_OK", "STATUS_EQ_FAIL", "STATUS_BAD_POINT",
    "STATUS_BAD_SCALAR", "STATUS_IDENTITY", "STATUS_ZERO_S", "default_generators", "verify_each_multi", "verify_batch_multi",
]

MAX_BATCH_SIZE = 1000          # batch.rs:48
# Smallest Parameters group that BatchVerifier.verify sends to the RLC batch check (smaller
# groups: per-proof verification); rust/reference-patch/gpu.rs RLC_MIN_GROUP, cpz_batch.hpp.
RLC_MIN_GROUP = 1001
PROTOCOL_VERSION = 1           # gadgets.rs:12
L = 2**252 + 27742317777372353535851937790883648493   # group order (ristretto.rs scalars)


# --- error taxonomy (src/error.rs:5-17) -------------------------------------------------
class Error(Exception):
    pass


class InvalidParams(Error):
    pass


class InvalidScalar(Error):
    pass


class InvalidGroupElement(Error):
    pass


_STATUS_ERR = {
    STATUS_EQ_FAIL: (InvalidParams, "Proof verification failed"),
    STATUS_BAD_POINT: (InvalidGroupElement, "Bytes do not represent a valid Ristretto point"),
    STATUS_BAD_SCALAR: (InvalidScalar, "Bytes do not represent a valid scalar"),
    STATUS_IDENTITY: (InvalidParams, "Commitment contains identity element"),
    STATUS_ZERO_S: (InvalidParams, "Response scalar is zero"),
}


class VerifyResult:
    """Per-entry `Result<()>` of BatchVerifier::verify."""

    __slots__ = ("status",)

    def __init__(self, status: int):
        self.status = int(status)

    def is_ok(self) -> bool:
        return self.status == STATUS_OK

    def is_err(self) -> bool:
        return self.status != STATUS_OK

    def error(self) -> Optional[Error]:
        if self.status == STATUS_OK:
            return None
        cls, msg = _STATUS_ERR[self.status]
        return cls(msg)

    def __repr__(self) -> str:
        return "Ok(())" if self.is_ok() else "Err(%r)" % (self.error(),)


def default_generators():
    """(g, h) encodings: basepoint and hash-to-group of the h DST (ristretto.rs:79-91)."""
    return _native.default_generators()


def _b32(x, what: str) -> bytes:
    b = bytes(x)
    if len(b) != 32:
        raise InvalidGroupElement("Expected 32 bytes, got %d (%s)" % (len(b), what))
    return b


class Parameters:
    """Generators (g, h).  Parameters() gives the defaults (gadgets.rs:43-48)."""

    def __init__(self, g: Optional[bytes] = None, h: Optional[bytes] = None):
        dg, dh = default_generators()
        self.g = dg if g is None else _b32(g, "g")
        self.h = dh if h is None else _b32(h, "h")

    @classmethod
    def new(cls) -> "Parameters":
        return cls()

    @classmethod
    def with_generators(cls, g: bytes, h: bytes) -> "Parameters":
        """gadgets.rs:77-103: identity / equal generators rejected here; undecodable ones
        are rejected by the GPU table build (CPZ_EGENERATOR) on first use."""
        g, h = _b32(g, "g"), _b32(h, "h")
        if g == bytes(32):
            raise InvalidParams("Generator g cannot be identity")
        if h == bytes(32):
            raise InvalidParams("Generator h cannot be identity")
        if g == h:
            raise InvalidParams("Generators g and h must be different")
        return cls(g, h)

    def generator_g(self) -> bytes:
        return self.g

    def generator_h(self) -> bytes:
        return self.h

    def __eq__(self, other) -> bool:
        return isinstance(other, Parameters) and (self.g, self.h) == (other.g, other.h)

    def __hash__(self) -> int:
        return hash((self.g, self.h))


class Statement:
    """Public values (y1, y2) as 32-byte encodings (gadgets.rs:177-239)."""

    def __init__(self, y1: bytes, y2: bytes):
        self.y1 = _b32(y1, "y1")
        self.y2 = _b32(y2, "y2")

    @classmethod
    def from_witness(cls, params: "Parameters", x, gpu: Optional["Gpu"] = None) -> "Statement":
        """y1 = x g, y2 = x h (gadgets.rs:217-221), computed on the device (cpz_prove)."""
        out = (gpu or _gpu()).prove([_scalar_bytes(x)], [_scalar_bytes(1)], params=params)
        return cls(out["y1"][0].tobytes(), out["y2"][0].tobytes())


class Proof:
    """Commitment (r1, r2) and response s (gadgets.rs:307-489)."""

    def __init__(self, r1: bytes, r2: bytes, s: bytes, version: int = PROTOCOL_VERSION):
        self.r1 = _b32(r1, "r1")
        self.r2 = _b32(r2, "r2")
        self.s = bytes(s)
        if len(self.s) != 32:
            raise InvalidScalar("Expected 32 bytes, got %d" % len(self.s))
        self.version = version

    def to_bytes(self) -> bytes:
        """gadgets.rs:343-361: [ver][u32be 32][r1][u32be 32][r2][u32be 32][s] = 109 bytes."""
        out = bytearray([self.version])
        for part in (self.r1, self.r2, self.s):
            out += struct.pack(">I", len(part)) + part
        return bytes(out)

    @classmethod
    def from_bytes(cls, b: bytes, gpu: Optional["Gpu"] = None) -> "Proof":
        """gadgets.rs:364-489, exactly: the blob goes through the device parser
        (cpz_parse_proofs, one k_parse_proofs thread), which applies the reference's checks
        in its order -- each field's structure, then its decode (element_from_bytes /
        scalar_from_bytes), trailing bytes, identity commitment, zero s -- and the first
        failing check raises the reference's error type and message."""
        out = cls.from_bytes_many([b], gpu)[0]
        if isinstance(out, Error):
            raise out
        return out

    @classmethod
    def from_bytes_many(cls, blobs: Sequence[bytes], gpu: Optional["Gpu"] = None) -> List:
        """Proof::from_bytes for many blobs in one device pass: a Proof or the Error the
        reference would return, per blob."""
        if not blobs:
            return []
        r1, r2, s, codes, aux = (gpu or _gpu()).parse_proofs(blobs)
        return [cls(r1[i].tobytes(), r2[i].tobytes(), s[i].tobytes()) if codes[i] == 0
                else parse_error(int(codes[i]), int(aux[i])) for i in range(len(blobs))]

    def commitment(self):
        return self.r1, self.r2

    def response(self) -> bytes:
        return self.s


# Proof::from_bytes outcome codes of the bulk parser (cpz.h CPZ_PARSE_*), with the
# reference's error type and message (gadgets.rs:364-489, ristretto.rs:94-138).
PARSE_ERRORS = {
    1: (InvalidParams, "Proof too small: {} bytes"),
    2: (InvalidParams, "Unsupported proof version: {}"),
    3: (InvalidParams, "Truncated proof: missing r1 length"),
    4: (InvalidParams, "Invalid r1 length: {}"),
    5: (InvalidParams, "Truncated proof: incomplete r1 data"),
    6: (InvalidGroupElement, "Expected 32 bytes, got {}"),
    7: (InvalidGroupElement, "Bytes do not represent a valid Ristretto point"),
    8: (InvalidParams, "Truncated proof: missing r2 length"),
    9: (InvalidParams, "Invalid r2 length: {}"),
    10: (InvalidParams, "Truncated proof: incomplete r2 data"),
    11: (InvalidGroupElement, "Expected 32 bytes, got {}"),
    12: (InvalidGroupElement, "Bytes do not represent a valid Ristretto point"),
    13: (InvalidParams, "Truncated proof: missing s length"),
    14: (InvalidParams, "Invalid s length: {}"),
    15: (InvalidParams, "Truncated proof: incomplete s data"),
    16: (InvalidScalar, "Expected 32 bytes, got {}"),
    17: (InvalidScalar, "Bytes do not represent a valid scalar"),
    18: (InvalidParams, "Proof has {} trailing bytes"),
    19: (InvalidParams, "Commitment contains identity element"),
    20: (InvalidParams, "Response scalar is zero"),
}


def parse_error(code: int, aux: int = 0) -> Optional[Error]:
    """The exception Proof::from_bytes raises for a bulk-parser code (None for 0)."""
    if code == 0:
        return None
    cls, msg = PARSE_ERRORS[int(code)]
    return cls(msg.format(int(aux)))


def _scalar_bytes(x) -> bytes:
    """A scalar given as an int (taken mod l) or as 32 little-endian bytes."""
    if isinstance(x, (bytes, bytearray, memoryview)):
        b = bytes(x)
        if len(b) != 32:
            raise InvalidScalar("Expected 32 bytes, got %d" % len(b))
        return b
    return (int(x) % L).to_bytes(32, "little")


def _rows(data, n: int, name: str) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
    if a.shape != (n, 32):
        a = a.reshape(n, 32)
    return a


def _ctx_arrays(contexts: Optional[Sequence[Optional[bytes]]], n: int):
    """None -> no contexts.  Otherwise (blob, offsets[n+1], present[n])."""
    if contexts is None:
        return None, None, None
    if len(contexts) != n:
        raise InvalidParams("contexts length %d != %d" % (len(contexts), n))
    present = np.array([0 if c is None else 1 for c in contexts], dtype=np.uint8)
    if not present.any():
        return None, None, None
    lens = np.array([0 if c is None else len(c) for c in contexts], dtype=np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(c for c in contexts if c is not None) or b"\0", dtype=np.uint8).copy()
    return blob, off, present


def _ptr(a) -> Optional[int]:
    return None if a is None else a.ctypes.data


def _flags(equations_only: bool) -> int:
    return _native.CALL_EQUATIONS_ONLY if equations_only else 0


def _torch_stream(stream):
    """Device entry points default to torch's current stream, so kernels are ordered with
    the torch ops that produce / consume the tensors."""
    if stream is not None:
        return stream
    import torch
    return torch.cuda.current_stream().cuda_stream


class Gpu:
    """A verifier context on one GPU (cpz_ctx).  Bulk entry points, no batch cap."""

    def __init__(self, device: int = 0, timing_only: bool = False):
        """timing_only: open the context of a timing-only build (tools/time_verify.py); the
        product library has no such entry point and its verdicts are the only ones."""
        lib = _native.load()
        ndev = lib.cpz_device_count()
        if ndev <= 0:
            raise CpzError(_native.CPZ_EHIP, "no GPU visible to the HIP runtime")
        h = ctypes.c_void_p()
        create = lib.cpz_ctx_create
        if timing_only:
            if not hasattr(lib, "cpz_ctx_create_timing_only"):
                raise CpzError(_native.CPZ_EINVAL, "not a timing-only build")
            create = lib.cpz_ctx_create_timing_only
        _native.check(create(device, ctypes.byref(h)))
        self._lib = lib
        self._h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.cpz_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- per-kernel timing (HIP events on the launch stream) -------------------------------
    STAGES = ("challenge", "verify_each", "rlc_prepare", "rlc_msm", "fallback", "verify_span", "prove", "generators",
              "rlc_sort", "rlc_bucket", "rlc_bucket_fix", "rlc_reduce", "rlc_final", "generators_varbase", "part_acc",
              "part_acc_locate")

    def set_timing(self, enable: bool) -> None:
        _native.check(self._lib.cpz_ctx_set_timing(self._h, 1 if enable else 0))

    def stage_times(self):
        """{stage: (total_ms, launches)} since the previous call (synchronises)."""
        ms = (ctypes.c_double * _native.NUM_STAGES)()
        cnt = (ctypes.c_int * _native.NUM_STAGES)()
        _native.check(self._lib.cpz_ctx_stage_times_n(self._h, _native.NUM_STAGES, ms, cnt))
        return {self.STAGES[k]: (ms[k], cnt[k]) for k in range(_native.NUM_STAGES) if cnt[k]}

    def fallback_stats(self) -> dict:
        """What the last verify_batch call's fallback did (cpz_ctx_fallback_stats)."""
        out = (ctypes.c_uint64 * _native.FALLBACK_STATS)()
        _native.check(self._lib.cpz_ctx_fallback_stats(self._h, out))
        return {"path": _native.FALLBACK_PATHS.get(int(out[0]), str(out[0])), "probe_invalid": int(out[1]),
                "blocks_checked": int(out[2]), "blocks_failing": int(out[3]), "per_proof": int(out[4]),
                "bisection_msms": int(out[5]), "blocks_indexed": int(out[6]),
                "blocks_located": int(out[7])}

    # -- commitment checks (cpz_ctx_set_commitment_checks) ------------------------------------
    def set_commitment_checks(self, enable: bool) -> None:
        """The context's mode.  On (default): statuses 4 / 5 for identity commitments and zero s,
        the rejections of Proof::from_bytes (gadgets.rs:474-482).  Off: the equations alone
        decide, as verify_one (batch.rs:185-231) does for a Proof built with Proof::new.  The
        mode applies to every later call on this context from any thread; for one call alone
        pass equations_only=True to verify_each / verify_batch / verify_response."""
        _native.check(self._lib.cpz_ctx_set_commitment_checks(self._h, 1 if enable else 0))

    # -- host-buffer entry points ---------------------------------------------------------
    def verify_each(self, y1, y2, r1, r2, s, contexts=None, params: Optional[Parameters] = None,
                    equations_only: bool = False) -> np.ndarray:
        """Status per proof (uint8[n]) for (n, 32) byte arrays.  cpz_verify_each_ex;
        equations_only: commitment checks off for this call (CPZ_CALL_EQUATIONS_ONLY)."""
        params = params or Parameters()
        n = len(y1)
        arrs = [_rows(a, n, nm) for a, nm in ((y1, "y1"), (y2, "y2"), (r1, "r1"), (r2, "r2"), (s, "s"))]
        blob, off, present = _ctx_arrays(contexts, n)
        out = np.empty(n, dtype=np.uint8)
        _native.check(self._lib.cpz_verify_each_ex(
            self._h, _flags(equations_only), params.g, params.h, n, *[_ptr(a) for a in arrs], _ptr(blob), _ptr(off),
            _ptr(present), _ptr(out)))
        return out

    def challenges(self, y1, y2, r1, r2, contexts=None, params: Optional[Parameters] = None) -> np.ndarray:
        params = params or Parameters()
        n = len(y1)
        arrs = [_rows(a, n, nm) for a, nm in ((y1, "y1"), (y2, "y2"), (r1, "r1"), (r2, "r2"))]
        blob, off, present = _ctx_arrays(contexts, n)
        out = np.empty((n, 32), dtype=np.uint8)
        _native.check(self._lib.cpz_challenges(
            self._h, params.g, params.h, n, *[_ptr(a) for a in arrs], _ptr(blob), _ptr(off), _ptr(present),
            _ptr(out)))
        return out

    def verify_response(self, y1, y2, r1, r2, s, c, params: Optional[Parameters] = None,
                        equations_only: bool = False) -> np.ndarray:
        """Status per proof with caller-supplied challenges c ((n, 32) canonical scalars):
        Verifier::verify_response (verifier/mod.rs:144-171), cpz_verify_response_ex."""
        params = params or Parameters()
        n = len(y1)
        arrs = [_rows(a, n, nm) for a, nm in ((y1, "y1"), (y2, "y2"), (r1, "r1"), (r2, "r2"), (s, "s"), (c, "c"))]
        out = np.empty(n, dtype=np.uint8)
        _native.check(self._lib.cpz_verify_response_ex(self._h, _flags(equations_only), params.g, params.h, n,
                                                       *[_ptr(a) for a in arrs], _ptr(out)))
        return out

    def prove(self, x, k, contexts=None, params: Optional[Parameters] = None):
        """Proofs from caller witnesses x and nonces k (sequences of ints / 32-byte scalars, or
        (n, 32) arrays): dict of (n, 32) arrays y1, y2, r1, r2, s (cpz_prove)."""
        params = params or Parameters()
        n = len(x)
        xs = x if isinstance(x, np.ndarray) else np.frombuffer(b"".join(_scalar_bytes(v) for v in x), np.uint8)
        ks = k if isinstance(k, np.ndarray) else np.frombuffer(b"".join(_scalar_bytes(v) for v in k), np.uint8)
        xs, ks = _rows(xs, n, "x"), _rows(ks, n, "k")
        outs = {q: np.empty((n, 32), dtype=np.uint8) for q in ("y1", "y2", "r1", "r2", "s")}
        blob, off, present = _ctx_arrays(contexts, n)
        _native.check(self._lib.cpz_prove(self._h, params.g, params.h, n, _ptr(xs), _ptr(ks), _ptr(blob), _ptr(off),
                                          _ptr(present), *[_ptr(outs[q]) for q in ("y1", "y2", "r1", "r2", "s")]))
        return outs

    def decode_points(self, points):
        """Bulk element_from_bytes + element_to_bytes (cpz_decode_points): (ok uint8[n],
        re-encodings uint8[n, 32], zero where a point does not decode)."""
        n = len(points)
        arr = _rows(np.frombuffer(b"".join(bytes(p) for p in points), np.uint8) if not isinstance(points, np.ndarray)
                    else points, n, "points")
        ok = np.empty(n, dtype=np.uint8)
        enc = np.empty((n, 32), dtype=np.uint8)
        _native.check(self._lib.cpz_decode_points(self._h, n, _ptr(arr), _ptr(ok), _ptr(enc)))
        return ok, enc

    def verify_batch(self, y1, y2, r1, r2, s, seed: bytes, first_index: int = 0, contexts=None,
                     params: Optional[Parameters] = None, statuses: bool = True, equations_only: bool = False):
        """RLC batch check (cpz_verify_batch_ex).  Returns (partial: bytes, batch_ok: bool,
        status: uint8[n] or None).  With statuses=True a failing batch runs the fallback
        search and status holds the exact per-entry outcome."""
        params = params or Parameters()
        n = len(y1)
        arrs = [_rows(a, n, nm) for a, nm in ((y1, "y1"), (y2, "y2"), (r1, "r1"), (r2, "r2"), (s, "s"))]
        blob, off, present = _ctx_arrays(contexts, n)
        partial = ctypes.create_string_buffer(32)
        ok = ctypes.c_int(0)
        out = np.empty(n, dtype=np.uint8) if statuses else None
        _native.check(self._lib.cpz_verify_batch_ex(
            self._h, _flags(equations_only), params.g, params.h, n, *[_ptr(a) for a in arrs], _ptr(blob), _ptr(off),
            _ptr(present), bytes(seed), first_index, partial, ctypes.byref(ok), _ptr(out)))
        return partial.raw, bool(ok.value), out

    def verify_batch_device(self, y1, y2, r1, r2, s, status_out, seed: bytes, first_index: int = 0,
                            fallback: bool = False, params: Optional[Parameters] = None,
                            stream: Optional[int] = None, ctx_bytes=None, ctx_off=None, ctx_present=None):
        """Device-resident RLC batch check; returns (partial, batch_ok); fills status_out.
        Contexts, if any, are device tensors: bytes (uint8), n + 1 offsets (int64), n flags."""
        params = params or Parameters()
        partial = ctypes.create_string_buffer(32)
        ok = ctypes.c_int(0)
        dp = lambda t: None if t is None else t.data_ptr()
        _native.check(self._lib.cpz_verify_batch_device(
            self._h, params.g, params.h, int(y1.shape[0]), y1.data_ptr(), y2.data_ptr(), r1.data_ptr(),
            r2.data_ptr(), s.data_ptr(), dp(ctx_bytes), dp(ctx_off), dp(ctx_present), bytes(seed), first_index,
            partial, ctypes.byref(ok), status_out.data_ptr(), 1 if fallback else 0, _torch_stream(stream)))
        return partial.raw, bool(ok.value)

    def parse_proofs(self, blobs: Sequence[bytes]):
        """Bulk Proof::from_bytes on the device (cpz_parse_proofs): returns (r1, r2, s) as
        uint8[n, 32] rows (zero where not parsed), codes uint8[n] (CPZ_PARSE_*, 0 = ok) and
        aux uint32[n] (the value printed by the reference's message); parse_error(code, aux)
        gives the exception."""
        n = len(blobs)
        lens = np.fromiter((len(b) for b in blobs), dtype=np.uint64, count=n)
        off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        blob = np.frombuffer(b"".join(bytes(b) for b in blobs) + b"\0", dtype=np.uint8)
        rows = [np.empty((n, 32), dtype=np.uint8) for _ in range(3)]
        codes = np.empty(n, dtype=np.uint8)
        aux = np.empty(n, dtype=np.uint32)
        _native.check(self._lib.cpz_parse_proofs(self._h, n, _ptr(blob), _ptr(off), *[_ptr(r) for r in rows],
                                                 _ptr(codes), _ptr(aux)))
        return rows[0], rows[1], rows[2], codes, aux

    def parse_proofs_device(self, blob, off, r1, r2, s, codes, aux=None, stream: Optional[int] = None) -> None:
        """Device form: blob (uint8 tensor), off (int64/uint64 tensor of n + 1 offsets), row
        outputs uint8[n, 32], codes uint8[n], aux int32/uint32[n] or None."""
        n = int(off.numel()) - 1
        dp = lambda t: None if t is None else t.data_ptr()
        _native.check(self._lib.cpz_parse_proofs_device(
            self._h, n, dp(blob), dp(off), dp(r1), dp(r2), dp(s), dp(codes), dp(aux), _torch_stream(stream)))

    def msm(self, points: Sequence[bytes], scalars: Sequence[int]) -> bytes:
        """enc(sum [k_j] P_j) through the Pippenger kernels (cpz_msm)."""
        pb = b"".join(bytes(p) for p in points)
        sb = b"".join(int(k).to_bytes(32, "little") for k in scalars)
        out = ctypes.create_string_buffer(32)
        _native.check(self._lib.cpz_msm(self._h, len(points), pb, sb, out))
        return out.raw

    def combine_partials(self, partials: Sequence[bytes]):
        """(sum encoding, is_identity) of per-shard partials (cpz_combine_partials)."""
        blob = b"".join(bytes(p) for p in partials)
        out = ctypes.create_string_buffer(32)
        ident = ctypes.c_int(0)
        _native.check(self._lib.cpz_combine_partials(self._h, len(partials), blob, out, ctypes.byref(ident)))
        return out.raw, bool(ident.value)

    def prove_synthetic(self, n: int, seed_x: bytes, seed_k: bytes, first_index: int = 0, contexts=None,
                        params: Optional[Parameters] = None):
        """Synthetic proofs from ChaCha20-derived witnesses: dict of (n, 32) arrays."""
        params = params or Parameters()
        outs = {k: np.empty((n, 32), dtype=np.uint8) for k in ("y1", "y2", "r1", "r2", "s")}
        blob, off, present = _ctx_arrays(contexts, n)
        _native.check(self._lib.cpz_prove_synthetic(
            self._h, params.g, params.h, n, first_index, bytes(seed_x), bytes(seed_k), _ptr(blob), _ptr(off),
            _ptr(present), *[_ptr(outs[k]) for k in ("y1", "y2", "r1", "r2", "s")]))
        return outs

    # -- device-resident entry points (torch tensors on this GPU) ---------------------------
    def verify_each_device(self, y1, y2, r1, r2, s, status_out, params: Optional[Parameters] = None,
                           stream: Optional[int] = None, ctx_bytes=None, ctx_off=None, ctx_present=None) -> None:
        """Enqueue verification of device tensors (uint8, (n, 32), 16-B aligned) on `stream`."""
        params = params or Parameters()
        n = int(y1.shape[0])
        dp = lambda t: None if t is None else t.data_ptr()
        _native.check(self._lib.cpz_verify_each_device(
            self._h, params.g, params.h, n, dp(y1), dp(y2), dp(r1), dp(r2), dp(s), dp(ctx_bytes), dp(ctx_off),
            dp(ctx_present), dp(status_out), _torch_stream(stream)))

    def verify_response_device(self, y1, y2, r1, r2, s, c, status_out, params: Optional[Parameters] = None,
                               stream: Optional[int] = None) -> None:
        """Enqueue verify_response of device tensors (uint8 (n, 32) rows, challenges c)."""
        params = params or Parameters()
        _native.check(self._lib.cpz_verify_response_device(
            self._h, params.g, params.h, int(y1.shape[0]), y1.data_ptr(), y2.data_ptr(), r1.data_ptr(), r2.data_ptr(),
            s.data_ptr(), c.data_ptr(), status_out.data_ptr(), _torch_stream(stream)))

    def prove_device(self, x, k, y1, y2, r1, r2, s, params: Optional[Parameters] = None, stream: Optional[int] = None,
                     ctx_bytes=None, ctx_off=None, ctx_present=None) -> None:
        """Enqueue the prover on device tensors: witnesses x, nonces k ((n, 32) uint8) -> rows."""
        params = params or Parameters()
        dp = lambda t: None if t is None else t.data_ptr()
        _native.check(self._lib.cpz_prove_device(
            self._h, params.g, params.h, int(x.shape[0]), x.data_ptr(), k.data_ptr(), dp(ctx_bytes), dp(ctx_off),
            dp(ctx_present), y1.data_ptr(), y2.data_ptr(), r1.data_ptr(), r2.data_ptr(), s.data_ptr(),
            _torch_stream(stream)))

    def prove_synthetic_device(self, n: int, seed_x: bytes, seed_k: bytes, y1, y2, r1, r2, s, first_index: int = 0,
                               params: Optional[Parameters] = None, stream: Optional[int] = None,
                               ctx_bytes=None, ctx_off=None, ctx_present=None) -> None:
        params = params or Parameters()
        dp = lambda t: None if t is None else t.data_ptr()
        _native.check(self._lib.cpz_prove_synthetic_device(
            self._h, params.g, params.h, n, first_index, bytes(seed_x), bytes(seed_k), dp(ctx_bytes), dp(ctx_off),
            dp(ctx_present), y1.data_ptr(), y2.data_ptr(), r1.data_ptr(), r2.data_ptr(), s.data_ptr(),
            _torch_stream(stream)))


def _ctx_list(gpus: Sequence[Gpu]):
    if not gpus:
        raise InvalidParams("no GPU contexts")
    return (ctypes.c_void_p * len(gpus))(*[g._h.value for g in gpus])


def verify_each_multi(gpus: Sequence[Gpu], y1, y2, r1, r2, s, contexts=None,
                      params: Optional[Parameters] = None) -> np.ndarray:
    """Per-proof statuses with the proofs sharded over several contexts (one per GPU, in
    shard order; cpz_verify_each_multi, one host thread per shard)."""
    params = params or Parameters()
    n = len(y1)
    arrs = [_rows(a, n, nm) for a, nm in ((y1, "y1"), (y2, "y2"), (r1, "r1"), (r2, "r2"), (s, "s"))]
    blob, off, present = _ctx_arrays(contexts, n)
    out = np.empty(n, dtype=np.uint8)
    lib = gpus[0]._lib if gpus else _native.load()
    _native.check(lib.cpz_verify_each_multi(_ctx_list(gpus), len(gpus), params.g, params.h, n,
                                            *[_ptr(a) for a in arrs], _ptr(blob), _ptr(off), _ptr(present), _ptr(out)))
    return out


def verify_batch_multi(gpus: Sequence[Gpu], y1, y2, r1, r2, s, seed: bytes, contexts=None,
                       params: Optional[Parameters] = None, statuses: bool = True):
    """RLC batch check sharded over several contexts (cpz_verify_batch_multi).  Returns
    (partials: [bytes] per shard, total: bytes, batch_ok: bool, status: uint8[n] or None)."""
    params = params or Parameters()
    n = len(y1)
    arrs = [_rows(a, n, nm) for a, nm in ((y1, "y1"), (y2, "y2"), (r1, "r1"), (r2, "r2"), (s, "s"))]
    blob, off, present = _ctx_arrays(contexts, n)
    k = len(gpus)
    parts = ctypes.create_string_buffer(32 * max(k, 1))
    total = ctypes.create_string_buffer(32)
    ok = ctypes.c_int(0)
    out = np.empty(n, dtype=np.uint8) if statuses else None
    lib = gpus[0]._lib if gpus else _native.load()
    _native.check(lib.cpz_verify_batch_multi(_ctx_list(gpus), k, params.g, params.h, n, *[_ptr(a) for a in arrs],
                                             _ptr(blob), _ptr(off), _ptr(present), bytes(seed), parts, total,
                                             ctypes.byref(ok), _ptr(out)))
    return [parts.raw[32 * i:32 * i + 32] for i in range(k)], total.raw, bool(ok.value), out


_default_gpu: Optional[Gpu] = None


def _gpu() -> Gpu:
    global _default_gpu
    if _default_gpu is None:
        _default_gpu = Gpu(0)
    return _default_gpu


class Transcript:
    """Mirror of `Transcript` (transcript.rs:25-72) as far as callers shape it: new() plus an
    optional `append_context` (transcript.rs:42-44, once; the protocol appends parameters,
    statement and commitment itself).  The sponge runs on the device."""

    def __init__(self):
        self.context: Optional[bytes] = None

    @classmethod
    def new(cls) -> "Transcript":
        return cls()

    def append_context(self, context: bytes) -> None:
        if self.context is not None:
            raise InvalidParams("the device transcript takes one context per proof")
        self.context = bytes(context)


_VALID_STATEMENTS: "dict" = {}   # (y1, y2) -> decodes; a registered user's statement repeats


def _validate_statement(gpu: Gpu, statement: "Statement") -> None:
    """Statement::validate (gadgets.rs:234-238 -> ristretto.rs:173-185): both elements must be
    group elements -- here, both encodings must decode (device decode, cpz_decode_points).
    A Rust Statement holds decoded points, so its validate() cannot fail; bytes can.
    Statements already seen to decode are remembered (bounded), so a batch of one user's
    proofs costs one device call."""
    key = (statement.y1, statement.y2)
    if key not in _VALID_STATEMENTS:
        ok, _ = gpu.decode_points(np.frombuffer(statement.y1 + statement.y2, np.uint8).reshape(2, 32))
        if not ok.all():
            raise InvalidGroupElement("Element failed recompression validation")
        if len(_VALID_STATEMENTS) >= 4096:
            _VALID_STATEMENTS.clear()
        _VALID_STATEMENTS[key] = True


def _raise_status(st: int) -> None:
    if st != STATUS_OK:
        raise VerifyResult(st).error()


class Verifier:
    """Mirror of `Verifier` (verifier/mod.rs:42-172): one statement, one proof at a time
    (each call is a 1-entry device call; batches belong in BatchVerifier / Gpu)."""

    def __init__(self, params: Parameters, statement: Statement, gpu: Optional[Gpu] = None):
        self.params, self.statement, self._gpu = params, statement, gpu

    def verify(self, proof: Proof) -> None:
        """verifier/mod.rs:85-88: a fresh transcript."""
        self.verify_with_transcript(proof, Transcript.new())

    def verify_with_transcript(self, proof: Proof, transcript: Transcript) -> None:
        """verifier/mod.rs:120-139; raises the reference's error, returns None on Ok(())."""
        g = self._gpu or _gpu()
        _validate_statement(g, self.statement)  # verifier/mod.rs:121
        one = lambda b: np.frombuffer(b, np.uint8).reshape(1, 32)
        # a Proof value: the equations only (verifier/mod.rs:144-171), for this call alone
        st = g.verify_each(one(self.statement.y1), one(self.statement.y2), one(proof.r1), one(proof.r2),
                           one(proof.s), contexts=[transcript.context], params=self.params, equations_only=True)
        _raise_status(int(st[0]))

    def verify_response(self, challenge, proof: Proof) -> None:
        """verifier/mod.rs:144-171: the caller's challenge (int mod l or 32 canonical bytes)."""
        g = self._gpu or _gpu()
        one = lambda b: np.frombuffer(b, np.uint8).reshape(1, 32)
        st = g.verify_response(one(self.statement.y1), one(self.statement.y2), one(proof.r1), one(proof.r2),
                               one(proof.s), one(_scalar_bytes(challenge)), params=self.params, equations_only=True)
        _raise_status(int(st[0]))


class Prover:
    """Mirror of `Prover` (prover/mod.rs:25-132) for one witness x; the point arithmetic
    and the transcript run on the device (cpz_prove)."""

    def __init__(self, params: Parameters, witness, gpu: Optional[Gpu] = None):
        self.params, self._x, self._gpu = params, _scalar_bytes(witness), gpu

    def statement(self) -> Statement:
        return Statement.from_witness(self.params, self._x, self._gpu)

    @staticmethod
    def _random_nonce(rng=None) -> bytes:
        import os
        raw = rng.randbytes(64) if rng is not None else os.urandom(64)
        return _scalar_bytes(int.from_bytes(raw, "little"))   # random_scalar: wide reduction

    def prove(self, rng=None) -> Proof:
        """prover/mod.rs:70-84: a fresh transcript."""
        return self.prove_with_transcript(rng, Transcript.new())

    def prove_with_transcript(self, rng, transcript: Transcript, nonce=None) -> Proof:
        """prover/mod.rs:86-110 (commit, transcript challenge, respond); `nonce` fixes k."""
        k = _scalar_bytes(nonce) if nonce is not None else self._random_nonce(rng)
        out = (self._gpu or _gpu()).prove([self._x], [k], contexts=[transcript.context], params=self.params)
        return Proof(out["r1"][0].tobytes(), out["r2"][0].tobytes(), out["s"][0].tobytes())

    def commit(self, rng=None, nonce=None):
        """prover/mod.rs:115-121: ((r1, r2), k) with r = (k g, k h)."""
        k = _scalar_bytes(nonce) if nonce is not None else self._random_nonce(rng)
        out = (self._gpu or _gpu()).prove([self._x], [k], params=self.params)
        return (out["r1"][0].tobytes(), out["r2"][0].tobytes()), k

    def respond(self, nonce, challenge) -> bytes:
        """prover/mod.rs:126-131: s = k + c x (mod l), scalar arithmetic only."""
        k = int.from_bytes(_scalar_bytes(nonce), "little")
        c = int.from_bytes(_scalar_bytes(challenge), "little")
        x = int.from_bytes(self._x, "little")
        return ((k + c * x) % L).to_bytes(32, "little")


class _Entry:
    __slots__ = ("params", "statement", "proof", "context")

    def __init__(self, params, statement, proof, context):
        self.params, self.statement, self.proof, self.context = params, statement, proof, context


class BatchVerifier:
    """Mirror of `verifier::batch::BatchVerifier` (batch.rs:82-324).

    Same cap (MAX_BATCH_SIZE, batch.rs:48, 151-156), same empty-batch error
    (batch.rs:172-176), results in entry order.  `verify` returns one VerifyResult per
    entry: exactly what the reference returns, because its n >= 2 batch equation falls
    back to per-entry verification and its n == 1 path is verify_one.
    """

    def __init__(self, gpu: Optional[Gpu] = None, capacity: int = 0):
        self._entries: List[_Entry] = []
        self._gpu = gpu
        self.capacity = min(int(capacity), MAX_BATCH_SIZE)   # batch.rs:113-118 (a reservation only)

    @classmethod
    def new(cls) -> "BatchVerifier":
        return cls()

    @classmethod
    def with_capacity(cls, capacity: int, gpu: Optional[Gpu] = None) -> "BatchVerifier":
        """batch.rs:113-118: capacity.min(MAX_BATCH_SIZE) reserved; no effect on results."""
        return cls(gpu, capacity)

    def len(self) -> int:
        return len(self._entries)

    __len__ = len

    def is_empty(self) -> bool:
        return not self._entries

    def remaining_capacity(self) -> int:
        return max(0, MAX_BATCH_SIZE - len(self._entries))

    def add(self, params: Parameters, statement: Statement, proof: Proof) -> None:
        self.add_with_context(params, statement, proof, None)

    def add_with_context(self, params: Parameters, statement: Statement, proof: Proof,
                         context: Optional[bytes]) -> None:
        if len(self._entries) >= MAX_BATCH_SIZE:
            raise InvalidParams("Batch size limit exceeded (max %d)" % MAX_BATCH_SIZE)
        _validate_statement(self._gpu or _gpu(), statement)   # batch.rs:158
        self._entries.append(_Entry(params, statement, proof, None if context is None else bytes(context)))

    def clear(self) -> None:
        self._entries.clear()

    def verify(self, rng=None, rlc_min_group: Optional[int] = None) -> List[VerifyResult]:
        """batch.rs:171-183, through the call sequence of the Rust drop-in
        (rust/reference-patch/gpu.rs; C++ mirror: include/cpz_batch.hpp): entries grouped by
        Parameters in order of first appearance; groups take consecutive weight indices, and a
        group of at least rlc_min_group entries (default RLC_MIN_GROUP) runs the RLC batch check
        with its exact fallback (cpz_verify_batch), a smaller one cpz_verify_each.

        `rng` is drawn exactly as the reference draws it: nothing for a one-entry batch
        (verify_one, batch.rs:178-180), otherwise one 64-byte random_scalar per entry
        (batch.rs:239-240), whatever entry point each group takes -- so a caller that keeps
        using a seeded rng sees the reference's stream.  The first draw's first 32 bytes key
        the RLC weights, so `rng` must be a CSPRNG (the reference requires CryptoRngCore):
        secrets.SystemRandom(), or None for os.urandom.  A predictable rng would let forgeries
        be built whose weighted errors cancel.  Only one such source is detected -- a
        random.Random (other than SystemRandom) is refused whenever a group takes the RLC
        check; any other caller-supplied rng is trusted to be a CSPRNG, as the reference's
        CryptoRngCore bound trusts its implementors.  A one-entry batch's RLC check (threshold lowered to 1) is
        keyed by os.urandom.  Entries are `Proof` values, which may have been built with
        Proof(...) (Proof::new: no identity / zero-s checks), so every call is equations-only:
        verify_one's equations alone decide (batch.rs:185-231).  Either entry point returns
        exactly verify_one's outcome per entry."""
        import os
        import random
        if not self._entries:
            raise InvalidParams("Cannot verify empty batch")
        gpu = self._gpu or _gpu()
        rlc_min = RLC_MIN_GROUP if rlc_min_group is None else int(rlc_min_group)
        status = np.empty(len(self._entries), dtype=np.uint8)
        groups = {}   # insertion order = order of first appearance
        for i, e in enumerate(self._entries):
            groups.setdefault((e.params.g, e.params.h), []).append(i)
        n = len(self._entries)
        uses_rlc = any(len(idx) >= rlc_min for idx in groups.values())
        if uses_rlc and n > 1 and isinstance(rng, random.Random) and not isinstance(rng, random.SystemRandom):
            raise InvalidParams("BatchVerifier.verify: the RLC weights need a cryptographic rng "
                                "(secrets.SystemRandom() or None), not random.Random")
        seed = None
        if n > 1:   # one random_scalar (64 bytes) per entry, batch.rs:239-240
            draws = [(rng.randbytes(64) if rng is not None else os.urandom(64)) for _ in range(n)]
            seed = draws[0][:32]
        elif uses_rlc:
            seed = os.urandom(32)
        first_index = 0
        for (g, h), idx in groups.items():
            ents = [self._entries[i] for i in idx]
            rows = [np.frombuffer(b"".join(getattr(e.statement if q in ("y1", "y2") else e.proof, q) for e in ents),
                                  np.uint8).reshape(-1, 32) for q in ("y1", "y2", "r1", "r2", "s")]
            ctxs = [e.context for e in ents]
            if len(idx) >= rlc_min:
                _, _, st = gpu.verify_batch(*rows, seed, first_index=first_index, contexts=ctxs,
                                            params=Parameters(g, h), equations_only=True)
            else:
                st = gpu.verify_each(*rows, contexts=ctxs, params=Parameters(g, h), equations_only=True)
            first_index += len(idx)
            status[np.array(idx)] = st
        return [VerifyResult(s) for s in status]
