"""The reference service's batch authentication (`AuthServiceImpl::verify_proof_batch`,
src/verifier/service.rs:407-616) over the GPU bulk path.

What the reference does per request, in order, and what this module keeps:

* request checks (service.rs:419-433): empty batch, mismatched array lengths, more than
  1000 entries -> the whole request fails (`InvalidArgument`, same messages);
* per entry, in entry order (service.rs:443-526): user-id / challenge-id / proof-size
  validation (service.rs:37-56, 446-470), `consume_challenge` (the challenge is consumed
  even when a later check fails), challenge owner == user, `get_user`, `Proof::from_bytes`
  ("Invalid proof: {e}"), then `add_with_context(Parameters::new(), statement, proof,
  Some(challenge_id))`;
* one `BatchVerifier::verify` over the entries that got that far (service.rs:528-540);
  its per-entry results are verify_one's, which is what `cpz_verify_each`
  computes, with the 32-byte challenge ids as transcript contexts (the fixed-schedule
  challenge kernel);
* results in entry order (service.rs:545-608): a session token (32 random bytes, hex)
  created per accepted entry in that order, "Authentication failed" for a rejected proof,
  the validation message otherwise.

The GPU work is two bulk calls per request: `cpz_parse_proofs` over every proof blob
(side-effect free, so it may run before the per-entry checks without changing which
challenges get consumed) and `cpz_verify_each` over the surviving entries.  Rate limiting,
metrics and gRPC framing (service.rs:411-413, counters/histograms) are control plane and
stay out; `state` is any object with the reference state's four calls (`MemoryState` below
is a minimal in-memory one for tests and examples).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import Error, InvalidGroupElement, InvalidParams, InvalidScalar, Parameters, parse_error

MAX_BATCH_REQUEST = 1000       # service.rs:429
MAX_CHALLENGE_ID_LEN = 64      # service.rs:456
MAX_PROOF_BYTES = 8192         # service.rs:467
MAX_USER_ID_LEN = 256          # service.rs:42


class InvalidArgument(Exception):
    """`Status::invalid_argument` for the whole request (service.rs:419-433)."""

    code = "INVALID_ARGUMENT"


class AlreadyExists(Exception):
    """`Status::already_exists`: the user id is taken (service.rs:108-112)."""

    code = "ALREADY_EXISTS"


@dataclass
class VerificationResult:
    """proto `VerificationResult` (proto/auth.proto): one per request entry."""
    success: bool
    message: str
    session_token: Optional[str] = None


def error_display(e: Error) -> str:
    """`Display` of the reference's `Error` (src/error.rs:5-17, thiserror formats)."""
    prefix = {InvalidParams: "Invalid group parameters: ", InvalidScalar: "Invalid scalar: ",
              InvalidGroupElement: "Invalid group element: "}
    for cls, p in prefix.items():
        if isinstance(e, cls):
            return p + str(e)
    return str(e)


def validate_user_id(user_id: str) -> Optional[str]:
    """service.rs:37-56 (length in UTF-8 bytes, as Rust's `str::len`)."""
    if not user_id:
        return "User ID cannot be empty"
    if len(user_id.encode("utf-8")) > MAX_USER_ID_LEN:
        return "User ID too long"
    if not all(c.isalnum() or c in "_-." for c in user_id):
        return "User ID contains invalid characters"
    return None


def _validate_entry(i: int, user_id: str, challenge_id: bytes, proof: bytes) -> Optional[str]:
    """service.rs:443-472."""
    msg = validate_user_id(user_id)
    if msg:
        return msg
    if len(challenge_id) == 0:
        return "Empty challenge ID for proof %d" % i
    if len(challenge_id) > MAX_CHALLENGE_ID_LEN:
        return "Challenge ID too long for proof %d" % i
    if len(proof) == 0:
        return "Empty proof %d" % i
    if len(proof) > MAX_PROOF_BYTES:
        return "Proof %d too large" % i
    return None


class MemoryState:
    """Minimal stand-in for `ServerState` (src/verifier/state.rs): users, single-use
    challenges with an expiry, sessions with the per-user cap.  Only what the batch path
    calls: consume_challenge (state.rs:204-230), get_user (:158-161), create_session
    (:252-276)."""

    def __init__(self, max_sessions_per_user: int = 5, clock: Callable[[], float] = time.time):
        self.users: Dict[str, Tuple[bytes, bytes]] = {}
        self.challenges: Dict[bytes, Tuple[str, float]] = {}
        self.sessions: Dict[str, str] = {}
        self.user_sessions: Dict[str, List[str]] = {}
        self.max_sessions_per_user = max_sessions_per_user
        self.clock = clock

    def register_user(self, user_id: str, y1: bytes, y2: bytes) -> None:
        """state.rs:136-157 (the state's own checks only).  Requests go through `register`,
        which validates the statement first as the handler does (service.rs:61-97)."""
        if user_id in self.users:
            raise InvalidParams("User '%s' already registered" % user_id)
        self.users[user_id] = (bytes(y1), bytes(y2))

    def create_challenge(self, user_id: str, challenge_id: bytes, ttl_s: float = 300.0) -> None:
        if user_id not in self.users:
            raise InvalidParams("User '%s' not found" % user_id)
        self.challenges[bytes(challenge_id)] = (user_id, self.clock() + ttl_s)

    def consume_challenge(self, challenge_id: bytes) -> str:
        """The challenge's user id; the challenge is removed (single use) either way."""
        rec = self.challenges.pop(bytes(challenge_id), None)
        if rec is None or self.clock() >= rec[1]:
            raise InvalidParams("Invalid or expired challenge")
        return rec[0]

    def get_user(self, user_id: str) -> Optional[Tuple[bytes, bytes]]:
        return self.users.get(user_id)

    def create_session(self, token: str, user_id: str) -> None:
        toks = self.user_sessions.setdefault(user_id, [])
        if len(toks) >= self.max_sessions_per_user:
            raise InvalidParams("User '%s' has reached maximum session limit (%d)"
                                % (user_id, self.max_sessions_per_user))
        self.sessions[token] = user_id
        toks.append(token)


MAX_STATEMENT_BYTES = 4096     # service.rs:78


def register(state, user_id: str, y1: bytes, y2: bytes, gpu=None) -> None:
    """The `register` handler (service.rs:61-131) minus rate limiting and metrics: user id
    checks, sizes, element_from_bytes of y1 and y2 (on the device, cpz_decode_points),
    identity statements rejected, then state.register_user.  Raises InvalidArgument with
    the reference's status message, or AlreadyExists ("Registration failed: ...",
    service.rs:108-112) for a taken id."""
    msg = validate_user_id(user_id)
    if msg:
        raise InvalidArgument(msg)
    y1, y2 = bytes(y1), bytes(y2)
    if not y1 or not y2:
        raise InvalidArgument("Empty y1 or y2 values")
    if len(y1) > MAX_STATEMENT_BYTES or len(y2) > MAX_STATEMENT_BYTES:
        raise InvalidArgument("y1 or y2 values too large")
    from . import _gpu
    pts = [p for p in (y1, y2) if len(p) == 32]
    ok = (gpu or _gpu()).decode_points(pts)[0] if pts else []
    j = 0
    for name, v in (("y1", y1), ("y2", y2)):
        if len(v) != 32:
            raise InvalidArgument("Invalid %s: %s" % (name, error_display(
                InvalidGroupElement("Expected 32 bytes, got %d" % len(v)))))
        if not ok[j]:
            raise InvalidArgument("Invalid %s: %s" % (name, error_display(
                InvalidGroupElement("Bytes do not represent a valid Ristretto point"))))
        j += 1
    if y1 == bytes(32) or y2 == bytes(32):   # the identity's (only) encoding
        raise InvalidArgument("Statement contains identity elements")
    try:
        state.register_user(user_id, y1, y2)
    except Error as e:
        raise AlreadyExists("Registration failed: %s" % error_display(e))


def verify_proof_batch(state, user_ids: Sequence[str], challenge_ids: Sequence[bytes], proofs: Sequence[bytes],
                       gpu=None, token_bytes: Callable[[int], bytes] = os.urandom,
                       params: Optional[Parameters] = None) -> List[VerificationResult]:
    """service.rs:407-616 with the verification on the GPU.  Raises InvalidArgument for
    request-level errors; otherwise one VerificationResult per entry, in entry order."""
    n = len(user_ids)
    if n == 0:
        raise InvalidArgument("Empty batch")
    if n != len(challenge_ids) or n != len(proofs):
        raise InvalidArgument("Mismatched array lengths in batch request")
    if n > MAX_BATCH_REQUEST:
        raise InvalidArgument("Batch size exceeds maximum limit of 1000")
    if gpu is None:
        from . import _gpu
        gpu = _gpu()
    params = params or Parameters()

    # Proof::from_bytes for every blob in one device pass; blobs the size checks reject
    # never reach the parser in the reference, so they are parsed as empty here.
    blobs = [bytes(p) if 0 < len(p) <= MAX_PROOF_BYTES else b"" for p in proofs]
    r1, r2, s, codes, aux = gpu.parse_proofs(blobs)

    entries: List[Tuple] = []      # ("err", message) or ("ok", user_id, slot)
    take: List[int] = []
    stmts: List[Tuple[bytes, bytes]] = []
    ctxs: List[bytes] = []
    for i in range(n):
        user_id, cid, proof = user_ids[i], bytes(challenge_ids[i]), proofs[i]
        msg = _validate_entry(i, user_id, cid, proof)
        if msg:
            entries.append(("err", msg))
            continue
        try:
            owner = state.consume_challenge(cid)
        except Exception:
            entries.append(("err", "Authentication failed"))
            continue
        if owner != user_id:
            entries.append(("err", "Authentication failed"))
            continue
        stmt = state.get_user(user_id)
        if stmt is None:
            entries.append(("err", "Authentication failed"))
            continue
        if codes[i]:
            entries.append(("err", "Invalid proof: " + error_display(parse_error(int(codes[i]), int(aux[i])))))
            continue
        # add_with_context (batch.rs:144-168): the capacity is the request size (<= 1000) and
        # registered statements were validated at registration, so it cannot fail here.
        entries.append(("ok", user_id, len(take)))
        take.append(i)
        stmts.append(stmt)
        ctxs.append(cid)

    status = None
    if take:
        idx = np.asarray(take, dtype=np.int64)
        y1 = np.frombuffer(b"".join(t[0] for t in stmts), np.uint8).reshape(-1, 32)
        y2 = np.frombuffer(b"".join(t[1] for t in stmts), np.uint8).reshape(-1, 32)
        status = gpu.verify_each(y1, y2, r1[idx], r2[idx], s[idx], contexts=ctxs, params=params)

    results: List[VerificationResult] = []
    for e in entries:
        if e[0] == "err":
            results.append(VerificationResult(False, e[1], None))
            continue
        user_id, slot = e[1], e[2]
        if int(status[slot]) != 0:
            results.append(VerificationResult(False, "Authentication failed", None))
            continue
        token = bytes(token_bytes(32)).hex()
        try:
            state.create_session(token, user_id)
        except Error as ex:
            results.append(VerificationResult(False, "Failed to create session: %s" % error_display(ex), None))
            continue
        results.append(VerificationResult(True, "User '%s' authenticated successfully" % user_id, token))
    return results
