"""The service's batch authentication path (service.rs:407-616) over the bulk entry points.

CPU test: the host logic (request checks, per-entry check order, challenge consumption,
error messages, result / session order) with an oracle-backed stand-in for the two bulk
calls (test infrastructure: the oracle is the checker here, never the product path).
GPU test: the same scenario through cpz_parse_proofs + cpz_verify_each on the device.
"""
import hashlib

import numpy as np
import pytest

import pyoracle as O


class OracleBulk:
    """parse_proofs / verify_each with the Gpu methods' signatures, computed by the oracle."""

    def parse_proofs(self, blobs):
        n = len(blobs)
        rows = [np.zeros((n, 32), np.uint8) for _ in range(3)]
        codes = np.zeros(n, np.uint8)
        aux = np.zeros(n, np.uint32)
        for i, b in enumerate(blobs):
            code, a = O.proof_from_bytes_code(bytes(b))
            codes[i], aux[i] = code, a
            if code == 0:
                for q in range(3):
                    off = 1 + 4 + q * 36
                    rows[q][i] = np.frombuffer(bytes(b)[off:off + 32], np.uint8)
        return rows[0], rows[1], rows[2], codes, aux

    def verify_each(self, y1, y2, r1, r2, s, contexts=None, params=None):
        return np.array([O.verify_one(O.ProofRecord(bytes(y1[i]), bytes(y2[i]), bytes(r1[i]), bytes(r2[i]),
                                                    bytes(s[i]), contexts[i]))
                         for i in range(len(y1))], np.uint8)


def _scenario():
    """Six users, one request of 12 entries exercising every per-entry outcome."""
    from chaum_pedersen.service import MemoryState
    st = MemoryState()
    users, xs = [], []
    for u in range(6):
        x = O.scalar_wide(hashlib.sha512(b"svc-x%d" % u).digest())
        rec = O.prove(x, 7)
        uid = "user_%d" % u
        st.register_user(uid, rec.y1, rec.y2)
        users.append(uid)
        xs.append(x)
    cid = [hashlib.sha256(b"cid%d" % i).digest() for i in range(12)]

    def proof_for(u, c, forge=False):
        k = O.scalar_wide(hashlib.sha512(b"svc-k" + c).digest())
        rec = O.prove(xs[u], k, ctx=c)
        s = (int.from_bytes(rec.s, "little") + (1 if forge else 0)) % O.L
        return O.proof_to_bytes(rec.r1, rec.r2, s.to_bytes(32, "little"))

    uids, cids, proofs, expect = [], [], [], []

    def add(uid, c, proof, exp, issue=True, owner=None):
        if issue:
            st.create_challenge(owner or uid, c)
        uids.append(uid)
        cids.append(c)
        proofs.append(proof)
        expect.append(exp)

    ok = "User '%s' authenticated successfully"
    add(users[0], cid[0], proof_for(0, cid[0]), (True, ok % users[0]))
    add(users[1], cid[1], proof_for(1, cid[1], forge=True), (False, "Authentication failed"))
    add("bad user!", cid[2], proof_for(2, cid[2]), (False, "User ID contains invalid characters"), issue=False)
    add(users[2], b"", proof_for(2, cid[2]), (False, "Empty challenge ID for proof 3"), issue=False)
    add(users[3], cid[4], proof_for(3, cid[4]), (False, "Authentication failed"), issue=False)  # never issued
    add(users[3], cid[5], proof_for(3, cid[5]), (False, "Authentication failed"), owner=users[4])  # someone else's
    p = bytearray(proof_for(4, cid[6]))
    p[0] = 2
    add(users[4], cid[6], bytes(p), (False, "Invalid proof: Invalid group parameters: Unsupported proof version: 2"))
    add(users[5], cid[7], proof_for(5, cid[7]) + b"\0\0", (False, "Invalid proof: Invalid group parameters: "
                                                                     "Proof has 2 trailing bytes"))
    add(users[5], cid[8], proof_for(5, cid[9]), (False, "Authentication failed"))  # proof bound to another context
    add(users[2], cid[10], b"\x01" * 9000, (False, "Proof 9 too large"))
    add(users[2], cid[11], proof_for(2, cid[11]), (True, ok % users[2]))
    add(users[0], cid[3], proof_for(0, cid[3]), (True, ok % users[0]))
    return st, uids, cids, proofs, expect


def _check(results, st, uids, expect):
    from chaum_pedersen.service import VerificationResult
    assert [(r.success, r.message) for r in results] == expect
    toks = [r.session_token for r in results if r.success]
    assert all(isinstance(t, str) and len(t) == 64 for t in toks)
    assert all(r.session_token is None for r in results if not r.success)
    # sessions issued in entry order, to the right users
    assert [st.sessions[t] for t in toks] == [u for u, e in zip(uids, expect) if e[0]]
    # every issued challenge that reached consume_challenge is gone (single use), including
    # the ones whose proof then failed to parse or verify
    assert not st.challenges


def test_service_batch_host_logic():
    from chaum_pedersen.service import InvalidArgument, verify_proof_batch
    st, uids, cids, proofs, expect = _scenario()
    # entry 9's challenge is issued but its proof is rejected by the size check before
    # consume_challenge (service.rs:466-468), so it stays; drop it before the final check
    res = verify_proof_batch(st, uids, cids, proofs, gpu=OracleBulk())
    assert cids[9] in st.challenges
    del st.challenges[cids[9]]
    _check(res, st, uids, expect)
    with pytest.raises(InvalidArgument, match="Empty batch"):
        verify_proof_batch(st, [], [], [], gpu=OracleBulk())
    with pytest.raises(InvalidArgument, match="Mismatched array lengths"):
        verify_proof_batch(st, ["a"], [b"x", b"y"], [b"p"], gpu=OracleBulk())
    with pytest.raises(InvalidArgument, match="maximum limit of 1000"):
        verify_proof_batch(st, ["a"] * 1001, [b"x"] * 1001, [b"p"] * 1001, gpu=OracleBulk())


def test_service_session_cap_and_replay():
    """A replayed challenge fails (consumed on first use); the per-user session cap turns
    an accepted proof into "Failed to create session: ..." (state.rs:252-276)."""
    from chaum_pedersen.service import MemoryState, verify_proof_batch
    st = MemoryState(max_sessions_per_user=1)
    x = 12345
    rec0 = O.prove(x, 1)
    st.register_user("alice", rec0.y1, rec0.y2)
    c1, c2 = b"\x11" * 32, b"\x22" * 32
    st.create_challenge("alice", c1)
    st.create_challenge("alice", c2)
    p1 = O.prove(x, 99, ctx=c1)
    p2 = O.prove(x, 98, ctx=c2)
    blobs = [O.proof_to_bytes(p.r1, p.r2, p.s) for p in (p1, p2)]
    res = verify_proof_batch(st, ["alice", "alice", "alice"], [c1, c2, c1], blobs + [blobs[0]], gpu=OracleBulk())
    assert [(r.success, r.message) for r in res] == [
        (True, "User 'alice' authenticated successfully"),
        (False, "Failed to create session: Invalid group parameters: User 'alice' has reached maximum session "
                "limit (1)"),
        (False, "Authentication failed")]


@pytest.mark.gpu
def test_service_batch_gpu(gpu):
    from chaum_pedersen.service import verify_proof_batch
    st, uids, cids, proofs, expect = _scenario()
    res = verify_proof_batch(st, uids, cids, proofs, gpu=gpu)
    del st.challenges[cids[9]]
    _check(res, st, uids, expect)
