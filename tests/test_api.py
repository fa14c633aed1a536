"""Host-side mirror of the reference interface (chaum_pedersen package), no GPU needed:
the 109-byte wire format (gadgets.rs:343-489 and its tests :555-652), Parameters
validation (gadgets.rs:77-103, tests :500-519) and the BatchVerifier's cap / empty /
bookkeeping behaviour (batch.rs:97-183, 321-323, tests :337-342, :464-511)."""
import pytest

import chaum_pedersen as cp

R1 = bytes.fromhex("e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76")
R2 = bytes.fromhex("6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919")
S = bytes(range(32))[:31] + b"\x01"


def test_proof_wire_layout():
    p = cp.Proof(R1, R2, S)
    b = p.to_bytes()
    assert len(b) == 109 and b[0] == cp.PROTOCOL_VERSION
    assert b[1:5] == b"\x00\x00\x00\x20" and b[5:37] == R1 and b[41:73] == R2 and b[77:109] == S


def test_from_bytes_needs_the_device():
    """Proof.from_bytes runs the device parser (the reference decodes points inside
    from_bytes, gadgets.rs:410-482); without a GPU it fails loudly instead of accepting
    blobs on structure alone."""
    import chaum_pedersen._native as nat
    if nat.load().cpz_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(cp.CpzError):
        cp.Proof.from_bytes(cp.Proof(R1, R2, S).to_bytes())


def test_parameters_validation():
    g, h = cp.default_generators()
    assert cp.Parameters().g == g and cp.Parameters.new().h == h
    with pytest.raises(cp.InvalidParams):
        cp.Parameters.with_generators(bytes(32), g)
    with pytest.raises(cp.InvalidParams):
        cp.Parameters.with_generators(g, bytes(32))
    with pytest.raises(cp.InvalidParams):
        cp.Parameters.with_generators(g, g)
    assert cp.Parameters.with_generators(g, h) == cp.Parameters()


class _DecodeStub:
    """Stands in for the device's bulk decode at add time (statement.validate, batch.rs:158):
    bookkeeping only -- nothing here verifies anything."""

    def __init__(self, ok=True):
        self.ok, self.calls = ok, 0

    def decode_points(self, pts):
        import numpy as np
        self.calls += 1
        return np.full(len(pts), 1 if self.ok else 0, np.uint8), None


def test_add_validates_the_statement():
    """batch.rs:158: add_with_context runs statement.validate(); an undecodable statement is
    refused at add time (InvalidGroupElement), before anything is queued; without a device
    the validation fails loudly."""
    b = cp.BatchVerifier(_DecodeStub(ok=False))
    with pytest.raises(cp.InvalidGroupElement):
        b.add(cp.Parameters(), cp.Statement(R1, R2), cp.Proof(R1, R2, S))
    assert b.is_empty()
    import chaum_pedersen._native as nat
    if nat.load().cpz_device_count() == 0:
        with pytest.raises(cp.CpzError):
            cp.BatchVerifier().add(cp.Parameters(), cp.Statement(bytes(31) + b"\x05", R2), cp.Proof(R1, R2, S))
    assert cp.BatchVerifier.with_capacity(10).capacity == 10
    assert cp.BatchVerifier.with_capacity(10 ** 6).capacity == cp.MAX_BATCH_SIZE   # batch.rs:113-118


def test_batch_bookkeeping_without_device():
    b = cp.BatchVerifier(_DecodeStub())
    assert b.len() == 0 and b.is_empty() and b.remaining_capacity() == cp.MAX_BATCH_SIZE == 1000
    with pytest.raises(cp.InvalidParams):
        b.verify()                                  # empty batch (batch.rs:172-176)
    st = cp.Statement(R1, R2)
    pr = cp.Proof(R1, R2, S)
    for _ in range(cp.MAX_BATCH_SIZE):
        b.add(cp.Parameters(), st, pr)
    assert b.remaining_capacity() == 0 and len(b) == 1000
    with pytest.raises(cp.InvalidParams):
        b.add_with_context(cp.Parameters(), st, pr, b"ctx")
    b.clear()
    assert b.is_empty()


def test_verify_result_mapping():
    assert cp.VerifyResult(0).is_ok() and cp.VerifyResult(0).error() is None
    assert isinstance(cp.VerifyResult(1).error(), cp.InvalidParams)
    assert isinstance(cp.VerifyResult(2).error(), cp.InvalidGroupElement)
    assert isinstance(cp.VerifyResult(3).error(), cp.InvalidScalar)
    assert isinstance(cp.VerifyResult(4).error(), cp.InvalidParams)
    assert str(cp.VerifyResult(4).error()) == "Commitment contains identity element"   # gadgets.rs:474-478
    assert str(cp.VerifyResult(5).error()) == "Response scalar is zero"                # gadgets.rs:480-482
    assert cp.STATUS_IDENTITY == 4 and cp.STATUS_ZERO_S == 5


def test_parse_error_messages():
    """Bulk-parser codes map to the reference's error types and messages (gadgets.rs:364-489)."""
    assert cp.parse_error(0) is None
    assert set(cp.PARSE_ERRORS) == set(range(1, 21))
    e = cp.parse_error(1, 17)
    assert isinstance(e, cp.InvalidParams) and str(e).endswith("Proof too small: 17 bytes")
    assert isinstance(cp.parse_error(7), cp.InvalidGroupElement)
    assert isinstance(cp.parse_error(16, 31), cp.InvalidScalar) and "got 31" in str(cp.parse_error(16, 31))
    assert "Proof has 5 trailing bytes" in str(cp.parse_error(18, 5))


def test_wire_golden_oracle_codes(golden):
    """The committed wire fixtures agree with the oracle's from_bytes, and every code maps to
    an exception of the reference's type."""
    import pyoracle as O
    for w in golden["wire"]:
        b = bytes.fromhex(w["blob"])
        assert O.proof_from_bytes_code(b) == (w["code"], w["aux"])
        if w["code"]:
            assert isinstance(cp.parse_error(w["code"], w["aux"]), cp.Error)


def test_transcript_mirror():
    t = cp.Transcript.new()
    assert t.context is None
    t.append_context(b"challenge-1")
    assert t.context == b"challenge-1"
    with pytest.raises(cp.InvalidParams):
        t.append_context(b"again")


def test_scalar_arguments():
    assert cp._scalar_bytes(cp.L + 5) == (5).to_bytes(32, "little")
    assert cp._scalar_bytes(bytes(range(32))) == bytes(range(32))
    with pytest.raises(cp.InvalidScalar):
        cp._scalar_bytes(b"\x01" * 31)
    # respond (prover/mod.rs:126-131) is scalar arithmetic: s = k + c x mod l
    pv = cp.Prover(cp.Parameters(), 7)
    assert pv.respond(3, 5) == (3 + 5 * 7).to_bytes(32, "little")
    assert pv.respond(cp.L - 1, 1) == (6).to_bytes(32, "little")
