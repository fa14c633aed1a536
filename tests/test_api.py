"""Host-side mirror of the reference interface (chaum_pedersen package), no GPU needed:
the 109-byte wire format (gadgets.rs:343-489 and its tests :555-652), Parameters
validation (gadgets.rs:77-103, tests :500-519) and the BatchVerifier's cap / empty /
bookkeeping behaviour (batch.rs:97-183, 321-323, tests :337-342, :464-511)."""
import pytest

import chaum_pedersen as cp

R1 = bytes.fromhex("e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76")
R2 = bytes.fromhex("6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919")
S = bytes(range(32))[:31] + b"\x01"


def test_proof_wire_roundtrip():
    p = cp.Proof(R1, R2, S)
    b = p.to_bytes()
    assert len(b) == 109 and b[0] == cp.PROTOCOL_VERSION
    assert b[1:5] == b"\x00\x00\x00\x20" and b[5:37] == R1 and b[41:73] == R2 and b[77:109] == S
    q = cp.Proof.from_bytes(b)
    assert (q.r1, q.r2, q.s, q.version) == (R1, R2, S, 1)


@pytest.mark.parametrize("data", [b"", bytes([1, 0, 0, 0]), bytes([0x00]), b"\xff" * 10, b"\x01" * 1000])
def test_from_bytes_rejects_malformed(data):
    with pytest.raises(cp.Error):
        cp.Proof.from_bytes(data)


def test_from_bytes_rejections():
    good = cp.Proof(R1, R2, S).to_bytes()
    with pytest.raises(cp.InvalidParams):          # wrong version (gadgets.rs:587-594)
        cp.Proof.from_bytes(bytes([99]) + good[1:])
    with pytest.raises(cp.InvalidParams):          # zero-length fields (:596-602)
        cp.Proof.from_bytes(bytes([1, 0, 0, 0, 0]) + good[5:])
    with pytest.raises(cp.InvalidParams):          # excessive length (:604-610)
        cp.Proof.from_bytes(bytes([1, 0xFF, 0xFF, 0xFF, 0xFF]) + good[5:])
    with pytest.raises(cp.InvalidParams):          # trailing data (:612-633)
        cp.Proof.from_bytes(good + b"\xff")
    with pytest.raises(cp.InvalidParams):          # truncated
        cp.Proof.from_bytes(good[:100])


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


def test_batch_bookkeeping_without_device():
    b = cp.BatchVerifier.new()
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
    """The committed wire fixtures agree with the oracle's from_bytes (structural Python mirror too)."""
    import pyoracle as O
    for w in golden["wire"]:
        b = bytes.fromhex(w["blob"])
        assert O.proof_from_bytes_code(b) == (w["code"], w["aux"])
        struct_codes = {1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 13, 14, 15, 16, 18}
        if w["code"] in struct_codes:
            with pytest.raises(cp.Error) as exc:
                cp.Proof.from_bytes(b)
            ref = cp.parse_error(w["code"], w["aux"])
            assert type(exc.value) is type(ref) and str(exc.value) == str(ref)
