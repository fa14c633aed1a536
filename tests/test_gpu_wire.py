"""Bulk wire-format ingestion: cpz_parse_proofs against the oracle's
Proof::from_bytes (gadgets.rs:364-489) on the golden blobs -- every truncation, bad
versions/lengths/points/scalars, trailing bytes, identity/zero, and doubly-malformed blobs
where the reference's order of checks decides the error -- then parse -> verify end to end."""
import numpy as np
import pytest

import chaum_pedersen as cp

pytestmark = pytest.mark.gpu


def test_parse_golden_blobs(gpu, golden):
    wire = golden["wire"]
    blobs = [bytes.fromhex(w["blob"]) for w in wire]
    r1, r2, s, codes, aux = gpu.parse_proofs(blobs)
    for i, w in enumerate(wire):
        assert (int(codes[i]), int(aux[i])) == (w["code"], w["aux"]), (i, w)
        if w["code"] == 0:
            b = blobs[i]
            assert r1[i].tobytes() == b[5:37] and r2[i].tobytes() == b[41:73] and s[i].tobytes() == b[77:109]
        err = cp.parse_error(int(codes[i]), int(aux[i]))
        assert (err is None) == (w["code"] == 0)


def test_parse_then_verify(gpu, golden):
    """Blobs of the golden proofs parse to the rows the verifier takes; statuses match."""
    ps = [p for p in golden["proofs"] if p["kind"] in ("valid", "s_plus_1", "wrong_statement")][:40]
    blobs = [bytes([1]) + b"".join(len(bytes.fromhex(p[k])).to_bytes(4, "big") + bytes.fromhex(p[k])
                                   for k in ("r1", "r2", "s")) for p in ps]
    r1, r2, s, codes, _ = gpu.parse_proofs(blobs)
    assert not codes.any()
    y1 = np.stack([np.frombuffer(bytes.fromhex(p["y1"]), np.uint8) for p in ps])
    y2 = np.stack([np.frombuffer(bytes.fromhex(p["y2"]), np.uint8) for p in ps])
    ctxs = [None if p["ctx"] is None else bytes.fromhex(p["ctx"]) for p in ps]
    st = gpu.verify_each(y1, y2, r1, r2, s, contexts=ctxs)
    assert list(st) == [p["status"] for p in ps]


def test_parse_device_large(gpu):
    """2^18 synthetic proofs serialised, 1 % corrupted (version byte), parsed on the device."""
    torch = pytest.importorskip("torch")
    import hashlib
    n = 1 << 18
    sx, sk = hashlib.sha256(b"cpz-bench-x").digest(), hashlib.sha256(b"cpz-bench-k").digest()
    rows = gpu.prove_synthetic(n, sx, sk)
    hdr = np.zeros((n, 109), dtype=np.uint8)
    hdr[:, 0] = 1
    for q, k in enumerate(("r1", "r2", "s")):
        o = 1 + 36 * q
        hdr[:, o:o + 4] = np.frombuffer((32).to_bytes(4, "big"), np.uint8)
        hdr[:, o + 4:o + 36] = rows[k]
    bad = np.arange(0, n, 100)
    hdr[bad, 0] = 2
    dev = torch.device("cuda:0")
    blob = torch.from_numpy(hdr.reshape(-1)).to(dev)
    off = torch.arange(0, 109 * (n + 1), 109, dtype=torch.int64, device=dev)
    out = {k: torch.empty((n, 32), dtype=torch.uint8, device=dev) for k in ("r1", "r2", "s")}
    codes = torch.empty(n, dtype=torch.uint8, device=dev)
    aux = torch.empty(n, dtype=torch.int32, device=dev)
    gpu.parse_proofs_device(blob, off, out["r1"], out["r2"], out["s"], codes, aux)
    c = codes.cpu().numpy()
    assert np.array_equal(np.nonzero(c)[0], bad) and set(c[bad].tolist()) == {2}
    good = np.setdiff1d(np.arange(n), bad)
    for k in ("r1", "r2", "s"):
        assert np.array_equal(out[k].cpu().numpy()[good], rows[k][good])
