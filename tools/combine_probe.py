"""Synchronous cpz_combine_partials latency at k = 1, 8, 64 partials (valid: the identity; and a
non-identity sum), median of 200 calls; run under rocprofv3 --kernel-trace for k_rlc_combine's
own duration (tools/gpu_r06_o.sh)."""
import json
import os
import statistics
import sys
import time

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "chaum-pedersen-zkp_amd"), os.path.join(root, "oracle")]
import pyoracle as O  # noqa: E402  (inputs only)
from chaum_pedersen import Gpu  # noqa: E402

gpu = Gpu(0)
rows = []
for k in (1, 8, 64):
    pts = [O.pt_mul(O.BASEPOINT, O.bench_scalar(b"combine", i)) for i in range(k)]
    enc = [O.ristretto_encode(p) for p in pts]
    acc = pts[0]
    for p in pts[1:]:
        acc = O.pt_add(acc, p)
    ident_set = enc[:-1] + [O.ristretto_encode(O.pt_neg(O.pt_add(acc, O.pt_neg(pts[-1]))))] if k > 1 else [bytes(32)]
    for name, parts in (("identity", ident_set), ("non_identity", enc)):
        for _ in range(20):
            gpu.combine_partials(parts)
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            out = gpu.combine_partials(parts)
            ts.append(time.perf_counter() - t0)
        rows.append({"k": k, "set": name, "identity": out[1], "median_ms": statistics.median(ts) * 1e3})
print(json.dumps({"combine_partials": rows}))
