#!/usr/bin/env python3
"""Per-call latency of the drop-in's own regime: BatchVerifier batches of n <= 1000
(batch.rs:48) at the reference bench's sizes (benches/batch_verification.rs:12-35), through
both GPU entry points from host buffers, beside the C oracle's single-thread
BatchVerifier::verify.  Prints one JSON object (bench.small_batch_table)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.small_batch_table(stages=True)), flush=True)
