//! Reference-side change (kobby-pentangeli/chaum-pedersen-zkp), part 2 of 2: the public
//! `BatchVerifier::verify` with the reference's exact signature (src/verifier/batch.rs:171),
//! dispatching to the GPU under the `gpu` feature and to the reference's own CPU code
//! otherwise.  Callers -- service.rs:529-540, examples/batch_verification.rs:46, 92,
//! benches/batch_verification.rs:33, 105, 144, the unit tests batch.rs:337-511 -- are unchanged.
//!
//! Edits to the reference (three, none of them in a caller):
//!   1. src/verifier/batch.rs, the existing `verify` (batch.rs:171): rename it to
//!      `verify_cpu` and make it private (its body stays as it is; its doc comment and
//!      doctest move to the `verify` below).
//!   2. src/verifier/batch.rs, after the imports: `mod dispatch;` and
//!      `#[cfg(feature = "gpu")] mod gpu;` -- this file is src/verifier/batch/dispatch.rs,
//!      gpu.rs is src/verifier/batch/gpu.rs.
//!   3. Cargo.toml: `[features] gpu = ["dep:chaum-pedersen-gpu"]` and
//!      `chaum-pedersen-gpu = { path = "<this repo>/rust/chaum-pedersen-gpu", optional = true }`.
//! Without the feature the crate builds and behaves exactly as before.
use rand_core::CryptoRngCore;

use super::BatchVerifier;
use crate::Result;

impl BatchVerifier {
    /// Verifies all proofs in the batch (batch.rs:171-183): `Err` for an empty batch,
    /// otherwise one `Result` per entry in entry order.  With the `gpu` feature the
    /// verification runs on the MI355X (gpu.rs: every `Parameters` group of this API's
    /// batches, at most 1000 entries, is verified per proof, `verify_one` by k_verify_wide
    /// (a six-wave workgroup per proof) or k_verify_small (three waves per 8 proofs); a group of at least RLC_MIN_GROUP entries would take the
    /// random-linear-combination check keyed by `rng`, with an exact per-entry fallback);
    /// the per-entry results are those of `verify_one`, and `rng` is drawn as the reference
    /// draws it (64 bytes per entry for n >= 2, nothing for n == 1).
    pub fn verify<R: CryptoRngCore>(&self, rng: &mut R) -> Result<Vec<Result<()>>> {
        #[cfg(feature = "gpu")]
        {
            super::gpu::verify(self, rng)
        }
        #[cfg(not(feature = "gpu"))]
        {
            self.verify_cpu(rng)
        }
    }
}
