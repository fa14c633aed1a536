//! Reference-side change (kobby-pentangeli/chaum-pedersen-zkp): `BatchVerifier::verify`
//! (src/verifier/batch.rs:171-183) served by the MI355X verifier when the crate is built with
//! a `gpu` feature.  Drop this file in as `src/verifier/batch/gpu.rs` (a child module of
//! `batch`, so it sees the private `entries` / `BatchEntry`), add `#[cfg(feature = "gpu")]
//! mod gpu;` to src/verifier/batch.rs, and in Cargo.toml:
//!
//!     [features]
//!     gpu = ["dep:chaum-pedersen-gpu"]
//!     [dependencies]
//!     chaum-pedersen-gpu = { path = "<this repo>/rust/chaum-pedersen-gpu", optional = true }
//!
//! No `unsafe` appears here, so the crate keeps `#![forbid(unsafe_code)]` (src/lib.rs:64): the
//! FFI lives in chaum-pedersen-gpu / chaum-pedersen-gpu-sys, whose build.rs runs hipcc (the
//! crate's own build.rs:1-12 keeps running tonic-build only).  The result vector equals the
//! reference's for every batch: its n >= 2 equation fails for valid batches and falls back to
//! verify_one per entry; the GPU reports exactly verify_one's outcome per entry.
//! The 1000-entry cap (batch.rs:48, 151-156) is unchanged; `rng` is not consumed.
use std::sync::OnceLock;

use chaum_pedersen_gpu::{EntryError, Entry, Gpu};

use super::BatchVerifier;
use crate::{Error, Ristretto255, Result};

fn gpu() -> Result<&'static Gpu> {
    static GPU: OnceLock<std::result::Result<Gpu, String>> = OnceLock::new();
    GPU.get_or_init(|| Gpu::new(0).map_err(|e| e.to_string()))
        .as_ref()
        .map_err(|e| Error::InvalidParams(e.clone()))
}

fn bytes32(v: Vec<u8>) -> [u8; 32] {
    v.try_into().expect("32-byte encoding")
}

fn entry_result(st: u8) -> Result<()> {
    match EntryError::from_status(st) {
        None => Ok(()),
        Some(e @ (EntryError::VerificationFailed | EntryError::IdentityCommitment | EntryError::ZeroResponse)) => {
            Err(Error::InvalidParams(e.message().to_string()))
        }
        Some(e @ EntryError::InvalidGroupElement) => Err(Error::InvalidGroupElement(e.message().to_string())),
        Some(e @ EntryError::InvalidScalar) => Err(Error::InvalidScalar(e.message().to_string())),
    }
}

impl BatchVerifier {
    /// `verify` (batch.rs:171-183) on the GPU: one bulk call per distinct Parameters.
    pub fn verify_gpu(&self) -> Result<Vec<Result<()>>> {
        if self.entries.is_empty() {
            return Err(Error::InvalidParams("Cannot verify empty batch".to_string()));
        }
        let gpu = gpu()?;
        let mut out: Vec<Option<Result<()>>> = (0..self.entries.len()).map(|_| None).collect();
        let mut groups: Vec<([u8; 32], [u8; 32], Vec<usize>)> = Vec::new();
        for (i, e) in self.entries.iter().enumerate() {
            let g = bytes32(Ristretto255::element_to_bytes(e.params.generator_g()));
            let h = bytes32(Ristretto255::element_to_bytes(e.params.generator_h()));
            match groups.iter_mut().find(|(gg, hh, _)| *gg == g && *hh == h) {
                Some(grp) => grp.2.push(i),
                None => groups.push((g, h, vec![i])),
            }
        }
        for (g, h, idx) in &groups {
            let entries: Vec<Entry<'_>> = idx
                .iter()
                .map(|&i| {
                    let e = &self.entries[i];
                    Entry {
                        y1: bytes32(Ristretto255::element_to_bytes(e.statement.y1())),
                        y2: bytes32(Ristretto255::element_to_bytes(e.statement.y2())),
                        r1: bytes32(Ristretto255::element_to_bytes(e.proof.commitment().r1())),
                        r2: bytes32(Ristretto255::element_to_bytes(e.proof.commitment().r2())),
                        s: bytes32(Ristretto255::scalar_to_bytes(e.proof.response().s())),
                        context: e.transcript_context.as_deref(),
                    }
                })
                .collect();
            let st = gpu.verify_each(g, h, &entries).map_err(|e| Error::InvalidParams(e.to_string()))?;
            for (k, &i) in idx.iter().enumerate() {
                out[i] = Some(entry_result(st[k]));
            }
        }
        Ok(out.into_iter().map(|r| r.expect("every entry grouped")).collect())
    }
}
