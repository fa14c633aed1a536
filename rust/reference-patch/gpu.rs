//! Reference-side change (kobby-pentangeli/chaum-pedersen-zkp): `BatchVerifier::verify`
//! (src/verifier/batch.rs:171-183) served by the MI355X verifier when the crate is built with
//! its `gpu` feature.  This file is `src/verifier/batch/gpu.rs`, a child module of `batch` (so
//! it sees the private `entries` / `BatchEntry` and `verify_cpu`); `dispatch.rs` next to it
//! holds the public `verify` with the reference's exact signature, so no caller changes
//! (service.rs:529-540, examples/batch_verification.rs:46, benches/batch_verification.rs:33).
//! The three edits to the reference are listed in dispatch.rs.
//!
//! What the GPU computes, per `Parameters` group of entries:
//!   * n == 1 (batch.rs:178-180): `verify_one` -- cpz_verify_each; `rng` is not touched,
//!     as in the reference.
//!   * n >= 2 (batch.rs:233-269): a 32-byte seed drawn from `rng` (the reference draws its
//!     weights from it, batch.rs:240) keys the random-linear-combination check
//!     (cpz_verify_batch: the batch equation with the weights on every term, one Pippenger
//!     MSM); a failing batch runs the fallback search, which returns exactly `verify_one`'s
//!     outcome per entry (verify_individually, batch.rs:262-268, 314-318).  Groups share the
//!     seed and take consecutive weight indices (`first_index`).
//! The context runs with commitment checks off: a `Proof` may have been built with
//! `Proof::new` (no identity / zero-s checks, gadgets.rs:252, 278, 317), and `verify_one`
//! judges it by the two equations alone -- so the result vector is the reference's for every
//! batch, not only for proofs that came through `Proof::from_bytes`.
//!
//! Host work per entry is the four compressions the C ABI's 32-byte rows need (y1, y2, r1,
//! r2) and one scalar copy; g and h are compressed once per group (entries are grouped by
//! `Element` equality, no compression), and the compressions are spread over scoped threads
//! for large batches.  No `unsafe` appears here, so the crate keeps `#![forbid(unsafe_code)]`
//! (src/lib.rs:64): the FFI lives in chaum-pedersen-gpu / chaum-pedersen-gpu-sys, whose
//! build.rs runs hipcc (the crate's own build.rs:1-12 keeps running tonic-build only).
use std::sync::OnceLock;

use chaum_pedersen_gpu::{Entry, EntryError, Gpu};
use rand_core::CryptoRngCore;

use super::{BatchEntry, BatchVerifier};
use crate::{Element, Error, Parameters, Ristretto255, Result};

/// The process's verifier context on GPU 0, with commitment checks off (see above).
fn gpu() -> Result<&'static Gpu> {
    static GPU: OnceLock<std::result::Result<Gpu, String>> = OnceLock::new();
    GPU.get_or_init(|| {
        let g = Gpu::new(0).map_err(|e| e.to_string())?;
        g.set_commitment_checks(false).map_err(|e| e.to_string())?;
        Ok(g)
    })
    .as_ref()
    .map_err(|e| Error::InvalidParams(e.clone()))
}

fn bytes32(v: Vec<u8>) -> [u8; 32] {
    v.try_into().expect("32-byte encoding")
}

/// The 32-byte encodings of a group's generators: once per group, never per entry.
fn compress_generators(params: &Parameters) -> ([u8; 32], [u8; 32]) {
    (
        bytes32(Ristretto255::element_to_bytes(params.generator_g())),
        bytes32(Ristretto255::element_to_bytes(params.generator_h())),
    )
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

/// One entry's rows: the statement and commitment compressions the C ABI takes.
fn entry_rows(e: &BatchEntry) -> Entry<'_> {
    Entry {
        y1: bytes32(Ristretto255::element_to_bytes(e.statement.y1())),
        y2: bytes32(Ristretto255::element_to_bytes(e.statement.y2())),
        r1: bytes32(Ristretto255::element_to_bytes(e.proof.commitment().r1())),
        r2: bytes32(Ristretto255::element_to_bytes(e.proof.commitment().r2())),
        s: bytes32(Ristretto255::scalar_to_bytes(e.proof.response().s())),
        context: e.transcript_context.as_deref(),
    }
}

/// The rows of `idx`, compressed on up to `available_parallelism` scoped threads when the
/// group is large enough to pay for them (4 compressions per entry, ~40 us).
fn group_rows<'a>(entries: &'a [BatchEntry], idx: &[usize]) -> Vec<Entry<'a>> {
    const PER_THREAD: usize = 128;
    let threads = std::thread::available_parallelism().map_or(1, |t| t.get()).min(idx.len() / PER_THREAD).max(1);
    if threads == 1 {
        return idx.iter().map(|&i| entry_rows(&entries[i])).collect();
    }
    let chunk = idx.len().div_ceil(threads);
    std::thread::scope(|sc| {
        let parts: Vec<_> = idx
            .chunks(chunk)
            .map(|part| sc.spawn(move || part.iter().map(|&i| entry_rows(&entries[i])).collect::<Vec<_>>()))
            .collect();
        parts.into_iter().flat_map(|h| h.join().expect("compression thread")).collect()
    })
}

/// A group of entries sharing (g, h): the generators as elements (for grouping by
/// `Element` equality) and encodings (for the device), and the entries' positions.
struct Group<'a> {
    g: &'a Element,
    h: &'a Element,
    enc: ([u8; 32], [u8; 32]),
    idx: Vec<usize>,
}

/// `BatchVerifier::verify` (batch.rs:171-183) on the GPU; called by `dispatch::verify`.
pub(super) fn verify<R: CryptoRngCore + ?Sized>(batch: &BatchVerifier, rng: &mut R) -> Result<Vec<Result<()>>> {
    let entries = &batch.entries;
    if entries.is_empty() {
        return Err(Error::InvalidParams("Cannot verify empty batch".to_string()));
    }
    let gpu = gpu()?;
    let mut groups: Vec<Group<'_>> = Vec::new();
    for (i, e) in entries.iter().enumerate() {
        let (g, h) = (e.params.generator_g(), e.params.generator_h());
        match groups.iter_mut().find(|grp| grp.g == g && grp.h == h) {
            Some(grp) => grp.idx.push(i),
            None => groups.push(Group { g, h, enc: compress_generators(&e.params), idx: vec![i] }),
        }
    }
    let mut out: Vec<Option<Result<()>>> = (0..entries.len()).map(|_| None).collect();
    let mut seed: Option<[u8; 32]> = None;
    let mut first_index = 0u64;
    for grp in &groups {
        let rows = group_rows(entries, &grp.idx);
        let (g, h) = &grp.enc;
        let status = if entries.len() == 1 {
            gpu.verify_each(g, h, &rows).map_err(|e| Error::InvalidParams(e.to_string()))?
        } else {
            let seed = seed.get_or_insert_with(|| {
                let mut s = [0u8; 32];
                rng.fill_bytes(&mut s);
                s
            });
            let (_partial, _ok, st) =
                gpu.verify_batch(g, h, &rows, seed, first_index).map_err(|e| Error::InvalidParams(e.to_string()))?;
            first_index += rows.len() as u64;
            st
        };
        for (k, &i) in grp.idx.iter().enumerate() {
            out[i] = Some(entry_result(status[k]));
        }
    }
    Ok(out.into_iter().map(|r| r.expect("every entry grouped")).collect())
}
