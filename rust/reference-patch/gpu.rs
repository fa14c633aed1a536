//! Reference-side change (kobby-pentangeli/chaum-pedersen-zkp): `BatchVerifier::verify`
//! (src/verifier/batch.rs:171-183) served by the MI355X verifier when the crate is built with
//! its `gpu` feature.  This file is `src/verifier/batch/gpu.rs`, a child module of `batch` (so
//! it sees the private `entries` / `BatchEntry` and `verify_cpu`); `dispatch.rs` next to it
//! holds the public `verify` with the reference's exact signature, so no caller changes
//! (service.rs:529-540, examples/batch_verification.rs:46, benches/batch_verification.rs:33).
//! The three edits to the reference are listed in dispatch.rs.
//!
//! What the GPU computes, per `Parameters` group of entries (groups in order of first
//! appearance):
//!   * a group of fewer than RLC_MIN_GROUP entries -- every group of this API's batches (at
//!     most 1000 entries), from the measured latencies -- runs cpz_verify_each: `verify_one`
//!     per entry (batch.rs:185-231): up to 512 proofs one proof per six-wave workgroup with
//!     its field products on 16-lane rows (k_verify_wide), up to 2048 three waves per 8
//!     proofs (k_verify_small);
//!   * a larger group takes the random-linear-combination check (cpz_verify_batch: the batch
//!     equation with the weights on every term, one Pippenger MSM), keyed by the first 32
//!     bytes `rng` yields -- or, for a one-entry batch, which the reference verifies with
//!     `verify_one` without touching `rng` (batch.rs:178-180), by 32 bytes from the OS
//!     (`OsRng`); a failing check runs the fallback search, which returns exactly
//!     `verify_one`'s outcome per entry (verify_individually, batch.rs:262-268, 314-318).
//!     Groups take consecutive weight indices (`first_index`).
//! `rng` is drawn exactly as the reference draws it, whatever entry point each group takes:
//! nothing for n == 1, one `random_scalar` -- 64 bytes, one `fill_bytes` call -- per entry for
//! n >= 2 (batch.rs:239-240, ristretto.rs:146-150), so a caller that keeps using a seeded rng
//! after `verify` sees the same stream as with the reference.
//! Every call passes EQUATIONS_ONLY: a `Proof` may have been built with `Proof::new` (no
//! identity / zero-s checks, gadgets.rs:252, 278, 317), and `verify_one` judges it by the
//! two equations alone -- so the result vector is the reference's for every batch, not only
//! for proofs that came through `Proof::from_bytes`.  The flag is per call: other users of
//! the library's contexts keep their own mode.
//!
//! Contexts: a pool of CONTEXTS_PER_DEVICE contexts on every visible GPU.  Each `verify`
//! checks one out for its duration (a free one, round-robin over the devices), so concurrent
//! callers -- the service's handlers, service.rs:529-540 -- run side by side on every GPU
//! instead of queueing on one context of GPU 0.  A context keeps the tables of its 4 most
//! recently used (g, h) pairs, so batches whose groups alternate Parameters rebuild nothing.
//!
//! The C++ mirror of this call sequence (include/cpz_batch.hpp, BatchVerifier::verify) is
//! what tests/test_gpu_dropin.py runs on the GPU against the oracle.
//!
//! Host work per entry is the four compressions the C ABI's 32-byte rows need (y1, y2, r1,
//! r2) and one scalar copy; g and h are compressed once per group (entries are grouped by
//! `Element` equality, no compression), and the compressions are spread over scoped threads
//! for large batches.  No `unsafe` appears here, so the crate keeps `#![forbid(unsafe_code)]`
//! (src/lib.rs:64): the FFI lives in chaum-pedersen-gpu / chaum-pedersen-gpu-sys, whose
//! build.rs runs hipcc (the crate's own build.rs:1-12 keeps running tonic-build only).
use std::sync::atomic::{AtomicUsize, Ordering};
use std::sync::{Mutex, MutexGuard, OnceLock, TryLockError};

use chaum_pedersen_gpu::{device_count, Entry, EntryError, Gpu, EQUATIONS_ONLY};
use rand_core::{CryptoRngCore, OsRng, RngCore};

use super::{BatchEntry, BatchVerifier};
use crate::{Element, Error, Parameters, Ristretto255, Result};

/// Contexts per visible GPU: two batches in flight on one GPU overlap one's latency-bound
/// MSM tails with the other's VALU-bound work (1.06-1.075x one at a time, BENCH_r03
/// rlc.two_in_flight).
const CONTEXTS_PER_DEVICE: usize = 2;

/// Smallest `Parameters` group sent to the RLC batch check; smaller groups are verified per
/// proof (cpz_verify_each).  Both return `verify_one`'s outcome; the threshold only picks the
/// faster entry point at the batch sizes this API carries (n <= 1000, batch.rs:48), from the
/// per-call latency table of bench.py's small_batch (profiles/r05_bench_i.json): per proof
/// 0.112-0.118 ms at n = 1 .. 100 (k_verify_wide) and 0.265 ms at 1000 (k_verify_small), the
/// RLC check 0.54-0.59 ms at n <= 100 and 0.73 ms at 1000, so no group of this API (at most
/// 1000 entries, batch.rs:48) takes the RLC check; the path stays for callers that lower it.
const RLC_MIN_GROUP: usize = 1001;

/// The process's verifier contexts (see above).
struct Pool {
    slots: Vec<Mutex<Gpu>>,
    next: AtomicUsize,
}

impl Pool {
    /// A free context, searched round-robin from a shared cursor (consecutive slots are on
    /// different GPUs); when every context is busy, the cursor's own slot, waited for.
    fn checkout(&self) -> MutexGuard<'_, Gpu> {
        let n = self.slots.len();
        let start = self.next.fetch_add(1, Ordering::Relaxed);
        for k in 0..n {
            match self.slots[(start + k) % n].try_lock() {
                Ok(g) => return g,
                Err(TryLockError::Poisoned(p)) => return p.into_inner(),
                Err(TryLockError::WouldBlock) => {}
            }
        }
        self.slots[start % n].lock().unwrap_or_else(|p| p.into_inner())
    }
}

/// Contexts on every visible GPU that opens; a device whose context fails to open is skipped
/// (its error kept for the message), so one bad GPU does not take `verify` down on the healthy
/// ones.  Fails only when no context opens at all.
fn pool() -> Result<&'static Pool> {
    static POOL: OnceLock<std::result::Result<Pool, String>> = OnceLock::new();
    POOL.get_or_init(|| {
        let devices = device_count();
        if devices == 0 {
            return Err("no GPU visible to the HIP runtime".to_string());
        }
        let mut slots = Vec::with_capacity(devices * CONTEXTS_PER_DEVICE);
        let mut last_err = String::new();
        for _ in 0..CONTEXTS_PER_DEVICE {
            for d in 0..devices {
                match Gpu::new(d) {
                    Ok(g) => slots.push(Mutex::new(g)),
                    Err(e) => last_err = format!("GPU {d}: {e}"),
                }
            }
        }
        if slots.is_empty() {
            return Err(format!("no verifier context could be opened ({last_err})"));
        }
        Ok(Pool { slots, next: AtomicUsize::new(0) })
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
    let gpu = pool()?.checkout();
    let mut groups: Vec<Group<'_>> = Vec::new();
    for (i, e) in entries.iter().enumerate() {
        let (g, h) = (e.params.generator_g(), e.params.generator_h());
        match groups.iter_mut().find(|grp| grp.g == g && grp.h == h) {
            Some(grp) => grp.idx.push(i),
            None => groups.push(Group { g, h, enc: compress_generators(&e.params), idx: vec![i] }),
        }
    }
    let mut out: Vec<Option<Result<()>>> = (0..entries.len()).map(|_| None).collect();
    // The reference's consumption of `rng` (batch.rs:178-180, 239-240), before any GPU work.
    let mut seed = [0u8; 32];
    if entries.len() == 1 {
        OsRng.fill_bytes(&mut seed); // verify_one draws nothing from the caller's rng
    } else {
        let mut draw = [0u8; 64];
        for i in 0..entries.len() {
            rng.fill_bytes(&mut draw); // one random_scalar per entry
            if i == 0 {
                seed.copy_from_slice(&draw[..32]);
            }
        }
    }
    let mut first_index = 0u64;
    for grp in &groups {
        let rows = group_rows(entries, &grp.idx);
        let (g, h) = &grp.enc;
        let status = if rows.len() < RLC_MIN_GROUP {
            gpu.verify_each_with(EQUATIONS_ONLY, g, h, &rows).map_err(|e| Error::InvalidParams(e.to_string()))?
        } else {
            let (_partial, _ok, st) = gpu
                .verify_batch_with(EQUATIONS_ONLY, g, h, &rows, &seed, first_index)
                .map_err(|e| Error::InvalidParams(e.to_string()))?;
            st
        };
        first_index += rows.len() as u64;
        for (k, &i) in grp.idx.iter().enumerate() {
            out[i] = Some(entry_result(status[k]));
        }
    }
    Ok(out.into_iter().map(|r| r.expect("every entry grouped")).collect())
}
