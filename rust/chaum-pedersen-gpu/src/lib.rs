//! Safe wrapper over `chaum-pedersen-gpu-sys` (include/cpz.h).  All `unsafe` of the GPU path
//! lives in this crate, so the reference crate (`#![forbid(unsafe_code)]`, src/lib.rs:64)
//! calls only safe functions.  Points and scalars cross as their 32-byte encodings; every
//! decode and check runs on the device.
#![deny(unsafe_op_in_unsafe_fn)]

use chaum_pedersen_gpu_sys as sys;
use std::ffi::CStr;
use std::os::raw::c_int;
use std::ptr;

/// A 32-byte encoding (compressed ristretto255 point or little-endian scalar).
pub type Bytes32 = [u8; 32];

/// Per-call flags (`CPZ_CALL_*`) of the `*_with` methods: options for that call alone.
pub type CallFlags = u32;
/// Commitment checks off for one call: the equations alone decide, as `verify_one`
/// (batch.rs:185-231) does for a `Proof` value (`CPZ_CALL_EQUATIONS_ONLY`).
pub const EQUATIONS_ONLY: CallFlags = sys::CPZ_CALL_EQUATIONS_ONLY;

/// A device / argument failure of a whole call (`CPZ_E*` code + `cpz_last_error`).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct GpuError {
    pub code: i32,
    pub message: String,
}

impl std::fmt::Display for GpuError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "cpz error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for GpuError {}

fn check(rc: c_int) -> Result<(), GpuError> {
    if rc == sys::CPZ_OK {
        return Ok(());
    }
    // SAFETY: cpz_last_error returns a NUL-terminated thread-local string (never null).
    let msg = unsafe { CStr::from_ptr(sys::cpz_last_error()) }.to_string_lossy().into_owned();
    Err(GpuError { code: rc, message: msg })
}

/// Per-entry outcome kinds with the reference's error variant and message
/// (batch.rs:224-228, ristretto.rs:120-138, ristretto.rs:94-112, gadgets.rs:474-482).
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub enum EntryError {
    /// `InvalidParams("Proof verification failed")`
    VerificationFailed,
    /// `InvalidGroupElement("Bytes do not represent a valid Ristretto point")`
    InvalidGroupElement,
    /// `InvalidScalar("Bytes do not represent a valid scalar")`
    InvalidScalar,
    /// `InvalidParams("Commitment contains identity element")`
    IdentityCommitment,
    /// `InvalidParams("Response scalar is zero")`
    ZeroResponse,
}

impl EntryError {
    /// The status byte of a per-entry result (0 = Ok).
    pub fn from_status(st: u8) -> Option<EntryError> {
        match st {
            sys::CPZ_STATUS_OK => None,
            sys::CPZ_STATUS_EQ_FAIL => Some(EntryError::VerificationFailed),
            sys::CPZ_STATUS_BAD_POINT => Some(EntryError::InvalidGroupElement),
            sys::CPZ_STATUS_BAD_SCALAR => Some(EntryError::InvalidScalar),
            sys::CPZ_STATUS_IDENTITY => Some(EntryError::IdentityCommitment),
            _ => Some(EntryError::ZeroResponse),
        }
    }

    /// The reference's message for this outcome.
    pub fn message(&self) -> &'static str {
        match self {
            EntryError::VerificationFailed => "Proof verification failed",
            EntryError::InvalidGroupElement => "Bytes do not represent a valid Ristretto point",
            EntryError::InvalidScalar => "Bytes do not represent a valid scalar",
            EntryError::IdentityCommitment => "Commitment contains identity element",
            EntryError::ZeroResponse => "Response scalar is zero",
        }
    }
}

/// One batch entry: statement, proof, optional transcript context (batch.rs:51-56).
#[derive(Debug, Clone)]
pub struct Entry<'a> {
    pub y1: Bytes32,
    pub y2: Bytes32,
    pub r1: Bytes32,
    pub r2: Bytes32,
    pub s: Bytes32,
    pub context: Option<&'a [u8]>,
}

/// Structure-of-arrays staging of entries for the C ABI.
struct Soa {
    rows: [Vec<u8>; 5],
    ctx_bytes: Vec<u8>,
    ctx_off: Vec<u64>,
    ctx_present: Vec<u8>,
    any_ctx: bool,
}

impl Soa {
    fn new(entries: &[Entry<'_>]) -> Soa {
        let n = entries.len();
        let mut rows: [Vec<u8>; 5] = Default::default();
        for r in rows.iter_mut() {
            r.reserve(32 * n);
        }
        let mut ctx_bytes = Vec::new();
        let mut ctx_off = Vec::with_capacity(n + 1);
        let mut ctx_present = Vec::with_capacity(n);
        ctx_off.push(0u64);
        let mut any_ctx = false;
        for e in entries {
            for (r, f) in rows.iter_mut().zip([&e.y1, &e.y2, &e.r1, &e.r2, &e.s]) {
                r.extend_from_slice(f);
            }
            if let Some(c) = e.context {
                any_ctx = true;
                ctx_bytes.extend_from_slice(c);
            }
            ctx_present.push(e.context.is_some() as u8);
            ctx_off.push(ctx_bytes.len() as u64);
        }
        if ctx_bytes.is_empty() {
            ctx_bytes.push(0);
        }
        Soa { rows, ctx_bytes, ctx_off, ctx_present, any_ctx }
    }
    fn ctx_ptrs(&self) -> (*const u8, *const u64, *const u8) {
        if self.any_ctx {
            (self.ctx_bytes.as_ptr(), self.ctx_off.as_ptr(), self.ctx_present.as_ptr())
        } else {
            (ptr::null(), ptr::null(), ptr::null())
        }
    }
}

/// A verifier context on one GPU (`cpz_ctx`).  The C side serialises concurrent calls on
/// one context, so it may be shared between threads.
pub struct Gpu {
    ctx: *mut sys::cpz_ctx,
}

// SAFETY: every entry point locks the context's mutex on the C side.
unsafe impl Send for Gpu {}
unsafe impl Sync for Gpu {}

impl Drop for Gpu {
    fn drop(&mut self) {
        // SAFETY: ctx came from cpz_ctx_create and is destroyed once.
        unsafe { sys::cpz_ctx_destroy(self.ctx) }
    }
}

/// `Ristretto255::generator_g` / `generator_h` encodings (ristretto.rs:79-91).
pub fn default_generators() -> (Bytes32, Bytes32) {
    let (mut g, mut h) = ([0u8; 32], [0u8; 32]);
    // SAFETY: two writable 32-byte buffers.
    unsafe { sys::cpz_default_generators(g.as_mut_ptr(), h.as_mut_ptr()) };
    (g, h)
}

/// Number of GPUs the HIP runtime sees.
pub fn device_count() -> usize {
    // SAFETY: no arguments.
    unsafe { sys::cpz_device_count() }.max(0) as usize
}

impl Gpu {
    /// A context on GPU `device`.  Refuses a library built against another `cpz.h`
    /// (`cpz_abi_version`), so no entry point is called with wrongly sized buffers.
    pub fn new(device: usize) -> Result<Gpu, GpuError> {
        // SAFETY: no arguments.
        let abi = unsafe { sys::cpz_abi_version() };
        if abi != sys::CPZ_ABI_VERSION {
            return Err(GpuError {
                code: sys::CPZ_EINVAL,
                message: format!("libcpz ABI {} but these bindings follow {}", abi, sys::CPZ_ABI_VERSION),
            });
        }
        let mut ctx = ptr::null_mut();
        // SAFETY: out-pointer to a local.
        check(unsafe { sys::cpz_ctx_create(device as c_int, &mut ctx) })?;
        Ok(Gpu { ctx })
    }

    /// Commitment checks (`cpz_ctx_set_commitment_checks`): on (the default) reports identity
    /// commitments and zero s as `Proof::from_bytes` would (gadgets.rs:474-482); off lets the
    /// two equations alone decide, as `verify_one` (batch.rs:185-231) does for a `Proof`
    /// built with `Proof::new` -- what a `BatchVerifier` holds.  This is the context's mode
    /// for every later call from any thread; `EQUATIONS_ONLY` on a `*_with` call is the same
    /// for that call alone.
    pub fn set_commitment_checks(&self, enable: bool) -> Result<(), GpuError> {
        // SAFETY: ctx is live; the C side locks it.
        check(unsafe { sys::cpz_ctx_set_commitment_checks(self.ctx, enable as c_int) })
    }

    /// Per-entry statuses of `BatchVerifier::verify` (batch.rs:171-231) for any n.
    pub fn verify_each(&self, g: &Bytes32, h: &Bytes32, entries: &[Entry<'_>]) -> Result<Vec<u8>, GpuError> {
        self.verify_each_with(0, g, h, entries)
    }

    /// `verify_each` with per-call flags (`cpz_verify_each_ex`).
    pub fn verify_each_with(&self, flags: CallFlags, g: &Bytes32, h: &Bytes32, entries: &[Entry<'_>])
                            -> Result<Vec<u8>, GpuError> {
        let soa = Soa::new(entries);
        let (cb, co, cp) = soa.ctx_ptrs();
        let mut st = vec![0u8; entries.len()];
        let r = &soa.rows;
        // SAFETY: every row holds 32 * n bytes; contexts hold n + 1 offsets / n flags.
        check(unsafe {
            sys::cpz_verify_each_ex(self.ctx, flags, g.as_ptr(), h.as_ptr(), entries.len(), r[0].as_ptr(),
                                    r[1].as_ptr(), r[2].as_ptr(), r[3].as_ptr(), r[4].as_ptr(), cb, co, cp,
                                    st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// `Verifier::verify_response` (verifier/mod.rs:144-171) with caller challenges.
    pub fn verify_response(&self, g: &Bytes32, h: &Bytes32, entries: &[Entry<'_>], challenges: &[Bytes32])
                           -> Result<Vec<u8>, GpuError> {
        self.verify_response_with(0, g, h, entries, challenges)
    }

    /// `verify_response` with per-call flags (`cpz_verify_response_ex`).
    pub fn verify_response_with(&self, flags: CallFlags, g: &Bytes32, h: &Bytes32, entries: &[Entry<'_>],
                                challenges: &[Bytes32]) -> Result<Vec<u8>, GpuError> {
        assert_eq!(entries.len(), challenges.len());
        let soa = Soa::new(entries);
        let c: Vec<u8> = challenges.iter().flatten().copied().collect();
        let mut st = vec![0u8; entries.len()];
        let r = &soa.rows;
        // SAFETY: as verify_each; c holds 32 * n bytes.
        check(unsafe {
            sys::cpz_verify_response_ex(self.ctx, flags, g.as_ptr(), h.as_ptr(), entries.len(), r[0].as_ptr(),
                                        r[1].as_ptr(), r[2].as_ptr(), r[3].as_ptr(), r[4].as_ptr(), c.as_ptr(),
                                        st.as_mut_ptr())
        })?;
        Ok(st)
    }

    /// Random-linear-combination batch check (corrected `verify_batch_equations`,
    /// batch.rs:271-312) with exact per-entry statuses on failure (verify_individually,
    /// batch.rs:314-318).  Returns (partial encoding, batch_ok, statuses).
    pub fn verify_batch(&self, g: &Bytes32, h: &Bytes32, entries: &[Entry<'_>], seed: &Bytes32, first_index: u64)
                        -> Result<(Bytes32, bool, Vec<u8>), GpuError> {
        self.verify_batch_with(0, g, h, entries, seed, first_index)
    }

    /// `verify_batch` with per-call flags (`cpz_verify_batch_ex`).
    pub fn verify_batch_with(&self, flags: CallFlags, g: &Bytes32, h: &Bytes32, entries: &[Entry<'_>], seed: &Bytes32,
                             first_index: u64) -> Result<(Bytes32, bool, Vec<u8>), GpuError> {
        let soa = Soa::new(entries);
        let (cb, co, cp) = soa.ctx_ptrs();
        let mut partial = [0u8; 32];
        let mut ok: c_int = 0;
        let mut st = vec![0u8; entries.len()];
        let r = &soa.rows;
        // SAFETY: as verify_each; partial holds 32 bytes, ok is a local.
        check(unsafe {
            sys::cpz_verify_batch_ex(self.ctx, flags, g.as_ptr(), h.as_ptr(), entries.len(), r[0].as_ptr(),
                                     r[1].as_ptr(), r[2].as_ptr(), r[3].as_ptr(), r[4].as_ptr(), cb, co, cp,
                                     seed.as_ptr(), first_index, partial.as_mut_ptr(), &mut ok, st.as_mut_ptr())
        })?;
        Ok((partial, ok != 0, st))
    }

    /// Proofs from witnesses x and nonces k (prover/mod.rs:86-131): (y1, y2, r1, r2, s) each.
    pub fn prove(&self, g: &Bytes32, h: &Bytes32, x: &[Bytes32], k: &[Bytes32], contexts: &[Option<&[u8]>])
                 -> Result<Vec<[Bytes32; 5]>, GpuError> {
        let n = x.len();
        assert!(k.len() == n && contexts.len() == n);
        let xs: Vec<u8> = x.iter().flatten().copied().collect();
        let ks: Vec<u8> = k.iter().flatten().copied().collect();
        let entries: Vec<Entry<'_>> = contexts
            .iter()
            .map(|c| Entry { y1: [0; 32], y2: [0; 32], r1: [0; 32], r2: [0; 32], s: [0; 32], context: *c })
            .collect();
        let soa = Soa::new(&entries);
        let (cb, co, cp) = soa.ctx_ptrs();
        let mut out: [Vec<u8>; 5] = Default::default();
        for o in out.iter_mut() {
            o.resize(32 * n, 0);
        }
        let [o0, o1, o2, o3, o4] = &mut out;
        // SAFETY: inputs hold 32 * n bytes; outputs are 32 * n writable bytes each.
        check(unsafe {
            sys::cpz_prove(self.ctx, g.as_ptr(), h.as_ptr(), n, xs.as_ptr(), ks.as_ptr(), cb, co, cp, o0.as_mut_ptr(),
                           o1.as_mut_ptr(), o2.as_mut_ptr(), o3.as_mut_ptr(), o4.as_mut_ptr())
        })?;
        Ok((0..n)
            .map(|i| {
                let mut p = [[0u8; 32]; 5];
                for (q, o) in out.iter().enumerate() {
                    p[q].copy_from_slice(&o[32 * i..32 * i + 32]);
                }
                p
            })
            .collect())
    }

    /// `Proof::from_bytes` (gadgets.rs:364-489) for many blobs: ((r1, r2, s), code, aux) per
    /// blob; code != 0 names the reference's error (CPZ_PARSE_*), aux the value it prints.
    pub fn parse_proofs(&self, blobs: &[&[u8]]) -> Result<Vec<([Bytes32; 3], u8, u32)>, GpuError> {
        let n = blobs.len();
        let mut blob = Vec::new();
        let mut off = vec![0u64];
        for b in blobs {
            blob.extend_from_slice(b);
            off.push(blob.len() as u64);
        }
        blob.push(0);
        let mut rows: [Vec<u8>; 3] = [vec![0; 32 * n], vec![0; 32 * n], vec![0; 32 * n]];
        let (mut code, mut aux) = (vec![0u8; n], vec![0u32; n]);
        let [a, b, c] = &mut rows;
        // SAFETY: n + 1 offsets into blob; outputs sized n.
        check(unsafe {
            sys::cpz_parse_proofs(self.ctx, n, blob.as_ptr(), off.as_ptr(), a.as_mut_ptr(), b.as_mut_ptr(),
                                  c.as_mut_ptr(), code.as_mut_ptr(), aux.as_mut_ptr())
        })?;
        Ok((0..n)
            .map(|i| {
                let mut f = [[0u8; 32]; 3];
                for (q, r) in rows.iter().enumerate() {
                    f[q].copy_from_slice(&r[32 * i..32 * i + 32]);
                }
                (f, code[i], aux[i])
            })
            .collect())
    }
}
