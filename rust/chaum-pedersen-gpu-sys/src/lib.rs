//! Raw bindings to `include/cpz.h` (libcpz.so: gfx950 HIP kernels + host runtime).
//!
//! Every item mirrors the header one for one (names, argument order, types);
//! `tests/test_rust_shim.py` checks this file against the header mechanically.  Safe
//! wrappers live in the `chaum-pedersen-gpu` crate, so the reference crate can keep
//! `#![forbid(unsafe_code)]` (src/lib.rs:64).
#![allow(non_camel_case_types)]
#![no_std]

use core::ffi::{c_char, c_int, c_void};

pub const CPZ_OK: c_int = 0;
pub const CPZ_EINVAL: c_int = -1;
pub const CPZ_EHIP: c_int = -2;
pub const CPZ_ENOMEM: c_int = -3;
pub const CPZ_EGENERATOR: c_int = -4;
pub const CPZ_EEMPTY: c_int = -5;

pub const CPZ_STATUS_OK: u8 = 0;
pub const CPZ_STATUS_EQ_FAIL: u8 = 1;
pub const CPZ_STATUS_BAD_POINT: u8 = 2;
pub const CPZ_STATUS_BAD_SCALAR: u8 = 3;
pub const CPZ_STATUS_IDENTITY: u8 = 4;
pub const CPZ_STATUS_ZERO_S: u8 = 5;

pub const CPZ_PARSE_OK: u8 = 0;
pub const CPZ_PARSE_TOO_SMALL: u8 = 1;
pub const CPZ_PARSE_BAD_VERSION: u8 = 2;
pub const CPZ_PARSE_R1_LEN_MISSING: u8 = 3;
pub const CPZ_PARSE_R1_LEN_INVALID: u8 = 4;
pub const CPZ_PARSE_R1_TRUNCATED: u8 = 5;
pub const CPZ_PARSE_R1_SIZE: u8 = 6;
pub const CPZ_PARSE_R1_POINT: u8 = 7;
pub const CPZ_PARSE_R2_LEN_MISSING: u8 = 8;
pub const CPZ_PARSE_R2_LEN_INVALID: u8 = 9;
pub const CPZ_PARSE_R2_TRUNCATED: u8 = 10;
pub const CPZ_PARSE_R2_SIZE: u8 = 11;
pub const CPZ_PARSE_R2_POINT: u8 = 12;
pub const CPZ_PARSE_S_LEN_MISSING: u8 = 13;
pub const CPZ_PARSE_S_LEN_INVALID: u8 = 14;
pub const CPZ_PARSE_S_TRUNCATED: u8 = 15;
pub const CPZ_PARSE_S_SIZE: u8 = 16;
pub const CPZ_PARSE_S_SCALAR: u8 = 17;
pub const CPZ_PARSE_TRAILING: u8 = 18;
pub const CPZ_PARSE_IDENTITY: u8 = 19;
pub const CPZ_PARSE_ZERO_S: u8 = 20;

pub const CPZ_NUM_STAGES: usize = 16;
pub const CPZ_ABI_VERSION: c_int = 5;
pub const CPZ_CALL_EQUATIONS_ONLY: u32 = 1;
pub const CPZ_FALLBACK_STATS: usize = 8;
pub const CPZ_FALLBACK_NONE: u64 = 0;
pub const CPZ_FALLBACK_BISECTION: u64 = 1;
pub const CPZ_FALLBACK_PARTITIONED: u64 = 2;
pub const CPZ_FALLBACK_PER_PROOF: u64 = 3;

/// Opaque verifier context (one GPU, its stream, cached generator tables, buffers).
#[repr(C)]
pub struct cpz_ctx {
    _private: [u8; 0],
}

extern "C" {
    pub fn cpz_abi_version() -> c_int;
    pub fn cpz_device_count() -> c_int;
    pub fn cpz_ctx_create(device_ordinal: c_int, out: *mut *mut cpz_ctx) -> c_int;
    pub fn cpz_ctx_destroy(ctx: *mut cpz_ctx);
    pub fn cpz_ctx_set_commitment_checks(ctx: *mut cpz_ctx, enable: c_int) -> c_int;
    pub fn cpz_ctx_fallback_stats(ctx: *mut cpz_ctx, out: *mut u64) -> c_int;
    pub fn cpz_last_error() -> *const c_char;
    pub fn cpz_default_generators(g: *mut u8, h: *mut u8);
    pub fn cpz_verify_each(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, y1: *const u8, y2: *const u8,
                           r1: *const u8, r2: *const u8, s: *const u8, ctx_bytes: *const u8, ctx_off: *const u64,
                           ctx_present: *const u8, status_out: *mut u8) -> c_int;
    pub fn cpz_verify_each_ex(ctx: *mut cpz_ctx, flags: u32, g: *const u8, h: *const u8, n: usize, y1: *const u8,
                              y2: *const u8, r1: *const u8, r2: *const u8, s: *const u8, ctx_bytes: *const u8,
                              ctx_off: *const u64, ctx_present: *const u8, status_out: *mut u8) -> c_int;
    pub fn cpz_verify_each_device(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, d_y1: *const c_void,
                                  d_y2: *const c_void, d_r1: *const c_void, d_r2: *const c_void, d_s: *const c_void,
                                  d_ctx_bytes: *const c_void, d_ctx_off: *const u64, d_ctx_present: *const u8,
                                  d_status_out: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn cpz_challenges(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, y1: *const u8, y2: *const u8,
                          r1: *const u8, r2: *const u8, ctx_bytes: *const u8, ctx_off: *const u64,
                          ctx_present: *const u8, c_out: *mut u8) -> c_int;
    pub fn cpz_verify_response(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, y1: *const u8, y2: *const u8,
                               r1: *const u8, r2: *const u8, s: *const u8, c: *const u8, status_out: *mut u8) -> c_int;
    pub fn cpz_verify_response_ex(ctx: *mut cpz_ctx, flags: u32, g: *const u8, h: *const u8, n: usize,
                                  y1: *const u8, y2: *const u8, r1: *const u8, r2: *const u8, s: *const u8,
                                  c: *const u8, status_out: *mut u8) -> c_int;
    pub fn cpz_verify_response_device(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, d_y1: *const c_void,
                                      d_y2: *const c_void, d_r1: *const c_void, d_r2: *const c_void,
                                      d_s: *const c_void, d_c: *const c_void, d_status_out: *mut c_void,
                                      stream: *mut c_void) -> c_int;
    pub fn cpz_prove(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, x: *const u8, k: *const u8,
                     ctx_bytes: *const u8, ctx_off: *const u64, ctx_present: *const u8, y1: *mut u8, y2: *mut u8,
                     r1: *mut u8, r2: *mut u8, s: *mut u8) -> c_int;
    pub fn cpz_prove_device(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, d_x: *const c_void,
                            d_k: *const c_void, d_ctx_bytes: *const c_void, d_ctx_off: *const u64,
                            d_ctx_present: *const u8, d_y1: *mut c_void, d_y2: *mut c_void, d_r1: *mut c_void,
                            d_r2: *mut c_void, d_s: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn cpz_prove_synthetic(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, first_index: u64,
                               seed_x: *const u8, seed_k: *const u8, ctx_bytes: *const u8, ctx_off: *const u64,
                               ctx_present: *const u8, y1: *mut u8, y2: *mut u8, r1: *mut u8, r2: *mut u8,
                               s: *mut u8) -> c_int;
    pub fn cpz_prove_synthetic_device(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, first_index: u64,
                                      seed_x: *const u8, seed_k: *const u8, d_ctx_bytes: *const c_void,
                                      d_ctx_off: *const u64, d_ctx_present: *const u8, d_y1: *mut c_void,
                                      d_y2: *mut c_void, d_r1: *mut c_void, d_r2: *mut c_void, d_s: *mut c_void,
                                      stream: *mut c_void) -> c_int;
    pub fn cpz_verify_batch(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, y1: *const u8, y2: *const u8,
                            r1: *const u8, r2: *const u8, s: *const u8, ctx_bytes: *const u8, ctx_off: *const u64,
                            ctx_present: *const u8, seed: *const u8, first_index: u64, partial_out: *mut u8,
                            batch_ok: *mut c_int, status_out: *mut u8) -> c_int;
    pub fn cpz_verify_batch_ex(ctx: *mut cpz_ctx, flags: u32, g: *const u8, h: *const u8, n: usize, y1: *const u8,
                               y2: *const u8, r1: *const u8, r2: *const u8, s: *const u8, ctx_bytes: *const u8,
                               ctx_off: *const u64, ctx_present: *const u8, seed: *const u8, first_index: u64,
                               partial_out: *mut u8, batch_ok: *mut c_int, status_out: *mut u8) -> c_int;
    pub fn cpz_verify_batch_device(ctx: *mut cpz_ctx, g: *const u8, h: *const u8, n: usize, d_y1: *const c_void,
                                   d_y2: *const c_void, d_r1: *const c_void, d_r2: *const c_void, d_s: *const c_void,
                                   d_ctx_bytes: *const c_void, d_ctx_off: *const u64, d_ctx_present: *const u8,
                                   seed: *const u8, first_index: u64, partial_out: *mut u8, batch_ok: *mut c_int,
                                   d_status_out: *mut c_void, fallback: c_int, stream: *mut c_void) -> c_int;
    pub fn cpz_decode_points(ctx: *mut cpz_ctx, n: usize, points: *const u8, ok_out: *mut u8,
                             reencoded_out: *mut u8) -> c_int;
    pub fn cpz_msm(ctx: *mut cpz_ctx, n: usize, points: *const u8, scalars: *const u8, out: *mut u8) -> c_int;
    pub fn cpz_combine_partials(ctx: *mut cpz_ctx, k: usize, partials: *const u8, out: *mut u8,
                                is_identity: *mut c_int) -> c_int;
    pub fn cpz_parse_proofs(ctx: *mut cpz_ctx, n: usize, blob: *const u8, off: *const u64, r1_out: *mut u8,
                            r2_out: *mut u8, s_out: *mut u8, code_out: *mut u8, aux_out: *mut u32) -> c_int;
    pub fn cpz_parse_proofs_device(ctx: *mut cpz_ctx, n: usize, d_blob: *const c_void, d_off: *const u64,
                                   d_r1: *mut c_void, d_r2: *mut c_void, d_s: *mut c_void, d_code: *mut c_void,
                                   d_aux: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn cpz_verify_each_multi(ctxs: *const *mut cpz_ctx, nctx: c_int, g: *const u8, h: *const u8, n: usize,
                                 y1: *const u8, y2: *const u8, r1: *const u8, r2: *const u8, s: *const u8,
                                 ctx_bytes: *const u8, ctx_off: *const u64, ctx_present: *const u8,
                                 status_out: *mut u8) -> c_int;
    pub fn cpz_verify_batch_multi(ctxs: *const *mut cpz_ctx, nctx: c_int, g: *const u8, h: *const u8, n: usize,
                                  y1: *const u8, y2: *const u8, r1: *const u8, r2: *const u8, s: *const u8,
                                  ctx_bytes: *const u8, ctx_off: *const u64, ctx_present: *const u8, seed: *const u8,
                                  partials_out: *mut u8, total_out: *mut u8, batch_ok: *mut c_int,
                                  status_out: *mut u8) -> c_int;
    pub fn cpz_ctx_set_timing(ctx: *mut cpz_ctx, enable: c_int) -> c_int;
    pub fn cpz_ctx_stage_times(ctx: *mut cpz_ctx, ms_out: *mut f64, launches_out: *mut c_int) -> c_int;
    pub fn cpz_ctx_stage_times_n(ctx: *mut cpz_ctx, nstages: c_int, ms_out: *mut f64, launches_out: *mut c_int)
                                 -> c_int;
}
