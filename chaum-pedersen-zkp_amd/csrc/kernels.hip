// gfx950 kernels for the Chaum-Pedersen verify path.
//
//   k_transcript_prefix  one thread: Merlin state after Transcript::new() (S0) and after
//                        append_parameters(g, h) (S1)          transcript.rs:29-50
//   k_challenge          1 thread / proof: Fiat-Shamir challenge c (bit-exact merlin),
//                        response-scalar checks (from_canonical_bytes, zero); entries
//                        without a context or with a 32-byte one on fixed schedules in
//                        registers, any other context length on an LDS sponge image
//                        batch.rs:188-206, gadgets.rs:466-482
//   k_challenge_noctx    the same for batches without contexts (registers only)
//   k_niels_bases /      (k * B) for k = 1..128, B in {g, h} x {2^(32 m): m = 0..7}: affine
//   k_build_niels        Niels tables
//   k_verify_each        1 thread / proof: challenge split v c = u (mod l) with
//                        u, |v| < 2^127 (verify.h), 4 ristretto decodes, then per equation
//                        [v s] B - [u] y - [v] r in E[4]  <=>  [s] B - [c] y == r
//                        by a half-length Straus loop: radix-16 signed digits of u and |v|
//                        against per-proof tables of 8 multiples of -y and -+r (HBM-backed
//                        scratch), then [v s mod l] B as 16 mixed additions from the
//                        fixed-base comb of B in HBM (radix-2^16 digits).
//                        batch.rs:185-231, verifier/mod.rs:144-171
//   k_parse_proofs       bulk Proof::from_bytes (gadgets.rs:364-489) into SoA rows + codes
//   k_prove_points /     synthetic-input generator: Prover::prove_with_transcript
//   k_prove_response     (prover/mod.rs:86-131) with ChaCha20-derived witnesses/nonces
//
// Status codes (uint8 per proof): 0 valid, 1 equation failed, 2 undecodable point,
// 3 non-canonical s, 4 identity commitment, 5 zero s.
#include <hip/hip_runtime.h>

#include "cpz_kernels.h"
#include "ristretto.h"
#include "scalar25519.h"
#include "transcript.h"
#include "scalarmul.h"
#include "verify.h"
#include "rlc_dev.h"
#include "fe16.h"
#include "keccak_wave.h"
#include "proof_digits.h"

namespace cpz {

// ---------------------------------------------------------------------------------------
// Loads
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool words_zero(const uint32_t w[8]) {
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) acc |= w[k];
  return acc == 0;
}

__device__ __forceinline__ void store_words8(uint32_t* base, int64_t i, const uint32_t w[8]) {
  uint4* p = reinterpret_cast<uint4*>(base + 8 * i);
  p[0] = make_uint4(w[0], w[1], w[2], w[3]);
  p[1] = make_uint4(w[4], w[5], w[6], w[7]);
}


__global__ void k_transcript_prefix(const uint32_t* __restrict__ gh_words, StrobeSnap* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ArrayState st;
  Strobe<ArrayState> s = transcript_new(st);
  for (int i = 0; i < 200; i++) out[0].state[i] = st.b[i];
  out[0].pos = s.pos; out[0].pos_begin = s.pos_begin; out[0].flags = s.cur_flags;
  transcript_parameters(s, gh_words, gh_words + 8);
  for (int i = 0; i < 200; i++) out[1].state[i] = st.b[i];
  out[1].pos = s.pos; out[1].pos_begin = s.pos_begin; out[1].flags = s.cur_flags;
}

constexpr int kChallengeBlock = 128;

// Generic transcript tail: the byte-wise STROBE code on this thread's dword-interleaved
// image of the sponge in LDS (any context length).
__device__ __forceinline__ sc challenge_generic(const ChallengeArgs& a, uint32_t* lds, bool has_ctx, uint64_t b0,
                                                uint64_t b1, const uint32_t y1[8], const uint32_t y2[8],
                                                const uint32_t r1[8], const uint32_t r2[8]) {
  LdsState st{lds, (int)threadIdx.x, kChallengeBlock};
  const StrobeSnap& snap = a.prefix[has_ctx ? 0 : 1];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(snap.state);
#pragma unroll
    for (int w = 0; w < 50; w++) lds[w * kChallengeBlock + threadIdx.x] = src[w];
  }
  Strobe<LdsState> s(st, snap.pos, snap.pos_begin, (uint8_t)snap.flags);
  if (has_ctx) {
    transcript_context(s, a.ctx_bytes + b0, (uint32_t)(b1 - b0));
    transcript_parameters(s, a.gh_words, a.gh_words + 8);
  }
  return transcript_challenge(s, y1, y2, r1, r2);
}

__global__ void __launch_bounds__(kChallengeBlock) k_challenge(ChallengeArgs a) {
  __shared__ uint32_t lds[50 * kChallengeBlock];
  const int64_t i = (int64_t)blockIdx.x * kChallengeBlock + threadIdx.x;
  if (i >= a.n) return;
  const bool has_ctx = a.ctx_off != nullptr && (a.ctx_present == nullptr || a.ctx_present[i] != 0);
  uint32_t y1[8], y2[8], r1[8], r2[8];
  load_words8(y1, a.y1, i);
  load_words8(y2, a.y2, i);
  load_words8(r1, a.r1, i);
  load_words8(r2, a.r2, i);
  const uint64_t b0 = has_ctx ? a.ctx_off[i] : 0;
  const uint64_t b1 = has_ctx ? (a.ctx_end ? a.ctx_end[i] : a.ctx_off[i + 1]) : 0;
  // Entries on a fixed schedule skip the LDS sponge: no context (k_challenge_noctx's tail)
  // or a 4-byte-aligned 32-byte context (the service's challenge ids).
  const bool fixed_noctx = !has_ctx && a.fast_noctx;
  // (the context's own address must be 4-byte aligned: the base pointer is the caller's)
  const bool fixed_ctx32 = has_ctx && a.fast_ctx32 && b1 - b0 == 32 &&
                           ((reinterpret_cast<uintptr_t>(a.ctx_bytes) + b0) & 3) == 0;
  sc c;
  if (fixed_noctx) {
    c = challenge_fixed(reinterpret_cast<const uint32_t*>(a.prefix[1].state), a.k1, a.k2, y1, y2, r1, r2);
  } else if (fixed_ctx32) {
    uint32_t cw[8];
    const uint32_t* cp = reinterpret_cast<const uint32_t*>(a.ctx_bytes + b0);  // 4-byte aligned (above)
#pragma unroll
    for (int k = 0; k < 8; k++) cw[k] = cp[k];
    c = challenge_fixed_ctx32(reinterpret_cast<const uint32_t*>(a.prefix[0].state), a.c32, cw, y1, y2, r1, r2);
  } else {
    c = challenge_generic(a, lds, has_ctx, b0, b1, y1, y2, r1, r2);
  }
  store_words8(a.c_out, i, c.w);
  if (a.s != nullptr) {
    uint32_t w[8];
    load_words8(w, a.s, i);
    a.status_out[i] = response_status(w, a.eq_only != 0);
  }
}
// No-context fast path (verify.h, challenge_fixed): the sponge in 50 registers, the
// framing as two constant masks, two permutations, no LDS.  Chosen by the runtime when the
// prefix snapshot sits at the fixed position.
__global__ void __launch_bounds__(256) k_challenge_noctx(ChallengeArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  uint32_t y1[8], y2[8], r1[8], r2[8];
  load_words8(y1, a.y1, i);
  load_words8(y2, a.y2, i);
  load_words8(r1, a.r1, i);
  load_words8(r2, a.r2, i);
  const sc c = challenge_fixed(reinterpret_cast<const uint32_t*>(a.prefix[1].state), a.k1, a.k2, y1, y2, r1, r2);
  store_words8(a.c_out, i, c.w);
  if (a.s != nullptr) {
    uint32_t w[8];
    load_words8(w, a.s, i);
    a.status_out[i] = response_status(w, a.eq_only != 0);
  }
}

// ---------------------------------------------------------------------------------------
// Fixed-base tables: tab[b * 128 + (k - 1)] = k * base_b in affine Niels form.
// ---------------------------------------------------------------------------------------
// Tables for kNielsLevels * nbases bases: [b0 .. b_{n-1}] at 2^0, 2^128, 2^64, 2^192, 2^32,
// 2^96, 2^160, 2^224 times (niels_level_doublings), 128 entries each.
// k_niels_bases: quad b decodes base b % nbases (every lane; ok flags from the first nbases
// quads) and doubles it as level b / nbases says, as quad-cooperative doublings (~0.25 ms
// for the longest chain, against ~0.6 ms on one lane per thread): B, 2^128 B (k_verify_quad's
// variable bases, the RLC extras), and all eight (k_verify_wide's eight 32-bit parts of s');
// k_build_niels: one thread per entry, [k] B_b by
// double-and-add and one inversion to affine Niels.  A variable-base call's cold (g, h) waits
// for both (ensure_generators).
__global__ void __launch_bounds__(64) k_niels_bases(const uint32_t* __restrict__ base_words, int nbases,
                                                     ge_p3* __restrict__ bases, int* __restrict__ ok) {
  const int b = threadIdx.x >> 2, q = threadIdx.x & 3;
  if (b >= kNielsLevels * nbases) return;  // whole quads
  ge_p3 B;
  const bool dec = ristretto_decode(B, base_words + 8 * (b % nbases));
  if (b < nbases && q == 0) ok[b] = dec ? 1 : 0;
  const int dbl = niels_level_doublings(b / nbases);
  if (dbl) B = p3_dbl_n_quad(B, dbl, q);
  if (q == 0) bases[b] = B;
}

__global__ void __launch_bounds__(64) k_build_niels(const ge_p3* __restrict__ bases, int nbases,
                                                    ge_niels* __restrict__ tab) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kNielsLevels * nbases * kNielsEntries) return;
  const int b = t / kNielsEntries;
  const int k = t % kNielsEntries + 1;
  tab[t] = p3_to_niels(small_mul(bases[b], k));
}

// ---------------------------------------------------------------------------------------
// Fixed-base combs (scalarmul.h): comb[b][k][j] = j * 2^(16 k) * base_b, affine Niels (j = 0: identity).
// k_comb_bases: thread (b, k) doubles base_b 16 k times.  k_comb_fill: one thread per
// entry, [j] Q_(b,k) by double-and-add over the 15-bit j, then one inversion to affine.
// 2^20 entries, a few milliseconds, once per (g, h) pair.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_comb_bases(const uint32_t* __restrict__ gh_words, ge_p3* __restrict__ q) {
  const int t = threadIdx.x;
  if (t >= 2 * kCombWindows) return;
  const int b = t / kCombWindows, k = t % kCombWindows;
  ge_p3 B;
  (void)ristretto_decode(B, gh_words + 8 * b);  // validity is checked by k_build_niels
#pragma unroll 1
  for (int d = 0; d < 16 * k; d++) B = p1p1_to_p3(p3_dbl(B));
  q[t] = B;
}

__global__ void __launch_bounds__(256) k_comb_fill(const ge_p3* __restrict__ q, ge_niels* __restrict__ comb) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * kCombPerBase) return;
  const int bk = (int)(t / kCombStride);  // b * kCombWindows + k
  const int j = (int)(t % kCombStride);
  if (j == 0) {
    comb[t] = ge_niels_identity();
    return;
  }
  const ge_p3 Q = q[bk];
  ge_p3 acc = Q;  // bit 15 of j set only for j = 2^15
  const int top = 31 - __builtin_clz((unsigned)j);
#pragma unroll 1
  for (int bit = top - 1; bit >= 0; bit--) {
    acc = p1p1_to_p3(p3_dbl(acc));
    if ((j >> bit) & 1) acc = ge_add(acc, Q);
  }
  comb[t] = p3_to_niels(acc);
}

// ---------------------------------------------------------------------------------------
// Bulk wire-format ingestion: Proof::from_bytes (gadgets.rs:364-489) for n blobs, one
// thread per blob, checks in the reference's order -- structural checks of each field,
// each field decoded (element_from_bytes / scalar_from_bytes) before the next field's
// structure is looked at, trailing bytes, then identity commitments and zero s -- so
// the first failing check, and hence the error, is the reference's.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t be32_at(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

__device__ __forceinline__ void words_at(uint32_t w[8], const uint8_t* p) {
#pragma unroll
  for (int k = 0; k < 8; k++)
    w[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
           ((uint32_t)p[4 * k + 3] << 24);
}

__global__ void __launch_bounds__(256) k_parse_proofs(ParseArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t o0 = a.off[i];
  const uint64_t len = a.off[i + 1] - o0;
  const uint8_t* b = a.blob + o0;
  uint32_t f0[8], f1[8], f2[8];  // r1, r2, s (separate arrays: q is a runtime index)
#pragma unroll
  for (int k = 0; k < 8; k++) f0[k] = f1[k] = f2[k] = 0;
  uint8_t code = kParseOk;
  uint32_t aux = 0;
  if (len < 1 + 4 + 1 + 4 + 1 + 4 + 1) {
    code = kParseTooSmall;
    aux = (uint32_t)len;
  } else if (b[0] != 1) {  // PROTOCOL_VERSION
    code = kParseBadVersion;
    aux = b[0];
  } else {
    uint64_t pos = 1;
#pragma unroll 1
    for (int q = 0; q < 3 && code == kParseOk; q++) {
      const uint8_t base = (uint8_t)(kParseR1LenMissing + 5 * q);
      const uint32_t maxlen = q < 2 ? 4096u : 512u;
      if (pos + 4 > len) { code = base; break; }
      const uint32_t fl = be32_at(b + pos);
      pos += 4;
      if (fl == 0 || fl > maxlen) { code = base + 1; aux = fl; break; }
      if (pos + fl > len) { code = base + 2; break; }
      if (fl != 32) { code = base + 3; aux = fl; break; }
      uint32_t w[8];
      words_at(w, b + pos);
      pos += 32;
      bool ok;
      if (q < 2) {
        ge_p3 P;
        ok = ristretto_decode(P, w);
      } else {
        ok = sc_is_canonical(w);
      }
      if (!ok) { code = base + 4; break; }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        f0[k] = q == 0 ? w[k] : f0[k];
        f1[k] = q == 1 ? w[k] : f1[k];
        f2[k] = q == 2 ? w[k] : f2[k];
      }
    }
    if (code == kParseOk && pos != len) {
      code = kParseTrailing;
      aux = (uint32_t)(len - pos);
    }
    if (code == kParseOk) {
      // validate_element (ristretto.rs:173-185) holds for every decoded point.
      if (words_zero(f0) || words_zero(f1)) code = kParseIdentity;
      else if (words_zero(f2)) code = kParseZeroS;
    }
  }
  store_words8(a.r1, i, f0);
  store_words8(a.r2, i, f1);
  store_words8(a.s, i, f2);
  a.code[i] = code;
  if (a.aux) a.aux[i] = aux;
}

// ---------------------------------------------------------------------------------------
// Per-proof verification
// ---------------------------------------------------------------------------------------

#ifndef CPZ_VERIFY_WAVES
#define CPZ_VERIFY_WAVES 2  // waves per SIMD (256 VGPRs each)
#endif
// The proof's four point encodings are staged in LDS (one word column per thread): they are
// read once per decode, and no row address has to stay live across the Straus loops.
__device__ __forceinline__ void verify_one_row(const VerifyArgs& a, int64_t i, const CombTable& comb_g,
                                               const CombTable& comb_h, const SlabTable& tab, uint32_t* dig,
                                               uint32_t* rows) {
  const uint32_t* src[4] = {a.y1, a.y2, a.r1, a.r2};
  uint32_t sw[8], cw[8];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t w[8];
    load_words8(w, src[q], i);
#pragma unroll
    for (int k = 0; k < 8; k++) rows[(8 * q + k) * kVerifyBlock] = w[k];
  }
  load_words8(sw, a.s, i);
  load_words8(cw, a.c, i);
  const uint8_t st_s = a.status[i];
  const DigitRef y1{rows, kVerifyBlock}, y2{rows + 8 * kVerifyBlock, kVerifyBlock},
      r1{rows + 16 * kVerifyBlock, kVerifyBlock}, r2{rows + 24 * kVerifyBlock, kVerifyBlock};
  a.status[i] = verify_proof(y1, y2, r1, r2, sw, cw, st_s, comb_g, comb_h, tab, dig, kVerifyBlock, nullptr,
                             a.eq_only != 0);
}

// The RLC fallback's per-proof pass (rlc_fallback): points, challenges and decode-level
// statuses come from the RLC prepare of the same batch, so only the equations are checked.
__global__ void __launch_bounds__(kVerifyBlock, CPZ_VERIFY_WAVES) k_verify_prepared(VerifyArgs a) {
  const CombTable comb_g{a.comb}, comb_h{a.comb + kCombPerBase};
  const int64_t l = (int64_t)blockIdx.x * kVerifyBlock + threadIdx.x;  // this launch's thread: its slab slot
  int64_t i = l;  // one proof per thread
  if (a.blocks) {
    const int64_t lb = (int64_t)blockIdx.x * (kVerifyBlock / a.block_proofs) + threadIdx.x / a.block_proofs;
    if (lb >= a.nblocks) return;
    i = (int64_t)a.blocks[lb] * a.block_proofs + threadIdx.x % a.block_proofs;
  }
  if (i >= a.n) return;
  const SlabTable tab{a.scratch, (uint32_t)l * (uint32_t)(kCachedEntries * sizeof(ge_cached))};
  __shared__ uint32_t dig[16 * kVerifyBlock];
  {
    if (a.status[i] != kStOk) return;  // decode-level rejection: already final
    uint32_t sw[8], cw[8];
    load_words8(sw, a.s, i);
    load_words8(cw, a.c, i);
    const DigitRef none{nullptr, 0};
    a.status[i] = verify_proof<true>(none, none, none, none, sw, cw, kStOk, comb_g, comb_h, tab, dig + threadIdx.x,
                                     kVerifyBlock, a.pre + 4 * i, a.eq_only != 0);
  }
}

__global__ void __launch_bounds__(kVerifyBlock, CPZ_VERIFY_WAVES) k_verify_each(VerifyArgs a) {
  const CombTable comb_g{a.comb}, comb_h{a.comb + kCombPerBase};
  // one proof per thread: the runtime cuts a batch into launches of at most grid x block
  // proofs (launch_verify_chunks), so there is no grid-stride loop state to keep live
  const int64_t i = (int64_t)blockIdx.x * kVerifyBlock + threadIdx.x;
  if (i >= a.n) return;
  // this thread's tables: kCachedEntries entries, contiguous (scalarmul.h, SlabTable)
#if defined(CPZ_EXP_SLAB_MOD)
  // timing experiment only (wrong verdicts: threads share slots; timing_only.h): an L2-sized slab
  const SlabTable tab{a.scratch, (uint32_t)(i % CPZ_EXP_SLAB_MOD) * (uint32_t)(kCachedEntries * sizeof(ge_cached))};
#else
  const SlabTable tab{a.scratch, (uint32_t)i * (uint32_t)(kCachedEntries * sizeof(ge_cached))};
#endif
  // digit words and point encodings in LDS, one column per thread (scalarmul.h, DigitRef)
  __shared__ uint32_t dig[16 * kVerifyBlock];
  __shared__ uint32_t rows[32 * kVerifyBlock];
#if defined(CPZ_CLOCK_PROBE)
  // Timing variant only (tools/time_verify.py; timing_only.h): the shader clock (s_memtime) and the constant
  // 100 MHz clock (s_memrealtime) around this wave's work and the wave's hardware id, written
  // over the wave's 64 status bytes (the verdicts are lost; the status buffer must be 8-byte
  // aligned, as the timing harness's is) -> the clock the kernel actually ran at and how many
  // of its waves each SIMD held over time.
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
#endif
  verify_one_row(a, i, comb_g, comb_h, tab, dig + threadIdx.x, rows + threadIdx.x);
#if defined(CPZ_CLOCK_PROBE)
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0 && i + 63 < a.n) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* out = reinterpret_cast<uint64_t*>(a.status + i);
    out[0] = t1 - t0;
    out[1] = q1 - q0;
    out[2] = q0;  // absolute 100 MHz stamps and the wave's SIMD: a per-SIMD occupancy timeline
    out[3] = q1;
    out[4] = (uint64_t)hw | ((uint64_t)xcc << 32);
  }
#endif
}

// ---------------------------------------------------------------------------------------
// Synthetic prover (input generator): x_i, k_i = wide(ChaCha20(seed_x / seed_k, block i)).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ sc chacha_scalar(const uint32_t key[8], uint64_t counter) {
  uint32_t blk[16];
  chacha20_block(blk, key, counter, 0);
  return sc_reduce_wide(blk);
}

// Witness / nonce of proof i: the caller's scalar (mod l), or the synthetic ChaCha20 one.
__device__ __forceinline__ sc prove_scalar(const uint32_t* in, const uint32_t seed[8], uint64_t idx, int64_t i) {
  if (in == nullptr) return chacha_scalar(seed, idx);
  uint32_t wide[16];
  load_words8(wide, in, i);
#pragma unroll
  for (int k = 8; k < 16; k++) wide[k] = 0;
  return sc_reduce_wide(wide);
}

__global__ void __launch_bounds__(kVerifyBlock, 2) k_prove_points(ProveArgs a) {
  const CombTable comb_g{a.comb}, comb_h{a.comb + kCombPerBase};
  const int64_t i = (int64_t)blockIdx.x * kVerifyBlock + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t idx = a.first_index + (uint64_t)i;
  uint32_t d[8], w[8];
  {
    const sc x = prove_scalar(a.x_in, a.seed_x, idx, i);
    sc_recode_radix65536(d, x.w);
  }
  ristretto_encode(w, comb_mul(comb_g, d));
  store_words8(a.y1, i, w);
  ristretto_encode(w, comb_mul(comb_h, d));
  store_words8(a.y2, i, w);
  {
    const sc k = prove_scalar(a.k_in, a.seed_k, idx, i);
    sc_recode_radix65536(d, k.w);
  }
  ristretto_encode(w, comb_mul(comb_g, d));
  store_words8(a.r1, i, w);
  ristretto_encode(w, comb_mul(comb_h, d));
  store_words8(a.r2, i, w);
}

__global__ void k_prove_response(ProveArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t idx = a.first_index + (uint64_t)i;
  const sc x = prove_scalar(a.x_in, a.seed_x, idx, i);
  const sc k = prove_scalar(a.k_in, a.seed_k, idx, i);
  sc c;
  load_words8(c.w, a.c, i);
  const sc s = sc_add(k, sc_mul(c, x));  // s = k + c x   (prover/mod.rs:126-131)
  store_words8(a.s_out, i, s.w);
}

// ---------------------------------------------------------------------------------------
// Bulk element_from_bytes (ristretto.rs:120-138) + element_to_bytes (:141-143): ok[i] = 1 iff
// point i decodes; out[i] = the encoding of the decoded point (equal to the input for every
// valid encoding -- ristretto encodings are canonical), zero when it does not decode.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_decode_encode(int64_t n, const uint32_t* __restrict__ pts,
                                                       uint8_t* __restrict__ ok, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  load_words8(w, pts, i);
  ge_p3 P;
  const bool dec = ristretto_decode(P, w);
  ok[i] = dec ? 1 : 0;
  if (out != nullptr) {
    ristretto_encode(w, P);
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = dec ? w[k] : 0u;
    store_words8(out, i, w);
  }
}

hipError_t launch_decode_encode(int64_t n, const uint32_t* pts, uint8_t* ok, uint32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_decode_encode, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, pts, ok, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// cpz_verify_response (Verifier::verify_response, verifier/mod.rs:144-171): the challenge is
// the caller's, so there is no transcript; only the response checks and a canonical copy of
// the challenge (a non-canonical one is reported, and zeroed so the split stays in range).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_response_prep(int64_t n, const uint32_t* __restrict__ s,
                                                       const uint32_t* __restrict__ c_in, uint32_t* __restrict__ c_out,
                                                       uint8_t* __restrict__ status, int eq_only) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8], c[8];
  load_words8(w, s, i);
  load_words8(c, c_in, i);
  uint8_t st = response_status(w, eq_only != 0);
  const bool c_ok = sc_is_canonical(c);
  if (st == kStOk && !c_ok) st = kStBadChallenge;
#pragma unroll
  for (int k = 0; k < 8; k++) c[k] = c_ok ? c[k] : 0u;
  store_words8(c_out, i, c);
  status[i] = st;
}

// ---------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------
hipError_t launch_transcript_prefix(const uint32_t* gh_words, StrobeSnap* out, hipStream_t st) {
  hipLaunchKernelGGL(k_transcript_prefix, dim3(1), dim3(64), 0, st, gh_words, out);
  return hipGetLastError();
}

bool challenge_prefix_is_fixed(const StrobeSnap& snap) {
  return snap.pos == kTailPrefixPos && snap.pos_begin == kTailPrefixBegin && snap.flags == kTailPrefixFlags;
}

bool challenge_prefix_is_ctx32(const StrobeSnap& snap) {
  return snap.pos == kC32PrefixPos && snap.pos_begin == kC32PrefixBegin && snap.flags == kC32PrefixFlags;
}

hipError_t launch_challenge(const ChallengeArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  if (a.ctx_off == nullptr && a.fast_noctx) {
    hipLaunchKernelGGL(k_challenge_noctx, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  const int64_t blocks = (a.n + kChallengeBlock - 1) / kChallengeBlock;
  hipLaunchKernelGGL(k_challenge, dim3((unsigned)blocks), dim3(kChallengeBlock), 0, st, a);
  return hipGetLastError();
}

// One thread per gathered proof: its five rows (two 16-byte loads each) and, with contexts,
// its context's [begin, end) in the batch's blob and its presence flag.
__global__ void __launch_bounds__(256) k_probe_gather(ProbeGatherArgs a) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= kProbeChunks * a.blk) return;
  const int64_t src = a.starts[j / a.blk] + j % a.blk;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    uint32_t w[8];
    load_words8(w, a.rows[q], src);
    store_words8(a.out_rows[q], j, w);
  }
  if (a.ctx_off) {
    a.out_begin[j] = a.ctx_off[src];
    a.out_end[j] = a.ctx_off[src + 1];
    a.out_present[j] = a.ctx_present ? a.ctx_present[src] : (uint8_t)1;
  }
}

hipError_t launch_probe_gather(const ProbeGatherArgs& a, hipStream_t st) {
  const int m = kProbeChunks * a.blk;
  hipLaunchKernelGGL(k_probe_gather, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_build_niels(const uint32_t* base_words, int nbases, ge_niels* tab, int* ok, ge_p3* bases,
                              hipStream_t st) {
  if (nbases < 1 || kNielsLevels * nbases > 16) return hipErrorInvalidValue;  // one wave of quads
  hipLaunchKernelGGL(k_niels_bases, dim3(1), dim3(64), 0, st, base_words, nbases, bases, ok);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int total = kNielsLevels * nbases * kNielsEntries;
  hipLaunchKernelGGL(k_build_niels, dim3((total + 63) / 64), dim3(64), 0, st, (const ge_p3*)bases, nbases, tab);
  return hipGetLastError();
}

__global__ void k_niels_r16(const ge_niels* __restrict__ tab, int32_t* __restrict__ out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // entry * 3 + field
  if (t >= 3 * n) return;
  const ge_niels& e = tab[t / 3];
  const int f = t % 3;
  uint32_t w[8];
  fe_towords(w, f == 0 ? e.ypx : (f == 1 ? e.ymx : e.xy2d));
#pragma unroll
  for (int k = 0; k < 16; k++) out[16 * t + k] = (int32_t)((w[k >> 1] >> (16 * (k & 1))) & 0xffffu);
}

hipError_t launch_niels_r16(const ge_niels* tab, int32_t* out, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_niels_r16, dim3((3 * n + 255) / 256), dim3(256), 0, st, tab, out, n);
  return hipGetLastError();
}

hipError_t launch_build_comb(const uint32_t* gh_words, ge_p3* bases_scratch, ge_niels* comb, hipStream_t st) {
  hipLaunchKernelGGL(k_comb_bases, dim3(1), dim3(64), 0, st, gh_words, bases_scratch);
  hipLaunchKernelGGL(k_comb_fill, dim3((unsigned)((2 * kCombPerBase + 255) / 256)), dim3(256), 0, st,
                     (const ge_p3*)bases_scratch, comb);
  return hipGetLastError();
}

int verify_each_blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_verify_each, kVerifyBlock, 0) != hipSuccess || nb < 1) nb = 2;
  return nb;
}

// ---------------------------------------------------------------------------------------
// Small batches: one proof on eight lanes, a quad per equation (rlc_dev.h's quad-cooperative
// point arithmetic: the four lanes hold the same point, each computes one of a round's four
// products).  k_verify_each gives every proof one lane, so a batch of a few proofs waits for
// one lane's whole verification (~1.1 ms: 31 x 4 doublings and 64 additions per equation
// issued one instruction per ~10 cycles by a lone wave); here the two equations run side by
// side and every point operation takes two product latencies instead of eight.  Lanes 0 / 1
// of a quad decode Y / R of its equation; the quad's tables (cached multiples 0..8 of -Y and
// of -R, or R when v < 0) live in the scratch slab, 160 bytes per entry, lane q storing and
// loading only field q (Y+X, Y-X, 2dT, Z: the operand fe_sel4 hands it), so a negative digit
// is lanes 0 / 1 swapping fields and lane 2 negating its own.  Same statuses as verify_proof.
// ---------------------------------------------------------------------------------------

__device__ __forceinline__ void fe_store_limbs(int32_t* dst, const fe& f) {
  uint2* d = reinterpret_cast<uint2*>(dst);
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = make_uint2((uint32_t)f.v[2 * k], (uint32_t)f.v[2 * k + 1]);
}

__device__ __forceinline__ fe fe_load_limbs(const int32_t* src) {
  const uint2* d = reinterpret_cast<const uint2*>(src);
  fe f;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint2 v = d[k];
    f.v[2 * k] = (int32_t)v.x;
    f.v[2 * k + 1] = (int32_t)v.y;
  }
  return f;
}

// field q of the cached form, in fe_sel4 order (Y+X, Y-X, 2dT, Z)
__device__ __forceinline__ fe cached_field(const ge_cached& c, int q) { return fe_sel4(q, c.YpX, c.YmX, c.T2d, c.Z); }

__device__ __forceinline__ ge_cached cached_of_field(const fe& x) {
  ge_cached c;
  c.YpX = x;
  c.YmX = x;
  c.T2d = x;
  c.Z = x;
  return c;
}

// entries 0..8 of the quad's table of P (lane q writes field q)
__device__ __forceinline__ void quad_table(int32_t* tab, const ge_p3& P, int q) {
  fe_store_limbs(tab + q * 10, cached_field(ge_cached_identity(), q));
  const ge_cached c1 = p3_to_cached(P);
  fe_store_limbs(tab + 40 + q * 10, cached_field(c1, q));
  ge_p3 acc = p3_dbl_n_quad(P, 1, q);
  fe_store_limbs(tab + 80 + q * 10, cached_field(p3_to_cached(acc), q));
#pragma unroll 1
  for (int k = 3; k <= 8; k++) {
    acc = ge_add_quad(acc, c1, q);
    fe_store_limbs(tab + 40 * k + q * 10, cached_field(p3_to_cached(acc), q));
  }
}

// lane q's operand of signed digit d: entry |d|; a negative digit swaps Y+X / Y-X and
// negates 2dT
__device__ __forceinline__ fe quad_lookup(const int32_t* tab, int d, int q) {
  const bool neg = d < 0;
  const int mag = neg ? -d : d;
  const int f = (neg && q < 2) ? 1 - q : q;
  const fe x = fe_load_limbs(tab + 40 * mag + 10 * f);
  return (neg && q == 2) ? fe_neg(x) : x;
}

// lane q's operand of the Niels multiple d (|d| <= 128, d = 0: the identity (1, 1, 0)) of a
// fixed base whose multiples 1..128 are at tab[0..127] (k_build_niels): Y+X, Y-X, 2dXY, and
// Z = 1 on lane 3; a negative digit swaps lanes 0 / 1's fields and negates lane 2's
__device__ __forceinline__ fe quad_niels_lookup(const ge_niels* tab, int d, int q) {
  const bool neg = d < 0;
  const int mag = neg ? -d : d;
  const int f = (neg && q < 2) ? 1 - q : q;
  const int32_t* e = reinterpret_cast<const int32_t*>(tab + (mag == 0 ? 0 : mag - 1));
  fe x = fe_load_limbs(e + 10 * (f < 3 ? f : 0));
  x = fe_select(x, fe_one(), mag == 0 || q == 3);
  x = fe_select(x, fe_zero(), mag == 0 && q == 2);
  return (neg && q == 2) ? fe_neg(x) : x;
}

__device__ __forceinline__ ge_p3 p3_bcast(const ge_p3& P, int from) {
  ge_p3 r;
  if (from == 0) {
    r.X = fe_quad_bcast<0>(P.X); r.Y = fe_quad_bcast<0>(P.Y); r.Z = fe_quad_bcast<0>(P.Z); r.T = fe_quad_bcast<0>(P.T);
  } else {
    r.X = fe_quad_bcast<1>(P.X); r.Y = fe_quad_bcast<1>(P.Y); r.Z = fe_quad_bcast<1>(P.Z); r.T = fe_quad_bcast<1>(P.T);
  }
  return r;
}

// kVar: no comb for this (g, h) -- [s'] B comes from the Niels multiples 1..128 of B and
// 2^128 B (a.vtab) as 2 x 16 signed radix-256 digits of s', one pair of mixed additions every
// second window of the Straus loop (32 additions per equation against the comb's 16).
template <bool kPre, bool kVar>
__global__ void __launch_bounds__(256) k_verify_quad(VerifyArgs a) {
  const int t = threadIdx.x;
  int64_t i = (int64_t)blockIdx.x * 32 + (t >> 3);
  const int e = (t >> 2) & 1, q = t & 3;
  if (a.blocks) {  // listed blocks of block_proofs proofs (the partitioned check's per-proof passes)
    const int64_t lb = i / a.block_proofs;
    if (lb >= a.nblocks) return;
    i = (int64_t)a.blocks[lb] * a.block_proofs + i % a.block_proofs;
  }
  if (i >= a.n) return;                          // a proof's eight lanes together
  if (kPre && a.status[i] != kStOk) return;      // decode-level rejection: already final
#if defined(CPZ_CLOCK_PROBE)
  // timing builds only: shader-clock stamps at the phase boundaries of block 0's first proof
  uint64_t stamp[kQuadPhases];
  stamp[0] = __builtin_amdgcn_s_memtime();
  stamp[7] = __builtin_amdgcn_s_memrealtime();
#define CPZ_QUAD_STAMP(k) stamp[k] = __builtin_amdgcn_s_memtime()
#else
#define CPZ_QUAD_STAMP(k) (void)0
#endif
  const CombTable comb{kVar ? nullptr : a.comb + (e ? kCombPerBase : 0)};
  int32_t* tab = reinterpret_cast<int32_t*>(a.scratch) + ((int64_t)blockIdx.x * 64 + (t >> 2)) * kQuadTableInts;  // by slot
  uint32_t sw[8], cw[8];
  load_words8(sw, a.s, i);
  load_words8(cw, a.c, i);
  const uint8_t st_s = kPre ? kStOk : a.status[i];
  // challenge split and digits, identical on every lane (verify_proof)
  uint32_t ud[4], vd[4], sd[8];
  bool vneg;
  {
    uint32_t u[4], va[4];
    sc_half_split(cw, u, va, vneg);
    sc_recode_radix16_half(ud, u);
    sc_recode_radix16_half(vd, va);
    sc vs, ss;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      vs.w[k] = k < 4 ? va[k] : 0u;
      ss.w[k] = sw[k];
    }
    sc sp = sc_mul(vs, ss);
    if (vneg) sp = sc_neg(sp);
    if constexpr (kVar)
      sc_recode_radix256(sd, sp.w);   // bytes 0..15: digits on B, bytes 16..31: on 2^128 B
    else
      sc_recode_radix65536(sd, sp.w);
  }
  CPZ_QUAD_STAMP(1);
  // lane 0 decodes this equation's Y, lane 1 its R
  ge_p3 P = ge_identity();
  bool ok = true;
  if (q < 2) {
    if constexpr (kPre) {
      P = affine_from_neg_niels(niels_load(a.pre + 4 * i + (q == 0 ? 1 + 2 * e : 2 * e)));
    } else {
      uint32_t enc[8];
      load_words8(enc, q == 0 ? (e ? a.y2 : a.y1) : (e ? a.r2 : a.r1), i);
      ok = ristretto_decode(P, enc);
    }
  }
  ge_p3 Y = p3_bcast(P, 0), R = p3_bcast(P, 1);
  CPZ_QUAD_STAMP(2);
  Y = ge_neg(Y);
  if (!vneg) R = ge_neg(R);
  quad_table(tab, Y, q);
  quad_table(tab + kQuadTableInts / 2, R, q);
  __threadfence_block();  // the quad's other lanes' fields (a negative digit reads them)
  CPZ_QUAD_STAMP(3);
  // Q = [u] Y' + [|v|] R' + [s'] B: identity (mod E[4]) iff the equation holds
  const ge_niels* gt = kVar ? a.vtab + e * kNielsEntries : nullptr;          // B = g or h
  const ge_niels* gt2 = kVar ? a.vtab + (2 + e) * kNielsEntries : nullptr;   // 2^128 B
  ge_p3 acc = ge_identity();
#pragma unroll 1
  for (int j = 0; j < 4; j++) {
    const uint32_t wu = ud[3], wv = vd[3];
    const uint32_t wg = kVar ? sd[3] : 0u, wg2 = kVar ? sd[7] : 0u;
#pragma unroll
    for (int k = 3; k > 0; k--) {
      ud[k] = ud[k - 1];
      vd[k] = vd[k - 1];
      if constexpr (kVar) {
        sd[k] = sd[k - 1];
        sd[4 + k] = sd[4 + k - 1];
      }
    }
#pragma unroll 1
    for (int m = 7; m >= 0; m--) {
      const int du = ((int32_t)(wu << (28 - 4 * m))) >> 28;
      const int dv = ((int32_t)(wv << (28 - 4 * m))) >> 28;
      const fe ey = quad_lookup(tab, du, q), er = quad_lookup(tab + kQuadTableInts / 2, dv, q);
      if (j != 0 || m != 7) acc = p3_dbl_n_quad(acc, 4, q);
      acc = ge_add_quad(acc, cached_of_field(ey), q);
      acc = ge_add_quad(acc, cached_of_field(er), q);
      if constexpr (kVar) {
        if ((m & 1) == 0) {  // byte 4 (3 - j) + m / 2 of s' (and of s' >> 128): weight 2^(4 t), t even
          const int dg = (int32_t)(wg << (24 - 4 * m)) >> 24;
          const int dg2 = (int32_t)(wg2 << (24 - 4 * m)) >> 24;
          acc = ge_add_quad(acc, cached_of_field(quad_niels_lookup(gt, dg, q)), q);
          acc = ge_add_quad(acc, cached_of_field(quad_niels_lookup(gt2, dg2, q)), q);
        }
      }
    }
  }
  CPZ_QUAD_STAMP(4);
#pragma unroll 1
  for (int j = 0; j < (kVar ? 0 : 8); j++) {
    const uint32_t w = sd[0];
#pragma unroll
    for (int k = 0; k < 7; k++) sd[k] = sd[k + 1];
#pragma unroll
    for (int m = 0; m < 2; m++) {
      const int d = (int32_t)(w << (16 - 16 * m)) >> 16;
      const ge_niels nl = comb.lookup(2 * j + m, d);
      ge_cached c;
      c.YpX = nl.ypx;
      c.YmX = nl.ymx;
      c.T2d = nl.xy2d;
      c.Z = fe_one();
      acc = ge_add_quad(acc, c, q);
    }
  }
  CPZ_QUAD_STAMP(5);
  // the proof's verdict from its two quads (lane 0 of quad e = 0 writes it)
  int eq = ristretto_is_identity(acc) ? 1 : 0;
  eq &= __shfl_xor(eq, 4);
  int bad = ok ? 0 : 1;
  bad |= __shfl_xor(bad, 1);
  bad |= __shfl_xor(bad, 2);
  bad |= __shfl_xor(bad, 4);
  if ((t & 7) != 0) return;
  bool rid = false;
  if constexpr (!kPre) {
    uint32_t w1[8], w2[8];
    load_words8(w1, a.r1, i);
    load_words8(w2, a.r2, i);
    rid = words8_zero(w1) || words8_zero(w2);
  }
  uint8_t st;
  if (bad) st = kStBadPoint;
  else if (st_s == kStBadScalar) st = kStBadScalar;
  else if (rid && !a.eq_only) st = kStIdentity;
  else if (st_s == kStZeroS) st = kStZeroS;
  else if (st_s == kStBadChallenge) st = kStBadScalar;
  else st = eq ? kStOk : kStEqFail;
  a.status[i] = st;
#if defined(CPZ_CLOCK_PROBE)
  CPZ_QUAD_STAMP(6);
  stamp[8] = __builtin_amdgcn_s_memrealtime();
  if (a.clock_probe && blockIdx.x == 0 && t == 0)
    for (int k = 0; k < kQuadPhases; k++) a.clock_probe[k] = stamp[k];
#endif
#undef CPZ_QUAD_STAMP
}


constexpr int kSmallProofs = 8;  // proofs per workgroup (3 waves of 64 lanes)

struct SmallShared {
  uint32_t dig[kSmallProofs][16];      // u (0..3), |v| (4..7), s' (8..15) digit words
  uint32_t meta[kSmallProofs];         // bit 0: v < 0; bits 8..15: response status
  int32_t tab[2][16][9 * 40];          // waves 0 / 1: per quad, entries 0..8 (4 fields x 10 limbs)
  ge_p3 part[3][16];                   // per quad: [u] (-Y), [|v|] (-+R), [s'] B
  uint8_t bad[2][16];                  // decode failures (waves 0 / 1)
  uint8_t rid[16];                     // R encodes the identity (wave 1)
  uint32_t sponge[50][kSmallProofs];   // wave 2's byte-wise transcript, one column per proof
};

__global__ void __launch_bounds__(64 * 3) k_verify_small(VerifyArgs a, ChallengeArgs ca) {
  __shared__ SmallShared sh;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int j = l >> 3, quad = l >> 2, e = (l >> 2) & 1, q = l & 3;
  const int64_t i = (int64_t)blockIdx.x * kSmallProofs + j;
  const bool live = i < a.n;
  const int64_t ii = live ? i : 0;  // dead proofs run the same code on proof 0's rows, unwritten
  ge_p3 acc = ge_identity();
#if defined(CPZ_CLOCK_PROBE)
  // timing builds only: shader-clock stamps of block 0 (wave 0 lane 0: start, decoded, table,
  // barrier A, Straus, barrier B, verdict; wave 2 lane 0: digits written, [s'] B done) and the
  // 100 MHz clock at wave 0's start and end -> a.clock_probe[0 .. kSmallStamps)
  uint64_t* const stamps = (a.clock_probe && blockIdx.x == 0 && l == 0 && w != 1) ? a.clock_probe : nullptr;
#define CPZ_SMALL_STAMP(k) do { if (stamps) stamps[k] = __builtin_amdgcn_s_memtime(); } while (0)
  if (stamps && w == 0) stamps[9] = __builtin_amdgcn_s_memrealtime();
  CPZ_SMALL_STAMP(w == 0 ? 0 : 11);
#else
#define CPZ_SMALL_STAMP(k) (void)0
#endif
  if (w < 2) {
    // ---- waves 0 / 1: decode Y (R) of equation e, its table --------------------------
    ge_p3 P = ge_identity();
    bool ok = true;
    uint32_t enc[8];
    load_words8(enc, w == 0 ? (e ? a.y2 : a.y1) : (e ? a.r2 : a.r1), ii);
    if (q == 0) ok = ristretto_decode(P, enc);
    P = p3_bcast(P, 0);
    if (w == 0) CPZ_SMALL_STAMP(1);
    if (q == 0) {
      sh.bad[w][quad] = ok ? 0 : 1;
      if (w == 1) sh.rid[quad] = words8_zero(enc) ? 1 : 0;
    }
    if (w == 0) P = ge_neg(P);
    int32_t* tab = &sh.tab[w][quad][0];
    quad_table(tab, P, q);
    if (w == 0) CPZ_SMALL_STAMP(2);
    __syncthreads();  // A: wave 2's digits; the quad's table fields
    if (w == 0) CPZ_SMALL_STAMP(3);
    // ---- the half-length Straus loop over one point ---------------------------------
    uint32_t d[4];
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = sh.dig[j][4 * w + k];
    // wave 1: [|v|] (v < 0 ? R : -R) = [+-|v|] R from the table of +R
    const bool flip = w == 1 && !(sh.meta[j] & 1u);
#pragma unroll 1
    for (int jj = 0; jj < 4; jj++) {
      const uint32_t wd = d[3 - jj];
#pragma unroll 1
      for (int m = 7; m >= 0; m--) {
        int dd = ((int32_t)(wd << (28 - 4 * m))) >> 28;
        dd = flip ? -dd : dd;
        const fe ex = quad_lookup(tab, dd, q);
        if (jj != 0 || m != 7) acc = p3_dbl_n_quad(acc, 4, q);
        acc = ge_add_quad(acc, cached_of_field(ex), q);
      }
    }
    if (q == 0) sh.part[w][quad] = acc;
    if (w == 0) CPZ_SMALL_STAMP(4);
  } else {
    // ---- wave 2: challenge, response checks, split, digits ------------------------------
    uint32_t dg[16], meta;
    proof_digits(dg, meta, a, ca, ii, (l & 7) == 0, &sh.sponge[0][0], j, kSmallProofs);
    if ((l & 7) == 0) {
#pragma unroll
      for (int k = 0; k < 16; k++) sh.dig[j][k] = dg[k];
      sh.meta[j] = meta;
    }
    uint32_t sd[8];
    CPZ_SMALL_STAMP(7);
    __syncthreads();  // A
    // the digits as the proof's first lane wrote them (its lanes differ on the byte-wise path)
#pragma unroll
    for (int k = 0; k < 8; k++) sd[k] = sh.dig[j][8 + k];
    // ---- [s'] B of equation e -------------------------------------------------------------
    if (a.vtab) {  // variable bases: 16 radix-256 windows of s' on B and of s' >> 128 on 2^128 B
      const ge_niels* gt = a.vtab + e * kNielsEntries;
      const ge_niels* gt2 = a.vtab + (2 + e) * kNielsEntries;
#pragma unroll 1
      for (int b = 15; b >= 0; b--) {
        const int dg = (int32_t)(sd[b >> 2] << (24 - 8 * (b & 3))) >> 24;
        const int dg2 = (int32_t)(sd[4 + (b >> 2)] << (24 - 8 * (b & 3))) >> 24;
        if (b != 15) acc = p3_dbl_n_quad(acc, 8, q);
        acc = ge_add_quad(acc, cached_of_field(quad_niels_lookup(gt, dg, q)), q);
        acc = ge_add_quad(acc, cached_of_field(quad_niels_lookup(gt2, dg2, q)), q);
      }
    } else {
      const CombTable comb{a.comb + (e ? kCombPerBase : 0)};
#pragma unroll 1
      for (int k = 0; k < 16; k++) {
        const int dgt = (int32_t)(sd[k >> 1] << (16 - 16 * (k & 1))) >> 16;
        const ge_niels nl = comb.lookup(k, dgt);
        ge_cached cc;
        cc.YpX = nl.ypx;
        cc.YmX = nl.ymx;
        cc.T2d = nl.xy2d;
        cc.Z = fe_one();
        acc = ge_add_quad(acc, cc, q);
      }
    }
    if (q == 0) sh.part[2][quad] = acc;
    CPZ_SMALL_STAMP(8);
  }
  __syncthreads();  // B: the three partial sums
  if (w != 0) return;
  CPZ_SMALL_STAMP(5);
  // ---- wave 0: Q = [u] (-Y) + [|v|] (-+R) + [s'] B, identity (mod E[4]) per equation ------
  acc = ge_add_quad(acc, sh.part[1][quad], q);
  acc = ge_add_quad(acc, sh.part[2][quad], q);
  int eq = ristretto_is_identity(acc) ? 1 : 0;
  eq &= __shfl_xor(eq, 4);
  if ((l & 7) != 0 || !live) return;
  const int q0 = 2 * j;
  const bool bad = sh.bad[0][q0] | sh.bad[0][q0 + 1] | sh.bad[1][q0] | sh.bad[1][q0 + 1];
  const bool rid = sh.rid[q0] | sh.rid[q0 + 1];
  const uint8_t st_s = (uint8_t)(sh.meta[j] >> 8);
  uint8_t st;
  if (bad) st = kStBadPoint;
  else if (st_s == kStBadScalar) st = kStBadScalar;
  else if (rid && !a.eq_only) st = kStIdentity;
  else if (st_s == kStZeroS) st = kStZeroS;
  else if (st_s == kStBadChallenge) st = kStBadScalar;
  else st = eq ? kStOk : kStEqFail;
  a.status[i] = st;
#if defined(CPZ_CLOCK_PROBE)
  CPZ_SMALL_STAMP(6);
  if (stamps) stamps[10] = __builtin_amdgcn_s_memrealtime();
#endif
#undef CPZ_SMALL_STAMP
}

hipError_t launch_verify_small(const VerifyArgs& a, const ChallengeArgs& ca, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  if (a.pre || a.blocks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_verify_small, dim3((unsigned)((a.n + kSmallProofs - 1) / kSmallProofs)), dim3(64 * 3), 0, st,
                     a, ca);
  return hipGetLastError();
}


hipError_t launch_verify_each(const VerifyArgs& a, int grid, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const int64_t slots = a.blocks ? a.nblocks * (int64_t)a.block_proofs : a.n;
  if (a.vtab && (a.pre || slots > a.quad_max)) return hipErrorInvalidValue;  // no comb: eight-lane kernel only
  if (a.vtab) {
    hipLaunchKernelGGL((k_verify_quad<false, true>), dim3((unsigned)((slots + 31) / 32)), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  if (CPZ_VERIFY_QUAD && slots <= a.quad_max) {  // small batches: eight lanes per proof
    const unsigned g = (unsigned)((slots + 31) / 32);
    if (a.pre)
      hipLaunchKernelGGL((k_verify_quad<true, false>), dim3(g), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((k_verify_quad<false, false>), dim3(g), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  if (a.pre)
    hipLaunchKernelGGL(k_verify_prepared, dim3(grid), dim3(kVerifyBlock), 0, st, a);
  else
    hipLaunchKernelGGL(k_verify_each, dim3(grid), dim3(kVerifyBlock), 0, st, a);
  return hipGetLastError();
}


hipError_t launch_prove_points(const ProveArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const int64_t blocks = (a.n + kVerifyBlock - 1) / kVerifyBlock;
  hipLaunchKernelGGL(k_prove_points, dim3((unsigned)blocks), dim3(kVerifyBlock), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_parse_proofs(const ParseArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_parse_proofs, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_response_prep(int64_t n, const uint32_t* s, const uint32_t* c_in, uint32_t* c_out, uint8_t* status,
                                int eq_only, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_response_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, s, c_in, c_out, status,
                     eq_only);
  return hipGetLastError();
}

hipError_t launch_prove_response(const ProveArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const int64_t blocks = (a.n + 255) / 256;
  hipLaunchKernelGGL(k_prove_response, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace cpz
