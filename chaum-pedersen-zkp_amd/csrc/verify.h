// Per-proof verification logic shared by the GPU kernels (kernels.hip) and the host
// build used by the CPU unit tests of the device library.
//
// Semantics (status precedence) follow the order in which the reference meets each
// rejection for one entry:
//   1. statement / commitment points must decode     -> 2  (Statement built at
//      registration, service.rs:82-86; Proof::from_bytes r1/r2, gadgets.rs:410, 437)
//   2. s must be canonical                           -> 3  (gadgets.rs:460, ristretto.rs:94-112)
//   3. r1, r2 not identity                           -> 4  (gadgets.rs:474-478)
//   4. s != 0                                        -> 5  (gadgets.rs:480-482)
//   5. g^s == r1 y1^c  and  h^s == r2 y2^c           -> 0 / 1 (batch.rs:216-228)
#pragma once
#include "timing_only.h"
#include "ristretto.h"
#include "scalar25519.h"
#include "scalarmul.h"
#include "transcript.h"

// Loops over the two points of an equation and over the two equations stay rolled (one
// copy of the decode / Straus code; unrolling them measured slower).
#define CPZ_EQ_LOOP _Pragma("unroll 1")

namespace cpz {

constexpr uint8_t kStOk = 0, kStEqFail = 1, kStBadPoint = 2, kStBadScalar = 3, kStIdentity = 4, kStZeroS = 5;
// Internal response status (never reported): the caller-supplied challenge of
// cpz_verify_response is not canonical.  It reports kStBadScalar, but only after the entry's
// own decode-level checks (pyoracle.verify_response).
constexpr uint8_t kStBadChallenge = 0x80;

CPZ_HD bool words8_zero(const uint32_t w[8]) {
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) acc |= w[k];
  return acc == 0;
}

// Status contributed by the response scalar alone.  eq_only (cpz_ctx_set_commitment_checks
// off): a zero s is not reported -- the entry stands for a Proof built with Response::new
// (gadgets.rs:278, no zero check), which verify_one judges by its equations alone.
CPZ_HD uint8_t response_status(const uint32_t s[8], bool eq_only = false) {
  if (!sc_is_canonical(s)) return kStBadScalar;
  if (sc_is_zero(s) && !eq_only) return kStZeroS;
  return kStOk;
}

// Merlin transcript tail shared by every entry (transcript.rs:47-71): statement,
// commitment, 64-byte challenge, wide reduction.  `s` must already hold the prefix
// (Transcript::new [+ append_context] + append_parameters).
template <class Acc>
CPZ_HD sc transcript_challenge(Strobe<Acc>& s, const uint32_t y1[8], const uint32_t y2[8], const uint32_t r1[8],
                               const uint32_t r2[8]) {
  s.merlin_append_words("y1", 2, y1);
  s.merlin_append_words("y2", 2, y2);
  s.merlin_append_words("r1", 2, r1);
  s.merlin_append_words("r2", 2, r2);
  uint8_t out[64];
  s.merlin_challenge("challenge", 9, out, 64);
  uint32_t wide[16];
#pragma unroll
  for (int k = 0; k < 16; k++)
    wide[k] = (uint32_t)out[4 * k] | ((uint32_t)out[4 * k + 1] << 8) | ((uint32_t)out[4 * k + 2] << 16) |
              ((uint32_t)out[4 * k + 3] << 24);
  return sc_reduce_wide(wide);
}

// Fixed-schedule transcript tail for entries WITHOUT a context.  Transcript::new +
// append_parameters always leave the sponge at byte 32 (begin 0, flags A): every message
// length is fixed, so the tail's schedule is fixed too -- y1, y2, r1 land at bytes 42, 84,
// 126 of the first segment, the r2 header crosses the rate (166) and forces the first
// permutation, r2 lands at byte 2 of the second segment, the challenge header's C flag
// forces the second permutation, and the 64 challenge bytes are state bytes 0..63.  All
// other bytes the framing XORs in are constants: k1 / k2 (50 words each, from
// challenge_masks).  The state is then 50 registers and no byte is touched individually.
constexpr int kTailPrefixPos = 32, kTailPrefixBegin = 0, kTailPrefixFlags = kFlagA;
constexpr int kTailY1 = 42, kTailY2 = 84, kTailR1 = 126, kTailR2 = 2;

// Fixed-schedule tail for entries whose context is exactly 32 bytes -- every entry of the
// reference service, whose challenge ids are 32 random bytes (service.rs:294-295, appended
// at :373 and in the batch path at :516).  The context follows Transcript::new directly,
// so the sponge enters it at byte 96 (begin 68, flags A); from there every position is
// fixed again: the context at byte 111 of segment 0, g and h (constants, folded into the
// masks) straddle into segment 1, y1 / y2 at bytes 89 / 131 of segment 1, r1 / r2 at 7 / 49
// of segment 2, and the challenge header's C flag forces the third permutation.
constexpr int kC32PrefixPos = 96, kC32PrefixBegin = 68, kC32PrefixFlags = kFlagA;
constexpr int kC32Ctx = 111, kC32Y1 = 89, kC32Y2 = 131, kC32R1 = 7, kC32R2 = 49;

// XOR a 32-byte message into the word image of the sponge at byte offset OFF (any
// alignment: a misaligned message is two funnel-shifted halves per word).
template <int OFF>
CPZ_HD void xor_message(uint32_t st[50], const uint32_t w[8]) {
  static_assert(OFF >= 0 && OFF + 32 <= kStrobeR, "a message must lie inside one sponge segment");
  constexpr int sh = 8 * (OFF % 4);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (sh == 0) {
      st[OFF / 4 + k] ^= w[k];
    } else {
      st[OFF / 4 + k] ^= w[k] << sh;
      st[OFF / 4 + k + 1] ^= w[k] >> (32 - sh);
    }
  }
}

CPZ_HD void keccak_words(uint32_t st[50]) {
  uint64_t a[25];
#pragma unroll
  for (int l = 0; l < 25; l++) a[l] = (uint64_t)st[2 * l] | ((uint64_t)st[2 * l + 1] << 32);
  keccak_f1600(a);
#pragma unroll
  for (int l = 0; l < 25; l++) {
    st[2 * l] = (uint32_t)a[l];
    st[2 * l + 1] = (uint32_t)(a[l] >> 32);
  }
}

// The permutation the fixed-schedule tails apply to their 50-word sponge image: Keccak-f on
// the image's registers (every lane its own sponge), or a caller's (k_verify_wide's wave 4
// spreads one sponge over the lanes of its wave, kernels.hip PermRows).
struct PermRegs {
  CPZ_HDM void operator()(uint32_t st[50]) const { keccak_words(st); }
};

template <class Perm = PermRegs>
CPZ_HD sc challenge_fixed(const uint32_t prefix[50], const uint32_t k1[50], const uint32_t k2[50],
                          const uint32_t y1[8], const uint32_t y2[8], const uint32_t r1[8], const uint32_t r2[8],
                          const Perm& perm = Perm()) {
  uint32_t st[50];
#pragma unroll
  for (int w = 0; w < 50; w++) st[w] = prefix[w] ^ k1[w];
  xor_message<kTailY1>(st, y1);
  xor_message<kTailY2>(st, y2);
  xor_message<kTailR1>(st, r1);
  perm(st);
#pragma unroll
  for (int w = 0; w < 50; w++) st[w] ^= k2[w];
  xor_message<kTailR2>(st, r2);
  perm(st);
  return sc_reduce_wide(st);  // challenge bytes 0..63 = state words 0..15
}

// 32-byte-context tail: prefix = the state after Transcript::new, m = the three segments'
// framing masks (challenge_masks_ctx32, g and h included), ctx = the context as 8 words.
template <class Perm = PermRegs>
CPZ_HD sc challenge_fixed_ctx32(const uint32_t prefix[50], const uint32_t m[3][50], const uint32_t ctx[8],
                                const uint32_t y1[8], const uint32_t y2[8], const uint32_t r1[8],
                                const uint32_t r2[8], const Perm& perm = Perm()) {
  uint32_t st[50];
#pragma unroll
  for (int w = 0; w < 50; w++) st[w] = prefix[w] ^ m[0][w];
  xor_message<kC32Ctx>(st, ctx);
  perm(st);
#pragma unroll
  for (int w = 0; w < 50; w++) st[w] ^= m[1][w];
  xor_message<kC32Y1>(st, y1);
  xor_message<kC32Y2>(st, y2);
  perm(st);
#pragma unroll
  for (int w = 0; w < 50; w++) st[w] ^= m[2][w];
  xor_message<kC32R1>(st, r1);
  xor_message<kC32R2>(st, r2);
  perm(st);
  return sc_reduce_wide(st);
}

template <class Acc>
CPZ_HD sc transcript_challenge(Strobe<Acc>& s, const uint32_t y1[8], const uint32_t y2[8], const uint32_t r1[8],
                               const uint32_t r2[8]);

CPZ_HD void mask_words(uint32_t out[50], const uint8_t m[200]) {
  for (int w = 0; w < 50; w++)
    out[w] = (uint32_t)m[4 * w] | ((uint32_t)m[4 * w + 1] << 8) | ((uint32_t)m[4 * w + 2] << 16) |
             ((uint32_t)m[4 * w + 3] << 24);
}

// The constant masks of challenge_fixed, derived by running the generic tail over zero
// messages with a recording accessor; false if the schedule is not the expected one (two
// permutations), in which case callers must use the generic path.
CPZ_HD bool challenge_masks(uint32_t k1[50], uint32_t k2[50]) {
  MaskState ms;
  for (int g = 0; g < 3; g++)
    for (int i = 0; i < 200; i++) ms.m[g][i] = 0;
  Strobe<MaskState> s(ms, kTailPrefixPos, kTailPrefixBegin, (uint8_t)kTailPrefixFlags);
  const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  (void)transcript_challenge(s, z, z, z, z);
  if (ms.seg != 2) return false;
  for (int w = 0; w < 50; w++) {
    uint32_t a = 0, b = 0;
    for (int k = 3; k >= 0; k--) {
      a = (a << 8) | ms.m[0][4 * w + k];
      b = (b << 8) | ms.m[1][4 * w + k];
    }
    k1[w] = a;
    k2[w] = b;
  }
  return true;
}

// Transcript::new() (transcript.rs:29-33) on a fresh sponge.
template <class Acc>
CPZ_HD Strobe<Acc> transcript_new(Acc& st) {
  Strobe<Acc> s = strobe_init_merlin(st);
  s.merlin_header("dom-sep", 7, 25);
  s.absorb((const uint8_t*)"Chaum-Pedersen ZKP v1.0.0", 25);
  s.merlin_header("protocol", 8, 27);
  s.absorb((const uint8_t*)"chaum-pedersen-ristretto255", 27);
  return s;
}

template <class Acc>
CPZ_HD void transcript_context(Strobe<Acc>& s, const uint8_t* ctx, uint32_t len) {
  s.merlin_header("context", 7, len);
  for (uint32_t b = 0; b < len; b++) s.absorb_byte(ctx[b]);
}

template <class Acc>
CPZ_HD void transcript_parameters(Strobe<Acc>& s, const uint32_t g[8], const uint32_t h[8]) {
  s.merlin_append_words("generator-g", 11, g);
  s.merlin_append_words("generator-h", 11, h);
}

// The masks of challenge_fixed_ctx32 for generators (g, h): the generic code run from the
// post-Transcript::new position over a zero context and zero messages, recording; false if
// the schedule is not the expected one (three permutations before the challenge bytes).
CPZ_HD bool challenge_masks_ctx32(uint32_t m[3][50], const uint32_t g[8], const uint32_t h[8]) {
  MaskState ms;
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 200; i++) ms.m[k][i] = 0;
  Strobe<MaskState> s(ms, kC32PrefixPos, kC32PrefixBegin, (uint8_t)kC32PrefixFlags);
  const uint8_t zc[32] = {0};
  const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  transcript_context(s, zc, 32);
  transcript_parameters(s, g, h);
  (void)transcript_challenge(s, z, z, z, z);
  if (ms.seg != 3) return false;
  for (int k = 0; k < 3; k++) mask_words(m[k], ms.m[k]);
  return true;
}

// One equation, [s] B - [c] Y == R (ristretto equality), checked through the half-size
// decomposition v c = u (mod l) of the challenge (sc_half_split):
//   Q = [v s mod l] B + [u] (-Y) + [v] (-R)  lies in E[4]   <=>   [s] B - [c] Y == R.
// (Decoded points lie in 2E = Z_l x Z_4; ristretto equality is equality modulo E[4].
// Multiplying by v != 0 (mod l) keeps the Z_l part zero iff it was; [v c] Y and [u] Y,
// [v s] B and [v s mod l] B differ by elements of E[4].)  [v s mod l] B comes from the
// fixed-base comb of B (sdig: radix-2^16 digits).  Also reports whether Y and R decode
// and whether R encodes the identity.
// The affine point P from the affine Niels form of -P that the RLC prepare stores (rlc.hip):
// -P = (-x, y), so q.ypx = y - x and q.ymx = y + x:  x = (q.ymx - q.ypx) / 2, y = (q.ypx +
// q.ymx) / 2, T = x y (3 multiplications instead of a decode's inverse square root).
CPZ_HD ge_p3 affine_from_neg_niels(const ge_niels& q) {
  ge_p3 P;
  P.X = fe_mul(fe_sub(q.ymx, q.ypx), FE_INV2());
  P.Y = fe_mul(fe_add(q.ypx, q.ymx), FE_INV2());
  P.Z = fe_one();
  P.T = fe_mul(P.X, P.Y);
  return P;
}

CPZ_HD ge_niels niels_load(const ge_niels* p) {
  ge_niels r;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* s = reinterpret_cast<const uint4*>(p);
  uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
  for (int v = 0; v < (int)(sizeof(ge_niels) / 16); v++) d[v] = s[v];
#else
  r = *p;
#endif
  return r;
}

// kPre: the points were decoded already (pre_y / pre_r: Niels of -Y / -R from the RLC
// prepare) and the entry's decode-level status is 0, so nothing is decoded here.
template <bool kPre, class Comb, class Dig>
CPZ_HD bool check_equation(const Dig& y, const Dig& r, const ge_niels* pre_y, const ge_niels* pre_r,
                           const Dig& udig, const Dig& vdig, bool vneg, const Dig& sdig, const Comb& comb,
                           const SlabTable& tab_y, const SlabTable& tab_r, bool& decoded, bool& r_identity) {
  // One copy of the decode + table code for both points (a rolled loop): the kernel's
  // instruction footprint, not its arithmetic, is what the 64 KB instruction cache sees.
  decoded = true;
CPZ_EQ_LOOP
  for (int k = 0; k < 2; k++) {
    ge_p3 P;
    if constexpr (kPre) {
      P = affine_from_neg_niels(niels_load(k ? pre_r : pre_y));
    } else {
      uint32_t w[8];
#pragma unroll
      for (int q = 0; q < 8; q++) w[q] = k ? r[q] : y[q];
      decoded = ristretto_decode(P, w) && decoded;
    }
    build_cached_table(k ? tab_r : tab_y, (k && vneg) ? P : ge_neg(P));
  }
  if constexpr (kPre) {
    r_identity = false;
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) acc |= r[q];
    r_identity = acc == 0;
  }
#if defined(CPZ_EXP_EXTRA_INV)
  // timing experiment only (timing_only.h: wrong verdicts): one field inversion per equation
  ge_p1p1 q = straus_half_comb(tab_y, tab_r, comb, udig, vdig, sdig);
  q.X = fe_mul(q.X, fe_invert(q.Z));
  return ristretto_is_identity(q);
#else
  return ristretto_is_identity(straus_half_comb(tab_y, tab_r, comb, udig, vdig, sdig));
#endif
}

// Full per-proof outcome given the challenge c (canonical) and the response status st_s.
// comb_g / comb_h: fixed-base combs of g and h; tab_v: 2 * kTableSlots entries of per-proof
// scratch (the y table, then the r table); dig: 16 words of digit storage at stride dstride
// (u: words 0-3, |v|: 4-7, v s mod l: 8-15).
// rows: the encodings y1, y2, r1, r2 (words at rows[4 q + ...], see DigitRef: the verify kernel
// stages them in LDS so that no per-row address stays live in registers); pre (kPre only):
// the entry's 4 prepared Niels points (-r1, -y1, -r2, -y2), st_s its decode-level status,
// which must be 0.  eq_only: an identity commitment is not reported (Commitment::new,
// gadgets.rs:252, has no identity check; verify_one, batch.rs:185-231, checks the equations
// only).
template <bool kPre = false, class Comb>
CPZ_HD uint8_t verify_proof(const DigitRef& y1, const DigitRef& y2, const DigitRef& r1, const DigitRef& r2,
                            const uint32_t s[8], const uint32_t c[8], uint8_t st_s, const Comb& comb_g,
                            const Comb& comb_h, const SlabTable& tab_v, uint32_t* dig, int dstride,
                            const ge_niels* pre = nullptr, bool eq_only = false) {
  bool vneg;
#if defined(CPZ_EXP_NOSPLIT)
  // timing experiment only (wrong verdicts, timing_only.h): the challenge split, v s and the
  // recodings skipped
  vneg = c[7] & 1;
  for (int k = 0; k < 8; k++) {
    dig[k * dstride] = c[k];
    dig[(8 + k) * dstride] = s[k];
  }
  if (0)
#endif
  {
    uint32_t u[4], va[4], w[8];
    sc_half_split(c, u, va, vneg);
    sc_recode_radix16_half(w, u);
    sc_recode_radix16_half(w + 4, va);
    for (int k = 0; k < 8; k++) dig[k * dstride] = w[k];
    sc vs, ss;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      vs.w[k] = k < 4 ? va[k] : 0u;
      ss.w[k] = s[k];
    }
    sc sp = sc_mul(vs, ss);
    if (vneg) sp = sc_neg(sp);
    sc_recode_radix65536(w, sp.w);
    for (int k = 0; k < 8; k++) dig[(8 + k) * dstride] = w[k];
  }
  const DigitRef udig{dig, dstride}, vdig{dig + 4 * dstride, dstride}, sdig{dig + 8 * dstride, dstride};
  // The two equations share one copy of the code too (rolled loop over e).
  bool dec = true, id = false, eq = true;
CPZ_EQ_LOOP
  for (int e = 0; e < 2; e++) {
    bool d, r_id;
    eq = check_equation<kPre>(e ? y2 : y1, e ? r2 : r1, kPre ? pre + 1 + 2 * e : nullptr, kPre ? pre + 2 * e : nullptr,
                              udig, vdig, vneg, sdig, e ? comb_h : comb_g, tab_v, tab_v.shifted(kTableSlots), d,
                              r_id) && eq;
    dec = dec && d;
    id = id || r_id;
  }
  if (!dec) return kStBadPoint;
  if (st_s == kStBadScalar) return kStBadScalar;
  if (id && !eq_only) return kStIdentity;
  if (st_s == kStZeroS) return kStZeroS;
  if (st_s == kStBadChallenge) return kStBadScalar;
  return eq ? kStOk : kStEqFail;
}

}  // namespace cpz
