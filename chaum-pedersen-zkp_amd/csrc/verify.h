// Per-proof verification logic shared by the GPU kernels (kernels.hip) and the host
// build used by the CPU unit tests of the device library.
//
// Semantics (status precedence) follow the order in which the reference meets each
// rejection for one entry:
//   1. statement / commitment points must decode     -> 2  (Statement built at
//      registration, service.rs:82-86; Proof::from_bytes r1/r2, gadgets.rs:410, 437)
//   2. s must be canonical                           -> 3  (gadgets.rs:460, ristretto.rs:94-112)
//   3. r1, r2 not identity; s != 0                   -> 4  (gadgets.rs:474-482)
//   4. g^s == r1 y1^c  and  h^s == r2 y2^c           -> 0 / 1 (batch.rs:216-228)
#pragma once
#include "ristretto.h"
#include "scalar25519.h"
#include "scalarmul.h"
#include "transcript.h"

namespace cpz {

constexpr uint8_t kStOk = 0, kStEqFail = 1, kStBadPoint = 2, kStBadScalar = 3, kStIdentityOrZero = 4;

CPZ_HD bool words8_zero(const uint32_t w[8]) {
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) acc |= w[k];
  return acc == 0;
}

// Status contributed by the response scalar alone.
CPZ_HD uint8_t response_status(const uint32_t s[8]) {
  if (!sc_is_canonical(s)) return kStBadScalar;
  if (sc_is_zero(s)) return kStIdentityOrZero;
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

// One equation, [s] B - [c] Y == R (ristretto equality), checked through the half-size
// decomposition v c = u (mod l) of the challenge (sc_half_split):
//   Q = [v s mod l] B + [u] (-Y) + [v] (-R)  lies in E[4]   <=>   [s] B - [c] Y == R.
// (Decoded points lie in 2E = Z_l x Z_4; ristretto equality is equality modulo E[4].
// Multiplying by v != 0 (mod l) keeps the Z_l part zero iff it was; [v c] Y and [u] Y,
// [v s] B and [v s mod l] B differ by elements of E[4].)  [v s mod l] B comes from the
// fixed-base comb of B (sdig: radix-2^16 digits).  Also reports whether Y and R decode
// and whether R encodes the identity.
template <class Comb>
CPZ_HD bool check_equation(const uint32_t y[8], const uint32_t r[8], const uint32_t udig[4], const uint32_t vdig[4],
                           bool vneg, const uint32_t sdig[8], const Comb& comb, ge_cached* tab_y, ge_cached* tab_r,
                           bool& decoded, bool& r_identity) {
  {
    ge_p3 P;
    decoded = ristretto_decode(P, y);
    build_cached_table(tab_y, ge_neg(P));
  }
  {
    ge_p3 R;
    decoded = ristretto_decode(R, r) && decoded;
    build_cached_table(tab_r, vneg ? R : ge_neg(R));
  }
  r_identity = words8_zero(r);
  return ristretto_is_identity(straus_half_comb(tab_y, tab_r, comb, udig, vdig, sdig));
}

// Full per-proof outcome given the challenge c (canonical) and the response status st_s.
// comb_g / comb_h: fixed-base combs of g and h; tab_v: 2 * kTableSlots entries of per-proof
// scratch.
template <class Comb>
CPZ_HD uint8_t verify_proof(const uint32_t y1[8], const uint32_t y2[8], const uint32_t r1[8], const uint32_t r2[8],
                            const uint32_t s[8], const uint32_t c[8], uint8_t st_s, const Comb& comb_g,
                            const Comb& comb_h, ge_cached* tab_v) {
  uint32_t udig[4], vdig[4], sdig[8];
  bool vneg;
  {
    uint32_t u[4], va[4];
    sc_half_split(c, u, va, vneg);
    sc_recode_radix16_half(udig, u);
    sc_recode_radix16_half(vdig, va);
    sc vs, ss;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      vs.w[k] = k < 4 ? va[k] : 0u;
      ss.w[k] = s[k];
    }
    sc sp = sc_mul(vs, ss);
    if (vneg) sp = sc_neg(sp);
    sc_recode_radix65536(sdig, sp.w);
  }
  bool dec1, dec2, id1, id2;
  const bool eq1 = check_equation(y1, r1, udig, vdig, vneg, sdig, comb_g, tab_v, tab_v + kTableSlots, dec1, id1);
  const bool eq2 = check_equation(y2, r2, udig, vdig, vneg, sdig, comb_h, tab_v, tab_v + kTableSlots, dec2, id2);
  if (!(dec1 && dec2)) return kStBadPoint;
  if (st_s == kStBadScalar) return kStBadScalar;
  if (id1 || id2 || st_s == kStIdentityOrZero) return kStIdentityOrZero;
  return (eq1 && eq2) ? kStOk : kStEqFail;
}

}  // namespace cpz
