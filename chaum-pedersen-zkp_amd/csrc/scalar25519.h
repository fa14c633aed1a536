// Scalars modulo l = 2^252 + 27742317777372353535851937790883648493 (8 x u32, little-endian).
//
// Replaces curve25519-dalek 4.1.3's Scalar as reached from the reference:
//   Scalar::from_canonical_bytes   (ristretto.rs:94-112)  -> sc_is_canonical
//   from_bytes_mod_order_wide      (ristretto.rs:146-150, transcript.rs:67-71) -> sc_reduce_wide
//   scalar_mul_scalar / scalar_add (ristretto.rs:198-200, prover/mod.rs:126-131) -> sc_mul / sc_add
//   scalar_is_zero                 (ristretto.rs:219-221) -> sc_is_zero
// plus the signed-digit recodings the scalar-multiplication loops consume.
// Reduction is Barrett (HAC 14.42, b = 2^32, k = 8, mu = floor(2^512 / l)); every
// 32x32 partial product is one v_mad_u64_u32.
#pragma once
#include <math.h>

#include "fe25519.h"

namespace cpz {

struct sc {
  uint32_t w[8];
};

CPZ_HD uint32_t SC_L(int i) {
  const uint32_t l[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                         0x00000000u, 0x00000000u, 0x00000000u, 0x10000000u};
  return l[i];
}

CPZ_HD uint32_t SC_MU(int i) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  return mu[i];
}

// a >= l ?
CPZ_HD bool sc_geq_l9(const uint32_t a[9]) {
  if (a[8] != 0) return true;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a[i] - SC_L(i) - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow == 0;
}

CPZ_HD void sc_sub_l9(uint32_t a[9]) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t d = (uint64_t)a[i] - (i < 8 ? SC_L(i) : 0u) - borrow;
    a[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
}

// s < l ?  (Scalar::from_canonical_bytes accepts exactly these.)
CPZ_HD bool sc_is_canonical(const uint32_t s[8]) {
  uint32_t t[9];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = s[i];
  t[8] = 0;
  return !sc_geq_l9(t);
}

CPZ_HD bool sc_is_zero(const uint32_t s[8]) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) acc |= s[i];
  return acc == 0;
}

// r = x mod l for a 512-bit x (16 words).
CPZ_HD sc sc_reduce_wide(const uint32_t x[16]) {
  // q1 = x >> 224 (9 words); q3 = (q1 * mu) >> 288.
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t t = (uint64_t)x[7 + i] * SC_MU(j) + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * l) mod 2^288.
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j < 9) {
        const uint64_t t = (uint64_t)q2[9 + i] * SC_L(j) + r2[i + j] + carry;
        r2[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
    if (i + 8 < 9) r2[i + 8] = (uint32_t)(r2[i + 8] + carry);
  }
  // r = (x mod 2^288) - r2 (mod 2^288); then at most two subtractions of l.
  uint32_t r[9];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  if (sc_geq_l9(r)) sc_sub_l9(r);
  if (sc_geq_l9(r)) sc_sub_l9(r);
  sc out;
#pragma unroll
  for (int i = 0; i < 8; i++) out.w[i] = r[i];
  return out;
}

// (a * b) mod l.
CPZ_HD sc sc_mul(const sc& a, const sc& b) {
  uint32_t p[16];
#pragma unroll
  for (int i = 0; i < 16; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)a.w[i] * b.w[j] + p[i + j] + carry;
      p[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    p[i + 8] = (uint32_t)carry;
  }
  return sc_reduce_wide(p);
}

// (a + b) mod l, a and b canonical.
CPZ_HD sc sc_add(const sc& a, const sc& b) {
  uint32_t t[9];
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t s = (uint64_t)a.w[i] + b.w[i] + carry;
    t[i] = (uint32_t)s;
    carry = s >> 32;
  }
  t[8] = (uint32_t)carry;
  if (sc_geq_l9(t)) sc_sub_l9(t);
  sc out;
#pragma unroll
  for (int i = 0; i < 8; i++) out.w[i] = t[i];
  return out;
}

// (l - a) mod l.
CPZ_HD sc sc_neg(const sc& a) {
  if (sc_is_zero(a.w)) return a;
  sc out;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)SC_L(i) - a.w[i] - borrow;
    out.w[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  return out;
}

// Signed radix-16 recoding of a scalar < 2^255: 64 digits in [-8, 7], packed as 4-bit
// two's-complement nibbles, digit i in bits 4(i%8) of word i/8.
CPZ_HD void sc_recode_radix16(uint32_t out[8], const uint32_t s[8]) {
  int32_t carry = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t packed = 0;
#pragma unroll
    for (int m = 0; m < 8; m++) {
      const int32_t n = (int32_t)((s[j] >> (4 * m)) & 15u) + carry;
      carry = (n + 8) >> 4;
      const int32_t d = n - (carry << 4);
      packed |= ((uint32_t)d & 15u) << (4 * m);
    }
    out[j] = packed;
  }
}

// Signed radix-256 recoding of a scalar < 2^253: 32 digits in [-128, 127] packed as
// bytes, digit i in byte i%4 of word i/4.
CPZ_HD void sc_recode_radix256(uint32_t out[8], const uint32_t s[8]) {
  int32_t carry = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t packed = 0;
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int32_t n = (int32_t)((s[j] >> (8 * m)) & 255u) + carry;
      carry = (n + 128) >> 8;
      const int32_t d = n - (carry << 8);
      packed |= ((uint32_t)d & 255u) << (8 * m);
    }
    out[j] = packed;
  }
}

// Signed radix-2^16 recoding of a scalar < 2^253: 16 digits in [-2^15, 2^15 - 1] packed
// as int16 halves, digit i in half i%2 of word i/2 (the fixed-base comb of scalarmul.h).
CPZ_HD void sc_recode_radix65536(uint32_t out[8], const uint32_t s[8]) {
  int32_t carry = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t packed = 0;
#pragma unroll
    for (int m = 0; m < 2; m++) {
      const int32_t n = (int32_t)((s[j] >> (16 * m)) & 0xffffu) + carry;
      carry = (n + 32768) >> 16;
      const int32_t d = n - (carry << 16);
      packed |= ((uint32_t)d & 0xffffu) << (16 * m);
    }
    out[j] = packed;
  }
}

// ---------------------------------------------------------------------------------------
// Half-size decomposition of a challenge (2-dimensional lattice reduction by the partial
// extended Euclidean algorithm, cf. T. Pornin, "Optimized Lattice Basis Reduction In
// Dimension 2, and Fast Schnorr and EdDSA Signature Verification", 2020).
//
// Finds u >= 0 and v != 0 with  v c == u (mod l)  and  u, |v| < 3 * 2^125.  The Euclid
// remainders r_k = s_k l + t_k c decrease; the first r_k below T = 3 * 2^125 gives
// u = r_k, v = t_k, and |t_k| <= l / r_{k-1} <= l / T < 2^127 / 1.5 (from the identity
// r_{k-1} |t_k| + r_k |t_{k-1}| = l).  Both fit 32 signed radix-16 digits with no carry
// out (top nibble <= 5, + carry <= 6).
//
// Quotients come from f64 estimates of r0 / r1 shrunk by a 2^-46 relative margin, so a
// step never subtracts more than the true quotient: one Euclid step may take several
// partial steps, but the (r, t) sequence at each swap is the exact Euclid sequence and
// (u, v) is unique.  Estimates >= 2^62 are applied as q * 2^k with a shifted divisor.
// ---------------------------------------------------------------------------------------
CPZ_HD double words8_to_f64(const uint32_t a[8]) {
  double d = (double)a[7];
#pragma unroll
  for (int j = 6; j >= 0; j--) d = d * 4294967296.0 + (double)a[j];
  return d;
}

// a < b (unsigned 256-bit)
CPZ_HD bool words8_lt(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t d = (uint64_t)a[j] - b[j] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow != 0;
}

// out = a << k (mod 2^256), 0 <= k < 256; selects instead of a dynamically indexed array.
CPZ_HD void words8_shl(uint32_t out[8], const uint32_t a[8], int k) {
  const int kl = k >> 5, kb = k & 31;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t hi = 0, lo = 0;
#pragma unroll
    for (int m = 0; m < 8; m++) {
      if (m == kl) {
        hi = j - m >= 0 ? a[j - m >= 0 ? j - m : 0] : 0u;
        lo = j - m - 1 >= 0 ? a[j - m - 1 >= 0 ? j - m - 1 : 0] : 0u;
      }
    }
    out[j] = kb ? ((hi << kb) | (lo >> (32 - kb))) : hi;
  }
}

// r -= q x (mod 2^256), q < 2^64.
CPZ_HD void words8_submul(uint32_t r[8], const uint32_t x[8], uint64_t q) {
  const uint32_t q0 = (uint32_t)q, q1 = (uint32_t)(q >> 32);
  uint32_t p[8];
  uint64_t carry = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t t = (uint64_t)x[j] * q0 + carry;
    p[j] = (uint32_t)t;
    carry = t >> 32;
  }
  carry = 0;
#pragma unroll
  for (int j = 1; j < 8; j++) {
    const uint64_t t = (uint64_t)x[j - 1] * q1 + p[j] + carry;
    p[j] = (uint32_t)t;
    carry = t >> 32;
  }
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t d = (uint64_t)r[j] - p[j] - borrow;
    r[j] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
}

CPZ_HD bool half_below(const uint32_t r[8]) {
  return (r[4] | r[5] | r[6] | r[7]) == 0 && r[3] < 0x60000000u;  // r < 3 * 2^125
}

// Bit length of a 256-bit value (0 for 0).
CPZ_HD int words8_bitlen(const uint32_t a[8]) {
  int n = 0;
#pragma unroll
  for (int j = 0; j < 8; j++)
    if (a[j]) n = 32 * j + 32 - __builtin_clz(a[j]);
  return n;
}

// floor(a / 2^sh) mod 2^64 for 0 <= sh < 192 (selects, no dynamically indexed array).
CPZ_HD uint64_t words8_extract64(const uint32_t a[8], int sh) {
  const int w = sh >> 5, b = sh & 31;
  uint32_t x0 = 0, x1 = 0, x2 = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (j == w) x0 = a[j];
    if (j == w + 1) x1 = a[j];
    if (j == w + 2) x2 = a[j];
  }
  const uint64_t lo = ((uint64_t)x1 << 32) | x0;
  return b ? (lo >> b) | ((uint64_t)x2 << (64 - b)) : lo;
}

// out = a x - b y (mod 2^256) for 32-bit a, b; x, y two's complement.
CPZ_HD void words8_mulsub2(uint32_t out[8], uint32_t a, const uint32_t x[8], uint32_t b, const uint32_t y[8]) {
  uint64_t cx = 0, cy = 0;
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t px = (uint64_t)x[j] * a + cx, py = (uint64_t)y[j] * b + cy;
    cx = px >> 32;
    cy = py >> 32;
    const uint64_t d = (uint64_t)(uint32_t)px - (uint32_t)py - borrow;
    out[j] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
}

// out = u x + v y (mod 2^256) for a cofactor row (u, v): u v <= 0 and |u|, |v| < 2^31.
CPZ_HD void words8_row(uint32_t out[8], int64_t u, int64_t v, const uint32_t x[8], const uint32_t y[8]) {
  const uint32_t au = (uint32_t)(u < 0 ? -u : u), av = (uint32_t)(v < 0 ? -v : v);
  if (u > 0 || v < 0)
    words8_mulsub2(out, au, x, av, y);
  else
    words8_mulsub2(out, av, y, au, x);
}

// One exact Euclid step (r0, r1, t0, t1 as in sc_half_split), partial when the f64
// quotient estimate is huge.
CPZ_HD void half_split_step(uint32_t r0[8], uint32_t r1[8], uint32_t t0[8], uint32_t t1[8]) {
  double qf = words8_to_f64(r0) / words8_to_f64(r1);
  int k = 0;
  if (qf >= 0x1p62) {
    k = ilogb(qf) - 61;
    qf = ldexp(qf, -k);
  }
  uint64_t q = (uint64_t)(qf * (1.0 - 0x1p-46));
  if (q == 0) q = 1;
  if (k) {
    uint32_t xs[8], ts[8];
    words8_shl(xs, r1, k);
    words8_shl(ts, t1, k);
    words8_submul(r0, xs, q);
    words8_submul(t0, ts, q);
  } else {
    words8_submul(r0, r1, q);
    words8_submul(t0, t1, q);
  }
  if (words8_lt(r0, r1)) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t x = r0[j]; r0[j] = r1[j]; r1[j] = x;
      x = t0[j]; t0[j] = t1[j]; t1[j] = x;
    }
  }
}

// c < l canonical.  u, vabs: 4 words each (128-bit); vneg: sign of v.
//
// Lehmer's acceleration of the Euclid loop: the quotients are computed on the top 63 bits
// a = r0 >> sh, b = r1 >> sh with 64-bit integers, accumulating the cofactor matrix
// (u0 v0; u1 v1), and applied to the 256-bit (r, t) once per batch (~30 bits of quotients,
// 4-5 batches instead of ~75 multi-word steps).  A step is taken only while it is provably
// the exact Euclid step of the full numbers: with A_k = u a + v b and |truncation| < 1,
// the full remainder lies within |u| + |v| of 2^sh R, so R >= e2 (+ T >> sh) and
// B - R >= e1 + e2 guarantee T <= r_full < previous r_full -- the quotient is the true
// one and the batch never passes the first remainder below T.  The last steps (and any
// huge quotient) go through the single-step path, so (u, v) is exactly the Euclid pair.
CPZ_HD void sc_half_split(const uint32_t c[8], uint32_t u[4], uint32_t vabs[4], bool& vneg) {
  uint32_t r0[8], r1[8], t0[8], t1[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    r0[j] = SC_L(j);
    r1[j] = c[j];
    t0[j] = 0;
    t1[j] = j == 0 ? 1u : 0u;
  }
#pragma unroll 1
  while (!half_below(r1)) {
    const int sh = words8_bitlen(r0) - 63;  // r0 >= r1 >= T > 2^126: sh > 63
    uint64_t A = words8_extract64(r0, sh), B = words8_extract64(r1, sh);
    const uint64_t tsh = sh <= 125 ? (3ull << (125 - sh)) : 0ull;  // T >> sh
    int64_t u0 = 1, v0 = 0, u1 = 0, v1 = 1;
    int steps = 0;
#pragma unroll 1
    while (B != 0) {
      const double qf = (double)A / (double)B;
      if (qf >= 0x1p30) break;
      uint64_t q = (uint64_t)qf;
      uint64_t qb = q * B;
      while (qb > A) {
        q--;
        qb -= B;
      }
      uint64_t R = A - qb;
      while (R >= B) {
        q++;
        R -= B;
      }
      const int64_t u2 = u0 - (int64_t)q * u1, v2 = v0 - (int64_t)q * v1;
      const int64_t au2 = u2 < 0 ? -u2 : u2, av2 = v2 < 0 ? -v2 : v2;
      const int64_t au1 = u1 < 0 ? -u1 : u1, av1 = v1 < 0 ? -v1 : v1;
      if (au2 >= (1ll << 31) || av2 >= (1ll << 31)) break;
      const uint64_t e2 = (uint64_t)(au2 + av2) + 1, e1 = (uint64_t)(au1 + av1) + 1;
      if (R < e2 + tsh || B - R < e1 + e2) break;
      A = B;
      B = R;
      u0 = u1;
      v0 = v1;
      u1 = u2;
      v1 = v2;
      steps++;
    }
    if (steps == 0) {
      half_split_step(r0, r1, t0, t1);
    } else {
      uint32_t nr0[8], nr1[8], nt0[8], nt1[8];
      words8_row(nr0, u0, v0, r0, r1);
      words8_row(nr1, u1, v1, r0, r1);
      words8_row(nt0, u0, v0, t0, t1);
      words8_row(nt1, u1, v1, t0, t1);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        r0[j] = nr0[j];
        r1[j] = nr1[j];
        t0[j] = nt0[j];
        t1[j] = nt1[j];
      }
    }
  }
  vneg = (t1[7] >> 31) != 0;
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    u[j] = r1[j];
    // |t1| = vneg ? 0 - t1 : t1
    const uint64_t d = (uint64_t)0 - t1[j] - borrow;
    borrow = (uint32_t)(d >> 63);
    vabs[j] = vneg ? (uint32_t)d : t1[j];
  }
}

// 1 / x to ~1 ulp (v_rcp_f32 on the device; the correction steps below absorb the error).
CPZ_HD float f32_rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}

// The same split with 31-bit Lehmer windows (k_verify_wide's wave 4, one challenge per wave).
// On a lone wave sc_half_split's inner step -- 64-bit quotient, cofactor and exactness
// arithmetic, each a chain of dependent 32-bit halves -- takes ~1000 shader cycles whatever
// the quotient's source (tools/ubench/w4_parts.hip: 73 K cycles for ~72 steps).  Here a step is
// 32-bit work: the quotient from an f32 reciprocal (exact after at most one correction for
// q < 2^15), cofactors below 2^15, the same two exactness conditions (T / 2^sh rounded up),
// so the same Euclid pair (u, v); twice the batches (~15 bits each), each batch the same four
// 8-word rows.
//
// kLanes (device, every lane of the wave splitting the same challenge): a batch's four 8-word
// rows are computed on lanes 0..3 at once and read back with v_readlane, instead of one after
// another on every lane.
template <bool kLanes = false>
CPZ_HD void sc_half_split32(const uint32_t c[8], uint32_t u[4], uint32_t vabs[4], bool& vneg) {
  uint32_t r0[8], r1[8], t0[8], t1[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    r0[j] = SC_L(j);
    r1[j] = c[j];
    t0[j] = 0;
    t1[j] = j == 0 ? 1u : 0u;
  }
#pragma unroll 1
  while (!half_below(r1)) {
    const int sh = words8_bitlen(r0) - 31;  // r0 >= r1 >= T > 2^126: sh > 95
    uint32_t A = (uint32_t)words8_extract64(r0, sh), B = (uint32_t)words8_extract64(r1, sh);
    // ceil(T / 2^sh), T = 3 * 2^125
    const uint32_t tsh = sh <= 125 ? (3u << (125 - sh)) : (sh == 126 ? 2u : 1u);
    int32_t u0 = 1, v0 = 0, u1 = 0, v1 = 1;
    int steps = 0;
    // Each step is straight-line selects and ONE exit test: a lone wave pays ~40 cycles per
    // divergent branch, and the step's five early exits were most of its time.
#pragma unroll 1
    for (;;) {
      // q = floor(A / B): the f32 estimate is within one of it for q < 2^15 (relative error
      // < 2^-21); larger quotients (and B = 0) end the batch
      const uint32_t qe = (uint32_t)((float)A * f32_rcp((float)(B | (B == 0u))));
      const uint32_t qb0 = qe * B;  // <= A + B < 2^32 when qe is within one of q
      const bool over = qb0 > A;
      const uint32_t q1 = over ? qe - 1u : qe, qb = over ? qb0 - B : qb0;
      const uint32_t R0 = A - qb;
      const bool under = R0 >= B;
      const uint32_t q = under ? q1 + 1u : q1, R = under ? R0 - B : R0;
      const int32_t u2 = u0 - (int32_t)q * u1, v2 = v0 - (int32_t)q * v1;
      const int32_t au2 = u2 < 0 ? -u2 : u2, av2 = v2 < 0 ? -v2 : v2;
      const int32_t au1 = u1 < 0 ? -u1 : u1, av1 = v1 < 0 ? -v1 : v1;
      const uint32_t e2 = (uint32_t)(au2 + av2) + 1, e1 = (uint32_t)(au1 + av1) + 1;
      const bool go = (B != 0u) & (qe < (1u << 15)) & (au2 < (1 << 15)) & (av2 < (1 << 15)) & (R >= e2 + tsh) &
                      (B - R >= e1 + e2);
      if (!go) break;
      A = B;
      B = R;
      u0 = u1;
      v0 = v1;
      u1 = u2;
      v1 = v2;
      steps++;
    }
    if (steps == 0) {
      half_split_step(r0, r1, t0, t1);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (kLanes) {
        // lane k & 3 computes row k: (u0, v0 | u1, v1) x (r0, r1 | t0, t1); branch-free form of
        // words8_row (the rows' signs differ between lanes)
        const int k = (int)(threadIdx.x & 3);
        const int32_t cu = (k & 1) ? u1 : u0, cv = (k & 1) ? v1 : v0;
        const bool pos = cu > 0 || cv < 0;
        const uint32_t au = (uint32_t)(cu < 0 ? -cu : cu), av = (uint32_t)(cv < 0 ? -cv : cv);
        uint32_t X[8], Y[8], out[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const uint32_t x = (k & 2) ? t0[j] : r0[j], y = (k & 2) ? t1[j] : r1[j];
          X[j] = pos ? x : y;
          Y[j] = pos ? y : x;
        }
        words8_mulsub2(out, pos ? au : av, X, pos ? av : au, Y);
#pragma unroll
        for (int j = 0; j < 8; j++) {
          r0[j] = __builtin_amdgcn_readlane(out[j], 0);
          r1[j] = __builtin_amdgcn_readlane(out[j], 1);
          t0[j] = __builtin_amdgcn_readlane(out[j], 2);
          t1[j] = __builtin_amdgcn_readlane(out[j], 3);
        }
        continue;
      }
#endif
      uint32_t nr0[8], nr1[8], nt0[8], nt1[8];
      words8_row(nr0, u0, v0, r0, r1);
      words8_row(nr1, u1, v1, r0, r1);
      words8_row(nt0, u0, v0, t0, t1);
      words8_row(nt1, u1, v1, t0, t1);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        r0[j] = nr0[j];
        r1[j] = nr1[j];
        t0[j] = nt0[j];
        t1[j] = nt1[j];
      }
    }
  }
  vneg = (t1[7] >> 31) != 0;
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    u[j] = r1[j];
    const uint64_t d = (uint64_t)0 - t1[j] - borrow;
    borrow = (uint32_t)(d >> 63);
    vabs[j] = vneg ? (uint32_t)d : t1[j];
  }
}

// Signed radix-16 recoding of a value < 6 * 2^124 held in 4 words: 32 digits in [-8, 7],
// packed as in sc_recode_radix16 (no carry out of the top digit for such values).
CPZ_HD void sc_recode_radix16_half(uint32_t out[4], const uint32_t s[4]) {
  int32_t carry = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint32_t packed = 0;
#pragma unroll
    for (int m = 0; m < 8; m++) {
      const int32_t n = (int32_t)((s[j] >> (4 * m)) & 15u) + carry;
      carry = (n + 8) >> 4;
      const int32_t d = n - (carry << 4);
      packed |= ((uint32_t)d & 15u) << (4 * m);
    }
    out[j] = packed;
  }
}

}  // namespace cpz
