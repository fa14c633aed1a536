/*
 * cpz_oracle.c -- CPU restatement (plain C) of the reference's verify path.
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY.  Used by tests/ (at-scale checker) and by
 * bench.py's cpu_baseline leg (timed on the GPU box's host cores).  Never linked into,
 * or called by, the product library.
 *
 * What it restates (reference: kobby-pentangeli/chaum-pedersen-zkp, Rust; arithmetic in
 * curve25519-dalek 4.1.3 / merlin 3.0.0, not vendored, algorithms restated from their
 * published descriptions, cf. oracle/pyoracle.py):
 *   - F_p arithmetic in radix 2^51 (dalek's u64 serial backend representation).
 *   - Edwards extended coordinates; dalek's constant-time variable-base scalar
 *     multiplication (radix-16 signed digits, 8-entry ProjectiveNiels table, CT select),
 *     which is what `Ristretto255::scalar_mul` (ristretto.rs:153-155) runs.
 *   - ristretto255 decode / encode / equality (RFC 9496).
 *   - Keccak-f[1600], STROBE-128, Merlin framing, the protocol transcript
 *     (transcript.rs:29-71), wide reduction mod l.
 *   - verify_one (batch.rs:185-231): 6 compressions for the transcript, 4 variable-base
 *     multiplications, 2 additions, 2 ristretto comparisons.
 *   - BatchVerifier::verify (batch.rs:171-318): n == 1 -> verify_one; n >= 2 ->
 *     per-entry weight + challenge, the batch equation AS WRITTEN (batch.rs:271-312,
 *     which omits alpha on y*c), then verify_individually when it fails.
 * Inputs are the same 32-byte encodings the GPU consumes, so each call first decodes
 * the statement and commitment (Statement construction, Proof::from_bytes) exactly as
 * the reference must before an entry can reach the batch.
 *
 * Pinned by tests/test_coracle.py against tests/golden/golden.json (generated from
 * oracle/pyoracle.py, itself pinned against libsodium, RFC 9496 and the merlin KAT).
 */
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------------ */
/* F_p, radix 2^51                                                                      */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint64_t v[5]; } fe51;

static const uint64_t M51 = (1ULL << 51) - 1;

static fe51 f_from(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e) {
  fe51 r = {{a, b, c, d, e}};
  return r;
}
static fe51 f_zero(void) { return f_from(0, 0, 0, 0, 0); }
static fe51 f_one(void) { return f_from(1, 0, 0, 0, 0); }

static fe51 f_weak(fe51 a) {
  uint64_t c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= M51; a.v[0] += 19 * c;
  return a;
}

/* No reduction (as dalek's Add): limbs stay below 2^54, which f_mul / f_sq accept. */
static fe51 f_add(fe51 a, fe51 b) {
  fe51 r;
  for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}

/* a - b + 16p, then weak reduction (inputs below 2^54). */
static fe51 f_sub(fe51 a, fe51 b) {
  fe51 r;
  r.v[0] = a.v[0] + 36028797018963664ULL - b.v[0]; /* 16 * (2^51 - 19) */
  for (int i = 1; i < 5; i++) r.v[i] = a.v[i] + 36028797018963952ULL - b.v[i]; /* 16 * (2^51 - 1) */
  return f_weak(r);
}

static fe51 f_neg(fe51 a) { return f_sub(f_zero(), a); }

static fe51 f_mul(fe51 a, fe51 b) {
  const uint64_t b1 = 19 * b.v[1], b2 = 19 * b.v[2], b3 = 19 * b.v[3], b4 = 19 * b.v[4];
  u128 c0 = (u128)a.v[0] * b.v[0] + (u128)a.v[1] * b4 + (u128)a.v[2] * b3 + (u128)a.v[3] * b2 + (u128)a.v[4] * b1;
  u128 c1 = (u128)a.v[0] * b.v[1] + (u128)a.v[1] * b.v[0] + (u128)a.v[2] * b4 + (u128)a.v[3] * b3 + (u128)a.v[4] * b2;
  u128 c2 = (u128)a.v[0] * b.v[2] + (u128)a.v[1] * b.v[1] + (u128)a.v[2] * b.v[0] + (u128)a.v[3] * b4 + (u128)a.v[4] * b3;
  u128 c3 = (u128)a.v[0] * b.v[3] + (u128)a.v[1] * b.v[2] + (u128)a.v[2] * b.v[1] + (u128)a.v[3] * b.v[0] + (u128)a.v[4] * b4;
  u128 c4 = (u128)a.v[0] * b.v[4] + (u128)a.v[1] * b.v[3] + (u128)a.v[2] * b.v[2] + (u128)a.v[3] * b.v[1] + (u128)a.v[4] * b.v[0];
  fe51 r;
  c1 += (uint64_t)(c0 >> 51); r.v[0] = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); r.v[1] = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); r.v[2] = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); r.v[3] = (uint64_t)c3 & M51;
  uint64_t carry = (uint64_t)(c4 >> 51);
  r.v[4] = (uint64_t)c4 & M51;
  r.v[0] += carry * 19;
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= M51;
  return r;
}

static fe51 f_carry128(u128 c0, u128 c1, u128 c2, u128 c3, u128 c4) {
  fe51 r;
  c1 += (uint64_t)(c0 >> 51); r.v[0] = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); r.v[1] = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); r.v[2] = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); r.v[3] = (uint64_t)c3 & M51;
  uint64_t carry = (uint64_t)(c4 >> 51);
  r.v[4] = (uint64_t)c4 & M51;
  r.v[0] += carry * 19;
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= M51;
  return r;
}

/* Dedicated squaring: 15 products. */
static fe51 f_sq(fe51 a) {
  const uint64_t d0 = 2 * a.v[0], d1 = 2 * a.v[1], d2 = 2 * a.v[2], d3 = 2 * a.v[3];
  const uint64_t a3_19 = 19 * a.v[3], a4_19 = 19 * a.v[4];
  u128 c0 = (u128)a.v[0] * a.v[0] + (u128)d1 * a4_19 + (u128)d2 * a3_19;
  u128 c1 = (u128)d0 * a.v[1] + (u128)d2 * a4_19 + (u128)a.v[3] * a3_19;
  u128 c2 = (u128)d0 * a.v[2] + (u128)a.v[1] * a.v[1] + (u128)d3 * a4_19;
  u128 c3 = (u128)d0 * a.v[3] + (u128)d1 * a.v[2] + (u128)a.v[4] * a4_19;
  u128 c4 = (u128)d0 * a.v[4] + (u128)d1 * a.v[3] + (u128)a.v[2] * a.v[2];
  return f_carry128(c0, c1, c2, c3, c4);
}

static fe51 f_sqn(fe51 a, int n) {
  for (int i = 0; i < n; i++) a = f_sq(a);
  return a;
}

/* Canonical little-endian encoding. */
static void f_tobytes(uint8_t out[32], fe51 a) {
  a = f_weak(f_weak(a));
  /* q = 1 iff a >= p */
  uint64_t q = (a.v[0] + 19) >> 51;
  q = (a.v[1] + q) >> 51;
  q = (a.v[2] + q) >> 51;
  q = (a.v[3] + q) >> 51;
  q = (a.v[4] + q) >> 51;
  a.v[0] += 19 * q;
  a.v[1] += a.v[0] >> 51; a.v[0] &= M51;
  a.v[2] += a.v[1] >> 51; a.v[1] &= M51;
  a.v[3] += a.v[2] >> 51; a.v[2] &= M51;
  a.v[4] += a.v[3] >> 51; a.v[3] &= M51;
  a.v[4] &= M51;
  uint64_t w0 = a.v[0] | (a.v[1] << 51);
  uint64_t w1 = (a.v[1] >> 13) | (a.v[2] << 38);
  uint64_t w2 = (a.v[2] >> 26) | (a.v[3] << 25);
  uint64_t w3 = (a.v[3] >> 39) | (a.v[4] << 12);
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
}

/* Bit 255 ignored (the caller checks canonicity). */
static fe51 f_frombytes(const uint8_t in[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int k = 7; k >= 0; k--) w[i] = (w[i] << 8) | in[8 * i + k];
  }
  fe51 r;
  r.v[0] = w[0] & M51;
  r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r.v[4] = (w[3] >> 12) & M51;
  return r;
}

static int f_iszero(fe51 a) {
  uint8_t b[32];
  f_tobytes(b, a);
  uint8_t acc = 0;
  for (int i = 0; i < 32; i++) acc |= b[i];
  return acc == 0;
}

static int f_isneg(fe51 a) {
  uint8_t b[32];
  f_tobytes(b, a);
  return b[0] & 1;
}

static int f_eq(fe51 a, fe51 b) { return f_iszero(f_sub(a, b)); }

static fe51 f_cmov(fe51 a, fe51 b, int c) { /* c ? b : a, branch-free */
  const uint64_t m = (uint64_t)0 - (uint64_t)(c & 1);
  fe51 r;
  for (int i = 0; i < 5; i++) r.v[i] = a.v[i] ^ (m & (a.v[i] ^ b.v[i]));
  return r;
}

static fe51 f_abs(fe51 a) { return f_cmov(a, f_neg(a), f_isneg(a)); }

static fe51 f_pow22523(fe51 z) {
  fe51 t0 = f_sq(z), t1 = f_sqn(t0, 2), t2;
  t1 = f_mul(z, t1);
  t0 = f_mul(t0, t1);
  t0 = f_sq(t0);
  t0 = f_mul(t1, t0);
  t1 = f_sqn(t0, 5); t0 = f_mul(t1, t0);
  t1 = f_sqn(t0, 10); t1 = f_mul(t1, t0);
  t2 = f_sqn(t1, 20); t1 = f_mul(t2, t1);
  t1 = f_sqn(t1, 10); t0 = f_mul(t1, t0);
  t1 = f_sqn(t0, 50); t1 = f_mul(t1, t0);
  t2 = f_sqn(t1, 100); t1 = f_mul(t2, t1);
  t1 = f_sqn(t1, 50); t0 = f_mul(t1, t0);
  t0 = f_sqn(t0, 2);
  return f_mul(t0, z);
}

/* constants (value mod p, radix 2^51) */
static fe51 C_D(void) { return f_from(929955233495203ULL, 466365720129213ULL, 1662059464998953ULL, 2033849074728123ULL, 1442794654840575ULL); }
static fe51 C_D2(void) { return f_from(1859910466990425ULL, 932731440258426ULL, 1072319116312658ULL, 1815898335770999ULL, 633789495995903ULL); }
static fe51 C_SQRT_M1(void) { return f_from(1718705420411056ULL, 234908883556509ULL, 2233514472574048ULL, 2117202627021982ULL, 765476049583133ULL); }
static fe51 C_INVSQRT_A_MINUS_D(void) { return f_from(278908739862762ULL, 821645201101625ULL, 8113234426968ULL, 1777959178193151ULL, 2118520810568447ULL); }

static int f_sqrt_ratio_m1(fe51 *out, fe51 u, fe51 v) {
  fe51 v3 = f_mul(f_sq(v), v);
  fe51 v7 = f_mul(f_sq(v3), v);
  fe51 r = f_mul(f_mul(u, v3), f_pow22523(f_mul(u, v7)));
  fe51 check = f_mul(v, f_sq(r));
  fe51 nu = f_neg(u);
  int correct = f_eq(check, u);
  int flipped = f_eq(check, nu);
  int flipped_i = f_eq(check, f_mul(nu, C_SQRT_M1()));
  r = f_cmov(r, f_mul(r, C_SQRT_M1()), flipped | flipped_i);
  *out = f_abs(r);
  return correct | flipped;
}

/* ------------------------------------------------------------------------------------ */
/* Edwards points                                                                       */
/* ------------------------------------------------------------------------------------ */
typedef struct { fe51 X, Y, Z, T; } ge;               /* extended */
typedef struct { fe51 YpX, YmX, Z, T2d; } ge_pniels;  /* ProjectiveNiels */

static ge g_identity(void) {
  ge r = {f_zero(), f_one(), f_one(), f_zero()};
  return r;
}

static ge_pniels g_to_pniels(ge p) {
  ge_pniels r = {f_add(p.Y, p.X), f_sub(p.Y, p.X), p.Z, f_mul(p.T, C_D2())};
  return r;
}

typedef struct { fe51 X, Y, Z, T; } ge_c;  /* completed ((X:Z), (Y:T)) */
typedef struct { fe51 X, Y, Z; } ge_p2;    /* projective */

static ge c_to_p3(ge_c c) {
  ge r = {f_mul(c.X, c.T), f_mul(c.Y, c.Z), f_mul(c.Z, c.T), f_mul(c.X, c.Y)};
  return r;
}

static ge_p2 c_to_p2(ge_c c) {
  ge_p2 r = {f_mul(c.X, c.T), f_mul(c.Y, c.Z), f_mul(c.Z, c.T)};
  return r;
}

/* p + q, q ProjectiveNiels -> completed (4M) */
static ge_c g_add_pn_c(ge p, ge_pniels q) {
  fe51 PP = f_mul(f_add(p.Y, p.X), q.YpX);
  fe51 MM = f_mul(f_sub(p.Y, p.X), q.YmX);
  fe51 TT = f_mul(p.T, q.T2d);
  fe51 ZZ = f_mul(p.Z, q.Z);
  fe51 ZZ2 = f_add(ZZ, ZZ);
  ge_c r = {f_sub(PP, MM), f_add(PP, MM), f_add(ZZ2, TT), f_sub(ZZ2, TT)};
  return r;
}

static ge g_add_pn(ge p, ge_pniels q) { return c_to_p3(g_add_pn_c(p, q)); }
static ge g_add(ge p, ge q) { return g_add_pn(p, g_to_pniels(q)); }

/* projective doubling -> completed: XX, YY, 2ZZ, (X+Y)^2 */
static ge_c p2_dbl(ge_p2 p) {
  fe51 XX = f_sq(p.X), YY = f_sq(p.Y), ZZ = f_sq(p.Z);
  fe51 ZZ2 = f_add(ZZ, ZZ);
  fe51 XpY2 = f_sq(f_add(p.X, p.Y));
  fe51 YpX = f_add(YY, XX), YmX = f_sub(YY, XX);
  ge_c r = {f_sub(XpY2, YpX), YpX, YmX, f_sub(ZZ2, YmX)};
  return r;
}

static ge g_neg(ge p) {
  ge r = {f_neg(p.X), p.Y, p.Z, f_neg(p.T)};
  return r;
}

/* Constant-time selection of d * P from [P..8P], d in [-8, 8]: every entry is read and
 * masked (dalek LookupTable::select: conditional_assign + conditional_negate). */
static ge_pniels pn_select(const ge_pniels tab[8], int d) {
  const uint64_t neg = (uint64_t)0 - (uint64_t)(d < 0);
  const int mag = d < 0 ? -d : d;
  ge_pniels r = {f_one(), f_one(), f_one(), f_zero()};
  uint64_t *o = (uint64_t *)&r;
  for (int j = 1; j <= 8; j++) {
    const uint64_t m = (uint64_t)0 - (uint64_t)(mag == j);
    const uint64_t *t = (const uint64_t *)&tab[j - 1];
    for (int k = 0; k < 20; k++) o[k] ^= m & (o[k] ^ t[k]);
  }
  for (int k = 0; k < 5; k++) { /* swap (Y+X, Y-X) when negative */
    const uint64_t x = neg & (r.YpX.v[k] ^ r.YmX.v[k]);
    r.YpX.v[k] ^= x;
    r.YmX.v[k] ^= x;
  }
  const fe51 nt = f_neg(r.T2d);
  for (int k = 0; k < 5; k++) r.T2d.v[k] ^= neg & (r.T2d.v[k] ^ nt.v[k]);
  return r;
}

/* Constant-time variable-base scalar multiplication, dalek's variable_base::mul:
 * radix-16 signed digits, LookupTable [P, 2P, ..., 8P] (ProjectiveNiels), per window
 * four projective doublings (completed -> projective 3M each, last -> extended 4M)
 * and one CT-selected addition. */
static ge g_mul_ct(ge P, const uint8_t k[32]) {
  ge_pniels tab[8];
  tab[0] = g_to_pniels(P);
  for (int i = 1; i < 8; i++) tab[i] = g_to_pniels(g_add_pn(P, tab[i - 1]));
  int8_t d[64];
  int carry = 0;
  for (int i = 0; i < 32; i++) {
    for (int h = 0; h < 2; h++) {
      int v = ((k[i] >> (4 * h)) & 15) + carry;
      carry = (v + 8) >> 4;
      d[2 * i + h] = (int8_t)(v - (carry << 4));
    }
  }
  ge_c t1 = g_add_pn_c(g_identity(), pn_select(tab, d[63]));
  for (int i = 62; i >= 0; i--) {
    ge_p2 t2 = c_to_p2(t1);
    t1 = p2_dbl(t2);
    t2 = c_to_p2(t1);
    t1 = p2_dbl(t2);
    t2 = c_to_p2(t1);
    t1 = p2_dbl(t2);
    t2 = c_to_p2(t1);
    t1 = p2_dbl(t2);
    t1 = g_add_pn_c(c_to_p3(t1), pn_select(tab, d[i]));
  }
  return c_to_p3(t1);
}

/* ------------------------------------------------------------------------------------ */
/* ristretto255                                                                         */
/* ------------------------------------------------------------------------------------ */
static int bytes_lt_p(const uint8_t s[32]) {
  /* p = 2^255 - 19 */
  if (s[31] > 0x7f) return 0;
  if (s[31] < 0x7f) return 1;
  for (int i = 30; i >= 1; i--) {
    if (s[i] < 0xff) return 1;
  }
  return s[0] < 0xed;
}

static int r_decode(ge *out, const uint8_t in[32]) {
  if (!bytes_lt_p(in) || (in[0] & 1)) return 0;
  fe51 s = f_frombytes(in);
  fe51 ss = f_sq(s);
  fe51 u1 = f_sub(f_one(), ss);
  fe51 u2 = f_add(f_one(), ss);
  fe51 u2s = f_sq(u2);
  fe51 v = f_sub(f_neg(f_mul(C_D(), f_sq(u1))), u2s);
  fe51 inv;
  int sq = f_sqrt_ratio_m1(&inv, f_one(), f_mul(v, u2s));
  fe51 dx = f_mul(inv, u2);
  fe51 dy = f_mul(f_mul(inv, dx), v);
  fe51 x = f_abs(f_mul(f_add(s, s), dx));
  fe51 y = f_mul(u1, dy);
  fe51 t = f_mul(x, y);
  if (!sq || f_isneg(t) || f_iszero(y)) return 0;
  out->X = x; out->Y = y; out->Z = f_one(); out->T = t;
  return 1;
}

static void r_encode(uint8_t out[32], ge p) {
  fe51 u1 = f_mul(f_add(p.Z, p.Y), f_sub(p.Z, p.Y));
  fe51 u2 = f_mul(p.X, p.Y);
  fe51 inv;
  f_sqrt_ratio_m1(&inv, f_one(), f_mul(u1, f_sq(u2)));
  fe51 den1 = f_mul(inv, u1), den2 = f_mul(inv, u2);
  fe51 zinv = f_mul(f_mul(den1, den2), p.T);
  fe51 ix = f_mul(p.X, C_SQRT_M1()), iy = f_mul(p.Y, C_SQRT_M1());
  fe51 ench = f_mul(den1, C_INVSQRT_A_MINUS_D());
  int rot = f_isneg(f_mul(p.T, zinv));
  fe51 x = f_cmov(p.X, iy, rot);
  fe51 y = f_cmov(p.Y, ix, rot);
  fe51 dinv = f_cmov(den2, ench, rot);
  y = f_cmov(y, f_neg(y), f_isneg(f_mul(x, zinv)));
  f_tobytes(out, f_abs(f_mul(dinv, f_sub(p.Z, y))));
}

static int r_eq(ge a, ge b) {
  return f_eq(f_mul(a.X, b.Y), f_mul(a.Y, b.X)) | f_eq(f_mul(a.Y, b.Y), f_mul(a.X, b.X));
}

/* ------------------------------------------------------------------------------------ */
/* scalars mod l                                                                        */
/* ------------------------------------------------------------------------------------ */
static const uint8_t L_BYTES[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                    0xa2, 0xde, 0xf9, 0xde, 0x14, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};

static int sc_canonical(const uint8_t s[32]) {
  for (int i = 31; i >= 0; i--) {
    if (s[i] < L_BYTES[i]) return 1;
    if (s[i] > L_BYTES[i]) return 0;
  }
  return 0;
}

/* x (nbytes little-endian, <= 64) mod l by binary long division over 64-bit words. */
static void sc_reduce(uint8_t out[32], const uint8_t *x, int nbytes) {
  uint64_t lw[4], r[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    lw[i] = 0;
    for (int k = 7; k >= 0; k--) lw[i] = (lw[i] << 8) | L_BYTES[8 * i + k];
  }
  for (int bit = nbytes * 8 - 1; bit >= 0; bit--) {
    /* r = 2r + bit */
    for (int i = 4; i > 0; i--) r[i] = (r[i] << 1) | (r[i - 1] >> 63);
    r[0] = (r[0] << 1) | ((x[bit >> 3] >> (bit & 7)) & 1);
    /* if r >= l: r -= l */
    int ge_l = r[4] != 0;
    if (!ge_l) {
      ge_l = 1;
      for (int i = 3; i >= 0; i--) {
        if (r[i] != lw[i]) { ge_l = r[i] > lw[i]; break; }
      }
    }
    if (ge_l) {
      uint64_t borrow = 0;
      for (int i = 0; i < 4; i++) {
        u128 d = (u128)r[i] - lw[i] - borrow;
        r[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 64) & 1;
      }
      r[4] -= borrow;
    }
  }
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(r[i] >> (8 * k));
}

static void sc_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
  uint32_t aw[8], bw[8], p[16] = {0};
  for (int i = 0; i < 8; i++) {
    aw[i] = (uint32_t)a[4 * i] | ((uint32_t)a[4 * i + 1] << 8) | ((uint32_t)a[4 * i + 2] << 16) | ((uint32_t)a[4 * i + 3] << 24);
    bw[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
  }
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t t = (uint64_t)aw[i] * bw[j] + p[i + j] + carry;
      p[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    p[i + 8] = (uint32_t)carry;
  }
  uint8_t x[64];
  for (int i = 0; i < 16; i++)
    for (int k = 0; k < 4; k++) x[4 * i + k] = (uint8_t)(p[i] >> (8 * k));
  sc_reduce(out, x, 64);
}

/* ------------------------------------------------------------------------------------ */
/* Keccak-f[1600], STROBE-128, Merlin, protocol transcript                              */
/* ------------------------------------------------------------------------------------ */
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static uint64_t rol(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

static void keccakf(uint8_t st[200]) {
  uint64_t a[25], b[25], c[5];
  for (int i = 0; i < 25; i++) {
    a[i] = 0;
    for (int k = 7; k >= 0; k--) a[i] = (a[i] << 8) | st[8 * i + k];
  }
  for (int r = 0; r < 24; r++) {
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++) {
      uint64_t d = c[(x + 4) % 5] ^ rol(c[(x + 1) % 5], 1);
      for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
    }
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rol(a[x + 5 * y], RHO[x + 5 * y]);
    for (int y = 0; y < 5; y++)
      for (int x = 0; x < 5; x++) a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= RC[r];
  }
  for (int i = 0; i < 25; i++)
    for (int k = 0; k < 8; k++) st[8 * i + k] = (uint8_t)(a[i] >> (8 * k));
}

enum { SR = 166 };
typedef struct { uint8_t st[200]; int pos, pos_begin; } strobe;

static void s_runf(strobe *s) {
  s->st[s->pos] ^= (uint8_t)s->pos_begin;
  s->st[s->pos + 1] ^= 0x04;
  s->st[SR + 1] ^= 0x80;
  keccakf(s->st);
  s->pos = 0;
  s->pos_begin = 0;
}
static void s_absorb(strobe *s, const uint8_t *d, size_t n) {
  for (size_t i = 0; i < n; i++) {
    s->st[s->pos++] ^= d[i];
    if (s->pos == SR) s_runf(s);
  }
}
static void s_begin(strobe *s, uint8_t flags) {
  uint8_t hdr[2] = {(uint8_t)s->pos_begin, flags};
  s->pos_begin = s->pos + 1;
  s_absorb(s, hdr, 2);
  if ((flags & 4) && s->pos != 0) s_runf(s);
}
static void s_meta_ad(strobe *s, const void *d, size_t n) { s_begin(s, 16 | 2); s_absorb(s, (const uint8_t *)d, n); }
static void m_append(strobe *s, const char *label, const uint8_t *msg, size_t n) {
  uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  s_meta_ad(s, label, strlen(label));
  s_absorb(s, len, 4);
  s_begin(s, 2);
  s_absorb(s, msg, n);
}
static void m_challenge(strobe *s, const char *label, uint8_t *out, size_t n) {
  uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  s_meta_ad(s, label, strlen(label));
  s_absorb(s, len, 4);
  s_begin(s, 1 | 2 | 4);
  for (size_t i = 0; i < n; i++) {
    out[i] = s->st[s->pos];
    s->st[s->pos] = 0;
    if (++s->pos == SR) s_runf(s);
  }
}
static void m_new(strobe *s, const char *label) {
  memset(s->st, 0, 200);
  const uint8_t hdr[6] = {1, SR + 2, 1, 0, 1, 96};
  memcpy(s->st, hdr, 6);
  memcpy(s->st + 6, "STROBEv1.0.2", 12);
  keccakf(s->st);
  s->pos = 0;
  s->pos_begin = 0;
  s_meta_ad(s, "Merlin v1.0", 11);
  m_append(s, "dom-sep", (const uint8_t *)label, strlen(label));
}

/* transcript.rs:29-71 as used by batch.rs:188-206 */
static void protocol_challenge(uint8_t c[32], const uint8_t g[32], const uint8_t h[32], const uint8_t y1[32],
                               const uint8_t y2[32], const uint8_t r1[32], const uint8_t r2[32], const uint8_t *ctx,
                               uint64_t ctx_len, int has_ctx) {
  strobe s;
  m_new(&s, "Chaum-Pedersen ZKP v1.0.0");
  m_append(&s, "protocol", (const uint8_t *)"chaum-pedersen-ristretto255", 27);
  if (has_ctx) m_append(&s, "context", ctx, ctx_len);
  m_append(&s, "generator-g", g, 32);
  m_append(&s, "generator-h", h, 32);
  m_append(&s, "y1", y1, 32);
  m_append(&s, "y2", y2, 32);
  m_append(&s, "r1", r1, 32);
  m_append(&s, "r2", r2, 32);
  uint8_t wide[64];
  m_challenge(&s, "challenge", wide, 64);
  sc_reduce(c, wide, 64);
}

/* ------------------------------------------------------------------------------------ */
/* ChaCha20 block (weights for the reference batch equation)                            */
/* ------------------------------------------------------------------------------------ */
static uint32_t rl32(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }
#define QR(a, b, c, d) a += b; d ^= a; d = rl32(d, 16); c += d; b ^= c; b = rl32(b, 12); \
                       a += b; d ^= a; d = rl32(d, 8); c += d; b ^= c; b = rl32(b, 7);
static void chacha_block(uint8_t out[64], const uint8_t key[32], uint64_t ctr, uint64_t stream) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; i++)
    in[4 + i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
  in[12] = (uint32_t)ctr; in[13] = (uint32_t)(ctr >> 32); in[14] = (uint32_t)stream; in[15] = (uint32_t)(stream >> 32);
  uint32_t x[16];
  memcpy(x, in, sizeof(x));
  for (int r = 0; r < 10; r++) {
    QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]); QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]); QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) {
    uint32_t v = x[i] + in[i];
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(v >> (8 * k));
  }
}

/* ------------------------------------------------------------------------------------ */
/* Protocol                                                                              */
/* ------------------------------------------------------------------------------------ */
enum { ST_OK = 0, ST_EQ = 1, ST_POINT = 2, ST_SCALAR = 3, ST_IDENT = 4, ST_ZERO_S = 5 };

typedef struct {
  ge y1, y2, r1, r2;
  uint8_t s[32];
} decoded;

static int is_zero32(const uint8_t *b) {
  uint8_t acc = 0;
  for (int i = 0; i < 32; i++) acc |= b[i];
  return acc == 0;
}

/* Statement construction + Proof::from_bytes rejections (gadgets.rs:364-489). */
static int decode_entry(decoded *d, const uint8_t *y1, const uint8_t *y2, const uint8_t *r1, const uint8_t *r2,
                        const uint8_t *s) {
  if (!r_decode(&d->y1, y1) || !r_decode(&d->y2, y2)) return ST_POINT;
  if (!r_decode(&d->r1, r1) || !r_decode(&d->r2, r2)) return ST_POINT;
  if (!sc_canonical(s)) return ST_SCALAR;
  if (is_zero32(r1) || is_zero32(r2)) return ST_IDENT; /* gadgets.rs:474-478; identity = 32 zero bytes */
  if (is_zero32(s)) return ST_ZERO_S;                     /* gadgets.rs:480-482 */
  memcpy(d->s, s, 32);
  return ST_OK;
}

/* batch.rs:185-231 on decoded points: 6 compressions, 4 CT multiplications. */
static int verify_one_decoded(const decoded *d, ge G, ge H, const uint8_t *ctx, uint64_t ctx_len, int has_ctx) {
  uint8_t ge_[32], he_[32], a[32], b[32], c_[32], e[32], c[32];
  r_encode(ge_, G); r_encode(he_, H);
  r_encode(a, d->y1); r_encode(b, d->y2);
  r_encode(c_, d->r1); r_encode(e, d->r2);
  protocol_challenge(c, ge_, he_, a, b, c_, e, ctx, ctx_len, has_ctx);
  ge lhs1 = g_mul_ct(G, d->s);
  ge rhs1 = g_add(d->r1, g_mul_ct(d->y1, c));
  ge lhs2 = g_mul_ct(H, d->s);
  ge rhs2 = g_add(d->r2, g_mul_ct(d->y2, c));
  return (r_eq(lhs1, rhs1) && r_eq(lhs2, rhs2)) ? ST_OK : ST_EQ;
}

/* Exported: per-proof status from encodings (decode + verify_one). */
int cpzo_verify_one(const uint8_t g[32], const uint8_t h[32], const uint8_t y1[32], const uint8_t y2[32],
                    const uint8_t r1[32], const uint8_t r2[32], const uint8_t s[32], const uint8_t *ctx,
                    uint64_t ctx_len, int has_ctx) {
  ge G, H;
  if (!r_decode(&G, g) || !r_decode(&H, h)) return -1;
  decoded d;
  int st = decode_entry(&d, y1, y2, r1, r2, s);
  if (st != ST_OK) return st;
  return verify_one_decoded(&d, G, H, ctx, ctx_len, has_ctx);
}

/* Exported: per-proof statuses for n SoA rows (no contexts). */
void cpzo_verify_many(const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t *y1, const uint8_t *y2,
                      const uint8_t *r1, const uint8_t *r2, const uint8_t *s, uint8_t *status) {
  for (size_t i = 0; i < n; i++)
    status[i] = (uint8_t)cpzo_verify_one(g, h, y1 + 32 * i, y2 + 32 * i, r1 + 32 * i, r2 + 32 * i, s + 32 * i, 0, 0, 0);
}

/* Exported: BatchVerifier::verify (batch.rs:171-318) on n <= 1000 entries, default or
 * given generators, no contexts.  Returns 1 if the (defective) batch equation held. */
int cpzo_reference_batch_verify(const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t *y1,
                                const uint8_t *y2, const uint8_t *r1, const uint8_t *r2, const uint8_t *s,
                                const uint8_t weight_seed[32], uint64_t first_index, uint8_t *status) {
  ge G, H;
  if (n == 0 || !r_decode(&G, g) || !r_decode(&H, h)) return -1;
  static __thread decoded ents[1000];
  if (n > 1000) return -1;
  int all_ok = 1;
  for (size_t i = 0; i < n; i++) {
    int st = decode_entry(&ents[i], y1 + 32 * i, y2 + 32 * i, r1 + 32 * i, r2 + 32 * i, s + 32 * i);
    status[i] = (uint8_t)st;
    if (st != ST_OK) all_ok = 0;  /* such an entry could not have been added to the batch */
  }
  if (n == 1 || !all_ok) {
    for (size_t i = 0; i < n; i++)
      if (status[i] == ST_OK) status[i] = (uint8_t)verify_one_decoded(&ents[i], G, H, 0, 0, 0);
    return 0;
  }
  /* verify_batch: per-entry alpha (random_scalar) and challenge */
  ge lhs1 = g_identity(), rhs1 = g_identity(), lhs2 = g_identity(), rhs2 = g_identity();
  uint8_t ge_[32], he_[32];
  for (size_t i = 0; i < n; i++) {
    uint8_t blk[64], alpha[32], c[32], a[32], b[32], c_[32], e[32], alpha_s[32];
    chacha_block(blk, weight_seed, first_index + i, 0);
    sc_reduce(alpha, blk, 64);
    r_encode(ge_, G); r_encode(he_, H);
    r_encode(a, ents[i].y1); r_encode(b, ents[i].y2);
    r_encode(c_, ents[i].r1); r_encode(e, ents[i].r2);
    protocol_challenge(c, ge_, he_, a, b, c_, e, 0, 0, 0);
    /* verify_batch_equations (batch.rs:279-309), as written */
    sc_mul(alpha_s, alpha, ents[i].s);
    lhs1 = g_add(lhs1, g_mul_ct(G, alpha_s));
    rhs1 = g_add(rhs1, g_add(g_mul_ct(ents[i].r1, alpha), g_mul_ct(ents[i].y1, c)));
    lhs2 = g_add(lhs2, g_mul_ct(H, alpha_s));
    rhs2 = g_add(rhs2, g_add(g_mul_ct(ents[i].r2, alpha), g_mul_ct(ents[i].y2, c)));
  }
  if (r_eq(lhs1, rhs1) && r_eq(lhs2, rhs2)) {
    for (size_t i = 0; i < n; i++) status[i] = ST_OK;
    return 1;
  }
  for (size_t i = 0; i < n; i++) status[i] = (uint8_t)verify_one_decoded(&ents[i], G, H, 0, 0, 0);
  return 0;
}

/* Exported helpers for tests. */
void cpzo_challenge(uint8_t c[32], const uint8_t g[32], const uint8_t h[32], const uint8_t y1[32], const uint8_t y2[32],
                    const uint8_t r1[32], const uint8_t r2[32], const uint8_t *ctx, uint64_t ctx_len, int has_ctx) {
  protocol_challenge(c, g, h, y1, y2, r1, r2, ctx, ctx_len, has_ctx);
}

int cpzo_decode_encode(uint8_t out[32], const uint8_t in[32]) {
  ge p;
  if (!r_decode(&p, in)) return 0;
  r_encode(out, p);
  return 1;
}

/* enc(k * P) through the constant-time ladder. */
int cpzo_scalar_mul(uint8_t out[32], const uint8_t p[32], const uint8_t k[32]) {
  ge P;
  if (!r_decode(&P, p)) return 0;
  r_encode(out, g_mul_ct(P, k));
  return 1;
}

/* Sum of points given as encodings, with a sign per point: enc(sum). Used to combine
 * per-GPU RLC partials in tests. */
int cpzo_point_sum(uint8_t out[32], size_t n, const uint8_t *pts) {
  ge acc = g_identity();
  for (size_t i = 0; i < n; i++) {
    ge p;
    if (!r_decode(&p, pts + 32 * i)) return 0;
    acc = g_add(acc, p);
  }
  r_encode(out, acc);
  return 1;
}

void cpzo_sc_reduce_wide(uint8_t out[32], const uint8_t in[64]) { sc_reduce(out, in, 64); }
void cpzo_sc_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) { sc_mul(out, a, b); }
void cpzo_chacha_block(uint8_t out[64], const uint8_t key[32], uint64_t ctr, uint64_t stream) {
  chacha_block(out, key, ctr, stream);
}

/* ------------------------------------------------------------------------------------ */
/* At-scale checkers (test infrastructure): per-entry statuses and challenges with         */
/* optional contexts, and the corrected RLC partial of a subset of a batch.                */
/* ------------------------------------------------------------------------------------ */
static void entry_ctx(const uint8_t *ctx_bytes, const uint64_t *ctx_off, const uint8_t *ctx_present, size_t i,
                      const uint8_t **p, uint64_t *len, int *has) {
  *has = ctx_off != 0 && (ctx_present == 0 || ctx_present[i] != 0);
  *p = *has ? ctx_bytes + ctx_off[i] : 0;
  *len = *has ? ctx_off[i + 1] - ctx_off[i] : 0;
}

/* Per-proof statuses (decode + verify_one, batch.rs:185-231) for n SoA rows with contexts
 * (ctx_off: n + 1 absolute offsets into ctx_bytes, or NULL: no contexts; ctx_present: NULL =
 * every entry Some). */
void cpzo_verify_many_ctx(const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t *y1, const uint8_t *y2,
                          const uint8_t *r1, const uint8_t *r2, const uint8_t *s, const uint8_t *ctx_bytes,
                          const uint64_t *ctx_off, const uint8_t *ctx_present, uint8_t *status) {
  for (size_t i = 0; i < n; i++) {
    const uint8_t *cp;
    uint64_t cl;
    int has;
    entry_ctx(ctx_bytes, ctx_off, ctx_present, i, &cp, &cl, &has);
    status[i] = (uint8_t)cpzo_verify_one(g, h, y1 + 32 * i, y2 + 32 * i, r1 + 32 * i, r2 + 32 * i, s + 32 * i, cp, cl,
                                         has);
  }
}

/* Transcript challenges (transcript.rs:29-71) for n rows with contexts. */
void cpzo_challenge_many(const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t *y1, const uint8_t *y2,
                         const uint8_t *r1, const uint8_t *r2, const uint8_t *ctx_bytes, const uint64_t *ctx_off,
                         const uint8_t *ctx_present, uint8_t *c_out) {
  for (size_t i = 0; i < n; i++) {
    const uint8_t *cp;
    uint64_t cl;
    int has;
    entry_ctx(ctx_bytes, ctx_off, ctx_present, i, &cp, &cl, &has);
    protocol_challenge(c_out + 32 * i, g, h, y1 + 32 * i, y2 + 32 * i, r1 + 32 * i, r2 + 32 * i, cp, cl, has);
  }
}

static void sc_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
  uint8_t wide[64] = {0};
  unsigned carry = 0;
  for (int i = 0; i < 32; i++) {
    unsigned v = (unsigned)a[i] + b[i] + carry;
    wide[i] = (uint8_t)v;
    carry = v >> 8;
  }
  wide[32] = (uint8_t)carry;
  sc_reduce(out, wide, 64);
}

static void sc_neg(uint8_t out[32], const uint8_t a[32]) { /* l - a (mod l), a canonical */
  static const uint8_t L_BYTES[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                      0xa2, 0xde, 0xf9, 0xde, 0x14, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};
  uint8_t d[64] = {0};
  int borrow = 0;
  for (int i = 0; i < 32; i++) {
    int v = (int)L_BYTES[i] - a[i] - borrow;
    borrow = v < 0;
    d[i] = (uint8_t)(v + (borrow ? 256 : 0));
  }
  sc_reduce(out, d, 64); /* l - 0 = l -> 0 */
}

/* The 128-bit RLC weight from 8 little-endian int16 words (pyoracle.rlc_weights):
 * sum_k w_k 2^(16k) mod l, each signed word reduced mod l and scaled separately. */
static void rlc_weight_words(uint8_t out[32], const uint8_t blk16[16]) {
  uint8_t acc[32] = {0};
  for (int k = 0; k < 8; k++) {
    const int16_t w = (int16_t)(blk16[2 * k] | (blk16[2 * k + 1] << 8));
    uint8_t mag[32] = {0}, term[32], pow2[32] = {0};
    const int m = w < 0 ? -(int)w : (int)w;
    mag[0] = (uint8_t)m;
    mag[1] = (uint8_t)(m >> 8);
    pow2[(16 * k) / 8] = 1; /* 2^(16k): byte 2k */
    sc_mul(term, mag, pow2);
    if (w < 0) sc_neg(term, term);
    sc_add(acc, acc, term);
  }
  memcpy(out, acc, 32);
}

/* The corrected RLC partial (rlc.hip; pyoracle.rlc_partial) of n entries whose GLOBAL batch
 * indices are gidx[i]:  sum over entries whose decode-level status is 0 of
 *   [a s] g - [a] r1 - [a c] y1 + [b s] h - [b] r2 - [b c] y2,
 * (a, b) = the weights of ChaCha20(seed) block gidx[i].  Returns the encoding in out and the
 * number of live (weighted) entries. */
long cpzo_rlc_partial(const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t *y1, const uint8_t *y2,
                      const uint8_t *r1, const uint8_t *r2, const uint8_t *s, const uint8_t *ctx_bytes,
                      const uint64_t *ctx_off, const uint8_t *ctx_present, const uint64_t *gidx,
                      const uint8_t seed[32], uint8_t out[32]) {
  ge G, H;
  if (!r_decode(&G, g) || !r_decode(&H, h)) return -1;
  ge acc = g_identity();
  uint8_t sg[32] = {0}, sh[32] = {0};
  long live = 0;
  for (size_t i = 0; i < n; i++) {
    decoded d;
    if (decode_entry(&d, y1 + 32 * i, y2 + 32 * i, r1 + 32 * i, r2 + 32 * i, s + 32 * i) != ST_OK) continue;
    live++;
    const uint8_t *cp;
    uint64_t cl;
    int has;
    entry_ctx(ctx_bytes, ctx_off, ctx_present, i, &cp, &cl, &has);
    uint8_t c[32], blk[64], a[32], b[32], t[32], na[32];
    protocol_challenge(c, g, h, y1 + 32 * i, y2 + 32 * i, r1 + 32 * i, r2 + 32 * i, cp, cl, has);
    chacha_block(blk, seed, gidx[i], 0);
    rlc_weight_words(a, blk);
    rlc_weight_words(b, blk + 16);
    sc_mul(t, a, d.s);
    sc_add(sg, sg, t);
    sc_mul(t, b, d.s);
    sc_add(sh, sh, t);
    sc_neg(na, a);
    acc = g_add(acc, g_mul_ct(d.r1, na));
    sc_mul(t, a, c);
    sc_neg(t, t);
    acc = g_add(acc, g_mul_ct(d.y1, t));
    sc_neg(na, b);
    acc = g_add(acc, g_mul_ct(d.r2, na));
    sc_mul(t, b, c);
    sc_neg(t, t);
    acc = g_add(acc, g_mul_ct(d.y2, t));
  }
  acc = g_add(acc, g_mul_ct(G, sg));
  acc = g_add(acc, g_mul_ct(H, sh));
  r_encode(out, acc);
  return live;
}
