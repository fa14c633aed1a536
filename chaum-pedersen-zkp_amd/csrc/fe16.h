// GF(2^255 - 19) and edwards25519 point operations on a 16-lane ROW of a wave: the latency
// form behind k_verify_wide (the drop-in's n = 1 .. few-proof calls).
//
// Replaces the same dalek arithmetic as fe25519.h / ristretto.h (FieldElement, the
// ristretto decode of src/primitives/ristretto.rs:120-138, EdwardsPoint addition and
// doubling), laid out for latency instead of throughput.  In fe25519.h one lane holds a
// whole element and a product is ~120 dependent instructions of that lane; a lone wave
// issues them at ~500 cycles per squaring (tools/ubench/wide_mul.hip: 218 ns).  Here a
// field element is spread over the 16 lanes of a row, one 16-bit limb per lane
// (value = sum_k x_k 2^(16k), limbs signed and loosely reduced), and a product is
// computed by all 16 lanes at once:
//   lane k accumulates column k = sum_i x_i * y_(k-i mod 16), with 38 y where the index
//   wraps (2^256 = 38 mod p): x_i by a row broadcast (DPP row_newbcast:i), the shifted y by
//   one v_mul_i32_i24 reading y through DPP row_ror:i times the lane's wrap factor, one
//   v_mad_i64_i32; then three rounds of a parallel carry through DPP row_ror:1.
// 143-148 ns per squaring on a lone wave (1.5x faster than one lane, same box).
//
// Bounds (|limb|): a product's output ("tight") lies in (-2^14.7, 2^16 + 2^14.7) on limb 0
// and (-2^9.4, 2^16 + 2^9.4) elsewhere, < 90.8K.  Operands may be sums/differences of at
// most FOUR tight elements (< 363K < 2^18.8): then |x_i * 38 y_j| < 2^42.9, a column of 16
// stays below 2^47, and alignbit's 32-bit window of a column is its exact floor / 2^16.
//
// Points ("replicated" layout): every row of the wave holds the whole point, X, Y, Z, T in
// four registers (lane k: limb k of each).  A point operation runs as two product STAGES:
// row r computes the stage's r-th product (operands picked per row by sel4), and one
// all-gather over the rows (gather4: v_permlane32_swap + two v_permlane16_swap) gives every
// row all four products in fixed registers, so the formulas' additions need no exchange.
// A doubling or an addition is two stages (dalek's ProjectivePoint::double and
// EdwardsPoint + ProjectiveNielsPoint, through CompletedPoint -> extended).
//
// Device-only (DPP, permlane); the CPU never runs it: parity is k_verify_wide's statuses
// against the oracle (tests/test_gpu_scale.py), like every other kernel's.
#pragma once
#include <stdint.h>

namespace cpz {
namespace r16 {

// Per-lane constants: limb index, wrap factors, row.
struct Lane {
  int k;         // limb index (lane & 15)
  int w;         // 38 on limb 0 (receives the wrapped carry), 1 elsewhere
  int row;       // 0..3
  int wrap[16];  // wrap[i] = 38 where a shift by i wraps (k < i), 1 elsewhere
};

__device__ __forceinline__ Lane lane_of(int lane) {
  Lane L;
  L.k = lane & 15;
  L.w = L.k == 0 ? 38 : 1;
  L.row = (lane >> 4) & 3;
#pragma unroll
  for (int i = 0; i < 16; i++) L.wrap[i] = L.k < i ? 38 : 1;
  return L;
}

// DPP move with zero fill of lanes whose source is outside the row.
template <int C>
__device__ __forceinline__ int dpp0(int x) {
  return __builtin_amdgcn_update_dpp(0, x, C, 0xf, 0xf, true);
}

// lane k of the row: y_(k-i) for k >= i, 38 y_(k-i+16) for k < i -- ONE instruction,
// v_mul_i32_i24 reading y through DPP row_ror:i (lane k <- lane k - i mod 16) times the lane's
// wrap factor.  The 24-bit multiplier needs |y| < 2^23: operands of mul are at most four
// tight elements (< 2^18.5); mul_pair's pre-shifted y at most 38 x two tight ones (< 2^22.3).
template <int I>
__device__ __forceinline__ int shifted(int y, const Lane& L) {
  if constexpr (I == 0) {
    return y;
  } else {
    return __mul24(dpp0<0x120 + I>(y), L.wrap[I]);
  }
}

template <int I>
__device__ __forceinline__ void col_step(int64_t (&a)[4], int x, int y, const Lane& L) {
  a[I & 3] += (int64_t)dpp0<0x150 + I>(x) * (int64_t)shifted<I>(y, L);  // row_newbcast:i
  if constexpr (I + 1 < 16) col_step<I + 1>(a, x, y, L);
}

// floor(v / 2^16) for |v| < 2^47 (bits 16..47 of the two's complement)
__device__ __forceinline__ int floor16(int64_t v) {
  return (int)__builtin_amdgcn_alignbit((uint32_t)((uint64_t)v >> 32), (uint32_t)v, 16);
}

// x * y mod p (both operands at most four tight elements); tight result.
__device__ __forceinline__ int mul(int x, int y, const Lane& L) {
  int64_t a[4] = {0, 0, 0, 0};
  col_step<0>(a, x, y, L);
  const int64_t acc = (a[0] + a[1]) + (a[2] + a[3]);
  const int c1 = floor16(acc);
  const int64_t t = (int64_t)dpp0<0x121>(c1) * L.w + (int64_t)((uint32_t)acc & 0xffffu);  // row_ror:1
  const int c2 = floor16(t);
  const int u = ((int)(uint32_t)t & 0xffff) + dpp0<0x121>(c2) * L.w;
  const int c3 = u >> 16;
  return (u & 0xffff) + dpp0<0x121>(c3) * L.w;
}

template <int I>
__device__ __forceinline__ void col_step_half(int64_t (&a)[4], int x, int y, const Lane& L) {
  a[I & 3] += (int64_t)dpp0<0x150 + I>(x) * (int64_t)shifted<I>(y, L);
  if constexpr (I + 1 < 8) col_step_half<I + 1>(a, x, y, L);
}

// x * y for values that are the same on every row (the decode): the column sums are split
// over row pairs -- even rows take i = 0..7, odd rows i = 8..15 from x rotated by 8 and y
// shifted by 8 (lanes k < 8 then hold 38 y_(k+8); a further shift by j < 8 wraps only lanes
// >= 9, which hold plain y, so 38 y is never taken twice) -- and one v_permlane16_swap adds
// the halves: 8 column steps per lane instead of 16.  Same result as mul; operands at most
// two tight elements (the decode's are), so the pre-shifted y fits shifted's 24-bit multiply.
__device__ __forceinline__ int mul_pair(int x, int y, const Lane& L) {
  const bool hi = (L.row & 1) != 0;
  // DPP moves are convergent: computed on every lane, then selected (a conditional DPP
  // becomes a divergent branch)
  const int xr = dpp0<0x128>(x);                         // row_ror:8: lane j holds x_(j+8)
  const int yr = shifted<8>(y, L);
  const int xs = hi ? xr : x;
  const int ys = hi ? yr : y;
  int64_t a[4] = {0, 0, 0, 0};
  col_step_half<0>(a, xs, ys, L);
  const int64_t h = (a[0] + a[1]) + (a[2] + a[3]);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)h, (uint32_t)h, false, false);
  const auto hw = __builtin_amdgcn_permlane16_swap((uint32_t)((uint64_t)h >> 32), (uint32_t)((uint64_t)h >> 32),
                                                   false, false);
  const int64_t acc = (int64_t)(((uint64_t)hw[0] << 32) | lo[0]) + (int64_t)(((uint64_t)hw[1] << 32) | lo[1]);
  const int c1 = floor16(acc);
  const int64_t t = (int64_t)dpp0<0x121>(c1) * L.w + (int64_t)((uint32_t)acc & 0xffffu);
  const int c2 = floor16(t);
  const int u = ((int)(uint32_t)t & 0xffff) + dpp0<0x121>(c2) * L.w;
  const int c3 = u >> 16;
  return (u & 0xffff) + dpp0<0x121>(c3) * L.w;
}

// The decode's products: split over row pairs unless CPZ_WIDE_PAIR=0.
#ifndef CPZ_WIDE_PAIR
#define CPZ_WIDE_PAIR 1
#endif
__device__ __forceinline__ int mulr(int x, int y, const Lane& L) {
#if CPZ_WIDE_PAIR
  return mul_pair(x, y, L);
#else
  return mul(x, y, L);
#endif
}

__device__ __forceinline__ int sq(int x, const Lane& L) { return mulr(x, x, L); }

__device__ __forceinline__ int sqn(int x, int n, const Lane& L) {
#pragma unroll 1
  for (int i = 0; i < n; i++) x = mulr(x, x, L);
  return x;
}

// Limb k of an element given as 8 little-endian words in memory (global or LDS).
__device__ __forceinline__ int limb_of(const uint32_t* w, const Lane& L) {
  return (int)reinterpret_cast<const uint16_t*>(w)[L.k];
}

__device__ __forceinline__ int one(const Lane& L) { return L.k == 0 ? 1 : 0; }

// Constants (canonical 16-bit limbs): limb k of d, 2d, sqrt(-1).
__device__ __forceinline__ int const_limb(const uint16_t (&c)[16], const Lane& L) {
  int v = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) v = L.k == i ? (int)c[i] : v;
  return v;
}

// d = -121665/121666, 2d, sqrt(-1) (RFC 7748 / RFC 9496 constants), 16-bit limbs.
__device__ __forceinline__ int K_D(const Lane& L) {
  constexpr uint16_t c[16] = {0x78a3, 0x1359, 0x4dca, 0x75eb, 0xd8ab, 0x4141, 0x0a4d, 0x0070,
                              0xe898, 0x7779, 0x4079, 0x8cc7, 0xfe73, 0x2b6f, 0x6cee, 0x5203};
  return const_limb(c, L);
}
__device__ __forceinline__ int K_D2(const Lane& L) {
  constexpr uint16_t c[16] = {0xf159, 0x26b2, 0x9b94, 0xebd6, 0xb156, 0x8283, 0x149a, 0x00e0,
                              0xd130, 0xeef3, 0x80f2, 0x198e, 0xfce7, 0x56df, 0xd9dc, 0x2406};
  return const_limb(c, L);
}
__device__ __forceinline__ int K_SQRT_M1(const Lane& L) {
  constexpr uint16_t c[16] = {0xa0b0, 0x4a0e, 0x1b27, 0xc4ee, 0xe478, 0xad2f, 0x1806, 0x2f43,
                              0xd7a7, 0x3dfb, 0x0099, 0x2b4d, 0xdf0b, 0x4fc1, 0x2480, 0x2b83};
  return const_limb(c, L);
}

// Canonical little-endian words of the row's element (every lane of the row gets them).
__device__ __forceinline__ void to_words(uint32_t out[8], int x) {
  int l[16];
  l[0] = dpp0<0x150>(x);
  l[1] = dpp0<0x151>(x);
  l[2] = dpp0<0x152>(x);
  l[3] = dpp0<0x153>(x);
  l[4] = dpp0<0x154>(x);
  l[5] = dpp0<0x155>(x);
  l[6] = dpp0<0x156>(x);
  l[7] = dpp0<0x157>(x);
  l[8] = dpp0<0x158>(x);
  l[9] = dpp0<0x159>(x);
  l[10] = dpp0<0x15a>(x);
  l[11] = dpp0<0x15b>(x);
  l[12] = dpp0<0x15c>(x);
  l[13] = dpp0<0x15d>(x);
  l[14] = dpp0<0x15e>(x);
  l[15] = dpp0<0x15f>(x);
  // V + 4p = V + 2^257 - 76 > 0 (|V| < 2^256): limbs to [0, 2^16) with carry c in [0, 4)
  uint32_t h[16];
  int64_t c = -76;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    c += l[i];
    h[i] = (uint32_t)c & 0xffffu;
    c >>= 16;
  }
  c += 2;
  // fold the carry (2^256 = 38), twice: the second fold cannot carry out again
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    int64_t d = c * 38;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      d += h[i];
      h[i] = (uint32_t)d & 0xffffu;
      d >>= 16;
    }
    c = d;
  }
  uint32_t x8[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x8[i] = h[2 * i] | (h[2 * i + 1] << 16);
  // [0, 2^256) -> [0, p): subtract p up to twice (x >= p iff x + 19 >= 2^255)
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    uint64_t cc = 19;
    uint32_t y[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      cc += x8[i];
      y[i] = (uint32_t)cc;
      cc >>= 32;
    }
    const bool ge = (y[7] >> 31) != 0 || cc != 0;
    y[7] &= 0x7fffffffu;
#pragma unroll
    for (int i = 0; i < 8; i++) x8[i] = ge ? y[i] : x8[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = x8[i];
}

__device__ __forceinline__ bool is_zero(int x) {
  uint32_t w[8];
  to_words(w, x);
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) a |= w[i];
  return a == 0;
}

__device__ __forceinline__ bool is_negative(int x) {
  uint32_t w[8];
  to_words(w, x);
  return (w[0] & 1u) != 0;
}

// x^((p-5)/8) = x^(2^252 - 3) (the chain of fe25519.h's fe_pow22523)
__device__ __forceinline__ int pow22523(int z, const Lane& L) {
  int t0 = sq(z, L);
  int t1 = sqn(t0, 2, L);
  t1 = mulr(z, t1, L);
  t0 = mulr(t0, t1, L);
  t0 = sq(t0, L);
  t0 = mulr(t1, t0, L);
  t1 = sqn(t0, 5, L);
  t0 = mulr(t1, t0, L);
  t1 = sqn(t0, 10, L);
  t1 = mulr(t1, t0, L);
  int t2 = sqn(t1, 20, L);
  t1 = mulr(t2, t1, L);
  t1 = sqn(t1, 10, L);
  t0 = mulr(t1, t0, L);
  t1 = sqn(t0, 50, L);
  t1 = mulr(t1, t0, L);
  t2 = sqn(t1, 100, L);
  t1 = mulr(t2, t1, L);
  t1 = sqn(t1, 50, L);
  t0 = mulr(t1, t0, L);
  t0 = sqn(t0, 2, L);
  return mulr(t0, z, L);
}

// SQRT_RATIO_M1(1, v) (RFC 9496 4.2, fe25519.h fe_invsqrt_m1): was_square, |1/sqrt(v)|
// or |sqrt(i/v)|.
__device__ __forceinline__ bool invsqrt_m1(int& out, int v, const Lane& L) {
  const int v3 = mulr(sq(v, L), v, L);
  const int v7 = mulr(sq(v3, L), v, L);
  int r = mulr(v3, pow22523(v7, L), L);
  uint32_t w[8];
  to_words(w, mulr(v, sq(r, L), L));
  const uint32_t kNegSqrtM1[8] = {0xb5f15f3du, 0x3b11e4d8u, 0x52d01b87u, 0xd0bce7f9u,
                                  0xc2042858u, 0xd4b2ff66u, 0xb03e20f4u, 0x547cdb7fu};
  uint32_t d_one = w[0] ^ 1u, d_neg = w[0] ^ 0xffffffecu, d_negi = w[0] ^ kNegSqrtM1[0];
#pragma unroll
  for (int k = 1; k < 8; k++) {
    d_one |= w[k];
    d_neg |= w[k] ^ (k == 7 ? 0x7fffffffu : 0xffffffffu);
    d_negi |= w[k] ^ kNegSqrtM1[k];
  }
  const bool correct = d_one == 0, flipped = d_neg == 0, flipped_i = d_negi == 0;
  const int ri = mulr(r, K_SQRT_M1(L), L);
  r = (flipped || flipped_i) ? ri : r;
  out = is_negative(r) ? -r : r;
  return correct || flipped;
}

// Replicated point: every row holds X, Y, Z, T (limb k on lane k of the row).
struct P4 {
  int X, Y, Z, T;
};
// Cached (ProjectiveNiels) point: Y + X, Y - X, Z, 2 d T.
struct C4 {
  int ypx, ymx, z, t2d;
};

__device__ __forceinline__ P4 identity(const Lane& L) {
  P4 p;
  p.X = 0;
  p.Y = one(L);
  p.Z = one(L);
  p.T = 0;
  return p;
}

// RFC 9496 4.3.1 DECODE of the 8 words at `w` (the same on every lane of the wave); every
// row computes it.  Returns false for non-canonical, negative, non-square, negative-t or
// y == 0 encodings (ristretto.h ristretto_decode).
__device__ __forceinline__ bool decode(P4& out, const uint32_t* w, const uint32_t wu[8], const Lane& L) {
  // canonical: s < p and even
  uint32_t borrow = 0;
  const uint32_t pw[8] = {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)wu[i] - pw[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  const bool canonical = borrow != 0 && (wu[0] & 1u) == 0;
  const int s = limb_of(w, L) & (L.k == 15 ? 0x7fff : 0xffff);
  const int ss = sq(s, L);
  const int u1 = one(L) - ss;
  const int u2 = one(L) + ss;
  const int u2_sqr = sq(u2, L);
  const int v = -mulr(K_D(L), sq(u1, L), L) - u2_sqr;
  int inv;
  const bool was_square = invsqrt_m1(inv, mulr(v, u2_sqr, L), L);
  const int den_x = mulr(inv, u2, L);
  const int den_y = mulr(mulr(inv, den_x, L), v, L);
  int x = mulr(s + s, den_x, L);
  x = is_negative(x) ? -x : x;
  const int y = mulr(u1, den_y, L);
  const int t = mulr(x, y, L);
  out.X = x;
  out.Y = y;
  out.Z = one(L);
  out.T = t;
  return canonical && was_square && !is_negative(t) && !is_zero(y);
}

// the row's pick among four values: a_row
__device__ __forceinline__ int sel4(int a0, int a1, int a2, int a3, const Lane& L) {
  const int lo = (L.row & 1) ? a1 : a0;
  const int hi = (L.row & 1) ? a3 : a2;
  return (L.row & 2) ? hi : lo;
}

// All-gather over the four rows: g[r] = row r's value, on every row.
struct G4 {
  int g0, g1, g2, g3;
};
__device__ __forceinline__ G4 gather4(int r) {
  const auto h = __builtin_amdgcn_permlane32_swap(r, r, false, false);          // [r0 r1 r0 r1], [r2 r3 r2 r3]
  const auto lo = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);   // [r0 x4], [r1 x4]
  const auto hi = __builtin_amdgcn_permlane16_swap(h[1], h[1], false, false);   // [r2 x4], [r3 x4]
  G4 g;
  g.g0 = (int)lo[0];
  g.g1 = (int)lo[1];
  g.g2 = (int)hi[0];
  g.g3 = (int)hi[1];
  return g;
}

// CompletedPoint ((X : Z), (Y : T)) -> extended: X T, Y Z, Z T, X Y (one stage).
__device__ __forceinline__ P4 completed_to_p4(int Xc, int Yc, int Zc, int Tc, const Lane& L) {
  const int a = sel4(Xc, Yc, Zc, Xc, L);
  const int b = sel4(Tc, Zc, Tc, Yc, L);
  const G4 g = gather4(mul(a, b, L));
  P4 p;
  p.X = g.g0;
  p.Y = g.g1;
  p.Z = g.g2;
  p.T = g.g3;
  return p;
}

// 2 P (dalek ProjectivePoint::double, then as_extended): two stages.
__device__ __forceinline__ P4 dbl(const P4& p, const Lane& L) {
  const int a = sel4(p.X, p.Y, p.Z, p.X + p.Y, L);
  const G4 g = gather4(mul(a, a, L));  // XX, YY, ZZ, (X + Y)^2
  const int yypxx = g.g1 + g.g0, yymxx = g.g1 - g.g0;
  return completed_to_p4(g.g3 - yypxx, yypxx, yymxx, (g.g2 + g.g2) - yymxx, L);
}

// P + C given the row's operand of C for the first stage (b: Y-X, Y+X, 2dT, Z per row;
// swapped / negated for -C by the caller): two stages.
__device__ __forceinline__ P4 add_b(const P4& p, int b, const Lane& L) {
  const int a = sel4(p.Y - p.X, p.Y + p.X, p.T, p.Z, L);
  const G4 g = gather4(mul(a, b, L));  // MM, PP, TT2d, ZZ
  const int zz2 = g.g3 + g.g3;
  return completed_to_p4(g.g1 - g.g0, g.g1 + g.g0, zz2 + g.g2, zz2 - g.g2, L);
}

// The first-stage operand row r takes from a cached point (+C, or -C when neg).
__device__ __forceinline__ int cached_b(const C4& c, bool neg, const Lane& L) {
  return sel4(neg ? c.ypx : c.ymx, neg ? c.ymx : c.ypx, neg ? -c.t2d : c.t2d, c.z, L);
}

// Extended -> cached (one product, 2 d T, computed by every row).
__device__ __forceinline__ C4 to_cached(const P4& p, const Lane& L) {
  C4 c;
  c.ypx = p.Y + p.X;
  c.ymx = p.Y - p.X;
  c.z = p.Z;
  c.t2d = mul(p.T, K_D2(L), L);
  return c;
}

__device__ __forceinline__ P4 neg(const P4& p) {
  P4 r;
  r.X = -p.X;
  r.Y = p.Y;
  r.Z = p.Z;
  r.T = -p.T;
  return r;
}

// Ristretto identity (mod E[4]): X == 0 or Y == 0 (ristretto.h ristretto_is_identity).
__device__ __forceinline__ bool is_identity(const P4& p) { return is_zero(p.X) || is_zero(p.Y); }

}  // namespace r16
}  // namespace cpz
