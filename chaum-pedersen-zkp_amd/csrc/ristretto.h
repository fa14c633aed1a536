// Edwards25519 group law and the ristretto255 encoding (RFC 9496) for gfx950.
//
// Replaces curve25519-dalek 4.1.3's EdwardsPoint / RistrettoPoint / CompressedRistretto
// as reached from the reference's src/primitives/ristretto.rs:
//   element_from_bytes  :120-138  -> ristretto_decode
//   element_to_bytes    :141-143  -> ristretto_encode
//   scalar_mul / element_mul :153-160 -> the point formulas below (used by kernels.hip)
//   RistrettoPoint ==  (dalek PartialEq)  -> ristretto_equal
//   is_identity         :168-170  -> ristretto_is_identity
//
// Coordinates follow the Hisil-Wong-Carter-Dawson extended model for a = -1:
//   ge_p3    extended (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z
//   ge_p2    projective (X:Y:Z)
//   ge_p1p1  "completed" ((X:Z), (Y:T))
//   ge_cached   (Y+X, Y-X, Z, 2d*T)        table entries for variable bases
//   ge_niels    (y+x, y-x, 2d*x*y), Z = 1  table entries for fixed bases (g, h)
// Operand bounds: every mul/sq input below is at most the sum of three tight elements
// (see fe25519.h).
#pragma once
#include "fe25519.h"

namespace cpz {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels {
  fe ypx, ymx, xy2d;
  int32_t pad[2];  // 128 B: whole 16-byte vectors for loads/stores
};
static_assert(sizeof(ge_niels) % 16 == 0, "ge_niels must be a whole number of 16-byte vectors");
static_assert(sizeof(ge_p3) % 16 == 0 && sizeof(ge_cached) % 16 == 0, "16-byte vector copies");

CPZ_HD ge_p3 ge_identity() {
  ge_p3 r;
  r.X = fe_zero(); r.Y = fe_one(); r.Z = fe_one(); r.T = fe_zero();
  return r;
}

CPZ_HD ge_cached ge_cached_identity() {
  ge_cached r;
  r.YpX = fe_one(); r.YmX = fe_one(); r.Z = fe_one(); r.T2d = fe_zero();
  return r;
}

CPZ_HD ge_niels ge_niels_identity() {
  ge_niels r;
  r.ypx = fe_one(); r.ymx = fe_one(); r.xy2d = fe_zero();
  return r;
}

// Operand roles: fe_mul(f, g) derives 2 f (odd limbs) and 19 g from its operands, so X and
// Z are always the left operand and T and Y the right one -- the derived limbs of each
// coordinate are then computed once and shared by the products that use it.
CPZ_HD ge_p2 p1p1_to_p2(const ge_p1p1& p) {
  ge_p2 r;
  r.X = fe_mul(p.X, p.T);
  r.Y = fe_mul(p.Z, p.Y);
  r.Z = fe_mul(p.Z, p.T);
  return r;
}

CPZ_HD ge_p3 p1p1_to_p3(const ge_p1p1& p) {
  ge_p3 r;
  r.X = fe_mul(p.X, p.T);
  r.Y = fe_mul(p.Z, p.Y);
  r.Z = fe_mul(p.Z, p.T);
  r.T = fe_mul(p.X, p.Y);
  return r;
}

CPZ_HD ge_p2 p3_to_p2(const ge_p3& p) {
  ge_p2 r;
  r.X = p.X; r.Y = p.Y; r.Z = p.Z;
  return r;
}

CPZ_HD ge_cached p3_to_cached(const ge_p3& p) {
  ge_cached r;
  r.YpX = fe_add(p.Y, p.X);
  r.YmX = fe_sub(p.Y, p.X);
  r.Z = p.Z;
  r.T2d = fe_mul(p.T, FE_D2());
  return r;
}

// 2P: 4S (one of them folded as 2Z^2) ; dbl-2008-hwcd with a = -1.
CPZ_HD ge_p1p1 p2_dbl(const ge_p2& p) {
  const fe XX = fe_sq(p.X);
  const fe YY = fe_sq(p.Y);
  const fe ZZ2 = fe_sq2(p.Z);
  const fe XpY2 = fe_sq(fe_add(p.X, p.Y));
  const fe YYpXX = fe_add(YY, XX);
  const fe YYmXX = fe_sub(YY, XX);
  ge_p1p1 r;
  r.X = fe_sub(XpY2, YYpXX);
  r.Y = YYpXX;
  r.Z = YYmXX;
  r.T = fe_sub(ZZ2, YYmXX);
  return r;
}

CPZ_HD ge_p1p1 p3_dbl(const ge_p3& p) { return p2_dbl(p3_to_p2(p)); }

// P + Q, Q cached: 4M.  add-2008-hwcd-3 with a = -1.
CPZ_HD ge_p1p1 ge_add_cached(const ge_p3& p, const ge_cached& q) {
  const fe PP = fe_mul(fe_add(p.Y, p.X), q.YpX);
  const fe MM = fe_mul(fe_sub(p.Y, p.X), q.YmX);
  const fe TT2d = fe_mul(p.T, q.T2d);
  const fe ZZ = fe_mul(p.Z, q.Z);
  const fe ZZ2 = fe_add(ZZ, ZZ);
  ge_p1p1 r;
  r.X = fe_sub(PP, MM);
  r.Y = fe_add(PP, MM);
  r.Z = fe_add(ZZ2, TT2d);
  r.T = fe_sub(ZZ2, TT2d);
  return r;
}

// P + Q, Q affine Niels (Z = 1): 3M.
CPZ_HD ge_p1p1 ge_add_niels(const ge_p3& p, const ge_niels& q) {
  const fe PP = fe_mul(fe_add(p.Y, p.X), q.ypx);
  const fe MM = fe_mul(fe_sub(p.Y, p.X), q.ymx);
  const fe Txy2d = fe_mul(p.T, q.xy2d);
  const fe Z2 = fe_add(p.Z, p.Z);
  ge_p1p1 r;
  r.X = fe_sub(PP, MM);
  r.Y = fe_add(PP, MM);
  r.Z = fe_add(Z2, Txy2d);
  r.T = fe_sub(Z2, Txy2d);
  return r;
}

CPZ_HD ge_p3 ge_add(const ge_p3& p, const ge_p3& q) { return p1p1_to_p3(ge_add_cached(p, p3_to_cached(q))); }

CPZ_HD ge_p3 ge_neg(const ge_p3& p) {
  ge_p3 r;
  r.X = fe_neg(p.X); r.Y = p.Y; r.Z = p.Z; r.T = fe_neg(p.T);
  return r;
}

// -Q for a cached / Niels entry: swap (Y+X, Y-X), negate 2dT.
CPZ_HD ge_cached ge_cached_cneg(const ge_cached& q, bool neg) {
  ge_cached r;
  r.YpX = fe_select(q.YpX, q.YmX, neg);
  r.YmX = fe_select(q.YmX, q.YpX, neg);
  r.Z = q.Z;
  r.T2d = fe_select(q.T2d, fe_neg(q.T2d), neg);
  return r;
}

CPZ_HD ge_niels ge_niels_cneg(const ge_niels& q, bool neg) {
  ge_niels r;
  r.ypx = fe_select(q.ypx, q.ymx, neg);
  r.ymx = fe_select(q.ymx, q.ypx, neg);
  r.xy2d = fe_select(q.xy2d, fe_neg(q.xy2d), neg);
  return r;
}

// Ristretto equality (RFC 9496 4.3.3): X1 Y2 == Y1 X2  or  Y1 Y2 == X1 X2.
CPZ_HD bool ristretto_equal(const ge_p3& a, const ge_p3& b) {
  const bool e1 = fe_equal(fe_mul(a.X, b.Y), fe_mul(a.Y, b.X));
  const bool e2 = fe_equal(fe_mul(a.Y, b.Y), fe_mul(a.X, b.X));
  return e1 || e2;
}

// Equal to the identity (0 : 1 : 1 : 0) in the ristretto sense: X == 0 or Y == 0.
CPZ_HD bool ristretto_is_identity(const ge_p3& a) { return fe_iszero(a.X) || fe_iszero(a.Y); }

// The same test on a completed point ((X:Z), (Y:T)), Z, T != 0: x == 0 or y == 0.
CPZ_HD bool ristretto_is_identity(const ge_p1p1& a) { return fe_iszero(a.X) || fe_iszero(a.Y); }

// 8 little-endian words of an encoding.
CPZ_HD bool words_lt_p(const uint32_t w[8]) {
  // p = 2^255 - 19 : words ffffffed ffffffff x6 7fffffff.  s < p iff s - p borrows.
  const uint32_t pw[8] = {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)w[i] - pw[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow != 0;
}

// RFC 9496 4.3.1 DECODE.  Returns false for non-canonical, negative, non-square,
// negative-t or y == 0 encodings (dalek CompressedRistretto::decompress == None).
CPZ_HD bool ristretto_decode(ge_p3& out, const uint32_t w[8]) {
  const bool canonical = words_lt_p(w) && ((w[0] & 1) == 0);
  const fe s = fe_fromwords(w);
  const fe ss = fe_sq(s);
  const fe u1 = fe_sub(fe_one(), ss);
  const fe u2 = fe_add(fe_one(), ss);
  const fe u2_sqr = fe_sq(u2);
  const fe v = fe_sub(fe_neg(fe_mul(FE_D(), fe_sq(u1))), u2_sqr);
  fe invsqrt;
  const bool was_square = fe_invsqrt_m1(invsqrt, fe_mul(v, u2_sqr));
  const fe den_x = fe_mul(invsqrt, u2);
  const fe den_y = fe_mul(fe_mul(invsqrt, den_x), v);
  const fe x = fe_abs(fe_mul(s, fe_add(den_x, den_x)));  // s limbs are < 2^26: double den_x
  const fe y = fe_mul(u1, den_y);
  const fe t = fe_mul(x, y);
  out.X = x;
  out.Y = y;
  out.Z = fe_one();
  out.T = t;
  return canonical && was_square && !fe_isnegative(t) && !fe_iszero(y);
}

// RFC 9496 4.3.2 ENCODE -> 8 little-endian words.
CPZ_HD void ristretto_encode(uint32_t w[8], const ge_p3& p) {
  const fe u1 = fe_mul(fe_add(p.Z, p.Y), fe_sub(p.Z, p.Y));
  const fe u2 = fe_mul(p.X, p.Y);
  fe invsqrt;
  fe_invsqrt_m1(invsqrt, fe_mul(u1, fe_sq(u2)));
  const fe den1 = fe_mul(invsqrt, u1);
  const fe den2 = fe_mul(invsqrt, u2);
  const fe z_inv = fe_mul(fe_mul(den1, den2), p.T);
  const fe ix0 = fe_mul(p.X, FE_SQRT_M1());
  const fe iy0 = fe_mul(p.Y, FE_SQRT_M1());
  const fe enchanted = fe_mul(den1, FE_INVSQRT_A_MINUS_D());
  const bool rotate = fe_isnegative(fe_mul(p.T, z_inv));
  const fe x = fe_select(p.X, iy0, rotate);
  fe y = fe_select(p.Y, ix0, rotate);
  const fe den_inv = fe_select(den2, enchanted, rotate);
  y = fe_select(y, fe_neg(y), fe_isnegative(fe_mul(x, z_inv)));
  const fe s = fe_abs(fe_mul(den_inv, fe_sub(p.Z, y)));
  fe_towords(w, s);
}

// Affine Niels form of a point (one inversion): table entries for fixed bases.
CPZ_HD ge_niels p3_to_niels(const ge_p3& p) {
  const fe zinv = fe_invert(p.Z);
  const fe x = fe_mul(p.X, zinv);
  const fe y = fe_mul(p.Y, zinv);
  ge_niels r;
  r.ypx = fe_add(y, x);
  r.ymx = fe_sub(y, x);
  r.xy2d = fe_mul(fe_mul(x, y), FE_D2());
  return r;
}

}  // namespace cpz
