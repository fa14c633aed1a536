// Device helpers shared by the RLC kernels (rlc.hip) and the partitioned batch check
// (part.hip): row loads, the 128-bit weights, signed radix-2^16 recoding, point stores, and
// the quad-cooperative point arithmetic of the latency-bound reduction kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "rlc.h"
#include "verify.h"

namespace cpz {

// In-kernel clock probe of the RLC kernels (CPZ_CLOCK_PROBE timing-only builds, timing_only.h;
// tools/time_verify.py MODE=rlc): per wave, lane 0 stores shader-clock (s_memtime) and
// constant 100 MHz (s_memrealtime) ticks of the wave's work, its absolute 100 MHz start and
// end, and its hardware id at probe[5 * wave] -- the clock the kernel ran at, against which
// bench.py prices its MAD rate.  Product builds compile none of it.
struct ClockStamp {
  uint64_t t0 = 0, q0 = 0;
  __device__ __forceinline__ void start() {
#if defined(CPZ_CLOCK_PROBE)
    t0 = __builtin_amdgcn_s_memtime();
    q0 = __builtin_amdgcn_s_memrealtime();
#endif
  }
  __device__ __forceinline__ void stop(uint64_t* probe, int64_t wave) const {
#if defined(CPZ_CLOCK_PROBE)
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
    if (probe && (threadIdx.x & 63) == 0) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t* out = probe + 5 * wave;
      out[0] = t1 - t0;
      out[1] = q1 - q0;
      out[2] = q0;
      out[3] = q1;
      out[4] = (uint64_t)hw | ((uint64_t)xcc << 32);
    }
#else
    (void)probe;
    (void)wave;
#endif
  }
};

__device__ __forceinline__ void rlc_load8(uint32_t w[8], const uint32_t* base, int64_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(base + 8 * i);
  const uint4 a = p[0], b = p[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// The weight sum_{k<8} w_k 2^(16k) (w_k the int16 halves of u[0..3]) reduced mod l: with
// U the unsigned 128-bit value of u, the signed value is U - 2 (U & 0x8000...8000).
__device__ __forceinline__ sc rlc_weight(const uint32_t u[4]) {
  uint32_t d[8];
  uint32_t borrow = 0, carry = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint32_t m = k < 4 ? (u[k] & 0x80008000u) : 0u;
    const uint32_t twice = (m << 1) | carry;  // bits shifted out of the previous word
    carry = m >> 31;
    const uint32_t x = k < 4 ? u[k] : 0u;
    const uint64_t t = (uint64_t)x - twice - borrow;
    d[k] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
#pragma unroll
  for (int k = 5; k < 8; k++) d[k] = borrow ? 0xffffffffu : 0u;  // sign extension
  sc r;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {  // negative: add l (wraps mod 2^256 to the value in [0, l))
    const uint64_t t = (uint64_t)d[k] + (borrow ? SC_L(k) : 0u) + c;
    r.w[k] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  return r;
}

// Signed radix-2^16 digits of a scalar < 2^253 (16 windows, digit in [-2^15, 2^15)).
__device__ __forceinline__ void recode16(int16_t d[kRlcWindows], const uint32_t s[8]) {
  int32_t carry = 0;
#pragma unroll
  for (int w = 0; w < kRlcWindows; w++) {
    const int32_t chunk = (int32_t)((s[w >> 1] >> (16 * (w & 1))) & 0xffffu) + carry;
    carry = (chunk + 0x8000) >> 16;
    d[w] = (int16_t)(chunk - (carry << 16));
  }
}

__device__ __forceinline__ ge_niels niels_from_p3_affine(const ge_p3& P, bool neg) {
  // P has Z = 1 (decoded): (y + x, y - x, 2d x y), negated by swapping and negating.
  ge_niels r;
  r.ypx = fe_add(P.Y, P.X);
  r.ymx = fe_sub(P.Y, P.X);
  r.xy2d = fe_mul(P.T, FE_D2());
  return ge_niels_cneg(r, neg);
}

__device__ __forceinline__ void store_niels(ge_niels* dst, const ge_niels& v) {
  const uint4* s = reinterpret_cast<const uint4*>(&v);
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(ge_niels) / 16); k++) d[k] = s[k];
}

__device__ __forceinline__ ge_niels load_niels(const ge_niels* src) {
  ge_niels v;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(&v);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(ge_niels) / 16); k++) d[k] = s[k];
  return v;
}

__device__ __forceinline__ void store_p3(ge_p3* dst, const ge_p3& v) {
  const uint4* s = reinterpret_cast<const uint4*>(&v);
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(ge_p3) / 16); k++) d[k] = s[k];
}

__device__ __forceinline__ ge_p3 load_p3(const ge_p3* src) {
  ge_p3 v;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(&v);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(ge_p3) / 16); k++) d[k] = s[k];
  return v;
}

// ---------------------------------------------------------------------------------------
// Quad-cooperative point arithmetic for the reduction kernels below, which are chains of
// dependent additions run by few waves (latency-bound: one wave issues ~1 VALU instruction
// per 4-8 cycles whatever the chip's width).  The four lanes of a quad hold the same
// points; each lane computes one of the four independent products of a round on operands
// it selects by its lane index, and the four products are broadcast inside the quad with
// DPP quad_perm moves (full-rate VALU, no LDS).  A cached addition (8 products) is then two
// product latencies instead of eight.  Quads must be whole (all four lanes active).
// ---------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ fe fe_quad_bcast(const fe& a) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = __builtin_amdgcn_mov_dpp(a.v[i], K * 0x55, 0xf, 0xf, false);
  return r;
}

__device__ __forceinline__ fe fe_sel4(int q, const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
  fe r = fe_select(a0, a1, q == 1);
  r = fe_select(r, a2, q == 2);
  return fe_select(r, a3, q == 3);
}

// lane q multiplies its own pair (a, b); every lane of the quad receives the four products
__device__ __forceinline__ void quad_mul(fe& m0, fe& m1, fe& m2, fe& m3, const fe& a, const fe& b) {
  const fe m = fe_mul(a, b);
  m0 = fe_quad_bcast<0>(m);
  m1 = fe_quad_bcast<1>(m);
  m2 = fe_quad_bcast<2>(m);
  m3 = fe_quad_bcast<3>(m);
}

// P + Q (Q cached) -> extended: ge_add_cached + p1p1_to_p3 as two quad rounds
__device__ __forceinline__ ge_p3 ge_add_quad(const ge_p3& p, const ge_cached& c, int q) {
  fe PP, MM, TT2d, ZZ;
  quad_mul(PP, MM, TT2d, ZZ, fe_sel4(q, fe_add(p.Y, p.X), fe_sub(p.Y, p.X), p.T, p.Z),
           fe_sel4(q, c.YpX, c.YmX, c.T2d, c.Z));
  const fe ZZ2 = fe_add(ZZ, ZZ);
  const fe X = fe_sub(PP, MM), Y = fe_add(PP, MM), Z = fe_add(ZZ2, TT2d), T = fe_sub(ZZ2, TT2d);
  ge_p3 r;  // p1p1_to_p3: X T, Z Y, Z T, X Y
  quad_mul(r.X, r.Y, r.Z, r.T, fe_sel4(q, X, Z, Z, X), fe_sel4(q, T, Y, T, Y));
  return r;
}

// cached form of an extended point: its one product (2d T) done by every lane of the quad
__device__ __forceinline__ ge_p3 ge_add_quad(const ge_p3& p, const ge_p3& o, int q) {
  return ge_add_quad(p, p3_to_cached(o), q);
}

// (X : Y : Z) -> extended (XZ : YZ : Z^2 : XY), one quad round
__device__ __forceinline__ ge_p3 p2_to_p3_quad(const ge_p2& t, int q) {
  ge_p3 d;
  quad_mul(d.X, d.Y, d.Z, d.T, fe_sel4(q, t.X, t.Y, t.Z, t.X), fe_sel4(q, t.Z, t.Z, t.Z, t.Y));
  return d;
}

// 2^k P with the chain kept distributed: lane q holds v_q = [X, Y, Z, X+Y][q] of the
// current point and squares it (lane 2: 2 Z^2); the four squares are broadcast, each lane
// forms its own product operands (lane 0: X1 T1, 1: Y1 Z1, 2: Z1 T1), so after the product
// lane q holds coordinate q of the double and lane 3 rebuilds X+Y from lanes 0 and 1.  Per
// doubling that is 6 broadcasts and 4 selects per limb instead of the 7 and 9 of p2_dbl_quad
// (the final's 240-doubling chain issues ~500 instructions per doubling from one wave).
__device__ __forceinline__ ge_p3 p3_dbl_n_quad(const ge_p3& p, int k, int q) {
  if (k == 0) return p;
  fe v = fe_sel4(q, p.X, p.Y, p.Z, fe_add(p.X, p.Y));
#pragma unroll 1
  for (int i = 0; i < k; i++) {
    int64_t h[10];
    fe_sq_wide(h, v, 1);
#pragma unroll
    for (int l = 0; l < 10; l++) h[l] = q == 2 ? 2 * h[l] - carry_bias(l) : h[l];  // 2 Z^2, bias once
    const fe sq = fe_carry_biased(h);
    const fe XX = fe_quad_bcast<0>(sq), YY = fe_quad_bcast<1>(sq), ZZ2 = fe_quad_bcast<2>(sq),
             XpY2 = fe_quad_bcast<3>(sq);
    const fe Y1 = fe_add(YY, XX), Z1 = fe_sub(YY, XX);
    const fe X1 = fe_sub(XpY2, Y1), T1 = fe_sub(ZZ2, Z1);
    const fe m = fe_mul(fe_select(fe_select(X1, Y1, q == 1), Z1, q == 2), fe_select(T1, Z1, q == 1));
    v = fe_select(m, fe_add(fe_quad_bcast<0>(m), fe_quad_bcast<1>(m)), q == 3);
  }
  ge_p2 t;
  t.X = fe_quad_bcast<0>(v);
  t.Y = fe_quad_bcast<1>(v);
  t.Z = fe_quad_bcast<2>(v);
  return p2_to_p3_quad(t, q);
}


}  // namespace cpz
