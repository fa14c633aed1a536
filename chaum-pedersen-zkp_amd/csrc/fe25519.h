// GF(2^255 - 19) arithmetic for gfx950, radix 2^25.5 (ten signed 32-bit limbs).
//
// Replaces curve25519-dalek 4.1.3's FieldElement (reached from the reference via
// src/primitives/ristretto.rs:120-185).  Limb i holds bits [off_i, off_i + w_i) with
// w = 26,25,26,25,...; off = 0,26,51,77,102,128,153,179,204,230.
//
// Why this radix on CDNA4: a 32x32->64 multiply-accumulate is ONE instruction
// (v_mad_i64_i32 / v_mad_u64_u32, measured at ~25 T lane-ops/s on MI355X, ~60% of the
// v_add_u32 rate), and with 25/26-bit limbs a whole column of ten products accumulates
// in a 64-bit register without any intermediate carry.  A full multiply is exactly 100
// MADs, a square 55, plus a 12-step carry chain.
//
// Limb bounds (checked by tests/test_device_arith.py through the host build of this
// header, CPZ_BOUNDS_CHECK): a "tight" element (output of mul/sq/carry) has
// |limb| <= 2^25 (+ 2^7 from the high-word carry, a few units more on limb 1); add/sub
// of two tight elements is "loose" (|limb| < 2^26.6) and is still a valid mul/sq operand:
// the worst column sum is 267 * 2^26.6 * 2^26.6 < 2^63.
//
// Everything is __host__ __device__ so the exact same code can be unit-tested on the
// CPU against the oracle; the product path only ever runs it on the GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CPZ_HD __host__ __device__ __forceinline__
#define CPZ_HDM __host__ __device__ __forceinline__
#else
#define CPZ_HD static inline
#define CPZ_HDM inline
#endif


#if defined(CPZ_BOUNDS_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <stdio.h>
#include <stdlib.h>
#define CPZ_ASSERT(c)                                                        \
  do {                                                                       \
    if (!(c)) {                                                              \
      fprintf(stderr, "cpz bound violated %s:%d: %s\n", __FILE__, __LINE__, #c); \
      abort();                                                               \
    }                                                                        \
  } while (0)
#else
#define CPZ_ASSERT(c) ((void)0)
#endif

namespace cpz {

#if defined(CPZ_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
// Host-only operation counters (tests/native/hostlib.cpp): the algorithmic work per
// proof that bench.py's roofline divides by the measured kernel time.
struct OpCounts {
  unsigned long long mul, sq;
};
inline OpCounts& op_counts() {
  static thread_local OpCounts c{0, 0};
  return c;
}
#define CPZ_COUNT(field) (++::cpz::op_counts().field)
#else
#define CPZ_COUNT(field) ((void)0)
#endif

struct fe {
  int32_t v[10];
};

// Largest |limb| a mul/sq operand may carry: 19 * bound must stay below 2^31 and the
// worst column sum (weight 267 in fe_mul) below 2^63.  Sums/differences of at most three
// tight elements stay below it.
constexpr int32_t kLooseBound = 108000000;  // ~2^26.69

CPZ_HD fe fe_const(int32_t a0, int32_t a1, int32_t a2, int32_t a3, int32_t a4, int32_t a5,
                   int32_t a6, int32_t a7, int32_t a8, int32_t a9) {
  fe r;
  r.v[0] = a0; r.v[1] = a1; r.v[2] = a2; r.v[3] = a3; r.v[4] = a4;
  r.v[5] = a5; r.v[6] = a6; r.v[7] = a7; r.v[8] = a8; r.v[9] = a9;
  return r;
}

CPZ_HD fe fe_zero() { return fe_const(0, 0, 0, 0, 0, 0, 0, 0, 0, 0); }
CPZ_HD fe fe_one() { return fe_const(1, 0, 0, 0, 0, 0, 0, 0, 0, 0); }

// Curve constants (value mod p, limb form); derived in oracle/pyoracle.py.
CPZ_HD fe FE_D() { return fe_const(56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712, 48412415, 21499315); }
CPZ_HD fe FE_D2() { return fe_const(45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993, 29715967, 9444199); }
CPZ_HD fe FE_SQRT_M1() { return fe_const(34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777, 326685, 11406482); }
CPZ_HD fe FE_INVSQRT_A_MINUS_D() { return fe_const(6111466, 4156064, 39310137, 12243467, 41204824, 120896, 20826367, 26493656, 6093567, 31568420); }
CPZ_HD fe FE_SQRT_AD_MINUS_ONE() { return fe_const(24849947, 33400850, 43495378, 6347714, 46036536, 32887293, 41837720, 18186727, 66238516, 14525638); }
CPZ_HD fe FE_ONE_MINUS_D_SQ() { return fe_const(6275446, 16937061, 44170319, 29780721, 11667076, 7397348, 39186143, 1766194, 42675006, 672202); }
CPZ_HD fe FE_INV2() { return fe_const(10, 0, 0, 0, 0, 0, 0, 0, 0, -16777216); }  // (p + 1) / 2
CPZ_HD fe FE_D_MINUS_ONE_SQ() { return fe_const(15551776, 22456977, 53683765, 23429360, 55212328, 10178283, 40474537, 4729243, 61826754, 23438029); }

CPZ_HD fe fe_add(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}

CPZ_HD fe fe_sub(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i] - b.v[i];
  return r;
}

CPZ_HD fe fe_neg(const fe& a) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = -a.v[i];
  return r;
}

// Conditional move: r = c ? b : a (c is 0/1 per lane; branch-free select).
CPZ_HD fe fe_select(const fe& a, const fe& b, bool c) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c ? b.v[i] : a.v[i];
  return r;
}

#if defined(CPZ_BOUNDS_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
CPZ_HD void fe_check_operand(const fe& a) {
  for (int i = 0; i < 10; i++) CPZ_ASSERT(a.v[i] < kLooseBound && a.v[i] > -kLooseBound);
}
#else
CPZ_HD void fe_check_operand(const fe&) {}
#endif

// Carry bias of column k: 2^(w_k - 1), w = 26, 25, 26, ...  Column accumulators start
// at this value (the first v_mad_i64_i32 adds it for free), so each carry step is just
//   c = H_k >> w_k,  H_(k+1) += c,  limb_k = (lo(H_k) & (2^w_k - 1)) - 2^(w_k - 1)
// (a 64-bit shift, a 64-bit add and two cheap 32-bit ops), which is the centred residue
// h_k - 2^w_k * round(h_k / 2^w_k) of the unbiased column h_k = H_k - bias_k.
CPZ_HD constexpr int64_t carry_bias(int k) { return (k & 1) ? (1LL << 24) : (1LL << 25); }

// Opaque copy of a column accumulator.  Every partial column sum goes through it, so
// LLVM cannot reassociate the sum (it would move the constant carry bias to the end, or
// split the chain into two halves, each costing an extra 64-bit add): column k is then
// exactly one v_mad_i64_i32 per product, the first one adding the bias from an SGPR pair.
// Non-volatile, so the scheduler still interleaves the ten columns freely.
CPZ_HD int64_t acc_pin(int64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}

// A constant the compiler must not see through (kept in an SGPR): (int64)x * opaque_sgpr(2^k)
// stays one v_mad_i64_i32 instead of becoming a 64-bit shift and add.
CPZ_HD int32_t opaque_sgpr(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(x));
#endif
  return x;
}

CPZ_HD int32_t unbias_limb(int64_t H, int k) {
  const uint32_t mask = (k & 1) ? 0x1ffffffu : 0x3ffffffu;
  return (int32_t)(((uint32_t)H & mask) - (uint32_t)carry_bias(k));
}

// Biased column sums -> tight limbs.  One chain 0 -> 1 -> ... -> 9 -> 0 (x19) -> 1: every
// column is carried once and the small wrap-around carry into limb 0 once more, so no
// reduced limb has to be widened back to 64 bits (the two-chain ref10 order needs that
// twice and is ~15 % more VALU work here).
//
// High-word carry: with H = hi 2^32 + lo, column k's high word
// moves into column k+1 as ONE v_mad_i64_i32 (hi * 2^(32-w) + H[k+1], the multiplier kept
// opaque in an SGPR so LLVM does not turn it back into a 64-bit shift + add), and the few
// bits of lo above the limb (lo >> w < 2^7) join limb k+1 in 32 bits (v_add3 with the
// unbias).  Per column: 1 MAD + 3 32-bit ops instead of a 64-bit shift, a 64-bit add and 2
// 32-bit ops; limbs end in [-2^(w-1), 2^(w-1) + 127).  k_verify_each 2.155 -> 2.105 ms per
// launch against the shift/add chain (A/B, two alternating runs each, one box).
CPZ_HD fe fe_carry_biased(int64_t H[10]) {
  fe r;
  uint32_t small = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int w = (k & 1) ? 25 : 26;
    const int32_t hi = (int32_t)(H[k] >> 32);
    const uint32_t lo = (uint32_t)H[k];
    H[k + 1] = acc_pin((int64_t)hi * (int64_t)opaque_sgpr(1 << (32 - w)) + H[k + 1]);
    r.v[k] = (int32_t)((lo & ((1u << w) - 1u)) - (uint32_t)carry_bias(k) + small);
    small = lo >> w;
  }
  const int32_t hi9 = (int32_t)(H[9] >> 32);
  const uint32_t lo9 = (uint32_t)H[9];
  r.v[9] = (int32_t)((lo9 & 0x1ffffffu) - (uint32_t)carry_bias(9) + small);
  // carry out of limb 9 = hi9 2^7 + (lo9 >> 25), times 19 into limb 0 (biased, then centred)
  const int64_t h0 = (int64_t)hi9 * (int64_t)opaque_sgpr(19 << 7) +
                     (int64_t)(uint64_t)(((uint32_t)r.v[0] + (uint32_t)carry_bias(0)) + 19u * (lo9 >> 25));
  r.v[1] += (int32_t)(h0 >> 26);
  r.v[0] = unbias_limb(h0, 0);
  return r;
}

// Unbiased 64-bit columns -> tight limbs.
CPZ_HD fe fe_carry_wide(int64_t h[10]) {
#pragma unroll
  for (int k = 0; k < 10; k++) h[k] += carry_bias(k);
  return fe_carry_biased(h);
}

// h = f * g.  Column k collects f_i g_j with (i + j) % 10 == k, times 19 when i + j >= 10
// (2^255 = 19 mod p) and times 2 when i and j are both odd (the half-bit offsets).
CPZ_HD fe fe_mul(const fe& f, const fe& g) {
  CPZ_COUNT(mul);
  fe_check_operand(f);
  fe_check_operand(g);
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = (int32_t)(19u * (uint32_t)g.v[i]);
    f2[i] = (int32_t)(2u * (uint32_t)f.v[i]);
  }
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int k = 0; k < 10; k++) {
      const int j = (k - i + 10) % 10;
      const int32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const int32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      h[k] = acc_pin((int64_t)a * (int64_t)b + (i == 0 ? carry_bias(k) : h[k]));
    }
  }
  fe r = fe_carry_biased(h);
  return r;
}

// Column sums of f^2 (using f_i f_j = f_j f_i: 55 products), each started at bias_k / div
// (div == 0: unbiased, for fe_carry_floor).
CPZ_HD void fe_sq_wide(int64_t h[10], const fe& f, int div) {
  CPZ_COUNT(sq);
  fe_check_operand(f);
  int32_t f2[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = (int32_t)(2u * (uint32_t)f.v[i]);
    f19[i] = (int32_t)(19u * (uint32_t)f.v[i]);
  }
  bool first[10] = {true, true, true, true, true, true, true, true, true, true};
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int k = (i + j) % 10;
      // coefficient = (i != j ? 2 : 1) * (both odd ? 2 : 1) * (i + j >= 10 ? 19 : 1)
      const int m2 = (i != j ? 2 : 1) * (((i & 1) && (j & 1)) ? 2 : 1);
      const int32_t a = (m2 == 1) ? f.v[i] : (m2 == 2 ? f2[i] : (int32_t)(2u * (uint32_t)f2[i]));
      const int32_t b = (i + j >= 10) ? f19[j] : f.v[j];
      h[k] = acc_pin((int64_t)a * (int64_t)b + (first[k] ? (div ? carry_bias(k) / div : 0) : h[k]));
      first[k] = false;
    }
  }
}

// h = f^2.
CPZ_HD fe fe_sq(const fe& f) {
  int64_t h[10];
  fe_sq_wide(h, f, 1);
  fe r = fe_carry_biased(h);
  return r;
}

// h = 2 f^2 (tight), as dalek's square2: the doubling is folded into the column sums
// (which start at half the bias, so the doubled sums carry the full bias).
CPZ_HD fe fe_sq2(const fe& f) {
  int64_t h[10];
  fe_sq_wide(h, f, 2);
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] += h[i];
  fe r = fe_carry_biased(h);
  return r;
}

// Unbiased columns -> limbs by floor carries: limb k in [0, 2^w_k) (limb 1 a few units
// above), one v_and_b32 per limb instead of the centred residue's and + subtract.  The
// limbs are twice as large as centred ones, which only a chain of squarings tolerates:
// there every operand is such an output, so 19 * limb < 2^30.3 and 4 * odd limb < 2^27.1
// fit the signed 32-bit multiplicands, and the worst column stays below 2^61.
CPZ_HD fe fe_carry_floor(int64_t H[10]) {
  fe r;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    H[k + 1] += H[k] >> ((k & 1) ? 25 : 26);
    r.v[k] = (int32_t)((uint32_t)H[k] & ((k & 1) ? 0x1ffffffu : 0x3ffffffu));
  }
  const int64_t h0 = (int64_t)r.v[0] + 19 * (H[9] >> 25);
  r.v[9] = (int32_t)((uint32_t)H[9] & 0x1ffffffu);
  r.v[1] += (int32_t)(h0 >> 26);
  r.v[0] = (int32_t)((uint32_t)h0 & 0x3ffffffu);
  return r;
}

// Repeated squaring (n >= 1): the intermediate squares use floor carries (above), the
// last one the centred carry, so the result is an ordinary tight element.
// The squaring loop stays rolled: letting the scheduler overlap one square's carry chain with
// the next square's products measured slower (k_verify_each 2.31 ms rolled vs 2.33 ms
// unrolled by 2 and 4, A/B).
CPZ_HD fe fe_sqn(fe f, int n) {
#pragma unroll 1
  for (int i = 1; i < n; i++) {
    int64_t h[10];
    fe_sq_wide(h, f, 0);
    f = fe_carry_floor(h);
  }
  return fe_sq(f);
}

// Reduce to the unique canonical representative and write 32 little-endian bytes.
CPZ_HD void fe_tobytes(uint8_t s[32], const fe& f) {
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  // Normalise to tight limbs first (handles loose inputs).
  fe t = fe_carry_wide(h);
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = t.v[i];
  // q = floor(value / p) in {0, 1} for tight input (value in (-2^255.1, 2^255.1)).
  int64_t q = (19 * h[9] + (1 << 24)) >> 25;
  q = (h[0] + q) >> 26;
  q = (h[1] + q) >> 25;
  q = (h[2] + q) >> 26;
  q = (h[3] + q) >> 25;
  q = (h[4] + q) >> 26;
  q = (h[5] + q) >> 25;
  q = (h[6] + q) >> 26;
  q = (h[7] + q) >> 25;
  q = (h[8] + q) >> 26;
  q = (h[9] + q) >> 25;
  h[0] += 19 * q;
  int64_t c;
  c = h[0] >> 26; h[1] += c; h[0] -= c * (1LL << 26);
  c = h[1] >> 25; h[2] += c; h[1] -= c * (1LL << 25);
  c = h[2] >> 26; h[3] += c; h[2] -= c * (1LL << 26);
  c = h[3] >> 25; h[4] += c; h[3] -= c * (1LL << 25);
  c = h[4] >> 26; h[5] += c; h[4] -= c * (1LL << 26);
  c = h[5] >> 25; h[6] += c; h[5] -= c * (1LL << 25);
  c = h[6] >> 26; h[7] += c; h[6] -= c * (1LL << 26);
  c = h[7] >> 25; h[8] += c; h[7] -= c * (1LL << 25);
  c = h[8] >> 26; h[9] += c; h[8] -= c * (1LL << 26);
  c = h[9] >> 25; h[9] -= c * (1LL << 25);  // drop 2^255 (value now in [0, p))
  uint32_t w[8];
  const uint32_t l0 = (uint32_t)h[0], l1 = (uint32_t)h[1], l2 = (uint32_t)h[2], l3 = (uint32_t)h[3],
                 l4 = (uint32_t)h[4], l5 = (uint32_t)h[5], l6 = (uint32_t)h[6], l7 = (uint32_t)h[7],
                 l8 = (uint32_t)h[8], l9 = (uint32_t)h[9];
  w[0] = l0 | (l1 << 26);
  w[1] = (l1 >> 6) | (l2 << 19);
  w[2] = (l2 >> 13) | (l3 << 13);
  w[3] = (l3 >> 19) | (l4 << 6);
  w[4] = l5 | (l6 << 25);
  w[5] = (l6 >> 7) | (l7 << 19);
  w[6] = (l7 >> 13) | (l8 << 12);
  w[7] = (l8 >> 20) | (l9 << 6);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    s[4 * i + 0] = (uint8_t)(w[i]);
    s[4 * i + 1] = (uint8_t)(w[i] >> 8);
    s[4 * i + 2] = (uint8_t)(w[i] >> 16);
    s[4 * i + 3] = (uint8_t)(w[i] >> 24);
  }
}

// Canonical little-endian words (8 x u32) of f.
CPZ_HD void fe_towords(uint32_t w[8], const fe& f) {
  uint8_t s[32];
  fe_tobytes(s, f);
#pragma unroll
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)s[4 * i] | ((uint32_t)s[4 * i + 1] << 8) | ((uint32_t)s[4 * i + 2] << 16) |
           ((uint32_t)s[4 * i + 3] << 24);
}

// Parse 8 little-endian words (bit 255 ignored) into limbs.  Not reduced mod p.
CPZ_HD fe fe_fromwords(const uint32_t w[8]) {
  fe r;
  r.v[0] = (int32_t)(w[0] & 0x3ffffff);
  r.v[1] = (int32_t)(((w[0] >> 26) | (w[1] << 6)) & 0x1ffffff);
  r.v[2] = (int32_t)(((w[1] >> 19) | (w[2] << 13)) & 0x3ffffff);
  r.v[3] = (int32_t)(((w[2] >> 13) | (w[3] << 19)) & 0x1ffffff);
  r.v[4] = (int32_t)((w[3] >> 6) & 0x3ffffff);
  r.v[5] = (int32_t)(w[4] & 0x1ffffff);
  r.v[6] = (int32_t)(((w[4] >> 25) | (w[5] << 7)) & 0x3ffffff);
  r.v[7] = (int32_t)(((w[5] >> 19) | (w[6] << 13)) & 0x1ffffff);
  r.v[8] = (int32_t)(((w[6] >> 12) | (w[7] << 20)) & 0x3ffffff);
  r.v[9] = (int32_t)((w[7] >> 6) & 0x1ffffff);
  return r;
}

CPZ_HD bool fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_towords(w, f);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) acc |= w[i];
  return acc == 0;
}

CPZ_HD bool fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_towords(w, f);
  return (w[0] & 1) != 0;
}

CPZ_HD bool fe_equal(const fe& a, const fe& b) { return fe_iszero(fe_sub(a, b)); }

CPZ_HD fe fe_abs(const fe& f) { return fe_select(f, fe_neg(f), fe_isnegative(f)); }

// f^((p-5)/8) = f^(2^252 - 3).
CPZ_HD fe fe_pow22523(const fe& z) {
  fe t0 = fe_sq(z);                        // 2
  fe t1 = fe_sqn(t0, 2);                   // 8
  t1 = fe_mul(z, t1);                      // 9
  t0 = fe_mul(t0, t1);                     // 11
  t0 = fe_sq(t0);                          // 22
  t0 = fe_mul(t1, t0);                     // 2^5 - 1
  t1 = fe_sqn(t0, 5);
  t0 = fe_mul(t1, t0);                     // 2^10 - 1
  t1 = fe_sqn(t0, 10);
  t1 = fe_mul(t1, t0);                     // 2^20 - 1
  fe t2 = fe_sqn(t1, 20);
  t1 = fe_mul(t2, t1);                     // 2^40 - 1
  t1 = fe_sqn(t1, 10);
  t0 = fe_mul(t1, t0);                     // 2^50 - 1
  t1 = fe_sqn(t0, 50);
  t1 = fe_mul(t1, t0);                     // 2^100 - 1
  t2 = fe_sqn(t1, 100);
  t1 = fe_mul(t2, t1);                     // 2^200 - 1
  t1 = fe_sqn(t1, 50);
  t0 = fe_mul(t1, t0);                     // 2^250 - 1
  t0 = fe_sqn(t0, 2);                      // 2^252 - 4
  return fe_mul(t0, z);                    // 2^252 - 3
}

// f^(p-2) = 1/f (0 -> 0).
CPZ_HD fe fe_invert(const fe& z) {
  fe t0 = fe_sq(z);                        // 2
  fe t1 = fe_sqn(t0, 2);                   // 8
  t1 = fe_mul(z, t1);                      // 9
  t0 = fe_mul(t0, t1);                     // 11
  fe t2 = fe_sq(t0);                       // 22
  t1 = fe_mul(t1, t2);                     // 2^5 - 1
  t2 = fe_sqn(t1, 5);
  t1 = fe_mul(t2, t1);                     // 2^10 - 1
  t2 = fe_sqn(t1, 10);
  t2 = fe_mul(t2, t1);                     // 2^20 - 1
  fe t3 = fe_sqn(t2, 20);
  t2 = fe_mul(t3, t2);                     // 2^40 - 1
  t2 = fe_sqn(t2, 10);
  t1 = fe_mul(t2, t1);                     // 2^50 - 1
  t2 = fe_sqn(t1, 50);
  t2 = fe_mul(t2, t1);                     // 2^100 - 1
  t3 = fe_sqn(t2, 100);
  t2 = fe_mul(t3, t2);                     // 2^200 - 1
  t2 = fe_sqn(t2, 50);
  t1 = fe_mul(t2, t1);                     // 2^250 - 1
  t1 = fe_sqn(t1, 5);                      // 2^255 - 32
  return fe_mul(t1, t0);                   // 2^255 - 21
}

// RFC 9496 section 4.2 SQRT_RATIO_M1(u, v): (was_square, |sqrt(u/v)| or |sqrt(i*u/v)|).
CPZ_HD bool fe_sqrt_ratio_m1(fe& out, const fe& u, const fe& v) {
  const fe v3 = fe_mul(fe_sq(v), v);
  const fe v7 = fe_mul(fe_sq(v3), v);
  fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  const fe check = fe_mul(v, fe_sq(r));
  const fe neg_u = fe_neg(u);
  const bool correct = fe_equal(check, u);
  const bool flipped = fe_equal(check, neg_u);
  const bool flipped_i = fe_equal(check, fe_mul(neg_u, FE_SQRT_M1()));
  r = fe_select(r, fe_mul(r, FE_SQRT_M1()), flipped || flipped_i);
  out = fe_abs(r);
  return correct || flipped;
}

// SQRT_RATIO_M1(1, v): the only form ristretto decode and encode use.  With u = 1 the
// products by u vanish and the three comparisons of `check` (with 1, -1 and -sqrt(-1))
// share one canonicalisation against constant words.
CPZ_HD bool fe_invsqrt_m1(fe& out, const fe& v) {
  const fe v3 = fe_mul(fe_sq(v), v);
  const fe v7 = fe_mul(fe_sq(v3), v);
  fe r = fe_mul(v3, fe_pow22523(v7));
  uint32_t w[8];
  fe_towords(w, fe_mul(v, fe_sq(r)));
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
  r = fe_select(r, fe_mul(r, FE_SQRT_M1()), flipped || flipped_i);
  out = fe_abs(r);
  return correct || flipped;
}

}  // namespace cpz
