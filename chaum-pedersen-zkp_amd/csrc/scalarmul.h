// Variable-time scalar multiplication loops (verification inputs are public, so
// data-dependent digits are allowed; SIMT divergence is avoided by using fixed windows:
// every lane adds at every window, digit 0 adds the identity).
//
// Replaces the reference's Ristretto255::scalar_mul (ristretto.rs:153-155) as used in
// verify_one (batch.rs:216-222): instead of four independent constant-time
// multiplications, each equation is one Straus double-scalar loop
//     Q = [s] B + [c] V        (B = g or h fixed, V = -y1 or -y2 per proof)
// whose result is compared with r by ristretto equality.
#pragma once
#include "ristretto.h"

namespace cpz {

constexpr int kTableV = 8;     // cached multiples 1..8 of a variable base (radix-16 digits)
constexpr int kTableSlots = kTableV + 1;  // + the identity at slot 0 (digit 0 needs no select)
constexpr int kTableB = 128;   // Niels multiples 1..128 of a fixed base (radix-256 digits)

// Fixed-base comb: for each of the 16 radix-2^16 windows k, the affine Niels multiples
// j * 2^(16 k) * B, j = 1..2^15, of one base (64 MiB per base in HBM).  [s] B for any
// s < 2^253 is then 16 mixed additions and no doubling.
constexpr int kCombWindows = 16;
constexpr int kCombEntries = 1 << 15;
constexpr int64_t kCombPerBase = (int64_t)kCombWindows * kCombEntries;

// Device view of one base's comb (entries in global memory).
struct CombTable {
  const ge_niels* p;
  CPZ_HDM ge_niels lookup(int k, int digit) const {
    const int mag = digit < 0 ? -digit : digit;
    const ge_niels* e = p + (int64_t)k * kCombEntries + (mag == 0 ? 0 : mag - 1);
    ge_niels r;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4* s = reinterpret_cast<const uint4*>(e);
    uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
    for (int v = 0; v < (int)(sizeof(ge_niels) / 16); v++) d[v] = s[v];
#else
    r = *e;
#endif
    return ge_niels_cneg(mag == 0 ? ge_niels_identity() : r, digit < 0);
  }
};

CPZ_HD ge_cached cached_load(const ge_cached* p) {
  ge_cached r;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* s = reinterpret_cast<const uint4*>(p);
  uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
  for (int v = 0; v < (int)(sizeof(ge_cached) / 16); v++) d[v] = s[v];
#else
  r = *p;
#endif
  return r;
}

CPZ_HD void cached_store(ge_cached* p, const ge_cached& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* s = reinterpret_cast<const uint4*>(&c);
  uint4* d = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int v = 0; v < (int)(sizeof(ge_cached) / 16); v++) d[v] = s[v];
#else
  *p = c;
#endif
}

CPZ_HD ge_niels niels_lookup(const ge_niels* tab, int digit) {
  const int mag = digit < 0 ? -digit : digit;
  const ge_niels e = tab[(mag == 0 ? 1 : mag) - 1];
  const ge_niels r = mag == 0 ? ge_niels_identity() : e;
  return ge_niels_cneg(r, digit < 0);
}

// tab[0] is the identity, tab[k] = k P: one load and a conditional negation.
CPZ_HD ge_cached cached_lookup(const ge_cached* tab, int digit) {
  const int mag = digit < 0 ? -digit : digit;
  return ge_cached_cneg(cached_load(tab + mag), digit < 0);
}
// Four doublings of a pending completed point.
CPZ_HD ge_p1p1 dbl4(const ge_p1p1& cur) {
  ge_p1p1 t = cur;
#pragma unroll 1
  for (int d = 0; d < 4; d++) t = p2_dbl(p1p1_to_p2(t));
  return t;
}

CPZ_HD ge_p1p1 p1p1_identity() {
  ge_p1p1 cur;
  cur.X = fe_zero(); cur.Y = fe_one(); cur.Z = fe_one(); cur.T = fe_one();
  return cur;
}

// Writes the identity and the cached multiples 1..8 of an AFFINE P (Z = 1, as decoded) to
// tab[0..8]: 1 doubling + 6 mixed additions of P in Niels form (3M each instead of 4M for a
// cached addition).
// (An unrolled 4-doubling / 3-addition schedule saves a few more multiplications but keeps
// three extended points live and measured slower from the extra spills.)
CPZ_HD void build_cached_table(ge_cached* tab, const ge_p3& P) {
  ge_niels n1;
  n1.ypx = fe_add(P.Y, P.X);
  n1.ymx = fe_sub(P.Y, P.X);
  n1.xy2d = fe_mul(P.T, FE_D2());
  cached_store(tab, ge_cached_identity());
  {
    ge_cached c1;
    c1.YpX = n1.ypx;
    c1.YmX = n1.ymx;
    c1.Z = P.Z;
    c1.T2d = n1.xy2d;
    cached_store(tab + 1, c1);
  }
  ge_p3 acc = p1p1_to_p3(p3_dbl(P));
  cached_store(tab + 2, p3_to_cached(acc));
#pragma unroll 1
  for (int k = 3; k <= kTableV; k++) {
    acc = p1p1_to_p3(ge_add_niels(acc, n1));
    cached_store(tab + k, p3_to_cached(acc));
  }
}

// Q = [s] B + [c] V.  tab_v: cached multiples 1..8 of V; tab_b: Niels multiples 1..128
// of B; cdig: radix-16 signed digits of c; sdig: radix-256 signed digits of s.
// 63 x 4 doublings, 64 cached additions, 32 Niels additions.
CPZ_HD ge_p3 straus_vartime(const ge_cached* tab_v, const ge_niels* tab_b, const uint32_t cdig_in[8],
                            const uint32_t sdig_in[8]) {
  uint32_t cdig[8], sdig[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { cdig[j] = cdig_in[j]; sdig[j] = sdig_in[j]; }
  ge_p1p1 cur = p1p1_identity();
#pragma unroll 1
  for (int j = 7; j >= 0; j--) {
    const uint32_t wc = cdig[7], wg = sdig[7];
#pragma unroll
    for (int t = 7; t > 0; t--) { cdig[t] = cdig[t - 1]; sdig[t] = sdig[t - 1]; }
#pragma unroll 1
    for (int m = 7; m >= 0; m--) {
      const int dc = ((int32_t)(wc << (28 - 4 * m))) >> 28;
      const ge_cached ev = cached_lookup(tab_v, dc);
      if (j != 7 || m != 7) cur = dbl4(cur);
      cur = ge_add_cached(p1p1_to_p3(cur), ev);
      if ((m & 1) == 0) {
        const int dg = ((int32_t)(wg << (24 - 8 * (m >> 1)))) >> 24;
        cur = ge_add_niels(p1p1_to_p3(cur), niels_lookup(tab_b, dg));
      }
    }
  }
  return p1p1_to_p3(cur);
}

// Adds [s] B to a pending completed point through the comb (16 mixed additions).
// sdig: 16 radix-2^16 signed digits (sc_recode_radix65536).
template <class Comb>
CPZ_HD ge_p1p1 comb_add(ge_p1p1 cur, const Comb& comb, const uint32_t sdig_in[8]) {
  uint32_t sd[8];
#pragma unroll
  for (int j = 0; j < 8; j++) sd[j] = sdig_in[j];
#pragma unroll 1
  for (int j = 0; j < 8; j++) {
    const uint32_t w = sd[0];
#pragma unroll
    for (int t = 0; t < 7; t++) sd[t] = sd[t + 1];
    // (requesting both entries of the pair before the first addition measured 2 % slower:
    // 30 more live VGPRs)
#pragma unroll
    for (int m = 0; m < 2; m++) {
      const int d = (int32_t)(w << (16 - 16 * m)) >> 16;
      cur = ge_add_niels(p1p1_to_p3(cur), comb.lookup(2 * j + m, d));
    }
  }
  return cur;
}

// Half-size per-proof check with the comb (see verify.h):
//   Q = [u] Y' + [v] R' (Straus, 31 x 4 doublings, 64 cached additions) + [s'] B (comb),
// returned as a completed point (callers only test it for the identity).
// tab_y / tab_r: cached multiples 1..8 of Y' / R'; udig, vdig: 32 radix-16 signed digits of
// u, |v| < 6 * 2^124; sdig: 16 radix-2^16 signed digits of s' < 2^253.
template <class Comb>
CPZ_HD ge_p1p1 straus_half_comb(const ge_cached* tab_y, const ge_cached* tab_r, const Comb& comb,
                              const uint32_t udig_in[4], const uint32_t vdig_in[4], const uint32_t sdig[8]) {
  uint32_t ud[4], vd[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    ud[j] = udig_in[j];
    vd[j] = vdig_in[j];
  }
  ge_p1p1 cur = p1p1_identity();
#pragma unroll 1
  for (int j = 3; j >= 0; j--) {
    const uint32_t wu = ud[3], wv = vd[3];
#pragma unroll
    for (int t = 3; t > 0; t--) {
      ud[t] = ud[t - 1];
      vd[t] = vd[t - 1];
    }
#pragma unroll 1
    for (int m = 7; m >= 0; m--) {
      const int du = ((int32_t)(wu << (28 - 4 * m))) >> 28;
      const int dv = ((int32_t)(wv << (28 - 4 * m))) >> 28;
      // both table loads issued before the four doublings, which hide their latency
      // (the tables live in the HBM-backed scratch slab; measured ~1 % faster)
      const ge_cached ey = cached_lookup(tab_y, du), er = cached_lookup(tab_r, dv);
      if (j != 3 || m != 7) cur = dbl4(cur);
      cur = ge_add_cached(p1p1_to_p3(cur), ey);
      cur = ge_add_cached(p1p1_to_p3(cur), er);
    }
  }
  return comb_add(cur, comb, sdig);
}

// [s] B through the comb (prover path): 16 mixed additions.
template <class Comb>
CPZ_HD ge_p3 comb_mul(const Comb& comb, const uint32_t sdig[8]) {
  return p1p1_to_p3(comb_add(p1p1_identity(), comb, sdig));
}

// [s] B by Horner over radix-256 signed digits (prover path).
CPZ_HD ge_p3 fixed_base_mul(const ge_niels* tab_b, const uint32_t sdig_in[8]) {
  uint32_t sdig[8];
#pragma unroll
  for (int j = 0; j < 8; j++) sdig[j] = sdig_in[j];
  ge_p1p1 cur = p1p1_identity();
#pragma unroll 1
  for (int j = 7; j >= 0; j--) {
    const uint32_t wg = sdig[7];
#pragma unroll
    for (int t = 7; t > 0; t--) sdig[t] = sdig[t - 1];
#pragma unroll 1
    for (int m = 3; m >= 0; m--) {
      if (j != 7 || m != 3) {
        cur = dbl4(cur);
        cur = dbl4(cur);
      }
      const int dg = ((int32_t)(wg << (24 - 8 * m))) >> 24;
      cur = ge_add_niels(p1p1_to_p3(cur), niels_lookup(tab_b, dg));
    }
  }
  return p1p1_to_p3(cur);
}

// k * B for 1 <= k <= 255 by double-and-add (table construction).
CPZ_HD ge_p3 small_mul(const ge_p3& B, int k) {
  ge_p3 acc = ge_identity();
#pragma unroll 1
  for (int bit = 7; bit >= 0; bit--) {
    acc = p1p1_to_p3(p3_dbl(acc));
    if ((k >> bit) & 1) acc = ge_add(acc, B);
  }
  return acc;
}

}  // namespace cpz
