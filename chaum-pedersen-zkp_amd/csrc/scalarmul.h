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
#include "timing_only.h"
#include "ristretto.h"

namespace cpz {

constexpr int kTableV = 8;     // cached multiples 1..8 of a variable base (radix-16 digits)
constexpr int kTableSlots = kTableV + 1;  // + the identity at slot 0 (digit 0 needs no select)
constexpr int kTableB = 128;   // Niels multiples 1..128 of a fixed base (radix-256 digits)

// Fixed-base comb: for each of the 16 radix-2^16 windows k, the affine Niels multiples
// j * 2^(16 k) * B, j = 0..2^15 (slot 0 the identity, so a zero digit needs no select), of one
// base (64 MiB per base in HBM).  [s] B for any s < 2^253 is then 16 mixed additions and no
// doubling.
constexpr int kCombWindows = 16;
constexpr int kCombEntries = 1 << 15;          // nonzero multiples per window
constexpr int kCombStride = kCombEntries + 1;  // + the identity at slot 0
constexpr int64_t kCombPerBase = (int64_t)kCombWindows * kCombStride;

// Device view of one base's comb (entries in global memory).
struct CombTable {
  const ge_niels* p;
  CPZ_HDM ge_niels lookup(int k, int digit) const {
    const int mag = digit < 0 ? -digit : digit;
    const ge_niels* e = p + (int64_t)k * kCombStride + mag;
    ge_niels r;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4* s = reinterpret_cast<const uint4*>(e);
    uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
    for (int v = 0; v < (int)(sizeof(ge_niels) / 16); v++) d[v] = s[v];
#else
    r = *e;
#endif
    return ge_niels_cneg(r, digit < 0);
  }
};

// Per-proof table of cached points (tab[0] = identity, tab[k] = k P), addressed as a base
// pointer plus a 32-bit byte offset per entry: entry e at col + 160 e, its 16-byte vectors
// contiguous.  The verify kernel keeps each thread's entries contiguous (col = the thread's
// slab slot).  Measured against two interleaved layouts in which one wave-wide load
// of a vector reads 1 KiB of consecutive slots (lane-interleaved over the whole slab, and
// wave-interleaved: 64 lanes per 184 KB region): 48.0 M and 48.2 M against 51.8 M proofs/s for
// the contiguous form (same gpurun call, two passes each) -- a lane's 9 entries in one 1.4 KB
// run beat full-line wave accesses spread over 10 separate 1-KiB rows per lookup.
constexpr int kCachedVecs = (int)(sizeof(ge_cached) / 16);

struct SlabTable {
  char* base;    // slab (wave-uniform)
  uint32_t col;  // byte offset of this thread's table (entry 0)
  static constexpr uint32_t kEntryBytes = kCachedVecs * 16;
  // entry e: one 32-bit offset per lookup; the 16-byte vectors of the entry are then
  // addressed as immediate offsets from it (computing base + 32-bit offset + 16 v in 32 bits
  // per vector made the compiler hoist one address register per (entry, vector) out of the
  // loops and spill)
  CPZ_HDM const char* entry(int e) const { return base + (col + (uint32_t)e * kEntryBytes); }
  // the table that starts e0 entries further on
  CPZ_HDM SlabTable shifted(int e0) const { return SlabTable{base, col + (uint32_t)e0 * kEntryBytes}; }
  CPZ_HDM ge_cached load(int e) const {
    ge_cached r;
    uint32_t* d = reinterpret_cast<uint32_t*>(&r);
    const char* p = entry(e);
#pragma unroll
    for (int v = 0; v < kCachedVecs; v++) {
#if defined(__HIP_DEVICE_COMPILE__)
      const uint4 x = *reinterpret_cast<const uint4*>(p + 16 * v);
      d[4 * v] = x.x; d[4 * v + 1] = x.y; d[4 * v + 2] = x.z; d[4 * v + 3] = x.w;
#else
      const uint32_t* s = reinterpret_cast<const uint32_t*>(p + 16 * v);
      for (int k = 0; k < 4; k++) d[4 * v + k] = s[k];
#endif
    }
    return r;
  }
  CPZ_HDM void store(int e, const ge_cached& c) const {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&c);
    char* p = const_cast<char*>(entry(e));
#pragma unroll
    for (int v = 0; v < kCachedVecs; v++) {
#if defined(__HIP_DEVICE_COMPILE__)
      *reinterpret_cast<uint4*>(p + 16 * v) = make_uint4(s[4 * v], s[4 * v + 1], s[4 * v + 2], s[4 * v + 3]);
#else
      uint32_t* d = reinterpret_cast<uint32_t*>(p + 16 * v);
      for (int k = 0; k < 4; k++) d[k] = s[4 * v + k];
#endif
    }
  }
};

// Digit words of a scalar multiplication held outside the registers: word k at p[k * stride].
// The verify kernel keeps them in LDS (one column per thread, conflict-free), which takes 16
// words per proof out of the Straus loop's register budget; the host build uses a plain array.
struct DigitRef {
  const uint32_t* p;
  int stride;
  CPZ_HDM uint32_t operator[](int k) const { return p[k * stride]; }
};
CPZ_HD DigitRef host_digits(const uint32_t* a) { return DigitRef{a, 1}; }

// A host array of cached points as a table (unit tests).
CPZ_HD SlabTable host_table(ge_cached* p) { return SlabTable{reinterpret_cast<char*>(p), 0u}; }

CPZ_HD ge_niels niels_lookup(const ge_niels* tab, int digit) {
  const int mag = digit < 0 ? -digit : digit;
  const ge_niels e = tab[(mag == 0 ? 1 : mag) - 1];
  const ge_niels r = mag == 0 ? ge_niels_identity() : e;
  return ge_niels_cneg(r, digit < 0);
}

// tab[0] is the identity, tab[k] = k P: one load and a conditional negation.
CPZ_HD ge_cached cached_lookup(const SlabTable& tab, int digit) {
  const int mag = digit < 0 ? -digit : digit;
  return ge_cached_cneg(tab.load(mag), digit < 0);
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
CPZ_HD void build_cached_table(const SlabTable& tab, const ge_p3& P) {
  ge_niels n1;
  n1.ypx = fe_add(P.Y, P.X);
  n1.ymx = fe_sub(P.Y, P.X);
  n1.xy2d = fe_mul(P.T, FE_D2());
  tab.store(0, ge_cached_identity());
  {
    ge_cached c1;
    c1.YpX = n1.ypx;
    c1.YmX = n1.ymx;
    c1.Z = P.Z;
    c1.T2d = n1.xy2d;
    tab.store(1, c1);
  }
  ge_p3 acc = p1p1_to_p3(p3_dbl(P));
  tab.store(2, p3_to_cached(acc));
#pragma unroll 1
  for (int k = 3; k <= kTableV; k++) {
    acc = p1p1_to_p3(ge_add_niels(acc, n1));
    tab.store(k, p3_to_cached(acc));
  }
}

// Q = [s] B + [c] V.  tab_v: cached multiples 1..8 of V; tab_b: Niels multiples 1..128
// of B; cdig: radix-16 signed digits of c; sdig: radix-256 signed digits of s.
// 63 x 4 doublings, 64 cached additions, 32 Niels additions.
CPZ_HD ge_p3 straus_vartime(const SlabTable& tab_v, const ge_niels* tab_b, const uint32_t cdig_in[8],
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
template <class Comb, class Dig>
CPZ_HD ge_p1p1 comb_add(ge_p1p1 cur, const Comb& comb, const Dig& sd) {
#pragma unroll 1
  for (int j = 0; j < 8; j++) {
    const uint32_t w = sd[j];
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
template <class Comb, class Dig>
CPZ_HD ge_p1p1 straus_half_comb(const SlabTable& tab_y, const SlabTable& tab_r, const Comb& comb, const Dig& ud,
                              const Dig& vd, const Dig& sdig) {
  ge_p1p1 cur = p1p1_identity();
#pragma unroll 1
  for (int j = 3; j >= 0; j--) {
    const uint32_t wu = ud[j], wv = vd[j];
#pragma unroll 1
    for (int m = 7; m >= 0; m--) {
      const int du = ((int32_t)(wu << (28 - 4 * m))) >> 28;
      const int dv = ((int32_t)(wv << (28 - 4 * m))) >> 28;
      // both table loads issued before the four doublings, which hide their latency
      // (the tables live in the HBM-backed scratch slab; measured ~1 % faster)
      const ge_cached ey = cached_lookup(tab_y, du), er = cached_lookup(tab_r, dv);
      if (j != 3 || m != 7) cur = dbl4(cur);
#if defined(CPZ_EXP_NIELS_TABLES)
      // timing experiment only (timing_only.h: wrong verdicts): the entries added as affine
      // Niels points, Z never read -- the best case of normalised per-proof tables
      cur = ge_add_niels(p1p1_to_p3(cur), ge_niels{ey.YpX, ey.YmX, ey.T2d, {0, 0}});
      cur = ge_add_niels(p1p1_to_p3(cur), ge_niels{er.YpX, er.YmX, er.T2d, {0, 0}});
#else
      cur = ge_add_cached(p1p1_to_p3(cur), ey);
      cur = ge_add_cached(p1p1_to_p3(cur), er);
#endif
    }
  }
  return comb_add(cur, comb, sdig);
}

// [s] B through the comb (prover path): 16 mixed additions.
template <class Comb>
CPZ_HD ge_p3 comb_mul(const Comb& comb, const uint32_t sdig[8]) {
  return p1p1_to_p3(comb_add(p1p1_identity(), comb, host_digits(sdig)));
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
