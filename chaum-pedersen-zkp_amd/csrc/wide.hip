// k_verify_wide (the drop-in's calls of at most CPZ_WIDE_MAX proofs), in a translation unit of
// its own so that it is compiled with -falign-loops=64 (build_native.py): its row loops are
// single-wave issue streams whose speed moved by 12 % with their placement.
#include <hip/hip_runtime.h>

#include "cpz_kernels.h"
#include "ristretto.h"
#include "scalar25519.h"
#include "transcript.h"
#include "scalarmul.h"
#include "verify.h"
#include "rlc_dev.h"
#include "fe16.h"
#include "keccak_wave.h"
#include "proof_digits.h"

namespace cpz {

// ---------------------------------------------------------------------------------------
// k_verify_wide: the drop-in's calls of a few proofs, one proof per workgroup of six waves
// (eight with custom generators) and every field product spread over a 16-lane row (fe16.h): a lone wave's product takes
// ~145 ns there against ~220 ns on one lane, and a point operation is two such stages
// (the four products of each on the four rows) instead of eight products on a quad.
// Four chains c = 2 e + R of equation e: a table of 9 cached multiples in LDS (of -Y_e, or
// of +R_e), then the half-length Straus loop [u] (-Y_e) or [|v|] (-+R_e) (k_verify_small's
// waves 0/1).  Phase 1:
//   waves 0, 1  decode Y_e on rows 0-1 and R_e on rows 2-3 of wave e (the decode's products
//               run on row pairs anyway), hand R_e over in LDS, build Y_e's table
//   waves 3, 4  R_1's / R_2's table once it is handed over
//   wave 2      the challenge, response checks, split and digits (proof_digits) -- on a SIMD
//               of its own: with one decode per chain wave it shared wave 0's, and the two
//               serial paths slowed each other by ~6 us
// Phase 2: waves 0, 3, 1, 2 run chains 0..3; waves 4 and 5 [s'] B of both equations from the
// comb on two quads, half of the 16 windows each, as canonical words.
// Barrier A: the digits and tables.  Barrier B: the R chains' sums and [s'] B; the Y chains'
// waves add their equation's three sums and test the identity.  Barrier C: wave 0 writes the status with
// verify_proof's precedence.  Custom generators (VerifyArgs::vtab16, the pair's Niels tables
// as 16-bit limbs): waves 4..7 compute [s'] g and [s'] h on rows instead of the comb -- s' in
// eight 32-bit parts on 2^(32 q) B, two waves per equation with four parts each: 24 doublings
// + 16 additions per wave.
// ---------------------------------------------------------------------------------------
struct WideShared {
  uint32_t dig[16];            // u (0..3), |v| (4..7), s' (8..15) digit words
  uint32_t meta;               // bit 0: v < 0; bits 8..15: response status
  int32_t tab[4][9][4][16];    // chain, multiple 0..8, field (Y+X, Y-X, Z, 2dT), limb
  int32_t part[4][4][16];      // the R chains' sums: X, Y, Z, T limbs
  uint32_t sB[2][2][4][8];     // [s'] B of each equation from the comb: half, canonical words of X, Y, Z, T
  int32_t sBv[2][2][4][16];    // the same from the variable-base waves: equation, half, X, Y, Z, T limbs
  uint32_t bad[4];             // decode failure per chain
  uint32_t rid[2];             // R_e encodes the identity
  uint32_t eq[2];              // equation e holds
  uint32_t sponge[50];         // byte-wise transcript image (contexts off the fixed schedules)
  int32_t pt[2][4][16];        // R_e handed from its decoding wave to its table's builder
  uint32_t ready[2];           // ... and the flag that releases it
};

__device__ __forceinline__ int niels16_b(const int32_t* t16, int d, const r16::Lane& L);

// [s'] B_e on the rows from the pair's R16 Niels tables: s' in eight 32-bit parts on
// 2^(32 q) B_e, 4 radix-256 windows each -- 24 doublings and 32 additions (four 64-bit parts
// took 56 doublings and 32 additions, ~65 us, longer than the Straus chains).  With
// CPZ_WIDE_VB_WAVES = 4 two waves share an equation, parts 4 h .. 4 h + 3 each (24 doublings,
// 16 additions), to sh.sBv[e][h]; with 2 one wave takes all eight parts, to sh.sBv[e][0].
#ifndef CPZ_WIDE_VB_WAVES
#define CPZ_WIDE_VB_WAVES 4
#endif
template <class Shared>
__device__ __forceinline__ void wide_varbase(Shared& sh, const VerifyArgs& a, int e, int h, const r16::Lane& L) {
  constexpr int kParts = CPZ_WIDE_VB_WAVES == 4 ? 4 : 8;
  uint32_t sd[kParts];
#pragma unroll
  for (int k = 0; k < kParts; k++) sd[k] = sh.dig[8 + kParts * h + k];
  const int32_t* tq[kParts];
#pragma unroll
  for (int k = 0; k < kParts; k++)
    tq[k] = a.vtab16 + (size_t)(2 * kNielsLevelOfPart[kParts * h + k] + e) * kNielsEntries * 48;  // 2^(32 q) B_e
  r16::P4 acc = r16::identity(L);
#pragma unroll 1
  for (int b = 3; b >= 0; b--) {
    // digit 4 q + b of s' (radix 256, 4 per word) on 2^(32 q) B_e
    int op[kParts];
#pragma unroll
    for (int k = 0; k < kParts; k++) op[k] = niels16_b(tq[k], (int32_t)(sd[k] << (24 - 8 * b)) >> 24, L);
    if (b != 3) {
#pragma unroll 1
      for (int k = 0; k < 8; k++) acc = r16::dbl(acc, L);
    }
#pragma unroll
    for (int k = 0; k < kParts; k++) acc = r16::add_b(acc, op[k], L);
  }
  sh.sBv[e][h][L.row][L.k] = r16::sel4(acc.X, acc.Y, acc.Z, acc.T, L);
}

// row r's first-stage operand for the Niels entry d (|d| <= 128) of an R16 table (k_niels_r16):
// +: Y-X, Y+X, 2dxy, Z = 1;  -: Y+X, Y-X, -2dxy, 1;  0: the identity (1, 1, 0, 1)
__device__ __forceinline__ int niels16_b(const int32_t* t16, int d, const r16::Lane& L) {
  const bool ng = d < 0;
  const int ad = ng ? -d : d;
  const int f = L.row == 0 ? (ng ? 0 : 1) : (L.row == 1 ? (ng ? 1 : 0) : 2);
  int v = (ad == 0 || L.row == 3) ? (L.row == 2 ? 0 : r16::one(L)) : t16[((ad - 1) * 3 + f) * 16 + L.k];
  return (ng && L.row == 2 && ad != 0) ? -v : v;
}

// Chain table: entry j = cached(j P), j = 0..8, of the replicated point P; row r stores field r
// (Y+X, Y-X, Z, 2dT) of each entry at tab[64 j + 16 r + k].
__device__ __forceinline__ void wide_table(int32_t* tab, const r16::P4& P, const r16::Lane& L) {
  const int slot = L.row * 16 + L.k;
  tab[slot] = L.row == 3 ? 0 : r16::one(L);  // identity: Y+X = Y-X = Z = 1, 2dT = 0
  const r16::C4 c1 = r16::to_cached(P, L);
  tab[64 + slot] = r16::sel4(c1.ypx, c1.ymx, c1.z, c1.t2d, L);
  // entries 2..8: Y+X, Y-X, Z, and for now T (row 3's field); their 2 d T afterwards, row r
  // multiplying entries 2 + r and 6 + r at once -- two products instead of seven in the chain
  r16::P4 M = r16::dbl(P, L);
#pragma unroll 1
  for (int j = 2; j <= 8; j++) {
    if (j > 2) M = r16::add_b(M, r16::cached_b(c1, false, L), L);
    tab[64 * j + slot] = r16::sel4(M.Y + M.X, M.Y - M.X, M.Z, M.T, L);
  }
  __builtin_amdgcn_wave_barrier();  // same-wave LDS: the T words are read back below
  const int ja = 2 + L.row, jb = L.row < 3 ? 6 + L.row : 5;
  const int ta = tab[64 * ja + 48 + L.k], tb = tab[64 * jb + 48 + L.k];
  __builtin_amdgcn_wave_barrier();
  const int d2 = r16::K_D2(L);
  const int pa = r16::mul(ta, d2, L), pb = r16::mul(tb, d2, L);
  tab[64 * ja + 48 + L.k] = pa;
  if (L.row < 3) tab[64 * jb + 48 + L.k] = pb;
}

// The half-length Straus loop of a chain over its table (after barrier A): [u] (-Y) for a Y
// chain, and for an R chain [|v|] (v < 0 ? R : -R) = -[v] R from the table of +R.
template <class Shared>
__device__ __forceinline__ r16::P4 wide_straus(const Shared& sh, const int32_t* tab, bool isR, const r16::Lane& L) {
  uint32_t d[4];
#pragma unroll
  for (int k = 0; k < 4; k++) d[k] = sh.dig[(isR ? 4 : 0) + k];
  const bool flip = isR && !(sh.meta & 1u);
  // the field row r reads for +C: Y-X, Y+X, 2dT, Z; for -C: Y+X, Y-X, -2dT, Z
  const int fpos = L.row == 0 ? 1 : (L.row == 1 ? 0 : (L.row == 2 ? 3 : 2));
  const int fneg = L.row == 0 ? 0 : (L.row == 1 ? 1 : fpos);
  r16::P4 acc = r16::identity(L);
#pragma unroll 1
  for (int jj = 0; jj < 4; jj++) {
    const uint32_t wd = d[3 - jj];
#pragma unroll 1
    for (int m = 7; m >= 0; m--) {
      int dd = ((int32_t)(wd << (28 - 4 * m))) >> 28;
      dd = flip ? -dd : dd;
      const bool ng = dd < 0;
      const int ad = ng ? -dd : dd;
      int b = tab[64 * ad + 16 * (ng ? fneg : fpos) + L.k];
      b = (ng && L.row == 2) ? -b : b;
      if (jj != 0 || m != 7) {
        acc = r16::dbl(acc, L);
        acc = r16::dbl(acc, L);
        acc = r16::dbl(acc, L);
        acc = r16::dbl(acc, L);
      }
      acc = r16::add_b(acc, b, L);
    }
  }
  return acc;
}

// [s'] B of both equations from the comb on two quads (lanes 0-3: g, 4-7: h), windows
// 8 h .. 8 h + 7 of s' (radix 2^16), as canonical words to sh.sB[e][h]: waves 4 and 5 take
// a half each (one wave took 37-49 us for all 16, as long as the Straus chains).
template <class Shared>
__device__ __forceinline__ void wide_comb(Shared& sh, const VerifyArgs& a, int h, int l) {
  const int e = l >> 2, q = l & 3;
  uint32_t sd[4];
#pragma unroll
  for (int k = 0; k < 4; k++) sd[k] = sh.dig[8 + 4 * h + k];
  const CombTable comb{a.comb + (e ? kCombPerBase : 0)};
  ge_p3 B = ge_identity();
#pragma unroll 1
  for (int k = 0; k < 8; k++) {
    const int dgt = (int32_t)(sd[k >> 1] << (16 - 16 * (k & 1))) >> 16;
    const ge_niels nl = comb.lookup(8 * h + k, dgt);
    ge_cached cc;
    cc.YpX = nl.ypx;
    cc.YmX = nl.ymx;
    cc.T2d = nl.xy2d;
    cc.Z = fe_one();
    B = ge_add_quad(B, cc, q);
  }
  if (q == 0) {
    fe_towords(sh.sB[e][h][0], B.X);
    fe_towords(sh.sB[e][h][1], B.Y);
    fe_towords(sh.sB[e][h][2], B.Z);
    fe_towords(sh.sB[e][h][3], B.T);
  }
}

__global__ void __launch_bounds__(64 * (4 + CPZ_WIDE_VB_WAVES)) k_verify_wide(VerifyArgs a, ChallengeArgs ca) {
  __shared__ WideShared sh;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t i = blockIdx.x;
  const r16::Lane L = r16::lane_of(l);
  r16::P4 acc = r16::identity(L);
  // Straus chain of each wave (0: Y_1, 1: R_1, 2: Y_2, 3: R_2); the challenge wave
  const int chain = w == 0 ? 0 : (w == 1 ? 2 : (w == 2 ? 3 : (w == 3 ? 1 : -1)));
  constexpr int kDigitWave = 2;
#if defined(CPZ_CLOCK_PROBE)
  // timing builds only: shader-clock stamps of block 0 (wave 0 lane 0: start, decoded, table,
  // barrier A, Straus, barrier B, identity test, end; the challenge wave's lane 0: challenge
  // (12), digits (8); wave 4 lane 0: [s'] B (9); wave 1 lane 0: decoded, table, Straus
  // (13..15)) and the 100 MHz clock at wave 0's start and end (10, 11) -> a.clock_probe
  // (waves 0, 1, 2, 4 as a bit test: with `w <= 1 || w == 2 || w == 4` this compiler left the
  // pointer null on waves 2 and 4 -- their stamps read back as 0)
  static_assert(kDigitWave == 2, "stamp waves");
  const bool stamp_wave = ((0x17u >> w) & 1u) != 0;
  uint64_t* const stamps = (a.clock_probe && blockIdx.x == 0 && l == 0 && stamp_wave) ? a.clock_probe : nullptr;
#define CPZ_WIDE_STAMP(k) do { if (stamps) stamps[k] = __builtin_amdgcn_s_memtime(); } while (0)
  if (stamps && w == 0) stamps[10] = __builtin_amdgcn_s_memrealtime();
  if (w == 0) CPZ_WIDE_STAMP(0);
#else
#define CPZ_WIDE_STAMP(k) (void)0
#endif
  if (threadIdx.x == 0) {
    sh.ready[0] = 0u;
    sh.ready[1] = 0u;
  }
  __syncthreads();  // the hand-off flags
  if (w <= 1) {
    // ---- waves 0, 1: decode Y_e (rows 0-1) and R_e (rows 2-3); Y_e's table -------------------
    const int e = w;
    const bool isR = L.row >= 2;
    const uint32_t* src = isR ? (e ? a.r2 : a.r1) : (e ? a.y2 : a.y1);
    uint32_t wu[8];
    load_words8(wu, src, i);
    r16::P4 P;
    const bool ok = r16::decode(P, src + 8 * i, wu, L);
    if (w == 0) CPZ_WIDE_STAMP(1);
    if (w == 1) CPZ_WIDE_STAMP(13);
    if (l == 0) sh.bad[2 * e] = ok ? 0u : 1u;
    if (l == 32) {
      sh.bad[2 * e + 1] = ok ? 0u : 1u;
      sh.rid[e] = words8_zero(wu) ? 1u : 0u;
    }
    if (L.row == 2) {
      sh.pt[e][0][L.k] = P.X;
      sh.pt[e][1][L.k] = P.Y;
      sh.pt[e][2][L.k] = P.Z;
      sh.pt[e][3][L.k] = P.T;
    }
    if (l == 32) __hip_atomic_store(&sh.ready[e], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    // Y_e on every row (rows 2-3 take rows 0-1's limbs)
    P.X = (int)__builtin_amdgcn_permlane32_swap(P.X, P.X, false, false)[0];
    P.Y = (int)__builtin_amdgcn_permlane32_swap(P.Y, P.Y, false, false)[0];
    P.Z = (int)__builtin_amdgcn_permlane32_swap(P.Z, P.Z, false, false)[0];
    P.T = (int)__builtin_amdgcn_permlane32_swap(P.T, P.T, false, false)[0];
    wide_table(&sh.tab[2 * e][0][0][0], r16::neg(P), L);
    if (w == 0) CPZ_WIDE_STAMP(2);
    if (w == 1) CPZ_WIDE_STAMP(14);
  } else if (w == 3 || w == 4) {
    // ---- waves 3, 4: R_e's table once wave e has handed R_e over -----------------------------
    const int e = w - 3;
#pragma unroll 1
    while (__hip_atomic_load(&sh.ready[e], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
      __builtin_amdgcn_s_sleep(2);
    r16::P4 P;
    P.X = sh.pt[e][0][L.k];
    P.Y = sh.pt[e][1][L.k];
    P.Z = sh.pt[e][2][L.k];
    P.T = sh.pt[e][3][L.k];
    wide_table(&sh.tab[2 * e + 1][0][0][0], P, L);
  }
  if (w == kDigitWave) {
    // ---- the challenge, response checks, split, digits -----------------------------------------
    uint32_t dg[16], meta;
#if defined(CPZ_CLOCK_PROBE)
    proof_digits<true>(dg, meta, a, ca, i, l == 0, sh.sponge, 0, 1, stamps ? stamps + 12 : nullptr);
#else
    proof_digits<true>(dg, meta, a, ca, i, l == 0, sh.sponge, 0, 1);
#endif
    if (l == 0) {
#pragma unroll
      for (int k = 0; k < 16; k++) sh.dig[k] = dg[k];
      sh.meta = meta;
    }
    CPZ_WIDE_STAMP(8);
  }
  __syncthreads();  // A: digits, tables
  if (w == 0) CPZ_WIDE_STAMP(3);
  if (chain >= 0) {
    // ---- the four Straus chains ------------------------------------------------------------------
    const bool isR = (chain & 1) != 0;
    acc = wide_straus(sh, &sh.tab[chain][0][0][0], isR, L);
    if (isR) sh.part[chain][L.row][L.k] = r16::sel4(acc.X, acc.Y, acc.Z, acc.T, L);
    if (w == 0) CPZ_WIDE_STAMP(4);
    if (w == 1) CPZ_WIDE_STAMP(15);
  } else if (w == 4) {
    // ---- wave 4: [s'] B of both equations (comb on two quads, or the variable-base rows) --------
    if (a.vtab16)
      wide_varbase(sh, a, 0, 0, L);
    else if (l < 8)
      wide_comb(sh, a, 0, l);
    CPZ_WIDE_STAMP(9);
  } else if (w >= 5) {
    // ---- waves 5.. : variable bases, wave 4 + e + 2 h takes half h of equation e; comb: wave 5
    // the second half of both equations' windows
    if (a.vtab16)
      wide_varbase(sh, a, (w - 4) & 1, (w - 4) >> 1, L);
    else if (w == 5 && l < 8)
      wide_comb(sh, a, 1, l);
  }
  __syncthreads();  // B: the R chains' sums, [s'] B
  if (w == 0) CPZ_WIDE_STAMP(5);
  if (chain == 0 || chain == 2) {
    // Q_e = [u] (-Y_e) + (-[v] R_e) + [s'] B_e, identity (mod E[4])
    const int e = chain >> 1;
    r16::P4 R;
    R.X = sh.part[chain + 1][0][L.k];
    R.Y = sh.part[chain + 1][1][L.k];
    R.Z = sh.part[chain + 1][2][L.k];
    R.T = sh.part[chain + 1][3][L.k];
    acc = r16::add_b(acc, r16::cached_b(r16::to_cached(R, L), false, L), L);
    r16::P4 S;
    if (a.vtab16) {
      if (CPZ_WIDE_VB_WAVES == 4) {
        S.X = sh.sBv[e][1][0][L.k];
        S.Y = sh.sBv[e][1][1][L.k];
        S.Z = sh.sBv[e][1][2][L.k];
        S.T = sh.sBv[e][1][3][L.k];
        acc = r16::add_b(acc, r16::cached_b(r16::to_cached(S, L), false, L), L);
      }
      S.X = sh.sBv[e][0][0][L.k];
      S.Y = sh.sBv[e][0][1][L.k];
      S.Z = sh.sBv[e][0][2][L.k];
      S.T = sh.sBv[e][0][3][L.k];
    } else {
      S.X = r16::limb_of(sh.sB[e][1][0], L);
      S.Y = r16::limb_of(sh.sB[e][1][1], L);
      S.Z = r16::limb_of(sh.sB[e][1][2], L);
      S.T = r16::limb_of(sh.sB[e][1][3], L);
      acc = r16::add_b(acc, r16::cached_b(r16::to_cached(S, L), false, L), L);
      S.X = r16::limb_of(sh.sB[e][0][0], L);
      S.Y = r16::limb_of(sh.sB[e][0][1], L);
      S.Z = r16::limb_of(sh.sB[e][0][2], L);
      S.T = r16::limb_of(sh.sB[e][0][3], L);
    }
    acc = r16::add_b(acc, r16::cached_b(r16::to_cached(S, L), false, L), L);
    const bool eq = r16::is_identity(acc);
    if (l == 0) sh.eq[e] = eq ? 1u : 0u;
    if (w == 0) CPZ_WIDE_STAMP(6);
  }
  __syncthreads();  // C
  if (threadIdx.x != 0) return;
  const bool bad = (sh.bad[0] | sh.bad[1] | sh.bad[2] | sh.bad[3]) != 0;
  const bool rid = (sh.rid[0] | sh.rid[1]) != 0;
  const uint8_t st_s = (uint8_t)(sh.meta >> 8);
  uint8_t st;
  if (bad) st = kStBadPoint;
  else if (st_s == kStBadScalar) st = kStBadScalar;
  else if (rid && !a.eq_only) st = kStIdentity;
  else if (st_s == kStZeroS) st = kStZeroS;
  else if (st_s == kStBadChallenge) st = kStBadScalar;
  else st = (sh.eq[0] & sh.eq[1]) ? kStOk : kStEqFail;
  a.status[i] = st;
#if defined(CPZ_CLOCK_PROBE)
  CPZ_WIDE_STAMP(7);
  if (stamps) stamps[11] = __builtin_amdgcn_s_memrealtime();
#endif
#undef CPZ_WIDE_STAMP
}

hipError_t launch_verify_wide(const VerifyArgs& a, const ChallengeArgs& ca, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  if (a.pre || a.blocks || (a.vtab && !a.vtab16) || (!a.vtab && !a.comb)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_verify_wide, dim3((unsigned)a.n), dim3(64 * (a.vtab16 ? 4 + CPZ_WIDE_VB_WAVES : 6)), 0, st, a, ca);
  return hipGetLastError();
}

}  // namespace cpz
