// Random-linear-combination batch verification on gfx950: one Pippenger multi-scalar
// multiplication per batch (or per shard / per sub-range during fallback).
//
// Replaces the reference's batch check (verify_batch / verify_batch_equations,
// batch.rs:233-312) with the CORRECT equation (the reference omits alpha on y*c,
// batch.rs:297-300):
//   P = sum_i  [a_i s_i] g - [a_i] r1_i - [a_i c_i] y1_i + [b_i s_i] h - [b_i] r2_i - [b_i c_i] y2_i
// with 128-bit weights in place of random_scalar (batch.rs:240): ChaCha20 block first+i of
// the seed read as 32 int16 words w_k, a_i = sum_{k<8} w_k 2^(16k), b_i = the same over
// w_8..w_15 (pyoracle.rlc_weights).  P is the identity iff every weighted proof satisfies
// both equations, except with probability <= 2^-128 per forged proof.  The r-points'
// scalars a_i, b_i ARE signed radix-2^16 digit vectors (8 windows, no recoding, windows
// 8..15 empty): 48 instead of 64 bucket additions per proof.  Proofs whose decode-level
// status is non-zero carry zero weight and are reported individually.
//
// Pipeline (all on one stream):
//   k_rlc_prepare   1 thread / proof: 4 decodes, weights, 4 scalar products, negated
//                   affine-Niels points, signed radix-2^16 digits (16 windows), per-block
//                   sums of a_i s_i and b_i s_i.
//   k_rlc_extra     g and h as two more MSM points with the summed scalars.
//   k_rlc_hist      per-(chunk, window) bucket histograms (LDS, 32768 buckets).
//   k_rlc_bscan     per-bucket prefix over chunks; bucket totals.
//   k_rlc_scan      exclusive scan -> bucket offsets.
//   k_rlc_coarse /  point ids sorted by bucket in two LDS-staged passes (256 coarse bins,
//   k_rlc_fine      then 128 buckets per bin) so that every global write is a contiguous run.
//   k_rlc_bucket    1 thread / (window, 64-entry chunk of the sorted list): mixed
//                   additions, partials of buckets spanning chunks fixed up by
//                   k_rlc_bucket_fix (load-balanced whatever the bucket sizes).
//   k_rlc_segment   1 thread / (window, 32-bucket segment): running sums.
//   k_rlc_window    1 block / window: sum_b b * B_b from the segments (LDS tree).
//   k_rlc_final16   2^(16w) combine (Horner on 16-lane rows, fe16.h), encode -> 32-byte
//                   partial + identity flag (k_rlc_final: the quad tree form).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "fe16.h"
#include "rlc.h"
#include "rlc_dev.h"
#include "verify.h"

namespace cpz {

// ---------------------------------------------------------------------------------------
// k_rlc_prepare
// ---------------------------------------------------------------------------------------
// Points are decoded one at a time and written out immediately (register pressure: one
// decoded point live, not four).  A proof that turns out not to be live afterwards gets
// all its digits zeroed, so its (possibly garbage) Niels entries never enter a bucket.
__global__ void __launch_bounds__(kRlcPrepBlock, 2) k_rlc_prepare(RlcPrepArgs a) {
  __shared__ sc red_a[kRlcPrepBlock];
  __shared__ sc red_b[kRlcPrepBlock];
  const int64_t i = (int64_t)blockIdx.x * kRlcPrepBlock + threadIdx.x;
  ClockStamp clk;
  clk.start();
  sc zero;
#pragma unroll
  for (int k = 0; k < 8; k++) zero.w[k] = 0;
  red_a[threadIdx.x] = zero;
  red_b[threadIdx.x] = zero;
  if (i < a.n) {
    // All scalar work first -- weights (replacing random_scalar, batch.rs:240: one ChaCha20
    // block per proof), the four points' digits and the block-sum terms a s, b s (parked in
    // LDS) -- so that nothing but the flags is live across the four decodes (56 VGPRs were
    // spilled when the weights, c and s stayed in registers through them).
    {
      uint32_t blk[16];
      chacha20_block(blk, a.seed, a.first_index + (uint64_t)i, 0);
      const sc wa = rlc_weight(blk), wb = rlc_weight(blk + 4);
      sc c, sv;
      rlc_load8(c.w, a.c, i);
      rlc_load8(sv.w, a.s, i);
      // q = 0: -r1 (a), 1: -y1 (a c), 2: -r2 (b), 3: -y2 (b c); the r-points' digits are the
      // weight words themselves (windows 8..15 empty)
#pragma unroll 1
      for (int q = 0; q < 4; q++) {
        int16_t d[kRlcWindows];
        if (q & 1) {
          recode16(d, sc_mul(q == 1 ? wa : wb, c).w);
        } else {
          const uint32_t* u = q == 0 ? blk : blk + 4;
#pragma unroll
          for (int wv = 0; wv < kRlcWindows; wv++)
            d[wv] = wv < 8 ? (int16_t)(u[wv >> 1] >> (16 * (wv & 1))) : (int16_t)0;
        }
#pragma unroll
        for (int wv = 0; wv < kRlcWindows; wv++) a.digits[(int64_t)wv * a.dstride + 4 * i + q] = d[wv];
      }
      red_a[threadIdx.x] = sc_mul(wa, sv);
      red_b[threadIdx.x] = sc_mul(wb, sv);
    }
    bool ok = true, ident = false;
#pragma unroll 1
    for (int q = 0; q < 4; q++) {
      const uint32_t* src = q == 0 ? a.r1 : (q == 1 ? a.y1 : (q == 2 ? a.r2 : a.y2));
      uint32_t w[8];
      rlc_load8(w, src, i);
      if (!(q & 1)) ident = words8_zero(w) || ident;
      ge_p3 P;
      ok = ristretto_decode(P, w) && ok;
      store_niels(a.pts + 4 * i + q, niels_from_p3_affine(P, true));
    }
    const uint8_t st_s = a.status[i];
    uint8_t st;
    if (!ok) st = kStBadPoint;
    else if (st_s == kStBadScalar) st = kStBadScalar;
    else if (ident && !a.eq_only) st = kStIdentity;
    else if (st_s == kStZeroS) st = kStZeroS;
    else st = kStOk;
    a.status[i] = st;
    if (st != kStOk) {  // zero weight: no digits, no block-sum terms
      atomicOr(a.any_bad, 1);
      red_a[threadIdx.x] = zero;
      red_b[threadIdx.x] = zero;
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int wv = 0; wv < kRlcWindows; wv++) a.digits[(int64_t)wv * a.dstride + 4 * i + q] = 0;
    }
  }
  clk.stop(a.clock_probe, i >> 6);
  // block sums of a_i s_i, b_i s_i (mod l), one per kRlcSumBlock proofs (two per workgroup)
  static_assert(kRlcPrepBlock == 2 * kRlcSumBlock, "two block sums per prepare workgroup");
  __syncthreads();
  for (int off = kRlcSumBlock / 2; off > 0; off >>= 1) {
    if ((threadIdx.x % kRlcSumBlock) < off) {
      red_a[threadIdx.x] = sc_add(red_a[threadIdx.x], red_a[threadIdx.x + off]);
      red_b[threadIdx.x] = sc_add(red_b[threadIdx.x], red_b[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x % kRlcSumBlock == 0) {
    const int64_t sb = 2 * (int64_t)blockIdx.x + threadIdx.x / kRlcSumBlock;
    a.block_sums[2 * sb] = red_a[threadIdx.x];
    a.block_sums[2 * sb + 1] = red_b[threadIdx.x];
  }
}

// Small batches (launch_rlc_prepare: n <= kRlcPrepWideMax): four lanes per proof -- lane q
// writes point q's digits and decodes point q -- so a BatchVerifier-sized batch waits for one
// decode per lane instead of four in sequence (on one lane per proof the prepare took 0.28 -
// 0.37 ms at n = 1 .. 1000, a latency, with most of the chip idle).  The weights' ChaCha20
// block is recomputed by each of the four lanes.  A block is 64 proofs: its a s and b s sums
// go to quarter_sums, and k_rlc_bsum4 adds each 128-proof block's two into block_sums.
__global__ void __launch_bounds__(256, 2) k_rlc_prepare4(RlcPrepArgs a) {
  __shared__ sc red_a[64];
  __shared__ sc red_b[64];
  const int q = threadIdx.x & 3, p = threadIdx.x >> 2;
  const int64_t i = (int64_t)blockIdx.x * 64 + p;
  sc zero;
#pragma unroll
  for (int k = 0; k < 8; k++) zero.w[k] = 0;
  if (q == 0) red_a[p] = zero;
  if (q == 2) red_b[p] = zero;
  bool ok = true, ident = false;
  if (i < a.n) {
    {
      // q = 0: -r1 (a), 1: -y1 (a c), 2: -r2 (b), 3: -y2 (b c), as k_rlc_prepare
      uint32_t blk[16];
      chacha20_block(blk, a.seed, a.first_index + (uint64_t)i, 0);
      const uint32_t* u = q < 2 ? blk : blk + 4;
      int16_t d[kRlcWindows];
      if (q & 1) {
        sc c;
        rlc_load8(c.w, a.c, i);
        recode16(d, sc_mul(rlc_weight(u), c).w);
      } else {
#pragma unroll
        for (int wv = 0; wv < kRlcWindows; wv++) d[wv] = wv < 8 ? (int16_t)(u[wv >> 1] >> (16 * (wv & 1))) : (int16_t)0;
        sc sv;
        rlc_load8(sv.w, a.s, i);
        (q == 0 ? red_a : red_b)[p] = sc_mul(rlc_weight(u), sv);
      }
#pragma unroll
      for (int wv = 0; wv < kRlcWindows; wv++) a.digits[(int64_t)wv * a.dstride + 4 * i + q] = d[wv];
    }
    const uint32_t* src = q == 0 ? a.r1 : (q == 1 ? a.y1 : (q == 2 ? a.r2 : a.y2));
    uint32_t w[8];
    rlc_load8(w, src, i);
    ident = !(q & 1) && words8_zero(w);
    ge_p3 P;
    ok = ristretto_decode(P, w);
    store_niels(a.pts + 4 * i + q, niels_from_p3_affine(P, true));
  }
  // the proof's four lanes are consecutive lanes of one wave: OR their flags
  int f = (ok ? 0 : 1) | (ident ? 2 : 0);
  f |= __shfl_xor(f, 1);
  f |= __shfl_xor(f, 2);
  if (i < a.n) {
    const uint8_t st_s = a.status[i];
    uint8_t st;
    if (f & 1) st = kStBadPoint;
    else if (st_s == kStBadScalar) st = kStBadScalar;
    else if ((f & 2) && !a.eq_only) st = kStIdentity;
    else if (st_s == kStZeroS) st = kStZeroS;
    else st = kStOk;
    if (q == 0) a.status[i] = st;  // after the quad's loads of it: one wave, in program order
    if (st != kStOk) {  // zero weight: no digits, no block-sum terms
      if (q == 0) {
        atomicOr(a.any_bad, 1);
        red_a[p] = zero;
      }
      if (q == 2) red_b[p] = zero;
#pragma unroll
      for (int wv = 0; wv < kRlcWindows; wv++) a.digits[(int64_t)wv * a.dstride + 4 * i + q] = 0;
    }
  }
  __syncthreads();
  for (int off = 32; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      red_a[threadIdx.x] = sc_add(red_a[threadIdx.x], red_a[threadIdx.x + off]);
      red_b[threadIdx.x] = sc_add(red_b[threadIdx.x], red_b[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.quarter_sums[2 * blockIdx.x] = red_a[0];
    a.quarter_sums[2 * blockIdx.x + 1] = red_b[0];
  }
}

// block_sums of a wide prepare: sum block b (kRlcSumBlock = 128 proofs) is quarters 2 b and
// 2 b + 1 (those that exist).
__global__ void __launch_bounds__(64) k_rlc_bsum4(const sc* __restrict__ quarter_sums, int64_t nq,
                                                  sc* __restrict__ block_sums, int64_t nb) {
  static_assert(kRlcSumBlock == 128, "two 64-proof quarters per block sum");
  const int64_t t = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= 2 * nb) return;
  const int64_t b = t >> 1;
  const int ab = (int)(t & 1);
  sc acc;
#pragma unroll
  for (int k = 0; k < 8; k++) acc.w[k] = 0;
  for (int64_t k = 2 * b; k < 2 * b + 2 && k < nq; k++) acc = sc_add(acc, quarter_sums[2 * k + ab]);
  block_sums[2 * b + ab] = acc;
}

// ---------------------------------------------------------------------------------------
// k_rlc_extra: g and h with scalars sum_{sum blocks in [b0, b1)} (a s), (b s).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_rlc_extra(RlcMsmArgs a, const sc* __restrict__ block_sums, int64_t b0,
                                                   int64_t b1, const ge_niels* __restrict__ tab) {
  __shared__ sc red_a[256];
  __shared__ sc red_b[256];
  sc sa, sb;
#pragma unroll
  for (int k = 0; k < 8; k++) { sa.w[k] = 0; sb.w[k] = 0; }
  for (int64_t b = b0 + threadIdx.x; b < b1; b += 256) {
    sa = sc_add(sa, block_sums[2 * b]);
    sb = sc_add(sb, block_sums[2 * b + 1]);
  }
  red_a[threadIdx.x] = sa;
  red_b[threadIdx.x] = sb;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      red_a[threadIdx.x] = sc_add(red_a[threadIdx.x], red_a[threadIdx.x + off]);
      red_b[threadIdx.x] = sc_add(red_b[threadIdx.x], red_b[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 2) {
    const sc s = threadIdx.x == 0 ? red_a[0] : red_b[0];
    const int64_t j = a.e0 + threadIdx.x;
    store_niels(a.pts + j, tab[threadIdx.x * kNielsEntriesRlc]);  // entry k = 1: g, h
    int16_t d[kRlcWindows];
    recode16(d, s.w);
#pragma unroll
    for (int wv = 0; wv < kRlcWindows; wv++) a.digits[(int64_t)wv * a.dstride + j] = d[wv];
  }
}

// point index for flat position t over [p0, p1) U [e0, e0 + 2)
__device__ __forceinline__ int64_t msm_point(const RlcMsmArgs& a, int64_t t) {
  const int64_t np = a.p1 - a.p0;
  return t < np ? a.p0 + t : a.e0 + (t - np);
}

// ---------------------------------------------------------------------------------------
// Counting sort by bucket, per window, without global atomics.  Window w's points are cut
// into `groups` chunks; sort block (g, w) owns chunk g:
//   k_rlc_hist     LDS histogram of its chunk -> bhist[w][g][*]
//   k_rlc_bscan    per (w, b): exclusive prefix of bhist[w][*][b] over g, total -> counts
//   k_rlc_scan     per w: exclusive scan of counts over b -> offsets
//   k_rlc_scatter  LDS cursors = offsets + block prefix; ranks from LDS atomics
// The order of points inside a bucket is not fixed, which does not matter: the bucket
// sum is the same group element whatever the order.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kRlcSortBlock) k_rlc_hist(RlcMsmArgs a) {
  extern __shared__ uint32_t hist[];  // kRlcBuckets counters (128 KB)
  const int g = blockIdx.x, w = blockIdx.y;
  for (int b = threadIdx.x; b < kRlcBuckets; b += kRlcSortBlock) hist[b] = 0;
  __syncthreads();
  const int64_t np = a.p1 - a.p0, total = np + 2;
  const int64_t t0 = (int64_t)g * a.chunk;
  const int64_t t1 = t0 + a.chunk < total ? t0 + a.chunk : total;
  const int16_t* dig = a.digits + (int64_t)w * a.dstride;
  // 8 digits per 16-byte load where the range is aligned (chunks are multiples of 64 points;
  // p0 is a multiple of 4 * 256 on every RLC path), so each thread has 8 entries per load
  // round trip instead of one
  int64_t ts = t0;
  if ((a.p0 & 7) == 0) {
    const int64_t v1 = t0 + (((t1 < np ? t1 : np) - t0) & ~(int64_t)7);
    for (int64_t t = t0 + 8 * threadIdx.x; t < v1; t += 8 * kRlcSortBlock) {
      const uint4 q = *reinterpret_cast<const uint4*>(dig + a.p0 + t);
      const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int d = (int16_t)(wv[k >> 1] >> (16 * (k & 1)));
        if (d != 0) atomicAdd(&hist[(d < 0 ? -d : d) - 1], 1u);
      }
    }
    ts = v1 > t0 ? v1 : t0;
  }
  for (int64_t t = ts + threadIdx.x; t < t1; t += kRlcSortBlock) {
    const int d = dig[msm_point(a, t)];
    if (d != 0) atomicAdd(&hist[(d < 0 ? -d : d) - 1], 1u);
  }
  __syncthreads();
  uint32_t* out = a.bhist + ((int64_t)w * a.groups + g) * kRlcBuckets;
  for (int b = threadIdx.x; b < kRlcBuckets; b += kRlcSortBlock) out[b] = hist[b];
}

__global__ void __launch_bounds__(256) k_rlc_bscan(RlcMsmArgs a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)kRlcWindows * kRlcBuckets) return;
  const int w = (int)(t / kRlcBuckets);
  const int b = (int)(t % kRlcBuckets);
  uint32_t* h = a.bhist + (int64_t)w * a.groups * kRlcBuckets + b;
  uint32_t run = 0;
  // 8 loads in flight, then their 8 stores (a load after a store to the same array would
  // otherwise wait for it)
  for (int g0 = 0; g0 < a.groups; g0 += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = g0 + k < a.groups ? h[(int64_t)(g0 + k) * kRlcBuckets] : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (g0 + k < a.groups) h[(int64_t)(g0 + k) * kRlcBuckets] = run;
      run += v[k];
    }
  }
  a.counts[t] = run;
}

// One block per window: exclusive scan of kRlcBuckets counts -> offsets.
__global__ void __launch_bounds__(1024) k_rlc_scan(RlcMsmArgs a) {
  __shared__ uint32_t part[1024];
  const int w = blockIdx.x;
  constexpr int per = kRlcBuckets / 1024;
  const uint32_t* cnt = a.counts + (int64_t)w * kRlcBuckets;
  uint32_t local[per];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < per; k++) {
    local[k] = cnt[threadIdx.x * per + k];
    sum += local[k];
  }
  part[threadIdx.x] = sum;
  __syncthreads();
  // Hillis-Steele inclusive scan over the 1024 partial sums
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - sum;  // exclusive
  uint32_t* off = a.offsets + (int64_t)w * (kRlcBuckets + 1);
#pragma unroll
  for (int k = 0; k < per; k++) {
    off[threadIdx.x * per + k] = run;
    run += local[k];
  }
  if (threadIdx.x == 1023) off[kRlcBuckets] = run;
}

// Scatter of the point ids into bucket order, in two LDS-staged passes so that every
// global write is part of a contiguous run.  (A direct scatter -- one 4-byte write per
// entry to a random position of a 16 MB window array -- costs a whole HBM burst per entry:
// measured 0.94 ms per 2^20 proofs, against 0.21 ms for the same kernel writing
// sequentially.)
//   k_rlc_coarse  block (chunk g, window w), tiles of 8192 points: an LDS counting sort of
//                 the tile by coarse bin (256 bins of 128 buckets), then each bin's run is
//                 appended to the bin's region of `inter` (runs of ~32 entries).
//   k_rlc_fine    block (coarse bin c, window w): the region's entries (~16 K for a full
//                 window) are ranked by bucket with LDS cursors into an LDS image of the
//                 region, which is then copied to idx contiguously.  A region too large for
//                 LDS (the top window's concentrated bins) is scattered directly instead;
//                 it spans < 1 MB, so its writes still merge in L2.
// A coarse bin's region of `inter` is the same range of positions its buckets occupy in
// idx, so both passes share the offsets from k_rlc_scan.
// Coarse-sorted entries are 32 bits: fine bucket (7 bits) << 25 | sign << 24 | flat position t
// of the point in this MSM (t < kRlcMaxMsmPoints); k_rlc_fine maps t back to the point id.
// (64-bit entries holding the id itself measured 0.61 against 0.53 ms per 2^20 proofs.)
constexpr int kRlcCoarse = 256;
constexpr int kRlcFinePerCoarse = kRlcBuckets / kRlcCoarse;  // 128
constexpr int kRlcTile = 8192;
// Entries k_rlc_fine stages in LDS (76 KB: two blocks per CU).  Larger regions -- the top
// window's bins, where every y-point lands in the first 64 -- are scattered directly.  A 144 KB
// image (one block per CU) measured 0.531 / 0.533 ms for the sort against 0.502 / 0.502 (A/B,
// one call); 48 KB (regions of windows 0-7 no longer fit) 0.656.
#ifndef CPZ_RLC_FINE_CAP
#define CPZ_RLC_FINE_CAP (19 * 1024)
#endif
constexpr int kRlcFineCap = CPZ_RLC_FINE_CAP;

__global__ void __launch_bounds__(kRlcSortBlock) k_rlc_coarse(RlcMsmArgs a) {
  __shared__ uint64_t buf[kRlcTile];
  __shared__ uint32_t gbase[kRlcCoarse], cnt[kRlcCoarse], start[kRlcCoarse];
  __shared__ uint32_t part[kRlcSortBlock];
  __shared__ uint32_t wtot[kRlcCoarse / 64];
  const int g = blockIdx.x, w = blockIdx.y;
  const int tid = threadIdx.x;
  const uint32_t* off = a.offsets + (int64_t)w * (kRlcBuckets + 1);
  const uint32_t* base = a.bhist + ((int64_t)w * a.groups + g) * kRlcBuckets;
  {  // this block's start in each coarse bin: off[first bucket] + its bucket bases
    constexpr int per = kRlcBuckets / kRlcSortBlock;  // 32 buckets per thread, 4 threads per bin
    uint32_t sum = 0;
    for (int k = 0; k < per; k++) sum += base[tid * per + k];
    part[tid] = sum;
  }
  __syncthreads();
  if (tid < kRlcCoarse) {
    constexpr int tpb = kRlcSortBlock / kRlcCoarse;
    uint32_t sum = off[tid * kRlcFinePerCoarse];
    for (int k = 0; k < tpb; k++) sum += part[tid * tpb + k];
    gbase[tid] = sum;
    cnt[tid] = 0;
  }
  __syncthreads();
  const int64_t total = (a.p1 - a.p0) + 2;
  const int64_t c0 = (int64_t)g * a.chunk;
  const int64_t c1 = c0 + a.chunk < total ? c0 + a.chunk : total;
  const int16_t* dig = a.digits + (int64_t)w * a.dstride;
  uint32_t* inter = a.inter + (int64_t)w * a.istride;
  constexpr int per_thread = kRlcTile / kRlcSortBlock;  // 8
  // A thread's 8 points of a tile are consecutive, so their digits are one 16-byte load where
  // the range is aligned (p0 is a multiple of 8 on every RLC path; the two extras at the end
  // go through msm_point one at a time; A/B against 8 strided 2-byte loads: sort 0.421 / 0.428
  // against 0.432 / 0.427 ms, within noise, kept for the 8x fewer load instructions).
  const int64_t np = a.p1 - a.p0;
  const bool vec = (a.p0 & 7) == 0;
  for (int64_t t0 = c0; t0 < c1; t0 += kRlcTile) {
    uint64_t ent[per_thread];
    uint32_t rank[per_thread];
    int dv[per_thread];
    const int64_t tb = t0 + (int64_t)per_thread * tid;
    if (vec && tb + per_thread <= c1 && tb + per_thread <= np) {
      const uint4 q = *reinterpret_cast<const uint4*>(dig + a.p0 + tb);
      const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < per_thread; k++) dv[k] = (int16_t)(wv[k >> 1] >> (16 * (k & 1)));
    } else {
#pragma unroll
      for (int k = 0; k < per_thread; k++) {
        const int64_t t = tb + k;
        dv[k] = t < c1 ? dig[msm_point(a, t)] : 0;
      }
    }
#pragma unroll
    for (int k = 0; k < per_thread; k++) {
      const int64_t t = tb + k;
      ent[k] = ~0ull;
      if (t < c1) {
        const int d = dv[k];
        if (d != 0) {
          const uint32_t b = (uint32_t)((d < 0 ? -d : d) - 1);
          const uint32_t c = b / kRlcFinePerCoarse;
          ent[k] = ((uint64_t)c << 40) | ((uint32_t)(b % kRlcFinePerCoarse) << 25) | (d < 0 ? (1u << 24) : 0u) |
                   (uint32_t)t;
          rank[k] = atomicAdd(&cnt[c], 1u);
        }
      }
    }
    __syncthreads();
    // exclusive scan of the 256 bin counts: a shuffle scan per wave, then the wave totals
    // (a one-thread loop here was ~8 us of LDS latency per tile)
    if (tid < kRlcCoarse) {
      const uint32_t v = cnt[tid];
      uint32_t x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if ((tid & 63) >= d) x += y;
      }
      start[tid] = x - v;
      if ((tid & 63) == 63) wtot[tid >> 6] = x;
    }
    __syncthreads();
    if (tid < kRlcCoarse) {
      uint32_t add = 0;
      for (int k = 0; k < (tid >> 6); k++) add += wtot[k];
      start[tid] += add;
      if (tid == kRlcCoarse - 1) part[0] = start[tid] + cnt[tid];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < per_thread; k++)
      if (ent[k] != ~0ull) buf[start[ent[k] >> 40] + rank[k]] = ent[k];
    __syncthreads();
    const uint32_t nt = part[0];
    for (uint32_t e = tid; e < nt; e += kRlcSortBlock) {
      const uint64_t v = buf[e];
      const uint32_t c = (uint32_t)(v >> 40);
      inter[gbase[c] + (e - start[c])] = (uint32_t)v;
    }
    __syncthreads();
    if (tid < kRlcCoarse) {
      gbase[tid] += cnt[tid];
      cnt[tid] = 0;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kRlcSortBlock) k_rlc_fine(RlcMsmArgs a) {
  __shared__ uint32_t img[kRlcFineCap];
  __shared__ uint32_t cur[kRlcFinePerCoarse];
  const int c = blockIdx.x, w = blockIdx.y;
  const int tid = threadIdx.x;
  const uint32_t* off = a.offsets + (int64_t)w * (kRlcBuckets + 1) + c * kRlcFinePerCoarse;
  const uint32_t r0 = off[0], r1 = off[kRlcFinePerCoarse];
  const bool staged = r1 - r0 <= (uint32_t)kRlcFineCap;
  if (tid < kRlcFinePerCoarse) cur[tid] = off[tid] - (staged ? r0 : 0u);
  __syncthreads();
  uint32_t* idx = a.idx + (int64_t)w * a.istride;
  constexpr int U = 4;  // loads in flight per thread
  const uint32_t* inter = a.inter + (int64_t)w * a.istride;
  for (uint32_t e0 = r0 + tid; e0 < r1; e0 += U * kRlcSortBlock) {
    uint32_t v[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
      const uint32_t e = e0 + k * kRlcSortBlock;
      v[k] = e < r1 ? inter[e] : ~0u;  // t < 2^24 - 1: an entry is never ~0
    }
#pragma unroll
    for (int k = 0; k < U; k++) {
      if (v[k] == ~0u) continue;
      const uint32_t pos = atomicAdd(&cur[v[k] >> 25], 1u);
      const uint32_t id = (uint32_t)msm_point(a, v[k] & 0xffffffu) | ((v[k] << 7) & 0x80000000u);
      if (staged) img[pos] = id; else idx[pos] = id;
    }
  }
  if (!staged) return;
  __syncthreads();
  for (uint32_t e = tid; e < r1 - r0; e += kRlcSortBlock) idx[r0 + e] = img[e];
}

// ---------------------------------------------------------------------------------------
// Bucket accumulation: B[w][b] = sum of (+/-) points in bucket b of window w, load-balanced.
// Window w's sorted entries [0, E_w) are cut into chunks of echunk; thread (w, t) adds
// exactly the points of chunk t (every lane of a wave does the same number of additions,
// whatever the bucket sizes -- the top window's 8x fuller buckets included).  A bucket that
// starts inside chunk t is owned by t, which writes its partial to B[w][b]; the partial of
// a bucket that started in an earlier chunk goes to heads[w][t], and k_rlc_bucket_fix adds
// the heads of the chunks a bucket spans (one or two for an average bucket).
// The running sum is kept as p1p1; its conversion to p3 (4 muls) is issued after the next
// point's gather, so the gather latency overlaps that work.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ ge_p1p1 p1p1_identity_rlc() {
  ge_p1p1 r;  // identity as p1p1: (0 : 1 : 1 : 1)
  r.X = fe_zero();
  r.Y = fe_one();
  r.Z = fe_one();
  r.T = fe_one();
  return r;
}

// The bucket holding sorted entry e, given that bucket b ended at e (off[b + 1] == e): the last
// b' > b with off[b'] <= e.  A gallop, then a binary search, so a sparse window costs O(log gap)
// dependent loads per bucket instead of one per empty bucket skipped -- a small batch spreads a
// few entries over 2^15 buckets, and walking them one by one made k_rlc_bucket 2.2 ms at n = 1
// (2^15 dependent offset loads on one lane) against 0.6 ms at n = 1000.  In a dense window the
// next bucket is non-empty and this is the one load the walk made.
__device__ __forceinline__ int next_bucket(const uint32_t* off, int b, uint32_t e) {
  int lo = b + 1, step = 1;
  while (lo + step < kRlcBuckets && off[lo + step] <= e) {
    lo += step;
    step <<= 1;
  }
  int hi = lo + step - 1 < kRlcBuckets - 1 ? lo + step - 1 : kRlcBuckets - 1;  // off[kRlcBuckets] > e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// (141 VGPRs, 3 waves/SIMD; forcing 4 waves -- 128 VGPRs with spills -- measured 7 % slower)
__global__ void __launch_bounds__(256) k_rlc_bucket(RlcMsmArgs a) {
  const int w = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  ClockStamp clk;
  clk.start();
  const uint32_t* off = a.offsets + (int64_t)w * (kRlcBuckets + 1);
  const uint32_t total = off[kRlcBuckets];
  const int64_t e0l = t * a.echunk;
  if (e0l >= (int64_t)total) return;
  const uint32_t e0 = (uint32_t)e0l;
  const uint32_t e1 = e0 + (uint32_t)a.echunk < total ? e0 + (uint32_t)a.echunk : total;
  const uint32_t* idx = a.idx + (int64_t)w * a.istride;
  ge_p3* bw = a.buckets + (int64_t)w * kRlcBuckets;
  ge_p3* heads = a.heads + (int64_t)w * a.hstride;
  // bucket of entry e0: the last b with off[b] <= e0
  int lo = 0, hi = kRlcBuckets - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e0) lo = mid; else hi = mid - 1;
  }
  int b = lo;
  uint32_t bend = off[b + 1];
  bool head = off[b] < e0;  // bucket b started in an earlier chunk
  ge_p1p1 r = p1p1_identity_rlc();
  uint32_t id = idx[e0];
  for (uint32_t e = e0; e < e1; e++) {
    const ge_niels p = load_niels(a.pts + (id & 0x7fffffffu));
    const bool neg = (id >> 31) != 0;
    id = e + 1 < e1 ? idx[e + 1] : 0u;
    ge_p3 acc = p1p1_to_p3(r);
    if (e == bend) {  // bucket b complete: emit it (a store, no extra field work), restart
      if (head) store_p3(heads + t, acc); else store_p3(bw + b, acc);
      head = false;
      acc = ge_identity();
      b = next_bucket(off, b, e);
      bend = off[b + 1];
    }
    r = ge_add_niels(acc, ge_niels_cneg(p, neg));
  }
  const ge_p3 v = p1p1_to_p3(r);
  if (head) store_p3(heads + t, v); else store_p3(bw + b, v);
  clk.stop(a.clock_probe, ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6));
}

// Buckets leave the fix-up in cached form (Y+X, Y-X, Z, 2dT, the same 160 bytes), so the
// reduction kernels add them with 2 quad rounds and no conversion of their own.
__device__ __forceinline__ void store_cached(ge_cached* dst, const ge_cached& v) {
  store_p3(reinterpret_cast<ge_p3*>(dst), *reinterpret_cast<const ge_p3*>(&v));
}

__device__ __forceinline__ ge_cached load_cached(const ge_cached* src) {
  const ge_p3 v = load_p3(reinterpret_cast<const ge_p3*>(src));
  return *reinterpret_cast<const ge_cached*>(&v);
}

// B[w][b] += heads of the chunks after the owner that bucket b spans, then B[w][b] is
// rewritten in cached form; empty buckets become the cached identity.
// 4 waves/SIMD (128 VGPRs, 16 B scratch): 0.124 / 0.122 ms against 0.130 / 0.129 at the
// compiler's 173 VGPRs (A/B, one call); prefetching the window kernel's segment sums one
// iteration ahead spilled and measured slower (reduce 0.39 against 0.34 ms).
#ifndef CPZ_RLC_FIX_WAVES
#define CPZ_RLC_FIX_WAVES 4
#endif
__global__ void __launch_bounds__(256, CPZ_RLC_FIX_WAVES) k_rlc_bucket_fix(RlcMsmArgs a) {
  __builtin_amdgcn_s_setprio(3);  // tails issue ahead of bucket waves sharing the SIMD (another batch in flight)
  const int64_t tl = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (tl >= (int64_t)kRlcWindows * kRlcBuckets) return;
  const int64_t t = tl;
  const int w = (int)(t / kRlcBuckets);
  const int b = (int)(t % kRlcBuckets);
  const uint32_t* off = a.offsets + (int64_t)w * (kRlcBuckets + 1);
  const uint32_t s = off[b], e = off[b + 1];
  ge_cached* dst = reinterpret_cast<ge_cached*>(a.buckets + t);
  if (s == e) {
    if (!a.sparse) store_cached(dst, ge_cached_identity());  // the sparse reduction reads non-empty buckets only
    return;
  }
  const uint32_t c0 = s / (uint32_t)a.echunk, c1 = (e - 1) / (uint32_t)a.echunk;
  const ge_p3* heads = a.heads + (int64_t)w * a.hstride;
  ge_p3 v = load_p3(a.buckets + t);
  for (uint32_t c = c0 + 1; c <= c1; c++) v = ge_add(v, load_p3(heads + c));
  store_cached(dst, p3_to_cached(v));
}

// One quad per (window, segment of kRlcSegLen buckets), buckets in cached form:
//   S = sum_{b in seg} B_b,   W = sum_{b in seg} (b - lo + 1) B_b   (lo = first bucket value)
// written in cached form for k_rlc_window.
// (2 waves/SIMD: the 2048 waves of a launch are resident at once)
__global__ void __launch_bounds__(256, 2) k_rlc_segment(RlcMsmArgs a) {
  __builtin_amdgcn_s_setprio(3);
  const int64_t tl = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 2;
  const int q = threadIdx.x & 3;
  constexpr int nseg = kRlcBuckets / kRlcSegLen;
  if (tl >= (int64_t)kRlcWindows * nseg) return;  // whole quads
  const int64_t t = tl;
  const int w = (int)(t / nseg);
  const int sg = (int)(t % nseg);
  const ge_cached* B =
      reinterpret_cast<const ge_cached*>(a.buckets + (int64_t)w * kRlcBuckets + (int64_t)sg * kRlcSegLen);
  ge_p3 run = ge_identity(), acc = ge_identity();
  ge_cached nb = load_cached(B + kRlcSegLen - 1);
#pragma unroll 1
  for (int k = kRlcSegLen - 1; k >= 0; k--) {
    const ge_cached cb = nb;
    if (k > 0) nb = load_cached(B + k - 1);
    run = ge_add_quad(run, cb, q);
    acc = ge_add_quad(acc, run, q);
  }
  if (q == 0) {
    store_cached(reinterpret_cast<ge_cached*>(a.seg_s) + t, p3_to_cached(run));
    store_cached(reinterpret_cast<ge_cached*>(a.seg_w) + t, p3_to_cached(acc));
  }
}

// One block of 512 threads (128 quads) per window.  Segment t covers bucket values L t + 1
// .. L t + L (L = kRlcSegLen):  T_w = sum_t W_t + L * sum_t t S_t.  Quad u owns the
// P = nseg / 128 segments P u .. P u + P - 1:  A_u = sum_j S_{Pu+j},  M_u = sum_j j S_{Pu+j},
//   sum_t t S_t = P sum_u u A_u + sum_u M_u,   sum_u u A_u = sum_{k>=1} suffix_k(A).
#ifndef CPZ_RLC_WIN_QUADS
#define CPZ_RLC_WIN_QUADS 128
#endif
constexpr int kRlcWinQuads = CPZ_RLC_WIN_QUADS;  // 512 threads: 256 VGPRs without spills (1024 spill)
__global__ void __launch_bounds__(4 * kRlcWinQuads) k_rlc_window(RlcMsmArgs a) {
  __shared__ ge_p3 lds[kRlcWinQuads], lds_m[kRlcWinQuads], lds_w[kRlcWinQuads];
  __builtin_amdgcn_s_setprio(3);
  const int w = blockIdx.x;
  const int u = threadIdx.x >> 2, q = threadIdx.x & 3;
  constexpr int nseg = kRlcBuckets / kRlcSegLen;
  constexpr int P = nseg / kRlcWinQuads;
  static_assert(P * kRlcWinQuads == nseg && (P & (P - 1)) == 0 && (kRlcSegLen & (kRlcSegLen - 1)) == 0,
                "window kernel assumes power-of-two segment counts");
  const ge_cached* S = reinterpret_cast<const ge_cached*>(a.seg_s) + (int64_t)w * nseg + P * u;
  const ge_cached* Wt = reinterpret_cast<const ge_cached*>(a.seg_w) + (int64_t)w * nseg + P * u;
  ge_p3 run = ge_identity(), M = ge_identity(), Wsum = ge_identity();
#pragma unroll 1
  for (int j = P - 1; j >= 1; j--) {  // M = sum_j j S_j = sum_{j>=1} suffix_j
    run = ge_add_quad(run, load_cached(S + j), q);
    M = ge_add_quad(M, run, q);
    Wsum = ge_add_quad(Wsum, load_cached(Wt + j), q);
  }
  const ge_p3 A = ge_add_quad(run, load_cached(S), q);
  Wsum = ge_add_quad(Wsum, load_cached(Wt), q);
  // suffix scan of A over u (inclusive): suf_u = sum_{v >= u} A_v
  if (q == 0) lds[u] = A;
  __syncthreads();
  ge_p3 suf = A;
#pragma unroll 1
  for (int off = 1; off < kRlcWinQuads; off <<= 1) {
    const ge_p3 other = u + off < kRlcWinQuads ? lds[u + off] : ge_identity();
    __syncthreads();
    suf = ge_add_quad(suf, other, q);
    if (q == 0) lds[u] = suf;
    __syncthreads();
  }
  // total = sum W + L * (P * sum_{u>=1} suf_u + sum M): the three sums side by side
  if (q == 0) {
    lds[u] = u >= 1 ? suf : ge_identity();
    lds_m[u] = M;
    lds_w[u] = Wsum;
  }
  __syncthreads();
#pragma unroll 1
  for (int off = kRlcWinQuads / 2; off > 0; off >>= 1) {
    ge_p3 x, m, ws;
    if (u < off) {
      x = ge_add_quad(lds[u], lds[u + off], q);
      m = ge_add_quad(lds_m[u], lds_m[u + off], q);
      ws = ge_add_quad(lds_w[u], lds_w[u + off], q);
    }
    __syncthreads();
    if (u < off && q == 0) {
      lds[u] = x;
      lds_m[u] = m;
      lds_w[u] = ws;
    }
    __syncthreads();
  }
  if (u == 0) {
    constexpr int lgP = __builtin_ctz(P), lgL = __builtin_ctz(kRlcSegLen);
    ge_p3 r = p3_dbl_n_quad(lds[0], lgP, q);                   // * P
    r = p3_dbl_n_quad(ge_add_quad(r, lds_m[0], q), lgL, q);    // * L
    r = ge_add_quad(r, lds_w[0], q);
    if (q == 0) store_p3(a.win + w, r);
  }
}

// Small MSMs (at most kRlcSparsePts points, BatchVerifier-sized batches): a window holds at
// most that many non-empty buckets, so T_w = sum_b b B_b is formed from them alone -- one
// double-and-add [b] B_b per non-empty bucket on a quad -- instead of the running sums over
// all 2^15 buckets (k_rlc_segment + k_rlc_window: 0.095 + 0.130 ms at n = 10, whatever the
// size).  A synchronous batch check of n = 1 .. 100 proofs: 0.63-0.68 ms against 0.77-0.81 ms;
// at n = 1000 (4002 points) it measured 0.84 against 0.82-0.83 ms, hence the 2048-point limit
// (profiles/r04_small_batch_sparse_ab.json).  G = RlcMsmArgs::sgroups workgroups per window (4 .. 32, ~2 buckets per quad) each
// take every G-th non-empty bucket (each workgroup lists the window's non-empty buckets itself
// from the offsets), reduce their quads' sums in LDS and write a partial; k_rlc_final adds a
// window's partials as it loads the window sums (a separate summing launch cost ~20 us).
constexpr int kRlcSparseMaxGroups = 32;
__global__ void __launch_bounds__(256) k_rlc_window_sparse(RlcMsmArgs a) {
  __shared__ uint32_t cnt[256];
  __shared__ uint16_t list[kRlcSparsePts + 2];
  __shared__ ge_p3 red[64];
  __builtin_amdgcn_s_setprio(3);
  const int w = blockIdx.y, g = blockIdx.x, t = threadIdx.x;
  const uint32_t* off = a.offsets + (int64_t)w * (kRlcBuckets + 1);
  constexpr int per = kRlcBuckets / 256;  // thread t scans buckets t, t + 256, ... (coalesced)
  uint32_t mine = 0;
  for (int k = 0; k < per; k++) mine += off[k * 256 + t + 1] > off[k * 256 + t] ? 1u : 0u;
  cnt[t] = mine;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive scan of the per-thread counts
    const uint32_t v = t >= d ? cnt[t - d] : 0u;
    __syncthreads();
    cnt[t] += v;
    __syncthreads();
  }
  const uint32_t K = cnt[255];  // non-empty buckets of the window (<= its entries <= the MSM's points)
  uint32_t pos = cnt[t] - mine;
  for (int k = 0; k < per && pos < (uint32_t)(kRlcSparsePts + 2); k++) {
    const int b = k * 256 + t;
    if (off[b + 1] > off[b]) list[pos++] = (uint16_t)b;
  }
  __syncthreads();
  const int u = t >> 2, q = t & 3;
  const ge_cached* B = reinterpret_cast<const ge_cached*>(a.buckets + (int64_t)w * kRlcBuckets);
  ge_p3 acc = ge_identity();
#pragma unroll 1
  for (uint32_t i = (uint32_t)(g * 64 + u); i < K; i += 64 * (uint32_t)a.sgroups) {  // uniform per quad
    const int b = list[i];
    const uint32_t v = (uint32_t)b + 1;  // bucket index b holds the digit magnitude b + 1
    const ge_cached Bc = load_cached(B + b);
    const ge_cached Z = ge_cached_identity();
    ge_p3 R = ge_identity();
#pragma unroll 1
    for (int bit = 15; bit >= 0; bit--) {  // branch-free: every quad of the wave adds
      R = p3_dbl_n_quad(R, 1, q);
      const bool on = (v >> bit) & 1u;
      ge_cached c;
      c.YpX = fe_select(Z.YpX, Bc.YpX, on);
      c.YmX = fe_select(Z.YmX, Bc.YmX, on);
      c.Z = fe_select(Z.Z, Bc.Z, on);
      c.T2d = fe_select(Z.T2d, Bc.T2d, on);
      R = ge_add_quad(R, c, q);
    }
    acc = ge_add_quad(acc, R, q);
  }
  if (q == 0) red[u] = acc;
  __syncthreads();
#pragma unroll 1
  for (int o = 32; o > 0; o >>= 1) {
    ge_p3 x;
    if (u < o) x = ge_add_quad(red[u], red[u + o], q);
    __syncthreads();
    if (u < o && q == 0) red[u] = x;
    __syncthreads();
  }
  if (t == 0) store_p3(a.seg_s + (int64_t)w * kRlcSparseMaxGroups + g, red[0]);
}

// Window sums T_j of the MSM into lds[j] (quad j's lane 0): from k_rlc_window_sparse's
// partials or k_rlc_window's sums.
__device__ __forceinline__ void rlc_final_windows(const RlcMsmArgs& a, ge_p3* lds, int j, int q) {
  if (a.sparse) {  // window j's sum from its k_rlc_window_sparse partials
    const ge_p3* part = a.seg_s + (int64_t)j * kRlcSparseMaxGroups;
    ge_p3 T = load_p3(part);
#pragma unroll 1
    for (int g = 1; g < a.sgroups; g++) T = ge_add_quad(T, load_p3(part + g), q);
    if (q == 0) lds[j] = T;
  } else if (q == 0) {
    lds[j] = load_p3(a.win + j);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Lanes 0..3 (one quad, each holding P): the span's identity flag, the multi-span running
// total, and the 32-byte partial with its identity flag.
__device__ __forceinline__ void rlc_final_tail(const RlcMsmArgs& a, ge_p3 P, int q) {
  if (a.span_identity && q == 0) a.span_identity[0] = ristretto_is_identity(P) ? 1 : 0;
  if (a.total) {  // one span of a multi-span batch
    if (!a.total_first) P = ge_add_quad(load_p3(a.total), P, q);
    if (!a.total_last) {
      if (q == 0) store_p3(a.total, P);
      return;
    }
  }
  if (q == 0) {
    // The identity (every valid batch) encodes to 32 zero bytes: only a failing batch pays
    // for the encoding's inverse square root, one lane's ~30 K instructions (~0.1 ms).
    const bool id = ristretto_is_identity(P);
    uint32_t enc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!id) ristretto_encode(enc, P);
    for (int k = 0; k < 8; k++) a.partial_out[k] = enc[k];
    a.identity_out[0] = id ? 1 : 0;
  }
}

// P = sum_w 2^(16 w) T_w by a tree on one wave: quad j owns window j; at level `span` the
// active quads double their upper partner 16 span times and add it to their own (240
// doublings deep), then the partial is encoded with its identity flag -- or, for one span of
// a multi-span batch, added into the batch's running total (RlcMsmArgs::total).
// CPZ_RLC_FINAL16=0 selects it; k_rlc_final16 below is the default.
__global__ void __launch_bounds__(64) k_rlc_final(RlcMsmArgs a) {
  __shared__ ge_p3 lds[kRlcWindows];
  __builtin_amdgcn_s_setprio(3);
  const int j = threadIdx.x >> 2, q = threadIdx.x & 3;
  rlc_final_windows(a, lds, j, q);
  for (int span = 1; span < kRlcWindows; span <<= 1) {  // one wave: LDS traffic stays in program order
    if ((j % (2 * span)) == 0) {
      const ge_p3 lo = ge_add_quad(lds[j], p3_dbl_n_quad(lds[j + span], 16 * span, q), q);
      if (q == 0) lds[j] = lo;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (threadIdx.x >= 4) return;
  rlc_final_tail(a, lds[0], q);
}

// The same combine as a Horner chain on the latency layout of fe16.h: the whole wave holds
// one point (a field element per 16-lane row, one 16-bit limb per lane), so each of the 240
// doublings is two row-parallel product stages instead of a quad's two one-lane products.
// The window sums arrive as canonical words (one fe_towords per lane: 16 windows x X, Y, Z,
// T), P = (..(T_15 2^16 + T_14) 2^16 + ..) + T_0, and the result goes back to radix 2^25.5
// for the shared tail.  The k_rlc_final tree is as deep (16 + 32 + 64 + 128 doublings).
__global__ void __launch_bounds__(64) k_rlc_final16(RlcMsmArgs a) {
  __shared__ ge_p3 lds[kRlcWindows];
  __shared__ uint32_t wd[kRlcWindows * 4 * 8];
  __builtin_amdgcn_s_setprio(3);
  const int lane = threadIdx.x, j = lane >> 2, q = lane & 3;
  rlc_final_windows(a, lds, j, q);
  fe_towords(wd + (j * 4 + q) * 8, reinterpret_cast<const fe*>(&lds[j])[q]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const r16::Lane L = r16::lane_of(lane);
  auto window = [&](int w) {
    r16::P4 p;
    p.X = r16::limb_of(wd + (w * 4 + 0) * 8, L);
    p.Y = r16::limb_of(wd + (w * 4 + 1) * 8, L);
    p.Z = r16::limb_of(wd + (w * 4 + 2) * 8, L);
    p.T = r16::limb_of(wd + (w * 4 + 3) * 8, L);
    return p;
  };
  r16::P4 P = window(kRlcWindows - 1);
#pragma unroll 1
  for (int w = kRlcWindows - 2; w >= 0; w--) {
#pragma unroll 1
    for (int i = 0; i < 16; i++) P = r16::dbl(P, L);
    const r16::C4 c = r16::to_cached(window(w), L);
    P = r16::add_b(P, r16::cached_b(c, false, L), L);
  }
  uint32_t out[8];
  r16::to_words(out, r16::sel4(P.X, P.Y, P.Z, P.T, L));  // row r: coordinate r
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (L.k == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) wd[L.row * 8 + k] = out[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane >= 4) return;
  // canonical words -> limbs in [0, 2^26), then one carry pass to the tight bounds the
  // tail's sums (Y - X, Y + X) assume
  auto tight = [](const uint32_t* w) {
    const fe f = fe_fromwords(w);
    int64_t h[10];
#pragma unroll
    for (int k = 0; k < 10; k++) h[k] = f.v[k];
    return fe_carry_wide(h);
  };
  ge_p3 R;
  R.X = tight(wd + 0);
  R.Y = tight(wd + 8);
  R.Z = tight(wd + 16);
  R.T = tight(wd + 24);
  rlc_final_tail(a, R, q);
}

// Generic MSM input: decode point j, store its Niels form and the digits of scalar j.
__global__ void __launch_bounds__(256) k_msm_load(int64_t n, const uint32_t* __restrict__ pts_enc,
                                                  const uint32_t* __restrict__ scalars, ge_niels* __restrict__ pts,
                                                  int16_t* __restrict__ digits, int64_t dstride, int* __restrict__ bad) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  uint32_t w[8];
  rlc_load8(w, pts_enc, j);
  ge_p3 P;
  const bool ok = ristretto_decode(P, w);
  if (!ok) atomicOr(bad, 1);
  store_niels(pts + j, niels_from_p3_affine(P, false));
  rlc_load8(w, scalars, j);
  int16_t d[kRlcWindows];
  recode16(d, w);
#pragma unroll
  for (int wv = 0; wv < kRlcWindows; wv++) digits[(int64_t)wv * dstride + j] = d[wv];
}

// Sum of k encoded partials (multi-GPU / fallback combine).  Lane l decodes partials l, l + 64,
// ... and sums them; a tree over the lanes that hold any adds the sums; lane 0 encodes the
// total unless it is the identity (every valid batch), whose encoding is 32 zero bytes.  One
// lane decoding the k partials in turn and always encoding took ~55 us per decode or encode.
__global__ void __launch_bounds__(64) k_rlc_combine(const uint32_t* __restrict__ parts, int k,
                                                    uint32_t* __restrict__ out, int* __restrict__ flags) {
  __shared__ ge_p3 lds[64];
  const int l = threadIdx.x;
  ge_p3 acc = ge_identity();
  bool ok = true;
#pragma unroll 1
  for (int j = l; j < k; j += 64) {
    ge_p3 P;
    ok = ristretto_decode(P, parts + 8 * (int64_t)j) && ok;
    acc = ge_add(acc, P);
  }
  const unsigned long long bad = __ballot(!ok);
  lds[l] = acc;
  __syncthreads();
  int m = 1;
  while (m < k && m < 64) m <<= 1;
#pragma unroll 1
  for (int off = m >> 1; off > 0; off >>= 1) {
    ge_p3 x;
    if (l < off) x = ge_add(lds[l], lds[l + off]);
    __syncthreads();
    if (l < off) lds[l] = x;
    __syncthreads();
  }
  if (l != 0) return;
  const ge_p3 S = lds[0];
  const bool id = ristretto_is_identity(S);
  uint32_t enc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!id) ristretto_encode(enc, S);
  for (int q = 0; q < 8; q++) out[q] = enc[q];
  flags[0] = bad == 0 ? 1 : 0;
  flags[1] = id ? 1 : 0;
}

// ---------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------
hipError_t launch_rlc_prepare(const RlcPrepArgs& a, hipStream_t st) {
  const int64_t blocks = (a.n + kRlcPrepBlock - 1) / kRlcPrepBlock;
  if (a.n <= kRlcPrepWideMax && a.quarter_sums) {
    const int64_t nq = (a.n + 63) / 64;
    hipLaunchKernelGGL(k_rlc_prepare4, dim3((unsigned)nq), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rlc_bsum4, dim3((unsigned)((4 * blocks + 63) / 64)), dim3(64), 0, st, a.quarter_sums, nq,
                       a.block_sums, 2 * blocks);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_rlc_prepare, dim3((unsigned)blocks), dim3(kRlcPrepBlock), 0, st, a);
  return hipGetLastError();
}

void rlc_sort_geometry(RlcMsmArgs& a, int64_t npts) {
  int64_t g = (npts + kRlcSortChunk - 1) / kRlcSortChunk;
  if (g > kRlcSortGroups) g = kRlcSortGroups;
  if (g < 1) g = 1;
  a.groups = (int)g;
  a.chunk = ((npts + g - 1) / g + 63) & ~(int64_t)63;  // whole 16-byte digit loads (k_rlc_hist)
  // Entries per k_rlc_bucket thread: kRlcChunk for a large MSM (load-balanced, enough threads
  // anyway); a small one (a BatchVerifier batch, a bisection leaf) is cut finer so that at
  // least ~2048 threads share each window, since a thread's additions are one dependent chain
  // -- 64 of them on one lane took 0.34-0.40 ms at n = 20 .. 1000 proofs.  A window holds at
  // most npts entries, so ceil(npts / echunk) <= max(npts / kRlcChunk, kRlcMinHeads) heads.
  int e = kRlcMinChunk;
  while (e < kRlcChunk && (int64_t)e * kRlcMinHeads < npts) e <<= 1;
  a.echunk = e;
}

hipError_t launch_rlc_msm(const RlcMsmArgs& a, const sc* block_sums, int64_t b0, int64_t b1, const ge_niels* tab,
                          hipStream_t st, hipEvent_t* marks, hipEvent_t final_wait, hipEvent_t final_done) {
  hipError_t e;
  auto mark = [&](int k) -> hipError_t { return marks ? hipEventRecord(marks[k], st) : hipSuccess; };
  if ((e = mark(0)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_rlc_extra, dim3(1), dim3(256), 0, st, a, block_sums, b0, b1, tab);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const size_t lds = sizeof(uint32_t) * kRlcBuckets;  // 128 KB of the 160 KB LDS
  // The attribute is per device: one bit per ordinal (contexts on several GPUs launch from
  // their own threads, cpz_verify_batch_multi; setting it twice is harmless).
  static std::atomic<uint64_t> attr_set{0};
  int dev = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? (uint64_t)1 << dev : 0;
  if (!bit || !(attr_set.load(std::memory_order_acquire) & bit)) {
    if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rlc_hist),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess)
      return e;
    attr_set.fetch_or(bit, std::memory_order_release);
  }
  const int64_t nb = (int64_t)kRlcWindows * kRlcBuckets;
  hipLaunchKernelGGL(k_rlc_hist, dim3(a.groups, kRlcWindows), dim3(kRlcSortBlock), lds, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_rlc_bscan, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_rlc_scan, dim3(kRlcWindows), dim3(1024), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_rlc_coarse, dim3(a.groups, kRlcWindows), dim3(kRlcSortBlock), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_rlc_fine, dim3(kRlcCoarse, kRlcWindows), dim3(kRlcSortBlock), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(1)) != hipSuccess) return e;
  const int64_t chunks = ((a.p1 - a.p0) + 2 + a.echunk - 1) / a.echunk;  // per window: entries <= points
  hipLaunchKernelGGL(k_rlc_bucket, dim3((unsigned)((chunks + 255) / 256), kRlcWindows), dim3(256), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(2)) != hipSuccess) return e;
  RlcMsmArgs a2 = a;
  a2.sparse = CPZ_RLC_SPARSE && (a.p1 - a.p0) + 2 <= kRlcSparsePts ? 1 : 0;
  a2.sgroups = (int)std::min<int64_t>(kRlcSparseMaxGroups, std::max<int64_t>(4, ((a.p1 - a.p0) + 2 + 127) / 128));
  hipLaunchKernelGGL(k_rlc_bucket_fix, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, a2);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(3)) != hipSuccess) return e;
  if (a2.sparse) {
    hipLaunchKernelGGL(k_rlc_window_sparse, dim3((unsigned)a2.sgroups, kRlcWindows), dim3(256), 0, st, a2);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  } else {
    const int64_t ns = (int64_t)kRlcWindows * (kRlcBuckets / kRlcSegLen);
    hipLaunchKernelGGL(k_rlc_segment, dim3((unsigned)((4 * ns + 255) / 256)), dim3(256), 0, st, a2);  // a quad each
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_rlc_window, dim3(kRlcWindows), dim3(4 * kRlcWinQuads), 0, st, a2);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if ((e = mark(4)) != hipSuccess) return e;
  if (final_wait && (e = hipStreamWaitEvent(st, final_wait, 0)) != hipSuccess) return e;
  static const bool final16 = [] {
    const char* v = getenv("CPZ_RLC_FINAL16");
    return !(v && v[0] == '0');
  }();
  if (final16)
    hipLaunchKernelGGL(k_rlc_final16, dim3(1), dim3(64), 0, st, a2);
  else
    hipLaunchKernelGGL(k_rlc_final, dim3(1), dim3(64), 0, st, a2);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (final_done && (e = hipEventRecord(final_done, st)) != hipSuccess) return e;
  return mark(5);
}

hipError_t launch_msm_load(int64_t n, const uint32_t* pts_enc, const uint32_t* scalars, ge_niels* pts,
                           int16_t* digits, int64_t dstride, int* bad, hipStream_t st) {
  hipLaunchKernelGGL(k_msm_load, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, pts_enc, scalars, pts, digits,
                     dstride, bad);
  return hipGetLastError();
}

hipError_t launch_rlc_combine(const uint32_t* parts, int k, uint32_t* out, int* flags, hipStream_t st) {
  hipLaunchKernelGGL(k_rlc_combine, dim3(1), dim3(64), 0, st, parts, k, out, flags);
  return hipGetLastError();
}

}  // namespace cpz
