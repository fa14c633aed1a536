// Partitioned batch check on gfx950: the random-linear-combination partial of every block of
// kPartProofs (128) proofs, so that a failing batch goes to per-proof verification only where a
// block fails, and within a failing block holding one forgery only to that entry -- the
// fallback of verify_batch (batch.rs:262-268) / verify_individually (batch.rs:314-318) at
// forgery densities where bisection cannot prune (configs[4]: 0.1 % forged leaves ~88 % of
// 128-proof blocks clean, but every range of a few thousand proofs dirty).
//
// Block b's partial is the corrected batch equation over its own proofs (rlc.hip header):
//   P_b = sum_{i in b} [a_i s_i] g - [a_i] r1_i - [a_i c_i] y1_i + [b_i s_i] h - [b_i] r2_i - [b_i c_i] y2_i
// with the same 128-bit weights, so sum_b P_b is the batch's partial, and P_b is the identity
// iff every proof of b satisfies both equations (except with probability 2^-128 per forged
// proof).  It is one Pippenger MSM per block over kPartPoints points (the block's 4 x kPartProofs
// prepared points and g, h with the block's weight sums): signed radix-2^8 digits (each
// radix-2^16 digit d of the prepare split as d = lo + 2^8 hi, lo in [-128, 128), hi in
// [-128, 128]), 32 windows of 128 buckets.
//   k_part_sort     1 workgroup / block: LDS counting sort of the block's entries by (window,
//                   bucket) -> a list of 16-bit point ids and per-window bucket offsets.
//   k_part_acc      1 wave / block; a lane walks two units -- (window v, share h): buckets
//                   Wh+1 .. Wh+W, W = 32, or 4 in the top window, whose digits are <= 16 (see
//                   part_width) -- one of windows 0..15 and one of 16..31, paired by size in
//                   k_part_sort, each from its lowest bucket up with the running-sum
//                   reduction: run += entry point, and at each bucket boundary acc += run, so
//                   run = sum_d B_d and acc = sum_d (Wh + W + 1 - d) B_d without storing a
//                   bucket.  Both kinds of step are the same extended + cached addition on
//                   selected operands, so lanes at different buckets never diverge.
//   k_part_combine  1 quad / block (16 blocks per wave): T_v = sum_d d B_d from the four lanes'
//                   (acc, run), P_b = sum_v 2^(8 v) T_v by Horner, quad-cooperative; P_b and its
//                   flags.
//   k_part_sum1/2   sum_b P_b -> the batch partial (encoded only when it is not the identity).
// The locate pass over the failing blocks (rlc.h): k_part_index_digits (the same scalars times
// j_t = kPartLocJ0 - 2 t), the same sort / walk (on the prepared points, through PartArgs::pmap)
// / combine -> P'_b, and k_part_locate (the one t with P'_b = [j_t] P_b, if there is one).
#include <hip/hip_runtime.h>

#include "rlc.h"
#include "rlc_dev.h"
#include "verify.h"

namespace cpz {

// d = lo + 2^8 hi with lo in [-128, 128) and hi in [-128, 128] for d in [-2^15, 2^15).
__device__ __forceinline__ void split8(int d, int& lo, int& hi) {
  lo = ((d + 128) & 255) - 128;
  hi = (d - lo) >> 8;
}

// Buckets per lane of window v's walk: 32 (a quarter of the 128), except in the top window.
// Its 8-bit digits are the high halves of radix-2^16 digit 15 of scalars < l < 2^252 + 2^125
// (a c, b c and the block sums are reduced mod l; the weights have no digit 15): digit 15 is
// s >> 240 <= 4096 plus the carry out of digit 14, so it lies in [0, 4097] and its high half
// in [0, 16] -- all in the first quarter.  A fixed 32-bucket split left one lane walking the
// whole window (512 entries) while the other 63 walked ~160 and doubled the kernel's time; 8
// per lane still left two lanes with ~250 (C5 134 ms for the partials); 4 per lane spreads
// the window over all four.
__device__ __forceinline__ int part_width(int v) { return v == kPartWindows - 1 ? kPartTopBuckets / kPartQuarters : 32; }

__device__ __forceinline__ int digit16(const uint2& g, int q) {
  const uint32_t w = q < 2 ? g.x : g.y;
  return (int)(int16_t)(uint16_t)(w >> (16 * (q & 1)));
}

// ---------------------------------------------------------------------------------------
// k_part_sort: thread t holds proof t's four points (prepared order -r1, -y1, -r2, -y2),
// threads 0 / 1 also g / h with the block's weight sums (ids 4 kPartProofs, + 1).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kPartProofs) k_part_sort(PartArgs a) {
  constexpr int kT = kPartProofs;  // threads: one per proof of the block
  __shared__ uint32_t cur[kPartWindows][kPartBuckets];
  __shared__ uint32_t wtot[kPartWindows];
  __shared__ uint32_t wbase[kPartWindows + 1];
  __shared__ uint32_t top_over;
  const int64_t b = blockIdx.x, gb = a.blk0 + b;
  const int t = threadIdx.x;
  for (int i = t; i < kPartWindows * kPartBuckets; i += kT) (&cur[0][0])[i] = 0;
  if (t == 0) top_over = 0;
  const int64_t pi = kPartProofs * gb + t;
  const int64_t j0 = 4 * pi;
  const bool in = pi < a.n;  // past the batch's end (last block): no entries
  int16_t ex[kRlcWindows];
  if (t < 2) {  // the block's sum of a s (t = 0) / b s (t = 1): its one or two block sums
    constexpr int R = kPartProofs / kRlcSumBlock;
    sc s = a.block_sums[2 * (R * gb) + t];
#pragma unroll
    for (int r = 1; r < R; r++) s = sc_add(s, a.block_sums[2 * (R * gb + r) + t]);
    recode16(ex, s.w);
  }
  __syncthreads();
#pragma unroll 4
  for (int w = 0; w < kRlcWindows; w++) {
    const uint2 g = in ? *reinterpret_cast<const uint2*>(a.digits + w * a.dstride + j0) : make_uint2(0u, 0u);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      int lo, hi;
      split8(digit16(g, q), lo, hi);
      if (lo) atomicAdd(&cur[2 * w][(lo < 0 ? -lo : lo) - 1], 1u);
      if (hi) atomicAdd(&cur[2 * w + 1][(hi < 0 ? -hi : hi) - 1], 1u);
    }
    if (t < 2) {
      int lo, hi;
      split8(ex[w], lo, hi);
      if (lo) atomicAdd(&cur[2 * w][(lo < 0 ? -lo : lo) - 1], 1u);
      if (hi) atomicAdd(&cur[2 * w + 1][(hi < 0 ? -hi : hi) - 1], 1u);
    }
  }
  __syncthreads();
  // The top window's walk covers buckets 1 .. kPartTopBuckets only (k_part_acc).  Its digits
  // never exceed that (kPartTopBuckets); should one ever do, the block is marked failing
  // here, so that it is verified per proof instead of being judged on a partial that would
  // miss the entry (k_part_combine ORs its identity test into this flag).
  if (t >= kPartTopBuckets && t < kPartBuckets && cur[kPartWindows - 1][t] != 0) top_over = 1;
  __syncthreads();
  if (t == 0) a.fail[gb] = top_over ? 2 : 0;
  // exclusive scan of each window's 128 counts: wave wv takes windows wv, wv + kT / 64, ...;
  // lane l buckets 2l and 2l + 1
  {
    const int lane = t & 63, wv = t >> 6;
    for (int v = wv; v < kPartWindows; v += kT / 64) {
      const uint32_t c0 = cur[v][2 * lane], c1 = cur[v][2 * lane + 1], s = c0 + c1;
      uint32_t x = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      cur[v][2 * lane] = x - s;
      cur[v][2 * lane + 1] = x - s + c0;
      if (lane == 63) wtot[v] = x;
    }
  }
  __syncthreads();
  if (t == 0) {
    uint32_t r = 0;
    for (int v = 0; v < kPartWindows; v++) {
      wbase[v] = r;
      r += wtot[v];
    }
    wbase[kPartWindows] = r;
  }
  __syncthreads();
  uint16_t* offs = a.offs + b * kPartOffs;
  for (int i = t; i < kPartOffs; i += kT) {
    const int v = i / (kPartBuckets + 1), k = i % (kPartBuckets + 1);
    offs[i] = (uint16_t)(k < kPartBuckets ? wbase[v] + cur[v][k] : wbase[v + 1]);
  }
  // Walk units: (window v, lane share h), 128 per block, 64 in windows 0..15 (the r- and
  // y-points' low digits: ~288 steps each) and 64 in windows 16..31 (y only: ~160).  Lane r of
  // k_part_acc walks the r-th largest low unit and then the r-th smallest high unit, so every
  // lane's total is close to the mean (~445 steps): pairing a fixed p with p + 16 made the
  // wave wait for its largest binomial sum (~485 in a simulation of the digit distribution).
  {
    __shared__ uint32_t usz[2 * kPartUnits];
    __shared__ uint8_t asg[2][kPartUnits];
    if (t < 2 * kPartUnits) {
      const int v = t >> 2, h = t & 3, w = part_width(v);
      const uint32_t e0 = cur[v][w * h];
      const uint32_t e1 = w * (h + 1) < kPartBuckets ? cur[v][w * (h + 1)] : wtot[v];
      usz[t] = e1 - e0 + w;
    }
    __syncthreads();
    if (t < 2 * kPartUnits) {
      const bool low = t < kPartUnits;
      const int base = low ? 0 : kPartUnits;
      const uint32_t me = usz[t];
      int rank = 0;
      for (int u = base; u < base + kPartUnits; u++) {  // low: descending, high: ascending
        const uint32_t o = usz[u];
        rank += low ? (o > me || (o == me && u < t)) : (o < me || (o == me && u < t));
      }
      asg[low ? 0 : 1][rank] = (uint8_t)t;
    }
    __syncthreads();
    if (t < kPartUnits) a.assign[b * kPartUnits + t] = (uint16_t)(asg[0][t] | (asg[1][t] << 8));
  }
  __syncthreads();
  for (int i = t; i < kPartWindows * kPartBuckets; i += kT) (&cur[0][0])[i] += wbase[i / kPartBuckets];
  __syncthreads();
  uint16_t* list = a.lists + b * kPartListCap;
#pragma unroll 1
  for (int w = 0; w < kRlcWindows; w++) {
    const uint2 g = in ? *reinterpret_cast<const uint2*>(a.digits + w * a.dstride + j0) : make_uint2(0u, 0u);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      int lo, hi;
      split8(digit16(g, q), lo, hi);
      const uint16_t id = (uint16_t)(4 * t + q);
      if (lo) list[atomicAdd(&cur[2 * w][(lo < 0 ? -lo : lo) - 1], 1u)] = id | (lo < 0 ? 0x8000 : 0);
      if (hi) list[atomicAdd(&cur[2 * w + 1][(hi < 0 ? -hi : hi) - 1], 1u)] = id | (hi < 0 ? 0x8000 : 0);
    }
    if (t < 2) {
      int lo, hi;
      split8(ex[w], lo, hi);
      const uint16_t id = (uint16_t)(4 * kPartProofs + t);
      if (lo) list[atomicAdd(&cur[2 * w][(lo < 0 ? -lo : lo) - 1], 1u)] = id | (lo < 0 ? 0x8000 : 0);
      if (hi) list[atomicAdd(&cur[2 * w + 1][(hi < 0 ? -hi : hi) - 1], 1u)] = id | (hi < 0 ? 0x8000 : 0);
    }
  }
}

// ---------------------------------------------------------------------------------------
// k_part_acc
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ ge_p3 p3_select(const ge_p3& x, const ge_p3& y, bool c) {  // c ? y : x
  ge_p3 r;
  r.X = fe_select(x.X, y.X, c);
  r.Y = fe_select(x.Y, y.Y, c);
  r.Z = fe_select(x.Z, y.Z, c);
  r.T = fe_select(x.T, y.T, c);
  return r;
}

// One step of the running-sum walk is one addition: entry (run += q, q an affine Niels point)
// or bucket boundary (acc += run).  run is always the extended operand; the cached operand is
// read from the lane's stage slot (q, Z = 1) or its acc slot, a per-lane LDS index, and a
// boundary writes acc back (cached form) under its lane mask: 9 M either way (4 + p1p1 -> p3 +
// acc's 2 d T), with no operand or result selects but run's.  (acc in registers, selected by
// v_cndmask: 233 -> 241 ms for C5, msm 109 -> 118 ms, A/B.)

// The next entry's Niels point is brought into the wave's LDS slot by direct-to-LDS loads
// (gfx950 global_load_lds_dwordx4: lane l's 16-byte vector v lands at slot[v][l]) while the
// current step's arithmetic runs, so the prefetch costs no VGPRs (the kernel sits at the
// 256-VGPR budget of 2 waves per SIMD).  The vmcnt wait at the top of a step waits for that
// prefetch and the id prefetch (and, once per lane, the stores of its first window's sums).
__device__ __forceinline__ void part_stage(uint4 (*slot)[64], const PartArgs& a, const ge_niels* P, uint32_t id) {
  const uint32_t j = id & 0x7fffu;
  const ge_niels* src = j < 4u * kPartProofs ? P + j : a.tab + (j == 4u * kPartProofs ? 0 : kNielsEntriesRlc);
  const uint4* g = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int v = 0; v < 8; v++) __builtin_amdgcn_global_load_lds(g + v, &slot[v][0], 16, 0, 0);
}

// A lane walks one unit (window v, share h) of windows 0..15 and one of windows 16..31, as
// k_part_sort paired them (a.assign), each UPWARD through its buckets (its entries are one
// contiguous run of the sorted list), the second without waiting for the other lanes:
// run += entry, and at each bucket boundary acc += run, so at the end of a window's share
// S = run = sum_d B_d and A = acc = sum_d (Wh + W + 1 - d) B_d (stored in cached form);
// k_part_combine forms sum_d (d - Wh) B_d = (W + 1) S - A.  (One walk over both windows: two
// separate walks made every lane wait for the slowest lane of the first window.)  76 KB of
// LDS per block of 4 waves: per wave the staged point and acc (below).
//
// acc's slots in LDS, written and read limb by limb (no local array is address-taken, so
// nothing goes to scratch): an = (Y+X, Y-X, 2dT) in the staged points' 8-vector layout, az = Z.
#define CPZ_LIMB(f, i) ((uint32_t)(f).v[i])
__device__ __forceinline__ uint32_t limb30(const ge_cached& c, int i) {  // word i of (Y+X, Y-X, 2dT, 0, 0)
  return i < 10 ? CPZ_LIMB(c.YpX, i) : i < 20 ? CPZ_LIMB(c.YmX, i - 10) : i < 30 ? CPZ_LIMB(c.T2d, i - 20) : 0u;
}
__device__ __forceinline__ void acc_store(uint4 (*an)[64], uint4 (*az)[64], int lane, const ge_cached& c) {
#pragma unroll
  for (int k = 0; k < 8; k++)
    an[k][lane] = make_uint4(limb30(c, 4 * k), limb30(c, 4 * k + 1), limb30(c, 4 * k + 2), limb30(c, 4 * k + 3));
  az[0][lane] = make_uint4(CPZ_LIMB(c.Z, 0), CPZ_LIMB(c.Z, 1), CPZ_LIMB(c.Z, 2), CPZ_LIMB(c.Z, 3));
  az[1][lane] = make_uint4(CPZ_LIMB(c.Z, 4), CPZ_LIMB(c.Z, 5), CPZ_LIMB(c.Z, 6), CPZ_LIMB(c.Z, 7));
  az[2][lane] = make_uint4(CPZ_LIMB(c.Z, 8), CPZ_LIMB(c.Z, 9), 0u, 0u);
}
#undef CPZ_LIMB
__device__ __forceinline__ fe acc_load_z(uint4 (*az)[64], int lane) {
  const uint4 a = az[0][lane], b = az[1][lane], c = az[2][lane];
  fe r;
  r.v[0] = (int32_t)a.x; r.v[1] = (int32_t)a.y; r.v[2] = (int32_t)a.z; r.v[3] = (int32_t)a.w;
  r.v[4] = (int32_t)b.x; r.v[5] = (int32_t)b.y; r.v[6] = (int32_t)b.z; r.v[7] = (int32_t)b.w;
  r.v[8] = (int32_t)c.x; r.v[9] = (int32_t)c.y;
  return r;
}

__global__ void __launch_bounds__(256, 2) k_part_acc(PartArgs a) {
  __shared__ uint4 lds[4][19][64];  // per wave: staged point (0..7), acc (8..15), acc's Z (16..18)
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + wv;
  if (b >= a.nblk) return;  // whole waves
  ClockStamp clk;
  clk.start();
  const int64_t gb = a.blk0 + b;
  const uint32_t units = a.assign[b * kPartUnits + lane];  // (low unit, high unit), k_part_sort
  int v = (units & 0xff) >> 2, h = units & 3;
  const uint16_t* list = a.lists + b * kPartListCap;
  const uint16_t* ob = a.offs + b * kPartOffs;
  const ge_niels* P = a.pts + (int64_t)4 * kPartProofs * (a.pmap ? (int64_t)a.pmap[gb] : gb);
  ge_p3* ws = a.wsum + gb * kPartWsum;  // indexed by the global block: one combine pass for all chunks
  uint4 (*slot)[64] = lds[wv];
  int width = part_width(v), klo = width * h, k = klo;
  const uint16_t* o = ob + v * (kPartBuckets + 1);
  uint32_t e = o[k], eend = o[k + 1], elast = o[klo + width];
  uint32_t cid = e < elast ? list[e] : 0u;
  uint32_t nid = e + 1 < elast ? list[e + 1] : 0u;
  if (e < eend) part_stage(slot, a, P, cid);
  ge_p3 run = ge_identity();
  uint4 (*an)[64] = lds[wv] + 8;   // acc's Y+X, Y-X, 2dT (the staged points' layout)
  uint4 (*az)[64] = lds[wv] + 16;  // acc's Z
  auto acc_get = [&]() -> ge_cached {
    uint32_t w[32];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint4 x = an[u][lane];
      w[4 * u] = x.x;
      w[4 * u + 1] = x.y;
      w[4 * u + 2] = x.z;
      w[4 * u + 3] = x.w;
    }
    ge_cached c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      c.YpX.v[i] = (int32_t)w[i];
      c.YmX.v[i] = (int32_t)w[10 + i];
      c.T2d.v[i] = (int32_t)w[20 + i];
    }
    c.Z = acc_load_z(az, lane);
    return c;
  };
  acc_store(an, az, lane, ge_cached_identity());
#pragma unroll 1
  for (;;) {
    const bool entry = e < eend;
    const bool wend = !entry && k == klo + width - 1;  // last boundary of this window's share
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this step's point (and ids) arrived
    ge_niels q;
    uint4* qv = reinterpret_cast<uint4*>(&q);
    // the cached operand: the staged point (vectors 0..7 of the wave's LDS) or acc (8..15),
    // a per-lane index
    const int src = entry ? 0 : 8;
#pragma unroll
    for (int u = 0; u < 8; u++) qv[u] = lds[wv][src + u][lane];
    const fe zq = acc_load_z(az, lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): read before the slot is refilled
    q = ge_niels_cneg(q, entry && (cid >> 15) != 0);
    // the next step's position; its point (if it is an entry) staged now
    uint32_t e2 = e, eend2 = eend;
    int k2 = k;
    uint32_t cid2 = cid, nid2 = nid;
    if (entry) {
      e2 = e + 1;
      cid2 = nid;
      nid2 = e + 2 < elast ? list[e + 2] : 0u;
    } else if (!wend) {
      k2 = k + 1;
      eend2 = o[k2 + 1];
    }
    if (!wend && e2 < eend2) part_stage(slot, a, P, cid2);
    {
      ge_cached oc;
      oc.YpX = q.ypx;
      oc.YmX = q.ymx;
      oc.T2d = q.xy2d;
      oc.Z = fe_select(zq, fe_one(), entry);
      const ge_p3 r = p1p1_to_p3(ge_add_cached(run, oc));
      if (!entry) acc_store(an, az, lane, p3_to_cached(r));
      run = p3_select(run, r, entry);
    }
    if (wend) {
      const ge_cached acc = acc_get();
      store_p3(ws + (v * kPartQuarters + h) * 2, *reinterpret_cast<const ge_p3*>(&acc));  // A_h (cached)
      store_p3(ws + (v * kPartQuarters + h) * 2 + 1, run);                                // S_h
      if (v >= 16) {
        clk.stop(a.clock_probe, b);
        break;
      }
      v = (units >> 8) >> 2;
      h = (units >> 8) & 3;
      width = part_width(v);
      klo = width * h;
      k2 = klo;
      o = ob + v * (kPartBuckets + 1);
      e2 = o[k2];
      eend2 = o[k2 + 1];
      elast = o[klo + width];
      cid2 = e2 < elast ? list[e2] : 0u;
      nid2 = e2 + 1 < elast ? list[e2 + 1] : 0u;
      if (e2 < eend2) part_stage(slot, a, P, cid2);
      run = ge_identity();
      acc_store(an, az, lane, ge_cached_identity());
    }
    e = e2;
    eend = eend2;
    k = k2;
    cid = cid2;
    nid = nid2;
  }
}

// ---------------------------------------------------------------------------------------
// k_part_combine: quad j of the wave owns block 16 x blockIdx + j.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_part_combine(PartArgs a) {
  const int j = threadIdx.x >> 2, q = threadIdx.x & 3;
  const int64_t b = (int64_t)blockIdx.x * 16 + j;
  const bool live = b < a.nblk;
  const ge_p3* ws = a.wsum + (a.blk0 + (live ? b : a.nblk - 1)) * kPartWsum;  // dead quads: any block, dropped
  ge_p3 P = ge_identity();
#pragma unroll 1
  for (int v = kPartWindows - 1; v >= 0; v--) {
    // T_v = sum_d d B_d = sum_h (W + 1 + W h) S_h - A_h = W (Stot + Sw) + Stot - Atot with
    // Stot = sum_h S_h, Sw = S_1 + 2 S_2 + 3 S_3 = U + V + X (U = S_3, V = S_2 + U, X = S_1 + V),
    // W = part_width(v) a power of two
    const ge_p3* w = ws + v * kPartQuarters * 2;
    const ge_p3 U = load_p3(w + 7);
    const ge_p3 V = ge_add_quad(load_p3(w + 5), U, q);
    const ge_p3 X = ge_add_quad(load_p3(w + 3), V, q);
    const ge_p3 Stot = ge_add_quad(X, load_p3(w + 1), q);
    const ge_p3 Sw = ge_add_quad(ge_add_quad(U, V, q), X, q);
    ge_p3 At = ge_identity();  // the A_h are stored in cached form
#pragma unroll 1
    for (int hh = 0; hh < kPartQuarters; hh++) {
      const ge_p3 c = load_p3(w + 2 * hh);
      At = ge_add_quad(At, *reinterpret_cast<const ge_cached*>(&c), q);
    }
    ge_p3 T = p3_dbl_n_quad(ge_add_quad(Stot, Sw, q), __builtin_ctz(part_width(v)), q);
    T = ge_add_quad(T, Stot, q);
    T = ge_add_quad(T, ge_neg(At), q);
    if (v == kPartWindows - 1) P = T;
    else P = ge_add_quad(p3_dbl_n_quad(P, 8, q), T, q);
  }
  if (live && q == 0) {
    store_p3(a.part + a.blk0 + b, P);
    a.fail[a.blk0 + b] = a.fail[a.blk0 + b] | (ristretto_is_identity(P) ? 0 : 1);  // k_part_sort's bit 1
  }
}

// The same with one lane per block (CPZ_PART_COMBINE_LANE, launches of at least
// kPartLaneMinBlocks blocks: C5's first pass, 131,072 blocks = 2,048 waves): the same point
// operations done once each instead of spread over a quad, whose product rounds pay DPP
// exchanges and per-lane operand selects.  T_v is formed in the order that keeps the fewest
// points live (P, the running sums and one loaded point), each A_h subtracted as it is loaded.
__device__ __forceinline__ ge_p3 part_dbl_n(const ge_p3& p, int n) {  // n >= 1 doublings
  ge_p1p1 t = p3_dbl(p);
#pragma unroll 1
  for (int k = 1; k < n; k++) t = p2_dbl(p1p1_to_p2(t));
  return p1p1_to_p3(t);
}

__global__ void __launch_bounds__(256, 2) k_part_combine_lane(PartArgs a) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= a.nblk) return;
  const ge_p3* ws = a.wsum + (a.blk0 + b) * kPartWsum;
  ge_p3 P = ge_identity();
#pragma unroll 1
  for (int v = kPartWindows - 1; v >= 0; v--) {
    // T_v = W (Stot + Sw) + Stot - sum_h A_h (k_part_combine), Sw = U + V + X
    const ge_p3* w = ws + v * kPartQuarters * 2;
    ge_p3 R = load_p3(w + 7);             // U = S_3
    ge_p3 Sw = R;
    R = ge_add(load_p3(w + 5), R);        // V = S_2 + U
    Sw = ge_add(Sw, R);
    R = ge_add(load_p3(w + 3), R);        // X = S_1 + V
    Sw = ge_add(Sw, R);
    R = ge_add(R, load_p3(w + 1));        // Stot = X + S_0
    ge_p3 T = ge_add(part_dbl_n(ge_add(R, Sw), __builtin_ctz(part_width(v))), R);
#pragma unroll 1
    for (int hh = 0; hh < kPartQuarters; hh++) {  // the A_h are stored in cached form
      const ge_p3 c = load_p3(w + 2 * hh);
      T = p1p1_to_p3(ge_add_cached(T, ge_cached_cneg(*reinterpret_cast<const ge_cached*>(&c), true)));
    }
    P = v == kPartWindows - 1 ? T : ge_add(part_dbl_n(P, 8), T);
  }
  store_p3(a.part + a.blk0 + b, P);
  a.fail[a.blk0 + b] = a.fail[a.blk0 + b] | (ristretto_is_identity(P) ? 0 : 1);  // k_part_sort's bit 1
}

// The same per block for very few blocks (the locate pass of a sparse failure: each wave of
// k_part_combine runs ~800 dependent quad operations, 1.7 ms, whatever the block count): one
// workgroup of 32 quads per block, quad v forming T_v, then P_b = sum_v 2^(8 v) T_v by a tree
// (depth 8 + 16 + 32 + 64 + 128 doublings).  Its upper levels leave most quads of a wave idle,
// so at scale it costs far more than the packed chain (C5's 15,776-block locate pass: 202 ms
// against 197.5; every size: 245 ms), hence kPartTreeMaxBlocks.
__device__ __forceinline__ ge_p3 part_window_sum(const ge_p3* ws, int v, int q) {
  const ge_p3* w = ws + v * kPartQuarters * 2;
  const ge_p3 U = load_p3(w + 7);
  const ge_p3 V = ge_add_quad(load_p3(w + 5), U, q);
  const ge_p3 X = ge_add_quad(load_p3(w + 3), V, q);
  const ge_p3 Stot = ge_add_quad(X, load_p3(w + 1), q);
  const ge_p3 Sw = ge_add_quad(ge_add_quad(U, V, q), X, q);
  ge_p3 At = ge_identity();  // the A_h are stored in cached form
#pragma unroll 1
  for (int hh = 0; hh < kPartQuarters; hh++) {
    const ge_p3 c = load_p3(w + 2 * hh);
    At = ge_add_quad(At, *reinterpret_cast<const ge_cached*>(&c), q);
  }
  ge_p3 T = p3_dbl_n_quad(ge_add_quad(Stot, Sw, q), __builtin_ctz(part_width(v)), q);
  T = ge_add_quad(T, Stot, q);
  return ge_add_quad(T, ge_neg(At), q);
}

__global__ void __launch_bounds__(4 * kPartWindows) k_part_combine_tree(PartArgs a) {
  __shared__ ge_p3 lds[kPartWindows];
  const int v = threadIdx.x >> 2, q = threadIdx.x & 3;
  const int64_t b = blockIdx.x;
  const ge_p3* ws = a.wsum + (a.blk0 + b) * kPartWsum;
  const ge_p3 T = part_window_sum(ws, v, q);
  if (q == 0) lds[v] = T;
  __syncthreads();
#pragma unroll 1
  for (int span = 1; span < kPartWindows; span <<= 1) {
    ge_p3 r;
    const bool act = (v % (2 * span)) == 0;
    if (act) r = ge_add_quad(lds[v], p3_dbl_n_quad(lds[v + span], 8 * span, q), q);
    __syncthreads();
    if (act && q == 0) lds[v] = r;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const ge_p3 P = lds[0];
    store_p3(a.part + a.blk0 + b, P);
    a.fail[a.blk0 + b] = a.fail[a.blk0 + b] | (ristretto_is_identity(P) ? 0 : 1);  // k_part_sort's bit 1
  }
}

// ---------------------------------------------------------------------------------------
// sum_b P_b: quads add 64 consecutive entries each, then one wave adds those.
// ---------------------------------------------------------------------------------------
constexpr int kPartSumRun = 64;

__global__ void __launch_bounds__(64) k_part_sum1(const ge_p3* part, int64_t n, ge_p3* tmp) {
  const int j = threadIdx.x >> 2, q = threadIdx.x & 3;
  const int64_t g = (int64_t)blockIdx.x * 16 + j;
  const int64_t lo = g * kPartSumRun;
  ge_p3 acc = ge_identity();
#pragma unroll 1
  for (int k = 0; k < kPartSumRun; k++)
    if (lo + k < n) acc = ge_add_quad(acc, load_p3(part + lo + k), q);  // uniform per quad
  if (q == 0 && lo < n) store_p3(tmp + g, acc);
}

__global__ void __launch_bounds__(64) k_part_sum2(const ge_p3* tmp, int64_t m, uint32_t* partial_out,
                                                  int* identity_out) {
  __shared__ ge_p3 lds[16];
  const int j = threadIdx.x >> 2, q = threadIdx.x & 3;
  ge_p3 acc = ge_identity();
#pragma unroll 1
  for (int64_t k = j; k < m; k += 16) acc = ge_add_quad(acc, load_p3(tmp + k), q);
  if (q == 0) lds[j] = acc;
  __syncthreads();
  if (threadIdx.x < 4) {
    ge_p3 s = lds[0];
#pragma unroll 1
    for (int k = 1; k < 16; k++) s = ge_add_quad(s, lds[k], q);
    if (q == 0) {
      const bool id = ristretto_is_identity(s);
      uint32_t enc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (!id) ristretto_encode(enc, s);
      for (int k = 0; k < 8; k++) partial_out[k] = enc[k];
      identity_out[0] = id ? 1 : 0;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Locating the forged entry of a failing block (rlc.h: P'_b = sum_i j_i E_i, j = kPartLocJ0 - 2 t).
// k_part_index_digits: listed block b, thread t = proof kPartProofs * blocks[b] + t of the
// prepared batch: the first pass's scalars (weights from the same ChaCha20 block, rlc.hip
// k_rlc_prepare) times j -- the r-points' j a_i as an integer (nine signed radix-2^16 digits;
// j < 2^16 - 256 keeps |digit 8| < 2^15 - 128), j a_i c_i mod l and j b_i c_i mod l recoded, and
// the block sums of j a_i s_i, j b_i s_i.  Zero digits and sum terms where the prepare gave zero
// weight.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void index_weight_digits(int16_t d[kRlcWindows], const uint32_t u[4], int64_t j) {
  int64_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int64_t chunk = j * (int64_t)(int16_t)(u[w >> 1] >> (16 * (w & 1))) + carry;  // |chunk| < 2^31
    const int64_t lo = ((chunk + 0x8000) & 0xffff) - 0x8000;
    d[w] = (int16_t)lo;
    carry = (chunk - lo) >> 16;
  }
  d[8] = (int16_t)carry;
#pragma unroll
  for (int w = 9; w < kRlcWindows; w++) d[w] = 0;
}

__global__ void __launch_bounds__(kPartProofs) k_part_index_digits(PartIdxArgs a) {
  static_assert(kPartLocJ0 < (1 << 16) - 256 && kPartLocJ0 - 2 * (kPartProofs - 1) > (1 << 15),
                "index multipliers: digit 8 of j a below 2^15 - 128, and above 2^15 so that it spreads");
  __shared__ sc red_a[kPartProofs];
  __shared__ sc red_b[kPartProofs];
  const int64_t b = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t i = (int64_t)a.blocks[b] * kPartProofs + t;  // proof of the prepared batch
  const int64_t o = b * kPartProofs + t;                      // its compact slot
  const int64_t j = kPartLocJ0 - 2 * t;
  sc zero;
#pragma unroll
  for (int k = 0; k < 8; k++) zero.w[k] = 0;
  red_a[t] = zero;
  red_b[t] = zero;
  const bool live = i < a.n && a.status[i] == kStOk;
  uint32_t blk[16];
  if (live) chacha20_block(blk, a.seed, a.first_index + (uint64_t)i, 0);
  sc J = zero;
  J.w[0] = (uint32_t)j;
#pragma unroll 1
  for (int q = 0; q < 4; q++) {
    int16_t d[kRlcWindows];
#pragma unroll
    for (int w = 0; w < kRlcWindows; w++) d[w] = 0;
    if (live) {
      const uint32_t* u = q < 2 ? blk : blk + 4;
      if (q & 1) {
        sc c;
        rlc_load8(c.w, a.c, i);
        recode16(d, sc_mul(J, sc_mul(rlc_weight(u), c)).w);
      } else {
        index_weight_digits(d, u, j);
        sc sv;
        rlc_load8(sv.w, a.s, i);
        (q == 0 ? red_a : red_b)[t] = sc_mul(J, sc_mul(rlc_weight(u), sv));
      }
    }
#pragma unroll
    for (int w = 0; w < kRlcWindows; w++) a.digits[(int64_t)w * a.dstride + 4 * o + q] = d[w];
  }
  __syncthreads();
  for (int off = kRlcSumBlock / 2; off > 0; off >>= 1) {
    if ((t % kRlcSumBlock) < off) {
      red_a[t] = sc_add(red_a[t], red_a[t + off]);
      red_b[t] = sc_add(red_b[t], red_b[t + off]);
    }
    __syncthreads();
  }
  if (t % kRlcSumBlock == 0) {  // kPartProofs / kRlcSumBlock sums per listed block (k_part_sort adds them)
    const int64_t sb = b * (kPartProofs / kRlcSumBlock) + t / kRlcSumBlock;
    a.block_sums[2 * sb] = red_a[t];
    a.block_sums[2 * sb + 1] = red_b[t];
  }
}

// [k] P for a small k > 0 (double and add from the top bit).
__device__ __forceinline__ ge_p3 p3_mul_small(const ge_p3& P, uint32_t k) {
  ge_p3 R = P;
#pragma unroll 1
  for (int bit = 30 - __builtin_clz(k); bit >= 0; bit--) {
    R = p1p1_to_p3(p3_dbl(R));
    if ((k >> bit) & 1u) R = ge_add(R, P);
  }
  return R;
}

// k_part_locate: kPartLocLanes lanes per listed block; lane q tests the proofs t = q, q + L, ...
// (L = kPartLocLanes), i.e. j = J0 - 2 q, J0 - 2 q - 2 L, ..., against P'_b by ristretto
// equality, stepping by -[2 L] P_b.  The block is located iff exactly one j matches (and
// neither partial is incomplete nor P_b the identity).
__global__ void __launch_bounds__(256) k_part_locate(PartLocArgs a) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t b = g / kPartLocLanes;
  const int q = (int)(g % kPartLocLanes);
  const bool live = b < a.nblk;
  const int64_t bb = live ? b : a.nblk - 1;  // dead lanes: any block, dropped (whole groups)
  const ge_p3 P = load_p3(a.part + a.blocks[bb]);
  const ge_p3 Pl = load_p3(a.lpart + bb);
  const bool usable = !(a.lfail[bb] & 2) && !ristretto_is_identity(P);
  ge_p3 Q = p3_mul_small(P, (uint32_t)(kPartLocJ0 - 2 * q));
  const ge_p3 step = ge_neg(p3_mul_small(P, 2u * kPartLocLanes));
  int hits = 0, found = 0;
#pragma unroll 1
  for (int t = q; t < kPartProofs; t += kPartLocLanes) {
    if (ristretto_equal(Q, Pl)) {
      hits++;
      found = t;
    }
    Q = ge_add(Q, step);
  }
  // the block's lanes are consecutive lanes of one wave
#pragma unroll
  for (int m = 1; m < kPartLocLanes; m <<= 1) {
    const int oh = __shfl_xor(hits, m), of = __shfl_xor(found, m);
    found = of > found ? of : found;
    hits += oh;
  }
  if (live && q == 0) a.loc[b] = (usable && hits == 1) ? (uint16_t)found : kPartNoLoc;
}

__global__ void __launch_bounds__(256) k_gather_status(const uint8_t* status, const uint32_t* idx, int64_t m,
                                                       uint8_t* out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < m) out[k] = status[idx[k]];
}

hipError_t launch_part_index_digits(const PartIdxArgs& a, hipStream_t st) {
  if (a.nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_part_index_digits, dim3((unsigned)a.nblk), dim3(kPartProofs), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_part_locate(const PartLocArgs& a, hipStream_t st) {
  if (a.nblk <= 0) return hipSuccess;
  static_assert(64 % kPartLocLanes == 0 && kPartProofs % kPartLocLanes == 0, "a block's lanes in one wave");
  const int64_t threads = a.nblk * kPartLocLanes;
  hipLaunchKernelGGL(k_part_locate, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gather_status(const uint8_t* status, const uint32_t* idx, int64_t m, uint8_t* out, hipStream_t st) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_status, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, status, idx, m, out);
  return hipGetLastError();
}

hipError_t launch_part_sort(const PartArgs& a, hipStream_t st) {
  if (a.nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_part_sort, dim3((unsigned)a.nblk), dim3(kPartProofs), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_part_acc(const PartArgs& a, hipStream_t st) {
  if (a.nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_part_acc, dim3((unsigned)((a.nblk + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_part_msm(const PartArgs& a, hipStream_t st) {
  hipError_t e = launch_part_sort(a, st);
  if (e != hipSuccess) return e;
  return launch_part_acc(a, st);
}

// One launch for every block of the batch: a block's combine is a chain of ~800 dependent
// quad operations, so a launch needs many blocks (16 per wave) to keep the SIMDs busy -- per
// 8192-block chunk it was 512 waves, 0.95 ms each, 7.6 ms per 2^24 proofs.
hipError_t launch_part_combine(const PartArgs& a, hipStream_t st) {
  if (a.nblk <= 0) return hipSuccess;
  if (CPZ_PART_COMBINE_TREE && a.nblk <= kPartTreeMaxBlocks)
    hipLaunchKernelGGL(k_part_combine_tree, dim3((unsigned)a.nblk), dim3(4 * kPartWindows), 0, st, a);
  else if (CPZ_PART_COMBINE_LANE && a.nblk >= kPartLaneMinBlocks)
    hipLaunchKernelGGL(k_part_combine_lane, dim3((unsigned)((a.nblk + 255) / 256)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(k_part_combine, dim3((unsigned)((a.nblk + 15) / 16)), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_part_sum(const ge_p3* part, int64_t nblk, ge_p3* tmp, uint32_t* partial_out, int* identity_out,
                           hipStream_t st) {
  const int64_t m = (nblk + kPartSumRun - 1) / kPartSumRun;
  hipLaunchKernelGGL(k_part_sum1, dim3((unsigned)((m + 15) / 16)), dim3(64), 0, st, part, nblk, tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_part_sum2, dim3(1), dim3(64), 0, st, tmp, m, partial_out, identity_out);
  return hipGetLastError();
}

}  // namespace cpz
