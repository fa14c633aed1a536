// Argument blocks and launchers of the RLC / Pippenger path (rlc.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "scalar25519.h"
#include "scalarmul.h"

namespace cpz {

constexpr int kRlcWindows = 16;          // 16-bit signed windows cover scalars < 2^255
constexpr int kRlcBuckets = 1 << 15;     // |digit| in [1, 2^15]
#ifndef CPZ_RLC_SEGLEN
#define CPZ_RLC_SEGLEN 32
#endif
constexpr int kRlcSegLen = CPZ_RLC_SEGLEN;  // buckets per reduction segment
constexpr int kRlcPrepBlock = 256;       // proofs per prepare workgroup (the bisection / shard / span granule)
constexpr int kRlcSumBlock = 128;        // proofs per block sum (block_sums granule; kRlcPrepBlock / 2)
#ifndef CPZ_RLC_PREP_WIDE_MAX
#define CPZ_RLC_PREP_WIDE_MAX (1 << 15)
#endif
constexpr int64_t kRlcPrepWideMax = CPZ_RLC_PREP_WIDE_MAX;  // up to this many proofs: four lanes per proof
constexpr int kRlcSortBlock = 1024;
#ifndef CPZ_RLC_SORT_CHUNK
#define CPZ_RLC_SORT_CHUNK (1 << 16)
#endif
constexpr int kRlcSortGroups = 64;      // max blocks per window in the counting sort
constexpr int64_t kRlcSortChunk = CPZ_RLC_SORT_CHUNK;  // target points per sort block
constexpr int kNielsEntriesRlc = kTableB;
constexpr int kRlcChunk = 64;            // sorted entries per bucket-accumulation thread (at most)
constexpr int kRlcMinChunk = 4;          // ... and at least (small MSMs, rlc_sort_geometry)
constexpr int64_t kRlcMinHeads = 2048;   // head slots per window whatever the MSM's size
#ifndef CPZ_RLC_SPARSE
#define CPZ_RLC_SPARSE 1
#endif
constexpr int kRlcSparsePts = 2048;      // MSMs of at most this many points reduce their non-empty buckets only
// Points of one MSM (its flat positions t, incl. the two extras): the 32-bit entries hold t
// in 24 bits and all-ones is their empty marker.
constexpr int64_t kRlcMaxMsmPoints = (1ll << 24) - 1;

struct RlcPrepArgs {
  int64_t n;
  uint64_t first_index;          // global index of proof 0 (weights are keyed by it)
  uint32_t seed[8];
  const uint32_t* y1;
  const uint32_t* y2;
  const uint32_t* r1;
  const uint32_t* r2;
  const uint32_t* s;
  const uint32_t* c;             // challenges from k_challenge
  uint8_t* status;               // in: response status; out: decode-level status (0/2/3/4)
  ge_niels* pts;                 // 4 n (+2 extra) negated affine points
  int16_t* digits;               // [16][dstride] signed radix-2^16 digits
  int64_t dstride;
  sc* block_sums;                // [2 ceil(n/256)][2]: sum a s, sum b s per 128 proofs
  sc* quarter_sums = nullptr;    // [ceil(n/64)][2]: scratch of the four-lanes-per-proof prepare
  int* any_bad;                  // set to 1 if some proof has a non-zero decode-level status
  int eq_only = 0;               // commitment checks off: identity r1 / r2 keep their weight
  uint64_t* clock_probe = nullptr;  // CPZ_CLOCK_PROBE builds only: 5 words per wave (rlc_dev.h)
};

struct RlcMsmArgs {
  int64_t p0, p1;                // point range [p0, p1)
  int64_t e0;                    // the two extra points (g, h) live at e0, e0 + 1
  ge_niels* pts;
  int16_t* digits;
  int64_t dstride;
  uint32_t* counts;              // [16][2^15]
  uint32_t* offsets;             // [16][2^15 + 1]
  uint32_t* bhist;               // [16][groups][2^15] per-sort-block histograms -> block bases
  int groups;                    // sort blocks per window
  int64_t chunk;                 // points per sort block
  int echunk = kRlcChunk;        // sorted entries per k_rlc_bucket thread (rlc_sort_geometry)
  int sparse = 0;                // set by launch_rlc_msm: small MSM, non-empty buckets reduced alone ...
  int sgroups = 4;               // ... by this many workgroups per window
  uint32_t* idx;                 // [16][istride]
  uint32_t* inter;               // [16][istride] coarse-sorted entries (32-bit)
  int64_t istride;
  ge_p3* buckets;                // [16][2^15]
  ge_p3* heads;                  // [16][hstride] partials of buckets begun in an earlier chunk
  int64_t hstride;               // >= ceil(points / echunk)
  ge_p3* seg_s;                  // [16][2^15 / kRlcSegLen]
  ge_p3* seg_w;                  // [16][2^15 / kRlcSegLen]
  ge_p3* win;                    // [16]
  uint32_t* partial_out;         // 8 words
  int* identity_out;             // 1
  // A batch verified as several MSMs over consecutive proof spans: the final of each span
  // adds its P into *total (the first span stores it), and only the last span encodes --
  // the sum -- into partial_out / identity_out.  total == nullptr: a single MSM.
  ge_p3* total = nullptr;
  int total_first = 1, total_last = 1;
  int* span_identity = nullptr;  // multi-span batches: 1 if this span's own P is the identity
                                 // (the batch-fail fallback then skips the span)
  uint64_t* clock_probe = nullptr;  // CPZ_CLOCK_PROBE builds only: k_rlc_bucket, 5 words per wave
};

// ---- partitioned batch check (part.hip) --------------------------------------------------
// The batch's prepared points cut into blocks of kPartProofs proofs (the weight blocks); one
// Pippenger MSM per block with signed 8-bit windows (the 16-bit digits of the prepare split in
// two), giving every block's partial P_b = sum over its proofs of the RLC terms.  A block with
// P_b the identity holds no forgery (w.o.p.); the others go to per-proof verification.
// 128: C5 210.8 / 210.0 ms against 221.3 / 221.8 ms with blocks of 256 proofs (A/B, one call): the
// failing blocks' per-proof pass halves (12 % of the proofs at 0.1 % forged instead of 23 %),
// the block partials cost 16 % more per proof (98 -> 114 ms: the 32 x 128 bucket boundaries per
// block are spread over half the entries).
#ifndef CPZ_PART_PROOFS
#define CPZ_PART_PROOFS 128
#endif
constexpr int kPartProofs = CPZ_PART_PROOFS;          // proofs per block (128 or 256)
static_assert(kPartProofs == 128 || kPartProofs == 256, "partition blocks are one or two block sums");
constexpr int kPartPoints = 4 * kPartProofs + 2;      // + g, h with the block's weight sums
constexpr int kPartWindows = 2 * kRlcWindows;         // 32 signed radix-2^8 windows
constexpr int kPartBuckets = 128;                     // |digit| in [1, 128]
constexpr int kPartQuarters = 4;                      // lanes per window pair (32 buckets each)
constexpr int kPartTopBuckets = 16;                   // |digit| bound of the top window (part.hip)
constexpr int kPartListCap = kPartWindows * kPartPoints;  // sorted entries per block, at most
constexpr int kPartOffs = kPartWindows * (kPartBuckets + 1);
constexpr int kPartWsum = kPartWindows * kPartQuarters * 2;  // (W, S) per window and quarter
constexpr int kPartUnits = kPartWindows * kPartQuarters / 2;  // walk units per half (64 = lanes)
// Combines of at most this many blocks run one workgroup per block (k_part_combine_tree).
// k_part_combine_lane (one lane per block) for launches of at least kPartLaneMinBlocks blocks
#ifndef CPZ_PART_COMBINE_LANE
#define CPZ_PART_COMBINE_LANE 1
#endif
#ifndef CPZ_PART_LANE_MIN
#define CPZ_PART_LANE_MIN (1 << 16)
#endif
constexpr int64_t kPartLaneMinBlocks = CPZ_PART_LANE_MIN;
#ifndef CPZ_PART_COMBINE_TREE
#define CPZ_PART_COMBINE_TREE 1
#endif
#ifndef CPZ_PART_TREE_MAX
#define CPZ_PART_TREE_MAX 256
#endif
constexpr int64_t kPartTreeMaxBlocks = CPZ_PART_TREE_MAX;

struct PartArgs {
  int64_t nblk;                  // blocks of this launch: [blk0, blk0 + nblk) of the prepared set
  int64_t blk0;
  int64_t n;                     // proofs of the prepared set (the last block may be partial)
  const ge_niels* pts;           // prepared negated Niels points, 4 per proof
  const int16_t* digits;         // [16][dstride] signed radix-2^16 digits
  int64_t dstride;
  const sc* block_sums;          // [sum blocks][2]: sum a s, sum b s per kRlcSumBlock proofs
  const ge_niels* tab;           // g at tab[0], h at tab[kNielsEntriesRlc]
  uint16_t* lists;               // [nblk][kPartListCap] point ids (bit 15: negate) sorted by (window, bucket)
  uint16_t* offs;                // [nblk][kPartOffs] bucket starts per window (+ window end)
  ge_p3* wsum;                   // [blocks][kPartWsum] (indexed by the global block)
  uint16_t* assign;              // [nblk][kPartUnits] lane -> (unit of windows 0..15, unit of 16..31)
  ge_p3* part;                   // [blocks] P_b (indexed by the global block)
  uint8_t* fail;                 // [blocks] bit 0: P_b is not the identity; bit 1: a top-window
                                 // digit exceeded kPartTopBuckets (the block is verified per proof)
  const uint32_t* pmap = nullptr;  // locate pass: listed block b's points are those of prepared
                                   // block pmap[b] (digits, sums and outputs are compact)
  uint64_t* clock_probe = nullptr;  // CPZ_CLOCK_PROBE builds only: k_part_acc, 5 words per wave
};

// ---- locating a failing block's forged entry (part.hip) ----------------------------------
// A failing block's second partial with the weights of its proof t multiplied by
// j_t = kPartLocJ0 - 2 t:  P'_b = sum_i j_i E_i  where  P_b = sum_i E_i  (E_i proof i's weighted
// terms; the identity, up to 4-torsion, for a valid proof).  With one forged proof f,
// P'_b = [j_f] P_b; with more, no j satisfies it except with probability ~2^-121 per block (128
// candidate j against 128-bit weights).  The r-points' scalars j a_i are kept as integers (signed
// radix-2^16 digits with a ninth digit), the others reduced mod l, so the pass has the first's
// window structure.  The j lie just below 2^16 so that the ninth digit spreads over its range:
// with j = t + 1 or 2 t + 1 the r-points' ninth digits were small and piled into the lowest
// buckets of 8-bit windows 16 / 17, and the walk waited for the lane holding them (C5's 15,776
// failing blocks: 18.1 - 20.9 ms, against 13.4 ms for the same walk with j = 1).
constexpr int64_t kPartLocJ0 = (1 << 16) - 257;
#ifndef CPZ_PART_LOCATE
#define CPZ_PART_LOCATE 1
#endif
constexpr int kPartLocLanes = 8;     // lanes per block in k_part_locate (t = q, q + 8, ...)
constexpr uint16_t kPartNoLoc = 0xffff;

struct PartIdxArgs {
  int64_t nblk;                  // listed blocks
  int64_t n;                     // proofs of the prepared batch
  const uint32_t* blocks;        // [nblk] prepared block of each listed block
  uint64_t first_index;          // the prepare's weight keys
  uint32_t seed[8];
  const uint32_t* s;
  const uint32_t* c;
  const uint8_t* status;         // decode-level statuses of the prepare (non-zero: zero weight)
  int16_t* digits;               // [16][dstride] compact: listed block b's proof t at 4 (kPartProofs b + t)
  int64_t dstride;
  sc* block_sums;                // [nblk * kPartProofs / kRlcSumBlock][2], compact
};

struct PartLocArgs {
  int64_t nblk;
  const uint32_t* blocks;        // [nblk] prepared block of each listed block
  const ge_p3* part;             // [prepared blocks] P_b of the first pass
  const ge_p3* lpart;            // [nblk] P'_b of the index-weighted pass
  const uint8_t* lfail;          // [nblk] its flags (bit 1: incomplete partial)
  uint16_t* loc;                 // [nblk] out: the forged proof's index in the block, or kPartNoLoc
};

hipError_t launch_part_index_digits(const PartIdxArgs& a, hipStream_t st);
hipError_t launch_part_locate(const PartLocArgs& a, hipStream_t st);
// out[k] = status[idx[k]] for k < m
hipError_t launch_gather_status(const uint8_t* status, const uint32_t* idx, int64_t m, uint8_t* out, hipStream_t st);

hipError_t launch_part_msm(const PartArgs& a, hipStream_t st);      // sort + walk of [blk0, blk0 + nblk)
hipError_t launch_part_sort(const PartArgs& a, hipStream_t st);     // the sort alone
hipError_t launch_part_acc(const PartArgs& a, hipStream_t st);      // the walk alone (k_part_acc)
hipError_t launch_part_combine(const PartArgs& a, hipStream_t st);  // P_b and fail flags of [blk0, blk0 + nblk)
// out = sum of part[0 .. nblk) (encoded, identity flag), through the scratch `tmp` of
// ceil(nblk / 16) ge_p3
hipError_t launch_part_sum(const ge_p3* part, int64_t nblk, ge_p3* tmp, uint32_t* partial_out, int* identity_out,
                           hipStream_t st);

hipError_t launch_rlc_prepare(const RlcPrepArgs& a, hipStream_t st);
// Sort and accumulation geometry for `npts` MSM points: sets a.groups / a.chunk / a.echunk.
void rlc_sort_geometry(RlcMsmArgs& a, int64_t npts);
// marks (optional, timing): kRlcMsmMarks events recorded on `st` at the phase boundaries
// (start | sort: extra, hist, bscan, scan, coarse, fine | bucket | bucket fix | segment + window
// | final).
constexpr int kRlcMsmMarks = 6;
// final_wait / final_done (overlapped spans, runtime.hip rlc_range_launch): the stream waits for
// final_wait before k_rlc_final (the previous span's final, which owns RlcMsmArgs::total) and
// records final_done after it; everything before the final overlaps freely.
hipError_t launch_rlc_msm(const RlcMsmArgs& a, const sc* block_sums, int64_t b0, int64_t b1, const ge_niels* tab,
                          hipStream_t st, hipEvent_t* marks = nullptr, hipEvent_t final_wait = nullptr,
                          hipEvent_t final_done = nullptr);
hipError_t launch_msm_load(int64_t n, const uint32_t* pts_enc, const uint32_t* scalars, ge_niels* pts,
                           int16_t* digits, int64_t dstride, int* bad, hipStream_t st);
hipError_t launch_rlc_combine(const uint32_t* parts, int k, uint32_t* out, int* flags, hipStream_t st);

}  // namespace cpz
