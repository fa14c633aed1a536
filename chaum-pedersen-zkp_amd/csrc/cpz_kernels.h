// Kernel argument blocks and launchers shared by kernels.hip and the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "scalarmul.h"

namespace cpz {

constexpr uint8_t kStatusOk = 0;
constexpr uint8_t kStatusEqFail = 1;
constexpr uint8_t kStatusBadPoint = 2;
constexpr uint8_t kStatusBadScalar = 3;
constexpr uint8_t kStatusIdentity = 4;
constexpr uint8_t kStatusZeroS = 5;

constexpr int kNielsEntries = kTableB;   // radix-256 signed digits: |d| <= 128
// Niels table bases per generator: 2^(32 m) B for the level order m = 0, 4, 2, 6, 1, 3, 5, 7
// (B, 2^128 B: the eight-lane kernels' two 128-bit parts; all eight: k_verify_wide's 32-bit
// parts), tables [level][generator]
constexpr int kNielsLevels = 8;
__host__ __device__ constexpr int niels_level_doublings(int level) {
  return level == 0 ? 0 : (level == 1 ? 128 : (level == 2 ? 64 : (level == 3 ? 192 : 32 * (2 * (level - 4) + 1))));
}
// the level holding 2^(32 q) B: k_verify_wide's part q of s'
constexpr int kNielsLevelOfPart[8] = {0, 4, 2, 5, 1, 6, 3, 7};
constexpr bool niels_parts_consistent() {
  for (int q = 0; q < 8; q++)
    if (niels_level_doublings(kNielsLevelOfPart[q]) != 32 * q) return false;
  return true;
}
static_assert(niels_parts_consistent(), "kNielsLevelOfPart must invert niels_level_doublings");
constexpr int kCachedEntries = 2 * kTableSlots;   // y and r tables (identity + 1..8): |d| <= 8
#ifndef CPZ_VERIFY_BLOCK
#define CPZ_VERIFY_BLOCK 256
#endif
constexpr int kVerifyBlock = CPZ_VERIFY_BLOCK;  // threads per k_verify_each block

// Merlin/STROBE sponge snapshot.
struct StrobeSnap {
  uint8_t state[200];
  int32_t pos;
  int32_t pos_begin;
  int32_t flags;
  int32_t pad;
};

struct ChallengeArgs {
  int64_t n;
  uint32_t gh_words[16];         // encodings of g and h
  const uint32_t* y1;            // n x 8 words each (SoA rows of 32 bytes)
  const uint32_t* y2;
  const uint32_t* r1;
  const uint32_t* r2;
  const uint32_t* s;             // may be null (prover)
  const uint8_t* ctx_bytes;      // concatenated contexts
  const uint64_t* ctx_off;       // n + 1 offsets, or null: no contexts
  const uint8_t* ctx_present;    // n flags (Some/None), or null: all Some when ctx_off set
  const uint64_t* ctx_end = nullptr;  // non-null: entry i's context ends at ctx_end[i], not at
                                      // ctx_off[i + 1] (gathered entries: the density probe)
  const StrobeSnap* prefix;      // [0] after Transcript::new(), [1] after append_parameters
  uint32_t* c_out;               // n x 8 words
  uint8_t* status_out;           // n (written when s != null)
  int fast_noctx = 0;            // prefix[1] at the fixed position: k_challenge_noctx with k1 / k2
  uint32_t k1[50];               // framing masks of the fixed-schedule tail (challenge_masks)
  uint32_t k2[50];
  int fast_ctx32 = 0;            // prefix[0] at the fixed position: 32-byte contexts take
  uint32_t c32[3][50];           // challenge_fixed_ctx32 with these masks (challenge_masks_ctx32)
  int eq_only = 0;               // commitment checks off: a zero s is not reported (response_status)
};

// Proof::from_bytes outcome codes (gadgets.rs:364-489); kept equal to CPZ_PARSE_* in cpz.h.
enum ParseCode : uint8_t {
  kParseOk = 0, kParseTooSmall, kParseBadVersion,
  kParseR1LenMissing, kParseR1LenInvalid, kParseR1Truncated, kParseR1Size, kParseR1Point,
  kParseR2LenMissing, kParseR2LenInvalid, kParseR2Truncated, kParseR2Size, kParseR2Point,
  kParseSLenMissing, kParseSLenInvalid, kParseSTruncated, kParseSSize, kParseSScalar,
  kParseTrailing, kParseIdentity, kParseZeroS
};

struct ParseArgs {
  int64_t n;
  const uint8_t* blob;           // concatenated Proof::to_bytes blobs
  const uint64_t* off;           // n + 1 offsets into blob
  uint32_t* r1;                  // n x 8 words out (zero where not parsed)
  uint32_t* r2;
  uint32_t* s;
  uint8_t* code;                 // n ParseCode
  uint32_t* aux;                 // n message values (length / version / trailing count), or null
};

// The batch check's density probe (runtime.hip, launch_probe): kProbeChunks chunks of `blk`
// proofs at `starts`, gathered into contiguous rows (5 x 32 B per proof) and, with contexts,
// per-entry [begin, end) offsets into the batch's own context blob and presence flags.
constexpr int kProbeChunks = 16;
struct ProbeGatherArgs {
  int64_t starts[kProbeChunks];
  int blk;
  const uint32_t* rows[5];       // the batch's y1, y2, r1, r2, s
  uint32_t* out_rows[5];         // kProbeChunks * blk rows each
  const uint64_t* ctx_off;       // the batch's n + 1 offsets, or null
  const uint8_t* ctx_present;    // the batch's flags, or null
  uint64_t* out_begin;           // kProbeChunks * blk each (when ctx_off is set)
  uint64_t* out_end;
  uint8_t* out_present;
};

// Launches of 2049 .. kQuadVerifyMax proofs are verified on eight lanes per proof
// (k_verify_quad), larger ones on one lane per proof (k_verify_each); at most 512 take
// k_verify_wide and up to 2048 k_verify_small (runtime.hip, launch_verify_chunks).  The
// crossover was measured in r04 (tools/quad_crossover.py, cpz_verify_each_device per call:
// eight lanes 0.78 / 1.52 ms at 16K / 32K proofs, one lane 1.26-1.31 ms).  The scratch slab
// holds kQuadProofScratch bytes of tables per proof for them (VerifyArgs::quad_max, the
// runtime's verify_quad_max: this constant capped by the slab, i.e. by the device's CUs).
#ifndef CPZ_VERIFY_QUAD
#define CPZ_VERIFY_QUAD 1
#endif
#ifndef CPZ_QUAD_MAX
#define CPZ_QUAD_MAX 16384
#endif
constexpr int64_t kQuadVerifyMax = CPZ_QUAD_MAX;
constexpr int kQuadTableInts = 2 * 9 * 40;  // per quad: two tables of 9 entries of 4 x 10 limbs
// Per-proof calls of at most this many proofs whose (g, h) has no comb in the context's cache
// verify against the pair's 128-entry Niels tables (VerifyArgs::vtab) instead of building the
// 128 MiB combs (~3 ms): [s'] B by radix-256 digits inside the Straus loop, +16 additions per
// equation against the comb's 16.  The default pair always gets its comb.
constexpr int64_t kVarBaseMax = kQuadVerifyMax;
// k_verify_quad phase stamps (CPZ_CLOCK_PROBE): start, split + digits, decode, tables, Straus,
// comb, verdict; then the 100 MHz clock at start and end.
constexpr int kQuadPhases = 9;
// k_verify_small's stamps (CPZ_CLOCK_PROBE): wave 0 start, decoded, table, barrier A, Straus,
// barrier B, verdict; wave 2 digits, [s'] B; 100 MHz at wave 0's start / end; wave 2's start.
constexpr int kSmallStamps = 16;
constexpr int64_t kQuadProofScratch = 2 * kQuadTableInts * 4;

struct VerifyArgs {
  int64_t n;
  const uint32_t* y1;
  const uint32_t* y2;
  const uint32_t* r1;
  const uint32_t* r2;
  const uint32_t* s;
  const uint32_t* c;
  uint8_t* status;               // in: response-scalar status; out: final status
  const ge_niels* comb;          // fixed-base combs of g then h, kCombPerBase entries each
  char* scratch;                 // table slab: grid * kVerifyBlock threads x kCachedEntries ge_cached
  const ge_niels* pre = nullptr; // RLC fallback: the prepared Niels points (-r1, -y1, -r2, -y2 of
                                 // proof i at 4 i ..), reused instead of decoding; entries whose
                                 // decode-level status is non-zero keep it
  int eq_only = 0;                  // commitment checks off: identity r1 / r2 and zero s are not
                                    // reported, the equations alone decide (verify_proof)
  const uint32_t* blocks = nullptr; // k_verify_prepared: the partitioned check's failing blocks of
                                    // block_proofs proofs each, nblocks of them; workgroup g takes
                                    // kVerifyBlock / block_proofs consecutive listed blocks; n bounds
                                    // the global proof index
  int block_proofs = 0;
  int64_t nblocks = 0;
  int64_t quad_max = 0;             // launches of at most this many proofs use k_verify_quad (the
                                    // runtime: kQuadVerifyMax, bounded by the slab's size)
  uint64_t* clock_probe = nullptr;  // CPZ_CLOCK_PROBE builds only: k_verify_quad's phase stamps
                                    // (kQuadPhases shader-clock words of block 0's first proof)
  const int32_t* vtab16 = nullptr;  // the same tables as 16-bit limbs for k_verify_wide (fe16.h):
                                    // [8 bases][128 entries][Y+X, Y-X, 2dxy][16 limbs]
  const ge_niels* vtab = nullptr;   // variable-base generators (no comb built for this (g, h)):
                                    // Niels multiples 1..128 of g, h, 2^128 g, 2^128 h
                                    // (k_build_niels), [s'] B from them inside the Straus loop;
                                    // k_verify_quad only (launches of at most quad_max proofs)
};

struct ProveArgs {
  int64_t n;
  uint64_t first_index;
  uint32_t seed_x[8];
  uint32_t seed_k[8];
  const uint32_t* x_in;          // caller witnesses / nonces (n x 8 words, taken mod l), or null:
  const uint32_t* k_in;          // derived from seed_x / seed_k (synthetic inputs)
  const ge_niels* comb;          // fixed-base combs of g then h
  uint32_t* y1;
  uint32_t* y2;
  uint32_t* r1;
  uint32_t* r2;
  const uint32_t* c;
  uint32_t* s_out;
};

hipError_t launch_transcript_prefix(const uint32_t* gh_words, StrobeSnap* out, hipStream_t st);
hipError_t launch_challenge(const ChallengeArgs& a, hipStream_t st);
hipError_t launch_probe_gather(const ProbeGatherArgs& a, hipStream_t st);
bool challenge_prefix_is_fixed(const StrobeSnap& snap);  // the no-context fast path applies
bool challenge_prefix_is_ctx32(const StrobeSnap& snap);  // prefix[0]: the 32-byte-context fast path applies
// Niels tables of kNielsLevels * nbases bases (nbases <= 2: one wave of quads); `bases` is
// scratch for kNielsLevels * nbases ge_p3.
hipError_t launch_build_niels(const uint32_t* base_words, int nbases, ge_niels* tab, int* ok, ge_p3* bases,
                              hipStream_t st);
// The Niels tables' fields as canonical 16-bit limbs (VerifyArgs::vtab16): n entries.
hipError_t launch_niels_r16(const ge_niels* tab, int32_t* out, int n, hipStream_t st);
hipError_t launch_parse_proofs(const ParseArgs& a, hipStream_t st);
// Fixed-base combs of 2 bases (g, h): bases_scratch holds 2 * kCombWindows ge_p3.
hipError_t launch_build_comb(const uint32_t* gh_words, ge_p3* bases_scratch, ge_niels* comb, hipStream_t st);
hipError_t launch_verify_each(const VerifyArgs& a, int grid, hipStream_t st);
// k_verify_small (kernels.hip): three waves per 8 proofs, the drop-in's latency path.  a.c null:
// the challenges and response statuses are computed in the kernel from ca (k_challenge's inputs).
hipError_t launch_verify_small(const VerifyArgs& a, const ChallengeArgs& ca, hipStream_t st);
// one proof per workgroup of six waves (4 + CPZ_WIDE_VB_WAVES = eight with vtab16), field products
// on 16-lane rows (fe16.h)
hipError_t launch_verify_wide(const VerifyArgs& a, const ChallengeArgs& ca, hipStream_t st);
int verify_each_blocks_per_cu();  // resident k_verify_each blocks per CU (occupancy API)
hipError_t launch_prove_points(const ProveArgs& a, hipStream_t st);
hipError_t launch_prove_response(const ProveArgs& a, hipStream_t st);
// Bulk decode (+ re-encode when out != null) of n encodings.
hipError_t launch_decode_encode(int64_t n, const uint32_t* pts, uint8_t* ok, uint32_t* out, hipStream_t st);
// cpz_verify_response: response status of s and the caller's challenge (sanitised copy to c_out).
hipError_t launch_response_prep(int64_t n, const uint32_t* s, const uint32_t* c_in, uint32_t* c_out, uint8_t* status,
                                int eq_only, hipStream_t st);

}  // namespace cpz
