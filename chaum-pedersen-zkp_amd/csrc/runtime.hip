// Host runtime behind the C ABI (include/cpz.h): device context, generator-table cache,
// reusable device buffers, kernel sequencing.  One HIP stream per context.
//
// Call sequence for cpz_verify_each (replaces BatchVerifier::verify, batch.rs:171-231):
//   [cache miss on (g, h)]  k_build_niels(g, h) + k_transcript_prefix(g, h)
//                           + k_comb_bases / k_comb_fill (128 MiB fixed-base combs)
//   k_challenge   -> c_i, response-scalar status          (transcript + gadgets checks)
//   k_verify_each -> final status                         (decode + two equations)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cpz.h"
#include "cpz_kernels.h"
#include "rlc.h"
#include "verify.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define CPZ_HIP(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(CPZ_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));           \
  } while (0)

const uint8_t kDefaultG[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                               0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                               0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
const uint8_t kDefaultH[32] = {0xc8, 0xdb, 0x6f, 0x46, 0xe1, 0xb9, 0x1e, 0x7e, 0x93, 0xac, 0xe6,
                               0x9e, 0xab, 0x46, 0x97, 0x6e, 0xfe, 0xbe, 0x07, 0xde, 0xaf, 0x5b,
                               0x9a, 0x2a, 0x74, 0x42, 0xfd, 0x02, 0x36, 0x40, 0x16, 0x23};

// Device buffer that only grows.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      hipError_t e = hipFree(p);
      p = nullptr;
      cap = 0;
      if (e != hipSuccess) return e;
    }
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Page-locked host memory (hipHostMalloc), grown on demand; dp = its device view.
struct PinnedBuf {
  void* p = nullptr;
  void* dp = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      hipError_t e = hipHostFree(p);
      p = dp = nullptr;
      cap = 0;
      if (e != hipSuccess) return e;
    }
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    cap = 0;
  }
};

// A stream on a hardware queue of its own.  HIP maps plain streams onto at most
// GPU_MAX_HW_QUEUES (4 by default) queues per process, reusing the least-used one beyond that,
// and two streams on one queue run one after the other: two torch streams created after the
// contexts' streams shared a queue (rocprofv3 Queue_Id), so the two batch checks issued on
// them never overlapped (0.996x one in flight, against 1.07x on the contexts' own streams).
// A stream with a CU mask always gets a queue of its own; the mask here holds every CU, so
// the verify streams (whose launches must overlap) stay concurrent whatever other streams
// the process creates.  Such a stream synchronises with the legacy default stream
// (hipStreamDefault semantics), which only adds ordering.
//
// Dedicated queues are capped per device (kMaxOwnQueues for the whole process): several
// contexts per GPU (a pool, the multi-context entry points) would otherwise claim 4 queues
// each and oversubscribe the hardware scheduler's queue slots.  Contexts take them in the
// order they create streams -- the context stream at creation, the verify stream with the
// first verify, the probe and copy streams last -- and streams beyond the cap are plain.
constexpr int kMaxOwnQueues = 16;
std::atomic<int> g_own_queues[64];

hipError_t stream_own_queue(hipStream_t* s, int cus, int device, int* taken) {
  std::atomic<int>* slot = device >= 0 && device < 64 ? &g_own_queues[device] : nullptr;
  if (slot && slot->fetch_add(1) < kMaxOwnQueues) {
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int c = 0; c < cus; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
    if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
      *taken += 1;
      return hipSuccess;
    }
    (void)hipGetLastError();
  }
  if (slot) slot->fetch_sub(1);
  return hipStreamCreateWithFlags(s, hipStreamDefault);
}

// Host-buffer pipeline chunk (proofs): 2^17 proofs = 20 MiB of inputs, ~2.8 ms of verify work.
constexpr size_t kPipeChunk = size_t(1) << 17;

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// partial_out of a batch check that skipped its MSM (dense fallback): 32 x 0xff, not an encoding
bool is_no_partial(const uint8_t p[32]) {
  for (int k = 0; k < 32; k++)
    if (p[k] != 0xff) return false;
  return true;
}

// RLC buffers come in two sets with their own capacities, and an MSM's arguments are derived
// from the sets it is handed, never from a context-wide size (rlc_msm_args):
//   RlcPrepared  the batch's prepared MSM input: 4 n + 2 negated Niels points, the digit rows
//                [16][dstride], per-128-proof block sums (kRlcSumBlock).  Capacity: proofs of the batch.
//   RlcMsmSet    sort / bucket / reduction buffers of ONE MSM, its partial and identity flag.
//                Capacity: proofs of one MSM (a span of at most CPZ_RLC_SPAN proofs).
struct RlcPrepared {
  DevBuf pts, dig, bsum, qsum;
  int64_t cap = 0;
  void release() {
    for (DevBuf* b : {&pts, &dig, &bsum, &qsum}) b->release();
    cap = 0;
  }
};

struct RlcMsmSet {
  DevBuf counts, offsets, bhist, idx, inter, buckets, heads, segs, segw, win, total, partial, flags;
  int64_t cap = 0;
  void release() {
    for (DevBuf* b : {&counts, &offsets, &bhist, &idx, &inter, &buckets, &heads, &segs, &segw, &win, &total, &partial,
                      &flags})
      b->release();
    cap = 0;
  }
};

// Fixed-base tables and transcript prefix of one (g, h) pair (ensure_generators).  A full set
// has the combs; a light set (a small per-proof call on a pair without one) only the Niels
// tables, which k_verify_quad reads as variable bases (VerifyArgs::vtab).
struct GenSet {
  bool valid = false;
  bool full = true;
  uint64_t used = 0;  // LRU stamp
  uint8_t gh[64];
  DevBuf tab;       // 16 x 128 ge_niels (g, h at 2^(32 m) times, build_niels_prefix's order)
  DevBuf tab16;     // the same as 16-bit limbs (k_verify_wide's variable bases)
  DevBuf comb;      // fixed-base combs of g and h: 2 x 16 x 2^15 ge_niels (128 MiB)
  DevBuf comb_q;    // 32 ge_p3: 2^(16 k) g, 2^(16 k) h
  DevBuf prefix;    // 2 StrobeSnap
  DevBuf gh_words;  // 16 words
  bool prefix_fixed = false;  // prefix[1] at the fixed position: k_challenge_noctx applies
  uint32_t chal_k1[50], chal_k2[50];  // its framing masks
  bool ctx32_fixed = false;   // prefix[0] at the fixed position: 32-byte contexts' fast path
  uint32_t chal_c32[3][50];   // its framing masks (g and h folded in)
  void release() {
    for (DevBuf* b : {&tab, &tab16, &comb, &comb_q, &prefix, &gh_words}) b->release();
    valid = false;
  }
};

// (g, h) pairs whose tables a context keeps (128 MiB of combs each): a service verifying
// batches of several Parameters groups rebuilds nothing while it uses at most this many.
#ifndef CPZ_GEN_CACHE
#define CPZ_GEN_CACHE 4
#endif
constexpr int kGenCache = CPZ_GEN_CACHE;
// Light sets a context keeps: each holds the pair's Niels tables (16 bases x 128 ge_niels, 245 KB)
// and their 16-bit-limb copy (16 x 128 x 48 int32, 196 KB) -- ~440 KB per set, ~28 MB for all 64 --
// plus the transcript prefix.
constexpr int kLightCache = 64;

}  // namespace

struct cpz_ctx {
  int device = 0;
  int cus = 0;
  int verify_blocks_per_cu = 2;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // fixed-base tables of the kGenCache most recently used (g, h) pairs; `gs` is the current one
  GenSet gen[kGenCache];
  int gen_cap = kGenCache;  // full sets kept (env CPZ_GEN_CACHE at creation: 1 .. kGenCache)
  GenSet light[kLightCache];
  GenSet* gs = nullptr;
  uint64_t gen_clock = 0;
  DevBuf ok_flags;  // 2 ints
  DevBuf gen_bases; // 4 ge_p3: g, h, 2^128 g, 2^128 h (k_niels_bases)
  // work buffers
  DevBuf c;         // n x 32
  DevBuf st;        // n
  DevBuf scratch;   // per-stream table slabs (kCachedEntries ge_cached per thread)
  // host-API staging (y1, y2, r1, r2, s, and challenges / witnesses / nonces)
  DevBuf in[7];
  DevBuf ctxb, ctxo, ctxp;
  // small host-buffer calls: inputs packed into one page-locked block and one copy (`in_all`),
  // and the RLC check's partial, flags and statuses read back with one synchronisation (`pin`
  // from kPinMail on; the mailbox words at its start)
  DevBuf in_all;
  PinnedBuf pin;
  // host-buffer pipeline (cpz_verify_each): H2D copies of chunk j+1 on their own stream
  // while chunk j verifies on `stream`
  hipStream_t copy_stream = nullptr;
  hipEvent_t copy_done = nullptr;
  // verify chunks round-robin over the launch stream and these (launch_verify_chunks)
  hipStream_t aux_stream[3] = {nullptr, nullptr, nullptr};
  hipEvent_t aux_start = nullptr;
  hipEvent_t aux_done[3] = {nullptr, nullptr, nullptr};
  // wire-format ingestion
  DevBuf pz_blob, pz_off, pz_rows, pz_code, pz_aux;
  // batch-check density probe (verify_batch_impl): sampled rows, challenges, statuses
  DevBuf probe;
  hipStream_t probe_stream = nullptr;
  hipEvent_t probe_done = nullptr;
  // RLC / Pippenger buffers: the prepared batch and one MSM set (each sized for the largest
  // batch / span seen), plus flags (any_bad at [3], cpz_msm's bad point at [2], the combine's
  // decode / identity flags at [0..1]) and the combine's inputs
  RlcPrepared rl_prep;
  RlcMsmSet rl_msm;
  // overlapped spans (rlc_range_launch): the second MSM set, its stream, and the events that
  // start it after the prepare ([0]) and chain the spans' finals ([1 + set])
  RlcMsmSet rl_msm2;
  DevBuf rl_span_ident;  // per span of the last multi-span MSM: its own P is the identity
  hipStream_t span_stream = nullptr;
  hipEvent_t span_ev[3] = {nullptr, nullptr, nullptr};
  DevBuf rl_flags, rl_parts;
  // partitioned batch check (part.hip): sorted lists / offsets / window sums of one chunk of
  // blocks, every block's partial and fail flag, the sum's scratch, the failing-block list
  DevBuf pt_lists, pt_offs, pt_wsum, pt_part, pt_fail, pt_tmp, pt_blocks, pt_assign;
  DevBuf pt_ldig, pt_lsum, pt_lpart, pt_lfail, pt_loc;  // the locate pass over failing blocks
  // what the last batch call's fallback did (cpz_ctx_fallback_stats)
  uint64_t fb_stats[CPZ_FALLBACK_STATS] = {};
  // commitment checks (statuses 4 and 5: the Proof::from_bytes rejections); off = equations only.
  // eq_only is the context's mode (cpz_ctx_set_commitment_checks); call_eq the mode of the call
  // in progress (CallLock: the context's, or equations only for that call alone).
  bool eq_only = false;
  bool call_eq = false;
  // streams this context created on hardware queues of their own (released with it)
  int own_queues = 0;
  // Completion of the last call's work on whatever stream it used: the *_device entry points
  // return without synchronising, and their kernels read context buffers (comb, tab, prefix,
  // c, scratch, RLC buffers) that the next call may rewrite on another stream.
  hipEvent_t last_done = nullptr;
  bool have_last = false;
#if defined(CPZ_CLOCK_PROBE)
  // timing-only builds: the in-kernel clock stamps of the last k_rlc_prepare [0],
  // k_rlc_bucket [1] and k_part_acc [2] launch (cpz_ctx_clock_probe), 5 words per wave
  DevBuf clk[4];
  size_t clk_waves[4] = {0, 0, 0, 0};
#endif
  // optional per-kernel timing
  bool timing = false;
  struct Mark { int stage; hipEvent_t a, b; };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> free_events;
};

namespace {

// One call's hold on the context: its mutex for the whole call, and the call's commitment-check
// mode -- the context's (cpz_ctx_set_commitment_checks), or equations only for this call alone
// (CPZ_CALL_EQUATIONS_ONLY), so callers sharing a context never change each other's mode.
struct CallLock {
  std::lock_guard<std::mutex> hold;
  explicit CallLock(cpz_ctx* ctx, uint32_t flags = 0) : hold(ctx->mu) {
    ctx->call_eq = ctx->eq_only || (flags & CPZ_CALL_EQUATIONS_ONLY) != 0;
  }
};

hipEvent_t take_event(cpz_ctx* ctx) {
  if (!ctx->free_events.empty()) {
    hipEvent_t e = ctx->free_events.back();
    ctx->free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Order the work this call enqueues on `st` after everything the previous call enqueued on
// its stream(s) (which may differ from `st`): the context's buffers are shared by all calls.
int order_after_last(cpz_ctx* ctx, hipStream_t st) {
  if (ctx->have_last) CPZ_HIP(hipStreamWaitEvent(st, ctx->last_done, 0));
  return CPZ_OK;
}

// Mark the end of this call's work on `st` (every aux stream already joined into it).
int record_last(cpz_ctx* ctx, hipStream_t st) {
  if (!ctx->last_done) CPZ_HIP(hipEventCreateWithFlags(&ctx->last_done, hipEventDisableTiming));
  CPZ_HIP(hipEventRecord(ctx->last_done, st));
  ctx->have_last = true;
  return CPZ_OK;
}

// RAII bracket: records events around one kernel launch on `st` when timing is enabled.
struct StageTimer {
  cpz_ctx* ctx;
  int stage;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  StageTimer(cpz_ctx* c, int s, hipStream_t stream) : ctx(c), stage(s), st(stream) {
    if (ctx->timing) {
      a = take_event(ctx);
      b = take_event(ctx);
      if (a) (void)hipEventRecord(a, st);
    }
  }
  ~StageTimer() {
    if (a && b) {
      (void)hipEventRecord(b, st);
      ctx->marks.push_back({stage, a, b});
    }
  }
};

// Build (or reuse) the fixed-base tables and transcript prefix for (g, h).
void words_from_bytes(uint32_t w[16], const uint8_t g[32], const uint8_t h[32]) {
  std::memcpy(w, g, 32);
  std::memcpy(w + 8, h, 32);
}

bool is_default_pair(const uint8_t g[32], const uint8_t h[32]) {
  return std::memcmp(g, kDefaultG, 32) == 0 && std::memcmp(h, kDefaultH, 32) == 0;
}

// The least recently used of sets[0 .. n) (an unused one first).
GenSet* lru_victim(GenSet* sets, int n) {
  GenSet* v = nullptr;
  for (int k = 0; k < n; k++) {
    GenSet& e = sets[k];
    if (!v || (!e.valid && v->valid) || (e.valid == v->valid && e.used < v->used)) v = &e;
  }
  return v;
}

// The Niels tables (g, h at 2^(32 m) times, kNielsLevels levels) and transcript prefix of
// (g, h) into e, and the fixed-schedule masks; CPZ_EGENERATOR if an encoding does not decode.
int build_niels_prefix(cpz_ctx* ctx, GenSet& e, const uint8_t both[64]) {
  // [level][generator]: g, h, 2^128 g, 2^128 h, 2^64 g, 2^64 h, 2^192 g, 2^192 h, 2^32 g, ...
  CPZ_HIP(e.tab.ensure(2 * cpz::kNielsLevels * cpz::kNielsEntries * sizeof(cpz::ge_niels)));
  CPZ_HIP(e.prefix.ensure(2 * sizeof(cpz::StrobeSnap)));
  CPZ_HIP(e.gh_words.ensure(64));
  CPZ_HIP(ctx->ok_flags.ensure(2 * sizeof(int)));
  CPZ_HIP(ctx->gen_bases.ensure(2 * cpz::kNielsLevels * sizeof(cpz::ge_p3)));
  CPZ_HIP(hipMemcpyAsync(e.gh_words.p, both, 64, hipMemcpyHostToDevice, ctx->stream));
  CPZ_HIP(cpz::launch_build_niels(static_cast<const uint32_t*>(e.gh_words.p), 2, static_cast<cpz::ge_niels*>(e.tab.p),
                                  static_cast<int*>(ctx->ok_flags.p), static_cast<cpz::ge_p3*>(ctx->gen_bases.p),
                                  ctx->stream));
  CPZ_HIP(e.tab16.ensure(2 * cpz::kNielsLevels * cpz::kNielsEntries * 48 * sizeof(int32_t)));
  CPZ_HIP(cpz::launch_niels_r16(static_cast<const cpz::ge_niels*>(e.tab.p), static_cast<int32_t*>(e.tab16.p),
                                2 * cpz::kNielsLevels * cpz::kNielsEntries, ctx->stream));
  CPZ_HIP(cpz::launch_transcript_prefix(static_cast<const uint32_t*>(e.gh_words.p),
                                        static_cast<cpz::StrobeSnap*>(e.prefix.p), ctx->stream));
  int ok[2] = {0, 0};
  cpz::StrobeSnap snap[2];
  CPZ_HIP(hipMemcpyAsync(ok, ctx->ok_flags.p, sizeof(ok), hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipMemcpyAsync(snap, e.prefix.p, sizeof(snap), hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  if (!ok[0] || !ok[1]) return fail(CPZ_EGENERATOR, "generator encoding does not decode to a ristretto255 point");
  e.prefix_fixed = cpz::challenge_prefix_is_fixed(snap[1]) && cpz::challenge_masks(e.chal_k1, e.chal_k2);
  uint32_t gw[16];
  std::memcpy(gw, both, 64);
  e.ctx32_fixed = cpz::challenge_prefix_is_ctx32(snap[0]) && cpz::challenge_masks_ctx32(e.chal_c32, gw, gw + 8);
  return CPZ_OK;
}

// Make the tables of (g, h) current.  A cached full set (combs) is reused.  need_comb false (a
// per-proof call of at most var_base_max(ctx) proofs on a pair other than the default one): a cached
// light set is reused, or one is built -- k_build_niels and k_transcript_prefix only, ~0.5 ms
// instead of the combs' ~3 ms, timed as stage 13 -- and the call verifies with variable bases.
// Otherwise the least recently used full set (an unused one first) is rebuilt: k_build_niels,
// k_transcript_prefix and the 128 MiB combs (~3 ms), timed as stage 7.  If the combs do not fit,
// the other full sets are freed and the allocation is tried once more.
int ensure_generators(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], bool need_comb = true) {
  uint8_t both[64];
  std::memcpy(both, g, 32);
  std::memcpy(both + 32, h, 32);
  for (int k = 0; k < ctx->gen_cap; k++) {
    GenSet& e = ctx->gen[k];
    if (e.valid && std::memcmp(e.gh, both, 64) == 0) {
      e.used = ++ctx->gen_clock;
      ctx->gs = &e;
      return CPZ_OK;
    }
  }
  const bool light = !need_comb && !is_default_pair(g, h);
  if (light) {
    for (GenSet& e : ctx->light) {
      if (e.valid && std::memcmp(e.gh, both, 64) == 0) {
        e.used = ++ctx->gen_clock;
        ctx->gs = &e;
        return CPZ_OK;
      }
    }
  }
  // Parameters::with_generators (gadgets.rs:77-103): valid, non-identity, distinct.
  static const uint8_t zero[32] = {0};
  if (std::memcmp(g, zero, 32) == 0 || std::memcmp(h, zero, 32) == 0)
    return fail(CPZ_EGENERATOR, "generator cannot be identity");
  if (std::memcmp(g, h, 32) == 0) return fail(CPZ_EGENERATOR, "generators g and h must be different");
  // a set is about to be rebuilt: no earlier call's kernels may still be reading it
  if (ctx->have_last) CPZ_HIP(hipEventSynchronize(ctx->last_done));
  GenSet& e = light ? *lru_victim(ctx->light, kLightCache) : *lru_victim(ctx->gen, ctx->gen_cap);
  e.valid = false;
  e.full = !light;
  if (ctx->gs == &e) ctx->gs = nullptr;
  StageTimer timer(ctx, light ? 13 : 7, ctx->stream);
  if (int rc = build_niels_prefix(ctx, e, both)) return rc;
  if (!light) {
    const size_t comb_bytes = (size_t)2 * cpz::kCombPerBase * sizeof(cpz::ge_niels);
    if (e.comb.ensure(comb_bytes) != hipSuccess) {
      (void)hipGetLastError();
      for (int k = 0; k < ctx->gen_cap; k++)  // trim: every other full set ...
        if (&ctx->gen[k] != &e) ctx->gen[k].release();
      for (GenSet& l : ctx->light) l.release();  // ... and every light set
      CPZ_HIP(e.comb.ensure(comb_bytes));
    }
    CPZ_HIP(e.comb_q.ensure((size_t)2 * cpz::kCombWindows * sizeof(cpz::ge_p3)));
    CPZ_HIP(cpz::launch_build_comb(static_cast<const uint32_t*>(e.gh_words.p), static_cast<cpz::ge_p3*>(e.comb_q.p),
                                   static_cast<cpz::ge_niels*>(e.comb.p), ctx->stream));
    CPZ_HIP(hipStreamSynchronize(ctx->stream));  // callers may launch on another stream
  }
  std::memcpy(e.gh, both, 64);
  e.valid = true;
  e.used = ++ctx->gen_clock;
  ctx->gs = &e;
  return CPZ_OK;
}

// The fixed-schedule challenge paths and their masks (set per (g, h) by ensure_generators).
void set_challenge_schedules(const cpz_ctx* ctx, cpz::ChallengeArgs& ca) {
  ca.eq_only = ctx->call_eq ? 1 : 0;
  ca.fast_noctx = ctx->gs->prefix_fixed ? 1 : 0;
  std::memcpy(ca.k1, ctx->gs->chal_k1, sizeof(ca.k1));
  std::memcpy(ca.k2, ctx->gs->chal_k2, sizeof(ca.k2));
  ca.fast_ctx32 = ctx->gs->ctx32_fixed ? 1 : 0;
  std::memcpy(ca.c32, ctx->gs->chal_c32, sizeof(ca.c32));
}

// Resident k_verify_each blocks on the whole chip (occupancy-limited).
int occupancy_grid(const cpz_ctx* ctx) { return ctx->cus * ctx->verify_blocks_per_cu; }

int verify_grid(cpz_ctx* ctx, size_t n) {
  const size_t want = (n + cpz::kVerifyBlock - 1) / cpz::kVerifyBlock;
  const size_t cap = (size_t)occupancy_grid(ctx);
  return (int)(want < cap ? want : cap);
}

// k_verify_each over va.n proofs as launches of one proof per thread: the grid is the
// occupancy-limited size (verify_grid), so a batch larger than grid * kVerifyBlock proofs is
// cut into that many proofs per launch rather than looping inside one launch.  Measured on
// MI355X at 2^20 proofs: 8 launches of 2^17 take 19.96 ms, one grid-stride launch 21.59 ms
// (tools/chunk_probe.py).  (Not an instruction-cache effect: a 3x smaller kernel measured
// the same.)
//
// The chunks go round-robin to CPZ_VERIFY_STREAMS streams (each with its own scratch slab),
// and a chunk is 1 / CPZ_VERIFY_CHUNK_DIV of the occupancy grid, so several launches are in
// flight and one launch's tail (waves finishing at different times) overlaps the next
// launch's start.  A/B on one box (tools/variants.sh, 2^20 proofs): 1 stream / full grid
// 49.5 M proofs/s, 2 / full 51.7 M, 3 / full 51.4 M, 4 / full 51.4 M, 2 / half 52.1 M,
// 4 / half 51.5 M, 3 / third 47.3 M, 4 / quarter 48.8 M.
// Challenges per verify chunk on the chunk's stream (hidden under the other stream's verify
// work; +0.5-1.1 % A/B on one box against one up-front challenge launch).
#ifndef CPZ_VERIFY_STREAMS
#define CPZ_VERIFY_STREAMS 2
#endif
// Launches of at most kSmallMax proofs (without prepared points or block lists) take
// k_verify_small: three waves per 8 proofs, the transcript challenge computed inside.
#ifndef CPZ_VERIFY_SMALL
#define CPZ_VERIFY_SMALL 1
#endif
#ifndef CPZ_SMALL_MAX
#define CPZ_SMALL_MAX 2048
#endif
constexpr int64_t kSmallMax = CPZ_SMALL_MAX;
// Launches of at most wide_max() proofs (default CPZ_WIDE_MAX, environment CPZ_WIDE_MAX for
// measurement) take k_verify_wide: a workgroup of six waves per proof (eight with a light set's
// variable-base generators), field products on 16-lane rows -- the shortest chain for a few
// proofs.  Light-set calls take it too (its variable-base waves read VerifyArgs::vtab16).
#ifndef CPZ_WIDE_MAX
#define CPZ_WIDE_MAX 512
#endif
// Synchronous host-buffer calls of at most kSmallMax proofs read their page-locked inputs and
// write their statuses in place (PinnedBuf::dp) instead of copying both ways on the stream;
// CPZ_ZERO_COPY=0 restores the copies.
bool zero_copy() {
  static const bool v = [] {
    const char* e = std::getenv("CPZ_ZERO_COPY");
    return !(e && e[0] == '0');
  }();
  return v;
}
int64_t wide_max() {
  static const int64_t v = [] {
    const char* e = std::getenv("CPZ_WIDE_MAX");
    return e ? (int64_t)std::atoll(e) : (int64_t)CPZ_WIDE_MAX;
  }();
  return v;
}
#ifndef CPZ_VERIFY_CHUNK_DIV
#define CPZ_VERIFY_CHUNK_DIV 2
#endif
// Blocks per verify launch (half the occupancy grid) and the bytes of one verify stream's table
// slab, which every stream owns at a fixed offset whatever a call's grid.
int verify_full_grid(const cpz_ctx* ctx) {
  return (occupancy_grid(ctx) + CPZ_VERIFY_CHUNK_DIV - 1) / CPZ_VERIFY_CHUNK_DIV;
}
size_t verify_slab_bytes(const cpz_ctx* ctx) {
  return (size_t)verify_full_grid(ctx) * cpz::kVerifyBlock * cpz::kCachedEntries * sizeof(cpz::ge_cached);
}
// Launches of at most this many proofs take the eight-lane kernel (k_verify_quad): kQuadVerifyMax,
// bounded by the tables one slab holds -- full * 128 proofs, which depends on the device's CUs
// (16384 on the 256-CU MI355X, 14080 on a 110-CU part).
int64_t verify_quad_max(const cpz_ctx* ctx) {
  return std::min<int64_t>(cpz::kQuadVerifyMax, (int64_t)(verify_slab_bytes(ctx) / cpz::kQuadProofScratch));
}
// Per-proof calls of at most this many proofs on a pair without cached combs verify with
// variable bases (light sets), which only the eight-lane and latency kernels support: the same
// bound as verify_quad_max, so a light-set call never reaches k_verify_each.
int64_t var_base_max(const cpz_ctx* ctx) { return std::min<int64_t>(cpz::kVarBaseMax, verify_quad_max(ctx)); }
// Round-robin position of the verify launches of one call that enqueues several batches
// (the host-buffer pipeline): launches keep alternating streams across batches, and the
// streams are joined once at the end.
struct VerifyRR {
  int64_t next = 0;
};

int join_verify_streams(cpz_ctx* ctx, hipStream_t st) {
  for (int k = 0; k < CPZ_VERIFY_STREAMS - 1; k++) {
    if (!ctx->aux_stream[k]) continue;
    CPZ_HIP(hipEventRecord(ctx->aux_done[k], ctx->aux_stream[k]));
    CPZ_HIP(hipStreamWaitEvent(st, ctx->aux_done[k], 0));
  }
  return CPZ_OK;
}

// ca != nullptr: each chunk's challenges are computed on the chunk's own stream right before
// its verify launch (so they overlap the other stream's verify work) instead of up front.
int launch_verify_chunks(cpz_ctx* ctx, const cpz::VerifyArgs& va, int stage, hipStream_t st, VerifyRR* rr,
                         bool join, const cpz::ChallengeArgs* ca = nullptr) {
  static_assert(CPZ_VERIFY_STREAMS >= 1 && CPZ_VERIFY_STREAMS <= 4, "1..4 verify streams");
  const int full = verify_full_grid(ctx);
  const int grid = std::min(full, verify_grid(ctx, (size_t)va.n));
  // every stream owns a full-size slab at a fixed offset, whatever this call's grid
  const size_t slab = verify_slab_bytes(ctx);
  const int64_t per = (int64_t)grid * cpz::kVerifyBlock;
  const int64_t chunks = (va.n + per - 1) / per;
  const int nst = rr ? CPZ_VERIFY_STREAMS : (int)std::min<int64_t>(CPZ_VERIFY_STREAMS, chunks);
  CPZ_HIP(ctx->scratch.ensure((size_t)CPZ_VERIFY_STREAMS * slab));
  if (nst > 1) {
    if (!ctx->aux_start) CPZ_HIP(hipEventCreateWithFlags(&ctx->aux_start, hipEventDisableTiming));
    CPZ_HIP(hipEventRecord(ctx->aux_start, st));  // the aux streams start after st's prior work
    for (int k = 0; k < nst - 1; k++) {
      if (!ctx->aux_stream[k]) CPZ_HIP(stream_own_queue(&ctx->aux_stream[k], ctx->cus, ctx->device, &ctx->own_queues));
      if (!ctx->aux_done[k]) CPZ_HIP(hipEventCreateWithFlags(&ctx->aux_done[k], hipEventDisableTiming));
      CPZ_HIP(hipStreamWaitEvent(ctx->aux_stream[k], ctx->aux_start, 0));
    }
  }
  for (int64_t c = 0; c < chunks; c++) {
    const int64_t a = c * per;
    cpz::VerifyArgs v = va;
    v.n = (va.n - a) < per ? (va.n - a) : per;
    v.y1 = va.y1 + 8 * a;
    v.y2 = va.y2 + 8 * a;
    v.r1 = va.r1 + 8 * a;
    v.r2 = va.r2 + 8 * a;
    v.s = va.s + 8 * a;
    v.c = va.c + 8 * a;
    if (va.pre) v.pre = va.pre + 4 * a;
    v.status = va.status + a;
    v.quad_max = verify_quad_max(ctx);
#if defined(CPZ_CLOCK_PROBE)
    CPZ_HIP(ctx->clk[3].ensure(cpz::kSmallStamps * sizeof(uint64_t)));
    ctx->clk_waves[3] = 1;
    v.clock_probe = static_cast<uint64_t*>(ctx->clk[3].p);
#endif
    const int k = (int)((rr ? rr->next++ : c) % nst);  // stream k owns scratch slab k
    v.scratch = static_cast<char*>(ctx->scratch.p) + (size_t)k * slab;
    hipStream_t sc = k == 0 ? st : ctx->aux_stream[k - 1];
    if (CPZ_VERIFY_SMALL && v.n <= kSmallMax && !v.pre && !v.blocks && (!ca || !ca->ctx_end)) {
      // the drop-in's regime: three waves per 8 proofs, the challenge inside (k_verify_small)
      cpz::ChallengeArgs cc{};
      if (ca) {
        cc = *ca;
        cc.n = v.n;
        if (ca->ctx_off) cc.ctx_off = ca->ctx_off + a;
        if (ca->ctx_present) cc.ctx_present = ca->ctx_present + a;
        v.c = nullptr;  // computed in the kernel
      }
      StageTimer t(ctx, stage, sc);
      if (v.n <= wide_max())  // a light set always carries vtab16 beside vtab (build_niels_prefix)
        CPZ_HIP(cpz::launch_verify_wide(v, cc, sc));
      else
        CPZ_HIP(cpz::launch_verify_small(v, cc, sc));
      continue;
    }
    if (ca) {
      cpz::ChallengeArgs cc = *ca;
      cc.n = v.n;
      cc.y1 = v.y1;
      cc.y2 = v.y2;
      cc.r1 = v.r1;
      cc.r2 = v.r2;
      cc.s = v.s;
      cc.c_out = ca->c_out + 8 * a;
      cc.status_out = ca->status_out + a;
      if (ca->ctx_off) cc.ctx_off = ca->ctx_off + a;  // absolute offsets into ctx_bytes
      if (ca->ctx_end) cc.ctx_end = ca->ctx_end + a;
      if (ca->ctx_present) cc.ctx_present = ca->ctx_present + a;
      StageTimer tc(ctx, 0, sc);
      CPZ_HIP(cpz::launch_challenge(cc, sc));
    }
    StageTimer t(ctx, stage, sc);
    CPZ_HIP(cpz::launch_verify_each(v, grid, sc));
  }
  if (join && nst > 1) return join_verify_streams(ctx, st);
  return CPZ_OK;
}

// Challenge + verify of n proofs on `st`.  c_buf: where k_challenge writes the challenges
// (default: the context's buffer from offset 0) -- launches of at most kSmallMax proofs compute
// them inside k_verify_small / k_verify_wide and leave c_buf unwritten, so no caller may read
// challenges back from it; rr / join: see VerifyRR; ctx_end: see ChallengeArgs.
int enqueue_verify(cpz_ctx* ctx, size_t n, const void* y1, const void* y2, const void* r1, const void* r2,
                   const void* s, const void* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                   uint8_t* status, hipStream_t st, uint32_t* c_buf = nullptr, VerifyRR* rr = nullptr,
                   bool join = true, const uint64_t* ctx_end = nullptr) {
  if (!c_buf) {
    CPZ_HIP(ctx->c.ensure(n * 32));
    c_buf = static_cast<uint32_t*>(ctx->c.p);
  }
  cpz::ChallengeArgs ca;
  set_challenge_schedules(ctx, ca);
  ca.n = (int64_t)n;
  words_from_bytes(ca.gh_words, ctx->gs->gh, ctx->gs->gh + 32);
  ca.y1 = static_cast<const uint32_t*>(y1);
  ca.y2 = static_cast<const uint32_t*>(y2);
  ca.r1 = static_cast<const uint32_t*>(r1);
  ca.r2 = static_cast<const uint32_t*>(r2);
  ca.s = static_cast<const uint32_t*>(s);
  ca.ctx_bytes = static_cast<const uint8_t*>(ctx_bytes);
  ca.ctx_off = ctx_off;
  ca.ctx_present = ctx_present;
  ca.ctx_end = ctx_end;
  ca.prefix = static_cast<const cpz::StrobeSnap*>(ctx->gs->prefix.p);
  ca.c_out = c_buf;
  ca.status_out = status;
  cpz::VerifyArgs va;
  va.n = (int64_t)n;
  va.y1 = ca.y1;
  va.y2 = ca.y2;
  va.r1 = ca.r1;
  va.r2 = ca.r2;
  va.s = ca.s;
  va.c = ca.c_out;
  va.status = status;
  va.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
  if (!ctx->gs->full) {  // a light set: variable-base generators (ensure_generators, n <= var_base_max)
    if ((int64_t)n > var_base_max(ctx)) return fail(CPZ_EINVAL, "internal: variable-base call above var_base_max");
    va.comb = nullptr;
    va.vtab = static_cast<const cpz::ge_niels*>(ctx->gs->tab.p);
    va.vtab16 = static_cast<const int32_t*>(ctx->gs->tab16.p);
  }
  va.scratch = nullptr;  // set per launch
  va.eq_only = ca.eq_only;
  StageTimer span(ctx, 5, st);  // all chunks, all streams (the launches overlap)
  return launch_verify_chunks(ctx, va, 1, st, rr, join, &ca);
}

// Stage host inputs on the device.  Returns device pointers through out[].
// Host-buffer calls of up to kPinStageMax input bytes: the rows (and transcript contexts) are
// packed into page-locked memory and sent with one copy.  A BatchVerifier-sized call made five
// to eight pageable copies, ~10 us of host round trip each (rocprofv3 timeline, n = 10).
constexpr size_t kPinMail = 256;                  // mailbox bytes at the start of ctx->pin
constexpr size_t kPinStageMax = size_t(8) << 20;  // larger inputs: one pageable copy per row
inline size_t pad16(size_t x) { return (x + 15) & ~size_t(15); }

// direct (a small synchronous call, zero_copy()): the kernels read the page-locked block
// itself through its device view -- no copy on the stream -- and *status_dev / *status_host
// point at n status bytes after it, which the kernels write the same way.
int stage_inputs(cpz_ctx* ctx, size_t n, const uint8_t* const host[5], int count, const uint8_t* ctx_bytes,
                 const uint64_t* ctx_off, const uint8_t* ctx_present, const void* dev[5], const void** dcb,
                 const uint64_t** dco, const uint8_t** dcp, bool direct = false, uint8_t** status_dev = nullptr,
                 uint8_t** status_host = nullptr) {
  if (status_dev) *status_dev = nullptr;
  if (ctx_off)
    for (size_t i = 0; i < n; i++)
      if (ctx_off[i + 1] < ctx_off[i]) return fail(CPZ_EINVAL, "ctx_off must be non-decreasing");
  const size_t nbytes = ctx_off ? (size_t)(ctx_off[n] - ctx_off[0]) : 0;
  const size_t rows = (size_t)count * n * 32;
  const size_t o_off = rows, o_pres = pad16(o_off + (ctx_off ? (n + 1) * 8 : 0));
  const size_t o_ctx = pad16(o_pres + (ctx_off && ctx_present ? n : 0));
  const size_t total = pad16(o_ctx + (ctx_off ? std::max<size_t>(nbytes, 1) : 0));
  // no copy of an earlier call may still read the block when it is rewritten or regrown
  // (host-buffer calls return synchronised; this covers one that failed part-way)
  if (total <= kPinStageMax) CPZ_HIP(hipStreamSynchronize(ctx->stream));
  if (total <= kPinStageMax && ctx->pin.ensure(kPinMail + total + pad16(n)) == hipSuccess &&
      ctx->in_all.ensure(total) == hipSuccess) {
    uint8_t* h = static_cast<uint8_t*>(ctx->pin.p) + kPinMail;
    for (int k = 0; k < count; k++) std::memcpy(h + (size_t)k * n * 32, host[k], n * 32);
    if (ctx_off) {
      uint64_t* rel = reinterpret_cast<uint64_t*>(h + o_off);
      for (size_t i = 0; i <= n; i++) rel[i] = ctx_off[i] - ctx_off[0];
      if (ctx_present) std::memcpy(h + o_pres, ctx_present, n);
      if (nbytes) std::memcpy(h + o_ctx, ctx_bytes + ctx_off[0], nbytes);
    }
    uint8_t* d = static_cast<uint8_t*>(ctx->in_all.p);
    if (direct && status_dev && status_host && ctx->pin.dp) {
      d = static_cast<uint8_t*>(ctx->pin.dp) + kPinMail;
      *status_dev = d + total;
      *status_host = h + total;
    } else if (total) {
      CPZ_HIP(hipMemcpyAsync(ctx->in_all.p, h, total, hipMemcpyHostToDevice, ctx->stream));
    }
    for (int k = 0; k < count; k++) dev[k] = d + (size_t)k * n * 32;
    *dcb = ctx_off ? d + o_ctx : nullptr;
    *dco = ctx_off ? reinterpret_cast<const uint64_t*>(d + o_off) : nullptr;
    *dcp = ctx_off && ctx_present ? d + o_pres : nullptr;
    return CPZ_OK;
  }
  (void)hipGetLastError();
  for (int k = 0; k < count; k++) {
    CPZ_HIP(ctx->in[k].ensure(n * 32));
    CPZ_HIP(hipMemcpyAsync(ctx->in[k].p, host[k], n * 32, hipMemcpyHostToDevice, ctx->stream));
    dev[k] = ctx->in[k].p;
  }
  *dcb = nullptr;
  *dco = nullptr;
  *dcp = nullptr;
  if (ctx_off) {
    std::vector<uint64_t> rel(n + 1);
    for (size_t i = 0; i <= n; i++) rel[i] = ctx_off[i] - ctx_off[0];
    CPZ_HIP(ctx->ctxb.ensure(nbytes ? nbytes : 1));
    CPZ_HIP(ctx->ctxo.ensure((n + 1) * sizeof(uint64_t)));
    if (nbytes)
      CPZ_HIP(hipMemcpyAsync(ctx->ctxb.p, ctx_bytes + ctx_off[0], nbytes, hipMemcpyHostToDevice, ctx->stream));
    CPZ_HIP(hipMemcpyAsync(ctx->ctxo.p, rel.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    // The copies above read pageable host memory synchronously, so rel may be freed.
    CPZ_HIP(hipStreamSynchronize(ctx->stream));
    *dcb = ctx->ctxb.p;
    *dco = static_cast<const uint64_t*>(ctx->ctxo.p);
    if (ctx_present) {
      CPZ_HIP(ctx->ctxp.ensure(n));
      CPZ_HIP(hipMemcpyAsync(ctx->ctxp.p, ctx_present, n, hipMemcpyHostToDevice, ctx->stream));
      *dcp = static_cast<const uint8_t*>(ctx->ctxp.p);
    }
  }
  return CPZ_OK;
}

// ---- RLC batch path --------------------------------------------------------------------
// digits row stride: 4 points per proof + g, h, rounded to 8 so that every window row starts
// 16-byte aligned (k_rlc_hist reads 8 digits per load)
// digit rows: 4 cap points + two MSM sets' extra points (g, h) each (kRlcExtraSlots)
constexpr int64_t kRlcExtraSlots = 4;
int64_t rlc_dstride(int64_t cap) { return (4 * cap + kRlcExtraSlots + 7) & ~(int64_t)7; }
// sorted-entry row stride: whole 4096-entry groups
int64_t rlc_istride(int64_t cap) { return (4 * cap + 2 + 4095) & ~(int64_t)4095; }
// bucket-head slots per window: one per k_rlc_bucket thread of any MSM the set can hold
// (rlc_sort_geometry: ceil(points / echunk) <= max(points / kRlcChunk, kRlcMinHeads))
int64_t rlc_hstride(int64_t cap) {
  return std::max<int64_t>((rlc_istride(cap) + cpz::kRlcChunk - 1) / cpz::kRlcChunk, cpz::kRlcMinHeads);
}

// The prepared set for a batch of n proofs.
int rlc_reserve_prepared(RlcPrepared& P, int64_t n) {
  if (n <= P.cap) return CPZ_OK;
  const int64_t npts = 4 * n + kRlcExtraSlots;
  const int64_t nblk = (n + cpz::kRlcPrepBlock - 1) / cpz::kRlcPrepBlock;
  P.cap = 0;  // stays 0 unless every buffer is in place
  CPZ_HIP(P.pts.ensure((size_t)npts * sizeof(cpz::ge_niels)));
  CPZ_HIP(P.dig.ensure((size_t)rlc_dstride(n) * cpz::kRlcWindows * sizeof(int16_t)));
  CPZ_HIP(P.bsum.ensure((size_t)nblk * 2 * 2 * sizeof(cpz::sc)));  // two sum blocks per prepare block
  CPZ_HIP(P.qsum.ensure((size_t)((std::min(n, cpz::kRlcPrepWideMax) + 63) / 64) * 2 * sizeof(cpz::sc)));
  P.cap = n;
  return CPZ_OK;
}

// An MSM set for MSMs over at most `span` proofs (4 span + 2 points).
int rlc_reserve_msm(RlcMsmSet& S, int64_t span) {
  if (span <= S.cap) return CPZ_OK;
  S.cap = 0;
  CPZ_HIP(S.counts.ensure(sizeof(uint32_t) * cpz::kRlcWindows * cpz::kRlcBuckets));
  CPZ_HIP(S.offsets.ensure(sizeof(uint32_t) * cpz::kRlcWindows * (cpz::kRlcBuckets + 1)));
  CPZ_HIP(S.bhist.ensure(sizeof(uint32_t) * cpz::kRlcWindows * cpz::kRlcSortGroups * cpz::kRlcBuckets));
  CPZ_HIP(S.idx.ensure((size_t)rlc_istride(span) * cpz::kRlcWindows * sizeof(uint32_t)));
  CPZ_HIP(S.inter.ensure((size_t)rlc_istride(span) * cpz::kRlcWindows * sizeof(uint32_t)));
  CPZ_HIP(S.buckets.ensure(sizeof(cpz::ge_p3) * cpz::kRlcWindows * cpz::kRlcBuckets));
  CPZ_HIP(S.heads.ensure(sizeof(cpz::ge_p3) * cpz::kRlcWindows * (size_t)rlc_hstride(span)));
  const size_t nseg = (size_t)cpz::kRlcWindows * (cpz::kRlcBuckets / cpz::kRlcSegLen);
  CPZ_HIP(S.segs.ensure(sizeof(cpz::ge_p3) * nseg));
  CPZ_HIP(S.segw.ensure(sizeof(cpz::ge_p3) * nseg));
  CPZ_HIP(S.win.ensure(sizeof(cpz::ge_p3) * cpz::kRlcWindows));
  CPZ_HIP(S.total.ensure(sizeof(cpz::ge_p3)));
  CPZ_HIP(S.partial.ensure(64));
  CPZ_HIP(S.flags.ensure(4 * sizeof(int)));
  S.cap = span;
  return CPZ_OK;
}

// Proofs per MSM: the points of a span (1 GiB) stay gather-friendly.
#ifndef CPZ_RLC_SPAN
#define CPZ_RLC_SPAN (1 << 21)
#endif

// Both sets for a batch of n proofs (the MSM set for one span of it).
int rlc_reserve(cpz_ctx* ctx, int64_t n) {
  int rc = rlc_reserve_prepared(ctx->rl_prep, n);
  if (rc) return rc;
  if ((rc = rlc_reserve_msm(ctx->rl_msm, std::min<int64_t>(n, CPZ_RLC_SPAN)))) return rc;
  CPZ_HIP(ctx->rl_flags.ensure(4 * sizeof(int)));
  return CPZ_OK;
}

// Arguments of the MSM over proofs [lo, hi) of the prepared set P, sorted / accumulated /
// reduced in the MSM set S.  Every stride and extra-point position comes from the set that
// owns the buffer: the prepared points' extras (g, h) sit at 4 P.cap, the digit rows have
// P's stride; the sorted-entry rows and bucket heads have S's strides.  (Round 2's attempt
// at a second, span-sized MSM set for overlapping spans took all of them from the prepared
// capacity, so a second set smaller than the batch was indexed with the batch's row stride:
// windows 1..15 of its sorted ids and heads fell outside the set -- the identity partials
// seen for every span that used it.  Fails with CPZ_EINVAL instead of misaddressing.)
int rlc_msm_args(const RlcPrepared& P, RlcMsmSet& S, int64_t lo, int64_t hi, cpz::RlcMsmArgs& m) {
  if (lo < 0 || hi < lo || hi > P.cap) return fail(CPZ_EINVAL, "MSM range outside the prepared set");
  if (hi - lo > S.cap) return fail(CPZ_EINVAL, "MSM range larger than its MSM set");
  m.p0 = 4 * lo;
  m.p1 = 4 * hi;
  m.e0 = 4 * P.cap;
  m.pts = static_cast<cpz::ge_niels*>(P.pts.p);
  m.digits = static_cast<int16_t*>(P.dig.p);
  m.dstride = rlc_dstride(P.cap);
  m.counts = static_cast<uint32_t*>(S.counts.p);
  m.offsets = static_cast<uint32_t*>(S.offsets.p);
  m.bhist = static_cast<uint32_t*>(S.bhist.p);
  cpz::rlc_sort_geometry(m, (m.p1 - m.p0) + 2);
  m.idx = static_cast<uint32_t*>(S.idx.p);
  m.inter = static_cast<uint32_t*>(S.inter.p);
  m.istride = rlc_istride(S.cap);
  m.buckets = static_cast<cpz::ge_p3*>(S.buckets.p);
  m.heads = static_cast<cpz::ge_p3*>(S.heads.p);
  m.hstride = rlc_hstride(S.cap);
  m.seg_s = static_cast<cpz::ge_p3*>(S.segs.p);
  m.seg_w = static_cast<cpz::ge_p3*>(S.segw.p);
  m.win = static_cast<cpz::ge_p3*>(S.win.p);
  m.partial_out = static_cast<uint32_t*>(S.partial.p);
  m.identity_out = static_cast<int*>(S.flags.p);
  return CPZ_OK;
}

// P over proofs [lo, hi) (lo a multiple of kRlcPrepBlock) of the prepared batch: one MSM per
// span of CPZ_RLC_SPAN proofs (aligned to the weight blocks), each span's P added on the
// device (RlcMsmArgs::total).  Random 128-byte gathers run at ~7 TB/s over a 512 MiB array
// but ~1.8 TB/s over 4 GiB (translation misses, tools/ubench/gather_bytes.hip), so a
// 2^26-proof MSM over one 32 GiB points array spent 2.8x the per-entry bucket time of a 2^20
// one.
//
// Several spans overlap (span_overlap(), default on): consecutive spans alternate between two
// MSM sets and two streams, so one span's latency-bound sort and tails run beside the other's
// VALU-bound bucket accumulation.  The only state the spans share is the running total, and
// the finals that own it are chained by events (launch_rlc_msm's final_wait / final_done);
// each set's two extra points (g, h with the span's summed scalars) have their own slots in
// the prepared set (e0 = 4 cap + 2 set).  The last span runs on set 0 and `st`, which waits
// for the other stream through that chain, so the readers of rl_msm (rlc_range and the
// fallbacks) and the order of later work on `st` are unchanged.  Synchronises nothing.
bool span_overlap() {
  static const bool v = [] {
    const char* e = std::getenv("CPZ_RLC_SPAN_OVERLAP");
    return !(e && e[0] == '0');
  }();
  return v;
}

int rlc_range_launch(cpz_ctx* ctx, int64_t lo, int64_t hi, hipStream_t st) {
  static_assert(CPZ_RLC_SPAN % cpz::kRlcPrepBlock == 0, "spans are whole weight blocks");
  static_assert(cpz::kRlcPrepBlock % cpz::kRlcSumBlock == 0, "ranges are whole block sums");
  static_assert(4ll * CPZ_RLC_SPAN + 2 <= cpz::kRlcMaxMsmPoints, "a span's MSM exceeds the sort-entry format");
  const int64_t nspan = (hi - lo + CPZ_RLC_SPAN - 1) / CPZ_RLC_SPAN;
#if defined(CPZ_CLOCK_PROBE)
  bool overlap = false;  // timing-only builds: one clock-probe buffer, spans in order
#else
  bool overlap = nspan > 1 && span_overlap();
#endif
  // the second MSM set (~1 GB for 2^21-proof spans): without room for it the spans run in order
  if (overlap && rlc_reserve_msm(ctx->rl_msm2, std::min<int64_t>(hi - lo, CPZ_RLC_SPAN)) != CPZ_OK) {
    ctx->rl_msm2.release();
    (void)hipGetLastError();
    overlap = false;
  }
  hipStream_t sts[2] = {st, st};
  if (overlap) {
    if (!ctx->span_stream) CPZ_HIP(stream_own_queue(&ctx->span_stream, ctx->cus, ctx->device, &ctx->own_queues));
    for (auto& e : ctx->span_ev)
      if (!e) CPZ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CPZ_HIP(hipEventRecord(ctx->span_ev[0], st));  // the second stream starts after st's prior work
    CPZ_HIP(hipStreamWaitEvent(ctx->span_stream, ctx->span_ev[0], 0));
    sts[1] = ctx->span_stream;
  }
  for (int64_t j = 0; j < nspan; j++) {
    const int64_t slo = lo + j * CPZ_RLC_SPAN, shi = std::min<int64_t>(hi, slo + CPZ_RLC_SPAN);
    const int set = overlap ? (int)((nspan - 1 - j) & 1) : 0;  // the last span on set 0 / st
    RlcMsmSet& S = set ? ctx->rl_msm2 : ctx->rl_msm;
    hipStream_t ss = sts[set];
    cpz::RlcMsmArgs m;
    if (int rc = rlc_msm_args(ctx->rl_prep, S, slo, shi, m)) return rc;
    m.e0 = 4 * ctx->rl_prep.cap + 2 * set;
    if (nspan > 1) {
      if (j == 0) CPZ_HIP(ctx->rl_span_ident.ensure((size_t)nspan * sizeof(int)));
      m.span_identity = static_cast<int*>(ctx->rl_span_ident.p) + j;
      m.total = static_cast<cpz::ge_p3*>(ctx->rl_msm.total.p);  // one running total for both sets
      m.total_first = j == 0;
      m.total_last = j == nspan - 1;
    }
    const int64_t b0 = slo / cpz::kRlcSumBlock;
    const int64_t b1 = (shi + cpz::kRlcSumBlock - 1) / cpz::kRlcSumBlock;
#if defined(CPZ_CLOCK_PROBE)
    {  // k_rlc_bucket's grid: (ceil(chunks / 256), 16) blocks of 4 waves (launch_rlc_msm)
      const int64_t chunks = ((m.p1 - m.p0) + 2 + m.echunk - 1) / m.echunk;
      ctx->clk_waves[1] = (size_t)((chunks + 255) / 256) * cpz::kRlcWindows * 4;
      CPZ_HIP(ctx->clk[1].ensure(ctx->clk_waves[1] * 40));
      CPZ_HIP(hipMemsetAsync(ctx->clk[1].p, 0, ctx->clk_waves[1] * 40, ss));
      m.clock_probe = static_cast<uint64_t*>(ctx->clk[1].p);
    }
#endif
    StageTimer t(ctx, 3, ss);
    // phase marks (stages 8-12) when timing: sort, bucket, bucket fix, segment + window, final
    hipEvent_t marks[cpz::kRlcMsmMarks];
    bool timed = ctx->timing;
    int got = 0;
    for (; got < cpz::kRlcMsmMarks && timed; got++) timed = (marks[got] = take_event(ctx)) != nullptr;
    if (!timed)
      for (int k = 0; k < got; k++)
        if (marks[k]) ctx->free_events.push_back(marks[k]);
    // overlapped: the final waits for the previous span's (the other set's event) and records its own
    hipEvent_t fwait = overlap && j > 0 ? ctx->span_ev[1 + (1 - set)] : nullptr;
    hipEvent_t fdone = overlap && j + 1 < nspan ? ctx->span_ev[1 + set] : nullptr;
    CPZ_HIP(cpz::launch_rlc_msm(m, static_cast<const cpz::sc*>(ctx->rl_prep.bsum.p), b0, b1,
                                static_cast<const cpz::ge_niels*>(ctx->gs->tab.p), ss, timed ? marks : nullptr,
                                fwait, fdone));
    if (timed)
      for (int k = 0; k + 1 < cpz::kRlcMsmMarks; k++) ctx->marks.push_back({8 + k, marks[k], marks[k + 1]});
  }
  return CPZ_OK;
}

// rlc_range_launch, then the partial and identity flag read back (synchronises).
int rlc_range(cpz_ctx* ctx, int64_t lo, int64_t hi, hipStream_t st, uint8_t partial[32], int* identity) {
  if (int rc = rlc_range_launch(ctx, lo, hi, st)) return rc;
  RlcMsmSet& S = ctx->rl_msm;
  int flags[1];
  CPZ_HIP(hipMemcpyAsync(partial, S.partial.p, 32, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(flags, S.flags.p, sizeof(int), hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipStreamSynchronize(st));
  *identity = flags[0];
  return CPZ_OK;
}

// Challenges of the whole batch into ctx->c, response statuses into `status`.
int batch_challenges(cpz_ctx* ctx, size_t n, const void* y1, const void* y2, const void* r1, const void* r2,
                     const void* s, const void* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                     uint8_t* status, hipStream_t st) {
  CPZ_HIP(ctx->c.ensure(n * 32));
  cpz::ChallengeArgs ca;
  set_challenge_schedules(ctx, ca);
  ca.n = (int64_t)n;
  words_from_bytes(ca.gh_words, ctx->gs->gh, ctx->gs->gh + 32);
  ca.y1 = static_cast<const uint32_t*>(y1);
  ca.y2 = static_cast<const uint32_t*>(y2);
  ca.r1 = static_cast<const uint32_t*>(r1);
  ca.r2 = static_cast<const uint32_t*>(r2);
  ca.s = static_cast<const uint32_t*>(s);
  ca.ctx_bytes = static_cast<const uint8_t*>(ctx_bytes);
  ca.ctx_off = ctx_off;
  ca.ctx_present = ctx_present;
  ca.prefix = static_cast<const cpz::StrobeSnap*>(ctx->gs->prefix.p);
  ca.c_out = static_cast<uint32_t*>(ctx->c.p);
  ca.status_out = status;
  StageTimer t(ctx, 0, st);
  CPZ_HIP(cpz::launch_challenge(ca, st));
  return CPZ_OK;
}

// Decode + weights + points/digits of the whole batch (after batch_challenges).
// need_msm = false (the partitioned check): the span-sized MSM set is not reserved.
int rlc_prepare_points(cpz_ctx* ctx, size_t n, const void* y1, const void* y2, const void* r1, const void* r2,
                       const void* s, uint8_t* status, const uint8_t seed[32], uint64_t first_index, hipStream_t st,
                       bool need_msm = true) {
  int rc = need_msm ? rlc_reserve(ctx, (int64_t)n) : rlc_reserve_prepared(ctx->rl_prep, (int64_t)n);
  if (rc) return rc;
  CPZ_HIP(ctx->rl_flags.ensure(4 * sizeof(int)));
  cpz::RlcPrepArgs pa;
  pa.n = (int64_t)n;
  pa.first_index = first_index;
  std::memcpy(pa.seed, seed, 32);
  pa.y1 = static_cast<const uint32_t*>(y1);
  pa.y2 = static_cast<const uint32_t*>(y2);
  pa.r1 = static_cast<const uint32_t*>(r1);
  pa.r2 = static_cast<const uint32_t*>(r2);
  pa.s = static_cast<const uint32_t*>(s);
  pa.c = static_cast<const uint32_t*>(ctx->c.p);
  pa.status = status;
  pa.pts = static_cast<cpz::ge_niels*>(ctx->rl_prep.pts.p);
  pa.digits = static_cast<int16_t*>(ctx->rl_prep.dig.p);
  pa.dstride = rlc_dstride(ctx->rl_prep.cap);
  pa.block_sums = static_cast<cpz::sc*>(ctx->rl_prep.bsum.p);
  pa.quarter_sums = static_cast<cpz::sc*>(ctx->rl_prep.qsum.p);
  pa.eq_only = ctx->call_eq ? 1 : 0;
  pa.any_bad = static_cast<int*>(ctx->rl_flags.p) + 3;
  CPZ_HIP(hipMemsetAsync(pa.any_bad, 0, sizeof(int), st));
#if defined(CPZ_CLOCK_PROBE)
  ctx->clk_waves[0] = (size_t)((n + cpz::kRlcPrepBlock - 1) / cpz::kRlcPrepBlock) * (cpz::kRlcPrepBlock / 64);
  CPZ_HIP(ctx->clk[0].ensure(ctx->clk_waves[0] * 40));
  CPZ_HIP(hipMemsetAsync(ctx->clk[0].p, 0, ctx->clk_waves[0] * 40, st));
  pa.clock_probe = static_cast<uint64_t*>(ctx->clk[0].p);
#endif
  {
    StageTimer t(ctx, 2, st);
    CPZ_HIP(cpz::launch_rlc_prepare(pa, st));
  }
  return CPZ_OK;
}

// Prepare (challenge + decode + weights + points/digits) for the whole batch.
int rlc_prepare(cpz_ctx* ctx, size_t n, const void* y1, const void* y2, const void* r1, const void* r2,
                const void* s, const void* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                uint8_t* status, const uint8_t seed[32], uint64_t first_index, hipStream_t st) {
  int rc = batch_challenges(ctx, n, y1, y2, r1, r2, s, ctx_bytes, ctx_off, ctx_present, status, st);
  if (rc) return rc;
  return rlc_prepare_points(ctx, n, y1, y2, r1, r2, s, status, seed, first_index, st);
}

// Batch-fail fallback by bisection (verify_individually, batch.rs:262-268, 314-318): locate
// the invalid entries of [lo, hi) exactly, for batches the density probe found sparse (or too
// small to sample, below kProbeMin).  The range is cut in kFanout parts aligned to the weight
// blocks, each part's partial is one more MSM over the prepared points, identity parts are
// accepted, failing parts recurse; a range is verified per proof (k_verify_prepared: the
// prepare's decoded points, challenges and decode-level statuses, the equations only) when it
// is <= kLeaf or when most of its parts fail.
constexpr int64_t kLeaf = 1 << 16;
constexpr int kFanout = 8;
constexpr int64_t kProbeMin = 1 << 20;
using cpz::kProbeChunks;

int rlc_fallback(cpz_ctx* ctx, int64_t lo, int64_t hi, const void* y1, const void* y2, const void* r1, const void* r2,
                 const void* s, uint8_t* status, hipStream_t st, int depth) {
  auto per_proof = [&](int64_t a, int64_t b) -> int {
    ctx->fb_stats[4] += (uint64_t)(b - a);
    cpz::VerifyArgs va;
    va.n = b - a;
    va.y1 = static_cast<const uint32_t*>(y1) + 8 * a;
    va.y2 = static_cast<const uint32_t*>(y2) + 8 * a;
    va.r1 = static_cast<const uint32_t*>(r1) + 8 * a;
    va.r2 = static_cast<const uint32_t*>(r2) + 8 * a;
    va.s = static_cast<const uint32_t*>(s) + 8 * a;
    va.c = static_cast<const uint32_t*>(ctx->c.p) + 8 * a;
    va.status = status + a;  // decode-level status in, final status out
    va.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
    va.scratch = nullptr;  // set per launch
    va.eq_only = ctx->call_eq ? 1 : 0;
    va.pre = static_cast<const cpz::ge_niels*>(ctx->rl_prep.pts.p) + 4 * a;
    return launch_verify_chunks(ctx, va, 4, st, nullptr, true);
  };
  if (hi - lo <= kLeaf || depth > 12) return per_proof(lo, hi);
  int64_t cuts[kFanout + 1];
  for (int k = 0; k <= kFanout; k++) {
    int64_t c = lo + ((hi - lo) * k) / kFanout;
    c = (c / cpz::kRlcPrepBlock) * cpz::kRlcPrepBlock;
    cuts[k] = k == 0 ? lo : (k == kFanout ? hi : (c < lo ? lo : c));
  }
  bool fail[kFanout];
  int nfail = 0;
  for (int k = 0; k < kFanout; k++) {
    fail[k] = false;
    if (cuts[k + 1] <= cuts[k]) continue;
    uint8_t part[32];
    int ident = 0;
    int rc = rlc_range(ctx, cuts[k], cuts[k + 1], st, part, &ident);
    if (rc) return rc;
    ctx->fb_stats[5] += 1;
    fail[k] = !ident;
    nfail += fail[k] ? 1 : 0;
  }
  if (2 * nfail > kFanout) return per_proof(lo, hi);  // dense failures: no pruning left
  for (int k = 0; k < kFanout; k++) {
    if (!fail[k]) continue;
    int rc = rlc_fallback(ctx, cuts[k], cuts[k + 1], y1, y2, r1, r2, s, status, st, depth + 1);
    if (rc) return rc;
  }
  return CPZ_OK;
}

// The density probe of a fallback-enabled batch check, launched BEFORE the prepare on its own
// stream so that it runs beside it: per-proof verification (challenge + k_verify_each) of
// kProbeChunks chunks of kRlcPrepBlock proofs spread over the batch, gathered by k_probe_gather
// into one small launch -- the rows, and with contexts each entry's [begin, end) in the batch's
// own context blob (the challenge kernel reads them through ChallengeArgs::ctx_end), so
// batches with contexts (the service's, service.rs:512-517) are sampled the same way.
// Returns the number of chunk starts.
int launch_probe(cpz_ctx* ctx, size_t n, const void* const rows[5], const void* cb, const uint64_t* co,
                 const uint8_t* cp, int64_t starts[kProbeChunks], hipStream_t st) {
  const int64_t blk = cpz::kRlcPrepBlock;
  const size_t m = (size_t)kProbeChunks * blk;
  // rows (5 x 32 B), challenges (32 B), statuses (1 B), then context begin / end (2 x 8 B) and
  // presence (1 B) per sampled entry
  CPZ_HIP(ctx->probe.ensure(m * (5 * 32 + 32 + 1 + 16 + 1) + 16));
  if (!ctx->probe_stream) CPZ_HIP(stream_own_queue(&ctx->probe_stream, ctx->cus, ctx->device, &ctx->own_queues));
  if (!ctx->probe_done) CPZ_HIP(hipEventCreateWithFlags(&ctx->probe_done, hipEventDisableTiming));
  if (!ctx->aux_start) CPZ_HIP(hipEventCreateWithFlags(&ctx->aux_start, hipEventDisableTiming));
  CPZ_HIP(hipEventRecord(ctx->aux_start, st));  // after everything before this call on st
  CPZ_HIP(hipStreamWaitEvent(ctx->probe_stream, ctx->aux_start, 0));
  uint8_t* base = static_cast<uint8_t*>(ctx->probe.p);
  cpz::ProbeGatherArgs ga;
  const int64_t span = (int64_t)n / kProbeChunks;
  for (int k = 0; k < kProbeChunks; k++) ga.starts[k] = starts[k] = ((k * span + span / 2) / blk) * blk;
  ga.blk = (int)blk;
  for (int q = 0; q < 5; q++) {
    ga.rows[q] = static_cast<const uint32_t*>(rows[q]);
    ga.out_rows[q] = reinterpret_cast<uint32_t*>(base + q * m * 32);
  }
  uint32_t* pc = reinterpret_cast<uint32_t*>(base + 5 * m * 32);
  uint8_t* pst = base + 6 * m * 32;
  uint64_t* pbeg = reinterpret_cast<uint64_t*>(base + ((6 * m * 32 + m + 15) & ~(size_t)15));
  ga.ctx_off = co;
  ga.ctx_present = cp;
  ga.out_begin = pbeg;
  ga.out_end = pbeg + m;
  ga.out_present = reinterpret_cast<uint8_t*>(pbeg + 2 * m);
  CPZ_HIP(cpz::launch_probe_gather(ga, ctx->probe_stream));
  int rc = enqueue_verify(ctx, m, ga.out_rows[0], ga.out_rows[1], ga.out_rows[2], ga.out_rows[3], ga.out_rows[4],
                          co ? cb : nullptr, co ? ga.out_begin : nullptr, co ? ga.out_present : nullptr, pst,
                          ctx->probe_stream, pc, nullptr, true, co ? ga.out_end : nullptr);
  if (rc) return rc;
  CPZ_HIP(hipEventRecord(ctx->probe_done, ctx->probe_stream));
  return kProbeChunks;
}

// Per-proof verification (k_verify_prepared) of the listed partition blocks (kPartProofs proofs
// each) of the prepared batch: a workgroup takes kVerifyBlock / kPartProofs consecutive listed
// blocks; launches of at most half the occupancy grid, round-robin over the verify streams and
// their scratch slabs (as launch_verify_chunks).
int verify_prepared_blocks(cpz_ctx* ctx, int64_t n, const void* s, uint8_t* status, const uint32_t* d_blocks,
                           int64_t nb, int block_proofs, hipStream_t st) {
  if (block_proofs <= 0 || cpz::kVerifyBlock % block_proofs != 0) return CPZ_EINVAL;
  const int64_t G = cpz::kVerifyBlock / block_proofs;
  if (nb <= 0) return CPZ_OK;
  const int full = verify_full_grid(ctx);
  const size_t slab = verify_slab_bytes(ctx);
  CPZ_HIP(ctx->scratch.ensure((size_t)CPZ_VERIFY_STREAMS * slab));
  const int64_t quad_max = verify_quad_max(ctx);
  if (CPZ_VERIFY_QUAD && nb * block_proofs <= quad_max) {  // one eight-lanes-per-proof launch (k_verify_quad)
    cpz::VerifyArgs v;
    v.n = n;
    v.s = static_cast<const uint32_t*>(s);
    v.c = static_cast<const uint32_t*>(ctx->c.p);
    v.status = status;
    v.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
    v.pre = static_cast<const cpz::ge_niels*>(ctx->rl_prep.pts.p);
    v.eq_only = ctx->call_eq ? 1 : 0;
    v.scratch = static_cast<char*>(ctx->scratch.p);
    v.blocks = d_blocks;
    v.block_proofs = block_proofs;
    v.nblocks = nb;
    v.quad_max = quad_max;
    StageTimer t(ctx, 1, st);
    CPZ_HIP(cpz::launch_verify_each(v, 0, st));
    return CPZ_OK;
  }
  const int64_t groups = (nb + G - 1) / G;
  const int64_t chunks = (groups + full - 1) / full;
  const int nst = (int)std::min<int64_t>(CPZ_VERIFY_STREAMS, chunks);
  if (nst > 1) {
    if (!ctx->aux_start) CPZ_HIP(hipEventCreateWithFlags(&ctx->aux_start, hipEventDisableTiming));
    CPZ_HIP(hipEventRecord(ctx->aux_start, st));
    for (int k = 0; k < nst - 1; k++) {
      if (!ctx->aux_stream[k]) CPZ_HIP(stream_own_queue(&ctx->aux_stream[k], ctx->cus, ctx->device, &ctx->own_queues));
      if (!ctx->aux_done[k]) CPZ_HIP(hipEventCreateWithFlags(&ctx->aux_done[k], hipEventDisableTiming));
      CPZ_HIP(hipStreamWaitEvent(ctx->aux_stream[k], ctx->aux_start, 0));
    }
  }
  cpz::VerifyArgs va;
  va.n = n;
  va.s = static_cast<const uint32_t*>(s);
  va.c = static_cast<const uint32_t*>(ctx->c.p);
  va.status = status;
  va.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
  va.pre = static_cast<const cpz::ge_niels*>(ctx->rl_prep.pts.p);
  va.eq_only = ctx->call_eq ? 1 : 0;
  va.block_proofs = block_proofs;
  for (int64_t c = 0; c < chunks; c++) {
    const int64_t g0 = c * full;
    const int g = (int)std::min<int64_t>(full, groups - g0);
    cpz::VerifyArgs v = va;
    v.blocks = d_blocks + g0 * G;
    v.nblocks = std::min<int64_t>(nb - g0 * G, (int64_t)g * G);
    const int k = (int)(c % nst);
    v.scratch = static_cast<char*>(ctx->scratch.p) + (size_t)k * slab;
    hipStream_t sc = k == 0 ? st : ctx->aux_stream[k - 1];
    StageTimer t(ctx, 1, sc);
    CPZ_HIP(cpz::launch_verify_each(v, g, sc));
  }
  if (nst > 1) {
    for (int k = 0; k < nst - 1; k++) {
      CPZ_HIP(hipEventRecord(ctx->aux_done[k], ctx->aux_stream[k]));
      CPZ_HIP(hipStreamWaitEvent(st, ctx->aux_done[k], 0));
    }
  }
  return CPZ_OK;
}

// Blocks per launch of the partitioned MSM's sort and walk: 2^24 proofs, ~4.8 GB of lists and
// offsets (~41 KB per 128-proof block); the window sums, 40 KB per block, are kept for the whole
// batch so that one combine launch covers every block.  Per 8192 blocks the launch tails cost C5
// 5 ms (227.9 / 229.5 ms against 223.7 / 223.6 at 65536, 224.6 / 224.9 at 32768; A/B, one call).
constexpr int64_t kPartChunkBlocks = (int64_t(1) << 24) / cpz::kPartProofs;
// Density probe outcomes (invalid entries among the kProbeChunks x 256 sampled) for which the
// partitioned check pays.  Relative to per-proof verification its prepare costs ~0.19, its
// block partials ~0.32 (blocks of 256 proofs) or ~0.36 (128), the locate pass ~0.5 per failing
// fraction, and the per-proof pass over a block holding two or more forgeries ~0.83 (no
// decodes); a block of B proofs is clean with probability (1 - rho)^B.  At B = 128 it pays up
// to rho ~ 0.65 % (~27 sampled; ~0.6 % without the locate pass), at 256 up to ~0.35 % (~14);
// the limits keep a margin.
constexpr int kPartMaxProbeBad = cpz::kPartProofs == 128 ? 20 : 12;
// A batch of at least this many proofs whose RLC check failed with the density probe seeing at
// most one invalid sample (or without a probe) takes the partitioned check instead of bisection.
#ifndef CPZ_SPARSE_PARTITIONED
#define CPZ_SPARSE_PARTITIONED 1
#endif
constexpr int64_t kPartSparseMin = 1 << 19;

// Every buffer the partitioned check of n proofs uses: the prepared batch, the partial / flag
// words of an MSM set, one chunk's sorted lists / assignment / offsets, and the whole batch's
// window sums, partials, fail flags and failing-block list.  A failure leaves CPZ_ENOMEM (or the
// HIP error) with no partial state: part_release frees the partitioned buffers.
int part_reserve(cpz_ctx* ctx, int64_t n) {
  const int64_t nblk = (n + cpz::kPartProofs - 1) / cpz::kPartProofs;
  const int64_t chunk = std::min<int64_t>(nblk, kPartChunkBlocks);
  if (int rc = rlc_reserve_prepared(ctx->rl_prep, n)) return rc;
  if (int rc = rlc_reserve_msm(ctx->rl_msm, 1)) return rc;  // its partial / flag words
  CPZ_HIP(ctx->rl_flags.ensure(4 * sizeof(int)));
  CPZ_HIP(ctx->pt_lists.ensure((size_t)chunk * cpz::kPartListCap * sizeof(uint16_t)));
  CPZ_HIP(ctx->pt_assign.ensure((size_t)chunk * cpz::kPartUnits * sizeof(uint16_t)));
  CPZ_HIP(ctx->pt_offs.ensure((size_t)chunk * cpz::kPartOffs * sizeof(uint16_t)));
  CPZ_HIP(ctx->pt_wsum.ensure((size_t)nblk * cpz::kPartWsum * sizeof(cpz::ge_p3)));  // 40 KB per block
  CPZ_HIP(ctx->pt_part.ensure((size_t)nblk * sizeof(cpz::ge_p3)));
  CPZ_HIP(ctx->pt_fail.ensure((size_t)nblk));
  CPZ_HIP(ctx->pt_tmp.ensure((size_t)((nblk + 63) / 64 + 16) * sizeof(cpz::ge_p3)));
  CPZ_HIP(ctx->pt_blocks.ensure((size_t)2 * nblk * sizeof(uint32_t)));  // failing blocks, then the per-proof lists
  return CPZ_OK;
}

// The partitioned check's own buffers (not the prepared batch).
void part_release_blocks(cpz_ctx* ctx) {
  for (DevBuf* b : {&ctx->pt_lists, &ctx->pt_offs, &ctx->pt_wsum, &ctx->pt_part, &ctx->pt_fail, &ctx->pt_tmp,
                    &ctx->pt_blocks, &ctx->pt_assign, &ctx->pt_ldig, &ctx->pt_lsum, &ctx->pt_lpart, &ctx->pt_lfail,
                    &ctx->pt_loc})
    b->release();
  (void)hipGetLastError();
}

void part_release(cpz_ctx* ctx) {
  part_release_blocks(ctx);
  ctx->rl_prep.release();
  (void)hipGetLastError();
}

// The locate pass (rlc.h, part.hip) over the failing blocks listed in pt_blocks: their
// index-weighted partials P'_b, then per block the one j with P'_b = [j] P_b if there is one.
// Fills `cand` with the located proofs and leaves in `whole` the blocks to verify per proof.
// Its buffers (16 KB of digits per failing block) are taken on demand; if they do not fit,
// every failing block is verified per proof, as without the pass.
int part_locate(cpz_ctx* ctx, int64_t n, const void* s, const uint8_t* d_status, const uint8_t seed[32],
                uint64_t first_index, const std::vector<uint32_t>& blocks, std::vector<uint32_t>& whole,
                std::vector<uint32_t>& cand, hipStream_t st) {
  const int64_t nf = (int64_t)blocks.size();
  const int64_t dstride = ((4 * cpz::kPartProofs * nf) + 7) & ~(int64_t)7;
  const int64_t nsum = nf * (cpz::kPartProofs / cpz::kRlcSumBlock);
  if (ctx->pt_ldig.ensure((size_t)cpz::kRlcWindows * dstride * sizeof(int16_t)) != hipSuccess ||
      ctx->pt_lsum.ensure((size_t)2 * nsum * sizeof(cpz::sc)) != hipSuccess ||
      ctx->pt_lpart.ensure((size_t)nf * sizeof(cpz::ge_p3)) != hipSuccess ||
      ctx->pt_lfail.ensure((size_t)nf) != hipSuccess || ctx->pt_loc.ensure((size_t)nf * sizeof(uint16_t)) != hipSuccess) {
    for (DevBuf* b : {&ctx->pt_ldig, &ctx->pt_lsum, &ctx->pt_lpart, &ctx->pt_lfail, &ctx->pt_loc}) b->release();
    (void)hipGetLastError();
    return CPZ_OK;  // `whole` keeps every failing block
  }
  const uint32_t* d_blocks = static_cast<const uint32_t*>(ctx->pt_blocks.p);
  {
    StageTimer t(ctx, 3, st);
    cpz::PartIdxArgs ia;
    ia.nblk = nf;
    ia.n = n;
    ia.blocks = d_blocks;
    ia.first_index = first_index;
    std::memcpy(ia.seed, seed, 32);
    ia.s = static_cast<const uint32_t*>(s);
    ia.c = static_cast<const uint32_t*>(ctx->c.p);
    ia.status = d_status;
    ia.digits = static_cast<int16_t*>(ctx->pt_ldig.p);
    ia.dstride = dstride;
    ia.block_sums = static_cast<cpz::sc*>(ctx->pt_lsum.p);
    CPZ_HIP(cpz::launch_part_index_digits(ia, st));
    cpz::PartArgs pa;
    pa.n = nf * cpz::kPartProofs;  // compact; proofs past the batch's end have zero digits
    pa.pts = static_cast<const cpz::ge_niels*>(ctx->rl_prep.pts.p);
    pa.pmap = d_blocks;
    pa.digits = ia.digits;
    pa.dstride = dstride;
    pa.block_sums = ia.block_sums;
    pa.tab = static_cast<const cpz::ge_niels*>(ctx->gs->tab.p);
    pa.lists = static_cast<uint16_t*>(ctx->pt_lists.p);
    pa.assign = static_cast<uint16_t*>(ctx->pt_assign.p);
    pa.offs = static_cast<uint16_t*>(ctx->pt_offs.p);
    pa.wsum = static_cast<cpz::ge_p3*>(ctx->pt_wsum.p);  // the first pass's window sums are spent
    pa.part = static_cast<cpz::ge_p3*>(ctx->pt_lpart.p);
    pa.fail = static_cast<uint8_t*>(ctx->pt_lfail.p);
    const int64_t chunk = std::min<int64_t>(nf, kPartChunkBlocks);
    for (int64_t b0 = 0; b0 < nf; b0 += chunk) {
      pa.blk0 = b0;
      pa.nblk = std::min<int64_t>(chunk, nf - b0);
      CPZ_HIP(cpz::launch_part_sort(pa, st));
      StageTimer ta(ctx, 15, st);  // the locate pass's walk (k_part_acc)
      CPZ_HIP(cpz::launch_part_acc(pa, st));
    }
    pa.blk0 = 0;
    pa.nblk = nf;
    CPZ_HIP(cpz::launch_part_combine(pa, st));
    cpz::PartLocArgs la;
    la.nblk = nf;
    la.blocks = d_blocks;
    la.part = static_cast<const cpz::ge_p3*>(ctx->pt_part.p);
    la.lpart = pa.part;
    la.lfail = pa.fail;
    la.loc = static_cast<uint16_t*>(ctx->pt_loc.p);
    CPZ_HIP(cpz::launch_part_locate(la, st));
  }
  std::vector<uint16_t> loc((size_t)nf);
  CPZ_HIP(hipMemcpyAsync(loc.data(), ctx->pt_loc.p, (size_t)nf * sizeof(uint16_t), hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipStreamSynchronize(st));
  ctx->fb_stats[6] = (uint64_t)nf;
  whole.clear();
  for (int64_t k = 0; k < nf; k++) {
    const int64_t e = (int64_t)blocks[(size_t)k] * cpz::kPartProofs + loc[(size_t)k];
    if (loc[(size_t)k] == cpz::kPartNoLoc || e >= n) whole.push_back(blocks[(size_t)k]);  // (past the end: w.o.p. never)
    else cand.push_back((uint32_t)e);
  }
  ctx->fb_stats[7] = (uint64_t)cand.size();
  return CPZ_OK;
}

// Per-proof verification (k_verify_prepared) of the located proofs alone and of the `whole`
// blocks.  A located proof that verifies (a 2^-121 event: the locate pass accepted its block's
// other proofs on P'_b = [j] P_b) sends its block to per-proof verification as well.
int part_verify_lists(cpz_ctx* ctx, int64_t n, const void* s, uint8_t* d_status, const std::vector<uint32_t>& blocks,
                      std::vector<uint32_t> whole, const std::vector<uint32_t>& cand, hipStream_t st) {
  uint32_t* d_list = static_cast<uint32_t*>(ctx->pt_blocks.p) + blocks.size();  // after the failing blocks
  StageTimer span(ctx, 4, st);  // wall time of the per-proof pass; launches timed as verify_each
  if (!cand.empty()) {
    ctx->fb_stats[4] += (uint64_t)cand.size();
    CPZ_HIP(hipMemcpyAsync(d_list, cand.data(), cand.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    if (int rc = verify_prepared_blocks(ctx, n, s, d_status, d_list, (int64_t)cand.size(), 1, st)) return rc;
    std::vector<uint8_t> cst(cand.size());
    uint8_t* d_cst = static_cast<uint8_t*>(ctx->pt_lfail.p);  // |cand| <= failing blocks bytes, spent
    CPZ_HIP(cpz::launch_gather_status(d_status, d_list, (int64_t)cand.size(), d_cst, st));
    CPZ_HIP(hipMemcpyAsync(cst.data(), d_cst, cand.size(), hipMemcpyDeviceToHost, st));
    CPZ_HIP(hipStreamSynchronize(st));
    for (size_t k = 0; k < cand.size(); k++)
      if (cst[k] == cpz::kStatusOk) whole.push_back(cand[k] / (uint32_t)cpz::kPartProofs);
  }
  if (whole.empty()) return CPZ_OK;
  for (uint32_t b : whole) ctx->fb_stats[4] += (uint64_t)std::min<int64_t>(cpz::kPartProofs, n - (int64_t)b * cpz::kPartProofs);
  CPZ_HIP(hipMemcpyAsync(d_list, whole.data(), whole.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (int rc = verify_prepared_blocks(ctx, n, s, d_status, d_list, (int64_t)whole.size(), cpz::kPartProofs, st))
    return rc;
  CPZ_HIP(hipStreamSynchronize(st));  // the host lists are pageable memory read by the copies above
  return CPZ_OK;
}

// The partitioned fallback over the prepared batch (buffers from part_reserve): every block's
// partial (k_part_*), the batch partial as their sum, and per-proof verification of the
// failing blocks only.
int part_fallback(cpz_ctx* ctx, int64_t n, const void* s, uint8_t* d_status, const uint8_t seed[32],
                  uint64_t first_index, uint8_t partial[32], int* identity, hipStream_t st) {
  const int64_t nblk = (n + cpz::kPartProofs - 1) / cpz::kPartProofs;
  const int64_t chunk = std::min<int64_t>(nblk, kPartChunkBlocks);
  {
    StageTimer t(ctx, 3, st);
    cpz::PartArgs pa;
    pa.n = n;
    pa.pts = static_cast<const cpz::ge_niels*>(ctx->rl_prep.pts.p);
    pa.digits = static_cast<const int16_t*>(ctx->rl_prep.dig.p);
    pa.dstride = rlc_dstride(ctx->rl_prep.cap);
    pa.block_sums = static_cast<const cpz::sc*>(ctx->rl_prep.bsum.p);
    pa.tab = static_cast<const cpz::ge_niels*>(ctx->gs->tab.p);
    pa.lists = static_cast<uint16_t*>(ctx->pt_lists.p);
    pa.assign = static_cast<uint16_t*>(ctx->pt_assign.p);
    pa.offs = static_cast<uint16_t*>(ctx->pt_offs.p);
    pa.wsum = static_cast<cpz::ge_p3*>(ctx->pt_wsum.p);
    pa.part = static_cast<cpz::ge_p3*>(ctx->pt_part.p);
    pa.fail = static_cast<uint8_t*>(ctx->pt_fail.p);
#if defined(CPZ_CLOCK_PROBE)
    {  // k_part_acc's clock stamps: one record per wave (= per block) of the last chunk's launch
      ctx->clk_waves[2] = (size_t)chunk;
      CPZ_HIP(ctx->clk[2].ensure(ctx->clk_waves[2] * 40));
      CPZ_HIP(hipMemsetAsync(ctx->clk[2].p, 0, ctx->clk_waves[2] * 40, st));
      pa.clock_probe = static_cast<uint64_t*>(ctx->clk[2].p);
    }
#endif
    for (int64_t b0 = 0; b0 < nblk; b0 += chunk) {
      pa.blk0 = b0;
      pa.nblk = std::min<int64_t>(chunk, nblk - b0);
      CPZ_HIP(cpz::launch_part_sort(pa, st));
      StageTimer ta(ctx, 14, st);  // every block's walk (k_part_acc), the C5 roofline's kernel
      CPZ_HIP(cpz::launch_part_acc(pa, st));
    }
    pa.blk0 = 0;
    pa.nblk = nblk;
    CPZ_HIP(cpz::launch_part_combine(pa, st));
    CPZ_HIP(cpz::launch_part_sum(pa.part, nblk, static_cast<cpz::ge_p3*>(ctx->pt_tmp.p),
                                 static_cast<uint32_t*>(ctx->rl_msm.partial.p), static_cast<int*>(ctx->rl_msm.flags.p),
                                 st));
  }
  std::vector<uint8_t> dirty((size_t)nblk);
  int flags[1];
  CPZ_HIP(hipMemcpyAsync(dirty.data(), ctx->pt_fail.p, (size_t)nblk, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(partial, ctx->rl_msm.partial.p, 32, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(flags, ctx->rl_msm.flags.p, sizeof(int), hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipStreamSynchronize(st));
  *identity = flags[0];
  std::vector<uint32_t> blocks;
  for (int64_t b = 0; b < nblk; b++)
    if (dirty[(size_t)b]) blocks.push_back((uint32_t)b);
  ctx->fb_stats[2] = (uint64_t)nblk;
  ctx->fb_stats[3] = blocks.size();
  if (blocks.empty()) return CPZ_OK;
  CPZ_HIP(hipMemcpyAsync(ctx->pt_blocks.p, blocks.data(), blocks.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  std::vector<uint32_t> whole = blocks;  // blocks verified per proof
  std::vector<uint32_t> cand;            // located forged proofs, verified alone
  // The locate pass pays while most failing blocks hold one forgery; with more than half of the
  // blocks failing (density above ~0.5 %) the failing blocks are verified whole.
  if (CPZ_PART_LOCATE && 2 * (int64_t)blocks.size() <= nblk) {
    int rc = part_locate(ctx, n, s, d_status, seed, first_index, blocks, whole, cand, st);
    if (rc) return rc;
  }
  return part_verify_lists(ctx, n, s, d_status, blocks, whole, cand, st);
}

int verify_batch_impl(cpz_ctx* ctx, size_t n, const void* y1, const void* y2, const void* r1, const void* r2,
                      const void* s, const void* cb, const uint64_t* co, const uint8_t* cp, uint8_t* d_status,
                      const uint8_t seed[32], uint64_t first_index, uint8_t partial_out[32], int* batch_ok,
                      int fallback, uint8_t* host_status, hipStream_t st) {
  // A fallback-enabled check of a large batch (with or without contexts) first samples its
  // density, beside the batch's challenges (the probe's ~0.5 ms of per-proof latency hides under
  // them).  Two or more invalid entries among the kProbeChunks x 256 sampled: the batch
  // cannot pass and bisection cannot prune it (every range of a few thousand proofs fails).
  //   * up to kPartMaxProbeBad = 20 sampled (density up to ~0.5 %, configs[4]'s 0.1 %): the
  //     partitioned check -- prepare, every 128-proof block's partial in one pass, the failing
  //     blocks' index-weighted partials (part_locate), per-proof verification of the located
  //     entries and of the blocks holding more; partial_out is the batch's partial.
  //   * denser: nothing is prepared, every entry is verified per proof (k_verify_each on the
  //     challenges just computed), and partial_out is 32 x 0xff ("no partial": not an
  //     encoding) -- the cost of the per-proof path plus the probe.
  for (auto& v : ctx->fb_stats) v = 0;
  int64_t starts[kProbeChunks];
  const bool probe = fallback && (int64_t)n >= kProbeMin;
  if (probe) {
    const void* rows[5] = {y1, y2, r1, r2, s};
    int rc = launch_probe(ctx, n, rows, cb, co, cp, starts, st);
    if (rc < 0) return rc;
  }
  int rc = batch_challenges(ctx, n, y1, y2, r1, r2, s, cb, co, cp, d_status, st);
  if (rc) return rc;
  if (probe) {
    const size_t m = (size_t)kProbeChunks * cpz::kRlcPrepBlock;
    std::vector<uint8_t> pst(m);
    CPZ_HIP(hipStreamWaitEvent(st, ctx->probe_done, 0));  // the probe used scratch slab 0 too
    CPZ_HIP(hipMemcpyAsync(pst.data(), static_cast<uint8_t*>(ctx->probe.p) + 6 * m * 32, m, hipMemcpyDeviceToHost,
                           ctx->probe_stream));
    CPZ_HIP(hipStreamSynchronize(ctx->probe_stream));
    int bad = 0;
    for (uint8_t v : pst) bad += (v == cpz::kStatusEqFail) ? 1 : 0;
    ctx->fb_stats[1] = (uint64_t)bad;
    // The partitioned check's buffers (the prepared batch, ~40 KB of window sums per block,
    // one chunk's sorted lists) are reserved first; if the device cannot hold them they are
    // released and the batch takes the per-proof path, which needs no extra memory.
    if (bad >= 2 && bad <= kPartMaxProbeBad && part_reserve(ctx, (int64_t)n) != CPZ_OK) {
      part_release(ctx);
      bad = kPartMaxProbeBad + 1;
    }
    if (bad >= 2 && bad <= kPartMaxProbeBad) {
      ctx->fb_stats[0] = CPZ_FALLBACK_PARTITIONED;
      if ((rc = rlc_prepare_points(ctx, n, y1, y2, r1, r2, s, d_status, seed, first_index, st, false))) return rc;
      uint8_t part[32];
      int ident = 0;
      if ((rc = part_fallback(ctx, (int64_t)n, s, d_status, seed, first_index, part, &ident, st))) return rc;
      if (partial_out) std::memcpy(partial_out, part, 32);
      if (batch_ok) *batch_ok = 0;  // the probe saw invalid entries
      if (host_status) {
        CPZ_HIP(hipMemcpyAsync(host_status, d_status, n, hipMemcpyDeviceToHost, st));
        CPZ_HIP(hipStreamSynchronize(st));
      }
      return CPZ_OK;
    }
    if (bad > kPartMaxProbeBad) {
      ctx->fb_stats[0] = CPZ_FALLBACK_PER_PROOF;
      ctx->fb_stats[4] = (uint64_t)n;
      if (partial_out) std::memset(partial_out, 0xff, 32);
      if (batch_ok) *batch_ok = 0;
      cpz::VerifyArgs va;
      va.n = (int64_t)n;
      va.y1 = static_cast<const uint32_t*>(y1);
      va.y2 = static_cast<const uint32_t*>(y2);
      va.r1 = static_cast<const uint32_t*>(r1);
      va.r2 = static_cast<const uint32_t*>(r2);
      va.s = static_cast<const uint32_t*>(s);
      va.c = static_cast<const uint32_t*>(ctx->c.p);
      va.status = d_status;  // response statuses from batch_challenges -> final statuses
      va.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
      va.scratch = nullptr;  // set per launch
      va.eq_only = ctx->call_eq ? 1 : 0;
      {
        StageTimer span(ctx, 4, st);  // wall time of the fallback; launches timed as verify_each
        if ((rc = launch_verify_chunks(ctx, va, 1, st, nullptr, true))) return rc;
      }
      CPZ_HIP(hipStreamSynchronize(st));
      if (host_status) {
        CPZ_HIP(hipMemcpyAsync(host_status, d_status, n, hipMemcpyDeviceToHost, st));
        CPZ_HIP(hipStreamSynchronize(st));
      }
      return CPZ_OK;
    }
  }
  if ((rc = rlc_prepare_points(ctx, n, y1, y2, r1, r2, s, d_status, seed, first_index, st))) return rc;
  // The partial, its identity flag, the any-bad word and (host-buffer calls) the statuses come
  // back with one synchronisation, into page-locked memory when it is there: a valid batch
  // needs no second round trip.  A failing one re-reads the statuses after its fallback.
  if ((rc = rlc_range_launch(ctx, 0, (int64_t)n, st))) return rc;
  const bool stage_st = host_status && n <= kPinStageMax;  // (the staged inputs there are spent)
  const bool pinned = ctx->pin.ensure(kPinMail + (stage_st ? pad16(n) : 0)) == hipSuccess;
  (void)hipGetLastError();
  uint8_t part_buf[32];
  int word_buf[2] = {0, 0};
  uint8_t* part = pinned ? static_cast<uint8_t*>(ctx->pin.p) : part_buf;
  int* words = pinned ? reinterpret_cast<int*>(static_cast<uint8_t*>(ctx->pin.p) + 32) : word_buf;
  uint8_t* st_stage = pinned && stage_st ? static_cast<uint8_t*>(ctx->pin.p) + kPinMail : host_status;
  CPZ_HIP(hipMemcpyAsync(part, ctx->rl_msm.partial.p, 32, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(&words[0], ctx->rl_msm.flags.p, sizeof(int), hipMemcpyDeviceToHost, st));
  // every entry must also have decoded (zero-weight entries are not "verified")
  CPZ_HIP(hipMemcpyAsync(&words[1], static_cast<int*>(ctx->rl_flags.p) + 3, sizeof(int), hipMemcpyDeviceToHost, st));
  if (host_status) CPZ_HIP(hipMemcpyAsync(st_stage, d_status, n, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipStreamSynchronize(st));
  const int ident = words[0];
  const int any_bad = words[1];
  if (partial_out) std::memcpy(partial_out, part, 32);
  const bool all_live = any_bad == 0;
  if (batch_ok) *batch_ok = (ident && all_live) ? 1 : 0;
  if (!ident && fallback) {
    // A batch of several MSM spans whose failure lies in at most half of them: each span's own
    // P was tested by its final (RlcMsmArgs::span_identity), so only the failing spans are
    // searched, each by bisection over its prepared points (configs[3]'s forged variant: 2 of
    // 32 spans) -- the partitioned pass below would walk every block of the whole batch.
    const int64_t nspan = ((int64_t)n + CPZ_RLC_SPAN - 1) / CPZ_RLC_SPAN;
    if (nspan > 1) {
      std::vector<int> sid((size_t)nspan);
      CPZ_HIP(hipMemcpyAsync(sid.data(), ctx->rl_span_ident.p, (size_t)nspan * sizeof(int), hipMemcpyDeviceToHost, st));
      CPZ_HIP(hipStreamSynchronize(st));
      int64_t nfail = 0;
      for (int v : sid) nfail += v ? 0 : 1;
      if (nfail > 0 && 2 * nfail <= nspan) {
        part_release_blocks(ctx);
        ctx->fb_stats[0] = CPZ_FALLBACK_BISECTION;
        for (int64_t j = 0; j < nspan; j++) {
          if (sid[(size_t)j]) continue;
          const int64_t slo = j * CPZ_RLC_SPAN, shi = std::min<int64_t>((int64_t)n, slo + CPZ_RLC_SPAN);
          if ((rc = rlc_fallback(ctx, slo, shi, y1, y2, r1, r2, s, d_status, st, 0))) return rc;
        }
        CPZ_HIP(hipStreamSynchronize(st));
        if (host_status) {
          CPZ_HIP(hipMemcpyAsync(host_status, d_status, n, hipMemcpyDeviceToHost, st));
          CPZ_HIP(hipStreamSynchronize(st));
        }
        return CPZ_OK;
      }
    }
    // A large batch that failed: every block's partial over the points just prepared, then
    // the locate pass and per-proof verification of what it leaves (part_fallback) -- at 2^20
    // cheaper than bisection from one forged entry up (sub-range MSMs of 1/8 of the range, each
    // with the whole MSM's sort and tails).  Smaller batches, or no room for the block buffers:
    // bisection.
    if (CPZ_SPARSE_PARTITIONED && (int64_t)n >= kPartSparseMin && part_reserve(ctx, (int64_t)n) == CPZ_OK) {
      ctx->fb_stats[0] = CPZ_FALLBACK_PARTITIONED;
      uint8_t part2[32];
      int ident2 = 0;
      if ((rc = part_fallback(ctx, (int64_t)n, s, d_status, seed, first_index, part2, &ident2, st))) return rc;
    } else {
      part_release_blocks(ctx);
      ctx->fb_stats[0] = CPZ_FALLBACK_BISECTION;
      rc = rlc_fallback(ctx, 0, (int64_t)n, y1, y2, r1, r2, s, d_status, st, 0);
      if (rc) return rc;
    }
    CPZ_HIP(hipStreamSynchronize(st));  // statuses complete on return (documented)
    if (host_status) {
      CPZ_HIP(hipMemcpyAsync(host_status, d_status, n, hipMemcpyDeviceToHost, st));
      CPZ_HIP(hipStreamSynchronize(st));
    }
    return CPZ_OK;
  }
  if (host_status && st_stage != host_status) std::memcpy(host_status, st_stage, n);
  return CPZ_OK;
}

}  // namespace

extern "C" {

int cpz_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* cpz_last_error(void) { return g_last_error.c_str(); }

void cpz_default_generators(uint8_t g[32], uint8_t h[32]) {
  if (g) std::memcpy(g, kDefaultG, 32);
  if (h) std::memcpy(h, kDefaultH, 32);
}

}  // extern "C"

namespace {

int ctx_create(int device_ordinal, cpz_ctx** out) {
  if (!out) return fail(CPZ_EINVAL, "out is null");
  *out = nullptr;
  int ndev = 0;
  CPZ_HIP(hipGetDeviceCount(&ndev));
  if (device_ordinal < 0 || device_ordinal >= ndev) return fail(CPZ_EINVAL, "device ordinal out of range");
  CPZ_HIP(hipSetDevice(device_ordinal));
  cpz_ctx* ctx = new (std::nothrow) cpz_ctx();
  if (!ctx) return fail(CPZ_ENOMEM, "host allocation failed");
  ctx->device = device_ordinal;
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device_ordinal);
  // A blocking stream: it orders with the legacy default stream, so work queued by other
  // libraries (e.g. torch's default stream, handle 0, which the C ABI reads as "use the
  // context stream") is ordered with the verifier's kernels in both directions.
  if (e == hipSuccess) e = stream_own_queue(&ctx->stream, prop.multiProcessorCount, device_ordinal, &ctx->own_queues);
  if (e != hipSuccess) {
    delete ctx;
    return fail(CPZ_EHIP, std::string("context setup: ") + hipGetErrorString(e));
  }
  ctx->cus = prop.multiProcessorCount;
  // CPZ_CUS (tests): size grids and slabs as on a part with fewer CUs, e.g. the 110-CU case whose
  // eight-lane bound (verify_quad_max) is 14080 rather than 16384
  if (const char* v = std::getenv("CPZ_CUS")) {
    const int k = std::atoi(v);
    if (k >= 1 && k < ctx->cus) ctx->cus = k;
  }
  ctx->verify_blocks_per_cu = cpz::verify_each_blocks_per_cu();  // the grid-stride verify grid fills the chip once
  // full (g, h) sets (128 MiB of combs each) this context may keep: CPZ_GEN_CACHE=1..4
  if (const char* v = std::getenv("CPZ_GEN_CACHE")) {
    const int k = std::atoi(v);
    if (k >= 1 && k <= kGenCache) ctx->gen_cap = k;
  }
  *out = ctx;
  return CPZ_OK;
}

}  // namespace

extern "C" {

int cpz_ctx_create(int device_ordinal, cpz_ctx** out) {
#if defined(CPZ_WRONG_VERDICT_FLAG)
  // a timing-only build (timing_only.h): its verdicts are wrong by construction
  if (out) *out = nullptr;
  (void)device_ordinal;
  return fail(CPZ_EINVAL, std::string("timing-only build (") + CPZ_WRONG_VERDICT_FLAG +
                              "): verdicts are wrong by design; only cpz_ctx_create_timing_only opens a context");
#else
  return ctx_create(device_ordinal, out);
#endif
}

#if defined(CPZ_WRONG_VERDICT_FLAG)
// Timing harness entry (tools/time_verify.py): exported by timing-only builds alone.
int cpz_ctx_create_timing_only(int device_ordinal, cpz_ctx** out) { return ctx_create(device_ordinal, out); }
#endif

#if defined(CPZ_CLOCK_PROBE)
// The clock stamps of the last k_rlc_prepare (kernel 0), k_rlc_bucket (kernel 1) or, of the
// partitioned check's first pass, k_part_acc (kernel 2) launch: up to max_waves records of 5
// words (a wave that did no work leaves zeros); *got = the launch's waves.  Kernel 3: the last
// k_verify_quad launch's kQuadPhases phase stamps (one 72-byte record; max_waves counts 40-byte
// records, so pass at least 2; k_verify_small's or k_verify_wide's kSmallStamps words when one of them ran instead).  Exported by CPZ_CLOCK_PROBE builds alone
// (tools/time_verify.py MODE=rlc / MODE=c5, tools/quad_phases.py).
int cpz_ctx_clock_probe(cpz_ctx* ctx, int kernel, uint64_t* out, size_t max_waves, size_t* got) {
  if (!ctx || !out || !got || kernel < 0 || kernel > 3) return fail(CPZ_EINVAL, "bad arguments");
  if (kernel == 3) {
    CallLock lock(ctx);
    CPZ_HIP(hipSetDevice(ctx->device));
    CPZ_HIP(hipDeviceSynchronize());
    if (max_waves < 2 || !ctx->clk[3].p) return fail(CPZ_EINVAL, "no k_verify_quad stamps");
    CPZ_HIP(hipMemcpy(out, ctx->clk[3].p, cpz::kSmallStamps * sizeof(uint64_t), hipMemcpyDeviceToHost));
    *got = 1;
    return CPZ_OK;
  }
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  CPZ_HIP(hipDeviceSynchronize());
  const size_t w = std::min(max_waves, ctx->clk_waves[kernel]);
  if (w) CPZ_HIP(hipMemcpy(out, ctx->clk[kernel].p, w * 40, hipMemcpyDeviceToHost));
  *got = ctx->clk_waves[kernel];
  return CPZ_OK;
}
#endif

int cpz_abi_version(void) { return CPZ_ABI_VERSION; }

int cpz_ctx_fallback_stats(cpz_ctx* ctx, uint64_t out[CPZ_FALLBACK_STATS]) {
  if (!ctx || !out) return fail(CPZ_EINVAL, "null argument");
  CallLock lock(ctx);
  std::memcpy(out, ctx->fb_stats, sizeof(ctx->fb_stats));
  return CPZ_OK;
}

int cpz_ctx_set_commitment_checks(cpz_ctx* ctx, int enable) {
  if (!ctx) return fail(CPZ_EINVAL, "null context");
  CallLock lock(ctx);
  ctx->eq_only = enable == 0;
  return CPZ_OK;
}

int cpz_verify_batch(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                     const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s,
                     const uint8_t* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                     const uint8_t seed[32], uint64_t first_index, uint8_t partial_out[32], int* batch_ok,
                     uint8_t* status_out) {
  return cpz_verify_batch_ex(ctx, 0, g, h, n, y1, y2, r1, r2, s, ctx_bytes, ctx_off, ctx_present, seed, first_index,
                              partial_out, batch_ok, status_out);
}

int cpz_verify_batch_ex(cpz_ctx* ctx, uint32_t flags, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                     const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s,
                     const uint8_t* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                     const uint8_t seed[32], uint64_t first_index, uint8_t partial_out[32], int* batch_ok,
                     uint8_t* status_out) {
  if (!ctx || !g || !h || !seed) return fail(CPZ_EINVAL, "null context, generators or seed");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!y1 || !y2 || !r1 || !r2 || !s) return fail(CPZ_EINVAL, "null input pointer");
  CallLock lock(ctx, flags);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h);
  if (rc) return rc;
  if ((rc = order_after_last(ctx, ctx->stream))) return rc;
  const uint8_t* host[5] = {y1, y2, r1, r2, s};
  const void* dev[5];
  const void* dcb;
  const uint64_t* dco;
  const uint8_t* dcp;
  rc = stage_inputs(ctx, n, host, 5, ctx_bytes, ctx_off, ctx_present, dev, &dcb, &dco, &dcp);
  if (rc) return rc;
  CPZ_HIP(ctx->st.ensure(n));
  return verify_batch_impl(ctx, n, dev[0], dev[1], dev[2], dev[3], dev[4], dcb, dco, dcp,
                           static_cast<uint8_t*>(ctx->st.p), seed, first_index, partial_out, batch_ok,
                           status_out != nullptr, status_out, ctx->stream);
}

int cpz_verify_batch_device(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const void* d_y1,
                            const void* d_y2, const void* d_r1, const void* d_r2, const void* d_s,
                            const void* d_ctx_bytes, const uint64_t* d_ctx_off, const uint8_t* d_ctx_present,
                            const uint8_t seed[32], uint64_t first_index, uint8_t partial_out[32], int* batch_ok,
                            void* d_status_out, int fallback, void* stream) {
  if (!ctx || !g || !h || !seed) return fail(CPZ_EINVAL, "null context, generators or seed");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!d_y1 || !d_y2 || !d_r1 || !d_r2 || !d_s || !d_status_out) return fail(CPZ_EINVAL, "null input pointer");
  if (!aligned16(d_y1) || !aligned16(d_y2) || !aligned16(d_r1) || !aligned16(d_r2) || !aligned16(d_s))
    return fail(CPZ_EINVAL, "device inputs must be 16-byte aligned");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h);
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = order_after_last(ctx, st))) return rc;
  rc = verify_batch_impl(ctx, n, d_y1, d_y2, d_r1, d_r2, d_s, d_ctx_bytes, d_ctx_off, d_ctx_present,
                         static_cast<uint8_t*>(d_status_out), seed, first_index, partial_out, batch_ok, fallback,
                         nullptr, st);
  if (rc) return rc;
  return record_last(ctx, st);
}

int cpz_msm(cpz_ctx* ctx, size_t n, const uint8_t* points, const uint8_t* scalars, uint8_t out[32]) {
  if (!ctx || !points || !scalars || !out || n == 0) return fail(CPZ_EINVAL, "bad arguments");
  if ((int64_t)n + 2 > cpz::kRlcMaxMsmPoints) return fail(CPZ_EINVAL, "too many points for one MSM call");
  for (size_t j = 0; j < n; j++)
    if (scalars[32 * j + 31] & 0xe0) return fail(CPZ_EINVAL, "scalars must be below 2^253");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  uint8_t g[32], h[32];
  cpz_default_generators(g, h);
  int rc = ctx->gs ? CPZ_OK : ensure_generators(ctx, g, h);
  if (rc) return rc;
  if ((rc = order_after_last(ctx, ctx->stream))) return rc;
  // n points occupy the prepared set's point / digit rows from 0 (room for ceil(n / 4)
  // proofs), and the MSM set must hold all of them in one MSM
  const int64_t nproofs = (int64_t)(n + 3) / 4;
  if ((rc = rlc_reserve_prepared(ctx->rl_prep, nproofs))) return rc;
  if ((rc = rlc_reserve_msm(ctx->rl_msm, nproofs))) return rc;
  CPZ_HIP(ctx->rl_flags.ensure(4 * sizeof(int)));
  CPZ_HIP(ctx->in[0].ensure(n * 32));
  CPZ_HIP(ctx->in[1].ensure(n * 32));
  CPZ_HIP(hipMemcpyAsync(ctx->in[0].p, points, n * 32, hipMemcpyHostToDevice, ctx->stream));
  CPZ_HIP(hipMemcpyAsync(ctx->in[1].p, scalars, n * 32, hipMemcpyHostToDevice, ctx->stream));
  CPZ_HIP(hipMemsetAsync(ctx->rl_flags.p, 0, 4 * sizeof(int), ctx->stream));
  cpz::RlcMsmArgs m;
  if ((rc = rlc_msm_args(ctx->rl_prep, ctx->rl_msm, 0, nproofs, m))) return rc;
  m.p0 = 0;
  m.p1 = (int64_t)n;  // the points themselves, not 4 per proof
  cpz::rlc_sort_geometry(m, (int64_t)n + 2);
  CPZ_HIP(cpz::launch_msm_load((int64_t)n, static_cast<const uint32_t*>(ctx->in[0].p),
                               static_cast<const uint32_t*>(ctx->in[1].p), m.pts, m.digits, m.dstride,
                               static_cast<int*>(ctx->rl_flags.p) + 2, ctx->stream));
  // the extra points (g, h at e0) get zero scalars: empty block range
  CPZ_HIP(cpz::launch_rlc_msm(m, static_cast<const cpz::sc*>(ctx->rl_prep.bsum.p), 0, 0,
                              static_cast<const cpz::ge_niels*>(ctx->gs->tab.p), ctx->stream, nullptr));
  int flags[3];
  CPZ_HIP(hipMemcpyAsync(out, ctx->rl_msm.partial.p, 32, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipMemcpyAsync(flags, ctx->rl_flags.p, sizeof(flags), hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  if (flags[2]) return fail(CPZ_EINVAL, "a point does not decode");
  return CPZ_OK;
}

int cpz_decode_points(cpz_ctx* ctx, size_t n, const uint8_t* points, uint8_t* ok_out, uint8_t* reencoded_out) {
  if (!ctx || !points || !ok_out) return fail(CPZ_EINVAL, "null argument");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = order_after_last(ctx, ctx->stream);
  if (rc) return rc;
  CPZ_HIP(ctx->in[0].ensure(n * 32));
  CPZ_HIP(ctx->in[1].ensure(n * 32));
  CPZ_HIP(ctx->st.ensure(n));
  CPZ_HIP(hipMemcpyAsync(ctx->in[0].p, points, n * 32, hipMemcpyHostToDevice, ctx->stream));
  CPZ_HIP(cpz::launch_decode_encode((int64_t)n, static_cast<const uint32_t*>(ctx->in[0].p),
                                    static_cast<uint8_t*>(ctx->st.p),
                                    reencoded_out ? static_cast<uint32_t*>(ctx->in[1].p) : nullptr, ctx->stream));
  CPZ_HIP(hipMemcpyAsync(ok_out, ctx->st.p, n, hipMemcpyDeviceToHost, ctx->stream));
  if (reencoded_out) CPZ_HIP(hipMemcpyAsync(reencoded_out, ctx->in[1].p, n * 32, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  return CPZ_OK;
}

int cpz_combine_partials(cpz_ctx* ctx, size_t k, const uint8_t* partials, uint8_t out[32], int* is_identity) {
  if (!ctx || !partials || !out || k == 0 || k > 4096) return fail(CPZ_EINVAL, "bad arguments");
  // A shard whose fallback found it dense skipped its MSM and reports the no-partial marker
  // (cpz_verify_batch): the batch cannot pass, and the sum is the marker too.
  for (size_t j = 0; j < k; j++)
    if (is_no_partial(partials + 32 * j)) {
      std::memset(out, 0xff, 32);
      if (is_identity) *is_identity = 0;
      return CPZ_OK;
    }
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  {
    int rc = order_after_last(ctx, ctx->stream);  // rl_flags is shared with the batch path
    if (rc) return rc;
  }
  CPZ_HIP(ctx->rl_parts.ensure(k * 32 + 64));
  CPZ_HIP(ctx->rl_flags.ensure(4 * sizeof(int)));
  CPZ_HIP(hipMemcpyAsync(ctx->rl_parts.p, partials, k * 32, hipMemcpyHostToDevice, ctx->stream));
  uint32_t* outw = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->rl_parts.p) + k * 32);
  CPZ_HIP(cpz::launch_rlc_combine(static_cast<const uint32_t*>(ctx->rl_parts.p), (int)k, outw,
                                  static_cast<int*>(ctx->rl_flags.p), ctx->stream));
  int flags[2];
  CPZ_HIP(hipMemcpyAsync(out, outw, 32, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipMemcpyAsync(flags, ctx->rl_flags.p, sizeof(flags), hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  if (!flags[0]) return fail(CPZ_EINVAL, "a partial does not decode");
  if (is_identity) *is_identity = flags[1];
  return CPZ_OK;
}

// ---- single-process multi-GPU ------------------------------------------------------------
}  // extern "C" (the helpers below are C++)

namespace {

constexpr size_t kShardAlign = cpz::kRlcPrepBlock;  // shard boundaries on weight blocks

// [lo, hi) of shard k of nctx (chaum_pedersen/shard.py:shard_range).
void shard_bounds(size_t n, int nctx, int k, size_t& lo, size_t& hi) {
  const size_t units = (n + kShardAlign - 1) / kShardAlign;
  lo = std::min(units * (size_t)k / (size_t)nctx * kShardAlign, n);
  hi = std::min(units * (size_t)(k + 1) / (size_t)nctx * kShardAlign, n);
}

// Runs fn(k, lo, hi) for every non-empty shard on its own thread; returns the first failing
// shard's code with its message moved to the calling thread.
template <class Fn>
int run_shards(int nctx, size_t n, Fn fn) {
  std::vector<int> rc(nctx, CPZ_OK);
  std::vector<std::string> msg(nctx);
  std::vector<std::thread> th;
  for (int k = 0; k < nctx; k++) {
    size_t lo, hi;
    shard_bounds(n, nctx, k, lo, hi);
    if (hi <= lo) continue;
    th.emplace_back([&, k, lo, hi] {
      rc[k] = fn(k, lo, hi);
      if (rc[k] != CPZ_OK) msg[k] = cpz_last_error();
    });
  }
  for (auto& t : th) t.join();
  for (int k = 0; k < nctx; k++)
    if (rc[k] != CPZ_OK) return fail(rc[k], "shard " + std::to_string(k) + ": " + msg[k]);
  return CPZ_OK;
}

int check_multi(cpz_ctx* const* ctxs, int nctx) {
  if (!ctxs || nctx <= 0) return fail(CPZ_EINVAL, "no contexts");
  for (int k = 0; k < nctx; k++)
    if (!ctxs[k]) return fail(CPZ_EINVAL, "null context in the list");
  for (int a = 0; a < nctx; a++)
    for (int b = a + 1; b < nctx; b++)
      if (ctxs[a] == ctxs[b]) return fail(CPZ_EINVAL, "a context appears twice (one context per shard)");
  return CPZ_OK;
}

}  // namespace

extern "C" {

int cpz_verify_each_multi(cpz_ctx* const* ctxs, int nctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                          const uint8_t* y1, const uint8_t* y2, const uint8_t* r1, const uint8_t* r2,
                          const uint8_t* s, const uint8_t* ctx_bytes, const uint64_t* ctx_off,
                          const uint8_t* ctx_present, uint8_t* status_out) {
  int rc = check_multi(ctxs, nctx);
  if (rc) return rc;
  if (!g || !h) return fail(CPZ_EINVAL, "null generators");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!y1 || !y2 || !r1 || !r2 || !s || !status_out) return fail(CPZ_EINVAL, "null input pointer");
  return run_shards(nctx, n, [&](int k, size_t lo, size_t hi) {
    // ctx_off keeps absolute offsets into ctx_bytes: the shard passes its n + 1 slice
    return cpz_verify_each(ctxs[k], g, h, hi - lo, y1 + 32 * lo, y2 + 32 * lo, r1 + 32 * lo, r2 + 32 * lo,
                           s + 32 * lo, ctx_bytes, ctx_off ? ctx_off + lo : nullptr,
                           ctx_present ? ctx_present + lo : nullptr, status_out + lo);
  });
}

int cpz_verify_batch_multi(cpz_ctx* const* ctxs, int nctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                           const uint8_t* y1, const uint8_t* y2, const uint8_t* r1, const uint8_t* r2,
                           const uint8_t* s, const uint8_t* ctx_bytes, const uint64_t* ctx_off,
                           const uint8_t* ctx_present, const uint8_t seed[32], uint8_t* partials_out,
                           uint8_t total_out[32], int* batch_ok, uint8_t* status_out) {
  int rc = check_multi(ctxs, nctx);
  if (rc) return rc;
  if (!g || !h || !seed || !partials_out || !total_out || !batch_ok) return fail(CPZ_EINVAL, "null argument");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!y1 || !y2 || !r1 || !r2 || !s) return fail(CPZ_EINVAL, "null input pointer");
  std::memset(partials_out, 0, (size_t)nctx * 32);  // empty shards contribute the identity
  std::vector<int> ok(nctx, 1);
  rc = run_shards(nctx, n, [&](int k, size_t lo, size_t hi) {
    return cpz_verify_batch(ctxs[k], g, h, hi - lo, y1 + 32 * lo, y2 + 32 * lo, r1 + 32 * lo, r2 + 32 * lo,
                            s + 32 * lo, ctx_bytes, ctx_off ? ctx_off + lo : nullptr,
                            ctx_present ? ctx_present + lo : nullptr, seed, (uint64_t)lo, partials_out + 32 * k,
                            &ok[k], status_out ? status_out + lo : nullptr);
  });
  if (rc) return rc;
  int ident = 0;
  rc = cpz_combine_partials(ctxs[0], (size_t)nctx, partials_out, total_out, &ident);
  if (rc) return rc;
  int all = ident;
  for (int k = 0; k < nctx; k++) all = all && ok[k];
  *batch_ok = all ? 1 : 0;
  return CPZ_OK;
}

int cpz_ctx_set_timing(cpz_ctx* ctx, int enable) {
  if (!ctx) return fail(CPZ_EINVAL, "null context");
  CallLock lock(ctx);
  ctx->timing = enable != 0;
  return CPZ_OK;
}

int cpz_ctx_stage_times(cpz_ctx* ctx, double ms_out[CPZ_NUM_STAGES], int launches_out[CPZ_NUM_STAGES]) {
  return cpz_ctx_stage_times_n(ctx, CPZ_NUM_STAGES, ms_out, launches_out);
}

int cpz_ctx_stage_times_n(cpz_ctx* ctx, int nstages, double* ms_out, int* launches_out) {
  if (!ctx || !ms_out || nstages <= 0) return fail(CPZ_EINVAL, "null argument or no stages");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  for (int k = 0; k < nstages; k++) {
    ms_out[k] = 0.0;
    if (launches_out) launches_out[k] = 0;
  }
  std::vector<hipEvent_t> done;  // consecutive RLC phase marks share events: return each once
  for (auto& m : ctx->marks) {
    CPZ_HIP(hipEventSynchronize(m.b));
    float ms = 0.f;
    CPZ_HIP(hipEventElapsedTime(&ms, m.a, m.b));
    if (m.stage >= 0 && m.stage < nstages) {
      ms_out[m.stage] += ms;
      if (launches_out) launches_out[m.stage] += 1;
    }
    done.push_back(m.a);
    done.push_back(m.b);
  }
  std::sort(done.begin(), done.end());
  done.erase(std::unique(done.begin(), done.end()), done.end());
  ctx->free_events.insert(ctx->free_events.end(), done.begin(), done.end());
  ctx->marks.clear();
  return CPZ_OK;
}

void cpz_ctx_destroy(cpz_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  {
    std::vector<hipEvent_t> all(ctx->free_events);
    for (auto& m : ctx->marks) {
      all.push_back(m.a);
      all.push_back(m.b);
    }
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    for (auto e : all) (void)hipEventDestroy(e);
  }
  if (ctx->last_done) (void)hipEventDestroy(ctx->last_done);
  for (GenSet& e : ctx->gen) e.release();
  ctx->ok_flags.release();
  ctx->c.release();
  ctx->st.release();
  ctx->scratch.release();
  for (auto& b : ctx->in) b.release();
  ctx->in_all.release();
  ctx->pin.release();
  ctx->ctxb.release();
  ctx->ctxo.release();
  ctx->ctxp.release();
  if (ctx->copy_done) (void)hipEventDestroy(ctx->copy_done);
  if (ctx->probe_done) (void)hipEventDestroy(ctx->probe_done);
  if (ctx->probe_stream) {
    (void)hipStreamSynchronize(ctx->probe_stream);
    (void)hipStreamDestroy(ctx->probe_stream);
  }
  ctx->probe.release();
  if (ctx->aux_start) (void)hipEventDestroy(ctx->aux_start);
  for (auto& e : ctx->aux_done)
    if (e) (void)hipEventDestroy(e);
  for (auto& a : ctx->aux_stream)
    if (a) {
      (void)hipStreamSynchronize(a);
      (void)hipStreamDestroy(a);
    }
  if (ctx->copy_stream) {
    (void)hipStreamSynchronize(ctx->copy_stream);
    (void)hipStreamDestroy(ctx->copy_stream);
  }
  for (DevBuf* b : {&ctx->pz_blob, &ctx->pz_off, &ctx->pz_rows, &ctx->pz_code, &ctx->pz_aux}) b->release();
  if (ctx->span_stream) {
    (void)hipStreamSynchronize(ctx->span_stream);
    (void)hipStreamDestroy(ctx->span_stream);
  }
  for (auto& e : ctx->span_ev)
    if (e) (void)hipEventDestroy(e);
  ctx->rl_prep.release();
  ctx->rl_msm.release();
  ctx->rl_msm2.release();
  ctx->rl_span_ident.release();
  for (DevBuf* b : {&ctx->pt_lists, &ctx->pt_offs, &ctx->pt_wsum, &ctx->pt_part, &ctx->pt_fail, &ctx->pt_tmp,
                    &ctx->pt_blocks, &ctx->pt_assign, &ctx->pt_ldig, &ctx->pt_lsum, &ctx->pt_lpart, &ctx->pt_lfail,
                    &ctx->pt_loc})
    b->release();
  ctx->rl_flags.release();
  ctx->rl_parts.release();
#if defined(CPZ_CLOCK_PROBE)
  for (DevBuf& b : ctx->clk) b.release();
#endif
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->device >= 0 && ctx->device < 64) g_own_queues[ctx->device].fetch_sub(ctx->own_queues);
  delete ctx;
}

namespace {

// Host-buffer per-proof verification in chunks of kPipeChunk proofs: the five input
// arrays of chunk j + 1 are copied (pageable H2D, on ctx->copy_stream) while chunk j's
// challenge + verify kernels run on ctx->stream, which waits on an event recorded after
// each chunk's copies.  Each chunk lands at its own offset of the full-size device arrays,
// so no copy overwrites data a queued kernel still reads.  Contexts (if any) are staged
// whole first; chunk j passes its slice of the offsets / presence flags (the offsets stay
// relative to the staged blob).  Statuses come back in one D2H copy at the end.
int verify_each_pipelined(cpz_ctx* ctx, size_t n, const uint8_t* const host[5], const uint8_t* ctx_bytes,
                          const uint64_t* ctx_off, const uint8_t* ctx_present, uint8_t* status_out) {
  const void* unused[5];
  const void* dcb;
  const uint64_t* dco;
  const uint8_t* dcp;
  int rc = stage_inputs(ctx, n, host, 0, ctx_bytes, ctx_off, ctx_present, unused, &dcb, &dco, &dcp);
  if (rc) return rc;
  for (int k = 0; k < 5; k++) CPZ_HIP(ctx->in[k].ensure(n * 32));
  CPZ_HIP(ctx->st.ensure(n));
  CPZ_HIP(ctx->c.ensure(n * 32));  // each chunk's challenges at its own offset
  VerifyRR rr;
  if (!ctx->copy_stream) CPZ_HIP(stream_own_queue(&ctx->copy_stream, ctx->cus, ctx->device, &ctx->own_queues));
  if (!ctx->copy_done) CPZ_HIP(hipEventCreateWithFlags(&ctx->copy_done, hipEventDisableTiming));
  uint8_t* st = static_cast<uint8_t*>(ctx->st.p);
  for (size_t off = 0; off < n; off += kPipeChunk) {
    const size_t m = (n - off) < kPipeChunk ? (n - off) : kPipeChunk;
    uint8_t* d[5];
    for (int k = 0; k < 5; k++) {
      d[k] = static_cast<uint8_t*>(ctx->in[k].p) + off * 32;
      CPZ_HIP(hipMemcpyAsync(d[k], host[k] + off * 32, m * 32, hipMemcpyHostToDevice, ctx->copy_stream));
    }
    CPZ_HIP(hipEventRecord(ctx->copy_done, ctx->copy_stream));
    CPZ_HIP(hipStreamWaitEvent(ctx->stream, ctx->copy_done, 0));
    rc = enqueue_verify(ctx, m, d[0], d[1], d[2], d[3], d[4], dcb, dco ? dco + off : nullptr,
                        dcp ? dcp + off : nullptr, st + off, ctx->stream,
                        static_cast<uint32_t*>(ctx->c.p) + 8 * off, &rr, false);
    if (rc) {
      (void)join_verify_streams(ctx, ctx->stream);
      (void)hipStreamSynchronize(ctx->stream);
      return rc;
    }
  }
  rc = join_verify_streams(ctx, ctx->stream);
  if (rc) return rc;
  CPZ_HIP(hipMemcpyAsync(status_out, st, n, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  return CPZ_OK;
}

}  // namespace

int cpz_verify_each_device(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const void* d_y1,
                           const void* d_y2, const void* d_r1, const void* d_r2, const void* d_s,
                           const void* d_ctx_bytes, const uint64_t* d_ctx_off, const uint8_t* d_ctx_present,
                           void* d_status_out, void* stream) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!d_y1 || !d_y2 || !d_r1 || !d_r2 || !d_s || !d_status_out) return fail(CPZ_EINVAL, "null input pointer");
  if (!aligned16(d_y1) || !aligned16(d_y2) || !aligned16(d_r1) || !aligned16(d_r2) || !aligned16(d_s))
    return fail(CPZ_EINVAL, "device inputs must be 16-byte aligned");
  if (d_ctx_off && !d_ctx_bytes) return fail(CPZ_EINVAL, "ctx_off given without ctx_bytes");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h, (int64_t)n > var_base_max(ctx));
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = order_after_last(ctx, st))) return rc;
  rc = enqueue_verify(ctx, n, d_y1, d_y2, d_r1, d_r2, d_s, d_ctx_bytes, d_ctx_off, d_ctx_present,
                      static_cast<uint8_t*>(d_status_out), st);
  if (rc) return rc;
  return record_last(ctx, st);
}

int cpz_verify_each(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                    const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s,
                    const uint8_t* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                    uint8_t* status_out) {
  return cpz_verify_each_ex(ctx, 0, g, h, n, y1, y2, r1, r2, s, ctx_bytes, ctx_off, ctx_present, status_out);
}

int cpz_verify_each_ex(cpz_ctx* ctx, uint32_t flags, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                    const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s,
                    const uint8_t* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present,
                    uint8_t* status_out) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!y1 || !y2 || !r1 || !r2 || !s || !status_out) return fail(CPZ_EINVAL, "null input pointer");
  if (ctx_off && !ctx_bytes && ctx_off[n] != ctx_off[0]) return fail(CPZ_EINVAL, "ctx_off given without ctx_bytes");
  CallLock lock(ctx, flags);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h, (int64_t)n > var_base_max(ctx));
  if (rc) return rc;
  if ((rc = order_after_last(ctx, ctx->stream))) return rc;
  const uint8_t* host[5] = {y1, y2, r1, r2, s};
  if (n > kPipeChunk) return verify_each_pipelined(ctx, n, host, ctx_bytes, ctx_off, ctx_present, status_out);
  const void* dev[5];
  const void* dcb;
  const uint64_t* dco;
  const uint8_t* dcp;
  uint8_t *st_dev = nullptr, *st_host = nullptr;
  rc = stage_inputs(ctx, n, host, 5, ctx_bytes, ctx_off, ctx_present, dev, &dcb, &dco, &dcp,
                    zero_copy() && (int64_t)n <= kSmallMax, &st_dev, &st_host);
  if (rc) return rc;
  if (st_dev) {  // zero-copy: inputs read and statuses written through the page-locked block
    rc = enqueue_verify(ctx, n, dev[0], dev[1], dev[2], dev[3], dev[4], dcb, dco, dcp, st_dev, ctx->stream);
    if (rc) return rc;
    CPZ_HIP(hipStreamSynchronize(ctx->stream));
    std::memcpy(status_out, st_host, n);
    return CPZ_OK;
  }
  CPZ_HIP(ctx->st.ensure(n));
  rc = enqueue_verify(ctx, n, dev[0], dev[1], dev[2], dev[3], dev[4], dcb, dco, dcp,
                      static_cast<uint8_t*>(ctx->st.p), ctx->stream);
  if (rc) return rc;
  // statuses through the page-locked block when stage_inputs used it (its inputs are spent)
  const bool pinned = ctx->pin.cap >= kPinMail + pad16(n);
  uint8_t* dst = pinned ? static_cast<uint8_t*>(ctx->pin.p) + kPinMail : status_out;
  CPZ_HIP(hipMemcpyAsync(dst, ctx->st.p, n, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  if (pinned) std::memcpy(status_out, dst, n);
  return CPZ_OK;
}

int cpz_challenges(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                   const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* ctx_bytes,
                   const uint64_t* ctx_off, const uint8_t* ctx_present, uint8_t* c_out) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  if (!y1 || !y2 || !r1 || !r2 || !c_out) return fail(CPZ_EINVAL, "null input pointer");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h, false);
  if (rc) return rc;
  if ((rc = order_after_last(ctx, ctx->stream))) return rc;
  const uint8_t* host[5] = {y1, y2, r1, r2, nullptr};
  const void* dev[5];
  const void* dcb;
  const uint64_t* dco;
  const uint8_t* dcp;
  rc = stage_inputs(ctx, n, host, 4, ctx_bytes, ctx_off, ctx_present, dev, &dcb, &dco, &dcp);
  if (rc) return rc;
  CPZ_HIP(ctx->c.ensure(n * 32));
  cpz::ChallengeArgs ca;
  set_challenge_schedules(ctx, ca);
  ca.n = (int64_t)n;
  words_from_bytes(ca.gh_words, ctx->gs->gh, ctx->gs->gh + 32);
  ca.y1 = static_cast<const uint32_t*>(dev[0]);
  ca.y2 = static_cast<const uint32_t*>(dev[1]);
  ca.r1 = static_cast<const uint32_t*>(dev[2]);
  ca.r2 = static_cast<const uint32_t*>(dev[3]);
  ca.s = nullptr;
  ca.ctx_bytes = static_cast<const uint8_t*>(dcb);
  ca.ctx_off = dco;
  ca.ctx_present = dcp;
  ca.prefix = static_cast<const cpz::StrobeSnap*>(ctx->gs->prefix.p);
  ca.c_out = static_cast<uint32_t*>(ctx->c.p);
  ca.status_out = nullptr;
  CPZ_HIP(cpz::launch_challenge(ca, ctx->stream));
  CPZ_HIP(hipMemcpyAsync(c_out, ctx->c.p, n * 32, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  return CPZ_OK;
}

int cpz_parse_proofs_device(cpz_ctx* ctx, size_t n, const void* d_blob, const uint64_t* d_off, void* d_r1,
                            void* d_r2, void* d_s, void* d_code, void* d_aux, void* stream) {
  if (!ctx) return fail(CPZ_EINVAL, "null context");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  if (!d_blob || !d_off || !d_r1 || !d_r2 || !d_s || !d_code) return fail(CPZ_EINVAL, "null input pointer");
  if (!aligned16(d_r1) || !aligned16(d_r2) || !aligned16(d_s))
    return fail(CPZ_EINVAL, "device row outputs must be 16-byte aligned");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  cpz::ParseArgs pa;
  pa.n = (int64_t)n;
  pa.blob = static_cast<const uint8_t*>(d_blob);
  pa.off = d_off;
  pa.r1 = static_cast<uint32_t*>(d_r1);
  pa.r2 = static_cast<uint32_t*>(d_r2);
  pa.s = static_cast<uint32_t*>(d_s);
  pa.code = static_cast<uint8_t*>(d_code);
  pa.aux = static_cast<uint32_t*>(d_aux);
  CPZ_HIP(cpz::launch_parse_proofs(pa, st));
  CPZ_HIP(hipStreamSynchronize(st));
  return CPZ_OK;
}

int cpz_parse_proofs(cpz_ctx* ctx, size_t n, const uint8_t* blob, const uint64_t* off, uint8_t* r1_out,
                     uint8_t* r2_out, uint8_t* s_out, uint8_t* code_out, uint32_t* aux_out) {
  if (!ctx) return fail(CPZ_EINVAL, "null context");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  if (!blob || !off || !r1_out || !r2_out || !s_out || !code_out) return fail(CPZ_EINVAL, "null input pointer");
  for (size_t i = 0; i < n; i++)
    if (off[i + 1] < off[i]) return fail(CPZ_EINVAL, "offsets must be non-decreasing");
  const size_t bytes = (size_t)(off[n] - off[0]);
  std::vector<uint64_t> rel(n + 1);
  for (size_t i = 0; i <= n; i++) rel[i] = off[i] - off[0];
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  CPZ_HIP(ctx->pz_blob.ensure(bytes + 16));
  CPZ_HIP(ctx->pz_off.ensure((n + 1) * sizeof(uint64_t)));
  CPZ_HIP(ctx->pz_rows.ensure(3 * n * 32));
  CPZ_HIP(ctx->pz_code.ensure(n));
  CPZ_HIP(ctx->pz_aux.ensure(n * sizeof(uint32_t)));
  if (bytes) CPZ_HIP(hipMemcpyAsync(ctx->pz_blob.p, blob + off[0], bytes, hipMemcpyHostToDevice, st));
  CPZ_HIP(hipMemcpyAsync(ctx->pz_off.p, rel.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  uint8_t* rows = static_cast<uint8_t*>(ctx->pz_rows.p);
  cpz::ParseArgs pa;
  pa.n = (int64_t)n;
  pa.blob = static_cast<const uint8_t*>(ctx->pz_blob.p);
  pa.off = static_cast<const uint64_t*>(ctx->pz_off.p);
  pa.r1 = reinterpret_cast<uint32_t*>(rows);
  pa.r2 = reinterpret_cast<uint32_t*>(rows + n * 32);
  pa.s = reinterpret_cast<uint32_t*>(rows + 2 * n * 32);
  pa.code = static_cast<uint8_t*>(ctx->pz_code.p);
  pa.aux = static_cast<uint32_t*>(ctx->pz_aux.p);
  CPZ_HIP(cpz::launch_parse_proofs(pa, st));
  CPZ_HIP(hipMemcpyAsync(r1_out, rows, n * 32, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(r2_out, rows + n * 32, n * 32, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(s_out, rows + 2 * n * 32, n * 32, hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipMemcpyAsync(code_out, ctx->pz_code.p, n, hipMemcpyDeviceToHost, st));
  if (aux_out) CPZ_HIP(hipMemcpyAsync(aux_out, ctx->pz_aux.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  CPZ_HIP(hipStreamSynchronize(st));
  return CPZ_OK;
}

}  // extern "C"

namespace {

// Prover::prove_with_transcript (prover/mod.rs:86-131) for n proofs on the device: x_i, k_i
// from the caller (d_x / d_k, mod l) or, when those are null, from ChaCha20(seed, first_index
// + i) (synthetic inputs).  y = x g, x h (gadgets.rs:217-221); r = k g, k h (commit,
// :115-121); c from the transcript (contexts as in verify); s = k + c x (respond, :126-131).
int prove_impl(cpz_ctx* ctx, size_t n, uint64_t first_index, const uint8_t* seed_x, const uint8_t* seed_k,
               const void* d_x, const void* d_k, const void* d_ctx_bytes, const uint64_t* d_ctx_off,
               const uint8_t* d_ctx_present, void* d_y1, void* d_y2, void* d_r1, void* d_r2, void* d_s,
               hipStream_t st) {
  CPZ_HIP(ctx->c.ensure(n * 32));
  cpz::ProveArgs pa;
  pa.n = (int64_t)n;
  pa.first_index = first_index;
  std::memset(pa.seed_x, 0, 32);
  std::memset(pa.seed_k, 0, 32);
  if (seed_x) std::memcpy(pa.seed_x, seed_x, 32);
  if (seed_k) std::memcpy(pa.seed_k, seed_k, 32);
  pa.x_in = static_cast<const uint32_t*>(d_x);
  pa.k_in = static_cast<const uint32_t*>(d_k);
  pa.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
  pa.y1 = static_cast<uint32_t*>(d_y1);
  pa.y2 = static_cast<uint32_t*>(d_y2);
  pa.r1 = static_cast<uint32_t*>(d_r1);
  pa.r2 = static_cast<uint32_t*>(d_r2);
  pa.c = static_cast<const uint32_t*>(ctx->c.p);
  pa.s_out = static_cast<uint32_t*>(d_s);
  {
    StageTimer t(ctx, 6, st);
    CPZ_HIP(cpz::launch_prove_points(pa, st));
  }
  cpz::ChallengeArgs ca;
  set_challenge_schedules(ctx, ca);
  ca.n = (int64_t)n;
  words_from_bytes(ca.gh_words, ctx->gs->gh, ctx->gs->gh + 32);
  ca.y1 = pa.y1;
  ca.y2 = pa.y2;
  ca.r1 = pa.r1;
  ca.r2 = pa.r2;
  ca.s = nullptr;
  ca.ctx_bytes = static_cast<const uint8_t*>(d_ctx_bytes);
  ca.ctx_off = d_ctx_off;
  ca.ctx_present = d_ctx_present;
  ca.prefix = static_cast<const cpz::StrobeSnap*>(ctx->gs->prefix.p);
  ca.c_out = static_cast<uint32_t*>(ctx->c.p);
  ca.status_out = nullptr;
  StageTimer t(ctx, 6, st);
  CPZ_HIP(cpz::launch_challenge(ca, st));
  CPZ_HIP(cpz::launch_prove_response(pa, st));
  return CPZ_OK;
}

bool rows_aligned(const void* const* p, int k) {
  for (int i = 0; i < k; i++)
    if (!aligned16(p[i])) return false;
  return true;
}

// Host-buffer prover: stage witnesses / nonces (or none) and contexts, prove on the device,
// copy the five rows back.
int prove_host(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, uint64_t first_index,
               const uint8_t* seed_x, const uint8_t* seed_k, const uint8_t* x, const uint8_t* k,
               const uint8_t* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present, uint8_t* y1, uint8_t* y2,
               uint8_t* r1, uint8_t* r2, uint8_t* s) {
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h);
  if (rc) return rc;
  if ((rc = order_after_last(ctx, ctx->stream))) return rc;
  const void* dcb = nullptr;
  const uint64_t* dco = nullptr;
  const uint8_t* dcp = nullptr;
  const void* unused[5];
  const uint8_t* none[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  rc = stage_inputs(ctx, n, none, 0, ctx_bytes, ctx_off, ctx_present, unused, &dcb, &dco, &dcp);
  if (rc) return rc;
  for (int q = 0; q < 5; q++) CPZ_HIP(ctx->in[q].ensure(n * 32));
  const void* dx = nullptr;
  const void* dk = nullptr;
  if (x) {
    CPZ_HIP(ctx->in[5].ensure(n * 32));
    CPZ_HIP(ctx->in[6].ensure(n * 32));
    CPZ_HIP(hipMemcpyAsync(ctx->in[5].p, x, n * 32, hipMemcpyHostToDevice, ctx->stream));
    CPZ_HIP(hipMemcpyAsync(ctx->in[6].p, k, n * 32, hipMemcpyHostToDevice, ctx->stream));
    dx = ctx->in[5].p;
    dk = ctx->in[6].p;
  }
  rc = prove_impl(ctx, n, first_index, seed_x, seed_k, dx, dk, dcb, dco, dcp, ctx->in[0].p, ctx->in[1].p,
                  ctx->in[2].p, ctx->in[3].p, ctx->in[4].p, ctx->stream);
  if (rc) return rc;
  uint8_t* outs[5] = {y1, y2, r1, r2, s};
  for (int q = 0; q < 5; q++)
    CPZ_HIP(hipMemcpyAsync(outs[q], ctx->in[q].p, n * 32, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  return CPZ_OK;
}

// Verifier::verify_response (verifier/mod.rs:144-171) with caller challenges c (device rows).
int verify_response_impl(cpz_ctx* ctx, size_t n, const void* y1, const void* y2, const void* r1, const void* r2,
                         const void* s, const void* c, uint8_t* status, hipStream_t st) {
  CPZ_HIP(ctx->c.ensure(n * 32));
  CPZ_HIP(cpz::launch_response_prep((int64_t)n, static_cast<const uint32_t*>(s), static_cast<const uint32_t*>(c),
                                    static_cast<uint32_t*>(ctx->c.p), status, ctx->call_eq ? 1 : 0, st));
  cpz::VerifyArgs va;
  va.n = (int64_t)n;
  va.y1 = static_cast<const uint32_t*>(y1);
  va.y2 = static_cast<const uint32_t*>(y2);
  va.r1 = static_cast<const uint32_t*>(r1);
  va.r2 = static_cast<const uint32_t*>(r2);
  va.s = static_cast<const uint32_t*>(s);
  va.c = static_cast<const uint32_t*>(ctx->c.p);
  va.status = status;
  va.comb = static_cast<const cpz::ge_niels*>(ctx->gs->comb.p);
  if (!ctx->gs->full) {  // a light set: variable-base generators (ensure_generators, n <= var_base_max)
    if ((int64_t)n > var_base_max(ctx)) return fail(CPZ_EINVAL, "internal: variable-base call above var_base_max");
    va.comb = nullptr;
    va.vtab = static_cast<const cpz::ge_niels*>(ctx->gs->tab.p);
    va.vtab16 = static_cast<const int32_t*>(ctx->gs->tab16.p);
  }
  va.scratch = nullptr;  // set per launch
  va.eq_only = ctx->call_eq ? 1 : 0;
  StageTimer span(ctx, 5, st);
  return launch_verify_chunks(ctx, va, 1, st, nullptr, true);
}

}  // namespace

extern "C" {

int cpz_prove_device(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const void* d_x,
                     const void* d_k, const void* d_ctx_bytes, const uint64_t* d_ctx_off, const uint8_t* d_ctx_present,
                     void* d_y1, void* d_y2, void* d_r1, void* d_r2, void* d_s, void* stream) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  const void* rows[7] = {d_x, d_k, d_y1, d_y2, d_r1, d_r2, d_s};
  for (const void* p : rows)
    if (!p) return fail(CPZ_EINVAL, "null input or output pointer");
  if (!rows_aligned(rows, 7)) return fail(CPZ_EINVAL, "device rows must be 16-byte aligned");
  if (d_ctx_off && !d_ctx_bytes) return fail(CPZ_EINVAL, "ctx_off given without ctx_bytes");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h);
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = order_after_last(ctx, st))) return rc;
  rc = prove_impl(ctx, n, 0, nullptr, nullptr, d_x, d_k, d_ctx_bytes, d_ctx_off, d_ctx_present, d_y1, d_y2, d_r1,
                  d_r2, d_s, st);
  if (rc) return rc;
  return record_last(ctx, st);
}

int cpz_prove(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* x, const uint8_t* k,
              const uint8_t* ctx_bytes, const uint64_t* ctx_off, const uint8_t* ctx_present, uint8_t* y1, uint8_t* y2,
              uint8_t* r1, uint8_t* r2, uint8_t* s) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  if (!x || !k || !y1 || !y2 || !r1 || !r2 || !s) return fail(CPZ_EINVAL, "null input or output pointer");
  if (ctx_off && !ctx_bytes && ctx_off[n] != ctx_off[0]) return fail(CPZ_EINVAL, "ctx_off given without ctx_bytes");
  return prove_host(ctx, g, h, n, 0, nullptr, nullptr, x, k, ctx_bytes, ctx_off, ctx_present, y1, y2, r1, r2, s);
}

int cpz_prove_synthetic_device(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n,
                               uint64_t first_index, const uint8_t seed_x[32], const uint8_t seed_k[32],
                               const void* d_ctx_bytes, const uint64_t* d_ctx_off, const uint8_t* d_ctx_present,
                               void* d_y1, void* d_y2, void* d_r1, void* d_r2, void* d_s, void* stream) {
  if (!ctx || !g || !h || !seed_x || !seed_k) return fail(CPZ_EINVAL, "null argument");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  if (!d_y1 || !d_y2 || !d_r1 || !d_r2 || !d_s) return fail(CPZ_EINVAL, "null output pointer");
  const void* rows[5] = {d_y1, d_y2, d_r1, d_r2, d_s};
  if (!rows_aligned(rows, 5)) return fail(CPZ_EINVAL, "device outputs must be 16-byte aligned");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h);
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = order_after_last(ctx, st))) return rc;
  rc = prove_impl(ctx, n, first_index, seed_x, seed_k, nullptr, nullptr, d_ctx_bytes, d_ctx_off, d_ctx_present, d_y1,
                  d_y2, d_r1, d_r2, d_s, st);
  if (rc) return rc;
  return record_last(ctx, st);
}

int cpz_prove_synthetic(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, uint64_t first_index,
                        const uint8_t seed_x[32], const uint8_t seed_k[32], const uint8_t* ctx_bytes,
                        const uint64_t* ctx_off, const uint8_t* ctx_present, uint8_t* y1, uint8_t* y2,
                        uint8_t* r1, uint8_t* r2, uint8_t* s) {
  if (!ctx || !g || !h || !seed_x || !seed_k) return fail(CPZ_EINVAL, "null argument");
  if (n == 0) return fail(CPZ_EEMPTY, "empty input");
  if (!y1 || !y2 || !r1 || !r2 || !s) return fail(CPZ_EINVAL, "null output pointer");
  return prove_host(ctx, g, h, n, first_index, seed_x, seed_k, nullptr, nullptr, ctx_bytes, ctx_off, ctx_present, y1,
                    y2, r1, r2, s);
}

int cpz_verify_response_device(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const void* d_y1,
                               const void* d_y2, const void* d_r1, const void* d_r2, const void* d_s, const void* d_c,
                               void* d_status_out, void* stream) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  const void* rows[6] = {d_y1, d_y2, d_r1, d_r2, d_s, d_c};
  for (const void* p : rows)
    if (!p) return fail(CPZ_EINVAL, "null input pointer");
  if (!d_status_out) return fail(CPZ_EINVAL, "null output pointer");
  if (!rows_aligned(rows, 6)) return fail(CPZ_EINVAL, "device inputs must be 16-byte aligned");
  CallLock lock(ctx);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h, (int64_t)n > var_base_max(ctx));
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = order_after_last(ctx, st))) return rc;
  rc = verify_response_impl(ctx, n, d_y1, d_y2, d_r1, d_r2, d_s, d_c, static_cast<uint8_t*>(d_status_out), st);
  if (rc) return rc;
  return record_last(ctx, st);
}

int cpz_verify_response(cpz_ctx* ctx, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                        const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s, const uint8_t* c,
                        uint8_t* status_out) {
  return cpz_verify_response_ex(ctx, 0, g, h, n, y1, y2, r1, r2, s, c, status_out);
}

int cpz_verify_response_ex(cpz_ctx* ctx, uint32_t flags, const uint8_t g[32], const uint8_t h[32], size_t n, const uint8_t* y1,
                        const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s, const uint8_t* c,
                        uint8_t* status_out) {
  if (!ctx || !g || !h) return fail(CPZ_EINVAL, "null context or generators");
  if (n == 0) return fail(CPZ_EEMPTY, "Cannot verify empty batch");
  if (!y1 || !y2 || !r1 || !r2 || !s || !c || !status_out) return fail(CPZ_EINVAL, "null input pointer");
  CallLock lock(ctx, flags);
  CPZ_HIP(hipSetDevice(ctx->device));
  int rc = ensure_generators(ctx, g, h, (int64_t)n > var_base_max(ctx));
  if (rc) return rc;
  if ((rc = order_after_last(ctx, ctx->stream))) return rc;
  const uint8_t* host[5] = {y1, y2, r1, r2, s};
  const void* dev[5];
  const void* dcb;
  const uint64_t* dco;
  const uint8_t* dcp;
  rc = stage_inputs(ctx, n, host, 5, nullptr, nullptr, nullptr, dev, &dcb, &dco, &dcp);
  if (rc) return rc;
  CPZ_HIP(ctx->in[5].ensure(n * 32));
  CPZ_HIP(hipMemcpyAsync(ctx->in[5].p, c, n * 32, hipMemcpyHostToDevice, ctx->stream));
  CPZ_HIP(ctx->st.ensure(n));
  rc = verify_response_impl(ctx, n, dev[0], dev[1], dev[2], dev[3], dev[4], ctx->in[5].p,
                            static_cast<uint8_t*>(ctx->st.p), ctx->stream);
  if (rc) return rc;
  CPZ_HIP(hipMemcpyAsync(status_out, ctx->st.p, n, hipMemcpyDeviceToHost, ctx->stream));
  CPZ_HIP(hipStreamSynchronize(ctx->stream));
  return CPZ_OK;
}

}  // extern "C"
