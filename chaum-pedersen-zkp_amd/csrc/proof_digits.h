// Loads, the LDS sponge image and the per-proof digit computation (challenge, response checks,
// split, recodings) shared by kernels.hip's k_verify_small and wide.hip's k_verify_wide.
#pragma once
#include <hip/hip_runtime.h>

#include "cpz_kernels.h"
#include "keccak_wave.h"
#include "scalar25519.h"
#include "transcript.h"
#include "verify.h"

namespace cpz {

__device__ __forceinline__ void load_words8(uint32_t w[8], const uint32_t* base, int64_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(base + 8 * i);
  const uint4 a = p[0], b = p[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// ---------------------------------------------------------------------------------------
// Transcript: per-thread STROBE image in LDS, dword-interleaved across the block so the
// Keccak load/store of all threads is bank-conflict free.
// ---------------------------------------------------------------------------------------
struct LdsState {
  uint32_t* base;  // __shared__ uint32_t[50 * T]
  int tid;
  int T;
  __device__ __forceinline__ uint8_t* byte_ptr(int i) const {
    return reinterpret_cast<uint8_t*>(base + (i >> 2) * T + tid) + (i & 3);
  }
  __device__ __forceinline__ uint8_t get(int i) const { return *byte_ptr(i); }
  __device__ __forceinline__ void put(int i, uint8_t v) { *byte_ptr(i) = v; }
  __device__ __forceinline__ void xor_(int i, uint8_t v) { *byte_ptr(i) ^= v; }
  __device__ __forceinline__ void permute() {
    uint64_t a[25];
#pragma unroll
    for (int l = 0; l < 25; l++)
      a[l] = (uint64_t)base[(2 * l) * T + tid] | ((uint64_t)base[(2 * l + 1) * T + tid] << 32);
    keccak_f1600(a);
#pragma unroll
    for (int l = 0; l < 25; l++) {
      base[(2 * l) * T + tid] = (uint32_t)a[l];
      base[(2 * l + 1) * T + tid] = (uint32_t)(a[l] >> 32);
    }
  }
};

// ---------------------------------------------------------------------------------------
// The drop-in's own regime (a BatchVerifier batch, at most 1000 entries): a call is one
// dependent chain -- challenge, decodes, tables, 124 doublings, additions -- so its latency is
// the longest chain, not the work.  k_verify_small splits each proof's chain over three waves of
// one workgroup (8 proofs per workgroup, a quad per (proof, equation) in each wave):
//   wave 0  decodes Y of each equation (lane 0 of the quad), builds the table of -Y in LDS,
//           then [u] (-Y): 124 doublings + 32 additions;
//   wave 1  the same for R: the table of +R, then [|v|] (-+R) (digits negated unless v < 0);
//   wave 2  the transcript challenge (fixed schedules without a context or with a 32-byte one;
//           the byte-wise sponge on one lane per proof otherwise), the response checks, the
//           challenge split and recodings -- while waves 0 and 1 decode -- then [s'] B: 16 comb
//           additions, or with variable-base generators (VerifyArgs::vtab) 120 doublings and
//           32 Niels additions, beside waves 0 and 1's loops.
// k_verify_quad ran all of it on one quad per equation: the challenge in a separate launch,
// then decode, both tables, 124 doublings + 64 additions, the 16 comb additions in sequence.
// The waves meet at two barriers (digits ready; partial sums ready), and wave 0 adds the three
// partial sums and writes the statuses (verify_proof's precedence).  a.c != nullptr: the
// challenges and response statuses were computed before (cpz_verify_response, or the
// challenge kernel), wave 2 only splits.
// ---------------------------------------------------------------------------------------
// The transcript challenge, response checks, challenge split and digit words of proof ii
// (k_verify_small's wave 2, k_verify_wide's wave 4): dig = u (0..3) and |v| (4..7) as radix-16
// signed digits, s' = v s mod l (8..15) as radix-2^16 digits (radix-256 with variable-base
// tables); meta bit 0 = v < 0, bits 8..15 = the response status.  With a.c the challenge and
// status were computed before.  The fixed transcript schedules (no context, 32-byte context)
// run on every lane; any other context runs the byte-wise sponge on the lanes with
// `sponge_lane` set, on column `col` of the LDS image `sponge` (50 x ncols words) -- the other
// lanes' results are then meaningless and the caller takes the sponge lane's from LDS.
template <bool kWave = false>
__device__ __forceinline__ void proof_digits(uint32_t dig[16], uint32_t& meta, const VerifyArgs& a,
                                             const ChallengeArgs& ca, int64_t ii, bool sponge_lane,
                                             uint32_t* sponge, int col, int ncols,
                                             uint64_t* stamp_challenge = nullptr) {
  uint32_t sw[8], cw[8];
  load_words8(sw, a.s, ii);
  uint8_t st_s;
  if (a.c) {
    load_words8(cw, a.c, ii);
    st_s = a.status[ii];
  } else {
    uint32_t y1[8], y2[8], r1[8], r2[8];
    load_words8(y1, a.y1, ii);
    load_words8(y2, a.y2, ii);
    load_words8(r1, a.r1, ii);
    load_words8(r2, a.r2, ii);
    const bool has_ctx = ca.ctx_off != nullptr && (ca.ctx_present == nullptr || ca.ctx_present[ii] != 0);
    const uint64_t b0 = has_ctx ? ca.ctx_off[ii] : 0, b1 = has_ctx ? ca.ctx_off[ii + 1] : 0;
    const bool fixed_noctx = !has_ctx && ca.fast_noctx;
    const bool fixed_ctx32 = has_ctx && ca.fast_ctx32 && b1 - b0 == 32 &&
                             ((reinterpret_cast<uintptr_t>(ca.ctx_bytes) + b0) & 3) == 0;
    sc c;
    if (fixed_noctx) {
      const uint32_t* pre = reinterpret_cast<const uint32_t*>(ca.prefix[1].state);
      if constexpr (kWave)
        c = challenge_fixed(pre, ca.k1, ca.k2, y1, y2, r1, r2, PermRows{sponge, (int)(threadIdx.x & 63)});
      else
        c = challenge_fixed(pre, ca.k1, ca.k2, y1, y2, r1, r2);
    } else if (fixed_ctx32) {
      uint32_t cx[8];
      const uint32_t* cp = reinterpret_cast<const uint32_t*>(ca.ctx_bytes + b0);
#pragma unroll
      for (int k = 0; k < 8; k++) cx[k] = cp[k];
      const uint32_t* pre = reinterpret_cast<const uint32_t*>(ca.prefix[0].state);
      if constexpr (kWave)
        c = challenge_fixed_ctx32(pre, ca.c32, cx, y1, y2, r1, r2, PermRows{sponge, (int)(threadIdx.x & 63)});
      else
        c = challenge_fixed_ctx32(pre, ca.c32, cx, y1, y2, r1, r2);
    } else {
      for (int k = 0; k < 8; k++) c.w[k] = 0;
      if (sponge_lane) {
        LdsState lst{sponge, col, ncols};
        const StrobeSnap& snap = ca.prefix[has_ctx ? 0 : 1];
        const uint32_t* src = reinterpret_cast<const uint32_t*>(snap.state);
        for (int k = 0; k < 50; k++) sponge[k * ncols + col] = src[k];
        Strobe<LdsState> st(lst, snap.pos, snap.pos_begin, (uint8_t)snap.flags);
        if (has_ctx) {
          transcript_context(st, ca.ctx_bytes + b0, (uint32_t)(b1 - b0));
          transcript_parameters(st, ca.gh_words, ca.gh_words + 8);
        }
        c = transcript_challenge(st, y1, y2, r1, r2);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) cw[k] = c.w[k];
    st_s = response_status(sw, ca.eq_only != 0);
  }
  if (stamp_challenge) *stamp_challenge = __builtin_amdgcn_s_memtime();  // timing builds only
  if constexpr (kWave) {
    // the byte-wise sponge ran on the first lane alone; the split's rows are shared by lanes
#pragma unroll
    for (int k = 0; k < 8; k++) cw[k] = __builtin_amdgcn_readfirstlane(cw[k]);
  }
  bool vneg;
  uint32_t u[4], va[4];
  if (kWave)
    sc_half_split32<true>(cw, u, va, vneg);
  else
    sc_half_split(cw, u, va, vneg);
  sc_recode_radix16_half(dig, u);
  sc_recode_radix16_half(dig + 4, va);
  sc vs, ss;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    vs.w[k] = k < 4 ? va[k] : 0u;
    ss.w[k] = sw[k];
  }
  sc sp = sc_mul(vs, ss);
  if (vneg) sp = sc_neg(sp);
  if (a.vtab)
    sc_recode_radix256(dig + 8, sp.w);
  else
    sc_recode_radix65536(dig + 8, sp.w);
  meta = (vneg ? 1u : 0u) | ((uint32_t)st_s << 8);
}

}  // namespace cpz
