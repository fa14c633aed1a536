// Keccak-f[1600] spread over the lanes of one wave (k_verify_wide's wave 4, which computes
// ONE transcript challenge per workgroup).  Replaces, for that wave, the register form of
// transcript.h keccak_f1600 (the permutation of STROBE-128 under merlin, transcript.rs:29-71).
// Device-only; parity: tools/ubench/w4_parts.hip checks it against the register form, and
// k_verify_wide's challenges are compared with the oracle's in tests/test_gpu_scale.py.
#pragma once
#include <stdint.h>

#include "transcript.h"

namespace cpz {

// ---------------------------------------------------------------------------------------
// The layout: state lane j = x + 5 y (0..24) on wave lane j (lanes 25..63
// repeat lane j mod 25), 64 bits as (lo, hi).  theta's column sums, D's neighbours, pi's moves
// and chi's two neighbours are ds_bpermute reads of other lanes (18 per round); rho is a
// per-lane rotation.  chi's neighbours are read straight from pi's sources (B[x + 1, y] and
// B[x + 2, y] are rotated lanes of A like B[x, y]), so a round is three dependent exchange
// levels, not four (33.2 K against 35.2 K cycles for the challenge, profiles/r05_keccak_fused_ab.txt).  For k_verify_wide's wave 4, which computes ONE
// transcript challenge: on a lone wave the register form's ~190 instructions a round issue one
// after another, here each lane does ~30.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bperm(int src_lane_x4, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane_x4, (int)v);
}

// pi's source (x 4) of B[x, y]: A[(3 (y - 3 x)) % 5, x]... as a lane: (3 (y + 5 - 3 x % 5)) % 5 + 5 x
__device__ __forceinline__ int keccak_pi_src(int x, int y) { return 4 * ((3 * (y + 5 - (3 * x) % 5)) % 5 + 5 * x); }

__device__ __forceinline__ void keccak_lanes(uint32_t& lo, uint32_t& hi, int j) {
  constexpr int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                           25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  const int x = j % 5, y = j / 5;
  int r = 0;
#pragma unroll
  for (int k = 0; k < 25; k++) r = j == k ? rho[k] : r;
  const bool swap = (r & 32) != 0;
  const int rs = r & 31;
  // source lanes (x 4 for ds_bpermute): column mates, theta's neighbours, pi's source, chi's
  const int c1 = 4 * (x + 5 * ((y + 1) % 5)), c2 = 4 * (x + 5 * ((y + 2) % 5)), c3 = 4 * (x + 5 * ((y + 3) % 5)),
            c4 = 4 * (x + 5 * ((y + 4) % 5));
  const int dm = 4 * ((x + 4) % 5), dp = 4 * ((x + 1) % 5);
  const int pi = keccak_pi_src(x, y);  // B[X = x, Y = y] <- A[(3 (Y - 3 X)) % 5, X]
  const int h1 = keccak_pi_src((x + 1) % 5, y), h2 = keccak_pi_src((x + 2) % 5, y);  // B[x+1, y], B[x+2, y]
#pragma unroll 1
  for (int round = 0; round < 24; round++) {
    // theta: C[x] (every lane of column x), D[x] = C[x-1] ^ rot(C[x+1], 1)
    uint64_t c = ((uint64_t)hi << 32) | lo;
    c = bitop3_64<kXor3>(c, ((uint64_t)bperm(c1, hi) << 32) | bperm(c1, lo),
                         ((uint64_t)bperm(c2, hi) << 32) | bperm(c2, lo));
    c = bitop3_64<kXor3>(c, ((uint64_t)bperm(c3, hi) << 32) | bperm(c3, lo),
                         ((uint64_t)bperm(c4, hi) << 32) | bperm(c4, lo));
    const uint32_t cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
    const uint64_t cm = ((uint64_t)bperm(dm, ch) << 32) | bperm(dm, cl);
    const uint64_t cp = ((uint64_t)bperm(dp, ch) << 32) | bperm(dp, cl);
    uint64_t a = bitop3_64<kXor3>(((uint64_t)hi << 32) | lo, cm, rol64(cp, 1));
    // rho: rotate left by r (lane 0: r = 0)
    uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32);
    if (swap) {
      const uint32_t t = al;
      al = ah;
      ah = t;
    }
    const uint32_t nh = rs ? __builtin_amdgcn_alignbit(ah, al, 32 - rs) : ah;
    const uint32_t nl = rs ? __builtin_amdgcn_alignbit(al, ah, 32 - rs) : al;
    // pi: B[x, y] = rotated A of its source lane
    const uint32_t bl = bperm(pi, nl), bh = bperm(pi, nh);
    // chi: A = B ^ (~B[x + 1] & B[x + 2]); iota on lane 0
    const uint64_t b = ((uint64_t)bh << 32) | bl;
    const uint64_t b1 = ((uint64_t)bperm(h1, nh) << 32) | bperm(h1, nl);
    const uint64_t b2 = ((uint64_t)bperm(h2, nh) << 32) | bperm(h2, nl);
    uint64_t na = bitop3_64<kChi>(b, b1, b2);
    if (j == 0) na ^= KECCAK_RC(round);
    lo = (uint32_t)na;
    hi = (uint32_t)(na >> 32);
  }
}

// The fixed-schedule tails' permutation on a wave (challenge_fixed's Perm): the 50-word image
// (the same on every lane) goes to LDS, each lane takes its state lane, permutes, and the
// image comes back to every lane.  `lds` = 50 words of the workgroup's shared memory.
struct PermRows {
  uint32_t* lds;
  int lane;
  __device__ void operator()(uint32_t st[50]) const {
    const int j = lane % 25;
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 50; k++) lds[k] = st[k];
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t lo = lds[2 * j], hi = lds[2 * j + 1];
    __builtin_amdgcn_wave_barrier();
    keccak_lanes(lo, hi, j);
    if (lane < 25) {
      lds[2 * j] = lo;
      lds[2 * j + 1] = hi;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 50; k++) st[k] = lds[k];
    __builtin_amdgcn_wave_barrier();
  }
};

}  // namespace cpz
