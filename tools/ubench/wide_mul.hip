// Microbenchmark for the drop-in's latency (VERDICT r04 missing #2): how long one field
// product takes on the critical path of a lone wave, in two layouts.
//   r25   the product code (csrc/fe25519.h): one element per lane, ten signed limbs of
//         radix 2^25.5; a squaring is 55 v_mad_i64_i32 plus the 11-step carry chain, all
//         dependent work of one lane
//   r16   one element per 16-lane row, one 16-bit limb per lane (value = sum x_k 2^(16k)):
//         lane k accumulates column k = sum_i x_i * x_(k-i mod 16) (x 38 where the index
//         wraps, 2^256 = 38 mod p) from a row broadcast of x_i (DPP row_newbcast) and a
//         shifted x (two DPP moves, the wrapped lanes taking 38 x), 16 MADs per lane, then
//         three rounds of a parallel carry (DPP row_ror:1); r16b builds the shifted y
//         incrementally, r16c uses a two-level carry, r16p splits the columns over row pairs
//         (timed only: its rows 2k+1 repeat rows 2k's inputs)
// Both run chains of squarings from the same inputs on one wave per CU; the JSON lines give
// ns and shader cycles per squaring (one lane's chain / one row's chain), and the outputs
// are written to a file for tools/ubench/wide_mul_check.py to compare against Python's pow.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../chaum-pedersen-zkp_amd/csrc/fe25519.h"

#define CHECK(x)                                                                               \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

constexpr int kChain = 250;

// DPP move; lanes whose source is outside the row keep `old` (zero when old is 0 -- then the
// bound-control zero fill is used, so no copy of `old` is needed)
template <int C>
__device__ __forceinline__ int dpp(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, C, 0xf, 0xf, false);
}
template <int C>
__device__ __forceinline__ int dpp0(int x) {
  return __builtin_amdgcn_update_dpp(0, x, C, 0xf, 0xf, true);
}

// lane k of the row gets y_(k-i) for k >= i and 38 y_(k-i+16) for k < i
template <int I>
__device__ __forceinline__ int shifted(int y, int y38) {
  if constexpr (I == 0) {
    return y;
  } else {
    const int w = dpp0<0x100 + (16 - I)>(y38);  // row_shl:(16-i): lanes k < i
    return dpp<0x110 + I>(w, y);                    // row_shr:i, lanes k >= i; others keep w
  }
}

template <int I>
__device__ __forceinline__ void col_step(int64_t (&a)[4], int x, int y, int y38) {
  const int xi = dpp0<0x150 + I>(x);  // row_newbcast:i
  a[I & 3] += (int64_t)xi * (int64_t)shifted<I>(y, y38);
  if constexpr (I + 1 < 16) col_step<I + 1>(a, x, y, y38);
}

__device__ __forceinline__ int align16(int64_t v) {
  return (int)__builtin_amdgcn_alignbit((uint32_t)((uint64_t)v >> 32), (uint32_t)v, 16);
}

// x * y, both in r16 form with |limb| < 2^18.8; result limbs in (-2^11.5, 2^16 + 2^11.5).
// w = 38 on lane 0 of the row, 1 elsewhere.
__device__ __forceinline__ int r16_mul(int x, int y, int w) {
  int64_t a[4] = {0, 0, 0, 0};
  col_step<0>(a, x, y, y * 38);
  const int64_t acc = (a[0] + a[1]) + (a[2] + a[3]);  // |acc| < 16 * 38 * 2^37.6 < 2^47
  const int c1 = align16(acc);                        // floor(acc / 2^16)
  const int64_t t = (int64_t)dpp0<0x121>(c1) * w + (int64_t)((uint32_t)acc & 0xffffu);
  const int c2 = align16(t);
  const int u = ((int)(uint32_t)t & 0xffff) + dpp0<0x121>(c2) * w;
  const int c3 = u >> 16;
  return (u & 0xffff) + dpp0<0x121>(c3) * w;
}

// r16b: y's shifted copy built incrementally -- y^(i) = row_ror:1(y^(i-1)), lane 0 times 38
// (one v_mul_i32_i24 reading its source through DPP) -- and operands held to |limb| < 2^17.2
// so 38 y fits the 24-bit multiplier; per column step: broadcast, shifted y, MAD.
template <int I>
__device__ __forceinline__ void col_step_b(int64_t (&a)[4], int x, int yi, int w) {
  const int xi = dpp0<0x150 + I>(x);
  a[I & 3] += (int64_t)xi * (int64_t)yi;
  if constexpr (I + 1 < 16) col_step_b<I + 1>(a, x, __mul24(dpp0<0x121>(yi), w), w);
}

__device__ __forceinline__ int r16_mul_b(int x, int y, int w) {
  int64_t a[4] = {0, 0, 0, 0};
  col_step_b<0>(a, x, y, w);
  const int64_t acc = (a[0] + a[1]) + (a[2] + a[3]);
  const int c1 = align16(acc);
  const int64_t t = (int64_t)dpp0<0x121>(c1) * w + (int64_t)((uint32_t)acc & 0xffffu);
  const int c2 = align16(t);
  const int u = ((int)(uint32_t)t & 0xffff) + dpp0<0x121>(c2) * w;
  const int c3 = u >> 16;
  return (u & 0xffff) + dpp0<0x121>(c3) * w;
}

// r16c: the same columns, a two-level carry -- the column splits into three pieces
// (bits 0..15, 16..31, the signed high word), added into limbs k, k+1, k+2 at once through two
// DPP moves (38x where they wrap), then one parallel carry round: 6 dependent steps instead of
// three rounds of 3.
__device__ __forceinline__ int r16_mul_c(int x, int y, int w, int w2) {
  int64_t a[4] = {0, 0, 0, 0};
  col_step<0>(a, x, y, y * 38);
  const int64_t acc = (a[0] + a[1]) + (a[2] + a[3]);
  const uint32_t lo = (uint32_t)acc;
  const int p0 = (int)(lo & 0xffffu), p1 = (int)(lo >> 16), p2 = (int)(acc >> 32);
  const int u = p0 + __mul24(dpp0<0x121>(p1), w) + __mul24(dpp0<0x122>(p2), w2);  // row_ror:1, row_ror:2
  const int c = u >> 16;
  return (u & 0xffff) + dpp0<0x121>(c) * w;
}

// r16p: the column sums split over row pairs (fe16.h mul_pair, the decode's product): even
// rows i = 0..7, odd rows i = 8..15 from x rotated and y shifted by 8, one permlane16 swap adds
// the halves -- every row of a pair must hold the same value.
template <int I>
__device__ __forceinline__ void col_step_h(int64_t (&a)[4], int x, int y, int y38) {
  a[I & 3] += (int64_t)dpp0<0x150 + I>(x) * (int64_t)shifted<I>(y, y38);
  if constexpr (I + 1 < 8) col_step_h<I + 1>(a, x, y, y38);
}

__device__ __forceinline__ int r16_mul_p(int x, int y, int w, bool hi) {
  // DPP moves are convergent: computed on every lane, then selected (a conditional DPP
  // becomes a divergent branch)
  const int xr = dpp0<0x128>(x);                         // row_ror:8: lane j holds x_(j+8)
  const int yr = shifted<8>(y, y * 38);
  const int xs = hi ? xr : x;
  const int ys = hi ? yr : y;
  int64_t a[4] = {0, 0, 0, 0};
  col_step_h<0>(a, xs, ys, ys * 38);
  const int64_t h = (a[0] + a[1]) + (a[2] + a[3]);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)h, (uint32_t)h, false, false);
  const auto hw = __builtin_amdgcn_permlane16_swap((uint32_t)((uint64_t)h >> 32), (uint32_t)((uint64_t)h >> 32),
                                                   false, false);
  const int64_t acc = (int64_t)(((uint64_t)hw[0] << 32) | lo[0]) + (int64_t)(((uint64_t)hw[1] << 32) | lo[1]);
  const int c1 = align16(acc);
  const int64_t t = (int64_t)dpp0<0x121>(c1) * w + (int64_t)((uint32_t)acc & 0xffffu);
  const int c2 = align16(t);
  const int u = ((int)(uint32_t)t & 0xffff) + dpp0<0x121>(c2) * w;
  const int c3 = u >> 16;
  return (u & 0xffff) + dpp0<0x121>(c3) * w;
}

template <int V>
__global__ void __launch_bounds__(64) k_r16(const uint32_t* in, int32_t* out, int reps) {
  const int lane = threadIdx.x;
  const int row = lane >> 4, k = lane & 15;
  const int e = blockIdx.x * 4 + row;  // element index
  const uint32_t word = in[8 * e + (k >> 1)];
  int x = (int)((k & 1) ? (word >> 16) : (word & 0xffffu));
  const int w = k == 0 ? 38 : 1;
  const int w2 = k < 2 ? 38 : 1;
  const bool hi = (row & 1) != 0;
  if (V == 3) {  // the pair product needs the same value on both rows of a pair
    const uint32_t word0 = in[8 * (blockIdx.x * 4 + (row & 2)) + (k >> 1)];
    x = (int)((k & 1) ? (word0 >> 16) : (word0 & 0xffffu));
  }
  for (int r = 0; r < reps; r++) {
#pragma unroll 1
    for (int s = 0; s < kChain; s++)
      x = V == 1 ? r16_mul_b(x, x, w)
                 : (V == 2 ? r16_mul_c(x, x, w, w2) : (V == 3 ? r16_mul_p(x, x, w, hi) : r16_mul(x, x, w)));
  }
  out[16 * e + k] = x;
}

__global__ void __launch_bounds__(64) k_r25(const uint32_t* in, uint32_t* out, int reps) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = in[8 * t + i];
  cpz::fe a = cpz::fe_fromwords(w);
  for (int r = 0; r < reps; r++) a = cpz::fe_sqn(a, kChain);
  cpz::fe_towords(w, a);
  for (int i = 0; i < 8; i++) out[8 * t + i] = w[i];
}

int main(int argc, char** argv) {
  const char* dump = argc > 1 ? argv[1] : "wide_mul_out.bin";
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount;  // one wave per CU
  const int nelem = blocks * 64;
  std::vector<uint32_t> in((size_t)nelem * 8);
  uint64_t s = 88172645463325252ull;
  for (auto& v : in) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    v = (uint32_t)s;
  }
  for (int e = 0; e < nelem; e++) in[8 * e + 7] &= 0x7fffffffu;
  uint32_t *din, *d25;
  int32_t* d16;
  CHECK(hipMalloc(&din, in.size() * 4));
  CHECK(hipMalloc(&d25, in.size() * 4));
  CHECK(hipMalloc(&d16, (size_t)nelem * 16 * 4));
  CHECK(hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 40;
  const double chain = (double)reps * kChain;
  float ms25 = 0, ms16 = 0, ms16b = 0, ms16c = 0, ms16p = 0;
  auto timed = [&](auto kern, auto* out, float* ms) -> int {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, din, out, 1);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, din, out, reps);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(ms, e0, e1));
    return 0;
  };
  std::vector<int32_t> o16a((size_t)blocks * 4 * 16), o16c((size_t)blocks * 4 * 16);
  for (int pass = 0; pass < 2; pass++) {
    if (timed(k_r25, d25, &ms25)) return 1;
    if (timed(k_r16<0>, d16, &ms16)) return 1;
    CHECK(hipMemcpy(o16a.data(), d16, o16a.size() * 4, hipMemcpyDeviceToHost));
    if (timed(k_r16<2>, d16, &ms16c)) return 1;
    CHECK(hipMemcpy(o16c.data(), d16, o16c.size() * 4, hipMemcpyDeviceToHost));
    if (timed(k_r16<3>, d16, &ms16p)) return 1;
    if (timed(k_r16<1>, d16, &ms16b)) return 1;
    printf("{\"pass\": %d, \"chain\": %d, \"r25_ns_per_sq\": %.2f, \"r16_ns_per_sq\": %.2f, "
           "\"r16b_ns_per_sq\": %.2f, \"r16c_ns_per_sq\": %.2f, \"r16p_ns_per_sq\": %.2f}\n",
           pass, (int)chain, ms25 * 1e6 / chain, ms16 * 1e6 / chain, ms16b * 1e6 / chain, ms16c * 1e6 / chain,
           ms16p * 1e6 / chain);
  }
  // outputs after `reps` chains: r25 canonical words for elements 0..nelem-1; r16 limbs for
  // elements 0..4*blocks-1 (the first four of each block's inputs... element e = 4 b + row)
  std::vector<uint32_t> o25(in.size());
  std::vector<int32_t> o16((size_t)blocks * 4 * 16);
  CHECK(hipMemcpy(o25.data(), d25, o25.size() * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(o16.data(), d16, o16.size() * 4, hipMemcpyDeviceToHost));
  FILE* f = fopen(dump, "wb");
  if (!f) return 3;
  const int hdr[3] = {nelem, blocks * 4, reps * kChain};
  fwrite(hdr, 4, 3, f);
  fwrite(in.data(), 4, in.size(), f);
  fwrite(o25.data(), 4, o25.size(), f);
  fwrite(o16.data(), 4, o16.size(), f);
  fwrite(o16a.data(), 4, o16a.size(), f);
  fwrite(o16c.data(), 4, o16c.size(), f);
  fclose(f);
  return 0;
}
