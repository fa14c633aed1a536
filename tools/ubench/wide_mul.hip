// Microbenchmark for the drop-in's latency (VERDICT r04 missing #2): how long one field
// product takes on the critical path of a lone wave, in two layouts.
//   r25   the product code (csrc/fe25519.h): one element per lane, ten signed limbs of
//         radix 2^25.5; a squaring is 55 v_mad_i64_i32 plus the 11-step carry chain, all
//         dependent work of one lane
//   r16   one element per 16-lane row, one 16-bit limb per lane (value = sum x_k 2^(16k)):
//         lane k accumulates column k = sum_i x_i * x_(k-i mod 16) (x 38 where the index
//         wraps, 2^256 = 38 mod p) from a row broadcast of x_i (DPP row_newbcast) and a
//         shifted x (two DPP moves, the wrapped lanes taking 38 x), 16 MADs per lane, then
//         three rounds of a parallel carry (DPP row_ror:1)
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

template <bool kB>
__global__ void __launch_bounds__(64) k_r16(const uint32_t* in, int32_t* out, int reps) {
  const int lane = threadIdx.x;
  const int row = lane >> 4, k = lane & 15;
  const int e = blockIdx.x * 4 + row;  // element index
  const uint32_t word = in[8 * e + (k >> 1)];
  int x = (int)((k & 1) ? (word >> 16) : (word & 0xffffu));
  const int w = k == 0 ? 38 : 1;
  for (int r = 0; r < reps; r++) {
#pragma unroll 1
    for (int s = 0; s < kChain; s++) x = kB ? r16_mul_b(x, x, w) : r16_mul(x, x, w);
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
  float ms25 = 0, ms16 = 0, ms16b = 0;
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
  std::vector<int32_t> o16a((size_t)blocks * 4 * 16);
  for (int pass = 0; pass < 2; pass++) {
    if (timed(k_r25, d25, &ms25)) return 1;
    if (timed(k_r16<false>, d16, &ms16)) return 1;
    CHECK(hipMemcpy(o16a.data(), d16, o16a.size() * 4, hipMemcpyDeviceToHost));
    if (timed(k_r16<true>, d16, &ms16b)) return 1;
    printf("{\"pass\": %d, \"chain\": %d, \"r25_ns_per_sq\": %.2f, \"r16_ns_per_sq\": %.2f, "
           "\"r16b_ns_per_sq\": %.2f, \"r25_over_r16b\": %.3f}\n",
           pass, (int)chain, ms25 * 1e6 / chain, ms16 * 1e6 / chain, ms16b * 1e6 / chain, ms25 / ms16b);
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
  fclose(f);
  return 0;
}
