// Microbenchmark: the inverse-square-root exponent chain of a ristretto
// decode is ~250 field squarings (fe_sqn in csrc/fe25519.h).  This times a chain of 250
// squarings per thread two ways, on the same inputs, and checks that both give the same
// canonical value:
//   r25  the product code: radix 2^25.5, ten signed limbs, 55 v_mad_i64_i32 + floor carries
//   r32  radix 2^32, eight unsigned limbs: 36 products (28 cross products doubled + 8
//        squares) accumulated per column in 64 bits plus an overflow word, then the upper
//        half folded in with 2^256 = 38 (mod p)
// Occupancy is swept (1, 2, 4 waves per SIMD); the JSON line per variant gives ns per
// squaring per lane and the shader-clock cycles per squaring per wave.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../chaum-pedersen-zkp_amd/csrc/fe25519.h"

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
      return 1;                                                                                   \
    }                                                                                             \
  } while (0)

constexpr int kSquarings = 250;

// ---- radix 2^32 ---------------------------------------------------------------------------
struct fe32 {
  uint32_t w[8];
};

__device__ __forceinline__ void mac(uint64_t& acc, uint32_t& ov, uint32_t a, uint32_t b) {
  const uint64_t p = (uint64_t)a * b;
  acc += p;
  ov += acc < p ? 1u : 0u;
}

// a^2 mod p, result < 2^256 (not canonical); input any value < 2^256.
__device__ __forceinline__ fe32 sq32(const fe32& a) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t ov = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t c = 0;
    uint32_t co = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j > i && j < 8) mac(c, co, a.w[i], a.w[j]);
    }
    // double the cross sum (co:c) and add the square and the carried-in (ov:acc)
    co = (co << 1) | (uint32_t)(c >> 63);
    c <<= 1;
    if ((k & 1) == 0) mac(c, co, a.w[k / 2], a.w[k / 2]);
    c += acc;
    co += (c < acc ? 1u : 0u) + ov;
    t[k] = (uint32_t)c;
    acc = (c >> 32) | ((uint64_t)co << 32);
    ov = 0;
  }
  t[15] = (uint32_t)acc;
  // fold: r = t_lo + 38 t_hi (2^256 = 38 mod p)
  fe32 r;
  uint64_t cr = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    cr += (uint64_t)t[i] + (uint64_t)t[8 + i] * 38u;
    r.w[i] = (uint32_t)cr;
    cr >>= 32;
  }
  // carry < 39: fold once more (the second carry out is 0 or 1 and folds trivially)
  uint64_t c2 = (uint64_t)r.w[0] + cr * 38u;
  r.w[0] = (uint32_t)c2;
  c2 >>= 32;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    c2 += r.w[i];
    r.w[i] = (uint32_t)c2;
    c2 >>= 32;
  }
  r.w[0] += (uint32_t)c2 * 38u;  // c2 set only if r was >= 2^256 - 38 * 39: then r.w[0] is small
  return r;
}

__device__ __forceinline__ void canon32(uint32_t out[8], const fe32& a) {
  // a < 2^256 -> a mod p, canonical (subtract p up to twice)
  uint32_t x[8];
  for (int i = 0; i < 8; i++) x[i] = a.w[i];
  for (int rep = 0; rep < 2; rep++) {
    // y = x + 19; if y >= 2^255 then x - p = y - 2^255
    uint64_t c = 19;
    uint32_t y[8];
    for (int i = 0; i < 8; i++) {
      c += x[i];
      y[i] = (uint32_t)c;
      c >>= 32;
    }
    const bool ge = (y[7] >> 31) != 0 || c != 0;
    y[7] &= 0x7fffffffu;
    for (int i = 0; i < 8; i++) x[i] = ge ? y[i] : x[i];
  }
  for (int i = 0; i < 8; i++) out[i] = x[i];
}

__global__ void __launch_bounds__(256) k_r32(const uint32_t* in, uint32_t* out, int reps) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  fe32 a;
  for (int i = 0; i < 8; i++) a.w[i] = in[8 * t + i];
  for (int r = 0; r < reps; r++) {
#pragma unroll 1
    for (int s = 0; s < kSquarings; s++) a = sq32(a);
  }
  uint32_t w[8];
  canon32(w, a);
  for (int i = 0; i < 8; i++) out[8 * t + i] = w[i];
}

__global__ void __launch_bounds__(256) k_r25(const uint32_t* in, uint32_t* out, int reps) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = in[8 * t + i];
  cpz::fe a = cpz::fe_fromwords(w);
  for (int r = 0; r < reps; r++) a = cpz::fe_sqn(a, kSquarings);
  cpz::fe_towords(w, a);
  for (int i = 0; i < 8; i++) out[8 * t + i] = w[i];
}

template <class K>
static int run(K kern, const char* name, int cus, int wps, int reps, uint32_t* din, uint32_t* dout, hipEvent_t e0,
               hipEvent_t e1, std::vector<uint32_t>& host_out) {
  const int grid = cus * wps;  // 4 waves per block: wps waves per SIMD
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, dout, 1);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, dout, reps);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double sq = (double)grid * 256 * reps * kSquarings;
  host_out.resize((size_t)grid * 256 * 8);
  CHECK(hipMemcpy(host_out.data(), dout, host_out.size() * 4, hipMemcpyDeviceToHost));
  printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"squarings_per_s\": %.4e, "
         "\"ps_per_squaring_chip\": %.3f}\n",
         name, wps, ms, sq / (ms * 1e-3), ms * 1e9 / sq);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int maxw = 4;
  const size_t nthr = (size_t)cus * maxw * 256;
  std::vector<uint32_t> in(nthr * 8);
  uint64_t x = 88172645463325252ull;
  for (auto& v : in) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    v = (uint32_t)x;
  }
  for (size_t t = 0; t < nthr; t++) in[8 * t + 7] &= 0x7fffffffu;  // < 2^255
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, in.size() * 4));
  CHECK(hipMalloc(&dout, in.size() * 4));
  CHECK(hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 40;
  for (int w : {1, 2, 4}) {
    std::vector<uint32_t> a, b;
    if (run(k_r25, "r25", cus, w, reps, din, dout, e0, e1, a)) return 1;
    if (run(k_r32, "r32", cus, w, reps, din, dout, e0, e1, b)) return 1;
    size_t bad = 0;
    for (size_t i = 0; i < a.size(); i++) bad += a[i] != b[i];
    printf("{\"waves_per_simd\": %d, \"mismatched_words\": %zu}\n", w, bad);
    if (bad) return 2;
  }
  return 0;
}
