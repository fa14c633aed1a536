// Microbenchmark: does the per-proof Straus loop (4 doublings + 1 cached addition from a
// per-thread table in HBM, the inner step of straus_half_comb) run faster with more waves per
// SIMD?  The same loop body compiled for 160 VGPRs (fits 3 waves/SIMD, no spill) and for 128
// (4 waves, spilling) is launched with 1..4 blocks of 256 threads per CU (= waves per SIMD),
// timed with HIP events; the in-kernel shader clock (s_memtime / s_memrealtime) is reported too.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I chaum-pedersen-zkp_amd/csrc \
//     tools/ubench/occupancy_loop.hip -o tools/ubench/occupancy_loop
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "verify.h"
using namespace cpz;

#define CHECK(x)                                                                               \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

template <int W>
__global__ void __launch_bounds__(256, W) k_loop(char* slab, uint32_t* out, uint64_t* stamps, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const SlabTable tab{slab, (uint32_t)i * 9u * 160u};
  ge_p1p1 c = p1p1_identity();
  c.X.v[0] = i;
  uint32_t dg = 0x9e3779b9u * (i + 1);
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    dg = dg * 1664525u + 1013904223u;
    const int d = (int)(dg >> 28) - 8;
    const ge_cached e = cached_lookup(tab, d);
    c = dbl4(c);
    c = ge_add_cached(p1p1_to_p3(c), e);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
  out[i] = c.X.v[0] ^ c.Y.v[1] ^ c.Z.v[2] ^ c.T.v[3];
  if ((threadIdx.x & 63) == 0) {
    stamps[2 * (i >> 6)] = t1 - t0;
    stamps[2 * (i >> 6) + 1] = q1 - q0;
  }
}

template <int W>
static int run(int cus, int blocks_per_cu, int n, char* slab, uint32_t* out, uint64_t* stamps) {
  const int grid = cus * blocks_per_cu;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_loop<W>, dim3(grid), dim3(256), 0, 0, slab, out, stamps, n / 8);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_loop<W>, dim3(grid), dim3(256), 0, 0, slab, out, stamps, n);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = grid * 4;
  std::vector<uint64_t> h(2 * (size_t)nw);
  CHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  std::vector<double> f(nw);
  for (int w = 0; w < nw; w++) f[w] = h[2 * w + 1] ? (double)h[2 * w] / (double)h[2 * w + 1] * 0.1 : 0.0;
  std::nth_element(f.begin(), f.begin() + nw / 2, f.end());
  const double steps = (double)grid * 256 * n;
  printf("%s{\"regs_budget_waves\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"G_steps_per_s\": %.4f, \"clock_ghz\": %.3f}\n",
         (W == 3 && blocks_per_cu == 1) ? " " : ",", W, blocks_per_cu, ms, steps / (ms * 1e-3) / 1e9, f[nw / 2]);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, n = 2000;
  char* slab;
  uint32_t* out;
  uint64_t* stamps;
  const size_t threads = (size_t)cus * 4 * 256;
  CHECK(hipMalloc(&slab, threads * 9 * 160));
  {  // random limbs in (-2^24, 2^24): valid operands, and realistic switching activity
    std::vector<int32_t> h(threads * 9 * 40);
    uint32_t x = 12345;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = (int32_t)(x >> 7) - (1 << 24);
    }
    CHECK(hipMemcpy(slab, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  CHECK(hipMalloc(&out, threads * sizeof(uint32_t)));
  CHECK(hipMalloc(&stamps, threads / 64 * 2 * sizeof(uint64_t)));
  printf("{\"device\": \"%s\", \"cus\": %d, \"step\": \"4 doublings + 1 cached addition (table entry from HBM)\", \"rows\": [\n",
         p.gcnArchName, cus);
  for (int b = 1; b <= 3; b++)
    if (run<3>(cus, b, n, slab, out, stamps)) return 1;
  for (int b = 1; b <= 4; b++)
    if (run<4>(cus, b, n, slab, out, stamps)) return 1;
  printf("]}\n");
  return 0;
}
