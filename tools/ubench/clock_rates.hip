// Microbenchmark: issue cost (SIMD cycles per wave64 instruction) of the integer VALU
// instructions the GF(2^255-19) arithmetic is made of, measured with the in-kernel shader
// clock (s_memtime) and the constant 100 MHz clock (s_memrealtime), so the MAD peak that
// bench.py's roofline divides by is stated at the clock the chip actually holds under a
// VALU-dense load (MI355X_MICROARCH.md, DVFS give-back item 6) instead of at 2.4 GHz.
//
// Each wave runs 16 independent accumulation chains of one instruction; lane 0 stamps
// s_memtime / s_memrealtime around the loop and writes them to a buffer of its own (never
// an output).  W blocks of 256 threads per CU = W waves per SIMD.
//   clock (GHz)             = median over waves of dt / dreal * 0.1
//   cycles/instr (per SIMD) = SIMD cycles of the launch / wave instructions per SIMD
//                           = (event ms * clock) / (W * iters * 16)
// The launch's SIMD cycles come from the event time and the measured clock, so the figure
// holds whether or not all W waves of a SIMD were resident at once.  (Round 2 divided each
// wave's own stamp span by W, which assumes they were: at 4 and 8 waves/SIMD it reported
// 3.96 and 2.90 cycles while the launch's throughput implied ~4.5.)  The per-wave form is
// kept as wave_stamp_cycles for comparison.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
      return 1;                                                                                   \
    }                                                                                             \
  } while (0)

enum Op { MAD_I64_I32 = 0, ADD_U32, AND_B32, MUL_LO_U32, LSHL_ADD_U64, ASHR_I64, NOPS };
static const char* kNames[NOPS] = {"v_mad_i64_i32", "v_add_u32", "v_and_b32", "v_mul_lo_u32", "v_lshl_add_u64",
                                    "v_ashrrev_i64"};
constexpr int kChains = 16;

template <int OP>
__global__ void __launch_bounds__(256) kclock(int iters, uint64_t* sink, uint64_t* stamps, uint32_t seed) {
  const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  const uint32_t a = seed ^ (t * 2654435761u), b = a * 747796405u + 1;
  uint64_t acc[kChains];
#pragma unroll
  for (int j = 0; j < kChains; j++) acc[j] = ((uint64_t)(a + j) << 7) | (uint64_t)j;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < kChains; j++) {
      if constexpr (OP == MAD_I64_I32) {
        asm volatile("v_mad_i64_i32 %0, s[40:41], %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b) : "s40", "s41");
      } else if constexpr (OP == ADD_U32) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == AND_B32) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == MUL_LO_U32) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == LSHL_ADD_U64) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[j]) : "v"(acc[(j + 1) % kChains]));
      } else if constexpr (OP == ASHR_I64) {
        asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(acc[j]));
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < kChains; j++) r ^= acc[j];
  sink[t] = r;
  if ((threadIdx.x & 63) == 0) {
    const uint32_t w = t >> 6;
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
}

template <int OP>
static int run(int cus, int waves_per_simd, int iters, uint64_t* sink, uint64_t* stamps, hipEvent_t e0, hipEvent_t e1,
               double* cyc, double* wave_cyc, double* ghz, double* gops) {
  const int grid = cus * waves_per_simd;
  hipLaunchKernelGGL(kclock<OP>, dim3(grid), dim3(256), 0, 0, iters / 4, sink, stamps, 1u);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kclock<OP>, dim3(grid), dim3(256), 0, 0, iters, sink, stamps, 1u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = grid * 4;
  std::vector<uint64_t> h(2 * (size_t)nw);
  CHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  std::vector<double> c(nw), f(nw);
  for (int w = 0; w < nw; w++) {
    c[w] = (double)h[2 * w] / ((double)iters * kChains) / waves_per_simd;
    f[w] = h[2 * w + 1] ? (double)h[2 * w] / (double)h[2 * w + 1] * 0.1 : 0.0;
  }
  std::nth_element(c.begin(), c.begin() + nw / 2, c.end());
  std::nth_element(f.begin(), f.begin() + nw / 2, f.end());
  *wave_cyc = c[nw / 2];
  *ghz = f[nw / 2];
  *cyc = (double)ms * 1e-3 * (*ghz * 1e9) / ((double)waves_per_simd * iters * kChains);
  *gops = (double)grid * 256.0 * iters * kChains / (ms * 1e-3) / 1e9;
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint64_t *sink, *stamps;
  CHECK(hipMalloc(&sink, (size_t)cus * 8 * 256 * sizeof(uint64_t)));
  CHECK(hipMalloc(&stamps, (size_t)cus * 8 * 4 * 2 * sizeof(uint64_t)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 40000;
  printf("{\"device\": \"%s\", \"cus\": %d, \"unit\": \"SIMD cycles per wave64 instruction (in-kernel s_memtime)\", \"rows\": [\n",
         p.gcnArchName, cus);
  bool first = true;
  for (int op = 0; op < NOPS; op++) {
    for (int w : {1, 2, 4, 8}) {
      double cyc = 0, wcyc = 0, ghz = 0, gops = 0;
      int rc = 0;
      switch (op) {
        case MAD_I64_I32: rc = run<MAD_I64_I32>(cus, w, iters, sink, stamps, e0, e1, &cyc, &wcyc, &ghz, &gops); break;
        case ADD_U32: rc = run<ADD_U32>(cus, w, iters, sink, stamps, e0, e1, &cyc, &wcyc, &ghz, &gops); break;
        case AND_B32: rc = run<AND_B32>(cus, w, iters, sink, stamps, e0, e1, &cyc, &wcyc, &ghz, &gops); break;
        case MUL_LO_U32: rc = run<MUL_LO_U32>(cus, w, iters, sink, stamps, e0, e1, &cyc, &wcyc, &ghz, &gops); break;
        case LSHL_ADD_U64: rc = run<LSHL_ADD_U64>(cus, w, iters, sink, stamps, e0, e1, &cyc, &wcyc, &ghz, &gops); break;
        case ASHR_I64: rc = run<ASHR_I64>(cus, w, iters, sink, stamps, e0, e1, &cyc, &wcyc, &ghz, &gops); break;
      }
      if (rc) return rc;
      printf("%s {\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr\": %.3f, \"wave_stamp_cycles\": %.3f, "
             "\"clock_ghz\": %.3f, \"lanes_per_simd_cycle\": %.3f, \"gops\": %.1f, \"gops_at_2p4ghz\": %.1f}\n",
             first ? " " : ",", kNames[op], w, cyc, wcyc, ghz, 64.0 / cyc, gops, 4.0 * cus * 64.0 / cyc * 2.4);
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
