// Microbenchmark: integer / f64 VALU instruction throughput on gfx950.
// Measures lane-ops per second for the instructions a GF(2^255-19) limb
// multiply can be built from, at several waves-per-SIMD occupancies, so the
// limb choice and the roofline peak in DESIGN.md rest on measured numbers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

enum Op { MAD_U64_U32 = 0, MUL_LO_U32, MUL_HI_U32, ADD_U32, MUL_U32_U24, FMA_F64, ADD_CO_CI, LSHL_B64, MAD_U32_U24, NOPS };
static const char* kNames[NOPS] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_add_u32",
                                    "v_mul_u32_u24", "v_fma_f64", "v_add_co+v_addc_co(64b add)",
                                    "v_lshlrev_b64", "v_mad_u32_u24"};

template <int OP>
__global__ void __launch_bounds__(256) kbench(int iters, uint64_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  uint32_t a = seed ^ (t * 2654435761u), b = a * 747796405u + 1;
  uint64_t acc[8];
  double facc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = (uint64_t)(a + j) << 7 | j; facc[j] = (double)(a + j); }
  double fb = 1.0000001 + (double)(b & 7) * 1e-9;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if constexpr (OP == MAD_U64_U32) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %3" : "=v"(c) : "v"(a), "v"(b), "v"(acc[j]) : "s40", "s41");
        acc[j] = c;
      } else if constexpr (OP == MUL_LO_U32) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == MUL_HI_U32) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == ADD_U32) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == MUL_U32_U24) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      } else if constexpr (OP == FMA_F64) {
        asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(facc[j]) : "v"(fb));
      } else if constexpr (OP == ADD_CO_CI) {
        uint64_t x = acc[j];
        uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc"
                     : "+v"(lo), "+v"(hi) : "v"(b) : "vcc");
        acc[j] = ((uint64_t)hi << 32) | lo;
      } else if constexpr (OP == LSHL_B64) {
        asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(acc[j]));
      } else if constexpr (OP == MAD_U32_U24) {
        uint32_t x = (uint32_t)acc[j];
        asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(b));
        acc[j] = x;
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= acc[j] ^ (uint64_t)facc[j];
  out[t] = r;
}

template <int OP>
static int run(int blocks_per_cu, int cus, int iters, uint64_t* d_out, hipEvent_t e0, hipEvent_t e1,
               double* gops) {
  int grid = cus * blocks_per_cu;
  hipLaunchKernelGGL(kbench<OP>, dim3(grid), dim3(256), 0, 0, 4, d_out, 1u);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kbench<OP>, dim3(grid), dim3(256), 0, 0, iters, d_out, 1u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  double ops = (double)grid * 256.0 * iters * 8.0;
  *gops = ops / (ms * 1e-3) / 1e9;
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  uint64_t* d_out;
  CHECK(hipMalloc(&d_out, (size_t)cus * 32 * 256 * sizeof(uint64_t)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 20000;
  int bpcs[] = {1, 2, 4, 8};
  printf("{\"unit\": \"G lane-ops/s\", \"rows\": [\n");
  bool first = true;
  for (int op = 0; op < NOPS; op++) {
    for (int bpc : bpcs) {
      double g = 0;
      int rc = 0;
      switch (op) {
        case MAD_U64_U32: rc = run<MAD_U64_U32>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case MUL_LO_U32: rc = run<MUL_LO_U32>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case MUL_HI_U32: rc = run<MUL_HI_U32>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case ADD_U32: rc = run<ADD_U32>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case MUL_U32_U24: rc = run<MUL_U32_U24>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case FMA_F64: rc = run<FMA_F64>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case ADD_CO_CI: rc = run<ADD_CO_CI>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case LSHL_B64: rc = run<LSHL_B64>(bpc, cus, iters, d_out, e0, e1, &g); break;
        case MAD_U32_U24: rc = run<MAD_U32_U24>(bpc, cus, iters, d_out, e0, e1, &g); break;
      }
      if (rc) return rc;
      printf("%s {\"op\": \"%s\", \"waves_per_simd\": %d, \"gops\": %.1f}\n", first ? " " : ",", kNames[op], bpc, g);
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
