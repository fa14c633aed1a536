// Microbenchmark: cost model of the VALU instruction mix of the GF(2^255-19) kernels on
// gfx950.  Each variant runs NM independent v_mad_i64_i32 chains and NA independent
// chains of a cheap op per iteration (16 chains each at most, so latency is hidden),
// at 2 waves/SIMD (the verify kernel's occupancy) and 4 waves/SIMD.  Reported:
// ns per wave-iteration and the implied cycles per instruction, to tell whether MADs and
// simple ops share issue slots additively.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

enum Cheap { ADD32 = 0, LSHLADD64, ASHR64, BFE32, AND32, MUL_LO, ADD32_E64, ADD3, ANDLIT, ALIGNBIT, SUBCO, FMA64, MAD24, MULHI24, PKFMA32, MADU64, NCHEAP };
static const char* kCheap[NCHEAP] = {"v_add_u32", "v_lshl_add_u64", "v_ashrrev_i64", "v_bfe_i32", "v_and_b32",
                                     "v_mul_lo_u32", "v_add_u32_e64", "v_add3_u32", "v_and_b32(literal)", "v_alignbit_b32", "v_sub_co+v_subb_co", "v_fma_f64", "v_mad_u32_u24", "v_mul_hi_u32_u24", "v_pk_fma_f32", "v_mad_u64_u32"};

template <int NM, int NA, int OP>
__global__ void __launch_bounds__(256) kmix(int iters, uint64_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  uint32_t a = seed ^ (t * 2654435761u), b = a * 747796405u + 1;
  int64_t m[NM > 0 ? NM : 1];
  uint64_t x[NA > 0 ? NA : 1];
#pragma unroll
  for (int j = 0; j < (NM > 0 ? NM : 1); j++) m[j] = (int64_t)(a + j);
#pragma unroll
  for (int j = 0; j < (NA > 0 ? NA : 1); j++) x[j] = (uint64_t)(b + 3 * j) << 3 | j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (j < NM) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(m[j < NM ? j : 0]) : "v"(a), "v"(b) : "vcc");
      if (j < NA) {
        uint64_t& y = x[j < NA ? j : 0];
        if constexpr (OP == ADD32) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == LSHLADD64) {
          asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(y));
        } else if constexpr (OP == ASHR64) {
          asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(y));
        } else if constexpr (OP == BFE32) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_bfe_i32 %0, %0, 0, 26" : "+v"(lo));
          y = lo;
        } else if constexpr (OP == AND32) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_and_b32 %0, %0, %1" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == ADD32_E64) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == ADD3) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == ANDLIT) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_and_b32 %0, 0xfc000000, %0" : "+v"(lo));
          y = lo;
        } else if constexpr (OP == ALIGNBIT) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_alignbit_b32 %0, %1, %0, 26" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == SUBCO) {
          uint32_t lo = (uint32_t)y, hi = (uint32_t)(y >> 32);
          asm volatile("v_sub_co_u32 %0, vcc, %0, %2\n\tv_subb_co_u32 %1, vcc, %1, %2, vcc" : "+v"(lo), "+v"(hi) : "v"(b) : "vcc");
          y = ((uint64_t)hi << 32) | lo;
        } else if constexpr (OP == FMA64) {
          asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(y));
        } else if constexpr (OP == MADU64) {
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y) : "v"(a), "v"(b) : "vcc");
        } else if constexpr (OP == PKFMA32) {
          asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(y));
        } else if constexpr (OP == MAD24) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == MULHI24) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(lo) : "v"(b));
          y = lo;
        } else if constexpr (OP == MUL_LO) {
          uint32_t lo = (uint32_t)y;
          asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
          y = lo;
        }
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < (NM > 0 ? NM : 1); j++) r ^= (uint64_t)m[j];
#pragma unroll
  for (int j = 0; j < (NA > 0 ? NA : 1); j++) r ^= x[j];
  out[t] = r;
}

template <int NM, int NA, int OP>
static int run(int wps, int cus, int iters, uint64_t* d_out, hipEvent_t e0, hipEvent_t e1, int clock_khz) {
  const int grid = cus * wps;  // 256 threads = 4 waves = one per SIMD
  hipLaunchKernelGGL((kmix<NM, NA, OP>), dim3(grid), dim3(256), 0, 0, 4, d_out, 1u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((kmix<NM, NA, OP>), dim3(grid), dim3(256), 0, 0, iters, d_out, 1u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  // cycles per SIMD per wave-iteration at the nominal clock
  const double cyc = (double)ms * 1e-3 * clock_khz * 1e3 / ((double)iters * wps);
  printf("{\"mads\": %d, \"cheap\": %d, \"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_iter\": %.2f, "
         "\"cycles_per_instr\": %.3f}\n",
         NM, NA, kCheap[OP], wps, cyc, cyc / (NM + NA));
  return 0;
}

#define RUN(NM, NA, OP) if (run<NM, NA, OP>(w, cus, iters, d_out, e0, e1, clk)) return 1;

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, clk = p.clockRate;
  printf("# device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, clk);
  uint64_t* d_out;
  CHECK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(uint64_t)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 4000;
  for (int w : {2, 4}) {
    RUN(0, 16, FMA64)
    RUN(0, 16, MADU64)
    RUN(0, 16, PKFMA32)
    RUN(0, 16, MAD24)
    RUN(0, 16, MULHI24)
    RUN(8, 8, FMA64)
    RUN(0, 16, ADD32_E64)
    RUN(0, 16, ADD3)
    RUN(0, 16, ANDLIT)
    RUN(0, 16, ALIGNBIT)
    RUN(0, 8, SUBCO)
    RUN(16, 0, ADD32)
    RUN(0, 16, ADD32)
    RUN(0, 16, LSHLADD64)
    RUN(0, 16, ASHR64)
    RUN(0, 16, BFE32)
    RUN(0, 16, AND32)
    RUN(0, 16, MUL_LO)
    RUN(8, 8, ADD32)
    RUN(8, 8, LSHLADD64)
    RUN(8, 8, ASHR64)
    RUN(8, 8, BFE32)
    RUN(12, 4, ADD32)
    RUN(4, 12, ADD32)
  }
  return 0;
}
