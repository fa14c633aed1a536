// Microbenchmark: GF(2^255 - 19) products and squarings in 5 x 51-bit f64
// limbs, priced against the product code's radix 2^25.5 (csrc/fe25519.h: ten signed 32-bit
// limbs, 100 / 55 v_mad_i64_i32 per product / squaring plus one carry chain).
//
// The f64 form (the most favourable exact one found; tight inputs only):
//   * limbs are signed and centred, |f_i| <= 2^50 + 2^47, value = sum f_i 2^(51 i);
//   * column k of the 9-column product collects f_i g_j (i + j = k); each 51 x 51 product is
//     split exactly by two v_fma_f64: H = fma(a, b, H) accumulates the product rounded to the
//     2^52 grid (H lives in [2^104, 2^105), started at C = 1.5 * 2^104, so its ulp stays 2^52
//     for the whole column), d = H_new - H_old is this product's rounded part (exact), and
//     lo = fma(a, b, -d) is the exact remainder, |lo| <= 2^51, summed in f64 (at most four
//     per accumulator: |sum| <= 2^53, exact; column 4 of a product has five, so two);
//   * per column, L is folded into H (H' = H + L rounds L to the grid, rem = L - (H' - H) is
//     exact, |rem| <= 2^51) and both leave f64 by their bit patterns: h = bits(H') - bits(C)
//     = (H' - C) / 2^52, r = bits(rem + 1.5 * 2^52) - bits(1.5 * 2^52) -- column sums carried
//     in int64 from there: limb k = r_k + 2 h_(k-1), the upper five limbs folded in x 19
//     (2^255 = 19 mod p), one centred carry pass, and back to f64 through the same magic.
// That is 4 f64 ops per 51 x 51 product (3 for a column's first) against 4 v_mad_i64_i32 for
// the same 102-bit product in 25.5-bit limbs (which also accumulate): the products alone cost
// the same instruction count, and the f64 form adds per column 4 f64 ops + 2 int64 subtracts
// before its carry.  Squarings: 15 products (cross terms as (2 f_i) f_j, exact) against 55 MADs.
//
// Checked bit-exactly: every thread's single product and square of 2^20 random inputs
// (including p - 1, p, 2^255 - 1, 0, 1, 2^254 and all-ones words) against a host
// __int128 reference, and the two forms' canonical outputs after chains of 250 operations
// against each other.  Timed as chains of 250 dependent operations per thread at 1, 2 and 4
// waves per SIMD; the in-kernel shader clock (s_memtime) of each block's wave 0 gives the
// cycles per operation per wave, and the launch's throughput the chip rate.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
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

constexpr int kChain = 250;

// ---- 5 x 51-bit f64 limbs --------------------------------------------------------------------
struct fd {
  double v[5];
};

constexpr double kC = 0x1.8p104;    // column accumulator origin: ulp 2^52 over [2^104, 2^105)
constexpr double kM = 0x1.8p52;     // int64 <-> f64 magic: ulp 1 over [2^52, 2^53]
constexpr int64_t kMask51 = (1LL << 51) - 1;

__host__ __device__ inline int64_t dbits(double x) {
  int64_t r;
  memcpy(&r, &x, 8);
  return r;
}
__host__ __device__ inline double bitsd(int64_t x) {
  double r;
  memcpy(&r, &x, 8);
  return r;
}

struct Col {
  double H, L;
};

// first product of a column / every further product (see the header)
__device__ __forceinline__ void col_first(Col& c, double a, double b) {
  c.H = __builtin_fma(a, b, kC);
  const double d = c.H - kC;
  c.L = __builtin_fma(a, b, -d);
}
__device__ __forceinline__ void col_add(Col& c, double a, double b) {
  const double Hn = __builtin_fma(a, b, c.H);
  const double d = Hn - c.H;
  c.L += __builtin_fma(a, b, -d);
  c.H = Hn;
}
// (h, r): column value = h 2^52 + r, |r| <= 2^51 (extra: a second lo accumulator, or 0)
__device__ __forceinline__ void col_out(int64_t& h, int64_t& r, const Col& c, bool has_extra, double extra) {
  double H = c.H + c.L;
  double rem = c.L - (H - c.H);  // |rem| <= 2^51
  if (has_extra) {               // column 4's fifth lo (only a product has one): |rem + extra|
    const double s = rem + extra;  // <= 2^52 is exact, and folding it leaves |rem| <= 2^51
    const double H2 = H + s;
    rem = s - (H2 - H);
    H = H2;
  }
  h = dbits(H) - dbits(kC);
  r = dbits(rem + kM) - dbits(kM);
}

// int64 limbs (|x| < 2^57) -> tight centred f64 limbs
__device__ __forceinline__ fd fd_from_wide(int64_t o[5]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int64_t c = (o[k] + (1LL << 50)) >> 51;
    o[k] -= c << 51;
    o[k + 1] += c;
  }
  const int64_t c4 = (o[4] + (1LL << 50)) >> 51;
  o[4] -= c4 << 51;
  o[0] += 19 * c4;
  const int64_t c0 = (o[0] + (1LL << 50)) >> 51;
  o[0] -= c0 << 51;
  o[1] += c0;
  fd r;
#pragma unroll
  for (int k = 0; k < 5; k++) r.v[k] = bitsd(dbits(kM) + o[k]) - kM;
  return r;
}

// limbs from the nine columns' (h, r): lambda_k = r_k + 2 h_(k-1), upper five x 19
__device__ __forceinline__ fd fd_finish(const int64_t h[9], const int64_t r[9]) {
  int64_t lam[10];
  lam[0] = r[0];
#pragma unroll
  for (int k = 1; k < 9; k++) lam[k] = r[k] + 2 * h[k - 1];
  lam[9] = 2 * h[8];
  int64_t o[5];
#pragma unroll
  for (int k = 0; k < 5; k++) o[k] = lam[k] + 19 * lam[k + 5];
  return fd_from_wide(o);
}

__device__ __forceinline__ fd fd_mul(const fd& f, const fd& g) {
  Col c[9];
  double extra = 0.0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int i0 = k < 5 ? 0 : k - 4;
    const int i1 = k < 5 ? k : 4;
    col_first(c[k], f.v[i0], g.v[k - i0]);
#pragma unroll
    for (int i = i0 + 1; i <= i1; i++) {
      if (k == 4 && i == 4) {  // fifth product of column 4: its own lo (four per accumulator)
        const double Hn = __builtin_fma(f.v[4], g.v[0], c[4].H);
        const double d = Hn - c[4].H;
        extra = __builtin_fma(f.v[4], g.v[0], -d);
        c[4].H = Hn;
      } else {
        col_add(c[k], f.v[i], g.v[k - i]);
      }
    }
  }
  int64_t h[9], r[9];
#pragma unroll
  for (int k = 0; k < 9; k++) col_out(h[k], r[k], c[k], k == 4, extra);
  return fd_finish(h, r);
}

__device__ __forceinline__ fd fd_sq(const fd& f) {
  double f2[5];
#pragma unroll
  for (int i = 0; i < 5; i++) f2[i] = f.v[i] + f.v[i];  // exact
  Col c[9];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int j = k - i;
      if (j < i || j > 4) continue;
      const double a = (i == j) ? f.v[i] : f2[i];
      if (first) col_first(c[k], a, f.v[j]);
      else col_add(c[k], a, f.v[j]);
      first = false;
    }
  }
  int64_t h[9], r[9];
#pragma unroll
  for (int k = 0; k < 9; k++) col_out(h[k], r[k], c[k], false, 0.0);
  return fd_finish(h, r);
}

// 8 little-endian words -> tight f64 limbs; bit 255 ignored, as the product code's fe_fromwords
__device__ inline fd fd_fromwords(const uint32_t w[8]) {
  uint64_t q[4];
  for (int i = 0; i < 4; i++) q[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  int64_t o[5];
  o[0] = (int64_t)(q[0] & kMask51);
  o[1] = (int64_t)(((q[0] >> 51) | (q[1] << 13)) & kMask51);
  o[2] = (int64_t)(((q[1] >> 38) | (q[2] << 26)) & kMask51);
  o[3] = (int64_t)(((q[2] >> 25) | (q[3] << 39)) & kMask51);
  o[4] = (int64_t)((q[3] >> 12) & kMask51);
  return fd_from_wide(o);
}

// canonical words
__device__ inline void fd_towords(uint32_t w[8], const fd& f) {
  int64_t o[5];
  for (int k = 0; k < 5; k++) o[k] = dbits(f.v[k] + kM) - dbits(kM);
  // floor carries to [0, 2^51), twice around
  for (int rep = 0; rep < 2; rep++) {
    for (int k = 0; k < 4; k++) {
      const int64_t c = o[k] >> 51;
      o[k] &= kMask51;
      o[k + 1] += c;
    }
    const int64_t c = o[4] >> 51;
    o[4] &= kMask51;
    o[0] += 19 * c;
  }
  // value in [0, 2^255 + small): subtract p if >= p
  int64_t t[5];
  int64_t c = 19;
  for (int k = 0; k < 5; k++) {
    t[k] = o[k] + c;
    c = t[k] >> 51;
    t[k] &= kMask51;
  }
  if (c) for (int k = 0; k < 5; k++) o[k] = t[k];
  uint64_t q[4];
  q[0] = (uint64_t)o[0] | ((uint64_t)o[1] << 51);
  q[1] = ((uint64_t)o[1] >> 13) | ((uint64_t)o[2] << 38);
  q[2] = ((uint64_t)o[2] >> 26) | ((uint64_t)o[3] << 25);
  q[3] = ((uint64_t)o[3] >> 39) | ((uint64_t)o[4] << 12);
  for (int i = 0; i < 4; i++) {
    w[2 * i] = (uint32_t)q[i];
    w[2 * i + 1] = (uint32_t)(q[i] >> 32);
  }
}

// ---- kernels -----------------------------------------------------------------------------
// mode 0: chains of kChain products a <- a * b; mode 1: chains of squarings (fe_sq / fd_sq);
// mode 2: fe_sqn's floor-carry squarings (r25 only: the decode chains' form).  stamps: block b's
// wave 0 writes s_memtime at start and end.
__global__ void __launch_bounds__(256) k_r25(const uint32_t* in, uint32_t* out, int reps, int mode,
                                             uint64_t* stamps) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = in[16 * t + i];
  cpz::fe a = cpz::fe_fromwords(w);
  for (int i = 0; i < 8; i++) w[i] = in[16 * t + 8 + i];
  const cpz::fe b = cpz::fe_fromwords(w);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    if (mode == 0) {
#pragma unroll 1
      for (int s = 0; s < kChain; s++) a = cpz::fe_mul(a, b);
    } else if (mode == 1) {
#pragma unroll 1
      for (int s = 0; s < kChain; s++) a = cpz::fe_sq(a);
    } else {
      a = cpz::fe_sqn(a, kChain);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t1;
  }
  cpz::fe_towords(w, a);
  for (int i = 0; i < 8; i++) out[8 * t + i] = w[i];
}

__global__ void __launch_bounds__(256) k_f64(const uint32_t* in, uint32_t* out, int reps, int mode,
                                             uint64_t* stamps) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = in[16 * t + i];
  fd a = fd_fromwords(w);
  for (int i = 0; i < 8; i++) w[i] = in[16 * t + 8 + i];
  const fd b = fd_fromwords(w);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    if (mode == 0) {
#pragma unroll 1
      for (int s = 0; s < kChain; s++) a = fd_mul(a, b);
    } else {
#pragma unroll 1
      for (int s = 0; s < kChain; s++) a = fd_sq(a);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t1;
  }
  fd_towords(w, a);
  for (int i = 0; i < 8; i++) out[8 * t + i] = w[i];
}

// one product and one square per thread (exactness check against the host reference)
__global__ void __launch_bounds__(256) k_f64_once(const uint32_t* in, uint32_t* out, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = in[16 * t + i];
  const fd a = fd_fromwords(w);
  for (int i = 0; i < 8; i++) w[i] = in[16 * t + 8 + i];
  const fd b = fd_fromwords(w);
  fd_towords(w, fd_mul(a, b));
  for (int i = 0; i < 8; i++) out[16 * t + i] = w[i];
  fd_towords(w, fd_sq(a));
  for (int i = 0; i < 8; i++) out[16 * t + 8 + i] = w[i];
}

// ---- host reference: 2^255 - 19 with unsigned __int128 ---------------------------------------
typedef unsigned __int128 u128;
static void h_from(uint64_t l[5], const uint32_t* w) {
  uint64_t q[4];
  for (int i = 0; i < 4; i++) q[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  const uint64_t m = (1ULL << 51) - 1;
  l[0] = q[0] & m;
  l[1] = ((q[0] >> 51) | (q[1] << 13)) & m;
  l[2] = ((q[1] >> 38) | (q[2] << 26)) & m;
  l[3] = ((q[2] >> 25) | (q[3] << 39)) & m;
  l[4] = (q[3] >> 12) & m;
}
static void h_mul(uint64_t r[5], const uint64_t a[5], const uint64_t b[5]) {
  u128 t[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 5; j++) {
      const u128 p = (u128)a[i] * b[j];
      if (i + j < 5) t[i + j] += p;
      else t[i + j - 5] += p * 19;
    }
  const uint64_t m = (1ULL << 51) - 1;
  uint64_t c = 0;
  for (int k = 0; k < 5; k++) {
    t[k] += c;
    r[k] = (uint64_t)t[k] & m;
    c = (uint64_t)(t[k] >> 51);
  }
  r[0] += 19 * c;
  c = r[0] >> 51;
  r[0] &= m;
  r[1] += c;
}
static void h_words(uint32_t w[8], const uint64_t l0[5]) {
  uint64_t o[5];
  const uint64_t m = (1ULL << 51) - 1;
  for (int k = 0; k < 5; k++) o[k] = l0[k];
  for (int rep = 0; rep < 2; rep++) {
    for (int k = 0; k < 4; k++) {
      o[k + 1] += o[k] >> 51;
      o[k] &= m;
    }
    const uint64_t c = o[4] >> 51;
    o[4] &= m;
    o[0] += 19 * c;
  }
  uint64_t t[5], c = 19;
  for (int k = 0; k < 5; k++) {
    t[k] = o[k] + c;
    c = t[k] >> 51;
    t[k] &= m;
  }
  if (c) for (int k = 0; k < 5; k++) o[k] = t[k];
  uint64_t q[4];
  q[0] = o[0] | (o[1] << 51);
  q[1] = (o[1] >> 13) | (o[2] << 38);
  q[2] = (o[2] >> 26) | (o[3] << 25);
  q[3] = (o[3] >> 39) | (o[4] << 12);
  for (int i = 0; i < 4; i++) {
    w[2 * i] = (uint32_t)q[i];
    w[2 * i + 1] = (uint32_t)(q[i] >> 32);
  }
}

template <class K>
static int timed(K kern, const char* name, const char* op, int mode, int cus, int wps, int reps, const uint32_t* din,
                 uint32_t* dout, uint64_t* dst, hipEvent_t e0, hipEvent_t e1, std::vector<uint32_t>& host_out,
                 int ops_per_call, int products_per_call) {
  const int grid = cus * wps;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, dout, 1, mode, dst);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, dout, reps, mode, dst);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> st((size_t)2 * grid);
  CHECK(hipMemcpy(st.data(), dst, st.size() * 8, hipMemcpyDeviceToHost));
  double cyc = 0;
  for (int b = 0; b < grid; b++) cyc += (double)(st[2 * b + 1] - st[2 * b]);
  cyc /= grid;
  const double per_wave_ops = (double)reps * kChain;
  const double total = (double)grid * 256 * reps * kChain;
  host_out.resize((size_t)grid * 256 * 8);
  CHECK(hipMemcpy(host_out.data(), dout, host_out.size() * 4, hipMemcpyDeviceToHost));
  // wave cycles per operation / waves sharing the SIMD = SIMD cycles per operation (issue cost)
  printf("{\"form\": \"%s\", \"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"ops_per_s\": %.4e, "
         "\"wave_cycles_per_op\": %.1f, \"simd_cycles_per_op\": %.1f, \"simd_cycles_per_51x51_product\": %.2f, "
         "\"valu_ops_per_call_isa\": %d}\n",
         name, op, wps, ms, total / (ms * 1e-3), cyc / per_wave_ops, cyc / per_wave_ops / wps,
         cyc / per_wave_ops / wps / products_per_call, ops_per_call);
  return 0;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  // exactness: 2^20 single products and squares against the host reference
  const int n1 = 1 << 20;
  std::vector<uint32_t> in((size_t)n1 * 16);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (auto& v : in) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    v = (uint32_t)x;
  }
  // edge inputs (bit 255 is ignored by both forms, as by the product's fe_fromwords): p - 1,
  // 2^255 - 1, 0, 1, all-ones words, p, ragged limbs, 2^254
  const uint32_t P1[8] = {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
  for (int e = 0; e < 64; e++) {
    uint32_t* row = &in[(size_t)16 * e];
    for (int h = 0; h < 2; h++) {
      const int kind = (e >> (3 * h)) & 7;
      for (int i = 0; i < 8; i++) {
        uint32_t v = 0;
        switch (kind) {
          case 0: v = P1[i]; break;                                  // p - 1
          case 1: v = i == 7 ? 0x7fffffffu : 0xffffffffu; break;     // 2^255 - 1
          case 2: v = 0; break;
          case 3: v = i == 0 ? 1 : 0; break;
          case 4: v = 0xffffffffu; break;                            // 2^256 - 1
          case 5: v = i == 0 ? 0xffffffedu : P1[i]; break;           // p
          case 6: v = (i & 1) ? 0x0007ffffu : 0xffffffffu; break;    // ragged high bits
          default: v = i == 7 ? 0x40000000u : 0; break;              // 2^254
        }
        row[8 * h + i] = v;
      }
    }
  }
  uint32_t *din, *dout;
  uint64_t* dst;
  CHECK(hipMalloc(&din, in.size() * 4));
  CHECK(hipMalloc(&dout, in.size() * 4));
  CHECK(hipMalloc(&dst, (size_t)2 * cus * 4 * 8));
  CHECK(hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_f64_once, dim3(n1 / 256), dim3(256), 0, 0, din, dout, n1);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> got((size_t)n1 * 16);
  CHECK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
  size_t bad_mul = 0, bad_sq = 0;
  for (int t = 0; t < n1; t++) {
    uint64_t a[5], b[5], r[5];
    uint32_t w[8];
    h_from(a, &in[(size_t)16 * t]);
    h_from(b, &in[(size_t)16 * t + 8]);
    h_mul(r, a, b);
    h_words(w, r);
    bad_mul += memcmp(w, &got[(size_t)16 * t], 32) != 0;
    h_mul(r, a, a);
    h_words(w, r);
    bad_sq += memcmp(w, &got[(size_t)16 * t + 8], 32) != 0;
  }
  printf("{\"check\": \"f64 single product / square vs host __int128 reference\", \"inputs\": %d, "
         "\"edge_inputs\": 64, \"mismatched_products\": %zu, \"mismatched_squares\": %zu}\n",
         n1, bad_mul, bad_sq);
  if (bad_mul || bad_sq) return 2;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  // ISA VALU instruction counts per call, from the disassembly (tools/ubench/fe_f64_isa.txt)
  const int ops_r25_mul = argc > 2 ? atoi(argv[2]) : 0, ops_f64_mul = argc > 3 ? atoi(argv[3]) : 0;
  const int ops_r25_sq = argc > 4 ? atoi(argv[4]) : 0, ops_f64_sq = argc > 5 ? atoi(argv[5]) : 0;
  for (int w : {1, 2, 4}) {
    for (int mode = 0; mode < 2; mode++) {
      std::vector<uint32_t> a, b;
      if (timed(k_r25, "r25", mode ? "sq" : "mul", mode, cus, w, reps, din, dout, dst, e0, e1, a,
                mode ? ops_r25_sq : ops_r25_mul, mode ? 15 : 25)) return 1;
      if (timed(k_f64, "f64", mode ? "sq" : "mul", mode, cus, w, reps, din, dout, dst, e0, e1, b,
                mode ? ops_f64_sq : ops_f64_mul, mode ? 15 : 25)) return 1;
      size_t bad = 0;
      for (size_t i = 0; i < a.size(); i++) bad += a[i] != b[i];
      printf("{\"waves_per_simd\": %d, \"op\": \"%s\", \"chain\": %d, \"mismatched_words_r25_vs_f64\": %zu}\n", w,
             mode ? "sq" : "mul", kChain * reps, bad);
      if (bad) return 2;
    }
    std::vector<uint32_t> c;
    if (timed(k_r25, "r25_sqn_floor", "sq", 2, cus, w, reps, din, dout, dst, e0, e1, c, 0, 15)) return 1;
  }
  return 0;
}
