// Microbenchmark: the serial work of k_verify_wide's wave 4 (the challenge and the split that
// gate the Straus loops) timed piece by piece on a lone wave with the shader clock
// (s_memtime), to see where its ~65 us go:
//   challenge   challenge_fixed (two Keccak-f permutations + the wide reduction mod l) on the
//               register sponge, and with the permutations spread over the wave (keccak_wave.h),
//               which must give the same challenge
//   split       sc_half_split (63-bit Lehmer windows, f64 quotients) / sc_half_split32 (31-bit
//               windows, f32 reciprocal) / the latter with each batch's four rows on four lanes
//   digits      sc_mul (v s mod l) + the three recodings
// One workgroup of one wave; every lane computes the same values (as in wave 4).  Prints one
// JSON line of cycles per piece (median of the lanes' agreeing results over `reps` launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../chaum-pedersen-zkp_amd/csrc/cpz_kernels.h"
#include "../../chaum-pedersen-zkp_amd/csrc/scalar25519.h"
#include "../../chaum-pedersen-zkp_amd/csrc/transcript.h"
#include "../../chaum-pedersen-zkp_amd/csrc/verify.h"
#include "../../chaum-pedersen-zkp_amd/csrc/keccak_wave.h"

using namespace cpz;

__global__ void __launch_bounds__(64) k_parts(const uint32_t* in, uint32_t* out, uint64_t* cyc) {
  const int l = threadIdx.x;
  uint32_t y1[8], y2[8], r1[8], r2[8], sw[8];
  for (int k = 0; k < 8; k++) {
    y1[k] = in[k];
    y2[k] = in[8 + k];
    r1[k] = in[16 + k];
    r2[k] = in[24 + k];
    sw[k] = in[32 + k] & (k == 7 ? 0x0fffffffu : 0xffffffffu);
  }
  const uint32_t* prefix = in + 64;
  const uint32_t* k1 = in + 128;
  const uint32_t* k2 = in + 192;
  __shared__ uint32_t lds[50];
  uint64_t t[8];
  t[0] = __builtin_amdgcn_s_memtime();
  const sc c0 = challenge_fixed(prefix, k1, k2, y1, y2, r1, r2);
  t[1] = __builtin_amdgcn_s_memtime();
  const sc c = challenge_fixed(prefix, k1, k2, y1, y2, r1, r2, PermRows{lds, l});
  t[2] = __builtin_amdgcn_s_memtime();
  bool same_c = true;
  for (int k = 0; k < 8; k++) same_c = same_c && c.w[k] == c0.w[k];
  uint32_t u[4], va[4], u2[4], va2[4], u3[4], va3[4];
  bool vneg, vneg2, vneg3;
  sc_half_split(c.w, u, va, vneg);
  t[3] = __builtin_amdgcn_s_memtime();
  sc_half_split32(c.w, u2, va2, vneg2);
  t[4] = __builtin_amdgcn_s_memtime();
  uint32_t cs[8];
  for (int k = 0; k < 8; k++) cs[k] = __builtin_amdgcn_readfirstlane(c.w[k]);
  sc_half_split32<true>(cs, u3, va3, vneg3);
  t[5] = __builtin_amdgcn_s_memtime();
  uint32_t dig[16];
  sc_recode_radix16_half(dig, u3);
  sc_recode_radix16_half(dig + 4, va3);
  sc vs, ss;
  for (int k = 0; k < 8; k++) {
    vs.w[k] = k < 4 ? va3[k] : 0u;
    ss.w[k] = sw[k];
  }
  sc sp = sc_mul(vs, ss);
  if (vneg3) sp = sc_neg(sp);
  sc_recode_radix65536(dig + 8, sp.w);
  t[6] = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int k = 0; k < 4; k++) x ^= u[k] ^ va[k] ^ u2[k] ^ va2[k] ^ u3[k] ^ va3[k];
  for (int k = 0; k < 16; k++) x ^= dig[k];
  x ^= (vneg ? 1u : 0u) ^ (vneg2 ? 2u : 0u) ^ (vneg3 ? 4u : 0u);
  out[l] = x;
  // the three splits must agree
  bool same = vneg == vneg2 && vneg2 == vneg3;
  for (int k = 0; k < 4; k++) same = same && u[k] == u2[k] && u2[k] == u3[k] && va[k] == va2[k] && va2[k] == va3[k];
  out[64 + l] = (same ? 1u : 0u) | (same_c ? 0u : 2u);
  if (l == 0)
    for (int k = 0; k < 7; k++) cyc[k] = t[k];
}

int main() {
  std::vector<uint32_t> in(256);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (auto& v : in) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    v = (uint32_t)s;
  }
  uint32_t *din, *dout;
  uint64_t* dcyc;
  hipMalloc(&din, in.size() * 4);
  hipMalloc(&dout, 128 * 4);
  hipMalloc(&dcyc, 8 * 8);
  hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice);
  const char* names[6] = {"challenge_registers", "challenge_wave_lanes", "split63", "split31", "split31_lanes",
                          "digits_scmul"};
  std::vector<std::vector<double>> per(6);
  for (int rep = 0; rep < 21; rep++) {
    hipLaunchKernelGGL(k_parts, dim3(1), dim3(64), 0, 0, din, dout, dcyc);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    uint64_t t[7];
    uint32_t o[128];
    hipMemcpy(t, dcyc, sizeof(t), hipMemcpyDeviceToHost);
    hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l++)
      if (o[64 + l] != 1) {
        fprintf(stderr, "lane %d: %s\n", l, (o[64 + l] & 2) ? "wave Keccak != register Keccak" : "split variants disagree");
        return 2;
      }
    if (rep == 0) continue;  // cold instruction cache
    for (int k = 0; k < 6; k++) per[k].push_back((double)(t[k + 1] - t[k]));
    in[0] ^= (uint32_t)rep;  // another challenge each launch
    hipMemcpy(din, in.data(), 4, hipMemcpyHostToDevice);
  }
  printf("{\"unit\": \"shader cycles (s_memtime), median of 20 launches\"");
  for (int k = 0; k < 6; k++) {
    std::vector<double> v = per[k];
    std::sort(v.begin(), v.end());
    printf(", \"%s\": %.0f", names[k], v[v.size() / 2]);
  }
  printf("}\n");
  return 0;
}
