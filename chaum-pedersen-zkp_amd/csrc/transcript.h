// Keccak-f[1600], STROBE-128 v1.0.2 and Merlin v1.0 framing, plus the ChaCha20 block
// function, for gfx950.
//
// Replaces merlin 3.0.0 (Cargo.lock:1182-1191; keccak 0.1.5) as reached from the
// reference's src/primitives/transcript.rs:29-71, bit for bit:
//   Transcript::new        -> Merlin("Chaum-Pedersen ZKP v1.0.0") + append("protocol", ...)
//   append_context         -> append("context", ctx)
//   append_parameters      -> append("generator-g", g) ; append("generator-h", h)
//   append_statement       -> append("y1", y1) ; append("y2", y2)
//   append_commitment      -> append("r1", r1) ; append("r2", r2)
//   challenge_scalar       -> challenge_bytes("challenge", 64) -> wide reduction mod l
// and rand_chacha 0.3.1's ChaCha20 block (batch weights, synthetic witnesses).
//
// The sponge state is reached through an accessor so the same STROBE code drives a
// per-thread LDS image on the GPU (kernels.hip) and a plain array in host unit tests.
#pragma once
#include "fe25519.h"

namespace cpz {

constexpr int kStrobeR = 166;
constexpr uint8_t kFlagI = 1, kFlagA = 2, kFlagC = 4, kFlagM = 16;

// 64-bit rotation; n is a compile-time constant at every call site after unrolling.  On the
// device it is two v_alignbit_b32 (funnel shifts of the 32-bit halves) instead of two
// 64-bit shifts and an OR.
CPZ_HD uint64_t rol64(uint64_t v, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  if (n & 32) {
    const uint32_t t = lo;
    lo = hi;
    hi = t;
  }
  const int r = n & 31;
  if (r == 0) return ((uint64_t)hi << 32) | lo;
  const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
  const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
  return ((uint64_t)nhi << 32) | nlo;
#else
  return n ? ((v << n) | (v >> (64 - n))) : v;
#endif
}

CPZ_HD uint64_t KECCAK_RC(int i) {
  const uint64_t rc[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
      0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
      0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  return rc[i];
}

// Three-input bitwise function on 64-bit lanes: gfx950's v_bitop3_b32 on each half
// (truth table imm = f(S0 = 0xF0, S1 = 0xCC, S2 = 0xAA)), so theta's five-way XOR and chi
// are one instruction per 32 bits where plain code needs two.  LLVM does not form these
// from the 64-bit expressions below by itself.
template <int IMM>
CPZ_HD uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo, hi;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(lo) : "v"((uint32_t)a), "v"((uint32_t)b), "v"((uint32_t)c),
      "i"(IMM));
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(hi)
      : "v"((uint32_t)(a >> 32)), "v"((uint32_t)(b >> 32)), "v"((uint32_t)(c >> 32)), "i"(IMM));
  return ((uint64_t)hi << 32) | lo;
#else
  static_assert(IMM == 0x96 || IMM == 0xD2, "plain forms of the two truth tables Keccak uses");
  return IMM == 0x96 ? (a ^ b ^ c) : (a ^ (~b & c));
#endif
}
constexpr int kXor3 = 0x96;   // a ^ b ^ c
constexpr int kChi = 0xD2;    // a ^ (~b & c)

// One Keccak-f[1600] round on 25 lanes, lane index x + 5y.
CPZ_HD void keccak_round(uint64_t a[25], uint64_t rc) {
  // rho offsets and pi destinations in lane order.
  constexpr int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                           25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  uint64_t c[5], b[25];
#pragma unroll
  for (int x = 0; x < 5; x++)
    c[x] = bitop3_64<kXor3>(bitop3_64<kXor3>(a[x], a[x + 5], a[x + 10]), a[x + 15], a[x + 20]);
#pragma unroll
  for (int x = 0; x < 5; x++) {
    const uint64_t d = c[(x + 4) % 5] ^ rol64(c[(x + 1) % 5], 1);
#pragma unroll
    for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
  }
#pragma unroll
  for (int x = 0; x < 5; x++) {
#pragma unroll
    for (int y = 0; y < 5; y++) {
      // B[y, 2x + 3y] = rot(A[x, y], r[x, y])
      b[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(a[x + 5 * y], rho[x + 5 * y]);
    }
  }
#pragma unroll
  for (int y = 0; y < 5; y++) {
#pragma unroll
    for (int x = 0; x < 5; x++)
      a[x + 5 * y] = bitop3_64<kChi>(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
  }
  a[0] ^= rc;
}

// In-place Keccak-f[1600] (the compiler keeps the 24 rounds a loop: one round of code).
CPZ_HD void keccak_f1600(uint64_t a[25]) {
  for (int round = 0; round < 24; round++) keccak_round(a, KECCAK_RC(round));
}

// STROBE-128 restricted to the operations Merlin uses (meta-AD, AD, PRF).
// Acc provides: uint8_t get(int), void put(int, uint8_t), void xor_(int, uint8_t),
// void permute() (Keccak-f over its 200 bytes).
template <class Acc>
struct Strobe {
  Acc& st;
  int pos;
  int pos_begin;
  uint8_t cur_flags;

  CPZ_HDM explicit Strobe(Acc& s, int p = 0, int pb = 0, uint8_t f = 0) : st(s), pos(p), pos_begin(pb), cur_flags(f) {}

  CPZ_HDM void run_f() {
    st.xor_(pos, (uint8_t)pos_begin);
    st.xor_(pos + 1, 0x04);
    st.xor_(kStrobeR + 1, 0x80);
    st.permute();
    pos = 0;
    pos_begin = 0;
  }
  CPZ_HDM void absorb_byte(uint8_t b) {
    st.xor_(pos, b);
    pos++;
    if (pos == kStrobeR) run_f();
  }
  CPZ_HDM void absorb(const uint8_t* data, int n) {
#pragma unroll
    for (int i = 0; i < n; i++) absorb_byte(data[i]);
  }
  CPZ_HDM void absorb_u32le(uint32_t v) {
    absorb_byte((uint8_t)v);
    absorb_byte((uint8_t)(v >> 8));
    absorb_byte((uint8_t)(v >> 16));
    absorb_byte((uint8_t)(v >> 24));
  }
  CPZ_HDM void absorb_words(const uint32_t* w, int nwords) {
#pragma unroll
    for (int i = 0; i < nwords; i++) absorb_u32le(w[i]);
  }
  CPZ_HDM uint8_t squeeze_byte() {
    const uint8_t b = st.get(pos);
    st.put(pos, 0);
    pos++;
    if (pos == kStrobeR) run_f();
    return b;
  }
  CPZ_HDM void begin_op(uint8_t flags) {  // more == false
    const int old_begin = pos_begin;
    pos_begin = pos + 1;
    cur_flags = flags;
    absorb_byte((uint8_t)old_begin);
    absorb_byte(flags);
    if ((flags & kFlagC) && pos != 0) run_f();
  }
  // Merlin append_message framing: meta-AD(label) ; meta-AD(u32le len, more) ; AD(msg).
  CPZ_HDM void merlin_header(const char* label, int label_len, uint32_t msg_len) {
    begin_op(kFlagM | kFlagA);
    absorb((const uint8_t*)label, label_len);
    absorb_u32le(msg_len);  // "more" continuation of the meta-AD op
    begin_op(kFlagA);
  }
  CPZ_HDM void merlin_append_words(const char* label, int label_len, const uint32_t w[8]) {
    merlin_header(label, label_len, 32);
    absorb_words(w, 8);
  }
  // challenge_bytes(label, n): meta-AD(label) ; meta-AD(u32le n, more) ; PRF(n).
  CPZ_HDM void merlin_challenge(const char* label, int label_len, uint8_t* out, int n) {
    begin_op(kFlagM | kFlagA);
    absorb((const uint8_t*)label, label_len);
    absorb_u32le((uint32_t)n);
    begin_op(kFlagI | kFlagA | kFlagC);
#pragma unroll
    for (int i = 0; i < n; i++) out[i] = squeeze_byte();
  }
};

// Byte-array accessor (host tests, the prefix kernel).
struct ArrayState {
  uint8_t b[200];
  CPZ_HDM uint8_t get(int i) const { return b[i]; }
  CPZ_HDM void put(int i, uint8_t v) { b[i] = v; }
  CPZ_HDM void xor_(int i, uint8_t v) { b[i] ^= v; }
  CPZ_HDM void permute() {
    uint64_t a[25];
    for (int i = 0; i < 25; i++) {
      uint64_t v = 0;
      for (int k = 7; k >= 0; k--) v = (v << 8) | b[8 * i + k];
      a[i] = v;
    }
    keccak_f1600(a);
    for (int i = 0; i < 25; i++)
      for (int k = 0; k < 8; k++) b[8 * i + k] = (uint8_t)(a[i] >> (8 * k));
  }
};

// Records, per sponge segment (between permutations), the bytes XORed into the state:
// run over the transcript tail with all-zero messages it yields the constant framing masks
// of the fixed-schedule challenge (verify.h, challenge_fixed).
struct MaskState {
  uint8_t m[3][200];
  int seg = 0;
  CPZ_HDM uint8_t get(int) const { return 0; }
  CPZ_HDM void put(int, uint8_t) {}
  CPZ_HDM void xor_(int i, uint8_t v) {
    if (seg < 3) m[seg][i] ^= v;
  }
  CPZ_HDM void permute() { seg++; }
};

// Fresh STROBE-128 state for protocol label "Merlin v1.0" (state, pos, pos_begin, flags).
template <class Acc>
CPZ_HD Strobe<Acc> strobe_init_merlin(Acc& st) {
  for (int i = 0; i < 200; i++) st.put(i, 0);
  const uint8_t hdr[6] = {1, kStrobeR + 2, 1, 0, 1, 96};
  const char* ver = "STROBEv1.0.2";
  for (int i = 0; i < 6; i++) st.put(i, hdr[i]);
  for (int i = 0; i < 12; i++) st.put(6 + i, (uint8_t)ver[i]);
  st.permute();
  Strobe<Acc> s(st);
  // meta_ad(protocol_label = "Merlin v1.0", more = false)
  s.begin_op(kFlagM | kFlagA);
  s.absorb((const uint8_t*)"Merlin v1.0", 11);
  return s;
}

// ChaCha20 block (djb layout: words 12-13 = 64-bit block counter, 14-15 = stream id).
CPZ_HD uint32_t rotl32(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

#define CPZ_CHACHA_QR(a, b, c, d)          \
  a += b; d ^= a; d = rotl32(d, 16);       \
  c += d; b ^= c; b = rotl32(b, 12);       \
  a += b; d ^= a; d = rotl32(d, 8);        \
  c += d; b ^= c; b = rotl32(b, 7);

CPZ_HD void chacha20_block(uint32_t out[16], const uint32_t key[8], uint64_t counter, uint64_t stream) {
  uint32_t init[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                       key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                       (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = init[i];
  for (int r = 0; r < 10; r++) {
    CPZ_CHACHA_QR(x[0], x[4], x[8], x[12]);
    CPZ_CHACHA_QR(x[1], x[5], x[9], x[13]);
    CPZ_CHACHA_QR(x[2], x[6], x[10], x[14]);
    CPZ_CHACHA_QR(x[3], x[7], x[11], x[15]);
    CPZ_CHACHA_QR(x[0], x[5], x[10], x[15]);
    CPZ_CHACHA_QR(x[1], x[6], x[11], x[12]);
    CPZ_CHACHA_QR(x[2], x[7], x[8], x[13]);
    CPZ_CHACHA_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + init[i];
}

}  // namespace cpz
