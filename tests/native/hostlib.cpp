// Host (CPU) build of the device library headers, for unit tests only.
//
// Compiles chaum-pedersen-zkp_amd/csrc/{fe25519,ristretto,scalar25519,transcript,
// scalarmul,verify}.h with g++ and -DCPZ_BOUNDS_CHECK (every fe_mul / fe_sq operand is
// checked against the limb bound), and exports thin C entry points so
// tests/test_device_arith.py can compare the exact arithmetic the kernels run against
// the Python oracle without a GPU.  Never linked into the product library.
#include <cstring>
#include <vector>

#include "verify.h"

using namespace cpz;

namespace {

void words_from(uint32_t w[8], const uint8_t* b) { std::memcpy(w, b, 32); }
void bytes_from(uint8_t* b, const uint32_t w[8]) { std::memcpy(b, w, 32); }

fe fe_from(const uint8_t* b) {
  uint32_t w[8];
  words_from(w, b);
  return fe_fromwords(w);
}

void fe_out(uint8_t* b, const fe& f) { fe_tobytes(b, f); }

// Fixed-base tables (k * base, k = 1..128) for one base encoding, times 2^shift.
bool build_table(std::vector<ge_niels>& tab, const uint8_t* enc, int shift = 0) {
  uint32_t w[8];
  words_from(w, enc);
  ge_p3 B;
  if (!ristretto_decode(B, w)) return false;
  for (int d = 0; d < shift; d++) B = p1p1_to_p3(p3_dbl(B));
  tab.resize(kTableB);
  for (int k = 1; k <= kTableB; k++) tab[k - 1] = p3_to_niels(small_mul(B, k));
  return true;
}

// Host stand-in for the device comb (CombTable): the same entries, j * 2^(16 k) * B in
// affine Niels form, computed on demand (the 64 MiB table is not worth building on the
// CPU for a handful of proofs).  Operation counting is suspended inside lookup, which
// stands for a memory read on the device.
struct HostComb {
  ge_p3 q[kCombWindows];
  bool build(const uint8_t* enc) {
    uint32_t w[8];
    words_from(w, enc);
    ge_p3 B;
    if (!ristretto_decode(B, w)) return false;
    for (int k = 0; k < kCombWindows; k++) {
      q[k] = B;
      for (int d = 0; d < 16; d++) B = p1p1_to_p3(p3_dbl(B));
    }
    return true;
  }
  ge_niels lookup(int k, int digit) const {
    const OpCounts saved = op_counts();
    const int mag = digit < 0 ? -digit : digit;
    ge_niels r = ge_niels_identity();
    if (mag != 0) {
      ge_p3 acc = q[k];
      for (int bit = 30 - __builtin_clz((unsigned)mag); bit >= 0; bit--) {
        acc = p1p1_to_p3(p3_dbl(acc));
        if ((mag >> bit) & 1) acc = ge_add(acc, q[k]);
      }
      r = p3_to_niels(acc);
    }
    op_counts() = saved;
    return ge_niels_cneg(r, digit < 0);
  }
};

struct GenTables {
  HostComb g, h;
  bool build(const uint8_t* genc, const uint8_t* henc) { return g.build(genc) && h.build(henc); }
};

}  // namespace

extern "C" {

// Field multiplications / squarings performed on this thread since the last call.
void cpzt_opcount(unsigned long long* mul, unsigned long long* sq) {
  *mul = op_counts().mul;
  *sq = op_counts().sq;
  op_counts().mul = 0;
  op_counts().sq = 0;
}

void cpzt_fe_mul(uint8_t* out, const uint8_t* a, const uint8_t* b) { fe_out(out, fe_mul(fe_from(a), fe_from(b))); }
void cpzt_fe_sq(uint8_t* out, const uint8_t* a) { fe_out(out, fe_sq(fe_from(a))); }
void cpzt_fe_sq2(uint8_t* out, const uint8_t* a) { fe_out(out, fe_sq2(fe_from(a))); }
void cpzt_fe_add(uint8_t* out, const uint8_t* a, const uint8_t* b) { fe_out(out, fe_add(fe_from(a), fe_from(b))); }
void cpzt_fe_sub(uint8_t* out, const uint8_t* a, const uint8_t* b) { fe_out(out, fe_sub(fe_from(a), fe_from(b))); }
void cpzt_fe_invert(uint8_t* out, const uint8_t* a) { fe_out(out, fe_invert(fe_from(a))); }
void cpzt_fe_pow22523(uint8_t* out, const uint8_t* a) { fe_out(out, fe_pow22523(fe_from(a))); }
int cpzt_fe_sqrt_ratio(uint8_t* out, const uint8_t* u, const uint8_t* v) {
  fe r;
  const bool sq = fe_sqrt_ratio_m1(r, fe_from(u), fe_from(v));
  fe_out(out, r);
  return sq ? 1 : 0;
}
int cpzt_fe_invsqrt_m1(uint8_t* out, const uint8_t* v) {
  fe r;
  const bool sq = fe_invsqrt_m1(r, fe_from(v));
  fe_out(out, r);
  return sq ? 1 : 0;
}

// Decode then re-encode: returns 1 and writes the re-encoding when `in` decodes.
int cpzt_decode_encode(uint8_t* out, const uint8_t* in) {
  uint32_t w[8], o[8];
  words_from(w, in);
  ge_p3 P;
  if (!ristretto_decode(P, w)) return 0;
  ristretto_encode(o, P);
  bytes_from(out, o);
  return 1;
}

// out = enc(a + b), enc(2a), enc(-a) for decodable a, b.
int cpzt_point_ops(uint8_t* sum, uint8_t* dbl, uint8_t* neg, const uint8_t* a, const uint8_t* b) {
  uint32_t w[8], o[8];
  ge_p3 A, B;
  words_from(w, a);
  if (!ristretto_decode(A, w)) return 0;
  words_from(w, b);
  if (!ristretto_decode(B, w)) return 0;
  ristretto_encode(o, ge_add(A, B));
  bytes_from(sum, o);
  ristretto_encode(o, p1p1_to_p3(p3_dbl(A)));
  bytes_from(dbl, o);
  ristretto_encode(o, ge_neg(A));
  bytes_from(neg, o);
  return 1;
}

int cpzt_points_equal(const uint8_t* a, const uint8_t* b) {
  uint32_t w[8];
  ge_p3 A, B;
  words_from(w, a);
  if (!ristretto_decode(A, w)) return -1;
  words_from(w, b);
  if (!ristretto_decode(B, w)) return -1;
  return ristretto_equal(A, B) ? 1 : 0;
}

// enc([s] B + [c] V) through the Straus loop, and enc([s] B) through fixed_base_mul.
int cpzt_straus(uint8_t* out, uint8_t* out_fixed, const uint8_t* base, const uint8_t* v, const uint8_t* s,
                const uint8_t* c) {
  std::vector<ge_niels> tab;
  if (!build_table(tab, base)) return 0;
  uint32_t w[8], sw[8], cw[8], sdig[8], cdig[8], o[8];
  words_from(w, v);
  ge_p3 V;
  if (!ristretto_decode(V, w)) return 0;
  ge_cached tv[kTableSlots];
  build_cached_table(host_table(tv), V);
  words_from(sw, s);
  words_from(cw, c);
  sc_recode_radix256(sdig, sw);
  sc_recode_radix16(cdig, cw);
  ristretto_encode(o, straus_vartime(host_table(tv), tab.data(), cdig, sdig));
  bytes_from(out, o);
  ristretto_encode(o, fixed_base_mul(tab.data(), sdig));
  bytes_from(out_fixed, o);
  return 1;
}

void cpzt_sc_reduce_wide(uint8_t* out, const uint8_t* in64) {
  uint32_t x[16];
  std::memcpy(x, in64, 64);
  const sc r = sc_reduce_wide(x);
  bytes_from(out, r.w);
}

void cpzt_sc_mul(uint8_t* out, const uint8_t* a, const uint8_t* b) {
  sc A, B;
  words_from(A.w, a);
  words_from(B.w, b);
  bytes_from(out, sc_mul(A, B).w);
}

void cpzt_sc_add(uint8_t* out, const uint8_t* a, const uint8_t* b) {
  sc A, B;
  words_from(A.w, a);
  words_from(B.w, b);
  bytes_from(out, sc_add(A, B).w);
}

int cpzt_sc_canonical(const uint8_t* s) {
  uint32_t w[8];
  words_from(w, s);
  return sc_is_canonical(w) ? 1 : 0;
}

void cpzt_chacha20_block(uint8_t* out64, const uint8_t* key, uint64_t counter, uint64_t stream) {
  uint32_t k[8], o[16];
  std::memcpy(k, key, 32);
  chacha20_block(o, k, counter, stream);
  std::memcpy(out64, o, 64);
}

void cpzt_keccak_f1600(uint8_t* state200) {
  ArrayState st;
  std::memcpy(st.b, state200, 200);
  st.permute();
  std::memcpy(state200, st.b, 200);
}

// Merlin KAT form: Transcript(label) ; append(l1, m1) ; challenge(l2, n).
void cpzt_merlin_kat(uint8_t* out, const char* proto, int plen, const char* label, int llen, const uint8_t* msg,
                     int mlen, const char* clabel, int cllen, int n) {
  ArrayState st;
  Strobe<ArrayState> s = strobe_init_merlin(st);
  s.merlin_header("dom-sep", 7, (uint32_t)plen);
  s.absorb((const uint8_t*)proto, plen);
  s.merlin_header(label, llen, (uint32_t)mlen);
  s.absorb(msg, mlen);
  s.merlin_challenge(clabel, cllen, out, n);
}

// Protocol challenge (batch.rs:188-206).  has_ctx selects Some(ctx) vs None.
void cpzt_challenge(uint8_t* out, const uint8_t* g, const uint8_t* h, const uint8_t* y1, const uint8_t* y2,
                    const uint8_t* r1, const uint8_t* r2, const uint8_t* ctx, uint32_t ctx_len, int has_ctx) {
  ArrayState st;
  Strobe<ArrayState> s = transcript_new(st);
  if (has_ctx) transcript_context(s, ctx, ctx_len);
  uint32_t gw[8], hw[8], a[8], b[8], c[8], d[8];
  words_from(gw, g);
  words_from(hw, h);
  transcript_parameters(s, gw, hw);
  words_from(a, y1);
  words_from(b, y2);
  words_from(c, r1);
  words_from(d, r2);
  bytes_from(out, transcript_challenge(s, a, b, c, d).w);
}

// Field-op count of verify_proof alone (the k_verify_each work for one proof), tables
// for g/h excluded (built once per context).
int cpzt_verify_opcount(unsigned long long* mul, unsigned long long* sq, const uint8_t* g, const uint8_t* h,
                        const uint8_t* y1, const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s,
                        const uint8_t* c) {
  GenTables gt;
  if (!gt.build(g, h)) return -1;
  uint32_t a[8], b[8], cc[8], d[8], sw[8], cw[8];
  words_from(a, y1);
  words_from(b, y2);
  words_from(cc, r1);
  words_from(d, r2);
  words_from(sw, s);
  words_from(cw, c);
  ge_cached tv[2 * kTableSlots];
  uint32_t dig[16];
  unsigned long long m0, s0;
  cpzt_opcount(&m0, &s0);
  const int st = verify_proof(host_digits(a), host_digits(b), host_digits(cc), host_digits(d), sw, cw,
                              response_status(sw), gt.g, gt.h, host_table(tv), dig, 1);
  cpzt_opcount(mul, sq);
  return st;
}

// Field-op counts of the RLC path's per-unit work (rlc.hip), for bench.py's roofline:
//   which = 0: k_rlc_prepare per proof -- 4 decodes + the Niels conversion of each (1 M);
//   which = 1: k_rlc_bucket per sorted entry -- one p1p1 -> p3 conversion + one mixed
//              (affine Niels) addition;
//   which = 2: k_verify_prepared per proof (the fallback's per-proof pass) -- the equations
//              with the points rebuilt from the prepared Niels forms instead of decoded;
//   which = 3: one k_part_acc walk step as the kernel executes it (part.hip): run + the
//              cached operand (the staged Niels point with Z = 1, or acc), p1p1 -> p3, and
//              acc's cached form (2 d T) -- the same products for an entry and a boundary;
//   which = 4: the algorithmic entry step of that walk: run + an affine Niels point (a mixed
//              addition) and p1p1 -> p3 (a boundary step, acc += run, is which = 3's work).
int cpzt_rlc_opcount(int which, unsigned long long* mul, unsigned long long* sq, const uint8_t* g, const uint8_t* h,
                     const uint8_t* y1, const uint8_t* y2, const uint8_t* r1, const uint8_t* r2, const uint8_t* s,
                     const uint8_t* c) {
  uint32_t w[4][8];
  words_from(w[0], r1);
  words_from(w[1], y1);
  words_from(w[2], r2);
  words_from(w[3], y2);
  ge_niels pre[4];
  for (int q = 0; q < 4; q++) {
    ge_p3 P;
    if (!ristretto_decode(P, w[q])) return -1;
    ge_niels n;
    n.ypx = fe_add(P.Y, P.X);
    n.ymx = fe_sub(P.Y, P.X);
    n.xy2d = fe_mul(P.T, FE_D2());
    pre[q] = ge_niels_cneg(n, true);
  }
  unsigned long long m0, s0;
  cpzt_opcount(&m0, &s0);
  if (which == 0) {
    for (int q = 0; q < 4; q++) {
      ge_p3 P;
      (void)ristretto_decode(P, w[q]);
      (void)fe_mul(P.T, FE_D2());
    }
  } else if (which == 1) {
    ge_p1p1 r = p1p1_identity();
    r = ge_add_niels(p1p1_to_p3(r), pre[0]);
    cpzt_opcount(&m0, &s0);  // one steady-state step: conversion + addition
    r = ge_add_niels(p1p1_to_p3(r), pre[1]);
  } else if (which == 3) {
    ge_p3 run = p1p1_to_p3(ge_add_niels(ge_identity(), pre[0]));
    cpzt_opcount(&m0, &s0);
    ge_cached oc;  // the staged point as k_part_acc forms its cached operand (Z = 1 selected)
    oc.YpX = pre[1].ypx;
    oc.YmX = pre[1].ymx;
    oc.T2d = pre[1].xy2d;
    oc.Z = fe_one();
    const ge_p3 r = p1p1_to_p3(ge_add_cached(run, oc));
    (void)p3_to_cached(r);  // acc's cached form (written under the boundary lanes' mask)
  } else if (which == 4) {
    ge_p3 run = p1p1_to_p3(ge_add_niels(ge_identity(), pre[0]));
    cpzt_opcount(&m0, &s0);
    (void)p1p1_to_p3(ge_add_niels(run, pre[1]));
  } else {
    GenTables gt;
    if (!gt.build(g, h)) return -1;
    cpzt_opcount(&m0, &s0);
    uint32_t sw[8], cw[8], dig[16];
    words_from(sw, s);
    words_from(cw, c);
    ge_cached tv[2 * kTableSlots];
    const DigitRef none{nullptr, 0};
    const int st = verify_proof<true>(none, none, none, none, sw, cw, 0, gt.g, gt.h, host_table(tv), dig, 1, pre);
    cpzt_opcount(mul, sq);
    return st;
  }
  cpzt_opcount(mul, sq);
  return 0;
}

// Full per-proof verification exactly as k_challenge + k_verify_each compute it.
int cpzt_verify(const uint8_t* g, const uint8_t* h, const uint8_t* y1, const uint8_t* y2, const uint8_t* r1,
                const uint8_t* r2, const uint8_t* s, const uint8_t* ctx, uint32_t ctx_len, int has_ctx) {
  GenTables gt;
  if (!gt.build(g, h)) return -1;
  uint8_t cb[32];
  cpzt_challenge(cb, g, h, y1, y2, r1, r2, ctx, ctx_len, has_ctx);
  uint32_t a[8], b[8], c[8], d[8], sw[8], cw[8];
  words_from(a, y1);
  words_from(b, y2);
  words_from(c, r1);
  words_from(d, r2);
  words_from(sw, s);
  words_from(cw, cb);
  ge_cached tv[2 * kTableSlots];
  uint32_t dig[16];
  return verify_proof(host_digits(a), host_digits(b), host_digits(c), host_digits(d), sw, cw, response_status(sw),
                      gt.g, gt.h, host_table(tv), dig, 1);
}

// The fixed-schedule no-context challenge (k_challenge_noctx's arithmetic) from the prefix
// state of (g, h); returns -1 if the prefix is not at the fixed position or the masks fail.
int cpzt_challenge_fixed(uint8_t* out, const uint8_t* g, const uint8_t* h, const uint8_t* y1, const uint8_t* y2,
                         const uint8_t* r1, const uint8_t* r2) {
  ArrayState st;
  Strobe<ArrayState> s = transcript_new(st);
  uint32_t gw[8], hw[8];
  words_from(gw, g);
  words_from(hw, h);
  transcript_parameters(s, gw, hw);
  if (s.pos != kTailPrefixPos || s.pos_begin != kTailPrefixBegin || s.cur_flags != kTailPrefixFlags) return -1;
  uint32_t k1[50], k2[50], pre[50];
  if (!challenge_masks(k1, k2)) return -1;
  std::memcpy(pre, st.b, 200);
  uint32_t a[8], b[8], c[8], d[8];
  words_from(a, y1);
  words_from(b, y2);
  words_from(c, r1);
  words_from(d, r2);
  bytes_from(out, challenge_fixed(pre, k1, k2, a, b, c, d).w);
  return 0;
}

// 32-byte-context fast path (challenge_fixed_ctx32) over the host build.
int cpzt_challenge_ctx32(uint8_t* out, const uint8_t* g, const uint8_t* h, const uint8_t* ctx, const uint8_t* y1,
                         const uint8_t* y2, const uint8_t* r1, const uint8_t* r2) {
  ArrayState st;
  Strobe<ArrayState> s = transcript_new(st);
  if (s.pos != kC32PrefixPos || s.pos_begin != kC32PrefixBegin || s.cur_flags != kC32PrefixFlags) return -1;
  uint32_t gw[8], hw[8], m[3][50], pre[50];
  words_from(gw, g);
  words_from(hw, h);
  if (!challenge_masks_ctx32(m, gw, hw)) return -1;
  std::memcpy(pre, st.b, 200);
  uint32_t cw[8], a[8], b[8], c[8], d[8];
  words_from(cw, ctx);
  words_from(a, y1);
  words_from(b, y2);
  words_from(c, r1);
  words_from(d, r2);
  bytes_from(out, challenge_fixed_ctx32(pre, m, cw, a, b, c, d).w);
  return 0;
}

// Half-size challenge split: u, |v| (16 bytes each, little-endian), sign of v.
void cpzt_half_split(uint8_t* u_out, uint8_t* v_out, int* vneg, const uint8_t* c) {
  uint32_t cw[8], u[4], v[4];
  words_from(cw, c);
  bool neg;
  sc_half_split(cw, u, v, neg);
  std::memcpy(u_out, u, 16);
  std::memcpy(v_out, v, 16);
  *vneg = neg ? 1 : 0;
}

// The 31-bit-window split (k_verify_wide's wave 4).
void cpzt_half_split32(uint8_t* u_out, uint8_t* v_out, int* vneg, const uint8_t* c) {
  uint32_t cw[8], u[4], v[4];
  words_from(cw, c);
  bool neg;
  sc_half_split32(cw, u, v, neg);
  std::memcpy(u_out, u, 16);
  std::memcpy(v_out, v, 16);
  *vneg = neg ? 1 : 0;
}

}  // extern "C"
