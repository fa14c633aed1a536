// cpz_batch.hpp -- header-only C++ mirror of the reference's `verifier::batch::BatchVerifier`
// (kobby-pentangeli/chaum-pedersen-zkp, src/verifier/batch.rs:45-330) on top of the C ABI
// in cpz.h.  Same names, cap, error conditions and result order:
//
//   BatchVerifier()                      batch.rs:97       (new)
//   BatchVerifier::with_capacity(n)      batch.rs:113
//   len / is_empty / remaining_capacity  batch.rs:122-136
//   add / add_with_context               batch.rs:139-168  (cap MAX_BATCH_SIZE = 1000)
//   verify()                             batch.rs:171-183  -> one Result per entry
//   clear                                batch.rs:321-323
//   Proof::to_bytes / Proof::from_bytes  gadgets.rs:343-489 (from_bytes on the device parser)
//   Verifier: verify / verify_with_transcript / verify_response     verifier/mod.rs:42-172
//   Prover: prove_with_transcript (caller nonce) / statement        prover/mod.rs:86-131,
//                                                                    gadgets.rs:217-221
//
// Errors are returned, never thrown across the ABI; `Result` carries the reference's
// error kind (src/error.rs:5-17).  Points and scalars stay as their 32-byte encodings:
// decoding and all checks run on the GPU.  Verifier and BatchVerifier hold Proof values,
// which may have been built directly (Proof::new, gadgets.rs:317: no identity / zero-s
// checks), so their calls pass CPZ_CALL_EQUATIONS_ONLY -- the equations alone decide, as
// verify_one (batch.rs:185-231) and verify_with_transcript (verifier/mod.rs:120-171) do --
// for those calls only (the context's own mode, Device::set_commitment_checks, is untouched);
// proof_from_bytes still applies from_bytes' checks.
//
// BatchVerifier::verify issues exactly the call sequence of the Rust drop-in
// (rust/reference-patch/gpu.rs): entries grouped by Parameters in order of first appearance;
// a one-entry batch -> cpz_verify_each_ex (batch.rs:178-180, the rng untouched); otherwise
// 64 bytes per entry are drawn from the caller's rng, as the reference's random_scalar draws
// them (batch.rs:239-240), the first 32 keying every group's RLC check; groups take
// consecutive weight indices (first_index), and a group of at least rlc_min_group entries runs
// cpz_verify_batch_ex (RLC + exact fallback), a smaller one cpz_verify_each_ex.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <functional>
#include <optional>
#include <random>
#include <string>
#include <utility>
#include <vector>

#include "cpz.h"

namespace chaum_pedersen {

constexpr std::size_t MAX_BATCH_SIZE = 1000;  // batch.rs:48

// Smallest Parameters group that takes the RLC batch check rather than per-proof
// verification (both return verify_one's outcome per entry).  The same threshold as
// rust/reference-patch/gpu.rs (RLC_MIN_GROUP), from the per-call latency table
// bench.py's small_batch (profiles/r05_bench_i.json): one synchronous host-buffer call takes
// 0.112-0.118 ms per proof at n = 1 .. 100 (k_verify_wide) and 0.265 ms at 1000 (k_verify_small),
// against 0.54-0.59 ms through the RLC check at n <= 100 and 0.73 ms at 1000, so no group of at most MAX_BATCH_SIZE entries takes
// the RLC check (set_rlc_min_group lowers it; a one-entry batch is then keyed by the OS's
// randomness, not the caller's).
constexpr std::size_t RLC_MIN_GROUP = 1001;

using Bytes32 = std::array<uint8_t, 32>;

enum class ErrorKind { None, InvalidParams, InvalidScalar, InvalidGroupElement, Device };

struct Result {
  ErrorKind kind = ErrorKind::None;
  std::string message;
  bool is_ok() const { return kind == ErrorKind::None; }
  bool is_err() const { return !is_ok(); }
  static Result ok() { return Result{}; }
  static Result err(ErrorKind k, std::string m) { return Result{k, std::move(m)}; }
};

inline Result status_result(uint8_t st) {
  switch (st) {
    case CPZ_STATUS_OK: return Result::ok();
    case CPZ_STATUS_EQ_FAIL: return Result::err(ErrorKind::InvalidParams, "Proof verification failed");
    case CPZ_STATUS_BAD_POINT:
      return Result::err(ErrorKind::InvalidGroupElement, "Bytes do not represent a valid Ristretto point");
    case CPZ_STATUS_BAD_SCALAR: return Result::err(ErrorKind::InvalidScalar, "Bytes do not represent a valid scalar");
    case CPZ_STATUS_IDENTITY: return Result::err(ErrorKind::InvalidParams, "Commitment contains identity element");
    default: return Result::err(ErrorKind::InvalidParams, "Response scalar is zero");  // CPZ_STATUS_ZERO_S
  }
}

struct Parameters {  // gadgets.rs:25-118
  Bytes32 g, h;
  Parameters() { cpz_default_generators(g.data(), h.data()); }
  Parameters(const Bytes32& g_, const Bytes32& h_) : g(g_), h(h_) {}
};

struct Statement {  // gadgets.rs:177-239
  Bytes32 y1, y2;
};

struct Proof {  // gadgets.rs:245-311
  Bytes32 r1, r2, s;

  // gadgets.rs:343-361: [version 1][u32be 32][r1][u32be 32][r2][u32be 32][s] = 109 bytes.
  std::vector<uint8_t> to_bytes() const {
    std::vector<uint8_t> out{1};
    for (const Bytes32* f : {&r1, &r2, &s}) {
      const uint8_t len[4] = {0, 0, 0, 32};
      out.insert(out.end(), len, len + 4);
      out.insert(out.end(), f->begin(), f->end());
    }
    return out;
  }
};

// The reference's error for a CPZ_PARSE_* code (gadgets.rs:364-489).
inline Result parse_result(uint8_t code, uint32_t aux) {
  const std::string a = std::to_string(aux);
  switch (code) {
    case CPZ_PARSE_OK: return Result::ok();
    case CPZ_PARSE_TOO_SMALL: return Result::err(ErrorKind::InvalidParams, "Proof too small: " + a + " bytes");
    case CPZ_PARSE_BAD_VERSION: return Result::err(ErrorKind::InvalidParams, "Unsupported proof version: " + a);
    case CPZ_PARSE_R1_LEN_MISSING: return Result::err(ErrorKind::InvalidParams, "Truncated proof: missing r1 length");
    case CPZ_PARSE_R1_LEN_INVALID: return Result::err(ErrorKind::InvalidParams, "Invalid r1 length: " + a);
    case CPZ_PARSE_R1_TRUNCATED: return Result::err(ErrorKind::InvalidParams, "Truncated proof: incomplete r1 data");
    case CPZ_PARSE_R2_LEN_MISSING: return Result::err(ErrorKind::InvalidParams, "Truncated proof: missing r2 length");
    case CPZ_PARSE_R2_LEN_INVALID: return Result::err(ErrorKind::InvalidParams, "Invalid r2 length: " + a);
    case CPZ_PARSE_R2_TRUNCATED: return Result::err(ErrorKind::InvalidParams, "Truncated proof: incomplete r2 data");
    case CPZ_PARSE_R1_SIZE:
    case CPZ_PARSE_R2_SIZE: return Result::err(ErrorKind::InvalidGroupElement, "Expected 32 bytes, got " + a);
    case CPZ_PARSE_R1_POINT:
    case CPZ_PARSE_R2_POINT:
      return Result::err(ErrorKind::InvalidGroupElement, "Bytes do not represent a valid Ristretto point");
    case CPZ_PARSE_S_LEN_MISSING: return Result::err(ErrorKind::InvalidParams, "Truncated proof: missing s length");
    case CPZ_PARSE_S_LEN_INVALID: return Result::err(ErrorKind::InvalidParams, "Invalid s length: " + a);
    case CPZ_PARSE_S_TRUNCATED: return Result::err(ErrorKind::InvalidParams, "Truncated proof: incomplete s data");
    case CPZ_PARSE_S_SIZE: return Result::err(ErrorKind::InvalidScalar, "Expected 32 bytes, got " + a);
    case CPZ_PARSE_S_SCALAR: return Result::err(ErrorKind::InvalidScalar, "Bytes do not represent a valid scalar");
    case CPZ_PARSE_TRAILING: return Result::err(ErrorKind::InvalidParams, "Proof has " + a + " trailing bytes");
    case CPZ_PARSE_IDENTITY: return Result::err(ErrorKind::InvalidParams, "Commitment contains identity element");
    default: return Result::err(ErrorKind::InvalidParams, "Response scalar is zero");  // CPZ_PARSE_ZERO_S
  }
}

// One GPU context; shareable by many BatchVerifiers on one thread.
class Device {
 public:
  explicit Device(int ordinal = 0) { rc_ = cpz_ctx_create(ordinal, &ctx_); }
  ~Device() { cpz_ctx_destroy(ctx_); }
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;
  bool ok() const { return rc_ == CPZ_OK && ctx_ != nullptr; }
  cpz_ctx* get() const { return ctx_; }
  // cpz_ctx_set_commitment_checks: the context's mode for every later call on it (the mirrors
  // below do not use it: their calls pass CPZ_CALL_EQUATIONS_ONLY)
  int set_commitment_checks(bool on) { return cpz_ctx_set_commitment_checks(ctx_, on ? 1 : 0); }

 private:
  cpz_ctx* ctx_ = nullptr;
  int rc_ = CPZ_EINVAL;
};

// Statement::validate (gadgets.rs:234-238 -> ristretto.rs:173-185): y1 and y2 must be group
// elements, i.e. their encodings must decode (on the device).
inline Result validate_statement(Device& dev, const Statement& st) {
  uint8_t pts[64], ok[2] = {0, 0};
  std::memcpy(pts, st.y1.data(), 32);
  std::memcpy(pts + 32, st.y2.data(), 32);
  if (cpz_decode_points(dev.get(), 2, pts, ok, nullptr) != CPZ_OK) return Result::err(ErrorKind::Device, cpz_last_error());
  if (!ok[0] || !ok[1]) return Result::err(ErrorKind::InvalidGroupElement, "Element failed recompression validation");
  return Result::ok();
}

// Proof::from_bytes (gadgets.rs:364-489) through the device parser: the reference's checks
// in its order (point decodes and canonical-scalar checks included), first failure wins.
inline Result proof_from_bytes(Device& dev, const uint8_t* blob, std::size_t len, Proof* out) {
  const uint64_t off[2] = {0, len};
  Proof p;
  uint8_t code = 0;
  uint32_t aux = 0;
  const uint8_t pad = 0;
  const int rc = cpz_parse_proofs(dev.get(), 1, len ? blob : &pad, off, p.r1.data(), p.r2.data(), p.s.data(), &code,
                                  &aux);
  if (rc != CPZ_OK) return Result::err(ErrorKind::Device, cpz_last_error());
  Result r = parse_result(code, aux);
  if (r.is_ok() && out) *out = p;
  return r;
}

// Verifier (verifier/mod.rs:42-172) for one statement; each call is a 1-entry device call.
class Verifier {
 public:
  Verifier(Device& dev, Parameters params, Statement st) : dev_(&dev), params_(params), st_(st) {}
  // verifier/mod.rs:85-88 (fresh transcript) and :120-139 (transcript with an optional context)
  Result verify(const Proof& pr) const { return verify_with_transcript(pr, std::nullopt); }
  Result verify_with_transcript(const Proof& pr, const std::optional<std::vector<uint8_t>>& context) const {
    Result v = validate_statement(*dev_, st_);  // verifier/mod.rs:121
    if (v.is_err()) return v;
    uint8_t st = 0, present = context ? 1 : 0, pad = 0;
    const uint64_t off[2] = {0, context ? context->size() : 0};
    const uint8_t* cb = (context && !context->empty()) ? context->data() : &pad;
    const int rc = cpz_verify_each_ex(dev_->get(), CPZ_CALL_EQUATIONS_ONLY, params_.g.data(), params_.h.data(), 1,
                                      st_.y1.data(), st_.y2.data(), pr.r1.data(), pr.r2.data(), pr.s.data(),
                                      context ? cb : nullptr, context ? off : nullptr, context ? &present : nullptr,
                                      &st);
    if (rc != CPZ_OK) return Result::err(ErrorKind::Device, cpz_last_error());
    return status_result(st);
  }
  // verifier/mod.rs:144-171: the caller's challenge (32 canonical little-endian bytes)
  Result verify_response(const Bytes32& challenge, const Proof& pr) const {
    uint8_t st = 0;
    const int rc = cpz_verify_response_ex(dev_->get(), CPZ_CALL_EQUATIONS_ONLY, params_.g.data(), params_.h.data(), 1,
                                          st_.y1.data(), st_.y2.data(), pr.r1.data(), pr.r2.data(), pr.s.data(),
                                          challenge.data(), &st);
    if (rc != CPZ_OK) return Result::err(ErrorKind::Device, cpz_last_error());
    return status_result(st);
  }

 private:
  Device* dev_;
  Parameters params_;
  Statement st_;
};

// Prover (prover/mod.rs:25-132) for one witness x; the nonce k is the caller's (commit draws it
// from an rng in the reference, :115-121).
class Prover {
 public:
  Prover(Device& dev, Parameters params, Bytes32 x) : dev_(&dev), params_(params), x_(x) {}
  // prover/mod.rs:86-110: proof (and the statement y = x g, x h) for nonce k.
  Result prove_with_transcript(const Bytes32& k, const std::optional<std::vector<uint8_t>>& context, Proof* proof,
                               Statement* statement = nullptr) const {
    Statement st;
    Proof pr;
    uint8_t present = context ? 1 : 0, pad = 0;
    const uint64_t off[2] = {0, context ? context->size() : 0};
    const uint8_t* cb = (context && !context->empty()) ? context->data() : &pad;
    const int rc = cpz_prove(dev_->get(), params_.g.data(), params_.h.data(), 1, x_.data(), k.data(),
                             context ? cb : nullptr, context ? off : nullptr, context ? &present : nullptr,
                             st.y1.data(), st.y2.data(), pr.r1.data(), pr.r2.data(), pr.s.data());
    if (rc != CPZ_OK) return Result::err(ErrorKind::Device, cpz_last_error());
    if (proof) *proof = pr;
    if (statement) *statement = st;
    return Result::ok();
  }

 private:
  Device* dev_;
  Parameters params_;
  Bytes32 x_;
};

class BatchVerifier {
 public:
  explicit BatchVerifier(Device& dev) : dev_(&dev) {}
  static BatchVerifier with_capacity(Device& dev, std::size_t cap) {
    BatchVerifier b(dev);
    b.entries_.reserve(cap < MAX_BATCH_SIZE ? cap : MAX_BATCH_SIZE);
    return b;
  }

  std::size_t len() const { return entries_.size(); }
  bool is_empty() const { return entries_.empty(); }
  std::size_t remaining_capacity() const { return entries_.size() >= MAX_BATCH_SIZE ? 0 : MAX_BATCH_SIZE - entries_.size(); }

  Result add(const Parameters& p, const Statement& st, const Proof& pr) { return add_with_context(p, st, pr, std::nullopt); }

  Result add_with_context(const Parameters& p, const Statement& st, const Proof& pr,
                          std::optional<std::vector<uint8_t>> context) {
    if (entries_.size() >= MAX_BATCH_SIZE)
      return Result::err(ErrorKind::InvalidParams, "Batch size limit exceeded (max 1000)");
    Result v = validate_statement(*dev_, st);  // batch.rs:158
    if (v.is_err()) return v;
    entries_.push_back(Entry{p, st, pr, std::move(context)});
    return Result::ok();
  }

  void clear() { entries_.clear(); }

  // The caller's randomness (the reference's rng: &mut impl CryptoRngCore, batch.rs:171):
  // fills `len` bytes.  os_rng reads the OS entropy source.
  using FillBytes = std::function<void(uint8_t*, std::size_t)>;
  static void os_rng(uint8_t* out, std::size_t len) {
    std::random_device rd;
    for (std::size_t i = 0; i < len; i += 4) {
      const uint32_t v = rd();
      for (std::size_t k = 0; k < 4 && i + k < len; k++) out[i + k] = (uint8_t)(v >> (8 * k));
    }
  }

  // What verify issued for one Parameters group (tests: the drop-in's call sequence).
  struct Dispatch {
    bool rlc = false;             // cpz_verify_batch_ex (else cpz_verify_each_ex)
    std::size_t entries = 0;
    uint64_t first_index = 0;     // the group's first weight index
    Bytes32 seed{};               // the batch's seed (every group's)
    Bytes32 partial{};            // the group's RLC partial (rlc only)
    int batch_ok = 0;
  };

  // Groups of at least this many entries take the RLC check (RLC_MIN_GROUP by default).
  void set_rlc_min_group(std::size_t m) { rlc_min_group_ = m; }

  // batch.rs:171-183.  `overall` is Err for an empty batch (and device failures); otherwise
  // the vector holds one Result per entry, in entry order.  `log` (optional) receives one
  // Dispatch per group, in group order.
  std::vector<Result> verify(Result* overall = nullptr) const { return verify(os_rng, overall); }
  std::vector<Result> verify(const FillBytes& rng, Result* overall = nullptr,
                             std::vector<Dispatch>* log = nullptr) const {
    if (overall) *overall = Result::ok();
    if (entries_.empty()) {
      if (overall) *overall = Result::err(ErrorKind::InvalidParams, "Cannot verify empty batch");
      return {};
    }
    std::vector<Result> out(entries_.size());
    // Parameters groups in order of first appearance (gpu.rs: a Vec searched per entry)
    std::vector<std::pair<Parameters, std::vector<std::size_t>>> groups;
    for (std::size_t i = 0; i < entries_.size(); i++) {
      std::size_t k = 0;
      while (k < groups.size() && !(groups[k].first.g == entries_[i].params.g && groups[k].first.h == entries_[i].params.h))
        k++;
      if (k == groups.size()) groups.push_back({entries_[i].params, {}});
      groups[k].second.push_back(i);
    }
    // The caller's rng is drawn exactly as the reference draws it, so a caller that keeps using a
    // seeded rng after verify sees the reference's stream: a one-entry batch is verify_one and
    // draws nothing (batch.rs:178-180; its RLC check, when the threshold is lowered to 1, is keyed
    // by a seed from the OS entropy source); a batch of n >= 2 draws one random_scalar, 64 bytes,
    // per entry (batch.rs:239-240, ristretto.rs:146-150), whatever entry point each group takes.
    // The first 32 bytes of the first draw key every group's RLC weights.
    const bool single = entries_.size() == 1;
    Bytes32 seed{};
    if (single) {
      if (entries_.size() >= rlc_min_group_) os_rng(seed.data(), seed.size());
    } else {
      uint8_t draw[64];
      for (std::size_t i = 0; i < entries_.size(); i++) {
        rng(draw, sizeof(draw));
        if (i == 0) std::memcpy(seed.data(), draw, seed.size());
      }
    }
    uint64_t first_index = 0;
    for (const auto& grp : groups) {
      const auto& idx = grp.second;
      const std::size_t n = idx.size();
      std::vector<uint8_t> y1(32 * n), y2(32 * n), r1(32 * n), r2(32 * n), s(32 * n), ctx_bytes, present(n), st(n);
      std::vector<uint64_t> off(n + 1, 0);
      bool any_ctx = false;
      for (std::size_t k = 0; k < n; k++) {
        const Entry& e = entries_[idx[k]];
        std::memcpy(&y1[32 * k], e.statement.y1.data(), 32);
        std::memcpy(&y2[32 * k], e.statement.y2.data(), 32);
        std::memcpy(&r1[32 * k], e.proof.r1.data(), 32);
        std::memcpy(&r2[32 * k], e.proof.r2.data(), 32);
        std::memcpy(&s[32 * k], e.proof.s.data(), 32);
        present[k] = e.context.has_value() ? 1 : 0;
        if (e.context) {
          any_ctx = true;
          ctx_bytes.insert(ctx_bytes.end(), e.context->begin(), e.context->end());
        }
        off[k + 1] = ctx_bytes.size();
      }
      if (ctx_bytes.empty()) ctx_bytes.push_back(0);
      const uint8_t* cb = any_ctx ? ctx_bytes.data() : nullptr;
      const uint64_t* co = any_ctx ? off.data() : nullptr;
      const uint8_t* cp = any_ctx ? present.data() : nullptr;
      const Parameters& p = grp.first;
      Dispatch d;
      d.entries = n;
      d.first_index = first_index;
      int rc;
      if (n >= rlc_min_group_) {
        d.rlc = true;
        d.seed = seed;
        rc = cpz_verify_batch_ex(dev_->get(), CPZ_CALL_EQUATIONS_ONLY, p.g.data(), p.h.data(), n, y1.data(), y2.data(),
                                 r1.data(), r2.data(), s.data(), cb, co, cp, seed.data(), first_index,
                                 d.partial.data(), &d.batch_ok, st.data());
      } else {
        rc = cpz_verify_each_ex(dev_->get(), CPZ_CALL_EQUATIONS_ONLY, p.g.data(), p.h.data(), n, y1.data(), y2.data(),
                                r1.data(), r2.data(), s.data(), cb, co, cp, st.data());
      }
      if (rc != CPZ_OK) {
        if (overall) *overall = Result::err(ErrorKind::Device, cpz_last_error());
        return {};
      }
      first_index += n;
      if (log) log->push_back(d);
      for (std::size_t k = 0; k < n; k++) out[idx[k]] = status_result(st[k]);
    }
    return out;
  }

 private:
  struct Entry {
    Parameters params;
    Statement statement;
    Proof proof;
    std::optional<std::vector<uint8_t>> context;
  };
  Device* dev_;
  std::vector<Entry> entries_;
  std::size_t rlc_min_group_ = RLC_MIN_GROUP;
};

}  // namespace chaum_pedersen
