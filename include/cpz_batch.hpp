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
//
// Errors are returned, never thrown across the ABI; `Result` carries the reference's
// error kind (src/error.rs:5-17).  Points and scalars stay as their 32-byte encodings:
// decoding and all checks run on the GPU.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <map>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "cpz.h"

namespace chaum_pedersen {

constexpr std::size_t MAX_BATCH_SIZE = 1000;  // batch.rs:48

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
    default:
      return Result::err(ErrorKind::InvalidParams, "Commitment contains identity element or response scalar is zero");
  }
}

struct Parameters {  // gadgets.rs:25-118
  Bytes32 g, h;
  Parameters() { cpz_default_generators(g.data(), h.data()); }
  Parameters(const Bytes32& g_, const Bytes32& h_) : g(g_), h(h_) {}
  bool operator<(const Parameters& o) const { return std::make_pair(g, h) < std::make_pair(o.g, o.h); }
};

struct Statement {  // gadgets.rs:177-239
  Bytes32 y1, y2;
};

struct Proof {  // gadgets.rs:245-311
  Bytes32 r1, r2, s;
};

// One GPU context; shareable by many BatchVerifiers on one thread.
class Device {
 public:
  explicit Device(int ordinal = 0) { rc_ = cpz_ctx_create(ordinal, &ctx_); }
  ~Device() { cpz_ctx_destroy(ctx_); }
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;
  bool ok() const { return rc_ == CPZ_OK && ctx_ != nullptr; }
  cpz_ctx* get() const { return ctx_; }

 private:
  cpz_ctx* ctx_ = nullptr;
  int rc_ = CPZ_EINVAL;
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
    entries_.push_back(Entry{p, st, pr, std::move(context)});
    return Result::ok();
  }

  void clear() { entries_.clear(); }

  // batch.rs:171-183.  `overall` is Err for an empty batch (and device failures);
  // otherwise the vector holds one Result per entry, in entry order.
  std::vector<Result> verify(Result* overall = nullptr) const {
    if (overall) *overall = Result::ok();
    if (entries_.empty()) {
      if (overall) *overall = Result::err(ErrorKind::InvalidParams, "Cannot verify empty batch");
      return {};
    }
    std::vector<Result> out(entries_.size());
    std::map<Parameters, std::vector<std::size_t>> groups;  // one bulk call per Parameters
    for (std::size_t i = 0; i < entries_.size(); i++) groups[entries_[i].params].push_back(i);
    for (const auto& kv : groups) {
      const auto& idx = kv.second;
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
      const int rc = cpz_verify_each(dev_->get(), kv.first.g.data(), kv.first.h.data(), n, y1.data(), y2.data(),
                                     r1.data(), r2.data(), s.data(), any_ctx ? ctx_bytes.data() : nullptr,
                                     any_ctx ? off.data() : nullptr, any_ctx ? present.data() : nullptr, st.data());
      if (rc != CPZ_OK) {
        if (overall) *overall = Result::err(ErrorKind::Device, cpz_last_error());
        return {};
      }
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
};

}  // namespace chaum_pedersen
