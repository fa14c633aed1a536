// The drop-in's call sequence through the C++ mirror: BatchVerifier::verify (include/cpz_batch.hpp)
// issues what rust/reference-patch/gpu.rs issues -- Parameters groups in order of first
// appearance, 64 bytes per entry from the caller's rng (the first 32 the seed), consecutive first_index, CPZ_CALL_EQUATIONS_ONLY,
// cpz_verify_batch_ex for groups of at least rlc_min_group entries and cpz_verify_each_ex
// otherwise.  Driven by tests/test_gpu_dropin.py:
//   dropin_test <input> <output>
// input (little-endian): "CPZD", u32 n, u32 rlc_min_group, seed[32] (what the rng yields),
//   then two Parameters (g, h) x 2, then per entry: u8 group, y1 y2 r1 r2 s (5 x 32 B),
//   u8 has_ctx, u32 ctx_len, ctx bytes.
// output: text, one "status <i> <code>" line per entry (the reference's error as its cpz.h
// status code) and one "dispatch <rlc> <entries> <first_index> <batch_ok> <seed hex>
// <partial hex>" line per group.  Exit 0 unless the input or a device call failed.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cpz_batch.hpp"

using namespace chaum_pedersen;

static bool rd(FILE* f, void* p, size_t n) { return std::fread(p, 1, n, f) == n; }

static int code_of(const Result& r) {
  if (r.is_ok()) return CPZ_STATUS_OK;
  for (int c = 1; c <= 5; c++) {
    const Result e = status_result((uint8_t)c);
    if (e.kind == r.kind && e.message == r.message) return c;
  }
  return 255;
}

static std::string hex(const Bytes32& b) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (uint8_t v : b) {
    s += d[v >> 4];
    s += d[v & 15];
  }
  return s;
}

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  char magic[4];
  uint32_t n = 0, rlc_min = 0;
  Bytes32 seed;
  Parameters params[2];
  if (!rd(f, magic, 4) || std::memcmp(magic, "CPZD", 4) != 0 || !rd(f, &n, 4) || !rd(f, &rlc_min, 4) ||
      !rd(f, seed.data(), 32))
    return 2;
  for (auto& p : params)
    if (!rd(f, p.g.data(), 32) || !rd(f, p.h.data(), 32)) return 2;
  Device dev(0);
  if (!dev.ok()) {
    std::fprintf(stderr, "no device: %s\n", cpz_last_error());
    return 2;
  }
  BatchVerifier b(dev);
  b.set_rlc_min_group(rlc_min);
  for (uint32_t i = 0; i < n; i++) {
    uint8_t grp = 0, has = 0;
    uint32_t len = 0;
    Statement st;
    Proof pr;
    if (!rd(f, &grp, 1) || grp > 1 || !rd(f, st.y1.data(), 32) || !rd(f, st.y2.data(), 32) ||
        !rd(f, pr.r1.data(), 32) || !rd(f, pr.r2.data(), 32) || !rd(f, pr.s.data(), 32) || !rd(f, &has, 1) ||
        !rd(f, &len, 4))
      return 2;
    std::vector<uint8_t> ctx(len);
    if (len && !rd(f, ctx.data(), len)) return 2;
    const Result r = has ? b.add_with_context(params[grp], st, pr, ctx) : b.add(params[grp], st, pr);
    if (r.is_err()) {
      std::fprintf(stderr, "add %u: %s\n", i, r.message.c_str());
      return 3;
    }
  }
  std::fclose(f);
  int draws = 0;
  std::size_t drawn = 0;
  auto rng = [&](uint8_t* out, std::size_t len) {  // yields the given seed, repeated
    draws++;
    drawn += len;
    for (std::size_t k = 0; k < len; k++) out[k] = seed[k % 32];
  };
  Result overall;
  std::vector<BatchVerifier::Dispatch> log;
  const std::vector<Result> res = b.verify(rng, &overall, &log);
  if (overall.is_err()) {
    std::fprintf(stderr, "verify: %s\n", overall.message.c_str());
    return 4;
  }
  FILE* o = std::fopen(argv[2], "w");
  if (!o) return 2;
  for (std::size_t i = 0; i < res.size(); i++) std::fprintf(o, "status %zu %d\n", i, code_of(res[i]));
  for (const auto& d : log)
    std::fprintf(o, "dispatch %d %zu %llu %d %s %s\n", d.rlc ? 1 : 0, d.entries, (unsigned long long)d.first_index,
                 d.batch_ok, hex(d.seed).c_str(), hex(d.partial).c_str());
  std::fprintf(o, "rng_draws %d %zu\n", draws, drawn);
  std::fclose(o);
  return 0;
}
