// Microbenchmark: what the FETCH_SIZE counter reports for the access patterns of the RLC
// bucket kernel, against the bytes the kernels are known to read, so that the bucket
// kernel's HBM figure (profiles/rNN_rlc_bucket_pmc.json) can be read without guessing the
// gfx950 correction (MI355X_MICROARCH.md documents it for wide coalesced reads only).
//   k_stream     coalesced 16-byte loads over a 1 GiB buffer (the documented case)
//   k_gather128  one 128-byte record per thread (8 x 16-byte loads) at a random index of a
//                512 MiB array: the bucket kernel's Niels-point gathers
//   k_gather160  the same with 160-byte records (extended points, the fix-up's reads)
// The 128-byte gather runs over arrays of 64 MiB (inside the 256 MiB MALL), 512 MiB and
// 4 GiB, so a counter that skipped MALL hits would show it as a size-dependent ratio.
// Run:  rocprofv3 --pmc FETCH_SIZE -- tools/ubench/gather_bytes     (one pass per counter)
//       tools/ubench/gather_bytes    alone prints the known bytes and the achieved GB/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                               \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ src, uint64_t n16, uint4* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = src[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) sink[0] = acc;  // keeps the loads; never taken
}

template <int V>  // V 16-byte vectors per record
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ recs, const uint32_t* __restrict__ idx,
                                                uint64_t n, uint4* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4* r = recs + (uint64_t)idx[i] * V;
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < V; k++) {
    const uint4 v = r[k];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) sink[0] = acc;
}

int main() {
  const uint64_t stream_bytes = 1ull << 30;
  const uint64_t rec_bytes = 4096ull << 20;  // largest record array
  const uint64_t ngather = 1ull << 24;  // 16 M gathers per launch
  uint4 *buf, *recs, *sink;
  uint32_t* idx;
  CHECK(hipMalloc(&buf, stream_bytes));
  CHECK(hipMalloc(&recs, rec_bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&idx, ngather * 4));
  CHECK(hipMemset(buf, 1, stream_bytes));
  CHECK(hipMemset(recs, 2, rec_bytes));
  std::vector<uint32_t> base(ngather), h(ngather);
  uint64_t x = 0x243f6a8885a308d3ull;
  for (auto& v : base) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    v = (uint32_t)(x >> 33);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\"runs\": [\n");
  for (int rep = 0; rep < 3; rep++) {
    float ms;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, buf, stream_bytes / 16, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf(" {\"kernel\": \"k_stream\", \"bytes\": %llu, \"ms\": %.4f, \"GBps\": %.1f},\n",
           (unsigned long long)stream_bytes, ms, stream_bytes / (ms * 1e6));
    const uint64_t sizes[4] = {64ull << 20, 512ull << 20, 4096ull << 20, 512ull << 20};
    for (int v = 0; v < 4; v++) {
      const int V = v == 3 ? 10 : 8;
      const uint64_t nrec = sizes[v] / (16ull * V);
      for (uint64_t i = 0; i < ngather; i++) h[i] = (uint32_t)(base[i] % nrec);
      CHECK(hipMemcpy(idx, h.data(), ngather * 4, hipMemcpyHostToDevice));
      CHECK(hipEventRecord(e0));
      if (V == 8)
        hipLaunchKernelGGL(k_gather<8>, dim3((unsigned)(ngather / 256)), dim3(256), 0, 0, recs, idx, ngather, sink);
      else
        hipLaunchKernelGGL(k_gather<10>, dim3((unsigned)(ngather / 256)), dim3(256), 0, 0, recs, idx, ngather, sink);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const uint64_t bytes = ngather * 16ull * V;
      printf(" {\"kernel\": \"k_gather%d\", \"array_mib\": %llu, \"bytes\": %llu, \"index_bytes\": %llu, \"ms\": %.4f, "
             "\"GBps\": %.1f}%s\n",
             16 * V, (unsigned long long)(sizes[v] >> 20), (unsigned long long)bytes, (unsigned long long)(ngather * 4),
             ms, bytes / (ms * 1e6), rep == 2 && v == 3 ? "" : ",");
    }
  }
  printf("]}\n");
  CHECK(hipDeviceSynchronize());
  return 0;
}
