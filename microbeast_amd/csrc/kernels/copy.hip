// Multi-segment device copy: the per-step rollout scatter issued by the GPU
// actor engine (engine.cpp) in ONE launch instead of ~9 hipMemcpyAsync blits.
#include "../include/mbk_api.h"
#include "common.h"

#include <algorithm>

namespace {

struct SegPack {
  MbkCopySeg s[MBK_MAX_COPY_SEGS];
  int n;
};

// blockIdx.y = segment; grid-stride over 16-B chunks when both ends are
// 16-B aligned, otherwise bytes.
__global__ __launch_bounds__(256) void multi_copy_kernel(SegPack p) {
  const int k = blockIdx.y;
  if (k >= p.n) return;
  const char* src = (const char*)p.s[k].src;
  char* dst = (char*)p.s[k].dst;
  const uint64_t n = p.s[k].bytes;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const uint64_t n16 = n >> 4;
    const uint4* s4 = (const uint4*)src;
    uint4* d4 = (uint4*)dst;
    for (uint64_t i = tid; i < n16; i += stride) d4[i] = s4[i];
    for (uint64_t i = (n16 << 4) + tid; i < n; i += stride) dst[i] = src[i];
  } else if ((((uintptr_t)src | (uintptr_t)dst) & 3) == 0) {
    const uint64_t n4 = n >> 2;
    const uint32_t* s4 = (const uint32_t*)src;
    uint32_t* d4 = (uint32_t*)dst;
    for (uint64_t i = tid; i < n4; i += stride) d4[i] = s4[i];
    for (uint64_t i = (n4 << 2) + tid; i < n; i += stride) dst[i] = src[i];
  } else {
    for (uint64_t i = tid; i < n; i += stride) dst[i] = src[i];
  }
}

// Row gather: dst row i = src row idx[i] (rows of row_bytes, 16- or 4-byte granules).
// blockIdx.y = output row. The dynamic-batching policy server's request gather.
template <typename V>
__global__ __launch_bounds__(256) void row_gather_kernel(const V* __restrict__ src,
                                                         V* __restrict__ dst,
                                                         const int64_t* __restrict__ idx,
                                                         int nv) {
  const int64_t r = idx[blockIdx.y];
  const V* s = src + r * nv;
  V* d = dst + (int64_t)blockIdx.y * nv;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < nv; j += gridDim.x * 256) d[j] = s[j];
}

}  // namespace

// dst[i] = src[idx[i]] for i < k (idx: device int64), rows of row_bytes (% 4 == 0)
extern "C" int mbk_row_gather(const void* src, void* dst, const int64_t* idx, int k,
                              int64_t row_bytes, hipStream_t stream) {
  if (k <= 0) return 0;
  if (row_bytes <= 0 || row_bytes % 4 || row_bytes / 4 > (1LL << 30)) return (int)hipErrorInvalidValue;
  const bool v16 = row_bytes % 16 == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
  const int nv = (int)(row_bytes / (v16 ? 16 : 4));
  unsigned bx = (unsigned)std::min<int64_t>(64, (nv + 255) / 256);
  if (v16)
    hipLaunchKernelGGL(row_gather_kernel<uint4>, dim3(bx, k), dim3(256), 0, stream,
                       (const uint4*)src, (uint4*)dst, idx, nv);
  else
    hipLaunchKernelGGL(row_gather_kernel<uint32_t>, dim3(bx, k), dim3(256), 0, stream,
                       (const uint32_t*)src, (uint32_t*)dst, idx, nv);
  return (int)hipGetLastError();
}

// Byte fill (hipMemsetAsync), for zero-initialised buffers without an ATen fill kernel
extern "C" int mbk_memset(void* dst, int value, int64_t bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemsetAsync(dst, value, (size_t)bytes, stream);
}

extern "C" int mbk_multi_copy(const MbkCopySeg* segs, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > MBK_MAX_COPY_SEGS) return (int)hipErrorInvalidValue;
  SegPack p;
  uint64_t mx = 0;
  for (int i = 0; i < n; ++i) {
    p.s[i] = segs[i];
    if (segs[i].bytes > mx) mx = segs[i].bytes;
  }
  p.n = n;
  // ~4 x 16 B per thread per pass; cap the x-extent so small launches stay small
  uint64_t blocks = (mx / 16 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 512) blocks = 512;
  dim3 grid((unsigned)blocks, (unsigned)n);
  hipLaunchKernelGGL(multi_copy_kernel, grid, dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

// Learner-side half of the engine's policy gate (runtime/engine.h EngineConfig::policy_gate):
// `stream` waits until the flag reads 0 (no policy step's kernels in flight) before its next
// launch. A stream wait-value packet, polled by the command processor.
extern "C" int mbk_stream_wait_zero(const void* flag, hipStream_t stream) {
  return (int)hipStreamWaitValue32(stream, const_cast<void*>(flag), 0u, hipStreamWaitValueEq,
                                   0xFFFFFFFFu);
}
