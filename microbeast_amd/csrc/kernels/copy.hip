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

// Sparse-row I/O of the captured-graph policy step (the shapes the fused acting kernel does
// not cover: other map sizes, the deep encoder, GridNet). The env workers write occupied-cell
// rows (word 0 = n | resources << 16, then cell | code << 16) into pinned host memory; one
// wave per env expands its row into the graph's dense device codes through LDS (zero, scatter,
// one coalesced store), so only a row's n + 1 words cross PCIe instead of the whole
// [S] code row of the H2D blit copy (1.15 KB per env at 24x24).
constexpr int kRowEnvs = 4;  // envs (waves) per workgroup
constexpr int kRowMaxS = 1024;
__global__ __launch_bounds__(64 * kRowEnvs) void rows_to_codes_kernel(
    const uint32_t* __restrict__ rows, int stride, int E, int S, uint16_t* __restrict__ codes,
    int32_t* __restrict__ res) {
  __shared__ uint16_t lc[kRowEnvs][kRowMaxS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * kRowEnvs + w;
  if (e >= E) return;
  uint16_t* l = lc[w];
  for (int c = lane; c < S; c += 64) l[c] = 0;
  const uint32_t* row = rows + (size_t)e * stride;
  const uint32_t w0 = row[0];
  const int n = min((int)(w0 & 0xFFFFu), S);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the zeroing is in LDS
  __builtin_amdgcn_wave_barrier();
  for (int q = 1 + lane; q <= n; q += 64) {
    const uint32_t x = row[q];
    if ((x & 0xFFFFu) < (uint32_t)S) l[x & 0xFFFFu] = (uint16_t)(x >> 16);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  uint16_t* out = codes + (size_t)e * S;
  for (int c = lane; c < S; c += 64) out[c] = l[c];
  if (lane == 0) res[e] = (int32_t)(w0 >> 16);
}

// ... and back: the graph's dense packed actions [E][S] -> the env workers' pinned action rows
// (word 0 = n, then cell | code << 16 for the non-noop cells, ascending), one wave per env.
__global__ __launch_bounds__(64 * kRowEnvs) void codes_to_rows_kernel(
    const uint16_t* __restrict__ act16, int E, int S, uint32_t* __restrict__ rows, int stride) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kRowEnvs + (threadIdx.x >> 6);
  if (e >= E) return;
  const uint16_t* a = act16 + (size_t)e * S;
  uint32_t* row = rows + (size_t)e * stride;
  int nz = 0;
  for (int c0 = 0; c0 < S; c0 += 64) {
    const int c = c0 + lane;
    const uint32_t code = c < S ? a[c] : 0u;
    const uint64_t bal = __ballot(code != 0u);
    if (code != 0u) row[1 + nz + __popcll(bal & ((1ull << lane) - 1ull))] = (uint32_t)c | (code << 16);
    nz += __popcll(bal);
  }
  if (lane == 0) row[0] = (uint32_t)nz;
}

}  // namespace

extern "C" int mbk_rows_to_codes(const uint32_t* rows, int stride, int E, int S, void* codes,
                                 int32_t* res, hipStream_t stream) {
  if (E <= 0) return 0;
  if (S > kRowMaxS || stride < S + 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_to_codes_kernel, dim3((E + kRowEnvs - 1) / kRowEnvs),
                     dim3(64 * kRowEnvs), 0, stream, rows, stride, E, S, (uint16_t*)codes, res);
  return (int)hipGetLastError();
}

extern "C" int mbk_codes_to_rows(const void* act16, int E, int S, uint32_t* rows, int stride,
                                 hipStream_t stream) {
  if (E <= 0) return 0;
  if (stride < S + 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(codes_to_rows_kernel, dim3((E + kRowEnvs - 1) / kRowEnvs),
                     dim3(64 * kRowEnvs), 0, stream, (const uint16_t*)act16, E, S, rows, stride);
  return (int)hipGetLastError();
}

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

// Stand-in for one bucket's ring all-reduce at world size 1 (parallel/dist.py rehearsal):
// `passes` sweeps of scratch += g over the bucket (a ring all-reduce over N ranks moves the
// bucket 2 (N - 1) times through each GPU, half of them with a reduce add), on a small grid
// like RCCL's channels (one workgroup per channel), so the learner / policy kernels see the
// CU, HBM and queue footprint of the collective a multi-GPU run adds. g is only read.
__global__ __launch_bounds__(256) void comm_standin_kernel(const float* __restrict__ g,
                                                           float* __restrict__ s, int64_t n,
                                                           int passes) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = 0; p < passes; ++p) {
    for (int64_t i = t0; i < n4; i += stride) {
      const float4 a = ((const float4*)g)[i];
      float4 b = ((float4*)s)[i];
      b.x += a.x; b.y += a.y; b.z += a.z; b.w += a.w;
      ((float4*)s)[i] = b;
    }
    for (int64_t i = (n4 << 2) + t0; i < n; i += stride) s[i] += g[i];
  }
}

extern "C" int mbk_comm_standin(const float* g, float* scratch, int64_t n, int passes,
                                int channels, hipStream_t stream) {
  if (n <= 0 || passes <= 0) return 0;
  if (((uintptr_t)g & 15) || ((uintptr_t)scratch & 15) || channels < 1)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(comm_standin_kernel, dim3(channels), dim3(256), 0, stream, g, scratch, n,
                     passes);
  return (int)hipGetLastError();
}
