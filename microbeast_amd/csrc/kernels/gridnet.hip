// GridNet (BASELINE config 2) helpers around the pixel-major conv kernels (pixconv.hip,
// ops/pixconv.py), also used by the IMPALA trunk tail (ops/tail.py):
//
//   bits_pad      int32 bit-plane obs [n][h*w] -> zero-padded [n][ph*pw] (the conv.hip
//                 stage-0 kernels' input for maps padded to a multiple of 16)
//   colsum        deterministic two-stage column sums (bias gradients), bf16 or fp32 in
//   map_gather    multi-segment index gather (weight packing into the GEMM operand layouts,
//                 weight-gradient unpacking into the parameters' own layouts), one launch
//   value_bwd     critic output layer backward: dh = (dv * w2 + g_head) * (h > 0), partial
//                 dW2 / db2
//
// All index maths is 32-bit; the launchers check that every element count fits.
#include "common.h"

#include <algorithm>
#include <climits>

typedef __hip_bfloat16 bf16;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }
__device__ __forceinline__ uint32_t bf_bits(float v) {
  return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v));
}
__device__ __forceinline__ uint32_t pack2(float a, float b) { return bf_bits(a) | (bf_bits(b) << 16); }
__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16 v) { return __bfloat162float(v); }

int grid_for(long work) {
  long g = (work + kThreads - 1) / kThreads;
  return (int)(g < 1 ? 1 : g > 65535 * 4 ? 65535 * 4 : g);
}

// ------------------------------------------------------------------ bits -> padded bits
template <typename IDX>
__global__ __launch_bounds__(kThreads) void bits_pad_kernel(const uint32_t* __restrict__ bits,
                                                            int n, int h, int w, int ph, int pw,
                                                            uint32_t* __restrict__ out) {
  const IDX total = (IDX)n * ph * pw;
  for (IDX e = (IDX)blockIdx.x * kThreads + threadIdx.x; e < total; e += (IDX)gridDim.x * kThreads) {
    const int x = (int)(e % pw), t = (int)(e / pw);
    const int y = t % ph, b = t / ph;
    out[e] = (y < h && x < w) ? bits[(size_t)b * h * w + y * w + x] : 0u;
  }
}

// ------------------------------------------------------------------ column sums
// Stage 1: partial[P][C] = sums of row blocks of x [R][ld] (bf16 or fp32). Block (part,
// 64-column chunk); the 4 waves take interleaved rows, combined in LDS (fixed order).
template <typename T>
__global__ __launch_bounds__(kThreads) void colsum_part_kernel(const T* __restrict__ x, int R,
                                                               int C, int ld, int rpp,
                                                               float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.y * 64 + lane;
  const int r0 = blockIdx.x * rpp, r1 = min(R, r0 + rpp);
  float s = 0.f;
  if (col < C)
    for (int r = r0 + wave; r < r1; r += 4) s += to_f(x[(size_t)r * ld + col]);
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && col < C)
    partial[(size_t)blockIdx.x * C + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// Stage 1, vector form for bf16 rows (ld % 8 == 0, C <= 256): thread = (8-column group cg,
// row slot); 16-byte loads, 256 / CG rows per pass, fixed-order LDS combine per block.
__global__ __launch_bounds__(kThreads) void colsum_part_vec_kernel(const bf16* __restrict__ x,
                                                                   int R, int C, int ld, int rpp,
                                                                   float* __restrict__ partial) {
  __shared__ float red[kThreads][8];
  const int CG = (C + 7) >> 3, slots = kThreads / CG;
  const int cg = threadIdx.x % CG, rs = threadIdx.x / CG;
  const int r0 = blockIdx.x * rpp, r1 = min(R, r0 + rpp);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (rs < slots)
    for (int r = r0 + rs; r < r1; r += slots) {
      const uint4 u = *(const uint4*)(x + (size_t)r * ld + 8 * cg);
      const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (j & 1) ? bf_hi(uu[j >> 1]) : bf_lo(uu[j >> 1]);
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = acc[j];
  __syncthreads();
  if (threadIdx.x < CG) {
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    for (int q = 0; q < slots; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += red[q * CG + threadIdx.x][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * threadIdx.x + j;
      if (c < C) partial[(size_t)blockIdx.x * C + c] = s[j];
    }
  }
}

// Stage 2: out[c] = sum_p partial[p][c] (block per column, fixed-order tree); columns
// [0, c0) -> out0, [c0, C) -> out1 (so one reduction can fill two separate parameter
// gradients, e.g. dW2 and db2)
__global__ __launch_bounds__(kThreads) void colsum_fin_kernel(const float* __restrict__ partial,
                                                              int P, int C, float* out0, int c0,
                                                              float* out1) {
  __shared__ float red[kThreads];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int p = threadIdx.x; p < P; p += kThreads) s += partial[(size_t)p * C + c];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (c < c0) out0[c] = red[0];
    else out1[c - c0] = red[0];
  }
}

// ------------------------------------------------------------------ multi-segment gather
// dst_s[i] = map_s[i] >= 0 ? src_s[map_s[i]] : 0 for every segment s (fp32 source, fp32 or
// bf16 destination). blockIdx.y = segment.
constexpr int kMaxSeg = 24;
struct MapSeg {
  const float* src;
  void* dst;
  const int* map;
  int n, dst_bf16;
};
struct MapSegs {
  MapSeg s[kMaxSeg];
};

__global__ __launch_bounds__(kThreads) void map_gather_kernel(MapSegs a) {
  const MapSeg sg = a.s[blockIdx.y];
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < sg.n; i += gridDim.x * kThreads) {
    const int m = sg.map[i];
    const float v = m >= 0 ? sg.src[m] : 0.f;
    if (sg.dst_bf16) ((bf16*)sg.dst)[i] = __float2bfloat16(v);
    else ((float*)sg.dst)[i] = v;
  }
}

// ------------------------------------------------------------------ critic output layer
// v = h . w2 + b2 with h = relu(hidden) [R][K] bf16. Backward for dv [R] (fp32):
//   dh[r][k] = bf16(dv[r] * w2[k]) where h > 0 (the hidden relu folded in), else 0;
//   partial[part][k] = sum_r dv[r] * h[r][k] (dW2), partial[part][K] = sum_r dv[r] (db2).
// Thread = (row slot, 8 columns): G = K/8 column groups, 256/G rows per pass.
// gadd (optional, rows < gadd_rows): a second gradient of h added before the relu mask
// (fp32 or bf16 [gadd_rows][K]) -- the IMPALA actor head's dX, which consumes h too.
__global__ __launch_bounds__(kThreads) void value_bwd_kernel(const float* __restrict__ dv,
                                                             const bf16* __restrict__ h,
                                                             const float* __restrict__ w2, int R,
                                                             int K, int rpp, bf16* __restrict__ dh,
                                                             float* __restrict__ partial,
                                                             const void* __restrict__ gadd,
                                                             int gadd_rows, int gadd_f32) {
  __shared__ float red[kThreads][9];
  const int G = K >> 3, rows = kThreads / G;
  const int cg = threadIdx.x % G, rs = threadIdx.x / G;
  float w[8], sw[8], sb = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { w[j] = w2[8 * cg + j]; sw[j] = 0.f; }
  const int r0 = blockIdx.x * rpp, r1 = min(R, r0 + rpp);
  if (rs < rows)
    for (int r = r0 + rs; r < r1; r += rows) {
      const float d = dv[r];
      const uint4 u = *(const uint4*)(h + (size_t)r * K + 8 * cg);
      const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
      float ga[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) ga[j] = 0.f;
      if (r < gadd_rows) {
        if (gadd_f32) {
          const float4* gp = (const float4*)((const float*)gadd + (size_t)r * K + 8 * cg);
          const float4 a = gp[0], b = gp[1];
          ga[0] = a.x, ga[1] = a.y, ga[2] = a.z, ga[3] = a.w;
          ga[4] = b.x, ga[5] = b.y, ga[6] = b.z, ga[7] = b.w;
        } else {
          const uint4 gv = *(const uint4*)((const bf16*)gadd + (size_t)r * K + 8 * cg);
          const uint32_t gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) ga[j] = (j & 1) ? bf_hi(gg[j >> 1]) : bf_lo(gg[j >> 1]);
        }
      }
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float hj = (j & 1) ? bf_hi(uu[j >> 1]) : bf_lo(uu[j >> 1]);
        o[j] = hj > 0.f ? d * w[j] + ga[j] : 0.f;
        sw[j] += d * hj;
      }
      sb += d;
      *(uint4*)(dh + (size_t)r * K + 8 * cg) =
          make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = sw[j];
  red[threadIdx.x][8] = sb;
  __syncthreads();
  if (threadIdx.x < G) {  // fixed-order sum over the row slots of column group cg
    float acc[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[j] = 0.f;
    for (int s = 0; s < rows; ++s)
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[j] += red[s * G + threadIdx.x][j];
    float* out = partial + (size_t)blockIdx.x * (K + 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[8 * threadIdx.x + j] = acc[j];
    if (threadIdx.x == 0) out[K] = acc[8];
  }
}

bool fits(long v) { return v >= 0 && v < INT_MAX; }
// element counts past 2^31 (e.g. 262K-row learner batches) take the 64-bit index variant;
// pixel counts must still fit 32 bits
#define MBK_LAUNCH_IDX(kern, total, ...)                                                  \
  do {                                                                                   \
    if (fits(total))                                                                     \
      hipLaunchKernelGGL(kern<int>, dim3(grid_for(total)), dim3(kThreads), 0, __VA_ARGS__); \
    else                                                                                 \
      hipLaunchKernelGGL(kern<int64_t>, dim3(grid_for(total)), dim3(kThreads), 0,          \
                         __VA_ARGS__);                                                   \
  } while (0)

}  // namespace

extern "C" int mbk_bits_pad(const void* bits, int n, int h, int w, int ph, int pw, void* out,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  if (ph < h || pw < w) return (int)hipErrorInvalidValue;
  const long total = (long)n * ph * pw;
  MBK_LAUNCH_IDX(bits_pad_kernel, total, stream, (const uint32_t*)bits, n, h, w, ph, pw,
                 (uint32_t*)out);
  return (int)hipGetLastError();
}

int colsum_parts(long R) { return (int)std::max(1L, std::min(2048L, (R + 1023) / 1024)); }

// Column sums of x [R][ld] (x_f32: fp32, else bf16) into out0[0:c0] / out1[0:C-c0]
// (out1 may be null when c0 >= C). partial: colsum_parts(R) * C floats of scratch.
extern "C" int mbk_colsum(const void* x, int x_f32, int R, int C, int ld, float* partial,
                          float* out0, int c0, float* out1, hipStream_t stream) {
  if (C <= 0) return 0;
  if (R < 0 || ld < C) return (int)hipErrorInvalidValue;
  const int P = colsum_parts(R);
  const int rpp = std::max(1, (R + P - 1) / P);
  const dim3 g1(P, (C + 63) / 64);
  if (!x_f32 && ld % 8 == 0 && C <= 256 && ((uintptr_t)x & 15) == 0)
    hipLaunchKernelGGL(colsum_part_vec_kernel, dim3(P), dim3(kThreads), 0, stream, (const bf16*)x,
                       R, C, ld, rpp, partial);
  else if (x_f32)
    hipLaunchKernelGGL(colsum_part_kernel<float>, g1, dim3(kThreads), 0, stream, (const float*)x,
                       R, C, ld, rpp, partial);
  else
    hipLaunchKernelGGL(colsum_part_kernel<bf16>, g1, dim3(kThreads), 0, stream, (const bf16*)x, R,
                       C, ld, rpp, partial);
  hipLaunchKernelGGL(colsum_fin_kernel, dim3(C), dim3(kThreads), 0, stream, (const float*)partial,
                     P, C, out0, c0, out1);
  return (int)hipGetLastError();
}

extern "C" int mbk_colsum_parts(long R) { return colsum_parts(R); }

// nseg segments: src[s], dst[s], map[s], n[s], dst_bf16[s]
extern "C" int mbk_map_gather(int nseg, const void* const* src, void* const* dst,
                              const void* const* map, const int* n, const int* dst_bf16,
                              hipStream_t stream) {
  if (nseg <= 0) return 0;
  if (nseg > kMaxSeg) return (int)hipErrorInvalidValue;
  MapSegs a{};
  int mx = 0;
  for (int s = 0; s < nseg; ++s) {
    a.s[s] = MapSeg{(const float*)src[s], dst[s], (const int*)map[s], n[s], dst_bf16[s]};
    mx = std::max(mx, n[s]);
  }
  if (mx == 0) return 0;
  hipLaunchKernelGGL(map_gather_kernel, dim3(std::min(grid_for(mx), 1024), nseg), dim3(kThreads),
                     0, stream, a);
  return (int)hipGetLastError();
}

int value_parts(int R) { return std::max(1, std::min(256, (R + 1023) / 1024)); }
extern "C" int mbk_value_bwd_parts(int R) { return value_parts(R); }

// dh [R][K] bf16, partial [value_parts(R)][K+1] fp32; K % 8 == 0, K <= 2048;
// gadd: null or [gadd_rows][K] (fp32 if gadd_f32 else bf16)
extern "C" int mbk_value_bwd(const float* dv, const void* h, const float* w2, int R, int K,
                             void* dh, float* partial, const void* gadd, int gadd_rows,
                             int gadd_f32, hipStream_t stream) {
  if (R <= 0) return 0;
  if (K % 8 || K > 8 * kThreads || gadd_rows > R) return (int)hipErrorInvalidValue;
  const int P = value_parts(R);
  const int rpp = (R + P - 1) / P;
  hipLaunchKernelGGL(value_bwd_kernel, dim3(P), dim3(kThreads), 0, stream, dv, (const bf16*)h, w2,
                     R, K, rpp, (bf16*)dh, partial, gadd, gadd ? gadd_rows : 0, gadd_f32);
  return (int)hipGetLastError();
}
