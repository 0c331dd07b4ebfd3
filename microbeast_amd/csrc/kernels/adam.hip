// Flat multi-tensor Adam over ONE fp32 master buffer (all parameters are
// views of it), emitting the bf16 compute copy the kernels read in the same
// pass. Reference: torch.optim.Adam(lr=2.5e-4, eps=1e-5) over the learner
// model (microbeast.py:200, libs/utils.py:333-335) — one kernel launch here
// instead of a per-parameter loop. Optional global-norm clipping uses a
// deterministic two-pass norm (partials + finalize).
#include "../include/mbk_api.h"
#include "common.h"

using namespace mbk;

namespace {

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(const float* __restrict__ g,
                                                              int64_t n,
                                                              float* __restrict__ partials) {
  float s = 0.f;
  const int64_t n4 = n >> 2;
  const float4* g4 = (const float4*)g;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = g4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += g[i] * g[i];
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// scale[0] = min(1, max_norm / (norm + 1e-6)), scale[1] = norm (of g * gmul)
__global__ __launch_bounds__(64) void clip_scale_kernel(const float* __restrict__ partials, int nb,
                                                        float max_norm, float gmul,
                                                        float* __restrict__ scale) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 64) s += partials[i];
  s = wave_sum(s);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * gmul;  // norm of the gradient Adam will see (g * gmul)
    scale[0] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    scale[1] = norm;
  }
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   __hip_bfloat16* __restrict__ p_bf16, int64_t n,
                                                   float lr, float b1, float b2, float eps,
                                                   float wd, float bc1, float bc2,
                                                   const float* __restrict__ gscale, float gmul) {
  // gmul folds the data-parallel 1/world average into this pass (no separate scaling
  // sweep over the gradient buffer); gscale is the optional clip factor
  const float sc = (gscale ? gscale[0] : 1.f) * gmul;
  const float step = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * sc;
    float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step * mi / (sqrtf(vi) * rbc2 + eps);
    p[i] = pi;
    if (p_bf16) p_bf16[i] = __float2bfloat16(pi);
  }
}

__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ x, int64_t n,
                                                      __hip_bfloat16* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = __float2bfloat16(x[i]);
}

inline unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace

extern "C" int mbk_grad_clip_scale(const float* g, int64_t n, float max_norm, float gmul,
                                   float* partials /* >= 1024 */, float* scale /* 2 */,
                                   hipStream_t stream) {
  unsigned nb = grid_for(n / 4 + 1);
  if (nb > 1024) nb = 1024;
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nb), dim3(256), 0, stream, g, n, partials);
  hipLaunchKernelGGL(clip_scale_kernel, dim3(1), dim3(64), 0, stream, partials, (int)nb, max_norm,
                     gmul, scale);
  return (int)hipGetLastError();
}

extern "C" int mbk_adam(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n,
                        float lr, float b1, float b2, float eps, float wd, int64_t step,
                        const float* gscale, float gmul, hipStream_t stream) {
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, stream, p, g, m, v,
                     (__hip_bfloat16*)p_bf16, n, lr, b1, b2, eps, wd, bc1, bc2, gscale, gmul);
  return (int)hipGetLastError();
}

extern "C" int mbk_to_bf16(const float* x, int64_t n, void* y, hipStream_t stream) {
  hipLaunchKernelGGL(to_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, stream, x, n,
                     (__hip_bfloat16*)y);
  return (int)hipGetLastError();
}

namespace {
__global__ __launch_bounds__(256) void from_bf16_kernel(const __hip_bfloat16* __restrict__ x,
                                                        int64_t n, float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = __bfloat162float(x[i]);
}
}  // namespace

// bf16 -> fp32 widening copy (the bf16 gradient all-reduce payload back into the fp32 master
// gradient buffer, parallel/dist.py), instead of an ATen copy kernel
extern "C" int mbk_from_bf16(const void* x, int64_t n, float* y, hipStream_t stream) {
  hipLaunchKernelGGL(from_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                     (const __hip_bfloat16*)x, n, y);
  return (int)hipGetLastError();
}
