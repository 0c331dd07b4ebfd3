// Fused V-trace (Espeholt et al. 2018, from_importance_weights) + IMPALA
// losses + their gradients, one lane per trajectory column.
//
// Reference: libs/utils.py:277-329 (PPO_learn): a Python reverse loop over T
// with torch ops per step, then three means. Here the reverse scan runs in
// registers and the kernel writes the gradients the backward needs directly:
//   pg_loss    = -mean(logp * pg_adv)           (sign fixed)
//   value_loss = baseline_cost * mean((vs - V)^2)   (reference: 0.5*mean)
//   ent_loss   = mean(H);  total = pg + value - entropy_cost * ent
//   dL/dlogp_t = -pg_adv_t / M,  dL/dV_t = 2*bc*(V_t - vs_t)/M,
//   dL/dH_t = -entropy_cost / M,  M = T*B (the reference means over T*B).
// Inputs are time-major [T(+1), B]; values[T] is the bootstrap (no gradient).
#include "../include/mbk_api.h"
#include "common.h"

using namespace mbk;

namespace {

__global__ __launch_bounds__(256) void vtrace_kernel(
    const float* __restrict__ logp_new, const float* __restrict__ logp_old,
    const float* __restrict__ values, const float* __restrict__ reward,
    const uint8_t* __restrict__ done, const float* __restrict__ entropy, int T, int B,
    float gamma, float rho_bar, float c_bar, float pg_rho_bar, float baseline_cost,
    float entropy_cost, float reward_clip, float* __restrict__ vs_out,
    float* __restrict__ adv_out, float* __restrict__ g_logp, float* __restrict__ g_value,
    float* __restrict__ partials /* [gridDim.x][4] */) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const float invM = 1.f / ((float)T * (float)B);
  float s_pg = 0.f, s_v = 0.f, s_ent = 0.f, s_rho = 0.f;
  if (b < B) {
    const float boot = values[(size_t)T * B + b];
    float acc = 0.f;
    float vs_next = boot;  // vs_{t+1}, with vs_T = V(x_T)
    float v_next = boot;   // V_{t+1}
    g_value[(size_t)T * B + b] = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      const size_t i = (size_t)t * B + b;
      const float lpn = logp_new[i];
      const float ratio = __expf(lpn - logp_old[i]);
      const float rho = fminf(rho_bar, ratio), c = fminf(c_bar, ratio);
      float r = reward[i];
      if (reward_clip > 0.f) r = fmaxf(-reward_clip, fminf(reward_clip, r));
      const float disc = done[i] ? 0.f : gamma;
      const float v = values[i];
      const float delta = rho * (r + disc * v_next - v);
      acc = delta + disc * c * acc;
      const float vs = acc + v;
      const float adv = fminf(pg_rho_bar, ratio) * (r + disc * vs_next - v);
      if (vs_out) vs_out[i] = vs;
      if (adv_out) adv_out[i] = adv;
      g_logp[i] = -adv * invM;
      g_value[i] = 2.f * baseline_cost * (v - vs) * invM;
      s_pg -= lpn * adv;
      s_v += (vs - v) * (vs - v);
      if (entropy) s_ent += entropy[i];
      s_rho += rho;
      vs_next = vs;
      v_next = v;
    }
  }
  // block reduction -> one partial row per block (deterministic 2-pass)
  __shared__ float red[4][4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float v0 = wave_sum(s_pg), v1 = wave_sum(s_v), v2 = wave_sum(s_ent), v3 = wave_sum(s_rho);
  if (lane == 0) { red[wave][0] = v0; red[wave][1] = v1; red[wave][2] = v2; red[wave][3] = v3; }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w][threadIdx.x];
    partials[blockIdx.x * 4 + threadIdx.x] = s;
  }
}

// losses[0..4] = pg, value, entropy, total, mean_rho
__global__ __launch_bounds__(64) void vtrace_finalize_kernel(const float* __restrict__ partials,
                                                             int nblocks, int T, int B,
                                                             float baseline_cost,
                                                             float entropy_cost,
                                                             float* __restrict__ losses) {
  const int lane = threadIdx.x;
  float s[4] = {0, 0, 0, 0};
  for (int i = lane; i < nblocks; i += 64)
    for (int k = 0; k < 4; ++k) s[k] += partials[i * 4 + k];
  for (int k = 0; k < 4; ++k) s[k] = wave_sum(s[k]);
  if (lane == 0) {
    const float invM = 1.f / ((float)T * (float)B);
    const float pg = s[0] * invM, vl = baseline_cost * s[1] * invM, ent = s[2] * invM;
    losses[0] = pg;
    losses[1] = vl;
    losses[2] = ent;
    losses[3] = pg + vl - entropy_cost * ent;
    losses[4] = s[3] * invM;
  }
}

}  // namespace

extern "C" int mbk_vtrace(const float* logp_new, const float* logp_old, const float* values,
                          const float* reward, const uint8_t* done, const float* entropy, int T,
                          int B, float gamma, float rho_bar, float c_bar, float pg_rho_bar,
                          float baseline_cost, float entropy_cost, float reward_clip,
                          float* vs_out, float* adv_out, float* g_logp, float* g_value,
                          float* partials /* >= 4*ceil(B/256) */, float* losses /* 5 */,
                          hipStream_t stream) {
  const int nb = (B + 255) / 256;
  hipLaunchKernelGGL(vtrace_kernel, dim3(nb), dim3(256), 0, stream, logp_new, logp_old, values,
                     reward, done, entropy, T, B, gamma, rho_bar, c_bar, pg_rho_bar, baseline_cost,
                     entropy_cost, reward_clip, vs_out, adv_out, g_logp, g_value, partials);
  hipLaunchKernelGGL(vtrace_finalize_kernel, dim3(1), dim3(64), 0, stream, partials, nb, T, B,
                     baseline_cost, entropy_cost, losses);
  return (int)hipGetLastError();
}
