// GPU-side observation decode + action-mask generation, and env-action packing.
//
// The reference ships, per env step, a float32 (s,s,27) observation and a
// (s*s*78) uint8 mask from the JVM to Python (env_packer.py:8-14, 39-40, 87):
// 47 KB per 16x16 frame. The native engine ships 16-bit cell codes (512 B) plus
// the player's resource count and derives the 78-bit mask of every cell on the
// GPU with exactly the simulator's rules (include/microrts_rules.h), so the CPU
// never builds masks and PCIe carries 8x less. Actions go back as one packed
// 16-bit word per cell (the chosen type's parameter only).
#include "../include/mbk_api.h"
#include "../include/microrts_rules.h"
#include "common.h"

namespace {

using namespace mbr;

__device__ __forceinline__ void setb(uint32_t w[3], int j) { w[j >> 5] |= 1u << (j & 31); }

// Per-step sparse-head bookkeeping for acting (BUCKET): every active (env, cell) pair is
// appended to its cell's bucket (bucket[c * E + slot], slot from an atomic counter; order
// inside a bucket is irrelevant for sampling: the RNG is keyed by (frame, cell)), and the
// outputs of inactive cells (action, cell log-prob) are zeroed here instead of by a
// separate pass. head.hip's head_units_kernel turns the counters into the unit list.
struct Buckets {
  int* cnt;        // [S] (zero on entry; reset by head_units_kernel)
  int* bucket;     // [S][E]
  float* cell_lp;  // [E*S]
  uint8_t* action; // [E*S*7]
};

// one workgroup per env; LDS copy of the env's codes
template <bool BUCKET>
__global__ __launch_bounds__(256) void decode_obs_mask_kernel(const uint16_t* __restrict__ codes,
                                                              const int32_t* __restrict__ res,
                                                              int H, int W,
                                                              uint32_t* __restrict__ obs,
                                                              uint32_t* __restrict__ mask,
                                                              Buckets bk) {
  extern __shared__ uint16_t cs[];
  const int S = H * W;
  const size_t e = blockIdx.x;
  const uint16_t* ce = codes + e * S;
  for (int c = threadIdx.x; c < S; c += blockDim.x) cs[c] = ce[c];
  __syncthreads();
  const int r = res[e];
  for (int c = threadIdx.x; c < S; c += blockDim.x) {
    const uint16_t code = cs[c];
    obs[e * S + c] = code_bits(code);
    uint32_t w[3] = {0u, 0u, 0u};
    const int t = code_type(code);
    // own (owner 1), idle (act noop <=> busy == 0), not a resource
    if (code_owner(code) == 1 && code_act(code) == A_NOOP && t != RESOURCE && t != NONE) {
      const int x = c % W, y = c / W;
      setb(w, kSegOff[0] + A_NOOP);
      bool any_move = false, any_harv = false, any_ret = false, any_prod = false, any_att = false;
      const bool mobile = t >= WORKER;
      const int carried = code_res(code);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int nx = x + kDX[d], ny = y + kDY[d];
        if (nx < 0 || ny < 0 || nx >= W || ny >= H) continue;
        const uint16_t nc = cs[ny * W + nx];
        const int nt = code_type(nc);
        if (nt == NONE) {
          if (mobile) { setb(w, kSegOff[1] + d); any_move = true; }
          const bool can_prod = (t == BASE && r >= spec_cost(WORKER)) ||
                                (t == BARRACKS && r >= spec_cost(LIGHT)) ||
                                (t == WORKER && r >= spec_cost(BARRACKS));
          if (can_prod) { setb(w, kSegOff[4] + d); any_prod = true; }
        } else {
          if (t == WORKER && nt == RESOURCE && carried == 0 && code_res(nc) > 0) {
            setb(w, kSegOff[2] + d); any_harv = true;
          }
          if (t == WORKER && nt == BASE && code_owner(nc) == 1 && carried > 0) {
            setb(w, kSegOff[3] + d); any_ret = true;
          }
        }
      }
      if (any_prod) {
        if (t == BASE) setb(w, kSegOff[5] + (WORKER - 1));
        if (t == BARRACKS) {
          if (r >= spec_cost(LIGHT)) setb(w, kSegOff[5] + (LIGHT - 1));
          if (r >= spec_cost(HEAVY)) setb(w, kSegOff[5] + (HEAVY - 1));
          if (r >= spec_cost(RANGED)) setb(w, kSegOff[5] + (RANGED - 1));
        }
        if (t == WORKER) {
          if (r >= spec_cost(BASE)) setb(w, kSegOff[5] + (BASE - 1));
          if (r >= spec_cost(BARRACKS)) setb(w, kSegOff[5] + (BARRACKS - 1));
        }
      }
      if (spec_damage(t) > 0) {
        const int R = spec_range(t);
        for (int ay = -3; ay <= 3; ++ay)
          for (int ax = -3; ax <= 3; ++ax) {
            if (ax * ax + ay * ay > R * R || (ax == 0 && ay == 0)) continue;
            const int tx = x + ax, ty = y + ay;
            if (tx < 0 || ty < 0 || tx >= W || ty >= H) continue;
            if (code_owner(cs[ty * W + tx]) == 2) {
              setb(w, kSegOff[6] + (ay + 3) * 7 + (ax + 3)); any_att = true;
            }
          }
      }
      if (any_move) setb(w, kSegOff[0] + A_MOVE);
      if (any_harv) setb(w, kSegOff[0] + A_HARVEST);
      if (any_ret) setb(w, kSegOff[0] + A_RETURN);
      if (any_prod) setb(w, kSegOff[0] + A_PRODUCE);
      if (any_att) setb(w, kSegOff[0] + A_ATTACK);
    }
    uint32_t* m = mask + (e * S + c) * 3;
    m[0] = w[0];
    m[1] = w[1];
    m[2] = w[2];
    if (BUCKET && (w[0] | w[1] | w[2])) {
      const int slot = atomicAdd(&bk.cnt[c], 1);
      bk.bucket[(size_t)c * gridDim.x + slot] = (int)e;
    }
  }
  if (BUCKET) {
    // every cell's log-prob and 7 action bytes start at zero; the sparse head overwrites the
    // active cells later in stream order. Whole-env zeroing with 16-byte stores (the env's
    // S*7 action bytes and S floats are contiguous) instead of 1 + 7 scalar byte stores per
    // inactive cell: profile 18, decode was 10 % of the bench's GPU time
    if ((S & 15) == 0 && (((uintptr_t)bk.action | (uintptr_t)bk.cell_lp) & 15) == 0) {
      uint4* act4 = (uint4*)(bk.action + e * S * 7);
      uint4* lp4 = (uint4*)(bk.cell_lp + e * S);
      for (int i = threadIdx.x; i < S * 7 / 16; i += blockDim.x) act4[i] = make_uint4(0, 0, 0, 0);
      for (int i = threadIdx.x; i < S / 4; i += blockDim.x) lp4[i] = make_uint4(0, 0, 0, 0);
    } else {
      for (int i = threadIdx.x; i < S * 7; i += blockDim.x) bk.action[e * S * 7 + i] = 0;
      for (int i = threadIdx.x; i < S; i += blockDim.x) bk.cell_lp[e * S + i] = 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void pack_env_actions_kernel(const uint8_t* __restrict__ act,
                                                               int64_t ncells,
                                                               uint16_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ncells;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t a[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) a[k] = act[i * 7 + k];
    out[i] = pack_env_action(a);
  }
}

}  // namespace

extern "C" int mbk_decode_obs_mask(const uint16_t* codes, const int32_t* res, int n_envs, int H,
                                   int W, uint32_t* obs, uint32_t* mask, hipStream_t stream) {
  if (n_envs <= 0) return 0;
  hipLaunchKernelGGL(decode_obs_mask_kernel<false>, dim3(n_envs), dim3(256), H * W * 2, stream,
                     codes, res, H, W, obs, mask, Buckets{nullptr, nullptr, nullptr, nullptr});
  return (int)hipGetLastError();
}

extern "C" int mbk_decode_obs_mask_bucket(const uint16_t* codes, const int32_t* res, int n_envs,
                                          int H, int W, uint32_t* obs, uint32_t* mask,
                                          int* bucket_cnt, int* bucket, float* cell_lp,
                                          uint8_t* action, hipStream_t stream) {
  if (n_envs <= 0) return 0;
  hipLaunchKernelGGL(decode_obs_mask_kernel<true>, dim3(n_envs), dim3(256), H * W * 2, stream,
                     codes, res, H, W, obs, mask, Buckets{bucket_cnt, bucket, cell_lp, action});
  return (int)hipGetLastError();
}

extern "C" int mbk_pack_env_actions(const uint8_t* act, int64_t ncells, uint16_t* out,
                                    hipStream_t stream) {
  int64_t blocks = (ncells + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(pack_env_actions_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, act,
                     ncells, out);
  return (int)hipGetLastError();
}
