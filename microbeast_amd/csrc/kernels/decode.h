// Device helpers for decoding the engine's 16-bit cell codes on the GPU: the 78-bit action
// mask of a cell (exactly the simulator's rules, include/microrts_rules.h) and the bit-plane
// -> bf16 expansion of the stage-0 conv. Shared by obs_mask.hip (decode kernels) and
// trunk.hip (the fused acting step, which decodes inside its conv trunk launch).
#pragma once
#include "../include/microrts_rules.h"
#include "common.h"

namespace mbk {

__device__ __forceinline__ void setb3(uint32_t w[3], int j) { w[j >> 5] |= 1u << (j & 31); }

// 78-bit action mask of cell c (real frame, player 1 = "own" in the code) from the env's
// codes cs[] (LDS), exactly the simulator's rules.
__device__ __forceinline__ void cell_mask(const uint16_t* cs, int c, int H, int W, int r,
                                          uint32_t w[3]) {
  using namespace mbr;
  w[0] = w[1] = w[2] = 0u;
  const uint16_t code = cs[c];
  const int t = code_type(code);
  // own (owner 1), idle (act noop <=> busy == 0), not a resource
  if (!(code_owner(code) == 1 && code_act(code) == A_NOOP && t != RESOURCE && t != NONE)) return;
  const int y = c / W, x = c - y * W;
  setb3(w, kSegOff[0] + A_NOOP);
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
      if (mobile) { setb3(w, kSegOff[1] + d); any_move = true; }
      const bool can_prod = (t == BASE && r >= spec_cost(WORKER)) ||
                            (t == BARRACKS && r >= spec_cost(LIGHT)) ||
                            (t == WORKER && r >= spec_cost(BARRACKS));
      if (can_prod) { setb3(w, kSegOff[4] + d); any_prod = true; }
    } else {
      if (t == WORKER && nt == RESOURCE && carried == 0 && code_res(nc) > 0) {
        setb3(w, kSegOff[2] + d); any_harv = true;
      }
      if (t == WORKER && nt == BASE && code_owner(nc) == 1 && carried > 0) {
        setb3(w, kSegOff[3] + d); any_ret = true;
      }
    }
  }
  if (any_prod) {
    if (t == BASE) setb3(w, kSegOff[5] + (WORKER - 1));
    if (t == BARRACKS) {
      if (r >= spec_cost(LIGHT)) setb3(w, kSegOff[5] + (LIGHT - 1));
      if (r >= spec_cost(HEAVY)) setb3(w, kSegOff[5] + (HEAVY - 1));
      if (r >= spec_cost(RANGED)) setb3(w, kSegOff[5] + (RANGED - 1));
    }
    if (t == WORKER) {
      if (r >= spec_cost(BASE)) setb3(w, kSegOff[5] + (BASE - 1));
      if (r >= spec_cost(BARRACKS)) setb3(w, kSegOff[5] + (BARRACKS - 1));
    }
  }
  if (spec_damage(t) > 0 && spec_range(t) == 1) {
    // range 1 (workers, light, heavy): the 4 neighbours only, not the 7x7 scan (same bits)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int tx = x + kDX[d], ty = y + kDY[d];
      if (tx < 0 || ty < 0 || tx >= W || ty >= H) continue;
      if (code_owner(cs[ty * W + tx]) == 2) {
        setb3(w, kSegOff[6] + (kDY[d] + 3) * 7 + (kDX[d] + 3)); any_att = true;
      }
    }
  } else if (spec_damage(t) > 0) {
    const int R = spec_range(t);
    for (int ay = -3; ay <= 3; ++ay)
      for (int ax = -3; ax <= 3; ++ax) {
        if (ax * ax + ay * ay > R * R || (ax == 0 && ay == 0)) continue;
        const int tx = x + ax, ty = y + ay;
        if (tx < 0 || ty < 0 || tx >= W || ty >= H) continue;
        if (code_owner(cs[ty * W + tx]) == 2) {
          setb3(w, kSegOff[6] + (ay + 3) * 7 + (ax + 3)); any_att = true;
        }
      }
  }
  if (any_move) setb3(w, kSegOff[0] + A_MOVE);
  if (any_harv) setb3(w, kSegOff[0] + A_HARVEST);
  if (any_ret) setb3(w, kSegOff[0] + A_RETURN);
  if (any_prod) setb3(w, kSegOff[0] + A_PRODUCE);
  if (any_att) setb3(w, kSegOff[0] + A_ATTACK);
}

// 8 one-hot planes (the low byte of bits) -> 8 bf16 (1.0 / 0.0): one entry of the stage-0
// conv's byte -> fragment lookup table (conv.hip conv0_row_kernel)
__device__ __forceinline__ uint4 bits8_bf16(uint32_t bits) {
  uint32_t w4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w4[j] = (((bits >> (2 * j)) & 1u) ? 0x3F80u : 0u) |
            (((bits >> (2 * j + 1)) & 1u) ? 0x3F800000u : 0u);
  return make_uint4(w4[0], w4[1], w4[2], w4[3]);
}

// lane x <- lane x-1 / x+1 inside each 16-lane DPP row, zero at the row ends (the stage-0
// conv's zero padding for its kx = 0 / 2 taps)
__device__ __forceinline__ uint32_t dpp_shr1_zero(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shl1_zero(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xF, 0xF, true);
}
// the same for floats with -inf at the row ends (max-pool padding)
__device__ __forceinline__ float dpp_shr1_ninf(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp((int)0xFF800000u, __float_as_int(v), 0x111, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_shl1_ninf(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp((int)0xFF800000u, __float_as_int(v), 0x101, 0xF, 0xF, false));
}

}  // namespace mbk
