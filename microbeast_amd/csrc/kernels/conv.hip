// 3x3 / stride 1 / pad 1 convolutions of the IMPALA encoder on CDNA4 MFMA.
//
// Reference: every nn.Conv2d of ConvSequence / Residual_Block (reference
// model.py:60-61, 83) plus the relu / residual add / max_pool2d around them
// (model.py:69-73, 97) — 15 convs, 3 pools, 10 relus, 6 adds per forward, each a
// separate ATen kernel in the reference (and ~170 launches per policy step with
// MIOpen on ROCm, see profiles/). Here one launch per conv, with everything
// around it fused:
//
//   conv_fwd   : y = [pool3x3s2]( conv(relu?(x)) + bias ) * [mask_src > 0] + [add]
//                - input either NHWC bf16 (C = 16 | 32) or the env's uint32
//                  bit-plane observation expanded on the fly (27 planes -> 32 ch)
//                - implicit GEMM on v_mfma_f32_16x16x32_bf16: M = pixels (whole
//                  images per workgroup, halo'd NHWC tile in LDS, one
//                  ds_read_b128 A-fragment per lane), N = Cout, K = 9*Cin;
//                  all B fragments (weights) live in VGPRs for the launch
//                - the same kernel is the data-gradient (dgrad) with flipped /
//                  transposed weights: dx = convT(dy) * (x_pre > 0) + dres
//   conv_wgrad : dW[co][t][ci] = sum_p dy[p][co] * relu?(x)[p + t][ci]
//                K = pixels; BOTH operands come from plain NHWC LDS tiles via
//                ds_read_b64_tr_b16 (CDNA4 transposed LDS read: 4 pixels of one
//                channel per lane), so no im2col is ever materialised; per-WG
//                fp32 partials + a deterministic reduce (bias grad included)
//   pool_bwd   : gather form of max_pool2d(3,2,1) backward (no atomics)
//   conv_pack  : fp32 [Cout][Cin][3][3] params -> packed bf16 fwd / dgrad layouts
//
// Layouts: activations NHWC bf16. Packed fwd weights wf[co][chunk][32] with
// chunk = tap (Cin 32) or tap pair (Cin 16: k = h*16 + ci for tap 2c+h).
#include "../include/mbk_api.h"
#include "common.h"

#include <algorithm>
#include <map>
#include <mutex>

using namespace mbk;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float bf2f(bf16 v) { return __bfloat162float(v); }
__device__ __forceinline__ bf16 f2bf(float v) { return __float2bfloat16(v); }

typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t w) {
  // bf16 pair: sign bit set (negative, -0) -> +0 as ONE v_pk_max_i16 (a bf16 with the
  // sign bit set is a negative int16, a non-negative one a non-negative int16)
  s16x2 v = __builtin_bit_cast(s16x2, w);
  v = __builtin_elementwise_max(v, s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, v);
}

union Frag8 {
  bf16x8 v;
  uint4 u;
  s16x4 h[2];
};

template <int CIN>
struct Geo {
  static constexpr int NCH = CIN == 16 ? 5 : 9;  // K chunks of 32
  static constexpr int PIXB = CIN * 2 + 16;       // padded NHWC pixel stride in LDS (bytes)
  static constexpr int PIXB8 = CIN + 8;           // fp8 tile pixel stride
};

struct ConvFwdArgs {
  const void* x;
  const bf16* w;
  const float* bias;
  const bf16* add;
  const bf16* mask_src;
  bf16* y;
  bf16* y_full;
  uint8_t* pool_idx;  // pooled argmax (0..8 in the 3x3 window) for the backward
  int N, H, W, imgs, relu_in, pool;
  const float* wscale;  // fp8 path: per-output-channel dequant scale of the e4m3 weights
  int* queue = nullptr;  // conv0_row kernels: per-wave image queue (common.h), null: static
};

// ------------------------------------------------------------------ forward / dgrad
// Persistent: the grid is sized to the CUs' occupancy and each workgroup walks image
// groups blockIdx.x, +gridDim.x, ... holding the weights in VGPRs for the whole launch
// (a per-group launch re-read all B fragments from L2 for every 1-16 images). The next
// group's interior pixels are loaded into registers (kPF per thread) while the current
// group computes; the halo ring of the LDS tile is zeroed once and never rewritten.
// MFMA operands are (A = weights, B = pixels), so a lane's accumulators are 4
// consecutive channels of one pixel and the epilogue moves 8-byte vectors.
constexpr int kPF = 8;

__device__ __forceinline__ uint4 expand_bits8(uint32_t bits) {
  // 8 one-hot planes -> 8 bf16 (1.0 / 0.0)
  uint32_t w4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w4[j] = (((bits >> (2 * j)) & 1u) ? 0x3F80u : 0u) |
            (((bits >> (2 * j + 1)) & 1u) ? 0x3F800000u : 0u);
  return make_uint4(w4[0], w4[1], w4[2], w4[3]);
}

__device__ __forceinline__ uint2 expand_bits8_fp8(uint32_t bits) {
  // 8 one-hot planes -> 8 OCP e4m3 bytes (1.0 = 0x38)
  uint32_t w2[2] = {0u, 0u};
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if ((bits >> j) & 1u) w2[j >> 2] |= 0x38u << (8 * (j & 3));
  return make_uint2(w2[0], w2[1]);
}

__device__ __forceinline__ uint32_t cvt_fp8x4(float a, float b, float c, float d) {
  // round-to-nearest-even into OCP e4m3 (gfx950), saturated to +-448
  auto sat = [](float v) { return fminf(fmaxf(v, -448.f), 448.f); };
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(d), w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ uint2 bf16x8_to_fp8(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  float f[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w[j] << 16);
    f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
  return make_uint2(cvt_fp8x4(f[0], f[1], f[2], f[3]), cvt_fp8x4(f[4], f[5], f[6], f[7]));
}

template <int CIN, bool BITS, bool F8>
__device__ __forceinline__ int fwd_lds_off(int e, int H, int W) {
  // interior staging element e -> byte offset of its slot in the halo'd LDS tile
  constexpr int PIXB = F8 ? Geo<CIN>::PIXB8 : Geo<CIN>::PIXB;
  const int Hp = H + 2, Wp = W + 2, HW = H * W;
  if (BITS) {  // one u32 of bit planes per pixel, expanded to 32 channels
    const int im = e / HW, r = e - im * HW, y = r / W, x = r - y * W;
    return ((im * Hp + y + 1) * Wp + x + 1) * PIXB;
  } else {
    constexpr int CH16 = CIN / 8;
    const int q = e % CH16, p = e / CH16;
    const int im = p / HW, r = p - im * HW, y = r / W, x = r - y * W;
    return ((im * Hp + y + 1) * Wp + x + 1) * PIXB + q * (F8 ? 8 : 16);
  }
}

// F8: the tile holds OCP e4m3 activations (converted at staging: half the LDS bytes and
// read traffic), weights are e4m3 with a power-of-two per-output-channel scale, and the
// MFMA is v_mfma_f32_16x16x32_fp8_fp8 (same lane map as the bf16 form). Inference only.

template <int CIN, int COUT, bool BITS, bool F8>
__global__ __launch_bounds__(kThreads) void conv_fwd_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NCH = Geo<CIN>::NCH;
  constexpr int PIXB = F8 ? Geo<CIN>::PIXB8 : Geo<CIN>::PIXB;  // bits expanded at staging
  constexpr int NB = COUT / 16;
  constexpr int EPP = BITS ? 1 : CIN / 8;  // staging elements per pixel (u32 / uint4)
  constexpr int OSTR = COUT + 4;           // pool staging row stride (bf16, bank spread)
  const int H = a.H, W = a.W, HW = H * W, Hp = H + 2, Wp = W + 2;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  char* tile = smem;
  const int tile_bytes = ((a.imgs * Hp * Wp * PIXB) + 15) & ~15;
  // pool staging [imgs*HW][OSTR] of the bf16-rounded conv outputs (what y_full holds and
  // what the pool compares): half the LDS of an fp32 tile, so more images per iteration
  bf16* otile = (bf16*)(smem + tile_bytes);
  const int ngroups = (a.N + a.imgs - 1) / a.imgs;
  const int per_grp = a.imgs * HW * EPP;

  for (int e = tid; e < tile_bytes / 16; e += kThreads) ((uint4*)tile)[e] = make_uint4(0, 0, 0, 0);
  int loff[kPF];
#pragma unroll
  for (int k = 0; k < kPF; ++k) {
    const int e = tid + k * kThreads;
    loff[k] = e < per_grp ? fwd_lds_off<CIN, BITS, F8>(e, H, W) : 0;
  }
  // ---- weights -> registers (A fragments): lane holds w[co = nb*16 + li][c][8g..8g+7]
  Frag8 bw[NCH][NB];
  long bw8[NCH][NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if constexpr (F8) {
      const long* wp = (const long*)((const uint8_t*)a.w + (size_t)(nb * 16 + li) * NCH * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH; ++c) bw8[c][nb] = wp[c * 4];
    } else {
      const uint4* wp = (const uint4*)(a.w + (size_t)(nb * 16 + li) * NCH * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH; ++c) bw[c][nb].u = wp[c * 4];
    }
  }
  float bias_v[NB][4], wsc[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bias_v[nb][i] = a.bias ? a.bias[nb * 16 + 4 * g + i] : 0.f;
      wsc[nb][i] = F8 ? a.wscale[nb * 16 + 4 * g + i] : 1.f;
    }

  // ---- register prefetch of one group's interior pixels
  uint4 pv[kPF];
  uint32_t pw[kPF];
  auto prefetch = [&](int grp) {
    const size_t base = (size_t)grp * per_grp;
    const int lim = min(per_grp, (a.N - grp * a.imgs) * HW * EPP);
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int e = tid + k * kThreads;
      if (BITS) pw[k] = e < lim ? ((const uint32_t*)a.x)[base + e] : 0u;
      else pv[k] = e < lim ? ((const uint4*)a.x)[base + e] : make_uint4(0, 0, 0, 0);
    }
  };
  auto put = [&](int off, uint4 v) {
    if (a.relu_in) {
      v.x = relu_bf16x2(v.x); v.y = relu_bf16x2(v.y);
      v.z = relu_bf16x2(v.z); v.w = relu_bf16x2(v.w);
    }
    if constexpr (F8) *(uint2*)(tile + off) = bf16x8_to_fp8(v);
    else *(uint4*)(tile + off) = v;
  };
  auto put_bits = [&](int off, uint32_t bits) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (F8) *(uint2*)(tile + off + q * 8) = expand_bits8_fp8(bits >> (8 * q));
      else *(uint4*)(tile + off + q * 16) = expand_bits8(bits >> (8 * q));
    }
  };
  // per-lane byte offset of K chunk c from the block's tap-(0,0) pixel: this lane's K group
  // (g) reads tap 2c + (g >> 1), channels 8 (g & 1).. (CIN 16) or tap c, channels 8g.. (CIN
  // 32); computed once instead of per chunk and block (the kernels were VALU-bound, profile 15)
  int coff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    int tap, ch0;
    if (CIN == 16) { tap = 2 * c + (g >> 1); ch0 = 8 * (g & 1); }
    else { tap = c; ch0 = 8 * g; }
    const int tapc = tap < 9 ? tap : 8;  // CIN=16 pads chunk 4 with a zero tap
    coff[c] = ((tapc / 3) * Wp + (tapc % 3)) * PIXB + (F8 ? ch0 : ch0 * 2);
  }
  if ((int)blockIdx.x < ngroups) prefetch(blockIdx.x);
  __syncthreads();  // halo zeros visible

  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * a.imgs;
    const int nimg = min(a.imgs, a.N - img0);
    const int lim = nimg * HW * EPP;
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int e = tid + k * kThreads;
      if (e < lim) {
        if (BITS) put_bits(loff[k], pw[k]);
        else put(loff[k], pv[k]);
      }
    }
    for (int e = tid + kPF * kThreads; e < lim; e += kThreads) {  // groups beyond the prefetch
      const size_t src = (size_t)grp * per_grp + e;
      if (BITS) put_bits(fwd_lds_off<CIN, BITS, F8>(e, H, W), ((const uint32_t*)a.x)[src]);
      else put(fwd_lds_off<CIN, BITS, F8>(e, H, W), ((const uint4*)a.x)[src]);
    }
    __syncthreads();
    if (grp + (int)gridDim.x < ngroups) prefetch(grp + gridDim.x);

    const int M = nimg * HW;
    const int nblk = (M + 15) >> 4;
    const size_t gpix0 = (size_t)img0 * HW;
    for (int pb = wave; pb < nblk; pb += kThreads / 64) {
      const int m = pb * 16 + li;  // this lane's pixel (B column)
      const bool valid = m < M;
      const int mm = valid ? m : 0;  // rows past M compute garbage that is never stored
      // float-reciprocal index math (exact: index_math_ok() bounds imgs*H*W at launch): the
      // integer divisions by runtime H*W / W are ~20 VALU per block
      const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
      const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
      const int base_pos = (im * Hp + y) * Wp + x;  // padded position of tap (0,0)
      // epilogue operands (residual / relu-mask source) requested before the MFMA chain so
      // their global-load latency overlaps it instead of stalling each block's epilogue
      uint2 ep_ms[NB], ep_ad[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const size_t gi = (gpix0 + mm) * COUT + nb * 16 + 4 * g;
        ep_ms[nb] = (a.mask_src && valid) ? *(const uint2*)(a.mask_src + gi) : make_uint2(0, 0);
        ep_ad[nb] = (a.add && valid) ? *(const uint2*)(a.add + gi) : make_uint2(0, 0);
      }
      f32x4 acc[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* bp = tile + base_pos * PIXB;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        Frag8 av;
        // no zeroing: the CIN-16 pad tap has zero packed weights and rows past M are not
        // stored, so the (finite) fragment read for them cannot change a stored output
        if constexpr (F8) {
          long a8 = *(const long*)(bp + coff[c]);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(bw8[c][nb], a8, acc[nb], 0, 0, 0);
        } else {
          av.u = *(const uint4*)(bp + coff[c]);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[c][nb].v, av.v, acc[nb], 0, 0, 0);
        }
      }
      if (!valid) continue;
      // ---- epilogue: lane holds channels nb*16 + 4g + i of pixel m
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int co0 = nb * 16 + 4 * g;
        const size_t gi = (gpix0 + m) * COUT + co0;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[nb][i] * wsc[nb][i] + bias_v[nb][i];
        if (a.mask_src) {
          const uint2 ms = ep_ms[nb];
          const uint32_t mw[2] = {ms.x, ms.y};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            if (!(__uint_as_float(hb << 16) > 0.f)) v[i] = 0.f;
          }
        }
        if (a.add) {
          const uint2 ad = ep_ad[nb];
          const uint32_t aw[2] = {ad.x, ad.y};
#pragma unroll
          for (int i = 0; i < 4; ++i)
            v[i] += __uint_as_float(((aw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) << 16);
        }
        uint32_t o[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          o[j] = (uint32_t)__bfloat16_as_ushort(f2bf(v[2 * j])) |
                 ((uint32_t)__bfloat16_as_ushort(f2bf(v[2 * j + 1])) << 16);
        if (a.pool) {
          // pool over the bf16-rounded values (what y_full holds)
          *(uint2*)(otile + m * OSTR + co0) = make_uint2(o[0], o[1]);
          if (a.y_full) *(uint2*)(a.y_full + gi) = make_uint2(o[0], o[1]);
        } else {
          *(uint2*)(a.y + gi) = make_uint2(o[0], o[1]);
        }
      }
    }
    if (a.pool) {
      __syncthreads();
      // ---- max_pool2d(kernel 3, stride 2, pad 1), 4 channels per thread
      const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
      mbk::pool_tile<COUT, OSTR, kThreads>(otile, H, W, nimg, (size_t)img0 * Ho * Wo * COUT, a.y, a.pool_idx,
                            tid);
    }
    __syncthreads();  // tile / otile reads done before the next group is staged
  }
}


// ------------------------------------------------------------------ first conv, W == 16
// Stage-0 conv of the 16-wide maps straight from the uint32 bit planes, without an LDS
// im2col tile. One image row is exactly one 16-pixel MFMA block (lane li = pixel x), so a
// wave owns one image and walks its rows keeping the expanded input rows y-1 .. y+2 in
// VGPRs: every input pixel is read from HBM and expanded once (the generic kernel issues
// 9 LDS fragment reads per 16-pixel block, profile 12: LDS-bound at 11 % MFMA). The kx = 0
// and kx = 2 taps are the same row shifted by one pixel: DPP row_shr:1 / row_shl:1 move
// lane x-1 / x+1 into lane x inside each 16-lane row, and their zero fill at the row ends
// is the conv's zero padding. Two output rows per iteration give two independent MFMA
// chains; each chain runs the taps in the generic kernel's order, so results are
// bit-identical to it. Conv outputs (+bias, bf16) go to an LDS staging tile and the
// 3x3/2 max-pool (+argmax) runs over the workgroup's images as in conv_fwd_kernel.
constexpr int kRowImgs = kThreads / 64;  // images per workgroup iteration: one per wave

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {  // lane x <- lane x-1 (x=0: 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t v) {  // lane x <- lane x+1 (x=15: 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, false);
}
__device__ __forceinline__ bf16x8 shr_px(const Frag8& f) {
  Frag8 o;
  o.u = make_uint4(dpp_shr1(f.u.x), dpp_shr1(f.u.y), dpp_shr1(f.u.z), dpp_shr1(f.u.w));
  return o.v;
}
__device__ __forceinline__ bf16x8 shl_px(const Frag8& f) {
  Frag8 o;
  o.u = make_uint4(dpp_shl1(f.u.x), dpp_shl1(f.u.y), dpp_shl1(f.u.z), dpp_shl1(f.u.w));
  return o.v;
}

// Bit-plane expansion through a 256-entry LDS table (byte -> 8 bf16, 4 KB) instead of ~24
// VALU bit ops per row, and the kx = 0 / 2 taps from DPP-shifted 32-bit BIT words (2 DPP
// per row instead of 8 on the expanded fragments, each needing a zeroed destination): the
// kernel was VALU-bound (72 % VALU busy, 15 VALU per MFMA, counters in profile 20).
// HT > 0: compile-time map height, all HT input rows of an image loaded in one batch;
// HT == 0: runtime height, rows loaded one pair ahead.
constexpr int kLutBytes = 256 * 16;

__device__ __forceinline__ uint32_t dpp_shr1_b(uint32_t v) {  // lane x <- lane x-1 (x=0: 0)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shl1_b(uint32_t v) {  // lane x <- lane x+1 (x=15: 0)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xF, 0xF, true);
}

struct Row3 {  // one input row's LUT offsets for pixels x-1 (l), x (c), x+1 (h) of lane x
  uint32_t l, c, h;
};
struct XRow3 {  // the same row expanded: kx = 0, 1, 2 B fragments
  Frag8 f[3];
};

// max_pool2d(3, 2, 1) + argmax of ONE 16 x 16 image's conv outputs in LDS by its own wave
// (same values and argmax bytes as mbk::pool_tile): lane = (pooled column ox, 4-channel
// group c4, row half); each lane walks its pooled rows top to bottom. Separable: a row's
// 3-wide horizontal max (first maximising kx) is computed once and shared by the two windows
// that contain the row; the vertical pass keeps the first maximising ky, so the index is the
// first maximum in scan order. W = H = 16: only x = -1 / y = -1 fall outside the map.
template <int COUT, int OSTR>
__device__ __forceinline__ void pool_img16(const bf16* __restrict__ ot, size_t obase,
                                           bf16* __restrict__ y, uint8_t* __restrict__ pool_idx,
                                           int lane) {
  constexpr int C4 = COUT / 4, ROWS = C4;  // pooled rows per lane: 8 rows x 8 x C4 / 64 lanes
  static_assert(C4 == 4 || C4 == 8, "16 or 32 channels");
  const int ox = lane & 7, c4 = (lane >> 3) % C4, oy0 = (lane >> 3) / C4 * ROWS;
  struct HRow { float m[4]; int k[4]; };
  auto hrow = [&](int yy) {  // horizontal max of input row yy over x = 2 ox - 1 .. 2 ox + 1
    HRow h;
    const bf16* b = ot + (yy * 16 + 2 * ox) * OSTR + 4 * c4;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      float v[4];
      if (kx == 0 && ox == 0) {
        v[0] = v[1] = v[2] = v[3] = -INFINITY;
      } else {
        const uint2 u = *(const uint2*)(b + (kx - 1) * OSTR);
        v[0] = __uint_as_float(u.x << 16);
        v[1] = __uint_as_float(u.x & 0xFFFF0000u);
        v[2] = __uint_as_float(u.y << 16);
        v[3] = __uint_as_float(u.y & 0xFFFF0000u);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kx == 0 || v[j] > h.m[j]) { h.m[j] = v[j]; h.k[j] = kx; }
      }
    }
    return h;
  };
  HRow top;
  if (oy0 == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { top.m[j] = -INFINITY; top.k[j] = 0; }
  } else {
    top = hrow(2 * oy0 - 1);
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int oy = oy0 + r;
    const HRow mid = hrow(2 * oy), bot = hrow(2 * oy + 1);
    float m[4];
    uint32_t am = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int ix = top.k[j];          // ky = 0 (a -inf row never wins: mid is inside the map)
      m[j] = top.m[j];
      if (mid.m[j] > m[j]) { m[j] = mid.m[j]; ix = 3 + mid.k[j]; }
      if (bot.m[j] > m[j]) { m[j] = bot.m[j]; ix = 6 + bot.k[j]; }
      am |= (uint32_t)ix << (8 * j);
    }
    const size_t oi = obase + (size_t)(oy * 8 + ox) * COUT + 4 * c4;
    // the maxima are loaded bf16 values: their float bits carry the bf16 exactly
    *(uint2*)(y + oi) = make_uint2((__float_as_uint(m[0]) >> 16) | (__float_as_uint(m[1]) & 0xFFFF0000u),
                                   (__float_as_uint(m[2]) >> 16) | (__float_as_uint(m[3]) & 0xFFFF0000u));
    if (pool_idx) *(uint32_t*)(pool_idx + oi) = am;
    top = bot;
  }
}

// WIDE: maps 17..32 pixels wide (24x24: BASELINE config 4) in 16-column blocks; the DPP pixel
// shifts cannot cross a block, so lane 0's left and lane 15's right neighbour words come from
// the next column block's row word (loaded uniformly); the pre-pool LDS tile drops its row
// padding (OSTR = COUT) so 8 images of 24 x 24 x 16 fit next to the LUT (151 KB).
// Pre-pool tile row stride (bf16): 24 for 16 channels puts pool_img16's b64 reads on disjoint
// banks in each half-wave (2-way at 20; the epilogue's b64 writes go 1 -> 2-way, but the pool
// reads outnumber them, tools/lds_banks.py rules): 2.40 -> 2.27-2.31 ms per 524K images with
// the v_bfe LUT addresses below (profile 43).
constexpr int conv0_ostr(int cout, bool wide) { return wide ? cout : cout == 16 ? 24 : cout + 4; }

template <int HT, int COUT, bool WIDE>
__device__ __forceinline__ void conv0_row_body(const ConvFwdArgs& a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int OSTR = conv0_ostr(COUT, WIDE), CB = COUT / 16;
  const int W = WIDE ? a.W : 16;
  const int H = HT > 0 ? HT : a.H, HW = H * W;
  const int NCB = WIDE ? (W + 15) >> 4 : 1;  // column blocks
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  uint4* lut = (uint4*)smem;                 // [256] byte -> 8 bf16 planes
  bf16* otile = (bf16*)(smem + kLutBytes);   // [kRowImgs * HW][OSTR] conv outputs (pool mode)
  for (int i = tid; i < 256; i += kThreads) lut[i] = expand_bits8((uint32_t)i);
  Frag8 bw[CB][9];            // A fragments: w[co = 16 cb + li][tap][8g .. 8g+7]
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const uint4* wp = (const uint4*)(a.w + (size_t)(16 * cb + li) * 9 * 32 + g * 8);
#pragma unroll
    for (int c = 0; c < 9; ++c) bw[cb][c].u = wp[c * 4];
  }
  float bias_v[CB][4];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) bias_v[cb][i] = a.bias ? a.bias[16 * cb + 4 * g + i] : 0.f;
  const int ngroups = (a.N + kRowImgs - 1) / kRowImgs;
  __syncthreads();  // LUT ready
  const int sh = 8 * g;
  // bytes this lane's 8 planes (group g) take from the LUT; bl / bh: the words left of lane 0
  // and right of lane 15 (0 = the conv's zero padding; only WIDE blocks pass others)
  auto row = [&](uint32_t bits, uint32_t bl = 0u, uint32_t bh = 0u) {
    Row3 r;
    uint32_t lw = dpp_shr1_b(bits), hw = dpp_shl1_b(bits);
    if (WIDE) {
      lw = li == 0 ? bl : lw;
      hw = li == 15 ? bh : hw;
    }
    // one v_bfe_u32 per byte (shift + and of the plain form: 96 fewer VALU per 16x16 image)
    r.c = __builtin_amdgcn_ubfe(bits, (uint32_t)sh, 8u) * 16u;
    r.l = __builtin_amdgcn_ubfe(lw, (uint32_t)sh, 8u) * 16u;
    r.h = __builtin_amdgcn_ubfe(hw, (uint32_t)sh, 8u) * 16u;
    return r;
  };
  const char* lutb = (const char*)lut;
  // an input row's three expanded (kx) fragments, kept in registers while the row is in the
  // 4-row window: each row is expanded once (3 LUT reads) and serves two row pairs. (Time
  // unchanged: 2.2 ms per 524K images before and after, and with the next group's rows
  // prefetched; it scales with the MFMA count -- 4.4 ms at 32 channels.)
  auto xrow = [&](uint32_t bits, uint32_t bl = 0u, uint32_t bh = 0u) {
    const Row3 r = row(bits, bl, bh);
    XRow3 x;
    x.f[0].u = *(const uint4*)(lutb + r.l);
    x.f[1].u = *(const uint4*)(lutb + r.c);
    x.f[2].u = *(const uint4*)(lutb + r.h);
    return x;
  };
  XRow3 xzero;
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) xzero.f[kx].u = make_uint4(0, 0, 0, 0);
  // one output row pair (y, y+1) from input rows y-1 .. y+2; each (row, kx) fragment feeds
  // both rows' MFMA chains (and, for 32 output channels, both channel blocks) in their tap
  // order
  // skip: the pair's four input rows are all zero (a padded map's rows, e.g. GridNet's 10x10
  // maps padded to 16): the MFMA sums are exactly +0, so only the bias is written
  auto row_pair = [&](const XRow3 r[4], int y, int im, int img0, int x0 = 0, bool skip = false) {
    f32x4 acc0[CB], acc1[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc0[cb] = acc1[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (skip) break;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const Frag8& f = r[q].f[kx];
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          if (q < 3)
            acc0[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[cb][3 * q + kx].v, f.v, acc0[cb], 0, 0, 0);
          if (q > 0)
            acc1[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[cb][3 * (q - 1) + kx].v, f.v, acc1[cb], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int yy = y + h;
      if (yy >= H) break;
      if (WIDE && x0 + li >= W) break;
      const int m = yy * W + x0 + li;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const f32x4& acc = h ? acc1[cb] : acc0[cb];
        uint32_t o[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          o[j] = (uint32_t)__bfloat16_as_ushort(f2bf(acc[2 * j] * 1.f + bias_v[cb][2 * j])) |
                 ((uint32_t)__bfloat16_as_ushort(f2bf(acc[2 * j + 1] * 1.f + bias_v[cb][2 * j + 1]))
                  << 16);
        const int c = 16 * cb + 4 * g;
        const size_t gi = ((size_t)(img0 + im) * HW + m) * COUT + c;
        if (a.pool) {
          *(uint2*)(otile + (im * HW + m) * OSTR + c) = make_uint2(o[0], o[1]);
          if (a.y_full) *(uint2*)(a.y_full + gi) = make_uint2(o[0], o[1]);
        } else {
          *(uint2*)(a.y + gi) = make_uint2(o[0], o[1]);
        }
      }
    }
  };
  constexpr int NR = HT > 0 ? HT : 1;

  // this wave's image img0 + wave: conv rows, then its pool (each wave pools its own image's LDS
  // rows: no workgroup barrier, so one wave's pool (VALU / LDS) overlaps the other waves' MFMA
  // rows. LDS ops of a wave complete in order; the fences only keep the compiler from moving
  // them across)
  auto one = [&](int img0) {
    if constexpr (HT > 0) {
      uint32_t rows[NR];  // this wave's image, all rows (lane: column li)
      {
        const uint32_t* xb = (const uint32_t*)a.x + (size_t)(img0 + wave) * HW + li;
#pragma unroll
        for (int y = 0; y < NR; ++y) rows[y] = xb[y * W];
      }
      XRow3 r[4];
      r[0] = xzero;
      r[1] = xrow(rows[0]);
      r[2] = NR > 1 ? xrow(rows[1 % NR]) : xzero;
      r[3] = NR > 2 ? xrow(rows[2 % NR]) : xzero;
#pragma unroll
      for (int y = 0; y < NR; y += 2) {
        const uint32_t any = (y >= 1 ? rows[(y + NR - 1) % NR] : 0u) | rows[y % NR] |
                             (y + 1 < NR ? rows[(y + 1) % NR] : 0u) |
                             (y + 2 < NR ? rows[(y + 2) % NR] : 0u);
        row_pair(r, y, wave, img0, 0, __ballot(any != 0u) == 0ull);
        r[0] = r[2];
        r[1] = r[3];
        r[2] = y + 3 < NR ? xrow(rows[(y + 3) % NR]) : xzero;
        r[3] = y + 4 < NR ? xrow(rows[(y + 4) % NR]) : xzero;
      }
    } else if constexpr (WIDE) {
      const int im = wave;
      const uint32_t* xi = (const uint32_t*)a.x + (size_t)(img0 + im) * HW;
      for (int cbk = 0; cbk < NCB; ++cbk) {
        const int x0 = 16 * cbk;
        const bool in = x0 + li < W, has_r = x0 + 16 < W;
        // row yy of this column block: the lane's word and the block's two edge neighbours
        // (rows outside the image: zero words, which expand to zero fragments)
        auto ldw = [&](int yy) {
          uint3 v = make_uint3(0u, 0u, 0u);
          if (yy >= 0 && yy < H) {
            const uint32_t* rp = xi + (size_t)yy * W;
            v = make_uint3(in ? rp[x0 + li] : 0u, x0 > 0 ? rp[x0 - 1] : 0u,
                           has_r ? rp[x0 + 16] : 0u);
          }
          return v;
        };
        auto xrw = [&](uint3 v) { return xrow(v.x, v.y, v.z); };
        XRow3 r[4];
        r[0] = xzero;
        r[1] = xrw(ldw(0));
        r[2] = xrw(ldw(1));
        r[3] = xrw(ldw(2));
        for (int y = 0; y < H; y += 2) {
          // the next pair's input rows load during this pair's MFMAs (expanding them right
          // after their loads exposed two global-load latencies per row pair: 9.0 ms per
          // 524K 24x24 images)
          const uint3 n0 = ldw(y + 3), n1 = ldw(y + 4);
          row_pair(r, y, im, img0, x0);
          r[0] = r[2];
          r[1] = r[3];
          r[2] = xrw(n0);
          r[3] = xrw(n1);
        }
      }
    } else {
      const int im = wave;
      const uint32_t* xb = (const uint32_t*)a.x + (size_t)(img0 + im) * HW + li;
      XRow3 r[4];  // expanded input rows y-1, y, y+1, y+2 (zero outside the image)
      r[0] = xzero;
      r[1] = xrow(xb[0]);
      r[2] = H > 1 ? xrow(xb[W]) : xzero;
      r[3] = H > 2 ? xrow(xb[2 * W]) : xzero;
      for (int y = 0; y < H; y += 2) {
        const uint32_t n0 = y + 3 < H ? xb[(y + 3) * W] : 0u;  // next iteration's rows
        const uint32_t n1 = y + 4 < H ? xb[(y + 4) * W] : 0u;
        row_pair(r, y, im, img0);
        r[0] = r[2];
        r[1] = r[3];
        r[2] = y + 3 < H ? xrow(n0) : xzero;
        r[3] = y + 4 < H ? xrow(n1) : xzero;
      }
    }
    if (a.pool) {
      // each wave pools its own image's LDS rows: no workgroup barrier, so one wave's pool
      // (VALU / LDS) overlaps the other waves' MFMA rows. LDS ops of a wave complete in
      // order; the fences only keep the compiler from moving them across.
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int Ho = (H + 1) >> 1, Wo = W >> 1;
      if (HT == 16 && !WIDE)
        pool_img16<COUT, OSTR>(otile + (size_t)wave * HW * OSTR,
                               (size_t)(img0 + wave) * Ho * Wo * COUT, a.y, a.pool_idx, lane);
      else
        mbk::pool_tile<COUT, OSTR, 64>(otile + (size_t)wave * HW * OSTR, H, W, 1,
                                       (size_t)(img0 + wave) * Ho * Wo * COUT, a.y, a.pool_idx, lane);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();   // reads done before the next group's rows overwrite
    }
  };
  if (a.queue) {  // per-wave image queue (16-image chunks): the wave's LDS slot stays `wave`
    int cend = 0;
    for (int img = mbk::wave_next_item(a.queue, -1, cend, a.N); img < a.N;
         img = mbk::wave_next_item(a.queue, img, cend, a.N))
      one(img - wave);
    mbk::wave_queue_done(a.queue, (int)gridDim.x * (kThreads / 64));
    return;
  }
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * kRowImgs;
    if (wave < min(kRowImgs, a.N - img0)) one(img0);
  }
}

// The body is a device function over the arguments by const reference: as a kernel taking
// ConvFwdArgs by value, with the [&] lambdas above capturing it, the same code ran 2.27-2.31 ms
// per 524K 16x16 images against 1.77 ms (bit-identical, 184 VGPRs either way; profile 43).
template <int HT, int COUT, bool WIDE = false>
__global__ __launch_bounds__(kThreads) void conv0_row_kernel(ConvFwdArgs a) {
  conv0_row_body<HT, COUT, WIDE>(a);
}
// the 16x16 / 16-channel form (the learner's stage 0) at 3 waves per SIMD: 168 VGPRs with a
// 20-byte spill, 1.62 vs 1.77 ms at 2 waves; its 52 KB of LDS fits 3 workgroups per CU
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(3))) void conv0_row16_kernel(
    ConvFwdArgs a) {
  conv0_row_body<16, 16, false>(a);
}

// ------------------------------------------------------------------ weight gradient
struct ConvWgradArgs {
  const void* x;
  const bf16* dy;
  float* partial;  // [gridDim.x][COUT*9*CIN + COUT]
  int N, H, W, imgs, relu_in;
  // UNPOOL: dY is the max-pool backward of dp through the stored argmax bytes pidx
  const bf16* dp;       // [N][Ho][Wo][COUT]
  const uint8_t* pidx;  // [N][Ho][Wo][COUT]
  // work queue of rounds (common.h; thread 0 takes 16-round chunks, the next rounds reach the
  // workgroup through an LDS ring behind the LUT): a late-starting workgroup takes fewer
  // rounds. Its partial row still sums its own rounds in its order, so the weight gradient is
  // deterministic up to fp32 summation order only (null: static stride, bit-reproducible)
  int* queue = nullptr;
};

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}

constexpr int kPFW = 4;  // wgrad prefetch slots per thread for X and for dY
#ifndef MBK_WGRAD_TSH
#define MBK_WGRAD_TSH 1  // build knob (tools/variant.py): 0 = the tap shift on X (A/B only)
#endif

// Band layout of the weight-gradient tiles (WT > 0: compile-time map width 8 or 16, H % 4
// == 0). A tr read gives lanes 0-31 32 bytes of 4 consecutive pixels each for the lane
// groups G = 0 and 1. In the plain layout (WT = 0) the two groups read pixels 8 apart in
// one row, which sit on the same banks (2 LDS cycles per half-wave: the 41.7 % conflict
// rate of profile 22). Here the 32 pixels of a K block are 4 rows x 8 columns and group G
// takes row G, so G = 1 reads one row below G = 0; rows are padded so that one row down is
// the other half of the 256-byte bank window: every tr read is conflict-free
// (tools/lds_banks.py --wgrad) and every tap / channel-block offset is an immediate.
template <int XPB, int WT>
constexpr int wg_rbx() {  // X tile row bytes (halo'd row + pad)
  return (WT + 2) * XPB + (XPB == 64 ? 32 : 64);
}
template <int DPB, int WT>
constexpr int wg_rbd() {  // dY tile row bytes
  return WT * DPB + (DPB == 64 ? 32 : 128);
}
inline size_t wg_tile_bytes(int cin, int cout, int imgs, int H, int W, int wt) {
  if (wt == 0)
    return ((((size_t)imgs * (H + 2) * (W + 2) * cin * 2) + 15) & ~(size_t)15) + 64 +
           ((((size_t)imgs * H * W * cout * 2) + 15) & ~(size_t)15) + 64;
  const int rbx = (wt + 2) * cin * 2 + (cin == 32 ? 32 : 64);
  const int rbd = wt * cout * 2 + (cout == 32 ? 32 : 128);
  // (cin > cout: the tap-shifted dY tile carries a zero halo, see conv_wgrad_kernel TSH)
  return (size_t)imgs * (H + 2) * rbx + 64 + (size_t)imgs * (H + (cin > cout ? 2 : 0)) * rbd + 64;
}
// the band-layout instantiation for this shape (0: the plain layout); 24 (config 4's 24x24
// stage 0): three 8-column chunks per band, and 24 x XPB / DPB keep the 8 / 16-wide rows'
// residues mod 256 bytes, so the tr reads stay conflict-free
inline int wg_band_w(int H, int W) {
  return (W == 16 || W == 8 || W == 24) && H % 4 == 0 ? W : 0;
}

// Persistent over image rounds (grid = occupancy-sized, one partial per workgroup).
// Both GEMM operands come from NHWC LDS tiles through ds_read_b64_tr_b16 (band layout
// above when WT > 0); the next round's X interior and dY are prefetched into registers
// during the MFMAs.
// UNPOOL (the stage-0 layer of a 16-wide map: its dY is the pool backward of the next
// layer's input gradient): each round stages the pooled gradient and argmax bytes (3 of the
// 8 KB per image a materialised dY costs) and scatters them into the zeroed band-layout dY
// tile (one wave per image, four window-parity phases), so the full-resolution dY never
// touches HBM and no pool_bwd_idx launch runs.
template <int CIN, int COUT, bool BITS, int WT = 0, bool UNPOOL = false>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(ConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int XPB = CIN * 2;       // X tile pixel stride (bytes), NHWC bf16
  constexpr int DPB = COUT * 2;      // dY tile pixel stride
  constexpr int MB = COUT / 16;
  constexpr int CB = CIN / 16;
  constexpr int NBLK = 9 * CB;
  constexpr int KTOT = 9 * CIN;
  constexpr int XEPP = BITS ? 1 : CIN / 8;  // X staging elements per pixel (u32 / uint4)
  constexpr int DCH = COUT / 8;             // dY uint4 per pixel
  constexpr bool band = WT > 0;
  constexpr int RBX = wg_rbx<XPB, WT>(), RBD = wg_rbd<DPB, WT>();
  // TSH (band layout, CIN > COUT: the stage-0 layer, 32 bit planes -> 16 channels): the tap
  // shift moves from X to dY. dW[t] = sum_p dY[p] X[p + off_t] = sum_q dY[q - off_t] X[q], so a
  // K block reads its CB X fragments once and one shifted dY fragment per tap: 2 + 18 tr reads
  // per 19 MFMAs instead of 2 + 36 (the LDS array, not the MFMA, bounded the kernel). The dY
  // tile then carries a zero halo ((H + 2) rows, pixel x at column x + 1: the 128-byte row pad
  // already holds the two halo pixels, so the row stride and its bank residue are unchanged).
  constexpr bool TSH = MBK_WGRAD_TSH && band && CIN > COUT;
  static_assert(!TSH || (WT + 2) * DPB <= RBD, "dY halo fits the padded row");
  const int H = a.H, W = band ? WT : a.W, HW = H * W, Hp = H + 2, Wp = W + 2;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  // wave index in an SGPR: the K-block loop's (image, band, chunk) split of the wave-uniform
  // block index then runs on the scalar unit instead of as VALU divisions
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = (lane >> 4), li = lane & 15;
  const int IMGX = Hp * RBX, IMGD = (TSH ? Hp : H) * RBD;  // band layout image strides
  constexpr int DIN = TSH ? RBD + DPB : 0;  // dY tile offset of interior pixel (0, 0)
  // LDS carve: [X tile | zero row (64B) | dY tile | zero row]; reused for the final reduce
  const int xbytes = band ? a.imgs * IMGX : ((a.imgs * Hp * Wp * XPB) + 15) & ~15;
  char* xt = smem;
  char* xzero = smem + xbytes;
  char* dt = xzero + 64;
  const int dbytes = band ? a.imgs * IMGD : ((a.imgs * HW * DPB) + 15) & ~15;
  char* dzero = dt + dbytes;
  float* red = (float*)smem;  // [COUT][KTOT] after the loop
  // bit-plane staging: byte -> 8 bf16 lookup table (4 KB) after the tiles
  uint4* lut = (uint4*)(dzero + 64);

  // (TSH: the dY tile too, once: its halo is never written)
  for (int e = tid; e < (xbytes + 64 + (TSH ? dbytes : 0)) / 16; e += kThreads)
    ((uint4*)xt)[e] = make_uint4(0, 0, 0, 0);
  for (int e = tid; e < 4; e += kThreads) ((uint4*)dzero)[e] = make_uint4(0, 0, 0, 0);
  if constexpr (BITS)
    for (int e = tid; e < 256; e += kThreads) lut[e] = expand_bits8((uint32_t)e);
  const int xper = a.imgs * HW * XEPP, dper = a.imgs * HW * DCH;
  // UNPOOL scatter lanes (wave w = channels 4w .. 4w + 3, see the round): lane = (image of
  // the round, window k of a parity phase, channel pair)
  constexpr int WO2 = WT / 2;
  const int s_im = lane >> 5, s_k = (lane >> 1) & 15, s_c0 = 4 * wave + 2 * (lane & 1);
  int xoff[kPFW];
#pragma unroll
  for (int k = 0; k < kPFW; ++k) {
    const int e = tid + k * kThreads;
    int o = 0;
    if (e < xper) {
      const int q = e % XEPP, p = e / XEPP;
      const int im = p / HW, r = p - im * HW, y = r / W, x = r - y * W;
      o = band ? im * IMGX + (y + 1) * RBX + (x + 1) * XPB + q * 16
               : ((im * Hp + y + 1) * Wp + x + 1) * XPB + q * 16;
    }
    xoff[k] = o;
  }
  f32x4 acc[MB][NBLK];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias grad = dY^T . ones: one more MFMA per K block against a constant all-ones fragment
  // (every column of accb holds the channel sums) instead of VALU adds in the staging
  f32x4 accb[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) accb[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);

  // two register prefetch buffers: round rd + 2 * grid loads while round rd computes, so
  // twice the bytes are in flight (the tile loads are HBM-latency bound at one round ahead)
  struct PF {
    uint4 px[kPFW], pd[kPFW];
    uint32_t sd[UNPOOL ? 4 : 1], si[UNPOOL ? 4 : 1];  // UNPOOL: the lane's 4 phases' dp / argmax
    uint32_t pb[kPFW];
  };
  PF pf0, pf1;
  auto prefetch = [&](int rd, PF& f) {
    uint4 (&px)[kPFW] = f.px; uint4 (&pd)[kPFW] = f.pd;
    uint32_t (&pb)[kPFW] = f.pb;
    const int nimg = min(a.imgs, a.N - rd * a.imgs);
    const int xl = nimg * HW * XEPP, dl = nimg * HW * DCH;
    const size_t xb = (size_t)rd * xper, db = (size_t)rd * dper;
#pragma unroll
    for (int k = 0; k < kPFW; ++k) {
      const int e = tid + k * kThreads;
      if (BITS) pb[k] = e < xl ? ((const uint32_t*)a.x)[xb + e] : 0u;
      else px[k] = e < xl ? ((const uint4*)a.x)[xb + e] : make_uint4(0, 0, 0, 0);
      if constexpr (!UNPOOL) pd[k] = e < dl ? ((const uint4*)a.dy)[db + e] : make_uint4(0, 0, 0, 0);
    }
    if constexpr (UNPOOL) {
      const bool ok = s_im < nimg;
      const size_t img = (size_t)rd * a.imgs + (ok ? s_im : 0);
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int oy = 2 * (s_k >> 2) + (ph >> 1), ox = 2 * (s_k & 3) + (ph & 1);
        const size_t o = (img * WO2 * WO2 + oy * WO2 + ox) * COUT + s_c0;
        f.sd[ph] = ok ? *(const uint32_t*)(a.dp + o) : 0u;
        f.si[ph] = ok ? *(const uint16_t*)(a.pidx + o) : 0u;
      }
    }
  };
  auto put_x = [&](int off, uint4 v) {
    if (a.relu_in) {
      v.x = relu_bf16x2(v.x); v.y = relu_bf16x2(v.y);
      v.z = relu_bf16x2(v.z); v.w = relu_bf16x2(v.w);
    }
    *(uint4*)(xt + off) = v;
  };
  auto put_bits = [&](int off, uint32_t bits) {  // one pixel's 32 planes -> 4 x uint4
    // lanes (consecutive pixels, 64 B apart) rotate their chunk order so that each 8-lane
    // store group covers 8 distinct 16-byte slots of the 128-byte store bank window
    const int rot = band ? (lane >> 1) & 3 : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = (i + rot) & 3;
      *(uint4*)(xt + off + q * 16) = lut[(bits >> (8 * q)) & 255u];
    }
  };
  auto doff_of = [&](int e) {  // dY tile byte offset of staging chunk e
    if constexpr (!band) return e * 16;
    const int q = e % DCH, p = e / DCH;
    const int im = p / HW, r = p - im * HW, y = r / W, x = r - y * W;
    return im * IMGD + DIN + y * RBD + x * DPB + q * 16;
  };
  auto put_d = [&](int e, uint4 v) { *(uint4*)(dt + doff_of(e)) = v; };
  auto xoff_of = [&](int e) {
    const int q = e % XEPP, p = e / XEPP;
    const int im = p / HW, r = p - im * HW, y = r / W, x = r - y * W;
    if constexpr (band) return im * IMGX + (y + 1) * RBX + (x + 1) * XPB + q * 16;
    return ((im * Hp + y + 1) * Wp + x + 1) * XPB + q * 16;
  };

  const int nrounds = (a.N + a.imgs - 1) / a.imgs;
  const int gstep = gridDim.x;
  int* const wq = a.queue;
  int* const ring = (int*)(dzero + 64 + 4096);  // rounds k .. k + 3 (queue mode)
  int t_last = -1, t_cend = 0;                  // thread 0's queue cursor
  auto gen = [&]() {  // thread 0: the workgroup's next round (>= nrounds: none left)
    if (t_last >= nrounds) return t_last;
    if (t_last + 1 < t_cend) return ++t_last;
    const int t = __hip_atomic_fetch_add(wq, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) *
                  mbk::kQueueChunk;
    t_cend = min(nrounds, t + mbk::kQueueChunk);
    return t_last = t;
  };
  if (wq) {
    if (tid == 0) {
      ring[0] = gen();
      ring[1] = gen();
      ring[2] = gen();
    }
    __syncthreads();
    if (ring[0] < nrounds) prefetch(ring[0], pf0);
    if (ring[1] < nrounds) prefetch(ring[1], pf1);
  } else {
    if ((int)blockIdx.x < nrounds) prefetch(blockIdx.x, pf0);
    if ((int)blockIdx.x + gstep < nrounds) prefetch(blockIdx.x + gstep, pf1);
  }
  __syncthreads();  // zero halo / zero rows visible
  // rd2: the round this one prefetches for (two rounds ahead in this workgroup's sequence),
  // read after the round's first barrier (queue mode: from the ring)
  auto round = [&](int rd, PF& f, int k) {
    uint4 (&px)[kPFW] = f.px; uint4 (&pd)[kPFW] = f.pd;
    uint32_t (&pb)[kPFW] = f.pb;
    const int nimg = min(a.imgs, a.N - rd * a.imgs);
    const int xl = nimg * HW * XEPP, dl = nimg * HW * DCH;
#pragma unroll
    for (int k = 0; k < kPFW; ++k) {
      const int e = tid + k * kThreads;
      if (e < xl) {
        if (BITS) put_bits(xoff[k], pb[k]);
        else put_x(xoff[k], px[k]);
      }
      if constexpr (!UNPOOL)
        if (e < dl) put_d(e, pd[k]);
    }
    for (int e = tid + kPFW * kThreads; e < xl; e += kThreads) {
      if (BITS) put_bits(xoff_of(e), ((const uint32_t*)a.x)[(size_t)rd * xper + e]);
      else put_x(xoff_of(e), ((const uint4*)a.x)[(size_t)rd * xper + e]);
    }
    if constexpr (UNPOOL) {
      // scatter, wave w taking channels 4w .. 4w + 3 of every image of the round from its
      // lanes' prefetched registers: no two waves touch one element and a wave's LDS ops
      // complete in issue order, so neither the zeroing of its channel slice nor the 4 phases
      // need a barrier. Phase ph = the 16 windows of parity (oy % 2, ox % 2) = (ph / 2, ph % 2),
      // which never overlap; each element gets dY[pixel][c] += dp (bf16 storage, fp32 add: a
      // pixel 2 windows chose sees one extra bf16 rounding against pool_bwd_idx's fp32 sum)
      static_assert(!UNPOOL || (band && WT == 16 && COUT == 16 && kThreads == 256),
                    "16-wide stage-0 layout, 4 waves x 4 channels");
      {  // this wave's 8 bytes of every pixel: lane = (row y % 4, column), rows 4 apart (one
         // pointer add per store instead of the pixel -> (image, row, column) split per store)
        char* zp = dt + DIN + (lane >> 4) * RBD + (lane & 15) * DPB + 8 * wave;
        for (int im = 0; im < nimg; ++im, zp += IMGD - H * RBD)
          for (int y4 = 0; y4 < H; y4 += 4, zp += 4 * RBD) *(uint2*)zp = make_uint2(0, 0);
      }
      asm volatile("" ::: "memory");
      if (s_im < nimg) {
        char* dimg = dt + s_im * IMGD + DIN;
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
          const int oy = 2 * (s_k >> 2) + (ph >> 1), ox = 2 * (s_k & 3) + (ph & 1);
          const uint32_t d2 = f.sd[ph], i2 = f.si[ph];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int t = (int)((i2 >> (8 * j)) & 0xFFu);
            const int ky = (t * 11) >> 5, kx = t - 3 * ky;  // t / 3 for t < 9
            const int py = 2 * oy - 1 + ky, px = 2 * ox - 1 + kx;
            uint16_t* el = (uint16_t*)(dimg + py * RBD + px * DPB + (s_c0 + j) * 2);
            const float add = __uint_as_float(j ? (d2 & 0xFFFF0000u) : (d2 << 16));
            const float v = __uint_as_float((uint32_t)*el << 16) + add;
            *el = __bfloat16_as_ushort(f2bf(v));
          }
          asm volatile("" ::: "memory");
        }
      }
    } else {
      for (int e = tid + kPFW * kThreads; e < dl; e += kThreads)
        put_d(e, ((const uint4*)a.dy)[(size_t)rd * dper + e]);
    }
    __syncthreads();
    const int rd2 = wq ? ring[(k + 2) & 3] : rd + 2 * gstep;
    if (rd2 < nrounds) prefetch(rd2, f);

    if constexpr (band) {
      // K block kb = (image, 4-row band, 8-column chunk); lane group G takes row G of the
      // band, h the column half, li >> 2 the column: every pixel of the block is real
      constexpr int CPR = WT / 8;
      const int bpi = (H >> 2) * CPR;
      const int nk = nimg * bpi;
      for (int kb = wave; kb < nk; kb += kThreads / 64) {
        const int im = kb / bpi, rem = kb - im * bpi;
        const int y = (rem / CPR) * 4 + G, x0 = (rem % CPR) * 8 + (li >> 2);
        const char* db = dt + im * IMGD + y * RBD + x0 * DPB + 8 * (li & 3);
        const char* xb = xt + im * IMGX + y * RBX + x0 * XPB + 8 * (li & 3);
        if constexpr (TSH) {
          // K = the block's 32 X pixels q (B: the centre tap of the halo'd X tile); tap t's A
          // is dY at q - off_t = halo'd dY (y + 2 - t / 3, x + 2 - t % 3); the centre one
          // (t = 4, the unshifted dY) also feeds the bias MFMA
          Frag8 bx[CB];
#pragma unroll
          for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int h = 0; h < 2; ++h) bx[cb].h[h] = tr_read(xb + RBX + (1 + 4 * h) * XPB + cb * 32);
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            Frag8 at[MB];
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                at[mb].h[h] = tr_read(db + (2 - t / 3) * RBD + (2 - t % 3 + 4 * h) * DPB + mb * 32);
            if (t == 4)
#pragma unroll
              for (int mb = 0; mb < MB; ++mb)
                accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[mb].v, ones.v, accb[mb], 0, 0, 0);
#pragma unroll
            for (int cb = 0; cb < CB; ++cb)
#pragma unroll
              for (int mb = 0; mb < MB; ++mb)
                acc[mb][t * CB + cb] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[mb].v, bx[cb].v, acc[mb][t * CB + cb], 0, 0, 0);
          }
          continue;
        }
        Frag8 af[MB];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int h = 0; h < 2; ++h) af[mb].h[h] = tr_read(db + h * 4 * DPB + mb * 32);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, ones.v, accb[mb], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            Frag8 bf;
#pragma unroll
            for (int h = 0; h < 2; ++h)
              bf.h[h] = tr_read(xb + (t / 3) * RBX + (t % 3 + 4 * h) * XPB + cb * 32);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              acc[mb][t * CB + cb] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bf.v, acc[mb][t * CB + cb], 0, 0, 0);
          }
        }
      }
    } else {
      const int M = nimg * HW;
      const int nk = (M + 31) >> 5;
      for (int kb = wave; kb < nk; kb += kThreads / 64) {
        // this lane's two pixels (rows q = li>>2 of halves h = 0, 1)
        const char* dptr[2];
        int xpos[2];
        bool ok[2];
  #pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int p = kb * 32 + 8 * G + 4 * h + (li >> 2);
          ok[h] = p < M;
          const int pp = ok[h] ? p : 0;
          // float-reciprocal index math (exact here, see conv_fwd_kernel)
          const int im = (int)(((float)pp + 0.5f) * inv_hw), r = pp - im * HW;
          const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
          xpos[h] = (im * Hp + y) * Wp + x;
          dptr[h] = ok[h] ? dt + pp * DPB : dzero;
        }
        Frag8 af[MB];
  #pragma unroll
        for (int mb = 0; mb < MB; ++mb)
  #pragma unroll
          for (int h = 0; h < 2; ++h)
            af[mb].h[h] = tr_read(dptr[h] + (mb * 16 + 4 * (li & 3)) * 2);
  #pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, ones.v, accb[mb], 0, 0, 0);
        // X taps: out-of-range pixels read pixel 0's (finite) values; their dY column (the A
        // operand, dzero) is zero, so they add exactly nothing and need no per-tap zero select
        const char* xb0 = xt + xpos[0] * XPB + 8 * (li & 3);
        const char* xb1 = xt + xpos[1] * XPB + 8 * (li & 3);
  #pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int off = ((t / 3) * Wp + (t % 3)) * XPB;
  #pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            Frag8 bf;
            bf.h[0] = tr_read(xb0 + off + cb * 32);
            bf.h[1] = tr_read(xb1 + off + cb * 32);
  #pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              acc[mb][t * CB + cb] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bf.v, acc[mb][t * CB + cb], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // tile reads done before the next round is staged
  };
  if (wq) {
    // round k: thread 0 queues round k + 3 into the ring before the round's first barrier;
    // slot k & 3 was written three rounds (>= 2 barriers) earlier
    for (int k = 0;; k += 2) {
      if (tid == 0) ring[(k + 3) & 3] = gen();
      const int r0 = ring[k & 3];
      if (r0 >= nrounds) break;
      round(r0, pf0, k);
      if (tid == 0) ring[(k + 4) & 3] = gen();
      const int r1 = ring[(k + 1) & 3];
      if (r1 >= nrounds) break;
      round(r1, pf1, k + 1);
    }
    if (tid == 0 && __hip_atomic_fetch_add(wq + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        (int)gridDim.x - 1) {
      __hip_atomic_store(wq, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(wq + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {
    for (int rd = blockIdx.x; rd < nrounds; rd += 2 * gstep) {
      round(rd, pf0, 0);
      if (rd + gstep < nrounds) round(rd + gstep, pf1, 0);
    }
  }
  // ---- reduce the 4 waves through LDS (sequential adds, no atomics)
  for (int w = 0; w < kThreads / 64; ++w) {
    if (wave == w) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NBLK; ++nb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            // C layout: row (co) = 4G + i, col (n) = li
            const int co = mb * 16 + 4 * G + i, n = nb * 16 + li;
            float* p = red + co * KTOT + n;
            *p = (w == 0 ? 0.f : *p) + acc[mb][nb][i];
          }
    }
    __syncthreads();
  }
  float* out = a.partial + (size_t)blockIdx.x * (COUT * KTOT + COUT);
  for (int e = tid; e < COUT * KTOT / 4; e += kThreads) ((float4*)out)[e] = ((const float4*)red)[e];
  // bias grad: column 0 of each wave's accb (C layout: lane li = 0 holds rows 4G + i)
  __syncthreads();
  float* bred = red;  // reuse: [4 waves][COUT]
  if (li == 0) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int i = 0; i < 4; ++i) bred[wave * COUT + mb * 16 + 4 * G + i] = accb[mb][i];
  }
  __syncthreads();
  if (tid < COUT) {
    float s = 0.f;
    for (int w = 0; w < kThreads / 64; ++w) s += bred[w * COUT + tid];
    out[COUT * KTOT + tid] = s;
  }
}

// partial[nparts][COUT*9*CIN + COUT] -> dw[co][ci][ky][kx] (+)=, db[co] (+)=
// block = 64 output columns x 4 part-lanes over parts [y*pps, (y+1)*pps); with `stage`
// set the split sums go to stage[y][row] for a second pass (two-level: the persistent
// wgrad writes up to a few thousand partial rows). Fixed summation order (deterministic).
// One 64-column slice of a partial-row reduction: sums rows [split*pps, min(nparts, ..+pps))
// of ``partial`` (4 row lanes x 64 columns, then the 4 lane sums in order) and writes the
// split's row of ``stage`` or, with stage == nullptr, the fp32 weight / bias gradient.
__device__ __forceinline__ void wgrad_reduce_cols(const float* __restrict__ partial, int nparts,
                                                  int pps, int split, int colblk,
                                                  float* __restrict__ stage, int cin,
                                                  int cin_real, int cout, float* __restrict__ dw,
                                                  float* __restrict__ db, int accumulate,
                                                  float (*red)[64]) {
  const int ktot = 9 * cin, row = cout * ktot + cout;
  const int col = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int e = colblk * 64 + col;
  const int p0 = split * pps, p1 = min(nparts, p0 + pps);
  float s = 0.f;
  if (e < row) {
#pragma unroll 4
    for (int p = p0 + pl; p < p1; p += 4) s += partial[(size_t)p * row + e];
  }
  red[pl][col] = s;
  __syncthreads();
  if (pl != 0 || e >= row) return;
  s = red[0][col] + red[1][col] + red[2][col] + red[3][col];
  if (stage) {
    stage[(size_t)split * row + e] = s;
    return;
  }
  if (e < cout * ktot) {
    const int co = e / ktot, r = e - co * ktot, t = r / cin, ci = r - t * cin;
    if (ci >= cin_real) return;
    float* d = dw + ((size_t)co * cin_real + ci) * 9 + t;
    *d = accumulate ? *d + s : s;
  } else if (db) {
    const int co = e - cout * ktot;
    db[co] = accumulate ? db[co] + s : s;
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ partial,
                                                           int nparts, int pps,
                                                           float* __restrict__ stage, int cin,
                                                           int cin_real, int cout,
                                                           float* __restrict__ dw,
                                                           float* __restrict__ db, int accumulate) {
  __shared__ float red[4][64];
  wgrad_reduce_cols(partial, nparts, pps, blockIdx.y, blockIdx.x, stage, cin, cin_real, cout, dw,
                    db, accumulate, red);
}

// Many layers' reductions in one launch (blockIdx.z = job; the encoder defers every weight
// gradient reduce of a backward pass to one mbk_wgrad_reduce_batch call). Level 0 runs a
// job's split sums (two-level jobs) or its whole sum; level 1 the two-level jobs' second
// stage: per element the same adds in the same order as mbk_wgrad_reduce -> bit-identical.
struct MbkReduceJob {
  const float* partial;
  float* dw;
  float* db;
  int nparts, cin, cin_real, cout, accumulate;
};
constexpr int kReducePps = 32;
constexpr int kMaxReduceJobs = 32;
struct ReduceBatch {
  MbkReduceJob j[kMaxReduceJobs];
};

__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(ReduceBatch b, int level) {
  __shared__ float red[4][64];
  const MbkReduceJob J = b.j[blockIdx.z];
  const int row = J.cout * 9 * J.cin + J.cout;
  if ((int)blockIdx.x * 64 >= row) return;  // whole workgroup: before any barrier
  const bool two = J.nparts > 2 * kReducePps;
  const int splits = two ? (J.nparts + kReducePps - 1) / kReducePps : 1;
  float* stage = two ? (float*)J.partial + (size_t)J.nparts * row : nullptr;
  if (level == 0) {
    if ((int)blockIdx.y >= splits) return;
    wgrad_reduce_cols(J.partial, J.nparts, two ? kReducePps : J.nparts, blockIdx.y, blockIdx.x,
                      stage, J.cin, J.cin_real, J.cout, J.dw, J.db, J.accumulate, red);
  } else {
    if (!two || blockIdx.y != 0) return;
    wgrad_reduce_cols(stage, splits, splits, 0, blockIdx.x, nullptr, J.cin, J.cin_real, J.cout,
                      J.dw, J.db, J.accumulate, red);
  }
}

// ------------------------------------------------------------------ maxpool backward
// dc[n][y][x][c] = sum of dp over the (<= 4) windows whose first-in-scan-order
// argmax is (y, x) — matches ATen's max_pool2d index semantics.
__global__ __launch_bounds__(256) void pool_bwd_kernel(const bf16* __restrict__ cfull,
                                                       const bf16* __restrict__ dp, int N, int H,
                                                       int W, int C, bf16* __restrict__ dc) {
  const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
  const size_t tot = (size_t)N * H * W * C;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (size_t)gridDim.x * blockDim.x) {
    const int c = e % C;
    const size_t p = e / C;
    const int x = p % W, y = (p / W) % H;
    const size_t n = p / ((size_t)H * W);
    float g = 0.f;
    // windows (oy, ox) with 2*oy-1 <= y <= 2*oy+1
    const int oy_lo = y / 2, oy_hi = min(Ho - 1, (y + 1) / 2);
    const int ox_lo = x / 2, ox_hi = min(Wo - 1, (x + 1) / 2);
    for (int oy = max(0, oy_lo - 1); oy <= oy_hi; ++oy) {
      if (y < 2 * oy - 1 || y > 2 * oy + 1) continue;
      for (int ox = max(0, ox_lo - 1); ox <= ox_hi; ++ox) {
        if (x < 2 * ox - 1 || x > 2 * ox + 1) continue;
        float mx = -INFINITY;
        int ay = -1, ax = -1;
        for (int ky = 0; ky < 3; ++ky) {
          const int yy = 2 * oy - 1 + ky;
          if (yy < 0 || yy >= H) continue;
          for (int kx = 0; kx < 3; ++kx) {
            const int xx = 2 * ox - 1 + kx;
            if (xx < 0 || xx >= W) continue;
            const float v = bf2f(cfull[((n * H + yy) * W + xx) * C + c]);
            if (v > mx || ay < 0) { mx = v; ay = yy; ax = xx; }
          }
        }
        if (ay == y && ax == x) g += bf2f(dp[((n * Ho + oy) * Wo + ox) * C + c]);
      }
    }
    dc[e] = f2bf(g);
  }
}

// dc[n][y][x][c..c+7] = sum of dp over the (<= 4) windows whose stored argmax is (y, x).
// One thread per (image, 2x2 input block, 8 channels): the block's pixels are fed only by
// windows (oy, ox) in {j, j+1} x {k, k+1}, so four 24-byte window loads cover four
// pixels and the tap each window must match is a compile-time constant. 32-bit index
// math (the host splits launches that would overflow it).
template <int C>
__global__ __launch_bounds__(256) void pool_bwd_idx_kernel(const uint8_t* __restrict__ pidx,
                                                           const bf16* __restrict__ dp, int N,
                                                           int H, int W,
                                                           bf16* __restrict__ dc) {
  constexpr int C8 = C / 8;
  const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
  const uint32_t tot = (uint32_t)N * Ho * Wo * C8;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
    const int c8 = e % C8;
    uint32_t q = e / C8;
    const int k = q % Wo;
    q /= Wo;
    const int j = q % Ho;
    const uint32_t n = q / Ho;
    uint32_t ids[2][2][2];
    uint32_t dv[2][2][4];
#pragma unroll
    for (int dj = 0; dj < 2; ++dj)
#pragma unroll
      for (int dk = 0; dk < 2; ++dk) {
        const int oy = j + dj, ox = k + dk;
        if (oy < Ho && ox < Wo) {
          const uint32_t o = ((n * Ho + oy) * Wo + ox) * C + c8 * 8;
          const uint2 iv = *(const uint2*)(pidx + o);
          const uint4 d = *(const uint4*)(dp + o);
          ids[dj][dk][0] = iv.x; ids[dj][dk][1] = iv.y;
          dv[dj][dk][0] = d.x; dv[dj][dk][1] = d.y; dv[dj][dk][2] = d.z; dv[dj][dk][3] = d.w;
        } else {  // tap id 0xFF never matches
          ids[dj][dk][0] = ids[dj][dk][1] = 0xFFFFFFFFu;
          dv[dj][dk][0] = dv[dj][dk][1] = dv[dj][dk][2] = dv[dj][dk][3] = 0u;
        }
      }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int y = 2 * j + a, x = 2 * k + b;
        if (y >= H || x >= W) continue;
        float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        // window (j+dj, k+dk) sees this pixel at tap (a+1-2dj, b+1-2dk) when in [0, 2]
#pragma unroll
        for (int dj = 0; dj < 2; ++dj)
#pragma unroll
          for (int dk = 0; dk < 2; ++dk) {
            const int ky = a + 1 - 2 * dj, kx = b + 1 - 2 * dk;
            if (ky < 0 || kx < 0) continue;
            const uint32_t me = (uint32_t)(ky * 3 + kx);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const uint32_t id = (ids[dj][dk][t >> 2] >> (8 * (t & 3))) & 0xFFu;
              const uint32_t hb = (dv[dj][dk][t >> 1] >> (16 * (t & 1))) & 0xFFFFu;
              if (id == me) g[t] += __uint_as_float(hb << 16);
            }
          }
        uint32_t o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t lo = __bfloat16_as_ushort(f2bf(g[2 * t]));
          const uint32_t hi = __bfloat16_as_ushort(f2bf(g[2 * t + 1]));
          o[t] = lo | (hi << 16);
        }
        *(uint4*)(dc + ((size_t)(n * H + y) * W + x) * C + c8 * 8) =
            make_uint4(o[0], o[1], o[2], o[3]);
      }
  }
}

// ------------------------------------------------------------------ weight packing
struct PackJob {
  const float* w;   // [cout][cin_real][3][3]
  bf16* fwd;        // [cout][nch(cin)][32]
  bf16* bwd;        // dgrad weights: conv with cin'=cout, cout'=cin -> [cin][nch(cout)][32]
  int cin, cin_real, cout;
};
struct PackJobs {
  PackJob j[16];
  int n;
};

__device__ __forceinline__ int nch_of(int c) { return c == 16 ? 5 : 9; }

__global__ __launch_bounds__(256) void conv_pack_kernel(PackJobs jobs) {
  const PackJob& J = jobs.j[blockIdx.y];
  if (blockIdx.y >= jobs.n) return;
  const int nf = J.cout * nch_of(J.cin) * 32;
  const int nb = J.bwd ? J.cin * nch_of(J.cout) * 32 : 0;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nf + nb; e += gridDim.x * blockDim.x) {
    if (e < nf) {
      const int co = e / (nch_of(J.cin) * 32), r = e % (nch_of(J.cin) * 32);
      const int c = r / 32, k = r % 32;
      int tap, ci;
      if (J.cin == 16) { tap = 2 * c + k / 16; ci = k % 16; }
      else { tap = c; ci = k; }
      float v = 0.f;
      if (tap < 9 && ci < J.cin_real) v = J.w[((size_t)co * J.cin_real + ci) * 9 + tap];
      J.fwd[e] = f2bf(v);
    } else {
      // dgrad: out channel = original ci, input channel = original co, tap flipped
      const int f = e - nf;
      const int ci = f / (nch_of(J.cout) * 32), r = f % (nch_of(J.cout) * 32);
      const int c = r / 32, k = r % 32;
      int tap, co;
      if (J.cout == 16) { tap = 2 * c + k / 16; co = k % 16; }
      else { tap = c; co = k; }
      float v = 0.f;
      if (tap < 9 && ci < J.cin_real) v = J.w[((size_t)co * J.cin_real + ci) * 9 + (8 - tap)];
      J.bwd[f] = f2bf(v);
    }
  }
}

// fp32 [cout][cin_real][3][3] -> e4m3 [cout][nch][32] (fwd layout) with a power-of-two
// per-output-channel scale 2^k (amax * 2^k <= 224, exact dequant), one block per (co, job)
struct PackJob8 {
  const float* w;
  uint8_t* q;
  float* scale;  // [cout] dequant multipliers 2^-k
  int cin, cin_real, cout;
};
struct PackJobs8 {
  PackJob8 j[16];
  int n;
};

__global__ __launch_bounds__(256) void conv_pack_fp8_kernel(PackJobs8 jobs) {
  if ((int)blockIdx.y >= jobs.n) return;
  const PackJob8& J = jobs.j[blockIdx.y];
  const int co = blockIdx.x;
  if (co >= J.cout) return;
  __shared__ float red[256];
  const int nk = J.cin_real * 9;
  const float* wr = J.w + (size_t)co * nk;
  float m = 0.f;
  for (int e = threadIdx.x; e < nk; e += blockDim.x) m = fmaxf(m, fabsf(wr[e]));
  red[threadIdx.x] = m;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  const float amax = red[0];
  int k = 0;
  if (amax > 0.f) {
    k = (int)floorf(log2f(224.f / amax));
    k = max(-30, min(30, k));
  }
  const float sc = ldexpf(1.f, k);
  const int nch = J.cin == 16 ? 5 : 9;
  for (int e = threadIdx.x; e < nch * 32; e += blockDim.x) {
    const int c = e / 32, kk = e % 32;
    int tap, ci;
    if (J.cin == 16) { tap = 2 * c + kk / 16; ci = kk % 16; }
    else { tap = c; ci = kk; }
    float v = 0.f;
    if (tap < 9 && ci < J.cin_real) v = wr[ci * 9 + tap] * sc;
    v = fminf(fmaxf(v, -448.f), 448.f);
    const int b = __builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false);
    J.q[(size_t)co * nch * 32 + e] = (uint8_t)(b & 0xFF);
  }
  if (threadIdx.x == 0) J.scale[co] = ldexpf(1.f, -k);
}

inline size_t fwd_smem(int cin, bool bits, int imgs, int H, int W, int cout, bool pool,
                       bool fp8 = false) {
  (void)bits;  // bit planes are staged expanded (cin = 32)
  const int pixb = fp8 ? cin + 8 : cin * 2 + 16;
  size_t t = (((size_t)imgs * (H + 2) * (W + 2) * pixb) + 15) & ~(size_t)15;
  if (pool) t += (size_t)imgs * H * W * (cout + 4) * 2;
  return t;
}

inline size_t wgrad_smem(int cin, int cout, int imgs, int H, int W, bool unpool = false) {
  (void)unpool;  // (the pool-fused form keeps its pooled operands in registers)
  size_t t = wg_tile_bytes(cin, cout, imgs, H, W, wg_band_w(H, W));
  t += 4096;  // bit-plane lookup table (allocated for every variant: keeps the sizing simple)
  t += 64;    // the work queue's round ring
  size_t red = (size_t)cout * 9 * cin * 4;
  return t > red ? t : red;
}

int g_grid_cap = 0;    // tests force multi-group workgroups with a small cap
int g_conv0_row = 1;   // stage-0 conv of 16-wide maps on conv0_row_kernel (0: generic kernel)

// resident workgroups the whole device holds for (kernel, dynamic LDS)
// (occ: mbk_occ_f / mbk_occ_b, the forward / backward per-CU caps of common.h)
int resident_blocks(const void* kfn, size_t sm, int (*occ)(int) = nullptr) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  if (sm > 64 * 1024) hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, kThreads, sm) != hipSuccess || per < 1)
    per = 1;
  int r = cus * (occ ? occ(per) : per);
  if (g_grid_cap > 0 && r > g_grid_cap) r = g_grid_cap;
  return r;
}

// Forward / dgrad grids: persistent, one resident set of workgroups that walks the image
// groups (2x / 4x grids that retire workgroups early for the acting step measured level or
// slower on the bench: DESIGN.md §9 rejected variants)
int fwd_grid(int ngroups, const void* kfn, size_t sm) {
  const long r = (long)resident_blocks(kfn, sm, mbk_occ_f);
  return (int)std::max(1L, std::min((long)ngroups, r));
}

// The kernels map a tile-local pixel index m in [0, imgs*H*W) to (image, y, x) with float
// reciprocals ((m + 0.5) * (1/HW)): exact while imgs*H*W < 2^22 (the product's rounding
// error stays below the 0.5/HW distance to the next integer). LDS capacity keeps today's
// shapes far below that; this check turns a future larger-tile / larger-map config into a
// launch error instead of silently wrong indices.
bool index_math_ok(int imgs, int H, int W) {
  return H > 0 && W > 0 && H * W <= 1024 && (int64_t)imgs * H * W < (int64_t(1) << 22);
}

}  // namespace

static int conv_fwd_launch(const void* x, int in_bits, int cin, int cout, const void* w,
                           const float* wscale, const float* bias, const void* add,
                           const void* mask_src, void* y, void* y_full, void* pool_idx, int N,
                           int H, int W, int imgs, int relu_in, int pool, bool fp8,
                           hipStream_t stream) {
  if (N <= 0) return 0;
  if (fp8 && !wscale) return (int)hipErrorInvalidValue;
  if (!index_math_ok(imgs, H, W)) return (int)hipErrorInvalidValue;
  ConvFwdArgs a{x, (const bf16*)w, bias, (const bf16*)add, (const bf16*)mask_src, (bf16*)y,
                (bf16*)y_full, (uint8_t*)pool_idx, N, H, W, imgs, relu_in, pool, wscale};
  const size_t sm = fwd_smem(cin, in_bits != 0, imgs, H, W, cout, pool != 0, fp8);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  const int ngroups = (N + imgs - 1) / imgs;
#define LAUNCH(CI, CO, B)                                                                   \
  do {                                                                                      \
    auto kfn = fp8 ? conv_fwd_kernel<CI, CO, B, true> : conv_fwd_kernel<CI, CO, B, false>;  \
    if (sm > 64 * 1024) hipFuncSetAttribute((const void*)kfn,                               \
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm); \
    const int grid = fwd_grid(ngroups, (const void*)kfn, sm);                               \
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(kThreads), sm, stream, a);                     \
  } while (0)
  // 17..32 pixels wide (config 4's 24 x 24), 16 channels: the WIDE row kernel
  if (in_bits && cout == 16 && W > 16 && W <= 32 && !fp8 && g_conv0_row && !add && !mask_src &&
      !relu_in && kLutBytes + (size_t)kRowImgs * H * W * 16 * 2 <= 160 * 1024) {
    const size_t sm0 = kLutBytes + (pool ? (size_t)kRowImgs * H * W * 16 * 2 : 0);
    const auto kfn = conv0_row_kernel<0, 16, true>;
    const int grid = fwd_grid((N + kRowImgs - 1) / kRowImgs, (const void*)kfn, sm0);
    // (no work queue: on config 4 it measured 5.45 vs 5.85 M frames/s -- a faster learner
    // forward there leaves the acting-bound step slower, tools/gpu_r6_c0q.sh)
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(kThreads), sm0, stream, a);
    return (int)hipGetLastError();
  }
  if (in_bits && (cout == 16 || cout == 32) && W == 16 && !fp8 && g_conv0_row && !add &&
      !mask_src && !relu_in) {
    const size_t sm0 =
        kLutBytes + (pool ? (size_t)kRowImgs * H * 16 * conv0_ostr(cout, false) * 2 : 0);
    if (sm0 > 160 * 1024) return (int)hipErrorInvalidValue;
    const bool hb = H == 16;  // 16 x 16 maps: batched row loads
    const auto kfn = cout == 16 ? (hb ? conv0_row16_kernel : conv0_row_kernel<0, 16>)
                                : (hb ? conv0_row_kernel<16, 32> : conv0_row_kernel<0, 32>);
    const int grid = fwd_grid((N + kRowImgs - 1) / kRowImgs, (const void*)kfn, sm0);
    if (hb) a.queue = mbk_work_queue(stream, kQueueConv0);
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(kThreads), sm0, stream, a);
    return (int)hipGetLastError();
  }
  if (in_bits) {
    if (cout == 16) LAUNCH(32, 16, true);
    else if (cout == 32) LAUNCH(32, 32, true);
    else return (int)hipErrorInvalidValue;
  } else if (cin == 16 && cout == 16) LAUNCH(16, 16, false);
  else if (cin == 16 && cout == 32) LAUNCH(16, 32, false);
  else if (cin == 32 && cout == 16) LAUNCH(32, 16, false);
  else if (cin == 32 && cout == 32) LAUNCH(32, 32, false);
  else return (int)hipErrorInvalidValue;
#undef LAUNCH
  return (int)hipGetLastError();
}

extern "C" int mbk_conv_fwd(const void* x, int in_bits, int cin, int cout, const void* w,
                            const float* bias, const void* add, const void* mask_src, void* y,
                            void* y_full, void* pool_idx, int N, int H, int W, int imgs,
                            int relu_in, int pool, hipStream_t stream) {
  return conv_fwd_launch(x, in_bits, cin, cout, w, nullptr, bias, add, mask_src, y, y_full,
                         pool_idx, N, H, W, imgs, relu_in, pool, false, stream);
}

// Inference conv on fp8 MFMA: w = e4m3 packed weights (mbk_conv_pack_fp8), wscale = their
// per-output-channel dequant scale; activations in / out stay bf16 NHWC.
extern "C" int mbk_conv_fwd_fp8(const void* x, int in_bits, int cin, int cout, const void* w,
                                const float* wscale, const float* bias, const void* add, void* y,
                                int N, int H, int W, int imgs, int relu_in, int pool,
                                hipStream_t stream) {
  return conv_fwd_launch(x, in_bits, cin, cout, w, wscale, bias, add, nullptr, y, nullptr,
                         nullptr, N, H, W, imgs, relu_in, pool, true, stream);
}

#define WGRAD_DISPATCH(LAUNCH)                                                              \
  if (in_bits) {                                                                            \
    if (cout == 16) LAUNCH(32, 16, true);                                                   \
    else if (cout == 32) LAUNCH(32, 32, true);                                              \
    else return -(int)hipErrorInvalidValue;                                                 \
  } else if (cin == 16 && cout == 16) LAUNCH(16, 16, false);                                \
  else if (cin == 16 && cout == 32) LAUNCH(16, 32, false);                                  \
  else if (cin == 32 && cout == 16) LAUNCH(32, 16, false);                                  \
  else if (cin == 32 && cout == 32) LAUNCH(32, 32, false);                                  \
  else return -(int)hipErrorInvalidValue;

// the wgrad instantiation of (CI, CO, B) for this map width: band layout (WT = 8 / 16 / 24)
// or the plain one; unpool: the stage-0 layer of a 16-wide map only (null otherwise)
template <int CI, int CO, bool B>
const void* wgrad_kfn(int H, int W, bool unpool = false) {
  if (unpool) {
    if constexpr (CI == 32 && CO == 16 && B)
      if (wg_band_w(H, W) == 16) return (const void*)conv_wgrad_kernel<32, 16, true, 16, true>;
    return nullptr;
  }
  switch (wg_band_w(H, W)) {
    case 24: return (const void*)conv_wgrad_kernel<CI, CO, B, 24>;
    case 16: return (const void*)conv_wgrad_kernel<CI, CO, B, 16>;
    case 8: return (const void*)conv_wgrad_kernel<CI, CO, B, 8>;
    default: return (const void*)conv_wgrad_kernel<CI, CO, B>;
  }
}

static int occ_b2(int per) {  // twice the backward cap
  const int c = mbk_occ_cap(1);
  return c > 0 && per > 2 * c ? 2 * c : per;
}
// number of partial rows mbk_conv_wgrad will write for this shape (<= nrounds)
extern "C" int mbk_conv_wgrad_parts(int in_bits, int cin, int cout, int N, int H, int W,
                                    int imgs, int unpool) {
  const size_t sm = wgrad_smem(cin, cout, imgs, H, W, unpool != 0);
  if (sm > 160 * 1024 || !index_math_ok(imgs, H, W)) return -(int)hipErrorInvalidValue;
  const int nrounds = (N + imgs - 1) / imgs;
  int res = 1;
  const void* kq = nullptr;
#define Q(CI, CO, B) kq = wgrad_kfn<CI, CO, B>(H, W, unpool != 0)
  WGRAD_DISPATCH(Q)
#undef Q
  if (!kq) return -(int)hipErrorInvalidValue;
  // the backward cap leaves room for one acting workgroup (80 KB of LDS) beside the learner's:
  // a pool-fused stage-0 form small enough for two of its workgroups beside it may take two
  res = resident_blocks(kq, sm, unpool != 0 && 2 * sm + 80 * 1024 <= 160 * 1024 ? occ_b2 : mbk_occ_b);
  return (int)std::max(1L, std::min((long)nrounds, (long)res));
}

// dy == nullptr: the stage-0 pool-fused form, dY = max_pool2d backward of dp through pidx
extern "C" int mbk_conv_wgrad(const void* x, int in_bits, int cin, int cout, const void* dy,
                              const void* dp, const void* pidx, float* partial, int nparts,
                              int N, int H, int W, int imgs, int relu_in, hipStream_t stream) {
  const bool unpool = dy == nullptr;
  if (unpool && (!dp || !pidx || imgs > 2)) return (int)hipErrorInvalidValue;
  ConvWgradArgs a{x, (const bf16*)dy, partial, N, H, W, imgs, relu_in, (const bf16*)dp,
                  (const uint8_t*)pidx};
#ifndef MBK_WGRAD_QUEUE
#define MBK_WGRAD_QUEUE 1  // build knob (tools/variant.py): 0 = static stride (A/B)
#endif
  if (MBK_WGRAD_QUEUE) a.queue = mbk_work_queue(stream, kQueueWgrad);
  const size_t sm = wgrad_smem(cin, cout, imgs, H, W, unpool);
  if (sm > 160 * 1024 || nparts < 1 || !index_math_ok(imgs, H, W))
    return (int)hipErrorInvalidValue;
  dim3 grid(nparts);
#define LAUNCH(CI, CO, B)                                                                   \
  do {                                                                                      \
    const void* kfn = wgrad_kfn<CI, CO, B>(H, W, unpool);                    \
    if (!kfn) return (int)hipErrorInvalidValue;                              \
    if (sm > 64 * 1024)                                                                     \
      hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);        \
    void* args[] = {&a};                                                                    \
    hipLaunchKernel(kfn, grid, dim3(kThreads), args, sm, stream);                           \
  } while (0)
  if (in_bits) {
    if (cout == 16) LAUNCH(32, 16, true);
    else if (cout == 32) LAUNCH(32, 32, true);
    else return (int)hipErrorInvalidValue;
  } else if (cin == 16 && cout == 16) LAUNCH(16, 16, false);
  else if (cin == 16 && cout == 32) LAUNCH(16, 32, false);
  else if (cin == 32 && cout == 16) LAUNCH(32, 16, false);
  else if (cin == 32 && cout == 32) LAUNCH(32, 32, false);
  else return (int)hipErrorInvalidValue;
#undef LAUNCH
  return (int)hipGetLastError();
}

extern "C" void mbk_conv_set_grid_cap(int cap) { g_grid_cap = cap; }
extern "C" void mbk_conv0_row_set(int on) { g_conv0_row = on; }

// partial holds nparts rows plus ceil(nparts / kReducePps) scratch rows after them
extern "C" int mbk_wgrad_reduce(const float* partial, int nparts, int cin, int cin_real, int cout,
                                float* dw, float* db, int accumulate, hipStream_t stream) {
  const int row = cout * 9 * cin + cout;
  const dim3 cols((row + 63) / 64);
  if (nparts > 2 * kReducePps) {
    const int splits = (nparts + kReducePps - 1) / kReducePps;
    float* stage = (float*)partial + (size_t)nparts * row;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cols.x, splits), dim3(256), 0, stream, partial,
                       nparts, kReducePps, stage, cin, cin_real, cout, dw, db, accumulate);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cols.x, 1), dim3(256), 0, stream,
                       (const float*)stage, splits, splits, (float*)nullptr, cin, cin_real, cout,
                       dw, db, accumulate);
  } else {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cols.x, 1), dim3(256), 0, stream, partial,
                       nparts, nparts, (float*)nullptr, cin, cin_real, cout, dw, db, accumulate);
  }
  return (int)hipGetLastError();
}

// jobs[0..n): each as one mbk_wgrad_reduce call, in <= 2 launches per 32 jobs.
extern "C" int mbk_wgrad_reduce_batch(const MbkReduceJob* jobs, int n, hipStream_t stream) {
  for (int j0 = 0; j0 < n; j0 += kMaxReduceJobs) {
    const int nj = std::min(kMaxReduceJobs, n - j0);
    ReduceBatch b{};
    int cols = 1, splits = 1;
    bool two = false;
    for (int i = 0; i < nj; ++i) {
      const MbkReduceJob& J = jobs[j0 + i];
      if (!J.partial || !J.dw || J.nparts < 1 || J.cin < 1 || J.cout < 1 || J.cin_real > J.cin)
        return (int)hipErrorInvalidValue;
      b.j[i] = J;
      const int row = J.cout * 9 * J.cin + J.cout;
      cols = std::max(cols, (row + 63) / 64);
      if (J.nparts > 2 * kReducePps) {
        two = true;
        splits = std::max(splits, (J.nparts + kReducePps - 1) / kReducePps);
      }
    }
    hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3(cols, splits, nj), dim3(256), 0, stream,
                       b, 0);
    if (two)
      hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3(cols, 1, nj), dim3(256), 0, stream, b, 1);
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  return 0;
}

extern "C" int mbk_pool_bwd(const void* cfull, const void* dp, int N, int H, int W, int C,
                            void* dc, hipStream_t stream) {
  const size_t tot = (size_t)N * H * W * C;
  size_t blocks = (tot + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(pool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     (const bf16*)cfull, (const bf16*)dp, N, H, W, C, (bf16*)dc);
  return (int)hipGetLastError();
}

// dc = max_pool2d(3, 2, 1) backward of dp through the stored argmax bytes (2x2-block form:
// the output-order form measured level, DESIGN.md §9 rejected variants)
extern "C" int mbk_pool_bwd_idx(const void* pidx, const void* dp, int N, int H, int W, int C,
                                void* dc, hipStream_t stream) {
  if (C != 16 && C != 32) return (int)hipErrorInvalidValue;
  const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
  const size_t per_img_in = (size_t)H * W * C, per_img_out = (size_t)Ho * Wo * C;
  // keep every 32-bit index of one launch (input elements) below 2^31
  const int chunk = (int)std::max<size_t>(1, ((size_t)1 << 31) / per_img_in - 1);
  for (int n0 = 0; n0 < N; n0 += chunk) {
    const int n = std::min(chunk, N - n0);
    const size_t tot = (size_t)n * Ho * Wo * (C / 8);
    size_t blocks = (tot + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    const uint8_t* pi = (const uint8_t*)pidx + n0 * per_img_out;
    const bf16* d = (const bf16*)dp + n0 * per_img_out;
    bf16* o = (bf16*)dc + n0 * per_img_in;
    if (C == 16)
      hipLaunchKernelGGL(pool_bwd_idx_kernel<16>, dim3((unsigned)blocks), dim3(256), 0, stream, pi,
                         d, n, H, W, o);
    else
      hipLaunchKernelGGL(pool_bwd_idx_kernel<32>, dim3((unsigned)blocks), dim3(256), 0, stream, pi,
                         d, n, H, W, o);
  }
  return (int)hipGetLastError();
}

extern "C" int mbk_conv_pack_fp8(const MbkPackJob8* jobs, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > 16) return (int)hipErrorInvalidValue;
  PackJobs8 p;
  int maxc = 1;
  for (int i = 0; i < n; ++i) {
    p.j[i].w = jobs[i].w;
    p.j[i].q = (uint8_t*)jobs[i].q;
    p.j[i].scale = jobs[i].scale;
    p.j[i].cin = jobs[i].cin;
    p.j[i].cin_real = jobs[i].cin_real;
    p.j[i].cout = jobs[i].cout;
    maxc = std::max(maxc, jobs[i].cout);
  }
  p.n = n;
  hipLaunchKernelGGL(conv_pack_fp8_kernel, dim3(maxc, n), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

extern "C" int mbk_conv_pack(const MbkPackJob* jobs, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > 16) return (int)hipErrorInvalidValue;
  PackJobs p;
  for (int i = 0; i < n; ++i) {
    p.j[i].w = jobs[i].w;
    p.j[i].fwd = (bf16*)jobs[i].fwd;
    p.j[i].bwd = (bf16*)jobs[i].bwd;
    p.j[i].cin = jobs[i].cin;
    p.j[i].cin_real = jobs[i].cin_real;
    p.j[i].cout = jobs[i].cout;
  }
  p.n = n;
  hipLaunchKernelGGL(conv_pack_kernel, dim3(16, n), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

static int g_occ_cap[2] = {0, 0};  // learner forward / backward workgroups per CU (0: no cap)
static bool g_occ_read = false;    // a grid was sized with the caps: they are fixed from now on
int mbk_occ_cap(int bwd) {
  g_occ_read = true;
  return g_occ_cap[bwd ? 1 : 0];
}
// 0, or hipErrorInvalidValue when a grid / partial buffer was already sized with other caps
extern "C" int mbk_set_learner_occupancy(int fwd, int bwd) {
  fwd = fwd < 0 ? 0 : fwd;
  bwd = bwd < 0 ? 0 : bwd;
  if (g_occ_read && (fwd != g_occ_cap[0] || bwd != g_occ_cap[1])) return (int)hipErrorInvalidValue;
  g_occ_cap[0] = fwd;
  g_occ_cap[1] = bwd;
  return 0;
}

// ------------------------------------------------------------------ learner work queues
static int g_work_queues = 1;                 // mbk_set_work_queues (A/B)
static unsigned g_queue_sites = ~0u;          // mbk_set_work_queue_site: per call site
int* mbk_work_queue(hipStream_t stream, int site) {
  if (!g_work_queues || site < 0 || site >= kQueueSites || !((g_queue_sites >> site) & 1u))
    return nullptr;
  static std::mutex mu;
  static std::map<hipStream_t, int*> queues;
  std::lock_guard<std::mutex> lk(mu);
  auto it = queues.find(stream);
  if (it == queues.end()) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone)
      return nullptr;
    int* p = nullptr;
    if (hipMalloc(&p, kQueueSites * 2 * sizeof(int)) != hipSuccess ||
        hipMemsetAsync(p, 0, kQueueSites * 2 * sizeof(int), stream) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    it = queues.emplace(stream, p).first;
  }
  return it->second + 2 * site;
}
extern "C" int mbk_set_work_queues(int on) {
  g_work_queues = on ? 1 : 0;
  return 0;
}
// one call site's queue on / off (site: common.h kQueue*; 4 = the weight gradient, whose
// partial rows then sum their rounds in a run-dependent order: bit-identity tests turn it off)
extern "C" int mbk_set_work_queue_site(int site, int on) {
  if (site < 0 || site >= kQueueSites) return (int)hipErrorInvalidValue;
  g_queue_sites = on ? (g_queue_sites | (1u << site)) : (g_queue_sites & ~(1u << site));
  return 0;
}
