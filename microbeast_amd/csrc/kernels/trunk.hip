// Fused acting trunk: everything of the IMPALA encoder after the stage-0 conv + pool in
// ONE persistent launch (reference model.py:56-107: 2 residual blocks, then two more
// ConvSequences of conv -> maxpool -> 2 residual blocks; 14 convs, 2 pools, 12 relus,
// 6 residual adds).
//
// Per-layer launches (conv.hip) round-trip every activation through HBM and pay a
// launch each: at the acting batch (E = 4096 frames) the 14 convs cost ~125 us of the
// ~195 us policy step, mostly fixed latency. Here a workgroup owns TNI images at a time
// and keeps all of their activations in two LDS regions that the stages alias:
//
//   R1: X0 (stage-0 residual stream, 16 ch) -> X1 (32 ch) -> X2 (32 ch)
//   R2: U0 (inner conv output)  -> stage-1 pre-pool staging -> U1 -> stage-2 staging -> U2
//
// Tiles are halo'd NHWC (pixel stride 2*C + 16 bytes); a producer phase zeroes the halo
// of the tile it fills (disjoint from the interior it writes), so regions can change
// layout between stages without extra passes. Each conv is an implicit GEMM on
// v_mfma_f32_16x16x32_bf16 with (A = weights from L2 into VGPRs, B = pixels from LDS),
// so a lane ends with 4 consecutive channels of one pixel. ReLU-on-input is applied to
// the B fragments; the residual add reads the output tile in place. Inference only
// (no saved activations); numerics identical to the per-layer kernels (bf16 storage,
// fp32 accumulation, pool over bf16-rounded values).
#include "../include/mbk_api.h"
#include "common.h"
#include "decode.h"


#include <algorithm>
#include <cstdlib>
#include <string>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

constexpr int kThreads = 512;  // 8 waves: 2 per SIMD even at one workgroup per CU
constexpr int kMaxTNI = 16;  // images per workgroup iteration (host picks <= this)
constexpr int kWBufBytes = 32 * (9 * 64 + 16);  // one staged layer (largest: 32x32)

union Frag8 {
  bf16x8 v;
  uint4 u;
};

typedef short s16x2 __attribute__((ext_vector_type(2)));
// relu of a bf16 pair in ONE v_pk_max_i16: a bf16 with the sign bit set is a negative
// int16 (-0.0 = 0x8000 too), a non-negative one a non-negative int16, so the signed max
// with 0 is exactly relu (the bit-select form costs ~6 VALU per dword, and the trunk
// re-applies relu for all 9 taps of every input pixel: profile 15, VALU-bound)
__device__ __forceinline__ uint32_t relu2(uint32_t w) {
  s16x2 v = __builtin_bit_cast(s16x2, w);
  v = __builtin_elementwise_max(v, s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(a)) |
         ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(b)) << 16);
}
__device__ __forceinline__ float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

template <int C>
struct TG {
  static constexpr int PIXB = C * 2 + 16;
  static constexpr int PIXB8 = C + 8;  // fp8 (e4m3) tile pixel stride, as conv.hip's fp8 tile
  static constexpr int NCH = C == 16 ? 5 : 9;
};

// zero the halo ring of a halo'd tile [nimg][(H+2)][(W+2)] of PIXB-byte pixels (index math
// by float reciprocals: exact for these tiny ranges, no runtime integer division); 16-byte
// stores, or 8-byte ones for the fp8 tiles (PIXB = C + 8)
template <int PIXB, bool WV = false>  // WV: the calling wave alone (its own images)
__device__ __forceinline__ void zero_halo(char* t, int nimg, int H, int W) {
  const int Hp = H + 2, Wp = W + 2;
  const int per = 2 * Wp + 2 * H;  // halo pixels per image
  constexpr int U = PIXB % 16 == 0 ? 16 : 8;
  constexpr int qn = PIXB / U;
  const int tot = nimg * per * qn;
  const float inv_per = 1.f / (float)per;
  int e0 = WV ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  if (WV) asm volatile("" : "+v"(e0));  // opaque: not hoisted out of the acting tile loop
  for (int e = e0; e < tot; e += WV ? 64 : kThreads) {
    const int r = e / qn, q = e - r * qn;  // qn is a compile-time constant
    const int im = (int)(((float)r + 0.5f) * inv_per), k = r - im * per;
    int py, px;
    if (k < Wp) { py = 0; px = k; }
    else if (k < 2 * Wp) { py = Hp - 1; px = k - Wp; }
    else { const int j = k - 2 * Wp; py = 1 + (j >> 1); px = (j & 1) ? Wp - 1 : 0; }
    char* p = t + ((im * Hp + py) * Wp + px) * PIXB + q * U;
    if constexpr (U == 16) *(uint4*)p = make_uint4(0, 0, 0, 0);
    else *(uint2*)p = make_uint2(0, 0);
  }
}

// 4 floats -> 4 OCP e4m3 bytes, round-to-nearest-even saturated to +-448 (conv.hip's
// cvt_fp8x4: the per-layer fp8 kernel's staging conversion, so the fused fp8 trunk matches it)
__device__ __forceinline__ uint32_t fp8x4(float a, float b, float c, float d) {
  auto sat = [](float v) { return fminf(fmaxf(v, -448.f), 448.f); };
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(d), w, true);
  return (uint32_t)w;
}
// 4 bf16 (two packed words) -> e4m3, optionally through relu
__device__ __forceinline__ uint32_t bf16x4_fp8(uint2 o, bool relu) {
  if (relu) o = make_uint2(relu2(o.x), relu2(o.y));
  return fp8x4(lo_f(o.x), hi_f(o.x), lo_f(o.y), hi_f(o.y));
}

// conv3x3 (pad 1) of a halo'd LDS tile. Output either into a halo'd tile (with optional
// in-place residual add from the same tile) or into a dense bf16 staging [nimg][H][W][COUT]
// (for the pool). relu_in applies to the input fragments.
// A layer's packed weights [COUT][NCH][32] bf16 live in LDS with each output row padded
// by 16 bytes (row stride NCH*64 + 16: the 16 rows a wave reads hit distinct banks).
template <int CIN>
__device__ __forceinline__ int wrow_bytes() { return TG<CIN>::NCH * 64 + 16; }

constexpr int kWRegs = 3;  // uint4 per thread to stage the largest layer (32x9x32 bf16)

// global -> registers (issued early, overlapping the current conv)
__device__ __forceinline__ void wload(const bf16* __restrict__ gw, int n16, uint4 r[kWRegs]) {
#pragma unroll
  for (int k = 0; k < kWRegs; ++k) {
    const int e = threadIdx.x + k * kThreads;
    r[k] = e < n16 ? ((const uint4*)gw)[e] : make_uint4(0, 0, 0, 0);
  }
}
// registers -> padded LDS rows
__device__ __forceinline__ void wstore(char* lw, int n16, int nch, const uint4 r[kWRegs]) {
  const int per_row = nch * 4, stride = nch * 64 + 16;
#pragma unroll
  for (int k = 0; k < kWRegs; ++k) {
    const int e = threadIdx.x + k * kThreads;
    if (e < n16) *(uint4*)(lw + (e / per_row) * stride + (e % per_row) * 16) = r[k];
  }
}

// The whole dynamic LDS of trunk_tail_kernel. conv_lds below is noinline (see there), so it
// must address the tiles through this LDS array with 32-bit offsets: a generic char*
// argument lowered every fragment read / epilogue store to flat_load / flat_store with
// 64-bit address math and s_waitcnt vmcnt(0) lgkmcnt(0) (it could be global memory).
extern __shared__ __attribute__((aligned(16))) char trunk_smem[];

// OUT_TILE_RELU: the inner activation U of a residual block is consumed only by the block's
// second conv, through a relu: store relu(U) once in the epilogue instead of re-applying it
// to every one of U's 9 tap reads (bit-identical: relu commutes with the bf16 rounding)
enum ConvOut : int { OUT_TILE = 0, OUT_TILE_ADD = 1, OUT_STAGE = 2, OUT_TILE_RELU = 3 };

constexpr int kWFrag = 18;  // this lane's weight fragments of the largest layer (9 x 2)

// A lane's packed-weight fragments of tail layer l, (chunk c, block nb) at c * NB + nb.
// Issued one layer ahead by the kernel, so the L2 latency of a layer's weights hides
// behind the previous layer's MFMAs (loading them at the top of each conv exposed it 14
// times per image group).
__device__ __forceinline__ void wfetch(const bf16* gw, int cin, int cout, uint4 w[kWFrag]) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) u32x4* GU4;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int nch = cin == 16 ? TG<16>::NCH : TG<32>::NCH, nb = cout / 16;
#pragma unroll
  for (int k = 0; k < kWFrag; ++k) {
    const int c = k / 2, b = k % 2;  // fixed (c, nb) slot layout: c * 2 + nb
    if (c < nch && b < nb) {
      const u32x4 v = ((GU4)((const char*)gw + ((b * 16 + li) * nch * 64 + g * 16)))[c * 4];
      w[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
}
// the same for e4m3 packed weights [COUT][NCH][32] bytes (conv.hip conv_pack_fp8 layout):
// 8 bytes per (chunk, block) fragment
__device__ __forceinline__ void wfetch8(const uint8_t* gw, int cin, int cout, long w[kWFrag]) {
  typedef const __attribute__((address_space(1))) long* GL;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int nch = cin == 16 ? TG<16>::NCH : TG<32>::NCH, nb = cout / 16;
#pragma unroll
  for (int k = 0; k < kWFrag; ++k) {
    const int c = k / 2, b = k % 2;
    if (c < nch && b < nb) w[k] = ((GL)(gw + ((b * 16 + li) * nch * 32 + g * 8)))[c * 4];
  }
}

// F8 (fp8 trunk, conv.hip's per-layer fp8 numerics): the input tile holds e4m3 activations
// (pixel stride CIN + 8, already relu'd by their producer, so RELU is false), wreg8 holds the
// lane's e4m3 weight fragments, acc is dequantised by the per-output-channel wscale, and
//   MODE OUT_TILE_RELU writes fp8(relu(bf16(v))) into an fp8 tile (out, stride COUT + 8);
//   MODE OUT_TILE_ADD writes the bf16 residual stream (out) and, for cp = 1 / 2, its fp8 copy
//   relu'd / as is into the fp8 tile at out8 (the next conv's input).
// WV (wave-owned tiles, act_trunk_w_kernel): 0 = the workgroup's waves share the tile's pixel
// blocks (wave w takes blocks w, w + NW, ...); 1 = the calling wave alone runs every block of
// its own images, two blocks per iteration; 2 = the same one block at a time (maps whose pixel
// count is one block: no idle partner chain)
template <int CIN, int COUT, bool RELU, int MODE, bool WLDS, bool F8 = false, int WV = 0>
// in / out: byte offsets of halo'd tiles in trunk_smem (out of a MODE == OUT_STAGE call: a
// dense bf16 staging [nimg][H][W][COUT]); weights: LDS offset (WLDS, rows of wstride bytes)
// or this lane's fragments prefetched into registers by wfetch (wreg)
__device__ __forceinline__ void conv_lds(int in, int H, int W, int nimg, int lw_off,
                                         const uint4* wreg, int wstride,
                                         const float* __restrict__ bias, int out,
                                         const long* wreg8 = nullptr,
                                         const float* __restrict__ wscale = nullptr,
                                         int out8 = 0, int cp = 0) {
  constexpr int NCH = TG<CIN>::NCH, NB = COUT / 16;
  constexpr int PI = F8 ? TG<CIN>::PIXB8 : TG<CIN>::PIXB;
  constexpr int PO = (F8 && MODE == OUT_TILE_RELU) ? TG<COUT>::PIXB8 : TG<COUT>::PIXB;
  constexpr int PO8 = TG<COUT>::PIXB8;
  static_assert(!(F8 && (RELU || WLDS)), "fp8 tiles are stored relu'd; weights from L2");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int Hp = H + 2, Wp = W + 2, HW = H * W;
  Frag8 bw[NCH][NB];
  long bw8[NCH][NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if constexpr (F8) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) bw8[c][nb] = wreg8[c * 2 + nb];
    } else if constexpr (WLDS) {
      const int wr = lw_off + (nb * 16 + li) * wstride + g * 16;
#pragma unroll
      for (int c = 0; c < NCH; ++c) bw[c][nb].u = *(const uint4*)(trunk_smem + wr + c * 64);
    } else {
#pragma unroll
      for (int c = 0; c < NCH; ++c) bw[c][nb].u = wreg[c * 2 + nb];
    }
  }
  typedef const __attribute__((address_space(1))) f32x4* GF4;
  float bv[NB][4], wsc[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const f32x4 b4 = ((GF4)bias)[(nb * 16 + 4 * g) / 4];
    bv[nb][0] = b4[0]; bv[nb][1] = b4[1]; bv[nb][2] = b4[2]; bv[nb][3] = b4[3];
    if constexpr (F8) {
      const f32x4 s4 = ((GF4)wscale)[(nb * 16 + 4 * g) / 4];
      wsc[nb][0] = s4[0]; wsc[nb][1] = s4[1]; wsc[nb][2] = s4[2]; wsc[nb][3] = s4[3];
    }
  }
  const int M = nimg * HW, nblk = (M + 15) >> 4;
  constexpr int NW = kThreads / 64;
  // Two pixel blocks per wave iteration (pb, pb + NW): two independent MFMA chains and
  // their LDS fragment reads interleave, so neither the MFMA dependency latency of one
  // accumulator chain nor the LDS read latency is exposed per block. Each chain runs the
  // taps in the same order as before (bit-identical results).
  // pixel -> (image, y, x) with float reciprocals (exact for m < 2^16, HW <= 1024: the
  // distance of (m + 0.5) / HW to an integer is >= 0.5 / HW, far above the rounding error;
  // mbk_trunk_tail refuses shapes outside that bound);
  // the integer divisions by runtime H*W / W cost ~20 VALU per block (profile 15: VALU-bound)
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  auto epilogue = [&](int pb, const f32x4* acc) {
    const int m = pb * 16 + li;
    if (pb >= nblk || m >= M) return;
    const int im = (int)(((float)m + 0.5f) * inv_hw), r = m - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int co0 = nb * 16 + 4 * g;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (F8) v[i] = acc[nb][i] * wsc[nb][i] + bv[nb][i];
        else v[i] = acc[nb][i] + bv[nb][i];
      }
      const int pix = (im * Hp + y + 1) * Wp + x + 1;
      if constexpr (MODE == OUT_STAGE) {
        *(uint2*)(trunk_smem + out + (m * COUT + co0) * 2) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      } else if constexpr (F8 && MODE == OUT_TILE_RELU) {
        *(uint32_t*)(trunk_smem + out + pix * PO + co0) =
            bf16x4_fp8(make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3])), true);
      } else {
        char* p = trunk_smem + out + (pix * PO + co0 * 2);
        if constexpr (MODE == OUT_TILE_ADD) {
          const uint2 ad = *(const uint2*)p;
          v[0] += lo_f(ad.x); v[1] += hi_f(ad.x); v[2] += lo_f(ad.y); v[3] += hi_f(ad.y);
        }
        uint2 o = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if constexpr (MODE == OUT_TILE_RELU) o = make_uint2(relu2(o.x), relu2(o.y));
        *(uint2*)p = o;
        if constexpr (F8)
          if (cp) *(uint32_t*)(trunk_smem + out8 + pix * PO8 + co0) = bf16x4_fp8(o, cp == 1);
      }
    }
  };
  constexpr int NJ = WV == 2 ? 1 : 2;  // independent block chains per iteration
  const int pstart = WV ? 0 : wave;
  constexpr int pstep = WV ? NJ : 2 * NW, poff = WV ? 1 : NW;
  for (int pb0 = pstart; pb0 < nblk; pb0 += pstep) {
    int base[2];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int m = (pb0 + j * poff) * 16 + li;
      const int mm = m < M ? m : 0;  // rows past M compute garbage that is never stored
      const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
      const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
      base[j] = in + ((im * Hp + y) * Wp + x) * PI;
    }
    f32x4 acc[2][NB];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[j][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      int tap, ch0;
      if (CIN == 16) { tap = 2 * c + (g >> 1); ch0 = 8 * (g & 1); }
      else { tap = c; ch0 = 8 * g; }
      const int tapc = tap < 9 ? tap : 8;
      const int toff = ((tapc / 3) * Wp + (tapc % 3)) * PI + (F8 ? ch0 : ch0 * 2);
      if constexpr (F8) {
        long a8[2];
#pragma unroll
        for (int j = 0; j < NJ; ++j) a8[j] = *(const long*)(trunk_smem + base[j] + toff);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[j][nb] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(bw8[c][nb], a8[j], acc[j][nb], 0, 0, 0);
        continue;
      }
      Frag8 a[2];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        a[j].u = *(const uint4*)(trunk_smem + base[j] + toff);
        if constexpr (RELU)
          a[j].u = make_uint4(relu2(a[j].u.x), relu2(a[j].u.y), relu2(a[j].u.z), relu2(a[j].u.w));
        // (CIN 16, tap 9 = the pad half of chunk 4: its packed weights are zero, so the
        // finite pixel read for it adds exactly 0 and needs no zeroing)
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[j][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[c][nb].v, a[j].v, acc[j][nb], 0, 0, 0);
    }
    epilogue(pb0, acc[0]);
    if constexpr (NJ == 2) epilogue(pb0 + poff, acc[1]);
  }
}

// One wave's conv over all of its own pixel blocks at once (the wave-owned acting tile): the
// K-chunk loop is outside and the NBLK blocks (all the wave's pixels: NBLK * 16 >= M) inside,
// so every chunk's weight fragment feeds NBLK independent accumulator chains and its LDS reads
// issue together -- conv_lds WV = 1 ran two chains per iteration and paid the LDS latency, the
// MFMA dependency and the epilogue once per block pair. Same taps, K order and epilogue maths
// per output pixel as conv_lds (bit-identical). Pixel rows m >= M compute on pixel 0 and are not
// stored.
template <int CIN, int COUT, bool RELU, int MODE, int NBLK, int NPASS = 1>
__device__ __forceinline__ void conv_w(int in, int H, int W, int M, const uint4* wreg,
                                       const float* __restrict__ bias, int out) {
  // NPASS passes of NBLK blocks (pass p: blocks p * NBLK ..): bounds the live accumulators
#pragma unroll 1
  for (int pass = 0; pass < NPASS; ++pass) {
  const int jb = pass * NBLK;
  constexpr int NCH = TG<CIN>::NCH, NB = COUT / 16;
  constexpr int PI = TG<CIN>::PIXB, PO = TG<COUT>::PIXB;
  // an opaque lane index: every address below derives from it, so none of them is hoisted out
  // of the tile loop (LICM kept all phases' pixel offsets live across the whole tile: spills)
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int g = lane >> 4, li = lane & 15;
  const int Hp = H + 2, Wp = W + 2, HW = H * W;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  Frag8 bw[NCH][NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int c = 0; c < NCH; ++c) bw[c][nb].u = wreg[c * 2 + nb];
  typedef const __attribute__((address_space(1))) f32x4* GF4;
  float bv[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const f32x4 b4 = ((GF4)bias)[(nb * 16 + 4 * g) / 4];
    bv[nb][0] = b4[0]; bv[nb][1] = b4[1]; bv[nb][2] = b4[2]; bv[nb][3] = b4[3];
  }
  int base[NBLK];
#pragma unroll
  for (int j = 0; j < NBLK; ++j) {
    const int m = (jb + j) * 16 + li;
    const int mm = m < M ? m : 0;
    const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
    base[j] = in + ((im * Hp + y) * Wp + x) * PI;
  }
  f32x4 acc[NBLK][NB];
#pragma unroll
  for (int j = 0; j < NBLK; ++j)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[j][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // chunk c's LDS byte offset (tap, 8-channel group of this lane)
  auto toff = [&](int c) {
    int tap, ch0;
    if (CIN == 16) { tap = 2 * c + (g >> 1); ch0 = 8 * (g & 1); }
    else { tap = c; ch0 = 8 * g; }
    const int tapc = tap < 9 ? tap : 8;
    return ((tapc / 3) * Wp + (tapc % 3)) * PI + ch0 * 2;
  };
  // software pipeline: chunk c+1's NBLK fragment reads are issued before chunk c's MFMAs, so the
  // LDS latency hides behind NBLK x NB MFMAs instead of stalling every block
  Frag8 fr[2][NBLK];
#pragma unroll
  for (int j = 0; j < NBLK; ++j) fr[0][j].u = *(const uint4*)(trunk_smem + base[j] + toff(0));
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) {
      const int to = toff(c + 1);
#pragma unroll
      for (int j = 0; j < NBLK; ++j)
        fr[(c + 1) & 1][j].u = *(const uint4*)(trunk_smem + base[j] + to);
    }
#pragma unroll
    for (int j = 0; j < NBLK; ++j) {
      Frag8 a = fr[c & 1][j];
      if constexpr (RELU)
        a.u = make_uint4(relu2(a.u.x), relu2(a.u.y), relu2(a.u.z), relu2(a.u.w));
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[j][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[c][nb].v, a.v, acc[j][nb], 0, 0, 0);
    }
    // (no reads hoisted further: two chunks' fragments in flight at most)
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < NBLK; ++j) {
    const int m = (jb + j) * 16 + li;
    if (m >= M) continue;
    const int im = (int)(((float)m + 0.5f) * inv_hw), r = m - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
    const int pix = (im * Hp + y + 1) * Wp + x + 1;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int co0 = nb * 16 + 4 * g;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[j][nb][i] + bv[nb][i];
      if constexpr (MODE == OUT_STAGE) {
        *(uint2*)(trunk_smem + out + (m * COUT + co0) * 2) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      } else {
        char* p = trunk_smem + out + (pix * PO + co0 * 2);
        if constexpr (MODE == OUT_TILE_ADD) {
          const uint2 ad = *(const uint2*)p;
          v[0] += lo_f(ad.x); v[1] += hi_f(ad.x); v[2] += lo_f(ad.y); v[3] += hi_f(ad.y);
        }
        uint2 o = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if constexpr (MODE == OUT_TILE_RELU) o = make_uint2(relu2(o.x), relu2(o.y));
        *(uint2*)p = o;
      }
    }
  }
  }
}

// max_pool2d(3, 2, 1) of staging [nimg][H][W][C] into the interior of a halo'd tile (F8: and
// fp8(relu(.)) into the fp8 tile out8, the next residual block's conv input)
template <int C, bool F8 = false, bool WV = false>
__device__ __forceinline__ void pool_lds(const bf16* stg, int H, int W, int nimg, char* out,
                                         char* out8 = nullptr) {
  constexpr int PO = TG<C>::PIXB, C4 = C / 4;
  const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1, HWo = Ho * Wo;
  const int tot = nimg * HWo * C4;
  const float inv_hwo = 1.f / (float)HWo, inv_wo = 1.f / (float)Wo;
  int e0 = WV ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  if (WV) asm volatile("" : "+v"(e0));  // opaque: not hoisted out of the acting tile loop
  for (int e = e0; e < tot; e += WV ? 64 : kThreads) {
    const int c4 = e % C4, p = e / C4;  // C4: compile-time power of two
    const int im = (int)(((float)p + 0.5f) * inv_hwo), r = p - im * HWo;
    const int oy = (int)(((float)r + 0.5f) * inv_wo), ox = r - oy * Wo;
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = 2 * oy - 1 + ky;
      if (yy < 0 || yy >= H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = 2 * ox - 1 + kx;
        if (xx < 0 || xx >= W) continue;
        const uint2 v = *(const uint2*)(stg + ((size_t)(im * H + yy) * W + xx) * C + 4 * c4);
        mx[0] = fmaxf(mx[0], lo_f(v.x)); mx[1] = fmaxf(mx[1], hi_f(v.x));
        mx[2] = fmaxf(mx[2], lo_f(v.y)); mx[3] = fmaxf(mx[3], hi_f(v.y));
      }
    }
    const int pix = (im * (Ho + 2) + oy + 1) * (Wo + 2) + ox + 1;
    const uint2 o = make_uint2(pack2(mx[0], mx[1]), pack2(mx[2], mx[3]));
    *(uint2*)(out + pix * PO + c4 * 8) = o;
    if constexpr (F8) *(uint32_t*)(out8 + pix * TG<C>::PIXB8 + c4 * 4) = bf16x4_fp8(o, true);
  }
}

struct TrunkArgs {
  const bf16* x;        // stage-0 pooled output [N][H0][W0][16]
  bf16* y;              // trunk output [N][H2][W2][32] (null: not stored)
  // fused trunk head (f_out != null): f = relu(W5 relu(y) + b5) [N][256] bf16 and the
  // critic v = wc . f + bc [N] fp32, from the LDS-resident X2 tile (fc.hip fc_fwd's maths)
  const bf16* w5;       // [256][H2*W2*32], columns in NHWC flatten order
  const float* b5;
  const float* wc;
  const float* bc;
  bf16* f_out;
  float* v_out;
  const bf16* w[14];    // packed fwd weights of layers 1..14 (HipEncoder order)
  const float* b[14];
  const uint8_t* w8[14];  // fp8 trunk: e4m3 packed weights (conv_pack_fp8) ...
  const float* ws[14];    // ... and their per-output-channel dequant scales
  int N, H0, W0;
  int tni;              // images per workgroup iteration
  int r1_bytes;         // region sizes (host computed)
  int r2_bytes;         // (fp8 trunk: A = r1_bytes, B = r2_bytes)
};

// layer l of the tail (0..13): CIN / COUT of the (16, 32, 32) trunk
__device__ __forceinline__ int tail_cin(int l) { return l < 5 ? 16 : 32; }
__device__ __forceinline__ int tail_cout(int l) { return l < 4 ? 16 : 32; }
__device__ __forceinline__ int tail_n16(int l) {
  return tail_cout(l) * TG<16>::NCH * 4 * (tail_cin(l) == 16 ? 1 : 0) +
         tail_cout(l) * TG<32>::NCH * 4 * (tail_cin(l) == 32 ? 1 : 0);
}

__device__ __forceinline__ uint4 relu8(uint4 v) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = ((w[j] & 0x8000u) ? 0u : (w[j] & 0xFFFFu)) |
           ((w[j] & 0x80000000u) ? 0u : (w[j] & 0xFFFF0000u));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// relu -> network.5 (256 hidden) -> relu -> critic on the group's X2 tile (halo'd NHWC in
// LDS at x2): the same MFMA tiling, K order and value reduction as fc.hip fc_fwd_kernel<256>
// (waves 0-3 take images [0,16), waves 4-7 images [16,32) of each 32-image chunk; 4 hidden
// blocks of 16 per wave), so f and v match the separate launch bit for bit.
__device__ __forceinline__ void trunk_fc(const char* x2, int H2, int W2, int nimg, int img0,
                                         const TrunkArgs& a, float* vred) {
  constexpr int O = 256, NBW = 4, PX = TG<32>::PIXB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int half = wave >> 2, wq = wave & 3;
  const int I = H2 * W2 * 32, nks = H2 * W2;
  for (int c0 = 0; c0 < nimg; c0 += 32) {
    const int im = c0 + half * 16 + li;
    const bool valid = im < nimg;
    // one hidden block at a time (4 accumulators live, not 16): the head runs at the end of
    // a 256-VGPR kernel; x fragments are re-read from LDS per block instead
#pragma unroll 1
    for (int j = 0; j < NBW; ++j) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint4* wrow = (const uint4*)(a.w5 + (size_t)((wq * NBW + j) * 16 + li) * I) + G;
#pragma unroll 1
      for (int ks = 0; ks < nks; ++ks) {  // K step = one pixel's 32 channels
        const int py = ks / W2, px = ks - py * W2;
        Frag8 b, w;
        b.u = make_uint4(0, 0, 0, 0);
        if (valid)
          b.u = relu8(*(const uint4*)(x2 + ((im * (H2 + 2) + py + 1) * (W2 + 2) + px + 1) * PX +
                                      G * 16));
        w.u = wrow[ks * 4];
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.v, b.v, acc, 0, 0, 0);
      }
      const int h0 = (wq * NBW + j) * 16 + 4 * G;
      float hv[4], w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        hv[i] = __bfloat162float(__float2bfloat16(fmaxf(acc[i] + a.b5[h0 + i], 0.f)));
        w4[i] = a.wc[h0 + i];
      }
      const float q = mbk::crit_block(hv, w4);  // the critic order of every FC kernel
      if (G == 0) vred[(half * 16 + wq * NBW + j) * 16 + li] = q;
      uint32_t o[2];
#pragma unroll
      for (int k = 0; k < 2; ++k)
        o[k] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k])) |
               ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k + 1])) << 16);
      if (valid) *(uint2*)(a.f_out + (size_t)(img0 + im) * O + h0) = make_uint2(o[0], o[1]);
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      const int hh = threadIdx.x >> 4, t = threadIdx.x & 15, r = c0 + hh * 16 + t;
      if (r < nimg) a.v_out[img0 + r] = mbk::crit_sum(vred + hh * 256 + t, 16, 16, a.bc[0]);
    }
    __syncthreads();
  }
}

// group input (stage-0 pooled output, bf16 NHWC) -> interior of the halo'd X0 tile; F8: also
// fp8(relu(x)) into the fp8 tile f (layer 1's input)
template <bool F8>
__device__ __forceinline__ void load_input(const TrunkArgs& a, int img0, int nimg, char* x0,
                                           char* f) {
  constexpr int PX = TG<16>::PIXB, PX8 = TG<16>::PIXB8;
  const int H0 = a.H0, W0 = a.W0;
  const int tot = nimg * H0 * W0 * 2;  // 16-byte chunks
  const uint4* src = (const uint4*)(a.x + (size_t)img0 * H0 * W0 * 16);
  const float ihw = 1.f / (float)(H0 * W0), iw = 1.f / (float)W0;
  for (int e = threadIdx.x; e < tot; e += kThreads) {
    const int q = e & 1, p = e >> 1;
    const int im = (int)(((float)p + 0.5f) * ihw), r = p - im * H0 * W0;
    const int y = (int)(((float)r + 0.5f) * iw), x = r - y * W0;
    const int pix = (im * (H0 + 2) + y + 1) * (W0 + 2) + x + 1;
    const uint4 v = src[e];
    *(uint4*)(x0 + pix * PX + q * 16) = v;
    if constexpr (F8)
      *(uint2*)(f + pix * PX8 + q * 8) = make_uint2(bf16x4_fp8(make_uint2(v.x, v.y), true),
                                                    bf16x4_fp8(make_uint2(v.z, v.w), true));
  }
}

// X2 tile interior -> global NHWC trunk output (if requested)
__device__ __forceinline__ void store_output(const TrunkArgs& a, int img0, int nimg, int H2,
                                             int W2, const char* x2) {
  if (!a.y) return;
  constexpr int PX = TG<32>::PIXB;
  const int tot = nimg * H2 * W2 * 4;
  uint4* dst = (uint4*)(a.y + (size_t)img0 * H2 * W2 * 32);
  const float ihw = 1.f / (float)(H2 * W2), iw = 1.f / (float)W2;
  for (int e = threadIdx.x; e < tot; e += kThreads) {
    const int q = e & 3, p = e >> 2;
    const int im = (int)(((float)p + 0.5f) * ihw), r = p - im * H2 * W2;
    const int y = (int)(((float)r + 0.5f) * iw), x = r - y * W2;
    dst[e] = *(const uint4*)(x2 + ((im * (H2 + 2) + y + 1) * (W2 + 2) + x + 1) * PX + q * 16);
  }
}

// Weights read through L2 into registers one layer ahead (staging them in LDS, double-
// buffered, measured slower than L2 + 16 images per tile). FC: the fused trunk head runs
// after the last conv; the next group's first weight fetch then waits until after it (keeps
// the prefetch registers free across the head: no spills).
template <bool FC>
__global__ __launch_bounds__(kThreads) void trunk_tail_kernel(TrunkArgs a) {
  char* smem = trunk_smem;
  const int oR1 = 0, oR2 = a.r1_bytes;  // region offsets for conv_lds
  char* R1 = smem + oR1;
  char* R2 = smem + oR2;
  const int H0 = a.H0, W0 = a.W0, H1 = (H0 + 1) >> 1, W1 = (W0 + 1) >> 1;
  const int H2 = (H1 + 1) >> 1, W2 = (W1 + 1) >> 1;
  const int TNI = a.tni;
  const int ngroups = (a.N + TNI - 1) / TNI;
  uint4 wnext[kWFrag];  // register prefetch of the next layer's weights
  wfetch(a.w[0], tail_cin(0), tail_cout(0), wnext);
  // phase helper: take layer l's prefetched weights, prefetch layer l+1 (wrapping to 0 for
  // the next group), run conv l
#define TAIL_PHASE(l, CI, CO, RELU, MODE, IN, H_, W_, WBUF, OUT)                          \
  do {                                                                                      \
    uint4 wc[kWFrag];                                                                       \
    _Pragma("unroll") for (int k = 0; k < kWFrag; ++k) wc[k] = wnext[k];                    \
    if (!(FC && (l) == 13)) {                                                               \
      const int ln = ((l) + 1) % 14;                                                        \
      wfetch(a.w[ln], tail_cin(ln), tail_cout(ln), wnext);                                  \
    }                                                                                       \
    conv_lds<CI, CO, RELU, MODE, false>(IN, H_, W_, nimg, 0, wc, TG<CI>::NCH * 64, a.b[l],  \
                                        OUT);                                               \
  } while (0)
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * TNI, nimg = min(TNI, a.N - img0);
    // ---- stage 0: X0 <- input (R1), U0 halo zero (R2)
    load_input<false>(a, img0, nimg, R1, nullptr);
    zero_halo<TG<16>::PIXB>(R1, nimg, H0, W0);
    zero_halo<TG<16>::PIXB>(R2, nimg, H0, W0);
    __syncthreads();
#pragma unroll 1
    for (int rb = 0; rb < 2; ++rb) {
      TAIL_PHASE(2 * rb, 16, 16, true, OUT_TILE_RELU, oR1, H0, W0, oWB[0], oR2);
      __syncthreads();
      TAIL_PHASE(2 * rb + 1, 16, 16, false, OUT_TILE_ADD, oR2, H0, W0, oWB[1], oR1);
      __syncthreads();
    }
    // ---- stage 1: conv 16->32 (staging in R2) -> pool -> X1 (R1)
    TAIL_PHASE(4, 16, 32, false, OUT_STAGE, oR1, H0, W0, oWB[0], oR2);
    __syncthreads();
    pool_lds<32>((const bf16*)R2, H0, W0, nimg, R1);
    zero_halo<TG<32>::PIXB>(R1, nimg, H1, W1);
    __syncthreads();
    zero_halo<TG<32>::PIXB>(R2, nimg, H1, W1);  // U1 layout (staging consumed)
#pragma unroll 1
    for (int rb = 0; rb < 2; ++rb) {
      TAIL_PHASE(5 + 2 * rb, 32, 32, true, OUT_TILE_RELU, oR1, H1, W1, oWB[1], oR2);
      __syncthreads();
      TAIL_PHASE(6 + 2 * rb, 32, 32, false, OUT_TILE_ADD, oR2, H1, W1, oWB[0], oR1);
      __syncthreads();
    }
    // ---- stage 2
    TAIL_PHASE(9, 32, 32, false, OUT_STAGE, oR1, H1, W1, oWB[1], oR2);
    __syncthreads();
    pool_lds<32>((const bf16*)R2, H1, W1, nimg, R1);
    zero_halo<TG<32>::PIXB>(R1, nimg, H2, W2);
    __syncthreads();
    zero_halo<TG<32>::PIXB>(R2, nimg, H2, W2);
#pragma unroll 1
    for (int rb = 0; rb < 2; ++rb) {
      TAIL_PHASE(10 + 2 * rb, 32, 32, true, OUT_TILE_RELU, oR1, H2, W2, oWB[0], oR2);
      __syncthreads();
      TAIL_PHASE(11 + 2 * rb, 32, 32, false, OUT_TILE_ADD, oR2, H2, W2, oWB[1], oR1);
      __syncthreads();
    }
#undef TAIL_PHASE
    if (FC) {
      trunk_fc(R1, H2, W2, nimg, img0, a, (float*)R2);
      wfetch(a.w[0], tail_cin(0), tail_cout(0), wnext);  // next group's layer 0
    }
    // ---- X2 interior -> global NHWC
    store_output(a, img0, nimg, H2, W2, R1);
    __syncthreads();
  }
}

// fp8 trunk (BASELINE config 5's fp8 acting path, inference): the 14 convs on
// v_mfma_f32_16x16x32_fp8_fp8, numerics of the per-layer fp8 kernel (conv.hip F8: e4m3
// activations converted from the bf16-rounded producer output, relu before the
// conversion, per-output-channel weight scales, bf16 outputs / residual stream). LDS:
//   R1: residual stream X (bf16, halo'd): the residual adds and the trunk output read it
//   R2: U (inner activation, fp8 relu'd) / stage conv staging (dense bf16)
//   R3: F = fp8 copy of X as the next conv consumes it (relu'd for a residual block, as is
//       for the next stage's conv), written by the producer's epilogue / the pool
// so each conv reads 8-byte fragments with no per-tap relu. Weights are fetched one layer
// ahead into registers (half the VGPRs of the bf16 prefetch).
__global__ __launch_bounds__(kThreads) void trunk_tail8_kernel(TrunkArgs a) {
  // regions (trunk8_region_*): A = X0 (bf16) in stage 0, then the pool staging and U (fp8)
  // of stages 1-2; B = U0 (fp8) in stage 0, then X1 / X2 (bf16); F = the fp8 conv input.
  // Swapping the roles after stage 0 keeps the 16-image group of the bf16 trunk in LDS.
  char* smem = trunk_smem;
  const int oA = 0, oB = a.r1_bytes, oF = a.r1_bytes + a.r2_bytes;
  char* A = smem + oA;
  char* B = smem + oB;
  char* F = smem + oF;
  const int H0 = a.H0, W0 = a.W0, H1 = (H0 + 1) >> 1, W1 = (W0 + 1) >> 1;
  const int H2 = (H1 + 1) >> 1, W2 = (W1 + 1) >> 1;
  const int TNI = a.tni;
  const int ngroups = (a.N + TNI - 1) / TNI;
  long wnext[kWFrag];
  wfetch8(a.w8[0], tail_cin(0), tail_cout(0), wnext);
#define TAIL8(l, CI, CO, MODE, IN, H_, W_, OUT, CP)                                    \
  do {                                                                               \
    long wc[kWFrag];                                                                 \
    _Pragma("unroll") for (int k = 0; k < kWFrag; ++k) wc[k] = wnext[k];             \
    const int ln = ((l) + 1) % 14;                                                   \
    wfetch8(a.w8[ln], tail_cin(ln), tail_cout(ln), wnext);                           \
    conv_lds<CI, CO, false, MODE, false, true>(IN, H_, W_, nimg, 0, nullptr, 0, a.b[l], \
                                               OUT, wc, a.ws[l], oF, CP);            \
  } while (0)
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * TNI, nimg = min(TNI, a.N - img0);
    // ---- stage 0: X0 <- input (A), F <- fp8(relu(X0)); halos of A / U0 (B) / F
    load_input<true>(a, img0, nimg, A, F);
    zero_halo<TG<16>::PIXB>(A, nimg, H0, W0);
    zero_halo<TG<16>::PIXB8>(B, nimg, H0, W0);
    zero_halo<TG<16>::PIXB8>(F, nimg, H0, W0);
    __syncthreads();
#pragma unroll 1
    for (int rb = 0; rb < 2; ++rb) {
      TAIL8(2 * rb, 16, 16, OUT_TILE_RELU, oF, H0, W0, oB, 0);
      __syncthreads();
      TAIL8(2 * rb + 1, 16, 16, OUT_TILE_ADD, oB, H0, W0, oA, rb == 0 ? 1 : 2);
      __syncthreads();
    }
    // ---- stage 1: conv 16->32 (staging in A: X0 is dead) -> pool -> X1 (B) + F
    TAIL8(4, 16, 32, OUT_STAGE, oF, H0, W0, oA, 0);
    __syncthreads();
    pool_lds<32, true>((const bf16*)A, H0, W0, nimg, B, F);
    zero_halo<TG<32>::PIXB>(B, nimg, H1, W1);
    zero_halo<TG<32>::PIXB8>(F, nimg, H1, W1);
    __syncthreads();
    zero_halo<TG<32>::PIXB8>(A, nimg, H1, W1);  // U1 layout (staging consumed)
#pragma unroll 1
    for (int rb = 0; rb < 2; ++rb) {
      TAIL8(5 + 2 * rb, 32, 32, OUT_TILE_RELU, oF, H1, W1, oA, 0);
      __syncthreads();
      TAIL8(6 + 2 * rb, 32, 32, OUT_TILE_ADD, oA, H1, W1, oB, rb == 0 ? 1 : 2);
      __syncthreads();
    }
    // ---- stage 2 (X1 in B is dead once F holds its copy)
    TAIL8(9, 32, 32, OUT_STAGE, oF, H1, W1, oA, 0);
    __syncthreads();
    pool_lds<32, true>((const bf16*)A, H1, W1, nimg, B, F);
    zero_halo<TG<32>::PIXB>(B, nimg, H2, W2);
    zero_halo<TG<32>::PIXB8>(F, nimg, H2, W2);
    __syncthreads();
    zero_halo<TG<32>::PIXB8>(A, nimg, H2, W2);
#pragma unroll 1
    for (int rb = 0; rb < 2; ++rb) {
      TAIL8(10 + 2 * rb, 32, 32, OUT_TILE_RELU, oF, H2, W2, oA, 0);
      __syncthreads();
      TAIL8(11 + 2 * rb, 32, 32, OUT_TILE_ADD, oA, H2, W2, oB, rb == 0 ? 1 : 0);
      __syncthreads();
    }
#undef TAIL8
    store_output(a, img0, nimg, H2, W2, B);
    __syncthreads();
  }
}

// ------------------------------------------------------------------ fused acting step, launch A
// Everything of a policy step up to the sparse head in ONE launch (reference model.py:152-160,
// 205, 219-220, on the engine's compact codes instead of float planes). Per tile of TNI envs a
// workgroup
//   P1  reads the envs' 16-bit cell codes + resources (device or pinned host) into LDS;
//   P2  decodes them (one wave per env, 4 consecutive cells per lane: obs_mask.hip's maths) into
//       the obs bit planes and the 78-bit masks, stored straight into the rollout row (and the
//       previous slot's bootstrap row), lists the active (env, cell) pairs in LDS, zeroes the
//       env's action row and per-cell step scratch and sets its pending-cell count;
//   P3  reserves each active cell's bucket range with one global atomic per (tile, cell) and runs
//       the stage-0 conv (conv0_row_kernel's maths: bit planes through an LDS byte table, the
//       kx = 0 / 2 taps by DPP) with its 3x3/2 max-pool in registers (vertical max over the row
//       pair and the previous row, horizontal max by DPP row shifts with -inf fill), writing the
//       pooled 8x8x16 map into the X0 tile, so the stage-0 output never leaves LDS;
// then the 14 trunk convs + network.5 + critic exactly as trunk_tail_kernel<false, true>. The
// prologue's scratch lives in region R2, which stage 0 needs only from its first conv on.
struct ActTrunkArgs {
  TrunkArgs t;  // layers 1..14 and the fused head: f_out = feat, v_out = the rollout row's values
  const bf16* w0;  // stage-0 conv, packed [16][9][32]
  const float* b0;
  const uint16_t* codes;
  const int32_t* res;
  const uint32_t* code_list;  // sparse input rows (mbk_api.h MbkActStep), or null
  uint32_t* abits;             // optional active-cell bitmap rows [E][S / 32] (+ obs2 copy)
  uint32_t* abits2;
  uint32_t* act_list;         // sparse action rows: A writes n = 0 for envs with nothing to act
  int list_stride;
  uint32_t* obs;
  uint32_t* mask;
  uint32_t* obs2;
  uint32_t* mask2;
  uint8_t* action;
  float* logp;
  uint16_t* act16;
  int* pending;  // [2E]: pending active cells, then the env's active-cell total
  int* bucket_cnt;  // this step's half of the [2][S] counters
  int* bucket_cnt_prev;  // the previous step's half: zeroed by workgroup 0
  int* bucket;
  uint64_t* cellx;  // launch B's per-env granule rows; the wave-owned kernel spills lists there
  const float* reward_src;
  const uint8_t* done_src;
  float* reward_dst;
  uint8_t* done_dst;
  uint64_t* stamps;  // diagnostic phase stamps (null: off)
};

constexpr int kActS = 256;  // 16x16 maps: one map row = one 16-pixel MFMA block

// The env's active-cell bitmap row from its decode (lane l holds cells 4l .. 4l + 3, mk: their
// mask words): word w = cells 32 w .. 32 w + 31 = lanes 8 w .. 8 w + 7, bit 4 i + q = lane
// 8 w + i's cell q. Four ballots, then lanes 0..7 spread their byte of each to every 4th bit.
__device__ __forceinline__ uint32_t spread4(uint32_t x) {  // bit i -> bit 4 i (8 bits)
  x &= 0xFFu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return (x | (x << 3)) & 0x11111111u;
}
__device__ __forceinline__ void write_abits(const uint32_t mk[12], int lane, uint32_t* row,
                                            uint32_t* row2) {
  uint32_t w = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t b = __ballot((mk[3 * q] | mk[3 * q + 1] | mk[3 * q + 2]) != 0u);
    w |= spread4((uint32_t)(b >> (8 * (lane & 7)))) << q;
  }
  if (lane < 8) {
    row[lane] = w;
    if (row2) row2[lane] = w;
  }
}
// words of a sparse input row read in the first access (count + 31 entries: most envs); the
// rest only for envs with more occupied cells
constexpr int kActSpec = 32;
__device__ __forceinline__ float bf16_round(float v) { return lo_f(pack2(v, 0.f)); }

// stage-0 conv of one 16x16 image (bit planes [256] u32 in LDS) + max_pool2d(3, 2, 1), into the
// interior of the halo'd X0 tile at x0 (image im). A wave owns the image; lane (g, li) = column
// li, channels 4g .. 4g+3. MFMA order per output row = conv0_row_kernel's, values rounded to
// bf16 before the pool as it pools the bf16 staging tile, so the pooled map is bit-identical.
__device__ __forceinline__ void act_conv0(const uint32_t* bits_img, const char* lut,
                                          const Frag8 bw[9], const float bias[4], char* x0,
                                          int im) {
  constexpr int H0 = 8, W0 = 8, PX = TG<16>::PIXB;
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // opaque: no address hoisted out of the caller's tile loop
  const int g = lane >> 4, li = lane & 15;
  const int sh = 8 * g;
  struct R3 {
    uint32_t l, c, h;
  };
  auto row = [&](uint32_t b) {  // LUT offsets of pixels x-1, x, x+1 (this lane's plane byte)
    R3 r;  // one v_bfe_u32 per byte, as conv0_row_kernel
    r.c = __builtin_amdgcn_ubfe(b, (uint32_t)sh, 8u) * 16u;
    r.l = __builtin_amdgcn_ubfe(mbk::dpp_shr1_zero(b), (uint32_t)sh, 8u) * 16u;
    r.h = __builtin_amdgcn_ubfe(mbk::dpp_shl1_zero(b), (uint32_t)sh, 8u) * 16u;
    return r;
  };
  uint32_t rows[16];
#pragma unroll
  for (int y = 0; y < 16; ++y) rows[y] = bits_img[y * 16 + li];
  const R3 zero3 = {0u, 0u, 0u};  // LUT entry 0 = all-zero planes
  R3 r[4];
  r[0] = zero3;
  r[1] = row(rows[0]);
  r[2] = row(rows[1]);
  r[3] = row(rows[2]);
  float prev[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};  // conv row y-1
#pragma unroll
  for (int y = 0; y < 16; y += 2) {
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        Frag8 f;
        f.u = *(const uint4*)(lut + (kx == 0 ? r[q].l : kx == 1 ? r[q].c : r[q].h));
        if (q < 3) acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[3 * q + kx].v, f.v, acc0, 0, 0, 0);
        if (q > 0) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[3 * (q - 1) + kx].v, f.v, acc1, 0, 0, 0);
      }
    }
    float hm[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float o0 = bf16_round(acc0[i] + bias[i]), o1 = bf16_round(acc1[i] + bias[i]);
      const float vm = fmaxf(fmaxf(prev[i], o0), o1);  // pooled row y/2: conv rows y-1 .. y+1
      prev[i] = o1;
      hm[i] = fmaxf(fmaxf(mbk::dpp_shr1_ninf(vm), vm), mbk::dpp_shl1_ninf(vm));
    }
    if ((li & 1) == 0) {
      const int oy = y >> 1, ox = li >> 1;
      *(uint2*)(x0 + ((im * (H0 + 2) + oy + 1) * (W0 + 2) + ox + 1) * PX + 8 * g) =
          make_uint2(pack2(hm[0], hm[1]), pack2(hm[2], hm[3]));
    }
    r[0] = r[2];
    r[1] = r[3];
    r[2] = y + 3 < 16 ? row(rows[(y + 3) % 16]) : zero3;
    r[3] = y + 4 < 16 ? row(rows[(y + 4) % 16]) : zero3;
  }
}

// diagnostic phase stamps (a.stamps != null, tools/act_phases.py): wave 0 of each workgroup
// records the 100 MHz real-time counter at the phase boundaries of its first tile; the
// stamped run's total is not a timing (the stamps serialise nothing, but read their shares)
#define ACT_STAMP(k)                                                                     \
  do {                                                                                   \
    if (a.stamps && grp == (int)blockIdx.x && threadIdx.x < 64)                          \
      a.stamps[(size_t)blockIdx.x * 64 * kActStamps + (k) * 64 + threadIdx.x] =           \
          __builtin_amdgcn_s_memrealtime();                                              \
  } while (0)
constexpr int kActStamps = 21;

// ------------------------------------------------------------------ launch A, wave-owned tiles
// The acting trunk with the tile split by WAVE instead of by phase: wave w owns envs
// 2w, 2w+1 of the 8-env tile (4 waves, 80 KB of LDS: two workgroups per CU, round 6) from
// their sparse rows to their trunk output -- codes, decode,
// stage-0 conv + pool, the 14 convs (conv_lds WV = 1 / 2 over its own images), the pools and
// the halo zeroing -- in its own slices of the two regions, so the trunk needs no workgroup
// barrier at all (LDS is in order within a wave). The phase-split form ran ~25 workgroup-wide
// phases per tile with 2 waves per SIMD: every phase waited for its slowest wave, the 2x2 stage
// had 4 pixel blocks for 8 waves, and no tile's prologue overlapped another's convs
// (profiles/33: 52 % of wave cycles waiting, MFMA 9.7 %).
//
// Tile-wide, behind two barriers at the tile's end: the bucket reservation (one global atomic
// per (tile, cell), as before) and network.5 + critic. Decode appends each active pair to the
// tile's LDS list (LDS atomics for its index and its slot among the tile's pairs of that
// cell); list, counters and count are double-buffered by tile parity, so the next tile's decode
// never waits for the bucket writes; a tile with more than kWList pairs spills the rest into
// its envs' cellx rows (launch B writes those rows only later). The FC gives each wave four
// hidden blocks of all 8 images (its W5 fragments are loaded before the first barrier), the
// critic partials meet in LDS (mbk::crit_block / crit_sum: every FC kernel's order).
// Round 6 halved the tile (16 envs / 8 waves / 157 KB -> 8 envs / 4 waves / 80 KB): a
// workgroup's tile-end barrier now waits for 4 waves, not 8, while the CU's other workgroup
// keeps issuing, and under the learner a workgroup fits beside a learner workgroup of up to
// 80 KB. Isolated 170 -> 177 us per 8192-env step (twice the per-tile FC and bucket work), but
// 4 of 4 seed-paired bench runs faster (16.35 -> 16.91 M frames/s mean on one box).
//
// Memory order per wave and tile (vmcnt counts loads and stores in issue order): the stage-0
// weights, this tile's rows (first tile only), reward / done, then the NEXT tile's rows from
// pinned host memory right away, so their PCIe latency has the decode and stage-0 conv to
// hide behind before the first weight wait that orders after them.
constexpr int kWNW = 4;                                      // waves per workgroup
constexpr int kWThreads = 64 * kWNW;
constexpr int kWEnv = 2;                                     // envs (images) per wave
constexpr int kWTni = kWNW * kWEnv;                          // envs per tile
constexpr int kWImgB = 10 * 10 * TG<16>::PIXB;               // largest per-image footprint (X0)
constexpr int kWSlice = kWEnv * kWImgB;                      // a wave's slice of R1 / R2
constexpr int kWRegion = kWNW * kWSlice;                     // R1 = R2 = 38400 bytes
constexpr int kWCnt = 2 * kWRegion;                          // [2][256] pair counts per cell
constexpr int kWNp = kWCnt + 2 * kActS * 4;                  // [2] list lengths (+ pad)
constexpr int kWVred = kWNp + 16;                            // [16 blocks][8 images] critic
constexpr int kWList = 136;                                  // list entries per parity in LDS
constexpr int kWLst = kWVred + 16 * kWTni * 4;               // [2][kWList] packed pairs
constexpr int kWSmem = kWLst + 2 * kWList * 4;
// two workgroups per CU (160 KB): one workgroup's tile-end barrier wait and FC run beside the
// other's convs, and a learner workgroup of up to 80 KB can share the CU with one of them
// (round 5's 16-env workgroups took 157 KB: a whole CU)
static_assert(2 * kWSmem <= 160 * 1024, "two wave-owned acting workgroups per CU");
static_assert(8 * 8 * 32 * 2 <= kWImgB && 6 * 6 * TG<32>::PIXB <= kWImgB, "stage footprints");
// a wave's decode scratch inside its R2 slice (dead once its stage-0 conv has run) with the
// wave's own copy of the stage-0 byte -> 8 bf16 table behind it (written before each tile's
// stage-0 conv: 4 LDS stores per lane, instead of a workgroup-wide 4 KB that no longer fits),
// and the compacted decode's mask rows + own-idle-unit list inside its R1 slice (dead once the
// stage-0 conv writes X0 there)
constexpr int kWCodes = 0, kWBits = kWEnv * kActS * 2;
constexpr int kWLut = kWBits + kWEnv * kActS * 4;
static_assert(kWLut + 256 * 16 <= kWSlice, "decode scratch + LUT");
constexpr int kWMask = 0, kWList16 = kWEnv * kActS * 12;
static_assert(kWList16 + kWEnv * kActS * 2 <= kWSlice, "decode mask scratch");

// network.5 + critic of the tile: wave w computes hidden blocks 4w .. 4w+3 (wf: their W5
// fragments, loaded before the barrier) for the tile's 8 images, whose X2 tiles sit in the
// waves' R1 slices (image i: wave i / 2's slice, its image i % 2); critic partials -> vred
// [hidden block][image] (mbk::crit_sum then adds the blocks in hidden order, as every FC)
__device__ __forceinline__ void tile_fc(int nimg, int img0, const TrunkArgs& a,
                                        const uint4 wf[4][4], float* vred) {
  constexpr int H2 = 2, W2 = 2, PX = TG<32>::PIXB, NKS = H2 * W2;
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // opaque: no address hoisted out of the tile loop
  const int wave = threadIdx.x >> 6;
  const int G = lane >> 4, li = lane & 15;
  const bool valid = li < nimg;
  const int x2 = ((li >> 1) & (kWNW - 1)) * kWSlice + (li & 1) * (H2 + 2) * (W2 + 2) * PX;
  Frag8 b[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int py = ks / W2, px = ks - py * W2;
    b[ks].u = valid ? relu8(*(const uint4*)(trunk_smem + x2 + ((py + 1) * (W2 + 2) + px + 1) * PX +
                                            G * 16))
                    : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int hb = 4 * wave + jj;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      Frag8 w;
      w.u = wf[jj][ks];
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.v, b[ks].v, acc, 0, 0, 0);
    }
    const int h0 = hb * 16 + 4 * G;
    float hv[4], w4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hv[i] = __bfloat162float(__float2bfloat16(fmaxf(acc[i] + a.b5[h0 + i], 0.f)));
      w4[i] = a.wc[h0 + i];
    }
    const float q = mbk::crit_block(hv, w4);
    if (G == 0 && li < kWTni) vred[hb * kWTni + li] = q;
    uint32_t o[2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      o[k] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k])) |
             ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k + 1])) << 16);
    if (valid) *(uint2*)(a.f_out + (size_t)(img0 + li) * 256 + h0) = make_uint2(o[0], o[1]);
  }
}

__device__ __forceinline__ void act_trunk_w_kernel_body(const ActTrunkArgs& a) {
  const TrunkArgs& t = a.t;
  constexpr int S = kActS, H0 = 8, W0 = 8, H1 = 4, W1 = 4, H2 = 2, W2 = 2;
  constexpr int NW = kWNW, TNI = kWTni;
  const int E = t.N;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int oR1 = wave * kWSlice, oR2 = kWRegion + wave * kWSlice;  // this wave's slices
  char* R1 = trunk_smem + oR1;
  char* R2 = trunk_smem + oR2;
  const char* lut = R2 + kWLut;  // this wave's copy (rewritten before each stage-0 conv)
  uint16_t* lcodes = (uint16_t*)(R2 + kWCodes);
  uint32_t* lbits = (uint32_t*)(R2 + kWBits);
  float* vred = (float*)(trunk_smem + kWVred);
  const int ngroups = (E + TNI - 1) / TNI;
  const bool pl = lane < kActSpec && lane <= S;  // lanes that read a row's first words
  // once per launch: both parities' tile counters, the previous step's bucket half
  for (int c = tid; c < 2 * S; c += kWThreads) ((int*)(trunk_smem + kWCnt))[c] = 0;
  if (tid < 2) ((int*)(trunk_smem + kWNp))[tid] = 0;
  if (blockIdx.x == 0) {
    // the previous step's launch B is done with these
    for (int c = tid; c < S; c += kWThreads) a.bucket_cnt_prev[c] = 0;
  }
  mbk::lds_barrier();
  uint32_t pre0 = 0u, pre1 = 0u;  // this wave's rows (first words) for the current tile
  if (a.code_list && (int)blockIdx.x < ngroups) {
    const int en = blockIdx.x * TNI + wave * kWEnv;
    pre0 = (en < E && pl) ? a.code_list[(size_t)en * a.list_stride + lane] : 0u;
    pre1 = (en + 1 < E && pl) ? a.code_list[(size_t)(en + 1) * a.list_stride + lane] : 0u;
  }
  // conv layer l: its weight fragments are loaded at its start (a one-layer-ahead register
  // prefetch as in act_trunk_kernel needs 72 more VGPRs and spills here); each MFMA waits only
  // for its own fragment, so the loads stream behind the first pixel blocks' MFMAs
#define ACT_WPHASE(l, CI, CO, RELU, MODE, NBLK, IN, H_, W_, OUT)                          \
  do {                                                                                   \
    uint4 wc[kWFrag];                                                                    \
    wfetch(t.w[l], CI, CO, wc);                                                          \
    conv_w<CI, CO, RELU, MODE, (NBLK) < 4 ? (NBLK) : 4, (NBLK) < 4 ? 1 : (NBLK) / 4>(     \
        IN, H_, W_, nw * (H_) * (W_), wc, t.b[l], OUT);                                  \
    __builtin_amdgcn_wave_barrier();                                                     \
    ACT_STAMP(4 + (l));                                                                  \
  } while (0)
  int k = 0;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x, ++k) {
    const int par = k & 1;
    int* lcnt = (int*)(trunk_smem + kWCnt) + par * S;
    int* np = (int*)(trunk_smem + kWNp) + par;
    uint32_t* lst = (uint32_t*)(trunk_smem + kWLst) + par * kWList;
    const int img0 = grp * TNI, nimg = min(TNI, E - img0);
    const int e0 = wave * kWEnv;                   // this wave's first env within the tile
    const int nw = max(0, min(kWEnv, nimg - e0));  // ... and how many it has
    uint32_t* ovf = (uint32_t*)(a.cellx + (size_t)img0 * S);  // list spill (this tile's rows)
    bool spilled = false;
    uint4 wf[4][4];  // this wave's four W5 hidden blocks for the tile's FC
    if (nw > 0) {
      // stage-0 conv weights / bias first: their L2 latency hides behind the rows and decode
      Frag8 bw0[9];
      {
        const uint4* wp = (const uint4*)(a.w0 + (size_t)li * 9 * 32 + g * 8);
#pragma unroll
        for (int c = 0; c < 9; ++c) bw0[c].u = wp[c * 4];
      }
      float bias0[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bias0[i] = a.b0[4 * g + i];
      ACT_STAMP(0);
      // ---- loads first: reward / done of the last env step (lane j: env j), the next tile's
      // rows; then this tile's codes into the wave's LDS code rows
      float rwv = 0.f;
      uint8_t dnv = 0;
      if (lane < nw) {
        if (a.reward_dst) rwv = a.reward_src[img0 + e0 + lane];
        if (a.done_dst) dnv = a.done_src[img0 + e0 + lane];
      }
      const uint32_t cur0 = pre0, cur1 = pre1;
      if (a.code_list) {
        const int en = img0 + gridDim.x * TNI + e0;
        pre0 = (en < E && pl) ? a.code_list[(size_t)en * a.list_stride + lane] : 0u;
        pre1 = (en + 1 < E && pl) ? a.code_list[(size_t)(en + 1) * a.list_stride + lane] : 0u;
      }
      int res0 = 0, res1 = 0;  // (kWEnv = 2: named, so a rolled loop keeps them in registers)
#pragma unroll 1
      for (int j = 0; j < nw; ++j) {
        const int el = e0 + j;
        uint16_t* cs = lcodes + j * S;
        if (a.code_list) {
          for (int c = lane * 4; c < S; c += 256) *(uint2*)(cs + c) = make_uint2(0u, 0u);
          const uint32_t* row = a.code_list + (size_t)(img0 + el) * a.list_stride;
          const uint32_t w = j ? cur1 : cur0;
          const uint32_t w0 = (uint32_t)__shfl((int)w, 0, 64);
          const int n = min((int)(w0 & 0xFFFFu), S);
          (j ? res1 : res0) = (int)(w0 >> 16);
          __builtin_amdgcn_wave_barrier();
          if (lane >= 1 && lane < kActSpec && lane <= n && (w & 0xFFFFu) < (uint32_t)S)
            cs[w & 0xFFFFu] = (uint16_t)(w >> 16);
          for (int q = kActSpec + lane; q <= n; q += 64) {
            const uint32_t x = row[q];
            if ((x & 0xFFFFu) < (uint32_t)S) cs[x & 0xFFFFu] = (uint16_t)(x >> 16);
          }
        } else {
          ((uint4*)cs)[lane & 31] = ((const uint4*)(a.codes + (size_t)(img0 + el) * S))[lane & 31];
          (j ? res1 : res0) = a.res[img0 + el];
        }
      }
      __builtin_amdgcn_wave_barrier();
      ACT_STAMP(1);
      // ---- decode (act_trunk_kernel P2), compacted: only an own idle unit's cell has a non-zero
      // mask (cell_mask returns zero words for every other cell, and an own idle unit always
      // gets its NOOP bit), so pass 1 lists the wave's own idle units (both envs) and pass 2
      // runs the mask rules once per listed cell, one cell per lane, into the LDS mask rows.
      // (Round 5 ran cell_mask on all 4 cells of every lane per env: the wave executed the rule
      // path for every q slot in which any lane had an idle unit -- ~3 of 4 per env.)
      const int c0 = lane * 4;
      uint32_t* lmk = (uint32_t*)(R1 + kWMask);       // [kWEnv][S][3] mask words (R1: free
      uint16_t* llist = (uint16_t*)(R1 + kWList16);   // until the stage-0 conv) + the list
      uint32_t actq = 0u;  // bit 4 j + q: cell c0 + q of env j holds an own idle unit
      int kxj[kWEnv], nj[kWEnv];
#pragma unroll
      for (int j = 0; j < kWEnv; ++j) {
        kxj[j] = nj[j] = 0;
        if (j >= nw) break;
        const uint16_t* cs = lcodes + j * S;
        int nact = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint16_t code = cs[c0 + q];
          const int t = mbr::code_type(code);
          const bool idle = mbr::code_owner(code) == 1 && mbr::code_act(code) == mbr::A_NOOP &&
                            t != mbr::RESOURCE && t != mbr::NONE;
          actq |= (uint32_t)idle << (4 * j + q);
          nact += idle;
        }
        uint4* mz = (uint4*)(lmk + (j * S + c0) * 3);
        mz[0] = mz[1] = mz[2] = make_uint4(0u, 0u, 0u, 0u);
        int kx = nact;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(kx, o, 64);
          if (lane >= o) kx += y;
        }
        nj[j] = __shfl(kx, 63, 64);
        kxj[j] = kx - nact;
      }
      {  // the list: env 0's cells, then env 1's, each in cell order
        int pos = kxj[0];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if ((actq >> q) & 1u) llist[pos++] = (uint16_t)(c0 + q);
        pos = nj[0] + kxj[1];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if ((actq >> (4 + q)) & 1u) llist[pos++] = (uint16_t)(S | (c0 + q));
      }
      __builtin_amdgcn_wave_barrier();
      for (int i = lane; i < nj[0] + nj[1]; i += 64) {  // pass 2: the rules, one cell per lane
        const int en = llist[i], j = en >> 8, c = en & (S - 1);
        uint32_t w3[3];
        mbk::cell_mask(lcodes + j * S, c, 16, 16, j ? res1 : res0, w3);
        uint32_t* d = lmk + (j * S + c) * 3;
        d[0] = w3[0];
        d[1] = w3[1];
        d[2] = w3[2];
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll 1
      for (int j = 0; j < nw; ++j) {
        const int el = e0 + j, e = img0 + el;
        const uint16_t* cs = lcodes + j * S;
        uint32_t ob[4], mk[12];
        {
          const uint4* ms = (const uint4*)(lmk + (j * S + c0) * 3);
          const uint4 u0 = ms[0], u1 = ms[1], u2 = ms[2];
          mk[0] = u0.x; mk[1] = u0.y; mk[2] = u0.z; mk[3] = u0.w;
          mk[4] = u1.x; mk[5] = u1.y; mk[6] = u1.z; mk[7] = u1.w;
          mk[8] = u2.x; mk[9] = u2.y; mk[10] = u2.z; mk[11] = u2.w;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) ob[q] = mbr::code_bits(cs[c0 + q]);
        const int n = j ? nj[1] : nj[0];
        int kx = j ? kxj[1] : kxj[0];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if ((actq >> (4 * j + q)) & 1u) {
            const int c = c0 + q;
            const int i = atomicAdd(np, 1);
            const int slot = atomicAdd(&lcnt[c], 1);
            const uint32_t en = (uint32_t)c | ((uint32_t)slot << 8) | ((uint32_t)el << 12) |
                                ((uint32_t)kx << 16);
            if (i < kWList) {
              lst[i] = en;
            } else {
              ovf[i - kWList] = en;
              spilled = true;
            }
            ++kx;
          }
        }
        const uint4 o4 = make_uint4(ob[0], ob[1], ob[2], ob[3]);
        const uint4 m0 = make_uint4(mk[0], mk[1], mk[2], mk[3]);
        const uint4 m1 = make_uint4(mk[4], mk[5], mk[6], mk[7]);
        const uint4 m2 = make_uint4(mk[8], mk[9], mk[10], mk[11]);
        *(uint4*)(lbits + j * S + c0) = o4;
        if (a.abits) write_abits(mk, lane, a.abits + (size_t)e * (S / 32),
                                 a.abits2 ? a.abits2 + (size_t)e * (S / 32) : nullptr);
        const size_t eo = (size_t)e * S + c0;
        *(uint4*)(a.obs + eo) = o4;
        uint4* mp = (uint4*)(a.mask + eo * 3);
        mp[0] = m0;
        mp[1] = m1;
        mp[2] = m2;
        if (a.obs2) {
          *(uint4*)(a.obs2 + eo) = o4;
          uint4* mp2 = (uint4*)(a.mask2 + eo * 3);
          mp2[0] = m0;
          mp2[1] = m1;
          mp2[2] = m2;
        }
        const uint4 z4 = make_uint4(0, 0, 0, 0);
        uint4* act4 = (uint4*)(a.action + (size_t)e * S * 7);
        for (int i = lane; i < S * 7 / 16; i += 64) act4[i] = z4;
        if (lane == 0) {
          a.pending[e] = n;
          a.pending[E + e] = n;
          if (n == 0) a.logp[e] = 0.f;
        }
        if (a.act_list) {
          if (n == 0 && lane == 0) a.act_list[(size_t)e * a.list_stride] = 0u;
        } else {
          *(uint2*)(a.act16 + eo) = make_uint2(0u, 0u);
        }
      }
      if (lane < nw) {
        if (a.reward_dst) a.reward_dst[img0 + e0 + lane] = rwv;
        if (a.done_dst) a.done_dst[img0 + e0 + lane] = dnv;
      }
      __builtin_amdgcn_wave_barrier();
      ACT_STAMP(2);
      // ---- stage-0 conv + pool of the wave's images into its X0 slice
      for (int i = lane; i < 256; i += 64)  // this wave's byte -> 8 bf16 table
        ((uint4*)(R2 + kWLut))[i] = mbk::bits8_bf16((uint32_t)i);
      zero_halo<TG<16>::PIXB, true>(R1, nw, H0, W0);
      for (int j = 0; j < nw; ++j) act_conv0(lbits + j * S, lut, bw0, bias0, R1, j);
      __builtin_amdgcn_wave_barrier();
      zero_halo<TG<16>::PIXB, true>(R2, nw, H0, W0);  // U0 layout (decode scratch is dead)
      __builtin_amdgcn_wave_barrier();
      ACT_STAMP(3);
      // ---- stage 0 residual blocks, stages 1 and 2 on the wave's own images
#pragma unroll 1
      for (int rb = 0; rb < 2; ++rb) {
        ACT_WPHASE(2 * rb, 16, 16, true, OUT_TILE_RELU, 8, oR1, H0, W0, oR2);
        ACT_WPHASE(2 * rb + 1, 16, 16, false, OUT_TILE_ADD, 8, oR2, H0, W0, oR1);
      }
      ACT_WPHASE(4, 16, 32, false, OUT_STAGE, 8, oR1, H0, W0, oR2);
      pool_lds<32, false, true>((const bf16*)R2, H0, W0, nw, R1);
      zero_halo<TG<32>::PIXB, true>(R1, nw, H1, W1);
      zero_halo<TG<32>::PIXB, true>(R2, nw, H1, W1);
      __builtin_amdgcn_wave_barrier();
#pragma unroll 1
      for (int rb = 0; rb < 2; ++rb) {
        ACT_WPHASE(5 + 2 * rb, 32, 32, true, OUT_TILE_RELU, 2, oR1, H1, W1, oR2);
        ACT_WPHASE(6 + 2 * rb, 32, 32, false, OUT_TILE_ADD, 2, oR2, H1, W1, oR1);
      }
      ACT_WPHASE(9, 32, 32, false, OUT_STAGE, 2, oR1, H1, W1, oR2);
      pool_lds<32, false, true>((const bf16*)R2, H1, W1, nw, R1);
      zero_halo<TG<32>::PIXB, true>(R1, nw, H2, W2);
      zero_halo<TG<32>::PIXB, true>(R2, nw, H2, W2);
      __builtin_amdgcn_wave_barrier();
#pragma unroll 1
      for (int rb = 0; rb < 2; ++rb) {
        ACT_WPHASE(10 + 2 * rb, 32, 32, true, OUT_TILE_RELU, 1, oR1, H2, W2, oR2);
        ACT_WPHASE(11 + 2 * rb, 32, 32, false, OUT_TILE_ADD, 1, oR2, H2, W2, oR1);
      }
      ACT_STAMP(18);
    }
    // ---- tile end: W5 fragments in flight across the barrier
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const uint4* wrow = (const uint4*)(t.w5 + (size_t)((4 * wave + jj) * 16 + li) * (H2 * W2 * 32)) + g;
#pragma unroll
      for (int ks = 0; ks < H2 * W2; ++ks) wf[jj][ks] = wrow[ks * 4];
    }
    // spill rows in L2 first
    if (spilled) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mbk::lds_barrier();
    ACT_STAMP(19);
    for (int c = tid; c < S; c += kWThreads) {
      const int n = lcnt[c];
      if (n > 0) lcnt[c] = atomicAdd(&a.bucket_cnt[c], n);
    }
    {  // the other parity (the previous tile's, consumed before this barrier) for the next tile
      int* lc2 = (int*)(trunk_smem + kWCnt) + (par ^ 1) * S;
      for (int c = tid; c < S; c += kWThreads) lc2[c] = 0;
      if (tid == 0) ((int*)(trunk_smem + kWNp))[par ^ 1] = 0;
    }
    const int npr = *np;
    tile_fc(nimg, img0, t, wf, vred);
    mbk::lds_barrier();
    if (tid < nimg) a.t.v_out[img0 + tid] = mbk::crit_sum(vred + tid, 16, kWTni, t.bc[0]);
    for (int i = tid; i < npr; i += kWThreads) {
      const uint32_t en = i < kWList ? lst[i]
                                     : __hip_atomic_load(ovf + (i - kWList), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
      const int c = (int)(en & 0xFFu), slot = (int)((en >> 8) & 0xFu);
      const int el = (int)((en >> 12) & 0xFu), rank = (int)(en >> 16);
      a.bucket[(size_t)c * E + lcnt[c] + slot] = (img0 + el) | (rank << 16);
    }
    ACT_STAMP(20);
  }
#undef ACT_WPHASE
}
// thin wrapper: the body takes the arguments by const reference (conv0_row_kernel, profile 43)
__global__ __launch_bounds__(kWThreads, 2) void act_trunk_w_kernel(ActTrunkArgs a) {
  act_trunk_w_kernel_body(a);
}

size_t region_bytes(int H0, int W0, int TNI) {
  const int H1 = (H0 + 1) / 2, W1 = (W0 + 1) / 2, H2 = (H1 + 1) / 2, W2 = (W1 + 1) / 2;
  size_t r = (size_t)TNI * (H0 + 2) * (W0 + 2) * TG<16>::PIXB;                 // X0 / U0
  r = std::max(r, (size_t)TNI * H0 * W0 * 32 * 2);                            // stage-1 staging
  r = std::max(r, (size_t)TNI * (H1 + 2) * (W1 + 2) * TG<32>::PIXB);          // X1 / U1
  r = std::max(r, (size_t)TNI * (H2 + 2) * (W2 + 2) * TG<32>::PIXB);          // X2 / U2
  return (r + 15) & ~(size_t)15;
}
// fp8 trunk regions (see trunk_tail8_kernel): A, B and the fp8 conv-input tile F
size_t trunk8_region_a(int H0, int W0, int TNI) {
  const int H1 = (H0 + 1) / 2, W1 = (W0 + 1) / 2, H2 = (H1 + 1) / 2, W2 = (W1 + 1) / 2;
  size_t r = (size_t)TNI * (H0 + 2) * (W0 + 2) * TG<16>::PIXB;          // X0
  r = std::max(r, (size_t)TNI * H0 * W0 * 32 * 2);                     // stage-1 staging
  r = std::max(r, (size_t)TNI * (H1 + 2) * (W1 + 2) * TG<32>::PIXB8);  // U1
  r = std::max(r, (size_t)TNI * H1 * W1 * 32 * 2);                     // stage-2 staging
  r = std::max(r, (size_t)TNI * (H2 + 2) * (W2 + 2) * TG<32>::PIXB8);  // U2
  return (r + 15) & ~(size_t)15;
}
size_t trunk8_region_b(int H0, int W0, int TNI) {
  const int H1 = (H0 + 1) / 2, W1 = (W0 + 1) / 2, H2 = (H1 + 1) / 2, W2 = (W1 + 1) / 2;
  size_t r = (size_t)TNI * (H0 + 2) * (W0 + 2) * TG<16>::PIXB8;         // U0
  r = std::max(r, (size_t)TNI * (H1 + 2) * (W1 + 2) * TG<32>::PIXB);   // X1
  r = std::max(r, (size_t)TNI * (H2 + 2) * (W2 + 2) * TG<32>::PIXB);   // X2
  return (r + 15) & ~(size_t)15;
}
size_t trunk8_region_f(int H0, int W0, int TNI) {
  const int H1 = (H0 + 1) / 2, W1 = (W0 + 1) / 2;
  size_t r = (size_t)TNI * (H0 + 2) * (W0 + 2) * TG<16>::PIXB8;
  r = std::max(r, (size_t)TNI * (H1 + 2) * (W1 + 2) * TG<32>::PIXB8);
  return (r + 15) & ~(size_t)15;
}
size_t trunk_smem_bytes(int H0, int W0, int TNI, size_t wb, bool f8) {
  if (f8)
    return trunk8_region_a(H0, W0, TNI) + trunk8_region_b(H0, W0, TNI) +
           trunk8_region_f(H0, W0, TNI);
  return 2 * region_bytes(H0, W0, TNI) + wb;
}

}  // namespace

static int trunk_launch(TrunkArgs a, int N, int H0, int W0, hipStream_t stream);

// x: stage-0 pooled activations [N][H0][W0][16] bf16; w/b: layers 1..14 of the
// (16, 32, 32) IMPALA trunk (packed fwd weights, fp32 biases); y: [N][H2][W2][32] bf16.
extern "C" int mbk_trunk_tail(const void* x, const void* const* w, const float* const* b, int N,
                              int H0, int W0, void* y, hipStream_t stream) {
  TrunkArgs a{};
  a.x = (const bf16*)x;
  a.y = (bf16*)y;
  for (int i = 0; i < 14; ++i) {
    a.w[i] = (const bf16*)w[i];
    a.b[i] = b[i];
  }
  return trunk_launch(a, N, H0, W0, stream);
}

// mbk_trunk_tail + the fused trunk head: f_out [N][256] bf16 = relu(W5 relu(y) + b5),
// v_out [N] = wc . f + bc (fc.hip mbk_fc_fwd's result); y may be null (not stored).
// w5: [256][H2*W2*32] bf16, NHWC column order.
extern "C" int mbk_trunk_tail_fc(const void* x, const void* const* w, const float* const* b,
                                 int N, int H0, int W0, void* y, const void* w5, const float* b5,
                                 const float* wc, const float* bc, int hidden, void* f_out,
                                 float* v_out, hipStream_t stream) {
  if (hidden != 256 || !w5 || !b5 || !wc || !bc || !f_out || !v_out)
    return (int)hipErrorInvalidValue;
  TrunkArgs a{};
  a.x = (const bf16*)x;
  a.y = (bf16*)y;
  for (int i = 0; i < 14; ++i) {
    a.w[i] = (const bf16*)w[i];
    a.b[i] = b[i];
  }
  a.w5 = (const bf16*)w5;
  a.b5 = b5;
  a.wc = wc;
  a.bc = bc;
  a.f_out = (bf16*)f_out;
  a.v_out = v_out;
  return trunk_launch(a, N, H0, W0, stream);
}

// fp8 trunk: w8 = e4m3 packed weights of layers 1..14 (mbk_conv_pack_fp8), ws = their
// per-output-channel dequant scales; activations in / out bf16 as mbk_trunk_tail.
extern "C" int mbk_trunk_tail_fp8(const void* x, const void* const* w8, const float* const* ws,
                                  const float* const* b, int N, int H0, int W0, void* y,
                                  hipStream_t stream) {
  TrunkArgs a{};
  a.x = (const bf16*)x;
  a.y = (bf16*)y;
  for (int i = 0; i < 14; ++i) {
    if (!w8[i] || !ws[i] || !b[i]) return (int)hipErrorInvalidValue;
    a.w8[i] = (const uint8_t*)w8[i];
    a.ws[i] = ws[i];
    a.b[i] = b[i];
  }
  return trunk_launch(a, N, H0, W0, stream);
}

static int trunk_launch(TrunkArgs a, int N, int H0, int W0, hipStream_t stream) {
  if (N <= 0) return 0;
  if (H0 < 1 || W0 < 1 || H0 > 16 || W0 > 16) return (int)hipErrorInvalidValue;
  a.N = N;
  a.H0 = H0;
  a.W0 = W0;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  // images per iteration: as many as LDS allows (each conv phase pays one L2 round trip
  // for its weights, so more images amortise it) while keeping >= one group per CU
  const bool f8 = a.w8[0] != nullptr;
  int tni = 1;
  while (tni < kMaxTNI && trunk_smem_bytes(H0, W0, tni * 2, 0, f8) <= 160 * 1024 &&
         (N + tni * 2 - 1) / (tni * 2) >= cus)
    tni *= 2;
  a.tni = tni;
  // float-reciprocal pixel index math in the kernel is exact only for tni*H0*W0 < 2^16
  if (H0 * W0 > 1024 || (int64_t)tni * H0 * W0 >= (int64_t(1) << 16))
    return (int)hipErrorInvalidValue;
  const size_t r = region_bytes(H0, W0, tni);
  a.r1_bytes = f8 ? (int)trunk8_region_a(H0, W0, tni) : (int)r;
  a.r2_bytes = f8 ? (int)trunk8_region_b(H0, W0, tni) : (int)r;
  const size_t sm = trunk_smem_bytes(H0, W0, tni, 0, f8);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  const bool fc = a.f_out != nullptr;
  if (fc && f8) return (int)hipErrorInvalidValue;
  auto kfn = f8 ? trunk_tail8_kernel : fc ? trunk_tail_kernel<true> : trunk_tail_kernel<false>;
  if (sm > 64 * 1024)
    hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kfn, kThreads, sm) !=
          hipSuccess || per < 1)
    per = 1;
  const int ngroups = (N + tni - 1) / tni;
  // persistent grid over the whole device
  const int grid = std::min(ngroups, cus * per);
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(kThreads), sm, stream, a);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ fused acting step, launch A
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static uint64_t* g_act_stamps = nullptr;  // diagnostic phase stamps (tools/act_phases.py)
// stamps: device buffer of grid x 8 x 64 uint64 (null: off); returns the stamps per workgroup
extern "C" int mbk_act_set_stamps(void* stamps) {
  g_act_stamps = (uint64_t*)stamps;
  return kActStamps;
}

extern "C" int mbk_act_trunk(const MbkActModel* m, const MbkActStep* s, hipStream_t stream) {
  if (!m || !s || m->E <= 0 || m->H != 16 || m->W != 16) return (int)hipErrorInvalidValue;
  if (!m->w0 || !m->b0 || !m->w5 || !m->b5 || !m->wc || !m->bc || !m->feat || !m->cellx ||
      !m->pending || !m->bucket_cnt || !m->bucket)
    return (int)hipErrorInvalidValue;
  if ((!s->code_list && (!s->codes || !s->res)) || (!s->act_list && !s->act16) || !s->obs ||
      !s->mask || !s->action || !s->logp || !s->value)
    return (int)hipErrorInvalidValue;
  if ((s->code_list || s->act_list) && s->list_stride < m->H * m->W + 1)
    return (int)hipErrorInvalidValue;
  if ((s->obs2 == nullptr) != (s->mask2 == nullptr) ||
      (s->reward_dst == nullptr) != (s->reward_src == nullptr) ||
      (s->done_dst == nullptr) != (s->done_src == nullptr))
    return (int)hipErrorInvalidValue;
  // 16-byte vector accesses of whole rows (S = 256 cells per env)
  if ((s->codes && !al16(s->codes)) || !al16(s->obs) || !al16(s->mask) || !al16(s->action) ||
      !al16(m->w0) || !al16(m->feat) || ((uintptr_t)s->act16 & 7) ||
      (s->obs2 && (!al16(s->obs2) || !al16(s->mask2))))
    return (int)hipErrorInvalidValue;
  ActTrunkArgs a{};
  TrunkArgs& t = a.t;
  for (int i = 0; i < 14; ++i) {
    if (!m->w[i] || !m->b[i]) return (int)hipErrorInvalidValue;
    t.w[i] = (const bf16*)m->w[i];
    t.b[i] = m->b[i];
  }
  t.w5 = (const bf16*)m->w5;
  t.b5 = m->b5;
  t.wc = m->wc;
  t.bc = m->bc;
  t.f_out = (bf16*)m->feat;
  t.v_out = s->value;
  t.N = m->E;
  t.H0 = 8;
  t.W0 = 8;
  const int tni = kWTni;
  t.tni = tni;
  t.r1_bytes = t.r2_bytes = kWRegion;
  const size_t sm = (size_t)kWSmem;
  if (m->E > 65535) return (int)hipErrorInvalidValue;  // bucket entry: env | rank
  a.w0 = (const bf16*)m->w0;
  a.b0 = m->b0;
  a.codes = s->codes;
  a.res = s->res;
  a.code_list = s->code_list;
  a.act_list = s->act_list;
  a.list_stride = s->list_stride;
  a.obs = s->obs;
  a.mask = s->mask;
  a.obs2 = s->obs2;
  a.mask2 = s->mask2;
  if ((s->abits2 && !s->abits) || (s->abits2 && !s->obs2)) return (int)hipErrorInvalidValue;
  a.abits = s->abits;
  a.abits2 = s->abits2;
  a.action = s->action;
  a.logp = s->logp;
  a.act16 = s->act16;
  a.pending = m->pending;
  const int S = m->H * m->W;
  a.bucket_cnt = m->bucket_cnt + (s->step & 1) * S;
  a.bucket_cnt_prev = m->bucket_cnt + ((s->step + 1) & 1) * S;
  a.bucket = m->bucket;
  a.cellx = m->cellx;
  a.reward_src = s->reward_src;
  a.done_src = s->done_src;
  a.reward_dst = s->reward_dst;
  a.done_dst = s->done_dst;
  a.stamps = g_act_stamps;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const void* kfn = (const void*)act_trunk_w_kernel;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, kWThreads, sm) != hipSuccess ||
      per < 1)
    per = 1;
  const int ngroups = (m->E + tni - 1) / tni;
  const int grid = std::min(ngroups, cus * per);
  hipLaunchKernelGGL(act_trunk_w_kernel, dim3(grid), dim3(kWThreads), sm, stream, a);
  return (int)hipGetLastError();
}
