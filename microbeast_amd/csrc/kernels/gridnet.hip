// GridNet (BASELINE config 2) data movement around the shifted-row MFMA GEMMs.
//
// The GridNet convolutions themselves are gemm.hip (forward / input grad) and fc.hip
// (weight grad) launches over zero-padded NHWC bf16 grids ([B][H+2][W+2][C], border = 0,
// ops/gridconv.py). Everything between those launches is here, so the GridNet path runs no
// ATen kernel at all:
//
//   bits_grid     int32 bit-plane obs -> padded bf16 input grid (planes expanded in flight)
//   pool_fwd      NHWC max_pool(3, 2, 1) of the relu'd conv output -> padded grid for the
//                 next conv (+ plain copy for the critic) + per-channel argmax (uint8)
//   pool_bwd      pooled-grid gradient(s), relu mask (pooled > 0) and argmax routing ->
//                 padded conv-output gradient grid (a gather: no atomics, deterministic)
//   grid_gather   strided / cropped / channel-padded / relu-masked copy of a gradient into
//                 the 4 sub-pixel phase grids of a stride-2 transposed conv (fp32 or bf16 in)
//   colsum        deterministic two-stage column sums (bias gradients), bf16 or fp32 in
//   map_gather    multi-segment index gather (weight packing into the GEMM operand layouts,
//                 weight-gradient unpacking into the parameters' own layouts), one launch
//   value_bwd     critic output layer backward: dh = (dv * w2 + g_head) * (h > 0), partial
//                 dW2 / db2 (also the IMPALA trunk tail's, models/agent.py)
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

// ------------------------------------------------------------------ bits -> padded grid
// bits [n][h*w] (plane p = bit p, p < 32) -> out [n][Hp][Wp][32] bf16; pixel (y, x) of the
// map sits at (y + 1, x + 1); the border and the area past (h, w) (maps padded up to a
// multiple of 16) are zero. Thread = (pixel, 8 planes): one 16-byte store.
template <typename IDX>
__global__ __launch_bounds__(kThreads) void bits_grid_kernel(const uint32_t* __restrict__ bits,
                                                             int n, int h, int w, int Hp, int Wp,
                                                             uint4* __restrict__ out) {
  const IDX total = (IDX)n * Hp * Wp * 4;
  for (IDX e = (IDX)blockIdx.x * kThreads + threadIdx.x; e < total; e += (IDX)gridDim.x * kThreads) {
    const int q = (int)(e & 3);
    const int p = (int)(e >> 2);
    const int x = p % Wp, t = p / Wp;
    const int y = t % Hp, b = t / Hp;
    uint32_t v = 0;
    if (y >= 1 && y <= h && x >= 1 && x <= w)
      v = (bits[(size_t)b * h * w + (y - 1) * w + (x - 1)] >> (8 * q)) & 0xFFu;
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = ((v >> (2 * j)) & 1u ? 0x3F80u : 0u) | ((v >> (2 * j + 1)) & 1u ? 0x3F800000u : 0u);
    out[e] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// int32 bit-plane obs [n][h*w] -> the same planes on the padded map [n][ph*pw] (zero outside the
// h x w map): the first encoder layer then runs on conv.hip's bit-plane kernels
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

// g_pad [B][H+2][W+2][C] interior * (p > 0) -> plain [B][H][W][C] (bf16, C % 8 == 0): the
// pooled-output gradient of relu(pool(conv)) from the next layer's padded-grid dgrad
template <typename IDX>
__global__ __launch_bounds__(kThreads) void crop_relu_mask_kernel(const uint4* __restrict__ g,
                                                                  const uint4* __restrict__ p,
                                                                  int B, int H, int W, int C8,
                                                                  uint4* __restrict__ out) {
  const IDX total = (IDX)B * H * W * C8;
  for (IDX e = (IDX)blockIdx.x * kThreads + threadIdx.x; e < total; e += (IDX)gridDim.x * kThreads) {
    const int q = (int)(e % C8);
    const IDX px = e / C8;
    const int x = (int)(px % W), t = (int)(px / W);
    const int y = t % H, b = t / H;
    const uint4 gv = g[(((IDX)b * (H + 2) + y + 1) * (W + 2) + x + 1) * C8 + q];
    const uint4 pv = p[e];
    const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w}, pw[4] = {pv.x, pv.y, pv.z, pv.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // bf16 > 0: sign bit clear and not +0 (per 16-bit half)
      const uint32_t lo = (pw[j] & 0x8000u) == 0u && (pw[j] & 0x7FFFu) != 0u ? 0xFFFFu : 0u;
      const uint32_t hi = (pw[j] & 0x80000000u) == 0u && (pw[j] & 0x7FFF0000u) != 0u
                              ? 0xFFFF0000u : 0u;
      o[j] = gw[j] & (lo | hi);
    }
    out[e] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ------------------------------------------------------------------ max pool 3x3 / 2, pad 1
// y [B][H][W][C] (relu'd conv output) -> out [B][Ho][Wo][C] and / or out_pad
// [B][Ho+2][Wo+2][C] (zero border), idx [B][Ho][Wo][C] = ky*3+kx of the first maximum in
// scan order (ATen's tie rule). Thread = (pixel of the padded grid if out_pad, else of the
// plain grid; 8 channels).
template <typename IDX>
__global__ __launch_bounds__(kThreads) void pool_fwd_kernel(const bf16* __restrict__ y, int B,
                                                            int H, int W, int C, int Ho, int Wo,
                                                            bf16* __restrict__ out,
                                                            bf16* __restrict__ out_pad,
                                                            uint8_t* __restrict__ idx) {
  const int C8 = C >> 3;
  const int pad = out_pad ? 1 : 0;
  const int Hg = Ho + 2 * pad, Wg = Wo + 2 * pad;
  const IDX total = (IDX)B * Hg * Wg * C8;
  for (IDX e = (IDX)blockIdx.x * kThreads + threadIdx.x; e < total; e += (IDX)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8), p = (int)(e / C8);
    const int gx = p % Wg, t = p / Wg;
    const int gy = t % Hg, b = t / Hg;
    const int oy = gy - pad, ox = gx - pad;
    if (oy < 0 || oy >= Ho || ox < 0 || ox >= Wo) {  // border of the padded grid
      *(uint4*)(out_pad + (size_t)p * C + 8 * c8) = make_uint4(0, 0, 0, 0);
      continue;
    }
    float mx[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mx[j] = -INFINITY; am[j] = -1; }
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = 2 * oy - 1 + ky;
      if (yy < 0 || yy >= H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = 2 * ox - 1 + kx;
        if (xx < 0 || xx >= W) continue;
        const uint4 u = *(const uint4*)(y + ((size_t)(b * H + yy) * W + xx) * C + 8 * c8);
        const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = (j & 1) ? bf_hi(uu[j >> 1]) : bf_lo(uu[j >> 1]);
          if (v > mx[j] || am[j] < 0) { mx[j] = v; am[j] = ky * 3 + kx; }
        }
      }
    }
    const uint4 o = make_uint4(pack2(mx[0], mx[1]), pack2(mx[2], mx[3]), pack2(mx[4], mx[5]),
                               pack2(mx[6], mx[7]));
    const size_t q = ((size_t)(b * Ho + oy) * Wo + ox) * C + 8 * c8;
    if (out_pad) *(uint4*)(out_pad + (size_t)p * C + 8 * c8) = o;
    if (out) *(uint4*)(out + q) = o;
    uint32_t i0 = 0, i1 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      i0 |= (uint32_t)am[j] << (8 * j);
      i1 |= (uint32_t)am[j + 4] << (8 * j);
    }
    *(uint2*)(idx + q) = make_uint2(i0, i1);
  }
}

// Gradient of relu + max_pool: pooled-output gradients g1 (+ g2), each on a plain
// [B][Ho][Wo][C] or padded [B][Ho+2][Wo+2][C] grid (pad flags), pass where pooled > 0 (the
// relu of the conv output; pooled = the argmax element's value) and go to the argmax
// position. Output: dy on the padded conv-output grid [B][H+2][W+2][C] (zero border), i.e.
// directly the operand of the conv's dgrad / wgrad GEMMs. Thread = (padded pixel, 8 ch).
template <typename IDX>
__global__ __launch_bounds__(kThreads) void pool_bwd_kernel(
    const bf16* __restrict__ g1, int pad1, const bf16* __restrict__ g2, int pad2,
    const bf16* __restrict__ pooled, int padp, const uint8_t* __restrict__ idx, int B, int H,
    int W, int C, int Ho, int Wo, bf16* __restrict__ dy) {
  const int C8 = C >> 3;
  const int Hp = H + 2, Wp = W + 2;
  const IDX total = (IDX)B * Hp * Wp * C8;
  for (IDX e = (IDX)blockIdx.x * kThreads + threadIdx.x; e < total; e += (IDX)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8), p = (int)(e / C8);
    const int x = p % Wp, t = p / Wp;
    const int y = t % Hp, b = t / Hp;
    const int Y = y - 1, X = x - 1;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if (Y >= 0 && Y < H && X >= 0 && X < W) {
      // windows oy with 2*oy - 1 <= Y <= 2*oy + 1: oy in [ceil((Y-1)/2), floor((Y+1)/2)]
      for (int oy = Y >> 1; oy <= (Y + 1) >> 1; ++oy) {
        if (oy < 0 || oy >= Ho) continue;
        const int ky = Y - (2 * oy - 1);
        for (int ox = X >> 1; ox <= (X + 1) >> 1; ++ox) {
          if (ox < 0 || ox >= Wo) continue;
          const int tap = ky * 3 + X - (2 * ox - 1);
          const size_t q = ((size_t)(b * Ho + oy) * Wo + ox) * C + 8 * c8;
          const uint2 iv = *(const uint2*)(idx + q);
          const uint32_t ii[2] = {iv.x, iv.y};
          bool any = false;
#pragma unroll
          for (int j = 0; j < 8; ++j) any |= ((ii[j >> 2] >> (8 * (j & 3))) & 0xFFu) == (uint32_t)tap;
          if (!any) continue;
          auto at = [&](int padded) {
            return padded ? ((size_t)(b * (Ho + 2) + oy + 1) * (Wo + 2) + ox + 1) * C + 8 * c8 : q;
          };
          const uint4 pv = *(const uint4*)(pooled + at(padp));
          const uint4 a1 = *(const uint4*)(g1 + at(pad1));
          uint4 a2 = make_uint4(0, 0, 0, 0);
          if (g2) a2 = *(const uint4*)(g2 + at(pad2));
          const uint32_t pu[4] = {pv.x, pv.y, pv.z, pv.w};
          const uint32_t u1[4] = {a1.x, a1.y, a1.z, a1.w};
          const uint32_t u2[4] = {a2.x, a2.y, a2.z, a2.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = j >> 1;
            const float pj = (j & 1) ? bf_hi(pu[k]) : bf_lo(pu[k]);
            const float gj = ((j & 1) ? bf_hi(u1[k]) : bf_lo(u1[k])) +
                             ((j & 1) ? bf_hi(u2[k]) : bf_lo(u2[k]));
            if (((ii[j >> 2] >> (8 * (j & 3))) & 0xFFu) == (uint32_t)tap && pj > 0.f) acc[j] += gj;
          }
        }
      }
    }
    *(uint4*)(dy + (size_t)p * C + 8 * c8) =
        make_uint4(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]),
                   pack2(acc[6], acc[7]));
  }
}

// ------------------------------------------------------------------ phase / pad gather
// dst [S*S][B][Hd+2][Wd+2][Cd] bf16 (S = stride 1 or 2, phase (a, c) = a*S + c), zero border:
//   dst[a*S+c][b][y][x][ch] = src(b, S*(y-1) + a, S*(x-1) + c, ch) * (mask(...) > 0)
// for in-range source pixels (Y < Hv, X < Wv) and channels ch < Cs, zero otherwise.
// src / mask are addressed by element strides (per image, row, pixel; channels unit
// stride), so plain, padded (offset base) and cropped layouts are all one case.
struct GatherArgs {
  const void* src;
  int src_f32;
  int64_t sb;
  int sy, sx;
  int Hv, Wv, Cs;
  const bf16* mask;
  int64_t mb;
  int my, mx;
  bf16* dst;
  int S, B, Hd, Wd, Cd;
};

template <typename IDX>
__global__ __launch_bounds__(kThreads) void grid_gather_kernel(GatherArgs a) {
  const int Hp = a.Hd + 2, Wp = a.Wd + 2, C8 = a.Cd >> 3;
  const IDX total = (IDX)a.S * a.S * a.B * Hp * Wp * C8;
  for (IDX e = (IDX)blockIdx.x * kThreads + threadIdx.x; e < total; e += (IDX)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8), p = (int)(e / C8);
    const int x = p % Wp, t = p / Wp;
    const int y = t % Hp, t2 = t / Hp;
    const int b = t2 % a.B, ph = t2 / a.B;
    const int Y = a.S * (y - 1) + ph / a.S, X = a.S * (x - 1) + ph % a.S;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    if (y >= 1 && y <= a.Hd && x >= 1 && x <= a.Wd && Y < a.Hv && X < a.Wv) {
      const int64_t so = b * a.sb + (int64_t)Y * a.sy + X * a.sx;
      const int64_t mo = b * a.mb + (int64_t)Y * a.my + X * a.mx;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ch = 8 * c8 + j;
        if (ch >= a.Cs) break;
        float s = a.src_f32 ? ((const float*)a.src)[so + ch]
                            : __bfloat162float(((const bf16*)a.src)[so + ch]);
        if (a.mask && !(__bfloat162float(a.mask[mo + ch]) > 0.f)) s = 0.f;
        v[j] = s;
      }
    }
    *(uint4*)(a.dst + (size_t)p * a.Cd + 8 * c8) =
        make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
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

extern "C" int mbk_bits_grid(const void* bits, int n, int h, int w, int Hp, int Wp, void* out,
                             hipStream_t stream) {
  const long total = (long)n * Hp * Wp * 4;
  if (n <= 0) return 0;
  if (!fits((long)n * Hp * Wp) || Hp < h + 2 || Wp < w + 2) return (int)hipErrorInvalidValue;
  MBK_LAUNCH_IDX(bits_grid_kernel, total, stream, (const uint32_t*)bits, n, h, w, Hp, Wp,
                 (uint4*)out);
  return (int)hipGetLastError();
}

extern "C" int mbk_bits_pad(const void* bits, int n, int h, int w, int ph, int pw, void* out,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  if (ph < h || pw < w) return (int)hipErrorInvalidValue;
  const long total = (long)n * ph * pw;
  MBK_LAUNCH_IDX(bits_pad_kernel, total, stream, (const uint32_t*)bits, n, h, w, ph, pw,
                 (uint32_t*)out);
  return (int)hipGetLastError();
}

extern "C" int mbk_crop_relu_mask(const void* g_pad, const void* p, int B, int H, int W, int C,
                                  void* out, hipStream_t stream) {
  if (B <= 0) return 0;
  if (C % 8) return (int)hipErrorInvalidValue;
  const long total = (long)B * H * W * (C / 8);
  MBK_LAUNCH_IDX(crop_relu_mask_kernel, total, stream, (const uint4*)g_pad, (const uint4*)p, B, H,
                 W, C / 8, (uint4*)out);
  return (int)hipGetLastError();
}

// out / out_pad may be null (not both); idx required. C % 8 == 0.
extern "C" int mbk_pool_fwd(const void* y, int B, int H, int W, int C, void* out, void* out_pad,
                            void* idx, hipStream_t stream) {
  if (B <= 0) return 0;
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long total = (long)B * (Ho + 2) * (Wo + 2) * (C / 8);
  if (C % 8 || !fits((long)B * (H + 2) * (W + 2)) || (!out && !out_pad) || !idx)
    return (int)hipErrorInvalidValue;
  MBK_LAUNCH_IDX(pool_fwd_kernel, total, stream, (const bf16*)y, B, H, W, C, Ho, Wo, (bf16*)out,
                 (bf16*)out_pad, (uint8_t*)idx);
  return (int)hipGetLastError();
}

// g2 may be null. dy: [B][H+2][W+2][C].
extern "C" int mbk_pool_bwd_grid(const void* g1, int pad1, const void* g2, int pad2,
                                 const void* pooled, int padp, const void* idx, int B, int H,
                                 int W, int C, void* dy, hipStream_t stream) {
  if (B <= 0) return 0;
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long total = (long)B * (H + 2) * (W + 2) * (C / 8);
  if (C % 8 || !fits((long)B * (H + 2) * (W + 2))) return (int)hipErrorInvalidValue;
  MBK_LAUNCH_IDX(pool_bwd_kernel, total, stream, (const bf16*)g1, pad1, (const bf16*)g2, pad2,
                 (const bf16*)pooled, padp, (const uint8_t*)idx, B, H, W, C, Ho, Wo, (bf16*)dy);
  return (int)hipGetLastError();
}

// geo: 14 ints {src_f32, sb, sy, sx, Hv, Wv, Cs, mb, my, mx, S, B, Hd, Wd}; Cd % 8 == 0
extern "C" int mbk_grid_gather(const void* src, const void* mask, const int* geo, void* dst, int Cd,
                               hipStream_t stream) {
  GatherArgs a{};
  a.src = src;
  a.src_f32 = geo[0], a.sb = geo[1], a.sy = geo[2], a.sx = geo[3];
  a.Hv = geo[4], a.Wv = geo[5], a.Cs = geo[6];
  a.mask = (const bf16*)mask;
  a.mb = geo[7], a.my = geo[8], a.mx = geo[9];
  a.S = geo[10], a.B = geo[11], a.Hd = geo[12], a.Wd = geo[13];
  a.dst = (bf16*)dst;
  a.Cd = Cd;
  if (a.B <= 0) return 0;
  const long pixels = (long)a.S * a.S * a.B * (a.Hd + 2) * (a.Wd + 2);
  if (Cd % 8 || (a.S != 1 && a.S != 2) || a.Cs > Cd || !fits(pixels))
    return (int)hipErrorInvalidValue;
  MBK_LAUNCH_IDX(grid_gather_kernel, pixels * (Cd / 8), stream, a);
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
