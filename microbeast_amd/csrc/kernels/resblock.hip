// Fused residual-block backward for 16-channel blocks (IMPALA stage 0: 8x8 maps at 16x16).
//
// Reference block (model.py:56-73): y = x + conv1(relu(conv0(relu(x)))), u = conv0(relu x).
// Given g = dL/dy the per-layer path (ops/encoder.py) ran four launches per block, each
// round-tripping a full activation tensor through HBM:
//   wgrad1(relu u, g) | du = conv1^T(g) * [u > 0] | wgrad0(relu x, du) | dx = conv0^T(du) * [x > 0] + g
// = 12 B of HBM traffic per activation byte (x, u, g read twice or more, du written and
// re-read). Here one persistent kernel stages x, u, g of an image group into LDS once
// (relu'd where the consumer wants relu), computes du into an LDS tile, then dx, and keeps
// both weight gradients in MFMA accumulators for the whole launch: 4 B of HBM per
// activation byte (read x, u, g; write dx). Profile 18 timed the four launches at ~2.3 ms
// per block per 524K frames, near the HBM roofline for that traffic.
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16), identical to conv.hip so dx / du are
// bit-identical to the per-layer kernels:
//   dgrad : A = packed transposed weights (VGPRs), B = 16 pixels x 32 K from the halo'd
//           tile (K chunk = 2 taps x 16 channels), acc lane = 4 channels of one pixel;
//   wgrad : A = dY (16 co x 32 pixels) and B = X taps (32 pixels x 16 ci), both read with
//           ds_read_b64_tr_b16 from the same halo'd tiles; acc over the 9 taps.
// Weight grads go out as per-workgroup fp32 partial rows [2][16*144 + 16] reduced by
// conv.hip's deterministic wgrad_reduce (bias grads included).
#include "../include/mbk_api.h"
#include "common.h"

#include <algorithm>


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

extern "C" int mbk_wgrad_reduce(const float* partial, int nparts, int cin, int cin_real,
                                int cout, float* dw, float* db, int accumulate,
                                hipStream_t stream);

namespace {

constexpr int kThreads = 256;
constexpr int C = 16;                  // channels (in = out)
constexpr int PIXB = C * 2 + 16;       // halo'd tile pixel stride, bytes (bank spread)
constexpr int NCH = 5;                 // dgrad K chunks of 32 (2 taps x 16 ch; chunk 4 padded)
constexpr int KTOT = 9 * C;            // wgrad K per output channel
constexpr int ROW = C * KTOT + C;      // one partial row (weights + bias)
constexpr int kPF = 2;                 // staging prefetch slots per thread per tensor (imgs*HW <= 256)

union Frag8 {
  bf16x8 v;
  uint4 u;
  s16x4 h[2];
};

__device__ __forceinline__ uint32_t relu2(uint32_t w) {
  s16x2 v = __builtin_bit_cast(s16x2, w);
  v = __builtin_elementwise_max(v, s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ uint4 relu8(uint4 v) {
  return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}
__device__ __forceinline__ float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(a)) |
         ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(b)) << 16);
}
__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}

// 8x8-map tile geometry of the wave-owned kernels (res_fwd16_w88 / res_bwd16_w88): lay16(8, 8)
namespace w88 {
constexpr int H = 8, W = 8, HW = 64, PB = 32, RB = 512;
constexpr int IMGB = ((H + 1) * RB + (W + 2) * PB + 15) & ~15;  // lay16(8, 8).imgb
constexpr int REG = 3 * IMGB;  // a wave's LDS: Tx, Tr, Tu
constexpr int TX = 0, TR = IMGB, TU = 2 * IMGB;
}  // namespace w88

__device__ __forceinline__ uint32_t cvt_pk2(float a, float b) {  // v_cvt_pk_bf16_f32 (RNE)
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, b16x2));
}

// compiler-only ordering point between a wave's LDS writes and its later reads of them (the
// hardware completes one wave's LDS instructions in order)
__device__ __forceinline__ void wave_lds_order() { asm volatile("" ::: "memory"); }

struct ResBwdArgs {
  const bf16* x;     // block input (pre-relu)      [N][H][W][16]
  const bf16* u;     // conv0 output (pre-relu)     [N][H][W][16]
  const bf16* g;     // dL/dy                        [N][H][W][16]
  bf16* dx;          // dL/dx                        [N][H][W][16]
  const bf16* w1t;   // conv1 packed dgrad weights [16][5][32] (conv.hip packed_bwd layout)
  const bf16* w0t;   // conv0 packed dgrad weights
  float* partial;    // layer l's row of workgroup b at partial + l * lstride + b * ROW
  int64_t lstride;   // floats per layer block: (nparts + reduce scratch rows) * ROW
  int N, H, W, imgs;
};

// Halo'd tile layout of the 16-channel backward kernel: byte offset of halo'd pixel (yy, xx) of
// image im = im * imgb + yy * rowb + xx * pb. For 8-wide maps (IMPALA stage 0 at 16x16) the
// pixels are 32 bytes in 512-byte rows: the dgrad's ds_read_b128 lane groups (16 pixels of two
// map rows, two 16-byte channel halves) then hit 64 distinct banks, which the 48-byte stride
// with 480-byte rows served in 3 cycles instead of 1 (profile 22: 35 % extra LDS cycles; bank
// model in tools/lds_banks.py). The last row holds only its 10 pixels.
struct Lay16 {
  int pb, rowb, imgb;
};
__host__ __device__ inline Lay16 lay16(int H, int W) {
  const int Hp = H + 2, Wp = W + 2;
  if (W == 8) return {32, 512, ((Hp - 1) * 512 + Wp * 32 + 15) & ~15};
  return {PIXB, Wp * PIXB, Hp * Wp * PIXB};
}

// WC > 0: the map width as a compile-time constant (IMPALA stage-0 shapes), so every tap
// offset is an immediate of the LDS instruction instead of per-lane multiply-adds
// (PMC: the runtime-width form issued ~15 VALU per MFMA); WC == 0: any width
template <int WC>
__global__ __launch_bounds__(kThreads) void res_bwd16_kernel(ResBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, W = WC > 0 ? WC : a.W, HW = H * W, Hp = H + 2, Wp = W + 2;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // tile layout: 8-wide maps use 32-byte pixels in 512-byte rows (no bank conflicts for the
  // dgrad ds_read_b128 or the staging writes, lay16); other widths the 48-byte pixel stride
  const Lay16 L = lay16(H, W);
  const int PB = L.pb, RB = L.rowb;
  const int tb = ((a.imgs * L.imgb) + 15) & ~15;
  char* Tg = smem;            // g          (dgrad1 input, wgrad1 dY, + g of dx)
  char* Tu = smem + tb;       // relu(u)    (wgrad1 X, du mask)
  char* Tx = smem + 2 * tb;   // relu(x)    (wgrad0 X, dx mask)
  char* Td = smem + 3 * tb;   // du         (dgrad0 input, wgrad0 dY)
  char* zero = smem + 4 * tb; // 64 zero bytes for out-of-range wgrad pixels
  float* red = (float*)smem;  // [C][KTOT] reduction after the loop

  for (int e = tid; e < (4 * tb + 64) / 16; e += kThreads) ((uint4*)smem)[e] = make_uint4(0, 0, 0, 0);

  // dgrad weights (A fragments): lane holds w[co = li][chunk c][8g .. 8g+7]
  Frag8 w1[NCH], w0[NCH];
  {
    const uint4* p1 = (const uint4*)(a.w1t + (size_t)li * NCH * 32 + g * 8);
    const uint4* p0 = (const uint4*)(a.w0t + (size_t)li * NCH * 32 + g * 8);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      w1[c].u = p1[c * 4];
      w0[c].u = p0[c * 4];
    }
  }
  f32x4 acc1[9], acc0[9];  // wgrad accumulators, tap t: rows co = 4G + i, cols ci = li
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // per-lane byte offset of dgrad chunk c relative to the block's tap-(0,0) position: this
  // lane's K group (g) reads tap 2c + (g >> 1), channels 8 (g & 1) .. +8
  int coff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int tap = 2 * c + (g >> 1), tapc = tap < 9 ? tap : 8;  // chunk 4's pad half
    coff[c] = (tapc / 3) * RB + (tapc % 3) * PB + 16 * (g & 1);
  }
  float db1[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // sum g: this thread's 8-channel half (tid & 1)
  float db0[4] = {0, 0, 0, 0};              // sum du: channels 4g .. 4g+3 (dgrad lane map)

  const int per = a.imgs * HW * 2;  // uint4 staging elements per tensor per round
  const int nrounds = (a.N + a.imgs - 1) / a.imgs;
  uint4 px[kPF], pu[kPF], pg[kPF];
  auto prefetch = [&](int rd) {
    const int lim = min(per, (a.N - rd * a.imgs) * HW * 2);
    const size_t base = (size_t)rd * per;
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int e = tid + k * kThreads;
      const bool ok = e < lim;
      px[k] = ok ? ((const uint4*)a.x)[base + e] : make_uint4(0, 0, 0, 0);
      pu[k] = ok ? ((const uint4*)a.u)[base + e] : make_uint4(0, 0, 0, 0);
      pg[k] = ok ? ((const uint4*)a.g)[base + e] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lds_off = [&](int e) {  // staging element -> byte offset in a halo'd tile
    const int q = e & 1, p = e >> 1;
    const int im = (int)(((float)p + 0.5f) * inv_hw), r = p - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
    return im * L.imgb + (y + 1) * RB + (x + 1) * PB + q * 16;
  };
  auto put = [&](int e, uint4 vx, uint4 vu, uint4 vg) {
    const int o = lds_off(e);
    *(uint4*)(Tx + o) = relu8(vx);
    *(uint4*)(Tu + o) = relu8(vu);
    *(uint4*)(Tg + o) = vg;
    const uint32_t w[4] = {vg.x, vg.y, vg.z, vg.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      db1[2 * j] += lo_f(w[j]);
      db1[2 * j + 1] += hi_f(w[j]);
    }
  };

  if ((int)blockIdx.x < nrounds) prefetch(blockIdx.x);
  __syncthreads();  // zeroed tiles visible
  for (int rd = blockIdx.x; rd < nrounds; rd += gridDim.x) {
    const int img0 = rd * a.imgs, nimg = min(a.imgs, a.N - img0);
    const int lim = nimg * HW * 2;
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int e = tid + k * kThreads;
      if (e < lim) put(e, px[k], pu[k], pg[k]);
    }
    for (int e = tid + kPF * kThreads; e < lim; e += kThreads) {
      const size_t s = (size_t)rd * per + e;
      put(e, ((const uint4*)a.x)[s], ((const uint4*)a.u)[s], ((const uint4*)a.g)[s]);
    }
    __syncthreads();
    if (rd + (int)gridDim.x < nrounds) prefetch(rd + gridDim.x);

    const int M = nimg * HW, nblk = (M + 15) >> 4, nk = (M + 31) >> 5;
    // ---------------- phase A: du = conv1^T(g) * [u > 0] -> Td;  dW1 += relu(u) (x) g
    for (int pb = wave; pb < nblk; pb += kThreads / 64) {
      const int m = pb * 16 + li;
      const bool valid = m < M;
      const int mm = valid ? m : 0;
      const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
      const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
      const int base = im * L.imgb + y * RB + x * PB;  // byte offset of tap (0, 0)
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* bp = Tg + base;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        Frag8 av;
        av.u = *(const uint4*)(bp + coff[c]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[c].v, av.v, acc, 0, 0, 0);
      }
      if (!valid) continue;
      const int o = base + RB + PB + 4 * g * 2;  // interior pixel, channels 4g..
      const uint2 mu = *(const uint2*)(Tu + o);
      const uint32_t mw[2] = {mu.x, mu.y};
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        v[i] = (__uint_as_float(hb << 16) > 0.f) ? acc[i] : 0.f;
      }
      const uint2 du = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      *(uint2*)(Td + o) = du;
      db0[0] += lo_f(du.x); db0[1] += hi_f(du.x); db0[2] += lo_f(du.y); db0[3] += hi_f(du.y);
    }
    for (int kb = wave; kb < nk; kb += kThreads / 64) {
      const char* dptr[2];
      int xpos[2];
      bool ok[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = kb * 32 + 8 * g + 4 * h + (li >> 2);
        ok[h] = p < M;
        const int pp = ok[h] ? p : 0;
        const int im = (int)(((float)pp + 0.5f) * inv_hw), r = pp - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        xpos[h] = im * L.imgb + y * RB + x * PB;  // byte offset of tap (0, 0)
        dptr[h] = ok[h] ? Tg + xpos[h] + RB + PB : zero;
      }
      Frag8 af;
#pragma unroll
      for (int h = 0; h < 2; ++h) af.h[h] = tr_read(dptr[h] + (4 * (li & 3)) * 2);
      // X taps: out-of-range pixels read pixel 0's (finite) values; their dY column (A)
      // is zero, so they add exactly nothing and need no per-tap zero select
      const char* xb0 = Tu + xpos[0] + 8 * (li & 3);
      const char* xb1 = Tu + xpos[1] + 8 * (li & 3);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int off = (t / 3) * RB + (t % 3) * PB;
        Frag8 bf;
        bf.h[0] = tr_read(xb0 + off);
        bf.h[1] = tr_read(xb1 + off);
        acc1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bf.v, acc1[t], 0, 0, 0);
      }
    }
    __syncthreads();  // Td complete
    // ---------------- phase B: dx = conv0^T(du) * [x > 0] + g -> HBM;  dW0 += relu(x) (x) du
    const size_t gpix0 = (size_t)img0 * HW;
    for (int pb = wave; pb < nblk; pb += kThreads / 64) {
      const int m = pb * 16 + li;
      const bool valid = m < M;
      const int mm = valid ? m : 0;
      const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
      const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
      const int base = im * L.imgb + y * RB + x * PB;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* bp = Td + base;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        Frag8 av;
        av.u = *(const uint4*)(bp + coff[c]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[c].v, av.v, acc, 0, 0, 0);
      }
      if (!valid) continue;
      const int o = base + RB + PB + 4 * g * 2;
      const uint2 mx = *(const uint2*)(Tx + o), ad = *(const uint2*)(Tg + o);
      const uint32_t mw[2] = {mx.x, mx.y}, aw[2] = {ad.x, ad.y};
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        v[i] = (__uint_as_float(hb << 16) > 0.f) ? acc[i] : 0.f;
        v[i] += __uint_as_float(((aw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) << 16);
      }
      *(uint2*)(a.dx + (gpix0 + m) * C + 4 * g) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
    for (int kb = wave; kb < nk; kb += kThreads / 64) {
      const char* dptr[2];
      int xpos[2];
      bool ok[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = kb * 32 + 8 * g + 4 * h + (li >> 2);
        ok[h] = p < M;
        const int pp = ok[h] ? p : 0;
        const int im = (int)(((float)pp + 0.5f) * inv_hw), r = pp - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        xpos[h] = im * L.imgb + y * RB + x * PB;  // byte offset of tap (0, 0)
        dptr[h] = ok[h] ? Td + xpos[h] + RB + PB : zero;
      }
      Frag8 af;
#pragma unroll
      for (int h = 0; h < 2; ++h) af.h[h] = tr_read(dptr[h] + (4 * (li & 3)) * 2);
      // X taps: out-of-range pixels read pixel 0's (finite) values; their dY column (A)
      // is zero, so they add exactly nothing and need no per-tap zero select
      const char* xb0 = Tx + xpos[0] + 8 * (li & 3);
      const char* xb1 = Tx + xpos[1] + 8 * (li & 3);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int off = (t / 3) * RB + (t % 3) * PB;
        Frag8 bf;
        bf.h[0] = tr_read(xb0 + off);
        bf.h[1] = tr_read(xb1 + off);
        acc0[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bf.v, acc0[t], 0, 0, 0);
      }
    }
    __syncthreads();  // tiles consumed before the next round is staged
  }
  // ---- per-workgroup partial rows: the 4 waves' accumulators summed through LDS in a fixed
  // order (deterministic), then the bias sums
  for (int which = 0; which < 2; ++which) {
    float* out = a.partial + which * a.lstride + (size_t)blockIdx.x * ROW;
    for (int w = 0; w < kThreads / 64; ++w) {
      if (wave == w) {
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int co = 4 * g + i, n = t * C + li;
            float* p = red + co * KTOT + n;
            const float v = which == 0 ? acc1[t][i] : acc0[t][i];
            *p = (w == 0 ? 0.f : *p) + v;
          }
      }
      __syncthreads();
    }
    for (int e = tid; e < C * KTOT / 4; e += kThreads) ((float4*)out)[e] = ((const float4*)red)[e];
    __syncthreads();
  }
  float* out1 = a.partial + (size_t)blockIdx.x * ROW;
  float* out0 = a.partial + a.lstride + (size_t)blockIdx.x * ROW;
  // bias grads: db1 per thread covers channels 8 * (tid & 1) .. +8; db0 per lane channels 4g..
  float* bred = red;  // [kThreads][12]
#pragma unroll
  for (int j = 0; j < 8; ++j) bred[tid * 12 + j] = db1[j];
#pragma unroll
  for (int j = 0; j < 4; ++j) bred[tid * 12 + 8 + j] = db0[j];
  __syncthreads();
  if (tid < C) {
    const int half = tid / 8, j = tid % 8;
    float s = 0.f;
    for (int t = half; t < kThreads; t += 2) s += bred[t * 12 + j];
    out1[C * KTOT + tid] = s;  // conv1 bias
    const int gq = tid / 4, i = tid % 4;  // channel tid = 4 * gq + i lives in lanes g == gq
    float s0 = 0.f;
    for (int t = 0; t < kThreads; ++t)
      if (((t & 63) >> 4) == gq) s0 += bred[t * 12 + 8 + i];
    out0[C * KTOT + tid] = s0;  // conv0 bias
  }
}

// ------------------------------------------------------------------ wave-pair backward (8x8)
// res_bwd16_kernel for IMPALA stage 0 at 16x16 (8x8 maps). The generic kernel ran 3 workgroup
// barriers per round of 4 images at 19.9 % MFMA (profile r5a); a wave-owned version (each wave
// whole images, dgrads and weight gradients) needed 276 registers -- the two layers' 72
// weight-gradient accumulators next to the dgrad weights -- so one wave per SIMD, every latency
// exposed (1.28 ms, 21.7 % MFMA); splitting each image over a wave pair synchronised by
// workgroup barriers (3 per 4 images) left the waves parked 58 % of their cycles (1.25 ms).
// Here 8 waves form 4 independent producer / consumer pairs, each pair on one SIMD:
//   D-wave p (waves 0-3): du = conv1^T(g) * [u > 0] -> Td; dx = conv0^T(du) * [x > 0] + g ->
//     HBM (dgrad weights in VGPRs);
//   W-wave p + 4 (waves 4-7): stages x, u, g (HBM loads one image ahead); dW1 += relu(u) (x) g,
//     dW0 += relu(x) (x) du (accumulators for the whole launch),
// over two sets of the pair's LDS tiles (Tg = g, Tu = relu u, Tx = relu x, Td = du), image i in
// set i % 2, synchronised by three per-pair LDS flags per set (staged / du written / D done with
// the set) instead of workgroup barriers: a wave's LDS writes complete in issue order, so a flag
// written after the data publishes it. (The staging sat in the D-wave until round 5: with the
// epilogues too, the D-wave was the pair's critical path and its W-wave spun on the flags --
// 4.2 VALU per MFMA, 55 % of wave cycles waiting, profile r5n.) Block j of the dgrads is map row pair j and K block kb of the
// weight gradients rows 4 kb .. 4 kb + 3, so their offsets are immediates; tap reads are
// software-pipelined against the MFMA chains. du / dx are bit-identical to the per-layer
// kernels; the weight gradients differ by fp32 summation order (the W-waves' fixed-order sum).
namespace w88b {
constexpr int RB = w88::RB, PB = w88::PB, IMGB = w88::IMGB;
constexpr int SET = 4 * IMGB;  // one tile set: Tg, Tu, Tx, Td
// tile sets per pair: 1 (single-buffered: 79 KB per workgroup, so 2 workgroups -- 4 waves --
// share each SIMD and one pair's waits are the other's issue slots) or 2 (157 KB, 1 per CU)
constexpr int NSET = 1;
constexpr int REG = NSET * SET;  // a pair's LDS
constexpr int TG = 0, TU = IMGB, TX = 2 * IMGB, TD = 3 * IMGB;
constexpr int NP = 2;            // pairs per workgroup (3 workgroups of 2 pairs per CU at
                                 // 162 VGPRs: 3 waves per SIMD)
constexpr int kPT = 128 * NP;
constexpr int FLAGS = NP * REG;  // per pair, per set: staged, du written, D done (iteration #)
}  // namespace w88b

// LDS flags between the two waves of a pair. The hardware runs one wave's LDS instructions in
// issue order, so a flag store issued after a tile's stores is seen after them; what must not
// move is the ISSUE order, i.e. the compiler may not sink an ordinary LDS store below the
// volatile flag store (or hoist a tile load above the flag poll). Both helpers therefore carry
// the compiler fence themselves (wave_lds_order: asm memory clobber, no instruction), so no call
// site can forget it (two set_flag sites relied on the fence being written beside them).
// spin until an LDS flag reaches v (written by the other wave of the pair)
__device__ __forceinline__ void wait_flag(const int* f, int v) {
  while (*(const volatile int*)f < v) __builtin_amdgcn_s_sleep(1);
  wave_lds_order();  // acquire side: no tile load above the poll
}
__device__ __forceinline__ void set_flag(int* f, int v, int lane) {
  wave_lds_order();  // release side: every tile store issued before the flag
  if (lane == 0) *(volatile int*)f = v;
}

__global__ __launch_bounds__(w88b::kPT) void res_bwd16_w88_kernel(ResBwdArgs a) {
  using namespace w88b;
  constexpr int HW = 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const bool dw = wave < NP;  // D-wave (dgrads) or W-wave (weight gradients)
  const int pair = wave % NP;
  char* R = smem + pair * REG;
  int* fl = (int*)(smem + FLAGS) + pair * 6;  // [set][staged, du, D done]
  for (int e = tid; e < FLAGS / 16; e += kPT) ((uint4*)smem)[e] = make_uint4(0, 0, 0, 0);
  if (tid < 6 * NP) ((int*)(smem + FLAGS))[tid] = 0;
  // dgrad (D-waves): this lane's pixel of row pair 0, tap (0, 0) offset per K chunk
  const int lb = (li >> 3) * RB + (li & 7) * PB;
  int aoff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int tap = 2 * c + (g >> 1), tapc = tap < 9 ? tap : 8;
    aoff[c] = lb + (tapc / 3) * RB + (tapc % 3) * PB + 16 * (g & 1);
  }
  const int ob = lb + RB + PB + 8 * g;  // output pixel (interior), channels 4g..
  const uint32_t goff = (uint32_t)(li * C + 4 * g) * 2;
  // wgrad (W-waves) K block 0 (rows 0-3): any pixel order along K will do as long as dY (A)
  // and X (B) agree, so half h's pixel of lane group g is row 2 (g / 2) + h, column
  // 4 (g % 2) + li / 4: each 32-lane half of a transposed read then covers one whole map row,
  // 256 contiguous bytes = all 64 banks (rows g and g + 1, 512 B apart, were 2-way conflicts);
  // the dY read starts at channel 4 (li % 4), the X taps at 8 (li % 4) B
  int xo[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) xo[h] = (2 * (g >> 1) + h) * RB + (4 * (g & 1) + (li >> 2)) * PB;
  const int ao = RB + PB + 8 * (li & 3), bo = 8 * (li & 3);
  int so[2];  // staging: this lane's two 16-byte chunks of an image
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = lane + 64 * k, px = e >> 1;
    so[k] = ((px >> 3) + 1) * RB + ((px & 7) + 1) * PB + (e & 1) * 16;
  }
  const int step = gridDim.x * NP;
  const int first = blockIdx.x * NP + pair;  // the pair's images: first, first + step, ...
  __syncthreads();  // zeroed tiles and flags
  if (dw) {
    Frag8 w1[NCH], w0[NCH];  // dgrad weights (A fragments): lane holds w[co = li][chunk c][8g..]
    {
      const uint4* p1 = (const uint4*)(a.w1t + (size_t)li * NCH * 32 + g * 8);
      const uint4* p0 = (const uint4*)(a.w0t + (size_t)li * NCH * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        w1[c].u = p1[c * 4];
        w0[c].u = p0[c * 4];
      }
    }
    // one dgrad pass (4 row-pair blocks x 5 K chunks = 20 MFMAs, step st = 5 j + c) from tile
    // S with weights W; each tap read issued DD steps ahead of its MFMA
    auto dgrad = [&](const char* S, const Frag8* W, f32x4* acc) {
      constexpr int DD = 8;
      Frag8 fr[20];
      auto rd = [&](int st) {
        fr[st].u = *(const uint4*)(S + (st / NCH) * 2 * RB + aoff[st % NCH]);
      };
#pragma unroll
      for (int st = 0; st < DD; ++st) rd(st);
#pragma unroll
      for (int st = 0; st < 20; ++st) {
        const int j = st / NCH, c = st % NCH;
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            W[c].v, fr[st].v, c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[j], 0, 0, 0);
        if (st + DD < 20) rd(st + DD);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    int it = 1;
    for (int img = first; img < a.N; img += step, ++it) {
      const int b = it % NSET;
      char* T = R + b * SET;
      int* f = fl + 3 * b;
      wait_flag(f, it);  // staged (by the W-wave)
      wave_lds_order();
      f32x4 acc[4];
      // du = conv1^T(g) * [u > 0] -> Td (the epilogue's mask words read ahead of the MFMAs)
      uint2 mus[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) mus[j] = *(const uint2*)(T + TU + j * 2 * RB + ob);
      dgrad(T + TG, w1, acc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = j * 2 * RB + ob;
        const uint2 mu = mus[j];
        const uint32_t mw[2] = {mu.x, mu.y};
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
          v[i] = (__uint_as_float(hb << 16) > 0.f) ? acc[j][i] : 0.f;
        }
        *(uint2*)(T + TD + o) = make_uint2(cvt_pk2(v[0], v[1]), cvt_pk2(v[2], v[3]));
      }
      set_flag(f + 1, it, lane);  // du written
      wave_lds_order();
      // dx = conv0^T(du) * [x > 0] + g -> HBM
      uint2 mxs[4], ads[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mxs[j] = *(const uint2*)(T + TX + j * 2 * RB + ob);
        ads[j] = *(const uint2*)(T + TG + j * 2 * RB + ob);
      }
      dgrad(T + TD, w0, acc);
      char* gdx = (char*)(a.dx + (size_t)img * HW * C);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint2 mx = mxs[j], ad = ads[j];
        const uint32_t mw[2] = {mx.x, mx.y}, aw[2] = {ad.x, ad.y};
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
          v[i] = (__uint_as_float(hb << 16) > 0.f) ? acc[j][i] : 0.f;
          v[i] += __uint_as_float(((aw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) << 16);
        }
        *(uint2*)(gdx + j * 16 * C * 2 + goff) =
            make_uint2(cvt_pk2(v[0], v[1]), cvt_pk2(v[2], v[3]));
      }
      wave_lds_order();
      set_flag(f + 2, it, lane);  // done with the set (its reads completed in issue order)
    }
    __syncthreads();  // (the W-waves' matching barrier: every pair is done)
  } else {  // ---------------- W-waves
  f32x4 acc1[9], acc0[9];  // wgrad accumulators, tap t: rows co = 4G + i, cols ci = li
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // bias gradients as one more MFMA per K block: dY (A) times an all-ones B fragment, so every
  // column of accb* holds the row's pixel sum
  f32x4 accb1 = f32x4{0.f, 0.f, 0.f, 0.f}, accb0 = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  // one weight-gradient pass over the image's 2 K blocks (18 MFMAs: K block kb = s / 9, tap
  // t = s % 9): dY from tile D (interior), X taps from tile X, each tap read DW steps ahead
  auto wgrad = [&](const char* D, const char* X, f32x4* acc, f32x4& accb) {
    constexpr int DW = 8;
    Frag8 af[2], bf[18];
    auto rd_b = [&](int st) {
      const int kb = st / 9, t = st % 9;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        bf[st].h[h] = tr_read(X + kb * 4 * RB + xo[h] + bo + (t / 3) * RB + (t % 3) * PB);
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) af[0].h[h] = tr_read(D + xo[h] + ao);
#pragma unroll
    for (int st = 0; st < DW; ++st) rd_b(st);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      const int kb = st / 9, t = st % 9;
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kb].v, bf[st].v, acc[t], 0, 0, 0);
      if (t == 8) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kb].v, ones.v, accb, 0, 0, 0);
      if (st + DW < 18) rd_b(st + DW);
      if (st == 4) {  // K block 1 = rows 4-7: its dY fragment
#pragma unroll
        for (int h = 0; h < 2; ++h) af[1].h[h] = tr_read(D + 4 * RB + xo[h] + ao);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // (named registers: the indexed [2] arrays of the first form went to scratch)
  uint4 px0, px1, pu0, pu1, pg0, pg1;
  auto fetch = [&](int im) {
    const size_t o = (size_t)im * HW * 2 + lane;
    px0 = ((const uint4*)a.x)[o];
    px1 = ((const uint4*)a.x)[o + 64];
    pu0 = ((const uint4*)a.u)[o];
    pu1 = ((const uint4*)a.u)[o + 64];
    pg0 = ((const uint4*)a.g)[o];
    pg1 = ((const uint4*)a.g)[o + 64];
  };
  if (first < a.N) fetch(first);
  int it = 1;
  for (int img = first; img < a.N; img += step, ++it) {
    const int b = it % NSET;
    char* T = R + b * SET;
    int* f = fl + 3 * b;
    if (it > NSET) wait_flag(f + 2, it - NSET);  // the D-wave is done with this set's last image
    *(uint4*)(T + TX + so[0]) = relu8(px0);
    *(uint4*)(T + TU + so[0]) = relu8(pu0);
    *(uint4*)(T + TG + so[0]) = pg0;
    *(uint4*)(T + TX + so[1]) = relu8(px1);
    *(uint4*)(T + TU + so[1]) = relu8(pu1);
    *(uint4*)(T + TG + so[1]) = pg1;
    set_flag(f, it, lane);  // staged
    if (img + step < a.N) fetch(img + step);
    wave_lds_order();
    wgrad(T + TG, T + TU, acc1, accb1);  // dW1 += relu(u) (x) g
    wait_flag(f + 1, it);  // du written
    wave_lds_order();
    wgrad(T + TD, T + TX, acc0, accb0);  // dW0 += relu(x) (x) du
    wave_lds_order();
  }
  __syncthreads();  // every pair is done: the tiles are dead
  // every tile is dead after the last (3): each W-wave parks its accumulators in its own slot
  float* red = (float*)smem;
#pragma unroll
  for (int which = 0; which < 2; ++which) {
    float* sl = red + (which * NP + pair) * (C * KTOT);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sl[(4 * g + i) * KTOT + t * C + li] = which == 0 ? acc1[t][i] : acc0[t][i];
    if (li == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[2 * NP * C * KTOT + (which * NP + pair) * C + 4 * g + i] =
            which == 0 ? accb1[i] : accb0[i];
  }
  }
  __syncthreads();
  // ---- per-workgroup partial rows: the NP W-waves' slots summed in a fixed order
  // (deterministic); bias = column 0 of the all-ones accumulators
  const float* red = (const float*)smem;
  for (int which = 0; which < 2; ++which) {
    float* out = a.partial + which * a.lstride + (size_t)blockIdx.x * ROW;
    const float* sl = red + which * NP * (C * KTOT);
    for (int e = tid; e < C * KTOT; e += kPT) {
      float v = sl[e];
#pragma unroll
      for (int p = 1; p < NP; ++p) v += sl[p * C * KTOT + e];
      out[e] = v;
    }
    if (tid < C) {
      const float* b = red + 2 * NP * C * KTOT + which * NP * C;
      float v = b[tid];
#pragma unroll
      for (int p = 1; p < NP; ++p) v += b[p * C + tid];
      out[C * KTOT + tid] = v;
    }
  }
}

// NP pairs' tile sets + their flags; the final reduction (2 NP slots of C x KTOT floats +
// biases) reuses the tiles
constexpr size_t res_w88b_smem() { return (size_t)w88b::FLAGS + w88b::NP * 6 * 4; }
static_assert((2 * w88b::NP * C * KTOT + 2 * w88b::NP * C) * 4 <= w88b::FLAGS,
              "reduction slots must fit the tiles");
static_assert(res_w88b_smem() <= 160 * 1024, "LDS");

size_t res_smem(int imgs, int H, int W) {
  const size_t tb = ((size_t)imgs * lay16(H, W).imgb + 15) & ~(size_t)15;
  return 4 * tb + 64;
}

// the wave-owned 8x8 backward runs whole images per wave: any imgs, 4 images per round
bool res_bwd_w88(int H, int W) { return H == 8 && W == 8; }

int res_grid(int N, int H, int W, int imgs) {
  if (res_bwd_w88(H, W)) imgs = w88b::NP;  // NP wave pairs, an image each
  const size_t sm = res_bwd_w88(H, W) ? res_w88b_smem() : res_smem(imgs, H, W);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ncu = cus;
  const void* kfn = res_bwd_w88(H, W) ? (const void*)res_bwd16_w88_kernel
                                       : (const void*)res_bwd16_kernel<0>;  // (every width)
  if (sm > 64 * 1024) (void)hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, res_bwd_w88(H, W) ? w88b::kPT : kThreads,
                                                   sm) != hipSuccess || per < 1)
    per = 1;
  const int nrounds = (N + imgs - 1) / imgs;
  return (int)std::max(1L, std::min((long)nrounds, (long)ncu * mbk_occ_b(per)));
}

}  // namespace

// Number of partial row PAIRS mbk_res_bwd16 writes (= its grid); <= 0: unsupported shape.
extern "C" int mbk_res_bwd16_parts(int N, int H, int W, int imgs) {
  if (N <= 0 || imgs < 1 || H * W > 1024 || (int64_t)imgs * H * W >= (int64_t(1) << 22))
    return -1;
  if (res_smem(imgs, H, W) > 160 * 1024) return -1;
  if ((int64_t)imgs * H * W * 2 > (int64_t)kPF * kThreads * 4) return -1;  // sane staging
  return res_grid(N, H, W, imgs);
}

namespace {

// ------------------------------------------------------------------ fused forward
// Both residual blocks of a 16-channel stage in one launch, saving what the backward needs:
//   u0 = conv0(relu p); y0 = p + conv1(relu u0); u1 = conv2(relu y0); y1 = y0 + conv3(relu u1)
// Writes u0, y0, u1, y1 (bf16) once each and reads p once (5 activation passes instead of the
// per-layer path's 10: every layer re-read its input and the residual from HBM). The stream
// tile Tx holds p, then y0 (updated in place: a conv's residual add touches only its own
// output pixel), the inner tile Tu holds relu(u) for the second conv of each block.
// Accumulation order = conv.hip's conv_fwd chains, so outputs are bit-identical.
struct ResFwdArgs {
  const bf16* p;                 // [N][H][W][16] block-pair input
  bf16 *u0, *y0, *u1, *y1;       // outputs (saved activations + stage output)
  const bf16* w[4];              // packed fwd weights [16][5][32] of conv0..conv3
  const float* b[4];             // fp32 biases
  int N, H, W, imgs;
  // STAGE: the next stage's conv (16 -> 32, no input relu) + max_pool2d(3, 2, 1) on y1 while
  // it is in LDS: ps [N][Ho][Wo][32] pooled output, pidx its argmax bytes (may be null)
  const bf16* ws;                // packed fwd weights [32][5][32]
  const float* bs;
  bf16* ps;
  uint8_t* pidx;
  int* queue = nullptr;          // wave-owned 8x8 form: per-wave image queue (common.h)
};

// STAGE: + the next ConvSequence's conv and pool (conv.hip conv_fwd<16, 32> with its pooled
// epilogue, bit-identical): its input y1 never goes back through HBM and the 8x8 maps'
// launch (profile 20: ~1.5 ms per 524K frames, latency-bound at 4 images per group) is gone.
// The pre-pool staging tile aliases Tu (relu(u1) is dead after conv3).
template <int WC, bool STAGE>
__global__ __launch_bounds__(kThreads) void res_fwd16_kernel(ResFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, W = WC > 0 ? WC : a.W, HW = H * W, Hp = H + 2, Wp = W + 2;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const Lay16 L = lay16(H, W);  // res_bwd16's bank-conflict-free layout for 8-wide maps
  const int PB = L.pb, RB = L.rowb;
  const int tb = ((a.imgs * L.imgb) + 15) & ~15;
  char* Tx = smem;       // residual stream p -> y0 (raw)
  char* Tu = smem + tb;  // relu(u) of the current block
  for (int e = tid; e < 2 * tb / 16; e += kThreads) ((uint4*)smem)[e] = make_uint4(0, 0, 0, 0);
  Frag8 w[4][NCH];
  float bv[4][4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const uint4* wp = (const uint4*)(a.w[l] + (size_t)li * NCH * 32 + g * 8);
#pragma unroll
    for (int c = 0; c < NCH; ++c) w[l][c].u = wp[c * 4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[l][i] = a.b[l][4 * g + i];
  }
  int coff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int tap = 2 * c + (g >> 1), tapc = tap < 9 ? tap : 8;
    coff[c] = (tapc / 3) * RB + (tapc % 3) * PB + 16 * (g & 1);
  }
  const int per = a.imgs * HW * 2;
  const int nrounds = (a.N + a.imgs - 1) / a.imgs;
  uint4 pp[kPF];
  auto prefetch = [&](int rd) {
    const int lim = min(per, (a.N - rd * a.imgs) * HW * 2);
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int e = tid + k * kThreads;
      pp[k] = e < lim ? ((const uint4*)a.p)[(size_t)rd * per + e] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lds_off = [&](int e) {
    const int q = e & 1, p = e >> 1;
    const int im = (int)(((float)p + 0.5f) * inv_hw), r = p - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
    return im * L.imgb + (y + 1) * RB + (x + 1) * PB + q * 16;
  };
  if ((int)blockIdx.x < nrounds) prefetch(blockIdx.x);
  __syncthreads();
  for (int rd = blockIdx.x; rd < nrounds; rd += gridDim.x) {
    const int img0 = rd * a.imgs, nimg = min(a.imgs, a.N - img0);
    const int lim = nimg * HW * 2;
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int e = tid + k * kThreads;
      if (e < lim) *(uint4*)(Tx + lds_off(e)) = pp[k];
    }
    for (int e = tid + kPF * kThreads; e < lim; e += kThreads)
      *(uint4*)(Tx + lds_off(e)) = ((const uint4*)a.p)[(size_t)rd * per + e];
    __syncthreads();
    if (rd + (int)gridDim.x < nrounds) prefetch(rd + gridDim.x);
    const int M = nimg * HW, nblk = (M + 15) >> 4;
    const size_t gpix0 = (size_t)img0 * HW;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const bool inner = (l & 1) == 0;  // conv0 / conv2: relu(Tx) -> u;  conv1 / conv3: + Tx
      const char* src = inner ? Tx : Tu;
      bf16* gout = l == 0 ? a.u0 : l == 1 ? a.y0 : l == 2 ? a.u1 : a.y1;
      for (int pb = wave; pb < nblk; pb += kThreads / 64) {
        const int m = pb * 16 + li;
        const bool valid = m < M;
        const int mm = valid ? m : 0;
        const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        const int base = im * L.imgb + y * RB + x * PB;  // byte offset of tap (0, 0)
        const char* bp = src + base;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          Frag8 av;
          av.u = *(const uint4*)(bp + coff[c]);
          if (inner) av.u = relu8(av.u);  // Tu already holds relu(u)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[l][c].v, av.v, acc, 0, 0, 0);
        }
        if (!valid) continue;
        const int o = base + RB + PB + 4 * g * 2;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[i] + bv[l][i];
        if (!inner) {
          const uint2 ad = *(const uint2*)(Tx + o);
          v[0] += lo_f(ad.x); v[1] += hi_f(ad.x); v[2] += lo_f(ad.y); v[3] += hi_f(ad.y);
        }
        const uint2 out = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        *(uint2*)(gout + (gpix0 + m) * C + 4 * g) = out;
        if (inner) *(uint2*)(Tu + o) = make_uint2(relu2(out.x), relu2(out.y));
        else if (l == 1 || STAGE) *(uint2*)(Tx + o) = out;  // y0 (y1) replaces the stream
      }
      __syncthreads();
    }
    if constexpr (STAGE) {
      // ---- next stage's conv (16 -> 32) over y1 in Tx -> bf16 staging (Tu) -> pooled output
      // (12-wide maps, BASELINE config 4's 24x24 stage 0: unpadded rows, so the staging still
      // fits the relu(u) tile it aliases: 12 x 12 x 64 B <= 14 x 14 x 48 B)
      constexpr int NB = 2, OSTR = WC == 12 ? 2 * C : 2 * C + 4;
      bf16* otile = (bf16*)Tu;
      Frag8 ws[NCH][NB];  // L2 reads per round (10 KB, every workgroup): keeps the persistent
      float bsv[NB][4];   // registers at the 4-layer set (occupancy 3 waves / SIMD)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const uint4* wp = (const uint4*)(a.ws + (size_t)(nb * 16 + li) * NCH * 32 + g * 8);
#pragma unroll
        for (int c = 0; c < NCH; ++c) ws[c][nb].u = wp[c * 4];
#pragma unroll
        for (int i = 0; i < 4; ++i) bsv[nb][i] = a.bs[nb * 16 + 4 * g + i];
      }
      for (int pb = wave; pb < nblk; pb += kThreads / 64) {
        const int m = pb * 16 + li;
        const bool valid = m < M;
        const int mm = valid ? m : 0;
        const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        const char* bp = Tx + im * L.imgb + y * RB + x * PB;
        f32x4 acc[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          Frag8 av;
          av.u = *(const uint4*)(bp + coff[c]);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws[c][nb].v, av.v, acc[nb], 0, 0, 0);
        }
        if (!valid) continue;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          *(uint2*)(otile + m * OSTR + nb * 16 + 4 * g) =
              make_uint2(pack2(acc[nb][0] + bsv[nb][0], acc[nb][1] + bsv[nb][1]),
                         pack2(acc[nb][2] + bsv[nb][2], acc[nb][3] + bsv[nb][3]));
      }
      __syncthreads();
      const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
      mbk::pool_tile<2 * C, OSTR, kThreads>(otile, H, W, nimg, (size_t)img0 * Ho * Wo * 2 * C,
                                            a.ps, a.pidx, tid);
      __syncthreads();  // Tu / Tx reads done before the next round restages them
      // (Tu's halo ring, which the staging overwrote, is never read before conv0 rewrites the
      // interior... the halo must be zero for conv1's taps: restored below)
      for (int e = tid; e < tb / 16; e += kThreads) ((uint4*)Tu)[e] = make_uint4(0, 0, 0, 0);
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ wave-owned forward (8x8)
// res_fwd16_kernel for IMPALA stage 0 at 16x16 (8x8 maps): every wave owns whole images, so
// the kernel has no workgroup barrier. Profile r5a (PMC, learner_only): the generic kernel
// issued ~13 VALU per MFMA -- per 16-pixel block and layer ~20 for the runtime pixel ->
// (image, y, x) split, 20 v_pk_max for relu on every tap fragment of conv0 / conv2, ~15 in
// the epilogue -- at 14.9 % MFMA, and its 5 barriers per round of 4 images left the waves
// parked half of their cycles. Here:
//  * a wave runs the 4 convs (+ the stage conv and pool) of one image at a time in its own
//    LDS tiles: the taps another row pair needs were written by the same wave, whose LDS
//    accesses complete in issue order, so nothing synchronises with the other waves;
//  * a 16-pixel block is a map row pair, so block j's offsets are the lane's own offset plus
//    j * 2 rows: instruction immediates, no per-block address math;
//  * the residual stream is staged twice, raw (Tx: the residual adds, the stage conv) and
//    relu'd (Tr: conv0 / conv2's taps), the relu applied once per pixel at staging and in
//    conv1's epilogue instead of once per tap read;
//  * block j + 1's tap fragments are read while block j's MFMA chain runs;
//  * the next image's input is loaded into registers during the current image.
// Same accumulation order and rounding as conv.hip conv_fwd: bit-identical outputs (test).
template <bool STAGE>
__global__ __launch_bounds__(kThreads) void res_fwd16_w88_kernel(ResFwdArgs a) {
  using namespace w88;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  char* R = smem + wave * REG;  // this wave's tiles
  for (int e = lane; e < REG / 16; e += 64) ((uint4*)R)[e] = make_uint4(0, 0, 0, 0);
  Frag8 w[4][NCH];
  float bv[4][4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const uint4* wp = (const uint4*)(a.w[l] + (size_t)li * NCH * 32 + g * 8);
#pragma unroll
    for (int c = 0; c < NCH; ++c) w[l][c].u = wp[c * 4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[l][i] = a.b[l][4 * g + i];
  }
  // STAGE: the next stage's conv weights stay in registers too (an L2 reload per image left
  // that conv's first MFMAs waiting on it)
  constexpr int NB = 2;
  Frag8 ws[NCH][NB];
  float bsv[NB][4];
  if constexpr (STAGE) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const uint4* wp = (const uint4*)(a.ws + (size_t)(nb * 16 + li) * NCH * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH; ++c) ws[c][nb].u = wp[c * 4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bsv[nb][i] = a.bs[nb * 16 + 4 * g + i];
    }
  }
  // this lane's pixel of block 0 (row li / 8, column li % 8): tap (0, 0) offset per K chunk
  const int lb = (li >> 3) * RB + (li & 7) * PB;
  int aoff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int tap = 2 * c + (g >> 1), tapc = tap < 9 ? tap : 8;
    aoff[c] = lb + (tapc / 3) * RB + (tapc % 3) * PB + 16 * (g & 1);
  }
  const int ob = lb + RB + PB + 8 * g;              // output pixel (interior), channels 4g..
  const uint32_t goff = (uint32_t)(li * C + 4 * g) * 2;  // its bytes in a block's HBM rows
  // staging: this lane's two 16-byte chunks of an image (pixel e / 2, channel half e % 2)
  int so[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = lane + 64 * k, px = e >> 1;
    so[k] = ((px >> 3) + 1) * RB + ((px & 7) + 1) * PB + (e & 1) * 16;
  }
  const int nw = gridDim.x * (kThreads / 64);
  // images: a static stride, or (a.queue) the next tickets of the per-wave queue; the next
  // image's ticket and rows are in flight during the current one
  int* const q = a.queue;
  int cend = 0;
  int img = q ? mbk::wave_next_item(q, -1, cend, a.N) : (int)blockIdx.x * (kThreads / 64) + wave;
  int nxt = q ? (img < a.N ? mbk::wave_next_item(q, img, cend, a.N) : a.N) : img + nw, nn = a.N;
  uint4 pp[2];
  auto fetch = [&](int im) {
    const uint4* src = (const uint4*)(a.p + (size_t)im * HW * C);
    pp[0] = src[lane];
    pp[1] = src[lane + 64];
  };
  if (img < a.N) fetch(img);
  for (; img < a.N; img = nxt, nxt = nn) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      *(uint4*)(R + TX + so[k]) = pp[k];
      *(uint4*)(R + TR + so[k]) = relu8(pp[k]);
    }
    if (nxt < a.N) fetch(nxt);
    nn = q ? (nxt < a.N ? mbk::wave_next_item(q, nxt, cend, a.N) : a.N) : nxt + nw;
    wave_lds_order();
    const size_t gpix = (size_t)img * HW;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const bool inner = (l & 1) == 0;  // conv0 / conv2: Tr -> u;  conv1 / conv3: Tu, + Tx
      const int src = inner ? TR : TU;
      char* gw = (char*)((l == 0 ? a.u0 : l == 1 ? a.y0 : l == 2 ? a.u1 : a.y1) + gpix * C);
      f32x4 acc[4];
      Frag8 fr[2][NCH];
#pragma unroll
      for (int c = 0; c < NCH; ++c) fr[0][c].u = *(const uint4*)(R + src + aoff[c]);
      // software pipeline in issue order: each MFMA of block j, then one tap read of block
      // j + 1 (hipcc's scheduler otherwise reuses one fragment register and waits for every
      // read); the scheduling barriers keep this order, the waitcnt pass then waits only for
      // the oldest of the five reads in flight
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              w[l][c].v, fr[j & 1][c].v, c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[j], 0, 0, 0);
          if (j + 1 < 4)
            fr[(j + 1) & 1][c].u = *(const uint4*)(R + src + (j + 1) * 2 * RB + aoff[c]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = j * 2 * RB + ob;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[j][i] + bv[l][i];
        if (!inner) {
          const uint2 ad = *(const uint2*)(R + TX + o);
          v[0] += lo_f(ad.x); v[1] += hi_f(ad.x); v[2] += lo_f(ad.y); v[3] += hi_f(ad.y);
        }
        const uint2 out = make_uint2(cvt_pk2(v[0], v[1]), cvt_pk2(v[2], v[3]));
        *(uint2*)(gw + j * 16 * C * 2 + goff) = out;
        const uint2 rl = make_uint2(relu2(out.x), relu2(out.y));
        if (inner) {
          *(uint2*)(R + TU + o) = rl;
        } else if (l == 1) {  // y0: the residual of conv3 (raw) and conv2's input (relu'd)
          *(uint2*)(R + TX + o) = out;
          *(uint2*)(R + TR + o) = rl;
        } else if (STAGE) {
          *(uint2*)(R + TX + o) = out;  // y1: the stage conv's input (no relu)
        }
      }
      wave_lds_order();
    }
    if constexpr (STAGE) {
      // next stage's conv (16 -> 32) over y1 in Tx -> bf16 staging (aliases Tu) -> pooled output
      constexpr int OSTR = 2 * C + 4;
      static_assert(HW * OSTR * 2 <= IMGB, "pre-pool staging must fit the relu(u) tile");
      bf16* otile = (bf16*)(R + TU);
      Frag8 fr[2][NCH];
#pragma unroll
      for (int c = 0; c < NCH; ++c) fr[0][c].u = *(const uint4*)(R + TX + aoff[c]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 ac2[NB];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {  // (the conv layers' software pipeline)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            ac2[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                ws[c][nb].v, fr[j & 1][c].v, c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : ac2[nb], 0,
                0, 0);
          if (j + 1 < 4)
            fr[(j + 1) & 1][c].u = *(const uint4*)(R + TX + (j + 1) * 2 * RB + aoff[c]);
          __builtin_amdgcn_sched_barrier(0);
        }
        const int m = j * 16 + li;  // pixel of the image
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          *(uint2*)(otile + m * OSTR + nb * 16 + 4 * g) =
              make_uint2(cvt_pk2(ac2[nb][0] + bsv[nb][0], ac2[nb][1] + bsv[nb][1]),
                         cvt_pk2(ac2[nb][2] + bsv[nb][2], ac2[nb][3] + bsv[nb][3]));
      }
      wave_lds_order();
      constexpr int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
      mbk::pool_tile<2 * C, OSTR, 64>(otile, H, W, 1, (size_t)img * Ho * Wo * 2 * C, a.ps, a.pidx,
                                      lane);
      wave_lds_order();
      // restore Tu's halo ring (conv1 / conv3 read it as zero padding): rows 0 and 9 (10
      // pixels each) and columns 0 and 9 of rows 1-8, 32 B per pixel
      if (lane < 36) {
        const int q = lane;
        const int off = q < 10 ? q * PB : q < 20 ? 9 * RB + (q - 10) * PB
                      : q < 28 ? (q - 19) * RB : (q - 27) * RB + 9 * PB;
        *(uint4*)(R + TU + off) = make_uint4(0, 0, 0, 0);
        *(uint4*)(R + TU + off + 16) = make_uint4(0, 0, 0, 0);
      }
      wave_lds_order();
    }
  }
  if (q) mbk::wave_queue_done(q, nw);
}

// One 32-channel residual block per launch (stages 1-2 of the IMPALA trunk):
//   u = conv0(relu x); y = x + conv1(relu u)
// x is staged once into a halo'd LDS tile (and serves as the residual), relu(u) stays in
// LDS for conv1; u and y are written once (3 activation passes instead of the per-layer
// path's 5). Both layers' weight fragments (2 x 9 K-chunks x 2 output blocks) stay in VGPRs
// for the whole persistent launch; all four 32-channel layers would not fit. Accumulation
// order = conv.hip's conv_fwd<32, 32> chains, so outputs are bit-identical to it.
constexpr int C32 = 32, PIXB32 = C32 * 2 + 16, NCH32 = 9, NB32 = 2;

struct Geo32f {
  int pb, rs, is;
};

struct ResBlk32Args {
  const bf16* x;     // [N][H][W][32] block input (pre-relu)
  bf16 *u, *y;       // outputs
  const bf16* w[2];  // packed fwd weights [32][9][32] of conv0, conv1
  const float* b[2];
  int N, H, W, imgs;
  int* queue = nullptr;  // res_blk32_wave_kernel: per-wave queue of 16-pixel blocks (common.h)
};

// Tile geometry (halo'd pixel (hy, hx) of image im at im * is + hy * rs + hx * pb). 4-wide maps
// (stage 1 at 16x16): 64-byte pixels in 416-byte rows (= 32 mod 64): the 16 B tap reads of a
// ds_read_b128 lane group -- 4 pixels of each of the image's 4 rows, two channel chunks --
// start at 16 distinct 16-byte slots of the 256-byte bank window (the generic 80-byte pixels:
// 32 % bank conflicts, profile 40)
__host__ __device__ inline Geo32f geo32f(int H, int W) {
  if (W == 4) return {64, 416, ((H + 1) * 416 + (W + 2) * 64 + 15) & ~15};
  return {PIXB32, (W + 2) * PIXB32, (H + 2) * (W + 2) * PIXB32};
}

template <int WC>
__global__ __launch_bounds__(kThreads) void res_blk32_kernel(ResBlk32Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, W = WC > 0 ? WC : a.W, HW = H * W;
  const Geo32f G3 = geo32f(H, W);
  const int PB = WC == 4 ? 64 : G3.pb, RS = WC == 4 ? 416 : G3.rs, IS = G3.is;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int tb = ((a.imgs * IS) + 15) & ~15;
  char* Tx = smem;       // x (raw): conv0's input (relu at read) and the residual
  char* Tu = smem + tb;  // relu(u): conv1's input
  for (int e = tid; e < 2 * tb / 16; e += kThreads) ((uint4*)smem)[e] = make_uint4(0, 0, 0, 0);
  Frag8 w[2][NCH32][NB32];
  float bv[2][NB32][4];
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int nb = 0; nb < NB32; ++nb) {
      const uint4* wp = (const uint4*)(a.w[l] + (size_t)(nb * 16 + li) * NCH32 * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH32; ++c) w[l][c][nb].u = wp[c * 4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[l][nb][i] = a.b[l][nb * 16 + 4 * g + i];
    }
  int coff[NCH32];  // K chunk c = tap c, channels 8g.. of this lane
#pragma unroll
  for (int c = 0; c < NCH32; ++c) coff[c] = (c / 3) * RS + (c % 3) * PB + 16 * g;
  constexpr int EPP = C32 / 8;  // uint4 per pixel
  const int per = a.imgs * HW * EPP;
  const int nrounds = (a.N + a.imgs - 1) / a.imgs;
  auto lds_off = [&](int e) {
    const int q = e & (EPP - 1), p = e / EPP;
    const int im = (int)(((float)p + 0.5f) * inv_hw), r = p - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
    return im * IS + (y + 1) * RS + (x + 1) * PB + q * 16;
  };
  // The next round's x is fetched into registers while this round computes (when a round
  // is at most kPF uint4 per thread), so the global-load latency leaves the critical path.
  constexpr int kPF = 4;
  const bool pf_ok = per <= kPF * kThreads;
  uint4 pf0, pf1, pf2, pf3;
#define MBK_RB32_FETCH(RD)                                                        \
  {                                                                               \
    const int lim_ = min(a.imgs, a.N - (RD) * a.imgs) * HW * EPP;                 \
    const uint4* src_ = (const uint4*)a.x + (size_t)(RD) * per + tid;             \
    if (tid < lim_) pf0 = src_[0];                                                \
    if (tid + kThreads < lim_) pf1 = src_[kThreads];                              \
    if (tid + 2 * kThreads < lim_) pf2 = src_[2 * kThreads];                      \
    if (tid + 3 * kThreads < lim_) pf3 = src_[3 * kThreads];                      \
  }
  if (pf_ok && (int)blockIdx.x < nrounds) MBK_RB32_FETCH((int)blockIdx.x)
  __syncthreads();
  for (int rd = blockIdx.x; rd < nrounds; rd += gridDim.x) {
    const int img0 = rd * a.imgs, nimg = min(a.imgs, a.N - img0);
    const int lim = nimg * HW * EPP;
    if (pf_ok) {
      if (tid < lim) *(uint4*)(Tx + lds_off(tid)) = pf0;
      if (tid + kThreads < lim) *(uint4*)(Tx + lds_off(tid + kThreads)) = pf1;
      if (tid + 2 * kThreads < lim) *(uint4*)(Tx + lds_off(tid + 2 * kThreads)) = pf2;
      if (tid + 3 * kThreads < lim) *(uint4*)(Tx + lds_off(tid + 3 * kThreads)) = pf3;
    } else {
      for (int e = tid; e < lim; e += kThreads)
        *(uint4*)(Tx + lds_off(e)) = ((const uint4*)a.x)[(size_t)rd * per + e];
    }
    __syncthreads();
    if (pf_ok && rd + (int)gridDim.x < nrounds) MBK_RB32_FETCH(rd + (int)gridDim.x)
    const int M = nimg * HW, nblk = (M + 15) >> 4;
    const size_t gpix0 = (size_t)img0 * HW;
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const char* src = l == 0 ? Tx : Tu;
      bf16* gout = l == 0 ? a.u : a.y;
      for (int pb = wave; pb < nblk; pb += kThreads / 64) {
        const int m = pb * 16 + li;
        const bool valid = m < M;
        const int mm = valid ? m : 0;
        const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        const int base = im * IS + y * RS + x * PB;
        const char* bp = src + base;
        f32x4 acc[NB32];
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NCH32; ++c) {
          Frag8 av;
          av.u = *(const uint4*)(bp + coff[c]);
          if (l == 0) av.u = relu8(av.u);  // Tu already holds relu(u)
#pragma unroll
          for (int nb = 0; nb < NB32; ++nb)
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[l][c][nb].v, av.v, acc[nb], 0, 0, 0);
        }
        if (!valid) continue;
        const int o = base + RS + PB;
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) {
          const int co0 = nb * 16 + 4 * g;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[nb][i] + bv[l][nb][i];
          if (l == 1) {
            const uint2 ad = *(const uint2*)(Tx + o + co0 * 2);
            v[0] += lo_f(ad.x); v[1] += hi_f(ad.x); v[2] += lo_f(ad.y); v[3] += hi_f(ad.y);
          }
          const uint2 out = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          *(uint2*)(gout + (gpix0 + m) * C32 + co0) = out;
          if (l == 0) *(uint2*)(Tu + o + co0 * 2) = make_uint2(relu2(out.x), relu2(out.y));
        }
      }
      __syncthreads();
    }
  }
}

#undef MBK_RB32_FETCH

// The same block on 4x4 and 2x2 maps (IMPALA stages 1 / 2 at 16x16) with wave-owned 16-pixel
// blocks: one MFMA block is one 4x4 image or four 2x2 images, so a wave stages its block
// (1 KB: one uint4 per lane, prefetched a block ahead), runs conv0 -> relu(u) in its own LDS
// tile -> conv1 + the residual, and never meets a workgroup barrier (the round form spent most
// of its time in three barriers per round and its staging: ~2.8 us per 16-image round on 2x2
// maps for 36 MFMAs per wave). Both layers' weights stay in VGPRs for the launch; chains and
// epilogues are res_blk32_kernel's, so bit-identical to it.
namespace rbw {
constexpr int NW = 4, kPT = 64 * NW;
constexpr int PB = 64;  // 64-byte pixels
// MW = 4: one halo'd 6x6 image, 416-byte rows; MW = 2: four halo'd 4x4 images, 288-byte rows,
// 1152 bytes apart. Both put the 16 pixels of a tap read's lane groups on distinct bank slots
// (tools/lds_banks.py model: 1.0 cycles per group; 4.0 for 256-byte rows / 1024-byte images).
template <int MW> struct Geo;
template <> struct Geo<4> { static constexpr int RS = 416, IS = 0, TB = (5 * 416 + 6 * 64 + 15) & ~15; };
template <> struct Geo<2> { static constexpr int RS = 288, IS = 4 * 288, TB = 4 * 4 * 288; };
template <int MW> constexpr int smem() { return NW * 2 * Geo<MW>::TB; }
}  // namespace rbw

template <int MW>
__global__ __launch_bounds__(rbw::kPT) void res_blk32_wave_kernel(ResBlk32Args a) {
  using namespace rbw;
  constexpr int RS = Geo<MW>::RS, IS = Geo<MW>::IS, TB = Geo<MW>::TB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  char* Tx = smem + wave * 2 * TB;
  char* Tu = Tx + TB;
  for (int e = lane; e < 2 * TB / 16; e += 64) ((uint4*)Tx)[e] = make_uint4(0, 0, 0, 0);
  Frag8 w[2][NCH32][NB32];
  float bv[2][NB32][4];
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int nb = 0; nb < NB32; ++nb) {
      const uint4* wp = (const uint4*)(a.w[l] + (size_t)(nb * 16 + li) * NCH32 * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH32; ++c) w[l][c][nb].u = wp[c * 4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[l][nb][i] = a.b[l][nb * 16 + 4 * g + i];
    }
  // pixel p (0..15) of the block: image, row, column inside the halo'd tile set
  auto pix = [](int p) {
    return MW == 4 ? (p >> 2) * RS + (p & 3) * PB
                   : (p >> 2) * IS + ((p >> 1) & 1) * RS + (p & 1) * PB;
  };
  const int pbase = pix(li);        // MFMA lanes: pixel li, tap (0, 0) of its window
  const int pout = pbase + RS + PB;  // the pixel itself
  // staging lanes: uint4 #lane of the block = pixel lane / 4, 16-byte chunk lane % 4
  const int sofs = pix(lane >> 2) + RS + PB + 16 * (lane & 3);
  const int64_t npix = (int64_t)a.N * MW * MW;
  const int nq = (int)((npix + 15) >> 4);
  const int step = gridDim.x * NW;
  // blocks: a static stride, or (a.queue) the per-wave queue's chunks (next block in flight)
  int* const wq = a.queue;
  int cend = 0;
  const int first = wq ? mbk::wave_next_item(wq, -1, cend, nq) : (int)blockIdx.x * NW + wave;
  int nxt = wq ? (first < nq ? mbk::wave_next_item(wq, first, cend, nq) : nq) : first + step;
  int nn = nq;
  uint4 pf;
  auto fetch = [&](int q) {
    const int64_t e = (int64_t)q * 64 + lane;  // uint4 index (4 per pixel)
    pf = e < npix * 4 ? ((const uint4*)a.x)[e] : make_uint4(0, 0, 0, 0);
  };
  wave_lds_order();
  if (first < nq) fetch(first);
  for (int q = first; q < nq; q = nxt, nxt = nn) {
    *(uint4*)(Tx + sofs) = pf;
    if (nxt < nq) fetch(nxt);
    nn = wq ? (nxt < nq ? mbk::wave_next_item(wq, nxt, cend, nq) : nq) : nxt + step;
    wave_lds_order();
    const int64_t m = (int64_t)q * 16 + li;  // global pixel of this lane
    const bool valid = m < npix;
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const char* src = (l == 0 ? Tx : Tu) + pbase;
      f32x4 acc[NB32];
#pragma unroll
      for (int nb = 0; nb < NB32; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NCH32; ++c) {
        Frag8 av;
        av.u = *(const uint4*)(src + (c / 3) * RS + (c % 3) * PB + 16 * g);
        if (l == 0) av.u = relu8(av.u);  // Tu already holds relu(u)
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb)
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[l][c][nb].v, av.v, acc[nb], 0, 0, 0);
      }
      bf16* gout = l == 0 ? a.u : a.y;
#pragma unroll
      for (int nb = 0; nb < NB32; ++nb) {
        const int co0 = nb * 16 + 4 * g;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[nb][i] + bv[l][nb][i];
        if (l == 1) {
          const uint2 ad = *(const uint2*)(Tx + pout + co0 * 2);
          v[0] += lo_f(ad.x); v[1] += hi_f(ad.x); v[2] += lo_f(ad.y); v[3] += hi_f(ad.y);
        }
        const uint2 out = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if (valid) *(uint2*)(gout + m * C32 + co0) = out;
        if (l == 0) *(uint2*)(Tu + pout + co0 * 2) = make_uint2(relu2(out.x), relu2(out.y));
      }
      wave_lds_order();
    }
  }
  if (wq) mbk::wave_queue_done(wq, step);
}

// ------------------------------------------------------------------ fused backward, 32 ch
// Backward of one 32-channel residual block (stages 1-2), the res_bwd16 dataflow
// (x, u, g staged once; du kept in LDS; dx written once) with the 32-channel operands split
// over 8 waves so that no wave holds more than one layer's weights and 9 wgrad tiles:
//   phase A: waves 0-3  du = conv1^T(g) * [u > 0] -> Td   (conv1 dgrad weights in VGPRs)
//            waves 4-7  dW1[cb][cib] += relu(u) (x) g      (9 tap tiles each)
//   phase B: waves 4-7  dx = conv0^T(du) * [x > 0] + g     (conv0 dgrad weights in VGPRs)
//            waves 0-3  dW0[cb][cib] += relu(x) (x) du
// (cb, cib) = this wave's 16-channel output / input block of the 32 x 32 weight, so every
// weight-gradient tile has exactly one owner: no cross-wave reduction, partial rows are
// written straight from the accumulators. dgrad = conv_fwd<32, 32> chains on the packed
// transposed weights (bit-identical du / dx to the per-layer kernels); wgrad = the
// ds_read_b64_tr_b16 operand form of res_bwd16 / conv_wgrad.
constexpr int kT32 = 512;                      // 8 waves
constexpr int KTOT32 = 9 * C32;                // wgrad K per output channel
constexpr int ROW32 = C32 * KTOT32 + C32;      // one partial row (weights + bias)
constexpr int kPF32 = 2;                       // staging prefetch slots per thread per tensor

struct ResBwd32Args {
  const bf16* x;     // block input (pre-relu)      [N][H][W][32]
  const bf16* u;     // conv0 output (pre-relu)     [N][H][W][32]
  const bf16* g;     // dL/dy                        [N][H][W][32]
  bf16* dx;          // dL/dx                        [N][H][W][32]
  const bf16* w1t;   // conv1 packed dgrad weights [32][9][32]
  const bf16* w0t;   // conv0 packed dgrad weights
  float* partial;    // layer l (0: conv1, 1: conv0) row of workgroup b at l * lstride + b * ROW32
  int64_t lstride;
  int N, H, W, imgs;
};

// Tile geometry: halo'd pixel (hy, hx) of image im at im * is + hy * rs + hx * pb. 4-wide maps
// (IMPALA stage 1 at 16x16): unpadded 64-byte pixels in 400-byte rows, so the 4 pixels of a
// transposed read's lane group span 4 x 64 B and the group two map rows down starts 800 = 32
// (mod 256) bytes later: a half-wave's 8 x 32 B reads cover 256 distinct bytes (the 80-byte
// pixels of the generic layout overlapped: 32.8 % bank conflicts, profile 40)
struct Geo32 {
  int pb, rs, is;
};
__host__ __device__ inline Geo32 geo32(int H, int W) {
  if (W == 4) return {64, 400, ((H + 1) * 400 + (W + 2) * 64 + 15) & ~15};
  return {PIXB32, (W + 2) * PIXB32, (H + 2) * (W + 2) * PIXB32};
}

template <int WC>
__global__ __launch_bounds__(kT32) void res_bwd32_kernel(ResBwd32Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, W = WC > 0 ? WC : a.W, HW = H * W;
  const Geo32 G3 = geo32(H, W);
  const int PB = WC == 4 ? 64 : G3.pb, RS = WC == 4 ? 400 : G3.rs, IS = G3.is;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const bool lo = wave < 4;          // waves 0-3: dgrad1 (A) + wgrad0 (B)
  const int wq = wave & 3;           // rank inside the half
  const int cb = wq >> 1, cib = wq & 1;
  const int tb = ((a.imgs * IS) + 15) & ~15;
  char* Tg = smem;
  char* Tu = smem + tb;       // relu(u)
  char* Tx = smem + 2 * tb;   // relu(x)
  char* Td = smem + 3 * tb;   // du
  char* zero = smem + 4 * tb; // 128 zero bytes for out-of-range wgrad pixels
  for (int e = tid; e < (4 * tb + 128) / 16; e += kT32) ((uint4*)smem)[e] = make_uint4(0, 0, 0, 0);

  // this wave's dgrad weights (lane: rows nb * 16 + li, chunk c, elements 8g..8g+7)
  Frag8 w[NCH32][NB32];
  {
    const bf16* wt = lo ? a.w1t : a.w0t;
#pragma unroll
    for (int nb = 0; nb < NB32; ++nb) {
      const uint4* wp = (const uint4*)(wt + (size_t)(nb * 16 + li) * NCH32 * 32 + g * 8);
#pragma unroll
      for (int c = 0; c < NCH32; ++c) w[c][nb].u = wp[c * 4];
    }
  }
  f32x4 acc[9];  // this wave's wgrad tiles (tap t): rows co = cb*16 + 4g + i, cols ci = cib*16 + li
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  int coff[NCH32];  // K chunk c = tap c, channels 8g.. of this lane
#pragma unroll
  for (int c = 0; c < NCH32; ++c) coff[c] = (c / 3) * RS + (c % 3) * PB + 16 * g;
  float db1[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // sum g: channels 8 (tid & 3) .. +8 (staging)
  float db0[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // sum du: channels nb*16 + 4g + i (waves 0-3)

  constexpr int EPP = C32 / 8;
  const int per = a.imgs * HW * EPP;  // uint4 per tensor per round
  const int nrounds = (a.N + a.imgs - 1) / a.imgs;
  uint4 px[kPF32], pu[kPF32], pg[kPF32];
  auto prefetch = [&](int rd) {
    const int lim = min(per, (a.N - rd * a.imgs) * HW * EPP);
    const size_t base = (size_t)rd * per;
#pragma unroll
    for (int k = 0; k < kPF32; ++k) {
      const int e = tid + k * kT32;
      const bool ok = e < lim;
      px[k] = ok ? ((const uint4*)a.x)[base + e] : make_uint4(0, 0, 0, 0);
      pu[k] = ok ? ((const uint4*)a.u)[base + e] : make_uint4(0, 0, 0, 0);
      pg[k] = ok ? ((const uint4*)a.g)[base + e] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lds_off = [&](int e) {
    const int q = e & (EPP - 1), p = e / EPP;
    const int im = (int)(((float)p + 0.5f) * inv_hw), r = p - im * HW;
    const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
    return im * IS + (y + 1) * RS + (x + 1) * PB + q * 16;
  };
  auto put = [&](int e, uint4 vx, uint4 vu, uint4 vg) {
    const int o = lds_off(e);
    *(uint4*)(Tx + o) = relu8(vx);
    *(uint4*)(Tu + o) = relu8(vu);
    *(uint4*)(Tg + o) = vg;
    const uint32_t wv[4] = {vg.x, vg.y, vg.z, vg.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      db1[2 * j] += lo_f(wv[j]);
      db1[2 * j + 1] += hi_f(wv[j]);
    }
  };
  // wgrad K block kb (32 pixels) of this wave's tile: dY tile D (block cb), X taps from X
  auto wgrad_kb = [&](int kb, int M, const char* D, const char* X) {
    const char* dptr[2];
    int xpos[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = kb * 32 + 8 * g + 4 * h + (li >> 2);
      const bool ok = p < M;
      const int pp = ok ? p : 0;
      const int im = (int)(((float)pp + 0.5f) * inv_hw), r = pp - im * HW;
      const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
      xpos[h] = im * IS + y * RS + x * PB;  // byte offset of the pixel's window top-left
      dptr[h] = ok ? D + xpos[h] + RS + PB + cb * 32 : zero;
    }
    Frag8 af;
#pragma unroll
    for (int h = 0; h < 2; ++h) af.h[h] = tr_read(dptr[h] + (4 * (li & 3)) * 2);
    // out-of-range pixels read pixel 0's (finite) X values against a zero dY column
    const char* xb0 = X + xpos[0] + cib * 32 + 8 * (li & 3);
    const char* xb1 = X + xpos[1] + cib * 32 + 8 * (li & 3);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int off = (t / 3) * RS + (t % 3) * PB;
      Frag8 bf;
      bf.h[0] = tr_read(xb0 + off);
      bf.h[1] = tr_read(xb1 + off);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bf.v, acc[t], 0, 0, 0);
    }
  };

  if ((int)blockIdx.x < nrounds) prefetch(blockIdx.x);
  __syncthreads();  // zeroed tiles visible
  for (int rd = blockIdx.x; rd < nrounds; rd += gridDim.x) {
    const int img0 = rd * a.imgs, nimg = min(a.imgs, a.N - img0);
    const int lim = nimg * HW * EPP;
#pragma unroll
    for (int k = 0; k < kPF32; ++k) {
      const int e = tid + k * kT32;
      if (e < lim) put(e, px[k], pu[k], pg[k]);
    }
    for (int e = tid + kPF32 * kT32; e < lim; e += kT32) {
      const size_t s = (size_t)rd * per + e;
      put(e, ((const uint4*)a.x)[s], ((const uint4*)a.u)[s], ((const uint4*)a.g)[s]);
    }
    __syncthreads();
    if (rd + (int)gridDim.x < nrounds) prefetch(rd + gridDim.x);
    const int M = nimg * HW, nblk = (M + 15) >> 4, nk = (M + 31) >> 5;
    const size_t gpix0 = (size_t)img0 * HW;
    // ---------------- phase A
    if (lo) {  // du = conv1^T(g) * [u > 0]
      for (int pb = wq; pb < nblk; pb += 4) {
        const int m = pb * 16 + li;
        const bool valid = m < M;
        const int mm = valid ? m : 0;
        const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        const int base = im * IS + y * RS + x * PB;
        const char* bp = Tg + base;
        f32x4 ac[NB32];
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) ac[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NCH32; ++c) {
          Frag8 av;
          av.u = *(const uint4*)(bp + coff[c]);
#pragma unroll
          for (int nb = 0; nb < NB32; ++nb)
            ac[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[c][nb].v, av.v, ac[nb], 0, 0, 0);
        }
        if (!valid) continue;
        const int o = base + RS + PB;
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) {
          const int co0 = nb * 16 + 4 * g;
          const uint2 mu = *(const uint2*)(Tu + o + co0 * 2);
          const uint32_t mw[2] = {mu.x, mu.y};
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            v[i] = (__uint_as_float(hb << 16) > 0.f) ? ac[nb][i] : 0.f;
          }
          const uint2 du = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          *(uint2*)(Td + o + co0 * 2) = du;
          db0[nb * 4 + 0] += lo_f(du.x); db0[nb * 4 + 1] += hi_f(du.x);
          db0[nb * 4 + 2] += lo_f(du.y); db0[nb * 4 + 3] += hi_f(du.y);
        }
      }
    } else {  // dW1 += relu(u) (x) g
      for (int kb = 0; kb < nk; ++kb) wgrad_kb(kb, M, Tg, Tu);  // this wave's tile: every K block
    }
    __syncthreads();  // Td complete
    // ---------------- phase B
    if (!lo) {  // dx = conv0^T(du) * [x > 0] + g
      for (int pb = wq; pb < nblk; pb += 4) {
        const int m = pb * 16 + li;
        const bool valid = m < M;
        const int mm = valid ? m : 0;
        const int im = (int)(((float)mm + 0.5f) * inv_hw), r = mm - im * HW;
        const int y = (int)(((float)r + 0.5f) * inv_w), x = r - y * W;
        const int base = im * IS + y * RS + x * PB;
        const char* bp = Td + base;
        f32x4 ac[NB32];
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) ac[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NCH32; ++c) {
          Frag8 av;
          av.u = *(const uint4*)(bp + coff[c]);
#pragma unroll
          for (int nb = 0; nb < NB32; ++nb)
            ac[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[c][nb].v, av.v, ac[nb], 0, 0, 0);
        }
        if (!valid) continue;
        const int o = base + RS + PB;
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) {
          const int co0 = nb * 16 + 4 * g;
          const uint2 mx = *(const uint2*)(Tx + o + co0 * 2), ad = *(const uint2*)(Tg + o + co0 * 2);
          const uint32_t mw[2] = {mx.x, mx.y}, aw[2] = {ad.x, ad.y};
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            v[i] = (__uint_as_float(hb << 16) > 0.f) ? ac[nb][i] : 0.f;
            v[i] += __uint_as_float(((aw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) << 16);
          }
          *(uint2*)(a.dx + (gpix0 + m) * C32 + co0) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
    } else {  // dW0 += relu(x) (x) du
      for (int kb = 0; kb < nk; ++kb) wgrad_kb(kb, M, Td, Tx);
    }
    __syncthreads();  // tiles consumed before the next round is staged
  }
  // ---- partial rows: each tile straight from its owner wave (layer 1 = waves 4-7 -> block 0)
  float* out = a.partial + (lo ? a.lstride : 0) + (size_t)blockIdx.x * ROW32;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      out[(cb * 16 + 4 * g + i) * KTOT32 + t * C32 + cib * 16 + li] = acc[t][i];
  // bias grads through LDS (fixed order): red1[tid][8] = db1, red0[tid][8] = db0 (waves 0-3)
  float* red = (float*)smem;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[tid * 16 + j] = db1[j];
    red[tid * 16 + 8 + j] = db0[j];
  }
  __syncthreads();
  if (tid < C32) {
    float s = 0.f;  // conv1 bias: channel tid = 8 q + j lives in threads with (t & 3) == q
    const int q = tid >> 3, j = tid & 7;
    for (int t = q; t < kT32; t += 4) s += red[t * 16 + j];
    a.partial[(size_t)blockIdx.x * ROW32 + C32 * KTOT32 + tid] = s;
    // conv0 bias: channel tid = nb * 16 + 4 G + i lives in waves 0-3, lanes with g == G
    const int nb = tid >> 4, G = (tid & 15) >> 2, i = tid & 3;
    float s0 = 0.f;
    for (int t = 0; t < 256; ++t)
      if (((t & 63) >> 4) == G) s0 += red[t * 16 + 8 + nb * 4 + i];
    a.partial[a.lstride + (size_t)blockIdx.x * ROW32 + C32 * KTOT32 + tid] = s0;
  }
}

// ------------------------------------------------------------------ team backward, 32 ch
// The 32-channel block backward on 4x4 / 2x2 maps (IMPALA stages 1 / 2 at 16x16) without
// workgroup barriers. res_bwd32_kernel ran rounds of 14-29 images with two barriers each (on
// 2x2 maps ~5 us per round for ~36 MFMAs per wave). One wave per role cannot hold a layer's
// 36 weight-gradient tiles next to the dgrad weights, so a TEAM of four waves shares a stream
// of 32-pixel items (two 16-pixel groups: two 4x4 images or eight 2x2 images), each role with
// its own operands in VGPRs for the whole launch:
//   W1 (stager): stages relu(x), relu(u), g of the item (prefetched an item ahead); dW1 +=
//       relu(u) (x) g over the item's 32 pixels (36 tiles + the bias column by an all-ones MFMA)
//   D1: du = conv1^T(g) * [u > 0] -> the item's du tiles (conv1 dgrad weights)
//   D0: dx = conv0^T(du) * [x > 0] + g -> HBM (conv0 dgrad weights)
//   W0: dW0 += relu(x) (x) du (36 tiles + bias)
// over NSET tile sets per team, synchronised by per-team LDS flags holding iteration numbers
// (staged / du written / D0 done / W0 done): a wave's LDS writes complete in issue order, so a
// flag written after the data publishes it, and W1 re-stages a set only once D0 and W0 are done
// with it (D1 finished reading it before it wrote du). Every role walks the same item sequence
// and each wait is on a flag another role sets in that same iteration, so every wave reaches
// the end. du / dx: res_bwd32's chains and epilogues (bit-identical); weight gradients: one
// partial row per team (fp32 order differs from the round kernel's).
namespace rbt {
constexpr int NT = 2, kPT = 64 * 4 * NT;  // teams per workgroup, threads
constexpr int NSET = 2;
constexpr int PB = 64;
template <int MW> constexpr int TB() { return rbw::Geo<MW>::TB; }  // one 16-pixel group's tile
// a set: g, relu(u), relu(x), du tiles of the item's two groups
template <int MW> constexpr int SETB() { return 4 * 2 * TB<MW>(); }
template <int MW> constexpr int TEAMB() { return NSET * SETB<MW>(); }
constexpr int FLAGS_PER_TEAM = 4 * NSET;
template <int MW> constexpr int smem() { return NT * TEAMB<MW>() + NT * FLAGS_PER_TEAM * 4; }
static_assert(smem<2>() <= 160 * 1024 && smem<4>() <= 160 * 1024, "LDS");
}  // namespace rbt

template <int MW>
__global__ __launch_bounds__(rbt::kPT) void res_bwd32_team_kernel(ResBwd32Args a) {
  using namespace rbt;
  constexpr int RS = rbw::Geo<MW>::RS, IS = rbw::Geo<MW>::IS, T = TB<MW>();
  constexpr int OG = 0, OU = 2 * T, OX = 4 * T, OD = 6 * T;  // tensor offsets in a set
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int team = wave >> 2, role = wave & 3;  // 0 W1, 1 D1, 2 D0, 3 W0
  char* base = smem + team * TEAMB<MW>();
  int* fl = (int*)(smem + NT * TEAMB<MW>()) + team * FLAGS_PER_TEAM;  // [kind][set]
  int* f_staged = fl;
  int* f_du = fl + NSET;
  int* f_d0 = fl + 2 * NSET;
  int* f_w0 = fl + 3 * NSET;
  for (int e = tid; e < NT * TEAMB<MW>() / 16; e += kPT) ((uint4*)smem)[e] = make_uint4(0, 0, 0, 0);
  if (tid < NT * FLAGS_PER_TEAM) ((int*)(smem + NT * TEAMB<MW>()))[tid] = 0;
  __syncthreads();  // zeroed tiles (halos) and flags
  auto pix = [](int p) {  // pixel p (0..15) of a group: window top-left inside its tile
    return MW == 4 ? (p >> 2) * RS + (p & 3) * PB
                   : (p >> 2) * IS + ((p >> 1) & 1) * RS + (p & 1) * PB;
  };
  const int64_t npix = (int64_t)a.N * MW * MW;
  const int nitems = (int)((npix + 31) >> 5);
  const int step = gridDim.x * NT;
  const int first = blockIdx.x * NT + team;
  const int pbase = pix(li), pin = pbase + RS + PB;  // dgrad lanes: pixel li of a group

  if (role == 1 || role == 2) {
    // ---- D1 / D0: dgrad weights (lane: rows nb * 16 + li, chunk c, elements 8g..)
    Frag8 w[NCH32][NB32];
    {
      const bf16* wt = role == 1 ? a.w1t : a.w0t;
#pragma unroll
      for (int nb = 0; nb < NB32; ++nb) {
        const uint4* wp = (const uint4*)(wt + (size_t)(nb * 16 + li) * NCH32 * 32 + g * 8);
#pragma unroll
        for (int c = 0; c < NCH32; ++c) w[c][nb].u = wp[c * 4];
      }
    }
    int it = 0;
    for (int item = first; item < nitems; item += step, ++it) {
      const int b = it % NSET;
      char* S = base + b * SETB<MW>();
      wait_flag(role == 1 ? f_staged + b : f_du + b, it + 1);
      wave_lds_order();
      // both groups' chains interleaved: 4 independent accumulators behind each tap read pair
      const char* src = S + (role == 1 ? OG : OD) + pbase;
      f32x4 acj[2][NB32];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) acj[j][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NCH32; ++c) {
        Frag8 av[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          av[j].u = *(const uint4*)(src + j * T + (c / 3) * RS + (c % 3) * PB + 16 * g);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int nb = 0; nb < NB32; ++nb)
            acj[j][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[c][nb].v, av[j].v, acj[j][nb], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4* ac = acj[j];
        const int o = j * T + pin;
        const int64_t m = (int64_t)item * 32 + 16 * j + li;
#pragma unroll
        for (int nb = 0; nb < NB32; ++nb) {
          const int co0 = nb * 16 + 4 * g;
          if (role == 1) {  // du = conv1^T(g) * [u > 0]
            const uint2 mu = *(const uint2*)(S + OU + o + co0 * 2);
            const uint32_t mw[2] = {mu.x, mu.y};
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
              v[i] = (__uint_as_float(hb << 16) > 0.f) ? ac[nb][i] : 0.f;
            }
            *(uint2*)(S + OD + o + co0 * 2) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          } else {  // dx = conv0^T(du) * [x > 0] + g
            const uint2 mx = *(const uint2*)(S + OX + o + co0 * 2);
            const uint2 ad = *(const uint2*)(S + OG + o + co0 * 2);
            const uint32_t mw[2] = {mx.x, mx.y}, aw[2] = {ad.x, ad.y};
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint32_t hb = (mw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
              v[i] = (__uint_as_float(hb << 16) > 0.f) ? ac[nb][i] : 0.f;
              v[i] += __uint_as_float(((aw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) << 16);
            }
            if (m < npix)
              *(uint2*)(a.dx + m * C32 + co0) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          }
        }
      }
      wave_lds_order();
      set_flag(role == 1 ? f_du + b : f_d0 + b, it + 1, lane);
    }
    return;
  }

  // ---- W1 (stager) / W0: weight gradients over the item's 32 pixels (K index
  // k = 8g + 4hh + q: group g / 2, pixel 8 (g % 2) + 4 hh + q of it; q = li / 4)
  f32x4 acc[2][2][9], accb[2];  // [co block][ci block][tap]
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    accb[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[mb][nb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  int kp[2];  // this lane's K-row pixel (window top-left) for hh = 0, 1
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) kp[hh] = (g >> 1) * T + pix(8 * (g & 1) + 4 * hh + (li >> 2));
  const int c8 = 8 * (li & 3);
  const bool w1 = role == 0;
  // staging (W1): uint4 e = lane + 64 k of a tensor's item (group k, pixel lane / 4, chunk)
  const int sofs = pix(lane >> 2) + RS + PB + 16 * (lane & 3);
  uint4 px0, px1, pu0, pu1, pg0, pg1;  // (named registers: indexed arrays go to scratch)
  auto fetch = [&](int item) {
    // (branches, not selects: a select between a global element and a local zero became a
    // flat load through a scratch copy)
    const int64_t e = (int64_t)item * 128 + lane;
    const int64_t lim = npix * 4;
    px0 = pu0 = pg0 = px1 = pu1 = pg1 = make_uint4(0, 0, 0, 0);
    if (e < lim) {
      px0 = ((const uint4*)a.x)[e];
      pu0 = ((const uint4*)a.u)[e];
      pg0 = ((const uint4*)a.g)[e];
    }
    if (e + 64 < lim) {
      px1 = ((const uint4*)a.x)[e + 64];
      pu1 = ((const uint4*)a.u)[e + 64];
      pg1 = ((const uint4*)a.g)[e + 64];
    }
  };
  if (w1 && first < nitems) fetch(first);
  int it = 0;
  for (int item = first; item < nitems; item += step, ++it) {
    const int b = it % NSET;
    char* S = base + b * SETB<MW>();
    if (w1) {
      if (it >= NSET) {  // D0 and W0 are done with this set's last item
        wait_flag(f_d0 + b, it + 1 - NSET);
        wait_flag(f_w0 + b, it + 1 - NSET);
      }
      wave_lds_order();
      *(uint4*)(S + OX + sofs) = relu8(px0);
      *(uint4*)(S + OU + sofs) = relu8(pu0);
      *(uint4*)(S + OG + sofs) = pg0;
      *(uint4*)(S + OX + T + sofs) = relu8(px1);
      *(uint4*)(S + OU + T + sofs) = relu8(pu1);
      *(uint4*)(S + OG + T + sofs) = pg1;
      wave_lds_order();
      set_flag(f_staged + b, it + 1, lane);
      if (item + step < nitems) fetch(item + step);
    } else {
      wait_flag(f_du + b, it + 1);
      wave_lds_order();
    }
    // W1: dW1 += relu(u) (x) g (A = g, B = relu(u) taps); W0: dW0 += relu(x) (x) du
    const char* D = S + (w1 ? OG : OD) + RS + PB + c8;
    const char* X = S + (w1 ? OU : OX) + c8;
    Frag8 af[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) af[mb].h[hh] = tr_read(D + kp[hh] + mb * 32);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int off = (t / 3) * RS + (t % 3) * PB;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        Frag8 bf;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) bf.h[hh] = tr_read(X + kp[hh] + off + nb * 32);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          acc[mb][nb][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bf.v, acc[mb][nb][t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
      accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, ones.v, accb[mb], 0, 0, 0);
    wave_lds_order();
    if (!w1) set_flag(f_w0 + b, it + 1, lane);
  }
  // ---- this team's partial row of its layer (conv1 rows at partial, conv0 rows at + lstride)
  float* out = a.partial + (w1 ? 0 : a.lstride) + (size_t)(blockIdx.x * NT + team) * ROW32;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          out[(mb * 16 + 4 * g + i) * KTOT32 + t * C32 + nb * 16 + li] = acc[mb][nb][t][i];
    if (li == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i) out[C32 * KTOT32 + mb * 16 + 4 * g + i] = accb[mb][i];
  }
}

size_t res32b_smem(int imgs, int H, int W) {
  const size_t tb = ((size_t)imgs * geo32(H, W).is + 15) & ~(size_t)15;
  return std::max(4 * tb + 128, (size_t)kT32 * 16 * 4);
}

size_t resb32_smem(int imgs, int H, int W) {
  return 2 * (((size_t)imgs * geo32f(H, W).is + 15) & ~(size_t)15);
}

size_t resf_smem(int imgs, int H, int W) {
  return 2 * (((size_t)imgs * lay16(H, W).imgb + 15) & ~(size_t)15);
}

// the wave-owned 8x8 forward (res_fwd16_w88_kernel): three tiles per wave
constexpr size_t resf_w88_smem() { return (size_t)(kThreads / 64) * w88::REG; }

}  // namespace

static int res_fwd16_launch(ResFwdArgs a, hipStream_t stream);

// Forward of both residual blocks of a 16-channel stage (see res_fwd16_kernel).
extern "C" int mbk_res_fwd16(const void* p, void* u0, void* y0, void* u1, void* y1,
                             const void* const* w, const float* const* b, int N, int H, int W,
                             int imgs, hipStream_t stream) {
  ResFwdArgs a{(const bf16*)p, (bf16*)u0, (bf16*)y0, (bf16*)u1, (bf16*)y1,
               {(const bf16*)w[0], (const bf16*)w[1], (const bf16*)w[2], (const bf16*)w[3]},
               {b[0], b[1], b[2], b[3]}, N, H, W, imgs, nullptr, nullptr, nullptr, nullptr};
  return res_fwd16_launch(a, stream);
}

// mbk_res_fwd16 + the next stage's conv (16 -> 32, packed fwd weights ws, bias bs) and
// max_pool2d(3, 2, 1): ps [N][(H+1)/2][(W+1)/2][32] bf16, pidx the same shape of argmax
// bytes (null: not written); conv.hip's pooled conv_fwd results bit for bit.
extern "C" int mbk_res_fwd16_stage(const void* p, void* u0, void* y0, void* u1, void* y1,
                                   const void* const* w, const float* const* b, const void* ws,
                                   const float* bs, void* ps, void* pidx, int N, int H, int W,
                                   int imgs, hipStream_t stream) {
  if (!ws || !bs || !ps) return (int)hipErrorInvalidValue;
  ResFwdArgs a{(const bf16*)p, (bf16*)u0, (bf16*)y0, (bf16*)u1, (bf16*)y1,
               {(const bf16*)w[0], (const bf16*)w[1], (const bf16*)w[2], (const bf16*)w[3]},
               {b[0], b[1], b[2], b[3]}, N, H, W, imgs, (const bf16*)ws, bs, (bf16*)ps,
               (uint8_t*)pidx};
  return res_fwd16_launch(a, stream);
}

static int res_fwd16_launch(ResFwdArgs a, hipStream_t stream) {
  const int N = a.N, H = a.H, W = a.W, imgs = a.imgs;
  if (N <= 0) return 0;
  if (imgs < 1 || H * W > 1024 || (int64_t)imgs * H * W >= (int64_t(1) << 22))
    return (int)hipErrorInvalidValue;
  const size_t sm = resf_smem(imgs, H, W);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  const bool st = a.ws != nullptr;
  // the stage conv's pre-pool staging [imgs*H*W][36] bf16 lives in Tu
  if (st && (size_t)imgs * H * W * (W == 12 ? 2 * C : 2 * C + 4) * 2 > sm / 2)
    return (int)hipErrorInvalidValue;
  const bool fast = H == 8 && W == 8;  // (imgs: the generic kernel's round size only)
  const size_t smf = fast ? resf_w88_smem() : sm;
  if (fast) a.queue = mbk_work_queue(stream, kQueueResFwd16);
  auto kfn = fast ? (st ? res_fwd16_w88_kernel<true> : res_fwd16_w88_kernel<false>)
           : st ? (W == 8 ? res_fwd16_kernel<8, true> : W == 5 ? res_fwd16_kernel<5, true>
                   : W == 12 ? res_fwd16_kernel<12, true> : W == 4 ? res_fwd16_kernel<4, true>
                   : res_fwd16_kernel<0, true>)
                : (W == 8 ? res_fwd16_kernel<8, false> : W == 5 ? res_fwd16_kernel<5, false>
                   : W == 12 ? res_fwd16_kernel<12, false> : W == 4 ? res_fwd16_kernel<4, false>
                   : res_fwd16_kernel<0, false>);
  if (smf > 64 * 1024) (void)hipFuncSetAttribute((const void*)kfn,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smf);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ncu = cus;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kfn, kThreads, smf) !=
          hipSuccess || per < 1)
    per = 1;
  // work items: images per wave (wave-owned) or rounds of imgs images per workgroup
  const int nrounds = fast ? (N + kThreads / 64 - 1) / (kThreads / 64) : (N + imgs - 1) / imgs;
  hipLaunchKernelGGL(kfn, dim3(std::max(1L, std::min((long)nrounds, (long)ncu * mbk_occ_f(per)))),
                     dim3(kThreads), smf, stream, a);
  return (int)hipGetLastError();
}

// floats mbk_res_bwd16 needs in ``partial``: per layer, nparts rows + the two-level
// reduce's scratch rows (conv.hip wgrad_reduce stages its split sums after the rows)
extern "C" int64_t mbk_res_bwd16_partial_floats(int nparts) {
  return 2 * (int64_t)(nparts + (nparts + 31) / 32) * ROW;
}

// dx = conv0^T(conv1^T(g) * [u>0]) * [x>0] + g and both layers' weight / bias gradients.
// partial: mbk_res_bwd16_partial_floats(nparts) floats. dw1/db1/dw0/db0: fp32 parameter
// gradients [16][16][3][3] / [16] (overwritten); dw1 == nullptr: only the partial rows are
// written (layer 1's at partial, layer 0's at partial + partial_floats / 2) and the caller
// reduces them later.
extern "C" int mbk_res_bwd16(const void* x, const void* u, const void* g, void* dx,
                             const void* w1t, const void* w0t, float* partial, int nparts,
                             float* dw1, float* db1, float* dw0, float* db0, int N, int H, int W,
                             int imgs, int accumulate, hipStream_t stream) {
  if (N <= 0) return 0;
  if (nparts < 1 || nparts != mbk_res_bwd16_parts(N, H, W, imgs)) return (int)hipErrorInvalidValue;
  const bool fast = res_bwd_w88(H, W);
  const size_t sm = fast ? res_w88b_smem() : res_smem(imgs, H, W);
  const int64_t lstride = (int64_t)(nparts + (nparts + 31) / 32) * ROW;
  ResBwdArgs a{(const bf16*)x, (const bf16*)u, (const bf16*)g, (bf16*)dx,
               (const bf16*)w1t, (const bf16*)w0t, partial, lstride, N, H, W, imgs};
  auto kfn = fast ? res_bwd16_w88_kernel : W == 5 ? res_bwd16_kernel<5>
           : W == 12 ? res_bwd16_kernel<12> : W == 4 ? res_bwd16_kernel<4> : res_bwd16_kernel<0>;
  if (sm > 64 * 1024) (void)hipFuncSetAttribute((const void*)kfn,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  hipLaunchKernelGGL(kfn, dim3(nparts), dim3(fast ? w88b::kPT : kThreads), sm, stream, a);
  int rc = (int)hipGetLastError();
  if (rc || !dw1) return rc;  // dw1 == nullptr: the caller reduces (mbk_wgrad_reduce_batch)
  rc = mbk_wgrad_reduce(partial, nparts, C, C, C, dw1, db1, accumulate, stream);
  if (rc) return rc;
  return mbk_wgrad_reduce(partial + lstride, nparts, C, C, C, dw0, db0, accumulate, stream);
}

// Partial-row PAIRS mbk_res_bwd32 writes (= its grid: one 8-wave workgroup per CU);
// <= 0: unsupported shape.
extern "C" int mbk_res_bwd32_parts(int N, int H, int W, int imgs) {
  if (N <= 0 || imgs < 1 || H * W > 1024 || (int64_t)imgs * H * W >= (int64_t(1) << 22))
    return -1;
  if (res32b_smem(imgs, H, W) > 160 * 1024) return -1;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ncu = cus;
  const int nrounds = (N + imgs - 1) / imgs;
  return std::max(1, std::min(nrounds, ncu));
}

// Partial-row PAIRS mbk_res_bwd32_team writes (teams of its grid); <= 0: unsupported shape.
extern "C" int mbk_res_bwd32_team_parts(int N, int H, int W) {
  if (N <= 0 || H != W || (W != 4 && W != 2)) return -1;
  static int cus = 0, per4 = 0, per2 = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    (void)hipFuncSetAttribute((const void*)res_bwd32_team_kernel<4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, rbt::smem<4>());
    (void)hipFuncSetAttribute((const void*)res_bwd32_team_kernel<2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, rbt::smem<2>());
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per4, (const void*)res_bwd32_team_kernel<4>,
                                                     rbt::kPT, rbt::smem<4>()) != hipSuccess || per4 < 1)
      per4 = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, (const void*)res_bwd32_team_kernel<2>,
                                                     rbt::kPT, rbt::smem<2>()) != hipSuccess || per2 < 1)
      per2 = 1;
  }
  const int64_t nitems = ((int64_t)N * H * W + 31) / 32;
  const int64_t wgs = (nitems + rbt::NT - 1) / rbt::NT;
  return (int)(rbt::NT * std::max<int64_t>(1, std::min<int64_t>(wgs, (int64_t)cus * mbk_occ_b(W == 4 ? per4 : per2))));
}

// The 32-channel block backward on 4x4 / 2x2 maps by wave teams (res_bwd32_team_kernel):
// dx (bit-identical to mbk_res_bwd32) and the two layers' partial rows (conv1 at partial,
// conv0 at partial + partial_floats / 2); the caller reduces them (mbk_wgrad_reduce_batch).
extern "C" int mbk_res_bwd32_team(const void* x, const void* u, const void* g, void* dx,
                                  const void* w1t, const void* w0t, float* partial, int nparts,
                                  int N, int H, int W, hipStream_t stream) {
  if (N <= 0) return 0;
  if (nparts < 1 || nparts != mbk_res_bwd32_team_parts(N, H, W)) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)x | (uintptr_t)u | (uintptr_t)g | (uintptr_t)w1t | (uintptr_t)w0t) & 15) ||
      ((uintptr_t)dx & 7))
    return (int)hipErrorInvalidValue;
  const int64_t lstride = (int64_t)(nparts + (nparts + 31) / 32) * ROW32;
  ResBwd32Args a{(const bf16*)x, (const bf16*)u, (const bf16*)g, (bf16*)dx,
                 (const bf16*)w1t, (const bf16*)w0t, partial, lstride, N, H, W, 1};
  const void* kfn = W == 4 ? (const void*)res_bwd32_team_kernel<4> : (const void*)res_bwd32_team_kernel<2>;
  const int sm = W == 4 ? rbt::smem<4>() : rbt::smem<2>();
  void* args[] = {(void*)&a};
  (void)hipLaunchKernel(kfn, dim3(nparts / rbt::NT), dim3(rbt::kPT), args, sm, stream);
  return (int)hipGetLastError();
}

extern "C" int64_t mbk_res_bwd32_partial_floats(int nparts) {
  return 2 * (int64_t)(nparts + (nparts + 31) / 32) * ROW32;
}

// 32-channel block backward (see res_bwd32_kernel): dx and both layers' weight / bias
// gradients dw1/db1/dw0/db0 (fp32 [32][32][3][3] / [32], overwritten; dw1 == nullptr: partial
// rows only, as mbk_res_bwd16).
extern "C" int mbk_res_bwd32(const void* x, const void* u, const void* g, void* dx,
                             const void* w1t, const void* w0t, float* partial, int nparts,
                             float* dw1, float* db1, float* dw0, float* db0, int N, int H, int W,
                             int imgs, int accumulate, hipStream_t stream) {
  if (N <= 0) return 0;
  if (nparts < 1 || nparts != mbk_res_bwd32_parts(N, H, W, imgs)) return (int)hipErrorInvalidValue;
  const size_t sm = res32b_smem(imgs, H, W);
  const int64_t lstride = (int64_t)(nparts + (nparts + 31) / 32) * ROW32;
  ResBwd32Args a{(const bf16*)x, (const bf16*)u, (const bf16*)g, (bf16*)dx,
                 (const bf16*)w1t, (const bf16*)w0t, partial, lstride, N, H, W, imgs};
  auto kfn = W == 4 ? res_bwd32_kernel<4> : W == 2 ? res_bwd32_kernel<2>
           : W == 8 ? res_bwd32_kernel<8> : W == 3 ? res_bwd32_kernel<3>
           : W == 6 ? res_bwd32_kernel<6> : res_bwd32_kernel<0>;
  if (sm > 64 * 1024) (void)hipFuncSetAttribute((const void*)kfn,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  hipLaunchKernelGGL(kfn, dim3(nparts), dim3(kT32), sm, stream, a);
  int rc = (int)hipGetLastError();
  if (rc || !dw1) return rc;  // dw1 == nullptr: the caller reduces (mbk_wgrad_reduce_batch)
  rc = mbk_wgrad_reduce(partial, nparts, C32, C32, C32, dw1, db1, accumulate, stream);
  if (rc) return rc;
  return mbk_wgrad_reduce(partial + lstride, nparts, C32, C32, C32, dw0, db0, accumulate, stream);
}

// One 32-channel residual block's forward (see res_blk32_kernel): u = conv0(relu x),
// y = x + conv1(relu u), bit-identical to two conv_fwd<32, 32> launches.
// One 32-channel residual block on 4x4 or 2x2 maps with wave-owned 16-pixel blocks
// (res_blk32_wave_kernel): bit-identical to mbk_res_blk32_fwd.
extern "C" int mbk_res_blk32_fwd_wave(const void* x, void* u, void* y, const void* const* w,
                                      const float* const* b, int N, int H, int W,
                                      hipStream_t stream) {
  if (N <= 0) return 0;
  if (H != W || (W != 4 && W != 2)) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)x | (uintptr_t)w[0] | (uintptr_t)w[1]) & 15) || (((uintptr_t)u | (uintptr_t)y) & 7))
    return (int)hipErrorInvalidValue;
  const void* kfn = W == 4 ? (const void*)res_blk32_wave_kernel<4> : (const void*)res_blk32_wave_kernel<2>;
  const int sm = W == 4 ? rbw::smem<4>() : rbw::smem<2>();
  static int cus = 0, per4 = 0, per2 = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per4, (const void*)res_blk32_wave_kernel<4>,
                                                     rbw::kPT, rbw::smem<4>()) != hipSuccess || per4 < 1)
      per4 = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, (const void*)res_blk32_wave_kernel<2>,
                                                     rbw::kPT, rbw::smem<2>()) != hipSuccess || per2 < 1)
      per2 = 1;
  }
  ResBlk32Args a{(const bf16*)x, (bf16*)u, (bf16*)y, {(const bf16*)w[0], (const bf16*)w[1]},
                 {b[0], b[1]}, N, H, W, 1};
  a.queue = mbk_work_queue(stream, kQueueBlk32);
  const int64_t nq = ((int64_t)N * H * W + 15) / 16;
  const int64_t groups = (nq + rbw::NW - 1) / rbw::NW;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(groups, (int64_t)cus * mbk_occ_f(W == 4 ? per4 : per2)));
  void* args[] = {(void*)&a};
  (void)hipLaunchKernel(kfn, dim3(grid), dim3(rbw::kPT), args, sm, stream);
  return (int)hipGetLastError();
}

extern "C" int mbk_res_blk32_fwd(const void* x, void* u, void* y, const void* const* w,
                                 const float* const* b, int N, int H, int W, int imgs,
                                 hipStream_t stream) {
  if (N <= 0) return 0;
  if (imgs < 1 || H * W > 1024 || (int64_t)imgs * H * W >= (int64_t(1) << 22))
    return (int)hipErrorInvalidValue;
  const size_t sm = resb32_smem(imgs, H, W);
  if (sm > 160 * 1024) return (int)hipErrorInvalidValue;
  ResBlk32Args a{(const bf16*)x, (bf16*)u, (bf16*)y, {(const bf16*)w[0], (const bf16*)w[1]},
                 {b[0], b[1]}, N, H, W, imgs};
  auto kfn = W == 4 ? res_blk32_kernel<4> : W == 2 ? res_blk32_kernel<2>
           : W == 8 ? res_blk32_kernel<8> : W == 3 ? res_blk32_kernel<3>
           : W == 6 ? res_blk32_kernel<6> : res_blk32_kernel<0>;
  if (sm > 64 * 1024) (void)hipFuncSetAttribute((const void*)kfn,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ncu = cus;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kfn, kThreads, sm) !=
          hipSuccess || per < 1)
    per = 1;
  const int nrounds = (N + imgs - 1) / imgs;
  hipLaunchKernelGGL(kfn, dim3(std::max(1, std::min(nrounds, ncu * mbk_occ_f(per)))), dim3(kThreads), sm,
                     stream, a);
  return (int)hipGetLastError();
}
