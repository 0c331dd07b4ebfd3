// Forward of a pooled stage conv on 4x4 maps (IMPALA stage 2 at 16x16: conv 32 -> 32, then
// max_pool2d(3, 2, 1) to 2x2) with wave-owned images.
//
// Reference: model.py:76-92 (a stage is conv -> max-pool -> 2 residual blocks). The generic
// conv_fwd<32, 32> (conv.hip) ran this shape in workgroup rounds of 8 images: stage, MFMA,
// barrier, pool_tile on half the threads, barrier -- 0.49-0.52 ms per 524K-frame update
// against 0.27 ms for the same conv without the pool (profile 42). Here every wave owns image
// pairs from its global load to its pooled store, with no workgroup barrier:
//   * x (1 KB per image: one uint4 per lane) is prefetched a pair ahead into registers and
//     staged into the wave's halo'd tiles (64-byte pixels in 416-byte rows: the 4-wide map
//     geometry of res_blk32, conflict-free tap reads);
//   * 9 tap chunks x 2 output blocks of MFMAs per image, with the weights in VGPRs for the
//     whole launch: conv_fwd's chain and epilogue (acc + bias, one RNE rounding), so the
//     pre-pool values are bit-identical to it;
//   * the pool: lane = (image, pooled pixel, 4 channels), the 3x3 window scanned in order with
//     strict > (the first maximising tap: mbk::pool_tile's values and argmax bytes).
#include "../include/mbk_api.h"
#include "common.h"

#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

union Frag8 {
  bf16x8 v;
  uint4 u;
};

__device__ __forceinline__ uint32_t cvt_pk2(float a, float b) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, b16x2));
}
__device__ __forceinline__ void wave_lds_order() { asm volatile("" ::: "memory"); }

namespace s2 {
constexpr int H = 4, W = 4, HW = 16, C = 32, HO = 2, WO = 2;
constexpr int NW = 4, kPT = 64 * NW;  // waves per workgroup
constexpr int NI = 2;                 // images per wave iteration (the pool's 64 lanes)
constexpr int PB = 64, RS = 416;      // halo'd x tile: pixel / row strides (bytes)
constexpr int XB = ((H + 1) * RS + (W + 2) * PB + 15) & ~15;
constexpr int OSTR = C + 4;           // pre-pool row (bf16), conv_fwd's OSTR
constexpr int OB = HW * OSTR * 2;
constexpr int SLICE = NI * (XB + OB);
constexpr int SMEM = NW * SLICE;
static_assert(XB % 16 == 0 && OB % 16 == 0, "alignment");
}  // namespace s2

struct PoolConvFwd4Args {
  const bf16* x;      // [N][4][4][32]
  const bf16* w;      // packed fwd weights [32][9][32] (conv.hip layout)
  const float* bias;  // [32]
  bf16* y;            // [N][2][2][32] pooled
  uint8_t* pidx;      // [N][2][2][32] argmax taps (nullable)
  int N;
  int* queue = nullptr;  // per-wave queue of image pairs (common.h), null: static stride
};

__global__ __launch_bounds__(s2::kPT) void pool_conv_fwd4_kernel(PoolConvFwd4Args a) {
  using namespace s2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  char* R = smem + wave * SLICE;
  // halos zero once: interiors are rewritten per image
  for (int e = lane; e < SLICE / 16; e += 64) ((uint4*)R)[e] = make_uint4(0, 0, 0, 0);
  Frag8 wv[9][2];  // A: w[co = 16 nb + li][tap c][ci 8g .. 8g+7]
  float bv[2][4];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const uint4* wp = (const uint4*)(a.w + (size_t)(nb * 16 + li) * 9 * C + g * 8);
#pragma unroll
    for (int c = 0; c < 9; ++c) wv[c][nb].u = wp[c * 4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nb][i] = a.bias[nb * 16 + 4 * g + i];
  }
  // B reads: pixel li (row li / 4, column li % 4), tap c, channels 8g .. 8g+7
  const int bofs = (li >> 2) * RS + (li & 3) * PB + 16 * g;
  // staging: lane = uint4 #lane of an image (pixel lane / 4, channel chunk lane % 4)
  const int sofs = ((lane >> 4) + 1) * RS + (((lane >> 2) & 3) + 1) * PB + 16 * (lane & 3);
  // pool lanes: image pj, pooled pixel (oy, ox), channels 4 c4 .. 4 c4 + 3
  const int pj = lane >> 5, opx = (lane >> 3) & 3, c4 = lane & 7;
  const int oy = opx >> 1, ox = opx & 1;
  const int npairs = (a.N + NI - 1) / NI;
  const int step = gridDim.x * NW;
  int* const wq = a.queue;
  int cend = 0;
  const int first = wq ? mbk::wave_next_item(wq, -1, cend, npairs) : (int)blockIdx.x * NW + wave;
  int nxt = wq ? (first < npairs ? mbk::wave_next_item(wq, first, cend, npairs) : npairs)
               : first + step;
  int nn = npairs;
  static_assert(NI == 2, "named prefetch registers");
  uint4 pf0, pf1;  // (named: an indexed register array went to scratch)
  auto fetch = [&](int pr) {
    const int i0 = NI * pr, i1 = min(i0 + 1, a.N - 1);  // a lone last image: repeated
    pf0 = ((const uint4*)(a.x + (size_t)i0 * HW * C))[lane];
    pf1 = ((const uint4*)(a.x + (size_t)i1 * HW * C))[lane];
  };
  wave_lds_order();
  if (first < npairs) fetch(first);
  for (int pr = first; pr < npairs; pr = nxt, nxt = nn) {
    *(uint4*)(R + sofs) = pf0;
    *(uint4*)(R + XB + sofs) = pf1;
    if (nxt < npairs) fetch(nxt);
    nn = wq ? (nxt < npairs ? mbk::wave_next_item(wq, nxt, cend, npairs) : npairs) : nxt + step;
    wave_lds_order();
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const char* xt = R + j * XB + bofs;
      Frag8 fr[9];
#pragma unroll
      for (int c = 0; c < 9; ++c) fr[c].u = *(const uint4*)(xt + (c / 3) * RS + (c % 3) * PB);
      f32x4 acc[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 9; ++c)
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[c][nb].v, fr[c].v, acc[nb], 0, 0, 0);
      }
      bf16* ot = (bf16*)(R + NI * XB + j * OB);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[nb][i] * 1.f + bv[nb][i];
        *(uint2*)(ot + li * OSTR + nb * 16 + 4 * g) =
            make_uint2(cvt_pk2(v[0], v[1]), cvt_pk2(v[2], v[3]));
      }
    }
    wave_lds_order();
    // ---- max_pool2d(3, 2, 1): the window's taps in scan order, first maximum kept
    {
      const int img = NI * pr + pj;
      const bf16* ot = (const bf16*)(R + NI * XB + pj * OB) + 4 * c4;
      float m[4];
      int ix[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) { m[j] = -INFINITY; ix[j] = 0; }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int py = 2 * oy - 1 + ky;
        if (py < 0 || py >= H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int px = 2 * ox - 1 + kx;
          if (px < 0 || px >= W) continue;
          const uint2 u = *(const uint2*)(ot + (py * W + px) * OSTR);
          float v[4];
          v[0] = __uint_as_float(u.x << 16);
          v[1] = __uint_as_float(u.x & 0xFFFF0000u);
          v[2] = __uint_as_float(u.y << 16);
          v[3] = __uint_as_float(u.y & 0xFFFF0000u);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (v[j] > m[j]) { m[j] = v[j]; ix[j] = 3 * ky + kx; }
        }
      }
      if (img < a.N) {
        const size_t oi = ((size_t)img * HO * WO + opx) * C + 4 * c4;
        *(uint2*)(a.y + oi) =
            make_uint2((__float_as_uint(m[0]) >> 16) | (__float_as_uint(m[1]) & 0xFFFF0000u),
                       (__float_as_uint(m[2]) >> 16) | (__float_as_uint(m[3]) & 0xFFFF0000u));
        if (a.pidx)
          *(uint32_t*)(a.pidx + oi) = (uint32_t)ix[0] | ((uint32_t)ix[1] << 8) |
                                      ((uint32_t)ix[2] << 16) | ((uint32_t)ix[3] << 24);
      }
    }
    wave_lds_order();  // the next pair's staging overwrites the tiles
  }
  if (wq) mbk::wave_queue_done(wq, step);
}

}  // namespace

// y = max_pool2d(conv(x) + bias, 3, 2, 1) with argmax bytes (pidx nullable) for 4x4x32 ->
// 2x2x32 maps; bit-identical to conv_fwd<32, 32> with pool. w: packed fwd weights [32][9][32].
extern "C" int mbk_pool_conv_fwd4(const void* x, const void* w, const float* bias, void* y,
                                  void* pidx, int N, hipStream_t stream) {
  if (N <= 0) return 0;
  if (!x || !w || !bias || !y || (((uintptr_t)x | (uintptr_t)w) & 15) || ((uintptr_t)y & 7) ||
      ((uintptr_t)pidx & 3))
    return (int)hipErrorInvalidValue;
  static int cus = 0, per = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)pool_conv_fwd4_kernel,
                                                     s2::kPT, s2::SMEM) != hipSuccess || per < 1)
      per = 1;
  }
  const int npairs = (N + s2::NI - 1) / s2::NI;
  const int groups = (npairs + s2::NW - 1) / s2::NW;
  PoolConvFwd4Args a{(const bf16*)x, (const bf16*)w, bias, (bf16*)y, (uint8_t*)pidx, N};
  a.queue = mbk_work_queue(stream, kQueuePoolConv4);
  hipLaunchKernelGGL(pool_conv_fwd4_kernel, dim3(std::max(1, std::min(groups, cus * mbk_occ_f(per)))),
                     dim3(s2::kPT), s2::SMEM, stream, a);
  return (int)hipGetLastError();
}
