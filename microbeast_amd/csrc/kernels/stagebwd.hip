// Backward of a pooled stage conv in one launch (IMPALA stage 1 at 16x16: conv 16 -> 32 on
// 8x8 maps, then max_pool2d(3, 2, 1) to 4x4).
//
// Reference: model.py:76-92, a stage is conv -> max-pool -> 2 residual blocks. Given dp =
// dL/d(pooled output) and the stored argmax bytes, the per-layer path (ops/encoder.py) ran
//   pool_bwd_idx (dc = pool backward of dp, 8x8x32, written to HBM)
//   | conv_wgrad (dW += x (x) dc, reads dc and x) | conv_fwd on dc (dx = conv^T(dc))
// = 0.66 + 0.57 + 0.82 ms per 524K-frame update (profile r5n), ~17.5 KB of HBM per image. Here
// each wave owns whole images, with no workgroup barrier until the final reduction:
//   * the pooled gradient and argmax bytes (1.5 KB) are scattered into an fp32 image of dc in
//     the wave's LDS (4 window-parity phases: windows of one parity never overlap, so no two
//     lanes of a phase add into the same element), then rounded once into a halo'd bf16 tile;
//   * dgrad (dx = conv^T(dc), the packed transposed weights in VGPRs, 4 row-pair blocks x 9 K
//     chunks: conv_fwd's MFMA chain, so dx is bit-identical whenever dc is) -> HBM;
//   * wgrad (dW += x (x) dc: A = dc^T and B = x taps through ds_read_b64_tr_b16, bias = dc^T
//     times an all-ones fragment), accumulated in VGPRs over the wave's images.
// ~5.5 KB of HBM per image (read dp, argmax, x; write dx). The fp32 sums of the <= 4 windows
// that share a pixel are exact whenever the pooled gradients' exponents are within 16 bits of
// each other (bf16 operands), i.e. the same values as pool_bwd_idx's raster-order sum.
#include "../include/mbk_api.h"
#include "common.h"

#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

extern "C" int mbk_wgrad_reduce(const float* partial, int nparts, int cin, int cin_real,
                                int cout, float* dw, float* db, int accumulate,
                                hipStream_t stream);

namespace {

union Frag8 {
  bf16x8 v;
  uint4 u;
  s16x4 h[2];
};

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}
__device__ __forceinline__ uint32_t cvt_pk2(float a, float b) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, b16x2));
}
__device__ __forceinline__ void wave_lds_order() { asm volatile("" ::: "memory"); }

// ---- geometry (stage 1 at 16x16): x 8x8x16, dc 8x8x32, pooled 4x4x32
namespace s1 {
constexpr int H = 8, W = 8, HW = 64, CI = 16, CO = 32, HO = 4, WO = 4;
constexpr int NW = 4, kPT = 64 * NW;  // waves per workgroup (2 workgroups per CU)
// halo'd x tile: 32-byte pixels, rows 384 B apart (= 128 mod 256: the two map rows of a
// transposed read's half-wave land on opposite bank halves)
constexpr int PBX = 32, RBX = 384, XB = (H + 1) * RBX + (W + 2) * PBX;
// halo'd dc tile: 64-byte pixels, rows 672 B apart (= 160 mod 256: a half-wave's 2 x 4 pixel
// chunks of 32 B fall in 8 distinct bank slots)
constexpr int PBD = 64, RBD = 672, DB = (H + 1) * RBD + (W + 2) * PBD;
// fp32 scatter image of dc: 33-dword pixel rows (lanes adding to different pixels spread banks)
constexpr int FST = 33 * 4, FB = HW * FST;
constexpr int PB_P = HO * WO * CO * 2, PB_I = HO * WO * CO;  // staged dp / argmax bytes
constexpr int OX = 0, OD = OX + XB, OF = OD + DB, OP = OF + FB, OI = OP + PB_P;
constexpr int SLICE = (OI + PB_I + 15) & ~15;
constexpr int KTOT = 9 * CI, ROWF = CO * KTOT + CO;  // one partial row (weights + bias)
constexpr int SMEM = NW * SLICE;
static_assert(XB % 16 == 0 && DB % 16 == 0 && OF % 16 == 0 && OP % 16 == 0, "alignment");
static_assert(2 * SMEM <= 160 * 1024, "two workgroups per CU");
static_assert(NW * ROWF * 4 <= SMEM, "reduction slots must fit the tiles");
}  // namespace s1

struct PoolConvBwdArgs {
  const bf16* dp;       // [N][4][4][32] pooled gradient
  const uint8_t* pidx;  // [N][4][4][32] argmax tap in the 3x3 window
  const bf16* x;        // [N][8][8][16] the conv's input
  const bf16* wt;       // packed transposed weights [16][9][32] (conv.hip dgrad layout)
  bf16* dx;             // [N][8][8][16]
  float* partial;       // [gridDim.x][ROWF]
  int N;
};

__global__ __launch_bounds__(s1::kPT) void pool_conv_bwd_s1_kernel(PoolConvBwdArgs a) {
  using namespace s1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  char* R = smem + wave * SLICE;
  char* X = R + OX;
  char* D = R + OD;
  float* F = (float*)(R + OF);
  char* P = R + OP;
  char* I = R + OI;
  // halos (and everything else) zero once: interiors are rewritten per image
  for (int e = lane; e < SLICE / 16; e += 64) ((uint4*)R)[e] = make_uint4(0, 0, 0, 0);
  // dgrad weights (A fragments): lane holds w[ci = li][chunk c = tap][co 8g..8g+7]
  Frag8 wd[9];
  {
    const uint4* wp = (const uint4*)(a.wt + (size_t)li * 9 * 32 + g * 8);
#pragma unroll
    for (int c = 0; c < 9; ++c) wd[c].u = wp[c * 4];
  }
  // dgrad B reads: pixel li of row-pair block j, tap c: row 2j + li/8 + c/3, col li%8 + c%3
  const int db0 = (li >> 3) * RBD + (li & 7) * PBD + 16 * g;
  // wgrad K order: half h of lane group g = map row 4 kb + 2 (g / 2) + g % 2, column 4 h + q
  // (q = li / 4 selects the row the lane's address supplies); channel block 4 (li % 4)
  int tro[2];  // the lane's map column in half h
#pragma unroll
  for (int h = 0; h < 2; ++h) tro[h] = 4 * h + (li >> 2);
  const int trow = 2 * (g >> 1) + (g & 1);  // ... and its row within the K block
  f32x4 acc[2][9], accb[2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    accb[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[mb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  // scatter lanes: phase ph's 4 windows (oy % 2, ox % 2) = (ph / 2, ph % 2); lane = (window k
  // of the phase, channel pair cp)
  const int sk = lane >> 4, cp = lane & 15;
  const int step = gridDim.x * NW;
  const int first = blockIdx.x * NW + wave;
  uint4 pxv[2], pdv;
  uint2 piv;
  auto fetch = [&](int im) {
    const uint4* xs = (const uint4*)(a.x + (size_t)im * HW * CI);
    pxv[0] = xs[2 * lane];
    pxv[1] = xs[2 * lane + 1];
    pdv = ((const uint4*)(a.dp + (size_t)im * HO * WO * CO))[lane];
    piv = ((const uint2*)(a.pidx + (size_t)im * HO * WO * CO))[lane];
  };
  wave_lds_order();
  if (first < a.N) fetch(first);
  for (int img = first; img < a.N; img += step) {
    // ---- stage: x interior (lane = pixel), pooled chunks (lane = 8 channels of a window)
    {
      char* xp = X + ((lane >> 3) + 1) * RBX + ((lane & 7) + 1) * PBX;
      *(uint4*)xp = pxv[0];
      *(uint4*)(xp + 16) = pxv[1];
      *(uint4*)(P + lane * 16) = pdv;
      *(uint2*)(I + lane * 8) = piv;
      float* fr = F + lane * 33;
#pragma unroll
      for (int c = 0; c < 32; ++c) fr[c] = 0.f;
    }
    if (img + step < a.N) fetch(img + step);
    wave_lds_order();
    // ---- scatter the pooled gradient into the fp32 image of dc
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int oy = 2 * (sk >> 1) + (ph >> 1), ox = 2 * (sk & 1) + (ph & 1);
      const int w = oy * WO + ox;
      const uint32_t d2 = *(const uint32_t*)(P + (w * CO + 2 * cp) * 2);
      const uint32_t i2 = *(const uint16_t*)(I + w * CO + 2 * cp);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int t = (int)((i2 >> (8 * k)) & 0xFFu);
        const int ky = t / 3, kx = t - 3 * ky;
        const int py = 2 * oy - 1 + ky, px = 2 * ox - 1 + kx;
        float* f = F + (py * W + px) * 33 + 2 * cp + k;
        *f = *f + __uint_as_float(k ? (d2 & 0xFFFF0000u) : (d2 << 16));
      }
      wave_lds_order();
    }
    // ---- round into the halo'd bf16 dc tile (lane = pixel)
    {
      const float* fr = F + lane * 33;
      uint32_t o[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) o[c] = cvt_pk2(fr[2 * c], fr[2 * c + 1]);
      char* dq = D + ((lane >> 3) + 1) * RBD + ((lane & 7) + 1) * PBD;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        *(uint4*)(dq + 16 * k) = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
    }
    wave_lds_order();
    // ---- dx = conv^T(dc): 4 row-pair blocks x 9 K chunks (tap c, 32 channels)
    {
      bf16* gdx = a.dx + (size_t)img * HW * CI;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Frag8 fr[9];
#pragma unroll
        for (int c = 0; c < 9; ++c)
          fr[c].u = *(const uint4*)(D + db0 + (2 * j + c / 3) * RBD + (c % 3) * PBD);
        f32x4 acc_d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 9; ++c)
          acc_d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wd[c].v, fr[c].v, acc_d, 0, 0, 0);
        // lane: pixel li of the block (row 2j + li / 8, column li % 8), channels 4g .. 4g+3
        const int pix = (2 * j + (li >> 3)) * W + (li & 7);
        *(uint2*)(gdx + pix * CI + 4 * g) =
            make_uint2(cvt_pk2(acc_d[0], acc_d[1]), cvt_pk2(acc_d[2], acc_d[3]));
      }
    }
    // ---- dW += x (x) dc over the image's 2 K blocks (rows 4 kb .. 4 kb + 3)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int row = 4 * kb + trow;
      Frag8 af[2];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          af[mb].h[h] = tr_read(D + (row + 1) * RBD + (tro[h] + 1) * PBD + mb * 32 + 8 * (li & 3));
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        Frag8 bf;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          bf.h[h] = tr_read(X + (row + t / 3) * RBX + (tro[h] + t % 3) * PBX + 8 * (li & 3));
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          acc[mb][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bf.v, acc[mb][t], 0, 0, 0);
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
        accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, ones.v, accb[mb], 0, 0, 0);
    }
    wave_lds_order();  // the next image's staging overwrites the tiles
  }
  __syncthreads();
  // ---- per-workgroup partial row: the waves' accumulators summed in a fixed order
  float* red = (float*)smem;
  {
    float* sl = red + wave * ROWF;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sl[(mb * 16 + 4 * g + i) * KTOT + t * CI + li] = acc[mb][t][i];
      if (li == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) sl[CO * KTOT + mb * 16 + 4 * g + i] = accb[mb][i];
    }
  }
  __syncthreads();
  float* out = a.partial + (size_t)blockIdx.x * ROWF;
  for (int e = tid; e < ROWF; e += kPT) {
    float s = red[e];
#pragma unroll
    for (int w = 1; w < NW; ++w) s += red[w * ROWF + e];
    out[e] = s;
  }
}

}  // namespace

// Partial rows mbk_pool_conv_bwd writes (= its grid) for N images of the supported shape
// (16 -> 32 channels on 8x8 maps, pooled 4x4); <= 0: unsupported.
extern "C" int mbk_pool_conv_bwd_parts(int N, int cin, int cout, int H, int W) {
  if (N <= 0 || cin != s1::CI || cout != s1::CO || H != s1::H || W != s1::W) return -1;
  static int cus = 0, per = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    (void)hipFuncSetAttribute((const void*)pool_conv_bwd_s1_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, s1::SMEM);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)pool_conv_bwd_s1_kernel,
                                                     s1::kPT, s1::SMEM) != hipSuccess || per < 1)
      per = 1;
  }
  const int rounds = (N + s1::NW - 1) / s1::NW;
  return std::max(1, std::min(rounds, cus * per));
}

// dx = conv^T(pool_bwd(dp, pidx)) and the conv's weight / bias gradients (dw [32][16][3][3],
// db [32], fp32; accumulate: add instead of overwrite). partial: nparts x (32*144 + 32) floats
// plus the reduce's scratch rows (conv.hip mbk_wgrad_reduce).
extern "C" int mbk_pool_conv_bwd(const void* dp, const void* pidx, const void* x, const void* wt,
                                 void* dx, float* partial, int nparts, float* dw, float* db,
                                 int N, int cin, int cout, int H, int W, int accumulate,
                                 hipStream_t stream) {
  if (N <= 0) return 0;
  if (nparts < 1 || nparts != mbk_pool_conv_bwd_parts(N, cin, cout, H, W))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)dp | (uintptr_t)x | (uintptr_t)wt) & 15 || ((uintptr_t)pidx & 7) ||
      ((uintptr_t)dx & 7))
    return (int)hipErrorInvalidValue;
  PoolConvBwdArgs a{(const bf16*)dp, (const uint8_t*)pidx, (const bf16*)x, (const bf16*)wt,
                    (bf16*)dx, partial, N};
  hipLaunchKernelGGL(pool_conv_bwd_s1_kernel, dim3(nparts), dim3(s1::kPT), s1::SMEM, stream, a);
  const int rc = (int)hipGetLastError();
  if (rc || !dw) return rc;  // dw == nullptr: the caller reduces (mbk_wgrad_reduce_batch)
  return mbk_wgrad_reduce(partial, nparts, cin, cin, cout, dw, db, accumulate, stream);
}

extern "C" int64_t mbk_pool_conv_bwd_partial_floats(int nparts) {
  return (int64_t)(nparts + (nparts + 31) / 32) * s1::ROWF;
}
