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
//
// Stage 2 (conv 32 -> 32 on 4x4 maps, pooled 2x2; pool_conv_bwd_s2_kernel): the per-layer
// path ran pool_bwd_idx 0.14 + conv_wgrad 0.26 + dgrad conv_fwd 0.27 ms per update (profile 42).
// The same dataflow with 32 input channels would need 36 weight-gradient tiles and 18 dgrad
// weight fragments per wave; instead the two waves of a pair take the SAME image pairs and
// split the input channels: wave h stages its 16-channel half of x, rebuilds the whole dc
// tile itself (the scatter is cheap, no cross-wave flags), and computes dx and dW for input
// channels 16h .. 16h + 15 only (9 dgrad fragments, 18 weight-gradient tiles). Two images form
// one 32-pixel K block of the weight gradient.
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

// ---- geometry (stage 2 at 16x16): x 4x4x32, dc 4x4x32, pooled 2x2x32
namespace s2 {
constexpr int H = 4, W = 4, HW = 16, CI = 32, CO = 32, HO = 2, WO = 2, CH = 16;
constexpr int NW = 4, kPT = 64 * NW;  // two wave pairs per workgroup
constexpr int NI = 2;                 // images per iteration: one 32-pixel wgrad K block
// halo'd x half tile: 32-byte pixels (16 channels), 192-byte rows (two map rows = 128 mod
// 256: the two K-row groups of a half-wave's transposed read fill opposite bank halves)
constexpr int PBX = 32, RBX = 192, XB = 6 * RBX;
// halo'd dc tile: 64-byte pixels, 400-byte rows (res_bwd32's 4-wide geometry)
constexpr int PBD = 64, RBD = 400, DB = ((H + 1) * RBD + (W + 2) * PBD + 15) & ~15;
constexpr int FST = 33, FB = HW * FST * 4;  // fp32 scatter image, 33-float pixel rows
constexpr int PB_P = HO * WO * CO * 2, PB_I = HO * WO * CO;
constexpr int OX = 0, OD = OX + NI * XB, OF = OD + NI * DB, OP = OF + NI * FB,
              OI = OP + NI * PB_P;
constexpr int SLICE = (OI + NI * PB_I + 15) & ~15;
constexpr int KTOT = 9 * CI, ROWF = CO * KTOT + CO;
constexpr int SMEM = NW * SLICE > ROWF * 4 ? NW * SLICE : ROWF * 4;
static_assert(XB % 16 == 0 && DB % 16 == 0 && FB % 16 == 0 && OF % 16 == 0 && OP % 16 == 0,
              "alignment");
static_assert(SMEM <= 64 * 1024, "no dynamic-LDS attribute needed");
}  // namespace s2

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
  uint4 pxv0, pxv1, pdv;  // (named: an indexed register array went to scratch)
  uint2 piv;
  auto fetch = [&](int im) {
    const uint4* xs = (const uint4*)(a.x + (size_t)im * HW * CI);
    pxv0 = xs[2 * lane];
    pxv1 = xs[2 * lane + 1];
    pdv = ((const uint4*)(a.dp + (size_t)im * HO * WO * CO))[lane];
    piv = ((const uint2*)(a.pidx + (size_t)im * HO * WO * CO))[lane];
  };
  wave_lds_order();
  if (first < a.N) fetch(first);
  for (int img = first; img < a.N; img += step) {
    // ---- stage: x interior (lane = pixel), pooled chunks (lane = 8 channels of a window)
    {
      char* xp = X + ((lane >> 3) + 1) * RBX + ((lane & 7) + 1) * PBX;
      *(uint4*)xp = pxv0;
      *(uint4*)(xp + 16) = pxv1;
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

__global__ __launch_bounds__(s2::kPT) void pool_conv_bwd_s2_kernel(PoolConvBwdArgs a) {
  using namespace s2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int h = wave & 1;  // this wave's input-channel half
  char* R = smem + wave * SLICE;
  char* X = R + OX;
  char* D = R + OD;
  float* F = (float*)(R + OF);
  char* P = R + OP;
  char* I = R + OI;
  for (int e = lane; e < SLICE / 16; e += 64) ((uint4*)R)[e] = make_uint4(0, 0, 0, 0);
  // dgrad weights (A fragments): lane holds w[ci = 16h + li][tap c][co 8g .. 8g+7]
  Frag8 wd[9];
  {
    const uint4* wp = (const uint4*)(a.wt + (size_t)(CH * h + li) * 9 * CO + g * 8);
#pragma unroll
    for (int c = 0; c < 9; ++c) wd[c].u = wp[c * 4];
  }
  // wgrad K index 8g + 4hh + q (q = li / 4): image g / 2, map row 2 (g % 2) + hh, column q;
  // channel block 4 (li % 4) of the transposed reads
  const int wj = g >> 1, wrow = 2 * (g & 1), q = li >> 2, p4 = li & 3;
  f32x4 acc[2][9], accb[2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    accb[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[mb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  // staging lanes: image sj; x: pixel sp, 16-byte chunk sc of the half; dp / pidx: word sw
  const int sj = lane >> 5, sp = (lane >> 1) & 15, sc = lane & 1, sw = lane & 31;
  const int npairs = (a.N + NI - 1) / NI;
  const int step = gridDim.x * (NW / 2);
  const int first = blockIdx.x * (NW / 2) + (wave >> 1);
  uint4 pxv;
  uint2 pdv;
  uint32_t piv;
  auto fetch = [&](int pr) {
    const int im = NI * pr + sj;
    if (im < a.N) {
      pxv = *(const uint4*)(a.x + ((size_t)im * HW + sp) * CI + CH * h + 8 * sc);
      pdv = ((const uint2*)(a.dp + (size_t)im * HO * WO * CO))[sw];
      piv = ((const uint32_t*)(a.pidx + (size_t)im * HO * WO * CO))[sw];
    } else {  // a pair's missing last image: zero gradient, centre taps (in the map)
      pxv = make_uint4(0, 0, 0, 0);
      pdv = make_uint2(0, 0);
      piv = 0x04040404u;
    }
  };
  wave_lds_order();
  if (first < npairs) fetch(first);
  for (int pr = first; pr < npairs; pr += step) {
    // ---- stage: the x half, the pooled gradient and argmax bytes; clear the scatter image
    *(uint4*)(X + sj * XB + ((sp >> 2) + 1) * RBX + ((sp & 3) + 1) * PBX + 16 * sc) = pxv;
    *(uint2*)(P + sj * PB_P + sw * 8) = pdv;
    *(uint32_t*)(I + sj * PB_I + sw * 4) = piv;
    for (int e = lane; e < NI * FB / 16; e += 64) ((uint4*)F)[e] = make_uint4(0, 0, 0, 0);
    if (pr + step < npairs) fetch(pr + step);
    wave_lds_order();
    // ---- scatter: lane = (image, channel); the 4 windows of a 2x2 map have 4 distinct
    // parities, one phase each, so no two lanes of a phase add into the same element
    {
      const int j = lane >> 5, ch = lane & 31;
      const bf16* pd = (const bf16*)(P + j * PB_P);
      const uint8_t* pi = (const uint8_t*)(I + j * PB_I);
      float* fj = F + j * (FB / 4);
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int t = pi[w * CO + ch];
        const int ky = t / 3, kx = t - 3 * ky;
        const int py = 2 * (w >> 1) - 1 + ky, px = 2 * (w & 1) - 1 + kx;
        float* f = fj + (py * W + px) * FST + ch;
        *f = *f + __bfloat162float(pd[w * CO + ch]);
        wave_lds_order();
      }
    }
    // ---- round into the halo'd bf16 dc tiles (lane = image, pixel, 16-channel half)
    {
      const float* fr = F + sj * (FB / 4) + sp * FST + 16 * sc;
      uint32_t o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = cvt_pk2(fr[2 * c], fr[2 * c + 1]);
      char* dq = D + sj * DB + ((sp >> 2) + 1) * RBD + ((sp & 3) + 1) * PBD + 32 * sc;
      *(uint4*)dq = make_uint4(o[0], o[1], o[2], o[3]);
      *(uint4*)(dq + 16) = make_uint4(o[4], o[5], o[6], o[7]);
    }
    wave_lds_order();
    // ---- dx[ci half] = conv^T(dc): one 16-pixel block x 9 K chunks per image
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      Frag8 fr[9];
#pragma unroll
      for (int c = 0; c < 9; ++c)
        fr[c].u = *(const uint4*)(D + j * DB + ((li >> 2) + c / 3) * RBD + ((li & 3) + c % 3) * PBD +
                                  16 * g);
      f32x4 acc_d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 9; ++c)
        acc_d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wd[c].v, fr[c].v, acc_d, 0, 0, 0);
      const int img = NI * pr + j;
      if (img < a.N)
        *(uint2*)(a.dx + ((size_t)img * HW + li) * CI + CH * h + 4 * g) =
            make_uint2(cvt_pk2(acc_d[0], acc_d[1]), cvt_pk2(acc_d[2], acc_d[3]));
    }
    // ---- dW[:, :, ci half] += x (x) dc over the pair's 32 pixels
    {
      Frag8 af[2];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          af[mb].h[hh] = tr_read(D + wj * DB + (wrow + hh + 1) * RBD + (q + 1) * PBD + mb * 32 +
                                 8 * p4);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        Frag8 bf;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          bf.h[hh] = tr_read(X + wj * XB + (wrow + hh + t / 3) * RBX + (q + t % 3) * PBX + 8 * p4);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          acc[mb][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bf.v, acc[mb][t], 0, 0, 0);
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
        accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, ones.v, accb[mb], 0, 0, 0);
    }
    wave_lds_order();  // the next pair's staging overwrites the tiles
  }
  // ---- per-workgroup partial row: pair 0 writes, pair 1 adds (fixed order); the two waves
  // of a pair own disjoint input channels, wave 0 of a pair the bias
  float* red = (float*)smem;
  for (int pp = 0; pp < NW / 2; ++pp) {
    __syncthreads();
    if ((wave >> 1) != pp) continue;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* e = red + (mb * 16 + 4 * g + i) * KTOT + t * CI + CH * h + li;
          *e = pp ? *e + acc[mb][t][i] : acc[mb][t][i];
        }
      if (h == 0 && li == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* e = red + CO * KTOT + mb * 16 + 4 * g + i;
          *e = pp ? *e + accb[mb][i] : accb[mb][i];
        }
    }
  }
  __syncthreads();
  float* out = a.partial + (size_t)blockIdx.x * ROWF;
  for (int e = tid; e < ROWF; e += kPT) out[e] = red[e];
}

}  // namespace

static bool pool_conv_s1(int cin, int cout, int H, int W) {
  return cin == s1::CI && cout == s1::CO && H == s1::H && W == s1::W;
}
static bool pool_conv_s2(int cin, int cout, int H, int W) {
  return cin == s2::CI && cout == s2::CO && H == s2::H && W == s2::W;
}

// Partial rows mbk_pool_conv_bwd writes (= its grid) for N images of a supported shape
// (16 -> 32 channels on 8x8 maps pooled 4x4; 32 -> 32 on 4x4 pooled 2x2); <= 0: unsupported.
extern "C" int mbk_pool_conv_bwd_parts(int N, int cin, int cout, int H, int W) {
  const bool one = pool_conv_s1(cin, cout, H, W);
  if (N <= 0 || !(one || pool_conv_s2(cin, cout, H, W))) return -1;
  static int cus = 0, per1 = 0, per2 = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    (void)hipFuncSetAttribute((const void*)pool_conv_bwd_s1_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, s1::SMEM);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per1, (const void*)pool_conv_bwd_s1_kernel,
                                                     s1::kPT, s1::SMEM) != hipSuccess || per1 < 1)
      per1 = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, (const void*)pool_conv_bwd_s2_kernel,
                                                     s2::kPT, s2::SMEM) != hipSuccess || per2 < 1)
      per2 = 1;
  }
  const int rounds = one ? (N + s1::NW - 1) / s1::NW
                         : ((N + s2::NI - 1) / s2::NI + s2::NW / 2 - 1) / (s2::NW / 2);
  return std::max(1, std::min(rounds, cus * mbk_occ_b(one ? per1 : per2)));
}

// dx = conv^T(pool_bwd(dp, pidx)) and the conv's weight / bias gradients (dw [cout][cin][3][3],
// db [cout], fp32; accumulate: add instead of overwrite). partial:
// mbk_pool_conv_bwd_partial_floats(nparts, cin, cout) floats (the rows plus the reduce's scratch
// rows, conv.hip mbk_wgrad_reduce).
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
  if (pool_conv_s1(cin, cout, H, W))
    hipLaunchKernelGGL(pool_conv_bwd_s1_kernel, dim3(nparts), dim3(s1::kPT), s1::SMEM, stream, a);
  else
    hipLaunchKernelGGL(pool_conv_bwd_s2_kernel, dim3(nparts), dim3(s2::kPT), s2::SMEM, stream, a);
  const int rc = (int)hipGetLastError();
  if (rc || !dw) return rc;  // dw == nullptr: the caller reduces (mbk_wgrad_reduce_batch)
  return mbk_wgrad_reduce(partial, nparts, cin, cin, cout, dw, db, accumulate, stream);
}

extern "C" int64_t mbk_pool_conv_bwd_partial_floats(int nparts, int cin, int cout) {
  return (int64_t)(nparts + (nparts + 31) / 32) * (cout * 9 * cin + cout);
}
