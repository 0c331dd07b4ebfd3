// Split-K weight gradient of the trunk-tail dense layers: dW[O][I] = sum_n g[n][o] x[n][i].
//
// Reference: the backward of nn.Linear(32*h/8*w/8, 256) and of the critic
// nn.Linear(256, 1) (model.py:119-137) on the learner batch, N = (T+1)*B ~ 266K rows.
// The output has only O*I/256 MFMA tiles (128 for network.5, 16 for the critic), so a
// library GEMM that parallelises over output tiles runs a handful of workgroups down a
// 266K-long K (0.57 ms measured, profiles/06); batched split-K through aten::bmm
// blocks the host. Here grid.x splits K, grid.y splits the output into 64x64 chunks,
// both operands are staged row-major in LDS and read K-major with ds_read_b64_tr_b16,
// fp32 partials are reduced by a deterministic two-level column sum. No host sync.
#include "common.h"

#include <cstdlib>

#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

constexpr int kThreads = 256;
constexpr int MBC = 4;          // output row blocks (16) per workgroup: 64 rows of W
constexpr int CBC = 4;          // output col blocks (16) per workgroup: 64 cols of W
constexpr int OC = MBC * 16, IC = CBC * 16;
constexpr int R = 128;          // K rows per LDS stage
constexpr int GROW = OC * 2;    // g tile row bytes
constexpr int XROW = IC * 2;    // x tile row bytes

union Frag8 {
  bf16x8 v;
  s16x4 h[2];
  uint4 u;
};

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}

// relu of 8 packed bf16 (sign bit set -> 0)
__device__ __forceinline__ uint4 relu8(uint4 v) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = ((w[j] & 0x8000u) ? 0u : (w[j] & 0xFFFFu)) |
           ((w[j] & 0x80000000u) ? 0u : (w[j] & 0xFFFF0000u));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// element e of the staged tile rows [r, r+R) x cols [c0, c0+W) of a row-major bf16 [N][ld]
// matrix (16 bytes: 8 columns of one row), zero-filled outside it
template <int W, bool VEC>
__device__ __forceinline__ uint4 stage_elem(const bf16* src, int r, int N, int c0, int ld, int e) {
  constexpr int C8 = W / 8;
  const int row = e / C8, c = c0 + (e % C8) * 8, n = r + row;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (n < N) {
    if (VEC && c + 8 <= ld) {
      v = *(const uint4*)(src + (size_t)n * ld + c);
    } else {
      uint16_t h[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        h[j] = c + j < ld ? __bfloat16_as_ushort(src[(size_t)n * ld + c + j]) : (uint16_t)0;
      v = make_uint4(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16,
                     h[4] | (uint32_t)h[5] << 16, h[6] | (uint32_t)h[7] << 16);
    }
  }
  return v;
}
// tile elements per thread per stage (R rows x 64 columns / 8 per element / kThreads)
constexpr int kSPF = R * 8 / kThreads;

// Row shifts of the x operand, one per output column block ("tap"): dW[o][t*I + i] =
// sum_n g[n][o] x[n + shift_t][i] -- the weight gradient of the shifted-row (implicit
// im2col) convolution GEMM in gemm.hip, all taps in one launch.
constexpr int kMaxTaps = 9;
struct XShifts {
  int s[kMaxTaps];
  int ntap;
  int relu_x;  // ntap == 1 only: dW = g^T relu(x)
};

// x tile element of the shifted-row weight gradient: output column c (of ntap * I) is
// channel c % I of tap c / I, i.e. x row n + shift[c / I]; each 8-column group lies in one tap
__device__ __forceinline__ uint4 stage_taps_elem(const bf16* src, int r, int N, int c0, int I,
                                                 int TI, const XShifts& xs, int nsrc, int e) {
  constexpr int C8 = IC / 8;
  const int row = e / C8, c = c0 + (e % C8) * 8;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (r + row < N && c < TI) {
    const int tap = c / I;
    const int n = r + row + xs.s[tap];
    if (n >= 0 && n < nsrc) v = *(const uint4*)(src + (size_t)n * I + (c - tap * I));
  }
  return v;
}

template <bool GVEC>
__global__ __launch_bounds__(kThreads) void fc_wgrad_kernel(const bf16* __restrict__ g,
                                                            const bf16* __restrict__ x, int N,
                                                            int O, int I, int rows_per_part,
                                                            float* __restrict__ partial,
                                                            XShifts xs, int chunk_fast) {
  __shared__ __attribute__((aligned(16))) char smem[R * GROW + R * XROW];
  char* gt = smem;
  char* xt = smem + R * GROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int TI = xs.ntap * I;  // output row width: ntap blocks of I columns
  const int ncb = (TI + IC - 1) / IC;
  // chunk_fast: blockIdx.x = output chunk (fastest in dispatch order: the chunks of one row
  // range run together and share its g / x rows through L2 / MALL), blockIdx.y = row range
  const int chunk = chunk_fast ? blockIdx.x : blockIdx.y;
  const int part = chunk_fast ? blockIdx.y : blockIdx.x;
  const int o0 = (chunk / ncb) * OC, i0 = (chunk % ncb) * IC;
  const int r0 = part * rows_per_part, r1 = min(N, r0 + rows_per_part);
  f32x4 acc[MBC][CBC];
#pragma unroll
  for (int mb = 0; mb < MBC; ++mb)
#pragma unroll
    for (int cb = 0; cb < CBC; ++cb) acc[mb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the next stage's g / x tile elements are loaded into registers before this stage's
  // MFMAs (the loads were issued between two barriers and exposed every stage)
  uint4 pg[kSPF], px[kSPF];
  auto load = [&](int rs) {
#pragma unroll
    for (int k = 0; k < kSPF; ++k) {
      const int e = tid + k * kThreads;
      pg[k] = stage_elem<OC, GVEC>(g, rs, r1, o0, O, e);
      px[k] = xs.ntap == 1 ? stage_elem<IC, true>(x, rs, r1, i0, I, e)
                           : stage_taps_elem(x, rs, r1, i0, I, TI, xs, N, e);
    }
  };
  if (r0 < r1) load(r0);
  for (int rs = r0; rs < r1; rs += R) {
    __syncthreads();  // previous stage's reads done
#pragma unroll
    for (int k = 0; k < kSPF; ++k) {
      const int e = tid + k * kThreads;
      *(uint4*)(gt + e * 16) = pg[k];
      *(uint4*)(xt + e * 16) = xs.relu_x ? relu8(px[k]) : px[k];
    }
    __syncthreads();
    if (rs + R < r1) load(rs + R);
    const int nk = (min(R, r1 - rs) + 31) >> 5;
    for (int kb = wave; kb < nk; kb += kThreads / 64) {
      int prow[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) prow[h] = kb * 32 + 8 * G + 4 * h + (li >> 2);
      Frag8 af[MBC];
#pragma unroll
      for (int mb = 0; mb < MBC; ++mb)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          af[mb].h[h] = tr_read(gt + prow[h] * GROW + (mb * 16 + 4 * (li & 3)) * 2);
#pragma unroll
      for (int cb = 0; cb < CBC; ++cb) {
        Frag8 bfr;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          bfr.h[h] = tr_read(xt + prow[h] * XROW + (cb * 16 + 4 * (li & 3)) * 2);
#pragma unroll
        for (int mb = 0; mb < MBC; ++mb)
          acc[mb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bfr.v, acc[mb][cb], 0, 0, 0);
      }
    }
  }
  // ---- reduce the 4 waves through LDS (fixed order), write this part's chunk
  __syncthreads();
  float* red = (float*)smem;  // [OC][IC] fp32 = 32 KB of the 48 KB stage buffers
  static_assert(R * GROW + R * XROW >= OC * IC * 4, "reduction buffer");
  for (int w = 0; w < kThreads / 64; ++w) {
    if (wave == w) {
#pragma unroll
      for (int mb = 0; mb < MBC; ++mb)
#pragma unroll
        for (int cb = 0; cb < CBC; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* p = red + (mb * 16 + 4 * G + i) * IC + cb * 16 + li;
            *p = (w == 0 ? 0.f : *p) + acc[mb][cb][i];
          }
    }
    __syncthreads();
  }
  float* out = partial + (size_t)part * O * TI;
  for (int e = tid; e < OC * IC; e += kThreads) {
    const int o = o0 + e / IC, i = i0 + e % IC;
    if (o < O && i < TI) out[(size_t)o * TI + i] = red[e];
  }
}

// out[e] (+)= sum_p partial[p][e] over parts [y*pps, (y+1)*pps); `stage` set: write the
// split sums to stage[y][e] for a second pass. 64 columns x 4 part-lanes per block.
// out_b (or null): columns >= split go to out_b[e - split] instead (a W + b partial row)
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ partial, int nparts,
                                                     int pps, long row, float* __restrict__ stage,
                                                     float* __restrict__ out, int accumulate,
                                                     float* __restrict__ out_b = nullptr,
                                                     long split = 0) {
  __shared__ float red[4][64];
  const int col = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + col;
  const int p0 = blockIdx.y * pps, p1 = min(nparts, p0 + pps);
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
    stage[(size_t)blockIdx.y * row + e] = s;
    return;
  }
  float* o = out_b && e >= split ? out_b + (e - split) : out + e;
  *o = accumulate ? *o + s : s;
}

// Acting-path trunk tail, one launch: f = relu(relu(x) . W5^T + b5) (bf16 out) and the
// critic v = f . wc + bc (fp32 out). One workgroup per 16 frames; its 4 waves split the
// O hidden units (O/64 independent 16-wide blocks each). MFMA operands (A = W5 rows,
// B = x rows) so a lane holds 4 consecutive hidden units of one frame: 8-byte stores of
// f; critic partials reduce over lanes (shuffles) and waves (LDS). W5 (bf16,
// NHWC-permuted) is read through L2; x rows are relu'd at load, once per wave.
template <int O>
__global__ __launch_bounds__(256) void fc_fwd_kernel(const bf16* __restrict__ x, int relu_in,
                                                     const bf16* __restrict__ w5,
                                                     const float* __restrict__ b5,
                                                     const float* __restrict__ wc,
                                                     const float* __restrict__ bc, int F, int I,
                                                     bf16* __restrict__ f_out,
                                                     float* __restrict__ v_out) {
  constexpr int NBW = O / 64;  // 16-wide hidden blocks per wave
  __shared__ float vred[O / 16][16];  // per hidden block: the critic partial of each row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int r0 = blockIdx.x * 16;
  const int row = r0 + li;
  const bool valid = row < F;
  const uint4* xr = (const uint4*)(x + (size_t)(valid ? row : r0) * I) + G;
  const int nks = I / 32;
  f32x4 acc[NBW];
#pragma unroll
  for (int j = 0; j < NBW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < nks; ++ks) {
    uint4 xv = valid ? xr[ks * 4] : make_uint4(0, 0, 0, 0);
    if (relu_in) {
      uint32_t w[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = (w[j] & 0x8000u) ? 0u : (w[j] & 0xFFFFu);
        const uint32_t hi = (w[j] & 0x80000000u) ? 0u : (w[j] & 0xFFFF0000u);
        w[j] = lo | hi;
      }
      xv = make_uint4(w[0], w[1], w[2], w[3]);
    }
    Frag8 b;
    __builtin_memcpy(&b, &xv, 16);
    uint4 wv[NBW];
#pragma unroll
    for (int j = 0; j < NBW; ++j)
      wv[j] = ((const uint4*)(w5 + (size_t)((wave * NBW + j) * 16 + li) * I) + G)[ks * 4];
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      Frag8 a;
      __builtin_memcpy(&a, &wv[j], 16);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc[j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int h0 = (wave * NBW + j) * 16 + 4 * G;  // lane: hidden units h0..h0+3 of `row`
    float hv[4], w4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // the critic consumes the bf16-rounded activations (what the head sees)
      hv[i] = __bfloat162float(__float2bfloat16(fmaxf(acc[j][i] + b5[h0 + i], 0.f)));
      w4[i] = wc[h0 + i];
    }
    const float q = mbk::crit_block(hv, w4);
    if (G == 0) vred[wave * NBW + j][li] = q;
    uint32_t o[2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      o[k] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k])) |
             ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k + 1])) << 16);
    if (valid) *(uint2*)(f_out + (size_t)row * O + h0) = make_uint2(o[0], o[1]);
  }
  __syncthreads();
  if (threadIdx.x < 16 && r0 + (int)threadIdx.x < F) {
    const int t = threadIdx.x;
    v_out[r0 + t] = mbk::crit_sum(&vred[0][t], O / 16, 16, bc[0]);
  }
}

// fc_fwd_kernel's maths (same MFMA operands, K order and critic reduction: bit-identical)
// for small I (NKS = I / 32 <= 4, the 16x16 IMPALA trunk's I = 128): the workgroup is
// persistent over 16-row blocks and keeps its wave's W5 fragments (NBW x NKS uint4) and the
// bias / critic weights in VGPRs for the whole launch. fc_fwd_kernel re-read all of W5
// (64 KB at O = 256) through L2 for every 16 rows: 2.1 GB of L2 reads per 524K-row learner
// batch, which bound it (0.38 ms vs ~0.1 ms of HBM traffic). The next row block's x
// fragments are loaded before the current block's MFMAs.
template <int O, int NKS>
__global__ __launch_bounds__(256) void fc_fwd_rb_kernel(const bf16* __restrict__ x, int relu_in,
                                                        const bf16* __restrict__ w5,
                                                        const float* __restrict__ b5,
                                                        const float* __restrict__ wc,
                                                        const float* __restrict__ bc, int F,
                                                        bf16* __restrict__ f_out,
                                                        float* __restrict__ v_out) {
  // two 16-row blocks per iteration (one barrier per 32 rows: the per-block barrier and
  // critic reduction bounded the one-block form, 190 us per 524K rows)
  constexpr int NBW = O / 64, I = NKS * 32, RB = 2;
  __shared__ float vred[2][RB][O / 16][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int nrb = (F + 16 * RB - 1) / (16 * RB);  // 32-row groups
  Frag8 wf[NBW][NKS];
  float bb[NBW][4], ww[NBW][4];
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const uint4* wr = (const uint4*)(w5 + (size_t)((wave * NBW + j) * 16 + li) * I) + G;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const uint4 v = wr[ks * 4];
      __builtin_memcpy(&wf[j][ks], &v, 16);
    }
    const int h0 = (wave * NBW + j) * 16 + 4 * G;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bb[j][i] = b5[h0 + i];
      ww[j][i] = wc[h0 + i];
    }
  }
  const float bcv = bc[0];
  // named registers per block (indexed arrays filled in a lambda can land in scratch)
  uint4 xn0[NKS], xn1[NKS];
  auto load_x = [&](int rg) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int row = (rg * RB + r) * 16 + li;
      const uint4* xr = (const uint4*)(x + (size_t)(row < F ? row : 0) * I) + G;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) (r ? xn1 : xn0)[ks] = xr[ks * 4];
    }
  };
  if ((int)blockIdx.x < nrb) load_x(blockIdx.x);
  int buf = 0;
  for (int rg = blockIdx.x; rg < nrb; rg += gridDim.x, buf ^= 1) {
    uint4 xv0[NKS], xv1[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      xv0[ks] = xn0[ks];
      xv1[ks] = xn1[ks];
    }
    if (rg + (int)gridDim.x < nrb) load_x(rg + gridDim.x);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int row = (rg * RB + r) * 16 + li;
      const bool valid = row < F;
      f32x4 acc[NBW];
#pragma unroll
      for (int j = 0; j < NBW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        uint4 v = valid ? (r ? xv1[ks] : xv0[ks]) : make_uint4(0, 0, 0, 0);
        if (relu_in) v = relu8(v);
        Frag8 b;
        __builtin_memcpy(&b, &v, 16);
#pragma unroll
        for (int j = 0; j < NBW; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks].v, b.v, acc[j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        const int h0 = (wave * NBW + j) * 16 + 4 * G;
        float hv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          hv[i] = __bfloat162float(__float2bfloat16(fmaxf(acc[j][i] + bb[j][i], 0.f)));
        const float q = mbk::crit_block(hv, ww[j]);
        if (G == 0) vred[buf][r][wave * NBW + j][li] = q;
        uint32_t o[2];
#pragma unroll
        for (int k = 0; k < 2; ++k)
          o[k] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k])) |
                 ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hv[2 * k + 1])) << 16);
        if (valid) *(uint2*)(f_out + (size_t)row * O + h0) = make_uint2(o[0], o[1]);
      }
    }
    __syncthreads();  // (double-buffered: the next group's writes go to the other half)
    if (threadIdx.x < 16 * RB) {
      const int r = threadIdx.x >> 4, t = threadIdx.x & 15;
      const int row = (rg * RB + r) * 16 + t;
      if (row < F) v_out[row] = mbk::crit_sum(&vred[buf][r][0][t], O / 16, 16, bcv);
    }
  }
}


// ---- FC weight + bias gradient of the IMPALA tail, one pass: dW = g^T x, db = g^T 1 with
// O = 256 outputs and I = 16 CB inputs (128 on 16x16 maps). fc_wgrad_kernel's 64 x 64 output
// chunks re-read every g / x row per chunk (8 chunks) from 128-row stages holding 16 MFMAs per
// wave between two barriers (297 us per 524K rows, 1.3 TB/s); colsum then re-read g for db
// (76 us). Here a 512-thread workgroup (one per CU) owns all of W: wave w computes W rows
// 32 w .. 32 w + 31 against all I columns (A = g^T and B = x through ds_read_b64_tr_b16, row
// strides 32 mod 256 bytes with the 4-row block swap of head_bwd2: conflict-free), plus the
// bias as one more MFMA per K block against an all-ones B fragment; every g / x row is read
// from HBM once (the next stage's rows are in registers during this stage's MFMAs).
constexpr int FW_NW = 8, FW_RS = 128, FW_GR = 544, FW_XR = 288;
constexpr int FW_LDS = FW_RS * (FW_GR + FW_XR);

__device__ __forceinline__ int fw_phi(int r) {
  const int b = (r >> 2) & 3;
  return (b == 1 || b == 2) ? r ^ 12 : r;
}

template <int CB>
__global__ __launch_bounds__(64 * FW_NW, 1) void fc_wgrad_wide_kernel(
    const bf16* __restrict__ g, const bf16* __restrict__ x, int N, int relu_x,
    int stages_per_part, float* __restrict__ partial) {
  constexpr int O = 256, I = 16 * CB, MB = 2;
  constexpr int GQ = O / 8, XQ = I / 8;                    // uint4 per g / x row
  constexpr int NG = FW_RS * GQ / (64 * FW_NW), NX = (FW_RS * XQ + 64 * FW_NW - 1) / (64 * FW_NW);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* gt = smem;
  char* xt = smem + FW_RS * FW_GR;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int nst = (N + FW_RS - 1) / FW_RS;
  const int s0 = blockIdx.x * stages_per_part, s1 = min(nst, s0 + stages_per_part);
  f32x4 acc[MB][CB], accb[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    accb[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[mb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  uint4 pg[NG], px[NX];
  auto load = [&](int st) {
    const int n0 = st * FW_RS;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int e = tid + k * 64 * FW_NW, row = e / GQ, q = e % GQ;
      pg[k] = n0 + row < N ? ((const uint4*)(g + (size_t)(n0 + row) * O))[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int e = tid + k * 64 * FW_NW, row = e / XQ, q = e % XQ;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < FW_RS * XQ && n0 + row < N) v = ((const uint4*)(x + (size_t)(n0 + row) * I))[q];
      px[k] = relu_x ? relu8(v) : v;
    }
  };
  if (s0 < s1) load(s0);
  for (int st = s0; st < s1; ++st) {
    __syncthreads();  // the previous stage's tile reads are done
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int e = tid + k * 64 * FW_NW, row = e / GQ, q = e % GQ;
      *(uint4*)(gt + fw_phi(row) * FW_GR + q * 16) = pg[k];
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int e = tid + k * 64 * FW_NW, row = e / XQ, q = e % XQ;
      if (e < FW_RS * XQ) *(uint4*)(xt + fw_phi(row) * FW_XR + q * 16) = px[k];
    }
    __syncthreads();
    if (st + 1 < s1) load(st + 1);
#pragma unroll
    for (int kb = 0; kb < FW_RS / 32; ++kb) {
      int pr[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) pr[h] = fw_phi(kb * 32 + 8 * G + 4 * h + (li >> 2));
      Frag8 af[MB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          af[mb].h[h] = tr_read(gt + pr[h] * FW_GR + (32 * wave + mb * 16 + 4 * (li & 3)) * 2);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        accb[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, ones.v, accb[mb], 0, 0, 0);
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        Frag8 bfr;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          bfr.h[h] = tr_read(xt + pr[h] * FW_XR + (cb * 16 + 4 * (li & 3)) * 2);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bfr.v, acc[mb][cb], 0, 0, 0);
      }
    }
  }
  // this part's row of partials: W [O][I] then b [O]; lane (li, G) holds column cb*16 + li of
  // W rows 32 w + mb*16 + 4G + i
  float* out = partial + (size_t)blockIdx.x * (O * I + O);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 32 * wave + mb * 16 + 4 * G + i;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) out[o * I + cb * 16 + li] = acc[mb][cb][i];
      if (li == 0) out[O * I + o] = accb[mb][i];
    }
}

}  // namespace

extern "C" int mbk_fc_fwd(const void* x, int relu_in, const void* w5, const float* b5,
                          const float* wc, const float* bc, int F, int I, int O, void* f_out,
                          float* v_out, hipStream_t stream) {
  if (F <= 0) return 0;
  if (I % 32) return (int)hipErrorInvalidValue;
  const int blocks = (F + 15) / 16;
  if ((O == 256 || O == 128) && I <= 128) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (cus <= 0) cus = 256;
    }
    const int grid = std::min((blocks + 1) / 2, cus * 2);  // 32-row groups; 2 workgroups per CU
#define FC_RB(OO, KS)                                                                        \
  hipLaunchKernelGGL((fc_fwd_rb_kernel<OO, KS>), dim3(grid), dim3(256), 0, stream,          \
                     (const bf16*)x, relu_in, (const bf16*)w5, b5, wc, bc, F, (bf16*)f_out, \
                     v_out)
    const int nks = I / 32;
    if (O == 256) {
      if (nks == 1) FC_RB(256, 1); else if (nks == 2) FC_RB(256, 2);
      else if (nks == 3) FC_RB(256, 3); else FC_RB(256, 4);
    } else {
      if (nks == 1) FC_RB(128, 1); else if (nks == 2) FC_RB(128, 2);
      else if (nks == 3) FC_RB(128, 3); else FC_RB(128, 4);
    }
#undef FC_RB
    return (int)hipGetLastError();
  }
  if (O == 256)
    hipLaunchKernelGGL(fc_fwd_kernel<256>, dim3(blocks), dim3(256), 0, stream, (const bf16*)x,
                       relu_in, (const bf16*)w5, b5, wc, bc, F, I, (bf16*)f_out, v_out);
  else if (O == 128)
    hipLaunchKernelGGL(fc_fwd_kernel<128>, dim3(blocks), dim3(256), 0, stream, (const bf16*)x,
                       relu_in, (const bf16*)w5, b5, wc, bc, F, I, (bf16*)f_out, v_out);
  else if (O == 512)
    hipLaunchKernelGGL(fc_fwd_kernel<512>, dim3(blocks), dim3(256), 0, stream, (const bf16*)x,
                       relu_in, (const bf16*)w5, b5, wc, bc, F, I, (bf16*)f_out, v_out);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// number of K splits (partial rows) for an N x (O, I) problem
extern "C" int mbk_fc_wgrad_parts(int N, int O, int I) {
  (void)O;
  (void)I;
  const int stages = (N + R - 1) / R;
  return std::max(1, std::min(512, stages / 8));  // >= 8 stages (1024 rows) per split
}

namespace {
int fc_wgrad_impl(const void* g, const void* x, int N, int O, int I, const XShifts& xs,
                  float* partial, int nparts, float* out, int accumulate, hipStream_t stream) {
  if (N <= 0 || O <= 0 || I <= 0 || nparts < 1 || I % 8) return (int)hipErrorInvalidValue;
  const int stages = (N + R - 1) / R;
  const int rpp = ((stages + nparts - 1) / nparts) * R;
  const int chunks = ((O + OC - 1) / OC) * ((xs.ntap * I + IC - 1) / IC);
  // dispatch order: chunk-fastest for the shifted (conv) form, whose chunks re-read the same
  // rows
  const int cf = xs.ntap > 1 ? 1 : 0;
  const dim3 grid = cf ? dim3(chunks, nparts) : dim3(nparts, chunks);
  if (O % 8 == 0)
    hipLaunchKernelGGL(fc_wgrad_kernel<true>, grid, dim3(kThreads), 0, stream, (const bf16*)g,
                       (const bf16*)x, N, O, I, rpp, partial, xs, cf);
  else  // e.g. the critic, O = 1
    hipLaunchKernelGGL(fc_wgrad_kernel<false>, grid, dim3(kThreads), 0, stream, (const bf16*)g,
                       (const bf16*)x, N, O, I, rpp, partial, xs, cf);
  const long row = (long)O * I * xs.ntap;
  const unsigned cols = (unsigned)((row + 63) / 64);
  constexpr int kPps = 32;
  if (nparts > 2 * kPps) {
    const int splits = (nparts + kPps - 1) / kPps;
    float* st = partial + (size_t)nparts * row;
    hipLaunchKernelGGL(colsum_kernel, dim3(cols, splits), dim3(256), 0, stream,
                       (const float*)partial, nparts, kPps, row, st, (float*)nullptr, 0);
    hipLaunchKernelGGL(colsum_kernel, dim3(cols, 1), dim3(256), 0, stream, (const float*)st,
                       splits, splits, row, (float*)nullptr, out, accumulate);
  } else {
    hipLaunchKernelGGL(colsum_kernel, dim3(cols, 1), dim3(256), 0, stream,
                       (const float*)partial, nparts, nparts, row, (float*)nullptr, out,
                       accumulate);
  }
  return (int)hipGetLastError();
}
}  // namespace

// partial: (nparts + ceil(nparts / 32)) * O * I floats of scratch; out: fp32 [O][I]
extern "C" int mbk_fc_wgrad(const void* g, const void* x, int N, int O, int I, float* partial,
                            int nparts, float* out, int accumulate, hipStream_t stream) {
  XShifts xs{};
  xs.ntap = 1;
  return fc_wgrad_impl(g, x, N, O, I, xs, partial, nparts, out, accumulate, stream);
}

// fc_wgrad_wide_kernel's part count for N rows (one workgroup per CU, >= 4 stages each);
// 0: the shape (O = 256, I in {32, 64, 128}) is not covered
extern "C" int mbk_fc_wgrad_wide_parts(int N, int O, int I) {
  if (O != 256 || (I != 32 && I != 64 && I != 128) || N <= 0) return 0;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int nst = (N + FW_RS - 1) / FW_RS;
  return std::max(1, std::min(cus, (nst + 3) / 4));
}

// dW = g^T relu?(x) and db = column sums of g in one pass (fc_wgrad_wide_kernel) for
// O = 256, I in {32, 64, 128}: out = fp32 [O][I], out_b = fp32 [O]. partial: (nparts +
// ceil(nparts / 32)) * (O * I + O) floats of scratch.
extern "C" int mbk_fc_wgrad_wide(const void* g, const void* x, int N, int O, int I, int relu_x,
                                 float* partial, int nparts, float* out, float* out_b,
                                 hipStream_t stream) {
  if (mbk_fc_wgrad_wide_parts(N, O, I) == 0 || nparts < 1) return (int)hipErrorInvalidValue;
  const int nst = (N + FW_RS - 1) / FW_RS;
  const int spp = (nst + nparts - 1) / nparts;
  const void* kfn = I == 128 ? (const void*)fc_wgrad_wide_kernel<8>
                    : I == 64 ? (const void*)fc_wgrad_wide_kernel<4>
                              : (const void*)fc_wgrad_wide_kernel<2>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)fc_wgrad_wide_kernel<8>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, FW_LDS);
    hipFuncSetAttribute((const void*)fc_wgrad_wide_kernel<4>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, FW_LDS);
    hipFuncSetAttribute((const void*)fc_wgrad_wide_kernel<2>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, FW_LDS);
    attr = true;
  }
  const bf16* gp = (const bf16*)g;
  const bf16* xp = (const bf16*)x;
  void* args[] = {&gp, &xp, &N, &relu_x, (void*)&spp, &partial};
  hipLaunchKernel(kfn, dim3(nparts), dim3(64 * FW_NW), args, FW_LDS, stream);
  const long row = (long)O * I + O;
  const unsigned cols = (unsigned)((row + 63) / 64);
  constexpr int kPps = 32;
  if (nparts > 2 * kPps) {
    const int splits = (nparts + kPps - 1) / kPps;
    float* st = partial + (size_t)nparts * row;
    hipLaunchKernelGGL(colsum_kernel, dim3(cols, splits), dim3(256), 0, stream,
                       (const float*)partial, nparts, kPps, row, st, (float*)nullptr, 0);
    hipLaunchKernelGGL(colsum_kernel, dim3(cols, 1), dim3(256), 0, stream, (const float*)st,
                       splits, splits, row, (float*)nullptr, out, 0, out_b, (long)O * I);
  } else {
    hipLaunchKernelGGL(colsum_kernel, dim3(cols, 1), dim3(256), 0, stream,
                       (const float*)partial, nparts, nparts, row, (float*)nullptr, out, 0, out_b,
                       (long)O * I);
  }
  return (int)hipGetLastError();
}

// mbk_fc_wgrad with relu_x: dW = g^T relu(x) (the pre-relu trunk output is what is saved)
extern "C" int mbk_fc_wgrad_ex(const void* g, const void* x, int N, int O, int I, float* partial,
                               int nparts, float* out, int accumulate, int relu_x,
                               hipStream_t stream) {
  XShifts xs{};
  xs.ntap = 1;
  xs.relu_x = relu_x;
  return fc_wgrad_impl(g, x, N, O, I, xs, partial, nparts, out, accumulate, stream);
}
