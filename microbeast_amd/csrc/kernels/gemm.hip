// General bf16 GEMM on v_mfma_f32_16x16x32_bf16: C[M][N] = A[M][K] . B[N][K]^T (+ bias[N])
// (+ relu), fp32 accumulation, bf16 or fp32 output (optionally accumulated into fp32 C).
//
// Both operands are K-contiguous ("NT"), the layout every caller here has natively:
// Linear forward (x . W^T) and its input gradient (g . W with W pre-transposed once per
// call, a few hundred KB): the trunk tail's dX and GridNet's critic output layer. The weight
// gradient (g^T x, K = batch) is the split-K kernel in fc.hip; GridNet's convolutions are
// pixconv.hip.
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (4 waves as 2 x 2, each 64 x 64 =
// 4 x 4 MFMA tiles), or 256 x 64 / 256 x 32 for narrow N (waves stacked along M), K step 32, A / B tiles double-buffered in LDS with a 16-byte row pad
// (conflict-free ds_read_b128 of the 8-element fragments). Global loads for step k+1 are
// issued before the MFMAs of step k. Edges are zero-filled, so any M, N and K % 8 == 0 work.
// blockIdx.x walks M (the large dimension in every use) and XCD-interleaves nothing: the
// B operand (weights) is the shared one and sits in every XCD's L2 after first touch.
#include "common.h"

#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

constexpr int kThreads = 256;
constexpr int TK = 32;
constexpr int ROWB = TK * 2 + 16;  // LDS row stride (bytes): 32 bf16 + pad

union Frag8 {
  bf16x8 v;
  uint4 u;
};

// K step TK of a ROWS-row tile = ROWS * 4 uint4; thread e moves elements e, e + 256, ...
template <int ROWS>
struct TileRegs {
  static constexpr int kN = (ROWS * 4 + kThreads - 1) / kThreads;
  uint4 r[kN];
};

template <int ROWS>
__device__ __forceinline__ void load_tile(const bf16* __restrict__ g, int rows, int ld, int r0,
                                          int k0, int K, TileRegs<ROWS>& t) {
#pragma unroll
  for (int j = 0; j < TileRegs<ROWS>::kN; ++j) {
    const int e = threadIdx.x + j * kThreads;
    const int row = e >> 2, q = e & 3;
    const int gr = r0 + row, gk = k0 + q * 8;
    t.r[j] = (row < ROWS && gr < rows && gk < K) ? *(const uint4*)(g + (size_t)gr * ld + gk)
                                                 : make_uint4(0, 0, 0, 0);
  }
}

// epilogue options: optional relu-backward mask in the output's layout (C[o] = 0 where
// mask[o] <= 0)
struct Epi {
  const bf16* mask;
};

template <int ROWS>
__device__ __forceinline__ void store_tile(char* t, const TileRegs<ROWS>& tr) {
#pragma unroll
  for (int j = 0; j < TileRegs<ROWS>::kN; ++j) {
    const int e = threadIdx.x + j * kThreads;
    if (e < ROWS * 4) *(uint4*)(t + (e >> 2) * ROWB + (e & 3) * 16) = tr.r[j];
  }
}

// Tile shapes: TN = 128 -> 128 x 128 tile, waves 2 x 2 of 64 x 64; TN = 64 / 32 (narrow N)
// -> 256 x TN tile, waves stacked along M, 64 x TN each, so no MFMA work is spent on padding
// columns.
template <int TN_>
struct Shape {
  static constexpr int TM = TN_ == 128 ? 128 : 256;
  static constexpr int WN = TN_ == 128 ? 2 : 1;  // waves along N
  static constexpr int NJ = TN_ / WN / 16;      // 16-col MFMA tiles per wave
};

template <bool OUT_BF16, int TN_>
__global__ __launch_bounds__(kThreads) void gemm_nt_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, void* __restrict__ C,
    const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int relu,
    int accumulate, Epi epi, int vec_out) {
  using S = Shape<TN_>;
  constexpr int TM_ = S::TM, NJ = S::NJ;
  // A / B double buffers; the bf16 output tile of the vectorised epilogue reuses them
  constexpr int kAB = 2 * TM_ * ROWB + 2 * TN_ * ROWB, OROW = TN_ * 2 + 16;
  static_assert(kAB >= TM_ * OROW, "output tile");
  __shared__ __attribute__((aligned(16))) char sab[kAB];
  char (*sa)[TM_ * ROWB] = (char (*)[TM_ * ROWB])sab;
  char (*sb)[TN_ * ROWB] = (char (*)[TN_ * ROWB])(sab + 2 * TM_ * ROWB);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wm = wave / S::WN, wn = wave % S::WN;
  const int m0 = blockIdx.x * TM_, n0 = blockIdx.y * TN_;
  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  TileRegs<TM_> ra;
  TileRegs<TN_> rb;
  load_tile<TM_>(A, M, lda, m0, 0, K, ra);
  load_tile<TN_>(B, N, ldb, n0, 0, K, rb);
  store_tile<TM_>(sa[0], ra);
  store_tile<TN_>(sb[0], rb);
  __syncthreads();
  const int nk = (K + TK - 1) / TK;
  for (int kk = 0; kk < nk; ++kk) {
    const int cur = kk & 1;
    if (kk + 1 < nk) {  // prefetch the next K step into registers
      load_tile<TM_>(A, M, lda, m0, (kk + 1) * TK, K, ra);
      load_tile<TN_>(B, N, ldb, n0, (kk + 1) * TK, K, rb);
    }
    const char* ta = sa[cur];
    const char* tb = sb[cur];
    Frag8 fa[4], fb[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i].u = *(const uint4*)(ta + (wm * 64 + i * 16 + li) * ROWB + g * 16);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      fb[j].u = *(const uint4*)(tb + (wn * NJ * 16 + j * 16 + li) * ROWB + g * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
    if (kk + 1 < nk) {
      store_tile<TM_>(sa[cur ^ 1], ra);
      store_tile<TN_>(sb[cur ^ 1], rb);
    }
    __syncthreads();
  }
  if constexpr (OUT_BF16) {
    if (vec_out) {
      // bf16 output through an LDS tile: 16-byte mask loads and C stores (the per-element
      // form issued 2-byte loads / stores, 64 of each per lane: the masked dX GEMM of
      // network.5 ran at ~1/3 of its HBM roofline). Same values: bias / relu before the
      // bf16 rounding, the mask zeroes a rounded value.
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int trow = wm * 64 + i * 16 + 4 * g + r;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int tcol = wn * NJ * 16 + j * 16 + li, col = n0 + tcol;
            float v = acc[i][j][r] + ((bias && col < N) ? bias[col] : 0.f);
            if (relu) v = fmaxf(v, 0.f);
            *(bf16*)(sab + trow * OROW + tcol * 2) = __float2bfloat16(v);
          }
        }
      __syncthreads();
      constexpr int C8 = TN_ / 8;
      for (int e = threadIdx.x; e < TM_ * C8; e += kThreads) {
        const int trow = e / C8, c8 = e % C8, row = m0 + trow, col = n0 + c8 * 8;
        if (row >= M || col >= N) continue;
        uint4 v = *(const uint4*)(sab + trow * OROW + c8 * 16);
        const size_t o = (size_t)row * ldc + col;
        if (epi.mask) {
          const uint4 mk = *(const uint4*)(epi.mask + o);
          const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
          uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t keep = (__uint_as_float(mw[q] << 16) > 0.f ? 0xFFFFu : 0u) |
                                  (__uint_as_float(mw[q] & 0xFFFF0000u) > 0.f ? 0xFFFF0000u : 0u);
            vw[q] &= keep;
          }
          v = make_uint4(vw[0], vw[1], vw[2], vw[3]);
        }
        *(uint4*)((bf16*)C + o) = v;
      }
      return;
    }
  }
  // epilogue: C layout row = 4g + r (M), col = li (N) within each 16 x 16 tile
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 64 + i * 16 + 4 * g + r;
      if (row >= M) continue;
      const size_t orow = row;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn * NJ * 16 + j * 16 + li;
        if (col >= N) continue;
        float v = acc[i][j][r] + (bias ? bias[col] : 0.f);
        if (relu) v = fmaxf(v, 0.f);
        const size_t o = orow * ldc + col;
        if (epi.mask && !(__bfloat162float(epi.mask[o]) > 0.f)) v = 0.f;
        if (OUT_BF16) {
          ((bf16*)C)[o] = __float2bfloat16(v);
        } else {
          float* c = (float*)C + o;
          *c = accumulate ? *c + v : v;
        }
      }
    }
}

template <int TN_>
void launch(const void* A, const void* B, void* C, const float* bias, int M, int N, int K,
            int lda, int ldb, int ldc, int relu, int out_bf16, int accumulate, const Epi& t,
            hipStream_t stream) {
  dim3 grid((M + Shape<TN_>::TM - 1) / Shape<TN_>::TM, (N + TN_ - 1) / TN_);
  // 16-byte output rows (and mask rows) for the vectorised bf16 epilogue
  const int vec = (out_bf16 && N % 8 == 0 && ldc % 8 == 0 &&
                   ((uintptr_t)C & 15) == 0 && ((uintptr_t)t.mask & 15) == 0) ? 1 : 0;
  if (out_bf16)
    hipLaunchKernelGGL((gemm_nt_kernel<true, TN_>), grid, dim3(kThreads), 0, stream,
                       (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, relu, 0,
                       t, vec);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<false, TN_>), grid, dim3(kThreads), 0, stream,
                       (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, relu,
                       accumulate, t, 0);
}

// narrowest tile that covers N (N = 78 -> one 128-wide tile rather than two of 64)
void launch_any(const void* A, const void* B, void* C, const float* bias, int M, int N, int K,
                int lda, int ldb, int ldc, int relu, int out_bf16, int accumulate,
                const Epi& t, hipStream_t stream) {
  if (N <= 32)
    launch<32>(A, B, C, bias, M, N, K, lda, ldb, ldc, relu, out_bf16, accumulate, t, stream);
  else if (N <= 64)
    launch<64>(A, B, C, bias, M, N, K, lda, ldb, ldc, relu, out_bf16, accumulate, t, stream);
  else
    launch<128>(A, B, C, bias, M, N, K, lda, ldb, ldc, relu, out_bf16, accumulate, t, stream);
}

}  // namespace

// C = A . B^T (+ bias) (+ relu). A: [M][K] (row stride lda), B: [N][K] (ldb), bf16, K % 8 == 0,
// 16-byte aligned rows. out_bf16: C bf16 [M][ldc], else fp32 (accumulate: C += result).
extern "C" int mbk_gemm_nt(const void* A, const void* B, void* C, const float* bias, int M, int N,
                           int K, int lda, int ldb, int ldc, int relu, int out_bf16,
                           int accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 8 || lda % 8 || ldb % 8) return (int)hipErrorInvalidValue;
  Epi none{};
  launch_any(A, B, C, bias, M, N, K, lda, ldb, ldc, relu, out_bf16, accumulate, none,
                    stream);
  return (int)hipGetLastError();
}

// mbk_gemm_nt with a relu-backward mask: C[m][n] = 0 where mask[m * ldc + n] <= 0 (bf16,
// the forward activation in C's layout), e.g. dX of network.5 through the trunk-output relu
extern "C" int mbk_gemm_nt_mask(const void* A, const void* B, void* C, const float* bias, int M,
                                int N, int K, int lda, int ldb, int ldc, int relu, int out_bf16,
                                const void* mask, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 8 || lda % 8 || ldb % 8) return (int)hipErrorInvalidValue;
  Epi t{};
  t.mask = (const bf16*)mask;
  launch_any(A, B, C, bias, M, N, K, lda, ldb, ldc, relu, out_bf16, 0, t, stream);
  return (int)hipGetLastError();
}
