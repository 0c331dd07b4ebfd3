// General bf16 GEMM on v_mfma_f32_16x16x32_bf16: C[M][N] = A[M][K] . B[N][K]^T (+ bias[N])
// (+ relu), fp32 accumulation, bf16 or fp32 output (optionally accumulated into fp32 C).
//
// Both operands are K-contiguous ("NT"), the layout every caller here has natively:
// Linear forward (x . W^T), its input gradient (g . W with W pre-transposed once per
// call, a few hundred KB) and convolutions as im2col . W^T (GridNet). The weight
// gradient (g^T x, K = batch) is the split-K kernel in fc.hip.
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (4 waves as 2 x 2, each 64 x 64 =
// 4 x 4 MFMA tiles), K step 32, A / B tiles double-buffered in LDS with a 16-byte row pad
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
constexpr int TM = 128, TN = 128, TK = 32;
constexpr int ROWB = TK * 2 + 16;  // LDS row stride (bytes): 32 bf16 + pad

union Frag8 {
  bf16x8 v;
  uint4 u;
};

// one 128 x 32 bf16 tile = 512 uint4; each thread moves 2
__device__ __forceinline__ void load_tile(const bf16* __restrict__ g, int rows, int ld, int r0,
                                          int k0, int K, uint4 r[2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = threadIdx.x + j * kThreads;
    const int row = e >> 2, q = e & 3;
    const int gr = r0 + row, gk = k0 + q * 8;
    r[j] = (gr < rows && gk < K) ? *(const uint4*)(g + (size_t)gr * ld + gk)
                                 : make_uint4(0, 0, 0, 0);
  }
}

// Shifted-row A operand ("implicit im2col"): K is split into ntap blocks of tk columns
// (tk % 32 == 0, so a 32-wide K step never straddles two taps); block t reads row
// m + shift[t] of its own matrix base[t] ([rows][lda], K-contiguous), zero outside [0, rows).
// A 3x3 conv over a zero-padded NHWC grid is then ONE GEMM (tap shifts dy*Wp + dx), and a
// stride-2 transposed conv is four sub-pixel phase GEMMs of 1 / 2 / 2 / 4 taps.
constexpr int kMaxTaps = 9;
struct ATaps {
  const bf16* base[kMaxTaps];
  int shift[kMaxTaps];
  int ntap, tk;
};

__device__ __forceinline__ void load_tile_taps(const ATaps& t, int rows, int ld, int r0, int k0,
                                               uint4 r[2]) {
  const int tap = k0 / t.tk, kin = k0 - tap * t.tk;
  const bf16* g = t.base[tap];
  const int sh = t.shift[tap];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = threadIdx.x + j * kThreads;
    const int row = e >> 2, q = e & 3;
    const int gr = r0 + row + sh;
    r[j] = (gr >= 0 && gr < rows && tap < t.ntap)
               ? *(const uint4*)(g + (size_t)gr * ld + kin + q * 8)
               : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void store_tile(char* t, const uint4 r[2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = threadIdx.x + j * kThreads;
    *(uint4*)(t + (e >> 2) * ROWB + (e & 3) * 16) = r[j];
  }
}

template <bool OUT_BF16, bool TAPS>
__global__ __launch_bounds__(kThreads) void gemm_nt_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, void* __restrict__ C,
    const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int relu,
    int accumulate, ATaps taps) {
  __shared__ __attribute__((aligned(16))) char sm[2][2][TM * ROWB];  // [buf][A|B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;  // 2 x 2 waves of 64 x 64
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 ra[2], rb[2];
  if (TAPS) load_tile_taps(taps, M, lda, m0, 0, ra);
  else load_tile(A, M, lda, m0, 0, K, ra);
  load_tile(B, N, ldb, n0, 0, K, rb);
  store_tile(sm[0][0], ra);
  store_tile(sm[0][1], rb);
  __syncthreads();
  const int nk = (K + TK - 1) / TK;
  for (int kk = 0; kk < nk; ++kk) {
    const int cur = kk & 1;
    if (kk + 1 < nk) {  // prefetch the next K step into registers
      if (TAPS) load_tile_taps(taps, M, lda, m0, (kk + 1) * TK, ra);
      else load_tile(A, M, lda, m0, (kk + 1) * TK, K, ra);
      load_tile(B, N, ldb, n0, (kk + 1) * TK, K, rb);
    }
    const char* ta = sm[cur][0];
    const char* tb = sm[cur][1];
    Frag8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i].u = *(const uint4*)(ta + (wm * 64 + i * 16 + li) * ROWB + g * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      fb[j].u = *(const uint4*)(tb + (wn * 64 + j * 16 + li) * ROWB + g * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
    if (kk + 1 < nk) {
      store_tile(sm[cur ^ 1][0], ra);
      store_tile(sm[cur ^ 1][1], rb);
    }
    __syncthreads();
  }
  // epilogue: C layout row = 4g + r (M), col = li (N) within each 16 x 16 tile
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + li;
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + 4 * g + r;
        if (row >= M) continue;
        float v = acc[i][j][r] + bv;
        if (relu) v = fmaxf(v, 0.f);
        const size_t o = (size_t)row * ldc + col;
        if (OUT_BF16) {
          ((bf16*)C)[o] = __float2bfloat16(v);
        } else {
          float* c = (float*)C + o;
          *c = accumulate ? *c + v : v;
        }
      }
    }
}

}  // namespace

// C = A . B^T (+ bias) (+ relu). A: [M][K] (row stride lda), B: [N][K] (ldb), bf16, K % 8 == 0,
// 16-byte aligned rows. out_bf16: C bf16 [M][ldc], else fp32 (accumulate: C += result).
extern "C" int mbk_gemm_nt(const void* A, const void* B, void* C, const float* bias, int M, int N,
                           int K, int lda, int ldb, int ldc, int relu, int out_bf16,
                           int accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 8 || lda % 8 || ldb % 8) return (int)hipErrorInvalidValue;
  dim3 grid((M + TM - 1) / TM, (N + TN - 1) / TN);
  ATaps none{};
  if (out_bf16)
    hipLaunchKernelGGL((gemm_nt_kernel<true, false>), grid, dim3(kThreads), 0, stream,
                       (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, relu, 0,
                       none);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<false, false>), grid, dim3(kThreads), 0, stream,
                       (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, relu,
                       accumulate, none);
  return (int)hipGetLastError();
}

// Shifted-row ("implicit im2col") GEMM: C[M][N] = sum_t A_t[m + shift_t][:] . B[:, t*tk ...]^T
// A_t: bases[t] [M][lda] bf16 (rows outside [0, M) read as zero), tk % 32 == 0,
// B: [N][ntap*tk] bf16 (tap-major K).
extern "C" int mbk_gemm_nt_taps(const void* const* bases, const int* shifts, int ntap, int tk,
                                const void* B, void* C, const float* bias, int M, int N, int lda,
                                int ldb, int ldc, int relu, int out_bf16, int accumulate,
                                hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (ntap < 1 || ntap > kMaxTaps || tk % 32 || lda % 8 || ldb % 8) return (int)hipErrorInvalidValue;
  ATaps t{};
  for (int i = 0; i < ntap; ++i) {
    t.base[i] = (const bf16*)bases[i];
    t.shift[i] = shifts[i];
  }
  t.ntap = ntap;
  t.tk = tk;
  const int K = ntap * tk;
  dim3 grid((M + TM - 1) / TM, (N + TN - 1) / TN);
  if (out_bf16)
    hipLaunchKernelGGL((gemm_nt_kernel<true, true>), grid, dim3(kThreads), 0, stream,
                       (const bf16*)nullptr, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc,
                       relu, 0, t);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<false, true>), grid, dim3(kThreads), 0, stream,
                       (const bf16*)nullptr, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc,
                       relu, accumulate, t);
  return (int)hipGetLastError();
}
