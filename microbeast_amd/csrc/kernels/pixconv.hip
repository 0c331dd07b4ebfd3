// GridNet layers on the pixel-major "PBC" layout: activations [pixel][image][channel] (bf16).
//
// GridNet (BASELINE config 2, models/gridnet.py) is a conv / max-pool encoder down to 1x1 and
// a stride-2 transposed-conv decoder back to the map, on tiny spatial grids (16x16 .. 1x1)
// with 32..256 channels. With the image index INSIDE the pixel, every layer is a set of
// per-output-pixel GEMMs whose rows are images:
//
//   out[P][b][:] = bias + sum_{(q, t) in pairs(P)} A[q][b][:] . W_t^T
//
// pairs(P) = the (source pixel, weight tap) pairs that are in range for output pixel P -- a
// conv3x3 at a map corner has 4, in the interior 9; a stride-2 transposed conv 1, 2 or 4
// (its sub-pixel phases). A workgroup owns one output pixel x 128 images x one output-channel
// tile, so the tap validity is uniform over the tile: no zero-padded halo rows are computed
// (the padded-grid shifted-row GEMM this replaces spent 1.6x..9x the useful MFMA work on the
// 8x8..1x1 grids), no im2col exists, and a row of A is one image's channels at one pixel --
// 64..512 contiguous bytes. The same kernel runs
//   * conv / transposed-conv forward (bias + relu epilogue),
//   * their input gradient (the inverse pair lists, transposed weights, relu-mask epilogue),
//   * the critic's first Linear (pairs = the z pixels),
// and any A / C layout given as (pixel stride, image stride) in elements, so the first layer's
// NHWC output (conv.hip) is read in place (relu on load) and its input gradient written in
// place (mask = relu of that output).
//
// The weight gradient dW_t = sum_{(P, q) in pairs(t)} sum_b g[P][b]^T x[q][b] is a split-K
// GEMM over (pair, image) rows with both operands staged row-major and read K-major by
// ds_read_b64_tr_b16; fp32 partials are reduced straight into the parameter's own layout
// through an index map. Max-pool 3x3/2 (+ uint8 argmax) and its gather-form backward are
// elementwise kernels on the same layout.
//
// All shapes are checked on the host (mbk_pconv_* return hipErrorInvalidValue).
#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

constexpr int kThreads = 256;
constexpr int BK = 64;              // K step: two 32-wide MFMA K blocks
constexpr int ROWB = BK * 2 + 16;   // LDS row bytes (16-byte pad: conflict-free b128 reads)
constexpr int kMaxPairs = 16;

union Frag8 {
  bf16x8 v;
  uint4 u;
  s16x4 h[2];
};

__device__ __forceinline__ uint4 relu8(uint4 v) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = ((w[j] & 0x8000u) ? 0u : (w[j] & 0xFFFFu)) |
           ((w[j] & 0x80000000u) ? 0u : (w[j] & 0xFFFF0000u));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// keep v's bf16 halves where the mask's bf16 halves are > 0
__device__ __forceinline__ uint4 mask8(uint4 v, uint4 m) {
  const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
  uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = ((mw[q] & 0x8000u) == 0u && (mw[q] & 0x7FFFu) != 0u) ? 0xFFFFu : 0u;
    const uint32_t hi = ((mw[q] & 0x80000000u) == 0u && (mw[q] & 0x7FFF0000u) != 0u)
                            ? 0xFFFF0000u : 0u;
    vw[q] &= lo | hi;
  }
  return make_uint4(vw[0], vw[1], vw[2], vw[3]);
}

// ------------------------------------------------------------------ pixel GEMM (fwd / dgrad)
struct PConvArgs {
  const bf16* A;
  long long a_ps, a_bs;  // A element (pixel q, image b, channel c) = A[q*a_ps + b*a_bs + c]
  int cin, a_relu;
  const bf16* B;         // tap t, row n (output channel), k = c: B[(t*N + n)*cin + c]
  const int* tab;        // per output-pixel row: [P_out, count, (q << 8 | t) x count], width tab_w
  int tab_w;
  const float* bias;
  int relu;
  bf16* C;
  long long c_ps, c_bs;  // output (P, b, n) = C[P*c_ps + b*c_bs + n]
  const bf16* mask;      // optional, C's layout: output 0 where mask <= 0
  int M, N, ntn;         // images, output channels, N tiles
};

template <int TM, int TN, int WM, int WN>
struct PCfg {
  static constexpr int WR = TM / WM, WC = TN / WN;
  static constexpr int MI = WR / 16, NJ = WC / 16;
  static constexpr int AE = TM * (BK / 8) / kThreads;
  static constexpr int BE = (TN * (BK / 8) + kThreads - 1) / kThreads;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(MI >= 1 && NJ >= 1 && WR % 16 == 0 && WC % 16 == 0, "wave tile");
  static_assert(TM * (BK / 8) % kThreads == 0, "A staging");
};

template <int TM, int TN, int WM, int WN>
__global__ __launch_bounds__(kThreads) void pconv_kernel(PConvArgs a) {
  using S = PCfg<TM, TN, WM, WN>;
  constexpr int MI = S::MI, NJ = S::NJ, AE = S::AE, BE = S::BE;
  constexpr int kAB = 2 * TM * ROWB + 2 * TN * ROWB, OROW = TN * 2 + 16;
  static_assert(kAB >= TM * OROW, "output tile");
  __shared__ __attribute__((aligned(16))) char sab[kAB];
  __shared__ int stab[2 + kMaxPairs];
  char* sa = sab;
  char* sb = sab + 2 * TM * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int z = blockIdx.x / a.ntn, nt = blockIdx.x - z * a.ntn;
  const int m0 = blockIdx.y * TM, n0 = nt * TN;
  if (tid < 2 + kMaxPairs && tid < a.tab_w) stab[tid] = a.tab[(size_t)z * a.tab_w + tid];
  __syncthreads();
  const int Pout = stab[0], cnt = stab[1];
  const int K = cnt * a.cin, nk = (K + BK - 1) / BK;
  // this thread's fixed 16-byte column segment of a staged row: chunk h (32-wide K half)
  const int seg = tid & 7, h = seg >> 2, cs = (seg & 3) * 8;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[AE], rb[BE];
  auto load = [&](int kk) {
    const int k = kk * BK + h * 32;
    const int pair = k / a.cin, c = k - pair * a.cin + cs;
    const bool on = pair < cnt;
    const int ent = on ? stab[2 + pair] : 0;
    const bf16* ap = a.A + (long long)(ent >> 8) * a.a_ps + c;
    const bf16* bp = a.B + ((size_t)(ent & 255) * a.N) * a.cin + c;
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int r = (tid + j * kThreads) >> 3, m = m0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (on && m < a.M) v = *(const uint4*)(ap + (long long)m * a.a_bs);
      ra[j] = a.a_relu ? relu8(v) : v;
    }
#pragma unroll
    for (int j = 0; j < BE; ++j) {
      const int r = (tid + j * kThreads) >> 3, n = n0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (on && r < TN && n < a.N) v = *(const uint4*)(bp + (size_t)n * a.cin);
      rb[j] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int r = (tid + j * kThreads) >> 3;
      *(uint4*)(sa + buf * TM * ROWB + r * ROWB + seg * 16) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < BE; ++j) {
      const int r = (tid + j * kThreads) >> 3;
      if (r < TN) *(uint4*)(sb + buf * TN * ROWB + r * ROWB + seg * 16) = rb[j];
    }
  };
  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int kk = 0; kk < nk; ++kk) {
    const int cur = kk & 1;
    if (kk + 1 < nk) load(kk + 1);
    const char* ta = sa + cur * TM * ROWB;
    const char* tb = sb + cur * TN * ROWB;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      Frag8 fa[MI], fb[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        fa[i].u = *(const uint4*)(ta + (wm * S::WR + i * 16 + li) * ROWB + kh * 64 + g * 16);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        fb[j].u = *(const uint4*)(tb + (wn * S::WC + j * 16 + li) * ROWB + kh * 64 + g * 16);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
    }
    if (kk + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
  // epilogue: bias / relu -> bf16 tile in LDS -> 16-byte row stores (masked)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int trow = wm * S::WR + i * 16 + 4 * g + r;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int tcol = wn * S::WC + j * 16 + li, col = n0 + tcol;
        float v = acc[i][j][r] + ((a.bias && col < a.N) ? a.bias[col] : 0.f);
        if (a.relu) v = fmaxf(v, 0.f);
        *(bf16*)(sab + trow * OROW + tcol * 2) = __float2bfloat16(v);
      }
    }
  __syncthreads();
  constexpr int C8 = TN / 8;
  bf16* cbase = a.C + (long long)Pout * a.c_ps;
  const bf16* mbase = a.mask ? a.mask + (long long)Pout * a.c_ps : nullptr;
  for (int e = tid; e < TM * C8; e += kThreads) {
    const int trow = e / C8, c8 = e - trow * C8, m = m0 + trow, col = n0 + c8 * 8;
    if (m >= a.M || col >= a.N) continue;
    const long long o = (long long)m * a.c_bs + col;
    uint4 v = *(const uint4*)(sab + trow * OROW + c8 * 16);
    if (col + 8 <= a.N) {
      if (mbase) v = mask8(v, *(const uint4*)(mbase + o));
      *(uint4*)(cbase + o) = v;
    } else {
      const bf16* pv = (const bf16*)&v;
      for (int q = 0; q < a.N - col; ++q) {
        bf16 x = pv[q];
        if (mbase && !(__bfloat162float(mbase[o + q]) > 0.f)) x = __float2bfloat16(0.f);
        cbase[o + q] = x;
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
// partial[part][t][o][i] = sum over tap t's pairs (P, q) and this part's images b of
// g[P][b][o] * x[q][b][i]. Output tile OC x IC per workgroup; a stage stages R images of one
// pair (g rows and x rows, row-major) and each wave takes 32-row K blocks, read K-major by
// ds_read_b64_tr_b16; the 4 waves' accumulators are summed through LDS at the end.
struct PWgradArgs {
  const bf16* g;
  long long g_ps, g_bs;
  int O;
  const bf16* x;
  long long x_ps, x_bs;
  int I, x_relu;
  const int* tab;  // per tap: [count, (P << 16 | q) x count], width tab_w
  int tab_w;
  int M, rows_per_part, nic;
  float* partial;  // [part][ntap][O][I]
  int ntap;
};

constexpr int WR_ = 128;  // K rows (images) per stage

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}

template <int OC, int IC>
__global__ __launch_bounds__(kThreads) void pwgrad_kernel(PWgradArgs a) {
  constexpr int MBC = OC / 16, CBC = IC / 16;
  constexpr int GROW = OC * 2 + 16, XROW = IC * 2 + 16;
  constexpr int GE = WR_ * (OC / 8) / kThreads, XE = WR_ * (IC / 8) / kThreads;
  constexpr int kStage = WR_ * GROW + WR_ * XROW;
  constexpr int kRed = OC * IC * 4;
  __shared__ __attribute__((aligned(16))) char smem[kStage > kRed ? kStage : kRed];
  char* gt = smem;
  char* xt = smem + WR_ * GROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int chunk = blockIdx.x, t = blockIdx.y, part = blockIdx.z;
  const int o0 = (chunk / a.nic) * OC, i0 = (chunk % a.nic) * IC;
  const int b0 = part * a.rows_per_part, b1 = min(a.M, b0 + a.rows_per_part);
  const int* trow = a.tab + (size_t)t * a.tab_w;
  const int cnt = trow[0];
  f32x4 acc[MBC][CBC];
#pragma unroll
  for (int mb = 0; mb < MBC; ++mb)
#pragma unroll
    for (int cb = 0; cb < CBC; ++cb) acc[mb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nst = b1 > b0 ? (b1 - b0 + WR_ - 1) / WR_ : 0;
  const int total = cnt * nst;
  uint4 pg[GE], px[XE];
  auto load = [&](int s) {
    const int pr = s / nst, rs = b0 + (s - pr * nst) * WR_;
    const int ent = trow[1 + pr];
    const bf16* gp = a.g + (long long)(ent >> 16) * a.g_ps;
    const bf16* xp = a.x + (long long)(ent & 0xFFFF) * a.x_ps;
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads, row = e / (OC / 8), c = o0 + (e % (OC / 8)) * 8;
      const int b = rs + row;
      pg[k] = (b < b1 && c < a.O) ? *(const uint4*)(gp + (long long)b * a.g_bs + c)
                                  : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = tid + k * kThreads, row = e / (IC / 8), c = i0 + (e % (IC / 8)) * 8;
      const int b = rs + row;
      uint4 v = (b < b1 && c < a.I) ? *(const uint4*)(xp + (long long)b * a.x_bs + c)
                                    : make_uint4(0, 0, 0, 0);
      px[k] = a.x_relu ? relu8(v) : v;
    }
  };
  if (total > 0) load(0);
  for (int s = 0; s < total; ++s) {
    __syncthreads();  // previous stage's reads done
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads;
      *(uint4*)(gt + (e / (OC / 8)) * GROW + (e % (OC / 8)) * 16) = pg[k];
    }
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = tid + k * kThreads;
      *(uint4*)(xt + (e / (IC / 8)) * XROW + (e % (IC / 8)) * 16) = px[k];
    }
    __syncthreads();
    if (s + 1 < total) load(s + 1);
    const int kb = wave;  // 4 waves x 32 rows = the stage's 128 rows
    int prow[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) prow[hh] = kb * 32 + 8 * G + 4 * hh + (li >> 2);
    Frag8 af[MBC];
#pragma unroll
    for (int mb = 0; mb < MBC; ++mb)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        af[mb].h[hh] = tr_read(gt + prow[hh] * GROW + (mb * 16 + 4 * (li & 3)) * 2);
#pragma unroll
    for (int cb = 0; cb < CBC; ++cb) {
      Frag8 bfr;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        bfr.h[hh] = tr_read(xt + prow[hh] * XROW + (cb * 16 + 4 * (li & 3)) * 2);
#pragma unroll
      for (int mb = 0; mb < MBC; ++mb)
        acc[mb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb].v, bfr.v, acc[mb][cb], 0, 0, 0);
    }
  }
  __syncthreads();
  float* red = (float*)smem;
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
  float* out = a.partial + ((size_t)part * a.ntap + t) * a.O * a.I;
  for (int e = tid; e < OC * IC; e += kThreads) {
    const int o = o0 + e / IC, i = i0 + e % IC;
    if (o < a.O && i < a.I) out[(size_t)o * a.I + i] = red[e];
  }
}

// dst[j] = sum_p partial[p * stride + map[j]] (map[j] < 0: 0), fixed order: the weight
// gradient in the parameter's own layout
__global__ __launch_bounds__(kThreads) void reduce_map_kernel(const float* __restrict__ partial,
                                                              int nparts, long long stride,
                                                              const int* __restrict__ map,
                                                              long long n, float* __restrict__ dst) {
  const long long j = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (j >= n) return;
  const int m = map[j];
  float s = 0.f;
  if (m >= 0)
    for (int p = 0; p < nparts; ++p) s += partial[(size_t)p * stride + m];
  dst[j] = s;
}

// ------------------------------------------------------------------ max pool 3x3 / 2 / pad 1
// y [H*W][n][C] (relu'd) -> out [Ho*Wo][n][C], idx (uint8, ky*3+kx of the first maximum in
// scan order). Thread = (pooled pixel, image, 8 channels).
__global__ __launch_bounds__(kThreads) void ppool_fwd_kernel(const bf16* __restrict__ y, int H,
                                                             int W, int n, int C,
                                                             bf16* __restrict__ out,
                                                             uint8_t* __restrict__ idx) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, C8 = C / 8;
  const long long total = (long long)Ho * Wo * n * C8;
  for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (long long)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8);
    const long long pb = e / C8;
    const int b = (int)(pb % n), P = (int)(pb / n);
    const int Y = P / Wo, X = P - Y * Wo;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = 2 * Y - 1 + ky;
      if (yy < 0 || yy >= H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = 2 * X - 1 + kx;
        if (xx < 0 || xx >= W) continue;
        const uint4 v = *(const uint4*)(y + ((long long)(yy * W + xx) * n + b) * C + c8 * 8);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = __uint_as_float((j & 1) ? (w[j >> 1] & 0xFFFF0000u) : (w[j >> 1] << 16));
          if (f > best[j]) { best[j] = f; bi[j] = (uint8_t)(ky * 3 + kx); }
        }
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = (__float_as_uint(best[2 * q]) >> 16) | (__float_as_uint(best[2 * q + 1]) & 0xFFFF0000u);
    const long long off = ((long long)P * n + b) * C + c8 * 8;
    *(uint4*)(out + off) = make_uint4(o[0], o[1], o[2], o[3]);
    uint2 iv;
    iv.x = bi[0] | (uint32_t)bi[1] << 8 | (uint32_t)bi[2] << 16 | (uint32_t)bi[3] << 24;
    iv.y = bi[4] | (uint32_t)bi[5] << 8 | (uint32_t)bi[6] << 16 | (uint32_t)bi[7] << 24;
    *(uint2*)(idx + off) = iv;
  }
}

// Gradient of relu(max_pool(conv)) w.r.t. the conv output, gather form (no atomics):
// dy[q][b][c] = sum over the <= 4 pooled windows P holding q with idx == q's tap and
// pooled > 0 of (g1[P][b][c] (b < n1) + g2[P][b][c] (b < n2)). g1 / g2: pixel strides
// g1_ps / g2_ps, image stride C.
__global__ __launch_bounds__(kThreads) void ppool_bwd_kernel(
    const bf16* __restrict__ g1, long long g1_ps, int n1, const bf16* __restrict__ g2,
    long long g2_ps, int n2, const bf16* __restrict__ pooled, const uint8_t* __restrict__ idx,
    int H, int W, int n, int C, bf16* __restrict__ dy) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, C8 = C / 8;
  const long long total = (long long)H * W * n * C8;
  for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (long long)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8);
    const long long qb = e / C8;
    const int b = (int)(qb % n), q = (int)(qb / n);
    const int yq = q / W, xq = q - yq * W;
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    const int Y0 = yq / 2, X0 = xq / 2;  // windows Y with 2Y-1 <= yq <= 2Y+1
    for (int Y = Y0; Y <= min(Ho - 1, (yq + 1) / 2); ++Y) {
      for (int X = X0; X <= min(Wo - 1, (xq + 1) / 2); ++X) {
        const int tap = (yq - 2 * Y + 1) * 3 + (xq - 2 * X + 1);
        const int P = Y * Wo + X;
        const long long po = ((long long)P * n + b) * C + c8 * 8;
        const uint2 iv = *(const uint2*)(idx + po);
        const uint4 pv = *(const uint4*)(pooled + po);
        uint4 gv1 = make_uint4(0, 0, 0, 0), gv2 = make_uint4(0, 0, 0, 0);
        if (b < n1) gv1 = *(const uint4*)(g1 + (long long)P * g1_ps + (long long)b * C + c8 * 8);
        if (g2 && b < n2) gv2 = *(const uint4*)(g2 + (long long)P * g2_ps + (long long)b * C + c8 * 8);
        const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
        const uint32_t w1[4] = {gv1.x, gv1.y, gv1.z, gv1.w}, w2[4] = {gv2.x, gv2.y, gv2.z, gv2.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t ib = ((j < 4 ? iv.x : iv.y) >> (8 * (j & 3))) & 0xFFu;
          const float pf = __uint_as_float((j & 1) ? (pw[j >> 1] & 0xFFFF0000u) : (pw[j >> 1] << 16));
          if ((int)ib == tap && pf > 0.f) {
            const float a1 = __uint_as_float((j & 1) ? (w1[j >> 1] & 0xFFFF0000u) : (w1[j >> 1] << 16));
            const float a2 = __uint_as_float((j & 1) ? (w2[j >> 1] & 0xFFFF0000u) : (w2[j >> 1] << 16));
            s[j] += a1 + a2;
          }
        }
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const bf16 lo = __float2bfloat16(s[2 * qq]), hi = __float2bfloat16(s[2 * qq + 1]);
      o[qq] = (uint32_t)__bfloat16_as_ushort(lo) | ((uint32_t)__bfloat16_as_ushort(hi) << 16);
    }
    *(uint4*)(dy + ((long long)q * n + b) * C + c8 * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

int grid_for(long long total) {
  long long g = (total + kThreads - 1) / kThreads;
  return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

template <int TM, int TN, int WM, int WN>
void launch_pconv(PConvArgs& a, int nz, hipStream_t st) {
  a.ntn = (a.N + TN - 1) / TN;
  dim3 grid(nz * a.ntn, (a.M + TM - 1) / TM);
  hipLaunchKernelGGL((pconv_kernel<TM, TN, WM, WN>), grid, dim3(kThreads), 0, st, a);
}

}  // namespace

// args (int64): [A, a_ps, a_bs, cin, a_relu, B, tab, tab_w, nz, bias, relu, C, c_ps, c_bs, mask,
//                M, N]
extern "C" int mbk_pconv(const long long* v, hipStream_t st) {
  PConvArgs a{};
  a.A = (const bf16*)v[0]; a.a_ps = v[1]; a.a_bs = v[2]; a.cin = (int)v[3]; a.a_relu = (int)v[4];
  a.B = (const bf16*)v[5]; a.tab = (const int*)v[6]; a.tab_w = (int)v[7];
  const int nz = (int)v[8];
  a.bias = (const float*)v[9]; a.relu = (int)v[10];
  a.C = (bf16*)v[11]; a.c_ps = v[12]; a.c_bs = v[13]; a.mask = (const bf16*)v[14];
  a.M = (int)v[15]; a.N = (int)v[16];
  if (a.M <= 0 || a.N <= 0 || nz <= 0) return 0;
  if (a.cin < 32 || a.cin % 32 || a.tab_w < 2 || a.tab_w > 2 + kMaxPairs || a.a_bs % 8 || a.a_ps % 8 ||
      a.c_bs % 8 || a.c_ps % 8 || ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15) ||
      ((uintptr_t)a.C & 15) || ((uintptr_t)a.mask & 15))
    return (int)hipErrorInvalidValue;
  if (a.N <= 32) launch_pconv<128, 32, 4, 1>(a, nz, st);
  else if (a.N <= 64) launch_pconv<128, 64, 2, 2>(a, nz, st);
  else if (a.N <= 96) launch_pconv<128, 96, 4, 1>(a, nz, st);
  else launch_pconv<128, 128, 2, 2>(a, nz, st);
  return (int)hipGetLastError();
}

extern "C" int mbk_pwgrad_parts(int M, int O, int I, int ntap) {
  const int oc = O <= 32 ? 32 : 64, ic = I <= 32 ? 32 : 64;
  const long long chunks = (long long)((O + oc - 1) / oc) * ((I + ic - 1) / ic) * ntap;
  long long parts = (2048 + chunks - 1) / chunks;
  const long long maxp = (M + WR_ - 1) / WR_;
  if (parts > maxp) parts = maxp;
  if (parts > 256) parts = 256;
  return (int)(parts < 1 ? 1 : parts);
}

// args: [g, g_ps, g_bs, O, x, x_ps, x_bs, I, x_relu, tab, tab_w, ntap, M, nparts, partial]
extern "C" int mbk_pwgrad(const long long* v, hipStream_t st) {
  PWgradArgs a{};
  a.g = (const bf16*)v[0]; a.g_ps = v[1]; a.g_bs = v[2]; a.O = (int)v[3];
  a.x = (const bf16*)v[4]; a.x_ps = v[5]; a.x_bs = v[6]; a.I = (int)v[7]; a.x_relu = (int)v[8];
  a.tab = (const int*)v[9]; a.tab_w = (int)v[10]; a.ntap = (int)v[11]; a.M = (int)v[12];
  const int nparts = (int)v[13];
  a.partial = (float*)v[14];
  if (a.M <= 0 || a.ntap <= 0) return 0;
  if (a.tab_w < 1 || a.O % 8 || a.I % 8 || a.g_bs % 8 || a.x_bs % 8 ||
      a.g_ps % 8 || a.x_ps % 8 || nparts < 1 || ((uintptr_t)a.g & 15) || ((uintptr_t)a.x & 15))
    return (int)hipErrorInvalidValue;
  long long rpp = ((long long)a.M + nparts - 1) / nparts;
  rpp = (rpp + WR_ - 1) / WR_ * WR_;
  a.rows_per_part = (int)rpp;
  const int oc = a.O <= 32 ? 32 : 64, ic = a.I <= 32 ? 32 : 64;
  a.nic = (a.I + ic - 1) / ic;
  dim3 grid(((a.O + oc - 1) / oc) * a.nic, a.ntap, nparts);
  if (oc == 32 && ic == 32) hipLaunchKernelGGL((pwgrad_kernel<32, 32>), grid, dim3(kThreads), 0, st, a);
  else if (oc == 32) hipLaunchKernelGGL((pwgrad_kernel<32, 64>), grid, dim3(kThreads), 0, st, a);
  else if (ic == 32) hipLaunchKernelGGL((pwgrad_kernel<64, 32>), grid, dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL((pwgrad_kernel<64, 64>), grid, dim3(kThreads), 0, st, a);
  return (int)hipGetLastError();
}

extern "C" int mbk_reduce_map(const float* partial, int nparts, long long stride, const int* map,
                              long long n, float* dst, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(reduce_map_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, st, partial, nparts, stride, map, n, dst);
  return (int)hipGetLastError();
}

extern "C" int mbk_ppool_fwd(const void* y, int H, int W, int n, int C, void* out, void* idx,
                             hipStream_t st) {
  if (n <= 0) return 0;
  if (C % 8) return (int)hipErrorInvalidValue;
  const long long total = (long long)((H + 1) / 2) * ((W + 1) / 2) * n * (C / 8);
  hipLaunchKernelGGL(ppool_fwd_kernel, dim3(grid_for(total)), dim3(kThreads), 0, st,
                     (const bf16*)y, H, W, n, C, (bf16*)out, (uint8_t*)idx);
  return (int)hipGetLastError();
}

extern "C" int mbk_ppool_bwd(const void* g1, long long g1_ps, int n1, const void* g2,
                             long long g2_ps, int n2, const void* pooled, const void* idx, int H,
                             int W, int n, int C, void* dy, hipStream_t st) {
  if (n <= 0) return 0;
  if (C % 8 || g1_ps % 8 || g2_ps % 8) return (int)hipErrorInvalidValue;
  const long long total = (long long)H * W * n * (C / 8);
  hipLaunchKernelGGL(ppool_bwd_kernel, dim3(grid_for(total)), dim3(kThreads), 0, st,
                     (const bf16*)g1, g1_ps, n1, (const bf16*)g2, g2_ps, n2,
                     (const bf16*)pooled, (const uint8_t*)idx, H, W, n, C, (bf16*)dy);
  return (int)hipGetLastError();
}
