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

#include <algorithm>

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
// Sparse logits layer (MODE 1, ops/pixconv.py Cells): the active cells of a batch (any legal
// action) are compacted into rows bucketed by map cell P, in (P, image) order (cells_* kernels
// below); the logits forward runs over those rows only: a persistent grid walks the (bucket,
// 128-row) tiles, A rows are gathered by image, C rows are the compact rows. (Its input
// gradient is sparse_dgrad_kernel.)
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
  // MODE 1: bucket b = table row b; tiles [tile_off[b], tile_off[b+1]); rows of bucket b are
  // compact rows bucket_off[b] + r (r < bucket_cnt[b]) of image rowimg[bucket_off[b] + r];
  // totals[1] = number of tiles
  const int *bucket_off, *bucket_cnt, *tile_off, *totals, *rowimg;
  int nbucket;
  // sparse_dgrad_kernel: compact A row of (source cell P, image m) = cellrow[P * M + m]
  const int* cellrow;
};

template <int TM, int TN, int WM, int WN>
struct PCfg {
  static constexpr int NT = WM * WN * 64;   // threads: 8 waves (2 per SIMD per workgroup)
  static constexpr int WR = TM / WM, WC = TN / WN;
  static constexpr int MI = WR / 16, NJ = WC / 16;
  static constexpr int AE = TM * (BK / 8) / NT;
  static constexpr int BE = (TN * (BK / 8) + NT - 1) / NT;
  static_assert(MI >= 1 && NJ >= 1 && WR % 16 == 0 && WC % 16 == 0, "wave tile");
  static_assert(TM * (BK / 8) % NT == 0, "A staging");
};

// One (output pixel / bucket z, 128-row, TN-column) tile. Rows r < mcnt are valid; row r is
// image m0 + r (MODE 0 / 2) or compact row rbase + m0 + r of image rowimg[..] (MODE 1).
template <int TM, int TN, int WM, int WN, int MODE>
__device__ __forceinline__ void pconv_tile(const PConvArgs& a, char* sab, int* stab, int z,
                                           int m0, int mcnt, int nt, int rbase) {
  using S = PCfg<TM, TN, WM, WN>;
  constexpr int MI = S::MI, NJ = S::NJ, AE = S::AE, BE = S::BE;
  constexpr int OROW = TN * 2 + 16;
  char* sa = sab;
  char* sb = sab + 2 * TM * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int n0 = nt * TN;
  if (tid < 2 + kMaxPairs && tid < a.tab_w) stab[tid] = a.tab[(size_t)z * a.tab_w + tid];
  __syncthreads();
  const int Pout = stab[0], cnt = stab[1];
  const int K = cnt * a.cin, nk = (K + BK - 1) / BK;
  // this thread's fixed 16-byte column segment of a staged row: chunk h (32-wide K half)
  const int seg = tid & 7, h = seg >> 2, cs = (seg & 3) * 8;
  // per staged row: its image (MODE 1: gathered once per tile)
  int img[AE];
#pragma unroll
  for (int j = 0; j < AE; ++j) {
    const int r = (tid + j * S::NT) >> 3;
    img[j] = r < mcnt - m0 ? (MODE == 1 ? a.rowimg[rbase + m0 + r] : m0 + r) : -1;
  }

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
      uint4 v = make_uint4(0, 0, 0, 0);
      if (on && img[j] >= 0) v = *(const uint4*)(ap + (long long)img[j] * a.a_bs);
      ra[j] = a.a_relu ? relu8(v) : v;
    }
#pragma unroll
    for (int j = 0; j < BE; ++j) {
      const int r = (tid + j * S::NT) >> 3, n = n0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (on && r < TN && n < a.N) v = *(const uint4*)(bp + (size_t)n * a.cin);
      rb[j] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int r = (tid + j * S::NT) >> 3;
      *(uint4*)(sa + buf * TM * ROWB + r * ROWB + seg * 16) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < BE; ++j) {
      const int r = (tid + j * S::NT) >> 3;
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
      for (int j = 0; j < NJ; ++j)
        fb[j].u = *(const uint4*)(tb + (wn * S::WC + j * 16 + li) * ROWB + kh * 64 + g * 16);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r0 = wm * S::WR + i * 16;
        fa[i].u = *(const uint4*)(ta + (r0 + li) * ROWB + kh * 64 + g * 16);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
      }
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
  bf16* cbase = a.C + (MODE == 1 ? (long long)rbase * a.c_bs : (long long)Pout * a.c_ps);
  const bf16* mbase = a.mask ? a.mask + (long long)Pout * a.c_ps : nullptr;
  for (int e = tid; e < TM * C8; e += S::NT) {
    const int trow = e / C8, c8 = e - trow * C8, m = m0 + trow, col = n0 + c8 * 8;
    if (m >= mcnt || col >= a.N) continue;
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

template <int TM, int TN, int WM, int WN, int MODE>
__global__ __launch_bounds__(WM * WN * 64) void pconv_kernel(PConvArgs a) {
  constexpr int kAB = 2 * TM * ROWB + 2 * TN * ROWB, OROW = TN * 2 + 16;
  static_assert(kAB >= TM * OROW, "output tile");
  __shared__ __attribute__((aligned(16))) char sab[kAB];
  __shared__ int stab[2 + kMaxPairs];
  if (MODE != 1) {
    const int z = blockIdx.x / a.ntn, nt = blockIdx.x - z * a.ntn;
    pconv_tile<TM, TN, WM, WN, MODE>(a, sab, stab, z, blockIdx.y * TM, a.M, nt, 0);
    return;
  }
  // persistent walk over the (bucket, row tile, column tile) list; every workgroup ends when
  // the list does (totals is written before the launch, on the same stream)
  const int ntiles = a.totals[1] * a.ntn;
  for (int tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int tile = tt / a.ntn, nt = tt - tile * a.ntn;
    int lo = 0, hi = a.nbucket - 1;  // last bucket with tile_off[b] <= tile
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.tile_off[mid] <= tile) lo = mid; else hi = mid - 1;
    }
    const int m0 = (tile - a.tile_off[lo]) * TM;
    pconv_tile<TM, TN, WM, WN, 1>(a, sab, stab, lo, m0, a.bucket_cnt[lo], nt,
                                  a.bucket_off[lo]);
    __syncthreads();  // LDS reuse by the next tile
  }
}

// ------------------------------------------------------------------ sparse input gradient
// dX[q][m] = sum over the pairs (P, t) of q of dZ[cellrow[P][m]] . B[t]^T, only for the active
// (pair, image) entries: the logits layer's input gradient when only the active cells carry a
// logit gradient. Per (q, 128-image) tile: the pairs' compact row indices are read once
// (coalesced over images), compacted per pair in LDS, and each pair's active entries run as
// 16-row MFMA groups (A = their dZ rows, B = that tap's weights, both straight from global /
// L2: the MFMA work is tiny and a small LDS footprint keeps ~5 workgroups per CU to hide the
// per-tile load chain); pairs are summed in order into an fp32 LDS tile (deterministic),
// which is written back dense (bf16, relu-masked). Persistent grid.
template <int NOUT>
__global__ __launch_bounds__(kThreads) void sparse_dgrad_kernel(PConvArgs a, int ntiles_m, int ntap) {
  constexpr int TMs = 128, NJ = NOUT / 16;
  constexpr int OSTR = NOUT + 1;                  // fp32 output tile row (odd: conflict-free)
  __shared__ float otile[TMs * OSTR];
  __shared__ int ridx[kMaxPairs * TMs];
  __shared__ short lst[kMaxPairs * TMs];
  __shared__ int lcnt[kMaxPairs];
  __shared__ int stab[2 + kMaxPairs];
  const int K = a.cin, KS = K / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  (void)ntap;
  const int total_tiles = a.tab_w > 0 ? ntiles_m * a.ntn : 0;  // ntn = table rows here
  for (int tile = blockIdx.x; tile < total_tiles; tile += gridDim.x) {
    const int z = tile / ntiles_m, m0 = (tile - z * ntiles_m) * TMs;
    __syncthreads();  // previous tile done with the LDS tiles
    if (tid < 2 + kMaxPairs && tid < a.tab_w) stab[tid] = a.tab[(size_t)z * a.tab_w + tid];
    for (int e = tid; e < TMs * OSTR; e += kThreads) otile[e] = 0.f;
    __syncthreads();
    const int q = stab[0], cnt = stab[1];
    // phase 1: compact row of every (pair, image)
    for (int e = tid; e < cnt * TMs; e += kThreads) {
      const int pr = e / TMs, m = e - pr * TMs;
      const int P = stab[2 + pr] >> 8;
      ridx[pr * TMs + m] = m0 + m < a.M ? a.cellrow[(long long)P * a.M + m0 + m] : -1;
    }
    __syncthreads();
    // phase 2: per pair, wave pr % 4 compacts its active images (ascending)
    for (int pr = wave; pr < cnt; pr += 4) {
      int base = 0;
      for (int h = 0; h < TMs / 64; ++h) {
        const bool on = ridx[pr * TMs + h * 64 + lane] >= 0;
        const uint64_t bal = __ballot(on);
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        if (on) lst[pr * TMs + base + __popcll(bal & below)] = (short)(h * 64 + lane);
        base += __popcll(bal);
      }
      if (lane == 0) lcnt[pr] = base;
    }
    __syncthreads();
    // phase 3: pairs in order; 16-entry MFMA groups over the waves
    for (int pr = 0; pr < cnt; ++pr) {
      const int c = lcnt[pr], t = stab[2 + pr] & 255;
      const bf16* wt = a.B + (size_t)t * NOUT * K;   // [NOUT][K], L2-resident
      for (int gi = wave; gi * 16 < c; gi += 4) {
        const int eidx = gi * 16 + li;
        const bool on = eidx < c;
        const int m = on ? lst[pr * TMs + eidx] : 0;
        const int row = on ? ridx[pr * TMs + m] : 0;
        f32x4 acc[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < KS; ++ks) {
          Frag8 fa;
          fa.u = on ? *(const uint4*)(a.A + (long long)row * a.a_bs + ks * 32 + g * 8)
                    : make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            Frag8 fb;
            fb.u = *(const uint4*)(wt + (j * 16 + li) * K + ks * 32 + g * 8);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa.v, fb.v, acc[j], 0, 0, 0);
          }
        }
        // C rows = entries 4g + i, col = li: add into the images' output rows
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ei = gi * 16 + 4 * g + i;
          if (ei < c) {
            const int mi = lst[pr * TMs + ei];
#pragma unroll
            for (int j = 0; j < NJ; ++j) otile[mi * OSTR + j * 16 + li] += acc[j][i];
          }
        }
      }
      __syncthreads();  // pair pr's adds land before pair pr + 1's (fixed order)
    }
    // epilogue: dense bf16 rows, relu-masked
    constexpr int C8 = NOUT / 8;
    bf16* cbase = a.C + (long long)q * a.c_ps;
    const bf16* mbase = a.mask ? a.mask + (long long)q * a.c_ps : nullptr;
    for (int e = tid; e < TMs * C8; e += kThreads) {
      const int r = e / C8, c8 = e - r * C8, m = m0 + r;
      if (m >= a.M) continue;
      uint32_t w[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const float lo = otile[r * OSTR + c8 * 8 + 2 * qq], hi = otile[r * OSTR + c8 * 8 + 2 * qq + 1];
        w[qq] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(lo)) |
                ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hi)) << 16);
      }
      uint4 v = make_uint4(w[0], w[1], w[2], w[3]);
      const long long o = (long long)m * a.c_bs + c8 * 8;
      if (mbase) v = mask8(v, *(const uint4*)(mbase + o));
      *(uint4*)(cbase + o) = v;
    }
  }
}

// ------------------------------------------------------------------ image-tile conv3x3
// conv3x3 / stride 1 / pad 1 on H x H maps with the input of TI = 256 / H^2 whole images held
// in a halo'd LDS tile, so all 9 taps read A from LDS (the per-pixel GEMM above re-reads every
// input row once per tap through L2: 7.6x at 8x8). Rows = TI images x H^2 pixels (one image per
// wave at 8x8), N = NOUT output channels, K = 9 taps x CIN. Input / output are addressed as
// (pixel stride, image stride) like pconv (NHWC or pixel-major), with relu-on-load, bias, relu
// and a relu-mask epilogue, so the same kernel runs GridNet conv2's forward (NHWC in, pixel-
// major out) and its input gradient (pixel-major dY in, flipped / transposed weights, NHWC out
// masked by the first layer's output). Weight fragments come from L1 / L2 (36 KB), so only the
// image tile takes LDS (37 / 58 KB: 2-4 workgroups per CU); the next tile's input is
// prefetched into registers during this tile's MFMAs.
template <int CIN, int NOUT, int H>
struct ImgCfg {
  static constexpr int HP = H + 2, NPIX = H * H, TI = 256 / NPIX;
  static constexpr int PST = CIN * 2 + 16;                 // LDS pixel stride (bytes)
  static constexpr int IN_BYTES = TI * HP * HP * PST;
  static constexpr int OROW = NOUT * 2 + 16;
  static constexpr int OUT_BYTES = 256 * OROW;
  static constexpr int TILE_BYTES = IN_BYTES > OUT_BYTES ? IN_BYTES : OUT_BYTES;
  static constexpr int WROW = CIN * 2 + 16;
  static constexpr int W_BYTES = 9 * NOUT * WROW;
  static constexpr int C8 = CIN / 8;
  static constexpr int LE = TI * NPIX * C8 / kThreads;     // 16-byte input chunks per thread
  static constexpr int NJ = NOUT / 16;
  static_assert(TI * NPIX == 256 && H * H % 16 == 0, "one 64-row slab per wave");
  static_assert(TI * NPIX * C8 % kThreads == 0, "input staging");
};

template <int CIN, int NOUT, int H>
__global__ __launch_bounds__(kThreads) void imgconv_kernel(PConvArgs a, int ntiles) {
  using S = ImgCfg<CIN, NOUT, H>;
  extern __shared__ __attribute__((aligned(16))) char ism[];
  char* tile = ism;                       // input tile, then the output staging tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // zero the whole input tile once: the halo ring is never written again
  for (int e = tid * 16; e < S::IN_BYTES; e += kThreads * 16)
    *(uint4*)(tile + e) = make_uint4(0, 0, 0, 0);
  uint4 ra[S::LE];
  auto load = [&](int t) {
#pragma unroll
    for (int j = 0; j < S::LE; ++j) {
      const int e = tid + j * kThreads, c8 = e % S::C8, rp = e / S::C8;   // rp = (image, pixel)
      const int i = rp / S::NPIX, p = rp - i * S::NPIX, m = t * S::TI + i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m < a.M) v = *(const uint4*)(a.A + (long long)p * a.a_ps + (long long)m * a.a_bs + c8 * 8);
      ra[j] = a.a_relu ? relu8(v) : v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < S::LE; ++j) {
      const int e = tid + j * kThreads, c8 = e % S::C8, rp = e / S::C8;
      const int i = rp / S::NPIX, p = rp - i * S::NPIX, y = p / H, x = p - y * H;
      *(uint4*)(tile + ((i * S::HP + y + 1) * S::HP + x + 1) * S::PST + c8 * 16) = ra[j];
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  __syncthreads();   // weights + zeroed tile
  for (; t < ntiles; t += gridDim.x) {
    store();
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);
    // wave w: rows [64 w, 64 w + 64) = 4 row blocks of 16 (image / pixel from the row index)
    f32x4 acc[4][S::NJ];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int j = 0; j < S::NJ; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pbase[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int r = wave * 64 + mb * 16 + li, i = r / S::NPIX, p = r - i * S::NPIX;
      const int y = p / H, x = p - y * H;
      pbase[mb] = ((i * S::HP + y) * S::HP + x) * S::PST;   // tap (0, 0) of this row
    }
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int ky = tp / 3, kx = tp % 3, toff = (ky * S::HP + kx) * S::PST;
#pragma unroll
      for (int c0 = 0; c0 < CIN; c0 += 32) {
        Frag8 fb[S::NJ];
#pragma unroll
        for (int j = 0; j < S::NJ; ++j)   // weights [9][NOUT][CIN]: 36 KB, L1 / L2 resident
          fb[j].u = *(const uint4*)(a.B + (size_t)(tp * NOUT + j * 16 + li) * CIN + c0 + 8 * g);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          Frag8 fa;
          fa.u = *(const uint4*)(tile + pbase[mb] + toff + (c0 + 8 * g) * 2);
#pragma unroll
          for (int j = 0; j < S::NJ; ++j)
            acc[mb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa.v, fb[j].v, acc[mb][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();   // all waves done reading the input tile: it becomes the output tile
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int trow = wave * 64 + mb * 16 + 4 * g + r;
#pragma unroll
        for (int j = 0; j < S::NJ; ++j) {
          const int col = j * 16 + li;
          float v = acc[mb][j][r] + (a.bias ? a.bias[col] : 0.f);
          if (a.relu) v = fmaxf(v, 0.f);
          *(bf16*)(tile + trow * S::OROW + col * 2) = __float2bfloat16(v);
        }
      }
    __syncthreads();
    constexpr int OC8 = NOUT / 8;
    for (int e = tid; e < 256 * OC8; e += kThreads) {
      const int trow = e / OC8, c8 = e - trow * OC8;
      const int i = trow / S::NPIX, p = trow - i * S::NPIX, m = t * S::TI + i;
      if (m >= a.M) continue;
      const long long o = (long long)p * a.c_ps + (long long)m * a.c_bs + c8 * 8;
      uint4 v = *(const uint4*)(tile + trow * S::OROW + c8 * 16);
      if (a.mask) v = mask8(v, *(const uint4*)(a.mask + o));
      *(uint4*)(a.C + o) = v;
    }
    __syncthreads();   // output tile read before the next input tile is stored
    // (the halo ring of the input tile was overwritten by the output staging: re-zero it)
    for (int e = tid; e < S::TI * (S::HP * S::HP - S::NPIX) * S::C8; e += kThreads) {
      const int c8 = e % S::C8, hp = e / S::C8, i = hp / (S::HP * S::HP - S::NPIX);
      int q = hp - i * (S::HP * S::HP - S::NPIX);      // q-th halo pixel of image i
      int y, x;
      if (q < S::HP) { y = 0; x = q; }
      else if (q < 2 * S::HP) { y = S::HP - 1; x = q - S::HP; }
      else { q -= 2 * S::HP; y = 1 + (q >> 1); x = (q & 1) ? S::HP - 1 : 0; }
      *(uint4*)(tile + ((i * S::HP + y) * S::HP + x) * S::PST + c8 * 16) = make_uint4(0, 0, 0, 0);
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
  // rows mode (sparse logits layer): pair (P, q) runs over the compact rows of cell bucket P,
  // g row = bucket_off[P] + r (image stride g_bs), x row = image rowimg[bucket_off[P] + r]
  const int *bucket_off, *bucket_cnt, *rowimg;
};

constexpr int WR_ = 128;  // K rows (images) per stage

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}

constexpr int kMaxWgPairs = 256;  // pairs per tap held in LDS

template <int OC, int IC, bool ROWS>
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
  __shared__ int trow[1 + kMaxWgPairs];
  for (int e = tid; e < a.tab_w; e += kThreads) trow[e] = a.tab[(size_t)t * a.tab_w + e];
  __syncthreads();
  const int cnt = trow[0];
  f32x4 acc[MBC][CBC];
#pragma unroll
  for (int mb = 0; mb < MBC; ++mb)
#pragma unroll
    for (int cb = 0; cb < CBC; ++cb) acc[mb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr bool rows = ROWS;
  // stage iterator over (pair, 128-row block) with empty pairs skipped
  auto pair_end = [&](int pr) -> int {
    return rows ? min(b1, a.bucket_cnt[trow[1 + pr] >> 16]) : b1;
  };
  auto advance = [&](int& pr, int& rs) {
    rs += WR_;
    while (pr < cnt && rs >= pair_end(pr)) {
      ++pr;
      rs = b0;
    }
  };
  uint4 pg[GE], px[XE];
  auto load = [&](int pr, int rs) {
    const int ent = trow[1 + pr], P = ent >> 16, q = ent & 0xFFFF;
    const int end = pair_end(pr);
    const int boff = rows ? a.bucket_off[P] : 0;
    const bf16* gp = rows ? a.g + (long long)boff * a.g_bs : a.g + (long long)P * a.g_ps;
    const bf16* xp = a.x + (long long)q * a.x_ps;
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads, row = e / (OC / 8), c = o0 + (e % (OC / 8)) * 8;
      const int b = rs + row;
      pg[k] = (b < end && c < a.O) ? *(const uint4*)(gp + (long long)b * a.g_bs + c)
                                   : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = tid + k * kThreads, row = e / (IC / 8), c = i0 + (e % (IC / 8)) * 8;
      const int b = rs + row;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b < end && c < a.I) {
        const int img = rows ? a.rowimg[boff + b] : b;
        v = *(const uint4*)(xp + (long long)img * a.x_bs + c);
      }
      px[k] = a.x_relu ? relu8(v) : v;
    }
  };
  int pr = 0, rs = b0 - WR_;
  advance(pr, rs);
  if (pr < cnt) load(pr, rs);
  while (pr < cnt) {
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
    int npr = pr, nrs = rs;
    advance(npr, nrs);
    if (npr < cnt) load(npr, nrs);
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
    pr = npr;
    rs = nrs;
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

// All-taps weight gradient over OUTPUT pixels: for each output pixel P (forward pair table)
// and 64-image stage, g[P] is staged once together with x[q] of every pair (q, t) of P, and
// each tap's accumulator takes g^T x[q] -- g is read once per stage instead of once per tap
// (the per-tap form above re-reads it 4-9x: 49 GB for GridNet's 8x8 conv), the x rows of
// neighbouring pixels are re-read from L2. Wave w owns W rows [16 w, 16 w + 16) of the 64-row
// chunk, all 32 input channels of the chunk and all taps (acc[tap][2 col blocks] in
// registers; the tap loop is unrolled over a per-P slot table, so no dynamic register index).
// Loads of the next (P, stage) are issued before this one's MFMAs. The I-chunk-0 workgroups
// also sum g per output channel (one MFMA per K block against an all-ones fragment): the bias
// gradient, stored after the ntap O I weight block of the part.
constexpr int WA_R = 64;          // images per stage (K)
constexpr int WA_OC = 64, WA_IC = 32;
constexpr int WA_GROW = WA_OC * 2 + 16, WA_XROW = WA_IC * 2 + 16;
constexpr int WA_MAXT = 9;

struct PWgradAllArgs {
  const bf16* g;
  long long g_ps, g_bs;
  int O;
  const bf16* x;
  long long x_ps, x_bs;
  int I, x_relu;
  const int* tab;     // forward table rows [P_out, count, (q << 8 | t) x count]
  int tab_w, nrows;   // table width, number of output pixels
  int M, rows_per_part, nic;
  float* partial;     // [part][ntap O I + O]: weights, then the bias sums
  int ntap;
};

__global__ __launch_bounds__(kThreads) void pwgrad_all_kernel(PWgradAllArgs a) {
  constexpr int GE = WA_R * (WA_OC / 8) / kThreads;   // 2
  constexpr int XE = WA_R * (WA_IC / 8) / kThreads;   // 1 per pair
  __shared__ __attribute__((aligned(16))) char gt[WA_R * WA_GROW];
  __shared__ __attribute__((aligned(16))) char xt[WA_MAXT][WA_R * WA_XROW];
  __shared__ int stab[2 + kMaxPairs];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int chunk = blockIdx.x, part = blockIdx.y;
  const int o0 = (chunk / a.nic) * WA_OC, i0 = (chunk % a.nic) * WA_IC;
  const int b0 = part * a.rows_per_part, b1 = min(a.M, b0 + a.rows_per_part);
  const bool wave_on = o0 + 16 * wave < a.O;
  f32x4 acc[WA_MAXT][2];
#pragma unroll
  for (int t = 0; t < WA_MAXT; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = i0 == 0;
  f32x4 accb = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);   // bf16 1.0 x 8
  const int nst = b1 > b0 ? (b1 - b0 + WA_R - 1) / WA_R : 0;
  const int total = nst * a.nrows;
  uint4 pg[GE], px[WA_MAXT][XE];
  // step s = (stage, P) with P fastest: the next P reuses the same images' x rows (L2)
  auto load = [&](int st_) {
    const int stg = st_ / a.nrows, z = st_ - stg * a.nrows;
    const int* row = a.tab + (size_t)z * a.tab_w;
    const int P = row[0], cnt = row[1];
    const int rs = b0 + stg * WA_R;
    const bf16* gp = a.g + (long long)P * a.g_ps;
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads, r = e / (WA_OC / 8), c = o0 + (e % (WA_OC / 8)) * 8;
      const int b = rs + r;
      pg[k] = (b < b1 && c < a.O) ? *(const uint4*)(gp + (long long)b * a.g_bs + c)
                                  : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < WA_MAXT; ++j) {
      int ent = j < cnt ? row[2 + j] : -1;
      const bf16* xp = a.x + (long long)(ent >> 8) * a.x_ps;
#pragma unroll
      for (int k = 0; k < XE; ++k) {
        const int e = tid + k * kThreads, r = e / (WA_IC / 8), c = i0 + (e % (WA_IC / 8)) * 8;
        const int b = rs + r;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (ent >= 0 && b < b1 && c < a.I) v = *(const uint4*)(xp + (long long)b * a.x_bs + c);
        px[j][k] = a.x_relu ? relu8(v) : v;
      }
    }
  };
  if (total > 0) load(0);
  for (int s = 0; s < total; ++s) {
    __syncthreads();  // previous step's LDS reads done
    {
      const int z = s % a.nrows;
      if (tid < 2 + kMaxPairs && tid < a.tab_w) stab[tid] = a.tab[(size_t)z * a.tab_w + tid];
    }
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads;
      *(uint4*)(gt + (e / (WA_OC / 8)) * WA_GROW + (e % (WA_OC / 8)) * 16) = pg[k];
    }
#pragma unroll
    for (int j = 0; j < WA_MAXT; ++j)
#pragma unroll
      for (int k = 0; k < XE; ++k) {
        const int e = tid + k * kThreads;
        *(uint4*)(xt[j] + (e / (WA_IC / 8)) * WA_XROW + (e % (WA_IC / 8)) * 16) = px[j][k];
      }
    __syncthreads();
    if (s + 1 < total) load(s + 1);
    if (!wave_on) continue;
    const int cnt = min(stab[1], WA_MAXT);
    // tap t's pair index in this P (a tap appears at most once per output pixel)
    uint64_t tmap = 0;  // 4 bits per tap: pair index + 1
    for (int j = 0; j < cnt; ++j) tmap |= (uint64_t)(j + 1) << (4 * (stab[2 + j] & 15));
#pragma unroll
    for (int kb = 0; kb < WA_R / 32; ++kb) {
      int prow[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) prow[hh] = kb * 32 + 8 * G + 4 * hh + (li >> 2);
      Frag8 af;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        af.h[hh] = tr_read(gt + prow[hh] * WA_GROW + (16 * wave + 4 * (li & 3)) * 2);
      if (do_bias) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, ones.v, accb, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < WA_MAXT; ++t) {
        const int j = (int)((tmap >> (4 * t)) & 15u) - 1;
        if (j >= 0) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          Frag8 bfr;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
            bfr.h[hh] = tr_read(xt[j] + prow[hh] * WA_XROW + (cb * 16 + 4 * (li & 3)) * 2);
          acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bfr.v, acc[t][cb], 0, 0, 0);
        }
        }
      }
    }
  }
  if (!wave_on) return;
  float* out = a.partial + (size_t)part * (a.ntap * a.O * a.I + a.O);
  if (do_bias && li == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = o0 + 16 * wave + 4 * G + i;
      if (o < a.O) out[(size_t)a.ntap * a.O * a.I + o] = accb[i];
    }
#pragma unroll
  for (int t = 0; t < WA_MAXT; ++t) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int ci = i0 + cb * 16 + li;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = o0 + 16 * wave + 4 * G + i;
        if (t < a.ntap && o < a.O && ci < a.I) out[((size_t)t * a.O + o) * a.I + ci] = acc[t][cb][i];
      }
    }
  }
}

// Image-tile weight gradient of the 8x8 conv3x3 (GridNet conv2): dW[t][o][i] = sum over
// images b and pixels P of dy[P][b][o] x[b][P + s_t][i]. A workgroup stages TI = 4 images at
// a time -- dy as 256 K-rows (image, pixel) x O and x as a halo'd [4][10][10][I] tile -- and
// every tap reads its shifted x rows straight from the tile (per-lane tr-read addresses), so
// each input element is read from HBM once (the per-pixel forms read x once per tap or per
// output pixel). Wave w owns W rows [16 w, 16 w + 16) and all 9 taps x I columns in registers;
// persistent workgroups write one fp32 partial each (reduce_map sums them). The bias
// gradient sum_{b,P} dy[P][b][o] rides along as one more MFMA per K block against an all-ones
// B fragment (stored after the 9 O I weight block), so dy is not read a second time for it.
template <int I_, int O_, int H>
__global__ __launch_bounds__(kThreads) void imgwgrad_kernel(PWgradArgs a, int ntiles) {
  constexpr int HP = H + 2, NPIX = H * H, TI = 256 / NPIX;
  constexpr int XPST = I_ * 2 + 16, GROW = O_ * 2 + 16;
  constexpr int XBYTES = TI * HP * HP * XPST;
  constexpr int GE = 256 * (O_ / 8) / kThreads, XE = TI * NPIX * (I_ / 8) / kThreads;
  constexpr int CBC = I_ / 16;
  static_assert(O_ == 64 && TI * NPIX == 256, "4 waves x 16 W rows, 256 K rows per tile");
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  char* xt = wsm;
  char* gt = wsm + XBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  for (int e = tid * 16; e < XBYTES; e += kThreads * 16) *(uint4*)(xt + e) = make_uint4(0, 0, 0, 0);
  f32x4 acc[9][CBC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int cb = 0; cb < CBC; ++cb) acc[t][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag8 ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);   // bf16 1.0 x 8
  uint4 pg[GE], px[XE];
  auto load = [&](int tl) {
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads, c8 = e % (O_ / 8), r = e / (O_ / 8);   // r = (img, P)
      const int i = r / NPIX, P = r - i * NPIX, m = tl * TI + i;
      pg[k] = m < a.M ? *(const uint4*)(a.g + (long long)P * a.g_ps + (long long)m * a.g_bs + c8 * 8)
                      : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = tid + k * kThreads, c8 = e % (I_ / 8), r = e / (I_ / 8);
      const int i = r / NPIX, P = r - i * NPIX, m = tl * TI + i;
      uint4 v = m < a.M ? *(const uint4*)(a.x + (long long)P * a.x_ps + (long long)m * a.x_bs + c8 * 8)
                        : make_uint4(0, 0, 0, 0);
      px[k] = a.x_relu ? relu8(v) : v;
    }
  };
  int tl = blockIdx.x;
  if (tl < ntiles) load(tl);
  __syncthreads();   // zeroed halo
  for (; tl < ntiles; tl += gridDim.x) {
#pragma unroll
    for (int k = 0; k < GE; ++k) {
      const int e = tid + k * kThreads, c8 = e % (O_ / 8), r = e / (O_ / 8);
      *(uint4*)(gt + r * GROW + c8 * 16) = pg[k];
    }
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = tid + k * kThreads, c8 = e % (I_ / 8), r = e / (I_ / 8);
      const int i = r / NPIX, P = r - i * NPIX, y = P / H, x = P - y * H;
      *(uint4*)(xt + ((i * HP + y + 1) * HP + x + 1) * XPST + c8 * 16) = px[k];
    }
    __syncthreads();
    if (tl + gridDim.x < ntiles) load(tl + gridDim.x);
#pragma unroll 1
    for (int kb = 0; kb < 256 / 32; ++kb) {
      int prow[2], xrow[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = kb * 32 + 8 * G + 4 * hh + (li >> 2);
        const int i = r / NPIX, P = r - i * NPIX, y = P / H, x = P - y * H;
        prow[hh] = r * GROW;
        xrow[hh] = ((i * HP + y) * HP + x) * XPST;          // tap (0, 0) source pixel
      }
      Frag8 af;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        af.h[hh] = tr_read(gt + prow[hh] + (16 * wave + 4 * (li & 3)) * 2);
      accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, ones.v, accb, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int toff = ((t / 3) * HP + (t % 3)) * XPST;
#pragma unroll
        for (int cb = 0; cb < CBC; ++cb) {
          Frag8 bfr;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
            bfr.h[hh] = tr_read(xt + xrow[hh] + toff + (cb * 16 + 4 * (li & 3)) * 2);
          acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bfr.v, acc[t][cb], 0, 0, 0);
        }
      }
    }
    __syncthreads();   // tiles consumed before the next store
  }
  float* out = a.partial + (size_t)blockIdx.x * (9 * O_ * I_ + O_);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int cb = 0; cb < CBC; ++cb) {
      const int ci = cb * 16 + li;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 16 * wave + 4 * G + i;
        out[((size_t)t * O_ + o) * I_ + ci] = acc[t][cb][i];
      }
    }
  if (li == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[9 * O_ * I_ + 16 * wave + 4 * G + i] = accb[i];
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

// The same sum walked in partial order: thread m reads partial[p * stride + m] (consecutive
// lanes, consecutive addresses: coalesced, where reduce_map's gather through a transposing
// weight map touches one cache line per lane) and writes dst[inv[m]] (inv[m] < 0: unused).
// Destinations no partial maps to are zeroed by the caller. Entries m >= nw (the bias sums
// the weight-gradient kernels store after the weights) go to dst2[m - nw] in the same pass.
__global__ __launch_bounds__(kThreads) void reduce_inv_kernel(const float* __restrict__ partial,
                                                              int nparts, long long stride,
                                                              const int* __restrict__ inv,
                                                              long long nm, float* __restrict__ dst,
                                                              float* __restrict__ dst2, long long nw) {
  const long long m = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (m >= nm) return;
  const int j = m < nw ? inv[m] : 0;
  if (j < 0) return;
  const float* src = partial + m;
  float s = 0.f;
#pragma unroll 8
  for (int p = 0; p < nparts; ++p) s += src[(size_t)p * stride];
  if (m < nw) dst[j] = s;
  else dst2[m - nw] = s;
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

// ------------------------------------------------------------------ active-cell compaction
// mask [n][S][3] (78-bit legal-action masks per cell); a cell is active when any bit is set.
// Compact rows are ordered (cell P, image b) and bucketed by P; chunk = 256 images, one thread
// per image walking the S cells (its mask row is contiguous), wave ballots for counts / ranks.
constexpr int kChunk = 256;

__device__ __forceinline__ bool cell_active(const uint32_t* mask, long long cell) {
  const uint32_t* m = mask + cell * 3;
  return (m[0] | m[1] | m[2]) != 0u;
}

// the chunk's active flags [image][S] into LDS from coalesced mask reads (3 words per cell)
__device__ __forceinline__ void stage_flags(const uint32_t* __restrict__ mask, int n, int S,
                                            int chunk, uint8_t* fl) {
  const int b0 = chunk * kChunk, nb = min(kChunk, n - b0);
  const int ncell = nb * S;
  const uint32_t* m = mask + (size_t)b0 * S * 3;
  for (int c = threadIdx.x; c < ncell; c += kChunk)
    fl[c] = (m[(size_t)c * 3] | m[(size_t)c * 3 + 1] | m[(size_t)c * 3 + 2]) != 0u;
  for (int c = ncell + threadIdx.x; c < kChunk * S; c += kChunk) fl[c] = 0;
}

__global__ __launch_bounds__(kChunk) void cells_count_kernel(const uint32_t* __restrict__ mask,
                                                             int n, int S,
                                                             int* __restrict__ counts) {
  extern __shared__ uint8_t fl[];   // [kChunk][S]
  __shared__ int cnt[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int chunk = blockIdx.x, nchunk = gridDim.x;
  for (int P = tid; P < S; P += kChunk) cnt[P] = 0;
  stage_flags(mask, n, S, chunk, fl);
  __syncthreads();
  for (int P = 0; P < S; ++P) {
    const uint64_t bal = __ballot(fl[tid * S + P] != 0);
    if (lane == 0 && bal) atomicAdd(&cnt[P], __popcll(bal));
  }
  __syncthreads();
  for (int P = tid; P < S; P += kChunk) counts[(size_t)P * nchunk + chunk] = cnt[P];
}

// one workgroup: exclusive scan of counts [S][nchunk] (P-major) into offs; per bucket offset
// / count; tile offsets (ceil(count / TM) tiles per bucket, S + 1 entries); totals = {rows,
// tiles}
__global__ __launch_bounds__(1024) void cells_scan_kernel(const int* __restrict__ counts, int S,
                                                          int nchunk, int TM,
                                                          int* __restrict__ offs,
                                                          int* __restrict__ bucket_off,
                                                          int* __restrict__ bucket_cnt,
                                                          int* __restrict__ tile_off,
                                                          int* __restrict__ totals) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const long long L = (long long)S * nchunk;
  const long long seg = (L + 1023) / 1024;
  const long long s0 = tid * seg, s1 = s0 + seg < L ? s0 + seg : L;
  int sum = 0;
  for (long long i = s0; i < s1; ++i) sum += counts[i];
  part[tid] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
    const int v = tid >= d ? part[tid - d] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = part[tid] - sum;
  for (long long i = s0; i < s1; ++i) {
    offs[i] = run;
    run += counts[i];
  }
  __syncthreads();  // offs visible to the workgroup (global writes, same workgroup)
  __threadfence_block();
  const int total = part[1023];
  for (int P = tid; P < S; P += 1024) {
    const int o = offs[(size_t)P * nchunk];
    const int e = P + 1 < S ? offs[(size_t)(P + 1) * nchunk] : total;
    bucket_off[P] = o;
    bucket_cnt[P] = e - o;
  }
  __syncthreads();
  __threadfence_block();
  if (tid == 0) {
    int t = 0;
    for (int P = 0; P < S; ++P) {
      tile_off[P] = t;
      t += (bucket_cnt[P] + TM - 1) / TM;
    }
    tile_off[S] = t;
    totals[0] = total;
    totals[1] = t;
  }
}

// rowimg[r] = image, rowcell[r] = image * S + P of compact row r; cellrow[P * n + b] = compact
// row of cell (b, P) or -1
__global__ __launch_bounds__(kChunk) void cells_scatter_kernel(const uint32_t* __restrict__ mask,
                                                               int n, int S,
                                                               const int* __restrict__ offs,
                                                               int* __restrict__ rowimg,
                                                               int* __restrict__ rowcell,
                                                               int* __restrict__ cellrow) {
  extern __shared__ uint8_t fl[];   // [kChunk][S]
  __shared__ int wcnt[kChunk / 64][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = blockIdx.x, nchunk = gridDim.x;
  const int b = chunk * kChunk + tid;
  stage_flags(mask, n, S, chunk, fl);
  __syncthreads();
  for (int P = 0; P < S; ++P) {
    const uint64_t bal = __ballot(fl[tid * S + P] != 0);
    if (lane == 0) wcnt[wave][P] = __popcll(bal);
  }
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int P = 0; P < S; ++P) {
    const bool on = fl[tid * S + P] != 0;
    const uint64_t bal = __ballot(on);
    int base = offs[(size_t)P * nchunk + chunk];
    for (int w = 0; w < wave; ++w) base += wcnt[w][P];
    if (b < n) {
      int row = -1;
      if (on) {
        row = base + __popcll(bal & below);
        rowimg[row] = b;
        rowcell[row] = b * S + P;
      }
      cellrow[(size_t)P * n + b] = row;
    }
  }
}

// column sums of the first C columns of the compact rows [totals[0]][ld] (bf16): partial
// [gridDim.x][C] (fixed order; reduce_map finishes), block = 4 row lanes x 64 columns
__global__ __launch_bounds__(kThreads) void rows_colsum_kernel(const bf16* __restrict__ Z, int ld,
                                                               int C, const int* __restrict__ totals,
                                                               float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = blockIdx.y * 64 + lane;
  const int nrows = totals[0];
  float s = 0.f;
  if (col < C)
    for (int r = blockIdx.x * 4 + rl; r < nrows; r += gridDim.x * 4)
      s += __bfloat162float(Z[(size_t)r * ld + col]);
  red[rl][lane] = s;
  __syncthreads();
  if (rl == 0 && col < C)
    partial[(size_t)blockIdx.x * C + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// Max-pool forward, one thread per (image, 8 channels) walking its map: each conv pixel is
// read once (three conv rows in registers as packed bf16, the last one reused as the next
// window row's first) instead of once per window covering it. Same scan order and tie rule
// as ppool_fwd_kernel: bit-identical.
template <int W>
__global__ __launch_bounds__(kThreads) void ppool_fwd_img_kernel(const bf16* __restrict__ y,
                                                                 int H, int n, int C,
                                                                 bf16* __restrict__ out,
                                                                 uint8_t* __restrict__ idx) {
  constexpr int Wo = (W + 1) / 2;
  const int Ho = (H + 1) / 2, C8 = C / 8;
  const long long total = (long long)n * C8;
  for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (long long)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8), b = (int)(e / C8);
    uint4 r[3][W];
    auto load = [&](int yy, uint4 (&row)[W]) {
#pragma unroll
      for (int xx = 0; xx < W; ++xx)
        row[xx] = (yy >= 0 && yy < H)
                      ? *(const uint4*)(y + ((long long)(yy * W + xx) * n + b) * C + c8 * 8)
                      : make_uint4(0, 0, 0, 0);
    };
    load(-1, r[0]);
    load(0, r[1]);
    load(1, r[2]);
    for (int Y = 0; Y < Ho; ++Y) {
#pragma unroll
      for (int X = 0; X < Wo; ++X) {
        float best[8];
        uint32_t bi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int yy = 2 * Y - 1 + ky;
          if (yy < 0 || yy >= H) continue;
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int xx = 2 * X - 1 + kx;
            if (xx < 0 || xx >= W) continue;
            const uint4 v = r[ky][xx];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float f = __uint_as_float((j & 1) ? (w[j >> 1] & 0xFFFF0000u) : (w[j >> 1] << 16));
              if (f > best[j]) { best[j] = f; bi[j] = (uint32_t)(ky * 3 + kx); }
            }
          }
        }
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = (__float_as_uint(best[2 * q]) >> 16) | (__float_as_uint(best[2 * q + 1]) & 0xFFFF0000u);
        const long long off = ((long long)(Y * Wo + X) * n + b) * C + c8 * 8;
        *(uint4*)(out + off) = make_uint4(o[0], o[1], o[2], o[3]);
        uint2 iv;
        iv.x = bi[0] | bi[1] << 8 | bi[2] << 16 | bi[3] << 24;
        iv.y = bi[4] | bi[5] << 8 | bi[6] << 16 | bi[7] << 24;
        *(uint2*)(idx + off) = iv;
      }
      if (Y + 1 < Ho) {  // window rows 2Y+1, 2Y+2, 2Y+3
#pragma unroll
        for (int xx = 0; xx < W; ++xx) r[0][xx] = r[2][xx];
        load(2 * Y + 2, r[1]);
        load(2 * Y + 3, r[2]);
      }
    }
  }
}

// Pool backward, one thread per (image, 8 channels) walking its whole map: the pooled
// windows are read once (two pooled rows in registers) instead of once per conv pixel they
// cover (2.25x on average, 4x in the interior), every conv pixel written once. Same summation
// order as ppool_bwd_kernel (windows by row, then column): bit-identical.
template <int W>
__global__ __launch_bounds__(kThreads) void ppool_bwd_img_kernel(
    const bf16* __restrict__ g1, long long g1_ps, int n1, const bf16* __restrict__ g2,
    long long g2_ps, int n2, const bf16* __restrict__ pooled, const uint8_t* __restrict__ idx,
    int H, int n, int C, bf16* __restrict__ dy) {
  constexpr int Wo = (W + 1) / 2;
  const int Ho = (H + 1) / 2, C8 = C / 8;
  const long long total = (long long)n * C8;
  for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < total;
       e += (long long)gridDim.x * kThreads) {
    const int c8 = (int)(e % C8), b = (int)(e / C8);
    float gc[Wo][8], gn[Wo][8];
    uint32_t ic[Wo][2], in_[Wo][2];
    auto load_row = [&](int Y, float (&gs)[Wo][8], uint32_t (&is)[Wo][2]) {
#pragma unroll
      for (int X = 0; X < Wo; ++X) {
        const int P = Y * Wo + X;
        const long long po = ((long long)P * n + b) * C + c8 * 8;
        const uint2 iv = *(const uint2*)(idx + po);
        const uint4 pv = *(const uint4*)(pooled + po);
        uint4 v1 = make_uint4(0, 0, 0, 0), v2 = make_uint4(0, 0, 0, 0);
        if (b < n1) v1 = *(const uint4*)(g1 + (long long)P * g1_ps + (long long)b * C + c8 * 8);
        if (g2 && b < n2) v2 = *(const uint4*)(g2 + (long long)P * g2_ps + (long long)b * C + c8 * 8);
        const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
        const uint32_t w1[4] = {v1.x, v1.y, v1.z, v1.w}, w2[4] = {v2.x, v2.y, v2.z, v2.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float pf = __uint_as_float((j & 1) ? (pw[j >> 1] & 0xFFFF0000u) : (pw[j >> 1] << 16));
          const float a1 = __uint_as_float((j & 1) ? (w1[j >> 1] & 0xFFFF0000u) : (w1[j >> 1] << 16));
          const float a2 = __uint_as_float((j & 1) ? (w2[j >> 1] & 0xFFFF0000u) : (w2[j >> 1] << 16));
          gs[X][j] = pf > 0.f ? a1 + a2 : 0.f;
        }
        is[X][0] = iv.x;
        is[X][1] = iv.y;
      }
    };
    // conv row yq from the windows of pooled rows (ra: ky_a) and optionally (rb: ky_b)
    auto emit = [&](int yq, const float (&ga)[Wo][8], const uint32_t (&ia)[Wo][2], int kya,
                    const float (&gb)[Wo][8], const uint32_t (&ib)[Wo][2], int kyb) {
#pragma unroll
      for (int xq = 0; xq < W; ++xq) {
        float s[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = 0.f;
        auto add = [&](const float (&gs)[Wo][8], const uint32_t (&is)[Wo][2], int ky) {
#pragma unroll
          for (int X = 0; X < Wo; ++X) {
            const int kx = xq - 2 * X + 1;
            if (kx < 0 || kx > 2) continue;
            const uint32_t tap = (uint32_t)(ky * 3 + kx);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t ibyte = (is[X][j >> 2] >> (8 * (j & 3))) & 0xFFu;
              if (ibyte == tap) s[j] += gs[X][j];
            }
          }
        };
        add(ga, ia, kya);
        if (kyb >= 0) add(gb, ib, kyb);
        uint32_t o[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          o[qq] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(s[2 * qq])) |
                  ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(s[2 * qq + 1])) << 16);
        *(uint4*)(dy + ((long long)(yq * W + xq) * n + b) * C + c8 * 8) =
            make_uint4(o[0], o[1], o[2], o[3]);
      }
    };
    load_row(0, gc, ic);
    for (int Y = 0; Y < Ho; ++Y) {
      const bool has_next = Y + 1 < Ho;
      if (has_next) load_row(Y + 1, gn, in_);
      emit(2 * Y, gc, ic, 1, gc, ic, -1);                 // even conv row: centre tap row
      if (2 * Y + 1 < H) emit(2 * Y + 1, gc, ic, 2, gn, in_, has_next ? 0 : -1);
      if (has_next) {
#pragma unroll
        for (int X = 0; X < Wo; ++X) {
#pragma unroll
          for (int j = 0; j < 8; ++j) gc[X][j] = gn[X][j];
          ic[X][0] = in_[X][0];
          ic[X][1] = in_[X][1];
        }
      }
    }
  }
}

int grid_for(long long total) {
  long long g = (total + kThreads - 1) / kThreads;
  return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

template <int TM, int TN, int WM, int WN, int MODE>
void launch_pconv(PConvArgs& a, int nz, int grid_cap, hipStream_t st) {
  a.ntn = (a.N + TN - 1) / TN;
  dim3 grid(nz * a.ntn, (a.M + TM - 1) / TM);
  if (MODE == 1) grid = dim3(grid_cap);
  hipLaunchKernelGGL((pconv_kernel<TM, TN, WM, WN, MODE>), grid, dim3(WM * WN * 64), 0, st, a);
}

}  // namespace

// args (int64): [A, a_ps, a_bs, cin, a_relu, B, tab, tab_w, nz, bias, relu, C, c_ps, c_bs, mask,
//                M, N, mode, bucket_off, bucket_cnt, tile_off, totals, rowimg, nbucket, cellrow,
//                grid_cap]
// mode 0: dense; 1: sparse rows (nz = nbucket = table rows, persistent grid of grid_cap
// workgroups, C = compact rows with image stride c_bs); 2: gathered A through cellrow.
extern "C" int mbk_pconv(const long long* v, hipStream_t st) {
  PConvArgs a{};
  a.A = (const bf16*)v[0]; a.a_ps = v[1]; a.a_bs = v[2]; a.cin = (int)v[3]; a.a_relu = (int)v[4];
  a.B = (const bf16*)v[5]; a.tab = (const int*)v[6]; a.tab_w = (int)v[7];
  const int nz = (int)v[8];
  a.bias = (const float*)v[9]; a.relu = (int)v[10];
  a.C = (bf16*)v[11]; a.c_ps = v[12]; a.c_bs = v[13]; a.mask = (const bf16*)v[14];
  a.M = (int)v[15]; a.N = (int)v[16];
  const int mode = (int)v[17];
  a.bucket_off = (const int*)v[18]; a.bucket_cnt = (const int*)v[19];
  a.tile_off = (const int*)v[20]; a.totals = (const int*)v[21]; a.rowimg = (const int*)v[22];
  a.nbucket = (int)v[23]; a.cellrow = (const int*)v[24];
  const int grid_cap = (int)v[25];
  if (a.M <= 0 || a.N <= 0 || nz <= 0) return 0;
  if (a.cin < 32 || a.cin % 32 || a.tab_w < 2 || a.tab_w > 2 + kMaxPairs || a.a_bs % 8 || a.a_ps % 8 ||
      a.c_bs % 8 || a.c_ps % 8 || ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15) ||
      ((uintptr_t)a.C & 15) || ((uintptr_t)a.mask & 15))
    return (int)hipErrorInvalidValue;
  if (mode == 1) {
    if (!a.bucket_off || !a.bucket_cnt || !a.tile_off || !a.totals || !a.rowimg ||
        a.nbucket != nz || grid_cap < 1 || a.mask || a.N > 128)
      return (int)hipErrorInvalidValue;
    if (a.N <= 96) launch_pconv<128, 96, 4, 2, 1>(a, nz, grid_cap, st);
    else launch_pconv<128, 128, 4, 2, 1>(a, nz, grid_cap, st);
  } else if (mode == 2) {
    // sparse input gradient: every pair's tap < ntap = (largest tap + 1) is read from B
    const int ntap = grid_cap;
    if (!a.cellrow || (a.N != 32 && a.N != 64) || a.a_relu || a.bias || a.relu || a.cin > 128 ||
        ntap < 1 || ntap > 16)
      return (int)hipErrorInvalidValue;
    const int ntm = (a.M + 127) / 128;
    a.ntn = nz;  // table rows
    const long long tiles = (long long)nz * ntm;
    const int grid = (int)std::min<long long>(tiles, 4096);   // ~5 resident per CU (29 KB LDS)
    if (a.N == 32)
      hipLaunchKernelGGL(sparse_dgrad_kernel<32>, dim3(grid), dim3(kThreads), 0, st, a, ntm, ntap);
    else
      hipLaunchKernelGGL(sparse_dgrad_kernel<64>, dim3(grid), dim3(kThreads), 0, st, a, ntm, ntap);
  } else {
    if (a.N <= 32) launch_pconv<128, 32, 4, 1, 0>(a, nz, 0, st);
    else if (a.N <= 64) launch_pconv<128, 64, 4, 2, 0>(a, nz, 0, st);
    else if (a.N <= 96) launch_pconv<128, 96, 4, 2, 0>(a, nz, 0, st);
    else launch_pconv<128, 128, 4, 2, 0>(a, nz, 0, st);
  }
  return (int)hipGetLastError();
}

// image-tile conv3x3 (args as mbk_pconv; B = [9][N][cin] in tap order 0..8, no table):
// supported (cin, N, H) = (32, 64, 8), (64, 32, 8)
extern "C" int mbk_imgconv(const long long* v, int H, hipStream_t st) {
  PConvArgs a{};
  a.A = (const bf16*)v[0]; a.a_ps = v[1]; a.a_bs = v[2]; a.cin = (int)v[3]; a.a_relu = (int)v[4];
  a.B = (const bf16*)v[5];
  a.bias = (const float*)v[9]; a.relu = (int)v[10];
  a.C = (bf16*)v[11]; a.c_ps = v[12]; a.c_bs = v[13]; a.mask = (const bf16*)v[14];
  a.M = (int)v[15]; a.N = (int)v[16];
  if (a.M <= 0) return 0;
  if (a.a_bs % 8 || a.a_ps % 8 || a.c_bs % 8 || a.c_ps % 8 || ((uintptr_t)a.A & 15) ||
      ((uintptr_t)a.B & 15) || ((uintptr_t)a.C & 15) || ((uintptr_t)a.mask & 15))
    return (int)hipErrorInvalidValue;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
#define MBK_IC(CI, NO, HH)                                                                       \
  do {                                                                                           \
    using S = ImgCfg<CI, NO, HH>;                                                                \
    const size_t sm = S::TILE_BYTES;                                                             \
    (void)hipFuncSetAttribute((const void*)imgconv_kernel<CI, NO, HH>,                            \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);              \
    const int ntiles = (a.M + S::TI - 1) / S::TI;                                                \
    const int grid = std::min(ntiles, ncu * std::min(4, (int)(160 * 1024 / sm)));                \
    hipLaunchKernelGGL((imgconv_kernel<CI, NO, HH>), dim3(grid), dim3(kThreads), sm, st, a, ntiles); \
  } while (0)
  if (a.cin == 32 && a.N == 64 && H == 8) MBK_IC(32, 64, 8);
  else if (a.cin == 64 && a.N == 32 && H == 8) MBK_IC(64, 32, 8);
  else return (int)hipErrorInvalidValue;
#undef MBK_IC
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

// args: [g, g_ps, g_bs, O, x, x_ps, x_bs, I, x_relu, tab, tab_w, ntap, M, nparts, partial,
//        bucket_off, bucket_cnt, rowimg] (the last three non-null: rows mode, M = the largest
//        bucket)
extern "C" int mbk_pwgrad(const long long* v, hipStream_t st) {
  PWgradArgs a{};
  a.g = (const bf16*)v[0]; a.g_ps = v[1]; a.g_bs = v[2]; a.O = (int)v[3];
  a.x = (const bf16*)v[4]; a.x_ps = v[5]; a.x_bs = v[6]; a.I = (int)v[7]; a.x_relu = (int)v[8];
  a.tab = (const int*)v[9]; a.tab_w = (int)v[10]; a.ntap = (int)v[11]; a.M = (int)v[12];
  const int nparts = (int)v[13];
  a.partial = (float*)v[14];
  a.bucket_off = (const int*)v[15]; a.bucket_cnt = (const int*)v[16]; a.rowimg = (const int*)v[17];
  if ((a.bucket_off == nullptr) != (a.bucket_cnt == nullptr) ||
      (a.bucket_off == nullptr) != (a.rowimg == nullptr))
    return (int)hipErrorInvalidValue;
  if (a.M <= 0 || a.ntap <= 0) return 0;
  if (a.tab_w < 1 || a.tab_w > 1 + kMaxWgPairs || a.O % 8 || a.I % 8 || a.g_bs % 8 || a.x_bs % 8 ||
      a.g_ps % 8 || a.x_ps % 8 || nparts < 1 || ((uintptr_t)a.g & 15) || ((uintptr_t)a.x & 15))
    return (int)hipErrorInvalidValue;
  long long rpp = ((long long)a.M + nparts - 1) / nparts;
  rpp = (rpp + WR_ - 1) / WR_ * WR_;
  a.rows_per_part = (int)rpp;
  const int oc = a.O <= 32 ? 32 : 64, ic = a.I <= 32 ? 32 : 64;
  a.nic = (a.I + ic - 1) / ic;
  dim3 grid(((a.O + oc - 1) / oc) * a.nic, a.ntap, nparts);
#define MBK_PW(OC_, IC_)                                                                        \
  do {                                                                                          \
    if (a.bucket_off)                                                                           \
      hipLaunchKernelGGL((pwgrad_kernel<OC_, IC_, true>), grid, dim3(kThreads), 0, st, a);      \
    else                                                                                        \
      hipLaunchKernelGGL((pwgrad_kernel<OC_, IC_, false>), grid, dim3(kThreads), 0, st, a);     \
  } while (0)
  if (oc == 32 && ic == 32) MBK_PW(32, 32);
  else if (oc == 32) MBK_PW(32, 64);
  else if (ic == 32) MBK_PW(64, 32);
  else MBK_PW(64, 64);
#undef MBK_PW
  return (int)hipGetLastError();
}

// all-taps weight gradient over output pixels (forward table), ntap <= 9, partial
// [nparts][ntap][O][I]; args: [g, g_ps, g_bs, O, x, x_ps, x_bs, I, x_relu, tab, tab_w, nrows,
// ntap, M, nparts, partial]
extern "C" int mbk_pwgrad_all_parts(int M, int O, int I) {
  const long long chunks = (long long)((O + WA_OC - 1) / WA_OC) * ((I + WA_IC - 1) / WA_IC);
  long long parts = (1024 + chunks - 1) / chunks;
  const long long maxp = (M + WA_R - 1) / WA_R;
  if (parts > maxp) parts = maxp;
  if (parts > 512) parts = 512;
  return (int)(parts < 1 ? 1 : parts);
}

extern "C" int mbk_pwgrad_all(const long long* v, hipStream_t st) {
  PWgradAllArgs a{};
  a.g = (const bf16*)v[0]; a.g_ps = v[1]; a.g_bs = v[2]; a.O = (int)v[3];
  a.x = (const bf16*)v[4]; a.x_ps = v[5]; a.x_bs = v[6]; a.I = (int)v[7]; a.x_relu = (int)v[8];
  a.tab = (const int*)v[9]; a.tab_w = (int)v[10]; a.nrows = (int)v[11]; a.ntap = (int)v[12];
  a.M = (int)v[13];
  const int nparts = (int)v[14];
  a.partial = (float*)v[15];
  if (a.M <= 0 || a.nrows <= 0) return 0;
  if (a.ntap < 1 || a.ntap > WA_MAXT || a.tab_w < 2 || a.tab_w > 2 + kMaxPairs || a.O % 8 ||
      a.I % 8 || a.g_bs % 8 || a.x_bs % 8 || a.g_ps % 8 || a.x_ps % 8 || nparts < 1 ||
      ((uintptr_t)a.g & 15) || ((uintptr_t)a.x & 15))
    return (int)hipErrorInvalidValue;
  long long rpp = ((long long)a.M + nparts - 1) / nparts;
  rpp = (rpp + WA_R - 1) / WA_R * WA_R;
  a.rows_per_part = (int)rpp;
  a.nic = (a.I + WA_IC - 1) / WA_IC;
  dim3 grid(((a.O + WA_OC - 1) / WA_OC) * a.nic, nparts);
  hipLaunchKernelGGL(pwgrad_all_kernel, grid, dim3(kThreads), 0, st, a);
  return (int)hipGetLastError();
}

// active-cell compaction of mask [n][S][3]: scratch counts / offs of S * ceil(n / 256) ints;
// outputs bucket_off / bucket_cnt [S], tile_off [S + 1], totals [2], rowimg / rowcell
// [n * S] (capacity), cellrow [S][n]
extern "C" int mbk_cells_nchunk(int n) { return (n + kChunk - 1) / kChunk; }
extern "C" int mbk_cells_compact(const void* mask, int n, int S, int TM, int* counts, int* offs,
                                 int* bucket_off, int* bucket_cnt, int* tile_off, int* totals,
                                 int* rowimg, int* rowcell, int* cellrow, hipStream_t st) {
  if (n <= 0 || S <= 0) return 0;
  if (S > 256 || TM < 1 || (long long)n * S >= (1ll << 31)) return (int)hipErrorInvalidValue;
  const int nchunk = (n + kChunk - 1) / kChunk;
  const size_t fsm = (size_t)kChunk * S;  // active flags of the chunk (<= 64 KB)
  hipLaunchKernelGGL(cells_count_kernel, dim3(nchunk), dim3(kChunk), fsm, st,
                     (const uint32_t*)mask, n, S, counts);
  hipLaunchKernelGGL(cells_scan_kernel, dim3(1), dim3(1024), 0, st, counts, S, nchunk, TM, offs,
                     bucket_off, bucket_cnt, tile_off, totals);
  hipLaunchKernelGGL(cells_scatter_kernel, dim3(nchunk), dim3(kChunk), fsm, st,
                     (const uint32_t*)mask, n, S, offs, rowimg, rowcell, cellrow);
  return (int)hipGetLastError();
}

extern "C" int mbk_rows_colsum(const void* Z, int ld, int C, const int* totals, int nblk,
                               float* partial, hipStream_t st) {
  if (C <= 0) return 0;
  hipLaunchKernelGGL(rows_colsum_kernel, dim3(nblk, (C + 63) / 64), dim3(kThreads), 0, st,
                     (const bf16*)Z, ld, C, totals, partial);
  return (int)hipGetLastError();
}

// image-tile weight gradient (args as mbk_pwgrad minus the table: g = dY, x = input, both
// (pixel stride, image stride); nparts = grid; partial [nparts][9][O][I]); supported
// (I, O, H) = (32, 64, 8)
extern "C" int mbk_imgwgrad_parts() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return 2 * ncu;
}
extern "C" int mbk_imgwgrad(const long long* v, int H, hipStream_t st) {
  PWgradArgs a{};
  a.g = (const bf16*)v[0]; a.g_ps = v[1]; a.g_bs = v[2]; a.O = (int)v[3];
  a.x = (const bf16*)v[4]; a.x_ps = v[5]; a.x_bs = v[6]; a.I = (int)v[7]; a.x_relu = (int)v[8];
  a.M = (int)v[12];
  const int nparts = (int)v[13];
  a.partial = (float*)v[14];
  if (a.M <= 0) return 0;
  if (a.I != 32 || a.O != 64 || H != 8 || nparts < 1 || a.g_bs % 8 || a.x_bs % 8 ||
      a.g_ps % 8 || a.x_ps % 8 || ((uintptr_t)a.g & 15) || ((uintptr_t)a.x & 15))
    return (int)hipErrorInvalidValue;
  constexpr int TI = 4;
  const int ntiles = (a.M + TI - 1) / TI;
  const size_t sm = (size_t)TI * 10 * 10 * (32 * 2 + 16) + 256 * (64 * 2 + 16);
  (void)hipFuncSetAttribute((const void*)imgwgrad_kernel<32, 64, 8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  hipLaunchKernelGGL((imgwgrad_kernel<32, 64, 8>), dim3(nparts), dim3(kThreads), sm, st, a, ntiles);
  return (int)hipGetLastError();
}

extern "C" int mbk_reduce_map(const float* partial, int nparts, long long stride, const int* map,
                              long long n, float* dst, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(reduce_map_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, st, partial, nparts, stride, map, n, dst);
  return (int)hipGetLastError();
}

extern "C" int mbk_reduce_inv(const float* partial, int nparts, long long stride, const int* inv,
                              long long nm, float* dst, float* dst2, long long nw, hipStream_t st) {
  if (nm <= 0) return 0;
  if (nm > nw && !dst2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(reduce_inv_kernel, dim3((unsigned)((nm + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, st, partial, nparts, stride, inv, nm, dst, dst2, nw);
  return (int)hipGetLastError();
}

extern "C" int mbk_ppool_fwd(const void* y, int H, int W, int n, int C, void* out, void* idx,
                             hipStream_t st) {
  if (n <= 0) return 0;
  if (C % 8) return (int)hipErrorInvalidValue;
  const long long total_img = (long long)n * (C / 8);
#define MBK_PF(WW)                                                                              \
  hipLaunchKernelGGL(ppool_fwd_img_kernel<WW>, dim3(grid_for(total_img)), dim3(kThreads), 0, st, \
                     (const bf16*)y, H, n, C, (bf16*)out, (uint8_t*)idx)
  if (W == 8) { MBK_PF(8); return (int)hipGetLastError(); }
  if (W == 4) { MBK_PF(4); return (int)hipGetLastError(); }
  if (W == 2) { MBK_PF(2); return (int)hipGetLastError(); }
#undef MBK_PF
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
  const long long total_img = (long long)n * (C / 8);
#define MBK_PB(WW)                                                                             \
  hipLaunchKernelGGL(ppool_bwd_img_kernel<WW>, dim3(grid_for(total_img)), dim3(kThreads), 0, st, \
                     (const bf16*)g1, g1_ps, n1, (const bf16*)g2, g2_ps, n2, (const bf16*)pooled, \
                     (const uint8_t*)idx, H, n, C, (bf16*)dy)
  if (W == 8) { MBK_PB(8); return (int)hipGetLastError(); }
  if (W == 4) { MBK_PB(4); return (int)hipGetLastError(); }
  if (W == 2) { MBK_PB(2); return (int)hipGetLastError(); }
#undef MBK_PB
  const long long total = (long long)H * W * n * (C / 8);
  hipLaunchKernelGGL(ppool_bwd_kernel, dim3(grid_for(total)), dim3(kThreads), 0, st,
                     (const bf16*)g1, g1_ps, n1, (const bf16*)g2, g2_ps, n2,
                     (const bf16*)pooled, (const uint8_t*)idx, H, W, n, C, (bf16*)dy);
  return (int)hipGetLastError();
}
