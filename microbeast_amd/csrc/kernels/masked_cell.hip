// Masked multi-discrete microRTS action head epilogue as standalone kernels
// (materialised logits). Replaces the reference's Python loop over 7*s*s
// CategoricalMasked objects per forward (model.py:168-200; 1,792 objects at
// 16x16), each doing where(mask, l, -1e8) + logsumexp + sample/log_prob/entropy.
//
// One thread owns one cell (78 logits, 7 segments). The active cells of a 64-cell tile of the
// contiguous cell-major logits are staged through LDS (one row per wave-wide load pair) into
// rows padded to 79 floats (odd stride => conflict-free per-lane reads).
// Used by the GridNet arch (logits from a deconv decoder) and as the parity
// oracle of the fused GEMM+epilogue head (head.hip).
#include "../include/mbk_api.h"
#include "common.h"

using namespace mbk;

namespace {

constexpr int kTile = 64;        // cells per block (one wave)
constexpr int kRow = kCell + 1;  // padded LDS row

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return (float)*p; }
template <>
__device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __bfloat162float(*p);
}

// Only cells with a legal action are staged: a cell whose 78 mask bits are all zero takes no
// logit read in cell_forward / cell_backward (log-prob 0, entropy 0, gradient 0 exactly), and
// on real states ~1-5 % of cells are active, so the tile's logits (156 B per cell in bf16) are
// read for those rows only. am: the tile's active-cell ballot (one wave per tile).
// Logits layout: cell c = (sample, cell-of-map) -> row; element j of the cell at row * ld + j.
// Cell-major (pbc_n == 0): row = c, ld = 78. Pixel-major GridNet logits (pbc_n = images):
// [cell-of-map][image][ld] (ops/pixconv.py), row = (c % cps) * pbc_n + c / cps.
struct Lay {
  int cps, pbc_n, ld;
  __device__ __forceinline__ int64_t row(int64_t c) const {
    return pbc_n ? (c % cps) * pbc_n + c / cps : c;
  }
};

template <typename TZ>
__device__ __forceinline__ void stage_active(const TZ* __restrict__ logits, int64_t c0,
                                             uint64_t am, float* zs, Lay L) {
  const int lane = threadIdx.x;
  while (am) {
    const int r = __builtin_ctzll(am);
    am &= am - 1;
    const TZ* src = logits + L.row(c0 + r) * L.ld;
    zs[r * kRow + lane] = ld(src + lane);
    if (lane < kCell - 64) zs[r * kRow + 64 + lane] = ld(src + 64 + lane);
  }
}

template <typename TZ>
__global__ __launch_bounds__(kTile) void masked_cell_fwd_kernel(
    const TZ* __restrict__ logits, const uint32_t* __restrict__ mask, uint8_t* __restrict__ action,
    const uint64_t* __restrict__ rng, int sample, int64_t ncells, float* __restrict__ cell_logp,
    float* __restrict__ cell_ent, Lay L) {
  __shared__ float zs[kTile * kRow];
  const int64_t c0 = (int64_t)blockIdx.x * kTile;
  const int nc = (int)min((int64_t)kTile, ncells - c0);
  const int i = threadIdx.x;
  const int64_t cell = c0 + i;
  uint32_t m[3] = {0u, 0u, 0u};
  if (i < nc) { m[0] = mask[cell * 3 + 0]; m[1] = mask[cell * 3 + 1]; m[2] = mask[cell * 3 + 2]; }
  stage_active(logits, c0, __ballot((m[0] | m[1] | m[2]) != 0u), zs, L);
  __syncthreads();
  if (i >= nc) return;
  uint8_t a[kComps];
  float u[kComps];
  if (sample) {
    const uint64_t seed = rng[0], step = rng[1];
    u32x4 c = {(uint32_t)cell, (uint32_t)(cell >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
    u32x4 r0 = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    c.y ^= 0x80000000u;
    u32x4 r1 = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    u[0] = u01(r0.x); u[1] = u01(r0.y); u[2] = u01(r0.z); u[3] = u01(r0.w);
    u[4] = u01(r1.x); u[5] = u01(r1.y); u[6] = u01(r1.z);
  } else {
#pragma unroll
    for (int k = 0; k < kComps; ++k) a[k] = action[cell * kComps + k];
  }
  float lp, ent;
  cell_forward(zs + i * kRow, m, a, sample != 0, u, &lp, &ent);
  if (sample) {
#pragma unroll
    for (int k = 0; k < kComps; ++k) action[cell * kComps + k] = a[k];
  }
  cell_logp[cell] = lp;
  if (cell_ent) cell_ent[cell] = ent;
}

template <typename TZ, typename TD>
__global__ __launch_bounds__(kTile) void masked_cell_bwd_kernel(
    const TZ* __restrict__ logits, const uint32_t* __restrict__ mask,
    const uint8_t* __restrict__ action, const float* __restrict__ g_logp,
    const float* __restrict__ g_ent, int cells_per_sample, int64_t ncells,
    TD* __restrict__ dlogits, Lay L) {
  __shared__ float zs[kTile * kRow];
  const int64_t c0 = (int64_t)blockIdx.x * kTile;
  const int nc = (int)min((int64_t)kTile, ncells - c0);
  const int i = threadIdx.x;
  uint32_t m[3] = {0u, 0u, 0u};
  if (i < nc) {
    const int64_t cell = c0 + i;
    m[0] = mask[cell * 3 + 0]; m[1] = mask[cell * 3 + 1]; m[2] = mask[cell * 3 + 2];
  }
  const uint64_t am = __ballot((m[0] | m[1] | m[2]) != 0u);
  stage_active(logits, c0, am, zs, L);
  __syncthreads();
  if (i < nc && ((am >> i) & 1ull)) {
    const int64_t cell = c0 + i;
    const int64_t smp = cell / cells_per_sample;
    uint8_t a[kComps];
#pragma unroll
    for (int k = 0; k < kComps; ++k) a[k] = action[cell * kComps + k];
    // in place: each segment's logits are read before its gradients overwrite them
    float* row = zs + i * kRow;
    cell_backward(row, m, a, g_logp[smp], g_ent ? g_ent[smp] : 0.f, row);
  }
  __syncthreads();
  // every cell's gradients are written (ld columns: 78 + zero padding): inactive rows are
  // exactly zero (not staged)
  if (!L.pbc_n) {
    const int64_t base = c0 * kCell;
    const int total = nc * kCell;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e / kCell, c = e - r * kCell;
      dlogits[base + e] = (TD)(((am >> r) & 1ull) ? zs[r * kRow + c] : 0.f);
    }
  } else if constexpr (sizeof(TD) == 2) {
    // pixel-major rows (ld % 8 == 0): 16-byte stores of 8 bf16, zero rows / padding unread
    const int c8n = L.ld / 8, total = nc * c8n;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e / c8n, c8 = e - r * c8n;
      const bool on = (am >> r) & 1ull;
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c8 * 8 + 2 * q;
        const float lo = (on && c < kCell) ? zs[r * kRow + c] : 0.f;
        const float hi = (on && c + 1 < kCell) ? zs[r * kRow + c + 1] : 0.f;
        w[q] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(lo)) |
               ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hi)) << 16);
      }
      *(uint4*)(dlogits + L.row(c0 + r) * L.ld + c8 * 8) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// Compact-row forms (sparse GridNet logits layer, ops/pixconv.py Cells): logits / gradients
// are rows r < totals[0] of [rows][ld] bf16, row r = cell rowcell[r] (= sample * S + map cell,
// every row active). Per-cell outputs go to the cell's index (the caller zeroes the others).
// 64-row tiles per wave, grid-stride over tiles (the row count is on the device).
__device__ __forceinline__ void stage_rows(const __hip_bfloat16* __restrict__ Z, int ld,
                                           int64_t r0, int nr, float* zs) {
  const int lane = threadIdx.x;
  for (int r = 0; r < nr; ++r) {
    const __hip_bfloat16* src = Z + (r0 + r) * ld;
    zs[r * kRow + lane] = __bfloat162float(src[lane]);
    if (lane < kCell - 64) zs[r * kRow + 64 + lane] = __bfloat162float(src[64 + lane]);
  }
}

__global__ __launch_bounds__(kTile) void masked_cell_rows_fwd_kernel(
    const __hip_bfloat16* __restrict__ Z, int ld, const int* __restrict__ rowcell,
    const int* __restrict__ totals, const uint32_t* __restrict__ mask, uint8_t* __restrict__ action,
    const uint64_t* __restrict__ rng, int sample, float* __restrict__ cell_logp,
    float* __restrict__ cell_ent) {
  __shared__ float zs[kTile * kRow];
  const int64_t nrows = totals[0];
  const int i = threadIdx.x;
  for (int64_t r0 = (int64_t)blockIdx.x * kTile; r0 < nrows; r0 += (int64_t)gridDim.x * kTile) {
    const int nr = (int)min((int64_t)kTile, nrows - r0);
    __syncthreads();  // previous tile's reads done
    stage_rows(Z, ld, r0, nr, zs);
    __syncthreads();
    if (i >= nr) continue;
    const int64_t cell = rowcell[r0 + i];
    const uint32_t m[3] = {mask[cell * 3 + 0], mask[cell * 3 + 1], mask[cell * 3 + 2]};
    uint8_t a[kComps];
    float u[kComps];
    if (sample) {  // same Philox stream as the dense kernel: keyed by the cell index
      const uint64_t seed = rng[0], step = rng[1];
      u32x4 c = {(uint32_t)cell, (uint32_t)(cell >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
      u32x4 q0 = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      c.y ^= 0x80000000u;
      u32x4 q1 = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      u[0] = u01(q0.x); u[1] = u01(q0.y); u[2] = u01(q0.z); u[3] = u01(q0.w);
      u[4] = u01(q1.x); u[5] = u01(q1.y); u[6] = u01(q1.z);
    } else {
#pragma unroll
      for (int k = 0; k < kComps; ++k) a[k] = action[cell * kComps + k];
    }
    float lp, ent;
    cell_forward(zs + i * kRow, m, a, sample != 0, u, &lp, &ent);
    if (sample) {
#pragma unroll
      for (int k = 0; k < kComps; ++k) action[cell * kComps + k] = a[k];
    }
    cell_logp[cell] = lp;
    if (cell_ent) cell_ent[cell] = ent;
  }
}

__global__ __launch_bounds__(kTile) void masked_cell_rows_bwd_kernel(
    const __hip_bfloat16* __restrict__ Z, int ld, const int* __restrict__ rowcell,
    const int* __restrict__ totals, int cps, const uint32_t* __restrict__ mask,
    const uint8_t* __restrict__ action, const float* __restrict__ g_logp,
    const float* __restrict__ g_ent, __hip_bfloat16* __restrict__ dZ) {
  __shared__ float zs[kTile * kRow];
  const int64_t nrows = totals[0];
  const int i = threadIdx.x;
  for (int64_t r0 = (int64_t)blockIdx.x * kTile; r0 < nrows; r0 += (int64_t)gridDim.x * kTile) {
    const int nr = (int)min((int64_t)kTile, nrows - r0);
    __syncthreads();
    stage_rows(Z, ld, r0, nr, zs);
    __syncthreads();
    if (i < nr) {
      const int64_t cell = rowcell[r0 + i];
      const int64_t smp = cell / cps;
      const uint32_t m[3] = {mask[cell * 3 + 0], mask[cell * 3 + 1], mask[cell * 3 + 2]};
      uint8_t a[kComps];
#pragma unroll
      for (int k = 0; k < kComps; ++k) a[k] = action[cell * kComps + k];
      float* row = zs + i * kRow;
      cell_backward(row, m, a, g_logp[smp], g_ent ? g_ent[smp] : 0.f, row);
    }
    __syncthreads();
    // 16-byte stores of 8 bf16 per row chunk, padding columns zero
    const int c8n = ld / 8, total = nr * c8n;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = e / c8n, c8 = e - r * c8n;
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c8 * 8 + 2 * q;
        const float lo = c < kCell ? zs[r * kRow + c] : 0.f;
        const float hi = c + 1 < kCell ? zs[r * kRow + c + 1] : 0.f;
        w[q] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(lo)) |
               ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(hi)) << 16);
      }
      *(uint4*)(dZ + (r0 + r) * ld + c8 * 8) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// Per-sample sums of per-cell values: out[n] = sum_c in[n, c] (one wave per sample).
__global__ __launch_bounds__(256) void row_sum_kernel(const float* __restrict__ in, int64_t rows,
                                                       int cols, float* __restrict__ out,
                                                       uint64_t* __restrict__ rng) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (rng && blockIdx.x == 0 && threadIdx.x == 0) rng[1] += 1;  // fused sampler step advance
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) s += in[r * cols + c];
  s = wave_sum(s);
  if (lane == 0) out[r] = s;
}

__global__ void rng_advance_kernel(uint64_t* rng) { rng[1] += 1; }

}  // namespace

extern "C" int mbk_masked_cell_fwd(const void* logits, int logits_bf16, const uint32_t* mask,
                                   uint8_t* action, const uint64_t* rng, int sample,
                                   int64_t ncells, float* cell_logp, float* cell_ent,
                                   hipStream_t stream) {
  dim3 grid((unsigned)((ncells + kTile - 1) / kTile));
  if (logits_bf16)
    hipLaunchKernelGGL(masked_cell_fwd_kernel<__hip_bfloat16>, grid, dim3(kTile), 0, stream,
                       (const __hip_bfloat16*)logits, mask, action, rng, sample, ncells, cell_logp,
                       cell_ent, Lay{1, 0, kCell});
  else
    hipLaunchKernelGGL(masked_cell_fwd_kernel<float>, grid, dim3(kTile), 0, stream,
                       (const float*)logits, mask, action, rng, sample, ncells, cell_logp, cell_ent,
                       Lay{1, 0, kCell});
  return (int)hipGetLastError();
}

// pixel-major bf16 logits [cps][n][ld] (cell c of sample s at row (c % cps) * n + s)
extern "C" int mbk_masked_cell_fwd_pbc(const void* logits, int cps, int n, int ld,
                                       const uint32_t* mask, uint8_t* action, const uint64_t* rng,
                                       int sample, int64_t ncells, float* cell_logp,
                                       float* cell_ent, hipStream_t stream) {
  if (ncells <= 0) return 0;
  if (ld < kCell || ncells != (int64_t)cps * n) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((ncells + kTile - 1) / kTile));
  hipLaunchKernelGGL(masked_cell_fwd_kernel<__hip_bfloat16>, grid, dim3(kTile), 0, stream,
                     (const __hip_bfloat16*)logits, mask, action, rng, sample, ncells, cell_logp,
                     cell_ent, Lay{cps, n, ld});
  return (int)hipGetLastError();
}

// gradient of the pixel-major logits, written in the same layout (padding columns zero)
extern "C" int mbk_masked_cell_bwd_pbc(const void* logits, int cps, int n, int ld,
                                       const uint32_t* mask, const uint8_t* action,
                                       const float* g_logp, const float* g_ent, int64_t ncells,
                                       void* dlogits, hipStream_t stream) {
  if (ncells <= 0) return 0;
  if (ld < kCell || ld % 8 || ((uintptr_t)dlogits & 15) || ncells != (int64_t)cps * n)
    return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((ncells + kTile - 1) / kTile));
  hipLaunchKernelGGL((masked_cell_bwd_kernel<__hip_bfloat16, __hip_bfloat16>), grid, dim3(kTile),
                     0, stream, (const __hip_bfloat16*)logits, mask, action, g_logp, g_ent, cps,
                     ncells, (__hip_bfloat16*)dlogits, Lay{cps, n, ld});
  return (int)hipGetLastError();
}

extern "C" int mbk_masked_cell_bwd(const void* logits, int logits_bf16, const uint32_t* mask,
                                   const uint8_t* action, const float* g_logp, const float* g_ent,
                                   int cells_per_sample, int64_t ncells, void* dlogits,
                                   int dlogits_bf16, hipStream_t stream) {
  dim3 grid((unsigned)((ncells + kTile - 1) / kTile));
#define MBK_BWD(TZ, TD)                                                                        \
  hipLaunchKernelGGL((masked_cell_bwd_kernel<TZ, TD>), grid, dim3(kTile), 0, stream,           \
                     (const TZ*)logits, mask, action, g_logp, g_ent, cells_per_sample, ncells, \
                     (TD*)dlogits, Lay{1, 0, kCell})
  if (logits_bf16 && dlogits_bf16) MBK_BWD(__hip_bfloat16, __hip_bfloat16);
  else if (logits_bf16) MBK_BWD(__hip_bfloat16, float);
  else if (dlogits_bf16) MBK_BWD(float, __hip_bfloat16);
  else MBK_BWD(float, float);
#undef MBK_BWD
  return (int)hipGetLastError();
}

extern "C" int mbk_row_sum(const float* in, int64_t rows, int cols, float* out,
                           hipStream_t stream) {
  dim3 grid((unsigned)((rows + 3) / 4));
  hipLaunchKernelGGL(row_sum_kernel, grid, dim3(256), 0, stream, in, rows, cols, out,
                     (uint64_t*)nullptr);
  return (int)hipGetLastError();
}

// row sums + advance the sampler's step counter (after the sampling kernel read it)
extern "C" int mbk_row_sum_rng(const float* in, int64_t rows, int cols, float* out, uint64_t* rng,
                               hipStream_t stream) {
  if (rows <= 0) return 0;
  dim3 grid((unsigned)((rows + 3) / 4));
  hipLaunchKernelGGL(row_sum_kernel, grid, dim3(256), 0, stream, in, rows, cols, out, rng);
  return (int)hipGetLastError();
}

extern "C" int mbk_rng_advance(uint64_t* rng, hipStream_t stream) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, stream, rng);
  return (int)hipGetLastError();
}

// compact-row forms: Z / dZ [rows][ld] bf16 (ld % 8 == 0), rows = totals[0] on the device,
// grid of nblk 64-thread workgroups
extern "C" int mbk_masked_cell_rows_fwd(const void* Z, int ld, const int* rowcell,
                                        const int* totals, int nblk, const uint32_t* mask,
                                        uint8_t* action, const uint64_t* rng, int sample,
                                        float* cell_logp, float* cell_ent, hipStream_t stream) {
  if (ld < kCell || ld % 8 || nblk < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(masked_cell_rows_fwd_kernel, dim3(nblk), dim3(kTile), 0, stream,
                     (const __hip_bfloat16*)Z, ld, rowcell, totals, mask, action, rng, sample,
                     cell_logp, cell_ent);
  return (int)hipGetLastError();
}

extern "C" int mbk_masked_cell_rows_bwd(const void* Z, int ld, const int* rowcell,
                                        const int* totals, int nblk, int cps,
                                        const uint32_t* mask, const uint8_t* action,
                                        const float* g_logp, const float* g_ent, void* dZ,
                                        hipStream_t stream) {
  if (ld < kCell || ld % 8 || nblk < 1 || ((uintptr_t)dZ & 15)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(masked_cell_rows_bwd_kernel, dim3(nblk), dim3(kTile), 0, stream,
                     (const __hip_bfloat16*)Z, ld, rowcell, totals, cps, mask, action, g_logp,
                     g_ent, (__hip_bfloat16*)dZ);
  return (int)hipGetLastError();
}
