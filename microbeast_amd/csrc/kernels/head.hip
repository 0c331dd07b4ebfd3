// Sparse per-cell action head: active-cell compaction + grouped MFMA GEMM with
// the masked segmented softmax fused into the epilogue.
//
// Reference: actor Linear(256, 78*h*w) + 7*h*w CategoricalMasked objects
// (model.py:136, 167-200) — a dense N x 256 x 19,968 GEMM (65 % of the model's
// FLOPs at 16x16) followed by a masked softmax over every cell.
//
// Observation: a cell whose 78 mask bits are all zero (no own idle unit — the
// vast majority of cells) contributes EXACTLY nothing under the reference's fp32
// semantics: its logits are replaced by -1e8, so log-prob = -1e8 - (-1e8 +
// log n) rounds to 0, the masked entropy is 0 and torch.where passes no
// gradient. So only "active" (frame, cell) pairs need logits at all:
//
//   head_count / head_scan / head_scatter : deterministic, stable counting sort
//       of active pairs by cell (frames ascending inside a cell group), a tile
//       list of 16-pair units, and pidx[f][c] (pair slot or -1). Inactive cells
//       get action 0 / log-prob 0 / entropy 0 written here.
//   head_fwd   : one wave per 16-pair unit: Z[16x80] = X[f rows] . W_c^T + b_c on
//                v_mfma_f32_16x16x32_bf16 (W_c = that cell's 78 rows, padded to 80),
//                then sample (Philox, inverse CDF) or score per row.
//   head_bwd   : one workgroup per cell: recompute Z, dZ in the epilogue, then
//                dX_pair = dZ . W_c (MFMA) and dW_c += dZ^T . X accumulated in
//                registers over all the cell's pairs (both operands via
//                ds_read_b64_tr_b16 from LDS tiles) -> written straight into the
//                actor.weight/bias gradient rows of that cell (deterministic).
//   head_dx_gather : dX[f] = sum of dX_pair over f's active cells (no atomics).
#include "../include/mbk_api.h"
#include "../include/microrts_rules.h"
#include "common.h"

using namespace mbk;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

namespace {

constexpr int KD = 256;      // feature width
constexpr int NP = 80;       // 78 logits padded to 5 x 16
constexpr int NPT = 96;      // 78 padded to 3 x 32 (K of dZ . W)

union Frag8 {
  bf16x8 v;
  uint4 u;
  s16x4 h[2];
};

__device__ __forceinline__ float bf2f(bf16 v) { return __bfloat162float(v); }
__device__ __forceinline__ bf16 f2bf(float v) { return __float2bfloat16(v); }

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(lds_addr));
}

__device__ __forceinline__ bool active3(const uint32_t* m) { return (m[0] | m[1] | m[2]) != 0u; }

// ------------------------------------------------------------------ compaction
// cnt[c * nfb + b] = active pairs of cell c among frames [b*FB, (b+1)*FB)
__global__ __launch_bounds__(256) void head_count_kernel(const uint32_t* __restrict__ mask,
                                                         int F, int S, int FB,
                                                         int* __restrict__ cnt) {
  const int b = blockIdx.x, nfb = gridDim.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= S) return;
  const int f0 = b * FB, f1 = min(F, f0 + FB);
  int n = 0;
#pragma unroll 8
  for (int f = f0; f < f1; ++f) n += active3(mask + ((size_t)f * S + c) * 3);
  cnt[c * nfb + b] = n;
}

// exclusive scan in (c, b) order + per-cell groups + 16-pair unit list
constexpr int CHUNK = 512;  // pairs per backward work item (heavy cells are split)
constexpr int MAX_S = 1024; // cells per map supported by the single-block scan (32x32)

// Per-cell frame-block scan: one workgroup per cell. off[c][b] = active pairs of cell c in
// frame blocks < b (relative to the cell's group start; head_scatter adds grp_start[c]),
// tot[c] = the cell's total. Block-wide scan of 256-element tiles with a carry.
__global__ __launch_bounds__(256) void head_cell_scan_kernel(const int* __restrict__ cnt, int nfb,
                                                             int* __restrict__ off,
                                                             int* __restrict__ tot) {
  __shared__ int ws[4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int carry = 0;
  for (int b0 = 0; b0 < nfb; b0 += 256) {
    const int b = b0 + tid;
    const int x = b < nfb ? cnt[c * nfb + b] : 0;
    int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; ++w) wbase += ws[w];
    const int total = ws[0] + ws[1] + ws[2] + ws[3];
    if (b < nfb) off[c * nfb + b] = carry + wbase + incl - x;
    carry += total;
    __syncthreads();  // ws reused
  }
  if (tid == 0) tot[c] = carry;
}

// Exclusive scans over cells of pairs / 16-pair units / CHUNK-pair chunks -> per-cell
// groups, the unit list and the chunk list. One workgroup (S <= 1024).
__global__ __launch_bounds__(1024) void head_scan_kernel(const int* __restrict__ cell_tot, int S,
                                                         int* __restrict__ grp_start,
                                                         int* __restrict__ grp_count,
                                                         int* __restrict__ unit_cell,
                                                         int* __restrict__ unit_row,
                                                         int* __restrict__ chunk_cell,
                                                         int* __restrict__ chunk_row,
                                                         int* __restrict__ chunk_start,
                                                         int* __restrict__ totals /* [3] */) {
  __shared__ int ust[MAX_S], cst[MAX_S], gst[MAX_S];
  __shared__ int sv[1024], su[1024], sq[1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  int v = 0, u = 0, q = 0;
  if (tid < S) {
    v = cell_tot[tid];
    u = (v + 15) / 16;
    q = (v + CHUNK - 1) / CHUNK;
  }
  sv[tid] = v; su[tid] = u; sq[tid] = q;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int a = tid >= o ? sv[tid - o] : 0, b = tid >= o ? su[tid - o] : 0,
              d = tid >= o ? sq[tid - o] : 0;
    __syncthreads();
    sv[tid] += a; su[tid] += b; sq[tid] += d;
    __syncthreads();
  }
  if (tid < S) {
    const int gs = sv[tid] - v;
    grp_start[tid] = gs;
    grp_count[tid] = v;
    chunk_start[tid] = sq[tid] - q;
    gst[tid] = gs;
    ust[tid] = su[tid] - u;
    cst[tid] = sq[tid] - q;
  }
  if (tid == 1023) {
    totals[0] = sv[1023];
    totals[1] = su[1023];
    totals[2] = sq[1023];
  }
  __syncthreads();
  for (int c = wave; c < S; c += nw) {  // unit / chunk lists, lane-parallel per cell
    const int gs = gst[c], n = sv[c] - gs;
    for (int r = lane * 16; r < n; r += 64 * 16) {
      const int k = ust[c] + r / 16;
      unit_cell[k] = c;
      unit_row[k] = gs + r;
    }
    for (int r = lane * CHUNK; r < n; r += 64 * CHUNK) {
      const int k = cst[c] + r / CHUNK;
      chunk_cell[k] = c;
      chunk_row[k] = gs + r;
    }
  }
}

// pairs[] (frame ids, grouped by cell), pidx[f][c]; zero outputs of inactive cells
__global__ __launch_bounds__(256) void head_scatter_kernel(
    const uint32_t* __restrict__ mask, int F, int S, int FB, const int* __restrict__ off,
    const int* __restrict__ grp_start,
    int* __restrict__ pairs, int* __restrict__ pidx, uint8_t* __restrict__ action_zero,
    float* __restrict__ cell_lp, float* __restrict__ cell_ent) {
  const int b = blockIdx.x, nfb = gridDim.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= S) return;
  const int f0 = b * FB, f1 = min(F, f0 + FB);
  int pos = grp_start[c] + off[c * nfb + b];
  for (int f = f0; f < f1; ++f) {
    const size_t fc = (size_t)f * S + c;
    if (active3(mask + fc * 3)) {
      pairs[pos] = f;
      pidx[fc] = pos;
      ++pos;
    } else {
      pidx[fc] = -1;
      if (action_zero) {
#pragma unroll
        for (int k = 0; k < kComps; ++k) action_zero[fc * kComps + k] = 0;
      }
      if (cell_lp) cell_lp[fc] = 0.f;
      if (cell_ent) cell_ent[fc] = 0.f;
    }
  }
}

// Acting path: per-cell bucket counters (filled by decode_obs_mask's BUCKET variant) ->
// group ranges (cell c's pairs are bucket[c*E, c*E + cnt)) and the 16-pair unit list; the
// counters are reset for the next step. One workgroup, S <= MAX_S.
__global__ __launch_bounds__(1024) void head_units_kernel(int* __restrict__ cnt, int S, int E,
                                                          int* __restrict__ grp_start,
                                                          int* __restrict__ grp_count,
                                                          int* __restrict__ unit_cell,
                                                          int* __restrict__ unit_row,
                                                          int* __restrict__ totals) {
  __shared__ int su[1024];
  const int tid = threadIdx.x;
  int v = 0, u = 0;
  if (tid < S) {
    v = cnt[tid];
    u = (v + 15) / 16;
  }
  su[tid] = u;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int b = tid >= o ? su[tid - o] : 0;
    __syncthreads();
    su[tid] += b;
    __syncthreads();
  }
  if (tid < S) {
    grp_start[tid] = tid * E;
    grp_count[tid] = v;
    cnt[tid] = 0;
    const int u0 = su[tid] - u;
    for (int k = 0; k < u; ++k) {
      unit_cell[u0 + k] = tid;
      unit_row[u0 + k] = tid * E + 16 * k;
    }
  }
  if (tid == 1023) totals[1] = su[1023];
}

// Z[16 pairs][80] of one 16-pair unit of cell c into the wave's LDS tile z: the X rows of the
// unit's frames times W_c^T + b_c on v_mfma_f32_16x16x32_bf16 (C layout: row = pair 4G+i,
// col = logit nb*16 + li). Shared by head_fwd_kernel and the acting step's head_act_kernel.
__device__ __forceinline__ void unit_z(const bf16* __restrict__ X, const bf16* __restrict__ Wp,
                                       const float* __restrict__ bp, int f, bool valid, int c,
                                       float (*z)[NP + 1]) {
  const int lane = threadIdx.x & 63, G = lane >> 4, li = lane & 15;
  f32x4 acc[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint4* xrow = (const uint4*)(X + (size_t)f * KD) + G;  // 8 bf16 per uint4
  const bf16* wc = Wp + (size_t)c * NP * KD;
#pragma unroll
  for (int ks = 0; ks < KD / 32; ++ks) {
    Frag8 a;
    a.u = valid ? xrow[ks * 4] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) {
      Frag8 b;
      b.u = *((const uint4*)(wc + (size_t)(nb * 16 + li) * KD + ks * 32) + G);
      acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc[nb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    const int col = nb * 16 + li;
    const float bias = bp[c * NP + col];
#pragma unroll
    for (int i = 0; i < 4; ++i) z[4 * G + i][col] = acc[nb][i] + bias;
  }
}

// exclusive prefix of ceil(cnt / 16) over the S <= kMaxUnitCells cells into upre (wave 0, 16
// cells per lane; upre[kMaxUnitCells] = the unit total). Caller barriers before reading it.
constexpr int kMaxUnitCells = 1024;
__device__ __forceinline__ void unit_prefix(const int* __restrict__ cnt, int S, int* upre) {
  const int lane = threadIdx.x & 63;
  if ((threadIdx.x >> 6) != 0) return;
  int loc[16], run = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = lane * 16 + k;
    loc[k] = run;
    run += c < S ? (cnt[c] + 15) / 16 : 0;
  }
  int x = run;  // inclusive wave scan of the lane totals
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  const int base = x - run;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = lane * 16 + k;
    if (c <= S) upre[c] = base + loc[k];
  }
  if (lane == 63) upre[kMaxUnitCells] = x;
}

// ------------------------------------------------------------------ forward
// Persistent: each wave takes 16-pair units until none is left.
// cnt != null (acting, decode-bucketed pairs): the unit list is derived in every workgroup from
// the per-cell bucket counts (a 16-pair-unit prefix over the S cells in LDS, then a binary
// search per unit) -- head_units_kernel's unit_cell / unit_row / grp_* / totals without its
// launch; the counters are reset by the step's last launch (row_sum_pack).
__global__ __launch_bounds__(256) void head_fwd_kernel(
    const bf16* __restrict__ X, const bf16* __restrict__ Wp, const float* __restrict__ bp,
    const uint32_t* __restrict__ mask, uint8_t* __restrict__ action, const uint64_t* __restrict__ rng,
    int sample, const int* __restrict__ pairs, const int* __restrict__ unit_cell,
    const int* __restrict__ unit_row, const int* __restrict__ grp_start,
    const int* __restrict__ grp_count, const int* __restrict__ totals, int S,
    float* __restrict__ cell_lp, float* __restrict__ cell_ent, int pair_out,
    const int* __restrict__ cnt, int E) {
  __shared__ float zs[4][16][NP + 1];
  __shared__ int upre[kMaxUnitCells + 1];  // count mode: units before cell c
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, li = lane & 15;
  int nunits;
  if (cnt) {
    unit_prefix(cnt, S, upre);
    __syncthreads();
    nunits = upre[kMaxUnitCells];
  } else {
    nunits = totals[1];
  }
  float (*z)[NP + 1] = zs[wave];
  for (int u = blockIdx.x * 4 + wave; u < nunits; u += gridDim.x * 4) {
    int c, r0, gend;
    if (cnt) {  // last cell whose prefix <= u (cells without units share the next one's)
      int lo = 0, hi = S - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (upre[mid] <= u) lo = mid; else hi = mid - 1;
      }
      c = lo;
      r0 = c * E + 16 * (u - upre[c]);
      gend = c * E + cnt[c];
    } else {
      c = unit_cell[u];
      r0 = unit_row[u];
      gend = grp_start[c] + grp_count[c];
    }
    const int r = r0 + li;
    const bool valid = r < gend;
    const int f = valid ? pairs[r] : pairs[r0];
    unit_z(X, Wp, bp, f, valid, c, z);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes of this wave visible
    __builtin_amdgcn_wave_barrier();
    if (lane < 16 && valid) {
      const size_t fc = (size_t)f * S + c;
      uint32_t m[3] = {mask[fc * 3], mask[fc * 3 + 1], mask[fc * 3 + 2]};
      uint8_t a[kComps];
      float uu[kComps];
      if (sample) {
        const uint64_t seed = rng[0], step = rng[1];
        u32x4 ctr = {(uint32_t)fc, (uint32_t)(fc >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
        u32x4 q0 = philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        ctr.y ^= 0x80000000u;
        u32x4 q1 = philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        uu[0] = u01(q0.x); uu[1] = u01(q0.y); uu[2] = u01(q0.z); uu[3] = u01(q0.w);
        uu[4] = u01(q1.x); uu[5] = u01(q1.y); uu[6] = u01(q1.z);
      } else {
#pragma unroll
        for (int k = 0; k < kComps; ++k) a[k] = action[fc * kComps + k];
      }
      float lp, ent;
      cell_forward(&z[lane][0], m, a, sample != 0, uu, &lp, &ent);
      if (sample) {
#pragma unroll
        for (int k = 0; k < kComps; ++k) action[fc * kComps + k] = a[k];
      }
      // pair_out: results indexed by pair (the learner's scoring: per-frame sums come from
      // head_pair_rowsum over pidx, so inactive cells are never written or read)
      const size_t o = pair_out ? (size_t)r : fc;
      cell_lp[o] = lp;
      if (cell_ent) cell_ent[o] = ent;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ acting step, launch B
// head_fwd_kernel's count-mode sampling (same units, GEMM, Philox stream and cell epilogue) with
// the policy step's finale folded in, so a step is two launches (trunk.hip act_trunk_kernel +
// this one) instead of head + row_sum_pack:
//   * each sampled pair stores {log-prob, packed env action} as ONE 8-byte write-through (sc1)
//     granule in its env's per-cell row, drains it (vmcnt(0)), then decrements its env's
//     pending-cell counter (agent-scope atomic, set by launch A);
//   * the lane whose decrement empties the counter hands the env to its wave, which reads the
//     env's row with sc1 loads only (no fence: MI355X_MICROARCH.md "Valid forms" -- every byte
//     stored sc1 and drained before the signal, every load of it sc1) and writes the env's
//     log-prob (row_sum_pack's lane-strided sum + wave_sum: bit-identical) and its 16-bit
//     action codes (one coalesced 128-byte store per 64 cells, also to pinned host memory);
//   * the bucket counters are double-buffered by step parity (launch A of the next step zeroes
//     this step's half) and the Philox step comes from the host, so no workgroup waits for or
//     counts the others (a 512-way arrival ticket cost ~6 us).
struct HeadActArgs {
  const bf16* X;
  const bf16* Wp;
  const float* bp;
  const uint32_t* mask;
  uint8_t* action;
  uint64_t* rng;
  const int* bucket;
  int* cnt;
  uint64_t* cellx;
  uint16_t* act16;
  uint32_t* act_list;  // sparse action rows (mbk_api.h) instead of act16, or null
  int list_stride;
  float* logp;
  int* pending;
  uint64_t step;  // Philox step (the host's per-lane step count)
  int S, E;
};

__global__ __launch_bounds__(256) void head_act_kernel(HeadActArgs a) {
  __shared__ float zs[4][16][NP + 1];
  __shared__ int upre[kMaxUnitCells + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15;
  const int S = a.S, E = a.E;
  unit_prefix(a.cnt, S, upre);
  __syncthreads();
  const int nunits = upre[kMaxUnitCells];
  const uint64_t seed = a.rng[0], step = a.step;
  // the device copy of the step counter follows the graph path's (nobody reads it in here)
  if (blockIdx.x == 0 && threadIdx.x == 0) a.rng[1] = step + 1;
  float (*z)[NP + 1] = zs[wave];
  for (int u = blockIdx.x * 4 + wave; u < nunits; u += gridDim.x * 4) {
    int lo = 0, hi = S - 1;  // last cell whose prefix <= u
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (upre[mid] <= u) lo = mid; else hi = mid - 1;
    }
    const int c = lo;
    const int r0 = c * E + 16 * (u - upre[c]);
    const int gend = c * E + a.cnt[c];
    const int r = r0 + li;
    const bool valid = r < gend;
    const int ent = valid ? a.bucket[r] : a.bucket[r0];
    const int f = ent & 0xFFFF, rank = ent >> 16;  // env, rank among its active cells
    unit_z(a.X, a.Wp, a.bp, f, valid, c, z);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes of this wave visible
    __builtin_amdgcn_wave_barrier();
    const bool mine = lane < 16 && valid;
    if (mine) {
      const size_t fc = (size_t)f * S + c;
      uint32_t m[3] = {a.mask[fc * 3], a.mask[fc * 3 + 1], a.mask[fc * 3 + 2]};
      uint8_t act[kComps];
      float uu[kComps];
      u32x4 ctr = {(uint32_t)fc, (uint32_t)(fc >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
      u32x4 q0 = philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
      ctr.y ^= 0x80000000u;
      u32x4 q1 = philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
      uu[0] = u01(q0.x); uu[1] = u01(q0.y); uu[2] = u01(q0.z); uu[3] = u01(q0.w);
      uu[4] = u01(q1.x); uu[5] = u01(q1.y); uu[6] = u01(q1.z);
      float lp, ent;
      cell_forward(&z[lane][0], m, act, true, uu, &lp, &ent);
#pragma unroll
      for (int k = 0; k < kComps; ++k) a.action[fc * kComps + k] = act[k];
      const uint64_t x = (uint64_t)__float_as_uint(lp) |
                         ((uint64_t)((uint32_t)c | ((uint32_t)mbr::pack_env_action(act) << 16))
                          << 32);
      __hip_atomic_store(a.cellx + (size_t)f * S + rank, x, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every granule drained before its signal
    bool fin = false;
    if (mine)
      fin = __hip_atomic_fetch_add(a.pending + f, -1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == 1;
    uint64_t bm = __ballot(fin);
    while (bm) {  // envs whose last active cell this wave sampled
      const int l = __builtin_ctzll(bm);
      bm &= bm - 1;
      const int fe = __shfl(f, l, 64);
      // the env's n granules (rank k = k-th active cell in cell order), sc1 loads only
      const uint64_t* row = a.cellx + (size_t)fe * S;
      const int n = a.pending[E + fe];
      float s = 0.f;
      int nz = 0;  // sparse rows: entries written so far
      uint32_t* lrow = a.act_list ? a.act_list + (size_t)fe * a.list_stride : nullptr;
      for (int k0 = 0; k0 < n; k0 += 64) {
        const int k = k0 + lane;
        const uint64_t x = k < n ? __hip_atomic_load(row + k, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const uint32_t hi = (uint32_t)(x >> 32);
        // row_sum_pack's lane-strided sum (lane l adds cells l, l + 64, ... in order) without
        // its +0.0 terms: walk the granules in cell order, each lane keeps its own cells
        const int kn = min(64, n - k0);
        for (int q = 0; q < kn; ++q) {
          const uint32_t lo_q = (uint32_t)__shfl((int)(uint32_t)x, q, 64);
          const uint32_t hi_q = (uint32_t)__shfl((int)hi, q, 64);
          if ((int)(hi_q & 63u) == lane) s += __uint_as_float(lo_q);
        }
        const uint32_t code = hi >> 16;
        if (lrow) {  // only the non-noop cells travel back to the env
          const uint64_t bal = __ballot(k < n && code != 0u);
          const int pos = nz + __popcll(bal & ((1ull << lane) - 1ull));
          if (k < n && code != 0u) lrow[1 + pos] = (hi & 0xFFFFu) | (code << 16);
          nz += __popcll(bal);
        } else if (k < n) {
          a.act16[(size_t)fe * S + (hi & 0xFFFFu)] = (uint16_t)code;
        }
      }
      s = wave_sum(s);
      if (lane == 0) {
        a.logp[fe] = s;
        if (lrow) lrow[0] = (uint32_t)nz;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// logp[f] = sum over f's active cells of the pair log-probs (ent likewise): one wave per
// frame walking pidx[f][:] (4 B per cell instead of reading dense per-cell outputs that
// head_scatter had to zero), fixed-order butterfly reduction (deterministic)
__global__ __launch_bounds__(256) void head_pair_rowsum_kernel(const int* __restrict__ pidx, int F,
                                                               int S, const float* __restrict__ plp,
                                                               const float* __restrict__ pent,
                                                               float* __restrict__ logp,
                                                               float* __restrict__ ent) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= F) return;
  float a = 0.f, b = 0.f;
  const int* pr = pidx + (size_t)f * S;
  auto add = [&](int p) {
    if (p >= 0) {
      a += plp[p];
      if (pent) b += pent[p];
    }
  };
  if ((S & 3) == 0) {  // 16-byte loads: 4 cells per lane per pass
    for (int c = 4 * lane; c < S; c += 256) {
      const int4 q = *(const int4*)(pr + c);
      add(q.x);
      add(q.y);
      add(q.z);
      add(q.w);
    }
  } else {
    for (int c = lane; c < S; c += 64) add(pr[c]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (lane == 0) {
    logp[f] = a;
    if (ent) ent[f] = b;
  }
}

// ------------------------------------------------------------------ backward
// One workgroup (4 waves) per 512-pair chunk of a cell; 64-pair tiles.
// LDS: X tile [64][256] bf16 | dZ tile [64][96] bf16 | z [64][81] f32 (65 KB: two
// workgroups per CU, so one's gather / scalar softmax-backward phase overlaps the other's
// MFMA phases -- at one per CU (W_c staged in LDS too, 105 KB) the kernel was 80 % waits).
// W_c (40 KB) is read through L2 like W_c^T in the dX GEMM.
constexpr int BW_TM = 64;
constexpr int LDS_WC = 0;
constexpr int LDS_XT = BW_TM * KD * 2;
constexpr int LDS_DZ = BW_TM * NPT * 2;
constexpr int LDS_Z = BW_TM * (NP + 1) * 4;

__global__ __launch_bounds__(256, 2) void head_bwd_kernel(
    const bf16* __restrict__ X, const bf16* __restrict__ Wp, const bf16* __restrict__ WpT,
    const float* __restrict__ bp, const uint32_t* __restrict__ mask,
    const uint8_t* __restrict__ action, const int* __restrict__ pairs,
    const int* __restrict__ grp_start, const int* __restrict__ grp_count,
    const int* __restrict__ chunk_cell, const int* __restrict__ chunk_row,
    const int* __restrict__ totals, const float* __restrict__ g_logp,
    const float* __restrict__ g_ent, int S, float* __restrict__ dXp,
    float* __restrict__ dWp /* [nchunks][78][256] */, float* __restrict__ dbp /* [nchunks][78] */) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wc_l = smem;
  char* xt = wc_l + LDS_WC;
  char* dzt = xt + LDS_XT;
  float* zb = (float*)(dzt + LDS_DZ);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int nchunks = totals[2];
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
  const int c = chunk_cell[ch];
  const int g0 = chunk_row[ch];
  const int gn = min(CHUNK, grp_start[c] + grp_count[c] - g0);
  __syncthreads();  // previous chunk's LDS reads done

  const bf16* wcg = Wp + (size_t)c * NP * KD;  // W_c rows [80][256] (L2)
  f32x4 accw[5][4];  // dW_c rows 16mb.., cols 64*wave + 16nb..
#pragma unroll
  for (int mb = 0; mb < 5; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) accw[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbias = 0.f;  // thread tid < 78 owns logit column tid

  for (int t0 = 0; t0 < gn; t0 += BW_TM) {
    const int nr = min(BW_TM, gn - t0);
    __syncthreads();  // previous tile fully consumed
    // stage X rows of this tile (zero rows past the group end)
    for (int e = tid; e < BW_TM * KD / 8; e += 256) {
      const int row = e / (KD / 8), q = e % (KD / 8);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < nr) v = ((const uint4*)(X + (size_t)pairs[g0 + t0 + row] * KD))[q];
      ((uint4*)xt)[e] = v;
    }
    __syncthreads();
    // ---- Z = X . Wc^T + b (wave w: rows 16w..16w+15)
    {
      f32x4 acc[5];
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2  // bounded: every W_c fragment of an unrolled K loop would be in flight
      for (int ks = 0; ks < KD / 32; ++ks) {
        Frag8 a;
        a.u = *(const uint4*)(xt + ((16 * wave + li) * KD + ks * 32 + 8 * G) * 2);
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) {
          Frag8 b;
          b.u = *(const uint4*)(wcg + (nb * 16 + li) * KD + ks * 32 + 8 * G);
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc[nb], 0, 0, 0);
        }
      }
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) {
        const int col = nb * 16 + li;
        const float bias = bp[c * NP + col];
#pragma unroll
        for (int i = 0; i < 4; ++i) zb[(16 * wave + 4 * G + i) * (NP + 1) + col] = acc[nb][i] + bias;
      }
    }
    __syncthreads();
    // ---- dZ per row (threads 0..63 one row each), in place in zb
    if (tid < BW_TM) {
      float* zr = zb + tid * (NP + 1);
      if (tid < nr) {
        const int f = pairs[g0 + t0 + tid];
        const size_t fc = (size_t)f * S + c;
        uint32_t m[3] = {mask[fc * 3], mask[fc * 3 + 1], mask[fc * 3 + 2]};
        uint8_t a[kComps];
#pragma unroll
        for (int k = 0; k < kComps; ++k) a[k] = action[fc * kComps + k];
        cell_backward(zr, m, a, g_logp[f], g_ent ? g_ent[f] : 0.f, zr);
      } else {
        for (int j = 0; j < kCell; ++j) zr[j] = 0.f;
      }
      zr[78] = 0.f;
      zr[79] = 0.f;
    }
    __syncthreads();
    // ---- dZ -> bf16 tile [64][96] (cols >= 78 zero); bias grad column sums
    for (int e = tid; e < BW_TM * NPT; e += 256) {
      const int row = e / NPT, col = e % NPT;
      const float v = col < kCell ? zb[row * (NP + 1) + col] : 0.f;
      ((bf16*)dzt)[e] = f2bf(v);
    }
    if (tid < kCell) {
      float s = 0.f;
      for (int row = 0; row < nr; ++row) s += zb[row * (NP + 1) + tid];
      dbias += s;
    }
    __syncthreads();
    // ---- dX_pair = dZ . Wc (wave w: rows 16w..16w+15, 256 cols; K = 96), in two halves of
    // 128 columns (8 accumulators + 8 fragments in flight instead of 16 + 48)
    {
      const bf16* wt = WpT + (size_t)c * KD * NPT;
#pragma unroll 1
      for (int hc = 0; hc < 2; ++hc) {
        f32x4 acc[8];
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int ks = 0; ks < NPT / 32; ++ks) {
          Frag8 a;
          a.u = *(const uint4*)(dzt + ((16 * wave + li) * NPT + ks * 32 + 8 * G) * 2);
#pragma unroll
          for (int nb = 0; nb < 8; ++nb) {
            Frag8 b;
            b.u = *((const uint4*)(wt + (size_t)((hc * 8 + nb) * 16 + li) * NPT + ks * 32) + G);
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc[nb], 0, 0, 0);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * wave + 4 * G + i;
          if (row < nr) {
            float* dst = dXp + (size_t)(g0 + t0 + row) * KD + hc * 128;
#pragma unroll
            for (int nb = 0; nb < 8; ++nb) dst[nb * 16 + li] = acc[nb][i];
          }
        }
      }
    }
    // ---- dW_c += dZ^T . X  (rows = logits, cols = features 64*wave.., K = 64 pairs)
#pragma unroll
    for (int ks = 0; ks < BW_TM / 32; ++ks) {
      Frag8 a[5];
#pragma unroll
      for (int mb = 0; mb < 5; ++mb)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int prow = ks * 32 + 8 * G + 4 * h + (li >> 2);
          a[mb].h[h] = tr_read(dzt + (prow * NPT + mb * 16 + 4 * (li & 3)) * 2);
        }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        Frag8 b;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int prow = ks * 32 + 8 * G + 4 * h + (li >> 2);
          b.h[h] = tr_read(xt + (prow * KD + 64 * wave + nb * 16 + 4 * (li & 3)) * 2);
        }
#pragma unroll
        for (int mb = 0; mb < 5; ++mb)
          accw[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mb].v, b.v, accw[mb][nb], 0, 0, 0);
      }
    }
  }
  // ---- this chunk's partial dW / db (reduced per cell by head_dw_reduce)
#pragma unroll
  for (int mb = 0; mb < 5; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = mb * 16 + 4 * G + i;
      if (n >= kCell) continue;
      float* dst = dWp + ((size_t)ch * kCell + n) * KD + 64 * wave;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) dst[nb * 16 + li] = accw[mb][nb][i];
    }
  if (tid < kCell) dbp[(size_t)ch * kCell + tid] = dbias;
  }  // chunks
}

// dW[c*78+n][d] = sum over the cell's chunks (fixed order); zero for idle cells
__global__ __launch_bounds__(256) void head_dw_reduce_kernel(const float* __restrict__ dWp,
                                                             const float* __restrict__ dbp,
                                                             const int* __restrict__ chunk_start,
                                                             const int* __restrict__ grp_count,
                                                             int S, float* __restrict__ dW,
                                                             float* __restrict__ db) {
  const int c = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;  // within [78][256] (+78 bias entries)
  const int nch = (grp_count[c] + CHUNK - 1) / CHUNK, c0 = chunk_start[c];
  if (e < kCell * KD) {
    float s = 0.f;
    for (int q = 0; q < nch; ++q) s += dWp[(size_t)(c0 + q) * kCell * KD + e];
    dW[(size_t)c * kCell * KD + e] = s;
  } else if (e < kCell * KD + kCell) {
    const int n = e - kCell * KD;
    float s = 0.f;
    for (int q = 0; q < nch; ++q) s += dbp[(size_t)(c0 + q) * kCell + n];
    db[c * kCell + n] = s;
  }
}

// dX[f][:] = sum over active cells c of dXp[pidx[f][c]][:]; one wave per frame
__global__ __launch_bounds__(256) void head_dx_gather_kernel(const float* __restrict__ dXp,
                                                             const int* __restrict__ pidx, int F,
                                                             int S, float* __restrict__ dX) {
  // one wave per frame: 64 cells' pair indices per coalesced load, ballot the active
  // ones (~1% of cells) and sum only their dXp rows
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= F) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int* pr = pidx + (size_t)f * S;
  for (int c0 = 0; c0 < S; c0 += 64) {
    const int p = c0 + lane < S ? pr[c0 + lane] : -1;
    uint64_t m = __ballot(p >= 0);
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      const int pp = __shfl(p, b);
      const float4 v = ((const float4*)(dXp + (size_t)pp * KD))[lane];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  ((float4*)(dX + (size_t)f * KD))[lane] = acc;
}

// head_dx_gather fused with the critic's backward (gridnet.hip value_bwd, same maths):
//   dh[r][:] = (dv[r] * wc[:] + sum of frame r's active pair rows of dXp) * (h[r][:] > 0)
// written once as bf16, plus per-workgroup partial rows [K + 1] of dWc = sum dv h and
// dbc = sum dv (reduced by the caller's column sum). Frames r >= F (rows the head did not
// score) take only the value term. The fp32 dX [F][256] of the separate kernels (1 KB per
// frame written, then re-read with h by value_bwd) never exists. One wave per frame row,
// a lane owns hidden units 4 lane .. 4 lane + 3 (the gather's float4 layout).
__global__ __launch_bounds__(256) void head_dx_value_kernel(const float* __restrict__ dXp,
                                                            const int* __restrict__ pidx, int F,
                                                            int S, const float* __restrict__ dv,
                                                            const bf16* __restrict__ h,
                                                            const float* __restrict__ wc, int R,
                                                            bf16* __restrict__ dh,
                                                            float* __restrict__ partial) {
  __shared__ float red[4][KD + 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float4 w = ((const float4*)wc)[lane];
  float sw[4] = {0.f, 0.f, 0.f, 0.f}, sb = 0.f;
  // the next frame's dv, h and pair-index row are loaded before this frame's gathers (one
  // wave walks ~R / (4 * grid) frames: without it every frame paid two dependent HBM trips)
  constexpr int kMaxCh = MAX_S / 64;
  const int nch = (S + 63) / 64;
  const int stride = gridDim.x * 4;
  float dn = 0.f;
  uint2 hn = make_uint2(0, 0);
  int pn[kMaxCh];
  auto fetch = [&](int r) {
    dn = dv[r];
    hn = ((const uint2*)(h + (size_t)r * KD))[lane];
    const int* pr = pidx + (size_t)r * S;
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q)
      pn[q] = (r < F && q < nch && q * 64 + lane < S) ? pr[q * 64 + lane] : -1;
  };
  const int rfirst = blockIdx.x * 4 + wave;
  if (rfirst < R) fetch(rfirst);
  for (int r = rfirst; r < R; r += stride) {
    const float d = dn;
    const uint2 hv = hn;
    int pc[kMaxCh];
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q) pc[q] = pn[q];
    if (r + stride < R) fetch(r + stride);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q) {
      if (q >= nch) break;
      const int p = pc[q];
      uint64_t m = __ballot(p >= 0);
      while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        const int pp = __shfl(p, b);
        const float4 v = ((const float4*)(dXp + (size_t)pp * KD))[lane];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    const float hj[4] = {__uint_as_float(hv.x << 16), __uint_as_float(hv.x & 0xFFFF0000u),
                         __uint_as_float(hv.y << 16), __uint_as_float(hv.y & 0xFFFF0000u)};
    const float wj[4] = {w.x, w.y, w.z, w.w}, gj[4] = {acc.x, acc.y, acc.z, acc.w};
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = hj[i] > 0.f ? d * wj[i] + gj[i] : 0.f;
      sw[i] += d * hj[i];
    }
    sb += d;
    const uint32_t o0 = (uint32_t)__bfloat16_as_ushort(f2bf(o[0])) |
                        ((uint32_t)__bfloat16_as_ushort(f2bf(o[1])) << 16);
    const uint32_t o1 = (uint32_t)__bfloat16_as_ushort(f2bf(o[2])) |
                        ((uint32_t)__bfloat16_as_ushort(f2bf(o[3])) << 16);
    ((uint2*)(dh + (size_t)r * KD))[lane] = make_uint2(o0, o1);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][4 * lane + i] = sw[i];
  if (lane == 0) red[wave][KD] = sb;
  __syncthreads();
  for (int e = threadIdx.x; e < KD + 1; e += 256)
    partial[(size_t)blockIdx.x * (KD + 1) + e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
}

// W [S*78][256] fp32, b [S*78] -> Wp [S][80][256] bf16, bp [S][80], WpT [S][256][96] bf16
__global__ __launch_bounds__(256) void head_pack_kernel(const float* __restrict__ W,
                                                        const float* __restrict__ b, int S,
                                                        bf16* __restrict__ Wp,
                                                        float* __restrict__ bp,
                                                        bf16* __restrict__ WpT) {
  const size_t nWp = (size_t)S * NP * KD;
  const size_t nWt = WpT ? (size_t)S * KD * NPT : 0;
  const size_t nb = (size_t)S * NP;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < nWp + nWt + nb;
       e += (size_t)gridDim.x * blockDim.x) {
    if (e < nWp) {
      const size_t c = e / (NP * KD), r = e % (NP * KD), n = r / KD, k = r % KD;
      Wp[e] = f2bf(n < (size_t)kCell ? W[(c * kCell + n) * KD + k] : 0.f);
    } else if (e < nWp + nWt) {
      const size_t q = e - nWp, c = q / (KD * NPT), r = q % (KD * NPT), d = r / NPT, n = r % NPT;
      WpT[q] = f2bf(n < (size_t)kCell ? W[(c * kCell + n) * KD + d] : 0.f);
    } else {
      const size_t q = e - nWp - nWt, c = q / NP, n = q % NP;
      bp[q] = n < (size_t)kCell ? b[c * kCell + n] : 0.f;
    }
  }
}

}  // namespace

// frames per counting block: small batches (policy steps) use short blocks so the
// serial per-thread frame loop stays short; big learner batches cap the scan length.
extern "C" int mbk_head_fb(int F) {
  int fb = F / 64;
  if (fb < 8) fb = 8;
  if (fb > 256) fb = 256;
  return fb;
}

extern "C" int mbk_head_compact(const uint32_t* mask, int F, int S, int* cnt, int* off,
                                int* grp_start, int* grp_count, int* unit_cell, int* unit_row,
                                int* chunk_cell, int* chunk_row, int* chunk_start,
                                int* totals, int* pairs, int* pidx, uint8_t* action_zero,
                                float* cell_lp, float* cell_ent, hipStream_t stream) {
  if (S > MAX_S) return (int)hipErrorInvalidValue;
  const int FB = mbk_head_fb(F);
  const int nfb = (F + FB - 1) / FB;
  dim3 g1(nfb, (S + 255) / 256);
  hipLaunchKernelGGL(head_count_kernel, g1, dim3(256), 0, stream, mask, F, S, FB, cnt);
  // per-cell totals go to grp_count (overwritten with the same values by the scan)
  hipLaunchKernelGGL(head_cell_scan_kernel, dim3(S), dim3(256), 0, stream, cnt, nfb, off,
                     grp_count);
  hipLaunchKernelGGL(head_scan_kernel, dim3(1), dim3(1024), 0, stream, grp_count, S, grp_start,
                     grp_count, unit_cell, unit_row, chunk_cell, chunk_row, chunk_start, totals);
  hipLaunchKernelGGL(head_scatter_kernel, g1, dim3(256), 0, stream, mask, F, S, FB, off,
                     grp_start, pairs, pidx, action_zero, cell_lp, cell_ent);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_units(int* bucket_cnt, int S, int E, int* grp_start, int* grp_count,
                              int* unit_cell, int* unit_row, int* totals, hipStream_t stream) {
  if (S > MAX_S) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(head_units_kernel, dim3(1), dim3(1024), 0, stream, bucket_cnt, S, E,
                     grp_start, grp_count, unit_cell, unit_row, totals);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_fwd(const void* X, const void* Wp, const float* bp, const uint32_t* mask,
                            uint8_t* action, const uint64_t* rng, int sample, const int* pairs,
                            const int* unit_cell, const int* unit_row, const int* grp_start,
                            const int* grp_count, const int* totals, int S, int grid,
                            float* cell_lp, float* cell_ent, int pair_out, hipStream_t stream) {
  hipLaunchKernelGGL(head_fwd_kernel, dim3(grid), dim3(256), 0, stream, (const bf16*)X,
                     (const bf16*)Wp, bp, mask, action, rng, sample, pairs, unit_cell, unit_row,
                     grp_start, grp_count, totals, S, cell_lp, cell_ent, pair_out,
                     (const int*)nullptr, 0);
  return (int)hipGetLastError();
}

// Acting head on decode-bucketed pairs (cell c's pairs at bucket[c * E, + cnt[c])) without
// head_units: every workgroup derives the 16-pair units from cnt (left for the caller to
// reset: mbk_row_sum_pack's cnt argument). S <= 1024.
extern "C" int mbk_head_fwd_counts(const void* X, const void* Wp, const float* bp,
                                   const uint32_t* mask, uint8_t* action, const uint64_t* rng,
                                   const int* bucket, const int* cnt, int E, int S, int grid,
                                   float* cell_lp, hipStream_t stream) {
  if (S < 1 || S > kMaxUnitCells - 1 || !cnt) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(grid), dim3(256), 0, stream, (const bf16*)X,
                     (const bf16*)Wp, bp, mask, action, rng, 1, bucket, (const int*)nullptr,
                     (const int*)nullptr, (const int*)nullptr, (const int*)nullptr,
                     (const int*)nullptr, S, cell_lp, (float*)nullptr, 0, cnt, E);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_pair_rowsum(const int* pidx, int F, int S, const float* plp,
                                    const float* pent, float* logp, float* ent,
                                    hipStream_t stream) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(head_pair_rowsum_kernel, dim3((F + 3) / 4), dim3(256), 0, stream, pidx, F, S,
                     plp, pent, logp, ent);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_bwd(const void* X, const void* Wp, const void* WpT, const float* bp,
                            const uint32_t* mask, const uint8_t* action, const int* pairs,
                            const int* grp_start, const int* grp_count, const int* chunk_cell,
                            const int* chunk_row, const int* chunk_start, const int* totals,
                            const float* g_logp, const float* g_ent, int S, int grid, float* dXp,
                            float* dWp, float* dbp, float* dW, float* db, hipStream_t stream) {
  const size_t sm = LDS_WC + LDS_XT + LDS_DZ + LDS_Z;
  hipFuncSetAttribute((const void*)head_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)sm);
  hipLaunchKernelGGL(head_bwd_kernel, dim3(grid), dim3(256), sm, stream, (const bf16*)X,
                     (const bf16*)Wp, (const bf16*)WpT, bp, mask, action, pairs, grp_start,
                     grp_count, chunk_cell, chunk_row, totals, g_logp, g_ent, S, dXp, dWp, dbp);
  dim3 g2((kCell * KD + kCell + 255) / 256, S);
  hipLaunchKernelGGL(head_dw_reduce_kernel, g2, dim3(256), 0, stream, dWp, dbp, chunk_start,
                     grp_count, S, dW, db);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_dx_gather(const float* dXp, const int* pidx, int F, int S, float* dX,
                                  hipStream_t stream) {
  hipLaunchKernelGGL(head_dx_gather_kernel, dim3((F + 3) / 4), dim3(256), 0, stream, dXp, pidx, F,
                     S, dX);
  return (int)hipGetLastError();
}

// partial rows mbk_head_dx_value writes ([parts][257] fp32)
extern "C" int mbk_head_dx_value_parts(int R) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int need = (R + 3) / 4;
  return need < 1 ? 1 : (need < cus * 4 ? need : cus * 4);
}

// dh [R][256] bf16 = (dv wc + gathered head dX) * (h > 0); partial [parts][257] fp32 rows of
// (dWc, dbc); rows >= F take the value term only. parts = mbk_head_dx_value_parts(R).
extern "C" int mbk_head_dx_value(const float* dXp, const int* pidx, int F, int S, const float* dv,
                                 const void* h, const float* wc, int R, void* dh, float* partial,
                                 int parts, hipStream_t stream) {
  if (R <= 0) return 0;
  if (F > R || parts < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(head_dx_value_kernel, dim3(parts), dim3(256), 0, stream, dXp, pidx, F, S, dv,
                     (const bf16*)h, wc, R, (bf16*)dh, partial);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_pack(const float* W, const float* b, int S, void* Wp, float* bp, void* WpT,
                             hipStream_t stream) {
  size_t tot = (size_t)S * (NP * KD + (WpT ? KD * NPT : 0) + NP);
  size_t blocks = (tot + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(head_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, W, b, S,
                     (bf16*)Wp, bp, (bf16*)WpT);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ fused acting step, launch B
extern "C" int mbk_act_head(const MbkActModel* m, const MbkActStep* s, hipStream_t stream) {
  if (!m || !s || m->E <= 0) return (int)hipErrorInvalidValue;
  const int S = m->H * m->W;
  if (S < 1 || S > kMaxUnitCells - 1 || (S & 3)) return (int)hipErrorInvalidValue;
  if (!m->feat || !m->Wp || !m->bp || !m->rng || !m->bucket || !m->bucket_cnt || !m->cellx ||
      !m->pending || !s->mask || !s->action || (!s->act16 && !s->act_list) ||
      !s->logp)
    return (int)hipErrorInvalidValue;
  if ((uintptr_t)m->cellx & 7) return (int)hipErrorInvalidValue;
  HeadActArgs a{};
  a.X = (const bf16*)m->feat;
  a.Wp = (const bf16*)m->Wp;
  a.bp = m->bp;
  a.mask = s->mask;
  a.action = s->action;
  a.rng = m->rng;
  a.bucket = m->bucket;
  a.cnt = m->bucket_cnt + (s->step & 1) * S;  // this step's half (launch A filled it)
  a.cellx = m->cellx;
  a.act16 = s->act16;
  a.act_list = s->act_list;
  a.list_stride = s->list_stride;
  a.logp = s->logp;
  a.pending = m->pending;
  a.step = s->step;
  a.S = S;
  a.E = m->E;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  hipLaunchKernelGGL(head_act_kernel, dim3(2 * cus), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" int mbk_act_trunk(const MbkActModel* m, const MbkActStep* s, hipStream_t stream);

// the whole acting step: A (decode + trunk + network.5 + critic) then B (sample + finale)
extern "C" int mbk_act_step(const MbkActModel* m, const MbkActStep* s, hipStream_t stream) {
  const int rc = mbk_act_trunk(m, s, stream);
  if (rc) return rc;
  return mbk_act_head(m, s, stream);
}
