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
//       list of 16-pair units, and pidx[f][c] (the pair slot, written for active
//       cells only). head_count reads the masks once (F x S x 12 B, the only pass
//       over them) and leaves a per-frame active-cell bitmap abits[f][S/32]: the
//       scatter and every per-frame consumer (row sums, dX gathers) walk that
//       instead of the masks / a dense pidx. Sampling: inactive cells get action 0
//       / log-prob 0 / entropy 0 written here.
//   head_fwd   : one wave per 16-pair unit: Z[16x80] = X[f rows] . W_c^T + b_c on
//                v_mfma_f32_16x16x32_bf16 (W_c = that cell's 78 rows, padded to 80),
//                then sample (Philox, inverse CDF) or score per row.
//   head_bwd2  : one workgroup per CU over 512-pair chunks of a cell, 128-pair tiles: recompute
//                Z, the masked-softmax backward from the MFMA C layout, dX_pair = dZ . W_c
//                (bf16 pair rows) and dW_c += dZ^T . X in registers over the chunk (both
//                operands via ds_read_b64_tr_b16); per-chunk partials reduced in a fixed
//                order per cell by head_dw_reduce (deterministic).
//   head_dx_gather : dX[f] = sum of dX_pair (bf16 rows) over f's active cells (no atomics).
#include <cstdio>
#include <vector>

#include "../include/mbk_api.h"
#include "../include/microrts_rules.h"
#include "common.h"

#ifndef MBK_HA_MB
#define MBK_HA_MB 4
#endif

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
// cnt[c * nfb + b] = active pairs of cell c among frames [b*FB, (b+1)*FB), and the frames'
// active-cell bitmap abits[f][(S + 31) / 32] (bit c & 31 of word c >> 5): a wave ballots its
// 64 cells per frame
__device__ __forceinline__ int abits_words(int S) { return (S + 31) >> 5; }

__global__ __launch_bounds__(256) void head_count_kernel(const uint32_t* __restrict__ mask,
                                                         int F, int S, int FB,
                                                         int* __restrict__ cnt,
                                                         uint32_t* __restrict__ abits) {
  const int b = blockIdx.x, nfb = gridDim.x;
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.y * 256 + threadIdx.x, c0 = c - lane;
  if (c0 >= S) return;  // whole waves only: the ballot needs every lane
  const bool in = c < S;
  const int SW = abits_words(S), w0 = c0 >> 5;
  const bool two = c0 + 32 < S;
  const int f0 = b * FB, f1 = min(F, f0 + FB);
  int n = 0;
#pragma unroll 8
  for (int f = f0; f < f1; ++f) {
    const bool a = in && active3(mask + ((size_t)f * S + c) * 3);
    n += a;
    const uint64_t bal = __ballot(a);
    if (lane == 0) abits[(size_t)f * SW + w0] = (uint32_t)bal;
    if (lane == 1 && two) abits[(size_t)f * SW + w0 + 1] = (uint32_t)(bal >> 32);
  }
  if (in) cnt[c * nfb + b] = n;
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

// head_count from a bitmap the acting step already wrote (the rollout's abits rows): 32 B
// per frame instead of the F x S x 12 B of masks
__global__ __launch_bounds__(256) void head_count_bits_kernel(const uint32_t* __restrict__ abits,
                                                              int F, int S, int FB,
                                                              int* __restrict__ cnt) {
  const int b = blockIdx.x, nfb = gridDim.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= S) return;
  const int SW = abits_words(S), w = c >> 5, bit = c & 31;
  const int f0 = b * FB, f1 = min(F, f0 + FB);
  int n = 0;
#pragma unroll 8
  for (int f = f0; f < f1; ++f) n += (abits[(size_t)f * SW + w] >> bit) & 1u;
  cnt[c * nfb + b] = n;
}

// pairs[] (frame ids, grouped by cell) and pidx[f][c] of the active cells from head_count's
// bitmap (32 B per frame at 16x16 instead of the 3 KB of masks); sampling also zeroes the
// outputs of inactive cells
__global__ __launch_bounds__(256) void head_scatter_kernel(
    const uint32_t* __restrict__ abits, int F, int S, int FB, const int* __restrict__ off,
    const int* __restrict__ grp_start,
    int* __restrict__ pairs, int* __restrict__ pidx, uint8_t* __restrict__ action_zero,
    float* __restrict__ cell_lp, float* __restrict__ cell_ent) {
  const int b = blockIdx.x, nfb = gridDim.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= S) return;
  const int f0 = b * FB, f1 = min(F, f0 + FB);
  const int SW = abits_words(S), w = c >> 5, bit = c & 31;
  const bool dense = action_zero || cell_lp || cell_ent;
  int pos = grp_start[c] + off[c * nfb + b];
#pragma unroll 4
  for (int f = f0; f < f1; ++f) {
    const size_t fc = (size_t)f * S + c;
    if ((abits[(size_t)f * SW + w] >> bit) & 1u) {
      pairs[pos] = f;
      pidx[fc] = pos;
      ++pos;
    } else if (dense) {
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
// head_fwd_kernel's count-mode sampling (same GEMM chain per logit, same Philox stream, same
// cell epilogue, so the two are bit-identical) with the policy step's finale folded in, so a step
// is two launches (trunk.hip act_trunk_w_kernel + this one) instead of head + row_sum_pack:
//   * work item = a JOB of up to 64 pairs of one cell (4 of head_fwd's 16-pair units): the wave
//     loads each W_c fragment once per job and feeds it to the 4 row blocks' MFMA chains (the
//     16-pair units of round 5 re-read the cell's whole 40 KB W_c from L2 per 16 pairs: ~150 MB
//     per 8192-env step, the kernel's dominant cost under the learner's HBM traffic);
//   * jobs are dealt to the XCDs in contiguous ranges of the cell-sorted job list (blockIdx % 8
//     labels the blocks of one XCD): an XCD's L2 then holds only ~1/8 of the 10.5 MB of packed
//     head weights instead of all of it;
//   * the 64 rows' logits go to the wave's LDS tile and the masked-cell epilogue (Philox, the
//     inverse-CDF sample, cell_forward) runs ONE PAIR PER LANE on all 64 lanes (head_fwd's unit
//     runs it on 16 lanes of 64);
//   * each sampled pair stores {log-prob, packed env action} as ONE 8-byte write-through (sc1)
//     granule in its env's per-cell row, drains it (vmcnt(0)), then decrements its env's
//     pending-cell counter (agent-scope atomic, set by launch A);
//   * the lane whose decrement empties the counter runs the env's finale itself (lane-parallel
//     over the wave's finishing envs): it reads the env's row with sc1 loads only (no fence:
//     MI355X_MICROARCH.md "Valid forms" -- every byte stored sc1 and drained before the signal,
//     every load of it sc1) and writes the env's log-prob (its cells' log-probs summed in cell
//     order, as row_sum_pack sums them: bit-identical) and its action codes / sparse action row
//     (also to pinned host memory);
//   * the bucket counters are double-buffered by step parity (launch A of the next step zeroes
//     this step's half) and the Philox step comes from the host, so no workgroup waits for or
//     counts the others.
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

#ifndef MBK_HA_NW
#define MBK_HA_NW 2
#endif
constexpr int HA_NW = MBK_HA_NW;    // waves per workgroup (LDS: ~3 workgroups per CU)
constexpr int HA_MB = MBK_HA_MB;     // 16-row blocks per job
constexpr int HA_JOB = 16 * HA_MB;  // pairs per job
constexpr int HA_ZS = NP + 1;       // logit tile row stride (floats): one row per lane

// exclusive prefix of ceil(cnt / HA_JOB) over the S <= kMaxUnitCells cells into jpre (wave 0,
// 16 cells per lane; jpre[kMaxUnitCells] = the job total). Caller barriers before reading it.
__device__ __forceinline__ void job_prefix(const int* __restrict__ cnt, int S, int* jpre) {
  const int lane = threadIdx.x & 63;
  if ((threadIdx.x >> 6) != 0) return;
  int loc[16], run = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = lane * 16 + k;
    loc[k] = run;
    run += c < S ? (cnt[c] + HA_JOB - 1) / HA_JOB : 0;
  }
  int x = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  const int base = x - run;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = lane * 16 + k;
    if (c <= S) jpre[c] = base + loc[k];
  }
  if (lane == 63) jpre[kMaxUnitCells] = x;
}

__device__ __forceinline__ void head_act_kernel_body(const HeadActArgs& a) {
  __shared__ float zs[HA_NW][HA_JOB * HA_ZS];
  __shared__ int jpre[kMaxUnitCells + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int S = a.S, E = a.E;
  job_prefix(a.cnt, S, jpre);
  __syncthreads();
  const int njobs = jpre[kMaxUnitCells];
  const uint64_t seed = a.rng[0], step = a.step;
  // the device copy of the step counter follows the graph path's (nobody reads it in here)
  if (blockIdx.x == 0 && threadIdx.x == 0) a.rng[1] = step + 1;
  // XCD-contiguous job ranges: the blocks b with b % ng == x (one XCD under the round-robin
  // placement; speed only) take jobs [x J / ng, (x + 1) J / ng)
  const int ng = min(8, (int)gridDim.x), xg = (int)blockIdx.x % ng;
  const int nbx = ((int)gridDim.x - xg + ng - 1) / ng, bx = (int)blockIdx.x / ng;
  const int j0 = (int)((long long)njobs * xg / ng), j1 = (int)((long long)njobs * (xg + 1) / ng);
  float* zt = zs[wave];
  for (int j = j0 + bx * HA_NW + wave; j < j1; j += nbx * HA_NW) {
    int lo = 0, hi = S - 1;  // last cell whose job prefix <= j
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jpre[mid] <= j) lo = mid; else hi = mid - 1;
    }
    const int c = lo;
    const int rb = c * E + HA_JOB * (j - jpre[c]);
    const int nr = min(HA_JOB, c * E + a.cnt[c] - rb);  // rows of this job (1 .. 64)
    // this lane's pair (the epilogue's row = lane) and the MFMA rows' frames (block mb, row li)
    const bool mine = lane < nr;
    const int ent = mine ? a.bucket[rb + lane] : 0;
    const int f = ent & 0xFFFF, rank = ent >> 16;  // env, rank among its active cells
    const size_t fc = (size_t)f * S + c;
    uint32_t m[3] = {0u, 0u, 0u};
    if (mine) { m[0] = a.mask[fc * 3]; m[1] = a.mask[fc * 3 + 1]; m[2] = a.mask[fc * 3 + 2]; }
    f32x4 acc[HA_MB][5];
#pragma unroll
    for (int mb = 0; mb < HA_MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint4* xr[HA_MB];
    bool xv[HA_MB];
#pragma unroll
    for (int mb = 0; mb < HA_MB; ++mb) {
      const int fr = __shfl(f, 16 * mb + li, 64);
      xv[mb] = 16 * mb + li < nr;
      xr[mb] = (const uint4*)(a.X + (size_t)fr * KD) + G;  // 8 bf16 per uint4
    }
    const bf16* wc = a.Wp + (size_t)c * NP * KD;
    // Z = X W_c^T + b: per logit the MFMA chain of unit_z (ks ascending from 0, then + bias).
    // Straight-line code over all 4 row blocks (a partial job's empty blocks multiply zero
    // rows): a wave-uniform skip inside the ks loop kept the compiler from hoisting the next
    // k-step's loads above it, one L2 round trip per k-step
#pragma unroll
    for (int ks = 0; ks < KD / 32; ++ks) {
      Frag8 bw[5];
#pragma unroll
      for (int nb = 0; nb < 5; ++nb)
        bw[nb].u = *((const uint4*)(wc + (size_t)(nb * 16 + li) * KD + ks * 32) + G);
#pragma unroll
      for (int mb = 0; mb < HA_MB; ++mb) {
        Frag8 xa;
        xa.u = xv[mb] ? xr[mb][ks * 4] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int nb = 0; nb < 5; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa.v, bw[nb].v, acc[mb][nb], 0, 0, 0);
      }
    }
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) {
      const int col = nb * 16 + li;
      const float bias = a.bp[c * NP + col];
#pragma unroll
      for (int mb = 0; mb < HA_MB; ++mb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) zt[(16 * mb + 4 * G + i) * HA_ZS + col] = acc[mb][nb][i] + bias;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes of this wave visible
    __builtin_amdgcn_wave_barrier();
    if (mine) {
      uint8_t act[kComps];
      float uu[kComps];
      u32x4 ctr = {(uint32_t)fc, (uint32_t)(fc >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
      u32x4 q0 = philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
      ctr.y ^= 0x80000000u;
      u32x4 q1 = philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
      uu[0] = u01(q0.x); uu[1] = u01(q0.y); uu[2] = u01(q0.z); uu[3] = u01(q0.w);
      uu[4] = u01(q1.x); uu[5] = u01(q1.y); uu[6] = u01(q1.z);
      float lp, en;
      cell_forward(zt + lane * HA_ZS, m, act, true, uu, &lp, &en);
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
    if (fin) {  // this lane sampled its env's last active cell: the env's finale, lane-parallel
      // (round 5 ran one env at a time on the whole wave: with 64 pairs per job a wave can finish
      // dozens of envs, each a dependent sc1 round trip)
      const uint64_t* row = a.cellx + (size_t)f * S;
      const int n = a.pending[E + f];  // the env's active cells (granules, rank = cell order)
      uint32_t* lrow = a.act_list ? a.act_list + (size_t)f * a.list_stride : nullptr;
      float s = 0.f;  // the env's log-prob: its cells' log-probs in cell order (row_sum_pack's)
      int nz = 0;     // sparse rows: entries written so far
      for (int k0 = 0; k0 < n; k0 += 8) {
        uint64_t xs[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)  // sc1 loads only (see above), 8 in flight
          xs[i] = k0 + i < n ? __hip_atomic_load(row + k0 + i, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) : 0ull;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (k0 + i >= n) break;
          const uint32_t hi = (uint32_t)(xs[i] >> 32), code = hi >> 16;
          s += __uint_as_float((uint32_t)xs[i]);
          if (lrow) {  // only the non-noop cells travel back to the env
            if (code != 0u) lrow[1 + nz++] = (hi & 0xFFFFu) | (code << 16);
          } else {
            a.act16[(size_t)f * S + (hi & 0xFFFFu)] = (uint16_t)code;
          }
        }
      }
      a.logp[f] = s;
      if (lrow) lrow[0] = (uint32_t)nz;
    }
    __builtin_amdgcn_wave_barrier();  // the logit tile is rewritten by the next job
  }
}
// thin wrapper: the body takes the arguments by const reference (conv0_row_kernel, profile 43)
__global__ __launch_bounds__(64 * HA_NW, 2) void head_act_kernel(HeadActArgs a) {
  head_act_kernel_body(a);
}

// logp[f] = sum over f's active cells of the pair log-probs (ent likewise), in cell order
// (deterministic): one lane per frame walking its bitmap row's set bits (~2 of 256 cells), so
// 64 frames share a wave. (One wave per frame -- 524K tiny waves, each paying the bitmap ->
// pidx -> log-prob chain with 1 to 2 of its 64 lanes busy -- took 183 us per learner update.)
__global__ __launch_bounds__(256) void head_pair_rowsum_kernel(const int* __restrict__ pidx,
                                                               const uint32_t* __restrict__ abits,
                                                               int F,
                                                               int S, const float* __restrict__ plp,
                                                               const float* __restrict__ pent,
                                                               float* __restrict__ logp,
                                                               float* __restrict__ ent) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= F) return;
  const int SW = abits_words(S);
  const uint32_t* ab = abits + (size_t)f * SW;
  const int* pr = pidx + (size_t)f * S;
  float a = 0.f, b = 0.f;
  for (int w = 0; w < SW; ++w) {
    uint32_t bits = ab[w];
    if (32 * w + 32 > S) bits &= (1u << (S - 32 * w)) - 1u;  // (the last word's tail)
    while (bits) {
      const int p = pr[32 * w + __builtin_ctz(bits)];
      bits &= bits - 1u;
      a += plp[p];
      if (pent) b += pent[p];
    }
  }
  logp[f] = a;
  if (ent) ent[f] = b;
}

// ------------------------------------------------------------------ backward
// ------------------------------------------------------------------ backward, v2
// head_bwd2: 8 waves, 128-pair tiles, everything a tile needs in LDS:
//   W_c  [96 rows][544 B]  the cell's 78 (+2 zero, +16 zero) logit rows, staged once per chunk
//   X    [128][544 B]      the tile's gathered feature rows (next tile prefetched in registers)
//   dZ   [128][288 B]      bf16 logit gradients
// Z = X W_c^T + b on MFMA, then the masked-softmax backward straight from the MFMA C layout
// (a row's 80 logits sit in the 16 lanes of one lane group, 5 registers: per-segment max /
// sum / sum z*e are 16-lane DPP reductions; segments with no valid logit anywhere in the
// wave are skipped), dX = dZ W_c (B operand = W_c through ds_read_b64_tr_b16), dW_c += dZ^T X.
// Rows are stored at phi(r) (4-row blocks 1 and 2 of each 16 swapped) with a row stride of
// 32 mod 256 bytes: the tr reads (rows r..r+3 and r+8..r+11 per half-wave) and the b128
// row reads are then bank-conflict-free. The old kernel (one 64-row workgroup, W_c read from
// L2 by every wave, a 64-thread scalar softmax backward) spent ~88 % of its wave cycles
// waiting (profile 27).
constexpr int HB_NW = 8;
constexpr int HB_TM = 16 * HB_NW;
constexpr int HB_RX = 544, HB_RW = 544, HB_RZ = 288;
constexpr int HB_LW = 0, HB_LX = 96 * HB_RW, HB_LZ = HB_LX + HB_TM * HB_RX;
constexpr int HB_LB = HB_LZ + HB_TM * HB_RZ;           // bias-grad reduce [8 waves][80] f32
constexpr int HB_LDS = HB_LB + HB_NW * NP * 4;

__device__ __forceinline__ int hb_phi(int r) {
  const int b = (r >> 2) & 3;
  return (b == 1 || b == 2) ? r ^ 12 : r;
}
// (bound_ctrl set: these patterns never leave the row, and it lets the compiler fold the move
// into the consuming add / max as a DPP operand)
template <int CTRL>
__device__ __forceinline__ float hb_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// reductions over the 16 lanes of a DPP row (quad swaps, half-row mirror, row mirror) of N
// independent values, interleaved step by step (no DPP read right after its VALU write)
constexpr int kHbDpp[4] = {0xB1, 0x4E, 0x141, 0x140};
template <int N>
__device__ __forceinline__ void hb_max16(float (&v)[N]) {
#pragma unroll
  for (int st = 0; st < 4; ++st)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float o = st == 0 ? hb_dpp<0xB1>(v[j]) : st == 1 ? hb_dpp<0x4E>(v[j])
                    : st == 2 ? hb_dpp<0x141>(v[j]) : hb_dpp<0x140>(v[j]);
      v[j] = fmaxf(v[j], o);
    }
}
template <int N>
__device__ __forceinline__ void hb_sum16(float (&v)[N]) {
#pragma unroll
  for (int st = 0; st < 4; ++st)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float o = st == 0 ? hb_dpp<0xB1>(v[j]) : st == 1 ? hb_dpp<0x4E>(v[j])
                    : st == 2 ? hb_dpp<0x141>(v[j]) : hb_dpp<0x140>(v[j]);
      v[j] += o;
    }
}

// ST: the forward's per-pair softmax statistics (head_score_kernel's stats: lse and entropy of
// each segment) are staged with the row metadata, and the epilogue is per logit: no segment
// max / sum reductions (a row's 16 lanes reducing by DPP were ~40 % of the kernel, VALU-bound).
template <bool ST>
__global__ __launch_bounds__(64 * HB_NW, 1) void head_bwd2_kernel(
    const bf16* __restrict__ X, const bf16* __restrict__ Wp, const float* __restrict__ bp,
    const uint32_t* __restrict__ mask, const uint8_t* __restrict__ action,
    const int* __restrict__ pairs, const int* __restrict__ grp_start,
    const int* __restrict__ grp_count, const int* __restrict__ chunk_cell,
    const int* __restrict__ chunk_row, const int* __restrict__ totals,
    const float* __restrict__ g_logp, const float* __restrict__ g_ent, int S,
    bf16* __restrict__ dXp, float* __restrict__ dWp, float* __restrict__ dbp,
    uint64_t* __restrict__ stamps, const float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem + HB_LW;
  int nst = 0;  // diagnostic phase stamps (MBK_HB_STAMPS): thread 0, first 8 tiles
#define HB_STAMP(k)                                                                        \
  do {                                                                                     \
    if (stamps && threadIdx.x == 0 && nst < 8)                                             \
      stamps[((size_t)blockIdx.x * 8 + nst) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  char* xl = smem + HB_LX;
  char* zl = smem + HB_LZ;
  float* bl = (float*)(smem + HB_LB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  const int nchunks = totals[2];
  // a contiguous range of chunks per workgroup (chunks are in cell order): consecutive chunks
  // of one cell keep W_c staged and accumulate dW / db in registers, and only the last chunk
  // of each such run writes a partial (head_dw_reduce reads exactly those: hb_run_end)
  const int qn = (nchunks + (int)gridDim.x - 1) / (int)gridDim.x;
  const int ch_begin = (int)blockIdx.x * qn, ch_end = min(nchunks, ch_begin + qn);
  if (ch_begin >= nchunks) return;
  // W rows 80..95 stay zero (the dX GEMM's K runs to 96)
  for (int e = tid; e < 16 * HB_RW / 16; e += 64 * HB_NW)
    ((uint4*)(wl + 80 * HB_RW))[e] = make_uint4(0, 0, 0, 0);

  // this lane's logit column per MFMA block: segment index and position inside it
  int sk[5], so[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    const int col = nb * 16 + li;
    int k = 0;
#pragma unroll
    for (int q = 1; q < kComps; ++q) k += col >= seg_off(q) ? 1 : 0;
    sk[nb] = col < kCell ? k : kComps;
    so[nb] = col - seg_off(k);
  }

  // staging map: thread -> 16-byte chunk q of rows r0 + 16 k
  const int sq = tid & 31, sr0 = tid >> 5;
  uint4 xr[8];
  // tile cursor: chunk ch (cell c, first row g0, n rows), tile offset t0; ch >= nchunks = end
  struct Cur {
    int ch, t0, c, g0, n;
  };
  auto chunk_cur = [&](int ch) {
    if (ch >= ch_end) ch = nchunks;  // past this workgroup's range: the end
    Cur u{ch, 0, 0, 0, 0};
    if (ch < nchunks) {
      u.c = chunk_cell[ch];
      u.g0 = chunk_row[ch];
      u.n = min(CHUNK, grp_start[u.c] + grp_count[u.c] - u.g0);
    }
    return u;
  };
  auto advance = [&](const Cur& u) {
    if (u.ch >= nchunks) return u;
    if (u.t0 + HB_TM < u.n) return Cur{u.ch, u.t0 + HB_TM, u.c, u.g0, u.n};
    return chunk_cur(u.ch + 1);
  };
  // Per-row metadata (mask words, the aligned action words, g_logp, g_ent, frame) goes through
  // the dZ tile's row padding (bytes 192..227 of each 288-byte row): threads 0..383 each load
  // one third of one row's 9 words for the NEXT tile (3 loads instead of 32 per wave) and write
  // them at the tile start; the epilogue reads its rows' 36 bytes back as broadcasts.
  // fx / fr: frames of the rows this thread stages / loads metadata for, two tiles ahead.
  const int mrow = tid / 3, mpart = tid - 3 * (tid / 3);
  int fx[8], fr = -1;
  uint32_t mt[3] = {0u, 0u, 0u};
  auto load_fx = [&](const Cur& u) {
    const int nr = u.ch < nchunks ? min(HB_TM, u.n - u.t0) : 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) fx[k] = sr0 + 16 * k < nr ? pairs[u.g0 + u.t0 + sr0 + 16 * k] : -1;
    fr = tid < 3 * HB_TM && mrow < nr ? pairs[u.g0 + u.t0 + mrow] : -1;
  };
  auto load_meta = [&](int c) {  // this thread's third of row mrow's metadata (frame fr, cell c)
    mt[0] = mt[1] = mt[2] = 0u;
    if (fr < 0) {
      if (mpart == 2) mt[2] = 0xFFFFFFFFu;  // frame -1: padding row
      return;
    }
    const size_t fc = (size_t)fr * S + c;
    if (mpart == 0) {
      mt[0] = mask[fc * 3]; mt[1] = mask[fc * 3 + 1]; mt[2] = mask[fc * 3 + 2];
    } else if (mpart == 1) {
      // only words holding one of the row's 7 action bytes (never past the buffer's end)
      const size_t ab0 = fc * kComps;
      const uint32_t* aw4 = (const uint32_t*)(action + (ab0 & ~(size_t)3));
      mt[0] = aw4[0]; mt[1] = aw4[1]; mt[2] = (ab0 & 3) >= 2 ? aw4[2] : 0u;
    } else {
      mt[0] = __float_as_uint(g_logp[fr]);
      mt[1] = g_ent ? __float_as_uint(g_ent[fr]) : 0u;
      mt[2] = (uint32_t)fr;
    }
  };
  auto store_meta = [&]() {
    if (tid < 3 * HB_TM) {
      uint32_t* d = (uint32_t*)(zl + hb_phi(mrow) * HB_RZ + 192 + mpart * 12);
      d[0] = mt[0]; d[1] = mt[1]; d[2] = mt[2];
    }
  };
  // ST: a quarter (16 B) of one row's 64-byte statistics {lse[7], H[7], 0, 0} per thread,
  // stored at bytes 228.. of the dZ tile row's padding (lse at 228 + 4k, H at 256 + 4k)
  const int srow = tid >> 2, squ = tid & 3;
  uint4 st4 = make_uint4(0u, 0u, 0u, 0u);
  auto load_stats = [&](const Cur& u) {
    if constexpr (ST) {
      const int nr = u.ch < nchunks ? min(HB_TM, u.n - u.t0) : 0;
      st4 = srow < nr ? ((const uint4*)(stats + (size_t)(u.g0 + u.t0 + srow) * 16))[squ]
                      : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store_stats = [&]() {
    if constexpr (ST) {
      uint32_t* d = (uint32_t*)(zl + hb_phi(srow) * HB_RZ + 228 + squ * 16);
      d[0] = st4.x; d[1] = st4.y;
      if (squ < 3) {
        d[2] = st4.z; d[3] = st4.w;
      }
    }
  };
  auto load_x = [&]() {  // the rows of fx into registers
#pragma unroll
    for (int k = 0; k < 8; ++k)
      xr[k] = fx[k] >= 0 ? ((const uint4*)(X + (size_t)fx[k] * KD))[sq] : make_uint4(0, 0, 0, 0);
  };
  auto store_x = [&]() {
#pragma unroll
    for (int k = 0; k < 8; ++k) *(uint4*)(xl + hb_phi(sr0 + 16 * k) * HB_RX + sq * 16) = xr[k];
  };
  auto stage_w = [&](int c) {  // rows 0..79 of W_c
    const uint4* src = (const uint4*)(Wp + (size_t)c * NP * KD);
    uint4 v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) v[k] = src[(sr0 + 16 * k) * (KD / 8) + sq];
#pragma unroll
    for (int k = 0; k < 5; ++k) *(uint4*)(wl + hb_phi(sr0 + 16 * k) * HB_RW + sq * 16) = v[k];
  };

  Cur cur = chunk_cur(ch_begin);
  Cur nx1 = advance(cur);
  load_fx(cur);
  load_x();           // tile 0's rows and metadata
  load_meta(cur.c);
  load_stats(cur);
  load_fx(nx1);       // tile 1's frames
  f32x4 accw[5][2];
  float dbs[5], bcol[5];
  bool new_chunk = true;
  for (;;) {
    const int ch = cur.ch, c = cur.c, g = cur.g0 + cur.t0, nr = min(HB_TM, cur.n - cur.t0);
    HB_STAMP(0);
    lds_barrier();  // previous tile's LDS reads done
    store_x();
    store_meta();
    store_stats();
    if (new_chunk) {
      stage_w(c);
#pragma unroll
      for (int mb = 0; mb < 5; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) accw[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) {
        dbs[nb] = 0.f;
        bcol[nb] = bp[(size_t)c * NP + nb * 16 + li];
      }
      new_chunk = false;
    }
    lds_barrier();
    HB_STAMP(1);
    const bool last = nx1.ch != ch, has_next = nx1.ch < nchunks;
    // the last tile of a run of this cell's chunks (the next tile is another cell's, or none)
    const bool run_end = last && !(has_next && nx1.c == c);
    // ---- Z = X W_c^T + b (this wave's 16 rows x 80)
    f32x4 z[5];
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) z[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* xa = xl + hb_phi(16 * wave + li) * HB_RX + 16 * G;
#pragma unroll 2
    for (int ks = 0; ks < KD / 32; ++ks) {
      Frag8 a;
      a.u = *(const uint4*)(xa + ks * 64);
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) {
        Frag8 b;
        b.u = *(const uint4*)(wl + hb_phi(nb * 16 + li) * HB_RW + ks * 64 + 16 * G);
        z[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, z[nb], 0, 0, 0);
      }
    }

    HB_STAMP(2);
    // ---- dZ from the C layout: lane (li, G) holds column nb*16+li of rows 4G+i
    // this wave's rows 16 wave + 4 G + i: metadata from the dZ tile's row padding
    uint32_t mw[4][3], aw[4][3];
    int ab[4];
    float gl[4], ge[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t* m = (const uint32_t*)(zl + hb_phi(16 * wave + 4 * G + i) * HB_RZ + 192);
      const uint4 q0 = *(const uint4*)m, q1 = *(const uint4*)(m + 4);
      const uint32_t fw = m[8];
      mw[i][0] = q0.x; mw[i][1] = q0.y; mw[i][2] = q0.z;
      aw[i][0] = q0.w; aw[i][1] = q1.x; aw[i][2] = q1.y;
      gl[i] = __uint_as_float(q1.z);
      ge[i] = __uint_as_float(q1.w);
      ab[i] = (int)((((size_t)(int)fw * S + c) * kComps) & 3);
    }
    // zz: the logits, overwritten in place by their gradient as each segment is finished
    // (every logit belongs to exactly one segment); ok: valid (masked-in) logits
    uint32_t okm = 0u;  // bit nb*4+i: logit (nb, i) valid
    float zz[5][4];
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) {
      const float b = bcol[nb];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        zz[nb][i] = z[nb][i] + b;
        const int bit = (nb & 1) * 16 + li;
        okm |= (sk[nb] < kComps && ((mw[i][nb >> 1] >> bit) & 1u)) ? 1u << (nb * 4 + i) : 0u;
      }
    }
    if constexpr (ST) {
      // per logit: lp = z - lse_k, p = e^lp, dz = gl (1[j == a_k] - p) - ge p (lp + H_k)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* rowp = zl + hb_phi(16 * wave + 4 * G + i) * HB_RZ;
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) {
          const int k = min(sk[nb], kComps - 1);
          const float lse = *(const float*)(rowp + 228 + 4 * k);
          const float H = *(const float*)(rowp + 256 + 4 * k);
          const int bi = ab[i] + k;
          const uint32_t wsel = bi < 4 ? aw[i][0] : bi < 8 ? aw[i][1] : aw[i][2];
          const int a = (int)((wsel >> (8 * (bi & 3))) & 0xFFu);
          const float lp = zz[nb][i] - lse;
          const float p = __expf(lp);
          zz[nb][i] = gl[i] * ((so[nb] == a ? 1.f : 0.f) - p) - ge[i] * p * (lp + H);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < (ST ? 0 : kComps); ++k) {
      const int c0 = seg_off(k), c1 = seg_off(k + 1);
      const int nb0 = c0 / 16, nb1 = (c1 - 1) / 16;
      bool any = false;
#pragma unroll
      for (int nb = nb0; nb <= nb1; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) any |= ((okm >> (nb * 4 + i)) & 1u) && sk[nb] == k;
      if (__ballot(any) == 0ull) continue;  // wave-uniform: no valid logit of segment k
      // the 4 rows' reductions interleaved
      float mx[4], sm[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mx[i] = -INFINITY;
#pragma unroll
        for (int nb = nb0; nb <= nb1; ++nb)
          if (((okm >> (nb * 4 + i)) & 1u) && sk[nb] == k) mx[i] = fmaxf(mx[i], zz[nb][i]);
      }
      hb_max16(mx);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float e_s = 0.f, e_sz = 0.f;
#pragma unroll
        for (int nb = nb0; nb <= nb1; ++nb) {
          const bool in = ((okm >> (nb * 4 + i)) & 1u) && sk[nb] == k;
          const float e = in ? __expf(zz[nb][i] - mx[i]) : 0.f;
          e_s += e;
          e_sz += e * zz[nb][i];
        }
        sm[2 * i] = e_s;
        sm[2 * i + 1] = e_sz;
      }
      hb_sum16(sm);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // lse = log sum exp, H = entropy = lse - sum p z; p = exp(z - lse)
        const float lse = mx[i] + __logf(sm[2 * i]);
        const float H = lse - sm[2 * i + 1] * __builtin_amdgcn_rcpf(sm[2 * i]);
        // action of segment k in this row: byte ab + k of the 3 words
        const int bi = ab[i] + k;
        const uint32_t wsel = bi < 4 ? aw[i][0] : bi < 8 ? aw[i][1] : aw[i][2];
        const int a = (int)((wsel >> (8 * (bi & 3))) & 0xFFu);
#pragma unroll
        for (int nb = nb0; nb <= nb1; ++nb) {
          const bool in = ((okm >> (nb * 4 + i)) & 1u) && sk[nb] == k;
          const float lp = zz[nb][i] - lse;
          const float p = __expf(lp);
          const float v = gl[i] * ((so[nb] == a ? 1.f : 0.f) - p) - ge[i] * p * (lp + H);
          zz[nb][i] = in ? v : zz[nb][i];
        }
      }
    }
    float d[5][4];
#pragma unroll
    for (int nb = 0; nb < 5; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) d[nb][i] = ((okm >> (nb * 4 + i)) & 1u) ? zz[nb][i] : 0.f;
    // dZ -> bf16 tile (rows phi(16 wave + 4 G + i), column nb*16 + li); bias-grad column sums
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) {
      float cs = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * wave + 4 * G + i;
        *(bf16*)(zl + hb_phi(r) * HB_RZ + (nb * 16 + li) * 2) = f2bf(d[nb][i]);
        cs += d[nb][i];
      }
      dbs[nb] += cs;
    }
    // columns 80..95 of the dZ tile are the dX GEMM's zero K tail
    if (li < 8) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * wave + 4 * G + i;
        *(uint32_t*)(zl + hb_phi(r) * HB_RZ + 160 + li * 4) = 0u;
      }
    }
    // next tile's rows and metadata: in flight through both GEMMs (issued after the epilogue,
    // whose register peak they would otherwise add to)
    if (has_next) {
      load_x();
      load_meta(nx1.c);
      load_stats(nx1);
    }
    // then the tile after next: its cursor (scalar loads when it starts a chunk) and frames
    // (fx / fr hold the next tile's frames until the two gathers above are issued)
    const Cur nx2 = advance(nx1);
    if (nx2.ch < nchunks) load_fx(nx2);
    HB_STAMP(3);
    lds_barrier();  // dZ tile complete
    HB_STAMP(4);

    // ---- dW_c += dZ^T X (logit rows x feature columns 32 wave.., K = the tile's rows)
#pragma unroll 1
    for (int ks = 0; ks < HB_TM / 32; ++ks) {
      Frag8 a[5];
#pragma unroll
      for (int mb = 0; mb < 5; ++mb)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int pr = hb_phi(ks * 32 + 8 * G + 4 * h + (li >> 2));
          a[mb].h[h] = tr_read(zl + pr * HB_RZ + (mb * 16 + 4 * (li & 3)) * 2);
        }
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        Frag8 b;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int pr = hb_phi(ks * 32 + 8 * G + 4 * h + (li >> 2));
          b.h[h] = tr_read(xl + pr * HB_RX + (32 * wave + nb * 16 + 4 * (li & 3)) * 2);
        }
#pragma unroll
        for (int mb = 0; mb < 5; ++mb)
          accw[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mb].v, b.v, accw[mb][nb], 0, 0, 0);
      }
    }
    // ---- dX_pair = dZ W_c (this wave's rows, 256 columns in two halves; K = 96), bf16. The
    // X tile is free once every wave's dW is done: each wave stages its 16 x 256 rows there
    // (C-layout 2-byte writes, 528-byte rows) and stores them as 16-byte chunks (the pair-row
    // writes are this kernel's largest HBM traffic: 512 B per pair)
    lds_barrier();
    HB_STAMP(5);
    const char* za = zl + hb_phi(16 * wave + li) * HB_RZ + 16 * G;
    char* stg = xl + wave * 16 * 528;
#pragma unroll 1
    for (int hc = 0; hc < 2; ++hc) {
      f32x4 acc[8];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int ks = 0; ks < NPT / 32; ++ks) {
        Frag8 a;
        a.u = *(const uint4*)(za + ks * 64);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) {
          Frag8 b;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int kr = ks * 32 + 8 * G + 4 * h + (li >> 2);
            b.h[h] = tr_read(wl + hb_phi(kr) * HB_RW + ((hc * 8 + nb) * 16 + 4 * (li & 3)) * 2);
          }
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc[nb], 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          *(bf16*)(stg + (4 * G + i) * 528 + ((hc * 8 + nb) * 16 + li) * 2) = f2bf(acc[nb][i]);
    }
    // Every load of this wave is complete before the stores go out: vmcnt counts stores too,
    // and a later wait on any load would otherwise also wait for these stores' completion
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // same wave, in-order LDS: the reads see the writes above; 2 rows x 512 B per instruction
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int rr = 2 * q + (lane >> 5), r = 16 * wave + rr;
      const uint4 v = *(const uint4*)(stg + rr * 528 + (lane & 31) * 16);
      if (r < nr) *(uint4*)(dXp + (size_t)(g + r) * KD + (lane & 31) * 8) = v;
    }
    HB_STAMP(6);
    if (run_end) {
      // ---- this run's partial dW / db, in the slot of its last chunk (reduced per cell by
      // head_dw_reduce)
      // one base per lane, compile-time offsets (no per-row 64-bit pointers kept live)
      float* dwb = dWp + ((size_t)ch * kCell + 4 * G) * KD + 32 * wave + li;
#pragma unroll
      for (int mb = 0; mb < 5; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (mb == 4 && 4 * G + i >= kCell - 64) continue;  // logit rows 78, 79
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) dwb[(mb * 16 + i) * KD + nb * 16] = accw[mb][nb][i];
        }
      // bias grad: the 4 lane groups' column sums, then the 8 waves through LDS
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) {
        float v = dbs[nb];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (G == 0) bl[wave * NP + nb * 16 + li] = v;
      }
      lds_barrier();
      if (tid < kCell) {
        float v = 0.f;
        for (int w = 0; w < HB_NW; ++w) v += bl[w * NP + tid];
        dbp[(size_t)ch * kCell + tid] = v;
      }
      if (!has_next) break;
      new_chunk = true;
    }
    HB_STAMP(7);
    ++nst;
    cur = nx1;
    nx1 = nx2;
  }
}

// ------------------------------------------------------------------ learner scoring
// The learner's forward over the compacted pairs (pair-indexed log-prob / entropy of the given
// actions; head_pair_rowsum sums them per frame). head_fwd_kernel's 16-pair units read all of
// W_c (40 KB) from L2 per unit and ran the 78-logit epilogue on 16 lanes of 64 (560 us per
// 524K-frame update). Here a workgroup takes a contiguous range of 256-row work items (half of
// one 512-pair chunk of one cell), so W_c is staged in LDS once per cell run. Each wave MFMAs
// its 64 rows as four 16-row blocks (A straight from X, B from LDS), parks the logits in its
// LDS tile and reads them back one row per lane: the epilogue (cell_forward, the sampling
// path's) then runs on all 64 lanes. (A C-layout epilogue -- a row's 16 lanes reducing each
// segment by DPP -- issued ~8x the VALU instructions per row: 356 us, VALU-bound.)
constexpr int HS_NW = 4, HS_TM = 64 * HS_NW, HS_IPC = CHUNK / HS_TM;  // items per chunk
constexpr int HS_ZS = NP + 1;                        // Z tile row stride (floats): conflict-free
constexpr int HS_LZ = 80 * HB_RW;                    // per-wave Z tiles [64][HS_ZS] f32
constexpr int HS_LDS = HS_LZ + HS_NW * 64 * HS_ZS * 4;

__global__ __launch_bounds__(64 * HS_NW, 1) void head_score_kernel(
    const bf16* __restrict__ X, const bf16* __restrict__ Wp, const float* __restrict__ bp,
    const uint32_t* __restrict__ mask, const uint8_t* __restrict__ action,
    const int* __restrict__ pairs, const int* __restrict__ grp_start,
    const int* __restrict__ grp_count, const int* __restrict__ chunk_cell,
    const int* __restrict__ chunk_row, const int* __restrict__ totals, int S,
    float* __restrict__ plp, float* __restrict__ pent, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, li = lane & 15;
  float* zt = (float*)(smem + HS_LZ) + wave * 64 * HS_ZS;
  // items: HS_IPC per chunk (rows 0, HS_TM, .. of it); workgroup b takes items [b q, b q + q)
  const int nitems = HS_IPC * totals[2];
  const int q = (nitems + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = (int)blockIdx.x * q, i1 = min(nitems, i0 + q);
  const int sq = tid & 31, sr0 = tid >> 5;  // W staging: 16-byte chunk sq of rows sr0 + RS k
  float bcol[5];
  int wc = -1;
  // item cursor: the next non-empty item from it on (it == i1: none), its cell, this wave's
  // first row and row count, and the frame of row `lane` (loaded one item ahead)
  struct Item {
    int it, c, rb, nr, f;
  };
  auto item_at = [&](int it) {
    Item u{i1, 0, 0, 0, -1};
    for (; it < i1; ++it) {
      const int ch = it / HS_IPC, t0 = (it % HS_IPC) * HS_TM;
      const int c = chunk_cell[ch], g0 = chunk_row[ch];
      const int n = min(CHUNK, grp_start[c] + grp_count[c] - g0);
      if (t0 >= n) continue;  // workgroup-uniform
      u.it = it;
      u.c = c;
      u.rb = g0 + t0 + 64 * wave;
      u.nr = min(64, n - t0 - 64 * wave);
      u.f = lane < u.nr ? pairs[u.rb + lane] : -1;
      break;
    }
    return u;
  };
  Item nx = item_at(i0);
  while (nx.it < i1) {
    const Item cu = nx;
    const int c = cu.c, rb = cu.rb, nr = cu.nr, f = cu.f;
    // this lane's row: mask words and the words holding its 7 action bytes
    uint32_t m[3] = {0u, 0u, 0u}, aw[3] = {0u, 0u, 0u};
    int ab = 0;
    if (f >= 0) {
      const size_t fc = (size_t)f * S + c;
      m[0] = mask[fc * 3]; m[1] = mask[fc * 3 + 1]; m[2] = mask[fc * 3 + 2];
      const size_t ab0 = fc * kComps;
      const uint32_t* aw4 = (const uint32_t*)(action + (ab0 & ~(size_t)3));
      aw[0] = aw4[0]; aw[1] = aw4[1]; aw[2] = (ab0 & 3) >= 2 ? aw4[2] : 0u;
      ab = (int)(ab0 & 3);
    }
    nx = item_at(cu.it + 1);  // the next item's frames: in flight through this one
    if (c != wc) {  // stage W_c (rows 0..79) once per run of the cell's items
      // (rare: a workgroup's items are contiguous, so this runs once or twice per workgroup)
      constexpr int RS = 64 * HS_NW / 32;  // rows per pass
      const uint4* src = (const uint4*)(Wp + (size_t)c * NP * KD) + sr0 * (KD / 8) + sq;
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) bcol[nb] = bp[(size_t)c * NP + nb * 16 + li];
      lds_barrier();  // every wave is done with the previous W_c
#pragma unroll
      for (int k = 0; k < 80 / RS; ++k)
        *(uint4*)(wl + hb_phi(sr0 + RS * k) * HB_RW + sq * 16) = src[RS * k * (KD / 8)];
      wc = c;
      lds_barrier();  // W_c staged
    }
    if (nr <= 0) continue;  // wave-uniform: a partial item's idle waves
    // ---- Z = X W_c^T + b for the wave's 4 row blocks -> Z tile (C layout: lane (li, G) holds
    // column nb*16+li of rows 16 mb + 4G+i); the next block's A fragments load during each GEMM
    uint4 xa[2][KD / 32];
    auto load_a = [&](int mb, uint4 (&d)[KD / 32]) {
      const int fr = __shfl(f, 16 * mb + li, 64);
      const uint4* xr = (const uint4*)(X + (size_t)max(fr, 0) * KD) + G;
#pragma unroll
      for (int ks = 0; ks < KD / 32; ++ks) d[ks] = fr >= 0 ? xr[ks * 4] : make_uint4(0, 0, 0, 0);
    };
    load_a(0, xa[0]);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      if (mb + 1 < 4 && 16 * (mb + 1) < nr) load_a(mb + 1, xa[(mb + 1) & 1]);
      if (16 * mb >= nr) break;  // wave-uniform
      f32x4 z[5];
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) z[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KD / 32; ++ks) {
        Frag8 a;
        a.u = xa[mb & 1][ks];
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) {
          Frag8 b;
          b.u = *(const uint4*)(wl + hb_phi(nb * 16 + li) * HB_RW + ks * 64 + 16 * G);
          z[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, z[nb], 0, 0, 0);
        }
      }
#pragma unroll
      for (int nb = 0; nb < 5; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) zt[(16 * mb + 4 * G + i) * HS_ZS + nb * 16 + li] = z[nb][i] + bcol[nb];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's Z tile writes are done
    __builtin_amdgcn_wave_barrier();
    // ---- one row per lane: the 78 logits into registers, then the masked cell epilogue
    if (lane < nr) {
      float zr[kCell];
      const float* zrow = zt + lane * HS_ZS;
#pragma unroll
      for (int j = 0; j < kCell; ++j) zr[j] = zrow[j];
      // cell_forward's scoring with the action's logit read from the tile (a register array
      // indexed by the action would live in scratch)
      float lp = 0.f, ent = 0.f;
      float sl[kComps], sh[kComps];  // per segment: lse and entropy (0: fully masked)
#pragma unroll
      for (int k = 0; k < kComps; ++k) {
        const int off = seg_off(k), n = seg_off(k + 1) - off;
        sl[k] = sh[k] = 0.f;
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < n; ++j)
          if (mask_bit(m, off + j)) mx = fmaxf(mx, zr[off + j]);
        if (mx == -INFINITY) continue;  // fully masked segment: log-prob 0, entropy 0
        float sm = 0.f, sz = 0.f;
#pragma unroll
        for (int j = 0; j < n; ++j) {
          const float e = mask_bit(m, off + j) ? __expf(zr[off + j] - mx) : 0.f;
          sm += e;
          sz += e * zr[off + j];
        }
        const float lse = mx + __logf(sm);
        const float h = lse - sz * (1.f / sm);
        ent += h;
        sl[k] = lse;
        sh[k] = h;
        const int bi = ab + k;
        const uint32_t w = bi < 4 ? aw[0] : bi < 8 ? aw[1] : aw[2];
        const int a = (int)((w >> (8 * (bi & 3))) & 0xFFu);
        const uint32_t mj = (uint32_t)(off + a);
        const uint32_t mwd = mj < 32 ? m[0] : mj < 64 ? m[1] : m[2];
        const bool valid = a < n && ((mwd >> (mj & 31)) & 1u);
        lp += (valid ? zrow[off + a] : -1e8f) - lse;
      }
      plp[rb + lane] = lp;
      if (pent) pent[rb + lane] = ent;
      if (stats) {  // the backward's softmax statistics of this pair: {lse[7], H[7], 0, 0}
        float4* st = (float4*)(stats + (size_t)(rb + lane) * 16);
        st[0] = make_float4(sl[0], sl[1], sl[2], sl[3]);
        st[1] = make_float4(sl[4], sl[5], sl[6], sh[0]);
        st[2] = make_float4(sh[1], sh[2], sh[3], sh[4]);
        st[3] = make_float4(sh[5], sh[6], 0.f, 0.f);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the Z tile is rewritten by the next item
  }
}

// dW[c*78+n][d] = sum over the cell's chunks (fixed order); zero for idle cells
// head_bwd2 (grid bwd_grid) wrote a partial only at the last chunk of each run of one cell's
// chunks inside a workgroup's contiguous range: chunk ch of a cell whose chunks end at c_end
__device__ __forceinline__ bool hb_run_end(int ch, int c_end, int nchunks, int bwd_grid) {
  const int qn = (nchunks + bwd_grid - 1) / bwd_grid;
  return ch + 1 == c_end || (ch + 1) % qn == 0;
}

__global__ __launch_bounds__(256) void head_dw_reduce_kernel(const float* __restrict__ dWp,
                                                             const float* __restrict__ dbp,
                                                             const int* __restrict__ chunk_start,
                                                             const int* __restrict__ grp_count,
                                                             const int* __restrict__ totals,
                                                             int bwd_grid, int S,
                                                             float* __restrict__ dW,
                                                             float* __restrict__ db) {
  const int c = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;  // within [78][256] (+78 bias entries)
  const int nch = (grp_count[c] + CHUNK - 1) / CHUNK, c0 = chunk_start[c];
  const int nchunks = totals[2];
  if (e < kCell * KD) {
    float s = 0.f;
    for (int q = 0; q < nch; ++q)
      if (hb_run_end(c0 + q, c0 + nch, nchunks, bwd_grid))
        s += dWp[(size_t)(c0 + q) * kCell * KD + e];
    dW[(size_t)c * kCell * KD + e] = s;
  } else if (e < kCell * KD + kCell) {
    const int n = e - kCell * KD;
    float s = 0.f;
    for (int q = 0; q < nch; ++q)
      if (hb_run_end(c0 + q, c0 + nch, nchunks, bwd_grid)) s += dbp[(size_t)(c0 + q) * kCell + n];
    db[c * kCell + n] = s;
  }
}

// the active bit of cell c in frame row ab (head_count's bitmap)
__device__ __forceinline__ bool abit(const uint32_t* ab, int c, int S) {
  return c < S && ((ab[c >> 5] >> (c & 31)) & 1u);
}

// dX[f][:] = sum over active cells c of dXp[pidx[f][c]][:]; one wave per frame
__global__ __launch_bounds__(256) void head_dx_gather_kernel(const bf16* __restrict__ dXp,
                                                             const int* __restrict__ pidx,
                                                             const uint32_t* __restrict__ abits,
                                                             int F, int S,
                                                             float* __restrict__ dX) {
  // one wave per frame: the active cells (~1 %) of 64 from the bitmap, their pair indices,
  // and only their dXp rows
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= F) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int* pr = pidx + (size_t)f * S;
  const uint32_t* ab = abits + (size_t)f * abits_words(S);
  for (int c0 = 0; c0 < S; c0 += 64) {
    const int p = abit(ab, c0 + lane, S) ? pr[c0 + lane] : -1;
    uint64_t m = __ballot(p >= 0);
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      const int pp = __shfl(p, b);
      const uint2 v = ((const uint2*)(dXp + (size_t)pp * KD))[lane];  // 4 bf16
      acc.x += __uint_as_float(v.x << 16); acc.y += __uint_as_float(v.x & 0xFFFF0000u);
      acc.z += __uint_as_float(v.y << 16); acc.w += __uint_as_float(v.y & 0xFFFF0000u);
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
__global__ __launch_bounds__(256) void head_dx_value_kernel(const bf16* __restrict__ dXp,
                                                            const int* __restrict__ pidx,
                                                            const uint32_t* __restrict__ abits,
                                                            int F,
                                                            int S, const float* __restrict__ dv,
                                                            const bf16* __restrict__ h,
                                                            const float* __restrict__ wc, int R,
                                                            bf16* __restrict__ dh,
                                                            float* __restrict__ partial) {
  __shared__ float red[4][KD + 4];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float4 w = ((const float4*)wc)[lane];
  float sw[4] = {0.f, 0.f, 0.f, 0.f}, sb = 0.f;
  // the next frame's dv, h and pair-index row are loaded before this frame's gathers (one
  // wave walks ~R / (4 * grid) frames: without it every frame paid two dependent HBM trips)
  constexpr int kMaxCh = MAX_S / 64;
  const int nch = (S + 63) / 64;
  const int stride = gridDim.x * 4;
  // The bitmap words run one frame further ahead: a frame's pair indices are loaded (active
  // lanes only) from bits that already arrived, so no iteration waits on two dependent trips.
  float dn = 0.f;
  uint2 hn = make_uint2(0, 0);
  int pn[kMaxCh];
  uint32_t wn[kMaxCh];  // bitmap word of cell q * 64 + lane, frame r + stride
  auto fetch_bits = [&](int r) {
    const uint32_t* ab = abits + (size_t)r * abits_words(S);
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q)
      wn[q] = (r < F && q < nch && q * 64 + lane < S) ? ab[(q * 64 + lane) >> 5] : 0u;
  };
  auto fetch = [&](int r) {  // uses wn = r's bitmap words
    dn = dv[r];
    hn = ((const uint2*)(h + (size_t)r * KD))[lane];
    const int* pr = pidx + (size_t)r * S;
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q)
      pn[q] = ((wn[q] >> (lane & 31)) & 1u) ? pr[q * 64 + lane] : -1;
  };
  const int rfirst = blockIdx.x * 4 + wave;
  if (rfirst < R) {
    fetch_bits(rfirst);
    fetch(rfirst);
    if (rfirst + stride < R) fetch_bits(rfirst + stride);
  }
  for (int r = rfirst; r < R; r += stride) {
    const float d = dn;
    const uint2 hv = hn;
    int pc[kMaxCh];
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q) pc[q] = pn[q];
    if (r + stride < R) {
      fetch(r + stride);
      if (r + 2 * stride < R) fetch_bits(r + 2 * stride);
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < kMaxCh; ++q) {
      if (q >= nch) break;
      const int p = pc[q];
      uint64_t m = __ballot(p >= 0);
      // up to 4 pair rows in flight per trip (one dependent HBM latency per 4 pairs instead
      // of per pair), added in the same order
      while (m) {
        int pp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pp[j] = -1;
          if (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            pp[j] = __shfl(p, b);
          }
        }
        uint2 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = pp[j] >= 0 ? ((const uint2*)(dXp + (size_t)pp[j] * KD))[lane]  // 4 bf16
                            : make_uint2(0u, 0u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (pp[j] < 0) break;
          acc.x += __uint_as_float(v[j].x << 16); acc.y += __uint_as_float(v[j].x & 0xFFFF0000u);
          acc.z += __uint_as_float(v[j].y << 16); acc.w += __uint_as_float(v[j].y & 0xFFFF0000u);
        }
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

// abits [F][(S + 31) / 32] uint32: the active-cell bitmap the consumers of pidx read, written
// here from the masks (abits_given 0) or already written by the acting step (1: the masks are
// not read at all)
extern "C" int mbk_head_compact(const uint32_t* mask, int F, int S, int* cnt, int* off,
                                int* grp_start, int* grp_count, int* unit_cell, int* unit_row,
                                int* chunk_cell, int* chunk_row, int* chunk_start,
                                int* totals, int* pairs, int* pidx, uint32_t* abits,
                                int abits_given, uint8_t* action_zero, float* cell_lp,
                                float* cell_ent, hipStream_t stream) {
  if (S > MAX_S) return (int)hipErrorInvalidValue;
  const int FB = mbk_head_fb(F);
  const int nfb = (F + FB - 1) / FB;
  dim3 g1(nfb, (S + 255) / 256);
  if (!abits) return (int)hipErrorInvalidValue;
  if (abits_given)
    hipLaunchKernelGGL(head_count_bits_kernel, g1, dim3(256), 0, stream, abits, F, S, FB, cnt);
  else
    hipLaunchKernelGGL(head_count_kernel, g1, dim3(256), 0, stream, mask, F, S, FB, cnt, abits);
  // per-cell totals go to grp_count (overwritten with the same values by the scan)
  hipLaunchKernelGGL(head_cell_scan_kernel, dim3(S), dim3(256), 0, stream, cnt, nfb, off,
                     grp_count);
  hipLaunchKernelGGL(head_scan_kernel, dim3(1), dim3(1024), 0, stream, grp_count, S, grp_start,
                     grp_count, unit_cell, unit_row, chunk_cell, chunk_row, chunk_start, totals);
  hipLaunchKernelGGL(head_scatter_kernel, g1, dim3(256), 0, stream, abits, F, S, FB, off,
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

extern "C" int mbk_head_pair_rowsum(const int* pidx, const uint32_t* abits, int F, int S,
                                    const float* plp, const float* pent, float* logp, float* ent,
                                    hipStream_t stream) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(head_pair_rowsum_kernel, dim3((F + 255) / 256), dim3(256), 0, stream, pidx,
                     abits, F, S, plp, pent, logp, ent);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_bwd(const void* X, const void* Wp, const void* WpT, const float* bp,
                            const uint32_t* mask, const uint8_t* action, const int* pairs,
                            const int* grp_start, const int* grp_count, const int* chunk_cell,
                            const int* chunk_row, const int* chunk_start, const int* totals,
                            const float* g_logp, const float* g_ent, int S, int grid, void* dXp,
                            float* dWp, float* dbp, float* dW, float* db, const float* stats,
                            hipStream_t stream) {
  int bwd_grid = 1;
  {
    static int cus = 0;
    static uint64_t* hb_stamps = nullptr;
    if (!cus) {
      int dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (cus <= 0) cus = 256;
      hipFuncSetAttribute((const void*)head_bwd2_kernel<false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, HB_LDS);
      hipFuncSetAttribute((const void*)head_bwd2_kernel<true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, HB_LDS);
      if (getenv("MBK_HB_STAMPS")) {
        hipMalloc(&hb_stamps, (size_t)cus * 64 * 8);
        hipMemset(hb_stamps, 0, (size_t)cus * 64 * 8);
      }
    }
    // one 158 KB workgroup per CU; the caller's grid (chunk count bound) caps it
    const int g2 = std::max(1, std::min(grid, cus));
    bwd_grid = g2;
    // stats (mbk_head_score's, same batch and weights): the per-logit epilogue
    hipLaunchKernelGGL(stats ? head_bwd2_kernel<true> : head_bwd2_kernel<false>, dim3(g2),
                       dim3(64 * HB_NW), HB_LDS, stream, (const bf16*)X, (const bf16*)Wp, bp,
                       mask, action, pairs, grp_start, grp_count, chunk_cell, chunk_row, totals,
                       g_logp, g_ent, S, (bf16*)dXp, dWp, dbp, hb_stamps, stats);
    if (hb_stamps) {  // per-phase mean over workgroups and their tiles 1..7 (us)
      std::vector<uint64_t> h((size_t)g2 * 64);
      hipMemcpyAsync(h.data(), hb_stamps, h.size() * 8, hipMemcpyDeviceToHost, stream);
      hipStreamSynchronize(stream);
      double acc[8] = {0};
      int n = 0;
      for (int b = 0; b < g2; ++b)
        for (int t = 1; t < 8; ++t) {
          const uint64_t* r = &h[((size_t)b * 8 + t) * 8];
          if (!r[0] || !r[7]) continue;
          for (int k = 0; k < 7; ++k) acc[k] += (double)(r[k + 1] - r[k]) * 0.01;
          ++n;
        }
      fprintf(stderr, "head_bwd2 phases (us, %d tiles): store+W %.2f | loads+Z %.2f | dZ %.2f | "
              "B2 %.2f | dX %.2f | dW %.2f | end %.2f\n", n, acc[0] / n, acc[1] / n, acc[2] / n,
              acc[3] / n, acc[4] / n, acc[5] / n, acc[6] / n);
      hipMemsetAsync(hb_stamps, 0, h.size() * 8, stream);
    }
  }
  dim3 g2((kCell * KD + kCell + 255) / 256, S);
  hipLaunchKernelGGL(head_dw_reduce_kernel, g2, dim3(256), 0, stream, dWp, dbp, chunk_start,
                     grp_count, totals, bwd_grid, S, dW, db);
  return (int)hipGetLastError();
}

// Learner scoring of the compacted pairs (head_score_kernel): pair-indexed log-prob and
// entropy (pent may be null) of the given actions over the backward's chunk list, one 127 KB
// workgroup per CU (no host sync: the chunk count is read on the device). stats (or null):
// per pair 16 floats {lse[7], H[7], 0, 0} for mbk_head_bwd's epilogue.
extern "C" int mbk_head_score(const void* X, const void* Wp, const float* bp,
                              const uint32_t* mask, const uint8_t* action, const int* pairs,
                              const int* grp_start, const int* grp_count, const int* chunk_cell,
                              const int* chunk_row, const int* totals, int S, float* plp,
                              float* pent, float* stats, hipStream_t stream) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    hipFuncSetAttribute((const void*)head_score_kernel,
                        hipFuncAttributeMaxDynamicSharedMemorySize, HS_LDS);
  }
  hipLaunchKernelGGL(head_score_kernel, dim3(cus), dim3(64 * HS_NW), HS_LDS, stream,
                     (const bf16*)X, (const bf16*)Wp, bp, mask, action, pairs, grp_start,
                     grp_count, chunk_cell, chunk_row, totals, S, plp, pent, stats);
  return (int)hipGetLastError();
}

extern "C" int mbk_head_dx_gather(const void* dXp, const int* pidx, const uint32_t* abits, int F,
                                  int S, float* dX, hipStream_t stream) {
  hipLaunchKernelGGL(head_dx_gather_kernel, dim3((F + 3) / 4), dim3(256), 0, stream,
                     (const bf16*)dXp, pidx, abits, F, S, dX);
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
extern "C" int mbk_head_dx_value(const void* dXp, const int* pidx, const uint32_t* abits, int F,
                                 int S, const float* dv, const void* h, const float* wc, int R,
                                 void* dh, float* partial, int parts, hipStream_t stream) {
  if (R <= 0) return 0;
  if (F > R || parts < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(head_dx_value_kernel, dim3(parts), dim3(256), 0, stream, (const bf16*)dXp,
                     pidx, abits, F, S, dv, (const bf16*)h, wc, R, (bf16*)dh, partial);
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
  // three 2-wave workgroups per CU (the LDS logit tiles allow three): ~1500 waves for the
  // ~800 64-pair jobs of a settled 8192-env step
  hipLaunchKernelGGL(head_act_kernel, dim3(std::max(1, cus * 6 / HA_NW)), dim3(64 * HA_NW), 0,
                     stream, a);
  return (int)hipGetLastError();
}

extern "C" int mbk_act_trunk(const MbkActModel* m, const MbkActStep* s, hipStream_t stream);

// the whole acting step: A (decode + trunk + network.5 + critic) then B (sample + finale)
extern "C" int mbk_act_step(const MbkActModel* m, const MbkActStep* s, hipStream_t stream) {
  const int rc = mbk_act_trunk(m, s, stream);
  if (rc) return rc;
  return mbk_act_head(m, s, stream);
}
