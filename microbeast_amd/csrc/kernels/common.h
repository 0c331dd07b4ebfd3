// Device-side helpers shared by the microbeast_amd HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define MBK_WAVE 64

// Learner persistent grids: resident workgroups per CU capped at mbk_occ_cap(0) (forward
// kernels) / mbk_occ_cap(1) (backward kernels), 0 = no cap. The acting kernels (215-256
// VGPRs) cannot co-reside with two learner workgroups per CU (2 waves x ~224 VGPRs per SIMD)
// and wait for the learner kernel's end; one backward workgroup per CU leaves them a slot
// (profile 45). Default: no caps; the GPU actor runtime sets the backward cap to 1 for the
// IMPALA-flat model (config.bwd_occupancy; the learner-heavy GridNet / deep configs keep none)
// (mbk_set_learner_occupancy, conv.hip: before the first learner allocation only, since the
// partial-buffer sizes -- the *_parts queries -- follow it).
int mbk_occ_cap(int bwd);
inline int mbk_occ_f(int per) { const int c = mbk_occ_cap(0); return c > 0 && per > c ? c : per; }
inline int mbk_occ_b(int per) { const int c = mbk_occ_cap(1); return c > 0 && per > c ? c : per; }

// Dynamic work queues for the learner's persistent kernels (round 6). A persistent grid walking
// its items by a static stride (blockIdx.x, + gridDim.x, ...) lasts as long as its latest-
// starting workgroup: under the GPU actor runtime an acting launch holds a CU's slots for
// 0.2-1 ms, so some of the grid's workgroups start that much later and still own a full share.
// With a queue, each wave takes its next items (16-item chunks) from a counter, so early waves
// take more and the kernel ends when the work does. The counter pair {next ticket, waves done}
// lives per (stream, call site) and resets itself: the last wave to finish zeroes it for the
// next launch on that stream (launches on one stream are ordered). The forward kernels' items
// only write their own outputs: bit-identical in any order. The stage-0 weight gradient
// (kQueueWgrad, workgroup-level: conv.hip) sums a run-dependent set of rounds per partial row:
// reproducible up to fp32 summation order (its site can be switched off:
// mbk_set_work_queue_site).
// mbk_work_queue: nullptr (static striding) while queues are off, or the stream is capturing a
// graph before its counters exist.
int* mbk_work_queue(hipStream_t stream, int site);
constexpr int kQueueConv0 = 0, kQueueResFwd16 = 1, kQueueBlk32 = 2, kQueuePoolConv4 = 3,
              kQueueWgrad = 4, kQueueSites = 8;

namespace mbk {

// the wave's next item: lane 0 takes a ticket (a vector atomic: the branch is per lane)
__device__ __forceinline__ int wave_ticket(int* q) {
  int t = 0;
  if ((threadIdx.x & 63) == 0)
    t = __hip_atomic_fetch_add(q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __shfl(t, 0, 64);
}
// Tickets hand out chunks of kQueueChunk items (one atomic per image on one address serialised
// in L2: 26 vs 17 ms per learner update): the wave's next item after `it` inside its chunk
// [.., cend), else the first of a new chunk (>= n: no work left; cend is updated)
constexpr int kQueueChunk = 16;
__device__ __forceinline__ int wave_next_item(int* q, int it, int& cend, int n) {
  if (it + 1 < cend) return it + 1;
  const int t = wave_ticket(q) * kQueueChunk;
  cend = min(n, t + kQueueChunk);
  return t;
}
// after the wave's last ticket (one past the work): the grid's last such wave resets the queue
__device__ __forceinline__ void wave_queue_done(int* q, int total_waves) {
  if ((threadIdx.x & 63) == 0 &&
      __hip_atomic_fetch_add(q + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total_waves - 1) {
    __hip_atomic_store(q, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// microRTS GridMode per-cell action components (reference model.py:168,
// libs/utils.py:40-44): nvec = [6,4,4,4,4,7,49], 78 logits per cell.
constexpr int kComps = 7;
constexpr int kCell = 78;
__host__ __device__ constexpr int seg_off(int k) {
  return k == 0 ? 0 : k == 1 ? 6 : k == 2 ? 10 : k == 3 ? 14 : k == 4 ? 18 : k == 5 ? 22
       : k == 6 ? 29 : 78;
}

__device__ __forceinline__ bool mask_bit(const uint32_t m[3], int j) {
  // selects, not m[j >> 5]: a runtime index would put the caller's m[] in scratch memory
  const uint32_t w = j < 32 ? m[0] : (j < 64 ? m[1] : m[2]);
  return (w >> (j & 31)) & 1u;
}
// the same on three named words (the compiler folded the array form's selects back into a
// runtime index -- a scratch store + load per call -- inside cell_forward's segment loops)
__device__ __forceinline__ bool mask_bit3(uint32_t m0, uint32_t m1, uint32_t m2, int j) {
  const uint32_t w = j < 32 ? m0 : (j < 64 ? m1 : m2);
  return (w >> (j & 31)) & 1u;
}

// ------------------------------------------------------------------ Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    u32x4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t x) {  // (0,1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// ------------------------------------------------------------------ cell epilogue
// One microRTS cell: 78 logits z (fp32, any stride-1 storage), 78 mask bits,
// 7 categorical segments. Semantics match the reference CategoricalMasked
// (model.py:33-52): masked logits are replaced by -1e8, so a masked entry has
// probability 0 and contributes 0 to the entropy; a fully-masked segment has
// log-prob 0 and entropy 0 in fp32 (as in the reference); we sample index 0
// there (the env ignores it — no unit to command).
//
// mode 0 = score the given actions; mode 1 = sample (writes actions).
template <typename ZPtr>
__device__ __forceinline__ void cell_forward(const ZPtr z, const uint32_t m[3], uint8_t* act,
                                             bool sample, const float u[kComps], float* logp_out,
                                             float* ent_out) {
  uint32_t m0 = m[0], m1 = m[1], m2 = m[2];
  asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));  // opaque: no array to re-index
  float lp = 0.f, ent = 0.f;
#pragma unroll
  for (int k = 0; k < kComps; ++k) {
    const int off = seg_off(k), n = seg_off(k + 1) - off;
    float mx = -INFINITY;
    for (int j = 0; j < n; ++j)
      if (mask_bit3(m0, m1, m2, off + j)) mx = fmaxf(mx, (float)z[off + j]);
    if (mx == -INFINITY) {  // fully masked segment
      if (sample) act[k] = 0;
      continue;
    }
    float s = 0.f, sz = 0.f;
    for (int j = 0; j < n; ++j)
      if (mask_bit3(m0, m1, m2, off + j)) {
        const float zj = (float)z[off + j];
        const float e = __expf(zj - mx);
        s += e;
        sz += e * zj;
      }
    const float inv = 1.f / s;
    const float lse = mx + __logf(s);
    ent += lse - sz * inv;  // -sum p log p = lse - sum p z
    int a;
    if (sample) {
      const float target = u[k] * s;
      float c = 0.f;
      a = -1;
      int last = 0;
      for (int j = 0; j < n; ++j)
        if (mask_bit3(m0, m1, m2, off + j)) {
          last = j;
          c += __expf((float)z[off + j] - mx);
          if (a < 0 && c >= target) a = j;
        }
      if (a < 0) a = last;
      act[k] = (uint8_t)a;
    } else {
      a = act[k];
    }
    const bool valid = a < n && mask_bit3(m0, m1, m2, off + a);
    lp += (valid ? (float)z[off + a] : -1e8f) - lse;
  }
  *logp_out = lp;
  *ent_out = ent;
}

// dL/dz for one cell given dL/dlogp (gl) and dL/dentropy (ge) of its sample.
//   valid j: gl*(1[j==a] - p_j) - ge*p_j*(log p_j + H_seg);  masked j: 0
template <typename ZPtr, typename DPtr>
__device__ __forceinline__ void cell_backward(const ZPtr z, const uint32_t m[3],
                                              const uint8_t* act, float gl, float ge, DPtr dz) {
#pragma unroll
  for (int k = 0; k < kComps; ++k) {
    const int off = seg_off(k), n = seg_off(k + 1) - off;
    float mx = -INFINITY;
    for (int j = 0; j < n; ++j)
      if (mask_bit(m, off + j)) mx = fmaxf(mx, (float)z[off + j]);
    if (mx == -INFINITY) {
      for (int j = 0; j < n; ++j) dz[off + j] = 0.f;
      continue;
    }
    float s = 0.f, sz = 0.f;
    for (int j = 0; j < n; ++j)
      if (mask_bit(m, off + j)) {
        const float zj = (float)z[off + j];
        const float e = __expf(zj - mx);
        s += e;
        sz += e * zj;
      }
    const float inv = 1.f / s;
    const float lse = mx + __logf(s);
    const float H = lse - sz * inv;
    const int a = act[k];
    for (int j = 0; j < n; ++j) {
      float d = 0.f;
      if (mask_bit(m, off + j)) {
        const float zj = (float)z[off + j];
        const float p = __expf(zj - mx) * inv;
        const float logp = zj - lse;
        d = gl * ((j == a ? 1.f : 0.f) - p) - ge * p * (logp + H);
      }
      dz[off + j] = d;
    }
  }
}

// ------------------------------------------------------------------ barriers
// Workgroup barrier that orders LDS only: the fences are restricted to the local address space,
// so no s_waitcnt vmcnt(0) is emitted and the waves' global stores stay in flight across it
// (__syncthreads() drains every outstanding global access of every wave first). For phases
// whose cross-wave hand-off is through LDS and whose global writes nobody in the workgroup
// reads back.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------------------------------------------ critic order
// The critic value v = wc . f + bc from the MFMA C layout of network.5 (lane (G, li) holds
// hidden units 4G .. 4G+3 of a 16-unit block for row li): every FC kernel (fc.hip fc_fwd /
// fc_fwd_rb, trunk.hip trunk_fc and the acting tile's FC) sums in THIS order, so the graph,
// fused-acting and learner values agree bit for bit: per block, the lane's 4 products as an
// explicit fma chain from 0 (llvm.fmuladd fuses differently per kernel), then the xor-16 /
// xor-32 butterfly over the lane groups (crit_block); then the blocks in hidden order, then
// the bias (crit_sum over the blocks' partials).
__device__ __forceinline__ float crit_block(const float hv[4], const float w[4]) {
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) q = __builtin_fmaf(hv[i], w[i], q);
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  return q;
}
// part[hb * stride] for hb = 0 .. nb-1, in order, then + bc
__device__ __forceinline__ float crit_sum(const float* part, int nb, int stride, float bc) {
  float v = part[0];
  for (int hb = 1; hb < nb; ++hb) v += part[hb * stride];
  return v + bc;
}

// ------------------------------------------------------------------ reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------ pooled epilogue
// max_pool2d(3, 2, 1) of the workgroup's conv outputs staged in LDS (otile [(im*H+y)*W+x]
// [OSTR] bf16) -> pooled y + per-channel argmax (ky*3+kx, first maximum in scan order as
// ATen). A thread owns one (image, pooled column, 4 channels) and walks its pooled rows top to
// bottom, separably: an input row's 3-wide horizontal max (first maximising kx, strict >) is
// computed once and shared by the two windows containing the row, and the vertical pass keeps
// the first maximising ky -- so the index is the smallest maximising tap, 6 tap reads per
// output instead of 9. Out-of-map taps read as -inf; the centre (2 oy, 2 ox) is always inside.
// Index maths by float reciprocals (exact: pixel counts are tiny, see conv.hip index_math_ok).
// Shared by conv.hip (conv_fwd / conv0_row epilogues) and resblock.hip (fused stage conv).
template <int COUT, int OSTR>
struct PoolHRow {
  float m[4];
  int k[4];
};

template <int COUT, int OSTR, int NT>
__device__ __forceinline__ void pool_tile(const __hip_bfloat16* __restrict__ otile, int H, int W, int nimg,
                                          size_t obase, __hip_bfloat16* __restrict__ y,
                                          uint8_t* __restrict__ pool_idx, int tid) {
  const int Ho = (H + 1) >> 1, Wo = (W + 1) >> 1;
  constexpr int C4 = COUT / 4;
  const int tot = nimg * Wo * C4;
  const float inv_wo = 1.f / (float)Wo;
  using HRow = PoolHRow<COUT, OSTR>;
  for (int e = tid; e < tot; e += NT) {
    const int c4 = e % C4, col = e / C4;
    const int im = (int)(((float)col + 0.5f) * inv_wo), ox = col - im * Wo;
    const __hip_bfloat16* base = otile + ((size_t)im * H * W + 2 * ox) * OSTR + 4 * c4;
    const bool lo_ok = ox > 0, hi_ok = 2 * ox + 1 < W;
    auto hrow = [&](int yy) {  // input row yy, x = 2 ox - 1 .. 2 ox + 1
      HRow h;
      const __hip_bfloat16* b = base + yy * W * OSTR;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const bool ok = kx == 1 || (kx == 0 ? lo_ok : hi_ok);
        const uint2 u = *(const uint2*)(b + (ok ? (kx - 1) * OSTR : 0));
        float v[4];
        v[0] = __uint_as_float(u.x << 16);
        v[1] = __uint_as_float(u.x & 0xFFFF0000u);
        v[2] = __uint_as_float(u.y << 16);
        v[3] = __uint_as_float(u.y & 0xFFFF0000u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!ok) v[j] = -INFINITY;
          if (kx == 0 || v[j] > h.m[j]) { h.m[j] = v[j]; h.k[j] = kx; }
        }
      }
      return h;
    };
    HRow top;
#pragma unroll
    for (int j = 0; j < 4; ++j) { top.m[j] = -INFINITY; top.k[j] = 0; }
    for (int oy = 0; oy < Ho; ++oy) {
      const HRow mid = hrow(2 * oy);
      HRow bot;
      if (2 * oy + 1 < H) {
        bot = hrow(2 * oy + 1);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) { bot.m[j] = -INFINITY; bot.k[j] = 0; }
      }
      float mx[4];
      uint32_t am = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int ix = top.k[j];   // ky = 0; an out-of-map top row never wins (mid is inside)
        mx[j] = top.m[j];
        if (mid.m[j] > mx[j]) { mx[j] = mid.m[j]; ix = 3 + mid.k[j]; }
        if (bot.m[j] > mx[j]) { mx[j] = bot.m[j]; ix = 6 + bot.k[j]; }
        am |= (uint32_t)ix << (8 * j);
      }
      const size_t oi = obase + ((size_t)(im * Ho + oy) * Wo + ox) * COUT + 4 * c4;
      // the maxima are loaded bf16 values: their float bits carry the bf16 exactly
      *(uint2*)(y + oi) =
          make_uint2((__float_as_uint(mx[0]) >> 16) | (__float_as_uint(mx[1]) & 0xFFFF0000u),
                     (__float_as_uint(mx[2]) >> 16) | (__float_as_uint(mx[3]) & 0xFFFF0000u));
      if (pool_idx) *(uint32_t*)(pool_idx + oi) = am;
      top = bot;
    }
  }
}

}  // namespace mbk
