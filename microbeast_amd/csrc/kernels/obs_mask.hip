// GPU-side observation decode + action-mask generation, and env-action packing.
//
// The reference ships, per env step, a float32 (s,s,27) observation and a
// (s*s*78) uint8 mask from the JVM to Python (env_packer.py:8-14, 39-40, 87):
// 47 KB per 16x16 frame. The native engine ships 16-bit cell codes (512 B) plus
// the player's resource count and derives the 78-bit mask of every cell on the
// GPU with exactly the simulator's rules (include/microrts_rules.h), so the CPU
// never builds masks and PCIe carries 8x less. Actions go back as one packed
// 16-bit word per cell (the chosen type's parameter only).
#include "../include/mbk_api.h"
#include "../include/microrts_rules.h"
#include "common.h"
#include "decode.h"

namespace {

using namespace mbr;
using mbk::cell_mask;

// Per-step sparse-head bookkeeping for acting (BUCKET): every active (env, cell) pair is
// appended to its cell's bucket (bucket[c * E + slot], slot from an atomic counter; order
// inside a bucket is irrelevant for sampling: the RNG is keyed by (frame, cell)), and the
// outputs of inactive cells (action, cell log-prob) are zeroed here instead of by a
// separate pass. head.hip's head_units_kernel turns the counters into the unit list.
struct Buckets {
  int* cnt;        // [S] (zero on entry; reset by head_units_kernel)
  int* bucket;     // [S][E]
  float* cell_lp;  // [E*S]
  uint8_t* action; // [E*S*7]
};

// One WAVE per env, EPW envs per workgroup, persistent over env groups (grid sized
// to the device). A lane owns Q = ceil(S/64) consecutive cells, so an env's obs words and
// mask triples leave as contiguous 16-byte vector stores (Q = 4 at 16x16: one uint4 of obs
// and three uint4 of mask per lane) and the inactive-output zeroing is a few wave-wide
// 16-byte stores. The previous form (one 256-thread workgroup per env, one cell per thread,
// 3 scalar mask stores per cell) ran at ~0.4-0.6 TB/s: 8192 short workgroups per step, each
// a global-load -> barrier -> store chain (profiles/16: ~99 us per 8192-env step).
//
// BUCKET: the (env, cell) pairs are first counted per cell in LDS (LDS atomics) and listed in
// LDS; after the workgroup's last env group, ONE global atomicAdd per (workgroup, active
// cell) reserves the workgroup's range of that cell's bucket. Unit start positions are the
// same in every env, so direct per-pair global atomics all hit a handful of counters
// (8192-way contention on the base cells: the kernel ran at 109 us, profile 20).
constexpr int kEnvsPerWG = 4;
constexpr int kBucketEPW = 8;          // envs per pass of the bucketing variant (512 threads)
constexpr int kBucketGroupsPerWG = 2;  // passes per workgroup before its bucket flush
constexpr int kMaxLocalPairs = 2048;   // LDS pair list; overflow takes the direct atomic path

template <bool BUCKET>
__global__ __launch_bounds__(512) void decode_obs_mask_kernel(const uint16_t* __restrict__ codes,
                                                              const int32_t* __restrict__ res,
                                                              int E, int H, int W,
                                                              uint32_t* __restrict__ obs,
                                                              uint32_t* __restrict__ mask,
                                                              Buckets bk) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_codes[];
  constexpr int EPW = BUCKET ? kBucketEPW : kEnvsPerWG;
  const int S = H * W;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint16_t* cs = smem_codes + wave * S;
  // BUCKET LDS: per-cell counts, then the pair list (cell << 19 | local slot, env)
  int* lcnt = (int*)(smem_codes + ((EPW * S + 7) & ~7));
  int* npairs = lcnt + S;
  int2* pairs = (int2*)(npairs + 2);
  const int Q = (S + 63) >> 6;  // cells per lane
  const int c0 = lane * Q, c1 = min(S, c0 + Q);
  const bool vec4 = Q == 4 && (S & 3) == 0;  // 16x16: whole-lane vector stores
  const int ngroups = (E + EPW - 1) / EPW;
  if (BUCKET) {
    for (int c = threadIdx.x; c < S; c += blockDim.x) lcnt[c] = 0;
    if (threadIdx.x == 0) *npairs = 0;
    __syncthreads();
  }
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {  // uniform trip count
    const int e = grp * EPW + wave;
    const bool live = e < E;
    if (live) {
      const uint16_t* ce = codes + (size_t)e * S;
      if (vec4) *(uint2*)(cs + c0) = *(const uint2*)(ce + c0);
      else
        for (int c = lane; c < S; c += 64) cs[c] = ce[c];  // coalesced
    }
    __syncthreads();
    if (live) {
      const int r = res[e];
      uint32_t ob[4], mk[12];
      // 16x16: 4 consecutive cells per lane (one 16-byte store each); other sizes: cells
      // lane, lane + 64, ... so a wave's obs / mask stores are coalesced (the contiguous split
      // strided them Q cells apart: 9 at 24x24)
      const int cstart = vec4 ? c0 : lane, cend = vec4 ? c1 : S, cstep = vec4 ? 1 : 64;
      for (int c = cstart; c < cend; c += cstep) {
        uint32_t w[3];
        cell_mask(cs, c, H, W, r, w);
        const uint32_t bits = code_bits(cs[c]);
        if (vec4) {
          const int j = c - c0;
          ob[j] = bits;
          mk[3 * j] = w[0]; mk[3 * j + 1] = w[1]; mk[3 * j + 2] = w[2];
        } else {
          obs[(size_t)e * S + c] = bits;
          uint32_t* m = mask + ((size_t)e * S + c) * 3;
          m[0] = w[0]; m[1] = w[1]; m[2] = w[2];
        }
        if (BUCKET && (w[0] | w[1] | w[2])) {
          const int i = atomicAdd(npairs, 1);
          if (i < kMaxLocalPairs) {
            pairs[i] = make_int2((c << 19) | atomicAdd(&lcnt[c], 1), e);
          } else {  // list full: direct global slot
            const int slot = atomicAdd(&bk.cnt[c], 1);
            bk.bucket[(size_t)c * E + slot] = e;
          }
        }
      }
      if (vec4) {
        *(uint4*)(obs + (size_t)e * S + c0) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
        uint4* m4 = (uint4*)(mask + ((size_t)e * S + c0) * 3);
        m4[0] = make_uint4(mk[0], mk[1], mk[2], mk[3]);
        m4[1] = make_uint4(mk[4], mk[5], mk[6], mk[7]);
        m4[2] = make_uint4(mk[8], mk[9], mk[10], mk[11]);
      }
      if (BUCKET) {
        // every cell's log-prob and 7 action bytes start at zero; the sparse head overwrites
        // the active cells later in stream order (whole-env 16-byte zeroing: the env's S*7
        // action bytes and S floats are contiguous)
        if ((S & 15) == 0 && (((uintptr_t)bk.action | (uintptr_t)bk.cell_lp) & 15) == 0) {
          uint4* act4 = (uint4*)(bk.action + (size_t)e * S * 7);
          uint4* lp4 = (uint4*)(bk.cell_lp + (size_t)e * S);
          for (int i = lane; i < S * 7 / 16; i += 64) act4[i] = make_uint4(0, 0, 0, 0);
          for (int i = lane; i < S / 4; i += 64) lp4[i] = make_uint4(0, 0, 0, 0);
        } else {
          for (int i = lane; i < S * 7; i += 64) bk.action[(size_t)e * S * 7 + i] = 0;
          for (int i = lane; i < S; i += 64) bk.cell_lp[(size_t)e * S + i] = 0.f;
        }
      }
    }
    __syncthreads();  // cs reused by the next group
  }
  if (BUCKET) {
    // one global reservation per active cell of this workgroup; lcnt becomes the base
    for (int c = threadIdx.x; c < S; c += blockDim.x) {
      const int n = lcnt[c];
      if (n > 0) lcnt[c] = atomicAdd(&bk.cnt[c], n);
    }
    __syncthreads();
    const int np = min(*npairs, kMaxLocalPairs);
    for (int i = threadIdx.x; i < np; i += blockDim.x) {
      const int2 pr = pairs[i];
      const int c = pr.x >> 19, slot = pr.x & 0x7FFFF;
      bk.bucket[(size_t)c * E + lcnt[c] + slot] = pr.y;
    }
  }
}

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

int decode_grid(int E) {
  const int ngroups = (E + kEnvsPerWG - 1) / kEnvsPerWG;
  return max(1, min(ngroups, device_cus() * 8));  // 8 resident 256-thread workgroups per CU
}

int bucket_grid(int E) {
  const int ngroups = (E + kBucketEPW - 1) / kBucketEPW;
  return max(1, (ngroups + kBucketGroupsPerWG - 1) / kBucketGroupsPerWG);
}

size_t bucket_smem(int S) {
  return (size_t)((kBucketEPW * S + 7) & ~7) * 2 + (size_t)(S + 2) * 4 + (size_t)kMaxLocalPairs * 8;
}

__global__ __launch_bounds__(256) void pack_env_actions_kernel(const uint8_t* __restrict__ act,
                                                               int64_t ncells,
                                                               uint16_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ncells;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t a[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) a[k] = act[i * 7 + k];
    out[i] = pack_env_action(a);
  }
}

// Policy-step finale in one launch (one wave per env): the env's log-prob = sum of its
// cells' log-probs in cell order (the fused step's finale order, bit-identical),
// its cells' 7 action bytes packed into the 16-bit codes the env reads, and the sampler's
// step counter advanced (block 0) -- row_sum_rng + pack_env_actions without the second
// launch (each dependent launch of the policy graph waits for CUs behind the learner).
__global__ __launch_bounds__(256) void row_sum_pack_kernel(const float* __restrict__ cell_lp,
                                                           int64_t rows, int cols,
                                                           float* __restrict__ logp,
                                                           uint64_t* __restrict__ rng,
                                                           const uint8_t* __restrict__ act,
                                                           uint16_t* __restrict__ act16,
                                                           int* __restrict__ cnt, int ncnt) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (rng && blockIdx.x == 0 && threadIdx.x == 0) rng[1] += 1;
  // the decode kernel's per-cell bucket counters, read by the head launch before this one
  if (cnt && blockIdx.x == 0)
    for (int c = threadIdx.x; c < ncnt; c += blockDim.x) cnt[c] = 0;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  // the cells' log-probs summed in cell order: the order the fused step's finale (head.hip
  // head_act_kernel) sums an env's active cells in. Zero entries (inactive cells) are skipped:
  // adding +-0 to the running sum is exact, so only the few non-zero cells are added serially
  // (adding all 576 cells of a 24x24 row one by one took 52 us per 8192-env step)
  float s = 0.f;
  for (int c0 = 0; c0 < cols; c0 += 64) {
    const float v = c0 + lane < cols ? cell_lp[r * cols + c0 + lane] : 0.f;
    uint64_t nz = __ballot(v != 0.f);
    while (nz) {
      const int q = __builtin_ctzll(nz);
      nz &= nz - 1;
      s += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), q));
    }
  }
  if (lane == 0) logp[r] = s;
  for (int c = lane; c < cols; c += 64) {
    const int64_t i = r * cols + c;
    uint8_t a[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) a[k] = act[i * 7 + k];
    act16[i] = pack_env_action(a);
  }
}

}  // namespace

// logp[r] = sum_c cell_lp[r][c], act16[r][c] = packed act[r][c][0..6], rng step advance.
// cnt (may be null): ncnt bucket counters zeroed for the next step (head_fwd_counts mode).
extern "C" int mbk_row_sum_pack(const float* cell_lp, int64_t rows, int cols, float* logp,
                                uint64_t* rng, const uint8_t* act, uint16_t* act16, int* cnt,
                                int ncnt, hipStream_t stream) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(row_sum_pack_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                     cell_lp, rows, cols, logp, rng, act, act16, cnt, ncnt);
  return (int)hipGetLastError();
}

extern "C" int mbk_decode_obs_mask(const uint16_t* codes, const int32_t* res, int n_envs, int H,
                                   int W, uint32_t* obs, uint32_t* mask, hipStream_t stream) {
  if (n_envs <= 0) return 0;
  if (H * W > 4096) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(decode_obs_mask_kernel<false>, dim3(decode_grid(n_envs)), dim3(256),
                     kEnvsPerWG * H * W * 2, stream, codes, res, n_envs, H, W, obs, mask,
                     Buckets{nullptr, nullptr, nullptr, nullptr});
  return (int)hipGetLastError();
}

extern "C" int mbk_decode_obs_mask_bucket(const uint16_t* codes, const int32_t* res, int n_envs,
                                          int H, int W, uint32_t* obs, uint32_t* mask,
                                          int* bucket_cnt, int* bucket, float* cell_lp,
                                          uint8_t* action, hipStream_t stream) {
  if (n_envs <= 0) return 0;
  if (H * W > 4096) return (int)hipErrorInvalidValue;
  const size_t sm = bucket_smem(H * W);
  if (sm > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)decode_obs_mask_kernel<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  hipLaunchKernelGGL(decode_obs_mask_kernel<true>, dim3(bucket_grid(n_envs)),
                     dim3(64 * kBucketEPW), sm, stream, codes, res, n_envs, H, W, obs, mask,
                     Buckets{bucket_cnt, bucket, cell_lp, action});
  return (int)hipGetLastError();
}

extern "C" int mbk_pack_env_actions(const uint8_t* act, int64_t ncells, uint16_t* out,
                                    hipStream_t stream) {
  int64_t blocks = (ncells + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(pack_env_actions_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, act,
                     ncells, out);
  return (int)hipGetLastError();
}
