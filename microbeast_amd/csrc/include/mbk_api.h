// C ABI of the microbeast_amd HIP kernel library (libmbk_kernels.so).
// Every launcher enqueues on the given HIP stream, never synchronises and never
// allocates, so callers can capture sequences of them into hipGraphs.
// Return value: hipError_t of the launch (0 = success).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MBK_MAX_COPY_SEGS 16
typedef struct {
  const void* src;
  void* dst;
  uint64_t bytes;
} MbkCopySeg;

// Many independent D2D copies in ONE launch (rollout scatter).
int mbk_multi_copy(const MbkCopySeg* segs, int n, hipStream_t stream);

typedef struct {
  const float* w;  // fp32 [cout][cin_real][3][3]
  void* fwd;       // bf16 packed fwd weights
  void* bwd;       // bf16 packed dgrad weights (nullable)
  int cin, cin_real, cout;
} MbkPackJob;

int mbk_conv_pack(const MbkPackJob* jobs, int n, hipStream_t stream);

typedef struct {
  const float* w;  // fp32 [cout][cin_real][3][3]
  void* q;         // e4m3 packed fwd weights [cout][nch][32]
  float* scale;    // [cout] dequant multipliers
  int cin, cin_real, cout;
} MbkPackJob8;

int mbk_conv_pack_fp8(const MbkPackJob8* jobs, int n, hipStream_t stream);

// ---- fused acting step (act.hip-level API; kernels in trunk.hip + head.hip) ----------------
// One policy step of the flat IMPALA agent on a 16x16 map in TWO launches:
//   A (trunk.hip act_trunk_kernel): per 16-env tile, 16-bit codes -> obs bit planes + 78-bit
//     masks (written straight into the rollout row), per-cell buckets of active pairs, stage-0
//     conv with the max-pool in registers, the 14 trunk convs in LDS, network.5 + critic;
//   B (head.hip head_act_kernel): sparse head GEMM + masked sampling per 16-pair unit, per-env
//     completion counters: the wave that finishes an env's last active cell sums its log-prob
//     and writes its packed 16-bit actions; the last workgroup resets the buckets and advances
//     the sampler's step counter.
// Model / workspace pointers are fixed per policy lane; step pointers change every step.
typedef struct {
  const void* w0;          // stage-0 conv packed fwd weights [16][9][32] bf16
  const float* b0;         // [16]
  const void* w[14];       // trunk layers 1..14 packed fwd weights (bf16)
  const float* b[14];
  const void* w5;          // network.5 [256][H2*W2*32] bf16, NHWC column order
  const float* b5;         // [256]
  const float* wc;         // critic [256]
  const float* bc;         // [1]
  const void* Wp;          // sparse head [S][80][256] bf16
  const float* bp;         // [S][80]
  uint64_t* rng;           // Philox (seed, step): the step is MbkActStep.step; [1] is set
                           // to step + 1 after the step (the graph path's counter)
  void* feat;              // workspace: network.5 output [E][256] bf16
  int* bucket_cnt;         // [2][S]: step t counts in half t & 1; launch A of step t zeroes
                           // the other half (step t-1's, read by its launch B)
  int* bucket;             // [S][E]
  uint64_t* cellx;         // [E][S] per active cell (rank k): {log-prob, cell | action << 16}
  int* pending;            // [2E]: active cells not yet sampled, then each env's total
  int E, H, W;
} MbkActModel;

typedef struct {
  // input: dense codes + resources, or (code_list != null) the sparse rows of list_stride
  // uint32 per env: word 0 = n | resources << 16, then n entries cell | code << 16 (occupied
  // cells only: empty cells are code 0)
  const uint16_t* codes;   // [E][S] (device or pinned host)
  const int32_t* res;      // [E]
  const uint32_t* code_list;
  uint32_t* obs;           // rollout row [E][S]
  uint32_t* mask;          // [E][S][3]
  uint32_t* obs2;          // optional second destination (previous slot's bootstrap row)
  uint32_t* mask2;
  uint8_t* action;         // [E][S][7]
  float* logp;             // [E]
  float* value;            // [E]
  // output actions: dense packed codes [E][S] (device or pinned host), or (act_list != null)
  // sparse rows: word 0 = n, then n entries cell | code << 16 for the non-noop cells
  uint16_t* act16;
  uint32_t* act_list;
  int list_stride;
  const float* reward_src; // optional reward / done of the previous env step -> dst
  const uint8_t* done_src;
  float* reward_dst;
  uint8_t* done_dst;
  uint64_t step;           // Philox step of this policy step (the lane's step count)
  uint32_t* abits;         // optional [E][S/32] active-cell bitmap of the row (bit c & 31 of
  uint32_t* abits2;        // word c >> 5: the cell's mask is non-zero), + the obs2 copy; the
                           // learner's head compaction then never reads the masks in full
} MbkActStep;

int mbk_act_step(const MbkActModel* m, const MbkActStep* s, hipStream_t stream);
// sparse-row I/O of the captured-graph policy step (copy.hip): pinned occupied-cell rows ->
// dense device codes + resources, and dense packed actions -> pinned non-noop action rows
int mbk_rows_to_codes(const uint32_t* rows, int stride, int E, int S, void* codes, int32_t* res,
                      hipStream_t stream);
int mbk_codes_to_rows(const void* act16, int E, int S, uint32_t* rows, int stride,
                      hipStream_t stream);
// the two launches separately (mbk_act_step = A then B)
int mbk_act_trunk(const MbkActModel* m, const MbkActStep* s, hipStream_t stream);
int mbk_act_head(const MbkActModel* m, const MbkActStep* s, hipStream_t stream);

#ifdef __cplusplus
}
#endif
