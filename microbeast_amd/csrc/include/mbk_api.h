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

#ifdef __cplusplus
}
#endif
