// Shared device helpers for the featurenet_amd gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * activations are channels-last ([N][D][H][W][C], 2-D = D==1) bf16;
//   * accumulation, BN statistics and optimizer state are fp32;
//   * a wavefront is 64 lanes (never 32) and workgroups are multiples of 64;
//   * kernels take raw device pointers plus a hipStream_t so they can be
//     captured into hipGraphs by the caller (no allocation / sync inside).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define FN_WAVE 64

#define FN_CHECK_LAUNCH()                                                     \
  do {                                                                        \
    hipError_t e__ = hipGetLastError();                                       \
    if (e__ != hipSuccess) return (int)e__;                                   \
  } while (0)

enum ActKind : int { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_SIGMOID = 3 };

__device__ __forceinline__ float act_fwd(float x, int act) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return tanhf(x);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    default: return x;
  }
}

// derivative expressed through the activation OUTPUT y (cheap, no re-eval).
__device__ __forceinline__ float act_bwd_from_out(float y, int act) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_TANH: return 1.f - y * y;
    case ACT_SIGMOID: return y * (1.f - y);
    default: return 1.f;
  }
}

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// 16-byte vector of 8 bf16 viewed as raw bits for loads/stores.
union Pack8 {
  uint4 u;
  bf16x8 v;
  bf16 e[8];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D block id: consecutive logical tiles land
// on the same XCD (shared L2) instead of being round-robined over the 8 XCDs.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

// dst[e] (+)= sum over p = 0 .. W-1 of part[p * n + e], in a fixed order (conv_wtile.hip): the
// deterministic replacement of per-workgroup float atomics -- kernels store their partial
// weight gradients into rows of `part` and this pass adds the rows, so the result is bitwise
// the same run to run whatever the workgroup timing
extern "C" int fn_part_reduce(const float* part, float* dst, long long n, int W, int accumulate, hipStream_t st);
extern "C" int fn_part_reduce2(const float* part, float* dst, long long n, const float* part2, float* dst2,
                               long long n2, int W, int accumulate, hipStream_t st);
extern "C" int fn_part_reduce_wdot(const float* part, float* dst, long long n, int W, int accumulate,
                                  const float* wsrc, float* wdp, int C, hipStream_t st);
