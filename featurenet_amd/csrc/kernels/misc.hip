// Loss, optimizer and elementwise kernels (gfx950).
//
//   softmax_xent   : fused log-softmax + NLL forward and d(logits) in one pass,
//                    one 64-lane wave per row, plus per-row correctness flags
//                    (top-1 accuracy without a host sync).
//   adam_flat      : multi-tensor Adam over ONE flat fp32 parameter buffer
//                    (all parameters of a model live in a single allocation),
//                    optionally refreshing the bf16 compute shadow in the same
//                    pass; torch-style and Keras-2.2-style epsilon placement.
//   sgd_flat       : momentum SGD (Nesterov optional) over the flat buffer.
//   act / bias_act : standalone activation and bias+activation (fallback when
//                    no producer epilogue can absorb them).
//   dropout        : counter-based hash RNG so backward regenerates the mask.
//   cast           : fp32 <-> bf16.
#include "common.h"

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ logits,
                                                           const long long* __restrict__ labels,
                                                           float* __restrict__ loss, float* __restrict__ dlogits,
                                                           int* __restrict__ correct, int B, int NC, float gscale,
                                                           float smoothing) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= B) return;
  const float* row = logits + (long long)wave * NC;
  float mx = -INFINITY;
  int amax = 0;
  for (int c = lane; c < NC; c += 64) {
    const float v = row[c];
    if (v > mx) { mx = v; amax = c; }
  }
  // wave arg-max (lowest index on ties)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < NC; c += 64) se += __expf(row[c] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const long long y = labels[wave];
  const float off = smoothing / (float)NC;
  const float on = 1.f - smoothing + off;
  float lrow = 0.f;
  for (int c = lane; c < NC; c += 64) {
    const float lp = row[c] - lse;
    const float tgt = (c == y) ? on : off;
    lrow -= tgt * lp;
    if (dlogits) dlogits[(long long)wave * NC + c] = (__expf(lp) - tgt) * gscale;
  }
  lrow = wave_sum(lrow);
  if (lane == 0) {
    loss[wave] = lrow;
    if (correct) correct[wave] = (amax == y) ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        bf16* __restrict__ pb, long long n, float lr, float b1,
                                                        float b2, float eps, float wd, float bc1, float bc2,
                                                        float gscale, int keras_eps) {
  const float rb2 = rsqrtf(bc2);  // 1/sqrt(bc2)
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float gi = g[i] * gscale;
    float pi = p[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    if (wd != 0.f) pi -= lr * wd * pi;  // decoupled (AdamW) decay
    float upd;
    if (keras_eps) {
      // Keras 2.2: lr_t = lr*sqrt(1-b2^t)/(1-b1^t); p -= lr_t*m/(sqrt(v)+eps)
      upd = (lr * sqrtf(bc2) / bc1) * mi / (sqrtf(vi) + eps);
    } else {
      upd = lr * (mi / bc1) / (sqrtf(vi) * rb2 + eps);
    }
    pi -= upd;
    p[i] = pi;
    if (pb) pb[i] = f2bf(pi);
  }
}

__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ buf, bf16* __restrict__ pb, long long n,
                                                       float lr, float momentum, float wd, int nesterov,
                                                       float gscale) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float gi = g[i] * gscale;
    float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    if (momentum != 0.f) {
      const float b = momentum * buf[i] + gi;
      buf[i] = b;
      gi = nesterov ? gi + momentum * b : b;
    }
    pi -= lr * gi;
    p[i] = pi;
    if (pb) pb[i] = f2bf(pi);
  }
}

// ---------------------------------------------------------------------------
// y = act(x + bias[c]) on [rows][C] bf16; x may alias y
__global__ __launch_bounds__(256) void bias_act_kernel(const bf16* __restrict__ x, const float* __restrict__ bias,
                                                       bf16* __restrict__ y, long long total, int C, int act) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const float b = bias ? bias[i % C] : 0.f;
    y[i] = f2bf(act_fwd(bf2f(x[i]) + b, act));
  }
}

// dx = dy * act'(y) (through the output)
__global__ __launch_bounds__(256) void act_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                                                      bf16* __restrict__ dx, long long total, int act) {
  const long long n8 = total / 8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    Pack8 a, b, o;
    a.u = *(const uint4*)(dy + i * 8);
    b.u = *(const uint4*)(y + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) o.e[j] = f2bf(bf2f(a.e[j]) * act_bwd_from_out(bf2f(b.e[j]), act));
    *(uint4*)(dx + i * 8) = o.u;
  }
  if (blockIdx.x == 0)
    for (long long i = n8 * 8 + threadIdx.x; i < total; i += 256)
      dx[i] = f2bf(bf2f(dy[i]) * act_bwd_from_out(bf2f(y[i]), act));
}

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // lowbias32-style mixing of (seed, offset, index)
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x85EBCA77u) * 0xC2B2AE3Du ^ c * 0x27D4EB2Fu;
  h ^= h >> 16; h *= 0x7FEB352Du;
  h ^= h >> 15; h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

// y = x * mask / (1-p), mask regenerated identically in backward
__global__ __launch_bounds__(256) void dropout_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                      long long total, float p, uint32_t seed, uint32_t offset) {
  const float scale = 1.f / (1.f - p);
  const uint32_t thr = (uint32_t)(p * 4294967295.0f);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const uint32_t r = hash3(seed, offset, (uint32_t)i ^ (uint32_t)(i >> 32) * 0x632BE5ABu);
    y[i] = (r >= thr) ? f2bf(bf2f(x[i]) * scale) : (bf16)0.f;
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y,
                                                            long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) y[i] = f2bf(x[i]);
}

// Bit-packed voxel grids (1 bit/voxel, LSB first) -> bf16 occupancy {0,1}.
// One thread expands one byte into 8 bf16 (16 B store); the host/PCIe side
// moves 1/16 of the bf16 bytes (csrc/runtime/voxel.cpp packs them).
__global__ __launch_bounds__(256) void unpack_bits_kernel(const uint8_t* __restrict__ bits, bf16* __restrict__ out,
                                                          long long nbytes) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nbytes; i += (long long)gridDim.x * 256) {
    const unsigned b = bits[i];
    Pack8 p;
#pragma unroll
    for (int j = 0; j < 8; ++j) p.e[j] = (b >> j) & 1u ? (bf16)1.f : (bf16)0.f;
    *(uint4*)(out + i * 8) = p.u;
  }
}

// ---------------------------------------------------------------------------
static unsigned blocks_for(long long work) {
  long long b = (work + 255) / 256;
  if (b < 1) b = 1;
  if (b > 8192) b = 8192;
  return (unsigned)b;
}

extern "C" int fn_softmax_xent(const float* logits, const long long* labels, float* loss, float* dlogits,
                               int* correct, int B, int NC, float gscale, float smoothing, hipStream_t st) {
  const unsigned blocks = (unsigned)((B + 3) / 4);
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(blocks), dim3(256), 0, st, logits, labels, loss, dlogits, correct, B, NC,
                     gscale, smoothing);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_adam_flat(float* p, const float* g, float* m, float* v, void* pb, long long n, float lr, float b1,
                            float b2, float eps, float wd, float bc1, float bc2, float gscale, int keras_eps,
                            hipStream_t st) {
  hipLaunchKernelGGL(adam_flat_kernel, dim3(blocks_for(n)), dim3(256), 0, st, p, g, m, v, (bf16*)pb, n, lr, b1, b2,
                     eps, wd, bc1, bc2, gscale, keras_eps);
  FN_CHECK_LAUNCH();
  return 0;
}

// Graph-capturable Adam: hyper-parameters and the step counter live in device
// memory, so a captured training step replays with the current lr / step.
// hp = {lr, b1, b2, eps, wd, grad_scale}; *t is incremented by the 1-thread
// kernel that precedes this one in the same stream.
__global__ void step_inc_kernel(int* t) { *t += 1; }

__global__ __launch_bounds__(256) void adam_flat_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                            float* __restrict__ m, float* __restrict__ v,
                                                            bf16* __restrict__ pb, long long n,
                                                            const float* __restrict__ hp, const int* __restrict__ t,
                                                            int keras_eps) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4], gscale = hp[5];
  const float tf = (float)*t;
  const float bc1 = 1.f - powf(b1, tf), bc2 = 1.f - powf(b2, tf);
  const float rb2 = rsqrtf(bc2);
  const float lr_t = lr * sqrtf(bc2) / bc1;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float gi = g[i] * gscale;
    float pi = p[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    if (wd != 0.f) pi -= lr * wd * pi;
    pi -= keras_eps ? lr_t * mi / (sqrtf(vi) + eps) : lr * (mi / bc1) / (sqrtf(vi) * rb2 + eps);
    p[i] = pi;
    if (pb) pb[i] = f2bf(pi);
  }
}

extern "C" int fn_adam_flat_dev(float* p, const float* g, float* m, float* v, void* pb, long long n, const float* hp,
                                int* t, int keras_eps, hipStream_t st) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, t);
  hipLaunchKernelGGL(adam_flat_dev_kernel, dim3(blocks_for(n)), dim3(256), 0, st, p, g, m, v, (bf16*)pb, n, hp, t,
                     keras_eps);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_sgd_flat(float* p, const float* g, float* buf, void* pb, long long n, float lr, float momentum,
                           float wd, int nesterov, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(blocks_for(n)), dim3(256), 0, st, p, g, buf, (bf16*)pb, n, lr, momentum,
                     wd, nesterov, gscale);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_bias_act(const void* x, const float* bias, void* y, long long total, int C, int act,
                           hipStream_t st) {
  hipLaunchKernelGGL(bias_act_kernel, dim3(blocks_for(total)), dim3(256), 0, st, (const bf16*)x, bias, (bf16*)y, total,
                     C, act);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_act_bwd(const void* dy, const void* y, void* dx, long long total, int act, hipStream_t st) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(blocks_for(total / 8 + 1)), dim3(256), 0, st, (const bf16*)dy,
                     (const bf16*)y, (bf16*)dx, total, act);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_dropout(const void* x, void* y, long long total, float p, unsigned seed, unsigned offset,
                          hipStream_t st) {
  hipLaunchKernelGGL(dropout_kernel, dim3(blocks_for(total)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, total, p,
                     seed, offset);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_unpack_bits(const void* bits, void* out, long long nbytes, hipStream_t st) {
  hipLaunchKernelGGL(unpack_bits_kernel, dim3(blocks_for(nbytes)), dim3(256), 0, st, (const uint8_t*)bits,
                     (bf16*)out, nbytes);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_cast_f32_bf16(const float* x, void* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(blocks_for(n)), dim3(256), 0, st, x, (bf16*)y, n);
  FN_CHECK_LAUNCH();
  return 0;
}
