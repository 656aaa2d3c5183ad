// Loss, optimizer and elementwise kernels (gfx950).
//
//   softmax_xent   : fused log-softmax + NLL forward and d(logits) in one pass
//                    (8 lanes per row for NC <= 64, bf16 or fp32 in/out),
//                    per-block loss partials and per-row correctness flags
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

#include <type_traits>

// ---------------------------------------------------------------------------
// Dense-prediction form (per-voxel segmentation: millions of rows, NC ~ 25):
// LPR lanes per row (8 for NC <= 64, so a wave covers 8 rows and the loads of a
// wave are one contiguous run), bf16 or fp32 logits read directly, d(logits)
// written in the logits' dtype with 1/B folded in, per-block partial loss sums
// (no per-row loss array, no host sync); grid-stride over rows.
template <typename TIn, int LPR, int EPL>
__global__ __launch_bounds__(256) void softmax_xent_rows_kernel(const TIn* __restrict__ logits,
                                                                const long long* __restrict__ labels,
                                                                float* __restrict__ block_loss, TIn* __restrict__ dlogits,
                                                                int* __restrict__ correct, long long B, int NC,
                                                                float gscale, float smoothing, float lscale) {
  // EPL > 0: the row (<= LPR*EPL classes) is read ONCE into registers; EPL = 0: any NC,
  // re-read per pass
  constexpr int RPB = 256 / LPR;
  __shared__ float red[256 / 64];
  const int sub = threadIdx.x % LPR, rloc = threadIdx.x / LPR;
  const float off = smoothing / (float)NC, on = 1.f - smoothing + off;
  float acc = 0.f;
  auto ld = [](const TIn* p) -> float {
    if constexpr (sizeof(TIn) == 2) return bf2f(*p); else return (float)*p;
  };
  for (long long r0 = (long long)blockIdx.x * RPB; r0 < B; r0 += (long long)gridDim.x * RPB) {
    const long long row = r0 + rloc;
    const bool live = row < B;
    const TIn* rp = logits + (live ? row : 0) * NC;
    float mx = -INFINITY;
    int am = 0;
    float v[EPL > 0 ? EPL : 1];
    if constexpr (EPL > 0) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = sub + e * LPR;
        v[e] = c < NC ? ld(rp + c) : -INFINITY;
        if (v[e] > mx) { mx = v[e]; am = c; }
      }
    } else {
      for (int c = sub; c < NC; c += LPR) {
        const float x = ld(rp + c);
        if (x > mx) { mx = x; am = c; }
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) {          // group arg-max, lowest index on ties
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    float se = 0.f;
    if constexpr (EPL > 0) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) se += sub + e * LPR < NC ? __expf(v[e] - mx) : 0.f;
    } else {
      for (int c = sub; c < NC; c += LPR) se += __expf(ld(rp + c) - mx);
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
    const float lse = mx + __logf(se);
    const long long y = live ? labels[row] : -1;
    float lrow = 0.f;
    auto out = [&](int c, float x) {
      const float lp = x - lse;
      const float tgt = (c == y) ? on : off;
      lrow -= tgt * lp;
      if (live) {
        const float d = (__expf(lp) - tgt) * gscale;
        if constexpr (sizeof(TIn) == 2) dlogits[row * NC + c] = f2bf(d); else dlogits[row * NC + c] = d;
      }
    };
    if constexpr (EPL > 0) {
#pragma unroll
      for (int e = 0; e < EPL; ++e)
        if (sub + e * LPR < NC) out(sub + e * LPR, v[e]);
    } else {
      for (int c = sub; c < NC; c += LPR) out(c, ld(rp + c));
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) lrow += __shfl_xor(lrow, o, 64);
    if (live && sub == 0) {
      acc += lrow;
      if (correct) correct[row] = (am == y) ? 1 : 0;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) block_loss[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) * lscale;
}

// Tile form for bf16 logits with NC <= NCMAX (the per-voxel segmentation loss):
// 256 rows per tile move between HBM and LDS as 16-byte vectors (the tile is one
// contiguous run of 256*NC bf16), then every thread owns one row entirely in
// registers -- no cross-lane reductions, every global access coalesced.
template <int NCMAX>
__global__ __launch_bounds__(256) void softmax_xent_tile_kernel(const bf16* __restrict__ logits,
                                                                const long long* __restrict__ labels,
                                                                float* __restrict__ block_loss,
                                                                bf16* __restrict__ dlogits, int* __restrict__ correct,
                                                                long long B, int NC, float gscale, float smoothing,
                                                                float lscale) {
  __shared__ __attribute__((aligned(16))) bf16 tile[256 * NCMAX];
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const float off = smoothing / (float)NC, on = 1.f - smoothing + off;
  float acc = 0.f;
  for (long long r0 = (long long)blockIdx.x * 256; r0 < B; r0 += (long long)gridDim.x * 256) {
    const int rows = (int)(B - r0 < 256 ? B - r0 : 256);
    const int nel = rows * NC;
    const bf16* src = logits + r0 * NC;           // 16-B aligned: r0 * NC * 2 = 512 * NC * k
    const int nvec = nel >> 3;
    __syncthreads();                               // previous tile's stores are done with `tile`
    for (int i = tid; i < nvec; i += 256) *(uint4*)(tile + i * 8) = *(const uint4*)(src + i * 8);
    for (int i = (nvec << 3) + tid; i < nel; i += 256) tile[i] = src[i];
    __syncthreads();
    if (tid < rows) {
      const long long row = r0 + tid;
      float v[NCMAX];
      float mx = -INFINITY;
      int am = 0;
#pragma unroll
      for (int c = 0; c < NCMAX; ++c) {
        v[c] = c < NC ? bf2f(tile[tid * NC + c]) : -INFINITY;
        if (v[c] > mx) { mx = v[c]; am = c; }
      }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < NCMAX; ++c) se += c < NC ? __expf(v[c] - mx) : 0.f;
      const float lse = mx + __logf(se);
      const long long y = labels[row];
      float lrow = 0.f;
#pragma unroll
      for (int c = 0; c < NCMAX; ++c) {
        if (c < NC) {
          const float lp = v[c] - lse;
          const float tgt = (c == y) ? on : off;
          lrow -= tgt * lp;
          tile[tid * NC + c] = f2bf((__expf(lp) - tgt) * gscale);   // own row only: no race
        }
      }
      acc += lrow;
      if (correct) correct[row] = (am == y) ? 1 : 0;
    }
    __syncthreads();
    bf16* dst = dlogits + r0 * NC;
    for (int i = tid; i < nvec; i += 256) *(uint4*)(dst + i * 8) = *(const uint4*)(tile + i * 8);
    for (int i = (nvec << 3) + tid; i < nel; i += 256) dst[i] = tile[i];
  }
  acc = wave_sum(acc);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) block_loss[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) * lscale;
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

// ---------------------------------------------------------------------------
// Nearest-neighbour x2 upsampling of a channels-last [N, D, H, W, C] grid (the
// segmentation decoder) and its backward (sum over each 2x2x2 block, fp32).
// One thread per 8-channel source vector: forward = 1 load, 8 stores;
// backward = 8 loads, 1 store.  C % 8 == 0.
// Index decode in 32-bit (IDX = unsigned) when the chunk count fits: the 64-bit divisions of
// the general form cost more VALU than the 16-B copies themselves (2.8 TB/s at 64^3 x 64).
template <typename IDX>
__global__ __launch_bounds__(256) void upsample2x_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int D,
                                                         int H, int W, int C, long long total) {
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= total) return;
  const IDX cpr = (IDX)(C >> 3);
  IDX t = (IDX)i;
  const int cv = (int)(t % cpr); t /= cpr;
  const int w = (int)(t % (IDX)W); t /= (IDX)W;
  const int h = (int)(t % (IDX)H); t /= (IDX)H;
  const int d = (int)(t % (IDX)D);
  const long long n = (long long)(t / (IDX)D);
  const uint4 v = *(const uint4*)(x + i * 8);
  const long long W2 = 2LL * W, H2 = 2LL * H;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const long long base = (((n * 2 * D + 2 * d + a) * H2 + 2 * h + b) * W2 + 2 * w) * C + cv * 8;
      *(uint4*)(y + base) = v;
      *(uint4*)(y + base + C) = v;
    }
}

template <typename IDX>
__global__ __launch_bounds__(256) void upsample2x_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                             int D, int H, int W, int C, long long total) {
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= total) return;
  const IDX cpr = (IDX)(C >> 3);
  IDX t = (IDX)i;
  const int cv = (int)(t % cpr); t /= cpr;
  const int w = (int)(t % (IDX)W); t /= (IDX)W;
  const int h = (int)(t % (IDX)H); t /= (IDX)H;
  const int d = (int)(t % (IDX)D);
  const long long n = (long long)(t / (IDX)D);
  const long long W2 = 2LL * W, H2 = 2LL * H;
  Pack8 p[8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const long long base = (((n * 2 * D + 2 * d + a) * H2 + 2 * h + b) * W2 + 2 * w) * C + cv * 8;
      p[(a * 2 + b) * 2].u = *(const uint4*)(dy + base);
      p[(a * 2 + b) * 2 + 1].u = *(const uint4*)(dy + base + C);
    }
  Pack8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += bf2f(p[k].e[j]);
    o.e[j] = f2bf(s);
  }
  *(uint4*)(dx + i * 8) = o.u;
}

// Output-row-major variants (C / 8 a power of two <= 32): lane i covers output chunk (w2, cv) of
// an output row, so every store (forward) / load (backward) instruction of a wave touches one
// contiguous 1-KB run instead of 128-B pieces two voxels apart.  Forward: one input chunk ->
// the same chunk of the four output rows (2d+a, 2h+b).  Backward: the four rows' chunks are
// summed per lane, then the pair (w2 = 2w, 2w+1) -- lanes cpr apart in the same wave -- is
// folded with one shuffle and the even lane stores dx.
__global__ __launch_bounds__(256) void upsample2x_rows_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                              int D, int H, int W, int lcpr, unsigned total) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i >= total) return;
  const unsigned cpr = 1u << lcpr, C = cpr * 8u, W2 = 2u * W;
  const unsigned cv = i & (cpr - 1);
  unsigned t = i >> lcpr;
  const unsigned w2 = t % W2; t /= W2;
  const unsigned h = t % (unsigned)H; t /= (unsigned)H;
  const unsigned d = t % (unsigned)D;
  const long long n = t / (unsigned)D;
  const uint4 v = *(const uint4*)(x + ((((n * D + d) * H + h) * (long long)W + (w2 >> 1)) * C + cv * 8));
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
      *(uint4*)(y + ((((n * 2 * D + 2 * d + a) * 2LL * H + 2 * h + b) * W2 + w2) * C + cv * 8)) = v;
}

__global__ __launch_bounds__(256) void upsample2x_rows_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                                  int D, int H, int W, int lcpr, unsigned total) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i >= total) return;                        // (total is a multiple of 2 cpr: pairs stay together)
  const unsigned cpr = 1u << lcpr, C = cpr * 8u, W2 = 2u * W;
  const unsigned cv = i & (cpr - 1);
  unsigned t = i >> lcpr;
  const unsigned w2 = t % W2; t /= W2;
  const unsigned h = t % (unsigned)H; t /= (unsigned)H;
  const unsigned d = t % (unsigned)D;
  const long long n = t / (unsigned)D;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      Pack8 p;
      p.u = *(const uint4*)(dy + ((((n * 2 * D + 2 * d + a) * 2LL * H + 2 * h + b) * W2 + w2) * C + cv * 8));
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f(p.e[j]);
    }
  Pack8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.e[j] = f2bf(s[j] + __shfl_down(s[j], (int)cpr, 64));
  if ((w2 & 1u) == 0)
    *(uint4*)(dx + ((((n * D + d) * H + h) * (long long)W + (w2 >> 1)) * C + cv * 8)) = o.u;
}

extern "C" int fn_upsample2x(const void* x, void* y, int N, int D, int H, int W, int C, int backward,
                             hipStream_t st) {
  if (C % 8) return -2;
  {
    const int cpr = C / 8;
    int lcpr = 0;
    while ((1 << lcpr) < cpr) ++lcpr;
    const long long tot_rows = (long long)N * D * H * (2LL * W) * cpr;
    if ((1 << lcpr) == cpr && cpr <= 32 && tot_rows < (1LL << 32)) {
      const unsigned blocks = (unsigned)((tot_rows + 255) / 256);
      if (backward)
        hipLaunchKernelGGL(upsample2x_rows_bwd_kernel, dim3(blocks), dim3(256), 0, st, (const bf16*)x, (bf16*)y, D, H,
                           W, lcpr, (unsigned)tot_rows);
      else
        hipLaunchKernelGGL(upsample2x_rows_kernel, dim3(blocks), dim3(256), 0, st, (const bf16*)x, (bf16*)y, D, H, W,
                           lcpr, (unsigned)tot_rows);
      FN_CHECK_LAUNCH();
      return 0;
    }
  }
  const long long total = (long long)N * D * H * W * (C / 8);
  const unsigned blocks = (unsigned)((total + 255) / 256);
  const bool small = total < (1LL << 32);
#define UP_LAUNCH(K, T) hipLaunchKernelGGL(K<T>, dim3(blocks), dim3(256), 0, st, (const bf16*)x, (bf16*)y, D, H, W, C, total)
  if (backward) {
    if (small) UP_LAUNCH(upsample2x_bwd_kernel, unsigned); else UP_LAUNCH(upsample2x_bwd_kernel, unsigned long long);
  } else {
    if (small) UP_LAUNCH(upsample2x_kernel, unsigned); else UP_LAUNCH(upsample2x_kernel, unsigned long long);
  }
#undef UP_LAUNCH
  FN_CHECK_LAUNCH();
  return 0;
}

static int sx_lpr(int NC) { return NC <= 64 ? 8 : 64; }

// number of partial loss sums softmax_xent_rows writes (= its grid); the bf16 tile
// kernel (NC <= 32) covers 256 rows per block, the lane-group kernel 256/LPR.  Classifier
// batches (<= 2048 rows) take ONE block: its partial is then the mean loss itself (no reduction
// and division launches after the loss kernel)
extern "C" int fn_softmax_xent_blocks(long long B, int NC) {
  if (B <= 2048) return 1;
  const long long rpb = NC <= 32 ? 256 : 256 / sx_lpr(NC);
  const long long need = (B + rpb - 1) / rpb;
  return (int)(need < 8192 ? (need > 0 ? need : 1) : 8192);
}

// logits / dlogits bf16 (in_bf16 = 1) or fp32; block_loss: fp32 [fn_softmax_xent_blocks] partial
// sums, or with one block the sum x gscale (the mean loss when gscale = 1/B)
extern "C" int fn_softmax_xent_rows(const void* logits, int in_bf16, const long long* labels, float* block_loss,
                                    void* dlogits, int* correct, long long B, int NC, float gscale, float smoothing,
                                    hipStream_t st) {
  const unsigned blocks = (unsigned)fn_softmax_xent_blocks(B, NC);
  const float lscale = blocks == 1 ? gscale : 1.f;
#define SX(T, L, E)                                                                                                \
  hipLaunchKernelGGL((softmax_xent_rows_kernel<T, L, E>), dim3(blocks), dim3(256), 0, st, (const T*)logits, labels, \
                     block_loss, (T*)dlogits, correct, B, NC, gscale, smoothing, lscale)
#define SX_T(T)                                         \
  do {                                                  \
    if (NC <= 32) SX(T, 8, 4);                          \
    else if (NC <= 64) SX(T, 8, 8);                     \
    else SX(T, 64, 0);                                  \
  } while (0)
  if (in_bf16 && NC <= 32)
    hipLaunchKernelGGL(softmax_xent_tile_kernel<32>, dim3(blocks), dim3(256), 0, st, (const bf16*)logits, labels,
                       block_loss, (bf16*)dlogits, correct, B, NC, gscale, smoothing, lscale);
  else if (in_bf16) SX_T(bf16);
  else SX_T(float);
#undef SX_T
#undef SX
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
// hp = {lr, b1, b2, eps, wd, grad_scale}; *t is incremented by the 1-thread kernel that
// precedes this one in the same stream.  (A finished-block count with the last block storing the
// step back, to save that launch, serialised 8192 same-address atomics: 40 -> 407 us.)
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

// x *= *s in place, unless *s == 1 (the loss gradient of a plain loss.backward()): every
// workgroup reads the device scalar first and leaves at once, so the common case costs one
// near-empty launch instead of a pass over d(logits) -- no host sync, graph-capturable.
// (SoftmaxXentFn.backward: 838M d(logits) elements for the 64^3 segmentation head.)
template <typename T>
__global__ __launch_bounds__(256) void scale_unless_one_kernel(T* __restrict__ x, const float* __restrict__ s,
                                                               long long n) {
  const float f = *s;
  if (f == 1.0f) return;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    if constexpr (std::is_same<T, float>::value) x[i] *= f;
    else x[i] = f2bf(bf2f(x[i]) * f);
  }
}

extern "C" int fn_scale_unless_one(void* x, int is_bf16, const float* s, long long n, hipStream_t st) {
  if (n <= 0) return 0;
  if (is_bf16)
    hipLaunchKernelGGL(scale_unless_one_kernel<bf16>, dim3(blocks_for(n)), dim3(256), 0, st, (bf16*)x, s, n);
  else
    hipLaunchKernelGGL(scale_unless_one_kernel<float>, dim3(blocks_for(n)), dim3(256), 0, st, (float*)x, s, n);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Batch copy-in: up to two device buffers (the step's input voxels and labels) in ONE launch,
// 16-B vector loads with four chunks in flight per thread over a resident-sized grid (the
// runtime's blit kernel moved the 33.5 MB FeatureNet-3D batch at ~1.3 TB/s in 25 us, plus a
// second launch for the labels).  Pointers 16-B aligned (host-checked); tail bytes one by one.
struct CopyJob {
  unsigned char* d;
  const unsigned char* s;
  long long n;
};

__global__ __launch_bounds__(256) void copy2_kernel(CopyJob a, CopyJob b) {
  const long long stride = (long long)gridDim.x * 256;
  const long long t0 = (long long)blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const CopyJob c = j == 0 ? a : b;
    const long long nv = c.n >> 4;
    const uint4* sv = reinterpret_cast<const uint4*>(c.s);
    uint4* dv = reinterpret_cast<uint4*>(c.d);
    long long i = t0;
    for (; i + 3 * stride < nv; i += 4 * stride) {
      const uint4 v0 = sv[i], v1 = sv[i + stride], v2 = sv[i + 2 * stride], v3 = sv[i + 3 * stride];
      dv[i] = v0;
      dv[i + stride] = v1;
      dv[i + 2 * stride] = v2;
      dv[i + 3 * stride] = v3;
    }
    for (; i < nv; i += stride) dv[i] = sv[i];
    for (long long k = nv * 16 + t0; k < c.n; k += stride) c.d[k] = c.s[k];
  }
}

extern "C" int fn_copy2(void* d0, const void* s0, long long n0, void* d1, const void* s1, long long n1,
                        hipStream_t st) {
  if (n0 < 0 || n1 < 0 || ((uintptr_t)d0 | (uintptr_t)s0) % 16 || (n1 > 0 && ((uintptr_t)d1 | (uintptr_t)s1) % 16))
    return -2;
  const long long nv = ((n0 > n1 ? n0 : n1) + 15) / 16;
  long long blocks = (nv + 4 * 256 - 1) / (4 * 256);
  if (blocks > 2048) blocks = 2048;              // 8 per CU, grid-stride beyond
  if (blocks < 1) blocks = 1;
  const CopyJob a{(unsigned char*)d0, (const unsigned char*)s0, n0};
  const CopyJob b{(unsigned char*)d1, (const unsigned char*)s1, n1 > 0 ? n1 : 0};
  hipLaunchKernelGGL(copy2_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, b);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// CU occupier (measurement only: scripts/dp_interference.py).  `nwg` workgroups of 256 threads,
// each holding `lds` bytes of LDS and spinning VALU work for `usec` microseconds of wall time
// (s_memrealtime, 100 MHz), so that a side stream pins that many CUs the way an RCCL ring
// kernel does while the training step runs on the main stream.  lds >= 16 KB keeps a big-tile
// conv workgroup (>= 144 KB) off the CU for the whole spin; lds = 0 only shares its issue
// slots.  Every wave leaves after `usec` (bounded: no flag, no dependence on other work); a
// nonzero `sink` word is written only if the impossible happens, so the loop is not dead code.
__global__ __launch_bounds__(256) void cu_occupy_kernel(int usec, unsigned* __restrict__ sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long dt = (unsigned long long)usec * 100ull;   // 100 MHz ticks
  float a = (float)threadIdx.x, b = 1.0001f;
  while (__builtin_amdgcn_s_memrealtime() - t0 < dt) {
#pragma unroll
    for (int i = 0; i < 64; ++i) a = a * b + 1e-7f;
  }
  if (a == -1.f) sink[threadIdx.x] = 1u;          // never true: keeps the spin alive
}

extern "C" int fn_cu_occupy(int nwg, int usec, int lds, void* sink, hipStream_t st) {
  if (nwg <= 0 || nwg > 1024 || usec <= 0 || usec > 200000 || lds < 0 || lds > 160 * 1024) return -2;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)cu_occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -5;
  hipLaunchKernelGGL(cu_occupy_kernel, dim3((unsigned)nwg), dim3(256), (size_t)lds, st, usec, (unsigned*)sink);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Row softmax of fp32 rows (a Dense layer with a softmax activation inside a NAS candidate; the
// classifier head's softmax lives in softmax_xent): one wave per row, 8 rows per 512-thread
// block, any N (lanes stride the row); the backward dx = y * (g - sum(g * y)) the same way.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sm_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float sm_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(512) void softmax_rows_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               long long M, int N) {
  const long long m = (long long)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  const float* xr = x + m * N;
  float mx = -INFINITY;
  for (int i = lane; i < N; i += 64) mx = fmaxf(mx, xr[i]);
  mx = sm_wave_max(mx);
  float s = 0.f;
  for (int i = lane; i < N; i += 64) s += __expf(xr[i] - mx);
  const float inv = 1.f / sm_wave_sum(s);
  float* yr = y + m * N;
  for (int i = lane; i < N; i += 64) yr[i] = __expf(xr[i] - mx) * inv;
}

__global__ __launch_bounds__(512) void softmax_rows_bwd_kernel(const float* __restrict__ y, const float* __restrict__ g,
                                                               float* __restrict__ dx, long long M, int N) {
  const long long m = (long long)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  const float* yr = y + m * N;
  const float* gr = g + m * N;
  float s = 0.f;
  for (int i = lane; i < N; i += 64) s += gr[i] * yr[i];
  s = sm_wave_sum(s);
  float* dr = dx + m * N;
  for (int i = lane; i < N; i += 64) dr[i] = yr[i] * (gr[i] - s);
}

extern "C" int fn_softmax_rows(const float* x, float* y, long long M, int N, int backward, const float* g,
                               hipStream_t st) {
  if (M <= 0 || N <= 0 || (backward && !g)) return -2;
  const dim3 grid((unsigned)((M + 7) / 8));
  if (backward)
    hipLaunchKernelGGL(softmax_rows_bwd_kernel, grid, dim3(512), 0, st, x, g, y, M, N);
  else
    hipLaunchKernelGGL(softmax_rows_fwd_kernel, grid, dim3(512), 0, st, x, y, M, N);
  FN_CHECK_LAUNCH();
  return 0;
}
