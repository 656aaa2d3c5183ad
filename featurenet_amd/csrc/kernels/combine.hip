// Branch-combination and padding kernels of the NAS cell (reference model/operation.py:
// Add :214-222, Concatenate :224-238, Multiply :240-248, ZeroPadding2D :116-137).
//
// All memory-bound, bf16, channels-last; 16-B vectors whenever the contiguous run allows
// (every FeatureNet / NAS channel count is a multiple of 8), scalar otherwise.  Each op is
// one pass: the padded tensor is written border and interior together (no zero-fill
// pass), concat writes both inputs into their column ranges of the output directly.
#include "common.h"

#define CB_THREADS 256

__device__ __forceinline__ unsigned cb_pack(float lo, float hi) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const b2 p = {f2bf(lo), f2bf(hi)};
  return __builtin_bit_cast(unsigned, p);
}
__device__ __forceinline__ float cb_lo(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float cb_hi(unsigned w) { return __uint_as_float(w & 0xffff0000u); }

// ---- out = a + b / a * b -------------------------------------------------------------
__global__ __launch_bounds__(CB_THREADS) void ew_binary_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                               bf16* __restrict__ out, long long n, int op) {
  const long long i = ((long long)blockIdx.x * CB_THREADS + threadIdx.x) * 8;
  if (i + 8 <= n) {
    const uint4 va = *(const uint4*)(a + i), vb = *(const uint4*)(b + i);
    const unsigned xa[4] = {va.x, va.y, va.z, va.w}, xb[4] = {vb.x, vb.y, vb.z, vb.w};
    unsigned o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float l = op ? cb_lo(xa[k]) * cb_lo(xb[k]) : cb_lo(xa[k]) + cb_lo(xb[k]);
      const float h = op ? cb_hi(xa[k]) * cb_hi(xb[k]) : cb_hi(xa[k]) + cb_hi(xb[k]);
      o[k] = cb_pack(l, h);
    }
    *(uint4*)(out + i) = make_uint4(o[0], o[1], o[2], o[3]);
  } else {
    for (long long j = i; j < n; ++j) {
      const float x = bf2f(a[j]), y = bf2f(b[j]);
      out[j] = f2bf(op ? x * y : x + y);
    }
  }
}

// ---- da = g * b, db = g * a (multiply backward, one pass) ----------------------------
__global__ __launch_bounds__(CB_THREADS) void ew_mul_bwd_kernel(const bf16* __restrict__ g, const bf16* __restrict__ a,
                                                                const bf16* __restrict__ b, bf16* __restrict__ da,
                                                                bf16* __restrict__ db, long long n) {
  const long long i = ((long long)blockIdx.x * CB_THREADS + threadIdx.x) * 8;
  if (i + 8 <= n) {
    const uint4 vg = *(const uint4*)(g + i), va = *(const uint4*)(a + i), vb = *(const uint4*)(b + i);
    const unsigned xg[4] = {vg.x, vg.y, vg.z, vg.w}, xa[4] = {va.x, va.y, va.z, va.w}, xb[4] = {vb.x, vb.y, vb.z, vb.w};
    unsigned oa[4], ob[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      oa[k] = cb_pack(cb_lo(xg[k]) * cb_lo(xb[k]), cb_hi(xg[k]) * cb_hi(xb[k]));
      ob[k] = cb_pack(cb_lo(xg[k]) * cb_lo(xa[k]), cb_hi(xg[k]) * cb_hi(xa[k]));
    }
    *(uint4*)(da + i) = make_uint4(oa[0], oa[1], oa[2], oa[3]);
    *(uint4*)(db + i) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
  } else {
    for (long long j = i; j < n; ++j) {
      const float x = bf2f(g[j]);
      da[j] = f2bf(x * bf2f(b[j]));
      db[j] = f2bf(x * bf2f(a[j]));
    }
  }
}

// ---- concat of two tensors along one axis: [outer][ia] ++ [outer][ib] -> [outer][ia+ib]
// dir 0: out <- (a, b);  dir 1: (a, b) <- out (the gradient split)
__global__ __launch_bounds__(CB_THREADS) void concat2_kernel(bf16* __restrict__ a, bf16* __restrict__ b,
                                                             bf16* __restrict__ out, long long outer, int ia, int ib,
                                                             int vec, int dir) {
  const int io = ia + ib;
  const int step = vec ? 8 : 1;
  const long long chunks = outer * (io / step);
  const long long c = (long long)blockIdx.x * CB_THREADS + threadIdx.x;
  if (c >= chunks) return;
  const long long row = c / (io / step);
  const int col = (int)(c % (io / step)) * step;
  bf16* o = out + row * io + col;
  bf16* s = col < ia ? a + row * ia + col : b + row * ib + (col - ia);
  if (vec) {
    if (dir == 0) *(uint4*)o = *(const uint4*)s;
    else *(uint4*)s = *(const uint4*)o;
  } else {
    if (dir == 0) *o = *s;
    else *s = *o;
  }
}

// ---- zero padding of a channels-last [N][D][H][W][C] grid by (pd, ph, pw) per side ----
// dir 0: out [N][D+2pd][H+2ph][W+2pw][C] <- x (border zeros written in the same pass)
// dir 1: x <- the interior of out (the gradient crop)
__global__ __launch_bounds__(CB_THREADS) void pad3_kernel(bf16* __restrict__ x, bf16* __restrict__ out, int N, int D,
                                                          int H, int W, int C, int pd, int ph, int pw, int vec,
                                                          int dir) {
  const int OD = D + 2 * pd, OH = H + 2 * ph, OW = W + 2 * pw;
  const int step = vec ? 8 : 1;
  const int cc = C / step;
  const long long total = dir == 0 ? (long long)N * OD * OH * OW * cc : (long long)N * D * H * W * cc;
  const long long i = (long long)blockIdx.x * CB_THREADS + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % cc) * step;
  long long p = i / cc;
  if (dir == 0) {
    const int ow = (int)(p % OW); p /= OW;
    const int oh = (int)(p % OH); p /= OH;
    const int od = (int)(p % OD);
    const int n = (int)(p / OD);
    const int d = od - pd, h = oh - ph, w = ow - pw;
    const bool in = (unsigned)d < (unsigned)D && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    bf16* o = out + ((((long long)n * OD + od) * OH + oh) * OW + ow) * C + c;
    const bf16* s = x + ((((long long)n * D + d) * H + h) * W + w) * C + c;
    if (vec) {
      *(uint4*)o = in ? *(const uint4*)s : make_uint4(0u, 0u, 0u, 0u);
    } else {
      *o = in ? *s : f2bf(0.f);
    }
  } else {
    const int w = (int)(p % W); p /= W;
    const int h = (int)(p % H); p /= H;
    const int d = (int)(p % D);
    const int n = (int)(p / D);
    const bf16* s = out + ((((long long)n * OD + d + pd) * OH + h + ph) * OW + w + pw) * C + c;
    bf16* o = x + ((((long long)n * D + d) * H + h) * W + w) * C + c;
    if (vec) *(uint4*)o = *(const uint4*)s;
    else *o = *s;
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
// ---- channel padding: [rows][C] <-> [rows][CP] (CP a multiple of 8, CP >= C) ----------
// dir 0: out[r][c] = c < C ? x[r][c] : 0 -- one 16-B store per thread (NAS convs with
//        C % 8 != 0 then gather 16-B channel vectors instead of single elements);
// dir 1: x[r][c] = out[r][c] for c < C (the gradient of the padding, a crop).
__global__ __launch_bounds__(CB_THREADS) void pad_channels_kernel(bf16* __restrict__ x, bf16* __restrict__ out,
                                                                  long long rows, int C, int CP, int dir) {
  const int cc = CP >> 3;
  const long long i = (long long)blockIdx.x * CB_THREADS + threadIdx.x;
  if (i >= rows * cc) return;
  const long long r = i / cc;
  const int c0 = (int)(i - r * cc) * 8;
  const unsigned short* xs = reinterpret_cast<const unsigned short*>(x) + r * C;
  unsigned short* os = reinterpret_cast<unsigned short*>(out) + r * CP + c0;
  if (dir == 0) {
    unsigned short v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = c0 + j < C ? xs[c0 + j] : (unsigned short)0;
    *reinterpret_cast<uint4*>(os) = make_uint4(v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                                               v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16));
  } else {
    const uint4 q = *reinterpret_cast<const uint4*>(os);
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
    unsigned short* xd = reinterpret_cast<unsigned short*>(x) + r * C;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c0 + j < C) xd[c0 + j] = (unsigned short)(w[j >> 1] >> (16 * (j & 1)));
  }
}

static unsigned cb_blocks(long long items) { return (unsigned)((items + CB_THREADS - 1) / CB_THREADS); }

extern "C" int fn_ew_binary(const void* a, const void* b, void* out, long long n, int op, hipStream_t st) {
  if (n <= 0 || (op != 0 && op != 1)) return -2;
  hipLaunchKernelGGL(ew_binary_kernel, dim3(cb_blocks((n + 7) / 8)), dim3(CB_THREADS), 0, st, (const bf16*)a,
                     (const bf16*)b, (bf16*)out, n, op);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_ew_mul_bwd(const void* g, const void* a, const void* b, void* da, void* db, long long n,
                             hipStream_t st) {
  if (n <= 0) return -2;
  hipLaunchKernelGGL(ew_mul_bwd_kernel, dim3(cb_blocks((n + 7) / 8)), dim3(CB_THREADS), 0, st, (const bf16*)g,
                     (const bf16*)a, (const bf16*)b, (bf16*)da, (bf16*)db, n);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_concat2(void* a, void* b, void* out, long long outer, int ia, int ib, int dir, hipStream_t st) {
  if (outer <= 0 || ia <= 0 || ib <= 0 || (dir != 0 && dir != 1)) return -2;
  const int vec = (ia % 8 == 0 && ib % 8 == 0) ? 1 : 0;
  const long long chunks = outer * ((ia + ib) / (vec ? 8 : 1));
  hipLaunchKernelGGL(concat2_kernel, dim3(cb_blocks(chunks)), dim3(CB_THREADS), 0, st, (bf16*)a, (bf16*)b, (bf16*)out,
                     outer, ia, ib, vec, dir);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_pad3(void* x, void* out, const int* g8, int dir, hipStream_t st) {
  const int N = g8[0], D = g8[1], H = g8[2], W = g8[3], C = g8[4], pd = g8[5], ph = g8[6], pw = g8[7];
  if (N <= 0 || C <= 0 || pd < 0 || ph < 0 || pw < 0 || (dir != 0 && dir != 1)) return -2;
  const int vec = C % 8 == 0 ? 1 : 0;
  const long long cc = C / (vec ? 8 : 1);
  const long long total = dir == 0 ? (long long)N * (D + 2 * pd) * (H + 2 * ph) * (W + 2 * pw) * cc
                                   : (long long)N * D * H * W * cc;
  hipLaunchKernelGGL(pad3_kernel, dim3(cb_blocks(total)), dim3(CB_THREADS), 0, st, (bf16*)x, (bf16*)out, N, D, H, W,
                     C, pd, ph, pw, vec, dir);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_pad_channels(void* x, void* out, long long rows, int C, int CP, int dir, hipStream_t st) {
  if (rows <= 0 || C <= 0 || CP < C || CP % 8 || (dir != 0 && dir != 1)) return -2;
  hipLaunchKernelGGL(pad_channels_kernel, dim3(cb_blocks(rows * (CP / 8))), dim3(CB_THREADS), 0, st, (bf16*)x,
                     (bf16*)out, rows, C, CP, dir);
  FN_CHECK_LAUNCH();
  return 0;
}
