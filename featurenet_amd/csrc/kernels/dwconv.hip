// Depthwise convolution (Keras DepthwiseConv2D / the first half of
// SeparableConv2D, reference model/input.py:296-306), channels-last, depth
// multiplier 1.  No MFMA: a depthwise conv has no reduction over channels, so
// it is a VALU/bandwidth kernel.  One thread owns VW consecutive channels of
// one output position (16-B vector loads for VW = 8), loops over the taps
// with clamped-address loads, and fuses bias + activation.
//   fwd  : y[m][c]  = act(b[c] + sum_tap x[pos(m)+tap][c] * w[c][tap])
//   dgrad: dx[p][c] = sum_tap sum_{o: o*s - pad + tap*dil = p} dy[o][c] * w[c][tap]
//   wgrad: dw[c][tap] = sum_m dy[m][c] * x[pos(m)+tap][c]  (block-reduced, per-split partials)
#include "common.h"

struct DwGeom {
  int N, D, H, W, C;
  int OD, OH, OW;
  int KD, KH, KW;
  int sd, sh, sw;
  int pd, ph, pw;
  int dd, dh, dw;
};

template <int VW>
struct Vec {
  float v[VW];
};

template <int VW>
__device__ __forceinline__ void load_vec(const bf16* p, bool ok, float* out) {
  if constexpr (VW == 8) {
    Pack8 u;
    u.u = ok ? *(const uint4*)p : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = bf2f(u.e[j]);
  } else {
    out[0] = ok ? bf2f(*p) : 0.f;
  }
}

template <int VW, int ACT, bool HB>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias, bf16* __restrict__ y, DwGeom g,
                                                     long long total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cg = g.C / VW;
  const int c0 = (int)(i % cg) * VW;
  long long m = i / cg;
  const int ow = (int)(m % g.OW); m /= g.OW;
  const int oh = (int)(m % g.OH); m /= g.OH;
  const int od = (int)(m % g.OD);
  const long long n = m / g.OD;
  const int T = g.KD * g.KH * g.KW;
  float acc[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) acc[j] = HB ? bias[c0 + j] : 0.f;
  for (int kd = 0; kd < g.KD; ++kd) {
    const int id = od * g.sd - g.pd + kd * g.dd;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.sh - g.ph + kh * g.dh;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.sw - g.pw + kw * g.dw;
        const bool ok = (unsigned)id < (unsigned)g.D && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const long long off = ok ? ((((n * g.D + id) * g.H + ih) * g.W + iw) * g.C + c0) : 0;
        float xv[VW];
        load_vec<VW>(x + off, ok, xv);
        const int t = (kd * g.KH + kh) * g.KW + kw;
#pragma unroll
        for (int j = 0; j < VW; ++j) acc[j] += xv[j] * w[(long long)(c0 + j) * T + t];
      }
    }
  }
  const long long o = i / cg * g.C + c0;
  if constexpr (VW == 8) {
    Pack8 u;
#pragma unroll
    for (int j = 0; j < 8; ++j) u.e[j] = f2bf(act_fwd(acc[j], ACT));
    *(uint4*)(y + o) = u.u;
  } else {
    y[o] = f2bf(act_fwd(acc[0], ACT));
  }
}

template <int VW>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const bf16* __restrict__ dy, const float* __restrict__ w,
                                                       bf16* __restrict__ dx, DwGeom g, long long total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cg = g.C / VW;
  const int c0 = (int)(i % cg) * VW;
  long long m = i / cg;
  const int iw = (int)(m % g.W); m /= g.W;
  const int ih = (int)(m % g.H); m /= g.H;
  const int id = (int)(m % g.D);
  const long long n = m / g.D;
  const int T = g.KD * g.KH * g.KW;
  float acc[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) acc[j] = 0.f;
  for (int kd = 0; kd < g.KD; ++kd) {
    const int td = id + g.pd - kd * g.dd;
    const int od = td / g.sd;
    if (td < 0 || td % g.sd || od >= g.OD) continue;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int th = ih + g.ph - kh * g.dh;
      const int oh = th / g.sh;
      if (th < 0 || th % g.sh || oh >= g.OH) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int tw = iw + g.pw - kw * g.dw;
        const int ow = tw / g.sw;
        if (tw < 0 || tw % g.sw || ow >= g.OW) continue;
        float dv[VW];
        load_vec<VW>(dy + (((n * g.OD + od) * g.OH + oh) * g.OW + ow) * g.C + c0, true, dv);
        const int t = (kd * g.KH + kh) * g.KW + kw;
#pragma unroll
        for (int j = 0; j < VW; ++j) acc[j] += dv[j] * w[(long long)(c0 + j) * T + t];
      }
    }
  }
  const long long o = i / cg * g.C + c0;
  if constexpr (VW == 8) {
    Pack8 u;
#pragma unroll
    for (int j = 0; j < 8; ++j) u.e[j] = f2bf(acc[j]);
    *(uint4*)(dx + o) = u.u;
  } else {
    dx[o] = f2bf(acc[0]);
  }
}

// grid: (taps, C/VW, splits); each block reduces a contiguous range of output positions.
template <int VW>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                       float* __restrict__ dw, DwGeom g, long long M,
                                                       long long per_split) {
  __shared__ float red[VW][256 / 64];
  const int t = blockIdx.x;
  const int c0 = blockIdx.y * VW;
  const int kw = t % g.KW, kh = (t / g.KW) % g.KH, kd = t / (g.KW * g.KH);
  const int T = g.KD * g.KH * g.KW;
  const long long mb = (long long)blockIdx.z * per_split;
  const long long me = mb + per_split < M ? mb + per_split : M;
  float acc[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) acc[j] = 0.f;
  for (long long m = mb + threadIdx.x; m < me; m += 256) {
    long long r = m;
    const int ow = (int)(r % g.OW); r /= g.OW;
    const int oh = (int)(r % g.OH); r /= g.OH;
    const int od = (int)(r % g.OD);
    const long long n = r / g.OD;
    const int id = od * g.sd - g.pd + kd * g.dd, ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
    const bool ok = (unsigned)id < (unsigned)g.D && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    float xv[VW], dv[VW];
    load_vec<VW>(x + (ok ? (((n * g.D + id) * g.H + ih) * g.W + iw) * g.C + c0 : 0), ok, xv);
    load_vec<VW>(dy + m * g.C + c0, true, dv);
#pragma unroll
    for (int j = 0; j < VW; ++j) acc[j] += xv[j] * dv[j];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    const float s = wave_sum(acc[j]);
    if (lane == 0) red[j][wave] = s;
  }
  __syncthreads();
  if (threadIdx.x < VW) {
    const int j = threadIdx.x;
    // this split's partial row (fn_part_reduce adds the splits in a fixed order)
    dw[(long long)blockIdx.z * g.C * T + (long long)(c0 + j) * T + t] = red[j][0] + red[j][1] + red[j][2] + red[j][3];
  }
}

static DwGeom parse_dw(const int* v) {
  DwGeom g;
  g.N = v[0]; g.D = v[1]; g.H = v[2]; g.W = v[3]; g.C = v[4];
  g.OD = v[5]; g.OH = v[6]; g.OW = v[7];
  g.KD = v[8]; g.KH = v[9]; g.KW = v[10];
  g.sd = v[11]; g.sh = v[12]; g.sw = v[13];
  g.pd = v[14]; g.ph = v[15]; g.pw = v[16];
  g.dd = v[17]; g.dh = v[18]; g.dw = v[19];
  return g;
}

extern "C" int fn_dw_fwd(const void* x, const float* w, const float* bias, void* y, const int* geom20, int act,
                         hipStream_t st) {
  const DwGeom g = parse_dw(geom20);
  const bool v8 = g.C % 8 == 0;
  const long long total = (long long)g.N * g.OD * g.OH * g.OW * (v8 ? g.C / 8 : g.C);
  const dim3 grid((unsigned)((total + 255) / 256));
  const bf16* xs = (const bf16*)x;
  bf16* ys = (bf16*)y;
  const bool hb = bias != nullptr;
#define DWF(VW, A)                                                                                          \
  do {                                                                                                      \
    if (hb) hipLaunchKernelGGL((dw_fwd_kernel<VW, A, true>), grid, dim3(256), 0, st, xs, w, bias, ys, g, total); \
    else hipLaunchKernelGGL((dw_fwd_kernel<VW, A, false>), grid, dim3(256), 0, st, xs, w, bias, ys, g, total);  \
  } while (0)
#define DWA(VW)                                  \
  do {                                           \
    if (act == ACT_RELU) DWF(VW, ACT_RELU);      \
    else if (act == ACT_TANH) DWF(VW, ACT_TANH); \
    else if (act == ACT_SIGMOID) DWF(VW, ACT_SIGMOID); \
    else DWF(VW, ACT_NONE);                      \
  } while (0)
  if (v8) DWA(8); else DWA(1);
#undef DWA
#undef DWF
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_dw_dgrad(const void* dy, const float* w, void* dx, const int* geom20, hipStream_t st) {
  const DwGeom g = parse_dw(geom20);
  const bool v8 = g.C % 8 == 0;
  const long long total = (long long)g.N * g.D * g.H * g.W * (v8 ? g.C / 8 : g.C);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (v8) hipLaunchKernelGGL((dw_dgrad_kernel<8>), grid, dim3(256), 0, st, (const bf16*)dy, w, (bf16*)dx, g, total);
  else hipLaunchKernelGGL((dw_dgrad_kernel<1>), grid, dim3(256), 0, st, (const bf16*)dy, w, (bf16*)dx, g, total);
  FN_CHECK_LAUNCH();
  return 0;
}

// dw: fp32 [C][taps], accumulated into (+=); part: fp32 scratch [splits][C][taps]
extern "C" int fn_dw_wgrad(const void* dy, const void* x, float* dw, const int* geom20, int splits, hipStream_t st,
                           float* part) {
  const DwGeom g = parse_dw(geom20);
  if (!part || splits < 1) return -6;
  const bool v8 = g.C % 8 == 0;
  const long long M = (long long)g.N * g.OD * g.OH * g.OW;
  const long long per = (M + splits - 1) / splits;
  const dim3 grid((unsigned)(g.KD * g.KH * g.KW), (unsigned)(v8 ? g.C / 8 : g.C), (unsigned)splits);
  if (v8) hipLaunchKernelGGL((dw_wgrad_kernel<8>), grid, dim3(256), 0, st, (const bf16*)dy, (const bf16*)x, part, g, M, per);
  else hipLaunchKernelGGL((dw_wgrad_kernel<1>), grid, dim3(256), 0, st, (const bf16*)dy, (const bf16*)x, part, g, M, per);
  FN_CHECK_LAUNCH();
  return fn_part_reduce(part, dw, (long long)g.C * g.KD * g.KH * g.KW, splits, 1, st);
}
