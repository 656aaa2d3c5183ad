// BatchNorm(+activation) and pooling kernels, channels-last, bf16 I/O, fp32 math.
//
// Forward training path of a BN layer that follows an implicit-GEMM conv:
//   conv epilogue -> per-block (sum, sumsq) slabs  (conv_igemm.hip, STATS=true)
//   bn_finalize   -> mean / invstd / scale / shift + running-stat update
//   bn_apply      -> z = act(y*scale + shift)          (or fused into pooling)
// Backward:
//   bn_bwd_reduce -> per-block (sum g, sum g*xhat) slabs, g = dz * act'(z)
//   bn_finalize   -> dbeta / dgamma
//   bn_bwd_apply  -> dy = gamma*invstd*(g - dbeta/M - xhat*dgamma/M)
// MaxPool/AvgPool take an optional BN+act prologue so the normalised
// activation of the layer feeding a pool is never written to HBM
// (FeatureNet-3D conv4 -> BN -> ReLU -> MaxPool3d is one read of y4).
#include "common.h"

#include <algorithm>
#include <type_traits>

// ---------------------------------------------------------------------------
// Column statistics: per-block partial sums over rows of a [M][C] tensor.
//   MODE 0: (sum x, sum x^2)                       -- forward stats
//   MODE 1: (sum g, sum g*xhat), g = dz*act'(z)     -- BN backward
// VW = channels per thread (8 -> 16-B vector loads, 1 -> scalar fallback).
// ---------------------------------------------------------------------------
template <int VW, int MODE, int ACT>
__global__ __launch_bounds__(256) void colstats_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dz,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       const float* __restrict__ mean, const float* __restrict__ invstd,
                                                       float* __restrict__ part, long long M, int C,
                                                       long long rows_per_block) {
  constexpr int act = ACT;          // compile-time activation: no per-element switch
  __shared__ float red[256][2 * VW + 1];
  const int tid = threadIdx.x;
  const int cpr = C / VW;           // chunks per row
  const int rpp = 256 / cpr;        // rows per pass
  const bool active = tid < rpp * cpr;
  const int ch = active ? tid % cpr : 0;
  const int r0 = active ? tid / cpr : 0;
  const long long mbeg = (long long)blockIdx.x * rows_per_block;
  long long mend = mbeg + rows_per_block;
  if (mend > M) mend = M;
  float s0[VW], s1[VW], sc[VW], sh[VW], mu[VW], is[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    s0[j] = 0.f; s1[j] = 0.f;
    if (MODE == 1 && active) {
      const int c = ch * VW + j;
      sc[j] = scale[c]; sh[j] = shift[c]; mu[j] = mean[c]; is[j] = invstd[c];
    }
  }
  if (active) {
#pragma unroll 4
    for (long long m = mbeg + r0; m < mend; m += rpp) {
      const long long off = m * C + (long long)ch * VW;
      if constexpr (VW == 8) {
        Pack8 px;
        px.u = *(const uint4*)(x + off);
        if constexpr (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { const float v = bf2f(px.e[j]); s0[j] += v; s1[j] += v * v; }
        } else {
          Pack8 pd;
          pd.u = *(const uint4*)(dz + off);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float y = bf2f(px.e[j]);
            const float z = act_fwd(y * sc[j] + sh[j], act);
            const float g = bf2f(pd.e[j]) * act_bwd_from_out(z, act);
            s0[j] += g;
            s1[j] += g * (y - mu[j]) * is[j];
          }
        }
      } else {
        const float y = bf2f(x[off]);
        if constexpr (MODE == 0) { s0[0] += y; s1[0] += y * y; }
        else {
          const float z = act_fwd(y * sc[0] + sh[0], act);
          const float g = bf2f(dz[off]) * act_bwd_from_out(z, act);
          s0[0] += g;
          s1[0] += g * (y - mu[0]) * is[0];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VW; ++j) { red[tid][j] = active ? s0[j] : 0.f; red[tid][VW + j] = active ? s1[j] : 0.f; }
  __syncthreads();
  // one thread per channel sums the rpp partials that share its chunk
  for (int c = tid; c < C; c += 256) {
    const int chk = c / VW, j = c % VW;
    float a = 0.f, b = 0.f;
    for (int i = 0; i < rpp; ++i) { a += red[i * cpr + chk][j]; b += red[i * cpr + chk][VW + j]; }
    part[(long long)blockIdx.x * 2 * C + c] = a;
    part[(long long)blockIdx.x * 2 * C + C + c] = b;
  }
}

// Column sums (MODE 0) of a [M][C] tensor whose C is not a multiple of 8 (bias gradients of
// 25-class heads, odd NAS widths): 16-B vector loads over "super rows" of lcm(8, C) elements
// = Q = C / gcd(8, C) chunks, in which chunk q always covers channels (8q + j) mod C -- so a
// thread that keeps chunk position q keeps 8 fixed channels, like the VW = 8 path.  Needs
// M * C to be whole super rows (the host checks) and Q <= 256.
__global__ __launch_bounds__(256) void colstats_sr_kernel(const bf16* __restrict__ x, float* __restrict__ part,
                                                          long long nsr, int C, int Q, long long sr_per_block) {
  __shared__ float red[256][17];
  const int tid = threadIdx.x;
  const int rpp = 256 / Q;                   // super rows per pass
  const bool active = tid < rpp * Q;
  const int q = active ? tid % Q : 0, r0 = active ? tid / Q : 0;
  const long long sbeg = (long long)blockIdx.x * sr_per_block;
  long long send = sbeg + sr_per_block;
  if (send > nsr) send = nsr;
  float s0[8], s1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
  if (active) {
#pragma unroll 4
    for (long long r = sbeg + r0; r < send; r += rpp) {
      Pack8 px;
      px.u = *(const uint4*)(x + (r * Q + q) * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float v = bf2f(px.e[j]); s0[j] += v; s1[j] += v * v; }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[tid][j] = active ? s0[j] : 0.f; red[tid][8 + j] = active ? s1[j] : 0.f; }
  __syncthreads();
  // (1) per chunk position q: sum the rpp threads that held it (fixed order)
  __shared__ float red2[256][17];
  if (tid < Q) {
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = 0.f;
    for (int r = 0; r < rpp; ++r)
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] += red[r * Q + tid][j];
#pragma unroll
    for (int j = 0; j < 16; ++j) red2[tid][j] = a[j];
  }
  __syncthreads();
  // (2) channel c sits at super-row offsets e = c + C*i, i < 8/gcd(8, C) (<= 8 terms)
  for (int c = tid; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int e = c; e < 8 * Q; e += C) {
      a += red2[e >> 3][e & 7];
      b += red2[e >> 3][8 + (e & 7)];
    }
    part[(long long)blockIdx.x * 2 * C + c] = a;
    part[(long long)blockIdx.x * 2 * C + C + c] = b;
  }
}

// ---------------------------------------------------------------------------
// Reduce [nb][2][C] slabs per channel in fp64 and finalise.
//   MODE 0 (forward): mean, invstd, scale=gamma*invstd, shift=beta-mean*scale,
//                     running stats update (unbiased var, Keras/torch style).
//   MODE 1 (backward): out0 = dbeta = sum g, out1 = dgamma = sum g*xhat.
// One 256-thread block per channel.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ part, int nb, int C, double count,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          float momentum, float eps, float* __restrict__ out0,
                                                          float* __restrict__ out1, float* __restrict__ out2,
                                                          float* __restrict__ out3) {
  __shared__ double sa[256], sb[256];
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
#pragma unroll 4   // (the conv_tile chunk slabs have thousands of rows: keep several loads in flight)
  for (int i = threadIdx.x; i < nb; i += 256) {
    a += (double)part[(long long)i * 2 * C + c];
    b += (double)part[(long long)i * 2 * C + C + c];
  }
  sa[threadIdx.x] = a; sb[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) { sa[threadIdx.x] += sa[threadIdx.x + s]; sb[threadIdx.x] += sb[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (MODE == 0) {
      const double mean = sa[0] / count;
      double var = sb[0] / count - mean * mean;
      if (var < 0.0) var = 0.0;
      const float invstd = (float)(1.0 / sqrt(var + (double)eps));
      const float g = gamma ? gamma[c] : 1.f;
      const float bt = beta ? beta[c] : 0.f;
      out0[c] = (float)mean;
      out1[c] = invstd;
      out2[c] = g * invstd;
      out3[c] = bt - (float)mean * g * invstd;
      if (run_mean) {
        const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
      }
    } else if (MODE == 1) {
      out0[c] = (float)sa[0];
      out1[c] = (float)sb[0];
    } else {
      // MODE 2: raw backward moments (sum g, sum g*y) from the conv_tile dgrad epilogue; the
      // mean / invstd of the forward pass come in run_mean / run_var (read only):
      // dbeta = sum g, dgamma = sum g*xhat = invstd * (sum g*y - mean * sum g), in fp64
      out0[c] = (float)sa[0];
      out1[c] = (float)((double)run_var[c] * (sb[0] - (double)run_mean[c] * sa[0]));
    }
  }
}

// z = act(y*scale + shift)
// When the channel-chunk count divides 256 (C = 8..2048 powers of two) every
// thread keeps ONE channel chunk for the whole grid-stride loop, so the
// per-channel parameters live in registers and no 64-bit modulo runs per
// element.
// mask (VW = 8, fixed-chunk path only; host-checked): also one byte per 8-channel chunk, bit j =
// (z_j > 0) -- the relu mask of the BN-backward statistics identity (bn_bwd_prep_kernel), which
// the consuming conv's dgrad epilogue applies to dz
template <int VW, int ACT>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, bf16* __restrict__ z,
                                                       long long total, int C, unsigned char* __restrict__ mask) {
  constexpr int act = ACT;
  const long long nvec = total / VW;
  const int cpr = C / VW;
  const long long stride = (long long)gridDim.x * 256;
  const long long i0 = blockIdx.x * 256LL + threadIdx.x;
  if ((256 % cpr) == 0) {
    const int c0 = (int)(threadIdx.x % cpr) * VW;
    float sc[VW], sh[VW];
#pragma unroll
    for (int j = 0; j < VW; ++j) { sc[j] = scale[c0 + j]; sh[j] = shift[c0 + j]; }
#pragma unroll 2
    for (long long i = i0; i < nvec; i += stride) {
      Pack8 p;
      if constexpr (VW == 8) p.u = *(const uint4*)(y + i * 8); else p.e[0] = y[i];
      unsigned bits = 0;
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const float v = act_fwd(bf2f(p.e[j]) * sc[j] + sh[j], act);
        bits |= (v > 0.f ? 1u : 0u) << j;
        p.e[j] = f2bf(v);
      }
      if constexpr (VW == 8) *(uint4*)(z + i * 8) = p.u; else z[i] = p.e[0];
      if (mask) mask[i] = (unsigned char)bits;
    }
    return;
  }
  for (long long i = i0; i < nvec; i += stride) {
    const int c0 = (int)((i * VW) % C);
    Pack8 p;
    if constexpr (VW == 8) p.u = *(const uint4*)(y + i * 8); else p.e[0] = y[i];
#pragma unroll
    for (int j = 0; j < VW; ++j) p.e[j] = f2bf(act_fwd(bf2f(p.e[j]) * scale[c0 + j] + shift[c0 + j], act));
    if constexpr (VW == 8) *(uint4*)(z + i * 8) = p.u; else z[i] = p.e[0];
  }
}

// dy = gamma*invstd*(g - dbeta/M - xhat*dgamma/M), g = dz*act'(z)
//    = k1*g + k2*y + k3 per channel with k1 = scale,
//      k2 = -scale*invstd*dgamma/M, k3 = -scale*(dbeta/M - mean*invstd*dgamma/M)
template <int VW, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ y,
                                                           const float* __restrict__ scale, const float* __restrict__ shift,
                                                           const float* __restrict__ mean, const float* __restrict__ invstd,
                                                           const float* __restrict__ dbeta, const float* __restrict__ dgamma,
                                                           bf16* __restrict__ dy, long long total, int C, float inv_count) {
  constexpr int act = ACT;
  const long long nvec = total / VW;
  const int cpr = C / VW;
  const long long stride = (long long)gridDim.x * 256;
  const long long i0 = blockIdx.x * 256LL + threadIdx.x;
  const bool fixed = (256 % cpr) == 0;
  float sc[VW], sh[VW], k2[VW], k3[VW];
  auto load_params = [&](int c0) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const int c = c0 + j;
      sc[j] = scale[c];
      sh[j] = shift[c];
      const float is = invstd[c];
      k2[j] = -sc[j] * is * dgamma[c] * inv_count;
      k3[j] = -sc[j] * (dbeta[c] * inv_count - mean[c] * is * dgamma[c] * inv_count);
    }
  };
  if (fixed) load_params((int)(threadIdx.x % cpr) * VW);
#pragma unroll 2
  for (long long i = i0; i < nvec; i += stride) {
    if (!fixed) load_params((int)((i * VW) % C));
    Pack8 py, pd, po;
    if constexpr (VW == 8) {
      py.u = *(const uint4*)(y + i * 8);
      pd.u = *(const uint4*)(dz + i * 8);
    } else {
      py.e[0] = y[i];
      pd.e[0] = dz[i];
    }
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const float yv = bf2f(py.e[j]);
      const float zv = act_fwd(yv * sc[j] + sh[j], act);
      const float g = bf2f(pd.e[j]) * act_bwd_from_out(zv, act);
      po.e[j] = f2bf(sc[j] * g + k2[j] * yv + k3[j]);
    }
    if constexpr (VW == 8) *(uint4*)(dy + i * 8) = po.u;
    else dy[i] = po.e[0];
  }
}

// ---------------------------------------------------------------------------
// BN backward without the colstats pass over (dz, y): the statistics identity.
//
// z = relu(bn(y)) feeds a conv (weights W [K][T][C], weight gradient dW, both fp32 [K*T][C]);
// its dgrad gives dz = conv^T(dy', W).  Per input channel c the adjoint identity
//     sum_p dz[p,c] * z[p,c] = sum_{k,t} W[k,t,c] * dW[k,t,c]
// holds exactly (dW = sum_q dy'[q,k] z[q+t,c]), so with g = dz * relu'(z) and, where
// relu' = 1, z = gamma * xhat + beta:
//     gamma * sum g*xhat = S - beta * sum g,      S = sum_{k,t} W * dW
// The consuming conv's dgrad epilogue sums g (dz masked by the bit mask bn_apply wrote; dz is
// stored unmasked, the true gradient of z); bn_wdot_kernel gives S; bn_bwd_prep_kernel the
// apply constants
//     dy = k1*g + k2*y + k3,  k1 = scale, k2 = -invstd^2 * G / M,
//                            k3 = -scale * sum g / M + mean * invstd^2 * G / M,  G = S - beta sum g
// (no division by gamma; channels whose gamma is too small against beta for z's bf16 resolution
// take G from (g, y) directly, see bn_bwd_prep_kernel).  dgamma itself, only read by the
// optimizer, is summed exactly from (g, y) inside the apply pass (bn_bwd_apply_k_kernel).
// W is rounded to bf16 as the dgrad's packed weights are.
// ---------------------------------------------------------------------------

// per-block partial sums part[block][c] = sum_rows bf16(W[r][c]) * dW[r][c] over rows of [R][C]
// (C divides 256: a thread keeps one channel)
__global__ __launch_bounds__(256) void bn_wdot_kernel(const float* __restrict__ w, const float* __restrict__ dw,
                                                      float* __restrict__ part, int R, int C, int rows_per_block) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int c = tid % C, r0 = tid / C, rpp = 256 / C;
  const int rb = blockIdx.x * rows_per_block;
  int re = rb + rows_per_block;
  if (re > R) re = R;
  float a = 0.f;
  for (int r = rb + r0; r < re; r += rpp) {
    const long long o = (long long)r * C + c;
    a += (float)(bf16)w[o] * dw[o];
  }
  red[tid] = a;
  __syncthreads();
  if (tid < C) {
    float t = 0.f;
    for (int i = 0; i < rpp; ++i) t += red[i * C + tid];
    part[(long long)blockIdx.x * C + tid] = t;
  }
}

// One block per channel: sum g (the dgrad epilogue's slab rows, [nbg][2][C] row 0) and S (the
// wdot partials [nbw][C]) in fp64 -> dbeta = sum g and the apply constants kc[3][C].
// Conditioning: z is stored in bf16, so S = sum dz * z carries ~2^-9 |z| of rounding per term,
// and G = S - beta * sum g cancels down to gamma * sum g * xhat -- a channel whose |gamma| is
// small against |beta| (z ~ beta: gamma * xhat below z's bf16 resolution) cannot get G from the
// identity.  Such a channel (|gamma| < |beta| / 4) sums g * (y - mean) exactly from g and y
// itself (a strided pass over that one channel: rare, and only the unsafe channels pay it).
__global__ __launch_bounds__(256) void bn_bwd_prep_kernel(const float* __restrict__ gslab, int nbg,
                                                          const float* __restrict__ wpart, int nbw, int C,
                                                          double count, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float* __restrict__ dbeta,
                                                          float* __restrict__ kc, const bf16* __restrict__ g,
                                                          const bf16* __restrict__ y, long long M) {
  __shared__ double sa[256], sb[256];
  const int c = blockIdx.x;
  const double gm = gamma ? (double)gamma[c] : 1.0, bt = beta ? (double)beta[c] : 0.0;
  const bool exact = fabs(gm) < 0.25 * fabs(bt);
  double a = 0.0, b = 0.0;
#pragma unroll 4
  for (int i = threadIdx.x; i < nbg; i += 256) a += (double)gslab[(long long)i * 2 * C + c];
  if (exact) {
    const float mu = mean[c], scf = scale[c], shf = shift[c];
    float t = 0.f;
    for (long long m = threadIdx.x; m < M; m += 256) {
      const float yv = bf2f(y[m * C + c]);
      if (yv * scf + shf > 0.f) t += bf2f(g[m * C + c]) * (yv - mu);
    }
    b = (double)t;                              // sum g * (y - mean), g = dz * relu'
  } else {
    for (int i = threadIdx.x; i < nbw; i += 256) b += (double)wpart[(long long)i * C + c];
  }
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = b;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      sa[threadIdx.x] += sa[threadIdx.x + st];
      sb[threadIdx.x] += sb[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double sg = sa[0];
    const double is = (double)invstd[c], sc = (double)scale[c];
    // G = gamma * sum g * xhat: from the identity, or exactly (gamma * invstd * sum g (y - mean))
    const double G = exact ? gm * is * sb[0] : sb[0] - bt * sg;
    dbeta[c] = (float)sg;
    kc[c] = (float)sc;
    kc[C + c] = (float)(-is * is * G / count);
    kc[2 * C + c] = (float)(-sc * sg / count + (double)mean[c] * is * is * G / count);
  }
}

// dy = k1*g + k2*y + k3 (g = dz * relu'(y * scale + shift)) and the exact dgamma partials
// sum g*(y-mean)*invstd as
// rows part[block][2][C] (row 0 zero; bn_finalize mode 1 turns row 1 into dgamma).  8 channels
// per thread, fixed (C / 8 divides 256, the stride a multiple of 256); grid-stride over a
// resident-sized grid.
__global__ __launch_bounds__(256) void bn_bwd_apply_k_kernel(const bf16* __restrict__ g, const bf16* __restrict__ y,
                                                             const float* __restrict__ kc,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ shift, bf16* __restrict__ dy,
                                                             long long nvec, int C, float* __restrict__ part) {
  const int cpr = C / 8;
  const int tid = threadIdx.x;
  const int c0 = (tid % cpr) * 8;
  float k1[8], k2[8], k3[8], mu[8], sh[8], s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k1[j] = kc[c0 + j];                          // (= scale)
    k2[j] = kc[C + c0 + j];
    k3[j] = kc[2 * C + c0 + j];
    mu[j] = mean[c0 + j];
    sh[j] = shift[c0 + j];
    s[j] = 0.f;
  }
  const long long stride = (long long)gridDim.x * 256;
#pragma unroll 2
  for (long long i = blockIdx.x * 256LL + tid; i < nvec; i += stride) {
    Pack8 pg, py, po;
    pg.u = *(const uint4*)(g + i * 8);
    py.u = *(const uint4*)(y + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float yv = bf2f(py.e[j]);
      const float gv = yv * k1[j] + sh[j] > 0.f ? bf2f(pg.e[j]) : 0.f;   // relu' of z (k1 = scale)
      po.e[j] = f2bf(k1[j] * gv + k2[j] * yv + k3[j]);
      s[j] += gv * (yv - mu[j]);
    }
    *(uint4*)(dy + i * 8) = po.u;
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid][j] = s[j] * invstd[c0 + j];
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int chk = c / 8, j = c % 8;
    float b = 0.f;
    for (int t = chk; t < 256; t += cpr) b += red[t][j];
    part[(long long)blockIdx.x * 2 * C + c] = 0.f;
    part[(long long)blockIdx.x * 2 * C + C + c] = b;
  }
}

// The same BN backward, writing dy in the SHIFTED space-to-depth layout of the sub-pixel
// decoder (ops/subpixel.py): output [N, FD/2+1, FH/2+1, FW/2+1, 8, C], cell c' sub-position
// j' = full-resolution position q = 2c' - 1 + j' (zero where q is outside the grid).
// Output-major: consecutive threads write consecutive 16-B chunks (the whole tensor, border
// zeros included -- no separate fill); the reads are 64-B position rows, adjacent
// sub-positions along W contiguous.  VW = 8 channels per thread, C / 8 dividing 256.
template <int ACT>
__global__ __launch_bounds__(256) void bn_bwd_apply_s2d_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ y,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ dbeta,
                                                               const float* __restrict__ dgamma, bf16* __restrict__ dsh,
                                                               int N, int FD, int FH, int FW, int C, float inv_count) {
  constexpr int act = ACT;
  const int cpr = C / 8;
  const int D2 = FD / 2 + 1, H2 = FH / 2 + 1, W2 = FW / 2 + 1;
  const long long nvec = (long long)N * D2 * H2 * W2 * 8 * cpr;
  const long long stride = (long long)gridDim.x * 256;   // a multiple of cpr: the chunk is fixed
  const long long i0 = blockIdx.x * 256LL + threadIdx.x;
  const int k = (int)(threadIdx.x % cpr);
  float sc[8], sh[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = k * 8 + j;
    sc[j] = scale[c];
    sh[j] = shift[c];
    const float is = invstd[c];
    k2[j] = -sc[j] * is * dgamma[c] * inv_count;
    k3[j] = -sc[j] * (dbeta[c] * inv_count - mean[c] * is * dgamma[c] * inv_count);
  }
  for (long long i = i0; i < nvec; i += stride) {
    const long long s = i / cpr;
    const int jp = (int)(s & 7);
    long long cell = s >> 3;
    const int cw = (int)(cell % W2);
    cell /= W2;
    const int ch = (int)(cell % H2);
    cell /= H2;
    const int cd = (int)(cell % D2);
    const int n = (int)(cell / D2);
    const int qd = 2 * cd - 1 + (jp >> 2), qh = 2 * ch - 1 + ((jp >> 1) & 1), qw = 2 * cw - 1 + (jp & 1);
    Pack8 po;
    if ((unsigned)qd < (unsigned)FD && (unsigned)qh < (unsigned)FH && (unsigned)qw < (unsigned)FW) {
      const long long off = ((((long long)n * FD + qd) * FH + qh) * FW + qw) * C + k * 8;
      Pack8 py, pd;
      py.u = *(const uint4*)(y + off);
      pd.u = *(const uint4*)(dz + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float yv = bf2f(py.e[j]);
        const float zv = act_fwd(yv * sc[j] + sh[j], act);
        const float g = bf2f(pd.e[j]) * act_bwd_from_out(zv, act);
        po.e[j] = f2bf(sc[j] * g + k2[j] * yv + k3[j]);
      }
    } else {
      po.u = make_uint4(0u, 0u, 0u, 0u);
    }
    *(uint4*)(dsh + i * 8) = po.u;
  }
}

// The same pass, one (n, cell-d, cell-h) row of the shifted grid at a time (grid-stride over the
// rows): a row is W2 cells x 8 sub-positions x C / 8 chunks, so every per-chunk index is a shift of
// the thread's offset in the row -- the flat form above spent six 64-bit divisions per 16-B chunk
// (1.28-1.44 ms per seg step, VALU-bound).  Same arithmetic, same bits.
// U: chunks per thread per pass -- ceil(row length / 256) where that is small, so a row is one
// pass (the seg decoder's rows are 1056 chunks: 4 per thread left a 32-chunk second pass per row)
template <int ACT, int LCPR, int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_s2d_rows_kernel(const bf16* __restrict__ dz,
                                                                    const bf16* __restrict__ y,
                                                                    const float* __restrict__ scale,
                                                                    const float* __restrict__ shift,
                                                                    const float* __restrict__ mean,
                                                                    const float* __restrict__ invstd,
                                                                    const float* __restrict__ dbeta,
                                                                    const float* __restrict__ dgamma,
                                                                    bf16* __restrict__ dsh, int N, int FD, int FH,
                                                                    int FW, int C, float inv_count) {
  constexpr int act = ACT;
  constexpr int cpr = 1 << LCPR;
  const int D2 = FD / 2 + 1, H2 = FH / 2 + 1, W2 = FW / 2 + 1;
  const int k = (int)(threadIdx.x & (cpr - 1));   // (256 is a multiple of cpr: the chunk is fixed)
  float sc[8], sh[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = k * 8 + j;
    sc[j] = scale[c];
    sh[j] = shift[c];
    const float is = invstd[c];
    k2[j] = -sc[j] * is * dgamma[c] * inv_count;
    k3[j] = -sc[j] * (dbeta[c] * inv_count - mean[c] * is * dgamma[c] * inv_count);
  }
  const int rowlen = W2 * 8 * cpr;
  const int nrows = N * D2 * H2;
  for (int row = blockIdx.x; row < nrows; row += gridDim.x) {
    const int chh = row % H2, r2 = row / H2;
    const int cd = r2 % D2, n = r2 / D2;
    bf16* orow = dsh + (long long)row * rowlen * 8;
    // U chunks per thread per pass, their 2U loads issued before any is used
    for (int t0 = threadIdx.x; t0 < rowlen; t0 += U * 256) {
      Pack8 py[U], pd[U];
      bool in[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 + u * 256;
        const int jp = (t >> LCPR) & 7, cw = t >> (LCPR + 3);
        const int qd = 2 * cd - 1 + (jp >> 2), qh = 2 * chh - 1 + ((jp >> 1) & 1), qw = 2 * cw - 1 + (jp & 1);
        in[u] = t < rowlen && (unsigned)qd < (unsigned)FD && (unsigned)qh < (unsigned)FH && (unsigned)qw < (unsigned)FW;
        const long long off = in[u] ? ((((long long)n * FD + qd) * FH + qh) * FW + qw) * C + k * 8 : 0;
        py[u].u = *(const uint4*)(y + off);
        pd[u].u = *(const uint4*)(dz + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 + u * 256;
        Pack8 po;
        if (in[u]) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float yv = bf2f(py[u].e[j]);
            const float zv = act_fwd(yv * sc[j] + sh[j], act);
            const float g = bf2f(pd[u].e[j]) * act_bwd_from_out(zv, act);
            po.e[j] = f2bf(sc[j] * g + k2[j] * yv + k3[j]);
          }
        } else {
          po.u = make_uint4(0u, 0u, 0u, 0u);
        }
        if (t < rowlen) *(uint4*)(orow + t * 8) = po.u;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pooling (max / avg), 1-D/2-D/3-D channels-last with optional BN+act prologue.
// geom: N, D, H, W, C, OD, OH, OW, KD, KH, KW, SD, SH, SW, PD, PH, PW
// ---------------------------------------------------------------------------
struct PoolGeom {
  int N, D, H, W, C, OD, OH, OW, KD, KH, KW, sd, sh, sw, pd, ph, pw;
};

__device__ __forceinline__ float load_pre(const bf16* x, long long idx, int c, const float* scale, const float* shift,
                                          int act) {
  float v = bf2f(x[idx]);
  if (scale) v = act_fwd(v * scale[c] + shift[c], act);
  return v;
}

template <int VW>
__global__ __launch_bounds__(256) void pool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ out,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       PoolGeom g, int is_max, int count_pad, int act) {
  const int cpr = g.C / VW;
  const long long total = (long long)g.N * g.OD * g.OH * g.OW * cpr;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % cpr);
    long long t = i / cpr;
    const int ow = (int)(t % g.OW); t /= g.OW;
    const int oh = (int)(t % g.OH); t /= g.OH;
    const int od = (int)(t % g.OD);
    const long long n = t / g.OD;
    float accv[VW];
#pragma unroll
    for (int j = 0; j < VW; ++j) accv[j] = is_max ? -INFINITY : 0.f;
    int cnt = 0;
    for (int kd = 0; kd < g.KD; ++kd) {
      const int id = od * g.sd - g.pd + kd;
      if ((unsigned)id >= (unsigned)g.D) continue;
      for (int kh = 0; kh < g.KH; ++kh) {
        const int ih = oh * g.sh - g.ph + kh;
        if ((unsigned)ih >= (unsigned)g.H) continue;
        for (int kw = 0; kw < g.KW; ++kw) {
          const int iw = ow * g.sw - g.pw + kw;
          if ((unsigned)iw >= (unsigned)g.W) continue;
          ++cnt;
          const long long base = (((n * g.D + id) * g.H + ih) * (long long)g.W + iw) * g.C + ch * VW;
          if constexpr (VW == 8) {
            Pack8 p;
            p.u = *(const uint4*)(x + base);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float v = bf2f(p.e[j]);
              if (scale) v = act_fwd(v * scale[ch * 8 + j] + shift[ch * 8 + j], act);
              accv[j] = is_max ? fmaxf(accv[j], v) : accv[j] + v;
            }
          } else {
            const float v = load_pre(x, base, ch, scale, shift, act);
            accv[0] = is_max ? fmaxf(accv[0], v) : accv[0] + v;
          }
        }
      }
    }
    const float div = count_pad ? (float)(g.KD * g.KH * g.KW) : (float)(cnt > 0 ? cnt : 1);
    const long long ob = i * VW;
    if constexpr (VW == 8) {
      Pack8 p;
#pragma unroll
      for (int j = 0; j < 8; ++j) p.e[j] = f2bf(is_max ? accv[j] : accv[j] / div);
      *(uint4*)(out + ob) = p.u;
    } else {
      out[ob] = f2bf(is_max ? accv[0] : accv[0] / div);
    }
  }
}

// Non-overlapping 2x2x2 (or 1x2x2) windows with 8-channel vectors: the common
// FeatureNet / CNN pooling.  Per-channel BN params live in registers, all window
// loads are issued before the reduction, 32-bit index math.
template <int KD, int ACT = -1>
__global__ __launch_bounds__(256) void pool2_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ out,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        PoolGeom g, int is_max, int act, int total) {
  const int actc = ACT >= 0 ? ACT : act;         // (compile-time relu / none: a runtime switch kept
                                                 //  tanh / sigmoid code in every element's path)
  const int cpr = g.C >> 3;
  // grid-stride over a resident-sized grid (the stride is a multiple of 256, so with
  // 256 % cpr == 0 -- host-checked -- a thread keeps its 8-channel chunk and the BN parameters
  // are loaded once); the next window's loads are issued before this one is reduced
  const int ch = threadIdx.x % cpr;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale ? scale[ch * 8 + j] : 1.f;
    sh[j] = scale ? shift[ch * 8 + j] : 0.f;
  }
  const long long rowW = (long long)g.W * g.C, plane = (long long)g.H * rowW;
  auto origin = [&](int ii) -> long long {
    int t = ii / cpr;
    const int ow = t % g.OW; t /= g.OW;
    const int oh = t % g.OH; t /= g.OH;
    const int od = t % g.OD;
    const int n = t / g.OD;
    return ((long long)(n * g.D + od * KD) * g.H + oh * 2) * rowW + (long long)ow * 2 * g.C + ch * 8;
  };
  auto fetch = [&](long long b0, Pack8* p) {
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int kw = 0; kw < 2; ++kw) p[(kd * 2 + kh) * 2 + kw].u = *(const uint4*)(x + b0 + kd * plane + kh * rowW + kw * g.C);
  };
  const int stride = gridDim.x * 256;
  int i = blockIdx.x * 256 + threadIdx.x;
  Pack8 p[KD * 4];
  if (i < total) fetch(origin(i), p);
  while (i < total) {
    const int inx = i + stride;
    Pack8 p2[KD * 4];
    fetch(origin(inx < total ? inx : i), p2);
    Pack8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float acc = is_max ? -INFINITY : 0.f;
#pragma unroll
      for (int w = 0; w < KD * 4; ++w) {
        float v = bf2f(p[w].e[j]);
        if (scale) v = act_fwd(v * sc[j] + sh[j], actc);
        acc = is_max ? fmaxf(acc, v) : acc + v;
      }
      o.e[j] = f2bf(is_max ? acc : acc * (1.f / (KD * 4)));
    }
    *(uint4*)(out + (long long)i * 8) = o.u;
#pragma unroll
    for (int w = 0; w < KD * 4; ++w) p[w] = p2[w];
    i = inx;
  }
}

// Gather-form backward: every input element collects from the windows that
// contain it (deterministic, no atomics, works for overlapping windows).
// For max pooling the window's arg-max is recomputed (first max wins, matching
// the forward's fmaxf scan order).
template <int VW>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ x,
                                                       bf16* __restrict__ dx, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, PoolGeom g, int is_max,
                                                       int count_pad, int act) {
  const int cpr = g.C / VW;
  const long long total = (long long)g.N * g.D * g.H * g.W * cpr;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % cpr);
    long long t = i / cpr;
    const int iw = (int)(t % g.W); t /= g.W;
    const int ih = (int)(t % g.H); t /= g.H;
    const int id = (int)(t % g.D);
    const long long n = t / g.D;
    float gacc[VW];
    float self[VW];
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      gacc[j] = 0.f;
      const int c = ch * VW + j;
      self[j] = is_max ? load_pre(x, i * VW + j, c, scale, shift, act) : 0.f;
    }
    // output windows covering (id, ih, iw): o*s - p <= i <= o*s - p + k - 1
    const int od0 = max(0, (id + g.pd - g.KD + g.sd) / g.sd), od1 = min(g.OD - 1, (id + g.pd) / g.sd);
    const int oh0 = max(0, (ih + g.ph - g.KH + g.sh) / g.sh), oh1 = min(g.OH - 1, (ih + g.ph) / g.sh);
    const int ow0 = max(0, (iw + g.pw - g.KW + g.sw) / g.sw), ow1 = min(g.OW - 1, (iw + g.pw) / g.sw);
    for (int od = od0; od <= od1; ++od)
      for (int oh = oh0; oh <= oh1; ++oh)
        for (int ow = ow0; ow <= ow1; ++ow) {
          // guard the floor-division edge cases of negative numerators
          if (id < od * g.sd - g.pd || id >= od * g.sd - g.pd + g.KD) continue;
          if (ih < oh * g.sh - g.ph || ih >= oh * g.sh - g.ph + g.KH) continue;
          if (iw < ow * g.sw - g.pw || iw >= ow * g.sw - g.pw + g.KW) continue;
          const long long obase = (((n * g.OD + od) * g.OH + oh) * (long long)g.OW + ow) * g.C + ch * VW;
          if (!is_max) {
            int cnt = g.KD * g.KH * g.KW;
            if (!count_pad) {
              cnt = 0;
              for (int kd = 0; kd < g.KD; ++kd) {
                const int a = od * g.sd - g.pd + kd;
                if ((unsigned)a >= (unsigned)g.D) continue;
                for (int kh = 0; kh < g.KH; ++kh) {
                  const int b = oh * g.sh - g.ph + kh;
                  if ((unsigned)b >= (unsigned)g.H) continue;
                  for (int kw = 0; kw < g.KW; ++kw) {
                    const int cc = ow * g.sw - g.pw + kw;
                    if ((unsigned)cc < (unsigned)g.W) ++cnt;
                  }
                }
              }
            }
            const float inv = 1.f / (float)(cnt > 0 ? cnt : 1);
#pragma unroll
            for (int j = 0; j < VW; ++j) gacc[j] += bf2f(dout[obase + j]) * inv;
          } else {
            // find first arg-max position of this window for each channel
            bool won[VW];
            float best[VW];
#pragma unroll
            for (int j = 0; j < VW; ++j) { best[j] = -INFINITY; won[j] = false; }
            bool done = false;
            for (int kd = 0; kd < g.KD && !done; ++kd) {
              const int a = od * g.sd - g.pd + kd;
              if ((unsigned)a >= (unsigned)g.D) continue;
              for (int kh = 0; kh < g.KH; ++kh) {
                const int b = oh * g.sh - g.ph + kh;
                if ((unsigned)b >= (unsigned)g.H) continue;
                for (int kw = 0; kw < g.KW; ++kw) {
                  const int cc = ow * g.sw - g.pw + kw;
                  if ((unsigned)cc >= (unsigned)g.W) continue;
                  const long long base = (((n * g.D + a) * g.H + b) * (long long)g.W + cc) * g.C + ch * VW;
                  const bool me = (a == id && b == ih && cc == iw);
#pragma unroll
                  for (int j = 0; j < VW; ++j) {
                    const float v = me ? self[j] : load_pre(x, base + j, ch * VW + j, scale, shift, act);
                    if (v > best[j]) { best[j] = v; won[j] = me; }
                  }
                }
              }
            }
#pragma unroll
            for (int j = 0; j < VW; ++j)
              if (won[j]) gacc[j] += bf2f(dout[obase + j]);
          }
        }
    if constexpr (VW == 8) {
      Pack8 p;
#pragma unroll
      for (int j = 0; j < 8; ++j) p.e[j] = f2bf(gacc[j]);
      *(uint4*)(dx + i * 8) = p.u;
    } else {
#pragma unroll
      for (int j = 0; j < VW; ++j) dx[i * VW + j] = f2bf(gacc[j]);
    }
  }
}

// Non-overlapping windows (stride == kernel, no padding, dims divisible):
// one thread per (output window, 8-channel chunk) reads the window once
// (16-B vectors), recomputes the BN+act prologue, picks the first arg-max and
// writes the whole window of dx -- every input element is written exactly
// once, so no zero-fill pass and no gather recomputation.
//
// STATS (max pool after BN+act, VW = 8, 256 % (C/8) == 0 so a thread keeps its channel chunk):
// also the BN backward's raw moments (sum g, sum g*y), g = dx * act'(z) -- nonzero only at a
// window's arg-max, where z is the window max and y its pre-BN value -- as per-block rows
// part[block][2][C] (bn_finalize MODE 2), so no colstats pass over dx and y follows.
template <int VW, bool STATS = false>
__global__ __launch_bounds__(256) void pool_bwd_tiled_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ x,
                                                             bf16* __restrict__ dx, const float* __restrict__ scale,
                                                             const float* __restrict__ shift, PoolGeom g, int is_max,
                                                             int act, float* __restrict__ part = nullptr) {
  const int cpr = g.C / VW;
  const long long total = (long long)g.N * g.OD * g.OH * g.OW * cpr;
  const int win = g.KD * g.KH * g.KW;
  const float inv = 1.f / (float)win;
  float s0[STATS ? VW : 1], s1[STATS ? VW : 1];
#pragma unroll
  for (int j = 0; j < (STATS ? VW : 1); ++j) s0[j] = s1[j] = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % cpr);
    long long t = i / cpr;
    const int ow = (int)(t % g.OW); t /= g.OW;
    const int oh = (int)(t % g.OH); t /= g.OH;
    const int od = (int)(t % g.OD);
    const long long n = t / g.OD;
    float go[VW], sc[VW], sh[VW], best[VW], yarg[VW];
    int arg[VW];
    Pack8 pg;
    if constexpr (VW == 8) pg.u = *(const uint4*)(dout + i * 8); else pg.e[0] = dout[i];
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      go[j] = bf2f(pg.e[j]);
      best[j] = -INFINITY;
      yarg[j] = 0.f;
      arg[j] = 0;
      sc[j] = scale ? scale[ch * VW + j] : 1.f;
      sh[j] = scale ? shift[ch * VW + j] : 0.f;
    }
    auto base_of = [&](int w) {
      const int kw = w % g.KW, kh = (w / g.KW) % g.KH, kd = w / (g.KW * g.KH);
      return ((((n * g.D + od * g.KD + kd) * g.H + oh * g.KH + kh) * (long long)g.W + ow * g.KW + kw) * g.C) +
             ch * VW;
    };
    if (is_max) {
      for (int w = 0; w < win; ++w) {
        Pack8 p;
        const long long b = base_of(w);
        if constexpr (VW == 8) p.u = *(const uint4*)(x + b); else p.e[0] = x[b];
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const float yv = bf2f(p.e[j]);
          float v = yv;
          if (scale) v = act_fwd(v * sc[j] + sh[j], act);
          if (v > best[j]) { best[j] = v; arg[j] = w; yarg[j] = yv; }
        }
      }
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const float gv = go[j] * act_bwd_from_out(best[j], act);   // bf16 dout: exactly the stored dx
          s0[j] += gv;
          s1[j] += gv * yarg[j];
        }
      }
    }
    if (!STATS || dx) {                          // (STATS with dx null: the moments only -- the
      for (int w = 0; w < win; ++w) {            //  fused apply below recomputes dx)
        Pack8 p;
#pragma unroll
        for (int j = 0; j < VW; ++j) p.e[j] = f2bf(is_max ? (arg[j] == w ? go[j] : 0.f) : go[j] * inv);
        const long long b = base_of(w);
        if constexpr (VW == 8) *(uint4*)(dx + b) = p.u; else dx[b] = p.e[0];
      }
    }
  }
  if constexpr (STATS) {
    __shared__ float red[256][2 * VW + 1];
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < VW; ++j) { red[tid][j] = s0[j]; red[tid][VW + j] = s1[j]; }
    __syncthreads();
    for (int c = tid; c < g.C; c += 256) {       // thread t holds chunk t % cpr (256 % cpr == 0)
      const int chk = c / VW, j = c % VW;
      float a = 0.f, b = 0.f;
      for (int t = chk; t < 256; t += cpr) { a += red[t][j]; b += red[t][VW + j]; }
      part[(long long)blockIdx.x * 2 * g.C + c] = a;
      part[(long long)blockIdx.x * 2 * g.C + g.C + c] = b;
    }
  }
}

// BN backward moments of a BN+act+max-pool block without writing dz (the fused apply below
// recomputes it): pool_bwd_tiled_kernel<8, true> with dx = null, restructured for bandwidth --
// all <= 8 window loads of a thread in flight together (the generic kernel's runtime window
// loop issued one 16-B load at a time: 2.6 TB/s), 32-bit index math (I = int when the host
// checked the sizes), a grid-stride loop over a resident-sized grid.
template <typename I, int ACT = -1>
__global__ __launch_bounds__(256) void pool_bn_moments8_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, PoolGeom g, int act,
                                                               float* __restrict__ part) {
  const int actc = ACT >= 0 ? ACT : act;         // (compile-time relu / none: a runtime switch kept
                                                 //  tanh / sigmoid code in every element's path)
  const int cpr = g.C / 8;
  const I total = (I)g.N * g.OD * g.OH * g.OW * cpr;
  const int win = g.KD * g.KH * g.KW;            // (<= 8: host-checked)
  const int ch = (int)(threadIdx.x % cpr);       // fixed: the stride is a multiple of cpr (256 % cpr == 0)
  float sc[8], sh[8], s0[8], s1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[ch * 8 + j];
    sh[j] = shift[ch * 8 + j];
    s0[j] = s1[j] = 0.f;
  }
  I wofs[8];                                     // window member offsets from the window origin
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    const int ww = w < win ? w : 0;
    const int kw = ww % g.KW, kh = (ww / g.KW) % g.KH, kd = ww / (g.KW * g.KH);
    wofs[w] = (((I)kd * g.H + kh) * g.W + kw) * g.C;
  }
  // software-pipelined: the next window's 9 loads are issued before this one is reduced (an
  // index past the end re-loads the current window: unconditional loads, so hipcc's wait
  // counts stay exact)
  auto fetch = [&](I ii, Pack8& q, Pack8* qy) {
    I t = ii / cpr;
    const int ow = (int)(t % g.OW); t /= g.OW;
    const int oh = (int)(t % g.OH); t /= g.OH;
    const int od = (int)(t % g.OD);
    const I n = t / g.OD;
    const I b0 = (((n * g.D + (I)od * g.KD) * g.H + (I)oh * g.KH) * g.W + (I)ow * g.KW) * g.C + ch * 8;
    q.u = *(const uint4*)(dout + ii * 8);
#pragma unroll
    for (int w = 0; w < 8; ++w)
      if (w < win) qy[w].u = *(const uint4*)(y + b0 + wofs[w]);
  };
  const I stride = (I)gridDim.x * 256;
  I i = (I)blockIdx.x * 256 + threadIdx.x;
  Pack8 pg, py[8];
  if (i < total) fetch(i, pg, py);
  while (i < total) {
    const I inx = i + stride;
    Pack8 pg2, py2[8];
    fetch(inx < total ? inx : i, pg2, py2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float best = -INFINITY, yarg = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        if (w < win) {
          const float yv = bf2f(py[w].e[j]);
          const float v = act_fwd(yv * sc[j] + sh[j], actc);
          if (v > best) { best = v; yarg = yv; }   // (first arg-max, as the forward's scan)
        }
      }
      const float gv = bf2f(pg.e[j]) * act_bwd_from_out(best, actc);
      s0[j] += gv;
      s1[j] += gv * yarg;
    }
    pg = pg2;
#pragma unroll
    for (int w = 0; w < 8; ++w) py[w] = py2[w];
    i = inx;
  }
  __shared__ float red[256][17];
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[tid][j] = s0[j]; red[tid][8 + j] = s1[j]; }
  __syncthreads();
  for (int c = tid; c < g.C; c += 256) {
    const int chk = c / 8, j = c % 8;
    float a = 0.f, b = 0.f;
    for (int u = chk; u < 256; u += cpr) { a += red[u][j]; b += red[u][8 + j]; }
    part[(long long)blockIdx.x * 2 * g.C + c] = a;
    part[(long long)blockIdx.x * 2 * g.C + g.C + c] = b;
  }
}

// Max-pool backward and the BN backward's input gradient in one pass (non-overlapping windows
// of <= 8 positions, C % 8 == 0): one thread per (window, 8-channel chunk) reads the window's y
// once, recomputes z = act(bn(y)) and the first arg-max, and writes
//   dy = scale*g + k2*y + k3,  g = dout * act'(z) at the arg-max, 0 elsewhere
// for the whole window (bn_bwd_apply_kernel's k2 / k3).  Replaces pool_bwd (writes the sparse
// dz) + bn_bwd_apply (reads dz and y again): two full-size passes fewer -- the moments come
// from pool_bwd_tiled_kernel<8, true> with dx = null beforehand.
// (I = int: 32-bit index math, when the host checked that every offset fits)
template <typename I, int ACT = -1>
__global__ __launch_bounds__(256) void pool_bn_bwd_apply_kernel(
    const bf16* __restrict__ dout, const bf16* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ dbeta, const float* __restrict__ dgamma, bf16* __restrict__ dy, PoolGeom g, int act,
    float inv_count) {
  const int actc = ACT >= 0 ? ACT : act;         // (compile-time relu / none: a runtime switch kept
                                                 //  tanh / sigmoid code in every element's path)
  const int cpr = g.C / 8;
  const I total = (I)g.N * g.OD * g.OH * g.OW * cpr;
  const int win = g.KD * g.KH * g.KW;            // (<= 8: host-checked)
  // a fixed 8-channel chunk per thread (256 % cpr == 0 and the grid stride a multiple of 256,
  // host-checked): the per-channel constants are loaded once, not per window
  const int ch = (int)(threadIdx.x % cpr);
  float sc[8], sh[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = ch * 8 + j;
    sc[j] = scale[c];
    sh[j] = shift[c];
    const float is = invstd[c];
    k2[j] = -sc[j] * is * dgamma[c] * inv_count;
    k3[j] = -sc[j] * (dbeta[c] * inv_count - mean[c] * is * dgamma[c] * inv_count);
  }
  I wofs[8];                                     // window member offsets from the window origin
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    const int ww = w < win ? w : 0;
    const int kw = ww % g.KW, kh = (ww / g.KW) % g.KH, kd = ww / (g.KW * g.KH);
    wofs[w] = (((I)kd * g.H + kh) * g.W + kw) * g.C;
  }
  auto origin = [&](I ii) -> I {
    I t = ii / cpr;
    const int ow = (int)(t % g.OW); t /= g.OW;
    const int oh = (int)(t % g.OH); t /= g.OH;
    const int od = (int)(t % g.OD);
    const I n = t / g.OD;
    return (((n * g.D + (I)od * g.KD) * g.H + (I)oh * g.KH) * g.W + (I)ow * g.KW) * g.C + ch * 8;
  };
  // software-pipelined as pool_bn_moments8_kernel: the next window's loads are in flight
  // while this one is reduced and stored
  auto fetch = [&](I ii, I b0, Pack8& q, Pack8* qy) {
    q.u = *(const uint4*)(dout + ii * 8);
#pragma unroll
    for (int w = 0; w < 8; ++w)
      if (w < win) qy[w].u = *(const uint4*)(y + b0 + wofs[w]);
  };
  const I stride = (I)gridDim.x * 256;
  I i = (I)blockIdx.x * 256 + threadIdx.x;
  Pack8 pg, py[8];
  I b0 = 0;
  if (i < total) {
    b0 = origin(i);
    fetch(i, b0, pg, py);
  }
  while (i < total) {
    const I inx = i + stride;
    const I in2 = inx < total ? inx : i;
    const I b1 = origin(in2);
    Pack8 pg2, py2[8];
    fetch(in2, b1, pg2, py2);
    float best[8], gm[8];
    int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      arg[j] = 0;
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      if (w < win) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = act_fwd(bf2f(py[w].e[j]) * sc[j] + sh[j], actc);
          if (v > best[j]) { best[j] = v; arg[j] = w; }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) gm[j] = bf2f(pg.e[j]) * act_bwd_from_out(best[j], actc);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      if (w < win) {
        Pack8 po;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          po.e[j] = f2bf(sc[j] * (arg[j] == w ? gm[j] : 0.f) + k2[j] * bf2f(py[w].e[j]) + k3[j]);
        *(uint4*)(dy + b0 + wofs[w]) = po.u;
      }
    }
    pg = pg2;
#pragma unroll
    for (int w = 0; w < 8; ++w) py[w] = py2[w];
    b0 = b1;
    i = inx;
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
// workgroups of `kernel` (256 threads, no dynamic LDS) resident on the whole device at once
// (0 when the runtime cannot say)
static int bn_resident_blocks(const void* kernel) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess)
    return 0;
  return cus > 0 && per > 0 ? cus * per : 0;
}

static unsigned ew_blocks(long long work) {
  long long b = (work + 255) / 256;
  if (b < 1) b = 1;
  if (b > 8192) b = 8192;
  return (unsigned)b;
}

// Workgroups for a colstats launch over M rows: one per 256 rows, capped at what the device
// holds resident at once (the kernel walks its rows in a loop; a grid of 2048 over 768 resident
// slots -- 134 VGPRs, 3 workgroups per CU -- spent its last third at 2/3 occupancy)
extern "C" int fn_colstats_blocks(long long M, int C, int mode, int act) {
  long long nb = M / 256;
  if (nb < 1) nb = 1;
  long long cap = 2048;
  if (C % 8 == 0 && C / 8 <= 256) {
    static int res[2][4] = {{-1, -1, -1, -1}, {-1, -1, -1, -1}};
    const int m = mode ? 1 : 0;
    const int a = mode == 0 ? 0 : (act == ACT_RELU ? 1 : act == ACT_TANH ? 2 : act == ACT_SIGMOID ? 3 : 0);
    if (res[m][a] < 0) {
      const void* k = mode == 0 ? (const void*)colstats_kernel<8, 0, ACT_NONE>
                    : a == 1 ? (const void*)colstats_kernel<8, 1, ACT_RELU>
                    : a == 2 ? (const void*)colstats_kernel<8, 1, ACT_TANH>
                    : a == 3 ? (const void*)colstats_kernel<8, 1, ACT_SIGMOID>
                             : (const void*)colstats_kernel<8, 1, ACT_NONE>;
      res[m][a] = bn_resident_blocks(k);
    }
    if (res[m][a] > 0) cap = res[m][a];
  }
  return (int)(nb > cap ? cap : nb);
}

extern "C" int fn_colstats(const void* x, const void* dz, const float* scale, const float* shift, const float* mean,
                           const float* invstd, float* part, long long M, int C, int act, int mode, int nb,
                           hipStream_t st) {
  const bool vec = (C % 8) == 0 && C / 8 <= 256;
  if (!vec && C > 256) return -2;
  if (!vec && mode == 0) {                       // super-row vector path (see colstats_sr_kernel)
    int gg = 8;
    while (C % gg) gg >>= 1;                     // gcd(8, C)
    const int Q = C / gg, rows_sr = 8 / gg;      // chunks / rows per super row
    if (Q <= 256 && M % rows_sr == 0) {
      const long long nsr = M / rows_sr;
      hipLaunchKernelGGL(colstats_sr_kernel, dim3(nb), dim3(256), 0, st, (const bf16*)x, part, nsr, C, Q,
                         (nsr + nb - 1) / nb);
      FN_CHECK_LAUNCH();
      return 0;
    }
  }
  const long long rpb = (M + nb - 1) / nb;
  const bf16* xx = (const bf16*)x;
  const bf16* dd = (const bf16*)dz;
#define CS_CASE(VW, MD, A) \
  hipLaunchKernelGGL((colstats_kernel<VW, MD, A>), dim3(nb), dim3(256), 0, st, xx, dd, scale, shift, mean, invstd, part, M, C, rpb)
#define CS_ACT(VW)                                                                                  \
  do {                                                                                              \
    if (mode == 0) CS_CASE(VW, 0, ACT_NONE);                                                        \
    else if (act == ACT_RELU) CS_CASE(VW, 1, ACT_RELU);                                             \
    else if (act == ACT_TANH) CS_CASE(VW, 1, ACT_TANH);                                             \
    else if (act == ACT_SIGMOID) CS_CASE(VW, 1, ACT_SIGMOID);                                       \
    else CS_CASE(VW, 1, ACT_NONE);                                                                  \
  } while (0)
  if (vec) CS_ACT(8); else CS_ACT(1);
#undef CS_ACT
#undef CS_CASE
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_bn_finalize(const float* part, int nb, int C, double count, const float* gamma, const float* beta,
                              float* run_mean, float* run_var, float momentum, float eps, float* o0, float* o1,
                              float* o2, float* o3, int mode, hipStream_t st) {
  if (mode == 0)
    hipLaunchKernelGGL(bn_finalize_kernel<0>, dim3(C), dim3(256), 0, st, part, nb, C, count, gamma, beta, run_mean,
                       run_var, momentum, eps, o0, o1, o2, o3);
  else if (mode == 1)
    hipLaunchKernelGGL(bn_finalize_kernel<1>, dim3(C), dim3(256), 0, st, part, nb, C, count, gamma, beta, run_mean,
                       run_var, momentum, eps, o0, o1, o2, o3);
  else if (mode == 2 && run_mean && run_var)
    hipLaunchKernelGGL(bn_finalize_kernel<2>, dim3(C), dim3(256), 0, st, part, nb, C, count, gamma, beta, run_mean,
                       run_var, momentum, eps, o0, o1, o2, o3);
  else
    return -2;
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_bn_apply(const void* y, const float* scale, const float* shift, void* z, long long total, int C,
                           int act, hipStream_t st, void* mask) {
  if (mask && (C % 8 || 256 % (C / 8))) return -2;   // (the fixed-chunk path writes the mask)
#define BA_CASE(VW, A)                                                                                  \
  hipLaunchKernelGGL((bn_apply_kernel<VW, A>), dim3(ew_blocks(total / VW)), dim3(256), 0, st, (const bf16*)y, scale, \
                     shift, (bf16*)z, total, C, (unsigned char*)mask)
#define BA_ACT(VW)                                                                                      \
  do {                                                                                                  \
    if (act == ACT_RELU) BA_CASE(VW, ACT_RELU);                                                         \
    else if (act == ACT_TANH) BA_CASE(VW, ACT_TANH);                                                    \
    else if (act == ACT_SIGMOID) BA_CASE(VW, ACT_SIGMOID);                                              \
    else BA_CASE(VW, ACT_NONE);                                                                         \
  } while (0)
  if (C % 8 == 0) BA_ACT(8); else BA_ACT(1);
#undef BA_ACT
#undef BA_CASE
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_bn_bwd_apply(const void* dz, const void* y, const float* scale, const float* shift,
                               const float* mean, const float* invstd, const float* dbeta, const float* dgamma,
                               void* dy, long long total, int C, float inv_count, int act, hipStream_t st) {
#define BB_CASE(VW, A)                                                                                  \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<VW, A>), dim3(ew_blocks(total / VW)), dim3(256), 0, st,            \
                     (const bf16*)dz, (const bf16*)y, scale, shift, mean, invstd, dbeta, dgamma, (bf16*)dy, total, C, \
                     inv_count)
#define BB_ACT(VW)                                                                                      \
  do {                                                                                                  \
    if (act == ACT_RELU) BB_CASE(VW, ACT_RELU);                                                         \
    else if (act == ACT_TANH) BB_CASE(VW, ACT_TANH);                                                    \
    else if (act == ACT_SIGMOID) BB_CASE(VW, ACT_SIGMOID);                                              \
    else BB_CASE(VW, ACT_NONE);                                                                         \
  } while (0)
  if (C % 8 == 0) BB_ACT(8); else BB_ACT(1);
#undef BB_ACT
#undef BB_CASE
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_bn_bwd_apply_s2d(const void* dz, const void* y, const float* scale, const float* shift,
                                   const float* mean, const float* invstd, const float* dbeta, const float* dgamma,
                                   void* dsh, int N, int FD, int FH, int FW, int C, float inv_count, int act,
                                   hipStream_t st) {
  if (C % 8 || 256 % (C / 8) || FD % 2 || FH % 2 || FW % 2 || N < 1) return -2;
  const long long nvec = (long long)N * (FD / 2 + 1) * (FH / 2 + 1) * (FW / 2 + 1) * 8 * (C / 8);
  const long long nrows = (long long)N * (FD / 2 + 1) * (FH / 2 + 1);
  if ((act == ACT_RELU || act == ACT_NONE) && nrows < (1LL << 31) && nvec * 8 < (1LL << 40)) {
    // the row form (grid-stride over the (n, cell-d, cell-h) rows)
    int lc = 0;
    while ((1 << lc) < C / 8) ++lc;
    const unsigned grid = (unsigned)std::min<long long>(nrows, 8192);
    const long long rowlen = (long long)(FW / 2 + 1) * 8 * (C / 8);
    const int u = rowlen > 4 * 256 && rowlen <= 5 * 256 ? 5 : (rowlen > 5 * 256 && rowlen <= 8 * 256 ? 8 : 4);
#define BR_CASE(A, L)                                                                                        \
    if (lc == L) {                                                                                           \
      if (u == 5) hipLaunchKernelGGL((bn_bwd_apply_s2d_rows_kernel<A, L, 5>), dim3(grid), dim3(256), 0, st,  \
                                     (const bf16*)dz, (const bf16*)y, scale, shift, mean, invstd, dbeta, dgamma, \
                                     (bf16*)dsh, N, FD, FH, FW, C, inv_count);                              \
      else if (u == 8) hipLaunchKernelGGL((bn_bwd_apply_s2d_rows_kernel<A, L, 8>), dim3(grid), dim3(256), 0, \
                                          st, (const bf16*)dz, (const bf16*)y, scale, shift, mean, invstd,  \
                                          dbeta, dgamma, (bf16*)dsh, N, FD, FH, FW, C, inv_count);          \
      else hipLaunchKernelGGL((bn_bwd_apply_s2d_rows_kernel<A, L, 4>), dim3(grid), dim3(256), 0, st,         \
                              (const bf16*)dz, (const bf16*)y, scale, shift, mean, invstd, dbeta, dgamma,   \
                              (bf16*)dsh, N, FD, FH, FW, C, inv_count);                                     \
    }
#define BR_ACT(A) BR_CASE(A, 0) BR_CASE(A, 1) BR_CASE(A, 2) BR_CASE(A, 3) BR_CASE(A, 4) BR_CASE(A, 5)
    if (act == ACT_RELU) { BR_ACT(ACT_RELU) } else { BR_ACT(ACT_NONE) }
#undef BR_ACT
#undef BR_CASE
    FN_CHECK_LAUNCH();
    return 0;
  }
#define BS_CASE(A)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_s2d_kernel<A>), dim3(ew_blocks(nvec)), dim3(256), 0, st, (const bf16*)dz, \
                     (const bf16*)y, scale, shift, mean, invstd, dbeta, dgamma, (bf16*)dsh, N, FD, FH, FW, C, inv_count)
  if (act == ACT_RELU) BS_CASE(ACT_RELU);
  else if (act == ACT_TANH) BS_CASE(ACT_TANH);
  else if (act == ACT_SIGMOID) BS_CASE(ACT_SIGMOID);
  else BS_CASE(ACT_NONE);
#undef BS_CASE
  FN_CHECK_LAUNCH();
  return 0;
}

static PoolGeom pool_geom(const int* g) {
  PoolGeom p;
  p.N = g[0]; p.D = g[1]; p.H = g[2]; p.W = g[3]; p.C = g[4];
  p.OD = g[5]; p.OH = g[6]; p.OW = g[7];
  p.KD = g[8]; p.KH = g[9]; p.KW = g[10];
  p.sd = g[11]; p.sh = g[12]; p.sw = g[13];
  p.pd = g[14]; p.ph = g[15]; p.pw = g[16];
  return p;
}

extern "C" int fn_pool_fwd(const void* x, void* out, const float* scale, const float* shift, const int* geom17,
                           int is_max, int count_pad, int act, hipStream_t st) {
  PoolGeom g = pool_geom(geom17);
  const long long outs = (long long)g.N * g.OD * g.OH * g.OW;
  const bool win2 = g.KH == 2 && g.KW == 2 && (g.KD == 2 || g.KD == 1) && g.sd == g.KD && g.sh == 2 && g.sw == 2 &&
                    g.pd == 0 && g.ph == 0 && g.pw == 0 && g.D >= g.OD * g.KD && g.H >= g.OH * 2 &&
                    g.W >= g.OW * 2 && g.C % 8 == 0 && 256 % (g.C / 8) == 0 &&
                    outs * (g.C / 8) + 256LL * 8192 < (1LL << 31);
  if (win2) {
    const int total = (int)(outs * (g.C / 8));
    // (relu / none / no BN: compile-time instances; other activations the runtime one)
    const int ka = !scale ? ACT_NONE : ((act == ACT_RELU || act == ACT_NONE) ? act : -1);
#define P2_CASE(K, A)                                                                                         \
    if (g.KD == K && ka == A) {                                                                               \
      static const int res = bn_resident_blocks((const void*)pool2_fwd_kernel<K, A>);                         \
      long long nbl = (total + 255) / 256;                                                                    \
      if (res > 0 && nbl > res) nbl = res;                                                                    \
      const unsigned nb = (unsigned)(nbl < 1 ? 1 : (nbl > 8192 ? 8192 : nbl));                                 \
      hipLaunchKernelGGL((pool2_fwd_kernel<K, A>), dim3(nb), dim3(256), 0, st, (const bf16*)x, (bf16*)out,    \
                         scale, shift, g, is_max, act, total);                                                \
    }
    P2_CASE(2, ACT_RELU) P2_CASE(2, ACT_NONE) P2_CASE(2, -1) P2_CASE(1, ACT_RELU) P2_CASE(1, ACT_NONE) P2_CASE(1, -1)
#undef P2_CASE
  } else if (g.C % 8 == 0)
    hipLaunchKernelGGL(pool_fwd_kernel<8>, dim3(ew_blocks(outs * (g.C / 8))), dim3(256), 0, st, (const bf16*)x,
                       (bf16*)out, scale, shift, g, is_max, count_pad, act);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<1>, dim3(ew_blocks(outs * g.C)), dim3(256), 0, st, (const bf16*)x, (bf16*)out,
                       scale, shift, g, is_max, count_pad, act);
  FN_CHECK_LAUNCH();
  return 0;
}

// every element offset of the pool's input / output (and the loop bound) fits a 32-bit int
static bool pool_i32(const PoolGeom& g) {
  const long long ins = (long long)g.N * g.D * g.H * g.W * g.C;
  const long long outs = (long long)g.N * g.OD * g.OH * g.OW * g.C;
  return ins + 256LL * 8192 * 8 < (1LL << 31) && outs + 256LL * 8192 * 8 < (1LL << 31);
}

static bool pool_bwd_stats_ok(const PoolGeom& g) {
  return g.sd == g.KD && g.sh == g.KH && g.sw == g.KW && g.pd == 0 && g.ph == 0 && g.pw == 0 &&
         g.D == g.OD * g.KD && g.H == g.OH * g.KH && g.W == g.OW * g.KW && g.C % 8 == 0 && 256 % (g.C / 8) == 0;
}

// blocks of the STATS launch (rows of its part slab); 0 when the geometry has no such path
extern "C" int fn_pool_bwd_stats_blocks(const int* geom17) {
  const PoolGeom g = pool_geom(geom17);
  if (!pool_bwd_stats_ok(g)) return 0;
  const long long w = ((long long)g.N * g.OD * g.OH * g.OW * (g.C / 8) + 255) / 256;
  long long cap = 2048;
  if (g.KD * g.KH * g.KW <= 8) {
    // the moments kernel's grid-stride loop: one resident wave of workgroups (no tail round)
    static const int res = bn_resident_blocks((const void*)pool_bn_moments8_kernel<int>);
    if (res > 0) cap = res;
  }
  return (int)(w < 1 ? 1 : (w > cap ? cap : w));
}

// max-pool backward of a BN+act output plus that BN's raw backward moments (see
// pool_bwd_tiled_kernel STATS); part: fp32 [fn_pool_bwd_stats_blocks][2][C]
extern "C" int fn_pool_bwd_stats(const void* dout, const void* x, void* dx, const float* scale, const float* shift,
                                 const int* geom17, int act, float* part, hipStream_t st) {
  const PoolGeom g = pool_geom(geom17);
  const int nb = fn_pool_bwd_stats_blocks(geom17);
  if (nb <= 0 || !scale || !shift || !part) return -2;
  if (!dx && g.KD * g.KH * g.KW <= 8) {          // moments only: the bandwidth form
    const bool i32 = pool_i32(g);
    const int ka = (act == ACT_RELU || act == ACT_NONE) ? act : -1;
#define PM_CASE(I, A)                                                                                          \
    if (i32 == std::is_same<I, int>::value && ka == A)                                                         \
      hipLaunchKernelGGL((pool_bn_moments8_kernel<I, A>), dim3(nb), dim3(256), 0, st, (const bf16*)dout,        \
                         (const bf16*)x, scale, shift, g, act, part);
    PM_CASE(int, ACT_RELU) PM_CASE(int, ACT_NONE) PM_CASE(int, -1)
    PM_CASE(long long, ACT_RELU) PM_CASE(long long, ACT_NONE) PM_CASE(long long, -1)
#undef PM_CASE
  } else
    hipLaunchKernelGGL((pool_bwd_tiled_kernel<8, true>), dim3(nb), dim3(256), 0, st, (const bf16*)dout, (const bf16*)x,
                       (bf16*)dx, scale, shift, g, 1, act, part);
  FN_CHECK_LAUNCH();
  return 0;
}

// dy of BN+act+max-pool in one pass (pool_bn_bwd_apply_kernel); the tiled-window geometry of
// fn_pool_bwd_stats with windows of <= 8 positions
extern "C" int fn_pool_bn_bwd_apply(const void* dout, const void* y, const float* scale, const float* shift,
                                    const float* mean, const float* invstd, const float* dbeta, const float* dgamma,
                                    void* dy, const int* geom17, int act, float inv_count, hipStream_t st) {
  const PoolGeom g = pool_geom(geom17);
  const bool tiled = g.sd == g.KD && g.sh == g.KH && g.sw == g.KW && g.pd == 0 && g.ph == 0 && g.pw == 0 &&
                     g.D == g.OD * g.KD && g.H == g.OH * g.KH && g.W == g.OW * g.KW;
  if (!tiled || g.C % 8 || 256 % (g.C / 8) || g.KD * g.KH * g.KW > 8) return -2;
  const long long outs = (long long)g.N * g.OD * g.OH * g.OW;
  static const int res = bn_resident_blocks((const void*)pool_bn_bwd_apply_kernel<int>);
  long long nbl = (outs * (g.C / 8) + 255) / 256;
  if (res > 0 && nbl > res) nbl = res;           // one resident wave of workgroups, grid-stride
  const unsigned nb = (unsigned)(nbl < 1 ? 1 : (nbl > 8192 ? 8192 : nbl));
  const bool i32 = pool_i32(g);
  const int ka = (act == ACT_RELU || act == ACT_NONE) ? act : -1;
#define PA_CASE(I, A)                                                                                           \
  if (i32 == std::is_same<I, int>::value && ka == A)                                                            \
    hipLaunchKernelGGL((pool_bn_bwd_apply_kernel<I, A>), dim3(nb), dim3(256), 0, st, (const bf16*)dout,          \
                       (const bf16*)y, scale, shift, mean, invstd, dbeta, dgamma, (bf16*)dy, g, act, inv_count);
  PA_CASE(int, ACT_RELU) PA_CASE(int, ACT_NONE) PA_CASE(int, -1)
  PA_CASE(long long, ACT_RELU) PA_CASE(long long, ACT_NONE) PA_CASE(long long, -1)
#undef PA_CASE
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_pool_bwd(const void* dout, const void* x, void* dx, const float* scale, const float* shift,
                           const int* geom17, int is_max, int count_pad, int act, hipStream_t st) {
  PoolGeom g = pool_geom(geom17);
  const long long ins = (long long)g.N * g.D * g.H * g.W;
  const bool tiled = g.sd == g.KD && g.sh == g.KH && g.sw == g.KW && g.pd == 0 && g.ph == 0 && g.pw == 0 &&
                     g.D == g.OD * g.KD && g.H == g.OH * g.KH && g.W == g.OW * g.KW;
  if (tiled) {
    const long long outs = (long long)g.N * g.OD * g.OH * g.OW;
    if (g.C % 8 == 0)
      hipLaunchKernelGGL(pool_bwd_tiled_kernel<8>, dim3(ew_blocks(outs * (g.C / 8))), dim3(256), 0, st,
                         (const bf16*)dout, (const bf16*)x, (bf16*)dx, scale, shift, g, is_max, act);
    else
      hipLaunchKernelGGL(pool_bwd_tiled_kernel<1>, dim3(ew_blocks(outs * g.C)), dim3(256), 0, st, (const bf16*)dout,
                         (const bf16*)x, (bf16*)dx, scale, shift, g, is_max, act);
    FN_CHECK_LAUNCH();
    return 0;
  }
  if (g.C % 8 == 0)
    hipLaunchKernelGGL(pool_bwd_kernel<8>, dim3(ew_blocks(ins * (g.C / 8))), dim3(256), 0, st, (const bf16*)dout,
                       (const bf16*)x, (bf16*)dx, scale, shift, g, is_max, count_pad, act);
  else if (g.C % 2 == 0)                         // (channel pairs: the window walk once per two, e.g.
    hipLaunchKernelGGL(pool_bwd_kernel<2>, dim3(ew_blocks(ins * (g.C / 2))), dim3(256), 0, st,   // LeNet's 18)
                       (const bf16*)dout, (const bf16*)x, (bf16*)dx, scale, shift, g, is_max, count_pad, act);
  else
    hipLaunchKernelGGL(pool_bwd_kernel<1>, dim3(ew_blocks(ins * g.C)), dim3(256), 0, st, (const bf16*)dout,
                       (const bf16*)x, (bf16*)dx, scale, shift, g, is_max, count_pad, act);
  FN_CHECK_LAUNCH();
  return 0;
}

// S partials of the statistics identity: part[nb][C], W / dW fp32 [R][C] (R = K * taps)
extern "C" int fn_bn_wdot(const float* w, const float* dw, float* part, int R, int C, int nb, hipStream_t st) {
  if (C <= 0 || C > 256 || 256 % C || nb < 1) return -2;
  const int rpb = (R + nb - 1) / nb;
  hipLaunchKernelGGL(bn_wdot_kernel, dim3(nb), dim3(256), 0, st, w, dw, part, R, C, rpb);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_bn_bwd_prep(const float* gslab, int nbg, const float* wpart, int nbw, int C, double count,
                              const float* gamma, const float* beta, const float* mean, const float* invstd,
                              const float* scale, const float* shift, float* dbeta, float* kc, const void* g,
                              const void* y, long long M, hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_prep_kernel, dim3(C), dim3(256), 0, st, gslab, nbg, wpart, nbw, C, count, gamma, beta,
                     mean, invstd, scale, shift, dbeta, kc, (const bf16*)g, (const bf16*)y, M);
  FN_CHECK_LAUNCH();
  return 0;
}

// workgroups of bn_bwd_apply_k (its partial-sum rows): one resident wave of them
extern "C" int fn_bn_bwd_apply_k_blocks(long long M, int C) {
  static const int res = bn_resident_blocks((const void*)bn_bwd_apply_k_kernel);
  long long nb = (M * (C / 8) + 255) / 256;
  const long long cap = res > 0 ? res : 2048;
  if (nb > cap) nb = cap;
  return (int)(nb < 1 ? 1 : nb);
}

extern "C" int fn_bn_bwd_apply_k(const void* g, const void* y, const float* kc, const float* mean,
                                 const float* invstd, const float* shift, void* dy, long long M, int C, float* part,
                                 int nb, hipStream_t st) {
  if (C % 8 || 256 % (C / 8) || nb < 1) return -2;
  hipLaunchKernelGGL(bn_bwd_apply_k_kernel, dim3(nb), dim3(256), 0, st, (const bf16*)g, (const bf16*)y, kc, mean,
                     invstd, shift, (bf16*)dy, M * (C / 8), C, part);
  FN_CHECK_LAUNCH();
  return 0;
}
