// Dense (fully connected) layer on MFMA: y = act(x W^T + b) and its gradients.
//
// Reference parity: Keras Dense (reference model/input.py:174-190) and the classifier head
// (model/keras_model.py:124).  FeatureNet-3D's FC1 is 128 x 64000 -> 128 (skinny: M*N tiny,
// K huge); NAS candidates put Dense layers of up to 2048 features after small feature maps.
//
//   dense_fwd_part  split-K partial products, x bf16 [M][K] x W fp32 [N][K] (the fp32 master
//                   weights converted to bf16 on the fly: no per-step weight cast pass) or a
//                   bf16 W copy (inference), fp32 partial slabs [S][M][N]; 128x64 or 128x128
//                   output tile per workgroup, 4 or 8 waves x (32 rows x 64 cols), operands
//                   straight from global (16-B loads, no LDS)
//   dense_fwd_reduce  y = act(sum_s part[s] + b) -> bf16 or fp32 (one pass over M*N); with one
//                   slice the partial kernel's epilogue writes y itself (no slab, no reduction)
//   dense_dgrad     dx [M][K] = g [M][N] W [N][K] -> bf16.  C^T form: A = W^T from an LDS
//                   tile written transposed ([kk][n], converted to bf16), B = g rows from
//                   global; a lane ends with 4 consecutive kk of one row (8-B stores)
//   dense_wgrad     dW [N][K] = g^T x -> fp32 straight into the parameter's (flat) gradient,
//                   db = column sums of g (workgroup 0).  Both operands from LDS tiles written
//                   transposed ([kk][m], [n][m]); a lane ends with 4 consecutive kk of one n
//                   (16-B stores)
//
// MFMA v_mfma_f32_16x16x32_bf16: A lane (r = lane&15, g = lane>>4) holds A[r][8g..8g+7],
// B lane holds B[8g..8g+7][r], C lane holds C[4g..4g+3][r].
#include "common.h"

#define DN_THREADS 256
#define DN_WG_MCH 512                            // weight gradient: batch rows per LDS chunk

__device__ __forceinline__ bf16x8 dn_cvt8(const float4 a, const float4 b) {
  bf16x8 v;
  v[0] = f2bf(a.x); v[1] = f2bf(a.y); v[2] = f2bf(a.z); v[3] = f2bf(a.w);
  v[4] = f2bf(b.x); v[5] = f2bf(b.y); v[6] = f2bf(b.z); v[7] = f2bf(b.w);
  return v;
}

// 8 consecutive bf16 of a row of n elements from column c (zeros past n), as wide as the row
// pitch allows: one 16-B load (n % 8 == 0), two 8-B loads (n % 4 == 0: the 84-wide Dense of the
// LeNet template, whose element loads ran its dgrad at 30 us), 4-B loads (n even), else elements
__device__ inline bf16x8 dn_load8(const bf16* __restrict__ row, int c, int n) {
  bf16x8 v = {};
  if ((n & 7) == 0 && c + 8 <= n) return *(const bf16x8*)(row + c);
  if ((n & 3) == 0) {
    if (c + 4 <= n) {
      const bf16x4 a = *(const bf16x4*)(row + c);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    }
    if (c + 8 <= n) {
      const bf16x4 b = *(const bf16x4*)(row + c + 4);
      v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    }
    return v;
  }
  if ((n & 1) == 0) {
#pragma unroll
    for (int e = 0; e < 8; e += 2)
      if (c + e + 2 <= n) {
        const unsigned u = *(const unsigned*)(row + c + e);
        v[e] = __builtin_bit_cast(bf16, (unsigned short)(u & 0xffffu));
        v[e + 1] = __builtin_bit_cast(bf16, (unsigned short)(u >> 16));
      }
    return v;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = c + e < n ? row[c + e] : f2bf(0.f);
  return v;
}

// ---------------------------------------------------------------------------
// forward: split-K partials
// ---------------------------------------------------------------------------
// grid (ceil(N/(64 NCW)), ceil(M/128), S); slice s covers k in [s*kc, min(K, (s+1)*kc)),
// kc % 32 == 0.  4 NCW waves: wave w takes rows 32 (w & 3).., columns 64 (w >> 2)..  -- with
// NCW = 2 (N > 64) a workgroup covers 128 columns, so each x row is fetched from HBM once and
// shared by the two column waves through the CU's L1 / L2 (with 64-column workgroups the two
// column tiles of a row landed on different XCDs and x, 2.3 GB at 128^3 inference, came from
// HBM twice).
// VEC (K % 8 == 0): 16-B x rows and 16-B weight loads; otherwise element loads masked at kend
// (the 84-wide LeNet layers).  WB: bf16 weights (the inference copy, half the weight bytes, no
// conversion), else the fp32 master weights converted on the fly.  D k-steps of raw operands
// in flight (a register ring): with one step ahead the loop waited a full memory latency per
// 32-k step (FC1 at 128^3 inference: 1100 steps per slice)
// FINAL (one slice, gridDim.z == 1): the epilogue writes y = act(acc + b) itself (bf16 or fp32)
// -- no partial slab and no reduction launch (the small Dense layers of NAS candidates)
template <bool VEC, int D, bool WB, int NCW, bool FINAL = false>
__global__ __launch_bounds__(DN_THREADS * NCW) void dense_fwd_part_kernel(const bf16* __restrict__ x,
                                                                          const void* __restrict__ wv,
                                                                          float* __restrict__ part, int M, int N,
                                                                          int K, int kc, const float* __restrict__ bias,
                                                                          int act, int out_fp32) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, gq = lane >> 4;
  const int row0 = blockIdx.y * 128 + (wave & 3) * 32, col0 = (blockIdx.x * NCW + (wave >> 2)) * 64;
  const int kbeg = blockIdx.z * kc, kend = min(K, kbeg + kc);
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // row / column validity is per lane; out-of-range rows read row 0 and are zeroed
  bool rok[2], cok[4];
  const bf16* xr[2];
  const float* wr[4];
  const bf16* wh[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = row0 + i * 16 + r;
    rok[i] = m < M;
    xr[i] = x + (long long)(rok[i] ? m : 0) * K;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = col0 + j * 16 + r;
    cok[j] = n < N;
    wr[j] = (const float*)wv + (long long)(cok[j] ? n : 0) * K;
    wh[j] = (const bf16*)wv + (long long)(cok[j] ? n : 0) * K;
  }
  const bf16x8 zero8 = {};
  // D k-steps of operands in flight ahead of the MFMAs (raw loads; conversion and masking
  // happen when the step is consumed; steps past kend read chunk 0 and are never consumed)
  bf16x8 ra[D][2];
  float4 rb[D][4][2];
  bf16x8 rh[D][4];
  auto load = [&](int st, int k0) {
    const int k = k0 + 8 * gq;
    const int ks = k < kend ? k : 0;
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) ra[st][i] = *(const bf16x8*)(xr[i] + ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (WB) {
          rh[st][j] = *(const bf16x8*)(wh[j] + ks);
        } else {
          const float4* p = (const float4*)(wr[j] + ks);
          rb[st][j][0] = p[0];
          rb[st][j][1] = p[1];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) ra[st][i][e] = ks + e < kend ? xr[i][ks + e] : f2bf(0.f);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (WB) {
#pragma unroll
          for (int e = 0; e < 8; ++e) rh[st][j][e] = ks + e < kend ? wh[j][ks + e] : f2bf(0.f);
        } else {
          float t[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = ks + e < kend ? wr[j][ks + e] : 0.f;
          rb[st][j][0] = make_float4(t[0], t[1], t[2], t[3]);
          rb[st][j][1] = make_float4(t[4], t[5], t[6], t[7]);
        }
      }
    }
  };
  // branch-free ring: every group of D steps loads and multiplies unconditionally (steps past
  // kend read chunk 0 and are zeroed by kok): hipcc's vmcnt counting stays exact (a conditional
  // load or step made it wait for the whole ring)
#pragma unroll
  for (int st = 0; st < D; ++st) load(st, kbeg + 32 * st);
  __builtin_amdgcn_sched_barrier(0);             // (the scheduler otherwise sinks every load to its use)
  for (int k0 = kbeg; k0 < kend; k0 += 32 * D) {
#pragma unroll
    for (int st = 0; st < D; ++st) {
      const int kk = k0 + 32 * st;
      {
        // rows / columns past M / N read row / column 0 and their outputs are never stored: only
        // chunks past kend (the tail of K) need zeroing.  Conversion first, then a select: a
        // conditional conversion became an exec-masked branch with a vmcnt(0) wait inside,
        // which drained the whole ring every step
        const bool kok = kk + 8 * gq < kend;
        bf16x8 fa[2], fb[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = kok ? ra[st][i] : zero8;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf16x8 t;
          if constexpr (WB) t = rh[st][j];
          else t = dn_cvt8(rb[st][j][0], rb[st][j][1]);
          fb[j] = kok ? t : zero8;
        }
        load(st, kk + 32 * D);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  if constexpr (FINAL) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = col0 + j * 16 + r;
      const float b = (bias && n < N) ? bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = row0 + i * 16 + 4 * gq + q;
          if (m < M && n < N) {
            const float v = act_fwd(acc[i][j][q] + b, act);
            if (out_fp32) ((float*)part)[(long long)m * N + n] = v;
            else ((bf16*)part)[(long long)m * N + n] = f2bf(v);
          }
        }
    }
    return;
  }
  float* ps = part + (long long)blockIdx.z * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = col0 + j * 16 + r;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = row0 + i * 16 + 4 * gq + q;
        if (m < M && n < N) ps[(long long)m * N + n] = acc[i][j][q];
      }
    }
}

// y[m][n] = act(sum_s part[s][m][n] + b[n]); bf16 or fp32 output.  A workgroup takes 64
// outputs; its 4 waves sum every 4th slice (coalesced 256-B rows, 4 loads in flight per
// lane) and combine through LDS -- one thread per output with a serial walk over hundreds
// of slices left FC1's reduction latency-bound (59 us for 16 MB)
__global__ __launch_bounds__(DN_THREADS) void dense_fwd_reduce_kernel(const float* __restrict__ part,
                                                                      const float* __restrict__ bias, void* out,
                                                                      int M, int N, int S, int act, int out_fp32) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long MN = (long long)M * N;
  const long long i = (long long)blockIdx.x * 64 + lane;
  float v = 0.f;
  if (i < MN) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = wave;
    for (; s + 12 < S; s += 16) {
      a0 += part[(long long)s * MN + i];
      a1 += part[(long long)(s + 4) * MN + i];
      a2 += part[(long long)(s + 8) * MN + i];
      a3 += part[(long long)(s + 12) * MN + i];
    }
    for (; s < S; s += 4) a0 += part[(long long)s * MN + i];
    v = (a0 + a1) + (a2 + a3);
  }
  red[wave][lane] = v;
  __syncthreads();
  if (wave == 0 && i < MN) {
    v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if (bias) v += bias[i % N];
    v = act_fwd(v, act);
    if (out_fp32) {
      ((float*)out)[i] = v;
    } else {
      ((bf16*)out)[i] = f2bf(v);
    }
  }
}

// ---------------------------------------------------------------------------
// dgrad: dx = g W   (C^T = W^T g^T: lane ends with dx[m][4 consecutive kk])
// ---------------------------------------------------------------------------
// grid (ceil(K/64), ceil(M/64)); block tile: 64 rows m x 64 columns kk; any N (the MFMA k dim
// is padded to NP = ceil(N/32)*32 with zero weights; g rows load as 16-B vectors when N % 8 == 0,
// element-wise otherwise -- the 10 / 24 / 84-wide NAS heads).
// LDS (dynamic): W tile transposed to [64 kk][NP + 8] bf16.
// ya (optional): the layer's activation output -- g is then dy * act'(y) (the activation
// backward applied as g is loaded, no separate pass).  (Batched, double-buffered g loads -- all
// 16 fragments of a 128-wide n chunk issued together, the first during the W staging -- ran
// FC1's dgrad at 31.1 us against 24.7 us: 196 registers, half the waves per SIMD)
__global__ __launch_bounds__(DN_THREADS) void dense_dgrad_kernel(const bf16* __restrict__ g,
                                                                 const float* __restrict__ w,
                                                                 bf16* __restrict__ dx, int M, int N, int K,
                                                                 const bf16* __restrict__ ya, int act, int mrep) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dn_lds[];
  const int NP = (N + 31) & ~31;
  const int LDN = NP + 8;                        // row pitch (bf16): 16-B aligned rows, bank shift
  bf16* wt = reinterpret_cast<bf16*>(dn_lds);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, gq = lane >> 4;
  // a workgroup covers mrep consecutive 64-row blocks with one staged W tile (the W tile is the
  // expensive part: FC1's 128 x 64000 weights were read -- and LDS-transposed -- once per row
  // block before)
  const int kk0 = blockIdx.x * 64;
  // stage W[0:N][kk0:kk0+64] -> wt[kk][n] (bf16): thread = (n, 4 consecutive kk)
  for (int idx = tid; idx < NP * 16; idx += DN_THREADS) {
    const int n = idx >> 4, q = idx & 15;
    const int kk = kk0 + 4 * q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n >= N) {
      // zero rows of the padded k dimension
    } else if (kk + 4 <= K && (K & 3) == 0) {   // (16-B aligned rows only)
      v = *(const float4*)(w + (long long)n * K + kk);
    } else {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int e = 0; e < 4; ++e)
        if (kk + e < K) t[e] = w[(long long)n * K + kk + e];
      v = make_float4(t[0], t[1], t[2], t[3]);
    }
    wt[(4 * q + 0) * LDN + n] = f2bf(v.x);
    wt[(4 * q + 1) * LDN + n] = f2bf(v.y);
    wt[(4 * q + 2) * LDN + n] = f2bf(v.z);
    wt[(4 * q + 3) * LDN + n] = f2bf(v.w);
  }
  __syncthreads();
  // wave: 16 kk rows (A = W^T rows kk) x 64 m columns (B = g^T columns m): 4 tiles
  const int kkw = wave * 16;
  const bf16x8 zero8 = {};
  for (int mi = 0; mi < mrep; ++mi) {
  const int m0 = (blockIdx.y * mrep + mi) * 64;
  if (m0 >= M) break;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int n0 = 0; n0 < NP; n0 += 32) {
    const bf16x8 fa = *(const bf16x8*)(wt + (kkw + r) * LDN + n0 + 8 * gq);
    const int nc = n0 + 8 * gq;                  // this lane group's 8 k (= n) values
    const bool vec = (N & 7) == 0 && nc + 8 <= N;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + j * 16 + r;
      const bf16* grow = g + (long long)(m < M ? m : 0) * N;
      bf16x8 v = vec ? *(const bf16x8*)(grow + nc) : dn_load8(grow, nc, N);
      if (ya) {
        const bf16* yrow = ya + (long long)(m < M ? m : 0) * N;
        const bf16x8 yv = vec ? *(const bf16x8*)(yrow + nc) : dn_load8(yrow, nc, N);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) * act_bwd_from_out(bf2f(yv[e]), act));
      }
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, m < M ? v : zero8, acc[j], 0, 0, 0);
    }
  }
  // C^T[kk][m]: lane holds m = col r of tile j, kk = kkw + 4gq .. +3
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + j * 16 + r;
    const int kk = kk0 + kkw + 4 * gq;
    if (m >= M) continue;
    bf16* o = dx + (long long)m * K + kk;
    if (kk + 4 <= K && (K & 3) == 0) {
      bf16x4 v;
      v[0] = f2bf(acc[j][0]); v[1] = f2bf(acc[j][1]); v[2] = f2bf(acc[j][2]); v[3] = f2bf(acc[j][3]);
      *(bf16x4*)o = v;
    } else {
      for (int e = 0; e < 4; ++e)
        if (kk + e < K) o[e] = f2bf(acc[j][e]);
    }
  }
  }
}

// ---------------------------------------------------------------------------
// wgrad: dW = g^T x (fp32, overwrite), db = colsum(g)
// ---------------------------------------------------------------------------
// grid (ceil(K/64), ceil(N/64)); block tile: 64 n x 64 kk; reduction over all M (padded with
// zero rows to a multiple of 32); any K, N (element loads where rows are not 16-B aligned).
// LDS (dynamic): x tile transposed [64 kk][M + 8], g tile transposed [64 n][M + 8].
// NB = 2: 128 n columns per workgroup (the x tile -- FC1's 16 MB activation -- staged once for
// both 64-column halves instead of once per half; a wave then holds 8 accumulator tiles).
// (Staging four items' loads before their LDS writes ran FC1's wgrad at 29.1 us against 25.0 us.)
template <int NB>
__global__ __launch_bounds__(DN_THREADS) void dense_wgrad_kernel(const bf16* __restrict__ g,
                                                                 const bf16* __restrict__ x,
                                                                 float* __restrict__ dw, float* __restrict__ db,
                                                                 int M, int N, int K, int mc,
                                                                 const bf16* __restrict__ ya, int act) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dn_lds[];
  // split over the batch (blockIdx.z = slice of mc rows -> its own dW / db slab, summed by
  // fn_part_reduce in a fixed order) so small dW tiles still fill the GPU
  const int mz0 = blockIdx.z * mc, mz1 = min(M, mz0 + mc);
  dw += (long long)blockIdx.z * N * K;
  if (db) db += (long long)blockIdx.z * N;
  // rows in chunks of up to DN_WG_MCH (LDS tiles), each padded with zero rows to a multiple of 32
  const int MCH = mc < DN_WG_MCH ? ((mc + 31) & ~31) : DN_WG_MCH;
  const int LDM = MCH + 8;
  bf16* xt = reinterpret_cast<bf16*>(dn_lds);
  bf16* gt = xt + 64 * LDM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, gq = lane >> 4;
  const int kk0 = blockIdx.x * 64, n0 = blockIdx.y * 64 * NB;
  const int kkw = wave * 16;
  f32x4 acc[4 * NB];
#pragma unroll
  for (int j = 0; j < 4 * NB; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbs[NB];                                 // bias gradient (first column block, tid < 64)
#pragma unroll
  for (int b = 0; b < NB; ++b) dbs[b] = 0.f;
  for (int mb = mz0; mb < mz1; mb += MCH) {
    const int rows = mz1 - mb < MCH ? mz1 - mb : MCH;
    const int MP = (rows + 31) & ~31;
    if (mb > mz0) __syncthreads();               // previous chunk's MFMA / db reads are done
    // x[mb:mb+rows][kk0:kk0+64] -> xt[kk][m]; g[..][n0:n0+64 NB] -> gt[n][m]: thread = (m, 8 columns)
    for (int idx = tid; idx < MP * 8 * NB; idx += DN_THREADS) {
      const int ml = idx / (8 * NB), q = idx % (8 * NB);
      const int m = mb + ml;
      const int kk = kk0 + 8 * q, n = n0 + 8 * q;
      const bool xq = q < 8;                     // (NB = 2: columns 8..15 stage g only)
      Pack8 vx, vg;
      if (ml >= rows) {
        vx.u = vg.u = make_uint4(0u, 0u, 0u, 0u);
      } else {
        if (!xq) {
          vx.u = make_uint4(0u, 0u, 0u, 0u);
        } else {                                 // (16-B loads when K % 8 == 0, narrower otherwise)
          vx.v = dn_load8(x + (long long)m * K, kk, K);
        }
        vg.v = dn_load8(g + (long long)m * N, n, N);
        if (ya) {                                // g = dy * act'(y) (see dense_dgrad_kernel)
          Pack8 vy;
          vy.v = dn_load8(ya + (long long)m * N, n, N);
#pragma unroll
          for (int e = 0; e < 8; ++e) vg.e[e] = f2bf(bf2f(vg.e[e]) * act_bwd_from_out(bf2f(vy.e[e]), act));
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (xq) xt[(8 * q + e) * LDM + ml] = vx.e[e];
        gt[(8 * q + e) * LDM + ml] = vg.e[e];
      }
    }
    __syncthreads();
    // C^T[kk][n] = sum_m x^T[kk][m] g[m][n]: wave = 16 kk rows x 64 NB n columns
    for (int mm = 0; mm < MP; mm += 32) {
      const bf16x8 fa = *(const bf16x8*)(xt + (kkw + r) * LDM + mm + 8 * gq);
#pragma unroll
      for (int j = 0; j < 4 * NB; ++j) {
        const bf16x8 fb = *(const bf16x8*)(gt + (j * 16 + r) * LDM + mm + 8 * gq);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[j], 0, 0, 0);
      }
    }
    if (db && blockIdx.x == 0 && tid < 64) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (n0 + 64 * b + tid < N)
          for (int m = 0; m < rows; ++m) dbs[b] += bf2f(gt[(64 * b + tid) * LDM + m]);
    }
  }
  // lane: n = n0 + 16j + r, kk = kk0 + kkw + 4gq .. +3 -> dW[n][kk..kk+3]
#pragma unroll
  for (int j = 0; j < 4 * NB; ++j) {
    const int n = n0 + j * 16 + r;
    const int kk = kk0 + kkw + 4 * gq;
    if (n >= N) continue;
    float* o = dw + (long long)n * K + kk;
    if (kk + 4 <= K && (K & 3) == 0) {
      *(float4*)o = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
    } else {
      for (int e = 0; e < 4; ++e)
        if (kk + e < K) o[e] = acc[j][e];
    }
  }
  // bias gradient: the first column block summed g over M for its 64 NB n
  if (db && blockIdx.x == 0 && tid < 64) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (n0 + 64 * b + tid < N) db[n0 + 64 * b + tid] = dbs[b];
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
// column waves per forward workgroup: 2 (128 columns, x rows read once) when N > 64 and the
// batch spans row blocks (inference chunks); one 128-row block (FC1 at training batch 128) takes
// 64-column workgroups -- 250 of them over K, one per CU: 30.6 us against 37.8 us for 128-column
// workgroups over 250 K slices (scripts/bench_fc_native.py, round-4 A/B)
// -- and so does a layer too shallow to split over K whose 128-column tiles would leave CUs idle
// (LeNet's 120 -> 84 Dense on 16,384 rows: 128 workgroups of 128 columns)
static int dn_ncw(int M, int N, int K) {
  if (N <= 64 || M <= 128) return 1;
  if (K < 512 && ((N + 127) / 128) * ((M + 127) / 128) < 256) return 1;
  return 2;
}

extern "C" int fn_dense_splits(int M, int N, int K) {
  const int ncw = dn_ncw(M, N, K);
  const int tiles = ((N + 64 * ncw - 1) / (64 * ncw)) * ((M + 127) / 128);
  // workgroups: ~256 (one per CU) for one row block -- longer K per slice, half the partial
  // slab (the same FC1 A/B: 500 workgroups 39.2 us, 250 30.6 us) -- else ~2048 waves, 2 per SIMD
  const int target = M <= 128 ? 256 : 512 / ncw;
  int S = (target + tiles - 1) / tiles;
  const int maxS = K / 256 > 0 ? K / 256 : 1;   // >= 256 k per slice
  return S < 1 ? 1 : (S > maxS ? maxS : S);
}

template <bool WB, int NCW, bool FINAL>
static void dn_fwd_part(const void* x, const void* w, void* part, int M, int N, int K, int kc, int Sr,
                        const float* bias, int act, int out_fp32, hipStream_t st) {
  const dim3 grid((N + 64 * NCW - 1) / (64 * NCW), (M + 127) / 128, Sr), blk(DN_THREADS * NCW);
  if (K % 8 == 0)
    hipLaunchKernelGGL((dense_fwd_part_kernel<true, 4, WB, NCW, FINAL>), grid, blk, 0, st, (const bf16*)x, w,
                       (float*)part, M, N, K, kc, bias, act, out_fp32);
  else
    hipLaunchKernelGGL((dense_fwd_part_kernel<false, 1, WB, NCW, FINAL>), grid, blk, 0, st, (const bf16*)x, w,
                       (float*)part, M, N, K, kc, bias, act, out_fp32);
}

template <bool WB, int NCW>
static void dn_fwd(const void* x, const void* w, const float* bias, void* out, float* part, int M, int N, int K,
                   int kc, int Sr, int act, int out_fp32, hipStream_t st) {
  if (Sr == 1) {                                 // one slice: bias + activation in the epilogue
    dn_fwd_part<WB, NCW, true>(x, w, out, M, N, K, kc, 1, bias, act, out_fp32, st);
    return;
  }
  dn_fwd_part<WB, NCW, false>(x, w, part, M, N, K, kc, Sr, nullptr, 0, 0, st);
  const long long tot = (long long)M * N;
  hipLaunchKernelGGL(dense_fwd_reduce_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(DN_THREADS), 0, st,
                     (const float*)part, bias, out, M, N, Sr, act, out_fp32);
}

// y = act(sum of S fp32 slabs [S][M][N] + b) -> bf16 (or fp32), slices added in order
extern "C" int fn_dense_fwd_reduce(const float* part, const float* bias, void* out, int M, int N, int S, int act,
                                   int out_fp32, hipStream_t st) {
  const long long tot = (long long)M * N;
  if (tot <= 0) return 0;
  hipLaunchKernelGGL(dense_fwd_reduce_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(DN_THREADS), 0, st, part, bias,
                     out, M, N, S, act, out_fp32);
  FN_CHECK_LAUNCH();
  return 0;
}

// w: fp32 [N][K] (training: the master weights) or, wbf16, a bf16 copy (inference)
extern "C" int fn_dense_fwd(const void* x, const void* w, const float* bias, void* out, float* part, int M, int N,
                            int K, int S, int act, int out_fp32, int wbf16, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || S < 1) return -2;
  int kc = (K + S - 1) / S;
  kc = (kc + 31) / 32 * 32;
  const int Sr = (K + kc - 1) / kc;              // slices actually covering K
  const int ncw = dn_ncw(M, N, K);
  if (wbf16) {
    if (ncw == 2) dn_fwd<true, 2>(x, w, bias, out, part, M, N, K, kc, Sr, act, out_fp32, st);
    else dn_fwd<true, 1>(x, w, bias, out, part, M, N, K, kc, Sr, act, out_fp32, st);
  } else {
    if (ncw == 2) dn_fwd<false, 2>(x, w, bias, out, part, M, N, K, kc, Sr, act, out_fp32, st);
    else dn_fwd<false, 1>(x, w, bias, out, part, M, N, K, kc, Sr, act, out_fp32, st);
  }
  FN_CHECK_LAUNCH();
  return 0;
}

static int dn_lds_attr(const void* fn, size_t lds) {
  if (lds <= 64 * 1024) return 0;
  return (int)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// ya / act: see dense_dgrad_kernel (null: g is the gradient itself)
extern "C" int fn_dense_dgrad(const void* g, const float* w, void* dx, int M, int N, int K, hipStream_t st,
                              const void* ya, int act) {
  if (M <= 0 || K <= 0 || N <= 0) return -2;   // (any K: rows of W and dx not 4-aligned go scalar)
  const size_t lds = (size_t)64 * (((N + 31) & ~31) + 8) * 2;
  if (lds > 160 * 1024) return -4;
  if (int e = dn_lds_attr((const void*)dense_dgrad_kernel, lds)) return e;
  // row blocks per workgroup: up to 4 when the K tiles alone fill the GPU
  const int mblk = (M + 63) / 64;
  const int mrep = (K + 63) / 64 >= 512 ? (mblk < 4 ? mblk : 4) : 1;
  hipLaunchKernelGGL(dense_dgrad_kernel, dim3((K + 63) / 64, (mblk + mrep - 1) / mrep), dim3(DN_THREADS), lds, st,
                     (const bf16*)g, w, (bf16*)dx, M, N, K, (const bf16*)ya, act, mrep);
  FN_CHECK_LAUNCH();
  return 0;
}

// batch slices of the weight gradient: enough (dW tile, slice) workgroups for the 256 CUs, at
// least 128 rows per slice (a 128-row batch -- FeatureNet-3D's FC layers -- stays one launch)
extern "C" int fn_dense_wgrad_slices(int M, int N, int K) {
  const int tiles = ((K + 63) / 64) * ((N + 63) / 64);
  int S = (256 + tiles - 1) / tiles;
  const int maxS = M / 128 > 1 ? M / 128 : 1;
  return S < 1 ? 1 : (S > maxS ? maxS : S);
}

// part: fp32 [S][N*K] + [S][N] workspace when S > 1 (fn_dense_wgrad_slices), else unused
extern "C" int fn_dense_wgrad(const void* g, const void* x, float* dw, float* db, int M, int N, int K, float* part,
                              int S, hipStream_t st, const void* ya, int act) {
  if (M <= 0 || N <= 0 || K <= 0 || S < 1 || (S > 1 && !part)) return -2;
  int mc = (M + S - 1) / S;
  mc = (mc + 31) & ~31;
  S = (M + mc - 1) / mc;                         // slices actually covering M
  const int mch = mc < DN_WG_MCH ? mc : DN_WG_MCH;
  // 128-column workgroups when N > 64 and the K tiles alone fill the GPU (FC1: 1000 tiles)
  // (NB = 2 -- x staged once for both 64-column halves -- measured slower on FC1: 42.8 vs 29.6 us)
  const int nb = 1;
  const size_t lds = (size_t)(64 + 64 * nb) * (mch + 8) * 2;
  if (lds > 160 * 1024) return -4;
  const long long NK = (long long)N * K;
  float* pdw = S > 1 ? part : dw;
  float* pdb = S > 1 ? (db ? part + (long long)S * NK : nullptr) : db;
  if (nb == 2) {
    if (int e = dn_lds_attr((const void*)dense_wgrad_kernel<2>, lds)) return e;
    hipLaunchKernelGGL(dense_wgrad_kernel<2>, dim3((K + 63) / 64, (N + 127) / 128, S), dim3(DN_THREADS), lds, st,
                       (const bf16*)g, (const bf16*)x, pdw, pdb, M, N, K, mc, (const bf16*)ya, act);
  } else {
    if (int e = dn_lds_attr((const void*)dense_wgrad_kernel<1>, lds)) return e;
    hipLaunchKernelGGL(dense_wgrad_kernel<1>, dim3((K + 63) / 64, (N + 63) / 64, S), dim3(DN_THREADS), lds, st,
                       (const bf16*)g, (const bf16*)x, pdw, pdb, M, N, K, mc, (const bf16*)ya, act);
  }
  FN_CHECK_LAUNCH();
  if (S > 1) {                                   // (fixed slice order: fn_part_reduce, overwrite)
    return fn_part_reduce2(part, dw, NK, db ? part + (long long)S * NK : nullptr, db, db ? (long long)N : 0, S, 0, st);
  }
  return 0;
}
