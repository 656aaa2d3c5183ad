// Pointwise (1x1x1, stride 1) convolutions = skinny GEMMs over every voxel:
//   forward  Y[M][N] = act(X[M][K] @ W^T + b)      (W: [N][K])
//   dgrad    dX[M][K] = dY[M][N] @ W               (same kernel, W passed as [K][N])
//   wgrad    dW[N][K] += dY^T @ X                  (reduction over M)
// with K, N <= 64 (the segmentation classifier is 32 -> 25, SqueezeNet squeeze /
// expand and the reference's combination projections are 1x1 as well).
//
// These are HBM-bound (two tiny matrices per voxel row), so the design goal is
// streaming: persistent workgroups walk 256-row tiles; a tile of a channels-last
// tensor is ONE contiguous run of 256*K bf16, loaded with 16-byte vectors
// regardless of K (25 is fine) and scattered into a padded LDS layout that the
// MFMA fragments read with aligned ds_read_b128; the next tile's loads are in
// flight while the current one computes.  Weights live in registers as MFMA B
// fragments for the whole kernel.  Output goes back through LDS so the global
// stores are 16-byte vectors too.
//
// Reference parity: Keras Conv2D with kernel (1,1) (model/input.py:294) and the
// combination projection (model/operation.py:179-186).
#include "common.h"

#define PW_BM 256
#define PW_NTHR 256


__device__ __forceinline__ int pw_tiles(long long M) { return (int)((M + PW_BM - 1) / PW_BM); }

// Y = act(X W^T + b).  KP / NP: K, N padded to 32 / 64.  Dynamic LDS: the A tile
// [256][KP+8] and the output staging [256][NP+8] share one region (bf16).
// PRO: -1 = plain input; ACT_NONE / ACT_RELU = input prologue x <- act(x * psc[k] + psh[k])
// BWS: ACT_NONE / ACT_RELU = the output is the gradient dz of a BN+act layer whose pre-BN input
//   sy [M][N] (scale ssc, shift ssh) is read alongside: each workgroup also sums that BN's raw
//   backward moments (sum g, sum g*y), g = dz * act'(y*ssc+ssh), into spart[block][2][N]
//   (bn_finalize MODE 2) -- the colstats pass over dz and y disappears (N % 8 == 0, 2048 % N == 0)
// XENT: the layer is a classifier head whose logits feed softmax + categorical cross-entropy against
//   int64 labels[M] (the per-voxel segmentation loss): every thread takes one row of the staged
//   logit tile, computes its log-sum-exp loss, top-1 hit and d(logits) = (softmax - target) * xscale
//   (label smoothing as softmax_xent_tile_kernel), and the tile's d(logits) -- not the logits --
//   are stored; per-workgroup (loss sum, hits) go to xpart[block][2].  The logits never reach HBM
//   and the separate loss kernel (one read of the logits + one write of d(logits)) disappears.
template <int KP, int NP, int ACT, bool HAS_BIAS, int PRO = -1, int BWS = -1, bool XENT = false>
__global__ __launch_bounds__(PW_NTHR, 2) void pw_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ y,
                                                           long long M, int K, int N, const float* __restrict__ psc,
                                                           const float* __restrict__ psh,
                                                           const bf16* __restrict__ sy = nullptr,
                                                           const float* __restrict__ ssc = nullptr,
                                                           const float* __restrict__ ssh = nullptr,
                                                           float* __restrict__ spart = nullptr,
                                                           const long long* __restrict__ labels = nullptr,
                                                           float* __restrict__ xpart = nullptr, float xscale = 0.f,
                                                           float smoothing = 0.f) {
  constexpr int LDA = KP + 8, LDO = NP + 8;
  constexpr int KS = KP / 32, NT = NP / 16;
  constexpr int CH = KP / 8;                     // 16-B chunks per thread of a 256 x KP tile
  extern __shared__ __attribute__((aligned(16))) unsigned char pw_dsm[];
  bf16* As = reinterpret_cast<bf16*>(pw_dsm);
  bf16* Os = As;                                 // aliased: staged only after the MFMAs have read As
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;

  auto zero_pad = [&]() {                       // K padding of the A tile (the scatter never writes it)
    for (int i = tid; i < PW_BM * (LDA - K); i += PW_NTHR) As[(i / (LDA - K)) * LDA + K + i % (LDA - K)] = f2bf(0.f);
  };
  // weights -> B fragments (k rows beyond K and n cols beyond N are zero)
  bf16x8 fb[KS][NT];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nt * 16 + lr;
      Pack8 p;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = ks * 32 + lg * 8 + j;
        p.e[j] = (n < N && k < K) ? w[(long long)n * K + k] : f2bf(0.f);
      }
      fb[ks][nt] = __builtin_bit_cast(bf16x8, p.u);
    }
  float bv[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nt * 16 + lr;
    bv[nt] = (HAS_BIAS && n < N) ? bias[n] : 0.f;
  }

  // optional input prologue x <- act(x * psc[k] + psh[k]) (a BatchNorm + activation whose
  // normalised output is never written): with K % 8 == 0 and 2048 % K == 0 (host check)
  // every chunk this thread loads starts at channel (8 tid) mod K, so 8 scale/shift pairs
  // in registers cover all of them
  constexpr int NPV = PRO >= 0 ? 8 : 1;
  float psv[NPV], phv[NPV];
  if constexpr (PRO >= 0) {
    const int pk0 = (tid * 8) % K;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      psv[j] = psc[pk0 + j];
      phv[j] = psh[pk0 + j];
    }
  }
  constexpr int NSV = BWS >= 0 ? 8 : 1;
  float ssv[NSV], shv[NSV], sg[NSV], sgy[NSV];
  if constexpr (BWS >= 0) {                      // this thread's output chunks start at channel 8 tid mod N
    const int sn0 = (tid * 8) % N;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ssv[j] = ssc[sn0 + j];
      shv[j] = ssh[sn0 + j];
      sg[j] = sgy[j] = 0.f;
    }
  }
  const int ntiles = pw_tiles(M);
  float xl = 0.f, xc = 0.f;                      // XENT: this thread's loss / top-1 hit sums
  uint4 rb[CH];
  auto load = [&](int t) {                       // tile t: 256*K contiguous bf16 (16-B aligned: 512*K*t)
    const long long e0 = (long long)t * PW_BM * K;
    const long long nel = (M - (long long)t * PW_BM < PW_BM ? M - (long long)t * PW_BM : PW_BM) * K;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = i * PW_NTHR + tid;
      // M % 8 == 0 (host check): every tile is a whole number of 16-B chunks
      rb[i] = *(const uint4*)(x + e0 + (c * 8 < nel ? c * 8 : 0));
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    const int rows = (int)(M - (long long)t * PW_BM < PW_BM ? M - (long long)t * PW_BM : PW_BM);
    __syncthreads();                             // previous tile's Os readers are done
    zero_pad();                                  // Os staging overwrote the padding
#pragma unroll
    for (int i = 0; i < CH; ++i) {            // scatter flat chunk -> padded rows
      const int c = i * PW_NTHR + tid;
      if (c * 8 < rows * K) {
        int r = (c * 8) / K, k = c * 8 - r * K;   // one division per chunk, then walk
        if (K % 8 == 0) {                          // chunk inside one row: one 16-B LDS store
          if constexpr (PRO >= 0) {
            Pack8 p;
            p.u = rb[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) p.e[j] = f2bf(act_fwd(bf2f(p.e[j]) * psv[j] + phv[j], PRO));
            *(uint4*)(As + r * LDA + k) = p.u;
          } else {
            *(uint4*)(As + r * LDA + k) = rb[i];
          }
        } else {
          Pack8 p;
          p.u = rb[i];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            As[r * LDA + k] = p.e[j];
            if (++k == K) { k = 0; ++r; }
          }
        }
      }
    }
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);   // next tile in flight during the MFMAs
    f32x4 acc[4][NT];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 fa = *(const bf16x8*)(As + (wave * 64 + mt * 16 + lr) * LDA + ks * 32 + lg * 8);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[ks][nt], acc[mt][nt], 0, 0, 0);
      }
    __syncthreads();                             // all MFMA reads of As done before Os overwrites it
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Os[(wave * 64 + mt * 16 + lg * 4 + r) * LDO + nt * 16 + lr] = f2bf(act_fwd(acc[mt][nt][r] + bv[nt], ACT));
    __syncthreads();
    if constexpr (XENT) {
      // one row per thread, from the stored bf16 logits (the values the unfused loss would read)
      if (tid < rows) {
        bf16* orow = Os + tid * LDO;
        const long long yl = labels[(long long)t * PW_BM + tid];
        const float off = smoothing / (float)N, on = 1.f - smoothing + off;
        float v[NP];
        float mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int c = 0; c < NP; ++c) {
          v[c] = c < N ? bf2f(orow[c]) : -INFINITY;
          if (v[c] > mx) { mx = v[c]; am = c; }
        }
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < NP; ++c) se += c < N ? __expf(v[c] - mx) : 0.f;
        const float lse = mx + __logf(se);
        float lrow = 0.f;
#pragma unroll
        for (int c = 0; c < NP; ++c) {
          if (c < N) {
            const float lp = v[c] - lse;
            const float tgt = (c == yl) ? on : off;
            lrow -= tgt * lp;
            orow[c] = f2bf((__expf(lp) - tgt) * xscale);   // own row only: no race
          }
        }
        xl += lrow;
        xc += (am == yl) ? 1.f : 0.f;
      }
      __syncthreads();
    }
    // gather padded rows -> flat 256*N run, 16-B stores
    const long long o0 = (long long)t * PW_BM * N;
    const int nel = rows * N;
    for (int c = tid; c * 8 < nel; c += PW_NTHR) {
      Pack8 p;
      int r = (c * 8) / N, n = c * 8 - r * N;
      if (N % 8 == 0) {
        p.u = *(const uint4*)(Os + r * LDO + n);
        if constexpr (BWS >= 0) {
          Pack8 q;
          q.u = *(const uint4*)(sy + o0 + c * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float yv = bf2f(q.e[j]);
            const float gv = bf2f(p.e[j]) * act_bwd_from_out(act_fwd(yv * ssv[j] + shv[j], BWS), BWS);
            sg[j] += gv;
            sgy[j] += gv * yv;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          p.e[j] = Os[r * LDO + n];
          if (++n == N) { n = 0; ++r; }
        }
      }
      *(uint4*)(y + o0 + c * 8) = p.u;           // rows * N is a multiple of 8 (M % 8 == 0)
    }
  }
  if constexpr (XENT) {
    // (loss sum, hits) of the workgroup, fixed order: waves, then the 4 wave sums
    xl = wave_sum(xl);
    xc = wave_sum(xc);
    __syncthreads();
    float* red = reinterpret_cast<float*>(pw_dsm);
    if (lane == 0) {
      red[wave] = xl;
      red[4 + wave] = xc;
    }
    __syncthreads();
    if (tid == 0) {
      xpart[2 * blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
      xpart[2 * blockIdx.x + 1] = (red[4] + red[5]) + (red[6] + red[7]);
    }
  }
  if constexpr (BWS >= 0) {
    // block reduction of the BN-backward moments (fixed order): thread t holds channels
    // (8t mod N) .. +7; the dynamic LDS (>= 256 x 40 bf16) is free after the last tile
    __syncthreads();
    float* red = reinterpret_cast<float*>(pw_dsm);   // [256][16]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[tid * 16 + j] = sg[j];
      red[tid * 16 + 8 + j] = sgy[j];
    }
    __syncthreads();
    const int cpr = N / 8;
    for (int c = tid; c < N; c += PW_NTHR) {
      float a = 0.f, b2 = 0.f;
      for (int t2 = c / 8; t2 < PW_NTHR; t2 += cpr) {
        a += red[t2 * 16 + (c & 7)];
        b2 += red[t2 * 16 + 8 + (c & 7)];
      }
      spart[(long long)blockIdx.x * 2 * N + c] = a;
      spart[(long long)blockIdx.x * 2 * N + N + c] = b2;
    }
  }
}

// dW[N][K] += sum_rows dY[row][n] * X[row][k].  Both tiles are scattered into LDS
// TRANSPOSED ([channel][row]) so the MFMA operands (k = rows) are contiguous
// 8-row runs; per-wave fp32 accumulators over a static (strided) tile set, added across the
// waves in a fixed order and stored into the workgroup's partial row of `dw` ([gridDim.x][N][K]),
// summed by fn_part_reduce in a fixed order (bitwise repeatable).
template <int KP, int NP, int PRO = -1>
__global__ __launch_bounds__(PW_NTHR, 2) void pw_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                             float* __restrict__ dw, long long M, int K, int N,
                                                             const float* __restrict__ psc,
                                                             const float* __restrict__ psh) {
  constexpr int LDR = PW_BM + 8;                 // row stride of the transposed tiles
  constexpr int NTN = NP / 16, NTK = KP / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char pw_dsm[];
  bf16* Yt = reinterpret_cast<bf16*>(pw_dsm);    // [NP][LDR]
  bf16* Xt = Yt + NP * LDR;                      // [KP][LDR]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  // padded channels (n >= N, k >= K) stay zero
  for (int i = tid; i < NP * LDR; i += PW_NTHR) Yt[i] = f2bf(0.f);
  for (int i = tid; i < KP * LDR; i += PW_NTHR) Xt[i] = f2bf(0.f);

  // each wave owns a 64-row quarter of the tile's k dimension (2 k-steps of 32 rows)
  f32x4 acc[NTN][NTK];
#pragma unroll
  for (int a = 0; a < NTN; ++a)
#pragma unroll
    for (int b = 0; b < NTK; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int ntiles = pw_tiles(M);
  constexpr int CY = NP / 8, CX = KP / 8;        // 16-B chunks per thread of the dy / x tiles
  uint4 ry[CY], rx[CX];
  auto load = [&](const bf16* src, int C, int t, uint4* rb, int nch) {
    const long long e0 = (long long)t * PW_BM * C;
    const long long nel = (M - (long long)t * PW_BM < PW_BM ? M - (long long)t * PW_BM : PW_BM) * C;
#pragma unroll
    for (int i = 0; i < nch; ++i) {
      const int c = i * PW_NTHR + tid;
      rb[i] = *(const uint4*)(src + e0 + (c * 8 < nel ? c * 8 : 0));
    }
  };
  // optional prologue on x (as pw_fwd_kernel): x <- act(x * psc[k] + psh[k])
  auto scatter_t = [&](bf16* dst, const uint4* rb, int C, int rows, int nch) {
#pragma unroll
    for (int i = 0; i < nch; ++i) {
      const int c = i * PW_NTHR + tid;
      if (c * 8 < rows * C) {
        Pack8 p;
        p.u = rb[i];
        int r = (c * 8) / C, k = c * 8 - r * C;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dst[k * LDR + r] = p.e[j];
          if (++k == C) { k = 0; ++r; }
        }
      }
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) { load(dy, N, t, ry, CY); load(x, K, t, rx, CX); }
  for (; t < ntiles; t += gridDim.x) {
    const int rows = (int)(M - (long long)t * PW_BM < PW_BM ? M - (long long)t * PW_BM : PW_BM);
    __syncthreads();
    scatter_t(Yt, ry, N, rows, CY);
    scatter_t(Xt, rx, K, rows, CX);
    if (rows < PW_BM) {                          // ragged last tile: zero the unused rows
      for (int i = tid; i < NP * (PW_BM - rows); i += PW_NTHR) Yt[(i / (PW_BM - rows)) * LDR + rows + i % (PW_BM - rows)] = f2bf(0.f);
    }
    __syncthreads();
    if constexpr (PRO >= 0) {
      // input prologue x <- act(x * psc[k] + psh[k]) on the transposed tile in LDS: channel k is
      // one LDS row, so a thread takes 32 consecutive rows of one channel with two scalars
      // (no per-element parameter registers; rows past a ragged tile's end meet dy = 0)
      for (int k = tid >> 3; k < K; k += PW_NTHR / 8) {
        const float a = psc[k], c = psh[k];
        bf16* row = Xt + k * LDR + (tid & 7) * 32;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          Pack8 p;
          p.u = *(const uint4*)(row + v * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) p.e[j] = f2bf(act_fwd(bf2f(p.e[j]) * a + c, PRO));
          *(uint4*)(row + v * 8) = p.u;
        }
      }
      __syncthreads();
    }
    if (t + gridDim.x < ntiles) { load(dy, N, t + gridDim.x, ry, CY); load(x, K, t + gridDim.x, rx, CX); }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = wave * 64 + kk * 32 + lg * 8;
      bf16x8 fa[NTN], fb[NTK];
#pragma unroll
      for (int a = 0; a < NTN; ++a) fa[a] = *(const bf16x8*)(Yt + (a * 16 + lr) * LDR + r0);
#pragma unroll
      for (int b = 0; b < NTK; ++b) fb[b] = *(const bf16x8*)(Xt + (b * 16 + lr) * LDR + r0);
#pragma unroll
      for (int a = 0; a < NTN; ++a)
#pragma unroll
        for (int b = 0; b < NTK; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
  }
  // D[row = n][col = k]: lane holds n = a*16 + lg*4 + r, k = b*16 + lr.  Every wave holds a partial
  // of the WHOLE [N][K] block (its quarter of the rows): the four are added through LDS in wave
  // order (4 x NP x KP fp32 fit in the tiles' LDS), then stored as the workgroup's partial row
  __syncthreads();
  float* red = reinterpret_cast<float*>(pw_dsm);
#pragma unroll
  for (int a = 0; a < NTN; ++a)
#pragma unroll
    for (int b = 0; b < NTK; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wave * NP + a * 16 + lg * 4 + r) * KP + b * 16 + lr] = acc[a][b][r];
  __syncthreads();
  for (int i = tid; i < NP * KP; i += PW_NTHR) {
    const int n = i / KP, k = i % KP;
    if (n < N && k < K)
      dw[((long long)blockIdx.x * N + n) * K + k] =
          ((red[i] + red[NP * KP + i]) + red[2 * NP * KP + i]) + red[3 * NP * KP + i];
  }
}

static int g_pw_cus = 0;
static int pw_grid(long long M, int per_cu) {
  if (g_pw_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_pw_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_pw_cus <= 0)
      g_pw_cus = 256;
  }
  const int tiles = (int)((M + PW_BM - 1) / PW_BM);
  const int g = g_pw_cus * per_cu;
  return tiles < g ? (tiles > 0 ? tiles : 1) : g;
}

// x: bf16 [M][K], w: bf16 [N][K] (row n = output channel), y: bf16 [M][N]; K, N <= 64
// psc / psh (optional, fp32 [K]): input prologue x <- pact(x * psc + psh); needs K % 8 == 0 and
// 2048 % K == 0
static bool pw_pro_ok(const float* psc, const float* psh, int K) {
  return !psc || (psh && K % 8 == 0 && 2048 % K == 0);
}

// grid of the BWS (dgrad + BN-backward moments) launch = rows of its spart slab: 3 workgroups per
// CU (165 VGPRs: occupancy 3, so a 4-per-CU persistent grid would leave a serial tail)
extern "C" int fn_pw_fwd_blocks(long long M, int K, int N) {
  (void)K; (void)N;
  return pw_grid(M, 3);
}

extern "C" int fn_pw_fwd(const void* x, const void* w, const float* bias, void* y, long long M, int K, int N, int act,
                         hipStream_t st, const float* psc, const float* psh, int pact, const void* sy,
                         const float* ssc, const float* ssh, float* spart, int sact) {
  if (K < 1 || K > 64 || N < 1 || N > 64 || M < 8 || M % 8) return -2;
  if (!pw_pro_ok(psc, psh, K)) return -2;
  // ~110-200 VGPRs and <= 37 KB LDS: 4 workgroups per CU for the 32-channel variants
  const dim3 grid((unsigned)pw_grid(M, (K <= 32 && N <= 32) ? 4 : 2));
  if (sy) {                                      // dgrad + BN-backward moments (see BWS)
    if (psc || bias || act != ACT_NONE || !ssc || !ssh || !spart || N % 8 || 2048 % N ||
        (sact != ACT_NONE && sact != ACT_RELU) || K > 32 || N > 32)
      return -2;
#define PWS(SA)                                                                                              \
  hipLaunchKernelGGL((pw_fwd_kernel<32, 32, ACT_NONE, false, -1, SA>), dim3((unsigned)fn_pw_fwd_blocks(M, K, N)),  \
                     dim3(PW_NTHR),                                                                            \
                     (size_t)PW_BM * (32 + 8) * 2, st, (const bf16*)x, (const bf16*)w, nullptr, (bf16*)y, M, K, N, \
                     nullptr, nullptr, (const bf16*)sy, ssc, ssh, spart)
    if (sact == ACT_RELU) PWS(ACT_RELU); else PWS(ACT_NONE);
#undef PWS
    FN_CHECK_LAUNCH();
    return 0;
  }
  const bool hb = bias != nullptr;
  // (the 64-channel prologue instances need > 64 KB of LDS only for KP = NP = 64: not emitted)
#define PWF(KP, NP, A, HB)                                                                                   \
  do {                                                                                                         \
    const size_t lds = (size_t)PW_BM * ((KP > NP ? KP : NP) + 8) * 2;                                        \
    if (lds > 64 * 1024 &&                                                                                     \
        hipFuncSetAttribute((const void*)pw_fwd_kernel<KP, NP, A, HB>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                            (int)lds) != hipSuccess)                                                           \
      return -4;                                                                                               \
    hipLaunchKernelGGL((pw_fwd_kernel<KP, NP, A, HB>), grid, dim3(PW_NTHR), lds, st, (const bf16*)x,          \
                       (const bf16*)w, bias, (bf16*)y, M, K, N, nullptr, nullptr);                             \
  } while (0)
  // prologue instances (the BN + act of the producing layer): identity output, bias or not,
  // K <= 32 or 64, N <= 32 or 64
#define PWP(KP, NP, HB, PA)                                                                                  \
  hipLaunchKernelGGL((pw_fwd_kernel<KP, NP, ACT_NONE, HB, PA>), grid, dim3(PW_NTHR),                           \
                     (size_t)PW_BM * ((KP > NP ? KP : NP) + 8) * 2, st, (const bf16*)x, (const bf16*)w, bias,    \
                     (bf16*)y, M, K, N, psc, psh)
  if (psc) {
    if (act != ACT_NONE || (pact != ACT_NONE && pact != ACT_RELU)) return -2;
#define PWP2(KP, NP)                                                                                         \
    do {                                                                                                     \
      if (pact == ACT_RELU) { if (hb) PWP(KP, NP, true, ACT_RELU); else PWP(KP, NP, false, ACT_RELU); }      \
      else { if (hb) PWP(KP, NP, true, ACT_NONE); else PWP(KP, NP, false, ACT_NONE); }                       \
    } while (0)
    if (K <= 32) { if (N <= 32) PWP2(32, 32); else PWP2(32, 64); }
    else { if (N <= 32) PWP2(64, 32); else PWP2(64, 64); }
#undef PWP2
#undef PWP
    FN_CHECK_LAUNCH();
    return 0;
  }
#define PWA(KP, NP)                                                          \
  do {                                                                       \
    if (act == ACT_RELU) { if (hb) PWF(KP, NP, ACT_RELU, true); else PWF(KP, NP, ACT_RELU, false); } \
    else if (act == ACT_NONE) { if (hb) PWF(KP, NP, ACT_NONE, true); else PWF(KP, NP, ACT_NONE, false); } \
    else if (act == ACT_TANH) PWF(KP, NP, ACT_TANH, true);                  \
    else PWF(KP, NP, ACT_SIGMOID, true);                                     \
  } while (0)
  if ((act == ACT_TANH || act == ACT_SIGMOID) && !hb) return -5;
  if (K <= 32) { if (N <= 32) PWA(32, 32); else PWA(32, 64); }
  else { if (N <= 32) PWA(64, 32); else PWA(64, 64); }
#undef PWA
#undef PWF
  FN_CHECK_LAUNCH();
  return 0;
}

// Classifier head + softmax cross-entropy (XENT instances): dlog [M][N] bf16 = d(mean loss)/d(logits)
// with xscale = 1/M folded in (the unscaled loss is sum(xpart[:, 0]) * xscale ... / M), labels
// int64 [M] (no ignore index), xpart fp32 [fn_pw_xent_blocks(M)][2] = per-workgroup (loss sum, top-1
// hits).  K, N <= 32, identity activation; psc / psh: the optional BN + act input prologue.
extern "C" int fn_pw_xent_blocks(long long M) { return pw_grid(M, 3); }   // (143-159 VGPRs: 3 per CU)

extern "C" int fn_pw_fwd_xent(const void* x, const void* w, const float* bias, void* dlog, long long M, int K, int N,
                              const float* psc, const float* psh, int pact, const long long* labels, float* xpart,
                              float xscale, float smoothing, hipStream_t st) {
  if (K < 1 || K > 32 || N < 2 || N > 32 || M < 8 || M % 8 || !labels || !xpart) return -2;
  if (!pw_pro_ok(psc, psh, K) || (psc && pact != ACT_NONE && pact != ACT_RELU)) return -2;
  const dim3 grid((unsigned)fn_pw_xent_blocks(M));
  const size_t lds = (size_t)PW_BM * (32 + 8) * 2;
  const bool hb = bias != nullptr;
#define PWX(HB, PA)                                                                                          \
  hipLaunchKernelGGL((pw_fwd_kernel<32, 32, ACT_NONE, HB, PA, -1, true>), grid, dim3(PW_NTHR), lds, st,       \
                     (const bf16*)x, (const bf16*)w, bias, (bf16*)dlog, M, K, N, psc, psh, nullptr, nullptr,     \
                     nullptr, nullptr, labels, xpart, xscale, smoothing)
  if (!psc) { if (hb) PWX(true, -1); else PWX(false, -1); }
  else if (pact == ACT_RELU) { if (hb) PWX(true, ACT_RELU); else PWX(false, ACT_RELU); }
  else { if (hb) PWX(true, ACT_NONE); else PWX(false, ACT_NONE); }
#undef PWX
  FN_CHECK_LAUNCH();
  return 0;
}

// rows of the partial slab fn_pw_wgrad needs ([rows][N][K] fp32)
extern "C" int fn_pw_wgrad_blocks(long long M, int K, int N) { return pw_grid(M, (K <= 32 && N <= 32) ? 3 : 2); }

// dw: fp32 [N][K], accumulated into (zero it for a fresh gradient); part: fp32 scratch
// [fn_pw_wgrad_blocks][N][K]
extern "C" int fn_pw_wgrad(const void* dy, const void* x, float* dw, long long M, int K, int N, hipStream_t st,
                           const float* psc, const float* psh, int pact, float* part) {
  if (K < 1 || K > 64 || N < 1 || N > 64 || M < 8 || M % 8) return -2;
  if (!pw_pro_ok(psc, psh, K)) return -2;
  if (!part) return -6;
  const dim3 grid((unsigned)fn_pw_wgrad_blocks(M, K, N));
#define PWW(KP, NP)                                                                                          \
  do {                                                                                                     \
    const size_t lds = (size_t)(KP + NP) * (PW_BM + 8) * 2;                                                \
    if (lds > 64 * 1024 &&                                                                                 \
        hipFuncSetAttribute((const void*)pw_wgrad_kernel<KP, NP>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                            (int)lds) != hipSuccess)                                                       \
      return -4;                                                                                           \
    if (!psc)                                                                                              \
      hipLaunchKernelGGL((pw_wgrad_kernel<KP, NP>), grid, dim3(PW_NTHR), lds, st, (const bf16*)dy,        \
                         (const bf16*)x, part, M, K, N, nullptr, nullptr);                                 \
    else if (pact == ACT_RELU)                                                                             \
      hipLaunchKernelGGL((pw_wgrad_kernel<KP, NP, ACT_RELU>), grid, dim3(PW_NTHR), lds, st, (const bf16*)dy, \
                         (const bf16*)x, part, M, K, N, psc, psh);                                         \
    else                                                                                                   \
      hipLaunchKernelGGL((pw_wgrad_kernel<KP, NP, ACT_NONE>), grid, dim3(PW_NTHR), lds, st, (const bf16*)dy, \
                         (const bf16*)x, part, M, K, N, psc, psh);                                         \
  } while (0)
  if (psc && pact != ACT_NONE && pact != ACT_RELU) return -2;
  if (K <= 32) { if (N <= 32) PWW(32, 32); else PWW(32, 64); }
  else { if (N <= 32) PWW(64, 32); else PWW(64, 64); }
#undef PWW
  FN_CHECK_LAUNCH();
  return fn_part_reduce(part, dw, (long long)N * K, (int)grid.x, 1, st);
}
