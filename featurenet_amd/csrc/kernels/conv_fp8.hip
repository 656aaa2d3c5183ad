// FP8 (OCP e4m3) LDS-halo convolution for the inference path (CDNA4).
//
// Same tiling as the bf16 halo kernel (conv_halo.hip): an output tile of
// TD x TH x OW rows, its input halo staged in LDS per 16-channel slice, two
// taps per MFMA k-step, weights streamed through a double-buffered 128-k LDS
// stage -- but every operand byte is fp8, so the halo, the weight stages and
// every LDS fragment read are half the size of the bf16 kernel's (the bf16
// kernel is LDS-bandwidth-bound) and MFMA runs the CDNA4 block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 (k = 128 per instruction, twice the bf16 MFMA
// rate; the older mfma_f32_16x16x32_fp8_fp8 runs at the bf16 rate).
// Dequantisation is one multiply in the epilogue:
//   y = act(acc * scale[co] + bias[co])     scale[co] = s_x * s_w[co]
// and the result is either re-quantised to fp8 (y * inv_out_scale, saturated
// to +-448) for the next layer or stored as bf16.
#include "common.h"

struct F8Geom {
  int N, ID, IH, IW, C;
  int OD, OH, OW;
  int KD, KH, KW;
  int pd, ph, pw;
  int TD, TH;
};

#define F8_BM 256
#define F8_BK 128   // k (bytes) per weight stage: 8 taps x 16 channels = one MFMA k-step
#define F8_UNIT_SCALE 127   // E8M0 exponent of 1.0

typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned char f32_to_fp8(float v) {
  v = fminf(fmaxf(v, -448.f), 448.f);
  const int p = __builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
  return (unsigned char)(p & 0xff);
}

template <int BN, bool OUT_F8, bool RELU>
__global__ __launch_bounds__(256, 2) void conv_halo_f8_kernel(const unsigned char* __restrict__ src,
                                                              const unsigned char* __restrict__ wt,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ bias, void* __restrict__ out,
                                                              float inv_out_scale, const int* __restrict__ toffs,
                                                              F8Geom g, int Ncol) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  constexpr int NT = BN / 16;
  constexpr int B_STAGE = BN * F8_BK;           // bytes
  constexpr int B_CHUNKS = BN * (F8_BK / 16);
  constexpr int B_PER_T = (B_CHUNKS + 255) / 256;
  const int HD = g.TD + g.KD - 1, HH = g.TH + g.KH - 1, HW = g.OW + g.KW - 1;
  const int HP = HD * HH * HW;
  const int T = g.KD * g.KH * g.KW;
  const int T8 = (T + 7) & ~7;
  const int spp = T8 >> 3;
  const int npass = g.C >> 4;
  const int nq = spp * npass;
  const int ldw = npass * T8 * 16;
  const int rows = g.TD * g.TH * g.OW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH;

  unsigned char* halo = dsm;                                   // [HP][16]
  unsigned char* Bs = dsm + (((size_t)HP * 16 + 15) & ~(size_t)15);
  int* toffs_s = reinterpret_cast<int*>(Bs + 2 * B_STAGE);      // [T8] tap offsets (LDS, not scalar loads)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int th_i = tile % thn, td_i = (tile / thn) % tdn, n = tile / (thn * tdn);
  const int d0 = td_i * g.TD, h0 = th_i * g.TH;
  const int n0 = blockIdx.y * BN;

  int hbase[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int r = wave * 64 + mt * 16 + lr;
    const int rr = r < rows ? r : 0;
    const int w = rr % g.OW, th = (rr / g.OW) % g.TH, td = rr / (g.OW * g.TH);
    hbase[mt] = (td * HH + th) * HW + w;
  }

  auto fill_halo = [&](int p) {
    for (int c0 = 0; c0 < HP; c0 += 256 * 4) {
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pos = c0 + j * 256 + tid;
        const int hw = pos % HW, hh = (pos / HW) % HH, hd = pos / (HW * HH);
        const int gd = d0 - g.pd + hd, gh = h0 - g.ph + hh, gw = hw - g.pw;
        const bool ok = pos < HP && (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
                        (unsigned)gw < (unsigned)g.IW;
        const long long off = ((((long long)n * g.ID + gd) * g.IH + gh) * g.IW + gw) * g.C + p * 16;
        const uint4 x = *(const uint4*)(src + (ok ? off : 0));
        v[j] = ok ? x : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pos = c0 + j * 256 + tid;
        if (pos < HP) *(uint4*)(halo + (size_t)pos * 16) = v[j];
      }
    }
  };
  uint4 rb[B_PER_T];
  auto load_b = [&](int q) {
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int idx = tid + i * 256;
      const int r = (idx >> 3) < BN ? (idx >> 3) : BN - 1;
      const bool ok = idx < B_CHUNKS && n0 + r < Ncol;
      const uint4 v = *(const uint4*)(wt + (ok ? (long long)(n0 + r) * ldw + q * F8_BK + (idx & 7) * 16 : 0));
      rb[i] = ok ? v : make_uint4(0, 0, 0, 0);
    }
  };
  auto write_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int idx = tid + i * 256;
      if (idx < B_CHUNKS) {
        const int r = idx >> 3, c = idx & 7;
        *(uint4*)(Bs + buf * B_STAGE + r * F8_BK + ((c ^ (r & 7)) << 4)) = rb[i];
      }
    }
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int t = tid; t < T8; t += 256) toffs_s[t] = toffs[t];
  fill_halo(0);
  load_b(0);
  write_b(0);
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    if (q > 0 && q % spp == 0) {
      fill_halo(q / spp);
      __syncthreads();
    }
    const bool more = q + 1 < nq;
    if (more) load_b(q + 1);
    const unsigned char* b = Bs + (q & 1) * B_STAGE;
    // one block-scaled MFMA per (mt, nt) covers the whole 128-byte stage: lane group
    // lg holds k = 32 lg .. 32 lg + 31 = taps 2 lg, 2 lg + 1 of the stage's 8, all 16
    // channels of each (two 16-B halo reads per row block, two swizzled 16-B chunks of
    // the weight row)
    const int* tp = toffs_s + (q % spp) * 8 + 2 * lg;
    const int to0 = tp[0], to1 = tp[1];
    i32x8 fa[4], fb[NT];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const uint4 lo = *(const uint4*)(halo + (size_t)(hbase[mt] + to0) * 16);
      const uint4 hi = *(const uint4*)(halo + (size_t)(hbase[mt] + to1) * 16);
      fa[mt] = (i32x8){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int r = nt * 16 + lr;
      const uint4 lo = *(const uint4*)(b + r * F8_BK + (((2 * lg) ^ (r & 7)) << 4));
      const uint4 hi = *(const uint4*)(b + r * F8_BK + (((2 * lg + 1) ^ (r & 7)) << 4));
      fb[nt] = (i32x8){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
    // branch-free: rows past the tile compute on a valid halo position and are dropped.
    // Formats 0/0 = e4m3 x e4m3; E8M0 block scales 127 = 2^0 (the per-channel
    // dequantisation stays one multiply in the epilogue)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0,
                                                                         F8_UNIT_SCALE, 0, F8_UNIT_SCALE);
    __syncthreads();
    if (more) {
      write_b((q + 1) & 1);
      __syncthreads();
    }
  }

  // ---- epilogue: dequantise, bias, act, (re)quantise; staged through LDS ----
  constexpr int ESZ = OUT_F8 ? 1 : 2;
  constexpr int LDO = BN * ESZ + 16;            // bytes per staged row
  unsigned char* Os = dsm;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = nt * 16 + lr;
    const bool cv = n0 + col < Ncol;
    const float sc = cv ? scale[n0 + col] : 0.f, bv = cv ? bias[n0 + col] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 64 + mt * 16 + lg * 4 + r;
        float v = acc[mt][nt][r] * sc + bv;
        if (RELU) v = fmaxf(v, 0.f);
        if constexpr (OUT_F8) Os[row * LDO + col] = f32_to_fp8(v * inv_out_scale);
        else *(bf16*)(Os + row * LDO + col * 2) = f2bf(v);
      }
  }
  __syncthreads();
  constexpr int CB = BN * ESZ / 16;             // 16-B chunks per row
  for (int idx = tid; idx < F8_BM * CB; idx += 256) {
    const int row = idx / CB, ch = idx % CB;
    if (row >= rows) continue;
    const int w = row % g.OW, th = (row / g.OW) % g.TH, td = row / (g.OW * g.TH);
    if (d0 + td >= g.OD || h0 + th >= g.OH) continue;
    const long long m = (((long long)n * g.OD + d0 + td) * g.OH + h0 + th) * g.OW + w;
    const int col0 = ch * 16 / ESZ;
    unsigned char* dst = (unsigned char*)out + (m * Ncol + n0 + col0) * ESZ;
    if (n0 + col0 + 16 / ESZ <= Ncol && (Ncol * ESZ) % 16 == 0) {
      *(uint4*)dst = *(const uint4*)(Os + row * LDO + ch * 16);
    } else {
      for (int j = 0; j < 16 / ESZ; ++j)
        if (n0 + col0 + j < Ncol)
          for (int b2 = 0; b2 < ESZ; ++b2) dst[j * ESZ + b2] = Os[row * LDO + ch * 16 + j * ESZ + b2];
    }
  }
}

static F8Geom parse_f8(const int* v) {
  F8Geom g;
  g.N = v[0]; g.ID = v[1]; g.IH = v[2]; g.IW = v[3]; g.C = v[4];
  g.OD = v[5]; g.OH = v[6]; g.OW = v[7];
  g.KD = v[8]; g.KH = v[9]; g.KW = v[10];
  g.pd = v[11]; g.ph = v[12]; g.pw = v[13];
  g.TD = v[14]; g.TH = v[15];
  return g;
}

static size_t f8_lds(const F8Geom& g, int BN, bool out_f8) {
  const size_t hp = (size_t)(g.TD + g.KD - 1) * (g.TH + g.KH - 1) * (g.OW + g.KW - 1);
  const size_t T8 = ((size_t)g.KD * g.KH * g.KW + 7) & ~(size_t)7;
  const size_t main_ = ((hp * 16 + 15) & ~(size_t)15) + 2 * (size_t)BN * F8_BK + T8 * 4;
  const size_t epi = (size_t)F8_BM * (BN * (out_f8 ? 1 : 2) + 16);
  return (main_ > epi ? main_ : epi) + 16;
}

// src / wt: fp8 e4m3 bytes; wt [Ncol][C/16][T8][16]; scale/bias fp32 [Ncol]; out fp8 or bf16.
extern "C" int fn_conv_halo_f8(const void* src, const void* wt, const float* scale, const float* bias, void* out,
                               float inv_out_scale, const int* toffs, const int* geom16, int Ncol, int out_f8,
                               int relu, hipStream_t st) {
  const F8Geom g = parse_f8(geom16);
  if (g.C % 16 != 0 || g.TD * g.TH * g.OW > F8_BM || Ncol % 16 != 0) return -2;
  const int BN = Ncol <= 32 ? 32 : 64;
  const size_t lds = f8_lds(g, BN, out_f8 != 0);
  if (lds > 160 * 1024) return -4;
  const int tiles = g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH);
  dim3 grid((unsigned)tiles, (Ncol + BN - 1) / BN);
  const unsigned char* s = (const unsigned char*)src;
  const unsigned char* w = (const unsigned char*)wt;
#define F8CASE(B, O, R)                                                                                   \
  do {                                                                                                    \
    static size_t cfg = 0;                                                                                \
    if (lds > cfg) {                                                                                      \
      hipError_t e = hipFuncSetAttribute((const void*)conv_halo_f8_kernel<B, O, R>,                       \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);           \
      if (e != hipSuccess) return (int)e;                                                                 \
      cfg = lds;                                                                                          \
    }                                                                                                     \
    hipLaunchKernelGGL((conv_halo_f8_kernel<B, O, R>), grid, dim3(256), lds, st, s, w, scale, bias, out, \
                       inv_out_scale, toffs, g, Ncol);                                                    \
  } while (0)
#define F8BN(B)                                                        \
  do {                                                                 \
    if (out_f8) { if (relu) F8CASE(B, true, true); else F8CASE(B, true, false); }   \
    else { if (relu) F8CASE(B, false, true); else F8CASE(B, false, false); }        \
  } while (0)
  if (BN == 32) F8BN(32); else F8BN(64);
#undef F8BN
#undef F8CASE
  FN_CHECK_LAUNCH();
  return 0;
}

// x (bf16) -> fp8 e4m3 of x * inv_scale, saturated (activation quantisation between layers).
__global__ void quant_fp8_kernel(const bf16* __restrict__ x, unsigned char* __restrict__ y, long long n,
                                 float inv_scale) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  if (i + 8 <= n) {
    Pack8 p;
    p.u = *(const uint4*)(x + i);
    unsigned int lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) lo |= (unsigned)f32_to_fp8(bf2f(p.e[j]) * inv_scale) << (8 * j);
#pragma unroll
    for (int j = 0; j < 4; ++j) hi |= (unsigned)f32_to_fp8(bf2f(p.e[4 + j]) * inv_scale) << (8 * j);
    *(uint2*)(y + i) = make_uint2(lo, hi);
  } else {
    for (long long j = i; j < n; ++j) y[j] = f32_to_fp8(bf2f(x[j]) * inv_scale);
  }
}

extern "C" int fn_quant_fp8(const void* x, void* y, long long n, float inv_scale, hipStream_t st) {
  const long long threads = (n + 7) / 8;
  hipLaunchKernelGGL(quant_fp8_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (const bf16*)x,
                     (unsigned char*)y, n, inv_scale);
  FN_CHECK_LAUNCH();
  return 0;
}

// x (bf16 [M][C], C % 32 == 0, C <= 128) -> OCP MX-style block-scaled e4m3: per (row, 32-channel
// block) the E8M0 exponent e = ceil(log2(amax / 448)), y = e4m3(x * 2^-e), and byte j of the row's
// scale dword = e_j + 127 (the layout the block-scaled fp8 conv kernels read).  One thread per
// (row, block): 64 B in, 32 B + 1 scale byte out.
__global__ void quant_fp8_block_kernel(const bf16* __restrict__ x, unsigned char* __restrict__ y,
                                       unsigned char* __restrict__ sc, long long M, int C) {
  const int nb = C >> 5;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * nb) return;
  const long long row = i / nb;
  const int b = (int)(i - row * nb);
  const bf16* xs = x + row * C + 32 * b;
  Pack8 p[4];
  float am = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p[q].u = *(const uint4*)(xs + 8 * q);
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(bf2f(p[q].e[j])));
  }
  const unsigned bits = __float_as_uint(am * (1.f / 448.f));
  int e = (int)((bits >> 23) & 255u) - 127 + ((bits & 0x7fffffu) != 0u ? 1 : 0);
  if ((bits & 0x7f800000u) == 0u) e = -127;
  e = e < -127 ? -127 : (e > 126 ? 126 : e);
  const float inv = __uint_as_float((unsigned)(127 - e) << 23);
  unsigned char* ys = y + row * C + 32 * b;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) lo |= (unsigned)f32_to_fp8(bf2f(p[q].e[j]) * inv) << (8 * j);
#pragma unroll
    for (int j = 0; j < 4; ++j) hi |= (unsigned)f32_to_fp8(bf2f(p[q].e[4 + j]) * inv) << (8 * j);
    *(uint2*)(ys + 8 * q) = make_uint2(lo, hi);
  }
  sc[row * 4 + b] = (unsigned char)(e + 127);
}

// sc: uint32 [M] (one scale dword per row; bytes past C/32 are left as they are)
extern "C" int fn_quant_fp8_block(const void* x, void* y, void* sc, long long M, int C, hipStream_t st) {
  if (C % 32 || C > 128 || M < 0) return -2;
  const long long n = M * (C / 32);
  if (n == 0) return 0;
  hipLaunchKernelGGL(quant_fp8_block_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const bf16*)x,
                     (unsigned char*)y, (unsigned char*)sc, M, C);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// fp8 stem input: space-to-depth (factor 2^3) of a 1-channel volume, with J consecutive
// w-taps of the packed grid folded into the channels, quantised to e4m3.
// ---------------------------------------------------------------------------
// x: bf16 [N, D, H, W] (1 channel).  y: e4m3 [N, D2, H2, W2o, 8J] with
//   y[n, d, h, w, 8j + (pd*4 + ph*2 + pw)] = e4m3(x[n, 2d+pd, 2h+ph, 2(w+j)+pw] * inv_scale)
// (zero outside x).  A 2^3-stride conv of kernel k^3 over x is then a stride-1 conv of
// taps (k2, k2, 1) over y (k2 = ceil(k/2), J = k2; the weight is the space-to-depth weight
// [K][k2][k2][k2][8] viewed as [K][k2][k2][1][8 k2]): 8J = 32 channels fit the fp8 tile
// kernel's 32-channel slices, where the plain space-to-depth input has 8.
// Block = 4 packed rows (n, d, h) x 64 w: each thread quantises the 8 space-to-depth bytes of
// ONE packed position (4 dword loads: two bf16 of each (pd, ph)) into LDS, then assembles
// the 32 output bytes of its position from LDS slots w .. w+3 (the rows of 64 cover W2o + 3
// <= 64 packed positions) -- every x element is loaded once, stores are 16 B.
// I8: int8 bytes of rint(x * inv_scale) saturated to [-127, 127] instead of e4m3 (the int8 stem:
// binary voxels are exact either way).
template <bool I8>
__global__ __launch_bounds__(256) void s2d_tap_f8_kernel(const bf16* __restrict__ x, unsigned char* __restrict__ y,
                                                         int N, int D, int H, int W, int D2, int H2, int W2o, int J,
                                                         float inv_scale) {
  __shared__ uint2 s8[4][64];
  const int lane = threadIdx.x & 63, rw = threadIdx.x >> 6;
  const long long row = (long long)blockIdx.x * 4 + rw;          // (n, d, h) packed row
  const long long nrows = (long long)N * D2 * H2;
  const int h = (int)(row % H2), d = (int)((row / H2) % D2), n = (int)(row / ((long long)H2 * D2));
  unsigned char b[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) b[q] = 0;
  const int xw = 2 * lane;
  if (row < nrows) {
#pragma unroll
    for (int pd = 0; pd < 2; ++pd)
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        const int xd = 2 * d + pd, xh = 2 * h + ph;
        if (xd >= D || xh >= H) continue;
        const bf16* xr = x + (((long long)n * D + xd) * H + xh) * W;
        float v0 = 0.f, v1 = 0.f;
        if (xw + 1 < W && (W & 1) == 0) {        // (even W: a 4-byte aligned pair)
          const unsigned u = *(const unsigned*)(xr + xw);
          v0 = __uint_as_float(u << 16);
          v1 = __uint_as_float(u & 0xffff0000u);
        } else {
          if (xw < W) v0 = bf2f(xr[xw]);
          if (xw + 1 < W) v1 = bf2f(xr[xw + 1]);
        }
        if constexpr (I8) {
          b[pd * 4 + ph * 2] = (unsigned char)(signed char)(int)fminf(fmaxf(rintf(v0 * inv_scale), -127.f), 127.f);
          b[pd * 4 + ph * 2 + 1] = (unsigned char)(signed char)(int)fminf(fmaxf(rintf(v1 * inv_scale), -127.f), 127.f);
        } else {
          b[pd * 4 + ph * 2] = f32_to_fp8(v0 * inv_scale);
          b[pd * 4 + ph * 2 + 1] = f32_to_fp8(v1 * inv_scale);
        }
      }
  }
  s8[rw][lane] = make_uint2((unsigned)b[0] | ((unsigned)b[1] << 8) | ((unsigned)b[2] << 16) | ((unsigned)b[3] << 24),
                            (unsigned)b[4] | ((unsigned)b[5] << 8) | ((unsigned)b[6] << 16) | ((unsigned)b[7] << 24));
  __syncthreads();
  if (row >= nrows || lane >= W2o) return;
  uint2 t[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = (j < J && lane + j < 64) ? s8[rw][lane + j] : make_uint2(0u, 0u);
  uint4* o = reinterpret_cast<uint4*>(y + (row * W2o + lane) * (8LL * J));
  o[0] = make_uint4(t[0].x, t[0].y, t[1].x, t[1].y);
  if (J == 4) o[1] = make_uint4(t[2].x, t[2].y, t[3].x, t[3].y);
}

extern "C" int fn_s2d_tap_f8(const void* x, void* y, int N, int D, int H, int W, int D2, int H2, int W2o, int J,
                             float inv_scale, int i8, hipStream_t st) {
  if (N <= 0 || D <= 0 || H <= 0 || W <= 0 || D2 <= 0 || H2 <= 0 || W2o <= 0 || (J != 2 && J != 4)) return -2;
  if (2 * (D2 - 1) >= D || 2 * (H2 - 1) >= H || 2 * (W2o - 1) >= W) return -3;   // every position reads x
  if (W2o + J - 1 > 64) return -2;               // one 64-lane row of packed positions per (n, d, h)
  const long long rows = (long long)N * D2 * H2;
  if (i8)
    hipLaunchKernelGGL(s2d_tap_f8_kernel<true>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, (const bf16*)x,
                       (unsigned char*)y, N, D, H, W, D2, H2, W2o, J, inv_scale);
  else
    hipLaunchKernelGGL(s2d_tap_f8_kernel<false>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, (const bf16*)x,
                       (unsigned char*)y, N, D, H, W, D2, H2, W2o, J, inv_scale);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) on one wave: lane l supplies the 32 A
// bytes a[l][0..31], the 32 B bytes b[l][0..31], the scale dwords sa[l] / sb[l] (opsel 0: low
// byte) and gets its 4 accumulator values d[l][0..3] -- the numerics test pins the operand
// K-layout and the block-scale lane mapping against an fp32 emulation (tests/test_fp8_block_gpu.py)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void mfma_scale_probe_kernel(const unsigned char* __restrict__ a,
                                                              const unsigned char* __restrict__ b,
                                                              const int* __restrict__ sa, const int* __restrict__ sb,
                                                              float* __restrict__ d) {
  const int l = threadIdx.x;
  i32x8 va, vb;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    va[j] = *(const int*)(a + l * 32 + 4 * j);
    vb[j] = *(const int*)(b + l * 32 + 4 * j);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(va, vb, acc, 0, 0, 0, sa[l], 0, sb[l]);
#pragma unroll
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

extern "C" int fn_mfma_scale_probe(const void* a, const void* b, const int* sa, const int* sb, float* d,
                                   hipStream_t st) {
  hipLaunchKernelGGL(mfma_scale_probe_kernel, dim3(1), dim3(64), 0, st, (const unsigned char*)a,
                     (const unsigned char*)b, sa, sb, d);
  FN_CHECK_LAUNCH();
  return 0;
}
