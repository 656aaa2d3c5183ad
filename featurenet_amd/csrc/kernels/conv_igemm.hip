// Implicit-GEMM convolution (1-D/2-D/3-D, channels-last) on CDNA4 MFMA.
//
// One kernel family covers the three products a conv layer needs:
//   fwd  : y[m][co]  = sum_k  A[m][k] * W[co][k]      A = im2col(x)   (gathered)
//   dgrad: dx[m][ci] = sum_k' A'[m][k'] * WT[ci][k']  A' = "im2col" of dy with
//          negated tap offsets (stride-1 transposed conv; stride-2 layers are
//          handled by the caller through zero insertion of dy)
//   wgrad: dW[co][k] = sum_m dy[m][co] * A[m][k]     (split over m, fixed-order partial sums)
//
// Nothing is materialised: the gather is driven by a per-layer tap table
// (built once on the host and cached) whose entries hold the element offset of
// a k-chunk relative to a row's base plus the tap displacement for the
// bounds test.  For C % 8 == 0 a table entry covers 8 consecutive channels of
// one tap, so one 16-byte load feeds one 8-element MFMA fragment slice; for
// C < 8 (first layers: FeatureNet-3D's 1-channel voxels, RGB images) the
// (kw, c) run of a (kd, kh) kernel row is contiguous and one unaligned 16-byte
// load covers 8 (kw, c) pairs ("packed-W").
//
// gfx950 specifics:
//   * mfma_f32_16x16x32_bf16, 64-lane waves, 256-thread workgroups;
//   * forward/dgrad: BM=256 rows x BN output channels x BK=64.  ONE LDS stage
//     (40 KB at BN=64) so 4 workgroups (16 waves) fit a CU; the next stage's
//     gathers are issued into registers BEFORE the MFMAs of the current stage
//     and written after the barrier (issue-early / write-late), and the
//     uniform tap-table entries of the stage after that are prefetched into
//     SGPRs, so no load sits behind another load on the critical path.
//     XOR swizzle (chunk ^= row & 7) makes the 16-lane ds_read_b128 groups
//     conflict-free on the 128-B rows;
//   * every gather is branchless (clamped address + select): hipcc otherwise
//     wraps each conditional load in exec-mask branches with per-load waits;
//   * wgrad: the reduction runs over m, the slow axis of both operands in
//     memory, so operands are staged row-major and read with
//     ds_read_b64_tr_b16 (hardware transpose); rows are padded to 32 mod 256 B
//     and the MFMA k-order is permuted (same permutation on both operands) so
//     every transposed read is bank-conflict-free.  A thread's k-columns are
//     fixed for the whole kernel, so its tap-table entries load once;
//   * XCD-aware block remap so neighbouring tiles (which share input halos /
//     the same rows of x) run on the same XCD's L2.
#include "common.h"
#include "pack_w.h"

struct GatherGeom {
  int RD, RH, RW;          // row decode dims: m -> (n, r1, r2, r3)
  int md, mh, mw;          // base coord = r * mul + add
  int ad, ah, aw;
  int SD, SH, SW, SC;      // gathered source tensor dims (channels-last)
  int kwc;                 // packed-W mode: KW*C valid elements per (kd, kh) row
};

// gather modes
#define GM_SCALAR 0   // one table entry per k element (any C)
#define GM_VEC 1      // C % 8 == 0: one entry per 8 channels of one tap, 16-B load
#define GM_PACKW 2    // C < 8, W-dilation 1: (kw, c) run of a (kd, kh) row contiguous

struct RowBase {
  long long base;   // element offset of (n, bd, bh, bw, 0); may be "outside"
  int bd, bh, bw;
  bool valid;
};

__device__ __forceinline__ RowBase make_row(long long n, int c1, int c2, int c3, bool valid, const GatherGeom& g) {
  RowBase r;
  r.valid = valid;
  r.bd = c1 * g.md + g.ad;
  r.bh = c2 * g.mh + g.ah;
  r.bw = c3 * g.mw + g.aw;
  r.base = (((n * g.SD + r.bd) * g.SH + r.bh) * (long long)g.SW + r.bw) * g.SC;
  return r;
}

__device__ __forceinline__ RowBase decode_row(long long m, long long M, const GatherGeom& g) {
  const bool valid = m < M;
  long long mm = valid ? m : 0;
  const int c3 = (int)(mm % g.RW); mm /= g.RW;
  const int c2 = (int)(mm % g.RH); mm /= g.RH;
  const int c1 = (int)(mm % g.RD);
  return make_row(mm / g.RD, c1, c2, c3, valid, g);
}

__device__ __forceinline__ bool tap_ok(const RowBase& r, const int4& e, const GatherGeom& g) {
  return r.valid && (unsigned)(r.bd + e.y) < (unsigned)g.SD && (unsigned)(r.bh + e.z) < (unsigned)g.SH &&
         (unsigned)(r.bw + e.w) < (unsigned)g.SW;
}

typedef uint4 uint4_u2 __attribute__((aligned(2)));

// 8 consecutive k of one row.  VEC / PACKW take the chunk's (prefetched) table
// entry `e`; SCALAR reads its 8 per-element entries itself.  Loads are issued
// unconditionally from a clamped address and masked with a select.
template <int GM>
__device__ __forceinline__ uint4 gather8(const bf16* __restrict__ src, const int4* __restrict__ tab, const int4& e,
                                         const RowBase& r, int k0, int Kdim, const GatherGeom& g) {
  const uint4 zero = make_uint4(0, 0, 0, 0);
  if constexpr (GM == GM_VEC) {
    const bool ok = k0 < Kdim && tap_ok(r, e, g);
    const uint4 v = *(const uint4*)(src + (ok ? r.base + e.x : 0));
    return ok ? v : zero;
  } else if constexpr (GM == GM_PACKW) {
    // entry: {row offset + p0, (zd<<16)|zh, (kw_lo<<16)|kw_hi, p0}
    const int zd = e.y >> 16, zh = e.y & 0xffff;
    const int lo = e.z >> 16, hi = e.z & 0xffff;
    const bool rowok = k0 < Kdim && r.valid && (unsigned)(r.bd + zd) < (unsigned)g.SD &&
                       (unsigned)(r.bh + zh) < (unsigned)g.SH;
    const bool fast = rowok && r.bw + lo >= 0 && r.bw + hi < g.SW;
    const uint4 vv = *(const uint4_u2*)(src + (fast ? r.base + e.x : 0));
    const unsigned fm = fast ? 0xffffffffu : 0u;
    unsigned w0 = vv.x & fm, w1 = vv.y & fm, w2 = vv.z & fm, w3 = vv.w & fm;
    if (rowok && !fast) {   // row touches the W border: per-element (rare lanes)
      const unsigned short* s16 = reinterpret_cast<const unsigned short*>(src);
      const long long rowb = r.base + e.x - e.w;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int pp = e.w + j;
        const int kw = pp / g.SC;
        const bool okj = pp < g.kwc && (unsigned)(r.bw + kw) < (unsigned)g.SW;
        const unsigned x = (okj ? (unsigned)s16[okj ? rowb + pp : 0] : 0u) << (16 * (j & 1));
        if (j < 2) w0 |= x; else if (j < 4) w1 |= x; else if (j < 6) w2 |= x; else w3 |= x;
      }
    }
    (void)zero;
    return make_uint4(w0, w1, w2, w3);
  } else {
    Pack8 p;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j;
      const int4 ee = tab[k < Kdim ? k : 0];
      const bool ok = k < Kdim && tap_ok(r, ee, g);
      const bf16 x = src[ok ? r.base + ee.x : 0];
      p.e[j] = ok ? x : (bf16)0.f;
    }
    return p.u;
  }
}

template <int GM>
__device__ __forceinline__ int4 entry_for(const int4* __restrict__ tab, int k0, int Kdim) {
  if constexpr (GM == GM_SCALAR) return make_int4(0, 0, 0, 0);
  const int nchunk = (Kdim + 7) >> 3;
  const int kc = k0 >> 3;
  return tab[kc < nchunk ? kc : nchunk - 1];
}

// ---------------------------------------------------------------------------
// Forward / dgrad kernel
// ---------------------------------------------------------------------------
#define FWD_BM 256
#define FWD_BK 64

// SPLIT (split-K, ACT_NONE / no bias / no stats): workgroup z takes k-stages [z * spz, (z+1) * spz)
// and writes its fp32 partial tile to part[z][M][Ncol] straight from the accumulators; the slices
// are added in slice order by dense_fwd_reduce_kernel (+ bias, activation, bf16).  For the small-M,
// deep-K layers of NAS candidates (the dgrad of a 5x5x16 -> 120 LeNet conv: 7 row blocks for a
// 3000-deep reduction ran 67 us on 7 CUs)
template <int BN, int GM, int ACT, bool HAS_BIAS, bool STATS, bool SPLIT = false>
__global__ __launch_bounds__(256, (BN >= 64 || GM != GM_VEC ? 3 : 4)) void igemm_fwd_kernel(
    const bf16* __restrict__ src, const bf16* __restrict__ wt, const float* __restrict__ bias,
    bf16* __restrict__ out, float* __restrict__ stats, const int4* __restrict__ tab, GatherGeom g,
    long long M, int Ncol, int Kdim, int ldw, float* __restrict__ part = nullptr, int spz = 0) {
  static_assert(!SPLIT || (ACT == ACT_NONE && !HAS_BIAS && !STATS), "split-K: the reduce applies bias / act");
  constexpr int A_STAGE = FWD_BM * FWD_BK;      // elements
  constexpr int B_STAGE = BN * FWD_BK;
  constexpr int LDO = BN + 8;                   // epilogue staging row (16-B aligned)
  constexpr int NT = BN / 16;                   // n-tiles per wave
  constexpr int B_CHUNKS = BN * (FWD_BK / 8);   // 16-B chunks per B stage
  constexpr int B_PER_T = (B_CHUNKS + 255) / 256;
  static_assert(FWD_BM * LDO + 16 * BN <= A_STAGE + B_STAGE, "epilogue staging + stats must fit the stage");
  __shared__ __attribute__((aligned(16))) bf16 smem[A_STAGE + B_STAGE];
  bf16* As = smem;
  bf16* Bs = smem + A_STAGE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nmb = gridDim.x;
  const int mb = xcd_remap(blockIdx.x, nmb);
  const long long m0 = (long long)mb * FWD_BM;
  const int n0 = blockIdx.y * BN;

  const RowBase rb = decode_row(m0 + tid, M, g);

  uint4 ra[8];
  uint4 rbv[B_PER_T];
  int4 te[8];   // uniform tap-table entries of the next stage to gather

  auto fetch_entries = [&](int kt) {
#pragma unroll
    for (int c = 0; c < 8; ++c) te[c] = entry_for<GM>(tab, kt * FWD_BK + c * 8, Kdim);
  };
  auto load_stage = [&](int kt) {
    const int kbase = kt * FWD_BK;
#pragma unroll
    for (int c = 0; c < 8; ++c) ra[c] = gather8<GM>(src, tab, te[c], rb, kbase + c * 8, Kdim, g);
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int idx = tid + i * 256;
      const int r = (idx >> 3) < BN ? (idx >> 3) : BN - 1;
      const int k = kbase + (idx & 7) * 8;
      const bool ok = idx < B_CHUNKS && n0 + r < Ncol && k < ldw;
      const uint4 v = *(const uint4*)(wt + (ok ? (long long)(n0 + r) * ldw + k : 0));
      rbv[i] = ok ? v : make_uint4(0, 0, 0, 0);
    }
  };
  auto write_stage = [&]() {
    bf16* a = As + tid * FWD_BK;
#pragma unroll
    for (int c = 0; c < 8; ++c) *(uint4*)(a + ((c ^ (tid & 7)) << 3)) = ra[c];
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int idx = tid + i * 256;
      if (idx < B_CHUNKS) {
        const int r = idx >> 3, c = idx & 7;
        *(uint4*)(Bs + r * FWD_BK + ((c ^ (r & 7)) << 3)) = rbv[i];
      }
    }
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk_all = (Kdim + FWD_BK - 1) / FWD_BK;
  const int kt0 = SPLIT ? (int)blockIdx.z * spz : 0;
  const int nk = SPLIT ? min(nk_all, kt0 + spz) : nk_all;   // (stage index range [kt0, nk))
  fetch_entries(kt0);
  load_stage(kt0);
  if (nk > kt0 + 1) fetch_entries(kt0 + 1);
  write_stage();
  __syncthreads();

  const int lr = lane & 15;     // row inside a 16-row fragment
  const int lg = lane >> 4;     // k-group (8 elements each)
  for (int kt = kt0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      load_stage(kt + 1);                 // gathers in flight during the MFMAs below
      if (kt + 2 < nk) fetch_entries(kt + 2);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + lg;
      bf16x8 fa[4], fb[NT];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int row = wave * 64 + mt * 16 + lr;
        fa[mt] = *(const bf16x8*)(As + row * FWD_BK + ((ch ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int row = nt * 16 + lr;
        fb[nt] = *(const bf16x8*)(Bs + row * FWD_BK + ((ch ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
    }
    __syncthreads();                       // every wave done reading the stage
    if (more) {
      write_stage();
      __syncthreads();
    }
  }

  if constexpr (SPLIT) {                        // fp32 partial tile, straight from the accumulators
    float* ps = part + (long long)blockIdx.z * M * Ncol;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int col = n0 + nt * 16 + lr;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long m = m0 + wave * 64 + mt * 16 + lg * 4 + r;
          if (m < M && col < Ncol) ps[m * Ncol + col] = acc[mt][nt][r];
        }
    }
    return;
  }
  // ---- epilogue: bias + activation, bf16 staging in LDS, BN partial stats ----
  bf16* Os = smem;  // reuse the A stage (all waves passed the final barrier)
  float csum[NT], csq[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) { csum[nt] = 0.f; csq[nt] = 0.f; }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = nt * 16 + lr;
    const bool cv = (n0 + col) < Ncol;
    float bv = 0.f;
    if constexpr (HAS_BIAS) bv = cv ? bias[n0 + col] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 64 + mt * 16 + lg * 4 + r;
        float v = acc[mt][nt][r] + bv;
        v = act_fwd(v, ACT);
        const bf16 bvv = f2bf(v);
        Os[row * LDO + col] = bvv;
        if constexpr (STATS) {
          const bool rv = cv && (m0 + row) < M;
          const float f = rv ? bf2f(bvv) : 0.f;
          csum[nt] += f;
          csq[nt] += f * f;
        }
      }
    }
  }
  if constexpr (STATS) {
    // cross-wave reduction scratch right after the staged output tile
    float* red = reinterpret_cast<float*>(smem + FWD_BM * LDO);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float s = csum[nt], q = csq[nt];
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (lg == 0) { red[(wave * 2 + 0) * BN + nt * 16 + lr] = s; red[(wave * 2 + 1) * BN + nt * 16 + lr] = q; }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < Ncol) {
      const float s = red[0 * BN + tid] + red[2 * BN + tid] + red[4 * BN + tid] + red[6 * BN + tid];
      const float q = red[1 * BN + tid] + red[3 * BN + tid] + red[5 * BN + tid] + red[7 * BN + tid];
      stats[(long long)mb * 2 * Ncol + n0 + tid] = s;
      stats[(long long)mb * 2 * Ncol + Ncol + n0 + tid] = q;
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  const bool vec_out = (Ncol % 8) == 0;
#pragma unroll
  for (int i = 0; i < CPR; ++i) {
    const int idx = tid + i * 256;
    const int row = idx / CPR, ch = idx % CPR;
    const long long m = m0 + row;
    const int col = n0 + ch * 8;
    if (m < M) {
      if (vec_out && col + 8 <= Ncol) {
        *(uint4*)(out + m * Ncol + col) = *(const uint4*)(Os + row * LDO + ch * 8);
      } else {
        for (int j = 0; j < 8; ++j)
          if (col + j < Ncol) out[m * Ncol + col + j] = Os[row * LDO + ch * 8 + j];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight-gradient kernel
// ---------------------------------------------------------------------------
#define WG_BR 64     // m-rows per stage (two MFMA k-steps)
#define WG_BK 256    // k-columns per block (64 per wave)
#define WG_LDX (WG_BK + 16)

template <int BCO>
struct WgLds {
  static constexpr int LDY = (BCO == 16) ? 48 : BCO + 16;
};

// k-order permutation shared by both operands: MFMA k-index (group G, elem j)
// of k-step s reads stage row 32s + (j<4 ? 4G+j : 16+4G+j-4).
__device__ __forceinline__ bf16x8 tr_frag(const bf16* base, int ld, int col0, int lane) {
  const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  typedef short s4 __attribute__((ext_vector_type(4)));
  const bf16* p0 = base + (4 * G + q) * ld + col0 + 4 * p;
  const bf16* p1 = base + (16 + 4 * G + q) * ld + col0 + 4 * p;
  s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p0));
  s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p1));
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int BCO, int GM, bool VECN>
__global__ __launch_bounds__(256, 2) void igemm_wgrad_kernel(
    const bf16* __restrict__ dy, const bf16* __restrict__ src, float* __restrict__ dw,
    const int4* __restrict__ tab, GatherGeom g, long long M, int Cout, int Kdim, long long rows_per_split,
    int gx, int gy, int ccrop, int cpad, const bf16* __restrict__ ya, int act, float* __restrict__ db, int kout) {
  constexpr int LDY = WgLds<BCO>::LDY;
  constexpr int X_STAGE = WG_BR * WG_LDX;
  constexpr int Y_STAGE = WG_BR * LDY;
  constexpr int MT = BCO / 16;
  constexpr int Y_CHUNKS = WG_BR * (BCO / 8);
  constexpr int Y_PER_T = (Y_CHUNKS + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[X_STAGE + Y_STAGE];
  bf16* Xs = smem;
  bf16* Ys = smem + X_STAGE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware remap: consecutive logical blocks (same split, neighbouring
  // column tiles -> same rows of x and dy) share an XCD.
  const int nwg = gx * gy * gridDim.z;
  const int lin = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), nwg);
  const int bx = lin % gx, by = (lin / gx) % gy, bz = lin / (gx * gy);
  const int kc0 = bx * WG_BK;
  const int co0 = by * BCO;
  const long long mbeg = (long long)bz * rows_per_split;
  long long mend = mbeg + rows_per_split;
  if (mend > M) mend = M;

  // X-tile loader: thread -> (row xr, 8 consecutive 8-col chunks of its wave)
  const int xr = tid & 63;
  const int xc = __builtin_amdgcn_readfirstlane(wave) * 8;
  int4 te[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) te[i] = entry_for<GM>(tab, kc0 + (xc + i) * 8, Kdim);

  // incremental row decode for row mbeg + xr (advances by WG_BR per stage)
  long long mcur = mbeg + xr;
  int c3, c2, c1;
  long long nn;
  {
    long long mm = mcur < M ? mcur : 0;
    c3 = (int)(mm % g.RW); mm /= g.RW;
    c2 = (int)(mm % g.RH); mm /= g.RH;
    c1 = (int)(mm % g.RD); nn = mm / g.RD;
  }
  auto advance_row = [&]() {
    mcur += WG_BR;
    c3 += WG_BR;
    while (c3 >= g.RW) {
      c3 -= g.RW;
      if (++c2 >= g.RH) {
        c2 = 0;
        if (++c1 >= g.RD) { c1 = 0; ++nn; }
      }
    }
  };

  uint4 rx[8];
  uint4 ry[Y_PER_T];
  auto load_stage = [&](long long ms) {
    const RowBase r = make_row(nn, c1, c2, c3, mcur < mend, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) rx[i] = gather8<GM>(src, tab, te[i], r, kc0 + (xc + i) * 8, Kdim, g);
#pragma unroll
    for (int i = 0; i < Y_PER_T; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / (BCO / 8), ch = idx % (BCO / 8);
      const long long m = ms + row;
      const int co = co0 + ch * 8;
      const bool ok = idx < Y_CHUNKS && m < mend;
      if constexpr (VECN) {
        const bool okc = ok && co < Cout;
        const uint4 v = *(const uint4*)(dy + (okc ? m * Cout + co : 0));
        ry[i] = okc ? v : make_uint4(0, 0, 0, 0);
        if (ya && okc) {                         // dy * act'(y): the activation backward on load
          Pack8 p, q;
          p.u = ry[i];
          q.u = *(const uint4*)(ya + m * Cout + co);
#pragma unroll
          for (int j = 0; j < 8; ++j) p.e[j] = f2bf(bf2f(p.e[j]) * act_bwd_from_out(bf2f(q.e[j]), act));
          ry[i] = p.u;
        }
      } else {
        Pack8 p;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool okj = ok && co + j < Cout;
          const bf16 x = dy[okj ? m * Cout + co + j : 0];
          p.e[j] = okj ? x : (bf16)0.f;
          if (ya && okj) p.e[j] = f2bf(bf2f(p.e[j]) * act_bwd_from_out(bf2f(ya[m * Cout + co + j]), act));
        }
        ry[i] = p.u;
      }
    }
    advance_row();
  };
  auto write_stage = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) *(uint4*)(Xs + xr * WG_LDX + (xc + i) * 8) = rx[i];
#pragma unroll
    for (int i = 0; i < Y_PER_T; ++i) {
      const int idx = tid + i * 256;
      if (idx < Y_CHUNKS) {
        const int row = idx / (BCO / 8), ch = idx % (BCO / 8);
        *(uint4*)(Ys + row * LDY + ch * 8) = ry[i];
      }
    }
  };

  f32x4 acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // db (optional): the bias gradient = column sums of (activated) dy, taken from the LDS dy tile by
  // the first column-tile's workgroups (one thread per output channel), one atomic per channel
  // and workgroup into the zeroed db -- no separate column-sum pass
  const bool dsum = db != nullptr && bx == 0 && tid < BCO;
  float dbs = 0.f;
  const long long nst = (mend - mbeg + WG_BR - 1) / WG_BR;
  if (nst > 0) {
    load_stage(mbeg);
    write_stage();
  }
  __syncthreads();
  for (long long s = 0; s < nst; ++s) {
    const bool more = s + 1 < nst;
    if (dsum)
      for (int row = 0; row < WG_BR; ++row) dbs += bf2f(Ys[row * LDY + tid]);
    if (more) load_stage(mbeg + (s + 1) * WG_BR);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[MT], fb[4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) fa[mt] = tr_frag(Ys + ks * 32 * LDY, LDY, mt * 16, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) fb[nt] = tr_frag(Xs + ks * 32 * WG_LDX, WG_LDX, wave * 64 + nt * 16, lane);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
    }
    __syncthreads();
    if (more) {
      write_stage();
      __syncthreads();
    }
  }

  // D[row=co][col=k]: lane holds rows (lane>>4)*4+r, col lane&15.
  // Split-m partial sums are stored into this split's partial rows (dw / db point at the
  // partial slabs [splits][kout][ldo] / [splits][kout]); fn_part_reduce adds the splits in a
  // fixed order (bitwise repeatable; through round 4 these were float atomics into dW).
  const long long ldo = ccrop > 0 ? (long long)(Kdim / cpad) * ccrop : Kdim;
  dw += (long long)bz * kout * ldo;
  if (dsum && co0 + tid < kout) db[(long long)bz * kout + co0 + tid] = dbs;
  // ccrop > 0: k = t*cpad + c lands at dw[co][t*ccrop + c] of the real weight, columns
  // c >= ccrop dropped -- the zero channels of a channel-padded input (cpad = its channels,
  // ccrop = the real ones) or the row padding of the packed-W layout (cpad = R, ccrop = KW*C):
  // straight into the parameter's zeroed flat gradient (no padded dW buffer, fill or crop copy)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int k = kc0 + wave * 64 + nt * 16 + (lane & 15);
      long long kdst = k;
      bool kok = k < Kdim;
      if (ccrop > 0) {
        const int t = k / cpad, c = k - t * cpad;
        kok = kok && c < ccrop;
        kdst = (long long)t * ccrop + c;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + mt * 16 + (lane >> 4) * 4 + r;
        if (co < kout && kok) dw[(long long)co * ldo + kdst] = acc[mt][nt][r];
      }
    }
}

// ---------------------------------------------------------------------------
// Host launchers (C ABI, used by bind.cpp)
// ---------------------------------------------------------------------------
static GatherGeom parse_geom(const int* g14) {
  GatherGeom g;
  g.RD = g14[0]; g.RH = g14[1]; g.RW = g14[2];
  g.md = g14[3]; g.mh = g14[4]; g.mw = g14[5];
  g.ad = g14[6]; g.ah = g14[7]; g.aw = g14[8];
  g.SD = g14[9]; g.SH = g14[10]; g.SW = g14[11]; g.SC = g14[12]; g.kwc = g14[13];
  return g;
}

template <int BN, int GMV>
static void launch_fwd_bn(dim3 grid, hipStream_t st, const bf16* src, const bf16* wt, const float* bias, bf16* out,
                          float* stats, const int4* tab, const GatherGeom& g, long long M, int N, int K, int ldw,
                          int act) {
#define FWD_ARGS src, wt, bias, out, stats, tab, g, M, N, K, ldw
#define FWD_CASE(ACTV, HB, ST) \
  hipLaunchKernelGGL((igemm_fwd_kernel<BN, GMV, ACTV, HB, ST>), grid, dim3(256), 0, st, FWD_ARGS)
  const bool hb = bias != nullptr, stt = stats != nullptr;
  if (act == ACT_NONE) {
    if (hb) { if (stt) FWD_CASE(ACT_NONE, true, true); else FWD_CASE(ACT_NONE, true, false); }
    else { if (stt) FWD_CASE(ACT_NONE, false, true); else FWD_CASE(ACT_NONE, false, false); }
  } else if (act == ACT_RELU) {
    if (hb) FWD_CASE(ACT_RELU, true, false); else FWD_CASE(ACT_RELU, false, false);
  } else if (act == ACT_TANH) {
    if (hb) FWD_CASE(ACT_TANH, true, false); else FWD_CASE(ACT_TANH, false, false);
  } else {
    if (hb) FWD_CASE(ACT_SIGMOID, true, false); else FWD_CASE(ACT_SIGMOID, false, false);
  }
#undef FWD_CASE
#undef FWD_ARGS
}

extern "C" int fn_dense_fwd_reduce(const float* part, const float* bias, void* out, int M, int N, int S, int act,
                                   int out_fp32, hipStream_t st);

// k-slices of the split-K form for (M, Ncol, Kdim): enough workgroups for the 256 CUs, >= 4
// k-stages per slice, 1 = no split (the caller sizes part = splits x M x Ncol floats)
extern "C" int fn_igemm_fwd_splits(long long M, int Ncol, int Kdim) {
  const int BN = Ncol <= 16 ? 16 : (Ncol <= 32 ? 32 : 64);
  const long long tiles = (M + FWD_BM - 1) / FWD_BM * ((Ncol + BN - 1) / BN);
  const int nk = (Kdim + FWD_BK - 1) / FWD_BK;
  if (tiles >= 128 || nk < 8) return 1;
  int s = (int)((256 + tiles - 1) / tiles);
  if (s > nk / 4) s = nk / 4;
  return s < 2 ? 1 : s;
}

extern "C" int fn_igemm_fwd(const void* src, const void* wt, const float* bias, void* out, float* stats,
                            const int* tab, const int* geom14, long long M, int Ncol, int Kdim, int ldw, int gm,
                            int act, hipStream_t st, float* part, int splits) {
  const GatherGeom g = parse_geom(geom14);
  if (stats && act != ACT_NONE) return -1;  // stats are taken on the pre-BN output
  if (ldw % 8 != 0) return -3;
  const int BN = Ncol <= 16 ? 16 : (Ncol <= 32 ? 32 : 64);
  const long long mblocks = (M + FWD_BM - 1) / FWD_BM;
  dim3 grid((unsigned)mblocks, (Ncol + BN - 1) / BN);
  const bf16* s = (const bf16*)src;
  const bf16* w = (const bf16*)wt;
  bf16* o = (bf16*)out;
  const int4* t = (const int4*)tab;
  if (splits > 1 && !stats) {
    if (!part) return -6;
    const int nk = (Kdim + FWD_BK - 1) / FWD_BK;
    const int spz = (nk + splits - 1) / splits;
    const int sr = (nk + spz - 1) / spz;        // slices actually covering the k-stages
    grid.z = (unsigned)sr;
#define SPLIT_CASE(BNV, GMV)                                                                              \
  hipLaunchKernelGGL((igemm_fwd_kernel<BNV, GMV, ACT_NONE, false, false, true>), grid, dim3(256), 0, st, s, w, \
                     nullptr, o, nullptr, t, g, M, Ncol, Kdim, ldw, part, spz)
#define SPLIT_GM(GMV)                                                                                     \
  do {                                                                                                  \
    if (BN == 16) SPLIT_CASE(16, GMV); else if (BN == 32) SPLIT_CASE(32, GMV); else SPLIT_CASE(64, GMV);   \
  } while (0)
    if (gm == GM_VEC) SPLIT_GM(GM_VEC);
    else if (gm == GM_PACKW) SPLIT_GM(GM_PACKW);
    else SPLIT_GM(GM_SCALAR);
#undef SPLIT_GM
#undef SPLIT_CASE
    FN_CHECK_LAUNCH();
    return fn_dense_fwd_reduce(part, bias, out, (int)M, Ncol, sr, act, 0, st);
  }
#define FWD_GM(GMV)                                                                                      \
  do {                                                                                                   \
    if (BN == 16) launch_fwd_bn<16, GMV>(grid, st, s, w, bias, o, stats, t, g, M, Ncol, Kdim, ldw, act);      \
    else if (BN == 32) launch_fwd_bn<32, GMV>(grid, st, s, w, bias, o, stats, t, g, M, Ncol, Kdim, ldw, act); \
    else launch_fwd_bn<64, GMV>(grid, st, s, w, bias, o, stats, t, g, M, Ncol, Kdim, ldw, act);              \
  } while (0)
  if (gm == GM_VEC) FWD_GM(GM_VEC);
  else if (gm == GM_PACKW) FWD_GM(GM_PACKW);
  else FWD_GM(GM_SCALAR);
#undef FWD_GM
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_igemm_fwd_mblocks(long long M) { return (int)((M + FWD_BM - 1) / FWD_BM); }

// fp32 floats of the partial slab fn_igemm_wgrad needs: splits x kout x (columns of dw) (+ splits x
// kout for the bias gradient)
extern "C" long long fn_igemm_wgrad_part(int Cout, int Kdim, int splits, int ccrop, int cpad, int kout, int with_db) {
  if (kout <= 0) kout = Cout;
  const long long ldo = ccrop > 0 ? (long long)(Kdim / cpad) * ccrop : Kdim;
  return (long long)splits * kout * (ldo + (with_db ? 1 : 0));
}

// ccrop > 0: dw is the real [Cout][Kdim / cpad][ccrop] weight gradient; column t*cpad + c of the
// gather layout (c < ccrop) maps to t*ccrop + c (channel-padded inputs; the packed-W rows)
// ya / act (optional): dy is the gradient of the activation output ya (the activation backward
// is applied as dy is loaded); db (optional): receives (+=) the bias gradient (column sums of
// the activated dy).  kout (0 = Cout): only output channels co < kout are written (dy channel-
// padded to Cout for 16-B loads, dW / db of the real kout channels).  dw and db are accumulated
// into (+=) from the split partials in `part` (fn_igemm_wgrad_part floats), in a fixed order.
extern "C" int fn_igemm_wgrad(const void* dy, const void* src, float* dw, const int* tab, const int* geom14,
                              long long M, int Cout, int Kdim, int splits, int gm, hipStream_t st, int ccrop,
                              int cpad, const void* ya, int act, float* db, int kout, float* part) {
  if (kout <= 0) kout = Cout;
  if (kout > Cout) return -2;
  const GatherGeom g = parse_geom(geom14);
  if (ccrop > 0 && (cpad < ccrop || Kdim % cpad)) return -2;
  if (!part || splits < 1) return -6;
  const long long ldo = ccrop > 0 ? (long long)(Kdim / cpad) * ccrop : Kdim;
  float* pdw = part;
  float* pdb = db ? part + (long long)splits * kout * ldo : nullptr;
  const int BCO = Cout <= 16 ? 16 : (Cout <= 32 ? 32 : 64);
  const long long rps = ((M + splits - 1) / splits + WG_BR - 1) / WG_BR * WG_BR;
  const int gx = (Kdim + WG_BK - 1) / WG_BK, gy = (Cout + BCO - 1) / BCO;
  dim3 grid(gx, gy, splits);
  const bool vecn = (Cout % 8) == 0;
  const bf16* d = (const bf16*)dy;
  const bf16* s = (const bf16*)src;
  const int4* t = (const int4*)tab;
#define WG_CASE(B, V, VN) \
  hipLaunchKernelGGL((igemm_wgrad_kernel<B, V, VN>), grid, dim3(256), 0, st, d, s, pdw, t, g, M, Cout, Kdim, rps, gx, gy, \
                     ccrop, cpad, (const bf16*)ya, act, pdb, kout)
#define WG_GM(GMV)                                                                        \
  do {                                                                                    \
    if (vecn) {                                                                           \
      if (BCO == 16) WG_CASE(16, GMV, true); else if (BCO == 32) WG_CASE(32, GMV, true); \
      else WG_CASE(64, GMV, true);                                                        \
    } else {                                                                              \
      if (BCO == 16) WG_CASE(16, GMV, false); else if (BCO == 32) WG_CASE(32, GMV, false); \
      else WG_CASE(64, GMV, false);                                                       \
    }                                                                                     \
  } while (0)
  if (gm == GM_VEC) WG_GM(GM_VEC);
  else if (gm == GM_PACKW) WG_GM(GM_PACKW);
  else WG_GM(GM_SCALAR);
#undef WG_GM
#undef WG_CASE
  FN_CHECK_LAUNCH();
  int rc = fn_part_reduce2(pdw, dw, (long long)kout * ldo, db ? pdb : nullptr, db, db ? kout : 0, splits, 1, st);
  return rc;
}

// ---------------------------------------------------------------------------
// B-operand packing for the gather kernels: fp32 weight -> bf16 rows in one launch
// (cast + transpose + zero padding of rows / channels / the row stride).
// ---------------------------------------------------------------------------
// w: fp32 [K0][T][C0] (the parameter, possibly fewer output / input channels than the
// conv runs with).  out: bf16 [rows][ld] with
//   mode 0 (forward): rows = K, element (k, t*C + c) = w[k][t][c]; kdim = T*C
//   mode 1 (dgrad):   rows = C, element (c, t*K + k) = w[k][t][c] (the dgrad gather table
//                     walks the taps mirrored itself)
//   mode 2 (packed-W forward, C < 8): rows = K, row k = [KD*KH][R] with R >= KW*C, element
//                     (k, r*R + p) = w[k][r*KW + p / C][p % C] for p < KW*C
// and zeros for k >= K0, c >= C0 and the padding columns.
__global__ __launch_bounds__(256) void igemm_pack_w_kernel(const float* __restrict__ w, bf16* __restrict__ out,
                                                           int K0, int C0, int K, int T, int C, int mode, int ld,
                                                           int KW, int R, long long total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  out[i] = f2bf(ig_pack_val(w, K0, C0, K, T, C, mode, ld, KW, R, i));
}

// Many weight packs in one launch (a model's forward and dgrad B operands at the start of its
// forward, ops/conv.py pack_scope): thread i finds its job by a scan of the (<= 24) job starts
// -- the NAS candidate step ran one 3-5 us launch per conv per direction
// Every job starts on a 256-element boundary, so a workgroup lies in one job: the job search and
// the job's parameters are wave-uniform (scalar loads; a per-lane search over the by-value job
// table made the FeatureNet-3D pack launch as slow as the three it replaced)
__global__ __launch_bounds__(256) void pack_w_multi_kernel(const PackJobs js) {
  const long long b0 = (long long)blockIdx.x * 256;
  int k = 0;
  while (k + 1 < js.n && b0 >= js.j[k + 1].start) ++k;
  k = __builtin_amdgcn_readfirstlane(k);
  const PackJob& jb = js.j[k];
  const long long e = b0 - jb.start + threadIdx.x;
  if (e >= jb.count) return;
  const int* a = jb.a;
  if (jb.kind == 5) {                            // (tile stream: one uint4 per index)
    tile_pack_w_one(jb.w, reinterpret_cast<uint4*>(jb.out), a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], e);
    return;
  }
  const float v = jb.kind <= 2 ? ig_pack_val(jb.w, a[0], a[1], a[2], a[3], a[4], jb.kind, a[5], a[6], a[7], e)
                               : halo_pack_val(jb.w, a[0], a[1], a[2], a[3], a[4], a[5], a[6], jb.kind - 3, e);
  jb.out[e] = f2bf(v);
}

extern "C" int fn_igemm_pack_w(const float* w, void* out, int K0, int C0, int K, int T, int C, int mode, int ld, int KW,
                               int R, hipStream_t st) {
  if (K0 <= 0 || C0 <= 0 || K0 > K || C0 > C || T <= 0 || mode < 0 || mode > 2 || ld <= 0) return -2;
  const int rows = mode == 1 ? C : K;
  const long long need = mode == 0 ? (long long)T * C : (mode == 1 ? (long long)T * K : (long long)(T / KW) * R);
  if (ld < need || (mode == 2 && (KW <= 0 || T % KW || R < KW * C || ld != (T / KW) * R))) return -2;
  const long long total = (long long)rows * ld;
  hipLaunchKernelGGL(igemm_pack_w_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, (bf16*)out, K0, C0,
                     K, T, C, mode, ld, KW, R, total);
  FN_CHECK_LAUNCH();
  return 0;
}

// jobs: n rows of 12 int64 (w, out, kind, a[0..8]); the element counts follow from kind and a
// (checked as fn_igemm_pack_w / fn_halo_pack_w / fn_tile_pack_w check their arguments)
extern "C" int fn_pack_w_multi(const long long* jobs, int n, hipStream_t st) {
  if (n <= 0 || n > FN_PACK_MAXJ) return -2;
  PackJobs js{};
  long long start = 0;
  for (int k = 0; k < n; ++k) {
    const long long* r = jobs + 12 * k;
    PackJob& jb = js.j[k];
    jb.w = reinterpret_cast<const float*>(r[0]);
    jb.out = reinterpret_cast<bf16*>(r[1]);
    jb.kind = (int)r[2];
    for (int q = 0; q < 9; ++q) jb.a[q] = (int)r[3 + q];
    const int* a = jb.a;
    long long cnt;
    if (jb.kind <= 2) {
      const int K0 = a[0], C0 = a[1], K = a[2], T = a[3], C = a[4], mode = jb.kind, ld = a[5], KW = a[6], R = a[7];
      if (K0 <= 0 || C0 <= 0 || K0 > K || C0 > C || T <= 0 || ld <= 0) return -2;
      const long long need = mode == 0 ? (long long)T * C : (mode == 1 ? (long long)T * K : (long long)(T / KW) * R);
      if (ld < need || (mode == 2 && (KW <= 0 || T % KW || R < KW * C || ld != (T / KW) * R))) return -2;
      cnt = (long long)(mode == 1 ? C : K) * ld;
    } else if (jb.kind <= 4) {
      const int K0 = a[0], C0 = a[1], K = a[2], T = a[3], C = a[4], CS = a[5], Tp = a[6];
      const int Csrc = jb.kind == 3 ? C : K;
      if (K0 <= 0 || C0 <= 0 || K0 > K || C0 > C || CS <= 0 || Csrc % CS || T <= 0 || Tp < T) return -2;
      cnt = (long long)(jb.kind == 3 ? K : C) * Csrc * Tp;
    } else if (jb.kind == 5) {                   // (fn_tile_pack_w's checks)
      const int CS = a[3], nks = a[4], nct = a[5], nslice = a[6], nt = a[8];
      if (CS != 8 && CS != 16 && CS % 32 != 0) return -2;
      if ((nt != 2 && nt != 4 && nt != 32) || nct % (nt == 4 ? 4 : 2) || nks <= 0 || nslice <= 0) return -2;
      cnt = ((long long)nslice * nks + 4) * nct * 64;
    } else {
      return -2;
    }
    if (!jb.w || !jb.out) return -2;
    jb.start = start;
    jb.count = cnt;
    start += (cnt + 255) / 256 * 256;              // (workgroup-aligned job starts)
  }
  js.n = n;
  js.total = start;
  hipLaunchKernelGGL(pack_w_multi_kernel, dim3((unsigned)((start + 255) / 256)), dim3(256), 0, st, js);
  FN_CHECK_LAUNCH();
  return 0;
}
