// LDS-halo implicit-GEMM convolution for stride-1 3-D convs (CDNA4 MFMA).
//
// The gather-based igemm kernel (conv_igemm.hip) re-fetches the im2col row of
// every output position once per tap: for FeatureNet-3D's 5x5x5 / 4x4x4 /
// 3x3x3 stride-1 layers that is 27-125 reads of every input voxel, so those
// layers run L2-bandwidth-bound at 15-25 % of MFMA peak.  This kernel stages
// a 3-D input tile (the output tile plus its kernel halo) in LDS ONCE per
// 16-channel slice and builds every MFMA A-fragment straight from it:
//
//   output tile  TD x TH x TW   (<= 256 rows; TW = OW, or a W split for wide outputs)
//   LDS halo     (TD+KD-1) x (TH+KH-1) x (TW+KW-1) positions x CS channels
//   K loop       pass p over C/CS channel slices (CS = 16, or 8 for 8-channel
//                inputs), 32/CS taps per MFMA k-step (k = [tap][CS ch]),
//                weights streamed through a double-buffered 128-k LDS stage
//                (all stages resident for short-K 8-channel convs)
//
// so global/L2 traffic drops from ~taps x |x| to ~halo/tile x |x| and the
// kernel becomes MFMA/LDS-bound.  Used for forward (with fused bias/act or BN
// statistics epilogue) and for dgrad (dx = conv(dy, flip(W)^T), stride 1).
//
// A-fragment LDS reads: lane (row lr, k-group lg) reads 16 B at
// (hbase[row] + tapoff[tap(lg)]) * 32 B + (lg & 1) * 16 B.  Rows are
// consecutive halo positions, so a ds_read_b128 lane group {lr 0-3,12-15 @ lg,
// lr 4-11 @ lg^1} touches 16 distinct 16-B slots of a 256-B bank line.
#include "common.h"
#include "pack_w.h"

struct HaloGeom {
  int N, ID, IH, IW, C;    // gathered source (x for fwd, dy for dgrad), channels-last
  int OD, OH, OW;          // output dims
  int KD, KH, KW;          // kernel
  int pd, ph, pw;          // leading pads (stride 1)
  int TD, TH;              // output tile (rows = TD * TH * TW <= 256)
  int TW;                  // tile width in W (OW, or OW split into ceil(OW / TW) column tiles)
};

// tile index -> (n, td_i, th_i, tw_i); W tiles vary fastest, so consecutive tiles of a
// workgroup share halo rows
struct TileIdx { int n, td, th, tw; };
__device__ __forceinline__ TileIdx tile_idx(int tile, int tdn, int thn, int twn) {
  TileIdx t;
  t.tw = twn == 1 ? 0 : tile % twn;               // full-width tiles (the common case): no division
  const int r = twn == 1 ? tile : tile / twn;
  t.th = r % thn;
  t.td = (r / thn) % tdn;
  t.n = r / (thn * tdn);
  return t;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt) but NOT for outstanding global loads, unlike __syncthreads(), whose
// fence drains vmcnt -- the register prefetches of the next halo / weight stage
// stay in flight across the barrier (hipcc waits for them, counted, at first use).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#define H_BM 256
#define H_BK 64
#define H_BKS 128   // weight-stage depth of the forward halo kernel

// 16-B halo chunks per thread prefetched in registers (the rest of a larger
// halo is loaded synchronously at the job boundary); BN=64 keeps 64 VGPRs of
// accumulators, so it prefetches fewer.
#define H_HC(BN) ((BN) == 32 ? 2 : 0)
#define H_NTHR 512   // 8 waves: 4 row blocks x 2-way split of every weight stage's k-steps

// Persistent form: each workgroup owns a contiguous run of output tiles
// (adjacent tiles share halo rows -> same XCD L2) and walks the sequence of
// (tile, channel-slice) jobs.  The NEXT job's halo is loaded into registers
// while the current job computes (written to LDS at the job boundary), and
// weight stages are prefetched two stages ahead, so neither halo nor weight
// latency sits on the critical path.
// RES: every weight stage stays resident in LDS for the whole kernel (short-K convs
// such as the space-to-depth stem, K = 512): no per-stage weight loads or barriers,
// the k-loop of a job is pure LDS reads + MFMAs.
template <int BN, int ACT, bool HAS_BIAS, bool STATS, int CS, bool RES>
__global__ __launch_bounds__(H_NTHR, 4) void conv_halo_kernel(const bf16* __restrict__ src, const bf16* __restrict__ wt,
                                                           const float* __restrict__ bias, bf16* __restrict__ out,
                                                           float* __restrict__ stats, const int* __restrict__ toffs,
                                                           HaloGeom g, int Ncol, int region_bytes,
                                                           int* __restrict__ sched, int chunk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  // 8 waves = 4 row blocks x 2: BN=32 splits every stage's 4 k-steps between
  // the two waves of a row block (partials reduced per tile); BN=64 gives each
  // of them 32 of the 64 columns.  Either way a wave owns 64 rows x 32 cols.
  // CS = channels per halo slice: 16 (k-step = 2 taps x 16 ch) or 8 (k-step =
  // 4 taps x 8 ch, for 8-channel inputs such as the space-to-depth stem).
  constexpr bool KSPLIT = BN == 32;
  constexpr int NT = 2;
  constexpr int CPP = CS / 8;                    // 16-B chunks per halo position
  constexpr int TPS = H_BKS / CS;                // taps per weight stage
  constexpr int B_STAGE = BN * H_BKS;            // elements (128 k = TPS taps x CS channels)
  constexpr int B_CHUNKS = BN * (H_BKS / 8);
  constexpr int B_PER_T = (B_CHUNKS + H_NTHR - 1) / H_NTHR;
  constexpr int LDO = BN + 8;

  const int HD = g.TD + g.KD - 1, HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const int HP = HD * HH * HW;                   // halo positions
  const int nchunk = HP * CPP;
  const int T = g.KD * g.KH * g.KW;
  const int Tp = (T + TPS - 1) / TPS * TPS;
  const int spp = Tp / TPS;                      // 128-k stages per channel pass
  const int npass = g.C / CS;
  const int nq = spp * npass;
  const int ldw = npass * Tp * CS;
  const int rows = g.TD * g.TH * g.TW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH, twn = (g.OW + g.TW - 1) / g.TW;
  const int ntiles = g.N * tdn * thn * twn;

  bf16* halo = reinterpret_cast<bf16*>(dsm);                      // also the epilogue staging area
  bf16* Bs = reinterpret_cast<bf16*>(dsm + region_bytes);
  int* posinfo = reinterpret_cast<int*>(dsm + region_bytes + (RES ? nq : 2) * B_STAGE * 2);  // packed (hd, hh, hw)
  int* toffs_s = posinfo + HP;                                    // [Tp] tap offsets (LDS: no scalar
                                                                  // loads inside the k-loop)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wrow = wave & 3;                                   // 64-row block of the tile
  const int khalf = __builtin_amdgcn_readfirstlane(wave >> 2);   // k-half (BN=32) or column half (BN=64)
  const int ccol = KSPLIT ? 0 : khalf * 32;                      // this wave's first column
  const int lr = lane & 15, lg = lane >> 4;
  const int n0 = blockIdx.y * BN;
  // BN statistics: one (sum, sumsq) partial per workgroup (not per tile), so the
  // finalize pass reduces gridDim.x rows instead of thousands
  float st_sum = 0.f, st_sq = 0.f;
  auto write_stats = [&]() {
    if (STATS && tid < BN && n0 + tid < Ncol) {
      stats[(long long)blockIdx.x * 2 * Ncol + n0 + tid] = st_sum;
      stats[(long long)blockIdx.x * 2 * Ncol + Ncol + n0 + tid] = st_sq;
    }
  };
  // Dynamic tile schedule: workgroups take chunks of `chunk` consecutive tiles from
  // a global counter (sched[1 + blockIdx.y]).  A static partition would make the
  // whole kernel wait for its last workgroups whenever some CU slots are held by a
  // concurrent kernel (RCCL all-reduce overlapping backward); with chunks the
  // resident workgroups simply take more of them.  The last workgroup to finish
  // (sched[0] counts finished ones) resets the counters for the next launch.
  // chunk < 0: static partition instead (one contiguous run of -chunk tiles per
  // workgroup, XCD-aware order) -- the host's choice whenever BN statistics are taken
  // (per-workgroup partials over a fixed tile set: repeatable run to run)
  const bool dyn = chunk > 0;
  const int run = dyn ? chunk : -chunk;
  int nstatic = 0;
  __shared__ int s_grab;
  auto grab = [&]() -> int {                     // first tile of a fresh chunk, or -1
    if (!dyn) {
      const int t0 = nstatic++ == 0 ? xcd_remap(blockIdx.x, gridDim.x) * run : ntiles;
      return t0 < ntiles ? t0 : -1;
    }
    if (tid == 0) s_grab = atomicAdd(sched + 1 + blockIdx.y, 1) * chunk;
    lds_barrier();
    const int t0 = __builtin_amdgcn_readfirstlane(s_grab);
    lds_barrier();                               // everyone has read s_grab before it can change
    return t0 < ntiles ? t0 : -1;
  };
  auto finish = [&]() {
    write_stats();
    if (tid == 0 && dyn) {
      __threadfence();
      if (atomicAdd(sched, 1) == (int)(gridDim.x * gridDim.y) - 1) {
        for (int i = 0; i < (int)gridDim.y; ++i) atomicExch(sched + 1 + i, 0);
        atomicExch(sched, 0);
      }
    }
  };
  int tile = grab();
  if (tile < 0) {                                // whole workgroup exits together
    finish();
    return;
  }
  int cend = min(tile + run, ntiles);

  for (int pos = tid; pos < HP; pos += H_NTHR)
    posinfo[pos] = ((pos / (HW * HH)) << 20) | (((pos / HW) % HH) << 10) | (pos % HW);
  for (int t = tid; t < Tp; t += H_NTHR) toffs_s[t] = toffs[t];
  int hbase[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int r = wrow * 64 + mt * 16 + lr;
    const int rr = r < rows ? r : 0;
    const int w = rr % g.TW, th = (rr / g.TW) % g.TH, td = rr / (g.TW * g.TH);
    hbase[mt] = (td * HH + th) * HW + w;
  }
  __syncthreads();

  constexpr int HC = RES ? 3 : H_HC(BN);   // RES (s2d stem): the whole 8-channel halo prefetched in registers
  uint4 hreg[HC > 0 ? HC : 1];
  // halo origin of a job = (tile, channel pass p) (wave-uniform; decoded once per job)
  auto job_origin = [&](int jt, int p, const bf16*& base, int& dlo, int& hlo, int& wlo) {
    const TileIdx ti = tile_idx(jt, tdn, thn, twn);
    dlo = ti.td * g.TD - g.pd;
    hlo = ti.th * g.TH - g.ph;
    wlo = ti.tw * g.TW - g.pw;
    base = src + (long long)ti.n * g.ID * g.IH * g.IW * g.C + p * CS;
  };
  auto prefetch_halo = [&](int jt, int p) {
    const bf16* base;
    int dlo, hlo, wlo;
    job_origin(jt, p, base, dlo, hlo, wlo);
#pragma unroll
    for (int i = 0; i < HC; ++i) {
      // chunks past the halo are clamped to the last one (a duplicate, identical
      // LDS write), so every load is consumed by an unconditional store and the
      // compiler never has to assume a load still in flight at the k-loop top
      const int c = min(i * H_NTHR + tid, nchunk - 1);
      const int info = posinfo[c / CPP];
      const int gd = dlo + (info >> 20), gh = hlo + ((info >> 10) & 1023), gw = wlo + (info & 1023);
      const bool ok = (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH && (unsigned)gw < (unsigned)g.IW;
      const int off = ((gd * g.IH + gh) * g.IW + gw) * g.C + (c % CPP) * 8;
      const uint4 x = *(const uint4*)(base + (ok ? off : 0));
      hreg[i] = ok ? x : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_halo = [&](int jt, int p) {
#pragma unroll
    for (int i = 0; i < HC; ++i) {
      const int c = min(i * H_NTHR + tid, nchunk - 1);
      *(uint4*)(halo + (size_t)c * 8) = hreg[i];
    }
    if (HC * H_NTHR >= nchunk) return;
    const bf16* base;
    int dlo, hlo, wlo;
    job_origin(jt, p, base, dlo, hlo, wlo);
    for (int c0 = HC * H_NTHR; c0 < nchunk; c0 += 4 * H_NTHR) {   // tail of a large halo: synchronous
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = min(c0 + j * H_NTHR + tid, nchunk - 1);
        const int info = posinfo[c / CPP];
        const int gd = dlo + (info >> 20), gh = hlo + ((info >> 10) & 1023), gw = wlo + (info & 1023);
        const bool ok = (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH && (unsigned)gw < (unsigned)g.IW;
        const int off = ((gd * g.IH + gh) * g.IW + gw) * g.C + (c % CPP) * 8;
        const uint4 x = *(const uint4*)(base + (ok ? off : 0));
        v[j] = ok ? x : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = min(c0 + j * H_NTHR + tid, nchunk - 1);
        *(uint4*)(halo + (size_t)c * 8) = v[j];
      }
    }
  };

  // BN=32: stage s+1's weights are loaded at the top of stage s and written after
  // its MFMAs, so their latency hides behind a whole stage.  BN=64 has no VGPRs
  // to keep them in flight across the stage (they would spill) and instead loads
  // stage s+2 at the end of stage s, writing it in the middle of stage s+1.
  constexpr bool EARLY_B = KSPLIT || RES;
  uint4 rbA[B_PER_T];
  auto load_b = [&](int q, uint4* dst) {
    const int kbase = (q % nq) * H_BKS;
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int idx = tid + i * H_NTHR;
      // rows past Ncol re-read the last valid row: a B column only feeds its own
      // output column, which the epilogue drops, so no zero-fill (and no exec-masked
      // load whose register init forces a vmcnt(0) at the stage top) is needed
      const int r = (idx >> 4) < BN ? (idx >> 4) : BN - 1;
      const int k = kbase + (idx & 15) * 8;
      if constexpr (EARLY_B) {
        const int row = n0 + r < Ncol ? n0 + r : Ncol - 1;
        dst[i] = *(const uint4*)(wt + (long long)row * ldw + k);
      } else {
        const bool ok = idx < B_CHUNKS && n0 + r < Ncol;
        const uint4 v = *(const uint4*)(wt + (ok ? (long long)(n0 + r) * ldw + k : 0));
        dst[i] = ok ? v : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto write_b = [&](int buf, const uint4* srcr) {
    bf16* b = Bs + buf * B_STAGE;
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int idx = tid + i * H_NTHR;
      if (B_CHUNKS % H_NTHR == 0 || idx < B_CHUNKS) {
        const int r = idx >> 4, c = idx & 15;
        *(uint4*)(b + r * H_BKS + ((c ^ (r & 15)) << 3)) = srcr[i];
      }
    }
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  prefetch_halo(tile, 0);
  if constexpr (RES) {
    for (int q = 0; q < nq; ++q) {        // all stages, once (the job loop's first barrier publishes them)
      load_b(q, rbA);
      write_b(q, rbA);
    }
  } else {
    load_b(0, rbA);
    write_b(0, rbA);
    if constexpr (!EARLY_B) load_b(1, rbA);
  }

  int s = 0;                              // global stage counter
  int pass = 0;
  while (true) {
    lds_barrier();                      // previous halo / epilogue staging fully consumed
    store_halo(tile, pass);
    lds_barrier();
    // the next job (same tile / next pass, next tile of the chunk, or a new chunk)
    int ntile = tile, npass_i = pass + 1, ncend = cend;
    if (npass_i == npass) {
      npass_i = 0;
      ntile = tile + 1;
      if (ntile == cend) {
        ntile = grab();
        ncend = ntile < 0 ? -1 : min(ntile + run, ntiles);
      }
    }
    if (ntile >= 0) prefetch_halo(ntile, npass_i);   // lands during this job's MFMAs
    for (int local = 0; local < spp; ++local, ++s) {
      if constexpr (EARLY_B && !RES) {
        load_b(s + 1, rbA);
        __builtin_amdgcn_sched_barrier(0);  // keep the loads here (the scheduler would sink them to their use)
      }
      const bf16* b = Bs + (RES ? pass * spp + local : (s & 1)) * B_STAGE;
      // lane group lg reads tap lg>>1 / channel half lg&1 (CS = 16) or tap lg (CS = 8)
      const int* tp = toffs_s + local * TPS + (KSPLIT ? khalf * (TPS / 2) : 0) + (CS == 16 ? (lg >> 1) : lg);
#pragma unroll
      for (int kk = 0; kk < (KSPLIT ? 2 : 4); ++kk) {
        const int ks = (KSPLIT ? khalf * 2 : 0) + kk;
        const int toff = tp[kk * (32 / CS)];
        const int hsub = CS == 16 ? (lg & 1) * 8 : 0;
        bf16x8 fa[4], fb[NT];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          fa[mt] = *(const bf16x8*)(halo + (size_t)(hbase[mt] + toff) * CS + hsub);
        const int ch = ks * 4 + lg;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int row = ccol + nt * 16 + lr;
          fb[nt] = *(const bf16x8*)(b + row * H_BKS + ((ch ^ (row & 15)) << 3));
        }
        // every row block runs all 4 MFMA row tiles (no branch in the k-loop: rows past
        // the tile read a valid halo position and are dropped by the epilogue)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
      }
      if constexpr (!RES) {
        write_b((s + 1) & 1, rbA);        // stage s+1 (its buffer's last readers passed the previous barrier)
        if constexpr (!EARLY_B) load_b(s + 2, rbA);
        lds_barrier();
      }
    }
    if constexpr (RES) lds_barrier();     // all waves are done with the halo before it is reused
    if (pass != npass - 1) {
      pass = npass_i;                   // same tile, next channel pass
      continue;
    }

    // ---- epilogue of a finished tile (staging in the halo region) ----
    const TileIdx ti = tile_idx(tile, tdn, thn, twn);
    const int th_i = ti.th, td_i = ti.td, n = ti.n;
    const int d0 = td_i * g.TD, h0 = th_i * g.TH, w0 = ti.tw * g.TW;
    const bool wfull = w0 + g.TW <= g.OW;          // uniform: the tile's columns are all inside OW
    // split-K reduction: the khalf=1 wave of each row block hands its partial
    // sums to its khalf=0 partner through LDS (lane-major, conflict-free)
    if constexpr (KSPLIT) {
      float* part = reinterpret_cast<float*>(dsm);
      {
        float* slot = part + (size_t)wrow * (4 * NT * 4 * 64);
        if (khalf == 1) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
              for (int r = 0; r < 4; ++r) slot[((mt * NT + nt) * 4 + r) * 64 + lane] = acc[mt][nt][r];
        }
        // epilogue hand-offs are LDS-only: lds_barrier, not __syncthreads, whose fence
        // would drain vmcnt and stall on the next job's halo prefetch
        lds_barrier();
        if (khalf == 0) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[mt][nt][r] += slot[((mt * NT + nt) * 4 + r) * 64 + lane];
        }
        lds_barrier();
      }
    }
    bf16* Os = reinterpret_cast<bf16*>(dsm);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int col = ccol + nt * 16 + lr;
      float bv = 0.f;
      if constexpr (HAS_BIAS) bv = (n0 + col) < Ncol ? bias[n0 + col] : 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if (!KSPLIT || khalf == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wrow * 64 + mt * 16 + lg * 4 + r;
            Os[row * LDO + col] = f2bf(act_fwd(acc[mt][nt][r] + bv, ACT));
          }
        }
        acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
    if constexpr (STATS) {
      // BN partial sums over the valid rows of the staged (bf16-rounded) tile
      constexpr int NPART = H_NTHR / BN;
      float* red = reinterpret_cast<float*>(dsm + (size_t)H_BM * LDO * 2);
      lds_barrier();
      const int col = tid % BN, part = tid / BN;
      float sm = 0.f, qq = 0.f;
      for (int row = part; row < rows; row += NPART) {
        const int td = row / (g.TW * g.TH), th = (row / g.TW) % g.TH;
        if (d0 + td < g.OD && h0 + th < g.OH && (wfull || w0 + row % g.TW < g.OW)) {
          const float f = bf2f(Os[row * LDO + col]);
          sm += f;
          qq += f * f;
        }
      }
      red[part * 2 * BN + col] = sm;
      red[part * 2 * BN + BN + col] = qq;
      lds_barrier();
      if (tid < BN) {
#pragma unroll
        for (int q2 = 0; q2 < NPART; ++q2) { st_sum += red[q2 * 2 * BN + tid]; st_sq += red[q2 * 2 * BN + BN + tid]; }
      }
    }
    lds_barrier();
    constexpr int CPR = BN / 8;
    const bool vec_out = (Ncol % 8) == 0;
#pragma unroll
    for (int i = 0; i < (H_BM * CPR + H_NTHR - 1) / H_NTHR; ++i) {
      const int idx = tid + i * H_NTHR;
      const int row = idx / CPR, ch = idx % CPR;
      if (row >= rows) continue;
      const int w = row % g.TW, th = (row / g.TW) % g.TH, td = row / (g.TW * g.TH);
      if (d0 + td >= g.OD || h0 + th >= g.OH || w0 + w >= g.OW) continue;
      const long long m = (((long long)n * g.OD + d0 + td) * g.OH + h0 + th) * g.OW + w0 + w;
      const int col = n0 + ch * 8;
      if (vec_out && col + 8 <= Ncol) {
        *(uint4*)(out + m * Ncol + col) = *(const uint4*)(Os + row * LDO + ch * 8);
      } else {
        for (int j = 0; j < 8; ++j)
          if (col + j < Ncol) out[m * Ncol + col + j] = Os[row * LDO + ch * 8 + j];
      }
    }
    tile = ntile;
    pass = npass_i;
    cend = ncend;
    if (tile < 0) break;
  }
  finish();
}

// ---------------------------------------------------------------------------
// Weight gradient on the same halo tiles
// ---------------------------------------------------------------------------
// dW[co][tap][ci] = sum_rows dy[row][co] * x[pos(row) + tap][ci]
// One workgroup: a 16-channel input slice (grid.z), a group of 4*TPW taps
// (grid.y, TPW per wave) and a strided set of output tiles (grid.x,
// persistent).  Per tile the dy tile [256][Cout] and the x halo slice are
// staged in LDS once; both MFMA operands are read with ds_read_b64_tr_b16
// (k = tile rows is the slow axis of both), the x operand at per-lane halo
// positions row -> pos(row) + tapoff.  fp32 accumulators live across all the
// workgroup's tiles (a static set) and are stored into the workgroup's partial
// dW row (part[blockIdx.x]); fn_part_reduce adds the rows in a fixed order, so
// dW is bitwise repeatable (no float atomics).
template <int MT>
__device__ __forceinline__ bf16x8 tr_pair(const bf16* lo, const bf16* hi) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lo));
  s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(hi));
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// halo / dy chunks per thread prefetched into registers for the NEXT tile
#define WG_HC(MT) ((MT) <= 2 ? 8 : 4)

// CS = channels per halo slice (grid.z walks C/CS slices).  CS = 16: the MFMA
// N axis is the slice's 16 input channels, one accumulator per (tap, co
// block).  CS = 8: the N axis is (tap pair, 8 channels) -- lanes p = 0,1 of a
// transposed-read quad fetch tap 2j, lanes p = 2,3 tap 2j+1 -- so a wave covers
// the same taps with half the accumulators.
// DIV = 2 halves the taps per wave (and the accumulators) for convs with few taps
// (3^3 = 27: 4 waves x 16 taps would leave half the waves idle).
template <int MT, int CS, int DIV>
__global__ __launch_bounds__(256, 2) void conv_halo_wgrad_kernel(const bf16* __restrict__ dy,
                                                                 const bf16* __restrict__ src,
                                                                 float* __restrict__ dw, HaloGeom g, int Cout) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  // 16x16 accumulator column blocks per (wave, co block); both slice widths give a
  // wave the same taps (CS = 8 packs two taps per block, so half the blocks)
  constexpr int NACC = (MT == 1 ? 16 : 32 / MT) / (16 / CS) / DIV;
  constexpr int TPW = CS == 16 ? NACC : 2 * NACC;   // taps per wave
  constexpr int CPP = CS / 8;
  constexpr int BCO = MT * 16;
  constexpr int LDY = BCO + 16;            // conflict-free transposed reads (as igemm wgrad)
  constexpr int YC = BCO / 8;              // 16-B chunks per dy row
  constexpr int HC = WG_HC(MT);
  const int HD = g.TD + g.KD - 1, HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const int HP = HD * HH * HW;
  const int nchunk = HP * CPP;
  const int T = g.KD * g.KH * g.KW;
  const int rows = g.TD * g.TH * g.TW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH, twn = (g.OW + g.TW - 1) / g.TW;
  const int ntiles = g.N * tdn * thn * twn;

  bf16* Ys = reinterpret_cast<bf16*>(dsm);                                   // [256][LDY]
  bf16* halo = reinterpret_cast<bf16*>(dsm + (size_t)H_BM * LDY * 2);        // [HP][CS]
  int* rowpos = reinterpret_cast<int*>(dsm + (size_t)H_BM * LDY * 2 + (size_t)HP * CS * 2);  // [256]
  int* rowinfo = rowpos + H_BM;                                               // packed (td, th, w) per row
  int* posinfo = rowinfo + H_BM;                                              // packed (hd, hh, hw) per position

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int slice = blockIdx.z;
  const int tap0 = (blockIdx.y * 4 + wave) * TPW;          // uniform: tap offsets stay in SGPRs
  // Static schedule: one contiguous run of ntiles / gridDim.x tiles per workgroup x (the
  // grid.y/grid.z workgroups -- tap groups, slices -- of a tile walk it in near lockstep and
  // share its dy / halo in L2), then at most one of the remaining tiles (tile per * gx + x).
  // The workgroup's tile set is fixed, so its partial dW is the same run to run.  (Through
  // round 4 the remainder and the last 1/8 were taken from a counter: dW changed in the last
  // bits with the schedule.)
  const int per = ntiles / (int)gridDim.x;
  int ngrab = 0;
  auto grab = [&](int& end) -> int {
    const int k = ngrab++;
    if (k == 0 && per > 0) {
      end = (int)(blockIdx.x + 1) * per;
      return (int)blockIdx.x * per;
    }
    if (k > 1 || (k == 1 && per == 0)) return -1;
    const int t0 = per * (int)gridDim.x + (int)blockIdx.x;
    end = t0 + 1;
    return t0 < ntiles ? t0 : -1;
  };

  for (int r = tid; r < H_BM; r += 256) {
    int pos = 0, info = -1;
    if (r < rows) {
      const int w = r % g.TW, th = (r / g.TW) % g.TH, td = r / (g.TW * g.TH);
      pos = (td * HH + th) * HW + w;
      info = (td << 20) | (th << 10) | w;
    }
    rowpos[r] = pos;
    rowinfo[r] = info;
  }
  for (int pos = tid; pos < HP; pos += 256)
    posinfo[pos] = ((pos / (HW * HH)) << 20) | (((pos / HW) % HH) << 10) | (pos % HW);
  int toff[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = tap0 + i < T ? tap0 + i : 0;
    const int kw = t % g.KW, kh = (t / g.KW) % g.KH, kd = t / (g.KW * g.KH);
    toff[i] = (kd * HH + kh) * HW + kw;
  }
  const int ntap = T - tap0 < TPW ? (T - tap0 > 0 ? T - tap0 : 0) : TPW;   // live taps of this wave
  __syncthreads();

  uint4 yreg[YC], hreg[HC];
  // validity of the prefetched chunks as bit masks: the loads themselves are
  // unconditional (invalid ones read offset 0) and are zeroed only when stored, so
  // no load is exec-masked over a zero-initialised register -- that pattern makes
  // hipcc's wait-count pass drain vmcnt at the top of the k-loop, i.e. it turns the
  // prefetch synchronous
  unsigned ymask = 0, hmask = 0;
  // per-tile origins (wave-uniform; decoded once per tile, not per chunk)
  struct TileOrg { long long ybase, xbase; int d0, h0, w0, dlo, hlo, wlo; };
  auto tile_org = [&](int tile) -> TileOrg {
    const TileIdx ti = tile_idx(tile, tdn, thn, twn);
    TileOrg o;
    o.d0 = ti.td * g.TD;
    o.h0 = ti.th * g.TH;
    o.w0 = ti.tw * g.TW;
    o.dlo = o.d0 - g.pd;
    o.hlo = o.h0 - g.ph;
    o.wlo = o.w0 - g.pw;
    o.ybase = (long long)ti.n * g.OD * g.OH * g.OW;
    o.xbase = (long long)ti.n * g.ID * g.IH * g.IW;
    return o;
  };
  auto dy_src = [&](const TileOrg& o, int idx, long long& m) -> bool {
    const int r = idx / YC, c = idx % YC;
    const int info = rowinfo[r];
    const int td = o.d0 + (info >> 20), th = o.h0 + ((info >> 10) & 1023), w = o.w0 + (info & 1023);
    m = (o.ybase + ((long long)td * g.OH + th) * g.OW + w) * Cout + c * 8;
    return info >= 0 && td < g.OD && th < g.OH && w < g.OW && c * 8 < Cout;
  };
  auto halo_src = [&](const TileOrg& o, int c, long long& off) -> bool {
    const int info = posinfo[c < nchunk ? c / CPP : 0];
    const int gd = o.dlo + (info >> 20), gh = o.hlo + ((info >> 10) & 1023), gw = o.wlo + (info & 1023);
    off = (o.xbase + ((long long)gd * g.IH + gh) * g.IW + gw) * g.C + slice * CS + (c % CPP) * 8;
    return c < nchunk && (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
           (unsigned)gw < (unsigned)g.IW;
  };
  auto masked = [](uint4 v, bool ok) -> uint4 {
    const unsigned m = ok ? ~0u : 0u;
    return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
  };
  auto prefetch = [&](int tile) {
    const TileOrg o = tile_org(tile);
    ymask = hmask = 0;
#pragma unroll
    for (int i = 0; i < YC; ++i) {
      long long m;
      const bool ok = dy_src(o, i * 256 + tid, m);
      yreg[i] = *(const uint4*)(dy + (ok ? m : 0));
      ymask |= (unsigned)ok << i;
    }
#pragma unroll
    for (int i = 0; i < HC; ++i) {
      long long off;
      // chunks past the halo clamp to the last one: a duplicate, identical LDS write
      const bool ok = halo_src(o, min(i * 256 + tid, nchunk - 1), off);
      hreg[i] = *(const uint4*)(src + (ok ? off : 0));
      hmask |= (unsigned)ok << i;
    }
  };
  auto store = [&](int tile) {
#pragma unroll
    for (int i = 0; i < YC; ++i) {
      const int idx = i * 256 + tid;
      *(uint4*)(Ys + (idx / YC) * LDY + (idx % YC) * 8) = masked(yreg[i], (ymask >> i) & 1);
    }
#pragma unroll
    for (int i = 0; i < HC; ++i) {
      const int c = min(i * 256 + tid, nchunk - 1);
      *(uint4*)(halo + (size_t)c * 8) = masked(hreg[i], (hmask >> i) & 1);
    }
    if (HC * 256 >= nchunk) return;
    const TileOrg o = tile_org(tile);
    for (int c0 = HC * 256; c0 < nchunk; c0 += 4 * 256) {   // tail of a large halo: synchronous
      uint4 v[4];
      bool okv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        long long off;
        okv[j] = halo_src(o, min(c0 + j * 256 + tid, nchunk - 1), off);
        v[j] = *(const uint4*)(src + (okv[j] ? off : 0));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = min(c0 + j * 256 + tid, nchunk - 1);
        *(uint4*)(halo + (size_t)c * 8) = masked(v[j], okv[j]);
      }
    }
  };

  f32x4 acc[NACC][MT];
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  int cend = 0;
  int tile = grab(cend);
  if (tile >= 0) prefetch(tile);
  while (tile >= 0) {
    lds_barrier();                 // previous tile's reads are done
    store(tile);
    lds_barrier();
    int ntile = tile + 1, ncend = cend;
    if (ntile == cend) ntile = grab(ncend);
    if (ntile >= 0) prefetch(ntile);   // lands during this tile's MFMAs
    const int kst = ntap > 0 ? (rows + 31) >> 5 : 0;   // waves past the last tap only stage
    for (int ks = 0; ks < kst; ++ks) {
      bf16x8 fa[MT];
      const int r_lo = ks * 32 + 4 * G + q, r_hi = r_lo + 16;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        fa[mt] = tr_pair<MT>(Ys + r_lo * LDY + mt * 16 + 4 * p4, Ys + r_hi * LDY + mt * 16 + 4 * p4);
      const int plo = rowpos[r_lo], phi = rowpos[r_hi];
      // no per-tap branch: dead taps (past T) read halo position offset 0 and
      // their accumulators are never stored
      auto read_b = [&](int i) -> bf16x8 {
        if constexpr (CS == 16) {
          return tr_pair<MT>(halo + (size_t)(plo + toff[i]) * 16 + 4 * p4,
                             halo + (size_t)(phi + toff[i]) * 16 + 4 * p4);
        } else {
          const int to = (p4 & 2) ? toff[2 * i + 1] : toff[2 * i];
          return tr_pair<MT>(halo + (size_t)(plo + to) * 8 + 4 * (p4 & 1),
                             halo + (size_t)(phi + to) * 8 + 4 * (p4 & 1));
        }
      };
      // B fragments double-buffered in registers: tap i+1 is read while tap i's
      // MFMAs run, so the LDS latency is not exposed once per tap
      bf16x8 fb_next = read_b(0);
#pragma unroll
      for (int i = 0; i < NACC; ++i) {
        const bf16x8 fb = fb_next;
        if (i + 1 < NACC) fb_next = read_b(i + 1);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb, acc[i][mt], 0, 0, 0);
      }
    }
    tile = ntile;
    cend = ncend;
  }
  // D[row=co][col=n]: lane holds co = mt*16 + (lane>>4)*4 + r, n = lane & 15
  // (CS=16: n = input channel; CS=8: n = (tap of the pair) * 8 + channel); plain stores into
  // this workgroup's partial row (the (y, z) workgroups of one x write disjoint (tap, channel)
  // columns of it, every element exactly once)
  float* part = dw + (long long)blockIdx.x * Cout * T * g.C;
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    const int t = CS == 16 ? tap0 + i : tap0 + 2 * i + ((lane & 15) >> 3);
    const int ci = CS == 16 ? (lane & 15) : (lane & 7);
    if (t < T && t - tap0 < ntap) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = mt * 16 + (lane >> 4) * 4 + r;
          if (co < Cout) part[((long long)co * T + t) * g.C + slice * CS + ci] = acc[i][mt][r];
        }
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static HaloGeom parse_halo(const int* v) {
  HaloGeom g;
  g.N = v[0]; g.ID = v[1]; g.IH = v[2]; g.IW = v[3]; g.C = v[4];
  g.OD = v[5]; g.OH = v[6]; g.OW = v[7];
  g.KD = v[8]; g.KH = v[9]; g.KW = v[10];
  g.pd = v[11]; g.ph = v[12]; g.pw = v[13];
  g.TD = v[14]; g.TH = v[15]; g.TW = v[16];
  return g;
}

static int halo_cs(int C) { return C % 16 == 0 ? 16 : (C % 8 == 0 ? 8 : 0); }

static size_t halo_region_bytes(const HaloGeom& g, int BN, int CS) {
  const size_t hp = (size_t)(g.TD + g.KD - 1) * (g.TH + g.KH - 1) * (g.TW + g.KW - 1);
  size_t epi = (size_t)H_BM * (BN + 8) * 2 + 2 * H_NTHR * 4;
  if (epi < 32 * 1024) epi = 32 * 1024;          // split-K partial sums (one round)
  const size_t r = hp * CS * 2 > epi ? hp * CS * 2 : epi;
  return (r + 15) & ~(size_t)15;
}

// weight stages of 128 k (TPS taps x CS channels) over all channel slices
static int halo_nq(const HaloGeom& g, int CS) {
  const int T = g.KD * g.KH * g.KW, tps = H_BKS / CS;
  return (g.C / CS) * ((T + tps - 1) / tps);
}

static size_t halo_lds_bytes(const HaloGeom& g, int BN, int CS, bool res) {
  const size_t hp = (size_t)(g.TD + g.KD - 1) * (g.TH + g.KH - 1) * (g.TW + g.KW - 1);
  const size_t T = (size_t)g.KD * g.KH * g.KW;
  const size_t stages = res ? (size_t)halo_nq(g, CS) : 2;
  return halo_region_bytes(g, BN, CS) + stages * BN * H_BKS * 2 + hp * 4 + (T + 15) / 16 * 64 + 16;
}

// weights-resident variant: 8-channel slices, BN = 32, <= 4 stages (32 KB), and
// still two workgroups per CU
static bool halo_resident(const HaloGeom& g, int BN, int CS) {
  return BN == 32 && CS == 8 && halo_nq(g, CS) <= 4 && halo_lds_bytes(g, BN, CS, true) <= 80 * 1024;
}

template <int BN, int ACT, bool HB, bool ST, int CS, bool RES>
static int launch_halo(dim3 grid, size_t lds, int region, hipStream_t st, const bf16* s, const bf16* w,
                       const float* b, bf16* o, float* stats, const int* toffs, const HaloGeom& g, int Ncol,
                       int* sched, int chunk) {
  static size_t configured = 0;
  if (lds > configured) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_halo_kernel<BN, ACT, HB, ST, CS, RES>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    configured = lds;
  }
  hipLaunchKernelGGL((conv_halo_kernel<BN, ACT, HB, ST, CS, RES>), grid, dim3(H_NTHR), lds, st, s, w, b, o, stats, toffs,
                     g, Ncol, region, sched, chunk);
  return 0;
}

static int g_num_cus = 0;
extern "C" int fn_conv_halo_workers(const int* geom17, int Ncol);

// wt: [Ncol][C/CS][Tp][CS] bf16 (taps padded to a multiple of 128/CS), CS = 16 when
// C % 16 == 0 else 8; toffs: int [>= Tp] halo position offsets of the taps (0 for
// padding taps); returns 0 on success.
// sched: int[1 + column blocks] tile-schedule counters, zero before the first launch
// (every launch leaves them zero again); at most one launch in flight per buffer.
extern "C" int fn_conv_halo(const void* src, const void* wt, const float* bias, void* out, float* stats,
                            const int* toffs, const int* geom17, int Ncol, int act, int* sched, hipStream_t st) {
  const HaloGeom g = parse_halo(geom17);
  const int CS = halo_cs(g.C);
  if (CS == 0 || g.TD * g.TH * g.TW > H_BM || g.TW < 1 || g.TW > g.OW || g.TD < 1 || g.TH < 1) return -2;
  if (stats && act != ACT_NONE) return -1;
  const int BN = Ncol <= 32 ? 32 : 64;
  const bool res = halo_resident(g, BN, CS);
  const size_t lds = halo_lds_bytes(g, BN, CS, res);
  const int region = (int)halo_region_bytes(g, BN, CS);
  if (lds > 160 * 1024) return -4;
  const int ncb = (Ncol + BN - 1) / BN;
  const int workers = fn_conv_halo_workers(geom17, Ncol);
  if (!sched || ncb > 63) return -6;
  const int ntiles_all = g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) * ((g.OW + g.TW - 1) / g.TW);
  // ~4 chunks per workgroup: enough slack to absorb late or missing workgroups,
  // few enough that consecutive tiles (shared halo rows) stay on one workgroup
  int chunk = ntiles_all / (4 * workers) > 1 ? ntiles_all / (4 * workers) : 1;
  // BN statistics: one partial row per workgroup, so its tiles must not depend on the dynamic
  // schedule (bitwise-repeatable statistics): the static partition
  if (stats) chunk = -((ntiles_all + workers - 1) / workers);
  dim3 grid((unsigned)workers, ncb);
  const bf16* s = (const bf16*)src;
  const bf16* w = (const bf16*)wt;
  bf16* o = (bf16*)out;
  const bool hb = bias != nullptr;
  int rc;
#define HCASE(B, A, H, S, C)                                                                     \
  rc = (B == 32 && C == 8 && res)                                                                \
           ? launch_halo<B, A, H, S, C, (B == 32 && C == 8)>(grid, lds, region, st, s, w, bias, o, stats, toffs, g, Ncol, \
                                                               sched, chunk)                                    \
           : launch_halo<B, A, H, S, C, false>(grid, lds, region, st, s, w, bias, o, stats, toffs, g, Ncol, sched, chunk)
#define HBN(B, C)                                                   \
  do {                                                              \
    if (stats) HCASE(B, ACT_NONE, false, true, C);                  \
    else if (act == ACT_NONE) { if (hb) HCASE(B, ACT_NONE, true, false, C); else HCASE(B, ACT_NONE, false, false, C); } \
    else if (act == ACT_RELU) HCASE(B, ACT_RELU, true, false, C);    \
    else if (act == ACT_TANH) HCASE(B, ACT_TANH, true, false, C);    \
    else HCASE(B, ACT_SIGMOID, true, false, C);                      \
  } while (0)
  if (act != ACT_NONE && !hb) return -5;   // activation variants are instantiated with bias only
  if (CS == 16) {
    if (BN == 32) HBN(32, 16); else HBN(64, 16);
  } else {
    if (BN == 32) HBN(32, 8); else HBN(64, 8);
  }
#undef HBN
#undef HCASE
  if (rc) return rc;
  FN_CHECK_LAUNCH();
  return 0;
}

// number of persistent workgroups (= rows of the BN-statistics slab) fn_conv_halo launches
extern "C" int fn_conv_halo_workers(const int* geom17, int Ncol) {
  const HaloGeom g = parse_halo(geom17);
  const int CS = halo_cs(g.C);
  if (CS == 0) return -2;
  const int BN = Ncol <= 32 ? 32 : 64;
  const size_t lds = halo_lds_bytes(g, BN, CS, halo_resident(g, BN, CS));
  if (g_num_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_num_cus <= 0)
      g_num_cus = 256;
  }
  const int ntiles = g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) * ((g.OW + g.TW - 1) / g.TW);
  const int ncb = (Ncol + BN - 1) / BN;
  const int per_cu = (int)((160 * 1024) / lds) < 2 ? 1 : 2;
  int workers = (g_num_cus * per_cu + ncb - 1) / ncb;
  return workers > ntiles ? ntiles : workers;
}

extern "C" long long fn_conv_halo_lds(const int* geom17, int Ncol) {
  const HaloGeom g = parse_halo(geom17);
  const int BN = Ncol <= 32 ? 32 : 64, CS = halo_cs(g.C) ? halo_cs(g.C) : 16;
  return (long long)halo_lds_bytes(g, BN, CS, halo_resident(g, BN, CS));
}

static size_t halo_wgrad_lds(const HaloGeom& g, int MT, int CS) {
  const size_t hp = (size_t)(g.TD + g.KD - 1) * (g.TH + g.KH - 1) * (g.TW + g.KW - 1);
  return (size_t)H_BM * (MT * 16 + 16) * 2 + hp * CS * 2 + 2 * H_BM * 4 + hp * 4 + 16;
}

// taps-per-wave divisor: 2 when halving the taps per wave fills >= 15 % more of the
// 4-wave tap slots (few-tap kernels, e.g. 3^3 with Cout <= 32)
static int halo_wgrad_div(int T, int MT) {
  const int tpw = MT == 1 ? 16 : 32 / MT;
  auto used = [&](int t) { const int slots = (T + 4 * t - 1) / (4 * t) * 4 * t; return (double)T / slots; };
  return (tpw % 2 == 0 && used(tpw / 2) >= 1.15 * used(tpw)) ? 2 : 1;
}

// grid.y of fn_conv_halo_wgrad (tap groups); the caller sizes grid.x from it
extern "C" int fn_conv_halo_wgrad_yblocks(const int* geom17, int Cout) {
  const HaloGeom g = parse_halo(geom17);
  const int MT = (Cout + 15) / 16, T = g.KD * g.KH * g.KW;
  const int tpw = (MT == 1 ? 16 : 32 / MT) / halo_wgrad_div(T, MT);
  return (T + 4 * tpw - 1) / (4 * tpw);
}

// effective grid.x of fn_conv_halo_wgrad (the partial rows `part` must hold)
extern "C" int fn_conv_halo_wgrad_gx(const int* geom17, int grid_x) {
  const HaloGeom g = parse_halo(geom17);
  if (g.TD < 1 || g.TH < 1 || g.TW < 1) return -2;
  const int ntiles = g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) * ((g.OW + g.TW - 1) / g.TW);
  return grid_x < ntiles ? (grid_x > 0 ? grid_x : 1) : ntiles;
}

// dw: fp32 [Cout][T][C], accumulated into (+=); part: fp32 scratch [fn_conv_halo_wgrad_gx][Cout][T][C]
// (every element written by the kernel, then summed over the rows in a fixed order)
extern "C" int fn_conv_halo_wgrad(const void* dy, const void* src, float* dw, float* part, const int* geom17, int Cout,
                                  int grid_x, hipStream_t st) {
  const HaloGeom g = parse_halo(geom17);
  const int CS = halo_cs(g.C);
  if (CS == 0 || g.TD * g.TH * g.TW > H_BM || g.TW < 1 || g.TW > g.OW || Cout > 64 || Cout % 8 != 0) return -2;
  const int MT = (Cout + 15) / 16;
  const size_t lds = halo_wgrad_lds(g, MT, CS);
  if (lds > 160 * 1024) return -4;
  const int T = g.KD * g.KH * g.KW;
  const int DIV = halo_wgrad_div(T, MT);
  const int TPW = (MT == 1 ? 16 : 32 / MT) / DIV;   // taps per wave (either slice width)
  const int ntiles = g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) * ((g.OW + g.TW - 1) / g.TW);
  const int gx = grid_x < ntiles ? (grid_x > 0 ? grid_x : 1) : ntiles;
  dim3 grid((unsigned)gx, (unsigned)((T + 4 * TPW - 1) / (4 * TPW)), (unsigned)(g.C / CS));
  if (!part) return -6;
  const bf16* d = (const bf16*)dy;
  const bf16* s = (const bf16*)src;
#define WCASE1(M, C, D)                                                                                    \
  do {                                                                                                     \
    static size_t cfg = 0;                                                                                 \
    if (lds > cfg) {                                                                                       \
      hipError_t e = hipFuncSetAttribute((const void*)conv_halo_wgrad_kernel<M, C, D>,                     \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);            \
      if (e != hipSuccess) return (int)e;                                                                  \
      cfg = lds;                                                                                           \
    }                                                                                                      \
    hipLaunchKernelGGL((conv_halo_wgrad_kernel<M, C, D>), grid, dim3(256), lds, st, d, s, part, g, Cout);  \
  } while (0)
#define WCASE(M, C) do { if (DIV == 2) WCASE1(M, C, 2); else WCASE1(M, C, 1); } while (0)
  if (CS == 16) {
    if (MT == 1) WCASE(1, 16); else if (MT == 2) WCASE(2, 16); else if (MT == 3) WCASE(3, 16); else WCASE(4, 16);
  } else {
    if (MT == 1) WCASE(1, 8); else if (MT == 2) WCASE(2, 8); else if (MT == 3) WCASE(3, 8); else WCASE(4, 8);
  }
#undef WCASE
#undef WCASE1
  FN_CHECK_LAUNCH();
  return fn_part_reduce(part, dw, (long long)Cout * T * g.C, gx, 1, st);
}

// ---------------------------------------------------------------------------
// space-to-depth packing for strided few-channel convs (the FeatureNet-3D stem)
// ---------------------------------------------------------------------------
// out[n][d2][h2][w2][CO] (CO = 8 or 16 channels, zero padded) with channel
// ((a * sh + b) * sw + c) * C + ci = x[n][d2*sd + a][h2*sh + b][w2*sw + c][ci]
// (zero outside x).  One thread per output position, one 16-B store per 8
// channels; a 1-channel stride-2 stem reads 4 bf16 pairs per position.
// T: bf16, or uint8 (binary voxel occupancy stored as bytes -- a quarter of the copy-in and of this
// kernel's reads; 0 / 1 convert exactly)
__device__ __forceinline__ float s2d_in(bf16 v) { return bf2f(v); }
__device__ __forceinline__ float s2d_in(unsigned char v) { return (float)v; }

template <typename T>
__global__ __launch_bounds__(256) void s2d_pack_kernel(const T* __restrict__ x, bf16* __restrict__ out,
                                                        int N, int D, int H, int W, int C, int sd, int sh, int sw,
                                                        int D2, int H2, int W2, int CO, int pd, int ph, int pw) {
  const long long npos = (long long)N * D2 * H2 * W2;
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npos) return;
  const int w2 = (int)(p % W2), h2 = (int)((p / W2) % H2), d2 = (int)((p / ((long long)W2 * H2)) % D2);
  const long long n = p / ((long long)W2 * H2 * D2);
  const int creal = sd * sh * sw * C;
  if (C == 1 && sd == 2 && sh == 2 && sw == 2 && !((D | H | W | pd | ph | pw) & 1)) {
    // the 1-channel stride-2 stem with even extents and even leading pads (FeatureNet-3D's valid
    // stem, the seg model's 'same' one): every (w, w+1) pair is aligned and wholly inside or
    // outside the input -- 4 pair loads -> one 16-B store
    const int d0 = 2 * d2 - pd, h0 = 2 * h2 - ph, w0 = 2 * w2 - pw;
    const bool wok = (unsigned)w0 < (unsigned)W;
    unsigned q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = d0 + (k >> 1), h = h0 + (k & 1);
      q[k] = 0u;
      if (!wok || (unsigned)d >= (unsigned)D || (unsigned)h >= (unsigned)H) continue;
      const long long off = ((n * D + d) * H + h) * (long long)W + w0;
      if constexpr (sizeof(T) == 2) {
        q[k] = reinterpret_cast<const unsigned*>(x)[off >> 1];
      } else {
        const unsigned short b = reinterpret_cast<const unsigned short*>(x)[off >> 1];
        q[k] = (unsigned)__builtin_bit_cast(unsigned short, f2bf((float)(b & 0xffu))) |
               ((unsigned)__builtin_bit_cast(unsigned short, f2bf((float)(b >> 8))) << 16);
      }
    }
    *(uint4*)(out + p * CO) = make_uint4(q[0], q[1], q[2], q[3]);
    if (CO == 16) *(uint4*)(out + p * CO + 8) = make_uint4(0, 0, 0, 0);
    return;
  }
  for (int c0 = 0; c0 < CO; c0 += 8) {
    Pack8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = c0 + j;
      float f = 0.f;
      if (ch < creal) {
        const int ci = ch % C, blk = ch / C;
        const int c = blk % sw, b = (blk / sw) % sh, a = blk / (sw * sh);
        // (leading zero pads of a padded strided conv: the packed grid covers the padded input)
        const int d = d2 * sd + a - pd, h = h2 * sh + b - ph, w = w2 * sw + c - pw;
        if ((unsigned)d < (unsigned)D && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
          f = s2d_in(x[(((n * D + d) * H + h) * W + w) * C + ci]);
      }
      v.e[j] = f2bf(f);
    }
    *(uint4*)(out + p * CO + c0) = v.u;
  }
}

// geom: N D H W C sd sh sw D2 H2 W2 CO [pd ph pw] (leading pads, default 0); u8: x is uint8
extern "C" int fn_s2d_pack(const void* x, void* out, const int* geom, int glen, hipStream_t st, int u8) {
  const int N = geom[0], D = geom[1], H = geom[2], W = geom[3], C = geom[4];
  const int sd = geom[5], sh = geom[6], sw = geom[7], D2 = geom[8], H2 = geom[9], W2 = geom[10];
  const int CO = geom[11];
  const int pd = glen >= 15 ? geom[12] : 0, ph = glen >= 15 ? geom[13] : 0, pw = glen >= 15 ? geom[14] : 0;
  if (CO % 8 != 0 || sd * sh * sw * C > CO || pd < 0 || ph < 0 || pw < 0 || pd >= sd * D2 || ph >= sh * H2 ||
      pw >= sw * W2)
    return -2;
  const long long npos = (long long)N * D2 * H2 * W2;
  const unsigned blocks = (unsigned)((npos + 255) / 256);
  if (u8)
    hipLaunchKernelGGL(s2d_pack_kernel<unsigned char>, dim3(blocks), dim3(256), 0, st, (const unsigned char*)x,
                       (bf16*)out, N, D, H, W, C, sd, sh, sw, D2, H2, W2, CO, pd, ph, pw);
  else
    hipLaunchKernelGGL(s2d_pack_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (const bf16*)x, (bf16*)out, N, D, H, W,
                       C, sd, sh, sw, D2, H2, W2, CO, pd, ph, pw);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// space-to-depth weight map (one launch instead of pad + permute copies)
// ---------------------------------------------------------------------------
// w [K][KD][KH][KW][C] (the strided conv) <-> w2 [K][kd][kh][kw][CO] (the stride-1 conv over
// the packed input): w2[k][i][j][l][((a*sh + b)*sw + c)*C + ci] = w[k][i*sd+a][j*sh+b][l*sw+c][ci]
// (zero for taps past KD/KH/KW and channels past sd*sh*sw*C).  dir 0 writes w2 from w
// (forward), dir 1 writes w from w2 (the gradient back onto the strided conv's weight).
__global__ __launch_bounds__(256) void s2d_weight_map_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                             int K, int KD, int KH, int KW, int C, int sd, int sh,
                                                             int sw, int kd, int kh, int kw, int CO, int dir) {
  const long long total = dir == 0 ? (long long)K * kd * kh * kw * CO : (long long)K * KD * KH * KW * C;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  if (dir == 0) {
    long long r = i;
    const int c2 = (int)(r % CO); r /= CO;
    const int l = (int)(r % kw); r /= kw;
    const int j = (int)(r % kh); r /= kh;
    const int ii = (int)(r % kd);
    const int k = (int)(r / kd);
    float v = 0.f;
    if (c2 < sd * sh * sw * C) {
      const int ci = c2 % C, q = c2 / C;
      const int c = q % sw, b = (q / sw) % sh, a = q / (sw * sh);
      const int zd = ii * sd + a, zh = j * sh + b, zw = l * sw + c;
      if (zd < KD && zh < KH && zw < KW) v = src[((((long long)k * KD + zd) * KH + zh) * KW + zw) * C + ci];
    }
    dst[i] = v;
  } else {
    long long r = i;
    const int ci = (int)(r % C); r /= C;
    const int zw = (int)(r % KW); r /= KW;
    const int zh = (int)(r % KH); r /= KH;
    const int zd = (int)(r % KD);
    const int k = (int)(r / KD);
    const int c2 = (((zd % sd) * sh + zh % sh) * sw + zw % sw) * C + ci;
    dst[i] = src[((((long long)k * kd + zd / sd) * kh + zh / sh) * kw + zw / sw) * CO + c2];
  }
}

// ---------------------------------------------------------------------------
// sub-pixel decoder weight maps (ops/subpixel.py: conv3^3_same(upsample2x(x)) as 8 parity-class
// 2^3 convs).  1-D selections, per dimension: forward S[j][e][t] = 1 iff e = floor((j + t - 1) / 2)
// - (j - 1) (parity j output, low-res offset e, full-res tap t); dgrad D[e][j'][t] = 1 iff
// 0 <= 2e + j' + t - 2 <= 1 (shifted cell offset e, sub-position j').  One launch per map instead
// of an einsum (a hipBLASLt GEMM and its copies) plus a contiguous copy per class:
//   mode 0  wf [8 classes (jd,jh,jw)][K][8 offsets (ed,eh,ew)][C] = sum_t S S S w[K][3][3][3][C]
//   mode 1  wd [C][8 offsets][8 sub-positions (jd,jh,jw)][K]     = sum_t D D D w
//   mode 2  dW [K][3][3][3][C] = sum over classes and offsets of S S S dwf[8][K][8][C] (mode 0's
//           adjoint, the per-class weight gradients folded back)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool sp_sel_fwd(int j, int e, int t) { return e == ((j + t - 1) >> 1) - (j - 1); }
__device__ __forceinline__ bool sp_sel_dgrad(int e, int j, int t) {
  const int v = 2 * e + j + t - 2;
  return v >= 0 && v <= 1;
}

__global__ __launch_bounds__(256) void subpixel_wmap_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                            int K, int C, int mode) {
  const long long total = mode == 2 ? 27LL * K * C : 64LL * K * C;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  float v = 0.f;
  if (mode == 0) {
    long long r = i / C;
    const int e = (int)(r % 8); r /= 8;
    const int k = (int)(r % K);
    const int j = (int)(r / K);
    const int jd = j >> 2, jh = (j >> 1) & 1, jw = j & 1, ed = e >> 2, eh = (e >> 1) & 1, ew = e & 1;
    for (int x = 0; x < 3; ++x) {
      if (!sp_sel_fwd(jd, ed, x)) continue;
      for (int y = 0; y < 3; ++y) {
        if (!sp_sel_fwd(jh, eh, y)) continue;
        for (int z = 0; z < 3; ++z)
          if (sp_sel_fwd(jw, ew, z)) v += src[(((long long)k * 3 + x) * 3 + y) * 3 * C + (long long)z * C + c];
      }
    }
  } else if (mode == 1) {
    // dst[c][e][j][k]: the fastest index is k here
    const int k = (int)(i % K);
    long long r = i / K;
    const int j = (int)(r % 8); r /= 8;
    const int e = (int)(r % 8);
    const int ci = (int)(r / 8);
    const int jd = j >> 2, jh = (j >> 1) & 1, jw = j & 1, ed = e >> 2, eh = (e >> 1) & 1, ew = e & 1;
    for (int x = 0; x < 3; ++x) {
      if (!sp_sel_dgrad(ed, jd, x)) continue;
      for (int y = 0; y < 3; ++y) {
        if (!sp_sel_dgrad(eh, jh, y)) continue;
        for (int z = 0; z < 3; ++z)
          if (sp_sel_dgrad(ew, jw, z)) v += src[(((long long)k * 3 + x) * 3 + y) * 3 * C + (long long)z * C + ci];
      }
    }
    dst[i] = v;
    return;
  } else {
    long long r = i / C;
    const int t = (int)(r % 27);
    const int k = (int)(r / 27);
    const int x = t / 9, y = (t / 3) % 3, z = t % 3;
    for (int j = 0; j < 8; ++j) {
      const int jd = j >> 2, jh = (j >> 1) & 1, jw = j & 1;
      for (int e = 0; e < 8; ++e) {
        const int ed = e >> 2, eh = (e >> 1) & 1, ew = e & 1;
        if (sp_sel_fwd(jd, ed, x) && sp_sel_fwd(jh, eh, y) && sp_sel_fwd(jw, ew, z))
          v += src[(((long long)j * K + k) * 8 + e) * C + c];
      }
    }
  }
  dst[i] = v;
}

extern "C" int fn_subpixel_wmap(const float* src, float* dst, int K, int C, int mode, hipStream_t st) {
  if (K < 1 || C < 1 || mode < 0 || mode > 2) return -2;
  const long long total = mode == 2 ? 27LL * K * C : 64LL * K * C;
  hipLaunchKernelGGL(subpixel_wmap_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, dst, K, C,
                     mode);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_s2d_weight_map(const float* src, float* dst, const int* geom13, int dir, hipStream_t st) {
  const int K = geom13[0], KD = geom13[1], KH = geom13[2], KW = geom13[3], C = geom13[4];
  const int sd = geom13[5], sh = geom13[6], sw = geom13[7], kd = geom13[8], kh = geom13[9], kw = geom13[10];
  const int CO = geom13[11];
  if (sd * sh * sw * C > CO || kd * sd < KD || kh * sh < KH || kw * sw < KW || (dir != 0 && dir != 1)) return -2;
  const long long total = dir == 0 ? (long long)K * kd * kh * kw * CO : (long long)K * KD * KH * KW * C;
  hipLaunchKernelGGL(s2d_weight_map_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, dst, K, KD,
                     KH, KW, C, sd, sh, sw, kd, kh, kw, CO, dir);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// weight packing for the halo kernels (one launch instead of zero-fill + copies)
// ---------------------------------------------------------------------------
// w: fp32 [K][T][C] (the conv weight, taps kd-kh-kw major); the layouts: pack_w.h halo_pack_val
__global__ __launch_bounds__(256) void halo_pack_w_kernel(const float* __restrict__ w, bf16* __restrict__ out, int K0,
                                                          int C0, int K, int T, int C, int CS, int Tp, int mode) {
  const long long total = (long long)K * C * Tp;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  out[i] = f2bf(halo_pack_val(w, K0, C0, K, T, C, CS, Tp, mode, i));
}

// w: [K0][T][C0] fp32 (K0 <= K, C0 <= C)
extern "C" int fn_halo_pack_w(const float* w, void* out, int K0, int C0, int K, int T, int C, int mode, int stage_k,
                              hipStream_t st) {
  const int Csrc = mode == 0 ? C : K;
  const int CS = Csrc % 16 == 0 ? 16 : (Csrc % 8 == 0 ? 8 : 0);
  if (CS == 0 || stage_k % CS || K0 <= 0 || C0 <= 0 || K0 > K || C0 > C) return -2;
  const int tps = stage_k / CS;
  const int Tp = (T + tps - 1) / tps * tps;
  const long long total = (long long)K * C * Tp;
  hipLaunchKernelGGL(halo_pack_w_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, (bf16*)out, K0, C0,
                     K, T, C, CS, Tp, mode);
  FN_CHECK_LAUNCH();
  return 0;
}
