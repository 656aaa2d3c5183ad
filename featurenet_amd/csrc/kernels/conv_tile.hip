// Big-tile LDS-halo implicit-GEMM convolution (stride 1, 3-D) -- forward and dgrad.
//
// Successor of conv_halo.hip for the wide-channel FeatureNet-3D layers.  Where
// conv_halo runs 8 waves on <= 256-row tiles with 16-channel halo slices, a
// double-buffered 128-k weight stage in LDS (one barrier per stage) and a
// mostly synchronous halo reload per job, this kernel is built around ONE wave
// per SIMD:
//
//   * workgroup = 4 waves, each owning 16*MT output rows (MT = 8..10) x all
//     NT*16 columns of the workgroup: 512-640-row tiles (cubic-ish output
//     blocks, 2-4x less halo overhead than conv_halo's plane slabs);
//   * the input halo of a CS-channel slice of a tile ("job") sits in one of two
//     LDS buffers; the NEXT job's halo streams into the other buffer by LDS-DMA
//     (global_load_lds_dwordx4, one wave-instruction per k-step, zero page for
//     padding) while the current job computes -- the only barriers are one per
//     job (plus the epilogue's);
//   * weights never touch LDS: pre-packed in MFMA-fragment order
//     ([slice][k-step][16-col tile][lane][8]) and streamed global -> VGPRs by
//     every wave (1 KB per fragment, L1/L2 hits), PD k-steps ahead in a register
//     ring;
//   * A-fragment reads are bank-conflict free: the halo is stored chunk-planar
//     (16-B chunk c of position p at c*PLANE + 16p, PLANE a multiple of 1 KB), so
//     the bank slot of a read is p mod 16, and the host permutes the tile rows
//     (rowtab) so that the 16 rows of every MFMA fragment have 16 distinct halo
//     positions mod 16: every ds_read_b128 lane group touches 16 distinct slots;
//   * per-k-step LDS offsets come from a scalar tap walker, not a table (a
//     scalar load shares lgkmcnt with the ds_reads and would drain them).
//
// MFMA: v_mfma_f32_16x16x32_bf16.  A = halo rows (lane: row lr, 8 k of group lg),
// B = weights, k-step = 32 k = one tap x 32 channels (CS >= 32) or two taps x 16
// channels (CS = 16).  Epilogue: fp32 acc (+bias) -> bf16 staged in LDS in natural
// tile order -> activation -> 16-B stores; optional BN statistics (per workgroup
// column sums of the bf16 outputs).
//
// Dgrad uses the same kernel: dx = conv(dy, flip(W)^T) with leading pads K-1-p.
#include "common.h"

struct TileGeom {
  int N, ID, IH, IW, C;     // gathered source (x for fwd, dy for dgrad), channels-last
  int OD, OH, OW;           // output dims
  int KD, KH, KW;           // kernel
  int pd, ph, pw;           // leading pads (stride 1)
  int TD, TH, TW;           // output tile
  int CS;                   // channels per halo slice (jobs per tile = C / CS)
  int HPpad;                // halo positions rounded up to a multiple of 64 (whole DMA rows)
  int nks;                  // k-steps per job (multiple of the B prefetch depth)
  int nct;                  // 16-column tiles of the packed weights (ceil(Ncol / 16))
  unsigned mHW, mHHW;       // magic multipliers: p / HW == umulhi(p, mHW) (host-verified)
  int BUF;                  // bytes per LDS buffer (halo or epilogue staging), multiple of 16
};

__device__ __forceinline__ void tile_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#define CT_NTHR 256

// LDS-DMA of one 16-B chunk per lane into lds_dst + 16 * lane (lds_dst wave-uniform).
// Inline asm (M0 saved/restored in the same statement), so hipcc does not count it:
// its waitcnt pass drains vmcnt(0) at every use of an ordinary load while a counted
// LDS-DMA is in flight.  The kernel waits for these with explicit vmcnt counts.
__device__ __forceinline__ void ct_glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// 16-B global load into a B fragment, hidden from hipcc's waitcnt bookkeeping (see
// ct_glds16): uniform base in SGPRs + per-lane byte offset; completion is waited by
// ct_wait_b with an explicit count
template <int IMM>
__device__ __forceinline__ void ct_gload16(bf16x8& dst, const void* sbase, unsigned voff) {
  asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(dst) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}

__device__ __forceinline__ unsigned ct_lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

template <int MT, int NT, int CPP>
__global__ __launch_bounds__(CT_NTHR, 1) void conv_tile_kernel(const bf16* __restrict__ src,
                                                               const uint4* __restrict__ wp,
                                                               const int2* __restrict__ rowtab,
                                                               const bf16* __restrict__ zp,
                                                               const float* __restrict__ bias, bf16* __restrict__ out,
                                                               float* __restrict__ stats, TileGeom g, int Ncol,
                                                               int act, int* __restrict__ sched) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  constexpr int PD = NT == 2 ? 4 : 3;            // B prefetch depth (k-steps in flight)
  constexpr int LDO = NT * 16 + 8;               // epilogue staging row pitch (bf16)
  constexpr int CPR = NT * 2;                    // 16-B chunks per output row

  const int HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1, HD = g.TD + g.KD - 1;
  const int HP = HD * HH * HW;
  const int PLANE = g.HPpad * 16;                // bytes per 16-B chunk plane
  const int rows = g.TD * g.TH * g.TW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH, twn = (g.OW + g.TW - 1) / g.TW;
  const int ntiles = g.N * tdn * thn * twn;
  const int nslice = g.C / g.CS;
  const int nks = g.nks;
  const int T = g.KD * g.KH * g.KW;
  const int prow = g.HPpad / 64;                 // DMA rows (64 positions) per chunk plane
  const int NQ = CPP * prow;                     // DMA wave-instructions per job halo

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int ct0 = blockIdx.y * NT;               // first 16-column tile of this workgroup
  // LDS: [halo / staging buffer 0][buffer 1][grab slot, 64 B][1 KB DMA scratch row][row map]
  int* s_grab = reinterpret_cast<int*>(dsm + 2 * g.BUF);
  int* s_orow = reinterpret_cast<int*>(dsm + 2 * g.BUF + 64 + 1024);   // natural tile row of every MFMA row
  for (int i = tid; i < 4 * MT * 16; i += CT_NTHR) s_orow[i] = rowtab[i].y;
  float bcol[NT];                                // bias of this lane's epilogue columns
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int gcol = (blockIdx.y * NT + nt) * 16 + (threadIdx.x & 15);
    bcol[nt] = (bias && gcol < Ncol) ? bias[gcol] : 0.f;
  }

  // ---- per-lane constants -------------------------------------------------
  int lbase[MT];                                 // LDS byte offset of the row's tap-(0,0,0) chunk
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int2 rt = rowtab[(wave * MT + mt) * 16 + lr];
    lbase[mt] = rt.x * 16 + (CPP >= 4 ? lg : (lg & 1)) * PLANE;
  }

  // ---- tile schedule (dynamic, one tile per grab; see conv_halo.hip) ------
  auto grab = [&]() -> int {
    if (tid == 0) *s_grab = atomicAdd(sched + 1 + blockIdx.y, 1);
    tile_lds_barrier();
    const int t = __builtin_amdgcn_readfirstlane(*s_grab);
    tile_lds_barrier();
    return t < ntiles ? t : -1;
  };

  // ---- halo DMA ---------------------------------------------------------------
  struct Org { const bf16* base; int dlo, hlo, wlo; };
  auto job_org = [&](int tile, int slice) -> Org {
    int t = tile;
    const int tw = t % twn; t /= twn;
    const int th = t % thn; t /= thn;
    const int td = t % tdn;
    const int n = t / tdn;
    Org o;
    o.dlo = td * g.TD - g.pd;
    o.hlo = th * g.TH - g.ph;
    o.wlo = tw * g.TW - g.pw;
    o.base = src + (long long)n * g.ID * g.IH * g.IW * g.C + slice * g.CS;
    return o;
  };
  // DMA row q of a job halo (wave-uniform): chunk plane c = q / prow, positions
  // p0 .. p0+63; lane l moves position p0 + l (zero page outside the input).  Rows
  // q >= NQ are dummies (zero page -> the scratch row past both buffers) so that every
  // k-step issues exactly one DMA and the explicit vmcnt counts stay constant.
  const unsigned lds_base = ct_lds_addr(dsm);
  auto dma_row = [&](const Org& o, int bufoff, int q) {
    const bool live = q < NQ;
    const int qq = live ? q : 0;
    const int c = qq / prow;
    const int p0 = (qq - c * prow) * 64;
    const int p = p0 + lane;
    const int hd = (int)__umulhi((unsigned)p, g.mHHW);
    const int rem = p - hd * HH * HW;
    const int hh = (int)__umulhi((unsigned)rem, g.mHW);
    const int hw = rem - hh * HW;
    const int gd = o.dlo + hd, gh = o.hlo + hh, gw = o.wlo + hw;
    const bool ok = live && p < HP && (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
                    (unsigned)gw < (unsigned)g.IW;
    const bf16* gsrc = ok ? o.base + ((gd * g.IH + gh) * g.IW + gw) * g.C + c * 8 : zp;
    const unsigned dst = lds_base + (live ? (unsigned)(bufoff + c * PLANE + p0 * 16) : (unsigned)(2 * g.BUF + 64));
    ct_glds16(gsrc, __builtin_amdgcn_readfirstlane(dst));
  };

  // ---- accumulators and operand registers ---------------------------------
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[MT];                                 // rotating: fragment mt of k-step k+1 is read right
                                                 // after the NT MFMAs of (mt, k) consumed it
  bf16x8 fb[PD][NT];

  const uint4* wjob = wp;                        // this job's first k-step (uniform)
  const int wstride = g.nct * 64;                // uint4 per k-step
  auto load_b = [&](int ks, int slot) {
    const int k = ks < nks ? ks : nks - 1;       // past the end: a redundant (never used) load
    const uint4* p = wjob + k * wstride;
    ct_gload16<0>(fb[slot][0], p, lane * 16);
    ct_gload16<1024>(fb[slot][1], p, lane * 16);
    if constexpr (NT == 4) {
      ct_gload16<2048>(fb[slot][2], p, lane * 16);
      ct_gload16<3072>(fb[slot][3], p, lane * 16);
    }
  };
  // wait until ring slot `slot` has landed: per k-step the kernel issues NT B loads then
  // one DMA row, so the loads younger than slot's are that DMA + (PD-1) whole k-steps
  constexpr int VM_B = 1 + (PD - 1) * (NT + 1);
  auto wait_b = [&](int slot) {
    if constexpr (NT == 2) {
      asm volatile("s_waitcnt vmcnt(%2)" : "+v"(fb[slot][0]), "+v"(fb[slot][1]) : "n"(VM_B));
    } else {
      asm volatile("s_waitcnt vmcnt(%4)"
                   : "+v"(fb[slot][0]), "+v"(fb[slot][1]), "+v"(fb[slot][2]), "+v"(fb[slot][3])
                   : "n"(VM_B));
    }
  };

  // scalar tap walker: LDS offset of the k-step for this lane, then advance one k-step
  constexpr int SUB = CPP >= 4 ? CPP / 4 : 1;    // k-steps per tap (32 channels each)
  struct Walk { int t, kw, kh, kd, sub; };
  auto tap_next = [&](Walk& w) {                 // branch-free (selects), so the waitcnt pass
    ++w.t;                                       // keeps exact counts across k-steps
    const int kw1 = w.kw + 1;
    const bool c1 = kw1 == g.KW;
    w.kw = c1 ? 0 : kw1;
    const int kh1 = w.kh + (c1 ? 1 : 0);
    const bool c2 = kh1 == g.KH;
    w.kh = c2 ? 0 : kh1;
    w.kd += c2 ? 1 : 0;
  };
  auto tap_off = [&](const Walk& w) -> int {    // byte offset of the walker's tap (0 past the last tap)
    return w.t < T ? ((w.kd * HH + w.kh) * HW + w.kw) * 16 : 0;
  };
  auto kofs_next = [&](Walk& w) -> int {
    int ko;
    if constexpr (CPP >= 4) {
      ko = tap_off(w) + w.sub * 4 * PLANE;
      if constexpr (SUB == 1) {
        tap_next(w);
      } else {
        const int s1 = w.sub + 1;
        if (s1 == SUB) { w.sub = 0; tap_next(w); } else { w.sub = s1; }
      }
    } else {                                     // CS = 16: lanes lg < 2 tap 2ks, lg >= 2 tap 2ks+1
      const int lo = tap_off(w);
      tap_next(w);
      const int hi = tap_off(w);
      tap_next(w);
      ko = lg < 2 ? lo : hi;
    }
    return ko;
  };
  Walk walk;
  int bufoff = 0;
  // MFMAs of the current k-step from ring slot `slot`; fragment mt of the next k-step
  // is read right after its own NT MFMAs.  sched_barrier pins that order: left
  // alone, hipcc sinks every read to just before its MFMA (exposing the LDS latency)
  // and every ring refill to the end of the turn (exposing the L2 latency).
  auto kstep = [&](int slot) {
    const int ko = kofs_next(walk) + bufoff;
    wait_b(slot);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[slot][nt], acc[mt][nt], 0, 0, 0);
      fa[mt] = *(const bf16x8*)(dsm + lbase[mt] + ko);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  int tile = grab();
  int slice = 0;
  if (tile >= 0) {
    const Org o = job_org(tile, 0);
    for (int q = wave; q < NQ; q += 4) dma_row(o, 0, q);
  }
  while (tile >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA rows of the job halo
    tile_lds_barrier();                                 // ... and everyone's; previous buffer free
    // next job: next slice of this tile, or a new tile
    int ntile = tile, nslc = slice + 1;
    if (nslc == nslice) {
      nslc = 0;
      ntile = grab();
    }
    const Org no = job_org(ntile >= 0 ? ntile : 0, nslc);
    const int nq = ntile >= 0 ? NQ : 0;          // live DMA rows of the next job's halo
    const int nbuf = bufoff ^ g.BUF;
    wjob = wp + ((size_t)slice * nks * g.nct + ct0) * 64;
    int q = nq > 0 ? wave : NQ;                  // next DMA row of this wave (NQ.. = dummies)
    // ring prologue: each load followed by one DMA row, the pattern of every k-step, so
    // wait_b's constant count holds from the first k-step on
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      load_b(u, u);
      dma_row(no, nbuf, q);
      q += 4;
    }
    walk.t = walk.kw = walk.kh = walk.kd = walk.sub = 0;
    {
      const int ko = kofs_next(walk) + bufoff;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) fa[mt] = *(const bf16x8*)(dsm + lbase[mt] + ko);
    }
    for (int ks = 0; ks < nks; ks += PD) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        kstep(u);
        load_b(ks + u + PD, u);
        dma_row(no, nbuf, q);
        q += 4;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    for (; q < nq; q += 4) dma_row(no, nbuf, q);  // short jobs: the rest of the next halo

    if (slice == nslice - 1) {
      // ---- epilogue: acc -> (bias) -> bf16 staging -> act -> 16-B stores (+BN stats) ----
      int t = tile;
      const int tw_i = t % twn; t /= twn;
      const int th_i = t % thn; t /= thn;
      const int td_i = t % tdn;
      const int n = t / tdn;
      const int d0 = td_i * g.TD, h0 = th_i * g.TH, w0 = tw_i * g.TW;
      tile_lds_barrier();                        // all waves are done reading this job's halo
      bf16* Os = reinterpret_cast<bf16*>(dsm + bufoff);
      // dummy rows write row 64*MT, a scratch row past the tile
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int4 o4 = *(const int4*)(s_orow + (wave * MT + mt) * 16 + lg * 4);   // rows 4lg .. 4lg+3
        const int orow[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int col = nt * 16 + lr;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int orr = orow[r] >= 0 ? orow[r] : 64 * MT;
            Os[orr * LDO + col] = f2bf(acc[mt][nt][r] + bcol[nt]);
          }
          acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
      tile_lds_barrier();
      const long long obase = (long long)n * g.OD * g.OH * g.OW;
      const int ch = tid % CPR;                  // fixed per thread (CT_NTHR % CPR == 0)
      const int gc = ct0 * 16 + ch * 8;
      float st_s[8], st_q[8];                    // this tile's BN partial sums of the thread's 8 columns
#pragma unroll
      for (int j = 0; j < 8; ++j) st_s[j] = st_q[j] = 0.f;
      for (int idx = tid; idx < rows * CPR; idx += CT_NTHR) {
        const int r = idx / CPR;
        const int tw = r % g.TW, th = (r / g.TW) % g.TH, td = r / (g.TW * g.TH);
        if (d0 + td >= g.OD || h0 + th >= g.OH || w0 + tw >= g.OW) continue;
        const long long m = obase + ((long long)(d0 + td) * g.OH + h0 + th) * g.OW + w0 + tw;
        Pack8 v;
        v.u = *(const uint4*)(Os + r * LDO + ch * 8);
        if (act != ACT_NONE) {
          for (int j = 0; j < 8; ++j) v.e[j] = f2bf(act_fwd(bf2f(v.e[j]), act));
        }
        if (stats) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = bf2f(v.e[j]);
            st_s[j] += f;
            st_q[j] += f * f;
          }
        }
        if (gc + 8 <= Ncol && (Ncol & 7) == 0) {
          *(uint4*)(out + m * Ncol + gc) = v.u;
        } else {
          for (int j = 0; j < 8; ++j)
            if (gc + j < Ncol) out[m * Ncol + gc + j] = v.e[j];
        }
      }
      if (stats) {
        // per-tile column reduction in LDS, folded into this workgroup's slab row (it
        // owns the row: plain read-modify-write; the caller zeroes the slab)
        tile_lds_barrier();
        float* red = reinterpret_cast<float*>(dsm + bufoff);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red[tid * 16 + j] = st_s[j];
          red[tid * 16 + 8 + j] = st_q[j];
        }
        tile_lds_barrier();
        if (tid < NT * 16) {
          const int c8 = tid / 8, j = tid % 8;   // column tid = c8 * 8 + j
          float s = 0.f, qq = 0.f;
          for (int u = c8; u < CT_NTHR; u += CPR) {
            s += red[u * 16 + j];
            qq += red[u * 16 + 8 + j];
          }
          const int gcol = ct0 * 16 + tid;
          if (gcol < Ncol) {
            stats[(long long)blockIdx.x * 2 * Ncol + gcol] += s;
            stats[(long long)blockIdx.x * 2 * Ncol + Ncol + gcol] += qq;
          }
        }
      }
    }
    tile = ntile;
    slice = nslc;
    bufoff = nbuf;
  }

  if (tid == 0) {                                // the last workgroup out resets the counters
    __threadfence();
    if (atomicAdd(sched, 1) == (int)(gridDim.x * gridDim.y) - 1) {
      for (int i = 0; i < (int)gridDim.y; ++i) atomicExch(sched + 1 + i, 0);
      atomicExch(sched, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// weight packing: conv weight [K][T][C] (fp32) -> MFMA B fragments
// ---------------------------------------------------------------------------
// out[((slice * nks + ks) * nct + ct) * 64 + lane][j] (8 bf16 per lane) =
//   Wsrc[col = ct*16 + (lane & 15)][tap][ch], k-step ks of slice:
//     CS >= 32: tap = ks / (CS/32), ch = slice*CS + (ks % (CS/32))*32 + (lane>>4)*8 + j
//     CS == 16: tap = 2*ks + (lane>>5), ch = slice*16 + ((lane>>4)&1)*8 + j
//   forward: Wsrc[col][tap][ch] = w[col][tap][ch]          (Ncol = K, Csrc = C)
//   dgrad:   Wsrc[col][tap][ch] = w[ch][T-1-tap][col]      (Ncol = C, Csrc = K)
// zero for tap >= T or col >= Ncol.
__global__ __launch_bounds__(256) void tile_pack_w_kernel(const float* __restrict__ w, uint4* __restrict__ out, int K,
                                                          int T, int C, int CS, int nks, int nct, int nslice,
                                                          int dgrad) {
  const long long total = (long long)nslice * nks * nct * 64;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int lane = (int)(i % 64);
  long long r = i / 64;
  const int ct = (int)(r % nct);
  r /= nct;
  const int ks = (int)(r % nks);
  const int slice = (int)(r / nks);
  const int Ncol = dgrad ? C : K;
  const int col = ct * 16 + (lane & 15);
  int tap, ch0;
  if (CS >= 32) {
    const int sub = CS / 32;
    tap = ks / sub;
    ch0 = slice * CS + (ks % sub) * 32 + (lane >> 4) * 8;
  } else {
    tap = 2 * ks + (lane >> 5);
    ch0 = slice * 16 + ((lane >> 4) & 1) * 8;
  }
  Pack8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float f = 0.f;
    if (tap < T && col < Ncol) {
      const int ch = ch0 + j;
      f = dgrad ? w[((long long)ch * T + (T - 1 - tap)) * C + col] : w[((long long)col * T + tap) * C + ch];
    }
    v.e[j] = f2bf(f);
  }
  out[i] = v.u;
}

extern "C" int fn_tile_pack_w(const float* w, void* out, int K, int T, int C, int CS, int nks, int nct, int nslice,
                              int dgrad, hipStream_t st) {
  if (CS != 16 && CS % 32 != 0) return -2;
  const long long total = (long long)nslice * nks * nct * 64;
  hipLaunchKernelGGL(tile_pack_w_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, (uint4*)out, K, T,
                     C, CS, nks, nct, nslice, dgrad);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------
#define CT_GEOM_LEN 24
static TileGeom parse_tile(const int* v) {
  TileGeom g;
  g.N = v[0]; g.ID = v[1]; g.IH = v[2]; g.IW = v[3]; g.C = v[4];
  g.OD = v[5]; g.OH = v[6]; g.OW = v[7];
  g.KD = v[8]; g.KH = v[9]; g.KW = v[10];
  g.pd = v[11]; g.ph = v[12]; g.pw = v[13];
  g.TD = v[14]; g.TH = v[15]; g.TW = v[16];
  g.CS = v[17]; g.HPpad = v[18]; g.nks = v[19]; g.nct = v[20];
  g.mHW = (unsigned)v[21]; g.mHHW = (unsigned)v[22]; g.BUF = v[23];
  return g;
}

static int g_tile_cus = 0;

extern "C" int fn_conv_tile_workers(const int* geom, int Ncol, int NT) {
  const TileGeom g = parse_tile(geom);
  if (g_tile_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_tile_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_tile_cus <= 0)
      g_tile_cus = 256;
  }
  const int ncb = (Ncol + NT * 16 - 1) / (NT * 16);
  const int ntiles = g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) * ((g.OW + g.TW - 1) / g.TW);
  const int w = (g_tile_cus + ncb - 1) / ncb;
  return w > ntiles ? ntiles : w;
}

template <int MT, int NT, int CPP>
static int launch_tile(dim3 grid, size_t lds, hipStream_t st, const bf16* s, const uint4* w, const int2* rt,
                       const bf16* zp, const float* b, bf16* o, float* stats, const TileGeom& g, int Ncol, int act,
                       int* sched) {
  static size_t configured = 0;
  if (lds > configured) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_tile_kernel<MT, NT, CPP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    configured = lds;
  }
  hipLaunchKernelGGL((conv_tile_kernel<MT, NT, CPP>), grid, dim3(CT_NTHR), lds, st, s, w, rt, zp, b, o, stats, g,
                     Ncol, act, sched);
  return 0;
}

// instantiations (MT, NT, CPP) -- the Python planner only emits these
#define CT_INSTANCES(X) \
  X(8, 2, 2) X(9, 2, 2) X(10, 2, 2) X(8, 2, 4) X(9, 2, 4) X(10, 2, 4) \
  X(8, 4, 2) X(9, 4, 2) X(10, 4, 2) X(8, 4, 4) X(9, 4, 4) X(10, 4, 4)

extern "C" int fn_conv_tile_supported(int MT, int NT, int CPP) {
#define CT_SUP(M, N, C) if (MT == M && NT == N && CPP == C) return 1;
  CT_INSTANCES(CT_SUP)
#undef CT_SUP
  return 0;
}

// geom: halo geometry (17) + CS, HPpad, nks, nct, mHW, mHHW, BUF (see TileGeom).
// wp: packed weights (fn_tile_pack_w); rowtab: int2[4 * MT * 16] (halo position of the
// row, natural tile row or -1); zp: >= 16 zero bytes; sched: int[64] zeroed counters
// (left zero); stats: fp32 [workers][2][Ncol] zero-initialised, or null.
extern "C" int fn_conv_tile(const void* src, const void* wp, const void* rowtab, const void* zp, const float* bias,
                            void* out, float* stats, const int* geom, int Ncol, int act, int MT, int NT,
                            int* sched, hipStream_t st) {
  const TileGeom g = parse_tile(geom);
  if (g.CS != 16 && g.CS % 32 != 0) return -2;
  const int CPP = g.CS / 8;
  if (!fn_conv_tile_supported(MT, NT, CPP)) return -2;
  if (g.C % g.CS || g.TD * g.TH * g.TW > 64 * MT || g.TD < 1 || g.TH < 1 || g.TW < 1) return -3;
  const long long HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const long long HP = (g.TD + g.KD - 1) * HH * HW;
  if (g.HPpad < HP || g.HPpad % 64) return -3;
  const int PD = NT == 2 ? 4 : 3;
  const int T = g.KD * g.KH * g.KW;
  const int need_ks = g.CS >= 32 ? T * (g.CS / 32) : (T + 1) / 2;
  if (g.nks % PD || g.nks < need_ks || g.nct < (Ncol + 15) / 16) return -3;
  // the magic divisors must be exact for every position the DMA rows touch
  for (long long p = 0; p < g.HPpad; p += 1) {
    const unsigned long long hd = ((unsigned long long)p * g.mHHW) >> 32;
    const unsigned long long rem = p - hd * HH * HW;
    if (hd != (unsigned long long)(p / (HH * HW)) || (((rem * g.mHW) >> 32) != rem / HW)) return -3;
  }
  const size_t halo = (size_t)g.HPpad * CPP * 16;
  const size_t stage = (size_t)(64 * MT + 1) * (NT * 16 + 8) * 2;
  if ((size_t)g.BUF < halo || (size_t)g.BUF < stage || (size_t)g.BUF < (size_t)CT_NTHR * 64 || g.BUF % 16) return -3;
  const size_t lds = 2 * (size_t)g.BUF + 64 + 1024 + 4 * 64 * MT * 4;
  if (lds > 160 * 1024) return -4;
  const int ncb = (Ncol + NT * 16 - 1) / (NT * 16);
  if (!sched || !zp || ncb > 63 || ncb * NT > g.nct) return -6;
  dim3 grid((unsigned)fn_conv_tile_workers(geom, Ncol, NT), (unsigned)ncb);
  int rc = -2;
#define CT_CASE(M, N, C)                                                                                          \
  if (MT == M && NT == N && CPP == C)                                                                             \
    rc = launch_tile<M, N, C>(grid, lds, st, (const bf16*)src, (const uint4*)wp, (const int2*)rowtab,            \
                              (const bf16*)zp, bias, (bf16*)out, stats, g, Ncol, act, sched);
  CT_INSTANCES(CT_CASE)
#undef CT_CASE
  if (rc) return rc;
  FN_CHECK_LAUNCH();
  return 0;
}
