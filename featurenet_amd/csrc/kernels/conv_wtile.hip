// Weight gradient of a stride-1 3-D convolution on big tiles with a loader wave.
//
//   dW[co][tap][ci] = sum over output positions p of dy[p][co] * x[p + tap][ci]
//
// The MFMA K axis is the output positions of a tile, so both operands are read from
// LDS "transposed" (ds_read_b64_tr_b16: each lane names one position row and 4
// channels; a pair of reads gives the 8 k-values of a 16x16x32 bf16 fragment):
//   A = dy^T  (16 output channels x 32 positions), MT fragments per k-step
//   B = x     (32 positions x 16 input channels) at tap offset t, NACC fragments
// and a wave accumulates MT x NACC 16x16 blocks: all Cout rows x NACC taps of one
// 16-channel input slice, over every tile its workgroup processes; the blocks are
// stored into this workgroup's partial dW once, at the end (summed in a fixed order by
// wtile_reduce_kernel).
//
// Structure (as conv_tile.hip): one workgroup per CU = 4 MFMA waves (one per SIMD) + 1
// loader wave.  A job is one output tile; its x halo (the slice's 16 channels, 32 B per
// position, position-major) and its dy rows (all Cout channels) are LDS-DMA'd by the
// loader into one of two buffers while the compute waves run the other -- one barrier
// per job.  Bank-conflict-free transposed reads:
//   * x: a 32-lane half reads 8 rows x 4 channel quads at 32*pos + 8*quad -- conflict free
//     when the 8 rows' halo positions are distinct mod 8; the host orders each aligned
//     group of 8 k-rows so (rowtab, the same order for dy and x);
//   * dy: rows of Cout*2 bytes with the 16-B chunks XOR-swizzled per row (the DMA source
//     chunk of each LDS slot is permuted) so the 8 rows of a half land on 8 distinct bank
//     groups.
// Column groups (grid): tap groups (4 waves x NACC taps) x input slices.  Workgroups are
// XCD-aware: the G column-group workgroups of an XCD share that XCD's contiguous tile
// range (per-(XCD, group) counters), so a tile's dy and halo are fetched into one L2 and
// neighbouring tiles' overlapping halos stay there.
//
// Reference semantics: the weight gradient of Keras Conv3D (reference model/input.py:294
// via TF autodiff); the layout / schedule here is MI355X-specific.
#include "common.h"
#include "conv_tile_shared.h"
#include "tile_dma.h"

#include <cstdlib>

#define WT_GEOM_LEN 24
// NW = 4: 4 MFMA waves (one per SIMD) + 1 loader wave; NW = 8: 8 MFMA waves (two per SIMD,
// twice the VALU/LDS issue slots of a lone wave) that LDS-DMA each job's halo and dy rows
// themselves (1/8 each) -- no loader, and a workgroup covers twice the taps
__host__ __device__ constexpr int wt_nthr(int NW) { return NW == 4 ? 64 * 5 : 64 * NW; }

struct WGeom {
  int N, ID, IH, IW, C;      // x, channels-last
  int OD, OH, OW, K;         // dy dims and channels (Cout)
  int KD, KH, KW;
  int pd, ph, pw;            // leading pads
  int TD, TH, TW;            // output tile
  int HPpad;                 // halo positions, multiple of 32 (whole DMA instructions)
  int kst;                   // 32-row k-steps per tile
  int XB;                    // bytes of the x halo of a buffer (HPpad * 32)
  int BUF;                   // bytes per buffer (XB + kst * 32 * K * 2)
  int G;                     // column groups (ntg tap groups x C/16 slices)
  int ntg;                   // tap groups
};

typedef short wt_s4 __attribute__((ext_vector_type(4)));
typedef short wt_s8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 wt_tr_pair(const unsigned char* lo, const unsigned char* hi) {
  const wt_s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) wt_s4*)(lo));
  const wt_s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) wt_s4*)(hi));
  const wt_s8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int MT, int NACC, int NW, bool C8 = false, bool KS2 = false, bool SP = false>
__global__ __launch_bounds__(wt_nthr(NW), 1) void conv_wtile_kernel(const bf16* __restrict__ x,
                                                                const bf16* __restrict__ dy,
                                                                float* __restrict__ dw,   // partials
                                                                const int2* __restrict__ rowtab,
                                                                const int* __restrict__ postab,
                                                                const bf16* __restrict__ zp, WGeom g,
                                                                int* __restrict__ sched, int dbg,
                                                                const float* __restrict__ pst, int pact) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  constexpr int CO = MT * 16;
  // SP: the sub-pixel (upsample x2 + 3^3 conv) weight gradient.  Rows are low-resolution
  // cells; wave w is parity class j = (w>>2, (w>>1)&1, w&1) and accumulates the 8 folded
  // taps e of its class (low-res offsets j - 1 + e, inside a 3^3 footprint with pad 1) for
  // two 16-channel x slices (two halo planes: 16 fragments).  The dy rows in LDS hold all 8
  // classes (8 x 32 channels = 512 B per cell: full-resolution positions 2c + j, gathered
  // from the shifted space-to-depth dy, ops/subpixel.py); wave w reads its class's 64 B.
  static_assert(!SP || (NW == 8 && MT == 2 && NACC == 16 && !C8 && !KS2), "sub-pixel form");
  constexpr int CO_L = SP ? 256 : CO;            // dy channels per LDS row
  constexpr int CPR = CO_L / 8;                  // 16-B chunks per dy row
  constexpr int R64 = SP ? 1 : 256 / (CO * 2);   // dy rows per 64 banks
  constexpr int NSW = 8 / R64;                   // swizzle classes over 8 rows
  constexpr int XPL = SP ? 2 : 1;                // x halo planes (16-channel slices) per job
  constexpr int PF = NACC < 4 ? NACC : 4;       // B fragments in flight (register ring)
  // C8 (8-channel input, the space-to-depth stem): 16-B halo positions, and each 16-column
  // B fragment holds TWO taps x 8 channels (columns 0-7: tap 2i, 8-15: tap 2i + 1 of the
  // wave's range -- lanes 4q + 2, 4q + 3 of a transposed read address the second tap)
  static_assert(!C8 || NW == 8, "the 8-channel form is loaderless");
  constexpr int XR = C8 ? 16 : 32;               // halo bytes per position
  constexpr int XSH = C8 ? 0 : 1;                // DMA slot -> halo position shift
  constexpr int TPF = C8 ? 2 : 1;                // taps per B fragment
  // KS2: the k-steps of a job are split between the wave halves (waves 0-3 even, 4-7 odd
  // k-steps; a wave and its SIMD partner w + 4 in different halves), each half covering
  // all of the workgroup's taps with twice the fragments per wave: twice the MFMAs per
  // k-step for the per-k-step bookkeeping (short k-steps were issue-bound).  The halves
  // accumulate the same dW entries into separate partial slabs.
  static_assert(!KS2 || NW == 8, "k-step split: loaderless form");
  constexpr int WPT = KS2 ? NW / 2 : NW;         // waves sharing one k-step stream
  constexpr int KSTEP = KS2 ? 2 : 1;
  const int ROWS = g.kst * 32;
  const int HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const int T = g.KD * g.KH * g.KW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH, twn = (g.OW + g.TW - 1) / g.TW;
  const int ntiles = g.N * tdn * thn * twn;

  constexpr int NTHR = wt_nthr(NW);
  constexpr bool HAS_LOADER = NW == 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = HAS_LOADER && wave == NW;
  // XCD-aware decomposition of the 1-D grid (gridDim.x = 8 * G * workers per group)
  const int xcd = blockIdx.x & 7, lid = blockIdx.x >> 3;
  const int grp = lid % g.G;
  const int tg = grp % g.ntg, slice = grp / g.ntg;
  const int per = (ntiles + 7) / 8;
  const int t_lo = xcd * per, t_hi = min(ntiles, t_lo + per);

  // LDS: [buffer 0][buffer 1][s_job 64 B][rows int2 ROWS][positions int HPpad]
  //      [x offsets int HPpad][dy row offsets int ROWS]
  int* s_job = reinterpret_cast<int*>(dsm + 2 * g.BUF);
  int2* s_rows = reinterpret_cast<int2*>(dsm + 2 * g.BUF + 64);
  int* s_pos = reinterpret_cast<int*>(s_rows + ROWS);
  int* s_xoff = s_pos + g.HPpad;
  int* s_yoff = s_xoff + g.HPpad;
  for (int i = tid; i < ROWS; i += NTHR) {
    const int2 rt = rowtab[i];
    s_rows[i] = rt;
    // byte offset of the row's dy from the tile origin (interior tiles), -1 for a dummy row
    const int e = rt.y;
    if constexpr (SP)   // dy grid = the shifted space-to-depth cells, one more per dimension
      s_yoff[i] = e < 0 ? -1 : (((e >> 16) * (g.OH + 1) + ((e >> 8) & 255)) * (g.OW + 1) + (e & 255)) * CO_L * 2;
    else
      s_yoff[i] = e < 0 ? -1 : (((e >> 16) * g.OH + ((e >> 8) & 255)) * g.OW + (e & 255)) * CO * 2;
  }
  for (int i = tid; i < g.HPpad; i += NTHR) {
    const int e = postab[i];
    s_pos[i] = e;
    // byte offset of the position from the halo origin (interior tiles; 0 past the halo:
    // those slots are never read)
    s_xoff[i] = e < 0 ? 0 : (((e >> 16) * g.IH + ((e >> 8) & 255)) * g.IW + (e & 255)) * g.C * 2;
  }
  // ---- job protocol ---------------------------------------------------------
  // s_job[j % 3] = tile of job j (-1: done).  Jobs 0 and 1 are taken before the first
  // barrier; in iteration j (between barriers A(j) and A(j+1)) the loader takes job j+2's
  // tile and publishes it and LDS-DMAs job j+1's x halo into the free buffer, and the
  // compute waves -- after reading jobs j and j+1, before running job j -- DMA a quarter
  // each of job j+1's dy rows (one wave alone could not keep the LDS fed at this job
  // size; giving the compute waves part of the x halo as well measured slower).
  // Static round-robin tiles for both forms: job j of worker wid of this (XCD, group) is tile
  // t_lo + wid + j * nwk.  The workgroup's partial dW is then a sum over a fixed tile set in a
  // fixed order, and wtile_reduce_kernel adds the partials in a fixed order: the weight
  // gradient is bitwise the same run to run (no atomic round trip on any wave's critical path
  // either).  (The 4-wave loader form took tiles from a per-(XCD, group) counter through round
  // 4, which made its partials -- and dW -- depend on the dynamic schedule.)
  const int nwk = (int)(gridDim.x >> 3) / g.G, wid = lid / g.G;
  auto tile_of = [&](int j) -> int {
    const int t = t_lo + wid + j * nwk;
    return t < t_hi ? t : -1;
  };
  if constexpr (HAS_LOADER) {
    if (tid == 0) {
      s_job[0] = tile_of(0);
      s_job[1] = tile_of(1);
    }
  }
  tile_lds_barrier();

  auto decode = [&](int tile, int& n, int& d0, int& h0, int& w0) {
    int t = tile;
    const int tw = t % twn; t /= twn;
    const int th = t % thn; t /= thn;
    const int td = t % tdn;
    n = t / tdn;
    d0 = td * g.TD;
    h0 = th * g.TH;
    w0 = tw * g.TW;
  };
  // dy rows of job `tile` in k order, DMA instructions first, first + step, ... (8 in
  // flight): slot s = CPR * row + chunk slot, holding source chunk slot ^ swizzle(row)
  const int ny = (ROWS * CPR) >> 6;
  auto dma_dy = [&](int tile, int bufoff, int first, int step, int mlo = 0, int mhi = 1 << 20) {
    tile = __builtin_amdgcn_readfirstlane(tile);
    int n, d0, h0, w0;
    decode(tile, n, d0, h0, w0);
    const unsigned dst0 = ct_lds_addr(dsm) + (unsigned)bufoff + (unsigned)g.XB;
    const int YH = SP ? g.OH + 1 : g.OH, YW = SP ? g.OW + 1 : g.OW;
    const bf16* ys = dy + (long long)n * (SP ? g.OD + 1 : g.OD) * YH * YW * CO_L;
    const bool y_in = d0 + g.TD <= g.OD && h0 + g.TH <= g.OH && w0 + g.TW <= g.OW;
    const unsigned char* yo =
        reinterpret_cast<const unsigned char*>(ys + ((long long)(d0 * YH + h0) * YW + w0) * CO_L);
    const int jend = min((dbg & 8) ? 0 : ny, first + mhi * step);   // (dbg 8, timing only: no dy DMA)
    for (int j0 = first + mlo * step; j0 < jend; j0 += 8 * step) {
      int o[8], e[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = (64 * min(j0 + i * step, ny - 1) + lane) / CPR;
        o[i] = s_yoff[r];
        e[i] = y_in ? 0 : s_rows[r].y;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int j = j0 + i * step;
        if (j < jend) {
          const int sl = 64 * j + lane;
          const int r = sl / CPR;
          const int c = (sl % CPR) ^ (2 * (((unsigned)r / R64) % NSW));
          bool ok = o[i] >= 0;
          if (!y_in) ok = ok && d0 + (e[i] >> 16) < g.OD && h0 + ((e[i] >> 8) & 255) < g.OH && w0 + (e[i] & 255) < g.OW;
          int co16 = c * 16;
          if constexpr (SP) {
            // chunk c = class j (c >> 2), quarter c & 3: full-res position 2 cell + j sits in
            // shifted cell (cell + j), sub-position (1 - j)
            const int j = c >> 2, jd = j >> 2, jh = (j >> 1) & 1, jw = j & 1;
            co16 = (((jd * YH + jh) * YW + jw) * 8 + (7 - j)) * 64 + (c & 3) * 16;
          }
          const void* src = ok ? (const void*)(yo + o[i] + co16) : (const void*)zp;
          if constexpr (HAS_LOADER) ct_glds16(src, dst0 + (unsigned)(j << 10));
          else ct_glds16_nc(src, dst0 + (unsigned)(j << 10));
        }
      }
    }
  };

  // x halo of job `tile` (HPpad positions x 2 chunks, one LDS-DMA per 64 slots),
  // instructions first, first + step, ...  Interior tiles take
  // precomputed per-slot offsets from an SGPR base (table reads in batches of 8, one LDS
  // latency per batch); edge tiles check every slot against the input bounds and read
  // the zero page outside.
  auto dma_x = [&](int tile, int bufoff, int first, int step, int mlo = 0, int mhi = 1 << 20) {
    tile = __builtin_amdgcn_readfirstlane(tile);
    bufoff = __builtin_amdgcn_readfirstlane(bufoff);
    int n, d0, h0, w0;
    decode(tile, n, d0, h0, w0);
    const int dlo = d0 - g.pd, hlo = h0 - g.ph, wlo = w0 - g.pw;
    const unsigned dst0 = ct_lds_addr(dsm) + bufoff;
    const bf16* xs = x + (long long)n * g.ID * g.IH * g.IW * g.C + slice * 16 * XPL;
    const int nxp = (g.HPpad * XR) >> 10;        // DMA instructions per halo plane
    const int nx = min(nxp * XPL, first + mhi * step);   // DMA instructions of the x halo (this range)
    const bool x_in = dlo >= 0 && hlo >= 0 && wlo >= 0 && dlo + g.TD + g.KD - 1 <= g.ID && hlo + HH <= g.IH &&
                      wlo + HW <= g.IW;
    if (dbg & 4) {                             // (timing only: no x halo DMA)
    } else if (x_in) {
      const bf16* xo = xs + ((long long)(dlo * g.IH + hlo) * g.IW + wlo) * g.C;
      {                                          // wave-uniform (an SGPR operand of the DMA)
        const unsigned long long a = (unsigned long long)xo;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
        xo = (const bf16*)(((unsigned long long)hi << 32) | lo);
      }
      for (int j0 = first + mlo * step; j0 < nx; j0 += 8 * step) {
        int o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int jj = min(j0 + i * step, nx - 1);
          const int pl = SP ? (jj >= nxp ? 1 : 0) : 0;   // (SP: plane = second 16-channel slice)
          o[i] = s_xoff[((64 * (jj - pl * nxp) + lane) >> XSH)] + pl * 32;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (j0 + i * step < nx)
            if constexpr (HAS_LOADER) ct_glds16_s(xo, (unsigned)(o[i] + (lane & 1) * 16), dst0 + (unsigned)((j0 + i * step) << 10));
            else ct_glds16_s_nc(xo, (unsigned)(o[i] + (C8 ? 0 : (lane & 1) * 16)), dst0 + (unsigned)((j0 + i * step) << 10));
      }
    } else {
      for (int j0 = first + mlo * step; j0 < nx; j0 += 8 * step) {
        int e[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int jj = min(j0 + i * step, nx - 1);
          const int pl = SP ? (jj >= nxp ? 1 : 0) : 0;
          e[i] = s_pos[((64 * (jj - pl * nxp) + lane) >> XSH)];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (j0 + i * step < nx) {
            const int pl = SP ? (j0 + i * step >= nxp ? 1 : 0) : 0;
            const int gd = dlo + (e[i] >> 16), gh = hlo + ((e[i] >> 8) & 255), gw = wlo + (e[i] & 255);
            const bool ok = e[i] >= 0 && (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
                            (unsigned)gw < (unsigned)g.IW;
            const bf16* src =
                ok ? xs + ((long long)(gd * g.IH + gh) * g.IW + gw) * g.C + pl * 16 + (C8 ? 0 : (lane & 1) * 8) : zp;
            if constexpr (HAS_LOADER) ct_glds16(src, dst0 + (unsigned)((j0 + i * step) << 10));
            else ct_glds16_nc(src, dst0 + (unsigned)((j0 + i * step) << 10));
          }
        }
      }
    }
  };

  // BN prologue (pst != null; 16-channel slices of a plain conv, host-checked): x is the previous
  // layer's pre-BN output y and the conv's input is z = act(y * scale + shift) (pst = [scale C]
  // [shift C]) -- the forward's conv_tile loader normalised its halos the same way and never wrote
  // z.  Whoever DMA'd a job's x slots rewrites them in LDS once they have landed (the loader, or
  // in the loaderless form each wave its own 1/NW), with bn_apply_kernel's fma, activation and
  // rounding; zero-page slots (padding) stay zero.
  // (experiment builds only: in the default instances this code raised the VGPR count and doubled
  // the SGPR spills of the weight-gradient kernels the FeatureNet-3D step runs)
  auto xform_x = [&](int tile, int bufoff, int first, int step) {
#ifdef FN_EXPERIMENTS
    if constexpr (!SP && !C8) {
      if (!pst) return;
      tile = __builtin_amdgcn_readfirstlane(tile);
      int n, d0, h0, w0;
      decode(tile, n, d0, h0, w0);
      const int dlo = d0 - g.pd, hlo = h0 - g.ph, wlo = w0 - g.pw;
      const bool x_in = dlo >= 0 && hlo >= 0 && wlo >= 0 && dlo + g.TD + g.KD - 1 <= g.ID && hlo + HH <= g.IH &&
                        wlo + HW <= g.IW;
      const int nx = (g.HPpad * XR) >> 10;
      const int ch0 = slice * 16 + (lane & 1) * 8;   // (a lane's slots: one 8-channel half)
      ct_f32x2 sc[4], sh[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        sc[qq] = *(const ct_f32x2*)(pst + ch0 + 2 * qq);
        sh[qq] = *(const ct_f32x2*)(pst + g.C + ch0 + 2 * qq);
      }
      unsigned char* buf = dsm + bufoff + lane * 16;
      if (first >= nx) return;
      // the next slot's LDS reads go out before this slot's write (the compiler would otherwise
      // wait out every read alone)
      uint4 v = *(const uint4*)(buf + (first << 10));
      int e = s_pos[(64 * first + lane) >> 1];
      for (int j = first; j < nx; j += step) {
        const int jn = j + step < nx ? j + step : j;
        const uint4 vn = *(const uint4*)(buf + (jn << 10));
        const int en = s_pos[(64 * jn + lane) >> 1];
        const int gd = dlo + (e >> 16), gh = hlo + ((e >> 8) & 255), gw = wlo + (e & 255);
        const bool ok = e >= 0 && (x_in || ((unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
                                            (unsigned)gw < (unsigned)g.IW));
        unsigned bits;
        const uint4 o = ct_bn_chunk(v, sc, sh, true, bits);
        if (ok) *(uint4*)(buf + (j << 10)) = o;
        v = vn;
        e = en;
      }
    }
#else
    (void)tile; (void)bufoff; (void)first; (void)step;
#endif
  };

  if constexpr (!HAS_LOADER) {                  // job 0, 1/NW of it by each wave
    const int t0 = tile_of(0);
    if (t0 >= 0) {
      dma_x(t0, 0, wave, NW);
      dma_dy(t0, 0, wave, NW);
    }
  }
  if (loader) {
    // ======================= loader wave =======================
    int cur = __builtin_amdgcn_readfirstlane(s_job[0]);
    int nxt = __builtin_amdgcn_readfirstlane(s_job[1]);
    if (cur >= 0) {                              // job 0 entirely by the loader
      dma_x(cur, 0, 0, 1);
      dma_dy(cur, 0, 0, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (cur >= 0) xform_x(cur, 0, 0, 1);
    int par = 0, j = 0;
    while (true) {
      tile_lds_barrier();                        // A(j): job j's buffer landed, the other is free
      if (cur < 0) break;
      int t2 = -1;
      if (nxt >= 0) {
        t2 = tile_of(j + 2);                     // job j+2
        if (!(dbg & 1)) dma_x(nxt, (par ^ 1) * g.BUF, 0, 1);   // (dbg 1: timing only, stale data)
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (nxt >= 0 && !(dbg & 1)) xform_x(nxt, (par ^ 1) * g.BUF, 0, 1);
      if (lane == 0) s_job[(j + 2) % 3] = t2;
      cur = nxt;
      nxt = t2;
      par ^= 1;
      ++j;
    }
    return;
  }

  // ======================= compute waves =======================
  const int G4 = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int hp = KS2 ? (wave >= NW / 2 ? 1 : 0) : 0;   // first k-step of this wave
  const int tap0 = (tg * WPT + (KS2 ? (wave & (NW / 2 - 1)) : wave)) * NACC * TPF;
  int toff[NACC];                                // byte offsets of this wave's taps in the halo
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    if constexpr (SP) {                          // class (wave) taps j + e in the 3^3 footprint, plane i >> 3
      const int e = i & 7;
      const int kd = (wave >> 2) + (e >> 2), kh = ((wave >> 1) & 1) + ((e >> 1) & 1), kw = (wave & 1) + (e & 1);
      toff[i] = (i >> 3) * g.HPpad * XR + ((kd * HH + kh) * HW + kw) * XR;
    } else {
      const int ti = tap0 + TPF * i + (C8 ? (p4 >> 1) : 0);
      const int t = ti < T ? ti : 0;             // dead taps read tap 0 (never stored)
      const int kw = t % g.KW, kh = (t / g.KW) % g.KH, kd = t / (g.KW * g.KH);
      toff[i] = ((kd * HH + kh) * HW + kw) * XR;
    }
  }
  const bool live = SP || tap0 < T;
  f32x4 acc[NACC][MT];
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // dy fragment address of k-row r, 16-channel block mt: this lane's 4-channel quad
  auto dy_addr = [&](int r, int mt) -> int {
    const int c = (SP ? wave * 4 : 0) + 2 * mt + (p4 >> 1);   // (SP: this wave's class)
    return r * (CO_L * 2) + ((c ^ (2 * (((unsigned)r / R64) % NSW))) << 4) + (p4 & 1) * 8;
  };
  // One flat loop over (job, k-step): the accumulators are carried by a single loop (with
  // a job loop around a k-step loop, hipcc copied all of them at every job start).
  // Every wave runs it (dead taps read tap 0 and are never stored).  B fragments run PF
  // taps ahead in a register ring, across the k-step boundary; a job starts with a ring
  // fill after its barrier.
  int par = 0, ks = hp;
  const unsigned char* xb = dsm;
  const unsigned char* yb = dsm;
  int plo = 0, phi = 0, plo_n = 0, phi_n = 0;   // row offsets of k-steps ks and ks + 1
  bf16x8 ring[PF], fa[MT];
  auto rows_of = [&](int k, int& lo, int& hi) {
    const int r_lo = k * 32 + 4 * G4 + q;
    lo = s_rows[r_lo].x + 8 * (C8 ? (p4 & 1) : p4);
    hi = s_rows[r_lo + 16].x + 8 * (C8 ? (p4 & 1) : p4);
  };
  auto read_b = [&](int lo, int hi, int i) -> bf16x8 { return wt_tr_pair(xb + lo + toff[i], xb + hi + toff[i]); };
  auto read_a = [&](int k, bf16x8* f) {
    const int r_lo = k * 32 + 4 * G4 + q;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) f[mt] = wt_tr_pair(yb + dy_addr(r_lo, mt), yb + dy_addr(r_lo + 16, mt));
  };
  int jc = 0;                                   // job index (s_job ring slot jc % 3)
  int dnext = -1;                               // NW = 8: the tile this wave DMAs during the current job
  // issued at k-step 0 by waves 0-3 and at mid-job by waves 4-7 (the two waves of a SIMD
  // never both stop their MFMAs for the DMA burst at the same time)
  const int kdma = KS2 ? (hp == 0 ? 0 : ((g.kst / 2) | 1) < g.kst ? ((g.kst / 2) | 1) : 1)
                      : (wave < NW / 2 ? 0 : g.kst / 2);
  auto dma_slice = [&](int k) {
    if (dnext < 0 || k != kdma) return;
    const int bo = (par ^ 1) * g.BUF;
    dma_x(dnext, bo, wave, NW);
    dma_dy(dnext, bo, wave, NW);
  };
  auto start_job = [&]() -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of the job about to start
    if constexpr (!HAS_LOADER) {                 // (this wave's x slots of it: the BN prologue)
      const int tj = tile_of(jc);
      if (tj >= 0 && !(dbg & 1)) xform_x(tj, par * g.BUF, wave, NW);
    }
    tile_lds_barrier();                          // A
    const int tile = HAS_LOADER ? __builtin_amdgcn_readfirstlane(s_job[jc % 3]) : tile_of(jc);
    if (tile < 0) return false;
    const int nxt = HAS_LOADER ? __builtin_amdgcn_readfirstlane(s_job[(jc + 1) % 3]) : tile_of(jc + 1);
    if constexpr (HAS_LOADER) {
      if (nxt >= 0 && !(dbg & 1)) dma_dy(nxt, (par ^ 1) * g.BUF, wave, NW);   // a quarter of job j+1's dy
    } else {
      dnext = (dbg & 1) ? -1 : nxt;              // 1/NW of job j+1's halo and dy rows, a slice per k-step
    }
    ++jc;
    xb = dsm + par * g.BUF;
    yb = xb + g.XB;
    rows_of(hp, plo, phi);
    rows_of(hp + KSTEP < g.kst ? hp + KSTEP : hp, plo_n, phi_n);
    read_a(hp, fa);
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = read_b(plo, phi, p);
    return true;
  };
  // (Measured, C8 stem: alternating two A/B register sets so every read had a whole k-step
  // to land changed nothing -- 191 vs 192 us; with 8 MFMAs per k-step that kernel is bound
  // by the ~12 non-MFMA instructions issued per MFMA, SQ_INSTS_* in profiles/.)
  if (start_job()) {
    while (true) {
      // this k-step's A fragments were read during the previous one (or at the job start);
      // the next k-step's rows and A fragments are read here, a whole k-step ahead
      // row offsets two k-steps ahead (read here, used for the next k-step's ring refill: a
      // read consumed in the same k-step made hipcc drain every LDS read in flight)
      if constexpr (!HAS_LOADER) dma_slice(ks);
      const int ksn = ks + KSTEP < g.kst ? ks + KSTEP : ks;   // (a job's last k-steps re-read themselves: unused)
      const int ksnn = ks + 2 * KSTEP < g.kst ? ks + 2 * KSTEP : ksn;
      int plo_nn, phi_nn;
      rows_of(ksnn, plo_nn, phi_nn);
      bf16x8 fa_n[MT];
#pragma unroll
      for (int i = 0; i < NACC; ++i) {
        // the MFMAs read the ring slot in place; its refill (tap i + PF) is issued after
        // them (a copy of the slot would be a VALU write in front of every MFMA)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], ring[i % PF], acc[i][mt], 0, 0, 0);
        if (i == 0) read_a(ksn, fa_n);
        if (i + PF < NACC) ring[i % PF] = read_b(plo, phi, i + PF);
        else ring[i % PF] = read_b(plo_n, phi_n, i + PF - NACC);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) fa[mt] = fa_n[mt];
      plo = plo_n;
      phi = phi_n;
      plo_n = plo_nn;
      phi_n = phi_nn;
      ks += KSTEP;
      if (ks >= g.kst) {
        ks = hp;
        par ^= 1;
        if (!start_job()) break;
      }
    }
  }
  // D[row = co][col = ci]: lane holds co = mt*16 + (lane>>4)*4 + r, ci = lane & 15.
  // Plain stores into this workgroup's partial dW (partial = XCD x worker: the G
  // column-group workgroups of one (XCD, worker) write disjoint columns of it), summed
  // in a fixed order by wtile_reduce_kernel: deterministic, no atomics.
  float* part = dw + ((long long)(xcd * ((int)(gridDim.x >> 3) / g.G) + lid / g.G) * KSTEP + hp) *
                         (SP ? 8LL * CO * 8 : (long long)g.K * T) * g.C;
  if (live) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if constexpr (SP) {                        // part [class][co][e][ci] (T = 8 folded taps)
        const int ci = (slice * 2 + (i >> 3)) * 16 + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int co = wave * CO + mt * 16 + G4 * 4 + r;
            part[((long long)co * 8 + (i & 7)) * g.C + ci] = acc[i][mt][r];
          }
        continue;
      }
      const int t = tap0 + TPF * i + (C8 ? ((lane & 15) >> 3) : 0);
      const int ci = C8 ? (lane & 7) : slice * 16 + (lane & 15);
      if (t < T) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int co = mt * 16 + G4 * 4 + r;
            part[((long long)co * T + t) * g.C + ci] = acc[i][mt][r];
          }
      }
    }
  }
}

// dw[e] (+)= sum over the partials p = 0 .. W-1 of part[p][e], in a fixed order: each of the
// 4 waves of a block sums a quarter of the partials for the block's 64 float4 columns, and
// the quarters are added in wave order (deterministic; 4x the parallelism of one thread per
// column walking all W partials)
// wsrc (optional, C | 256): also the per-block partials wdp[block][c] = sum over the block's 256
// elements of channel c of bf16(wsrc) * dW (the BN statistics identity's S = sum W . dW, which
// bn_wdot_kernel would otherwise compute in a launch of its own after this one)
__global__ __launch_bounds__(256) void wtile_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                           long long n, int W, int accumulate,
                                                           const float* __restrict__ wsrc, float* __restrict__ wdp,
                                                           int C) {
  __shared__ float4 s_q[4][64];
  __shared__ float s_p[256];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long long i = ((long long)blockIdx.x * 64 + l) * 4;
  const int q = (W + 3) / 4, p0 = w * q, p1 = min(W, p0 + q);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i + 4 <= n) {
#pragma unroll 4
    for (int p = p0; p < p1; ++p) {
      const float4 v = *(const float4*)(part + (long long)p * n + i);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  } else if (i < n) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = p0; p < p1; ++p)
      for (long long j = i; j < n; ++j) t[j - i] += part[(long long)p * n + j];
    a = make_float4(t[0], t[1], t[2], t[3]);
  }
  s_q[w][l] = a;
  __syncthreads();
  if (w == 0 && i < n) {
    float4 r = accumulate ? (i + 4 <= n ? *(const float4*)(dw + i) : make_float4(0.f, 0.f, 0.f, 0.f))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    if (accumulate && i + 4 > n) {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (long long j = i; j < n; ++j) t[j - i] = dw[j];
      r = make_float4(t[0], t[1], t[2], t[3]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = s_q[k][l];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    if (i + 4 <= n) {
      *(float4*)(dw + i) = r;
    } else {
      const float t[4] = {r.x, r.y, r.z, r.w};
      for (long long j = i; j < n; ++j) dw[j] = t[j - i];
    }
    if (wsrc) {
      const float t[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) s_p[4 * l + k] = i + k < n ? (float)(bf16)wsrc[i + k] * t[k] : 0.f;
    }
  } else if (w == 0 && wsrc) {
#pragma unroll
    for (int k = 0; k < 4; ++k) s_p[4 * l + k] = 0.f;
  }
  if (wsrc) {                                    // (uniform: every thread reaches the barrier)
    __syncthreads();
    if ((int)threadIdx.x < C) {
      float t = 0.f;
      for (int e = threadIdx.x; e < 256; e += C) t += s_p[e];
      wdp[(long long)blockIdx.x * C + threadIdx.x] = t;
    }
  }
}

// Few outputs, many slices (the small layers of NAS candidates: a 4K-element dW over 1K
// partial rows ran 23 us in the 256-element blocks above, each thread walking a quarter of
// the rows): E elements per block in vectors of V (16-B loads when V = 4), the 256 V / E thread
// groups take every (256 V / E)-th row, then the groups' sums are added in group order -- fixed
// for a given (n, W), so still repeatable.  (Scalar loads -- V = 1 -- made the FeatureNet-3D stem's
// 16K-element reduce over its 1K+ partial rows 19.2 us against 11.7 us in the 256-element form.)
// (a second job -- part2 / dst2 / n2, the bias gradient beside a weight gradient -- takes the
// blocks past the first job's: one launch for both)
template <int E, int V>
__global__ __launch_bounds__(256) void part_reduce_narrow_kernel(const float* __restrict__ part, float* __restrict__ dst,
                                                                 long long n, int W, int accumulate,
                                                                 const float* __restrict__ part2 = nullptr,
                                                                 float* __restrict__ dst2 = nullptr, long long n2 = 0) {
  constexpr int T = E / V;                       // threads per row group
  constexpr int G = 256 / T;                     // row groups
  __shared__ float s_r[G][E];
  const int t = threadIdx.x % T, gq = threadIdx.x / T;
  long long b = blockIdx.x;
  const long long nb1 = (n + E - 1) / E;
  if (b >= nb1) {                                // (uniform per block)
    part = part2;
    dst = dst2;
    n = n2;
    b -= nb1;
  }
  const long long i = b * E + (long long)t * V;  // (V > 1: n % V == 0, whole vectors)
  float a0[V], a1[V];
#pragma unroll
  for (int v = 0; v < V; ++v) a0[v] = a1[v] = 0.f;
  auto add = [&](float (&acc)[V], int p) {
    if constexpr (V == 4) {
      const float4 x = *(const float4*)(part + (long long)p * n + i);
      acc[0] += x.x; acc[1] += x.y; acc[2] += x.z; acc[3] += x.w;
    } else {
      acc[0] += part[(long long)p * n + i];
    }
  };
  if (i < n) {
    int p = gq;
    for (; p + G < W; p += 2 * G) {
      add(a0, p);
      add(a1, p + G);
    }
    if (p < W) add(a0, p);
  }
#pragma unroll
  for (int v = 0; v < V; ++v) s_r[gq][t * V + v] = a0[v] + a1[v];
  __syncthreads();
  const long long o = b * E + threadIdx.x;
  if (threadIdx.x < E && o < n) {
    float r = accumulate ? dst[o] : 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) r += s_r[g][threadIdx.x];
    dst[o] = r;
  }
}

extern "C" int fn_part_reduce_wdot(const float* part, float* dst, long long n, int W, int accumulate,
                                  const float* wsrc, float* wdp, int C, hipStream_t st) {
  if (n <= 0) return 0;
  if (!part || !dst || W < 1) return -6;
  if (wsrc && (!wdp || C < 1 || 256 % C || n % C)) return -2;
  if (!wsrc && W >= 16 && (n + 255) / 256 < 192) {   // (narrow form: at least ~192 blocks)
    const bool v4 = n % 4 == 0 && ((uintptr_t)part & 15) == 0;
    const unsigned nb16 = (unsigned)((n + 15) / 16), nb64 = (unsigned)((n + 63) / 64);
    if (n <= 192 * 16) {
      if (v4) hipLaunchKernelGGL((part_reduce_narrow_kernel<16, 4>), dim3(nb16), dim3(256), 0, st, part, dst, n, W, accumulate);
      else hipLaunchKernelGGL((part_reduce_narrow_kernel<16, 1>), dim3(nb16), dim3(256), 0, st, part, dst, n, W, accumulate);
    } else {
      if (v4) hipLaunchKernelGGL((part_reduce_narrow_kernel<64, 4>), dim3(nb64), dim3(256), 0, st, part, dst, n, W, accumulate);
      else hipLaunchKernelGGL((part_reduce_narrow_kernel<64, 1>), dim3(nb64), dim3(256), 0, st, part, dst, n, W, accumulate);
    }
    FN_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(wtile_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, dst, n, W,
                     accumulate, wsrc, wdp, C);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_part_reduce(const float* part, float* dst, long long n, int W, int accumulate, hipStream_t st) {
  return fn_part_reduce_wdot(part, dst, n, W, accumulate, nullptr, nullptr, 0, st);
}

// two reductions over the same slice count (a weight gradient and its bias gradient) in one
// launch when both take the narrow form, else two
extern "C" int fn_part_reduce2(const float* part, float* dst, long long n, const float* part2, float* dst2,
                               long long n2, int W, int accumulate, hipStream_t st) {
  if (!part2 || !dst2 || n2 <= 0) return fn_part_reduce(part, dst, n, W, accumulate, st);
  if (n <= 0 || !part || !dst || W < 1) return -6;
  if (W >= 16 && (n + 255) / 256 < 192 && n <= 192 * 16 && n2 <= 192 * 16) {
    const unsigned nb = (unsigned)((n + 15) / 16 + (n2 + 15) / 16);
    if (n % 4 == 0 && n2 % 4 == 0 && !(((uintptr_t)part | (uintptr_t)part2) & 15))
      hipLaunchKernelGGL((part_reduce_narrow_kernel<16, 4>), dim3(nb), dim3(256), 0, st, part, dst, n, W, accumulate,
                         part2, dst2, n2);
    else
      hipLaunchKernelGGL((part_reduce_narrow_kernel<16, 1>), dim3(nb), dim3(256), 0, st, part, dst, n, W, accumulate,
                         part2, dst2, n2);
    FN_CHECK_LAUNCH();
    return 0;
  }
  if (int e = fn_part_reduce(part, dst, n, W, accumulate, st)) return e;
  return fn_part_reduce(part2, dst2, n2, W, accumulate, st);
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------
static WGeom parse_wgeom(const int* v) {
  WGeom g;
  g.N = v[0]; g.ID = v[1]; g.IH = v[2]; g.IW = v[3]; g.C = v[4];
  g.OD = v[5]; g.OH = v[6]; g.OW = v[7]; g.K = v[8];
  g.KD = v[9]; g.KH = v[10]; g.KW = v[11];
  g.pd = v[12]; g.ph = v[13]; g.pw = v[14];
  g.TD = v[15]; g.TH = v[16]; g.TW = v[17];
  g.HPpad = v[18]; g.kst = v[19]; g.XB = v[20]; g.BUF = v[21]; g.G = v[22]; g.ntg = v[23];
  return g;
}

static size_t wtile_lds(const WGeom& g) {
  return 2 * (size_t)g.BUF + 64 + (size_t)g.kst * 32 * 12 + (size_t)g.HPpad * 8;
}

// the BN prologue of the x halos is compiled into experiment builds only (FN_BUILD_EXPERIMENTS=1)
extern "C" int fn_conv_wtile_prologue_built() {
#ifdef FN_EXPERIMENTS
  return 1;
#else
  return 0;
#endif
}

extern "C" int fn_conv_wtile_supported(int K, int nacc) {
  const int c8 = (nacc >> 12) & 1, ks2 = (nacc >> 13) & 1, sp = (nacc >> 14) & 1;
  const int nw = (nacc >> 8) & 15;
  nacc &= 255;
  if (sp) return nw == 8 && nacc == 16 && K == 32 && !c8 && !ks2;
  if (ks2) return nw == 8 && nacc == 8 && (K == 32 || (K == 64 && !c8));
  if (c8) return nw == 8 && (K == 32 || K == 64) && nacc == 4;
  if (nw == 8) return (K == 32 && (nacc == 4 || nacc == 8 || nacc == 16)) || (K == 64 && (nacc == 4 || nacc == 8));
  return (K == 16 && nacc == 16) || (K == 32 && (nacc == 8 || nacc == 16)) || (K == 64 && nacc == 8);
}

// dw: fp32 [K][T][C], accumulated into (+=); part: fp32 scratch [8 * workers (x2 with ks2)][K][T][C]; rowtab int2[kst*32] (halo byte offset of
// the row's tap-0 position, packed tile coords or -1), k order with distinct halo positions
// mod 8 per aligned group of 8; postab int[HPpad] packed halo coords (-1 past the halo);
// zp >= 16 zero bytes; sched int[64] zeroed (left zero); workers = workgroups per (XCD,
// column group).
// wsrc / wdp (optional): the reduce also writes the S = sum W . dW partials [ceil(n / 256)][C]
// (fn_part_reduce_wdot)
extern "C" int fn_conv_wtile(const void* x, const void* dy, float* dw, float* part, const void* rowtab,
                             const void* postab, const void* zp, const int* geom, int nacc, int workers, int* sched,
                             hipStream_t st, const float* wsrc, float* wdp, const float* pst, int pact) {
  const WGeom g = parse_wgeom(geom);
  // nacc | (8 << 8): the loaderless 8-wave variant; | (1 << 12): its 8-input-channel form;
  // | (1 << 13): k-steps split between the wave halves; | (1 << 14): the sub-pixel form
  // (K = 32 per parity class, dy = the shifted space-to-depth view with 8 x K channels per
  // cell, a 3^3 footprint, dw = [8 classes][K][8 folded taps][C])
  const bool c8 = ((nacc >> 12) & 1) != 0, ks2 = ((nacc >> 13) & 1) != 0, sp = ((nacc >> 14) & 1) != 0;
  const int nw = ((nacc >> 8) & 15) == 8 ? 8 : 4;
  if (!fn_conv_wtile_supported(g.K, nacc)) return -2;
  // the BN prologue (x = pre-BN y; pst = [scale C][shift C]): 16-channel slices only, act none / relu
  if (pst && (c8 || sp || pact != ACT_RELU || !fn_conv_wtile_prologue_built())) return -2;   // (relu only)
  nacc &= 255;
  const int xr = c8 ? 16 : 32, tpf = c8 ? 2 : 1;
  if ((c8 ? g.C != 8 : g.C % (sp ? 32 : 16)) || g.TD < 1 || g.TH < 1 || g.TW < 1) return -2;
  if (sp && (g.KD != 3 || g.KH != 3 || g.KW != 3)) return -2;
  const int HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const long long HP = (long long)(g.TD + g.KD - 1) * HH * HW;
  const int T = g.KD * g.KH * g.KW;
  if (g.HPpad < HP || g.HPpad % (c8 ? 64 : 32) || g.TD + g.KD - 1 > 255 || HH > 255 || HW > 255) return -3;
  if ((long long)g.TD * g.TH * g.TW > 32LL * g.kst || g.kst < 1 || g.kst > 32) return -3;
  const int kl = sp ? 8 * g.K : g.K;             // dy channels per LDS row
  if (g.XB != g.HPpad * xr * (sp ? 2 : 1) || g.BUF < g.XB + g.kst * 32 * kl * 2 || g.BUF % 1024) return -3;
  const int wpt = ks2 ? nw / 2 : nw;
  if (sp ? (g.ntg != 1 || g.G != g.C / 32)
         : (g.ntg != (T + wpt * nacc * tpf - 1) / (wpt * nacc * tpf) || g.G != g.ntg * (c8 ? 1 : g.C / 16)))
    return -3;
  if (8 * g.G > 63) return -3;
  if (ks2 && g.kst < 2) return -3;
  if ((g.kst * 32 * (kl / 8)) % 64) return -3;
  const size_t lds = wtile_lds(g);
  if (lds > 160 * 1024) return -4;
  if (!sched || !zp || !part || workers < 1) return -6;
  const unsigned grid = 8u * (unsigned)g.G * (unsigned)workers;
  static const int dbg = [] { const char* e = getenv("FN_WTILE_DBG"); return e ? atoi(e) : 0; }();
#define WT_CASE(M, A, W, C, S, P)                                                                              \
  if (g.K == M * 16 && nacc == A && nw == W && c8 == C && ks2 == S && sp == P) {                               \
    static size_t cfg = 0;                                                                                     \
    if (lds > cfg) {                                                                                           \
      hipError_t e = hipFuncSetAttribute((const void*)conv_wtile_kernel<M, A, W, C, S, P>,                     \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                \
      if (e != hipSuccess) return (int)e;                                                                      \
      cfg = lds;                                                                                               \
    }                                                                                                          \
    hipLaunchKernelGGL((conv_wtile_kernel<M, A, W, C, S, P>), dim3(grid), dim3(wt_nthr(W)), lds, st,           \
                       (const bf16*)x, (const bf16*)dy, part, (const int2*)rowtab, (const int*)postab,         \
                       (const bf16*)zp, g, sched, dbg, pst, pact);                                             \
  }
  WT_CASE(1, 16, 4, false, false, false)
  WT_CASE(2, 8, 4, false, false, false)
  WT_CASE(2, 16, 4, false, false, false)
  WT_CASE(4, 8, 4, false, false, false)
  WT_CASE(2, 4, 8, false, false, false)
  WT_CASE(2, 8, 8, false, false, false)
  WT_CASE(2, 16, 8, false, false, false)
  WT_CASE(4, 4, 8, false, false, false)
  WT_CASE(4, 8, 8, false, false, false)
  WT_CASE(2, 4, 8, true, false, false)
  WT_CASE(4, 4, 8, true, false, false)
  WT_CASE(2, 8, 8, false, true, false)
  WT_CASE(4, 8, 8, false, true, false)
  WT_CASE(2, 8, 8, true, true, false)
  WT_CASE(2, 16, 8, false, false, true)
#undef WT_CASE
  FN_CHECK_LAUNCH();
  const long long n = sp ? 64LL * g.K * g.C : (long long)g.K * T * g.C;
  return fn_part_reduce_wdot(part, dw, n, 8 * workers * (ks2 ? 2 : 1), 1, sp ? nullptr : wsrc, wdp, g.C, st);
}
