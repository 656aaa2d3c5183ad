// Big-tile LDS-halo implicit-GEMM convolution (stride 1, 3-D) -- forward and dgrad.
//
// Successor of conv_halo.hip for the wide-channel FeatureNet-3D layers.  Where
// conv_halo runs 8 waves on <= 256-row tiles with 16-channel halo slices, a
// double-buffered 128-k weight stage in LDS (one barrier per stage) and a
// mostly synchronous halo reload per job, this kernel is built around ONE MFMA
// wave per SIMD:
//
//   * workgroup = 4 compute waves, each owning 16*MT output positions (MT = 8, 9)
//     x all NT*16 columns of the workgroup (512-576-position tiles: cubic-ish
//     output blocks, 2-4x less halo overhead than conv_halo's plane slabs), plus
//     one loader wave;
//   * the input halo of a CS-channel slice of a tile ("job") sits in one of two
//     LDS buffers; the loader LDS-DMAs the NEXT job's halo into the other buffer
//     (global_load_lds_dwordx4 from SGPR base + per-position offsets, zero page
//     for padding) while the compute waves run the current one -- one barrier per
//     job, nothing else;
//   * weights never touch LDS: pre-packed in MFMA-fragment order
//     ([slice][k-step][16-col tile][lane][8]) and streamed global -> VGPRs by
//     every compute wave (1 KB per fragment, L1/L2 hits), PD k-steps ahead in a
//     register ring that runs on across jobs;
//   * halo fragment reads are bank-conflict free: the halo is stored chunk-planar
//     (16-B chunk c of position p at c*PLANE + 16p, PLANE a multiple of 1 KB), so
//     the bank slot of a read is p mod 16, and the host permutes the tile
//     positions (rowtab) so that the 16 of every MFMA fragment have 16 distinct
//     halo positions mod 16: every ds_read_b128 lane group touches 16 distinct slots;
//   * per-k-step tap offsets come from a small LDS table (a scalar-memory table
//     would share lgkmcnt with the halo reads and drain them; an SALU tap walker
//     costs issue slots the single wave per SIMD cannot spare).
//
// MFMA: v_mfma_f32_16x16x32_bf16 with A = weights (16 output channels x 32 k) and
// B = halo (32 k x 16 positions): the accumulator is C^T, so a lane holds 4
// consecutive output channels of one position and the epilogue stores them
// straight from registers (+bias, bf16, activation, 8-B stores; optional BN
// statistics as per-workgroup column sums of the stored bf16 values) -- no LDS
// staging and no epilogue barriers.  k-step = 32 k = one tap x 32 channels
// (CS >= 32), two taps x 16 channels (CS = 16) or four taps x 8 channels (CS = 8).
//
// Dgrad uses the same kernel: dx = conv(dy, flip(W)^T) with leading pads K-1-p.
#include "conv_tile_shared.h"
#include "pack_w.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

// F8 = false: bf16 operands, v_mfma_f32_16x16x32_bf16, k-step 32; CPP = 16-B chunks (8
//   channels) per halo position.
// F8 = true (inference): OCP e4m3 halo and weights, v_mfma_scale_f32_16x16x128_f8f6f4 (unit
//   block scales), k-step 128 = each lane group's 32 bytes: tap 4ks+lg x 32 channels (CS =
//   32, CPP = 2 chunks of 16 channels) or tap 2ks+lg/2 x channels 32(lg&1).. (CS = 64, CPP =
//   4); the epilogue dequantises (acc * scale[co] + bias[co]), applies ReLU and stores bf16
//   or re-quantised e4m3 (x oscale).
// Q8O: the bf16 instance with an e4m3 output epilogue (fp8 inference: the bf16 stem writes the
// fp8 layers' input; its own register allocation)
// (A raw-moment BN-backward statistics epilogue for dgrad -- the statistics of the BN whose output
// this conv consumed, read from y at the tile's positions -- measured 5.37 vs 5.00 ms per step in
// round 4 and 5.14 vs 4.80 in round 3, and was removed; the relu-mask epilogue (MSK) replaced it.)
// I8 (with F8: the fp8 kernel's 32-byte fragments holding int8 instead): two
//   v_mfma_i32_16x16x64_i8 per fragment pair (bytes 0-15 and 16-31 of every lane: A and B split
//   the same way, so the k sum is complete), exact int32 accumulation, converted to float in
//   the epilogue before the dequantisation -- the binary-voxel stem of the fp8 inference path
//   (0/1 inputs are exact; per-channel int8 weights keep ~8 bits, where e4m3 kept 4).
// BS (block-scaled fp8, OCP MX style): with F8 the e4m3 input carries one E8M0 scale per (position,
//   32-channel block) -- xsc: a dword per position, byte j = block j -- that the loader LDS-DMAs with
//   each job's halo and every MFMA takes as its B-operand scale (the halo is the B operand); with an
//   e4m3 output (F8 fp8 output, or Q8O) the epilogue scales every (position, 32-column block) by its
//   own power of two and writes the scale byte into osc (the same dword-per-position layout)
// NCW: compute waves (4: one per SIMD, MT fragments each; 8: two per SIMD at MT / 2 -- the same
// 4 * 8 fragment rows, so the same row tables -- where a partner wave can issue while the other
// waits: the one-wave-per-SIMD k-loop ran its MFMAs at 72 % of its cycles)
// WL (bf16): the weight fragments through an LDS ring of `wring` k-step slots that the loader wave
// LDS-DMAs (one copy per workgroup instead of one per compute wave through L1), with per-k-step
// counters in LDS for the hand-off (see the loader); wring = 0 / WL false: every compute wave
// streams the fragments global -> VGPRs itself (the PD-deep register ring).
// PRO: the BN prologue instances (xform_job below; opt-in, measured slower) -- a template flag so the
// default instances carry none of its code (it doubled their SGPR spills)
// CHK: the instances with the chunked BN-statistics schedule (data parallelism); the others run the
// static one only (the chunk walk's state cost the one-GPU instances ~25 SGPR spills and 1-4 % of
// their time)
template <int MT, int NT, int CPP, int DBG = 0, bool F8 = false, bool Q8O = false, bool I8 = false, bool BS = false,
          int NCW = CT_NCW, bool WL = false, bool PRO = false, bool CHK = true>
__global__ __launch_bounds__(64 * (NCW + 1), 1) void conv_tile_kernel(const unsigned char* __restrict__ src,
                                                               const uint4* __restrict__ wp,
                                                               const int2* __restrict__ rowtab,
                                                               const int4* __restrict__ ktab,
                                                               const unsigned char* __restrict__ zp,
                                                               const float* __restrict__ bias, void* __restrict__ out,
                                                               float* __restrict__ stats, TileGeom g, int Ncol,
                                                               int act, int* __restrict__ sched,
                                                               long long* __restrict__ stamps,
                                                               const float* __restrict__ scale, float oscale,
                                                               const unsigned char* __restrict__ gmask,
                                                               const unsigned* __restrict__ xsc,
                                                               unsigned char* __restrict__ osc, int chunk,
                                                               int wring, const float* __restrict__ pst,
                                                               bf16* __restrict__ pz,
                                                               unsigned char* __restrict__ pmask, int pact) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  static_assert(!BS || F8 || Q8O, "block scales: fp8 operands or an e4m3 output");
  constexpr int NTHR = 64 * (NCW + 1);
  constexpr int PD = ct_pd(NT, F8);
  constexpr int ESZ = F8 ? 1 : 2;                // bytes per element of the source / weights
  constexpr int FRAG = F8 ? 32 : 16;             // bytes per lane of one MFMA operand fragment
  // NT = 2: 32-column blocks (a lane stores 8 consecutive columns).  NT = 4 (bf16, MT = 4: the
  // same 64 accumulator registers): 64-column workgroups over 256 rows, for loader-bound convs whose
  // 32-column blocks would each DMA the whole halo (the sub-pixel decoder's dgrad: 8 taps over 256
  // channels into 64 columns).  (Round 3 measured MT 8 x NT 4 3-4 % slower on the classifier --
  // 256 VGPRs -- and a 32x32x16-MFMA form measured 2-8 % slower per layer in round 4.)
  static_assert(NT == 2 || (NT == 4 && !F8), "32-column blocks, or 64 for the bf16 kernel");
  constexpr int RC = NT * 16;                    // columns of the workgroup (BN partial row length)
  constexpr int NV = 4 * NT;                     // consecutive columns per lane in the epilogue
  static_assert(!F8 || CPP == 2 || CPP == 4, "fp8: 32- or 64-channel slices");
  using Frag = std::conditional_t<F8, ct_i32x8, bf16x8>;

  const int HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const int HP = (g.TD + g.KD - 1) * HH * HW;
  const int PLANE = g.HPpad * 16;                // bytes per 16-B chunk plane
  const int rows = g.TD * g.TH * g.TW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH, twn = (g.OW + g.TW - 1) / g.TW;
  const int ntiles = g.N * tdn * thn * twn;
  const int nslice = g.C / g.CS;
  const int nks = g.nks;
  const int NQ = CPP * g.HPpad / 64;             // DMA wave-instructions per job halo

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = wave == NCW;
  const int lr = lane & 15, lg = lane >> 4;
  const int ct0 = blockIdx.y * NT;               // first 16-column tile of this workgroup
  // LDS: [buffer 0][buffer 1][job slots 64 B][BN partials][k-step offsets (nks+PD+2) int4]
  // [halo positions HPpad int2: (byte offset from the halo origin, packed hd|hh|hw)]
  int* s_job = reinterpret_cast<int*>(dsm + 2 * g.BUF);                    // [2][4] (tile, slice, flush) by parity
  // BN partials: [0] the waves' running per-tile sums (MT = 9), [1 + parity] the chunk flush rows;
  // each [4 waves][2][32]
  float* s_red = reinterpret_cast<float*>(dsm + 2 * g.BUF + 64);
  // BS (F8): two int4 per k-step -- the tap offset of the scale each lane group supplies, then the
  // lane group's packed (lo | hi << 16) data offsets (the block-scaled operand layout, below)
  constexpr int KTW = (F8 && BS) ? 2 : 1;
  int4* s_kt = reinterpret_cast<int4*>(dsm + 2 * g.BUF + 64 + ct_red_bytes(NT, NCW, F8));
  int2* s_pos = reinterpret_cast<int2*>(s_kt + KTW * (nks + PD + 2));
  for (int i = tid; i < KTW * (nks + PD + 2); i += NTHR) s_kt[i] = ktab[i];
  for (int i = tid; i < ct_red_bytes(NT, NCW, F8) / 4; i += NTHR) s_red[i] = 0.f;
  // F8: the dequantisation scale and bias of this workgroup's 32 columns ([scale 32][bias 32]),
  // read by the epilogue from LDS (global loads there serialised every tile's stores)
  float* s_sb = reinterpret_cast<float*>(s_pos + g.HPpad);
  // relu-mask dgrad (gmask): two buffers (by job parity) of the tile's mask bytes,
  // [natural tile row][Ncol / 8], after everything else
  const int mask_off = 64 + ct_red_bytes(NT, NCW, F8) + KTW * (nks + PD + 2) * 16 + g.HPpad * 8 + (F8 ? NT * 16 * 8 : 0);
  // (the buffers hold the bytes in FRAGMENT order -- slot f = (wave * MT + mt) * 16 + lr -- so
  // the epilogue reads slot (wave * MT + mt) * 16 + lr: a per-lane base plus a constant per mt)
  const int mask_bytes = ct_mask_bytes(NCW * MT * 16, Ncol, gmask != nullptr);
  // BS (F8): two planes (by job parity) of the halo positions' scale dwords, after s_sb
  const int scl_off = 2 * g.BUF + 64 + ct_red_bytes(NT, NCW, F8) + KTW * (nks + PD + 2) * 16 + g.HPpad * 8 + NT * 16 * 8;
  // ... and after them each fragment slot's (output offset from the tile origin in positions,
  // packed td|th|tw; dummy rows: the origin) for the loader's mask DMA, built once per kernel
  int2* s_mrow = reinterpret_cast<int2*>(dsm + 2 * g.BUF + mask_off + 2 * mask_bytes);
  if (!F8 && gmask) {
    for (int f = tid; f < NCW * MT * 16; f += NTHR) {
      const int r = rowtab[f].y;
      if (r < 0) {
        s_mrow[f] = make_int2(0, 0);
      } else {
        const int tw = r % g.TW, th = (r / g.TW) % g.TH, td = r / (g.TW * g.TH);
        s_mrow[f] = make_int2(td * g.osd + th * g.osh + tw * g.osw, (td << 16) | (th << 8) | tw);
      }
    }
  }
  // WL: the weight ring after everything else; counters in the job area: [8] k-steps published
  // (landed in the ring) by the loader, [12 + w] k-steps whose fragments compute wave w has read
  static_assert(!WL || !F8, "the LDS weight ring is the bf16 kernel's");
  constexpr unsigned WSLOT = NT * 1024u;         // bytes of one ring slot (NT 1-KB bf16 fragments)
  const int ring_off = 2 * g.BUF + mask_off + ct_mask_lds(NCW * MT * 16, Ncol, gmask != nullptr);
  int* s_wrdy = s_job + 8;
  int* s_wdone = s_job + 12;
  int* s_wabort = s_job + 9;                     // set by a wave whose bounded wait ran out: no more waits
  // (relaxed workgroup-scope atomics: plain ds_read / ds_write that the compiler may not merge,
  // drop or hoist out of a polling loop, and -- unlike volatile -- with no wait behind them)
  auto ld_cnt = [](int* p) -> int { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto st_cnt = [](int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  if constexpr (F8) {
    if (tid < NT * 16) {
      const int c = blockIdx.y * NT * 16 + tid;
      s_sb[tid] = c < Ncol ? scale[c] : 0.f;
      s_sb[NT * 16 + tid] = (bias && c < Ncol) ? bias[c] : 0.f;
    }
  }
  for (int p = tid; p < g.HPpad; p += NTHR) {  // positions past HP repeat the last one
    const int pc = p < HP ? p : HP - 1;
    const int hd = pc / (HH * HW), hh = (pc / HW) % HH, hw = pc % HW;
    s_pos[p] = make_int2(((hd * g.IH + hh) * g.IW + hw) * g.C * ESZ, (hd << 16) | (hh << 8) | hw);
  }
  // per compute lane: fragment row (output position) lr of each MFMA tile mt -- its LDS halo
  // offset lb (toggled between the buffers per job), its output offset relative to the
  // tile origin (-1: dummy row) and its packed tile coordinates (edge-tile bounds)
  int lb[MT], roff[MT], rpk[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int2 rt = rowtab[((loader ? 0 : wave) * MT + mt) * 16 + lr];
    // this lane group's (first) plane
    // (BS: lane group lg reads chunk plane lg & 1 (CPP 2) or lg (CPP 4) of two taps, see read_a)
    if constexpr (F8 && BS) lb[mt] = rt.x * 16 + (CPP == 4 ? lg : (lg & 1)) * PLANE;
    else if constexpr (F8) lb[mt] = rt.x * 16 + (CPP == 4 ? 2 * (lg & 1) : 0) * PLANE;
    else lb[mt] = rt.x * 16 + (CPP >= 4 ? lg : (CPP == 2 ? (lg & 1) : 0)) * PLANE;
    const int tw = rt.y % g.TW, th = (rt.y / g.TW) % g.TH, td = rt.y / (g.TW * g.TH);
    roff[mt] = rt.y < 0 ? -1 : td * g.osd + th * g.osh + tw * g.osw;
    rpk[mt] = (td << 16) | (th << 8) | tw;
  }

  // ---- loader: job decode and halo DMA --------------------------------------
  // Halo of job (tile, slice) into the buffer at bufoff.  Interior halos (the common
  // case for unpadded convs) use SGPR base + the per-position byte offsets of s_pos: no
  // address math per DMA row; halos crossing the input boundary check every position
  // and read the zero page outside.
  auto dma_job = [&](int tile, int slice, int bufoff) {
    ct_dma_job<CPP, ESZ>(g, src, zp, dsm, s_pos, tile, slice, bufoff, lane, tdn, thn, twn);
  };
  auto dma_job_rows = [&](int tile, int slice, int bufoff, int r_lo, int r_hi) {
    ct_dma_job<CPP, ESZ>(g, src, zp, dsm, s_pos, tile, slice, bufoff, lane, tdn, thn, twn, r_lo, r_hi);
  };
  // BS: the scale dwords of the job's halo positions into scale plane `which` (64 positions per
  // DMA row; positions outside the input read the zero page: scale 2^-127 on zero data)
  auto dma_scl = [&](int tile, int which) {
    if constexpr (F8 && BS) {
      int t = __builtin_amdgcn_readfirstlane(tile);
      const int tw_ = t % twn; t /= twn;
      const int th_ = t % thn; t /= thn;
      const int td_ = t % tdn;
      const int n = t / tdn;
      const int dlo = td_ * g.TD - g.pd, hlo = th_ * g.TH - g.ph, wlo = tw_ * g.TW - g.pw;
      const unsigned dst0 = ct_lds_addr(dsm) + (unsigned)(scl_off + which * g.HPpad * 4);
      const unsigned* base = xsc + (long long)n * g.ID * g.IH * g.IW;
      for (int r = 0; r < (g.HPpad >> 6); ++r) {
        const int e = s_pos[(r << 6) + lane].y;
        const int gd = dlo + (e >> 16), gh = hlo + ((e >> 8) & 255), gw = wlo + (e & 255);
        const bool ok = (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH && (unsigned)gw < (unsigned)g.IW;
        ct_glds4(ok ? (const void*)(base + ((long long)gd * g.IH + gh) * g.IW + gw) : (const void*)zp,
                 dst0 + (unsigned)(r << 8));
      }
    }
  };
  // the mask bytes of `tile` into mask buffer mpar, with the halo of the tile's last job: one
  // dword per lane (Ncol / 32 per position), natural row order; rows past the tile or the
  // output read the tile origin's bytes (never used)
  auto dma_mask = [&](int tile, int mpar) {
    if (!gmask) return;
    int t = __builtin_amdgcn_readfirstlane(tile);
    const int tw_ = t % twn; t /= twn;
    const int th_ = t % thn; t /= thn;
    const int td_ = t % tdn;
    const int n = t / tdn;
    const int d0 = td_ * g.TD, h0 = th_ * g.TH, w0 = tw_ * g.TW;
    const long long pb = (long long)n * g.osn + g.ob + (long long)d0 * g.osd + (long long)h0 * g.osh + w0 * g.osw;
    const int lg2 = Ncol == 64 ? 1 : 0;          // log2 dwords per position (Ncol 32 / 64)
    const int nslot = NCW * MT * 16;
    const int ndw = nslot << lg2;
    const int ld = g.OD - d0, lh = g.OH - h0, lw = g.OW - w0;
    const unsigned char* mb0 = gmask + pb * (Ncol >> 3);
    const unsigned dst = ct_lds_addr(dsm) + 2 * g.BUF + mask_off + mpar * mask_bytes;
    for (int k0 = 0; k0 < ndw; k0 += 64) {
      const int dd = k0 + lane;
      const int2 e = s_mrow[dd >> lg2];             // (ndw is a whole number of DMA rows)
      const bool in = (e.y >> 16) < ld && ((e.y >> 8) & 255) < lh && (e.y & 255) < lw;
      ct_glds4(mb0 + (long long)(in ? e.x : 0) * (Ncol >> 3) + (dd & ((1 << lg2) - 1)) * 4, dst + (unsigned)(k0 * 4));
    }
  };

  // BN prologue (pst != null; bf16 forward only, host-checked): the source is the PREVIOUS layer's
  // pre-BN output y, and the layer's input is z = relu(y * scale + shift) per input channel
  // (pst = [scale C][shift C]).  Once a job's halo has landed the loader rewrites it in LDS as z --
  // the same fma, activation and bf16 rounding as bn_apply_kernel, so the conv sees the same bits --
  // leaving the zero page's padding positions alone (the conv pads z, not y), and for the positions
  // the tile OWNS (per dimension the input rows [t*T - pad, (t+1)*T - pad) of output tile t, the
  // last tile also everything past them: every input position has exactly one owner) the first
  // column block also writes z (pz, for the weight gradient) and the relu-mask byte of each 8
  // channels (pmask, bit j = z_j > 0: the statistics identity of the backward, ops/bnfuse.py).
  // bn_apply's separate pass over y -- and its re-read of y here -- disappears.
  auto xform_job = [&](int tile, int slice, int bufoff) {
    if constexpr (!F8 && PRO) {
      if (!pst) return;
      int t = __builtin_amdgcn_readfirstlane(tile);
      const int tw_ = t % twn; t /= twn;
      const int th_ = t % thn; t /= thn;
      const int td_ = t % tdn;
      const int n = t / tdn;
      const int dlo = td_ * g.TD - g.pd, hlo = th_ * g.TH - g.ph, wlo = tw_ * g.TW - g.pw;
      const int HD = g.TD + g.KD - 1;
      const bool interior = dlo >= 0 && hlo >= 0 && wlo >= 0 && dlo + HD <= g.ID && hlo + HH <= g.IH &&
                            wlo + HW <= g.IW;
      // owned halo rows per dimension: [0, T) (all of them for the last tile)
      const int od = td_ == tdn - 1 ? 255 : g.TD, oh = th_ == thn - 1 ? 255 : g.TH, ow = tw_ == twn - 1 ? 255 : g.TW;
      const bool writer = blockIdx.y == 0 && (pz || pmask);
      const long long nbase = (long long)n * g.ID * g.IH * g.IW;
      // (the loader shares SIMD 0 with compute wave 0, whose MFMA stream wins the issue arbitration
      // at equal priority: the transform -- on the loader's critical path -- runs at a raised one)
      __builtin_amdgcn_s_setprio(2);
      unsigned char* buf = dsm + bufoff + lane * 16;
      // the slice's scale / shift pairs in VGPRs (an opaque zero in the index: uniform loads would
      // take 16 SGPRs per chunk, and the kernel already spills SGPRs)
      int z0;
      asm("v_mov_b32 %0, 0" : "=v"(z0));
      const float* ps = pst + slice * g.CS + z0;
      ct_f32x2 sc[CPP][4], sh[CPP][4];
#pragma unroll
      for (int c = 0; c < CPP; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sc[c][q] = *(const ct_f32x2*)(ps + c * 8 + 2 * q);
          sh[c][q] = *(const ct_f32x2*)(ps + g.C + c * 8 + 2 * q);
        }
      // a position's CPP chunks together (one s_pos read, one bounds test); every LDS read of a row
      // -- its chunks and the next row's s_pos entry -- is issued before the row's writes (the
      // compiler cannot tell the planes apart and would otherwise wait out each read alone)
      const int NR = g.HPpad >> 6;
      int e = s_pos[lane].y;
      for (int r = 0; r < NR; ++r) {
        const int p = (r << 6) + lane;
        uint4 v[CPP];
#pragma unroll
        for (int c = 0; c < CPP; ++c) v[c] = *(const uint4*)(buf + c * PLANE + (r << 10));
        const int e_next = s_pos[(r + 1 < NR ? p + 64 : p)].y;
        const int hd = e >> 16, hh = (e >> 8) & 255, hw = e & 255;
        const int gd = dlo + hd, gh = hlo + hh, gw = wlo + hw;
        const bool ok = interior || ((unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
                                     (unsigned)gw < (unsigned)g.IW);
        uint4 o[CPP];
        unsigned bits[CPP];
#pragma unroll
        for (int c = 0; c < CPP; ++c) {
          o[c] = ct_bn_chunk(v[c], sc[c], sh[c], true, bits[c]);
          if (ok) *(uint4*)(buf + c * PLANE + (r << 10)) = o[c];
        }
        if (writer && ok && p < HP && hd < od && hh < oh && hw < ow) {
          const long long pos = nbase + ((long long)gd * g.IH + gh) * g.IW + gw;
          if (pz) {
#pragma unroll
            for (int c = 0; c < CPP; ++c) *(uint4*)(pz + pos * g.C + slice * g.CS + c * 8) = o[c];
          }
          if (pmask) {                             // (CPP consecutive mask bytes, CPP-aligned)
            unsigned char* mp = pmask + pos * (g.C >> 3) + slice * (g.CS >> 3);
            if constexpr (CPP == 1) {
              *mp = (unsigned char)bits[0];
            } else if constexpr (CPP == 2) {
              *(unsigned short*)mp = (unsigned short)(bits[0] | (bits[1] << 8));
            } else {
#pragma unroll
              for (int c = 0; c < CPP; c += 4)
                *(unsigned*)(mp + c) = bits[c] | (bits[c + 1] << 8) | (bits[c + 2] << 16) | (bits[c + 3] << 24);
            }
          }
        }
        e = e_next;
      }
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // DBG & 16: cycle stamps of wave 0 and the loader (barrier-A wait, job work, tile end)
  long long st_a = 0, st_k = 0, st_e = 0, st_0 = 0, st_1 = 0;
  auto stamp = [&]() -> long long { return (DBG & 16) ? (long long)__builtin_amdgcn_s_memtime() : 0; };
  auto lap = [&](long long& acc_t) {
    if constexpr ((DBG & 16) != 0) {
      const long long t2 = stamp();
      acc_t += t2 - st_1;
      st_1 = t2;
    }
  };
  st_0 = stamp();

  // ---- job protocol ---------------------------------------------------------
  // s_job[4*par ..] = (tile, slice, flush) of the job whose halo sits in buffer par (tile -1:
  // done; flush: see below).  The loader publishes job j+1 in slot par^1 right after barrier
  // A(j) and lands its halo before barrier A(j+1); every wave reads its job after barrier A.
  // The compute waves never wait on anything else: the epilogue stores straight from registers.
  // Tile schedule.  Without BN statistics every output element is written by exactly one tile
  // whatever the order, and tiles are handed out one at a time from a counter.  With statistics
  // (stats != null) the partial sums must not depend on which workgroup ran which tiles, or the
  // statistics -- and everything downstream -- would change in the last bits run to run:
  //   * chunk > 0 (the default): the tiles are cut into fixed CHUNKS of `chunk` consecutive
  //     tiles (the host sizes them from the tile count alone, never from the grid or the CU
  //     count); workgroups grab whole chunks from a counter, and each compute wave writes its
  //     partial sums over a chunk into the chunk's own slab row (chunk * NCW + wave) when the
  //     chunk's last job ends (s_job flush = the chunk id).  The sums are fixed per chunk and
  //     the finalize adds the rows in a fixed order, so the result is the same bits whatever
  //     the grab order -- and a workgroup that starts late (its CU held by another kernel, e.g.
  //     an RCCL ring of the data-parallel all-reduce) simply takes fewer chunks
  //     (profiles/r6_dp_interference.md);
  //   * chunk == 0: the round-5 STATIC schedule (job k = tile k * G + slot, slots XCD-major;
  //     per-workgroup partial rows), kept for the A/B of that measurement: a CU held by another
  //     kernel there delays its workgroup's whole fixed share.
  const bool stat_static = stats != nullptr && (!CHK || chunk <= 0);
  const bool stat_chunk = CHK && stats != nullptr && chunk > 0;
  const int G = (int)gridDim.x;
  const int slot = (G & 7) == 0 ? ((int)blockIdx.x & 7) * (G >> 3) + ((int)blockIdx.x >> 3) : (int)blockIdx.x;
  const int nchunk = stat_chunk ? (ntiles + chunk - 1) / chunk : 0;
  // Dynamic grabs (chunks with statistics, single tiles without) come from 8 XCD queues: the units
  // are cut into 8 contiguous ranges, queue x's counter at sched[1 + 8 * blockIdx.y + x]; a
  // workgroup takes from the queue of its own XCD (workgroups are dispatched to the XCDs round
  // robin: linear id & 7 -- a locality hint only, any mapping is correct), so neighbouring tiles
  // run together on one XCD and share halo rows in its L2, and once that range is done it takes
  // from the others in turn (the tail balances across the chip).
  const int nunit = stat_chunk ? nchunk : ntiles;
  const int xcd0 = (int)((blockIdx.x + blockIdx.y * gridDim.x) & 7);
  int qdone = 0;                                 // (loader, uniform) bit x: queue x found empty
  auto grab = [&]() -> int {                     // the next unit for this workgroup, or -1
    for (int i = 0; i < 8; ++i) {
      const int x = (xcd0 + i) & 7;
      if (qdone & (1 << x)) continue;
      const int lo = (int)(((long long)nunit * x) >> 3), hi = (int)(((long long)nunit * (x + 1)) >> 3);
      int c = 0;
      if (lane == 0) c = atomicAdd(sched + 1 + 8 * blockIdx.y + x, 1);
      c = lo + __builtin_amdgcn_readfirstlane(c);
      if (c < hi) return c;
      qdone |= 1 << x;
    }
    return -1;
  };
  // loader state of the chunk walk (wave-uniform): the chunk being handed out, its next tile, its end
  int ch_id = -1, ch_next = 0, ch_end = 0;
  auto next_tile = [&](int k) -> int {           // tile of this workgroup's job k (-1: none)
    if (stat_chunk) {
      if (ch_next >= ch_end) {
        const int c = grab();
        if (c < 0) return -1;
        ch_id = c;
        ch_next = c * chunk;
        ch_end = min(ntiles, ch_next + chunk);
      }
      return ch_next++;
    }
    if (stat_static) {
      const int t = k * G + slot;
      return t < ntiles ? t : -1;
    }
    return grab();
  };
  // the chunk to flush after job (tile, slice): its id when this is the chunk's last job, else -1
  auto flush_of = [&](int tile, int slice) -> int {
    return (stat_chunk && tile >= 0 && tile == ch_end - 1 && slice == nslice - 1) ? ch_id : -1;
  };
  if (loader) {                                  // (the loader runs the tile walk; its first job here)
    const int t0 = next_tile(0);
    if (lane == 0) {
      s_job[0] = t0;
      s_job[1] = 0;
      s_job[2] = flush_of(t0, 0);
    }
    if (WL && lane < 2 + NCW) s_job[lane == 0 ? 8 : (lane == 1 ? 9 : 10 + lane)] = 0;   // (ring counters, abort)
  }
  tile_lds_barrier();

  if (WL && loader) {
    // ================ loader wave, LDS weight ring (WL) ================
    // The weights are one cyclic stream: job j runs slice j % nslice (a tile's jobs are its slices in
    // order), so k-step q of the workgroup is packed row (slice (q / nks) % nslice, k-step q % nks)
    // whatever the tiles.  Step q goes to ring slot q % wring once every compute wave has read the
    // step wring before it (s_wdone); after its DMA has landed the loader publishes it (s_wrdy).
    // The next job's halo rows are interleaved with the weight steps, one per step, so a wait for
    // landed weights never waits behind a whole halo.
    int tile = __builtin_amdgcn_readfirstlane(s_job[0]), slice = 0, t_next = -1, kjob = 1;
    const int NR = g.HPpad >> 6;
    const unsigned char* wsrc = reinterpret_cast<const unsigned char*>(wp) + (size_t)ct0 * 1024;
    const unsigned ring0 = ct_lds_addr(dsm) + (unsigned)ring_off;
    int qi = 0, wsl = 0, wk = 0, wslot = 0;      // next step to issue: its slice, k-step, ring slot
    // (the compute waves hand slots back a whole turn -- PD k-steps -- at a time, and the loader
    // issues and publishes whole turns: one credit poll, one wait for the landing per PD steps)
    auto issue_w = [&]() {
      const unsigned char* src = wsrc + ((size_t)(wsl * nks + wk) * g.nct) * 1024;
      const unsigned dst = ring0 + (unsigned)wslot * WSLOT;
      if (!(act & 0x800)) {                      // (0x800, timing only: no weight DMAs at all)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) ct_glds16_s(src + nt * 1024, (unsigned)lane * 16u, dst + (unsigned)nt * 1024u);
      }
      ++qi;
      if (++wk == nks) {
        wk = 0;
        if (++wsl == nslice) wsl = 0;
      }
      if (++wslot == wring) wslot = 0;
    };
    auto credit = [&]() -> int {                 // steps the ring can hold now: the slowest reader + wring
      if (act & 0x400) return 1 << 30;           // (timing only: no hand-off, wrong results)
      int m = ld_cnt(s_wdone);
#pragma unroll
      for (int w = 1; w < NCW; ++w) m = min(m, ld_cnt(s_wdone + w));
      return __builtin_amdgcn_readfirstlane(m) + wring;
    };
    auto publish = [&]() {                       // everything issued so far has landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) st_cnt(s_wrdy, qi);
    };
    // Turns stay in flight while the next one is issued: DMA instructions issued so far (nis:
    // weights and halo rows; anything uncounted only lengthens a wait below), and for the last
    // three issued batches the step count and nis right after them (uniform shift registers).
    // Publishing batch b waits vmcnt(DMAs issued after it) -- the newer batches stay in flight.
    int nis = 0, nfl = 0;                        // (nfl: batches in flight, <= 3)
    int bq0 = 0, bq1 = 0, bq2 = 0, bn0 = 0, bn1 = 0, bn2 = 0;   // [0] = the oldest in flight
    auto wait_vm = [&](int n) {                  // s_waitcnt vmcnt(n), n rounded down to a multiple of 4
      switch (min(n, 60) >> 2) {
#define CT_VMW(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * k) : "memory"); break;
        CT_VMW(0) CT_VMW(1) CT_VMW(2) CT_VMW(3) CT_VMW(4) CT_VMW(5) CT_VMW(6) CT_VMW(7)
        CT_VMW(8) CT_VMW(9) CT_VMW(10) CT_VMW(11) CT_VMW(12) CT_VMW(13) CT_VMW(14)
        default: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
#undef CT_VMW
      }
    };
    auto push_batch = [&]() {                    // a batch just issued (qi, nis after it)
      if (nfl == 0) { bq0 = qi; bn0 = nis; }
      else if (nfl == 1) { bq1 = qi; bn1 = nis; }
      else { bq2 = qi; bn2 = nis; }
      ++nfl;
    };
    auto publish_oldest = [&]() {                // the oldest batch in flight has landed
      wait_vm(nis - bn0);
      if (lane == 0) st_cnt(s_wrdy, bq0);
      bq0 = bq1; bn0 = bn1; bq1 = bq2; bn1 = bn2;
      --nfl;
    };
    if (tile >= 0) {
      dma_job(tile, 0, 0);
      if (nslice == 1) dma_mask(tile, 0);
      if (!stat_chunk) t_next = next_tile(kjob);
      ++kjob;
    }
    while (qi < wring) issue_w();                // (credit: nothing read yet)
    publish();
    int par = 0, jcur = 0;
    int fl_prev = -1;
    int fl_cur = __builtin_amdgcn_readfirstlane(s_job[2]);
    while (true) {
      tile_lds_barrier();                        // A: job halo landed; the other buffer is free
      if (fl_prev >= 0) {
        const float* fl = s_red + (1 + (par ^ 1)) * NCW * 2 * RC;
        float* row = stats + (long long)fl_prev * 2 * Ncol;
        for (int i = lane; i < 2 * RC; i += 64) {
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < NCW; ++w) v += fl[w * 2 * RC + i];
          const int c = ct0 * 16 + (i < RC ? i : i - RC);
          if (c < Ncol) row[(i < RC ? 0 : Ncol) + c] = v;
        }
      }
      fl_prev = fl_cur;
      if (tile < 0) break;
      int ntile = tile, nslc = slice + 1;
      if (nslc == nslice) {
        nslc = 0;
        ntile = stat_chunk ? next_tile(kjob) : t_next;
      }
      fl_cur = flush_of(ntile, nslc);
      if (lane == 0) {
        s_job[4 * (par ^ 1)] = ntile;
        s_job[4 * (par ^ 1) + 1] = nslc;
        s_job[4 * (par ^ 1) + 2] = fl_cur;
      }
      // this period: job jcur's steps (and the compute waves' read-ahead of the next job's first)
      // must all be issued before barrier A(jcur + 1), and the next job's first turn too, so it
      // starts without waiting for the loader.  The next job's halo rows go in one per issued
      // step (two when no step can be issued), and must have landed before the barrier.
      const int qneed = (jcur + 1) * nks + 1;
      const int qmax = qneed + wring - 1;
      const int bo = (par ^ 1) * g.BUF;
      int hr = ntile >= 0 ? 0 : NR;
      if (ntile >= 0 && nslc == nslice - 1) dma_mask(ntile, par ^ 1);
      int guard = 0;
      while (true) {
        const int lim = min(credit(), qmax + 1);
        if (lim - qi >= PD || (lim > qi && lim == qmax + 1)) {   // a whole turn (or the period's rest)
          const int n = min(lim - qi, PD);
          for (int b = 0; b < n; ++b) {
            issue_w();
            nis += NT;
            if (hr < NR) {
              dma_job_rows(ntile, nslc, bo, hr, hr + 1);
              nis += CPP;
              ++hr;
            }
          }
          push_batch();
          if (nfl > 2) publish_oldest();         // (two batches stay in flight)
          guard = 0;
          continue;
        }
        if (hr < NR) {                           // no credit yet: halo rows
          for (int b = 0; b < 2 && hr < NR; ++b) {
            dma_job_rows(ntile, nslc, bo, hr, hr + 1);
            nis += CPP;
            ++hr;
          }
          continue;
        }
        if (nfl > 0) {                           // nothing to issue: the oldest batch lands
          publish_oldest();
          continue;
        }
        // the job's steps and the next job's first turn issued and landed: on to the barrier (the
        // compute waves finish this job from the ring without the loader, and find the next one's
        // first turn there -- no bubble at the job boundary)
        if (qi >= qneed + PD) break;
        // (no credit: the compute waves are behind by the whole ring.  The loop is bounded: after
        // 2^20 empty polls -- tens of ms, far past any k-step -- it gives up and sets the abort flag
        // that ends every wait of the workgroup, rather than hang the GPU)
        if (++guard > (1 << 20) || ld_cnt(s_wabort)) {
          if (lane == 0) st_cnt(s_wabort, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the halo of the next job has landed)
      if (nslc == 0 && ntile >= 0) {
        if (!stat_chunk) t_next = next_tile(kjob);
        ++kjob;
      }
      tile = ntile;
      slice = nslc;
      par ^= 1;
      ++jcur;
    }
    tile_lds_barrier();                          // R
  } else if (loader) {
    // ======================= loader wave =======================
    int tile = __builtin_amdgcn_readfirstlane(s_job[0]), slice = 0, t_next = -1, kjob = 1;
    // (the chunk walk hands out the next tile only once the current one is published: t_next is
    // taken when the loader moves to a new tile, so flush_of sees the chunk of the published job)
    if (tile >= 0) {
      dma_job(tile, 0, 0);
      dma_scl(tile, 0);
      if (nslice == 1) dma_mask(tile, 0);
      if (!stat_chunk) t_next = next_tile(kjob);
      ++kjob;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tile >= 0) xform_job(tile, 0, 0);
    int par = 0;
    int fl_prev = -1;                            // flush (chunk id) of the job before the current one
    int fl_cur = __builtin_amdgcn_readfirstlane(s_job[2]);
    while (true) {
      st_1 = stamp();
      tile_lds_barrier();                        // A: job halo landed; the other buffer is free
      lap(st_a);
      if (!F8 && fl_prev >= 0) {
        // the chunk that ended with the previous job: its 4 waves' flush rows (that job's parity,
        // par ^ 1 now), added in wave order, into the chunk's slab row
        const float* fl = s_red + (1 + (par ^ 1)) * NCW * 2 * RC;
        float* row = stats + (long long)fl_prev * 2 * Ncol;
        for (int i = lane; i < 2 * RC; i += 64) {
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < NCW; ++w) v += fl[w * 2 * RC + i];
          const int c = ct0 * 16 + (i < RC ? i : i - RC);
          if (c < Ncol) row[(i < RC ? 0 : Ncol) + c] = v;
        }
      }
      fl_prev = fl_cur;
      if (tile < 0) break;
      int ntile = tile, nslc = slice + 1;
      if (nslc == nslice) {
        nslc = 0;
        ntile = stat_chunk ? next_tile(kjob) : t_next;
      }
      const int nfl = flush_of(ntile, nslc);
      fl_cur = nfl;
      if (lane == 0) {
        s_job[4 * (par ^ 1)] = ntile;
        s_job[4 * (par ^ 1) + 1] = nslc;
        s_job[4 * (par ^ 1) + 2] = nfl;
      }
      if (!(DBG & 4) && ntile >= 0) dma_job(ntile, nslc, (par ^ 1) * g.BUF);
      if (ntile >= 0) dma_scl(ntile, par ^ 1);
      if (ntile >= 0 && nslc == nslice - 1) dma_mask(ntile, par ^ 1);
      if (nslc == 0 && ntile >= 0) {
        if (!stat_chunk) t_next = next_tile(kjob);
        ++kjob;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lap(st_k);
      if (ntile >= 0) xform_job(ntile, nslc, (par ^ 1) * g.BUF);
      lap(st_e);                                 // (the loader's "epilogue" stamp: the BN prologue)
      tile = ntile;
      slice = nslc;
      par ^= 1;
    }
    tile_lds_barrier();                          // R: the compute waves' BN partials (uniform count)
  } else {
    // ======================= compute waves =======================
    if constexpr ((DBG & 64) != 0) __builtin_amdgcn_s_setprio(1);   // (timing variant: compute waves first)
    // MFMA with the weights as A (16 output channels) and the halo as B (16 positions):
    // acc[mt][nt] = C^T, lane (lr, lg) holds channels (ct0+nt)*16 + 4lg + r of position
    // lr of tile mt -- 4 consecutive channels of one output row, stored as one 8-B write
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    Frag fa[MT];                                 // rotating: fragment mt of k-step k+1 is read right
                                                 // after the NT MFMAs of (mt, k) consumed it
    // BS: E8M0 scales (low byte) of fragment rows, a ring of SR read SR - 1 fragments ahead of their
    // MFMAs (not a full k-step like fa: 8 more live registers made the kernel spill)
    static_assert(!(F8 && BS) || MT % 4 == 0, "block-scaled instances: MT a multiple of the scale ring");
    constexpr int SR = (F8 && BS) ? 4 : 1;
    unsigned fs[SR];
    int scl_job = 0;                             // BS: the lane's scale byte of the job's scale plane
                                                 // (less the lane's halo plane offset, see read_s)
    // B operand: the PD-deep register ring of weight fragments streamed from global memory, or (WL)
    // two k-steps of fragments read from the LDS weight ring one k-step ahead
    Frag fb[WL ? 2 : PD][NT];
    // the packed weight columns are ordered so that fragment nt row 4lg+r is output column
    // ct0*16 + 4*NT*lg + 4nt + r: a lane ends with NV = 4*NT consecutive columns of one position
    const int gc8 = ct0 * 16 + NV * lg;
    ct_f32x2 bias2[NT / 2][4];                   // (fp8: read in the epilogue from LDS, no live
#pragma unroll                                   // registers across the k-loop)
    for (int h = 0; h < NT / 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = gc8 + 8 * h + 2 * q + e;
          bias2[h][q][e] = (!F8 && bias && c < Ncol) ? bias[c] : 0.f;
        }
    constexpr unsigned FTILE = 64u * FRAG;       // bytes of one 16-column fragment of a k-step
    const unsigned wstep = (unsigned)g.nct * FTILE;   // bytes per k-step of the packed weights
    unsigned voffb[PD];                          // per-lane B offsets of the PD ring slots
#pragma unroll
    for (int u = 0; u < PD; ++u) voffb[u] = (unsigned)lane * FRAG + (unsigned)u * wstep;
    // weight loads are ordinary loads: hipcc counts them (vmcnt waits before the consuming
    // MFMAs, correct across its own register copies); the compute waves issue no hidden
    // VMEM, so its counts are exact
    auto load_b = [&](const unsigned char* base, int slot) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) fb[slot][nt] = *(const Frag*)(base + voffb[slot] + nt * FTILE);
    };
    // A fragment of row block mt at k-step offset ko: one 16-B read (bf16) or the lane
    // group's two consecutive chunk planes (fp8)
    // BS: v_mfma_scale_f32_16x16x128_f8f6f4 reads a lane's bytes 0-15 as k = 16 lg .. and bytes 16-31 as
    // k = 64 + 16 lg .., and takes the scale of 32-k block j from lane group j
    // (tests/test_fp8_block_gpu.py::test_scaled_mfma_operand_layout), so every block must be one
    // (position, 32-channel block): lane group lg reads its low 16 B at the packed offset's low half
    // and its high 16 B at the high half (two taps, one chunk plane), and supplies the scale of
    // block lg (kofs_s)
    auto read_a = [&](int mt, int ko) -> Frag {
      if constexpr (F8 && BS) {
        const uint4 lo = *(const uint4*)(dsm + lb[mt] + (ko & 0xffff));
        const uint4 hi = *(const uint4*)(dsm + lb[mt] + (ko >> 16));
        return (ct_i32x8){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      } else if constexpr (F8) {
        const uint4 lo = *(const uint4*)(dsm + lb[mt] + ko);
        const uint4 hi = *(const uint4*)(dsm + lb[mt] + ko + PLANE);
        return (ct_i32x8){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      } else {
        return *(const bf16x8*)(dsm + lb[mt] + ko);
      }
    };
    // k-step offsets: s_kt[k][lg] = byte offset of the tap lane group lg reads in k-step k
    // (all four equal for CS >= 32, pairs for CS = 16, four taps for CS = 8).  Reading
    // them per lane keeps the offset a per-lane value even where it is uniform: hipcc then
    // keeps the halo reads interleaved with the MFMAs (with a wave-uniform offset it
    // hoisted a turn's reads into a double-buffered block)
    auto kofs = [&](int k) -> int { return *((const int*)(s_kt + KTW * k + (KTW - 1)) + lg); };
    // (BS: the scale tap, as kq = the lane's scale byte base + tap / 4 -- read_s adds lb / 4)
    auto kofs_s = [&](int k) -> int { return scl_job + (*((const int*)(s_kt + KTW * k) + lg) >> 2); };
    // BS: the scale of fragment mt's rows at k-step scale base ko = kq (kofs_s: the byte of the
    // row's tap position dword).  lb[mt] = 16 row + halo plane + buffer, tap offsets 16 tap:
    // lb / 4 + tap / 4 is the dword index 4 (row + tap) plus terms scl_job takes back off.  One byte
    // read (ds_read_u8, zero-extended: the MFMA takes the low byte), no shift after it -- a shift
    // right behind each read made hipcc wait for every scale read on the spot (lgkmcnt(0) per
    // fragment: the block-scaled kernel ran 1.47x the per-tensor one)
    auto read_s = [&](int mt, int ko) -> unsigned {
      if constexpr (F8 && BS) return *(const unsigned char*)(dsm + ko + (lb[mt] >> 2));   // (ko: kq, below)
      else return 127u;
    };
    // epilogue variant (wave-uniform); columns come in whole 8-column groups (Ncol % 8 == 0)
    // (fp8: bit 0 relu, bit 1 fp8 output)
    // (fp8: act bit CT_F8_POOL = the 2^3 max-pool epilogue, relu + bf16 output of the pooled grid)
    const int emode = F8 ? (((act & 0xff) == ACT_RELU ? 1 : 0) | (oscale > 0.f ? 2 : 0) | ((act & CT_F8_POOL) ? 4 : 0))
                         : ((stats ? 1 : 0) | ((act & 0xff) == ACT_RELU ? 2 : 0) | (Q8O ? 8 : 0));   // (ACT_NONE /
                                                                                          // ACT_RELU only; 8: e4m3 out)
    // relu-mask dgrad (stats, no activation; host-checked) -- selected inside case 1, so every
    // emode value still reaches an epilogue (a reachable no-epilogue path kept the accumulators
    // live across it: 227 -> 256 VGPRs with spills)
    const bool msk = !F8 && gmask != nullptr && !(act & 0x200);   // (0x200: timing only, DMA without the mask epilogue)
    // BN partial sums of this lane's columns over every tile the workgroup runs (the epilogues
    // add into them; one DPP + LDS reduction after the last tile instead of one per tile:
    // stem fwd epilogue ~40 % of its cycles in round 4 stamps).  MT = 9 keeps the per-tile
    // reduction (16 more live registers made it spill)
    constexpr bool RSACC = MT <= 8;
    // (column pairs: the epilogue's adds are packed v_pk_add / v_pk_fma of two columns)
    ct_f32x2 rsum[NT / 2][4], rsq[NT / 2][4];
#pragma unroll
    for (int h = 0; h < NT / 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) rsum[h][q] = rsq[h][q] = (ct_f32x2){0.f, 0.f};
    // ring prologue: the first job's k-steps 0..PD-1 (slice 0); every later job's come from
    // the previous job's last turn, so no job starts on an exposed L2 latency
    if constexpr (!WL) {
#pragma unroll
      for (int u = 0; u < PD; ++u) load_b(reinterpret_cast<const unsigned char*>(wp) + (size_t)ct0 * FTILE, u);
    }
    // WL: the workgroup's k-step counter (uniform), the ring slot of the NEXT step, the published
    // count as read during the previous step (one LDS read per step, used a step later)
    int wq = 0, wslot1 = wring > 1 ? 1 : 0, wr_v = 0;
    const unsigned char* rbase = dsm + ring_off + lane * 16;
    // (bounded wait for the loader: no hang, whatever happens to it)
    auto ring_wait = [&](int need) -> int {
      int c = __builtin_amdgcn_readfirstlane(wr_v);
      for (int guard = 0; c <= need; ++guard) {
        if (guard > (1 << 20) || ld_cnt(s_wabort)) {   // (bounded: give up, and make every other
          st_cnt(s_wabort, 1);                         //  wait of the workgroup give up at once)
          return need + 1;
        }
        __builtin_amdgcn_s_sleep(1);
        c = __builtin_amdgcn_readfirstlane(ld_cnt(s_wrdy));
      }
      return c;
    };
    bool wfirst = true;
    int par = 0;
    while (true) {
      st_1 = stamp();
      tile_lds_barrier();                        // A
      lap(st_a);
      const int tile = __builtin_amdgcn_readfirstlane(s_job[4 * par]);
      const int slice = __builtin_amdgcn_readfirstlane(s_job[4 * par + 1]);
      const int flush = __builtin_amdgcn_readfirstlane(s_job[4 * par + 2]);
      if (tile < 0) break;
      const int nslc = slice + 1 == nslice ? 0 : slice + 1;
      if constexpr (F8 && BS) {
        scl_job = scl_off + par * g.HPpad * 4 - (((CPP == 4 ? lg : (lg & 1)) * PLANE + par * g.BUF) >> 2) +
                  (CPP == 4 ? 2 * slice + (lg & 1) : slice);   // (+ the byte of this lane group's 32-channel block)
      }
      // ---- k-loop: MFMA + A reads + B loads, nothing else ----
      const unsigned char* wbase = reinterpret_cast<const unsigned char*>(wp) +
                                   ((size_t)slice * nks * g.nct + ct0) * FTILE + PD * wstep;
      // weights of the next job: its slice (slice 0 for a new tile, whatever the tile)
      const unsigned char* wnext =
          reinterpret_cast<const unsigned char*>(wp) + ((size_t)nslc * nks * g.nct + ct0) * FTILE;
      int kos_c = (F8 && BS) ? kofs_s(0) : 0;   // BS: scale offsets of the current k-step
      {
        const int ko = kofs(0);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) fa[mt] = read_a(mt, ko);
        if constexpr (F8 && BS) {
#pragma unroll
          for (int mt = 0; mt < SR - 1; ++mt) fs[mt] = read_s(mt, kos_c);
        }
      }
      int ko_n = kofs(1);                        // offsets of the next k-step
      if constexpr (WL) {
        if (wfirst) {                            // (every later job's first step: read ahead by the
          wfirst = false;                        //  previous job's last one)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) fb[0][nt] = *(const Frag*)(rbase + nt * 1024);
          wr_v = ld_cnt(s_wrdy);
        }
      }
      for (int ks = 0; ks < nks; ks += PD) {
        const unsigned char* wl = ks + PD >= nks ? wnext : wbase;   // last turn: next job's steps
#pragma unroll
        for (int u = 0; u < PD; ++u) {
          const int ko = (DBG & 32) ? u * 16 * 37 : ko_n;   // (DBG 32, timing only: constant tap offsets)
          const int kos_x = (F8 && BS) ? kofs_s(ks + u + 1) : 0;   // (BS: the next k-step's)
          if constexpr (!(DBG & 32)) ko_n = kofs(ks + u + 2);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              if constexpr (F8 && I8) {   // int8 x int8 -> int32 (the accumulator's bits)
                typedef int ct_i32x4 __attribute__((ext_vector_type(4)));
                const ct_i32x8 b8 = fb[u][nt], a8 = fa[mt];
                ct_i32x4 c = __builtin_bit_cast(ct_i32x4, acc[mt][nt]);
                c = __builtin_amdgcn_mfma_i32_16x16x64_i8((ct_i32x4){b8[0], b8[1], b8[2], b8[3]},
                                                         (ct_i32x4){a8[0], a8[1], a8[2], a8[3]}, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_i32_16x16x64_i8((ct_i32x4){b8[4], b8[5], b8[6], b8[7]},
                                                         (ct_i32x4){a8[4], a8[5], a8[6], a8[7]}, c, 0, 0, 0);
                acc[mt][nt] = __builtin_bit_cast(f32x4, c);
              } else if constexpr (F8 && BS)   // e4m3 x e4m3, weights unscaled (127 = 1.0; per-channel
                acc[mt][nt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(   // scale in the epilogue),
                    fb[u][nt], fa[mt], acc[mt][nt], 0, 0, 0, 127, 0, (int)fs[mt % SR]);  // halo block-scaled
              else if constexpr (F8)   // e4m3 x e4m3 (formats 0, 0), E8M0 scales 127 = 1.0
                acc[mt][nt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[u][nt], fa[mt], acc[mt][nt], 0, 0,
                                                                                 0, 127, 0, 127);
              else
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[WL ? (u & 1) : u][nt], fa[mt], acc[mt][nt],
                                                                      0, 0, 0);
            }
            if constexpr (!(DBG & 2)) {
              fa[mt] = read_a(mt, ko);
              if constexpr (F8 && BS) {          // row mt + SR - 1: this k-step's or (wrapped) the next's
                const int r = mt + SR - 1;
                fs[r % SR] = read_s(r < MT ? r : r - MT, r < MT ? kos_c : kos_x);
              }
            }
            if constexpr (WL) {
              if (mt == 0) {
                // the next k-step's fragments from the ring.  Once per turn: are the turn's reads
                // (steps wq + 1 .. wq + PD) published?  (the count read a step ago; rarely short --
                // then wait).  At the turn's end: this wave is done with the slots of the steps
                // before wq + 2 (the reads, the count store and the next count read stay in order:
                // LDS runs one wave's accesses in order; the relaxed atomics keep the compiler's)
                int so = wslot1 * (int)WSLOT;
                if (u == 0) {
                  int c = __builtin_amdgcn_readfirstlane(wr_v);
                  if (c <= wq + PD && !(act & 0x400)) c = ring_wait(wq + PD);   // (0x400: timing only)
                  // (the slot offset through an opaque copy that takes the checked count as an
                  // input: the turn's reads cannot be hoisted above the check)
                  asm volatile("s_mov_b32 %0, %1" : "=s"(so) : "s"(so), "s"(c));
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) fb[(u + 1) & 1][nt] = *(const Frag*)(rbase + so + nt * 1024);
                if (u == PD - 1) {
                  st_cnt(s_wdone + wave, wq + 2);
                  // (once per turn, for the next turn's check: a count read every step would be dead
                  // until overwritten, and the overwrite waits for it -- lgkmcnt(0) every step)
                  wr_v = ld_cnt(s_wrdy);
                }
              }
            }
            if constexpr (!(DBG & 128)) __builtin_amdgcn_sched_barrier(0);   // (DBG 128: free scheduling
          }                                                                  //  within a k-step)
          // k-step ks+u+PD, or the next job's step u
          if constexpr (WL) {
            ++wq;
            wslot1 = wslot1 + 1 == wring ? 0 : wslot1 + 1;
          } else if constexpr (!(DBG & 1)) {
            load_b(wl, u);
          }
          if constexpr (F8 && BS) kos_c = kos_x;
          __builtin_amdgcn_sched_barrier(0);
        }
        wbase += PD * wstep;
      }
      lap(st_k);
      if (slice == nslice - 1) {
        // ---- epilogue: acc (+bias) -> bf16 -> activation -> 8-B stores (+BN sums) ----
        int t = tile;
        const int tw_i = t % twn; t /= twn;
        const int th_i = t % thn; t /= thn;
        const int td_i = t % tdn;
        const int n = t / tdn;
        const int d0 = td_i * g.TD, h0 = th_i * g.TH, w0 = tw_i * g.TW;
        const int ld = g.OD - d0, lh = g.OH - h0, lw = g.OW - w0;   // in-bounds tile extent
        const bool edge = ld < g.TD || lh < g.TH || lw < g.TW;
        const long long obase_e =
            ((long long)n * g.osn + g.ob + (long long)d0 * g.osd + (long long)h0 * g.osh + w0 * g.osw) * Ncol + gc8;
        bf16* obase = reinterpret_cast<bf16*>(out) + obase_e;
        // straight-line variants per (statistics, activation): runtime branches inside the
        // unrolled per-tile loop made hipcc emit ~1000 basic blocks
        auto epilogue = [&](auto mode) {
          // bit 0: forward BN statistics (sum v, sum v^2) of the stored values; bit 1: relu.
          constexpr int M = decltype(mode)::value;
          constexpr bool RELU_OUT = (M & 2) != 0;
          constexpr bool ST = (M & 1) != 0;
          // bit 3: e4m3 output of v * oscale (saturated; fp8 inference: the bf16 stem writes the
          // fp8 layers' input directly), 8-B stores; no statistics
          constexpr bool Q8 = (M & 8) != 0;
          // bit 4: relu-mask dgrad -- the column sums are of g = dx * relu'(z) (z's mask bits, from
          // LDS); dx itself is stored unmasked (it is the true gradient of z)
          constexpr bool MSK = (M & 16) != 0;
          // (MSK: the loader DMA'd the tile's mask bytes into the LDS mask buffer of this job's
          // parity, [fragment slot][Ncol / 8])
          const unsigned char* mb = dsm + 2 * g.BUF + mask_off + par * mask_bytes +
                                    ((wave * MT * 16 + lr) * (Ncol >> 3) + (gc8 >> 3));
          unsigned mrows[MSK ? MT : 1][NT / 2];  // (all the byte reads in flight together; byte h:
          if constexpr (MSK) {                   //  the lane's columns 8h .. 8h + 7)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
              for (int h = 0; h < NT / 2; ++h) mrows[mt][h] = mb[mt * 16 * (Ncol >> 3) + h];
          }
          bool okm[MT];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            bool ok = roff[mt] >= 0 && gc8 < Ncol;
            if (edge) ok = ok && (rpk[mt] >> 16) < ld && ((rpk[mt] >> 8) & 255) < lh && (rpk[mt] & 255) < lw;
            okm[mt] = ok;
          }
          // one pass per 8 consecutive columns of the lane (fragments 2h, 2h+1): one 16-B store
          // per row; the BN partial sums go into the lane's running sums (rsum / rsq).  Column
          // pairs throughout: packed bias add, one v_cvt_pk_bf16_f32 per pair gives the stored
          // word (relu on the packed bf16 as a signed 16-bit max), the statistics unpack that
          // word (the stored values) into packed adds -- ~3 VALU per value instead of ~6
#pragma unroll
          for (int h = 0; h < NT / 2; ++h) {
            ct_f32x2 tsl[4], tql[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) tsl[q] = tql[q] = (ct_f32x2){0.f, 0.f};
            ct_f32x2* ts = RSACC ? rsum[h] : tsl;
            ct_f32x2* tq = RSACC ? rsq[h] : tql;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              const bool ok = okm[mt];
              const unsigned mrow = MSK ? mrows[mt][h] : 0u;
              unsigned pw[4];                    // the stored bf16 pairs (columns 2q, 2q+1)
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const f32x4 a4 = acc[mt][2 * h + (q >> 1)];
                const ct_f32x2 v = (ct_f32x2){a4[(2 * q) & 3], a4[(2 * q + 1) & 3]} + bias2[h][q];
                unsigned w = bf16x2_pack(v[0], v[1]);
                if constexpr (RELU_OUT) w = ct_relu_bf16x2(w);
                pw[q] = w;
              }
              if constexpr (ST) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  unsigned w = ok ? pw[q] : 0u;
                  if constexpr (MSK) {               // the sums see g = dx * relu'(z): bits 2q, 2q+1
                    const unsigned b = mrow >> (2 * q);   // of the row's mask byte (dx is stored whole)
                    w &= ((b & 1u) ? 0x0000ffffu : 0u) | ((b & 2u) ? 0xffff0000u : 0u);
                  }
                  const ct_f32x2 x = (ct_f32x2){bf16_lo(w), bf16_hi(w)};
                  ts[q] += x;
                  if constexpr (!MSK) tq[q] += x * x;      // (the identity needs sum g only)
                }
              }
              if constexpr (Q8) {
                float qs = oscale;               // BS: 2^-e of the (row, 32-column) block instead
                if constexpr (BS) {
                  float am = 0.f;
#pragma unroll
                  for (int q = 0; q < 4; ++q) am = fmaxf(am, fmaxf(fabsf(bf16_lo(pw[q])), fabsf(bf16_hi(pw[q]))));
                  am = fmaxf(am, __shfl_xor(am, 16, 64));
                  am = fmaxf(am, __shfl_xor(am, 32, 64));
                  const int e = ct_e8m0_exp(am);
                  qs = ct_exp2_neg(e);
                  if (ok && lg == 0) {
                    const long long pos = (long long)n * g.osn + g.ob + (long long)d0 * g.osd + (long long)h0 * g.osh +
                                          w0 * g.osw + roff[mt];
                    osc[pos * 4 + blockIdx.y] = (unsigned char)(e + 127);
                  }
                }
                if (ok) {
                  unsigned wd[2];
#pragma unroll
                  for (int qq = 0; qq < 2; ++qq) {
                    float e[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                      const unsigned w = pw[2 * qq + (j >> 1)];
                      const float v = (j & 1) ? bf16_hi(w) : bf16_lo(w);
                      e[j] = __builtin_amdgcn_fmed3f(v * qs, RELU_OUT ? 0.f : -448.f, 448.f);
                    }
                    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(e[0], e[1], 0, false);
                    pk = __builtin_amdgcn_cvt_pk_fp8_f32(e[2], e[3], pk, true);
                    wd[qq] = (unsigned)pk;
                  }
                  *(uint2*)(reinterpret_cast<unsigned char*>(out) + obase_e + (long long)roff[mt] * Ncol + 8 * h) =
                      make_uint2(wd[0], wd[1]);
                }
              } else if (ok && !(DBG & 8))      // (DBG 8, timing only: no output stores)
                *(uint4*)(obase + (long long)roff[mt] * Ncol + 8 * h) = make_uint4(pw[0], pw[1], pw[2], pw[3]);
              acc[mt][2 * h] = (f32x4){0.f, 0.f, 0.f, 0.f};
              acc[mt][2 * h + 1] = (f32x4){0.f, 0.f, 0.f, 0.f};
            }
            if constexpr (ST && !RSACC) {        // (per-tile: DPP over the 16 lanes, LDS adds)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float a = ct_sum16(ts[j >> 1][j & 1]), b = ct_sum16(tq[j >> 1][j & 1]);
                if (lr == 0) {
                  s_red[wave * 2 * RC + NV * lg + 8 * h + j] += a;
                  s_red[wave * 2 * RC + RC + NV * lg + 8 * h + j] += b;
                }
              }
            }
          }
        };
        // fp8 inference epilogue: dequantise + bias (+ReLU) -> bf16 (16-B store) or e4m3 of
        // y * oscale (8-B store)
        auto epilogue_f8 = [&](auto mode) {
          constexpr int M = decltype(mode)::value;   // bit 0 relu, bit 1 fp8 output, bit 2 max-pool
          constexpr bool POOL = (M & 4) != 0;
          float sc8[8], bs8[8];
          {
            const float4* q = reinterpret_cast<const float4*>(s_sb + 8 * lg);
            const float4 a = q[0], b = q[1], c = q[NT * 4], d = q[NT * 4 + 1];
            sc8[0] = a.x; sc8[1] = a.y; sc8[2] = a.z; sc8[3] = a.w;
            sc8[4] = b.x; sc8[5] = b.y; sc8[6] = b.z; sc8[7] = b.w;
            bs8[0] = c.x; bs8[1] = c.y; bs8[2] = c.z; bs8[3] = c.w;
            bs8[4] = d.x; bs8[5] = d.y; bs8[6] = d.z; bs8[7] = d.w;
          }
          if constexpr ((M & 2) != 0 && !BS) {   // fp8 output: fold the requantisation scale into the
#pragma unroll                                   // dequantisation (one FMA + one med3 per value)
            for (int j = 0; j < 8; ++j) {
              sc8[j] *= oscale;
              bs8[j] *= oscale;
            }
          }
          // BS fp8 output: position index of the tile origin (the output view), for the scale bytes
          const long long pbase = (long long)n * g.osn + g.ob + (long long)d0 * g.osd + (long long)h0 * g.osh +
                                  w0 * g.osw;
          // POOL: the pool row table puts the 8 members of one 2^3 window in one lane, member m
          // in fragment m (MT = 8): the lane's running max over the fragments is the pooled value
          float pm[POOL ? 8 : 1];
          if constexpr (POOL) {
#pragma unroll
            for (int j = 0; j < 8; ++j) pm[j] = 0.f;   // (relu: pooled values are >= 0)
          }
          bool pok = false;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            bool ok = roff[mt] >= 0 && gc8 < Ncol;
            if (edge) ok = ok && (rpk[mt] >> 16) < ld && ((rpk[mt] >> 8) & 255) < lh && (rpk[mt] & 255) < lw;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              // (the element is copied out first: __builtin_bit_cast of a vector-element lvalue
              // compiled to element 0 of the vector -- every lane's 4 columns got column 0's sum)
              const float ae = acc[mt][j >> 2][j & 3];
              const float a = I8 ? (float)__builtin_bit_cast(int, ae) : ae;
              v[j] = a * sc8[j] + bs8[j];
              if constexpr ((M & 2) != 0 && !BS)   // (already x oscale) relu / saturate in one med3
                v[j] = __builtin_amdgcn_fmed3f(v[j], (M & 1) != 0 ? 0.f : -448.f, 448.f);
              else if constexpr ((M & 1) != 0 || POOL)
                v[j] = fmaxf(v[j], 0.f);
            }
            if constexpr ((M & 2) != 0 && BS) {
              // block scale of (row, the workgroup's 32 columns): the 4 lanes lr + 16 lg hold them
              float am = 0.f;
#pragma unroll
              for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[j]));
              am = fmaxf(am, __shfl_xor(am, 16, 64));
              am = fmaxf(am, __shfl_xor(am, 32, 64));
              const int e = ct_e8m0_exp(am);
              const float inv = ct_exp2_neg(e);
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_fmed3f(v[j] * inv, -448.f, 448.f);
              if (ok && lg == 0) osc[(pbase + roff[mt]) * 4 + blockIdx.y] = (unsigned char)(e + 127);
            }
            if constexpr (POOL) {
              if (mt == 0) pok = ok;             // (windows lie wholly inside or outside the output)
#pragma unroll
              for (int j = 0; j < 8; ++j) pm[j] = fmaxf(pm[j], v[j]);
            } else if (ok) {
              if constexpr ((M & 2) != 0) {
                unsigned wd[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                  int p = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * h], v[4 * h + 1], 0, false);
                  p = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * h + 2], v[4 * h + 3], p, true);
                  wd[h] = (unsigned)p;
                }
                *(uint2*)(reinterpret_cast<unsigned char*>(out) + obase_e + (long long)roff[mt] * Ncol) =
                    make_uint2(wd[0], wd[1]);
              } else {
                *(uint4*)(obase + (long long)roff[mt] * Ncol) =
                    make_uint4(bf16x2_pack(v[0], v[1]), bf16x2_pack(v[2], v[3]), bf16x2_pack(v[4], v[5]),
                               bf16x2_pack(v[6], v[7]));
              }
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
          }
          if constexpr (POOL) {
            if (pok) {                           // pooled grid [N][OD/2][OH/2][OW/2][Ncol]
              const int PDm = g.OD >> 1, PHm = g.OH >> 1, PWm = g.OW >> 1;
              const int pd_ = (d0 + (rpk[0] >> 16)) >> 1, ph_ = (h0 + ((rpk[0] >> 8) & 255)) >> 1,
                        pw_ = (w0 + (rpk[0] & 255)) >> 1;
              bf16* po = reinterpret_cast<bf16*>(out) +
                         ((((long long)n * PDm + pd_) * PHm + ph_) * PWm + pw_) * Ncol + gc8;
              *(uint4*)po = make_uint4(bf16x2_pack(pm[0], pm[1]), bf16x2_pack(pm[2], pm[3]),
                                       bf16x2_pack(pm[4], pm[5]), bf16x2_pack(pm[6], pm[7]));
            }
          }
        };
        if constexpr (F8) {
          switch (emode) {
            case 0: epilogue_f8(std::integral_constant<int, 0>{}); break;
            case 1: epilogue_f8(std::integral_constant<int, 1>{}); break;
            case 2: epilogue_f8(std::integral_constant<int, 2>{}); break;
            case 3: epilogue_f8(std::integral_constant<int, 3>{}); break;
            default: if constexpr (MT == 8) epilogue_f8(std::integral_constant<int, 5>{}); break;
          }
        } else {
          switch (emode) {
            case 0: epilogue(std::integral_constant<int, 0>{}); break;
            case 1:
              if (msk) epilogue(std::integral_constant<int, 17>{});
              else epilogue(std::integral_constant<int, 1>{});
              break;
            case 2: epilogue(std::integral_constant<int, 2>{}); break;
            case 3: epilogue(std::integral_constant<int, 3>{}); break;
            case 8: if constexpr (Q8O) epilogue(std::integral_constant<int, 8>{}); break;
            default: if constexpr (Q8O) epilogue(std::integral_constant<int, 10>{}); break;
          }
        }
        lap(st_e);
        if (!F8 && stat_chunk && flush >= 0) {
          // the chunk's last job: this wave's partial sums over the chunk into its LDS flush row
          // of this job's parity; after the next barrier A the loader adds the 4 waves' rows in
          // wave order and stores the chunk's slab row (every row written once per column block)
          float* fl = s_red + (1 + par) * NCW * 2 * RC + wave * 2 * RC;
          if constexpr (RSACC) {
#pragma unroll
            for (int h = 0; h < NT / 2; ++h) {
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float a = ct_sum16(rsum[h][j >> 1][j & 1]), b = ct_sum16(rsq[h][j >> 1][j & 1]);
                if (lr == 0) {
                  fl[NV * lg + 8 * h + j] = a;
                  fl[RC + NV * lg + 8 * h + j] = b;
                }
              }
#pragma unroll
              for (int q = 0; q < 4; ++q) rsum[h][q] = rsq[h][q] = (ct_f32x2){0.f, 0.f};
            }
          } else {                               // (per-tile sums in this wave's own LDS row)
            for (int i = lane; i < 2 * RC; i += 64) {
              fl[i] = s_red[wave * 2 * RC + i];
              s_red[wave * 2 * RC + i] = 0.f;
            }
          }
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) lb[mt] += (1 - 2 * par) * g.BUF;   // the other buffer
      par ^= 1;
    }
    if (!F8 && RSACC && stat_static) {
      // (static schedule) the lane's running sums over the 16 lanes holding the same columns
      // (DPP), into the wave's LDS row: the workgroup's tiles are a fixed sequence, so every
      // partial -- and the finalize's fixed-order sum over the slab rows -- is the same run to run
#pragma unroll
      for (int h = 0; h < NT / 2; ++h) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = ct_sum16(rsum[h][j >> 1][j & 1]), b = ct_sum16(rsq[h][j >> 1][j & 1]);
          if (lr == 0) {
            s_red[wave * 2 * RC + NV * lg + 8 * h + j] = a;
            s_red[wave * 2 * RC + RC + NV * lg + 8 * h + j] = b;
          }
        }
      }
    }
    tile_lds_barrier();                          // R
    if (!F8 && stat_static && tid < RC && ct0 * 16 + tid < Ncol) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < NCW; ++w) {
        s1 += s_red[w * 2 * RC + tid];
        s2 += s_red[w * 2 * RC + RC + tid];
      }
      float* row = stats + (long long)blockIdx.x * 2 * Ncol;   // this workgroup's slab row
      row[ct0 * 16 + tid] = s1;
      row[Ncol + ct0 * 16 + tid] = s2;
    }
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the last job's unused ring loads
  if constexpr ((DBG & 16) != 0) {
    if (lane == 0 && (wave == 0 || loader)) {
      long long* d = stamps + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16 + (loader ? 8 : 0);
      d[0] = st_a;
      d[1] = st_k;
      d[2] = st_e;
      d[6] = stamp() - st_0;
    }
    if (lane == 0 && wave == 1) {                // (compute wave 1, alone on SIMD 1: slots 3, 4, 5, 7)
      long long* d = stamps + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16;
      d[3] = st_a;
      d[4] = st_k;
      d[5] = st_e;
      d[7] = stamp() - st_0;
    }
  }
  if (tid == 0 && !stat_static) {                // the last workgroup out resets the counters
    __threadfence();                             // (static schedules never touch them)
    if (atomicAdd(sched, 1) == (int)(gridDim.x * gridDim.y) - 1) {
      for (int i = 0; i < 8 * (int)gridDim.y; ++i) atomicExch(sched + 1 + i, 0);
      atomicExch(sched, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// weight packing: conv weight [K][T][C] (fp32) -> MFMA B fragments
// ---------------------------------------------------------------------------
// (the element map: pack_w.h tile_pack_w_one)
__global__ __launch_bounds__(256) void tile_pack_w_kernel(const float* __restrict__ w, uint4* __restrict__ out, int K,
                                                          int T, int C, int CS, int nks, int nct, int nslice,
                                                          int dgrad, int nt) {
  const long long total = ((long long)nslice * nks + 4) * nct * 64;   // + the ring's 4 zero k-steps
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < total) tile_pack_w_one(w, out, K, T, C, CS, nks, nct, nslice, dgrad, nt, i);
}

// The forward and the dgrad packing of one weight in one launch (the conv's forward packs its
// backward's dgrad operand too: one graph node fewer on the backward's critical path)
struct TilePackJob {
  uint4* out;
  int CS, nks, nct, nslice, dgrad, nt;
};

__global__ __launch_bounds__(256) void tile_pack_w2_kernel(const float* __restrict__ w, int K, int T, int C,
                                                           TilePackJob j0, TilePackJob j1) {
  const long long t0 = ((long long)j0.nslice * j0.nks + 4) * j0.nct * 64;
  const long long t1 = ((long long)j1.nslice * j1.nks + 4) * j1.nct * 64;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < t0)
    tile_pack_w_one(w, j0.out, K, T, C, j0.CS, j0.nks, j0.nct, j0.nslice, j0.dgrad, j0.nt, i);
  else if (i < t0 + t1)
    tile_pack_w_one(w, j1.out, K, T, C, j1.CS, j1.nks, j1.nct, j1.nslice, j1.dgrad, j1.nt, i - t0);
}

// two packings of one weight (p = {CS, nks, nct, nslice, dgrad, nt} each) in one launch
extern "C" int fn_tile_pack_w2(const float* w, void* out0, void* out1, int K, int T, int C, const int* p0,
                               const int* p1, hipStream_t st) {
  const int* ps[2] = {p0, p1};
  TilePackJob j[2];
  long long total = 0;
  for (int q = 0; q < 2; ++q) {
    const int* p = ps[q];
    if (p[0] != 8 && p[0] != 16 && p[0] % 32 != 0) return -2;
    if ((p[5] != 2 && p[5] != 4) || p[2] % p[5]) return -2;   // (nt: the workgroup's 16-column tiles)
    j[q] = TilePackJob{(uint4*)(q ? out1 : out0), p[0], p[1], p[2], p[3], p[4], p[5]};
    total += ((long long)p[3] * p[1] + 4) * p[2] * 64;
  }
  hipLaunchKernelGGL(tile_pack_w2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, K, T, C, j[0],
                     j[1]);
  FN_CHECK_LAUNCH();
  return 0;
}

extern "C" int fn_tile_pack_w(const float* w, void* out, int K, int T, int C, int CS, int nks, int nct, int nslice,
                              int dgrad, int nt, hipStream_t st) {
  if (CS != 8 && CS != 16 && CS % 32 != 0) return -2;
  if ((nt != 2 && nt != 4) || nct % nt) return -2;
  const long long total = ((long long)nslice * nks + 4) * nct * 64;
  hipLaunchKernelGGL(tile_pack_w_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, (uint4*)out, K, T,
                     C, CS, nks, nct, nslice, dgrad, nt);
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------

static int g_tile_cus = 0;
static int g_tile_grid_cap = 0;   // tests: at most this many workgroups per column block (0: none)

extern "C" void fn_conv_tile_grid_cap(int cap) { g_tile_grid_cap = cap > 0 ? cap : 0; }

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

// Schedule of the BN-statistics launches (both deterministic, see conv_tile_kernel):
//   static  -- fixed tiles per workgroup, one partial row per workgroup: the fastest when the
//              kernel has the GPU to itself (1 GPU: 4.61-4.62 vs 4.73-4.76 ms per training step,
//              profiles/r6_dp_interference.md);
//   chunked -- fixed chunks of tiles grabbed dynamically from XCD queues, one partial row per
//              chunk: degrades gracefully when other kernels hold CUs (the RCCL rings of the
//              data-parallel all-reduce overlapping the backward).
// fn_conv_tile_set_schedule: 0 static, 1 chunked; the data-parallel gradient bucketer selects the
// chunked one when the world has more than one rank (parallel/ddp.py).  FN_TILE_SCHED=static /
// chunked overrides.  Chunks: tiles per chunk from the tile count alone (never the grid or the CU
// count: the partial rows -- so the statistics' bits -- are the same on every box), at most
// CT_MAX_CHUNKS chunks, so every workgroup takes dozens and the tail of the dynamic grab is about one
// chunk.
#define CT_MAX_CHUNKS 8192
static int g_tile_sched = -1;     // -1: FN_TILE_SCHED (default static); 0 static, 1 chunked
extern "C" void fn_conv_tile_set_schedule(int mode) { g_tile_sched = mode < 0 ? -1 : (mode ? 1 : 0); }
extern "C" int fn_conv_tile_schedule() {
  static const int env = [] {
    const char* e = getenv("FN_TILE_SCHED");
    return (e && std::string(e) == "chunked") ? 1 : 0;
  }();
  return g_tile_sched < 0 ? env : g_tile_sched;
}
static bool tile_stat_static() { return fn_conv_tile_schedule() == 0; }
static int tile_chunk(const TileGeom& g) {
  if (tile_stat_static()) return 0;
  const long long nt = (long long)g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) *
                       ((g.OW + g.TW - 1) / g.TW);
  return (int)std::max(1LL, (nt + CT_MAX_CHUNKS - 1) / CT_MAX_CHUNKS);
}

// rows of the BN-statistics slab [rows][2][Ncol] a statistics launch writes: one per chunk (or, with
// the static schedule, one per workgroup)
extern "C" int fn_conv_tile_wring(const int* geom, int Ncol, int MT, int NT, int mask);
extern "C" int fn_conv_tile_slab_rows(const int* geom, int Ncol, int NT) {
  const TileGeom g = parse_tile(geom);
  const int c = tile_chunk(g);
  if (c == 0) return fn_conv_tile_workers(geom, Ncol, NT);
  const long long nt = (long long)g.N * ((g.OD + g.TD - 1) / g.TD) * ((g.OH + g.TH - 1) / g.TH) *
                       ((g.OW + g.TW - 1) / g.TW);
  return (int)((nt + c - 1) / c);
}

template <int MT, int NT, int CPP, int DBG = 0, bool F8 = false, bool Q8O = false, bool I8 = false, bool BS = false,
          int NCW = CT_NCW, bool WL = false, bool PRO = false, bool CHK = true>
static int launch_tile(dim3 grid, size_t lds, hipStream_t st, const void* s, const uint4* w, const int2* rt,
                       const int4* kt, const void* zp, const float* b, void* o, float* stats, const TileGeom& g,
                       int Ncol, int act, int* sched, long long* stamps = nullptr, const float* scale = nullptr,
                       float oscale = 0.f, const void* gmask = nullptr, const void* xsc = nullptr,
                       void* osc = nullptr, int chunk = 0, int wring = 0, const float* pst = nullptr,
                       void* pz = nullptr, void* pmask = nullptr, int pact = 0) {
  static size_t configured = 0;
  if (lds > configured) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_tile_kernel<MT, NT, CPP, DBG, F8, Q8O, I8, BS, NCW, WL, PRO, CHK>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    configured = lds;
  }
  hipLaunchKernelGGL((conv_tile_kernel<MT, NT, CPP, DBG, F8, Q8O, I8, BS, NCW, WL, PRO, CHK>), grid, dim3(64 * (NCW + 1)), lds,
                     st, (const unsigned char*)s, w, rt, kt, (const unsigned char*)zp, b, o, stats, g, Ncol, act,
                     sched, stamps, scale, oscale, (const unsigned char*)gmask, (const unsigned*)xsc,
                     (unsigned char*)osc, chunk, wring, pst, (bf16*)pz, (unsigned char*)pmask, pact);
  return 0;
}

// The LDS weight ring (conv_tile_kernel WL): off unless FN_TILE_WLDS=1 (measured slower than the
// register path, profiles/r6_bn_prologue.md), for the bf16 instances whose
// plan leaves room for at least CT_WRING_MIN k-step slots (up to CT_WRING_MAX) in the 160 KiB
#define CT_WRING_MIN 8
#define CT_WRING_MAX 12
static int g_tile_wlds = -1;      // -1: FN_TILE_WLDS (default off); 0 / 1 set by fn_conv_tile_set_wlds (tests)
extern "C" void fn_conv_tile_set_wlds(int mode) { g_tile_wlds = mode < 0 ? -1 : (mode ? 1 : 0); }
static int tile_wring(size_t lds, int NT) {
  static const bool env_on = [] { const char* e = getenv("FN_TILE_WLDS"); return e && atoi(e) == 1; }();
  const bool on = g_tile_wlds < 0 ? env_on : g_tile_wlds == 1;
  if (!on || lds >= 160 * 1024) return 0;
  const int r = (int)std::min<size_t>(CT_WRING_MAX, (160 * 1024 - lds) / ((size_t)NT * 1024));
  return r >= CT_WRING_MIN ? r : 0;
}

// instantiations (MT, NT, CPP) -- the Python planner only emits these
#define CT_INSTANCES(X) X(8, 2, 1) X(9, 2, 1) X(8, 2, 2) X(9, 2, 2) X(8, 2, 4) X(9, 2, 4) X(4, 4, 4)

extern "C" int fn_conv_tile_supported(int MT, int NT, int CPP) {
#define CT_SUP(M, N, C) if (MT == M && NT == N && CPP == C) return 1;
  CT_INSTANCES(CT_SUP)
#undef CT_SUP
  return 0;
}

static size_t tile_lds_total(const TileGeom& g, int MT, int NT, bool f8 = false, int Ncol = 0, bool mask = false,
                             bool bs = false, int ncw = CT_NCW) {
  const int PD = ct_pd(NT, f8);
  return 2 * (size_t)g.BUF + 64 + ct_red_bytes(NT, ncw, f8) + (size_t)(g.nks + PD + 2) * 16 * (f8 && bs ? 2 : 1) +
         (size_t)g.HPpad * 8 +
         (f8 ? (size_t)NT * 16 * 8 : 0) + (size_t)ct_mask_lds(ncw * MT * 16, Ncol, mask) +
         (f8 && bs ? 2 * (size_t)g.HPpad * 4 : 0);    // (BS: the two scale planes)
}

// geom: halo geometry (17) + CS, HPpad, nks, nct, mHW, mHHW, BUF (see TileGeom).
// wp: packed weights (fn_tile_pack_w) with PD zero k-steps past the last slice; rowtab:
// int2[4 * MT * 16] (halo position of the row, natural tile row or -1); ktab: int4[nks + PD
// + 2] byte offsets of the tap each lane group reads per k-step (zero past nks);
// zp: >= 16 zero bytes; sched: int[1 + 8 * column blocks] zeroed counters (left zero); stats: fp32
// [fn_conv_tile_slab_rows][2][Ncol], or null.  bny (bnp null): the relu-mask bytes [output
// positions][Ncol / 8] of the BN whose output this dgrad's conv consumed -- the epilogue's column
// sums are of g = dx * mask (dx stored as is); stats required, act none.
// osc (oscale > 0 only): block-scaled e4m3 output -- one E8M0 byte per (position, 32-column block)
// into the dword-per-position array osc (byte j = block j); oscale is then only the flag
extern "C" int fn_conv_tile(const void* src, const void* wp, const void* rowtab, const void* ktab, const void* zp,
                            const float* bias, void* out, float* stats, const int* geom, int Ncol, int act, int MT,
                            int NT, int* sched, hipStream_t st, const void* bny, const float* bnp, float oscale,
                            void* osc, const float* pst, void* pz, void* pmask, int pact) {
  const TileGeom g = parse_tile(geom);
  if (g.CS != 8 && g.CS != 16 && g.CS != 32 && g.CS != 64) return -2;
  const int CPP = g.CS / 8;
  if (!fn_conv_tile_supported(MT, NT, CPP)) return -2;
  if (g.C % g.CS || g.TD * g.TH * g.TW > 64 * MT || g.TD < 1 || g.TH < 1 || g.TW < 1) return -3;
  const long long HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const long long HP = (g.TD + g.KD - 1) * HH * HW;
  if (g.HPpad < HP || g.HPpad % 64) return -3;
  if (g.TD + g.KD - 1 > 255 || HH > 255 || HW > 255) return -3;   // packed 8-bit hd/hh/hw
  const int PD = ct_pd(NT, false);
  const int T = g.KD * g.KH * g.KW;
  const int need_ks = g.CS >= 32 ? T * (g.CS / 32) : (g.CS == 16 ? (T + 1) / 2 : (T + 3) / 4);
  if (g.nks % PD || g.nks < need_ks || g.nct < (Ncol + 15) / 16) return -3;
  for (long long r = 0; r < 64LL * MT; ++r) {    // epilogue row decode
    const unsigned long long q = (r * (unsigned long long)g.mTW) >> 32;
    if (q != (unsigned long long)(r / g.TW) || ((q * g.mTH) >> 32) != q / g.TH) return -3;
  }
  // the magic divisors must be exact for every position the DMA rows touch
  for (long long p = 0; p < g.HPpad; p += 1) {
    const unsigned long long hd = ((unsigned long long)p * g.mHHW) >> 32;
    const unsigned long long rem = p - hd * HH * HW;
    if (hd != (unsigned long long)(p / (HH * HW)) || (((rem * g.mHW) >> 32) != rem / HW)) return -3;
  }
  const size_t halo = (size_t)g.HPpad * CPP * 16;
  if ((size_t)g.BUF < halo || g.BUF % 1024) return -3;
  if (bnp || (bny && ((act & 0xff) != ACT_NONE || oscale != 0.f || (Ncol != 32 && Ncol != 64) || !stats))) return -2;
  const size_t lds = tile_lds_total(g, MT, NT, false, Ncol, bny != nullptr);
  if (lds > 160 * 1024) return -4;
  const int ncb = (Ncol + NT * 16 - 1) / (NT * 16);
  if (!sched || !zp || !ktab || ncb > 63 || ncb * NT > g.nct) return -6;   // (sched: int[1 + 8 * 63] and more)
  if (Ncol % 8 || ((act & 0xff) != ACT_NONE && (act & 0xff) != ACT_RELU)) return -2;   // 16-B column groups
  // oscale > 0: e4m3 output of y * oscale (no statistics; the 8-channel-slice instances: the
  // space-to-depth stem of the fp8 inference path)
  if (!(oscale >= 0.f) || (oscale > 0.f && (stats || NT != 2 || CPP != 1))) return -2;
  if (osc && (oscale <= 0.f || Ncol > 128)) return -2;
  // the BN prologue: a bf16 forward (no relu-mask dgrad, no fp8 output), z none / relu
  if (pst && (bny || oscale != 0.f || osc || pact != ACT_RELU)) return -2;   // (relu only)
  if (!pst && (pz || pmask)) return -2;
  dim3 grid((unsigned)fn_conv_tile_workers(geom, Ncol, NT), (unsigned)ncb);
  // (tests: a smaller grid must give the same bits -- only the dynamic schedules take it)
  if (g_tile_grid_cap > 0 && (!stats || tile_chunk(g) > 0)) grid.x = std::min<unsigned>(grid.x, g_tile_grid_cap);
  const int wring = (oscale > 0.f || osc || pst) ? 0 : tile_wring(lds, NT);   // (the ring's loader: no prologue)
  // (timing only: FN_TILE_WLDBG=1 the ring without its hand-off, 3 also without the weight DMAs)
  static const int wl_dbg = [] { const char* e = getenv("FN_TILE_WLDBG"); return e ? atoi(e) : 0; }();
  if (wring && (wl_dbg & 1)) act |= 0x400;
  if (wring && (wl_dbg & 2)) act |= 0x800;
  int rc = -2;
#ifdef FN_EXPERIMENTS
  static const int dbg = [] { const char* e = getenv("FN_TILE_DBG"); return e ? atoi(e) : 0; }();
  if (dbg && MT == 8 && NT == 2 && oscale == 0.f) {   // experiment variants (timing only; 1-7, 32 give
                                                              // wrong results; 64, 128, 192 schedule variants)
    static long long* stamps = nullptr;
    const size_t nst = (size_t)grid.x * grid.y * 16;
    if ((dbg & 16) && !stamps && hipMalloc(&stamps, 256 * 64 * 16 * sizeof(long long)) != hipSuccess) return -5;
    if ((dbg & 16) && hipMemsetAsync(stamps, 0, nst * sizeof(long long), st) != hipSuccess) return -5;
#define CT_DBG(C, D) if (CPP == C && dbg == D) rc = launch_tile<8, 2, C, D>(grid, lds, st, src, \
      (const uint4*)wp, (const int2*)rowtab, (const int4*)ktab, zp, bias, out, stats, g, Ncol, act, sched, stamps, \
      nullptr, 0.f, bny, nullptr, nullptr, stats ? tile_chunk(g) : 0);
    CT_DBG(1, 1) CT_DBG(1, 2) CT_DBG(1, 4) CT_DBG(1, 16)   // (the space-to-depth stem)
    CT_DBG(1, 8) CT_DBG(1, 24) CT_DBG(2, 8) CT_DBG(2, 24)
    CT_DBG(2, 1) CT_DBG(2, 2) CT_DBG(2, 4) CT_DBG(2, 3) CT_DBG(2, 7) CT_DBG(2, 16) CT_DBG(4, 16) CT_DBG(2, 23)
    CT_DBG(4, 23) CT_DBG(2, 32) CT_DBG(4, 32) CT_DBG(4, 1) CT_DBG(4, 2) CT_DBG(4, 3) CT_DBG(4, 4) CT_DBG(4, 8)
    CT_DBG(2, 64) CT_DBG(2, 128) CT_DBG(2, 192) CT_DBG(4, 64) CT_DBG(4, 128) CT_DBG(4, 192)   // (correct results)
#undef CT_DBG
    if (rc) return rc;
    FN_CHECK_LAUNCH();
    if (dbg & 16) {                              // mean cycles per workgroup: wave 0 and the loader
      std::vector<long long> h(nst);
      if (hipStreamSynchronize(st) != hipSuccess ||
          hipMemcpy(h.data(), stamps, nst * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -5;
      double m[16] = {0};
      for (size_t i = 0; i < nst; ++i) m[i % 16] += (double)h[i] / (grid.x * grid.y);
      for (int w = 0; w < 2; ++w)
        fprintf(stderr,
                "[conv_tile stamps MT8 CPP%d dbg%d %s] barrierA %.0f job %.0f epilogue %.0f | total %.0f\n", CPP, dbg,
                w ? "loader" : "wave0 ", m[8 * w], m[8 * w + 1], m[8 * w + 2], m[8 * w + 6]);
      fprintf(stderr, "[conv_tile stamps MT8 CPP%d dbg%d wave1 ] barrierA %.0f job %.0f epilogue %.0f | total %.0f\n",
              CPP, dbg, m[3], m[4], m[5], m[7]);
    }
    return 0;
  }
#endif  // FN_EXPERIMENTS
#define CT_CASE(M, N, C)                                                                                          \
  if (MT == M && NT == N && CPP == C)                                                                             \
    rc = oscale > 0.f ? (osc ? launch_tile<M, N, C, 0, false, C == 1 && N == 2, false, C == 1 && N == 2>(        \
                                   grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab, (const int4*)ktab, zp,  \
                                   bias, out, stats, g, Ncol, act, sched, nullptr, nullptr, oscale, nullptr, nullptr, \
                                   osc)                                                                           \
                             : launch_tile<M, N, C, 0, false, C == 1 && N == 2>(                                  \
                                   grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab, (const int4*)ktab, zp,  \
                                   bias, out, stats, g, Ncol, act, sched, nullptr, nullptr, oscale))              \
                      : (wring ? launch_tile<M, N, C, 0, false, false, false, false, CT_NCW, true>(                \
                                     grid, lds + (size_t)wring * N * 1024, st, src, (const uint4*)wp,                 \
                                     (const int2*)rowtab, (const int4*)ktab, zp, bias, out, stats, g, Ncol, act,       \
                                     sched, nullptr, nullptr, 0.f, bny, nullptr, nullptr, stats ? tile_chunk(g) : 0,   \
                                     wring)                                                                            \
                               : (pst ? launch_tile<M, N, C, 0, false, false, false, false, CT_NCW, false, true>(      \
                                            grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab,                 \
                                            (const int4*)ktab, zp, bias, out, stats, g, Ncol, act, sched, nullptr,     \
                                            nullptr, 0.f, bny, nullptr, nullptr, stats ? tile_chunk(g) : 0, 0, pst, pz, \
                                            pmask, pact)                                                              \
                                      : ((stats && tile_chunk(g) > 0)                                          \
                                             ? launch_tile<M, N, C>(grid, lds, st, src, (const uint4*)wp,              \
                                                                    (const int2*)rowtab, (const int4*)ktab, zp, bias,  \
                                                                    out, stats, g, Ncol, act, sched, nullptr, nullptr, \
                                                                    0.f, bny, nullptr, nullptr, tile_chunk(g))         \
                                             : launch_tile<M, N, C, 0, false, false, false, false, CT_NCW, false,      \
                                                           false, false>(grid, lds, st, src, (const uint4*)wp,         \
                                                                         (const int2*)rowtab, (const int4*)ktab, zp,   \
                                                                         bias, out, stats, g, Ncol, act, sched,        \
                                                                         nullptr, nullptr, 0.f, bny, nullptr,          \
                                                                         nullptr, 0))));
  CT_INSTANCES(CT_CASE)
#undef CT_CASE
  if (rc) return rc;
  FN_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// fp8 (e4m3) inference launcher
// ---------------------------------------------------------------------------
// As fn_conv_tile with fp8 bytes for src / wp (packed by the host: [slice][k-step][16-col
// tile][lane][32 B], the same column order, + 4 zero k-steps) and per-column dequantisation
// scale[Ncol] (s_x * s_w[co]); oscale > 0 stores e4m3 of y * oscale, 0 stores bf16.
// (MT = 9 spills at the fp8 fragment sizes: 8 only)
#define CT_F8_INSTANCES(X) X(8, 2, 2) X(8, 2, 4)

extern "C" int fn_conv_tile_f8_supported(int MT, int NT, int CPP) {
#define CT_SUP(M, N, C) if (MT == M && NT == N && CPP == C) return 1;
  CT_F8_INSTANCES(CT_SUP)
#undef CT_SUP
  return 0;
}

// xsc (optional): block-scaled input -- one E8M0 byte per (input position, 32-channel block) in a
// dword per position; scale then holds the weights' per-column dequantisation only.  osc (with
// xsc, oscale > 0): block-scaled e4m3 output (the same layout; oscale is then only the flag).
extern "C" int fn_conv_tile_f8(const void* src, const void* wp, const void* rowtab, const void* ktab, const void* zp,
                               const float* scale, const float* bias, void* out, float oscale, const int* geom, int Ncol,
                               int relu, int MT, int NT, int* sched, hipStream_t st, const void* xsc, void* osc) {
  const TileGeom g = parse_tile(geom);
  if (g.CS != 32 && g.CS != 64) return -2;
  const int CPP = g.CS / 16;
  if (!fn_conv_tile_f8_supported(MT, NT, CPP) || !scale || !(oscale >= 0.f)) return -2;
  // relu: bit 0 relu, bit 1 the fused 2^3 max-pool (relu, bf16 output [N][OD/2][OH/2][OW/2][Ncol];
  // even tile dims so every window lies in one tile, the pool row table, MT = 8), bit 2 int8
  // operands (src / wp hold int8, scale dequantises the int32 sums; 32-channel slices, no pool)
  const bool pool = (relu & 2) != 0;
  const bool i8 = (relu & 4) != 0;
  if (i8 && (pool || CPP != 2 || MT != 8 || NT != 2)) return -2;
  const bool bs = xsc != nullptr;
  if ((bs && (i8 || g.C > 128)) || (osc && (!bs || oscale <= 0.f || Ncol > 128))) return -2;
  if (pool && (MT != 8 || oscale != 0.f || (g.TD | g.TH | g.TW | g.OD | g.OH | g.OW) & 1)) return -2;
  const int f8act = ((relu & 1) || pool ? ACT_RELU : ACT_NONE) | (pool ? CT_F8_POOL : 0);
  if (g.C % g.CS || g.TD * g.TH * g.TW > 64 * MT || g.TD < 1 || g.TH < 1 || g.TW < 1) return -3;
  const long long HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const long long HP = (g.TD + g.KD - 1) * HH * HW;
  if (g.HPpad < HP || g.HPpad % 64) return -3;
  if (g.TD + g.KD - 1 > 255 || HH > 255 || HW > 255) return -3;
  const int PD = ct_pd(NT, true);
  const int T = g.KD * g.KH * g.KW;
  const int need_ks = g.CS == 32 ? (T + 3) / 4 : (T + 1) / 2;
  if (g.nks % PD || g.nks < need_ks || g.nct < (Ncol + 15) / 16) return -3;
  for (long long p = 0; p < g.HPpad; p += 1) {
    const unsigned long long hd = ((unsigned long long)p * g.mHHW) >> 32;
    const unsigned long long rem = p - hd * HH * HW;
    if (hd != (unsigned long long)(p / (HH * HW)) || (((rem * g.mHW) >> 32) != rem / HW)) return -3;
  }
  if ((size_t)g.BUF < (size_t)g.HPpad * CPP * 16 || g.BUF % 1024) return -3;
  const size_t lds = tile_lds_total(g, MT, NT, true, 0, false, bs);
  if (lds > 160 * 1024) return -4;
  const int ncb = (Ncol + NT * 16 - 1) / (NT * 16);
  if (!sched || !zp || !ktab || ncb > 63 || ncb * NT > g.nct) return -6;
  if (Ncol % 8) return -2;
  if (bs) {                                      // (block-scaled operands: the production instances only)
#define CT_F8_BS(M, N, C)                                                                                          \
    if (MT == M && NT == N && CPP == C)                                                                            \
      rc = launch_tile<M, N, C, 0, true, false, false, true>(grid, lds, st, src, (const uint4*)wp,                  \
                                                             (const int2*)rowtab, (const int4*)ktab, zp, bias, out, \
                                                             nullptr, g, Ncol, f8act, sched, nullptr, scale, oscale, \
                                                             nullptr, xsc, osc);
    dim3 grid((unsigned)fn_conv_tile_workers(geom, Ncol, NT), (unsigned)ncb);
    int rc = -2;
    CT_F8_INSTANCES(CT_F8_BS)
#undef CT_F8_BS
    if (rc) return rc;
    FN_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((unsigned)fn_conv_tile_workers(geom, Ncol, NT), (unsigned)ncb);
  int rc = -2;
  // FN_F8_DBG (timing experiments only, wrong results): 1 no weight loads, 2 no halo reads,
  // 4 no halo DMA (and sums of them), 16 cycle stamps (barrier-A wait, job, epilogue)
#ifdef FN_EXPERIMENTS
  static const int f8dbg = [] { const char* e = getenv("FN_F8_DBG"); return e ? atoi(e) : 0; }();
  if (f8dbg) {
    static long long* stamps = nullptr;
    const size_t nst = (size_t)grid.x * grid.y * 16;
    if ((f8dbg & 16) && !stamps && hipMalloc(&stamps, 256 * 64 * 16 * sizeof(long long)) != hipSuccess) return -5;
    if ((f8dbg & 16) && hipMemsetAsync(stamps, 0, nst * sizeof(long long), st) != hipSuccess) return -5;
#define CT_F8_DBG(C, D) if (MT == 8 && NT == 2 && CPP == C && f8dbg == D) \
    rc = launch_tile<8, 2, C, D, true>(grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab, (const int4*)ktab, \
                                       zp, bias, out, nullptr, g, Ncol, f8act, sched, stamps, scale, oscale);
    CT_F8_DBG(2, 1) CT_F8_DBG(2, 2) CT_F8_DBG(2, 3) CT_F8_DBG(2, 4) CT_F8_DBG(2, 7) CT_F8_DBG(2, 16)
    CT_F8_DBG(4, 1) CT_F8_DBG(4, 2) CT_F8_DBG(4, 3) CT_F8_DBG(4, 4) CT_F8_DBG(4, 7) CT_F8_DBG(4, 16)
#undef CT_F8_DBG
    if (rc) return rc;
    FN_CHECK_LAUNCH();
    if (f8dbg & 16) {
      std::vector<long long> h(nst);
      if (hipStreamSynchronize(st) != hipSuccess ||
          hipMemcpy(h.data(), stamps, nst * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -5;
      double m[16] = {0};
      for (size_t i = 0; i < nst; ++i) m[i % 16] += (double)h[i] / (grid.x * grid.y);
      for (int w = 0; w < 2; ++w)
        fprintf(stderr, "[conv_tile_f8 stamps CPP%d %s] barrierA %.0f job %.0f epilogue %.0f | total %.0f\n", CPP,
                w ? "loader" : "wave0 ", m[8 * w], m[8 * w + 1], m[8 * w + 2], m[8 * w + 6]);
    }
    return 0;
  }
#endif  // FN_EXPERIMENTS
#ifdef FN_EXPERIMENTS
#define CT_F8_CASE(M, N, C)                                                                                        \
  if (MT == M && NT == N && CPP == C)                                                                              \
    rc = i8 ? launch_tile<M, N, C, 0, true, false, C == 2>(grid, lds, st, src, (const uint4*)wp,                     \
                                                                  (const int2*)rowtab, (const int4*)ktab, zp, bias, \
                                                                  out, nullptr, g, Ncol, f8act, sched, nullptr,    \
                                                                  scale, oscale)                                   \
            : launch_tile<M, N, C, 0, true>(grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab,              \
                                            (const int4*)ktab, zp, bias, out, nullptr, g, Ncol, f8act, sched,      \
                                            nullptr, scale, oscale);
#else   // (the int8 stem instance is an experiment build: measured no faster, and seed-dependent top-1)
  if (i8) return -2;
#define CT_F8_CASE(M, N, C)                                                                                        \
  if (MT == M && NT == N && CPP == C)                                                                              \
    rc = launch_tile<M, N, C, 0, true>(grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab,                   \
                                       (const int4*)ktab, zp, bias, out, nullptr, g, Ncol, f8act, sched, nullptr,  \
                                       scale, oscale);
#endif
  CT_F8_INSTANCES(CT_F8_CASE)
#undef CT_F8_CASE
  if (rc) return rc;
  FN_CHECK_LAUNCH();
  return 0;
}

// k-step slots of the LDS weight ring a bf16 launch of this plan gets (0: the register path) --
// the test / profile hook for which path a layer takes
extern "C" int fn_conv_tile_wring(const int* geom, int Ncol, int MT, int NT, int mask) {
  const TileGeom g = parse_tile(geom);
  return tile_wring(tile_lds_total(g, MT, NT, false, Ncol, mask != 0), NT);
}
