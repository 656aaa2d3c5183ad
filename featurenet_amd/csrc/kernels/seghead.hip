// Segmentation classifier head + per-voxel softmax cross-entropy + the head's whole backward in ONE
// streaming pass (FeatureNet3DSeg training, ops/subpixel.py SubpixelDecoderHeadLossFn).
//
// The 1x1x1 head maps the decoder output z = act(bn(y)) [M][32] to per-voxel logits [M][NC] and
// the loss is their mean cross-entropy.  Unfused, a training step writes the logits (1.7 GB at
// 128 x 64^3), the loss kernel reads them and writes d(logits), and the backward reads
// d(logits) three more times: head weight gradient (with z), bias gradient, head dgrad (with y,
// plus the decoder BN's backward moments).  Everything the backward needs from d(logits) is
// linear in it and local to a voxel row, so this kernel computes it while the tile is in LDS:
//
//   per 256-row tile:  y (raw, for the BN moments) and z = act(y*sc + sh) into LDS
//                      logits = z W^T + b            (MFMA 16x16x32, W^T fragments in registers)
//                      one row per thread: log-sum-exp loss, top-1 hit,
//                      d = (softmax - target) * xscale  (bf16, the unfused kernel's values)
//                      dW^T += z^T d, db += 1^T d    (MFMA; both operands ds_read_b64_tr_b16)
//                      dz = d W                      (MFMA; W fragments in registers)
//                      BN moments: g = dz * act'(y*sc + sh), sum g, sum g * y per channel
//                      dz -> HBM (16-B stores through LDS)
//
// HBM traffic: y and the labels in, dz out -- the logits and d(logits) never exist.  Partials are
// per workgroup (fixed-order reductions: deterministic); the host sums them.
//
// Reference parity: the softmax head + categorical cross-entropy (reference
// model/keras_model.py:124, tensorflow_generator.py:232-235), Keras Conv (1,1) head
// (model/input.py:294).
#include "common.h"
#include "conv_tile_shared.h"

#include <type_traits>

#define SH_BM 256
#define SH_NTHR 256
#define SH_K 32                                  // decoder channels (the head's input)
#define SH_LD 40                                 // LDS row stride (bf16): 80 B

typedef short sh_s4 __attribute__((ext_vector_type(4)));
typedef short sh_s8 __attribute__((ext_vector_type(8)));

// 8 consecutive rows of one column (rows lo..lo+3 and hi..hi+3 of the lane's 16-lane group) as
// an MFMA operand fragment: lane 4q+p of the group addresses row q, columns 4p..4p+3
__device__ __forceinline__ bf16x8 sh_tr8(const bf16* lo, const bf16* hi) {
  sh_s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sh_s4*)(lo));
  sh_s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sh_s4*)(hi));
  sh_s8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ sh_s4 sh_tr4(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sh_s4*)(p));
}

__device__ __forceinline__ float sh_bf(short s) { return __uint_as_float(((unsigned)(unsigned short)s) << 16); }
__device__ __forceinline__ unsigned sh_pack2(float lo, float hi) { return bf16x2_pack(lo, hi); }
__device__ __forceinline__ float bf16_round(float x) { return bf2f(f2bf(x)); }

// ACT: the decoder BN's activation (ACT_NONE / ACT_RELU); LT: the label type (int64, or uint8 --
// NC <= 32 classes fit a byte: 8x fewer label bytes to copy in and read).
// y [M][32] bf16; sc / sh [32]; w [NC][32] bf16; bias [NC] fp32 or null; labels LT [M];
// dz [M][32] bf16 out; part: per workgroup [loss, hits | db[32] | dWt[32][32] | msum[32] | msq[32]]
// (fp32; dWt[ch][cls] = sum z[r][ch] d[r][cls]).
// NCT: the class count when it is 25 (the FeatureNet3DSeg head: loops of exactly 25 classes, 25
// live logits per row), 32 for any NC <= 32 (runtime bound).  XF: the extras -- top-1 hits and label
// smoothing; the lean instance (a training step that asks for neither, smoothing == 0) skips the
// arg-max and the logit sum, a third of the row's VALU work.
template <int ACT, typename LT, int NCT = 32, bool XF = true>
__global__ __launch_bounds__(SH_NTHR, 2) void seghead_loss_kernel(const bf16* __restrict__ y,
                                                                 const float* __restrict__ sc,
                                                                 const float* __restrict__ shf,
                                                                 const bf16* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 const LT* __restrict__ labels,
                                                                 bf16* __restrict__ dz, float* __restrict__ part,
                                                                 long long M, int NC, float xscale, float smoothing) {
  __shared__ __attribute__((aligned(16))) bf16 Ys[SH_BM * SH_LD];   // raw y
  __shared__ __attribute__((aligned(16))) bf16 Zs[SH_BM * SH_LD];   // z = act(y*sc + sh)
  __shared__ __attribute__((aligned(16))) bf16 Os[SH_BM * SH_LD];   // logits -> d -> dz staging
  constexpr int PW = 2 + 32 + 32 * 32 + 64;      // partial floats per wave / workgroup
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int q = (lane & 15) >> 2, pp = lane & 3;                    // tr_b16 address roles
  const int ntiles = (int)((M + SH_BM - 1) / SH_BM);

  // head weights as MFMA fragments: logits B[k = ch][n = cls] = w[cls][ch] (8 consecutive ch of
  // row cls: 16-B loads), dz B[k = cls][n = ch] = w[cls][ch] (a column gather, once)
  bf16x8 wl[2], wd[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int cls = 16 * nb + lr;
    Pack8 p, r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p.e[j] = cls < NC ? w[cls * SH_K + 8 * lg + j] : f2bf(0.f);
      const int c2 = 8 * lg + j;                                     // class of the dz B fragment
      r.e[j] = c2 < NC ? w[c2 * SH_K + 16 * nb + lr] : f2bf(0.f);
    }
    wl[nb] = __builtin_bit_cast(bf16x8, p.u);
    wd[nb] = __builtin_bit_cast(bf16x8, r.u);
  }
  // (the MFMAs take the weights as A and the voxel rows as B: a lane's accumulator holds 4
  // consecutive classes / channels 16 nb + 4 lg + i of one voxel row 16 mt + lr -- one 8-B LDS
  // store per fragment instead of four 2-B ones)
  // scale / shift / bias in LDS, read where each phase uses them (held in registers for the whole
  // kernel they pushed it past 256 VGPRs: spills)
  __shared__ __attribute__((aligned(16))) float Ps[3 * SH_K];   // [scale 32][shift 32][bias 32]
  if (tid < SH_K) {
    Ps[tid] = sc[tid];
    Ps[SH_K + tid] = shf[tid];
    Ps[2 * SH_K + tid] = (bias && tid < NC) ? bias[tid] : 0.f;
  }
  __syncthreads();
  Pack8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones.e[j] = f2bf(1.f);
  const bf16x8 fone = __builtin_bit_cast(bf16x8, ones.u);

  f32x4 adw[2][2], adb[2];                       // dW^T [ch block][cls block], db [cls block]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    adb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) adw[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  ct_f32x2 ms[2][2], mq[2][2];                   // BN moments of columns 16 nb + 4 lg + 2 h + (0, 1)
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int h = 0; h < 2; ++h) ms[nb][h] = mq[nb][h] = (ct_f32x2){0.f, 0.f};
  float xl = 0.f, xc = 0.f;                       // loss, hits (row threads)

  uint4 rb[4];
  auto load = [&](int t) {                       // tile t: 256 x 32 contiguous bf16 = 1024 chunks
    const long long e0 = (long long)t * SH_BM * SH_K;
    const long long nel = (M - (long long)t * SH_BM < SH_BM ? M - (long long)t * SH_BM : SH_BM) * SH_K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = i * SH_NTHR + tid;
      rb[i] = *(const uint4*)(y + e0 + (c * 8 < nel ? c * 8 : 0));
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    const int rows = (int)(M - (long long)t * SH_BM < SH_BM ? M - (long long)t * SH_BM : SH_BM);
    __syncthreads();                             // the previous tile's LDS readers are done
    // y and z = act(y*sc + sh) into LDS; the zero rows of a partial tile in their own (uniform)
    // branch, so full tiles carry no per-dword selects
    auto stage = [&](auto partial) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = i * SH_NTHR + tid, r = c >> 2, k = (c & 3) * 8;
        Pack8 raw, zz;
        raw.u = rb[i];
        if constexpr (decltype(partial)::value)
          if (r >= rows) raw.u = make_uint4(0u, 0u, 0u, 0u);
        unsigned bits;
        ct_f32x2 psc[4], psh[4];                 // (this thread's chunk: channels 8 (tid mod 4) ..)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          psc[j] = *(const ct_f32x2*)(Ps + 8 * (tid & 3) + 2 * j);
          psh[j] = *(const ct_f32x2*)(Ps + SH_K + 8 * (tid & 3) + 2 * j);
        }
        zz.u = ct_bn_chunk(raw.u, psc, psh, ACT == ACT_RELU, bits);
        if constexpr (decltype(partial)::value)
          if (r >= rows) zz.u = make_uint4(0u, 0u, 0u, 0u);
        *(uint4*)(Ys + r * SH_LD + k) = raw.u;
        *(uint4*)(Zs + r * SH_LD + k) = zz.u;
      }
    };
    if (rows == SH_BM) stage(std::false_type{});
    else stage(std::true_type{});
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);   // next tile in flight
    // ---- logits = z W^T + b: wave rows 64 wave + 16 mt ----
    {
      f32x4 acc[4][2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 fa = *(const bf16x8*)(Zs + (64 * wave + 16 * mt + lr) * SH_LD + 8 * lg);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mt][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[nb], fa, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          *(uint2*)(Os + (64 * wave + 16 * mt + lr) * SH_LD + 16 * nb + 4 * lg) =
              make_uint2(sh_pack2(acc[mt][nb][0] + Ps[2 * SH_K + 16 * nb + 4 * lg], acc[mt][nb][1] + Ps[2 * SH_K + 16 * nb + 4 * lg + 1]),
                         sh_pack2(acc[mt][nb][2] + Ps[2 * SH_K + 16 * nb + 4 * lg + 2], acc[mt][nb][3] + Ps[2 * SH_K + 16 * nb + 4 * lg + 3]));
    }
    __syncthreads();
    // ---- softmax cross-entropy, one row per thread: d (bf16) replaces the logits ----
    {
      // (the row moves as four 16-B LDS accesses each way: rows are 80 B apart, so the 16-lane
      // groups of ds_read_b128 hit 16 distinct bank slots; scalar 2-B accesses were 4-way)
      bf16* orow = Os + tid * SH_LD;
      if (tid < rows) {
        const long long yl = (long long)labels[(long long)t * SH_BM + tid];
        const float off = XF ? smoothing / (float)NC : 0.f, on = XF ? 1.f - smoothing + off : 1.f;
        Pack8 lv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) lv[j].u = *(const uint4*)(orow + 8 * j);
        // (NCT = 25: the loops end at the real class count, no padded-class selects)
        auto live = [&](int c) { return NCT != 32 || c < NC; };
        // the target class enters through its own LDS read and a fix-up store, not a compare and
        // select per class (the one-hot selects were a third of the row's VALU work)
        const int ylab = (int)yl;
        const bool yin = yl >= 0 && yl < NC;
        const float vy = yin ? bf2f(orow[ylab]) : 0.f;
        float v[NCT];
        float mx = -INFINITY, vs = 0.f;
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
          v[c] = live(c) ? bf2f(lv[c >> 3].e[c & 7]) : -INFINITY;
          mx = fmaxf(mx, v[c]);
          if constexpr (XF)
            if (live(c)) vs += v[c];
        }
        int am = 0;                              // the first arg-max (bf16 logits tie often)
        if constexpr (XF) {
#pragma unroll
          for (int c = NCT - 1; c >= 0; --c)
            if (live(c) && v[c] == mx) am = c;
        }
        // one exp per class: e_c = exp(v_c - max) = exp2(v_c log2e - max log2e) (one fma, one
        // v_exp_f32, pairs on v_pk_fma_f32) serves the sum and the softmax (e_c / sum); padded
        // classes are -inf -> 0.  The loss -sum_c tgt_c (v_c - lse) = lse - off * sum_c v_c - (on - off) v_y
        constexpr float L2E = 1.4426950408889634f;
        const ct_f32x2 l2e = {L2E, L2E}, nml = {-mx * L2E, -mx * L2E};
        ct_f32x2 sp = {0.f, 0.f};
#pragma unroll
        for (int c = 0; c + 1 < NCT; c += 2) {
          const ct_f32x2 a = __builtin_elementwise_fma((ct_f32x2){v[c], v[c + 1]}, l2e, nml);
          v[c] = __builtin_amdgcn_exp2f(a.x);
          v[c + 1] = __builtin_amdgcn_exp2f(a.y);
          sp += (ct_f32x2){v[c], v[c + 1]};
        }
        if constexpr (NCT % 2) {
          v[NCT - 1] = __builtin_amdgcn_exp2f(__builtin_fmaf(v[NCT - 1], L2E, nml.x));
          sp.x += v[NCT - 1];
        }
        const float se = sp.x + sp.y;
        const float lse = mx + __logf(se), inv = 1.f / se;
        const float lrow = XF ? lse - (off * vs + (yin ? (on - off) * vy : 0.f)) : lse - (yin ? vy : 0.f);
        // d = (softmax - off) * xscale = e * (inv xscale) - off xscale, pairs on v_pk_fma_f32
        const ct_f32x2 ix = {inv * xscale, inv * xscale}, ox = {-off * xscale, -off * xscale};
#pragma unroll
        for (int c = 0; c < 32; c += 2) {
          ct_f32x2 d = {0.f, 0.f};
          if (c < NCT) {
            d = __builtin_elementwise_fma((ct_f32x2){v[c], v[c + 1 < NCT ? c + 1 : c]}, ix, ox);
            if (!live(c)) d.x = 0.f;
            if (!(c + 1 < NCT && live(c + 1))) d.y = 0.f;   // (padded classes: 0)
          }
          lv[c >> 3].e[c & 7] = f2bf(d.x);
          lv[(c + 1) >> 3].e[(c + 1) & 7] = f2bf(d.y);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) *(uint4*)(orow + 8 * j) = lv[j].u;
        if (yin)                                 // the target's d
          orow[ylab] = f2bf(__builtin_amdgcn_exp2f(__builtin_fmaf(vy, L2E, nml.x)) * ix.x - on * xscale);
        xl += lrow;
        if constexpr (XF) xc += (am == ylab) ? 1.f : 0.f;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) *(uint4*)(orow + 8 * j) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    __syncthreads();
    // ---- dW^T += z^T d and db += 1^T d over the wave's 64 rows (2 k-steps of 32 rows) ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = 64 * wave + 32 * ks + 8 * lg;      // this lane group's 8 rows
      bf16x8 fz[2], fd[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        fz[b] = sh_tr8(Zs + (r0 + q) * SH_LD + 16 * b + 4 * pp, Zs + (r0 + 4 + q) * SH_LD + 16 * b + 4 * pp);
        fd[b] = sh_tr8(Os + (r0 + q) * SH_LD + 16 * b + 4 * pp, Os + (r0 + 4 + q) * SH_LD + 16 * b + 4 * pp);
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          adw[cb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fz[cb], fd[nb], adw[cb][nb], 0, 0, 0);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) adb[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fone, fd[nb], adb[nb], 0, 0, 0);
    }
    // ---- dz = d W (rows 64 wave + 16 mt), the BN moments from y ----
    f32x4 dzc[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const bf16x8 fa = *(const bf16x8*)(Os + (64 * wave + 16 * mt + lr) * SH_LD + 8 * lg);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        dzc[mt][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wd[nb], fa, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int row = 64 * wave + 16 * mt + lr;      // the lane's voxel row, channels 16 nb + 4 lg + i
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const uint2 y4 = *(const uint2*)(Ys + row * SH_LD + 16 * nb + 4 * lg);
        const unsigned yw[2] = {y4.x, y4.y};
#pragma unroll
        for (int h = 0; h < 2; ++h) {               // channel pairs: v_pk_fma_f32 / v_pk_add_f32
          const unsigned dp = bf16x2_pack(dzc[mt][nb][2 * h], dzc[mt][nb][2 * h + 1]);   // the stored dz
          ct_f32x2 g = {bf16_lo(dp), bf16_hi(dp)};
          const ct_f32x2 yy = {bf16_lo(yw[h]), bf16_hi(yw[h])};
          if constexpr (ACT == ACT_RELU) {          // g = dz * relu'(z), z > 0 <=> y * sc + sh > 0
            const ct_f32x2 msc = *(const ct_f32x2*)(Ps + 16 * nb + 4 * lg + 2 * h);
            const ct_f32x2 msh = *(const ct_f32x2*)(Ps + SH_K + 16 * nb + 4 * lg + 2 * h);
            const ct_f32x2 tz = __builtin_elementwise_fma(yy, msc, msh);
            g.x = tz.x > 0.f ? g.x : 0.f;
            g.y = tz.y > 0.f ? g.y : 0.f;
          }
          ms[nb][h] += g;
          mq[nb][h] = __builtin_elementwise_fma(g, yy, mq[nb][h]);
        }
      }
    }
    __syncthreads();                             // every wave is done with d (Os) of this tile
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        *(uint2*)(Os + (64 * wave + 16 * mt + lr) * SH_LD + 16 * nb + 4 * lg) =
            make_uint2(sh_pack2(dzc[mt][nb][0], dzc[mt][nb][1]), sh_pack2(dzc[mt][nb][2], dzc[mt][nb][3]));
    __syncthreads();
    // dz rows -> HBM: 256 x 32 contiguous bf16, 16-B chunks
    {
      bf16* dst = dz + (long long)t * SH_BM * SH_K;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = i * SH_NTHR + tid, r = c >> 2, k = (c & 3) * 8;
        if (r < rows) *(uint4*)(dst + c * 8) = *(const uint4*)(Os + r * SH_LD + k);
      }
    }
  }
  // ---- workgroup partials (fixed order) ----
  // moments: the 16 lanes lr of lane group lg hold columns 16 nb + 4 lg + i
  float msf[2][4], mqf[2][4];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      msf[nb][i] = ms[nb][i >> 1][i & 1];
      mqf[nb][i] = mq[nb][i >> 1][i & 1];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        msf[nb][i] += __shfl_xor(msf[nb][i], o, 64);
        mqf[nb][i] += __shfl_xor(mqf[nb][i], o, 64);
      }
    }
  xl = wave_sum(xl);
  xc = wave_sum(xc);
  __syncthreads();                               // (Ys / Zs are free: the per-wave partials go there)
  float* red = reinterpret_cast<float*>(Ys);     // [4][PW] floats = 18 KB of the 40 KB of Ys + Zs
  float* rw = red + wave * PW;
  if (lane == 0) {
    rw[0] = xl;
    rw[1] = xc;
  }
  // db: every row of the C fragment holds the column sums; lanes of group 0 row 0
  if (lg == 0) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) rw[2 + 16 * nb + lr] = adb[nb][0];
  }
  // dW^T [ch][cls]: C row = ch = 16 cb + 4 lg + i, column = cls = 16 nb + lr
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) rw[34 + (16 * cb + 4 * lg + i) * 32 + 16 * nb + lr] = adw[cb][nb][i];
  if (lr == 0) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        rw[34 + 1024 + 16 * nb + 4 * lg + i] = msf[nb][i];
        rw[34 + 1024 + 32 + 16 * nb + 4 * lg + i] = mqf[nb][i];
      }
  }
  __syncthreads();
  float* out = part + (long long)blockIdx.x * PW;
  for (int i = tid; i < PW; i += SH_NTHR) out[i] = (red[i] + red[PW + i]) + (red[2 * PW + i] + red[3 * PW + i]);
}

extern "C" int fn_seghead_part_len() { return 2 + 32 + 32 * 32 + 64; }

extern "C" int fn_seghead_blocks(long long M) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus <= 0)
      cus = 256;
  }
  const long long tiles = (M + SH_BM - 1) / SH_BM;
  const long long g = 2LL * cus;                 // (~60 KB of LDS: 2 workgroups per CU)
  return (int)(tiles < g ? (tiles > 0 ? tiles : 1) : g);
}

// y [M][32] bf16 (M % 8 == 0), sc / sh [32], w [NC][32] bf16 (NC <= 32), bias [NC] or null,
// labels int64 [M] (lab8 = 0) or uint8 [M] (lab8 = 1), dz [M][32] bf16, part fp32
// [fn_seghead_blocks(M)][fn_seghead_part_len()]; hits = 0: the caller does not read part's hits
// column (0 there with smoothing == 0 and 25 classes)
extern "C" int fn_seghead_loss(const void* y, const float* sc, const float* sh, const void* w, const float* bias,
                               const void* labels, void* dz, float* part, long long M, int K, int NC, int act,
                               float xscale, float smoothing, hipStream_t st, int lab8, int hits) {
  if (K != SH_K || NC < 2 || NC > 32 || M < 8 || M % 8 || !sc || !sh || !labels || !part) return -2;
  if (act != ACT_RELU && act != ACT_NONE) return -2;
  const dim3 grid((unsigned)fn_seghead_blocks(M));
  // the lean instances (no hits, no smoothing: a training step) for the 25-class head
  const bool lean = !hits && smoothing == 0.f;
#define SH_LAUNCH(A, T)                                                                                       \
  if (NC == 25 && lean)                                                                                       \
    hipLaunchKernelGGL((seghead_loss_kernel<A, T, 25, false>), grid, dim3(SH_NTHR), 0, st, (const bf16*)y, sc,  \
                       sh, (const bf16*)w, bias, (const T*)labels, (bf16*)dz, part, M, NC, xscale, smoothing);   \
  else if (NC == 25)                                                                                          \
    hipLaunchKernelGGL((seghead_loss_kernel<A, T, 25>), grid, dim3(SH_NTHR), 0, st, (const bf16*)y, sc, sh,     \
                       (const bf16*)w, bias, (const T*)labels, (bf16*)dz, part, M, NC, xscale, smoothing);       \
  else                                                                                                        \
    hipLaunchKernelGGL((seghead_loss_kernel<A, T>), grid, dim3(SH_NTHR), 0, st, (const bf16*)y, sc, sh,         \
                       (const bf16*)w, bias, (const T*)labels, (bf16*)dz, part, M, NC, xscale, smoothing)
  if (act == ACT_RELU) {
    if (lab8) SH_LAUNCH(ACT_RELU, unsigned char); else SH_LAUNCH(ACT_RELU, long long);
  } else {
    if (lab8) SH_LAUNCH(ACT_NONE, unsigned char); else SH_LAUNCH(ACT_NONE, long long);
  }
#undef SH_LAUNCH
  FN_CHECK_LAUNCH();
  return 0;
}
