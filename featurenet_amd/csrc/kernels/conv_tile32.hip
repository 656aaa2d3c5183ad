// Big-tile LDS-halo implicit-GEMM convolution (stride 1, 3-D, bf16) on v_mfma_f32_32x32x16_bf16.
//
// The same workgroup, job protocol, halo layout (chunk-planar, LDS-DMA double buffer filled by
// a loader wave), row table and weight stream as conv_tile_kernel (conv_tile.hip), with the
// k-loop on the 32x32x16 MFMA instead of 16x16x32:
//
//   * a compute wave owns MB blocks of 32 output positions x the workgroup's 32 columns; per
//     32-k step and block it issues 2 MFMAs (k halves j = 0, 1) of 32 cycles each, with one
//     halo fragment read (32 positions x 16 k = 1 KB) per MFMA;
//   * per MFMA cycle that is half the MFMA instructions of the 16x16x32 loop (which issues two
//     16-cycle MFMAs per halo read): each MFMA holds the SIMD's vector issue for 8 of its 32
//     cycles instead of 8 of 16, so the per-read bookkeeping (address add, wait, B-ring load)
//     has room beside the MFMAs -- the 16x16x32 loop measured at ~72 % MFMA issue, bound by
//     exactly that (profiles/r3_pmc_train_step.md);
//   * MFMA operands: A = weights (32 output channels x 16 k; packed by tile_pack_w mode 32 so
//     MFMA row m is output column 16*((m>>2)&1) + (m&3) + 4*(m>>3)), B = halo (16 k x 32
//     positions).  The accumulator is C^T with lane l holding position l&31 and, after the
//     row permutation, the 16 consecutive channels 16*(l>>5) .. +15: two 16-B stores per
//     position straight from registers;
//   * k-table: per k-step and lane half h, the byte offsets (tap + chunk plane) of the two
//     sub-steps: CS >= 32 one tap x 32 channels (chunk 4s + 2j + h), CS = 16 taps 2k + j (chunk
//     h), CS = 8 taps 4k + 2j + h (chunk 0).
//
// Reference parity: Keras Conv2D/Conv3D (reference model/input.py:294); dgrad uses the same
// kernel on dy with the flipped, transposed kernel (as conv_tile_kernel).
#include "conv_tile_shared.h"

#include <type_traits>

#define C32_PD 4                               // weight-ring depth (k-steps in flight)

__device__ __forceinline__ float c32_sum32(float x) {
  // sum over the 32 lanes of a wave half (rows 0-1 / rows 2-3): DPP row sum, then the partner row
  x = ct_sum16(x);
  return x + __shfl_xor(x, 16, 64);
}

// MB: 32-row MFMA blocks per compute wave (tile rows <= 128 MB); CPP: 16-B chunks per halo position
// of a slice (CS / 8); Q8O: e4m3 output of v * oscale (the fp8 inference stem), no statistics.
// BWS: the dgrad of a conv whose input was act(bn(y)) (ops/bnfuse.py): the stored dx is that BN's
// dz, and the epilogue also sums the BN's raw backward moments (sum g, sum g*y; g = dz * act'(z))
// from y (bny) at the tile's positions and the BN's scale / shift (bnp rows 2, 3) -- the separate
// colstats pass over dz and y disappears (bn_finalize mode 2 centres the moments in fp64).
template <int MB, int CPP, bool Q8O = false, bool BWS = false>
__global__ __launch_bounds__(CT_NTHR, 1) void conv_tile32_kernel(const unsigned char* __restrict__ src,
                                                                 const uint4* __restrict__ wp,
                                                                 const int2* __restrict__ rowtab,
                                                                 const int4* __restrict__ ktab,
                                                                 const unsigned char* __restrict__ zp,
                                                                 const float* __restrict__ bias, void* __restrict__ out,
                                                                 float* __restrict__ stats, TileGeom g, int Ncol,
                                                                 int act, int* __restrict__ sched, float oscale,
                                                                 const bf16* __restrict__ bny,
                                                                 const float* __restrict__ bnp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  constexpr int PD = C32_PD;
  constexpr int RC = 32;                         // columns of the workgroup
  constexpr int ESZ = 2;
  const int HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const int HP = (g.TD + g.KD - 1) * HH * HW;
  const int tdn = (g.OD + g.TD - 1) / g.TD, thn = (g.OH + g.TH - 1) / g.TH, twn = (g.OW + g.TW - 1) / g.TW;
  const int ntiles = g.N * tdn * thn * twn;
  const int nslice = g.C / g.CS;
  const int nks = g.nks;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = wave == CT_NCW;
  const int r32 = lane & 31, hf = lane >> 5;     // position row of the block, k / channel half
  const int ct0 = blockIdx.y * 2;                // first 16-column fragment of the workgroup
  // LDS: [buffer 0][buffer 1][job slots 64 B][BN partials 4 x 2 x 32][k-table (nks+PD+2) int4]
  // [halo positions HPpad int2][bias 32 floats][BWS: (scale, shift) 32 float2]
  int* s_job = reinterpret_cast<int*>(dsm + 2 * g.BUF);
  float* s_red = reinterpret_cast<float*>(dsm + 2 * g.BUF + 64);
  int4* s_kt = reinterpret_cast<int4*>(dsm + 2 * g.BUF + 64 + ct_red_bytes(2));
  int2* s_pos = reinterpret_cast<int2*>(s_kt + (nks + PD + 2));
  float* s_bias = reinterpret_cast<float*>(s_pos + g.HPpad);
  float2* s_bn = reinterpret_cast<float2*>(s_bias + RC);
  for (int i = tid; i < nks + PD + 2; i += CT_NTHR) s_kt[i] = ktab[i];
  for (int i = tid; i < ct_red_bytes(2) / 4; i += CT_NTHR) s_red[i] = 0.f;
  if (tid < RC) {
    const int c = blockIdx.y * RC + tid;
    s_bias[tid] = (bias && c < Ncol) ? bias[c] : 0.f;
    if constexpr (BWS) s_bn[tid] = c < Ncol ? make_float2(bnp[2 * Ncol + c], bnp[3 * Ncol + c]) : make_float2(0.f, 0.f);
  }
  for (int p = tid; p < g.HPpad; p += CT_NTHR) {  // positions past HP repeat the last one
    const int pc = p < HP ? p : HP - 1;
    const int hd = pc / (HH * HW), hh = (pc / HW) % HH, hw = pc % HW;
    s_pos[p] = make_int2(((hd * g.IH + hh) * g.IW + hw) * g.C * ESZ, (hd << 16) | (hh << 8) | hw);
  }
  // per compute lane: position row r32 of each 32-row block mb (row-table fragments 2mb, 2mb+1)
  int lb[MB], roff[MB], rpk[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int2 rt = rowtab[((loader ? 0 : wave) * MB + mb) * 32 + r32];
    lb[mb] = rt.x * 16;
    const int tw = rt.y % g.TW, th = (rt.y / g.TW) % g.TH, td = rt.y / (g.TW * g.TH);
    roff[mb] = rt.y < 0 ? -1 : td * g.osd + th * g.osh + tw * g.osw;
    rpk[mb] = (td << 16) | (th << 8) | tw;
  }

  if (tid == 0) {
    const int t0 = atomicAdd(sched + 1 + blockIdx.y, 1);
    s_job[0] = t0 < ntiles ? t0 : -1;
    s_job[1] = 0;
  }
  tile_lds_barrier();

  if (loader) {
    // ======================= loader wave (as conv_tile_kernel) =======================
    int tile = __builtin_amdgcn_readfirstlane(s_job[0]), slice = 0, t_next = -1;
    if (tile >= 0) {
      ct_dma_job<CPP, ESZ>(g, src, zp, dsm, s_pos, tile, 0, 0, lane, tdn, thn, twn);
      if (lane == 0) t_next = atomicAdd(sched + 1 + blockIdx.y, 1);
      t_next = __builtin_amdgcn_readfirstlane(t_next);
      if (t_next >= ntiles) t_next = -1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int par = 0;
    while (true) {
      tile_lds_barrier();                        // A: job halo landed; the other buffer is free
      if (tile < 0) break;
      int ntile = tile, nslc = slice + 1;
      if (nslc == nslice) {
        nslc = 0;
        ntile = t_next;
      }
      if (lane == 0) {
        s_job[2 * (par ^ 1)] = ntile;
        s_job[2 * (par ^ 1) + 1] = nslc;
      }
      if (ntile >= 0) ct_dma_job<CPP, ESZ>(g, src, zp, dsm, s_pos, ntile, nslc, (par ^ 1) * g.BUF, lane, tdn, thn, twn);
      if (nslc == 0 && ntile >= 0) {
        if (lane == 0) t_next = atomicAdd(sched + 1 + blockIdx.y, 1);
        t_next = __builtin_amdgcn_readfirstlane(t_next);
        if (t_next >= ntiles) t_next = -1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tile = ntile;
      slice = nslc;
      par ^= 1;
    }
    tile_lds_barrier();                          // R: the compute waves' BN partials (uniform count)
  } else {
    // ======================= compute waves =======================
    f32x16 acc[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    bf16x8 fa[MB][2];                            // halo (B) fragments of sub-steps 0 / 1, rotating
    bf16x8 fb[PD][2];                            // weight (A) fragments of PD k-steps in flight
    constexpr unsigned FTILE = 64u * 16u;        // bytes of one fragment (32 columns x 16 k)
    const unsigned wstep = (unsigned)g.nct * FTILE;   // bytes per k-step of the packed weights
    unsigned voffb[PD];
#pragma unroll
    for (int u = 0; u < PD; ++u) voffb[u] = (unsigned)lane * 16u + (unsigned)u * wstep;
    auto load_b = [&](const unsigned char* base, int slot) {
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[slot][j] = *(const bf16x8*)(base + voffb[slot] + j * FTILE);
    };
    auto read_a = [&](int mb, int o) -> bf16x8 { return *(const bf16x8*)(dsm + lb[mb] + o); };
    // k-step offsets of this lane half: (sub-step 0, sub-step 1); per-lane LDS reads keep the
    // halo reads interleaved with the MFMAs (see conv_tile_kernel)
    auto kofs = [&](int k) -> int2 { return *reinterpret_cast<const int2*>((const int*)(s_kt + k) + 2 * hf); };
    const int emode = Q8O ? (8 | ((act & 0xff) == ACT_RELU ? 2 : 0))
                          : (BWS ? (4 | ((act & 0xff) == ACT_RELU ? 2 : 0))
                                 : ((stats ? 1 : 0) | ((act & 0xff) == ACT_RELU ? 2 : 0)));
#pragma unroll
    for (int u = 0; u < PD; ++u) load_b(reinterpret_cast<const unsigned char*>(wp) + (size_t)ct0 * FTILE, u);
    int par = 0;
    while (true) {
      tile_lds_barrier();                        // A
      const int tile = __builtin_amdgcn_readfirstlane(s_job[2 * par]);
      const int slice = __builtin_amdgcn_readfirstlane(s_job[2 * par + 1]);
      if (tile < 0) break;
      const int nslc = slice + 1 == nslice ? 0 : slice + 1;
      const unsigned char* wbase = reinterpret_cast<const unsigned char*>(wp) +
                                   ((size_t)slice * nks * g.nct + ct0) * FTILE + PD * wstep;
      const unsigned char* wnext =
          reinterpret_cast<const unsigned char*>(wp) + ((size_t)nslc * nks * g.nct + ct0) * FTILE;
      {
        const int2 ko = kofs(0);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          fa[mb][0] = read_a(mb, ko.x);
          fa[mb][1] = read_a(mb, ko.y);
        }
      }
      int2 ko_n = kofs(1);
      for (int ks = 0; ks < nks; ks += PD) {
        const unsigned char* wl = ks + PD >= nks ? wnext : wbase;   // last turn: next job's steps
#pragma unroll
        for (int u = 0; u < PD; ++u) {
          const int2 ko = ko_n;
          ko_n = kofs(ks + u + 2);
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[u][0], fa[mb][0], acc[mb], 0, 0, 0);
            fa[mb][0] = read_a(mb, ko.x);
            acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[u][1], fa[mb][1], acc[mb], 0, 0, 0);
            fa[mb][1] = read_a(mb, ko.y);
            __builtin_amdgcn_sched_barrier(0);
          }
          load_b(wl, u);                         // k-step ks+u+PD, or the next job's step u
          __builtin_amdgcn_sched_barrier(0);
        }
        wbase += PD * wstep;
      }
      if (slice == nslice - 1) {
        // ---- epilogue: acc (+bias) -> bf16 -> activation -> 2 x 16-B stores (+BN sums) ----
        int t = tile;
        const int tw_i = t % twn; t /= twn;
        const int th_i = t % thn; t /= thn;
        const int td_i = t % tdn;
        const int n = t / tdn;
        const int d0 = td_i * g.TD, h0 = th_i * g.TH, w0 = tw_i * g.TW;
        const int ld = g.OD - d0, lh = g.OH - h0, lw = g.OW - w0;
        const bool edge = ld < g.TD || lh < g.TH || lw < g.TW;
        const int gc = ct0 * 16 + 16 * hf;       // this lane's first output column
        const long long obase_e =
            ((long long)n * g.osn + g.ob + (long long)d0 * g.osd + (long long)h0 * g.osh + w0 * g.osw) * Ncol + gc;
        auto epilogue = [&](auto mode) {
          // bit 0 BN statistics, bit 1 relu, bit 2 BN-backward moments (bit 1 is then the BN's relu,
          // dx itself has no activation), bit 3 e4m3 out
          constexpr int M = decltype(mode)::value;
          constexpr bool BW = (M & 4) != 0;
          constexpr bool ST = BW || (M & 1) != 0, RELU = !BW && (M & 2) != 0, Q8 = (M & 8) != 0;
          bool okm[MB];
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            bool ok = roff[mb] >= 0 && gc < Ncol;
            if (edge) ok = ok && (rpk[mb] >> 16) < ld && ((rpk[mb] >> 8) & 255) < lh && (rpk[mb] & 255) < lw;
            okm[mb] = ok;
          }
          // two passes of 8 consecutive columns (one 16-B store per position each): 8 + 8 live
          // partial sums instead of 16 + 16 (the MB = 5 instance spilled with all 16 columns')
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            float ts[ST ? 8 : 1], tq[ST ? 8 : 1];
            if constexpr (ST) {
#pragma unroll
              for (int j = 0; j < 8; ++j) ts[j] = tq[j] = 0.f;
            }
            // BW: the BN input y of this pass's 8 columns at every block's position (all MB loads
            // in flight together) and the BN's scale / shift (the relu mask)
            uint4 yb[BW ? MB : 1];
            float bsc[BW ? 8 : 1], bsh[BW ? 8 : 1];
            if constexpr (BW) {
#pragma unroll
              for (int mb = 0; mb < MB; ++mb)
                yb[mb] = okm[mb] ? *(const uint4*)(bny + obase_e + (long long)roff[mb] * Ncol + 8 * p)
                                 : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float2 q = s_bn[16 * hf + 8 * p + j];
                bsc[j] = q.x;
                bsh[j] = q.y;
              }
            }
            float bb[8];
            {
              const float4* b4 = reinterpret_cast<const float4*>(s_bias + 16 * hf + 8 * p);
              const float4 x0 = b4[0], x1 = b4[1];
              bb[0] = x0.x; bb[1] = x0.y; bb[2] = x0.z; bb[3] = x0.w;
              bb[4] = x1.x; bb[5] = x1.y; bb[6] = x1.z; bb[7] = x1.w;
            }
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
              const bool ok = okm[mb];
              float v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                float x = bf16_lo(bf16x2_pack(acc[mb][8 * p + j] + bb[j], 0.f));   // the stored bf16 value
                if constexpr (RELU) x = fmaxf(x, 0.f);
                v[j] = x;
              }
              if constexpr (BW) {
                const unsigned yw[4] = {yb[mb].x, yb[mb].y, yb[mb].z, yb[mb].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const float y = (j & 1) ? bf16_hi(yw[j >> 1]) : bf16_lo(yw[j >> 1]);
                  float gv = ok ? v[j] : 0.f;
                  if constexpr ((M & 2) != 0) gv = (y * bsc[j] + bsh[j]) > 0.f ? gv : 0.f;
                  ts[j] += gv;
                  tq[j] += gv * y;
                }
              } else if constexpr (ST) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const float x = ok ? v[j] : 0.f;
                  ts[j] += x;
                  tq[j] += x * x;
                }
              }
              if (ok) {
                if constexpr (Q8) {
                  unsigned wd[2];
#pragma unroll
                  for (int q = 0; q < 2; ++q) {
                    float e[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                      e[j] = __builtin_amdgcn_fmed3f(v[4 * q + j] * oscale, RELU ? 0.f : -448.f, 448.f);
                    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(e[0], e[1], 0, false);
                    pk = __builtin_amdgcn_cvt_pk_fp8_f32(e[2], e[3], pk, true);
                    wd[q] = (unsigned)pk;
                  }
                  *(uint2*)(reinterpret_cast<unsigned char*>(out) + obase_e + (long long)roff[mb] * Ncol + 8 * p) =
                      make_uint2(wd[0], wd[1]);
                } else {
                  *(uint4*)(reinterpret_cast<bf16*>(out) + obase_e + (long long)roff[mb] * Ncol + 8 * p) =
                      make_uint4(bf16x2_pack(v[0], v[1]), bf16x2_pack(v[2], v[3]), bf16x2_pack(v[4], v[5]),
                                 bf16x2_pack(v[6], v[7]));
                }
              }
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[mb][8 * p + j] = 0.f;
            }
            if constexpr (ST) {
              // over the 32 lanes holding the same columns, into the wave's LDS sums (lanes 0 and
              // 32 write disjoint columns; a fixed summation order: deterministic statistics)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                ts[j] = c32_sum32(ts[j]);
                tq[j] = c32_sum32(tq[j]);
              }
              if (r32 == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  s_red[wave * 2 * RC + 16 * hf + 8 * p + j] += ts[j];
                  s_red[wave * 2 * RC + RC + 16 * hf + 8 * p + j] += tq[j];
                }
              }
            }
          }
        };
        if constexpr (BWS) {
          if (emode == 6) epilogue(std::integral_constant<int, 6>{});
          else epilogue(std::integral_constant<int, 4>{});
        } else switch (emode) {
          case 0: epilogue(std::integral_constant<int, 0>{}); break;
          case 1: epilogue(std::integral_constant<int, 1>{}); break;
          case 2: epilogue(std::integral_constant<int, 2>{}); break;
          case 3: epilogue(std::integral_constant<int, 3>{}); break;
          case 8: if constexpr (Q8O) epilogue(std::integral_constant<int, 8>{}); break;
          default: if constexpr (Q8O) epilogue(std::integral_constant<int, 10>{}); break;
        }
      }
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) lb[mb] += (1 - 2 * par) * g.BUF;   // the other buffer
      par ^= 1;
    }
    tile_lds_barrier();                          // R
    if (stats && tid < RC && ct0 * 16 + tid < Ncol) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < CT_NCW; ++w) {
        s1 += s_red[w * 2 * RC + tid];
        s2 += s_red[w * 2 * RC + RC + tid];
      }
      float* row = stats + (long long)blockIdx.x * 2 * Ncol;
      row[ct0 * 16 + tid] = s1;
      row[Ncol + ct0 * 16 + tid] = s2;
    }
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the last job's unused ring loads
  if (tid == 0) {                                // the last workgroup out resets the counters
    __threadfence();
    if (atomicAdd(sched, 1) == (int)(gridDim.x * gridDim.y) - 1) {
      for (int i = 0; i < (int)gridDim.y; ++i) atomicExch(sched + 1 + i, 0);
      atomicExch(sched, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------
// instantiations (MB, CPP) -- the Python planner only emits these (tile rows <= 128 MB)
#define C32_INSTANCES(X) X(4, 1) X(5, 1) X(4, 2) X(5, 2) X(4, 4) X(5, 4)

extern "C" int fn_conv_tile32_supported(int MB, int CPP) {
#ifndef FN_EXPERIMENTS
  return 0;   // (measured 3.5 % slower per step, profiles/r4_m32_ab.md: an experiment build only)
#endif
#define C32_SUP(M, C) if (MB == M && CPP == C) return 1;
  C32_INSTANCES(C32_SUP)
#undef C32_SUP
  return 0;
}

static size_t tile32_lds_total(const TileGeom& g) {
  return 2 * (size_t)g.BUF + 64 + ct_red_bytes(2) + (size_t)(g.nks + C32_PD + 2) * 16 + (size_t)g.HPpad * 8 + 32 * 4 +
         32 * 8;
}

template <int MB, int CPP, bool Q8O, bool BWS = false>
static int launch_tile32(dim3 grid, size_t lds, hipStream_t st, const void* s, const uint4* w, const int2* rt,
                         const int4* kt, const void* zp, const float* b, void* o, float* stats, const TileGeom& g,
                         int Ncol, int act, int* sched, float oscale, const void* bny = nullptr,
                         const float* bnp = nullptr) {
  static size_t configured = 0;
  if (lds > configured) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_tile32_kernel<MB, CPP, Q8O, BWS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    configured = lds;
  }
  hipLaunchKernelGGL((conv_tile32_kernel<MB, CPP, Q8O, BWS>), grid, dim3(CT_NTHR), lds, st, (const unsigned char*)s, w,
                     rt, kt, (const unsigned char*)zp, b, o, stats, g, Ncol, act, sched, oscale, (const bf16*)bny, bnp);
  return 0;
}

// As fn_conv_tile (same geometry vector, row table of 4 * 2MB 16-row fragments, sched / zero
// page), for the 32x32x16 kernel: wp packed by fn_tile_pack_w mode 32, ktab int4[nks + PD + 2]
// = per k-step {h0 j0, h0 j1, h1 j0, h1 j1} byte offsets; Ncol % 32 == 0; oscale > 0: e4m3 out.
// bny / bnp (dgrad only, with stats): as fn_conv_tile -- the BN input y [out shape] and (mean,
// invstd, scale, shift) [4][Ncol] of the BN+act layer whose output the conv consumed; stats then
// receives that BN's raw backward sums and act is the BN's activation (none / relu).
extern "C" int fn_conv_tile32(const void* src, const void* wp, const void* rowtab, const void* ktab, const void* zp,
                              const float* bias, void* out, float* stats, const int* geom, int Ncol, int act, int MB,
                              int* sched, hipStream_t st, float oscale, const void* bny, const float* bnp) {
  const TileGeom g = parse_tile(geom);
  if (g.CS != 8 && g.CS != 16 && g.CS != 32 && g.CS != 64) return -2;
  const int CPP = g.CS / 8;
  if (!fn_conv_tile32_supported(MB, CPP)) return -2;
  if (g.C % g.CS || g.TD * g.TH * g.TW > 128 * MB || g.TD < 1 || g.TH < 1 || g.TW < 1) return -3;
  const long long HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const long long HP = (g.TD + g.KD - 1) * HH * HW;
  if (g.HPpad < HP || g.HPpad % 64) return -3;
  if (g.TD + g.KD - 1 > 255 || HH > 255 || HW > 255) return -3;
  const int T = g.KD * g.KH * g.KW;
  const int need_ks = g.CS >= 32 ? T * (g.CS / 32) : (g.CS == 16 ? (T + 1) / 2 : (T + 3) / 4);
  if (g.nks % C32_PD || g.nks < need_ks || g.nct < (Ncol + 15) / 16 || g.nct % 2) return -3;
  for (long long p = 0; p < g.HPpad; p += 1) {   // the magic divisors must be exact for every DMA row
    const unsigned long long hd = ((unsigned long long)p * g.mHHW) >> 32;
    const unsigned long long rem = p - hd * HH * HW;
    if (hd != (unsigned long long)(p / (HH * HW)) || (((rem * g.mHW) >> 32) != rem / HW)) return -3;
  }
  if ((size_t)g.BUF < (size_t)g.HPpad * CPP * 16 || g.BUF % 1024) return -3;
  const size_t lds = tile32_lds_total(g);
  if (lds > 160 * 1024) return -4;
  const int ncb = Ncol / 32;
  if (!sched || !zp || !ktab || ncb > 63 || ncb * 2 > g.nct) return -6;
  if (Ncol % 32 || (act != ACT_NONE && act != ACT_RELU)) return -2;   // whole 32-column blocks
  if (!(oscale >= 0.f) || (oscale > 0.f && (stats || CPP != 1 || bny))) return -2;   // (e4m3 out: the s2d stem)
  if ((bny != nullptr) != (bnp != nullptr) || (bny && (!stats || bias))) return -2;
  dim3 grid((unsigned)fn_conv_tile_workers(geom, Ncol, 2), (unsigned)ncb);
  int rc = -2;
#define C32_CASE(M, C)                                                                                            \
  if (MB == M && CPP == C)                                                                                        \
    rc = bny ? launch_tile32<M, C, false, true>(grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab,        \
                                                 (const int4*)ktab, zp, bias, out, stats, g, Ncol, act, sched, 0.f, \
                                                 bny, bnp) :                                                       \
         oscale > 0.f ? launch_tile32<M, C, C == 1>(grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab,     \
                                                     (const int4*)ktab, zp, bias, out, stats, g, Ncol, act, sched,  \
                                                     oscale)                                                        \
                      : launch_tile32<M, C, false>(grid, lds, st, src, (const uint4*)wp, (const int2*)rowtab,      \
                                                   (const int4*)ktab, zp, bias, out, stats, g, Ncol, act, sched, 0.f);
#ifdef FN_EXPERIMENTS
  C32_INSTANCES(C32_CASE)
#endif
#undef C32_CASE
  if (rc) return rc;
  FN_CHECK_LAUNCH();
  return 0;
}
