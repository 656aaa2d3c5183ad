// Shared pieces of the big-tile LDS-halo conv kernels (conv_tile.hip: the 16x16x32 bf16 and
// the fp8 kernels): the tile geometry, the halo DMA of one job, small helpers.
#pragma once
#include "common.h"
#include "tile_dma.h"

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
  unsigned mTW, mTH;        // magic multipliers for the epilogue's tile-row decode
  // output view: output position (n, d, h, w) is stored at position index
  // n*osn + ob + d*osd + h*osh + w*osw (x Ncol elements); natural layout = (OD*OH*OW, 0,
  // OH*OW, OW, 1).  A strided view writes one parity class of a sub-pixel (upsample x2)
  // convolution straight into the full-resolution output.
  int osn, ob, osd, osh, osw;
};

#define CT_NCW 4                       // compute (MFMA) waves
#define CT_F8_POOL 0x100               // fp8 act flag: fused 2^3 max-pool epilogue
#define CT_NTHR (64 * (CT_NCW + 1))     // + one loader wave
// per-compute-wave BN sums of the workgroup's NT*16 columns: the running sums and the chunk flush
// rows of the two job parities (conv_tile.hip's chunked statistics schedule)
// (fp8 inference instances: no statistics, one set)
__host__ __device__ constexpr int ct_red_bytes(int NT, int ncw = CT_NCW, bool f8 = false) {
  return (f8 ? 1 : 3) * ncw * 2 * NT * 16 * 4;
}

// packed bf16 pairs (low half = element 0)
__device__ __forceinline__ float bf16_lo(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(unsigned w) { return __uint_as_float(w & 0xffff0000u); }
// (one vector conversion: a pair of scalar f2bf's feeding bit operations is emitted as two
// half-empty v_cvt_pk_bf16_f32 and a v_perm_b32; the vector form is one v_cvt_pk_bf16_f32, same RNE bits)
__device__ __forceinline__ unsigned bf16x2_pack(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

// sum over the 16 lanes of a DPP row (every lane of the row gets it): quad swaps, then
// half-row and row mirrors
__device__ __forceinline__ float ct_sum16(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));    // quad [1,0,3,2]
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));    // quad [2,3,0,1]
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));   // row_half_mirror
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));   // row_mirror
  return x;
}

// OCP MX block scale of a block whose largest magnitude is amax: the E8M0 exponent e = ceil(log2(amax /
// 448)) (the smallest power of two that maps the block into e4m3's range), clamped to [-127, 126]
// (byte e + 127: never 0xFF, the E8M0 NaN; 2^-e stays a normal float); amax 0 gives -127
__device__ __forceinline__ int ct_e8m0_exp(float amax) {
  const unsigned b = __float_as_uint(amax * (1.f / 448.f));
  int e = (int)((b >> 23) & 255u) - 127 + ((b & 0x7fffffu) != 0u ? 1 : 0);
  if ((b & 0x7f800000u) == 0u) e = -127;          // zero / subnormal block
  return e < -127 ? -127 : (e > 126 ? 126 : e);
}
// 2^-e for e in [-127, 126]
__device__ __forceinline__ float ct_exp2_neg(int e) { return __uint_as_float((unsigned)(127 - e) << 23); }

typedef int ct_i32x8 __attribute__((ext_vector_type(8)));
typedef float ct_f32x2 __attribute__((ext_vector_type(2)));
typedef short ct_s16x2 __attribute__((ext_vector_type(2)));

// relu of a packed bf16 pair: a negative bf16 (sign bit set) is a negative int16, so a signed
// 16-bit max with 0 zeroes it (-0.0 -> +0.0) and keeps every non-negative value (one v_pk_max_i16)
__device__ __forceinline__ unsigned ct_relu_bf16x2(unsigned w) {
  const ct_s16x2 s = __builtin_elementwise_max(__builtin_bit_cast(ct_s16x2, w), (ct_s16x2){0, 0});
  return __builtin_bit_cast(unsigned, s);
}

// BN (+ relu) of 8 bf16 values (one 16-B chunk, packed pairs) with per-channel scale / shift pairs:
// z = act(y * scale + shift) as bn_apply_kernel computes it -- one fma, bf16 rounding, then relu on
// the bf16 bits (the same bits as relu before the rounding, NaN aside).  Packed: per pair two
// unpacks, one v_pk_fma_f32, one v_cvt_pk_bf16_f32, one v_pk_max_i16.  bits (relu): bit j = z_j > 0.
typedef unsigned short ct_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ct_bn_chunk(uint4 v, const ct_f32x2* sc, const ct_f32x2* sh, bool relu,
                                             unsigned& bits) {
  const unsigned vi[4] = {v.x, v.y, v.z, v.w};
  unsigned o[4];
  bits = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const ct_f32x2 x = {bf16_lo(vi[q]), bf16_hi(vi[q])};
    const ct_f32x2 r = __builtin_elementwise_fma(x, sc[q], sh[q]);
    unsigned w = bf16x2_pack(r.x, r.y);
    if (relu) w = ct_relu_bf16x2(w);
    o[q] = w;
    const unsigned m = __builtin_bit_cast(unsigned, __builtin_elementwise_min(__builtin_bit_cast(ct_u16x2, w),
                                                                               (ct_u16x2){1, 1}));
    bits |= ((m | (m >> 15)) & 3u) << (2 * q);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// B-ring depth (k-steps in flight): a bf16 k-step is MT*NT 16-cycle MFMAs, an fp8 one
// MT*NT 32-cycle block-scaled MFMAs, so 2 fp8 steps cover the latency 4 bf16 steps do; NT = 4
// (MT = 4) holds 2: four 4-fragment slots are 64 registers, past the budget (spills)
__host__ __device__ constexpr int ct_pd(int NT, bool F8) { return F8 ? 2 : (NT == 4 ? 2 : 4); }

// Halo of job (tile, slice) into the LDS buffer at bufoff, issued by one wave (the
// loader): interior halos (the common case for unpadded convs) use SGPR base + the
// per-position byte offsets of s_pos, no address math per DMA row; halos crossing the input
// boundary check every position and read the zero page outside.
// (r_lo, r_hi: only DMA rows [r_lo, r_hi) of the job's HPpad / 64 -- the LDS-weight-ring loader
// interleaves a job's halo with the weight stream; -1: to the last row)
template <int CPP, int ESZ>
__device__ __forceinline__ void ct_dma_job(const TileGeom& g, const unsigned char* __restrict__ src,
                                           const unsigned char* __restrict__ zp, unsigned char* dsm,
                                           const int2* s_pos, int tile, int slice, int bufoff, int lane, int tdn,
                                           int thn, int twn, int r_lo = 0, int r_hi = -1) {
  const int HH = g.TH + g.KH - 1, HW = g.TW + g.KW - 1;
  const int PLANE = g.HPpad * 16;
  tile = __builtin_amdgcn_readfirstlane(tile);   // (wave-uniform: the SGPR operands need proof)
  slice = __builtin_amdgcn_readfirstlane(slice);
  bufoff = __builtin_amdgcn_readfirstlane(bufoff);
  int t = tile;
  const int tw = t % twn; t /= twn;
  const int th = t % thn; t /= thn;
  const int td = t % tdn;
  const int n = t / tdn;
  const int dlo = td * g.TD - g.pd, hlo = th * g.TH - g.ph, wlo = tw * g.TW - g.pw;
  const bool interior = dlo >= 0 && hlo >= 0 && wlo >= 0 && dlo + g.TD + g.KD - 1 <= g.ID &&
                        hlo + HH <= g.IH && wlo + HW <= g.IW;
  const unsigned char* base = src + ((long long)n * g.ID * g.IH * g.IW * g.C + slice * g.CS) * ESZ;
  const unsigned dst0 = ct_lds_addr(dsm) + bufoff;
  // position rows in batches of 8: the s_pos reads of a batch are in flight together
  // (one LDS latency per batch, not per DMA row)
  const int NR = r_hi < 0 ? (g.HPpad >> 6) : r_hi;
  if (interior) {
    const unsigned char* obase = base + (((long long)dlo * g.IH + hlo) * g.IW + wlo) * g.C * ESZ;
    for (int r0 = r_lo; r0 < NR; r0 += 8) {
      int po[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) po[i] = s_pos[((r0 + i < NR ? r0 + i : NR - 1) << 6) + lane].x;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (r0 + i < NR) {
#pragma unroll
          for (int c = 0; c < CPP; ++c)
            ct_glds16_s(obase, (unsigned)(po[i] + c * 16), dst0 + (unsigned)(c * PLANE + ((r0 + i) << 10)));
        }
      }
    }
  } else {
    for (int r0 = r_lo; r0 < NR; r0 += 8) {
      int e[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = s_pos[((r0 + i < NR ? r0 + i : NR - 1) << 6) + lane].y;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (r0 + i < NR) {
          const int gd = dlo + (e[i] >> 16), gh = hlo + ((e[i] >> 8) & 255), gw = wlo + (e[i] & 255);
          const bool ok = (unsigned)gd < (unsigned)g.ID && (unsigned)gh < (unsigned)g.IH &&
                          (unsigned)gw < (unsigned)g.IW;
          const unsigned char* gsrc = ok ? base + (long long)((gd * g.IH + gh) * g.IW + gw) * g.C * ESZ : zp;
#pragma unroll
          for (int c = 0; c < CPP; ++c)
            ct_glds16(ok ? gsrc + c * 16 : zp, dst0 + (unsigned)(c * PLANE + ((r0 + i) << 10)));
        }
      }
    }
  }
}

// bytes of one LDS mask buffer of the relu-mask dgrad epilogue: slots (4 waves x MT x 16 fragment
// rows) x Ncol / 8, rounded up to whole 64-dword DMA rows
__host__ __device__ constexpr int ct_mask_bytes(int rows, int Ncol, bool on) {
  return on ? (rows * (Ncol >> 3) + 255) / 256 * 256 : 0;
}
// LDS bytes of the relu-mask dgrad: the two mask buffers and the slot table (int2 per slot)
__host__ __device__ constexpr int ct_mask_lds(int rows, int Ncol, bool on) {
  return on ? 2 * ct_mask_bytes(rows, Ncol, on) + rows * 8 : 0;
}

#define CT_GEOM_LEN 31
static inline TileGeom parse_tile(const int* v) {
  TileGeom g;
  g.N = v[0]; g.ID = v[1]; g.IH = v[2]; g.IW = v[3]; g.C = v[4];
  g.OD = v[5]; g.OH = v[6]; g.OW = v[7];
  g.KD = v[8]; g.KH = v[9]; g.KW = v[10];
  g.pd = v[11]; g.ph = v[12]; g.pw = v[13];
  g.TD = v[14]; g.TH = v[15]; g.TW = v[16];
  g.CS = v[17]; g.HPpad = v[18]; g.nks = v[19]; g.nct = v[20];
  g.mHW = (unsigned)v[21]; g.mHHW = (unsigned)v[22]; g.BUF = v[23];
  g.mTW = (unsigned)v[24]; g.mTH = (unsigned)v[25];
  g.osn = v[26]; g.ob = v[27]; g.osd = v[28]; g.osh = v[29]; g.osw = v[30];
  return g;
}

extern "C" int fn_conv_tile_workers(const int* geom, int Ncol, int NT);
