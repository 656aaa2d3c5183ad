// Weight packing element maps shared by the single-layer pack kernels (igemm_pack_w in
// conv_igemm.hip, halo_pack_w in conv_halo.hip) and the many-layer pack launch
// (pack_w_multi_kernel, conv_igemm.hip): output element i of a packed bf16 B operand and the fp32
// weight element it comes from.
#pragma once
#include "common.h"

// gather (igemm) layouts of an fp32 w [K0][T][C0] (K0 <= K, C0 <= C: missing rows / channels
// are zeros), row stride ld:
//   mode 0 (forward):   out[co][t*C + c]
//   mode 1 (dgrad):     out[ci][t*K + k]
//   mode 2 (packed-W):  out[co][r*R + p] = w[co][r*KW + p/C][p%C]  (p < KW*C; rows of R = KW*C
//                       rounded up to 8)
__device__ inline float ig_pack_val(const float* __restrict__ w, int K0, int C0, int K, int T, int C, int mode, int ld,
                                    int KW, int R, long long i) {
  const int row = (int)(i / ld), col = (int)(i % ld);
  if (mode == 0) {
    const int t = col / C, c = col % C;
    return (t < T && row < K0 && c < C0) ? w[((long long)row * T + t) * C0 + c] : 0.f;
  }
  if (mode == 1) {
    const int t = col / K, k = col % K;
    return (t < T && k < K0 && row < C0) ? w[((long long)k * T + t) * C0 + row] : 0.f;
  }
  const int r = col / R, p = col % R;
  if (p >= KW * C || row >= K0) return 0.f;
  const int t = r * KW + p / C, c = p % C;
  return (t < T && c < C0) ? w[((long long)row * T + t) * C0 + c] : 0.f;
}

// halo-kernel layouts of an fp32 w [K0][T][C0] (K0 <= K, C0 <= C: missing output / input
// channels are zeros -- channel-padded NAS convs), CS = channels per halo slice of the source,
// taps padded to Tp:
//   mode 0 (forward):  out[n = co][p][t][j] = w[co][t][p*CS + j]            n < K,  src C channels
//   mode 1 (dgrad):    out[n = ci][p][t][j] = w[p*CS + j][T-1-t][ci]        n < C,  src K channels
__device__ inline float halo_pack_val(const float* __restrict__ w, int K0, int C0, int K, int T, int C, int CS, int Tp,
                                      int mode, long long i) {
  const int Csrc = mode == 0 ? C : K;
  const int j = (int)(i % CS);
  long long r = i / CS;
  const int t = (int)(r % Tp);
  r /= Tp;
  const int p = (int)(r % (Csrc / CS));
  const int n = (int)(r / (Csrc / CS));
  const int cs = p * CS + j;
  if (t >= T) return 0.f;
  if (mode == 0) return (n < K0 && cs < C0) ? w[((long long)n * T + t) * C0 + cs] : 0.f;
  return (cs < K0 && n < C0) ? w[((long long)cs * T + (T - 1 - t)) * C0 + n] : 0.f;
}

// tile-kernel (conv_tile) B stream of an fp32 w [K][T][C], one uint4 (8 bf16) per index:
// out[((slice * nks + ks) * nct + ct) * 64 + lane][j] (8 bf16 per lane) =
//   Wsrc[col = ct*16 + (lane & 15)][tap][ch], k-step ks of slice:
//     CS >= 32: tap = ks / (CS/32), ch = slice*CS + (ks % (CS/32))*32 + (lane>>4)*8 + j
//     CS == 16: tap = 2*ks + (lane>>5), ch = slice*16 + ((lane>>4)&1)*8 + j
//     CS == 8:  tap = 4*ks + (lane>>4), ch = slice*8 + j
//   forward: Wsrc[col][tap][ch] = w[col][tap][ch]          (Ncol = K, Csrc = C)
//   dgrad:   Wsrc[col][tap][ch] = w[ch][T-1-tap][col]      (Ncol = C, Csrc = K)
// zero for tap >= T or col >= Ncol.
__device__ __forceinline__ void tile_pack_w_one(const float* __restrict__ w, uint4* __restrict__ out, int K, int T,
                                                int C, int CS, int nks, int nct, int nslice, int dgrad, int nt,
                                                long long i) {
  if (i >= (long long)nslice * nks * nct * 64) {
    out[i] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  const int lane = (int)(i % 64);
  long long r = i / 64;
  const int ct = (int)(r % nct);
  r /= nct;
  const int ks = (int)(r % nks);
  const int slice = (int)(r / nks);
  const int Ncol = dgrad ? C : K;
  // column order inside each nt*16-column block: fragment ct%nt, row i holds output column
  // 4nt*(i/4) + 4*(ct%nt) + i%4, so after the kernel's C^T MFMA a lane's nt fragments give 4nt
  // consecutive output columns (one 16-B store per 8)
  int tap, ch0;
  const int fi = lane & 15;
  const int col = (ct / nt) * nt * 16 + 4 * nt * (fi >> 2) + 4 * (ct % nt) + (fi & 3);
  if (CS >= 32) {
    const int sub = CS / 32;
    tap = ks / sub;
    ch0 = slice * CS + (ks % sub) * 32 + (lane >> 4) * 8;
  } else if (CS == 16) {
    tap = 2 * ks + (lane >> 5);
    ch0 = slice * 16 + ((lane >> 4) & 1) * 8;
  } else {                                       // CS = 8: four taps per k-step
    tap = 4 * ks + (lane >> 4);
    ch0 = slice * 8;
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

// one job of the many-layer pack launch: indices [start, start + count) of the launch's index
// space go to out[0 .. count); kind 0-2 = ig_pack_val modes (a = K0, C0, K, T, C, ld, KW, R),
// 3 / 4 = halo_pack_val forward / dgrad (a = K0, C0, K, T, C, CS, Tp), 5 = tile_pack_w_one (a = K, T,
// C, CS, nks, nct, nslice, dgrad, nt; uint4 elements)
#define FN_PACK_MAXJ 24
struct PackJob {
  const float* w;
  bf16* out;
  long long start;                               // (a multiple of 256: one job per workgroup)
  long long count;
  int a[9];
  int kind;
};
struct PackJobs {
  PackJob j[FN_PACK_MAXJ];
  int n;
  long long total;
};
