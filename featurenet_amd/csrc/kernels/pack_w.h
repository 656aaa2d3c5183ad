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

// one job of the many-layer pack launch: output elements [start, start + count) of the launch's
// index space go to out[0 .. count); kind 0-2 = ig_pack_val modes (a = K0, C0, K, T, C, ld, KW, R),
// 3 / 4 = halo_pack_val forward / dgrad (a = K0, C0, K, T, C, CS, Tp)
#define FN_PACK_MAXJ 24
struct PackJob {
  const float* w;
  bf16* out;
  long long start;
  int a[9];
  int kind;
};
struct PackJobs {
  PackJob j[FN_PACK_MAXJ];
  int n;
  long long total;
};
