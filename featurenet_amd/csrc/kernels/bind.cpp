// pybind11 surface of the featurenet_amd HIP kernel library (module `_C`).
//
// Every entry point takes raw device addresses (Python ints from
// tensor.data_ptr()) and the HIP stream handle of the caller's current torch
// stream, so the Python op layer owns allocation and the kernels can be
// captured into hipGraphs.  Errors raise RuntimeError with the HIP message.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

extern "C" {
int fn_igemm_fwd(const void*, const void*, const float*, void*, float*, const int*, const int*, long long, int, int,
                 int, int, int, hipStream_t, float*, int);
int fn_igemm_fwd_splits(long long, int, int);
int fn_igemm_fwd_mblocks(long long);
int fn_conv_halo(const void*, const void*, const float*, void*, float*, const int*, const int*, int, int, int*,
                 hipStream_t);
long long fn_conv_halo_lds(const int*, int);
int fn_conv_halo_workers(const int*, int);
int fn_pw_fwd(const void*, const void*, const float*, void*, long long, int, int, int, hipStream_t, const float*,
              const float*, int, const void*, const float*, const float*, float*, int);
int fn_seghead_part_len();
int fn_part_reduce(const float*, float*, long long, int, int, hipStream_t);
int fn_seghead_blocks(long long);
int fn_seghead_loss(const void*, const float*, const float*, const void*, const float*, const void*, void*, float*,
                    long long, int, int, int, float, float, hipStream_t, int, int);
int fn_pw_xent_blocks(long long);
int fn_pw_fwd_xent(const void*, const void*, const float*, void*, long long, int, int, const float*, const float*, int,
                   const long long*, float*, float, float, hipStream_t);
int fn_pw_fwd_blocks(long long, int, int);
int fn_pw_wgrad(const void*, const void*, float*, long long, int, int, hipStream_t, const float*, const float*, int,
                float*);
int fn_pw_wgrad_blocks(long long, int, int);
int fn_conv_halo_wgrad_yblocks(const int*, int);
int fn_conv_halo_f8(const void*, const void*, const float*, const float*, void*, float, const int*, const int*, int,
                    int, int, hipStream_t);
int fn_quant_fp8(const void*, void*, long long, float, hipStream_t);
int fn_quant_fp8_block(const void*, void*, void*, long long, int, hipStream_t);
int fn_mfma_scale_probe(const void*, const void*, const int*, const int*, float*, hipStream_t);
int fn_s2d_tap_f8(const void*, void*, int, int, int, int, int, int, int, int, float, int, hipStream_t);
int fn_dw_fwd(const void*, const float*, const float*, void*, const int*, int, hipStream_t);
int fn_dw_dgrad(const void*, const float*, void*, const int*, hipStream_t);
int fn_dw_wgrad(const void*, const void*, float*, const int*, int, hipStream_t, float*);
int fn_conv_halo_wgrad(const void*, const void*, float*, float*, const int*, int, int, hipStream_t);
int fn_conv_halo_wgrad_gx(const int*, int);
int fn_s2d_pack(const void*, void*, const int*, int, hipStream_t, int);
int fn_dense_splits(int, int, int);
int fn_ew_binary(const void*, const void*, void*, long long, int, hipStream_t);
int fn_ew_mul_bwd(const void*, const void*, const void*, void*, void*, long long, hipStream_t);
int fn_concat2(void*, void*, void*, long long, int, int, int, hipStream_t);
int fn_pad3(void*, void*, const int*, int, hipStream_t);
int fn_pad_channels(void*, void*, long long, int, int, int, hipStream_t);
int fn_dense_fwd(const void*, const void*, const float*, void*, float*, int, int, int, int, int, int, int, hipStream_t);
int fn_dense_dgrad(const void*, const float*, void*, int, int, int, hipStream_t, const void*, int);
int fn_dense_wgrad(const void*, const void*, float*, float*, int, int, int, float*, int, hipStream_t, const void*, int);
int fn_dense_wgrad_slices(int, int, int);
int fn_s2d_weight_map(const float*, float*, const int*, int, hipStream_t);
int fn_subpixel_wmap(const float*, float*, int, int, int, hipStream_t);
int fn_halo_pack_w(const float*, void*, int, int, int, int, int, int, int, hipStream_t);
int fn_igemm_pack_w(const float*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
int fn_pack_w_multi(const long long*, int, hipStream_t);
int fn_igemm_wgrad(const void*, const void*, float*, const int*, const int*, long long, int, int, int, int,
                   hipStream_t, int, int, const void*, int, float*, int, float*);
long long fn_igemm_wgrad_part(int, int, int, int, int, int, int);
int fn_colstats(const void*, const void*, const float*, const float*, const float*, const float*, float*, long long,
                int, int, int, int, hipStream_t);
int fn_bn_finalize(const float*, int, int, double, const float*, const float*, float*, float*, float, float, float*,
                   float*, float*, float*, int, hipStream_t);
int fn_bn_apply(const void*, const float*, const float*, void*, long long, int, int, hipStream_t, void*);
int fn_bn_wdot(const float*, const float*, float*, int, int, int, hipStream_t);
int fn_bn_bwd_prep(const float*, int, const float*, int, int, double, const float*, const float*, const float*,
                   const float*, const float*, const float*, float*, float*, const void*, const void*, long long,
                   hipStream_t);
int fn_bn_bwd_apply_k_blocks(long long, int);
int fn_bn_bwd_apply_k(const void*, const void*, const float*, const float*, const float*, const float*, void*,
                      long long, int, float*, int, hipStream_t);
int fn_bn_bwd_apply(const void*, const void*, const float*, const float*, const float*, const float*, const float*,
                    const float*, void*, long long, int, float, int, hipStream_t);
int fn_bn_bwd_apply_s2d(const void*, const void*, const float*, const float*, const float*, const float*,
                        const float*, const float*, void*, int, int, int, int, int, float, int, hipStream_t);
int fn_pool_fwd(const void*, void*, const float*, const float*, const int*, int, int, int, hipStream_t);
int fn_pool_bwd(const void*, const void*, void*, const float*, const float*, const int*, int, int, int, hipStream_t);
int fn_pool_bwd_stats_blocks(const int*);
int fn_colstats_blocks(long long, int, int, int);
int fn_pool_bn_bwd_apply(const void*, const void*, const float*, const float*, const float*, const float*,
                         const float*, const float*, void*, const int*, int, float, hipStream_t);
int fn_pool_bwd_stats(const void*, const void*, void*, const float*, const float*, const int*, int, float*,
                      hipStream_t);
int fn_softmax_xent_blocks(long long, int);
int fn_upsample2x(const void*, void*, int, int, int, int, int, int, hipStream_t);
int fn_softmax_xent_rows(const void*, int, const long long*, float*, void*, int*, long long, int, float, float,
                         hipStream_t);
int fn_adam_flat_dev(float*, const float*, float*, float*, void*, long long, const float*, int*, int, hipStream_t);
int fn_adam_flat(float*, const float*, float*, float*, void*, long long, float, float, float, float, float, float,
                 float, float, int, hipStream_t);
int fn_sgd_flat(float*, const float*, float*, void*, long long, float, float, float, int, float, hipStream_t);
int fn_bias_act(const void*, const float*, void*, long long, int, int, hipStream_t);
int fn_act_bwd(const void*, const void*, void*, long long, int, hipStream_t);
int fn_dropout(const void*, void*, long long, float, unsigned, unsigned, hipStream_t);
int fn_cast_f32_bf16(const float*, void*, long long, hipStream_t);
int fn_scale_unless_one(void*, int, const float*, long long, hipStream_t);
int fn_copy2(void*, const void*, long long, void*, const void*, long long, hipStream_t);
int fn_cu_occupy(int, int, int, void*, hipStream_t);
int fn_softmax_rows(const float*, float*, long long, int, int, const float*, hipStream_t);
int fn_unpack_bits(const void*, void*, long long, hipStream_t);
int fn_conv_tile(const void*, const void*, const void*, const void*, const void*, const float*, void*, float*,
                 const int*, int, int, int, int, int*, hipStream_t, const void*, const float*, float, void*,
                 const float*, void*, void*, int);
int fn_conv_tile_workers(const int*, int, int);
int fn_conv_tile_slab_rows(const int*, int, int);
void fn_conv_tile_grid_cap(int);
void fn_conv_tile_set_wlds(int);
void fn_conv_tile_set_schedule(int);
int fn_conv_tile_schedule();
int fn_conv_tile_wring(const int*, int, int, int, int);
int fn_conv_tile_f8(const void*, const void*, const void*, const void*, const void*, const float*, const float*, void*,
                    float, const int*, int, int, int, int, int*, hipStream_t, const void*, void*);
int fn_conv_tile_f8_supported(int, int, int);
int fn_conv_wtile(const void*, const void*, float*, float*, const void*, const void*, const void*, const int*, int, int,
                  int*, hipStream_t, const float*, float*, const float*, int);
int fn_conv_wtile_supported(int, int);
int fn_conv_wtile_prologue_built();
int fn_tile_pack_w(const float*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
int fn_tile_pack_w2(const float*, void*, void*, int, int, int, const int*, const int*, hipStream_t);
}

template <typename T>
static T P(uintptr_t a) {
  return reinterpret_cast<T>(a);
}
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void chk(int rc, const char* what) {
  if (rc == 0) return;
  if (rc < 0) throw std::runtime_error(std::string(what) + ": unsupported configuration (code " + std::to_string(rc) + ")");
  throw std::runtime_error(std::string(what) + ": " + hipGetErrorString((hipError_t)rc));
}

static void need(const std::vector<int>& v, size_t n, const char* what) {
  if (v.size() != n) throw std::runtime_error(std::string(what) + ": bad geometry length");
}

// Extent checks: the geometry implies how many elements every kernel operand
// spans; the caller passes the numel of the tensors it hands over (``ext``),
// and a geometry/tensor mismatch raises here instead of reading or writing
// out of bounds on the GPU.  ``ext`` may be empty (no check) for internal
// callers that size their own scratch.
static void fits(const std::vector<long long>& ext, size_t i, long long need_elems, const char* what,
                 const char* operand) {
  if (ext.empty()) return;
  if (i >= ext.size()) throw std::runtime_error(std::string(what) + ": missing extent for " + operand);
  if (need_elems < 0 || ext[i] < need_elems)
    throw std::runtime_error(std::string(what) + ": " + operand + " has " + std::to_string(ext[i]) +
                             " elements, geometry needs " + std::to_string(need_elems));
}
static long long prod(std::initializer_list<long long> v) {
  long long r = 1;
  for (long long x : v) {
    if (x < 0) return -1;
    r *= x;
  }
  return r;
}
// halo geometry: N ID IH IW C | OD OH OW | KD KH KW | pd ph pw | TD TH TW
static void check_halo(const std::vector<int>& g, const std::vector<long long>& ext, int ncol, bool wgrad,
                       const char* what) {
  const long long src = prod({g[0], g[1], g[2], g[3], g[4]});
  const long long out = prod({g[0], g[5], g[6], g[7], ncol});
  const int T = g[8] * g[9] * g[10];
  if (g[4] <= 0 || ncol <= 0 || T <= 0) throw std::runtime_error(std::string(what) + ": empty geometry");
  if (g[5] > g[1] + 2 * g[11] || g[6] > g[2] + 2 * g[12] || g[7] > g[3] + 2 * g[13])
    throw std::runtime_error(std::string(what) + ": output larger than the padded input");
  if (wgrad) {                       // ext = {dy, src, dw}
    fits(ext, 0, out, what, "dy");
    fits(ext, 1, src, what, "src");
    fits(ext, 2, prod({ncol, T, g[4]}), what, "dw");
  } else {                           // ext = {src, wt, out, toffs}
    const int cs = g[4] % 16 == 0 ? 16 : 8, tps = 128 / cs;
    const long long Tp = (T + tps - 1) / tps * tps;
    fits(ext, 0, src, what, "src");
    fits(ext, 1, prod({ncol, g[4], Tp}), what, "wt");
    fits(ext, 2, out, what, "out");
    fits(ext, 3, Tp, what, "toffs");
  }
}

// tile geometry: halo geometry (17) | CS HPpad nks nct mHW mHHW BUF mTW mTH; ext = {src, wpk, out, rowtab rows}
// elements an output view (geometry entries 26-30: osn, ob, osd, osh, osw) spans
static long long view_extent(const std::vector<int>& g, int ncol) {
  if (g[26] < 0 || g[27] < 0 || g[28] < 0 || g[29] < 0 || g[30] < 0) throw std::runtime_error("conv_tile: bad output view");
  return ((long long)(g[0] - 1) * g[26] + g[27] + (long long)(g[5] - 1) * g[28] + (long long)(g[6] - 1) * g[29] +
          (long long)(g[7] - 1) * g[30] + 1) * ncol;
}

static void check_tile(const std::vector<int>& g, const std::vector<long long>& ext, int ncol, int MT,
                       const char* what, int NT = 2) {
  if (g[4] <= 0 || ncol <= 0 || g[17] <= 0 || g[4] % g[17]) throw std::runtime_error(std::string(what) + ": bad slice");
  if (g[5] > g[1] + 2 * g[11] + g[8] || g[6] > g[2] + 2 * g[12] + g[9] || g[7] > g[3] + 2 * g[13] + g[10])
    throw std::runtime_error(std::string(what) + ": output larger than the padded input");
  fits(ext, 0, prod({g[0], g[1], g[2], g[3], g[4]}), what, "src");
  // the stream's rows (+ 4 zero ring k-steps) x nct fragments, of which the last row is read up to the
  // ncol columns' fragments (a view may start inside a wider stream: the sub-pixel class weights)
  const long long ncb = (ncol + NT * 16 - 1) / (NT * 16);
  fits(ext, 1, ((long long)(g[4] / g[17] * g[19] + 3) * g[20] + ncb * NT) * 64 * 8, what, "wpk");
  fits(ext, 2, view_extent(g, ncol), what, "out");
  fits(ext, 3, 4LL * MT * 16, what, "rowtab");
  fits(ext, 4, g[19] + 6LL, what, "ktab");
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "featurenet_amd gfx950 HIP kernels";
  m.attr("ARCH") = "gfx950";

  // part / splits (optional): the split-K form (fn_igemm_fwd_splits), part = splits x M x N floats
  m.def("igemm_fwd", [](uintptr_t src, uintptr_t wt, uintptr_t bias, uintptr_t out, uintptr_t stats, uintptr_t tab,
                        std::vector<int> geom, long long M, int N, int K, int ldw, int vec, int act, uintptr_t st,
                        uintptr_t part, int splits, long long part_elems) {
    need(geom, 14, "igemm_fwd");
    if (splits > 1 && part_elems < (long long)splits * M * N)
      throw std::runtime_error("igemm_fwd: part has " + std::to_string(part_elems) + " elements, split-K needs " +
                               std::to_string((long long)splits * M * N));
    chk(fn_igemm_fwd(P<const void*>(src), P<const void*>(wt), P<const float*>(bias), P<void*>(out), P<float*>(stats),
                     P<const int*>(tab), geom.data(), M, N, K, ldw, vec, act, S(st), P<float*>(part), splits),
        "igemm_fwd");
  }, py::arg("src"), py::arg("wt"), py::arg("bias"), py::arg("out"), py::arg("stats"), py::arg("tab"), py::arg("geom"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("ldw"), py::arg("vec"), py::arg("act"), py::arg("st"),
     py::arg("part") = 0, py::arg("splits") = 1, py::arg("part_elems") = 0);
  m.def("igemm_fwd_splits", &fn_igemm_fwd_splits);
  m.def("igemm_fwd_mblocks", &fn_igemm_fwd_mblocks);
  m.def("conv_halo", [](uintptr_t src, uintptr_t wt, uintptr_t bias, uintptr_t out, uintptr_t stats,
                        uintptr_t toffs, std::vector<int> geom, int ncol, int act, uintptr_t sched, uintptr_t st,
                        std::vector<long long> ext) {
    need(geom, 17, "conv_halo");
    check_halo(geom, ext, ncol, false, "conv_halo");
    chk(fn_conv_halo(P<const void*>(src), P<const void*>(wt), P<const float*>(bias), P<void*>(out), P<float*>(stats),
                     P<const int*>(toffs), geom.data(), ncol, act, P<int*>(sched), S(st)),
        "conv_halo");
  }, py::arg("src"), py::arg("wt"), py::arg("bias"), py::arg("out"), py::arg("stats"), py::arg("toffs"),
     py::arg("geom"), py::arg("ncol"), py::arg("act"), py::arg("sched"), py::arg("st"),
     py::arg("ext") = std::vector<long long>());
  // part: fp32 scratch of conv_halo_wgrad_gx(geom, grid_x) x cout x taps x C (the per-workgroup
  // partial weight gradients, added into dw in a fixed order); ext = {dy, src, dw, part}
  m.def("conv_halo_wgrad", [](uintptr_t dy, uintptr_t src, uintptr_t dw, uintptr_t part, std::vector<int> geom,
                              int cout, int grid_x, uintptr_t st, std::vector<long long> ext) {
    need(geom, 17, "conv_halo_wgrad");
    check_halo(geom, ext, cout, true, "conv_halo_wgrad");
    const int gx = fn_conv_halo_wgrad_gx(geom.data(), grid_x);
    fits(ext, 3, prod({gx, cout, geom[8] * geom[9] * geom[10], geom[4]}), "conv_halo_wgrad", "part");
    chk(fn_conv_halo_wgrad(P<const void*>(dy), P<const void*>(src), P<float*>(dw), P<float*>(part), geom.data(), cout,
                           grid_x, S(st)),
        "conv_halo_wgrad");
  }, py::arg("dy"), py::arg("src"), py::arg("dw"), py::arg("part"), py::arg("geom"), py::arg("cout"),
     py::arg("grid_x"), py::arg("st"), py::arg("ext") = std::vector<long long>());
  m.def("conv_halo_wgrad_gx", [](std::vector<int> geom, int grid_x) {
    need(geom, 17, "conv_halo_wgrad_gx");
    return fn_conv_halo_wgrad_gx(geom.data(), grid_x);
  });
  m.def("conv_tile", [](uintptr_t src, uintptr_t wpk, uintptr_t rowtab, uintptr_t ktab, uintptr_t zp, uintptr_t bias,
                        uintptr_t out, uintptr_t stats, std::vector<int> geom, int ncol, int act, int MT, int NT,
                        uintptr_t sched, uintptr_t st, std::vector<long long> ext, uintptr_t bny, uintptr_t bnp,
                        float oscale, uintptr_t osc, long long osc_n, uintptr_t pst, uintptr_t pz, uintptr_t pmask,
                        int pact, std::vector<long long> pext) {
    need(geom, 31, "conv_tile");
    check_tile(geom, ext, ncol, MT, "conv_tile", NT);
    // osc: block scales of an e4m3 output, one dword per output position
    if (osc && osc_n < view_extent(geom, 1)) throw std::runtime_error("conv_tile: osc smaller than the output");
    if (bny && bnp) {   // ext[5] = numel of the BN input (the output's shape), ext[6] = numel of bnp
      fits(ext, 5, view_extent(geom, ncol), "conv_tile", "bny");
      fits(ext, 6, 4LL * ncol, "conv_tile", "bnp");
    } else if (bny) {   // the relu-mask bytes: ext[5] = their count (one per 8 output columns)
      fits(ext, 5, view_extent(geom, ncol) / 8, "conv_tile", "mask");
    }
    // the BN prologue: pext = {pst, pz, pmask} element counts -- [scale C][shift C] of the source's
    // channels, z of the source's shape, one mask byte per 8 source elements
    if (pst) {
      if (pext.size() < 3) throw std::runtime_error("conv_tile: the BN prologue needs pext = {pst, pz, pmask}");
      const long long nsrc = prod({geom[0], geom[1], geom[2], geom[3], geom[4]});
      fits(pext, 0, 2LL * geom[4], "conv_tile", "pst");
      if (pz) fits(pext, 1, nsrc, "conv_tile", "pz");
      if (pmask) fits(pext, 2, nsrc / 8, "conv_tile", "pmask");
    }
    chk(fn_conv_tile(P<const void*>(src), P<const void*>(wpk), P<const void*>(rowtab), P<const void*>(ktab),
                     P<const void*>(zp), P<const float*>(bias), P<void*>(out), P<float*>(stats), geom.data(), ncol,
                     act, MT, NT, P<int*>(sched), S(st), P<const void*>(bny), P<const float*>(bnp), oscale,
                     P<void*>(osc), P<const float*>(pst), P<void*>(pz), P<void*>(pmask), pact),
        "conv_tile");
  }, py::arg("src"), py::arg("wpk"), py::arg("rowtab"), py::arg("ktab"), py::arg("zp"), py::arg("bias"), py::arg("out"),
     py::arg("stats"), py::arg("geom"), py::arg("ncol"), py::arg("act"), py::arg("MT"), py::arg("NT"),
     py::arg("sched"), py::arg("st"), py::arg("ext") = std::vector<long long>(), py::arg("bny") = 0,
     py::arg("bnp") = 0, py::arg("oscale") = 0.f, py::arg("osc") = 0, py::arg("osc_n") = 0, py::arg("pst") = 0,
     py::arg("pz") = 0, py::arg("pmask") = 0, py::arg("pact") = 0, py::arg("pext") = std::vector<long long>());
  m.def("conv_tile_f8", [](uintptr_t src, uintptr_t wpk, uintptr_t rowtab, uintptr_t ktab, uintptr_t zp,
                           uintptr_t scale, uintptr_t bias, uintptr_t out, float oscale, std::vector<int> geom, int ncol,
                           int relu, int MT, int NT, uintptr_t st, uintptr_t sched, std::vector<long long> ext,
                           uintptr_t xsc, uintptr_t osc) {
    need(geom, 31, "conv_tile_f8");
    // xsc / osc: block scales (a dword per input / output position): ext[5] / ext[6] their counts
    if (xsc) fits(ext, 5, prod({geom[0], geom[1], geom[2], geom[3]}), "conv_tile_f8", "xsc");
    if (osc) fits(ext, 6, view_extent(geom, 1), "conv_tile_f8", "osc");
    if (geom[4] <= 0 || ncol <= 0 || geom[17] <= 0 || geom[4] % geom[17])
      throw std::runtime_error("conv_tile_f8: bad slice");
    fits(ext, 0, prod({geom[0], geom[1], geom[2], geom[3], geom[4]}), "conv_tile_f8", "src");
    fits(ext, 1, prod({geom[4] / geom[17] * geom[19] + 4, geom[20], 64, 32}), "conv_tile_f8", "wpk");
    fits(ext, 2, (relu & 2) ? prod({geom[0], geom[5] / 2, geom[6] / 2, geom[7] / 2, ncol}) : view_extent(geom, ncol),
         "conv_tile_f8", "out");
    fits(ext, 3, 4LL * MT * 16, "conv_tile_f8", "rowtab");
    fits(ext, 4, geom[19] + 6LL, "conv_tile_f8", "ktab");
    chk(fn_conv_tile_f8(P<const void*>(src), P<const void*>(wpk), P<const void*>(rowtab), P<const void*>(ktab),
                        P<const void*>(zp), P<const float*>(scale), P<const float*>(bias), P<void*>(out), oscale,
                        geom.data(), ncol, relu, MT, NT, P<int*>(sched), S(st), P<const void*>(xsc), P<void*>(osc)),
        "conv_tile_f8");
  }, py::arg("src"), py::arg("wpk"), py::arg("rowtab"), py::arg("ktab"), py::arg("zp"), py::arg("scale"),
     py::arg("bias"), py::arg("out"), py::arg("oscale"), py::arg("geom"), py::arg("ncol"), py::arg("relu"),
     py::arg("MT"), py::arg("NT"), py::arg("st"), py::arg("sched"), py::arg("ext") = std::vector<long long>(),
     py::arg("xsc") = 0, py::arg("osc") = 0);
  m.def("conv_tile_f8_supported", &fn_conv_tile_f8_supported);
  m.def("conv_wtile", [](uintptr_t x, uintptr_t dy, uintptr_t dw, uintptr_t part, uintptr_t rowtab, uintptr_t postab,
                         uintptr_t zp, std::vector<int> geom, int nacc, int workers, uintptr_t sched, uintptr_t st,
                         std::vector<long long> ext, uintptr_t wsrc, uintptr_t wdp, uintptr_t pst, int pact) {
    need(geom, 24, "conv_wtile");
    // the BN prologue: pst = [scale C][shift C] of x's channels (ext[8] = its element count)
    if (pst) fits(ext, 8, 2LL * geom[4], "conv_wtile", "pst");
    const long long T = (long long)geom[9] * geom[10] * geom[11];
    fits(ext, 0, prod({geom[0], geom[1], geom[2], geom[3], geom[4]}), "conv_wtile", "x");
    const bool sp = (nacc >> 14) & 1;             // sub-pixel form: dy = [N, OD+1, OH+1, OW+1, 8 K]
    if (sp)
      fits(ext, 1, prod({geom[0], geom[5] + 1, geom[6] + 1, geom[7] + 1, 8 * geom[8]}), "conv_wtile", "dy");
    else
      fits(ext, 1, prod({geom[0], geom[5], geom[6], geom[7], geom[8]}), "conv_wtile", "dy");
    const long long tw = sp ? 64 : T;             // (sub-pixel form: 8 classes x 8 folded taps)
    fits(ext, 2, prod({geom[8], tw, geom[4]}), "conv_wtile", "dw");
    fits(ext, 3, 32LL * geom[19], "conv_wtile", "rowtab");
    fits(ext, 4, geom[18], "conv_wtile", "postab");
    fits(ext, 5, 8LL * workers * ((nacc >> 13) & 1 ? 2 : 1) * geom[8] * tw * geom[4], "conv_wtile", "part");
    if (wsrc) {                                   // S = sum W . dW partials: [ceil(dW / 256)][C], W like dW
      fits(ext, 6, prod({geom[8], tw, geom[4]}), "conv_wtile", "wsrc");
      fits(ext, 7, (prod({geom[8], tw, geom[4]}) + 255) / 256 * geom[4], "conv_wtile", "wdp");
    }
    if (geom[5] > geom[1] + 2 * geom[12] || geom[6] > geom[2] + 2 * geom[13] || geom[7] > geom[3] + 2 * geom[14])
      throw std::runtime_error("conv_wtile: output larger than the padded input");
    chk(fn_conv_wtile(P<const void*>(x), P<const void*>(dy), P<float*>(dw), P<float*>(part), P<const void*>(rowtab),
                      P<const void*>(postab), P<const void*>(zp), geom.data(), nacc, workers, P<int*>(sched), S(st),
                      P<const float*>(wsrc), P<float*>(wdp), P<const float*>(pst), pact),
        "conv_wtile");
  }, py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("part"), py::arg("rowtab"), py::arg("postab"), py::arg("zp"),
     py::arg("geom"), py::arg("nacc"), py::arg("workers"), py::arg("sched"), py::arg("st"),
     py::arg("ext") = std::vector<long long>(), py::arg("wsrc") = 0, py::arg("wdp") = 0, py::arg("pst") = 0,
     py::arg("pact") = 0);
  m.def("conv_wtile_supported", &fn_conv_wtile_supported);
  m.def("conv_wtile_prologue_built", &fn_conv_wtile_prologue_built);
  m.def("conv_tile_workers", [](std::vector<int> geom, int ncol, int NT) {
    need(geom, 31, "conv_tile_workers");
    return fn_conv_tile_workers(geom.data(), ncol, NT);
  });
  m.def("conv_tile_grid_cap", [](int cap) { fn_conv_tile_grid_cap(cap); });   // (tests: grid independence)
  // the LDS weight ring: -1 = FN_TILE_WLDS (default on), 0 off, 1 on (tests / A/B in one process)
  m.def("conv_tile_set_wlds", [](int mode) { fn_conv_tile_set_wlds(mode); });
  // the BN-statistics tile schedule: -1 = FN_TILE_SCHED (default static), 0 static, 1 chunked
  m.def("conv_tile_set_schedule", [](int mode) { fn_conv_tile_set_schedule(mode); });
  m.def("conv_tile_schedule", [] { return fn_conv_tile_schedule(); });
  m.def("conv_tile_wring", [](std::vector<int> geom, int ncol, int MT, int NT, int mask) {
    need(geom, 31, "conv_tile_wring");
    return fn_conv_tile_wring(geom.data(), ncol, MT, NT, mask);
  });
  m.def("conv_tile_slab_rows", [](std::vector<int> geom, int ncol, int NT) {
    // rows of the BN-statistics slab a conv_tile launch with statistics writes (one per tile chunk)
    need(geom, 31, "conv_tile_slab_rows");
    return fn_conv_tile_slab_rows(geom.data(), ncol, NT);
  });
  m.def("tile_pack_w", [](uintptr_t w, uintptr_t out, int K, int T, int C, int CS, int nks, int nct, int nslice,
                          int dgrad, uintptr_t st, int nt) {
    chk(fn_tile_pack_w(P<const float*>(w), P<void*>(out), K, T, C, CS, nks, nct, nslice, dgrad, nt, S(st)),
        "tile_pack_w");
  });
  m.def("tile_pack_w2", [](uintptr_t w, uintptr_t out0, uintptr_t out1, int K, int T, int C, std::vector<int> p0,
                           std::vector<int> p1, uintptr_t st, std::vector<long long> ext) {
    // p = {CS, nks, nct, nslice, dgrad, nt}; ext = {numel(w), numel(out0) and numel(out1) in uint4 x 2 bf16x4}
    need(p0, 6, "tile_pack_w2");
    need(p1, 6, "tile_pack_w2");
    fits(ext, 0, (long long)K * T * C, "tile_pack_w2", "w");
    fits(ext, 1, ((long long)p0[3] * p0[1] + 4) * p0[2] * 64 * 8, "tile_pack_w2", "out0");
    fits(ext, 2, ((long long)p1[3] * p1[1] + 4) * p1[2] * 64 * 8, "tile_pack_w2", "out1");
    chk(fn_tile_pack_w2(P<const float*>(w), P<void*>(out0), P<void*>(out1), K, T, C, p0.data(), p1.data(), S(st)),
        "tile_pack_w2");
  });
  m.def("igemm_pack_w", [](uintptr_t w, uintptr_t out, int K0, int C0, int K, int T, int C, int mode, int ld, int KW,
                           int R, uintptr_t st, std::vector<long long> ext) {
    // ext = {numel(w), numel(out)}
    fits(ext, 0, (long long)K0 * T * C0, "igemm_pack_w", "w");
    fits(ext, 1, (long long)(mode == 1 ? C : K) * ld, "igemm_pack_w", "out");
    chk(fn_igemm_pack_w(P<const float*>(w), P<void*>(out), K0, C0, K, T, C, mode, ld, KW, R, S(st)), "igemm_pack_w");
  });
  m.def("pack_w_multi", [](std::vector<long long> jobs, uintptr_t st, std::vector<long long> ext) {
    // jobs: n rows of (w, out, kind, a0..a8) (pack_w.h PackJob); ext: n rows of (numel(w), numel(out))
    if (jobs.size() % 12 || ext.size() != jobs.size() / 6)
      throw std::invalid_argument("pack_w_multi: 12 values per job and 2 extents per job");
    const int n = (int)(jobs.size() / 12);
    for (int k = 0; k < n; ++k) {
      const long long* r = jobs.data() + 12 * k;
      const long long kind = r[2];
      long long wn, on;
      if (kind >= 0 && kind <= 2) {                // K0, C0, K, T, C, ld
        wn = r[3] * r[6] * r[4];
        on = (kind == 1 ? r[7] : r[5]) * r[8];
      } else if (kind <= 4) {                      // K0, C0, K, T, C, CS, Tp
        wn = r[3] * r[6] * r[4];
        on = r[5] * r[7] * r[9];
      } else {                                     // K, T, C, CS, nks, nct, nslice, dgrad, nt: bf16 x 8 per index
        wn = r[3] * r[4] * r[5];
        on = (r[9] * r[7] + 4) * r[8] * 64 * 8;
      }
      std::vector<long long> e = {ext[2 * k], ext[2 * k + 1]};
      fits(e, 0, wn, "pack_w_multi", "w");
      fits(e, 1, on, "pack_w_multi", "out");
    }
    chk(fn_pack_w_multi(jobs.data(), n, S(st)), "pack_w_multi");
  });
  m.def("halo_pack_w", [](uintptr_t w, uintptr_t out, int K0, int C0, int K, int T, int C, int mode, int stage_k,
                          uintptr_t st, std::vector<long long> ext) {
    // ext = {numel(w), numel(out)}; out holds K * C * (taps padded to the stage) elements
    fits(ext, 0, (long long)K0 * T * C0, "halo_pack_w", "w");
    // (the kernel writes K * C * Tp elements: the tap count padded to whole stages, as
    // fn_halo_pack_w derives it -- checking K * C * T would let an output sized by T overrun)
    {
      const int Csrc = mode == 0 ? C : K;
      const int CS = Csrc % 16 == 0 ? 16 : (Csrc % 8 == 0 ? 8 : 0);
      const int tps = CS > 0 && stage_k > 0 ? stage_k / CS : 0;
      const long long Tp = tps > 0 ? (long long)(T + tps - 1) / tps * tps : T;
      fits(ext, 1, (long long)K * C * Tp, "halo_pack_w", "out");
    }
    chk(fn_halo_pack_w(P<const float*>(w), P<void*>(out), K0, C0, K, T, C, mode, stage_k, S(st)), "halo_pack_w");
  });
  m.def("ew_binary", [](uintptr_t a, uintptr_t b, uintptr_t out, long long n, int op, uintptr_t st) {
    chk(fn_ew_binary(P<const void*>(a), P<const void*>(b), P<void*>(out), n, op, S(st)), "ew_binary");
  });
  m.def("ew_mul_bwd", [](uintptr_t g, uintptr_t a, uintptr_t b, uintptr_t da, uintptr_t db, long long n,
                         uintptr_t st) {
    chk(fn_ew_mul_bwd(P<const void*>(g), P<const void*>(a), P<const void*>(b), P<void*>(da), P<void*>(db), n, S(st)),
        "ew_mul_bwd");
  });
  m.def("concat2", [](uintptr_t a, uintptr_t b, uintptr_t out, long long outer, int ia, int ib, int dir,
                      uintptr_t st) {
    chk(fn_concat2(P<void*>(a), P<void*>(b), P<void*>(out), outer, ia, ib, dir, S(st)), "concat2");
  });
  m.def("pad3", [](uintptr_t x, uintptr_t out, std::vector<int> geom, int dir, uintptr_t st) {
    need(geom, 8, "pad3");
    chk(fn_pad3(P<void*>(x), P<void*>(out), geom.data(), dir, S(st)), "pad3");
  });
  m.def("pad_channels", [](uintptr_t x, uintptr_t out, long long rows, int C, int CP, int dir, uintptr_t st,
                           std::vector<long long> ext) {
    // dir 0: x [rows, C] -> out [rows, CP]; dir 1: x [rows, CP] -> out [rows, C]
    fits(ext, 0, rows * (dir == 0 ? C : CP), "pad_channels", "x");
    fits(ext, 1, rows * (dir == 0 ? CP : C), "pad_channels", "out");
    chk(fn_pad_channels(P<void*>(x), P<void*>(out), rows, C, CP, dir, S(st)), "pad_channels");
  }, py::arg("x"), py::arg("out"), py::arg("rows"), py::arg("C"), py::arg("CP"), py::arg("dir"), py::arg("st"),
     py::arg("ext"));
  m.def("dense_splits", &fn_dense_splits);
  m.def("dense_fwd", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t out, uintptr_t part, int M, int N, int K,
                        int nsplit, int act, int out_fp32, uintptr_t st, std::vector<long long> ext, int wbf16) {
    fits(ext, 0, (long long)M * K, "dense_fwd", "x");
    fits(ext, 1, (long long)N * K, "dense_fwd", "w");
    fits(ext, 2, (long long)M * N, "dense_fwd", "out");
    fits(ext, 3, (long long)nsplit * M * N, "dense_fwd", "part");
    chk(fn_dense_fwd(P<const void*>(x), P<const void*>(w), P<const float*>(bias), P<void*>(out), P<float*>(part), M,
                     N, K, nsplit, act, out_fp32, wbf16, S(st)),
        "dense_fwd");
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("out"), py::arg("part"), py::arg("M"), py::arg("N"),
     py::arg("K"), py::arg("S"), py::arg("act"), py::arg("out_fp32"), py::arg("st"),
     py::arg("ext") = std::vector<long long>(), py::arg("wbf16") = 0);
  // ya / act: g is dy and the layer's activation backward is applied as it is loaded (ya =
  // the activation output [M][N], the same extent as g)
  m.def("dense_dgrad", [](uintptr_t g, uintptr_t w, uintptr_t dx, int M, int N, int K, uintptr_t st,
                          std::vector<long long> ext, uintptr_t ya, int act) {
    fits(ext, 0, (long long)M * N, "dense_dgrad", "g");
    fits(ext, 1, (long long)N * K, "dense_dgrad", "w");
    fits(ext, 2, (long long)M * K, "dense_dgrad", "dx");
    if (ya) fits(ext, 3, (long long)M * N, "dense_dgrad", "ya");
    chk(fn_dense_dgrad(P<const void*>(g), P<const float*>(w), P<void*>(dx), M, N, K, S(st), P<const void*>(ya), act),
        "dense_dgrad");
  }, py::arg("g"), py::arg("w"), py::arg("dx"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("st"),
     py::arg("ext") = std::vector<long long>(), py::arg("ya") = 0, py::arg("act") = 0);
  m.def("dense_wgrad_slices", &fn_dense_wgrad_slices);
  // part: fp32 workspace of S * (N*K + N) elements when S > 1 (dense_wgrad_slices)
  m.def("dense_wgrad", [](uintptr_t g, uintptr_t x, uintptr_t dw, uintptr_t db, int M, int N, int K, uintptr_t st,
                          std::vector<long long> ext, uintptr_t part, int slices, uintptr_t ya, int act) {
    fits(ext, 0, (long long)M * N, "dense_wgrad", "g");
    fits(ext, 1, (long long)M * K, "dense_wgrad", "x");
    fits(ext, 2, (long long)N * K, "dense_wgrad", "dw");
    if (slices > 1) fits(ext, 3, (long long)slices * ((long long)N * K + N), "dense_wgrad", "part");
    if (ya) fits(ext, 4, (long long)M * N, "dense_wgrad", "ya");   // (the activation output dy is taken through)
    chk(fn_dense_wgrad(P<const void*>(g), P<const void*>(x), P<float*>(dw), P<float*>(db), M, N, K, P<float*>(part),
                       slices, S(st), P<const void*>(ya), act),
        "dense_wgrad");
  }, py::arg("g"), py::arg("x"), py::arg("dw"), py::arg("db"), py::arg("M"), py::arg("N"), py::arg("K"),
     py::arg("st"), py::arg("ext") = std::vector<long long>(), py::arg("part") = 0, py::arg("slices") = 1,
     py::arg("ya") = 0, py::arg("act") = 0);
  // sub-pixel decoder weight maps (conv_halo.hip): mode 0 class weights [8][K][8][C] from w
  // [K][27][C], 1 dgrad weights [C][8][8][K], 2 the folded weight gradient [K][27][C] from [8][K][8][C]
  m.def("subpixel_wmap", [](uintptr_t src, uintptr_t dst, int K, int C, int mode, uintptr_t st,
                            std::vector<long long> ext) {
    const long long small = 27LL * K * C, big = 64LL * K * C;
    fits(ext, 0, mode == 2 ? big : small, "subpixel_wmap", "src");
    fits(ext, 1, mode == 2 ? small : big, "subpixel_wmap", "dst");
    chk(fn_subpixel_wmap(P<const float*>(src), P<float*>(dst), K, C, mode, S(st)), "subpixel_wmap");
  });
  m.def("s2d_weight_map", [](uintptr_t src, uintptr_t dst, std::vector<int> geom, int dir, uintptr_t st,
                             std::vector<long long> ext) {
    need(geom, 12, "s2d_weight_map");
    const long long big = prod({geom[0], geom[8], geom[9], geom[10], geom[11]});
    const long long small = prod({geom[0], geom[1], geom[2], geom[3], geom[4]});
    fits(ext, 0, dir == 0 ? small : big, "s2d_weight_map", "src");
    fits(ext, 1, dir == 0 ? big : small, "s2d_weight_map", "dst");
    chk(fn_s2d_weight_map(P<const float*>(src), P<float*>(dst), geom.data(), dir, S(st)), "s2d_weight_map");
  }, py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("dir"), py::arg("st"),
     py::arg("ext") = std::vector<long long>());
  m.def("s2d_pack", [](uintptr_t x, uintptr_t out, std::vector<int> geom, uintptr_t st, int u8) {
    // u8: x holds uint8 voxels (binary occupancy), else bf16
    if (geom.size() != 12 && geom.size() != 15) throw std::runtime_error("s2d_pack: geometry of 12 or 15 ints");
    chk(fn_s2d_pack(P<const void*>(x), P<void*>(out), geom.data(), (int)geom.size(), S(st), u8), "s2d_pack");
  });
  m.def("conv_halo_f8", [](uintptr_t src, uintptr_t wt, uintptr_t scale, uintptr_t bias, uintptr_t out,
                           float inv_out_scale, uintptr_t toffs, std::vector<int> geom, int ncol, int out_f8, int relu,
                           uintptr_t st) {
    need(geom, 16, "conv_halo_f8");
    chk(fn_conv_halo_f8(P<const void*>(src), P<const void*>(wt), P<const float*>(scale), P<const float*>(bias),
                        P<void*>(out), inv_out_scale, P<const int*>(toffs), geom.data(), ncol, out_f8, relu, S(st)),
        "conv_halo_f8");
  });
  m.def("s2d_tap_f8", [](uintptr_t x, uintptr_t y, std::vector<int> g, float inv_scale, uintptr_t st,
                         std::vector<long long> ext, int i8) {
    // g = {N, D, H, W, D2, H2, W2o, J}; ext = {numel(x), numel(y)}
    need(g, 8, "s2d_tap_f8");
    fits(ext, 0, prod({g[0], g[1], g[2], g[3]}), "s2d_tap_f8", "x");
    fits(ext, 1, prod({g[0], g[4], g[5], g[6], 8LL * g[7]}), "s2d_tap_f8", "y");
    chk(fn_s2d_tap_f8(P<const void*>(x), P<void*>(y), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], inv_scale, i8, S(st)),
        "s2d_tap_f8");
  });
  // block-scaled e4m3 of a bf16 [M][C] tensor: y [M][C] bytes, sc a scale dword per row (ext = {x, y, sc})
  m.def("quant_fp8_block", [](uintptr_t x, uintptr_t y, uintptr_t sc, long long M, int C, uintptr_t st,
                              std::vector<long long> ext) {
    fits(ext, 0, M * C, "quant_fp8_block", "x");
    fits(ext, 1, M * C, "quant_fp8_block", "y");
    fits(ext, 2, M, "quant_fp8_block", "sc");
    chk(fn_quant_fp8_block(P<const void*>(x), P<void*>(y), P<void*>(sc), M, C, S(st)), "quant_fp8_block");
  }, py::arg("x"), py::arg("y"), py::arg("sc"), py::arg("M"), py::arg("C"), py::arg("st"),
     py::arg("ext") = std::vector<long long>());
  // one v_mfma_scale_f32_16x16x128_f8f6f4 on one wave (a, b: 64 x 32 bytes; sa, sb: 64 int32; d: 64 x 4 fp32)
  m.def("mfma_scale_probe", [](uintptr_t a, uintptr_t b, uintptr_t sa, uintptr_t sb, uintptr_t d, uintptr_t st) {
    chk(fn_mfma_scale_probe(P<const void*>(a), P<const void*>(b), P<const int*>(sa), P<const int*>(sb), P<float*>(d),
                            S(st)),
        "mfma_scale_probe");
  });
  m.def("quant_fp8", [](uintptr_t x, uintptr_t y, long long n, float inv_scale, uintptr_t st) {
    chk(fn_quant_fp8(P<const void*>(x), P<void*>(y), n, inv_scale, S(st)), "quant_fp8");
  });
  m.def("dw_fwd", [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t y, std::vector<int> geom, int act,
                     uintptr_t st) {
    need(geom, 20, "dw_fwd");
    chk(fn_dw_fwd(P<const void*>(x), P<const float*>(w), P<const float*>(b), P<void*>(y), geom.data(), act, S(st)),
        "dw_fwd");
  });
  m.def("dw_dgrad", [](uintptr_t dy, uintptr_t w, uintptr_t dx, std::vector<int> geom, uintptr_t st) {
    need(geom, 20, "dw_dgrad");
    chk(fn_dw_dgrad(P<const void*>(dy), P<const float*>(w), P<void*>(dx), geom.data(), S(st)), "dw_dgrad");
  });
  // part: fp32 scratch [splits][C][taps] (the per-split partials, added into dw in a fixed order)
  m.def("dw_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw, std::vector<int> geom, int splits, uintptr_t st,
                       uintptr_t part, long long part_n) {
    need(geom, 20, "dw_wgrad");
    if (part_n < prod({splits, geom[4], geom[8] * geom[9] * geom[10]}))
      throw std::runtime_error("dw_wgrad: part scratch too small");
    chk(fn_dw_wgrad(P<const void*>(dy), P<const void*>(x), P<float*>(dw), geom.data(), splits, S(st), P<float*>(part)),
        "dw_wgrad");
  });
  m.def("conv_halo_wgrad_yblocks", [](std::vector<int> geom, int cout) {
    need(geom, 17, "conv_halo_wgrad_yblocks");
    return fn_conv_halo_wgrad_yblocks(geom.data(), cout);
  });
  // psc / psh / pact: optional input prologue x <- pact(x * psc[k] + psh[k]) (BN + act of the
  // producing layer, never materialised)
  // sy / ssc / ssh / spart / sact: BN-backward moments of the layer whose dz this call computes
  // (spart fp32 [pw_fwd_blocks][2][N])
  m.def("pw_fwd", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, long long M, int K, int N, int act,
                     uintptr_t st, uintptr_t psc, uintptr_t psh, int pact, uintptr_t sy, uintptr_t ssc,
                     uintptr_t ssh, uintptr_t spart, int sact) {
    chk(fn_pw_fwd(P<const void*>(x), P<const void*>(w), P<const float*>(bias), P<void*>(y), M, K, N, act, S(st),
                  P<const float*>(psc), P<const float*>(psh), pact, P<const void*>(sy), P<const float*>(ssc),
                  P<const float*>(ssh), P<float*>(spart), sact),
        "pw_fwd");
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("M"), py::arg("K"), py::arg("N"),
     py::arg("act"), py::arg("st"), py::arg("psc") = 0, py::arg("psh") = 0, py::arg("pact") = 0, py::arg("sy") = 0,
     py::arg("ssc") = 0, py::arg("ssh") = 0, py::arg("spart") = 0, py::arg("sact") = 0);
  m.def("pw_fwd_blocks", &fn_pw_fwd_blocks);
  m.def("pw_xent_blocks", &fn_pw_xent_blocks);
  m.def("part_reduce", [](uintptr_t part, uintptr_t dst, long long n, int W, int accumulate, uintptr_t st,
                          std::vector<long long> ext) {
    // dst[i] (+)= sum over the W partial rows part[w][i], added in row order; ext = {numel(part), numel(dst)}
    fits(ext, 0, n * W, "part_reduce", "part");
    fits(ext, 1, n, "part_reduce", "dst");
    chk(fn_part_reduce(P<const float*>(part), P<float*>(dst), n, W, accumulate, S(st)), "part_reduce");
  });
  m.def("seghead_part_len", &fn_seghead_part_len);
  m.def("seghead_blocks", &fn_seghead_blocks);
  m.def("seghead_loss", [](uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t w, uintptr_t bias, uintptr_t labels,
                           uintptr_t dz, uintptr_t part, long long M, int K, int NC, int act, float xscale,
                           float smoothing, uintptr_t st, std::vector<long long> ext, int lab8, int hits) {
    fits(ext, 0, M * K, "seghead_loss", "y");
    fits(ext, 1, (long long)NC * K, "seghead_loss", "w");
    fits(ext, 2, M, "seghead_loss", "labels");
    fits(ext, 3, M * K, "seghead_loss", "dz");
    fits(ext, 4, (long long)fn_seghead_blocks(M) * fn_seghead_part_len(), "seghead_loss", "part");
    chk(fn_seghead_loss(P<const void*>(y), P<const float*>(sc), P<const float*>(sh), P<const void*>(w),
                        P<const float*>(bias), P<const void*>(labels), P<void*>(dz), P<float*>(part), M, K, NC,
                        act, xscale, smoothing, S(st), lab8, hits),
        "seghead_loss");
  }, py::arg("y"), py::arg("sc"), py::arg("sh"), py::arg("w"), py::arg("bias"), py::arg("labels"), py::arg("dz"),
     py::arg("part"), py::arg("M"), py::arg("K"), py::arg("NC"), py::arg("act"), py::arg("xscale"),
     py::arg("smoothing"), py::arg("st"), py::arg("ext"), py::arg("lab8") = 0, py::arg("hits") = 1);
  m.def("pw_fwd_xent", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t dlog, long long M, int K, int N,
                          uintptr_t psc, uintptr_t psh, int pact, uintptr_t labels, uintptr_t xpart, float xscale,
                          float smoothing, uintptr_t st, std::vector<long long> ext) {
    fits(ext, 0, M * K, "pw_fwd_xent", "x");
    fits(ext, 1, M * N, "pw_fwd_xent", "dlog");
    fits(ext, 2, M, "pw_fwd_xent", "labels");
    fits(ext, 3, 2LL * fn_pw_xent_blocks(M), "pw_fwd_xent", "xpart");
    chk(fn_pw_fwd_xent(P<const void*>(x), P<const void*>(w), P<const float*>(bias), P<void*>(dlog), M, K, N,
                       P<const float*>(psc), P<const float*>(psh), pact, P<const long long*>(labels), P<float*>(xpart),
                       xscale, smoothing, S(st)),
        "pw_fwd_xent");
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("dlog"), py::arg("M"), py::arg("K"), py::arg("N"),
     py::arg("psc"), py::arg("psh"), py::arg("pact"), py::arg("labels"), py::arg("xpart"), py::arg("xscale"),
     py::arg("smoothing"), py::arg("st"), py::arg("ext"));
  // part: fp32 scratch of pw_wgrad_blocks(M, K, N) x N x K floats (per-workgroup partials)
  m.def("pw_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t dw, long long M, int K, int N, uintptr_t st,
                       uintptr_t psc, uintptr_t psh, int pact, uintptr_t part, long long part_n) {
    if (part_n < (long long)fn_pw_wgrad_blocks(M, K, N) * N * K) throw std::runtime_error("pw_wgrad: part scratch too small");
    chk(fn_pw_wgrad(P<const void*>(dy), P<const void*>(x), P<float*>(dw), M, K, N, S(st), P<const float*>(psc),
                    P<const float*>(psh), pact, P<float*>(part)),
        "pw_wgrad");
  }, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("M"), py::arg("K"), py::arg("N"), py::arg("st"),
     py::arg("psc") = 0, py::arg("psh") = 0, py::arg("pact") = 0, py::arg("part") = 0, py::arg("part_n") = 0);
  m.def("pw_wgrad_blocks", &fn_pw_wgrad_blocks);
  m.def("conv_halo_workers", [](std::vector<int> geom, int ncol) {
    need(geom, 17, "conv_halo_workers");
    return fn_conv_halo_workers(geom.data(), ncol);
  });
  m.def("conv_halo_lds", [](std::vector<int> geom, int ncol) {
    need(geom, 17, "conv_halo_lds");
    return fn_conv_halo_lds(geom.data(), ncol);
  });
  // dw (and db) are accumulated into from the split partials in `scratch` (igemm_wgrad_part floats)
  m.def("igemm_wgrad", [](uintptr_t dy, uintptr_t src, uintptr_t dw, uintptr_t tab, std::vector<int> geom,
                          long long M, int Cout, int K, int splits, int vec, uintptr_t st, int ccrop, int cpad,
                          uintptr_t ya, int act, uintptr_t db, int kout, uintptr_t scratch, long long scratch_n) {
    need(geom, 14, "igemm_wgrad");
    if (scratch_n < fn_igemm_wgrad_part(Cout, K, splits, ccrop, cpad, kout, db ? 1 : 0))
      throw std::runtime_error("igemm_wgrad: partial scratch too small");
    chk(fn_igemm_wgrad(P<const void*>(dy), P<const void*>(src), P<float*>(dw), P<const int*>(tab), geom.data(), M,
                       Cout, K, splits, vec, S(st), ccrop, cpad, P<const void*>(ya), act, P<float*>(db), kout,
                       P<float*>(scratch)),
        "igemm_wgrad");
  }, py::arg("dy"), py::arg("src"), py::arg("dw"), py::arg("tab"), py::arg("geom"), py::arg("M"), py::arg("Cout"),
     py::arg("K"), py::arg("splits"), py::arg("vec"), py::arg("st"), py::arg("ccrop") = 0, py::arg("cpad") = 0,
     py::arg("ya") = 0, py::arg("act") = 0, py::arg("db") = 0, py::arg("kout") = 0, py::arg("scratch") = 0,
     py::arg("scratch_n") = 0);
  m.def("igemm_wgrad_part", &fn_igemm_wgrad_part);
  m.def("colstats", [](uintptr_t x, uintptr_t dz, uintptr_t scale, uintptr_t shift, uintptr_t mean, uintptr_t invstd,
                       uintptr_t part, long long M, int C, int act, int mode, int nb, uintptr_t st) {
    chk(fn_colstats(P<const void*>(x), P<const void*>(dz), P<const float*>(scale), P<const float*>(shift),
                    P<const float*>(mean), P<const float*>(invstd), P<float*>(part), M, C, act, mode, nb, S(st)),
        "colstats");
  });
  m.def("experiments_built", [] {
    // FN_BUILD_EXPERIMENTS=1 builds: the int8 fp8-stem instance, timing variants
#ifdef FN_EXPERIMENTS
    return true;
#else
    return false;
#endif
  });
  m.def("colstats_blocks", &fn_colstats_blocks, py::arg("M"), py::arg("C"), py::arg("mode"), py::arg("act"));
  m.def("bn_finalize", [](uintptr_t part, int nb, int C, double count, uintptr_t gamma, uintptr_t beta,
                          uintptr_t rmean, uintptr_t rvar, float momentum, float eps, uintptr_t o0, uintptr_t o1,
                          uintptr_t o2, uintptr_t o3, int mode, uintptr_t st) {
    chk(fn_bn_finalize(P<const float*>(part), nb, C, count, P<const float*>(gamma), P<const float*>(beta),
                       P<float*>(rmean), P<float*>(rvar), momentum, eps, P<float*>(o0), P<float*>(o1), P<float*>(o2),
                       P<float*>(o3), mode, S(st)),
        "bn_finalize");
  });
  m.def("bn_apply", [](uintptr_t y, uintptr_t scale, uintptr_t shift, uintptr_t z, long long total, int C, int act,
                       uintptr_t st, uintptr_t mask, long long mask_numel) {
    // mask: optional uint8 [total / 8] relu-mask bytes (one per 8-channel chunk)
    if (mask && mask_numel * 8 != total) throw std::runtime_error("bn_apply: mask needs total / 8 bytes");
    chk(fn_bn_apply(P<const void*>(y), P<const float*>(scale), P<const float*>(shift), P<void*>(z), total, C, act,
                    S(st), P<void*>(mask)),
        "bn_apply");
  }, py::arg("y"), py::arg("scale"), py::arg("shift"), py::arg("z"), py::arg("total"), py::arg("C"), py::arg("act"),
     py::arg("st"), py::arg("mask") = 0, py::arg("mask_numel") = 0);
  m.def("bn_wdot", [](uintptr_t w, uintptr_t dw, uintptr_t part, int R, int C, int nb, uintptr_t st,
                      std::vector<long long> ext) {
    fits(ext, 0, (long long)R * C, "bn_wdot", "w");
    fits(ext, 1, (long long)R * C, "bn_wdot", "dw");
    fits(ext, 2, (long long)nb * C, "bn_wdot", "part");
    chk(fn_bn_wdot(P<const float*>(w), P<const float*>(dw), P<float*>(part), R, C, nb, S(st)), "bn_wdot");
  });
  m.def("bn_bwd_prep", [](uintptr_t gslab, int nbg, uintptr_t wpart, int nbw, int C, double count, uintptr_t gamma,
                          uintptr_t beta, uintptr_t mean, uintptr_t invstd, uintptr_t scale, uintptr_t shift,
                          uintptr_t dbeta, uintptr_t kc, uintptr_t g, uintptr_t y, long long M, uintptr_t st,
                          std::vector<long long> ext) {
    fits(ext, 0, 2LL * nbg * C, "bn_bwd_prep", "gslab");
    fits(ext, 1, (long long)nbw * C, "bn_bwd_prep", "wpart");
    fits(ext, 2, 3LL * C, "bn_bwd_prep", "kc");
    fits(ext, 3, M * C, "bn_bwd_prep", "g");
    fits(ext, 4, M * C, "bn_bwd_prep", "y");
    chk(fn_bn_bwd_prep(P<const float*>(gslab), nbg, P<const float*>(wpart), nbw, C, count, P<const float*>(gamma),
                       P<const float*>(beta), P<const float*>(mean), P<const float*>(invstd), P<const float*>(scale),
                       P<const float*>(shift), P<float*>(dbeta), P<float*>(kc), P<const void*>(g), P<const void*>(y),
                       M, S(st)),
        "bn_bwd_prep");
  });
  m.def("bn_bwd_apply_k_blocks", &fn_bn_bwd_apply_k_blocks);
  m.def("bn_bwd_apply_k", [](uintptr_t g, uintptr_t y, uintptr_t kc, uintptr_t mean, uintptr_t invstd,
                             uintptr_t shift, uintptr_t dy, long long M, int C, uintptr_t part, int nb, uintptr_t st,
                             std::vector<long long> ext) {
    fits(ext, 0, M * C, "bn_bwd_apply_k", "g");
    fits(ext, 1, M * C, "bn_bwd_apply_k", "y");
    fits(ext, 2, M * C, "bn_bwd_apply_k", "dy");
    fits(ext, 3, 2LL * nb * C, "bn_bwd_apply_k", "part");
    chk(fn_bn_bwd_apply_k(P<const void*>(g), P<const void*>(y), P<const float*>(kc), P<const float*>(mean),
                          P<const float*>(invstd), P<const float*>(shift), P<void*>(dy), M, C, P<float*>(part), nb,
                          S(st)),
        "bn_bwd_apply_k");
  });
  m.def("bn_bwd_apply", [](uintptr_t dz, uintptr_t y, uintptr_t scale, uintptr_t shift, uintptr_t mean,
                           uintptr_t invstd, uintptr_t dbeta, uintptr_t dgamma, uintptr_t dy, long long total, int C,
                           float inv_count, int act, uintptr_t st) {
    chk(fn_bn_bwd_apply(P<const void*>(dz), P<const void*>(y), P<const float*>(scale), P<const float*>(shift),
                        P<const float*>(mean), P<const float*>(invstd), P<const float*>(dbeta),
                        P<const float*>(dgamma), P<void*>(dy), total, C, inv_count, act, S(st)),
        "bn_bwd_apply");
  });
  // ext = {dz / y numel, dsh numel}
  m.def("bn_bwd_apply_s2d", [](uintptr_t dz, uintptr_t y, uintptr_t scale, uintptr_t shift, uintptr_t mean,
                               uintptr_t invstd, uintptr_t dbeta, uintptr_t dgamma, uintptr_t dsh, int N, int FD,
                               int FH, int FW, int C, float inv_count, int act, uintptr_t st,
                               std::vector<long long> ext) {
    fits(ext, 0, prod({N, FD, FH, FW, C}), "bn_bwd_apply_s2d", "dz/y");
    fits(ext, 1, prod({N, FD / 2 + 1, FH / 2 + 1, FW / 2 + 1, 8LL * C}), "bn_bwd_apply_s2d", "dsh");
    chk(fn_bn_bwd_apply_s2d(P<const void*>(dz), P<const void*>(y), P<const float*>(scale), P<const float*>(shift),
                            P<const float*>(mean), P<const float*>(invstd), P<const float*>(dbeta),
                            P<const float*>(dgamma), P<void*>(dsh), N, FD, FH, FW, C, inv_count, act, S(st)),
        "bn_bwd_apply_s2d");
  }, py::arg("dz"), py::arg("y"), py::arg("scale"), py::arg("shift"), py::arg("mean"), py::arg("invstd"),
     py::arg("dbeta"), py::arg("dgamma"), py::arg("dsh"), py::arg("N"), py::arg("FD"), py::arg("FH"), py::arg("FW"),
     py::arg("C"), py::arg("inv_count"), py::arg("act"), py::arg("st"), py::arg("ext"));
  // pool geometry: N D H W C | OD OH OW | KD KH KW | sd sh sw | pd ph pw; ext = {x, out}
  auto check_pool = [](const std::vector<int>& g, const std::vector<long long>& ext, const char* what) {
    fits(ext, 0, prod({g[0], g[1], g[2], g[3], g[4]}), what, "x");
    fits(ext, 1, prod({g[0], g[5], g[6], g[7], g[4]}), what, "out");
  };
  m.def("pool_fwd", [check_pool](uintptr_t x, uintptr_t out, uintptr_t scale, uintptr_t shift, std::vector<int> geom,
                       int is_max, int count_pad, int act, uintptr_t st, std::vector<long long> ext) {
    need(geom, 17, "pool_fwd");
    check_pool(geom, ext, "pool_fwd");
    chk(fn_pool_fwd(P<const void*>(x), P<void*>(out), P<const float*>(scale), P<const float*>(shift), geom.data(),
                    is_max, count_pad, act, S(st)),
        "pool_fwd");
  }, py::arg("x"), py::arg("out"), py::arg("scale"), py::arg("shift"), py::arg("geom"), py::arg("is_max"),
     py::arg("count_pad"), py::arg("act"), py::arg("st"), py::arg("ext") = std::vector<long long>());
  m.def("pool_bwd", [check_pool](uintptr_t dout, uintptr_t x, uintptr_t dx, uintptr_t scale, uintptr_t shift,
                       std::vector<int> geom, int is_max, int count_pad, int act, uintptr_t st,
                       std::vector<long long> ext) {
    need(geom, 17, "pool_bwd");
    check_pool(geom, ext, "pool_bwd");   // ext = {x (and dx), dout}
    chk(fn_pool_bwd(P<const void*>(dout), P<const void*>(x), P<void*>(dx), P<const float*>(scale),
                    P<const float*>(shift), geom.data(), is_max, count_pad, act, S(st)),
        "pool_bwd");
  }, py::arg("dout"), py::arg("x"), py::arg("dx"), py::arg("scale"), py::arg("shift"), py::arg("geom"),
     py::arg("is_max"), py::arg("count_pad"), py::arg("act"), py::arg("st"), py::arg("ext") = std::vector<long long>());
  m.def("pool_bwd_stats_blocks", [](std::vector<int> geom) {
    need(geom, 17, "pool_bwd_stats_blocks");
    return fn_pool_bwd_stats_blocks(geom.data());
  });
  m.def("pool_bwd_stats", [check_pool](uintptr_t dout, uintptr_t x, uintptr_t dx, uintptr_t scale, uintptr_t shift,
                             std::vector<int> geom, int act, uintptr_t part, uintptr_t st, std::vector<long long> ext) {
    need(geom, 17, "pool_bwd_stats");
    check_pool(geom, ext, "pool_bwd_stats");   // ext = {x (and dx), dout, part}
    fits(ext, 2, 2LL * fn_pool_bwd_stats_blocks(geom.data()) * geom[4], "pool_bwd_stats", "part");
    chk(fn_pool_bwd_stats(P<const void*>(dout), P<const void*>(x), P<void*>(dx), P<const float*>(scale),
                          P<const float*>(shift), geom.data(), act, P<float*>(part), S(st)),
        "pool_bwd_stats");
  }, py::arg("dout"), py::arg("x"), py::arg("dx"), py::arg("scale"), py::arg("shift"), py::arg("geom"),
     py::arg("act"), py::arg("part"), py::arg("st"), py::arg("ext") = std::vector<long long>());
  m.def("pool_bn_bwd_apply", [check_pool](uintptr_t dout, uintptr_t y, uintptr_t scale, uintptr_t shift,
                                uintptr_t mean, uintptr_t invstd, uintptr_t dbeta, uintptr_t dgamma, uintptr_t dy,
                                std::vector<int> geom, int act, float inv_count, uintptr_t st,
                                std::vector<long long> ext) {
    need(geom, 17, "pool_bn_bwd_apply");
    check_pool(geom, ext, "pool_bn_bwd_apply");   // ext = {y (and dy), dout}
    chk(fn_pool_bn_bwd_apply(P<const void*>(dout), P<const void*>(y), P<const float*>(scale), P<const float*>(shift),
                             P<const float*>(mean), P<const float*>(invstd), P<const float*>(dbeta),
                             P<const float*>(dgamma), P<void*>(dy), geom.data(), act, inv_count, S(st)),
        "pool_bn_bwd_apply");
  }, py::arg("dout"), py::arg("y"), py::arg("scale"), py::arg("shift"), py::arg("mean"), py::arg("invstd"),
     py::arg("dbeta"), py::arg("dgamma"), py::arg("dy"), py::arg("geom"), py::arg("act"), py::arg("inv_count"),
     py::arg("st"), py::arg("ext") = std::vector<long long>());
  m.def("upsample2x", [](uintptr_t x, uintptr_t y, int N, int D, int H, int W, int C, int backward, uintptr_t st) {
    chk(fn_upsample2x(P<const void*>(x), P<void*>(y), N, D, H, W, C, backward, S(st)), "upsample2x");
  });
  m.def("softmax_xent_blocks", [](long long B, int NC) { return fn_softmax_xent_blocks(B, NC); });
  m.def("softmax_xent_rows", [](uintptr_t logits, int in_bf16, uintptr_t labels, uintptr_t block_loss,
                                uintptr_t dlogits, uintptr_t correct, long long B, int NC, float gscale,
                                float smoothing, uintptr_t st) {
    chk(fn_softmax_xent_rows(P<const void*>(logits), in_bf16, P<const long long*>(labels), P<float*>(block_loss),
                             P<void*>(dlogits), P<int*>(correct), B, NC, gscale, smoothing, S(st)),
        "softmax_xent_rows");
  });
  m.def("softmax_rows", [](uintptr_t x, uintptr_t y, long long M, int N, int backward, uintptr_t g, uintptr_t st,
                           std::vector<long long> ext) {
    // forward: y = softmax(x) over rows of N fp32; backward (x = y, y = dx): dx = y * (g - sum g y)
    fits(ext, 0, M * N, "softmax_rows", "x");
    fits(ext, 1, M * N, "softmax_rows", "y");
    if (backward) fits(ext, 2, M * N, "softmax_rows", "g");
    chk(fn_softmax_rows(P<const float*>(x), P<float*>(y), M, N, backward, P<const float*>(g), S(st)), "softmax_rows");
  });
  m.def("cu_occupy", [](int nwg, int usec, int lds, uintptr_t sink, uintptr_t st) {
    // (measurement only: pins nwg CUs on the given stream for usec microseconds; sink >= 1 KB)
    chk(fn_cu_occupy(nwg, usec, lds, P<void*>(sink), S(st)), "cu_occupy");
  });
  m.def("adam_flat_dev", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t pb, long long n,
                            uintptr_t hp, uintptr_t t, int keras_eps, uintptr_t st) {
    chk(fn_adam_flat_dev(P<float*>(p), P<const float*>(g), P<float*>(mm), P<float*>(v), P<void*>(pb), n,
                         P<const float*>(hp), P<int*>(t), keras_eps, S(st)),
        "adam_flat_dev");
  });
  m.def("adam_flat", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t pb, long long n, float lr,
                        float b1, float b2, float eps, float wd, float bc1, float bc2, float gscale, int keras_eps,
                        uintptr_t st) {
    chk(fn_adam_flat(P<float*>(p), P<const float*>(g), P<float*>(mm), P<float*>(v), P<void*>(pb), n, lr, b1, b2, eps,
                     wd, bc1, bc2, gscale, keras_eps, S(st)),
        "adam_flat");
  });
  m.def("sgd_flat", [](uintptr_t p, uintptr_t g, uintptr_t buf, uintptr_t pb, long long n, float lr, float momentum,
                       float wd, int nesterov, float gscale, uintptr_t st) {
    chk(fn_sgd_flat(P<float*>(p), P<const float*>(g), P<float*>(buf), P<void*>(pb), n, lr, momentum, wd, nesterov,
                    gscale, S(st)),
        "sgd_flat");
  });
  m.def("bias_act", [](uintptr_t x, uintptr_t bias, uintptr_t y, long long total, int C, int act, uintptr_t st) {
    chk(fn_bias_act(P<const void*>(x), P<const float*>(bias), P<void*>(y), total, C, act, S(st)), "bias_act");
  });
  m.def("act_bwd", [](uintptr_t dy, uintptr_t y, uintptr_t dx, long long total, int act, uintptr_t st) {
    chk(fn_act_bwd(P<const void*>(dy), P<const void*>(y), P<void*>(dx), total, act, S(st)), "act_bwd");
  });
  m.def("dropout", [](uintptr_t x, uintptr_t y, long long total, float p, unsigned seed, unsigned offset,
                      uintptr_t st) {
    chk(fn_dropout(P<const void*>(x), P<void*>(y), total, p, seed, offset, S(st)), "dropout");
  });
  m.def("unpack_bits", [](uintptr_t bits, uintptr_t out, long long nbytes, uintptr_t st) {
    chk(fn_unpack_bits(P<const void*>(bits), P<void*>(out), nbytes, S(st)), "unpack_bits");
  });
  m.def("copy2", [](uintptr_t d0, uintptr_t s0, long long n0, uintptr_t d1, uintptr_t s1, long long n1, uintptr_t st) {
    chk(fn_copy2(P<void*>(d0), P<const void*>(s0), n0, P<void*>(d1), P<const void*>(s1), n1, S(st)), "copy2");
  });
  m.def("scale_unless_one", [](uintptr_t x, int is_bf16, uintptr_t s, long long n, uintptr_t st) {
    chk(fn_scale_unless_one(P<void*>(x), is_bf16, P<const float*>(s), n, S(st)), "scale_unless_one");
  });
  m.def("cast_f32_bf16", [](uintptr_t x, uintptr_t y, long long n, uintptr_t st) {
    chk(fn_cast_f32_bf16(P<const float*>(x), P<void*>(y), n, S(st)), "cast_f32_bf16");
  });
}
