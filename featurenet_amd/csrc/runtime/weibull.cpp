// Batched reverse-Weibull maximum-likelihood fits for the CLEVER robustness score.
//
// Reference: the vendored ART metrics (reference model/metrics.py:242-324, clever_t) fit
// scipy.stats.weibull_min to the negated per-batch maxima of the class-gradient norms with
// `weibull_min.fit(-values, c_init, optimizer=fmin)` -- one Nelder-Mead run of ~300 Python-level
// likelihood evaluations per (sample, target class): ~34 ms each, 2.5 minutes of host time for
// the reference's 500-sample x 9-target robustness set.  This file is the same estimator in
// C++, run for every (sample, target) problem of a robustness evaluation in one call on a
// thread pool:
//
//   * the start point of scipy 1.15 weibull_min.fit with a shape guess: c = c_init,
//     scale = sqrt(var / (G(1+2/c) - G(1+1/c)^2)), loc = mean - scale * G(1+1/c)
//     (numpy's pairwise summation for the moments);
//   * the penalized negative log-likelihood of rv_continuous._penalized_nnlf (points outside
//     the support and non-finite log-pdf terms cost log(DBL_MAX) * 100 each);
//   * scipy.optimize.fmin's Nelder-Mead (rho 1, chi 2, psi 0.5, sigma 0.5, initial simplex
//     +5 % per coordinate, xtol / ftol termination, the function-call cap), step for step,
//     with the stable small-array argsort numpy uses for the 4-point simplex.
//
// tests/test_robust.py checks the fitted parameters against scipy on random problems.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

// numpy's pairwise summation (umath pairwise_sum, contiguous float64) for the lengths the
// fits see; blocks of 128 are split recursively as numpy does
double np_sum(const double* a, long n) {
  if (n < 8) {
    double res = 0.0;
    for (long i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    long i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  long n2 = n / 2;
  n2 -= n2 % 8;
  return np_sum(a, n2) + np_sum(a + n2, n - n2);
}

const double kLogXMax = std::log(DBL_MAX);
const double kInf = std::numeric_limits<double>::infinity();

struct Nnlf {
  const double* data;
  int n;
  mutable std::vector<double> terms;
  double operator()(const double* th) const {
    const double c = th[0], loc = th[1], scale = th[2];
    if (!(c > 0.0) || !(scale > 0.0)) return kInf;       // _argcheck(c) and scale > 0
    terms.clear();
    long bad = 0;
    const double logc = std::log(c);
    for (int i = 0; i < n; ++i) {
      const double x = (data[i] - loc) / scale;
      if (!(0.0 < x && x < kInf)) {                     // _support_mask
        ++bad;
        continue;
      }
      const double xl = (c - 1.0) == 0.0 ? 0.0 : (c - 1.0) * std::log(x);   // xlogy(c - 1, x)
      const double t = logc + xl - std::pow(x, c);
      if (std::isfinite(t)) terms.push_back(t);
      else ++bad;
    }
    const double total = np_sum(terms.data(), (long)terms.size());
    return (-total + (double)bad * kLogXMax * 100.0) + (double)n * std::log(scale);
  }
};

// stable insertion sort of the simplex by f (numpy argsort on <= 16 elements)
void sort_simplex(double sim[4][3], double f[4]) {
  for (int i = 1; i < 4; ++i) {
    double fv = f[i], sv[3] = {sim[i][0], sim[i][1], sim[i][2]};
    int j = i - 1;
    while (j >= 0 && f[j] > fv) {
      f[j + 1] = f[j];
      for (int k = 0; k < 3; ++k) sim[j + 1][k] = sim[j][k];
      --j;
    }
    f[j + 1] = fv;
    for (int k = 0; k < 3; ++k) sim[j + 1][k] = sv[k];
  }
}

struct Fit {
  double c, loc, scale;
  int nfev;
};

Fit fit_one(const double* data, int n, double c0, double xtol, double ftol, int maxfun) {
  // start point (weibull_min.fit with a shape guess)
  const double mean = np_sum(data, n) / n;
  std::vector<double> dev(n);
  for (int i = 0; i < n; ++i) {
    const double d = data[i] - mean;
    dev[i] = d * d;
  }
  const double var = np_sum(dev.data(), n) / n;
  const double g1 = std::tgamma(1.0 + 1.0 / c0), g2 = std::tgamma(1.0 + 2.0 / c0);
  const double scale0 = std::sqrt(var / (g2 - g1 * g1));
  const double loc0 = mean - scale0 * g1;

  Nnlf f{data, n, {}};
  f.terms.reserve(n);
  const double x0[3] = {c0, loc0, scale0};
  double sim[4][3], fs[4];
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 3; ++j) sim[k][j] = x0[j];
  for (int k = 0; k < 3; ++k) sim[k + 1][k] = x0[k] != 0.0 ? (1.0 + 0.05) * x0[k] : 0.00025;
  int fcalls = 0;
  bool capped = false;
  auto call = [&](const double* th, double& out) -> bool {   // false: the call cap was hit
    if (fcalls >= maxfun) return false;
    ++fcalls;
    out = f(th);
    return true;
  };
  for (int k = 0; k < 4; ++k) fs[k] = kInf;
  for (int k = 0; k < 4 && !capped; ++k)
    if (!call(sim[k], fs[k])) capped = true;
  sort_simplex(sim, fs);

  const double rho = 1.0, chi = 2.0, psi = 0.5, sigma = 0.5;
  while (fcalls < maxfun) {
    double mx = 0.0, mf = 0.0;
    for (int k = 1; k < 4; ++k) {
      for (int j = 0; j < 3; ++j) mx = std::max(mx, std::fabs(sim[k][j] - sim[0][j]));
      mf = std::max(mf, std::fabs(fs[0] - fs[k]));
    }
    if (mx <= xtol && mf <= ftol) break;
    double xbar[3];
    for (int j = 0; j < 3; ++j) xbar[j] = ((sim[0][j] + sim[1][j]) + sim[2][j]) / 3.0;
    double xr[3];
    for (int j = 0; j < 3; ++j) xr[j] = (1 + rho) * xbar[j] - rho * sim[3][j];
    double fxr;
    bool ok = call(xr, fxr);
    if (ok) {
      if (fxr < fs[0]) {
        double xe[3], fxe;
        for (int j = 0; j < 3; ++j) xe[j] = (1 + rho * chi) * xbar[j] - rho * chi * sim[3][j];
        ok = call(xe, fxe);
        if (ok) {
          if (fxe < fxr) {
            for (int j = 0; j < 3; ++j) sim[3][j] = xe[j];
            fs[3] = fxe;
          } else {
            for (int j = 0; j < 3; ++j) sim[3][j] = xr[j];
            fs[3] = fxr;
          }
        }
      } else if (fxr < fs[2]) {
        for (int j = 0; j < 3; ++j) sim[3][j] = xr[j];
        fs[3] = fxr;
      } else {
        bool shrink = false;
        if (fxr < fs[3]) {
          double xc[3], fxc;
          for (int j = 0; j < 3; ++j) xc[j] = (1 + psi * rho) * xbar[j] - psi * rho * sim[3][j];
          ok = call(xc, fxc);
          if (ok) {
            if (fxc <= fxr) {
              for (int j = 0; j < 3; ++j) sim[3][j] = xc[j];
              fs[3] = fxc;
            } else {
              shrink = true;
            }
          }
        } else {
          double xcc[3], fxcc;
          for (int j = 0; j < 3; ++j) xcc[j] = (1 - psi) * xbar[j] + psi * sim[3][j];
          ok = call(xcc, fxcc);
          if (ok) {
            if (fxcc < fs[3]) {
              for (int j = 0; j < 3; ++j) sim[3][j] = xcc[j];
              fs[3] = fxcc;
            } else {
              shrink = true;
            }
          }
        }
        if (ok && shrink) {
          for (int k = 1; k < 4 && ok; ++k) {
            for (int j = 0; j < 3; ++j) sim[k][j] = sim[0][j] + sigma * (sim[k][j] - sim[0][j]);
            ok = call(sim[k], fs[k]);
          }
        }
      }
    }
    sort_simplex(sim, fs);
    if (!ok) break;                               // (the cap: scipy's _MaxFuncCallError)
  }
  return {sim[0][0], sim[0][1], sim[0][2], fcalls};
}

// data [P, n] float64 (each row one problem, already negated like the reference's call) ->
// [P, 3] (c, loc, scale); non-finite rows give NaN
py::array_t<double> weibull_min_fit_batch(py::array_t<double, py::array::c_style | py::array::forcecast> data,
                                          double c_init, double xtol, double ftol, int maxfun, int threads) {
  if (data.ndim() != 2) throw std::runtime_error("weibull_min_fit_batch: data must be [problems, values]");
  const long P = data.shape(0);
  const int n = (int)data.shape(1);
  if (n < 2) throw std::runtime_error("weibull_min_fit_batch: need >= 2 values per problem");
  if (!(c_init > 0.0)) throw std::runtime_error("weibull_min_fit_batch: c_init must be > 0");
  py::array_t<double> out({P, (long)3});
  const double* d = data.data();
  double* o = out.mutable_data();
  {
    py::gil_scoped_release nogil;
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = (int)std::min<long>(nt, std::max<long>(1, P / 8));
    auto work = [&](long lo, long hi) {
      for (long p = lo; p < hi; ++p) {
        const double* row = d + p * n;
        bool finite = true;
        for (int i = 0; i < n; ++i) finite = finite && std::isfinite(row[i]);
        if (!finite) {
          o[3 * p] = o[3 * p + 1] = o[3 * p + 2] = std::nan("");
          continue;
        }
        const Fit r = fit_one(row, n, c_init, xtol, ftol, maxfun);
        o[3 * p] = r.c;
        o[3 * p + 1] = r.loc;
        o[3 * p + 2] = r.scale;
      }
    };
    if (nt <= 1) {
      work(0, P);
    } else {
      std::vector<std::thread> pool;
      const long chunk = (P + nt - 1) / nt;
      for (int t = 0; t < nt; ++t) {
        const long lo = t * chunk, hi = std::min(P, lo + chunk);
        if (lo < hi) pool.emplace_back(work, lo, hi);
      }
      for (auto& th : pool) th.join();
    }
  }
  return out;
}

}  // namespace

void register_weibull(py::module_& m) {
  m.def("weibull_min_fit_batch", &weibull_min_fit_batch, py::arg("data"), py::arg("c_init") = 1.0,
        py::arg("xtol") = 1e-6, py::arg("ftol") = 1e-4, py::arg("maxfun") = 1000, py::arg("threads") = 0,
        "scipy weibull_min.fit(row, c_init, optimizer=fmin(xtol, ftol, maxfun)) for every row -> [P, 3] (c, loc, "
        "scale)");
}
