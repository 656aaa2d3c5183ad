// Native PLEDGE-style product sampler (host C++17, no GPU).
//
// Replaces the reference's external Java tool PLEDGE.jar (SAT4J + SPLAR,
// invoked by pledge_evolution.py:36-47): given a feature model lowered to
// CNF (featurenet_amd/fm/splot.py), generate N valid products that are as
// different from each other as possible within a time budget.
//
//   * RandomSolver   -- DPLL with two-watched-literal unit propagation,
//                       randomised decision order and polarity, restarts.
//                       Each call yields an independent "unpredictable"
//                       valid product (PLEDGE's getUnpredictableProducts).
//   * Diversity EA   -- (1+1) evolutionary algorithm over a SET of N
//                       products; fitness = sum of pairwise Jaccard
//                       distances (bitset popcounts); mutation replaces the
//                       product with the smallest distance contribution
//                       (or a random one) by a fresh random product.
//   * prioritize     -- SimilarityGreedy ordering: start from the product
//                       farthest from the rest, then repeatedly append the
//                       product maximising its minimum distance to the
//                       already-ordered ones.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <numeric>
#include <random>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

using Clock = std::chrono::steady_clock;

struct Cnf {
  int nvars = 0;
  std::vector<std::vector<int>> clauses;  // literals: +v / -v (1-based)
};

// ------------------------------------------------------------------ solver
class RandomSolver {
 public:
  RandomSolver(const Cnf& cnf, uint64_t seed) : n_(cnf.nvars), rng_(seed) {
    for (const auto& c : cnf.clauses) {
      if (c.empty()) throw std::runtime_error("empty clause: formula is unsatisfiable");
      if (c.size() == 1) {
        units_.push_back(c[0]);
        continue;
      }
      clauses_.push_back(c);
    }
    watches_.assign(2 * (n_ + 1), {});
    for (int ci = 0; ci < (int)clauses_.size(); ++ci) {
      watches_[idx(-clauses_[ci][0])].push_back(ci);
      watches_[idx(-clauses_[ci][1])].push_back(ci);
    }
    val_.assign(n_ + 1, 0);
    order_.resize(n_);
    std::iota(order_.begin(), order_.end(), 1);
  }

  // returns a full assignment (val[v] in {+1,-1}) or empty on failure
  std::vector<int8_t> sample(int max_conflicts = 20000, int restarts = 50) {
    for (int r = 0; r < restarts; ++r) {
      if (attempt(max_conflicts)) return val_;
    }
    return {};
  }

 private:
  static int idx(int lit) { return lit > 0 ? 2 * lit : 2 * (-lit) + 1; }
  int value(int lit) const {
    const int v = val_[std::abs(lit)];
    return lit > 0 ? v : -v;
  }

  bool assign(int lit) {
    const int v = std::abs(lit);
    const int8_t want = lit > 0 ? 1 : -1;
    if (val_[v] != 0) return val_[v] == want;
    val_[v] = want;
    trail_.push_back(lit);
    return true;
  }

  // propagate from qhead_; returns false on conflict
  bool propagate() {
    while (qhead_ < (int)trail_.size()) {
      const int lit = trail_[qhead_++];            // lit became true -> clauses watching -lit
      auto& ws = watches_[idx(lit)];
      for (size_t i = 0; i < ws.size();) {
        const int ci = ws[i];
        auto& c = clauses_[ci];
        // make c[1] the false watch
        if (c[0] == -lit) std::swap(c[0], c[1]);
        if (value(c[0]) == 1) { ++i; continue; }
        bool moved = false;
        for (size_t k = 2; k < c.size(); ++k) {
          if (value(c[k]) != -1) {
            std::swap(c[1], c[k]);
            watches_[idx(-c[1])].push_back(ci);
            ws[i] = ws.back();
            ws.pop_back();
            moved = true;
            break;
          }
        }
        if (moved) continue;
        if (value(c[0]) == -1) return false;       // conflict
        if (!assign(c[0])) return false;           // unit
        ++i;
      }
    }
    return true;
  }

  void undo_to(size_t level_start) {
    while (trail_.size() > level_start) {
      val_[std::abs(trail_.back())] = 0;
      trail_.pop_back();
    }
    qhead_ = (int)trail_.size();
  }

  bool attempt(int max_conflicts) {
    std::fill(val_.begin(), val_.end(), 0);
    trail_.clear();
    qhead_ = 0;
    for (int u : units_)
      if (!assign(u)) return false;
    if (!propagate()) return false;
    std::shuffle(order_.begin(), order_.end(), rng_);
    std::bernoulli_distribution coin(0.5);
    // decision stack: (trail size before decision, decided literal, flipped?)
    struct Dec { size_t start; int lit; bool flipped; };
    std::vector<Dec> stack;
    size_t next = 0;
    int conflicts = 0;
    while (true) {
      while (next < order_.size() && val_[order_[next]] != 0) ++next;
      if (next == order_.size()) return true;     // complete assignment
      const int v = order_[next];
      const int lit = coin(rng_) ? v : -v;
      stack.push_back({trail_.size(), lit, false});
      assign(lit);
      bool backtracked = false;
      while (!propagate()) {
        backtracked = true;
        if (++conflicts > max_conflicts) return false;
        // chronological backtracking: flip the most recent unflipped decision
        while (!stack.empty() && stack.back().flipped) {
          undo_to(stack.back().start);
          stack.pop_back();
        }
        if (stack.empty()) return false;
        Dec& d = stack.back();
        undo_to(d.start);
        d.flipped = true;
        d.lit = -d.lit;
        assign(d.lit);
      }
      if (backtracked) next = 0;  // positions before `next` may have been unassigned
    }
  }

  int n_;
  std::mt19937_64 rng_;
  std::vector<std::vector<int>> clauses_;
  std::vector<int> units_;
  std::vector<std::vector<int>> watches_;
  std::vector<int8_t> val_;
  std::vector<int> trail_;
  std::vector<int> order_;
  int qhead_ = 0;
};

// ------------------------------------------------------------------ bitsets
struct Product {
  std::vector<uint64_t> bits;
  int count = 0;
};

Product to_product(const std::vector<int8_t>& val, int n) {
  Product p;
  p.bits.assign((n + 64) / 64, 0);
  for (int v = 1; v <= n; ++v)
    if (val[v] > 0) {
      p.bits[v >> 6] |= (1ULL << (v & 63));
      ++p.count;
    }
  return p;
}

double jaccard(const Product& a, const Product& b) {
  int inter = 0, uni = 0;
  for (size_t i = 0; i < a.bits.size(); ++i) {
    inter += __builtin_popcountll(a.bits[i] & b.bits[i]);
    uni += __builtin_popcountll(a.bits[i] | b.bits[i]);
  }
  return uni == 0 ? 0.0 : 1.0 - (double)inter / (double)uni;
}

Cnf make_cnf(int nvars, const std::vector<std::vector<int>>& clauses) {
  Cnf c;
  c.nvars = nvars;
  c.clauses = clauses;
  for (const auto& cl : clauses)
    for (int l : cl)
      if (l == 0 || std::abs(l) > nvars) throw std::runtime_error("literal out of range");
  return c;
}

std::vector<int> signed_ids(const Product& p, int n) {
  std::vector<int> out;
  out.reserve(n);
  for (int v = 1; v <= n; ++v) out.push_back(((p.bits[v >> 6] >> (v & 63)) & 1ULL) ? v : -v);
  return out;
}

// ------------------------------------------------------------------ API
std::vector<std::vector<int>> random_products(int nvars, const std::vector<std::vector<int>>& clauses, int n,
                                              uint64_t seed) {
  Cnf cnf = make_cnf(nvars, clauses);
  RandomSolver s(cnf, seed);
  std::vector<std::vector<int>> out;
  for (int i = 0; i < n; ++i) {
    auto a = s.sample();
    if (a.empty()) throw std::runtime_error("no valid product found (formula unsatisfiable or too hard)");
    out.push_back(signed_ids(to_product(a, nvars), nvars));
  }
  return out;
}

double set_fitness(const std::vector<Product>& ps, std::vector<double>* contrib) {
  const int n = (int)ps.size();
  double total = 0.0;
  if (contrib) contrib->assign(n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const double d = jaccard(ps[i], ps[j]);
      total += d;
      if (contrib) { (*contrib)[i] += d; (*contrib)[j] += d; }
    }
  return total;
}

std::vector<int> prioritize_idx(const std::vector<Product>& ps) {
  const int n = (int)ps.size();
  std::vector<int> order;
  if (n == 0) return order;
  std::vector<double> contrib;
  set_fitness(ps, &contrib);
  std::vector<char> used(n, 0);
  int first = (int)(std::max_element(contrib.begin(), contrib.end()) - contrib.begin());
  order.push_back(first);
  used[first] = 1;
  std::vector<double> mind(n, 1e30);
  for (int k = 1; k < n; ++k) {
    const int last = order.back();
    int best = -1;
    double bestv = -1.0;
    for (int i = 0; i < n; ++i) {
      if (used[i]) continue;
      mind[i] = std::min(mind[i], jaccard(ps[i], ps[last]));
      if (mind[i] > bestv) { bestv = mind[i]; best = i; }
    }
    order.push_back(best);
    used[best] = 1;
  }
  return order;
}

py::dict sample_diverse(int nvars, const std::vector<std::vector<int>>& clauses, int n, double time_ms,
                        uint64_t seed, int max_iters, bool prioritize) {
  Cnf cnf = make_cnf(nvars, clauses);
  RandomSolver s(cnf, seed);
  std::mt19937_64 rng(seed ^ 0x9E3779B97F4A7C15ULL);
  const auto t0 = Clock::now();
  auto fresh = [&]() {
    auto a = s.sample();
    if (a.empty()) throw std::runtime_error("no valid product found (formula unsatisfiable or too hard)");
    return to_product(a, nvars);
  };
  std::vector<Product> cur;
  for (int i = 0; i < n; ++i) cur.push_back(fresh());
  std::vector<double> contrib;
  double fit = set_fitness(cur, &contrib);
  const double init_fit = fit;
  int iters = 0, accepted = 0;
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  {
    py::gil_scoped_release nogil;
    while (n > 1) {
      const double el = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
      if (el >= time_ms || (max_iters > 0 && iters >= max_iters)) break;
      ++iters;
      // mutate: replace the least-diverse product (p=0.7) or a random one
      int victim;
      if (u01(rng) < 0.7) victim = (int)(std::min_element(contrib.begin(), contrib.end()) - contrib.begin());
      else victim = (int)(rng() % (uint64_t)n);
      Product cand = fresh();
      // incremental fitness delta
      double old_c = 0.0, new_c = 0.0;
      for (int j = 0; j < n; ++j) {
        if (j == victim) continue;
        old_c += jaccard(cur[victim], cur[j]);
        new_c += jaccard(cand, cur[j]);
      }
      if (new_c >= old_c) {
        for (int j = 0; j < n; ++j) {
          if (j == victim) continue;
          const double dold = jaccard(cur[victim], cur[j]);
          const double dnew = jaccard(cand, cur[j]);
          contrib[j] += dnew - dold;
        }
        contrib[victim] = new_c;
        cur[victim] = std::move(cand);
        fit += new_c - old_c;
        ++accepted;
      }
    }
  }
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  if (prioritize) order = prioritize_idx(cur);
  std::vector<std::vector<int>> prods;
  for (int i : order) prods.push_back(signed_ids(cur[i], nvars));
  py::dict d;
  d["products"] = prods;
  d["fitness"] = fit;
  d["initial_fitness"] = init_fit;
  d["iterations"] = iters;
  d["accepted"] = accepted;
  d["elapsed_ms"] = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
  return d;
}

std::vector<std::vector<double>> jaccard_matrix(const std::vector<std::vector<int>>& prods, int nvars) {
  std::vector<Product> ps;
  for (const auto& pr : prods) {
    Product p;
    p.bits.assign((nvars + 64) / 64, 0);
    for (int l : pr)
      if (l > 0 && l <= nvars) { p.bits[l >> 6] |= (1ULL << (l & 63)); ++p.count; }
    ps.push_back(std::move(p));
  }
  std::vector<std::vector<double>> m(ps.size(), std::vector<double>(ps.size(), 0.0));
  for (size_t i = 0; i < ps.size(); ++i)
    for (size_t j = i + 1; j < ps.size(); ++j) m[i][j] = m[j][i] = jaccard(ps[i], ps[j]);
  return m;
}

bool check(int nvars, const std::vector<std::vector<int>>& clauses, const std::vector<int>& product) {
  std::vector<int8_t> val(nvars + 1, -1);
  for (int l : product)
    if (l > 0 && l <= nvars) val[l] = 1;
  for (const auto& c : clauses) {
    bool sat = false;
    for (int l : c) {
      const int v = val[std::abs(l)];
      if ((l > 0 && v > 0) || (l < 0 && v < 0)) { sat = true; break; }
    }
    if (!sat) return false;
  }
  return true;
}

}  // namespace

void register_sampler(py::module_& m) {
  m.def("random_products", &random_products, py::arg("nvars"), py::arg("clauses"), py::arg("n"),
        py::arg("seed") = 0, "n independent randomised-SAT valid products (signed id lists)");
  m.def("sample_diverse", &sample_diverse, py::arg("nvars"), py::arg("clauses"), py::arg("n"),
        py::arg("time_ms") = 1000.0, py::arg("seed") = 0, py::arg("max_iters") = 0, py::arg("prioritize") = true,
        "(1+1) EA maximising the sum of pairwise Jaccard distances of n products");
  m.def("jaccard_matrix", &jaccard_matrix, py::arg("products"), py::arg("nvars"));
  m.def("check", &check, py::arg("nvars"), py::arg("clauses"), py::arg("product"));
}
