// Native voxel data pipeline (host C++17): synthetic machining-feature parts,
// binvox I/O and bit-packing.
//
// FeatureNet-3D (the north-star workload) classifies 24 machining features
// in 64^3 occupancy grids of a stock block.  No dataset can be downloaded
// here, so the framework ships a procedural generator of the same task:
// a solid stock with ONE subtractive feature of random size / position /
// depth, in one of 6 orientations (the access face).  Classes follow the
// FeatureNet taxonomy:
//
//   0 O-ring               8 rect. blind slot      16 2-sides through step
//   1 through hole         9 triangular pocket     17 slanted through step
//   2 blind hole          10 rectangular pocket    18 chamfer
//   3 triangular passage  11 circular end pocket   19 round
//   4 rect. passage       12 triangular blind step 20 vertical circ.-end blind slot
//   5 circ. through slot  13 circular blind step   21 horizontal circ.-end blind slot
//   6 tri. through slot   14 rect. blind step      22 6-sides passage
//   7 rect. through slot  15 rect. through step    23 6-sides pocket
//
// Output is bit-packed (1 bit per voxel, x fastest) so a 64^3 sample is
// 32 KiB on the host / over PCIe; the GPU unpacks to bf16 (misc.hip,
// unpack_bits).  Generation is multi-threaded and deterministic per
// (seed, sample index).  binvox (RLE) read/write keeps the classic voxelised
// CAD file format usable.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int kNumClasses = 24;

struct Grid {
  int S;
  std::vector<uint8_t> v;  // S^3, index (z*S + y)*S + x
  explicit Grid(int s) : S(s), v((size_t)s * s * s, 1) {}
  uint8_t& at(int x, int y, int z) { return v[((size_t)z * S + y) * S + x]; }
};

// 2-D cross-section predicates in (u, v) plane coordinates relative to a centre
bool in_circle(double u, double v, double r) { return u * u + v * v <= r * r; }
bool in_rect(double u, double v, double a, double b) { return std::fabs(u) <= a && std::fabs(v) <= b; }
bool in_tri(double u, double v, double r) {  // equilateral, pointing +v
  const double h = r * 1.5;
  if (v < -r * 0.5 || v > r) return false;
  const double half = (r - v) / h * (r * std::sqrt(3.0));
  return std::fabs(u) <= half * 0.5 + 1e-9;
}
bool in_hex(double u, double v, double r) {
  u = std::fabs(u);
  v = std::fabs(v);
  return v <= r * std::sqrt(3.0) / 2 && u * std::sqrt(3.0) / 2 + v * 0.5 <= r * std::sqrt(3.0) / 2;
}

// Carve the feature with the access face at z = S-1 (top); depth measured down.
void carve(Grid& g, int cls, std::mt19937_64& rng) {
  const int S = g.S;
  auto U = [&](double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); };
  const double c = (S - 1) / 2.0;
  const double cu = c + U(-0.12, 0.12) * S, cv = c + U(-0.12, 0.12) * S;
  const double r = U(0.12, 0.25) * S;
  const double a = U(0.10, 0.22) * S, b = U(0.10, 0.30) * S;
  const double depth = U(0.25, 0.6) * S;          // blind features
  const double top = S - 1;
  auto sweep = [&](auto&& inside, double d) {       // extrude a section from the top face
    for (int z = 0; z < S; ++z) {
      if (top - z > d) continue;
      for (int y = 0; y < S; ++y)
        for (int x = 0; x < S; ++x)
          if (inside(x - cu, y - cv)) g.at(x, y, z) = 0;
    }
  };
  const double thru = S + 1.0;
  switch (cls) {
    case 0: {  // O-ring groove on the top face
      const double r2 = r * U(0.55, 0.8);
      sweep([&](double u, double v) { return in_circle(u, v, r) && !in_circle(u, v, r2); }, depth * 0.5);
      break;
    }
    case 1: sweep([&](double u, double v) { return in_circle(u, v, r * 0.8); }, thru); break;
    case 2: sweep([&](double u, double v) { return in_circle(u, v, r * 0.8); }, depth); break;
    case 3: sweep([&](double u, double v) { return in_tri(u, v, r); }, thru); break;
    case 4: sweep([&](double u, double v) { return in_rect(u, v, a, b); }, thru); break;
    case 5: {  // circular-ended through slot: rectangle + two half discs, through
      sweep([&](double u, double v) {
        return in_rect(u, v, a, r * 0.5) || in_circle(u - a, v, r * 0.5) || in_circle(u + a, v, r * 0.5);
      }, thru);
      break;
    }
    case 6:  // triangular through slot: V groove across the whole top face
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x) {
            const double dz = top - z;
            if (dz <= depth && std::fabs(x - cu) <= (depth - dz) * 0.6) g.at(x, y, z) = 0;
          }
      break;
    case 7:  // rectangular through slot across the top face
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && std::fabs(x - cu) <= a * 0.6) g.at(x, y, z) = 0;
      break;
    case 8:  // rectangular blind slot: open on one side face only
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && std::fabs(x - cu) <= a * 0.6 && y <= cv + b) g.at(x, y, z) = 0;
      break;
    case 9: sweep([&](double u, double v) { return in_tri(u, v, r); }, depth); break;
    case 10: sweep([&](double u, double v) { return in_rect(u, v, a, b); }, depth); break;
    case 11:
      sweep([&](double u, double v) {
        return in_rect(u, v, a, r * 0.5) || in_circle(u - a, v, r * 0.5) || in_circle(u + a, v, r * 0.5);
      }, depth);
      break;
    case 12:  // triangular blind step (corner)
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && x + y <= 2.2 * r) g.at(x, y, z) = 0;
      break;
    case 13:  // circular blind step at a corner
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && in_circle(x, y, 2.0 * r)) g.at(x, y, z) = 0;
      break;
    case 14:  // rectangular blind step at a corner
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && x <= 2 * a && y <= 2 * b) g.at(x, y, z) = 0;
      break;
    case 15:  // rectangular through step along one edge
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && x <= 2 * a) g.at(x, y, z) = 0;
      break;
    case 16:  // 2-sides through step (two opposite edges)
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && (x <= a || x >= S - 1 - a)) g.at(x, y, z) = 0;
      break;
    case 17:  // slanted through step
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if ((top - z) <= depth && x <= 2 * a * (1.0 - (top - z) / depth) + a * 0.5) g.at(x, y, z) = 0;
      break;
    case 18: {  // chamfer on a top edge (45 degree)
      const double w = U(0.15, 0.35) * S;
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (x + (top - z) < w) g.at(x, y, z) = 0;
      break;
    }
    case 19: {  // round (convex fillet) on a top edge
      const double w = U(0.15, 0.35) * S;
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x) {
            const double dx = w - x, dz = w - (top - z);
            if (x < w && (top - z) < w && dx * dx + dz * dz > w * w) g.at(x, y, z) = 0;
          }
      break;
    }
    case 20:  // vertical circular end blind slot: slot from a side face ending in a half disc
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x)
            if (top - z <= depth && ((std::fabs(x - cu) <= r * 0.5 && y <= cv) || in_circle(x - cu, y - cv, r * 0.5)))
              g.at(x, y, z) = 0;
      break;
    case 21:  // horizontal circular end blind slot (semicircular floor)
      for (int z = 0; z < S; ++z)
        for (int y = 0; y < S; ++y)
          for (int x = 0; x < S; ++x) {
            const double dz = top - z;
            if (y <= cv + b && ((dz <= depth - r * 0.5 && std::fabs(x - cu) <= r * 0.5) ||
                                in_circle(x - cu, dz - (depth - r * 0.5), r * 0.5)))
              g.at(x, y, z) = 0;
          }
      break;
    case 22: sweep([&](double u, double v) { return in_hex(u, v, r); }, thru); break;
    case 23: sweep([&](double u, double v) { return in_hex(u, v, r); }, depth); break;
    default: throw std::runtime_error("bad class");
  }
}

// rotate so the access face becomes one of the 6 faces (axis permutation + flip)
void orient(const Grid& src, Grid& dst, int o) {
  const int S = src.S;
  for (int z = 0; z < S; ++z)
    for (int y = 0; y < S; ++y)
      for (int x = 0; x < S; ++x) {
        int X = x, Y = y, Z = z;
        switch (o) {
          case 0: break;                                  // +z
          case 1: Z = S - 1 - z; Y = S - 1 - y; break;    // -z
          case 2: X = z; Z = S - 1 - x; break;            // +x
          case 3: X = S - 1 - z; Z = x; break;            // -x
          case 4: Y = z; Z = S - 1 - y; break;            // +y
          default: Y = S - 1 - z; Z = y; break;           // -y
        }
        dst.v[((size_t)Z * S + Y) * S + X] = src.v[((size_t)z * S + y) * S + x];
      }
}

void gen_one(int S, int cls, uint64_t seed, uint8_t* packed, bool random_orient) {
  std::mt19937_64 rng(seed);
  Grid g(S), o(S);
  carve(g, cls, rng);
  const int ori = random_orient ? (int)(rng() % 6) : 0;
  orient(g, o, ori);
  const size_t n = (size_t)S * S * S;
  std::memset(packed, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i)
    if (o.v[i]) packed[i >> 3] |= (uint8_t)(1u << (i & 7));
}

py::tuple generate(int n, int size, uint64_t seed, int num_classes, bool random_orient, int threads,
                   py::object labels_in) {
  if (size < 8) throw std::runtime_error("voxel grid too small");
  if (num_classes < 1 || num_classes > kNumClasses) throw std::runtime_error("num_classes must be in [1, 24]");
  const size_t per = ((size_t)size * size * size + 7) / 8;
  py::array_t<uint8_t> bits({(py::ssize_t)n, (py::ssize_t)per});
  py::array_t<int64_t> labels(n);
  auto L = labels.mutable_unchecked<1>();
  if (!labels_in.is_none()) {
    auto li = labels_in.cast<py::array_t<int64_t>>();
    auto r = li.unchecked<1>();
    if (r.shape(0) != n) throw std::runtime_error("labels length mismatch");
    for (int i = 0; i < n; ++i) L(i) = r(i);
  } else {
    std::mt19937_64 lr(seed * 7919 + 17);
    for (int i = 0; i < n; ++i) L(i) = (int64_t)(lr() % (uint64_t)num_classes);
  }
  uint8_t* out = bits.mutable_data();
  std::vector<int64_t> lab(n);
  for (int i = 0; i < n; ++i) lab[i] = L(i);
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = std::min(threads, std::max(1, n));
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&, t]() {
        for (int i = t; i < n; i += threads)
          gen_one(size, (int)lab[i], seed * 1000003ULL + (uint64_t)i * 2654435761ULL + 1, out + (size_t)i * per,
                  random_orient);
      });
    for (auto& th : pool) th.join();
  }
  return py::make_tuple(bits, labels);
}

py::array_t<uint8_t> pack_bits(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> dense) {
  const size_t n = (size_t)dense.size();
  py::array_t<uint8_t> out((py::ssize_t)((n + 7) / 8));
  const uint8_t* d = dense.data();
  uint8_t* o = out.mutable_data();
  std::memset(o, 0, (n + 7) / 8);
  for (size_t i = 0; i < n; ++i)
    if (d[i]) o[i >> 3] |= (uint8_t)(1u << (i & 7));
  return out;
}

py::array_t<uint8_t> unpack_bits(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> packed, size_t n) {
  py::array_t<uint8_t> out((py::ssize_t)n);
  const uint8_t* p = packed.data();
  uint8_t* o = out.mutable_data();
  for (size_t i = 0; i < n; ++i) o[i] = (p[i >> 3] >> (i & 7)) & 1u;
  return out;
}

// binvox: "#binvox 1\ndim D D D\ntranslate tx ty tz\nscale s\ndata\n" + RLE (value, count) bytes,
// voxel order x-major in the file (index = x*W*H + z*W + y); we convert to our (z, y, x) layout.
py::tuple read_binvox(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string line;
  std::getline(f, line);
  if (line.rfind("#binvox", 0) != 0) throw std::runtime_error("not a binvox file");
  int d = 0, h = 0, w = 0;
  double tx = 0, ty = 0, tz = 0, sc = 1;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string key;
    is >> key;
    if (key == "dim") is >> d >> h >> w;
    else if (key == "translate") is >> tx >> ty >> tz;
    else if (key == "scale") is >> sc;
    else if (key == "data") break;
  }
  if (d <= 0 || d != h || h != w) throw std::runtime_error("binvox: only cubic grids supported");
  const size_t n = (size_t)d * h * w;
  std::vector<uint8_t> raw;
  raw.reserve(n);
  uint8_t pair[2];
  while (raw.size() < n && f.read(reinterpret_cast<char*>(pair), 2)) raw.insert(raw.end(), pair[1], pair[0] ? 1 : 0);
  if (raw.size() < n) throw std::runtime_error("binvox: truncated data");
  const int S = d;
  py::array_t<uint8_t> out({S, S, S});
  auto o = out.mutable_unchecked<3>();
  for (int x = 0; x < S; ++x)
    for (int z = 0; z < S; ++z)
      for (int y = 0; y < S; ++y) o(z, y, x) = raw[((size_t)x * S + z) * S + y];
  return py::make_tuple(out, py::make_tuple(tx, ty, tz), sc);
}

void write_binvox(const std::string& path, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> grid,
                  std::vector<double> translate, double scale) {
  if (grid.ndim() != 3 || grid.shape(0) != grid.shape(1) || grid.shape(1) != grid.shape(2))
    throw std::runtime_error("write_binvox: need a cubic [S,S,S] grid");
  const int S = (int)grid.shape(0);
  auto g = grid.unchecked<3>();
  std::ofstream f(path, std::ios::binary);
  f << "#binvox 1\ndim " << S << " " << S << " " << S << "\n";
  if (translate.size() != 3) translate = {0, 0, 0};
  f << "translate " << translate[0] << " " << translate[1] << " " << translate[2] << "\nscale " << scale
    << "\ndata\n";
  uint8_t cur = 2;
  int run = 0;
  auto flush = [&]() {
    if (run > 0) {
      const uint8_t b[2] = {cur, (uint8_t)run};
      f.write(reinterpret_cast<const char*>(b), 2);
    }
  };
  for (int x = 0; x < S; ++x)
    for (int z = 0; z < S; ++z)
      for (int y = 0; y < S; ++y) {
        const uint8_t v = g(z, y, x) ? 1 : 0;
        if (v == cur && run < 255) ++run;
        else { flush(); cur = v; run = 1; }
      }
  flush();
}

}  // namespace

void register_voxel(py::module_& m) {
  m.attr("NUM_FEATURE_CLASSES") = kNumClasses;
  m.def("generate_voxels", &generate, py::arg("n"), py::arg("size") = 64, py::arg("seed") = 0,
        py::arg("num_classes") = 24, py::arg("random_orient") = true, py::arg("threads") = 0,
        py::arg("labels") = py::none(),
        "n synthetic machining-feature parts -> (bit-packed uint8 [n, S^3/8], int64 labels [n])");
  m.def("pack_bits", &pack_bits);
  m.def("unpack_bits", &unpack_bits, py::arg("packed"), py::arg("n"));
  m.def("read_binvox", &read_binvox);
  m.def("write_binvox", &write_binvox, py::arg("path"), py::arg("grid"),
        py::arg("translate") = std::vector<double>{0, 0, 0}, py::arg("scale") = 1.0);
}
