// pybind11 module `_rt`: the host-side native runtime of featurenet_amd.
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_sampler(py::module_& m);
void register_voxel(py::module_& m);
void register_weibull(py::module_& m);

PYBIND11_MODULE(_rt, m) {
  m.doc() = "featurenet_amd native host runtime (sampler, voxel pipeline, CLEVER Weibull fits)";
  register_sampler(m);
  register_voxel(m);
  register_weibull(m);
}
