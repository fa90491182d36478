// pybind11 bindings of the amd-smi collector (module yoda_scheduler_amd._native._yoda_sniffer).
#include <pybind11/pybind11.h>

#include "build_id.h"
#include <pybind11/stl.h>

#include "collector.hpp"

namespace py = pybind11;
using namespace yoda;

PYBIND11_MODULE(_yoda_sniffer, m) {
  m.def("build_id", [] { return std::string(YODA_BUILD_ID); }, "hash of the sources this module was built from");
  m.doc() = "amd-smi telemetry collector (C++)";
  py::class_<Collector>(m, "Collector")
      .def(py::init<>())
      .def("init",
           [](Collector& c) {
             std::string err;
             bool ok = c.init(&err);
             return py::make_tuple(ok, err);
           })
      .def_property_readonly("count", &Collector::count)
      .def("sample_json", [](Collector& c) { return to_json(c.sample()); })
      .def("shutdown", &Collector::shutdown);
}
