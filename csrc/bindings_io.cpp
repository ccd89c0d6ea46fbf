// fedmi — Python bindings for the native checkpoint writer (csrc/runtime/ckpt_writer.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <string>
#include <tuple>

#include "runtime/ckpt_writer.h"

namespace py = pybind11;
using fedmi::CkptRecord;
using fedmi::CkptSegment;
using fedmi::CkptWriter;

void fedmi_bind_io(py::module_& m) {
  py::class_<CkptWriter>(m, "CkptWriter")
      .def(py::init([](py::bytes tmpl, const std::vector<std::tuple<uintptr_t, long long, long long>>& segs,
                       const std::vector<std::tuple<long long, long long, long long, std::vector<long long>>>& recs,
                       long long epoch_at, const std::vector<std::string>& paths, bool device, int slots,
                       bool coalesce, bool link) {
             std::string t = tmpl;
             std::vector<CkptSegment> s;
             for (const auto& x : segs) s.push_back({std::get<0>(x), std::get<1>(x), std::get<2>(x)});
             std::vector<CkptRecord> r;
             for (const auto& x : recs) r.push_back({std::get<0>(x), std::get<1>(x), std::get<2>(x), std::get<3>(x)});
             return new CkptWriter(std::vector<uint8_t>(t.begin(), t.end()), std::move(s), std::move(r), epoch_at,
                                   paths, device, slots, coalesce, link);
           }),
           py::arg("template"), py::arg("segments"), py::arg("records"), py::arg("epoch_at"), py::arg("paths"),
           py::arg("device"), py::arg("slots") = 4, py::arg("coalesce") = false,
           py::arg("link") = false)
      .def("submit", [](CkptWriter& w, uintptr_t st, int32_t epoch) {
             w.submit(reinterpret_cast<hipStream_t>(st), epoch);
           }, py::arg("stream"), py::arg("epoch"), py::call_guard<py::gil_scoped_release>())
      .def("flush", &CkptWriter::flush, py::call_guard<py::gil_scoped_release>())
      .def("last_file", [](const CkptWriter& w) {
        auto v = w.last_file();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def_property_readonly("written", &CkptWriter::written)
      .def_property_readonly("coalesced", &CkptWriter::coalesced)
      .def_property_readonly("submitted", &CkptWriter::submitted);
}
