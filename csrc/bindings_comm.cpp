// fedmi — Python bindings for the peer-to-peer (hipIpc / xGMI) collectives.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <string>

#include "comm/peer_comm.h"

namespace py = pybind11;
using fedmi::PeerComm;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

void fedmi_bind_comm(py::module_& m) {
  m.attr("PEER_MAX_RANKS") = fedmi::kPeerMaxRanks;
  m.attr("PEER_ONESHOT") = (int)fedmi::kPeerOneShot;
  m.attr("PEER_TWOSHOT") = (int)fedmi::kPeerTwoShot;
  py::class_<PeerComm>(m, "PeerComm")
      .def(py::init<int, int, long long>(), py::arg("rank"), py::arg("world"), py::arg("capacity_bytes"))
      .def("handle", [](const PeerComm& c) {
        auto h = c.handle();
        return py::bytes(reinterpret_cast<const char*>(h.data()), h.size());
      })
      .def("connect", [](PeerComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::vector<uint8_t>> v;
        for (const auto& b : hs) {
          std::string s = b;
          v.emplace_back(s.begin(), s.end());
        }
        c.connect(v);
      })
      .def("allreduce_f32", [](PeerComm& c, uintptr_t st, uintptr_t in, uintptr_t out, long long n, float scale,
                               int algo, int blocks) {
             c.allreduce_f32(S(st), reinterpret_cast<const float*>(in), reinterpret_cast<float*>(out), n, scale, algo,
                             blocks);
           }, py::arg("stream"), py::arg("src"), py::arg("dst"), py::arg("n"), py::arg("scale"), py::arg("algo") = 0,
           py::arg("blocks") = 0)
      .def("allreduce_int8_ef", [](PeerComm& c, uintptr_t st, uintptr_t x, uintptr_t g, uintptr_t r, long long n,
                                   float scale, int blocks) {
             c.allreduce_int8_ef(S(st), reinterpret_cast<float*>(x), reinterpret_cast<float*>(g),
                                 reinterpret_cast<float*>(r), n, scale, blocks);
           }, py::arg("stream"), py::arg("x"), py::arg("g"), py::arg("r"), py::arg("n"), py::arg("scale"),
           py::arg("blocks") = 0)
      .def("allreduce_i64_mean_floor", [](PeerComm& c, uintptr_t st, uintptr_t in, uintptr_t out, long long n) {
        c.allreduce_i64_mean_floor(S(st), reinterpret_cast<const int64_t*>(in), reinterpret_cast<int64_t*>(out), n);
      })
      .def("allgather", [](PeerComm& c, uintptr_t st, uintptr_t in, uintptr_t out, long long nbytes, int blocks) {
             c.allgather(S(st), reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out), nbytes, blocks);
           }, py::arg("stream"), py::arg("src"), py::arg("dst"), py::arg("nbytes"), py::arg("blocks") = 0)
      .def("error", &PeerComm::error)
      .def("epochs", &PeerComm::epochs)
      .def("clear_error", &PeerComm::clear_error)
      .def("request_abort", &PeerComm::request_abort)
      .def("abort_requested", &PeerComm::abort_requested)
      .def("set_timeout_ms", &PeerComm::set_timeout_ms)
      .def("disconnect", &PeerComm::disconnect, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("connected", &PeerComm::connected)
      .def_property_readonly("colocated", &PeerComm::colocated)
      .def_property_readonly("rank", &PeerComm::rank)
      .def_property_readonly("world", &PeerComm::world)
      .def_property_readonly("capacity", &PeerComm::capacity)
      .def_static("default_blocks", &PeerComm::default_blocks);
}
