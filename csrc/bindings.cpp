// fedmi — Python bindings for the native runtime and HIP kernels.
//
// Device memory is owned by PyTorch tensors (caching allocator); the native
// side receives raw device pointers and the torch stream handle, so every
// launch is ordered on torch's current stream and can be graph-captured.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>

#include "kernels/common.h"
#include "kernels/lenet_layout.h"
#include "runtime/lenet_engine.h"

namespace py = pybind11;

namespace fedmi {
void launch_lenet_conv_fwd(hipStream_t, const uint8_t*, int, int, const bf16*, const float*, uint32_t, const int*, int,
                           bf16*, bf16*, int, bf16*, uint8_t*, uint8_t*, lenet::Stats*);
void launch_lenet_fc_eval(hipStream_t, const bf16*, const int*, int, const bf16*, const float*, float*, long,
                          lenet::Stats*);
bool stamps_enabled();
void read_stamps(unsigned long long*, bool);
void set_ks1_diag(int);
void launch_lenet_pack(hipStream_t, const float*, bf16*);
void launch_sgd_flat(hipStream_t, float*, const float*, float*, long, float, float, float, float, int, int);
void launch_ef_delta(hipStream_t, const float*, const float*, const float*, float*, long);
size_t topk_state_bytes();
size_t topk_overflow_offset();
void launch_topk_ef(hipStream_t, const float*, const float*, float*, long, int, void*, int*, unsigned*, int*, float*);
void launch_scatter_add_ranked(hipStream_t, float*, const int*, const float*, int, long, float, long);
void launch_quant_int8(hipStream_t, const float*, long, signed char*, float*, float*);
void launch_dequant_accum(hipStream_t, const signed char*, const float*, int, long, float*, float);
}  // namespace fedmi

using namespace fedmi;

void fedmi_bind_cnn(py::module_& m);   // bindings_cnn.cpp
void fedmi_bind_comm(py::module_& m);  // bindings_comm.cpp
void fedmi_bind_zoo(py::module_& m);   // bindings_zoo.cpp
void fedmi_bind_io(py::module_& m);    // bindings_io.cpp

template <typename T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void check_last(const char* what) { check_hip(hipGetLastError(), what); }

static LeNetBuffers buffers_from(const py::dict& d) {
  auto get = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
  LeNetBuffers b;
  b.train_images = P<const uint8_t>(get("train_images"));
  b.train_labels = P<const int>(get("train_labels"));
  b.n_train = d.contains("n_train") ? d["n_train"].cast<int>() : 0;
  b.params = P<float>(get("params"));
  b.mom = P<float>(get("mom"));
  b.pk = P<bf16>(get("pk"));
  b.act2 = P<bf16>(get("act2"));
  b.act2_rows = d.contains("act2_rows") ? d["act2_rows"].cast<int>() : 0;
  b.act2T = P<bf16>(get("act2T"));
  b.h1 = P<bf16>(get("h1"));
  b.dact2 = P<float>(get("dact2"));
  b.dZ1T = P<bf16>(get("dZ1T"));
  b.conv_slab = P<float>(get("conv_slab"));
  b.eval_part = P<float>(get("eval_part"));
  b.eval_part_floats = d.contains("eval_part_floats") ? d["eval_part_floats"].cast<long>() : 0;
  b.train_stats = P<lenet::Stats>(get("train_stats"));
  b.eval_stats = P<lenet::Stats>(get("eval_stats"));
  b.round_ctr = P<int>(get("round_ctr"));
  return b;
}

static void fedmi_bind(py::module_& m) {
  fedmi_bind_cnn(m);
  fedmi_bind_comm(m);
  fedmi_bind_zoo(m);
  fedmi_bind_io(m);
  m.def("stamps_enabled", &stamps_enabled);
  m.def("set_ks1_diag", &set_ks1_diag);
  m.def("read_stamps", [](bool clear) {
    const size_t n = (size_t)FEDMI_STAMP_KERNELS * FEDMI_STAMP_WGS * FEDMI_STAMP_SLOTS;
    std::vector<unsigned long long> buf(n, 0ull);
    read_stamps(buf.data(), clear);
    return py::bytes(reinterpret_cast<const char*>(buf.data()), n * sizeof(unsigned long long));
  }, py::arg("clear") = true);
  m.attr("STAMP_SHAPE") = py::make_tuple(FEDMI_STAMP_KERNELS, FEDMI_STAMP_WGS, FEDMI_STAMP_SLOTS);
  m.doc() = "fedmi native runtime: fused LeNet HIP kernels, graph executor, flat-buffer and compression kernels (gfx950)";

  m.def("lenet_layout", []() {
    using namespace lenet;
    py::dict d;
    d["P_C1W"] = P_C1W; d["P_C1B"] = P_C1B; d["P_C2W"] = P_C2W; d["P_C2B"] = P_C2B;
    d["P_F1W"] = P_F1W; d["P_F1B"] = P_F1B; d["P_F2W"] = P_F2W; d["P_F2B"] = P_F2B;
    d["P_F3W"] = P_F3W; d["P_F3B"] = P_F3B; d["P_TOTAL"] = P_TOTAL;
    d["CS"] = CS; d["FS"] = FS; d["F1W_N"] = F1W_N; d["DZ1_LD"] = DZ1_LD; d["PK_TOTAL"] = PK_TOTAL; d["F0"] = F0; d["F0P"] = F0P; d["NP1"] = NP1;
    d["MAX_TRAIN_BATCH"] = MAX_TRAIN_BATCH; d["FC_SPW"] = FC_SPW;
    d["IMG_BYTES"] = IMG_BYTES; d["STATS_BYTES"] = (int)sizeof(Stats);
    return d;
  });

  py::class_<SgdConfig>(m, "SgdConfig")
      .def(py::init<>())
      .def_readwrite("lr", &SgdConfig::lr)
      .def_readwrite("momentum", &SgdConfig::momentum)
      .def_readwrite("weight_decay", &SgdConfig::weight_decay);

  py::class_<LeNetEngine>(m, "LeNetEngine")
      .def(py::init([](const py::dict& bufs, float lr, float momentum, float wd, uint32_t seed, bool augment) {
             SgdConfig c;
             c.lr = lr; c.momentum = momentum; c.weight_decay = wd;
             return new LeNetEngine(buffers_from(bufs), c, seed, augment);
           }),
           py::arg("buffers"), py::arg("lr"), py::arg("momentum"), py::arg("weight_decay"), py::arg("seed"),
           py::arg("augment"))
      .def("set_schedule", &LeNetEngine::set_schedule)
      .def("schedule_len", &LeNetEngine::schedule_len)
      .def("step", [](LeNetEngine& e, uintptr_t st, int start, int nb, bool bump, bool reset) {
             e.step(S(st), start, nb, bump, reset);
           }, py::arg("stream"), py::arg("start"), py::arg("nb"), py::arg("bump_round") = false,
           py::arg("reset_stats") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("run_epoch", [](LeNetEngine& e, uintptr_t st, bool use_graph) { e.run_epoch(S(st), use_graph); },
           py::call_guard<py::gil_scoped_release>())
      .def("eval", [](LeNetEngine& e, uintptr_t st, uintptr_t images, uintptr_t labels, int n) {
             e.eval(S(st), P<const uint8_t>(images), P<const int>(labels), n);
           }, py::arg("st"), py::arg("images"), py::arg("labels"), py::arg("n"), py::call_guard<py::gil_scoped_release>())
      .def("pack", [](LeNetEngine& e, uintptr_t st) { e.pack(S(st)); }, py::call_guard<py::gil_scoped_release>())
      .def("set_sgd", [](LeNetEngine& e, float lr, float m, float wd) {
             SgdConfig c; c.lr = lr; c.momentum = m; c.weight_decay = wd; e.set_sgd(c);
           })
      .def("graph_ready", &LeNetEngine::graph_ready);

  // ---- raw LeNet kernels (numerics tests drive them one by one) -------------
  m.def("lenet_conv_fwd", [](uintptr_t st, uintptr_t images, int base, int nb, uintptr_t pk, uintptr_t params,
                             uint32_t seed, uintptr_t round_ctr, int augment, uintptr_t act2, uintptr_t act2T,
                             int tstride, uintptr_t pool1, uintptr_t am1, uintptr_t am2, uintptr_t zero_stats) {
    launch_lenet_conv_fwd(S(st), P<const uint8_t>(images), base, nb, P<const bf16>(pk), P<const float>(params), seed,
                          P<const int>(round_ctr), augment, P<bf16>(act2), P<bf16>(act2T), tstride, P<bf16>(pool1),
                          P<uint8_t>(am1), P<uint8_t>(am2), P<lenet::Stats>(zero_stats));
    check_last("lenet_conv_fwd");
  });
  m.def("lenet_pack", [](uintptr_t st, uintptr_t params, uintptr_t pk) {
    launch_lenet_pack(S(st), P<const float>(params), P<bf16>(pk));
    check_last("lenet_pack");
  });

  // ---- flat-buffer ops --------------------------------------------------------
  m.def("sgd_flat", [](uintptr_t st, uintptr_t p, uintptr_t g, uintptr_t buf, long n, float lr, float mo, float wd,
                       float damp, bool nesterov, bool first) {
    launch_sgd_flat(S(st), P<float>(p), P<const float>(g), P<float>(buf), n, lr, mo, wd, damp, nesterov ? 1 : 0,
                    first ? 1 : 0);
    check_last("sgd_flat");
  });

  // ---- compression ---------------------------------------------------------------
  m.def("topk_state_bytes", &topk_state_bytes);
  m.def("topk_overflow_offset", &topk_overflow_offset);
  m.def("topk_ef", [](uintptr_t st, uintptr_t x, uintptr_t g, uintptr_t residual, long n, int k, uintptr_t state,
                      uintptr_t cidx, uintptr_t ckey, uintptr_t idx, uintptr_t val) {
    if (k <= 0 || k > n) throw std::invalid_argument("topk_ef: need 0 < k <= n");
    if (n >= (1L << 30)) throw std::invalid_argument("topk_ef: n must be < 2^30 (int32 indices, 2n scratch)");
    launch_topk_ef(S(st), P<const float>(x), P<const float>(g), P<float>(residual), n, k, P<void>(state), P<int>(cidx),
                   P<unsigned>(ckey), P<int>(idx), P<float>(val));
    check_last("topk_ef");
  }, py::arg("stream"), py::arg("x"), py::arg("g"), py::arg("residual"), py::arg("n"), py::arg("k"), py::arg("state"),
     py::arg("cidx"), py::arg("ckey"), py::arg("idx"), py::arg("val"));
  m.def("ef_delta", [](uintptr_t st, uintptr_t local, uintptr_t global, uintptr_t residual, uintptr_t d, long n) {
    launch_ef_delta(S(st), P<const float>(local), P<const float>(global), P<const float>(residual), P<float>(d), n);
    check_last("ef_delta");
  });
  m.def("scatter_add_ranked", [](uintptr_t st, uintptr_t out, uintptr_t idx, uintptr_t val, int R, long m_, float scale,
                                 long n) {
    if (R <= 0) throw std::invalid_argument("scatter_add_ranked: R must be > 0");
    launch_scatter_add_ranked(S(st), P<float>(out), P<const int>(idx), P<const float>(val), R, m_, scale, n);
    check_last("scatter_add_ranked");
  });
  m.def("quant_int8", [](uintptr_t st, uintptr_t d, long n, uintptr_t q, uintptr_t scales, uintptr_t residual) {
    launch_quant_int8(S(st), P<const float>(d), n, P<signed char>(q), P<float>(scales), P<float>(residual));
    check_last("quant_int8");
  });
  m.def("dequant_accum", [](uintptr_t st, uintptr_t q, uintptr_t scales, int R, long n, uintptr_t out, float scale) {
    launch_dequant_accum(S(st), P<const signed char>(q), P<const float>(scales), R, n, P<float>(out), scale);
    check_last("dequant_accum");
  });
}

// the module name carries the build variant (fedmi/_build.py VARIANTS): -DFEDMI_MODULE=_fedmi_native_<v>
#ifndef FEDMI_MODULE
#define FEDMI_MODULE _fedmi_native
#endif
PYBIND11_MODULE(FEDMI_MODULE, m) { fedmi_bind(m); }
