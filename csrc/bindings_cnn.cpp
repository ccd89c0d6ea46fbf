// fedmi — Python bindings for the CNN-zoo kernels (implicit-GEMM conv, BN,
// classifier head, input prep).  Raw device pointers + torch stream handle,
// like the rest of the extension; every call is graph-capturable.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "kernels/common.h"
#include "kernels/wgrad_reduce.h"

namespace py = pybind11;

namespace fedmi {
struct ConvShape {
  int N, H, W, C, Cw, O, P, Q, R, S, st, pad;
};
void launch_conv_fwd(hipStream_t, const ConvShape&, const bf16*, const bf16*, bf16*, double*, const float*, float*, long,
                     const bf16*);
void launch_conv_dgrad(hipStream_t, const ConvShape&, const bf16*, const bf16*, bf16*, float*, long, const bf16*, int,
                       const bf16*, const BnSums*);
int conv_dgrad_fusable(const ConvShape&, int);
struct DPackItem {
  const float* w;
  bf16* wd;
  int O, Cw, C, R, S, st, pad;
};
void launch_dgrad_pack_multi(hipStream_t, const DPackItem*, int);
long conv_fd_ws_floats(const ConvShape&);
struct PackItem {
  const float* w;
  bf16* wr;
  int O, Cw, C, RS;
  int O8;
  int G;
};
void launch_conv_pack_multi(hipStream_t, const PackItem*, int);
void launch_conv_wgrad(hipStream_t, const ConvShape&, const bf16*, const bf16*, float*, float*, long, int, int, int, int,
                       WredItem*, int);
long conv_wgrad_ws_floats(const ConvShape&);
void launch_conv_pack(hipStream_t, const float*, bf16*, int, int, int, int, int, int);
struct SgdPackConv {
  long off;
  bf16* wr;
  bf16* wd;
  int O, Cw, C, R, S, st, pad;
};
struct SgdPackPlan {
  std::vector<char> table;
  int n_entries, n_blocks, lds_bytes;
};
SgdPackPlan build_sgd_pack_plan(const SgdPackConv*, int, const long*, int);
void launch_sgd_pack(hipStream_t, const void*, int, int, int, float*, const float*, float*, float, float, float, float,
                     int, int);

struct BNDesc {
  const double* stats; const float* gamma; const float* beta; float* rmean; float* rvar; long long* nbt;
  float* smean; float* sinv; const float* shift; const float* cbias;
};
void launch_maxpool2(hipStream_t, const bf16*, bf16*, int, int, int, int);
void launch_maxpool3(hipStream_t, const bf16*, bf16*, uint8_t*, int, int, int, int, int);
void launch_maxpool3_bwd(hipStream_t, const bf16*, const uint8_t*, bf16*, int, int, int, int, int, int);
void launch_maxpool2_bwd(hipStream_t, const bf16*, const bf16*, bf16*, int, int, int, int);
struct BNBwdDesc {
  const bf16* dya; const bf16* dyb; const bf16* y;
  const bf16* za; const float* meanA; const float* invA; const float* gammaA; float* dgammaA; float* dbetaA; bf16* dza;
  const bf16* zb; const float* meanB; const float* invB; const float* gammaB; float* dgammaB; float* dbetaB; bf16* dzb;
  bf16* gout;
  float* shiftA; float* shiftB;
  const bf16* dadd;
  const float* msc;
};
struct DwShape {
  int N, H, W, C, R, S, st, pad;
};
void launch_dw_fwd(hipStream_t, const DwShape&, const bf16*, const float*, bf16*, double*, const float*);
void launch_dw_dgrad(hipStream_t, const DwShape&, const bf16*, const float*, bf16*, const BnSums*);
long dw_wgrad_ws_floats(const DwShape&);
void launch_dw_wgrad(hipStream_t, const DwShape&, const bf16*, const bf16*, float*, float*, long, int, WredItem*);
void launch_prep_input(hipStream_t, const uint8_t*, int, const int*, int, int, uint32_t, const int*, bf16*);
void launch_sched_next(hipStream_t, const int*, int*, int*, double*, long);
void launch_bn_apply(hipStream_t, const bf16*, const BNDesc&, const bf16*, const BNDesc*, const bf16*, bf16*, int, int,
                     float, float, int, int, int, float*);
void launch_bn_bwd(hipStream_t, const BNBwdDesc&, double*, int, int, double*, long, int, int, int, int);
long bn_bwd_ws_floats(int, int);
int bn_bwd_chain_reps(int);
void launch_head(hipStream_t, const bf16*, const int*, int, const int*, int, int, int, int, const float*,
                 const float*, float*, float*, bf16*, float*, float*, float*, float*, int, float*, long);
}  // namespace fedmi

using namespace fedmi;

namespace {
template <typename T>
T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

void check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

ConvShape shape_from(const py::tuple& t) {
  if (t.size() != 12) throw std::invalid_argument("conv shape: (N,H,W,C,Cw,O,P,Q,R,S,stride,pad)");
  ConvShape s;
  int* f = &s.N;
  for (int i = 0; i < 12; ++i) f[i] = t[i].cast<int>();
  return s;
}

uintptr_t dget(const py::dict& d, const char* k) {
  return d.contains(k) && !d[k].is_none() ? d[k].cast<uintptr_t>() : 0;
}

DwShape dw_from(const py::tuple& t) {
  if (t.size() != 8) throw std::invalid_argument("dwconv shape: (N,H,W,C,R,S,stride,pad)");
  DwShape s;
  int* f = &s.N;
  for (int i = 0; i < 8; ++i) f[i] = t[i].cast<int>();
  return s;
}

// deferred WGRAD reduction <-> (ws, dw, kind, splits, O, C, Cw, RS, accumulate, Ow, G)
py::object wred_tuple(const WredItem& e) {
  return py::make_tuple(reinterpret_cast<uintptr_t>(e.ws), reinterpret_cast<uintptr_t>(e.dw), e.kind, e.splits, e.O,
                        e.C, e.Cw, e.RS, e.accumulate, e.Ow, e.G);
}

WredItem wred_from(const py::tuple& t) {
  if (t.size() != 11) throw std::invalid_argument("wgrad reduce item: (ws, dw, kind, splits, O, C, Cw, RS, acc, Ow, G)");
  WredItem e{};
  e.ws = P<const float>(t[0].cast<uintptr_t>());
  e.dw = P<float>(t[1].cast<uintptr_t>());
  e.kind = t[2].cast<int>();
  if (e.kind < WRED_TILE || e.kind > WRED_DW || !e.ws || !e.dw) throw std::invalid_argument("wgrad reduce item: bad kind / pointers");
  e.splits = t[3].cast<int>(); e.O = t[4].cast<int>(); e.C = t[5].cast<int>(); e.Cw = t[6].cast<int>();
  e.RS = t[7].cast<int>(); e.accumulate = t[8].cast<int>(); e.Ow = t[9].cast<int>(); e.G = t[10].cast<int>();
  return e;
}

BnSums bnsums_from(const py::dict& d) {
  return BnSums{P<double>(dget(d, "rep")), P<const bf16>(dget(d, "z")), P<const bf16>(dget(d, "y")),
                P<const float>(dget(d, "mean")), P<const float>(dget(d, "inv")), d["reps"].cast<int>(),
                P<const bf16>(dget(d, "zb")), P<const float>(dget(d, "meanb")), P<const float>(dget(d, "invb")),
                P<const float>(dget(d, "msc")), d.contains("msc_ld") ? d["msc_ld"].cast<int>() : 0};
}

BNDesc bn_from(const py::dict& d) {
  return BNDesc{P<const double>(dget(d, "stats")), P<const float>(dget(d, "gamma")), P<const float>(dget(d, "beta")),
                P<float>(dget(d, "rmean")),       P<float>(dget(d, "rvar")),        P<long long>(dget(d, "nbt")),
                P<float>(dget(d, "smean")),       P<float>(dget(d, "sinv")),        P<const float>(dget(d, "shift")),
                P<const float>(dget(d, "cbias"))};
}
}  // namespace

void read_conv_stamps(unsigned long long* host, bool clear);

void fedmi_bind_cnn(py::module_& m) {
  m.def("read_conv_stamps", [](bool clear) {
    const size_t n = (size_t)FEDMI_STAMP_WGS * FEDMI_STAMP_SLOTS;
    std::vector<unsigned long long> buf(n, 0ull);
    read_conv_stamps(buf.data(), clear);
    return py::bytes(reinterpret_cast<const char*>(buf.data()), n * sizeof(unsigned long long));
  }, py::arg("clear") = true);
  m.attr("STAT_REP") = STAT_REP;
  m.def("conv_fwd", [](uintptr_t st, const py::tuple& shp, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats,
                       uintptr_t shift, uintptr_t ws, long ws_floats, uintptr_t res) {
    launch_conv_fwd(S(st), shape_from(shp), P<const bf16>(x), P<const bf16>(w), P<bf16>(y), P<double>(stats),
                    P<const float>(shift), P<float>(ws), ws ? ws_floats : 0, P<const bf16>(res));
    check("conv_fwd");
  }, py::arg("st"), py::arg("shape"), py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stats"), py::arg("shift"),
     py::arg("ws") = 0, py::arg("ws_floats") = 0, py::arg("res") = 0);
  // add: dx = dgrad + add;  bsum (dict rep/reps/z/y/mean/inv): the producer BN's backward sums in the epilogue
  m.def("conv_dgrad", [](uintptr_t st, const py::tuple& shp, uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t ws,
                         long ws_floats, uintptr_t wd, int acc, uintptr_t add, py::object bsum) {
    BnSums bs{};
    const bool has_bs = !bsum.is_none();
    if (has_bs) bs = bnsums_from(bsum.cast<py::dict>());
    launch_conv_dgrad(S(st), shape_from(shp), P<const bf16>(dy), P<const bf16>(w), P<bf16>(dx), P<float>(ws),
                      ws ? ws_floats : 0, P<const bf16>(wd), acc, P<const bf16>(add), has_bs ? &bs : nullptr);
    check("conv_dgrad");
  }, py::arg("st"), py::arg("shape"), py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("ws") = 0,
     py::arg("ws_floats") = 0, py::arg("wd") = 0, py::arg("acc") = 0, py::arg("add") = 0, py::arg("bsum") = py::none());
  m.def("conv_dgrad_fusable", [](const py::tuple& shp, int has_wd) { return conv_dgrad_fusable(shape_from(shp), has_wd); });
  m.def("dgrad_pack_multi", [](uintptr_t st, const py::list& items) {
    std::vector<DPackItem> v;
    for (const auto& it : items) {
      const py::tuple t = it.cast<py::tuple>();
      if (t.size() != 9) throw std::invalid_argument("dgrad_pack_multi item: (w, wd, O, Cw, C, R, S, stride, pad)");
      v.push_back(DPackItem{P<const float>(t[0].cast<uintptr_t>()), P<bf16>(t[1].cast<uintptr_t>()), t[2].cast<int>(),
                            t[3].cast<int>(), t[4].cast<int>(), t[5].cast<int>(), t[6].cast<int>(), t[7].cast<int>(),
                            t[8].cast<int>()});
    }
    if (!v.empty()) launch_dgrad_pack_multi(S(st), v.data(), (int)v.size());
    check("dgrad_pack_multi");
  });
  m.def("conv_fd_ws_floats", [](const py::tuple& shp) { return conv_fd_ws_floats(shape_from(shp)); });
  // fused SGD + weight images: convs (off, wr, wd, O, Cw, C, R, S, stride, pad) inside the flat master and flat
  // segments (off, len) -> (table bytes for device memory, entries, workgroups, LDS bytes)
  m.def("sgd_pack_plan", [](const py::list& convs, const py::list& segs) {
    std::vector<SgdPackConv> cv;
    for (const auto& it : convs) {
      const py::tuple t = it.cast<py::tuple>();
      if (t.size() != 10) throw std::invalid_argument("sgd_pack_plan conv: (off, wr, wd, O, Cw, C, R, S, stride, pad)");
      cv.push_back(SgdPackConv{t[0].cast<long>(), P<bf16>(t[1].cast<uintptr_t>()), P<bf16>(t[2].cast<uintptr_t>()),
                               t[3].cast<int>(), t[4].cast<int>(), t[5].cast<int>(), t[6].cast<int>(),
                               t[7].cast<int>(), t[8].cast<int>(), t[9].cast<int>()});
    }
    std::vector<long> sg;
    for (const auto& it : segs) {
      const py::tuple t = it.cast<py::tuple>();
      if (t.size() != 2) throw std::invalid_argument("sgd_pack_plan segment: (off, len)");
      sg.push_back(t[0].cast<long>());
      sg.push_back(t[1].cast<long>());
    }
    const SgdPackPlan p = build_sgd_pack_plan(cv.data(), (int)cv.size(), sg.data(), (int)(sg.size() / 2));
    return py::make_tuple(py::bytes(p.table.data(), p.table.size()), p.n_entries, p.n_blocks, p.lds_bytes);
  });
  m.def("sgd_pack", [](uintptr_t st, uintptr_t table, int n_entries, int n_blocks, int lds_bytes, uintptr_t p,
                       uintptr_t g, uintptr_t b, float lr, float mom, float wd, float damp, int nesterov, int first) {
    launch_sgd_pack(S(st), reinterpret_cast<const void*>(table), n_entries, n_blocks, lds_bytes, P<float>(p),
                    P<const float>(g), P<float>(b), lr, mom, wd, damp, nesterov, first);
    check("sgd_pack");
  });
  m.def("conv_pack_multi", [](uintptr_t st, const py::list& items) {
    std::vector<PackItem> v;
    for (const auto& it : items) {
      const py::tuple t = it.cast<py::tuple>();
      if (t.size() < 6 || t.size() > 8) throw std::invalid_argument("conv_pack_multi item: (w, wr, O, Cw, C, RS[, O8[, G]])");
      v.push_back(PackItem{P<const float>(t[0].cast<uintptr_t>()), P<bf16>(t[1].cast<uintptr_t>()), t[2].cast<int>(),
                           t[3].cast<int>(), t[4].cast<int>(), t[5].cast<int>(), t.size() >= 7 ? t[6].cast<int>() : 0,
                           t.size() >= 8 ? t[7].cast<int>() : 1});
    }
    if (!v.empty()) launch_conv_pack_multi(S(st), v.data(), (int)v.size());
    check("conv_pack_multi");
  });
  // defer != 0: the partial reduction is not launched; its descriptor comes back (wred_tuple) for wgrad_reduce_multi
  m.def("conv_wgrad", [](uintptr_t st, const py::tuple& shp, uintptr_t x, uintptr_t dy, uintptr_t dw, uintptr_t ws,
                         long ws_floats, int splits, int accumulate, int Ow, int G, int defer, int allow_1x1) -> py::object {
    WredItem it{};
    launch_conv_wgrad(S(st), shape_from(shp), P<const bf16>(x), P<const bf16>(dy), P<float>(dw), P<float>(ws),
                      ws_floats, splits, accumulate, Ow, G, defer ? &it : nullptr, allow_1x1);
    check("conv_wgrad");
    return defer ? wred_tuple(it) : py::object(py::none());
  }, py::arg("st"), py::arg("shp"), py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("ws"), py::arg("ws_floats"),
     py::arg("splits"), py::arg("accumulate"), py::arg("Ow") = 0, py::arg("G") = 1, py::arg("defer") = 0,
     py::arg("allow_1x1") = 1);
  m.def("wgrad_reduce_multi", [](uintptr_t st, const py::list& items) {
    std::vector<WredItem> v;
    for (const auto& o : items) v.push_back(wred_from(o.cast<py::tuple>()));
    if (!v.empty()) launch_wgrad_reduce_multi(S(st), v.data(), (int)v.size());
    check("wgrad_reduce_multi");
  });
  m.def("conv_wgrad_ws_floats", [](const py::tuple& shp) { return conv_wgrad_ws_floats(shape_from(shp)); });
  m.def("conv_pack", [](uintptr_t st, uintptr_t w, uintptr_t wr, int O, int Cw, int C, int RS, int O8, int G) {
    launch_conv_pack(S(st), P<const float>(w), P<bf16>(wr), O, Cw, C, RS, O8, G);
    check("conv_pack");
  }, py::arg("st"), py::arg("w"), py::arg("wr"), py::arg("O"), py::arg("Cw"), py::arg("C"), py::arg("RS"),
     py::arg("O8") = 0, py::arg("G") = 1);
  m.def("dw_fwd", [](uintptr_t st, const py::tuple& shp, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats,
                     uintptr_t shift) {
    launch_dw_fwd(S(st), dw_from(shp), P<const bf16>(x), P<const float>(w), P<bf16>(y), P<double>(stats),
                  P<const float>(shift));
    check("dw_fwd");
  }, py::arg("st"), py::arg("shp"), py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stats"), py::arg("shift"));
  m.def("dw_dgrad", [](uintptr_t st, const py::tuple& shp, uintptr_t dy, uintptr_t w, uintptr_t dx,
                       py::object bsum) {
    BnSums bs{};
    const bool has_bs = !bsum.is_none();
    if (has_bs) bs = bnsums_from(bsum.cast<py::dict>());
    launch_dw_dgrad(S(st), dw_from(shp), P<const bf16>(dy), P<const float>(w), P<bf16>(dx), has_bs ? &bs : nullptr);
    check("dw_dgrad");
  }, py::arg("st"), py::arg("shp"), py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("bsum") = py::none());
  m.def("dw_wgrad_ws_floats", [](const py::tuple& shp) { return dw_wgrad_ws_floats(dw_from(shp)); });
  m.def("dw_wgrad", [](uintptr_t st, const py::tuple& shp, uintptr_t x, uintptr_t dy, uintptr_t dw, uintptr_t ws,
                       long ws_floats, int accumulate, int defer) -> py::object {
    WredItem it{};
    launch_dw_wgrad(S(st), dw_from(shp), P<const bf16>(x), P<const bf16>(dy), P<float>(dw), P<float>(ws), ws_floats,
                    accumulate, defer ? &it : nullptr);
    check("dw_wgrad");
    return defer ? wred_tuple(it) : py::object(py::none());
  }, py::arg("st"), py::arg("shp"), py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("ws"), py::arg("ws_floats"),
     py::arg("accumulate"), py::arg("defer") = 0);
  m.def("prep_input", [](uintptr_t st, uintptr_t images, int base, uintptr_t dbase, int nb, int augment,
                         uint32_t seed, uintptr_t round_ctr, uintptr_t out) {
    launch_prep_input(S(st), P<const uint8_t>(images), base, P<const int>(dbase), nb, augment, seed,
                      P<const int>(round_ctr), P<bf16>(out));
    check("prep_input");
  });
  m.def("maxpool3", [](uintptr_t st, uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int stride) {
    launch_maxpool3(S(st), P<const bf16>(x), P<bf16>(y), P<uint8_t>(idx), N, H, W, C, stride);
    check("maxpool3");
  });
  m.def("maxpool3_bwd", [](uintptr_t st, uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int H, int W, int C,
                           int stride, int acc) {
    launch_maxpool3_bwd(S(st), P<const bf16>(dy), P<const uint8_t>(idx), P<bf16>(dx), N, H, W, C, stride, acc);
    check("maxpool3_bwd");
  });
  m.def("maxpool2", [](uintptr_t st, uintptr_t x, uintptr_t y, int N, int H, int W, int C) {
    launch_maxpool2(S(st), P<const bf16>(x), P<bf16>(y), N, H, W, C);
    check("maxpool2");
  });
  m.def("maxpool2_bwd", [](uintptr_t st, uintptr_t x, uintptr_t dy, uintptr_t dx, int N, int H, int W, int C) {
    launch_maxpool2_bwd(S(st), P<const bf16>(x), P<const bf16>(dy), P<bf16>(dx), N, H, W, C);
    check("maxpool2_bwd");
  });
  m.def("sched_next", [](uintptr_t st, uintptr_t sched, uintptr_t counter, uintptr_t cur, uintptr_t zero, long n) {
    launch_sched_next(S(st), P<const int>(sched), P<int>(counter), P<int>(cur), P<double>(zero), n);
    check("sched_next");
  });
  m.def("bn_apply", [](uintptr_t st, uintptr_t z, const py::dict& a, uintptr_t z2, py::object b, uintptr_t res,
                       uintptr_t y, int M, int C, float eps, float mom, int train, int relu, int ldy,
                       uintptr_t co_out) {
    BNDesc bd{};
    const bool has_b = !b.is_none();
    if (has_b) bd = bn_from(b.cast<py::dict>());
    launch_bn_apply(S(st), P<const bf16>(z), bn_from(a), P<const bf16>(z2), has_b ? &bd : nullptr, P<const bf16>(res),
                    P<bf16>(y), M, C, eps, mom, train, relu, ldy, P<float>(co_out));
    check("bn_apply");
  }, py::arg("st"), py::arg("z"), py::arg("a"), py::arg("z2"), py::arg("b"), py::arg("res"), py::arg("y"), py::arg("M"),
     py::arg("C"), py::arg("eps"), py::arg("mom"), py::arg("train"), py::arg("relu"), py::arg("ldy") = 0,
     py::arg("co_out") = 0);
  m.def("bn_bwd_ws_floats", [](int M, int C) { return bn_bwd_ws_floats(M, C); });
  m.def("bn_bwd", [](uintptr_t st, const py::dict& d, uintptr_t red, int M, int C, uintptr_t ws, long ws_floats,
                     int ldd, int ldy, int chained, int presummed) {
    BNBwdDesc b{P<const bf16>(dget(d, "dya")),     P<const bf16>(dget(d, "dyb")),     P<const bf16>(dget(d, "y")),
                P<const bf16>(dget(d, "za")),      P<const float>(dget(d, "meanA")),  P<const float>(dget(d, "invA")),
                P<const float>(dget(d, "gammaA")), P<float>(dget(d, "dgammaA")),      P<float>(dget(d, "dbetaA")),
                P<bf16>(dget(d, "dza")),           P<const bf16>(dget(d, "zb")),      P<const float>(dget(d, "meanB")),
                P<const float>(dget(d, "invB")),   P<const float>(dget(d, "gammaB")), P<float>(dget(d, "dgammaB")),
                P<float>(dget(d, "dbetaB")),       P<bf16>(dget(d, "dzb")),           P<bf16>(dget(d, "gout")),
                P<float>(dget(d, "shiftA")),       P<float>(dget(d, "shiftB")),       P<const bf16>(dget(d, "dadd")),
                P<const float>(dget(d, "msc"))};
    if (!b.dya || !b.za || !b.meanA || !b.invA || !b.gammaA || !b.dza) throw std::invalid_argument("bn_bwd: missing A");
    launch_bn_bwd(S(st), b, P<double>(red), M, C, P<double>(ws), ws ? ws_floats : 0, ldd, ldy, chained, presummed);
    check("bn_bwd");
  }, py::arg("st"), py::arg("desc"), py::arg("red"), py::arg("M"), py::arg("C"), py::arg("ws") = 0,
     py::arg("ws_floats") = 0, py::arg("ldd") = 0, py::arg("ldy") = 0, py::arg("chained") = 0,
     py::arg("presummed") = 0);
  m.def("bn_bwd_chain_reps", [](int C) { return bn_bwd_chain_reps(C); });
  m.def("head", [](uintptr_t st, uintptr_t y, uintptr_t labels, int base, uintptr_t dbase, int N, int HW, int C, int J,
                   uintptr_t W, uintptr_t b, uintptr_t pooled, uintptr_t dlog, uintptr_t dy, uintptr_t stats,
                   uintptr_t dW, uintptr_t db, int train, uintptr_t zero_buf, long zero_n, uintptr_t lossv) {
    launch_head(S(st), P<const bf16>(y), P<const int>(labels), base, P<const int>(dbase), N, HW, C, J, P<const float>(W),
                P<const float>(b), P<float>(pooled), P<float>(dlog), P<bf16>(dy), P<float>(stats), P<float>(lossv),
                P<float>(dW), P<float>(db), train, P<float>(zero_buf), zero_n);
    check("head");
  }, py::arg("st"), py::arg("y"), py::arg("labels"), py::arg("base"), py::arg("dbase"), py::arg("N"), py::arg("HW"),
     py::arg("C"), py::arg("J"), py::arg("W"), py::arg("b"), py::arg("pooled"), py::arg("dlog"), py::arg("dy"),
     py::arg("stats"), py::arg("dW"), py::arg("db"), py::arg("train"), py::arg("zero_buf") = 0, py::arg("zero_n") = 0,
     py::arg("lossv") = 0);
}
