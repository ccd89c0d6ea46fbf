// fedmi — Python bindings for the generic zoo kernels (csrc/kernels/zoo_ops.hip).
// A tensor crosses as (data_ptr, dtype code, sizes, strides); dtype codes: 0 fp32, 1 bf16, 2 int64.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <vector>

namespace py = pybind11;

#include "kernels/common.h"

namespace fedmi {
constexpr int ZMAXD = 6;
struct ZTensor {
  void* p;
  int dtype;
  int ndim;
  long long size[ZMAXD];
  long long stride[ZMAXD];
};
void launch_ew(hipStream_t, const ZTensor&, const ZTensor*, int, int, float, float, uint32_t, const int*, int, int);
void launch_ctr_bump(hipStream_t, int*);
long long reduce_rows_ws_floats(long long, int);
int rows_tune(int);
void launch_pad_rows(hipStream_t, const bf16*, long long, int, bf16*, int, long long);
void launch_reduce_rows(hipStream_t, const void*, int, long long, const void*, int, long long, const float*, int,
                        long long, int, float*, long long, float*, float*, void*, int, float);
void launch_reduce(hipStream_t, const ZTensor&, const ZTensor&, const ZTensor&, const ZTensor&, const void*, int,
                   const void*, int, const float*, float*, float*, int, float*, long long, void*, int, float);
long long reduce_ws_floats(long long, long long);
void launch_bn_rows_fwd(hipStream_t, const void*, int, long long, const float*, int, long long, float*, long long,
                        const float*, const float*, float*, float*, float, float, float*, float*, float*, float*,
                        long long*);
void launch_bn_rows_bwd(hipStream_t, const void*, int, long long, const void*, int, long long, const void*, int,
                        long long, float, const float*, const float*, const float*, int, long long, float*, long long,
                        float*, float*, float*, float*, float*);
void launch_bn_fwd_coeffs(hipStream_t, const float*, const float*, const float*, int, long long, const float*,
                          const float*, float*, float*, float, float, int, float*, float*, float*, float*);
void launch_bn_bwd_coeffs(hipStream_t, const float*, const float*, const float*, const float*, const float*, int,
                          long long, float*, float*, float*, float*, float*);
void launch_pool_fwd(hipStream_t, const ZTensor&, const ZTensor&, const ZTensor&, int, int, int, int, int, int, int, int,
                     int);
void launch_pool_bwd(hipStream_t, const ZTensor&, const ZTensor&, const ZTensor&, int, int, int, int, int, int, int, int,
                     int);
void launch_gemm(hipStream_t, const ZTensor&, const ZTensor&, const ZTensor&, const ZTensor&, float, float);
void launch_log_softmax(hipStream_t, const ZTensor&, const ZTensor&, int, const ZTensor&);
void launch_nll_fwd(hipStream_t, const ZTensor&, const long long*, long long, int, int, void*, int, void*, int);
void launch_nll_bwd(hipStream_t, const ZTensor&, const void*, int, const void*, int, const long long*, long long, int,
                    int);
void launch_ce_stats(hipStream_t, const ZTensor&, const long long*, float*);
void launch_gconv(hipStream_t, int, const ZTensor&, const ZTensor&, const ZTensor&, int, int, int, int, int, float*,
                  long long);
long long gconv_wgrad_ws_floats(long long, long long, long long, long long);
}  // namespace fedmi

using fedmi::ZTensor;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// (ptr, dtype, sizes, strides) or None
static ZTensor zt(const py::object& o) {
  ZTensor t{};
  if (o.is_none()) return t;
  py::tuple tp = o.cast<py::tuple>();
  if (tp.size() != 4) throw std::invalid_argument("tensor descriptor: (ptr, dtype, sizes, strides)");
  t.p = reinterpret_cast<void*>(tp[0].cast<uintptr_t>());
  t.dtype = tp[1].cast<int>();
  auto sz = tp[2].cast<std::vector<long long>>();
  auto sd = tp[3].cast<std::vector<long long>>();
  if (sz.size() != sd.size() || sz.size() > (size_t)fedmi::ZMAXD) throw std::invalid_argument("tensor descriptor: rank");
  t.ndim = (int)sz.size();
  for (int d = 0; d < t.ndim; ++d) {
    t.size[d] = sz[d];
    t.stride[d] = sd[d];
  }
  return t;
}

void fedmi_bind_zoo(py::module_& m) {
  // vmask < 0: scalar launch; otherwise the 8-wide vector launch (descriptors pre-divided by the caller)
  m.def("z_ew", [](uintptr_t st, py::object out, std::vector<py::object> ins, int op, float s0, float s1,
                   uint32_t seed, uintptr_t ctr, int vmask, int vw) {
    std::vector<ZTensor> v;
    for (auto& o : ins) v.push_back(zt(o));
    fedmi::launch_ew(S(st), zt(out), v.data(), (int)v.size(), op, s0, s1, seed, reinterpret_cast<const int*>(ctr),
                     vmask, vw);
  }, py::arg("st"), py::arg("out"), py::arg("ins"), py::arg("op"), py::arg("s0"), py::arg("s1"), py::arg("seed"),
        py::arg("ctr"), py::arg("vmask") = -1, py::arg("vw") = 8);
  m.def("z_ctr_bump", [](uintptr_t st, uintptr_t ctr) { fedmi::launch_ctr_bump(S(st), reinterpret_cast<int*>(ctr)); });
  m.def("z_reduce", [](uintptr_t st, py::object outer, py::object inner, py::object outer_b, py::object inner_b,
                       uintptr_t a, int a_dt, uintptr_t b, int b_dt, uintptr_t shift, uintptr_t acc, uintptr_t acc2,
                       int op, uintptr_t part, long long part_floats, uintptr_t out, int out_dt, float scale) {
    fedmi::launch_reduce(S(st), zt(outer), zt(inner), zt(outer_b), zt(inner_b), reinterpret_cast<const void*>(a), a_dt,
                         reinterpret_cast<const void*>(b), b_dt, reinterpret_cast<const float*>(shift),
                         reinterpret_cast<float*>(acc), reinterpret_cast<float*>(acc2), op,
                         reinterpret_cast<float*>(part), part_floats, reinterpret_cast<void*>(out), out_dt, scale);
  }, py::arg("st"), py::arg("outer"), py::arg("inner"), py::arg("outer_b"), py::arg("inner_b"), py::arg("a"),
     py::arg("a_dt"), py::arg("b"), py::arg("b_dt"), py::arg("shift"), py::arg("acc"), py::arg("acc2"), py::arg("op"),
     py::arg("part"), py::arg("part_floats"), py::arg("out") = 0, py::arg("out_dt") = 0, py::arg("scale") = 1.f);
  m.def("z_reduce_ws_floats", &fedmi::reduce_ws_floats);
  m.def("z_reduce_rows_ws_floats", &fedmi::reduce_rows_ws_floats);
  m.def("z_rows_tune", &fedmi::rows_tune);   // rows per row lane of the row reductions (benchmark sweeps)
  m.def("z_pad_rows", [](uintptr_t st, uintptr_t src, long long lds, int C, uintptr_t dst, int C8, long long rows) {
    fedmi::launch_pad_rows(S(st), reinterpret_cast<const bf16*>(src), lds, C, reinterpret_cast<bf16*>(dst), C8, rows);
  });
  m.def("z_reduce_rows", [](uintptr_t st, uintptr_t a, int a_dt, long long lda, uintptr_t b, int b_dt, long long ldb,
                            uintptr_t shift, int C, long long M, int op, uintptr_t part, long long part_floats,
                            uintptr_t acc, uintptr_t acc2, uintptr_t out, int out_dt, float scale) {
    fedmi::launch_reduce_rows(S(st), reinterpret_cast<const void*>(a), a_dt, lda, reinterpret_cast<const void*>(b), b_dt,
                              ldb, reinterpret_cast<const float*>(shift), C, M, op, reinterpret_cast<float*>(part),
                              part_floats, reinterpret_cast<float*>(acc), reinterpret_cast<float*>(acc2),
                              reinterpret_cast<void*>(out), out_dt, scale);
  }, py::arg("st"), py::arg("a"), py::arg("a_dt"), py::arg("lda"), py::arg("b"), py::arg("b_dt"), py::arg("ldb"),
     py::arg("shift"), py::arg("C"), py::arg("M"), py::arg("op"), py::arg("part"), py::arg("part_floats"),
     py::arg("acc"), py::arg("acc2"), py::arg("out") = 0, py::arg("out_dt") = 0, py::arg("scale") = 1.f);
  m.def("z_bn_fwd_coeffs", [](uintptr_t st, uintptr_t s1, uintptr_t s2, uintptr_t shift, int C, long long M, uintptr_t w,
                              uintptr_t b, uintptr_t rmean, uintptr_t rvar, float eps, float mom, int train,
                              uintptr_t save_mean, uintptr_t save_invstd, uintptr_t scale, uintptr_t bias) {
    auto f = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
    fedmi::launch_bn_fwd_coeffs(S(st), f(s1), f(s2), f(shift), C, M, f(w), f(b), f(rmean), f(rvar), eps, mom, train,
                                f(save_mean), f(save_invstd), f(scale), f(bias));
  });
  m.def("z_bn_rows_fwd", [](uintptr_t st, uintptr_t x, int x_dt, long long ldx, uintptr_t shift, int C, long long M,
                            uintptr_t part, long long part_floats, uintptr_t w, uintptr_t b, uintptr_t rmean,
                            uintptr_t rvar, float eps, float mom, uintptr_t save_mean, uintptr_t save_invstd,
                            uintptr_t scale, uintptr_t bias, uintptr_t ctr) {
    auto f = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
    fedmi::launch_bn_rows_fwd(S(st), reinterpret_cast<const void*>(x), x_dt, ldx, f(shift), C, M, f(part), part_floats,
                              f(w), f(b), f(rmean), f(rvar), eps, mom, f(save_mean), f(save_invstd), f(scale), f(bias),
                              reinterpret_cast<long long*>(ctr));
  }, py::arg("st"), py::arg("x"), py::arg("x_dt"), py::arg("ldx"), py::arg("shift"), py::arg("C"), py::arg("M"),
     py::arg("part"), py::arg("part_floats"), py::arg("w"), py::arg("b"), py::arg("rmean"), py::arg("rvar"),
     py::arg("eps"), py::arg("mom"), py::arg("save_mean"), py::arg("save_invstd"), py::arg("scale"), py::arg("bias"),
     py::arg("ctr") = 0);
  m.def("z_bn_rows_bwd", [](uintptr_t st, uintptr_t g, int g_dt, long long ldg, uintptr_t x, int x_dt, long long ldx,
                            uintptr_t fm, int f_dt, long long ldf, float thr, uintptr_t mean, uintptr_t invstd,
                            uintptr_t w, int C, long long M, uintptr_t part, long long part_floats, uintptr_t k,
                            uintptr_t bb, uintptr_t cc, uintptr_t dw, uintptr_t db) {
    auto f = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
    fedmi::launch_bn_rows_bwd(S(st), reinterpret_cast<const void*>(g), g_dt, ldg, reinterpret_cast<const void*>(x), x_dt,
                              ldx, reinterpret_cast<const void*>(fm), f_dt, ldf, thr, f(mean), f(invstd), f(w), C, M,
                              f(part), part_floats, f(k), f(bb), f(cc), f(dw), f(db));
  });
  m.def("z_bn_bwd_coeffs", [](uintptr_t st, uintptr_t sg, uintptr_t sgx, uintptr_t mean, uintptr_t invstd, uintptr_t w,
                              int C, long long M, uintptr_t k, uintptr_t bb, uintptr_t cc, uintptr_t dw, uintptr_t db) {
    auto f = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
    fedmi::launch_bn_bwd_coeffs(S(st), f(sg), f(sgx), f(mean), f(invstd), f(w), C, M, f(k), f(bb), f(cc), f(dw), f(db));
  });
  m.def("z_pool_fwd", [](uintptr_t st, py::object x, py::object y, py::object idx, int kh, int kw, int sh, int sw,
                         int ph, int pw, int cip, int divisor, int is_max) {
    fedmi::launch_pool_fwd(S(st), zt(x), zt(y), zt(idx), kh, kw, sh, sw, ph, pw, cip, divisor, is_max);
  });
  m.def("z_pool_bwd", [](uintptr_t st, py::object dx, py::object dy, py::object idx, int kh, int kw, int sh, int sw,
                         int ph, int pw, int cip, int divisor, int is_max) {
    fedmi::launch_pool_bwd(S(st), zt(dx), zt(dy), zt(idx), kh, kw, sh, sw, ph, pw, cip, divisor, is_max);
  });
  m.def("z_gemm", [](uintptr_t st, py::object a, py::object b, py::object c, py::object bias, float alpha, float beta) {
    fedmi::launch_gemm(S(st), zt(a), zt(b), zt(c), zt(bias), alpha, beta);
  });
  m.def("z_log_softmax", [](uintptr_t st, py::object x, py::object y, int bwd, py::object gy) {
    fedmi::launch_log_softmax(S(st), zt(x), zt(y), bwd, zt(gy));
  });
  m.def("z_nll_fwd", [](uintptr_t st, py::object lp, uintptr_t tgt, long long tstride, int ignore, int mean,
                        uintptr_t out, int out_bf16, uintptr_t tw, int tw_bf16) {
    fedmi::launch_nll_fwd(S(st), zt(lp), reinterpret_cast<const long long*>(tgt), tstride, ignore, mean,
                          reinterpret_cast<void*>(out), out_bf16, reinterpret_cast<void*>(tw), tw_bf16);
  });
  m.def("z_nll_bwd", [](uintptr_t st, py::object gx, uintptr_t g, int g_bf16, uintptr_t tw, int tw_bf16, uintptr_t tgt,
                        long long tstride, int ignore, int mean) {
    fedmi::launch_nll_bwd(S(st), zt(gx), reinterpret_cast<const void*>(g), g_bf16, reinterpret_cast<const void*>(tw),
                          tw_bf16, reinterpret_cast<const long long*>(tgt), tstride, ignore, mean);
  });
  m.def("z_ce_stats", [](uintptr_t st, py::object logits, uintptr_t y, uintptr_t stats) {
    fedmi::launch_ce_stats(S(st), zt(logits), reinterpret_cast<const long long*>(y), reinterpret_cast<float*>(stats));
  });
  m.def("z_gconv", [](uintptr_t st, int mode, py::object x, py::object w, py::object y, int G, int sth, int stw,
                      int padh, int padw, uintptr_t ws, long long ws_floats) {
    fedmi::launch_gconv(S(st), mode, zt(x), zt(w), zt(y), G, sth, stw, padh, padw, reinterpret_cast<float*>(ws),
                        ws_floats);
  }, py::arg("st"), py::arg("mode"), py::arg("x"), py::arg("w"), py::arg("y"), py::arg("G"), py::arg("sth"),
        py::arg("stw"), py::arg("padh"), py::arg("padw"), py::arg("ws") = 0, py::arg("ws_floats") = 0);
  m.def("z_gconv_wgrad_ws_floats", &fedmi::gconv_wgrad_ws_floats);
}
