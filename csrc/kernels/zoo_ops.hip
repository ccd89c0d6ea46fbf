// fedmi — generic native kernels for the zoo families without a whole-network
// engine (DenseNet, ResNeXt, DPN, ShuffleNet v1/v2, SENet, EfficientNet, RegNet,
// PNASNet, DLA, SimpleDLA).  They back the aten ops of a
// training step through fedmi.ops.native_mode (a TorchDispatchMode): every
// elementwise / reduction / BatchNorm / pooling / GEMM / loss / grouped-conv op of
// those models runs here or on the MFMA / depthwise conv kernels, none on ATen.
//
// Tensors are described by (ptr, dtype, sizes, strides) so one kernel serves any
// layout (channels-last activations, broadcast operands, channel slices of a
// concatenation); dtypes are fp32 / bf16 / int64.  Integer index math is 64-bit
// only where a tensor can exceed 2^31 elements' byte range (never, in practice).
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>

#include "common.h"

namespace fedmi {
void check_hip(hipError_t e, const char* what);

constexpr int ZMAXD = 6;
enum ZDtype : int { Z_F32 = 0, Z_BF16 = 1, Z_I64 = 2 };

struct ZTensor {
  void* p;
  int dtype;
  int ndim;
  long long size[ZMAXD];
  long long stride[ZMAXD];
};
}  // namespace fedmi

namespace {
using fedmi::ZTensor;
using fedmi::ZMAXD;

FEDMI_DEV float zload(const ZTensor& t, long long off) {
  if (t.dtype == 0) return reinterpret_cast<const float*>(t.p)[off];
  if (t.dtype == 1) return (float)reinterpret_cast<const bf16*>(t.p)[off];
  return (float)reinterpret_cast<const long long*>(t.p)[off];
}
FEDMI_DEV void zstore(const ZTensor& t, long long off, float v) {
  if (t.dtype == 0) reinterpret_cast<float*>(t.p)[off] = v;
  else if (t.dtype == 1) reinterpret_cast<bf16*>(t.p)[off] = (bf16)v;
  else reinterpret_cast<long long*>(t.p)[off] = (long long)v;
}

// ---- elementwise ------------------------------------------------------------------
enum EwOp : int {
  EW_COPY = 0,       // o = a
  EW_ADD = 1,        // o = a + s0 * b
  EW_MUL = 2,        // o = a * b
  EW_MULS = 3,       // o = a * s0
  EW_RELU = 4,       // o = max(a, 0)
  EW_THR_BWD = 5,    // o = b > s0 ? a : 0          (threshold_backward(grad=a, self=b))
  EW_SIGMOID = 6,    // o = 1 / (1 + exp(-a))
  EW_SIG_BWD = 7,    // o = a * b * (1 - b)         (sigmoid_backward(grad=a, out=b))
  EW_FILL = 8,       // o = s0
  EW_FMA = 9,        // o = a * b + c
  EW_BNB = 11,       // o = a * b + c * d + e      (BatchNorm backward apply: g*k + x*bb + cc)
  EW_BERN = 12,      // o = hash(seed, ctr, i) < s0 ? 1 : 0   (bernoulli_(p = s0))
  EW_SUB = 13,       // o = a - s0 * b
  EW_DIV = 14,       // o = a / b
  EW_ADDS = 15,      // o = a + s0
  EW_FMA_RELU = 16,  // o = max(a * b + c, 0)      (BatchNorm apply + ReLU in one pass)
  EW_BNB_THR = 17,   // o = (f > s0 ? a : 0) * b + c * d + e   (threshold_backward fused into BN backward)
  EW_FMA_ADD = 18,   // o = r(a * b + c) + d       (BatchNorm apply + residual add; r = bf16 rounding if s1)
  EW_FMA_ADD_RELU = 19,  // o = max(r(a * b + c) + d, 0)  (BatchNorm apply + residual add + ReLU)
  EW_BNB_ADD = 20,   // o = r(a * b + c * d + e) + f          (BN backward apply + the gradient accumulation add)
  EW_BNB_THR_ADD = 21,  // o = r((f > s0 ? a : 0) * b + c * d + e) + g
};

// NIN input descriptors: 6 for every op but the 7-operand BN-backward + accumulation pass, so the common
// launches do not carry (or unroll over) a seventh descriptor
template <int NIN>
struct EwArgs {
  ZTensor o;
  ZTensor in[NIN];
  float s0, s1;
  int op;
  uint32_t seed;
  const int* ctr;    // EW_BERN: device step counter
  int vmask;         // vector launch: bit k set = input k is contiguous over the 8-element group
};

// offset of linear element `i` of the output iteration space in tensor t
// (32-bit index decode: the host guarantees every tensor has < 2^31 elements; the host also
// coalesces dims, so activations + per-channel operands arrive as 1-2 dims: 0-1 divisions)
FEDMI_DEV long long zoffset(const ZTensor& shape, const ZTensor& t, long long i64) {
  uint32_t i = (uint32_t)i64;
  long long off = 0;
#pragma unroll
  for (int d = ZMAXD - 1; d >= 1; --d) {
    if (d < shape.ndim) {
      const uint32_t sz = (uint32_t)shape.size[d];
      const uint32_t q = i / sz;
      off += (long long)(i - q * sz) * t.stride[d];
      i = q;
    }
  }
  return off + (long long)i * t.stride[0];
}

// The N-d coordinates of linear index i in `shape` (the divisions), computed ONCE per element and shared by
// every operand of an elementwise op; zoff() is then one multiply-add per dimension per operand (zoffset per
// operand repeated the divisions: the index math, not memory, bounded the 4-6 operand BN passes).
struct ZCoord {
  uint32_t c[ZMAXD];
};

FEDMI_DEV ZCoord zcoords(const ZTensor& shape, long long i64) {
  ZCoord k;
  uint32_t i = (uint32_t)i64;
#pragma unroll
  for (int d = ZMAXD - 1; d >= 1; --d) {
    k.c[d] = 0u;
    if (d < shape.ndim) {
      const uint32_t sz = (uint32_t)shape.size[d];
      const uint32_t q = i / sz;
      k.c[d] = i - q * sz;
      i = q;
    }
  }
  k.c[0] = i;
  return k;
}

FEDMI_DEV long long zoff(const ZCoord& k, const ZTensor& t, int ndim) {
  long long off = (long long)k.c[0] * t.stride[0];
#pragma unroll
  for (int d = 1; d < ZMAXD; ++d)
    if (d < ndim) off += (long long)k.c[d] * t.stride[d];
  return off;
}

template <class A>
FEDMI_DEV float ew_apply(const A& a, float x0, float x1, float x2, float x3, float x4, float x5 = 0.f,
                         float x6 = 0.f) {
  switch (a.op) {
    case EW_COPY: return x0;
    case EW_ADD: return x0 + a.s0 * x1;
    case EW_SUB: return x0 - a.s0 * x1;
    case EW_MUL: return x0 * x1;
    case EW_DIV: return x0 / x1;
    case EW_ADDS: return x0 + a.s0;
    case EW_MULS: return x0 * a.s0;
    case EW_RELU: return fmaxf(x0, 0.f);
    case EW_THR_BWD: return x1 > a.s0 ? x0 : 0.f;
    case EW_SIGMOID: return 1.f / (1.f + __expf(-x0));
    case EW_SIG_BWD: return x0 * x1 * (1.f - x1);
    case EW_FILL: return a.s0;
    case EW_FMA: return x0 * x1 + x2;
    case EW_BNB: return x0 * x1 + x2 * x3 + x4;
    case EW_FMA_RELU: return fmaxf(x0 * x1 + x2, 0.f);
    case EW_BNB_THR: return (x5 > a.s0 ? x0 : 0.f) * x1 + x2 * x3 + x4;
    // s1 != 0: the BN output is rounded to bf16 before the add, exactly as the unfused pair stores it
    case EW_FMA_ADD: return (a.s1 != 0.f ? (float)(bf16)(x0 * x1 + x2) : x0 * x1 + x2) + x3;
    case EW_FMA_ADD_RELU: return fmaxf((a.s1 != 0.f ? (float)(bf16)(x0 * x1 + x2) : x0 * x1 + x2) + x3, 0.f);
    // the BN-backward gradient is rounded (s1) as the unfused pair stores it before autograd's accumulation add
    case EW_BNB_ADD: {
      const float gi = x0 * x1 + x2 * x3 + x4;
      return (a.s1 != 0.f ? (float)(bf16)gi : gi) + x5;
    }
    case EW_BNB_THR_ADD: {
      const float gi = (x5 > a.s0 ? x0 : 0.f) * x1 + x2 * x3 + x4;
      return (a.s1 != 0.f ? (float)(bf16)gi : gi) + x6;
    }
    default: return 0.f;
  }
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// VW consecutive elements (VW = 8 or 4) as 16- / 8-byte bf16 or 16-byte fp32 vector accesses
template <int VW>
FEDMI_DEV void vload(const void* p, int dt, long long off, float* v) {
  if (dt == 1) {
    if constexpr (VW == 8) {
      const bf16x8 q = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(p) + off);
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = (float)q[u];
    } else {
      const bf16x4 q = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(p) + off);
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (float)q[u];
    }
  } else {
#pragma unroll
    for (int h = 0; h < VW / 4; ++h) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p) + off + 4 * h);
#pragma unroll
      for (int u = 0; u < 4; ++u) v[4 * h + u] = q[u];
    }
  }
}

template <int VW>
FEDMI_DEV void vstore(void* p, int dt, long long off, const float* v) {
  if (dt == 1) {
    if constexpr (VW == 8) {
      bf16x8 q;
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = (bf16)v[u];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(p) + off) = q;
    } else {
      bf16x4 q;
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = (bf16)v[u];
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p) + off) = q;
    }
  } else {
#pragma unroll
    for (int h = 0; h < VW / 4; ++h) {
      f32x4 q;
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = v[4 * h + u];
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p) + off + 4 * h) = q;
    }
  }
}

// VW consecutive innermost elements per thread (host-checked alignment); the descriptors' innermost
// size is already divided by VW and unit strides scaled by VW; a broadcast input (vmask bit clear)
// is one scalar load
template <int VW, int NIN>
__global__ __launch_bounds__(256) void ew_vec_kernel(EwArgs<NIN> a, long long nv) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const ZCoord kc = zcoords(a.o, i);
    float x[7][VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) x[6][u] = 0.f;
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      if (a.in[k].p && ((a.vmask >> k) & 1)) {
        vload<VW>(a.in[k].p, a.in[k].dtype, zoff(kc, a.in[k], a.o.ndim), x[k]);
      } else {
        const float sv = a.in[k].p ? zload(a.in[k], zoff(kc, a.in[k], a.o.ndim)) : 0.f;
#pragma unroll
        for (int u = 0; u < VW; ++u) x[k][u] = sv;
      }
    }
    float v[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) v[u] = ew_apply(a, x[0][u], x[1][u], x[2][u], x[3][u], x[4][u], x[5][u], x[6][u]);
    vstore<VW>(a.o.p, a.o.dtype, zoff(kc, a.o, a.o.ndim), v);
  }
}

template <int NIN>
__global__ __launch_bounds__(256) void ew_kernel(EwArgs<NIN> a, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const uint32_t ctr = a.ctr ? (uint32_t)a.ctr[0] : 0u;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const ZCoord kc = zcoords(a.o, i);
    float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f, x4 = 0.f, x5 = 0.f, x6 = 0.f;
    if (a.in[0].p) x0 = zload(a.in[0], zoff(kc, a.in[0], a.o.ndim));
    if (a.in[1].p) x1 = zload(a.in[1], zoff(kc, a.in[1], a.o.ndim));
    if (a.in[2].p) x2 = zload(a.in[2], zoff(kc, a.in[2], a.o.ndim));
    if (a.in[3].p) x3 = zload(a.in[3], zoff(kc, a.in[3], a.o.ndim));
    if (a.in[4].p) x4 = zload(a.in[4], zoff(kc, a.in[4], a.o.ndim));
    if (a.in[5].p) x5 = zload(a.in[5], zoff(kc, a.in[5], a.o.ndim));
    if constexpr (NIN > 6) {
      if (a.in[6].p) x6 = zload(a.in[6], zoff(kc, a.in[6], a.o.ndim));
    }
    float v;
    if (a.op == EW_BERN) {
      const uint32_t h = hash3(a.seed, ctr, (uint32_t)i ^ (uint32_t)(i >> 32));
      v = ((float)(h >> 8) * (1.f / 16777216.f)) < a.s0 ? 1.f : 0.f;
    } else {
      v = ew_apply(a, x0, x1, x2, x3, x4, x5, x6);
    }
    zstore(a.o, zoff(kc, a.o, a.o.ndim), v);
  }
}

__global__ void ctr_bump_kernel(int* ctr) {
  if (threadIdx.x == 0) ctr[0] += 1;
}

// ---- reduction: out[outer] (+)= sum over inner of f(in...) ----------------------------
// outer / inner index spaces with their own sizes and per-tensor strides.
// RD_DOT_R: sum a, sum bf16(a * b) -- the product rounded as a stored bf16 product would be (exact fusion)
enum RdOp : int { RD_SUM = 0, RD_SUMSQ_SHIFT = 1, RD_DOT_SHIFT = 2, RD_DOT_R = 3 };
struct RdArgs {
  ZTensor outer;     // sizes of the kept dims; strides of input a along them
  ZTensor inner;     // sizes of the reduced dims; strides of input a along them
  ZTensor outer_b;   // strides of input b along the kept dims (RD_DOT_SHIFT)
  ZTensor inner_b;
  const void* a;
  int a_dtype;
  const void* b;
  int b_dtype;
  const float* shift;   // per-outer shift (moments of (a - shift)), or null
  float* acc;           // fp32 [n_outer] accumulator, zeroed by the host
  float* acc2;          // second accumulator (RD_SUMSQ_SHIFT: sum of squares; RD_DOT_SHIFT: sum a*(b-shift))
  float* part;          // [2][splits][n_outer] per-split partials (splits > 1), summed in split order afterwards
  int op;
  void* out;            // RD_SUM with out: out[o] = scale * sum, stored in out_dt (overwrite; acc unused)
  int out_dt;
  float scale;
};

FEDMI_DEV float rload(const void* p, int dt, long long off) {
  if (dt == 0) return reinterpret_cast<const float*>(p)[off];
  return (float)reinterpret_cast<const bf16*>(p)[off];
}

FEDMI_DEV void rstore(void* p, int dt, long long off, float v) {
  if (dt == 0) reinterpret_cast<float*>(p)[off] = v;
  else reinterpret_cast<bf16*>(p)[off] = (bf16)v;
}

// block = 64 outer lanes x 4 inner lanes; grid = (outer tiles, inner splits)
__global__ __launch_bounds__(256) void reduce_kernel(RdArgs r, long long n_outer, long long n_inner) {
  __shared__ float red[2][4][64];
  const int lo = threadIdx.x & 63, li = threadIdx.x >> 6;
  const long long o = (long long)blockIdx.x * 64 + lo;
  float s1 = 0.f, s2 = 0.f;
  if (o < n_outer) {
    const long long base_a = zoffset(r.outer, r.outer, o);
    const long long base_b = r.b ? zoffset(r.outer, r.outer_b, o) : 0;
    const float sh = r.shift ? r.shift[o] : 0.f;
    const long long per = (n_inner + gridDim.y - 1) / gridDim.y;
    const long long i0 = (long long)blockIdx.y * per, i1 = i0 + per < n_inner ? i0 + per : n_inner;
    long long i = i0 + li;
    if (r.op == RD_SUM) {
      // 8 inner elements per pass, every load issued before the first add (clamped index, masked value):
      // one memory latency per 8 elements instead of per element
      constexpr int U = 8;
      for (; i < i1; i += 4 * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long iu = i + 4 * u < i1 ? i + 4 * u : i;
          v[u] = rload(r.a, r.a_dtype, base_a + zoffset(r.inner, r.inner, iu));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) s1 += i + 4 * u < i1 ? v[u] : 0.f;
      }
    }
    for (; i < i1; i += 4) {
      const float va = rload(r.a, r.a_dtype, base_a + zoffset(r.inner, r.inner, i));
      if (r.op == RD_SUM) {
        s1 += va;
      } else if (r.op == RD_SUMSQ_SHIFT) {
        const float d = va - sh;
        s1 += d;
        s2 += d * d;
      } else if (r.op == RD_DOT_R) {
        const float vb = rload(r.b, r.b_dtype, base_b + zoffset(r.inner, r.inner_b, i));
        s1 += va;
        s2 += (float)(bf16)(va * vb);
      } else {
        const float vb = rload(r.b, r.b_dtype, base_b + zoffset(r.inner, r.inner_b, i));
        s1 += va;
        s2 += va * (vb - sh);
      }
    }
  }
  red[0][li][lo] = s1;
  red[1][li][lo] = s2;
  __syncthreads();
  if (li == 0 && o < n_outer) {
    // no atomics: one writer per (split, outer), so the result does not depend on workgroup order
    const float t1 = red[0][0][lo] + red[0][1][lo] + red[0][2][lo] + red[0][3][lo];
    const float t2 = red[1][0][lo] + red[1][1][lo] + red[1][2][lo] + red[1][3][lo];
    if (gridDim.y == 1 && r.out) {
      rstore(r.out, r.out_dt, o, r.scale * (r.op == RD_SUM ? t1 : t2));
    } else if (gridDim.y == 1) {
      r.acc[o] += t1;
      if (r.op != RD_SUM) r.acc2[o] += t2;
    } else {
      r.part[(long long)blockIdx.y * n_outer + o] = t1;
      if (r.op != RD_SUM) r.part[((long long)gridDim.y + blockIdx.y) * n_outer + o] = t2;
    }
  }
}

__global__ __launch_bounds__(256) void reduce_splits_kernel(const float* part, int splits, long long n_outer,
                                                            float* acc, float* acc2, void* out, int out_dt,
                                                            float scale, int two) {
  const long long o = (long long)blockIdx.x * 256 + threadIdx.x;
  if (o >= n_outer) return;
  float s1 = 0.f, s2 = 0.f;
  for (int y = 0; y < splits; ++y) {
    s1 += part[(long long)y * n_outer + o];
    if (two) s2 += part[((long long)splits + y) * n_outer + o];
  }
  if (out) {
    rstore(out, out_dt, o, scale * (two ? s2 : s1));   // RD_DOT_SHIFT: the dot sums
    return;
  }
  acc[o] += s1;
  if (acc2) acc2[o] += s2;
}

// sum over slabs of part[slab * pitch + i], 64 elements x 4 slab lanes per block, lanes combined in
// a fixed order (deterministic); returns the total on lane 0 (others: 0)
FEDMI_DEV float ordered_slab_sum(const float* part, int slabs, long long pitch, long long i, bool valid) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x >> 6, el = threadIdx.x & 63;
  float v = 0.f;
  if (valid) {
#pragma unroll 8
    for (int b = lane; b < slabs; b += 4) v += part[(long long)b * pitch + i];
  }
  red[lane][el] = v;
  __syncthreads();
  return lane == 0 ? red[0][el] + red[1][el] + red[2][el] + red[3][el] : 0.f;
}

// bf16 load of VW channels, no dtype branch (fast path of the row reduction)
template <int VW>
FEDMI_DEV void vload_bf(const void* p, long long off, float* v) {
  if constexpr (VW == 8) {
    const bf16x8 q = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(p) + off);
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (float)q[u];
  } else {
    const bf16x4 q = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(p) + off);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (float)q[u];
  }
}

// rows [r0 + rl, r1) step RL of one channel vector, U rows per pass with every load issued first (OPK 0: sum
// of a, 1: sum / sum of squares of a - shift, 2: sum a / sum a * (b - shift); HF: a masked by f > thr)
template <int VW, bool BF, bool HF, int OPK>
FEDMI_DEV void rows_pass(const void* a, long long lda, const void* b, long long ldb, const void* f, long long ldf,
                         float thr, const float* sh, int v, int rl, int RL, long long r0, long long r1, float* s1,
                         float* s2) {
  static_assert(BF, "bf16 operands only");
  constexpr int U = 4;
  for (long long rb = r0 + rl; rb < r1; rb += (long long)U * RL) {
    float x[U][VW], m[U][VW], y[U][VW];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long rr = rb + (long long)k * RL;
      const long long r = rr < r1 ? rr : rb;
      vload_bf<VW>(a, r * lda + v * VW, x[k]);
      if constexpr (HF) vload_bf<VW>(f, r * ldf + v * VW, m[k]);
      if constexpr (OPK == 2) vload_bf<VW>(b, r * ldb + v * VW, y[k]);
    }
    // dead rows (past r1) contribute exact zeros through selects, never through an extra multiply; the
    // products are explicit fmas, so the rounding cannot depend on how the compiler contracts each
    // instantiation (a masked and a pre-masked gradient give bit-identical sums)
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool live = rb + (long long)k * RL < r1;
#pragma unroll
      for (int u = 0; u < VW; ++u) {
        float xv = live ? x[k][u] : 0.f;
        if constexpr (HF) xv = m[k][u] > thr ? xv : 0.f;
        if constexpr (OPK == 0) {
          s1[u] += xv;
        } else if constexpr (OPK == 1) {
          const float d = live ? xv - sh[u] : 0.f;
          s1[u] += d;
          s2[u] = __builtin_fmaf(d, d, s2[u]);
        } else {
          const float yv = live ? y[k][u] - sh[u] : 0.f;
          s1[u] += xv;
          s2[u] = __builtin_fmaf(xv, yv, s2[u]);
        }
      }
    }
  }
}

// ---- channel pad: dst [rows][C8] (compact) = src [rows][C] (row stride lds, any 2-byte alignment), zero
// channels C..C8; one launch for the fill + copy pair.  One thread per 8-channel destination vector.
__global__ __launch_bounds__(256) void pad_rows_kernel(const bf16* __restrict__ src, long long lds, int C,
                                                       bf16* __restrict__ dst, int C8, long long rows, int vec) {
  const int VD = C8 >> 3;
  const long long n = rows * VD;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long r = i / VD;
    const int c0 = (int)(i - r * VD) * 8;
    bf16x8 o;
    const bf16* sp = src + r * lds + c0;
    if (vec && c0 + 8 <= C) {
      o = *reinterpret_cast<const bf16x8*>(sp);
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) o[u] = c0 + u < C ? sp[u] : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(dst + r * C8 + c0) = o;
  }
}

// Finalize arguments of a row pass, applied per channel by rows_fin_kernel
// (mode 1: forward statistics -> coefficients / running stats, 2: backward sums -> coefficients, 0: none)
struct BnFin {
  int mode;
  long long M;
  const float* shift; const float* w; const float* b; float* rmean; float* rvar; float eps, mom;
  float* save_mean; float* save_invstd; float* scale; float* bias;
  const float* mean; const float* invstd; float* k; float* bb; float* cc; float* dw; float* db;
  long long* ctr;         // mode 1: the module's num_batches_tracked, += 1 by the finalizing workgroup (or null)
  void* out; int out_dt; float out_scale;   // mode 3 (row sums): out[c] = out_scale * sum (dot sum if two), in out_dt
  int two;
};

FEDMI_DEV void bn_fwd_fin(const BnFin& f, int c, float s1, float s2) {
  const long long M = f.M;
  const float ms = s1 / (float)M;
  const float var = fmaxf(s2 / (float)M - ms * ms, 0.f);
  const float mean = ms + (f.shift ? f.shift[c] : 0.f);
  const float inv = rsqrtf(var + f.eps);
  if (f.save_mean) f.save_mean[c] = mean;
  if (f.save_invstd) f.save_invstd[c] = inv;
  if (f.rmean) {
    f.rmean[c] = (1.f - f.mom) * f.rmean[c] + f.mom * mean;
    f.rvar[c] = (1.f - f.mom) * f.rvar[c] + f.mom * var * ((float)M / (float)(M > 1 ? M - 1 : 1));
  }
  const float sc = (f.w ? f.w[c] : 1.f) * inv;
  f.scale[c] = sc;
  f.bias[c] = (f.b ? f.b[c] : 0.f) - mean * sc;
}

FEDMI_DEV void bn_bwd_fin(const BnFin& f, int c, float sg, float sgx) {
  const long long M = f.M;
  const float inv = f.invstd[c];
  const float kk = (f.w ? f.w[c] : 1.f) * inv;
  const float b = -kk * inv * inv * sgx / (float)M;
  f.k[c] = kk;
  f.bb[c] = b;
  f.cc[c] = -kk * sg / (float)M - b * f.mean[c];
  if (f.dw) f.dw[c] = sgx * inv;
  if (f.db) f.db[c] = sg;
}

constexpr int kRowsTileC = 64;   // channels per workgroup column tile

// ---- row reduction of a [M, C] row-major matrix (ld = row stride), C % 4 == 0 ------------------
// The channels-last case of the BN moments / bias gradients.  Grid = (64-channel column tiles, row slabs): a
// thread owns VW channels (one 16- / 8-byte load per row), RL = 256 / (tile vectors) row lanes per block, the
// row lanes are combined by a fixed-order LDS tree and each block stores its slab's sums to `part`
// [slabs][2][C]; rows_fin_kernel then adds the slabs in slab order (deterministic) and applies the BN
// finalize.  A kernel boundary publishes the partials: the one-launch form, whose last-arriving workgroups
// summed the slabs after an agent-scope release per workgroup, measured 1.1-2x slower at every zoo BN shape
// (profiles/r4_zoo/rows_ab).
template <int VW>
__global__ __launch_bounds__(256) void reduce_rows_kernel(const void* a, int a_dt, long long lda, const void* b,
                                                          int b_dt, long long ldb, const float* shift, int C,
                                                          long long M, int op, float* part, const void* f = nullptr,
                                                          int f_dt = 0, long long ldf = 0, float thr = 0.f) {
  __shared__ float red[2][256 * VW];
  const int VL = C / VW;
  const int vt = min(VL, kRowsTileC / VW);
  const int RL = 256 / vt;
  const int vl = threadIdx.x % vt;
  const int v = blockIdx.x * vt + vl;
  const int rl = threadIdx.x / vt;
  const bool act = rl < RL && v < VL;
  float s1[VW], s2[VW];
#pragma unroll
  for (int u = 0; u < VW; ++u) { s1[u] = 0.f; s2[u] = 0.f; }
  if (act) {
    float sh[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) sh[u] = shift ? shift[v * VW + u] : 0.f;
    const long long per = (M + gridDim.y - 1) / gridDim.y;
    const long long r0 = (long long)blockIdx.y * per, r1 = min(M, r0 + per);
    // U rows per pass, every load of the pass issued before the first use (clamped rows, masked): one
    // memory latency per U rows instead of per row; dtypes / operands are compile-time in the pass
    const bool dot = op != RD_SUM && op != RD_SUMSQ_SHIFT;
    const bool bf = a_dt == 1 && (!f || f_dt == 1) && (!dot || b_dt == 1);   // the prefetching bf16 pass
    const int opk = op == RD_SUM ? 0 : op == RD_SUMSQ_SHIFT ? 1 : 2;
#define FEDMI_ROWS(BF, HF, OPK) rows_pass<VW, BF, HF, OPK>(a, lda, b, ldb, f, ldf, thr, sh, v, rl, RL, r0, r1, s1, s2)
    if (bf) {
      if (f) { if (opk == 0) FEDMI_ROWS(true, true, 0); else if (opk == 1) FEDMI_ROWS(true, true, 1); else FEDMI_ROWS(true, true, 2); }
      else { if (opk == 0) FEDMI_ROWS(true, false, 0); else if (opk == 1) FEDMI_ROWS(true, false, 1); else FEDMI_ROWS(true, false, 2); }
    } else {
      for (long long r = r0 + rl; r < r1; r += RL) {   // generic dtypes (fp32 operands): one row at a time
        float x[VW];
        vload<VW>(a, a_dt, r * lda + v * VW, x);
        if (f) {
          float m[VW];
          vload<VW>(f, f_dt, r * ldf + v * VW, m);
#pragma unroll
          for (int u = 0; u < VW; ++u) x[u] = m[u] > thr ? x[u] : 0.f;
        }
        if (opk == 0) {
#pragma unroll
          for (int u = 0; u < VW; ++u) s1[u] += x[u];
        } else if (opk == 1) {
#pragma unroll
          for (int u = 0; u < VW; ++u) { const float d = x[u] - sh[u]; s1[u] += d; s2[u] = __builtin_fmaf(d, d, s2[u]); }
        } else {
          float y[VW];
          vload<VW>(b, b_dt, r * ldb + v * VW, y);
#pragma unroll
          for (int u = 0; u < VW; ++u) { s1[u] += x[u]; s2[u] = __builtin_fmaf(x[u], y[u] - sh[u], s2[u]); }
        }
      }
    }
#undef FEDMI_ROWS
  }
  // fixed-order tree over the row lanes of each channel vector: fold lanes >= P2 (largest power of two <= RL)
  // onto lanes < RL - P2, then halve
  auto put = [&]() {
#pragma unroll
    for (int u = 0; u < VW; ++u) { red[0][threadIdx.x * VW + u] = s1[u]; red[1][threadIdx.x * VW + u] = s2[u]; }
  };
  auto take = [&](int src_rl) {
    const int t = (src_rl * vt + vl) * VW;
#pragma unroll
    for (int u = 0; u < VW; ++u) { s1[u] += red[0][t + u]; s2[u] += red[1][t + u]; }
  };
  int P2 = 1;
  while (P2 * 2 <= RL) P2 *= 2;
  put();
  __syncthreads();
  if (rl < RL - P2) { take(rl + P2); put(); }
  __syncthreads();
  for (int sstep = P2 / 2; sstep >= 1; sstep /= 2) {
    if (rl < sstep) { take(rl + sstep); put(); }
    __syncthreads();
  }
  if (rl == 0 && v < VL) {
    float* dst = part + (long long)blockIdx.y * 2 * C;
#pragma unroll
    for (int u = 0; u < VW; ++u) { dst[v * VW + u] = s1[u]; dst[C + v * VW + u] = s2[u]; }
  }
}

// the slab sums of kFinCB channels per block, 256 / kFinCB lanes per channel (a lane's slab loads all in flight:
// one memory latency, where 4 lanes per channel walked the slabs in ~slabs / 32 dependent rounds), both sums in
// the same pass, lanes combined by a fixed-order LDS tree (deterministic); then per channel: the BN forward
// finalize (fin.mode 1), the BN backward coefficients (2), a direct store (3), or acc += sums (0)
constexpr int kFinCB = 16;
__global__ __launch_bounds__(256) void rows_fin_kernel(const float* part, int slabs, int C, int two, float* acc,
                                                       float* acc2, BnFin fin) {
  constexpr int L = 256 / kFinCB;
  __shared__ float red[2][256];
  const int l = threadIdx.x / kFinCB, el = threadIdx.x % kFinCB;
  const int c = blockIdx.x * kFinCB + el;
  const bool ok = c < C;
  const long long pitch = 2LL * C;
  float v1 = 0.f, v2 = 0.f;
  if (ok) {
#pragma unroll 4
    for (int b = l; b < slabs; b += L) {
      v1 += part[(long long)b * pitch + c];
      if (two) v2 += part[(long long)b * pitch + C + c];
    }
  }
  red[0][threadIdx.x] = v1;
  red[1][threadIdx.x] = v2;
  __syncthreads();
#pragma unroll
  for (int sstep = L / 2; sstep >= 1; sstep /= 2) {
    if (l < sstep) {
      red[0][threadIdx.x] += red[0][threadIdx.x + sstep * kFinCB];
      red[1][threadIdx.x] += red[1][threadIdx.x + sstep * kFinCB];
    }
    __syncthreads();
  }
  if (fin.ctr && blockIdx.x == 0 && threadIdx.x == 0) fin.ctr[0] += 1;
  if (l != 0 || !ok) return;
  const float t1 = red[0][el], t2 = two ? red[1][el] : 0.f;
  if (fin.mode == 1) bn_fwd_fin(fin, c, t1, t2);
  else if (fin.mode == 2) bn_bwd_fin(fin, c, t1, t2);
  else if (fin.mode == 3) rstore(fin.out, fin.out_dt, c, fin.out_scale * (fin.two ? t2 : t1));
  else {
    acc[c] += t1;
    if (two) acc2[c] += t2;
  }
}

int rows_vw(int C) { return C % 8 == 0 ? 8 : 4; }

int rows_tile_vecs(int C) {
  const int VL = C / rows_vw(C), tv = kRowsTileC / rows_vw(C);
  return VL < tv ? VL : tv;
}

int rows_tiles(int C) {
  const int VL = C / rows_vw(C), vt = rows_tile_vecs(C);
  return (VL + vt - 1) / vt;
}

int g_rows_per_lane = 16;   // rows per row lane (tools/bench_rows.py sweeps it through fedmi::rows_tune)

int rows_slabs(long long M, int C) {
  const int RL = 256 / rows_tile_vecs(C);
  const long long tiles = rows_tiles(C);
  const long long per_lane = g_rows_per_lane;
  long long sl = M / ((long long)RL * per_lane);    // >= per_lane rows per row lane
  const long long cap = (2048 + tiles - 1) / tiles;  // ~2048 blocks in flight at most
  if (sl > cap) sl = cap;
  if (sl < 1) sl = 1;
  return (int)sl;
}

// ---- BatchNorm per-channel coefficients --------------------------------------------
// forward (train): from sum(x - shift), sum((x - shift)^2) over M rows:
//   mean, invstd -> save_mean / save_invstd; scale = w * invstd, bias = b - mean * scale;
//   running stats (momentum, unbiased var) updated in place.
// forward (eval): from running stats.
__global__ void bn_fwd_coeffs_kernel(const float* s1, const float* s2, const float* shift, int C, long long M,
                                     const float* w, const float* b, float* rmean, float* rvar, float eps,
                                     float mom, int train, float* save_mean, float* save_invstd, float* scale,
                                     float* bias) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean, inv;
  if (train) {
    const float ms = s1[c] / (float)M;
    const float var = fmaxf(s2[c] / (float)M - ms * ms, 0.f);
    mean = ms + (shift ? shift[c] : 0.f);
    inv = rsqrtf(var + eps);
    if (save_mean) save_mean[c] = mean;
    if (save_invstd) save_invstd[c] = inv;
    if (rmean) {
      rmean[c] = (1.f - mom) * rmean[c] + mom * mean;
      rvar[c] = (1.f - mom) * rvar[c] + mom * var * ((float)M / (float)(M > 1 ? M - 1 : 1));
    }
  } else {
    mean = rmean[c];
    inv = rsqrtf(rvar[c] + eps);
  }
  const float sc = (w ? w[c] : 1.f) * inv;
  scale[c] = sc;
  bias[c] = (b ? b[c] : 0.f) - mean * sc;
}

// backward: from sg = sum g, sgx = sum g * (x - mean):
//   k = w * invstd, dx = g * k + x * bb + cc with bb = -k * invstd^2 * sgx / M, cc = -k * sg / M - bb * mean
__global__ void bn_bwd_coeffs_kernel(const float* sg, const float* sgx, const float* mean, const float* invstd,
                                     const float* w, int C, long long M, float* k, float* bb, float* cc,
                                     float* dw, float* db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = invstd[c];
  const float kk = (w ? w[c] : 1.f) * inv;
  const float b = -kk * inv * inv * sgx[c] / (float)M;
  k[c] = kk;
  bb[c] = b;
  cc[c] = -kk * sg[c] / (float)M - b * mean[c];
  if (dw) dw[c] = sgx[c] * inv;
  if (db) db[c] = sg[c];
}

// ---- pooling (any layout via strides; 4-D [N, C, H, W] logical) ----------------------
struct PoolArgs {
  ZTensor x;    // [N, C, H, W]
  ZTensor y;    // [N, C, P, Q]
  ZTensor idx;  // int64 [N, C, P, Q] (max pool) or p == null
  int kh, kw, sh, sw, ph, pw;
  int count_include_pad;
  int divisor;  // 0: default
};

__global__ __launch_bounds__(256) void pool_fwd_kernel(PoolArgs a, int is_max, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long P = a.y.size[2], Q = a.y.size[3], C = a.y.size[1], H = a.x.size[2], W = a.x.size[3];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    long long t = i;
    const long long q = t % Q; t /= Q;
    const long long p = t % P; t /= P;
    const long long c = t % C; t /= C;
    const long long nn = t;
    const long long h0 = p * a.sh - a.ph, w0 = q * a.sw - a.pw;
    const long long xb = nn * a.x.stride[0] + c * a.x.stride[1];
    float acc = is_max ? -INFINITY : 0.f;
    long long arg = -1;
    int cnt = 0;
    for (int r = 0; r < a.kh; ++r) {
      const long long h = h0 + r;
      for (int s = 0; s < a.kw; ++s) {
        const long long w = w0 + s;
        const bool in = h >= 0 && h < H && w >= 0 && w < W;
        if (is_max) {
          if (in) {
            const float v = zload(a.x, xb + h * a.x.stride[2] + w * a.x.stride[3]);
            if (v > acc || arg < 0 || v != v) { acc = v; arg = h * W + w; }
          }
        } else {
          if (in) acc += zload(a.x, xb + h * a.x.stride[2] + w * a.x.stride[3]);
          // count_include_pad counts the padded window clipped to the padded input
          if (in || (a.count_include_pad && h < H + a.ph && w < W + a.pw)) ++cnt;
        }
      }
    }
    const long long yo = nn * a.y.stride[0] + c * a.y.stride[1] + p * a.y.stride[2] + q * a.y.stride[3];
    if (is_max) {
      zstore(a.y, yo, acc);
      if (a.idx.p)
        reinterpret_cast<long long*>(a.idx.p)[nn * a.idx.stride[0] + c * a.idx.stride[1] + p * a.idx.stride[2] +
                                              q * a.idx.stride[3]] = arg;
    } else {
      const int div = a.divisor ? a.divisor : (cnt > 0 ? cnt : 1);
      zstore(a.y, yo, acc / (float)div);
    }
  }
}

// dx gather: every input element sums the grads of the windows covering it
__global__ __launch_bounds__(256) void pool_bwd_kernel(PoolArgs a, ZTensor dy, int is_max, long long n) {
  // here a.x describes dx (output), dy the incoming grad [N, C, P, Q]
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long P = dy.size[2], Q = dy.size[3], C = a.x.size[1], H = a.x.size[2], W = a.x.size[3];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    long long t = i;
    const long long w = t % W; t /= W;
    const long long h = t % H; t /= H;
    const long long c = t % C; t /= C;
    const long long nn = t;
    // windows p with p*sh - ph <= h < p*sh - ph + kh
    const long long pl = (h + a.ph - a.kh) >= 0 ? (h + a.ph - a.kh) / a.sh + 1 : 0;
    const long long ph_ = (h + a.ph) / a.sh;
    const long long ql = (w + a.pw - a.kw) >= 0 ? (w + a.pw - a.kw) / a.sw + 1 : 0;
    const long long qh = (w + a.pw) / a.sw;
    float acc = 0.f;
    for (long long p = pl; p <= ph_ && p < P; ++p) {
      for (long long q = ql; q <= qh && q < Q; ++q) {
        const long long o = nn * dy.stride[0] + c * dy.stride[1] + p * dy.stride[2] + q * dy.stride[3];
        if (is_max) {
          const long long arg = reinterpret_cast<const long long*>(a.idx.p)[nn * a.idx.stride[0] + c * a.idx.stride[1] +
                                                                            p * a.idx.stride[2] + q * a.idx.stride[3]];
          if (arg == h * W + w) acc += zload(dy, o);
        } else {
          int cnt;
          if (a.divisor) {
            cnt = a.divisor;
          } else {
            const long long hs = p * a.sh - a.ph, ws = q * a.sw - a.pw;
            long long he = hs + a.kh, we = ws + a.kw;
            if (a.count_include_pad) {
              he = he < H + a.ph ? he : H + a.ph;
              we = we < W + a.pw ? we : W + a.pw;
              cnt = (int)((he - hs) * (we - ws));
            } else {
              const long long h0 = hs > 0 ? hs : 0, w0 = ws > 0 ? ws : 0;
              he = he < H ? he : H;
              we = we < W ? we : W;
              cnt = (int)((he - h0) * (we - w0));
            }
          }
          acc += zload(dy, o) / (float)(cnt > 0 ? cnt : 1);
        }
      }
    }
    zstore(a.x, nn * a.x.stride[0] + c * a.x.stride[1] + h * a.x.stride[2] + w * a.x.stride[3], acc);
  }
}

// ---- small GEMM: C[M,N] = alpha * A[M,K] B[K,N] + beta * bias (broadcast over rows) ------
// 16 x 16 output tile per 256-thread block, K in LDS chunks of 16; fp32 accumulate.
__global__ __launch_bounds__(256) void gemm_kernel(ZTensor A, ZTensor B, ZTensor Cm, ZTensor bias, float alpha,
                                                   float beta) {
  __shared__ float as[16][17], bs[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const long long M = Cm.size[0], N = Cm.size[1], K = A.size[1];
  const long long row = (long long)blockIdx.y * 16 + ty, col = (long long)blockIdx.x * 16 + tx;
  float acc = 0.f;
  for (long long k0 = 0; k0 < K; k0 += 16) {
    const long long ka = k0 + tx, kb = k0 + ty;
    const long long ar = (long long)blockIdx.y * 16 + ty, bc = (long long)blockIdx.x * 16 + tx;
    as[ty][tx] = (ar < M && ka < K) ? zload(A, ar * A.stride[0] + ka * A.stride[1]) : 0.f;
    bs[ty][tx] = (kb < K && bc < N) ? zload(B, kb * B.stride[0] + bc * B.stride[1]) : 0.f;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) acc += as[ty][kk] * bs[kk][tx];
    __syncthreads();
  }
  if (row < M && col < N) {
    float v = alpha * acc;
    if (bias.p) v += beta * zload(bias, (bias.ndim == 2 ? row * bias.stride[0] : 0) + col * bias.stride[bias.ndim - 1]);
    zstore(Cm, row * Cm.stride[0] + col * Cm.stride[1], v);
  }
}

// ---- bf16 GEMM on MFMA: C[M,N] = alpha * A[M,K] B[K,N] + beta * bias --------------------
// 64 x 64 output tile per 256-thread workgroup, each wave a 32 x 32 quadrant of 2 x 2
// v_mfma_f32_16x16x32_bf16 tiles; K in steps of 32 staged through LDS with any operand strides
// (the aten mm operands are often transposed views), both tiles stored k-contiguous so every
// fragment is one 16-byte ds_read.  Used when both operands are bf16 (autocast linear layers and
// their backward); fp32 operands keep the exact-fp32 gemm_kernel above.
constexpr int kGmPitch = 40;   // bf16 per LDS row: 32 + 8 pad (80 B rows: 16-B aligned, bank-spread)

__global__ __launch_bounds__(256) void gemm_mfma_kernel(ZTensor A, ZTensor B, ZTensor Cm, ZTensor bias, float alpha,
                                                        float beta) {
  __shared__ __attribute__((aligned(16))) bf16 as[64 * kGmPitch];
  __shared__ __attribute__((aligned(16))) bf16 bs[64 * kGmPitch];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const long long M = Cm.size[0], N = Cm.size[1], K = A.size[1];
  const long long m0 = (long long)blockIdx.y * 64, n0 = (long long)blockIdx.x * 64;
  const bf16* Ap = reinterpret_cast<const bf16*>(A.p);
  const bf16* Bp = reinterpret_cast<const bf16*>(B.p);
  const int lr = t >> 2, lk = (t & 3) * 8;      // loader: tile row / column lr, 8 consecutive k
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
  for (long long k0 = 0; k0 < K; k0 += 32) {
    bf16x8 va, vb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long long k = k0 + lk + e, m = m0 + lr, n = n0 + lr;
      va[e] = (m < M && k < K) ? Ap[m * A.stride[0] + k * A.stride[1]] : (bf16)0.f;
      vb[e] = (n < N && k < K) ? Bp[k * B.stride[0] + n * B.stride[1]] : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(as + lr * kGmPitch + lk) = va;
    *reinterpret_cast<bf16x8*>(bs + lr * kGmPitch + lk) = vb;
    __syncthreads();
    const int fr = lane & 15, fk = (lane >> 4) * 8;
    bf16x8 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(as + (wm + i * 16 + fr) * kGmPitch + fk);
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(bs + (wn + j * 16 + fr) * kGmPitch + fk);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    __syncthreads();
  }
  // 16x16x32 result layout: lane holds rows 4 * (lane / 16) + r of column lane % 16
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long row = m0 + wm + i * 16 + (lane >> 4) * 4 + r, col = n0 + wn + j * 16 + (lane & 15);
        if (row < M && col < N) {
          float v = alpha * acc[i][j][r];
          if (bias.p)
            v += beta * zload(bias, (bias.ndim == 2 ? row * bias.stride[0] : 0) + col * bias.stride[bias.ndim - 1]);
          zstore(Cm, row * Cm.stride[0] + col * Cm.stride[1], v);
        }
      }
}

// ---- log_softmax over dim 1 of a 2-D tensor; NLL loss (mean, ignore_index) -------------
__global__ void log_softmax_kernel(ZTensor x, ZTensor y, int bwd, ZTensor gy) {
  // fwd: y = x - logsumexp(x); bwd (x = output of fwd): y = gy - exp(x) * sum(gy)
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= x.size[0]) return;
  const long long J = x.size[1];
  if (!bwd) {
    float mx = -INFINITY;
    for (long long j = 0; j < J; ++j) mx = fmaxf(mx, zload(x, r * x.stride[0] + j * x.stride[1]));
    float se = 0.f;
    for (long long j = 0; j < J; ++j) se += __expf(zload(x, r * x.stride[0] + j * x.stride[1]) - mx);
    const float lse = mx + __logf(se);
    for (long long j = 0; j < J; ++j) zstore(y, r * y.stride[0] + j * y.stride[1], zload(x, r * x.stride[0] + j * x.stride[1]) - lse);
  } else {
    float sg = 0.f;
    for (long long j = 0; j < J; ++j) sg += zload(gy, r * gy.stride[0] + j * gy.stride[1]);
    for (long long j = 0; j < J; ++j)
      zstore(y, r * y.stride[0] + j * y.stride[1],
             zload(gy, r * gy.stride[0] + j * gy.stride[1]) - __expf(zload(x, r * x.stride[0] + j * x.stride[1])) * sg);
  }
}

// nll fwd: out = -sum_r lp[r][t_r] / n_valid ; total_weight = n_valid.  One workgroup.
__global__ __launch_bounds__(256) void nll_fwd_kernel(ZTensor lp, const long long* tgt, long long tstride,
                                                      int ignore, int reduction_mean, float* out_f32, bf16* out_bf16,
                                                      float* tw_f32, bf16* tw_bf16) {
  __shared__ float sl[256], sc[256];
  float l = 0.f, c = 0.f;
  for (long long r = threadIdx.x; r < lp.size[0]; r += 256) {
    const long long t = tgt[r * tstride];
    if (t != ignore) { l -= zload(lp, r * lp.stride[0] + t * lp.stride[1]); c += 1.f; }
  }
  sl[threadIdx.x] = l; sc[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) { sl[threadIdx.x] += sl[threadIdx.x + s]; sc[threadIdx.x] += sc[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float v = reduction_mean ? sl[0] / fmaxf(sc[0], 1.f) : sl[0];
    if (out_f32) *out_f32 = v; else *out_bf16 = (bf16)v;
    if (tw_f32) *tw_f32 = sc[0]; else if (tw_bf16) *tw_bf16 = (bf16)sc[0];
  }
}

// nll bwd: gx[r][j] = (j == t_r) ? -g / total_weight : 0   (mean); -g (sum)
__global__ void nll_bwd_kernel(ZTensor gx, const float* g, const float* tw, const long long* tgt, long long tstride,
                               int ignore, int reduction_mean, int g_bf16, int tw_bf16) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= gx.size[0]) return;
  const float gv = g_bf16 ? (float)*reinterpret_cast<const bf16*>(g) : *g;
  const float twv = tw_bf16 ? (float)*reinterpret_cast<const bf16*>(tw) : *tw;
  const long long t = tgt[r * tstride];
  const float v = reduction_mean ? -gv / fmaxf(twv, 1.f) : -gv;
  for (long long j = 0; j < gx.size[1]; ++j) zstore(gx, r * gx.stride[0] + j * gx.stride[1], (t != ignore && j == t) ? v : 0.f);
}

// training statistics of a classifier output: loss_sum += CE, correct += argmax == y, count += n
__global__ __launch_bounds__(256) void ce_stats_kernel(ZTensor logits, const long long* y, float* stats) {
  __shared__ float sl[256], sc[256];
  float l = 0.f, c = 0.f;
  const long long J = logits.size[1];
  for (long long r = threadIdx.x; r < logits.size[0]; r += 256) {
    float mx = -INFINITY;
    long long am = 0;
    for (long long j = 0; j < J; ++j) {
      const float v = zload(logits, r * logits.stride[0] + j * logits.stride[1]);
      if (v > mx) { mx = v; am = j; }
    }
    float se = 0.f;
    for (long long j = 0; j < J; ++j) se += __expf(zload(logits, r * logits.stride[0] + j * logits.stride[1]) - mx);
    const long long t = y[r];
    l += mx + __logf(se) - zload(logits, r * logits.stride[0] + t * logits.stride[1]);
    c += (am == t) ? 1.f : 0.f;
  }
  sl[threadIdx.x] = l; sc[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) { sl[threadIdx.x] += sl[threadIdx.x + s]; sc[threadIdx.x] += sc[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[0] += sl[0];
    stats[1] += sc[0];
    stats[2] += (float)logits.size[0];
  }
}

// ---- direct (VALU) grouped convolution, any channel counts ---------------------------
// x [N, C, H, W], w [O, C/G, R, S], y [N, O, P, Q] -- logical NCHW, any strides (channels-last in
// practice).  Grouped convs with narrow groups (RegNet group width 8, DPN / ResNeXt cardinality 32,
// ShuffleNet g2/g3 widths) and odd channel counts have no MFMA-shaped tile; they run here.
// FWD: a thread owns one output pixel x GT output channels of one group; the (group, channel
// chunk)'s weights sit in LDS as [r*S+s][c][GT] and are read as wave-wide broadcasts, the input
// channels of a tap are contiguous (channels-last), so each tap costs one cached load per channel
// and GT FMAs.  DGRAD: the same with the roles of x and y swapped (one input pixel x GT input
// channels).  WGRAD: a thread owns weights (o, r, s, c) with c fastest -- neighbouring lanes read
// neighbouring channels of the same pixel (coalesced) and share the dy value (broadcast) -- and
// sums over the pixels of an image slab; per-slab partials go to a workspace and a second pass
// adds them in slab order (deterministic, no atomics).
constexpr int GT = 8;          // output (FWD) / input (DGRAD) channels per thread
constexpr int GC_LDS = 8192;   // floats of LDS for a weight chunk (32 KiB)

struct GConv {
  ZTensor x, w, y;
  int G, st_h, st_w, pad_h, pad_w, R, S;
  int vec_x, vec_y;    // channels of x (resp. y) load as aligned bf16x8 vectors (host-checked)
};

FEDMI_DEV void load8(const ZTensor& t, long long off, long long cstride, bool vec, float v[8]) {
  if (vec) {
    const bf16x8 q = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(t.p) + off);
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (float)q[u];
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = zload(t, off + u * cstride);
  }
}

__global__ __launch_bounds__(256) void gconv_fwd_kernel(GConv g) {
  __shared__ float wl[GC_LDS];
  const long long N = g.y.size[0], O = g.y.size[1], P = g.y.size[2], Q = g.y.size[3];
  const long long H = g.x.size[2], W = g.x.size[3];
  const int Cg = (int)g.w.size[1], Og = (int)(O / g.G), RS = g.R * g.S;
  const int grp = blockIdx.y, o0 = blockIdx.z * GT;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  const bool valid = pix < N * P * Q;
  long long t = valid ? pix : 0;
  const long long q = t % Q; t /= Q;
  const long long p = t % P;
  const long long n = t / P;
  float acc[GT];
#pragma unroll
  for (int j = 0; j < GT; ++j) acc[j] = 0.f;
  const int cch = max(8, GC_LDS / (RS * GT) / 8 * 8);
  const long long xb = n * g.x.stride[0] + (long long)grp * Cg * g.x.stride[1];
  for (int c0 = 0; c0 < Cg; c0 += cch) {
    const int cn = min(cch, Cg - c0);
    __syncthreads();
    for (int e = threadIdx.x; e < RS * cn * GT; e += 256) {
      const int j = e % GT, c = (e / GT) % cn, rs = e / (GT * cn);
      const int o = o0 + j;
      wl[e] = o < Og ? zload(g.w, (long long)(grp * Og + o) * g.w.stride[0] + (long long)(c0 + c) * g.w.stride[1] +
                                      (rs / g.S) * g.w.stride[2] + (rs % g.S) * g.w.stride[3])
                     : 0.f;
    }
    __syncthreads();
    if (!valid) continue;
    if (g.R == 3 && g.S == 3 && g.vec_x && g.x.dtype == 1 && cn % 8 == 0) {
      // 3x3, bf16 channels-last: per 8-channel group the nine tap vectors are loaded together (clamped
      // addresses, 0/1 masks), then the FMAs -- one memory latency per group instead of one per tap
      const bf16* xp = reinterpret_cast<const bf16*>(g.x.p);
      long long toff[9];
      float tok[9];
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const long long h = p * g.st_h - g.pad_h + tp / 3, w = q * g.st_w - g.pad_w + tp % 3;
        const bool ok = h >= 0 && h < H && w >= 0 && w < W;
        tok[tp] = ok ? 1.f : 0.f;
        toff[tp] = xb + (ok ? h * g.x.stride[2] + w * g.x.stride[3] : 0) + (long long)c0;
      }
      for (int c = 0; c < cn; c += 8) {
        bf16x8 xq[9];
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) xq[tp] = *reinterpret_cast<const bf16x8*>(xp + toff[tp] + c);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const float* wr = wl + tp * cn * GT;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float xv = tok[tp] * (float)xq[tp][u];
#pragma unroll
            for (int j = 0; j < GT; ++j) acc[j] += xv * wr[(c + u) * GT + j];
          }
        }
      }
      continue;
    }
    // general path, in the fast path's accumulation order (8-channel group, then tap, then channel): the sums
    // do not depend on which path a layout takes
    for (int c = 0; c < cn; c += 8) {
      const int cw = min(8, cn - c);
      for (int r = 0; r < g.R; ++r) {
        const long long h = p * g.st_h - g.pad_h + r;
        if (h < 0 || h >= H) continue;
        for (int s = 0; s < g.S; ++s) {
          const long long w = q * g.st_w - g.pad_w + s;
          if (w < 0 || w >= W) continue;
          const long long base = xb + h * g.x.stride[2] + w * g.x.stride[3] + (long long)(c0 + c) * g.x.stride[1];
          const float* wr = wl + (r * g.S + s) * cn * GT;
          float xv[8];
          if (g.vec_x && cw == 8) {
            load8(g.x, base, 1, true, xv);
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) xv[u] = u < cw ? zload(g.x, base + (long long)u * g.x.stride[1]) : 0.f;
          }
          for (int u = 0; u < cw; ++u)
#pragma unroll
            for (int j = 0; j < GT; ++j) acc[j] += xv[u] * wr[(c + u) * GT + j];
        }
      }
    }
  }
  if (!valid) return;
  const long long yb = n * g.y.stride[0] + p * g.y.stride[2] + q * g.y.stride[3];
#pragma unroll
  for (int j = 0; j < GT; ++j)
    if (o0 + j < Og) zstore(g.y, yb + (long long)(grp * Og + o0 + j) * g.y.stride[1], acc[j]);
}

// g.x = dx (output), g.y = dy (input)
__global__ __launch_bounds__(256) void gconv_dgrad_kernel(GConv g) {
  __shared__ float wl[GC_LDS];
  const long long N = g.x.size[0], H = g.x.size[2], W = g.x.size[3];
  const long long O = g.y.size[1], P = g.y.size[2], Q = g.y.size[3];
  const int Cg = (int)g.w.size[1], Og = (int)(O / g.G), RS = g.R * g.S;
  const int grp = blockIdx.y, c0 = blockIdx.z * GT;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  const bool valid = pix < N * H * W;
  long long t = valid ? pix : 0;
  const long long w = t % W; t /= W;
  const long long h = t % H;
  const long long n = t / H;
  float acc[GT];
#pragma unroll
  for (int j = 0; j < GT; ++j) acc[j] = 0.f;
  const int och = max(8, GC_LDS / (RS * GT) / 8 * 8);
  const long long yb = n * g.y.stride[0] + (long long)grp * Og * g.y.stride[1];
  for (int o0 = 0; o0 < Og; o0 += och) {
    const int on = min(och, Og - o0);
    __syncthreads();
    for (int e = threadIdx.x; e < RS * on * GT; e += 256) {
      const int j = e % GT, o = (e / GT) % on, rs = e / (GT * on);
      const int c = c0 + j;
      wl[e] = c < Cg ? zload(g.w, (long long)(grp * Og + o0 + o) * g.w.stride[0] + (long long)c * g.w.stride[1] +
                                      (rs / g.S) * g.w.stride[2] + (rs % g.S) * g.w.stride[3])
                     : 0.f;
    }
    __syncthreads();
    if (!valid) continue;
    if (g.R == 3 && g.S == 3 && g.vec_y && g.y.dtype == 1 && on % 8 == 0) {
      // 3x3, bf16 channels-last dy: the nine tap vectors of an 8-channel group loaded together (see fwd)
      const bf16* yp = reinterpret_cast<const bf16*>(g.y.p);
      long long toff[9];
      float tok[9];
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const long long hp = h + g.pad_h - tp / 3, wp = w + g.pad_w - tp % 3;
        const bool okd = hp >= 0 && wp >= 0 && hp % g.st_h == 0 && wp % g.st_w == 0;
        const long long p = okd ? hp / g.st_h : 0, q = okd ? wp / g.st_w : 0;
        const bool ok = okd && p < P && q < Q;
        tok[tp] = ok ? 1.f : 0.f;
        toff[tp] = yb + (ok ? p * g.y.stride[2] + q * g.y.stride[3] : 0) + (long long)o0;
      }
      for (int o = 0; o < on; o += 8) {
        bf16x8 yq[9];
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) yq[tp] = *reinterpret_cast<const bf16x8*>(yp + toff[tp] + o);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const float* wr = wl + tp * on * GT;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float dv = tok[tp] * (float)yq[tp][u];
#pragma unroll
            for (int j = 0; j < GT; ++j) acc[j] += dv * wr[(o + u) * GT + j];
          }
        }
      }
      continue;
    }
    // general path in the fast path's order (8-channel group, tap, channel), as in gconv_fwd_kernel
    for (int o = 0; o < on; o += 8) {
      const int ow = min(8, on - o);
      for (int r = 0; r < g.R; ++r) {
        const long long hp = h + g.pad_h - r;
        if (hp < 0 || hp % g.st_h) continue;
        const long long p = hp / g.st_h;
        if (p >= P) continue;
        for (int s = 0; s < g.S; ++s) {
          const long long wp = w + g.pad_w - s;
          if (wp < 0 || wp % g.st_w) continue;
          const long long q = wp / g.st_w;
          if (q >= Q) continue;
          const long long base = yb + p * g.y.stride[2] + q * g.y.stride[3] + (long long)(o0 + o) * g.y.stride[1];
          const float* wr = wl + (r * g.S + s) * on * GT;
          float dv[8];
          if (g.vec_y && ow == 8) {
            load8(g.y, base, 1, true, dv);
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) dv[u] = u < ow ? zload(g.y, base + (long long)u * g.y.stride[1]) : 0.f;
          }
          for (int u = 0; u < ow; ++u)
#pragma unroll
            for (int j = 0; j < GT; ++j) acc[j] += dv[u] * wr[(o + u) * GT + j];
        }
      }
    }
  }
  if (!valid) return;
  const long long xo = n * g.x.stride[0] + h * g.x.stride[2] + w * g.x.stride[3];
#pragma unroll
  for (int j = 0; j < GT; ++j)
    if (c0 + j < Cg) zstore(g.x, xo + (long long)(grp * Cg + c0 + j) * g.x.stride[1], acc[j]);
}

// partial[slab][O][Cg][R][S] = sum over the output rows [slab*rps, +rps) of the flattened (n, p)
// space.  A thread owns one (o, r, s) and 8 consecutive input channels of o's group (one bf16x8 load
// per pixel when x is channels-last); blocks tile the flattened (o, rs, channel block) space of ALL
// groups, grid.y = row slabs -- enough lanes in flight even for 8-wide groups.
__global__ __launch_bounds__(256) void gconv_wgrad_kernel(GConv g, float* part, int rps) {
  const long long N = g.x.size[0], H = g.x.size[2], W = g.x.size[3];
  const long long O = g.y.size[1], P = g.y.size[2], Q = g.y.size[3];
  const int Cg = (int)g.w.size[1], Og = (int)(O / g.G), RS = g.R * g.S;
  const int CB = (Cg + 7) / 8;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= O * RS * CB) return;
  // e = (og * RS + rs) * CB + cb, og = the global output channel
  const int cb = (int)(e % CB);
  const int rs = (int)((e / CB) % RS);
  const int og = (int)(e / ((long long)CB * RS));
  const int grp = og / Og;
  const int r = rs / g.S, s = rs % g.S;
  const int c0 = cb * 8, cn = min(8, Cg - c0);
  const bool vec = g.vec_x && cn == 8;
  const long long xc = (long long)(grp * Cg + c0) * g.x.stride[1];
  const long long yc = (long long)og * g.y.stride[1];
  const long long row0 = (long long)blockIdx.y * rps, row1 = min(N * P, row0 + rps);
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
  if (vec && g.y.dtype == 1) {
    // bf16 channels-last fast path: 8 output columns per pass, all 16 loads (8 dy scalars, 8 x vectors)
    // issued before the first use -- clamped addresses and a 0/1 mask instead of per-load branches, so the
    // pass costs one memory latency (the scalar loop paid one per pixel: ~300 us per RegNetY launch)
    const bf16* yp = reinterpret_cast<const bf16*>(g.y.p);
    const bf16* xp = reinterpret_cast<const bf16*>(g.x.p);
    const long long ys3 = g.y.stride[3], xs3 = g.x.stride[3];
    for (long long row = row0; row < row1; ++row) {
      const long long n = row / P, p = row - n * P;
      const long long h = p * g.st_h - g.pad_h + r;
      if (h < 0 || h >= H) continue;
      const long long xr = n * g.x.stride[0] + h * g.x.stride[2] + xc;
      const long long yr = n * g.y.stride[0] + p * g.y.stride[2] + yc;
      for (long long q0 = 0; q0 < Q; q0 += 8) {
        bf16 dq[8];
        bf16x8 xq[8];
        float okm[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const long long q = q0 + k, w = q * g.st_w - g.pad_w + s;
          const bool ok = q < Q && w >= 0 && w < W;
          okm[k] = ok ? 1.f : 0.f;
          dq[k] = yp[yr + (ok ? q : 0) * ys3];
          xq[k] = *reinterpret_cast<const bf16x8*>(xp + xr + (ok ? w : 0) * xs3);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dv = okm[k] * (float)dq[k];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc[u] += dv * (float)xq[k][u];
        }
      }
    }
  } else
  for (long long row = row0; row < row1; ++row) {
    const long long n = row / P, p = row - n * P;
    const long long h = p * g.st_h - g.pad_h + r;
    if (h < 0 || h >= H) continue;
    const long long xr = n * g.x.stride[0] + h * g.x.stride[2] + xc;
    const long long yr = n * g.y.stride[0] + p * g.y.stride[2] + yc;
    for (long long q = 0; q < Q; ++q) {
      const long long w = q * g.st_w - g.pad_w + s;
      if (w < 0 || w >= W) continue;
      const float dv = zload(g.y, yr + q * g.y.stride[3]);
      float xv[8];
      if (vec) {
        load8(g.x, xr + w * g.x.stride[3], 1, true, xv);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) xv[u] = u < cn ? zload(g.x, xr + w * g.x.stride[3] + u * g.x.stride[1]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += dv * xv[u];
    }
  }
  float* dst = part + (long long)blockIdx.y * O * Cg * RS;
  for (int u = 0; u < cn; ++u) dst[((long long)og * Cg + c0 + u) * RS + rs] = acc[u];
}

// dw[i] = sum_slab part[slab][i] (dw: any strides over the contiguous [O, Cg, R, S] order)
__global__ __launch_bounds__(256) void gconv_wgrad_sum_kernel(const float* part, int slabs, long long total,
                                                              ZTensor dw) {
  const long long i = (long long)blockIdx.x * 64 + (threadIdx.x & 63);
  const float v = ordered_slab_sum(part, slabs, total, i, i < total);
  if ((threadIdx.x >> 6) || i >= total) return;
  const long long RS = dw.size[2] * dw.size[3], Cg = dw.size[1];
  const long long rs = i % RS, c = (i / RS) % Cg, o = i / (RS * Cg);
  zstore(dw, o * dw.stride[0] + c * dw.stride[1] + (rs / dw.size[3]) * dw.stride[2] + (rs % dw.size[3]) * dw.stride[3], v);
}

// output rows per wgrad slab (>= ~256 pixels per thread) and the slab count, with the partials
// capped at 8M floats
void gconv_slabs(long long N, long long P, long long Q, long long total, long long* rps, long long* slabs) {
  const long long rows = N * P > 0 ? N * P : 1;
  long long r = (256 + Q - 1) / (Q > 0 ? Q : 1);
  if (r < 1) r = 1;
  long long sl = (rows + r - 1) / r;
  const long long cap = total > 0 ? (8LL << 20) / total : 1;
  if (sl > cap) sl = cap > 0 ? cap : 1;
  if (sl > 65535) sl = 65535;
  r = (rows + sl - 1) / sl;
  *rps = r;
  *slabs = (rows + r - 1) / r;
}

int grid1(long long n) {
  long long b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (int)b;
}

}  // namespace

namespace fedmi {

template <int NIN>
static void launch_ew_n(hipStream_t st, const ZTensor& o, const ZTensor* ins, int nin, int op, float s0, float s1,
                        uint32_t seed, const int* ctr, int vmask, int vw) {
  EwArgs<NIN> a{};
  a.o = o;
  for (int i = 0; i < nin; ++i) a.in[i] = ins[i];
  a.op = op;
  a.s0 = s0;
  a.s1 = s1;
  a.seed = seed;
  a.ctr = ctr;
  a.vmask = vmask < 0 ? 0 : vmask;
  long long n = 1;
  for (int d = 0; d < o.ndim; ++d) n *= o.size[d];
  if (n <= 0) return;
  if (vmask >= 0) {
    if (op == EW_BERN) throw std::invalid_argument("ew: no vector launch for bernoulli");
    if (vw == 8)
      hipLaunchKernelGGL((ew_vec_kernel<8, NIN>), dim3(grid1(n)), dim3(256), 0, st, a, n);
    else if (vw == 4)
      hipLaunchKernelGGL((ew_vec_kernel<4, NIN>), dim3(grid1(n)), dim3(256), 0, st, a, n);
    else
      throw std::invalid_argument("ew: vector width 8 or 4");
  } else {
    hipLaunchKernelGGL(ew_kernel<NIN>, dim3(grid1(n)), dim3(256), 0, st, a, n);
  }
}

void launch_ew(hipStream_t st, const ZTensor& o, const ZTensor* ins, int nin, int op, float s0, float s1,
               uint32_t seed, const int* ctr, int vmask, int vw) {
  if (nin > 7) throw std::invalid_argument("ew: at most 7 inputs");
  if (nin > 6)
    launch_ew_n<7>(st, o, ins, nin, op, s0, s1, seed, ctr, vmask, vw);
  else
    launch_ew_n<6>(st, o, ins, nin, op, s0, s1, seed, ctr, vmask, vw);
  check_hip(hipGetLastError(), "ew_kernel");
}

void launch_ctr_bump(hipStream_t st, int* ctr) {
  hipLaunchKernelGGL(ctr_bump_kernel, dim3(1), dim3(64), 0, st, ctr);
}

static long long reduce_splits(long long no, long long ni) {
  const long long tiles = (no + 63) / 64;
  long long splits = (1024 + tiles - 1) / tiles;             // ~1024 workgroups in flight
  const long long max_split = (ni + 255) / 256;              // >= 64 inner elements per lane group
  if (splits > max_split) splits = max_split;
  if (splits > 256) splits = 256;                            // bounds the partials workspace
  if (splits < 1) splits = 1;
  return splits;
}

long long reduce_ws_floats(long long no, long long ni) {
  const long long sp = reduce_splits(no, ni);
  return sp > 1 ? 2 * sp * no : 0;
}

void launch_reduce(hipStream_t st, const ZTensor& outer, const ZTensor& inner, const ZTensor& outer_b,
                   const ZTensor& inner_b, const void* a, int a_dt, const void* b, int b_dt, const float* shift,
                   float* acc, float* acc2, int op, float* part, long long part_floats, void* out, int out_dt,
                   float scale) {
  if (out && op == RD_SUMSQ_SHIFT) throw std::invalid_argument("launch_reduce: no direct output of moments");
  long long no = 1, ni = 1;
  for (int d = 0; d < outer.ndim; ++d) no *= outer.size[d];
  for (int d = 0; d < inner.ndim; ++d) ni *= inner.size[d];
  if (no <= 0) return;
  RdArgs r{};
  r.outer = outer; r.inner = inner; r.outer_b = outer_b; r.inner_b = inner_b;
  r.a = a; r.a_dtype = a_dt; r.b = b; r.b_dtype = b_dt; r.shift = shift; r.acc = acc; r.acc2 = acc2; r.op = op;
  r.part = part; r.out = out; r.out_dt = out_dt; r.scale = scale;
  const long long tiles = (no + 63) / 64;
  const long long splits = reduce_splits(no, ni);
  if (splits > 1 && (part == nullptr || part_floats < 2 * splits * no))
    throw std::invalid_argument("launch_reduce: partials workspace too small");
  hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)tiles, (unsigned)splits), dim3(256), 0, st, r, no, ni);
  check_hip(hipGetLastError(), "reduce_kernel");
  if (splits > 1) {
    hipLaunchKernelGGL(reduce_splits_kernel, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, st, part, (int)splits,
                       no, acc, op != RD_SUM ? acc2 : nullptr, out, out_dt, scale, op != RD_SUM ? 1 : 0);
    check_hip(hipGetLastError(), "reduce_splits_kernel");
  }
}

void launch_pad_rows(hipStream_t st, const bf16* src, long long lds, int C, bf16* dst, int C8, long long rows) {
  if (C8 % 8 || C > C8 || C <= 0 || lds < C || rows <= 0) throw std::invalid_argument("pad_rows: bad shape");
  const int vec = (reinterpret_cast<uintptr_t>(src) % 16 == 0 && lds % 8 == 0) ? 1 : 0;
  const long long n = rows * (C8 / 8);
  const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(pad_rows_kernel, dim3(blocks), dim3(256), 0, st, src, lds, C, dst, C8, rows, vec);
  check_hip(hipGetLastError(), "pad_rows");
}

long long reduce_rows_ws_floats(long long M, int C) { return (long long)rows_slabs(M, C) * 2 * C; }

int rows_tune(int per_lane) {
  const int prev = g_rows_per_lane;
  if (per_lane > 0) g_rows_per_lane = per_lane;
  return prev;
}

// phase 1 (row slabs -> part) + rows_fin_kernel (slab sums -> fin / out / acc)
static void rows_launch(hipStream_t st, const void* a, int a_dt, long long lda, const void* b, int b_dt, long long ldb,
                        const float* shift, int C, long long M, int op, float* part, long long part_floats,
                        const void* f, int f_dt, long long ldf, float thr, float* acc, float* acc2, const BnFin& fin,
                        const char* what) {
  if (C % 4 || C <= 0 || M <= 0) throw std::invalid_argument(std::string(what) + ": C % 4 == 0 and M > 0 required");
  const int slabs = rows_slabs(M, C);
  if (part_floats < reduce_rows_ws_floats(M, C)) throw std::invalid_argument(std::string(what) + ": workspace too small");
  const dim3 grid((unsigned)rows_tiles(C), (unsigned)slabs);
  if (rows_vw(C) == 8)
    hipLaunchKernelGGL(reduce_rows_kernel<8>, grid, dim3(256), 0, st, a, a_dt, lda, b, b_dt, ldb, shift, C, M, op, part,
                       f, f_dt, ldf, thr);
  else
    hipLaunchKernelGGL(reduce_rows_kernel<4>, grid, dim3(256), 0, st, a, a_dt, lda, b, b_dt, ldb, shift, C, M, op, part,
                       f, f_dt, ldf, thr);
  hipLaunchKernelGGL(rows_fin_kernel, dim3((unsigned)((C + kFinCB - 1) / kFinCB)), dim3(256), 0, st, part, slabs, C,
                     op != RD_SUM ? 1 : 0, acc, acc2, fin);
  check_hip(hipGetLastError(), what);
}

void launch_reduce_rows(hipStream_t st, const void* a, int a_dt, long long lda, const void* b, int b_dt,
                        long long ldb, const float* shift, int C, long long M, int op, float* part, long long part_floats,
                        float* acc, float* acc2, void* out, int out_dt, float scale) {
  if (out && op == RD_SUMSQ_SHIFT) throw std::invalid_argument("reduce_rows: no direct output of moments");
  BnFin fin{};
  if (out) {   // the sums stored directly: no zeroed accumulator, no copy
    fin.mode = 3; fin.out = out; fin.out_dt = out_dt; fin.out_scale = scale; fin.two = op != RD_SUM;
  }
  rows_launch(st, a, a_dt, lda, b, b_dt, ldb, shift, C, M, op, part, part_floats, nullptr, 0, 0LL, 0.f, acc, acc2, fin,
              "reduce_rows");
}

// BN forward statistics + coefficients of a channels-last [M, C] activation
void launch_bn_rows_fwd(hipStream_t st, const void* x, int x_dt, long long ldx, const float* shift, int C, long long M,
                        float* part, long long part_floats, const float* w, const float* b, float* rmean, float* rvar,
                        float eps, float mom, float* save_mean, float* save_invstd, float* scale, float* bias,
                        long long* ctr) {
  BnFin fin{};
  fin.mode = 1; fin.M = M; fin.shift = shift; fin.w = w; fin.b = b; fin.rmean = rmean; fin.rvar = rvar;
  fin.eps = eps; fin.mom = mom; fin.save_mean = save_mean; fin.save_invstd = save_invstd; fin.scale = scale;
  fin.bias = bias; fin.ctr = ctr;
  rows_launch(st, x, x_dt, ldx, nullptr, 0, 0LL, shift, C, M, (int)RD_SUMSQ_SHIFT, part, part_floats, nullptr, 0, 0LL,
              0.f, nullptr, nullptr, fin, "bn_rows_fwd");
}

// BN backward sums + coefficients; f (optional): the ReLU output whose threshold_backward is fused in
void launch_bn_rows_bwd(hipStream_t st, const void* g, int g_dt, long long ldg, const void* x, int x_dt, long long ldx,
                        const void* f, int f_dt, long long ldf, float thr, const float* mean, const float* invstd,
                        const float* w, int C, long long M, float* part, long long part_floats, float* k, float* bb,
                        float* cc, float* dw, float* db) {
  BnFin fin{};
  fin.mode = 2; fin.M = M; fin.mean = mean; fin.invstd = invstd; fin.w = w; fin.k = k; fin.bb = bb; fin.cc = cc;
  fin.dw = dw; fin.db = db;
  rows_launch(st, g, g_dt, ldg, x, x_dt, ldx, mean, C, M, (int)RD_DOT_SHIFT, part, part_floats, f, f_dt, ldf, thr,
              nullptr, nullptr, fin, "bn_rows_bwd");
}

void launch_bn_fwd_coeffs(hipStream_t st, const float* s1, const float* s2, const float* shift, int C, long long M,
                          const float* w, const float* b, float* rmean, float* rvar, float eps, float mom, int train,
                          float* save_mean, float* save_invstd, float* scale, float* bias) {
  hipLaunchKernelGGL(bn_fwd_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, st, s1, s2, shift, C, M, w, b, rmean,
                     rvar, eps, mom, train, save_mean, save_invstd, scale, bias);
  check_hip(hipGetLastError(), "bn_fwd_coeffs");
}

void launch_bn_bwd_coeffs(hipStream_t st, const float* sg, const float* sgx, const float* mean, const float* invstd,
                          const float* w, int C, long long M, float* k, float* bb, float* cc, float* dw, float* db) {
  hipLaunchKernelGGL(bn_bwd_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, st, sg, sgx, mean, invstd, w, C, M, k,
                     bb, cc, dw, db);
  check_hip(hipGetLastError(), "bn_bwd_coeffs");
}

void launch_pool_fwd(hipStream_t st, const ZTensor& x, const ZTensor& y, const ZTensor& idx, int kh, int kw, int sh,
                     int sw, int ph, int pw, int count_include_pad, int divisor, int is_max) {
  PoolArgs a{};
  a.x = x; a.y = y; a.idx = idx; a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.count_include_pad = count_include_pad; a.divisor = divisor;
  long long n = y.size[0] * y.size[1] * y.size[2] * y.size[3];
  if (n <= 0) return;
  hipLaunchKernelGGL(pool_fwd_kernel, dim3(grid1(n)), dim3(256), 0, st, a, is_max, n);
  check_hip(hipGetLastError(), "pool_fwd");
}

void launch_pool_bwd(hipStream_t st, const ZTensor& dx, const ZTensor& dy, const ZTensor& idx, int kh, int kw, int sh,
                     int sw, int ph, int pw, int count_include_pad, int divisor, int is_max) {
  PoolArgs a{};
  a.x = dx; a.idx = idx; a.kh = kh; a.kw = kw; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.count_include_pad = count_include_pad; a.divisor = divisor;
  long long n = dx.size[0] * dx.size[1] * dx.size[2] * dx.size[3];
  if (n <= 0) return;
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(grid1(n)), dim3(256), 0, st, a, dy, is_max, n);
  check_hip(hipGetLastError(), "pool_bwd");
}

void launch_gemm(hipStream_t st, const ZTensor& A, const ZTensor& B, const ZTensor& Cm, const ZTensor& bias, float alpha,
                 float beta) {
  const long long M = Cm.size[0], N = Cm.size[1];
  if (M <= 0 || N <= 0) return;
  if (A.dtype == 1 && B.dtype == 1) {
    dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64));
    hipLaunchKernelGGL(gemm_mfma_kernel, grid, dim3(256), 0, st, A, B, Cm, bias, alpha, beta);
    check_hip(hipGetLastError(), "gemm_mfma");
    return;
  }
  dim3 grid((unsigned)((N + 15) / 16), (unsigned)((M + 15) / 16));
  hipLaunchKernelGGL(gemm_kernel, grid, dim3(256), 0, st, A, B, Cm, bias, alpha, beta);
  check_hip(hipGetLastError(), "gemm");
}

void launch_log_softmax(hipStream_t st, const ZTensor& x, const ZTensor& y, int bwd, const ZTensor& gy) {
  const long long R = x.size[0];
  hipLaunchKernelGGL(log_softmax_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, st, x, y, bwd, gy);
  check_hip(hipGetLastError(), "log_softmax");
}

void launch_nll_fwd(hipStream_t st, const ZTensor& lp, const long long* tgt, long long tstride, int ignore, int mean,
                    void* out, int out_bf16, void* tw, int tw_bf16) {
  hipLaunchKernelGGL(nll_fwd_kernel, dim3(1), dim3(256), 0, st, lp, tgt, tstride, ignore, mean,
                     out_bf16 ? nullptr : reinterpret_cast<float*>(out), out_bf16 ? reinterpret_cast<bf16*>(out) : nullptr,
                     tw_bf16 ? nullptr : reinterpret_cast<float*>(tw), tw_bf16 ? reinterpret_cast<bf16*>(tw) : nullptr);
  check_hip(hipGetLastError(), "nll_fwd");
}

void launch_nll_bwd(hipStream_t st, const ZTensor& gx, const void* g, int g_bf16, const void* tw, int tw_bf16,
                    const long long* tgt, long long tstride, int ignore, int mean) {
  const long long R = gx.size[0];
  hipLaunchKernelGGL(nll_bwd_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, st, gx,
                     reinterpret_cast<const float*>(g), reinterpret_cast<const float*>(tw), tgt, tstride, ignore, mean,
                     g_bf16, tw_bf16);
  check_hip(hipGetLastError(), "nll_bwd");
}

void launch_ce_stats(hipStream_t st, const ZTensor& logits, const long long* y, float* stats) {
  hipLaunchKernelGGL(ce_stats_kernel, dim3(1), dim3(256), 0, st, logits, y, stats);
  check_hip(hipGetLastError(), "ce_stats");
}

long long gconv_wgrad_ws_floats(long long N, long long P, long long Q, long long w_numel) {
  long long rps, slabs;
  gconv_slabs(N, P, Q, w_numel, &rps, &slabs);
  return slabs * w_numel;
}

void launch_gconv(hipStream_t st, int mode, const ZTensor& x, const ZTensor& w, const ZTensor& y, int G, int sth,
                  int stw, int padh, int padw, float* ws, long long ws_floats) {
  GConv g{};
  g.x = x; g.w = w; g.y = y; g.G = G; g.st_h = sth; g.st_w = stw; g.pad_h = padh; g.pad_w = padw;
  g.R = (int)w.size[2]; g.S = (int)w.size[3];
  const long long O = y.size[1], Cg = w.size[1], Og = O / G;
  // bf16x8 channel vectors: bf16, unit channel stride, every other stride and the group offset a
  // multiple of 8 elements, 16-byte aligned base
  auto vec_ok = [](const ZTensor& t, long long per_group) {
    if (t.dtype != 1 || t.ndim != 4 || t.stride[1] != 1 || per_group % 8) return 0;
    if (reinterpret_cast<uintptr_t>(t.p) % 16) return 0;
    for (int d : {0, 2, 3})
      if (t.stride[d] % 8) return 0;
    return 1;
  };
  g.vec_x = vec_ok(x, Cg);
  g.vec_y = vec_ok(y, Og);
  if (G <= 0 || O % G || x.size[1] != Cg * G || w.size[0] != O || g.R * g.S * GT > GC_LDS)
    throw std::invalid_argument("gconv: inconsistent shapes");
  if (mode == 0) {
    const long long n = y.size[0] * y.size[2] * y.size[3];
    if (n <= 0) return;
    hipLaunchKernelGGL(gconv_fwd_kernel, dim3((unsigned)((n + 255) / 256), G, (unsigned)((Og + GT - 1) / GT)), dim3(256),
                       0, st, g);
  } else if (mode == 1) {
    const long long n = x.size[0] * x.size[2] * x.size[3];
    if (n <= 0) return;
    hipLaunchKernelGGL(gconv_dgrad_kernel, dim3((unsigned)((n + 255) / 256), G, (unsigned)((Cg + GT - 1) / GT)),
                       dim3(256), 0, st, g);
  } else {
    const long long N = x.size[0], P = y.size[2], Q = y.size[3];
    const long long total = w.size[0] * w.size[1] * w.size[2] * w.size[3];
    long long rps, slabs;
    gconv_slabs(N, P, Q, total, &rps, &slabs);
    if (!ws || ws_floats < slabs * total) throw std::invalid_argument("gconv wgrad: workspace too small");
    const long long threads = O * g.R * g.S * ((Cg + 7) / 8);
    hipLaunchKernelGGL(gconv_wgrad_kernel, dim3((unsigned)((threads + 255) / 256), (unsigned)slabs), dim3(256), 0, st,
                       g, ws, (int)rps);
    hipLaunchKernelGGL(gconv_wgrad_sum_kernel, dim3((unsigned)((total + 63) / 64)), dim3(256), 0, st, ws, (int)slabs,
                       total, w);
  }
  check_hip(hipGetLastError(), "gconv");
}

}  // namespace fedmi
