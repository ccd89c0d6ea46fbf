// fedmi — flat-buffer elementwise kernels for the generic (model-zoo) engine
// and the aggregation paths.
//
//  * sgd_flat:       torch.optim.SGD(momentum, weight_decay) over ONE flat fp32
//                    parameter buffer (multi-tensor apply in a single launch;
//                    the reference issues 4 ops x #tensors, src/main.py:151).
//  * fedavg_reduce:  out = sum_k w_k * in_k over K flat fp32 buffers — the
//                    coordinator-side FedAvg of gathered checkpoints
//                    (reference: CPU Python loop, src/server.py:155-179).
//  * scale_inplace:  x *= alpha (sum -> mean after a SUM all-reduce).
// All kernels stream 16 B per lane and grid-stride (memory-bound; HBM roof).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ buf, long n, float lr, float m,
                                                       float wd, float dampening, int nesterov, int first) {
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 bv = reinterpret_cast<float4*>(buf)[i];
    float* pp = reinterpret_cast<float*>(&pv);
    const float* gg = reinterpret_cast<const float*>(&gv);
    float* bb = reinterpret_cast<float*>(&bv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float d = gg[j] + wd * pp[j];
      if (m != 0.f) {
        bb[j] = first ? d : m * bb[j] + (1.f - dampening) * d;
        d = nesterov ? d + m * bb[j] : bb[j];
      }
      pp[j] -= lr * d;
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(buf)[i] = bv;
  }
  // tail
  for (long i = (n4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float d = g[i] + wd * p[i];
    if (m != 0.f) {
      buf[i] = first ? d : m * buf[i] + (1.f - dampening) * d;
      d = nesterov ? d + m * buf[i] : buf[i];
    }
    p[i] -= lr * d;
  }
}

constexpr int kMaxFedAvgInputs = 64;
struct FedAvgArgs {
  const float* in[kMaxFedAvgInputs];
  float w[kMaxFedAvgInputs];
};

__global__ __launch_bounds__(256) void fedavg_reduce_kernel(FedAvgArgs args, int k, float* __restrict__ out, long n) {
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < k; ++q) {
      const float4 v = reinterpret_cast<const float4*>(args.in[q])[i];
      const float w = args.w[q];
      acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
  for (long i = (n4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int q = 0; q < k; ++q) acc += args.w[q] * args.in[q][i];
    out[i] = acc;
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, long n, float alpha) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= alpha;
}

int grid_for(long n) {
  long blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;   // 256 CUs x 8: grid-stride the rest (Guideline 11)
  return (int)blocks;
}

}  // namespace

namespace fedmi {

void launch_sgd_flat(hipStream_t st, float* p, const float* g, float* buf, long n, float lr, float m, float wd,
                     float dampening, int nesterov, int first) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, buf, n, lr, m, wd, dampening,
                     nesterov, first);
}

int fedavg_max_inputs() { return kMaxFedAvgInputs; }

void launch_fedavg_reduce(hipStream_t st, const float* const* ins, const float* weights, int k, float* out, long n) {
  if (n <= 0 || k <= 0) return;
  FedAvgArgs a;
  for (int q = 0; q < k && q < kMaxFedAvgInputs; ++q) {
    a.in[q] = ins[q];
    a.w[q] = weights[q];
  }
  hipLaunchKernelGGL(fedavg_reduce_kernel, dim3(grid_for(n)), dim3(256), 0, st, a, k, out, n);
}

void launch_scale(hipStream_t st, float* x, long n, float alpha) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n * 4)), dim3(256), 0, st, x, n, alpha);
}

}  // namespace fedmi
