// fedmi — flat-buffer elementwise kernels for the generic (model-zoo) engine
// (FedAvg itself is one collective over the flat buffer: fedmi/parallel/fedavg.py).
//
//  * sgd_flat:       torch.optim.SGD(momentum, weight_decay) over ONE flat fp32
//                    parameter buffer (multi-tensor apply in a single launch;
//                    the reference issues 4 ops x #tensors, src/main.py:151).
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
    for (int j = 0; j < 4; ++j) fedmi::sgd_elem(pp[j], gg[j], bb[j], lr, m, wd, dampening, nesterov, first);
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(buf)[i] = bv;
  }
  // tail
  for (long i = (n4 << 2) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pv = p[i], bv = buf[i];
    fedmi::sgd_elem(pv, g[i], bv, lr, m, wd, dampening, nesterov, first);
    p[i] = pv;
    buf[i] = bv;
  }
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


}  // namespace fedmi
