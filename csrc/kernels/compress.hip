// fedmi — `-c Y` update compression on the device.
//
// The reference's -c Y is gRPC gzip over base64 fp32 checkpoints
// (src/server.py:103-107, src/client.py:39-43), which saves ~1-2 % because fp32
// weights are incompressible.  fedmi keeps the flag and makes
// it mean lossy *update* compression on the data plane:
//
//   top-k:  d = (w_local - w_global) + residual      (error feedback)
//           exact k-th largest |d| by a 4-pass 8-bit radix select
//           (LDS-privatised histograms, no sort), deterministic compaction
//           (block scans, ties taken in index order), residual <- d - sparse(d)
//   int8:   per-256-element-chunk absmax scaling, residual <- d - deq(q(d))
//
// The compressed payloads are all-gathered over RCCL and folded back with
// scatter_add_ranked (rank-ordered, atomic-free) / dequant_accum.
#include "common.h"

namespace {

struct SelectState {
  unsigned prefix;       // selected high bits of the threshold key so far
  unsigned mask;         // which bits of prefix are decided
  int k_rem;             // elements still to take at/below the current prefix
  int n_gt;              // elements strictly above the final threshold (set by the last pick)
  unsigned hist[256];
};

FEDMI_DEV unsigned key_of(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__global__ __launch_bounds__(256) void ef_delta_kernel(const float* __restrict__ local, const float* __restrict__ global,
                                                       const float* __restrict__ residual, float* __restrict__ d, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    d[i] = local[i] - global[i] + (residual ? residual[i] : 0.f);
}

__global__ void select_init_kernel(SelectState* st, int k) {
  const int t = threadIdx.x;
  if (t == 0) { st->prefix = 0u; st->mask = 0u; st->k_rem = k; st->n_gt = 0; }
  if (t < 256) st->hist[t] = 0u;
}

__global__ __launch_bounds__(256) void radix_hist_kernel(const float* __restrict__ d, long n, SelectState* st, int shift) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const unsigned prefix = st->prefix, mask = st->mask;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const unsigned k = key_of(d[i]);
    if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
  }
  __syncthreads();
  const unsigned v = h[threadIdx.x];
  if (v) atomicAdd(&st->hist[threadIdx.x], v);
}

// One workgroup: choose the digit holding the k_rem-th largest key.
__global__ __launch_bounds__(256) void radix_pick_kernel(SelectState* st, int shift) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = st->hist[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    int k = st->k_rem;
    unsigned above = 0u;
    int digit = 0;
    for (int b = 255; b >= 0; --b) {
      if (above + h[b] >= (unsigned)k) { digit = b; break; }
      above += h[b];
    }
    st->k_rem = k - (int)above;
    st->n_gt += (int)above;
    st->prefix |= ((unsigned)digit) << shift;
    st->mask |= 255u << shift;
  }
  __syncthreads();
  st->hist[threadIdx.x] = 0u;
}

constexpr int kChunk = 2048;   // elements per compaction block (256 thr x 8)

// per-block counts of (key > T) and (key == T)
__global__ __launch_bounds__(256) void compact_count_kernel(const float* __restrict__ d, long n, const SelectState* st,
                                                            int* __restrict__ counts) {
  __shared__ int sg[4], se[4];
  const unsigned T = st->prefix;
  const long base = (long)blockIdx.x * kChunk;
  int gt = 0, eq = 0;
  for (int j = threadIdx.x; j < kChunk; j += 256) {
    const long i = base + j;
    if (i < n) {
      const unsigned k = key_of(d[i]);
      gt += k > T;
      eq += k == T;
    }
  }
  for (int off = 32; off > 0; off >>= 1) { gt += __shfl_xor(gt, off, 64); eq += __shfl_xor(eq, off, 64); }
  if ((threadIdx.x & 63) == 0) { sg[threadIdx.x >> 6] = gt; se[threadIdx.x >> 6] = eq; }
  __syncthreads();
  if (threadIdx.x == 0) {
    counts[2 * blockIdx.x] = sg[0] + sg[1] + sg[2] + sg[3];
    counts[2 * blockIdx.x + 1] = se[0] + se[1] + se[2] + se[3];
  }
}

// single workgroup exclusive scan of the per-block counts (in place)
__global__ __launch_bounds__(256) void compact_scan_kernel(int* __restrict__ counts, int nblocks) {
  if (threadIdx.x == 0) {
    int ag = 0, ae = 0;
    for (int b = 0; b < nblocks; ++b) {
      const int g = counts[2 * b], e = counts[2 * b + 1];
      counts[2 * b] = ag;
      counts[2 * b + 1] = ae;
      ag += g;
      ae += e;
    }
  }
}

FEDMI_DEV int block_excl_scan(int flag, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(flag);
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int in_wave = __popcll(bal & lt);
  if (lane == 0) wsum[w] = __popcll(bal);
  __syncthreads();
  int before = 0;
  for (int q = 0; q < w; ++q) before += wsum[q];
  total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return before + in_wave;
}

__global__ __launch_bounds__(256) void compact_write_kernel(const float* __restrict__ d, long n, const SelectState* st,
                                                            const int* __restrict__ offs, int* __restrict__ idx,
                                                            float* __restrict__ val, float* __restrict__ residual) {
  __shared__ int wsum[4];
  const unsigned T = st->prefix;
  const int take_eq = st->k_rem, n_gt = st->n_gt;
  int og = offs[2 * blockIdx.x], oe = offs[2 * blockIdx.x + 1];
  const long base = (long)blockIdx.x * kChunk;
  for (int j0 = 0; j0 < kChunk; j0 += 256) {
    const long i = base + j0 + threadIdx.x;
    float v = 0.f;
    unsigned k = 0u;
    const bool in = i < n;
    if (in) { v = d[i]; k = key_of(v); }
    const int fg = in && k > T, fe = in && k == T;
    int tg, te;
    const int rg = block_excl_scan(fg, wsum, tg);
    const int re = block_excl_scan(fe, wsum, te);
    bool sel = false;
    if (fg) { idx[og + rg] = (int)i; val[og + rg] = v; sel = true; }
    if (fe && oe + re < take_eq) { idx[n_gt + oe + re] = (int)i; val[n_gt + oe + re] = v; sel = true; }
    if (in && residual) residual[i] = sel ? 0.f : v;
    og += tg;
    oe += te;
  }
}

// out[idx[i]] += scale * val[i] for ONE rank's payload.  Indices are unique within a
// rank (top-k), so no atomics: the launcher applies the ranks' payloads one launch
// after another in rank order, and every client computes the same fp32 sums in the
// same order -> bit-identical global models (atomics would add in arrival order).
__global__ __launch_bounds__(256) void scatter_add_rank_kernel(float* __restrict__ out, const int* __restrict__ idx,
                                                               const float* __restrict__ val, long m, float scale, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const int j = idx[i];
    if (j >= 0 && j < n) out[j] += scale * val[i];
  }
}

// int8: one workgroup per 256-element chunk
__global__ __launch_bounds__(256) void quant_int8_kernel(const float* __restrict__ d, long n, signed char* __restrict__ q,
                                                         float* __restrict__ scales, float* __restrict__ residual) {
  __shared__ float wmax[4];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const float v = i < n ? d[i] : 0.f;
  float a = fabsf(v);
  for (int off = 32; off > 0; off >>= 1) a = fmaxf(a, __shfl_xor(a, off, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = a;
  __syncthreads();
  const float amax = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  if (i < n) {
    const float r = rintf(v / s);
    const int qi = (int)fminf(fmaxf(r, -127.f), 127.f);
    q[i] = (signed char)qi;
    if (residual) residual[i] = v - (float)qi * s;
  }
  if (threadIdx.x == 0) scales[blockIdx.x] = s;
}

// out[i] += scale * sum_r q[r][i] * scales[r][i/256]
__global__ __launch_bounds__(256) void dequant_accum_kernel(const signed char* __restrict__ q, const float* __restrict__ scales,
                                                            int R, long n, long nchunks, float* __restrict__ out, float scale) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int r = 0; r < R; ++r) acc += (float)q[(long)r * n + i] * scales[(long)r * nchunks + (i >> 8)];
    out[i] += scale * acc;
  }
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

}  // namespace

namespace fedmi {

size_t select_state_bytes() { return sizeof(SelectState); }
int compact_chunk() { return kChunk; }

void launch_ef_delta(hipStream_t st, const float* local, const float* global, const float* residual, float* d, long n) {
  hipLaunchKernelGGL(ef_delta_kernel, dim3(grid_for(n)), dim3(256), 0, st, local, global, residual, d, n);
}

// Exact top-k by magnitude.  counts: int[2*ceil(n/kChunk)] scratch.
// Writes exactly k (idx, val) pairs; residual (optional) keeps the rest.
void launch_topk(hipStream_t st, const float* d, long n, int k, void* state, int* counts, int* idx, float* val,
                 float* residual) {
  SelectState* s = reinterpret_cast<SelectState*>(state);
  hipLaunchKernelGGL(select_init_kernel, dim3(1), dim3(256), 0, st, s, k);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(grid_for(n)), dim3(256), 0, st, d, n, s, shift);
    hipLaunchKernelGGL(radix_pick_kernel, dim3(1), dim3(256), 0, st, s, shift);
  }
  const int nb = (int)((n + kChunk - 1) / kChunk);
  hipLaunchKernelGGL(compact_count_kernel, dim3(nb), dim3(256), 0, st, d, n, s, counts);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(64), 0, st, counts, nb);
  hipLaunchKernelGGL(compact_write_kernel, dim3(nb), dim3(256), 0, st, d, n, s, counts, idx, val, residual);
}

// idx/val: [R][m] gathered payloads, applied in rank order 0..R-1.
void launch_scatter_add_ranked(hipStream_t st, float* out, const int* idx, const float* val, int R, long m, float scale,
                               long n) {
  if (m <= 0) return;
  for (int r = 0; r < R; ++r)
    hipLaunchKernelGGL(scatter_add_rank_kernel, dim3(grid_for(m)), dim3(256), 0, st, out, idx + (long)r * m,
                       val + (long)r * m, m, scale, n);
}

void launch_quant_int8(hipStream_t st, const float* d, long n, signed char* q, float* scales, float* residual) {
  const long nchunks = (n + 255) / 256;
  hipLaunchKernelGGL(quant_int8_kernel, dim3((unsigned)nchunks), dim3(256), 0, st, d, n, q, scales, residual);
}

void launch_dequant_accum(hipStream_t st, const signed char* q, const float* scales, int R, long n, float* out, float scale) {
  const long nchunks = (n + 255) / 256;
  hipLaunchKernelGGL(dequant_accum_kernel, dim3(grid_for(n)), dim3(256), 0, st, q, scales, R, n, nchunks, out, scale);
}

}  // namespace fedmi
