// fedmi — `-c Y` update compression on the device.
//
// The reference's -c Y is gRPC gzip over base64 fp32 checkpoints
// (src/server.py:103-107, src/client.py:39-43), which saves ~1-2 % because fp32
// weights are incompressible.  fedmi keeps the flag and makes
// it mean lossy *update* compression on the data plane:
//
//   top-k:  d = (w_local - w_global) + residual      (error feedback)
//           exact k-th largest |d|: an 11-bit histogram of the top key bits
//           fused with the delta pass, one compaction pass that takes the bins
//           above the boundary outright and keeps the boundary bin as
//           candidates, an exact LDS radix select among those (ties: smallest
//           indices); residual <- d - sparse(d)  (the tk_* kernels below)
//   int8:   per-256-element-chunk absmax scaling, residual <- d - deq(q(d))
//
// The compressed payloads are all-gathered over RCCL and folded back with
// scatter_add_ranked (rank-ordered, atomic-free) / dequant_accum.
#include <algorithm>
#include <cstddef>

#include "common.h"

namespace {

FEDMI_DEV unsigned key_of(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__global__ __launch_bounds__(256) void ef_delta_kernel(const float* __restrict__ local, const float* __restrict__ global,
                                                       const float* __restrict__ residual, float* __restrict__ d, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    d[i] = local[i] - global[i] + (residual ? residual[i] : 0.f);
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

// ---------------------------------------------------------------------------
// Fused error-feedback top-k (the default path): 3 launches (6 from 1 M entries), 2 full passes over the state.
//
//   K1 tk_delta_hist   r <- x - g + r (the residual buffer holds d from here on), and a
//                      histogram of the top 11 bits of |d| (key bits 30..20: exponent + 3
//                      mantissa bits, each bin ~9 % of magnitude), LDS-privatised per
//                      workgroup, nonzero bins added to the global histogram.  The bin b1 holding the
//                      k-th largest key is picked by every K2 workgroup from that histogram (n < 1 M; a
//                      one-workgroup tk_pick1 launch from 1 M entries); tk_select2 / tk_pick1 leave the
//                      histogram and the append counters zero for the next call.
//   K2 tk_compact1     keys in bins > b1 are selected outright (idx/val appended, r <- 0);
//                      keys in bin b1 become candidates (index + key appended).  Appends are
//                      staged in LDS (one pair of LDS atomics per wave per pass) and flushed with
//                      one global atomic per list per workgroup.  Large n: also the level-2
//                      histogram of the candidates (picked by tk_pick2); tk_compact2 then splits the
//                      candidates the same way one level down.
//   K3 tk_select2      one workgroup: exact selection of the remaining `need` among the
//                      candidates (LDS radix passes over the undecided key bits; exact ties
//                      resolved by the smallest indices, 3 more passes only when needed).
//
// The selected SET is exact and deterministic (ties: smallest indices); the order of the
// (idx, val) list depends on arrival order, which no consumer sees: a rank's indices are
// unique and scatter_add_ranked applies the ranks one after another.
constexpr int kTkBins1 = 2048;
constexpr long kTkThreeLevel = 1 << 20;   // n at which the 3-level path takes over
struct TopKState {
  unsigned hist[kTkBins1];
  int b1, n_above, need, out_cnt, cand_cnt, pad[3];   // pad[0]: sticky overflow flag (topk_overflow_offset)
  // 3-level path (large n): level-2 histogram of the candidates' key bits 19..9
  unsigned hist2[kTkBins1];
  int b2, n_above2, need2, out2_cnt, cand2_cnt;
  int pad2[3];
};

// NT threads: bin b of h[0..nb) (nb = 1024 or 2048, nb >= NT) such that above(b) < k <= above(b) + h[b],
// scanning from the TOP bin down; above(b) = sum of the bins > b.  Result in res[0..1].
template <int NT = 1024>
FEDMI_DEV void tk_find_top(const unsigned* h, int nb, unsigned k, unsigned* scratch, unsigned* res) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, per = nb / NT;
  unsigned s = 0u;
  for (int j = 0; j < per; ++j) s += h[nb - 1 - (t * per + j)];
  unsigned inc = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned v = __shfl_up(inc, off, 64);
    if (lane >= off) inc += v;
  }
  if (lane == 63) scratch[w] = inc;
  __syncthreads();
  if (t == 0) {
    unsigned a = 0u;
    for (int q = 0; q < NW; ++q) { const unsigned v = scratch[q]; scratch[16 + q] = a; a += v; }
  }
  __syncthreads();
  const unsigned excl = scratch[16 + w] + inc - s;
  if (excl < k && k <= excl + s) {
    unsigned above = excl;
    for (int j = 0; j < per; ++j) {
      const int b = nb - 1 - (t * per + j);
      if (above + h[b] >= k) { res[0] = (unsigned)b; res[1] = above; break; }
      above += h[b];
    }
  }
  __syncthreads();
}

FEDMI_DEV void tk_hist_add(unsigned* h, float v) { atomicAdd(&h[key_of(v) >> 20], 1u); }

template <bool VEC>
__global__ __launch_bounds__(256) void tk_delta_hist_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                            float* __restrict__ r, long n, TopKState* __restrict__ st,
                                                            int k) {
  __shared__ unsigned h[kTkBins1];
  for (int i = threadIdx.x; i < kTkBins1; i += 256) h[i] = 0u;
  __syncthreads();
  const long stride = (long)gridDim.x * 256;
  if (VEC) {
    const long n4 = n >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* r4 = reinterpret_cast<float4*>(r);
    // 4 float4 per thread per iteration, all 12 loads issued before the first use
    for (long i0 = (long)blockIdx.x * 1024 + threadIdx.x; i0 < n4; i0 += stride * 4) {
      float4 a[4], b[4], c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long i = i0 + u * 256;
        if (i < n4) { a[u] = x4[i]; b[u] = g4[i]; c[u] = r4[i]; }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long i = i0 + u * 256;
        if (i < n4) {
          const float4 d = make_float4(a[u].x - b[u].x + c[u].x, a[u].y - b[u].y + c[u].y, a[u].z - b[u].z + c[u].z,
                                       a[u].w - b[u].w + c[u].w);
          r4[i] = d;
          tk_hist_add(h, d.x);
          tk_hist_add(h, d.y);
          tk_hist_add(h, d.z);
          tk_hist_add(h, d.w);
        }
      }
    }
    if (blockIdx.x == 0 && threadIdx.x < (int)(n & 3)) {
      const long i = (n4 << 2) + threadIdx.x;
      const float d = x[i] - g[i] + r[i];
      r[i] = d;
      tk_hist_add(h, d);
    }
  } else {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const float d = x[i] - g[i] + r[i];
      r[i] = d;
      tk_hist_add(h, d);
    }
  }
  __syncthreads();
  // rotated bin order per workgroup: concurrent workgroups hit different global bins at a time
  for (int j = threadIdx.x; j < kTkBins1; j += 256) {
    const int i = (j + (int)blockIdx.x * 64) & (kTkBins1 - 1);
    if (h[i]) atomicAdd(&st->hist[i], h[i]);
  }
}

__global__ __launch_bounds__(1024) void tk_pick1_kernel(TopKState* __restrict__ st, int k) {
  __shared__ unsigned h[kTkBins1];
  __shared__ unsigned scratch[32], res[2];
  for (int i = threadIdx.x; i < kTkBins1; i += 1024) {
    h[i] = st->hist[i];
    st->hist[i] = 0u;                        // zero for the next call (graph-safe: no memset node)
  }
  __syncthreads();
  tk_find_top(h, kTkBins1, (unsigned)k, scratch, res);
  if (threadIdx.x == 0) {
    st->b1 = (int)res[0];
    st->n_above = (int)res[1];
    st->need = k - (int)res[1];
    st->out_cnt = 0;
    st->cand_cnt = 0;
  }
}

// level 2 (large n): the bin b2 of key bits 19..9 holding the need-th largest candidate
__global__ __launch_bounds__(1024) void tk_pick2_kernel(TopKState* __restrict__ st) {
  __shared__ unsigned h[kTkBins1];
  __shared__ unsigned scratch[32], res[2];
  for (int i = threadIdx.x; i < kTkBins1; i += 1024) {
    h[i] = st->hist2[i];
    st->hist2[i] = 0u;
  }
  __syncthreads();
  const int need = st->need;
  tk_find_top(h, kTkBins1, (unsigned)need, scratch, res);
  if (threadIdx.x == 0) {
    st->b2 = (int)res[0];
    st->n_above2 = (int)res[1];
    st->need2 = need - (int)res[1];
    st->out2_cnt = 0;
    st->cand2_cnt = 0;
  }
}

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its outstanding
// global loads (a __syncthreads() would also drain prefetched loads of the next pass)
FEDMI_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Winners and candidates are staged in LDS and appended to the global lists once per workgroup (two
// global atomics per flush): per-wave global atomics on the two list counters serialise at one L2
// address each (2.4 ms at 11 M entries, measured).
constexpr int kTkStage = 4096;   // >= 2 iterations' worth (8 x 256 per iteration)
template <int LEVELS, int NT>
FEDMI_DEV void tk_select_body(float* __restrict__ r, int c, int nab, unsigned m, const int* __restrict__ cidx,
                              const unsigned* __restrict__ ckey, int* __restrict__ idx, float* __restrict__ val,
                              int* overflow, unsigned* h, unsigned* scratch, unsigned* res, int* wcount_p);

// PICK (2-level path, n < kTkThreeLevel): every workgroup finds the boundary bin b1 itself from the global
// histogram (one 8 KB read + an LDS scan) instead of a one-workgroup tk_pick1 launch in between; workgroup 0
// publishes (b1, n_above, need) for tk_select2, which also re-zeroes the histogram and the list counters for the
// next call once every compaction workgroup has read them.
template <bool H2, bool PICK>
__global__ __launch_bounds__(256) void tk_compact1_kernel(float* __restrict__ r, long n, TopKState* __restrict__ st,
                                                          int* __restrict__ idx, float* __restrict__ val,
                                                          int* __restrict__ cidx, unsigned* __restrict__ ckey, int k) {
  __shared__ int s_si[kTkStage], s_ci[kTkStage];   // 4 x 16 KB of LDS
  __shared__ float s_sv[kTkStage];
  __shared__ unsigned s_ck[kTkStage];
  __shared__ unsigned h2[(H2 || PICK) ? kTkBins1 : 1];
  __shared__ int n_s, n_c, b_s, b_c;
  __shared__ unsigned pscr[32], pres[2];
  unsigned b1;
  if constexpr (PICK) {
    for (int i = threadIdx.x; i < kTkBins1; i += 256) h2[i] = st->hist[i];
    __syncthreads();
    tk_find_top<256>(h2, kTkBins1, (unsigned)k, pscr, pres);
    b1 = pres[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->b1 = (int)pres[0];
      st->n_above = (int)pres[1];
      st->need = k - (int)pres[1];
    }
    __syncthreads();      // h2 is reused as the level-2 histogram only when H2 (never together with PICK)
  } else {
    b1 = (unsigned)st->b1;
  }
  const long stride = (long)gridDim.x * 256;
  if (threadIdx.x == 0) { n_s = 0; n_c = 0; }
  if (H2)
    for (int i = threadIdx.x; i < kTkBins1; i += 256) h2[i] = 0u;
  __syncthreads();
  // uniform trip count per workgroup: every lane takes part in every ballot and barrier.  8 elements per
  // thread per pass; the NEXT pass's 8 loads are issued before this pass is processed, and the pass's
  // barriers wait for LDS operations only (lds_barrier), so they stay in flight across it
  // (loads are unconditional -- clamped address, masked value -- so no branch splits them and the compiler can
  // wait for the older pass only)
  float nx[8];
  long i0 = (long)blockIdx.x * 2048;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const long i = i0 + u * 256 + threadIdx.x;
    const float v = r[i < n ? i : n - 1];
    nx[u] = i < n ? v : 0.f;
  }
  for (; i0 < n; i0 += stride * 8) {
    float dv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) dv[u] = nx[u];
    const long i1 = i0 + stride * 8;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long i = i1 + u * 256 + threadIdx.x;
      const float v = r[i < n ? i : n - 1];   // disjoint from this pass's elements (zeroed below when selected)
      nx[u] = i < n ? v : 0.f;
    }
    // classify all 8 first, then ONE pair of LDS appends per wave for the whole pass (two independent
    // returning atomics instead of 16 dependent ones); slots follow from the 8 ballots
    unsigned key[8];
    unsigned long long ms[8], mc[8];
    int ts = 0, tc = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long i = i0 + u * 256 + threadIdx.x;
      const bool in = i < n;
      key[u] = key_of(dv[u]);
      const unsigned bin = key[u] >> 20;
      ms[u] = __ballot(in && bin > b1);
      mc[u] = __ballot(in && bin == b1);
      ts += (int)__popcll(ms[u]);
      tc += (int)__popcll(mc[u]);
    }
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int bs = 0, bc = 0;
    if (lane == 0) {
      if (ts) bs = atomicAdd(&n_s, ts);
      if (tc) bc = atomicAdd(&n_c, tc);
    }
    bs = __shfl(bs, 0, 64);
    bc = __shfl(bc, 0, 64);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long i = i0 + u * 256 + threadIdx.x;
      if ((ms[u] >> lane) & 1ull) {
        const int ps = bs + (int)__popcll(ms[u] & lt);
        s_si[ps] = (int)i; s_sv[ps] = dv[u]; r[i] = 0.f;
      }
      if ((mc[u] >> lane) & 1ull) {
        const int pc = bc + (int)__popcll(mc[u] & lt);
        s_ci[pc] = (int)i;
        s_ck[pc] = key[u];
        if (H2) atomicAdd(&h2[(key[u] >> 9) & (kTkBins1 - 1)], 1u);
      }
      bs += (int)__popcll(ms[u]);
      bc += (int)__popcll(mc[u]);
    }
    lds_barrier();
    const bool last = i1 >= n;
    if (last || n_s > kTkStage - 8 * 256 || n_c > kTkStage - 8 * 256) {
      if (threadIdx.x == 0) {
        b_s = n_s ? atomicAdd(&st->out_cnt, n_s) : 0;
        b_c = n_c ? atomicAdd(&st->cand_cnt, n_c) : 0;
      }
      __syncthreads();
      for (int j = threadIdx.x; j < n_s; j += 256) { idx[b_s + j] = s_si[j]; val[b_s + j] = s_sv[j]; }
      for (int j = threadIdx.x; j < n_c; j += 256) { cidx[b_c + j] = s_ci[j]; ckey[b_c + j] = s_ck[j]; }
      lds_barrier();
      if (threadIdx.x == 0) { n_s = 0; n_c = 0; }
      lds_barrier();
    }
  }
  if (H2) {
    __syncthreads();
    for (int j = threadIdx.x; j < kTkBins1; j += 256) {
      const int i = (j + (int)blockIdx.x * 64) & (kTkBins1 - 1);
      if (h2[i]) atomicAdd(&st->hist2[i], h2[i]);
    }
  }
}

// level 2 (large n): candidates with key bits 19..9 above b2 are winners (positions n_above + [0, n_above2)),
// those in b2 go to the level-3 list; workgroup-staged appends like tk_compact1
__global__ __launch_bounds__(256) void tk_compact2_kernel(float* __restrict__ r, TopKState* __restrict__ st,
                                                          const int* __restrict__ cidx, const unsigned* __restrict__ ckey,
                                                          int* __restrict__ idx, float* __restrict__ val,
                                                          int* __restrict__ cidx2, unsigned* __restrict__ ckey2) {
  __shared__ int s_si[kTkStage], s_ci[kTkStage];
  __shared__ float s_sv[kTkStage];
  __shared__ unsigned s_ck[kTkStage];
  __shared__ int n_s, n_c, b_s, b_c;
  const int c = st->cand_cnt, nab = st->n_above;
  const unsigned b2 = (unsigned)st->b2;
  const long stride = (long)gridDim.x * 256;
  if (threadIdx.x == 0) { n_s = 0; n_c = 0; }
  __syncthreads();
  for (long j0 = (long)blockIdx.x * 2048; j0 < c; j0 += stride * 8) {
    int ci[8];
    unsigned kk[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long j = j0 + u * 256 + threadIdx.x;
      ci[u] = j < c ? cidx[j] : 0;
      kk[u] = j < c ? ckey[j] : 0u;
    }
    float dv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long j = j0 + u * 256 + threadIdx.x;
      dv[u] = (j < c && ((kk[u] >> 9) & (kTkBins1 - 1)) > b2) ? r[ci[u]] : 0.f;
    }
    // one pair of LDS appends per wave per pass (see tk_compact1_kernel)
    unsigned long long ms[8], mc[8];
    int ts = 0, tc = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long j = j0 + u * 256 + threadIdx.x;
      const unsigned bin = (kk[u] >> 9) & (kTkBins1 - 1);
      ms[u] = __ballot(j < c && bin > b2);
      mc[u] = __ballot(j < c && bin == b2);
      ts += (int)__popcll(ms[u]);
      tc += (int)__popcll(mc[u]);
    }
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int bs = 0, bc = 0;
    if (lane == 0) {
      if (ts) bs = atomicAdd(&n_s, ts);
      if (tc) bc = atomicAdd(&n_c, tc);
    }
    bs = __shfl(bs, 0, 64);
    bc = __shfl(bc, 0, 64);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if ((ms[u] >> lane) & 1ull) {
        const int ps = bs + (int)__popcll(ms[u] & lt);
        s_si[ps] = ci[u]; s_sv[ps] = dv[u]; r[ci[u]] = 0.f;
      }
      if ((mc[u] >> lane) & 1ull) {
        const int pc = bc + (int)__popcll(mc[u] & lt);
        s_ci[pc] = ci[u]; s_ck[pc] = kk[u];
      }
      bs += (int)__popcll(ms[u]);
      bc += (int)__popcll(mc[u]);
    }
    __syncthreads();
    const bool last = j0 + stride * 8 >= c;
    if (last || n_s > kTkStage - 8 * 256 || n_c > kTkStage - 8 * 256) {
      if (threadIdx.x == 0) {
        b_s = n_s ? atomicAdd(&st->out2_cnt, n_s) : 0;
        b_c = n_c ? atomicAdd(&st->cand2_cnt, n_c) : 0;
      }
      __syncthreads();
      for (int q = threadIdx.x; q < n_s; q += 256) { idx[nab + b_s + q] = s_si[q]; val[nab + b_s + q] = s_sv[q]; }
      for (int q = threadIdx.x; q < n_c; q += 256) { cidx2[b_c + q] = s_ci[q]; ckey2[b_c + q] = s_ck[q]; }
      __syncthreads();
      if (threadIdx.x == 0) { n_s = 0; n_c = 0; }
      __syncthreads();
    }
  }
}

// Exact selection of the remaining m among c candidates (cidx / ckey), one 1024-thread workgroup; winners land at
// idx / val [nab, nab + m).  LEVELS == 2: the level-1 candidates (key bits 19..0 undecided, 2 radix passes);
// LEVELS == 1: the level-3 list of the 3-level path (bits 19..9 decided; one pass over bits 9..0, bit 9 common
// to all).  h: >= kTkBins1 LDS words, scratch: 32, res: 2.
template <int LEVELS, int NT = 1024>
FEDMI_DEV void tk_select_body(float* __restrict__ r, int c, int nab, unsigned m, const int* __restrict__ cidx,
                              const unsigned* __restrict__ ckey, int* __restrict__ idx, float* __restrict__ val,
                              int* overflow, unsigned* h, unsigned* scratch, unsigned* res, int* wcount_p) {
  int& wcount = *wcount_p;
  const int t = threadIdx.x;
  constexpr unsigned LOWMASK = LEVELS == 2 ? 0xfffffu : 0x3ffu;
  // pass A: key bits 19..10
  unsigned bA = 0u, mA = m;
  if (LEVELS == 2) {
    for (int i = t; i < 1024; i += NT) h[i] = 0u;
    __syncthreads();
    for (int j0 = t; j0 < c; j0 += 8 * NT) {         // 8 loads in flight per thread
      unsigned kk[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) kk[u] = j0 + u * NT < c ? ckey[j0 + u * NT] : 0u;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (j0 + u * NT < c) atomicAdd(&h[(kk[u] >> 10) & 1023u], 1u);
    }
    __syncthreads();
    tk_find_top<NT>(h, 1024, m, scratch, res);
    bA = res[0];
    mA = m - res[1];
  }
  // pass B: key bits 9..0 of the keys in bin bA
  for (int i = t; i < 1024; i += NT) h[i] = 0u;
  __syncthreads();
  for (int j0 = t; j0 < c; j0 += 8 * NT) {
    unsigned kk[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) kk[u] = j0 + u * NT < c ? ckey[j0 + u * NT] : 0u;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + u * NT < c && (LEVELS == 1 || ((kk[u] >> 10) & 1023u) == bA)) atomicAdd(&h[kk[u] & 1023u], 1u);
  }
  __syncthreads();
  tk_find_top<NT>(h, 1024, mA, scratch, res);
  const unsigned bB = res[0];
  const unsigned T = LEVELS == 2 ? ((bA << 10) | bB) : bB;   // undecided low bits of the k-th largest key
  const unsigned ties_take = mA - res[1], ties = h[bB];
  __syncthreads();
  // exact ties beyond what is needed: keep the smallest indices (radix on the index, smallest first:
  // digit' = nb-1-digit makes "top" the smallest)
  unsigned ilim = 0xffffffffu;
  if (ties > ties_take) {
    unsigned pre = 0u, pmask = 0u, kk = ties_take;
    const int shifts[3] = {20, 10, 0};
    const int widths[3] = {11, 10, 10};
    for (int ps = 0; ps < 3; ++ps) {
      const int nb = 1 << widths[ps], sh = shifts[ps];
      for (int i = t; i < kTkBins1; i += NT) h[i] = 0u;
      __syncthreads();
      for (int j = t; j < c; j += NT) {
        const unsigned ix = (unsigned)cidx[j];
        if ((ckey[j] & LOWMASK) == T && (ix & pmask) == pre) atomicAdd(&h[nb - 1 - ((ix >> sh) & (nb - 1))], 1u);
      }
      __syncthreads();
      tk_find_top<NT>(h, nb < 1024 ? 1024 : nb, kk, scratch, res);
      pre |= (unsigned)(nb - 1 - (int)res[0]) << sh;
      pmask |= (unsigned)(nb - 1) << sh;
      kk -= res[1];
      __syncthreads();
    }
    ilim = pre;                               // the ties_take-th smallest tied index
  }
  if (t == 0) wcount = 0;
  __syncthreads();
  for (int j0 = 0; j0 < c; j0 += 4 * NT) {      // uniform trip count: every lane takes part in the ballots
    unsigned kk[4];
    int ci[4];
    float dv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * NT + t;
      kk[u] = j < c ? ckey[j] : 0u;
      ci[u] = j < c ? cidx[j] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) dv[u] = j0 + u * NT + t < c ? r[ci[u]] : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned low = kk[u] & LOWMASK;
      const bool sel = j0 + u * NT + t < c && (low > T || (low == T && (unsigned)ci[u] <= ilim));
      const unsigned long long msk = __ballot(sel);
      int base = 0;
      if ((t & 63) == 0 && msk) base = atomicAdd(&wcount, (int)__popcll(msk));
      base = __shfl(base, 0, 64);
      if (sel) {
        const int lane = t & 63;
        const int pos = nab + base + (int)__popcll(msk & (lane ? (~0ull >> (64 - lane)) : 0ull));
        // never past the k-entry payload (a selection larger than need would otherwise write beyond idx /
        // val into whatever the allocator placed after them); an overflow is flagged in the state
        if (pos < nab + (int)m) {
          idx[pos] = ci[u];
          val[pos] = dv[u];
          r[ci[u]] = 0.f;
        } else {
          *overflow = 1;
        }
      }
    }
  }
}

template <int LEVELS>
__global__ __launch_bounds__(1024) void tk_select2_kernel(float* __restrict__ r, TopKState* __restrict__ st,
                                                          const int* __restrict__ cidx, const unsigned* __restrict__ ckey,
                                                          int* __restrict__ idx, float* __restrict__ val) {
  __shared__ unsigned h[kTkBins1];
  __shared__ unsigned scratch[32], res[2];
  __shared__ int wcount;
  const int c = LEVELS == 2 ? st->cand_cnt : st->cand2_cnt;
  const int nab = LEVELS == 2 ? st->n_above : st->n_above + st->n_above2;
  const unsigned m = (unsigned)(LEVELS == 2 ? st->need : st->need2);
  tk_select_body<LEVELS>(r, c, nab, m, cidx, ckey, idx, val, &st->pad[0], h, scratch, res, &wcount);
  // leave the level-1 histogram and list counters zero for the next call, on BOTH paths: the 2-level path has
  // no pick launch that would reset them, so a 3-level call followed by a 2-level one must not leave its
  // counters behind (the 2-level compaction would append past the end of idx / cidx)
  if (LEVELS == 2)
    for (int i = threadIdx.x; i < kTkBins1; i += blockDim.x) st->hist[i] = 0u;
  if (threadIdx.x == 0) { st->out_cnt = 0; st->cand_cnt = 0; }
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

}  // namespace

namespace fedmi {

void launch_ef_delta(hipStream_t st, const float* local, const float* global, const float* residual, float* d, long n) {
  hipLaunchKernelGGL(ef_delta_kernel, dim3(grid_for(n)), dim3(256), 0, st, local, global, residual, d, n);
}

size_t topk_state_bytes() { return sizeof(TopKState); }
// byte offset of the int overflow word (set if a select ever produced more than k entries; sticky)
size_t topk_overflow_offset() { return offsetof(TopKState, pad); }

// Fused error-feedback exact top-k (see tk_* kernels).  residual: d is built IN it and the
// selected entries are zeroed (= the new residual); state: topk_state_bytes(), zero on first
// use (left zero by every call); cidx/ckey: candidate scratch of 2n entries each.
void launch_topk_ef(hipStream_t st, const float* x, const float* g, float* residual, long n, int k, void* state,
                    int* cidx, unsigned* ckey, int* idx, float* val) {
  TopKState* s = reinterpret_cast<TopKState*>(state);
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g) |
                     reinterpret_cast<uintptr_t>(residual)) & 15) == 0;
  // ~8 float4 per thread, at most 2048 workgroups (their nonzero bins go to the global histogram).  The
  // boundary-bin picks run as their own one-workgroup launches: doing them in the last-arriving workgroup of
  // the histogram / compaction kernels measured slower (132 vs 94.6 us at 11.2 M entries, 23.4 vs 22.7 us at
  // 62 k: every workgroup pays an agent-scope release and a drained flush for one launch saved), and so did
  // the select in the compaction's last workgroup (34 vs 24 us at 62 k) and a one-workgroup kernel for small
  // states (38.5 vs 22.7 us at 62 k) -- profiles/r3_dataplane/topk_ab.txt.
  const int blocks = (int)std::min<long>(2048, std::max<long>(1, (n + 8 * 1024 - 1) / (8 * 1024)));
  if (vec)
    hipLaunchKernelGGL(tk_delta_hist_kernel<true>, dim3(blocks), dim3(256), 0, st, x, g, residual, n, s, k);
  else
    hipLaunchKernelGGL(tk_delta_hist_kernel<false>, dim3(blocks), dim3(256), 0, st, x, g, residual, n, s, k);
  // compaction grid cap: 2 workgroups per CU (512) measured 103.5 vs 128 us at 11.2 M entries (2048: 4x the
  // per-workgroup flushes of the staged lists and of the level-2 histogram)
  const int cblocks = (int)std::min<long>(512, std::max<long>(1, (n + 2 * 2048 - 1) / (2 * 2048)));
  if (n < kTkThreeLevel) {   // 3 launches: the bin pick runs inside every compaction workgroup
    hipLaunchKernelGGL((tk_compact1_kernel<false, true>), dim3(cblocks), dim3(256), 0, st, residual, n, s, idx, val,
                       cidx, ckey, k);
    hipLaunchKernelGGL(tk_select2_kernel<2>, dim3(1), dim3(1024), 0, st, residual, s, cidx, ckey, idx, val);
    return;
  }
  hipLaunchKernelGGL(tk_pick1_kernel, dim3(1), dim3(1024), 0, st, s, k);
  // large n: the boundary bin holds ~1-3 % of the entries -- too many for one workgroup; a second histogram
  // level over the candidates (built by compact1) and a multi-workgroup compaction of them leave a
  // level-3 list of a few hundred for the single-workgroup exact select
  int* cidx2 = cidx + n;                     // second half of the 2n-entry candidate scratch
  unsigned* ckey2 = ckey + n;
  hipLaunchKernelGGL((tk_compact1_kernel<true, false>), dim3(cblocks), dim3(256), 0, st, residual, n, s, idx, val, cidx,
                     ckey, k);
  hipLaunchKernelGGL(tk_pick2_kernel, dim3(1), dim3(1024), 0, st, s);
  const int c2blocks = (int)std::min<long>(1024, std::max<long>(1, (n / 50 + 2047) / 2048));
  hipLaunchKernelGGL(tk_compact2_kernel, dim3(c2blocks), dim3(256), 0, st, residual, s, cidx, ckey, idx, val, cidx2,
                     ckey2);
  hipLaunchKernelGGL(tk_select2_kernel<1>, dim3(1), dim3(1024), 0, st, residual, s, cidx2, ckey2, idx, val);
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
