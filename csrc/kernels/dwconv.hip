// fedmi — depthwise 2-D convolution (groups == channels) on NHWC bf16, the
// MobileNet / MobileNetV2 / EfficientNet / ShuffleNet / PNASNet building block
// (src/models/mobilenet.py:11-23, mobilenetv2.py:11-37, ...).
//
// Depthwise work has K = R*S (9 for 3x3) per output: no reduction dimension
// for MFMA to chew on, so these are VALU kernels built around 16-byte
// channel vectors: one thread owns 8 consecutive channels of one pixel, the
// R*S taps stream through registers, and the per-channel filter taps are
// loaded once per thread.  Memory-bound by design (HBM roofline), with the
// BatchNorm batch statistics of the output fused into the forward epilogue.
//
//   fwd    y[n,p,q,c]  = sum_rs x[n, p*st-pad+r, q*st-pad+s, c] * w[c,r,s]
//   dgrad  dx[n,h,w,c] = sum_rs dy[n, (h+pad-r)/st, (w+pad-s)/st, c] * w[c,r,s]
//   wgrad  dw[c,r,s]   = sum_npq dy[n,p,q,c] * x[n, p*st-pad+r, q*st-pad+s, c]
//          (per-block partials -> workspace -> deterministic reduce)
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "wgrad_reduce.h"

namespace {

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

struct DwGeom {
  int N, H, W, C, P, Q, R, S, st, pad;
};

FEDMI_DEV void ld8f(const bf16* p, float* v) {
  const bf16x8v b = *reinterpret_cast<const bf16x8v*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
}

constexpr int MAXRS = 49;   // up to 7x7 (PNASNet)

// Filter taps staged in LDS as [tap][C] fp32 (8 consecutive channels = 32 B).  8 loads in flight per
// thread: a load-use loop paid one memory round trip per C*RS/blockDim taps (18 for a 512-channel 3x3
// filter, ~half of those layers' 16 us).
FEDMI_DEV void stage_taps(const float* __restrict__ w, float* wl, int C, int RS) {
  const int n = C * RS, step = blockDim.x;
  for (int i0 = threadIdx.x; i0 < n; i0 += 8 * step) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = i0 + u * step < n ? w[i0 + u * step] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * step;
      if (i < n) {
        const int c = i / RS, t = i - c * RS;
        wl[t * C + c] = v[u];
      }
    }
  }
}

// one thread per (output pixel, 8-channel group); the block size is a multiple
// of C/8, so the grid stride is too and a thread's channel group is fixed
__global__ __launch_bounds__(256) void dw_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                     bf16* __restrict__ y, double* __restrict__ stats,
                                                     const float* __restrict__ shift, DwGeom g) {
  extern __shared__ float wl[];   // [RS][C]
  __shared__ float red[2][256][8];
  const int VC = g.C >> 3, RS = g.R * g.S;
  stage_taps(w, wl, g.C, RS);
  __syncthreads();
  const long total = (long)g.N * g.P * g.Q * VC;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  const int c0 = (int)(threadIdx.x % VC) * 8;
  float sh[8];   // statistics are of (y - shift): see conv_igemm's epilogue
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[j] = shift ? shift[c0 + j] : 0.f;
  // 32-bit index math (host guarantees < 2^31 elements): 64-bit div/mod are software loops
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = i / (uint32_t)VC;
    const uint32_t t2 = pix / (uint32_t)g.Q;
    const int q = (int)(pix - t2 * g.Q);
    const int n = (int)(t2 / (uint32_t)g.P), p = (int)(t2 - (uint32_t)n * g.P);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const long nb = (long)n * g.H;
    if (g.R == 3) {   // the MobileNet case: 9 independent 16-B loads in flight
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int h = p * g.st - g.pad + r;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int ww = q * g.st - g.pad + s;
          const bool ok = (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
          float v[8];
          ld8f(x + (ok ? ((nb + h) * g.W + ww) * g.C + c0 : c0), v);
          const float* wt = wl + (r * 3 + s) * g.C + c0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += ok ? v[j] * wt[j] : 0.f;
        }
      }
    } else {
      for (int r = 0; r < g.R; ++r) {
        const int h = p * g.st - g.pad + r;
        if ((unsigned)h >= (unsigned)g.H) continue;
        for (int s = 0; s < g.S; ++s) {
          const int ww = q * g.st - g.pad + s;
          if ((unsigned)ww >= (unsigned)g.W) continue;
          float v[8];
          ld8f(x + ((nb + h) * g.W + ww) * g.C + c0, v);
          const float* wt = wl + (r * g.S + s) * g.C + c0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += v[j] * wt[j];
        }
      }
    }
    bf16x8v o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (bf16)acc[j];
      const float vb = (float)o[j] - sh[j];
      s1[j] += vb;
      s2[j] += vb * vb;
    }
    *reinterpret_cast<bf16x8v*>(y + (long)pix * g.C + c0) = o;
  }
  if (stats == nullptr) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][threadIdx.x][j] = s1[j]; red[1][threadIdx.x][j] = s2[j]; }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * g.C; e += blockDim.x) {   // threads t == grp (mod VC) own group grp
    const int qn = e / g.C, c = e - qn * g.C;
    const int grp = c >> 3, j = c & 7;
    float sum = 0.f;
    for (int t = grp; t < (int)blockDim.x; t += VC) sum += red[qn][t][j];
    unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + qn) * g.C + c, (double)sum);
  }
}

// 3x3 depthwise forward, register-blocked along the output row: one thread per (2 adjacent output
// pixels, 8-channel group).  The 4 (stride 1) / 5 (stride 2) input columns of a filter row are loaded
// once for both outputs (6 / 7.5 loads per output instead of 9), and each tap's 8 filter values read from
// LDS feed two outputs; same fused BN statistics and input-BN option as dw_fwd_kernel.
template <int ST>
__global__ __launch_bounds__(256) void dw_fwd3_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                      bf16* __restrict__ y, double* __restrict__ stats,
                                                      const float* __restrict__ shift, DwGeom g) {
  constexpr int NCOL = ST == 1 ? 4 : 5;
  extern __shared__ float wl[];   // [9][C]
  __shared__ float red[2][256][8];
  const int VC = g.C >> 3;
  stage_taps(w, wl, g.C, 9);
  __syncthreads();
  const int Q2 = (g.Q + 1) >> 1;
  const long total = (long)g.N * g.P * Q2 * VC;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  const int c0 = (int)(threadIdx.x % VC) * 8;
  float sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[j] = shift ? shift[c0 + j] : 0.f;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)total; i += gridDim.x * blockDim.x) {
    const uint32_t pr = i / (uint32_t)VC;            // pair index
    const uint32_t t2 = pr / (uint32_t)Q2;
    const int q0 = (int)(pr - t2 * Q2) * 2;
    const int n = (int)(t2 / (uint32_t)g.P), p = (int)(t2 - (uint32_t)n * g.P);
    float a0[8], a1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a0[j] = a1[j] = 0.f;
    const long nb = (long)n * g.H;
    const int w0 = q0 * ST - 1;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = p * ST - 1 + r;
      const bool hok = (unsigned)h < (unsigned)g.H;
      float v[NCOL][8];
#pragma unroll
      for (int k = 0; k < NCOL; ++k) {
        const int ww = w0 + k;
        const bool ok = hok && (unsigned)ww < (unsigned)g.W;
        ld8f(x + (ok ? ((nb + h) * g.W + ww) * g.C + c0 : c0), v[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = ok ? v[k][j] : 0.f;
      }
#pragma unroll
      for (int s2i = 0; s2i < 3; ++s2i) {
        const float* wt = wl + (r * 3 + s2i) * g.C + c0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a0[j] += v[s2i][j] * wt[j];
          a1[j] += v[ST + s2i][j] * wt[j];
        }
      }
    }
    const long pix0 = (((long)n * g.P + p) * g.Q + q0);
    bf16x8v o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (bf16)a0[j];
      const float vb = (float)o[j] - sh[j];
      s1[j] += vb;
      s2[j] += vb * vb;
    }
    *reinterpret_cast<bf16x8v*>(y + pix0 * g.C + c0) = o;
    if (q0 + 1 < g.Q) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (bf16)a1[j];
        const float vb = (float)o[j] - sh[j];
        s1[j] += vb;
        s2[j] += vb * vb;
      }
      *reinterpret_cast<bf16x8v*>(y + (pix0 + 1) * g.C + c0) = o;
    }
  }
  if (stats == nullptr) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][threadIdx.x][j] = s1[j]; red[1][threadIdx.x][j] = s2[j]; }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * g.C; e += blockDim.x) {
    const int qn = e / g.C, c = e - qn * g.C;
    const int grp = c >> 3, j = c & 7;
    float sum = 0.f;
    for (int t = grp; t < (int)blockDim.x; t += VC) sum += red[qn][t][j];
    unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + qn) * g.C + c, (double)sum);
  }
}

// one thread per (input pixel, 8-channel group): gather form, no atomics.
// bs (optional): the BatchNorm-backward channel sums of dx's producer BN (fedmi::BnSums, the dense
// DGRAD epilogue's contract), from the stored bf16 dx; blockDim is a multiple of C/8, so a thread's
// channel group is fixed and its sums reduce through LDS behind the filter image.
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const bf16* __restrict__ dy, const float* __restrict__ w,
                                                       bf16* __restrict__ dx, DwGeom g, fedmi::BnSums bs) {
  extern __shared__ float wl[];
  const int VC = g.C >> 3;
  stage_taps(w, wl, g.C, g.R * g.S);
  __syncthreads();
  const bool bsum = bs.rep != nullptr;
  float bq[3][8], bm[3][8], bi[3][8];
  fedmi::bnsum_coeffs(bs, (int)(threadIdx.x % VC) * 8, bsum, bm, bi, bq);
  const long total = (long)g.N * g.H * g.W * VC;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = i / (uint32_t)VC;
    const int c0 = (int)(i - pix * VC) * 8;
    const uint32_t t2 = pix / (uint32_t)g.W;
    const int wq = (int)(pix - t2 * g.W);
    const int n = (int)(t2 / (uint32_t)g.H), h = (int)(t2 - (uint32_t)n * g.H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const long nb = (long)n * g.P;
    if (g.R == 3 && g.st == 1) {   // unrolled: all taps in flight
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int y = h + g.pad - r;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int xx = wq + g.pad - s;
          const bool ok = (unsigned)y < (unsigned)g.P && (unsigned)xx < (unsigned)g.Q;
          float v[8];
          ld8f(dy + (ok ? ((nb + y) * g.Q + xx) * g.C + c0 : c0), v);
          const float* wt = wl + (r * 3 + s) * g.C + c0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += ok ? v[j] * wt[j] : 0.f;
        }
      }
    } else {
      for (int r = 0; r < g.R; ++r) {
        int y = h + g.pad - r;
        if (y < 0 || y % g.st) continue;
        y /= g.st;
        if (y >= g.P) continue;
        for (int s = 0; s < g.S; ++s) {
          int xx = wq + g.pad - s;
          if (xx < 0 || xx % g.st) continue;
          xx /= g.st;
          if (xx >= g.Q) continue;
          float v[8];
          ld8f(dy + ((nb + y) * g.Q + xx) * g.C + c0, v);
          const float* wt = wl + (r * g.S + s) * g.C + c0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += v[j] * wt[j];
        }
      }
    }
    bf16x8v o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)acc[j];
    *reinterpret_cast<bf16x8v*>(dx + (long)pix * g.C + c0) = o;
    if (bsum) fedmi::bnsum_acc(bs, (long)pix * g.C + c0, o, bm, bi, bq);
  }
  if (!bsum) return;
  float* red = wl + g.C * g.R * g.S;   // [3][blockDim][8]
  const int tb = blockDim.x;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(q * tb + threadIdx.x) * 8 + j] = bq[q][j];
  __syncthreads();
  const int nq = bs.zb ? 3 : 2;
  for (int e = threadIdx.x; e < nq * g.C; e += tb) {
    const int q = e / g.C, c = e - q * g.C, grp = c >> 3, j = c & 7;
    float sum = 0.f;
    for (int t = grp; t < tb; t += VC) sum += red[(q * tb + t) * 8 + j];
    unsafeAtomicAdd(bs.rep + ((long)(blockIdx.x % bs.reps) * 3 + q) * g.C + c, (double)sum);
  }
}

// 3x3 / stride 2 / pad 1 DGRAD, one thread per (2x2 block of dX, 8-channel group): the block's four input
// pixels draw on the same four dY pixels (i, j), (i, j+1), (i+1, j), (i+1, j+1) --
//   dx[2i][2j]     = dy[i][j] w11
//   dx[2i][2j+1]   = dy[i][j+1] w10 + dy[i][j] w12
//   dx[2i+1][2j]   = dy[i+1][j] w01 + dy[i][j] w21
//   dx[2i+1][2j+1] = dy[i+1][j+1] w00 + dy[i+1][j] w02 + dy[i][j+1] w20 + dy[i][j] w22
// -- so 4 loads feed 4 outputs with no per-tap parity test (dw_dgrad_kernel's generic path walks all 9 taps
// per output behind divergent stride checks: 4x the forward's time).  Taps are summed in dw_dgrad_kernel's
// (r, s) order; same BN-sums epilogue.
__global__ __launch_bounds__(256) void dw_dgrad3s2_kernel(const bf16* __restrict__ dy, const float* __restrict__ w,
                                                          bf16* __restrict__ dx, DwGeom g, fedmi::BnSums bs) {
  extern __shared__ float wl[];
  const int VC = g.C >> 3;
  stage_taps(w, wl, g.C, 9);
  __syncthreads();
  const bool bsum = bs.rep != nullptr;
  float bq[3][8], bm[3][8], bi[3][8];
  const int c0 = (int)(threadIdx.x % VC) * 8;
  fedmi::bnsum_coeffs(bs, c0, bsum, bm, bi, bq);
  const float* wc = wl + c0;   // tap t, channel k: wc[t * C + k]
  const uint32_t total = (uint32_t)g.N * g.P * g.Q * VC;
  for (uint32_t it = blockIdx.x * blockDim.x + threadIdx.x; it < total; it += gridDim.x * blockDim.x) {
    const uint32_t cell = it / (uint32_t)VC;
    const uint32_t t2 = cell / (uint32_t)g.Q;
    const int j = (int)(cell - t2 * g.Q);
    const int n = (int)(t2 / (uint32_t)g.P), i = (int)(t2 - (uint32_t)n * g.P);
    const bool okr = i + 1 < g.P, okc = j + 1 < g.Q;
    const long b00 = (((long)n * g.P + i) * g.Q + j) * g.C + c0;
    float d00[8], d01[8], d10[8], d11[8];
    ld8f(dy + b00, d00);
    ld8f(dy + (okc ? b00 + g.C : b00), d01);
    ld8f(dy + (okr ? b00 + (long)g.Q * g.C : b00), d10);
    ld8f(dy + (okr && okc ? b00 + (long)(g.Q + 1) * g.C : b00), d11);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d01[k] = okc ? d01[k] : 0.f;
      d10[k] = okr ? d10[k] : 0.f;
      d11[k] = okr && okc ? d11[k] : 0.f;
    }
    // taps: t = r * 3 + s
    const int C = g.C;
    float a[4][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a[0][k] = 0.f + d00[k] * wc[4 * C + k];
      a[1][k] = 0.f + d01[k] * wc[3 * C + k];
      a[1][k] += d00[k] * wc[5 * C + k];
      a[2][k] = 0.f + d10[k] * wc[1 * C + k];
      a[2][k] += d00[k] * wc[7 * C + k];
      a[3][k] = 0.f + d11[k] * wc[0 * C + k];
      a[3][k] += d10[k] * wc[2 * C + k];
      a[3][k] += d01[k] * wc[6 * C + k];
      a[3][k] += d00[k] * wc[8 * C + k];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = 2 * i + (q >> 1), ww = 2 * j + (q & 1);
      if (h >= g.H || ww >= g.W) continue;
      const long pix = ((long)n * g.H + h) * g.W + ww;
      bf16x8v o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (bf16)a[q][k];
      *reinterpret_cast<bf16x8v*>(dx + pix * g.C + c0) = o;
      if (bsum) fedmi::bnsum_acc(bs, pix * g.C + c0, o, bm, bi, bq);
    }
  }
  if (!bsum) return;
  float* red = wl + g.C * 9;   // [3][blockDim][8]
  const int tb = blockDim.x;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[(q * tb + threadIdx.x) * 8 + k] = bq[q][k];
  __syncthreads();
  const int nq = bs.zb ? 3 : 2;
  for (int e = threadIdx.x; e < nq * g.C; e += tb) {
    const int q = e / g.C, c = e - q * g.C, grp = c >> 3, k = c & 7;
    float sum = 0.f;
    for (int t = grp; t < tb; t += VC) sum += red[(q * tb + t) * 8 + k];
    unsafeAtomicAdd(bs.rep + ((long)(blockIdx.x % bs.reps) * 3 + q) * g.C + c, (double)sum);
  }
}

// 3x3 / stride 1 / pad 1 DGRAD, register-blocked like dw_fwd3_kernel<1>: one thread per (2 horizontally adjacent
// dX pixels, 8-channel group); the 3 x 4 dY pixels they draw on are loaded once (6 loads per output instead of
// 9).  dx[h][w] = sum_{r,s} dy[h+1-r][w+1-s] w[r][s], taps summed in dw_dgrad_kernel's (r, s) order; same BN-sums
// epilogue.
__global__ __launch_bounds__(256) void dw_dgrad3s1_kernel(const bf16* __restrict__ dy, const float* __restrict__ w,
                                                          bf16* __restrict__ dx, DwGeom g, fedmi::BnSums bs) {
  extern __shared__ float wl[];
  const int VC = g.C >> 3;
  stage_taps(w, wl, g.C, 9);
  __syncthreads();
  const bool bsum = bs.rep != nullptr;
  float bq[3][8], bm[3][8], bi[3][8];
  const int c0 = (int)(threadIdx.x % VC) * 8;
  fedmi::bnsum_coeffs(bs, c0, bsum, bm, bi, bq);
  const int W2 = (g.W + 1) >> 1;
  const uint32_t total = (uint32_t)g.N * g.H * W2 * VC;
  for (uint32_t it = blockIdx.x * blockDim.x + threadIdx.x; it < total; it += gridDim.x * blockDim.x) {
    const uint32_t pr = it / (uint32_t)VC;
    const uint32_t t2 = pr / (uint32_t)W2;
    const int w0 = (int)(pr - t2 * W2) * 2;
    const int n = (int)(t2 / (uint32_t)g.H), h = (int)(t2 - (uint32_t)n * g.H);
    float a0[8], a1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a0[k] = a1[k] = 0.f;
    const long nb = (long)n * g.P;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int yy = h + 1 - r;
      const bool rok = (unsigned)yy < (unsigned)g.P;
      float v[4][8];   // dY columns w0-1 .. w0+2
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int xx = w0 - 1 + k;
        const bool ok = rok && (unsigned)xx < (unsigned)g.Q;
        ld8f(dy + (ok ? ((nb + yy) * g.Q + xx) * g.C + c0 : c0), v[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = ok ? v[k][j] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const float* wt = wl + (r * 3 + s) * g.C + c0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a0[j] += v[2 - s][j] * wt[j];
          a1[j] += v[3 - s][j] * wt[j];
        }
      }
    }
    const long pix0 = ((long)n * g.H + h) * g.W + w0;
    bf16x8v o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)a0[j];
    *reinterpret_cast<bf16x8v*>(dx + pix0 * g.C + c0) = o;
    if (bsum) fedmi::bnsum_acc(bs, pix0 * g.C + c0, o, bm, bi, bq);
    if (w0 + 1 < g.W) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)a1[j];
      *reinterpret_cast<bf16x8v*>(dx + (pix0 + 1) * g.C + c0) = o;
      if (bsum) fedmi::bnsum_acc(bs, (pix0 + 1) * g.C + c0, o, bm, bi, bq);
    }
  }
  if (!bsum) return;
  float* red = wl + g.C * 9;   // [3][blockDim][8]
  const int tb = blockDim.x;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[(q * tb + threadIdx.x) * 8 + k] = bq[q][k];
  __syncthreads();
  const int nq = bs.zb ? 3 : 2;
  for (int e = threadIdx.x; e < nq * g.C; e += tb) {
    const int q = e / g.C, c = e - q * g.C, grp = c >> 3, k = c & 7;
    float sum = 0.f;
    for (int t = grp; t < tb; t += VC) sum += red[(q * tb + t) * 8 + k];
    unsafeAtomicAdd(bs.rep + ((long)(blockIdx.x % bs.reps) * 3 + q) * g.C + c, (double)sum);
  }
}

// Sum acc over the pstep threads of the block that share a channel group (LDS, one tap at a
// time) and write this block's partial ws[blockIdx.x][C][RS] for the chunk's channels.
template <int RS>
__device__ __forceinline__ void wgrad_block_reduce(const float (&acc)[RS][8], float* __restrict__ ws, const DwGeom& g,
                                                   int VCB) {
  __shared__ float red[256][8];
  float* out = ws + (long)blockIdx.x * g.C * RS;
#pragma unroll
  for (int t = 0; t < RS; ++t) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = acc[t][j];
    __syncthreads();
    for (int c = threadIdx.x; c < VCB * 8; c += blockDim.x) {
      const int grp = c >> 3, j = c & 7;
      float sum = 0.f;
      for (int tt = grp; tt < (int)blockDim.x; tt += VCB) sum += red[tt][j];
      out[(long)(blockIdx.y * VCB * 8 + c) * RS + t] = sum;
    }
    __syncthreads();
  }
}

// Partial weight gradients: block (b, chunk) sums a contiguous range of output pixels for
// the VCB channel groups of its chunk (thread -> fixed group), writes ws[b][C][RS] for those
// channels.  Wide layers are split into channel chunks so that small-spatial / many-channel
// layers still launch ~100+ workgroups (round 1: 8 workgroups for MobileNet's 2x2x1024 layer).
template <int RS>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                       float* __restrict__ ws, DwGeom g, int pix_per_block, int VCB) {
  const int VC = VCB;        // channel groups of this block's chunk; host: blockDim.x % VCB == 0
  const int cg = threadIdx.x % VC, lane_pix = threadIdx.x / VC, pstep = blockDim.x / VC;
  const int c0 = blockIdx.y * VCB * 8 + cg * 8;
  const long npix = (long)g.N * g.P * g.Q;
  const long pb = (long)blockIdx.x * pix_per_block, pe = std::min<long>(npix, pb + pix_per_block);
  float acc[RS][8];
#pragma unroll
  for (int t = 0; t < RS; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  for (uint32_t pix = (uint32_t)(pb + lane_pix); pix < (uint32_t)pe; pix += pstep) {
    const uint32_t t2 = pix / (uint32_t)g.Q;
    const int q = (int)(pix - t2 * g.Q);
    const int n = (int)(t2 / (uint32_t)g.P), p = (int)(t2 - (uint32_t)n * g.P);
    float d[8];
    ld8f(dy + (long)pix * g.C + c0, d);
#pragma unroll
    for (int t = 0; t < RS; ++t) {
      const int r = t / g.S, s = t - r * g.S;
      const int h = p * g.st - g.pad + r, ww = q * g.st - g.pad + s;
      const bool ok = (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
      float v[8];
      ld8f(x + (ok ? (((long)n * g.H + h) * g.W + ww) * g.C + c0 : c0), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[t][j] += ok ? v[j] * d[j] : 0.f;
    }
  }
  wgrad_block_reduce<RS>(acc, ws, g, VCB);
}

// Row-pair 3x3 wgrad (pad 1, stride ST): a thread takes two horizontally adjacent output
// pixels per step, so the 3 x (ST==1 ? 4 : 5) input columns they share are loaded once:
// 2 + 12 (15) loads for 18 tap updates instead of 2 x 10.  Pixel blocks range over pairs.
// The launcher uses it for stride 1 only (see dw_wgrad_pair).
template <int ST>
__global__ __launch_bounds__(256) void dw_wgrad3_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        float* __restrict__ ws, DwGeom g, int pairs_per_block,
                                                        int VCB) {
  constexpr int NCOL = ST == 1 ? 4 : 5;
  const int VC = VCB;
  const int cg = threadIdx.x % VC, lane_pix = threadIdx.x / VC, pstep = blockDim.x / VC;
  const int c0 = blockIdx.y * VCB * 8 + cg * 8;
  const int Q2 = (g.Q + 1) >> 1;
  const long npair = (long)g.N * g.P * Q2;
  const long pb = (long)blockIdx.x * pairs_per_block, pe = std::min<long>(npair, pb + pairs_per_block);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  for (uint32_t pr = (uint32_t)(pb + lane_pix); pr < (uint32_t)pe; pr += pstep) {
    const uint32_t t2 = pr / (uint32_t)Q2;
    const int q0 = (int)(pr - t2 * Q2) * 2;
    const int n = (int)(t2 / (uint32_t)g.P), p = (int)(t2 - (uint32_t)n * g.P);
    const long pix0 = ((long)n * g.P + p) * g.Q + q0;
    const bool q1ok = q0 + 1 < g.Q;
    float d0[8], d1[8];
    ld8f(dy + pix0 * g.C + c0, d0);
    ld8f(dy + (q1ok ? pix0 + 1 : pix0) * g.C + c0, d1);
#pragma unroll
    for (int j = 0; j < 8; ++j) d1[j] = q1ok ? d1[j] : 0.f;
    const long nb = (long)n * g.H;
    const int w0 = q0 * ST - 1;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = p * ST - 1 + r;
      const bool hok = (unsigned)h < (unsigned)g.H;
      float v[NCOL][8];
#pragma unroll
      for (int k = 0; k < NCOL; ++k) {
        const int ww = w0 + k;
        const bool ok = hok && (unsigned)ww < (unsigned)g.W;
        ld8f(x + (ok ? ((nb + h) * g.W + ww) * g.C + c0 : c0), v[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = ok ? v[k][j] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[r * 3 + s][j] += v[s][j] * d0[j] + v[ST + s][j] * d1[j];
    }
  }
  wgrad_block_reduce<9>(acc, ws, g, VCB);
}

// dw[i] (+)= sum_b ws[b][i] (body: wgrad_reduce.h wred_dw_body)
__global__ __launch_bounds__(256) void dw_wgrad_reduce(const float* __restrict__ ws, int nblk, int n,
                                                       float* __restrict__ dw, int accumulate) {
  __shared__ float part[16 * 17];
  fedmi::wred_dw_body(part, blockIdx.x, ws, nblk, n, dw, accumulate);
}

int blocks_for(long items, int tb = 256) { return (int)std::max<long>(1, std::min<long>((items + tb - 1) / tb, 4096)); }

// largest multiple of C/8 that fits in 256 threads
int block_threads(int C) { const int vc = C / 8; return (256 / vc) * vc; }

}  // namespace

namespace fedmi {

struct DwShape {
  int N, H, W, C, R, S, st, pad;
};

static DwGeom dw_geom(const DwShape& s) {
  if (s.C % 8 || s.C / 8 > 256) throw std::invalid_argument("dwconv: need C % 8 == 0 and C <= 2048");
  if (s.R != s.S || (s.R != 3 && s.R != 5 && s.R != 7)) throw std::invalid_argument("dwconv: square 3/5/7 kernels");
  if ((long)s.C * s.R * s.S * 4 > 128 * 1024) throw std::invalid_argument("dwconv: filter image exceeds LDS");
  if ((long)s.N * s.H * s.W * s.C >= (1l << 31)) throw std::invalid_argument("dwconv: tensor too large for 32-bit indexing");
  DwGeom g{s.N, s.H, s.W, s.C, (s.H + 2 * s.pad - s.R) / s.st + 1, (s.W + 2 * s.pad - s.S) / s.st + 1,
           s.R, s.S, s.st, s.pad};
  return g;
}

// w: fp32 [C][1][R][S] (PyTorch depthwise layout, used directly)
void launch_dw_fwd(hipStream_t st, const DwShape& s, const bf16* x, const float* w, bf16* y, double* stats,
                   const float* shift) {
  const DwGeom g = dw_geom(s);
  const int tb = block_threads(g.C);
  if (g.R == 3 && (g.st == 1 || g.st == 2) && g.pad == 1) {   // the MobileNet family: row-pair kernel
    const long items = (long)g.N * g.P * ((g.Q + 1) / 2) * (g.C / 8);
    const size_t lds = (size_t)g.C * 9 * sizeof(float);
    if (g.st == 1)
      hipLaunchKernelGGL(dw_fwd3_kernel<1>, dim3(blocks_for(items, tb)), dim3(tb), lds, st, x, w, y, stats, shift, g);
    else
      hipLaunchKernelGGL(dw_fwd3_kernel<2>, dim3(blocks_for(items, tb)), dim3(tb), lds, st, x, w, y, stats, shift, g);
    return;
  }
  const long items = (long)g.N * g.P * g.Q * (g.C / 8);
  hipLaunchKernelGGL(dw_fwd_kernel, dim3(blocks_for(items, tb)), dim3(tb), g.C * g.R * g.S * sizeof(float), st, x, w,
                     y, stats, shift, g);
}

// bs: optional BN-backward sums of dx's producer (see dw_dgrad_kernel); fewer, longer workgroups then
// (their per-channel fp64 atomics land on 2-3 x C x reps addresses)
void launch_dw_dgrad(hipStream_t st, const DwShape& s, const bf16* dy, const float* w, bf16* dx,
                     const BnSums* bs) {
  const DwGeom g = dw_geom(s);
  if (bs && (!bs->rep || !bs->z || !bs->mean || !bs->inv || bs->reps < 1 || (bs->zb && (!bs->meanb || !bs->invb)) ||
             (bs->msc && (bs->y || bs->msc_ld <= 0))))
    throw std::invalid_argument("dw_dgrad: incomplete BN sums descriptor");
  const int tb = block_threads(g.C);
  const size_t lds = g.C * g.R * g.S * sizeof(float) + (bs ? 3 * tb * 8 * sizeof(float) : 0);
  if (g.R == 3 && g.st == 2 && g.pad == 1) {   // 2x2 dX blocks (dw_dgrad3s2_kernel): H <= 2P, W <= 2Q always
    const long items = (long)g.N * g.P * g.Q * (g.C / 8);
    const int nblk = bs ? std::min(blocks_for(items, tb), 2048) : blocks_for(items, tb);
    hipLaunchKernelGGL(dw_dgrad3s2_kernel, dim3(nblk), dim3(tb), lds, st, dy, w, dx, g, bs ? *bs : BnSums{});
    return;
  }
  if (g.R == 3 && g.st == 1 && g.pad == 1) {   // row pairs (dw_dgrad3s1_kernel)
    const long items = (long)g.N * g.H * ((g.W + 1) / 2) * (g.C / 8);
    const int nblk = bs ? std::min(blocks_for(items, tb), 2048) : blocks_for(items, tb);
    hipLaunchKernelGGL(dw_dgrad3s1_kernel, dim3(nblk), dim3(tb), lds, st, dy, w, dx, g, bs ? *bs : BnSums{});
    return;
  }
  const long items = (long)g.N * g.H * g.W * (g.C / 8);
  const int nblk = bs ? std::min(blocks_for(items, tb), 2048) : blocks_for(items, tb);
  hipLaunchKernelGGL(dw_dgrad_kernel, dim3(nblk), dim3(tb), lds, st, dy, w, dx, g, bs ? *bs : BnSums{});
}

// channel groups per wgrad workgroup (<= 32: >= 8 pixel lanes) and pixel blocks (>= 2 pixels per lane)
static int dw_wgrad_vcb(const DwGeom& g) {   // largest divisor of C/8 that is <= 32
  const int vc = g.C / 8;
  for (int d = std::min(vc, 32); d > 1; --d)
    if (vc % d == 0) return d;
  return 1;
}
// stride 1 only: at stride 2 the pair shares 3 of 5 columns, and measured slower (MobileNet 37 -> 64 us)
static bool dw_wgrad_pair(const DwGeom& g) { return g.R == 3 && g.st == 1 && g.pad == 1; }
static long dw_wgrad_items(const DwGeom& g) {   // output pixels, or pixel pairs for the row-pair kernel
  return dw_wgrad_pair(g) ? (long)g.N * g.P * ((g.Q + 1) / 2) : (long)g.N * g.P * g.Q;
}
static int dw_wgrad_blocks(const DwGeom& g) {
  const long npix = dw_wgrad_items(g);
  const int pstep = block_threads(dw_wgrad_vcb(g) * 8) / dw_wgrad_vcb(g);
  const int per_lane = dw_wgrad_pair(g) ? 1 : 2;   // a pair is already two pixels
  return (int)std::max<long>(1, std::min<long>(512, (npix + per_lane * pstep - 1) / (per_lane * pstep)));
}

long dw_wgrad_ws_floats(const DwShape& s) {
  const DwGeom g = dw_geom(s);
  return (long)dw_wgrad_blocks(g) * g.C * g.R * g.S;
}

void launch_dw_wgrad_reduce(hipStream_t st, const WredItem& e) {
  hipLaunchKernelGGL(dw_wgrad_reduce, dim3((unsigned)wred_blocks(e)), dim3(256), 0, st, e.ws, e.splits, e.C, e.dw,
                     e.accumulate);
}

// defer: fill the reduction's WredItem instead of launching it (see launch_wgrad_reduce_multi)
void launch_dw_wgrad(hipStream_t st, const DwShape& s, const bf16* x, const bf16* dy, float* dw, float* ws,
                     long ws_floats, int accumulate, WredItem* defer) {
  const DwGeom g = dw_geom(s);
  const int nblk = dw_wgrad_blocks(g);
  const int n = g.C * g.R * g.S;
  if ((long)nblk * n > ws_floats) throw std::invalid_argument("dw_wgrad: workspace too small");
  const long npix = dw_wgrad_items(g);
  const int ppb = (int)((npix + nblk - 1) / nblk);
  const int vcb = dw_wgrad_vcb(g);
  const int tb = block_threads(vcb * 8);
  const dim3 grid(nblk, (g.C / 8) / vcb);
  if (dw_wgrad_pair(g))
    hipLaunchKernelGGL(dw_wgrad3_kernel<1>, grid, dim3(tb), 0, st, x, dy, ws, g, ppb, vcb);
  else if (g.R == 3) hipLaunchKernelGGL(dw_wgrad_kernel<9>, grid, dim3(tb), 0, st, x, dy, ws, g, ppb, vcb);
  else if (g.R == 5) hipLaunchKernelGGL(dw_wgrad_kernel<25>, grid, dim3(tb), 0, st, x, dy, ws, g, ppb, vcb);
  else hipLaunchKernelGGL(dw_wgrad_kernel<49>, grid, dim3(tb), 0, st, x, dy, ws, g, ppb, vcb);
  WredItem it{};
  it.ws = ws; it.dw = dw; it.kind = WRED_DW; it.splits = nblk; it.C = n; it.accumulate = accumulate;
  if (defer) *defer = it;
  else launch_dw_wgrad_reduce(st, it);
}

}  // namespace fedmi
