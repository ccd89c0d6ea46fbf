// Weight-gradient partial reductions shared by the standalone reduce kernels (conv_igemm.hip conv_wgrad_reduce /
// conv_wgrad_reduce_cols, dwconv.hip dw_wgrad_reduce) and the deferred multi-reduce (conv_igemm.hip
// wgrad_reduce_multi): the same device bodies, so a deferred reduction is bit-identical to the immediate one.
// Every body is a 256-thread workgroup `bx` of its own launch grid; `lds` is the workgroup's scratch.
#pragma once

#include <hip/hip_runtime.h>

namespace fedmi {

// dW[o][c][r][s] (+)= sum_z ws[z][o][(r*S + s)*C + c]     (c < Cw)
// Block = one output channel o x 64 input channels, all R*S taps, 4 split groups: each wave reads 256 contiguous
// bytes per (tap, split), the groups combine in LDS in a fixed order (deterministic), and the block writes its
// 64 x RS results as ONE contiguous run of dW[o][c0:c0+64][:][:].  lds: [4][RS][65] floats.
__device__ __forceinline__ void wred_tile_body(float* __restrict__ part_, int bx, const float* __restrict__ ws,
                                               int splits, int O, int C, int Cw, int RS, float* __restrict__ dw,
                                               int accumulate, int Ow, int G) {
  auto part = [&](int zg, int rs, int ci) -> float& { return part_[(zg * RS + rs) * 65 + ci]; };
  const long plane = (long)O * RS * C;
  const int ncb = (C + 63) / 64;
  const int o = bx / ncb, c0 = (bx % ncb) * 64;
  if (o >= Ow) return;                             // zero-padded filters: no output row (workgroup-uniform)
  const int cl = threadIdx.x & 63, zg = threadIdx.x >> 6;
  const int c = c0 + cl;
  if (splits <= 12 && RS <= 9) {
    // <= 3 splits per group: every tap's load of a split in flight at once (the loop below has one load per
    // tap in flight); the same sequential per-tap order as the general loop takes for splits <= 12
    float v[9];
#pragma unroll
    for (int rs = 0; rs < 9; ++rs) v[rs] = 0.f;
    if (c < C) {
      const float* p = ws + (long)o * RS * C + c;
      for (int z = zg; z < splits; z += 4) {
        float t[9];
#pragma unroll
        for (int rs = 0; rs < 9; ++rs) t[rs] = rs < RS ? p[(long)z * plane + (long)rs * C] : 0.f;
#pragma unroll
        for (int rs = 0; rs < 9; ++rs) v[rs] += t[rs];
      }
    }
#pragma unroll
    for (int rs = 0; rs < 9; ++rs)
      if (rs < RS) part(zg, rs, cl) = v[rs];
  } else {
    for (int rs = 0; rs < RS; ++rs) {
      float v = 0.f;
      if (c < C) {
        const float* p = ws + ((long)o * RS + rs) * C + c;
        int z = zg;
        for (; z + 12 < splits; z += 16) {   // 4 independent loads in flight per lane
          const float a = p[(long)z * plane], b = p[(long)(z + 4) * plane];
          const float cc = p[(long)(z + 8) * plane], d = p[(long)(z + 12) * plane];
          v += (a + b) + (cc + d);
        }
        for (; z < splits; z += 4) v += p[(long)z * plane];
      }
      part(zg, rs, cl) = v;
    }
  }
  __syncthreads();
  // this filter's channels: [cg0, cg0 + Cw) (G > 1: the block-diagonal group of a densified grouped conv)
  const int cg0 = G > 1 ? (o / (O / G)) * Cw : 0;
  const int lo = max(c0, cg0), hi = min(c0 + 64, cg0 + Cw);
  if (hi <= lo) return;
  float* out = dw + ((long)o * Cw + (lo - cg0)) * RS;
  for (int e = threadIdx.x; e < (hi - lo) * RS; e += 256) {
    const int ci = e / RS + (lo - c0), rs = e - (e / RS) * RS;
    const float s = (part(0, rs, ci) + part(1, rs, ci)) + (part(2, rs, ci) + part(3, rs, ci));
    out[e] = accumulate ? out[e] + s : s;
  }
}

// Column-mapped variant (one lane per workspace column, scattered stores): more workgroups, so it wins when the
// plane is small and the split count large (ResNet-18's 64-channel layers).  Block = 64 consecutive workspace
// columns x 4 split groups: every wave reads 256 contiguous bytes per split (the workspace is read exactly once,
// fully coalesced), the 4 groups are combined in LDS, and the 64 sums are written to their permuted [O][Cw][R][S]
// positions.  Deterministic (fixed order).  lds: [4][64] floats.
__device__ __forceinline__ void wred_cols_body(float* __restrict__ part, int bx, const float* __restrict__ ws,
                                               int splits, int O, int C, int Cw, int RS, float* __restrict__ dw,
                                               int accumulate, int Ow, int G) {
  const long plane = (long)O * RS * C;
  const long e = (long)bx * 64 + (threadIdx.x & 63);
  const int zg = threadIdx.x >> 6;
  float v = 0.f;
  if (e < plane) {
    const float* p = ws + e;
    int z = zg;
    for (; z + 12 < splits; z += 16) {   // 4 independent loads in flight per lane
      const float a = p[(long)z * plane], b = p[(long)(z + 4) * plane];
      const float c = p[(long)(z + 8) * plane], d = p[(long)(z + 12) * plane];
      v += (a + b) + (c + d);
    }
    for (; z < splits; z += 4) v += p[(long)z * plane];
  }
  part[zg * 64 + (threadIdx.x & 63)] = v;
  __syncthreads();
  if (threadIdx.x < 64 && e < plane) {
    const int l = threadIdx.x;
    const float s = (part[l] + part[64 + l]) + (part[128 + l] + part[192 + l]);
    const long t = e / C;
    const int rs = (int)(t % RS), o = (int)(t / RS);
    const int c = (int)(e % C) - (G > 1 ? (o / (O / G)) * Cw : 0);   // channel within filter o's group
    if (c >= 0 && c < Cw && o < Ow) {
      const long i = ((long)o * Cw + c) * RS + rs;
      dw[i] = accumulate ? dw[i] + s : s;
    }
  }
}

// Depthwise: dw[i] (+)= sum_b ws[b][i].  Block = 16 outputs x 16 partial groups (each thread sums nblk/16
// partials, 4 loads in flight), fixed-order LDS combine.  lds: [16][17] floats.
__device__ __forceinline__ void wred_dw_body(float* __restrict__ part, int bx, const float* __restrict__ ws, int nblk,
                                             int n, float* __restrict__ dw, int accumulate) {
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int i = bx * 16 + col;
  float a = 0.f, b = 0.f, c = 0.f, d = 0.f;
  if (i < n) {
    int k = grp;
    for (; k + 48 < nblk; k += 64) {
      a += ws[(long)k * n + i];
      b += ws[(long)(k + 16) * n + i];
      c += ws[(long)(k + 32) * n + i];
      d += ws[(long)(k + 48) * n + i];
    }
    for (; k < nblk; k += 16) a += ws[(long)k * n + i];
  }
  part[grp * 17 + col] = (a + b) + (c + d);
  __syncthreads();
  if (threadIdx.x < 16 && i < n) {
    float v = 0.f;
#pragma unroll
    for (int g2 = 0; g2 < 16; ++g2) v += part[g2 * 17 + col];
    dw[i] = accumulate ? dw[i] + v : v;
  }
}

// One deferred reduction (the arguments its standalone launch would have taken).
enum WredKind : int { WRED_TILE = 0, WRED_COLS = 1, WRED_DW = 2 };
struct WredItem {
  const float* ws;
  float* dw;
  int kind;                    // WredKind
  int splits;                  // WRED_DW: partial blocks (nblk)
  int O, C, Cw, RS;            // WRED_DW: C = n (elements), the rest unused
  int accumulate, Ow, G;
};

inline long wred_blocks(const WredItem& e) {
  if (e.kind == WRED_TILE) return (long)e.O * ((e.C + 63) / 64);
  if (e.kind == WRED_COLS) return ((long)e.O * e.RS * e.C + 63) / 64;
  return (e.C + 15) / 16;
}
inline size_t wred_lds_bytes(const WredItem& e) {
  if (e.kind == WRED_TILE) return (size_t)4 * e.RS * 65 * sizeof(float);
  if (e.kind == WRED_COLS) return 4 * 64 * sizeof(float);
  return 16 * 17 * sizeof(float);
}

// launchers (conv_igemm.hip / dwconv.hip)
void launch_wgrad_reduce_multi(hipStream_t st, const WredItem* items, int n);
void launch_dw_wgrad_reduce(hipStream_t st, const WredItem& e);

}  // namespace fedmi
