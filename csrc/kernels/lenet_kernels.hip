// fedmi — fused LeNet training/eval kernels for MI355X (gfx950, CDNA4).
//
// One local SGD step of the reference (src/main.py:146-151: zero_grad,
// forward, CE loss, backward, SGD(m=0.9, wd=5e-4)) is FOUR launches:
//
//   K1 lenet_conv_fwd   one workgroup per sample: uint8 image -> on-device
//                       RandomCrop(32,pad4)+HFlip+Normalize (src/main.py:37-42)
//                       -> conv1 (MFMA) +bias+ReLU -> maxpool2 -> conv2 (MFMA)
//                       +bias+ReLU -> maxpool2, all staged in LDS.  Saves the
//                       pooled activations and 2-bit argmax codes for backward.
//   K2 lenet_fc_head    32 samples per workgroup: fc1/fc2/fc3 forward (MFMA),
//                       cross-entropy + accuracy counters, full FC backward
//                       (dgrad + wgrad on MFMA) -> per-workgroup grad slab and
//                       d(pool2) for K3.  Also the eval head (train=0).
//   K3 lenet_conv_bwd   one workgroup per sample: maxpool/ReLU backward by the
//                       saved argmax, conv2 wgrad + dgrad, conv1 wgrad (MFMA),
//                       bias grads -> per-sample grad slab.
//   K4 lenet_sgd        reduces the grad slabs (split-K combine at the kernel
//                       boundary: deterministic, no atomics), applies
//                       wd/momentum/lr to the fp32 master weights and rewrites
//                       the packed bf16 MFMA operand images.
//
// The whole local epoch is replayed from a hipGraph built by the native
// executor (csrc/runtime/lenet_engine.cpp), so the host issues one launch per
// round instead of 4 x #batches.
#include "common.h"
#include "lenet_layout.h"

using namespace lenet;

namespace {

__constant__ float kMean[3] = {0.4914f, 0.4822f, 0.4465f};
__constant__ float kInvStd[3] = {1.f / 0.2023f, 1.f / 0.1994f, 1.f / 0.2010f};

// Stage one CIFAR uint8 image into LDS (raw), then augment + normalize into a
// bf16 [3][32][32] image.  Reference transform: src/main.py:36-46.
// RandomCrop(32, padding=4) pads with pixel value 0 *before* ToTensor/Normalize,
// so an out-of-image pixel becomes (0 - mean)/std.
FEDMI_DEV void stage_image(const uint8_t* __restrict__ img, uint8_t* raw, bf16* xs,
                           int augment, uint32_t h) {
  const int tid = threadIdx.x;
  if (tid < IMG_BYTES / 16) {
    reinterpret_cast<uint4*>(raw)[tid] = reinterpret_cast<const uint4*>(img)[tid];
  }
  __syncthreads();
  int i0 = 4, j0 = 4, flip = 0;
  if (augment) {
    i0 = (int)(h % 9u);
    j0 = (int)((h >> 8) % 9u);
    flip = (int)((h >> 16) & 1u);
  }
  for (int e = tid; e < IMG_BYTES; e += blockDim.x) {
    const int c = e >> 10, y = (e >> 5) & 31, x = e & 31;
    const int sy = y + i0 - 4;
    const int sx = (flip ? 31 - x : x) + j0 - 4;
    float v = 0.f;
    if (sy >= 0 && sy < IMG && sx >= 0 && sx < IMG) v = (float)raw[c * 1024 + sy * 32 + sx] * (1.f / 255.f);
    xs[e] = (bf16)((v - kMean[c]) * kInvStd[c]);
  }
}

FEDMI_DEV bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

}  // namespace

// ---------------------------------------------------------------------------
// K1: conv stack forward, one workgroup (4 waves) per sample.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lenet_conv_fwd(
    const uint8_t* __restrict__ images, int sample_base, int nb,
    const bf16* __restrict__ pk, const float* __restrict__ params,
    uint32_t seed, const int* __restrict__ round_ctr, int augment,
    bf16* __restrict__ act2,        // [nb][F0P]
    bf16* __restrict__ act2T,       // [F0P][tstride] (train) or null
    int tstride,
    bf16* __restrict__ pool1_out,   // [nb][NP1] or null
    uint8_t* __restrict__ am1_out,  // [nb][NP1] or null
    uint8_t* __restrict__ am2_out)  // [nb][F0]  or null
{
  __shared__ __attribute__((aligned(16))) unsigned char smem[3072 + 6144 + 18816 + 2368 + 6400];
  uint8_t* raw = smem;
  bf16* xs = reinterpret_cast<bf16*>(smem + 3072);
  float* c1 = reinterpret_cast<float*>(smem + 3072 + 6144);
  bf16* p1 = reinterpret_cast<bf16*>(smem + 3072 + 6144 + 18816);
  float* c2 = reinterpret_cast<float*>(smem + 3072 + 6144 + 18816 + 2368);

  const int s = blockIdx.x;
  if (s >= nb) return;
  const int gidx = sample_base + s;
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8;
  const int n16 = lane & 15;

  const uint32_t h = augment ? hash3(seed, (uint32_t)round_ctr[0], (uint32_t)gidx) : 0u;
  stage_image(images + (size_t)gidx * IMG_BYTES, raw, xs, augment, h);

  // conv1 B fragments (weights) stay in registers for all 49 tiles.
  bf16x8 wb1[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) wb1[ks] = ld8(pk + PK_W1C + n16 * K1P + ks * 32 + kq);
  int offs1[24];
#pragma unroll
  for (int q = 0; q < 24; ++q) {
    const int k = (q >> 3) * 32 + kq + (q & 7);
    const int c = k / 25, rs = k - c * 25, r = rs / 5, sc = rs - r * 5;
    offs1[q] = (k < K1) ? c * 1024 + r * 32 + sc : 0;   // pad k -> any finite pixel (weight is 0)
  }
  __syncthreads();

  // ---- conv1: M = 784 positions (49 tiles), N = 6 (pad 16), K = 75 (pad 96)
  {
    const float bias = n16 < C1 ? params[P_C1B + n16] : 0.f;
    for (int t = wave; t < NPOS1 / 16; t += 4) {
      const int pos = t * 16 + n16;
      const int py = pos / O1, px = pos - py * O1;
      const bf16* xb = xs + py * IMG + px;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = xb[offs1[ks * 8 + j]];
        acc = mfma16(a, wb1[ks], acc);
      }
      if (n16 < C1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) c1[n16 * NPOS1 + t * 16 + (lane >> 4) * 4 + r] = fmaxf(acc[r] + bias, 0.f);
      }
    }
  }
  __syncthreads();

  // ---- maxpool2 #1 (+ argmax code: 0=(0,0) 1=(0,1) 2=(1,0) 3=(1,1), first max wins)
  for (int e = tid; e < NP1; e += 256) {
    const int o = e / 196, rem = e - o * 196, py = rem / P1, px = rem - py * P1;
    const float* w = c1 + o * NPOS1 + (2 * py) * O1 + 2 * px;
    float m = w[0]; int a = 0;
    if (w[1] > m) { m = w[1]; a = 1; }
    if (w[O1] > m) { m = w[O1]; a = 2; }
    if (w[O1 + 1] > m) { m = w[O1 + 1]; a = 3; }
    const bf16 mb = (bf16)m;
    p1[e] = mb;
    if (pool1_out) {
      pool1_out[(size_t)s * NP1 + e] = mb;
      am1_out[(size_t)s * NP1 + e] = (uint8_t)a;
    }
  }

  bf16x8 wb2[5];
#pragma unroll
  for (int ks = 0; ks < 5; ++ks) wb2[ks] = ld8(pk + PK_W2C + n16 * K2P + ks * 32 + kq);
  int offs2[40];
#pragma unroll
  for (int q = 0; q < 40; ++q) {
    const int k = (q >> 3) * 32 + kq + (q & 7);
    const int c = k / 25, rs = k - c * 25, r = rs / 5, sc = rs - r * 5;
    offs2[q] = (k < K2) ? c * 196 + r * P1 + sc : 0;
  }
  __syncthreads();

  // ---- conv2: M = 100 positions (7 tiles), N = 16, K = 150 (pad 160)
  {
    const float bias = params[P_C2B + n16];
    for (int t = wave; t < 7; t += 4) {
      int pos = t * 16 + n16;
      if (pos >= NPOS2) pos = 0;
      const int py = pos / O2, px = pos - py * O2;
      const bf16* pb = p1 + py * P1 + px;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = pb[offs2[ks * 8 + j]];
        acc = mfma16(a, wb2[ks], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = t * 16 + (lane >> 4) * 4 + r;
        if (p < NPOS2) c2[n16 * NPOS2 + p] = fmaxf(acc[r] + bias, 0.f);
      }
    }
  }
  __syncthreads();

  // ---- maxpool2 #2 -> flattened act2 row (torch .view order: o*25 + py*5 + px)
  for (int e = tid; e < F0P; e += 256) {
    bf16 mb = (bf16)0.f;
    if (e < F0) {
      const int o = e / 25, rem = e - o * 25, py = rem / P2, px = rem - py * P2;
      const float* w = c2 + o * NPOS2 + (2 * py) * O2 + 2 * px;
      float m = w[0]; int a = 0;
      if (w[1] > m) { m = w[1]; a = 1; }
      if (w[O2] > m) { m = w[O2]; a = 2; }
      if (w[O2 + 1] > m) { m = w[O2 + 1]; a = 3; }
      mb = (bf16)m;
      if (am2_out) am2_out[(size_t)s * F0 + e] = (uint8_t)a;
    }
    act2[(size_t)s * F0P + e] = mb;
    if (act2T) act2T[(size_t)e * tstride + s] = mb;
  }
}

// ---------------------------------------------------------------------------
// K2: FC head. 32 samples per workgroup (2 MFMA row tiles), 4 waves.
//   fwd: H1 = relu(X W1^T + b1), H2 = relu(H1 W2^T + b2), Z = H2 W3^T + b3
//   CE:  loss/acc counters; dZ = (softmax - onehot) / nb  (mean reduction)
//   bwd: dW3/db3, dH2, dW2/db2, dH1, dW1/db1, dX (masked by pool2 ReLU)
// Wgrad GEMMs reduce over the 32 samples (K = 32 = one MFMA k-step), so the
// activations are also kept sample-contiguous ("T" images) in LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lenet_fc_head(
    const bf16* __restrict__ act2,   // [nb][F0P]
    const bf16* __restrict__ act2T,  // [F0P][tstride]  (train only)
    int tstride,
    const int* __restrict__ labels,  // labels of this batch (already offset)
    int nb, int train,
    const bf16* __restrict__ pk, const float* __restrict__ params,
    float* __restrict__ dact2,       // [nb][F0]      (train)
    float* __restrict__ fc_slab,     // [grid][FS]    (train)
    Stats* __restrict__ stats)
{
  constexpr int SZ_H1 = 32 * 128, SZ_H2 = 32 * 96, SZ_Z3 = 32 * 32;
  __shared__ __attribute__((aligned(16))) bf16 sH1[SZ_H1], sH1T[SZ_H1];
  __shared__ __attribute__((aligned(16))) bf16 sH2[SZ_H2], sH2T[SZ_H2];
  __shared__ __attribute__((aligned(16))) bf16 sdZ3[SZ_Z3], sdZ3T[16 * 32];
  __shared__ __attribute__((aligned(16))) bf16 sdZ2[SZ_H2], sdZ2T[SZ_H2];
  __shared__ __attribute__((aligned(16))) bf16 sdZ1[SZ_H1], sdZ1T[SZ_H1];
  __shared__ float sZ[32 * 16];
  __shared__ float sdb[128 + 96 + 16];

  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  const int s0 = blockIdx.x * FC_SPW;
  const int ns = min(FC_SPW, nb - s0);
  if (ns <= 0) return;

  for (int e = tid; e < 240; e += 256) sdb[e] = 0.f;

  // ---- fc1 fwd: [32 x 128] = X[32 x 416] . W1p^T, 16 output tiles, K = 13 steps
  for (int q = wave; q < 16; q += 4) {
    const int m = q & 1, nt = q >> 1;
    const int srow = m * 16 + n16;
    const bool valid = srow < ns;
    const bf16* xa = act2 + (size_t)(s0 + (valid ? srow : 0)) * F0P + kq;
    const bf16* wb = pk + PK_FC1 + (nt * 16 + n16) * F0P + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < F0P / 32; ++ks) {
      const bf16x8 a = valid ? ld8(xa + ks * 32) : zero8();
      acc = mfma16(a, ld8(wb + ks * 32), acc);
    }
    const int n = nt * 16 + n16;
    const float b = n < F1 ? params[P_F1B + n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = m * 16 + rq + r;
      const float hv = (n < F1 && sr < ns) ? fmaxf(acc[r] + b, 0.f) : 0.f;
      sH1[sr * 128 + n] = (bf16)hv;
      sH1T[n * 32 + sr] = (bf16)hv;
    }
  }
  __syncthreads();

  // ---- fc2 fwd: [32 x 96] = H1[32 x 128] . W2p^T, 12 tiles, K = 4 steps
  for (int q = wave; q < 12; q += 4) {
    const int m = q & 1, nt = q >> 1;
    const bf16* ha = sH1 + (m * 16 + n16) * 128 + kq;
    const bf16* wb = pk + PK_FC2 + (nt * 16 + n16) * 128 + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) acc = mfma16(ld8(ha + ks * 32), ld8(wb + ks * 32), acc);
    const int n = nt * 16 + n16;
    const float b = n < F2 ? params[P_F2B + n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = m * 16 + rq + r;
      const float hv = (n < F2 && sr < ns) ? fmaxf(acc[r] + b, 0.f) : 0.f;
      sH2[sr * 96 + n] = (bf16)hv;
      sH2T[n * 32 + sr] = (bf16)hv;
    }
  }
  __syncthreads();

  // ---- fc3 fwd: logits [32 x 16] = H2[32 x 96] . W3p^T, 2 tiles, K = 3 steps
  if (wave < 2) {
    const int m = wave;
    const bf16* ha = sH2 + (m * 16 + n16) * 96 + kq;
    const bf16* wb = pk + PK_FC3 + n16 * 96 + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) acc = mfma16(ld8(ha + ks * 32), ld8(wb + ks * 32), acc);
    const float b = n16 < NCLS ? params[P_F3B + n16] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) sZ[(m * 16 + rq + r) * 16 + n16] = acc[r] + b;
  }
  __syncthreads();

  // ---- cross-entropy (mean over the global batch nb), accuracy, dZ
  if (wave == 0) {
    float loss = 0.f, corr = 0.f;
    const int sr = lane;
    if (sr < 32) {
      float dz[NCLS];
      const bool valid = sr < ns;
      if (valid) {
        float z[NCLS];
#pragma unroll
        for (int n = 0; n < NCLS; ++n) z[n] = sZ[sr * 16 + n];
        float mx = z[0]; int am = 0;
#pragma unroll
        for (int n = 1; n < NCLS; ++n) if (z[n] > mx) { mx = z[n]; am = n; }
        float se = 0.f;
#pragma unroll
        for (int n = 0; n < NCLS; ++n) se += __expf(z[n] - mx);
        const float lse = mx + __logf(se);
        const int y = labels[s0 + sr];
        float zy = 0.f;
#pragma unroll
        for (int n = 0; n < NCLS; ++n) zy = (n == y) ? z[n] : zy;
        loss = lse - zy;
        corr = (am == y) ? 1.f : 0.f;
        const float inv = 1.f / (float)nb;
#pragma unroll
        for (int n = 0; n < NCLS; ++n) dz[n] = (__expf(z[n] - lse) - (n == y ? 1.f : 0.f)) * inv;
      } else {
#pragma unroll
        for (int n = 0; n < NCLS; ++n) dz[n] = 0.f;
      }
      if (train) {
#pragma unroll
        for (int n = 0; n < 32; ++n) {
          const float v = n < NCLS ? dz[n < NCLS ? n : 0] : 0.f;
          sdZ3[sr * 32 + n] = (bf16)v;
          if (n < 16) sdZ3T[n * 32 + sr] = (bf16)v;
        }
#pragma unroll
        for (int n = 0; n < NCLS; ++n) sZ[sr * 16 + n] = dz[n];   // fp32 dZ for db3
      }
    }
    loss = wave_sum(loss);
    corr = wave_sum(corr);
    if (lane == 0) {
      atomicAdd(&stats->loss_sum, loss);
      atomicAdd(&stats->correct, (int)(corr + 0.5f));
      atomicAdd(&stats->count, ns);
    }
  }
  if (!train) return;
  __syncthreads();

  float* slab = fc_slab + (size_t)blockIdx.x * FS;
  constexpr int OF3W = P_F3W - P_F1W, OF2W = P_F2W - P_F1W, OF1W = 0;

  if (tid < NCLS) {   // db3
    float acc = 0.f;
    for (int sr = 0; sr < 32; ++sr) acc += sZ[sr * 16 + tid];
    sdb[224 + tid] = acc;
  }

  // ---- phase 5: dW3 (6 tiles) and dH2 = dZ3 . W3 (12 tiles)
  for (int q = wave; q < 18; q += 4) {
    if (q < 6) {
      const int ft = q;
      f32x4 acc = mfma16(ld8(sdZ3T + n16 * 32 + kq), ld8(sH2T + (ft * 16 + n16) * 32 + kq), zero4());
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = rq + r, f = ft * 16 + n16;
        if (n < NCLS && f < F2) slab[OF3W + n * F2 + f] = acc[r];
      }
    } else {
      const int qq = q - 6, m = qq & 1, ft = qq >> 1;
      const int f = ft * 16 + n16;
      f32x4 acc = mfma16(ld8(sdZ3 + (m * 16 + n16) * 32 + kq), ld8(pk + PK_FC3T + f * 32 + kq), zero4());
      float colsum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sr = m * 16 + rq + r;
        const float g = (f < F2 && (float)sH2[sr * 96 + f] > 0.f) ? acc[r] : 0.f;
        sdZ2[sr * 96 + f] = (bf16)g;
        sdZ2T[f * 32 + sr] = (bf16)g;
        colsum += g;
      }
      colsum += __shfl_xor(colsum, 16, 64);
      colsum += __shfl_xor(colsum, 32, 64);
      if (lane < 16 && f < F2) atomicAdd(&sdb[128 + f], colsum);
    }
  }
  __syncthreads();

  // ---- phase 6: dW2 = dZ2^T H1 (48 tiles) and dH1 = dZ2 . W2 (16 tiles)
  for (int q = wave; q < 64; q += 4) {
    if (q < 48) {
      const int mt = q / 8, ft = q - mt * 8;
      f32x4 acc = mfma16(ld8(sdZ2T + (mt * 16 + n16) * 32 + kq), ld8(sH1T + (ft * 16 + n16) * 32 + kq), zero4());
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = mt * 16 + rq + r, f = ft * 16 + n16;
        if (n < F2 && f < F1) slab[OF2W + n * F1 + f] = acc[r];
      }
    } else {
      const int qq = q - 48, m = qq & 1, ft = qq >> 1;
      const int f = ft * 16 + n16;
      const bf16* za = sdZ2 + (m * 16 + n16) * 96 + kq;
      const bf16* wb = pk + PK_FC2T + f * 96 + kq;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) acc = mfma16(ld8(za + ks * 32), ld8(wb + ks * 32), acc);
      float colsum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sr = m * 16 + rq + r;
        const float g = (f < F1 && (float)sH1[sr * 128 + f] > 0.f) ? acc[r] : 0.f;
        sdZ1[sr * 128 + f] = (bf16)g;
        sdZ1T[f * 32 + sr] = (bf16)g;
        colsum += g;
      }
      colsum += __shfl_xor(colsum, 16, 64);
      colsum += __shfl_xor(colsum, 32, 64);
      if (lane < 16 && f < F1) atomicAdd(&sdb[f], colsum);
    }
  }
  __syncthreads();

  // ---- phase 7: dW1 = dZ1^T X (200 tiles) and dX = dZ1 . W1 (50 tiles)
  for (int q = wave; q < 250; q += 4) {
    if (q < 200) {
      const int mt = q / 25, ft = q - mt * 25;
      const int f = ft * 16 + n16;
      f32x4 acc = mfma16(ld8(sdZ1T + (mt * 16 + n16) * 32 + kq),
                         ld8(act2T + (size_t)f * tstride + s0 + kq), zero4());
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = mt * 16 + rq + r;
        if (n < F1) slab[OF1W + n * F0 + f] = acc[r];
      }
    } else {
      const int qq = q - 200, m = qq & 1, ft = qq >> 1;
      const int f = ft * 16 + n16;
      const bf16* za = sdZ1 + (m * 16 + n16) * 128 + kq;
      const bf16* wb = pk + PK_FC1T + f * 128 + kq;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma16(ld8(za + ks * 32), ld8(wb + ks * 32), acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sr = m * 16 + rq + r;
        if (sr < ns) {
          const size_t row = (size_t)(s0 + sr);
          const float x = (float)act2[row * F0P + f];
          dact2[row * F0 + f] = x > 0.f ? acc[r] : 0.f;
        }
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < F1; e += 256) slab[P_F1B - P_F1W + e] = sdb[e];
  for (int e = tid; e < F2; e += 256) slab[P_F2B - P_F1W + e] = sdb[128 + e];
  if (tid < NCLS) slab[P_F3B - P_F1W + tid] = sdb[224 + tid];
}

// ---------------------------------------------------------------------------
// K3: conv stack backward, one workgroup per sample.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lenet_conv_bwd(
    const uint8_t* __restrict__ images, int sample_base, int nb,
    uint32_t seed, const int* __restrict__ round_ctr, int augment,
    const float* __restrict__ dact2,       // [nb][F0]
    const bf16* __restrict__ pool1,        // [nb][NP1]
    const uint8_t* __restrict__ am1,       // [nb][NP1]
    const uint8_t* __restrict__ am2,       // [nb][F0]
    const bf16* __restrict__ pk,
    float* __restrict__ conv_slab)         // [nb][CS]
{
  constexpr int DY2P = 18;                 // dY2 with a 4-pixel zero border
  constexpr int SZ_DY2P = C2 * DY2P * DY2P;   // 5184
  constexpr int DY1S = 800;                // conv1-grad row stride (784 -> 25 k-steps)
  __shared__ __attribute__((aligned(16))) unsigned char raw[IMG_BYTES];
  __shared__ __attribute__((aligned(16))) bf16 xs[IMG_BYTES];
  __shared__ __attribute__((aligned(16))) bf16 p1[1184];
  __shared__ __attribute__((aligned(16))) bf16 dY2[C2 * 128];
  __shared__ __attribute__((aligned(16))) bf16 dY2p[SZ_DY2P];
  __shared__ __attribute__((aligned(16))) bf16 dY1[C1 * DY1S];
  __shared__ float dW1acc[16 * 80];
  __shared__ float db[32];

  const int s = blockIdx.x;
  if (s >= nb) return;
  const int gidx = sample_base + s;
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;

  // zero the scatter targets
  {
    const uint4 z = make_uint4(0, 0, 0, 0);
    for (int e = tid; e < C2 * 128 / 8; e += 256) reinterpret_cast<uint4*>(dY2)[e] = z;
    for (int e = tid; e < SZ_DY2P / 8; e += 256) reinterpret_cast<uint4*>(dY2p)[e] = z;
    for (int e = tid; e < C1 * DY1S / 8; e += 256) reinterpret_cast<uint4*>(dY1)[e] = z;
    for (int e = tid; e < 16 * 80; e += 256) dW1acc[e] = 0.f;
    if (tid < 32) db[tid] = 0.f;
    if (tid < NP1 / 8) reinterpret_cast<uint4*>(p1)[tid] = reinterpret_cast<const uint4*>(pool1 + (size_t)s * NP1)[tid];
  }
  const uint32_t h = augment ? hash3(seed, (uint32_t)round_ctr[0], (uint32_t)gidx) : 0u;
  stage_image(images + (size_t)gidx * IMG_BYTES, raw, xs, augment, h);   // contains __syncthreads

  // pool2 / relu backward: route each pooled grad to its argmax position
  for (int f = tid; f < F0; f += 256) {
    const int o = f / 25, rem = f - o * 25, py = rem / P2, px = rem - py * P2;
    const int a = am2[(size_t)s * F0 + f];
    const int y = 2 * py + (a >> 1), x = 2 * px + (a & 1);
    const float g = dact2[(size_t)s * F0 + f];   // already masked by (pool2 > 0) in K2
    const bf16 gb = (bf16)g;
    dY2[o * 128 + y * O2 + x] = gb;
    dY2p[o * DY2P * DY2P + (y + 4) * DY2P + (x + 4)] = gb;
    atomicAdd(&db[o], g);
  }
  __syncthreads();

  float* slab = conv_slab + (size_t)s * CS;

  // ---- conv2 wgrad: dW2[o][kk] = sum_p dY2[o][p] * im2col(pool1)[p][kk]
  //      M = 16 (o), N = 160 (10 tiles, kk < 150), K = 128 (4 steps, p < 100)
  for (int t = wave; t < 10; t += 4) {
    const int kk = t * 16 + n16;
    const int kc = kk < K2 ? kk : 0;
    const int c = kc / 25, rs = kc - c * 25, r = rs / 5, sc = rs - r * 5;
    const bf16* pb = p1 + c * 196 + r * P1 + sc;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int p = ks * 32 + kq + j;
        if (p >= NPOS2) p = 0;                 // dY2 is zero there
        const int py = p / O2, px = p - py * O2;
        b[j] = pb[py * P1 + px];
      }
      acc = mfma16(ld8(dY2 + n16 * 128 + ks * 32 + kq), b, acc);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int o = rq + rr;
      if (kk < K2) slab[P_C2W + o * K2 + kk] = acc[rr];
    }
  }

  // ---- conv2 dgrad: dP1[c][pos] = sum_(o,r,s) dY2[o][y-r][x-s] W2[o][c][r][s]
  //      M = 196 positions (13 tiles), N = 6 (pad 16), K = 400 (13 steps)
  {
    bf16x8 wb[13];
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) wb[ks] = ld8(pk + PK_W2DG + n16 * KDGP + ks * 32 + kq);
    for (int t = wave; t < 13; t += 4) {
      int pos = t * 16 + n16;
      if (pos >= 196) pos = 0;
      const int y = pos / P1, x = pos - y * P1;
      const bf16* gb = dY2p + (y + 4) * DY2P + (x + 4);
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 13; ++ks) {
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          int k = ks * 32 + kq + j;
          if (k >= KDG) k = 0;                 // W2dg pad is zero
          const int o = k / 25, rs = k - o * 25, r = rs / 5, sc = rs - r * 5;
          a[j] = gb[o * DY2P * DY2P - r * DY2P - sc];
        }
        acc = mfma16(a, wb[ks], acc);
      }
      if (n16 < C1) {
        const int c = n16;
        float csum = 0.f;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int p = t * 16 + rq + rr;
          if (p < 196) {
            const float pooled = (float)p1[c * 196 + p];
            const float g = pooled > 0.f ? acc[rr] : 0.f;
            const int a = am1[(size_t)s * NP1 + c * 196 + p];
            const int py = p / P1, px = p - py * P1;
            const int yy = 2 * py + (a >> 1), xx = 2 * px + (a & 1);
            dY1[c * DY1S + yy * O1 + xx] = (bf16)g;
            csum += g;
          }
        }
        atomicAdd(&db[16 + c], csum);
      }
    }
  }
  __syncthreads();

  // ---- conv1 wgrad: dW1[o][kk] = sum_p dY1[o][p] * im2col(x)[p][kk]
  //      M = 16 (o < 6), N = 80 (5 tiles, kk < 75), K = 800 (25 steps, p < 784)
  //      K split over the 4 waves, combined with LDS float atomics.
  {
    int coff[5];
#pragma unroll
    for (int nt = 0; nt < 5; ++nt) {
      const int kk = nt * 16 + n16;
      const int kc = kk < K1 ? kk : 0;
      const int c = kc / 25, rs = kc - c * 25, r = rs / 5, sc = rs - r * 5;
      coff[nt] = c * 1024 + r * 32 + sc;
    }
    f32x4 acc[5];
#pragma unroll
    for (int nt = 0; nt < 5; ++nt) acc[nt] = zero4();
    for (int ks = wave; ks < 25; ks += 4) {
      const bf16x8 a = n16 < C1 ? ld8(dY1 + n16 * DY1S + ks * 32 + kq) : zero8();
      int poff[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int p = ks * 32 + kq + j;
        if (p >= NPOS1) p = 0;                 // dY1 pad is zero
        const int py = p / O1, px = p - py * O1;
        poff[j] = py * IMG + px;
      }
#pragma unroll
      for (int nt = 0; nt < 5; ++nt) {
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = xs[coff[nt] + poff[j]];
        acc[nt] = mfma16(a, b, acc[nt]);
      }
    }
#pragma unroll
    for (int nt = 0; nt < 5; ++nt) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int o = rq + rr, kk = nt * 16 + n16;
        if (o < C1 && kk < K1) atomicAdd(&dW1acc[o * 80 + kk], acc[nt][rr]);
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < C1 * K1; e += 256) {
    const int o = e / K1, kk = e - o * K1;
    slab[P_C1W + e] = dW1acc[o * 80 + kk];
  }
  if (tid < C1) slab[P_C1B + tid] = db[16 + tid];
  if (tid < C2) slab[P_C2B + tid] = db[tid];
}

// ---------------------------------------------------------------------------
// Packing: fp32 master -> bf16 MFMA operand images.
// ---------------------------------------------------------------------------
FEDMI_DEV void pack_one(int i, float w, bf16* __restrict__ pk) {
  const bf16 v = (bf16)w;
  if (i < P_C1B) {
    const int o = i / K1, k = i - o * K1;
    pk[PK_W1C + o * K1P + k] = v;
  } else if (i < P_C2W) {
  } else if (i < P_C2B) {
    const int j = i - P_C2W, o = j / K2, k = j - o * K2;
    pk[PK_W2C + o * K2P + k] = v;
    const int c = k / 25, rs = k - c * 25;
    pk[PK_W2DG + c * KDGP + o * 25 + rs] = v;
  } else if (i < P_F1W) {
  } else if (i < P_F1B) {
    const int j = i - P_F1W, n = j / F0, f = j - n * F0;
    pk[PK_FC1 + n * F0P + f] = v;
    pk[PK_FC1T + f * 128 + n] = v;
  } else if (i < P_F2W) {
  } else if (i < P_F2B) {
    const int j = i - P_F2W, n = j / F1, f = j - n * F1;
    pk[PK_FC2 + n * 128 + f] = v;
    pk[PK_FC2T + f * 96 + n] = v;
  } else if (i < P_F3W) {
  } else if (i < P_F3B) {
    const int j = i - P_F3W, n = j / F2, f = j - n * F2;
    pk[PK_FC3 + n * 96 + f] = v;
    pk[PK_FC3T + f * 32 + n] = v;
  }
}

__global__ __launch_bounds__(256) void lenet_pack(const float* __restrict__ params, bf16* __restrict__ pk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < P_TOTAL) pack_one(i, params[i], pk);
}

// ---------------------------------------------------------------------------
// K4: slab reduction + SGD(momentum, weight decay) + repack.
// 64 parameters x 4 reduction lanes per workgroup.
// torch.optim.SGD semantics (src/main.py:99-100): d = g + wd*p;
// buf = m*buf + d (buf starts at 0 == torch's clone on first step); p -= lr*buf
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lenet_sgd(
    float* __restrict__ params, float* __restrict__ mom, bf16* __restrict__ pk,
    const float* __restrict__ conv_slab, int n_conv,
    const float* __restrict__ fc_slab, int n_fc,
    float lr, float momentum, float wd, int* __restrict__ round_ctr)
{
  __shared__ float red[4][64];
  const int pl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + pl;
  float sum = 0.f;
  if (i < P_TOTAL) {
    const float* src; int stride, cnt;
    if (i < CS) { src = conv_slab + i; stride = CS; cnt = n_conv; }
    else { src = fc_slab + (i - CS); stride = FS; cnt = n_fc; }
    for (int q = g; q < cnt; q += 4) sum += src[(size_t)q * stride];
  }
  red[g][pl] = sum;
  __syncthreads();
  if (g == 0 && i < P_TOTAL) {
    const float grad = red[0][pl] + red[1][pl] + red[2][pl] + red[3][pl];
    const float p = params[i];
    const float d = grad + wd * p;
    const float b = momentum * mom[i] + d;
    const float np = p - lr * b;
    mom[i] = b;
    params[i] = np;
    pack_one(i, np, pk);
  }
  if (round_ctr && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(round_ctr, 1);
}

// ---------------------------------------------------------------------------
// Host launchers (called by the native executor, csrc/runtime/lenet_engine.cpp)
// ---------------------------------------------------------------------------
namespace fedmi {

void launch_lenet_conv_fwd(hipStream_t st, const uint8_t* images, int sample_base, int nb,
                           const bf16* pk, const float* params, uint32_t seed, const int* round_ctr,
                           int augment, bf16* act2, bf16* act2T, int tstride, bf16* pool1,
                           uint8_t* am1, uint8_t* am2) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(lenet_conv_fwd, dim3(nb), dim3(256), 0, st, images, sample_base, nb, pk, params,
                     seed, round_ctr, augment, act2, act2T, tstride, pool1, am1, am2);
}

void launch_lenet_fc_head(hipStream_t st, const bf16* act2, const bf16* act2T, int tstride,
                          const int* labels, int nb, int train, const bf16* pk, const float* params,
                          float* dact2, float* fc_slab, Stats* stats) {
  if (nb <= 0) return;
  const int grid = (nb + FC_SPW - 1) / FC_SPW;
  hipLaunchKernelGGL(lenet_fc_head, dim3(grid), dim3(256), 0, st, act2, act2T, tstride, labels, nb,
                     train, pk, params, dact2, fc_slab, stats);
}

void launch_lenet_conv_bwd(hipStream_t st, const uint8_t* images, int sample_base, int nb,
                           uint32_t seed, const int* round_ctr, int augment, const float* dact2,
                           const bf16* pool1, const uint8_t* am1, const uint8_t* am2,
                           const bf16* pk, float* conv_slab) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(lenet_conv_bwd, dim3(nb), dim3(256), 0, st, images, sample_base, nb, seed,
                     round_ctr, augment, dact2, pool1, am1, am2, pk, conv_slab);
}

void launch_lenet_sgd(hipStream_t st, float* params, float* mom, bf16* pk, const float* conv_slab,
                      int n_conv, const float* fc_slab, int n_fc, float lr, float momentum, float wd,
                      int* round_ctr) {
  hipLaunchKernelGGL(lenet_sgd, dim3((P_TOTAL + 63) / 64), dim3(256), 0, st, params, mom, pk,
                     conv_slab, n_conv, fc_slab, n_fc, lr, momentum, wd, round_ctr);
}

void launch_lenet_pack(hipStream_t st, const float* params, bf16* pk) {
  hipLaunchKernelGGL(lenet_pack, dim3((P_TOTAL + 255) / 256), dim3(256), 0, st, params, pk);
}

}  // namespace fedmi
