// fedmi — fused LeNet training/eval kernels for MI355X (gfx950, CDNA4).
//
// One local SGD step of the reference (src/main.py:146-151: zero_grad,
// forward, CE loss, backward, SGD(m=0.9, wd=5e-4)) is FOUR launches:
//
//   K1 lenet_conv_fwd   one 8-wave workgroup per sample: uint8 image ->
//                       on-device RandomCrop(32,pad4)+HFlip+Normalize
//                       (src/main.py:37-42) -> conv1 (MFMA, channels-last LDS
//                       image: one 16-B read per operand fragment) +bias+ReLU
//                       -> maxpool2 -> conv2 (MFMA) +bias+ReLU -> maxpool2.
//                       Saves pooled activations + 2-bit argmax codes.
//   K2 lenet_fc_head    16 samples (one MFMA row tile) per workgroup: fc1/fc2/
//                       fc3 forward, cross-entropy + accuracy counters, FC
//                       backward down to dZ1 (fc2/fc3 wgrad + bias grads).
//                       Also the eval head (train=0).
//   K3 lenet_conv_bwd   one workgroup per sample: d(pool2) = dZ1.W1 (MFMA),
//                       maxpool/ReLU backward by argmax, conv2 wgrad + dgrad,
//                       conv1 wgrad (MFMA; the im2col operands come from
//                       5 column-shifted LDS copies so every fragment is one
//                       aligned 16-B read).  25 extra workgroups of the same
//                       launch compute fc1.weight's gradient (dZ1^T X).
//   K4 lenet_sgd        combines the gradient slabs (split-K combine at the
//                       kernel boundary: deterministic, no global atomics),
//                       applies wd/momentum/lr to the fp32 master weights and
//                       rewrites the packed bf16 MFMA operand images.
//
// The whole local epoch is replayed from a hipGraph built by the native
// executor (csrc/runtime/lenet_engine.cpp).
#include "common.h"
#include "lenet_layout.h"

using namespace lenet;

namespace {

constexpr int NT = 512;         // threads per workgroup (8 waves) for K1/K2/K3
constexpr int NW = NT / 64;

__constant__ float kMean[3] = {0.4914f, 0.4822f, 0.4465f};
__constant__ float kInvStd[3] = {1.f / 0.2023f, 1.f / 0.1994f, 1.f / 0.2010f};

FEDMI_DEV bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

FEDMI_DEV bf16x8 ld8_b64x2(const bf16* p) {   // 8-byte aligned 8 x bf16
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 4);
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) { r[j] = lo[j]; r[j + 4] = hi[j]; }
  return r;
}

// Crop/flip parameters of the reference train transform (src/main.py:37-38).
struct Aug { int i0, j0, flip; };
FEDMI_DEV Aug aug_params(int augment, uint32_t seed, const int* round_ctr, int gidx) {
  Aug a{4, 4, 0};
  if (augment) {
    const uint32_t h = hash3(seed, (uint32_t)round_ctr[0], (uint32_t)gidx);
    a.i0 = (int)(h % 9u);
    a.j0 = (int)((h >> 8) % 9u);
    a.flip = (int)((h >> 16) & 1u);
  }
  return a;
}

// Normalised pixel of the augmented image (RandomCrop pads with pixel 0 BEFORE
// ToTensor/Normalize, so out-of-image pixels become (0 - mean) / std).
FEDMI_DEV float aug_pixel(const uint8_t* raw, const Aug& a, int c, int y, int x) {
  const int sy = y + a.i0 - 4;
  const int sx = (a.flip ? 31 - x : x) + a.j0 - 4;
  float v = 0.f;
  if (sy >= 0 && sy < IMG && sx >= 0 && sx < IMG) v = (float)raw[c * 1024 + sy * 32 + sx] * (1.f / 255.f);
  return (v - kMean[c]) * kInvStd[c];
}

FEDMI_DEV void load_raw(const uint8_t* __restrict__ img, uint8_t* raw) {
  if ((int)threadIdx.x < IMG_BYTES / 16)
    reinterpret_cast<uint4*>(raw)[threadIdx.x] = reinterpret_cast<const uint4*>(img)[threadIdx.x];
}

FEDMI_DEV void zero_lds(void* p, int bytes) {
  uint4* q = reinterpret_cast<uint4*>(p);
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int e = threadIdx.x; e < bytes / 16; e += blockDim.x) q[e] = z;
}

}  // namespace

// ---------------------------------------------------------------------------
// K1: conv stack forward, one 8-wave workgroup per sample.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void lenet_conv_fwd(
    const uint8_t* __restrict__ images, int sample_base, int nb,
    const bf16* __restrict__ pk, const float* __restrict__ params,
    uint32_t seed, const int* __restrict__ round_ctr, int augment,
    bf16* __restrict__ act2,        // [nb][F0P]
    bf16* __restrict__ act2T,       // [F0P][tstride] (train) or null
    int tstride,
    bf16* __restrict__ pool1_out,   // [nb][NP1] CHW, or null
    uint8_t* __restrict__ am1_out,  // [nb][NP1] or null
    uint8_t* __restrict__ am2_out,  // [nb][F0]  or null
    Stats* __restrict__ zero_stats) // stats block to reset before K2 accumulates (or null)
{
  // LDS: raw u8 | x channels-last [36][40][4] bf16 | conv1 out f32 [6][784]
  //      | pool1 channels-last [14][14][8] bf16 | conv2 out f32 [16][100]
  constexpr int XCL = 36 * 40 * 4, P1CL = 14 * 14 * 8;
  constexpr int O_X = 3072, O_C1 = O_X + XCL * 2, O_P1 = O_C1 + C1 * NPOS1 * 4, O_C2 = O_P1 + P1CL * 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[O_C2 + C2 * NPOS2 * 4];
  uint8_t* raw = smem;
  bf16* xcl = reinterpret_cast<bf16*>(smem + O_X);
  float* c1 = reinterpret_cast<float*>(smem + O_C1);
  bf16* p1cl = reinterpret_cast<bf16*>(smem + O_P1);
  float* c2 = reinterpret_cast<float*>(smem + O_C2);

  const int s = blockIdx.x;
  if (s >= nb) return;
  const int gidx = sample_base + s;
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  // Reset the statistics the following FC-head launch accumulates into (a kernel
  // write instead of a memset node: ordered by the K1 -> K2 boundary in the graph).
  if (zero_stats != nullptr && s == 0 && tid == 0) *zero_stats = Stats{0.f, 0, 0, 0};

  load_raw(images + (size_t)gidx * IMG_BYTES, raw);
  // conv1 weights (B fragments) + per-lane group offsets, while the image lands
  bf16x8 wb1[4];
  int go1[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    wb1[ks] = ld8(pk + PK_W1C + n16 * K1C + ks * 32 + kq);
    const int g = ks * 4 + (lane >> 4);
    go1[ks] = g < 15 ? ((g / 3) * 40 + 2 * (g % 3)) * 4 : 0;
  }
  const Aug a = aug_params(augment, seed, round_ctr, gidx);
  __syncthreads();
  for (int e = tid; e < XCL; e += NT) {
    const int y = e / 160, rem = e - y * 160, x = rem >> 2, c = rem & 3;
    const float v = (c < 3 && y < IMG && x < IMG) ? aug_pixel(raw, a, c, y, x) : 0.f;
    xcl[e] = (bf16)v;
  }
  __syncthreads();

  // ---- conv1: M = 784 positions (49 tiles), N = 6 (pad 16), K = 128 (4 steps)
  {
    const float bias = n16 < C1 ? params[P_C1B + n16] : 0.f;
    for (int t = wave; t < NPOS1 / 16; t += NW) {
      const int pos = t * 16 + n16;
      const int py = pos / O1, px = pos - py * O1;
      const bf16* xb = xcl + (py * 40 + px) * 4;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma16(ld8_b64x2(xb + go1[ks]), wb1[ks], acc);
      if (n16 < C1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) c1[n16 * NPOS1 + t * 16 + rq + r] = fmaxf(acc[r] + bias, 0.f);
      }
    }
  }
  bf16x8 wb2[7];
  int go2[7];
#pragma unroll
  for (int ks = 0; ks < 7; ++ks) {
    wb2[ks] = ld8(pk + PK_W2C + n16 * K2C + ks * 32 + kq);
    const int g = ks * 4 + (lane >> 4);
    go2[ks] = g < 25 ? ((g / 5) * P1 + (g % 5)) * 8 : 0;
  }
  __syncthreads();

  // ---- maxpool2 #1 (+ argmax code: 0=(0,0) 1=(0,1) 2=(1,0) 3=(1,1), first max wins)
  for (int e = tid; e < P1CL; e += NT) {
    const int pos = e >> 3, c = e & 7;
    bf16 mb = (bf16)0.f;
    if (c < C1) {
      const int py = pos / P1, px = pos - py * P1;
      const float* w = c1 + c * NPOS1 + (2 * py) * O1 + 2 * px;
      float m = w[0]; int am = 0;
      if (w[1] > m) { m = w[1]; am = 1; }
      if (w[O1] > m) { m = w[O1]; am = 2; }
      if (w[O1 + 1] > m) { m = w[O1 + 1]; am = 3; }
      mb = (bf16)m;
      if (pool1_out) {
        pool1_out[(size_t)s * NP1 + c * 196 + pos] = mb;
        am1_out[(size_t)s * NP1 + c * 196 + pos] = (uint8_t)am;
      }
    }
    p1cl[e] = mb;
  }
  __syncthreads();

  // ---- conv2: M = 100 positions (7 tiles), N = 16, K = 224 (7 steps)
  if (wave < 7) {
    const int t = wave;
    const float bias = params[P_C2B + n16];
    int pos = t * 16 + n16;
    if (pos >= NPOS2) pos = 0;
    const int py = pos / O2, px = pos - py * O2;
    const bf16* pb = p1cl + (py * P1 + px) * 8;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) acc = mfma16(ld8(pb + go2[ks]), wb2[ks], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = t * 16 + rq + r;
      if (p < NPOS2) c2[n16 * NPOS2 + p] = fmaxf(acc[r] + bias, 0.f);
    }
  }
  __syncthreads();

  // ---- maxpool2 #2 -> flattened act2 row (torch .view order: o*25 + py*5 + px)
  for (int e = tid; e < F0P; e += NT) {
    bf16 mb = (bf16)0.f;
    if (e < F0) {
      const int o = e / 25, rem = e - o * 25, py = rem / P2, px = rem - py * P2;
      const float* w = c2 + o * NPOS2 + (2 * py) * O2 + 2 * px;
      float m = w[0]; int am = 0;
      if (w[1] > m) { m = w[1]; am = 1; }
      if (w[O2] > m) { m = w[O2]; am = 2; }
      if (w[O2 + 1] > m) { m = w[O2 + 1]; am = 3; }
      mb = (bf16)m;
      if (am2_out) am2_out[(size_t)s * F0 + e] = (uint8_t)am;
    }
    act2[(size_t)s * F0P + e] = mb;
    if (act2T) act2T[(size_t)e * tstride + s] = mb;
  }
}

// ---------------------------------------------------------------------------
// K2: FC head, 16 samples per workgroup (one MFMA row tile), 8 waves.
//   fwd: H1 = relu(X W1^T + b1), H2 = relu(H1 W2^T + b2), Z = H2 W3^T + b3
//   CE:  loss/acc counters; dZ = (softmax - onehot) / nb  (mean reduction)
//   bwd: dW3/db3, dH2, dW2/db2, dH1 -> dZ1 (+db1).  dZ1 goes to global for K3.
// Wgrad GEMMs reduce over samples (K = 32, samples 16..31 zero), so the
// activations are also kept sample-contiguous ("T" images) in LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void lenet_fc_head(
    const bf16* __restrict__ act2,   // [nb][F0P]
    const int* __restrict__ labels,  // labels of this batch (already offset)
    int nb, int train,
    const bf16* __restrict__ pk, const float* __restrict__ params,
    bf16* __restrict__ dZ1,          // [128][DZ1_LD]  (train)
    bf16* __restrict__ dZ1T,         // [128][DZ1_LD]  (train)
    float* __restrict__ fc_slab,     // [grid][FS]     (train)
    Stats* __restrict__ stats)
{
  __shared__ __attribute__((aligned(16))) bf16 sH1[16 * 128], sH1T[128 * 32];
  __shared__ __attribute__((aligned(16))) bf16 sH2[16 * 96], sH2T[96 * 32];
  __shared__ __attribute__((aligned(16))) bf16 sdZ3[16 * 32], sdZ3T[16 * 32];
  __shared__ __attribute__((aligned(16))) bf16 sdZ2[16 * 96], sdZ2T[96 * 32];
  __shared__ float sZ[16 * 16];
  __shared__ float sdb[128 + 96 + 16];

  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  const int s0 = blockIdx.x * FC_SPW;
  const int ns = min(FC_SPW, nb - s0);
  if (ns <= 0) return;

  zero_lds(sH1T, sizeof(sH1T));
  zero_lds(sH2T, sizeof(sH2T));
  zero_lds(sdZ3T, sizeof(sdZ3T));
  zero_lds(sdZ2T, sizeof(sdZ2T));
  for (int e = tid; e < 240; e += NT) sdb[e] = 0.f;

  // ---- fc1 fwd: wave w -> output tile n in [16w, 16w+16); K = 416 (13 steps)
  {
    const bool valid = n16 < ns;
    const bf16* xa = act2 + (size_t)(s0 + (valid ? n16 : 0)) * F0P + kq;
    const bf16* wb = pk + PK_FC1 + (wave * 16 + n16) * F0P + kq;
    bf16x8 af[13], bfr[13];
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) {
      af[ks] = valid ? ld8(xa + ks * 32) : zero8();
      bfr[ks] = ld8(wb + ks * 32);
    }
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) acc = mfma16(af[ks], bfr[ks], acc);
    const int n = wave * 16 + n16;
    const float b = n < F1 ? params[P_F1B + n] : 0.f;
    __syncthreads();   // T images zeroed before they are written
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = rq + r;
      const float hv = (n < F1 && sr < ns) ? fmaxf(acc[r] + b, 0.f) : 0.f;
      sH1[sr * 128 + n] = (bf16)hv;
      sH1T[n * 32 + sr] = (bf16)hv;
    }
  }
  __syncthreads();

  // ---- fc2 fwd: waves 0..5 -> 16 outputs each; K = 128 (4 steps)
  if (wave < 6) {
    const bf16* ha = sH1 + n16 * 128 + kq;
    const bf16* wb = pk + PK_FC2 + (wave * 16 + n16) * 128 + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) acc = mfma16(ld8(ha + ks * 32), ld8(wb + ks * 32), acc);
    const int n = wave * 16 + n16;
    const float b = n < F2 ? params[P_F2B + n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = rq + r;
      const float hv = (n < F2 && sr < ns) ? fmaxf(acc[r] + b, 0.f) : 0.f;
      sH2[sr * 96 + n] = (bf16)hv;
      sH2T[n * 32 + sr] = (bf16)hv;
    }
  }
  __syncthreads();

  // ---- fc3 fwd: logits [16 x 16]; K = 96 (3 steps)
  if (wave == 0) {
    const bf16* ha = sH2 + n16 * 96 + kq;
    const bf16* wb = pk + PK_FC3 + n16 * 96 + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) acc = mfma16(ld8(ha + ks * 32), ld8(wb + ks * 32), acc);
    const float b = n16 < NCLS ? params[P_F3B + n16] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) sZ[(rq + r) * 16 + n16] = acc[r] + b;
  }
  __syncthreads();

  // ---- cross-entropy (mean over the batch nb), accuracy, dZ3
  if (wave == 0) {
    float loss = 0.f, corr = 0.f;
    if (lane < 16) {
      const int sr = lane;
      float dz[NCLS];
      if (sr < ns) {
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
        for (int n = 0; n < NCLS; ++n) sZ[sr * 16 + n] = dz[n];   // fp32 dZ3 for db3
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
  constexpr int OF3W = P_F3W - P_F1B, OF2W = P_F2W - P_F1B;

  if (tid < NCLS) {   // db3
    float acc = 0.f;
    for (int sr = 0; sr < 16; ++sr) acc += sZ[sr * 16 + tid];
    sdb[224 + tid] = acc;
  }

  // ---- dW3 (6 tiles) and dH2 = dZ3 . W3 (6 tiles)
  for (int q = wave; q < 12; q += NW) {
    if (q < 6) {
      const int ft = q;
      const f32x4 acc = mfma16(ld8(sdZ3T + n16 * 32 + kq), ld8(sH2T + (ft * 16 + n16) * 32 + kq), zero4());
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = rq + r, f = ft * 16 + n16;
        if (n < NCLS && f < F2) slab[OF3W + n * F2 + f] = acc[r];
      }
    } else {
      const int f = (q - 6) * 16 + n16;
      const f32x4 acc = mfma16(ld8(sdZ3 + n16 * 32 + kq), ld8(pk + PK_FC3T + f * 32 + kq), zero4());
      float colsum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sr = rq + r;
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

  // ---- dW2 = dZ2^T H1 (48 tiles) and dH1 = dZ2 . W2 (8 tiles) -> dZ1
  for (int q = wave; q < 56; q += NW) {
    if (q < 48) {
      const int mt = q >> 3, ft = q & 7;
      const f32x4 acc = mfma16(ld8(sdZ2T + (mt * 16 + n16) * 32 + kq), ld8(sH1T + (ft * 16 + n16) * 32 + kq), zero4());
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = mt * 16 + rq + r, f = ft * 16 + n16;
        if (n < F2 && f < F1) slab[OF2W + n * F1 + f] = acc[r];
      }
    } else {
      const int f = (q - 48) * 16 + n16;
      const bf16* za = sdZ2 + n16 * 96 + kq;
      const bf16* wb = pk + PK_FC2T + f * 96 + kq;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) acc = mfma16(ld8(za + ks * 32), ld8(wb + ks * 32), acc);
      float colsum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sr = rq + r;
        const float g = (f < F1 && (float)sH1[sr * 128 + f] > 0.f) ? acc[r] : 0.f;
        const bf16 gb = (bf16)g;
        dZ1[(size_t)(s0 + sr) * DZ1_LD + f] = gb;
        dZ1T[(size_t)f * DZ1_LD + s0 + sr] = gb;
        colsum += g;
      }
      colsum += __shfl_xor(colsum, 16, 64);
      colsum += __shfl_xor(colsum, 32, 64);
      if (lane < 16 && f < F1) atomicAdd(&sdb[f], colsum);
    }
  }
  __syncthreads();
  for (int e = tid; e < F1; e += NT) slab[e] = sdb[e];                       // fc1.bias
  for (int e = tid; e < F2; e += NT) slab[P_F2B - P_F1B + e] = sdb[128 + e];
  if (tid < NCLS) slab[P_F3B - P_F1B + tid] = sdb[224 + tid];
  // the last workgroup zeroes dZ1T columns [nb, 128): they are K-padding of the fc1 wgrad
  if (s0 + FC_SPW >= nb) {
    const int pad = DZ1_LD - nb;
    for (int e = tid; e < 128 * pad; e += NT) {
      const int f = e / pad, c = nb + (e - f * pad);
      dZ1T[(size_t)f * DZ1_LD + c] = (bf16)0.f;
    }
  }
}

// ---------------------------------------------------------------------------
// K3: conv stack backward (one workgroup per sample) + fc1 wgrad workgroups.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void lenet_conv_bwd(
    const uint8_t* __restrict__ images, int sample_base, int nb,
    uint32_t seed, const int* __restrict__ round_ctr, int augment,
    const bf16* __restrict__ act2,         // [nb][F0P]
    const bf16* __restrict__ act2T,        // [F0P][128]
    const bf16* __restrict__ dZ1,          // [128][128]
    const bf16* __restrict__ dZ1T,         // [128][128]
    const bf16* __restrict__ pool1,        // [nb][NP1]
    const uint8_t* __restrict__ am1,       // [nb][NP1]
    const uint8_t* __restrict__ am2,       // [nb][F0]
    const bf16* __restrict__ pk,
    float* __restrict__ conv_slab,         // [nb][CS]
    float* __restrict__ fc1w_grad)         // [F1W_N]
{
  // LDS carve (bytes)
  constexpr int XSH = 5 * 3 * 32 * 32;        // x shifted copies [s][c][y][x']
  constexpr int P1SH = 5 * 6 * 14 * 16;       // pool1 shifted copies [s][c][y][x']
  constexpr int DY2W = 16 * 160;              // conv2 out-grad [o][i*16+j]
  constexpr int DY2C = 18 * 18 * 16;          // conv2 out-grad channels-last, 4-px zero border
  constexpr int DY1 = 6 * 896;                // conv1 out-grad [o][i*32+j]
  constexpr int O_RAW = 0, O_XSH = 3072, O_P1SH = O_XSH + XSH * 2, O_DY2W = O_P1SH + P1SH * 2,
                O_DY2C = O_DY2W + DY2W * 2, O_DY1 = O_DY2C + DY2C * 2, O_DX = O_DY1 + DY1 * 2,
                O_DW1 = O_DX + F0 * 4, O_DB = O_DW1 + 16 * 80 * 4, O_END = O_DB + 32 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[O_END];

  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;

  if ((int)blockIdx.x >= nb) {
    // ---- fc1.weight grad: dW1[n][f] = sum_s dZ1[s][n] X[s][f], f in [16e, 16e+16)
    const int e = blockIdx.x - nb;
    if (e >= N_DW1_WG) return;
    const int nks = (nb + 31) >> 5;
    const bf16* ap = dZ1T + (wave * 16 + n16) * DZ1_LD + kq;
    const bf16* bp = act2T + (size_t)(e * 16 + n16) * MAX_TRAIN_BATCH + kq;
    f32x4 acc = zero4();
    for (int ks = 0; ks < nks; ++ks) acc = mfma16(ld8(ap + ks * 32), ld8(bp + ks * 32), acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = wave * 16 + rq + r;
      if (n < F1) fc1w_grad[n * F0 + e * 16 + n16] = acc[r];
    }
    return;
  }

  uint8_t* raw = smem + O_RAW;
  bf16* xsh = reinterpret_cast<bf16*>(smem + O_XSH);
  bf16* p1sh = reinterpret_cast<bf16*>(smem + O_P1SH);
  bf16* dY2w = reinterpret_cast<bf16*>(smem + O_DY2W);
  bf16* dY2c = reinterpret_cast<bf16*>(smem + O_DY2C);
  bf16* dY1 = reinterpret_cast<bf16*>(smem + O_DY1);
  float* dx = reinterpret_cast<float*>(smem + O_DX);
  float* dW1acc = reinterpret_cast<float*>(smem + O_DW1);
  float* db = reinterpret_cast<float*>(smem + O_DB);

  const int s = blockIdx.x;
  const int gidx = sample_base + s;

  load_raw(images + (size_t)gidx * IMG_BYTES, raw);
  zero_lds(dY2w, DY2W * 2);
  zero_lds(dY2c, DY2C * 2);
  zero_lds(dY1, DY1 * 2);
  for (int e = tid; e < 16 * 80; e += NT) dW1acc[e] = 0.f;
  if (tid < 32) db[tid] = 0.f;
  // pool1 shifted copies straight from global (one writer per element)
  for (int e = tid; e < P1SH; e += NT) {
    const int xp = e & 15, rest = e >> 4, y = rest % 14, sc = rest / 14, c = sc % 6, sh = sc / 6;
    const int xx = xp + sh;
    p1sh[e] = (xx < P1) ? pool1[(size_t)s * NP1 + c * 196 + y * P1 + xx] : (bf16)0.f;
  }

  // ---- d(pool2) = dZ1[s] . W1 (masked by the pool2 ReLU): M = 1 (of 16), N = 400, K = 128
  {
    const bf16x8 z = zero8();
    bf16x8 af[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) af[ks] = n16 == 0 ? ld8(dZ1 + (size_t)s * DZ1_LD + ks * 32 + kq) : z;
    for (int nt = wave; nt < F0 / 16; nt += NW) {
      const int f = nt * 16 + n16;
      const bf16* wb = pk + PK_FC1T + f * 128 + kq;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma16(af[ks], ld8(wb + ks * 32), acc);
      if (lane < 16) dx[f] = (float)act2[(size_t)s * F0P + f] > 0.f ? acc[0] : 0.f;
    }
  }
  __syncthreads();   // raw image, dx, zeroed buffers visible

  // x shifted copies (augmented, normalised)
  {
    const Aug a = aug_params(augment, seed, round_ctr, gidx);
    for (int e = tid; e < XSH; e += NT) {
      const int xp = e & 31, y = (e >> 5) & 31, sc = e >> 10, c = sc % 3, sh = sc / 3;
      const int xx = xp + sh;
      xsh[e] = (bf16)(xx < IMG ? aug_pixel(raw, a, c, y, xx) : 0.f);
    }
  }
  // pool2 / relu backward: route each pooled grad to its argmax position
  for (int f = tid; f < F0; f += NT) {
    const int o = f / 25, rem = f - o * 25, py = rem / P2, px = rem - py * P2;
    const int am = am2[(size_t)s * F0 + f];
    const int y = 2 * py + (am >> 1), x = 2 * px + (am & 1);
    const float g = dx[f];
    const bf16 gb = (bf16)g;
    dY2w[o * 160 + y * 16 + x] = gb;
    dY2c[((y + 4) * 18 + (x + 4)) * 16 + o] = gb;
    atomicAdd(&db[o], g);
  }
  __syncthreads();

  float* slab = conv_slab + (size_t)s * CS;

  // ---- conv2 wgrad: dW2[o][k'] = sum_p dY2[o][p] * im2col(pool1)[p][k']
  //      M = 16 (o), N = 150 (10 tiles), K = 160 (p' = i*16 + j, 5 steps)
  for (int t = wave; t < 10; t += NW) {
    const int kk = t * 16 + n16;
    const int kc = kk < 150 ? kk : 0;
    const int c = kc / 25, rs = kc - c * 25, r = rs / 5, sc = rs - r * 5;
    const bf16* bb = p1sh + ((sc * 6 + c) * 14 + r) * 16 + (kq & 15);
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 5; ++ks) {
      const int i = 2 * ks + (kq >> 4);
      acc = mfma16(ld8(dY2w + n16 * 160 + ks * 32 + kq), ld8(bb + i * 16), acc);
    }
    if (kk < 150) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) slab[P_C2W + (rq + rr) * 150 + kk] = acc[rr];
    }
  }

  // ---- conv2 dgrad: dP1[c][pos] = sum_(r,s,o) dY2[o][y-r][x-s] W2[o][c][r][s]
  //      M = 196 positions (13 tiles), N = 6 (pad 16), K = 416 (13 steps)
  {
    for (int t = wave; t < 13; t += NW) {
      int pos = t * 16 + n16;
      if (pos >= 196) pos = 0;
      const int y = pos / P1, x = pos - y * P1;
      const bf16* wb = pk + PK_W2DG + n16 * KDGP + kq;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < 13; ++ks) {
        const int G = ks * 4 + (lane >> 4), g = G >> 1;
        int off = 0;
        if (g < 25) {
          const int r = g / 5, sc = g - r * 5;
          off = ((y - r + 4) * 18 + (x - sc + 4)) * 16 + (G & 1) * 8;
        }
        acc = mfma16(ld8(dY2c + off), ld8(wb + ks * 32), acc);
      }
      if (n16 < C1) {
        const int c = n16;
        float csum = 0.f;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int p = t * 16 + rq + rr;
          if (p < 196) {
            const int py = p / P1, px = p - py * P1;
            const float pooled = (float)p1sh[(c * 14 + py) * 16 + px];
            const float g = pooled > 0.f ? acc[rr] : 0.f;
            const int am = am1[(size_t)s * NP1 + c * 196 + p];
            const int yy = 2 * py + (am >> 1), xx = 2 * px + (am & 1);
            dY1[c * 896 + yy * 32 + xx] = (bf16)g;
            csum += g;
          }
        }
        atomicAdd(&db[16 + c], csum);
      }
    }
  }
  __syncthreads();

  // ---- conv1 wgrad: dW1[o][k'] = sum_p dY1[o][p] * im2col(x)[p][k']
  //      M = 16 (o < 6), N = 75 (5 tiles), K = 896 (p' = i*32 + j: step = row i)
  //      K split over the 8 waves, combined with LDS float atomics.
  {
    const bf16* bb[5];
#pragma unroll
    for (int nt = 0; nt < 5; ++nt) {
      const int kk = nt * 16 + n16;
      const int kc = kk < 75 ? kk : 0;
      const int c = kc / 25, rs = kc - c * 25, r = rs / 5, sc = rs - r * 5;
      bb[nt] = xsh + ((sc * 3 + c) * 32 + r) * 32 + kq;
    }
    f32x4 acc[5];
#pragma unroll
    for (int nt = 0; nt < 5; ++nt) acc[nt] = zero4();
    const bf16x8 z = zero8();
    for (int ks = wave; ks < O1; ks += NW) {
      const bf16x8 a = n16 < C1 ? ld8(dY1 + n16 * 896 + ks * 32 + kq) : z;
#pragma unroll
      for (int nt = 0; nt < 5; ++nt) acc[nt] = mfma16(a, ld8(bb[nt] + ks * 32), acc[nt]);
    }
#pragma unroll
    for (int nt = 0; nt < 5; ++nt) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int o = rq + rr, kk = nt * 16 + n16;
        if (o < C1 && kk < 75) atomicAdd(&dW1acc[o * 80 + kk], acc[nt][rr]);
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < C1 * 75; e += NT) {
    const int o = e / 75, kk = e - o * 75;
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
    const int o = i / 75, k = i - o * 75, c = k / 25, rs = k - c * 25, r = rs / 5, s = rs - r * 5;
    pk[PK_W1C + o * K1C + (r * 3 + (s >> 1)) * 8 + (s & 1) * 4 + c] = v;
  } else if (i < P_C2W) {
  } else if (i < P_C2B) {
    const int j = i - P_C2W, o = j / 150, k = j - o * 150, c = k / 25, rs = k - c * 25;
    pk[PK_W2C + o * K2C + rs * 8 + c] = v;
    pk[PK_W2DG + c * KDGP + rs * 16 + o] = v;
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
// K4: gradient combine + SGD(momentum, weight decay) + repack.
// torch.optim.SGD semantics (src/main.py:99-100): d = g + wd*p;
// buf = m*buf + d (buf starts at 0 == torch's clone on first step); p -= lr*buf
// Workgroup ranges: [0, NA) conv params: 16 params x 16 slab lanes;
//                   [NA, NA+NB) fc1.weight: 256 params, complete grads;
//                   [NA+NB, ..) fc tail: 256 params x <= 8 slabs.
// ---------------------------------------------------------------------------
constexpr int SGD_NA = (CS + 15) / 16;           // 180
constexpr int SGD_NB = (F1W_N + 255) / 256;      // 188
constexpr int SGD_NC = (FS + 255) / 256;         // 44

FEDMI_DEV void sgd_update(int i, float grad, float* __restrict__ params, float* __restrict__ mom,
                          bf16* __restrict__ pk, float lr, float momentum, float wd) {
  const float p = params[i];
  const float d = grad + wd * p;
  const float b = momentum * mom[i] + d;
  const float np = p - lr * b;
  mom[i] = b;
  params[i] = np;
  pack_one(i, np, pk);
}

__global__ __launch_bounds__(256) void lenet_sgd(
    float* __restrict__ params, float* __restrict__ mom, bf16* __restrict__ pk,
    const float* __restrict__ conv_slab, int n_conv,
    const float* __restrict__ fc1w_grad,
    const float* __restrict__ fc_slab, int n_fc,
    float lr, float momentum, float wd, int* __restrict__ round_ctr)
{
  __shared__ float red[16][17];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b < SGD_NA) {
    const int pl = tid & 15, g = tid >> 4;
    const int i = b * 16 + pl;
    float sum = 0.f;
    if (i < CS)
      for (int q = g; q < n_conv; q += 16) sum += conv_slab[(size_t)q * CS + i];
    red[g][pl] = sum;
    __syncthreads();
    if (g == 0 && i < CS) {
      float tot = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) tot += red[q][pl];
      sgd_update(i, tot, params, mom, pk, lr, momentum, wd);
    }
  } else if (b < SGD_NA + SGD_NB) {
    const int j = (b - SGD_NA) * 256 + tid;
    if (j < F1W_N) sgd_update(P_F1W + j, fc1w_grad[j], params, mom, pk, lr, momentum, wd);
  } else {
    const int j = (b - SGD_NA - SGD_NB) * 256 + tid;
    if (j < FS) {
      float sum = 0.f;
      for (int q = 0; q < n_fc; ++q) sum += fc_slab[(size_t)q * FS + j];
      sgd_update(P_F1B + j, sum, params, mom, pk, lr, momentum, wd);
    }
  }
  if (round_ctr && b == 0 && tid == 0) atomicAdd(round_ctr, 1);
}

// ---------------------------------------------------------------------------
// Host launchers (called by the native executor, csrc/runtime/lenet_engine.cpp)
// ---------------------------------------------------------------------------
namespace fedmi {

void launch_lenet_conv_fwd(hipStream_t st, const uint8_t* images, int sample_base, int nb,
                           const bf16* pk, const float* params, uint32_t seed, const int* round_ctr,
                           int augment, bf16* act2, bf16* act2T, int tstride, bf16* pool1,
                           uint8_t* am1, uint8_t* am2, Stats* zero_stats) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(lenet_conv_fwd, dim3(nb), dim3(NT), 0, st, images, sample_base, nb, pk, params,
                     seed, round_ctr, augment, act2, act2T, tstride, pool1, am1, am2, zero_stats);
}

void launch_lenet_fc_head(hipStream_t st, const bf16* act2, const int* labels, int nb, int train,
                          const bf16* pk, const float* params, bf16* dZ1, bf16* dZ1T, float* fc_slab,
                          Stats* stats) {
  if (nb <= 0) return;
  const int grid = (nb + FC_SPW - 1) / FC_SPW;
  hipLaunchKernelGGL(lenet_fc_head, dim3(grid), dim3(NT), 0, st, act2, labels, nb, train, pk, params,
                     dZ1, dZ1T, fc_slab, stats);
}

void launch_lenet_conv_bwd(hipStream_t st, const uint8_t* images, int sample_base, int nb,
                           uint32_t seed, const int* round_ctr, int augment, const bf16* act2,
                           const bf16* act2T, const bf16* dZ1, const bf16* dZ1T, const bf16* pool1,
                           const uint8_t* am1, const uint8_t* am2, const bf16* pk, float* conv_slab,
                           float* fc1w_grad) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(lenet_conv_bwd, dim3(nb + N_DW1_WG), dim3(NT), 0, st, images, sample_base, nb, seed,
                     round_ctr, augment, act2, act2T, dZ1, dZ1T, pool1, am1, am2, pk, conv_slab, fc1w_grad);
}

void launch_lenet_sgd(hipStream_t st, float* params, float* mom, bf16* pk, const float* conv_slab,
                      int n_conv, const float* fc1w_grad, const float* fc_slab, int n_fc, float lr,
                      float momentum, float wd, int* round_ctr) {
  hipLaunchKernelGGL(lenet_sgd, dim3(SGD_NA + SGD_NB + SGD_NC), dim3(256), 0, st, params, mom, pk,
                     conv_slab, n_conv, fc1w_grad, fc_slab, n_fc, lr, momentum, wd, round_ctr);
}

void launch_lenet_pack(hipStream_t st, const float* params, bf16* pk) {
  hipLaunchKernelGGL(lenet_pack, dim3((P_TOTAL + 255) / 256), dim3(256), 0, st, params, pk);
}

}  // namespace fedmi
