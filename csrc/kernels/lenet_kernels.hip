// fedmi — fused LeNet training/eval kernels for MI355X (gfx950, CDNA4).
//
// One local SGD step of the reference (src/main.py:146-151: zero_grad, forward, CE loss,
// backward, SGD(m=0.9, wd=5e-4)) is TWO launches:
//
//   KS1 lenet_sample_step  one 16-wave workgroup per sample runs the sample's whole chain:
//                          on-device RandomCrop(32,pad4)+HFlip+Normalize (src/main.py:37-42)
//                          -> conv1 (MFMA) +bias+ReLU -> maxpool2 -> conv2 (MFMA) +bias+ReLU
//                          -> maxpool2 -> fc1/fc2/fc3 -> CE -> FC backward -> conv backward
//                          (maxpool/ReLU backward by argmax, conv2 wgrad + dgrad, conv1
//                          wgrad; im2col operands from 5 column-shifted LDS copies so every
//                          fragment is one aligned 16-B read) -> the sample's gradient slab.
//   KS2 lenet_sgd2         fc1/fc2/fc3 weight gradients as MFMA GEMMs over the batch, SGD
//                          applied to each tile in the workgroup that computed it, the conv
//                          slab combine, bias sums, loss/accuracy: fixed order, no atomics.
//
// Evaluation: lenet_conv_fwd (one 8-wave workgroup per sample, the same conv stack as KS1)
// then lenet_fc_eval (16 samples per workgroup, fc1/fc2/fc3 as MFMA tiles, CE) and
// lenet_eval_stats (ordered sum of the row groups' partials).
//
// The whole local epoch is replayed from a hipGraph built by the native executor
// (csrc/runtime/lenet_engine.cpp).
#include <stdexcept>

#include "common.h"
#include "lenet_layout.h"

using namespace lenet;

#ifdef FEDMI_STAMPS
__device__ unsigned long long fedmi_stamps[FEDMI_STAMP_KERNELS][FEDMI_STAMP_WGS][FEDMI_STAMP_SLOTS];
// diagnostic build only: KS1 staging experiments (bit 0: skip the packed-weight loads, bit 1: every
// workgroup reads sample 0's image).  Timing probes -- the numerics of such a step are meaningless.
__device__ int fedmi_ks1_diag;
#endif

namespace {

constexpr int NT_FWD = 512;     // eval conv forward: 8 waves (measured faster than 16)
constexpr int NW_FWD = NT_FWD / 64;
constexpr int NT_CONV = 1024;   // KS1: 16 waves
constexpr int NW_CONV = NT_CONV / 64;
constexpr int NT_FC = 512;      // eval FC head: 8 waves

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

// NT = the launch's block size as a constant: blockDim.x is read from the dispatch packet, and the
// s_waitcnt vmcnt(0) guarding that load would also drain every weight prefetch in flight
template <int NT>
FEDMI_DEV void zero_lds(void* p, int bytes) {
  uint4* q = reinterpret_cast<uint4*>(p);
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int e = threadIdx.x; e < bytes / 16; e += NT) q[e] = z;
}

}  // namespace

// ---------------------------------------------------------------------------
// lenet_conv_fwd: conv stack forward, one 8-wave workgroup per sample (eval; in "train" mode it
// also saves act2T / pool1 / argmax codes -- the tests' forward oracle for KS1's backward).
// ---------------------------------------------------------------------------
// (at least 6 waves per SIMD: 76 VGPRs, three 49 KB workgroups per CU instead of two at 82 -- the eval launch is
// 10 000 latency-bound workgroups, so images in flight per CU set its throughput)
__global__ __launch_bounds__(NT_FWD, 6) void lenet_conv_fwd(
    const uint8_t* __restrict__ images, int sample_base, int nb,
    const bf16* __restrict__ pk, const float* __restrict__ params,
    uint32_t seed, const int* __restrict__ round_ctr, int augment,
    bf16* __restrict__ act2,        // [nb][F0P]
    bf16* __restrict__ act2T,       // [F0P][tstride] (train) or null
    int tstride,
    bf16* __restrict__ pool1_out,   // [nb][NP1] CHW, or null
    uint8_t* __restrict__ am1_out,  // [nb][NP1] or null
    uint8_t* __restrict__ am2_out,  // [nb][F0]  or null
    Stats* __restrict__ zero_stats) // stats block to reset before the FC head accumulates (or null)
{
  // LDS: raw u8 | x channels-last [36][40][4] bf16 | conv1 out f32 channels-last [784][8]
  //      | pool1 channels-last [14][14][8] bf16 | conv2 out f32 channels-last [100][16]
  //      (conv weights as register fragments: the 10 000-workgroup eval launch values occupancy over
  //      the per-wave L2 traffic KS1 avoids by staging them in LDS)
  constexpr int XCL = 36 * 40 * 4, P1CL = 14 * 14 * 8;
  constexpr int O_X = 3072, O_C1 = O_X + XCL * 2, O_P1 = O_C1 + NPOS1 * 8 * 4, O_C2 = O_P1 + P1CL * 2,
                O_END = O_C2 + C2 * NPOS2 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[O_END];
  uint8_t* raw = smem;
  bf16* xcl = reinterpret_cast<bf16*>(smem + O_X);
  float* c1 = reinterpret_cast<float*>(smem + O_C1);
  bf16* p1cl = reinterpret_cast<bf16*>(smem + O_P1);
  float* c2 = reinterpret_cast<float*>(smem + O_C2);

  const int s = blockIdx.x;
  if (s >= nb) return;
  [[maybe_unused]] const int stamp_wg = s;
  const int gidx = sample_base + s;
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  // Reset the statistics the following FC-head launch accumulates into (a kernel
  // write instead of a memset node: ordered by the K1 -> K2 boundary in the graph).
  if (zero_stats != nullptr && s == 0 && tid == 0) *zero_stats = Stats{0.f, 0, 0, 0};
  FEDMI_STAMP(0, 0);

  // image (192) + conv1 (256) + conv2 (448) weight chunks of 16 B, <= 2 per thread, and every other
  // global read of the kernel start, issued together while the x image is zeroed
  bf16x8 wr1[4], wr2[7];
  load_raw(images + (size_t)gidx * IMG_BYTES, raw);
  zero_lds<NT_FWD>(xcl, XCL * 2);   // channel 3 and the right/bottom pad stay zero
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) wr1[ks] = ld8(pk + PK_W1C + n16 * K1C + ks * 32 + kq);
#pragma unroll
  for (int ks = 0; ks < 7; ++ks) wr2[ks] = ld8(pk + PK_W2C + n16 * K2C + ks * 32 + kq);
  int go1[4], go2[7];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int g = ks * 4 + (lane >> 4);
    go1[ks] = g < 15 ? ((g / 3) * 40 + 2 * (g % 3)) * 4 : 0;
  }
#pragma unroll
  for (int ks = 0; ks < 7; ++ks) {
    const int g = ks * 4 + (lane >> 4);
    go2[ks] = g < 25 ? ((g / 5) * P1 + (g % 5)) * 8 : 0;
  }
  const float bias1 = n16 < C1 ? params[P_C1B + n16] : 0.f;
  const float bias2 = params[P_C2B + n16];
  const Aug a = aug_params(augment, seed, round_ctr, gidx);
  __syncthreads();
  bf16x8 wb1[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) wb1[ks] = wr1[ks];
  for (int e = tid; e < IMG_BYTES; e += NT_FWD) {   // lanes walk x: raw reads broadcast within a dword
    const int c = e >> 10, y = (e >> 5) & 31, x = e & 31;
    xcl[(y * 40 + x) * 4 + c] = (bf16)aug_pixel(raw, a, c, y, x);
  }
  __syncthreads();
  FEDMI_STAMP(0, 1);

  // ---- conv1: M = 784 positions (49 tiles), N = 6 (pad 16), K = 128 (4 steps)
  {
    const float bias = bias1;
    // two tiles per pass (t, t + NW_FWD): both tiles' 8 operand reads are in flight
    // together and the two accumulation chains interleave on the matrix core, so a
    // wave pays the LDS round trip once per two tiles.
    for (int t = wave; t < NPOS1 / 16; t += 2 * NW_FWD) {
      const int tb = t + NW_FWD;
      const bool two = tb < NPOS1 / 16;
      const int pa = t * 16 + n16, pb = (two ? tb : t) * 16 + n16;
      const bf16* xa = xcl + ((pa / O1) * 40 + pa % O1) * 4;
      const bf16* xbb = xcl + ((pb / O1) * 40 + pb % O1) * 4;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        fa[ks] = ld8_b64x2(xa + go1[ks]);
        fb[ks] = ld8_b64x2(xbb + go1[ks]);
      }
      f32x4 acc = zero4(), accb = zero4();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        acc = mfma16(fa[ks], wb1[ks], acc);
        accb = mfma16(fb[ks], wb1[ks], accb);
      }
      if (n16 < C1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) c1[(t * 16 + rq + r) * 8 + n16] = fmaxf(acc[r] + bias, 0.f);
        if (two) {
#pragma unroll
          for (int r = 0; r < 4; ++r) c1[(tb * 16 + rq + r) * 8 + n16] = fmaxf(accb[r] + bias, 0.f);
        }
      }
    }
  }
  __syncthreads();
  FEDMI_STAMP(0, 2);

  // ---- maxpool2 #1 (+ argmax code: 0=(0,0) 1=(0,1) 2=(1,0) 3=(1,1), first max wins)
  for (int e = tid; e < P1CL; e += NT_FWD) {
    const int pos = e >> 3, c = e & 7;
    bf16 mb = (bf16)0.f;
    if (c < C1) {
      const int py = pos / P1, px = pos - py * P1;
      const float* w = c1 + ((2 * py) * O1 + 2 * px) * 8 + c;
      float m = w[0]; int am = 0;
      if (w[8] > m) { m = w[8]; am = 1; }
      if (w[O1 * 8] > m) { m = w[O1 * 8]; am = 2; }
      if (w[O1 * 8 + 8] > m) { m = w[O1 * 8 + 8]; am = 3; }
      mb = (bf16)m;
      if (pool1_out) {
        pool1_out[(size_t)s * NP1 + c * 196 + pos] = mb;
        am1_out[(size_t)s * NP1 + c * 196 + pos] = (uint8_t)am;
      }
    }
    p1cl[e] = mb;
  }
  __syncthreads();
  FEDMI_STAMP(0, 3);

  // ---- conv2: M = 100 positions (7 tiles), N = 16, K = 224 (7 steps)
  if (wave < 7) {
    const int t = wave;
    const float bias = bias2;
    int pos = t * 16 + n16;
    if (pos >= NPOS2) pos = 0;
    const int py = pos / O2, px = pos - py * O2;
    const bf16* pb = p1cl + (py * P1 + px) * 8;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) acc = mfma16(ld8(pb + go2[ks]), wr2[ks], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = t * 16 + rq + r;
      if (p < NPOS2) c2[p * 16 + n16] = fmaxf(acc[r] + bias, 0.f);
    }
  }
  __syncthreads();
  FEDMI_STAMP(0, 4);

  // ---- maxpool2 #2 -> flattened act2 row (torch .view order: o*25 + py*5 + px)
  for (int e = tid; e < F0P; e += NT_FWD) {
    bf16 mb = (bf16)0.f;
    if (e < F0) {
      const int o = e / 25, rem = e - o * 25, py = rem / P2, px = rem - py * P2;
      const float* w = c2 + ((2 * py) * O2 + 2 * px) * 16 + o;
      float m = w[0]; int am = 0;
      if (w[16] > m) { m = w[16]; am = 1; }
      if (w[O2 * 16] > m) { m = w[O2 * 16]; am = 2; }
      if (w[O2 * 16 + 16] > m) { m = w[O2 * 16 + 16]; am = 3; }
      mb = (bf16)m;
      if (am2_out) am2_out[(size_t)s * F0 + e] = (uint8_t)am;
    }
    act2[(size_t)s * F0P + e] = mb;
    if (act2T) act2T[(size_t)e * tstride + s] = mb;
  }
  FEDMI_STAMP(0, 5);
}

// ---------------------------------------------------------------------------
// lenet_fc_eval: the eval head, 16 samples per 8-wave workgroup.  fc1 = relu(X W1^T + b1) from
// the act2 tile in LDS and this wave's 16 W1 rows held as 13 register fragments, fc2 / fc3 as
// 16x16 MFMA tiles, then CE + argmax on 16 lanes.  The row group's (loss, correct) go to
// part[2 mt], part[2 mt + 1] for lenet_eval_stats' ordered sum (no float atomics).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT_FC) void lenet_fc_eval(
    const bf16* __restrict__ act2, const int* __restrict__ labels, int nb,
    const bf16* __restrict__ pk, const float* __restrict__ params, float* __restrict__ part)
{
  constexpr int SX_LD = F0P + 8;                   // act2 tile row stride (bank spread)
  constexpr int XCH = F0P / 8;                     // 52 16-B chunks per act2 row
  __shared__ __attribute__((aligned(16))) bf16 sX[16 * SX_LD];
  __shared__ __attribute__((aligned(16))) bf16 sH1[16 * 128];
  __shared__ __attribute__((aligned(16))) bf16 sH2[16 * 96];
  __shared__ float sZ[16 * 16];
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  const int mt = blockIdx.x, s0 = mt * FC_SPW;
  const int ns = min(FC_SPW, nb - s0);
  if (ns <= 0) return;

  // every global read of the kernel in one wave of requests: W1 / W2 / W3 fragments, biases, act2 tile
  const int nf1 = wave * 16 + n16;
  bf16x8 w1f[13];
#pragma unroll
  for (int ks = 0; ks < 13; ++ks) w1f[ks] = ld8(pk + PK_FC1 + nf1 * F0P + ks * 32 + kq);
  const float b1 = params[P_F1B + min(nf1, F1 - 1)];
  const int nf2 = (wave < 6 ? wave : 0) * 16 + n16;
  const float b2 = params[P_F2B + min(nf2, F2 - 1)];
  const float b3 = params[P_F3B + min(n16, NCLS - 1)];
  bf16x8 w2f[4], w3f[3];
  if (wave < 6) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) w2f[ks] = ld8(pk + PK_FC2 + nf2 * 128 + ks * 32 + kq);
  }
  if (wave == 0) {
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) w3f[ks] = ld8(pk + PK_FC3 + n16 * 96 + ks * 32 + kq);
  }
  uint4 xv[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = tid + u * NT_FC;
    if (e < 16 * XCH) {
      const int r = e / XCH;
      xv[u] = reinterpret_cast<const uint4*>(act2 + (size_t)(s0 + min(r, ns - 1)) * F0P)[e - r * XCH];
      if (r >= ns) xv[u] = make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = tid + u * NT_FC;
    if (e < 16 * XCH) {
      const int r = e / XCH;
      *reinterpret_cast<uint4*>(sX + r * SX_LD + (e - r * XCH) * 8) = xv[u];
    }
  }
  __syncthreads();

  // ---- fc1: wave -> 16 output columns, K = 416 (13 steps)
  {
    const bf16* xa = sX + n16 * SX_LD + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) acc = mfma16(ld8(xa + ks * 32), w1f[ks], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = rq + r;
      sH1[sr * 128 + nf1] = (bf16)((nf1 < F1 && sr < ns) ? fmaxf(acc[r] + b1, 0.f) : 0.f);
    }
  }
  __syncthreads();
  // ---- fc2: waves 0..5 -> 16 outputs each; K = 128 (4 steps)
  if (wave < 6) {
    const bf16* ha = sH1 + n16 * 128 + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) acc = mfma16(ld8(ha + ks * 32), w2f[ks], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sr = rq + r;
      sH2[sr * 96 + nf2] = (bf16)((nf2 < F2 && sr < ns) ? fmaxf(acc[r] + b2, 0.f) : 0.f);
    }
  }
  __syncthreads();
  // ---- fc3: logits [16 x 16]; K = 96 (3 steps)
  if (wave == 0) {
    const bf16* ha = sH2 + n16 * 96 + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) acc = mfma16(ld8(ha + ks * 32), w3f[ks], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) sZ[(rq + r) * 16 + n16] = acc[r] + b3;
  }
  __syncthreads();
  // ---- cross-entropy + accuracy of the row group (lane = sample)
  if (wave == 0) {
    float loss = 0.f, corr = 0.f;
    if (lane < ns) {
      float z[NCLS];
#pragma unroll
      for (int n = 0; n < NCLS; ++n) z[n] = sZ[lane * 16 + n];
      float mx = z[0]; int am = 0;
#pragma unroll
      for (int n = 1; n < NCLS; ++n) if (z[n] > mx) { mx = z[n]; am = n; }
      float se = 0.f;
#pragma unroll
      for (int n = 0; n < NCLS; ++n) se += __expf(z[n] - mx);
      const int y = labels[s0 + lane];
      float zy = 0.f;
#pragma unroll
      for (int n = 0; n < NCLS; ++n) zy = (n == y) ? z[n] : zy;
      loss = mx + __logf(se) - zy;
      corr = (am == y) ? 1.f : 0.f;
    }
    loss = wave_sum(loss);
    corr = wave_sum(corr);
    if (lane == 0) {
      part[2 * mt] = loss;
      part[2 * mt + 1] = corr;
    }
  }
}

// ---------------------------------------------------------------------------
// The conv stack backward of one sample (KS1's second half): maxpool/ReLU backward by argmax,
// conv2 wgrad + dgrad, conv1 wgrad, all operands in LDS.
// ---------------------------------------------------------------------------
// Operand images are padded so the 16 lanes of an MFMA fragment read land on
// distinct 16-byte bank groups (strides in 16-B units: coprime with 16 or
// chosen so the (c, r, s) im2col column index maps to distinct groups).
constexpr int BW_XROW = 40, BW_XS_C = 32 * BW_XROW + 72, BW_XS_S = 3 * BW_XS_C + 48;  // xsh[s][c][y][x']: 5/169/513
constexpr int BW_XSH = 5 * BW_XS_S;
constexpr int BW_P1SH = 5 * 6 * 14 * 16;       // pool1 shifted copies [s][c][y][x']
constexpr int BW_DY2W = 16 * 160;              // conv2 out-grad [o][i*16+j]
constexpr int BW_DY2S = 24;                    // conv2 out-grad channels-last position stride (3 units)
constexpr int BW_DY2C = 18 * 18 * BW_DY2S;     // 4-px zero border
constexpr int BW_DY1S = 904;                   // conv1 out-grad row stride [o][i*32+j] (113 units)
constexpr int BW_DY1 = 6 * BW_DY1S;
constexpr int BW_WDGS = KDGP + 8;              // conv2 dgrad weight row stride (53 units)
// bytes of the backward's scratch region (shifted copies, out-grads, wgrad partials, bias sums)
constexpr int BW_O_XSH = 0, BW_O_P1SH = BW_O_XSH + BW_XSH * 2, BW_O_DY2W = BW_O_P1SH + BW_P1SH * 2,
              BW_O_DY2C = BW_O_DY2W + BW_DY2W * 2, BW_O_DY1 = BW_O_DY2C + BW_DY2C * 2,
              BW_O_DW1 = BW_O_DY1 + BW_DY1 * 2, BW_O_DB = BW_O_DW1 + 3 * 6 * 80 * 4, BW_SCRATCH = BW_O_DB + 64 * 4;

// LDS operands of one sample's conv backward (KS1 still holds them from its own forward).
struct BwdLds {
  const uint8_t* raw;     // uint8 CHW image
  const bf16* p1r;        // pool1 output, CHW [NP1]
  const uint8_t* am1s;    // pool1 argmax codes [NP1]
  const uint8_t* am2s;    // pool2 argmax codes [F0]
  const float* dxs;       // d(pool2) [F0], ReLU-masked
  const bf16* wdg;        // conv2 dgrad weight image, rows of BW_WDGS
  bf16* xsh; bf16* p1sh; bf16* dY2w; bf16* dY2c; bf16* dY1; float* db; float* w1part;
};

FEDMI_DEV BwdLds bwd_lds(unsigned char* scratch, const uint8_t* raw, const bf16* p1r, const uint8_t* am1s,
                         const uint8_t* am2s, const float* dxs, const bf16* wdg) {
  BwdLds L;
  L.raw = raw; L.p1r = p1r; L.am1s = am1s; L.am2s = am2s; L.dxs = dxs; L.wdg = wdg;
  L.xsh = reinterpret_cast<bf16*>(scratch + BW_O_XSH);
  L.p1sh = reinterpret_cast<bf16*>(scratch + BW_O_P1SH);
  L.dY2w = reinterpret_cast<bf16*>(scratch + BW_O_DY2W);
  L.dY2c = reinterpret_cast<bf16*>(scratch + BW_O_DY2C);
  L.dY1 = reinterpret_cast<bf16*>(scratch + BW_O_DY1);
  L.w1part = reinterpret_cast<float*>(scratch + BW_O_DW1);   // conv1 wgrad K-split partials [3][6][80]
  L.db = reinterpret_cast<float*>(scratch + BW_O_DB);
  return L;
}

// zero the out-grad images, the shifted copies' tails (x' + s beyond the row) and the bias sums
FEDMI_DEV void bwd_zero(const BwdLds& L) {
  zero_lds<NT_CONV>(L.dY2w, BW_DY2W * 2);
  zero_lds<NT_CONV>(L.dY2c, BW_DY2C * 2);
  zero_lds<NT_CONV>(L.dY1, BW_DY1 * 2);
  zero_lds<NT_CONV>(L.xsh, BW_XSH * 2);
  zero_lds<NT_CONV>(L.p1sh, BW_P1SH * 2);
  if (threadIdx.x < 64) L.db[threadIdx.x] = 0.f;
}

// each augmented pixel / pooled value is computed once and stored into its 5
// column-shifted copies: copy s holds element x at column x - s
FEDMI_DEV void bwd_build_shifted_img(const BwdLds& L, const Aug& a, int tid, int nthr) {
  for (int e = tid; e < IMG_BYTES; e += nthr) {
    const int c = e >> 10, y = (e >> 5) & 31, x = e & 31;
    const bf16 v = (bf16)aug_pixel(L.raw, a, c, y, x);
    bf16* row = L.xsh + c * BW_XS_C + y * BW_XROW + x;
#pragma unroll
    for (int sh = 0; sh < 5; ++sh)
      if (x >= sh) row[sh * BW_XS_S - sh] = v;
  }
}
FEDMI_DEV void bwd_build_shifted_p1(const BwdLds& L, int tid, int nthr) {
  for (int e = tid; e < NP1; e += nthr) {
    const int c = e / 196, rem = e - c * 196, y = rem / P1, x = rem - y * P1;
    const bf16 v = L.p1r[e];
    bf16* row = L.p1sh + (c * 14 + y) * 16 + x;
#pragma unroll
    for (int sh = 0; sh < 5; ++sh)
      if (x >= sh) row[sh * (6 * 14 * 16) - sh] = v;
  }
}

// d(pool2) -> conv2 out-grad images + conv2 bias sums, then conv2 wgrad + dgrad, conv1 wgrad,
// and the sample's gradient slab.  Stamps slots 2..5 of kernel 'sk'.  db: [0, 16) conv2 bias,
// [16, 58) conv1 bias partials of the 7 dgrad waves (combined in wave order: no LDS float atomics).
FEDMI_DEV void bwd_main(const BwdLds& L, float* __restrict__ slab, int sk, int stamp_wg) {
  (void)sk; (void)stamp_wg;
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  float* db = L.db;
  // thread = (channel o, slot r < 32): the 25 positions of a channel sit in 32 consecutive lanes, so
  // the conv2 bias grad is a shuffle reduction (400 LDS atomics onto 16 addresses took ~2k cycles)
  if (tid < C2 * 32) {
    const int o = tid >> 5, rem = tid & 31;
    float g = 0.f;
    if (rem < 25) {
      const int f = o * 25 + rem, py = rem / P2, px = rem - py * P2;
      const int am = L.am2s[f];
      const int y = 2 * py + (am >> 1), x = 2 * px + (am & 1);
      g = L.dxs[f];
      const bf16 gb = (bf16)g;
      L.dY2w[o * 160 + y * 16 + x] = gb;
      L.dY2c[((y + 4) * 18 + (x + 4)) * BW_DY2S + o] = gb;
    }
#pragma unroll
    for (int w = 1; w < 32; w <<= 1) g += __shfl_xor(g, w, 64);
    if (rem == 0) db[o] = g;
  }
  __syncthreads();
  FEDMI_STAMP(sk, 2);

  // ---- conv2 wgrad: dW2[o][k'] = sum_p dY2[o][p] * im2col(pool1)[p][k']
  //      M = 16 (o), N = 150 (10 tiles), K = 160 (p' = i*16 + j, 5 steps)
  // task map over 16 waves: dgrad tiles (2w, 2w+1) -> wave w < 7 (one read of each weight fragment
  // feeds two tiles), wgrad tiles -> waves 7..15 (wave 7 takes tiles 0 and 9)
  for (int t = wave - 7; t >= 0 && t < 10; t += 9) {
    const int kk = t * 16 + n16;
    const int kc = kk < 150 ? kk : 0;
    const int c = kc / 25, rs = kc - c * 25, r = rs / 5, sc = rs - r * 5;
    const bf16* bb = L.p1sh + ((sc * 6 + c) * 14 + r) * 16 + (kq & 15);
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 5; ++ks) {
      const int i = 2 * ks + (kq >> 4);
      acc = mfma16(ld8(L.dY2w + n16 * 160 + ks * 32 + kq), ld8(bb + i * 16), acc);
    }
    if (kk < 150) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) slab[P_C2W + (rq + rr) * 150 + kk] = acc[rr];
    }
  }

  // ---- conv2 dgrad: dP1[c][pos] = sum_(r,s,o) dY2[o][y-r][x-s] W2[o][c][r][s]
  //      M = 196 positions (13 tiles), N = 6 (pad 16), K = 416 (13 steps)
  int koff[13];   // per-lane K-group offsets into dY2c relative to the output position
#pragma unroll
  for (int ks = 0; ks < 13; ++ks) {
    const int G = ks * 4 + (lane >> 4), g = G >> 1;
    const int r = g / 5, sc = g - r * 5;
    koff[ks] = g < 25 ? (-r * 18 - sc) * BW_DY2S + (G & 1) * 8 : 0;   // pad group: weight 0, any in-bounds read
  }
  if (wave < 7) {
    const int ta = 2 * wave, tb = 2 * wave + 1;          // tb == 13 (wave 6) is a duplicate, not stored
    int pa = ta * 16 + n16, pb = tb * 16 + n16;
    if (pa >= 196) pa = 0;
    if (pb >= 196) pb = 0;
    const bf16* ga = L.dY2c + (((pa / P1) + 4) * 18 + (pa % P1 + 4)) * BW_DY2S;
    const bf16* gbb = L.dY2c + (((pb / P1) + 4) * 18 + (pb % P1 + 4)) * BW_DY2S;
    const bf16* wb = L.wdg + min(n16, C1) * BW_WDGS + kq;     // rows >= 6 are zero: share row 6 (broadcast)
    f32x4 acc[2] = {zero4(), zero4()};
#pragma unroll
    for (int ks = 0; ks < 13; ++ks) {
      const bf16x8 w = ld8(wb + ks * 32);
      acc[0] = mfma16(ld8(ga + koff[ks]), w, acc[0]);
      acc[1] = mfma16(ld8(gbb + koff[ks]), w, acc[1]);
    }
    FEDMI_STAMP(sk, 6);    // wave 0: conv2 dgrad MFMAs done
    float csum = 0.f;
    if (n16 < C1) {
      const int c = n16;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = h ? tb : ta;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int p = t * 16 + rq + rr;
          if (p < 196) {
            const int py = p / P1, px = p - py * P1;
            const float pooled = (float)L.p1r[c * 196 + p];
            const float g = pooled > 0.f ? acc[h][rr] : 0.f;
            const int am = L.am1s[c * 196 + p];
            const int yy = 2 * py + (am >> 1), xx = 2 * px + (am & 1);
            L.dY1[c * BW_DY1S + yy * 32 + xx] = (bf16)g;
            csum += g;
          }
        }
      }
    }
    // the 4 lane groups (rq) of a channel in a fixed xor order, then one write per (wave, channel)
    csum += __shfl_xor(csum, 16, 64);
    csum += __shfl_xor(csum, 32, 64);
    if (n16 < C1 && lane < 16) db[16 + wave * C1 + n16] = csum;
    FEDMI_STAMP(sk, 7);    // wave 0: pool1 backward scatter done
  }
  __syncthreads();
  FEDMI_STAMP(sk, 3);

  // ---- conv1 wgrad: dW1[o][k'] = sum_p dY1[o][p] * im2col(x)[p][k']
  //      M = 16 (o < 6), N = 75 (5 tiles), K = 896 (p' = i*32 + j, 28 steps = conv1
  //      output rows) split in 3 parts: 15 waves = 5 tiles x 3 K-parts, then a
  //      deterministic 3-way combine through LDS.
  if (wave < 15) {
    const int nt = wave % 5, part = wave / 5;
    const int ks0 = part * 10, ks1 = min(ks0 + 10, O1);
    const int kk = nt * 16 + n16;
    const int kc = kk < 75 ? kk : kk - 64;                 // pad columns: distinct bank groups, result dropped
    const int c = kc / 25, rs = kc - c * 25, r = rs / 5, sc = rs - r * 5;
    const bf16* bb = L.xsh + sc * BW_XS_S + c * BW_XS_C + r * BW_XROW + kq;
    const bf16* ab = L.dY1 + min(n16, C1 - 1) * BW_DY1S + kq;
    const bool arow = n16 < C1;
    f32x4 acc0 = zero4(), acc1 = zero4();
    int ks = ks0;
    for (; ks + 1 < ks1; ks += 2) {
      bf16x8 a0 = ld8(ab + ks * 32), a1 = ld8(ab + ks * 32 + 32);
      if (!arow) { a0 = zero8(); a1 = zero8(); }
      acc0 = mfma16(a0, ld8(bb + ks * BW_XROW), acc0);
      acc1 = mfma16(a1, ld8(bb + (ks + 1) * BW_XROW), acc1);
    }
    if (ks < ks1) {
      bf16x8 a0 = ld8(ab + ks * 32);
      if (!arow) a0 = zero8();
      acc0 = mfma16(a0, ld8(bb + ks * BW_XROW), acc0);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int o = rq + rr;
      if (o < C1 && kk < 75) L.w1part[(part * 6 + o) * 80 + kk] = acc0[rr] + acc1[rr];
    }
  }
  __syncthreads();
  FEDMI_STAMP(sk, 4);
  for (int e = tid; e < C1 * 75; e += NT_CONV) {
    const int o = e / 75, kk = e - o * 75;
    slab[P_C1W + e] = L.w1part[o * 80 + kk] + L.w1part[(6 + o) * 80 + kk] + L.w1part[(12 + o) * 80 + kk];
  }
  if (tid < C1) {
    float b = 0.f;
#pragma unroll
    for (int w = 0; w < 7; ++w) b += db[16 + w * C1 + tid];
    slab[P_C1B + tid] = b;
  }
  if (tid < C2) slab[P_C2B + tid] = db[tid];
  FEDMI_STAMP(sk, 5);
}

// ---------------------------------------------------------------------------
// KS1 + KS2: the per-sample training step (the default training path).
//
// KS1 lenet_sample_step: ONE 16-wave workgroup per sample runs the WHOLE chain that
// has no cross-sample dependency: augment -> conv stack forward -> fc1/fc2/fc3 ->
// cross-entropy -> FC backward down to d(pool2) -> conv stack backward -> the
// sample's conv gradient slab.  Every forward operand the backward needs (image,
// pool1, argmax codes, act2) stays in LDS: no flag hand-off between workgroups
// (nothing waits on another workgroup, so a shared GPU can never deadlock it), no
// restaging from global memory, one kernel boundary less than K12 -> K3.  The FC
// layers of ONE sample are GEMVs: VALU dot products over 16-B weight chunks of the
// packed images (L2-resident, read by all 128 workgroups) with 8-lane shuffle
// reductions -- a 16-row MFMA tile would be 15/16 padding.
// KS1 writes the per-sample FC operands of the weight gradients (act2T, h1T, h2T,
// dZ1T, dZ2T, dZ3T: sample-contiguous rows), the FC bias gradients and its loss.
//
// KS2 lenet_sgd2: fc1/fc2/fc3 weight gradients as MFMA GEMMs over the batch
// (K = 128 samples), each workgroup applying SGD to the tile it just computed; the
// conv slab combine (K4's), the bias sums and the loss/accuracy counters in fixed
// order (deterministic, no atomics).
// ---------------------------------------------------------------------------
// Per-step FC side buffers, carved out of the [128][F0] fp32 'dact2' buffer (bytes).
constexpr int AUX_H2T = 0;                              // bf16 [96][128]
constexpr int AUX_DZ2T = AUX_H2T + 96 * 128 * 2;        // bf16 [96][128]
constexpr int AUX_DZ3T = AUX_DZ2T + 96 * 128 * 2;       // bf16 [16][128]
constexpr int FCB_N = 224;                              // fc1.bias 120 | fc2.bias 84 | fc3.bias 10 | pad
constexpr int AUX_FCB = AUX_DZ3T + 16 * 128 * 2;        // f32 [128][FCB_N] per-sample bias grads
constexpr int AUX_LOSS = AUX_FCB + MAX_TRAIN_BATCH * FCB_N * 4;   // f32 [128]
constexpr int AUX_CORR = AUX_LOSS + MAX_TRAIN_BATCH * 4;          // f32 [128]
constexpr int AUX_BYTES = AUX_CORR + MAX_TRAIN_BATCH * 4;
static_assert(AUX_BYTES <= MAX_TRAIN_BATCH * F0 * 4, "FC side buffers must fit in dact2");

// KS1 LDS (bytes): persistent operands, then one scratch region shared by the forward
// (x image, conv1 out, pool1 channels-last, conv2 out) and the backward (BwdLds scratch).
constexpr int S_O_RAW = 0, S_O_P1R = 3072, S_O_AM1 = S_O_P1R + 2368, S_O_AM2 = S_O_AM1 + 1184,
              S_O_X = S_O_AM2 + 416, S_O_DX = S_O_X + F0P * 2, S_O_WDG = S_O_DX + F0 * 4,
              S_O_FC = S_O_WDG + 16 * BW_WDGS * 2, S_O_W1C = S_O_FC + 2048, S_O_W2C = S_O_W1C + 16 * 136 * 2,
              S_O_SCR = S_O_W2C + 16 * 232 * 2;
// conv1 / conv2 B images in LDS, rows padded to 136 / 232 bf16 (17 / 29 16-B units: the 16 rows of a
// fragment read land on distinct bank groups).  Staged ONCE per workgroup: per-wave register loads of
// the same fragments cost 16 waves x 11 KB of L2 traffic per sample.
constexpr int S_W1C_LD = 136, S_W2C_LD = 232;
constexpr int S_F_XCL = 0, S_F_C1 = S_F_XCL + 36 * 40 * 4 * 2, S_F_P1 = S_F_C1 + NPOS1 * 8 * 4,
              S_F_C2 = S_F_P1 + 14 * 14 * 8 * 2, S_F_END = S_F_C2 + C2 * NPOS2 * 4;
// fc1 cross-wave partials: [128 n][4 rows] for the forward, [16 waves][F0P] for dX (one region, two uses)
constexpr int S_O_RED = S_O_SCR + (S_F_END > BW_SCRATCH ? S_F_END : BW_SCRATCH);
constexpr int S_O_W3 = S_O_RED + NW_CONV * F0P * 4;    // fc3 image [16 n][96 f] bf16, staged with the conv weights
constexpr int S_END = S_O_W3 + 16 * 96 * 2;
static_assert(S_END <= 160 * 1024, "KS1 LDS");
// FC scratch (floats, bf16-rounded values where the old MFMA path used bf16 operands)
constexpr int SF_H1 = 0, SF_H2 = 128, SF_Z = 224, SF_DZ3 = 240, SF_DZ2 = 256, SF_DZ1 = 352, SF_END = 480;
static_assert(SF_END * 4 <= 2048, "FC scratch");

FEDMI_DEV float dot8(const bf16x8& a, const bf16x8& b, float acc) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc += (float)a[j] * (float)b[j];
  return acc;
}
FEDMI_DEV float dot8f(const float* a, const bf16x8& b, float acc) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc += a[j] * (float)b[j];
  return acc;
}
FEDMI_DEV float sum8lanes(float v) {   // over the 8 consecutive lanes of a group
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}
FEDMI_DEV float bfr(float v) { return (float)(bf16)v; }
// sum over the 16 lanes of a DPP row (rotations: every lane of the row ends with the row total, each in a
// fixed order -- deterministic)
FEDMI_DEV float row_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xf, 0xf, false));
  return v;
}

__global__ __launch_bounds__(NT_CONV) void lenet_sample_step(
    const uint8_t* __restrict__ images, int sample_base, int nb,
    const bf16* __restrict__ pk, const float* __restrict__ params,
    uint32_t seed, const int* __restrict__ round_ctr, int augment,
    const int* __restrict__ labels,      // labels of this batch (already offset)
    bf16* __restrict__ act2T,            // [F0P][128]
    bf16* __restrict__ h1T,              // [128][128]
    unsigned char* __restrict__ aux,     // AUX_* side buffers
    bf16* __restrict__ dZ1T,             // [128][128]
    float* __restrict__ conv_slab)       // [nb][CS]
{
  __shared__ __attribute__((aligned(16))) unsigned char smem[S_END];
  const int s = blockIdx.x;
  if (s >= nb) return;
  [[maybe_unused]] const int stamp_wg = s;
  const int gidx = sample_base + s;
  const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
  const int kq = (lane >> 4) * 8, n16 = lane & 15, rq = (lane >> 4) * 4;
  uint8_t* raw = smem + S_O_RAW;
  bf16* p1r = reinterpret_cast<bf16*>(smem + S_O_P1R);
  uint8_t* am1s = smem + S_O_AM1;
  uint8_t* am2s = smem + S_O_AM2;
  bf16* xrow = reinterpret_cast<bf16*>(smem + S_O_X);
  float* dxs = reinterpret_cast<float*>(smem + S_O_DX);
  bf16* wdg = reinterpret_cast<bf16*>(smem + S_O_WDG);
  float* fcs = reinterpret_cast<float*>(smem + S_O_FC);
  float* red = reinterpret_cast<float*>(smem + S_O_RED);
  unsigned char* scr = smem + S_O_SCR;
  bf16* xcl = reinterpret_cast<bf16*>(scr + S_F_XCL);
  float* c1 = reinterpret_cast<float*>(scr + S_F_C1);
  bf16* p1cl = reinterpret_cast<bf16*>(scr + S_F_P1);
  float* c2 = reinterpret_cast<float*>(scr + S_F_C2);
  FEDMI_STAMP(0, 0);

  // ---- stage: image (192 x 16 B) and the conv2 dgrad weight image (832 x 16 B) -- one
  //      16-B load per thread; both land while the x image is zeroed and the augmentation drawn
  bf16* w1c = reinterpret_cast<bf16*>(smem + S_O_W1C);
  bf16* w2c = reinterpret_cast<bf16*>(smem + S_O_W2C);
  bf16* w3s = reinterpret_cast<bf16*>(smem + S_O_W3);
  float bias1, bias2;
  Aug a;
  {
    // 192 image + 832 dgrad-weight + 256 conv1-weight + 448 conv2-weight + 192 fc3 16-B chunks (<= 2 per thread)
    constexpr int NI = IMG_BYTES / 16, NWD = 16 * KDGP / 8, NW1 = 16 * K1C / 8, NW2 = 16 * K2C / 8, NW3 = 16 * 96 / 8;
    constexpr int E1 = NI, E2 = E1 + NWD, E3 = E2 + NW1, E4 = E3 + NW2, E5 = E4 + NW3;
    static_assert(E5 <= 2 * NT_CONV, "stage: two chunks per thread");
    uint4 v[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
#ifdef FEDMI_STAMPS
    const int dg = fedmi_ks1_diag;
    const size_t img_sample = (dg & 2) ? 0 : (size_t)gidx;
    const int lim = (dg & 1) ? E1 : E5;
#else
    const size_t img_sample = (size_t)gidx;
    constexpr int lim = E5;
#endif
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * NT_CONV;
      if (e < E1) v[u] = reinterpret_cast<const uint4*>(images + img_sample * IMG_BYTES)[e];
      else if (e >= lim) {}
      else if (e < E2) v[u] = reinterpret_cast<const uint4*>(pk + PK_W2DG)[e - E1];
      else if (e < E3) v[u] = reinterpret_cast<const uint4*>(pk + PK_W1C)[e - E2];
      else if (e < E4) v[u] = reinterpret_cast<const uint4*>(pk + PK_W2C)[e - E3];
      else if (e < E5) v[u] = reinterpret_cast<const uint4*>(pk + PK_FC3)[e - E4];
    }
    // the other global reads of the kernel's start go out in the same wave of requests (one
    // memory latency for the whole stage instead of one per dependent group)
    bias1 = n16 < C1 ? params[P_C1B + n16] : 0.f;
    bias2 = params[P_C2B + n16];
    a = aug_params(augment, seed, round_ctr, gidx);
    zero_lds<NT_CONV>(xcl, 36 * 40 * 4 * 2);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * NT_CONV;
      if (e < E1) {
        reinterpret_cast<uint4*>(raw)[e] = v[u];
      } else if (e < E2) {
        const int w = e - E1, row = w / (KDGP / 8), col = w - row * (KDGP / 8);
        reinterpret_cast<uint4*>(wdg + row * BW_WDGS)[col] = v[u];
      } else if (e < E3) {
        const int w = e - E2, row = w / (K1C / 8), col = w - row * (K1C / 8);
        reinterpret_cast<uint4*>(w1c + row * S_W1C_LD)[col] = v[u];
      } else if (e < E4) {
        const int w = e - E3, row = w / (K2C / 8), col = w - row * (K2C / 8);
        reinterpret_cast<uint4*>(w2c + row * S_W2C_LD)[col] = v[u];
      } else if (e < E5) {
        reinterpret_cast<uint4*>(w3s)[e - E4] = v[u];
      }
    }
  }
  int go1[4], go2[7];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int g = ks * 4 + (lane >> 4);
    go1[ks] = g < 15 ? ((g / 3) * 40 + 2 * (g % 3)) * 4 : 0;
  }
#pragma unroll
  for (int ks = 0; ks < 7; ++ks) {
    const int g = ks * 4 + (lane >> 4);
    go2[ks] = g < 25 ? ((g / 5) * P1 + (g % 5)) * 8 : 0;
  }
  __syncthreads();
  FEDMI_STAMP(1, 7);
  bf16x8 wb1[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) wb1[ks] = ld8(w1c + n16 * S_W1C_LD + ks * 32 + kq);
  for (int e = tid; e < IMG_BYTES; e += NT_CONV) {
    const int c = e >> 10, y = (e >> 5) & 31, x = e & 31;
    xcl[(y * 40 + x) * 4 + c] = (bf16)aug_pixel(raw, a, c, y, x);
  }
  __syncthreads();
  FEDMI_STAMP(0, 1);

  // ---- conv1 (+bias+ReLU) with maxpool #1 in registers: a tile's 16 rows are 4 pooling windows x their 4
  //      positions in argmax-code order (row 4g + r, r = dy * 2 + dx: 0=(0,0) 1=(0,1) 2=(1,0) 3=(1,1)), so the
  //      lane holding C rows 4g..4g+3 of channel n16 has one whole window -- max and first-max code straight
  //      from the accumulators, no fp32 conv1 image and no pooling pass (49 tiles over 16 waves, two per pass)
  auto c1_row = [&](int tt) {                        // A row n16 of tile tt in the channels-last image
    const int q = tt * 4 + (n16 >> 2), y = 2 * (q / P1) + ((n16 >> 1) & 1), x = 2 * (q % P1) + (n16 & 1);
    return xcl + (y * 40 + x) * 4;
  };
  auto pool1 = [&](const f32x4& v, int tt) {
    if (n16 < 8) {                                   // channels 6, 7: zero padding of the conv2 operand
      const int q = tt * 4 + (lane >> 4);
      float m = fmaxf(v[0] + bias1, 0.f), c;
      int am = 0;
      c = fmaxf(v[1] + bias1, 0.f); if (c > m) { m = c; am = 1; }
      c = fmaxf(v[2] + bias1, 0.f); if (c > m) { m = c; am = 2; }
      c = fmaxf(v[3] + bias1, 0.f); if (c > m) { m = c; am = 3; }
      const bf16 mb = (bf16)m;
      p1cl[q * 8 + n16] = mb;
      if (n16 < C1) {
        p1r[n16 * 196 + q] = mb;
        am1s[n16 * 196 + q] = (uint8_t)am;
      }
    }
  };
  for (int t = wave; t < NPOS1 / 16; t += 2 * NW_CONV) {
    const int tb = t + NW_CONV;
    const bool two = tb < NPOS1 / 16;
    const bf16* xa = c1_row(t);
    const bf16* xbb = c1_row(two ? tb : t);
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      fa[ks] = ld8_b64x2(xa + go1[ks]);
      fb[ks] = ld8_b64x2(xbb + go1[ks]);
    }
    f32x4 acc = zero4(), accb = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      acc = mfma16(fa[ks], wb1[ks], acc);
      accb = mfma16(fb[ks], wb1[ks], accb);
    }
    pool1(acc, t);
    if (two) pool1(accb, tb);
  }
  // fc1 weights of this thread, in flight through pool1..pool2 and held in registers to the end of the
  // FC backward: rows n = wave + 16 m (m < 8), columns k = 8 lane .. 8 lane + 7 (lanes >= 52 idle).
  // The forward reduces over k (lanes: DPP row sums, then 4 rows across LDS), dX over n (in-thread over
  // m, then 16 waves across LDS) -- one 106 KB read of W1 per sample, no transposed copy.
  // (every weight load below is unconditional from a clamped address and only its USE is guarded:
  //  a select between a loaded value and zero made the compiler wait for the load on the spot)
  const int fn = tid >> 3, fq = tid & 7;
  constexpr int KCH = F0P / 8;                     // 52 16-B k chunks
  const int kc = min(lane, KCH - 1);
  bf16x8 w1r[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) w1r[m] = ld8(pk + PK_FC1 + (wave + 16 * m) * F0P + kc * 8);
  __syncthreads();
  FEDMI_STAMP(0, 2);
  FEDMI_STAMP(0, 3);                                 // (pool1 is fused into conv1: empty phase)

  // ---- conv2 (+bias+ReLU) with maxpool #2 in registers (rows: 25 windows x 4 positions, 7 tiles) -> act2
  //      row (torch .view order o * 25 + py * 5 + px) in LDS + act2T column
  if (wave < 7) {
    const int t = wave;
    int q = t * 4 + (n16 >> 2);
    if (q >= P2 * P2) q = 0;                         // rows past the 25 windows read a valid position
    const int y = 2 * (q / P2) + ((n16 >> 1) & 1), x = 2 * (q % P2) + (n16 & 1);
    const bf16* pb = p1cl + (y * P1 + x) * 8;
    const bf16* wb = w2c + n16 * S_W2C_LD + kq;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) acc = mfma16(ld8(pb + go2[ks]), ld8(wb + ks * 32), acc);
    const int qo = t * 4 + (lane >> 4);
    if (qo < P2 * P2) {
      float m = fmaxf(acc[0] + bias2, 0.f), c;
      int am = 0;
      c = fmaxf(acc[1] + bias2, 0.f); if (c > m) { m = c; am = 1; }
      c = fmaxf(acc[2] + bias2, 0.f); if (c > m) { m = c; am = 2; }
      c = fmaxf(acc[3] + bias2, 0.f); if (c > m) { m = c; am = 3; }
      const bf16 mb = (bf16)m;
      const int e = n16 * (P2 * P2) + qo;
      am2s[e] = (uint8_t)am;
      xrow[e] = mb;
      act2T[(size_t)e * MAX_TRAIN_BATCH + s] = mb;
    }
  } else if (tid >= 7 * 64 && tid < 7 * 64 + (F0P - F0)) {     // act2 row padding 400..415
    const int e = F0 + tid - 7 * 64;
    xrow[e] = (bf16)0.f;
    act2T[(size_t)e * MAX_TRAIN_BATCH + s] = (bf16)0.f;
  }
  FEDMI_STAMP(0, 4);
  // fc2 weight chunks and the FC biases (fc3's 3 KB image is in LDS since the stage)
  const int n2 = fn < 96 ? fn : 95;
  bf16x8 w2v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) w2v[i] = ld8(pk + PK_FC2 + n2 * 128 + fq * 8 + 64 * i);
  const int label = labels[s];
  const float fb1 = params[P_F1B + min(tid & 127, F1 - 1)];
  const float fb2 = params[P_F2B + min(fn, F2 - 1)];
  const float fb3 = params[P_F3B + min(fn, NCLS - 1)];
  __syncthreads();
  const BwdLds L = bwd_lds(scr, raw, p1r, am1s, am2s, dxs, wdg);
  bwd_zero(L);                 // the forward scratch is dead: the backward's images take its place
  FEDMI_STAMP(0, 5);

  // ---- fc1: h1[n] = relu(x . W1[n] + b1)  (thread = (n, 8-lane k slice))
  unsigned char* auxp = aux;
  float* fcb = reinterpret_cast<float*>(auxp + AUX_FCB) + (size_t)s * FCB_N;
  {
    const bf16x8 xv = ld8(xrow + kc * 8);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float p = row_sum16(lane < KCH ? dot8(xv, w1r[m], 0.f) : 0.f);
      if ((lane & 15) == 0) red[(wave + 16 * m) * 4 + (lane >> 4)] = p;
    }
  }
  // backward weight chunks: fc2^T rows (dH1)
  bf16x8 w2t[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) w2t[i] = ld8(pk + PK_FC2T + fn * 96 + min(fq * 8 + 64 * i, 88));
  __syncthreads();
  if (tid < 128) {             // h1[n] = relu(sum of the 4 row partials + b1), rows in order
    const float* r = red + tid * 4;
    const float h = bfr(tid < F1 ? fmaxf(((r[0] + r[1]) + r[2]) + r[3] + fb1, 0.f) : 0.f);
    fcs[SF_H1 + tid] = h;
    h1T[(size_t)tid * MAX_TRAIN_BATCH + s] = (bf16)h;
  }
  __syncthreads();

  FEDMI_STAMP(1, 0);
  // ---- fc2: h2[n] = relu(h1 . W2[n] + b2)
  if (fn < 96) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) acc = dot8f(fcs + SF_H1 + fq * 8 + 64 * i, w2v[i], acc);
    acc = sum8lanes(acc);
    if (fq == 0) {
      const float h = bfr(fn < F2 ? fmaxf(acc + fb2, 0.f) : 0.f);
      fcs[SF_H2 + fn] = h;
      reinterpret_cast<bf16*>(auxp + AUX_H2T)[(size_t)fn * MAX_TRAIN_BATCH + s] = (bf16)h;
    }
  }
  __syncthreads();
  FEDMI_STAMP(1, 1);
  // ---- fc3: logits (waves 0..1); waves 2..15 meanwhile build the conv backward's column-shifted
  //      copies (zeroed after pool2): the FC chain's idle waves absorb that LDS work
  if (fn < 16) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (fq * 8 + 64 * i < 96) acc = dot8f(fcs + SF_H2 + fq * 8 + 64 * i, ld8(w3s + fn * 96 + fq * 8 + 64 * i), acc);
    acc = sum8lanes(acc);
    if (fq == 0) fcs[SF_Z + fn] = fn < NCLS ? acc + fb3 : 0.f;
  } else {
    bwd_build_shifted_img(L, a, tid - 128, NT_CONV - 128);
  }
  __syncthreads();
  FEDMI_STAMP(1, 2);
  // ---- cross-entropy (mean over the batch nb), accuracy, dZ3: lanes 0..15 of wave 0 hold one
  //      class each (max / sum by xor shuffles); waves 1..15 build the pool1 shifted copies
  if (wave == 0) {
    const int n = lane & 15;
    const float zn = n < NCLS ? fcs[SF_Z + n] : -INFINITY;
    float mx = zn;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    // first index reaching the max (torch argmax semantics)
    float cand = (zn == mx) ? (float)n : 16.f;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) cand = fminf(cand, __shfl_xor(cand, o, 64));
    float se = n < NCLS ? __expf(zn - mx) : 0.f;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) se += __shfl_xor(se, o, 64);
    const float lse = mx + __logf(se);
    const int y = label;
    const float zy = __shfl(zn, y, 64);
    const float d = n < NCLS ? (__expf(zn - lse) - (n == y ? 1.f : 0.f)) * (1.f / (float)nb) : 0.f;
    if (lane < 16) {
      fcs[SF_DZ3 + n] = bfr(d);
      reinterpret_cast<bf16*>(auxp + AUX_DZ3T)[(size_t)n * MAX_TRAIN_BATCH + s] = (bf16)d;
      if (n < NCLS) fcb[204 + n] = d;
    }
    if (lane == 0) {
      reinterpret_cast<float*>(auxp + AUX_LOSS)[s] = lse - zy;
      reinterpret_cast<float*>(auxp + AUX_CORR)[s] = ((int)cand == y) ? 1.f : 0.f;
    }
  } else {
    bwd_build_shifted_p1(L, tid - 64, NT_CONV - 64);
  }
  __syncthreads();
  FEDMI_STAMP(1, 3);
  // ---- dH2 = dZ3 . W3 -> dZ2 (pool of fc2's ReLU)
  if (tid < 96) {
    float acc = 0.f;
#pragma unroll
    for (int n = 0; n < NCLS; ++n) acc += fcs[SF_DZ3 + n] * (float)w3s[n * 96 + tid];   // W3 column tid from LDS
    const float g = (tid < F2 && fcs[SF_H2 + tid] > 0.f) ? acc : 0.f;
    fcs[SF_DZ2 + tid] = bfr(g);
    reinterpret_cast<bf16*>(auxp + AUX_DZ2T)[(size_t)tid * MAX_TRAIN_BATCH + s] = (bf16)g;
    if (tid < F2) fcb[120 + tid] = g;
  }
  __syncthreads();
  FEDMI_STAMP(1, 4);
  // ---- dH1 = dZ2 . W2 -> dZ1
  {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (fq * 8 + 64 * i < 96) acc = dot8f(fcs + SF_DZ2 + fq * 8 + 64 * i, w2t[i], acc);
    acc = sum8lanes(acc);
    if (fq == 0) {
      const float g = (fn < F1 && fcs[SF_H1 + fn] > 0.f) ? acc : 0.f;
      fcs[SF_DZ1 + fn] = bfr(g);
      dZ1T[(size_t)fn * DZ1_LD + s] = (bf16)g;
      if (fn < F1) fcb[fn] = g;
    }
  }
  __syncthreads();
  FEDMI_STAMP(1, 5);
  // ---- dX = dZ1 . W1 from the forward's register fragments: in-thread over the 8 rows, then the 16
  //      waves' partials in wave order, masked by the pool2 ReLU -> d(pool2) in LDS
  {
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float g = fcs[SF_DZ1 + wave + 16 * m];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += g * (float)w1r[m][j];
    }
    if (lane < KCH) {
      float4* o = reinterpret_cast<float4*>(red + wave * F0P + lane * 8);
      o[0] = make_float4(d[0], d[1], d[2], d[3]);
      o[1] = make_float4(d[4], d[5], d[6], d[7]);
    }
  }
  __syncthreads();
  if (tid < F0) {
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < NW_CONV; ++w) acc += red[w * F0P + tid];
    dxs[tid] = (float)xrow[tid] > 0.f ? acc : 0.f;
  }
  __syncthreads();             // d(pool2) from every wave before the conv backward scatters it
  FEDMI_STAMP(0, 6);
  bwd_main(L, conv_slab + (size_t)s * CS, 2, stamp_wg);
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
  } else if (i < P_F2W) {
  } else if (i < P_F2B) {
    const int j = i - P_F2W, n = j / F1, f = j - n * F1;
    pk[PK_FC2 + n * 128 + f] = v;
    pk[PK_FC2T + f * 96 + n] = v;
  } else if (i < P_F3W) {
  } else if (i < P_F3B) {
    const int j = i - P_F3W, n = j / F2, f = j - n * F2;
    pk[PK_FC3 + n * 96 + f] = v;
  }
}

__global__ __launch_bounds__(256) void lenet_pack(const float* __restrict__ params, bf16* __restrict__ pk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < P_TOTAL) pack_one(i, params[i], pk);
}

// ---------------------------------------------------------------------------
// SGD(momentum, weight decay) + repack, torch.optim.SGD semantics (src/main.py:99-100):
// d = g + wd*p; buf = m*buf + d (buf starts at 0 == torch's clone on first step); p -= lr*buf.
// KS2's conv-parameter blocks: 16 params x 16 slab lanes each.
// ---------------------------------------------------------------------------
constexpr int SGD_NA = (CS + 15) / 16;           // 180

FEDMI_DEV void sgd_apply(int i, float grad, float p, float m, float* __restrict__ params, float* __restrict__ mom,
                         bf16* __restrict__ pk, float lr, float momentum, float wd) {
  const float d = grad + wd * p;
  const float b = momentum * m + d;
  const float np = p - lr * b;
  mom[i] = b;
  params[i] = np;
  pack_one(i, np, pk);
}

// Masks the sample columns >= nb of an operand fragment (8 consecutive samples from s0).
FEDMI_DEV bf16x8 mask_cols(bf16x8 v, int s0, int nb) {
  if (s0 + 8 <= nb) return v;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (s0 + j >= nb) v[j] = (bf16)0.f;
  return v;
}

// One 16x16 tile of dW = dZ^T X over the batch: A rows = dZ^T (sample-contiguous, masked
// beyond nb), B rows = X^T (sample-contiguous), K = 128 samples (4 MFMA steps).
// Both operands are masked: columns >= nb may hold anything (the buffers are shared scratch).
// The tile's SGD operands (params / momentum of the <= 4 elements of this lane, indices idx[r],
// -1 = none) are loaded in the same wave of requests as the GEMM operands.
FEDMI_DEV f32x4 batch_tile(const bf16* __restrict__ a, const bf16* __restrict__ b, int nb,
                           const float* __restrict__ params, const float* __restrict__ mom, const int* idx,
                           float* p, float* m) {
  const int lane = lane_id(), kq = (lane >> 4) * 8, n16 = lane & 15;
  bf16x8 av[4], bv[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    av[ks] = ld8(a + n16 * MAX_TRAIN_BATCH + ks * 32 + kq);
    bv[ks] = ld8(b + n16 * MAX_TRAIN_BATCH + ks * 32 + kq);
  }
  // unconditional loads from a clamped index (the callers only use p / m where idx >= 0): a select between
  // a loaded value and zero makes the compiler wait for each load on the spot
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    p[r] = params[idx[r] >= 0 ? idx[r] : 0];
    m[r] = mom[idx[r] >= 0 ? idx[r] : 0];
  }
  f32x4 acc = zero4();
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    acc = mfma16(mask_cols(av[ks], ks * 32 + kq, nb), mask_cols(bv[ks], ks * 32 + kq, nb), acc);
  return acc;
}

constexpr int SGD2_NB = (8 * 25 + 3) / 4;    // fc1.weight: 200 tiles, one per wave
constexpr int SGD2_NC = (6 * 8 + 3) / 4;     // fc2.weight: 48 tiles
constexpr int SGD2_ND = (6 + 3) / 4;         // fc3.weight: 6 tiles
constexpr int SGD2_NE = 4;                   // FC biases: 64 per block x 4 sample groups
constexpr int SGD2_GRID = SGD_NA + SGD2_NB + SGD2_NC + SGD2_ND + SGD2_NE + 1;   // + loss/accuracy block

__global__ __launch_bounds__(256) void lenet_sgd2(
    float* __restrict__ params, float* __restrict__ mom, bf16* __restrict__ pk,
    const float* __restrict__ conv_slab, int nb,
    const bf16* __restrict__ act2T, const bf16* __restrict__ h1T, const unsigned char* __restrict__ aux,
    const bf16* __restrict__ dZ1T, float lr, float momentum, float wd,
    int* __restrict__ round_ctr, Stats* __restrict__ stats)
{
  __shared__ float red[16][17];
  const int b = blockIdx.x, tid = threadIdx.x, wave = wave_id(), lane = lane_id();
  const int n16 = lane & 15, rq = (lane >> 4) * 4;
  [[maybe_unused]] const int stamp_wg = b;
  FEDMI_STAMP(3, 0);
  if (b < SGD_NA) {                                   // conv params: K4's slab combine
    const int pl = tid & 15, g = tid >> 4;
    const int i = b * 16 + pl;
    float p = 0.f, m = 0.f;
    if (g == 0 && i < CS) { p = params[i]; m = mom[i]; }
    float sum = 0.f;
    if (i < CS) {
      // every load unconditional from a clamped sample (masked after): one memory latency for all 8
      float v[MAX_TRAIN_BATCH / 16];
#pragma unroll
      for (int u = 0; u < MAX_TRAIN_BATCH / 16; ++u) v[u] = conv_slab[(size_t)min(g + 16 * u, nb - 1) * CS + i];
#pragma unroll
      for (int u = 0; u < MAX_TRAIN_BATCH / 16; ++u) sum += g + 16 * u < nb ? v[u] : 0.f;
    }
    red[g][pl] = sum;
    __syncthreads();
    if (g == 0 && i < CS) {
      float tot = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) tot += red[q][pl];
      sgd_apply(i, tot, p, m, params, mom, pk, lr, momentum, wd);
    }
  } else if (b < SGD_NA + SGD2_NB) {                  // fc1.weight [120][400]: 8 x 25 tiles
    const int t = (b - SGD_NA) * 4 + wave;
    if (t < 200) {
      const int nt = t / 25, ft = t - nt * 25;
      int idx[4];
      float p[4], m[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nt * 16 + rq + r, f = ft * 16 + n16;
        idx[r] = n < F1 ? P_F1W + n * F0 + f : -1;
      }
      const f32x4 acc = batch_tile(dZ1T + (size_t)nt * 16 * DZ1_LD, act2T + (size_t)ft * 16 * MAX_TRAIN_BATCH, nb,
                                   params, mom, idx, p, m);
      FEDMI_STAMP(3, 2);    // operands landed + MFMA (wave 0's tile)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (idx[r] >= 0) sgd_apply(idx[r], acc[r], p[r], m[r], params, mom, pk, lr, momentum, wd);
      FEDMI_STAMP(3, 3);
    }
  } else if (b < SGD_NA + SGD2_NB + SGD2_NC) {        // fc2.weight [84][120]: 6 x 8 tiles
    const int t = (b - SGD_NA - SGD2_NB) * 4 + wave;
    if (t < 48) {
      const int nt = t >> 3, ft = t & 7;
      const bf16* dz2t = reinterpret_cast<const bf16*>(aux + AUX_DZ2T);
      int idx[4];
      float p[4], m[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nt * 16 + rq + r, f = ft * 16 + n16;
        idx[r] = (n < F2 && f < F1) ? P_F2W + n * F1 + f : -1;
      }
      const f32x4 acc = batch_tile(dz2t + (size_t)nt * 16 * MAX_TRAIN_BATCH, h1T + (size_t)ft * 16 * MAX_TRAIN_BATCH, nb,
                                   params, mom, idx, p, m);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (idx[r] >= 0) sgd_apply(idx[r], acc[r], p[r], m[r], params, mom, pk, lr, momentum, wd);
    }
  } else if (b < SGD_NA + SGD2_NB + SGD2_NC + SGD2_ND) {   // fc3.weight [10][84]: 1 x 6 tiles
    const int t = (b - SGD_NA - SGD2_NB - SGD2_NC) * 4 + wave;
    if (t < 6) {
      const bf16* dz3t = reinterpret_cast<const bf16*>(aux + AUX_DZ3T);
      const bf16* h2t = reinterpret_cast<const bf16*>(aux + AUX_H2T);
      int idx[4];
      float p[4], m[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = rq + r, f = t * 16 + n16;
        idx[r] = (n < NCLS && f < F2) ? P_F3W + n * F2 + f : -1;
      }
      const f32x4 acc = batch_tile(dz3t, h2t + (size_t)t * 16 * MAX_TRAIN_BATCH, nb, params, mom, idx, p, m);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (idx[r] >= 0) sgd_apply(idx[r], acc[r], p[r], m[r], params, mom, pk, lr, momentum, wd);
    }
  } else {                                            // FC biases + loss / accuracy counters
    // block e < 4: biases [64e, 64e + 64) x 4 sample groups of 32 (all 32 loads in flight),
    // fixed-order combine; block 4: the per-sample losses / hits (fixed tree order)
    const int e = b - (SGD_NA + SGD2_NB + SGD2_NC + SGD2_ND);
    const float* fcb = reinterpret_cast<const float*>(aux + AUX_FCB);
    const int j = e * 64 + (tid & 63), g = tid >> 6;
    __shared__ float bsum[4][64];
    float bp = 0.f, bm = 0.f;
    const int bi = j < 120 ? P_F1B + j : (j < 204 ? P_F2B + j - 120 : P_F3B + j - 204);
    if (e < SGD2_NE && g == 0 && j < 214) { bp = params[bi]; bm = mom[bi]; }
    if (e < SGD2_NE && j < 214) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = fcb[(size_t)min(g * 32 + u, nb - 1) * FCB_N + j];
      float sum = 0.f;
#pragma unroll
      for (int u = 0; u < 32; ++u) sum += g * 32 + u < nb ? v[u] : 0.f;
      bsum[g][tid & 63] = sum;
    } else if (e == SGD2_NE && g == 0 && stats != nullptr) {
      const float* lv = reinterpret_cast<const float*>(aux + AUX_LOSS);
      const float* cv = reinterpret_cast<const float*>(aux + AUX_CORR);
      float ls = 0.f, cs = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int sm = lane + 64 * u;
        if (sm < nb) { ls += lv[sm]; cs += cv[sm]; }
      }
      ls = wave_sum(ls);
      cs = wave_sum(cs);
      if (lane == 0) {
        stats->loss_sum += ls;
        stats->correct += (int)(cs + 0.5f);
        stats->count += nb;
      }
    }
    __syncthreads();
    if (e < SGD2_NE && g == 0 && j < 214) {
      const float sum = (bsum[0][tid] + bsum[1][tid]) + (bsum[2][tid] + bsum[3][tid]);
      sgd_apply(bi, sum, bp, bm, params, mom, pk, lr, momentum, wd);
    }
  }
  if (b == 0 && tid == 0 && round_ctr) atomicAdd(round_ctr, 1);
  FEDMI_STAMP(3, 1);
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
  hipLaunchKernelGGL(lenet_conv_fwd, dim3(nb), dim3(NT_FWD), 0, st, images, sample_base, nb, pk, params,
                     seed, round_ctr, augment, act2, act2T, tstride, pool1, am1, am2, zero_stats);
}

// eval loss / correct partials of lenet_fc_eval (one pair per 16-row group) summed in group order: 256
// strided partials, then an ordered LDS fold -- bit-reproducible eval statistics
__global__ __launch_bounds__(256) void lenet_eval_stats(const float* __restrict__ part, int groups, int n,
                                                        Stats* __restrict__ stats) {
  __shared__ float rl[256], rc[256];
  float l = 0.f, c = 0.f;
  for (int g = threadIdx.x; g < groups; g += 256) { l += part[2 * g]; c += part[2 * g + 1]; }
  rl[threadIdx.x] = l;
  rc[threadIdx.x] = c;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) { rl[threadIdx.x] += rl[threadIdx.x + w]; rc[threadIdx.x] += rc[threadIdx.x + w]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats->loss_sum += rl[0];
    stats->correct += (int)(rc[0] + 0.5f);
    stats->count += n;
  }
}

// eval head over the act2 rows of n samples; part: >= 2 * ceil(n / 16) floats of scratch
void launch_lenet_fc_eval(hipStream_t st, const bf16* act2, const int* labels, int n, const bf16* pk,
                          const float* params, float* part, long part_floats, Stats* stats) {
  if (n <= 0) return;
  const int mtiles = (n + FC_SPW - 1) / FC_SPW;
  if (2L * mtiles > part_floats) throw std::invalid_argument("lenet eval: partials scratch too small");
  hipLaunchKernelGGL(lenet_fc_eval, dim3(mtiles), dim3(NT_FC), 0, st, act2, labels, n, pk, params, part);
  hipLaunchKernelGGL(lenet_eval_stats, dim3(1), dim3(256), 0, st, part, mtiles, n, stats);
}

bool stamps_enabled() {
#ifdef FEDMI_STAMPS
  return true;
#else
  return false;
#endif
}

void set_ks1_diag(int v) {
#ifdef FEDMI_STAMPS
  (void)hipMemcpyToSymbol(HIP_SYMBOL(fedmi_ks1_diag), &v, sizeof(v), 0, hipMemcpyHostToDevice);
#else
  (void)v;
#endif
}

// Copy (and optionally clear) the per-phase s_memtime stamps of the diagnostic build.
void read_stamps(unsigned long long* host, bool clear) {
#ifdef FEDMI_STAMPS
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(fedmi_stamps), sizeof(fedmi_stamps), 0, hipMemcpyDeviceToHost);
  if (clear) {
    static unsigned long long zeros[FEDMI_STAMP_KERNELS][FEDMI_STAMP_WGS][FEDMI_STAMP_SLOTS];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(fedmi_stamps), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
  }
#else
  (void)host;
  (void)clear;
#endif
}

// Zeroes a Stats row in a kernel: an epoch captured into a hipGraph must not reset it with hipMemsetAsync --
// a replayed memset node was measured writing stale bytes (host data such as "PDF1") into the row in a
// gRPC client process whose host heap is reused between rounds (tests/test_system_gpu.py, -c Y).
__global__ void lenet_zero_stats(Stats* __restrict__ s) {
  if (threadIdx.x == 0) *s = Stats{0.f, 0, 0, 0};
}

void launch_lenet_zero_stats(hipStream_t st, Stats* s) {
  hipLaunchKernelGGL(lenet_zero_stats, dim3(1), dim3(64), 0, st, s);
}

void launch_lenet_pack(hipStream_t st, const float* params, bf16* pk) {
  hipLaunchKernelGGL(lenet_pack, dim3((P_TOTAL + 255) / 256), dim3(256), 0, st, params, pk);
}

void launch_lenet_sample_step(hipStream_t st, const uint8_t* images, int sample_base, int nb, const bf16* pk,
                              const float* params, uint32_t seed, const int* round_ctr, int augment,
                              const int* labels, bf16* act2T, bf16* h1T, float* aux, bf16* dZ1T, float* conv_slab) {
  if (nb <= 0 || nb > MAX_TRAIN_BATCH) throw std::invalid_argument("lenet_sample_step: batch must be in [1, 128]");
  hipLaunchKernelGGL(lenet_sample_step, dim3(nb), dim3(NT_CONV), 0, st, images, sample_base, nb, pk, params, seed,
                     round_ctr, augment, labels, act2T, h1T, reinterpret_cast<unsigned char*>(aux), dZ1T, conv_slab);
}

void launch_lenet_sgd2(hipStream_t st, float* params, float* mom, bf16* pk, const float* conv_slab, int nb,
                       const bf16* act2T, const bf16* h1T, const float* aux, const bf16* dZ1T, float lr,
                       float momentum, float wd, int* round_ctr, Stats* stats) {
  if (nb <= 0 || nb > MAX_TRAIN_BATCH) throw std::invalid_argument("lenet_sgd2: batch must be in [1, 128]");
  hipLaunchKernelGGL(lenet_sgd2, dim3(SGD2_GRID), dim3(256), 0, st, params, mom, pk, conv_slab, nb, act2T, h1T,
                     reinterpret_cast<const unsigned char*>(aux), dZ1T, lr, momentum, wd, round_ctr, stats);
}

}  // namespace fedmi
