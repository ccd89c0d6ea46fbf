// fedmi — memory-bound companions of the implicit-GEMM convolution for the
// CIFAR CNN zoo (ResNet family first), all on NHWC bf16 activations:
//
//  * prep_input:     uint8 NCHW image batch -> RandomCrop(32, pad 4) + HFlip +
//                    Normalize (src/main.py:36-41, on-device counter RNG shared
//                    with the LeNet engine) -> bf16 NHWC, channels padded to 8.
//  * bn_apply:       training BatchNorm from the batch statistics the conv
//                    epilogue accumulated (sum, sum of squares) or eval BN
//                    from running stats; running-stat momentum update and
//                    num_batches_tracked += 1 (torch BatchNorm2d semantics);
//                    fused residual (identity or a second BN branch: the
//                    projection shortcut) and ReLU.
//  * bn_bwd_reduce / bn_bwd_apply: BatchNorm backward through the ReLU mask,
//                    for one or two BN branches sharing the same output grad,
//                    with an optional second incoming grad (residual fan-in);
//                    writes dgamma/dbeta into the flat gradient buffer.
//  * head_fwd_bwd / head_wgrad: global average pool + linear + softmax CE
//                    (+ correct count) and its backward, deterministic weight
//                    gradient (no atomics across samples).
//
// Reference parity: native_batch_norm(_backward), relu/threshold_backward,
// add, avg_pool2d(4), addmm/mm, _log_softmax + nll_loss of SURVEY.md §2.4b
// (src/models/resnet.py:14-104, src/main.py:146-156).
#include <stdexcept>

#include "common.h"

namespace {

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

__constant__ float cMean[3] = {0.4914f, 0.4822f, 0.4465f};
__constant__ float cInvStd[3] = {1.f / 0.2023f, 1.f / 0.1994f, 1.f / 0.2010f};

FEDMI_DEV void load8f(const bf16* p, float* v) {
  const bf16x8v b = *reinterpret_cast<const bf16x8v*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
}
FEDMI_DEV void store8f(bf16* p, const float* v) {
  bf16x8v b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)v[j];
  *reinterpret_cast<bf16x8v*>(p) = b;
}

// ---------------------------------------------------------------------------
// dbase (optional): device-side batch start added to ``base``, so one captured
// graph serves every batch of an epoch (see sched_next_kernel).
__global__ __launch_bounds__(256) void prep_input_kernel(const uint8_t* __restrict__ images, int base,
                                                         const int* __restrict__ dbase, int nb, int augment,
                                                         uint32_t seed, const int* __restrict__ round_ctr,
                                                         bf16* __restrict__ out) {
  // one thread per output pixel: 8 channels (3 real + 5 zero) = one 16-B store
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb * 1024) return;
  const int s = t >> 10, y = (t >> 5) & 31, x = t & 31;
  const int gidx = base + (dbase ? dbase[0] : 0) + s;
  int i0 = 4, j0 = 4, flip = 0;
  if (augment) {
    const uint32_t h = hash3(seed, (uint32_t)round_ctr[0], (uint32_t)gidx);
    i0 = (int)(h % 9u); j0 = (int)((h >> 8) % 9u); flip = (int)((h >> 16) & 1u);
  }
  const int sy = y + i0 - 4, sx = (flip ? 31 - x : x) + j0 - 4;
  const bool in = sy >= 0 && sy < 32 && sx >= 0 && sx < 32;
  const uint8_t* img = images + (size_t)gidx * 3072 + (in ? sy * 32 + sx : 0);
  float v[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) v[c] = 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float px = (float)img[c * 1024];
    v[c] = ((in ? px : 0.f) * (1.f / 255.f) - cMean[c]) * cInvStd[c];
  }
  store8f(out + (size_t)t * 8, v);
}

// ---------------------------------------------------------------------------
struct BNArgs {
  const double* stats;    // [STAT_REP][2][C] fp64: sum, sum of squares over M rows (train)
  const float* gamma;
  const float* beta;
  float* rmean;           // running stats (updated in train mode, read in eval)
  float* rvar;
  long long* nbt;         // num_batches_tracked
  float* smean;           // saved batch mean / invstd for the backward
  float* sinv;
  const float* shift;     // the sums in ``stats`` are of (z - shift[c]) (null: 0)
  const float* cbias;     // bias of the producing conv, NOT included in z (null: none):
                          // BN(z + b) in train mode == BN(z); running_mean tracks mean(z) + b
};

// per-channel scale/shift of channels [c_lo, c_lo + CC) into LDS sc[0..CC), sh[0..CC); the
// commit block (its row chunk 0) also commits the running stats of those channels
FEDMI_DEV void bn_coeffs(const BNArgs& a, int C, int M, float eps, float mom, int train, float* sc, float* sh,
                         int c_lo = 0, int CC = -1, bool commit = true, bool count = true) {
  if (CC < 0) CC = C;
  for (int cc = threadIdx.x; cc < CC; cc += blockDim.x) {
    const int c = c_lo + cc;
    float mean, inv;
    if (train) {
      // fp64 replicas (the epilogues add float block partials with fp64 atomics: the totals do not
      // depend on the order the workgroups arrive in, up to fp64 rounding far below the fp32 result)
      double s1 = 0.0, s2 = 0.0;
#pragma unroll 4
      for (int r = 0; r < STAT_REP; ++r) {
        s1 += a.stats[(2 * r) * C + c];
        s2 += a.stats[(2 * r + 1) * C + c];
      }
      const double msd = s1 / (double)M;   // mean of (z - shift)
      const float ms = (float)msd;
      const float var = (float)fmax(s2 / (double)M - msd * msd, 0.0);
      mean = ms + (a.shift ? a.shift[c] : 0.f);
      inv = rsqrtf(var + eps);
      if (commit) {
        a.smean[c] = mean;
        a.sinv[c] = inv;
        if (a.rmean) {
          a.rmean[c] = (1.f - mom) * a.rmean[c] + mom * (mean + (a.cbias ? a.cbias[c] : 0.f));
          a.rvar[c] = (1.f - mom) * a.rvar[c] + mom * var * ((float)M / (float)max(M - 1, 1));
        }
      }
    } else {
      mean = a.rmean[c] - (a.cbias ? a.cbias[c] : 0.f);
      inv = rsqrtf(a.rvar[c] + eps);
    }
    sc[cc] = a.gamma[c] * inv;
    sh[cc] = a.beta[c] - mean * sc[cc];
  }
  if (train && commit && count && threadIdx.x == 0 && a.nbt) a.nbt[0] += 1;
}

// BN scale / shift only ([2][C] fp32), with bn_apply's running-stat / saved-stat commit: for a BN whose
// consumer applies it on load (bn_apply's output is never written).  One workgroup.

// Channel-chunked grid of the apply kernels: blockIdx.y = chunk of CC <= 64 channels, blockIdx.x = chunk
// of rows.  A block derives the BN coefficients of ITS channels only (16 fp64 replica reads x 2 per
// channel): with the whole channel range per block, every block re-read all C channels' replicas --
// 256 KB per block at C = 1024, which made the late small layers' applies latency-bound.
constexpr int kBnChunk = 64;

// Flat grid (C < 256 or C % 64 != 0: the coefficient prologue is cheap, every row load coalesced)
// y = act(bnA(z) [+ res | + bnB(z2)])      res_mode: 0 none, 1 identity residual, 2 second BN branch
// y rows have stride ldy (>= C): a channel slice of a concatenated output (GoogLeNet)
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ z, BNArgs A, const bf16* __restrict__ z2,
                                                       BNArgs B, const bf16* __restrict__ res, bf16* __restrict__ y,
                                                       int M, int C, float eps, float mom, int train, int relu,
                                                       int res_mode, int ldy, float* __restrict__ co_out) {
  extern __shared__ float co[];   // [4][C]
  float* sc = co;
  float* sh = co + C;
  float* sc2 = co + 2 * C;
  float* sh2 = co + 3 * C;
  bn_coeffs(A, C, M, eps, mom, train, sc, sh, 0, C, blockIdx.x == 0);
  if (res_mode == 2) bn_coeffs(B, C, M, eps, mom, train, sc2, sh2, 0, C, blockIdx.x == 0);
  if (co_out != nullptr && blockIdx.x == 0)   // the coefficients, for a backward that derives the ReLU mask from z
    for (int c = threadIdx.x; c < C; c += blockDim.x) { co_out[c] = sc[c]; co_out[C + c] = sh[c]; }
  __syncthreads();
  const int VR = C >> 3;
  const long nv = (long)M * VR;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % VR) * 8;
    float v[8];
    load8f(z + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[c0 + j] + sh[c0 + j];
    if (res_mode == 1) {
      float r[8];
      load8f(res + i * 8, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    } else if (res_mode == 2) {
      float r[8];
      load8f(z2 + i * 8, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j] * sc2[c0 + j] + sh2[c0 + j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    store8f(y + (ldy == C ? i * 8 : (i / VR) * ldy + c0), v);
  }
}

// y = act(bnA(z) [+ res | + bnB(z2)])      res_mode: 0 none, 1 identity residual, 2 second BN branch
// y rows have stride ldy (>= C): a channel slice of a concatenated output (GoogLeNet)
__global__ __launch_bounds__(256) void bn_apply_chunk_kernel(const bf16* __restrict__ z, BNArgs A,
                                                             const bf16* __restrict__ z2, BNArgs B,
                                                             const bf16* __restrict__ res, bf16* __restrict__ y, int M,
                                                             int C, float eps, float mom, int train, int relu,
                                                             int res_mode, int ldy, int rows_per_block,
                                                             float* __restrict__ co_out) {
  __shared__ float co[4][kBnChunk];
  const int CC = min(kBnChunk, C), c_lo = blockIdx.y * CC;
  const bool commit = blockIdx.x == 0;
  bn_coeffs(A, C, M, eps, mom, train, co[0], co[1], c_lo, CC, commit, blockIdx.y == 0);
  if (res_mode == 2) bn_coeffs(B, C, M, eps, mom, train, co[2], co[3], c_lo, CC, commit, blockIdx.y == 0);
  if (co_out != nullptr && commit)
    for (int cc = threadIdx.x; cc < CC; cc += blockDim.x) { co_out[c_lo + cc] = co[0][cc]; co_out[C + c_lo + cc] = co[1][cc]; }
  __syncthreads();
  const int VC = CC >> 3, rstep = 256 / VC;
  const int cv = threadIdx.x % VC, c0 = cv * 8, cg = c_lo + c0;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  if ((int)threadIdx.x >= rstep * VC) return;
  float sa[8], ha[8], sb[8], hb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sa[j] = co[0][c0 + j]; ha[j] = co[1][c0 + j];
    sb[j] = res_mode == 2 ? co[2][c0 + j] : 0.f; hb[j] = res_mode == 2 ? co[3][c0 + j] : 0.f;
  }
  // two rows per thread-slot, every load issued before the first use (the kernel is latency-bound on
  // the small late layers)
  for (int r0 = rb + (int)threadIdx.x / VC; r0 < re; r0 += 2 * rstep) {
    float v[2][8], t[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * rstep;
      if (r < re) {
        const long i = (long)r * C + cg;
        load8f(z + i, v[u]);
        if (res_mode == 1) load8f(res + i, t[u]);
        else if (res_mode == 2) load8f(z2 + i, t[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * rstep;
      if (r >= re) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = v[u][j] * sa[j] + ha[j];
        if (res_mode == 1) x += t[u][j];
        else if (res_mode == 2) x += t[u][j] * sb[j] + hb[j];
        v[u][j] = relu ? fmaxf(x, 0.f) : x;
      }
      store8f(y + (long)r * ldy + cg, v[u]);
    }
  }
}

// ---------------------------------------------------------------------------
// BN backward. g = (dya [+ dyb]) * (y > 0 if relu).  Per channel:
//   red[0] = sum g,  red[1] = sum g * xhatA,  red[2] = sum g * xhatB
constexpr int BN_REP = 16;   // atomic replicas of the two-level BN-backward channel sums (fp64)

struct BwdIn {
  const bf16* dya;
  const bf16* dyb;        // optional second incoming grad (residual fan-in)
  const bf16* y;          // forward output (ReLU mask) or null
  const bf16* za;
  const float* meanA;
  const float* invA;
  const bf16* zb;         // optional second BN branch (projection shortcut)
  const float* meanB;
  const float* invB;
  int ldd;                // row stride of dya / dyb (elements; C = compact)
  int ldy;                // row stride of y
  const float* msc;       // [2][C] (optional, y == null): ReLU mask from za, relu(za * sc + sh) > 0 -- the
                          // forward never materialised y (its consumer applied this BN on load)
};

// row r, channel group cg (8 channels); z: the 8 za values of the row (for the msc mask)
FEDMI_DEV void load_g(const BwdIn& in, long r, int cg, float* g, const float* z) {
  const long od = r * in.ldd + cg * 8;
  load8f(in.dya + od, g);
  if (in.dyb) {
    float t[8];
    load8f(in.dyb + od, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] += t[j];
  }
  if (in.y) {
    float t[8];
    load8f(in.y + r * in.ldy + cg * 8, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = t[j] > 0.f ? g[j] : 0.f;
  } else if (in.msc) {
    const int C = in.ldd;   // msc mode: compact rows (host checks ldd == C)
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = z[j] * in.msc[cg * 8 + j] + in.msc[C + cg * 8 + j] > 0.f ? g[j] : 0.f;
  }
}

// red: [3][C] fp64 accumulated with atomics (partials == nullptr), or two-level: the
// block sums are added into one of BN_REP replicas partials[rep][3][C]
// (rep = block % BN_REP: 1/BN_REP of the same-address atomic contention) and
// bn_bwd_finalize sums the replicas into red and re-zeroes them.  fp64 atomics of the
// float block sums: the channel sums do not depend on the workgroups' arrival order
// (up to fp64 rounding, far below the fp32 coefficients derived from them).
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BwdIn in, double* __restrict__ red, int M, int C,
                                                            int rows_per_block, double* __restrict__ partials,
                                                            int reps) {
  __shared__ float part[3][256][8];
  const int VR = C >> 3;                 // host: blockDim.x % VR == 0
  const int cg = threadIdx.x % VR, rstep = blockDim.x / VR, r0 = threadIdx.x / VR;
  const int c0 = cg * 8;
  float ma[8], ia[8], mb[8], ib[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ma[j] = in.meanA[c0 + j]; ia[j] = in.invA[c0 + j];
    mb[j] = in.zb ? in.meanB[c0 + j] : 0.f; ib[j] = in.zb ? in.invB[c0 + j] : 0.f;
  }
  float s0[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = s2[j] = 0.f;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  for (int r = rb + r0; r < re; r += rstep) {
    const long i = (long)r * VR + cg;
    float g[8], z[8];
    load8f(in.za + i * 8, z);
    load_g(in, r, cg, g, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0[j] += g[j];
      s1[j] += g[j] * (z[j] - ma[j]) * ia[j];
    }
    if (in.zb) {
      load8f(in.zb + i * 8, z);
#pragma unroll
      for (int j = 0; j < 8; ++j) s2[j] += g[j] * (z[j] - mb[j]) * ib[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    part[0][threadIdx.x][j] = s0[j];
    part[1][threadIdx.x][j] = s1[j];
    part[2][threadIdx.x][j] = s2[j];
  }
  __syncthreads();
  // threads < 3*C: one (quantity, channel) sum over the rstep partials
  for (int e = threadIdx.x; e < 3 * C; e += blockDim.x) {
    const int qn = e / C, c = e - qn * C;
    if (qn == 2 && !in.zb) continue;
    const int g = c >> 3, j = c & 7;
    float s = 0.f;
    for (int t = g; t < (int)blockDim.x; t += VR) s += part[qn][t][j];
    unsafeAtomicAdd((partials ? partials + (long)(blockIdx.x % reps) * 3 * C : red) + qn * C + c, (double)s);
  }
}

// red[q][c] = sum_r partials[r][q][c]; the replicas are left zero for the next BN
// (launches of a step are stream-serial, so one scratch serves every BN layer).
__global__ __launch_bounds__(256) void bn_bwd_finalize(double* __restrict__ partials, int C, double* __restrict__ red) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 3 * C) return;
  const long stride = 3l * C;
  double v[BN_REP];
#pragma unroll
  for (int r = 0; r < BN_REP; ++r) v[r] = partials[r * stride + e];
#pragma unroll
  for (int r = 0; r < BN_REP; ++r) partials[r * stride + e] = 0.0;
#pragma unroll
  for (int w = BN_REP / 2; w >= 1; w >>= 1)
#pragma unroll
    for (int r = 0; r < w; ++r) v[r] += v[r + w];
  red[e] = v[0];
}

struct BwdOut {
  bf16* dza;              // grad wrt za (conv output of branch A)
  bf16* dzb;              // grad wrt zb (branch B) or null
  bf16* gout;             // masked incoming grad g (identity-shortcut grad) or null
  float* dgammaA;
  float* dbetaA;
  float* dgammaB;
  float* dbetaB;
  const float* gammaA;
  const float* gammaB;
  float* shiftA;          // <- this step's batch mean: the next step's statistics shift
  float* shiftB;
  const bf16* dadd;       // optional grad added to dza (a residual edge that bypasses this BN)
};

// Raw operands of one 8-channel vector of the BN backward (row r, channel offset c; i = the compact element index
// r * C + c), all loads issued together; bwd_g then forms load_g's g from them.  The apply kernels issue their
// first vector this way BEFORE the coefficient prologue, so its latency overlaps the fp64 channel-sum reads.
struct BwdRaw {
  float z[8], g[8], gb[8], ym[8], zb[8], da[8];
};
FEDMI_DEV void bwd_issue(const BwdIn& in, const BwdOut& out, long r, int c, long i, BwdRaw& x) {
  load8f(in.za + i, x.z);
  const long od = r * in.ldd + c;
  load8f(in.dya + od, x.g);
  if (in.dyb) load8f(in.dyb + od, x.gb);
  if (in.y) load8f(in.y + r * in.ldy + c, x.ym);
  if (in.zb) load8f(in.zb + i, x.zb);
  if (out.dadd) load8f(out.dadd + i, x.da);
}
FEDMI_DEV void bwd_g(const BwdIn& in, int c, BwdRaw& x) {
  if (in.dyb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x.g[j] += x.gb[j];
  }
  if (in.y) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x.g[j] = x.ym[j] > 0.f ? x.g[j] : 0.f;
  } else if (in.msc) {
    const int C = in.ldd;   // msc mode: compact rows (host checks ldd == C)
#pragma unroll
    for (int j = 0; j < 8; ++j) x.g[j] = x.z[j] * in.msc[c + j] + in.msc[C + c + j] > 0.f ? x.g[j] : 0.f;
  }
}

// Flat grid variant (see bn_apply_kernel).
// partials != null (chained mode): the channel sums are read straight from the reduce kernel's
// 'reps' atomic replicas (no finalize launch); the caller zeroes them before the next step.
__global__ __launch_bounds__(256) void bn_bwd_apply_flat_kernel(BwdIn in, BwdOut out, const double* __restrict__ red,
                                                           int M, int C, const double* __restrict__ partials,
                                                           int reps) {
  extern __shared__ float co[];   // [6][C]: kA, bA, cA, kB, bB, cB  (dz = k*g + b*xhat + c)
  const float invM = 1.f / (float)M;
  const int VR = C >> 3;
  const int nv = M * VR;          // host: < 2^31
  const int stride = gridDim.x * blockDim.x;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  BwdRaw x;
  if (i < nv) {
    const int row = i / VR;
    bwd_issue(in, out, row, (i - row * VR) * 8, (long)i * 8, x);
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double dg = 0.0, dgx = 0.0, dgx2 = 0.0;
    if (partials) {
      for (int r = 0; r < reps; ++r) {           // fixed order: every block derives identical coefficients
        const double* pr = partials + (long)r * 3 * C;
        dg += pr[c];
        dgx += pr[C + c];
        if (in.zb) dgx2 += pr[2 * C + c];
      }
    } else {
      dg = red[c];
      dgx = red[C + c];
      if (in.zb) dgx2 = red[2 * C + c];
    }
    const float sg = (float)dg, sgx = (float)dgx, sgx2 = (float)dgx2;
    const float scA = out.gammaA[c] * in.invA[c];
    // dz = scA * (g - sg/M - xhat * sgx/M),  xhat = (z - mean) * inv
    co[c] = scA;
    co[C + c] = -scA * sgx * invM * in.invA[c];
    co[2 * C + c] = -scA * sg * invM + scA * sgx * invM * in.invA[c] * in.meanA[c];
    if (blockIdx.x == 0) {
      out.dgammaA[c] = sgx;
      out.dbetaA[c] = sg;
      if (out.shiftA) out.shiftA[c] = in.meanA[c];
    }
    if (in.zb) {
      const float scB = out.gammaB[c] * in.invB[c];
      co[3 * C + c] = scB;
      co[4 * C + c] = -scB * sgx2 * invM * in.invB[c];
      co[5 * C + c] = -scB * sg * invM + scB * sgx2 * invM * in.invB[c] * in.meanB[c];
      if (blockIdx.x == 0) {
        out.dgammaB[c] = sgx2;
        out.dbetaB[c] = sg;
        if (out.shiftB) out.shiftB[c] = in.meanB[c];
      }
    }
  }
  __syncthreads();
  for (bool first = true; i < nv; i += stride, first = false) {
    const int row = i / VR, c0 = (i - row * VR) * 8;
    if (!first) bwd_issue(in, out, row, c0, (long)i * 8, x);
    bwd_g(in, c0, x);
    if (out.gout) store8f(out.gout + (long)i * 8, x.g);
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = co[c0 + j] * x.g[j] + co[C + c0 + j] * x.z[j] + co[2 * C + c0 + j];
    if (out.dadd) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += x.da[j];
    }
    store8f(out.dza + (long)i * 8, d);
    if (in.zb) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = co[3 * C + c0 + j] * x.g[j] + co[4 * C + c0 + j] * x.zb[j] + co[5 * C + c0 + j];
      store8f(out.dzb + (long)i * 8, d);
    }
  }
}

// partials != null (chained mode): the channel sums are read straight from the reduce kernel's
// 'reps' atomic replicas (no finalize launch); the caller zeroes them before the next step.
// Channel-chunked grid like bn_apply_kernel: a block derives the coefficients of its CC channels only.
__global__ __launch_bounds__(256) void bn_bwd_apply_chunk_kernel(BwdIn in, BwdOut out, const double* __restrict__ red,
                                                                 int M, int C, const double* __restrict__ partials,
                                                                 int reps, int rows_per_block) {
  __shared__ float co[6][kBnChunk];   // kA, bA, cA, kB, bB, cB  (dz = k*g + b*z + c)
  const int CC = min(kBnChunk, C), c_lo = blockIdx.y * CC;
  const float invM = 1.f / (float)M;
  const int VC = CC >> 3, rstep = 256 / VC;
  const int cv = threadIdx.x % VC, c0 = cv * 8, cg = c_lo + c0;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  const bool lane_ok = (int)threadIdx.x < rstep * VC;
  // two rows per thread-slot, every load issued before the first use; the first pair before the prologue
  BwdRaw x[2];
  auto issue_pair = [&](int r0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * rstep;
      if (r < re) bwd_issue(in, out, r, cg, (long)r * C + cg, x[u]);
    }
  };
  int r0 = rb + (int)threadIdx.x / VC;
  if (lane_ok) issue_pair(r0);
  for (int cc = threadIdx.x; cc < CC; cc += blockDim.x) {
    const int c = c_lo + cc;
    double dg = 0.0, dgx = 0.0, dgx2 = 0.0;
    if (partials) {
      for (int r = 0; r < reps; ++r) {           // fixed order: every block derives identical coefficients
        const double* pr = partials + (long)r * 3 * C;
        dg += pr[c];
        dgx += pr[C + c];
        if (in.zb) dgx2 += pr[2 * C + c];
      }
    } else {
      dg = red[c];
      dgx = red[C + c];
      if (in.zb) dgx2 = red[2 * C + c];
    }
    const float sg = (float)dg, sgx = (float)dgx, sgx2 = (float)dgx2;
    const float scA = out.gammaA[c] * in.invA[c];
    // dz = scA * (g - sg/M - xhat * sgx/M),  xhat = (z - mean) * inv
    co[0][cc] = scA;
    co[1][cc] = -scA * sgx * invM * in.invA[c];
    co[2][cc] = -scA * sg * invM + scA * sgx * invM * in.invA[c] * in.meanA[c];
    if (blockIdx.x == 0) {
      out.dgammaA[c] = sgx;
      out.dbetaA[c] = sg;
      if (out.shiftA) out.shiftA[c] = in.meanA[c];
    }
    if (in.zb) {
      const float scB = out.gammaB[c] * in.invB[c];
      co[3][cc] = scB;
      co[4][cc] = -scB * sgx2 * invM * in.invB[c];
      co[5][cc] = -scB * sg * invM + scB * sgx2 * invM * in.invB[c] * in.meanB[c];
      if (blockIdx.x == 0) {
        out.dgammaB[c] = sgx2;
        out.dbetaB[c] = sg;
        if (out.shiftB) out.shiftB[c] = in.meanB[c];
      }
    }
  }
  __syncthreads();
  if (!lane_ok) return;
  for (bool first = true; r0 < re; r0 += 2 * rstep, first = false) {
    if (!first) issue_pair(r0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * rstep;
      if (r >= re) continue;
      const long i = (long)r * C + cg;
      bwd_g(in, cg, x[u]);
      if (out.gout) store8f(out.gout + i, x[u].g);
      float d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        d[j] = co[0][c0 + j] * x[u].g[j] + co[1][c0 + j] * x[u].z[j] + co[2][c0 + j];
        if (out.dadd) d[j] += x[u].da[j];
      }
      store8f(out.dza + i, d);
      if (in.zb) {
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = co[3][c0 + j] * x[u].g[j] + co[4][c0 + j] * x[u].zb[j] + co[5][c0 + j];
        store8f(out.dzb + i, d);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Classifier head: y [N][HW][C] -> avgpool -> linear (J <= 16) -> CE.
// One workgroup per sample. Stats layout as lenet::Stats {loss_sum, correct, count, pad}.
__global__ __launch_bounds__(256) void head_fwd_bwd_kernel(const bf16* __restrict__ y, const int* __restrict__ labels,
                                                           int base, const int* __restrict__ dbase, int HW, int C, int J, const float* __restrict__ W,
                                                           const float* __restrict__ b, float* __restrict__ pooled,
                                                           float* __restrict__ dlog, bf16* __restrict__ dy,
                                                           float* __restrict__ stats, float* __restrict__ lossv,
                                                           int N, int train, float4* __restrict__ zero_buf,
                                                           long zero_n4) {
  // the step's BN-backward replica arena (chained mode) is cleared here: the head runs after every
  // BN backward of the previous step and before any of this step
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < zero_n4; i += (long)gridDim.x * 256)
    zero_buf[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  // Every phase issues ALL of a thread's global loads before consuming any of them: with
  // one workgroup per sample the kernel is latency-bound, and a load-use loop paid one
  // memory round trip per position / weight (round 1: 25 us for ResNet-18's 4x4x512 head).
  extern __shared__ float sm[];   // pooled[C], logits[16], dl[16], partial sums [pg][C]
  float* pl = sm;
  float* lg = sm + C;
  float* dl = lg + 16;
  float* ps = dl + 16;
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* yn = y + (size_t)n * HW * C;
  const float invHW = 1.f / (float)HW;
  {
    // thread = (position group pg, 8-channel group cg); 8 positions' 16-B loads in flight
    const int VC = C >> 3, npg = max(1, 256 / VC), cg = tid % VC, pg = tid / VC;
    if (pg < npg && cg < VC) {
      float s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = 0.f;
      for (int p0 = pg; p0 < HW; p0 += 8 * npg) {
        bf16x8v v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = p0 + u * npg;
          if (p < HW) v[u] = *reinterpret_cast<const bf16x8v*>(yn + (size_t)p * C + cg * 8);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (p0 + u * npg < HW) {
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += (float)v[u][j];
          }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ps[pg * C + cg * 8 + j] = s[j];
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      for (int g = 0; g < npg; ++g) s += ps[g * C + c];   // fixed order: deterministic
      pl[c] = s * invHW;
      if (train) pooled[(size_t)n * C + c] = s * invHW;
    }
  }
  __syncthreads();
  for (int j = wave; j < J; j += 4) {
    float s = 0.f;
    for (int c0 = lane; c0 < C; c0 += 64 * 8) {
      float w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = c0 + 64 * u < C ? W[(size_t)j * C + c0 + 64 * u] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (c0 + 64 * u < C) s += w[u] * pl[c0 + 64 * u];
    }
    s = wave_sum(s);
    if (lane == 0) lg[j] = s + b[j];
  }
  __syncthreads();
  if (tid == 0) {
    const int lab = labels[base + (dbase ? dbase[0] : 0) + n];
    float mx = lg[0];
    int am = 0;
    for (int j = 1; j < J; ++j)
      if (lg[j] > mx) { mx = lg[j]; am = j; }
    float se = 0.f;
    for (int j = 0; j < J; ++j) se += __expf(lg[j] - mx);
    const float lse = mx + __logf(se);
    lossv[n] = lse - lg[lab];   // summed in sample order by head_wgrad / head_loss (no float atomics)
    atomicAdd(reinterpret_cast<int*>(stats) + 1, am == lab ? 1 : 0);
    atomicAdd(reinterpret_cast<int*>(stats) + 2, 1);
    for (int j = 0; j < J; ++j) {
      const float p = __expf(lg[j] - lse);
      dl[j] = (p - (j == lab ? 1.f : 0.f)) / (float)N;
      if (train) dlog[(size_t)n * J + j] = dl[j];
    }
  }
  if (!train) return;
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = j < J ? W[(size_t)j * C + c] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < J) s += w[j] * dl[j];
    pl[c] = s * invHW;   // reuse: d pooled / HW
  }
  __syncthreads();
  bf16* dyn = dy + (size_t)n * HW * C;
  const int VR = C >> 3;   // C % 8 == 0: 16-B stores of 8 channels
  for (int e = tid; e < HW * VR; e += 256) {
    const int c0 = (e % VR) * 8;
    bf16x8v v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)pl[c0 + j];
    *reinterpret_cast<bf16x8v*>(dyn + (size_t)e * 8) = v;
  }
}

constexpr int HEAD_MAXN = 512;
// dW[j][c] = sum_n dlog[n][j] * pooled[n][c];  db[j] = sum_n dlog[n][j]   (N <= HEAD_MAXN)
// Block = 64 channels x 4 sample groups (fixed-order LDS combine: deterministic);
// block 0 also reduces db.  Loads are issued 8 at a time before use (the kernel has
// C/64 workgroups, so a load-use loop was one memory round trip per sample: 30 us).
// stats[0] += sum_n lossv[n] in a fixed order (256 strided partials, then an ordered LDS fold): the loss sum
// is bit-reproducible, unlike a float atomicAdd per sample.  Called by ONE workgroup.
FEDMI_DEV void ordered_loss_sum(const float* __restrict__ lossv, int N, float* __restrict__ stats, float* red) {
  float s = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) s += lossv[n];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) stats[0] += red[0];
}

__global__ __launch_bounds__(256) void head_loss_kernel(const float* __restrict__ lossv, int N, float* __restrict__ stats) {
  __shared__ float red[256];
  ordered_loss_sum(lossv, N, stats, red);
}

__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ pooled, const float* __restrict__ dlog,
                                                         int N, int C, int J, float* __restrict__ dW,
                                                         float* __restrict__ db, const float* __restrict__ lossv,
                                                         float* __restrict__ stats) {
  __shared__ float part[4][16][64];
  __shared__ float dls[HEAD_MAXN * 16];   // dlog staged once per block, read as LDS broadcasts
  const int cl = threadIdx.x & 63, ng = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  for (int i0 = threadIdx.x; i0 < N * J; i0 += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = i0 + 256 * u < N * J ? dlog[i0 + 256 * u] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + 256 * u;
      if (i < N * J) dls[(i / J) * 16 + i % J] = v[u];
    }
  }
  __syncthreads();
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int n0 = ng; n0 < N; n0 += 32) {
    float pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int n = n0 + 4 * u;
      pv[u] = (c < C && n < N) ? pooled[(size_t)n * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int n = n0 + 4 * u;
      if (n < N) {
        const float* dl = dls + n * 16;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j < J) acc[j] += dl[j] * pv[u];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) part[ng][j][cl] = acc[j];
  __syncthreads();
  for (int e = threadIdx.x; e < J * 64; e += 256) {
    const int j = e >> 6, cc = e & 63;
    if (blockIdx.x * 64 + cc < C)
      dW[(size_t)j * C + blockIdx.x * 64 + cc] = (part[0][j][cc] + part[1][j][cc]) + (part[2][j][cc] + part[3][j][cc]);
  }
  if (blockIdx.x == 0) {   // db: 16 classes x 16 sample groups from the staged dlog, then a fixed-order combine
    __syncthreads();
    const int j = threadIdx.x & 15, g = threadIdx.x >> 4;
    float s = 0.f;
    if (j < J)
      for (int n = g; n < N; n += 16) s += dls[n * 16 + j];
    float* red = &part[0][0][0];   // reuse: [16 groups][16 classes]
    red[g * 16 + j] = s;
    __syncthreads();
    if (threadIdx.x < J) {
      float t = 0.f;
      for (int q = 0; q < 16; ++q) t += red[q * 16 + threadIdx.x];
      db[threadIdx.x] = t;
    }
    __syncthreads();
    ordered_loss_sum(lossv, N, stats, red);
  }
}

// ---------------------------------------------------------------------------
// MaxPool2d(2, 2) on NHWC bf16 (VGG, src/models/vgg.py:24-25): one thread per
// (output pixel, 8 channels).  The backward recomputes the window argmax from
// the saved input (first maximum in window order, as max_pool2d_with_indices)
// instead of storing indices, and writes every input element (0 off-argmax).
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                           int H, int W, int C) {
  const int P = H >> 1, Q = W >> 1, VC = C >> 3;
  const uint32_t total = (uint32_t)N * P * Q * VC;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = i / VC;
    const int c0 = (int)(i - pix * VC) * 8;
    const uint32_t t = pix / Q;
    const int q = (int)(pix - t * Q);
    const int n = (int)(t / P), p = (int)(t - (uint32_t)n * P);
    const bf16* b = x + (((long)n * H + 2 * p) * W + 2 * q) * C + c0;
    const bf16x8v v0 = *reinterpret_cast<const bf16x8v*>(b);
    const bf16x8v v1 = *reinterpret_cast<const bf16x8v*>(b + C);
    const bf16x8v v2 = *reinterpret_cast<const bf16x8v*>(b + (long)W * C);
    const bf16x8v v3 = *reinterpret_cast<const bf16x8v*>(b + (long)W * C + C);
    bf16x8v o;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = (bf16)fmaxf(fmaxf((float)v0[j], (float)v1[j]), fmaxf((float)v2[j], (float)v3[j]));
    *reinterpret_cast<bf16x8v*>(y + (long)pix * C + c0) = o;
  }
}

__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                           bf16* __restrict__ dx, int N, int H, int W, int C) {
  const int P = H >> 1, Q = W >> 1, VC = C >> 3;
  const uint32_t total = (uint32_t)N * P * Q * VC;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = i / VC;
    const int c0 = (int)(i - pix * VC) * 8;
    const uint32_t t = pix / Q;
    const int q = (int)(pix - t * Q);
    const int n = (int)(t / P), p = (int)(t - (uint32_t)n * P);
    const long o00 = (((long)n * H + 2 * p) * W + 2 * q) * C + c0;
    const long offs[4] = {o00, o00 + C, o00 + (long)W * C, o00 + (long)W * C + C};
    bf16x8v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const bf16x8v*>(x + offs[k]);
    const bf16x8v g = *reinterpret_cast<const bf16x8v*>(dy + (long)pix * C + c0);
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float best = (float)v[0][j];
      am[j] = 0;
#pragma unroll
      for (int k = 1; k < 4; ++k)
        if ((float)v[k][j] > best) { best = (float)v[k][j]; am[j] = k; }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16x8v o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = am[j] == k ? g[j] : (bf16)0.f;
      *reinterpret_cast<bf16x8v*>(dx + offs[k]) = o;
    }
  }
}

// ---------------------------------------------------------------------------
// MaxPool2d(3, stride 1|2, padding 1) on NHWC bf16 (GoogLeNet branch 4 and its
// stage pools, src/models/googlenet.py:27-30, 79): forward saves the window
// argmax (tap 0..8, first maximum as max_pool2d_with_indices, padding never
// wins) as one byte per output element; backward is a gather over the <= 9
// windows covering each input pixel (no atomics), optionally accumulating into
// dx (the branch's share of a fan-in gradient).
// stride as a template parameter: the window / phase index math compiles to shifts instead of
// runtime integer divisions (GoogLeNet's inception pools: 63 us per backward launch with runtime st).
// maxpool3_bwd_kernel serves stride 2; the forward and the stride-1 backward are the register-blocked
// kernels below.
template <int ST>
__global__ __launch_bounds__(256) void maxpool3_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                           bf16* __restrict__ dx, int N, int H, int W, int C,
                                                           int P, int Q, int acc) {
  constexpr int st = ST;
  const int VC = C >> 3;
  const uint32_t total = (uint32_t)N * H * W * VC;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = i / VC;
    const int c0 = (int)(i - pix * VC) * 8;
    const uint32_t t = pix / W;
    const int w = (int)(pix - t * W);
    const int n = (int)(t / H), h = (int)(t - (uint32_t)n * H);
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ph = h + 1 - r;              // = p * st
      if (ph < 0 || ph % st) continue;
      const int p = ph / st;
      if (p >= P) continue;
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const int qw = w + 1 - s2;
        if (qw < 0 || qw % st) continue;
        const int q = qw / st;
        if (q >= Q) continue;
        const long o = (((long)n * P + p) * Q + q) * C + c0;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        const bf16x8v d = *reinterpret_cast<const bf16x8v*>(dy + o);
        const int tap = r * 3 + s2;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((int)((packed >> (8 * j)) & 0xff) == tap) g[j] += (float)d[j];
      }
    }
    bf16* dst = dx + (long)pix * C + c0;
    if (acc) {
      const bf16x8v e = *reinterpret_cast<const bf16x8v*>(dst);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] += (float)e[j];
    }
    bf16x8v o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)g[j];
    *reinterpret_cast<bf16x8v*>(dst) = o;
  }
}

// cur[0] = sched[counter[0]++]  (first node of a captured training step); the other lanes / workgroups zero the
// step's fp64 BN-statistics accumulators (n doubles, 16-B stores): one fedmi launch instead of sched + an ATen fill
__global__ __launch_bounds__(256) void sched_next_kernel(const int* __restrict__ sched, int* __restrict__ counter,
                                                         int* __restrict__ cur, double* __restrict__ zero, long n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int i = counter[0];
    cur[0] = sched[i];
    counter[0] = i + 1;
  }
  const long n2 = n >> 1;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256)
    reinterpret_cast<double2*>(zero)[i] = make_double2(0.0, 0.0);
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 64) zero[n - 1] = 0.0;
}

int grid_for(long nv) { return (int)std::min<long>((nv + 255) / 256, 2048); }

// bn_apply / bn_bwd_apply grid: y = channel chunks of kBnChunk, x = row chunks of ~8 rows per thread-row
// slot (C % 8 == 0; chunks of 64 channels need C % 64 == 0 when C > 64)
bool use_chunked(int C) { return C >= 256 && C % kBnChunk == 0; }

dim3 apply_grid(int M, int C) {
  const int CC = std::min(kBnChunk, C), nch = C / CC, rstep = 256 / (CC / 8);
  const long want = ((long)M + 2L * rstep - 1) / (2L * rstep);   // ~2 rows per thread-slot
  const int bx = (int)std::max<long>(1, std::min<long>(want, std::max(1, 2048 / nch)));
  return dim3(bx, nch);
}

}  // namespace

namespace fedmi {

struct BNDesc {
  const double* stats; const float* gamma; const float* beta; float* rmean; float* rvar; long long* nbt;
  float* smean; float* sinv; const float* shift; const float* cbias;
};

static BNArgs to_args(const BNDesc& d) {
  return BNArgs{d.stats, d.gamma, d.beta, d.rmean, d.rvar, d.nbt, d.smean, d.sinv, d.shift, d.cbias};
}

// Register-blocked forms (QB horizontally adjacent outputs per thread): the (QB - 1) * ST + 3 input columns of
// the QB windows are loaded once (stride 1, QB 4: 18 loads for 4 outputs instead of 36), and every output scans its
// window in the same (r, s) order with the same strict '>' as maxpool3_fwd_kernel -- bit-identical values and
// argmax codes.  GoogLeNet's 32x32x192/256 branch pools spent 40 us (fwd) / 53 us (bwd) per call re-reading each
// input vector 9 times.
template <int ST, int QB>
__global__ __launch_bounds__(256) void maxpool3_fwd_blk_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                               uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                               int P, int Q) {
  constexpr int NCOL = (QB - 1) * ST + 3;
  const int VC = C >> 3;
  const int QBk = (Q + QB - 1) / QB;
  const uint32_t total = (uint32_t)N * P * QBk * VC;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pb = i / VC;
    const int c0 = (int)(i - pb * VC) * 8;
    const uint32_t t = pb / QBk;
    const int q0 = (int)(pb - t * QBk) * QB;
    const int n = (int)(t / P), p = (int)(t - (uint32_t)n * P);
    const int w0 = q0 * ST - 1;
    float best[QB][8];
    int am[QB][8];
#pragma unroll
    for (int k = 0; k < QB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[k][j] = -INFINITY; am[k][j] = 0; }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = p * ST - 1 + r;
      const bool hok = (unsigned)h < (unsigned)H;
      bf16x8v v[NCOL];
      bool ok[NCOL];
#pragma unroll
      for (int cc = 0; cc < NCOL; ++cc) {
        const int w = w0 + cc;
        ok[cc] = hok && (unsigned)w < (unsigned)W;
        v[cc] = *reinterpret_cast<const bf16x8v*>(x + (ok[cc] ? (((long)n * H + h) * W + w) * C + c0 : c0));
      }
#pragma unroll
      for (int k = 0; k < QB; ++k)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
          const int cc = k * ST + s2;
          if (!ok[cc]) continue;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if ((float)v[cc][j] > best[k][j]) { best[k][j] = (float)v[cc][j]; am[k][j] = r * 3 + s2; }
        }
    }
#pragma unroll
    for (int k = 0; k < QB; ++k) {
      if (q0 + k >= Q) break;
      bf16x8v o;
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (bf16)best[k][j];
        packed |= (uint64_t)am[k][j] << (8 * j);
      }
      const long pix = ((long)n * P + p) * Q + q0 + k;
      *reinterpret_cast<bf16x8v*>(y + pix * C + c0) = o;
      *reinterpret_cast<uint64_t*>(idx + pix * C + c0) = packed;
    }
  }
}

// stride-1 backward, QB adjacent input pixels per thread: the (QB + 2) x 3 covering windows' (code, grad) pairs are
// loaded once; each pixel sums its windows in maxpool3_bwd_kernel's (r, s) order (bit-identical)
template <int QB>
__global__ __launch_bounds__(256) void maxpool3_bwd1_blk_kernel(const bf16* __restrict__ dy,
                                                                const uint8_t* __restrict__ idx, bf16* __restrict__ dx,
                                                                int N, int H, int W, int C, int acc) {
  constexpr int NCOL = QB + 2;
  const int VC = C >> 3;
  const int WBk = (W + QB - 1) / QB;
  const uint32_t total = (uint32_t)N * H * WBk * VC;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pb = i / VC;
    const int c0 = (int)(i - pb * VC) * 8;
    const uint32_t t = pb / WBk;
    const int w0 = (int)(pb - t * WBk) * QB;
    const int n = (int)(t / H), h = (int)(t - (uint32_t)n * H);
    float g[QB][8];
#pragma unroll
    for (int k = 0; k < QB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) g[k][j] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int p = h + 1 - r;                // output row whose window holds input row h at tap row r
      if ((unsigned)p >= (unsigned)H) continue;
      uint64_t pk[NCOL];
      bf16x8v d[NCOL];
      bool ok[NCOL];
#pragma unroll
      for (int cc = 0; cc < NCOL; ++cc) {     // output columns q = w0 - 1 + cc
        const int q = w0 - 1 + cc;
        ok[cc] = (unsigned)q < (unsigned)W;
        const long o = ok[cc] ? (((long)n * H + p) * W + q) * C + c0 : c0;
        pk[cc] = *reinterpret_cast<const uint64_t*>(idx + o);
        d[cc] = *reinterpret_cast<const bf16x8v*>(dy + o);
      }
#pragma unroll
      for (int k = 0; k < QB; ++k)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
          const int cc = k + 2 - s2;          // q = (w0 + k) + 1 - s2
          if (!ok[cc]) continue;
          const int tap = r * 3 + s2;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if ((int)((pk[cc] >> (8 * j)) & 0xff) == tap) g[k][j] += (float)d[cc][j];
        }
    }
#pragma unroll
    for (int k = 0; k < QB; ++k) {
      if (w0 + k >= W) break;
      bf16* dst = dx + (((long)n * H + h) * W + w0 + k) * C + c0;
      if (acc) {
        const bf16x8v e = *reinterpret_cast<const bf16x8v*>(dst);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[k][j] += (float)e[j];
      }
      bf16x8v o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)g[k][j];
      *reinterpret_cast<bf16x8v*>(dst) = o;
    }
  }
}

void launch_maxpool3(hipStream_t st, const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C, int stride) {
  if (C % 8 || (stride != 1 && stride != 2)) throw std::invalid_argument("maxpool3: need C % 8 == 0, stride 1|2");
  const int P = (H + 2 - 3) / stride + 1, Q = (W + 2 - 3) / stride + 1;
  if (stride == 1)
    hipLaunchKernelGGL((maxpool3_fwd_blk_kernel<1, 4>), dim3(grid_for((long)N * P * ((Q + 3) / 4) * (C / 8))),
                       dim3(256), 0, st, x, y, idx, N, H, W, C, P, Q);
  else
    hipLaunchKernelGGL((maxpool3_fwd_blk_kernel<2, 2>), dim3(grid_for((long)N * P * ((Q + 1) / 2) * (C / 8))),
                       dim3(256), 0, st, x, y, idx, N, H, W, C, P, Q);
}

void launch_maxpool3_bwd(hipStream_t st, const bf16* dy, const uint8_t* idx, bf16* dx, int N, int H, int W, int C,
                         int stride, int acc) {
  if (C % 8 || (stride != 1 && stride != 2)) throw std::invalid_argument("maxpool3_bwd: need C % 8 == 0, stride 1|2");
  const int P = (H + 2 - 3) / stride + 1, Q = (W + 2 - 3) / stride + 1;
  if (stride == 1)
    hipLaunchKernelGGL(maxpool3_bwd1_blk_kernel<4>, dim3(grid_for((long)N * H * ((W + 3) / 4) * (C / 8))), dim3(256), 0,
                       st, dy, idx, dx, N, H, W, C, acc);
  else
    hipLaunchKernelGGL(maxpool3_bwd_kernel<2>, dim3(grid_for((long)N * H * W * (C / 8))), dim3(256), 0, st, dy, idx, dx,
                       N, H, W, C, P, Q, acc);
}

void launch_maxpool2(hipStream_t st, const bf16* x, bf16* y, int N, int H, int W, int C) {
  if (C % 8 || H % 2 || W % 2) throw std::invalid_argument("maxpool2: need C % 8 == 0 and even H, W");
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid_for((long)N * (H / 2) * (W / 2) * (C / 8))), dim3(256), 0, st, x,
                     y, N, H, W, C);
}

void launch_maxpool2_bwd(hipStream_t st, const bf16* x, const bf16* dy, bf16* dx, int N, int H, int W, int C) {
  if (C % 8 || H % 2 || W % 2) throw std::invalid_argument("maxpool2_bwd: need C % 8 == 0 and even H, W");
  hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(grid_for((long)N * (H / 2) * (W / 2) * (C / 8))), dim3(256), 0, st, x,
                     dy, dx, N, H, W, C);
}

void launch_prep_input(hipStream_t st, const uint8_t* images, int base, const int* dbase, int nb, int augment,
                       uint32_t seed, const int* round_ctr, bf16* out) {
  hipLaunchKernelGGL(prep_input_kernel, dim3((nb * 1024 + 255) / 256), dim3(256), 0, st, images, base, dbase, nb,
                     augment, seed, round_ctr, out);
}

void launch_sched_next(hipStream_t st, const int* sched, int* counter, int* cur, double* zero, long n) {
  if (zero == nullptr) n = 0;
  const int grid = (int)std::max<long>(1, std::min<long>(((n >> 1) + 255) / 256, 256));
  hipLaunchKernelGGL(sched_next_kernel, dim3(grid), dim3(256), 0, st, sched, counter, cur, zero, n);
}

// co_out (optional): BN-A's scale / shift [2][C] as applied (a backward that derives the ReLU mask from z)
void launch_bn_apply(hipStream_t st, const bf16* z, const BNDesc& a, const bf16* z2, const BNDesc* b, const bf16* res,
                     bf16* y, int M, int C, float eps, float mom, int train, int relu, int ldy, float* co_out) {
  if (C % 8) throw std::invalid_argument("bn_apply: C % 8 != 0");
  if (ldy <= 0) ldy = C;
  if (ldy < C || ldy % 8) throw std::invalid_argument("bn_apply: bad output row stride");
  if ((long)M * (C / 8) >= (1l << 31)) throw std::invalid_argument("bn_apply: tensor too large for 32-bit indexing");
  const int res_mode = b ? 2 : (res ? 1 : 0);
  const BNArgs bb = b ? to_args(*b) : BNArgs{};
  if (use_chunked(C)) {
    const dim3 grid = apply_grid(M, C);
    hipLaunchKernelGGL(bn_apply_chunk_kernel, grid, dim3(256), 0, st, z, to_args(a), z2, bb, res, y, M, C, eps, mom,
                       train, relu, res_mode, ldy, (M + (int)grid.x - 1) / (int)grid.x, co_out);
  } else {
    hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for((long)M * (C / 8))), dim3(256), 4 * C * sizeof(float), st, z,
                       to_args(a), z2, bb, res, y, M, C, eps, mom, train, relu, res_mode, ldy, co_out);
  }
}


struct BNBwdDesc {
  const bf16* dya; const bf16* dyb; const bf16* y;
  const bf16* za; const float* meanA; const float* invA; const float* gammaA; float* dgammaA; float* dbetaA; bf16* dza;
  const bf16* zb; const float* meanB; const float* invB; const float* gammaB; float* dgammaB; float* dbetaB; bf16* dzb;
  bf16* gout;
  float* shiftA; float* shiftB;
  const bf16* dadd;
  const float* msc;
};

static void bn_bwd_grid(int M, int C, int* tb, int* rows_per_block, int* nblk) {
  const int VR = C / 8;
  *tb = (256 / VR) * VR;   // block size a multiple of C/8: fixed channel group per thread
  const int rstep = *tb / VR;
  // <= 1024 row-blocks (~4 per CU), each >= 2 row passes of the block
  *rows_per_block = std::max(2 * rstep, (M + 1023) / 1024);
  *nblk = (M + *rows_per_block - 1) / *rows_per_block;
}

// Scratch (fp64 elements) the two-level reduction of launch_bn_bwd needs (ZERO-initialised
// once by the caller; every launch leaves it zero again).
long bn_bwd_ws_floats(int M, int C) {
  (void)M;
  return (long)BN_REP * 3 * C;
}

// red: [3][C] fp64.  With ``ws`` (fp64, >= bn_bwd_ws_floats elements, zero): replica atomics + a
// finalize launch (red needs no zeroing).  Without: atomics into red, which must
// be zero on entry.
// Replicas per channel sum in chained mode: <= 2048 values per quantity, 4..16 (a replica spreads
// the reduce workgroups' same-address atomics; the apply prologue reads them all).
int bn_bwd_chain_reps(int C) { return std::max(4, std::min(16, 2048 / std::max(C, 1))); }

// presummed (chained mode only): the channel sums are already in ``ws`` -- the DGRAD that produced dya
// took them in its epilogue (conv_igemm.hip BnSums) -- so only the apply pass runs.
void launch_bn_bwd(hipStream_t st, const BNBwdDesc& d, double* red, int M, int C, double* ws, long ws_floats, int ldd,
                   int ldy, int chained, int presummed) {
  const int VR = C / 8;
  if (C % 8 || VR > 256) throw std::invalid_argument("bn_bwd: need C % 8 == 0 and C <= 2048");
  if (ldd <= 0) ldd = C;
  if (ldy <= 0) ldy = C;
  if (ldd < C || ldy < C || ldd % 8 || ldy % 8) throw std::invalid_argument("bn_bwd: bad row strides");
  if ((long)M * VR >= (1l << 31)) throw std::invalid_argument("bn_bwd: tensor too large for 32-bit indexing");
  if (d.msc && (d.y || ldd != C)) throw std::invalid_argument("bn_bwd: the z-derived ReLU mask needs y == null, compact rows");
  BwdIn in{d.dya, d.dyb, d.y, d.za, d.meanA, d.invA, d.zb, d.meanB, d.invB, ldd, ldy, d.msc};
  BwdOut out{d.dza, d.dzb, d.gout, d.dgammaA, d.dbetaA, d.dgammaB, d.dbetaB, d.gammaA, d.gammaB, d.shiftA, d.shiftB,
             d.dadd};
  int tb, rows_per_block, nblk;
  bn_bwd_grid(M, C, &tb, &rows_per_block, &nblk);
  if (chained) {
    // ws: this BN's own replica buffer, ZERO on entry (the head kernel clears the arena every step)
    const int reps = bn_bwd_chain_reps(C);
    if (!ws || ws_floats < (long)reps * 3 * C) throw std::invalid_argument("bn_bwd: chained replicas too small");
    if (presummed && d.dyb)
      throw std::invalid_argument("bn_bwd: presummed sums cover one incoming grad");
    if (!presummed)
      hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(tb), 0, st, in, red, M, C, rows_per_block, ws, reps);
    if (use_chunked(C)) {
      const dim3 ag = apply_grid(M, C);
      hipLaunchKernelGGL(bn_bwd_apply_chunk_kernel, ag, dim3(256), 0, st, in, out, red, M, C, ws, reps,
                         (M + (int)ag.x - 1) / (int)ag.x);
    } else {
      const int gblk = (int)std::min<long>(((long)M * VR + 255) / 256, 1024);
      hipLaunchKernelGGL(bn_bwd_apply_flat_kernel, dim3(gblk), dim3(256), 6 * C * sizeof(float), st, in, out, red, M,
                         C, ws, reps);
    }
    return;
  }
  if (presummed) throw std::invalid_argument("bn_bwd: presummed needs chained replicas");
  const bool two = ws && ws_floats >= (long)BN_REP * 3 * C;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(tb), 0, st, in, red, M, C, rows_per_block,
                     two ? ws : nullptr, BN_REP);
  if (two) hipLaunchKernelGGL(bn_bwd_finalize, dim3((3 * C + 255) / 256), dim3(256), 0, st, ws, C, red);
  if (use_chunked(C)) {
    const dim3 ag = apply_grid(M, C);
    hipLaunchKernelGGL(bn_bwd_apply_chunk_kernel, ag, dim3(256), 0, st, in, out, red, M, C, nullptr, 0,
                       (M + (int)ag.x - 1) / (int)ag.x);
  } else {
    hipLaunchKernelGGL(bn_bwd_apply_flat_kernel, dim3(grid_for((long)M * VR)), dim3(256), 6 * C * sizeof(float), st,
                       in, out, red, M, C, nullptr, 0);
  }
}

void launch_head(hipStream_t st, const bf16* y, const int* labels, int base, const int* dbase, int N, int HW, int C, int J,
                 const float* W, const float* b, float* pooled, float* dlog, bf16* dy, float* stats, float* lossv,
                 float* dW, float* db, int train, float* zero_buf, long zero_n) {
  if (lossv == nullptr) throw std::invalid_argument("head: per-sample loss buffer required");
  if (zero_n % 4 || (reinterpret_cast<uintptr_t>(zero_buf) & 15)) throw std::invalid_argument("head: zero arena alignment");
  if (J > 16) throw std::invalid_argument("head: at most 16 classes");
  if (C % 8 || C > 2048) throw std::invalid_argument("head: need C % 8 == 0 and C <= 2048");
  const int npg = std::max(1, 256 / (C / 8));
  hipLaunchKernelGGL(head_fwd_bwd_kernel, dim3(N), dim3(256), (C + 32 + npg * C) * sizeof(float), st, y, labels, base, dbase, HW, C,
                     J, W, b, pooled, dlog, dy, stats, lossv, N, train,
                     reinterpret_cast<float4*>(zero_buf), zero_n / 4);
  if (train && N > HEAD_MAXN) throw std::invalid_argument("head: training batch > 512");
  if (train)
    hipLaunchKernelGGL(head_wgrad_kernel, dim3((C + 63) / 64), dim3(256), 0, st, pooled, dlog, N, C, J, dW, db, lossv,
                       stats);
  else
    hipLaunchKernelGGL(head_loss_kernel, dim3(1), dim3(256), 0, st, lossv, N, stats);
}

}  // namespace fedmi
