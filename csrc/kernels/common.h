// fedmi — shared device helpers for the CDNA4 (gfx950) kernels.
//
// Everything here is written for a 64-lane wavefront and the gfx950 MFMA
// fragment maps (cdna_hip_programming.md §3):
//   mfma_f32_16x16x32_bf16:  A lane l holds A[l&15][8*(l>>4)+j], j=0..7
//                            B lane l holds B[8*(l>>4)+j][l&15]
//                            C lane l holds C[(l>>4)*4+r][l&15],  r=0..3
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define FEDMI_DEV __device__ __forceinline__

// BatchNorm batch statistics are accumulated into STAT_REP replicas
// [STAT_REP][2][C] (replica = producing workgroup % STAT_REP): the per-channel
// atomics of hundreds of workgroups would otherwise serialise on 2*C addresses.
// Consumers (bn_apply) sum the replicas.
constexpr int STAT_REP = 16;

FEDMI_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

FEDMI_DEV f32x4 zero4() { f32x4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

FEDMI_DEV bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  return z;
}

FEDMI_DEV int lane_id() { return threadIdx.x & 63; }
FEDMI_DEV int wave_id() { return threadIdx.x >> 6; }

// Counter-based RNG (stateless): one 32-bit draw per (seed, a, b) triple.
// Used for the on-device RandomCrop/RandomHorizontalFlip augmentation so the
// whole local epoch can be captured in a graph and replayed.
FEDMI_DEV uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u;
  h ^= (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du;
  h ^= h >> 12; h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

// Wave64 sum via DPP-free shuffles.
FEDMI_DEV float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---- optional per-phase timestamps (diagnostic build: -DFEDMI_STAMPS) -------
// Lane 0 of each workgroup records s_memtime at phase boundaries (after the
// phase's barrier), so phase shares can be read without a profiler.
#define FEDMI_STAMP_KERNELS 4
#define FEDMI_STAMP_WGS 1024
#define FEDMI_STAMP_SLOTS 8
#ifdef FEDMI_STAMPS
extern __device__ unsigned long long fedmi_stamps[FEDMI_STAMP_KERNELS][FEDMI_STAMP_WGS][FEDMI_STAMP_SLOTS];
// 'stamp_wg' (a local of the enclosing function) is the workgroup's slot: kernels that host
// several roles in one launch stamp each role under its own index.
#define FEDMI_STAMP(k, i)                                                                   \
  do {                                                                                      \
    if (threadIdx.x == 0 && stamp_wg >= 0 && stamp_wg < FEDMI_STAMP_WGS)                    \
      fedmi_stamps[k][stamp_wg][i] = __builtin_amdgcn_s_memtime();                          \
  } while (0)
#else
#define FEDMI_STAMP(k, i) do {} while (0)
#endif

namespace fedmi {
// BatchNorm-backward channel sums of the BN that PRODUCED a DGRAD's output, taken in the DGRAD
// epilogue (tap kernel or split-K combine) instead of a separate pass over (dy, z, y):
//   g = bf16(dX)[row][c] * (y[row][c] > 0, or 1 without a ReLU)
//   rep[blk % reps][0][c] += sum g,   rep[blk % reps][1][c] += sum g * (z[row][c] - mean[c]) * inv[c]
//   (rep[..][2][c] += sum g * (zb - meanb) * invb: a projection-shortcut BN sharing g)
// -- the chained replica layout bn_bwd's apply kernel reads (cnn_ops.hip, launch_bn_bwd presummed).
struct BnSums {
  double* rep;          // [reps][3][C] fp64, zero at the step start (null: off)
  const bf16* z;        // the BN's input (its conv's output), compact [rows][C]
  const bf16* y;        // the BN's ReLU output (mask) or null
  const float* mean;    // saved batch mean / inverse std of the BN
  const float* inv;
  int reps;
  const bf16* zb;       // second BN branch (projection shortcut) or null
  const float* meanb;
  const float* invb;
  const float* msc;     // y == null: [2][C] scale / shift the forward applied; ReLU mask = z * sc + sh > 0
  int msc_ld;           // C (row stride of msc)
};

// one 8-channel group of a DGRAD output row into the BN-backward sums (bm/bi: [2][8] mean / inv of
// the two branches; q: [3][8])
// the same on operands already in registers (an epilogue that prefetched its rows' z / y / zb)
FEDMI_DEV void bnsum_acc_v(const BnSums& bs, const bf16x8& t, const bf16x8& z, const bf16x8& y, const bf16x8& zb,
                           const float (*bm)[8], const float (*bi)[8], float (*q)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float g = (float)t[j];
    if (bs.y && !((float)y[j] > 0.f)) g = 0.f;
    else if (!bs.y && bs.msc && !((float)z[j] * bm[2][j] + bi[2][j] > 0.f)) g = 0.f;
    q[0][j] += g;
    q[1][j] += g * ((float)z[j] - bm[0][j]) * bi[0][j];
    if (bs.zb) q[2][j] += g * ((float)zb[j] - bm[1][j]) * bi[1][j];
  }
}

FEDMI_DEV void bnsum_acc(const BnSums& bs, long idx, const bf16x8& t, const float (*bm)[8], const float (*bi)[8],
                         float (*q)[8]) {   // bm / bi: [3][8] (see bnsum_coeffs)
  const bf16x8 z = *reinterpret_cast<const bf16x8*>(bs.z + idx);
  bf16x8 y{}, zb{};
  if (bs.y) y = *reinterpret_cast<const bf16x8*>(bs.y + idx);
  if (bs.zb) zb = *reinterpret_cast<const bf16x8*>(bs.zb + idx);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float g = (float)t[j];
    if (bs.y && !((float)y[j] > 0.f)) g = 0.f;
    else if (!bs.y && bs.msc && !((float)z[j] * bm[2][j] + bi[2][j] > 0.f)) g = 0.f;
    q[0][j] += g;
    q[1][j] += g * ((float)z[j] - bm[0][j]) * bi[0][j];
    if (bs.zb) q[2][j] += g * ((float)zb[j] - bm[1][j]) * bi[1][j];
  }
}

// mean / inv of an 8-channel group (both branches; [2]: the z-mask scale / shift), zero past the last channel
FEDMI_DEV void bnsum_coeffs(const BnSums& bs, int c0, bool ok, float (*bm)[8], float (*bi)[8], float (*q)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    q[0][j] = q[1][j] = q[2][j] = 0.f;
    bm[0][j] = ok ? bs.mean[c0 + j] : 0.f;
    bi[0][j] = ok ? bs.inv[c0 + j] : 0.f;
    bm[1][j] = ok && bs.zb ? bs.meanb[c0 + j] : 0.f;
    bi[1][j] = ok && bs.zb ? bs.invb[c0 + j] : 0.f;
    bm[2][j] = ok && bs.msc ? bs.msc[c0 + j] : 0.f;
    bi[2][j] = ok && bs.msc ? bs.msc[bs.msc_ld + c0 + j] : 0.f;
  }
}

// torch.optim.SGD on one element (momentum buffer b): d = g + wd * p, b = m * b + (1 - dampening) * d (d on the
// first step), d = nesterov ? d + m * b : b, p -= lr * d.  sgd_flat_kernel and the fused SGD + weight-image pack
// (sgd_pack_kernel) both use it, so the two paths are bit-identical.
FEDMI_DEV void sgd_elem(float& p, float g, float& b, float lr, float m, float wd, float dampening, int nesterov,
                        int first) {
  float d = g + wd * p;
  if (m != 0.f) {
    b = first ? d : m * b + (1.f - dampening) * d;
    d = nesterov ? d + m * b : b;
  }
  p -= lr * d;
}

}  // namespace fedmi
