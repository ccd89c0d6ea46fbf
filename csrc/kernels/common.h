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
