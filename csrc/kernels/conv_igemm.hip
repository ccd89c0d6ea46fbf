// fedmi — implicit-GEMM 2-D convolution on gfx950 MFMA (bf16 in, fp32 acc).
//
// One kernel template serves the three convolution GEMMs of training, all on
// NHWC (channels-last) bf16 activations and an [O][R][S][C] bf16 weight image
// ("W_rsc", packed from the fp32 master [O][C][R][S] by conv_pack_weights):
//
//   FWD    Y[m=(n,p,q)][o]     = sum_{k=(r,s,c)} X[n][p*st-pad+r][q*st-pad+s][c] * W[o][r][s][c]
//   DGRAD  dX[m=(n,h,w)][c]    = sum_{k=(r,s,o)} dY[n][(h+pad-r)/st][(w+pad-s)/st][o] * W[o][r][s][c]
//   WGRAD  dW[o][j=(r,s,c)]   += sum_{k=m=(n,p,q)} dY[m][o] * X[n][p*st-pad+r][q*st-pad+s][c]   (split-K)
//
// Tiles: BM x BN output tile, BK = 64, 256 threads = 4 waves in a 2x2 grid,
// each wave (BM/2) x (BN/2) of 16x16 MFMA sub-tiles (v_mfma_f32_16x16x32_bf16).
// Operands are staged global -> registers -> LDS (double-buffered LDS, one
// barrier per K step, the next tile's loads in flight behind the MFMAs).
// Each operand tile is stored in the layout it has in global memory:
//   * "KC"  (K contiguous: im2col rows of X / dY, W_rsc rows)  -> [rows][BK+8]
//     image, MFMA fragments read with ds_read_b128 (16-B row reads; the +8
//     element pad makes the 16 rows of a fragment hit distinct bank groups).
//   * "MNC" (M/N contiguous: weight columns for DGRAD, pixel-major dY / X for
//     WGRAD) -> [BK][cols] image with a 32-byte-segment XOR swizzle, fragments
//     read with ds_read_b64_tr_b16 (gfx950 hardware transpose; conflict-free
//     for the swizzle below).
// So no operand is ever transposed in registers or through extra buffers.
//
// Epilogues: FWD writes bf16 Y and (optionally) per-channel sum / sum-of-
// squares for the following BatchNorm (training batch statistics fused into
// the conv); DGRAD writes bf16 dX; WGRAD atomically adds the
// fp32 partial into the PyTorch-layout [O][C][R][S] gradient (split-K over
// output pixels, gridDim.z splits).
//
// Reference parity: these are the convolution / convolution_backward ops of
// every zoo model (src/models/resnet.py:14-104 etc.).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>
#include <stdexcept>

#include "common.h"
#include "wgrad_reduce.h"

// diagnostic build (-DFEDMI_STAMPS): s_memtime per conv_tap phase, lane 0 of each workgroup
// (tools/diag_conv_stamps.py); device code is per translation unit, so conv stamps have their own array
#ifdef FEDMI_STAMPS
__device__ unsigned long long fedmi_conv_stamps[FEDMI_STAMP_WGS][FEDMI_STAMP_SLOTS];
#define CONV_STAMP(i)                                                                       \
  do {                                                                                      \
    if (threadIdx.x == 0 && stamp_wg >= 0 && stamp_wg < FEDMI_STAMP_WGS)                    \
      fedmi_conv_stamps[stamp_wg][i] = __builtin_amdgcn_s_memtime();                        \
  } while (0)
#else
#define CONV_STAMP(i) do {} while (0)
#endif

void read_conv_stamps(unsigned long long* host, bool clear) {
#ifdef FEDMI_STAMPS
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(fedmi_conv_stamps), sizeof(fedmi_conv_stamps), 0, hipMemcpyDeviceToHost);
  if (clear) {
    static unsigned long long zeros[FEDMI_STAMP_WGS][FEDMI_STAMP_SLOTS];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(fedmi_conv_stamps), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
  }
#else
  (void)host;
  (void)clear;
#endif
}

namespace {

struct FastDiv {   // q = x / d for 0 <= x < 2^31 (Granlund-Montgomery)
  uint32_t d, m, s;
};
FEDMI_DEV uint32_t fdiv(uint32_t x, const FastDiv& f) { return (__umulhi(x, f.m) + x) >> f.s; }

struct ConvGeom {
  int N, H, W, C;          // input (C = padded channel count, % 8 == 0)
  int O, P, Q;             // output channels / spatial
  int R, S, st, pad;
  int M, NC, K;            // GEMM rows / cols / reduction for the launched mode
  int Cw;                  // channel count of the fp32 master weight (unpadded; WGRAD epilogue)
  // DGRAD sub-pixel phase (stride 2: one launch per output parity (ph, pw), each
  // summing only the taps r = r0 + 2i, s = s0 + 2j that land on that parity;
  // stride 1: ph = pw = 0, r0 = s0 = 0, nr = R, ns = S, Hp = H, Wp = W)
  int ph, pw, r0, s0, nr, ns, Hp, Wp;
  FastDiv dC, dO, dS, dQ, dPQ, dW, dHW, dNS, dWp, dHWp;
};

// GEMM row m = (n, p, q) over an output grid P x Q -> row of the stored output:
// identity, or the stride-`st` sub-pixel scatter of a DGRAD phase:
// ((n * OH + p * st + ph) * OW + q * st + pw).
struct RowMap {
  int on;
  int P, Q, OH, OW, st, ph, pw;
  FastDiv dPQ, dQ;
};
FEDMI_DEV long map_row(const RowMap& r, int m) {
  if (!r.on) return m;
  const uint32_t n = fdiv(m, r.dPQ), pq = m - n * r.P * r.Q;
  const uint32_t p = fdiv(pq, r.dQ), q = pq - p * r.Q;
  return ((long)n * r.OH + p * r.st + r.ph) * r.OW + q * r.st + r.pw;
}

using fedmi::BnSums;

enum { FWD = 0, DGRAD = 1, WGRAD = 2 };
constexpr int BK = 64;
constexpr int KC_LD = BK + 8;   // KC image row stride (elements): 144 B = 9 x 16 B

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

FEDMI_DEV uint4 zero_u4() { return make_uint4(0u, 0u, 0u, 0u); }
FEDMI_DEV uint4 ld16(const bf16* p) { return *reinterpret_cast<const uint4*>(p); }

// MNC image: [BK rows][COLS] bf16, 32-byte segments XOR-swizzled by row so that
// a ds_read_b64_tr_b16 (per 32-lane half: rows k0..k0+3 and k0+8..k0+11 of one
// 16-column block) touches 64 distinct banks.
template <int COLS>
FEDMI_DEV int mnc_off(int row, int col) {
  if constexpr (COLS == 128) {
    const int f = (row & 3) | (((row >> 3) & 1) << 2);
    return row * 128 + ((((col >> 4) ^ f)) << 4) + (col & 15);
  } else {   // 64
    const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    return row * 64 + ((((col >> 4) ^ f)) << 4) + (col & 15);
  }
}

// Fragment readers (16x16x32 operand of rows/cols [i0, i0+16), k in [kk*32, kk*32+32)).
FEDMI_DEV bf16x8 frag_kc(const bf16* img, int i0, int kk, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + (i0 + (lane & 15)) * KC_LD + kk * 32 + (lane >> 4) * 8);
}

template <int COLS>
FEDMI_DEV bf16x8 frag_mnc(const bf16* img, int i0, int kk, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int row0 = kk * 32 + 8 * g + q;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const bf16* a0 = img + mnc_off<COLS>(row0, i0 + 4 * p);
  const bf16* a1 = img + mnc_off<COLS>(row0 + 4, i0 + 4 * p);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  // whole-vector bit casts: per-element short->bf16 casts of the tr16 result were
  // miscompiled (elements 2,3 duplicated from 0,1)
  const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo);
  const bf16x4 h4 = __builtin_bit_cast(bf16x4, hi);
  return __builtin_shufflevector(l4, h4, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ---------------------------------------------------------------------------
// Per-thread operand loaders. Each thread owns NCH 16-byte chunks of each
// operand tile per K step; the chunk -> (row, k-chunk) map is fixed across the
// K loop, so per-row decode work is hoisted out of it.
// ---------------------------------------------------------------------------
template <int MODE, int BM, int BN>
struct Loader {
  static constexpr int NA = BM * BK / 8 / 256;   // chunks per thread, A
  static constexpr int NB = BN * BK / 8 / 256;
  // A rows (KC: FWD/DGRAD) or k-rows (MNC: WGRAD)
  int a_row[NA], a_kc[NA];
  int a_n[NA], a_h[NA], a_w[NA];   // FWD: n, p*st-pad, q*st-pad ; DGRAD: n, h+pad, w+pad
  bool a_ok[NA];
  int b_row[NB], b_kc[NB];
  int b_r[NB], b_s[NB], b_c[NB];   // WGRAD: fixed (r,s,c) of the column chunk
  bool b_ok[NB];

  FEDMI_DEV void init(const ConvGeom& g, int m0, int n0, int tid) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int c = tid + 256 * u;
      if constexpr (MODE == WGRAD) {          // MNC: [BK][BM]
        a_row[u] = c / (BM / 8);
        a_kc[u] = c % (BM / 8);
        a_ok[u] = m0 + a_kc[u] * 8 < g.M;     // o chunk in range (O % 8 == 0)
      } else {                                // KC: [BM][BK]
        a_row[u] = c >> 3;
        a_kc[u] = c & 7;
        const int m = m0 + a_row[u];
        a_ok[u] = m < g.M;
        const uint32_t mm = a_ok[u] ? m : 0;
        if constexpr (MODE == FWD) {
          const uint32_t n = fdiv(mm, g.dPQ), pq = mm - n * g.P * g.Q;
          const uint32_t p = fdiv(pq, g.dQ), q = pq - p * g.Q;
          a_n[u] = n; a_h[u] = p * g.st - g.pad; a_w[u] = q * g.st - g.pad;
        } else {   // DGRAD: row -> (n, hh, ww) of this phase -> input pixel (h, w)
          const uint32_t n = fdiv(mm, g.dHWp), hw = mm - n * g.Hp * g.Wp;
          const uint32_t hh = fdiv(hw, g.dWp), ww = hw - hh * g.Wp;
          a_n[u] = n; a_h[u] = hh * g.st + g.ph + g.pad; a_w[u] = ww * g.st + g.pw + g.pad;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int c = tid + 256 * u;
      if constexpr (MODE == FWD) {            // KC: [BN][BK] rows o
        b_row[u] = c >> 3;
        b_kc[u] = c & 7;
        b_ok[u] = n0 + b_row[u] < g.NC;
      } else {                                // MNC: [BK][BN]
        b_row[u] = c / (BN / 8);
        b_kc[u] = c % (BN / 8);
        const int j = n0 + b_kc[u] * 8;
        b_ok[u] = j < g.NC;
        if constexpr (MODE == WGRAD) {
          const uint32_t jj = b_ok[u] ? j : 0;
          const uint32_t rs = fdiv(jj, g.dC), cc = jj - rs * g.C;
          const uint32_t r = fdiv(rs, g.dS), s = rs - r * g.S;
          b_r[u] = r; b_s[u] = s; b_c[u] = cc;
        }
      }
    }
  }

  // Load the K step starting at k0 into registers (unconditional loads from a
  // clamped address, then select: no per-load branches).
  FEDMI_DEV void load(const ConvGeom& g, const bf16* __restrict__ x, const bf16* __restrict__ w,
                      const bf16* __restrict__ dy, int k0, int m0, int n0, uint4* ra, uint4* rb) const {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      if constexpr (MODE == FWD) {
        const int k = k0 + a_kc[u] * 8;
        const uint32_t rs = fdiv(k, g.dC), cc = k - rs * g.C;
        const uint32_t r = fdiv(rs, g.dS), s = rs - r * g.S;
        const int h = a_h[u] + (int)r, ww = a_w[u] + (int)s;
        const bool ok = a_ok[u] && k < g.K && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
        const long off = ok ? (((long)a_n[u] * g.H + h) * g.W + ww) * g.C + cc : 0;
        const uint4 v = ld16(x + off);
        ra[u] = ok ? v : zero_u4();
      } else if constexpr (MODE == DGRAD) {
        const int k = k0 + a_kc[u] * 8;
        const uint32_t t = fdiv(k, g.dO), o = k - t * g.O;
        const uint32_t i = fdiv(t, g.dNS), j = t - i * g.ns;
        const int r = g.r0 + (int)i * g.st, s = g.s0 + (int)j * g.st;
        int y = a_h[u] - r, xx = a_w[u] - s;   // divisible by st by the phase's tap choice
        bool ok = a_ok[u] && k < g.K && y >= 0 && xx >= 0;
        if (g.st == 2) { y >>= 1; xx >>= 1; }
        ok = ok && y < g.P && xx < g.Q;
        const long off = ok ? (((long)a_n[u] * g.P + y) * g.Q + xx) * g.O + o : 0;
        const uint4 v = ld16(dy + off);
        ra[u] = ok ? v : zero_u4();
      } else {   // WGRAD A: dY[m][o], k-row = pixel
        const int m = k0 + a_row[u];
        const bool ok = a_ok[u] && m < g.K;
        const long off = ok ? (long)m * g.O + m0 + a_kc[u] * 8 : 0;
        const uint4 v = ld16(dy + off);
        ra[u] = ok ? v : zero_u4();
      }
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if constexpr (MODE == FWD) {   // W_rsc[o][k]
        const int k = k0 + b_kc[u] * 8;
        const bool ok = b_ok[u] && k < g.K;
        const long off = ok ? (long)(n0 + b_row[u]) * g.K + k : 0;
        const uint4 v = ld16(w + off);
        rb[u] = ok ? v : zero_u4();
      } else if constexpr (MODE == DGRAD) {   // k-row = (tap, o), cols c: W_rsc[o][r][s][c]
        const int k = k0 + b_row[u];
        const uint32_t kk = k < g.K ? k : 0;
        const uint32_t t = fdiv(kk, g.dO), o = kk - t * g.O;
        const uint32_t i = fdiv(t, g.dNS), j = t - i * g.ns;
        const int rs = (g.r0 + (int)i * g.st) * g.S + g.s0 + (int)j * g.st;
        const bool ok = b_ok[u] && k < g.K;
        const long off = ok ? ((long)o * g.R * g.S + rs) * g.C + n0 + b_kc[u] * 8 : 0;
        const uint4 v = ld16(w + off);
        rb[u] = ok ? v : zero_u4();
      } else {   // WGRAD B: k-row = pixel m=(n,p,q), cols (r,s,c)
        const int m = k0 + b_row[u];
        const uint32_t mm = m < g.K ? m : 0;
        const uint32_t n = fdiv(mm, g.dPQ), pq = mm - n * g.P * g.Q;
        const uint32_t p = fdiv(pq, g.dQ), q = pq - p * g.Q;
        const int h = (int)(p * g.st) - g.pad + b_r[u], ww = (int)(q * g.st) - g.pad + b_s[u];
        const bool ok = b_ok[u] && m < g.K && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
        const long off = ok ? (((long)n * g.H + h) * g.W + ww) * g.C + b_c[u] : 0;
        const uint4 v = ld16(x + off);
        rb[u] = ok ? v : zero_u4();
      }
    }
  }

  FEDMI_DEV void store(bf16* As, bf16* Bs, const uint4* ra, const uint4* rb) const {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      bf16* d = (MODE == WGRAD) ? As + mnc_off<BM>(a_row[u], a_kc[u] * 8) : As + a_row[u] * KC_LD + a_kc[u] * 8;
      *reinterpret_cast<uint4*>(d) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      bf16* d = (MODE == FWD) ? Bs + b_row[u] * KC_LD + b_kc[u] * 8 : Bs + mnc_off<BN>(b_row[u], b_kc[u] * 8);
      *reinterpret_cast<uint4*>(d) = rb[u];
    }
  }
};

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256) void conv_igemm(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                  const bf16* __restrict__ dy, bf16* __restrict__ out,
                                                  float* __restrict__ gout, double* __restrict__ stats,
                                                  const float* __restrict__ shift, ConvGeom g,
                                                  int ksteps_per_split, int partial) {
  // partial bit 0: fp32 split-K partial into gout; bit 1: out += result (bf16 outputs)
  constexpr int A_IMG = (MODE == WGRAD) ? BK * BM : BM * KC_LD;
  constexpr int B_IMG = (MODE == FWD) ? BN * KC_LD : BK * BN;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (A_IMG + B_IMG)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (g.NC + BN - 1) / BN;
  const int tile_n = blockIdx.x % ntn, tile_m = blockIdx.x / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int wm0 = (wave >> 1) * WM, wn0 = (wave & 1) * WN;

  const int ksteps = (g.K + BK - 1) / BK;
  const int kb = blockIdx.z * ksteps_per_split;
  const int ke = min(ksteps, kb + ksteps_per_split);
  if ((MODE == WGRAD || (partial & 1)) && kb >= ke) return;   // (never launched: every split owns >= 1 step)

  Loader<MODE, BM, BN> L;
  L.init(g, m0, n0, tid);
  uint4 ra[Loader<MODE, BM, BN>::NA], rb[Loader<MODE, BM, BN>::NB];

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();

  if (kb < ke) {   // a DGRAD phase with no taps (1x1 stride 2, odd parity) just writes zeros
    L.load(g, x, w, dy, kb * BK, m0, n0, ra, rb);
    L.store(smem, smem + A_IMG, ra, rb);
  }
  __syncthreads();

  for (int t = kb; t < ke; ++t) {
    const int buf = (t - kb) & 1;
    const bf16* As = smem + buf * (A_IMG + B_IMG);
    const bf16* Bs = As + A_IMG;
    const bool more = t + 1 < ke;
    if (more) L.load(g, x, w, dy, (t + 1) * BK, m0, n0, ra, rb);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = (MODE == WGRAD) ? frag_mnc<BM>(As, wm0 + 16 * i, kk, lane) : frag_kc(As, wm0 + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = (MODE == FWD) ? frag_kc(Bs, wn0 + 16 * j, kk, lane) : frag_mnc<BN>(Bs, wn0 + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      bf16* Ad = smem + (buf ^ 1) * (A_IMG + B_IMG);
      L.store(Ad, Ad + A_IMG, ra, rb);
    }
    __syncthreads();
  }

  // ---- epilogue
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  if (MODE == WGRAD || (partial & 1)) {
    // fp32 partial of this K split -> workspace [split][M][NC] (natural GEMM
    // layout, plain stores).  WGRAD: conv_wgrad_reduce sums the splits and
    // permutes into the PyTorch [O][Cw][R][S] gradient; split-K FWD / DGRAD:
    // conv_splitk_reduce sums, rounds to bf16 (+ BN statistics for FWD).
    float* ws = gout + (long)blockIdx.z * g.M * g.NC;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn0 + 16 * j + col_l;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int o = m0 + wm0 + 16 * i + row_l + e;
          if (o < g.M && col < g.NC) ws[(long)o * g.NC + col] = acc[i][j][e];
        }
    }
  } else {
    // Stage the bf16 tile through LDS, then 16-byte row stores; FWD also sums
    // each column (BatchNorm batch statistics) with one atomic per column per WG.
    constexpr int CT_LD = BN + 8;
    bf16* ct = smem;
    float* red = reinterpret_cast<float*>(smem + BM * CT_LD);   // [256/BN parts][2][BN]
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          ct[(wm0 + 16 * i + row_l + e) * CT_LD + wn0 + 16 * j + col_l] = (bf16)acc[i][j][e];
    __syncthreads();
    constexpr int CPR = BN / 8;   // 16-B chunks per tile row
    for (int c = tid; c < BM * CPR; c += 256) {
      const int row = c / CPR, cc = c % CPR;
      const int m = m0 + row, col = n0 + cc * 8;
      long orow = m;
      if (MODE == DGRAD && g.st != 1) {   // phase row -> input pixel row
        const uint32_t n = fdiv(m, g.dHWp), hw = m - n * g.Hp * g.Wp;
        const uint32_t hh = fdiv(hw, g.dWp), ww = hw - hh * g.Wp;
        orow = ((long)n * g.H + hh * g.st + g.ph) * g.W + ww * g.st + g.pw;
      }
      if (m < g.M && col < g.NC) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + row * CT_LD + cc * 8);
        if (partial & 2) {   // accumulate (gradient fan-in of a multi-branch block)
          const bf16x8 o = *reinterpret_cast<const bf16x8*>(out + orow * g.NC + col);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)o[j]);
        }
        *reinterpret_cast<bf16x8*>(out + orow * g.NC + col) = v;
      }
    }
    if (MODE == FWD && stats != nullptr) {
      // sums of (y - shift[c]): shift = the previous step's batch mean of this
      // BN (kept by bn_bwd), so E[d^2] - E[d]^2 does not cancel catastrophically
      constexpr int PARTS = 256 / BN;
      const int col = tid % BN, part = tid / BN;
      const int rows = min(BM, g.M - m0);
      const float sh = (shift != nullptr && n0 + col < g.NC) ? shift[n0 + col] : 0.f;
      float s1 = 0.f, s2 = 0.f;
      for (int r = part; r < rows; r += PARTS) {
        const float v = (float)ct[r * CT_LD + col] - sh;   // statistics of the values the next layer reads
        s1 += v;
        s2 += v * v;
      }
      red[(part * 2) * BN + col] = s1;
      red[(part * 2 + 1) * BN + col] = s2;
      __syncthreads();
      if (tid < 2 * BN) {
        const int q = tid / BN, cl = tid % BN;
        float t = 0.f;
#pragma unroll
        for (int pp = 0; pp < PARTS; ++pp) t += red[(pp * 2 + q) * BN + cl];
        if (n0 + cl < g.NC) unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + q) * g.NC + n0 + cl, (double)t);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Tap-major implicit GEMM with LDS-DMA staging (FWD, and DGRAD through
// flipped/transposed "dgrad weight images"; input channels C % 64 == 0).
//
//   out[m = (n,p,q)][o] = sum_{r,s,c} in[n][p*st - pad_h + r][q*st - pad_w + s][c] * wt[o][r][s][c]
//
// With C % 64 == 0 every BK = 64 K step is ONE tap (r, s) and 64 consecutive
// channels, so a row of the A tile is 128 contiguous bytes of one input pixel
// (or zeros in the halo).  Both operand tiles are therefore K-contiguous
// [rows][64] images filled by global_load_lds_dwordx4 (no VGPR staging, no
// ds_write): each wave-instruction writes 8 rows x 128 B linearly, and the
// per-lane GLOBAL address carries the XOR swizzle (16-B chunk kc of row r is
// stored at chunk kc ^ (r & 7)), which ds_read_b128 fragment reads undo.  Halo
// / tail lanes read a 16-B zero block instead of branching.
//
// Pipeline: three LDS stages, the DMA two K steps ahead, ONE raw s_barrier per
// step behind a counted `s_waitcnt vmcnt` (never vmcnt(0) or __syncthreads()
// while a DMA is in flight).  Tile 128 x BN (BN 128 | 64), 4 waves of 64 x BN/2.
// ---------------------------------------------------------------------------
struct TapGeom {
  int N, H, W, C;          // input [N][H][W][C], C % 64 == 0
  int O;                   // GEMM columns = weight rows [O][R][S][C]
  int P, Q;                // output grid, GEMM rows M = N * P * Q
  int R, S, st, pad_h, pad_w;
  int M, K;                // K = R * S * C
  FastDiv dPQ, dQ;
};

__device__ __attribute__((aligned(16))) const uint4 g_zero16[4] = {};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

FEDMI_DEV void glds16(const void* g, bf16* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_base, 16, 0, 0);
}

// Raw buffer resource over [base, base + bytes): a lane whose byte offset is >= bytes reads zeros (the
// hardware range check), so halo / tail lanes need no select and no zero block.  gfx9 descriptor word 3.
constexpr uint32_t BUF_OOB = 0x80000000u;   // a byte offset every resource here is shorter than
FEDMI_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// 16 bytes per lane from rsrc + voffset into LDS at lds_base + 16 * lane (M0 = lds_base, uniform)
FEDMI_DEV void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voffset, bf16* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_base, 16, (int)voffset, 0, 0, 0);
}

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left at their maxima (gfx9 encoding: vmcnt bits 3:0 + 15:14)
template <int N>
FEDMI_DEV void vmcnt_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// fragment of rows [i0, i0+16), k block kk (0/1) from a swizzled [rows][64] image
FEDMI_DEV bf16x8 frag_sw(const bf16* img, int i0, int kk, int lane) {
  const int row = i0 + (lane & 15);
  const int kc = kk * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((kc ^ (row & 7)) << 3));
}

// Three LDS stages, the DMA two K steps ahead (1 workgroup per CU at BN 128, 2 at BN 64).  Measured
// slower: a two-stage double buffer (one more workgroup per CU), and four stages at BN 128 (128 KiB, the
// DMA three steps ahead: +5..13 % per conv, profiles/r4_cnn/tap_stages_ab.txt).
// NW waves per workgroup (4 or 8) in an (NW / 2) x 2 grid over the 128 x BN tile: with 8 waves every SIMD
// holds two waves, so one wave's barrier / LDS / DMA latency is covered by its partner's MFMAs.
// GEN: input channels C % 8 == 0 but not % 64 (GoogLeNet's 16 / 24 / 32 / 48 / 96 / 112 / 144 / 160-channel inception
// branches, DenseNet's growth): a 64-deep K step then spans several taps, so every DMA lane tracks the (tap, channel)
// of its own 16-byte chunk (k = 64 t + 8 kc, incrementally, no division in the loop) and the last step's chunks
// past K = R * S * C read zeros on both operands.  The weight rows are K-contiguous for any C, so the B side only
// gains the K-tail mask.
template <int BN, int NW, bool GEN = false>
FEDMI_DEV void conv_tap_body(const bf16* __restrict__ in, const bf16* __restrict__ wt, bf16* __restrict__ out,
                             float* __restrict__ part, double* __restrict__ stats, const float* __restrict__ shift,
                             const TapGeom& g, const RowMap& rmap, int ksteps_per_split,
                             const bf16* __restrict__ res, const BnSums& bs, int tile, int split) {
  constexpr int BM = 128;
  constexpr int NT = 64 * NW;            // threads
  constexpr int RW = NW / 2;             // row waves
  constexpr int WMR = BM / RW;           // rows per wave
  constexpr int NA = BM / 8 / NW;        // A wave-instructions per stage per wave (8 rows each)
  constexpr int NB = BN / 8 / NW;
  static_assert(NA >= 1 && NB >= 1, "tile too small for the wave count");
  constexpr int STAGE = (BM + BN) * 64;  // elements
  constexpr int TM = WMR / 16, TN = BN / 32;    // 16x16 fragments per wave: WMR x BN/2
  constexpr int NST = 3;                 // LDS stages: step t being read, t+1 and t+2 in flight
  // the epilogue reuses the stages for the bf16 tile and its partial sums
  constexpr int EPI = BM * (BN + 8) + 2 * 3 * NT * 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[NST * STAGE > EPI ? NST * STAGE : EPI];

  [[maybe_unused]] const int stamp_wg = (int)(blockIdx.x + gridDim.x * blockIdx.z);
  CONV_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  // uniform (SGPR) wave index: the LDS-DMA destinations (M0) are scalar, no readfirstlane per piece
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = (g.O + BN - 1) / BN;
  const int tile_n = tile % ntn, tile_m = tile / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int wm0 = (wave >> 1) * WMR, wn0 = (wave & 1) * (BN / 2);

  const int ksteps = GEN ? (g.K + 63) / 64 : g.K / 64;
  const int kb = split * ksteps_per_split;
  const int ke = min(ksteps, kb + ksteps_per_split);

  // per-lane DMA sources: row (l >> 3) of each 8-row group, logical chunk kc.  Operands are read through
  // buffer resources (the host keeps them < 2 GiB): an A row is valid at tap (r, s) iff bit r * S + s of
  // its tap mask is set (the input pixel (p*st - pad + r, q*st - pad + s) is inside the image); invalid
  // rows / filters get an out-of-range offset and land as zeros.
  const int lrow = lane >> 3;
  const int kc = (lane & 7) ^ lrow;
  const __amdgpu_buffer_rsrc_t rin = buf_rsrc(in, (uint32_t)((long)g.N * g.H * g.W * g.C * 2));
  const __amdgpu_buffer_rsrc_t rwt = buf_rsrc(wt, (uint32_t)((long)g.O * g.K * 2));
  int a_off[NA];              // element offset of the row's pixel at tap (0, 0) (may be negative: halo)
  uint64_t a_mask[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + (wave * NA + i) * 8 + lrow;
    const bool ok = m < g.M;
    const uint32_t mm = ok ? m : 0;
    const uint32_t n = fdiv(mm, g.dPQ), pq = mm - n * g.P * g.Q;
    const uint32_t p = fdiv(pq, g.dQ), q = pq - p * g.Q;
    const int h0 = (int)(p * g.st) - g.pad_h, w0 = (int)(q * g.st) - g.pad_w;
    uint64_t mk = 0;
    for (int r = 0; r < g.R; ++r)
      for (int x = 0; x < g.S; ++x)
        if (ok && (unsigned)(h0 + r) < (unsigned)g.H && (unsigned)(w0 + x) < (unsigned)g.W) mk |= 1ull << (r * g.S + x);
    a_mask[i] = mk;
    a_off[i] = ((n * g.H + h0) * g.W + w0) * g.C + (GEN ? 0 : kc * 8);
  }
  uint32_t b_off[NB];         // byte offset of the filter row's chunk at k = 0 (BUF_OOB: o >= O)
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int o = n0 + (wave * NB + i) * 8 + lrow;
    b_off[i] = o < g.O ? (uint32_t)(o * g.K + kc * 8) * 2u : BUF_OOB;
  }

  // tap state of the next K step to issue, advanced incrementally (scalar; no per-step division):
  // K step t = tap (r, s), channels [c0, c0 + 64)
  int is_c0 = 0, is_s = 0, is_r = 0;
  if constexpr (!GEN) {
    const int k0 = kb * 64;
    const int rs = k0 / g.C;
    is_c0 = k0 - rs * g.C;
    is_r = rs / g.S;
    is_s = rs - is_r * g.S;
  }
  // GEN: this lane's chunk of the next K step to issue: k = 64 t + 8 kc -> tap (gr, gs), channel gc
  int gr = 0, gs = 0, gc = 0;
  uint32_t gk0b = 0;                      // byte offset of the step's first k along a weight row
  if constexpr (GEN) {
    const int k = kb * 64 + kc * 8;
    const int tp = k / g.C;
    gc = k - tp * g.C;
    gr = tp / g.S;
    gs = tp - gr * g.S;
    gk0b = (uint32_t)kb * 128u;
  }
  auto issue = [&](int stage) {
    bf16* As = smem + stage * STAGE;
    bf16* Bs = As + BM * 64;
    if constexpr (GEN) {
      const bool kok = gr < g.R;          // k < K (the last step's tail chunks read zeros on both sides)
      const int rs = kok ? gr * g.S + gs : 0;
      const int tap = (gr * g.W + gs) * g.C + gc;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const bool ok = kok && ((a_mask[i] >> rs) & 1);
        blds16(rin, ok ? (uint32_t)(a_off[i] + tap) * 2u : BUF_OOB, As + (wave * NA + i) * 8 * 64);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i)
        blds16(rwt, (b_off[i] == BUF_OOB || !kok) ? BUF_OOB : b_off[i] + gk0b, Bs + (wave * NB + i) * 8 * 64);
      gk0b += 128u;
      gc += 64;
      while (gc >= g.C) {
        gc -= g.C;
        if (++gs == g.S) { gs = 0; ++gr; }
      }
      return;
    }
    const int rs = is_r * g.S + is_s;
    const int tap = (is_r * g.W + is_s) * g.C + is_c0;
    const uint32_t k0b = (uint32_t)(rs * g.C + is_c0) * 2u;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const bool ok = (a_mask[i] >> rs) & 1;
      blds16(rin, ok ? (uint32_t)(a_off[i] + tap) * 2u : BUF_OOB, As + (wave * NA + i) * 8 * 64);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) blds16(rwt, b_off[i] == BUF_OOB ? BUF_OOB : b_off[i] + k0b, Bs + (wave * NB + i) * 8 * 64);
    is_c0 += 64;
    if (is_c0 == g.C) {
      is_c0 = 0;
      if (++is_s == g.S) { is_s = 0; ++is_r; }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();

  // One barrier per K step: wait for this wave's DMA of step t (leaving the up to AHEAD-1 later
  // steps already issued in flight), barrier (step t visible everywhere AND every wave is done
  // reading step t-1's stage), read every fragment of step t, refill step t-1's stage with step
  // t+AHEAD, MFMAs on step t.  (Measured slower with 8 waves: a software-pipelined loop that reads step
  // t+1's fragments into a second register set during step t's MFMAs, +2..8 % per conv -- the partner wave
  // on the SIMD already covers the LDS latency; profiles/r5_cnn/README.md.)
  constexpr int AHEAD = NST - 1;
#pragma unroll
  for (int a = 0; a < AHEAD; ++a)
    if (kb + a < ke) issue(a);
  CONV_STAMP(1);
  for (int t = kb; t < ke; ++t) {
    const int stg = (t - kb) % NST;
    const int later = min(ke - 1 - t, AHEAD - 1);     // issued steps after t still allowed in flight
    if (later >= 2) vmcnt_wait<2 * (NA + NB)>();
    else if (later == 1) vmcnt_wait<NA + NB>();
    else vmcnt_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#ifdef FEDMI_STAMPS
    if (t == kb) CONV_STAMP(2);
    if (t == kb + (ke - kb) / 2) CONV_STAMP(3);
#endif
    const bf16* As = smem + stg * STAGE;
    const bf16* Bs = As + BM * 64;
    // every fragment of the step (both 32-deep halves) requested at once, THEN the refill DMA and the
    // MFMAs: one LDS latency per step instead of one per half (the compiler otherwise reuses the
    // fragment registers and waits for lgkmcnt(0) before each MFMA group)
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < TM; ++i) af[kk][i] = frag_sw(As, wm0 + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[kk][j] = frag_sw(Bs, wn0 + 16 * j, kk, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t + AHEAD < ke) issue((stg + AHEAD) % NST);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[kk][i], bfr[kk][j], acc[i][j]);
  }
  __syncthreads();   // every wave done with the stages (no DMA in flight) before LDS reuse
  CONV_STAMP(4);

  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  // (Combining the splits in-kernel -- the last-arriving split sums the tile's partials and runs this
  // epilogue, no combine launch -- measured 1.3-2.2x slower at l3 / l4: each last arriver reads 3 x 64 KB of
  // partials serially, profiles/r4_cnn/README.md.)
  if (part != nullptr) {   // split-K partial -> [split][M][O] fp32
    // staged through LDS (free after the K loop) so every global store is a 16-byte row segment instead of
    // a guarded 4-byte scatter per accumulator element
    constexpr int PLD = BN + 4;
    float* pt = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) pt[(wm0 + 16 * i + row_l + e) * PLD + wn0 + 16 * j + col_l] = acc[i][j][e];
    __syncthreads();
    float* ws = part + (long)split * g.M * g.O;
    constexpr int C4 = BN / 4;
#pragma unroll
    for (int k = 0; k < BM * C4 / NT; ++k) {
      const int c = tid + k * NT, row = c / C4, c4 = c % C4;
      const int m = m0 + row, col = n0 + c4 * 4;
      if (m < g.M && col < g.O)
        *reinterpret_cast<float4*>(ws + (long)m * g.O + col) = *reinterpret_cast<const float4*>(pt + row * PLD + c4 * 4);
    }
    CONV_STAMP(5);
    return;
  }
  constexpr int CT_LD = BN + 8;
  bf16* ct = smem;
  float* red = reinterpret_cast<float*>(smem + BM * CT_LD);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ct[(wm0 + 16 * i + row_l + e) * CT_LD + wn0 + 16 * j + col_l] = (bf16)acc[i][j][e];
  if (stats != nullptr && res == nullptr) {
    // BN statistics of bf16(y) - shift straight from the accumulators (rows past M masked), the wave's
    // 4 row groups combined by cross-lane adds, the RW row parts of the tile through LDS
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn0 + 16 * j + col_l;
      const float sh = (shift != nullptr && col < g.O) ? shift[col] : 0.f;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = (m0 + wm0 + 16 * i + row_l + e < g.M) ? (float)(bf16)acc[i][j][e] - sh : 0.f;
          s1 += v;
          s2 += v * v;
        }
      s1 += __shfl_xor(s1, 16);
      s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      if (lane < 16) {
        red[((wave >> 1) * 2) * BN + wn0 + 16 * j + lane] = s1;
        red[((wave >> 1) * 2 + 1) * BN + wn0 + 16 * j + lane] = s2;
      }
    }
  }
  __syncthreads();
  if (stats != nullptr && res == nullptr && tid < 2 * BN) {
    const int q = tid / BN, cl = tid % BN;
    float tsum = 0.f;
#pragma unroll
    for (int rw = 0; rw < RW; ++rw) tsum += red[(rw * 2 + q) * BN + cl];
    if (n0 + cl < g.O) unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + q) * g.O + n0 + cl, (double)tsum);
  }
  constexpr int CPR = BN / 8;
  constexpr int RPT = BM * CPR / NT;      // output rows (8-channel vectors) per thread
  // DGRAD: BN-backward sums of the producer BN (each thread keeps one 8-channel group: NT % CPR == 0)
  const bool bsum = bs.rep != nullptr;
  float bq[3][8], bm[3][8], bi[3][8];
  if (bsum) bnsum_coeffs(bs, n0 + (tid % CPR) * 8, n0 + (tid % CPR) * 8 < g.O, bm, bi, bq);
  // every global operand of the epilogue (residual / second grad, z / y / zb of the BN sums) in flight
  // at once: one memory latency per tile instead of one per row (conditions hoisted out of the loads;
  // invalid rows read row 0)
  long pidx[RPT];
  bool pok[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int c = tid + k * NT, row = c / CPR, cc = c % CPR;
    const int m = m0 + row, col = n0 + cc * 8;
    pok[k] = m < g.M && col < g.O;
    pidx[k] = pok[k] ? map_row(rmap, m) * g.O + col : 0;
  }
  bf16x8 pr[RPT], pz[RPT], py[RPT], pzb[RPT];
  if (res != nullptr) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) pr[k] = *reinterpret_cast<const bf16x8*>(res + pidx[k]);
  }
  if (bsum) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) pz[k] = *reinterpret_cast<const bf16x8*>(bs.z + pidx[k]);
    if (bs.y) {
#pragma unroll
      for (int k = 0; k < RPT; ++k) py[k] = *reinterpret_cast<const bf16x8*>(bs.y + pidx[k]);
    }
    if (bs.zb) {
#pragma unroll
      for (int k = 0; k < RPT; ++k) pzb[k] = *reinterpret_cast<const bf16x8*>(bs.zb + pidx[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int c = tid + k * NT, row = c / CPR, cc = c % CPR;
    if (pok[k]) {
      bf16x8 t = *reinterpret_cast<const bf16x8*>(ct + row * CT_LD + cc * 8);
      if (res != nullptr) {   // fused residual add (pre-activation fwd) / second incoming grad (DGRAD)
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = (bf16)((float)t[j] + (float)pr[k][j]);
        if (stats != nullptr) *reinterpret_cast<bf16x8*>(ct + row * CT_LD + cc * 8) = t;
      }
      *reinterpret_cast<bf16x8*>(out + pidx[k]) = t;
      if (bsum) bnsum_acc_v(bs, t, pz[k], py[k], pzb[k], bm, bi, bq);
    }
  }
  if (bsum) {
    // [3][NT][8] partials behind the ct tile, then one (quantity, channel) per thread -> fp64 replica atomics
    float* rs = red;
    const int nq = bs.zb ? 3 : 2;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) rs[(q * NT + tid) * 8 + j] = bq[q][j];
    __syncthreads();
    for (int e = tid; e < nq * BN; e += NT) {
      const int q = e / BN, cl = e % BN, grp = cl >> 3, j = cl & 7;
      float s = 0.f;
      for (int th = grp; th < NT; th += CPR) s += rs[(q * NT + th) * 8 + j];
      if (n0 + cl < g.O) unsafeAtomicAdd(bs.rep + ((long)(blockIdx.x % bs.reps) * 3 + q) * g.O + n0 + cl, (double)s);
    }
  }
  if (stats != nullptr && res != nullptr) {   // statistics of y = conv + res, from the summed tile
    __syncthreads();
    constexpr int PARTS = NT / BN;
    const int col = tid % BN, prt = tid / BN;
    const int rows = min(BM, g.M - m0);
    const float sh = (shift != nullptr && n0 + col < g.O) ? shift[n0 + col] : 0.f;
    float s1 = 0.f, s2 = 0.f;
    for (int r = prt; r < rows; r += PARTS) {
      const float v = (float)ct[r * CT_LD + col] - sh;
      s1 += v;
      s2 += v * v;
    }
    red[(prt * 2) * BN + col] = s1;
    red[(prt * 2 + 1) * BN + col] = s2;
    __syncthreads();
    if (tid < 2 * BN) {
      const int q = tid / BN, cl = tid % BN;
      float t = 0.f;
#pragma unroll
      for (int pp = 0; pp < PARTS; ++pp) t += red[(pp * 2 + q) * BN + cl];
      if (n0 + cl < g.O) unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + q) * g.O + n0 + cl, (double)t);
    }
  }
  CONV_STAMP(5);
}

template <int BN, int NW, bool GEN = false>
__global__ __launch_bounds__(64 * NW) void conv_tap(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                bf16* __restrict__ out, float* __restrict__ part,
                                                double* __restrict__ stats, const float* __restrict__ shift,
                                                TapGeom g, RowMap rmap, int ksteps_per_split,
                                                const bf16* __restrict__ res, BnSums bs) {
  conv_tap_body<BN, NW, GEN>(in, wt, out, part, stats, shift, g, rmap, ksteps_per_split, res, bs, blockIdx.x,
                             blockIdx.z);
}

// The sub-pixel phases of a stride-2 DGRAD in ONE launch: blockIdx.x walks the phases' tiles in order,
// blockIdx.z is the K split (phases with fewer splits return early, before any barrier).  Each phase
// writes its own parity rows of dX (row maps), or its split-K partials into its own workspace slice.
constexpr int MAX_TAP_PHASES = 4;
struct TapMulti {
  TapGeom g[MAX_TAP_PHASES];
  RowMap rm[MAX_TAP_PHASES];
  long woff[MAX_TAP_PHASES];       // weight-image offset (elements)
  long wsoff[MAX_TAP_PHASES];      // workspace offset (floats), -1: no split (the epilogue writes dX)
  int kps[MAX_TAP_PHASES];         // K steps per split
  int splits[MAX_TAP_PHASES];
  int tile0[MAX_TAP_PHASES + 1];   // first tile of each phase; tile0[n] = total
  int n;
};

template <int BN, int NW>
__global__ __launch_bounds__(64 * NW) void conv_tap_phases(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                       bf16* __restrict__ out, float* __restrict__ ws,
                                                       TapMulti tm, const bf16* __restrict__ res, BnSums bs) {
  int p = 0;
  while (p + 1 < tm.n && (int)blockIdx.x >= tm.tile0[p + 1]) ++p;
  if ((int)blockIdx.z >= tm.splits[p]) return;
  const bool split = tm.wsoff[p] >= 0;
  conv_tap_body<BN, NW>(in, wt + tm.woff[p], out, split ? ws + tm.wsoff[p] : nullptr, nullptr, nullptr, tm.g[p],
                    tm.rm[p], tm.kps[p], split ? nullptr : res, split ? BnSums{} : bs,
                    (int)blockIdx.x - tm.tile0[p], blockIdx.z);
}

// ---------------------------------------------------------------------------
// Halo-patch geometry for 3x3 / stride 1 / pad 1: a 128-pixel tile is IMGS images x TH rows x W
// columns whose input window (TH + 2 rows x W + 2 columns per image, zero halo) is DMA'd into LDS
// once per 64-channel chunk; the nine taps read shifted rows of the same patch (conv_wgrad_halo).
// ---------------------------------------------------------------------------
struct HaloGeom {
  int N, H, W, C, O;
  int M, K;                // M = N * H * W output pixels, K = 9 * C (weight row length)
  int TH, IMGS;            // tile = IMGS images x TH rows x W columns = 128 pixels
  int PW, NPR;             // patch row width W + 2, patch rows IMGS * (TH + 2) * (W + 2)
  int nchunks;             // C / 64
  FastDiv dPI, dPW, dTHW, dW, dHW;   // by (TH + 2) * PW, PW, TH * W, W, H * W
};

// s_waitcnt vmcnt(n) for a run-time n <= N (expcnt / lgkmcnt left at their maxima)
template <int N>
FEDMI_DEV void vm_wait_le(int n) {
  if constexpr (N <= 0) {
    __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
  } else {
    if (n >= N) __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
    else vm_wait_le<N - 1>(n);
  }
}

// ---------------------------------------------------------------------------
// Halo-patch WGRAD for 3x3 / stride 1 / pad 1:
//   dW[o][(r, s, c)] = sum_{pixels m} dY[m][o] * X[m shifted by (r - 1, s - 1)][c]
// One workgroup owns 64 output channels x (9 taps x 64 input channels) = 64 x 576
// fp32 accumulators and walks 128-pixel blocks of its K split.  Per block the
// dY tile [128 px][64 o] and the block's input window [rows][64 c] (the fwd
// halo geometry) are DMA'd once; all nine taps read shifted rows of the same
// window, so each barrier amortises 144 MFMAs per wave (the generic WGRAD: 16)
// and no im2col row is ever re-fetched.  Both LDS images use the MNC swizzle
// (mnc_off<64>), written by the DMA through per-lane source columns, and are
// read with ds_read_b64_tr_b16 at precomputed per-lane offsets (kk, tap).
// Waves split the 64 input channels (16 each); the fp32 partial of a split goes
// to ws[split][o][(r, s, c)] -- the generic WGRAD's layout, so its reduce kernels
// sum the splits and permute into [O][Cw][3][3].
// ---------------------------------------------------------------------------
// KR = 1: the same kernel for a 1x1 / stride-1 conv -- the "patch" is the block's own 128 pixel rows (no halo,
// one tap), dW[o][c] = sum_m dY[m][o] X[m][c]: a plain GEMM over the pixels with both operands pixel-major.
template <int PP, int KR = 3>
__global__ __launch_bounds__(256) void conv_wgrad_halo(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                       float* __restrict__ ws, HaloGeom g, int blocks_per_split) {
  constexpr int TAPS = KR * KR;
  constexpr int PCAP = KR == 1 ? 128 : PP == 1 ? 208 : 288;
  constexpr int NPS = KR == 1 ? 4 : 7 * PP;   // patch wave-instructions per block per wave
  constexpr int DYE = 128 * 64;           // dY stage elements
  constexpr int PTE = PCAP * 64;          // patch stage elements
  constexpr int NST = 3;
  __shared__ __attribute__((aligned(16))) bf16 smem[NST * (DYE + PTE) + 512];
  bf16* const dummy = smem + NST * (DYE + PTE);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nct = g.nchunks;                       // c-chunk tiles
  const int o0 = (blockIdx.x / nct) * 64, c0 = (blockIdx.x % nct) * 64;
  const int nblk = g.M / 128;
  const int b_begin = blockIdx.z * blocks_per_split;
  const int b_end = min(nblk, b_begin + blocks_per_split);
  const int HW = g.H * g.W;
  const int per_img = (g.TH + 2) * g.PW;

  // ---- DMA lanes: row R = base + (lane >> 3), physical 16-B slot sl = lane & 7 holds logical
  // columns ((sl >> 1) ^ f(R)) * 16 + (sl & 1) * 8  (mnc_off<64> inverse)
  const int lr = lane >> 3, sl = lane & 7;
  auto lcol = [&](int R) {
    const int f = ((R >> 1) & 1) | (((R >> 3) & 1) << 1);
    return (((sl >> 1) ^ f) << 4) + ((sl & 1) << 3);
  };
  // dY rows: 128 per block -> 16 instructions, 4 per wave: rows (u * 4 + wave) * 8 + lr
  int dyo[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int R = (u * 4 + wave) * 8 + lr;
    dyo[u] = R * g.O + o0 + lcol(R);             // + block * 128 * O
  }
  // patch rows (q * 4 + wave) * 8 + lr: (image, row, column) of the window packed as i << 16 | hh << 8 | ww
  // (-1 past the window's rows)
  int pk[NPS];
#pragma unroll
  for (int q = 0; q < NPS; ++q) {
    const int pr = (q * 4 + wave) * 8 + lr;
    if constexpr (KR == 1) {
      pk[q] = pr;                                  // the block's pixel row (NPS * 32 == 128)
    } else {
      const int i = fdiv(pr, g.dPI), rem = pr - i * per_img;
      const int hh = fdiv(rem, g.dPW), ww = rem - hh * g.PW;
      pk[q] = pr < g.NPR ? (i << 16) | (hh << 8) | ww : -1;
    }
  }
  auto issue = [&](int b, int stage) {
    bf16* Ds = smem + stage * (DYE + PTE);
    bf16* Ps = Ds + DYE;
    const long mb = (long)b * 128;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds16(dy + mb * g.O + dyo[u], Ds + (u * 4 + wave) * 512);
    const int m0 = b * 128;
    if constexpr (KR == 1) {
#pragma unroll
      for (int q = 0; q < NPS; ++q) {
        const int base = (q * 4 + wave) * 8;
        glds16(x + ((long)m0 + pk[q]) * g.C + c0 + lcol(base + lr), Ps + base * 64);
      }
    } else {
      const int img0 = fdiv(m0, g.dHW), h0 = fdiv(m0 - img0 * HW, g.dW);
#pragma unroll
      for (int q = 0; q < NPS; ++q) {
        const int base = (q * 4 + wave) * 8;
        const int n = img0 + (pk[q] >> 16), h = h0 + ((pk[q] >> 8) & 255) - 1, w = (pk[q] & 255) - 1;
        const bool ok = pk[q] >= 0 && n < g.N && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        const void* src = ok ? (const void*)(x + (((long)n * g.H + h) * g.W + w) * g.C + c0 + lcol(base + lr))
                             : (const void*)g_zero16;
        glds16(src, base < PCAP ? Ps + base * 64 : dummy);
      }
    }
  };

  const int nb = b_end - b_begin;
  if (nb > 0) issue(b_begin, 0);         // the first two blocks load while the offset tables are built
  if (nb > 1) issue(b_begin + 1, 1);

  // ---- fragment offsets (elements, stage-relative).  frag_mnc's lane map: g4 = lane >> 4,
  // q4 = (lane & 15) >> 2, p4 = lane & 3; rows kk * 32 + 8 g4 + q4 and + 4; columns col0 + 4 p4.
  const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  int aoff[4][4][2];        // [kk][o block][row half] in the dY image
  int boff[4][TAPS][2];     // [kk][tap][row half] in the patch image
  const int thw = g.TH * g.W;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int k = kk * 32 + 8 * g4 + q4 + 4 * h2;        // pixel of the block
#pragma unroll
      for (int i = 0; i < 4; ++i) aoff[kk][i][h2] = mnc_off<64>(k, 16 * i + 4 * p4);
      if constexpr (KR == 1) {
        boff[kk][0][h2] = mnc_off<64>(k, wave * 16 + 4 * p4);
      } else {
        const int im = fdiv(k, g.dTHW), rem = k - im * thw;
        const int pp = fdiv(rem, g.dW), qq = rem - pp * g.W;
        const int prow = (im * (g.TH + 2) + pp) * g.PW + qq;  // patch row at tap (0, 0)
#pragma unroll
        for (int t = 0; t < 9; ++t)
          boff[kk][t][h2] = mnc_off<64>(prow + (t / 3) * g.PW + (t % 3), wave * 16 + 4 * p4);
      }
    }
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto tr = [&](const bf16* base, int o0_, int o1_) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + o0_));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + o1_));
    const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo);
    const bf16x4 h4 = __builtin_bit_cast(bf16x4, hi);
    return (bf16x8)__builtin_shufflevector(l4, h4, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[4][TAPS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < TAPS; ++t) acc[i][t] = zero4();

  constexpr int GRP = 4 + NPS;            // DMA instructions per block per wave
  auto step = [&](int it, auto stg) {
    constexpr int S = decltype(stg)::value;
    if (it + 1 < nb) vm_wait_le<GRP>(GRP);
    else vm_wait_le<0>(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 2 < nb) issue(b_begin + it + 2, (S + 2) % NST);
    const bf16* Ds = smem + S * (DYE + PTE);
    const bf16* Ps = Ds + DYE;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr(Ds, aoff[kk][i][0], aoff[kk][i][1]);
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const bf16x8 bfr = tr(Ps, boff[kk][t][0], boff[kk][t][1]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][t] = mfma16(af[i], bfr, acc[i][t]);
      }
    }
  };
  for (int it = 0; it < nb; it += NST) {
    step(it, std::integral_constant<int, 0>{});
    if (it + 1 < nb) step(it + 1, std::integral_constant<int, 1>{});
    if (it + 2 < nb) step(it + 2, std::integral_constant<int, 2>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- partial -> ws[split][o][tap * C + c], staged through LDS (free after the loop) so that every
  // global store is 16 bytes: two passes of 32 output channels; each lane drops its 4 consecutive-o
  // values of a column as one 16-B LDS write into a [576 col][32 o (+1 pad)] tile, then each thread
  // gathers 4 consecutive columns of one o and stores them as a float4.
  constexpr int TLD = 33;
  float* tile = reinterpret_cast<float*>(smem);    // (TAPS * 64) x 33 floats (76 KB at 9 taps)
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  const long NC = (long)TAPS * g.C;
  float* wsp = ws + (long)blockIdx.z * g.O * NC;
  __syncthreads();
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = 2 * half + ii;
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int col = t * 64 + wave * 16 + col_l;     // column within the tile (tap, c)
        float* d = tile + col * TLD + 16 * ii + row_l;
        d[0] = acc[i][t][0]; d[1] = acc[i][t][1]; d[2] = acc[i][t][2]; d[3] = acc[i][t][3];
      }
    }
    __syncthreads();
    // 32 o x (16 * TAPS) column quads
    for (int idx = tid; idx < 32 * 16 * TAPS; idx += 256) {
      const int ol = idx / (16 * TAPS), cq = idx - ol * (16 * TAPS);
      const int col = cq * 4;
      float4 v;
      v.x = tile[(col + 0) * TLD + ol];
      v.y = tile[(col + 1) * TLD + ol];
      v.z = tile[(col + 2) * TLD + ol];
      v.w = tile[(col + 3) * TLD + ol];
      const int t = col >> 6, c = col & 63;
      *reinterpret_cast<float4*>(wsp + (long)(o0 + 32 * half + ol) * NC + t * g.C + c0 + c) = v;
    }
    __syncthreads();
  }
}

// DGRAD weight images for conv_tap: for each sub-pixel phase (stride 1: the
// single phase r0 = s0 = 0, nr = R, ns = S, step 1)
//   wd[c][i][j][o] = W[o][c][r0 + step*(nr-1-i)][s0 + step*(ns-1-j)]   (c < Cw, else 0)
// One workgroup per (64 output channels o, DP_CB input channels c): the fp32 rows
// W[o][c0:c0+DP_CB][:][:] are read contiguously into LDS (one wave walks 16 rows, its
// lanes stride the row: no per-element division), the image rows wd[c][i][j][o0:o0+64]
// written as 128-B runs (lane = o).  Round 1's 4-channel blocks with per-element index
// divisions took 45 us for ResNet-18's layer-3/4 weights.
constexpr int DP_CB = 16;      // input channels per workgroup for R*S <= 9 (4 for larger filters: LDS)
struct DPackEntry {
  const float* w;    // fp32 master [O][Cw][R][S]
  bf16* wd;          // image [Cpad][nr][ns][O]
  int O, Cw, Cpad, R, S, r0, s0, nr, ns, step;
  int blk0;          // first workgroup of this entry
};
constexpr int MAX_DPACK = 16;
struct DPackTable {
  DPackEntry e[MAX_DPACK];
  int n;
  int cb;            // input channels per workgroup (DP_CB or 4)
};

__global__ __launch_bounds__(256) void dgrad_pack_kernel(DPackTable t) {
  extern __shared__ float tile_[];   // [64][cb * R*S + 1], sized by the launch for the largest R*S
  const int CB = t.cb;
  int k = 0;
  while (k + 1 < t.n && (int)blockIdx.x >= t.e[k + 1].blk0) ++k;
  const DPackEntry& p = t.e[k];
  const int b = blockIdx.x - p.blk0;
  const int ncb = (p.Cpad + CB - 1) / CB;
  const int o0 = (b / ncb) * 64, c0 = (b % ncb) * CB;
  const int RS = p.R * p.S;
  const int cw = max(0, min(CB, p.Cw - c0));               // real input channels of this block
  const int span = CB * RS, ld = span + 1, live = cw * RS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // wave w owns rows w, w+4, ..., w+60; 4 rows x 3 row chunks = 12 loads in flight per lane
  for (int k0 = 0; k0 < 16; k0 += 4) {
    for (int f0 = lane; f0 < span; f0 += 64 * 3) {
      float v[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int o = o0 + wave + 4 * (k0 + u);
        const float* src = p.w + ((long)o * p.Cw + c0) * RS;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int f = f0 + 64 * q;
          v[u][q] = (o < p.O && f < live) ? src[f] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (f0 + 64 * q < span) tile_[(wave + 4 * (k0 + u)) * ld + f0 + 64 * q] = v[u][q];
    }
  }
  __syncthreads();
  const int taps = p.nr * p.ns;
  const int o = o0 + lane;
  for (int idx = wave; idx < CB * taps; idx += 4) {      // (ci, tap) per wave: scalar index math
    const int ci = idx / taps, ij = idx - ci * taps;
    const int i = ij / p.ns, j = ij - i * p.ns;
    const int c = c0 + ci;
    if (c >= p.Cpad || o >= p.O) continue;
    const int r = p.r0 + p.step * (p.nr - 1 - i), sx = p.s0 + p.step * (p.ns - 1 - j);
    p.wd[(((long)c * p.nr + i) * p.ns + j) * p.O + o] = (bf16)tile_[lane * ld + ci * RS + r * p.S + sx];
  }
}

// ---------------------------------------------------------------------------
// Network-input ("stem") 3x3 / stride 1 / pad 1 conv on the 8-channel padded image (3 real channels), O = 16 * OT
// output channels (ResNet / VGG / PreAct: 64, MobileNet(V2): 32).  K = 9 taps x 8 channels is tiny, so the
// generic implicit GEMM (128-row tiles, LDS staging, 2 K steps) spent 16-17 us on a memory-bound 0.45 GFLOP
// conv.  Here every MFMA fragment is ONE 16-byte load: with the product transposed (A = filters [o][k],
// B = im2col^T [k][pixel]) a lane's 8 consecutive k are one tap's 8 channels -- of filter o (A, kept in registers
// for the whole kernel) or of one input pixel (B, straight from global memory, zero in the halo).  A wave takes
// 16 output pixels per step: 3 B loads per lane, 3 * OT MFMAs (taps 0-3, 4-7, 8 + zero pad), and the 16x16 output
// tiles land as 4 consecutive channels of one pixel per lane (8-byte stores).  BatchNorm statistics of
// bf16(y) - shift as in the other epilogues: per-lane sums, 16-lane shuffles, a workgroup LDS combine, fp64
// replica atomics.
// ---------------------------------------------------------------------------
struct StemGeom {
  int N, H, W, O, M;   // input [N][H][W][8], output [N][H][W][O], M = N * H * W
};

template <int OT>
__global__ __launch_bounds__(256) void conv_stem_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wr,
                                                        bf16* __restrict__ y, double* __restrict__ stats,
                                                        const float* __restrict__ shift, StemGeom g) {
  constexpr int O = 16 * OT;
  __shared__ float red[4][2][O];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = lane >> 4;        // k block of this lane: taps ks * 4 + kq
  const int col = lane & 15;       // A row (filter) / B column (pixel) of this lane
  bf16x8 a[OT][3];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int tap = ks * 4 + kq;
      a[ot][ks] = tap < 9 ? *reinterpret_cast<const bf16x8*>(wr + ((ot * 16 + col) * 9 + tap) * 8) : zero8();
    }
  float sh[OT][4], s1[OT][4], s2[OT][4];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sh[ot][e] = shift != nullptr ? shift[ot * 16 + kq * 4 + e] : 0.f;
      s1[ot][e] = s2[ot][e] = 0.f;
    }
  const int ntiles = (g.M + 15) >> 4;
  const int nwaves = gridDim.x * 4;
  for (int t = blockIdx.x * 4 + wave; t < ntiles; t += nwaves) {
    const int m = t * 16 + col;
    const bool mok = m < g.M;
    const int mm = mok ? m : 0;
    const int n = mm / (g.H * g.W), pq = mm - n * g.H * g.W;
    const int p = pq / g.W, q = pq - p * g.W;
    bf16x8 b[3];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int tap = ks * 4 + kq;
      const int r = tap / 3, s = tap - (tap / 3) * 3;
      const int h = p + r - 1, w = q + s - 1;
      const bool ok = mok && tap < 9 && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (ok ? ((long)(n * g.H + h) * g.W + w) * 8 : 0));
      b[ks] = ok ? v : zero8();
    }
    f32x4 acc[OT];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      acc[ot] = zero4();
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) acc[ot] = mfma16(a[ot][ks], b[ks], acc[ot]);
    }
    if (mok) {
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = (bf16)acc[ot][e];
          const float v = (float)o[e] - sh[ot][e];
          s1[ot][e] += v;
          s2[ot][e] += v * v;
        }
        *reinterpret_cast<bf16x4*>(y + (long)m * O + ot * 16 + kq * 4) = o;
      }
    }
  }
  if (stats == nullptr) return;
  // the 16 lanes of a k block hold the same 4 channels of 16 different pixels
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) {
        s1[ot][e] += __shfl_xor(s1[ot][e], d);
        s2[ot][e] += __shfl_xor(s2[ot][e], d);
      }
  if (col == 0) {
#pragma unroll
    for (int ot = 0; ot < OT; ++ot)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[wave][0][ot * 16 + kq * 4 + e] = s1[ot][e];
        red[wave][1][ot * 16 + kq * 4 + e] = s2[ot][e];
      }
  }
  __syncthreads();
  if ((int)threadIdx.x < 2 * O) {
    const int qn = threadIdx.x / O, c = threadIdx.x - qn * O;
    const float v = (red[0][qn][c] + red[1][qn][c]) + (red[2][qn][c] + red[3][qn][c]);
    unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + qn) * O + c, (double)v);
  }
}

// ---------------------------------------------------------------------------
// Fused SGD step + weight images (the CNN engines' per-step tail): one launch updates every parameter of the
// flat fp32 master (torch.optim.SGD with momentum / weight decay, fedmi::sgd_elem -- bit-identical to
// sgd_flat_kernel) and, for each dense conv, writes the forward image wr[o][r][s][c] and the DGRAD phase
// images wd[c][i][j][o] from the UPDATED values while they are still in LDS.  The unfused tail read the fp32
// weights three times (sgd_flat, conv_pack_multi, dgrad_pack) in 3-4 launches.
// Workgroup = one conv block of 64 filters x cb input channels (dgrad_pack_kernel's tiling: the image rows
// wd[c][i][j][o0:o0+64] are 128-B runs, the forward rows wr[o][rs][c0:c0+cb] 32-B runs) or SP_SEG elements of
// a flat segment (BatchNorm affine, classifier, depthwise filters: SGD only).  The table lives in device
// memory (built once per engine: all pointers are fixed), sorted by first workgroup.
// ---------------------------------------------------------------------------
constexpr int SP_SEG = 2048;   // flat-segment elements per workgroup (8 per thread)
struct SgdPackEntry {
  long off;                    // element offset into the flat params / grads / momentum
  bf16* wr;                    // kind 0: forward image [O][R][S][C] (nullptr: none)
  bf16* wd[4];                 // kind 0: DGRAD phase images (nph of them)
  int kind;                    // 0: conv weight [O][Cw][R][S]; 1: flat segment of O elements
  int O, Cw, C, R, S, cb, nph, step;
  int blk0;                    // first workgroup of this entry
  int r0[4], s0[4], nr[4], ns[4];
};

template <int RU>
__global__ __launch_bounds__(256) void sgd_pack_kernel(const SgdPackEntry* __restrict__ tab, int n,
                                                       float* __restrict__ P, const float* __restrict__ G,
                                                       float* __restrict__ B, float lr, float mom, float wdecay,
                                                       float damp, int nesterov, int first) {
  extern __shared__ float tile_[];   // [64][cb * R*S + 1] (conv blocks), sized by the launch
  const int bid = blockIdx.x;
  int lo = 0, hi = n - 1;            // last entry with blk0 <= bid (workgroup-uniform)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].blk0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const SgdPackEntry& e = tab[lo];
  const int b = bid - e.blk0;
  const int tid = threadIdx.x;
  if (e.kind == 1) {                 // flat segment: all loads of the chunk in flight, then update + store
    constexpr int U = SP_SEG / 256;
    const long base = e.off + (long)b * SP_SEG;
    const long end = e.off + e.O;
    float pv[U], gv[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + tid + 256 * u;
      const bool ok = i < end;
      pv[u] = ok ? P[i] : 0.f;
      gv[u] = ok ? G[i] : 0.f;
      bv[u] = ok ? B[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + tid + 256 * u;
      if (i < end) {
        fedmi::sgd_elem(pv[u], gv[u], bv[u], lr, mom, wdecay, damp, nesterov, first);
        P[i] = pv[u];
        B[i] = bv[u];
      }
    }
    return;
  }
  const int CB = e.cb, RS = e.R * e.S;
  const int ncb = (e.C + CB - 1) / CB;
  const int o0 = (b / ncb) * 64, c0 = (b % ncb) * CB;
  const int cw = max(0, min(CB, e.Cw - c0));                // real input channels of this block
  const int span = CB * RS, ld = span + 1, live = cw * RS;
  const int lane = tid & 63, wave = tid >> 6;
  // SGD on rows o0..o0+63 (wave w: rows w, w+4, ..): row o's channels [c0, c0+cw) are cw*RS contiguous floats
  // at a wave-uniform base; updated values -> LDS, channels past Cw as zeros.  8 rows x 3 row chunks x 3 operands
  // in flight per lane (RU = 4 rows per pass: 2 measured the same, 8 18-28 % slower -- its VGPRs cost occupancy;
  // profiles/r5_cnn/sgdpack/).
  for (int k0 = 0; k0 < 16; k0 += RU) {
    for (int f0 = lane; f0 < span; f0 += 64 * 3) {
      float pv[RU][3], gv[RU][3], bv[RU][3];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int o = o0 + wave + 4 * (k0 + u);
        const long rb = e.off + ((long)o * e.Cw + c0) * RS;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int f = f0 + 64 * q;
          const bool ok = o < e.O && f < live;
          pv[u][q] = ok ? P[rb + f] : 0.f;
          gv[u][q] = ok ? G[rb + f] : 0.f;
          bv[u][q] = ok ? B[rb + f] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int o = o0 + wave + 4 * (k0 + u);
        const long rb = e.off + ((long)o * e.Cw + c0) * RS;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int f = f0 + 64 * q;
          if (o < e.O && f < live) {
            fedmi::sgd_elem(pv[u][q], gv[u][q], bv[u][q], lr, mom, wdecay, damp, nesterov, first);
            P[rb + f] = pv[u][q];
            B[rb + f] = bv[u][q];
          }
          if (f < span) tile_[(wave + 4 * (k0 + u)) * ld + f] = pv[u][q];
        }
      }
    }
  }
  __syncthreads();
  // DGRAD phase images (dgrad_pack_kernel's write loop per phase)
  const int o = o0 + lane;
  for (int ph = 0; ph < e.nph; ++ph) {
    const int nr = e.nr[ph], ns = e.ns[ph], r0 = e.r0[ph], s0 = e.s0[ph], taps = nr * ns;
    bf16* wd = e.wd[ph];
    for (int idx = wave; idx < CB * taps; idx += 4) {
      const int ci = idx / taps, ij = idx - ci * taps;
      const int i = ij / ns, j = ij - i * ns;
      const int c = c0 + ci;
      if (c >= e.C || o >= e.O) continue;
      const int r = r0 + e.step * (nr - 1 - i), sx = s0 + e.step * (ns - 1 - j);
      wd[(((long)c * nr + i) * ns + j) * e.O + o] = (bf16)tile_[lane * ld + ci * RS + r * e.S + sx];
    }
  }
  // forward image rows wr[o][rs][c0 : c0 + cwr) (cwr: 8 / 16 at cb 16 since C % 8 == 0; 4 at cb 4)
  if (e.wr != nullptr) {
    const int cwr = min(CB, e.C - c0);
    for (int q = tid; q < 64 * RS; q += 256) {
      const int ol = q / RS, rs = q - ol * RS;
      if (o0 + ol >= e.O) continue;
      bf16* dst = e.wr + ((long)(o0 + ol) * RS + rs) * e.C + c0;
      const float* src = tile_ + ol * ld + rs;
      if (cwr == 4) {
        bf16x4 t;
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = (bf16)src[k * RS];
        *reinterpret_cast<bf16x4*>(dst) = t;
      } else {
        for (int v0 = 0; v0 < cwr; v0 += 8) {
          bf16x8 t;
#pragma unroll
          for (int k = 0; k < 8; ++k) t[k] = (bf16)src[(v0 + k) * RS];
          *reinterpret_cast<bf16x8*>(dst + v0) = t;
        }
      }
    }
  }
}

// Split-K WGRAD reductions (bodies in wgrad_reduce.h, shared with the deferred wgrad_reduce_multi below).
constexpr int WRED_MAX_RS = 49;
__global__ __launch_bounds__(256) void conv_wgrad_reduce(const float* __restrict__ ws, int splits, int O, int C, int Cw,
                                                         int RS, float* __restrict__ dw, int accumulate, int Ow, int G) {
  extern __shared__ float part_[];                 // [4][RS][65], sized by the launch
  fedmi::wred_tile_body(part_, blockIdx.x, ws, splits, O, C, Cw, RS, dw, accumulate, Ow, G);
}

__global__ __launch_bounds__(256) void conv_wgrad_reduce_cols(const float* __restrict__ ws, int splits, int O, int C, int Cw,
                                                         int RS, float* __restrict__ dw, int accumulate, int Ow, int G) {
  __shared__ float part[4 * 64];
  fedmi::wred_cols_body(part, blockIdx.x, ws, splits, O, C, Cw, RS, dw, accumulate, Ow, G);
}

// Deferred WGRAD reductions: every split-K / depthwise partial reduction of a backward pass in one launch
// (the engines run them all after the last WGRAD, before the SGD step).  Workgroup bid belongs to the last item
// with blk0 <= bid; each item runs its standalone kernel's body, so the result is bit-identical.
constexpr int WRED_MULTI_MAX = 32;
struct WredTable {
  fedmi::WredItem it[WRED_MULTI_MAX];
  int blk0[WRED_MULTI_MAX];
  int n;
};
__global__ __launch_bounds__(256) void wgrad_reduce_multi(const WredTable t) {
  extern __shared__ float lds_[];
  const int bid = blockIdx.x;
  int k = 0;
  while (k + 1 < t.n && t.blk0[k + 1] <= bid) ++k;   // workgroup-uniform
  const fedmi::WredItem& e = t.it[k];
  const int b = bid - t.blk0[k];
  if (e.kind == fedmi::WRED_TILE)
    fedmi::wred_tile_body(lds_, b, e.ws, e.splits, e.O, e.C, e.Cw, e.RS, e.dw, e.accumulate, e.Ow, e.G);
  else if (e.kind == fedmi::WRED_COLS)
    fedmi::wred_cols_body(lds_, b, e.ws, e.splits, e.O, e.C, e.Cw, e.RS, e.dw, e.accumulate, e.Ow, e.G);
  else
    fedmi::wred_dw_body(lds_, b, e.ws, e.splits, e.C, e.dw, e.accumulate);
}

// Split-K FWD / DGRAD combine: out[row][c] = bf16(sum_z ws[z][m][c]); FWD also
// accumulates the BatchNorm batch statistics (sum / sum of squares of
// bf16(y) - shift[c]) like the single-pass epilogue.  Each thread owns one
// 8-channel group (two 16-B loads per split) of rows r0, r0 + rstep, ...
// rows per thread per pass x splits' loads in flight per step (2: ResNet-18 814-816 vs 816-822 ms per round,
// GoogLeNet 3322 vs 3325-3338, MobileNet 643 vs 645-648; same VGPR count -- profiles/r6_cnn/splitk_z2/)
#ifndef SPLITK_U
#define SPLITK_U 4
#endif
#ifndef SPLITK_Z
#define SPLITK_Z 2
#endif
__global__ __launch_bounds__(256) void conv_splitk_reduce(const float* __restrict__ ws, int splits, int M, int NC,
                                                          RowMap rmap, bf16* __restrict__ out,
                                                          double* __restrict__ stats, const float* __restrict__ shift,
                                                          int rows_per_block, const bf16* __restrict__ res,
                                                          BnSums bs) {
  __shared__ float red[3][256][8];
  const int VR = NC >> 3;                 // host: blockDim.x % VR == 0
  const int cg = threadIdx.x % VR, rstep = blockDim.x / VR, r0 = threadIdx.x / VR;
  const int c0 = cg * 8;
  const long plane = (long)M * NC;
  const bool bsum = bs.rep != nullptr;    // DGRAD: BN-backward sums of the producer BN (conv_tap's epilogue)
  float sh[8], bq[3][8], bm[3][8], bi[3][8];
  bnsum_coeffs(bs, c0, bsum, bm, bi, bq);
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[j] = (stats && shift) ? shift[c0 + j] : 0.f;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  // U rows per thread per pass, every load of the pass issued before the first use (the partials of all
  // splits, the residual / second grad, the BN-sums operands): one memory latency per U rows
  constexpr int U = SPLITK_U;
  for (int m0 = rb + r0; m0 < re; m0 += U * rstep) {
    float v[U][8];
    bf16x8 rr[U], pz[U], py[U], pzb[U];
    long orow[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * rstep;
      ok[u] = m < re;
      const int mm = ok[u] ? m : rb + r0;
      orow[u] = map_row(rmap, mm);
      const float* p = ws + (long)mm * NC + c0;
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[u][0] = a.x; v[u][1] = a.y; v[u][2] = a.z; v[u][3] = a.w;
      v[u][4] = b.x; v[u][5] = b.y; v[u][6] = b.z; v[u][7] = b.w;
    }
    // SPLITK_Z splits' loads in flight per step (the adds stay in split order: bit-identical for any SPLITK_Z)
    for (int z = 1; z < splits; z += SPLITK_Z) {
      float4 ua[SPLITK_Z][U], ub[SPLITK_Z][U];
#pragma unroll
      for (int q = 0; q < SPLITK_Z; ++q)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int mm = ok[u] ? m0 + u * rstep : rb + r0;
          const float* p = ws + (long)mm * NC + c0 + (long)min(z + q, splits - 1) * plane;
          ua[q][u] = *reinterpret_cast<const float4*>(p);
          ub[q][u] = *reinterpret_cast<const float4*>(p + 4);
        }
#pragma unroll
      for (int q = 0; q < SPLITK_Z; ++q) {
        if (z + q >= splits) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          v[u][0] += ua[q][u].x; v[u][1] += ua[q][u].y; v[u][2] += ua[q][u].z; v[u][3] += ua[q][u].w;
          v[u][4] += ub[q][u].x; v[u][5] += ub[q][u].y; v[u][6] += ub[q][u].z; v[u][7] += ub[q][u].w;
        }
      }
    }
    if (res != nullptr) {
#pragma unroll
      for (int u = 0; u < U; ++u) rr[u] = *reinterpret_cast<const bf16x8*>(res + orow[u] * NC + c0);
    }
    if (bsum) {
#pragma unroll
      for (int u = 0; u < U; ++u) pz[u] = *reinterpret_cast<const bf16x8*>(bs.z + orow[u] * NC + c0);
      if (bs.y) {
#pragma unroll
        for (int u = 0; u < U; ++u) py[u] = *reinterpret_cast<const bf16x8*>(bs.y + orow[u] * NC + c0);
      }
      if (bs.zb) {
#pragma unroll
        for (int u = 0; u < U; ++u) pzb[u] = *reinterpret_cast<const bf16x8*>(bs.zb + orow[u] * NC + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      if (res != nullptr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] += (float)rr[u][j];
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)v[u][j];
      *reinterpret_cast<bf16x8*>(out + orow[u] * NC + c0) = o;
      if (stats) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)o[j] - sh[j];
          bq[0][j] += d;
          bq[1][j] += d * d;
        }
      } else if (bsum) {
        bnsum_acc_v(bs, o, pz[u], py[u], pzb[u], bm, bi, bq);
      }
    }
  }
  if (!stats && !bsum) return;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[q][threadIdx.x][j] = bq[q][j];
  __syncthreads();
  const int nq = (bsum && bs.zb) ? 3 : 2;
  for (int e = threadIdx.x; e < nq * NC; e += blockDim.x) {
    const int q = e / NC, c = e - q * NC;
    const int grp = c >> 3, j = c & 7;
    float t = 0.f;
    for (int th = grp; th < (int)blockDim.x; th += VR) t += red[q][th][j];
    if (stats) unsafeAtomicAdd(stats + ((blockIdx.x % STAT_REP) * 2 + q) * NC + c, (double)t);
    else unsafeAtomicAdd(bs.rep + ((long)(blockIdx.x % bs.reps) * 3 + q) * NC + c, (double)t);
  }
}

// Multi-tensor weight pack: every dense conv of a network in one launch.
// One workgroup per output-channel row: the fp32 [Cw][R*S] row is read
// coalesced into LDS, then written as the bf16 [R*S][C] row (zero channel pad),
// also coalesced (a direct element map reads with an R*S stride).
struct PackEntry {
  const float* w;
  bf16* wr;
  int O, Cw, C, RS;
  int O8;            // image rows: O..O8 are zero filters (the output-channel pad of odd widths)
  int G;             // groups > 1: block-diagonal image of a grouped conv (filter o reads channels of its group)
  int row0;          // first workgroup (row) of this entry in the launch
};
constexpr int MAX_PACK = 64;   // 64 x 40 B of kernel arguments
constexpr int PACK_ROW_MAX = 8192;   // Cw * R * S floats staged per row (32 KiB)
struct PackTable {
  PackEntry e[MAX_PACK];
  int n;
};

__global__ __launch_bounds__(256) void conv_pack_multi_kernel(PackTable t) {
  extern __shared__ float row[];   // sized by the launch: the table's longest Cw * R * S
  int k = 0;
  while (k + 1 < t.n && (int)blockIdx.x >= t.e[k + 1].row0) ++k;
  const PackEntry& p = t.e[k];
  const int o = blockIdx.x - p.row0;
  if (o >= p.O) {   // zero filter row (workgroup-uniform)
    bf16* dst = p.wr + (long)o * p.RS * p.C;
    for (int i = threadIdx.x; i < p.RS * p.C; i += 256) dst[i] = (bf16)0.f;
    return;
  }
  const int n_in = p.Cw * p.RS;
  const float* src = p.w + (long)o * n_in;
  for (int i0 = threadIdx.x; i0 < n_in; i0 += 256 * 8) {   // 8 loads in flight per thread
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = i0 + 256 * u < n_in ? src[i0 + 256 * u] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + 256 * u < n_in) row[i0 + 256 * u] = v[u];
  }
  __syncthreads();
  bf16* dst = p.wr + (long)o * p.RS * p.C;
  const int n_out = p.RS * p.C;
  const int cg0 = p.G > 1 ? (o / (p.O / p.G)) * p.Cw : 0;   // first input channel of filter o's group
  for (int i = threadIdx.x; i < n_out; i += 256) {
    const int rs = i / p.C, c = i - rs * p.C - cg0;
    dst[i] = c >= 0 && c < p.Cw ? (bf16)row[c * p.RS + rs] : (bf16)0.f;
  }
}

FastDiv make_div(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  return f;
}

}  // namespace

namespace fedmi {

struct ConvShape {
  int N, H, W, C, Cw, O, P, Q, R, S, st, pad;
};

static RowMap make_rowmap(int P, int Q, int OH, int OW, int st, int ph, int pw) {
  RowMap r{};
  r.on = 1;
  r.P = P; r.Q = Q; r.OH = OH; r.OW = OW; r.st = st; r.ph = ph; r.pw = pw;
  r.dPQ = make_div(P * Q); r.dQ = make_div(Q);
  return r;
}

static ConvGeom make_geom(const ConvShape& s) {
  ConvGeom g{};
  g.N = s.N; g.H = s.H; g.W = s.W; g.C = s.C; g.O = s.O; g.P = s.P; g.Q = s.Q;
  g.R = s.R; g.S = s.S; g.st = s.st; g.pad = s.pad; g.Cw = s.Cw;
  g.dC = make_div(s.C); g.dO = make_div(s.O); g.dS = make_div(s.S); g.dQ = make_div(s.Q);
  g.dPQ = make_div(s.P * s.Q); g.dW = make_div(s.W); g.dHW = make_div(s.H * s.W);
  g.ph = g.pw = 0; g.r0 = g.s0 = 0; g.nr = s.R; g.ns = s.S; g.Hp = s.H; g.Wp = s.W;
  g.dNS = make_div(s.S); g.dWp = make_div(s.W); g.dHWp = make_div(s.H * s.W);
  return g;
}

static void check_shape(const ConvShape& s) {
  if (s.C % 8 || s.O % 8 || s.C < s.Cw || s.st < 1 || s.st > 2 || s.R < 1 || s.S < 1)
    throw std::invalid_argument("conv_igemm: need C % 8 == 0, O % 8 == 0, stride 1|2");
  if (s.P != (s.H + 2 * s.pad - s.R) / s.st + 1 || s.Q != (s.W + 2 * s.pad - s.S) / s.st + 1)
    throw std::invalid_argument("conv_igemm: inconsistent output size");
  if ((long)s.N * s.H * s.W * s.C >= (1l << 31) || (long)s.N * s.P * s.Q * s.O >= (1l << 31))
    throw std::invalid_argument("conv_igemm: tensor too large for 32-bit index math");
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

struct TileCfg {
  int BM, BN;
};

static TileCfg pick_tiles(int M, int NC) {
  const int cus = num_cus();
  const int BN = NC <= 64 ? 64 : 128;
  const long t128 = (long)((M + 127) / 128) * ((NC + BN - 1) / BN);
  return TileCfg{(M > 64 && t128 >= cus) ? 128 : 64, BN};
}

// WGRAD always splits K, so the tile count never has to fill the chip: take the 128 x 128 tile
// (twice the MFMA work per loaded byte) for O >= 256 -- measured 44 -> 38 us (256x256 3x3) and
// 51 -> 47 us (512x512) at batch 128, but slower at O = 128.
static TileCfg pick_tiles_wgrad(int M, int NC) {
  TileCfg t = pick_tiles(M, NC);
  if (M >= 256 && NC > 64) t.BM = 128;
  return t;
}

template <int MODE, int BM, int BN>
static void launch_tiled(hipStream_t st, dim3 grid, const ConvGeom& g, const bf16* x, const bf16* w, const bf16* dy,
                         bf16* out, float* gout, double* stats, const float* shift, int kps, int partial) {
  hipLaunchKernelGGL((conv_igemm<MODE, BM, BN>), grid, dim3(256), 0, st, x, w, dy, out, gout, stats, shift, g, kps,
                     partial);
}

// FWD / DGRAD split-K: GEMMs with fewer output tiles than CUs and a long K loop
// (ResNet layer3/4 at batch 128: 128-256 tiles, 36-72 K steps) leave most of
// the chip idle behind a serial K chain.  Split K so that ~3 workgroups per CU
// run >= 8 K steps each, partials into ``ws``; 1 = no split.
// The split-K combine (conv_splitk_reduce) gives each lane one 8-channel vector of a row and needs a
// whole row in one 256-lane block: rows wider than 2048 channels never split.
static constexpr int SPLITK_MAX_NC = 2048;

static int fd_splits(const ConvGeom& g, long ws_floats) {
  if (ws_floats <= 0 || g.NC > SPLITK_MAX_NC) return 1;
  const TileCfg t = pick_tiles(g.M, g.NC);
  const long tiles = (long)((g.M + t.BM - 1) / t.BM) * ((g.NC + t.BN - 1) / t.BN);
  const int ksteps = (g.K + BK - 1) / BK;
  if (tiles >= 2l * num_cus() || ksteps < 16) return 1;
  long sp = std::min<long>((3l * num_cus() + tiles - 1) / tiles, ksteps / 8);
  sp = std::min<long>(sp, ws_floats / ((long)g.M * g.NC));
  if (sp < 2) return 1;
  const int kps = (int)((ksteps + sp - 1) / sp);
  return (ksteps + kps - 1) / kps;
}

template <int MODE>
static void launch_mode(hipStream_t st, const ConvGeom& g, const bf16* x, const bf16* w, const bf16* dy, bf16* out,
                        float* gout, double* stats, int splits, const float* shift = nullptr, int partial = 0) {
  const TileCfg t = MODE == WGRAD ? pick_tiles_wgrad(g.M, g.NC) : pick_tiles(g.M, g.NC);
  const long tiles = (long)((g.M + t.BM - 1) / t.BM) * ((g.NC + t.BN - 1) / t.BN);
  const int ksteps = (g.K + BK - 1) / BK;
  if (MODE != WGRAD && !(partial & 1)) splits = 1;
  splits = std::max(1, std::min(splits, ksteps));
  const int kps = std::max(1, (ksteps + splits - 1) / splits);
  splits = std::max(1, (ksteps + kps - 1) / kps);
  dim3 grid((unsigned)tiles, 1, (unsigned)splits);
  if (t.BM == 128 && t.BN == 128) launch_tiled<MODE, 128, 128>(st, grid, g, x, w, dy, out, gout, stats, shift, kps, partial);
  else if (t.BM == 128) launch_tiled<MODE, 128, 64>(st, grid, g, x, w, dy, out, gout, stats, shift, kps, partial);
  else if (t.BN == 128) launch_tiled<MODE, 64, 128>(st, grid, g, x, w, dy, out, gout, stats, shift, kps, partial);
  else launch_tiled<MODE, 64, 64>(st, grid, g, x, w, dy, out, gout, stats, shift, kps, partial);
}

// ---- tap-major LDS-DMA path (conv_tap)
static TapGeom make_tap(int N, int H, int W, int C, int O, int P, int Q, int R, int S, int st, int pad_h, int pad_w) {
  TapGeom g{};
  g.N = N; g.H = H; g.W = W; g.C = C; g.O = O; g.P = P; g.Q = Q;
  g.R = R; g.S = S; g.st = st; g.pad_h = pad_h; g.pad_w = pad_w;
  g.M = N * P * Q; g.K = R * S * C;
  g.dPQ = make_div(P * Q); g.dQ = make_div(Q);
  return g;
}

// conv_tap tile width: 128 columns (96 KiB of LDS stages, 1 workgroup per CU) while the 128-wide tiles fill the
// chip; 64 (72 KiB, 2 per CU) for O <= 64 and for problems whose 128-wide tiles would leave CUs idle (ResNet-18 l3 /
// l4: 128 / 64 tiles -> 256 / 128; -19 % / -8 % per conv, while l2's 256 tiles stay faster at 128: +7 % at 64,
// profiles/r5_cnn/).  FEDMI_TAP_BN=64|128 forces one width (A/B runs).  m_tiles: 128-row tiles of the problem.
static int tap_bn_for(int O, long m_tiles) {
  static const int force = [] {
    const char* e = std::getenv("FEDMI_TAP_BN");
    return e ? std::atoi(e) : 0;
  }();
  if (O <= 64) return 64;
  if (force == 64 || force == 128) return force;
  return m_tiles * ((O + 127) / 128) < num_cus() ? 64 : 128;
}
static int tap_bn(const TapGeom& g) { return tap_bn_for(g.O, (g.M + 127) / 128); }

// waves per conv_tap workgroup: 8 (two per SIMD, default: 8-15 % faster per conv, profiles/r5_cnn/) or 4 (one
// per SIMD); FEDMI_TAP_WAVES overrides (A/B runs)
static int tap_waves() {
  static int w = [] {
    const char* e = std::getenv("FEDMI_TAP_WAVES");
    const int v = e ? std::atoi(e) : 8;
    return v == 8 ? 8 : 4;
  }();
  return w;
}

// conv_tap reads its operands through 32-bit buffer offsets (out-of-range lanes read zeros) and keeps a
// per-row tap-validity mask of R * S <= 64 bits
static bool tap_fits(long in_elems, long w_elems, int R, int S) {
  return in_elems * 2 < (1l << 31) && w_elems * 2 < (1l << 31) && R * S <= 64;
}

// Split K only to fill one wave of workgroups: conv_tap keeps 1 (BN 128, 96 KiB
// LDS) or 2 (BN 64) workgroups per CU, and a split costs an fp32 round trip.
// With 8-wave workgroups a half-filled chip without split-K beats split-K + combine (ResNet-18 l3 forward:
// 24.7 vs 28.8 us, profiles/r5_cnn/): split only when the tiles fill at most a quarter of one wave of
// workgroups.  FEDMI_TAP_SPLITS=n forces n splits where a split applies (A/B runs).
static int tap_split_override() {
  static int v = [] {
    const char* e = std::getenv("FEDMI_TAP_SPLITS");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

static int tap_splits(const TapGeom& g, long ws_floats) {
  if (ws_floats <= 0 || g.O > SPLITK_MAX_NC) return 1;
  const int bn = tap_bn(g);
  const long tiles = (long)((g.M + 127) / 128) * ((g.O + bn - 1) / bn);
  const long target = (bn == 128 ? 1l : 2l) * num_cus();
  const int ksteps = (g.K + 63) / 64;
  // (a 40-step threshold saved 2.4 us on ResNet-18's layer-4 stride-2 forward but moved EfficientNetB0's
  // 3-epoch trajectory outside its parity bound -- profiles/r5_cnn/splits/; kept at 16)
  if (4 * tiles > target || ksteps < 16) return 1;
  long sp = std::min<long>((target + tiles / 2) / tiles, ksteps / 8);
  if (tap_split_override() > 0) sp = std::min<long>(tap_split_override(), ksteps / 8);
  sp = std::min<long>(sp, ws_floats / ((long)g.M * g.O));
  if (sp < 2) return 1;
  const int kps = (int)((ksteps + sp - 1) / sp);
  return (ksteps + kps - 1) / kps;
}

// halo geometry of a 3x3 / stride-1 / pad-1 problem (conv_wgrad_halo), or false
static bool halo_geom(const TapGeom& g, const RowMap& rm, HaloGeom* h) {
  if (rm.on || g.R != 3 || g.S != 3 || g.st != 1 || g.pad_h != 1 || g.pad_w != 1 || g.P != g.H ||
      g.Q != g.W || g.C % 64 || g.O % 8 || g.M % 128)
    return false;
  const int HW = g.H * g.W;
  HaloGeom x{};
  x.N = g.N; x.H = g.H; x.W = g.W; x.C = g.C; x.O = g.O; x.M = g.M; x.K = 9 * g.C;
  if (HW <= 128) {
    if (128 % HW) return false;
    x.IMGS = 128 / HW; x.TH = g.H;
  } else {
    if (128 % g.W || g.H % (128 / g.W)) return false;
    x.IMGS = 1; x.TH = 128 / g.W;
  }
  x.PW = g.W + 2;
  x.NPR = x.IMGS * (x.TH + 2) * x.PW;
  x.nchunks = g.C / 64;
  if (x.NPR > 288) return false;
  x.dPI = make_div((x.TH + 2) * x.PW); x.dPW = make_div(x.PW); x.dTHW = make_div(x.TH * g.W);
  x.dW = make_div(g.W); x.dHW = make_div(HW);
  *h = x;
  return true;
}

static void launch_tap_reduce(hipStream_t st, const TapGeom& g, const RowMap& rm, const float* ws, int splits,
                              bf16* out, double* stats, const float* shift, const bf16* res, const BnSums& bs) {
  const int VR = g.O / 8;
  const int tb = (256 / VR) * VR;
  const int rstep = tb / VR;
  // with BN statistics / BN-backward sums fewer blocks (their per-channel atomics contend on 2 x O addresses)
  const int rows_per_block = (stats || bs.rep) ? std::max(2 * rstep, (g.M + 255) / 256)
                                               : std::max(rstep, (g.M + 1023) / 1024);
  const int nblk = (g.M + rows_per_block - 1) / rows_per_block;
  hipLaunchKernelGGL(conv_splitk_reduce, dim3(nblk), dim3(tb), 0, st, ws, splits, g.M, g.O, rm, out, stats, shift,
                     rows_per_block, res, bs);
}

static void launch_tap(hipStream_t st, const TapGeom& g, const bf16* in, const bf16* wt, bf16* out, double* stats,
                       const float* shift, const RowMap& rm, float* ws, long ws_floats,
                       const bf16* res = nullptr, const BnSums& bs = BnSums{}) {
  if (g.C % 8 || g.C < 16 || g.O % 8) throw std::invalid_argument("conv_tap: need C % 8 == 0, C >= 16, O % 8 == 0");
  if (!tap_fits((long)g.N * g.H * g.W * g.C, (long)g.O * g.K, g.R, g.S))
    throw std::invalid_argument("conv_tap: operands over 2 GiB or R * S > 64");
  const bool gen = g.C % 64 != 0;         // several taps per K step (conv_tap_body GEN)
  const int BN = tap_bn(g);
  const long tiles = (long)((g.M + 127) / 128) * ((g.O + BN - 1) / BN);
  const int ksteps = (g.K + 63) / 64;
  const int sp = tap_splits(g, ws_floats);
  const int kps = (ksteps + sp - 1) / sp;
  const int splits = (ksteps + kps - 1) / kps;
  dim3 grid((unsigned)tiles, 1, (unsigned)splits);
  float* part = splits > 1 ? ws : nullptr;
  const BnSums tbs = part ? BnSums{} : bs;
  double* tst = part ? nullptr : stats;
  const bf16* trs = part ? nullptr : res;
  if (gen) {   // 8 waves only (the default shape)
    if (BN == 128)
      hipLaunchKernelGGL((conv_tap<128, 8, true>), grid, dim3(512), 0, st, in, wt, out, part, tst, shift, g, rm, kps, trs,
                         tbs);
    else
      hipLaunchKernelGGL((conv_tap<64, 8, true>), grid, dim3(512), 0, st, in, wt, out, part, tst, shift, g, rm, kps, trs,
                         tbs);
  } else if (BN == 128)
    if (tap_waves() == 8)
      hipLaunchKernelGGL((conv_tap<128, 8>), grid, dim3(512), 0, st, in, wt, out, part, tst, shift, g, rm, kps, trs, tbs);
    else
      hipLaunchKernelGGL((conv_tap<128, 4>), grid, dim3(256), 0, st, in, wt, out, part, tst, shift, g, rm, kps, trs, tbs);
  else if (tap_waves() == 8)
    hipLaunchKernelGGL((conv_tap<64, 8>), grid, dim3(512), 0, st, in, wt, out, part, tst, shift, g, rm, kps, trs, tbs);
  else
    hipLaunchKernelGGL((conv_tap<64, 4>), grid, dim3(256), 0, st, in, wt, out, part, tst, shift, g, rm, kps, trs, tbs);
  if (splits > 1) launch_tap_reduce(st, g, rm, ws, splits, out, stats, shift, res, bs);
}

// DGRAD phases as conv_tap problems over dY: (geometry, row map, image offset) per phase.
struct TapPhase {
  TapGeom g;
  RowMap rm;
  long img_off;
  int r0, s0, nr, ns;
  bool empty;   // no taps land on this parity (1x1 stride 2): output rows must be zero
  int ph, pw;
};

static int dgrad_tap_phases(const ConvShape& s, TapPhase* out) {
  int n = 0;
  if (s.st == 1) {
    TapPhase& t = out[n++];
    t = TapPhase{};
    t.g = make_tap(s.N, s.P, s.Q, s.O, s.C, s.H, s.W, s.R, s.S, 1, s.R - 1 - s.pad, s.S - 1 - s.pad);
    t.r0 = t.s0 = 0; t.nr = s.R; t.ns = s.S;
    return n;
  }
  long off = 0;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      const int r0 = (ph + s.pad) & 1, s0 = (pw + s.pad) & 1;
      const int nr = std::max(0, (s.R - r0 + 1) / 2), ns = std::max(0, (s.S - s0 + 1) / 2);
      const int Hp = (s.H - ph + 1) / 2, Wp = (s.W - pw + 1) / 2;
      if (Hp <= 0 || Wp <= 0) continue;
      TapPhase& t = out[n++];
      t = TapPhase{};
      t.ph = ph; t.pw = pw; t.r0 = r0; t.s0 = s0; t.nr = nr; t.ns = ns;
      t.empty = nr * ns == 0;
      const int d0 = (ph + s.pad - r0) / 2, e0 = (pw + s.pad - s0) / 2;
      t.g = make_tap(s.N, s.P, s.Q, s.O, s.C, Hp, Wp, std::max(nr, 1), std::max(ns, 1), 1, nr - 1 - d0, ns - 1 - e0);
      t.rm = make_rowmap(Hp, Wp, s.H, s.W, 2, ph, pw);
      t.img_off = off;
      off += (long)s.C * nr * ns * s.O;
    }
  return n;
}

// One-launch plan for the non-empty phases of a stride-2 DGRAD: no K split while their tiles fill the
// chip (the phases run side by side instead of one small launch after another); otherwise split the
// phase with the longest per-split K first (>= 8 K steps per split) until about one wave of workgroups,
// within the workspace.  ws_need: floats the plan's split phases use.
struct PhasePlan {
  TapMulti tm;
  int idx[MAX_TAP_PHASES];   // TapPhase index of each planned phase
  int maxsp;
  long ws_need;
  int bn;                    // tile width of the one launch (all phases share O)
};

static PhasePlan plan_tap_phases(const TapPhase* ph, int n, long ws_cap) {
  PhasePlan pl{};
  TapMulti& tm = pl.tm;
  long tiles[MAX_TAP_PHASES], total = 0;
  int ks[MAX_TAP_PHASES];
  long m_tiles = 0;
  for (int i = 0; i < n; ++i)
    if (!ph[i].empty) m_tiles += (ph[i].g.M + 127) / 128;
  int bn = 64;
  for (int i = 0; i < n; ++i)
    if (!ph[i].empty) { bn = tap_bn_for(ph[i].g.O, m_tiles); break; }
  pl.bn = bn;
  // tap-less parities (1x1 stride 2) ride along as K = 0 phases: their tiles only write zeros (or leave an
  // accumulated dX as it is) -- one launch instead of one zero-fill launch per empty parity
  for (int i = 0; i < n; ++i) {
    const int k = tm.n++;
    pl.idx[k] = i;
    tiles[k] = (long)((ph[i].g.M + 127) / 128) * ((ph[i].g.O + bn - 1) / bn);
    ks[k] = ph[i].empty ? 0 : ph[i].g.K / 64;
    tm.splits[k] = 1;
    if (!ph[i].empty) total += tiles[k];
  }
  auto need = [&](const int* sp) {
    long w = 0;
    for (int k = 0; k < tm.n; ++k)
      if (sp[k] > 1) w += (long)sp[k] * ph[pl.idx[k]].g.M * ph[pl.idx[k]].g.O;
    return w;
  };
  const long target = (bn == 128 ? 1l : 2l) * num_cus();
  if (4 * total < 3 * target) {
    long wgs = total;
    for (;;) {
      int best = -1;
      double bestv = 0.0;
      for (int k = 0; k < tm.n; ++k) {
        const double v = (double)ks[k] / tm.splits[k];
        if (ks[k] / (tm.splits[k] + 1) >= 8 && v > bestv) { best = k; bestv = v; }
      }
      if (best < 0 || wgs + tiles[best] > target) break;
      int trial[MAX_TAP_PHASES];
      for (int k = 0; k < tm.n; ++k) trial[k] = tm.splits[k] + (k == best ? 1 : 0);
      if (need(trial) > ws_cap) break;
      tm.splits[best] = trial[best];
      wgs += tiles[best];
    }
  }
  long off = 0, t0 = 0;
  pl.maxsp = 1;
  for (int k = 0; k < tm.n; ++k) {
    const TapPhase& q = ph[pl.idx[k]];
    tm.kps[k] = std::max(1, (ks[k] + tm.splits[k] - 1) / tm.splits[k]);
    tm.splits[k] = std::max(1, (ks[k] + tm.kps[k] - 1) / tm.kps[k]);
    tm.g[k] = q.g;
    if (q.empty) tm.g[k].K = 0;
    tm.rm[k] = q.rm;
    tm.woff[k] = q.img_off;
    tm.wsoff[k] = tm.splits[k] > 1 ? off : -1;
    if (tm.splits[k] > 1) off += (long)tm.splits[k] * q.g.M * q.g.O;
    tm.tile0[k] = (int)t0;
    t0 += tiles[k];
    pl.maxsp = std::max(pl.maxsp, tm.splits[k]);
  }
  tm.tile0[tm.n] = (int)t0;
  pl.ws_need = off;
  return pl;
}

// The phases of a stride-2 DGRAD as one conv_tap_phases launch (+ one split-K combine per split phase).
static void launch_tap_phases(hipStream_t st, const TapPhase* ph, int n, const bf16* dy, const bf16* wd, bf16* dx,
                              float* ws, long ws_floats, const bf16* res, const BnSums& bs) {
  const PhasePlan pl = plan_tap_phases(ph, n, ws_floats);
  const TapMulti& tm = pl.tm;
  if (tm.n == 0) return;
  for (int k = 0; k < tm.n; ++k) {
    if (tm.g[k].C % 64 || tm.g[k].O % 8 || tm.g[k].O != tm.g[0].O)
      throw std::invalid_argument("conv_tap_phases: need C % 64 == 0, O % 8 == 0 and one O");
    if (!tap_fits((long)tm.g[k].N * tm.g[k].H * tm.g[k].W * tm.g[k].C, (long)tm.g[k].O * tm.g[k].K, tm.g[k].R, tm.g[k].S))
      throw std::invalid_argument("conv_tap_phases: operands over 2 GiB or R * S > 64");
  }
  dim3 grid((unsigned)tm.tile0[tm.n], 1, (unsigned)pl.maxsp);
  if (pl.bn == 128)
    if (tap_waves() == 8)
      hipLaunchKernelGGL((conv_tap_phases<128, 8>), grid, dim3(512), 0, st, dy, wd, dx, ws, tm, res, bs);
    else
      hipLaunchKernelGGL((conv_tap_phases<128, 4>), grid, dim3(256), 0, st, dy, wd, dx, ws, tm, res, bs);
  else if (tap_waves() == 8)
    hipLaunchKernelGGL((conv_tap_phases<64, 8>), grid, dim3(512), 0, st, dy, wd, dx, ws, tm, res, bs);
  else
    hipLaunchKernelGGL((conv_tap_phases<64, 4>), grid, dim3(256), 0, st, dy, wd, dx, ws, tm, res, bs);
  for (int k = 0; k < tm.n; ++k)
    if (tm.splits[k] > 1)
      launch_tap_reduce(st, tm.g[k], tm.rm[k], ws + tm.wsoff[k], tm.splits[k], dx, nullptr, nullptr, res, bs);
}

// FWD / DGRAD with automatic split-K through ``ws`` (null / 0 floats: never split).
template <int MODE>
static void launch_fd(hipStream_t st, const ConvGeom& g, const bf16* x, const bf16* w, const bf16* dy, bf16* out,
                      double* stats, const float* shift, float* ws, long ws_floats, bool acc = false) {
  const int sp = fd_splits(g, ws_floats);
  if (sp <= 1) {
    launch_mode<MODE>(st, g, x, w, dy, out, nullptr, stats, 1, shift, acc ? 2 : 0);
    return;
  }
  launch_mode<MODE>(st, g, x, w, dy, nullptr, ws, nullptr, sp, nullptr, 1);
  const int VR = g.NC / 8;
  const int tb = (256 / VR) * VR;
  const int rstep = tb / VR;
  // plain combine: ~4 blocks per CU; with BN statistics fewer blocks (their
  // per-channel atomics contend on 2 x NC addresses)
  const int rows_per_block = stats ? std::max(2 * rstep, (g.M + 255) / 256) : std::max(rstep, (g.M + 1023) / 1024);
  const int nblk = (g.M + rows_per_block - 1) / rows_per_block;
  RowMap rm{};
  if (MODE == DGRAD && g.st != 1) rm = make_rowmap(g.Hp, g.Wp, g.H, g.W, g.st, g.ph, g.pw);
  hipLaunchKernelGGL(conv_splitk_reduce, dim3(nblk), dim3(tb), 0, st, ws, sp, g.M, g.NC, rm, out, stats, shift,
                     rows_per_block, acc ? out : nullptr, BnSums{});
}

// K-split count for the weight gradient: at most one wave of two workgroups per CU (rounded down: ResNet-18's
// layer-4 3x3 WGRAD, 144 tiles, 48.0 -> 40.5 us with 3 splits instead of 4 -- the fourth made a second, 64-workgroup
// wave; profiles/r5_cnn/experiments/wgrad_splits.jsonl), at least 8 K steps per split, a bounded workspace.
static int wgrad_splits(const ConvGeom& g, long ws_cap_floats) {
  const TileCfg t = pick_tiles_wgrad(g.M, g.NC);
  const long tiles = (long)((g.M + t.BM - 1) / t.BM) * ((g.NC + t.BN - 1) / t.BN);
  const int ksteps = (g.K + BK - 1) / BK;
  static const bool up = [] {
    const char* e = std::getenv("FEDMI_WGRAD_SPLITS_UP");   // A/B: round 5's rounded-up count
    return e && e[0] == '1';
  }();
  long sp = up ? (2l * num_cus() + tiles - 1) / tiles : std::max<long>(1, 2l * num_cus() / tiles);
  sp = std::min<long>(sp, std::max(1, ksteps / 8));
  if (ws_cap_floats > 0) sp = std::min<long>(sp, ws_cap_floats / ((long)g.M * g.NC));
  sp = std::max<long>(1, sp);
  const int kps = (int)((ksteps + sp - 1) / sp);
  return (ksteps + kps - 1) / kps;
}

// the forward runs on conv_tap for C % 64 == 0, and (GEN) for any C % 8 == 0 from 16 channels with O % 8 == 0;
// FEDMI_TAP_GEN=0 keeps those on the generic implicit GEMM (A/B runs, tests)
static bool tap_gen_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("FEDMI_TAP_GEN");
    return !(e && e[0] == '0');
  }();
  return on;
}
static bool fwd_tap_ok(const ConvShape& s) {
  const long K = (long)s.R * s.S * s.C;
  return s.O % 8 == 0 && (s.C % 64 == 0 || (tap_gen_enabled() && s.C % 8 == 0 && s.C >= 16)) &&
         tap_fits((long)s.N * s.H * s.W * s.C, (long)s.O * K, s.R, s.S);
}

// Y[N,P,Q,O] = conv(X[N,H,W,C], W_rsc); stats (optional) += [sum | sumsq] of (Y - shift) per output channel.
void launch_conv_fwd(hipStream_t st, const ConvShape& s, const bf16* x, const bf16* wrsc, bf16* y, double* stats,
                     const float* shift, float* ws, long ws_floats, const bf16* res) {
  check_shape(s);
  ConvGeom g = make_geom(s);
  g.M = s.N * s.P * s.Q; g.NC = s.O; g.K = s.R * s.S * s.C;
  if (fwd_tap_ok(s)) {
    const TapGeom t = make_tap(s.N, s.H, s.W, s.C, s.O, s.P, s.Q, s.R, s.S, s.st, s.pad, s.pad);
    launch_tap(st, t, x, wrsc, y, stats, shift, RowMap{}, ws, ws_floats, res);
    return;
  }
  if (res) throw std::invalid_argument("conv_fwd: a fused residual needs the tap path (C % 8 == 0, C >= 16)");
  static const bool stem_on = [] {
    const char* e = std::getenv("FEDMI_STEM");                // A/B: 0 = the generic implicit GEMM for the stem
    return !(e && e[0] == '0');
  }();
  if (stem_on && s.C == 8 && s.R == 3 && s.S == 3 && s.st == 1 && s.pad == 1 && (s.O == 32 || s.O == 64)) {
    // the network-input conv (conv_stem_kernel): ~4 pixel tiles of 16 per wave
    const StemGeom sg{s.N, s.H, s.W, s.O, s.N * s.H * s.W};
    const long ntiles = (sg.M + 15) / 16;
    const unsigned nblk = (unsigned)std::max<long>(1, std::min<long>(2048, (ntiles + 15) / 16));
    if (s.O == 64)
      hipLaunchKernelGGL(conv_stem_kernel<4>, dim3(nblk), dim3(256), 0, st, x, wrsc, y, stats, shift, sg);
    else
      hipLaunchKernelGGL(conv_stem_kernel<2>, dim3(nblk), dim3(256), 0, st, x, wrsc, y, stats, shift, sg);
    return;
  }
  launch_fd<FWD>(st, g, x, wrsc, nullptr, y, stats, shift, ws, ws_floats);
}

// dX[N,H,W,C] = conv_transpose(dY[N,P,Q,O], W_rsc)   (every element written).
// Stride 2 runs as 4 sub-pixel phases so no MFMA multiplies a structural zero.
// acc: dx += result (the data gradient of one branch of a multi-branch block)
//
// add: dx = result + add (a second incoming grad, e.g. the shortcut branch's; != dx) and bs: the
// producer BN's backward sums taken in the epilogue -- both only on the tap path without empty
// phases (conv_dgrad_fusable).
// O % 64 == 0 (every stride: conv_tap / conv_tap_phases), or stride 1 with O % 8 == 0 from 16 channels: one phase, a
// plain conv_tap problem over dY with O input channels -> conv_tap<GEN> (the GoogLeNet / zoo narrow branches)
static bool dgrad_gen_enabled() {   // FEDMI_DGRAD_GEN=0: the GEN DGRAD only off (A/B)
  static const bool on = [] {
    const char* e = std::getenv("FEDMI_DGRAD_GEN");
    return !(e && e[0] == '0');
  }();
  return on && tap_gen_enabled();
}
static bool dgrad_tap_ok(const ConvShape& s) {
  const bool gen = s.st == 1 && dgrad_gen_enabled() && s.O % 8 == 0 && s.O >= 16;
  return (s.O % 64 == 0 || gen) && tap_fits((long)s.N * s.P * s.Q * s.O, (long)s.C * s.R * s.S * s.O, s.R, s.S);
}

int conv_dgrad_fusable(const ConvShape& s, int has_wd) {
  check_shape(s);
  if (!has_wd || !dgrad_tap_ok(s)) return 0;
  TapPhase ph[4];
  const int n = dgrad_tap_phases(s, ph);
  for (int i = 0; i < n; ++i)
    if (ph[i].empty) return 0;
  return 1;
}

void launch_conv_dgrad(hipStream_t st, const ConvShape& s, const bf16* dy, const bf16* wrsc, bf16* dx, float* ws,
                       long ws_floats, const bf16* wd, int acc, const bf16* add, const BnSums* bs) {
  check_shape(s);
  if ((add || bs) && !conv_dgrad_fusable(s, wd != nullptr))
    throw std::invalid_argument("conv_dgrad: add / BN sums need the tap path (conv_dgrad_fusable)");
  if (add && acc) throw std::invalid_argument("conv_dgrad: add and accumulate are exclusive");
  if (bs && (!bs->rep || !bs->z || !bs->mean || !bs->inv || bs->reps < 1 || (bs->zb && (!bs->meanb || !bs->invb)) ||
             (bs->msc && (bs->y || bs->msc_ld <= 0))))
    throw std::invalid_argument("conv_dgrad: incomplete BN sums descriptor");
  if (wd != nullptr && dgrad_tap_ok(s)) {   // tap-major path on the dgrad weight image
    TapPhase ph[4];
    const int n = dgrad_tap_phases(s, ph);
    if (n > 1)   // stride 2: every parity in one launch (tap-less parities as K = 0 phases that write zeros)
      launch_tap_phases(st, ph, n, dy, wd, dx, ws, ws_floats, acc ? dx : add, bs ? *bs : BnSums{});
    else
      launch_tap(st, ph[0].g, dy, wd + ph[0].img_off, dx, nullptr, nullptr, ph[0].rm, ws, ws_floats,
                 acc ? dx : add, bs ? *bs : BnSums{});
    return;
  }
  ConvGeom g = make_geom(s);
  g.NC = s.C;
  if (s.st == 1) {
    g.M = s.N * s.H * s.W; g.K = s.R * s.S * s.O;
    launch_fd<DGRAD>(st, g, nullptr, wrsc, dy, dx, nullptr, nullptr, ws, ws_floats, acc != 0);
    return;
  }
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      ConvGeom q = g;
      q.ph = ph; q.pw = pw;
      q.r0 = (ph + s.pad) & 1; q.s0 = (pw + s.pad) & 1;
      q.nr = std::max(0, (s.R - q.r0 + 1) / 2); q.ns = std::max(0, (s.S - q.s0 + 1) / 2);
      q.Hp = (s.H - ph + 1) / 2; q.Wp = (s.W - pw + 1) / 2;
      if (q.Hp <= 0 || q.Wp <= 0) continue;
      q.dNS = make_div(std::max(q.ns, 1)); q.dWp = make_div(q.Wp); q.dHWp = make_div(q.Hp * q.Wp);
      q.M = s.N * q.Hp * q.Wp; q.K = q.nr * q.ns * s.O;
      if (q.K == 0) {   // phase with no taps (1x1 stride 2, odd parity): the kernel writes zeros
        launch_mode<DGRAD>(st, q, nullptr, wrsc, dy, dx, nullptr, nullptr, 1, nullptr, acc ? 2 : 0);
        continue;
      }
      launch_fd<DGRAD>(st, q, nullptr, wrsc, dy, dx, nullptr, nullptr, ws, ws_floats, acc != 0);
    }
}

static ConvGeom wgrad_geom(const ConvShape& s) {
  check_shape(s);
  ConvGeom g = make_geom(s);
  g.M = s.O; g.NC = s.R * s.S * s.C; g.K = s.N * s.P * s.Q;
  return g;
}

// Workspace (floats) split-K FWD + DGRAD want for this shape (0: they never split).
long conv_fd_ws_floats(const ConvShape& s) {
  check_shape(s);
  ConvGeom g = make_geom(s);
  g.M = s.N * s.P * s.Q; g.NC = s.O; g.K = s.R * s.S * s.C;
  long need = 0;
  const long cap = 1l << 40;
  int sp = fd_splits(g, cap);
  if (sp > 1) need = std::max(need, (long)sp * g.M * g.NC);
  if (fwd_tap_ok(s)) {
    const TapGeom t = make_tap(s.N, s.H, s.W, s.C, s.O, s.P, s.Q, s.R, s.S, s.st, s.pad, s.pad);
    const int tsp = tap_splits(t, cap);
    if (tsp > 1) need = std::max(need, (long)tsp * t.M * t.O);
  }
  if (dgrad_tap_ok(s)) {
    TapPhase ph[4];
    const int n = dgrad_tap_phases(s, ph);
    if (n > 1) {
      need = std::max(need, plan_tap_phases(ph, n, cap).ws_need);
    } else {
      for (int i = 0; i < n; ++i) {
        if (ph[i].empty) continue;
        const int tsp = tap_splits(ph[i].g, cap);
        if (tsp > 1) need = std::max(need, (long)tsp * ph[i].g.M * ph[i].g.O);
      }
    }
  }
  ConvGeom d = make_geom(s);
  d.NC = s.C;
  if (s.st == 1) {
    d.M = s.N * s.H * s.W; d.K = s.R * s.S * s.O;
    sp = fd_splits(d, cap);
    if (sp > 1) need = std::max(need, (long)sp * d.M * d.NC);
  } else {
    for (int ph = 0; ph < 2; ++ph) {
      const int r0 = (ph + s.pad) & 1;
      const int nr = std::max(0, (s.R - r0 + 1) / 2);
      const int Hp = (s.H - ph + 1) / 2;
      for (int pw = 0; pw < 2; ++pw) {
        const int s0 = (pw + s.pad) & 1;
        const int ns = std::max(0, (s.S - s0 + 1) / 2);
        const int Wp = (s.W - pw + 1) / 2;
        if (Hp <= 0 || Wp <= 0 || nr * ns == 0) continue;
        ConvGeom q = d;
        q.M = s.N * Hp * Wp; q.K = nr * ns * s.O;
        sp = fd_splits(q, cap);
        if (sp > 1) need = std::max(need, (long)sp * q.M * q.NC);
      }
    }
  }
  return need;
}

// conv_wgrad_halo applies to 3x3 / stride 1 / pad 1 with C and O % 64 and 128-pixel blocks; every other
// shape takes the generic WGRAD (split-K conv_igemm).
static bool wgrad_1x1_enabled() {   // FEDMI_WGRAD_1X1=0: 1x1 WGRADs on the generic split-K kernel (A/B)
  static const bool on = [] {
    const char* e = std::getenv("FEDMI_WGRAD_1X1");
    return !(e && e[0] == '0');
  }();
  return on;
}
static bool wgrad_halo_geom(const ConvShape& s, HaloGeom* h, bool allow_1x1 = true) {
  if (allow_1x1 && s.R == 1 && s.S == 1 && s.st == 1 && s.pad == 0 && s.C % 64 == 0 && s.O % 64 == 0 &&
      wgrad_1x1_enabled()) {
    // 1x1 / stride 1: conv_wgrad_halo<1, 1> over 128-pixel blocks (K = C marks the one-tap form).  Its 64 x 64
    // tiles re-read each operand chunk twice as often as the generic kernel's 128 x 128 ones, which the L2 absorbs
    // only for small problems: 1.3-2x faster at MobileNet's 16x16 / 8x8 pointwise shapes, 7-65 % slower from
    // M * (C + O) ~ 2e7 on (GoogLeNet 32x32 256 -> 128, 16x16 512 -> 192, 8x8 832 -> 256;
    // profiles/r6_cnn/wgrad1x1_halo/)
    const long M = (long)s.N * s.H * s.W;
    if (M % 128 || M >= (1l << 31) || M * (s.C + s.O) > 3l * (1l << 22)) return false;
    HaloGeom x{};
    x.N = s.N; x.H = s.H; x.W = s.W; x.C = s.C; x.O = s.O; x.M = (int)M; x.K = s.C;
    x.NPR = 128; x.nchunks = s.C / 64;
    *h = x;
    return true;
  }
  if (s.R != 3 || s.S != 3 || s.st != 1 || s.pad != 1 || s.C % 64 || s.O % 64) return false;
  const TapGeom t = make_tap(s.N, s.H, s.W, s.C, s.O, s.P, s.Q, 3, 3, 1, 1, 1);
  // the 288-row window (4x4 images) would spill the per-lane fragment offset tables: generic path
  return halo_geom(t, RowMap{}, h) && h->NPR <= 208;
}

// K splits of the halo WGRAD: about one workgroup per CU over the (O / 64) x (C / 64) tiles -- fewer
// splits mean fewer fp32 partial bytes to write and reduce.
static int wgrad_halo_splits(const HaloGeom& h, long ws_cap_floats) {
  const long want = num_cus();
  const long tiles = (long)(h.O / 64) * h.nchunks;
  const int nblk = h.M / 128;
  long sp = std::max<long>(1, (want + tiles / 2) / tiles);
  sp = std::min<long>(sp, nblk);
  if (ws_cap_floats > 0) sp = std::min<long>(sp, ws_cap_floats / ((long)h.O * h.K));   // K = taps * C
  sp = std::max<long>(1, sp);
  const int bps = (int)((nblk + sp - 1) / sp);
  return (nblk + bps - 1) / bps;
}

long conv_wgrad_ws_floats(const ConvShape& s) {
  const ConvGeom g = wgrad_geom(s);
  long need = (long)wgrad_splits(g, 0) * g.M * g.NC;
  HaloGeom h;
  if (wgrad_halo_geom(s, &h)) need = std::max(need, (long)wgrad_halo_splits(h, 0) * g.M * g.NC);
  return need;
}

// dW[O][Cw][R][S] (fp32, PyTorch layout) = (or +=) X^T dY.  ``ws`` holds
// ws_floats floats; splits <= 0 picks automatically within that capacity.
// dw: [Ow][Cw][R][S] (Ow <= 0: O) -- the first Ow filters of an O-padded conv land in the unpadded gradient.
// G > 1: a grouped conv run densely with a block-diagonal weight image; filter o keeps only its group's Cw
// channels of the dense gradient.
// allow_1x1 = 0: no conv_wgrad_halo<1, 1> route (the aten backend: mixed results across the zoo families)
void launch_conv_wgrad(hipStream_t st, const ConvShape& s, const bf16* x, const bf16* dy, float* dw, float* ws,
                       long ws_floats, int splits, int accumulate, int Ow, int G, WredItem* defer, int allow_1x1) {
  if (Ow <= 0 || Ow > s.O) Ow = s.O;
  if (G < 1) G = 1;
  if (G > 1 && (s.O % G || s.C < G * s.Cw || Ow != s.O))
    throw std::invalid_argument("conv_wgrad: grouped gradient needs O % G == 0, C >= G * Cw, no O pad");
  const ConvGeom g = wgrad_geom(s);
  const long plane = (long)g.M * g.NC;
  if (ws_floats < plane) throw std::invalid_argument("conv_wgrad: workspace smaller than one O x RSC plane");
  HaloGeom h;
  if (splits <= 0 && wgrad_halo_geom(s, &h, allow_1x1 != 0)) {
    splits = wgrad_halo_splits(h, ws_floats);
    const int nblk = h.M / 128;
    const int bps = (nblk + splits - 1) / splits;
    dim3 grid((unsigned)((h.O / 64) * h.nchunks), 1, (unsigned)splits);
    if (h.K == h.C)
      hipLaunchKernelGGL((conv_wgrad_halo<1, 1>), grid, dim3(256), 0, st, x, dy, ws, h, bps);
    else
      hipLaunchKernelGGL(conv_wgrad_halo<1>, grid, dim3(256), 0, st, x, dy, ws, h, bps);
  } else {
    if (splits <= 0) splits = wgrad_splits(g, ws_floats);
    const int ksteps = (g.K + BK - 1) / BK;
    splits = std::max(1, std::min<int>(splits, ksteps));
    const int kps = (ksteps + splits - 1) / splits;
    splits = (ksteps + kps - 1) / kps;
    if ((long)splits * plane > ws_floats) throw std::invalid_argument("conv_wgrad: workspace too small for splits");
    launch_mode<WGRAD>(st, g, x, nullptr, dy, nullptr, ws, nullptr, splits);
  }
  if (s.R * s.S > WRED_MAX_RS) throw std::invalid_argument("conv_wgrad: window larger than 7x7");
  const long blocks = (long)s.O * ((s.C + 63) / 64);
  // enough (o, channel-block) tiles: coalesced tile writes; else one lane per workspace column
  const WredItem it{ws, dw, blocks >= 1024 ? WRED_TILE : WRED_COLS, splits, s.O, s.C, s.Cw, s.R * s.S, accumulate, Ow, G};
  if (defer) {               // the caller runs it later in launch_wgrad_reduce_multi
    *defer = it;
    return;
  }
  launch_wgrad_reduce_multi(st, &it, 1);
}

// Deferred reductions (WredItem, filled by launch_conv_wgrad / launch_dw_wgrad with a `defer` slot): one launch
// per WRED_MULTI_MAX items; a single item launches its standalone kernel.
void launch_wgrad_reduce_multi(hipStream_t st, const WredItem* items, int n) {
  for (int i0 = 0; i0 < n; i0 += WRED_MULTI_MAX) {
    const int m = std::min(WRED_MULTI_MAX, n - i0);
    if (m == 1) {
      const WredItem& e = items[i0];
      const unsigned g = (unsigned)wred_blocks(e);
      if (e.kind == WRED_TILE)
        hipLaunchKernelGGL(conv_wgrad_reduce, dim3(g), dim3(256), wred_lds_bytes(e), st, e.ws, e.splits, e.O, e.C, e.Cw,
                           e.RS, e.dw, e.accumulate, e.Ow, e.G);
      else if (e.kind == WRED_COLS)
        hipLaunchKernelGGL(conv_wgrad_reduce_cols, dim3(g), dim3(256), 0, st, e.ws, e.splits, e.O, e.C, e.Cw, e.RS,
                           e.dw, e.accumulate, e.Ow, e.G);
      else
        launch_dw_wgrad_reduce(st, e);
      continue;
    }
    WredTable t{};
    long blk = 0;
    size_t lds = 0;
    for (int k = 0; k < m; ++k) {
      t.it[k] = items[i0 + k];
      t.blk0[k] = (int)blk;
      blk += wred_blocks(items[i0 + k]);
      lds = std::max(lds, wred_lds_bytes(items[i0 + k]));
    }
    t.n = m;
    if (blk >= (1l << 31)) throw std::invalid_argument("wgrad_reduce_multi: grid too large");
    hipLaunchKernelGGL(wgrad_reduce_multi, dim3((unsigned)blk), dim3(256), lds, st, t);
  }
}

struct PackItem {
  const float* w;
  bf16* wr;
  int O, Cw, C, RS;
  int O8;            // <= 0: O (no zero filters)
  int G;             // <= 1: dense; > 1: block-diagonal image of a grouped conv (C = G * Cw channels)
};

// All dense-conv weight images of a network from their fp32 masters, <= MAX_PACK per launch.
void launch_conv_pack_multi(hipStream_t st, const PackItem* items, int n) {
  for (int b = 0; b < n; b += MAX_PACK) {
    PackTable t{};
    t.n = std::min(MAX_PACK, n - b);
    int rows = 0, max_row = 1;
    for (int k = 0; k < t.n; ++k) {
      const PackItem& it = items[b + k];
      if (it.C % 8 || it.C < it.Cw) throw std::invalid_argument("conv_pack_multi: bad channel padding");
      if (it.G > 1 && (it.O % it.G || it.C < it.G * it.Cw || (it.O8 > it.O)))
        throw std::invalid_argument("conv_pack_multi: grouped image needs O % G == 0, C >= G * Cw, no O pad");
      if ((long)it.Cw * it.RS > PACK_ROW_MAX) throw std::invalid_argument("conv_pack_multi: row too long");
      const int o8 = it.O8 > it.O ? it.O8 : it.O;
      t.e[k] = PackEntry{it.w, it.wr, it.O, it.Cw, it.C, it.RS, o8, it.G > 1 ? it.G : 1, rows};
      rows += o8;
      max_row = std::max(max_row, it.Cw * it.RS);
    }
    hipLaunchKernelGGL(conv_pack_multi_kernel, dim3(rows), dim3(256), max_row * sizeof(float), st, t);
  }
}

// DGRAD weight images (conv_tap layout, phases concatenated) for several convs, one launch per <= MAX_DPACK phases.
struct DPackItem {
  const float* w;
  bf16* wd;
  int O, Cw, C, R, S, st, pad;
};

void launch_dgrad_pack_multi(hipStream_t st, const DPackItem* items, int n) {
  std::vector<DPackEntry> all;
  for (int k = 0; k < n; ++k) {
    const DPackItem& it = items[k];
    if (it.R * it.S > 49 || it.C % 8 || it.C < it.Cw) throw std::invalid_argument("dgrad_pack: unsupported shape");
    ConvShape s{};
    s.N = 1; s.H = 8; s.W = 8; s.P = 4; s.Q = 4;   // spatial sizes only gate empty phases here
    s.C = it.C; s.Cw = it.Cw; s.O = it.O; s.R = it.R; s.S = it.S; s.st = it.st; s.pad = it.pad;
    TapPhase ph[4];
    const int np = dgrad_tap_phases(s, ph);
    for (int i = 0; i < np; ++i) {
      if (ph[i].empty) continue;
      DPackEntry e{};
      e.w = it.w; e.wd = it.wd + ph[i].img_off;
      e.O = it.O; e.Cw = it.Cw; e.Cpad = it.C; e.R = it.R; e.S = it.S;
      e.r0 = ph[i].r0; e.s0 = ph[i].s0; e.nr = ph[i].nr; e.ns = ph[i].ns; e.step = it.st;
      all.push_back(e);
    }
  }
  for (size_t b = 0; b < all.size(); b += MAX_DPACK) {
    DPackTable t{};
    t.n = (int)std::min<size_t>(MAX_DPACK, all.size() - b);
    int max_rs = 1;
    for (int k = 0; k < t.n; ++k) max_rs = std::max(max_rs, all[b + k].R * all[b + k].S);
    t.cb = max_rs <= 9 ? DP_CB : 4;
    int blk = 0;
    for (int k = 0; k < t.n; ++k) {
      t.e[k] = all[b + k];
      t.e[k].blk0 = blk;
      blk += ((t.e[k].O + 63) / 64) * ((t.e[k].Cpad + t.cb - 1) / t.cb);
    }
    hipLaunchKernelGGL(dgrad_pack_kernel, dim3(blk), dim3(256), 64 * (t.cb * max_rs + 1) * sizeof(float), st, t);
  }
}

// Fused SGD + weight images (sgd_pack_kernel): the host builds the table once per engine (convs first, then the
// flat segments, in workgroup order); the caller copies `table` to device memory and launches with it.
struct SgdPackConv {
  long off;          // element offset of the fp32 weight [O][Cw][R][S] in the flat master
  bf16* wr;          // forward image [O][R][S][C] (nullptr: none)
  bf16* wd;          // DGRAD image, phases concatenated (nullptr: none; needs O % 64 == 0)
  int O, Cw, C, R, S, st, pad;
};
struct SgdPackPlan {
  std::vector<char> table;
  int n_entries, n_blocks, lds_bytes;
};

SgdPackPlan build_sgd_pack_plan(const SgdPackConv* convs, int nc, const long* segs, int nseg) {
  std::vector<SgdPackEntry> v;
  int blk = 0, lds = 0;
  for (int k = 0; k < nc; ++k) {
    const SgdPackConv& c = convs[k];
    if (c.C % 8 || c.C < c.Cw || c.Cw < 1 || c.O < 1 || c.R * c.S > 49 || (c.wd && (c.O % 8 || (c.O % 64 && c.st != 1))))
      throw std::invalid_argument("sgd_pack: unsupported conv (C % 8, C >= Cw, R*S <= 49; a DGRAD image needs O % 64, "
                                  "or O % 8 at stride 1)");
    SgdPackEntry e{};
    e.kind = 0; e.off = c.off; e.wr = c.wr;
    e.O = c.O; e.Cw = c.Cw; e.C = c.C; e.R = c.R; e.S = c.S; e.step = c.st;
    // input channels per block: 16 for 3x3 (144 floats per filter row), 4 past 3x3 (LDS), 64 for 1x1 (cold-cache
    // tail, MobileNet: 16 -> 53 us, 64 -> 37, 128 -> 40; profiles/r5_cnn/sgdpack/)
    e.cb = c.R * c.S > 9 ? 4 : c.R * c.S > 4 ? DP_CB : c.R * c.S > 1 ? 32 : 64;
    if (c.wd) {
      ConvShape s{};
      s.N = 1; s.H = 8; s.W = 8; s.P = 4; s.Q = 4;   // spatial sizes only gate empty phases (launch_dgrad_pack_multi)
      s.C = c.C; s.Cw = c.Cw; s.O = c.O; s.R = c.R; s.S = c.S; s.st = c.st; s.pad = c.pad;
      TapPhase ph[4];
      const int np = dgrad_tap_phases(s, ph);
      for (int i = 0; i < np; ++i) {
        if (ph[i].empty) continue;
        e.wd[e.nph] = c.wd + ph[i].img_off;
        e.r0[e.nph] = ph[i].r0; e.s0[e.nph] = ph[i].s0; e.nr[e.nph] = ph[i].nr; e.ns[e.nph] = ph[i].ns;
        ++e.nph;
      }
    }
    e.blk0 = blk;
    blk += ((c.O + 63) / 64) * ((c.C + e.cb - 1) / e.cb);
    lds = std::max(lds, (int)(64 * (e.cb * c.R * c.S + 1) * sizeof(float)));
    v.push_back(e);
  }
  for (int k = 0; k < nseg; ++k) {
    const long off = segs[2 * k], len = segs[2 * k + 1];
    if (len <= 0) continue;
    for (long s0 = 0; s0 < len; s0 += (1l << 30)) {   // entries count O in 32 bits
      SgdPackEntry e{};
      e.kind = 1; e.off = off + s0; e.O = (int)std::min<long>(len - s0, 1l << 30);
      e.blk0 = blk;
      blk += (e.O + SP_SEG - 1) / SP_SEG;
      v.push_back(e);
    }
  }
  if (v.empty()) throw std::invalid_argument("sgd_pack: empty plan");
  SgdPackPlan p;
  p.table.resize(v.size() * sizeof(SgdPackEntry));
  std::memcpy(p.table.data(), v.data(), p.table.size());
  p.n_entries = (int)v.size();
  p.n_blocks = blk;
  p.lds_bytes = lds;
  return p;
}

void launch_sgd_pack(hipStream_t st, const void* table, int n_entries, int n_blocks, int lds_bytes, float* P,
                     const float* G, float* B, float lr, float m, float wd, float dampening, int nesterov, int first) {
  if (n_entries <= 0 || n_blocks <= 0) return;
  hipLaunchKernelGGL(sgd_pack_kernel<4>, dim3((unsigned)n_blocks), dim3(256), lds_bytes, st,
                     static_cast<const SgdPackEntry*>(table), n_entries, P, G, B, lr, m, wd, dampening, nesterov, first);
}


void launch_conv_pack(hipStream_t st, const float* w, bf16* wrsc, int O, int Cw, int C, int RS, int O8, int G) {
  const PackItem it{w, wrsc, O, Cw, C, RS, O8, G};
  launch_conv_pack_multi(st, &it, 1);
}

}  // namespace fedmi
