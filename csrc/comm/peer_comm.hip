// fedmi — peer-to-peer collectives over hipIpc-mapped staging buffers (see peer_comm.h).
//
// Synchronisation (one barrier = one phase):
//   every wave of the workgroup waits for its own stores (vmcnt 0), workgroup
//   barrier, wave 0 issues a SYSTEM-scope release (L2 write-back: the peer may be
//   another GPU across xGMI or another XCD of this one), then lane p stores the
//   call's epoch into rank p's flag slot [phase][block][me] and polls its own slot
//   [phase][block][p]; a SYSTEM-scope acquire (L1/L2 invalidate) follows, then a
//   workgroup barrier releases the other waves to read peer data.
//   Flags live in uncached memory; polls are bounded by a wall-clock timeout that
//   sets PeerSignal::error instead of hanging when a peer died mid-collective, and
//   by a host-pinned abort word (PeerArgs::abort_flag) that the client's watchdog
//   sets as soon as the coordinator reports the loss (reference: a dead client is
//   dropped at its next failed RPC, src/server.py:59-62, 72-75) -- the survivors
//   then leave the barrier within one poll period instead of the full timeout.
//
// Buffer reuse: call k uses staging slot k & 1.  A rank rewrites slot k & 1 only
// in call k + 2, after call k + 1's barrier, which every peer enters only once
// its stream has finished call k — so one barrier per call suffices for oneshot.
//
// Call counter: every call advances ALL kPeerMaxBlocks epoch words, whatever its
// grid size (block b of a B-block call writes words b, b + B, b + 2B, ...), so the
// epoch -- and with it the slot parity -- is one communicator-wide call number.
// Calls of different grid sizes (fedavg's f32 reduce then a 1-block int64 call,
// the int8 compressor's gather then scale) therefore stay in step on every block.
// The words are read at the start of the NEXT call, which the stream orders after
// every block of this one has retired.
#include "peer_comm.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

namespace fedmi {
void check_hip(hipError_t e, const char* what);
}

namespace {

using fedmi::PeerArgs;
using fedmi::PeerSignal;
using fedmi::kPeerMaxRanks;

#define PDEV __device__ __forceinline__

PDEV uint32_t ld_sys(const uint32_t* p) { return __scoped_atomic_load_n(p, __ATOMIC_RELAXED, __MEMORY_SCOPE_SYSTEM); }
PDEV void st_sys(uint32_t* p, uint32_t v) { __scoped_atomic_store_n(p, v, __ATOMIC_RELAXED, __MEMORY_SCOPE_SYSTEM); }

PDEV char* region(const PeerArgs& a, int p, int slot, int which) {
  return a.data[p] + (long long)(slot * 2 + which) * a.cap;
}

// Epoch of this call for workgroup b (device-side counter: replays from a graph stay in step).
PDEV uint32_t begin_call(const PeerArgs& a, int b) {
  __shared__ uint32_t s_ep;
  if (threadIdx.x == 0) s_ep = ld_sys(&a.sig[a.rank]->epoch[b]) + 1u;
  __syncthreads();
  return s_ep;
}

PDEV void end_call(const PeerArgs& a, int b, uint32_t ep) {
  for (int j = b + (int)threadIdx.x * (int)gridDim.x; j < fedmi::kPeerMaxBlocks; j += (int)(blockDim.x * gridDim.x))
    st_sys(&a.sig[a.rank]->epoch[j], ep);
}

// Returns false (for the whole workgroup) when a peer never arrived: the caller then
// skips every further access to peer memory -- a dead peer's buffers are not touched.
PDEV bool peer_barrier(const PeerArgs& a, int phase, int b, uint32_t ep) {
  __shared__ int s_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) s_ok = 1;
  __syncthreads();
  if (threadIdx.x < 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int p = threadIdx.x;
    bool ok = true;
    if (p < a.world) {
      st_sys(&a.sig[p]->flags[phase][b][a.rank], ep);
      const uint32_t* mine = &a.sig[a.rank]->flags[phase][b][p];
      const unsigned long long t0 = wall_clock64();
      uint32_t polls = 0;
      while (ld_sys(mine) < ep) {
        __builtin_amdgcn_s_sleep(1);
        // the abort word lives in host memory (one PCIe read): looked at every 256 polls only
        const bool aborted = ((++polls & 255u) == 0u) && ld_sys(a.abort_flag) != 0u;
        if (aborted || (long long)(wall_clock64() - t0) > a.timeout_ticks) {
          st_sys(&a.sig[a.rank]->error, 1u);
          ok = false;
          break;
        }
      }
    }
    if (__ballot(!ok) != 0ull && threadIdx.x == 0) s_ok = 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return s_ok != 0;
}

PDEV float4 f4add(float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); }

// Sum of element i (float4 granule) over all ranks, in rank order 0..W-1.
PDEV float4 gather_sum4(const PeerArgs& a, int slot, long long i) {
  float4 v[kPeerMaxRanks];
#pragma unroll
  for (int p = 0; p < kPeerMaxRanks; ++p)
    if (p < a.world) v[p] = reinterpret_cast<const float4*>(region(a, p, slot, 0))[i];
  float4 acc = v[0];
#pragma unroll
  for (int p = 1; p < kPeerMaxRanks; ++p)
    if (p < a.world) acc = f4add(acc, v[p]);
  return acc;
}

PDEV float gather_sum1(const PeerArgs& a, int slot, long long i) {
  float acc = reinterpret_cast<const float*>(region(a, 0, slot, 0))[i];
  for (int p = 1; p < a.world; ++p) acc += reinterpret_cast<const float*>(region(a, p, slot, 0))[i];
  return acc;
}

__global__ __launch_bounds__(256) void peer_oneshot_f32_kernel(PeerArgs a, const float* in, float* out, long long n,
                                                               float scale) {
  const int b = blockIdx.x, t = threadIdx.x;
  const uint32_t ep = begin_call(a, b);
  const int slot = ep & 1;
  const long long n4 = n >> 2, stride = (long long)gridDim.x * 256;
  const int tail = (int)(n & 3);
  float* mine = reinterpret_cast<float*>(region(a, a.rank, slot, 0));
  for (long long i = (long long)b * 256 + t; i < n4; i += stride)
    reinterpret_cast<float4*>(mine)[i] = reinterpret_cast<const float4*>(in)[i];
  if (b == 0 && t < tail) mine[n4 * 4 + t] = in[n4 * 4 + t];
  if (!peer_barrier(a, 0, b, ep)) return;
  for (long long i = (long long)b * 256 + t; i < n4; i += stride) {
    float4 s = gather_sum4(a, slot, i);
    s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
    reinterpret_cast<float4*>(out)[i] = s;
  }
  if (b == 0 && t < tail) out[n4 * 4 + t] = scale * gather_sum1(a, slot, n4 * 4 + t);
  end_call(a, b, ep);
}

// Two-shot: slices of L float4 granules; rank r owns slice r.
__global__ __launch_bounds__(256) void peer_twoshot_f32_kernel(PeerArgs a, const float* in, float* out, long long n,
                                                               float scale) {
  const int b = blockIdx.x, t = threadIdx.x, W = a.world, r = a.rank;
  const uint32_t ep = begin_call(a, b);
  const int slot = ep & 1;
  const long long n4 = n >> 2, stride = (long long)gridDim.x * 256;
  const long long L = (n4 + W - 1) / W;
  const int tail = (int)(n & 3);
  float* mine_in = reinterpret_cast<float*>(region(a, r, slot, 0));
  float* mine_out = reinterpret_cast<float*>(region(a, r, slot, 1));
  // 1. stage the whole input (slice s, sub-range of workgroup b, for every s)
  for (int s = 0; s < W; ++s) {
    const long long lo = s * L, hi = (s + 1) * L < n4 ? (s + 1) * L : n4;
    for (long long i = lo + (long long)b * 256 + t; i < hi; i += stride)
      reinterpret_cast<float4*>(mine_in)[i] = reinterpret_cast<const float4*>(in)[i];
  }
  if (b == 0 && t < tail) mine_in[n4 * 4 + t] = in[n4 * 4 + t];
  if (!peer_barrier(a, 0, b, ep)) return;
  // 2. reduce my slice from every peer, push the result into every peer's result area
  {
    const long long lo = r * L, hi = (r + 1) * L < n4 ? (r + 1) * L : n4;
    for (long long i = lo + (long long)b * 256 + t; i < hi; i += stride) {
      float4 s = gather_sum4(a, slot, i);
      s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
      for (int p = 0; p < W; ++p) reinterpret_cast<float4*>(region(a, p, slot, 1))[i] = s;
    }
    if (r == 0 && b == 0 && t < tail) {
      const float v = scale * gather_sum1(a, slot, n4 * 4 + t);
      for (int p = 0; p < W; ++p) reinterpret_cast<float*>(region(a, p, slot, 1))[n4 * 4 + t] = v;
    }
  }
  if (!peer_barrier(a, 1, b, ep)) return;
  // 3. every slice of the result is now in my result area
  for (int s = 0; s < W; ++s) {
    const long long lo = s * L, hi = (s + 1) * L < n4 ? (s + 1) * L : n4;
    for (long long i = lo + (long long)b * 256 + t; i < hi; i += stride)
      reinterpret_cast<float4*>(out)[i] = reinterpret_cast<const float4*>(mine_out)[i];
  }
  if (b == 0 && t < tail) out[n4 * 4 + t] = mine_out[n4 * 4 + t];
  end_call(a, b, ep);
}

// int64 counters (BN num_batches_tracked): floor(sum / W), one workgroup.
__global__ __launch_bounds__(256) void peer_i64_mean_floor_kernel(PeerArgs a, const int64_t* in, int64_t* out,
                                                                  long long n) {
  const uint32_t ep = begin_call(a, 0);
  const int slot = ep & 1;
  int64_t* mine = reinterpret_cast<int64_t*>(region(a, a.rank, slot, 0));
  for (long long i = threadIdx.x; i < n; i += 256) mine[i] = in[i];
  if (!peer_barrier(a, 0, 0, ep)) return;
  for (long long i = threadIdx.x; i < n; i += 256) {
    int64_t s = 0;
    for (int p = 0; p < a.world; ++p) s += reinterpret_cast<const int64_t*>(region(a, p, slot, 0))[i];
    int64_t q = s / a.world;
    if ((s % a.world) != 0 && s < 0) --q;          // floor, like torch.div(..., rounding_mode="floor")
    out[i] = q;
  }
  end_call(a, 0, ep);
}

__global__ __launch_bounds__(256) void peer_allgather_kernel(PeerArgs a, const uint4* in, uint4* out, long long n16) {
  const int b = blockIdx.x, t = threadIdx.x;
  const uint32_t ep = begin_call(a, b);
  const int slot = ep & 1;
  const long long stride = (long long)gridDim.x * 256;
  uint4* mine = reinterpret_cast<uint4*>(region(a, a.rank, slot, 0));
  for (long long i = (long long)b * 256 + t; i < n16; i += stride) mine[i] = in[i];
  if (!peer_barrier(a, 0, b, ep)) return;
  for (int p = 0; p < a.world; ++p) {
    const uint4* src = reinterpret_cast<const uint4*>(region(a, p, slot, 0));
    for (long long i = (long long)b * 256 + t; i < n16; i += stride) out[(long long)p * n16 + i] = src[i];
  }
  end_call(a, b, ep);
}

// -c Y (int8 + error feedback) fused into the collective: ONE launch per FedAvg instead of delta + quantise +
// two all-gathers + dequantise-accumulate.  One WAVE owns one 256-entry chunk (4 consecutive entries per lane,
// 16-byte loads / stores, the chunk's absmax by wave shuffles only -- no workgroup barrier per chunk); block b's
// waves take chunks 4b + w, 4b + w + 4G, ... on every rank.  Phase 1: d = x - g + r, scale s = absmax / 127,
// q = rint(d / s) clamped to +-127, r <- d - q * s; q (int8) and s go to this rank's staging slot.  Peer barrier of
// block b.  Phase 2, same chunks: acc = sum over ranks 0..W-1 of q_p * s_p, g += scale * acc, x = g.  The formulas
// and the summation order are those of ef_delta / quant_int8 / dequant_accum (compress.hip), so the result is
// bit-identical to the unfused path and to every other rank.  Staging: q bytes [0, n16), scales (fp32) from n16.
// x, g, r: 16-byte aligned (the host checks); the tail chunk's lanes past n go element by element.
PDEV void i8_load4(const float* p, long long i, long long n, float v[4]) {
  if (i + 3 < n) {
    const float4 t = *reinterpret_cast<const float4*>(p + i);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = i + e < n ? p[i + e] : 0.f;
  }
}
PDEV void i8_store4(float* p, long long i, long long n, const float v[4]) {
  if (i + 3 < n) {
    *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i + e < n) p[i + e] = v[e];
  }
}

__global__ __launch_bounds__(256) void peer_int8_ef_kernel(PeerArgs a, float* __restrict__ x, float* __restrict__ g,
                                                           float* __restrict__ r, long long n, float scale) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t ep = begin_call(a, b);
  const int slot = ep & 1;
  const long long nchunks = (n + 255) >> 8, n16 = (n + 15) & ~15LL;
  const long long cstep = (long long)gridDim.x * 4;
  char* mine = region(a, a.rank, slot, 0);
  float* mys = reinterpret_cast<float*>(mine + n16);
  for (long long c = (long long)b * 4 + wave; c < nchunks; c += cstep) {
    const long long i = c * 256 + 4 * lane;
    float xv[4], gv[4], rv[4], v[4];
    i8_load4(x, i, n, xv);
    i8_load4(g, i, n, gv);
    i8_load4(r, i, n, rv);
    float am = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = i + e < n ? (xv[e] - gv[e]) + rv[e] : 0.f;
      am = fmaxf(am, fabsf(v[e]));
    }
    for (int off = 32; off > 0; off >>= 1) am = fmaxf(am, __shfl_xor(am, off, 64));
    const float sc = am > 0.f ? am / 127.f : 1.f;
    uint32_t packed = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float rq = rintf(v[e] / sc);
      const int qi = (int)fminf(fmaxf(rq, -127.f), 127.f);
      packed |= (uint32_t)(qi & 0xff) << (8 * e);
      rv[e] = v[e] - (float)qi * sc;
    }
    i8_store4(r, i, n, rv);
    if (i < n16) *reinterpret_cast<uint32_t*>(mine + i) = packed;     // (n16 % 4 == 0: whole words)
    if (lane == 0) mys[c] = sc;
  }
  if (!peer_barrier(a, 0, b, ep)) return;
  for (long long c = (long long)b * 4 + wave; c < nchunks; c += cstep) {
    const long long i = c * 256 + 4 * lane;
    if (i >= n) continue;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < a.world; ++p) {
      const char* base = region(a, p, slot, 0);
      const uint32_t qw = *reinterpret_cast<const uint32_t*>(base + i);
      const float sp = reinterpret_cast<const float*>(base + n16)[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += (float)(signed char)((qw >> (8 * e)) & 0xff) * sp;
    }
    float gv[4];
    i8_load4(g, i, n, gv);
#pragma unroll
    for (int e = 0; e < 4; ++e) gv[e] = gv[e] + scale * acc[e];
    i8_store4(g, i, n, gv);
    i8_store4(x, i, n, gv);
  }
  end_call(a, b, ep);
}

}  // namespace

namespace fedmi {

PeerComm::PeerComm(int rank, int world, long long cap_bytes) {
  if (world < 1 || world > kPeerMaxRanks) throw std::invalid_argument("PeerComm: world must be in [1, 16]");
  if (rank < 0 || rank >= world) throw std::invalid_argument("PeerComm: bad rank");
  if (cap_bytes <= 0) throw std::invalid_argument("PeerComm: capacity must be > 0");
  cap_bytes = (cap_bytes + 255) & ~255LL;
  check_hip(hipGetDevice(&device_), "hipGetDevice");
  // Both buffers are rounded up to whole 2 MiB fragments: the runtime may carve small uncached
  // allocations out of one shared block, and a later generation's buffer exported from a block
  // that an earlier (retired, still mapped) generation already exported failed with
  // hipIpcGetMemHandle: invalid argument (failover drill, third data-plane group of a client).
  constexpr size_t kFrag = 2u << 20;
  const size_t sig_bytes = (sizeof(PeerSignal) + kFrag - 1) / kFrag * kFrag;
  check_hip(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sig_bytes, hipDeviceMallocUncached),
            "PeerComm signal alloc");
  check_hip(hipMemset(sig_, 0, sizeof(PeerSignal)), "PeerComm signal memset");
  // Staging is uncached as well: the payload is read once per call by peers on other GPUs, and an
  // uncached mapping needs no cache maintenance to be coherent across xGMI.
  const size_t data_bytes = (4 * (size_t)cap_bytes + kFrag - 1) / kFrag * kFrag;
  check_hip(hipExtMallocWithFlags(reinterpret_cast<void**>(&data_), data_bytes, hipDeviceMallocUncached),
            "PeerComm staging alloc");
  check_hip(hipMemset(data_, 0, 4 * cap_bytes), "PeerComm staging memset");
  // abort word: host-pinned, coherent (device reads see host stores without any cache maintenance)
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&abort_host_), 64, hipHostMallocMapped | hipHostMallocCoherent),
            "PeerComm abort word alloc");
  *reinterpret_cast<volatile uint32_t*>(abort_host_) = 0u;
  void* abort_dev = nullptr;
  check_hip(hipHostGetDevicePointer(&abort_dev, abort_host_, 0), "PeerComm abort word device pointer");
  a_.abort_flag = reinterpret_cast<const uint32_t*>(abort_dev);
  check_hip(hipDeviceSynchronize(), "PeerComm init sync");
  a_.rank = rank;
  a_.world = world;
  a_.cap = cap_bytes;
  a_.sig[rank] = sig_;
  a_.data[rank] = data_;
  set_timeout_ms(30000.0);
}

PeerComm::~PeerComm() {
  try {
    disconnect();
  } catch (...) {
  }
  (void)hipFree(data_);
  (void)hipFree(sig_);
  (void)hipHostFree(abort_host_);
}

// Handle blob: [signal IPC handle][staging IPC handle][PCI bus id of the owner's GPU, 64 bytes].
constexpr int kBusIdLen = 64;

std::vector<uint8_t> PeerComm::handle() const {
  hipIpcMemHandle_t hs, hd;
  check_hip(hipIpcGetMemHandle(&hs, sig_), "hipIpcGetMemHandle(signal)");
  check_hip(hipIpcGetMemHandle(&hd, data_), "hipIpcGetMemHandle(staging)");
  std::vector<uint8_t> out(2 * sizeof(hipIpcMemHandle_t) + kBusIdLen, 0);
  std::memcpy(out.data(), &hs, sizeof(hs));
  std::memcpy(out.data() + sizeof(hs), &hd, sizeof(hd));
  check_hip(hipDeviceGetPCIBusId(reinterpret_cast<char*>(out.data() + 2 * sizeof(hs)), kBusIdLen - 1, device_),
            "hipDeviceGetPCIBusId");
  return out;
}

void PeerComm::connect(const std::vector<std::vector<uint8_t>>& handles) {
  if ((int)handles.size() != a_.world) throw std::invalid_argument("PeerComm::connect: need one handle per rank");
  if (connected_) return;
  check_hip(hipSetDevice(device_), "hipSetDevice");
  const size_t want = 2 * sizeof(hipIpcMemHandle_t) + kBusIdLen;
  // refuse BEFORE mapping anything when a peer's GPU is not directly addressable from ours: the
  // kernels dereference peer memory, and a missing xGMI / P2P path would fault instead of failing
  for (int p = 0; p < a_.world; ++p) {
    if (p == a_.rank) continue;
    if (handles[p].size() != want) throw std::invalid_argument("PeerComm: bad handle size");
    char bus[kBusIdLen];
    std::memcpy(bus, handles[p].data() + 2 * sizeof(hipIpcMemHandle_t), kBusIdLen);
    bus[kBusIdLen - 1] = 0;
    int dev = -1;
    check_hip(hipDeviceGetByPCIBusId(&dev, bus), "hipDeviceGetByPCIBusId");
    if (dev == device_) colocated_ = true;
    if (dev != device_) {
      int can = 0;
      check_hip(hipDeviceCanAccessPeer(&can, device_, dev), "hipDeviceCanAccessPeer");
      if (!can) throw std::runtime_error("PeerComm: GPU " + std::to_string(device_) + " cannot access peer GPU " +
                                         std::to_string(dev));
    }
  }
  for (int p = 0; p < a_.world; ++p) {
    if (p == a_.rank) continue;
    hipIpcMemHandle_t hs, hd;
    std::memcpy(&hs, handles[p].data(), sizeof(hs));
    std::memcpy(&hd, handles[p].data() + sizeof(hs), sizeof(hd));
    void* ps = nullptr;
    void* pd = nullptr;
    check_hip(hipIpcOpenMemHandle(&ps, hs, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(signal)");
    check_hip(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(staging)");
    a_.sig[p] = reinterpret_cast<PeerSignal*>(ps);
    a_.data[p] = reinterpret_cast<char*>(pd);
  }
  connected_ = true;
}

void PeerComm::disconnect() {
  if (!connected_) return;
  (void)hipDeviceSynchronize();
  for (int p = 0; p < a_.world; ++p) {
    if (p == a_.rank) continue;
    if (a_.sig[p]) (void)hipIpcCloseMemHandle(a_.sig[p]);
    if (a_.data[p]) (void)hipIpcCloseMemHandle(a_.data[p]);
    a_.sig[p] = nullptr;
    a_.data[p] = nullptr;
  }
  connected_ = false;
}

void PeerComm::set_timeout_ms(double ms) { a_.timeout_ticks = (long long)(ms * 1e5); }  // 100 MHz realtime clock

uint32_t PeerComm::error() const {
  uint32_t e = 0;
  check_hip(hipMemcpy(&e, &sig_->error, sizeof(e), hipMemcpyDeviceToHost), "PeerComm::error");
  return e;
}

std::vector<uint32_t> PeerComm::epochs() const {
  std::vector<uint32_t> e(kPeerMaxBlocks);
  check_hip(hipMemcpy(e.data(), sig_->epoch, sizeof(uint32_t) * kPeerMaxBlocks, hipMemcpyDeviceToHost),
            "PeerComm::epochs");
  return e;
}

void PeerComm::request_abort() {
  __atomic_store_n(abort_host_, 1u, __ATOMIC_RELEASE);
}

bool PeerComm::abort_requested() const { return __atomic_load_n(abort_host_, __ATOMIC_ACQUIRE) != 0u; }

void PeerComm::clear_error() { check_hip(hipMemset(&sig_->error, 0, sizeof(uint32_t)), "PeerComm::clear_error"); }

int PeerComm::default_blocks(long long bytes, int algo, int world) {
  long long g4 = bytes / 16;                         // float4 granules
  if (algo == kPeerTwoShot) g4 = (g4 + world - 1) / world;
  long long b = (g4 + 255) / 256;
  if (b < 1) b = 1;
  if (b > 128) b = 128;
  return (int)b;
}

static void need(bool ok, const char* msg) {
  if (!ok) throw std::invalid_argument(msg);
}

void PeerComm::allreduce_f32(hipStream_t st, const float* in, float* out, long long n, float scale, int algo,
                             int blocks) {
  need(connected_ || a_.world == 1, "PeerComm: not connected");
  need(n >= 0 && n * 4 <= a_.cap, "PeerComm::allreduce_f32: payload exceeds capacity");
  need((reinterpret_cast<uintptr_t>(in) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0,
       "PeerComm::allreduce_f32: buffers must be 16-byte aligned");
  if (n == 0) return;
  if (blocks <= 0) blocks = default_blocks(n * 4, algo, a_.world);
  need(blocks <= kPeerMaxBlocks, "PeerComm: too many blocks");
  if (algo == kPeerTwoShot)
    hipLaunchKernelGGL(peer_twoshot_f32_kernel, dim3(blocks), dim3(256), 0, st, a_, in, out, n, scale);
  else
    hipLaunchKernelGGL(peer_oneshot_f32_kernel, dim3(blocks), dim3(256), 0, st, a_, in, out, n, scale);
  check_hip(hipGetLastError(), "peer allreduce_f32 launch");
}

void PeerComm::allreduce_int8_ef(hipStream_t st, float* x, float* g, float* r, long long n, float scale, int blocks) {
  need(connected_ || a_.world == 1, "PeerComm: not connected");
  const long long nchunks = (n + 255) / 256, n16 = (n + 15) & ~15LL;
  need(n >= 0 && n16 + 4 * nchunks <= a_.cap, "PeerComm::allreduce_int8_ef: payload exceeds capacity");
  if (n == 0) return;
  need(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(r)) & 15) == 0,
       "PeerComm::allreduce_int8_ef: x, g, r must be 16-byte aligned");
  if (blocks <= 0) blocks = (int)std::min<long long>((nchunks + 3) / 4, kPeerMaxBlocks);   // a chunk per wave
  need(blocks <= kPeerMaxBlocks, "PeerComm: too many blocks");
  hipLaunchKernelGGL(peer_int8_ef_kernel, dim3(blocks), dim3(256), 0, st, a_, x, g, r, n, scale);
  check_hip(hipGetLastError(), "peer int8_ef launch");
}

void PeerComm::allreduce_i64_mean_floor(hipStream_t st, const int64_t* in, int64_t* out, long long n) {
  need(connected_ || a_.world == 1, "PeerComm: not connected");
  need(n >= 0 && n * 8 <= a_.cap, "PeerComm::allreduce_i64: payload exceeds capacity");
  if (n == 0) return;
  hipLaunchKernelGGL(peer_i64_mean_floor_kernel, dim3(1), dim3(256), 0, st, a_, in, out, n);
  check_hip(hipGetLastError(), "peer allreduce_i64 launch");
}

void PeerComm::allgather(hipStream_t st, const void* in, void* out, long long nbytes, int blocks) {
  need(connected_ || a_.world == 1, "PeerComm: not connected");
  need(nbytes >= 0 && nbytes <= a_.cap && nbytes % 16 == 0, "PeerComm::allgather: bad size (<= cap, % 16)");
  need((reinterpret_cast<uintptr_t>(in) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0,
       "PeerComm::allgather: buffers must be 16-byte aligned");
  if (nbytes == 0) return;
  if (blocks <= 0) blocks = default_blocks(nbytes * a_.world, kPeerOneShot, a_.world);
  need(blocks <= kPeerMaxBlocks, "PeerComm: too many blocks");
  hipLaunchKernelGGL(peer_allgather_kernel, dim3(blocks), dim3(256), 0, st, a_, reinterpret_cast<const uint4*>(in),
                     reinterpret_cast<uint4*>(out), nbytes / 16);
  check_hip(hipGetLastError(), "peer allgather launch");
}

}  // namespace fedmi
