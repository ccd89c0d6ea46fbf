// fedmi — intra-node peer-to-peer collectives over hipIpc mappings (xGMI).
//
// FedAvg of a LeNet-sized model is a 248 KB all-reduce: far below the size at
// which a ring collective is bandwidth-bound (~3 µs of link
// time at 8 GPUs), so the RCCL launch/protocol floor dominates.  PeerComm maps
// every rank's staging buffer into every other rank's address space once
// (hipIpcGetMemHandle / hipIpcOpenMemHandle) and then runs each collective as
// ONE kernel: a flag-guarded barrier between the same workgroup index of all
// ranks, then direct loads from all peers over all xGMI links at once.
//
//   oneshot  all-reduce: every rank reads the whole payload from every peer
//            (one barrier; best for tiny payloads).
//   twoshot  all-reduce: rank r reduces slice r (pull from all peers), pushes
//            the reduced slice into every peer's result area, barrier, copy out
//            (two barriers; 1/W of the reads of oneshot per rank).
//   allgather: rank r's payload lands in slot r of every rank's output.
//
// The reduction order is rank 0..W-1 on every rank, so every rank computes
// bit-identical results (the reference averages on one CPU, src/server.py:163-171;
// a per-rank atomic order would let clients drift apart).
//
// Replaces the reference's gRPC gather + CPU average + SendModel broadcast
// (src/server.py:51-75, 155-179) on the data plane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace fedmi {

constexpr int kPeerMaxRanks = 16;    // one GPU box allows <=16 GPU processes; a node has 8 GPUs
constexpr int kPeerMaxBlocks = 256;  // one workgroup per CU at most

// Lives in UNCACHED device memory (hipDeviceMallocUncached), one per rank,
// mapped by every peer.  flags[phase][block][src] is written by rank `src`.
struct PeerSignal {
  uint32_t flags[2][kPeerMaxBlocks][kPeerMaxRanks];
  uint32_t epoch[kPeerMaxBlocks];   // per-workgroup call counter (device-side: graph-capturable)
  uint32_t error;                   // set when a barrier timed out (a peer died or never arrived)
  uint32_t pad[63];
};

struct PeerArgs {
  PeerSignal* sig[kPeerMaxRanks];   // sig[p]: rank p's signal block (own one at [rank])
  char* data[kPeerMaxRanks];        // data[p]: rank p's staging buffer: [2 slots][2 regions][cap]
  int rank;
  int world;
  long long cap;                    // bytes per region
  long long timeout_ticks;          // s_memrealtime ticks (100 MHz)
  const uint32_t* abort_flag;       // host-pinned coherent word (device view): nonzero = the coordinator
                                    // reported a lost client, every barrier of this communicator fails now
};

enum PeerAlgo { kPeerOneShot = 0, kPeerTwoShot = 1 };

class PeerComm {
 public:
  PeerComm(int rank, int world, long long cap_bytes);
  ~PeerComm();
  PeerComm(const PeerComm&) = delete;
  PeerComm& operator=(const PeerComm&) = delete;

  // 2 x sizeof(hipIpcMemHandle_t) bytes: signal handle, staging handle.
  std::vector<uint8_t> handle() const;
  // handles[p] from every rank (own entry ignored); maps the peers.
  void connect(const std::vector<std::vector<uint8_t>>& handles);
  bool connected() const { return connected_; }
  // some peer runs on THIS GPU (one-GPU rehearsals): its kernels share our hardware queues, so a
  // barrier kernel spinning here can starve a peer that has not launched yet (callers then gate
  // each collective with a host-side barrier)
  bool colocated() const { return colocated_; }

  // out = scale * sum_p in_p  (fp32; in == out allowed)
  void allreduce_f32(hipStream_t st, const float* in, float* out, long long n, float scale, int algo, int blocks);
  // -c Y int8 + error feedback in ONE launch: d = x - g + r quantised per 256-chunk (r <- quantisation error),
  // g += scale * sum_p deq(q_p), x = g  (bit-identical to ef_delta + quant_int8 + all-gathers + dequant_accum)
  void allreduce_int8_ef(hipStream_t st, float* x, float* g, float* r, long long n, float scale, int blocks);
  // out = floor(sum_p in_p / world)  (int64 BN counters: reference float mean + int64 truncation)
  void allreduce_i64_mean_floor(hipStream_t st, const int64_t* in, int64_t* out, long long n);
  // out[p * nbytes .. ) = in_p  (nbytes % 16 == 0)
  void allgather(hipStream_t st, const void* in, void* out, long long nbytes, int blocks);

  uint32_t error() const;           // synchronous read of the timeout flag
  // Host-side abort (a watchdog thread, while a collective may be spinning on the stream): a plain store
  // into host-pinned coherent memory the barrier polls -- no stream, no HIP call, never blocks.  Sticky:
  // the communicator belongs to one data-plane generation, which the coordinator replaces after a loss.
  void request_abort();
  bool abort_requested() const;
  std::vector<uint32_t> epochs() const;   // synchronous read of the per-block call counters (tests)
  void clear_error();
  void set_timeout_ms(double ms);
  void disconnect();                // unmap peers (call after a host-side barrier)

  int rank() const { return a_.rank; }
  int world() const { return a_.world; }
  long long capacity() const { return a_.cap; }
  static int default_blocks(long long bytes, int algo, int world);

 private:
  PeerArgs a_{};
  PeerSignal* sig_ = nullptr;       // own (uncached)
  char* data_ = nullptr;            // own staging
  uint32_t* abort_host_ = nullptr;  // host-pinned abort word (a_.abort_flag is its device view)
  bool connected_ = false;
  bool colocated_ = false;
  int device_ = 0;
};

}  // namespace fedmi
