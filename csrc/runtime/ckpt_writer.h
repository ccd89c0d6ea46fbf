// fedmi — native per-round checkpoint writer (no Python, no GIL on the write path).
//
// The reference writes a torch.save checkpoint every round on every client and the
// averaged model on the coordinator (src/main.py:160-165, src/server.py:174-179).
// At 8 GPU-clients a LeNet round is ~1.3 ms; a Python writer thread that pickles
// and writes every round holds the GIL for about that long and stalls the round
// loop's launches (tools/bench_ckpt_writer.py).  This writer does the whole job in
// a C++ thread:
//
//   * the file is a TEMPLATE: torch.save's zip archive of the state dict, made once
//     by Python with a sentinel epoch, parsed there into record offsets.  Every
//     record is stored uncompressed (zip method 0), so a new checkpoint is the
//     template with the storage bytes replaced, the 4-byte pickled epoch patched,
//     and the CRC-32s of the changed records rewritten (data descriptor + central
//     directory) -- byte-for-byte what torch.save would have written.
//   * submit(): ONE async device->pinned-host copy per source storage on the
//     caller's stream + an event, into a free slot of a ring of `slots` pinned
//     snapshot buffers.  It never waits for the GPU or for I/O while a slot is free.
//   * every submission is written, in order (the reference writes every round).  A
//     host running more than `slots` rounds ahead of the writer waits for a slot --
//     the GPU queue then already holds that many rounds of work.  Optional
//     coalescing (`coalesce`): with every slot taken, a submission replaces the
//     newest queued one instead of waiting (the files hold the newest model either
//     way); the coordinator-side persister works like that.
//   * the writer thread waits for the event, assembles the archive, CRCs it and
//     writes every target path atomically (tmp file + rename).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace fedmi {

struct CkptSegment {     // one source storage span -> snapshot buffer
  uintptr_t src;         // device pointer (device mode) or host pointer (host mode)
  long long bytes;
  long long snap_off;    // offset inside a snapshot buffer
};

struct CkptRecord {      // one zip record whose bytes change per checkpoint
  long long data_off;    // file offset of the record's data
  long long bytes;
  long long snap_off;    // -1: not a storage (data.pkl: bytes come from the template)
  std::vector<long long> crc_at;   // file offsets of this record's CRC-32 fields
};

class CkptWriter {
 public:
  // device: true = segments are device pointers copied on a stream (pinned snapshots);
  //         false = host pointers copied synchronously (CPU hosts / tests).
  CkptWriter(std::vector<uint8_t> tmpl, std::vector<CkptSegment> segs, std::vector<CkptRecord> recs,
             long long epoch_at, std::vector<std::string> paths, bool device, int slots = 4, bool coalesce = false,
             bool link = false);   // link: extra targets are hard links to the first (opt-in, see write_one)
  ~CkptWriter();
  CkptWriter(const CkptWriter&) = delete;
  CkptWriter& operator=(const CkptWriter&) = delete;

  void submit(hipStream_t st, int32_t epoch);
  void flush();                     // newest submission on disk (or throws the writer's error)
  long long written() const;        // files written
  long long coalesced() const;      // submissions superseded before being written
  long long submitted() const;
  std::vector<uint8_t> last_file() const;   // bytes of the last archive written (tests)

 private:
  void run();
  void write_one(int buf, int32_t epoch);

  std::vector<uint8_t> tmpl_, out_;
  std::vector<CkptSegment> segs_;
  std::vector<CkptRecord> recs_;
  long long epoch_at_;
  std::vector<std::string> paths_;
  bool device_;
  bool coalesce_;
  bool link_;
  long long snap_bytes_ = 0;
  std::vector<uint8_t*> snap_;
  std::vector<hipEvent_t> ev_;
  std::vector<int32_t> epoch_;           // epoch of the snapshot in each slot

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::vector<int> free_;                // free slots
  std::deque<int> queue_;                // submitted, not yet picked up (FIFO)
  int busy_ = -1;                        // slot the writer is reading
  bool stop_ = false;
  std::string err_;
  long long written_ = 0, coalesced_ = 0, submitted_ = 0;
  std::thread th_;
};

}  // namespace fedmi
