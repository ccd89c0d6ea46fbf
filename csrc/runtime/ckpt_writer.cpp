// fedmi — native per-round checkpoint writer (see ckpt_writer.h).
#include "runtime/ckpt_writer.h"

#include <fcntl.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace fedmi {
void check_hip(hipError_t e, const char* what);
uint32_t crc32_fast(uint32_t crc, const uint8_t* p, size_t n);   // crc32_fast.cpp (PCLMULQDQ folding)

namespace {

void put_u32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

// Write all of `data` to `path` atomically: tmp file in the same directory, then rename.
std::string tmp_name(const std::string& path) { return path + ".tmpn" + std::to_string(::getpid()); }

void write_tmp(const std::string& tmp, const uint8_t* data, size_t n) {
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("ckpt writer: cannot open " + tmp);
  size_t off = 0;
  while (off < n) {
    const ssize_t w = ::write(fd, data + off, n - off);
    if (w < 0) {
      ::close(fd);
      ::unlink(tmp.c_str());
      throw std::runtime_error("ckpt writer: write failed for " + tmp);
    }
    off += (size_t)w;
  }
  if (::close(fd) != 0) throw std::runtime_error("ckpt writer: close failed for " + tmp);
}

void commit(const std::string& tmp, const std::string& path) {
  if (::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("ckpt writer: rename to " + path);
}

}  // namespace

CkptWriter::CkptWriter(std::vector<uint8_t> tmpl, std::vector<CkptSegment> segs, std::vector<CkptRecord> recs,
                       long long epoch_at, std::vector<std::string> paths, bool device, int slots, bool coalesce,
                       bool link)
    : tmpl_(std::move(tmpl)), segs_(std::move(segs)), recs_(std::move(recs)), epoch_at_(epoch_at),
      paths_(std::move(paths)), device_(device), coalesce_(coalesce), link_(link) {
  const long long n = (long long)tmpl_.size();
  if (slots < 1 || slots > 64) throw std::invalid_argument("CkptWriter: slots must be in [1, 64]");
  if (epoch_at_ < 0 || epoch_at_ + 4 > n) throw std::invalid_argument("CkptWriter: epoch offset outside template");
  for (const auto& s : segs_) {
    if (s.bytes < 0 || s.snap_off < 0) throw std::invalid_argument("CkptWriter: bad segment");
    snap_bytes_ = std::max(snap_bytes_, s.snap_off + s.bytes);
  }
  for (const auto& r : recs_) {
    if (r.data_off < 0 || r.bytes < 0 || r.data_off + r.bytes > n) throw std::invalid_argument("CkptWriter: record");
    if (r.snap_off >= 0 && r.snap_off + r.bytes > snap_bytes_) throw std::invalid_argument("CkptWriter: record src");
    for (long long c : r.crc_at)
      if (c < 0 || c + 4 > n) throw std::invalid_argument("CkptWriter: CRC offset outside template");
  }
  if (paths_.empty()) throw std::invalid_argument("CkptWriter: no target paths");
  const size_t sb = (size_t)std::max(snap_bytes_, 16LL);
  snap_.assign(slots, nullptr);
  ev_.assign(slots, nullptr);
  epoch_.assign(slots, 0);
  for (int i = 0; i < slots; ++i) {
    if (device_) {
      check_hip(hipHostMalloc(reinterpret_cast<void**>(&snap_[i]), sb, hipHostMallocDefault), "CkptWriter pinned");
      check_hip(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "CkptWriter event");
    } else {
      snap_[i] = new uint8_t[sb];
    }
    free_.push_back(slots - 1 - i);
  }
  out_ = tmpl_;
  th_ = std::thread([this] { run(); });
}

CkptWriter::~CkptWriter() {
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return (queue_.empty() && busy_ < 0) || !err_.empty(); });
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  for (size_t i = 0; i < snap_.size(); ++i) {
    if (device_) {
      if (ev_[i]) (void)hipEventDestroy(ev_[i]);
      if (snap_[i]) (void)hipHostFree(snap_[i]);
    } else {
      delete[] snap_[i];
    }
  }
}

void CkptWriter::submit(hipStream_t st, int32_t epoch) {
  std::unique_lock<std::mutex> lk(mu_);
  if (!err_.empty()) throw std::runtime_error("checkpoint writer failed: " + err_);
  ++submitted_;
  int slot;
  if (free_.empty() && coalesce_ && !queue_.empty()) {
    // every slot taken: supersede the newest queued snapshot (the writer has not touched it; this
    // copy is stream-ordered after the one it replaces)
    slot = queue_.back();
    ++coalesced_;
  } else {
    cv_.wait(lk, [this] { return !free_.empty() || !err_.empty(); });
    if (!err_.empty()) throw std::runtime_error("checkpoint writer failed: " + err_);
    slot = free_.back();
    free_.pop_back();
    queue_.push_back(slot);
  }
  // the copy is issued under the lock: the writer cannot pick the slot up before its event is recorded
  for (const auto& s : segs_) {
    if (s.bytes == 0) continue;
    if (device_)
      check_hip(hipMemcpyAsync(snap_[slot] + s.snap_off, reinterpret_cast<const void*>(s.src), (size_t)s.bytes,
                               hipMemcpyDeviceToHost, st),
                "CkptWriter snapshot copy");
    else
      std::memcpy(snap_[slot] + s.snap_off, reinterpret_cast<const void*>(s.src), (size_t)s.bytes);
  }
  if (device_) check_hip(hipEventRecord(ev_[slot], st), "CkptWriter event record");
  epoch_[slot] = epoch;
  lk.unlock();
  cv_.notify_all();
}

void CkptWriter::write_one(int slot, int32_t epoch) {
  if (device_) {
    // poll instead of hipEventSynchronize: a writer thread blocked inside the runtime's event wait was
    // measured stalling the round loop's own launches/copies on the main thread (host 1.15 ms per
    // submit at the 8-client LeNet cadence, profiles/r4_scale/README.md)
    for (;;) {
      const hipError_t q = hipEventQuery(ev_[slot]);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) check_hip(q, "CkptWriter snapshot wait");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  uint8_t* o = out_.data();
  put_u32(o + epoch_at_, (uint32_t)epoch);        // pickle BININT ('J' + int32 LE)
  for (const auto& r : recs_) {
    if (r.snap_off >= 0) std::memcpy(o + r.data_off, snap_[slot] + r.snap_off, (size_t)r.bytes);
    const uint32_t crc = crc32_fast(0u, o + r.data_off, (size_t)r.bytes);
    for (long long c : r.crc_at) put_u32(o + c, crc);
  }
  // Default: every target is its own file (tmp + atomic rename), so a peer that rewrites one of them in
  // place (the reference's torch.save, src/server.py:179, src/main.py:165) never touches another.  With
  // link_ (opt-in, for target sets in directories fedmi owns alone) the bytes are written ONCE and every
  // further target is a hard link to that file, committed by its own rename; a link that fails (another
  // filesystem) falls back to a copy.  Stale temp names are unlinked first: a temp left behind by a failed
  // round may share an inode with a committed target, and O_TRUNC on it would rewrite that file in place.
  const std::string first = tmp_name(paths_[0]);
  ::unlink(first.c_str());
  write_tmp(first, o, out_.size());
  for (size_t i = 1; i < paths_.size(); ++i) {
    const std::string t = tmp_name(paths_[i]);
    ::unlink(t.c_str());
    if (!link_ || ::link(first.c_str(), t.c_str()) != 0) write_tmp(t, o, out_.size());
    commit(t, paths_[i]);
  }
  commit(first, paths_[0]);
}

void CkptWriter::run() {
  for (;;) {
    int slot;
    int32_t epoch;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return !queue_.empty() || stop_; });
      if (queue_.empty()) return;
      slot = queue_.front();
      queue_.pop_front();
      epoch = epoch_[slot];
      busy_ = slot;
    }
    std::string e;
    try {
      write_one(slot, epoch);
    } catch (const std::exception& ex) {
      e = ex.what();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      busy_ = -1;
      free_.push_back(slot);
      if (e.empty())
        written_ += (long long)paths_.size();
      else
        err_ = e;
    }
    cv_.notify_all();
  }
}

void CkptWriter::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [this] { return (queue_.empty() && busy_ < 0) || !err_.empty(); });
  if (!err_.empty()) throw std::runtime_error("checkpoint writer failed: " + err_);
}

long long CkptWriter::written() const {
  std::lock_guard<std::mutex> lk(mu_);
  return written_;
}
long long CkptWriter::coalesced() const {
  std::lock_guard<std::mutex> lk(mu_);
  return coalesced_;
}
long long CkptWriter::submitted() const {
  std::lock_guard<std::mutex> lk(mu_);
  return submitted_;
}
std::vector<uint8_t> CkptWriter::last_file() const {
  std::lock_guard<std::mutex> lk(mu_);
  return out_;
}

}  // namespace fedmi
