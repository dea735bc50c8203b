// Asynchronous checkpoint engine core (header-only host C++; HIP runtime API for the D2H
// staging, no torch / pybind dependency so it can be unit-tested and sanitized standalone:
// tests/native/ckpt_engine_selftest.cpp). Python bindings: ckpt_engine.cpp.
//
// Replaces the reference's synchronous `torch.save` + whole-file re-read md5
// (reference pyrecover/checkpoint.py:58-84) with:
//   1. staging: device buffers -> a reusable pinned host pool (hipHostMalloc) via chunked
//      hipMemcpyAsync on a dedicated LOW-priority HIP stream that first waits on the caller's
//      compute stream; each 256 MiB chunk records a hipEvent. `fence()` makes the compute
//      stream wait (GPU-side, no host block) for the snapshot before the optimizer mutates
//      the parameters again.
//   2. a background writer thread that emits a torch.save-compatible zip archive
//      (stored records, 64-B aligned payloads, ZIP64 when needed, CRC32 patched into the
//      local headers) while each chunk's D2H lands, computing the CRC32 in parallel pieces
//      and the whole-file MD5 on a pipelined hashing thread. The archive is written to
//      `<path>.tmp`, fsync'ed and renamed, so a crash never leaves a torn "latest" file;
//      the `.md5` sidecar (32 hex chars, no newline, same as the reference) is written the
//      same way.
// The pickle stream itself is produced by torch's own serializer in Python (so the archive
// is byte-compatible with what torch.load expects); this engine only moves bytes.
#pragma once
#include <hip/hip_runtime_api.h>

#include <openssl/evp.h>
#include <zlib.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace pra {
namespace ckpt {


inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ckpt_engine: ") + what + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------------------------------------
// MD5 on its own thread, fed in file order.
class Md5Pipe {
 public:
  Md5Pipe() : ctx_(EVP_MD_CTX_new()) {
    EVP_DigestInit_ex(ctx_, EVP_md5(), nullptr);
    th_ = std::thread([this] { run(); });
  }
  ~Md5Pipe() {
    finish();
    EVP_MD_CTX_free(ctx_);
  }
  // `owned` payloads are copied; borrowed pointers must stay valid until finish().
  void push_copy(const void* p, size_t n) {
    auto buf = std::make_shared<std::vector<uint8_t>>((const uint8_t*)p, (const uint8_t*)p + n);
    enqueue({buf->data(), n, buf});
  }
  void push_borrowed(const void* p, size_t n) { enqueue({(const uint8_t*)p, n, nullptr}); }
  std::string finish() {
    if (th_.joinable()) {
      {
        std::lock_guard<std::mutex> g(mu_);
        done_ = true;
      }
      cv_.notify_all();
      th_.join();
      unsigned char dig[EVP_MAX_MD_SIZE];
      unsigned int len = 0;
      EVP_DigestFinal_ex(ctx_, dig, &len);
      static const char* hex = "0123456789abcdef";
      hexd_.clear();
      for (unsigned i = 0; i < len; ++i) {
        hexd_.push_back(hex[dig[i] >> 4]);
        hexd_.push_back(hex[dig[i] & 15]);
      }
    }
    return hexd_;
  }

 private:
  struct Item {
    const uint8_t* p;
    size_t n;
    std::shared_ptr<std::vector<uint8_t>> keep;
  };
  void enqueue(Item it) {
    std::unique_lock<std::mutex> g(mu_);
    cv_space_.wait(g, [&] { return q_.size() < 64; });
    q_.push_back(std::move(it));
    cv_.notify_one();
  }
  void run() {
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return done_ || !q_.empty(); });
        if (q_.empty()) return;
        it = std::move(q_.front());
        q_.pop_front();
        cv_space_.notify_one();
      }
      EVP_DigestUpdate(ctx_, it.p, it.n);
    }
  }
  EVP_MD_CTX* ctx_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_, cv_space_;
  std::deque<Item> q_;
  bool done_ = false;
  std::string hexd_;
};

inline uint32_t crc32_parallel(uint32_t crc, const uint8_t* p, size_t n) {
  constexpr size_t kPiece = 16u << 20;
  if (n <= kPiece) return (uint32_t)crc32_z(crc, p, n);
  const size_t np = (n + kPiece - 1) / kPiece;
  std::vector<std::future<uint32_t>> fut;
  std::vector<size_t> len(np);
  for (size_t i = 0; i < np; ++i) {
    const size_t off = i * kPiece;
    len[i] = std::min(kPiece, n - off);
    fut.push_back(std::async(std::launch::async, [p, off, l = len[i]] { return (uint32_t)crc32_z(0, p + off, l); }));
  }
  for (size_t i = 0; i < np; ++i) crc = (uint32_t)crc32_combine(crc, fut[i].get(), (z_off_t)len[i]);
  return crc;
}

inline void put16(std::vector<uint8_t>& b, uint16_t v) { b.push_back(v & 0xff); b.push_back(v >> 8); }
inline void put32(std::vector<uint8_t>& b, uint32_t v) { for (int i = 0; i < 4; ++i) b.push_back((v >> (8 * i)) & 0xff); }
inline void put64(std::vector<uint8_t>& b, uint64_t v) { for (int i = 0; i < 8; ++i) b.push_back((v >> (8 * i)) & 0xff); }

struct Record {
  std::string name;
  uintptr_t ptr;
  uint64_t nbytes;
};

// One file = a sequence of items: a zip archive built from records, or raw bytes copied verbatim.
struct Item {
  bool raw = false;
  uintptr_t ptr = 0;  // raw
  uint64_t n = 0;     // raw
  std::vector<Record> records;  // zip
};

struct Chunk {
  uintptr_t host;  // host address
  uint64_t n;
  hipEvent_t ev;
};

struct JobResult {
  bool ok = false;
  std::string error;
  std::string md5;
  uint64_t bytes = 0;
  double seconds = 0;
  double stage_wait_seconds = 0;
  std::vector<std::pair<uint64_t, uint64_t>> items;  // (offset, length) of each item in the file
};

// Streaming MD5 of an open file from its start (double-buffered reads on this thread, hashing
// on the Md5Pipe thread).
inline std::string md5_fd(int fd) {
  Md5Pipe md5;
  constexpr size_t kBuf = 32u << 20;
  uint64_t pos = 0;
  for (;;) {
    auto buf = std::make_shared<std::vector<uint8_t>>(kBuf);
    ssize_t n;
    do {
      n = ::pread(fd, buf->data(), kBuf, (off_t)pos);
    } while (n < 0 && errno == EINTR);
    if (n < 0) throw std::runtime_error("md5: read failed");
    if (n == 0) break;
    md5.push_copy(buf->data(), (size_t)n);
    pos += (uint64_t)n;
  }
  return md5.finish();
}

// ------------------------------------------------------------------------------------------
class CkptEngine {
 public:
  // device < 0: CPU mode (no HIP calls; regions are host pointers copied with memcpy).
  explicit CkptEngine(int device) : device_(device) {
    if (device_ < 0) return;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    // numerically larger = lower priority on HIP
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, lo), "stream create");
    hip_check(hipEventCreateWithFlags(&entry_ev_, hipEventDisableTiming), "event create");
  }
  ~CkptEngine() {
    try {
      wait_writer();
    } catch (...) {
    }
    release_chunks();
    free_pool();
    if (device_ >= 0) {
      (void)hipEventDestroy(entry_ev_);
      (void)hipStreamDestroy(stream_);
    }
  }

  // Ensure the pinned pool holds at least nbytes (must not be called while a job runs).
  void reserve(uint64_t nbytes) {
    wait_writer();
    if (nbytes <= pool_size_) return;
    release_chunks();
    free_pool();
    if (device_ >= 0) {
      hip_check(hipSetDevice(device_), "hipSetDevice");
      hip_check(hipHostMalloc(&pool_, nbytes, hipHostMallocDefault), "hipHostMalloc");
    } else {
      if (posix_memalign(&pool_, 4096, nbytes) != 0) throw std::runtime_error("ckpt_engine: host alloc failed");
    }
    pool_size_ = nbytes;
  }
  int device() const { return device_; }
  uintptr_t pool_ptr() const { return (uintptr_t)pool_; }
  uint64_t pool_size() const { return pool_size_; }

  // Enqueue D2H copies of (dev_ptr, nbytes) regions into the pool, packed at 64-B aligned
  // offsets. Returns the host offsets. Ordered after all work already queued on `cur` (the
  // caller's compute stream; ignored in CPU mode).
  std::vector<uint64_t> stage(const std::vector<std::pair<uintptr_t, uint64_t>>& regions, hipStream_t cur) {
    wait_writer();  // the pool is reused: the previous archive must be fully written
    release_chunks();
    uint64_t total = 0;
    std::vector<uint64_t> offs;
    for (auto& r : regions) {
      total = (total + 63) & ~uint64_t(63);
      offs.push_back(total);
      total += r.second;
    }
    if (total > pool_size_) throw std::runtime_error("ckpt_engine: pinned pool too small; call reserve()");
    if (device_ < 0) {  // CPU mode: parallel memcpy snapshot
      std::vector<std::future<void>> fut;
      for (size_t i = 0; i < regions.size(); ++i) {
        constexpr uint64_t kPiece = 64ull << 20;
        for (uint64_t o = 0; o < regions[i].second; o += kPiece) {
          const uint64_t n = std::min(kPiece, regions[i].second - o);
          uint8_t* dst = (uint8_t*)pool_ + offs[i] + o;
          const uint8_t* src = (const uint8_t*)regions[i].first + o;
          fut.push_back(std::async(std::launch::async, [dst, src, n] { std::memcpy(dst, src, n); }));
          if (fut.size() >= 8) { for (auto& f : fut) f.get(); fut.clear(); }
        }
      }
      for (auto& f : fut) f.get();
      staged_bytes_ = total;
      return offs;
    }
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipEventRecord(entry_ev_, cur), "event record");
    hip_check(hipStreamWaitEvent(stream_, entry_ev_, 0), "stream wait");
    constexpr uint64_t kChunk = 256ull << 20;
    for (size_t i = 0; i < regions.size(); ++i) {
      const uint8_t* src = (const uint8_t*)regions[i].first;
      uint8_t* dst = (uint8_t*)pool_ + offs[i];
      for (uint64_t o = 0; o < regions[i].second; o += kChunk) {
        const uint64_t n = std::min(kChunk, regions[i].second - o);
        hip_check(hipMemcpyAsync(dst + o, src + o, n, hipMemcpyDeviceToHost, stream_), "hipMemcpyAsync");
        hipEvent_t ev;
        hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event create");
        hip_check(hipEventRecord(ev, stream_), "event record");
        chunks_.push_back({(uintptr_t)(dst + o), n, ev});
      }
    }
    staged_bytes_ = total;
    return offs;
  }

  // GPU-side fence: `cur` (the caller's compute stream) waits for the whole snapshot, so the
  // next optimizer step cannot overwrite parameters that are still being copied out.
  void fence(hipStream_t cur) {
    if (device_ < 0 || chunks_.empty()) return;
    hip_check(hipStreamWaitEvent(cur, chunks_.back().ev, 0), "fence");
  }
  // Host-side: block until the snapshot has fully landed in host memory.
  void sync_stage() {
    if (!chunks_.empty()) hip_check(hipEventSynchronize(chunks_.back().ev), "event sync");
  }
  // Debug assertion support: true when every staged chunk has landed (hipEventQuery).
  bool staged_complete() const {
    for (auto& c : chunks_)
      if (hipEventQuery(c.ev) != hipSuccess) return false;
    return true;
  }

  // Start writing a zip archive on the background thread. Records point into the pinned pool
  // (waited per chunk) or into caller-owned host memory kept alive until wait().
  void write_items(const std::string& path, std::vector<Item> items, bool want_md5, bool do_fsync) {
    wait_writer();
    running_ = true;
    result_ = JobResult{};
    writer_ = std::thread([this, path, items = std::move(items), want_md5, do_fsync]() mutable {
      JobResult r;
      const auto t0 = std::chrono::steady_clock::now();
      try {
        write_impl(path, items, want_md5, do_fsync, r);
        r.ok = true;
      } catch (const std::exception& e) {
        r.ok = false;
        r.error = e.what();
        ::unlink((path + ".tmp").c_str());
      }
      r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      {
        std::lock_guard<std::mutex> g(mu_);
        result_ = r;
        running_ = false;
      }
    });
  }

  bool busy() {
    std::lock_guard<std::mutex> g(mu_);
    return running_;
  }

  JobResult wait() {
    wait_writer();
    return result_;
  }

 private:
  void wait_writer() {
    if (writer_.joinable()) writer_.join();
  }
  void free_pool() {
    if (!pool_) return;
    if (device_ >= 0) (void)hipHostFree(pool_);
    else ::free(pool_);
    pool_ = nullptr;
    pool_size_ = 0;
  }
  void release_chunks() {
    for (auto& c : chunks_) {
      (void)hipEventSynchronize(c.ev);
      (void)hipEventDestroy(c.ev);
    }
    chunks_.clear();
  }
  // wait for every staging chunk overlapping [p, p+n)
  void wait_range(uintptr_t p, uint64_t n, JobResult& r) {
    const uintptr_t lo = (uintptr_t)pool_, hi = lo + pool_size_;
    if (device_ < 0 || p + n <= lo || p >= hi) return;
    for (auto& c : chunks_) {
      if (c.host < p + n && c.host + c.n > p) {
        if (hipEventQuery(c.ev) != hipSuccess) {
          const auto t0 = std::chrono::steady_clock::now();
          hip_check(hipEventSynchronize(c.ev), "event sync");
          r.stage_wait_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
      }
    }
  }

  static void write_all(int fd, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    while (n) {
      const ssize_t w = ::write(fd, b, std::min<size_t>(n, 1u << 30));
      if (w < 0) {
        if (errno == EINTR) continue;
        throw std::runtime_error(std::string("ckpt_engine: write failed: ") + strerror(errno));
      }
      b += w;
      n -= (size_t)w;
    }
  }

  // Emit one zip archive (offsets inside it are relative to `base`, the archive's first byte).
  template <class Emit>
  void emit_zip(std::vector<Record>& recs, uint64_t& off, const uint64_t base, int fd, Md5Pipe* md5, Emit&& emit_copy,
                JobResult& r) {
    struct CdEnt {
      std::string name;
      uint32_t crc;
      uint64_t size, hdr_off;
    };
    std::vector<CdEnt> cd;
    for (auto& rec : recs) {
      const uint64_t hdr_off = off - base;
      const bool z64 = rec.nbytes >= 0xFFFFFFFFull;
      std::vector<uint8_t> h;
      put32(h, 0x04034b50);
      put16(h, z64 ? 45 : 20);  // version needed
      put16(h, 0x0800);         // UTF-8 names, no data descriptor
      put16(h, 0);              // stored
      put16(h, 0);
      put16(h, 0x21);           // dos time/date (1980-01-01)
      // CRC first (parallel pieces over the staged bytes), so every byte is final when written
      // and the MD5 pipe can hash the stream as it goes.
      wait_range(rec.ptr, rec.nbytes, r);
      const uint32_t crc = crc32_parallel(0, (const uint8_t*)rec.ptr, rec.nbytes);
      put32(h, crc);
      put32(h, z64 ? 0xFFFFFFFFu : (uint32_t)rec.nbytes);
      put32(h, z64 ? 0xFFFFFFFFu : (uint32_t)rec.nbytes);
      put16(h, (uint16_t)rec.name.size());
      const size_t extra_len_pos = h.size();
      put16(h, 0);
      h.insert(h.end(), rec.name.begin(), rec.name.end());
      std::vector<uint8_t> ex;
      if (z64) {
        put16(ex, 0x0001);
        put16(ex, 16);
        put64(ex, rec.nbytes);
        put64(ex, rec.nbytes);
      }
      // 64-byte alignment (relative to the archive start) of the payload via a padding extra
      // field ("FB", like torch's writer), so mmap'ed loads see aligned storages
      const uint64_t data_start = hdr_off + h.size() + ex.size();
      const uint64_t pad = (64 - (data_start + 4) % 64) % 64;
      put16(ex, 0x4246);
      put16(ex, (uint16_t)pad);
      ex.insert(ex.end(), pad, 0);
      h[extra_len_pos] = ex.size() & 0xff;
      h[extra_len_pos + 1] = ex.size() >> 8;
      h.insert(h.end(), ex.begin(), ex.end());
      emit_copy(h);
      constexpr uint64_t kPiece = 64ull << 20;
      for (uint64_t o = 0; o < rec.nbytes; o += kPiece) {
        const uint64_t n = std::min(kPiece, rec.nbytes - o);
        const uint8_t* p = (const uint8_t*)(rec.ptr + o);
        write_all(fd, p, n);
        if (md5) md5->push_borrowed(p, n);
        off += n;
      }
      cd.push_back({rec.name, crc, rec.nbytes, hdr_off});
    }
    const uint64_t cd_off = off - base;
    std::vector<uint8_t> c;
    for (auto& e : cd) {
      const bool zs = e.size >= 0xFFFFFFFFull, zo = e.hdr_off >= 0xFFFFFFFFull;
      std::vector<uint8_t> ex;
      if (zs || zo) {
        put16(ex, 0x0001);
        put16(ex, (uint16_t)((zs ? 16 : 0) + (zo ? 8 : 0)));
        if (zs) { put64(ex, e.size); put64(ex, e.size); }
        if (zo) put64(ex, e.hdr_off);
      }
      put32(c, 0x02014b50);
      put16(c, (3 << 8) | 45);  // made by: unix, 4.5
      put16(c, (zs || zo) ? 45 : 20);
      put16(c, 0x0800);
      put16(c, 0);
      put16(c, 0);
      put16(c, 0x21);
      put32(c, e.crc);
      put32(c, zs ? 0xFFFFFFFFu : (uint32_t)e.size);
      put32(c, zs ? 0xFFFFFFFFu : (uint32_t)e.size);
      put16(c, (uint16_t)e.name.size());
      put16(c, (uint16_t)ex.size());
      put16(c, 0);  // comment
      put16(c, 0);  // disk
      put16(c, 0);  // internal attr
      put32(c, 0100644u << 16);
      put32(c, zo ? 0xFFFFFFFFu : (uint32_t)e.hdr_off);
      c.insert(c.end(), e.name.begin(), e.name.end());
      c.insert(c.end(), ex.begin(), ex.end());
    }
    const uint64_t cd_size = c.size();
    const uint64_t n = cd.size();
    const bool z64e = cd_off >= 0xFFFFFFFFull || cd_size >= 0xFFFFFFFFull || n >= 0xFFFF;
    if (z64e) {
      const uint64_t z64_off = cd_off + cd_size;
      put32(c, 0x06064b50);
      put64(c, 44);
      put16(c, (3 << 8) | 45);
      put16(c, 45);
      put32(c, 0);
      put32(c, 0);
      put64(c, n);
      put64(c, n);
      put64(c, cd_size);
      put64(c, cd_off);
      put32(c, 0x07064b50);
      put32(c, 0);
      put64(c, z64_off);
      put32(c, 1);
    }
    put32(c, 0x06054b50);
    put16(c, 0);
    put16(c, 0);
    put16(c, z64e ? 0xFFFF : (uint16_t)n);
    put16(c, z64e ? 0xFFFF : (uint16_t)n);
    put32(c, z64e ? 0xFFFFFFFFu : (uint32_t)cd_size);
    put32(c, z64e ? 0xFFFFFFFFu : (uint32_t)cd_off);
    put16(c, 0);
    emit_copy(c);
  }

  void write_impl(const std::string& path, std::vector<Item>& items, bool want_md5, bool do_fsync, JobResult& r) {
    if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
    const std::string tmp = path + ".tmp";
    const int fd = ::open(tmp.c_str(), O_CREAT | O_TRUNC | O_RDWR | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("ckpt_engine: cannot open " + tmp + ": " + strerror(errno));
    std::unique_ptr<Md5Pipe> md5;
    if (want_md5) md5 = std::make_unique<Md5Pipe>();
    uint64_t off = 0;
    // Fault-injection hook (recovery tests): PYRECOVER_FAULT_HOLD_WRITE=<substring> parks the
    // writer after the first bytes of a matching archive, so a kill lands mid-write for certain.
    const char* hold = std::getenv("PYRECOVER_FAULT_HOLD_WRITE");
    bool hold_now = hold != nullptr && hold[0] != 0 && path.find(hold) != std::string::npos;
    auto emit_copy = [&](const std::vector<uint8_t>& b) {
      write_all(fd, b.data(), b.size());
      if (md5) md5->push_copy(b.data(), b.size());
      off += b.size();
      if (hold_now) {
        hold_now = false;
        std::this_thread::sleep_for(std::chrono::seconds(120));
      }
    };
    try {
      for (auto& it : items) {
        const uint64_t start = off;
        if (it.raw) {
          wait_range(it.ptr, it.n, r);
          write_all(fd, (const void*)it.ptr, it.n);
          if (md5) md5->push_borrowed((const void*)it.ptr, it.n);
          off += it.n;
        } else {
          emit_zip(it.records, off, start, fd, md5.get(), emit_copy, r);
        }
        r.items.push_back({start, off - start});
      }
      if (do_fsync && ::fsync(fd) != 0) throw std::runtime_error("ckpt_engine: fsync failed");
      // Whole-file MD5 (the reference's `.md5` sidecar: 32 hex chars, no newline).
      if (md5) r.md5 = md5->finish();
    } catch (...) {
      ::close(fd);
      if (md5) md5->finish();
      throw;
    }
    ::close(fd);
    r.bytes = off;
    if (::rename(tmp.c_str(), path.c_str()) != 0)
      throw std::runtime_error("ckpt_engine: rename failed: " + std::string(strerror(errno)));
    if (want_md5) {
      const std::string mp = path + ".md5", mt = mp + ".tmp";
      const int mfd = ::open(mt.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0644);
      if (mfd < 0) throw std::runtime_error("ckpt_engine: cannot open md5 sidecar");
      write_all(mfd, r.md5.data(), r.md5.size());
      if (do_fsync) ::fsync(mfd);
      ::close(mfd);
      if (::rename(mt.c_str(), mp.c_str()) != 0) throw std::runtime_error("ckpt_engine: md5 rename failed");
    }
  }

  int device_;
  hipStream_t stream_ = nullptr;
  hipEvent_t entry_ev_ = nullptr;
  void* pool_ = nullptr;
  uint64_t pool_size_ = 0;
  uint64_t staged_bytes_ = 0;
  std::vector<Chunk> chunks_;
  std::thread writer_;
  std::mutex mu_;
  bool running_ = false;
  JobResult result_;
};

// Streaming whole-file MD5 (used to verify on load without reading the file into RAM at
// once, unlike reference checkpoint.py:162-166).
inline std::string md5_file(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) throw std::runtime_error("md5_file: cannot open " + path);
  std::string h;
  try {
    h = md5_fd(fd);
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
  return h;
}


}  // namespace ckpt
}  // namespace pra
