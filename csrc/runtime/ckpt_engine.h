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

// the bandwidth-bound D2D copy kernel of csrc/kernels/comm.hip (linked into pyrecover_amd._C); weak,
// so the host-only engine self-test links without the kernels (it never takes the device path)
extern "C" hipError_t pra_copy_d2d(void* dst, const void* src, long nbytes, hipStream_t s) __attribute__((weak));

#include <openssl/evp.h>
#include <zlib.h>
#include <immintrin.h>

#include <fcntl.h>
#include <sys/mman.h>
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
#include <tuple>
#include <utility>
#include <vector>

namespace pra {
namespace ckpt {


// Pinned (DMA-mapped) pages are copied eagerly by fork() (Linux copies pinned anonymous pages at
// fork instead of sharing them copy-on-write), so a DataLoader forking its workers after a
// multi-GB staging pool exists stalls for minutes (measured: 147 s at 10.5 GiB, two workers). No
// child ever touches these buffers: keep them out of forks altogether.
inline void dont_fork(void* p, uint64_t n) {
  const uintptr_t pg = 4096, a = (uintptr_t)p & ~(pg - 1), e = ((uintptr_t)p + n + pg - 1) & ~(pg - 1);
  (void)::madvise((void*)a, e - a, MADV_DONTFORK);
}

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
  // drop everything still queued and stop (the digest is then meaningless)
  void abort() {
    if (!th_.joinable()) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.clear();
      done_ = true;
    }
    cv_.notify_all();
    cv_space_.notify_all();
    th_.join();
  }
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

// CRC-32 (zip/gzip polynomial, reflected) by carry-less multiplication: 4 x 128-bit lanes folded
// 64 bytes per step, then Barrett reduction (Intel's PCLMULQDQ folding; same constants as the
// Linux crc32-pclmul code). ~10x zlib 1.2.11's table CRC on the same core. Returns the RAW
// register update (no pre/post inversion); n >= 64 and n % 16 == 0.
#define PRA_CLMUL __attribute__((target("pclmul,sse4.1")))
PRA_CLMUL inline __m128i crc_ld(const uint8_t* q) { return _mm_loadu_si128((const __m128i*)q); }
PRA_CLMUL inline __m128i crc_fold(__m128i x, __m128i k, __m128i next) {
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), next);
}
PRA_CLMUL inline uint32_t crc32_fold_raw(uint32_t crc, const uint8_t* p, size_t n) {
  const __m128i k12 = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);  // hi R2, lo R1
  const __m128i k34 = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);  // hi R4, lo R3
  const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124LL);
  const __m128i pu = _mm_set_epi64x(0x1f7011641LL, 0x1db710641LL);   // hi u, lo P'
  const __m128i m32 = _mm_set_epi32(0, 0, 0, -1);
  __m128i x1 = _mm_xor_si128(crc_ld(p), _mm_cvtsi32_si128((int)crc)), x2 = crc_ld(p + 16), x3 = crc_ld(p + 32),
          x4 = crc_ld(p + 48);
  p += 64;
  n -= 64;
  for (; n >= 64; p += 64, n -= 64) {
    x1 = crc_fold(x1, k12, crc_ld(p));
    x2 = crc_fold(x2, k12, crc_ld(p + 16));
    x3 = crc_fold(x3, k12, crc_ld(p + 32));
    x4 = crc_fold(x4, k12, crc_ld(p + 48));
  }
  x1 = crc_fold(x1, k34, x2);
  x1 = crc_fold(x1, k34, x3);
  x1 = crc_fold(x1, k34, x4);
  for (; n >= 16; p += 16, n -= 16) x1 = crc_fold(x1, k34, crc_ld(p));
  // 128 -> 64 bits (appends 32 zero bits), 64 -> 32, Barrett
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), _mm_clmulepi64_si128(k34, x1, 0x01));
  __m128i t = _mm_and_si128(x1, m32);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 4), _mm_clmulepi64_si128(t, k5, 0x00));
  t = _mm_and_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, m32), pu, 0x10), m32);
  x1 = _mm_xor_si128(x1, _mm_clmulepi64_si128(t, pu, 0x00));
  return (uint32_t)_mm_extract_epi32(x1, 1);
}
#undef PRA_CLMUL

// zlib-convention CRC-32 (crc32(crc, p, n) of zlib) on the folding kernel.
inline uint32_t crc32_fast(uint32_t crc, const uint8_t* p, size_t n) {
  if (n < 64) return (uint32_t)crc32_z(crc, p, n);
  const size_t m = n & ~size_t(15);
  crc = ~crc32_fold_raw(~crc, p, m);
  return (uint32_t)crc32_z(crc, p + m, n - m);
}

inline uint32_t crc32_parallel(uint32_t crc, const uint8_t* p, size_t n) {
  constexpr size_t kPiece = 16u << 20;
  if (n <= kPiece) return crc32_fast(crc, p, n);
  const size_t np = (n + kPiece - 1) / kPiece;
  std::vector<std::future<uint32_t>> fut;
  std::vector<size_t> len(np);
  for (size_t i = 0; i < np; ++i) {
    const size_t off = i * kPiece;
    len[i] = std::min(kPiece, n - off);
    fut.push_back(std::async(std::launch::async, [p, off, l = len[i]] { return crc32_fast(0, p + off, l); }));
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

// A contiguous range of the output file whose bytes are at `p` (the pinned pool, caller memory
// or an engine-owned header buffer).
struct Piece {
  uint64_t off;
  const uint8_t* p;
  uint64_t n;
};

// Segment size of the `.md5parts` sidecar: MD5 is inherently serial (~1 GB/s per core), so
// besides the reference's whole-file `.md5` every checkpoint file carries the MD5 of each
// 256 MiB segment, written and verified by many threads in parallel.
constexpr uint64_t kSegBytes = 256ull << 20;
constexpr int kWriters = 16;  // 16 vs 8: vanilla save 9.4 -> 8.0 s, sharded 5.6 -> 5.2 s at 7B (profiles/ckpt_threads_ab_r2)

inline std::string digest_hex(EVP_MD_CTX* ctx) {
  unsigned char dig[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_DigestFinal_ex(ctx, dig, &len);
  static const char* hex = "0123456789abcdef";
  std::string out;
  for (unsigned i = 0; i < len; ++i) {
    out.push_back(hex[dig[i] >> 4]);
    out.push_back(hex[dig[i] & 15]);
  }
  return out;
}

// "pyrecover-md5parts 1 <segment bytes> <file bytes>\n" + one hex digest per line
inline std::string md5parts_text(uint64_t seg, uint64_t total, const std::vector<std::string>& md5s) {
  std::string t = "pyrecover-md5parts 1 " + std::to_string(seg) + " " + std::to_string(total) + "\n";
  for (auto& m : md5s) t += m + "\n";
  return t;
}

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
  double layout_seconds = 0;  // CRC32 + headers (after the staged bytes landed)
  double write_seconds = 0;   // parallel segment writes + MD5s (+ whole-file MD5)
  double fsync_seconds = 0;
  int writers = 0;
  bool direct = false;
  std::vector<std::pair<uint64_t, uint64_t>> items;  // (offset, length) of each item in the file
  struct Rec {
    std::string name;
    uint64_t data_off, nbytes;  // payload position of each zip record in the file
  };
  std::vector<Rec> records;
  uint64_t seg_bytes = 0;
  std::vector<std::string> seg_md5;  // MD5 of each kSegBytes segment of the file
  bool md5_deferred = false;  // the whole-file `.md5` sidecar is still being computed (flush())
};

struct CkptEngineIo {
  // 0, or the errno of the first failed pwrite
  static int try_pwrite_all(int fd, const uint8_t* b, size_t n, uint64_t pos) {
    while (n) {
      const ssize_t w = ::pwrite(fd, b, std::min<size_t>(n, 1u << 30), (off_t)pos);
      if (w < 0) {
        if (errno == EINTR) continue;
        return errno;
      }
      b += w;
      pos += (uint64_t)w;
      n -= (size_t)w;
    }
    return 0;
  }
};

// Streaming MD5 of an open file from its start (double-buffered reads on this thread, hashing
// on the Md5Pipe thread). `cancel` (optional) is checked between reads: once set, the digest is
// dropped and md5_fd throws.
// `left` (optional) is decremented by the bytes hashed, `consumed` (optional) counts them.
inline std::string md5_fd(int fd, const std::atomic<bool>* cancel = nullptr,
                          std::atomic<int64_t>* left = nullptr, int64_t* consumed = nullptr) {
  Md5Pipe md5;
  constexpr size_t kBuf = 32u << 20;
  uint64_t pos = 0;
  for (;;) {
    if (cancel != nullptr && cancel->load(std::memory_order_relaxed)) {
      md5.abort();
      throw std::runtime_error("md5: cancelled");
    }
    auto buf = std::make_shared<std::vector<uint8_t>>(kBuf);
    ssize_t n;
    do {
      n = ::pread(fd, buf->data(), kBuf, (off_t)pos);
    } while (n < 0 && errno == EINTR);
    if (n < 0) throw std::runtime_error("md5: read failed");
    if (n == 0) break;
    md5.push_copy(buf->data(), (size_t)n);
    pos += (uint64_t)n;
    if (left != nullptr) left->fetch_sub(n);
    if (consumed != nullptr) *consumed += n;
  }
  return md5.finish();
}

// Throughput probes for the time-aware stop (the final checkpoint's cost is budgeted from the
// bytes it will write and these rates before any save of the run has completed).
// Single-stream MD5 over an in-memory buffer: the rate of the reference's whole-file `.md5`.
inline double md5_probe_bps(uint64_t nbytes) {
  nbytes = std::max<uint64_t>(nbytes, 1u << 20);
  std::vector<uint8_t> buf(nbytes);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (uint64_t i = 0; i + 8 <= nbytes; i += 8) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    std::memcpy(buf.data() + i, &x, 8);
  }
  const auto t0 = std::chrono::steady_clock::now();
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  EVP_DigestInit_ex(ctx, EVP_md5(), nullptr);
  EVP_DigestUpdate(ctx, buf.data(), buf.size());
  unsigned char dig[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_DigestFinal_ex(ctx, dig, &len);
  EVP_MD_CTX_free(ctx);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return (double)nbytes / std::max(s, 1e-9);
}

// Parallel write throughput through the archive writer's path: `threads` threads pwrite 64 MiB
// aligned buffers of incompressible bytes at disjoint offsets of the probe file `path` (O_DIRECT
// when the filesystem takes it), then fsync; the file is removed. Returns bytes/s.
inline double write_probe_bps(const std::string& path, uint64_t nbytes, int threads, bool do_fsync) {
  constexpr uint64_t kBuf = 64ull << 20;
  threads = std::max(1, threads);
  const uint64_t nchunks = std::max<uint64_t>(1, (nbytes + kBuf - 1) / kBuf);
  const int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("write probe: cannot open " + path + ": " + strerror(errno));
  const int dfd = ::open(path.c_str(), O_WRONLY | O_CLOEXEC | O_DIRECT);
  std::atomic<bool> direct{dfd >= 0};
  std::atomic<uint64_t> next{0};
  std::string err;
  std::mutex err_mu;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ws;
  for (int t = 0; t < (int)std::min<uint64_t>((uint64_t)threads, nchunks); ++t)
    ws.emplace_back([&, t] {
      uint8_t* b = nullptr;
      if (posix_memalign((void**)&b, 4096, kBuf) != 0) {
        std::lock_guard<std::mutex> g(err_mu);
        err = "write probe: alloc failed";
        return;
      }
      uint64_t x = 0x243f6a8885a308d3ull ^ (uint64_t)t;
      for (uint64_t i = 0; i + 8 <= kBuf; i += 8) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        std::memcpy(b + i, &x, 8);
      }
      for (uint64_t c; (c = next.fetch_add(1)) < nchunks;) {
        int rc = EINVAL;
        if (direct.load()) {
          rc = CkptEngineIo::try_pwrite_all(dfd, b, kBuf, c * kBuf);
          if (rc == EINVAL) direct = false;
        }
        if (rc == EINVAL) rc = CkptEngineIo::try_pwrite_all(fd, b, kBuf, c * kBuf);
        if (rc != 0) {
          std::lock_guard<std::mutex> g(err_mu);
          err = std::string("write probe: ") + strerror(rc);
          break;
        }
      }
      ::free(b);
    });
  for (auto& w : ws) w.join();
  if (dfd >= 0) ::close(dfd);
  if (err.empty() && do_fsync && ::fsync(fd) != 0) err = "write probe: fsync failed";
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  ::close(fd);
  ::unlink(path.c_str());
  if (!err.empty()) throw std::runtime_error(err);
  return (double)(nchunks * kBuf) / std::max(s, 1e-9);
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
      flush();
    } catch (...) {
    }
    release_chunks();
    free_pool();
    if (device_ >= 0) {
      if (hbm_ev_ != nullptr) (void)hipEventDestroy(hbm_ev_);
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
      dont_fork(pool_, nbytes);
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
  //
  // hbm (device pointer, hbm_bytes >= the packed size): two-hop snapshot. The regions are first
  // copied device-to-device into this HBM buffer (tens of ms at HBM bandwidth); fence() waits for
  // THAT copy only, and the slow D2H into the pinned pool (~0.6 s for 38 GiB) then drains from the
  // HBM copy while the next optimizer steps overwrite the live buffers.
  std::vector<uint64_t> stage(const std::vector<std::pair<uintptr_t, uint64_t>>& regions, hipStream_t cur,
                              uintptr_t hbm = 0, uint64_t hbm_bytes = 0) {
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
    const bool two_hop = hbm != 0 && hbm_bytes >= total;
    if (two_hop) {
      for (size_t i = 0; i < regions.size(); ++i) {
        void* d = (uint8_t*)hbm + offs[i];
        const void* sp = (const void*)regions[i].first;
        if (pra_copy_d2d != nullptr)
          hip_check(pra_copy_d2d(d, sp, (long)regions[i].second, stream_), "snapshot D2D copy");
        else
          hip_check(hipMemcpyAsync(d, sp, regions[i].second, hipMemcpyDeviceToDevice, stream_), "snapshot D2D copy");
      }
      if (hbm_ev_ == nullptr) hip_check(hipEventCreateWithFlags(&hbm_ev_, hipEventDisableTiming), "event create");
      hip_check(hipEventRecord(hbm_ev_, stream_), "event record");
    }
    fence_ev_ = two_hop ? hbm_ev_ : nullptr;  // null: the last D2H chunk
    last_two_hop_ = two_hop;
    constexpr uint64_t kChunk = 256ull << 20;
    for (size_t i = 0; i < regions.size(); ++i) {
      const uint8_t* src = two_hop ? (const uint8_t*)hbm + offs[i] : (const uint8_t*)regions[i].first;
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
    hip_check(hipStreamWaitEvent(cur, fence_ev_ != nullptr ? fence_ev_ : chunks_.back().ev, 0), "fence");
  }
  bool last_two_hop() const { return last_two_hop_; }
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
  // defer_md5: the job completes once the archive and its `.md5parts` are durable; the reference's
  // whole-file `.md5` (serial MD5, ~0.9 GB/s: ~45 s at 7B) is computed by a background thread that
  // re-reads the file, and appears atomically later -- flush() (also run at destruction) waits.
  void write_items(const std::string& path, std::vector<Item> items, bool want_md5, bool do_fsync,
                   bool defer_md5 = false) {
    wait_writer();
    running_ = true;
    result_ = JobResult{};
    uint64_t est = 0;  // payload bytes (headers are added by the layout)
    for (auto& it : items) {
      est += it.n;
      for (auto& rc : it.records) est += rc.nbytes;
    }
    prog_total_ = est;
    prog_written_ = 0;
    prog_hashed_ = 0;
    const char* wm = std::getenv("PYRECOVER_WHOLE_MD5");
    const bool whole = want_md5 && !(wm != nullptr && wm[0] == '0');
    prog_md5_ = whole ? (defer_md5 ? 2 : 1) : 0;
    writer_ = std::thread([this, path, items = std::move(items), want_md5, do_fsync, defer_md5]() mutable {
      JobResult r;
      const auto t0 = std::chrono::steady_clock::now();
      try {
        write_impl(path, items, want_md5, do_fsync, defer_md5, r);
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

  // Progress of the current (or last) archive job: bytes of the file, bytes written, bytes of
  // the inline whole-file MD5 hashed, and its mode (0 none, 1 inline, 2 deferred). The time-aware
  // stop estimates the drain of an in-flight save from what is still to write.
  std::tuple<uint64_t, uint64_t, uint64_t, int> progress() const {
    return {prog_total_.load(), prog_written_.load(), prog_hashed_.load(), prog_md5_.load()};
  }
  // Bytes deferred digests still have to hash (queued and running), and the slowest completed
  // digest's rate in bytes/s (0 if none of at least 64 MiB completed).
  uint64_t md5_pending_bytes() const { return (uint64_t)std::max<int64_t>(0, md5st_->left.load()); }
  double md5_min_bps() {
    std::lock_guard<std::mutex> g(md5st_->mu);
    return md5st_->min_bps;
  }

  JobResult wait() {
    wait_writer();
    return result_;
  }

  // Wait for a deferred whole-file digest; returns its error ("" if none / nothing pending).
  std::string flush() {
    std::vector<std::thread> th;
    {
      std::lock_guard<std::mutex> g(md5_th_mu_);
      th.swap(md5_th_);
    }
    for (auto& t : th) t.join();
    std::lock_guard<std::mutex> g(md5st_->mu);
    std::string e;
    e.swap(md5st_->error);
    return e;
  }
  // Cancel deferred digests (a job about to be killed by its wall-clock limit): each stops at its
  // next 32 MiB read and is joined here, so no digest thread outlives the call (interpreter
  // shutdown, static destructors). A cancelled digest leaves no `.md5`; the `.md5parts` written
  // with the archive still verify it.
  // Returns the error of a digest that had failed on its own before the cancel ("" if none): a
  // cancelled digest records nothing, so what is left is a real failure.
  std::string abandon_md5() {
    md5st_->cancel = true;
    std::vector<std::thread> th;
    {
      std::lock_guard<std::mutex> g(md5_th_mu_);
      th.swap(md5_th_);
    }
    for (auto& t : th) t.join();
    std::lock_guard<std::mutex> g(md5st_->mu);
    std::string e;
    e.swap(md5st_->error);
    md5st_->cancel = false;  // later saves digest again
    return e;
  }
  double md5_max_seconds() {
    std::lock_guard<std::mutex> g(md5st_->mu);
    return md5st_->max_seconds;
  }
  bool md5_pending() {
    std::lock_guard<std::mutex> g(md5st_->mu);
    return md5st_->running > 0;
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

  // Lay out one zip archive (offsets inside it are relative to `base`, the archive's first byte):
  // CRC32 of every record (parallel pieces over the staged bytes), local headers, payload
  // pointers and the central directory become Pieces of the file at known offsets, so the bytes
  // can then be written by several threads at once.
  void layout_zip(std::vector<Record>& recs, const uint32_t* crcs, uint64_t& off, const uint64_t base,
                  std::vector<Piece>& pieces, std::deque<std::vector<uint8_t>>& owned, JobResult& r) {
    struct CdEnt {
      std::string name;
      uint32_t crc;
      uint64_t size, hdr_off;
    };
    auto own = [&](std::vector<uint8_t>&& b) {
      owned.push_back(std::move(b));
      pieces.push_back({off, owned.back().data(), owned.back().size()});
      off += owned.back().size();
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
      const uint32_t crc = crcs[&rec - recs.data()];
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
      own(std::move(h));
      r.records.push_back({rec.name, off, rec.nbytes});
      if (rec.nbytes) pieces.push_back({off, (const uint8_t*)rec.ptr, rec.nbytes});
      off += rec.nbytes;
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
    own(std::move(c));
  }

  static int try_pwrite_all(int fd, const uint8_t* b, size_t n, uint64_t pos) {
    return CkptEngineIo::try_pwrite_all(fd, b, n, pos);
  }
  static void pwrite_all(int fd, const uint8_t* b, size_t n, uint64_t pos) {
    if (const int e = try_pwrite_all(fd, b, n, pos))
      throw std::runtime_error(std::string("ckpt_engine: write failed: ") + strerror(e));
  }

  // The file is written segment by segment (kSegBytes) by kWriters threads, each hashing the
  // segments it writes (the `.md5parts` sidecar, verified in parallel on load); the reference's
  // whole-file MD5 (`.md5`) is computed over the same in-memory pieces on its own thread.
  void write_impl(const std::string& path, std::vector<Item>& items, bool want_md5, bool do_fsync, bool defer_md5,
                  JobResult& r) {
    if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
    using clk = std::chrono::steady_clock;
    const auto t_layout = clk::now();
    // every staged byte has landed; CRC-32 of all zip records in one parallel pass (64 MiB pieces
    // over kWriters threads, combined per record)
    std::vector<std::vector<uint32_t>> crcs(items.size());
    {
      struct Task {
        size_t item, rec;
        uint64_t o, n;
      };
      std::vector<Task> tasks;
      for (size_t i = 0; i < items.size(); ++i) {
        if (items[i].raw) {
          wait_range(items[i].ptr, items[i].n, r);
          continue;
        }
        crcs[i].assign(items[i].records.size(), 0);
        for (size_t j = 0; j < items[i].records.size(); ++j) {
          const Record& rec = items[i].records[j];
          wait_range(rec.ptr, rec.nbytes, r);
          constexpr uint64_t kPiece = 64ull << 20;
          for (uint64_t o = 0; o < rec.nbytes; o += kPiece) tasks.push_back({i, j, o, std::min(kPiece, rec.nbytes - o)});
        }
      }
      std::vector<uint32_t> part(tasks.size());
      std::atomic<size_t> nt{0};
      std::vector<std::thread> cth;
      for (int t = 0; t < kWriters; ++t)
        cth.emplace_back([&] {
          for (size_t k; (k = nt.fetch_add(1)) < tasks.size();)
            part[k] = crc32_fast(0, (const uint8_t*)items[tasks[k].item].records[tasks[k].rec].ptr + tasks[k].o,
                                 tasks[k].n);
        });
      for (auto& x : cth) x.join();
      for (size_t k = 0; k < tasks.size(); ++k) {  // pieces are in record order
        uint32_t& c = crcs[tasks[k].item][tasks[k].rec];
        c = tasks[k].o == 0 ? part[k] : (uint32_t)crc32_combine(c, part[k], (z_off_t)tasks[k].n);
      }
    }
    std::vector<Piece> pieces;
    std::deque<std::vector<uint8_t>> owned;
    uint64_t off = 0;
    for (size_t i = 0; i < items.size(); ++i) {
      auto& it = items[i];
      const uint64_t start = off;
      if (it.raw) {
        if (it.n) pieces.push_back({off, (const uint8_t*)it.ptr, it.n});
        off += it.n;
      } else {
        layout_zip(it.records, crcs[i].data(), off, start, pieces, owned, r);
      }
      r.items.push_back({start, off - start});
    }
    const uint64_t total = off;
    prog_total_ = total;
    r.layout_seconds = std::chrono::duration<double>(clk::now() - t_layout).count() - r.stage_wait_seconds;
    const auto t_write = clk::now();
    const std::string tmp = path + ".tmp";
    const int fd = ::open(tmp.c_str(), O_CREAT | O_TRUNC | O_RDWR | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("ckpt_engine: cannot open " + tmp + ": " + strerror(errno));
    // Fault-injection hook (recovery tests): PYRECOVER_FAULT_HOLD_WRITE=<substring> parks the
    // writer after the first bytes of a matching archive, so a kill lands mid-write for certain.
    const char* hold = std::getenv("PYRECOVER_FAULT_HOLD_WRITE");
    if (hold != nullptr && hold[0] != 0 && path.find(hold) != std::string::npos && !pieces.empty()) {
      pwrite_all(fd, pieces[0].p, pieces[0].n, pieces[0].off);
      std::this_thread::sleep_for(std::chrono::seconds(120));
    }
    const uint64_t nseg = (total + kSegBytes - 1) / kSegBytes;
    r.seg_bytes = want_md5 ? kSegBytes : 0;
    r.seg_md5.assign(want_md5 ? nseg : 0, std::string());
    std::mutex err_mu;
    std::string err;
    auto fail = [&](const char* what) {
      std::lock_guard<std::mutex> g(err_mu);
      if (err.empty()) err = what;
    };
    // PYRECOVER_WHOLE_MD5=0 skips the reference's whole-file `.md5` (serial, ~1 GB/s) and keeps
    // only the parallel `.md5parts`, for runs that never hand checkpoints to reference tooling
    const char* wm = std::getenv("PYRECOVER_WHOLE_MD5");
    const bool whole_md5 = want_md5 && !(wm != nullptr && wm[0] == '0');
    const bool deferred = whole_md5 && defer_md5;
    std::thread whole;
    if (whole_md5 && !deferred) {
      whole = std::thread([&] {
        try {
          EVP_MD_CTX* ctx = EVP_MD_CTX_new();
          EVP_DigestInit_ex(ctx, EVP_md5(), nullptr);
          for (auto& pc : pieces)
            for (uint64_t o = 0; o < pc.n; o += kHashStep) {
              const uint64_t n = std::min<uint64_t>(kHashStep, pc.n - o);
              EVP_DigestUpdate(ctx, pc.p + o, n);
              prog_hashed_ += n;
            }
          r.md5 = digest_hex(ctx);
          EVP_MD_CTX_free(ctx);
        } catch (const std::exception& e) {
          fail(e.what());
        }
      });
    }
    std::atomic<uint64_t> next{0};
    static const int writers_env = [] {
      const char* e = std::getenv("PYRECOVER_CKPT_WRITERS");
      return e ? std::max(1, atoi(e)) : kWriters;
    }();
    const int nthreads = (int)std::min<uint64_t>(writers_env, std::max<uint64_t>(nseg, 1));
    r.writers = nthreads;
    // O_DIRECT (PYRECOVER_CKPT_DIRECT_WRITE, default on): segments are assembled in aligned bounce
    // buffers and DMA'd to the device, skipping the page-cache copy and most of the fsync flush
    const char* dw = std::getenv("PYRECOVER_CKPT_DIRECT_WRITE");
    int dfd = (dw != nullptr && dw[0] == '0') ? -1 : ::open(tmp.c_str(), O_WRONLY | O_CLOEXEC | O_DIRECT);
    // Some filesystems (FUSE, overlay, network) accept the O_DIRECT open but refuse the aligned
    // pwrite with EINVAL: the first such refusal switches this and every later chunk of the save to
    // buffered writes on `fd` (as Reader::read_impl does for reads). PYRECOVER_FAULT_DIRECT_EINVAL=1
    // injects that refusal on the first direct write (tests).
    r.direct = dfd >= 0;
    std::atomic<bool> use_direct{dfd >= 0};
    static const bool inject_einval = [] {
      const char* e = std::getenv("PYRECOVER_FAULT_DIRECT_EINVAL");
      return e != nullptr && e[0] == '1';
    }();
    std::atomic<bool> injected{false};
    constexpr uint64_t kBounce = 64ull << 20;
    std::vector<std::thread> ws;
    for (int t = 0; t < nthreads; ++t) {
      ws.emplace_back([&] {
        EVP_MD_CTX* ctx = EVP_MD_CTX_new();
        uint8_t* bounce = nullptr;
        try {
          if (dfd >= 0 && posix_memalign((void**)&bounce, 4096, kBounce) != 0)
            throw std::runtime_error("ckpt_engine: bounce buffer alloc failed");
          for (uint64_t s; (s = next.fetch_add(1)) < nseg;) {
            const uint64_t a = s * kSegBytes, b = std::min(total, a + kSegBytes);
            if (want_md5) EVP_DigestInit_ex(ctx, EVP_md5(), nullptr);
            for (uint64_t c = a; c < b; c += kBounce) {
              const uint64_t e = std::min(b, c + kBounce);
              // pieces overlapping [c, e)
              auto it = std::upper_bound(pieces.begin(), pieces.end(), c,
                                         [](uint64_t x, const Piece& pc) { return x < pc.off + pc.n; });
              for (; it != pieces.end() && it->off < e; ++it) {
                const uint64_t lo = std::max(c, it->off), hi = std::min(e, it->off + it->n);
                const uint8_t* src = it->p + (lo - it->off);
                if (bounce) std::memcpy(bounce + (lo - c), src, hi - lo);
                else pwrite_all(fd, src, hi - lo, lo);
                if (want_md5 && !bounce) EVP_DigestUpdate(ctx, src, hi - lo);
                if (!bounce) prog_written_ += hi - lo;
              }
              if (bounce) {
                if (want_md5) EVP_DigestUpdate(ctx, bounce, e - c);
                int rc = EINVAL;
                if (use_direct.load()) {
                  const uint64_t len = (e - c + 4095) & ~uint64_t(4095);  // tail padded; truncated below
                  std::memset(bounce + (e - c), 0, len - (e - c));
                  rc = (inject_einval && !injected.exchange(true)) ? EINVAL : try_pwrite_all(dfd, bounce, len, c);
                  if (rc == EINVAL) use_direct = false;
                  else if (rc != 0) throw std::runtime_error(std::string("ckpt_engine: write failed: ") + strerror(rc));
                }
                if (rc == EINVAL) pwrite_all(fd, bounce, e - c, c);  // buffered, exact length
                prog_written_ += e - c;
              }
            }
            if (want_md5) r.seg_md5[s] = digest_hex(ctx);
          }
        } catch (const std::exception& e) {
          fail(e.what());
        }
        ::free(bounce);
        EVP_MD_CTX_free(ctx);
      });
    }
    for (auto& w : ws) w.join();
    if (whole.joinable()) whole.join();
    if (dfd >= 0) {
      ::close(dfd);
      if (err.empty() && total % 4096 && ::ftruncate(fd, (off_t)total) != 0) err = "ckpt_engine: ftruncate failed";
    }
    r.direct = r.direct && use_direct.load();
    r.write_seconds = std::chrono::duration<double>(clk::now() - t_write).count();
    const auto t_sync = clk::now();
    if (err.empty() && do_fsync && ::fsync(fd) != 0) err = "ckpt_engine: fsync failed";
    r.fsync_seconds = std::chrono::duration<double>(clk::now() - t_sync).count();
    ::close(fd);
    if (!err.empty()) throw std::runtime_error(err);
    r.bytes = total;
    {
      // under the sidecar lock: an earlier deferred digest of the same path either wrote its
      // sidecar before this unlink, or sees the new inode after the rename and writes nothing
      std::lock_guard<std::mutex> g(sidecar_mu());
      if (want_md5 && (!whole_md5 || deferred)) ::unlink((path + ".md5").c_str());  // no stale digest
      if (::rename(tmp.c_str(), path.c_str()) != 0)
        throw std::runtime_error("ckpt_engine: rename failed: " + std::string(strerror(errno)));
    }
    if (want_md5) {
      // whole-file MD5 (the reference's `.md5` sidecar: 32 hex chars, no newline) and the
      // per-segment list
      if (whole_md5 && !deferred) write_sidecar(path + ".md5", r.md5, do_fsync);
      write_sidecar(path + ".md5parts", md5parts_text(r.seg_bytes, total, r.seg_md5), do_fsync);
    }
    if (deferred) start_deferred_md5(path, do_fsync, r);
  }

  // The deferred digest re-reads the finished FILE (streaming, double-buffered preads; the serial
  // MD5 at ~1 GB/s, not the read, is its speed limit), so it holds no staging memory: the next
  // snapshot can reuse the pool at once, and several digests may be in flight (flush() joins all).
  void start_deferred_md5(const std::string& path, bool do_fsync, JobResult& r) {
    std::shared_ptr<Md5State> st = md5st_;  // shared: an abandoned (detached) digest outlives nothing it uses
    {
      std::lock_guard<std::mutex> g(st->mu);
      ++st->running;
    }
    const int64_t size = (int64_t)r.bytes;
    st->left += size;
    r.md5_deferred = true;
    std::lock_guard<std::mutex> g(md5_th_mu_);
    md5_th_.emplace_back([st, path, do_fsync, size] {
      int64_t consumed = 0;  // this digest's bytes hashed (the rest leaves `left` at the end)
      std::string err;
      const auto t0 = std::chrono::steady_clock::now();
      bool done = false;
      try {
        const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) throw std::runtime_error("ckpt_engine: deferred md5: cannot open " + path);
        struct stat before {};
        std::string md5;
        try {
          if (::fstat(fd, &before) != 0) throw std::runtime_error("ckpt_engine: deferred md5: fstat failed");
          md5 = md5_fd(fd, &st->cancel, &st->left, &consumed);
        } catch (...) {
          ::close(fd);
          throw;
        }
        ::close(fd);
        // write the sidecar only if `path` is still the file that was hashed: retention may have
        // deleted it meanwhile (no orphan `.md5`), or a new save of the same path may have
        // replaced it (its own digest owns the sidecar; no false mismatch on resume)
        // check and write under the lock a new save of the path takes around its unlink + rename
        std::lock_guard<std::mutex> g(sidecar_mu());
        struct stat now {};
        if (::stat(path.c_str(), &now) == 0 && now.st_ino == before.st_ino && now.st_dev == before.st_dev &&
            now.st_mtim.tv_sec == before.st_mtim.tv_sec && now.st_mtim.tv_nsec == before.st_mtim.tv_nsec &&
            now.st_size == before.st_size)
          write_sidecar(path + ".md5", md5, do_fsync);
        done = true;
      } catch (const std::exception& e) {
        if (!st->cancel.load()) err = e.what();
      }
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      st->left -= size - consumed;
      std::lock_guard<std::mutex> g2(st->mu);
      if (!err.empty()) st->error = err;
      if (done) st->max_seconds = std::max(st->max_seconds, sec);
      if (done && size >= (int64_t)(64u << 20)) {
        const double bps = (double)size / std::max(sec, 1e-9);
        st->min_bps = st->min_bps > 0 ? std::min(st->min_bps, bps) : bps;
      }
      --st->running;
    });
  }

  // Process-wide: orders a deferred digest's check-and-write of `<path>.md5` against a new save of
  // the same path (every engine instance, every thread).
  static std::mutex& sidecar_mu() {
    static std::mutex mu;
    return mu;
  }

  static void write_sidecar(const std::string& p, const std::string& text, bool do_fsync) {
    const std::string t = p + ".tmp";
    const int fd = ::open(t.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("ckpt_engine: cannot open " + t);
    write_all(fd, text.data(), text.size());
    if (do_fsync) ::fsync(fd);
    ::close(fd);
    if (::rename(t.c_str(), p.c_str()) != 0) throw std::runtime_error("ckpt_engine: sidecar rename failed");
  }

  int device_;
  hipStream_t stream_ = nullptr;
  hipEvent_t entry_ev_ = nullptr;
  hipEvent_t hbm_ev_ = nullptr;    // the D2D hop of a two-hop snapshot landed in the HBM buffer
  hipEvent_t fence_ev_ = nullptr;  // what fence() waits for (null: the last D2H chunk)
  bool last_two_hop_ = false;
  void* pool_ = nullptr;
  uint64_t pool_size_ = 0;
  uint64_t staged_bytes_ = 0;
  std::vector<Chunk> chunks_;
  std::thread writer_;
  struct Md5State {
    std::mutex mu;
    int running = 0;
    double max_seconds = 0;  // longest completed deferred digest (feeds the time-aware budget)
    double min_bps = 0;      // slowest completed digest of >= 64 MiB, bytes/s
    std::string error;
    std::atomic<bool> cancel{false};
    std::atomic<int64_t> left{0};  // bytes still to hash over every queued / running digest
  };
  std::vector<std::thread> md5_th_;  // deferred whole-file digests
  std::mutex md5_th_mu_;
  std::shared_ptr<Md5State> md5st_ = std::make_shared<Md5State>();
  std::mutex mu_;
  bool running_ = false;
  JobResult result_;
  static constexpr uint64_t kHashStep = 64ull << 20;
  std::atomic<uint64_t> prog_total_{0}, prog_written_{0}, prog_hashed_{0};
  std::atomic<int> prog_md5_{0};
};

// ------------------------------------------------------------------------------------------
// Parallel checkpoint reader: the resume path (replaces torch.load + load_state_dict, reference
// pyrecover/checkpoint.py:137-199 / 300-368). Byte ranges of a file go straight into their
// destination buffers (device pointers: pread into pinned staging buffers + hipMemcpyAsync H2D
// on one stream per thread; host pointers in CPU mode: pread + memcpy). The file is processed as
// kSegBytes work units by `threads` threads (64 MiB reads, double-buffered per thread), and
// the units listed in `hash_segs` are MD5-hashed on the way (the `.md5parts` check). O_DIRECT
// is used when the filesystem takes it (cold restarts do not fill the page cache twice).
struct ReadItem {
  uint64_t off, n;
  uintptr_t dst;
};

struct ReadResult {
  bool ok = false;
  std::string error;
  std::vector<std::string> seg_md5;  // "" for segments not hashed
  uint64_t bytes_read = 0;
  double seconds = 0;
  bool direct = false;
};

class Reader {
 public:
  static constexpr uint64_t kRead = 64ull << 20;
  explicit Reader(int device) : device_(device) {}
  ~Reader() { release(); }

  ReadResult read(const std::string& path, std::vector<ReadItem> items, const std::vector<int64_t>& hash_segs,
                  int threads, bool direct) {
    ReadResult r;
    const auto t0 = std::chrono::steady_clock::now();
    try {
      read_impl(path, items, hash_segs, threads, direct, r);
      r.ok = true;
    } catch (const std::exception& e) {
      r.ok = false;
      r.error = e.what();
    }
    r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return r;
  }

 private:
  struct Worker {
    uint8_t* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipStream_t stream = nullptr;
  };

  void ensure_workers(int n) {
    while ((int)workers_.size() < n) {
      Worker w;
      for (int i = 0; i < 2; ++i) {
        if (device_ >= 0) {
          hip_check(hipHostMalloc((void**)&w.buf[i], kRead + 4096, hipHostMallocDefault), "hipHostMalloc");
          dont_fork(w.buf[i], kRead + 4096);
          hip_check(hipEventCreateWithFlags(&w.ev[i], hipEventDisableTiming), "event create");
        } else if (posix_memalign((void**)&w.buf[i], 4096, kRead + 4096) != 0) {
          throw std::runtime_error("ckpt_reader: host alloc failed");
        }
      }
      if (device_ >= 0) hip_check(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking), "stream create");
      workers_.push_back(w);
    }
  }
  void release() {
    for (auto& w : workers_) {
      for (int i = 0; i < 2; ++i) {
        if (device_ >= 0) {
          if (w.ev[i]) (void)hipEventSynchronize(w.ev[i]), (void)hipEventDestroy(w.ev[i]);
          if (w.buf[i]) (void)hipHostFree(w.buf[i]);
        } else {
          ::free(w.buf[i]);
        }
      }
      if (w.stream) (void)hipStreamDestroy(w.stream);
    }
    workers_.clear();
  }

  static ssize_t pread_full(int fd, uint8_t* b, size_t n, uint64_t pos) {
    size_t got = 0;
    while (got < n) {
      const ssize_t k = ::pread(fd, b + got, n - got, (off_t)(pos + got));
      if (k < 0) {
        if (errno == EINTR) continue;
        return -1;
      }
      if (k == 0) break;
      got += (size_t)k;
    }
    return (ssize_t)got;
  }

  void read_impl(const std::string& path, std::vector<ReadItem>& items, const std::vector<int64_t>& hash_segs,
                 int threads, bool direct, ReadResult& r) {
    if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
    int fd = direct ? ::open(path.c_str(), O_RDONLY | O_CLOEXEC | O_DIRECT) : -1;
    r.direct = fd >= 0;
    if (fd < 0) fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) throw std::runtime_error("ckpt_reader: cannot open " + path + ": " + strerror(errno));
    struct stat st;
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      throw std::runtime_error("ckpt_reader: fstat failed");
    }
    const uint64_t size = (uint64_t)st.st_size;
    std::sort(items.begin(), items.end(), [](const ReadItem& a, const ReadItem& b) { return a.off < b.off; });
    for (size_t i = 0; i < items.size(); ++i) {
      if (items[i].off + items[i].n > size) {
        ::close(fd);
        throw std::runtime_error("ckpt_reader: item beyond the end of " + path);
      }
      if (i && items[i].off < items[i - 1].off + items[i - 1].n) {
        ::close(fd);
        throw std::runtime_error("ckpt_reader: overlapping items");
      }
    }
    const uint64_t nseg = (size + kSegBytes - 1) / kSegBytes;
    std::vector<char> want(nseg, 0), hash(nseg, 0);
    for (int64_t s : hash_segs) {
      if (s < 0 || (uint64_t)s >= nseg) {
        ::close(fd);
        throw std::runtime_error("ckpt_reader: hash segment out of range");
      }
      want[s] = hash[s] = 1;
    }
    for (auto& it : items)
      if (it.n)
        for (uint64_t s = it.off / kSegBytes; s <= (it.off + it.n - 1) / kSegBytes; ++s) want[s] = 1;
    std::vector<uint64_t> units;
    for (uint64_t s = 0; s < nseg; ++s)
      if (want[s]) units.push_back(s);
    r.seg_md5.assign(nseg, std::string());
    const int nt = std::max(1, std::min<int>(threads, (int)std::max<size_t>(units.size(), 1)));
    ensure_workers(nt);
    std::atomic<size_t> next{0};
    std::atomic<uint64_t> nread{0};
    std::atomic<bool> use_direct{r.direct};
    std::mutex err_mu;
    std::string err;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
      th.emplace_back([&, t] {
        Worker& w = workers_[t];
        EVP_MD_CTX* ctx = EVP_MD_CTX_new();
        int slot = 0;
        int bfd = -1;  // buffered fallback descriptor if O_DIRECT reads are refused
        try {
          if (device_ >= 0) hip_check(hipSetDevice(device_), "hipSetDevice");
          for (size_t u; (u = next.fetch_add(1)) < units.size();) {
            const uint64_t s = units[u];
            const uint64_t a = s * kSegBytes, b = std::min(size, a + kSegBytes);
            if (hash[s]) EVP_DigestInit_ex(ctx, EVP_md5(), nullptr);
            for (uint64_t c = a; c < b; c += kRead) {
              const uint64_t n = std::min(kRead, b - c);
              uint8_t* buf = w.buf[slot];
              if (device_ >= 0) hip_check(hipEventSynchronize(w.ev[slot]), "event sync");  // buffer free
              ssize_t got = -1;
              if (use_direct.load()) {
                got = pread_full(fd, buf, (n + 4095) & ~uint64_t(4095), c);
                if (got < 0 && errno == EINVAL) use_direct = false;
              }
              if (!use_direct.load()) {
                if (bfd < 0) bfd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
                got = bfd < 0 ? -1 : pread_full(bfd, buf, n, c);
              }
              if (got < (ssize_t)n) throw std::runtime_error("ckpt_reader: short read of " + path);
              nread += n;
              if (hash[s]) EVP_DigestUpdate(ctx, buf, n);
              // destination items overlapping [c, c + n)
              auto it = std::upper_bound(items.begin(), items.end(), c,
                                         [](uint64_t x, const ReadItem& i) { return x < i.off + i.n; });
              for (; it != items.end() && it->off < c + n; ++it) {
                const uint64_t lo = std::max(c, it->off), hi = std::min(c + n, it->off + it->n);
                void* dst = (void*)(it->dst + (lo - it->off));
                if (device_ >= 0)
                  hip_check(hipMemcpyAsync(dst, buf + (lo - c), hi - lo, hipMemcpyHostToDevice, w.stream),
                            "hipMemcpyAsync");
                else
                  std::memcpy(dst, buf + (lo - c), hi - lo);
              }
              if (device_ >= 0) hip_check(hipEventRecord(w.ev[slot], w.stream), "event record");
              slot ^= 1;
            }
            if (hash[s]) r.seg_md5[s] = digest_hex(ctx);
          }
          if (device_ >= 0) hip_check(hipStreamSynchronize(w.stream), "stream sync");
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> g(err_mu);
          if (err.empty()) err = e.what();
          if (device_ >= 0) (void)hipStreamSynchronize(w.stream);
        }
        if (bfd >= 0) ::close(bfd);
        EVP_MD_CTX_free(ctx);
      });
    }
    for (auto& x : th) x.join();
    ::close(fd);
    r.direct = r.direct && use_direct.load();
    r.bytes_read = nread.load();
    if (!err.empty()) throw std::runtime_error(err);
  }

  int device_;
  std::vector<Worker> workers_;
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
