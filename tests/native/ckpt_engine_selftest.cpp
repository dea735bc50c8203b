// Standalone self-test of the checkpoint engine core (csrc/runtime/ckpt_engine.h) in CPU mode
// (device -1: no HIP calls), built with -fsanitize=address,undefined or -fsanitize=thread by
// tests/test_native_sanitizers.py. Exercises: pool reserve, parallel host staging, the writer
// threads (zip records + raw blob in one file, CRC32 pieces, parallel segment writes + MD5s,
// whole-file MD5, tmp+rename, .md5 sidecar), the deferred whole-file digest (third round: the job
// returns before the `.md5` exists; the caller's raw bytes are freed before flush()), the parallel
// Reader (O_DIRECT and buffered), the error paths, and back-to-back jobs reusing the pool.
// usage: ckpt_engine_selftest <out_dir>   -> exit 0 on success; writes <out_dir>/t.bin
#include "runtime/ckpt_engine.h"

#include <cstdio>
#include <fstream>
#include <random>
#include <sstream>

using namespace pra::ckpt;

#define REQUIRE(c)                                                             \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "REQUIRE failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

static std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string dir = argv[1];
  std::mt19937_64 rng(1234);
  // three "tensors" (one larger than the 16 MiB CRC piece so the parallel CRC path runs)
  std::vector<std::vector<uint8_t>> src = {std::vector<uint8_t>(1000), std::vector<uint8_t>(40u << 20),
                                           std::vector<uint8_t>(77)};
  for (auto& v : src)
    for (auto& b : v) b = (uint8_t)rng();
  std::vector<uint8_t> raw(4096);
  for (auto& b : raw) b = (uint8_t)rng();

  CkptEngine eng(-1);
  eng.reserve(64u << 20);
  for (int round = 0; round < 3; ++round) {  // the pool is reused by later jobs; round 2 defers the .md5
    std::vector<std::pair<uintptr_t, uint64_t>> regions;
    for (auto& v : src) regions.push_back({(uintptr_t)v.data(), v.size()});
    const auto offs = eng.stage(regions, nullptr);
    REQUIRE(offs.size() == 3 && offs[0] % 64 == 0 && offs[1] % 64 == 0 && offs[2] % 64 == 0);
    REQUIRE(eng.staged_complete());
    const uintptr_t pool = eng.pool_ptr();
    for (size_t i = 0; i < src.size(); ++i) REQUIRE(std::memcmp((void*)(pool + offs[i]), src[i].data(), src[i].size()) == 0);
    Item zip;
    for (size_t i = 0; i < src.size(); ++i)
      zip.records.push_back({"archive/data/" + std::to_string(i), pool + offs[i], src[i].size()});
    const bool defer = round == 2;
    std::vector<uint8_t>* raw_copy = new std::vector<uint8_t>(raw);  // caller-owned, freed after wait()
    Item rawi;
    rawi.raw = true;
    rawi.ptr = (uintptr_t)raw_copy->data();
    rawi.n = raw_copy->size();
    const std::string path = dir + "/t.bin";
    eng.write_items(path, {zip, rawi}, /*md5=*/true, /*fsync=*/round == 0, defer);
    JobResult r = eng.wait();
    std::memset(raw_copy->data(), 0xEE, raw_copy->size());
    delete raw_copy;
    REQUIRE(r.ok);
    REQUIRE(r.md5_deferred == defer);
    if (defer) {
      REQUIRE(eng.flush().empty());
      r.md5 = slurp(path + ".md5");
      REQUIRE(r.md5.size() == 32);
    }
    REQUIRE(r.items.size() == 2);
    const std::string file = slurp(path);
    REQUIRE(file.size() == r.bytes);
    REQUIRE(r.items[1].second == raw.size());
    REQUIRE(std::memcmp(file.data() + r.items[1].first, raw.data(), raw.size()) == 0);
    REQUIRE(file.compare(0, 4, "PK\x03\x04") == 0);
    REQUIRE(md5_file(path) == r.md5);
    REQUIRE(slurp(path + ".md5") == r.md5);
    REQUIRE(access((path + ".tmp").c_str(), F_OK) != 0);
    REQUIRE(r.seg_md5.size() == (r.bytes + kSegBytes - 1) / kSegBytes);
    // every zip record's payload sits at the reported offset
    REQUIRE(r.records.size() == 3);
    for (size_t i = 0; i < src.size(); ++i)
      REQUIRE(std::memcmp(file.data() + r.records[i].data_off, src[i].data(), src[i].size()) == 0);
    // parallel reader (CPU mode, several threads): payloads back into fresh buffers, segment hash
    std::vector<std::vector<uint8_t>> back(src.size());
    std::vector<ReadItem> ri;
    for (size_t i = 0; i < src.size(); ++i) {
      back[i].assign(src[i].size(), 0);
      ri.push_back({r.records[i].data_off, src[i].size(), (uintptr_t)back[i].data()});
    }
    Reader rd(-1);
    const ReadResult rr = rd.read(path, ri, {0}, 4, /*direct=*/round == 0);
    REQUIRE(rr.ok);
    REQUIRE(rr.seg_md5.size() == r.seg_md5.size() && rr.seg_md5[0] == r.seg_md5[0]);
    for (size_t i = 0; i < src.size(); ++i) REQUIRE(back[i] == src[i]);
    // an item past the end of the file is an error, not a fault
    const ReadResult bad_rd = rd.read(path, {{r.bytes - 4, 64, (uintptr_t)back[0].data()}}, {}, 2, false);
    REQUIRE(!bad_rd.ok && !bad_rd.error.empty());
  }
  // an abandoned deferred digest (time-aware stop at the wall-clock limit) is cancelled and
  // joined: after abandon_md5() no digest thread runs, and the sidecar is either absent (cancelled)
  // or correct (finished first); the engine can then be destroyed at once
  {
    std::vector<uint8_t> big(96u << 20);
    for (size_t i = 0; i < big.size(); i += 8) big[i] = (uint8_t)rng();
    auto* e2 = new CkptEngine(-1);
    e2->reserve(big.size());
    const auto o2 = e2->stage({{(uintptr_t)big.data(), big.size()}}, nullptr);
    Item z2;
    z2.records.push_back({"archive/data/0", e2->pool_ptr() + o2[0], big.size()});
    const std::string p2 = dir + "/abandoned.bin";
    e2->write_items(p2, {z2}, /*md5=*/true, /*fsync=*/false, /*defer_md5=*/true);
    REQUIRE(e2->wait().ok);
    e2->abandon_md5();
    REQUIRE(!e2->md5_pending());
    REQUIRE(e2->flush().empty());  // cancelled is not an error
    delete e2;
    REQUIRE(access((p2 + ".md5").c_str(), F_OK) != 0 || slurp(p2 + ".md5") == md5_file(p2));
    // a later save on the same engine digests again (cancel is reset)
  }
  // a deferred digest whose file was deleted (retention) or replaced (same path saved again)
  // while it ran writes no sidecar: no orphan `.md5`, no stale digest over the new file
  {
    std::vector<uint8_t> big(128u << 20);
    for (size_t i = 0; i < big.size(); i += 8) big[i] = (uint8_t)rng();
    CkptEngine e3(-1);
    e3.reserve(big.size());
    const auto o3 = e3.stage({{(uintptr_t)big.data(), big.size()}}, nullptr);
    Item z3;
    z3.records.push_back({"archive/data/0", e3.pool_ptr() + o3[0], big.size()});
    const std::string p3 = dir + "/deleted.bin";
    e3.write_items(p3, {z3}, true, false, true);
    REQUIRE(e3.wait().ok);
    REQUIRE(::unlink(p3.c_str()) == 0);  // retention removes it while the digest reads
    REQUIRE(e3.flush().empty());
    REQUIRE(access((p3 + ".md5").c_str(), F_OK) != 0);
    const std::string p4 = dir + "/replaced.bin";
    e3.write_items(p4, {z3}, true, false, true);
    REQUIRE(e3.wait().ok);
    {
      std::ofstream f(p4 + ".new", std::ios::binary);
      f << "replacement";
    }
    REQUIRE(::rename((p4 + ".new").c_str(), p4.c_str()) == 0);  // a new file at the same path
    REQUIRE(e3.flush().empty());
    REQUIRE(access((p4 + ".md5").c_str(), F_OK) != 0);
  }
  // error path: unwritable destination -> ok=false, message, nothing left behind
  eng.write_items(dir + "/no/such/dir/x.bin", {}, true, false);
  const JobResult bad = eng.wait();
  REQUIRE(!bad.ok && !bad.error.empty());
  std::printf("ckpt_engine selftest ok\n");
  return 0;
}
