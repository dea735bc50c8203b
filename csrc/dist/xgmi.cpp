// Host side of the intra-node direct all-reduce over xGMI (SURVEY §5.8 option (b); N12/N13):
// IPC-shared device buffers and events, peer copies, and the rank-ordered reduction launch.
// XgmiEngine (below) runs the per-bucket schedule natively: one comm stream, one pull-reduce and one
// pull-gather kernel per bucket, a C++ worker thread (no Python in the backward's critical path).
// Setup (IPC handles, events, the shared host page) lives in pyrecover_amd/parallel/xgmi.py.
//
// Memory: gradient buffers that peers read are allocated here with hipMalloc (exportable with
// hipIpcGetMemHandle) and handed to torch as a tensor that frees them on destruction.
// Synchronisation across processes uses interprocess HIP events (hipEventInterprocess):
// a peer's stream waits GPU-side on this rank's event; no kernel ever spins on a flag.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels/launchers.h"

namespace py = pybind11;

namespace {

void hchk(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "pyrecover_amd xgmi: ", what, " failed: ", hipGetErrorString(e));
}

at::Tensor ipc_empty(int64_t numel, at::ScalarType dtype, int64_t device) {
  TORCH_CHECK(numel > 0, "ipc_empty: numel must be positive");
  hchk(hipSetDevice((int)device), "hipSetDevice");
  const size_t bytes = (size_t)numel * c10::elementSize(dtype);
  void* p = nullptr;
  hchk(hipMalloc(&p, bytes), "hipMalloc");
  hchk(hipMemset(p, 0, bytes), "hipMemset");
  auto opts = at::TensorOptions().dtype(dtype).device(at::Device(at::kCUDA, (c10::DeviceIndex)device));
  return torch::from_blob(p, {numel}, [](void* q) { (void)hipFree(q); }, opts);
}

py::bytes ipc_mem_handle(const at::Tensor& t) {
  hipIpcMemHandle_t h;
  hchk(hipIpcGetMemHandle(&h, t.data_ptr()), "hipIpcGetMemHandle");
  return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

uintptr_t ipc_open_mem(py::bytes handle, int64_t device) {
  std::string s = handle;
  TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "ipc_open_mem: bad handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, s.data(), sizeof(h));
  hchk(hipSetDevice((int)device), "hipSetDevice");
  void* p = nullptr;
  hchk(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return (uintptr_t)p;
}

void ipc_close_mem(uintptr_t p) { (void)hipIpcCloseMemHandle((void*)p); }

uintptr_t ipc_event_create(int64_t device) {
  hchk(hipSetDevice((int)device), "hipSetDevice");
  hipEvent_t e;
  hchk(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventInterprocess), "hipEventCreate(ipc)");
  return (uintptr_t)e;
}

py::bytes ipc_event_handle(uintptr_t e) {
  hipIpcEventHandle_t h;
  hchk(hipIpcGetEventHandle(&h, (hipEvent_t)e), "hipIpcGetEventHandle");
  return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

uintptr_t ipc_event_open(py::bytes handle, int64_t device) {
  std::string s = handle;
  TORCH_CHECK(s.size() == sizeof(hipIpcEventHandle_t), "ipc_event_open: bad handle size");
  hipIpcEventHandle_t h;
  std::memcpy(&h, s.data(), sizeof(h));
  hchk(hipSetDevice((int)device), "hipSetDevice");
  hipEvent_t e;
  hchk(hipIpcOpenEventHandle(&e, h), "hipIpcOpenEventHandle");
  return (uintptr_t)e;
}

void event_destroy(uintptr_t e) { (void)hipEventDestroy((hipEvent_t)e); }
void event_record(uintptr_t e, uintptr_t stream) { hchk(hipEventRecord((hipEvent_t)e, (hipStream_t)stream), "record"); }
void stream_wait_event(uintptr_t stream, uintptr_t e) {
  hchk(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)e, 0), "hipStreamWaitEvent");
}
void event_synchronize(uintptr_t e) {
  py::gil_scoped_release nogil;
  hchk(hipEventSynchronize((hipEvent_t)e), "hipEventSynchronize");
}

// Device-to-device copy on `stream` (a peer pointer on either side is fine: the copy engines
// move it over xGMI and the runtime makes the bytes visible when the copy completes).
void copy_async(uintptr_t dst, uintptr_t src, int64_t nbytes, uintptr_t stream) {
  TORCH_CHECK(nbytes >= 0, "copy_async: negative size");
  if (nbytes == 0) return;
  hchk(hipMemcpyAsync((void*)dst, (const void*)src, (size_t)nbytes, hipMemcpyDeviceToDevice, (hipStream_t)stream),
       "hipMemcpyAsync");
}

// dst[0:n) = sum_r srcs[r][0:n) (fp32 accumulation in list order, one rounding).
void sum_slices(const std::vector<uintptr_t>& srcs, uintptr_t dst, int64_t n, at::ScalarType dtype, uintptr_t stream) {
  TORCH_CHECK(!srcs.empty() && srcs.size() <= 16, "sum_slices: 1..16 sources");
  int dtc = dtype == at::kFloat ? 0 : dtype == at::kBFloat16 ? 1 : dtype == at::kHalf ? 2 : -1;
  TORCH_CHECK(dtc >= 0, "sum_slices: unsupported dtype");
  if (n == 0) return;
  std::vector<const void*> v;
  for (auto p : srcs) v.push_back((const void*)p);
  hchk(pra_sum_slices(dtc, v.data(), (int)v.size(), (void*)dst, n, (hipStream_t)stream), "sum_slices");
}

// ------------------------------------------------------------------------------------------
// Native pull all-reduce engine: one comm stream, two kernels per bucket, a C++ worker thread.
//
// Per bucket b (slices: rank r owns elements [cut_r, cut_{r+1}) of the bucket):
//   1. the backward thread records ev_ready[b] on the compute stream and enqueues b (launch);
//   2. the worker publishes "ready b" in the shared host page, waits until every peer has published
//      its own (its ev_ready[b] of THIS step is recorded), makes the comm stream wait (GPU-side) on
//      every rank's ev_ready[b], and launches ONE reduce kernel that reads this rank's slice from all
//      W gradient buffers (peers' over xGMI, IPC-mapped) and sums them in rank order in fp32 into
//      its own buffer -- all links at once, no staging copy, deterministic;
//   3. it records ev_rs[b], publishes "reduced b", waits for every peer's, and launches ONE gather
//      kernel pulling every peer's reduced slice into this rank's buffer; ev_done[b] marks the end.
// end_step: no rank may overwrite its gradient buffer (next backward) before every peer has read it.
// Cross-process ordering: interprocess HIP events (GPU-side waits) + host sequence words that say an
// event has been recorded for this step (a wait on a not-yet-recorded event would pass at once).
class XgmiEngine {
 public:
  XgmiEngine(int device, int rank, int world, int dtype, int64_t esz, std::vector<uintptr_t> peer_base,
             std::vector<int64_t> cuts, uintptr_t seq_words, std::vector<uintptr_t> ev_ready,
             std::vector<uintptr_t> ev_rs, uintptr_t ev_step, std::vector<uintptr_t> peer_ready,
             std::vector<uintptr_t> peer_rs, std::vector<uintptr_t> peer_step)
      : dev_(device), rank_(rank), world_(world), dtype_(dtype), esz_(esz), base_(std::move(peer_base)),
        cuts_(std::move(cuts)), words_(reinterpret_cast<int64_t*>(seq_words)), ev_ready_(std::move(ev_ready)),
        ev_rs_(std::move(ev_rs)), ev_step_(ev_step), peer_ready_(std::move(peer_ready)),
        peer_rs_(std::move(peer_rs)), peer_step_(std::move(peer_step)) {
    nb_ = (int)ev_ready_.size();
    TORCH_CHECK(world_ >= 2 && world_ <= 16 && (int)base_.size() == world_, "XgmiEngine: 2..16 ranks");
    TORCH_CHECK((int64_t)cuts_.size() == (int64_t)nb_ * (world_ + 1), "XgmiEngine: cuts [nb][world + 1]");
    TORCH_CHECK((int)peer_ready_.size() == world_ * nb_ && (int)peer_rs_.size() == world_ * nb_ &&
                    (int)peer_step_.size() == world_,
                "XgmiEngine: peer events");
    hchk(hipSetDevice(dev_), "hipSetDevice");
    int lo = 0, hi = 0;
    hchk(hipDeviceGetStreamPriorityRange(&lo, &hi), "priority range");
    hchk(hipStreamCreateWithPriority(&comm_, hipStreamNonBlocking, hi), "comm stream");
    done_.resize(nb_);
    for (auto& e : done_) hchk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event create");
    processed_.assign(nb_, 0);
    worker_ = std::thread([this] { run(); });
  }
  ~XgmiEngine() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
    for (auto e : done_) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(comm_);
  }
  int64_t seq() const { return seq_; }

  // backward thread: bucket b's gradients are enqueued on `cur`. Returns the step's sequence
  // number, the ticket wait() takes (a bucket may be waited on after end_step moved to the next)
  int64_t launch(int b, uintptr_t cur) {
    TORCH_CHECK(b >= 0 && b < nb_, "XgmiEngine.launch: bucket index");
    hchk(hipEventRecord((hipEvent_t)ev_ready_[b], (hipStream_t)cur), "record ready");
    push(b);
    std::lock_guard<std::mutex> g(mu_);
    return seq_;
  }
  // `cur` waits (GPU-side) for bucket b's all-reduce of step `seq`; blocks the host only until the
  // worker has enqueued it
  void wait(int b, int64_t seq, uintptr_t cur) {
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> g(mu_);
      if (!cv_done_.wait_for(g, std::chrono::seconds(600), [&] { return processed_[b] >= seq || !err_.empty(); }) &&
          err_.empty())
        err_ = "bucket " + std::to_string(b) + " of step " + std::to_string(seq) + " not processed in 600 s";
    }
    check_err();
    hchk(hipStreamWaitEvent((hipStream_t)cur, done_[b], 0), "wait done");
  }
  void end_step(uintptr_t cur) {
    push(kStep);
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> g(mu_);
      if (!cv_done_.wait_for(g, std::chrono::seconds(600), [&] { return step_done_ >= seq_ || !err_.empty(); }) &&
          err_.empty())
        err_ = "step barrier " + std::to_string(seq_) + " not reached in 600 s";
    }
    check_err();
    for (int r = 0; r < world_; ++r)
      if (r != rank_) hchk(hipStreamWaitEvent((hipStream_t)cur, (hipEvent_t)peer_step_[r], 0), "wait step");
    std::lock_guard<std::mutex> g(mu_);
    ++seq_;
  }

 private:
  static constexpr int kStep = -1;
  void push(int item) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(item);
    }
    cv_.notify_one();
  }
  void check_err() {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(err_.empty(), "xgmi all-reduce failed: ", err_);
  }
  int64_t& word(int r, int slot) { return words_[(int64_t)r * (2 * nb_ + 1) + slot]; }
  void publish(int slot, int64_t v) { __atomic_store_n(&word(rank_, slot), v, __ATOMIC_RELEASE); }
  void wait_word(int r, int slot, int64_t v) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int spins = 0; __atomic_load_n(&word(r, slot), __ATOMIC_ACQUIRE) < v; ++spins) {
      if (spins > 200) std::this_thread::sleep_for(std::chrono::microseconds(20));
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600))
        throw std::runtime_error("xgmi: rank " + std::to_string(r) + " did not publish slot " + std::to_string(slot));
    }
  }
  void bucket(int b, int64_t seq) {
    const int64_t* c = cuts_.data() + (int64_t)b * (world_ + 1);
    const int64_t s0 = c[rank_], n = c[rank_ + 1] - s0;
    hipStream_t st = comm_;
    // reduce-scatter: every rank's bucket b is complete (GPU-side waits), then one pull-reduce
    publish(b, seq);
    hchk(hipStreamWaitEvent(st, (hipEvent_t)ev_ready_[b], 0), "wait own ready");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      wait_word(r, b, seq);
      hchk(hipStreamWaitEvent(st, (hipEvent_t)peer_ready_[(int64_t)r * nb_ + b], 0), "wait peer ready");
    }
    std::vector<const void*> srcs(world_);
    for (int r = 0; r < world_; ++r) srcs[r] = (const void*)(base_[r] + s0 * esz_);
    if (n > 0) hchk(pra_sum_slices(dtype_, srcs.data(), world_, (void*)(base_[rank_] + s0 * esz_), n, st), "pull reduce");
    hchk(hipEventRecord((hipEvent_t)ev_rs_[b], st), "record reduced");
    publish(nb_ + b, seq);
    // all-gather: every owner has reduced its slice, then one pull of all peers' slices
    std::vector<const void*> gs;
    std::vector<void*> gd;
    std::vector<long> gn;
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      wait_word(r, nb_ + b, seq);
      hchk(hipStreamWaitEvent(st, (hipEvent_t)peer_rs_[(int64_t)r * nb_ + b], 0), "wait peer reduced");
      const int64_t p0 = c[r], pn = c[r + 1] - p0;
      if (pn > 0) {
        gs.push_back((const void*)(base_[r] + p0 * esz_));
        gd.push_back((void*)(base_[rank_] + p0 * esz_));
        gn.push_back((long)(pn * esz_));
      }
    }
    hchk(pra_pull_gather(gs.data(), gd.data(), gn.data(), (int)gs.size(), st), "pull gather");
    hchk(hipEventRecord(done_[b], st), "record done");
  }
  void step(int64_t seq) {
    hchk(hipEventRecord((hipEvent_t)ev_step_, comm_), "record step");
    publish(2 * nb_, seq);
    for (int r = 0; r < world_; ++r)
      if (r != rank_) wait_word(r, 2 * nb_, seq);
  }
  void run() {
    (void)hipSetDevice(dev_);
    for (;;) {
      int item;
      int64_t seq;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        item = q_.front();
        q_.pop_front();
        seq = seq_;
      }
      try {
        if (item == kStep) step(seq);
        else bucket(item, seq);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu_);
        if (err_.empty()) err_ = e.what();
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        if (item == kStep) step_done_ = seq;
        else processed_[item] = seq;
      }
      cv_done_.notify_all();
    }
  }

  int dev_, rank_, world_, dtype_, nb_ = 0;
  int64_t esz_;
  std::vector<uintptr_t> base_;
  std::vector<int64_t> cuts_;
  int64_t* words_;
  std::vector<uintptr_t> ev_ready_, ev_rs_;
  uintptr_t ev_step_;
  std::vector<uintptr_t> peer_ready_, peer_rs_, peer_step_;
  hipStream_t comm_ = nullptr;
  std::vector<hipEvent_t> done_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_, cv_done_;
  std::deque<int> q_;
  std::vector<int64_t> processed_;
  int64_t step_done_ = 0;
  int64_t seq_ = 1;  // current step's sequence number (published values start at 1)
  bool stop_ = false;
  std::string err_;
};

}  // namespace

void register_xgmi(py::module& m) {
  auto x = m.def_submodule("xgmi", "IPC buffers/events + peer copies for the direct xGMI all-reduce");
  x.def("ipc_empty", &ipc_empty);
  x.def("ipc_mem_handle", &ipc_mem_handle);
  x.def("ipc_open_mem", &ipc_open_mem);
  x.def("ipc_close_mem", &ipc_close_mem);
  x.def("ipc_event_create", &ipc_event_create);
  x.def("ipc_event_handle", &ipc_event_handle);
  x.def("ipc_event_open", &ipc_event_open);
  x.def("event_destroy", &event_destroy);
  x.def("event_record", &event_record);
  x.def("stream_wait_event", &stream_wait_event);
  x.def("event_synchronize", &event_synchronize);
  x.def("copy_async", &copy_async);
  x.def("sum_slices", &sum_slices);
  py::class_<XgmiEngine>(x, "XgmiEngine")
      .def(py::init<int, int, int, int, int64_t, std::vector<uintptr_t>, std::vector<int64_t>, uintptr_t,
                    std::vector<uintptr_t>, std::vector<uintptr_t>, uintptr_t, std::vector<uintptr_t>,
                    std::vector<uintptr_t>, std::vector<uintptr_t>>(),
           py::arg("device"), py::arg("rank"), py::arg("world"), py::arg("dtype"), py::arg("esz"),
           py::arg("peer_base"), py::arg("cuts"), py::arg("seq_words"), py::arg("ev_ready"), py::arg("ev_rs"),
           py::arg("ev_step"), py::arg("peer_ready"), py::arg("peer_rs"), py::arg("peer_step"))
      .def("launch", &XgmiEngine::launch)
      .def("wait", &XgmiEngine::wait)
      .def("end_step", &XgmiEngine::end_step)
      .def("seq", &XgmiEngine::seq);
}
