// Host side of the intra-node direct all-reduce over xGMI (SURVEY §5.8 option (b); N12/N13):
// IPC-shared device buffers and events, peer copies, and the rank-ordered reduction launch.
// Orchestration (bucket schedule, host barriers, comm thread) lives in
// pyrecover_amd/parallel/xgmi.py; this file only wraps HIP runtime calls with checks.
//
// Memory: gradient buffers that peers read are allocated here with hipMalloc (exportable with
// hipIpcGetMemHandle) and handed to torch as a tensor that frees them on destruction.
// Synchronisation across processes uses interprocess HIP events (hipEventInterprocess):
// a peer's stream waits GPU-side on this rank's event; no kernel ever spins on a flag.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstring>
#include <string>
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
}
