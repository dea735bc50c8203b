// Python bindings of the checkpoint engine (core: ckpt_engine.h). The torch adapter supplies the
// caller's current HIP stream to stage()/fence() and releases the GIL around blocking calls.
#include "runtime/ckpt_engine.h"

#include <c10/hip/HIPStream.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;
using namespace pra::ckpt;


void register_ckpt_engine(py::module& m) {
  py::class_<CkptEngine>(m, "CkptEngine")
      .def(py::init<int>())
      .def("reserve", &CkptEngine::reserve, py::call_guard<py::gil_scoped_release>())
      .def("pool_ptr", &CkptEngine::pool_ptr)
      .def("pool_size", &CkptEngine::pool_size)
      .def("stage",
           [](CkptEngine& e, const std::vector<std::pair<uintptr_t, uint64_t>>& regions, uintptr_t hbm,
              uint64_t hbm_bytes) {
             const int dev = e.device();
             return e.stage(regions, dev >= 0 ? c10::hip::getCurrentHIPStream(dev).stream() : nullptr, hbm,
                            hbm_bytes);
           },
           py::arg("regions"), py::arg("hbm") = 0, py::arg("hbm_bytes") = 0)
      .def("last_two_hop", &CkptEngine::last_two_hop)
      .def("fence",
           [](CkptEngine& e) {
             const int dev = e.device();
             if (dev >= 0) e.fence(c10::hip::getCurrentHIPStream(dev).stream());
           })
      .def("sync_stage", &CkptEngine::sync_stage, py::call_guard<py::gil_scoped_release>())
      .def("staged_complete", &CkptEngine::staged_complete)
      .def("write_items",
           [](CkptEngine& e, const std::string& path, py::list items, bool md5, bool fsync, bool defer_md5) {
             // items: [("raw", ptr, nbytes) | ("zip", [(name, ptr, nbytes), ...])]
             std::vector<Item> v;
             for (auto h : items) {
               auto t = h.cast<py::tuple>();
               Item it;
               const std::string kind = t[0].cast<std::string>();
               if (kind == "raw") {
                 it.raw = true;
                 it.ptr = t[1].cast<uintptr_t>();
                 it.n = t[2].cast<uint64_t>();
               } else if (kind == "zip") {
                 for (auto rh : t[1].cast<py::list>()) {
                   auto rt = rh.cast<py::tuple>();
                   it.records.push_back({rt[0].cast<std::string>(), rt[1].cast<uintptr_t>(), rt[2].cast<uint64_t>()});
                 }
               } else {
                 throw std::runtime_error("write_items: unknown item kind " + kind);
               }
               v.push_back(std::move(it));
             }
             e.write_items(path, std::move(v), md5, fsync, defer_md5);
           },
           py::arg("path"), py::arg("items"), py::arg("md5"), py::arg("fsync"), py::arg("defer_md5") = false)
      .def("busy", &CkptEngine::busy)
      .def("flush", &CkptEngine::flush, py::call_guard<py::gil_scoped_release>())
      .def("md5_pending", &CkptEngine::md5_pending)
      .def("abandon_md5", &CkptEngine::abandon_md5, py::call_guard<py::gil_scoped_release>())
      .def("md5_max_seconds", &CkptEngine::md5_max_seconds)
      .def("md5_min_bps", &CkptEngine::md5_min_bps)
      .def("md5_pending_bytes", &CkptEngine::md5_pending_bytes)
      .def("progress", &CkptEngine::progress)
      .def("wait", [](CkptEngine& e) {
        JobResult r;
        {
          py::gil_scoped_release nogil;
          r = e.wait();
        }
        py::dict d;
        d["ok"] = r.ok;
        d["error"] = r.error;
        d["md5"] = r.md5;
        d["bytes"] = r.bytes;
        d["seconds"] = r.seconds;
        d["stage_wait_seconds"] = r.stage_wait_seconds;
        d["layout_seconds"] = r.layout_seconds;
        d["write_seconds"] = r.write_seconds;
        d["fsync_seconds"] = r.fsync_seconds;
        d["writers"] = r.writers;
        d["direct"] = r.direct;
        py::list items;
        for (auto& it : r.items) items.append(py::make_tuple(it.first, it.second));
        d["items"] = items;
        py::list recs;
        for (auto& rc : r.records) recs.append(py::make_tuple(rc.name, rc.data_off, rc.nbytes));
        d["records"] = recs;
        d["seg_bytes"] = r.seg_bytes;
        d["seg_md5"] = r.seg_md5;
        d["md5_deferred"] = r.md5_deferred;
        return d;
      });
  py::class_<Reader>(m, "CkptReader")
      .def(py::init<int>())
      .def("read",
           [](Reader& rd, const std::string& path, const std::vector<std::tuple<uint64_t, uint64_t, uintptr_t>>& items,
              const std::vector<int64_t>& hash_segs, int threads, bool direct) {
             // items: (file offset, nbytes, destination pointer: device memory, or host memory in CPU mode)
             std::vector<ReadItem> v;
             v.reserve(items.size());
             for (auto& t : items) v.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
             ReadResult r;
             {
               py::gil_scoped_release nogil;
               r = rd.read(path, std::move(v), hash_segs, threads, direct);
             }
             py::dict d;
             d["ok"] = r.ok;
             d["error"] = r.error;
             d["seg_md5"] = r.seg_md5;
             d["bytes_read"] = r.bytes_read;
             d["seconds"] = r.seconds;
             d["direct"] = r.direct;
             return d;
           });
  m.attr("MD5PARTS_SEGMENT_BYTES") = py::int_(kSegBytes);
  m.def("md5_file", &md5_file, py::call_guard<py::gil_scoped_release>());
  m.def("md5_probe_bps", &md5_probe_bps, py::arg("nbytes"), py::call_guard<py::gil_scoped_release>());
  m.def("write_probe_bps", &write_probe_bps, py::arg("path"), py::arg("nbytes"), py::arg("threads") = kWriters,
        py::arg("fsync") = true, py::call_guard<py::gil_scoped_release>());
  m.attr("CKPT_WRITERS") = py::int_(kWriters);
  m.def("crc32_bytes", [](py::bytes b) {
    std::string s = b;
    return crc32_parallel(0, (const uint8_t*)s.data(), s.size());
  });
}
