// pybind11 bindings of the host runtime: netsdb_amd._native
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"

namespace py = pybind11;
using namespace nsdb_rt;

static py::dict spec_dict(const TupleSpec& t) {
  py::dict d;
  d["name"] = t.name;
  d["atts"] = t.atts;
  return d;
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "netsdb_amd host runtime: TCAP parser, buffer manager, page files, slab allocator, hashing";

  m.def("parse_tcap", [](const std::string& text) {
    std::vector<AtomicComputation> atoms;
    {
      py::gil_scoped_release rel;
      atoms = parse_tcap(text);
    }
    py::list out;
    for (const auto& a : atoms) {
      py::dict d;
      d["type"] = a.type;
      d["output"] = spec_dict(a.output);
      d["input"] = spec_dict(a.input);
      d["projection"] = spec_dict(a.projection);
      d["input2"] = spec_dict(a.input2);
      d["projection2"] = spec_dict(a.projection2);
      d["comp"] = a.comp;
      d["lambda"] = a.lambda;
      d["db"] = a.db;
      d["set"] = a.set;
      d["line"] = a.line;
      out.append(d);
    }
    return out;
  });

  py::class_<SlabAllocator>(m, "SlabAllocator")
      .def(py::init<uint64_t, uint64_t>(), py::arg("capacity"), py::arg("alignment") = 256)
      .def("alloc", &SlabAllocator::alloc)
      .def("free", &SlabAllocator::free)
      .def_property_readonly("capacity", &SlabAllocator::capacity)
      .def_property_readonly("used", &SlabAllocator::used)
      .def_property_readonly("largest_free", &SlabAllocator::largest_free)
      .def_property_readonly("num_allocations", &SlabAllocator::num_allocations);

  py::class_<PageFile>(m, "PageFile")
      .def(py::init<const std::string&, uint64_t>())
      .def("write_page", [](PageFile& f, uint64_t p, py::buffer b) {
        py::buffer_info bi = b.request();
        f.write_page(p, bi.ptr, (uint64_t)(bi.size * bi.itemsize));
      })
      .def("read_page", [](PageFile& f, uint64_t p) {
        std::string buf(f.page_size(), '\0');
        uint64_t n = f.read_page(p, buf.data(), f.page_size());
        return py::bytes(buf.data(), n);
      })
      .def("has_page", &PageFile::has_page)
      .def("pages", &PageFile::pages)
      .def("sync", &PageFile::sync)
      .def_property_readonly("page_size", &PageFile::page_size);

  py::class_<BufferManager>(m, "BufferManager")
      .def(py::init<uint64_t, uint64_t, const std::string&>(), py::arg("page_size"), py::arg("num_pages"),
           py::arg("spill_dir"))
      .def("pin", &BufferManager::pin, py::arg("set_id"), py::arg("page_no"), py::arg("create") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("unpin", &BufferManager::unpin, py::arg("set_id"), py::arg("page_no"), py::arg("dirty") = false,
           py::arg("bytes_used") = 0, py::call_guard<py::gil_scoped_release>())
      .def("slot_view", [](BufferManager& b, int64_t slot) {
        return py::memoryview::from_memory(b.slot_ptr(slot), (ssize_t)b.page_size(), false);
      })
      .def("drop_set", &BufferManager::drop_set)
      .def("drop_page", &BufferManager::drop_page)
      .def("flush_set", &BufferManager::flush_set, py::call_guard<py::gil_scoped_release>())
      .def("flush_all", &BufferManager::flush_all, py::call_guard<py::gil_scoped_release>())
      .def("prefetch", &BufferManager::prefetch, py::call_guard<py::gil_scoped_release>())
      .def("bytes_used", &BufferManager::bytes_used)
      .def("set_pages", &BufferManager::set_pages)
      .def_property_readonly("page_size", &BufferManager::page_size)
      .def_property_readonly("num_slots", &BufferManager::num_slots)
      .def_property_readonly("resident_pages", &BufferManager::resident_pages)
      .def_property_readonly("evictions", &BufferManager::evictions)
      .def_property_readonly("loads", &BufferManager::loads)
      .def_property_readonly("spill_dir", &BufferManager::spill_dir);

  py::class_<Buzzer, std::shared_ptr<Buzzer>>(m, "Buzzer")
      .def("wait", &Buzzer::wait, py::arg("timeout") = -1.0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("done", &Buzzer::done)
      .def_property_readonly("error", &Buzzer::error);

  py::class_<WorkerQueue>(m, "WorkerQueue")
      .def(py::init<int>(), py::arg("num_workers") = 4)
      .def("submit_flush", [](WorkerQueue& q, BufferManager& bm, int64_t set_id) {
        return q.submit([&bm, set_id] { bm.flush_set(set_id); });
      }, py::keep_alive<0, 2>())
      .def("submit_prefetch", [](WorkerQueue& q, BufferManager& bm, int64_t set_id, std::vector<int64_t> pages) {
        return q.submit([&bm, set_id, pages] {
          for (int64_t p : pages) bm.prefetch(set_id, p);
        });
      }, py::keep_alive<0, 2>())
      .def("drain", &WorkerQueue::drain, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("num_workers", &WorkerQueue::num_workers)
      .def_property_readonly("completed", &WorkerQueue::completed)
      .def_property_readonly("pending", &WorkerQueue::pending);

  m.def("hash_columns", [](std::vector<py::array_t<int64_t, py::array::c_style | py::array::forcecast>> cols) {
    if (cols.empty()) throw std::runtime_error("hash_columns: no columns");
    const int64_t n = (int64_t)cols[0].size();
    std::vector<const int64_t*> ptrs;
    for (auto& c : cols) {
      if ((int64_t)c.size() != n) throw std::runtime_error("hash_columns: length mismatch");
      ptrs.push_back(c.data());
    }
    py::array_t<uint64_t> out(n);
    {
      py::gil_scoped_release rel;
      hash_columns(ptrs.data(), (int)ptrs.size(), n, out.mutable_data());
    }
    return out;
  });
  m.def("partition_ids", [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> h, int nparts) {
    if (nparts <= 0) throw std::runtime_error("partition_ids: nparts must be > 0");
    py::array_t<int32_t> out(h.size());
    partition_ids(h.data(), (int64_t)h.size(), nparts, out.mutable_data());
    return out;
  });
  m.def("hash64", &hash64);
}
