// pybind11 bindings of the host runtime: `_cgs_runtime`.
//
//   SafeTensorsFile(path): keys(), metadata(), info(name) -> (dtype, shape, nbytes),
//                          tensor(name) -> (dtype, shape, buffer)  [zero-copy, keeps the mmap alive]
//                          read_into(names, addresses, threads)    [parallel copy into host memory]
//   save_safetensors(path, [(name, dtype, shape, bytes)], metadata)
//   BPE(merges, vocab).encode_word(word) -> [ids]
//   blake3_hex(bytes) / blake3_file_hex(path)
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"

namespace py = pybind11;
using namespace cgs;

namespace {

// A byte range of a mapped file exported through the buffer protocol; holds the mapping alive.
struct Span {
  std::shared_ptr<MappedFile> owner;
  uint8_t* ptr;
  size_t n;
};

}  // namespace

PYBIND11_MODULE(_cgs_runtime, m) {
  m.doc() = "comfy_gen_server_amd native host runtime (safetensors, BPE, BLAKE3)";

  py::class_<Span>(m, "Span", py::buffer_protocol())
      .def_buffer([](Span& s) -> py::buffer_info {
        return py::buffer_info(s.ptr, 1, py::format_descriptor<uint8_t>::format(), 1, {py::ssize_t(s.n)}, {1},
                               /*readonly=*/false);
      })
      .def("__len__", [](const Span& s) { return s.n; });

  py::class_<SafeTensors, std::shared_ptr<SafeTensors>>(m, "SafeTensorsFile")
      .def(py::init<const std::string&>(), py::call_guard<py::gil_scoped_release>())
      .def("keys", &SafeTensors::keys)
      .def("metadata", &SafeTensors::metadata)
      .def("info",
           [](const SafeTensors& f, const std::string& k) {
             const TensorInfo& t = f.info(k);
             return py::make_tuple(t.dtype, t.shape, t.end - t.begin);
           })
      .def("tensor",
           [](const SafeTensors& f, const std::string& k) {
             const TensorInfo& t = f.info(k);
             Span s{f.file(), f.tensor_ptr(k), size_t(t.end - t.begin)};
             return py::make_tuple(t.dtype, t.shape, py::memoryview(py::cast(s)));
           })
      .def("offsets",
           [](const SafeTensors& f, const std::string& k) {
             const TensorInfo& t = f.info(k);
             return py::make_tuple(t.begin, t.end);
           })
      .def("data_section",
           [](const SafeTensors& f) {
             // (address, size, keep-alive span): the address stays valid while the span lives
             Span s{f.file(), f.data_section(), f.data_section_size()};
             return py::make_tuple(reinterpret_cast<uintptr_t>(s.ptr), s.n, py::cast(s));
           })
      .def("read_into",
           [](const SafeTensors& f, const std::vector<std::string>& names, const std::vector<uintptr_t>& addrs,
              int threads) {
             if (names.size() != addrs.size()) throw std::invalid_argument("names/addresses length mismatch");
             std::vector<std::pair<std::string, uint8_t*>> dst;
             dst.reserve(names.size());
             for (size_t i = 0; i < names.size(); ++i) dst.emplace_back(names[i], reinterpret_cast<uint8_t*>(addrs[i]));
             py::gil_scoped_release nogil;
             f.copy_many(dst, threads);
           },
           py::arg("names"), py::arg("addresses"), py::arg("threads") = 8);

  m.def("save_safetensors",
        [](const std::string& path, const std::vector<py::tuple>& items, const std::map<std::string, std::string>& meta) {
          std::vector<SaveItem> v;
          v.reserve(items.size());
          for (auto& t : items) {
            SaveItem s;
            s.name = t[0].cast<std::string>();
            s.dtype = t[1].cast<std::string>();
            s.shape = t[2].cast<std::vector<int64_t>>();
            s.bytes = t[3].cast<std::string>();
            v.push_back(std::move(s));
          }
          py::gil_scoped_release nogil;
          save_safetensors(path, v, meta);
        });

  py::class_<BPE>(m, "BPE")
      .def(py::init<const std::vector<std::string>&, const std::vector<std::string>&>())
      .def("encode_word", &BPE::encode_word)
      .def("vocab_size", &BPE::vocab_size);

  py::class_<Arena>(m, "Arena")
      .def(py::init<uint64_t, uint64_t>(), py::arg("capacity"), py::arg("align") = 256)
      .def("alloc", &Arena::alloc)
      .def("free", &Arena::free)
      .def_property_readonly("align", &Arena::align)
      .def("stats", [](const Arena& a) {
        const ArenaStats s = a.stats();
        py::dict d;
        d["capacity"] = s.capacity;
        d["used"] = s.used;
        d["peak"] = s.peak;
        d["largest_free"] = s.largest_free;
        d["free_blocks"] = s.free_blocks;
        d["live_blocks"] = s.live_blocks;
        return d;
      });

  m.def("blake3_hex", [](py::bytes data, size_t out_len) {
    std::string s = data;
    py::gil_scoped_release nogil;
    return blake3_hex(reinterpret_cast<const uint8_t*>(s.data()), s.size(), out_len);
  }, py::arg("data"), py::arg("out_len") = 32);
  m.def("blake3_file_hex", [](const std::string& path) {
    py::gil_scoped_release nogil;
    return blake3_file_hex(path);
  });
}
