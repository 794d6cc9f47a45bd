// pybind11 module `_tpi_native`: host-side native runtime pieces.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>

#include "ctl.h"
#include "filter.h"
#include "../common/tpz.h"
#include "fileio.h"
#include "hostops.h"
#include "transfer.h"

namespace py = pybind11;

namespace {

const tpi_seg* seg_ptr(py::buffer& b, int& n) {
  py::buffer_info info = b.request();
  if (info.size * info.itemsize % (py::ssize_t)sizeof(tpi_seg))
    throw std::invalid_argument("segment buffer size is not a multiple of sizeof(tpi_seg)");
  n = (int)(info.size * info.itemsize / sizeof(tpi_seg));
  return (const tpi_seg*)info.ptr;
}

}  // namespace

PYBIND11_MODULE(_tpi_native, m) {
  m.doc() = "Host-side native runtime of the MI355X task orchestrator";
  m.attr("SEG_SIZE") = (int)sizeof(tpi_seg);
#ifdef TPI_VERSION_STRING
  m.attr("VERSION") = TPI_VERSION_STRING;
#else
  m.attr("VERSION") = "0.0.0-dev";
#endif

  py::class_<tpi::Filter>(m, "Filter")
      .def(py::init<>())
      .def(py::init([](const std::vector<std::string>& rules) {
        tpi::Filter f;
        for (auto& r : rules) f.add_rule(r);
        return f;
      }))
      .def("add_rule", &tpi::Filter::add_rule)
      .def("add", &tpi::Filter::add)
      .def("include_file", &tpi::Filter::include_file)
      .def("include_dir", &tpi::Filter::include_dir)
      .def("describe", &tpi::Filter::describe);

  m.def("glob_match", [](const std::string& glob, const std::string& path) {
    return tpi::Glob(glob).match(path);
  });

  m.def(
      "walk",
      [](const std::string& root, const tpi::Filter& f) {
        std::vector<tpi::Entry> es;
        {
          py::gil_scoped_release nogil;
          es = tpi::walk(root, f);
        }
        py::list out;
        for (auto& e : es)
          out.append(py::make_tuple(e.rel, e.size, e.mtime_ns, e.mode, e.is_dir));
        return out;
      },
      py::arg("root"), py::arg("filter"));

  m.def(
      "copy_dir",
      [](const std::string& src, const std::string& dst, const tpi::Filter& f, int threads,
         uint64_t piece) {
        tpi::TransferStats s;
        {
          py::gil_scoped_release nogil;
          s = tpi::copy_dir(src, dst, f, threads, piece);
        }
        py::dict d;
        d["files"] = s.files;
        d["bytes"] = s.bytes;
        d["dirs"] = s.dirs;
        d["skipped"] = s.skipped;
        d["skipped_bytes"] = s.skipped_bytes;
        d["cloned"] = s.cloned;
        d["seconds"] = s.seconds;
        return d;
      },
      py::arg("src"), py::arg("dst"), py::arg("filter"), py::arg("threads") = 8,
      py::arg("piece_bytes") = 256ull << 20);

  auto pieces_of = [](const py::list& items) {
    std::vector<tpi::ReadPiece> pieces;
    for (auto item : items) {
      auto t = item.cast<py::tuple>();
      pieces.push_back({t[0].cast<std::string>(), t[1].cast<uint64_t>(), t[2].cast<uint64_t>(),
                        t[3].cast<uint64_t>()});
    }
    return pieces;
  };
  m.def(
      "read_pieces",
      [pieces_of](const py::list& items, uintptr_t dst, int threads) {
        auto pieces = pieces_of(items);
        py::gil_scoped_release nogil;
        return tpi::read_pieces(pieces, (uint8_t*)dst, threads);
      },
      "read [(path, file_off, len, dst_off)] into the buffer at dst");
  m.def(
      "write_pieces",
      [pieces_of](const py::list& items, uintptr_t src, int threads) {
        auto pieces = pieces_of(items);
        py::gil_scoped_release nogil;
        return tpi::write_pieces(pieces, (const uint8_t*)src, threads);
      },
      "write buffer ranges [(path, file_off, len, src_off)] into files");

  m.def("remove_tree", [](const std::string& p) {
    py::gil_scoped_release nogil;
    return tpi::remove_tree(p);
  });

  m.def(
      "crc32c",
      [](py::buffer b, uint32_t crc) {
        py::buffer_info i = b.request();
        py::gil_scoped_release nogil;
        return tpi::crc32c(i.ptr, (size_t)(i.size * i.itemsize), crc);
      },
      py::arg("data"), py::arg("crc") = 0);
  m.def("crc32c_ptr", [](uintptr_t p, uint64_t n, uint32_t crc) {
    py::gil_scoped_release nogil;
    return tpi::crc32c((const void*)p, n, crc);
  });
  m.def("crc32c_combine", &tpi::crc32c_combine);
  m.def("crc32c_combine_tiles_ptr", [](uintptr_t crcs, uint64_t n, uint64_t tile,
                                       uint64_t total) {
    return tpi::crc32c_combine_tiles((const uint32_t*)crcs, n, tile, total);
  });
  m.def("crc32c_tiles_ptr", [](uintptr_t p, uint64_t n, uint64_t tile, uintptr_t out,
                               int threads) {
    py::gil_scoped_release nogil;
    tpi::crc32c_tiles((const void*)p, n, tile, (uint32_t*)out, threads);
  });
  m.def("shard_hash_ptr", [](uintptr_t p, uint64_t n, uint64_t shard, uint64_t seed,
                             uintptr_t out, int threads) {
    py::gil_scoped_release nogil;
    tpi::shard_hash((const void*)p, n, shard, seed, (uint64_t*)out, threads);
  });
  m.def("pack_ptr", [](py::buffer segs, uint64_t total, uintptr_t stream, uint64_t tile,
                       uintptr_t crcs, int threads) {
    int n = 0;
    const tpi_seg* s = seg_ptr(segs, n);
    py::gil_scoped_release nogil;
    tpi::pack(s, n, total, (void*)stream, tile, (uint32_t*)crcs, threads);
  });
  m.def("unpack_ptr", [](py::buffer segs, uint64_t total, uintptr_t stream, uint64_t tile,
                         uintptr_t crcs, int threads) {
    int n = 0;
    const tpi_seg* s = seg_ptr(segs, n);
    int64_t first = -1;
    uint64_t bad;
    {
      py::gil_scoped_release nogil;
      bad = tpi::unpack(s, n, total, (const void*)stream, tile, (const uint32_t*)crcs, threads,
                        &first);
    }
    return py::make_tuple(bad, first);
  });
  m.def("write_file_ptr", [](const std::string& path, uintptr_t src, uint64_t n, int threads,
                            bool sync) {
    std::string err;
    {
      py::gil_scoped_release nogil;
      err = tpi::write_file(path, (const void*)src, n, threads, sync);
    }
    if (!err.empty()) throw std::runtime_error(err);
  });
  m.def("read_stream_ptr", [](const std::string& path, uintptr_t dst, uint64_t offset,
                              uint64_t n, int threads, uint64_t chunk, uintptr_t words,
                              uintptr_t tile_ends, uint64_t ntiles) {
    std::string err;
    {
      py::gil_scoped_release nogil;
      err = tpi::read_stream(path, (void*)dst, offset, n, threads, chunk, (uint64_t*)words,
                             (const uint64_t*)tile_ends, ntiles);
    }
    if (!err.empty()) throw std::runtime_error(err);
  });
  m.def("resident_bytes", [](const std::string& path) {
    uint64_t size = 0;
    int tmpfs = 0;
    const int64_t r = tpi::resident_bytes(path.c_str(), &size, &tmpfs);
    return py::make_tuple(r, size, (bool)tmpfs);
  });
  // step-boundary agreement block (ctl.h); `base` is the address of a shared mapping
  m.def("ctl_bytes", &tpi::ctl::bytes);
  m.def("ctl_init", [](uintptr_t base, int world) { tpi::ctl::init((void*)base, world); });
  m.def("ctl_valid", [](uintptr_t base, int world) {
    return tpi::ctl::valid((const void*)base, world);
  });
  m.def("ctl_arrive", [](uintptr_t base, int rank, uint64_t ordinal) {
    uint64_t preempt = 0, periodic = 0;
    tpi::ctl::arrive((void*)base, rank, ordinal, &preempt, &periodic);
    return py::make_tuple(preempt, periodic);
  });
  m.def("ctl_propose_preempt", [](uintptr_t base, int world, int self) {
    return tpi::ctl::propose_preempt((void*)base, world, self);
  });
  m.def("ctl_propose_periodic", [](uintptr_t base, int world, int self) {
    return tpi::ctl::propose_periodic((void*)base, world, self);
  });
  m.def("ctl_ordinal", [](uintptr_t base, int rank) {
    return tpi::ctl::ordinal_of((const void*)base, rank);
  });

  m.def("tpz_bound", [](uint64_t len) { return tpz_bound(len); });
  m.def("tpz_meta_bytes", [](uint64_t ntiles) { return tpz_meta_bytes(ntiles); });
  m.def("tpz_encode_ptr", [](uintptr_t src, uint64_t total, uint64_t tile, uintptr_t dst,
                             uintptr_t csizes, int threads) {
    py::gil_scoped_release nogil;
    return tpi::tpz_encode_stream((const void*)src, total, tile, (void*)dst,
                                  (uint32_t*)csizes, threads);
  });
  m.def("tpz_decode_ptr", [](uintptr_t src, uintptr_t csizes, uint64_t total, uint64_t tile,
                             uintptr_t dst, int threads) {
    py::gil_scoped_release nogil;
    return tpi::tpz_decode_stream((const void*)src, (const uint32_t*)csizes, total, tile,
                                  (void*)dst, threads);
  });
}
