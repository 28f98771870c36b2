// pybind11 module `_dfs_native`: the native data plane exposed to the service layer.
// Every long-running call releases the GIL so gRPC worker threads run in parallel.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <cstring>

#include <chrono>

#include "trace.h"
#include "chunk_store.h"
#include "crc32.h"
#include "crypto.h"
#include "disk_gate.h"
#include "fastpath.h"
#include "gf256.h"
#include "gpu_kernels.h"
#include "replication.h"
#include "cs_agent.h"
#include "cs_grpc.h"
#include "cs_stats.h"
#include "grpc_server.h"
#include "http_lite.h"
#include "sigv4.h"
#include "tls.h"
#include "wal.h"

namespace py = pybind11;
using namespace dfs;

namespace {

struct Buf {
  const uint8_t* p;
  size_t n;
};

Buf view(const py::buffer& b, py::buffer_info& keep) {
  keep = b.request();
  return Buf{static_cast<const uint8_t*>(keep.ptr), static_cast<size_t>(keep.size * keep.itemsize)};
}

py::bytes new_bytes(size_t n, char** data) {
  PyObject* o = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(n));
  if (!o) throw py::error_already_set();
  *data = PyBytes_AS_STRING(o);
  return py::reinterpret_steal<py::bytes>(o);
}

py::bytes meta_image(const std::vector<uint32_t>& v) {
  char* d;
  py::bytes out = new_bytes(v.size() * 4, &d);
  for (size_t i = 0; i < v.size(); ++i) {
    uint32_t be = __builtin_bswap32(v[i]);
    std::memcpy(d + 4 * i, &be, 4);
  }
  return out;
}

gf::Matrix to_matrix(const std::vector<std::vector<int>>& m) {
  gf::Matrix out;
  for (auto& row : m) {
    std::vector<uint8_t> r;
    for (int v : row) r.push_back(static_cast<uint8_t>(v));
    out.push_back(r);
  }
  return out;
}

std::vector<std::vector<int>> from_matrix(const gf::Matrix& m) {
  std::vector<std::vector<int>> out;
  for (auto& row : m) out.emplace_back(row.begin(), row.end());
  return out;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // namespace

void bind_meta(py::module_& m);  // bindings_meta.cpp

// JSON (cs_stats.h) -> Python objects
py::object json_to_py(const Json& j) {
  switch (j.type()) {
    case Json::Type::Null: return py::none();
    case Json::Type::Bool: return py::bool_(j.as_bool());
    case Json::Type::Int: return py::int_(j.as_int());
    case Json::Type::Double: return py::float_(j.as_double());
    case Json::Type::String: return py::str(j.as_string());
    case Json::Type::Array: {
      py::list l;
      for (const auto& v : j.items()) l.append(json_to_py(v));
      return l;
    }
    case Json::Type::Object: {
      py::dict d;
      for (const auto& kv : j.fields()) d[py::str(kv.first)] = json_to_py(kv.second);
      return d;
    }
  }
  return py::none();
}

PYBIND11_MODULE(_dfs_native, m) {
  m.doc() = "MI355X-native data plane: HBM chunk store, CDNA4 CRC/RS kernels, RCCL replication, WAL";
  dfs::trace_init();  // at import, before the module starts a thread (trace.h)

  // ---------------- checksums
  m.def("copy_into", [](py::buffer dst, uint64_t off, py::buffer src) {
    // memcpy into a writable buffer (shared-memory slot) with the GIL released
    py::buffer_info d = dst.request(true);
    py::buffer_info sk;
    Buf sv = view(src, sk);
    uint64_t cap = static_cast<uint64_t>(d.size * d.itemsize);
    if (off > cap || sv.n > cap - off) throw std::out_of_range("copy_into: destination too small");
    py::gil_scoped_release r;
    std::memcpy(static_cast<uint8_t*>(d.ptr) + off, sv.p, sv.n);
  }, py::arg("dst"), py::arg("offset"), py::arg("src"));
  m.def("copy_out", [](py::buffer src, uint64_t off, uint64_t n) {
    // new bytes object holding src[off:off+n], memcpy with the GIL released
    py::buffer_info sk;
    Buf sv = view(src, sk);
    if (off > sv.n || n > sv.n - off) throw std::out_of_range("copy_out: range outside source");
    char* d;
    py::bytes out = new_bytes(n, &d);
    {
      py::gil_scoped_release r;
      std::memcpy(d, sv.p + off, n);
    }
    return out;
  }, py::arg("src"), py::arg("offset"), py::arg("length"));
  m.def("crc32", [](py::buffer b, uint32_t crc) {
    py::buffer_info k;
    Buf v = view(b, k);
    py::gil_scoped_release r;
    return crc32_update(crc, v.p, v.n);
  }, py::arg("data"), py::arg("crc") = 0);
  m.def("crc32_meta", [](py::buffer b) {
    py::buffer_info k;
    Buf v = view(b, k);
    std::vector<uint32_t> s(num_slices(v.n));
    {
      py::gil_scoped_release r;
      crc32_slices(v.p, v.n, s.data());
    }
    return meta_image(s);
  }, "Per-512B-slice CRC32 as the big-endian .meta image");
  m.def("crc32_combine", &crc32_combine);
  m.def("crc32_from_meta", [](py::buffer meta, uint64_t n) {
    py::buffer_info k;
    Buf v = view(meta, k);
    std::vector<uint32_t> s(v.n / 4);
    for (size_t i = 0; i < s.size(); ++i) {
      uint32_t be;
      std::memcpy(&be, v.p + 4 * i, 4);
      s[i] = __builtin_bswap32(be);
    }
    return crc32_from_slices(s.data(), n);
  });
  m.def("cpu_has_pclmul", &cpu_has_pclmul);
  m.def("device_count", &device_count);
  // hipDeviceSynchronize on `device` in the calling process (the chunkserver owns its GPU:
  // the benchmark brackets its timed region with this, through the server's /sync endpoint)
  // The same device synchronize on a native HTTP listener of its own (GET /sync): the
  // benchmark's timed region is bracketed by it, and no Python thread (GIL, thread start)
  // sits between the request and hipDeviceSynchronize.
  struct SyncServer {
    std::unique_ptr<HttpLiteServer> srv;
  };
  py::class_<SyncServer>(m, "DeviceSyncServer")
      .def(py::init([](const std::string& host, int port, int device) {
             auto s = std::make_unique<SyncServer>();
             s->srv = std::make_unique<HttpLiteServer>(host, port, [device](const HttpRequest& r) -> HttpResponse {
               if (r.path != "/sync") return HttpResponse{404, "text/plain", "Not Found"};
               const auto t0 = std::chrono::steady_clock::now();
               bool ok = device < 0 || (hipSetDevice(device) == hipSuccess && hipDeviceSynchronize() == hipSuccess);
               const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
               char body[160];
               std::snprintf(body, sizeof(body), "{\"synchronized\": %s, \"gpu\": %d, \"sync_ms\": %.3f, \"native\": true}",
                             ok ? "true" : "false", device, ms);
               return HttpResponse{200, "application/json", body};
             });
             return s;
           }),
           py::arg("host"), py::arg("port"), py::arg("device"))
      .def("start", [](SyncServer& s) {
        std::string err;
        bool ok = s.srv->start(&err);
        return py::make_tuple(ok, err);
      })
      .def_property_readonly("port", [](SyncServer& s) { return s.srv->port(); })
      .def("stop", [](SyncServer& s) {
        py::gil_scoped_release r;
        s.srv->stop();
      });
  m.def("device_synchronize", [](int device) {
    py::gil_scoped_release r;
    if (device < 0) return true;
    return hipSetDevice(device) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
  });
  // checksum-kernel selection (tests / A-B runs): (mfma, scrub ring buffers, K1/K2/K3 ring buffers)
  m.def("crc_kernels", [] { return py::make_tuple(crc_mfma_enabled(), crc_ring_buffers(), crc_tile_ring_buffers()); });
  m.def("set_crc_lds_max_mib", &set_crc_lds_max_mib, "K1/K2 size-based dispatch threshold (0 = matrix cores only)");
  m.def("crc_wide_mode", &crc_wide_mode);
  m.def("crc_fp4_enabled", &crc_fp4_enabled);
  m.def("set_crc_fp4", &set_crc_fp4, "wide K1/K2: chunk CRCs on the FP4 matrix cores (else i8)");
  m.def("set_crc_wide", &set_crc_wide, "K1/K2 one workgroup per CU: 0 off, 1 shared LDS image, 2 + LDS basis");
  m.def("set_crc_kernels", [](bool mfma, int scrub_ring, int tile_ring) {
    set_crc_mfma(mfma);
    set_crc_ring(scrub_ring, tile_ring);
  });

  // ---------------- GF(2^8) / Reed-Solomon
  m.def("rs_matrix", [](int k, int mm) { return from_matrix(gf::rs_matrix(k, mm)); });
  m.def("rs_decode_rows", [](int k, int mm, std::vector<int> present, std::vector<int> wanted) {
    return from_matrix(gf::rs_decode_rows(k, mm, present, wanted));
  });
  m.def("gf_mul", &gf::mul);
  m.def("gf_matmul_cpu", [](std::vector<std::vector<int>> mat, std::vector<py::buffer> inputs, uint64_t len) {
    gf::Matrix M = to_matrix(mat);
    std::vector<py::buffer_info> keep(inputs.size());
    std::vector<const uint8_t*> in;
    for (size_t i = 0; i < inputs.size(); ++i) {
      Buf v = view(inputs[i], keep[i]);
      if (v.n < len) throw std::runtime_error("shard shorter than len");
      in.push_back(v.p);
    }
    std::vector<py::bytes> outs;
    std::vector<uint8_t*> out;
    for (size_t r = 0; r < M.size(); ++r) {
      char* d;
      outs.push_back(new_bytes(len, &d));
      out.push_back(reinterpret_cast<uint8_t*>(d));
    }
    {
      py::gil_scoped_release rel;
      gf::matmul_cpu(M, in.data(), out.data(), len);
    }
    return outs;
  });

  // ---------------- chunk store
  py::class_<ChunkStore>(m, "ChunkStore")
      .def(py::init([](std::string storage_dir, std::string cold_dir, int device, uint64_t hbm_capacity,
                       int durability, int cache_blocks, int lanes, int spill_threads, bool sync_writes,
                       int journal) {
             StoreConfig c;
             c.journal = journal;
             c.storage_dir = storage_dir;
             c.cold_dir = cold_dir;
             c.device = device;
             c.hbm_capacity = hbm_capacity;
             c.durability = static_cast<Durability>(durability);
             c.cache_blocks = cache_blocks;
             c.lanes = lanes;
             c.spill_threads = spill_threads;
             c.sync_writes = sync_writes;
             py::gil_scoped_release r;
             return new ChunkStore(c);
           }),
           py::arg("storage_dir"), py::arg("cold_dir") = "", py::arg("device") = -1, py::arg("hbm_capacity") = 0,
           py::arg("durability") = 0, py::arg("cache_blocks") = 100, py::arg("lanes") = 8,
           py::arg("spill_threads") = 4, py::arg("sync_writes") = true, py::arg("journal") = -1)
      .def_property_readonly("gpu", &ChunkStore::gpu)
      .def_property_readonly("device", [](ChunkStore& s) { return s.config().device; })
      .def("write", [](ChunkStore& s, const std::string& id, py::buffer data, uint32_t expected) {
        py::buffer_info k;
        Buf v = view(data, k);
        WriteResult w;
        {
          py::gil_scoped_release r;
          w = s.write(id, v.p, v.n, expected);
        }
        return py::make_tuple(w.ok, w.actual_crc, w.error);
      }, py::arg("block_id"), py::arg("data"), py::arg("expected_crc") = 0)
      .def("stage", [](ChunkStore& s, const std::string& id, py::buffer data, uint32_t expected) {
        py::buffer_info k;
        Buf v = view(data, k);
        WriteResult w;
        {
          py::gil_scoped_release r;
          w = s.stage(id, v.p, v.n, expected);
        }
        return py::make_tuple(w.ok, w.actual_crc, w.error);
      }, py::arg("block_id"), py::arg("data"), py::arg("expected_crc") = 0)
      .def("persist", [](ChunkStore& s, const std::string& id, py::object data) {
        std::string err;
        bool ok;
        if (data.is_none()) {
          py::gil_scoped_release r;
          ok = s.persist(id, nullptr, 0, &err);
        } else {
          py::buffer_info k;
          Buf v = view(data.cast<py::buffer>(), k);
          py::gil_scoped_release r;
          ok = s.persist(id, v.p, v.n, &err);
        }
        return py::make_tuple(ok, err);
      }, py::arg("block_id"), py::arg("data") = py::none())
      .def("read", [](ChunkStore& s, const std::string& id, uint64_t offset, uint64_t length) -> py::tuple {
        ReadResult st;
        {
          py::gil_scoped_release r;
          st = s.stat(id, offset, length);
        }
        if (st.status != ReadStatus::Ok)
          return py::make_tuple(static_cast<int>(st.status), st.total_size, py::bytes(), false, (int64_t)-1, st.error);
        char* d;
        py::bytes out = new_bytes(st.bytes, &d);
        ReadResult rr;
        {
          py::gil_scoped_release r;
          rr = s.read_into(id, offset, st.bytes, reinterpret_cast<uint8_t*>(d));
        }
        if (rr.status == ReadStatus::NotFound || rr.status == ReadStatus::OutOfRange || rr.status == ReadStatus::IoError)
          return py::make_tuple(static_cast<int>(rr.status), rr.total_size, py::bytes(), false, (int64_t)-1, rr.error);
        return py::make_tuple(static_cast<int>(rr.status), rr.total_size, out, rr.partial_corrupt, rr.bad_slice,
                              rr.error);
      }, py::arg("block_id"), py::arg("offset") = 0, py::arg("length") = 0)
      .def("read_into", [](ChunkStore& s, const std::string& id, uint64_t offset, uint64_t length,
                           py::buffer out) -> py::tuple {
        // Zero-copy read into a caller-owned writable buffer (short-circuit shm slot).
        py::buffer_info bi = out.request(true);
        ReadResult st;
        {
          py::gil_scoped_release r;
          st = s.stat(id, offset, length);
        }
        if (st.status != ReadStatus::Ok)
          return py::make_tuple(static_cast<int>(st.status), st.total_size, (uint64_t)0, false, (int64_t)-1,
                                st.error);
        if (static_cast<uint64_t>(bi.size * bi.itemsize) < st.bytes)
          return py::make_tuple(static_cast<int>(ReadStatus::IoError), st.total_size, (uint64_t)0, false,
                                (int64_t)-1, std::string("destination buffer too small"));
        ReadResult rr;
        {
          py::gil_scoped_release r;
          rr = s.read_into(id, offset, st.bytes, static_cast<uint8_t*>(bi.ptr));
        }
        return py::make_tuple(static_cast<int>(rr.status), rr.total_size, rr.bytes, rr.partial_corrupt,
                              rr.bad_slice, rr.error);
      }, py::arg("block_id"), py::arg("offset"), py::arg("length"), py::arg("out"))
      // pin a caller buffer for device DMA / kernel stores, as the fast path pins a client's
      // shared-memory arena (tests and benches of the zero-copy and fused read paths)
      .def("register_host", [](ChunkStore& s, py::buffer b) {
        py::buffer_info bi = b.request(true);
        py::gil_scoped_release r;
        return s.register_host(bi.ptr, static_cast<uint64_t>(bi.size * bi.itemsize));
      }, py::arg("buffer"))
      .def("unregister_host", [](ChunkStore& s, py::buffer b) {
        py::buffer_info bi = b.request(true);
        py::gil_scoped_release r;
        s.unregister_host(bi.ptr);
      }, py::arg("buffer"))
      .def("exists", &ChunkStore::exists)
      .def("size", &ChunkStore::block_size)
      .def("crc", &ChunkStore::block_crc, py::call_guard<py::gil_scoped_release>())
      .def("remove", &ChunkStore::remove, py::call_guard<py::gil_scoped_release>())
      .def("move_to_cold", &ChunkStore::move_to_cold, py::call_guard<py::gil_scoped_release>())
      .def("verify_on_disk", &ChunkStore::verify_on_disk, py::call_guard<py::gil_scoped_release>())
      .def("meta", [](ChunkStore& s, const std::string& id) {
        std::vector<uint32_t> v;
        {
          py::gil_scoped_release r;
          v = s.meta(id);
        }
        return meta_image(v);
      })
      .def("scrub", &ChunkStore::scrub, py::call_guard<py::gil_scoped_release>())
      .def("scrub_resident", &ChunkStore::scrub_resident, py::call_guard<py::gil_scoped_release>(),
           "K1b only: verify the listed HBM-resident blocks against their .meta images")
      .def("list_blocks", &ChunkStore::list_blocks)
      .def("flush", &ChunkStore::flush, py::call_guard<py::gil_scoped_release>())
      .def("drop_resident", &ChunkStore::drop_resident, py::call_guard<py::gil_scoped_release>())
      .def("debug_corrupt", &ChunkStore::debug_corrupt, py::call_guard<py::gil_scoped_release>())
      .def("debug_pause_spill", &ChunkStore::debug_pause_spill, py::call_guard<py::gil_scoped_release>())
      .def("materialize", &ChunkStore::materialize_all, py::call_guard<py::gil_scoped_release>(),
           "write every journal record out as <id> + <id>.meta now and wait")
      .def("debug_pause_materializer", &ChunkStore::debug_pause_materializer,
           py::call_guard<py::gil_scoped_release>())
      .def("journaled", &ChunkStore::journaled)
      .def("compact", &ChunkStore::compact, py::call_guard<py::gil_scoped_release>(), py::arg("max_live") = 1.0,
           "relocate the live records of the oldest journal segment(s) holding at most max_live of their capacity")
      .def("stats", [](ChunkStore& s) { return json_to_py(stats_json(s.stats())); })
      .def("gpu_crc", [](ChunkStore& s, py::buffer data) {
        py::buffer_info k;
        Buf v = view(data, k);
        std::vector<uint32_t> sl;
        uint32_t c;
        {
          py::gil_scoped_release r;
          c = s.gpu_crc(v.p, v.n, &sl);
        }
        return py::make_tuple(c, meta_image(sl));
      })
      .def("gf_matmul", [](ChunkStore& s, std::vector<std::vector<int>> mat, std::vector<py::buffer> inputs,
                           uint64_t len) -> py::object {
        gf::Matrix M = to_matrix(mat);
        std::vector<py::buffer_info> keep(inputs.size());
        std::vector<const uint8_t*> in;
        for (size_t i = 0; i < inputs.size(); ++i) {
          Buf v = view(inputs[i], keep[i]);
          if (v.n < len) throw std::runtime_error("shard shorter than len");
          in.push_back(v.p);
        }
        std::vector<py::bytes> outs;
        std::vector<uint8_t*> out;
        for (size_t r = 0; r < M.size(); ++r) {
          char* d;
          outs.push_back(new_bytes(len, &d));
          out.push_back(reinterpret_cast<uint8_t*>(d));
        }
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = s.gf_matmul_gpu(M, in, out, len);
        }
        if (!ok) return py::none();
        return py::cast(outs);
      });

  // ---------------- native chunkserver control loop (csrc/cs_agent.cpp)
  py::class_<CsAgent>(m, "CsAgent")
      .def(py::init([](ChunkStore* store, FastPathServer* fp, const std::string& advertise, const std::string& rack_id,
                       const std::string& storage_dir, int gpu_rank, std::vector<std::string> masters,
                       std::vector<std::string> config_servers, double heartbeat_s, double scrub_s,
                       const std::string& ca_cert, const std::string& domain_name, bool tls) {
             CsAgentConfig c;
             c.advertise = advertise;
             c.rack_id = rack_id;
             c.storage_dir = storage_dir;
             c.gpu_rank = gpu_rank;
             c.masters = std::move(masters);
             c.config_servers = std::move(config_servers);
             c.heartbeat_ms = std::max(10, static_cast<int>(heartbeat_s * 1000));
             c.scrub_ms = std::max(10, static_cast<int>(scrub_s * 1000));
             c.tls = tls;
             std::shared_ptr<TlsContext> ctx;
             if (tls) {
               std::string err;
               ctx = TlsContext::client(ca_cert, domain_name, &err);
               if (!ctx) throw std::runtime_error(err);
             }
             return std::make_unique<CsAgent>(c, store, fp, ctx);
           }),
           py::arg("store"), py::arg("fastpath"), py::arg("advertise"), py::arg("rack_id") = "",
           py::arg("storage_dir") = "/tmp", py::arg("gpu_rank") = -1, py::arg("masters") = std::vector<std::string>{},
           py::arg("config_servers") = std::vector<std::string>{}, py::arg("heartbeat_interval") = 5.0,
           py::arg("scrub_interval") = 60.0, py::arg("ca_cert") = "", py::arg("domain_name") = "",
           py::arg("tls") = false, py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("start", &CsAgent::start)
      .def("stop", &CsAgent::stop, py::call_guard<py::gil_scoped_release>())
      .def("heartbeat_once", &CsAgent::heartbeat_once, py::call_guard<py::gil_scoped_release>())
      .def("scrub_once", &CsAgent::scrub_once, py::call_guard<py::gil_scoped_release>())
      .def("recover", &CsAgent::recover, py::call_guard<py::gil_scoped_release>())
      .def("queue_recovery", &CsAgent::queue_recovery)
      .def("submit_command", [](CsAgent& a, py::bytes cmd) {
        std::string c = cmd;
        py::gil_scoped_release r;
        a.submit_command(c);
      })
      .def("report_new_block", &CsAgent::report_new_block)
      .def("report_bad_block", &CsAgent::report_bad_block)
      .def("masters", &CsAgent::masters)
      .def_property_readonly("known_term", &CsAgent::known_term)
      .def("stats", [](CsAgent& a) { return json_to_py(stats_json(a.stats())); });

  // ---------------- RCCL replication
  py::class_<FastPathServer>(m, "FastPathServer")
      .def(py::init<ChunkStore*, std::string>(), py::arg("store"), py::arg("name"), py::keep_alive<1, 2>())
      .def("start", [](FastPathServer& f) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = f.start(&err);
        }
        return py::make_tuple(ok, err);
      })
      .def("stop", &FastPathServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("name", &FastPathServer::name)
      .def("fence", [](FastPathServer& f, uint64_t term) {
        uint64_t known = 0;
        bool ok = f.fence(term, &known);
        return py::make_tuple(ok, known);
      })
      .def("adopt_term", &FastPathServer::adopt_term)
      .def_property_readonly("term", &FastPathServer::term)
      .def("drain_suspects", &FastPathServer::drain_suspects)
      .def("recent_request_ids", &FastPathServer::recent_request_ids)
      .def("set_replication", [](FastPathServer& f, ReplicationEngine& e) {
        f.set_replication(&e);
        e.set_control([&f](int rank, const std::string& req, std::string* reply) { return f.control(rank, req, reply); });
      }, py::arg("engine"), py::keep_alive<1, 2>(), py::keep_alive<2, 1>())
      .def("debug_drop_descriptors", &FastPathServer::debug_drop_descriptors)
      .def("set_peer", &FastPathServer::set_peer, py::arg("addr"), py::arg("rank"), py::arg("name") = "")
      .def("set_self_host", &FastPathServer::set_self_host, py::arg("host"))
      .def("set_self_addr", &FastPathServer::set_self_addr, py::arg("addr"))
      .def("stats", [](FastPathServer& f) { return json_to_py(stats_json(f.stats())); })
      .def("replicate_block", [](FastPathServer& f, const std::string& id, const std::vector<std::string>& targets,
                                 uint64_t term) {
        std::vector<std::string> done;
        int n;
        {
          py::gil_scoped_release r;
          n = f.replicate_block(id, targets, term, &done);
        }
        return py::make_tuple(n, done);
      }, py::arg("block_id"), py::arg("targets"), py::arg("term"))
      .def("drain_healed", &FastPathServer::drain_healed);

  struct PyTicket {
    ReplTicket t;
    py::object keep;  // host source bytes stay alive until wait_send
  };
  py::class_<PyTicket>(m, "ReplTicket")
      .def_property_readonly("peer", [](PyTicket& k) { return k.t.peer; })
      .def_property_readonly("gen", [](PyTicket& k) { return k.t.gen; })
      .def_property_readonly("seq", [](PyTicket& k) { return k.t.seq; })
      .def_property_readonly("ch", [](PyTicket& k) { return k.t.ch; })
      .def_property_readonly("size", [](PyTicket& k) { return k.t.size; })
      .def_property_readonly("slice", [](PyTicket& k) { return k.t.slice; });

  m.def("rccl_loopback_probe", [](int device, uint64_t bytes, uint64_t abort_bytes, int timeout_ms) {
    RcclProbe p;
    {
      py::gil_scoped_release r;
      p = rccl_loopback_probe(device, bytes, abort_bytes, timeout_ms);
    }
    py::dict d;
    d["ok"] = p.ok;
    d["bytes_ok"] = p.bytes_ok;
    d["drained_after_abort"] = p.drained_after_abort;
    d["reinit_ok"] = p.reinit_ok;
    d["version"] = p.version;
    d["xfer_ms"] = p.xfer_ms;
    d["abort_ms"] = p.abort_ms;
    d["init_ms"] = p.init_ms;
    d["error"] = p.error;
    return d;
  }, py::arg("device"), py::arg("bytes"), py::arg("abort_bytes") = 0, py::arg("timeout_ms") = 20000);

  py::class_<ReplicationEngine>(m, "ReplicationEngine")
      .def(py::init([](ChunkStore* store, const std::string& transport, int rank, int world, const std::string& ns,
                       int open_timeout_ms, int turn_timeout_ms, int xfer_timeout_ms, int channels) {
             std::string err;
             std::unique_ptr<P2PTransport> t = make_transport(transport, store, rank, ns, channels, &err);
             if (!t) throw std::runtime_error(err);
             ReplOptions o;
             o.open_timeout_ms = open_timeout_ms;
             o.turn_timeout_ms = turn_timeout_ms;
             o.xfer_timeout_ms = xfer_timeout_ms;
             o.channels = t->channels();
             return std::make_unique<ReplicationEngine>(store, std::move(t), rank, world, o);
           }),
           py::keep_alive<1, 2>(), py::arg("store"), py::arg("transport"), py::arg("rank"), py::arg("world"),
           py::arg("ns") = "", py::arg("open_timeout_ms") = 20000, py::arg("turn_timeout_ms") = 3000,
           py::arg("xfer_timeout_ms") = 20000, py::arg("channels") = 0)
      .def_property_readonly("channels", &ReplicationEngine::channels)
      .def("start", &ReplicationEngine::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &ReplicationEngine::stop, py::call_guard<py::gil_scoped_release>())
      .def("wait_ready", &ReplicationEngine::wait_ready, py::call_guard<py::gil_scoped_release>(), py::arg("timeout_ms"),
           py::arg("give_up_after") = 3)
      .def_property_readonly("rank", &ReplicationEngine::rank)
      .def_property_readonly("world", &ReplicationEngine::world)
      .def_property_readonly("transport", &ReplicationEngine::transport_name)
      .def("pair_ok", &ReplicationEngine::pair_ok, py::call_guard<py::gil_scoped_release>())
      .def("generation", &ReplicationEngine::generation, py::call_guard<py::gil_scoped_release>())
      .def("fail_pair", &ReplicationEngine::fail_pair, py::call_guard<py::gil_scoped_release>(), py::arg("peer"),
           py::arg("why") = "debug")
      .def("slice_for", &ReplicationEngine::slice_for)
      .def("send", [](ReplicationEngine& e, int peer, const std::string& id, py::object data) -> py::tuple {
        auto k = std::make_unique<PyTicket>();
        std::string err;
        const uint8_t* src = nullptr;
        uint64_t n = 0;
        if (!data.is_none()) {
          py::buffer_info bi = py::buffer(data).request();
          src = static_cast<const uint8_t*>(bi.ptr);
          n = static_cast<uint64_t>(bi.size * bi.itemsize);
          k->keep = data;
        }
        bool ok;
        {
          py::gil_scoped_release r;
          ok = e.send(peer, id, src, n, &k->t, &err);
        }
        if (!ok) return py::make_tuple(py::none(), err);
        return py::make_tuple(py::cast(std::move(k)), std::string());
      }, py::arg("peer"), py::arg("block_id"), py::arg("data") = py::none())
      .def("wait_send", [](ReplicationEngine& e, PyTicket& k) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = e.wait_send(&k.t, &err);
        }
        k.keep = py::none();
        return py::make_tuple(ok, err);
      })
      .def("cancel_send", [](ReplicationEngine& e, PyTicket& k, const std::string& why) {
        {
          py::gil_scoped_release r;
          e.cancel_send(&k.t, why);
        }
        k.keep = py::none();
      })
      .def("recv", [](ReplicationEngine& e, int src, uint64_t gen, int64_t seq, const std::string& id, uint64_t size,
                      uint64_t slice, uint32_t crc, bool persist, int ch) {
        WriteResult w;
        {
          py::gil_scoped_release r;
          w = e.recv(src, gen, ch, seq, id, size, slice, crc, persist);
        }
        return py::make_tuple(w.ok, w.actual_crc, w.error);
      }, py::arg("src"), py::arg("gen"), py::arg("seq"), py::arg("block_id"), py::arg("size"), py::arg("slice"),
         py::arg("crc"), py::arg("persist") = true, py::arg("ch") = 0)
      .def("debug_drop_sends", [](ReplicationEngine& e, int peer, int n) { e.transport()->debug_drop_sends(peer, n); })
      .def("debug_stall", [](ReplicationEngine& e, int peer, int ms) { e.transport()->debug_stall(peer, ms); })
      .def("stats", [](ReplicationEngine& e) {
        Json d = stats_json(e.stats());
        d.set("channels", e.channels());
        return json_to_py(d);
      })
      .def_property_readonly("bytes_sent", [](ReplicationEngine& e) { return e.stats().bytes_sent; })
      .def_property_readonly("bytes_recv", [](ReplicationEngine& e) { return e.stats().bytes_recv; });

  // ---------------- native gRPC ChunkServerService (nghttp2)
  struct NativeGrpc {
    std::shared_ptr<py::object> fallback;
    std::unique_ptr<NativeChunkService> svc;
    std::unique_ptr<GrpcServer> srv;
  };
  py::class_<NativeGrpc>(m, "NativeGrpcChunkServer")
      .def(py::init([](ChunkStore* store, FastPathServer* fp, const std::string& host, int port, py::object fallback,
                       int workers, const std::string& tls_cert, const std::string& tls_key) {
             auto n = std::make_unique<NativeGrpc>();
             // the Python fallback is released with the GIL held, whichever thread drops it
             n->fallback = std::shared_ptr<py::object>(new py::object(std::move(fallback)), [](py::object* o) {
               py::gil_scoped_acquire g;
               delete o;
             });
             auto fb = n->fallback;
             n->svc = std::make_unique<NativeChunkService>(store, fp, [fb](const GrpcCall& c) -> GrpcReply {
               py::gil_scoped_acquire g;
               try {
                 py::tuple r = (*fb)(c.path, c.request_id,
                                     py::bytes(reinterpret_cast<const char*>(c.data()), c.size()));
                 return GrpcReply{r[0].cast<int>(), r[1].cast<std::string>()};
               } catch (py::error_already_set& e) {
                 return GrpcReply{13, std::string("python handler failed: ") + e.what()};
               }
             });
             NativeChunkService* svc = n->svc.get();
             n->srv = std::make_unique<GrpcServer>(host, port, [svc](const GrpcCall& c) { return svc->handle(c); },
                                                   workers);
             n->srv->set_body_allocator([svc](size_t len) { return svc->request_buffer(len); },
                                        NativeChunkService::kRequestBufferMin);
             if (!tls_cert.empty()) {
               std::string err;
               auto t = TlsContext::server(tls_cert, tls_key, &err);
               if (!t) throw std::runtime_error(err);
               n->srv->set_tls(std::move(t));
             }
             return n;
           }),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::arg("store"), py::arg("fastpath"), py::arg("host"),
           py::arg("port"), py::arg("fallback"), py::arg("workers") = 32, py::arg("tls_cert") = "",
           py::arg("tls_key") = "")
      .def("start", [](NativeGrpc& n) {
        std::string err;
        bool ok = n.srv->start(&err);
        return py::make_tuple(ok, err);
      })
      .def("stop", [](NativeGrpc& n) {
        py::gil_scoped_release r;  // workers may be waiting for the GIL in the fallback
        n.srv->stop();
      })
      .def_property_readonly("port", [](NativeGrpc& n) { return n.srv->port(); })
      .def("stats", [](NativeGrpc& n) { return json_to_py(stats_json(n.svc->stats(), n.srv->calls())); });

  // ---------------- WAL
  py::class_<Wal>(m, "Wal")
      .def(py::init<std::string, bool>(), py::arg("path"), py::arg("sync") = true)
      .def("replay", [](Wal& w) {
        std::vector<std::string> v;
        {
          py::gil_scoped_release r;
          v = w.replay();
        }
        py::list out;
        for (auto& s : v) out.append(py::bytes(s));
        return out;
      })
      .def("append", [](Wal& w, std::vector<std::string> recs) {
        py::gil_scoped_release r;
        w.append(recs);
      })
      .def("reset", [](Wal& w, std::vector<std::string> recs) {
        py::gil_scoped_release r;
        w.reset(recs);
      })
      .def_property_readonly("size_bytes", &Wal::size_bytes)
      .def_property_readonly("syncs", &Wal::syncs);
  m.def("atomic_write", [](std::string path, py::bytes data, bool sync) {
    std::string d = data;
    py::gil_scoped_release r;
    atomic_write_file(path, d, sync);
  }, py::arg("path"), py::arg("data"), py::arg("sync") = true);

  // ---------------- crypto
  m.def("aes256gcm_encrypt", [](py::bytes key, py::bytes nonce, py::bytes pt, py::bytes aad) {
    std::string k = key, n = nonce, p = pt, a = aad, o;
    {
      py::gil_scoped_release r;
      o = crypto::aes256gcm_encrypt(k, n, p, a);
    }
    return py::bytes(o);
  }, py::arg("key"), py::arg("nonce"), py::arg("plaintext"), py::arg("aad") = py::bytes());
  m.def("aes256gcm_decrypt", [](py::bytes key, py::bytes nonce, py::bytes ct, py::bytes aad) {
    std::string k = key, n = nonce, c = ct, a = aad, o;
    {
      py::gil_scoped_release r;
      o = crypto::aes256gcm_decrypt(k, n, c, a);
    }
    return py::bytes(o);
  }, py::arg("key"), py::arg("nonce"), py::arg("ciphertext"), py::arg("aad") = py::bytes());
  m.def("rsa_sha256_verify", [](py::bytes n, py::bytes e, py::bytes msg, py::bytes sig) {
    return crypto::rsa_sha256_verify(n, e, msg, sig);
  });
  m.def("random_bytes", [](size_t n) { return py::bytes(crypto::random_bytes(n)); });

  // ---------------- SigV4 (sigv4.h)
  m.def("sigv4_uri_encode", &sigv4::uri_encode, py::arg("s"), py::arg("encode_slash") = true);
  m.def("sigv4_normalize_query", &sigv4::normalize_query);
  m.def("sigv4_signing_key", [](const std::string& secret, const std::string& date, const std::string& region,
                                const std::string& service) {
    return py::bytes(sigv4::signing_key(secret, date, region, service));
  });
  m.def("sigv4_signature", [](py::bytes key, const std::string& sts) { return sigv4::signature(key, sts); });
  m.def("sigv4_canonical_request", [](const std::string& method, const std::string& path, const std::string& query,
                                      std::vector<std::pair<std::string, std::string>> headers,
                                      const std::string& signed_headers, const std::string& payload_hash) {
    return sigv4::canonical_request({method, path, query, std::move(headers), signed_headers, payload_hash});
  });
  m.def("sigv4_verify", [](const std::string& method, const std::string& path, const std::string& query,
                           std::vector<std::pair<std::string, std::string>> headers, const std::string& signed_headers,
                           const std::string& payload_hash, const std::string& timestamp, const std::string& scope,
                           py::bytes key, const std::string& sig) {
    std::string creq;
    bool ok = sigv4::verify({method, path, query, std::move(headers), signed_headers, payload_hash}, timestamp, scope,
                            key, sig, &creq);
    return py::make_tuple(ok, creq);
  });

  // ---------------- node-wide disk admission (disk_gate.h)
  py::class_<DiskGate::Slot>(m, "DiskSlot")
      .def("release", &DiskGate::Slot::release)
      .def_property_readonly("held", &DiskGate::Slot::held);
  py::class_<DiskGate>(m, "DiskGate")
      .def(py::init<const std::string&, int>(), py::arg("dir"), py::arg("slots"))
      .def_property_readonly("enabled", &DiskGate::enabled)
      .def_property_readonly("slots", &DiskGate::slots)
      .def_property_readonly("waits", &DiskGate::waits)
      .def("acquire", &DiskGate::acquire, py::call_guard<py::gil_scoped_release>(), py::keep_alive<0, 1>())
      .def("try_acquire", [](DiskGate& g) -> py::object {
        bool got = false;
        DiskGate::Slot s = g.try_acquire(&got);
        if (!got) return py::none();
        return py::cast(std::move(s));
      }, py::keep_alive<0, 1>());

  // ---------------- metadata plane (Raft)
  bind_meta(m);
}
