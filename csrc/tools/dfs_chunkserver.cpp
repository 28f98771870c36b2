// dfs_chunkserver — the native ChunkServer process, one per GPU (C43; reference
// dfs/chunkserver/src/bin/chunkserver.rs:74-375 for the process, chunkserver.rs:721-1088 for
// the service).
//
// Everything the Python shell (tests/models/chunkserver_shell.py + chunkserver_service.py) used to host runs here in
// C++, so no interpreter lives in a chunkserver process:
//   * the HBM chunk store on GPU --gpu (the host store with --gpu -1), its block journal,
//     exporter and scrubber (chunk_store.cpp);
//   * the same-host fast path (fastpath.cpp) and, with --rccl-world > 1, the replication
//     engine over the named transport, its ranks met through the --rccl-rendezvous directory
//     (one `addr_<rank>` file per rank: advertised address, fast-path socket);
//   * ChunkServerService on the native HTTP/2 gRPC server with every case native
//     (cs_grpc.cpp set_native): the reference's store-and-forward gRPC chain for hops without
//     a pair, engine descriptors, heal copies, shm-in-gRPC, recovery of corrupt reads;
//   * the control loop (cs_agent.cpp): heartbeats to every master, the masters' commands,
//     recovery, the scrubber;
//   * the HTTP side channel: /health, /metrics (Prometheus), /stats (JSON), /sync (device
//     synchronize; also on a listener of its own, reported as sync_port), /export (write every
//     journal-resident block out as <id> + <id>.meta now), /compact, and /debug/* with
//     DFS_DEBUG_ENDPOINTS=1.
//
// Flags are those of tests/models/chunkserver_shell.py (the reference's spelling plus the MI355X
// additions), so the launcher, bench.py, the helm chart and the tests start either process
// with the same command line.
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "chunk_store.h"
#include "thread_name.h"

#include <sys/prctl.h>
#include "crc32.h"
#include "cs_agent.h"
#include "cs_grpc.h"
#include "cs_stats.h"
#include "dfs_pb.h"
#include "fastpath.h"
#include "grpc_client.h"
#include "grpc_server.h"
#include "http_lite.h"
#include "json.h"
#include "node_shell.h"
#include "replication.h"
#include "tls.h"
#include "trace.h"

using namespace dfs;
using namespace dfs::shell;

namespace {

constexpr const char* kLog = "dfs.chunkserver";

const char* kUsage =
    "usage: dfs_chunkserver [--addr HOST:PORT] [--storage-dir DIR] [--cold-storage-dir DIR]\n"
    "  [--advertise-addr ADDR] [--http-port N] [--config-servers A,B] [--masters A,B] [--rack-id ID]\n"
    "  [--gpu N] [--hbm-capacity BYTES[K|M|G]] [--durability nvme-sync|hbm-ack] [--lanes N]\n"
    "  [--rccl-rank R --rccl-world W --rccl-rendezvous DIR] [--rccl-timeout-ms MS]\n"
    "  [--replication-transport hipipc|hipipc-spin|rccl|grpc|socket] [--repl-turn-timeout-ms MS]\n"
    "  [--heartbeat-interval S] [--scrub-interval S] [--workers N] [--no-fsync]\n"
    "  [--tls-cert F --tls-key F] [--ca-cert F] [--domain-name NAME]\n";

std::string strip_scheme(const std::string& a) {
  auto p = a.find("://");
  return p == std::string::npos ? a : a.substr(p + 3);
}

uint64_t parse_size(std::string s) {
  if (s.empty()) return 0;
  const char u = static_cast<char>(std::toupper(static_cast<unsigned char>(s.back())));
  uint64_t mult = 1;
  if (u == 'K') mult = 1ull << 10;
  else if (u == 'M') mult = 1ull << 20;
  else if (u == 'G') mult = 1ull << 30;
  else if (u == 'T') mult = 1ull << 40;
  if (mult != 1) s.pop_back();
  return static_cast<uint64_t>(std::atof(s.c_str()) * static_cast<double>(mult));
}

std::string abs_path(const std::string& p) {
  if (!p.empty() && p[0] == '/') return p;
  char cwd[4096];
  if (!::getcwd(cwd, sizeof(cwd))) return p;
  return std::string(cwd) + "/" + p;
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// Publish our advertised address and fast-path socket for our rank, then wait for every
// rank's (tests/models/chunkserver_shell.py rendezvous_ranks: the same files, so mixed shells still meet).
bool rendezvous(const std::string& dir, int rank, int world, const std::string& addr, const std::string& fp_name,
                double timeout_s, std::map<std::string, int>* ranks, std::map<std::string, std::string>* names) {
  ::mkdir(dir.c_str(), 0755);
  const std::string tmp = dir + "/.addr_" + std::to_string(rank) + ".tmp";
  {
    std::ofstream f(tmp, std::ios::trunc);
    f << addr << (fp_name.empty() ? "" : "\n" + fp_name);
  }
  if (::rename(tmp.c_str(), (dir + "/addr_" + std::to_string(rank)).c_str()) != 0) return false;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(static_cast<int>(timeout_s * 1000));
  while (std::chrono::steady_clock::now() < deadline) {
    ranks->clear();
    names->clear();
    for (int r = 0; r < world; ++r) {
      const std::string text = read_file(dir + "/addr_" + std::to_string(r));
      if (text.empty()) continue;
      const auto nl = text.find('\n');
      const std::string a = strip_scheme(text.substr(0, nl));
      (*ranks)[a] = r;
      if (nl != std::string::npos && nl + 1 < text.size()) (*names)[a] = text.substr(nl + 1);
    }
    if (static_cast<int>(ranks->size()) == world) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  return false;
}

// Masters named by the SHARD_CONFIG file ({"shards": {id: [peers]}, "ranges": ...}).
std::vector<std::string> shard_config_masters(const std::string& path) {
  std::vector<std::string> out;
  try {
    Json cfg = Json::parse(read_file(path));
    for (const auto& kv : cfg["shards"].fields())
      for (const auto& p : kv.second.items())
        if (std::find(out.begin(), out.end(), strip_scheme(p.str())) == out.end()) out.push_back(strip_scheme(p.str()));
  } catch (const std::exception& e) {
    log(kWarning, kLog, "SHARD_CONFIG %s unreadable: %s", path.c_str(), e.what());
  }
  return out;
}

std::map<std::string, std::string> parse_query(const std::string& q) {
  std::map<std::string, std::string> out;
  size_t pos = 0;
  while (pos < q.size()) {
    size_t amp = q.find('&', pos);
    std::string kv = q.substr(pos, amp == std::string::npos ? std::string::npos : amp - pos);
    size_t eq = kv.find('=');
    if (eq != std::string::npos) out[kv.substr(0, eq)] = kv.substr(eq + 1);
    else if (!kv.empty()) out[kv] = "";
    if (amp == std::string::npos) break;
    pos = amp + 1;
  }
  return out;
}

std::string from_hex(const std::string& h) {
  std::string out;
  for (size_t i = 0; i + 1 < h.size(); i += 2) out.push_back(static_cast<char>(std::stoi(h.substr(i, 2), nullptr, 16)));
  return out;
}

HttpResponse sync_device(int gpu) {
  const auto t0 = std::chrono::steady_clock::now();
  const bool ok = gpu < 0 || (hipSetDevice(gpu) == hipSuccess && hipDeviceSynchronize() == hipSuccess);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  char body[160];
  std::snprintf(body, sizeof(body), "{\"synchronized\": %s, \"gpu\": %d, \"sync_ms\": %.3f, \"native\": true}",
                ok ? "true" : "false", gpu, ms);
  return HttpResponse{200, "application/json", body};
}

}  // namespace

int main(int argc, char** argv) {
  // 1 us timer slack, inherited by every thread started from here (see name_thread)
  (void)::prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--help" || std::string(argv[i]) == "-h") {
      std::fputs(kUsage, stdout);
      return 0;
    }
  block_stop_signals();
  Args a(argc, argv, {"no-fsync", "no-fastpath"});
  if (!a.error().empty()) {
    std::fprintf(stderr, "dfs_chunkserver: %s\n", a.error().c_str());
    return 2;
  }
  if (a.flag("no-fastpath")) {
    std::fprintf(stderr, "dfs_chunkserver: --no-fastpath needs the Python shell (DFS_NATIVE_CHUNKSERVER=0)\n");
    return 2;
  }
  const std::string addr = strip_scheme(a.get("addr", "127.0.0.1:50052"));
  const std::string advertise = strip_scheme(a.get("advertise-addr", addr));
  const std::string host = addr.substr(0, addr.rfind(':'));
  const int port = std::atoi(addr.substr(addr.rfind(':') + 1).c_str());
  const int http_port = static_cast<int>(a.get_int("http-port", 8082));
  const int gpu = static_cast<int>(a.get_int("gpu", -1));
  const std::string tls_cert = a.get("tls-cert"), tls_key = a.get("tls-key");
  const bool tls = !tls_cert.empty() && !tls_key.empty();
  const std::string storage_dir = a.get("storage-dir", "/tmp/chunkserver_data");
  if (gpu >= 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || gpu >= n) {
      std::fprintf(stderr, "dfs_chunkserver: no HIP device %d (%d visible)\n", gpu, n);
      return 1;
    }
  }

  // ---------------- block store
  StoreConfig sc;
  sc.storage_dir = storage_dir;
  sc.cold_dir = a.get("cold-storage-dir");
  sc.device = gpu;
  sc.hbm_capacity = parse_size(a.get("hbm-capacity", "0"));
  sc.durability = a.get("durability", "nvme-sync") == "hbm-ack" ? Durability::HbmAck : Durability::NvmeSync;
  sc.cache_blocks = std::atoi(env("BLOCK_CACHE_SIZE", "100").c_str());
  sc.lanes = static_cast<int>(a.get_int("lanes", [] {  // DFS_CS_LANES: the default when --lanes is absent
    const char* e = std::getenv("DFS_CS_LANES");
    // 16: with 8, waiting stagings, receives, reads and spills queued for a stream context
    // (4,050 waits, 0.87 s in one 2-rank run; 16 lanes: 15 waits, profiles/r5_repl/laneab)
    return e && std::atoi(e) > 0 ? std::atoi(e) : 16;
  }()));
  sc.spill_threads = 4;
  sc.sync_writes = !a.flag("no-fsync");
  std::unique_ptr<ChunkStore> store;
  try {
    store = std::make_unique<ChunkStore>(sc);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "dfs_chunkserver: chunk store: %s\n", e.what());
    return 1;
  }

  // ---------------- fast path (same-host clients, replica descriptors, engine control)
  std::string err;
  FastPathServer fp(store.get(), "dfs_fp_" + std::to_string(port));
  if (!fp.start(&err)) log(kWarning, kLog, "native fast path disabled: %s", err.c_str());
  fp.set_self_host(advertise.substr(0, advertise.rfind(':')));
  fp.set_self_addr(advertise);

  // ---------------- replication engine
  std::unique_ptr<ReplicationEngine> engine;
  int pairs_up = 0;
  const std::string transport = a.get("replication-transport", "hipipc");
  const int rank = static_cast<int>(a.get_int("rccl-rank", -1)), world = static_cast<int>(a.get_int("rccl-world", 0));
  const std::string rdv = a.get("rccl-rendezvous");
  const int rccl_timeout = static_cast<int>(a.get_int("rccl-timeout-ms", 60000));
  if ((transport == "hipipc" || transport == "hipipc-spin" || transport == "rccl" || transport == "socket") &&
      world > 1 && rank >= 0 && !rdv.empty() && (gpu >= 0 || transport == "socket")) {
    std::map<std::string, int> ranks;
    std::map<std::string, std::string> names;
    if (!rendezvous(rdv, rank, world, advertise, fp.name(), 120.0, &ranks, &names)) {
      std::fprintf(stderr, "dfs_chunkserver: rendezvous: only %zu/%d chunkservers published in %s\n", ranks.size(),
                   world, rdv.c_str());
      return 1;
    }
    char ns[16];
    const std::string ap = abs_path(rdv);
    std::snprintf(ns, sizeof(ns), "%08x", crc32(reinterpret_cast<const uint8_t*>(ap.data()), ap.size()));
    auto t = make_transport(transport, store.get(), rank, ns, 0, &err);
    if (!t) {
      log(kError, kLog, "replication engine unavailable (%s); using gRPC replication", err.c_str());
    } else {
      ReplOptions o;
      o.open_timeout_ms = rccl_timeout;
      o.turn_timeout_ms = static_cast<int>(a.get_int("repl-turn-timeout-ms", 3000));
      o.xfer_timeout_ms = std::min(rccl_timeout, 20000);
      o.channels = t->channels();
      engine = std::make_unique<ReplicationEngine>(store.get(), std::move(t), rank, world, o);
      for (const auto& kv : ranks)
        if (kv.second != rank) fp.set_peer(kv.first, kv.second, names.count(kv.first) ? names[kv.first] : "");
      fp.set_replication(engine.get());
      engine->set_control([&fp](int r, const std::string& req, std::string* reply) { return fp.control(r, req, reply); });
      engine->start();
      // pairs come up in the background; wait a bounded time so a benchmark starts with its
      // channels ready (a pair that is not up just falls back per block)
      pairs_up = engine->wait_ready(rccl_timeout);
      log(kInfo, kLog, "%s replication: rank %d/%d, %d/%d pairs up, %d channels", transport.c_str(), rank, world,
          pairs_up, world - 1, engine->channels());
    }
  }

  // ---------------- control loop: heartbeats, commands, recovery, scrubber
  std::vector<std::string> masters;
  for (auto& m : split_csv(a.get("masters"))) masters.push_back(strip_scheme(m));
  const std::string shard_cfg = env("SHARD_CONFIG");
  if (!shard_cfg.empty())
    for (auto& m : shard_config_masters(shard_cfg))
      if (std::find(masters.begin(), masters.end(), m) == masters.end()) masters.push_back(m);
  std::shared_ptr<TlsContext> client_tls;
  if (tls) {
    client_tls = TlsContext::client(a.get("ca-cert"), a.get("domain-name"), &err);
    if (!client_tls) {
      std::fprintf(stderr, "dfs_chunkserver: client TLS: %s\n", err.c_str());
      return 1;
    }
  }
  CsAgentConfig ac;
  ac.advertise = advertise;
  ac.rack_id = a.get("rack-id");
  ac.storage_dir = storage_dir;
  ac.gpu_rank = rank;
  ac.masters = masters;
  for (auto& c : split_csv(a.get("config-servers"))) ac.config_servers.push_back(strip_scheme(c));
  ac.heartbeat_ms = std::max(10, static_cast<int>(a.get_double("heartbeat-interval", 5.0) * 1000));
  ac.scrub_ms = std::max(10, static_cast<int>(a.get_double("scrub-interval", 60.0) * 1000));
  ac.tls = tls;
  CsAgent agent(ac, store.get(), &fp, client_tls);

  // ---------------- ChunkServerService, every case native
  auto peers = std::make_shared<GrpcChannelPool>(120000, client_tls);
  NativeChunkService svc(store.get(), &fp, nullptr);
  svc.set_native(&agent, peers);
  GrpcServer grpc(host.empty() ? "0.0.0.0" : host, port, [&svc](const GrpcCall& c) { return svc.handle(c); },
                  static_cast<int>(a.get_int("workers", 64)));
  grpc.set_body_allocator([&svc](size_t len) { return svc.request_buffer(len); }, NativeChunkService::kRequestBufferMin);
  if (tls) {
    auto t = TlsContext::server(tls_cert, tls_key, &err);
    if (!t) {
      std::fprintf(stderr, "dfs_chunkserver: TLS: %s\n", err.c_str());
      return 1;
    }
    grpc.set_tls(std::move(t));
  }
  if (!grpc.start(&err)) {
    std::fprintf(stderr, "dfs_chunkserver: gRPC server: %s\n", err.c_str());
    return 1;
  }

  // ---------------- HTTP side channel
  auto stats_json_all = [&]() {
    Json d = stats_json(store->stats());
    merge_into(&d, stats_json(fp.stats()));
    const CsGrpcStats gs = svc.stats();
    merge_into(&d, stats_json(gs, grpc.calls()));
    merge_into(&d, stats_json(agent.stats()));
    // the Python service's counter names (bench.py and the tests read them)
    d.set("writes", gs.native_writes);
    d.set("reads", gs.native_reads);
    d.set("replicas_in", gs.native_replicates);
    d.set("grpc_forwards", gs.grpc_forwards);
    d.set("rccl_forwards", static_cast<uint64_t>(0));  // engine hops are fp_rccl_forwards
    d.set("rccl_fallbacks", static_cast<uint64_t>(0));
    d.set("recoveries", gs.recoveries);
    d.set("shm_writes", gs.shm_writes);
    d.set("shm_reads", gs.shm_reads);
    if (engine) {
      merge_into(&d, stats_json(engine->stats()), "repl_");
      d.set("repl_channels", engine->channels());
      d.set("repl_transport", engine->transport_name());
      int up = 0, pulls = 0;
      for (int r = 0; r < engine->world(); ++r)
        if (r != engine->rank() && engine->pair_ok(r)) {
          ++up;
          if (engine->transport()->pulls_from(r)) ++pulls;  // hipipc receiver pull from that peer
        }
      d.set("repl_pairs_up", up);
      d.set("repl_pull_peers", pulls);
    }
    d.set("native_chunkserver", true);
    // CPU milliseconds by thread name (live threads): what the process spends its cores on
    Json tc = Json::object();
    for (const auto& [name, ms] : thread_cpu_ms()) tc.set(name, static_cast<uint64_t>(ms));
    d.set("thread_cpu_ms", tc);
    return d;
  };
  Gauges metrics;
  auto disk = [&](bool used) {
    struct statvfs sv;
    if (::statvfs(storage_dir.c_str(), &sv) != 0) return 0.0;
    const double total = static_cast<double>(sv.f_blocks) * sv.f_frsize, avail = static_cast<double>(sv.f_bavail) * sv.f_frsize;
    return used ? total - avail : avail;
  };
  metrics.add("dfs_chunkserver_available_space_bytes", "free bytes on the storage fs", [&] { return disk(false); });
  metrics.add("dfs_chunkserver_used_space_bytes", "used bytes on the storage fs", [&] { return disk(true); });
  metrics.add("dfs_chunkserver_total_chunks", "blocks held", [&] { return static_cast<double>(store->stats().blocks); });
  for (const char* k : {"hbm_capacity", "hbm_used", "hbm_resident_blocks", "dirty_blocks", "spill_queue", "evictions",
                        "promotions", "crc_mismatches", "gpu_kernel_launches", "disk_gate_waits", "journal_live_bytes",
                        "journal_used_bytes", "materialized_blocks", "relocated_blocks"}) {
    const std::string key = k;
    metrics.add("dfs_chunkserver_" + key, "chunk store " + key,
                [&, key] { return stats_json(store->stats())[key].as_double(); });
  }
  metrics.add("dfs_chunkserver_rccl_bytes_sent", "bytes replicated over the engine",
              [&] { return engine ? static_cast<double>(engine->stats().bytes_sent) : 0.0; });
  metrics.add("dfs_chunkserver_rccl_bytes_recv", "bytes received over the engine",
              [&] { return engine ? static_cast<double>(engine->stats().bytes_recv) : 0.0; });
  for (const char* k : {"native_grpc_writes", "native_grpc_reads", "native_grpc_replicates", "native_grpc_forwards",
                        "native_grpc_recoveries"}) {
    const std::string key = k;
    metrics.add(std::string("dfs_chunkserver_") + k + "_total", key,
                [&, key] { return stats_json(svc.stats(), grpc.calls())[key].as_double(); });
  }
  const bool debug = env("DFS_DEBUG_ENDPOINTS") == "1";
  HttpLiteServer http(host.empty() ? "0.0.0.0" : host, http_port, [&](const HttpRequest& req) -> HttpResponse {
    if (req.path == "/health") return HttpResponse{200, "text/plain", "OK"};
    if (req.path == "/metrics") return HttpResponse{200, "text/plain", metrics.render()};
    if (req.path == "/sync") return sync_device(gpu);
    if (req.path == "/stats") return json_response(stats_json_all().dump());
    if (req.path == "/export") {  // every journal-resident block as <id> + <id>.meta, now
      store->materialize_all();
      return json_response(Json(Json::Object{{"exported", Json(store->stats().materialized_blocks)}}).dump());
    }
    if (req.path == "/compact") {
      const auto q = parse_query(req.query);
      const double ml = q.count("max_live") ? std::atof(q.at("max_live").c_str()) : 0.5;
      return json_response(Json(Json::Object{{"relocated", Json(store->compact(ml))}}).dump());
    }
    if (debug && req.path.rfind("/debug/", 0) == 0) {
      // fault injection for tests (off unless DFS_DEBUG_ENDPOINTS=1), as the Python shell
      const auto q = parse_query(req.query);
      auto qs = [&](const char* k, const char* d = "") { return q.count(k) ? q.at(k) : std::string(d); };
      if (req.path == "/debug/corrupt")
        return json_response(Json(Json::Object{{"corrupted", Json(store->debug_corrupt(
                                                                  qs("block"), std::stoull(qs("offset", "0"))))}})
                                 .dump());
      if (req.path == "/debug/scrub") {
        Json bad = Json::array();
        for (auto& b : agent.scrub_once()) bad.push_back(Json(b));
        return json_response(Json(Json::Object{{"bad", bad}}).dump());
      }
      if (req.path == "/debug/pause_spill") {
        store->debug_pause_spill(qs("on", "1") == "1");
        return json_response("{}");
      }
      if (req.path == "/debug/remove")
        return json_response(Json(Json::Object{{"removed", Json(store->remove(qs("block")))}}).dump());
      if (req.path == "/debug/command") {
        agent.submit_command(from_hex(qs("hex")));
        return json_response("{}");
      }
      if (req.path == "/debug/drop_resident") {
        store->drop_resident();
        return json_response("{}");
      }
      if (req.path == "/debug/drop_descriptors") {
        fp.debug_drop_descriptors(std::atoi(qs("n", "1").c_str()));
        return json_response("{}");
      }
      if (req.path == "/debug/drop_sends" && engine) {
        engine->transport()->debug_drop_sends(std::atoi(qs("peer").c_str()), std::atoi(qs("n", "1").c_str()));
        return json_response("{}");
      }
      if (req.path == "/debug/fail_pair" && engine) {
        engine->fail_pair(std::atoi(qs("peer").c_str()), "debug");
        return json_response("{}");
      }
    }
    return HttpResponse{404, "text/plain", "Not Found"};
  });
  if (!http.start(&err)) {
    std::fprintf(stderr, "dfs_chunkserver: HTTP: %s\n", err.c_str());
    return 1;
  }
  // GET /sync on a listener of its own: the benchmark's device-sync bracket never queues
  // behind a /stats or /metrics request
  HttpLiteServer sync_srv("127.0.0.1", 0, [gpu](const HttpRequest& r) -> HttpResponse {
    if (r.path != "/sync") return HttpResponse{404, "text/plain", "Not Found"};
    return sync_device(gpu);
  });
  int sync_port = 0;
  if (sync_srv.start(&err)) sync_port = sync_srv.port();

  agent.start();
  write_ready_file(Json(Json::Object{{"addr", Json(addr)},
                                     {"gpu", Json(gpu)},
                                     {"rccl", Json(engine != nullptr)},
                                     {"transport", Json(engine ? std::string(engine->transport_name()) : "grpc")},
                                     {"pairs_up", Json(pairs_up)},
                                     {"sync_port", Json(sync_port)},
                                     {"native", Json(true)}})
                       .dump());
  log(kInfo, kLog, "chunkserver %s serving (gpu=%d, durability=%s, journal=%s)", advertise.c_str(), gpu,
      a.get("durability", "nvme-sync").c_str(), store->stats().journal_mode.c_str());

  wait_for_stop();
  agent.stop();
  grpc.stop();
  http.stop();
  sync_srv.stop();
  if (engine) engine->stop();
  fp.stop();
  store->flush();
  engine.reset();
  store.reset();
  return 0;
}
