// dfs_config_server — the native config-server process (C36; reference
// dfs/metaserver/src/bin/config_server.rs:66-172). One Raft member of the configuration
// group: ConfigCore holds and applies the shard map + master registry on the Raft applier
// thread and answers every ConfigService RPC; this executable owns the process around it —
// the native Raft node, the HTTP/2 gRPC server (ConfigService + /dfs.RaftPeer/*), the
// same-host socket listener, and the HTTP side channel (/raft/{vote,append,snapshot,
// timeout_now}, /raft/state, /raft/endpoint, /shards, /health, /metrics). No Python runs in
// it.
//
// Flags (the reference's spelling and defaults, printed by --help): --addr, --id, --peers,
// --http-port, --advertise-addr, --storage-dir, --tls-cert, --tls-key, --ca-cert,
// --no-fsync, --snapshot-threshold.
#include <cstdio>
#include <memory>
#include <string>
#include <thread>

#include "config_core.h"
#include "grpc_server.h"
#include "localrpc.h"
#include "node_shell.h"
#include "raft.h"
#include "tls.h"
#include "trace.h"

using namespace dfs;
using namespace dfs::shell;

static const char* kUsage =
    "usage: dfs_config_server [--addr ADDR] [--id ID] [--peers PEERS] [--http-port HTTP_PORT]\n"
    "                         [--advertise-addr ADVERTISE_ADDR] [--storage-dir STORAGE_DIR] [--tls-cert TLS_CERT]\n"
    "                         [--tls-key TLS_KEY] [--ca-cert CA_CERT] [--no-fsync]\n"
    "                         [--snapshot-threshold SNAPSHOT_THRESHOLD]\n";

// The reference's defaults (bin/config_server.rs:19-48), printed by --help.
const std::map<std::string, std::string> kDefaults = {{"addr", "127.0.0.1:50052"},
                                                      {"id", "1"},
                                                      {"http-port", "8081"},
                                                      {"storage-dir", "/tmp/config-raft-logs"},
                                                      {"snapshot-threshold", "10000"}};

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--help" || std::string(argv[i]) == "-h") {
      std::fputs(kUsage, stdout);
      std::fputs(defaults_help(kDefaults).c_str(), stdout);
      return 0;
    }
  block_stop_signals();
  Args a(argc, argv, {"no-fsync"}, {}, kDefaults);
  if (!a.error().empty()) {
    std::fprintf(stderr, "dfs_config_server: %s\n", a.error().c_str());
    return 2;
  }
  const std::string addr = a.get("addr", "127.0.0.1:50052");
  const int id = static_cast<int>(a.get_int("id", 1));
  const int http_port = static_cast<int>(a.get_int("http-port", 8081));
  const std::string host = addr.find(':') != std::string::npos ? addr.substr(0, addr.find(':')) : "127.0.0.1";
  const std::string self_http = "http://" + host + ":" + std::to_string(http_port);
  const std::string client_addr = with_scheme(a.get("advertise-addr", addr));
  const std::string tls_cert = a.get("tls-cert"), tls_key = a.get("tls-key");
  const bool tls = !tls_cert.empty() && !tls_key.empty();

  auto core = std::make_shared<ConfigCore>();
  raft::Options o;
  o.id = id;
  o.members = initial_members(id, self_http, split_csv(a.get("peers")));
  o.client_address = client_addr;
  o.dir = a.get("storage-dir", "/tmp/config-raft-logs") + "/raft_node_" + std::to_string(id);
  o.sync = !a.flag("no-fsync");
  o.snapshot_threshold = static_cast<uint64_t>(a.get_int("snapshot-threshold", 10000));
  auto raft_host = std::make_shared<NativeRaftHost>(core);
  auto node = std::make_unique<raft::Node>(o, raft_host);
  core->attach(node.get());

  // ConfigService + Raft peer RPCs over HTTP/2
  std::atomic<uint64_t> raft_calls{0};
  static const std::string kPrefix = "/dfs.ConfigService/", kRaft = "/dfs.RaftPeer/";
  const std::string bind = addr.find(':') != std::string::npos ? addr : "0.0.0.0:" + addr;
  const std::string bhost = bind.substr(0, bind.rfind(':'));
  const int gport = std::atoi(bind.substr(bind.rfind(':') + 1).c_str());
  GrpcServer grpc(bhost, gport, [&](const GrpcCall& c) -> GrpcReply {
    GrpcReply r;
    RequestScope scope(c.request_id);
    if (c.path.compare(0, kRaft.size(), kRaft) == 0) {
      r.status = core->raft_rpc(c.path.substr(kRaft.size()), c.message, &r.message);
      raft_calls++;
    } else if (c.path.compare(0, kPrefix.size(), kPrefix) == 0) {
      r.status = core->handle(c.path.substr(kPrefix.size()), c.message, &r.message);
    } else {
      r.status = 12;
      r.message = "unknown service: " + c.path;
    }
    return r;
  }, 16);
  std::string err;
  if (tls) {
    auto t = TlsContext::server(tls_cert, tls_key, &err);
    if (!t) {
      std::fprintf(stderr, "dfs_config_server: TLS: %s\n", err.c_str());
      return 1;
    }
    grpc.set_tls(std::move(t));
  }
  if (!grpc.start(&err)) {
    std::fprintf(stderr, "dfs_config_server: gRPC server: %s\n", err.c_str());
    return 1;
  }
  std::unique_ptr<LocalRpcServer> local;
  if (!tls && env("DFS_NO_LOCALRPC") != "1") {
    local = std::make_unique<LocalRpcServer>(
        "dfs_rpc_" + std::to_string(gport),
        [&](const std::string& path, const std::string& rid, const std::string& payload, std::string* out) -> int {
          RequestScope scope(rid);
          if (path.compare(0, kPrefix.size(), kPrefix) != 0) return (*out = "unknown service: " + path, 12);
          return core->handle(path.substr(kPrefix.size()), payload, out);
        });
    if (!local->start(&err)) {
      log(kWarning, "dfs.config_server", "local RPC listener unavailable: %s", err.c_str());
      local.reset();
    }
  }

  Gauges metrics;
  metrics.add("raft_role", "0=follower 1=candidate 2=leader", [&] { return static_cast<double>(static_cast<int>(node->role())); });
  metrics.add("config_shards", "shards in the map", [&] {
    return static_cast<double>(ShardMap::from_json(Json::parse(core->shard_map_json())).shards().size());
  });
  metrics.add("config_native_requests", "ConfigService RPCs answered by the native core",
              [&] { return static_cast<double>(core->requests()); });
  metrics.add("config_native_raft_rpcs", "Raft peer RPCs received over the native server",
              [&] { return static_cast<double>(raft_calls.load()); });

  HttpLiteServer http(host, http_port, [&](const HttpRequest& req) -> HttpResponse {
    if (req.path.rfind("/raft/", 0) == 0 && req.method == "POST") return raft_http(*node, req);
    if (req.path == "/health") return HttpResponse{200, "text/plain", "OK"};
    if (req.path == "/metrics") return HttpResponse{200, "text/plain", metrics.render()};
    if (req.path == "/raft/state") return json_response(node->info_json());
    if (req.path == "/raft/endpoint") return json_response(Json(Json::Object{{"grpc", Json(client_addr)}}).dump());
    if (req.path == "/shards") {
      Json arr = Json::array();
      for (auto& s : ShardMap::from_json(Json::parse(core->shard_map_json())).shards()) arr.push_back(Json(s));
      return json_response(Json(Json::Object{{"shards", arr}}).dump());
    }
    return HttpResponse{404, "text/plain", "Not Found"};
  });
  if (!http.start(&err)) {
    std::fprintf(stderr, "dfs_config_server: %s\n", err.c_str());
    return 1;
  }
  node->start();
  std::atomic<bool> stop{false};
  std::thread resolver([&] { resolve_peers_loop(*node, *raft_host, stop); });
  write_ready_file(Json(Json::Object{{"addr", Json(addr)}, {"native", Json(true)}}).dump());
  log(kInfo, "dfs.config_server", "config server %d serving %s (http %d)", id, addr.c_str(), http_port);

  wait_for_stop();
  stop = true;
  resolver.join();
  if (local) local->stop();
  grpc.stop();
  http.stop();
  node->stop();
  core->detach();
  return 0;
}
