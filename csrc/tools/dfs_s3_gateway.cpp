// dfs_s3_gateway — the S3 gateway as one native process (C52-C57; reference
// dfs/s3_server/src/main.rs:243-274 for the process, handlers.rs for the object API,
// auth_middleware.rs for SigV4, sts_handler.rs for STS).
//
// The S3 front (csrc/s3_front.cpp) with no Python backend: every request is answered in this
// process. The object, multipart, bucket and policy API; SigV4 (header, presigned, aws-chunked
// chunk chains), STS sessions with their IAM role policies and bucket policies; STS
// AssumeRoleWithWebIdentity against the OIDC issuer (csrc/sts.cpp); SSE-S3; the error answers
// of every request the data path does not serve (auth errors with the reference's codes,
// NoSuchKey / NoSuchBucket / NoSuchUpload / MalformedXML ...); /health and /metrics. Audit
// records go to the native hash-chained writer (csrc/audit_log.cpp) in this process.
//
// Configuration is the Python gateway's environment (tests/models/s3_gateway.py S3Config): MASTER_ADDR,
// CONFIG_SERVERS, SHARD_CONFIG, LOCAL_CHUNKSERVER, CA_CERT, DOMAIN_NAME, PORT, TLS_CERT /
// TLS_KEY, S3_AUTH_ENABLED, S3_ACCESS_KEY / S3_SECRET_KEY, S3_REGION, S3_REQUIRE_TLS,
// S3_ALLOW_UNSIGNED_PAYLOAD, OIDC_ISSUER_URL / OIDC_CLIENT_ID / OIDC_ALLOW_HS256,
// STS_SIGNING_KEY, IAM_CONFIG_PATH, SSE_MASTER_KEY, AUDIT_LOG_* / AUDIT_HMAC_SECRET; plus
// S3_FRONT_THREADS, S3_FRONT_SLOTS and S3_FRONT_SLOT_MB (the largest single PUT). Flags:
// --port, --host, --workers (or S3_WORKERS). S3_METADATA_SIDECAR=true also writes the
// reference's `<key>.meta` sidecar files (objects without attributes are always described by
// theirs).
//
// S3_WORKERS=N > 1: this process (worker 0) owns the audit hash chain and the policy epoch page
// and starts N-1 copies of itself on the same port (SO_REUSEPORT: the kernel spreads the
// connections). The copies send their audit records to worker 0's ingest socket as datagrams,
// so one writer keeps one chain, and share its epoch page, so a bucket-policy change made
// through any worker reaches all of them. They exit with worker 0 (PR_SET_PDEATHSIG).
#include <signal.h>
#include <spawn.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "audit_log.h"
#include "client_fast.h"
#include "dfs_pb.h"
#include "front_store.h"
#include "grpc_client.h"
#include "json.h"
#include "node_shell.h"
#include "s3_front.h"
#include "shard_map.h"
#include "tls.h"

extern char** environ;

using namespace dfs;
using dfs::shell::log;
using dfs::shell::kError;
using dfs::shell::kInfo;
using dfs::shell::kWarning;

namespace {

const char* kLog = "dfs.s3";

std::string env(const char* k, const std::string& d = "") {
  const char* v = std::getenv(k);
  return v ? std::string(v) : d;
}

std::string read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::string with_scheme(const std::string& a, bool tls) {
  if (a.find("://") != std::string::npos) return a;
  return (tls ? "https://" : "http://") + a;
}

// The shard map of SHARD_CONFIG ({"shards": {id: [peers]}, "ranges": {...}}), as serde JSON.
std::string shard_config_json(const std::string& path) {
  Json cfg = Json::parse(read_file(path));
  ShardMap m = ShardMap::new_range();
  for (auto& kv : cfg["shards"].fields()) {
    std::vector<std::string> peers;
    for (auto& p : kv.second.items()) peers.push_back(p.str());
    m.add_shard(kv.first, peers);
  }
  Json j = m.to_json();
  if (cfg["ranges"].is_object()) {
    Json r = Json::object();
    for (auto& kv : cfg["ranges"].fields()) r.set(kv.first, kv.second.str());
    j.set("strategy", Json(Json::Object{{"Range", Json(Json::Object{{"ranges", r}})}}));
  }
  return ShardMap::from_json(j).to_json().dump();
}

// FetchShardMap from the first config server that answers (ShardMap.from_fetch).
std::string fetch_shard_map(GrpcChannelPool& pool, const std::vector<std::string>& servers, bool tls) {
  for (auto& c : servers) {
    GrpcResult r = pool.call(with_scheme(c, tls), "/dfs.ConfigService/FetchShardMap", std::string(), "", 5000);
    if (!r.transport_ok || r.status != 0) continue;
    pb::FetchShardMapResponse resp;
    if (!resp.decode(r.message) || resp.shards.empty()) continue;
    ShardMap m = ShardMap::new_range();
    for (auto& kv : resp.shards) m.add_shard(kv.first, kv.second.peers);
    Json j = m.to_json();
    if (!resp.ranges.empty()) {
      Json ranges = Json::object();
      for (auto& kv : resp.ranges)
        if (resp.shards.count(kv.second)) ranges.set(kv.first, Json(kv.second));
      j.set("strategy", Json(Json::Object{{"Range", Json(Json::Object{{"ranges", ranges}})}}));
    }
    return ShardMap::from_json(j).to_json().dump();
  }
  return std::string();
}

bool parse_hex32(const std::string& hex, std::string* out) {
  std::string h;
  for (char ch : hex)
    if (!std::isspace(static_cast<unsigned char>(ch))) h.push_back(ch);
  if (h.size() != 64) return false;
  out->clear();
  for (size_t i = 0; i < 64; i += 2) {
    char* end = nullptr;
    const std::string b = h.substr(i, 2);
    long v = std::strtol(b.c_str(), &end, 16);
    if (!end || *end) return false;
    out->push_back(static_cast<char>(v));
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  std::string host = "0.0.0.0";
  int port = std::atoi(env("PORT", "9000").c_str());
  int workers = std::max(1, std::atoi(env("S3_WORKERS", "1").c_str()));
  // a copy started by worker 0: its private directory (audit ingest socket, policy epoch page)
  const std::string parent_dir = env("DFS_S3_WORKER_OF");
  if (!parent_dir.empty()) ::prctl(PR_SET_PDEATHSIG, SIGTERM);
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--port") port = std::atoi(val().c_str());
    else if (a == "--host") host = val();
    else if (a == "--workers") workers = std::max(1, std::atoi(val().c_str()));
    else if (a == "-h" || a == "--help") {
      std::printf("usage: dfs_s3_gateway [--port PORT] [--host HOST] [--workers N]\n"
                  "configuration from the environment (see the header of csrc/tools/dfs_s3_gateway.cpp)\n");
      return 0;
    }
  }
  shell::block_stop_signals();
  S3FrontConfig cfg;
  cfg.metadata_sidecar = env("S3_METADATA_SIDECAR") == "true";
  cfg.reuse_port = workers > 1 || !parent_dir.empty();
  cfg.host = host;
  cfg.port = port;
  cfg.backend = "";  // no Python workers: every request is answered here
  cfg.workers = std::atoi(env("S3_FRONT_THREADS", "32").c_str());
  cfg.auth_enabled = env("S3_AUTH_ENABLED") == "true";
  cfg.region = env("S3_REGION", "us-east-1");
  cfg.access_key = env("S3_ACCESS_KEY");
  cfg.secret_key = env("S3_SECRET_KEY");
  cfg.allow_unsigned_payload = env("S3_ALLOW_UNSIGNED_PAYLOAD", "true") == "true";
  cfg.require_tls = env("S3_REQUIRE_TLS") == "true";
  const std::string tls_cert = env("TLS_CERT"), tls_key = env("TLS_KEY");
  if (!tls_cert.empty() && !tls_key.empty()) {
    cfg.tls_cert = tls_cert;
    cfg.tls_key = tls_key;
  }
  if (!env("SSE_MASTER_KEY").empty()) {
    std::string kek;
    if (parse_hex32(env("SSE_MASTER_KEY"), &kek)) {
      cfg.sse_enabled = true;
      cfg.sse_kek = kek;
    } else {
      log(kError, kLog, "SSE disabled: SSE_MASTER_KEY must be 32 bytes (64 hex chars)");
    }
  }
  if (!env("STS_SIGNING_KEY").empty()) cfg.sts_keys[1] = env("STS_SIGNING_KEY");
  if (!env("IAM_CONFIG_PATH").empty()) {
    try {
      cfg.iam_config = read_file(env("IAM_CONFIG_PATH"));
    } catch (const std::exception& e) {
      log(kError, kLog, "failed to load IAM config %s: %s", env("IAM_CONFIG_PATH").c_str(), e.what());
    }
  }
  cfg.oidc_issuer = env("OIDC_ISSUER_URL");
  cfg.oidc_client_id = env("OIDC_CLIENT_ID");
  cfg.oidc_allow_hs256 = env("OIDC_ALLOW_HS256") == "true";
  cfg.oidc_ca = env("OIDC_CA_CERT");

  // private directory: the policy epoch page and the audit ingest socket (worker 0's, shared
  // by the copies it starts)
  char tmpl[] = "/tmp/s3gw-XXXXXX";
  const std::string priv = !parent_dir.empty() ? parent_dir : ::mkdtemp(tmpl) ? tmpl : "/tmp";
  cfg.policy_epoch_path = priv + "/policy_epoch";
  std::unique_ptr<AuditLog> audit;
  int ingest_fd = -1;
  if (!parent_dir.empty()) {
    if (cfg.auth_enabled && env("AUDIT_LOG_ENABLED", "true") == "true" && env("AUDIT_HMAC_SECRET").size() >= 16)
      cfg.audit_socket = priv + "/ingest.sock";
  } else if (env("AUDIT_LOG_ENABLED", "true") == "true") {
    const std::string secret = env("AUDIT_HMAC_SECRET");
    if (secret.size() >= 16) {
      audit = std::make_unique<AuditLog>(env("AUDIT_LOG_DIR", "/tmp/s3_audit_log"),
                                         std::atoi(env("AUDIT_LOG_RETENTION_DAYS", "30").c_str()),
                                         std::atoi(env("AUDIT_LOG_BATCH_SIZE", "100").c_str()), secret);
      const std::string path = priv + "/ingest.sock";
      ingest_fd = ::socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
      sockaddr_un sa{};
      sa.sun_family = AF_UNIX;
      std::snprintf(sa.sun_path, sizeof sa.sun_path, "%s", path.c_str());
      int buf = 8 << 20;
      ::setsockopt(ingest_fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
      if (::bind(ingest_fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) == 0) {
        audit->start_ingest(ingest_fd);
        if (cfg.auth_enabled) cfg.audit_socket = path;
      } else {
        log(kError, kLog, "audit ingest socket %s: %s", path.c_str(), std::strerror(errno));
      }
    } else {
      log(kWarning, kLog, "audit logging disabled: AUDIT_HMAC_SECRET must be set and at least 16 characters");
    }
  }

  // the DFS side: co-located (FastClient over the chunkserver's shared memory) or remote (gRPC)
  const std::string ca = env("CA_CERT"), domain = env("DOMAIN_NAME");
  std::shared_ptr<TlsContext> ctls;
  if (!ca.empty()) {
    std::string err;
    ctls = TlsContext::client(ca, domain, &err);
    if (!ctls) {
      log(kError, kLog, "TLS client: %s", err.c_str());
      return 1;
    }
  }
  const bool tls = ctls != nullptr;
  std::vector<std::string> masters;
  for (auto& m : shell::split_csv(env("MASTER_ADDR", "http://127.0.0.1:8081"))) masters.push_back(with_scheme(m, tls));
  const std::vector<std::string> cfg_servers = shell::split_csv(env("CONFIG_SERVERS"));
  GrpcChannelPool pool(10000, ctls);
  std::string map_json;
  if (!env("SHARD_CONFIG").empty()) {
    try {
      map_json = shard_config_json(env("SHARD_CONFIG"));
    } catch (const std::exception& e) {
      log(kWarning, kLog, "SHARD_CONFIG: %s", e.what());
    }
  } else if (!cfg_servers.empty()) {
    map_json = fetch_shard_map(pool, cfg_servers, tls);
  }
  const size_t slot_bytes = static_cast<size_t>(std::atol(env("S3_FRONT_SLOT_MB", "128").c_str())) << 20;
  const size_t slots = static_cast<size_t>(std::max(1L, std::atol(env("S3_FRONT_SLOTS", "16").c_str())));
  std::unique_ptr<FastClient> fast;
  std::unique_ptr<LocalFirstFrontStore> local_first;
  std::unique_ptr<RemoteFrontStore> remote;
  std::unique_ptr<S3Front> front;
  const std::string local = env("LOCAL_CHUNKSERVER");
  if (!local.empty() && env("DFS_NATIVE_CLIENT", "1") == "1") {
    const std::string fp = "dfs_fp_" + local.substr(local.rfind(':') + 1);
    fast = std::make_unique<FastClient>(fp, local, slots * slot_bytes, slot_bytes,
                                        std::atoi(env("DFS_HASH_THREADS", "16").c_str()));
    if (!fast->ok()) {
      log(kWarning, kLog, "no shared-memory arena with %s: using gRPC", local.c_str());
      fast.reset();
    }
  }
  if (fast) {
    // the shared-memory client first; what it declines (a leader elsewhere, a dead local
    // master) over gRPC with leader following, the body still in the shared slot
    local_first = std::make_unique<LocalFirstFrontStore>(fast.get(), map_json, masters, 120000, ctls);
    front = std::make_unique<S3Front>(cfg, static_cast<FrontStore*>(local_first.get()));
  } else {
    remote = std::make_unique<RemoteFrontStore>(map_json, masters, slots, slot_bytes, 120000, ctls);
    front = std::make_unique<S3Front>(cfg, static_cast<FrontStore*>(remote.get()));
  }
  std::string err;
  if (!front->start(&err)) {
    log(kError, kLog, "S3 front failed to start: %s", err.c_str());
    return 1;
  }
  // the shard map follows the config servers (splits and merges move ranges)
  std::atomic<bool> stop{false};
  std::thread refresher;
  if (!cfg_servers.empty() && env("SHARD_CONFIG").empty()) {
    refresher = std::thread([&] {
      while (!stop.load()) {
        for (int i = 0; i < 50 && !stop.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (stop.load()) break;
        std::string js = fetch_shard_map(pool, cfg_servers, tls);
        if (js.empty() || js == map_json) continue;
        map_json = js;
        if (local_first) local_first->set_routing(js, masters);
        if (remote) remote->set_routing(js, masters);
      }
    });
  }
  log(kInfo, kLog, "S3 gateway on %s:%d (native process, auth=%d, sse=%d, audit=%d, %s)", host.c_str(), front->port(),
      cfg.auth_enabled, cfg.sse_enabled, audit != nullptr, fast ? "co-located: shared memory" : "remote: gRPC");
  // worker 0 starts the others on the port it bound (an ephemeral --port 0 included)
  std::vector<pid_t> kids;
  if (parent_dir.empty() && workers > 1) {
    char self[4096];
    const ssize_t sl = ::readlink("/proc/self/exe", self, sizeof self - 1);
    if (sl > 0) {
      self[sl] = 0;
      std::vector<std::string> envs;
      for (char** e = environ; *e; ++e) {
        const std::string kv = *e;
        if (kv.compare(0, 15, "DFS_READY_FILE=") != 0 && kv.compare(0, 17, "DFS_S3_WORKER_OF=") != 0) envs.push_back(kv);
      }
      envs.push_back("DFS_S3_WORKER_OF=" + priv);
      std::vector<char*> envp;
      for (auto& kv : envs) envp.push_back(const_cast<char*>(kv.c_str()));
      envp.push_back(nullptr);
      const std::string ps = std::to_string(front->port());
      for (int w = 1; w < workers; ++w) {
        std::vector<std::string> args = {self, "--port", ps, "--host", host, "--workers", "1"};
        std::vector<char*> argp;
        for (auto& s : args) argp.push_back(const_cast<char*>(s.c_str()));
        argp.push_back(nullptr);
        pid_t pid = -1;
        if (::posix_spawn(&pid, self, nullptr, nullptr, argp.data(), envp.data()) == 0) kids.push_back(pid);
        else log(kError, kLog, "starting gateway worker %d: %s", w, std::strerror(errno));
      }
    }
  }
  if (!parent_dir.empty()) {  // a copy: serves until worker 0 stops it
    shell::wait_for_stop();
    stop = true;
    if (refresher.joinable()) refresher.join();
    front->stop();
    return 0;
  }
  Json ready = Json::object();
  ready.set("port", front->port());
  ready.set("workers", static_cast<int>(1 + kids.size()));
  ready.set("native_front", true);
  ready.set("native_gateway", true);
  ready.set("store", fast ? "shm" : "grpc");
  shell::write_ready_file(ready.dump());
  shell::wait_for_stop();
  stop = true;
  for (pid_t k : kids) ::kill(k, SIGTERM);
  for (pid_t k : kids) ::waitpid(k, nullptr, 0);
  if (refresher.joinable()) refresher.join();
  front->stop();
  if (audit) audit->close();
  if (ingest_fd >= 0) ::close(ingest_fd);
  std::remove(cfg.policy_epoch_path.c_str());
  std::remove((priv + "/ingest.sock").c_str());
  ::rmdir(priv.c_str());
  return 0;
}
