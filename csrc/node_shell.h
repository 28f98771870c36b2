// Process shell shared by the native control-plane executables (dfs_master,
// dfs_config_server): flag parsing in the reference's spelling, the initial Raft membership,
// the Raft host that hands the node's peer RPCs to the native HTTP/2 path or to the peers'
// HTTP/JSON endpoints, peer-endpoint discovery, Prometheus text, readiness file and signals.
// (Reference: bin/master.rs:97-255, bin/config_server.rs:66-172, simple_raft.rs:791-807
// for peer ids, :1313-1651 for the HTTP retry policy.)
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "grpc_client.h"
#include "http_lite.h"
#include "raft.h"

namespace dfs::shell {

// --name value / --name=value / -a value; boolean flags take no value.
class Args {
 public:
  // `defaults`: the value of a flag that is not given (the reference's clap defaults); a
  // default passed to get() applies only to flags without one here.
  Args(int argc, char** argv, const std::set<std::string>& bool_flags,
       const std::map<std::string, std::string>& short_names = {},
       const std::map<std::string, std::string>& defaults = {});
  std::string get(const std::string& name, const std::string& dflt = "") const;
  int64_t get_int(const std::string& name, int64_t dflt) const;
  double get_double(const std::string& name, double dflt) const;
  bool flag(const std::string& name) const { return flags_.count(name) != 0; }
  bool has(const std::string& name) const { return kv_.count(name) != 0; }
  const std::string& error() const { return err_; }

 private:
  std::map<std::string, std::string> kv_, defaults_;
  std::set<std::string> flags_;
  std::string err_;
};

// "  --name default" lines of a defaults table (the --help text's defaults section).
std::string defaults_help(const std::map<std::string, std::string>& defaults);
std::string with_scheme(const std::string& addr, bool tls = false);
std::vector<std::string> split_csv(const std::string& s);
// "3@http://h:p" -> (3, url); "...metaserver-N..." -> (N + 1, url); else (-1, url)
std::pair<int, std::string> parse_peer(const std::string& spec);
std::map<int, std::string> initial_members(int id, const std::string& self_addr, const std::vector<std::string>& peers);
std::string env(const char* name, const std::string& dflt = "");
int64_t now_ms();

// raft::Host over a native state machine. Peer RPCs go to a peer's native endpoint
// (/dfs.RaftPeer/<kind> on its HTTP/2 port) once discovered, else POST JSON to
// <peer>/raft/<kind> with the reference's retries; `blocked` peers are unreachable.
class NativeRaftHost : public raft::Host {
 public:
  explicit NativeRaftHost(std::shared_ptr<raft::StateMachine> sm, std::shared_ptr<TlsContext> peer_tls = nullptr);
  std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) override;
  std::string snapshot() override;
  void restore(const std::string& state) override;
  bool send(const std::string& addr, const std::string& kind, const std::string& body, std::string* reply) override;
  void backup(const std::string& url, const std::string& data) override;
  void set_peer_endpoint(const std::string& addr, const std::string& endpoint) override;
  void set_blocked(const std::vector<std::string>& addrs) override;
  std::vector<std::string> blocked() const;
  bool has_endpoint(const std::string& addr) const;

 private:
  std::shared_ptr<raft::StateMachine> sm_;
  mutable std::mutex mu_;
  std::map<std::string, std::string> endpoints_;
  std::set<std::string> blocked_;
  std::unique_ptr<GrpcChannelPool> peers_;
};

// Asks every member without a known native endpoint for GET /raft/endpoint once a second
// until `stop` (the Python shell's resolve_native_peers).
void resolve_peers_loop(raft::Node& node, NativeRaftHost& host, const std::atomic<bool>& stop);

// POST /raft/<kind> on the HTTP side channel -> the node's blocking handler.
HttpResponse raft_http(raft::Node& node, const HttpRequest& req);
HttpResponse json_response(const std::string& body, int status = 200);

// Prometheus text exposition of gauges, in registration order.
class Gauges {
 public:
  void add(const std::string& name, const std::string& help, std::function<double()> fn);
  std::string render() const;

 private:
  struct G {
    std::string name, help;
    std::function<double()> fn;
  };
  std::vector<G> gs_;
};

// SIGTERM / SIGINT are blocked in every thread from here on (call first in main); wait_for_stop
// returns when one arrives.
void block_stop_signals();  // also installs install_crash_handler()
// SIGSEGV / SIGBUS / SIGFPE / SIGILL / SIGABRT print a backtrace to stderr before the default action
void install_crash_handler();
void wait_for_stop();
void write_ready_file(const std::string& json);  // $DFS_READY_FILE, if set

// Log lines in the Python services' layout ("<time> <LEVEL> <name> [req=-] <msg>") on stderr,
// filtered by DFS_LOG (debug|info|warning|error; default warning).
void log(int level, const char* name, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
enum { kDebug = 10, kInfo = 20, kWarning = 30, kError = 40 };

}  // namespace dfs::shell
