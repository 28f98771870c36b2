// Shared shell of the native control-plane executables (see node_shell.h).
#include "trace.h"
#include "node_shell.h"

#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <sys/time.h>
#include <unistd.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <regex>
#include <thread>

#include "json.h"
#include "tls.h"

namespace dfs::shell {

Args::Args(int argc, char** argv, const std::set<std::string>& bool_flags,
           const std::map<std::string, std::string>& short_names, const std::map<std::string, std::string>& defaults)
    : defaults_(defaults) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    std::string name, value;
    bool has_value = false;
    if (a.rfind("--", 0) == 0) {
      name = a.substr(2);
      size_t eq = name.find('=');
      if (eq != std::string::npos) {
        value = name.substr(eq + 1);
        name = name.substr(0, eq);
        has_value = true;
      }
    } else if (a.size() == 2 && a[0] == '-' && short_names.count(a.substr(1))) {
      name = short_names.at(a.substr(1));
    } else {
      err_ = "unexpected argument: " + a;
      return;
    }
    if (bool_flags.count(name)) {
      flags_.insert(name);
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argc) {
        err_ = "--" + name + " needs a value";
        return;
      }
      value = argv[++i];
    }
    kv_[name] = value;
  }
}

std::string Args::get(const std::string& name, const std::string& dflt) const {
  auto it = kv_.find(name);
  if (it != kv_.end()) return it->second;
  auto d = defaults_.find(name);
  return d == defaults_.end() ? dflt : d->second;
}

int64_t Args::get_int(const std::string& name, int64_t dflt) const {
  const std::string v = get(name, "");
  return v.empty() ? dflt : std::strtoll(v.c_str(), nullptr, 10);
}

double Args::get_double(const std::string& name, double dflt) const {
  const std::string v = get(name, "");
  return v.empty() ? dflt : std::strtod(v.c_str(), nullptr);
}

std::string defaults_help(const std::map<std::string, std::string>& defaults) {
  std::string o = "defaults:\n";
  for (auto& kv : defaults) o += "  --" + kv.first + " " + kv.second + "\n";
  return o;
}

std::string with_scheme(const std::string& addr, bool tls) {
  if (addr.rfind("http://", 0) == 0 || addr.rfind("https://", 0) == 0) return addr;
  return (tls ? "https://" : "http://") + addr;
}

std::vector<std::string> split_csv(const std::string& s) {
  std::vector<std::string> out;
  size_t pos = 0;
  while (pos <= s.size()) {
    size_t c = s.find(',', pos);
    if (c == std::string::npos) c = s.size();
    std::string t = s.substr(pos, c - pos);
    size_t a = t.find_first_not_of(" \t"), b = t.find_last_not_of(" \t");
    if (a != std::string::npos) out.push_back(t.substr(a, b - a + 1));
    pos = c + 1;
  }
  return out;
}

std::pair<int, std::string> parse_peer(const std::string& spec) {
  size_t at = spec.find('@');
  if (at != std::string::npos && at > 0) {
    std::string id = spec.substr(0, at);
    if (id.find_first_not_of("0123456789") == std::string::npos) return {std::atoi(id.c_str()), spec.substr(at + 1)};
  }
  static const std::regex pod("(?:configserver|metaserver)-(\\d+)");
  std::smatch m;
  if (std::regex_search(spec, m, pod)) return {std::atoi(m[1].str().c_str()) + 1, spec};
  return {-1, spec};
}

std::map<int, std::string> initial_members(int id, const std::string& self_addr, const std::vector<std::string>& peers) {
  std::map<int, std::string> members{{id, self_addr}};
  std::vector<std::string> unnamed;
  for (auto& p : peers) {
    auto [pid, addr] = parse_peer(p);
    if (pid < 0) unnamed.push_back(addr);
    else members[pid] = addr;
  }
  if (!unnamed.empty()) {
    // peers without an id: deterministic ids from the sorted address list of the whole group
    std::set<std::string> everyone(unnamed.begin(), unnamed.end());
    everyone.insert(self_addr);
    std::vector<std::string> sorted(everyone.begin(), everyone.end());
    for (auto& a : unnamed)
      members[static_cast<int>(std::find(sorted.begin(), sorted.end(), a) - sorted.begin()) + 1] = a;
  }
  return members;
}

std::string env(const char* name, const std::string& dflt) {
  const char* v = std::getenv(name);
  return v ? std::string(v) : dflt;
}

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// ---------------------------------------------------------------- Raft host
NativeRaftHost::NativeRaftHost(std::shared_ptr<raft::StateMachine> sm, std::shared_ptr<TlsContext> peer_tls)
    : sm_(std::move(sm)), peers_(std::make_unique<GrpcChannelPool>(1500, std::move(peer_tls))) {}

std::vector<std::string> NativeRaftHost::apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) {
  return sm_->apply(cmds);
}
std::string NativeRaftHost::snapshot() { return sm_->snapshot(); }
void NativeRaftHost::restore(const std::string& state) { sm_->restore(state); }

namespace {
std::string base_url(const std::string& addr) {
  std::string a = addr;
  while (!a.empty() && a.back() == '/') a.pop_back();
  return with_scheme(a);
}
}  // namespace

bool NativeRaftHost::send(const std::string& addr, const std::string& kind, const std::string& body,
                          std::string* reply) {
  std::string ep;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (blocked_.count(base_url(addr))) return false;
    auto it = endpoints_.find(addr);
    if (it != endpoints_.end()) ep = it->second;
  }
  if (!ep.empty()) {
    GrpcResult r = peers_->call(ep, "/dfs.RaftPeer/" + kind, body, "", kind == "snapshot" ? 30000 : 1500);
    if (!r.transport_ok || r.status != 0) return false;
    *reply = std::move(r.message);
    return true;
  }
  // HTTP/JSON peer (a node without a native endpoint): 3 tries / 50 ms x2 for vote and
  // snapshot, 2 tries / 20 ms for append, one for timeout_now
  int tries = 1, backoff_ms = 0;
  if (kind == "vote" || kind == "snapshot") tries = 3, backoff_ms = 50;
  else if (kind == "append") tries = 2, backoff_ms = 20;
  const std::string url = base_url(addr) + "/raft/" + kind;
  for (int a = 0; a < tries; ++a) {
    if (http_request("POST", url, body, "application/json", kind == "snapshot" ? 30000 : 1500, reply) == 200)
      return true;
    if (a + 1 < tries) std::this_thread::sleep_for(std::chrono::milliseconds(backoff_ms << a));
  }
  return false;
}

void NativeRaftHost::backup(const std::string& url, const std::string& data) {
  std::thread([url, data] {
    std::string err;
    int st = http_request("PUT", url, data, "application/octet-stream", 30000, nullptr, &err);
    if (st < 200 || st >= 300) log(kWarning, "dfs.raft", "snapshot backup to %s failed: %s", url.c_str(),
                                   err.empty() ? std::to_string(st).c_str() : err.c_str());
  }).detach();
}

void NativeRaftHost::set_peer_endpoint(const std::string& addr, const std::string& endpoint) {
  std::lock_guard<std::mutex> g(mu_);
  if (endpoint.empty()) endpoints_.erase(addr);
  else endpoints_[addr] = endpoint;
}

void NativeRaftHost::set_blocked(const std::vector<std::string>& addrs) {
  std::lock_guard<std::mutex> g(mu_);
  blocked_.clear();
  for (auto& a : addrs) blocked_.insert(base_url(a));
}

std::vector<std::string> NativeRaftHost::blocked() const {
  std::lock_guard<std::mutex> g(mu_);
  return {blocked_.begin(), blocked_.end()};
}

bool NativeRaftHost::has_endpoint(const std::string& addr) const {
  std::lock_guard<std::mutex> g(mu_);
  return endpoints_.count(addr) != 0;
}

void resolve_peers_loop(raft::Node& node, NativeRaftHost& host, const std::atomic<bool>& stop) {
  std::set<std::string> asked;
  while (!stop) {
    for (auto& [id, addr] : node.config().all()) {
      if (id == node.id() || asked.count(addr)) continue;
      std::string body;
      if (http_request("GET", base_url(addr) + "/raft/endpoint", "", "", 2000, &body) != 200) continue;
      asked.insert(addr);
      try {
        std::string ep = Json::parse(body)["grpc"].str();
        if (!ep.empty()) host.set_peer_endpoint(addr, ep);
      } catch (...) {
      }
    }
    for (int i = 0; i < 10 && !stop; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
}

HttpResponse json_response(const std::string& body, int status) {
  HttpResponse r;
  r.status = status;
  r.content_type = "application/json";
  r.body = body;
  return r;
}

HttpResponse raft_http(raft::Node& node, const HttpRequest& req) {
  static const std::set<std::string> kinds = {"vote", "append", "snapshot", "timeout_now"};
  std::string kind = req.path.substr(std::string("/raft/").size());
  if (req.method != "POST" || !kinds.count(kind)) return HttpResponse{404, "text/plain", "Not Found"};
  try {
    return json_response(node.handle(kind, req.body));
  } catch (...) {
    return HttpResponse{500, "text/plain", "Internal server error"};
  }
}

void Gauges::add(const std::string& name, const std::string& help, std::function<double()> fn) {
  gs_.push_back(G{name, help, std::move(fn)});
}

std::string Gauges::render() const {
  std::string out;
  char num[64];
  for (auto& g : gs_) {
    double v = 0;
    try {
      v = g.fn();
    } catch (...) {
    }
    std::snprintf(num, sizeof(num), "%.17g", v);
    out += "# HELP " + g.name + " " + g.help + "\n# TYPE " + g.name + " gauge\n" + g.name + " " + num + "\n";
  }
  return out;
}

namespace {
// A fatal signal's backtrace on stderr (async-signal-safe: backtrace + backtrace_symbols_fd
// write straight to the fd), then the default action, so the exit status still says which.
void on_fatal(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  // no snprintf / strsignal here (not async-signal-safe): the number, written by hand
  char head[48] = "FATAL signal ";
  size_t len = std::strlen(head);
  if (sig >= 10) head[len++] = static_cast<char>('0' + sig / 10);
  head[len++] = static_cast<char>('0' + sig % 10);
  const char tail[] = "; backtrace:\n";
  std::memcpy(head + len, tail, sizeof(tail) - 1);
  len += sizeof(tail) - 1;
  (void)!::write(2, head, len);
  backtrace_symbols_fd(frames, n, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}
}  // namespace

void install_crash_handler() {
  void* warm[1];
  (void)backtrace(warm, 1);  // loads libgcc's unwinder now, not inside the handler
  for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT}) ::signal(sig, on_fatal);
}

void block_stop_signals() {
  install_crash_handler();
  trace_init();  // before any thread: roctx's first range calls setenv (trace.h)
  sigset_t s;
  sigemptyset(&s);
  sigaddset(&s, SIGTERM);
  sigaddset(&s, SIGINT);
  pthread_sigmask(SIG_BLOCK, &s, nullptr);
  signal(SIGPIPE, SIG_IGN);
}

void wait_for_stop() {
  sigset_t s;
  sigemptyset(&s);
  sigaddset(&s, SIGTERM);
  sigaddset(&s, SIGINT);
  int sig = 0;
  while (sigwait(&s, &sig) != 0) {
  }
}

void write_ready_file(const std::string& json) {
  std::string path = env("DFS_READY_FILE");
  if (path.empty()) return;
  std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp);
    f << json;
  }
  std::rename(tmp.c_str(), path.c_str());
}

namespace {
int log_threshold() {
  static const int t = [] {
    std::string v = env("DFS_LOG", "warning");
    for (auto& c : v) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    if (v == "debug") return static_cast<int>(kDebug);
    if (v == "info") return static_cast<int>(kInfo);
    if (v == "error") return static_cast<int>(kError);
    return static_cast<int>(kWarning);
  }();
  return t;
}
}  // namespace

void log(int level, const char* name, const char* fmt, ...) {
  if (level < log_threshold()) return;
  char msg[2048];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  timeval tv;
  gettimeofday(&tv, nullptr);
  tm t;
  localtime_r(&tv.tv_sec, &t);
  char ts[64];
  std::strftime(ts, sizeof(ts), "%Y-%m-%d %H:%M:%S", &t);
  const char* lv = level >= kError ? "ERROR" : level >= kWarning ? "WARNING" : level >= kInfo ? "INFO" : "DEBUG";
  std::fprintf(stderr, "%s,%03d %s %s [req=-] %s\n", ts, static_cast<int>(tv.tv_usec / 1000), lv, name, msg);
}

}  // namespace dfs::shell
