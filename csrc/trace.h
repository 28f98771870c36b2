// roctx ranges around the data-path phases (kernels, RCCL sends and the
// phases around them visible in one rocprofv3 timeline). `rocprofv3 --marker-trace
// --kernel-trace -- <program>` records them next to the kernels; without a tool attached
// a range costs one call into the roctx stub.
//
// Request ids (reference dfs/common/src/lib.rs:8-50, x-request-id): the native data path
// carries the client's request id on every hop (local RPC, fast-path ops, replication
// descriptors); RequestScope makes it current for the thread, and every TraceRange opened
// under it is named "<phase> [rid]" so a rocprofv3 marker trace correlates kernels, RCCL
// transfers and fsyncs with the client request that caused them.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>

namespace dfs {

inline thread_local std::string t_request_id;

class RequestScope {
 public:
  explicit RequestScope(const std::string& rid) : saved_(t_request_id) {
    if (!rid.empty()) t_request_id = rid;
  }
  ~RequestScope() { t_request_id = saved_; }
  RequestScope(const RequestScope&) = delete;
  RequestScope& operator=(const RequestScope&) = delete;

 private:
  std::string saved_;
};

// roctx (and rocprofiler-register under it) calls setenv() while it initializes, on the
// first range. glibc's getenv() is not safe against a concurrent setenv(): a chunkserver's
// first ranges come from its worker threads while main still reads its environment, and one
// CPU test run died with SIGSEGV inside getenv at startup. Every process therefore starts
// roctx from main before it starts a thread (shell::block_stop_signals, the Python module).
inline void trace_init() {
  roctxRangePushA("dfs.init");
  roctxRangePop();
}

class TraceRange {
 public:
  explicit TraceRange(const char* name) {
    if (t_request_id.empty()) {
      roctxRangePushA(name);
    } else {
      std::string n = std::string(name) + " [" + t_request_id + "]";
      roctxRangePushA(n.c_str());
    }
  }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace dfs
