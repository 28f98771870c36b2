// roctx ranges around the data-path phases (kernels, RCCL sends and the
// phases around them visible in one rocprofv3 timeline). `rocprofv3 --marker-trace
// --kernel-trace -- <program>` records them next to the kernels; without a tool attached
// a range costs one call into the roctx stub.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace dfs {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace dfs
