// JSON key lists of the chunkserver components' statistics (cs_stats.cpp), shared by the
// Python bindings and the native dfs_chunkserver's /stats.
#pragma once
#include <string>

#include "json.h"

namespace dfs {

struct StoreStats;
struct CsAgentStats;
struct FpStats;
struct ReplStats;
struct CsGrpcStats;

Json stats_json(const StoreStats& t);
Json stats_json(const CsAgentStats& t);
Json stats_json(const FpStats& t);
Json stats_json(const ReplStats& t);  // replication engine (unprefixed; /stats prefixes "repl_")
Json stats_json(const CsGrpcStats& t, uint64_t calls);
// every field of `src` into `dst`, names prefixed
void merge_into(Json* dst, const Json& src, const std::string& prefix = "");

}  // namespace dfs
