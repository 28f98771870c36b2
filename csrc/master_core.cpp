#include "master_core.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <future>
#include <memory>

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

const char* kSafeModeMsg = "Cluster is in Safe Mode. Write operations are blocked.";
constexpr uint64_t kScheduleQuantum = 64ull << 20;
constexpr size_t kReplication = 3;

int64_t create_lease_ms() {
  static const int64_t v = [] {
    const char* e = std::getenv("DFS_CREATE_LEASE_MS");
    return e ? std::atoll(e) : 60000;
  }();
  return v;
}

// ---- serde layout of FileMetadata / BlockInfo (reference build.rs serde derives; models/meta.py)
Json block_json(const pb::BlockInfo& b) {
  Json d = Json::object();
  d.set("block_id", b.block_id);
  d.set("size", b.size);
  d.set("checksum_crc32c", b.checksum_crc32c);
  d.set("ec_data_shards", b.ec_data_shards);
  d.set("ec_parity_shards", b.ec_parity_shards);
  d.set("original_size", b.original_size);
  Json l = Json::array();
  for (auto& x : b.locations) l.push_back(x);
  d.set("locations", l);
  return d;
}

pb::BlockInfo block_from(const Json& d) {
  pb::BlockInfo b;
  b.block_id = d["block_id"].str();
  b.size = d["size"].as_u64();
  b.checksum_crc32c = static_cast<uint32_t>(d["checksum_crc32c"].as_u64());
  b.ec_data_shards = static_cast<int32_t>(d["ec_data_shards"].as_int());
  b.ec_parity_shards = static_cast<int32_t>(d["ec_parity_shards"].as_int());
  b.original_size = d["original_size"].as_u64();
  for (auto& x : d["locations"].items()) b.locations.push_back(x.str());
  return b;
}

Json attrs_json(const std::map<std::string, std::string>& a) {
  Json o = Json::object();
  for (auto& kv : a) o.set(kv.first, kv.second);
  return o;
}

void attrs_from(const Json& j, std::map<std::string, std::string>* out) {
  if (!j.is_object()) return;
  out->clear();
  for (auto& kv : j.fields()) (*out)[kv.first] = kv.second.str();
}

Json file_json(const pb::FileMetadata& m) {
  Json d = Json::object();
  d.set("path", m.path);
  d.set("size", m.size);
  d.set("etag_md5", m.etag_md5);
  d.set("created_at_ms", m.created_at_ms);
  d.set("ec_data_shards", m.ec_data_shards);
  d.set("ec_parity_shards", m.ec_parity_shards);
  d.set("last_access_ms", m.last_access_ms);
  d.set("access_count", m.access_count);
  d.set("moved_to_cold_at_ms", m.moved_to_cold_at_ms);
  Json bl = Json::array();
  for (auto& b : m.blocks) bl.push_back(block_json(b));
  d.set("blocks", bl);
  if (!m.attributes.empty()) d.set("attributes", attrs_json(m.attributes));  // absent: reference layout
  return d;
}

pb::FileMetadata file_from(const Json& d) {
  pb::FileMetadata m;
  m.path = d["path"].str();
  m.size = d["size"].as_u64();
  m.etag_md5 = d["etag_md5"].str();
  m.created_at_ms = d["created_at_ms"].as_u64();
  m.ec_data_shards = static_cast<int32_t>(d["ec_data_shards"].as_int());
  m.ec_parity_shards = static_cast<int32_t>(d["ec_parity_shards"].as_int());
  m.last_access_ms = d["last_access_ms"].as_u64();
  m.access_count = d["access_count"].as_u64();
  m.moved_to_cold_at_ms = d["moved_to_cold_at_ms"].as_u64();
  for (auto& b : d["blocks"].items()) m.blocks.push_back(block_from(b));
  attrs_from(d["attributes"], &m.attributes);
  return m;
}

Json block_list(const pb::FileMetadata& m) {  // [[block_id, [locations]], ...]
  Json out = Json::array();
  for (auto& b : m.blocks) {
    Json locs = Json::array();
    for (auto& l : b.locations) locs.push_back(l);
    out.push_back(Json(Json::Array{Json(b.block_id), locs}));
  }
  return out;
}

Json obj(std::initializer_list<std::pair<const char*, Json>> kv) {
  Json o = Json::object();
  for (auto& p : kv) o.set(p.first, p.second);
  return o;
}

std::string prefix_of(const std::string& path) {
  size_t i = 0;
  while (i < path.size() && path[i] == '/') ++i;
  if (i == path.size()) return "/";
  size_t j = path.find('/', i);
  return "/" + path.substr(i, j == std::string::npos ? std::string::npos : j - i) + "/";
}

std::string locked_path(const Json& rec) {
  const Json& ren = rec["tx_type"]["Rename"];
  const std::string& st = rec["state"].as_string();
  if (ren.is_null() || st == "Committed" || st == "Aborted") return "";
  const std::string& src = ren["source_path"].as_string();
  return src.empty() ? ren["dest_path"].str() : src;
}

}  // namespace

Json file_meta_json(const pb::FileMetadata& m) { return file_json(m); }
Json block_info_json(const pb::BlockInfo& b) { return block_json(b); }

// ---------------------------------------------------------------- placement
std::vector<std::string> select_servers_rack_aware(const std::vector<ChunkServerStatus>& servers, size_t n,
                                                   const std::string& preferred) {
  std::vector<std::string> selected;
  if (n == 0 || servers.empty()) return selected;
  // free space net of blocks scheduled since the last heartbeat (HDFS-style), so a burst of
  // allocations rotates over equally-free servers instead of piling onto the same ones
  std::vector<const ChunkServerStatus*> cands;
  for (auto& s : servers) cands.push_back(&s);
  auto net = [](const ChunkServerStatus* s) {
    return static_cast<int64_t>(s->available_space) - static_cast<int64_t>(s->scheduled);
  };
  std::sort(cands.begin(), cands.end(), [&](const ChunkServerStatus* a, const ChunkServerStatus* b) {
    int64_t na = net(a), nb = net(b);
    return na != nb ? na > nb : a->address < b->address;
  });
  std::string pref_rack;
  if (!preferred.empty()) {
    auto it = std::find_if(cands.begin(), cands.end(), [&](auto* s) { return s->address == preferred; });
    if (it != cands.end()) {
      selected.push_back(preferred);
      pref_rack = (*it)->rack_id;
      cands.erase(it);
    }
  }
  std::vector<std::string> order;
  std::map<std::string, std::vector<const ChunkServerStatus*>> buckets;
  for (auto* s : cands) {
    std::string key = s->rack_id.empty() ? "__addr__" + s->address : s->rack_id;
    if (!buckets.count(key)) order.push_back(key);
    buckets[key].push_back(s);
  }
  // the writer's rack goes last so the next replicas spread to other racks first
  if (!selected.empty() && !pref_rack.empty() && buckets.count(pref_rack)) {
    order.erase(std::find(order.begin(), order.end(), pref_rack));
    order.push_back(pref_rack);
  }
  std::vector<size_t> pos(order.size(), 0);
  while (selected.size() < n) {
    bool picked = false;
    for (size_t i = 0; i < order.size() && selected.size() < n; ++i) {
      auto& rack = buckets[order[i]];
      if (pos[i] < rack.size()) {
        selected.push_back(rack[pos[i]++]->address);
        picked = true;
      }
    }
    if (!picked) break;
  }
  selected.resize(std::min(selected.size(), n));
  return selected;
}

// ---------------------------------------------------------------- lifecycle
MasterCore::MasterCore() : rng_(std::random_device{}()) {
  access_thread_ = std::thread([this] { access_loop(); });
}

MasterCore::~MasterCore() {
  running_ = false;
  access_cv_.notify_all();
  if (access_thread_.joinable()) access_thread_.join();
}

void MasterCore::attach(raft::Node* node) { node_ = node; }
void MasterCore::detach() { node_ = nullptr; }

void MasterCore::set_access_stats(bool on, int flush_ms) {
  std::lock_guard<std::mutex> g(mu_);
  access_stats_ = on;
  access_flush_ms_ = flush_ms;
}

void MasterCore::set_shard_map(const std::string& json, const std::string& shard_id) {
  ShardMap m = json.empty() ? ShardMap::new_range() : ShardMap::from_json(Json::parse(json));
  std::lock_guard<std::mutex> g(mu_);
  shard_map_ = std::move(m);
  shard_id_ = shard_id;
  have_map_ = !json.empty();
}

static int64_t steady_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void MasterCore::note_shard_map_fresh() {
  std::lock_guard<std::mutex> g(mu_);
  map_fresh_ms_ = steady_ms();
}

void MasterCore::set_shard_map_max_age(int64_t ms) {
  std::lock_guard<std::mutex> g(mu_);
  map_max_age_ms_ = ms;
}

// ---------------------------------------------------------------- state machine
void MasterCore::put(const std::string& path, pb::FileMetadata m) {
  auto it = files_.find(path);
  if (it != files_.end())
    for (auto& b : it->second.blocks) {
      auto bi = block_index_.find(b.block_id);
      if (bi != block_index_.end() && bi->second == path) block_index_.erase(bi);
    }
  for (auto& b : m.blocks) block_index_[b.block_id] = path;
  files_[path] = std::move(m);
  ordered_.insert(path);
}

bool MasterCore::del(const std::string& path, pb::FileMetadata* out) {
  under_construction_.erase(path);
  uc_progress_.erase(path);
  auto it = files_.find(path);
  if (it == files_.end()) return false;
  for (auto& b : it->second.blocks) {
    auto bi = block_index_.find(b.block_id);
    if (bi != block_index_.end() && bi->second == path) block_index_.erase(bi);
  }
  if (out) *out = std::move(it->second);
  files_.erase(it);
  ordered_.erase(path);
  return true;
}

const pb::FileMetadata* MasterCore::visible(const std::string& path) const {
  if (under_construction_.count(path)) return nullptr;
  auto it = files_.find(path);
  return it == files_.end() ? nullptr : &it->second;
}

pb::BlockInfo* MasterCore::find_block_locked(const std::string& block_id, pb::FileMetadata** file) {
  auto bi = block_index_.find(block_id);
  if (bi == block_index_.end()) return nullptr;
  auto it = files_.find(bi->second);
  if (it == files_.end()) return nullptr;
  for (auto& b : it->second.blocks)
    if (b.block_id == block_id) {
      if (file) *file = &it->second;
      return &b;
    }
  return nullptr;
}

void MasterCore::relock(const Json& rec) {
  const std::string id = rec["tx_id"].str();
  for (auto it = tx_locks_.begin(); it != tx_locks_.end();) it = it->second == id ? tx_locks_.erase(it) : std::next(it);
  std::string p = locked_path(rec);
  if (!p.empty()) tx_locks_[p] = id;
}

std::vector<std::string> MasterCore::apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) {
  std::vector<std::string> out;
  out.reserve(cmds.size());
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& c : cmds) {
      try {
        Json j = Json::parse(c.second);
        const Json* m = j.find("Master");
        if (!m || m->fields().empty()) {
          out.push_back("null");
          continue;
        }
        auto& kv = m->fields().front();
        out.push_back(apply_one(kv.first, kv.second).dump());
      } catch (const std::exception& e) {
        out.push_back(std::string("!") + e.what());
      }
    }
  }
  applied_cv_.notify_all();
  return out;
}

Json MasterCore::apply_one(const std::string& name, const Json& a) {
  const std::string path = a["path"].str();
  if (name == "CreateFile" || name == "CreateComplete") {
    // existence is decided here, in log order: two racing creates cannot both succeed
    if (tx_locks_.count(path)) return obj({{"locked", path}});
    int64_t ts = a["ts"].as_int();
    pb::FileMetadata old;
    bool had_old = false;
    auto it = files_.find(path);
    if (it != files_.end()) {
      auto uc = under_construction_.find(path);
      if (uc == under_construction_.end()) return obj({{"exists", true}});
      auto pr = uc_progress_.find(path);
      int64_t last = pr == uc_progress_.end() ? uc->second : std::max(uc->second, pr->second);
      if (ts - last < create_lease_ms()) return obj({{"exists", true}});
      // a writer that made no progress (create / AllocateBlock) for a whole lease: take the
      // path over; its later AllocateBlock / CompleteFile carry the old generation and fail
      old = it->second;
      had_old = true;
    }
    pb::FileMetadata m;
    m.path = path;
    m.ec_data_shards = static_cast<int32_t>(a["ec_data_shards"].as_int());
    m.ec_parity_shards = static_cast<int32_t>(a["ec_parity_shards"].as_int());
    if (name == "CreateFile") {
      if (!a["block_id"].str().empty()) {
        pb::BlockInfo b;
        b.block_id = a["block_id"].str();
        b.ec_data_shards = m.ec_data_shards;
        b.ec_parity_shards = m.ec_parity_shards;
        for (auto& l : a["locations"].items()) b.locations.push_back(l.str());
        m.blocks.push_back(std::move(b));
      }
      put(path, std::move(m));
      under_construction_[path] = ts;
      uc_progress_[path] = ts;
    } else {
      for (auto& bd : a["blocks"].items()) m.blocks.push_back(block_from(bd));
      put(path, std::move(m));
      under_construction_.erase(path);
      uc_progress_.erase(path);
      apply_one("CompleteFile", a);
    }
    return obj({{"exists", false}, {"gen", ts}, {"orphans", had_old ? block_list(old) : Json::array()}});
  }
  if (name == "CompleteFile") {
    auto it = files_.find(path);
    if (it == files_.end()) return obj({{"found", false}});
    pb::FileMetadata& m = it->second;
    if (int64_t gen = a["gen"].as_int()) {
      auto uc = under_construction_.find(path);
      if (uc == under_construction_.end()) {
        // already complete: only an identical retry of the completion is accepted
        bool same = m.size == a["size"].as_u64() && (a["etag_md5"].str().empty() || m.etag_md5 == a["etag_md5"].str());
        if (!same) return obj({{"found", true}, {"stale", true}});
        return obj({{"found", true}});
      }
      if (uc->second != gen) return obj({{"found", true}, {"stale", true}});
    }
    under_construction_.erase(path);
    uc_progress_.erase(path);
    m.size = a["size"].as_u64();
    if (!a["etag_md5"].str().empty()) m.etag_md5 = a["etag_md5"].str();
    if (a["created_at_ms"].as_u64()) m.created_at_ms = a["created_at_ms"].as_u64();
    attrs_from(a["attributes"], &m.attributes);
    const Json& sums = a["block_checksums"];
    if (sums.size()) {
      for (auto& s : sums.items())
        for (auto& b : m.blocks)
          if (b.block_id == s["block_id"].as_string()) {
            b.checksum_crc32c = static_cast<uint32_t>(s["checksum_crc32c"].as_u64());
            b.size = s["actual_size"].as_u64();
            b.original_size = b.size;
          }
    } else if (!m.blocks.empty()) {
      uint64_t n = m.blocks.size(), per = m.size / n;
      for (size_t i = 0; i + 1 < n; ++i) m.blocks[i].size = per;
      m.blocks.back().size = m.size - per * (n - 1);
    }
    return obj({{"found", true}});
  }
  if (name == "DeleteFile") {
    if (tx_locks_.count(path)) return obj({{"locked", path}});
    if (!visible(path)) return obj({{"found", false}});
    pb::FileMetadata m;
    del(path, &m);
    return obj({{"found", true}, {"blocks", block_list(m)}});
  }
  if (name == "AllocateBlock") {
    auto it = files_.find(path);
    if (it == files_.end()) return Json();
    auto uc = under_construction_.find(path);
    if (int64_t gen = a["gen"].as_int())
      if (uc == under_construction_.end() || uc->second != gen) return obj({{"stale", true}});
    if (uc != under_construction_.end()) {  // progress renews the writer's lease
      int64_t& last = uc_progress_[path];
      last = std::max(last, a["ts"].as_int());
    }
    pb::BlockInfo b;
    b.block_id = a["block_id"].str();
    b.ec_data_shards = it->second.ec_data_shards;
    b.ec_parity_shards = it->second.ec_parity_shards;
    for (auto& l : a["locations"].items()) b.locations.push_back(l.str());
    block_index_[b.block_id] = path;
    it->second.blocks.push_back(std::move(b));
    return Json();
  }
  if (name == "RenameFile") {
    // decided in log order: the source must be complete, the destination must not exist
    std::string src = a["source_path"].str(), dst = a["dest_path"].str();
    for (auto* p : {&src, &dst})
      if (tx_locks_.count(*p)) return obj({{"locked", *p}});
    if (!visible(src)) return obj({{"error", "Source file not found: " + src}});
    if (files_.count(dst)) return obj({{"error", "Destination file already exists: " + dst}});
    pb::FileMetadata m;
    del(src, &m);
    m.path = dst;
    put(dst, std::move(m));
    return obj({{"error", Json()}});
  }
  if (name == "CreateTransactionRecord") {
    const Json& rec = a["record"];
    std::string id = rec["tx_id"].str();
    if (tx_records_.count(id)) return obj({{"conflict", Json()}});
    std::string p = locked_path(rec);
    const Json& ren = rec["tx_type"]["Rename"];
    if (!ren.is_null() && !p.empty()) {
      auto lk = tx_locks_.find(p);
      if (lk != tx_locks_.end() && lk->second != id) return obj({{"conflict", p + " is locked by another transaction"}});
      if (!ren["source_path"].str().empty()) {
        if (!visible(p)) return obj({{"conflict", "Source file not found: " + p}});
      } else if (files_.count(p)) {
        return obj({{"conflict", "Destination file already exists: " + p}});
      }
    }
    tx_records_[id] = rec;
    relock(rec);
    return obj({{"conflict", Json()}});
  }
  if (name == "UpdateTransactionState") {
    auto it = tx_records_.find(a["tx_id"].str());
    if (it != tx_records_.end()) {
      it->second.set("state", a["new_state"]);
      relock(it->second);
    }
    return Json();
  }
  if (name == "ApplyTransactionOperation") {
    const Json& op = a["operation"]["op_type"];
    if (const Json* d = op.find("Delete")) {
      del((*d)["path"].str(), nullptr);
    } else if (const Json* c = op.find("Create")) {
      std::string p = (*c)["path"].str();
      if (!files_.count(p)) {
        pb::FileMetadata m = file_from((*c)["metadata"]);
        m.path = p;
        put(p, std::move(m));
      }
    }
    return Json();
  }
  if (name == "DeleteTransactionRecord") {
    auto it = tx_records_.find(a["tx_id"].str());
    if (it != tx_records_.end()) {
      Json rec = it->second;
      tx_records_.erase(it);
      rec.set("state", "Aborted");
      relock(rec);
    }
    return Json();
  }
  if (name == "SplitShard") {
    if (const Json* ps = a.find("paths")) {  // explicit list: the files the post-split map routes away
      for (auto& p : ps->items()) del(p.str(), nullptr);
      return Json();
    }
    std::string key = a["split_key"].str();
    std::vector<std::string> moving;
    for (auto& kv : files_)
      if (kv.first >= key) moving.push_back(kv.first);
    for (auto& p : moving) del(p, nullptr);
    return Json();
  }
  if (name == "IngestBatch") {
    for (auto& f : a["files"].items()) {
      pb::FileMetadata m = file_from(f);
      std::string p = m.path;
      put(p, std::move(m));
    }
    return Json();
  }
  if (name == "TriggerShuffle") {
    shuffling_prefixes_.insert(a["prefix"].str());
    return Json();
  }
  if (name == "StopShuffle") {
    shuffling_prefixes_.erase(a["prefix"].str());
    return Json();
  }
  if (name == "UpdateAccessStats") {
    auto it = files_.find(path);
    if (it != files_.end()) {
      it->second.last_access_ms = a["accessed_at_ms"].as_u64();
      it->second.access_count++;
    }
    return Json();
  }
  if (name == "UpdateAccessStatsBatch") {
    uint64_t t = a["accessed_at_ms"].as_u64();
    for (auto& kv : a["paths"].fields()) {
      auto it = files_.find(kv.first);
      if (it != files_.end()) {
        it->second.last_access_ms = t;
        it->second.access_count += kv.second.as_u64();
      }
    }
    return Json();
  }
  if (name == "MoveToCold") {
    auto it = files_.find(path);
    if (it != files_.end()) it->second.moved_to_cold_at_ms = a["moved_at_ms"].as_u64();
    return Json();
  }
  if (name == "ConvertToEc") {
    auto it = files_.find(path);
    if (it == files_.end()) return Json();
    pb::FileMetadata& m = it->second;
    for (auto& b : m.blocks) block_index_.erase(b.block_id);
    m.ec_data_shards = static_cast<int32_t>(a["ec_data_shards"].as_int());
    m.ec_parity_shards = static_cast<int32_t>(a["ec_parity_shards"].as_int());
    m.blocks.clear();
    for (auto& bd : a["new_blocks"].items()) m.blocks.push_back(block_from(bd));
    for (auto& b : m.blocks) block_index_[b.block_id] = m.path;
    return Json();
  }
  if (name == "SetParticipantAcked" || name == "IncrementInquiryCount") {
    auto it = tx_records_.find(a["tx_id"].str());
    if (it != tx_records_.end()) {
      if (name == "SetParticipantAcked") it->second.set("participant_acked", true);
      else it->second.set("inquiry_count", it->second["inquiry_count"].as_int() + 1);
    }
    return Json();
  }
  if (name == "AddBlockLocation") {
    pb::BlockInfo* b = find_block_locked(a["block_id"].str(), nullptr);
    if (!b) return Json();
    std::string addr = a["address"].str();
    const Json& idx = a["shard_index"];
    if (!idx.is_null() && b->ec_data_shards > 0) {
      // EC locations are positional (shard i lives at locations[i]): a rebuilt shard
      // replaces its dead holder instead of being appended
      int64_t i = idx.as_int();
      if (i >= 0 && static_cast<size_t>(i) < b->locations.size()) b->locations[i] = addr;
      return Json();
    }
    if (std::find(b->locations.begin(), b->locations.end(), addr) == b->locations.end()) b->locations.push_back(addr);
    return Json();
  }
  if (name == "UpdateBlockLocations") {
    pb::BlockInfo* b = find_block_locked(a["block_id"].str(), nullptr);
    if (b) {
      b->locations.clear();
      for (auto& l : a["locations"].items()) b->locations.push_back(l.str());
    }
    return Json();
  }
  if (name == "MergeShard" || name == "RegisterChunkServer") return Json();
  std::fprintf(stderr, "master: unknown command %s\n", name.c_str());
  return Json();
}

// The replicated state is copied under the lock and serialized outside it, so a compaction
// of a large namespace holds the handlers up for the copy, not for the JSON text.
std::string MasterCore::snapshot() {
  std::vector<std::pair<std::string, pb::FileMetadata>> files;
  Json tx = Json::object(), sp = Json::array(), uc = Json::object(), up = Json::object();
  {
    std::lock_guard<std::mutex> g(mu_);
    files.assign(files_.begin(), files_.end());
    for (auto& kv : tx_records_) tx.set(kv.first, kv.second);
    for (auto& p : shuffling_prefixes_) sp.push_back(p);
    for (auto& kv : under_construction_) uc.set(kv.first, kv.second);
    for (auto& kv : uc_progress_) up.set(kv.first, kv.second);
  }
  std::sort(files.begin(), files.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::string out = "{\"Master\":{\"files\":{";
  bool first = true;
  for (auto& kv : files) {
    if (!first) out += ",";
    first = false;
    json_escape(kv.first, out);
    out += ":";
    file_json(kv.second).dump_to(out);
  }
  out += "},\"transaction_records\":";
  tx.dump_to(out);
  out += ",\"shuffling_prefixes\":";
  sp.dump_to(out);
  out += ",\"under_construction\":";
  uc.dump_to(out);
  out += ",\"uc_progress\":";
  up.dump_to(out);
  out += "}}";
  return out;
}

void MasterCore::restore(const std::string& text) {
  Json j = Json::parse(text);
  const Json* st = j.find("Master");
  const Json& s = st ? *st : j;  // a legacy raw MasterState is accepted too
  std::lock_guard<std::mutex> g(mu_);
  files_.clear();
  ordered_.clear();
  block_index_.clear();
  for (auto& kv : s["files"].fields()) put(kv.first, file_from(kv.second));
  tx_records_.clear();
  tx_locks_.clear();
  for (auto& kv : s["transaction_records"].fields()) {
    tx_records_[kv.first] = kv.second;
    relock(kv.second);
  }
  shuffling_prefixes_.clear();
  for (auto& p : s["shuffling_prefixes"].items()) shuffling_prefixes_.insert(p.str());
  under_construction_.clear();
  uc_progress_.clear();
  for (auto& kv : s["under_construction"].fields())
    if (files_.count(kv.first)) under_construction_[kv.first] = uc_progress_[kv.first] = kv.second.as_int();
  for (auto& kv : s["uc_progress"].fields())
    if (under_construction_.count(kv.first)) uc_progress_[kv.first] = kv.second.as_int();
}

// ---------------------------------------------------------------- chunkservers / safe mode
void MasterCore::upsert_chunk_server(const ChunkServerStatus& st) {
  std::lock_guard<std::mutex> g(mu_);
  chunk_servers_[st.address] = st;
}

bool MasterCore::remove_chunk_server(const std::string& addr) {
  std::lock_guard<std::mutex> g(mu_);
  return chunk_servers_.erase(addr) != 0;
}

std::vector<ChunkServerStatus> MasterCore::chunk_servers() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<ChunkServerStatus> out;
  for (auto& kv : chunk_servers_) out.push_back(kv.second);
  return out;
}

void MasterCore::enter_safe_mode(bool manual) {
  std::lock_guard<std::mutex> g(mu_);
  safe_mode_ = true;
  safe_mode_entered_at_ = now_ms();
  safe_mode_threshold_ = 0.99;
  uint64_t n = 0;
  for (auto& kv : files_) n += kv.second.blocks.size();
  expected_blocks_ = n;
  reported_blocks_ = 0;
  safe_mode_manual_ = manual;
}

void MasterCore::exit_safe_mode() {
  std::lock_guard<std::mutex> g(mu_);
  safe_mode_ = false;
  safe_mode_manual_ = false;
}

bool MasterCore::should_exit_safe_mode() const {
  std::lock_guard<std::mutex> g(mu_);
  if (safe_mode_manual_ || !safe_mode_ || chunk_servers_.empty()) return false;
  if (expected_blocks_ == 0) return true;
  if (static_cast<double>(reported_blocks_) / static_cast<double>(expected_blocks_) >= safe_mode_threshold_) return true;
  return now_ms() - safe_mode_entered_at_ > 60000;
}

void MasterCore::report_blocks(uint64_t n) {
  {
    std::lock_guard<std::mutex> g(mu_);
    reported_blocks_ += n;
  }
  if (should_exit_safe_mode()) exit_safe_mode();
}

Json MasterCore::safe_mode_status() const {
  std::lock_guard<std::mutex> g(mu_);
  return obj({{"is_safe_mode", safe_mode_},
              {"is_manual", safe_mode_manual_},
              {"chunk_server_count", static_cast<uint64_t>(chunk_servers_.size())},
              {"expected_blocks", expected_blocks_},
              {"reported_blocks", reported_blocks_},
              {"threshold", safe_mode_threshold_},
              {"entered_at", safe_mode_entered_at_}});
}

// ---------------------------------------------------------------- queries
bool MasterCore::get_file(const std::string& path, bool visible_only, std::string* out) const {
  std::lock_guard<std::mutex> g(mu_);
  const pb::FileMetadata* m = nullptr;
  if (visible_only) {
    m = visible(path);
  } else {
    auto it = files_.find(path);
    if (it != files_.end()) m = &it->second;
  }
  if (!m) return false;
  m->encode(*out);
  return true;
}

bool MasterCore::contains(const std::string& path) const {
  std::lock_guard<std::mutex> g(mu_);
  return files_.count(path) != 0;
}

bool MasterCore::under_construction(const std::string& path) const {
  std::lock_guard<std::mutex> g(mu_);
  return under_construction_.count(path) != 0;
}

size_t MasterCore::file_count() const {
  std::lock_guard<std::mutex> g(mu_);
  return files_.size();
}

std::vector<std::string> MasterCore::paths(const std::string& prefix, bool visible_only) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for_prefix(prefix, [&](const std::string& p) {
    if (!visible_only || !under_construction_.count(p)) out.push_back(p);
  });
  return out;
}

std::vector<std::string> MasterCore::files_pb(const std::string& prefix) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for_prefix(prefix, [&](const std::string& p) { out.push_back(files_.at(p).str()); });
  return out;
}

bool MasterCore::find_block(const std::string& block_id, std::string* file_pb) const {
  std::lock_guard<std::mutex> g(mu_);
  auto bi = block_index_.find(block_id);
  if (bi == block_index_.end()) return false;
  auto it = files_.find(bi->second);
  if (it == files_.end()) return false;
  it->second.encode(*file_pb);
  return true;
}

bool MasterCore::has_block(const std::string& block_id) const {
  std::lock_guard<std::mutex> g(mu_);
  return block_index_.count(block_id) != 0;
}

uint64_t MasterCore::total_blocks() const {
  std::lock_guard<std::mutex> g(mu_);
  uint64_t n = 0;
  for (auto& kv : files_) n += kv.second.blocks.size();
  return n;
}

std::string MasterCore::tx_record(const std::string& tx_id) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = tx_records_.find(tx_id);
  return it == tx_records_.end() ? std::string() : it->second.dump();
}

std::string MasterCore::tx_records() const {
  std::lock_guard<std::mutex> g(mu_);
  Json o = Json::object();
  for (auto& kv : tx_records_) o.set(kv.first, kv.second);
  return o.dump();
}

std::string MasterCore::tx_lock(const std::string& path) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = tx_locks_.find(path);
  return it == tx_locks_.end() ? std::string() : it->second;
}

std::vector<std::string> MasterCore::shuffling_prefixes() const {
  std::lock_guard<std::mutex> g(mu_);
  return {shuffling_prefixes_.begin(), shuffling_prefixes_.end()};
}

std::map<std::string, uint64_t> MasterCore::take_request_counts() {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, uint64_t> out;
  out.swap(request_counts_);
  return out;
}

int MasterCore::raft_rpc(const std::string& kind, const std::string& body, std::string* out) {
  raft::Node* node = node_.load();
  if (!node) return (*out = "raft node not attached", UNAVAILABLE);
  try {
    *out = node->handle(kind, body);
    return OK;
  } catch (const std::exception& e) {
    *out = e.what();
    return INTERNAL;
  }
}

std::vector<MasterCore::HealAction> MasterCore::heal_scan(
    int rf, const std::vector<std::string>& live, const std::map<std::string, std::vector<std::string>>& bad,
    const std::set<std::pair<std::string, std::string>>& queued) const {
  std::vector<HealAction> out;
  if (live.empty()) return out;
  const std::set<std::string> live_set(live.begin(), live.end());
  const size_t want = std::min<size_t>(static_cast<size_t>(std::max(rf, 0)), live.size());
  auto holds = [](const pb::BlockInfo& b, const std::string& s) {
    return std::find(b.locations.begin(), b.locations.end(), s) != b.locations.end();
  };
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : files_) {
    for (const pb::BlockInfo& b : kv.second.blocks) {
      if (b.ec_data_shards > 0) {
        const size_t total = static_cast<size_t>(b.ec_data_shards + b.ec_parity_shards);
        if (b.locations.size() != total) continue;
        size_t alive = 0;
        for (auto& l : b.locations) alive += live_set.count(l);
        for (size_t idx = 0; idx < b.locations.size(); ++idx) {
          if (live_set.count(b.locations[idx])) continue;
          if (alive < static_cast<size_t>(b.ec_data_shards)) break;  // not reconstructible
          auto t = std::find_if(live.begin(), live.end(), [&](const std::string& s) { return !holds(b, s); });
          if (t == live.end()) continue;
          HealAction a;
          a.reconstruct = true;
          a.queue_on = a.target = *t;
          a.block_id = b.block_id;
          a.shard_index = static_cast<int>(idx);
          a.ec_data = b.ec_data_shards;
          a.ec_parity = b.ec_parity_shards;
          for (auto& l : b.locations) a.sources.push_back(live_set.count(l) ? l : std::string());
          a.original_size = b.original_size;
          out.push_back(std::move(a));
        }
        continue;
      }
      auto bi = bad.find(b.block_id);
      std::vector<const std::string*> healthy;
      for (auto& l : b.locations)
        if (live_set.count(l) && (bi == bad.end() || std::find(bi->second.begin(), bi->second.end(), l) ==
                                                         bi->second.end()))
          healthy.push_back(&l);
      // copies already queued (not yet reported) count toward the target: a pass that runs
      // before the last one's replications land does not over-replicate
      size_t inflight = 0;
      for (auto q = queued.lower_bound({b.block_id, std::string()}); q != queued.end() && q->first == b.block_id; ++q)
        inflight += !holds(b, q->second);
      if (healthy.empty() || healthy.size() + inflight >= want) continue;
      size_t needed = want - healthy.size() - inflight;
      for (const std::string& s : live) {
        if (!needed) break;
        if (holds(b, s) || queued.count({b.block_id, s})) continue;
        HealAction a;
        a.queue_on = *healthy[0];
        a.block_id = b.block_id;
        a.target = s;
        out.push_back(std::move(a));
        --needed;
      }
    }
  }
  return out;
}

std::string MasterCore::pick_block(const std::string& src, const std::string& dst, const std::string* prefix) const {
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : files_) {
    if (prefix && kv.first.compare(0, prefix->size(), *prefix) != 0) continue;
    for (const pb::BlockInfo& b : kv.second.blocks) {
      if (b.ec_data_shards != 0) continue;
      const auto& l = b.locations;
      if (std::find(l.begin(), l.end(), src) != l.end() && std::find(l.begin(), l.end(), dst) == l.end())
        return b.block_id;
    }
  }
  return std::string();
}

std::vector<MasterCore::ColdFile> MasterCore::tiering_scan(uint64_t now_ms, uint64_t cold_ms) const {
  std::vector<ColdFile> out;
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : files_) {
    const pb::FileMetadata& f = kv.second;
    if (f.moved_to_cold_at_ms != 0 || f.ec_data_shards != 0 || f.last_access_ms == 0 ||
        now_ms <= f.last_access_ms || now_ms - f.last_access_ms <= cold_ms)
      continue;
    ColdFile c;
    c.path = f.path;
    for (const pb::BlockInfo& b : f.blocks) c.blocks.emplace_back(b.block_id, b.locations);
    out.push_back(std::move(c));
  }
  return out;
}

std::vector<std::string> MasterCore::ec_candidates(uint64_t now_ms, uint64_t ec_ms) const {
  std::vector<std::string> out;
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : files_) {
    const pb::FileMetadata& f = kv.second;
    if (f.moved_to_cold_at_ms == 0 || f.ec_data_shards != 0 || f.blocks.empty() || now_ms <= f.moved_to_cold_at_ms ||
        now_ms - f.moved_to_cold_at_ms <= ec_ms)
      continue;
    out.push_back(f.str());
  }
  return out;
}

std::vector<std::pair<std::string, std::vector<std::string>>> MasterCore::take_gc() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::pair<std::string, std::vector<std::string>>> out;
  out.swap(gc_);
  return out;
}

// ---------------------------------------------------------------- RPC plumbing
MasterCore::Result MasterCore::propose(const Json& cmd) {
  raft::Node* node = node_.load();
  if (!node) return {1, ""};
  auto prom = std::make_shared<std::promise<Result>>();
  auto fut = prom->get_future();
  node->propose(cmd.dump(), [prom](int code, const std::string& payload) { prom->set_value(Result{code, payload}); });
  if (fut.wait_for(std::chrono::seconds(30)) != std::future_status::ready) return {2, "proposal timed out"};
  return fut.get();
}

MasterCore::Result MasterCore::propose_unlocked(const std::string& name, const Json& args) {
  for (int attempt = 0; attempt < 50; ++attempt) {
    Json master = Json::object();
    master.set(name, args);
    Result r = propose(obj({{"Master", master}}));
    if (r.code != 0) return r;
    Json res = Json::parse(r.payload);
    const Json* lk = res.find("locked");
    if (!lk) return r;
    std::string err;
    if (!wait_unlocked(lk->str(), 5000, &err)) return {3, err};
  }
  return {3, name + ": path stays locked by cross-shard renames"};
}

int MasterCore::read_index(std::string* err) {
  raft::Node* node = node_.load();
  if (!node) {
    *err = "Not Leader";
    return FAILED_PRECONDITION;
  }
  auto prom = std::make_shared<std::promise<Result>>();
  auto fut = prom->get_future();
  node->read_index([prom](int code, const std::string& payload) { prom->set_value(Result{code, payload}); });
  if (fut.wait_for(std::chrono::seconds(10)) != std::future_status::ready) {
    *err = "ReadIndex timed out";
    return UNAVAILABLE;
  }
  Result r = fut.get();
  if (r.code == 0) return OK;
  if (r.code == 1) {
    *err = r.payload.empty() ? "Not Leader" : "Not Leader|" + r.payload;
    return FAILED_PRECONDITION;
  }
  *err = r.payload;
  return INTERNAL;
}

bool MasterCore::wait_unlocked(const std::string& path, int timeout_ms, std::string* err) {
  std::unique_lock<std::mutex> lk(mu_);
  if (!tx_locks_.count(path)) return true;
  if (applied_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return !tx_locks_.count(path); }))
    return true;
  auto it = tx_locks_.find(path);
  *err = path + " is locked by transaction " + (it == tx_locks_.end() ? std::string() : it->second);
  return false;
}

int MasterCore::check_ownership(const std::string& path, std::string* err) const {
  std::lock_guard<std::mutex> g(mu_);
  if (!have_map_) return OK;
  std::string target = shard_map_.get_shard(path);
  if (target.empty() || target == shard_id_) return OK;
  const auto* peers = shard_map_.peers(target);
  *err = "REDIRECT:" + (peers && !peers->empty() ? peers->front() : std::string());
  return OUT_OF_RANGE;
}

bool MasterCore::place(int ec_d, int ec_p, const std::string& preferred, std::vector<std::string>* out,
                       std::string* err) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<ChunkServerStatus> cands;
  for (auto& kv : chunk_servers_) cands.push_back(kv.second);
  size_t needed;
  bool ec = ec_d > 0 && ec_p > 0;
  if (ec) {
    size_t total = static_cast<size_t>(ec_d + ec_p);
    if (cands.size() < total) {
      *err = "Need " + std::to_string(total) + " chunk servers for EC(" + std::to_string(ec_d) + "," +
             std::to_string(ec_p) + "), only " + std::to_string(cands.size()) + " available";
      return false;
    }
    needed = total;
  } else {
    needed = std::min(kReplication, cands.size());
  }
  if (needed == 0) {
    *err = "No chunk servers available";
    return false;
  }
  *out = select_servers_rack_aware(cands, needed, ec ? std::string() : preferred);
  for (auto& a : *out) chunk_servers_[a].scheduled += kScheduleQuantum;
  return true;
}

void MasterCore::allocation(const std::string& block_id, const std::vector<std::string>& sel, int ec_d, int ec_p,
                            pb::AllocateBlockResponse* a) const {
  a->block.block_id = block_id;
  a->block.locations = sel;
  a->block.ec_data_shards = ec_d;
  a->block.ec_parity_shards = ec_p;
  a->has_block = true;
  a->chunk_server_addresses = sel;
  a->ec_data_shards = ec_d;
  a->ec_parity_shards = ec_p;
  raft::Node* node = node_.load();
  a->master_term = node ? node->term() : 0;
}

void MasterCore::record_request(const std::string& path) {
  std::string p = prefix_of(path);
  std::lock_guard<std::mutex> g(mu_);
  request_counts_[p]++;
  requests_++;
}

void MasterCore::record_access(const std::string& path) {
  raft::Node* node = node_.load();
  if (!node || !node->is_leader()) return;
  std::lock_guard<std::mutex> g(mu_);
  if (!access_stats_) return;
  access_buf_[path]++;
}

void MasterCore::access_loop() {
  // The reference fires one Raft write per GetFileInfo (master.rs:2187-2209); the same
  // statistics (last_access_ms, access_count) go out as ONE batched entry per window.
  while (running_) {
    std::map<std::string, uint64_t> buf;
    {
      std::unique_lock<std::mutex> lk(mu_);
      access_cv_.wait_for(lk, std::chrono::milliseconds(access_flush_ms_), [&] { return !running_.load(); });
      buf.swap(access_buf_);
    }
    raft::Node* node = node_.load();
    if (buf.empty() || !node || !node->is_leader()) continue;
    Json paths = Json::object();
    for (auto& kv : buf) paths.set(kv.first, kv.second);
    Json batch = obj({{"accessed_at_ms", now_ms()}, {"paths", paths}});
    Json master = obj({{"UpdateAccessStatsBatch", batch}});
    node->propose_nowait(obj({{"Master", master}}).dump());
  }
}

void MasterCore::queue_gc(const Json& blocks) {
  // Extension: blocks no file references any more get DELETE commands (the reference never
  // garbage-collects blocks; proto DELETE is "future use").
  std::lock_guard<std::mutex> g(mu_);
  for (auto& e : blocks.items()) {
    std::string bid = e[0].str();
    if (block_index_.count(bid)) continue;
    std::vector<std::string> locs;
    for (auto& l : e[1].items()) locs.push_back(l.str());
    gc_.emplace_back(bid, locs);
  }
}

std::string MasterCore::new_uuid() {
  uint64_t hi, lo;
  {
    std::lock_guard<std::mutex> g(mu_);
    hi = rng_();
    lo = rng_();
  }
  hi = (hi & ~0xF000ull) | 0x4000ull;                  // version 4
  lo = (lo & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;  // RFC 4122 variant
  char buf[40];
  std::snprintf(buf, sizeof buf, "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(hi >> 32),
                static_cast<unsigned>((hi >> 16) & 0xFFFF), static_cast<unsigned>(hi & 0xFFFF),
                static_cast<unsigned>(lo >> 48), static_cast<unsigned long long>(lo & 0xFFFFFFFFFFFFull));
  return buf;
}

// ---------------------------------------------------------------- handlers
bool MasterCore::native_method(const std::string& m) const {
  return m == "GetFileInfo" || m == "CreateFile" || m == "AllocateBlock" || m == "CompleteFile" ||
         m == "ListFiles" || m == "DeleteFile" || m == "GetBlockLocations" || m == "Rename" ||
         m == "PrepareTransaction" || m == "CommitTransaction" || m == "AbortTransaction" ||
         m == "InquireTransaction" || m == "Heartbeat" || m == "RegisterChunkServer" || m == "GetSafeModeStatus" ||
         m == "SetSafeMode";
}

int MasterCore::handle(const std::string& method, const std::string& req, std::string* out) {
  try {
    if (method == "GetFileInfo") return get_file_info(req, out);
    if (method == "CreateFile") return create_file(req, out);
    if (method == "CompleteFile") return complete_file(req, out);
    if (method == "AllocateBlock") return allocate_block(req, out);
    if (method == "ListFiles") return list_files(req, out);
    if (method == "DeleteFile") return delete_file(req, out);
    if (method == "Rename") return rename(req, out);
    if (method == "GetBlockLocations") return get_block_locations(req, out);
    if (method == "PrepareTransaction") return prepare_transaction(req, out);
    if (method == "CommitTransaction") return commit_transaction(req, out);
    if (method == "AbortTransaction") return abort_transaction(req, out);
    if (method == "InquireTransaction") return inquire_transaction(req, out);
    if (method == "Heartbeat") return heartbeat(req, out);
    if (method == "RegisterChunkServer") return register_chunk_server(req, out);
    if (method == "GetSafeModeStatus") return get_safe_mode_status(req, out);
    if (method == "SetSafeMode") return set_safe_mode(req, out);
  } catch (const std::exception& e) {
    *out = e.what();
    return INTERNAL;
  }
  *out = "unknown method " + method;
  return UNIMPLEMENTED;
}

int MasterCore::get_file_info(const std::string& raw, std::string* out) {
  pb::GetFileInfoRequest r;
  if (!r.decode(raw)) return (*out = "malformed GetFileInfoRequest", INTERNAL);
  record_request(r.path);
  record_access(r.path);
  int c;
  if ((c = check_ownership(r.path, out)) != OK) return c;
  if ((c = read_index(out)) != OK) return c;
  if (!wait_unlocked(r.path, 5000, out)) return UNAVAILABLE;
  pb::GetFileInfoResponse resp;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (const pb::FileMetadata* m = visible(r.path)) {
      resp.metadata = *m;
      resp.has_metadata = true;
      resp.found = true;
    }
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::create_file(const std::string& raw, std::string* out) {
  pb::CreateFileRequest r;
  if (!r.decode(raw)) return (*out = "malformed CreateFileRequest", INTERNAL);
  record_request(r.path);
  int c;
  if ((c = check_ownership(r.path, out)) != OK) return c;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (safe_mode_) return (*out = kSafeModeMsg, UNAVAILABLE);
  }
  if (!wait_unlocked(r.path, 5000, out)) return UNAVAILABLE;
  pb::CreateFileResponse resp;
  auto reply = [&]() {
    out->clear();
    resp.encode(*out);
    return static_cast<int>(OK);
  };
  {
    std::lock_guard<std::mutex> g(mu_);
    if (files_.count(r.path) && !under_construction_.count(r.path)) {
      resp.error_message = "File already exists";
      return reply();
    }
  }
  raft::Node* node = node_.load();
  std::vector<std::string> sel;
  if (r.allocate_block && r.defer_create) {
    // place the block now; the file appears with its data in CompleteFile{create}: one
    // Raft entry (one WAL fdatasync) per write instead of two
    std::string err;
    if (!place(r.ec_data_shards, r.ec_parity_shards, r.preferred_chunk_server, &sel, &err))
      return (*out = err, UNAVAILABLE);
    // no Raft entry here, so leadership must be known fresh: a leader cut off from its
    // majority (possibly already replaced) would hand out a stale master term
    if (!node || !node->is_leader() || !node->has_lease()) {
      resp.error_message = "Not Leader";
      resp.leader_hint = node && !node->is_leader() ? node->leader_address() : "";
      return reply();
    }
    resp.success = true;
    resp.deferred = true;
    allocation(new_uuid(), sel, r.ec_parity_shards ? r.ec_data_shards : 0, r.ec_data_shards ? r.ec_parity_shards : 0,
               &resp.allocation);
    resp.has_allocation = true;
    return reply();
  }
  Json args = obj({{"path", r.path},
                   {"ec_data_shards", r.ec_data_shards},
                   {"ec_parity_shards", r.ec_parity_shards},
                   {"ts", now_ms()}});
  std::string block_id;
  if (r.allocate_block) {
    // CreateFile + AllocateBlock as ONE Raft entry and one round trip
    std::string err;
    if (!place(r.ec_data_shards, r.ec_parity_shards, r.preferred_chunk_server, &sel, &err))
      return (*out = err, UNAVAILABLE);
    block_id = new_uuid();
    Json locs = Json::array();
    for (auto& s : sel) locs.push_back(s);
    args.set("block_id", block_id);
    args.set("locations", locs);
  }
  Result res = propose_unlocked("CreateFile", args);
  if (res.code == 1) {
    resp.error_message = "Not Leader";
    resp.leader_hint = res.payload;
    return reply();
  }
  if (res.code != 0) return (*out = res.payload, res.code == 3 ? UNAVAILABLE : INTERNAL);
  Json j = Json::parse(res.payload);
  if (j["exists"].as_bool()) {
    resp.error_message = "File already exists";
    return reply();
  }
  if (j["orphans"].size()) queue_gc(j["orphans"]);
  resp.success = true;
  resp.writer_generation = static_cast<uint64_t>(j["gen"].as_int());
  if (r.allocate_block) {
    int ec_d = 0, ec_p = 0;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = files_.find(r.path);
      if (it != files_.end()) {
        ec_d = it->second.ec_data_shards;
        ec_p = it->second.ec_parity_shards;
      }
    }
    allocation(block_id, sel, ec_d, ec_p, &resp.allocation);
    resp.has_allocation = true;
  }
  return reply();
}

int MasterCore::allocate_block(const std::string& raw, std::string* out) {
  pb::AllocateBlockRequest r;
  if (!r.decode(raw)) return (*out = "malformed AllocateBlockRequest", INTERNAL);
  record_request(r.path);
  int c;
  if ((c = check_ownership(r.path, out)) != OK) return c;
  int ec_d, ec_p;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (safe_mode_) return (*out = kSafeModeMsg, UNAVAILABLE);
    auto it = files_.find(r.path);
    if (it == files_.end()) return (*out = "File not found", NOT_FOUND);
    ec_d = it->second.ec_data_shards;
    ec_p = it->second.ec_parity_shards;
  }
  std::vector<std::string> sel;
  std::string err;
  if (!place(ec_d, ec_p, r.preferred_chunk_server, &sel, &err)) return (*out = err, UNAVAILABLE);
  std::string block_id = new_uuid();
  Json locs = Json::array();
  for (auto& s : sel) locs.push_back(s);
  Json args = obj({{"path", r.path}, {"block_id", block_id}, {"locations", locs}, {"ts", now_ms()}});
  if (r.writer_generation) args.set("gen", static_cast<int64_t>(r.writer_generation));
  Result res = propose(obj({{"Master", obj({{"AllocateBlock", args}})}}));
  pb::AllocateBlockResponse resp;
  if (res.code == 1) {
    resp.leader_hint = res.payload;
  } else if (res.code != 0) {
    return (*out = res.payload, INTERNAL);
  } else if (!res.payload.empty() && Json::parse(res.payload)["stale"].as_bool()) {
    return (*out = "Write lease lost: " + r.path + " was taken over by another writer", FAILED_PRECONDITION);
  } else {
    allocation(block_id, sel, ec_d, ec_p, &resp);
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::complete_file(const std::string& raw, std::string* out) {
  pb::CompleteFileRequest r;
  if (!r.decode(raw)) return (*out = "malformed CompleteFileRequest", INTERNAL);
  int c;
  if ((c = check_ownership(r.path, out)) != OK) return c;
  Json sums = Json::array();
  for (auto& s : r.block_checksums)
    sums.push_back(obj({{"block_id", s.block_id}, {"checksum_crc32c", s.checksum_crc32c}, {"actual_size", s.actual_size}}));
  Json args = obj({{"path", r.path},
                   {"size", r.size},
                   {"etag_md5", r.etag_md5.empty() ? Json() : Json(r.etag_md5)},
                   {"created_at_ms", r.created_at_ms ? Json(r.created_at_ms) : Json()},
                   {"block_checksums", sums}});
  if (!r.attributes.empty()) args.set("attributes", attrs_json(r.attributes));
  pb::CompleteFileResponse resp;
  auto not_leader = [&](const std::string& hint) {
    // CompleteFileResponse has no leader_hint: the read-path status makes clients follow it
    *out = hint.empty() ? "Not Leader" : "Not Leader|" + hint;
    return static_cast<int>(FAILED_PRECONDITION);
  };
  if (r.create) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (safe_mode_) return (*out = kSafeModeMsg, UNAVAILABLE);
    }
    if (!wait_unlocked(r.path, 5000, out)) return UNAVAILABLE;
    Json blocks = Json::array();
    for (auto& b : r.blocks) blocks.push_back(block_json(b));
    args.set("ts", now_ms());
    args.set("ec_data_shards", r.ec_data_shards);
    args.set("ec_parity_shards", r.ec_parity_shards);
    args.set("blocks", blocks);
    Result res = propose_unlocked("CreateComplete", args);
    if (res.code == 1) return not_leader(res.payload);
    if (res.code != 0) return (*out = res.payload, res.code == 3 ? UNAVAILABLE : INTERNAL);
    Json j = Json::parse(res.payload);
    if (j["exists"].as_bool()) {
      pb::FileMetadata tmp;
      tmp.blocks = r.blocks;
      queue_gc(block_list(tmp));  // our freshly written replicas belong to nobody
      resp.error_message = "File already exists";
    } else {
      if (j["orphans"].size()) queue_gc(j["orphans"]);
      resp.success = true;
    }
  } else {
    if (r.writer_generation) args.set("gen", static_cast<int64_t>(r.writer_generation));
    Result res = propose(obj({{"Master", obj({{"CompleteFile", args}})}}));
    if (res.code == 1) return not_leader(res.payload);
    if (res.code != 0) return (*out = res.payload, INTERNAL);
    Json j = Json::parse(res.payload);
    if (j["stale"].as_bool()) return (*out = "Write lease lost: " + r.path + " was taken over by another writer", FAILED_PRECONDITION);
    resp.success = j["found"].as_bool(true);
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::list_files(const std::string& raw, std::string* out) {
  pb::ListFilesRequest r;
  if (!r.decode(raw)) return (*out = "malformed ListFilesRequest", INTERNAL);
  int c;
  if ((c = read_index(out)) != OK) return c;
  pb::ListFilesResponse resp;
  if (!r.delimiter.empty()) {
    // one entry per distinct next component: after a prefix is seen, jump past every path
    // under it (they are contiguous in the ordered index)
    std::lock_guard<std::mutex> g(mu_);
    const std::string& pre = r.path;
    auto it = ordered_.lower_bound(pre);
    while (it != ordered_.end() && it->compare(0, pre.size(), pre) == 0) {
      const size_t d = it->find(r.delimiter, pre.size());
      if (d == std::string::npos) {
        if (!under_construction_.count(*it)) {
          resp.files.push_back(*it);
          if (r.with_metadata) resp.metadata.push_back(files_.at(*it));
        }
        ++it;
        continue;
      }
      std::string cp = it->substr(0, d + r.delimiter.size());
      std::string past = cp;
      // the smallest string greater than every path that starts with cp
      while (!past.empty() && static_cast<unsigned char>(past.back()) == 0xff) past.pop_back();
      if (past.empty()) {
        resp.common_prefixes.push_back(std::move(cp));
        break;
      }
      past.back() = static_cast<char>(static_cast<unsigned char>(past.back()) + 1);
      resp.common_prefixes.push_back(std::move(cp));
      it = ordered_.lower_bound(past);
    }
  } else if (!r.with_metadata) {
    resp.files = paths(r.path, true);
  } else {  // one consistent pass: paths and their metadata under the same lock
    std::lock_guard<std::mutex> g(mu_);
    for_prefix(r.path, [&](const std::string& p) {
      if (!under_construction_.count(p)) resp.files.push_back(p);
    });
    resp.metadata.reserve(resp.files.size());
    for (auto& p : resp.files) resp.metadata.push_back(files_.at(p));
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::delete_file(const std::string& raw, std::string* out) {
  pb::DeleteFileRequest r;
  if (!r.decode(raw)) return (*out = "malformed DeleteFileRequest", INTERNAL);
  record_request(r.path);
  int c;
  if ((c = check_ownership(r.path, out)) != OK) return c;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (safe_mode_) return (*out = kSafeModeMsg, UNAVAILABLE);
  }
  if (!wait_unlocked(r.path, 5000, out)) return UNAVAILABLE;
  pb::DeleteFileResponse resp;
  bool exists;
  {
    std::lock_guard<std::mutex> g(mu_);
    exists = visible(r.path) != nullptr;
  }
  if (!exists) {
    resp.error_message = "File not found";
  } else {
    Result res = propose_unlocked("DeleteFile", obj({{"path", r.path}}));
    if (res.code == 1) {
      resp.error_message = "Not Leader";
      resp.leader_hint = res.payload;
    } else if (res.code != 0) {
      return (*out = res.payload, res.code == 3 ? UNAVAILABLE : INTERNAL);
    } else {
      Json j = Json::parse(res.payload);
      if (!j["found"].as_bool(true)) {
        resp.error_message = "File not found";
      } else {
        queue_gc(j["blocks"]);
        resp.success = true;
      }
    }
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

// Same-shard Rename (reference master.rs rename, the local case): one Raft entry whose apply
// decides in log order. A rename whose destination another shard owns runs the 2PC below
// when a peer caller is configured (else it is declined to the Python coordinator,
// master/service.py, which is also where more than kMaxCoordinators concurrent ones go).
int MasterCore::rename(const std::string& raw, std::string* out) {
  pb::RenameRequest r;
  if (!r.decode(raw)) return (*out = "malformed RenameRequest", INTERNAL);
  int c;
  if ((c = check_ownership(r.source_path, out)) != OK) {
    record_request(r.source_path);
    return c;
  }
  std::string src_shard, dst_shard;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (safe_mode_) return (*out = kSafeModeMsg, UNAVAILABLE);
    if (have_map_ && map_max_age_ms_ > 0 && steady_ms() - map_fresh_ms_ > map_max_age_ms_) {
      // right after a split or merge the destination may have moved: a stale map could
      // commit locally a rename that belongs to another shard
      stale_map_declines_++;
      return kDecline;
    }
    if (have_map_) {
      std::string s = shard_map_.get_shard(r.source_path), d = shard_map_.get_shard(r.dest_path);
      src_shard = s.empty() ? shard_id_ : s;
      dst_shard = d.empty() ? shard_id_ : d;
    }
  }
  if (src_shard != dst_shard) {
    if (!peer_call_ || coordinators_.fetch_add(1) >= kMaxCoordinators) {
      if (peer_call_) coordinators_--;
      tx_declined_++;
      return kDecline;  // dfs_master waits for a slot and retries (rename_declined)
    }
    record_request(r.source_path);
    int rc = rename_2pc(r, src_shard, dst_shard, out);
    coordinators_--;
    return rc;
  }
  record_request(r.source_path);
  if (!wait_unlocked(r.source_path, 5000, out) || !wait_unlocked(r.dest_path, 5000, out)) return UNAVAILABLE;
  pb::RenameResponse resp;
  bool exists;
  {
    std::lock_guard<std::mutex> g(mu_);
    exists = visible(r.source_path) != nullptr;
  }
  if (!exists) {
    resp.error_message = "Source file not found: " + r.source_path;
  } else {
    Result res = propose_unlocked("RenameFile", obj({{"source_path", r.source_path}, {"dest_path", r.dest_path}}));
    if (res.code == 1) {
      resp.error_message = "Not Leader";
      resp.leader_hint = res.payload;
    } else if (res.code != 0) {
      return (*out = res.payload, res.code == 3 ? UNAVAILABLE : INTERNAL);
    } else {
      Json j = Json::parse(res.payload);
      const Json& e = j["error"];
      if (e.is_string() && !e.as_string().empty()) resp.error_message = e.as_string();
      else resp.success = true;
    }
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

namespace {
Json master_cmd(const char* name, Json args);  // below, with the 2PC helpers
}  // namespace

// ---------------------------------------------------------------- heartbeat (C33/C34)
void MasterCore::queue_command(const std::string& addr, const std::string& cmd) {
  std::lock_guard<std::mutex> g(mu_);
  cmd_q_[addr].push_back(cmd);
}

std::vector<std::string> MasterCore::take_commands(const std::string& addr) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  auto it = cmd_q_.find(addr);
  if (it != cmd_q_.end()) {
    out.swap(it->second);
    cmd_q_.erase(it);
  }
  return out;
}

std::map<std::string, std::vector<std::string>> MasterCore::peek_commands() const {
  std::lock_guard<std::mutex> g(mu_);
  return cmd_q_;
}

std::map<std::string, std::vector<std::string>> MasterCore::bad_blocks() const {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, std::vector<std::string>> out;
  for (auto& kv : bad_blocks_) out[kv.first].assign(kv.second.begin(), kv.second.end());
  return out;
}

void MasterCore::add_bad_block(const std::string& block_id, const std::string& addr) {
  std::lock_guard<std::mutex> g(mu_);
  bad_blocks_[block_id].insert(addr);
  heal_req_ = true;
}

std::pair<std::vector<std::string>, std::vector<std::string>> MasterCore::take_ec_reports() {
  std::lock_guard<std::mutex> g(mu_);
  std::pair<std::vector<std::string>, std::vector<std::string>> out;
  out.first.swap(ec_encoded_);
  out.second.swap(ec_failed_);
  return out;
}

bool MasterCore::take_heal_request() {
  std::lock_guard<std::mutex> g(mu_);
  bool r = heal_req_;
  heal_req_ = false;
  return r;
}

// Heartbeat (reference master.rs heartbeat handler): refresh the registry entry, record the
// replicas / rebuilt EC shards the server reports (AddBlockLocation, fire-and-forget Raft
// entries), safe-mode block accounting, bad-block reports (a heal pass is requested from the
// background healer), unreferenced blocks as DELETE commands, and the queued commands for
// this server with the current master term.
int MasterCore::heartbeat(const std::string& raw, std::string* out) {
  pb::HeartbeatRequest r;
  if (!r.decode(raw)) return (*out = "malformed HeartbeatRequest", INTERNAL);
  heartbeats_++;
  const std::string& addr = r.chunk_server_address;
  raft::Node* node = node_.load();
  bool is_new, safe;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = chunk_servers_.find(addr);
    is_new = it == chunk_servers_.end();
    ChunkServerStatus st;
    st.address = addr;
    st.last_heartbeat = now_ms();
    st.used_space = r.used_space;
    st.available_space = r.available_space;
    st.chunk_count = r.chunk_count;
    st.rack_id = !r.rack_id.empty() ? r.rack_id : (is_new ? std::string() : it->second.rack_id);
    st.gpu_rank = r.gpu_rank;
    st.hbm_capacity = r.hbm_capacity;
    st.hbm_used = r.hbm_used;
    chunk_servers_[addr] = st;
    for (auto& b : r.ec_encoded) ec_encoded_.push_back(b);
    for (auto& b : r.ec_failed) ec_failed_.push_back(b);
    for (auto& b : r.bad_blocks) bad_blocks_[b].insert(addr);
    if (!r.bad_blocks.empty()) heal_req_ = true;
    safe = safe_mode_;
  }
  if (node) {
    for (auto& bid : r.new_blocks)  // replicas created by REPLICATE / reconstruction
      node->propose_nowait(master_cmd("AddBlockLocation", obj({{"block_id", bid}, {"address", addr}})).dump());
    for (auto& ent : r.ec_rebuilt) {  // "<block>/<shard index>": the rebuilt shard's position
      size_t slash = ent.rfind('/');
      if (slash == std::string::npos || slash == 0 || slash + 1 >= ent.size()) continue;
      const std::string idx = ent.substr(slash + 1);
      if (idx.find_first_not_of("0123456789") != std::string::npos) continue;
      node->propose_nowait(master_cmd("AddBlockLocation", obj({{"block_id", ent.substr(0, slash)},
                                                               {"address", addr},
                                                               {"shard_index", static_cast<int64_t>(std::stoll(idx))}}))
                               .dump());
    }
  }
  if (safe && is_new) report_blocks(r.chunk_count);  // exits safe mode when due
  if (safe && should_exit_safe_mode()) exit_safe_mode();
  if (!r.bad_blocks.empty())
    std::fprintf(stderr, "dfs master: heartbeat: %zu bad block(s) reported by %s\n", r.bad_blocks.size(), addr.c_str());
  pb::HeartbeatResponse resp;
  {
    std::lock_guard<std::mutex> g(mu_);
    // blocks no file references any more: DELETE on every holder (Python's drain_gc)
    for (auto& e : gc_)
      for (auto& loc : e.second) {
        pb::ChunkServerCommand c;
        c.type = pb::ChunkServerCommand::DELETE;
        c.block_id = e.first;
        cmd_q_[loc].push_back(c.str());
      }
    gc_.clear();
    auto it = cmd_q_.find(addr);
    if (it != cmd_q_.end()) {
      for (auto& c : it->second) {
        pb::ChunkServerCommand cmd;
        if (cmd.decode(c)) resp.commands.push_back(std::move(cmd));
      }
      cmd_q_.erase(it);
    }
  }
  resp.success = true;
  resp.master_term = node ? node->term() : 0;
  out->clear();
  resp.encode(*out);
  return OK;
}

// RegisterChunkServer / GetSafeModeStatus / SetSafeMode (reference master.rs:258-367 and the
// handlers of the same names): the registry entry, the linearizable safe-mode view, manual
// enter / leave.
int MasterCore::register_chunk_server(const std::string& raw, std::string* out) {
  pb::RegisterChunkServerRequest r;
  if (!r.decode(raw)) return (*out = "malformed RegisterChunkServerRequest", INTERNAL);
  ChunkServerStatus st;
  st.address = r.address;
  st.last_heartbeat = now_ms();
  st.available_space = r.capacity;
  st.rack_id = r.rack_id;
  upsert_chunk_server(st);
  pb::RegisterChunkServerResponse resp;
  resp.success = true;
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::get_safe_mode_status(const std::string& raw, std::string* out) {
  pb::GetSafeModeStatusRequest r;
  if (!r.decode(raw)) return (*out = "malformed GetSafeModeStatusRequest", INTERNAL);
  int c;
  if ((c = read_index(out)) != OK) return c;
  pb::GetSafeModeStatusResponse resp;
  {
    std::lock_guard<std::mutex> g(mu_);
    resp.is_safe_mode = safe_mode_;
    resp.is_manual = safe_mode_manual_;
    resp.chunk_server_count = static_cast<uint32_t>(chunk_servers_.size());
    resp.expected_blocks = static_cast<uint32_t>(expected_blocks_);
    resp.reported_blocks = static_cast<uint32_t>(reported_blocks_);
    resp.threshold = safe_mode_threshold_;
    resp.entered_at = static_cast<uint64_t>(safe_mode_entered_at_);
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::set_safe_mode(const std::string& raw, std::string* out) {
  pb::SetSafeModeRequest r;
  if (!r.decode(raw)) return (*out = "malformed SetSafeModeRequest", INTERNAL);
  if (r.enter) enter_safe_mode(true);
  else exit_safe_mode();
  pb::SetSafeModeResponse resp;
  resp.success = true;
  {
    std::lock_guard<std::mutex> g(mu_);
    resp.is_safe_mode = safe_mode_;
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::get_block_locations(const std::string& raw, std::string* out) {
  pb::GetBlockLocationsRequest r;
  if (!r.decode(raw)) return (*out = "malformed GetBlockLocationsRequest", INTERNAL);
  int c;
  if ((c = read_index(out)) != OK) return c;
  pb::GetBlockLocationsResponse resp;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (pb::BlockInfo* b = find_block_locked(r.block_id, nullptr)) {
      resp.locations = b->locations;
      resp.found = true;
    }
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

// ---------------------------------------------------------------- cross-shard Rename (2PC)
// Coordinator (the source shard's leader) and participant (the destination shard's leader)
// of the reference's presumed-abort 2PC (master.rs:2562-2683, :2724-2900), same records and
// the same recovery contract as the Python coordinator (master/service.py, tx_recovery in
// master/background.py): Pending -> Prepared on the coordinator, PrepareTransaction pins the
// destination on the participant, CommitTransaction creates it, the coordinator deletes the
// source and marks the record Committed + acked. Differences: proposals whose outcomes do
// not gate each other are queued back to back and ride one WAL group commit (record +
// Prepared; source delete + Committed + acked; the participant's create + Committed), so a
// rename costs 3 sequential Raft commits instead of 7.
void MasterCore::enable_native_2pc(PeerCall call) { peer_call_ = std::move(call); }

Json MasterCore::txn_stats() const {
  return obj({{"native_started", tx_started_.load()},
              {"native_committed", tx_committed_.load()},
              {"native_aborted", tx_aborted_.load()},
              {"native_pending", tx_pending_.load()},
              {"declined", tx_declined_.load()},
              {"stale_map_declines", stale_map_declines_.load()},
              {"enabled", static_cast<bool>(peer_call_)}});
}

namespace {

Json master_cmd(const char* name, Json args) {
  Json m = Json::object();
  m.set(name, std::move(args));
  return obj({{"Master", m}});
}

Json state_cmd(const std::string& tx, const char* st) {
  return master_cmd("UpdateTransactionState", obj({{"tx_id", tx}, {"new_state", st}}));
}

Json op_json(const std::string& shard, const char* kind, Json body) {
  Json op = Json::object();
  op.set(kind, std::move(body));
  return obj({{"shard_id", shard}, {"op_type", op}});
}

Json strings(const std::vector<std::string>& v) {
  Json a = Json::array();
  for (auto& x : v) a.push_back(x);
  return a;
}

}  // namespace

template <class Resp>
bool MasterCore::call_peers(const std::vector<std::string>& peers, const std::string& method, const std::string& req) {
  std::set<std::string> tried;
  std::deque<std::string> queue(peers.begin(), peers.end());
  while (!queue.empty()) {
    std::string addr = queue.front();
    queue.pop_front();
    if (addr.empty() || !tried.insert(addr).second) continue;
    GrpcResult g = peer_call_(addr, "/dfs.MasterService/" + method, req, 5000);
    if (!g.transport_ok || g.status != 0) continue;  // unreachable, REDIRECT, ...: next peer
    Resp resp;
    if (!resp.decode(g.message)) continue;
    if (resp.success) return true;
    if (!resp.leader_hint.empty() && !tried.count(resp.leader_hint)) {
      queue.push_front(resp.leader_hint);
    } else if (!resp.error_message.empty() && resp.error_message != "Not Leader") {
      return false;  // a decided refusal (destination exists / locked): no other peer helps
    }
  }
  return false;
}

std::vector<MasterCore::Result> MasterCore::propose_all(const std::vector<Json>& cmds) {
  std::vector<Result> out(cmds.size(), Result{1, ""});
  raft::Node* node = node_.load();
  if (!node) return out;
  std::vector<std::future<Result>> futs;
  for (auto& c : cmds) {
    auto prom = std::make_shared<std::promise<Result>>();
    futs.push_back(prom->get_future());
    node->propose(c.dump(), [prom](int code, const std::string& payload) { prom->set_value(Result{code, payload}); });
  }
  auto deadline = Clock::now() + std::chrono::seconds(30);
  for (size_t i = 0; i < futs.size(); ++i)
    out[i] = futs[i].wait_until(deadline) == std::future_status::ready ? futs[i].get()
                                                                       : Result{2, "proposal timed out"};
  return out;
}

int MasterCore::rename_2pc(const pb::RenameRequest& r, const std::string& src_shard, const std::string& dst_shard,
                           std::string* out) {
  pb::RenameResponse resp;
  auto reply = [&]() {
    out->clear();
    resp.encode(*out);
    return static_cast<int>(OK);
  };
  const std::string& src = r.source_path;
  const std::string& dst = r.dest_path;
  if (!wait_unlocked(src, 5000, out)) return UNAVAILABLE;
  pb::FileMetadata dmeta;
  std::vector<std::string> dst_peers, my_peers;
  std::string my_shard;
  {
    std::lock_guard<std::mutex> g(mu_);
    const pb::FileMetadata* m = visible(src);
    if (!m) {
      resp.error_message = "Source file not found: " + src;
      return reply();
    }
    dmeta = *m;
    if (const auto* p = shard_map_.peers(dst_shard)) dst_peers = *p;
    if (const auto* p = shard_map_.peers(shard_id_)) my_peers = *p;
    my_shard = shard_id_;
  }
  dmeta.path = dst;
  const std::string tx = new_uuid();
  tx_started_++;
  Json ops = Json::array();
  ops.push_back(op_json(src_shard, "Delete", obj({{"path", src}})));
  ops.push_back(op_json(dst_shard, "Create", obj({{"path", dst}, {"metadata", file_json(dmeta)}})));
  Json rec = obj({{"tx_id", tx},
                  {"tx_type", obj({{"Rename", obj({{"source_path", src}, {"dest_path", dst}})}})},
                  {"state", "Pending"},
                  {"timestamp", now_ms()},
                  {"participants", strings({src_shard, dst_shard})},
                  {"operations", ops},
                  {"coordinator_shard", src_shard},
                  {"participant_acked", false},
                  {"inquiry_count", 0}});
  auto abort_all = [&]() {
    pb::AbortTransactionRequest a;
    a.tx_id = tx;
    call_peers<pb::AbortTransactionResponse>(dst_peers, "AbortTransaction", a.str());
    propose(state_cmd(tx, "Aborted"));
    tx_aborted_++;
  };
  // record (Pending) and Prepared back to back: a rejected record makes the update a no-op
  std::vector<Result> rs = propose_all({master_cmd("CreateTransactionRecord", obj({{"record", rec}})),
                                        state_cmd(tx, "Prepared")});
  if (rs[0].code == 1) {
    resp.error_message = "Not Leader";
    resp.leader_hint = rs[0].payload;
    return reply();
  }
  if (rs[0].code != 0) return (*out = rs[0].payload, INTERNAL);
  const Json parsed = Json::parse(rs[0].payload);
  const Json& conflict = parsed["conflict"];
  if (conflict.is_string() && !conflict.as_string().empty()) {
    resp.error_message = conflict.as_string();
    return reply();
  }
  if (rs[1].code != 0) {
    abort_all();
    resp.error_message = "Internal error: Raft commit failed";
    return reply();
  }
  pb::PrepareTransactionRequest prep;
  prep.tx_id = tx;
  prep.operation_type = "CREATE";
  prep.path = dst;
  prep.metadata = dmeta;
  prep.has_metadata = true;
  prep.coordinator_shard = my_shard;
  prep.coordinator_peers = my_peers;
  if (!call_peers<pb::PrepareTransactionResponse>(dst_peers, "PrepareTransaction", prep.str())) {
    abort_all();
    resp.error_message = "Cross-shard prepare failed";
    return reply();
  }
  const char* drop = std::getenv("DFS_DEBUG_2PC_DROP_COMMIT");
  pb::CommitTransactionRequest com;
  com.tx_id = tx;
  if ((drop && std::string(drop) == "1") ||
      !call_peers<pb::CommitTransactionResponse>(dst_peers, "CommitTransaction", com.str())) {
    // the record stays Prepared: tx_recovery (background) re-drives the commit
    tx_pending_++;
    resp.error_message = "Cross-shard commit pending, will be retried";
    return reply();
  }
  rs = propose_all({master_cmd("ApplyTransactionOperation",
                               obj({{"tx_id", tx}, {"operation", op_json(src_shard, "Delete", obj({{"path", src}}))}})),
                    state_cmd(tx, "Committed"), master_cmd("SetParticipantAcked", obj({{"tx_id", tx}}))});
  for (auto& x : rs)
    if (x.code != 0) std::fprintf(stderr, "dfs master: tx %s: coordinator finish failed: %s\n", tx.c_str(),
                                  x.payload.c_str());
  tx_committed_++;
  resp.success = true;
  return reply();
}

int MasterCore::prepare_transaction(const std::string& raw, std::string* out) {
  pb::PrepareTransactionRequest r;
  if (!r.decode(raw)) return (*out = "malformed PrepareTransactionRequest", INTERNAL);
  pb::PrepareTransactionResponse resp;
  auto reply = [&]() {
    out->clear();
    resp.encode(*out);
    return static_cast<int>(OK);
  };
  {
    std::lock_guard<std::mutex> g(mu_);
    if (tx_records_.count(r.tx_id)) {  // a retried prepare
      resp.success = true;
      return reply();
    }
  }
  int c;
  if ((c = check_ownership(r.path, out)) != OK) return c;
  std::string err;
  if (!wait_unlocked(r.path, 1000, &err)) {
    resp.error_message = "Destination is locked by another transaction: " + r.path;
    return reply();
  }
  std::string me;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (files_.count(r.path)) {
      resp.error_message = "Destination file already exists: " + r.path;
      return reply();
    }
    me = shard_id_;
  }
  Json ops = Json::array();
  ops.push_back(op_json(me, "Create", obj({{"path", r.path}, {"metadata", file_json(r.metadata)}})));
  Json rec = obj({{"tx_id", r.tx_id},
                  {"tx_type", obj({{"Rename", obj({{"source_path", ""}, {"dest_path", r.path}})}})},
                  {"state", "Prepared"},
                  {"timestamp", now_ms()},
                  {"participants", strings({r.coordinator_shard, me})},
                  {"operations", ops},
                  {"coordinator_shard", r.coordinator_shard},
                  {"participant_acked", false},
                  {"inquiry_count", 0},
                  {"coordinator_peers", strings(r.coordinator_peers)}});
  Result res = propose(master_cmd("CreateTransactionRecord", obj({{"record", rec}})));
  if (res.code == 1) {
    resp.error_message = "Not Leader";
    resp.leader_hint = res.payload;
    return reply();
  }
  if (res.code != 0) return (*out = res.payload, INTERNAL);
  const Json parsed = Json::parse(res.payload);
  const Json& conflict = parsed["conflict"];
  if (conflict.is_string() && !conflict.as_string().empty()) {
    resp.error_message = conflict.as_string();
    return reply();
  }
  resp.success = true;
  return reply();
}

int MasterCore::commit_transaction(const std::string& raw, std::string* out) {
  pb::CommitTransactionRequest r;
  if (!r.decode(raw)) return (*out = "malformed CommitTransactionRequest", INTERNAL);
  pb::CommitTransactionResponse resp;
  auto reply = [&]() {
    out->clear();
    resp.encode(*out);
    return static_cast<int>(OK);
  };
  Json op;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = tx_records_.find(r.tx_id);
    if (it != tx_records_.end() && it->second["state"].str() == "Committed") {
      resp.success = true;
      return reply();
    }
    if (it == tx_records_.end() || !it->second["operations"].size()) {
      resp.error_message = "Transaction not found: " + r.tx_id;
      return reply();
    }
    op = it->second["operations"][0];
  }
  std::vector<Result> rs =
      propose_all({master_cmd("ApplyTransactionOperation", obj({{"tx_id", r.tx_id}, {"operation", op}})),
                   state_cmd(r.tx_id, "Committed")});
  if (rs[0].code == 1) {
    resp.error_message = "Not Leader";
    resp.leader_hint = rs[0].payload;
    return reply();
  }
  if (rs[0].code != 0) return (*out = rs[0].payload, INTERNAL);
  resp.success = true;
  return reply();
}

int MasterCore::abort_transaction(const std::string& raw, std::string* out) {
  pb::AbortTransactionRequest r;
  if (!r.decode(raw)) return (*out = "malformed AbortTransactionRequest", INTERNAL);
  pb::AbortTransactionResponse resp;
  Result res = propose(state_cmd(r.tx_id, "Aborted"));
  if (res.code == 1) {
    resp.error_message = "Not Leader";
    resp.leader_hint = res.payload;
  } else if (res.code != 0) {
    return (*out = res.payload, INTERNAL);
  } else {
    resp.success = true;
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

int MasterCore::inquire_transaction(const std::string& raw, std::string* out) {
  pb::InquireTransactionRequest r;
  if (!r.decode(raw)) return (*out = "malformed InquireTransactionRequest", INTERNAL);
  int c;
  if ((c = read_index(out)) != OK) return c;
  pb::InquireTransactionResponse resp;
  resp.status = "UNKNOWN";
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = tx_records_.find(r.tx_id);
    if (it != tx_records_.end()) {
      const std::string& st = it->second["state"].str();
      if (st == "Committed") resp.status = "COMMITTED";
      else if (st == "Aborted") resp.status = "ABORTED";
    }
  }
  out->clear();
  resp.encode(*out);
  return OK;
}

}  // namespace dfs
