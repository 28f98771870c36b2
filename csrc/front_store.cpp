// RemoteFrontStore: the native S3 front's file-system side for a gateway on another host; see
// front_store.h.
#include "front_store.h"

#include <chrono>
#include <cstdlib>
#include <cstring>

namespace dfs {

RemoteFrontStore::RemoteFrontStore(const std::string& shard_map_json, const std::vector<std::string>& masters,
                                   size_t slots, size_t slot_bytes, int timeout_ms, std::shared_ptr<TlsContext> tls)
    : rc_(4, timeout_ms, std::move(tls)), slot_bytes_((slot_bytes + 63) / 64 * 64) {
  rc_.set_routing(shard_map_json, masters);
  slots = slots ? slots : 1;
  base_ = static_cast<uint8_t*>(std::aligned_alloc(64, slots * slot_bytes_));
  if (!base_) throw std::bad_alloc();
  for (size_t i = slots; i-- > 0;) free_.push_back(static_cast<int64_t>(i * slot_bytes_));
}

RemoteFrontStore::~RemoteFrontStore() { std::free(base_); }

int64_t RemoteFrontStore::acquire_slot(size_t n) {
  if (n > slot_bytes_) return -1;
  std::unique_lock<std::mutex> lk(mu_);
  if (!cv_.wait_for(lk, std::chrono::seconds(5), [&] { return !free_.empty(); })) return -1;
  const int64_t s = free_.back();
  free_.pop_back();
  return s;
}

void RemoteFrontStore::release(int64_t slot) {
  if (slot < 0) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(slot / static_cast<int64_t>(slot_bytes_) * static_cast<int64_t>(slot_bytes_));
  }
  cv_.notify_one();
}

FrontStore::Status RemoteFrontStore::write_slot(const std::string& path, int64_t slot, size_t n, int* replicas,
                                                std::string* msg, Times* t, const std::string& rid,
                                                const std::map<std::string, std::string>* attrs,
                                                const char* etag_attr, std::string* md5_out) {
  if (slot < 0 || n > slot_bytes_) return FastClient::NotHandled;
  return rc_.write_etag(path, base_ + slot, n, replicas, msg, t, rid, attrs, etag_attr, md5_out);
}

FrontStore::Status RemoteFrontStore::stat(const std::string& path, bool* found, std::string* meta_pb,
                                          std::string* msg, const std::string& rid) {
  return rc_.stat(path, found, meta_pb, msg, rid);
}

FrontStore::Status RemoteFrontStore::read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n,
                                                std::string* msg, Times* t, const std::string& rid, uint64_t offset,
                                                uint64_t length) {
  pb::FileMetadata m;
  if (!m.decode(meta_pb)) return FastClient::NotHandled;
  if (m.size == 0) {
    *slot = -1;
    *n = 0;
    return FastClient::Ok;
  }
  const uint64_t want = length > 0 ? std::min<uint64_t>(length, offset < m.size ? m.size - offset : 0) : m.size;
  if (want > slot_bytes_) return FastClient::NotHandled;
  std::string data;
  Status st = rc_.read_meta(m, &data, msg, t, rid, offset, length);
  if (st != FastClient::Ok) return st;
  if (data.size() > slot_bytes_) return FastClient::NotHandled;
  const int64_t s = acquire_slot(data.size());
  if (s < 0) return FastClient::NotHandled;
  std::memcpy(base_ + s, data.data(), data.size());
  *slot = s;
  *n = data.size();
  return FastClient::Ok;
}

FrontStore::Status RemoteFrontStore::remove(const std::string& path, std::string* msg, const std::string& rid) {
  return rc_.remove(path, msg, rid);
}

FrontStore::Status RemoteFrontStore::rename(const std::string& src, const std::string& dst, std::string* msg,
                                            const std::string& rid) {
  return rc_.rename(src, dst, msg, rid);
}

FrontStore::Status RemoteFrontStore::list(const std::string& prefix,
                                          std::vector<std::pair<std::string, pb::FileMetadata>>* out,
                                          const std::string& rid) {
  return rc_.list(prefix, out, rid);
}

LocalFirstFrontStore::LocalFirstFrontStore(FastClient* fc, const std::string& shard_map_json,
                                           const std::vector<std::string>& masters, int timeout_ms,
                                           std::shared_ptr<TlsContext> tls)
    : fc_(fc), rc_(4, timeout_ms, std::move(tls)) {
  fc_->set_routing(shard_map_json, masters);
  rc_.set_routing(shard_map_json, masters);
}

FrontStore::Status LocalFirstFrontStore::write_slot(const std::string& path, int64_t slot, size_t n, int* replicas,
                                                    std::string* msg, Times* t, const std::string& rid,
                                                    const std::map<std::string, std::string>* attrs,
                                                    const char* etag_attr, std::string* md5_out) {
  Status st = fc_->write_slot(path, slot, n, replicas, msg, t, rid, attrs, etag_attr, md5_out);
  if (st != FastClient::NotHandled || slot < 0 || n > fc_->slot_bytes()) return st;
  fallbacks_++;
  msg->clear();
  return rc_.write_etag(path, fc_->slot_ptr(slot), n, replicas, msg, t, rid, attrs, etag_attr, md5_out);
}

FrontStore::Status LocalFirstFrontStore::stat(const std::string& path, bool* found, std::string* meta_pb,
                                              std::string* msg, const std::string& rid) {
  Status st = fc_->stat(path, found, meta_pb, msg, rid);
  if (st != FastClient::NotHandled) return st;
  fallbacks_++;
  msg->clear();
  return rc_.stat(path, found, meta_pb, msg, rid);
}

FrontStore::Status LocalFirstFrontStore::read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n,
                                                    std::string* msg, Times* t, const std::string& rid,
                                                    uint64_t offset, uint64_t length) {
  Status st = fc_->read_known(meta_pb, slot, n, msg, t, rid, offset, length);
  if (st != FastClient::NotHandled) return st;
  pb::FileMetadata m;
  if (!m.decode(meta_pb)) return st;
  fallbacks_++;
  msg->clear();
  std::string data;
  st = rc_.read_meta(m, &data, msg, t, rid, offset, length);
  if (st != FastClient::Ok) return st;
  if (data.empty()) {
    *slot = -1;
    *n = 0;
    return FastClient::Ok;
  }
  if (data.size() > fc_->slot_bytes()) return FastClient::NotHandled;
  const int64_t s = fc_->acquire_slot(data.size());
  if (s < 0) return FastClient::NotHandled;
  std::memcpy(fc_->slot_mut(s), data.data(), data.size());
  *slot = s;
  *n = data.size();
  return FastClient::Ok;
}

FrontStore::Status LocalFirstFrontStore::remove(const std::string& path, std::string* msg, const std::string& rid) {
  Status st = fc_->remove(path, msg, rid);
  if (st != FastClient::NotHandled) return st;
  fallbacks_++;
  msg->clear();
  return rc_.remove(path, msg, rid);
}

FrontStore::Status LocalFirstFrontStore::rename(const std::string& src, const std::string& dst, std::string* msg,
                                                const std::string& rid) {
  Status st = fc_->rename(src, dst, msg, rid);
  if (st != FastClient::NotHandled) return st;
  fallbacks_++;
  msg->clear();
  return rc_.rename(src, dst, msg, rid);
}

FrontStore::Status LocalFirstFrontStore::list(const std::string& prefix,
                                              std::vector<std::pair<std::string, pb::FileMetadata>>* out,
                                              const std::string& rid) {
  Status st = fc_->list(prefix, out, rid);
  if (st != FastClient::NotHandled) return st;
  fallbacks_++;
  out->clear();
  return rc_.list(prefix, out, rid);
}

}  // namespace dfs
