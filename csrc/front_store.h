// FrontStore: what the native S3 front (s3_front.cpp) needs from the file system. Payloads are
// produced and consumed in place in slots: a PUT body is received straight into a slot and
// written from there; a GET is read into a slot and sent from there.
//
// Two implementations:
//  * FastClient (client_fast.h), a gateway co-located with a chunkserver: the slots are the
//    chunkserver-shared /dev/shm arena the chunkserver registers with HIP, blocks move slot <->
//    HBM in one DMA, and the masters are reached over their same-host sockets.
//  * RemoteFrontStore (below), a gateway on another host (reference s3_server/src/main.rs runs
//    the gateway as its own service, talking gRPC to masters and chunkservers): private slots,
//    and every master and chunkserver call over gRPC through RemoteClient (client_remote.h),
//    with its leader following, hedged reads and EC decode.
//  * LocalFirstFrontStore (below), the executable gateway co-located with a chunkserver: the
//    FastClient for everything it serves, and a RemoteClient (leader following over gRPC) for
//    the calls it declines (a shard leader that is not its first peer or on another host, a
//    dead local master, a multi-block file), with the body still in the FastClient's slot.
// Either way the front serves the same requests natively; NotHandled sends a request to the
// gateway's Python path (a hosted front) or its own error answer (the executable).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "client_fast.h"
#include "client_remote.h"

namespace dfs {

class FrontStore {
 public:
  using Status = FastClient::Status;
  using Times = FastClient::Times;
  virtual ~FrontStore() = default;
  virtual size_t slot_bytes() const = 0;
  virtual int64_t acquire_slot(size_t n) = 0;  // -1: none free within 5 s, or n > slot_bytes()
  virtual const uint8_t* slot_ptr(int64_t slot) const = 0;
  virtual uint8_t* slot_mut(int64_t slot) = 0;
  virtual void release(int64_t slot) = 0;
  virtual Status write_slot(const std::string& path, int64_t slot, size_t n, int* replicas, std::string* msg,
                            Times* t, const std::string& rid, const std::map<std::string, std::string>* attrs,
                            const char* etag_attr, std::string* md5_out) = 0;
  virtual Status stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg,
                      const std::string& rid) = 0;
  virtual Status read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg, Times* t,
                            const std::string& rid, uint64_t offset, uint64_t length) = 0;
  virtual Status remove(const std::string& path, std::string* msg, const std::string& rid) = 0;
  virtual Status rename(const std::string& src, const std::string& dst, std::string* msg, const std::string& rid) = 0;
  virtual Status list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
                      const std::string& rid) = 0;
  // The distinct next path components below `prefix` (ListBuckets). This default lists every
  // path; the co-located stores ask the masters for one entry per component instead.
  virtual Status list_components(const std::string& prefix, std::set<std::string>* out, const std::string& rid) {
    std::vector<std::pair<std::string, pb::FileMetadata>> files;
    Status st = list(prefix, &files, rid);
    if (st != FastClient::Ok) return st;
    for (auto& f : files) {
      const size_t e = f.first.find('/', prefix.size());
      if (f.first.compare(0, prefix.size(), prefix) == 0 && e != std::string::npos && e > prefix.size())
        out->insert(f.first.substr(prefix.size(), e - prefix.size()));
    }
    return FastClient::Ok;
  }
  // calls a first-choice path declined and a second one served (LocalFirstFrontStore)
  virtual uint64_t fallbacks() const { return 0; }
};

// The co-located form: every call goes to the FastClient (not owned).
class FastFrontStore final : public FrontStore {
 public:
  explicit FastFrontStore(FastClient* fc) : fc_(fc) {}
  size_t slot_bytes() const override { return fc_->slot_bytes(); }
  int64_t acquire_slot(size_t n) override { return fc_->acquire_slot(n); }
  const uint8_t* slot_ptr(int64_t slot) const override { return fc_->slot_ptr(slot); }
  uint8_t* slot_mut(int64_t slot) override { return fc_->slot_mut(slot); }
  void release(int64_t slot) override { fc_->release(slot); }
  Status write_slot(const std::string& path, int64_t slot, size_t n, int* replicas, std::string* msg, Times* t,
                    const std::string& rid, const std::map<std::string, std::string>* attrs, const char* etag_attr,
                    std::string* md5_out) override {
    return fc_->write_slot(path, slot, n, replicas, msg, t, rid, attrs, etag_attr, md5_out);
  }
  Status stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg,
              const std::string& rid) override {
    return fc_->stat(path, found, meta_pb, msg, rid);
  }
  Status read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg, Times* t,
                    const std::string& rid, uint64_t offset, uint64_t length) override {
    return fc_->read_known(meta_pb, slot, n, msg, t, rid, offset, length);
  }
  Status remove(const std::string& path, std::string* msg, const std::string& rid) override {
    return fc_->remove(path, msg, rid);
  }
  Status rename(const std::string& src, const std::string& dst, std::string* msg, const std::string& rid) override {
    return fc_->rename(src, dst, msg, rid);
  }
  Status list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
              const std::string& rid) override {
    return fc_->list(prefix, out, rid);
  }
  Status list_components(const std::string& prefix, std::set<std::string>* out, const std::string& rid) override {
    return fc_->list_components(prefix, out, rid);
  }

 private:
  FastClient* fc_;
};

// The remote form: `slots` private slots of `slot_bytes` (allocated once, 64 B aligned) and a
// RemoteClient. Reads land in the client's reply buffer and are copied into the slot once.
class RemoteFrontStore final : public FrontStore {
 public:
  RemoteFrontStore(const std::string& shard_map_json, const std::vector<std::string>& masters, size_t slots,
                   size_t slot_bytes, int timeout_ms = 120000, std::shared_ptr<TlsContext> tls = nullptr);
  ~RemoteFrontStore() override;
  RemoteFrontStore(const RemoteFrontStore&) = delete;
  void set_routing(const std::string& shard_map_json, const std::vector<std::string>& masters) {
    rc_.set_routing(shard_map_json, masters);
  }
  RemoteClient& client() { return rc_; }

  size_t slot_bytes() const override { return slot_bytes_; }
  int64_t acquire_slot(size_t n) override;
  const uint8_t* slot_ptr(int64_t slot) const override { return base_ + slot; }
  uint8_t* slot_mut(int64_t slot) override { return base_ + slot; }
  void release(int64_t slot) override;
  Status write_slot(const std::string& path, int64_t slot, size_t n, int* replicas, std::string* msg, Times* t,
                    const std::string& rid, const std::map<std::string, std::string>* attrs, const char* etag_attr,
                    std::string* md5_out) override;
  Status stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg,
              const std::string& rid) override;
  Status read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg, Times* t,
                    const std::string& rid, uint64_t offset, uint64_t length) override;
  Status remove(const std::string& path, std::string* msg, const std::string& rid) override;
  Status rename(const std::string& src, const std::string& dst, std::string* msg, const std::string& rid) override;
  Status list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
              const std::string& rid) override;

 private:
  RemoteClient rc_;
  size_t slot_bytes_;
  uint8_t* base_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<int64_t> free_;  // slot offsets
};

// The executable gateway's co-located store: FastClient first, RemoteClient for what it
// declines. Slots are the FastClient's (shared with the chunkserver), so a PUT body received
// into one is written over gRPC from there when the fast path cannot take it.
class LocalFirstFrontStore final : public FrontStore {
 public:
  LocalFirstFrontStore(FastClient* fc, const std::string& shard_map_json, const std::vector<std::string>& masters,
                       int timeout_ms = 120000, std::shared_ptr<TlsContext> tls = nullptr);
  void set_routing(const std::string& shard_map_json, const std::vector<std::string>& masters) {
    fc_->set_routing(shard_map_json, masters);
    rc_.set_routing(shard_map_json, masters);
  }

  size_t slot_bytes() const override { return fc_->slot_bytes(); }
  int64_t acquire_slot(size_t n) override { return fc_->acquire_slot(n); }
  const uint8_t* slot_ptr(int64_t slot) const override { return fc_->slot_ptr(slot); }
  uint8_t* slot_mut(int64_t slot) override { return fc_->slot_mut(slot); }
  void release(int64_t slot) override { fc_->release(slot); }
  Status write_slot(const std::string& path, int64_t slot, size_t n, int* replicas, std::string* msg, Times* t,
                    const std::string& rid, const std::map<std::string, std::string>* attrs, const char* etag_attr,
                    std::string* md5_out) override;
  Status stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg,
              const std::string& rid) override;
  Status read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg, Times* t,
                    const std::string& rid, uint64_t offset, uint64_t length) override;
  Status remove(const std::string& path, std::string* msg, const std::string& rid) override;
  Status rename(const std::string& src, const std::string& dst, std::string* msg, const std::string& rid) override;
  Status list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
              const std::string& rid) override;
  uint64_t fallbacks() const override { return fallbacks_.load(); }
  Status list_components(const std::string& prefix, std::set<std::string>* out, const std::string& rid) override {
    if (fc_->list_components(prefix, out, rid) == FastClient::Ok) return FastClient::Ok;
    ++fallbacks_;
    out->clear();
    return FrontStore::list_components(prefix, out, rid);
  }

 private:
  FastClient* fc_;
  RemoteClient rc_;
  std::atomic<uint64_t> fallbacks_{0};
};

}  // namespace dfs
