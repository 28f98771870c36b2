// Native S3 front end: the HTTP/1.1 listener of the S3 gateway (C52-C54 data path; reference
// dfs/s3_server/src/main.rs:243-256 router, handlers.rs:918-1365 object handlers,
// auth_middleware.rs:19-365 SigV4).
//
// The hot object operations run here in C++, with no interpreter on the path:
//   PUT object, UploadPart  -> body read from the socket straight into a FastClient slot
//                              (the /dev/shm arena the co-located chunkserver has pinned for
//                              its copy engines), CRC + MD5 in C++, then the native write
//                              (CreateFile -> fast path -> HBM -> CompleteFile with the
//                              object headers as attributes);
//   GET / HEAD / Range GET  -> GetFileInfo, then the chunkserver's fused verify+copy kernel
//                              lands the (range of the) block in a slot that is written to
//                              the socket as is; multipart objects are streamed part by
//                              part from the layout recorded at completion.
//   DELETE, DeleteObjects,  -> the object file, its multipart children and sidecar removed
//   AbortMultipartUpload       over the masters' sockets (a bulk delete's keys in parallel);
//   CopyObject              -> the source read into a slot (decrypted / re-encrypted under
//                              SSE, multipart sources concatenated there) and written back;
//   aws-chunked PUT         -> the chunk framing decoded from the socket into the slot, each
//                              chunk's signature checked against the seed-signature chain;
//   presigned URLs          -> query-string SigV4 (X-Amz-Credential/-Signature/-Expires).
// Everything else — bucket create/delete, policies, STS, errors this path does not model, any
// case it does not own — is handed, unchanged, to the Python gateway (aiohttp on a private
// UNIX socket, tests/models/s3_gateway.py), which keeps the reference semantics.
// Signed requests are verified here with csrc/sigv4.cpp (static credentials); anything
// that does not verify is handed over too, so Python produces the exact error and audit
// record. Native requests of an authenticated gateway send their audit record to the
// gateway's audit store over the same datagram socket the Python workers use, so one hash
// chain covers both.
//
// Concurrency: one epoll thread accepts and watches idle keep-alive connections
// (EPOLLONESHOT); a ready connection is handed to a worker thread, which serves its
// requests with blocking I/O (the DFS calls block) and re-arms it when it goes idle.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "client_fast.h"
#include "front_store.h"
#include "s3_policy.h"
#include "sts.h"
#include "tls.h"
#include "io_pool.h"

namespace dfs {

struct S3FrontConfig {
  std::string host = "0.0.0.0";
  int port = 9000;
  std::string backend;  // UNIX socket path of the Python gateway
  int workers = 32;
  bool auth_enabled = false;
  std::string region = "us-east-1";
  std::string access_key, secret_key;  // EnvCredentialProvider (S3_ACCESS_KEY / S3_SECRET_KEY)
  bool allow_unsigned_payload = true;
  bool require_tls = false;  // S3_REQUIRE_TLS: an authenticated request over plain HTTP is refused
  std::string audit_socket;  // datagram socket of the audit store ("" = no audit)
  bool sse_enabled = false;  // SSE-S3: objects are stored encrypted
  std::string sse_kek;       // the 32-byte KEK (SSE_MASTER_KEY): encryption here; empty: Python does it
  bool metadata_sidecar = false;
  // several gateway processes on one port (S3_WORKERS > 1): the listening socket is bound with
  // SO_REUSEPORT and the kernel spreads the connections over the processes
  bool reuse_port = false;
  // 8-byte shared counter the gateway's workers bump on every PutBucketPolicy /
  // DeleteBucketPolicy ("" = none): a change empties the front's policy cache at once
  std::string policy_epoch_path;
  // TLS terminated by the front itself (reference main.rs:263-274 binds rustls): PEM files
  std::string tls_cert, tls_key;
  // STS sessions verified here: the token keys by KID (StsTokenManager) and the IAM role
  // configuration (IAM_CONFIG_PATH document) that decides what a session may do
  std::map<uint32_t, std::string> sts_keys;
  std::string iam_config;
  // STS issuance in the front (a gateway without the Python workers, backend == ""): the
  // OIDC issuer and client id (OIDC_ISSUER_URL / OIDC_CLIENT_ID), HS256 test issuers, the CA
  // for an https issuer, and the KID new session tokens are sealed with
  std::string oidc_issuer, oidc_client_id, oidc_ca;
  bool oidc_allow_hs256 = false;
  uint32_t sts_active_kid = 1;
};

struct S3FrontStats {
  uint64_t connections = 0, requests = 0, native = 0, proxied = 0;
  uint64_t puts = 0, parts = 0, gets = 0, range_gets = 0, heads = 0, mpu_gets = 0;
  uint64_t bytes_in = 0, bytes_out = 0, auth_native = 0, audit_sent = 0, audit_dropped = 0;
  uint64_t policy_native = 0;  // requests on a bucket with a policy, evaluated here and served natively
  std::map<std::string, uint64_t> by_status;  // "METHOD status" -> count (native requests)
  std::map<std::string, uint64_t> proxy_reasons;
  // native GET/Range GET phases, summed microseconds: metadata stat, block read into the
  // slot, response send (where a GET's latency goes)
  uint64_t get_stat_us = 0, get_read_us = 0, get_send_us = 0, get_timed = 0;
  uint64_t tls_handshakes = 0, tls_failures = 0, sse_puts = 0, sse_gets = 0, iam_native = 0, lists = 0, mpu_completes = 0, mpu_initiates = 0;
  uint64_t deletes = 0, multi_deletes = 0, deleted_keys = 0, mpu_aborts = 0, copies = 0, copy_bytes = 0;
  uint64_t chunked_puts = 0, chunk_sigs = 0, chunk_sig_failures = 0, presigned = 0, bucket_ops = 0;
  uint64_t sidecar_reads = 0, sidecar_writes = 0;  // the reference's <key>.meta files
  // a gateway without Python workers: the IAM metrics the workers would export
  std::map<std::string, uint64_t> auth_results;  // "success|none", "failure|<error_type>"
  std::map<std::string, uint64_t> sts_results;   // "success|none", "failure|<code>"
  std::map<std::string, uint64_t> policy_results;  // "allow|s3:GetObject", "deny|s3:DeleteObject"
  std::map<std::string, uint64_t> oidc_results;  // "success", "failure"
  uint64_t sts_issued = 0, standalone_answers = 0;
  // answers of the executable gateway's own fallback path (errors, /health, /metrics) by the
  // reason a hosted front would have handed the request over for; never a hand-off
  std::map<std::string, uint64_t> standalone_reasons;
};

class S3Front {
 public:
  S3Front(S3FrontConfig cfg, FastClient* fc);     // co-located gateway
  S3Front(S3FrontConfig cfg, FrontStore* store);  // any store (not owned), e.g. RemoteFrontStore
  ~S3Front();
  S3Front(const S3Front&) = delete;
  bool start(std::string* err);
  void stop();
  int port() const { return cfg_.port; }
  S3FrontStats stats();

  struct Conn;
  struct Req;

 private:
  void epoll_loop();
  void worker_loop();
  void serve(Conn* c);  // all requests until the connection goes idle or closes
  bool handle(Conn* c, Req& r);
  bool proxy(Conn* c, Req& r, const uint8_t* body, uint64_t body_len, const std::string& why);
  bool native_put(Conn* c, Req& r, const std::string& path, bool part);
  bool native_get(Conn* c, Req& r, const std::string& path, bool head);
  // the reference's sidecar `<path>.meta` ({"headers": {...}}): read for objects without
  // attributes; written too with S3_METADATA_SIDECAR=true (false: the store failed)
  bool read_sidecar(const std::string& path, const std::string& rid, std::map<std::string, std::string>* out);
  bool write_sidecar(const std::string& path, const std::map<std::string, std::string>& attrs, const std::string& rid);
  bool native_mpu_get(Conn* c, Req& r, const std::string& path, const std::string& marker_meta);
  bool sse_get(Conn* c, Req& r, const std::string& meta, uint64_t size, const std::string& hdrs,
               const std::string& dek_b64);
  struct Session {  // an authenticated STS session (empty role_arn: the static key)
    std::string role_arn, secret;
    s3policy::Context ctx;
  };
  int open_session(const std::string& token, Session* out);  // 1 open, 0 invalid, -1 expired
  bool authorize(Req& r, const std::string& bucket, const std::map<std::string, std::string>& q, std::string* user,
                 Session* sess, std::string* why);
  bool native_list(Conn* c, Req& r, const std::string& bucket, std::map<std::string, std::string>& q);
  // InitiateMultipartUpload: the upload's marker file and the UploadId, no Python.
  bool native_initiate(Conn* c, Req& r, const std::string& bucket, const std::string& key,
                       std::map<std::string, std::string>& q);
  bool native_complete(Conn* c, Req& r, const std::string& bucket, const std::string& key,
                       std::map<std::string, std::string>& q);
  bool native_delete(Conn* c, Req& r, const std::string& path);
  bool native_abort(Conn* c, Req& r, const std::string& upload_id);
  bool native_delete_objects(Conn* c, Req& r, const std::string& bucket, std::map<std::string, std::string>& q);
  bool native_copy(Conn* c, Req& r, const std::string& dest);
  // Bucket-level requests: CreateBucket, HeadBucket, DeleteBucket, GetBucketLocation and
  // Get/Put/DeleteBucketPolicy; ListBuckets at the root.
  bool native_bucket(Conn* c, Req& r, const std::string& bucket, std::map<std::string, std::string>& q);
  bool native_list_buckets(Conn* c, Req& r);
  // Reads an aws-chunked body (Content-Length framed) into dst (cap bytes): 1 ok (*n = decoded
  // bytes), 0 connection error, -1 bad framing or a chunk signature that does not chain.
  int read_aws_chunked(Conn* c, Req& r, uint8_t* dst, uint64_t cap, uint64_t* n);
  // A response with an S3 XML body (or none); counts it as a native request.
  bool respond(Conn* c, Req& r, int status, const std::string& xml, const std::string& extra = "");
  bool s3_error(Conn* c, Req& r, int status, const std::string& code, const std::string& msg,
                const std::string& resource = "");
  int verify_auth(Req& r, std::string* user, Session* sess);  // 1 ok, 0 hand over
  // A front without a Python backend answers what it would hand over: the auth error, the
  // S3 error or the STS exchange, as tests/models/s3_gateway.py does.
  bool standalone(Conn* c, Req& r, const uint8_t* body, uint64_t n, const std::string& why);
  bool auth_error(Conn* c, Req& r);
  bool native_sts(Conn* c, Req& r, std::map<std::string, std::string>& q);
  // The bucket's policy: *known = false when it could not be read (the request is handed
  // over); a null pointer when the bucket has none (or an unparsable one, which the gateway
  // ignores too).
  std::shared_ptr<const s3policy::BucketPolicy> bucket_policy(const std::string& bucket, bool* known);
  void audit(const Conn* c, const Req& r, const std::string& user, int status, const std::string& role_arn = "",
             const std::string& error_code = "", const std::string& action = "", const std::string& resource = "");
  void count(const Req& r, int status);
  int backend_conn();
  void backend_done(int fd, bool reuse);
  void note_proxy(const std::string& why);
  std::string native_metrics();

  S3FrontConfig cfg_;
  std::unique_ptr<FrontStore> own_store_;  // the FastClient adapter
  FrontStore* fc_;
  std::shared_ptr<TlsContext> tls_;
  std::map<uint32_t, std::string> sts_keys_;
  std::unique_ptr<s3policy::IamPolicy> iam_;
  std::unique_ptr<sts::OidcValidator> oidc_;
  int lfd_ = -1, epfd_ = -1, evfd_ = -1, audit_fd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread epoller_;
  std::vector<std::thread> workers_;
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<Conn*> ready_;
  std::mutex conns_mu_;
  std::map<int, Conn*> conns_;
  std::mutex be_mu_;
  std::vector<int> be_idle_;
  std::mutex pol_mu_;
  // bucket -> (expiry, policy or null); the gateway's 1 s policy cache
  std::map<std::string, std::pair<double, std::shared_ptr<const s3policy::BucketPolicy>>> policy_cache_;
  static constexpr size_t kPolicyCacheMax = 4096;  // entries; the cache is emptied beyond this
  uint64_t cache_epoch_ = 0;                        // pol_mu_: epoch the cached entries belong to
  uint64_t* epoch_map_ = nullptr;                   // mmap of cfg_.policy_epoch_path (shared, writable)
  uint64_t policy_epoch() const { return epoch_map_ ? __atomic_load_n(epoch_map_, __ATOMIC_ACQUIRE) : 0; }
  // A bucket policy changed here: bump the shared epoch (every gateway process drops its
  // cached policies) and this front's own cache.
  void policy_changed();

 public:
  void drop_policies();  // the in-process form of an epoch bump

 private:
  std::mutex key_mu_;
  std::map<std::string, std::string> key_cache_;  // date -> signing key (the single static key)
  IoPool pool_{4};
  std::mutex st_mu_;
  S3FrontStats st_;
};

}  // namespace dfs
