// s3_load: a native HTTP/1.1 load generator for the S3 gateway (config 5). One keep-alive
// connection per client thread, requests back to back — the shape of the Python `requests`
// load generator in bench_configs.py, without an interpreter on the client side, so the
// numbers describe the gateway rather than the client.
//
//   s3_load --host 127.0.0.1 --port 9000 --op put|get|range|list|mpu|head|copy|rename|delete|
//                                              multidelete|chunked --bucket b --prefix p
//           [--key k] [--count N | --seconds S] --size BYTES --conc C [--range-size 65536]
//           [--verify] [--keys K] [--parts P] [--batch 100] [--chunk 65536]
//           [--tls] [--ak AK --sk SK [--token SESSION_TOKEN] [--region R]] [--sse]
//
// --seconds runs every thread for that long (keys cycle) instead of a fixed request count.
// --tls speaks HTTPS (the native front's own TLS; the certificate is not verified: a
// benchmark client). --ak/--sk sign every request with SigV4 (UNSIGNED-PAYLOAD, as the AWS
// SDKs do over TLS), with the STS session token when given; --sse asks for SSE-S3 on PUT.
// list: ListObjectsV2 of `--prefix` (req/s); mpu: initiate + P parts + complete per object
// (MB/s of object bytes). The S3A-shaped operations (Hadoop's S3AFileSystem over the gateway):
// head: HEAD of key i (getFileStatus); copy: CopyObject key i -> key i.cp; rename: CopyObject
// key i -> key i.mv then DELETE key i.mv (S3A's rename is copy + delete; the source stays so
// the phase can cycle); delete: DELETE key i.cp; multidelete: DeleteObjects of --batch keys
// i.cp (S3A's bulk delete of a directory; keys/s in "keys_per_s"); chunked: PUT with an
// aws-chunked body of --chunk byte chunks (STREAMING-AWS4-HMAC-SHA256-PAYLOAD with a
// chunk-signature chain when signing, STREAMING-UNSIGNED-PAYLOAD-TRAILER otherwise — what the
// AWS SDKs send over plain HTTP). Payload of object i: a xorshift stream seeded by i (`--verify`
// checks GET bodies against it). Prints one JSON object: ops, seconds, MB/s, req/s, p50/p99
// latency, errors.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "trace.h"
#include "sigv4.h"

namespace {

using Clock = std::chrono::steady_clock;

void fill(std::vector<char>& b, uint64_t seed) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  for (size_t i = 0; i < b.size(); i += 8) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    std::memcpy(b.data() + i, &x, std::min<size_t>(8, b.size() - i));
  }
}

struct Opts {
  std::string host = "127.0.0.1", op = "get", bucket = "bench", prefix = "nat", fixed_key;
  int port = 9000, conc = 10, parts = 4;
  uint64_t count = 100, size = 1 << 20, rsize = 65536, keys = 0, batch = 100, chunk = 65536;
  double seconds = 0;
  bool verify = false, tls = false, sse = false;
  std::string ak, sk, token, region = "us-east-1";
};

SSL_CTX* g_ssl = nullptr;

struct Conn {
  int fd = -1;
  SSL* ssl = nullptr;
  std::string buf;
  std::string etag;  // ETag header of the last response
  bool open(const Opts& o) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(o.port));
    ::inet_pton(AF_INET, o.host.c_str(), &a.sin_addr);
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) return false;
    if (!o.tls) return true;
    ssl = SSL_new(g_ssl);
    SSL_set_fd(ssl, fd);
    SSL_set_tlsext_host_name(ssl, o.host.c_str());
    return SSL_connect(ssl) == 1;
  }
  void close() {
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
      ssl = nullptr;
    }
    if (fd >= 0) ::close(fd);
    fd = -1;
  }
  ssize_t io_send(const char* p, size_t n) {
    if (ssl) {
      int w = SSL_write(ssl, p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
      return w > 0 ? w : -1;
    }
    return ::send(fd, p, n, MSG_NOSIGNAL);
  }
  ssize_t io_recv(char* p, size_t n) {
    if (ssl) {
      int r = SSL_read(ssl, p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
      return r > 0 ? r : -1;
    }
    return ::recv(fd, p, n, 0);
  }
  bool send_all(const char* p, size_t n) {
    while (n) {
      ssize_t w = io_send(p, n);
      if (w <= 0) return false;
      p += w;
      n -= static_cast<size_t>(w);
    }
    return true;
  }
  // Reads one response; returns the status (-1 on error); body into *body (if non-null).
  int response(std::string* body, bool no_body = false) {
    size_t end;
    char tmp[1 << 16];
    while ((end = buf.find("\r\n\r\n")) == std::string::npos) {
      ssize_t n = io_recv(tmp, sizeof tmp);
      if (n <= 0) return -1;
      buf.append(tmp, static_cast<size_t>(n));
    }
    std::string head = buf.substr(0, end);
    buf.erase(0, end + 4);
    int status = std::atoi(head.c_str() + head.find(' ') + 1);
    size_t clen = 0;
    etag.clear();
    for (size_t p = 0; (p = head.find("\r\n", p)) != std::string::npos;) {
      p += 2;
      if (strncasecmp(head.c_str() + p, "content-length:", 15) == 0) clen = std::strtoull(head.c_str() + p + 15, nullptr, 10);
      if (strncasecmp(head.c_str() + p, "etag:", 5) == 0) {
        size_t e = head.find("\r\n", p);
        etag = head.substr(p + 5, (e == std::string::npos ? head.size() : e) - p - 5);
        etag.erase(0, etag.find_first_not_of(' '));
      }
    }
    if (no_body || status == 204) clen = 0;  // HEAD, 204: no body follows the head
    std::string sink;
    std::string* out = body ? body : &sink;
    out->resize(clen);
    size_t have = std::min(clen, buf.size());
    std::memcpy(out->data(), buf.data(), have);
    buf.erase(0, have);
    while (have < clen) {
      ssize_t n = io_recv(out->data() + have, clen - have);
      if (n <= 0) return -1;
      have += static_cast<size_t>(n);
    }
    return status;
  }
};

// SigV4 request headers (UNSIGNED-PAYLOAD) for one request; "" when no credentials.
struct Signer {
  const Opts& o;
  std::mutex mu;
  std::string day, key;
  explicit Signer(const Opts& opts) : o(opts) {}
  std::string headers(const std::string& method, const std::string& path, const std::string& query,
                      uint64_t content_length, bool sse_header,
                      const std::vector<std::pair<std::string, std::string>>& extra = {},
                      const std::string& payload = "UNSIGNED-PAYLOAD", dfs::sigv4::ChunkChain* seed = nullptr) {
    std::string h = "Host: " + o.host + ":" + std::to_string(o.port) + "\r\n";
    if (sse_header) h += "x-amz-server-side-encryption: AES256\r\n";
    if (method == "PUT" || method == "POST") h += "Content-Length: " + std::to_string(content_length) + "\r\n";
    for (auto& kv : extra) h += kv.first + ": " + kv.second + "\r\n";
    if (o.ak.empty()) {
      if (payload != "UNSIGNED-PAYLOAD") h += "x-amz-content-sha256: " + payload + "\r\n";
      return h;
    }
    char amz[32], date[16];
    std::time_t now = std::time(nullptr);
    std::tm t;
    gmtime_r(&now, &t);
    std::strftime(amz, sizeof amz, "%Y%m%dT%H%M%SZ", &t);
    std::strftime(date, sizeof date, "%Y%m%d", &t);
    std::string k;
    {
      std::lock_guard<std::mutex> g(mu);
      if (day != date) {
        day = date;
        key = dfs::sigv4::signing_key(o.sk, date, o.region, "s3");
      }
      k = key;
    }
    dfs::sigv4::Request r;
    r.method = method;
    r.path = path;
    r.query = query;
    r.payload_hash = payload;
    r.headers.emplace_back("host", o.host + ":" + std::to_string(o.port));
    r.headers.emplace_back("x-amz-content-sha256", payload);
    r.headers.emplace_back("x-amz-date", amz);
    if (!o.token.empty()) r.headers.emplace_back("x-amz-security-token", o.token);
    if (sse_header) r.headers.emplace_back("x-amz-server-side-encryption", "AES256");
    for (auto& kv : extra) r.headers.emplace_back(kv.first, kv.second);
    std::sort(r.headers.begin(), r.headers.end());
    for (auto& kv : r.headers) r.signed_headers += (r.signed_headers.empty() ? "" : ";") + kv.first;
    const std::string scope = std::string(date) + "/" + o.region + "/s3/aws4_request";
    const std::string sig =
        dfs::sigv4::signature(k, dfs::sigv4::string_to_sign(amz, scope, dfs::sigv4::canonical_request(r)));
    if (seed) *seed = dfs::sigv4::ChunkChain{k, amz, scope, sig};  // what an aws-chunked body continues
    h += "x-amz-content-sha256: " + payload + "\r\nx-amz-date: " + std::string(amz) + "\r\n";
    if (!o.token.empty()) h += "x-amz-security-token: " + o.token + "\r\n";
    h += "Authorization: AWS4-HMAC-SHA256 Credential=" + o.ak + "/" + scope + ", SignedHeaders=" + r.signed_headers +
         ", Signature=" + sig + "\r\n";
    return h;
  }
};

std::string xml_text(const std::string& body, const std::string& tag) {
  size_t a = body.find("<" + tag + ">");
  if (a == std::string::npos) return "";
  a += tag.size() + 2;
  size_t b = body.find("</" + tag + ">", a);
  return b == std::string::npos ? "" : body.substr(a, b - a);
}

}  // namespace

int main(int argc, char** argv) {
  dfs::trace_init();  // before any thread: roctx's first range calls setenv (trace.h)
  Opts o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto nxt = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--host") o.host = nxt();
    else if (a == "--port") o.port = std::atoi(nxt().c_str());
    else if (a == "--op") o.op = nxt();
    else if (a == "--bucket") o.bucket = nxt();
    else if (a == "--prefix") o.prefix = nxt();
    else if (a == "--key") o.fixed_key = nxt();  // every request on this one key (e.g. a multipart object)
    else if (a == "--count") o.count = std::strtoull(nxt().c_str(), nullptr, 10);
    else if (a == "--seconds") o.seconds = std::strtod(nxt().c_str(), nullptr);
    else if (a == "--size") o.size = std::strtoull(nxt().c_str(), nullptr, 10);
    else if (a == "--conc") o.conc = std::atoi(nxt().c_str());
    else if (a == "--range-size") o.rsize = std::strtoull(nxt().c_str(), nullptr, 10);
    else if (a == "--verify") o.verify = true;
    else if (a == "--keys") o.keys = std::strtoull(nxt().c_str(), nullptr, 10);  // request i -> key i % keys
    else if (a == "--parts") o.parts = std::max(1, std::atoi(nxt().c_str()));
    else if (a == "--batch") o.batch = std::max<uint64_t>(1, std::strtoull(nxt().c_str(), nullptr, 10));
    else if (a == "--chunk") o.chunk = std::max<uint64_t>(1, std::strtoull(nxt().c_str(), nullptr, 10));
    else if (a == "--tls") o.tls = true;
    else if (a == "--sse") o.sse = true;
    else if (a == "--ak") o.ak = nxt();
    else if (a == "--sk") o.sk = nxt();
    else if (a == "--token") o.token = nxt();
    else if (a == "--region") o.region = nxt();
  }
  if (o.keys == 0) o.keys = o.count;
  if (o.tls) {
    g_ssl = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_verify(g_ssl, SSL_VERIFY_NONE, nullptr);
  }
  Signer signer(o);
  // Payloads are generated before the clock starts (PUT bodies, and the expected bytes of a
  // verified GET): generating 1 MiB of xorshift per request inside the timed loop costs the
  // client ~0.5 ms, which would be measured as gateway latency. Falls back to per-request
  // generation when the key set is too large to hold.
  std::vector<std::vector<char>> cache;
  const bool need = o.op == "put" || o.op == "chunked" || o.op == "mpu" || (o.verify && o.fixed_key.empty());
  const uint64_t ncache = o.op == "mpu" ? 1 : o.keys;
  if (need && ncache * o.size <= (4ull << 30)) {
    cache.resize(ncache);
    for (uint64_t k = 0; k < ncache; ++k) {
      cache[k].resize(o.size);
      fill(cache[k], k);
    }
  }
  std::vector<std::vector<double>> lat(o.conc);
  std::atomic<uint64_t> errors{0}, bytes{0}, keys_deleted{0};
  std::mutex err_mu;
  std::string first_error;
  auto note_error = [&](const std::string& e) {
    errors++;
    std::lock_guard<std::mutex> g(err_mu);
    if (first_error.empty()) first_error = e;
  };
  const auto t0 = Clock::now();
  const auto stop_at = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(o.seconds));
  std::vector<std::thread> th;
  for (int t = 0; t < o.conc; ++t)
    th.emplace_back([&, t] {
      Conn c;
      if (!c.open(o)) {
        note_error("connect failed");
        return;
      }
      std::vector<char> payload(o.size);
      std::string body;
      for (uint64_t i = static_cast<uint64_t>(t);; i += static_cast<uint64_t>(o.conc)) {
        if (o.seconds > 0 ? Clock::now() >= stop_at : i >= o.count) break;
        char key[96];
        if (o.fixed_key.empty())
          std::snprintf(key, sizeof key, "%s_%05llu", o.prefix.c_str(), static_cast<unsigned long long>(i % o.keys));
        else
          std::snprintf(key, sizeof key, "%s", o.fixed_key.c_str());
        const std::string path = "/" + o.bucket + "/" + key;
        auto s0 = Clock::now();
        int st = -1;
        if (o.op == "put") {
          const char* src = payload.data();
          if (!cache.empty()) src = cache[i % o.keys].data();
          else fill(payload, i % o.keys);
          std::string req = "PUT " + path + " HTTP/1.1\r\n" + signer.headers("PUT", path, "", o.size, o.sse) + "\r\n";
          st = c.send_all(req.data(), req.size()) && c.send_all(src, o.size) ? c.response(&body) : -1;
          if (st == 200) bytes += o.size;
        } else if (o.op == "chunked") {
          // aws-chunked body: <hex>[;chunk-signature=<64 hex>]\r\n<data>\r\n ... 0[;sig]\r\n\r\n
          const char* src = payload.data();
          if (!cache.empty()) src = cache[i % o.keys].data();
          else fill(payload, i % o.keys);
          const bool sign = !o.ak.empty();
          const size_t sig_len = sign ? 17 + 64 : 0;  // ";chunk-signature=" + signature
          uint64_t enc = 1 + sig_len + 4;             // the final empty chunk and the closing CRLF
          char hx[24];
          for (uint64_t off = 0; off < o.size; off += o.chunk) {
            const uint64_t len = std::min<uint64_t>(o.chunk, o.size - off);
            enc += static_cast<uint64_t>(std::snprintf(hx, sizeof hx, "%llx", static_cast<unsigned long long>(len))) +
                   sig_len + 2 + len + 2;
          }
          dfs::sigv4::ChunkChain chain;
          std::string req = "PUT " + path + " HTTP/1.1\r\n" +
                            signer.headers("PUT", path, "", enc, false,
                                           {{"content-encoding", "aws-chunked"},
                                            {"x-amz-decoded-content-length", std::to_string(o.size)}},
                                           sign ? "STREAMING-AWS4-HMAC-SHA256-PAYLOAD" : "STREAMING-UNSIGNED-PAYLOAD-TRAILER",
                                           &chain) +
                            "\r\n";
          std::string b;
          b.reserve(enc);
          auto piece = [&](const char* p, uint64_t len) {
            std::snprintf(hx, sizeof hx, "%llx", static_cast<unsigned long long>(len));
            b += hx;
            if (sign) b += ";chunk-signature=" + chain.next(p, len);
            b += "\r\n";
            b.append(p, len);
            b += "\r\n";
          };
          for (uint64_t off = 0; off < o.size; off += o.chunk) piece(src + off, std::min<uint64_t>(o.chunk, o.size - off));
          piece(src, 0);
          st = b.size() == enc && c.send_all(req.data(), req.size()) && c.send_all(b.data(), b.size()) ? c.response(&body) : -1;
          if (st == 200) bytes += o.size;
        } else if (o.op == "head") {
          std::string req = "HEAD " + path + " HTTP/1.1\r\n" + signer.headers("HEAD", path, "", 0, false) + "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body, true) : -1;
        } else if (o.op == "copy" || o.op == "rename") {
          const std::string dst = path + (o.op == "copy" ? ".cp" : ".mv");
          std::string req = "PUT " + dst + " HTTP/1.1\r\n" +
                            signer.headers("PUT", dst, "", 0, false, {{"x-amz-copy-source", path}}) + "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
          if (st == 200 && body.find("<CopyObjectResult") == std::string::npos) st = -5;
          if (st == 200 && o.op == "rename") {  // S3A rename: the copy, then the delete
            req = "DELETE " + dst + " HTTP/1.1\r\n" + signer.headers("DELETE", dst, "", 0, false) + "\r\n";
            st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
            if (st == 204) st = 200;
          }
          if (st == 200) bytes += o.size;
        } else if (o.op == "delete") {
          const std::string dst = path + ".cp";
          std::string req = "DELETE " + dst + " HTTP/1.1\r\n" + signer.headers("DELETE", dst, "", 0, false) + "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
          if (st == 204) st = 200;
        } else if (o.op == "multidelete") {
          std::string xml = "<Delete><Quiet>true</Quiet>";
          for (uint64_t j = 0; j < o.batch; ++j) {
            char k2[96];
            std::snprintf(k2, sizeof k2, "%s_%05llu.cp", o.prefix.c_str(),
                          static_cast<unsigned long long>((i * o.batch + j) % o.keys));
            xml += std::string("<Object><Key>") + k2 + "</Key></Object>";
          }
          xml += "</Delete>";
          const std::string bp = "/" + o.bucket;
          std::string req = "POST " + bp + "?delete= HTTP/1.1\r\n" +
                            signer.headers("POST", bp, "delete=", xml.size(), false) + "\r\n";
          st = c.send_all(req.data(), req.size()) && c.send_all(xml.data(), xml.size()) ? c.response(&body) : -1;
          if (st == 200 && body.find("<DeleteResult") == std::string::npos) st = -6;
          if (st == 200 && body.find("<Error>") != std::string::npos) st = -7;
          if (st == 200) keys_deleted += o.batch;
        } else if (o.op == "list") {
          const std::string q = "list-type=2&max-keys=1000&prefix=" + dfs::sigv4::uri_encode(o.prefix, true);
          std::string req = "GET /" + o.bucket + "?" + q + " HTTP/1.1\r\n" + signer.headers("GET", "/" + o.bucket, q, 0, false) +
                            "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
          if (st == 200 && body.find("<ListBucketResult") == std::string::npos) st = -3;
        } else if (o.op == "mpu") {
          // one multipart object per iteration: initiate, P parts, complete; each thread cycles
          // over --keys objects (a completion replaces the older object and frees its parts), so
          // a long window's live data stays bounded by threads x keys x object size
          char mkey[96];
          const uint64_t mk = o.keys > 0 ? i % o.keys : i;
          std::snprintf(mkey, sizeof mkey, "%s_mpu_%d_%llu", o.prefix.c_str(), t, static_cast<unsigned long long>(mk));
          const std::string mpath = "/" + o.bucket + "/" + mkey;
          std::string req = "POST " + mpath + "?uploads= HTTP/1.1\r\n" + signer.headers("POST", mpath, "uploads=", 0, o.sse) + "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
          std::string uid = st == 200 ? xml_text(body, "UploadId") : "";
          if (uid.empty()) {
            note_error("initiate: HTTP " + std::to_string(st));
            st = -1;
          } else {
            const uint64_t psz = (o.size + o.parts - 1) / o.parts;
            const char* src = cache.empty() ? payload.data() : cache[0].data();
            std::string xml = "<CompleteMultipartUpload>";
            for (int p = 0; p < o.parts && st == 200; ++p) {
              const uint64_t off = p * psz, len = std::min<uint64_t>(psz, o.size - off);
              const std::string q = "partNumber=" + std::to_string(p + 1) + "&uploadId=" + dfs::sigv4::uri_encode(uid, true);
              req = "PUT " + mpath + "?" + q + " HTTP/1.1\r\n" + signer.headers("PUT", mpath, q, len, false) + "\r\n";
              st = c.send_all(req.data(), req.size()) && c.send_all(src + off, len) ? c.response(&body) : -1;
              xml += "<Part><PartNumber>" + std::to_string(p + 1) + "</PartNumber><ETag>" + c.etag + "</ETag></Part>";
            }
            xml += "</CompleteMultipartUpload>";
            if (st == 200) {
              const std::string q = "uploadId=" + dfs::sigv4::uri_encode(uid, true);
              req = "POST " + mpath + "?" + q + " HTTP/1.1\r\n" + signer.headers("POST", mpath, q, xml.size(), false) + "\r\n";
              st = c.send_all(req.data(), req.size()) && c.send_all(xml.data(), xml.size()) ? c.response(&body) : -1;
              if (st == 200 && body.find("<CompleteMultipartUploadResult") == std::string::npos) st = -4;
            }
            if (st == 200) bytes += o.size;
          }
        } else {
          uint64_t off = 0, want = o.size;
          std::string extra;
          if (o.op == "range") {
            off = (i * 7919 * 4096) % (o.size - o.rsize);
            want = o.rsize;
            extra = "Range: bytes=" + std::to_string(off) + "-" + std::to_string(off + o.rsize - 1) + "\r\n";
          }
          std::string req = "GET " + path + " HTTP/1.1\r\n" + signer.headers("GET", path, "", 0, false) + extra + "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
          if ((st == 200 || st == 206) && body.size() == want) {
            bytes += want;
            if (o.verify && o.fixed_key.empty()) {
              const char* exp = payload.data();
              if (!cache.empty()) exp = cache[i % o.keys].data();
              else fill(payload, i % o.keys);
              if (std::memcmp(exp + off, body.data(), want) != 0) st = -2;
            }
          } else if (st > 0) {
            st = -st;
          }
        }
        if (st != 200 && st != 206) note_error(o.op + " " + key + ": status " + std::to_string(st) + " " + body.substr(0, 200));
        lat[t].push_back(std::chrono::duration<double>(Clock::now() - s0).count());
        if (st < 0 && (st > -2 || st < -7)) {  // connection state unknown: reconnect
          c.close();
          c.buf.clear();
          if (!c.open(o)) break;
        }
      }
      c.close();
    });
  for (auto& x : th) x.join();
  double secs = std::chrono::duration<double>(Clock::now() - t0).count();
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : 1e3 * all[std::min(all.size() - 1, size_t(all.size() * p))]; };
  std::string fe;
  for (char ch : first_error) fe += (ch == '"' || ch == '\\') ? '\'' : (ch < 32 ? ' ' : ch);
  std::printf("{\"op\": \"%s\", \"ops\": %zu, \"seconds\": %.4f, \"mb_per_s\": %.1f, \"req_per_s\": %.1f, "
              "\"p50_ms\": %.3f, \"p99_ms\": %.3f, \"keys_per_s\": %.1f, \"errors\": %llu, \"concurrency\": %d, \"size\": %llu, "
              "\"tls\": %s, \"signed\": %s, \"session\": %s, \"sse\": %s, \"first_error\": \"%s\"}\n",
              o.op.c_str(), all.size(), secs, bytes.load() / 1048576.0 / secs, all.size() / secs, pct(0.5), pct(0.99),
              keys_deleted.load() / secs,
              static_cast<unsigned long long>(errors.load()), o.conc, static_cast<unsigned long long>(o.size),
              o.tls ? "true" : "false", o.ak.empty() ? "false" : "true", o.token.empty() ? "false" : "true",
              o.sse ? "true" : "false", fe.c_str());
  if (g_ssl) SSL_CTX_free(g_ssl);
  return errors.load() ? 1 : 0;
}
