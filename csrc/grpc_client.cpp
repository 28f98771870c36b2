// Native gRPC client on nghttp2; design notes in grpc_client.h.
#include "grpc_client.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "tls.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

std::string percent_decode(const uint8_t* p, size_t n) {
  std::string o;
  o.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    int hi, lo;
    if (p[i] == '%' && i + 2 < n && (hi = hexval(static_cast<char>(p[i + 1]))) >= 0 &&
        (lo = hexval(static_cast<char>(p[i + 2]))) >= 0) {
      o.push_back(static_cast<char>(hi * 16 + lo));
      i += 2;
    } else {
      o.push_back(static_cast<char>(p[i]));
    }
  }
  return o;
}

std::string strip_scheme(const std::string& t) {
  for (const char* s : {"http://", "https://"})
    if (t.compare(0, std::strlen(s), s) == 0) return t.substr(std::strlen(s));
  return t;
}

nghttp2_nv nv(const std::string& name, const std::string& value) {
  return {reinterpret_cast<uint8_t*>(const_cast<char*>(name.data())),
          reinterpret_cast<uint8_t*>(const_cast<char*>(value.data())), name.size(), value.size(),
          NGHTTP2_NV_FLAG_NO_COPY_NAME | NGHTTP2_NV_FLAG_NO_COPY_VALUE};
}

int connect_to(const std::string& hostport, int timeout_ms, std::string* err) {
  size_t colon = hostport.rfind(':');
  if (colon == std::string::npos) {
    *err = "bad target " + hostport;
    return -1;
  }
  std::string host = hostport.substr(0, colon), port = hostport.substr(colon + 1);
  if (host.size() > 1 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  addrinfo hints{}, *res = nullptr;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_family = AF_UNSPEC;
  if (int rc = ::getaddrinfo(host.c_str(), port.c_str(), &hints, &res); rc != 0) {
    *err = std::string("resolve ") + hostport + ": " + gai_strerror(rc);
    return -1;
  }
  int fd = -1;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, ai->ai_protocol);
    if (fd < 0) continue;
    int rc = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      int soerr = 0;
      socklen_t sl = sizeof soerr;
      if (::poll(&p, 1, timeout_ms) == 1 && ::getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) == 0 && soerr == 0)
        rc = 0;
      else
        errno = soerr ? soerr : ETIMEDOUT;
    }
    if (rc == 0) break;
    *err = "connect " + hostport + ": " + std::strerror(errno);
    ::close(fd);
    fd = -1;
  }
  ::freeaddrinfo(res);
  if (fd < 0) return -1;
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int buf = 4 << 20;
  ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
  return fd;
}

}  // namespace

struct GrpcChannelPool::Conn {
  int fd = -1;
  std::unique_ptr<TlsConn> tls;  // TLS session on fd (https targets)
  nghttp2_session* s = nullptr;
  std::string authority;
  // the call in flight
  int32_t sid = -1;
  // request: 5-byte gRPC prefix + the caller's message (not copied; valid during the call)
  char prefix[5];
  const std::string* req = nullptr;
  size_t off = 0;       // bytes of prefix + *req written to the socket
  size_t read_off = 0;  // bytes of prefix + *req scheduled into DATA frames
  // response: its prefix kept apart, so the message is moved out, not copied
  char head[5];
  size_t head_len = 0;
  std::string in;
  bool closed = false, reset = false;
  int grpc_status = -1;
  std::string grpc_message;
  Clock::time_point deadline;

  ~Conn() {
    if (s) nghttp2_session_del(s);
    tls.reset();
    if (fd >= 0) ::close(fd);
  }

  static ssize_t on_send(nghttp2_session*, const uint8_t* data, size_t len, int, void* user) {
    auto* c = static_cast<Conn*>(user);
    if (c->tls) return c->tls->write_all(data, len, c->deadline) ? static_cast<ssize_t>(len) : NGHTTP2_ERR_CALLBACK_FAILURE;
    // the socket is non-blocking: wait for room until the call's deadline
    size_t done = 0;
    while (done < len) {
      ssize_t r = ::send(c->fd, data + done, len - done, MSG_NOSIGNAL);
      if (r > 0) {
        done += static_cast<size_t>(r);
      } else if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        int ms = static_cast<int>(
            std::chrono::duration_cast<std::chrono::milliseconds>(c->deadline - Clock::now()).count());
        pollfd p{c->fd, POLLOUT, 0};
        if (ms <= 0 || ::poll(&p, 1, ms) <= 0) return NGHTTP2_ERR_CALLBACK_FAILURE;
      } else if (r < 0 && errno == EINTR) {
        continue;
      } else {
        return NGHTTP2_ERR_CALLBACK_FAILURE;
      }
    }
    return static_cast<ssize_t>(len);
  }

  static int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t namelen,
                       const uint8_t* value, size_t valuelen, uint8_t, void* user) {
    auto* c = static_cast<Conn*>(user);
    if (f->hd.stream_id != c->sid) return 0;
    std::string n(reinterpret_cast<const char*>(name), namelen);
    if (n == "grpc-status") c->grpc_status = std::atoi(std::string(reinterpret_cast<const char*>(value), valuelen).c_str());
    else if (n == "grpc-message") c->grpc_message = percent_decode(value, valuelen);
    return 0;
  }

  static int on_data(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* user) {
    auto* c = static_cast<Conn*>(user);
    if (sid != c->sid) return 0;
    if (c->head_len < 5) {
      const size_t k = std::min<size_t>(5 - c->head_len, len);
      std::memcpy(c->head + c->head_len, data, k);
      c->head_len += k;
      data += k;
      len -= k;
      if (c->head_len == 5) {
        uint32_t n;
        std::memcpy(&n, c->head + 1, 4);
        c->in.reserve(std::min<uint32_t>(ntohl(n), 1u << 30));
      }
    }
    c->in.append(reinterpret_cast<const char*>(data), len);
    return 0;
  }

  static int on_close(nghttp2_session*, int32_t sid, uint32_t error_code, void* user) {
    auto* c = static_cast<Conn*>(user);
    if (sid == c->sid) {
      c->closed = true;
      c->reset = error_code != NGHTTP2_NO_ERROR;
    }
    return 0;
  }

  // The request body goes out without a copy into nghttp2's buffer (NGHTTP2_DATA_FLAG_NO_COPY):
  // read_body only sizes each DATA frame, send_data writes the frame header plus the prefix /
  // message bytes straight from the caller's buffer with one writev. With read_length the
  // frames are as large as the peer allows (1 MiB here) instead of nghttp2's default 16 KiB,
  // so a 1 MiB WriteBlock is one or two frames and syscalls, not 64 of each.
  static ssize_t read_body(nghttp2_session*, int32_t, uint8_t*, size_t len, uint32_t* flags, nghttp2_data_source*,
                           void* user) {
    auto* c = static_cast<Conn*>(user);
    if (!c->req) {  // a stream of an earlier call (never expected: calls end with their stream)
      *flags |= NGHTTP2_DATA_FLAG_EOF;
      return 0;
    }
    const size_t total = 5 + c->req->size();
    const size_t n = std::min(len, total - c->read_off);
    c->read_off += n;
    *flags |= NGHTTP2_DATA_FLAG_NO_COPY;
    if (c->read_off == total) *flags |= NGHTTP2_DATA_FLAG_EOF;
    return static_cast<ssize_t>(n);
  }

  static ssize_t read_length(nghttp2_session*, uint8_t, int32_t, int32_t session_window, int32_t stream_window,
                             uint32_t remote_max_frame, void*) {
    int64_t n = std::min<int64_t>({session_window, stream_window, static_cast<int64_t>(remote_max_frame)});
    return static_cast<ssize_t>(std::max<int64_t>(n, 1));
  }

  bool writev_all(iovec* iv, int k) {
    if (tls) {
      for (int i = 0; i < k; ++i)
        if (iv[i].iov_len && !tls->write_all(static_cast<const uint8_t*>(iv[i].iov_base), iv[i].iov_len, deadline))
          return false;
      return true;
    }
    while (k > 0) {
      // sendmsg, not writev: a peer that closed the connection must fail the call with EPIPE,
      // not raise SIGPIPE in the calling process (the unit tests' dead-server case)
      msghdr mh{};
      mh.msg_iov = iv;
      mh.msg_iovlen = static_cast<size_t>(k);
      ssize_t r = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
      if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        int ms = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count());
        pollfd p{fd, POLLOUT, 0};
        if (ms <= 0 || ::poll(&p, 1, ms) <= 0) return false;
        continue;
      }
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) return false;
      size_t done = static_cast<size_t>(r);
      while (k > 0 && done >= iv[0].iov_len) {
        done -= iv[0].iov_len;
        ++iv;
        --k;
      }
      if (k > 0) {
        iv[0].iov_base = static_cast<uint8_t*>(iv[0].iov_base) + done;
        iv[0].iov_len -= done;
      }
    }
    return true;
  }

  static int send_data(nghttp2_session*, nghttp2_frame* f, const uint8_t* framehd, size_t length,
                       nghttp2_data_source*, void* user) {
    auto* c = static_cast<Conn*>(user);
    if (!c->req || f->data.padlen > 0) return NGHTTP2_ERR_CALLBACK_FAILURE;  // no padding is ever selected
    iovec iv[3];
    int k = 0;
    iv[k++] = {const_cast<uint8_t*>(framehd), 9};
    size_t off = c->off, rem = length;
    if (off < 5 && rem) {
      const size_t m = std::min(rem, 5 - off);
      iv[k++] = {c->prefix + off, m};
      off += m;
      rem -= m;
    }
    if (rem) {
      iv[k++] = {const_cast<char*>(c->req->data()) + (off - 5), rem};
      off += rem;
    }
    if (!c->writev_all(iv, k)) return NGHTTP2_ERR_CALLBACK_FAILURE;
    c->off = off;
    return 0;
  }

  bool init(std::string* err) {
    nghttp2_session_callbacks* cb;
    nghttp2_session_callbacks_new(&cb);
    nghttp2_session_callbacks_set_send_callback(cb, &Conn::on_send);
    nghttp2_session_callbacks_set_on_header_callback(cb, &Conn::on_header);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cb, &Conn::on_data);
    nghttp2_session_callbacks_set_on_stream_close_callback(cb, &Conn::on_close);
    nghttp2_session_callbacks_set_send_data_callback(cb, &Conn::send_data);
    nghttp2_session_callbacks_set_data_source_read_length_callback(cb, &Conn::read_length);
    int rc = nghttp2_session_client_new(&s, cb, this);
    nghttp2_session_callbacks_del(cb);
    if (rc != 0) {
      *err = "nghttp2 session";
      return false;
    }
    nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_ENABLE_PUSH, 0},
                                   {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 64u << 20},
                                   {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 20}};
    if (nghttp2_submit_settings(s, NGHTTP2_FLAG_NONE, iv, 3) != 0 ||
        nghttp2_session_set_local_window_size(s, NGHTTP2_FLAG_NONE, 0, 1 << 30) != 0) {
      *err = "nghttp2 settings";
      return false;
    }
    return true;
  }

  // Drive the session until our stream closes; false on transport failure / timeout.
  bool pump() {
    std::vector<uint8_t> buf(1 << 18);
    for (;;) {
      if (nghttp2_session_send(s) != 0) return false;
      if (closed) return true;
      int ms = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count());
      if (ms <= 0) return false;
      if (!(tls && tls->pending())) {  // decrypted bytes already buffered need no poll
        pollfd p{fd, POLLIN, 0};
        int pr = ::poll(&p, 1, ms);
        if (pr < 0 && errno == EINTR) continue;
        if (pr <= 0) return false;
      }
      ssize_t n;
      if (tls) {
        n = static_cast<ssize_t>(tls->read(buf.data(), buf.size()));
        if (n == 0) continue;  // the record is not complete yet
      } else {
        n = ::recv(fd, buf.data(), buf.size(), 0);
        if (n < 0 && (errno == EINTR || errno == EAGAIN)) continue;
      }
      if (n <= 0) return false;
      if (nghttp2_session_mem_recv(s, buf.data(), static_cast<size_t>(n)) < 0) return false;
    }
  }
};

GrpcChannelPool::GrpcChannelPool(int timeout_ms, std::shared_ptr<TlsContext> tls)
    : timeout_ms_(timeout_ms), tls_(std::move(tls)) {}
GrpcChannelPool::~GrpcChannelPool() = default;

uint64_t GrpcChannelPool::connects() const {
  std::lock_guard<std::mutex> g(mu_);
  return connects_;
}

std::unique_ptr<GrpcChannelPool::Conn> GrpcChannelPool::take(const std::string& target, int timeout_ms,
                                                             std::string* err) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& v = idle_[target];
    if (!v.empty()) {
      auto c = std::move(v.back());
      v.pop_back();
      return c;
    }
    ++connects_;
  }
  auto c = std::make_unique<Conn>();
  c->authority = strip_scheme(target);
  c->fd = connect_to(c->authority, timeout_ms, err);
  if (c->fd < 0) return nullptr;
  if (tls_) {
    c->tls = std::make_unique<TlsConn>(tls_, c->fd);
    std::string host = c->authority.substr(0, c->authority.rfind(':'));
    if (host.size() > 1 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
    if (!c->tls->handshake(host, Clock::now() + std::chrono::milliseconds(timeout_ms), err)) return nullptr;
  }
  if (!c->init(err)) return nullptr;
  return c;
}

void GrpcChannelPool::give(const std::string& target, std::unique_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(mu_);
  idle_[target].push_back(std::move(c));
}

void GrpcChannelPool::set_host_aliases(std::vector<std::pair<std::string, std::string>> aliases) {
  std::lock_guard<std::mutex> g(mu_);
  aliases_ = std::move(aliases);
}

std::string GrpcChannelPool::resolve(const std::string& target) const {
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& a : aliases_) {
    auto p = target.find(a.first);
    if (!a.first.empty() && p != std::string::npos) return target.substr(0, p) + a.second + target.substr(p + a.first.size());
  }
  return target;
}

GrpcResult GrpcChannelPool::call(const std::string& target_in, const std::string& path, const std::string& request,
                                 const std::string& request_id, int timeout_ms) {
  const std::string target = resolve(target_in);
  GrpcResult res;
  if (timeout_ms < 0) timeout_ms = timeout_ms_;
  std::string err;
  std::unique_ptr<Conn> c = take(target, timeout_ms, &err);
  if (!c) {
    res.message = err;
    return res;
  }
  c->deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
  c->prefix[0] = 0;
  uint32_t be = htonl(static_cast<uint32_t>(request.size()));
  std::memcpy(c->prefix + 1, &be, 4);
  c->req = &request;
  c->off = 0;
  c->read_off = 0;
  c->head_len = 0;
  c->in.clear();
  c->closed = c->reset = false;
  c->grpc_status = -1;
  c->grpc_message.clear();
  static const std::string k_m = ":method", v_m = "POST", k_s = ":scheme", v_s = "http", k_p = ":path",
                           k_a = ":authority", k_ct = "content-type", v_ct = "application/grpc", k_te = "te",
                           v_te = "trailers", k_ua = "user-agent", v_ua = "dfs-native-client/1",
                           k_rid = "x-request-id";
  static const std::string v_https = "https";
  std::vector<nghttp2_nv> h = {nv(k_m, v_m), nv(k_s, tls_ ? v_https : v_s), nv(k_p, path), nv(k_a, c->authority),
                               nv(k_ct, v_ct), nv(k_te, v_te), nv(k_ua, v_ua)};
  if (!request_id.empty()) h.push_back(nv(k_rid, request_id));
  nghttp2_data_provider dp;
  dp.source.ptr = nullptr;
  dp.read_callback = &Conn::read_body;
  c->sid = nghttp2_submit_request(c->s, nullptr, h.data(), h.size(), &dp, nullptr);
  if (c->sid < 0 || !c->pump()) {
    res.message = "transport failure calling " + path + " on " + target;
    return res;  // the connection is dropped
  }
  res.transport_ok = true;
  if (c->grpc_status < 0) {
    res.status = c->reset ? 14 : 13;  // UNAVAILABLE on a reset stream, else INTERNAL
    res.message = c->reset ? "stream reset" : "response without grpc-status";
  } else if (c->grpc_status != 0) {
    res.status = c->grpc_status;
    res.message = std::move(c->grpc_message);
  } else if (c->head_len < 5) {
    res.status = 13;
    res.message = "empty response";
  } else {
    uint32_t n;
    std::memcpy(&n, c->head + 1, 4);
    n = ntohl(n);
    if (c->head[0] != 0 || c->in.size() < static_cast<size_t>(n)) {
      res.status = 13;
      res.message = "malformed or compressed response";
    } else {
      c->in.resize(n);
      res.status = 0;
      res.message = std::move(c->in);
    }
  }
  std::string().swap(c->in);
  c->req = nullptr;
  if (!c->reset && nghttp2_session_want_read(c->s)) give(target, std::move(c));
  return res;
}

}  // namespace dfs
