// Native gRPC server on nghttp2; design notes in grpc_server.h.
#include "grpc_server.h"
#include "thread_name.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <algorithm>
#include <cstring>
#include <map>

#include "tls.h"
#include "trace.h"

namespace dfs {

namespace {

bool writev_full(int fd, iovec* iv, int k) {
  while (k > 0) {
    msghdr mh{};
    mh.msg_iov = iv;
    mh.msg_iovlen = static_cast<size_t>(k);
    ssize_t r = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
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

bool write_full(int fd, const uint8_t* p, size_t n) {
  while (n > 0) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r > 0) {
      p += r;
      n -= static_cast<size_t>(r);
    } else if (r < 0 && errno == EINTR) {
      continue;
    } else {
      return false;
    }
  }
  return true;
}

// grpc-message is percent-encoded (gRPC over HTTP/2: printable ASCII except '%').
std::string percent_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7E && c != '%') {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

nghttp2_nv nv(const std::string& name, const std::string& value) {
  return {reinterpret_cast<uint8_t*>(const_cast<char*>(name.data())),
          reinterpret_cast<uint8_t*>(const_cast<char*>(value.data())), name.size(), value.size(),
          NGHTTP2_NV_FLAG_NONE};
}

}  // namespace

struct GrpcServer::Conn : std::enable_shared_from_this<Conn> {
  struct Stream {
    std::string path, rid;
    // request: the 5-byte gRPC prefix kept apart from the message, so the message moves to
    // the handler without a copy
    char head[5];
    size_t head_len = 0;
    std::string body;
    std::shared_ptr<uint8_t> ext;  // body from the server's allocator (body stays empty)
    size_t ext_len = 0;
    size_t received() const { return ext ? ext_len : body.size(); }
    // response: prefix + message, served by read_body without concatenating them
    char prefix[5];
    std::string out;
    std::shared_ptr<const void> keep;  // owner of body_p when the reply is external
    const uint8_t* body_p = nullptr;
    size_t body_n = 0;
    size_t off = 0;       // bytes of prefix + body written to the socket
    size_t read_off = 0;  // bytes of prefix + body scheduled into DATA frames
    std::string status_str = "0";
    bool dispatched = false;
    bool too_big = false;   // over kMaxMessage (or the connection's budget): refused
    uint32_t declared = 0;  // message length from the gRPC prefix
  };
  static constexpr uint32_t kMaxMessage = 100u << 20;       // MAX_GRPC_MESSAGE_SIZE of the reference
  static constexpr size_t kMaxConnBuffered = 1ull << 30;    // request bytes held per connection
  GrpcServer* srv = nullptr;
  int fd = -1;
  TlsConn* tc = nullptr;  // TLS session on fd (owned by serve())
  int efd = -1;
  size_t buffered = 0;  // request bytes buffered across this connection's streams
  nghttp2_session* session = nullptr;
  std::map<int32_t, Stream> streams;
  std::mutex mu;
  std::deque<std::pair<int32_t, GrpcReply>> done;

  ~Conn() {
    if (session) nghttp2_session_del(session);
    if (efd >= 0) ::close(efd);
  }

  void post(int32_t sid, GrpcReply r) {
    {
      std::lock_guard<std::mutex> g(mu);
      done.emplace_back(sid, std::move(r));
    }
    uint64_t one = 1;
    (void)!::write(efd, &one, sizeof one);
  }

  // Response bodies go out without a copy into nghttp2's buffer (NGHTTP2_DATA_FLAG_NO_COPY):
  // read_body sizes each DATA frame (up to the peer's max frame size via read_length), and
  // send_data writes header + prefix + body bytes straight from the reply buffer with one
  // sendmsg — a 1 MiB ReadBlock is one frame, not 64 frames of 16 KiB each copied twice.
  static ssize_t read_body(nghttp2_session* s, int32_t sid, uint8_t*, size_t len, uint32_t* flags,
                           nghttp2_data_source*, void* user) {
    auto* c = static_cast<Conn*>(user);
    auto it = c->streams.find(sid);
    if (it == c->streams.end()) return NGHTTP2_ERR_TEMPORAL_CALLBACK_FAILURE;
    Stream& st = it->second;
    const size_t total = 5 + st.body_n;
    const size_t n = std::min(len, total - st.read_off);
    st.read_off += n;
    *flags |= NGHTTP2_DATA_FLAG_NO_COPY;
    if (st.read_off == total) {
      *flags |= NGHTTP2_DATA_FLAG_EOF | NGHTTP2_DATA_FLAG_NO_END_STREAM;
      static const std::string k_status = "grpc-status";
      nghttp2_nv tr[] = {nv(k_status, st.status_str)};
      if (nghttp2_submit_trailer(s, sid, tr, 1) != 0) return NGHTTP2_ERR_CALLBACK_FAILURE;
    }
    return static_cast<ssize_t>(n);
  }

  static ssize_t read_length(nghttp2_session*, uint8_t, int32_t, int32_t session_window, int32_t stream_window,
                             uint32_t remote_max_frame, void*) {
    int64_t n = std::min<int64_t>({session_window, stream_window, static_cast<int64_t>(remote_max_frame)});
    return static_cast<ssize_t>(std::max<int64_t>(n, 1));
  }

  bool write_vec(iovec* iv, int k) {
    if (tc) {
      const auto far = std::chrono::steady_clock::now() + std::chrono::hours(24);
      for (int i = 0; i < k; ++i)
        if (iv[i].iov_len && !tc->write_all(static_cast<const uint8_t*>(iv[i].iov_base), iv[i].iov_len, far))
          return false;
      return true;
    }
    return writev_full(fd, iv, k);
  }

  static ssize_t on_send(nghttp2_session*, const uint8_t* data, size_t len, int, void* user) {
    iovec iv{const_cast<uint8_t*>(data), len};
    return static_cast<Conn*>(user)->write_vec(&iv, 1) ? static_cast<ssize_t>(len) : NGHTTP2_ERR_CALLBACK_FAILURE;
  }

  static int send_data(nghttp2_session*, nghttp2_frame* f, const uint8_t* framehd, size_t length,
                       nghttp2_data_source*, void* user) {
    auto* c = static_cast<Conn*>(user);
    auto it = c->streams.find(f->hd.stream_id);
    if (it == c->streams.end() || f->data.padlen > 0) return NGHTTP2_ERR_CALLBACK_FAILURE;
    Stream& st = it->second;
    iovec iv[3];
    int k = 0;
    iv[k++] = {const_cast<uint8_t*>(framehd), 9};
    size_t off = st.off, rem = length;
    if (off < 5 && rem) {
      const size_t m = std::min(rem, 5 - off);
      iv[k++] = {st.prefix + off, m};
      off += m;
      rem -= m;
    }
    if (rem) {
      iv[k++] = {const_cast<uint8_t*>(st.body_p) + (off - 5), rem};
      off += rem;
    }
    if (!c->write_vec(iv, k)) return NGHTTP2_ERR_CALLBACK_FAILURE;
    st.off = off;
    return 0;
  }

  void respond(int32_t sid, GrpcReply& r) {
    auto it = streams.find(sid);
    if (it == streams.end()) return;  // the client reset the stream meanwhile
    Stream& st = it->second;
    static const std::string k_status = ":status", v200 = "200", k_ct = "content-type", v_ct = "application/grpc",
                             k_gs = "grpc-status", k_gm = "grpc-message";
    if (r.status == 0) {
      st.prefix[0] = 0;
      if (r.ext) {
        st.keep = std::move(r.keep);
        st.body_p = r.ext;
        st.body_n = r.ext_len;
      } else {
        st.out = std::move(r.message);
        st.body_p = reinterpret_cast<const uint8_t*>(st.out.data());
        st.body_n = st.out.size();
      }
      uint32_t n = htonl(static_cast<uint32_t>(st.body_n));
      std::memcpy(st.prefix + 1, &n, 4);
      st.off = 0;
      st.read_off = 0;
      nghttp2_nv h[] = {nv(k_status, v200), nv(k_ct, v_ct)};
      nghttp2_data_provider dp;
      dp.source.ptr = nullptr;
      dp.read_callback = &Conn::read_body;
      nghttp2_submit_response(session, sid, h, 2, &dp);
    } else {
      // Trailers-Only response: status and message in the single HEADERS frame
      std::string code = std::to_string(r.status), msg = percent_encode(r.message);
      nghttp2_nv h[] = {nv(k_status, v200), nv(k_ct, v_ct), nv(k_gs, code), nv(k_gm, msg)};
      nghttp2_submit_response(session, sid, h, 4, nullptr);
    }
  }

  void dispatch(int32_t sid) {
    auto it = streams.find(sid);
    if (it == streams.end() || it->second.dispatched) return;
    Stream& st = it->second;
    st.dispatched = true;
    buffered -= std::min(buffered, st.received());
    GrpcReply bad;
    if (st.too_big) {
      bad = {8, "message larger than the " + std::to_string(kMaxMessage) + " byte limit"};
    } else if (st.head_len < 5) {
      bad = {13, "missing gRPC message"};
    } else if (st.head[0] != 0) {
      bad = {12, "compressed messages are not supported"};
    } else {
      uint32_t n;
      std::memcpy(&n, st.head + 1, 4);
      if (ntohl(n) != st.received()) bad = {13, "gRPC message length mismatch"};
    }
    if (bad.status) {
      respond(sid, bad);
      return;
    }
    auto call = std::make_shared<GrpcCall>();
    call->path = std::move(st.path);
    call->request_id = std::move(st.rid);
    if (st.ext) {
      call->body = st.ext.get();
      call->body_len = st.ext_len;
      call->body_keep = std::move(st.ext);
      st.ext_len = 0;
    } else {
      call->message = std::move(st.body);
      st.body = std::string();
    }
    auto self = shared_from_this();
    std::lock_guard<std::mutex> g(srv->mu_);
    srv->jobs_.emplace_back([self, sid, call] {
      GrpcReply r;
      try {
        r = self->srv->handler_(*call);
      } catch (const std::exception& e) {
        r = {13, std::string("internal error: ") + e.what()};
      }
      self->srv->calls_++;
      self->post(sid, std::move(r));
    });
    srv->cv_.notify_one();
  }

  // ---- nghttp2 callbacks
  static int on_begin_headers(nghttp2_session*, const nghttp2_frame* f, void* user) {
    if (f->hd.type == NGHTTP2_HEADERS && f->headers.cat == NGHTTP2_HCAT_REQUEST)
      static_cast<Conn*>(user)->streams[f->hd.stream_id];
    return 0;
  }
  static int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nlen,
                       const uint8_t* value, size_t vlen, uint8_t, void* user) {
    auto* c = static_cast<Conn*>(user);
    auto it = c->streams.find(f->hd.stream_id);
    if (it == c->streams.end()) return 0;
    std::string n(reinterpret_cast<const char*>(name), nlen);
    if (n == ":path") it->second.path.assign(reinterpret_cast<const char*>(value), vlen);
    else if (n == "x-request-id") it->second.rid.assign(reinterpret_cast<const char*>(value), vlen);
    return 0;
  }
  static int on_data(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* user) {
    auto* c = static_cast<Conn*>(user);
    auto it = c->streams.find(sid);
    if (it != c->streams.end()) {
      Stream& st = it->second;
      if (st.too_big) return 0;  // already refused: drop the rest of the upload
      if (st.head_len < 5) {
        const size_t k = std::min<size_t>(5 - st.head_len, len);
        std::memcpy(st.head + st.head_len, data, k);
        st.head_len += k;
        data += k;
        len -= k;
        if (st.head_len == 5) {
          uint32_t n;
          std::memcpy(&n, st.head + 1, 4);
          n = ntohl(n);
          // the reference's tonic servers cap messages at 100 MiB (RESOURCE_EXHAUSTED); the
          // buffer is sized from the prefix only once the prefix passed that check, and the
          // connection's buffered bytes stay under kMaxConnBuffered whatever the stream count
          if (n > kMaxMessage || c->buffered + n > kMaxConnBuffered) {
            c->refuse(st);
            return 0;
          }
          st.declared = n;
          if (c->srv->body_alloc_ && n >= c->srv->body_min_) st.ext = c->srv->body_alloc_(n);
          if (!st.ext) st.body.reserve(n);
        }
      }
      if (len && (st.head_len < 5 || st.received() + len > st.declared)) {
        c->refuse(st);  // more bytes than the prefix announced
        return 0;
      }
      if (st.ext) {
        std::memcpy(st.ext.get() + st.ext_len, data, len);
        st.ext_len += len;
      } else {
        st.body.append(reinterpret_cast<const char*>(data), len);
      }
      c->buffered += len;
    }
    return 0;
  }
  void refuse(Stream& st) {
    st.too_big = true;
    buffered -= std::min(buffered, st.received());
    st.body = std::string();
    st.ext.reset();
    st.ext_len = 0;
  }
  static int on_frame(nghttp2_session*, const nghttp2_frame* f, void* user) {
    if ((f->hd.type == NGHTTP2_DATA || f->hd.type == NGHTTP2_HEADERS) && (f->hd.flags & NGHTTP2_FLAG_END_STREAM))
      static_cast<Conn*>(user)->dispatch(f->hd.stream_id);
    return 0;
  }
  static int on_close(nghttp2_session*, int32_t sid, uint32_t, void* user) {
    auto* c = static_cast<Conn*>(user);
    auto it = c->streams.find(sid);
    if (it == c->streams.end()) return 0;
    if (!it->second.dispatched) c->buffered -= std::min(c->buffered, it->second.received());
    c->streams.erase(it);
    return 0;
  }
};

GrpcServer::GrpcServer(std::string host, int port, Handler handler, int workers)
    : host_(std::move(host)), port_(port), handler_(std::move(handler)), nworkers_(std::max(1, workers)) {}

GrpcServer::~GrpcServer() { stop(); }

bool GrpcServer::start(std::string* err) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) {
    *err = std::string("socket: ") + std::strerror(errno);
    return false;
  }
  int one = 1;
  ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port_));
  if (host_.empty() || host_ == "0.0.0.0") a.sin_addr.s_addr = INADDR_ANY;
  else if (host_ == "localhost") a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  else if (::inet_pton(AF_INET, host_.c_str(), &a.sin_addr) != 1) {
    *err = "bad bind address " + host_;
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || ::listen(lfd_, 512) != 0) {
    *err = std::string("bind/listen: ") + std::strerror(errno);
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  socklen_t al = sizeof a;
  ::getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &al);
  port_ = ntohs(a.sin_port);
  for (int i = 0; i < nworkers_; ++i)
    workers_.emplace_back([this] {
      name_thread("grpc-worker");
      worker_loop();
    });
  acceptor_ = std::thread([this] { accept_loop(); });
  return true;
}

void GrpcServer::stop() {
  if (stop_.exchange(true)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  {
    std::unique_lock<std::mutex> lk(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    conns_cv_.wait(lk, [this] { return live_conns_ == 0; });
  }
  cv_.notify_all();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
}

void GrpcServer::worker_loop() {
  for (;;) {
    std::function<void()> job;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_.load() || !jobs_.empty(); });
      if (jobs_.empty()) return;
      job = std::move(jobs_.front());
      jobs_.pop_front();
    }
    job();
  }
}

void GrpcServer::accept_loop() {
  while (!stop_.load()) {
    pollfd p{lfd_, POLLIN, 0};
    if (::poll(&p, 1, 200) <= 0) continue;
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    std::lock_guard<std::mutex> g(mu_);
    if (stop_.load()) {
      ::close(fd);
      break;
    }
    conns_.push_back(fd);
    live_conns_++;
    std::thread([this, fd] {
      name_thread("grpc-conn");
      serve(fd);
    }).detach();
  }
}

void GrpcServer::serve(int fd) {
  std::unique_ptr<TlsConn> tc;
  if (tls_) {
    // bounded handshake on the blocking socket (a silent client must not pin this thread)
    timeval tv{10, 0};
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    tc = std::make_unique<TlsConn>(tls_, fd);
    std::string err;
    if (!tc->handshake("", std::chrono::steady_clock::now() + std::chrono::seconds(10), &err)) {
      tc.reset();
      std::lock_guard<std::mutex> g(mu_);
      for (auto it = conns_.begin(); it != conns_.end(); ++it)
        if (*it == fd) {
          conns_.erase(it);
          break;
        }
      ::close(fd);
      if (--live_conns_ == 0) conns_cv_.notify_all();
      return;
    }
    timeval none{0, 0};
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof none);
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &none, sizeof none);
  }
  auto far = [] { return std::chrono::steady_clock::now() + std::chrono::hours(24); };
  auto c = std::make_shared<Conn>();
  c->srv = this;
  c->fd = fd;
  c->efd = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  nghttp2_session_callbacks* cbs;
  nghttp2_session_callbacks_new(&cbs);
  nghttp2_session_callbacks_set_on_begin_headers_callback(cbs, &Conn::on_begin_headers);
  nghttp2_session_callbacks_set_on_header_callback(cbs, &Conn::on_header);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, &Conn::on_data);
  nghttp2_session_callbacks_set_on_frame_recv_callback(cbs, &Conn::on_frame);
  nghttp2_session_callbacks_set_on_stream_close_callback(cbs, &Conn::on_close);
  nghttp2_session_callbacks_set_send_callback(cbs, &Conn::on_send);
  nghttp2_session_callbacks_set_send_data_callback(cbs, &Conn::send_data);
  nghttp2_session_callbacks_set_data_source_read_length_callback(cbs, &Conn::read_length);
  nghttp2_option* opt;
  nghttp2_option_new(&opt);
  nghttp2_option_set_no_http_messaging(opt, 0);
  nghttp2_session_server_new2(&c->session, cbs, c.get(), opt);
  nghttp2_option_del(opt);
  nghttp2_session_callbacks_del(cbs);
  nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 1024},
                                 {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 64u << 20},
                                 {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 20}};
  nghttp2_submit_settings(c->session, NGHTTP2_FLAG_NONE, iv, 3);
  nghttp2_session_set_local_window_size(c->session, NGHTTP2_FLAG_NONE, 0, 1 << 30);
  std::vector<uint8_t> buf(1 << 20);
  bool ok = true;
  c->tc = tc.get();
  // frames go out through on_send / send_data, in order, straight to the socket
  auto flush = [&] { return nghttp2_session_send(c->session) == 0; };
  ok = flush();
  while (ok && !stop_.load() && (nghttp2_session_want_read(c->session) || nghttp2_session_want_write(c->session))) {
    pollfd p[2] = {{fd, POLLIN, 0}, {c->efd, POLLIN, 0}};
    const bool buffered = tc && tc->pending();  // TLS records already decrypted: no poll
    if (::poll(p, 2, buffered ? 0 : 500) < 0 && errno != EINTR) break;
    if (buffered || (p[0].revents & (POLLIN | POLLHUP | POLLERR))) {
      ssize_t n = tc ? static_cast<ssize_t>(tc->read(buf.data(), buf.size())) : ::recv(fd, buf.data(), buf.size(), 0);
      if (tc && n == 0) continue;  // a record is still incomplete
      if (n <= 0) break;
      if (nghttp2_session_mem_recv(c->session, buf.data(), static_cast<size_t>(n)) < 0) break;
    }
    if (p[1].revents & POLLIN) {
      uint64_t v;
      (void)!::read(c->efd, &v, sizeof v);
      std::deque<std::pair<int32_t, GrpcReply>> ready;
      {
        std::lock_guard<std::mutex> g(c->mu);
        ready.swap(c->done);
      }
      for (auto& d : ready) c->respond(d.first, d.second);
    }
    ok = flush();
  }
  c->tc = nullptr;
  tc.reset();  // close_notify before the socket goes
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = conns_.begin(); it != conns_.end(); ++it)
    if (*it == fd) {
      conns_.erase(it);
      break;
    }
  ::close(fd);
  if (--live_conns_ == 0) conns_cv_.notify_all();
  // `c` (and its session) lives on while worker jobs still hold it; their replies are dropped
}

}  // namespace dfs
