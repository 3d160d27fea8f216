// Native HTTP/1.1 front end for the gateway (the reference's fiber server, core/http/app.go).
//
// One epoll I/O thread owns accept/read/parse; complete requests are queued for Python and an
// eventfd wakes the asyncio loop (loop.add_reader).  Responses are written by whichever thread
// produces them (asyncio loop, or the engine thread for token streams) directly into the socket,
// spilling into a per-connection buffer that the I/O thread drains on EPOLLOUT.
//
// Token streaming (the hot path): an SseSink is bound to a connection; the engine thread calls
// sink.push(text) per token and the chunk `head + json_escape(text) + mid + usage + tail` is
// built and written here without touching the asyncio loop (Python per token in the gateway
// was ~60-90 us; this is ~1-2 us).  Client disconnects flip the sink to closed so the engine
// aborts the sequence.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "text_stream.h"

#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace lahttp {

static inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void json_escape_append(std::string& out, const char* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  for (size_t i = 0; i < n; ++i) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          out += "\\u00";
          out += hex[c >> 4];
          out += hex[c & 15];
        } else if (c < 0x80) {
          out += static_cast<char>(c);
        } else {
          // a random-init (or byte-fallback) model can emit byte tokens that never complete a
          // UTF-8 sequence; JSON must stay valid UTF-8, so such bytes become U+FFFD
          const size_t len = c >= 0xF0 && c < 0xF5 ? 4 : c >= 0xE0 ? (c < 0xF0 ? 3 : 0) : c >= 0xC2 ? 2 : 0;
          bool ok = len != 0 && i + len <= n;
          for (size_t k = 1; ok && k < len; ++k) ok = (static_cast<unsigned char>(s[i + k]) & 0xC0) == 0x80;
          if (ok && len >= 3) {
            const unsigned char c1 = static_cast<unsigned char>(s[i + 1]);
            if (c == 0xE0 && c1 < 0xA0) ok = false;       // overlong
            if (c == 0xED && c1 >= 0xA0) ok = false;      // surrogate
            if (c == 0xF0 && c1 < 0x90) ok = false;       // overlong
            if (c == 0xF4 && c1 >= 0x90) ok = false;      // > U+10FFFF
          }
          if (ok) {
            out.append(s + i, len);
            i += len - 1;
          } else {
            out += "\xEF\xBF\xBD";
          }
        }
    }
  }
}

struct Request {
  uint64_t conn;
  std::string method, target, version;
  std::vector<std::pair<std::string, std::string>> headers;  // lower-cased names
  std::string body;
  std::string peer;
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::mutex mu;
  std::string in;       // unparsed input (I/O thread only)
  std::string out;      // pending output (guarded by mu)
  bool busy = false;    // a request is being served
  bool streaming = false;
  bool close_after = false;  // Connection: close
  bool closed = false;       // peer gone / fatal error
  bool drain_close = false;  // close once the output buffer is flushed
  bool want_out = false;     // EPOLLOUT armed
  bool rd_closed = false;    // peer half-closed (shutdown(SHUT_WR)); answer what is buffered, then close
  std::string peer;
  // request being received (I/O thread only): the head is parsed once and its bytes dropped from
  // `in`; a chunked body is decoded incrementally into head.body, consumed chunks leave `in` too
  bool have_head = false, chunked = false, expect = false, conn_close = false, sent_continue = false;
  size_t clen = 0;
  Request head;
};

class Server {
 public:
  Server(const std::string& host, int port, int backlog) {
    lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (lfd_ < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    if (host.empty() || host == "0.0.0.0") {
      a.sin_addr.s_addr = INADDR_ANY;
    } else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
      ::close(lfd_);
      throw std::runtime_error("bad listen address " + host);
    }
    if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
      const int e = errno;
      ::close(lfd_);
      throw std::runtime_error(std::string("bind failed: ") + strerror(e));
    }
    socklen_t al = sizeof(a);
    getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &al);
    port_ = ntohs(a.sin_port);
    if (::listen(lfd_, backlog) != 0) throw std::runtime_error("listen failed");
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    wake_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);   // I/O thread wake-up (stop)
    notify_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC); // Python wake-up (requests ready)
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = kListen;
    epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &ev);
    ev.data.u64 = kWake;
    epoll_ctl(ep_, EPOLL_CTL_ADD, wake_, &ev);
  }

  ~Server() { stop(); }

  int port() const { return port_; }
  int notify_fd() const { return notify_; }
  size_t max_body() const { return max_body_; }
  void set_max_body(size_t n) { max_body_ = n; }  // before start()

  void start() {
    if (th_.joinable()) return;
    running_ = true;
    th_ = std::thread([this] { loop(); });
  }

  void stop() {
    if (!running_.exchange(false)) return;
    uint64_t one = 1;
    (void)!::write(wake_, &one, 8);
    if (th_.joinable()) th_.join();
    std::lock_guard<std::mutex> g(map_mu_);
    for (auto& kv : conns_) ::close(kv.second->fd);
    conns_.clear();
    ::close(lfd_);
    ::close(ep_);
    ::close(wake_);
    ::close(notify_);
  }

  // Python: drain completed requests (non-blocking).
  py::list take_requests() {
    uint64_t v;
    (void)!::read(notify_, &v, 8);
    std::deque<Request> rs;
    {
      std::lock_guard<std::mutex> g(q_mu_);
      rs.swap(q_);
    }
    py::list out;
    for (auto& r : rs) {
      py::list hs;
      for (auto& h : r.headers) hs.append(py::make_tuple(py::bytes(h.first), py::bytes(h.second)));
      out.append(py::make_tuple(r.conn, r.method, py::bytes(r.target), r.version, hs, py::bytes(r.body), r.peer));
    }
    return out;
  }

  // Full response with Content-Length; the connection becomes ready for its next request.
  bool respond(uint64_t cid, int status, const std::vector<std::pair<std::string, std::string>>& headers,
               const std::string& body) {
    auto c = get(cid);
    if (!c) return false;
    std::string h = status_line(status);
    bool has_len = false;
    for (auto& kv : headers) {
      if (strcasecmp(kv.first.c_str(), "content-length") == 0) has_len = true;
      h += kv.first + ": " + kv.second + "\r\n";
    }
    if (!has_len) h += "content-length: " + std::to_string(body.size()) + "\r\n";
    if (c->close_after) h += "connection: close\r\n";
    h += "\r\n";
    h += body;
    return finish_response(c, std::move(h));
  }

  bool stream_start(uint64_t cid, int status, const std::vector<std::pair<std::string, std::string>>& headers) {
    auto c = get(cid);
    if (!c) return false;
    std::string h = status_line(status);
    for (auto& kv : headers) {
      if (strcasecmp(kv.first.c_str(), "content-length") == 0) continue;
      if (strcasecmp(kv.first.c_str(), "transfer-encoding") == 0) continue;
      h += kv.first + ": " + kv.second + "\r\n";
    }
    h += "transfer-encoding: chunked\r\n";
    if (c->close_after) h += "connection: close\r\n";
    h += "\r\n";
    {
      std::lock_guard<std::mutex> g(c->mu);
      c->streaming = true;
    }
    return send_raw(c, std::move(h));
  }

  bool stream_write(uint64_t cid, const std::string& data) {
    if (data.empty()) return is_open(cid);
    auto c = get(cid);
    if (!c) return false;
    return send_raw(c, chunk(data));
  }

  bool stream_end(uint64_t cid, const std::string& last) {
    auto c = get(cid);
    if (!c) return false;
    std::string s = last.empty() ? std::string() : chunk(last);
    s += "0\r\n\r\n";
    return finish_response(c, std::move(s));
  }

  bool is_open(uint64_t cid) {
    auto c = get(cid);
    if (!c) return false;
    std::lock_guard<std::mutex> g(c->mu);
    return !c->closed;
  }

  void close_conn(uint64_t cid) {
    auto c = get(cid);
    if (!c) return;
    {
      std::lock_guard<std::mutex> g(c->mu);
      c->closed = true;
    }
    schedule(cid);
  }

  size_t num_connections() {
    std::lock_guard<std::mutex> g(map_mu_);
    return conns_.size();
  }

  // ---- used by SseSink
  std::shared_ptr<Conn> get(uint64_t cid) {
    std::lock_guard<std::mutex> g(map_mu_);
    auto it = conns_.find(cid);
    return it == conns_.end() ? nullptr : it->second;
  }

  static std::string chunk(const std::string& data) {
    char hx[24];
    const int n = snprintf(hx, sizeof(hx), "%zx\r\n", data.size());
    std::string s;
    s.reserve(data.size() + n + 2);
    s.append(hx, n);
    s += data;
    s += "\r\n";
    return s;
  }

  bool send_raw(const std::shared_ptr<Conn>& c, std::string&& s) {
    std::lock_guard<std::mutex> g(c->mu);
    return send_locked(c.get(), s.data(), s.size());
  }

  bool finish_response(const std::shared_ptr<Conn>& c, std::string&& s) {
    bool ok;
    {
      std::lock_guard<std::mutex> g(c->mu);
      ok = send_locked(c.get(), s.data(), s.size());
      c->streaming = false;
      c->busy = false;
      if (c->close_after) c->drain_close = true;
    }
    // the I/O thread parses a pipelined request that may already be buffered, or closes
    schedule(c->id);
    return ok;
  }

  void schedule(uint64_t cid) {
    uint64_t one = 1;
    {
      std::lock_guard<std::mutex> g(resume_mu_);
      resume_.push_back(cid);
    }
    (void)!::write(wake_, &one, 8);
  }

 private:
  static constexpr uint64_t kListen = ~0ull, kWake = ~0ull - 1;

  static std::string status_line(int status) {
    const char* reason = "OK";
    switch (status) {
      case 200: reason = "OK"; break;
      case 201: reason = "Created"; break;
      case 204: reason = "No Content"; break;
      case 400: reason = "Bad Request"; break;
      case 401: reason = "Unauthorized"; break;
      case 403: reason = "Forbidden"; break;
      case 404: reason = "Not Found"; break;
      case 405: reason = "Method Not Allowed"; break;
      case 413: reason = "Payload Too Large"; break;
      case 422: reason = "Unprocessable Entity"; break;
      case 500: reason = "Internal Server Error"; break;
      case 501: reason = "Not Implemented"; break;
      case 503: reason = "Service Unavailable"; break;
      default: reason = "";
    }
    return "HTTP/1.1 " + std::to_string(status) + " " + reason + "\r\n";
  }

  // caller holds c->mu
  bool send_locked(Conn* c, const char* p, size_t n) {
    if (c->closed) return false;
    if (!c->out.empty()) {
      c->out.append(p, n);
      return true;
    }
    while (n) {
      const ssize_t w = ::send(c->fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (w > 0) {
        p += w;
        n -= static_cast<size_t>(w);
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      c->closed = true;
      return false;
    }
    if (n) {
      c->out.append(p, n);
      if (!c->want_out) {
        c->want_out = true;
        rearm(c);
      }
    }
    return true;
  }

  // caller holds c->mu: read interest until the peer half-closes, write interest while output is queued
  void rearm(Conn* c) {
    epoll_event ev{};
    ev.events = (c->rd_closed ? 0u : static_cast<uint32_t>(EPOLLIN | EPOLLRDHUP)) | (c->want_out ? EPOLLOUT : 0u);
    ev.data.u64 = c->id;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &ev);
  }

  void drop(const std::shared_ptr<Conn>& c) {
    {
      std::lock_guard<std::mutex> g(c->mu);
      if (c->fd < 0) return;
      c->closed = true;
      epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
      ::close(c->fd);
      c->fd = -1;
    }
    std::lock_guard<std::mutex> g(map_mu_);
    conns_.erase(c->id);
  }

  void accept_all() {
    for (;;) {
      sockaddr_in a{};
      socklen_t al = sizeof(a);
      const int fd = accept4(lfd_, reinterpret_cast<sockaddr*>(&a), &al, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      auto c = std::make_shared<Conn>();
      c->fd = fd;
      c->id = next_id_++;
      char buf[64];
      inet_ntop(AF_INET, &a.sin_addr, buf, sizeof(buf));
      c->peer = std::string(buf) + ":" + std::to_string(ntohs(a.sin_port));
      {
        std::lock_guard<std::mutex> g(map_mu_);
        conns_[c->id] = c;
      }
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    }
  }

  // Parse as many complete requests as allowed (one in flight per connection). The head is parsed
  // once; a body is taken when complete. Chunked bodies are decoded incrementally (each recv only
  // looks at new chunks) and both body kinds are held to max_body_ before they are buffered.
  void parse(const std::shared_ptr<Conn>& c) {
    for (;;) {
      {
        std::lock_guard<std::mutex> g(c->mu);
        if (c->busy || c->closed) return;
      }
      if (!c->have_head && !parse_head(c)) return;
      if (c->chunked) {
        size_t q = 0;
        bool complete = false;
        for (;;) {
          const size_t e = c->in.find("\r\n", q);
          if (e == std::string::npos) {
            if (c->in.size() - q > 4096) return bad(c, 400);  // chunk-size line without an end
            break;
          }
          char* endp = nullptr;
          const std::string line = c->in.substr(q, e - q);
          errno = 0;
          const unsigned long long n = strtoull(line.c_str(), &endp, 16);
          if (endp == line.c_str() || errno == ERANGE || (*endp && *endp != ';' && *endp != ' ' && *endp != '\t'))
            return bad(c, 400);
          if (n == 0) {
            // last-chunk, optional trailer fields, empty line
            size_t t;
            if (c->in.compare(e + 2, 2, "\r\n") == 0) t = e + 4;
            else {
              const size_t te = c->in.find("\r\n\r\n", e + 2);
              if (te == std::string::npos) break;
              t = te + 4;
            }
            q = t;
            complete = true;
            break;
          }
          if (n > max_body_ || c->head.body.size() + n > max_body_) return bad(c, 413);
          if (c->in.size() - (e + 2) < n + 2) break;
          c->head.body.append(c->in, e + 2, n);
          q = e + 2 + n + 2;
        }
        c->in.erase(0, q);
        if (!complete) {
          if (c->expect && !c->sent_continue) {
            c->sent_continue = true;
            send_continue(c);
          }
          return;
        }
      } else {
        if (c->in.size() < c->clen) {
          if (c->expect && !c->sent_continue) {
            c->sent_continue = true;
            send_continue(c);
          }
          return;
        }
        c->head.body = c->in.substr(0, c->clen);
        c->in.erase(0, c->clen);
      }
      c->have_head = false;
      {
        std::lock_guard<std::mutex> g(c->mu);
        c->busy = true;
        c->close_after = c->conn_close || c->rd_closed;
      }
      {
        std::lock_guard<std::mutex> g(q_mu_);
        q_.push_back(std::move(c->head));
      }
      c->head = Request();
      uint64_t one = 1;
      (void)!::write(notify_, &one, 8);
    }
  }

  // Request line + headers of the next request into c->head; false if incomplete or rejected.
  bool parse_head(const std::shared_ptr<Conn>& c) {
    const size_t he = c->in.find("\r\n\r\n");
    if (he == std::string::npos) {
      if (c->in.size() > (1u << 20)) bad(c, 431);
      return false;
    }
    Request& r = c->head;
    r = Request();
    r.conn = c->id;
    r.peer = c->peer;
    const size_t le = c->in.find("\r\n");
    {
      const std::string line = c->in.substr(0, le);
      const size_t s1 = line.find(' ');
      const size_t s2 = line.rfind(' ');
      if (s1 == std::string::npos || s2 == s1) {
        bad(c, 400);
        return false;
      }
      r.method = line.substr(0, s1);
      r.target = line.substr(s1 + 1, s2 - s1 - 1);
      r.version = line.substr(s2 + 1);
    }
    size_t p = le + 2;
    c->clen = 0;
    c->chunked = false;
    c->expect = false;
    c->sent_continue = false;
    c->conn_close = (r.version == "HTTP/1.0");
    bool bad_len = false;
    while (p < he) {
      const size_t e = c->in.find("\r\n", p);
      const size_t colon = c->in.find(':', p);
      if (colon != std::string::npos && colon < e) {
        std::string k = c->in.substr(p, colon - p);
        for (auto& ch : k) ch = static_cast<char>(tolower(ch));
        size_t vs = colon + 1;
        while (vs < e && (c->in[vs] == ' ' || c->in[vs] == '\t')) ++vs;
        size_t ve = e;
        while (ve > vs && (c->in[ve - 1] == ' ' || c->in[ve - 1] == '\t')) --ve;
        std::string v = c->in.substr(vs, ve - vs);
        if (k == "content-length") {
          char* endp = nullptr;
          errno = 0;
          c->clen = strtoull(v.c_str(), &endp, 10);
          if (v.empty() || *endp || errno == ERANGE) bad_len = true;
        } else if (k == "transfer-encoding" && v.find("chunked") != std::string::npos) {
          c->chunked = true;
        } else if (k == "connection") {
          std::string lv = v;
          for (auto& ch : lv) ch = static_cast<char>(tolower(ch));
          if (lv.find("close") != std::string::npos) c->conn_close = true;
          if (lv.find("keep-alive") != std::string::npos) c->conn_close = false;
        } else if (k == "expect") {
          c->expect = true;
        }
        r.headers.emplace_back(std::move(k), std::move(v));
      }
      p = e + 2;
    }
    c->in.erase(0, he + 4);
    if (bad_len && !c->chunked) {
      bad(c, 400);
      return false;
    }
    if (!c->chunked && c->clen > max_body_) {
      bad(c, 413);
      return false;
    }
    c->have_head = true;
    return true;
  }

  // bytes of unparsed input a connection may hold: one maximal body plus a head
  size_t in_cap() const { return max_body_ + (2u << 20); }

  void send_continue(const std::shared_ptr<Conn>& c) {
    static const char k100[] = "HTTP/1.1 100 Continue\r\n\r\n";
    std::lock_guard<std::mutex> g(c->mu);
    send_locked(c.get(), k100, sizeof(k100) - 1);
  }

  void bad(const std::shared_ptr<Conn>& c, int status) {
    std::string s = status_line(status) + "content-length: 0\r\nconnection: close\r\n\r\n";
    {
      std::lock_guard<std::mutex> g(c->mu);
      send_locked(c.get(), s.data(), s.size());
    }
    drop(c);
  }

  void loop() {
    std::vector<epoll_event> evs(256);
    char buf[65536];
    while (running_) {
      const int n = epoll_wait(ep_, evs.data(), static_cast<int>(evs.size()), 1000);
      for (int i = 0; i < n; ++i) {
        const uint64_t id = evs[i].data.u64;
        if (id == kListen) {
          accept_all();
          continue;
        }
        if (id == kWake) {
          uint64_t v;
          (void)!::read(wake_, &v, 8);
          std::vector<uint64_t> rs;
          {
            std::lock_guard<std::mutex> g(resume_mu_);
            rs.swap(resume_);
          }
          for (auto cid : rs) {
            auto c = get(cid);
            if (!c) continue;
            bool dead, drained;
            {
              std::lock_guard<std::mutex> g(c->mu);
              dead = c->closed;
              drained = c->drain_close && c->out.empty();
            }
            if (dead || drained) drop(c);
            else parse(c);
          }
          continue;
        }
        auto c = get(id);
        if (!c) continue;
        const uint32_t e = evs[i].events;
        if (e & EPOLLOUT) {
          std::lock_guard<std::mutex> g(c->mu);
          while (!c->out.empty() && !c->closed) {
            const ssize_t w = ::send(c->fd, c->out.data(), c->out.size(), MSG_NOSIGNAL | MSG_DONTWAIT);
            if (w > 0) {
              c->out.erase(0, static_cast<size_t>(w));
            } else if (w < 0 && errno == EINTR) {
              continue;
            } else if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
              break;
            } else {
              c->closed = true;
            }
          }
          if (c->out.empty() && c->drain_close) c->closed = true;
          if (c->out.empty() && c->want_out && !c->closed) {
            c->want_out = false;
            rearm(c.get());
          }
        }
        bool gone = false, eof = false;
        if (e & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          for (;;) {
            const ssize_t r = ::recv(c->fd, buf, sizeof(buf), MSG_DONTWAIT);
            if (r > 0) {
              c->in.append(buf, static_cast<size_t>(r));
              if (c->in.size() > in_cap()) break;  // checked below
              continue;
            }
            if (r == 0) eof = true;
            else if (errno == EINTR) continue;
            else if (errno != EAGAIN && errno != EWOULDBLOCK) gone = true;
            break;
          }
          if (e & (EPOLLHUP | EPOLLERR)) gone = true;
        }
        if (gone) {
          drop(c);
          continue;
        }
        bool busy;
        {
          std::lock_guard<std::mutex> g(c->mu);
          busy = c->busy;
        }
        // a client that keeps pipelining while its request is served cannot grow `in` without bound
        if (busy && c->in.size() > in_cap()) {
          drop(c);
          continue;
        }
        parse(c);
        if (eof) {
          // half-close after a complete request is legal: answer it, then close; nothing
          // complete buffered (or a partial request) -> the connection is finished
          std::lock_guard<std::mutex> g(c->mu);
          if (!c->busy && c->out.empty()) {
            c->closed = true;
          } else {
            c->rd_closed = true;
            c->close_after = true;
            if (!c->busy) c->drain_close = true;
            rearm(c.get());
          }
        }
        bool dead;
        {
          std::lock_guard<std::mutex> g(c->mu);
          dead = c->closed;
        }
        if (dead) drop(c);
      }
    }
  }

  int lfd_ = -1, ep_ = -1, wake_ = -1, notify_ = -1, port_ = 0;
  size_t max_body_ = 64u << 20;
  std::atomic<bool> running_{false};
  std::thread th_;
  std::mutex map_mu_, q_mu_, resume_mu_;
  std::unordered_map<uint64_t, std::shared_ptr<Conn>> conns_;
  std::deque<Request> q_;
  std::vector<uint64_t> resume_;
  std::atomic<uint64_t> next_id_{1};
};

// Per-request SSE token sink (engine thread -> socket).
class SseSink {
 public:
  SseSink(Server* srv, uint64_t conn, std::string head, std::string mid, std::string tail, int prompt_tokens)
      : srv_(srv), conn_(conn), head_(std::move(head)), mid_(std::move(mid)), tail_(std::move(tail)),
        prompt_(prompt_tokens), t0_(now_s()) {}

  // One token (or several coalesced) of text; returns false once the client is gone.
  bool push(const std::string& text, int completion_tokens) {
    if (done_) return false;
    if (completion_tokens > 0) ntok_ = completion_tokens;
    else ++ntok_;
    if (text.empty()) return srv_->is_open(conn_);
    if (t_first_ == 0) t_first_ = now_s();
    std::string s;
    s.reserve(head_.size() + text.size() + 96);
    s += head_;
    json_escape_append(s, text.data(), text.size());
    s += mid_;
    s += "{\"prompt_tokens\":" + std::to_string(prompt_) + ",\"completion_tokens\":" + std::to_string(ntok_) +
         ",\"total_tokens\":" + std::to_string(prompt_ + ntok_) + "}";
    s += tail_;
    return srv_->stream_write(conn_, s);
  }

  // Several tokens at once (one SSE event each, one socket write): n_gen[i] is the completion
  // count after piece i.
  bool push_many(const std::vector<std::string>& pieces, const std::vector<int>& n_gen) {
    if (done_) return false;
    std::string s;
    for (size_t i = 0; i < pieces.size(); ++i) {
      ntok_ = n_gen[i];
      const std::string& text = pieces[i];
      if (text.empty()) continue;
      if (t_first_ == 0) t_first_ = now_s();
      s += head_;
      json_escape_append(s, text.data(), text.size());
      s += mid_;
      s += "{\"prompt_tokens\":" + std::to_string(prompt_) + ",\"completion_tokens\":" + std::to_string(ntok_) +
           ",\"total_tokens\":" + std::to_string(prompt_ + ntok_) + "}";
      s += tail_;
    }
    if (s.empty()) return srv_->is_open(conn_);
    return srv_->stream_write(conn_, s);
  }

  // Raw final bytes (final chunk + [DONE]) and end of the chunked body.
  bool finish(const std::string& raw) {
    if (done_) return false;
    done_ = true;
    return srv_->stream_end(conn_, raw);
  }

  void set_prompt_tokens(int p) { prompt_ = p; }
  bool open() { return !done_ && srv_->is_open(conn_); }
  double ttft() const { return t_first_ == 0 ? -1.0 : t_first_ - t0_; }
  int tokens() const { return ntok_; }

 private:
  Server* srv_;
  uint64_t conn_;
  std::string head_, mid_, tail_;
  int prompt_ = 0, ntok_ = 0;
  double t0_, t_first_ = 0;
  bool done_ = false;
};

// Post-process one device-resident multi-step decode run for every row in C++ (the per-token
// Python path cost ~4 us x rows x steps on the engine thread): detokenise with stop-string
// hold-back, apply EOS / max_tokens / context limits, and write each streaming row's new SSE
// events with a single socket write.  reason: 0 running, 1 eos, 2 stop string, 3 length,
// 4 client gone.
py::tuple emit_run(py::array_t<int32_t, py::array::c_style | py::array::forcecast> hist, int K, int B,
                   py::list streams, py::list sinks, py::array_t<int32_t, py::array::c_style | py::array::forcecast> st,
                   std::vector<int32_t> eog, int ctx) {
  const int ld = (int)hist.shape(1);
  const int32_t* H = hist.data();
  const int32_t* S = st.data();
  std::vector<la::TextStream*> ts(B, nullptr);
  std::vector<SseSink*> sk(B, nullptr);
  for (int b = 0; b < B; ++b) {
    if (!streams[b].is_none()) ts[b] = streams[b].cast<la::TextStream*>();
    if (!sinks[b].is_none()) sk[b] = sinks[b].cast<SseSink*>();
  }
  std::vector<int> nacc(B, 0), reason(B, 0);
  std::vector<std::string> texts(B);
  // rows are independent (own TextStream, own connection): a wide batch is split over a few
  // threads so detokenisation + SSE formatting + the per-connection send of 256 streams does not
  // serialise on the engine thread between two graph runs (~20 us a row on one thread)
  auto rows = [&](int b0, int b1) {
    std::vector<std::string> pieces;
    std::vector<int> ngen;
    for (int b = b0; b < b1; ++b) {
      const int32_t* row = S + 5 * b;
      int n_gen = row[0];
      const int max_tokens = row[1], n_prompt = row[2], ignore_eos = row[3], active = row[4];
      if (!active || !ts[b]) continue;
      pieces.clear();
      ngen.clear();
      int rs = 0, acc = 0;
      for (int k = 0; k < K; ++k) {
        const int32_t tok = H[(long)k * ld + b];
        ++n_gen;
        ++acc;
        if (!ignore_eos && std::find(eog.begin(), eog.end(), tok) != eog.end()) {
          rs = 1;
          break;
        }
        auto r = ts[b]->push_raw(tok);
        pieces.push_back(std::move(r.first));
        ngen.push_back(n_gen);
        if (r.second) { rs = 2; break; }
        if (max_tokens > 0 && n_gen >= max_tokens) { rs = 3; break; }
        if (n_prompt + n_gen >= ctx) { rs = 3; break; }
      }
      if (sk[b]) {
        if (!sk[b]->push_many(pieces, ngen) && rs == 0) rs = 4;
      } else {
        for (auto& p : pieces) texts[b] += p;
      }
      nacc[b] = acc;
      reason[b] = rs;
    }
  };
  {
    py::gil_scoped_release rel;
    int nsink = 0;
    for (int b = 0; b < B; ++b) nsink += sk[b] != nullptr;
    const int T = nsink >= 64 ? std::min(8, std::max(1, nsink / 32)) : 1;
    if (T == 1) {
      rows(0, B);
    } else {
      std::vector<std::thread> th;
      const int per = (B + T - 1) / T;
      for (int t = 1; t < T; ++t) th.emplace_back(rows, std::min(B, t * per), std::min(B, (t + 1) * per));
      rows(0, std::min(B, per));
      for (auto& x : th) x.join();
    }
  }
  py::list out_texts;
  for (int b = 0; b < B; ++b) out_texts.append(texts[b].empty() ? py::object(py::none()) : py::object(py::bytes(texts[b])));
  return py::make_tuple(py::array_t<int32_t>(B, nacc.data()), py::array_t<int32_t>(B, reason.data()), out_texts);
}

}  // namespace lahttp

void register_http(py::module& m) {
  using namespace lahttp;
  py::class_<Server>(m, "Server")
      .def(py::init<const std::string&, int, int>(), py::arg("host"), py::arg("port"), py::arg("backlog") = 4096)
      .def_property_readonly("port", &Server::port)
      .def_property_readonly("notify_fd", &Server::notify_fd)
      .def_property("max_body", &Server::max_body, &Server::set_max_body)
      .def("start", &Server::start)
      .def("stop", &Server::stop, py::call_guard<py::gil_scoped_release>())
      .def("take_requests", &Server::take_requests)
      .def("respond", &Server::respond, py::call_guard<py::gil_scoped_release>())
      .def("stream_start", &Server::stream_start, py::call_guard<py::gil_scoped_release>())
      .def("stream_write", &Server::stream_write, py::call_guard<py::gil_scoped_release>())
      .def("stream_end", &Server::stream_end, py::arg("conn"), py::arg("last") = std::string(),
           py::call_guard<py::gil_scoped_release>())
      .def("is_open", &Server::is_open)
      .def("close", &Server::close_conn)
      .def("num_connections", &Server::num_connections);
  py::class_<SseSink>(m, "SseSink")
      .def(py::init<Server*, uint64_t, std::string, std::string, std::string, int>(), py::keep_alive<1, 2>())
      .def("push", &SseSink::push, py::arg("text"), py::arg("completion_tokens") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("push_many", &SseSink::push_many, py::call_guard<py::gil_scoped_release>())
      .def("finish", &SseSink::finish, py::call_guard<py::gil_scoped_release>())
      .def("set_prompt_tokens", &SseSink::set_prompt_tokens)
      .def("open", &SseSink::open)
      .def_property_readonly("ttft", &SseSink::ttft)
      .def_property_readonly("tokens", &SseSink::tokens);
  m.def("emit_run", &emit_run);
  m.def("json_escape", [](const std::string& s) {
    std::string o;
    json_escape_append(o, s.data(), s.size());
    return py::bytes(o);
  });
}
