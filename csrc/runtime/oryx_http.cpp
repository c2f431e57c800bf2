// oryx_http.cpp -- the serving layer's native HTTP/1.1 front end.
//
// The reference serves its REST endpoints from embedded Tomcat ([lserving]/ServingLayer.java:
// 194-245: a connector with its own acceptor and poller threads in front of the servlet
// worker pool).  Here an epoll loop on one native thread accepts connections and parses
// requests (request line, headers, Content-Length or chunked bodies, keep-alive and
// pipelining); complete requests wait in a queue that the Python handler threads take from
// (oryx_http_next blocks without the GIL), and their responses come back as ready bytes
// (oryx_http_respond) that the loop writes in request order per connection.  So the Python
// side does only routing and the endpoint's own work per request: no per-connection thread,
// no header parsing in Python, no socket calls.
//
// TLS is not handled here (the Python server keeps that path).

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr size_t kMaxHeader = 64 * 1024;

struct Req {
  uint64_t id = 0;
  std::string method, target, headers, body;
};

struct Conn {
  int fd = -1;
  uint64_t cid = 0;
  std::string in;                  // unparsed input
  size_t scan = 0;                 // header-end search resumes here
  // a request whose headers are parsed and whose body is still arriving
  bool in_body = false, chunked = false, close_after = false;
  long long body_len = 0;
  Req cur;
  // responses by request sequence; next_out = the next one to write
  uint64_t next_seq = 0, next_out = 0;
  std::map<uint64_t, std::pair<std::string, bool>> done;
  std::string out;                 // bytes being written
  size_t out_off = 0;
  bool closing = false;            // close once `out` drains
  bool read_shut = false;
  bool wout = false;               // EPOLLOUT armed
};

struct Server {
  int lfd = -1, efd = -1, wfd = -1;   // listener, epoll, eventfd (responses ready / stop)
  int port = 0;
  long long max_body = 64ll << 20;
  std::atomic<bool> stop{false};
  // requests ready for the handlers; `leader`: a handler thread is polling the sockets
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<Req> ready;
  bool leader = false;
  // connection state: taken by the loop per event and by a handler thread that writes its
  // response straight to the socket (oryx_http_respond: no hop through the loop thread)
  std::mutex cmu;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  std::unordered_map<uint64_t, std::pair<uint64_t, uint64_t>> inflight;  // id -> (cid, seq)
  std::unordered_map<uint64_t, int> fd_of_cid;
  uint64_t next_id = 1, next_cid = 1;
  std::atomic<long long> served{0};
};

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

bool ieq(const char* a, size_t n, const char* b) {
  if (strlen(b) != n) return false;
  for (size_t k = 0; k < n; ++k)
    if (tolower((unsigned char)a[k]) != tolower((unsigned char)b[k])) return false;
  return true;
}

std::string lower_trim(const char* a, size_t n) {
  while (n && (*a == ' ' || *a == '\t')) { ++a; --n; }
  while (n && (a[n - 1] == ' ' || a[n - 1] == '\t')) --n;
  std::string s(a, n);
  for (char& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

const char* status_text(int code) {
  switch (code) {
    case 400: return "Bad Request";
    case 413: return "Payload Too Large";
    case 431: return "Request Header Fields Too Large";
    case 501: return "Not Implemented";
    default: return "Error";
  }
}

// An error response produced by the loop itself (malformed request): written after the
// connection's earlier responses, then the connection closes.
void loop_error(Server* S, Conn* c, int code) {
  std::string body = std::string(status_text(code)) + "\n";
  std::string r = "HTTP/1.1 " + std::to_string(code) + " " + status_text(code) +
                  "\r\nContent-Type: text/plain; charset=UTF-8\r\nContent-Length: " +
                  std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
  c->done[c->next_seq++] = {r, true};
  c->read_shut = true;
  (void)S;
}

void close_conn(Server* S, int fd) {
  auto it = S->conns.find(fd);
  if (it == S->conns.end()) return;
  S->fd_of_cid.erase(it->second->cid);
  epoll_ctl(S->efd, EPOLL_CTL_DEL, fd, nullptr);
  close(fd);
  S->conns.erase(it);
}

void want_write(Server* S, Conn* c, bool on) {
  if (c->wout == on) return;
  c->wout = on;
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | (on ? EPOLLOUT : 0);
  ev.data.fd = c->fd;
  epoll_ctl(S->efd, EPOLL_CTL_MOD, c->fd, &ev);
}

// Moves finished responses into the write buffer in request order and writes what the
// socket takes.  Returns false when the connection is gone.
bool flush_conn(Server* S, Conn* c) {
  for (;;) {
    if (c->out_off >= c->out.size()) {
      c->out.clear();
      c->out_off = 0;
      if (c->closing) {
        close_conn(S, c->fd);
        return false;
      }
      auto it = c->done.find(c->next_out);
      if (it == c->done.end()) break;
      c->out = std::move(it->second.first);
      c->closing = it->second.second;
      c->done.erase(it);
      ++c->next_out;
      // batch every further ready response into the same write
      for (auto jt = c->done.find(c->next_out); jt != c->done.end() && !c->closing;
           jt = c->done.find(c->next_out)) {
        c->out += jt->second.first;
        c->closing = jt->second.second;
        c->done.erase(jt);
        ++c->next_out;
      }
    }
    const ssize_t w = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off,
                           MSG_NOSIGNAL);
    if (w > 0) {
      c->out_off += (size_t)w;
      continue;
    }
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      want_write(S, c, true);
      return true;
    }
    if (w < 0 && errno == EINTR) continue;
    close_conn(S, c->fd);
    return false;
  }
  want_write(S, c, false);
  if (c->read_shut && c->next_out == c->next_seq) {
    close_conn(S, c->fd);
    return false;
  }
  return true;
}

void submit(Server* S, Conn* c) {
  Req r = std::move(c->cur);
  c->cur = Req();
  r.id = S->next_id++;
  const uint64_t seq = c->next_seq++;
  S->inflight[r.id] = {c->cid, seq};
  // (no wake-up here: the polling thread takes a request itself when its poll returns)
  std::lock_guard<std::mutex> g(S->qmu);
  S->ready.push_back(std::move(r));
}

// Parses whatever complete requests c->in holds.
void parse_input(Server* S, Conn* c) {
  for (;;) {
    if (c->read_shut) return;
    if (!c->in_body) {
      const size_t from = c->scan >= 3 ? c->scan - 3 : 0;
      const size_t e = c->in.find("\r\n\r\n", from);
      if (e == std::string::npos) {
        c->scan = c->in.size();
        if (c->in.size() > kMaxHeader) loop_error(S, c, 431);
        return;
      }
      c->scan = 0;
      // request line
      const size_t le = c->in.find("\r\n");
      const std::string line = c->in.substr(0, le);
      const size_t sp1 = line.find(' ');
      const size_t sp2 = sp1 == std::string::npos ? std::string::npos : line.find(' ', sp1 + 1);
      if (sp1 == std::string::npos || sp2 == std::string::npos) {
        loop_error(S, c, 400);
        return;
      }
      c->cur.method = line.substr(0, sp1);
      c->cur.target = line.substr(sp1 + 1, sp2 - sp1 - 1);
      const std::string ver = line.substr(sp2 + 1);
      bool keep = ver == "HTTP/1.1";
      if (ver != "HTTP/1.1" && ver != "HTTP/1.0") {
        loop_error(S, c, 400);
        return;
      }
      c->cur.headers = c->in.substr(le + 2, e + 2 - (le + 2));
      c->body_len = 0;
      c->chunked = false;
      bool expect_continue = false;
      // the headers the loop needs: length, chunking, persistence
      const char* h = c->cur.headers.data();
      const size_t hn = c->cur.headers.size();
      for (size_t p = 0; p < hn;) {
        size_t q = c->cur.headers.find("\r\n", p);
        if (q == std::string::npos) q = hn;
        const size_t colon = c->cur.headers.find(':', p);
        if (colon != std::string::npos && colon < q) {
          const char* name = h + p;
          const size_t nn = colon - p;
          if (ieq(name, nn, "content-length")) {
            const std::string v = lower_trim(h + colon + 1, q - colon - 1);
            char* endp = nullptr;
            c->body_len = strtoll(v.c_str(), &endp, 10);
            if (v.empty() || *endp || c->body_len < 0) {
              loop_error(S, c, 400);
              return;
            }
          } else if (ieq(name, nn, "transfer-encoding")) {
            const std::string v = lower_trim(h + colon + 1, q - colon - 1);
            if (v == "chunked") c->chunked = true;
            else if (v != "identity") {
              loop_error(S, c, 501);
              return;
            }
          } else if (ieq(name, nn, "expect")) {
            expect_continue = lower_trim(h + colon + 1, q - colon - 1) == "100-continue";
          } else if (ieq(name, nn, "connection")) {
            const std::string v = lower_trim(h + colon + 1, q - colon - 1);
            if (v.find("close") != std::string::npos) keep = false;
            else if (v.find("keep-alive") != std::string::npos) keep = true;
          }
        }
        p = q + 2;
      }
      if (c->body_len > S->max_body) {
        loop_error(S, c, 413);
        return;
      }
      c->close_after = !keep;
      c->in.erase(0, e + 4);
      c->in_body = true;
      // a client that waits for "100 Continue" before its body gets it at once (when no
      // earlier response on the connection is still due, which it would have to follow)
      if (expect_continue && (c->chunked || (long long)c->in.size() < c->body_len) &&
          c->next_out == c->next_seq && c->out.empty()) {
        static const char k100[] = "HTTP/1.1 100 Continue\r\n\r\n";
        (void)!send(c->fd, k100, sizeof(k100) - 1, MSG_NOSIGNAL);
      }
    }
    // body
    if (c->chunked) {
      // chunks: hex size [;ext] CRLF data CRLF ... 0 CRLF [trailers] CRLF
      size_t p = 0;
      std::string body;
      for (;;) {
        const size_t le = c->in.find("\r\n", p);
        if (le == std::string::npos) return;           // need more
        const long long sz = strtoll(c->in.substr(p, le - p).c_str(), nullptr, 16);
        if (sz < 0 || (long long)body.size() + sz > S->max_body) {
          loop_error(S, c, 413);
          return;
        }
        if (sz == 0) {
          // trailers end at an empty line
          const size_t te = c->in.find("\r\n", le + 2);
          if (te == std::string::npos) return;
          size_t end = le + 2;
          while (true) {
            const size_t nl = c->in.find("\r\n", end);
            if (nl == std::string::npos) return;
            if (nl == end) { end += 2; break; }
            end = nl + 2;
          }
          c->cur.body = std::move(body);
          c->in.erase(0, end);
          break;
        }
        if (c->in.size() < le + 2 + (size_t)sz + 2) return;
        body.append(c->in, le + 2, (size_t)sz);
        p = le + 2 + (size_t)sz + 2;
      }
    } else {
      if ((long long)c->in.size() < c->body_len) return;
      c->cur.body = c->in.substr(0, (size_t)c->body_len);
      c->in.erase(0, (size_t)c->body_len);
    }
    c->in_body = false;
    const bool close_after = c->close_after;
    submit(S, c);
    if (close_after) {
      c->read_shut = true;     // no further requests on this connection
      return;
    }
  }
}

// One round of the event loop, run by the handler thread that currently leads (see
// oryx_http_next): waits up to wait_ms for socket events and handles them all.
void poll_once(Server* S, int wait_ms) {
  epoll_event evs[256];
  static thread_local char buf[64 * 1024];
  {
    const int n = epoll_wait(S->efd, evs, 256, wait_ms);
    for (int k = 0; k < n; ++k) {
      const int fd = evs[k].data.fd;
      std::lock_guard<std::mutex> g(S->cmu);
      if (fd == S->lfd) {
        for (;;) {
          const int cfd = accept4(S->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (cfd < 0) break;
          int one = 1;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          auto c = std::make_unique<Conn>();
          c->fd = cfd;
          c->cid = S->next_cid++;
          S->fd_of_cid[c->cid] = cfd;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = cfd;
          epoll_ctl(S->efd, EPOLL_CTL_ADD, cfd, &ev);
          S->conns[cfd] = std::move(c);
        }
        continue;
      }
      if (fd == S->wfd) {         // stop
        uint64_t v;
        (void)!read(S->wfd, &v, sizeof(v));
        continue;
      }
      auto it = S->conns.find(fd);
      if (it == S->conns.end()) continue;
      Conn* c = it->second.get();
      if (evs[k].events & EPOLLOUT) {
        if (!flush_conn(S, c)) continue;
      }
      if (evs[k].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
        bool eof = false;
        for (;;) {
          const ssize_t r = recv(fd, buf, sizeof(buf), 0);
          if (r > 0) {
            if (!c->read_shut) c->in.append(buf, (size_t)r);
            continue;
          }
          if (r == 0) eof = true;
          else if (errno == EINTR) continue;
          else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
          break;
        }
        parse_input(S, c);
        if (eof) {
          // the client closed: answer what it already sent only if it can still read
          if (c->next_out == c->next_seq) {
            close_conn(S, fd);
            continue;
          }
          c->read_shut = true;
        }
        flush_conn(S, c);
      }
    }
  }
}

}  // namespace

extern "C" {

// Binds host:port (port 0: any free port).  The sockets are polled by the threads calling
// oryx_http_next.  Returns a handle or null.
void* oryx_http_start(const char* host, int port, int backlog, long long max_body) {
  auto* S = new Server();
  if (max_body > 0) S->max_body = max_body;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host && *host ? host : nullptr, ps.c_str(), &hints, &res) != 0 || !res) {
    delete S;
    return nullptr;
  }
  S->lfd = socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(S->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (S->lfd < 0 || bind(S->lfd, res->ai_addr, res->ai_addrlen) != 0 ||
      listen(S->lfd, backlog > 0 ? backlog : 1024) != 0) {
    if (S->lfd >= 0) close(S->lfd);
    freeaddrinfo(res);
    delete S;
    return nullptr;
  }
  freeaddrinfo(res);
  sockaddr_storage sa{};
  socklen_t sl = sizeof(sa);
  getsockname(S->lfd, (sockaddr*)&sa, &sl);
  S->port = sa.ss_family == AF_INET6 ? ntohs(((sockaddr_in6*)&sa)->sin6_port)
                                     : ntohs(((sockaddr_in*)&sa)->sin_port);
  set_nonblock(S->lfd);
  S->efd = epoll_create1(EPOLL_CLOEXEC);
  S->wfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = S->lfd;
  epoll_ctl(S->efd, EPOLL_CTL_ADD, S->lfd, &ev);
  ev.data.fd = S->wfd;
  epoll_ctl(S->efd, EPOLL_CTL_ADD, S->wfd, &ev);
  return S;
}

int oryx_http_port(void* h) { return static_cast<Server*>(h)->port; }

long long oryx_http_served(void* h) { return static_cast<Server*>(h)->served.load(); }

// The next request, packed into out as
//   [u64 id][u32 method len][u32 target len][u32 headers len][u64 body len]
//   method target headers ("Name: value\r\n" lines) body
// Waits up to timeout_ms.  Returns the packed size, 0 on timeout, -1 once the server is
// stopping, or -(size needed) when out is too small (the request stays queued).
//
// Leader / followers: there is no loop thread.  A caller finding no request ready becomes
// the poller if no other thread is (the others wait); when its poll returns it hands the
// poller role on (waking one waiting thread) and takes the first request itself -- so at low
// concurrency a request goes from the socket to its handler on the same thread, with no
// thread wake-up in between.
long long oryx_http_next(void* h, char* out, long long cap, int timeout_ms) {
  auto* S = static_cast<Server*>(h);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  std::unique_lock<std::mutex> l(S->qmu);
  for (;;) {
    if (S->stop.load()) return -1;
    if (!S->ready.empty()) break;
    const auto now = std::chrono::steady_clock::now();
    if (now >= deadline) return 0;
    if (!S->leader) {
      S->leader = true;
      l.unlock();
      const long long left =
          std::chrono::duration_cast<std::chrono::milliseconds>(deadline - now).count();
      poll_once(S, (int)std::max<long long>(1, std::min<long long>(left, 50)));
      l.lock();
      S->leader = false;
      S->qcv.notify_one();     // the next poller (or a taker of further ready requests)
      continue;
    }
    S->qcv.wait_until(l, deadline);
  }
  const Req& r = S->ready.front();
  const long long need = 28 + (long long)(r.method.size() + r.target.size() + r.headers.size() +
                                          r.body.size());
  if (need > cap) return -need;
  char* o = out;
  const uint64_t id = r.id;
  const uint32_t ml = (uint32_t)r.method.size(), tl = (uint32_t)r.target.size(),
                 hl = (uint32_t)r.headers.size();
  const uint64_t bl = r.body.size();
  memcpy(o, &id, 8); memcpy(o + 8, &ml, 4); memcpy(o + 12, &tl, 4); memcpy(o + 16, &hl, 4);
  memcpy(o + 20, &bl, 8);
  o += 28;
  memcpy(o, r.method.data(), ml); o += ml;
  memcpy(o, r.target.data(), tl); o += tl;
  memcpy(o, r.headers.data(), hl); o += hl;
  memcpy(o, r.body.data(), bl);
  S->ready.pop_front();
  if (!S->ready.empty()) S->qcv.notify_one();
  return need;
}

// The complete response (status line, headers, body) to request `id`; close: end the
// connection after it.  Returns 0.
int oryx_http_respond(void* h, unsigned long long id, const char* data, long long len,
                      int close_after) {
  auto* S = static_cast<Server*>(h);
  std::string bytes(data, (size_t)len);
  std::lock_guard<std::mutex> g(S->cmu);
  S->served.fetch_add(1);
  auto it = S->inflight.find(id);
  if (it == S->inflight.end()) return 0;
  const uint64_t cid = it->second.first, seq = it->second.second;
  S->inflight.erase(it);
  auto ft = S->fd_of_cid.find(cid);
  if (ft == S->fd_of_cid.end()) return 0;                // the client went away
  auto ct = S->conns.find(ft->second);
  if (ct == S->conns.end()) return 0;
  Conn* c = ct->second.get();
  c->done[seq] = {std::move(bytes), close_after != 0};
  // written from this thread when it is the connection's next response (the socket is
  // non-blocking: what does not fit now is written by the loop on EPOLLOUT)
  flush_conn(S, c);
  return 0;
}

// Stops the loop, closes every connection; blocked oryx_http_next calls return -1.
void oryx_http_stop(void* h) {
  auto* S = static_cast<Server*>(h);
  if (!S || S->stop.exchange(true)) return;
  const uint64_t one = 1;
  (void)!write(S->wfd, &one, sizeof(one));     // ends a poll in progress
  {
    std::unique_lock<std::mutex> l(S->qmu);
    S->qcv.notify_all();
    S->qcv.wait_for(l, std::chrono::seconds(5), [&] { return !S->leader; });
  }
  std::lock_guard<std::mutex> g(S->cmu);
  for (auto& kv : S->conns) close(kv.first);
  S->conns.clear();
  close(S->lfd);
  close(S->efd);
  close(S->wfd);
}

// Frees a stopped server (no handler thread may still use it).
void oryx_http_free(void* h) { delete static_cast<Server*>(h); }

}  // extern "C"
