// oryx_http.cpp -- the serving layer's native HTTP/1.1 (and HTTPS) front end.
//
// The reference serves its REST endpoints from embedded Tomcat ([lserving]/ServingLayer.java:
// 194-245: one NIO connector, HTTP or HTTPS, with its own acceptor and poller threads in front
// of the servlet worker pool).  Here the sockets are polled by the handler threads themselves
// (leader / followers, see oryx_http_next): the poller accepts connections and parses requests
// (request line, headers, Content-Length or chunked bodies, keep-alive and pipelining);
// complete requests wait in a queue that the Python handler threads take from (oryx_http_next
// blocks without the GIL), and their responses come back as ready bytes (oryx_http_respond)
// that are written in request order per connection.  So the Python side does only routing and
// the endpoint's own work per request: no per-connection thread, no header parsing in Python,
// no socket calls.
//
// HTTPS (oryx_http_tls): the same loop with an OpenSSL session per connection in non-blocking
// mode -- the handshake runs inside the first reads and writes, a read that needs a write (or
// the reverse) waits for the matching epoll event.  Every SSL call on a connection is made
// under the connection-table lock, so a session is never used by two threads at once.
//
// Limits: headers <= 64 KB (431); bodies <= max_body (413), checked before they are buffered:
// a Content-Length above it, a chunk size that does not parse or that would take the body past
// it (written without the addition, so huge sizes cannot wrap) all end the connection.
// Chunked bodies are parsed incrementally (the state lives on the connection), so a body sent
// in many small pieces costs linear time.

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
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

#include "oryx_keystore.h"

namespace {

constexpr size_t kMaxHeader = 64 * 1024;

struct Req {
  uint64_t id = 0;
  std::string method, target, headers, body;
};

// chunked-body parse state
enum ChunkState { kSize, kData, kDataEnd, kTrailers };

struct Conn {
  int fd = -1;
  uint64_t cid = 0;
  SSL* ssl = nullptr;              // HTTPS session (null: plain HTTP)
  bool ssl_rd_wants_out = false;   // the last SSL_read needs the socket writable
  bool ssl_wr_wants_in = false;    // the last SSL_write needs the socket readable
  std::string in;                  // unparsed input
  size_t scan = 0;                 // header-end search resumes here
  // a request whose headers are parsed and whose body is still arriving
  bool in_body = false, chunked = false, close_after = false;
  long long body_len = 0;
  ChunkState cstate = kSize;
  long long chunk_left = 0;        // bytes of the current chunk still to come
  size_t trailer_bytes = 0;
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
  SSL_CTX* tls = nullptr;
  std::atomic<bool> stop{false};
  // requests ready for the handlers; `leader`: a handler thread is polling the sockets
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<Req> ready;
  bool leader = false;
  // connection state: taken by the poller per event and by a handler thread that writes its
  // response straight to the socket (oryx_http_respond: no hop through the poller)
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

// ---- transport: plain socket or TLS session.  Return > 0 bytes, 0 at EOF, -1 when the call
// would block (the connection's ssl_*_wants_* flags say on what), -2 on an error.
// The connection BIO of a TLS socket: OpenSSL's socket BIO writes with plain send(), which
// raises SIGPIPE in whichever thread writes to a connection the client already closed (a
// handler thread answering a vanished client); this one sends with MSG_NOSIGNAL and reads
// with recv(), keeping the socket BIO's retry semantics (EAGAIN / EINTR -> retry).
int nosig_write(BIO* b, const char* p, int n) {
  const int fd = (int)BIO_get_fd(b, nullptr);
  const ssize_t w = send(fd, p, (size_t)n, MSG_NOSIGNAL);
  BIO_clear_retry_flags(b);
  if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR))
    BIO_set_retry_write(b);
  return (int)w;
}

int nosig_read(BIO* b, char* p, int n) {
  const int fd = (int)BIO_get_fd(b, nullptr);
  const ssize_t r = recv(fd, p, (size_t)n, 0);
  BIO_clear_retry_flags(b);
  if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR))
    BIO_set_retry_read(b);
  return (int)r;
}

long nosig_ctrl(BIO* b, int cmd, long num, void* ptr) {
  switch (cmd) {
    case BIO_C_SET_FD:
      BIO_set_data(b, reinterpret_cast<void*>((intptr_t) * static_cast<int*>(ptr)));
      BIO_set_init(b, 1);
      return 1;
    case BIO_C_GET_FD: {
      const int fd = BIO_get_init(b) ? (int)reinterpret_cast<intptr_t>(BIO_get_data(b)) : -1;
      if (ptr) *static_cast<int*>(ptr) = fd;
      return fd;
    }
    case BIO_CTRL_FLUSH:
      return 1;
    default:
      (void)num;
      return 0;
  }
}

BIO_METHOD* nosig_method() {
  static BIO_METHOD* m = [] {
    BIO_METHOD* x = BIO_meth_new(BIO_get_new_index() | BIO_TYPE_SOURCE_SINK |
                                     BIO_TYPE_DESCRIPTOR,
                                 "oryx socket (MSG_NOSIGNAL)");
    BIO_meth_set_write(x, nosig_write);
    BIO_meth_set_read(x, nosig_read);
    BIO_meth_set_ctrl(x, nosig_ctrl);
    return x;
  }();
  return m;
}

ssize_t conn_recv(Conn* c, char* buf, size_t n) {
  if (!c->ssl) {
    for (;;) {
      const ssize_t r = recv(c->fd, buf, n, 0);
      if (r >= 0) return r;
      if (errno == EINTR) continue;
      return (errno == EAGAIN || errno == EWOULDBLOCK) ? -1 : -2;
    }
  }
  c->ssl_rd_wants_out = false;
  ERR_clear_error();
  const int r = SSL_read(c->ssl, buf, (int)std::min<size_t>(n, 1 << 30));
  if (r > 0) return r;
  switch (SSL_get_error(c->ssl, r)) {
    case SSL_ERROR_WANT_READ: return -1;
    case SSL_ERROR_WANT_WRITE: c->ssl_rd_wants_out = true; return -1;
    case SSL_ERROR_ZERO_RETURN: return 0;
    case SSL_ERROR_SYSCALL:
      if (errno == EINTR || errno == EAGAIN) return -1;
      return 0;
    default: return -2;
  }
}

ssize_t conn_send(Conn* c, const char* p, size_t n) {
  if (!c->ssl) {
    for (;;) {
      const ssize_t w = send(c->fd, p, n, MSG_NOSIGNAL);
      if (w >= 0) return w;
      if (errno == EINTR) continue;
      return (errno == EAGAIN || errno == EWOULDBLOCK) ? -1 : -2;
    }
  }
  c->ssl_wr_wants_in = false;
  ERR_clear_error();
  const int w = SSL_write(c->ssl, p, (int)std::min<size_t>(n, 1 << 30));
  if (w > 0) return w;
  switch (SSL_get_error(c->ssl, w)) {
    case SSL_ERROR_WANT_WRITE: return -1;
    case SSL_ERROR_WANT_READ: c->ssl_wr_wants_in = true; return -1;
    default: return -2;
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
  c->in.clear();
  (void)S;
}

void close_conn(Server* S, int fd) {
  auto it = S->conns.find(fd);
  if (it == S->conns.end()) return;
  Conn* c = it->second.get();
  S->fd_of_cid.erase(c->cid);
  epoll_ctl(S->efd, EPOLL_CTL_DEL, fd, nullptr);
  if (c->ssl) {
    SSL_shutdown(c->ssl);          // best effort close_notify (non-blocking socket)
    SSL_free(c->ssl);
    c->ssl = nullptr;
  }
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
    const ssize_t w = conn_send(c, c->out.data() + c->out_off, c->out.size() - c->out_off);
    if (w > 0) {
      c->out_off += (size_t)w;
      continue;
    }
    if (w == -1) {
      // blocked: on writability (or, TLS, on readability: the poller retries on EPOLLIN)
      want_write(S, c, !c->ssl_wr_wants_in || c->ssl_rd_wants_out);
      return true;
    }
    close_conn(S, c->fd);
    return false;
  }
  want_write(S, c, c->ssl_rd_wants_out);
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

// Parses a chunk-size line "HEX[;ext]": true and the size when it is 1-15 hex digits.
bool parse_chunk_size(const char* s, size_t n, long long& out) {
  size_t k = 0;
  long long v = 0;
  while (k < n && isxdigit((unsigned char)s[k])) {
    if (k == 15) return false;     // > 2^60: no body is that large (and no overflow below)
    const char ch = s[k];
    const int d = ch <= '9' ? ch - '0' : (tolower((unsigned char)ch) - 'a' + 10);
    v = v * 16 + d;
    ++k;
  }
  if (k == 0) return false;
  while (k < n && (s[k] == ' ' || s[k] == '\t')) ++k;
  if (k < n && s[k] != ';') return false;
  out = v;
  return true;
}

// Consumes what c->in holds of a chunked body, from its front: chunk sizes, data (appended
// to the request body), the CRLF after each chunk, trailers.  Returns 1 when the body is
// complete, 0 when more input is needed, or an HTTP error status.
int parse_chunked(Server* S, Conn* c) {
  size_t p = 0;
  int rc = 0;
  for (;;) {
    if (c->cstate == kSize) {
      const size_t le = c->in.find("\r\n", p);
      if (le == std::string::npos) {
        if (c->in.size() - p > 1024) rc = 400;     // a size line is short
        break;
      }
      long long sz = 0;
      if (!parse_chunk_size(c->in.data() + p, le - p, sz)) {
        rc = 400;
        break;
      }
      // sz > max_body - body: the remaining allowance, never a sum that could wrap
      if (sz > S->max_body - (long long)c->cur.body.size()) {
        rc = 413;
        break;
      }
      p = le + 2;
      if (sz == 0) {
        c->cstate = kTrailers;
        c->trailer_bytes = 0;
      } else {
        c->cstate = kData;
        c->chunk_left = sz;
      }
    } else if (c->cstate == kData) {
      const size_t avail = c->in.size() - p;
      if (avail == 0) break;
      const size_t take = (size_t)std::min<long long>(c->chunk_left, (long long)avail);
      c->cur.body.append(c->in, p, take);
      p += take;
      c->chunk_left -= (long long)take;
      if (c->chunk_left == 0) c->cstate = kDataEnd;
    } else if (c->cstate == kDataEnd) {
      if (c->in.size() - p < 2) break;
      if (c->in[p] != '\r' || c->in[p + 1] != '\n') {
        rc = 400;
        break;
      }
      p += 2;
      c->cstate = kSize;
    } else {   // trailers: header lines up to an empty line
      const size_t nl = c->in.find("\r\n", p);
      if (nl == std::string::npos) {
        if (c->trailer_bytes + (c->in.size() - p) > kMaxHeader) rc = 431;
        break;
      }
      c->trailer_bytes += nl + 2 - p;
      if (c->trailer_bytes > kMaxHeader) {
        rc = 431;
        break;
      }
      const bool end = nl == p;
      p = nl + 2;
      if (end) {
        c->cstate = kSize;
        rc = 1;
        break;
      }
    }
  }
  c->in.erase(0, p);
  return rc;
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
      if (e > kMaxHeader) {
        loop_error(S, c, 431);
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
            errno = 0;
            c->body_len = strtoll(v.c_str(), &endp, 10);
            if (v.empty() || *endp || c->body_len < 0 || errno == ERANGE) {
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
      c->cstate = kSize;
      // a client that waits for "100 Continue" before its body gets it at once (when no
      // earlier response on the connection is still due, which it would have to follow)
      if (expect_continue && (c->chunked || (long long)c->in.size() < c->body_len) &&
          c->next_out == c->next_seq && c->out.empty()) {
        static const char k100[] = "HTTP/1.1 100 Continue\r\n\r\n";
        (void)conn_send(c, k100, sizeof(k100) - 1);
      }
    }
    // body
    if (c->chunked) {
      const int rc = parse_chunked(S, c);
      if (rc == 0) return;                       // need more
      if (rc != 1) {
        loop_error(S, c, rc);
        return;
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
      c->in.clear();
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
          if (S->tls) {
            c->ssl = SSL_new(S->tls);
            BIO* bio = c->ssl ? BIO_new(nosig_method()) : nullptr;
            if (!bio) {
              if (c->ssl) SSL_free(c->ssl);
              close(cfd);
              continue;
            }
            int fd_arg = cfd;
            BIO_ctrl(bio, BIO_C_SET_FD, 0, &fd_arg);
            SSL_set_bio(c->ssl, bio, bio);   // (the SSL owns the BIO; the fd stays ours)
            SSL_set_accept_state(c->ssl);   // the handshake runs inside the first read
          }
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
      const uint32_t e = evs[k].events;
      // a TLS write blocked on readability retries on any event; so does a TLS read blocked
      // on writability (both below)
      if ((e & EPOLLOUT) || (c->ssl && c->ssl_wr_wants_in)) {
        if (!flush_conn(S, c)) continue;
      }
      if ((e & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) ||
          (c->ssl && c->ssl_rd_wants_out && (e & EPOLLOUT))) {
        bool eof = false;
        for (;;) {
          const ssize_t r = conn_recv(c, buf, sizeof(buf));
          if (r > 0) {
            if (!c->read_shut) {
              c->in.append(buf, (size_t)r);
              // parse as the bytes arrive: complete requests and chunk data leave c->in, so
              // what it holds stays bounded by one header block or one Content-Length body
              parse_input(S, c);
            }
            continue;
          }
          if (r == 0 || r == -2) eof = true;
          break;
        }
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

int tls_password_cb(char* buf, int size, int, void* u) {
  const char* pw = static_cast<const char*>(u);
  if (!pw) return 0;
  const int n = (int)std::min<size_t>(strlen(pw), (size_t)size);
  memcpy(buf, pw, (size_t)n);
  return n;
}

thread_local std::string tls_err;

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

// Serves HTTPS on the server's socket.  `cert` is a Java keystore -- JKS or PKCS#12, as the
// reference's keystore-file (oryx_keystore.cpp), `password` its keystore-password -- or a PEM
// certificate chain with private key `key` (null or empty: the key is in `cert`) and
// `password` for an encrypted key (may be null).  TLS 1.2 is the minimum (the reference's
// connector allows TLSv1.2 and 1.1; 1.1 is deprecated).  Call before the first
// oryx_http_next.  Returns 0, or -1 (oryx_http_tls_error says why).
int oryx_http_tls(void* h, const char* cert, const char* key, const char* password) {
  auto* S = static_cast<Server*>(h);
  tls_err.clear();
  SSL_CTX* ctx = SSL_CTX_new(TLS_server_method());
  if (!ctx) {
    tls_err = "SSL_CTX_new failed";
    return -1;
  }
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  // (no SSL_MODE_RELEASE_BUFFERS: a keep-alive connection would free and re-allocate its
  // record buffers around every request)
  SSL_CTX_set_mode(ctx, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  SSL_CTX_set_options(ctx, SSL_OP_NO_RENEGOTIATION);
  std::string pw = password ? password : "";
  SSL_CTX_set_default_passwd_cb(ctx, tls_password_cb);
  SSL_CTX_set_default_passwd_cb_userdata(ctx, password ? (void*)pw.c_str() : nullptr);
  const char* kf = key && *key ? key : cert;
  auto fail = [&](const char* what) {
    char eb[256];
    ERR_error_string_n(ERR_get_error(), eb, sizeof(eb));
    tls_err = std::string(what) + ": " + eb;
    SSL_CTX_free(ctx);
    return -1;
  };
  EVP_PKEY* ks_key = nullptr;
  X509* ks_cert = nullptr;
  STACK_OF(X509)* ks_chain = nullptr;
  std::string ks_why;
  const int ks = oryx::keystore_load(cert, password, nullptr, &ks_key, &ks_cert, &ks_chain,
                                     &ks_why);
  if (ks == oryx::kKeystoreOk) {
    // certificate, chain and key straight from the keystore (no PEM files)
    int ok = SSL_CTX_use_certificate(ctx, ks_cert) == 1 && SSL_CTX_use_PrivateKey(ctx, ks_key) == 1;
    for (int i = 0; ok && i < sk_X509_num(ks_chain); ++i)
      ok = SSL_CTX_add1_chain_cert(ctx, sk_X509_value(ks_chain, i)) == 1;
    EVP_PKEY_free(ks_key);
    X509_free(ks_cert);
    sk_X509_pop_free(ks_chain, X509_free);
    if (!ok) return fail("keystore");
  } else if (ks != oryx::kKeystoreNotKeystore) {
    tls_err = ks_why;
    SSL_CTX_free(ctx);
    return -1;
  } else {
    if (SSL_CTX_use_certificate_chain_file(ctx, cert) != 1) return fail("certificate");
    if (SSL_CTX_use_PrivateKey_file(ctx, kf, SSL_FILETYPE_PEM) != 1) return fail("private key");
  }
  if (SSL_CTX_check_private_key(ctx) != 1) return fail("key does not match certificate");
  // the password is only needed while loading
  SSL_CTX_set_default_passwd_cb_userdata(ctx, nullptr);
  std::lock_guard<std::mutex> g(S->cmu);
  if (S->tls) SSL_CTX_free(S->tls);
  S->tls = ctx;
  return 0;
}

const char* oryx_http_tls_error() { return tls_err.c_str(); }

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
    // timed waits on the system clock (pthread_cond_timedwait): the steady-clock form maps to
    // pthread_cond_clockwait, which ThreadSanitizer's runtime does not intercept
    S->qcv.wait_until(l, std::chrono::system_clock::now() + (deadline - now));
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
  // non-blocking: what does not fit now is written by the poller on EPOLLOUT)
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
    S->qcv.wait_until(l, std::chrono::system_clock::now() + std::chrono::seconds(5),
                      [&] { return !S->leader; });
  }
  std::lock_guard<std::mutex> g(S->cmu);
  for (auto& kv : S->conns) {
    if (kv.second->ssl) SSL_free(kv.second->ssl);
    close(kv.first);
  }
  S->conns.clear();
  close(S->lfd);
  close(S->efd);
  close(S->wfd);
}

// Frees a stopped server (no handler thread may still use it).
void oryx_http_free(void* h) {
  auto* S = static_cast<Server*>(h);
  if (S && S->tls) SSL_CTX_free(S->tls);
  delete S;
}

}  // extern "C"
