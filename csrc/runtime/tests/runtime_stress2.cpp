// runtime_stress2.cpp -- the round-4 native concurrency code under sanitizer builds
// (SURVEY.md section 5.2), alongside runtime_stress.cpp:
//
//   1. oryx_log_append_fill: writer threads on two topic handles whose fill callbacks format
//      the values straight into the mapped segment (the speed layer's hot path; fill runs on
//      the native pool for large appends), small segments so that appends roll; at the same
//      time a frame reader (oryx_reader_poll_frames) and a text reader (oryx_reader_read_text)
//      tail the partition across the rolls and check every record's content and order;
//   2. the native HTTP front end (oryx_http.cpp) with four handler threads (leader /
//      followers) and concurrent clients: keep-alive request loops, pipelined bursts, chunked
//      bodies sent in small pieces, 413 (oversized Content-Length and chunk size) and 431
//      (header flood), 400 (bad chunk size), and clients that close abruptly mid-request or
//      before reading their responses;
//   3. oryx_topn_prep from several threads at once on shared inputs (LSH bitmaps, exclusions);
//   4. the persistent ThreadPool (parallel_ranges) entered from several threads at once
//      (oryx_blob_hash64 and oryx_digest128 split their work over it);
//   5. the HTTP front end with TLS (oryx_http_tls: OpenSSL in non-blocking mode inside the
//      same leader / follower loop) under concurrent TLS clients: keep-alive pipelined
//      requests, handshakes abandoned halfway, plain HTTP sent to the TLS port, and clients
//      that close right after sending.  Needs a certificate: runtime_stress2 <dir> <cert> <key>.
//
// Exit status 0 = no check failed.

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <openssl/err.h>
#include <openssl/ssl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <random>
#include <cmath>
#include <algorithm>
#include <thread>
#include <vector>

extern "C" {
void* oryx_log_open(const char*, const char*, int, long long, long long);
void oryx_log_close(void*);
const char* oryx_log_last_error();
typedef void (*FillFn)(void* ctx, long long j, char* dst);
long long oryx_log_append_fill(void* h, int partition, const char* key, int key_len,
                               const long long* lens, int n, FillFn fill, void* ctx,
                               long long ts_ms, int do_fsync);
void* oryx_reader_open(void*, int, long long);
void oryx_reader_close(void*);
long long oryx_reader_poll_frames(void* rh, char* out, long long out_cap, int max_records,
                                  long long* out_used);
long long oryx_reader_read_text(void* rh, long long end_offset, char* out, long long out_cap,
                                long long* out_used, int* flags);
void* oryx_http_start(const char* host, int port, int backlog, long long max_body);
int oryx_http_port(void* h);
long long oryx_http_next(void* h, char* out, long long cap, int timeout_ms);
int oryx_http_respond(void* h, unsigned long long id, const char* data, long long len,
                      int close_after);
void oryx_http_stop(void* h);
int oryx_http_tls(void* h, const char* cert, const char* key, const char* password);
void oryx_http_free(void* h);
int oryx_keystore_to_pem(const char* path, const char* password, const char* alias,
                         char** cert_pem, long long* cert_len, char** key_pem,
                         long long* key_len);
void oryx_keystore_free(char* p);
const char* oryx_keystore_error();
long long oryx_topn_prep(int nq, int k, int kp, int max_batch, const float* targets,
                         const long long* cand_ptr, const long long* cand,
                         const unsigned char* cand_all, int num_buckets, int words,
                         const long long* bucket_start, long long n_rows, const long long* ex_ptr,
                         const long long* ex_rows, const long long* pos_of_row, long long n_pos,
                         long long delta_lo, long long delta_hi,
                         unsigned char* out, long long out_cap, long long* info);
void oryx_blob_hash64(const unsigned char* blob, const long long* ends, long long n,
                      unsigned long long seed, unsigned long long* out);
void oryx_digest128(const unsigned char* p, long long n, unsigned long long* out);
void* oryx_hostbuf_alloc(long long n);
void oryx_hostbuf_free(void* p, long long n);
void oryx_hostbuf_stats(long long* out);
long long oryx_hostbuf_quiesce(long long timeout_ms);
long long oryx_read_file_parallel(const char* path, char* out, long long n, int threads);
long long oryx_encode_spans(const char* base, const long long* off, const int* len, long long n,
                            long long stride, long long* codes, long long* first_row);
void* oryx_rowmap_new();
void oryx_rowmap_free(void* h);
void oryx_rowmap_set(void* h, const char* blob, const long long* ends, const long long* rows,
                     long long n);
void* oryx_speed_new();
void oryx_speed_free(void* h);
long long oryx_speed_parse(void* h, const char* buf, long long len, void* xm, void* ym,
                           long long default_ts);
long long oryx_speed_aggregate(void* h, int implicit, long long* out_u, long long* out_i,
                               double* out_s);
long long oryx_speed_counts(void* h, long long* out);
}

static std::atomic<int> g_errors{0};

#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_errors;                                                      \
    }                                                                  \
  } while (0)

// ---------------------------------------------------------------- 1. append_fill + readers

struct FillCtx {
  int writer, batch;
};

static std::string value_of(int w, int b, long long j) {
  char buf[64];
  const int n = snprintf(buf, sizeof(buf), "[\"X\",\"w%d-b%d-%lld\",%lld]", w, b, j, j * 7);
  std::string s(buf, (size_t)n);
  s.append((size_t)(j % 37), 'z');
  return s;
}

static void fill_fn(void* ctx, long long j, char* dst) {
  const auto* c = static_cast<const FillCtx*>(ctx);
  const std::string v = value_of(c->writer, c->batch, j);
  memcpy(dst, v.data(), v.size());
}

static void test_append_fill(const char* root) {
  const int writers = 2, batches = 6, n = 3000;
  const long long total = (long long)writers * batches * n;
  void* t1 = oryx_log_open(root, "Fill", 1, 1 << 20, 256 << 10);   // 256 KB segments: rolls
  void* t2 = oryx_log_open(root, "Fill", 1, 1 << 20, 256 << 10);
  CHECK(t1 && t2);
  if (!t1 || !t2) return;
  std::atomic<bool> done{false};
  std::vector<std::thread> th;
  for (int w = 0; w < writers; ++w) {
    th.emplace_back([&, w] {
      for (int b = 0; b < batches; ++b) {
        std::vector<long long> lens((size_t)n);
        for (long long j = 0; j < n; ++j) lens[(size_t)j] = (long long)value_of(w, b, j).size();
        FillCtx c{w, b};
        CHECK(oryx_log_append_fill(w ? t2 : t1, 0, "UP", 2, lens.data(), n, fill_fn, &c, -1,
                                   0) >= 0);
      }
    });
  }
  // frame reader: every frame's value parses back to its (writer, batch, j) and, per writer,
  // the batches arrive whole and in order
  th.emplace_back([&] {
    void* r = oryx_reader_open(t1, 0, 0);
    std::vector<char> out(1 << 20);
    long long got = 0, last_off = -1;
    auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    while (got < total && std::chrono::steady_clock::now() < t_end) {
      long long used = 0;
      const long long n_fr = oryx_reader_poll_frames(r, out.data(), (long long)out.size(), 4096,
                                                     &used);
      CHECK(n_fr >= 0);
      if (n_fr <= 0) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        continue;
      }
      long long pos = 0;
      for (long long i = 0; i < n_fr; ++i) {
        uint32_t kl, vl;
        long long off;
        memcpy(&off, out.data() + pos + 8, 8);
        memcpy(&kl, out.data() + pos + 24, 4);
        memcpy(&vl, out.data() + pos + 28, 4);
        CHECK(off == last_off + 1);
        last_off = off;
        CHECK(kl == 2 && memcmp(out.data() + pos + 32, "UP", 2) == 0);
        const char* v = out.data() + pos + 32 + kl;
        int w = -1, b = -1;
        long long j = -1;
        CHECK(sscanf(v, "[\"X\",\"w%d-b%d-%lld\"", &w, &b, &j) == 3);
        if (w >= 0 && b >= 0 && j >= 0) CHECK(value_of(w, b, j) == std::string(v, vl));
        pos += 32 + kl + vl;
      }
      got += n_fr;
    }
    CHECK(got == total);
    oryx_reader_close(r);
  });
  // text reader: the same records as text lines, up to whatever end offset it sees
  th.emplace_back([&] {
    void* r = oryx_reader_open(t2, 0, 0);
    std::vector<char> out(1 << 20);
    long long got = 0;
    auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    while (got < total && std::chrono::steady_clock::now() < t_end) {
      long long used = 0;
      int flags = 0;
      const long long n_rec = oryx_reader_read_text(r, got + 2000, out.data(),
                                                    (long long)out.size(), &used, &flags);
      CHECK(n_rec >= 0);
      if (n_rec <= 0) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        continue;
      }
      long long lines = 0;
      for (long long p = 0; p < used; ++p) lines += out[(size_t)p] == '\n';
      CHECK(lines == n_rec);
      got += n_rec;
    }
    CHECK(got == total);
    oryx_reader_close(r);
  });
  for (auto& x : th) x.join();
  done = true;
  oryx_log_close(t1);
  oryx_log_close(t2);
}

// ---------------------------------------------------------------- 2. HTTP front end

static int connect_to(int port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  timeval tv{10, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  return fd;
}

static bool send_all(int fd, const std::string& s) {
  size_t o = 0;
  while (o < s.size()) {
    const ssize_t w = send(fd, s.data() + o, s.size() - o, MSG_NOSIGNAL);
    if (w <= 0) return false;
    o += (size_t)w;
  }
  return true;
}

// n responses: status codes and bodies
static bool read_responses(int fd, int n, std::vector<int>& st, std::vector<std::string>& bodies) {
  std::string buf;
  char tmp[65536];
  while ((int)st.size() < n) {
    size_t he;
    while ((he = buf.find("\r\n\r\n")) == std::string::npos) {
      const ssize_t r = recv(fd, tmp, sizeof(tmp), 0);
      if (r <= 0) return false;
      buf.append(tmp, (size_t)r);
    }
    const int code = atoi(buf.c_str() + 9);
    size_t cl = 0;
    const size_t p = buf.find("Content-Length: ");
    if (p != std::string::npos && p < he) cl = (size_t)atoll(buf.c_str() + p + 16);
    while (buf.size() < he + 4 + cl) {
      const ssize_t r = recv(fd, tmp, sizeof(tmp), 0);
      if (r <= 0) return false;
      buf.append(tmp, (size_t)r);
    }
    st.push_back(code);
    bodies.push_back(buf.substr(he + 4, cl));
    buf.erase(0, he + 4 + cl);
  }
  return true;
}

static void test_http() {
  void* S = oryx_http_start("127.0.0.1", 0, 256, 1 << 20);
  CHECK(S != nullptr);
  if (!S) return;
  const int port = oryx_http_port(S);
  std::atomic<bool> stop{false};
  std::vector<std::thread> handlers;
  for (int h = 0; h < 4; ++h) {
    handlers.emplace_back([&] {
      std::vector<char> buf(1 << 16);
      while (!stop) {
        long long n = oryx_http_next(S, buf.data(), (long long)buf.size(), 50);
        if (n == -1) return;
        if (n == 0) continue;
        if (n < 0) {
          buf.resize((size_t)-n);
          continue;
        }
        uint64_t id;
        uint32_t ml, tl, hl;
        uint64_t bl;
        memcpy(&id, buf.data(), 8);
        memcpy(&ml, buf.data() + 8, 4);
        memcpy(&tl, buf.data() + 12, 4);
        memcpy(&hl, buf.data() + 16, 4);
        memcpy(&bl, buf.data() + 20, 8);
        const std::string target(buf.data() + 28 + ml, tl);
        const std::string body(buf.data() + 28 + ml + tl + hl, bl);
        const std::string payload = target + "|" + std::to_string(bl) + "|" +
                                    (body.size() > 64 ? body.substr(0, 64) : body);
        const std::string resp = "HTTP/1.1 200 OK\r\nContent-Length: " +
                                 std::to_string(payload.size()) + "\r\n\r\n" + payload;
        oryx_http_respond(S, id, resp.data(), (long long)resp.size(), 0);
      }
    });
  }
  std::vector<std::thread> clients;
  // keep-alive loops with pipelined bursts
  for (int c = 0; c < 6; ++c) {
    clients.emplace_back([&, c] {
      const int fd = connect_to(port);
      CHECK(fd >= 0);
      if (fd < 0) return;
      for (int rep = 0; rep < 20; ++rep) {
        std::string burst;
        for (int j = 0; j < 5; ++j)
          burst += "GET /c" + std::to_string(c) + "/" + std::to_string(rep * 5 + j) +
                   " HTTP/1.1\r\nHost: x\r\n\r\n";
        CHECK(send_all(fd, burst));
        std::vector<int> st;
        std::vector<std::string> b;
        CHECK(read_responses(fd, 5, st, b));
        for (int j = 0; j < (int)b.size(); ++j)
          CHECK(b[(size_t)j].rfind("/c" + std::to_string(c) + "/" +
                                   std::to_string(rep * 5 + j) + "|", 0) == 0);
      }
      close(fd);
    });
  }
  // chunked bodies in small pieces
  for (int c = 0; c < 3; ++c) {
    clients.emplace_back([&, c] {
      const int fd = connect_to(port);
      CHECK(fd >= 0);
      if (fd < 0) return;
      for (int rep = 0; rep < 4; ++rep) {
        std::string req = "POST /chunk HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n";
        std::string want;
        for (int k = 0; k < 300; ++k) {
          const std::string piece(1 + (k + c) % 13, (char)('a' + k % 26));
          char hx[16];
          snprintf(hx, sizeof(hx), "%zx\r\n", piece.size());
          req += hx + piece + "\r\n";
          want += piece;
        }
        req += "0\r\n\r\n";
        for (size_t o = 0; o < req.size(); o += 41) CHECK(send_all(fd, req.substr(o, 41)));
        std::vector<int> st;
        std::vector<std::string> b;
        CHECK(read_responses(fd, 1, st, b));
        if (!b.empty())
          CHECK(b[0] == "/chunk|" + std::to_string(want.size()) + "|" + want.substr(0, 64));
      }
      close(fd);
    });
  }
  // errors: 413 (Content-Length, chunk size), 431 (header flood), 400 (bad chunk size)
  clients.emplace_back([&] {
    const char* reqs[] = {
        "POST /x HTTP/1.1\r\nContent-Length: 99999999\r\n\r\n",
        "POST /x HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n1\r\na\r\nfffffffffffffff\r\n",
        "POST /x HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n"};
    const int want[] = {413, 413, 400};
    for (int k = 0; k < 3; ++k) {
      const int fd = connect_to(port);
      CHECK(fd >= 0);
      if (fd < 0) continue;
      CHECK(send_all(fd, reqs[k]));
      std::vector<int> st;
      std::vector<std::string> b;
      CHECK(read_responses(fd, 1, st, b));
      if (!st.empty()) CHECK(st[0] == want[k]);
      close(fd);
    }
    const int fd = connect_to(port);
    if (fd >= 0) {
      std::string flood = "GET /x HTTP/1.1\r\n";
      while (flood.size() < 70000) flood += "X-Pad: aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa\r\n";
      send_all(fd, flood);
      std::vector<int> st;
      std::vector<std::string> b;
      CHECK(read_responses(fd, 1, st, b));
      if (!st.empty()) CHECK(st[0] == 431);
      close(fd);
    }
  });
  // abrupt closes: mid-headers, mid-body, and after sending without reading the answers
  for (int c = 0; c < 4; ++c) {
    clients.emplace_back([&, c] {
      for (int rep = 0; rep < 25; ++rep) {
        const int fd = connect_to(port);
        if (fd < 0) continue;
        if (c == 0) send_all(fd, "GET /half HTTP/1.1\r\nHo");
        if (c == 1) send_all(fd, "POST /b HTTP/1.1\r\nContent-Length: 100\r\n\r\nabc");
        if (c == 2)
          send_all(fd, "GET /a HTTP/1.1\r\n\r\nGET /b HTTP/1.1\r\n\r\nGET /c HTTP/1.1\r\n\r\n");
        if (c == 3) {
          linger lg{1, 0};   // RST on close
          setsockopt(fd, SOL_SOCKET, SO_LINGER, &lg, sizeof(lg));
          send_all(fd, "GET /rst HTTP/1.1\r\n\r\n");
        }
        close(fd);
      }
    });
  }
  for (auto& x : clients) x.join();
  // the server still answers after all that
  {
    const int fd = connect_to(port);
    CHECK(fd >= 0);
    if (fd >= 0) {
      CHECK(send_all(fd, "GET /final HTTP/1.1\r\n\r\n"));
      std::vector<int> st;
      std::vector<std::string> b;
      CHECK(read_responses(fd, 1, st, b));
      if (!b.empty()) CHECK(b[0].rfind("/final|", 0) == 0);
      close(fd);
    }
  }
  stop = true;
  oryx_http_stop(S);
  for (auto& x : handlers) x.join();
  oryx_http_free(S);
}

// ---------------------------------------------------------------- 3. top-N prep

static void test_topn_prep() {
  const int nq = 8, k = 50, kp = 64, nb = 70, words = (nb + 31) / 32;
  const long long n_rows = 5000;
  std::vector<float> targets((size_t)nq * k);
  for (size_t i = 0; i < targets.size(); ++i) targets[i] = (float)(i % 17) * 0.25f;
  std::vector<long long> bstart(nb + 1);
  for (int b = 0; b <= nb; ++b) bstart[(size_t)b] = n_rows * b / nb;
  std::vector<long long> cand_ptr(nq + 1, 0), cand;
  std::vector<unsigned char> cand_all(nq, 0);
  for (int j = 0; j < nq; ++j) {
    for (int b = j; b < nb; b += 3 + j) cand.push_back(b);
    cand.push_back(-5);          // ignored
    cand.push_back(nb + 9);      // ignored
    cand_ptr[(size_t)j + 1] = (long long)cand.size();
  }
  cand_all[5] = 1;
  std::vector<long long> ex_ptr(nq + 1, 0), ex_rows, pos_of_row((size_t)n_rows);
  for (long long r = 0; r < n_rows; ++r) pos_of_row[(size_t)r] = (r * 7919) % n_rows;
  for (int j = 0; j < nq; ++j) {
    for (int e = 0; e < 40; ++e) ex_rows.push_back((j * 131 + e * 977) % (n_rows + 50) - 10);
    ex_ptr[(size_t)j + 1] = (long long)ex_rows.size();
  }
  auto run = [&](std::vector<unsigned char>& out, std::vector<long long>& info) {
    out.assign(1 << 20, 0);
    info.assign(9, 0);
    return oryx_topn_prep(nq, k, kp, 16, targets.data(), cand_ptr.data(), cand.data(),
                          cand_all.data(), nb, words, bstart.data(), n_rows, ex_ptr.data(),
                          ex_rows.data(), pos_of_row.data(), n_rows, n_rows - 300, n_rows,
                          out.data(), (long long)out.size(), info.data());
  };
  std::vector<unsigned char> ref;
  std::vector<long long> ref_info;
  CHECK(run(ref, ref_info) == 0);
  {
    std::vector<unsigned char> small(64);
    std::vector<long long> info(9);
    CHECK(oryx_topn_prep(nq, k, kp, 16, targets.data(), cand_ptr.data(), cand.data(),
                         cand_all.data(), nb, words, bstart.data(), n_rows, ex_ptr.data(),
                         ex_rows.data(), pos_of_row.data(), n_rows, 0, 0, small.data(),
                         (long long)small.size(), info.data()) == -1);
  }
  std::vector<std::thread> th;
  for (int t = 0; t < 6; ++t) {
    th.emplace_back([&] {
      for (int rep = 0; rep < 50; ++rep) {
        std::vector<unsigned char> out;
        std::vector<long long> info;
        CHECK(run(out, info) == 0);
        CHECK(info == ref_info);
        CHECK(memcmp(out.data(), ref.data(), (size_t)ref_info[7]) == 0);
      }
    });
  }
  for (auto& x : th) x.join();
}

// ---------------------------------------------------------------- 4. thread pool

static void test_pool() {
  std::string blob;
  std::vector<long long> ends;
  for (int i = 0; i < 200000; ++i) {
    blob += "user-" + std::to_string(i * 31);
    ends.push_back((long long)blob.size());
  }
  std::vector<unsigned long long> ref(ends.size());
  oryx_blob_hash64((const unsigned char*)blob.data(), ends.data(), (long long)ends.size(), 9,
                   ref.data());
  std::vector<unsigned char> big(64 << 20);
  for (size_t i = 0; i < big.size(); ++i) big[i] = (unsigned char)(i * 2654435761u >> 13);
  unsigned long long dref[2];
  oryx_digest128(big.data(), (long long)big.size(), dref);
  std::vector<std::thread> th;
  for (int t = 0; t < 6; ++t) {
    th.emplace_back([&, t] {
      for (int rep = 0; rep < 8; ++rep) {
        if ((t + rep) & 1) {
          std::vector<unsigned long long> h(ends.size());
          oryx_blob_hash64((const unsigned char*)blob.data(), ends.data(),
                           (long long)ends.size(), 9, h.data());
          CHECK(h == ref);
        } else {
          unsigned long long d[2];
          oryx_digest128(big.data(), (long long)big.size(), d);
          CHECK(d[0] == dref[0] && d[1] == dref[1]);
        }
      }
    });
  }
  for (auto& x : th) x.join();
}

// ---------------------------------------------------------------- 5. HTTPS

static void serve(void* S, std::atomic<bool>& stop, std::vector<std::thread>& handlers) {
  for (int h = 0; h < 4; ++h) {
    handlers.emplace_back([S, &stop] {
      std::vector<char> buf(1 << 16);
      while (!stop) {
        long long n = oryx_http_next(S, buf.data(), (long long)buf.size(), 50);
        if (n == -1) return;
        if (n == 0) continue;
        if (n < 0) {
          buf.resize((size_t)-n);
          continue;
        }
        uint64_t id;
        uint32_t ml, tl;
        memcpy(&id, buf.data(), 8);
        memcpy(&ml, buf.data() + 8, 4);
        memcpy(&tl, buf.data() + 12, 4);
        const std::string target(buf.data() + 28 + ml, tl);
        const std::string resp = "HTTP/1.1 200 OK\r\nContent-Length: " +
                                 std::to_string(target.size()) + "\r\n\r\n" + target;
        oryx_http_respond(S, id, resp.data(), (long long)resp.size(), 0);
      }
    });
  }
}

static bool ssl_write_all(SSL* ssl, const std::string& s) {
  size_t o = 0;
  while (o < s.size()) {
    const int w = SSL_write(ssl, s.data() + o, (int)(s.size() - o));
    if (w <= 0) return false;
    o += (size_t)w;
  }
  return true;
}

static bool ssl_read_responses(SSL* ssl, int n, std::vector<std::string>& bodies) {
  std::string buf;
  char tmp[16384];
  while ((int)bodies.size() < n) {
    size_t he;
    while ((he = buf.find("\r\n\r\n")) == std::string::npos) {
      const int r = SSL_read(ssl, tmp, sizeof(tmp));
      if (r <= 0) return false;
      buf.append(tmp, (size_t)r);
    }
    size_t cl = 0;
    const size_t p = buf.find("Content-Length: ");
    if (p != std::string::npos && p < he) cl = (size_t)atoll(buf.c_str() + p + 16);
    while (buf.size() < he + 4 + cl) {
      const int r = SSL_read(ssl, tmp, sizeof(tmp));
      if (r <= 0) return false;
      buf.append(tmp, (size_t)r);
    }
    bodies.push_back(buf.substr(he + 4, cl));
    buf.erase(0, he + 4 + cl);
  }
  return true;
}

static void test_https(const char* cert, const char* key) {
  void* S = oryx_http_start("127.0.0.1", 0, 256, 1 << 20);
  CHECK(S != nullptr);
  if (!S) return;
  CHECK(oryx_http_tls(S, cert, key, nullptr) == 0);
  const int port = oryx_http_port(S);
  std::atomic<bool> stop{false};
  std::vector<std::thread> handlers;
  serve(S, stop, handlers);
  SSL_CTX* cctx = SSL_CTX_new(TLS_client_method());
  SSL_CTX_set_verify(cctx, SSL_VERIFY_NONE, nullptr);
  std::vector<std::thread> clients;
  // keep-alive TLS connections with pipelined bursts
  for (int c = 0; c < 6; ++c) {
    clients.emplace_back([&, c] {
      const int fd = connect_to(port);
      CHECK(fd >= 0);
      if (fd < 0) return;
      SSL* ssl = SSL_new(cctx);
      SSL_set_fd(ssl, fd);
      CHECK(SSL_connect(ssl) == 1);
      for (int rep = 0; rep < 15; ++rep) {
        std::string burst;
        for (int j = 0; j < 4; ++j)
          burst += "GET /t" + std::to_string(c) + "/" + std::to_string(rep * 4 + j) +
                   " HTTP/1.1\r\nHost: x\r\n\r\n";
        CHECK(ssl_write_all(ssl, burst));
        std::vector<std::string> b;
        CHECK(ssl_read_responses(ssl, 4, b));
        for (int j = 0; j < (int)b.size(); ++j)
          CHECK(b[(size_t)j] == "/t" + std::to_string(c) + "/" + std::to_string(rep * 4 + j));
      }
      SSL_shutdown(ssl);
      SSL_free(ssl);
      close(fd);
    });
  }
  // abandoned handshakes, plain HTTP to the TLS port, closes right after a request
  for (int c = 0; c < 3; ++c) {
    clients.emplace_back([&, c] {
      for (int rep = 0; rep < 15; ++rep) {
        const int fd = connect_to(port);
        if (fd < 0) continue;
        if (c == 0) {
          send_all(fd, std::string("\x16\x03\x01\x02\x00\x01\x00\x01\xfc\x03\x03", 11));
        } else if (c == 1) {
          send_all(fd, "GET /plain HTTP/1.1\r\nHost: x\r\n\r\n");
          char tmp[256];
          (void)recv(fd, tmp, sizeof(tmp), 0);
        } else {
          SSL* ssl = SSL_new(cctx);
          SSL_set_fd(ssl, fd);
          if (SSL_connect(ssl) == 1) ssl_write_all(ssl, "GET /gone HTTP/1.1\r\n\r\n");
          SSL_free(ssl);
        }
        close(fd);
      }
    });
  }
  for (auto& x : clients) x.join();
  // the server still answers over TLS after all that
  {
    const int fd = connect_to(port);
    CHECK(fd >= 0);
    if (fd >= 0) {
      SSL* ssl = SSL_new(cctx);
      SSL_set_fd(ssl, fd);
      CHECK(SSL_connect(ssl) == 1);
      CHECK(ssl_write_all(ssl, "GET /final HTTP/1.1\r\n\r\n"));
      std::vector<std::string> b;
      CHECK(ssl_read_responses(ssl, 1, b));
      if (!b.empty()) CHECK(b[0] == "/final");
      SSL_free(ssl);
      close(fd);
    }
  }
  SSL_CTX_free(cctx);
  stop = true;
  oryx_http_stop(S);
  for (auto& x : handlers) x.join();
  oryx_http_free(S);
}

// ---------------------------------------------------------------- 6. host buffers, spans

// writers allocating / filling / freeing host buffers on several threads while the reaper
// unmaps them; the parallel file read of a file written here; the threaded categorical span
// encoding against a sequential first-appearance numbering
static void test_hostbuf(const char* dir) {
  std::vector<std::thread> ts;
  for (int w = 0; w < 6; ++w)
    ts.emplace_back([w] {
      for (int k = 0; k < 40; ++k) {
        const long long n = (1ll << 20) * (1 + (w + k) % 5) + 4096 * k;
        char* p = static_cast<char*>(oryx_hostbuf_alloc(n));
        CHECK(p != nullptr);
        if (!p) return;
        CHECK(p[n - 1] == 0);
        memset(p, 'a' + w, (size_t)n);
        CHECK(p[n / 2] == 'a' + w);
        oryx_hostbuf_free(p, n);
      }
    });
  for (auto& t : ts) t.join();
  CHECK(oryx_hostbuf_quiesce(10000) == 0);
  long long st[2];
  oryx_hostbuf_stats(st);
  CHECK(st[0] == 0 && st[1] > 0);

  const std::string path = std::string(dir) + "/hostbuf_read.txt";
  std::string data;
  for (int j = 0; j < 3000000; ++j) data += (char)('0' + j % 10), data += (j % 7 ? ',' : '\n');
  FILE* f = fopen(path.c_str(), "wb");
  CHECK(f != nullptr);
  if (f) {
    fwrite(data.data(), 1, data.size(), f);
    fclose(f);
    std::vector<char> got(data.size());
    CHECK(oryx_read_file_parallel(path.c_str(), got.data(), (long long)got.size(), 8) ==
          (long long)data.size());
    CHECK(memcmp(got.data(), data.data(), data.size()) == 0);
  }

  const long long n = 400000;
  std::string text;
  std::vector<long long> off(n);
  std::vector<int> len(n);
  unsigned long long z = 12345;
  for (long long j = 0; j < n; ++j) {
    z = z * 6364136223846793005ull + 1442695040888963407ull;
    const int v = (int)((z >> 33) % 3000);
    const std::string key = (z >> 20) % 19 == 0 ? std::string() : "v" + std::to_string(v * v % 997);
    off[j] = (long long)text.size();
    len[j] = (int)key.size();
    text += key;
    text += ',';
  }
  std::vector<long long> codes(n), first(n);
  const long long k = oryx_encode_spans(text.data(), off.data(), len.data(), n, 1, codes.data(),
                                        first.data());
  std::vector<std::string> seen;
  bool ok = true;
  for (long long j = 0; j < n && ok; ++j) {
    if (len[j] == 0) {
      ok = codes[j] == -1;
      continue;
    }
    const std::string key = text.substr((size_t)off[j], (size_t)len[j]);
    long long c = -1;
    for (size_t q = 0; q < seen.size(); ++q)
      if (seen[q] == key) c = (long long)q;
    if (c < 0) {
      c = (long long)seen.size();
      seen.push_back(key);
      ok = first[c] == j;
    }
    ok = ok && codes[j] == c;
  }
  CHECK(ok && k == (long long)seen.size());
}

// The keystore readers (oryx_keystore.cpp) from several threads at once on the same files, and
// on every truncation and a byte-flipped copy of each file: valid stores decode, damaged ones
// fail cleanly (no crash, no leak, no read past the buffer).
static void test_keystores(const char* dir, const char* const* stores, int n_stores) {
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int rep = 0; rep < 20; ++rep)
        for (int j = 0; j < n_stores; ++j) {
          char *c = nullptr, *k = nullptr;
          long long cn = 0, kn = 0;
          const int rc = oryx_keystore_to_pem(stores[j], "oryxpass", nullptr, &c, &cn, &k, &kn);
          if (rc != 0 || !c || !k || cn <= 0 || kn <= 0 ||
              strncmp(c, "-----BEGIN CERTIFICATE-----", 27) != 0) {
            fprintf(stderr, "keystore %s thread %d: rc %d (%s)\n", stores[j], t, rc,
                    oryx_keystore_error());
            g_errors++;
          }
          oryx_keystore_free(c);
          oryx_keystore_free(k);
          const int bad = oryx_keystore_to_pem(stores[j], "wrong", nullptr, &c, &cn, &k, &kn);
          if (bad != 2) {
            fprintf(stderr, "keystore %s: wrong password gave %d\n", stores[j], bad);
            g_errors++;
            if (bad == 0) {
              oryx_keystore_free(c);
              oryx_keystore_free(k);
            }
          }
        }
    });
  for (auto& x : th) x.join();
  // damaged copies: every prefix length (up to 4 KB) and one flipped byte per position step
  const std::string tmp = std::string(dir) + "/damaged_store";
  for (int j = 0; j < n_stores; ++j) {
    FILE* f = fopen(stores[j], "rb");
    if (!f) { g_errors++; continue; }
    std::vector<char> b;
    char buf[4096];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) b.insert(b.end(), buf, buf + got);
    fclose(f);
    for (size_t len = 0; len < b.size() && len < 4096; len += (len < 64 ? 1 : 37)) {
      for (int flip = 0; flip < 2; ++flip) {
        std::vector<char> d(b.begin(), b.begin() + (long)(flip ? b.size() : len));
        if (flip && len < d.size()) d[len] ^= 0x5a;
        FILE* o = fopen(tmp.c_str(), "wb");
        if (!o) { g_errors++; return; }
        if (!d.empty()) fwrite(d.data(), 1, d.size(), o);
        fclose(o);
        char *c = nullptr, *k = nullptr;
        long long cn = 0, kn = 0;
        const int rc = oryx_keystore_to_pem(tmp.c_str(), "oryxpass", nullptr, &c, &cn, &k, &kn);
        if (rc == 0) {
          oryx_keystore_free(c);
          oryx_keystore_free(k);
        }
      }
    }
  }
}

// ---------------------------------------------------------------- 7. speed micro-batch
// oryx_speed_parse (threaded parse + prefetched row-map probes) and oryx_speed_aggregate (hash
// grouping, time order per pair) against a std::map model of the same semantics: per (user,
// item) in (timestamp, arrival) order, implicit = sum after the last delete (a trailing delete
// drops the pair), explicit = the last value (a delete drops it).  Batches mix repeated pairs,
// out-of-order timestamps, deletes, quoted lines and keys the stores lack.

static void add_keys(void* m, const char* pre, int n, int stride) {
  std::string blob;
  std::vector<long long> ends, rows;
  for (int j = 0; j < n; ++j) {
    blob += pre + std::to_string(j);
    ends.push_back((long long)blob.size());
    rows.push_back((long long)j * stride + 1);
  }
  oryx_rowmap_set(m, blob.data(), ends.data(), rows.data(), n);
}

static void test_speed_batch() {
  void* xm = oryx_rowmap_new();
  void* ym = oryx_rowmap_new();
  add_keys(xm, "U", 3000, 3);
  add_keys(ym, "I", 800, 2);
  void* sb = oryx_speed_new();
  std::mt19937_64 g(7);
  for (int round = 0; round < 6; ++round) {
    const int n = round < 3 ? 25000 : 400 + 3000 * round;
    const int nu = round % 2 ? 60 : 3300, ni = round % 2 ? 20 : 900;   // dense: many repeats
    std::string buf;
    struct Ev { std::string u, i; double v; long long t; };
    std::vector<Ev> evs;
    for (int j = 0; j < n; ++j) {
      Ev e;
      e.u = "U" + std::to_string(g() % nu);
      e.i = "I" + std::to_string(g() % ni);
      const bool del = g() % 29 == 0;
      e.v = del ? std::nan("") : (double)(g() % 400) / 8.0;
      e.t = 1000 + (long long)(g() % 50);
      char vb[32];
      if (del) vb[0] = 0; else snprintf(vb, sizeof(vb), "%.3f", e.v);
      if (g() % 11 == 0)
        buf += "\"" + e.u + "\",\"" + e.i + "\"," + vb + "," + std::to_string(e.t) + "\n";
      else
        buf += e.u + "," + e.i + "," + vb + "," + std::to_string(e.t) + "\n";
      evs.push_back(e);
    }
    const long long got_n = oryx_speed_parse(sb, buf.data(), (long long)buf.size(), xm, ym, 0);
    CHECK(got_n == n);
    for (int implicit = 0; implicit < 2; ++implicit) {
      // model: stable sort by time, then fold per pair
      std::vector<int> ord(evs.size());
      for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
      std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return evs[a].t < evs[b].t; });
      std::map<std::pair<std::string, std::string>, double> want;
      for (int k : ord) {
        const auto key = std::make_pair(evs[k].u, evs[k].i);
        const double v = evs[k].v;
        if (!implicit) { want[key] = v; continue; }
        auto it = want.find(key);
        if (std::isnan(v)) want[key] = std::nan("");
        else if (it == want.end() || std::isnan(it->second)) want[key] = v;
        else it->second += v;
      }
      for (auto it = want.begin(); it != want.end();)
        it = std::isnan(it->second) ? want.erase(it) : std::next(it);
      std::vector<long long> u(evs.size()), i(evs.size());
      std::vector<double> v(evs.size());
      const long long m = oryx_speed_aggregate(sb, implicit, u.data(), i.data(), v.data());
      long long c[4];
      oryx_speed_counts(sb, c);
      CHECK(c[3] == m);
      // stores hold U0..U2999 (row 3j + 1) and I0..I799 (row 2j + 1): compare the pairs the
      // stores hold by row, and the count of the rest
      size_t known = 0;
      std::map<std::pair<long long, long long>, double> got;
      for (long long k = 0; k < m; ++k)
        if (u[k] >= 0 && i[k] >= 0) got[{u[k], i[k]}] = v[k];
      for (const auto& kv : want) {
        const long long uj = std::stoll(kv.first.first.substr(1)),
                        ij = std::stoll(kv.first.second.substr(1));
        if (uj >= 3000 || ij >= 800) continue;
        ++known;
        auto it = got.find({3 * uj + 1, 2 * ij + 1});
        CHECK(it != got.end() && std::fabs(it->second - kv.second) <= 1e-9 * (1 + std::fabs(kv.second)));
      }
      CHECK(got.size() == known);
      CHECK((size_t)m == want.size());
    }
  }
  oryx_speed_free(sb);
  oryx_rowmap_free(xm);
  oryx_rowmap_free(ym);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: runtime_stress2 <dir>\n");
    return 2;
  }
  test_append_fill(argv[1]);
  printf("append_fill + frame / text readers: errors %d\n", g_errors.load());
  test_http();
  printf("http: errors %d\n", g_errors.load());
  test_topn_prep();
  printf("topn_prep: errors %d\n", g_errors.load());
  test_pool();
  printf("thread pool: errors %d\n", g_errors.load());
  test_hostbuf(argv[1]);
  printf("host buffers / parallel read / span encoding: errors %d\n", g_errors.load());
  test_speed_batch();
  printf("speed micro-batch parse / aggregate: errors %d\n", g_errors.load());
  if (argc >= 4) {
    test_https(argv[2], argv[3]);
    printf("https: errors %d\n", g_errors.load());
  }
  if (argc >= 5) {
    test_keystores(argv[1], (const char* const*)(argv + 4), argc - 4);
    printf("keystores (JKS / PKCS#12, damaged copies): errors %d\n", g_errors.load());
  }
  return g_errors.load() == 0 ? 0 : 1;
}
