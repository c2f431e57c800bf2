// runtime_stress.cpp -- concurrency stress of the native runtime for sanitizer builds
// (the reference relies on coding discipline; here the host C++ runtime
// is exercised under -fsanitize=address,undefined and -fsanitize=thread).
//
// Producers append keyed records to a 4-partition topic from several threads (two Topic
// handles, as two processes would hold), readers tail every partition concurrently, consumer
// offsets are committed while reading, and the ingest dictionary/parser runs alongside.
// Exit status 0 = every record was read back exactly once per reader in per-partition order.

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* oryx_log_open(const char*, const char*, int, long long, long long);
void oryx_log_close(void*);
long long oryx_log_append_batch(void*, int, const char*, long long, int, long long, int,
                                long long*);
long long oryx_log_append_values_gap(void*, int, const char*, int, const char*,
                                     const long long*, int, int, long long, int);
void* oryx_reader_open(void*, int, long long);
void oryx_reader_close(void*);
long long oryx_reader_poll(void*, char*, long long, int, int, long long*);
int oryx_offsets_set(const char*, const char*, const char*, int, const int*, const long long*);
long long oryx_offsets_get(const char*, const char*, const char*, int);
const char* oryx_log_last_error();
void* oryx_dict_new();
void oryx_dict_free(void*);
long long oryx_parse_ratings(const char*, long long, void*, void*, long long*, long long*,
                             double*, long long*, long long, long long, int);
}

static void pack(std::string& buf, const std::string& key, const std::string& val) {
  int kl = (int)key.size();
  long long vl = (long long)val.size();
  buf.append(reinterpret_cast<const char*>(&kl), 4);
  buf.append(reinterpret_cast<const char*>(&vl), 8);
  buf += key;
  buf += val;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: runtime_stress <dir>\n");
    return 2;
  }
  const char* root = argv[1];
  const int P = 4, producers = 4, batches = 60, per_batch = 25;
  const long long total = (long long)producers * batches * per_batch;
  void* t1 = oryx_log_open(root, "Stress", P, 1 << 20, 1 << 16);   // small segments: rolls
  void* t2 = oryx_log_open(root, "Stress", P, 1 << 20, 1 << 16);
  if (!t1 || !t2) {
    fprintf(stderr, "open failed: %s\n", oryx_log_last_error());
    return 1;
  }
  std::atomic<int> errors{0};
  std::atomic<long long> read_total{0};
  std::vector<std::thread> th;
  for (int p = 0; p < producers; ++p) {
    th.emplace_back([&, p] {
      void* t = (p & 1) ? t2 : t1;
      for (int b = 0; b < batches; ++b) {
        std::string buf;
        for (int i = 0; i < per_batch; ++i) {
          const std::string key = "k" + std::to_string(p) + "-" + std::to_string(i % 7);
          pack(buf, key, "p" + std::to_string(p) + ":" + std::to_string(b * per_batch + i));
        }
        if (oryx_log_append_batch(t, -1, buf.data(), (long long)buf.size(), per_batch, -1, 0,
                                  nullptr) < 0)
          ++errors;
      }
    });
  }
  for (int part = 0; part < P; ++part) {
    th.emplace_back([&, part] {
      void* r = oryx_reader_open(t1, part, 0);
      std::vector<char> out(1 << 16);
      long long used = 0, last = -1, idle = 0;
      while (idle < 40) {
        long long n = oryx_reader_poll(r, out.data(), (long long)out.size(), 64, 50, &used);
        if (n < 0) {
          ++errors;
          break;
        }
        if (n == 0) {
          ++idle;
          continue;
        }
        idle = 0;
        long long pos = 0;
        for (long long i = 0; i < n; ++i) {
          long long off;
          int kl, vl;
          memcpy(&off, out.data() + pos, 8);
          memcpy(&kl, out.data() + pos + 16, 4);
          memcpy(&vl, out.data() + pos + 20, 4);
          if (off != last + 1) ++errors;          // offsets dense and in order
          last = off;
          pos += 24 + (kl > 0 ? kl : 0) + vl;
        }
        read_total += n;
        const int pp = part;
        const long long o = last + 1;
        if (oryx_offsets_set(root, "Stress", ("g" + std::to_string(part)).c_str(), 1, &pp,
                             &o) != 0)
          ++errors;
      }
      oryx_reader_close(r);
    });
  }
  th.emplace_back([&] {
    std::string text;
    for (int i = 0; i < 2000; ++i)
      text += "u" + std::to_string(i % 97) + ",i" + std::to_string(i % 31) + "," +
              std::to_string(i % 5) + "," + std::to_string(1000 + i) + "\n";
    for (int rep = 0; rep < 20; ++rep) {
      void* users = oryx_dict_new();
      void* items = oryx_dict_new();
      std::vector<long long> u(2000), it(2000), ts(2000);
      std::vector<double> s(2000);
      long long n = oryx_parse_ratings(text.data(), (long long)text.size(), users, items,
                                       u.data(), it.data(), s.data(), ts.data(), 2000, 0, 1);
      if (n != 2000) ++errors;
      oryx_dict_free(users);
      oryx_dict_free(items);
    }
  });
  // large blocks (frames built on several threads inside each append) from two writers
  const int big_batches = 3, big_n = 5000;
  void* b1 = oryx_log_open(root, "Big", 1, 1 << 20, 64ll << 20);
  void* b2 = oryx_log_open(root, "Big", 1, 1 << 20, 64ll << 20);
  for (int w = 0; w < 2; ++w) {
    th.emplace_back([&, w] {
      std::string blob;
      std::vector<long long> lens;
      for (int i = 0; i < big_n; ++i) {
        std::string v = "w" + std::to_string(w) + ":" + std::to_string(i) + ":";
        v.append(600, (char)('a' + i % 26));
        lens.push_back((long long)v.size());
        blob += v;
        blob += '\n';
      }
      for (int b = 0; b < big_batches; ++b)
        if (oryx_log_append_values_gap(w ? b2 : b1, -1, "UP", 2, blob.data(), lens.data(), big_n,
                                       1, -1, 0) < 0)
          ++errors;
    });
  }
  for (auto& x : th) x.join();
  {
    void* r = oryx_reader_open(b1, 0, 0);
    std::vector<char> out(1 << 22);
    long long used = 0, last = -1, got = 0;
    for (int idle = 0; idle < 5;) {
      const long long n = oryx_reader_poll(r, out.data(), (long long)out.size(), 4096, 20, &used);
      if (n <= 0) {
        ++idle;
        continue;
      }
      long long pos = 0;
      for (long long i = 0; i < n; ++i) {
        long long off;
        int kl, vl;
        memcpy(&off, out.data() + pos, 8);
        memcpy(&kl, out.data() + pos + 16, 4);
        memcpy(&vl, out.data() + pos + 20, 4);
        if (off != last + 1 || kl != 2 || vl < 600) ++errors;
        last = off;
        pos += 24 + (kl > 0 ? kl : 0) + vl;
      }
      got += n;
    }
    if (got != 2LL * big_batches * big_n) ++errors;
    oryx_reader_close(r);
  }
  oryx_log_close(b1);
  oryx_log_close(b2);
  oryx_log_close(t1);
  oryx_log_close(t2);
  for (int part = 0; part < P; ++part)
    if (oryx_offsets_get(root, "Stress", ("g" + std::to_string(part)).c_str(), part) < 0)
      ++errors;
  printf("records written %lld, read %lld, errors %d\n", total, read_total.load(),
         errors.load());
  return (errors.load() == 0 && read_total.load() == total) ? 0 : 1;
}
