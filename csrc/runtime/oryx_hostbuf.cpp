// oryx_hostbuf.cpp -- large host byte buffers of the batch layer (a generation's drained
// text, its train / test selections and concatenations: tens of GB per generation at
// BASELINE config #4's shape, 12.5M x 256 k-means points as CSV), mapped directly and unmapped
// off the caller's thread.
//
// The reference leaves these to Spark's executors (partitioned RDDs of the interval's and the
// history's records, [lambda]/batch/BatchUpdateFunction.java:103-130, reclaimed by the JVM
// garbage collector in the background).  Here a buffer freed by Python would be unmapped by
// the thread that drops the last reference -- with the GIL held, while the layer waits: with
// 4 KB pages that is ~65 ms per GB (a k-means generation spent ~2 s of 7 in its two "release"
// phases, profiles/r5_bb_kmeans_phases_v5.json).  oryx_hostbuf_free hands the mapping to one
// reaper thread instead and returns at once; the pages go back to the kernel while the layer
// continues.
//
// Mappings ask for transparent huge pages (MADV_HUGEPAGE: first-touch faults and the unmap
// walk 512x fewer page-table entries where the kernel grants them).
#include <errno.h>
#include <pthread.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>
#include <atomic>

namespace {

struct Reaper {
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<std::pair<void*, size_t>> q;
  long long pending = 0;     // bytes queued or being unmapped
  long long freed = 0;       // bytes unmapped by the reaper, ever
  bool started = false;

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return !q.empty(); });
      auto job = q.front();
      q.pop_front();
      lk.unlock();
      // The pages go first, by MADV_DONTNEED in 64 MB pieces (it holds the process's mmap
      // lock for reading only), then the emptied range is unmapped: munmap holds the lock for
      // writing while it frees pages, and a 17 GB munmap stalled the layer's own page faults
      // (a model publish went from 0.02 to 1.09 s) and the HIP runtime's pinning of pageable
      // memory for host -> device copies (the parse's upload ran at half speed beside it).
      constexpr size_t kPiece = 64u << 20;
      char* base = static_cast<char*>(job.first);
      for (size_t off = 0; off < job.second; off += kPiece)
        madvise(base + off, job.second - off < kPiece ? job.second - off : kPiece,
                MADV_DONTNEED);
      munmap(base, job.second);
      lk.lock();
      pending -= (long long)job.second;
      freed += (long long)job.second;
      if (pending == 0) idle.notify_all();
    }
  }
};

// Never destroyed: the detached thread may still be waiting on it at exit.  A forked child
// gets a fresh one (no reaper thread exists there, and the parent's lock may have been held
// at the fork): the parent's queued mappings are left to the child's exit.
std::atomic<Reaper*> g_reaper{nullptr};

void reaper_after_fork_child() { g_reaper.store(new Reaper()); }

Reaper& reaper() {
  static const bool once = [] {
    g_reaper.store(new Reaper());
    pthread_atfork(nullptr, nullptr, reaper_after_fork_child);
    return true;
  }();
  (void)once;
  return *g_reaper.load();
}

}  // namespace

extern "C" {

// A zero-filled private anonymous mapping of n bytes (huge pages advised), or nullptr.
void* oryx_hostbuf_alloc(long long n) {
  if (n <= 0) return nullptr;
  void* p = mmap(nullptr, (size_t)n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
#ifdef MADV_HUGEPAGE
  madvise(p, (size_t)n, MADV_HUGEPAGE);
#endif
  return p;
}

// Queues the unmapping of a buffer from oryx_hostbuf_alloc (same p and n) on the reaper
// thread; returns at once.  When the thread cannot be started the unmap happens here.
void oryx_hostbuf_free(void* p, long long n) {
  if (!p || n <= 0) return;
  Reaper& r = reaper();
  {
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.started) {
      try {
        std::thread([&r] { r.run(); }).detach();
        r.started = true;
      } catch (...) {
      }
    }
    if (r.started) {
      r.q.emplace_back(p, (size_t)n);
      r.pending += n;
      r.cv.notify_one();
      return;
    }
  }
  munmap(p, (size_t)n);
}

// Bytes queued for unmapping and not yet returned (out[0]), bytes unmapped by the reaper so
// far (out[1]).
void oryx_hostbuf_stats(long long* out) {
  Reaper& r = reaper();
  std::lock_guard<std::mutex> lk(r.mu);
  out[0] = r.pending;
  out[1] = r.freed;
}

// Waits until every queued unmap is done (at most timeout_ms; < 0: no limit).  Returns the
// bytes still pending.
long long oryx_hostbuf_quiesce(long long timeout_ms) {
  Reaper& r = reaper();
  std::unique_lock<std::mutex> lk(r.mu);
  auto done = [&] { return r.pending == 0; };
  if (timeout_ms < 0) {
    r.idle.wait(lk, done);
    return r.pending;
  }
  // (a bounded wait by polling: condition_variable::wait_for goes through
  // pthread_cond_clockwait, which ThreadSanitizer does not see release the mutex)
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (!done() && std::chrono::steady_clock::now() < until) {
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
    lk.lock();
  }
  return r.pending;
}

// Faults in [p, p + n) from `threads` threads (MADV_POPULATE_WRITE per slice where the kernel
// has it, else one store per 4 KB page): a buffer that several writers fill at once would
// otherwise take every first-touch fault inside their copies.
void oryx_hostbuf_prefault(void* p, long long n, int threads) {
  if (!p || n <= 0) return;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  constexpr long long kAlign = 2ll << 20;
  long long per = (n + threads - 1) / threads;
  per = (per + kAlign - 1) / kAlign * kAlign;
  auto work = [p, n, per](int t) {
    const long long lo = (long long)t * per;
    if (lo >= n) return;
    const long long len = lo + per < n ? per : n - lo;
    char* b = static_cast<char*>(p) + lo;
#ifdef MADV_POPULATE_WRITE
    if (madvise(b, (size_t)len, MADV_POPULATE_WRITE) == 0) return;
#endif
    for (long long o = 0; o < len; o += 4096) reinterpret_cast<volatile char*>(b)[o] = 0;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) {
    try {
      pool.emplace_back(work, t);
    } catch (...) {
      work(t);
    }
  }
  work(0);
  for (auto& th : pool) th.join();
}

// Reads bytes [0, n) of the file at path into out with up to `threads` concurrent preads of
// 32 MB pieces (a past interval's part file, tens of GB at config #4's shape: one read() call
// into a fresh Python bytes object ran at ~4 GB/s, single-threaded copy plus page faults).
// Returns the bytes read (n unless the file is shorter), or -errno.
long long oryx_read_file_parallel(const char* path, char* out, long long n, int threads) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -(long long)errno;
  constexpr long long kPiece = 32ll << 20;
  const long long pieces = (n + kPiece - 1) / kPiece;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  if ((long long)threads > pieces) threads = (int)(pieces > 0 ? pieces : 1);
  std::atomic<long long> next{0}, short_at{n};
  std::atomic<int> err{0};
  auto work = [&] {
    for (;;) {
      const long long k = next.fetch_add(1);
      if (k >= pieces || err.load()) return;
      long long off = k * kPiece;
      const long long end = off + kPiece < n ? off + kPiece : n;
      while (off < end) {
        const ssize_t got = pread(fd, out + off, (size_t)(end - off), (off_t)off);
        if (got < 0) {
          if (errno == EINTR) continue;
          err.store(errno);
          return;
        }
        if (got == 0) {   // end of file before n: remember the earliest short piece
          long long cur = short_at.load();
          while (off < cur && !short_at.compare_exchange_weak(cur, off)) {
          }
          break;
        }
        off += got;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) {
    try {
      pool.emplace_back(work);
    } catch (...) {
      break;
    }
  }
  work();
  for (auto& t : pool) t.join();
  close(fd);
  if (err.load()) return -(long long)err.load();
  return short_at.load();
}

}  // extern "C"
