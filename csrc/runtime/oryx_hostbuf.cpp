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
#include <sys/mman.h>

#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <mutex>
#include <thread>
#include <utility>

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
      munmap(job.first, job.second);
      lk.lock();
      pending -= (long long)job.second;
      freed += (long long)job.second;
      if (pending == 0) idle.notify_all();
    }
  }
};

Reaper& reaper() {
  // never destroyed: the detached thread may still be waiting on it at exit
  static Reaper* r = new Reaper();
  return *r;
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
  if (timeout_ms < 0)
    r.idle.wait(lk, done);
  else
    r.idle.wait_for(lk, std::chrono::milliseconds(timeout_ms), done);
  return r.pending;
}

}  // extern "C"
