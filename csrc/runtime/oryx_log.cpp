// oryx_log.cpp -- framework-owned append-only log (the Kafka/ZooKeeper replacement).
//
// The reference moves every inter-layer message over Kafka 0.8 topics (input: keyed,
// 4 partitions; update: 1 partition, replayed from the beginning by speed/serving) and keeps
// consumer-group offsets in ZooKeeper ([lambda]/TopicProducerImpl.java:32-84,
// [kafka]/KafkaUtils.java:57-161, deploy/bin/oryx-run.sh:330-344).  Nothing like that exists
// on an MI355X node, so this is a small native log with the same semantics:
//
//   <root>/<topic>/meta                     partitions, max message bytes, segment bytes
//   <root>/<topic>/<p>/<base-offset>.log    segment files of framed records
//   <root>/<topic>/.offsets/<group>         committed "partition offset" lines
//
// Record frame (little endian):  u32 magic | u32 crc32c | u64 offset | i64 ts_ms |
//                                u32 key_len (0xFFFFFFFF = null) | u32 value_len | key | value
// Appends from any process are serialised with flock() on the partition directory's lock
// file and written with one pwrite() (a block past 2 GB: consecutive ones); readers never
// consume a torn frame (a frame is only consumed once its full length and CRC check out).  Readers tail segment
// files by position, so consumers in other processes need no shared memory.
//
// C ABI for ctypes; every call releases nothing (ctypes drops the GIL around the call).

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <tuple>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <fcntl.h>
#include <memory>
#include <mutex>
#include <string>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "fastfloat.h"

namespace {

// "ORY2": frames checksummed with CRC-32C.  The first format, "ORYL", used the IEEE CRC-32
// over the same bytes; its frames are still read (the checksum is picked by magic) and new
// records are appended after them in the current format, so a log directory written by an
// older build keeps every record and offset.
constexpr uint32_t kMagic = 0x3259524Fu;
constexpr uint32_t kMagicV1 = 0x4F52594Cu;
constexpr size_t kHeader = 4 + 4 + 8 + 8 + 4 + 4;
constexpr uint32_t kNullKey = 0xFFFFFFFFu;

// CRC-32C (Castagnoli, the checksum of Kafka's v2 record batches): the SSE4.2 crc32
// instruction does 8 bytes per instruction (~10 GB/s on one core, ~6x the IEEE table loop this
// replaced) -- every poll and bulk read checks every record, model loads read gigabytes of
// update messages and the speed layer appends ~15 MB of UP rows per micro-batch.  CPUs without
// SSE4.2 take a slicing-by-8 table of the same polynomial.
uint32_t crc_tab[8][256];
uint32_t ieee_tab[8][256];   // legacy "ORYL" frames
bool crc_hw = false;

void init_table(uint32_t tab[8][256], uint32_t poly) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? poly ^ (c >> 1) : c >> 1;
    tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t)
      tab[t][i] = (tab[t - 1][i] >> 8) ^ tab[0][tab[t - 1][i] & 0xFF];
}

void init_crc() {
  init_table(crc_tab, 0x82F63B78u);
  init_table(ieee_tab, 0xEDB88320u);
  __builtin_cpu_init();
  crc_hw = __builtin_cpu_supports("sse4.2");
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}

uint32_t crc_sliced(const uint32_t (*crc_tab)[256], const uint8_t* p, size_t n, uint32_t crc) {
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = crc_tab[7][lo & 0xFF] ^ crc_tab[6][(lo >> 8) & 0xFF] ^
          crc_tab[5][(lo >> 16) & 0xFF] ^ crc_tab[4][lo >> 24] ^
          crc_tab[3][hi & 0xFF] ^ crc_tab[2][(hi >> 8) & 0xFF] ^
          crc_tab[1][(hi >> 16) & 0xFF] ^ crc_tab[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = crc_tab[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return crc;
}

// tables and CPU check once, at library load (a call_once per record cost more than the
// checksum of a short record)
struct CrcInit {
  CrcInit() { init_crc(); }
} crc_init_at_load;

inline uint32_t crc32(const uint8_t* p, size_t n, uint32_t crc = 0) {
  return ~(crc_hw ? crc32c_hw(p, n, ~crc) : crc_sliced(crc_tab, p, n, ~crc));
}

inline bool known_magic(uint32_t m) { return m == kMagic || m == kMagicV1; }

// Checksum of a complete frame at `f` with `plen` payload bytes: the 16 offset|ts bytes at
// +8, then the payload, under the polynomial its magic names.
inline uint32_t frame_crc(uint32_t magic, const uint8_t* f, size_t plen) {
  if (magic == kMagicV1)
    return ~crc_sliced(ieee_tab, f + kHeader, plen, crc_sliced(ieee_tab, f + 8, 16, ~0u));
  return crc32(f + kHeader, plen, crc32(f + 8, 16));
}

thread_local std::string g_err;

// large appends keep a preallocated, pre-faulted tail ahead of them (ORYX_LOG_PREALLOC=0
// disables)
const bool g_prealloc = [] {
  const char* v = std::getenv("ORYX_LOG_PREALLOC");
  return !(v && std::string(v) == "0");
}();

// One background thread faults preallocated segment ranges into the page cache
// (MADV_POPULATE_WRITE on a shared mapping: page tables and cache pages, no data change --
// an append writing the same range meanwhile is unaffected).  Jobs name the file by path: a
// segment deleted in between is skipped.
struct SegMap;
struct PrefaultQueue {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::tuple<std::shared_ptr<SegMap>, int64_t, int64_t>> jobs;
  bool started = false;
};

PrefaultQueue& prefault_queue() {
  static PrefaultQueue* q = new PrefaultQueue();   // never destroyed: the worker is detached
  return *q;
}

void prefault_run(const std::shared_ptr<SegMap>& m, int64_t off, int64_t len);

void prefault_async(const std::shared_ptr<SegMap>& m, int64_t off, int64_t len) {
  PrefaultQueue& q = prefault_queue();
  std::lock_guard<std::mutex> g(q.mu);
  q.jobs.emplace_back(m, off, len);
  if (!q.started) {
    q.started = true;
    std::thread([&q] {
      for (;;) {
        std::tuple<std::shared_ptr<SegMap>, int64_t, int64_t> j;
        {
          std::unique_lock<std::mutex> l(q.mu);
          q.cv.wait(l, [&] { return !q.jobs.empty(); });
          j = q.jobs.front();
          q.jobs.pop_front();
        }
        prefault_run(std::get<0>(j), std::get<1>(j), std::get<2>(j));
      }
    }).detach();
  }
  q.cv.notify_one();
}

// appends of at least this many bytes go through a shared mapping of the segment
// (ORYX_LOG_MMAP_MIN bytes; 0 disables)
const long long g_mmap_min = [] {
  const char* v = std::getenv("ORYX_LOG_MMAP_MIN");
  return v ? std::atoll(v) : (4ll << 20);
}();

int fail(const std::string& msg) {
  g_err = msg + (errno ? std::string(": ") + strerror(errno) : std::string());
  return -1;
}

bool mkdirs(const std::string& path) {
  if (path.empty()) return true;
  struct stat st;
  if (stat(path.c_str(), &st) == 0) return S_ISDIR(st.st_mode);
  size_t slash = path.find_last_of('/');
  if (slash != std::string::npos && slash > 0 && !mkdirs(path.substr(0, slash))) return false;
  return mkdir(path.c_str(), 0755) == 0 || errno == EEXIST;
}

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

std::vector<int64_t> list_segments(const std::string& dir) {
  std::vector<int64_t> bases;
  DIR* d = opendir(dir.c_str());
  if (!d) return bases;
  while (struct dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n.size() > 4 && n.compare(n.size() - 4, 4, ".log") == 0) {
      char* end = nullptr;
      long long v = strtoll(n.c_str(), &end, 10);
      if (end && std::string(end) == ".log") bases.push_back(v);
    }
  }
  closedir(d);
  std::sort(bases.begin(), bases.end());
  return bases;
}

std::string seg_name(const std::string& dir, int64_t base) {
  char buf[32];
  snprintf(buf, sizeof(buf), "%020lld.log", (long long)base);
  return dir + "/" + buf;
}

// MurmurHash2 (the hash Kafka's default partitioner uses), positive modulo partitions.
uint32_t murmur2(const uint8_t* data, int len) {
  const uint32_t seed = 0x9747b28c, m = 0x5bd1e995;
  const int r = 24;
  uint32_t h = seed ^ (uint32_t)len;
  int len4 = len / 4;
  for (int i = 0; i < len4; ++i) {
    int i4 = i * 4;
    uint32_t k = (data[i4 + 0] & 0xff) + ((data[i4 + 1] & 0xff) << 8) +
                 ((data[i4 + 2] & 0xff) << 16) + ((uint32_t)(data[i4 + 3] & 0xff) << 24);
    k *= m; k ^= k >> r; k *= m; h *= m; h ^= k;
  }
  switch (len % 4) {
    case 3: h ^= (uint32_t)(data[(len & ~3) + 2] & 0xff) << 16; [[fallthrough]];
    case 2: h ^= (uint32_t)(data[(len & ~3) + 1] & 0xff) << 8; [[fallthrough]];
    case 1: h ^= (uint32_t)(data[len & ~3] & 0xff); h *= m;
  }
  h ^= h >> 13; h *= m; h ^= h >> 15;
  return h;
}

// A writer's shared mapping of one segment file, kept across appends (the page tables of a
// mapping built per append cost more than the copy), sized to the segment's roll size plus
// the largest block seen; a background prefault job holds a reference while it works on it.
struct SegMap {
  int fd = -1;
  uint8_t* base = nullptr;
  size_t len = 0;
  int64_t seg_base = -1;
  ~SegMap() {
    if (base) munmap(base, len);
    if (fd >= 0) close(fd);
  }
};

// Faults [off, off + len) of a writer mapping in (page cache pages and this process's page
// tables; MADV_POPULATE_WRITE changes no data, so an append writing the range meanwhile is
// unaffected).  The range lies inside the file (the appender grew it under the lock).
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23     // Linux 5.14+ (older headers lack the name)
#endif
void prefault_run(const std::shared_ptr<SegMap>& m, int64_t off, int64_t len) {
  if (len < 0) {
    // a retired writer mapping (its segment is full): cut the file's unused preallocated
    // tail at `off`, the end of its data; the mapping itself goes with the last reference
    if (m && m->fd >= 0) (void)!ftruncate(m->fd, off);
    return;
  }
  {
  const long long page = sysconf(_SC_PAGESIZE);
  const int64_t a = off - off % page;
  if (!m || !m->base || a + len > (int64_t)m->len) return;
  madvise(m->base + a, (size_t)(off + len - a), MADV_POPULATE_WRITE);
  }
}

struct Partition {
  std::string dir;
  int lock_fd = -1;
  std::shared_ptr<SegMap> wmap;           // this handle's writer mapping of the active segment
  // flock() excludes other processes (and other handles); threads sharing this handle also
  // share the lock's open file description, for which flock is a no-op, so appends through
  // one handle are serialised by this mutex as well
  std::shared_ptr<std::mutex> mu = std::make_shared<std::mutex>();
  // cached tail of the active segment (validated under the lock on every append)
  int64_t c_base = -1, c_pos = 0, c_next = 0;
  // where oryx_log_end_offset's last scan stopped (it resumes from there)
  std::shared_ptr<std::mutex> end_mu_p = std::make_shared<std::mutex>();
  std::mutex& end_mu = *end_mu_p;
  int64_t e_base = -1, e_pos = 0, e_next = 0;
};

struct Topic {
  std::string root, name, dir;
  int partitions = 1;
  int64_t max_message = 16777216;
  int64_t segment_bytes = 64ll << 20;
  std::vector<Partition> parts;
  std::mutex mu;
  uint32_t rr = 0;
};

bool read_meta(Topic* t) {
  FILE* f = fopen((t->dir + "/meta").c_str(), "r");
  if (!f) return false;
  int p = 0;
  long long mm = 0, sb = 0;
  int n = fscanf(f, "partitions=%d\nmax-message=%lld\nsegment-bytes=%lld", &p, &mm, &sb);
  fclose(f);
  if (n < 1 || p <= 0) return false;
  t->partitions = p;
  if (n >= 2 && mm > 0) t->max_message = mm;
  if (n >= 3 && sb > 0) t->segment_bytes = sb;
  return true;
}

bool write_meta(Topic* t) {
  std::string tmp = t->dir + "/.meta.tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return false;
  fprintf(f, "partitions=%d\nmax-message=%lld\nsegment-bytes=%lld\n", t->partitions,
          (long long)t->max_message, (long long)t->segment_bytes);
  fflush(f);
  fsync(fileno(f));
  fclose(f);
  // first creator wins: link() fails if meta already exists
  if (link(tmp.c_str(), (t->dir + "/meta").c_str()) != 0) {
    unlink(tmp.c_str());
    return read_meta(t);
  }
  unlink(tmp.c_str());
  return true;
}

// Scan a segment from byte position `pos`; returns the next offset and fills `end_pos` with
// the position after the last complete frame.
int64_t scan_segment(const std::string& path, int64_t base, int64_t* end_pos,
                     int64_t start_pos = 0, int64_t start_next = -1) {
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) { *end_pos = 0; return base; }
  int64_t pos = start_pos, next = start_next >= 0 ? start_next : base;
  // block reads growing from 64 KB to 4 MB (a resumed scan usually finds a few frames and
  // then the end of the data -- possibly a preallocated zero tail, not worth 4 MB per look);
  // a frame straddling a block is re-read from its start
  std::vector<uint8_t> buf(64u << 10);
  for (;;) {
    const size_t cap = buf.size();
    ssize_t got = pread(fd, buf.data(), cap, pos);
    if (got < (ssize_t)kHeader) break;
    size_t at = 0;
    bool bad = false, straddle = false;
    while (at + kHeader <= (size_t)got) {
      const uint8_t* h = buf.data() + at;
      uint32_t magic, crc, klen, vlen;
      uint64_t off;
      memcpy(&magic, h, 4); memcpy(&crc, h + 4, 4); memcpy(&off, h + 8, 8);
      memcpy(&klen, h + 24, 4); memcpy(&vlen, h + 28, 4);
      if (!known_magic(magic)) { bad = true; break; }
      size_t plen = (klen == kNullKey ? 0 : klen) + (size_t)vlen;
      if (at + kHeader + plen > (size_t)got) {
        if (kHeader + plen > buf.size()) buf.resize(kHeader + plen);
        straddle = true;
        break;
      }
      if (frame_crc(magic, h, plen) != crc) { bad = true; break; }
      at += kHeader + plen;
      next = (int64_t)off + 1;
    }
    pos += (int64_t)at;
    if (bad) break;
    // a frame that runs past a short read ends where the file ends: a torn tail (a writer
    // that died mid-append); only a full block (or one just grown for a large frame) is
    // re-read from the frame's start
    if (straddle) {
      if ((size_t)got < cap) break;
      continue;
    }
    if (at == 0 || (size_t)got < cap) break;
    if (buf.size() < (4u << 20)) buf.resize(std::min<size_t>(buf.size() * 4, 4u << 20));
  }
  close(fd);
  *end_pos = pos;
  return next;
}

// The bytes past the end of the data: a zero header means nothing was ever written there (a
// preallocated tail, kept for the next append to write into) -- unlike a torn block, whose
// unpublished first frame has a zero magic but a written header.
bool zero_header_at(int fd, int64_t pos) {
  uint8_t h[kHeader];
  const ssize_t got = pread(fd, h, kHeader, pos);
  if (got != (ssize_t)kHeader) return false;
  for (size_t i = 0; i < kHeader; ++i)
    if (h[i]) return false;
  return true;
}

// Whether bytes [end_pos, size) of a segment can be the torn tail of an interrupted append:
// shorter than a frame header, all zeros (a crashed write on a filesystem that had already
// extended the file), or a single frame of a known format that runs to (or past) the end of
// the file.  Anything else -- an unknown magic with data behind it, or a bad frame followed by
// more bytes -- is not a torn write.
bool torn_tail(const std::string& path, int64_t end_pos, int64_t size) {
  const int64_t rem = size - end_pos;
  if (rem < (int64_t)kHeader) return true;
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  std::vector<uint8_t> buf((size_t)std::min<int64_t>(rem, 1 << 20));
  const ssize_t got = pread(fd, buf.data(), buf.size(), end_pos);
  bool zeros = got == (ssize_t)buf.size();
  for (ssize_t i = 0; zeros && i < got; ++i) zeros = buf[(size_t)i] == 0;
  if (zeros && rem > (int64_t)buf.size()) {
    // scan the rest of a large zero tail in blocks
    for (int64_t at = end_pos + (int64_t)buf.size(); zeros && at < size;) {
      const ssize_t g = pread(fd, buf.data(), buf.size(), at);
      if (g <= 0) break;
      for (ssize_t i = 0; zeros && i < g; ++i) zeros = buf[(size_t)i] == 0;
      at += g;
    }
  }
  close(fd);
  if (zeros) return true;
  if (got < (ssize_t)kHeader) return false;
  uint32_t magic, klen, vlen;
  memcpy(&magic, buf.data(), 4); memcpy(&klen, buf.data() + 24, 4);
  memcpy(&vlen, buf.data() + 28, 4);
  // a mapped append that never published its first frame's magic (the writer died): the
  // whole block is unpublished, nothing of it was ever readable
  if (magic == 0) return true;
  if (!known_magic(magic)) return false;
  const int64_t flen = (int64_t)kHeader + (klen == kNullKey ? 0 : (int64_t)klen) + (int64_t)vlen;
  return flen >= rem;
}

struct Reader {
  Topic* topic;
  int part;
  int64_t seg_base = -1;
  int64_t pos = 0;
  int64_t next_offset = 0;
  int fd = -1;
  // read-ahead block of the current segment file: polls parse frames out of it instead of
  // two preads per record (invalidated whenever fd changes or a frame is incomplete/bad)
  std::vector<uint8_t> blk;
  int64_t blk_pos = -1;
  size_t blk_len = 0;
  // at the end of the data (the last look found no complete frame): read small blocks until
  // more arrives (a segment may have a preallocated zero tail: 1 MB per idle poll would be
  // wasted copying)
  bool at_tail = false;
};

// Pointer to bytes [pos, pos + n) of the reader's segment (through the read-ahead block), or
// nullptr when the file does not hold them (yet).
const uint8_t* reader_bytes(Reader* r, int64_t pos, size_t n) {
  if (r->blk_pos >= 0 && pos >= r->blk_pos &&
      (size_t)(pos - r->blk_pos) + n <= r->blk_len)
    return r->blk.data() + (pos - r->blk_pos);
  const size_t ahead = r->at_tail ? (4u << 10) : (1u << 20);
  const size_t want = n > ahead ? n : ahead;
  if (r->blk.size() < want) r->blk.resize(want);
  const ssize_t got = pread(r->fd, r->blk.data(), want, pos);
  r->blk_pos = pos;
  r->blk_len = got > 0 ? (size_t)got : 0;
  if (r->blk_len < n) {
    r->blk_pos = -1;
    return nullptr;
  }
  return r->blk.data();
}

// Position a reader at `offset` (clamped to [begin, end]).  Frames before it are skipped in
// 4 MB block reads (not two syscalls per frame: a consumer seeking to the end of a 3M-record
// partition paid ~0.15 s), starting from the partition's cached end-of-log scan position
// when that lies at or before the target (the common seek: to the end offset just read).
void reader_seek(Reader* r, int64_t offset) {
  Partition& P = r->topic->parts[r->part];
  const std::string& dir = P.dir;
  std::vector<int64_t> segs = list_segments(dir);
  if (r->fd >= 0) { close(r->fd); r->fd = -1; }
  r->blk_pos = -1;
  if (segs.empty()) { r->seg_base = 0; r->pos = 0; r->next_offset = 0; return; }
  if (offset < segs.front()) offset = segs.front();
  size_t idx = 0;
  for (size_t i = 0; i < segs.size(); ++i) if (segs[i] <= offset) idx = i;
  r->seg_base = segs[idx];
  r->pos = 0;
  r->next_offset = segs[idx];
  {
    std::lock_guard<std::mutex> g(P.end_mu);
    if (P.e_base == segs[idx] && P.e_next <= offset && P.e_next >= segs[idx]) {
      r->pos = P.e_pos;
      r->next_offset = P.e_next;
    }
  }
  r->fd = open(seg_name(dir, segs[idx]).c_str(), O_RDONLY);
  if (r->fd < 0 || r->next_offset >= offset) return;
  std::vector<uint8_t> buf(4u << 20);
  while (r->next_offset < offset) {
    const ssize_t got = pread(r->fd, buf.data(), buf.size(), r->pos);
    if (got < (ssize_t)kHeader) break;
    size_t at = 0;
    bool straddle = false, stop = false;
    while (at + kHeader <= (size_t)got && r->next_offset < offset) {
      const uint8_t* h = buf.data() + at;
      uint32_t magic, klen, vlen;
      uint64_t off;
      memcpy(&magic, h, 4); memcpy(&off, h + 8, 8); memcpy(&klen, h + 24, 4);
      memcpy(&vlen, h + 28, 4);
      if (!known_magic(magic)) { stop = true; break; }
      const size_t plen = (klen == kNullKey ? 0 : klen) + (size_t)vlen;
      if (at + kHeader + plen > (size_t)got) {
        if (kHeader + plen > buf.size()) buf.resize(kHeader + plen);
        straddle = true;
        break;
      }
      at += kHeader + plen;
      r->pos += (int64_t)(kHeader + plen);
      r->next_offset = (int64_t)off + 1;
    }
    if (stop) break;
    if (straddle) {
      if ((size_t)got < buf.size() && at == 0) break;   // a frame still being written
      continue;
    }
    if ((size_t)got < buf.size()) break;
  }
}

}  // namespace

extern "C" {

const char* oryx_log_last_error() { return g_err.c_str(); }

// Opens (creating when `create_partitions` > 0) a topic.  Returns a handle or nullptr.
void* oryx_log_open(const char* root, const char* topic, int create_partitions,
                    long long max_message, long long segment_bytes) {
  errno = 0;
  auto* t = new Topic();
  t->root = root;
  t->name = topic;
  t->dir = std::string(root) + "/" + topic;
  if (!read_meta(t)) {
    if (create_partitions <= 0) {
      g_err = "topic does not exist: " + t->name;
      delete t;
      return nullptr;
    }
    if (!mkdirs(t->dir)) { fail("mkdir " + t->dir); delete t; return nullptr; }
    t->partitions = create_partitions;
    if (max_message > 0) t->max_message = max_message;
    if (segment_bytes > 0) t->segment_bytes = segment_bytes;
    if (!write_meta(t)) { fail("write meta"); delete t; return nullptr; }
  }
  t->parts.resize(t->partitions);
  for (int p = 0; p < t->partitions; ++p) {
    t->parts[p].dir = t->dir + "/" + std::to_string(p);
    if (!mkdirs(t->parts[p].dir)) { fail("mkdir partition"); delete t; return nullptr; }
    t->parts[p].lock_fd = open((t->parts[p].dir + "/.lock").c_str(), O_RDWR | O_CREAT, 0644);
  }
  return t;
}

int oryx_log_exists(const char* root, const char* topic) {
  std::string meta = std::string(root) + "/" + topic + "/meta";
  struct stat st;
  return stat(meta.c_str(), &st) == 0 ? 1 : 0;
}

void oryx_log_close(void* h) {
  auto* t = static_cast<Topic*>(h);
  if (!t) return;
  for (auto& p : t->parts) if (p.lock_fd >= 0) close(p.lock_fd);
  delete t;
}

int oryx_log_num_partitions(void* h) { return static_cast<Topic*>(h)->partitions; }
long long oryx_log_max_message(void* h) { return static_cast<Topic*>(h)->max_message; }

int oryx_log_partition_for(void* h, const char* key, int key_len) {
  auto* t = static_cast<Topic*>(h);
  if (key_len < 0 || !key) {
    std::lock_guard<std::mutex> g(t->mu);
    return (int)(t->rr++ % (uint32_t)t->partitions);
  }
  return (int)((murmur2((const uint8_t*)key, key_len) & 0x7fffffffu) % (uint32_t)t->partitions);
}

namespace {

// One record to append: key (nullptr / klen < 0 = null key) and value, both pointing into the
// caller's memory.
struct RecRef {
  const char* key;
  int32_t klen;
  const char* val;
  int64_t vlen;
};

// Frame buffer reused across appends by the same thread (a fresh multi-MB vector per append
// paid for its zero-filled pages in kernel time: ~45 ms per 12 MB block of UP messages).
std::vector<uint8_t>& frame_buffer(size_t need) {
  thread_local std::vector<uint8_t> out;
  if (out.size() < need) out.resize(need);
  return out;
}

// The segment just filled (its data reached the roll size): the next append starts a new
// segment at offset `next`.  Create and size it now and fault its first pages in on the
// background thread, so that append (a speed layer's next micro-batch) finds its pages ready
// instead of paying a fresh mapping's page faults; the full segment's mapping retires on
// the background thread, which also cuts its unused zero tail.  Readers treat the new,
// all-zero segment as the end of the data (a zero magic), as they do a preallocated tail.
// Called under the partition's locks.
void pre_roll(Topic* t, Partition& P, int64_t next, size_t total) {
  const std::string path = seg_name(P.dir, next);
  const int fd = open(path.c_str(), O_RDWR | O_CREAT, 0644);
  if (fd < 0) return;
  struct stat st;
  const int64_t want = std::min<int64_t>(std::max<int64_t>(2 * (int64_t)total, 16ll << 20),
                                         t->segment_bytes);
  if (fstat(fd, &st) != 0 || st.st_size != 0 || ftruncate(fd, want) != 0) {
    close(fd);
    return;
  }
  auto m = std::make_shared<SegMap>();
  m->fd = fd;
  m->seg_base = next;
  m->len = (size_t)t->segment_bytes + 4 * total;
  void* a = mmap(nullptr, m->len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (a == MAP_FAILED) return;           // (m closes fd)
  m->base = static_cast<uint8_t*>(a);
  std::shared_ptr<SegMap> old = std::move(P.wmap);
  P.wmap = m;
  if (old) prefault_async(old, P.c_pos, -1);
  prefault_async(m, 0, want);
  P.c_base = next;
  P.c_pos = 0;
  P.c_next = next;
}

// Appends `recs` (already validated) to partition `part` under its locks; records get
// consecutive offsets.  Frames are built straight from the records' memory, their CRCs over
// several threads for large batches.  Returns the last offset written, or -1.
// A producer that writes record j's value bytes straight into its frame (`vlen` bytes at
// dst) instead of the log copying them from the caller's memory.
typedef void (*FillFn)(void* ctx, long long j, char* dst);

long long append_partition(Topic* t, int part, const std::vector<RecRef>& recs,
                           const std::vector<int>& which, long long ts_ms, int do_fsync,
                           long long* out_offsets, FillFn fill = nullptr,
                           void* fill_ctx = nullptr) {
  const auto Ts = std::chrono::steady_clock::now();
  Partition& P = t->parts[part];
  std::lock_guard<std::mutex> in_process(*P.mu);
  if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_EX);
  std::vector<int64_t> segs = list_segments(P.dir);
  int64_t base = segs.empty() ? 0 : segs.back();
  int64_t end_pos = 0;
  int64_t next = 0;
  if (!segs.empty()) {
    if (P.c_base == base)
      next = scan_segment(seg_name(P.dir, base), base, &end_pos, P.c_pos, P.c_next);
    else
      next = scan_segment(seg_name(P.dir, base), base, &end_pos);
  }
  std::string path = seg_name(P.dir, base);
  if (!segs.empty() && end_pos >= t->segment_bytes) {
    base = next;
    path = seg_name(P.dir, base);
    end_pos = 0;
  }
  int fd = open(path.c_str(), O_RDWR | O_CREAT, 0644);
  if (fd < 0) {
    if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_UN);
    return fail("open segment");
  }
  // truncate a torn tail left by a crashed writer -- but only a tail that can be one: bytes
  // past the last good frame that are not themselves followed by more data (a frame with an
  // unknown magic or a bad checksum in the middle of a segment is corruption, and truncating
  // there would silently drop every later record and re-issue committed offsets)
  struct stat st;
  int64_t file_size = fstat(fd, &st) == 0 ? (int64_t)st.st_size : end_pos;
  if (file_size > end_pos && !zero_header_at(fd, end_pos)) {
    if (!torn_tail(path, end_pos, file_size)) {
      close(fd);
      if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_UN);
      errno = 0;
      return fail("refusing to append: segment " + path + " holds unreadable data at byte " +
                  std::to_string(end_pos) + " followed by more data (corrupt or unknown format)");
    }
    if (ftruncate(fd, end_pos) == 0) file_size = end_pos;
  }
  const size_t n = which.size();
  std::vector<size_t> at(n + 1);
  at[0] = 0;
  for (size_t j = 0; j < n; ++j) {
    const RecRef& r = recs[(size_t)which[j]];
    at[j + 1] = at[j] + kHeader + (r.klen < 0 ? 0 : (size_t)r.klen) + (size_t)r.vlen;
  }
  const size_t total = at[n];
  const int64_t first = next;
  // Large appends are built straight into the segment's page cache through a shared mapping
  // (one copy of the bytes instead of a frame buffer plus pwrite's kernel copy, and the
  // frames are written by all native threads).  The first frame's magic is stored last: until
  // then readers see an unknown magic at the old end of the log and stop there, so no reader
  // ever sees a later frame of the block before an earlier one is complete.
  const auto Tm = std::chrono::steady_clock::now();
  uint8_t* mapped = nullptr;
  if (g_mmap_min > 0 && (long long)total >= g_mmap_min &&
      (file_size >= end_pos + (int64_t)total ||
       ftruncate(fd, end_pos + (off_t)total) == 0)) {
    // (the file only ever grows here: a preallocated tail may already be longer)
    file_size = std::max<int64_t>(file_size, end_pos + (int64_t)total);
    std::shared_ptr<SegMap>& wm = P.wmap;
    const size_t need = (size_t)(end_pos + (int64_t)total);
    if (!wm || wm->seg_base != base || wm->len < need) {
      // (re)map the whole segment: its roll size, or more for a block that overshoots it
      auto m = std::make_shared<SegMap>();
      m->fd = open(path.c_str(), O_RDWR);
      m->seg_base = base;
      // (room for the block that overshoots the roll size too)
      m->len = std::max<size_t>((size_t)t->segment_bytes + 2 * total, 2 * need);
      if (m->fd >= 0) {
        void* a = mmap(nullptr, m->len, PROT_READ | PROT_WRITE, MAP_SHARED, m->fd, 0);
        if (a != MAP_FAILED) m->base = static_cast<uint8_t*>(a);
      }
      wm = m->base ? m : nullptr;
    }
    if (wm) mapped = wm->base;
  }
  const auto T0 = std::chrono::steady_clock::now();
  std::vector<uint8_t>* fb = mapped ? nullptr : &frame_buffer(total);
  uint8_t* dst = mapped ? mapped + end_pos : fb->data();
  auto build = [&](long long lo, long long hi, int) {
    for (long long j = lo; j < hi; ++j) {
      const RecRef& r = recs[(size_t)which[(size_t)j]];
      uint8_t* f = dst + at[(size_t)j];
      const uint32_t uk = r.klen < 0 ? kNullKey : (uint32_t)r.klen;
      const uint32_t uv = (uint32_t)r.vlen;
      const size_t kl = r.klen < 0 ? 0 : (size_t)r.klen;
      const uint64_t off = (uint64_t)(first + j);
      const int64_t ts = ts_ms;
      const uint32_t magic = j == 0 ? 0u : kMagic;     // published last, see below
      memcpy(f, &magic, 4);
      memcpy(f + 8, &off, 8);
      memcpy(f + 16, &ts, 8);
      memcpy(f + 24, &uk, 4);
      memcpy(f + 28, &uv, 4);
      if (kl) memcpy(f + kHeader, r.key, kl);
      if (fill)
        fill(fill_ctx, (long long)which[(size_t)j], reinterpret_cast<char*>(f + kHeader + kl));
      else
        memcpy(f + kHeader + kl, r.val, (size_t)r.vlen);
      const uint32_t crc = crc32(f + kHeader, kl + (size_t)r.vlen, crc32(f + 8, 16));
      memcpy(f + 4, &crc, 4);
    }
  };
  // threads only for batches worth it (~1 MB per thread)
  const long long per = total >= (2u << 20) ? std::max<long long>(64, (long long)(n * (1u << 20) / total)) : (long long)n + 1;
  oryx_ff::parallel_ranges((long long)n, per, build);
  const auto T1 = std::chrono::steady_clock::now();
  if (out_offsets)
    for (size_t j = 0; j < n; ++j) out_offsets[which[j]] = first + (long long)j;
  next = first + (int64_t)n;
  // Every append publishes its block by storing the first frame's magic after every other
  // byte of the block is in place: a reader stops at the zero magic (the end of the data)
  // until then, so it never meets a half-written frame followed by complete ones (which it
  // would report as corruption) -- also when the block lands in a preallocated zero tail.
  size_t done = 0;
  if (mapped) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __atomic_store_n(reinterpret_cast<uint32_t*>(dst), kMagic, __ATOMIC_RELEASE);
    if (do_fsync) {
      const long long page = sysconf(_SC_PAGESIZE);
      const int64_t a = end_pos - end_pos % page;
      msync(mapped + a, (size_t)(end_pos + (int64_t)total - a), MS_SYNC);
    }
    done = total;
  }
  // otherwise one pwrite per append (Linux caps a single write at 0x7ffff000 bytes, so a
  // block past 2 GB goes out in pieces), then the 4-byte magic
  while (done < total) {
    const ssize_t w = pwrite(fd, fb->data() + done, total - done, end_pos + (off_t)done);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) break;
    done += (size_t)w;
  }
  if (!mapped && done == total) {
    ssize_t w;
    do { w = pwrite(fd, &kMagic, 4, end_pos); } while (w < 0 && errno == EINTR);
    if (w != 4) done = 0;
  }
  const auto T2 = std::chrono::steady_clock::now();
  if (std::getenv("ORYX_LOG_DEBUG"))
    fprintf(stderr, "append %zu B mapped=%d open %.3f map %.3f build %.3f ms write %.3f ms\n",
            total, mapped != nullptr, std::chrono::duration<double, std::milli>(Tm - Ts).count(),
            std::chrono::duration<double, std::milli>(T0 - Tm).count(),
            std::chrono::duration<double, std::milli>(T1 - T0).count(),
            std::chrono::duration<double, std::milli>(T2 - T1).count());
  if (done == total && mapped && g_prealloc) {
    // keep the next large block's pages in the page cache ahead of it: grow the segment
    // (under the lock; never past its roll size) and fault the new range in on a
    // background thread -- the append itself then only copies bytes
    const int64_t new_end = end_pos + (int64_t)total;
    // (up to a block past the roll size: the block that crosses it lands there too, and the
    // unused rest is cut when the segment retires, see pre_roll)
    int64_t want = std::min<int64_t>(new_end + std::max<int64_t>(2 * (int64_t)total,
                                                                 16ll << 20),
                                     std::max<int64_t>(t->segment_bytes + (int64_t)total,
                                                       new_end));
    want = std::min<int64_t>(want, (int64_t)P.wmap->len);
    if (want > file_size && ftruncate(fd, want) == 0) file_size = want;
    if (file_size > new_end) prefault_async(P.wmap, new_end, file_size - new_end);
  }
  if (done != total) {
    close(fd);
    if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_UN);
    return fail("write");
  }
  if (do_fsync) fsync(fd);
  close(fd);
  P.c_base = base;
  P.c_pos = end_pos + (int64_t)total;
  P.c_next = next;
  if (mapped && g_prealloc && P.c_pos >= t->segment_bytes) pre_roll(t, P, next, total);
  if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_UN);
  if (std::getenv("ORYX_LOG_DEBUG"))
    fprintf(stderr, "append tail %.3f ms\n", std::chrono::duration<double, std::milli>(
        std::chrono::steady_clock::now() - T2).count());
  return next - 1;
}

// Validates the records, routes them to partitions (-1: by key / round robin) and appends.
long long append_records(Topic* t, void* h, int partition, const std::vector<RecRef>& recs,
                         long long ts_ms, int do_fsync, long long* out_offsets,
                         FillFn fill = nullptr, void* fill_ctx = nullptr) {
  errno = 0;
  if (ts_ms < 0) ts_ms = now_ms();
  const size_t n = recs.size();
  std::vector<std::vector<int>> idx(t->partitions);
  for (size_t i = 0; i < n; ++i) {
    const RecRef& r = recs[i];
    if (r.vlen + (r.klen < 0 ? 0 : r.klen) > t->max_message) {
      g_err = "message of " + std::to_string(r.vlen) + " bytes exceeds max message size " +
              std::to_string(t->max_message);
      return -2;
    }
    const int part = partition >= 0 ? partition : oryx_log_partition_for(h, r.key, r.klen);
    if (part >= t->partitions) { g_err = "bad partition"; return -1; }
    idx[part].push_back((int)i);
  }
  long long last = -1;
  for (int part = 0; part < t->partitions; ++part) {
    if (idx[part].empty()) continue;
    const long long l = append_partition(t, part, recs, idx[part], ts_ms, do_fsync, out_offsets,
                                         fill, fill_ctx);
    if (l < 0) return -1;
    last = l;
  }
  return last;
}

}  // namespace

// Appends `n` records packed as [i32 key_len(-1=null)][i64 value_len][key][value]... to one
// partition (-1: per record by key / round robin).  Returns the last offset written, or -1.
// Each record's offset is written to out_offsets when non-null.
long long oryx_log_append_batch(void* h, int partition, const char* buf, long long buf_len,
                                int n, long long ts_ms, int do_fsync, long long* out_offsets) {
  auto* t = static_cast<Topic*>(h);
  std::vector<RecRef> recs((size_t)n);
  const char* p = buf;
  const char* end = buf + buf_len;
  for (int i = 0; i < n; ++i) {
    if (p + 12 > end) { g_err = "truncated batch"; return -1; }
    int32_t klen; int64_t vlen;
    memcpy(&klen, p, 4); memcpy(&vlen, p + 4, 8);
    const int64_t rec_bytes = 12 + (klen < 0 ? 0 : klen) + vlen;
    if (vlen < 0 || p + rec_bytes > end) { g_err = "truncated batch"; return -1; }
    recs[(size_t)i] = RecRef{klen < 0 ? nullptr : p + 12, klen, p + 12 + (klen < 0 ? 0 : klen), vlen};
    p += rec_bytes;
  }
  return append_records(t, h, partition, recs, ts_ms, do_fsync, out_offsets);
}

long long oryx_log_begin_offset(void* h, int partition) {
  auto* t = static_cast<Topic*>(h);
  std::vector<int64_t> segs = list_segments(t->parts[partition].dir);
  return segs.empty() ? 0 : segs.front();
}

long long oryx_log_end_offset(void* h, int partition) {
  auto* t = static_cast<Topic*>(h);
  auto& P = t->parts[partition];
  const std::string& dir = P.dir;
  std::vector<int64_t> segs = list_segments(dir);
  if (segs.empty()) return 0;
  int64_t end_pos;
  int64_t next;
  // resume the scan where the previous call ended (valid frames only ever get appended)
  std::lock_guard<std::mutex> g(P.end_mu);
  if (P.e_base == segs.back())
    next = scan_segment(seg_name(dir, segs.back()), segs.back(), &end_pos, P.e_pos, P.e_next);
  else
    next = scan_segment(seg_name(dir, segs.back()), segs.back(), &end_pos);
  P.e_base = segs.back();
  P.e_pos = end_pos;
  P.e_next = next;
  return next;
}

// Deletes whole segments whose files were last modified before `older_than_ms` (keeping the
// active segment).  Returns the number of segments deleted.
int oryx_log_retain(void* h, long long older_than_ms) {
  auto* t = static_cast<Topic*>(h);
  int deleted = 0;
  for (auto& P : t->parts) {
    if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_EX);
    std::vector<int64_t> segs = list_segments(P.dir);
    for (size_t i = 0; i + 1 < segs.size(); ++i) {
      std::string path = seg_name(P.dir, segs[i]);
      struct stat st;
      if (stat(path.c_str(), &st) == 0 &&
          (int64_t)st.st_mtime * 1000 < older_than_ms) {
        if (unlink(path.c_str()) == 0) ++deleted;
      } else {
        break;
      }
    }
    if (P.lock_fd >= 0) flock(P.lock_fd, LOCK_UN);
  }
  return deleted;
}

void* oryx_reader_open(void* h, int partition, long long offset) {
  auto* t = static_cast<Topic*>(h);
  if (partition < 0 || partition >= t->partitions) { g_err = "bad partition"; return nullptr; }
  auto* r = new Reader();
  r->topic = t;
  r->part = partition;
  reader_seek(r, offset < 0 ? oryx_log_end_offset(h, partition) : offset);
  return r;
}

void oryx_reader_close(void* rh) {
  auto* r = static_cast<Reader*>(rh);
  if (!r) return;
  if (r->fd >= 0) close(r->fd);
  delete r;
}

long long oryx_reader_position(void* rh) { return static_cast<Reader*>(rh)->next_offset; }

void oryx_reader_seek(void* rh, long long offset) { reader_seek(static_cast<Reader*>(rh), offset); }

// Reads up to `max_records` complete records into `out` as
// [i64 offset][i64 ts][i32 key_len(-1 null)][i32 value_len][key][value]...
// Waits up to timeout_ms for the first record.  Returns the number of records read, -1 on
// error, -3 when the next record is corrupt (CRC mismatch with later data present), or
// -(needed bytes)-16 when the next record alone does not fit in `out`.
long long oryx_reader_poll(void* rh, char* out, long long out_cap, int max_records,
                           int timeout_ms, long long* out_used) {
  auto* r = static_cast<Reader*>(rh);
  const std::string& dir = r->topic->parts[r->part].dir;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  long long used = 0;
  int count = 0;
  int sleep_us = 200;
  for (;;) {
    if (r->fd < 0) {
      reader_seek(r, r->next_offset);
    }
    bool progressed = false;
    while (r->fd >= 0 && count < max_records) {
      const uint8_t* h = reader_bytes(r, r->pos, kHeader);
      if (!h) break;
      uint32_t magic, crc, klen, vlen;
      uint64_t off;
      int64_t ts;
      memcpy(&magic, h, 4); memcpy(&crc, h + 4, 4); memcpy(&off, h + 8, 8);
      memcpy(&ts, h + 16, 8); memcpy(&klen, h + 24, 4); memcpy(&vlen, h + 28, 4);
      if (!known_magic(magic)) { r->blk_pos = -1; r->at_tail = true; break; }
      size_t kl = klen == kNullKey ? 0 : klen;
      size_t plen = kl + vlen;
      // the whole frame, so header and payload are contiguous in the block
      const uint8_t* f = reader_bytes(r, r->pos, kHeader + plen);
      if (!f) break;
      const uint8_t* pl = f + kHeader;
      if (frame_crc(magic, f, plen) != crc) {
        r->blk_pos = -1;
        // A torn or in-progress write can only be the tail of the segment; a bad frame with
        // a complete frame header written after it is corruption, reported instead of being
        // waited on forever.
        struct stat st;
        if (fstat(r->fd, &st) == 0 &&
            (long long)st.st_size >= r->pos + (long long)(kHeader + plen + kHeader)) {
          if (count > 0) break;   // deliver the good records first; the next poll reports
          *out_used = 0;
          fail("corrupt record (crc mismatch) in " + dir + " at offset " +
               std::to_string(r->next_offset));
          return -3;
        }
        break;  // torn / in-progress write
      }
      long long need = 24 + (long long)plen;
      if (used + need > out_cap) {
        if (count == 0) { *out_used = 0; return -need - 16; }
        *out_used = used;
        return count;
      }
      char* o = out + used;
      int64_t o_off = (int64_t)off;
      int32_t o_kl = klen == kNullKey ? -1 : (int32_t)klen;
      int32_t o_vl = (int32_t)vlen;
      memcpy(o, &o_off, 8); memcpy(o + 8, &ts, 8); memcpy(o + 16, &o_kl, 4);
      memcpy(o + 20, &o_vl, 4); memcpy(o + 24, pl, plen);
      used += need;
      r->pos += kHeader + plen;
      r->next_offset = (int64_t)off + 1;
      ++count;
      progressed = true;
      r->at_tail = false;
    }
    if (count >= max_records) break;
    if (!progressed) {
      // maybe the writer rolled to a new segment
      std::vector<int64_t> segs = list_segments(dir);
      bool rolled = false;
      for (int64_t b : segs) {
        if (b > r->seg_base && b <= r->next_offset) {
          if (r->fd >= 0) close(r->fd);
          r->blk_pos = -1;
          r->seg_base = b;
          r->pos = 0;
          r->fd = open(seg_name(dir, b).c_str(), O_RDONLY);
          rolled = true;
          break;
        }
      }
      if (rolled) continue;
      if (count > 0 || std::chrono::steady_clock::now() >= deadline) break;
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      sleep_us = std::min(sleep_us * 2, 2000);   // <= 2 ms behind a new record
    } else if (count > 0) {
      break;  // deliver what we have
    }
  }
  *out_used = used;
  return count;
}

// Records sharing one key (or none: key_len -1) given as one blob of values plus their byte
// lengths (the producer's fast path: no per-record framing in the caller); same semantics
// as oryx_log_append_batch.
long long oryx_log_append_values_gap(void* h, int partition, const char* key, int key_len,
                                     const char* blob, const long long* lens, int n, int gap,
                                     long long ts_ms, int do_fsync);

long long oryx_log_append_values(void* h, int partition, const char* key, int key_len,
                                 const char* blob, const long long* lens, int n,
                                 long long ts_ms, int do_fsync) {
  return oryx_log_append_values_gap(h, partition, key, key_len, blob, lens, n, 0, ts_ms,
                                    do_fsync);
}

// As oryx_log_append_values with `gap` separator bytes after every value in blob (e.g. the
// '\n' between the messages of a native formatter's output).  Frames are built straight from
// the blob (no packed intermediate copy).
long long oryx_log_append_values_gap(void* h, int partition, const char* key, int key_len,
                                     const char* blob, const long long* lens, int n, int gap,
                                     long long ts_ms, int do_fsync) {
  auto* t = static_cast<Topic*>(h);
  std::vector<RecRef> recs((size_t)n);
  const char* v = blob;
  for (int i = 0; i < n; ++i) {
    recs[(size_t)i] = RecRef{key_len < 0 ? nullptr : key, key_len < 0 ? -1 : key_len, v,
                             (int64_t)lens[i]};
    v += lens[i] + gap;
  }
  return append_records(t, h, partition, recs, ts_ms, do_fsync, nullptr);
}

// Records sharing one key whose values a producer writes itself: record j has lens[j] value
// bytes, which fill(ctx, j, dst) stores at dst -- straight into the segment's mapped page
// cache on the large-append path, so a producer that formats its messages there (the speed
// layer's UP assembly, oryx_speed_append) costs one pass over the bytes, CRCs included (each
// frame's CRC is computed by the thread that just wrote it).  fill runs on several native
// threads at once for large appends.  Same results as oryx_log_append_values.
long long oryx_log_append_fill(void* h, int partition, const char* key, int key_len,
                               const long long* lens, int n, FillFn fill, void* ctx,
                               long long ts_ms, int do_fsync) {
  auto* t = static_cast<Topic*>(h);
  std::vector<RecRef> recs((size_t)n);
  for (int i = 0; i < n; ++i)
    recs[(size_t)i] = RecRef{key_len < 0 ? nullptr : key, key_len < 0 ? -1 : key_len, nullptr,
                             (int64_t)lens[i]};
  return append_records(t, h, partition, recs, ts_ms, do_fsync, nullptr, fill, ctx);
}

// Bulk poll for consumers that parse records natively (the serving model load): complete
// frames from the reader's position are read with ONE pread straight into `out`, in the
// log's own frame layout (u32 magic | u32 crc | u64 offset | i64 ts | u32 key len
// (0xFFFFFFFF = null) | u32 value len | key | value), and their CRCs are checked on the native
// threads -- no per-record copy through the read-ahead block.  Never waits.  Returns the
// number of frames (at most max_records; 0 when none is complete yet), -3 on a corrupt frame
// that later data follows, or -(bytes needed) - 16 when the next frame alone exceeds out_cap.
long long oryx_reader_poll_frames(void* rh, char* out, long long out_cap, int max_records,
                                  long long* out_used) {
  auto* r = static_cast<Reader*>(rh);
  const std::string& dir = r->topic->parts[r->part].dir;
  *out_used = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (r->fd < 0) reader_seek(r, r->next_offset);
    if (r->fd < 0) return 0;
    r->blk_pos = -1;   // the poll read-ahead block is bypassed from here on
    // the next frame's header first: at the end of the data (possibly a preallocated zero
    // tail) a bulk read of out_cap bytes would copy nothing useful
    {
      uint8_t h[kHeader];
      const ssize_t hg = pread(r->fd, h, kHeader, r->pos);
      uint32_t magic = 0;
      if (hg == (ssize_t)kHeader) memcpy(&magic, h, 4);
      if (hg == (ssize_t)kHeader && !known_magic(magic)) {
        bool rolled = false;
        for (int64_t b : list_segments(dir)) {
          if (b > r->seg_base && b <= r->next_offset) {
            close(r->fd);
            r->seg_base = b;
            r->pos = 0;
            r->fd = open(seg_name(dir, b).c_str(), O_RDONLY);
            rolled = true;
            break;
          }
        }
        if (!rolled) return 0;
        continue;
      }
    }
    // the bulk read in 8 MB chunks on the native threads: one pread is a single-threaded
    // page-cache copy (~5 GB/s), which bounded a 57 GB model load
    ssize_t got = 0;
    {
      constexpr long long kChunk = 8LL << 20;
      const long long nch = (out_cap + kChunk - 1) / kChunk;
      std::vector<long long> cgot((size_t)nch, 0);
      const int fd = r->fd;
      const long long base = r->pos;
      oryx_ff::parallel_ranges(nch, 1, [&](long long lo, long long hi, int) {
        for (long long c = lo; c < hi; ++c) {
          const long long off = c * kChunk;
          const long long len = std::min(kChunk, out_cap - off);
          long long done = 0;
          while (done < len) {
            const ssize_t g = pread(fd, out + off + done, (size_t)(len - done), base + off + done);
            if (g <= 0) break;
            done += g;
          }
          cgot[(size_t)c] = done;
        }
      });
      for (long long c = 0; c < nch; ++c) {
        got += (ssize_t)cgot[(size_t)c];
        if (cgot[(size_t)c] < std::min(kChunk, out_cap - c * kChunk)) break;   // end of data
      }
    }
    std::vector<size_t> at;
    size_t p = 0;
    while ((long long)at.size() < max_records && p + kHeader <= (size_t)got) {
      const uint8_t* h = reinterpret_cast<const uint8_t*>(out) + p;
      uint32_t magic, klen, vlen;
      memcpy(&magic, h, 4); memcpy(&klen, h + 24, 4); memcpy(&vlen, h + 28, 4);
      if (!known_magic(magic)) break;
      const size_t plen = (klen == kNullKey ? 0 : klen) + (size_t)vlen;
      if (p + kHeader + plen > (size_t)got) {
        if (at.empty() && (long long)(kHeader + plen) > out_cap)
          return -(long long)(kHeader + plen) - 16;
        break;
      }
      at.push_back(p);
      p += kHeader + plen;
    }
    const long long n = (long long)at.size();
    if (n == 0) {
      if (got > 0) return 0;          // a frame still being written
      // end of this segment file: move to the next one when the writer has rolled
      bool rolled = false;
      for (int64_t b : list_segments(dir)) {
        if (b > r->seg_base && b <= r->next_offset) {
          close(r->fd);
          r->seg_base = b;
          r->pos = 0;
          r->fd = open(seg_name(dir, b).c_str(), O_RDONLY);
          rolled = true;
          break;
        }
      }
      if (!rolled) return 0;
      continue;
    }
    std::vector<unsigned char> bad((size_t)n, 0);
    oryx_ff::parallel_ranges(n, 512, [&](long long lo, long long hi, int) {
      for (long long j = lo; j < hi; ++j) {
        const uint8_t* f = reinterpret_cast<const uint8_t*>(out) + at[(size_t)j];
        uint32_t magic, crc, klen, vlen;
        memcpy(&magic, f, 4); memcpy(&crc, f + 4, 4); memcpy(&klen, f + 24, 4);
        memcpy(&vlen, f + 28, 4);
        const size_t plen = (klen == kNullKey ? 0 : klen) + (size_t)vlen;
        if (frame_crc(magic, f, plen) != crc) bad[(size_t)j] = 1;
      }
    });
    long long good = n;
    for (long long j = 0; j < n; ++j)
      if (bad[(size_t)j]) { good = j; break; }
    if (good < n) {
      if (good == 0) {
        // a bad frame followed by more data is corruption; at the tail it is a torn or
        // in-progress write
        const size_t p0 = at[0];
        const uint8_t* f = reinterpret_cast<const uint8_t*>(out) + p0;
        uint32_t klen, vlen;
        memcpy(&klen, f + 24, 4); memcpy(&vlen, f + 28, 4);
        const size_t flen = kHeader + (klen == kNullKey ? 0 : klen) + (size_t)vlen;
        struct stat st;
        if (fstat(r->fd, &st) == 0 && (long long)st.st_size >= r->pos + (long long)(flen + kHeader)) {
          fail("corrupt record (crc mismatch) in " + dir + " at offset " +
               std::to_string(r->next_offset));
          return -3;
        }
        return 0;
      }
    }
    const size_t last = at[(size_t)good - 1];
    const uint8_t* f = reinterpret_cast<const uint8_t*>(out) + last;
    uint64_t off;
    uint32_t klen, vlen;
    memcpy(&off, f + 8, 8); memcpy(&klen, f + 24, 4); memcpy(&vlen, f + 28, 4);
    const size_t end = last + kHeader + (klen == kNullKey ? 0 : klen) + (size_t)vlen;
    r->pos += (int64_t)end;
    r->next_offset = (int64_t)off + 1;
    *out_used = (long long)end;
    return good;
  }
  return 0;
}

// Upper bound on the bytes oryx_reader_read_text delivers for the records from the reader's
// position up to `end_offset`: the segment bytes from the position to the current end of the
// log, less 31 per record (each frame has a 32-byte header; the text adds one '\n').  Lets
// the caller allocate the output once.
long long oryx_reader_text_bound(void* rh, long long end_offset) {
  auto* r = static_cast<Reader*>(rh);
  if (r->fd < 0) reader_seek(r, r->next_offset);
  if (r->next_offset >= end_offset) return 0;
  const std::string& dir = r->topic->parts[r->part].dir;
  long long bytes = 0;
  for (int64_t b : list_segments(dir)) {
    if (b < r->seg_base) continue;
    struct stat st;
    if (stat(seg_name(dir, b).c_str(), &st) != 0) continue;
    bytes += (long long)st.st_size - (b == r->seg_base ? (long long)r->pos : 0);
  }
  const long long bound = bytes - 31 * (end_offset - r->next_offset);
  return bound > 0 ? bound : 0;
}

// Bulk text read for the batch layer's drains: every record from the reader's position up
// to `end_offset` (exclusive) appended to `out` as `value '\n'`, reading the segment files in
// 4 MB blocks (one pread per block instead of two per record).  Returns the number of
// records consumed (fewer than asked when `out` is full: call again), or -3 on a corrupt
// frame.  *flags gets bit 0 when a record had a key and bit 1 when a value contained a newline
// (the caller then uses the per-record path for those semantics), and bit 2 when the next
// record alone is larger than out_cap (nothing delivered; *out_used is the size it needs).
long long oryx_reader_read_text(void* rh, long long end_offset, char* out, long long out_cap,
                                long long* out_used, int* flags) {
  auto* r = static_cast<Reader*>(rh);
  const std::string& dir = r->topic->parts[r->part].dir;
  constexpr size_t kBlock = 4u << 20;
  // per-thread block (a fresh 4 MB vector per call paid its page faults every time)
  thread_local std::vector<uint8_t> buf;
  if (buf.size() < kBlock) buf.resize(kBlock);
  long long used = 0, count = 0;
  *flags = 0;
  if (r->fd < 0) reader_seek(r, r->next_offset);
  while (r->next_offset < end_offset) {
    if (r->fd < 0) break;
    const size_t cap = buf.size();
    ssize_t got = pread(r->fd, buf.data(), cap, r->pos);
    size_t at = 0;
    bool need_more = false;
    while (got > 0 && at + kHeader <= (size_t)got && r->next_offset < end_offset) {
      const uint8_t* h = buf.data() + at;
      uint32_t magic, crc, klen, vlen;
      uint64_t off;
      memcpy(&magic, h, 4); memcpy(&crc, h + 4, 4); memcpy(&off, h + 8, 8);
      memcpy(&klen, h + 24, 4); memcpy(&vlen, h + 28, 4);
      if (!known_magic(magic)) { got = 0; break; }
      size_t kl = klen == kNullKey ? 0 : klen;
      size_t plen = kl + vlen;
      if (at + kHeader + plen > (size_t)got) {
        // frame straddles the block: re-read from its start (grow for huge frames)
        if (kHeader + plen > buf.size()) buf.resize(kHeader + plen);
        need_more = true;
        break;
      }
      // crc covers offset | ts | key | value (the 16 header bytes at +8 and the payload)
      if (frame_crc(magic, h, plen) != crc) {
        *out_used = used;
        fail("corrupt record (crc mismatch) in " + dir + " at offset " +
             std::to_string(r->next_offset));
        return -3;
      }
      if ((long long)off >= end_offset) { r->next_offset = end_offset; break; }
      if (used + (long long)vlen + 1 > out_cap) {
        // buffer full; with nothing delivered yet, report the size this record needs
        if (count == 0) {
          *flags |= 4;
          *out_used = (long long)vlen + 1;
        } else {
          *out_used = used;
        }
        return count;
      }
      if (klen != kNullKey) *flags |= 1;
      const uint8_t* v = h + kHeader + kl;
      if (memchr(v, '\n', vlen)) *flags |= 2;
      memcpy(out + used, v, vlen);
      out[used + vlen] = '\n';
      used += vlen + 1;
      at += kHeader + plen;
      r->pos += kHeader + plen;
      r->next_offset = (int64_t)off + 1;
      ++count;
    }
    if (r->next_offset >= end_offset) break;
    // a frame cut off by a short read is still being written (or torn): deliver what there is
    if (need_more) {
      if (got < (ssize_t)cap) break;
      continue;
    }
    if (at == 0) {
      // end of this segment file: move to the next one (records up to end_offset exist)
      std::vector<int64_t> segs = list_segments(dir);
      bool rolled = false;
      for (int64_t b : segs) {
        if (b > r->seg_base && b <= r->next_offset) {
          close(r->fd);
          r->seg_base = b;
          r->pos = 0;
          r->fd = open(seg_name(dir, b).c_str(), O_RDONLY);
          r->blk_pos = -1;   // the poll read-ahead block holds the previous file's bytes
          rolled = true;
          break;
        }
      }
      if (!rolled) break;   // not written yet: deliver what there is
    }
  }
  *out_used = used;
  return count;
}

// ---- consumer-group offsets (ZooKeeper replacement) ----

static std::string offsets_path(const char* root, const char* topic, const char* group) {
  return std::string(root) + "/" + topic + "/.offsets/" + group;
}

// Writes `n` (partition, offset) pairs atomically (tmp + fsync + rename).
int oryx_offsets_set(const char* root, const char* topic, const char* group, int n,
                     const int* partitions, const long long* offsets) {
  errno = 0;
  std::string path = offsets_path(root, topic, group);
  if (!mkdirs(path.substr(0, path.find_last_of('/')))) return fail("mkdir offsets");
  // merge with existing
  std::vector<long long> cur;
  {
    FILE* f = fopen(path.c_str(), "r");
    if (f) {
      int p; long long o;
      while (fscanf(f, "%d %lld", &p, &o) == 2) {
        if (p >= 0 && p < 1 << 20) {
          if ((int)cur.size() <= p) cur.resize(p + 1, -1);
          cur[p] = o;
        }
      }
      fclose(f);
    }
  }
  for (int i = 0; i < n; ++i) {
    if ((int)cur.size() <= partitions[i]) cur.resize(partitions[i] + 1, -1);
    cur[partitions[i]] = offsets[i];
  }
  std::string tmp = path + ".tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return fail("open offsets tmp");
  for (size_t p = 0; p < cur.size(); ++p)
    if (cur[p] >= 0) fprintf(f, "%zu %lld\n", p, cur[p]);
  fflush(f);
  fsync(fileno(f));
  fclose(f);
  if (rename(tmp.c_str(), path.c_str()) != 0) return fail("rename offsets");
  return 0;
}

// Returns the committed offset of one partition, or -1 if none.
long long oryx_offsets_get(const char* root, const char* topic, const char* group,
                           int partition) {
  FILE* f = fopen(offsets_path(root, topic, group).c_str(), "r");
  if (!f) return -1;
  int p; long long o, res = -1;
  while (fscanf(f, "%d %lld", &p, &o) == 2) if (p == partition) res = o;
  fclose(f);
  return res;
}

}  // extern "C"
