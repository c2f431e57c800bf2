// oryx_ingest.cpp -- native data loading for the batch/speed layers.
//
// The reference parses input lines inside Spark tasks ([app-common]/common/fn/MLFunctions.java:39-65,
// [mllib]/als/ALSUpdate.java:260-290) and maps string IDs to ints by parse-or-MD5-hash with a
// reverse lookup collected to the driver (C4 in SURVEY.md section 2.5).  Here one C++ pass turns a
// buffer of "user,item[,strength[,timestamp]]" lines (or JSON arrays) into dense dictionary
// codes, strengths (NaN = delete) and timestamps, ready to upload as device tensors; the
// dictionaries are collision-free (no hashing of IDs) and persist across intervals.
// Also: shortest-round-trip float formatting of factor rows for JSON update messages.

#include <algorithm>
#include <array>
#include <charconv>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <limits>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include <zlib.h>

#include "fastfloat.h"

namespace {

// Open-addressing string -> int32 index for the parse hot loop (std::unordered_map costs a
// node and a key indirection per lookup: two cache misses once the IDs number 1e5).  Keys of
// up to 16 bytes are stored inline, longer ones as views (into the input buffer or owned
// storage); the full 64-bit hash is compared first.
class FlatIndex {
 public:
  FlatIndex() { rehash(1024); }
  // grow once to hold about n keys (load <= 1/2) instead of doubling through every size
  void reserve(size_t n) {
    size_t cap = slots_.size();
    while (cap < 2 * n) cap *= 2;
    if (cap > slots_.size()) rehash(cap);
  }
  // value of key k, or -1
  int32_t find(std::string_view k) const {
    const uint64_t h = hash(k.data(), k.size());
    const size_t m = slots_.size() - 1;
    for (size_t j = (size_t)h & m;; j = (j + 1) & m) {
      const Slot& sl = slots_[j];
      if (sl.code < 0) return -1;
      if (sl.h == h && sl.len == k.size() &&
          std::memcmp(k.size() <= 16 ? sl.in : sl.ptr, k.data(), k.size()) == 0)
        return sl.code;
    }
  }
  // index of key k, inserting it with value `next` when absent (*inserted set)
  int32_t find_or_add(std::string_view k, int32_t next, bool* inserted) {
    const uint64_t h = hash(k.data(), k.size());
    size_t m = slots_.size() - 1, j = (size_t)h & m;
    while (true) {
      Slot& sl = slots_[j];
      if (sl.code < 0) {
        if ((used_ + 1) * 2 > slots_.size()) {
          rehash(slots_.size() * 2);
          return find_or_add(k, next, inserted);
        }
        sl.h = h;
        sl.len = (uint32_t)k.size();
        sl.code = next;
        if (k.size() <= 16) std::memcpy(sl.in, k.data(), k.size());
        else sl.ptr = k.data();
        ++used_;
        last_ = j;
        *inserted = true;
        return next;
      }
      if (sl.h == h && sl.len == k.size() &&
          std::memcmp(k.size() <= 16 ? sl.in : sl.ptr, k.data(), k.size()) == 0) {
        *inserted = false;
        return sl.code;
      }
      j = (j + 1) & m;
    }
  }
  // a long key inserted from a transient view is re-pointed at its stable copy
  void repoint_last(const char* p) {
    if (slots_[last_].len > 16) slots_[last_].ptr = p;
  }
  // empty, keeping the table's capacity (a reused dictionary allocates nothing)
  void clear() {
    for (Slot& sl : slots_) sl.code = -1;
    used_ = 0;
  }

 private:
  struct Slot {
    uint64_t h = 0;
    uint32_t len = 0;
    int32_t code = -1;
    union {
      char in[16];
      const char* ptr;
    };
    Slot() : in{} {}
  };
  static uint64_t mix(uint64_t a, uint64_t b) {
    const unsigned __int128 r = (unsigned __int128)a * b;
    return (uint64_t)r ^ (uint64_t)(r >> 64);
  }
  static uint64_t hash(const char* p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    while (n >= 8) {
      uint64_t v;
      std::memcpy(&v, p, 8);
      h = mix(h ^ v, 0xA0761D6478BD642Full);
      p += 8;
      n -= 8;
    }
    uint64_t v = 0;
    std::memcpy(&v, p, n);
    return mix(h ^ v, 0xE7037ED1A0B428DBull);
  }
  void rehash(size_t cap) {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(cap, Slot());
    used_ = 0;
    const size_t m = cap - 1;
    for (const Slot& sl : old) {
      if (sl.code < 0) continue;
      size_t j = (size_t)sl.h & m;
      while (slots_[j].code >= 0) j = (j + 1) & m;
      slots_[j] = sl;
      ++used_;
    }
  }
  std::vector<Slot> slots_;
  size_t used_ = 0;
  size_t last_ = 0;
};

// A key that is a canonical decimal integer below kNumLimit ("0", "17", not "017" / "+1" /
// "1.0"): such IDs (most real datasets') index a dense array instead of the hash table.  A
// random probe into a table of 1e5-1e6 string slots costs a cache and TLB miss (~100-200 ns);
// the array is 4 bytes per value and mostly cache resident.
constexpr uint32_t kNumLimit = 1u << 24;

inline bool numeric_key(std::string_view s, uint32_t* v) {
  const size_t n = s.size();
  if (n == 0 || n > 8 || (s[0] == '0' && n > 1)) return false;
  uint32_t x = 0;
  for (size_t j = 0; j < n; ++j) {
    const unsigned d = (unsigned char)s[j] - '0';
    if (d > 9) return false;
    x = x * 10 + d;
  }
  if (x >= kNumLimit) return false;
  *v = x;
  return true;
}

struct Dict {
  // the index's long keys are views of the strings in `keys` (a deque: elements never move);
  // open addressing (FlatIndex): a micro-batch's fresh dictionary of 10k IDs costs no node
  // allocations, and lookups in a 1e6-ID dictionary one cache miss
  FlatIndex map;
  std::deque<std::string> keys;
  // numeric keys: value -> code (-1 absent), and the values present (for clear())
  std::vector<int32_t> num;
  std::vector<uint32_t> num_present;
  std::mutex mu;
  int64_t encode_num(uint32_t v) {
    if (v >= num.size()) {
      size_t sz = std::max<size_t>({(size_t)v + 1, num.size() * 2, 1024});
      num.resize(std::min<size_t>(sz, kNumLimit), -1);
    }
    int32_t& c = num[v];
    if (c >= 0) return c;
    c = (int32_t)keys.size();
    char b[12];
    const auto r = std::to_chars(b, b + sizeof(b), v);
    keys.emplace_back(b, (size_t)(r.ptr - b));
    num_present.push_back(v);
    return c;
  }
  int64_t encode(std::string_view s) {
    uint32_t v;
    if (numeric_key(s, &v)) return encode_num(v);
    bool ins;
    const int32_t code = map.find_or_add(s, (int32_t)keys.size(), &ins);
    if (ins) {
      keys.emplace_back(s);
      map.repoint_last(keys.back().data());
    }
    return code;
  }
  int64_t find(std::string_view s) const {
    uint32_t v;
    if (numeric_key(s, &v)) return v < num.size() ? num[v] : -1;
    return map.find(s);
  }
  void clear() {
    map.clear();
    for (uint32_t v : num_present) num[v] = -1;
    num_present.clear();
    keys.clear();
  }
};

// Parse one CSV field starting at p (RFC 4180 quotes, backslash escapes).  Returns end position.
const char* csv_field(const char* p, const char* end, std::string& out) {
  out.clear();
  if (p < end && *p == '"') {
    ++p;
    while (p < end) {
      char c = *p;
      if (c == '\\' && p + 1 < end) { out.push_back(p[1]); p += 2; continue; }
      if (c == '"') {
        if (p + 1 < end && p[1] == '"') { out.push_back('"'); p += 2; continue; }
        ++p;
        break;
      }
      out.push_back(c);
      ++p;
    }
    while (p < end && *p != ',') out.push_back(*p++);
  } else {
    while (p < end && *p != ',') {
      if (*p == '\\' && p + 1 < end) { out.push_back(p[1]); p += 2; continue; }
      out.push_back(*p++);
    }
  }
  return p;
}

// Minimal JSON array-of-primitives parser: ["a", 1, "2.5", 123] -> tokens as strings.
bool json_fields(const char* p, const char* end, std::vector<std::string>& toks) {
  toks.clear();
  if (p >= end || *p != '[') return false;
  ++p;
  std::string cur;
  while (p < end) {
    while (p < end && (*p == ' ' || *p == '\t' || *p == ',')) ++p;
    if (p >= end) return false;
    if (*p == ']') return true;
    cur.clear();
    if (*p == '"') {
      ++p;
      while (p < end && *p != '"') {
        if (*p == '\\' && p + 1 < end) {
          char e = p[1];
          cur.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e);
          p += 2;
          continue;
        }
        cur.push_back(*p++);
      }
      ++p;
    } else {
      while (p < end && *p != ',' && *p != ']' && *p != ' ') cur.push_back(*p++);
      if (cur == "null") cur.clear();
    }
    toks.push_back(cur);
  }
  return false;
}

bool parse_double(const std::string& s, double* out) {
  if (s.empty()) return false;
  const char* b = s.data();
  const char* e = b + s.size();
  while (b < e && (*b == ' ' || *b == '+')) ++b;
  auto r = std::from_chars(b, e, *out);
  return r.ec == std::errc() && r.ptr == e;
}

}  // namespace

extern "C" {

void* oryx_dict_new() { return new Dict(); }
void oryx_dict_free(void* d) { delete static_cast<Dict*>(d); }
long long oryx_dict_size(void* d) { return (long long)static_cast<Dict*>(d)->keys.size(); }

// Empties a dictionary for reuse (the speed layer's per-micro-batch dictionaries): the hash
// table keeps its capacity, so the next batch's IDs are inserted without allocating it again.
void oryx_dict_clear(void* dh) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  d->clear();
}

// Encodes n strings packed back to back (lengths in lens) -> codes.  Returns n.
long long oryx_dict_encode(void* dh, const char* buf, long long buf_len, int n, long long* codes) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  // buf holds n NUL-terminated strings
  const char* p = buf;
  const char* end = buf + buf_len;
  for (int i = 0; i < n && p < end; ++i) {
    size_t len = strnlen(p, end - p);
    codes[i] = d->encode(std::string_view(p, len));
    p += len + 1;
  }
  return n;
}

// Encodes n canonical decimal keys given by value (each < 2^24: the dense-array keys of
// numeric_key) in order -> codes: what encoding their decimal strings would do, without the
// strings (the device rating parse numbers a segment's keys in first-appearance order and
// hands them over here).  Returns n, or -1 for a value out of range.
long long oryx_dict_encode_nums(void* dh, const int32_t* vals, long long n, long long* codes) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  for (long long j = 0; j < n; ++j)
    if (vals[j] < 0 || (uint32_t)vals[j] >= kNumLimit) return -1;
  for (long long j = 0; j < n; ++j) {
    const int64_t c = d->encode_num((uint32_t)vals[j]);
    if (codes) codes[j] = c;
  }
  return n;
}

// Inserts every key of src (in src's code order) into dst; map_out[c] = dst code of src key c.
// Merging per-segment dictionaries in segment order reproduces the codes a single parse of the
// concatenated segments assigns (first appearance order).  Returns src's size.
long long oryx_dict_merge(void* dst_h, void* src_h, long long* map_out) {
  Dict* d = static_cast<Dict*>(dst_h);
  Dict* s = static_cast<Dict*>(src_h);
  if (d == s) return -1;
  std::scoped_lock g(d->mu, s->mu);
  long long c = 0;
  for (const std::string& k : s->keys) map_out[c++] = d->encode(std::string_view(k));
  return c;
}

long long oryx_dict_get(void* dh, const char* s, long long len) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  return d->find(std::string_view(s, (size_t)len));
}

// ---- blob forms for the sharded batch layer's global dictionaries (parallel/shuffle.py):
// keys travel between ranks as one byte blob plus end offsets, never as Python strings.

// owner[c] = zlib crc32(key c) % world for keys [from, size) (the same owner function as
// shuffle.owner_of_strings).  Returns the number of keys written.
long long oryx_dict_owners(void* dh, long long from, int world, long long* owner) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  long long n = 0;
  for (size_t c = (size_t)from; c < d->keys.size(); ++c, ++n) {
    const std::string& k = d->keys[c];
    const uLong h = crc32(0L, reinterpret_cast<const Bytef*>(k.data()), (uInt)k.size());
    owner[n] = (long long)(h % (uLong)world);
  }
  return n;
}

// Inserts the n keys of blob (key j = blob[ends[j-1], ends[j])) in order; codes[j] = its
// code.  Returns n.
long long oryx_dict_encode_blob(void* dh, const char* blob, const long long* ends, long long n,
                                long long* codes) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  long long at = 0;
  for (long long j = 0; j < n; ++j) {
    codes[j] = d->encode(std::string_view(blob + at, (size_t)(ends[j] - at)));
    at = ends[j];
  }
  return n;
}

// As oryx_dict_encode_blob without inserting: codes[j] = -1 for keys not present.
long long oryx_dict_find_blob(void* dh, const char* blob, const long long* ends, long long n,
                              long long* codes) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  long long at = 0;
  for (long long j = 0; j < n; ++j) {
    codes[j] = d->find(std::string_view(blob + at, (size_t)(ends[j] - at)));
    at = ends[j];
  }
  return n;
}

// The keys of codes[0..n) back to back in out; ends[j] = end offset of key j.  Returns bytes
// used or -(bytes needed) when out is too small; an out-of-range code gives an empty key.
long long oryx_dict_keys_blob_sel(void* dh, const long long* codes, long long n, char* out,
                                  long long cap, long long* ends) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  const long long size = (long long)d->keys.size();
  long long need = 0;
  for (long long j = 0; j < n; ++j)
    if (codes[j] >= 0 && codes[j] < size) need += (long long)d->keys[(size_t)codes[j]].size();
  if (need > cap) return -need;
  long long pos = 0;
  for (long long j = 0; j < n; ++j) {
    if (codes[j] >= 0 && codes[j] < size) {
      const std::string& k = d->keys[(size_t)codes[j]];
      memcpy(out + pos, k.data(), k.size());
      pos += (long long)k.size();
    }
    ends[j] = pos;
  }
  return pos;
}

// Copies key `code` into out (cap bytes); returns its length (or -1).
long long oryx_dict_key(void* dh, long long code, char* out, long long cap) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  if (code < 0 || code >= (long long)d->keys.size()) return -1;
  const std::string& k = d->keys[code];
  if ((long long)k.size() <= cap) memcpy(out, k.data(), k.size());
  return (long long)k.size();
}

}  // extern "C"

namespace {

// One chunk of rating lines parsed by one thread: IDs get chunk-local codes (first-appearance
// order) from chunk-local maps of views; the caller merges the local dictionaries into the
// global ones in chunk order, which reproduces the global first-appearance numbering.
// Fields of one rating line [p, lend) ("user,item[,strength[,timestamp]]" CSV, RFC 4180
// quotes / backslash escapes, or a JSON array): f[0..] views of the fields, *sv the strength
// (NaN when empty = delete, 1 when missing), *tv the timestamp (left as given when missing).
// *stable: the views point into the line itself (plain CSV) rather than into `toks`.
// Returns false for a line that is not a rating.
inline bool parse_rating_fields(const char* p, const char* lend, std::vector<std::string>& toks,
                                std::string& field, std::string_view f[4], bool* stable,
                                double* sv, long long* tv) {
  int nf = 0;
  *sv = 1.0;
  // fast path: plain CSV (no quotes / escapes): fields are views of the line
  if (*p != '[' && !memchr(p, '"', (size_t)(lend - p)) &&
      !memchr(p, '\\', (size_t)(lend - p))) {
    const char* q = p;
    while (nf < 4) {
      const char* c = static_cast<const char*>(memchr(q, ',', (size_t)(lend - q)));
      const char* fe = c ? c : lend;
      f[nf++] = std::string_view(q, (size_t)(fe - q));
      if (!c) break;
      q = c + 1;
    }
    *stable = true;
  } else {
    toks.clear();
    if (*p == '[' && lend[-1] == ']') {
      if (!json_fields(p, lend, toks)) toks.clear();
    } else {
      const char* q = p;
      while (true) {
        q = csv_field(q, lend, field);
        toks.push_back(field);
        if (q >= lend) break;
        ++q;
        if (q >= lend) { toks.emplace_back(); break; }
      }
    }
    for (size_t t = 0; t < toks.size() && nf < 4; ++t) f[nf++] = toks[t];
    *stable = false;
  }
  bool ok = nf >= 2;
  if (ok && nf >= 3) {
    if (f[2].empty()) *sv = std::numeric_limits<double>::quiet_NaN();
    else ok = oryx_ff::parse_double(f[2].data(), f[2].data() + f[2].size(), *sv);
  }
  if (ok && nf >= 4 && !f[3].empty()) {
    // epoch milliseconds are plain digits: integer fast path, the float parser for anything
    // else ("1.7e12", signs, spaces)
    const char* a = f[3].data();
    const size_t m = f[3].size();
    size_t d = 0;
    long long iv = 0;
    while (d < m && d < 18 && a[d] >= '0' && a[d] <= '9') iv = iv * 10 + (a[d++] - '0');
    if (d == m) {
      *tv = iv;
    } else {
      double t;
      ok = oryx_ff::parse_double(a, a + m, t);
      *tv = (long long)t;
    }
  }
  return ok;
}

struct RatingChunk {
  // per side (users / items): chunk-local codes of string keys, and the chunk's keys in
  // first-appearance order (>= 0: a string key's local code; < 0: numeric key -(value + 1),
  // which is also what the row stores -- its global code is read from the dictionary's
  // dense array after the merge)
  struct Side {
    FlatIndex m;
    std::vector<std::string_view> keys;
    std::vector<int64_t> order;
    std::vector<uint64_t> seen;      // bitmap of numeric values met in this chunk
  };
  std::vector<int32_t> u, i;
  std::vector<double> s;
  std::vector<long long> ts;
  Side us, is;
  std::deque<std::string> owned;     // unescaped fields (quoted CSV / JSON lines)
  long long lines = 0, bad_line = -1;
  // single-chunk parse: codes straight from the global dictionaries (no chunk-local index
  // and merge; both dictionaries are locked by the caller)
  Dict* gu = nullptr;
  Dict* gi = nullptr;
  // timestamps / strengths only (the train/test split): IDs are not encoded at all
  bool no_ids = false;
  // the raw text span [begin, end) of every parsed row's line (the time split copies lines)
  bool want_spans = false;
  std::vector<const char*> sp_b, sp_e;
  // direct output (oryx_parse_ratings' multi-chunk path): rows go straight to these arrays
  // (room for every line of the chunk) instead of the vectors above -- no intermediate copy
  long long* d_u = nullptr;
  long long* d_i = nullptr;
  double* d_s = nullptr;
  long long* d_ts = nullptr;
  long long d_n = 0;

  int32_t code(Side& sd, std::string_view k, bool stable) {
    uint32_t v;
    if (numeric_key(k, &v)) {
      const size_t w = v >> 6;
      if (w >= sd.seen.size()) sd.seen.resize(std::max<size_t>(w + 1, sd.seen.size() * 2), 0);
      const uint64_t bit = 1ull << (v & 63);
      if (!(sd.seen[w] & bit)) {
        sd.seen[w] |= bit;
        sd.order.push_back(-(int64_t)v - 1);
      }
      return -(int32_t)v - 1;
    }
    if (!stable) {
      // an unescaped token lives in a per-line buffer: index a stable copy, made only for a
      // key not seen before
      const int32_t c = sd.m.find(k);
      if (c >= 0) return c;
      owned.emplace_back(k);
      k = owned.back();
    }
    bool inserted;
    const int32_t c = sd.m.find_or_add(k, (int32_t)sd.keys.size(), &inserted);
    if (inserted) {
      sd.keys.push_back(k);
      sd.order.push_back(c);
    }
    return c;
  }

  void parse(const char* p, const char* end, long long default_ts, bool strict) {
    std::vector<std::string> toks;
    std::string field;
    std::string_view f[4];
    while (p < end) {
      const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
      const char* le = nl ? nl : end;
      const char* lend = le;
      if (lend > p && lend[-1] == '\r') --lend;
      if (lend > p) {
        bool stable;
        double sv;
        long long tv = default_ts;
        const bool ok = parse_rating_fields(p, lend, toks, field, f, &stable, &sv, &tv);
        if (ok && d_u) {
          d_u[d_n] = code(us, f[0], stable);
          d_i[d_n] = code(is, f[1], stable);
          d_s[d_n] = sv;
          d_ts[d_n] = tv;
          ++d_n;
        } else if (ok) {
          if (no_ids) {
            u.push_back(0);
            i.push_back(0);
          } else if (gu) {
            u.push_back((int32_t)gu->encode(f[0]));
            i.push_back((int32_t)gi->encode(f[1]));
          } else {
            u.push_back(code(us, f[0], stable));
            i.push_back(code(is, f[1], stable));
          }
          s.push_back(sv);
          ts.push_back(tv);
          if (want_spans) {
            sp_b.push_back(p);
            sp_e.push_back(le);
          }
        } else if (strict && bad_line < 0) {
          bad_line = lines;
          return;
        }
      }
      ++lines;
      p = nl ? nl + 1 : end;
    }
  }
};

// oryx_parse_ratings' multi-chunk parse writing rows in place: chunk t parses into the
// outputs from index lines_at[t] (its first line), the chunk dictionaries are merged in
// order, then the rows' chunk-local codes become global ones -- in parallel when no line was
// dropped (rows then sit exactly where they belong), else in chunk order, moving each chunk's
// rows down to close the gaps (destinations never pass the rows still to be read).
long long parse_direct(Dict* du, Dict* di, std::vector<RatingChunk>& ch,
                       const std::vector<const char*>& cut, const std::vector<long long>& lines_at,
                       long long* out_u, long long* out_i, double* out_s, long long* out_ts,
                       long long default_ts, int strict) {
  const int P = (int)ch.size();
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      RatingChunk& c = ch[(size_t)t];
      const long long o = lines_at[(size_t)t];
      c.d_u = out_u + o;
      c.d_i = out_i + o;
      c.d_s = out_s + o;
      c.d_ts = out_ts + o;
      c.parse(cut[(size_t)t], cut[(size_t)t + 1], default_ts, strict != 0);
    }
  });
  long long lines_before = 0;
  for (int t = 0; t < P; ++t) {
    if (ch[(size_t)t].bad_line >= 0) return -(lines_before + ch[(size_t)t].bad_line + 1);
    lines_before += ch[(size_t)t].lines;
  }
  std::vector<std::vector<int64_t>> umap((size_t)P), imap((size_t)P);
  std::vector<long long> off((size_t)P + 1, 0);
  bool dense = true;
  auto merge = [](Dict* d, const RatingChunk::Side& sd, std::vector<int64_t>& to_global) {
    to_global.reserve(sd.keys.size());
    for (int64_t e : sd.order) {
      if (e < 0) d->encode_num((uint32_t)(-e - 1));
      else to_global.push_back(d->encode(sd.keys[(size_t)e]));
    }
  };
  for (int t = 0; t < P; ++t) {
    RatingChunk& c = ch[(size_t)t];
    merge(du, c.us, umap[(size_t)t]);
    merge(di, c.is, imap[(size_t)t]);
    off[(size_t)t + 1] = off[(size_t)t] + c.d_n;
    dense = dense && off[(size_t)t] == lines_at[(size_t)t];
  }
  const int32_t* unum = du->num.data();
  const int32_t* inum = di->num.data();
  auto remap = [&](long long t) {
    const RatingChunk& c = ch[(size_t)t];
    const long long src = lines_at[(size_t)t], dst = off[(size_t)t];
    const int64_t* um = umap[(size_t)t].data();
    const int64_t* im = imap[(size_t)t].data();
    for (long long r = 0; r < c.d_n; ++r) {
      const long long a = out_u[src + r], b = out_i[src + r];
      out_u[dst + r] = a < 0 ? unum[-(a + 1)] : um[a];
      out_i[dst + r] = b < 0 ? inum[-(b + 1)] : im[b];
      out_s[dst + r] = out_s[src + r];
      out_ts[dst + r] = out_ts[src + r];
    }
  };
  if (dense)
    oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
      for (long long t = lo; t < hi; ++t) remap(t);
    });
  else
    for (int t = 0; t < P; ++t) remap(t);
  return off[(size_t)P];
}

// Chunks at line boundaries over the native threads, no dictionaries (see oryx_parse_ratings).
long long parse_rows_no_ids(const char* buf, long long len, long long* out_u, long long* out_i,
                            double* out_s, long long* out_ts, long long max_rows,
                            long long default_ts, int strict) {
  int P = 1;
  if (len >= (1ll << 20))
    P = (int)std::max<long long>(1, std::min<long long>(len / (256ll << 10),
                                                       oryx_ff::native_threads()));
  std::vector<const char*> cut((size_t)P + 1);
  cut[0] = buf;
  cut[(size_t)P] = buf + len;
  for (int t = 1; t < P; ++t) {
    const char* c = buf + len * t / P;
    if (c < cut[(size_t)t - 1]) c = cut[(size_t)t - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(buf + len - c)));
    cut[(size_t)t] = nl ? nl + 1 : buf + len;
  }
  std::vector<RatingChunk> ch((size_t)P);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      ch[(size_t)t].no_ids = true;
      ch[(size_t)t].parse(cut[(size_t)t], cut[(size_t)t + 1], default_ts, strict != 0);
    }
  });
  long long lines_before = 0, o = 0;
  for (int t = 0; t < P; ++t) {
    if (ch[(size_t)t].bad_line >= 0) return -(lines_before + ch[(size_t)t].bad_line + 1);
    lines_before += ch[(size_t)t].lines;
  }
  for (int t = 0; t < P; ++t) {
    const RatingChunk& c = ch[(size_t)t];
    for (size_t r = 0; r < c.s.size() && o < max_rows; ++r, ++o) {
      if (out_u) out_u[o] = 0;
      if (out_i) out_i[o] = 0;
      out_s[o] = c.s[r];
      out_ts[o] = c.ts[r];
    }
  }
  return o;
}

// Line-aligned chunks of buf for P threads.
std::vector<const char*> line_chunks(const char* buf, long long len, int P) {
  std::vector<const char*> cut((size_t)P + 1);
  cut[0] = buf;
  cut[(size_t)P] = buf + len;
  for (int t = 1; t < P; ++t) {
    const char* c = buf + len * t / P;
    if (c < cut[(size_t)t - 1]) c = cut[(size_t)t - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(buf + len - c)));
    cut[(size_t)t] = nl ? nl + 1 : buf + len;
  }
  return cut;
}

// Calls fn(begin, end) for every non-empty line of [p, end) (end excludes the '\n' and a
// trailing '\r'), as RatingChunk::parse delimits them.
template <class Fn>
void for_each_line(const char* p, const char* end, Fn&& fn) {
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    const char* le = nl ? nl : end;
    const char* lend = le;
    if (lend > p && lend[-1] == '\r') --lend;
    if (lend > p) fn(p, lend);
    p = nl ? nl + 1 : end;
  }
}

// The timestamp of one rating line as parse_ratings reads it (default_ts when absent); false
// for a line parse_ratings would drop.
struct LineScratch {
  std::vector<std::string> toks;
  std::string field;
};

inline bool line_ts(const char* b, const char* e, long long default_ts, long long* ts,
                    LineScratch& sc) {
  std::vector<std::string>& toks = sc.toks;
  std::string& field = sc.field;
  std::string_view f[4];
  bool stable;
  double sv;
  *ts = default_ts;
  return parse_rating_fields(b, e, toks, field, f, &stable, &sv, ts);
}

template <class Fn>
void for_each_line_ts(const char* p, const char* end, long long default_ts, Fn&& fn) {
  LineScratch sc;
  for_each_line(p, end, [&](const char* b, const char* e) {
    long long v;
    if (line_ts(b, e, default_ts, &v, sc)) fn(b, e, v);
  });
}

int split_threads(long long len) {
  if (len < (1ll << 20)) return 1;
  return (int)std::max<long long>(1, std::min<long long>(len / (256ll << 10),
                                                         oryx_ff::native_threads()));
}

}  // namespace

extern "C" {

// Timestamp range of the rating lines of buf (the rows oryx_parse_ratings accepts; lines
// without a timestamp count as default_ts).  Returns the number of rows (0: no range).
long long oryx_ts_range(const char* buf, long long len, long long default_ts,
                        long long* out_min, long long* out_max) {
  const int P = split_threads(len);
  std::vector<const char*> cut = line_chunks(buf, len, P);
  std::vector<long long> mn((size_t)P, std::numeric_limits<long long>::max()),
      mx((size_t)P, std::numeric_limits<long long>::min()), cnt((size_t)P, 0);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long a = std::numeric_limits<long long>::max(), b = std::numeric_limits<long long>::min(), c = 0;
      for_each_line_ts(cut[(size_t)t], cut[(size_t)t + 1], default_ts,
                       [&](const char*, const char*, long long v) {
                         a = std::min(a, v);
                         b = std::max(b, v);
                         ++c;
                       });
      mn[(size_t)t] = a;
      mx[(size_t)t] = b;
      cnt[(size_t)t] = c;
    }
  });
  long long n = 0, a = std::numeric_limits<long long>::max(), b = std::numeric_limits<long long>::min();
  for (int t = 0; t < P; ++t) {
    n += cnt[(size_t)t];
    a = std::min(a, mn[(size_t)t]);
    b = std::max(b, mx[(size_t)t]);
  }
  *out_min = a;
  *out_max = b;
  return n;
}

// The time split of MLUpdate.splitNewDataToTrainTest for ALS (ALSUpdate.java:237-254) in one
// parallel pass: every parsable line of buf goes, in order and with its '\n', to out_lo when
// its timestamp (default_ts when missing) is < boundary, else to out_hi (lines that do not
// parse are dropped).  Both outputs need capacity len + 1.  Returns 0 (counts and byte sizes
// in the out parameters).
long long oryx_split_by_time(const char* buf, long long len, long long default_ts,
                             long long boundary, char* out_lo, char* out_hi, long long* n_lo,
                             long long* n_hi, long long* b_lo, long long* b_hi) {
  const auto T0 = std::chrono::steady_clock::now();
  const int P = split_threads(len);
  std::vector<const char*> cut = line_chunks(buf, len, P);
  // pass 1: each parsable line's side (1 byte per line) and the bytes per side per chunk
  // (raw arrays sized for the most lines a chunk can hold: a vector's push_back per line
  // cost 3x the parse -- its end pointer cannot stay in a register across byte stores)
  std::vector<std::unique_ptr<uint8_t[]>> side((size_t)P);
  std::vector<long long> blo((size_t)P, 0), bhi((size_t)P, 0), nlo((size_t)P, 0),
      nhi((size_t)P, 0);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      side[(size_t)t].reset(new uint8_t[(size_t)((cut[(size_t)t + 1] - cut[(size_t)t]) / 2 + 2)]);
      uint8_t* sd = side[(size_t)t].get();
      size_t r = 0;
      long long bl = 0, bh = 0, cl = 0, chh = 0;
      LineScratch sc;
      for_each_line(cut[(size_t)t], cut[(size_t)t + 1], [&](const char* b, const char* e) {
        long long v;
        const bool ok = line_ts(b, e, default_ts, &v, sc);
        const long long l = (long long)(e - b) + 1;
        const bool low = v < boundary;
        bl += ok && low ? l : 0;
        cl += ok && low;
        bh += ok && !low ? l : 0;
        chh += ok && !low;
        sd[r++] = ok ? (uint8_t)!low : (uint8_t)2;
      });
      blo[(size_t)t] = bl; bhi[(size_t)t] = bh; nlo[(size_t)t] = cl; nhi[(size_t)t] = chh;
    }
  });
  const auto T1 = std::chrono::steady_clock::now();
  std::vector<long long> olo((size_t)P + 1, 0), ohi((size_t)P + 1, 0);
  for (int t = 0; t < P; ++t) {
    olo[(size_t)t + 1] = olo[(size_t)t] + blo[(size_t)t];
    ohi[(size_t)t + 1] = ohi[(size_t)t] + bhi[(size_t)t];
  }
  // pass 2: copy runs of consecutive same-side lines
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      const uint8_t* sd = side[(size_t)t].get();
      char* wl = out_lo + olo[(size_t)t];
      char* wh = out_hi + ohi[(size_t)t];
      size_t r = 0;
      for_each_line(cut[(size_t)t], cut[(size_t)t + 1], [&](const char* b, const char* e) {
        const uint8_t k = sd[r++];
        if (k == 2) return;
        char*& w = k == 0 ? wl : wh;
        const size_t l = (size_t)(e - b);
        memcpy(w, b, l);
        w[l] = '\n';
        w += l + 1;
      });
    }
  });
  if (std::getenv("ORYX_LOG_DEBUG"))
    fprintf(stderr, "split P=%d pass1 %.3f ms pass2 %.3f ms\n", P,
            std::chrono::duration<double, std::milli>(T1 - T0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T1).count());
  long long a = 0, b = 0;
  for (int t = 0; t < P; ++t) { a += nlo[(size_t)t]; b += nhi[(size_t)t]; }
  *n_lo = a;
  *n_hi = b;
  *b_lo = olo[(size_t)P];
  *b_hi = ohi[(size_t)P];
  return 0;
}

// Parses newline-separated rating lines.  users/items: dictionaries; outputs per parsed row:
// user code, item code, strength (NaN when the field is empty = delete; 1 when missing),
// timestamp (default_ts when missing).  Returns rows parsed, or -(line number + 1) of the
// first malformed line when strict.  Large inputs are split at line boundaries over the
// native threads (per-chunk dictionaries merged in chunk order: the codes are the same as a
// sequential pass would give).
long long oryx_parse_ratings(const char* buf, long long len, void* users, void* items,
                             long long* out_u, long long* out_i, double* out_s,
                             long long* out_ts, long long max_rows, long long default_ts,
                             int strict) {
  if (!users || !items) {
    // no dictionaries: every parsed row's strength and timestamp, IDs not encoded (codes 0)
    return parse_rows_no_ids(buf, len, out_u, out_i, out_s, out_ts, max_rows, default_ts,
                             strict);
  }
  Dict* du = static_cast<Dict*>(users);
  Dict* di = static_cast<Dict*>(items);
  std::lock_guard<std::mutex> gu(du->mu);
  std::unique_lock<std::mutex> gi(di->mu, std::defer_lock);
  if (di != du) gi.lock();
  // chunk boundaries at newlines
  // several chunks from 1 MB on, at least 256 KB each (measured on 8 host cores: 100k lines,
  // 3 MB, 12.6 -> 8.6 ms; at 10k lines, 0.3 MB, thread start-up and the dictionary merge
  // cost more than they save: 1.1 ms on one thread, 1.7 ms on four)
  int P = 1;
  if (len >= (1ll << 20)) {
    const long long by_size = len / (256ll << 10);
    P = (int)std::min<long long>(by_size, oryx_ff::native_threads());
    if (P < 1) P = 1;
  }
  std::vector<const char*> cut((size_t)P + 1);
  cut[0] = buf;
  cut[(size_t)P] = buf + len;
  for (int t = 1; t < P; ++t) {
    const char* c = buf + len * t / P;
    if (c < cut[(size_t)t - 1]) c = cut[(size_t)t - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(buf + len - c)));
    cut[(size_t)t] = nl ? nl + 1 : buf + len;
  }
  std::vector<RatingChunk> ch((size_t)P);
  if (P == 1) {
    // a fresh dictionary (the speed layer's per-interval ones) is sized for the batch up front:
    // at most one new user and item per line (~24 bytes per line in practice; capped so an
    // 8 MB block of few distinct IDs does not allocate a table for 350k)
    const size_t est = std::min<size_t>((size_t)(len / 24) + 16, (size_t)1 << 17);
    if (du->keys.empty()) du->map.reserve(est);
    if (di != du && di->keys.empty()) di->map.reserve(est);
    ch[0].gu = du;
    ch[0].gi = di;
    const size_t rows_est = std::min<size_t>((size_t)max_rows, (size_t)(len / 4) + 1);
    ch[0].u.reserve(rows_est);
    ch[0].i.reserve(rows_est);
    ch[0].s.reserve(rows_est);
    ch[0].ts.reserve(rows_est);
    ch[0].parse(buf, buf + len, default_ts, strict != 0);
    const RatingChunk& c = ch[0];
    if (c.bad_line >= 0) return -(c.bad_line + 1);
    const long long n = (long long)c.u.size() < max_rows ? (long long)c.u.size() : max_rows;
    for (long long r = 0; r < n; ++r) {
      out_u[r] = c.u[(size_t)r];
      out_i[r] = c.i[(size_t)r];
      out_s[r] = c.s[(size_t)r];
      out_ts[r] = c.ts[(size_t)r];
    }
    return n;
  }
  // lines per chunk (an upper bound on its rows): when the output holds them all, every
  // chunk parses straight into the output at its first line's index
  std::vector<long long> lines_at((size_t)P + 1, 0);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      const char* b = cut[(size_t)t];
      const char* e = cut[(size_t)t + 1];
      lines_at[(size_t)t + 1] = (long long)std::count(b, e, '\n') + (e > b && e[-1] != '\n');
    }
  });
  for (int t = 0; t < P; ++t) lines_at[(size_t)t + 1] += lines_at[(size_t)t];
  if (lines_at[(size_t)P] <= max_rows)
    return parse_direct(du, di, ch, cut, lines_at, out_u, out_i, out_s, out_ts, default_ts,
                        strict);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t)
      ch[(size_t)t].parse(cut[(size_t)t], cut[(size_t)t + 1], default_ts, strict != 0);
  });
  // strict: the first malformed line in input order
  long long lines_before = 0;
  for (int t = 0; t < P; ++t) {
    if (ch[(size_t)t].bad_line >= 0) return -(lines_before + ch[(size_t)t].bad_line + 1);
    lines_before += ch[(size_t)t].lines;
  }
  // merge the chunk dictionaries in order (first appearances, numeric and string keys
  // interleaved as met), then write the rows at their offsets
  std::vector<std::vector<int64_t>> umap((size_t)P), imap((size_t)P);
  std::vector<long long> off((size_t)P + 1, 0);
  auto merge = [](Dict* d, const RatingChunk::Side& sd, std::vector<int64_t>& to_global) {
    to_global.reserve(sd.keys.size());
    for (int64_t e : sd.order) {
      if (e < 0) d->encode_num((uint32_t)(-e - 1));
      else to_global.push_back(d->encode(sd.keys[(size_t)e]));
    }
  };
  for (int t = 0; t < P; ++t) {
    RatingChunk& c = ch[(size_t)t];
    merge(du, c.us, umap[(size_t)t]);
    merge(di, c.is, imap[(size_t)t]);
    off[(size_t)t + 1] = off[(size_t)t] + (long long)c.u.size();
  }
  const long long total = off[(size_t)P] < max_rows ? off[(size_t)P] : max_rows;
  const int32_t* unum = du->num.data();
  const int32_t* inum = di->num.data();
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      const RatingChunk& c = ch[(size_t)t];
      const long long o = off[(size_t)t];
      const long long n = (long long)c.u.size();
      const int64_t* um = umap[(size_t)t].data();
      const int64_t* im = imap[(size_t)t].data();
      for (long long r = 0; r < n && o + r < total; ++r) {
        const int32_t a = c.u[(size_t)r], b = c.i[(size_t)r];
        out_u[o + r] = a < 0 ? unum[-(a + 1)] : um[a];
        out_i[o + r] = b < 0 ? inum[-(b + 1)] : im[b];
        out_s[o + r] = c.s[(size_t)r];
        out_ts[o + r] = c.ts[(size_t)r];
      }
    }
  });
  return total;
}

// ---- id -> row maps mirroring a Python feature store (the speed layer's ID lookups) ----

// Open addressing with linear probing and tombstones: a slot holds the 64-bit hash, the key
// (inline up to 16 bytes, else an index into owned storage) and the row, so a lookup of a
// short ID touches one cache line (std::unordered_map<std::string> took a bucket, a node and
// the key's heap copy: ~370 ns per ID of a 10k-event micro-batch against a 162k-row store).
struct RowMap {
  struct Slot {
    uint64_t h = 0;
    uint32_t len = 0;
    int32_t state = -1;     // -1 empty, -2 deleted, 0 live
    int64_t row = 0;
    union {
      char in[16];
      int64_t big;          // index into longs
    };
    Slot() : in{} {}
  };
  std::vector<Slot> slots = std::vector<Slot>(1024);
  std::vector<std::string> longs;
  size_t live = 0, used = 0;   // used: live + deleted slots

  static uint64_t mix(uint64_t a, uint64_t b) {
    const unsigned __int128 r = (unsigned __int128)a * b;
    return (uint64_t)r ^ (uint64_t)(r >> 64);
  }
  static uint64_t hash(const char* p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    while (n >= 8) {
      uint64_t v;
      std::memcpy(&v, p, 8);
      h = mix(h ^ v, 0xA0761D6478BD642Full);
      p += 8;
      n -= 8;
    }
    uint64_t v = 0;
    std::memcpy(&v, p, n);
    return mix(h ^ v, 0xE7037ED1A0B428DBull);
  }
  const char* key_of(const Slot& sl) const {
    return sl.len <= 16 ? sl.in : longs[(size_t)sl.big].data();
  }
  bool same(const Slot& sl, uint64_t h, const char* k, size_t n) const {
    return sl.state == 0 && sl.h == h && sl.len == n && std::memcmp(key_of(sl), k, n) == 0;
  }
  // slot of key k, or -1
  int64_t find(const char* k, size_t n, uint64_t h) const {
    const size_t m = slots.size() - 1;
    for (size_t j = (size_t)h & m;; j = (j + 1) & m) {
      const Slot& sl = slots[j];
      if (sl.state == -1) return -1;
      if (same(sl, h, k, n)) return (int64_t)j;
    }
  }
  void rehash(size_t cap) {
    std::vector<Slot> old;
    old.swap(slots);
    slots.assign(cap, Slot());
    used = 0;
    std::vector<std::string> kept;   // live long keys only
    const size_t m = cap - 1;
    for (const Slot& sl : old) {
      if (sl.state != 0) continue;
      size_t j = (size_t)sl.h & m;
      while (slots[j].state != -1) j = (j + 1) & m;
      slots[j] = sl;
      if (sl.len > 16) {
        slots[j].big = (int64_t)kept.size();
        kept.push_back(std::move(longs[(size_t)sl.big]));
      }
      ++used;
    }
    longs.swap(kept);
  }
  void set(const char* k, size_t n, int64_t row) {
    const uint64_t h = hash(k, n);
    const int64_t f = find(k, n, h);
    if (f >= 0) {
      slots[(size_t)f].row = row;
      return;
    }
    if ((used + 1) * 2 > slots.size()) {
      size_t cap = 1024;
      while (cap < (live + 1) * 4) cap *= 2;
      rehash(cap);
    }
    const size_t m = slots.size() - 1;
    size_t j = (size_t)h & m;
    while (slots[j].state == 0) j = (j + 1) & m;
    Slot& sl = slots[j];
    if (sl.state == -1) ++used;
    sl.h = h;
    sl.len = (uint32_t)n;
    sl.state = 0;
    sl.row = row;
    if (n <= 16) {
      std::memcpy(sl.in, k, n);
    } else {
      sl.big = (int64_t)longs.size();
      longs.emplace_back(k, n);
    }
    ++live;
  }
  void remove(const char* k, size_t n) {
    const int64_t f = find(k, n, hash(k, n));
    if (f < 0) return;
    slots[(size_t)f].state = -2;    // a long key's storage is reclaimed at the next rehash
    --live;
    if (live == 0) {
      slots.assign(1024, Slot());
      longs.clear();
      used = 0;
    }
  }
  int64_t row_of(const char* k, size_t n, uint64_t h) const {
    const int64_t f = find(k, n, h);
    return f < 0 ? -1 : slots[(size_t)f].row;
  }
  void prefetch(uint64_t h) const { __builtin_prefetch(&slots[(size_t)h & (slots.size() - 1)]); }
};

void* oryx_rowmap_new() { return new RowMap(); }
void oryx_rowmap_free(void* h) { delete static_cast<RowMap*>(h); }
long long oryx_rowmap_size(void* h) { return (long long)static_cast<RowMap*>(h)->live; }

// n ids back to back in blob (ends = end offsets) -> rows (set / overwrite).
void oryx_rowmap_set(void* h, const char* blob, const long long* ends, const long long* rows,
                     long long n) {
  RowMap* m = static_cast<RowMap*>(h);
  long long b = 0;
  for (long long j = 0; j < n; ++j) {
    m->set(blob + b, (size_t)(ends[j] - b), rows[j]);
    b = ends[j];
  }
}

void oryx_rowmap_remove(void* h, const char* blob, const long long* ends, long long n) {
  RowMap* m = static_cast<RowMap*>(h);
  long long b = 0;
  for (long long j = 0; j < n; ++j) {
    m->remove(blob + b, (size_t)(ends[j] - b));
    b = ends[j];
  }
}

// out[c] = row of dictionary key c (-1 when absent) for every code of the dictionary.
// The numeric suffix (trailing decimal digits, at most 18) of every live key, written at its
// row of out [n_rows] (rows without a key or without digits: -1).  For rescorers that select
// items by ID pattern: one pass over the map instead of a Python loop over every ID.
long long oryx_rowmap_key_suffixes(void* h, long long* out, long long n_rows) {
  const RowMap* m = static_cast<const RowMap*>(h);
  for (long long r = 0; r < n_rows; ++r) out[r] = -1;
  long long hit = 0;
  for (const auto& sl : m->slots) {
    if (sl.state != 0 || sl.row < 0 || sl.row >= n_rows) continue;
    const char* k = m->key_of(sl);
    size_t e = sl.len, b = e;
    while (b > 0 && e - b < 18 && (unsigned)(k[b - 1] - '0') < 10u) --b;
    if (b == e) continue;
    long long v = 0;
    for (size_t q = b; q < e; ++q) v = v * 10 + (k[q] - '0');
    out[sl.row] = v;
    ++hit;
  }
  return hit;
}

long long oryx_rowmap_translate(void* h, void* dh, long long* out) {
  const RowMap* m = static_cast<RowMap*>(h);
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  const long long n = (long long)d->keys.size();
  // a store of 1e5+ rows is a table of several MB: every probe is a cache miss, so hashes are
  // computed D keys ahead and their slots prefetched (~10 misses in flight instead of one),
  // and batches past 4k keys are split over the native threads
  oryx_ff::parallel_ranges(n, 4096, [&](long long lo, long long hi, int) {
    constexpr int D = 16;
    uint64_t hs[D];
    for (long long c = lo; c < hi && c < lo + D; ++c) {
      const std::string& k = d->keys[(size_t)c];
      hs[(c - lo) % D] = RowMap::hash(k.data(), k.size());
      m->prefetch(hs[(c - lo) % D]);
    }
    for (long long c = lo; c < hi; ++c) {
      const int q = (int)((c - lo) % D);
      const uint64_t h = hs[q];
      if (c + D < hi) {
        const std::string& kn = d->keys[(size_t)(c + D)];
        hs[q] = RowMap::hash(kn.data(), kn.size());
        m->prefetch(hs[q]);
      }
      const std::string& k = d->keys[(size_t)c];
      out[c] = m->row_of(k.data(), k.size(), h);
    }
  });
  return n;
}

// Plain CSV block -> a dense row-major double matrix (the classification / regression
// examples of the RDF and k-means speed layers and batch inputs): F fields per line, numeric
// columns (is_num[f] != 0) parsed with the exact fast-path double parser (empty -> NaN), the
// other columns returned as (offset, length) spans into buf for the caller's category maps.
// Lines are split over the native threads (newline counts first, then every chunk parses
// straight into its rows).  Returns the row count, or -(line + 1) of the first line that is
// not plain CSV with F fields (a quote, a backslash or a leading '[' included) or has an
// unparseable numeric field (the caller then takes the general path).
}  // extern "C"

namespace {

// A plain decimal field at p ("[-+]digits[.digits][e[-+]digits]", at most 19 significant
// digits, a value exactly representable by the one-rounding product D * 10^e) ending at ','
// or lend: the value and the field's end; nullptr when the field needs the general parser
// (oryx_ff::parse_double) -- more digits, exponents beyond 10^22, other characters.  Found
// in the same pass that parses it: no per-field memchr.
inline const char* fast_decimal_field(const char* p, const char* lend, double& out) {
  static const double kP10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  const char* q = p;
  bool neg = false;
  if (q < lend && (*q == '-' || *q == '+')) neg = *q++ == '-';
  uint64_t D = 0;
  int nd = 0, frac = 0;
  while (q < lend && (unsigned)(*q - '0') < 10u) {
    D = D * 10 + (uint64_t)(*q++ - '0');
    ++nd;
  }
  if (q < lend && *q == '.') {
    ++q;
    while (q < lend && (unsigned)(*q - '0') < 10u) {
      D = D * 10 + (uint64_t)(*q++ - '0');
      ++nd;
      ++frac;
    }
  }
  if (nd == 0 || nd > 19) return nullptr;
  int e10 = -frac;
  if (q < lend && (*q == 'e' || *q == 'E')) {
    ++q;
    bool eneg = false;
    if (q < lend && (*q == '-' || *q == '+')) eneg = *q++ == '-';
    int x = 0, ne = 0;
    while (q < lend && (unsigned)(*q - '0') < 10u && ne < 4) {
      x = x * 10 + (*q++ - '0');
      ++ne;
    }
    if (!ne) return nullptr;
    e10 += eneg ? -x : x;
  }
  if (q < lend && *q != ',') return nullptr;
  if (D > (1ull << 53) || e10 < -22 || e10 > 22) return nullptr;
  const double v = e10 < 0 ? (double)D / kP10[-e10] : (double)D * kP10[e10];
  out = neg ? -v : v;
  return q;
}

}  // namespace

extern "C" {

long long oryx_csv_numeric_block(const char* buf, long long len, int F,
                                 const unsigned char* is_num, double* out, long long* span_off,
                                 int* span_len, long long max_rows) {
  // threads for blocks past 256 KB (a 10k-event speed-layer batch is ~1 MB)
  long long np_ = len >> 18;
  if (np_ > oryx_ff::native_threads()) np_ = oryx_ff::native_threads();
  const int P = np_ > 1 ? (int)np_ : 1;
  std::vector<const char*> cut((size_t)P + 1);
  cut[0] = buf;
  cut[(size_t)P] = buf + len;
  for (int t = 1; t < P; ++t) {
    const char* c = buf + len * t / P;
    if (c < cut[(size_t)t - 1]) c = cut[(size_t)t - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(buf + len - c)));
    cut[(size_t)t] = nl ? nl + 1 : buf + len;
  }
  // rows per chunk (non-empty lines)
  std::vector<long long> rows((size_t)P + 1, 0), bad((size_t)P, -1), lines((size_t)P, 0);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long r = 0, l = 0;
      for (const char* p = cut[(size_t)t]; p < cut[(size_t)t + 1];) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(cut[(size_t)t + 1] - p)));
        const char* le = nl ? nl : cut[(size_t)t + 1];
        if (le > p && !(le - p == 1 && *p == '\r')) ++r;
        ++l;
        p = nl ? nl + 1 : cut[(size_t)t + 1];
      }
      rows[(size_t)t + 1] = r;
      lines[(size_t)t] = l;
    }
  });
  for (int t = 0; t < P; ++t) rows[(size_t)t + 1] += rows[(size_t)t];
  if (rows[(size_t)P] > max_rows) return -1;
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long row = rows[(size_t)t], line = 0;
      for (const char* p = cut[(size_t)t]; p < cut[(size_t)t + 1];) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(cut[(size_t)t + 1] - p)));
        const char* le = nl ? nl : cut[(size_t)t + 1];
        const char* lend = le;
        if (lend > p && lend[-1] == '\r') --lend;
        if (lend > p) {
          double* o = out + row * F;
          const char* q = p;
          int f = 0;
          // JSON-array lines and backslash escapes belong to the general parser
          bool ok = *p != '[' && !memchr(p, '\\', (size_t)(lend - p)) &&
                    !memchr(p, '"', (size_t)(lend - p));
          while (ok) {
            if (f < F && is_num[f]) {
              const char* fe = fast_decimal_field(q, lend, o[f]);
              if (fe) {
                ++f;
                if (fe >= lend) break;
                q = fe + 1;
                continue;
              }
            }
            const char* c = static_cast<const char*>(memchr(q, ',', (size_t)(lend - q)));
            const char* fe = c ? c : lend;
            if (f >= F) { ok = false; break; }
            if (is_num[f]) {
              if (fe == q) o[f] = std::numeric_limits<double>::quiet_NaN();
              else if (!oryx_ff::parse_double(q, fe, o[f])) ok = false;
            } else {
              o[f] = std::numeric_limits<double>::quiet_NaN();
              span_off[row * F + f] = q - buf;
              span_len[row * F + f] = (int)(fe - q);
            }
            ++f;
            if (!c) break;
            q = c + 1;
          }
          if (!ok || f != F) {
            bad[(size_t)t] = line;
            return;
          }
          ++row;
        }
        ++line;
        p = nl ? nl + 1 : cut[(size_t)t + 1];
      }
    }
  });
  long long before = 0;
  for (int t = 0; t < P; ++t) {
    if (bad[(size_t)t] >= 0) return -(before + bad[(size_t)t] + 1);
    before += lines[(size_t)t];
  }
  return rows[(size_t)P];
}

// Numeric CSV rows straight to a float32 matrix (the k-means / RDF batch layers' parse of
// millions of feature rows): every non-empty line of buf has exactly F comma-separated fields;
// field f goes to column out_col[f] of out ([rows][P], out_col -1: skipped).  Numeric fields
// (is_num[f]) are parsed exactly to double and rounded to float32 (as float(x) -> np.float32);
// an empty numeric field is NaN.  Fields that are not numeric are recorded as spans
// (span_off/span_len [rows][S], S = number of such fields, in field order; nullable when S =
// 0).  Lines with quotes, backslash escapes or JSON arrays, or a field count other than F,
// stop the parse: returns -(line + 1) of the first such line, else the number of rows (-2 when
// more than max_rows).  Threads over line-aligned chunks.
}  // extern "C"

namespace {

template <typename T>
long long csv_to_matrix(const char* buf, long long len, int F, const unsigned char* is_num,
                        const int* out_col, int P, T* out, long long* span_off, int* span_len,
                        long long max_rows) {
  int S = 0;
  std::vector<int> span_idx((size_t)F, -1);
  for (int f = 0; f < F; ++f)
    if (!is_num[f]) span_idx[(size_t)f] = S++;
  const int P_ = split_threads(len);
  std::vector<const char*> cut = line_chunks(buf, len, P_);
  std::vector<long long> rows((size_t)P_ + 1, 0), bad((size_t)P_, -1), lines((size_t)P_, 0);
  oryx_ff::parallel_ranges(P_, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long r = 0, l = 0;
      for (const char* p = cut[(size_t)t]; p < cut[(size_t)t + 1];) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(cut[(size_t)t + 1] - p)));
        const char* le = nl ? nl : cut[(size_t)t + 1];
        if (le > p && !(le - p == 1 && *p == '\r')) ++r;
        ++l;
        p = nl ? nl + 1 : cut[(size_t)t + 1];
      }
      rows[(size_t)t + 1] = r;
      lines[(size_t)t] = l;
    }
  });
  for (int t = 0; t < P_; ++t) rows[(size_t)t + 1] += rows[(size_t)t];
  if (rows[(size_t)P_] > max_rows) return -2;
  oryx_ff::parallel_ranges(P_, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long row = rows[(size_t)t], line = 0;
      for (const char* p = cut[(size_t)t]; p < cut[(size_t)t + 1];) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(cut[(size_t)t + 1] - p)));
        const char* le = nl ? nl : cut[(size_t)t + 1];
        const char* lend = le;
        if (lend > p && lend[-1] == '\r') --lend;
        if (lend > p) {
          T* o = out + row * P;
          const char* q = p;
          int f = 0;
          bool ok = *p != '[' && !memchr(p, '\\', (size_t)(lend - p)) &&
                    !memchr(p, '"', (size_t)(lend - p));
          while (ok) {
            if (f < F && is_num[f]) {
              double v;
              const char* fe = fast_decimal_field(q, lend, v);
              if (fe) {
                if (out_col[f] >= 0) o[out_col[f]] = (T)v;
                ++f;
                if (fe >= lend) break;
                q = fe + 1;
                continue;
              }
            }
            const char* c = static_cast<const char*>(memchr(q, ',', (size_t)(lend - q)));
            const char* fe = c ? c : lend;
            if (f >= F) { ok = false; break; }
            if (is_num[f]) {
              double v;
              if (fe == q) v = std::numeric_limits<double>::quiet_NaN();
              else if (!oryx_ff::parse_double(q, fe, v)) { ok = false; break; }
              if (out_col[f] >= 0) o[out_col[f]] = (T)v;
            } else {
              const int si = span_idx[(size_t)f];
              span_off[row * S + si] = q - buf;
              span_len[row * S + si] = (int)(fe - q);
              if (out_col[f] >= 0) o[out_col[f]] = std::numeric_limits<T>::quiet_NaN();
            }
            ++f;
            if (!c) break;
            q = c + 1;
          }
          if (!ok || f != F) {
            bad[(size_t)t] = line;
            return;
          }
          ++row;
        }
        ++line;
        p = nl ? nl + 1 : cut[(size_t)t + 1];
      }
    }
  });
  long long before = 0;
  for (int t = 0; t < P_; ++t) {
    if (bad[(size_t)t] >= 0) return -(before + bad[(size_t)t] + 1);
    before += lines[(size_t)t];
  }
  return rows[(size_t)P_];
}

}  // namespace

extern "C" {

long long oryx_csv_to_f32(const char* buf, long long len, int F, const unsigned char* is_num,
                          const int* out_col, int P, float* out, long long* span_off,
                          int* span_len, long long max_rows) {
  return csv_to_matrix<float>(buf, len, F, is_num, out_col, P, out, span_off, span_len,
                              max_rows);
}

long long oryx_csv_to_f64(const char* buf, long long len, int F, const unsigned char* is_num,
                          const int* out_col, int P, double* out, long long* span_off,
                          int* span_len, long long max_rows) {
  return csv_to_matrix<double>(buf, len, F, is_num, out_col, P, out, span_off, span_len,
                               max_rows);
}

// Formats rows of a float matrix as JSON arrays "[v0,v1,...]" with shortest round-trip
// float32 text (fastfloat.h), back to back in out; row_ends[r] = end offset of row r.  Rows are
// split over the native threads (each formats its range into its own buffer, then the parts
// are copied in order).  Returns bytes used or -1 when out is too small.
long long oryx_format_float_rows(const float* mat, long long n, int k, long long stride,
                                 char* out, long long cap, long long* row_ends) {
  const int T = oryx_ff::native_threads();
  std::vector<std::string> part((size_t)T);
  std::vector<long long> lo_of((size_t)T + 1, n);
  const int P = oryx_ff::parallel_ranges(n, 512, [&](long long lo, long long hi, int t) {
    lo_of[(size_t)t] = lo;
    std::string& o = part[(size_t)t];
    o.resize((size_t)(hi - lo) * (size_t)(2 + 18 * (long long)k));
    char* w = &o[0];
    for (long long r = lo; r < hi; ++r) {
      const float* row = mat + r * stride;
      *w++ = '[';
      for (int j = 0; j < k; ++j) {
        if (j) *w++ = ',';
        w = oryx_ff::write_float_json(row[j], w);
      }
      *w++ = ']';
      row_ends[r] = w - o.data();   // local end; rebased below
    }
    o.resize((size_t)(w - o.data()));
  });
  long long pos = 0;
  for (int t = 0; t < P; ++t) {
    const long long lo = lo_of[(size_t)t], hi = t + 1 < P ? lo_of[(size_t)t + 1] : n;
    const std::string& o = part[(size_t)t];
    if (pos + (long long)o.size() > cap) return -1;
    std::memcpy(out + pos, o.data(), o.size());
    for (long long r = lo; r < hi; ++r) row_ends[r] += pos;
    pos += (long long)o.size();
  }
  return pos;
}

// All keys from `from` on, back to back in out; ends[j] = end offset of key from + j.
// Returns bytes used, or -(bytes needed) when out is too small.
// Keys from .. to - 1 (clamped to the size) back to back into out, their end offsets into
// ends (to - from entries at most: a dictionary growing concurrently never writes past it).
long long oryx_dict_keys_blob(void* dh, long long from, long long to, char* out, long long cap,
                              long long* ends) {
  auto* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  const size_t end = std::min((size_t)std::max(to, 0LL), d->keys.size());
  long long need = 0;
  for (size_t c = (size_t)from; c < end; ++c) need += (long long)d->keys[c].size();
  if (need > cap) return -need;
  long long pos = 0;
  for (size_t c = (size_t)from; c < end; ++c) {
    memcpy(out + pos, d->keys[c].data(), d->keys[c].size());
    pos += (long long)d->keys[c].size();
    ends[c - from] = pos;
  }
  return pos;
}

}  // extern "C"

namespace {

// JSON string literal of UTF-8 text with Python json.dumps' default escaping (ensure_ascii:
// non-ASCII as \uXXXX, astral planes as surrogate pairs).
void json_quote(const char* s, size_t len, std::string& o) {
  static const char* hex = "0123456789abcdef";
  auto u4 = [&](unsigned v) {
    o += "\\u";
    o += hex[(v >> 12) & 15]; o += hex[(v >> 8) & 15]; o += hex[(v >> 4) & 15]; o += hex[v & 15];
  };
  o += '"';
  for (size_t p = 0; p < len;) {
    unsigned char c = (unsigned char)s[p];
    if (c < 0x80) {
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        default:
          if (c < 0x20) u4(c); else o += (char)c;
      }
      ++p;
      continue;
    }
    unsigned cp = 0;
    int extra = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : 1;
    cp = c & (0x3F >> extra);
    for (int q = 1; q <= extra && p + q < len; ++q) cp = (cp << 6) | (s[p + q] & 0x3F);
    p += 1 + extra;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u4(0xD800 + (cp >> 10));
      u4(0xDC00 + (cp & 0x3FF));
    } else {
      u4(cp);
    }
  }
  o += '"';
}

void json_quote(const std::string& s, std::string& o) { json_quote(s.data(), s.size(), o); }

void float_row(const float* row, int k, std::string& o) {
  const size_t at = o.size();
  o.resize(at + 2 + 18 * (size_t)k);
  char* w = &o[at];
  *w++ = '[';
  for (int j = 0; j < k; ++j) {
    if (j) *w++ = ',';
    w = oryx_ff::write_float_json(row[j], w);
  }
  *w++ = ']';
  o.resize((size_t)(w - o.data()));
}

}  // namespace

extern "C" {

// ---- bulk parsing of ALS model-update messages (the serving / speed model load) ----

struct JsonCursor {
  const char* p;
  const char* end;
  void ws() { while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
  bool eat(char c) { ws(); if (p < end && *p == c) { ++p; return true; } return false; }
  // a JSON string (escapes decoded to UTF-8) or a bare number / literal as text
  bool token(std::string& out) {
    ws();
    out.clear();
    if (p >= end) return false;
    if (*p != '"') {
      const char* b = p;
      while (p < end && *p != ',' && *p != ']' && *p != ' ') ++p;
      out.assign(b, p - b);
      return p > b;
    }
    ++p;
    while (p < end && *p != '"') {
      char c = *p++;
      if (c != '\\') { out += c; continue; }
      if (p >= end) return false;
      char e = *p++;
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          auto hex4 = [&](unsigned& v) {
            if (end - p < 4) return false;
            v = 0;
            for (int q = 0; q < 4; ++q) {
              char h = p[q];
              v <<= 4;
              if (h >= '0' && h <= '9') v |= h - '0';
              else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
              else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
              else return false;
            }
            p += 4;
            return true;
          };
          unsigned cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            unsigned lo;
            if (!hex4(lo)) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (cp < 0x80) out += (char)cp;
          else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 63)); }
          else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 63));
            out += (char)(0x80 | (cp & 63));
          } else {
            out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 63));
            out += (char)(0x80 | ((cp >> 6) & 63)); out += (char)(0x80 | (cp & 63));
          }
          break;
        }
        default: return false;
      }
    }
    if (p >= end) return false;
    ++p;
    return true;
  }
};

}  // extern "C"

namespace {
thread_local std::string g_up_ids, g_up_known;

// One ["X"|"Y", id, [k floats], optional [ids...]] message: returns 0 (X) / 1 (Y) / 2 (not
// parseable: nothing appended).  The id text is appended to ids, known ids ('\0'-terminated)
// to known; cnt = number of known ids, -1 when the list is absent.
int parse_one_up(const char* b, const char* e, int k, float* v, std::string& ids,
                 std::string& known, long long& cnt, std::string& tok) {
  JsonCursor c{b, e};
  cnt = -1;
  const size_t id_mark = ids.size(), known_mark = known.size();
  bool ok = c.eat('[') && c.token(tok) && (tok == "X" || tok == "Y");
  const int kind = ok && tok == "Y" ? 1 : 0;
  ok = ok && c.eat(',') && c.token(tok);
  if (ok) ids += tok;
  ok = ok && c.eat(',') && c.eat('[');
  for (int f = 0; ok && f < k; ++f) {
    if (f && !c.eat(',')) { ok = false; break; }
    c.ws();
    const char* fb = c.p;
    {
      // one pass over a plain number followed by its delimiter
      const char* stop;
      if (oryx_ff::parse_float_prefix(fb, c.end, v[f], &stop) && stop > fb && stop < c.end &&
          (*stop == ',' || *stop == ']' || *stop == ' ')) {
        c.p = stop;
        continue;
      }
    }
    while (c.p < c.end && *c.p != ',' && *c.p != ']' && *c.p != ' ') ++c.p;
    if (!oryx_ff::parse_float(fb, c.p, v[f])) {
      const std::string_view t(fb, (size_t)(c.p - fb));   // NaN / Infinity spellings
      if (t == "NaN") v[f] = std::numeric_limits<float>::quiet_NaN();
      else if (t == "Infinity") v[f] = std::numeric_limits<float>::infinity();
      else if (t == "-Infinity") v[f] = -std::numeric_limits<float>::infinity();
      else ok = false;
    }
  }
  ok = ok && c.eat(']');
  if (ok && c.eat(',')) {
    cnt = 0;
    ok = c.eat('[');
    if (ok && !c.eat(']')) {
      do {
        if (!c.token(tok)) { ok = false; break; }
        known += tok;
        known += '\0';
        ++cnt;
      } while (c.eat(','));
      ok = ok && c.eat(']');
    }
  }
  ok = ok && c.eat(']');
  if (!ok) {
    ids.resize(id_mark);
    known.resize(known_mark);
    cnt = -1;
    return 2;
  }
  return kind;
}

// Parses messages [begin[j], end[j]) for j < n over the native threads into the thread-local
// texts of the calling thread (id_ends are global offsets into them).  With stop_at_bad, the
// result is cut before the first unparseable message; returns the number of messages kept.
long long parse_up_spans(const char* buf, const long long* begin, const long long* end,
                         long long n, int k, unsigned char* kinds, float* vecs,
                         long long* id_ends, long long* known_cnt, bool stop_at_bad) {
  g_up_ids.clear();
  g_up_known.clear();
  const int T = oryx_ff::native_threads();
  std::vector<std::string> ids((size_t)T), known((size_t)T);
  std::vector<long long> lo_of((size_t)T + 1, n);
  const int P = oryx_ff::parallel_ranges(n, 128, [&](long long lo, long long hi, int t) {
    lo_of[(size_t)t] = lo;
    std::string tok;
    std::string& id = ids[(size_t)t];
    std::string& kn = known[(size_t)t];
    for (long long j = lo; j < hi; ++j) {
      kinds[j] = (unsigned char)parse_one_up(buf + begin[j], buf + end[j], k, vecs + j * k, id,
                                             kn, known_cnt[j], tok);
      id_ends[j] = (long long)id.size();   // local; rebased below
    }
  });
  long long keep = n;
  if (stop_at_bad)
    for (long long j = 0; j < n; ++j)
      if (kinds[j] == 2) { keep = j; break; }
  size_t id_total = 0, kn_total = 0;
  for (int t = 0; t < P; ++t) { id_total += ids[(size_t)t].size(); kn_total += known[(size_t)t].size(); }
  g_up_ids.reserve(id_total);
  g_up_known.reserve(kn_total);
  for (int t = 0; t < P; ++t) {
    const long long lo = lo_of[(size_t)t], hi = t + 1 < P ? lo_of[(size_t)t + 1] : n;
    const long long base = (long long)g_up_ids.size();
    for (long long j = lo; j < hi; ++j) id_ends[j] += base;
    g_up_ids += ids[(size_t)t];
    g_up_known += known[(size_t)t];
  }
  if (keep < n) {
    // drop what follows the first bad message from the texts
    g_up_ids.resize(keep ? (size_t)id_ends[keep - 1] : 0);
    size_t kb = 0;
    for (long long j = 0; j < keep; ++j)
      if (known_cnt[j] > 0) {
        for (long long q = 0; q < known_cnt[j]; ++q) kb = g_up_known.find('\0', kb) + 1;
      }
    g_up_known.resize(kb);
  }
  return keep;
}
}  // namespace

extern "C" {

// Parses n messages (back to back in buf, ends = message end offsets).  kinds[j] = 0 (X) /
// 1 (Y) / 2 (unparseable: the caller falls back); vecs [n][k]; id_ends[j] indexes the id
// texts, known_cnt[j] = number of known ids (-1: no list); the texts are fetched with
// oryx_up_texts (ids back to back, then known items '\0'-terminated).  Returns the total
// number of known items.
long long oryx_parse_up_batch(const char* buf, const long long* ends, long long n, int k,
                              unsigned char* kinds, float* vecs, long long* id_ends,
                              long long* known_cnt) {
  std::vector<long long> begin((size_t)n);
  for (long long j = 0; j < n; ++j) begin[(size_t)j] = j ? ends[j - 1] : 0;
  parse_up_spans(buf, begin.data(), ends, n, k, kinds, vecs, id_ends, known_cnt, false);
  long long total = 0;
  for (long long j = 0; j < n; ++j) if (known_cnt[j] > 0) total += known_cnt[j];
  return total;
}

// The leading run of "UP" records of a raw poll buffer (oryx_reader_poll layout: per record
// i64 offset, i64 timestamp, i32 key length (-1: none), i32 value length, key, value), parsed
// as oryx_parse_up_batch does, stopping before the first record that is not a parseable UP.
// At most max_n records; *consumed_bytes = buffer offset after the run.  Returns the run
// length (0 when the first record is not one).
long long oryx_parse_up_records(const char* raw, long long used, long long nrec, int k,
                                long long max_n, unsigned char* kinds, float* vecs,
                                long long* id_ends, long long* known_cnt,
                                long long* consumed_bytes) {
  std::vector<long long> begin, end, after;
  long long pos = 0;
  for (long long r = 0; r < nrec && r < max_n; ++r) {
    if (pos + 24 > used) break;
    int32_t kl, vl;
    std::memcpy(&kl, raw + pos + 16, 4);
    std::memcpy(&vl, raw + pos + 20, 4);
    const long long kpos = pos + 24;
    if (kl != 2 || raw[kpos] != 'U' || raw[kpos + 1] != 'P') break;
    begin.push_back(kpos + 2);
    end.push_back(kpos + 2 + vl);
    pos = kpos + 2 + vl;
    after.push_back(pos);
  }
  const long long n = (long long)begin.size();
  const long long keep = n ? parse_up_spans(raw, begin.data(), end.data(), n, k, kinds, vecs,
                                            id_ends, known_cnt, true) : 0;
  *consumed_bytes = keep ? after[(size_t)keep - 1] : 0;
  return keep;
}

// As oryx_parse_up_records over a buffer of log frames (oryx_reader_poll_frames layout: per
// frame u32 magic, u32 crc, u64 offset, i64 ts, u32 key length (0xFFFFFFFF: none), u32 value
// length, key, value).
long long oryx_parse_up_frames(const char* raw, long long used, long long nrec, int k,
                               long long max_n, unsigned char* kinds, float* vecs,
                               long long* id_ends, long long* known_cnt,
                               long long* consumed_bytes) {
  std::vector<long long> begin, end, after;
  long long pos = 0;
  for (long long r = 0; r < nrec && r < max_n; ++r) {
    if (pos + 32 > used) break;
    uint32_t kl, vl;
    std::memcpy(&kl, raw + pos + 24, 4);
    std::memcpy(&vl, raw + pos + 28, 4);
    const long long kpos = pos + 32;
    if (kl != 2 || raw[kpos] != 'U' || raw[kpos + 1] != 'P') break;
    begin.push_back(kpos + 2);
    end.push_back(kpos + 2 + vl);
    pos = kpos + 2 + vl;
    after.push_back(pos);
  }
  const long long n = (long long)begin.size();
  const long long keep = n ? parse_up_spans(raw, begin.data(), end.data(), n, k, kinds, vecs,
                                            id_ends, known_cnt, true) : 0;
  *consumed_bytes = keep ? after[(size_t)keep - 1] : 0;
  return keep;
}

// Factor part-file lines ([id,[k floats]] per line, the X/ Y/ text parts written by
// write_features / the reference's saveFeaturesRDD) -> vecs [n][k] and the id texts (fetched
// with oryx_up_texts, as after oryx_parse_up_batch).  Lines are split over the native threads.
// Empty lines are skipped.  Returns the number of rows, or -(line + 1) of the first line that
// does not parse (the caller then takes the general path); at most max_n rows.
long long oryx_parse_feature_lines(const char* buf, long long len, int k, long long max_n,
                                   float* vecs, long long* id_ends) {
  g_up_ids.clear();
  g_up_known.clear();
  std::vector<long long> begin, end;
  for (const char* p = buf; p < buf + len;) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(buf + len - p)));
    const char* le = nl ? nl : buf + len;
    const char* b = p;
    while (b < le && (*b == ' ' || *b == '\r')) ++b;
    if (b < le) {
      if ((long long)begin.size() >= max_n) return -((long long)begin.size() + 1);
      begin.push_back(p - buf);
      end.push_back(le - buf);
    }
    p = nl ? nl + 1 : buf + len;
  }
  const long long n = (long long)begin.size();
  const int T = oryx_ff::native_threads();
  std::vector<std::string> ids((size_t)T);
  std::vector<long long> lo_of((size_t)T + 1, n), bad((size_t)T, -1);
  const int P = oryx_ff::parallel_ranges(n, 256, [&](long long lo, long long hi, int t) {
    lo_of[(size_t)t] = lo;
    std::string tok;
    std::string& id = ids[(size_t)t];
    for (long long j = lo; j < hi; ++j) {
      JsonCursor c{buf + begin[(size_t)j], buf + end[(size_t)j]};
      float* v = vecs + j * k;
      bool ok = c.eat('[') && c.token(tok);
      if (ok) id += tok;
      ok = ok && c.eat(',') && c.eat('[');
      for (int f = 0; ok && f < k; ++f) {
        if (f && !c.eat(',')) { ok = false; break; }
        c.ws();
        const char* fb = c.p;
        while (c.p < c.end && *c.p != ',' && *c.p != ']' && *c.p != ' ') ++c.p;
        if (!oryx_ff::parse_float(fb, c.p, v[f])) {
          const std::string_view t(fb, (size_t)(c.p - fb));
          if (t == "NaN") v[f] = std::numeric_limits<float>::quiet_NaN();
          else if (t == "Infinity") v[f] = std::numeric_limits<float>::infinity();
          else if (t == "-Infinity") v[f] = -std::numeric_limits<float>::infinity();
          else ok = false;
        }
      }
      ok = ok && c.eat(']') && c.eat(']');
      if (ok) { c.ws(); while (c.p < c.end && *c.p == '\r') ++c.p; ok = c.p == c.end; }
      if (!ok) { bad[(size_t)t] = j; return; }
      id_ends[j] = (long long)id.size();   // local; rebased below
    }
  });
  for (int t = 0; t < P; ++t)
    if (bad[(size_t)t] >= 0) return -(bad[(size_t)t] + 1);
  for (int t = 0; t < P; ++t) {
    const long long lo = lo_of[(size_t)t], hi = t + 1 < P ? lo_of[(size_t)t + 1] : n;
    const long long base = (long long)g_up_ids.size();
    for (long long j = lo; j < hi; ++j) id_ends[j] += base;
    g_up_ids += ids[(size_t)t];
  }
  return n;
}

// The id texts (back to back) and the known-item texts ('\0'-terminated) of the last
// oryx_parse_up_batch call; returns -(bytes needed) when a buffer is too small.
long long oryx_up_texts(char* ids, long long ids_cap, char* known, long long known_cap) {
  if ((long long)g_up_ids.size() > ids_cap || (long long)g_up_known.size() > known_cap)
    return -(long long)(g_up_ids.size() + g_up_known.size());
  memcpy(ids, g_up_ids.data(), g_up_ids.size());
  memcpy(known, g_up_known.data(), g_up_known.size());
  return (long long)g_up_ids.size();
}

// IDs only (the known-item texts stay behind for oryx_up_known_codes).
long long oryx_up_ids(char* ids, long long ids_cap) {
  if ((long long)g_up_ids.size() > ids_cap) return -(long long)g_up_ids.size();
  memcpy(ids, g_up_ids.data(), g_up_ids.size());
  return (long long)g_up_ids.size();
}

// The known items of the last UP parse on this thread as codes of dictionary `dh` (the
// serving model keeps known items as item codes, not millions of Python strings).  Returns
// the number of items (only the first `cap` are written).
long long oryx_up_known_codes(void* dh, long long* out, long long cap) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  const std::string& s = g_up_known;
  // token spans, then lookups of the (mostly already known) items on the native threads --
  // finds are read-only -- and the misses inserted in order on this thread, which numbers
  // new items exactly as one sequential pass would
  std::vector<std::pair<size_t, size_t>> tok;
  tok.reserve(s.size() / 8 + 1);
  for (size_t p = 0; p < s.size();) {
    const size_t e = s.find('\0', p);
    if (e == std::string::npos) break;
    tok.emplace_back(p, e - p);
    p = e + 1;
  }
  const long long n = (long long)tok.size();
  std::vector<long long> code((size_t)n);
  oryx_ff::parallel_ranges(n, 1 << 15, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t)
      code[(size_t)t] = d->find(std::string_view(s.data() + tok[(size_t)t].first,
                                                 tok[(size_t)t].second));
  });
  for (long long t = 0; t < n; ++t) {
    if (code[(size_t)t] < 0)
      code[(size_t)t] = d->encode(std::string_view(s.data() + tok[(size_t)t].first,
                                                   tok[(size_t)t].second));
    if (t < cap) out[t] = code[(size_t)t];
  }
  return n;
}

}  // extern "C"

namespace {

// One event's messages: ["X",user,row,[item]] if vx, then ["Y",item,row,[user]] if vy.
void als_update_messages(Dict* du, Dict* di, long long ue, long long ie, const char* xrow,
                         size_t xlen, const char* yrow, size_t ylen, bool vx, bool vy,
                         bool with_known, std::string& o, std::string& qu, std::string& qi) {
  qu.clear();
  qi.clear();
  json_quote(du->keys[(size_t)ue], qu);
  json_quote(di->keys[(size_t)ie], qi);
  if (vx) {
    o += "[\"X\",";
    o += qu;
    o += ',';
    o.append(xrow, xlen);
    if (with_known) { o += ",["; o += qi; o += ']'; }
    o += "]\n";
  }
  if (vy) {
    o += "[\"Y\",";
    o += qi;
    o += ',';
    o.append(yrow, ylen);
    if (with_known) { o += ",["; o += qu; o += ']'; }
    o += "]\n";
  }
}

// Runs the per-event formatter over the native threads and joins the parts into out; with
// msg_ends (capacity 2n), the end offset of every '\n'-terminated message (its '\n' excluded)
// is written and *n_msgs set.
template <class Fn>
long long join_event_parts(long long n, char* out, long long cap, long long* msg_ends,
                           long long* n_msgs, Fn&& fn) {
  const int T = oryx_ff::native_threads();
  std::vector<std::string> part((size_t)T);
  const int P = oryx_ff::parallel_ranges(n, 256, [&](long long lo, long long hi, int t) {
    fn(lo, hi, part[(size_t)t]);
  });
  long long need = 0;
  for (int t = 0; t < P; ++t) need += (long long)part[(size_t)t].size();
  if (need > cap) return -need;
  long long pos = 0, m = 0;
  for (int t = 0; t < P; ++t) {
    const std::string& q = part[(size_t)t];
    std::memcpy(out + pos, q.data(), q.size());
    if (msg_ends) {
      const char* b = q.data();
      const char* e = b + q.size();
      for (const char* c = b; c < e;) {
        const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(e - c)));
        if (!nl) break;
        msg_ends[m++] = pos + (nl - b);
        c = nl + 1;
      }
    }
    pos += (long long)q.size();
  }
  if (n_msgs) *n_msgs = m;
  return pos;
}

}  // namespace

extern "C" {

// The ALS speed layer's update messages for n folded-in events, in the reference's order
// (per event: ["X",user,[Xu'],[item]] if vx, then ["Y",item,[Yi'],[user]] if vy;
// ALSSpeedModelManager.java:182-215), '\n'-separated into out.  IDs come straight from the
// parse dictionaries by code.  Returns bytes used or -(bytes needed).
long long oryx_format_als_updates(void* users, void* items, const long long* u,
                                  const long long* i, const float* nx, const float* ny,
                                  const unsigned char* vx, const unsigned char* vy, long long n,
                                  int k, int with_known, char* out, long long cap) {
  auto* du = static_cast<Dict*>(users);
  auto* di = static_cast<Dict*>(items);
  return join_event_parts(n, out, cap, nullptr, nullptr,
                          [&](long long lo, long long hi, std::string& o) {
    o.reserve((size_t)(hi - lo) * (size_t)(k * 24 + 96));
    std::string qu, qi, xr, yr;
    for (long long e = lo; e < hi; ++e) {
      xr.clear();
      yr.clear();
      if (vx[e]) float_row(nx + e * k, k, xr);
      if (vy[e]) float_row(ny + e * k, k, yr);
      als_update_messages(du, di, u[e], i[e], xr.data(), xr.size(), yr.data(), yr.size(),
                          vx[e] != 0, vy[e] != 0, with_known != 0, o, qu, qi);
    }
  });
}

// As oryx_format_als_updates with the rows already formatted (e.g. on the GPU): row e of
// X is xtext[xends[e-1], xends[e]) (xends[-1] = 0), likewise Y.  msg_ends (capacity 2n)
// receives each message's end offset ('\n' excluded), *n_msgs their number.  Two threaded
// passes: message sizes per event (the quoted IDs are the only unknowns), then every thread
// writes its events straight into out at their prefix offsets.
long long oryx_assemble_als_updates(void* users, void* items, const long long* u,
                                    const long long* i, const char* xtext,
                                    const long long* xends, const char* ytext,
                                    const long long* yends, const unsigned char* vx,
                                    const unsigned char* vy, long long n, int with_known,
                                    char* out, long long cap, long long* msg_ends,
                                    long long* n_msgs) {
  auto* du = static_cast<Dict*>(users);
  auto* di = static_cast<Dict*>(items);
  std::vector<long long> bytes((size_t)n + 1, 0), msgs((size_t)n + 1, 0);
  // "[\"X\"," id "," row (",[" other "]")? "]\n"
  oryx_ff::parallel_ranges(n, 256, [&](long long lo, long long hi, int) {
    std::string q;
    for (long long e = lo; e < hi; ++e) {
      q.clear();
      json_quote(du->keys[(size_t)u[e]], q);
      const long long lu = (long long)q.size();
      q.clear();
      json_quote(di->keys[(size_t)i[e]], q);
      const long long li = (long long)q.size();
      const long long xs = e ? xends[e - 1] : 0, ys = e ? yends[e - 1] : 0;
      long long b = 0;
      if (vx[e]) b += 5 + lu + 1 + (xends[e] - xs) + (with_known ? 3 + li : 0) + 2;
      if (vy[e]) b += 5 + li + 1 + (yends[e] - ys) + (with_known ? 3 + lu : 0) + 2;
      bytes[(size_t)e + 1] = b;
      msgs[(size_t)e + 1] = (vx[e] ? 1 : 0) + (vy[e] ? 1 : 0);
    }
  });
  for (long long e = 0; e < n; ++e) {
    bytes[(size_t)e + 1] += bytes[(size_t)e];
    msgs[(size_t)e + 1] += msgs[(size_t)e];
  }
  if (bytes[(size_t)n] > cap) return -bytes[(size_t)n];
  oryx_ff::parallel_ranges(n, 256, [&](long long lo, long long hi, int) {
    std::string qu, qi;
    for (long long e = lo; e < hi; ++e) {
      qu.clear();
      qi.clear();
      json_quote(du->keys[(size_t)u[e]], qu);
      json_quote(di->keys[(size_t)i[e]], qi);
      char* o = out + bytes[(size_t)e];
      long long m = msgs[(size_t)e];
      auto put = [&](const char* p, size_t len) { std::memcpy(o, p, len); o += len; };
      auto one = [&](const char* kind, const std::string& self, const char* row, size_t rl,
                     const std::string& other) {
        put(kind, 5);
        put(self.data(), self.size());
        *o++ = ',';
        put(row, rl);
        if (with_known) {
          put(",[", 2);
          put(other.data(), other.size());
          *o++ = ']';
        }
        *o++ = ']';
        if (msg_ends) msg_ends[m++] = o - out;
        *o++ = '\n';
      };
      const long long xs = e ? xends[e - 1] : 0, ys = e ? yends[e - 1] : 0;
      if (vx[e]) one("[\"X\",", qu, xtext + xs, (size_t)(xends[e] - xs), qi);
      if (vy[e]) one("[\"Y\",", qi, ytext + ys, (size_t)(yends[e] - ys), qu);
    }
  });
  if (n_msgs) *n_msgs = msgs[(size_t)n];
  return bytes[(size_t)n];
}

}  // extern "C"

namespace {

// Span j of a blob with end offsets (ends[-1] = 0).
struct Spans {
  const char* blob;
  const long long* ends;
  const char* ptr(long long j) const { return blob + (j ? ends[j - 1] : 0); }
  size_t len(long long j) const { return (size_t)(ends[j] - (j ? ends[j - 1] : 0)); }
};

}  // namespace

extern "C" {

// Model rows as update messages / part-file lines (ALSUpdate.publishAdditionalModelData,
// ALSUpdate.java:183-235; the X/ Y/ text parts of saveFeaturesRDD):
//   kind 'Y' (or 'X' without known): ["Y",id_e,row_e]
//   kind 'X' with known:            ["X",id_e,row_e,known_{kidx[e]}]  (kidx[e] < 0: skipped,
//                                    the reference's join drops users without events)
//   kind 0:                          [id_e,row_e]
// IDs are raw UTF-8 spans (quoted here as json.dumps does), rows and known arrays JSON text
// spans.  '\n'-terminated into out; msg_ends receives each line's end ('\n' excluded) and
// *n_msgs their number.  Two threaded passes (sizes, then direct writes at prefix offsets).
// Returns bytes used or -(bytes needed).
long long oryx_assemble_row_messages(int kind, const char* ids, const long long* id_ends,
                                     const char* rows, const long long* row_ends, long long n,
                                     const char* known, const long long* known_ends,
                                     const long long* kidx, char* out, long long cap,
                                     long long* msg_ends, long long* n_msgs) {
  const Spans id{ids, id_ends}, row{rows, row_ends}, kn{known, known_ends};
  const bool with_known = known != nullptr && kidx != nullptr;
  const size_t head = kind ? 5 : 1;   // "[\"X\"," or "["
  std::vector<long long> bytes((size_t)n + 1, 0), msgs((size_t)n + 1, 0);
  oryx_ff::parallel_ranges(n, 1024, [&](long long lo, long long hi, int) {
    std::string q;
    for (long long e = lo; e < hi; ++e) {
      if (with_known && kidx[e] < 0) continue;
      q.clear();
      json_quote(id.ptr(e), id.len(e), q);
      long long b = (long long)(head + q.size() + 1 + row.len(e) + 2);
      if (with_known) b += 1 + (long long)kn.len(kidx[e]);
      bytes[(size_t)e + 1] = b;
      msgs[(size_t)e + 1] = 1;
    }
  });
  for (long long e = 0; e < n; ++e) {
    bytes[(size_t)e + 1] += bytes[(size_t)e];
    msgs[(size_t)e + 1] += msgs[(size_t)e];
  }
  if (bytes[(size_t)n] > cap) return -bytes[(size_t)n];
  const char hdr[6] = {'[', '"', (char)kind, '"', ',', 0};
  oryx_ff::parallel_ranges(n, 1024, [&](long long lo, long long hi, int) {
    std::string q;
    for (long long e = lo; e < hi; ++e) {
      if (with_known && kidx[e] < 0) continue;
      q.clear();
      json_quote(id.ptr(e), id.len(e), q);
      char* o = out + bytes[(size_t)e];
      if (kind) { std::memcpy(o, hdr, 5); o += 5; } else { *o++ = '['; }
      std::memcpy(o, q.data(), q.size());
      o += q.size();
      *o++ = ',';
      std::memcpy(o, row.ptr(e), row.len(e));
      o += row.len(e);
      if (with_known) {
        *o++ = ',';
        std::memcpy(o, kn.ptr(kidx[e]), kn.len(kidx[e]));
        o += kn.len(kidx[e]);
      }
      *o++ = ']';
      if (msg_ends) msg_ends[msgs[(size_t)e]] = o - out;
      *o++ = '\n';
    }
  });
  if (n_msgs) *n_msgs = msgs[(size_t)n];
  return bytes[(size_t)n];
}

// Known-item JSON arrays per user code (the X messages' last element): the (user, item)
// code pairs come sorted by user; user c's array lists the quoted names (items dictionary)
// of its items in the given order, "[]" for a user without pairs.  ends[c], c < n_users.
// Returns bytes used or -(bytes needed).
long long oryx_known_items_text(void* items, const long long* uu, const long long* ii,
                                long long m, long long n_users, char* out, long long cap,
                                long long* ends) {
  auto* di = static_cast<Dict*>(items);
  const long long n_items = (long long)di->keys.size();
  std::vector<std::string> qname((size_t)n_items);
  oryx_ff::parallel_ranges(n_items, 4096, [&](long long lo, long long hi, int) {
    for (long long j = lo; j < hi; ++j) json_quote(di->keys[(size_t)j], qname[(size_t)j]);
  });
  // pair range of every user (uu ascending)
  std::vector<long long> first((size_t)n_users + 1);
  oryx_ff::parallel_ranges(n_users + 1, 4096, [&](long long lo, long long hi, int) {
    for (long long c = lo; c < hi; ++c)
      first[(size_t)c] = std::lower_bound(uu, uu + m, c) - uu;
  });
  std::vector<long long> bytes((size_t)n_users + 1, 0);
  oryx_ff::parallel_ranges(n_users, 1024, [&](long long lo, long long hi, int) {
    for (long long c = lo; c < hi; ++c) {
      const long long a = first[(size_t)c], b = first[(size_t)c + 1];
      long long sz = 2 + (b > a ? b - a - 1 : 0);
      for (long long p = a; p < b; ++p) sz += (long long)qname[(size_t)ii[p]].size();
      bytes[(size_t)c + 1] = sz;
    }
  });
  for (long long c = 0; c < n_users; ++c) bytes[(size_t)c + 1] += bytes[(size_t)c];
  if (bytes[(size_t)n_users] > cap) return -bytes[(size_t)n_users];
  oryx_ff::parallel_ranges(n_users, 1024, [&](long long lo, long long hi, int) {
    for (long long c = lo; c < hi; ++c) {
      char* o = out + bytes[(size_t)c];
      *o++ = '[';
      for (long long p = first[(size_t)c]; p < first[(size_t)c + 1]; ++p) {
        if (p > first[(size_t)c]) *o++ = ',';
        const std::string& q = qname[(size_t)ii[p]];
        std::memcpy(o, q.data(), q.size());
        o += q.size();
      }
      *o++ = ']';
      ends[c] = o - out;
    }
  });
  return bytes[(size_t)n_users];
}

// buf[0, n) written to path as concatenated gzip members, one per 2 MB slice, compressed on
// the native threads (a multi-member file is a single gzip stream to gzip / zlib / Hadoop
// readers).  Every member's header carries an extra subfield "OX" (RFC 1952 FEXTRA, ignored
// by other readers) with the member's total size and its uncompressed size, so that
// oryx_gzip_indexed_inflate can find the members without inflating and decompress them in
// parallel (the BGZF idea).  Returns 0, or -1 (file error) / -2 (zlib error).
int oryx_write_gzip(const char* path, const char* buf, long long n, int level) {
  const long long slice = 2ll << 20;
  const long long ns = n > 0 ? (n + slice - 1) / slice : 1;
  std::vector<std::string> part((size_t)ns);
  std::vector<int> bad((size_t)ns, 0);
  oryx_ff::parallel_ranges(ns, 1, [&](long long lo, long long hi, int) {
    for (long long k = lo; k < hi; ++k) {
      const long long a = k * slice, len = n > 0 ? std::min(slice, n - a) : 0;
      const Bytef* src = reinterpret_cast<const Bytef*>(buf + (len > 0 ? a : 0));
      z_stream z{};
      if (deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
        bad[(size_t)k] = 1;
        continue;
      }
      std::string& o = part[(size_t)k];
      const size_t H = 24;                     // 10 fixed + XLEN + "OX" subfield of 8 bytes
      o.resize(H + deflateBound(&z, (uLong)len) + 8);
      z.next_in = const_cast<Bytef*>(src);
      z.avail_in = (uInt)len;
      z.next_out = reinterpret_cast<Bytef*>(&o[H]);
      z.avail_out = (uInt)(o.size() - H - 8);
      if (deflate(&z, Z_FINISH) != Z_STREAM_END) bad[(size_t)k] = 1;
      const size_t body = z.total_out;
      deflateEnd(&z);
      const uint32_t total = (uint32_t)(H + body + 8), isize = (uint32_t)len;
      const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), src, (uInt)len);
      unsigned char* h = reinterpret_cast<unsigned char*>(&o[0]);
      const unsigned char fixed[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 255, 12, 0, 'O', 'X', 8, 0};
      std::memcpy(h, fixed, 16);
      std::memcpy(h + 16, &total, 4);
      std::memcpy(h + 20, &isize, 4);
      std::memcpy(h + H + body, &crc, 4);
      std::memcpy(h + H + body + 4, &isize, 4);
      o.resize(total);
    }
  });
  for (int b : bad)
    if (b) return -2;
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  for (const std::string& o : part)
    if (std::fwrite(o.data(), 1, o.size(), f) != o.size()) { std::fclose(f); return -1; }
  return std::fclose(f) == 0 ? 0 : -1;
}

namespace {

// The members of an "OX"-indexed gzip file: (offset, total size, output offset, out size);
// false when any member lacks the index (other writers).
bool gzip_members(const unsigned char* b, long long n,
                  std::vector<std::array<long long, 4>>& m) {
  long long pos = 0, out = 0;
  while (pos < n) {
    if (n - pos < 24 || b[pos] != 0x1f || b[pos + 1] != 0x8b || b[pos + 2] != 8 ||
        b[pos + 3] != 4)
      return false;
    const int xlen = b[pos + 10] | (b[pos + 11] << 8);
    if (xlen != 12 || b[pos + 12] != 'O' || b[pos + 13] != 'X' || b[pos + 14] != 8 ||
        b[pos + 15] != 0)
      return false;
    uint32_t total, isize;
    std::memcpy(&total, b + pos + 16, 4);
    std::memcpy(&isize, b + pos + 20, 4);
    if (total < 32 || pos + total > n) return false;
    m.push_back({pos, (long long)total, out, (long long)isize});
    pos += total;
    out += isize;
  }
  return !m.empty();
}

}  // namespace

// Uncompressed size of an "OX"-indexed gzip file (see oryx_write_gzip), -1 when it is not one.
long long oryx_gzip_indexed_size(const unsigned char* b, long long n) {
  std::vector<std::array<long long, 4>> m;
  if (!gzip_members(b, n, m)) return -1;
  return m.back()[2] + m.back()[3];
}

// Inflates an "OX"-indexed gzip file into out (cap >= oryx_gzip_indexed_size), members on the
// native threads, each checked against its CRC-32 and size.  Returns the size, -1 when the
// file is not indexed, -2 on a corrupt member.
long long oryx_gzip_indexed_inflate(const unsigned char* b, long long n, char* out,
                                    long long cap) {
  std::vector<std::array<long long, 4>> m;
  if (!gzip_members(b, n, m)) return -1;
  const long long size = m.back()[2] + m.back()[3];
  if (size > cap) return -2;
  std::vector<int> bad(m.size(), 0);
  oryx_ff::parallel_ranges((long long)m.size(), 1, [&](long long lo, long long hi, int) {
    for (long long k = lo; k < hi; ++k) {
      const auto& e = m[(size_t)k];
      z_stream z{};
      if (inflateInit2(&z, -15) != Z_OK) { bad[(size_t)k] = 1; continue; }
      z.next_in = const_cast<Bytef*>(b + e[0] + 24);
      z.avail_in = (uInt)(e[1] - 24 - 8);
      Bytef* dst = reinterpret_cast<Bytef*>(out + e[2]);
      z.next_out = dst;
      z.avail_out = (uInt)e[3];
      const int rc = inflate(&z, Z_FINISH);
      const bool ok = rc == Z_STREAM_END && (long long)z.total_out == e[3];
      inflateEnd(&z);
      uint32_t crc;
      std::memcpy(&crc, b + e[0] + e[1] - 8, 4);
      if (!ok || (uint32_t)crc32(crc32(0L, Z_NULL, 0), dst, (uInt)e[3]) != crc)
        bad[(size_t)k] = 1;
    }
  });
  for (int x : bad)
    if (x) return -2;
  return size;
}

}  // extern "C"

// ------------------------------------------------------------------ newline-delimited text
// (oryx_amd.textlines.TextLines: messages held as one buffer, every line ending in '\n')

extern "C" {

// End offset (position of the '\n') of every line of buf[0, len), threaded over blocks cut at
// newlines.  Returns the number of lines written to out_ends (at most max_lines).
long long oryx_line_ends(const char* buf, long long len, long long* out_ends,
                         long long max_lines) {
  if (len <= 0) return 0;
  const int P = len >= (16ll << 20) ? oryx_ff::native_threads() : 1;
  std::vector<const char*> cut((size_t)P + 1);
  cut[0] = buf;
  cut[(size_t)P] = buf + len;
  for (int t = 1; t < P; ++t) {
    const char* c = buf + len * t / P;
    if (c < cut[(size_t)t - 1]) c = cut[(size_t)t - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(buf + len - c)));
    cut[(size_t)t] = nl ? nl + 1 : buf + len;
  }
  std::vector<long long> cnt((size_t)P, 0);
  auto count = [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long c = 0;
      for (const char* p = cut[(size_t)t]; p < cut[(size_t)t + 1];) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(cut[(size_t)t + 1] - p)));
        if (!nl) break;
        ++c;
        p = nl + 1;
      }
      cnt[(size_t)t] = c;
    }
  };
  oryx_ff::parallel_ranges(P, 1, count);
  std::vector<long long> first((size_t)P + 1, 0);
  for (int t = 0; t < P; ++t) first[(size_t)t + 1] = first[(size_t)t] + cnt[(size_t)t];
  const long long total = first[(size_t)P];
  if (total > max_lines) return -total;
  auto fill = [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      long long k = first[(size_t)t];
      for (const char* p = cut[(size_t)t]; p < cut[(size_t)t + 1];) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(cut[(size_t)t + 1] - p)));
        if (!nl) break;
        out_ends[k++] = (long long)(nl - buf);
        p = nl + 1;
      }
    }
  };
  oryx_ff::parallel_ranges(P, 1, fill);
  return total;
}

// Copies lines idx[0..n) (line j = buf[ends[j-1] + 1, ends[j]), ends[-1] = -1) into out, each
// followed by '\n'; out must hold sum of their lengths + n bytes.  Returns bytes written.
long long oryx_gather_lines(const char* buf, const long long* ends, const long long* idx,
                            long long n, char* out) {
  std::vector<long long> at((size_t)n + 1, 0);
  for (long long k = 0; k < n; ++k) {
    const long long j = idx[k];
    const long long b = j ? ends[j - 1] + 1 : 0;
    at[(size_t)k + 1] = at[(size_t)k] + (ends[j] - b) + 1;
  }
  oryx_ff::parallel_ranges(n, 1 << 16, [&](long long lo, long long hi, int) {
    for (long long k = lo; k < hi; ++k) {
      const long long j = idx[k];
      const long long b = j ? ends[j - 1] + 1 : 0;
      const long long l = ends[j] - b + 1;   // the line and its '\n'
      memcpy(out + at[(size_t)k], buf + b, (size_t)l);
    }
  });
  return at[(size_t)n];
}

}  // extern "C"

extern "C" {

// Concatenates n buffers (ptrs[k], lens[k] bytes) into out, the copy split into equal byte
// ranges over the native threads (a drain's per-partition text buffers, hundreds of MB, into
// the one buffer the parser reads).  Returns the bytes written.
long long oryx_concat_buffers(const char* const* ptrs, const long long* lens, long long n,
                              char* out) {
  std::vector<long long> at((size_t)n + 1, 0);
  for (long long k = 0; k < n; ++k) at[(size_t)k + 1] = at[(size_t)k] + lens[k];
  const long long total = at[(size_t)n];
  constexpr long long kPiece = 4ll << 20;
  oryx_ff::parallel_ranges((total + kPiece - 1) / kPiece, 1, [&](long long lo, long long hi, int) {
    const long long b = lo * kPiece, e = std::min(total, hi * kPiece);
    // buffers overlapping [b, e)
    long long k = (long long)(std::upper_bound(at.begin(), at.end(), b) - at.begin()) - 1;
    for (; k < n && at[(size_t)k] < e; ++k) {
      const long long s0 = std::max(b, at[(size_t)k]);
      const long long s1 = std::min(e, at[(size_t)k + 1]);
      if (s1 > s0) memcpy(out + s0, ptrs[k] + (s0 - at[(size_t)k]), (size_t)(s1 - s0));
    }
  });
  return total;
}

}  // extern "C"

extern "C" {

// Time-ordered per-(user, item) aggregation of parsed events (ALSUpdate.aggregateScores with
// SUM_WITH_NAN): events ordered by (user, item), then timestamp, then arrival; implicit: the
// sum of the values after the group's last NaN (a trailing NaN drops the pair), explicit: the
// last value (NaN drops the pair).  Writes the surviving pairs in (user, item) order; returns
// their count.  One native sort of packed keys instead of a dozen numpy passes: a 10k-event
// speed-layer micro-batch aggregates in ~0.2 ms.
long long oryx_aggregate_scores(const long long* u, const long long* i, const double* s,
                                const long long* ts, long long n, int implicit,
                                long long* out_u, long long* out_i, double* out_s) {
  if (n <= 0) return 0;
  long long n_i = 0;
  for (long long k = 0; k < n; ++k) n_i = std::max(n_i, i[k] + 1);
  struct Ev {
    unsigned long long key;
    long long ts;
    long long at;
  };
  std::vector<Ev> ev((size_t)n);
  for (long long k = 0; k < n; ++k)
    ev[(size_t)k] = Ev{(unsigned long long)u[k] * (unsigned long long)n_i + (unsigned long long)i[k],
                       ts[k], k};
  std::sort(ev.begin(), ev.end(), [](const Ev& a, const Ev& b) {
    if (a.key != b.key) return a.key < b.key;
    if (a.ts != b.ts) return a.ts < b.ts;
    return a.at < b.at;
  });
  long long m = 0;
  for (size_t b = 0; b < ev.size();) {
    size_t e = b + 1;
    while (e < ev.size() && ev[e].key == ev[b].key) ++e;
    double v;
    if (implicit) {
      // sum after the last NaN (delete); a NaN last in time drops the pair
      size_t from = b;
      for (size_t k = b; k < e; ++k)
        if (std::isnan(s[ev[k].at])) from = k + 1;
      if (from == e) {
        v = std::numeric_limits<double>::quiet_NaN();
      } else {
        v = 0.0;
        for (size_t k = from; k < e; ++k) v += s[ev[k].at];
      }
    } else {
      v = s[ev[e - 1].at];
    }
    if (!std::isnan(v)) {
      out_u[m] = (long long)(ev[b].key / (unsigned long long)n_i);
      out_i[m] = (long long)(ev[b].key % (unsigned long long)n_i);
      out_s[m] = v;
      ++m;
    }
    b = e;
  }
  return m;
}

}  // extern "C"

// ---- speed-layer micro-batch (ALSSpeedModelManager.buildUpdates, [speed-app]/als/
// ALSSpeedModelManager.java:134-205) without per-batch dictionaries: each line's user and
// item are looked up straight in the stores' id -> row maps (read-only, so the lines are
// parsed on all native threads); only IDs the stores do not hold get a batch-local code.
// The pairs are then aggregated in time order (ALSUpdate.aggregateScores semantics) and the
// UP messages assembled from the events' own key bytes.

namespace {

// JSON-quoted length of a key, and the quoted key written at dst (returns the end): keys
// that need no escaping (the usual case) are '"' + bytes + '"' without a temporary string.
bool plain_json(const char* s, size_t n) {
  for (size_t k = 0; k < n; ++k) {
    const unsigned char c = (unsigned char)s[k];
    if (c < 0x20 || c >= 0x80 || c == '"' || c == '\\') return false;
  }
  return true;
}

size_t quoted_len(std::string_view k) {
  if (plain_json(k.data(), k.size())) return k.size() + 2;
  std::string q;
  json_quote(k.data(), k.size(), q);
  return q.size();
}

// (ql: the key's quoted_len; a key that needs escapes always quotes longer than size + 2)
char* put_quoted(std::string_view k, size_t ql, char* o) {
  if (ql == k.size() + 2) {
    *o++ = '"';
    memcpy(o, k.data(), k.size());
    o += k.size();
    *o++ = '"';
    return o;
  }
  std::string q;
  json_quote(k.data(), k.size(), q);
  memcpy(o, q.data(), q.size());
  return o + q.size();
}

struct SpeedBatch {
  // per event: store row (>= 0) or -(new key index) - 1; strength; timestamp; key views
  std::vector<int64_t> u, i;
  std::vector<uint32_t> uql, iql;       // the keys' JSON-quoted lengths (quoted_len)
  std::vector<double> s;
  std::vector<long long> ts;
  std::vector<std::string_view> uk, ik;
  // unescaped keys of quoted / JSON lines, per parse chunk (a moved deque keeps its
  // elements where they are, so the views into them stay valid)
  std::vector<std::deque<std::string>> owned;
  FlatIndex nu_idx, ni_idx;             // new keys -> index
  std::vector<std::string_view> nu_keys, ni_keys;
  // aggregated pairs: representative event (for the keys)
  std::vector<int64_t> rep;
  // aggregation scratch (kept for its capacity): pair hash table, per-pair first event and
  // count, per-event pair, grouped events
  std::vector<int32_t> tab, first, cnt, pid, start, ev;
  const char* buf = nullptr;

  void clear() {
    u.clear(); i.clear(); s.clear(); ts.clear(); uk.clear(); ik.clear(); owned.clear();
    uql.clear(); iql.clear();
    nu_idx.clear(); ni_idx.clear(); nu_keys.clear(); ni_keys.clear();
    rep.clear();
  }
};

struct SpeedChunk {
  std::vector<int64_t> u, i;
  std::vector<uint32_t> uql, iql;
  std::vector<double> s;
  std::vector<long long> ts;
  std::vector<std::string_view> uk, ik;
  std::vector<uint64_t> hu, hi;         // the keys' RowMap hashes
  std::deque<std::string> owned;
  bool has_new = false;                 // a key the stores lack
};

// splitmix64 finalizer: the aggregation's (user row, item row) pair hash
inline uint64_t pair_mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

}  // namespace

extern "C" {

void* oryx_speed_new() { return new SpeedBatch(); }
void oryx_speed_free(void* h) { delete static_cast<SpeedBatch*>(h); }

// Parses rating lines (see oryx_parse_ratings) resolving users / items in the row maps xm / ym
// (read-only here: the caller holds off writers).  Returns the number of events.
long long oryx_speed_parse(void* h, const char* buf, long long len, void* xm, void* ym,
                           long long default_ts) {
  SpeedBatch* b = static_cast<SpeedBatch*>(h);
  const RowMap* X = static_cast<const RowMap*>(xm);
  const RowMap* Y = static_cast<const RowMap*>(ym);
  b->clear();
  b->buf = buf;
  // ~32 KB of lines per thread (a 10k-event batch is ~250 KB)
  int P = 1;
  if (len >= (64ll << 10))
    P = (int)std::max<long long>(1, std::min<long long>(len / (32ll << 10),
                                                       oryx_ff::native_threads()));
  std::vector<const char*> cut = line_chunks(buf, len, P);
  std::vector<SpeedChunk> ch((size_t)P);
  oryx_ff::parallel_ranges(P, 1, [&](long long lo, long long hi, int) {
    for (long long t = lo; t < hi; ++t) {
      SpeedChunk& c = ch[(size_t)t];
      const char* p = cut[(size_t)t];
      const char* end = cut[(size_t)t + 1];
      const size_t est = (size_t)((end - p) / 20 + 1);
      c.u.reserve(est); c.i.reserve(est); c.s.reserve(est); c.ts.reserve(est);
      c.uk.reserve(est); c.ik.reserve(est); c.hu.reserve(est); c.hi.reserve(est);
      std::vector<std::string> toks;
      std::string field;
      std::string_view f[4];
      while (p < end) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        const char* le = nl ? nl : end;
        const char* lend = le;
        if (lend > p && lend[-1] == '\r') --lend;
        if (lend > p) {
          bool stable;
          double sv;
          long long tv = default_ts;
          if (parse_rating_fields(p, lend, toks, field, f, &stable, &sv, &tv)) {
            std::string_view a = f[0], bk = f[1];
            if (!stable) {
              c.owned.emplace_back(a);
              a = c.owned.back();
              c.owned.emplace_back(bk);
              bk = c.owned.back();
            }
            // the row-map probes wait for the second pass: the maps of a 20M-row store are
            // far larger than the caches, and probing as each line is parsed left one miss
            // in flight per thread; hashed and prefetched here, the chunk's misses overlap
            const uint64_t ha = RowMap::hash(a.data(), a.size());
            const uint64_t hb = RowMap::hash(bk.data(), bk.size());
            X->prefetch(ha);
            Y->prefetch(hb);
            c.hu.push_back(ha);
            c.hi.push_back(hb);
            c.s.push_back(sv);
            c.ts.push_back(tv);
            c.uk.push_back(a);
            c.ik.push_back(bk);
            c.uql.push_back((uint32_t)quoted_len(a));
            c.iql.push_back((uint32_t)quoted_len(bk));
          }
        }
        p = nl ? nl + 1 : end;
      }
      const size_t m = c.hu.size();
      c.u.resize(m);
      c.i.resize(m);
      for (size_t r = 0; r < m; ++r) {
        c.u[r] = X->row_of(c.uk[r].data(), c.uk[r].size(), c.hu[r]);
        c.i[r] = Y->row_of(c.ik[r].data(), c.ik[r].size(), c.hi[r]);
        c.has_new |= (c.u[r] < 0) | (c.i[r] < 0);
      }
    }
  });
  size_t n = 0;
  for (auto& c : ch) n += c.u.size();
  b->u.reserve(n); b->i.reserve(n); b->s.reserve(n); b->ts.reserve(n);
  b->uk.reserve(n); b->ik.reserve(n); b->uql.reserve(n); b->iql.reserve(n);
  for (auto& c : ch) {
    const size_t base = b->u.size();
    b->u.insert(b->u.end(), c.u.begin(), c.u.end());
    b->i.insert(b->i.end(), c.i.begin(), c.i.end());
    b->s.insert(b->s.end(), c.s.begin(), c.s.end());
    b->ts.insert(b->ts.end(), c.ts.begin(), c.ts.end());
    b->uk.insert(b->uk.end(), c.uk.begin(), c.uk.end());
    b->ik.insert(b->ik.end(), c.ik.begin(), c.ik.end());
    b->uql.insert(b->uql.end(), c.uql.begin(), c.uql.end());
    b->iql.insert(b->iql.end(), c.iql.begin(), c.iql.end());
    // keys the stores lack get batch codes in first-appearance order (chunks in order)
    if (c.has_new) {
      for (size_t r = 0; r < c.u.size(); ++r) {
        bool ins;
        if (c.u[r] < 0) {
          const int32_t k = b->nu_idx.find_or_add(c.uk[r], (int32_t)b->nu_keys.size(), &ins);
          if (ins) b->nu_keys.push_back(c.uk[r]);
          b->u[base + r] = -(int64_t)k - 1;
        }
        if (c.i[r] < 0) {
          const int32_t k = b->ni_idx.find_or_add(c.ik[r], (int32_t)b->ni_keys.size(), &ins);
          if (ins) b->ni_keys.push_back(c.ik[r]);
          b->i[base + r] = -(int64_t)k - 1;
        }
      }
    }
    b->owned.push_back(std::move(c.owned));
  }
  return (long long)n;
}

// Keys of the batch that the stores do not hold: which = 0 users, 1 items; back to back in
// out with end offsets.  Returns bytes, or -(bytes needed).
long long oryx_speed_new_keys(void* h, int which, char* out, long long cap, long long* ends) {
  SpeedBatch* b = static_cast<SpeedBatch*>(h);
  const auto& keys = which ? b->ni_keys : b->nu_keys;
  long long need = 0;
  for (auto k : keys) need += (long long)k.size();
  if (need > cap) return -need;
  long long pos = 0;
  for (size_t j = 0; j < keys.size(); ++j) {
    memcpy(out + pos, keys[j].data(), keys[j].size());
    pos += (long long)keys[j].size();
    ends[j] = pos;
  }
  return pos;
}

long long oryx_speed_counts(void* h, long long* out) {
  SpeedBatch* b = static_cast<SpeedBatch*>(h);
  out[0] = (long long)b->u.size();
  out[1] = (long long)b->nu_keys.size();
  out[2] = (long long)b->ni_keys.size();
  out[3] = (long long)b->rep.size();
  return out[0];
}

// Time-ordered aggregation per (user, item) (implicit: sum after the last delete, a trailing
// delete drops the pair; explicit: the last value, NaN drops it), pairs in the order of their
// first event.  Writes the pairs' user / item rows (-1: not in the store) and values; returns
// the number of pairs.  Pairs are found through a hash table over (user, item) rather than by
// sorting the events: a micro-batch's pairs are nearly all distinct, so one probe per event
// and a pass over the few repeated pairs replace four radix passes (0.38 -> ~0.05 ms per
// 10k events on the 8-core host).
long long oryx_speed_aggregate(void* h, int implicit, long long* out_u, long long* out_i,
                               double* out_s) {
  SpeedBatch* b = static_cast<SpeedBatch*>(h);
  const size_t n = b->u.size();
  b->rep.clear();
  if (n == 0) return 0;
  size_t cap = 64;
  while (cap < 2 * n) cap <<= 1;
  std::vector<int32_t>& tab = b->tab;
  tab.assign(cap, -1);
  std::vector<int32_t>& first = b->first;   // first event of each pair
  std::vector<int32_t>& cnt = b->cnt;       // events per pair
  std::vector<int32_t>& pid = b->pid;       // pair of each event
  first.clear();
  cnt.clear();
  pid.resize(n);
  const int64_t* U = b->u.data();
  const int64_t* I = b->i.data();
  const size_t msk = cap - 1;
  for (size_t r = 0; r < n; ++r) {
    size_t j = (size_t)pair_mix((uint64_t)U[r] * 0x9E3779B97F4A7C15ull ^ (uint64_t)I[r]) & msk;
    int32_t p;
    for (;; j = (j + 1) & msk) {
      p = tab[j];
      if (p < 0) {
        p = (int32_t)first.size();
        tab[j] = p;
        first.push_back((int32_t)r);
        cnt.push_back(0);
        break;
      }
      const int32_t f = first[(size_t)p];
      if (U[f] == U[r] && I[f] == I[r]) break;
    }
    pid[r] = p;
    ++cnt[(size_t)p];
  }
  const size_t np = first.size();
  std::vector<int64_t>& rep = b->rep;
  rep.resize(np);
  size_t m = 0;
  auto emit = [&](int64_t r, double v) {
    if (std::isnan(v)) return;
    out_u[m] = U[r] >= 0 ? U[r] : -1;
    out_i[m] = I[r] >= 0 ? I[r] : -1;
    out_s[m] = v;
    rep[m++] = r;
  };
  if (np == n) {
    // every pair has one event: its value (NaN = a delete drops the pair either way)
    for (size_t r = 0; r < n; ++r) emit((int64_t)r, b->s[r]);
  } else {
    // events grouped by pair, arrival order kept (counting sort), then each repeated pair's
    // events put in time order (stable: equal timestamps stay in arrival order)
    std::vector<int32_t>& start = b->start;
    std::vector<int32_t>& ev = b->ev;
    start.resize(np + 1);
    start[0] = 0;
    for (size_t p = 0; p < np; ++p) start[p + 1] = start[p] + cnt[p];
    ev.resize(n);
    {
      std::vector<int32_t>& at = b->cnt;   // reused as the fill cursors
      for (size_t p = 0; p < np; ++p) at[p] = start[p];
      for (size_t r = 0; r < n; ++r) ev[(size_t)at[(size_t)pid[r]]++] = (int32_t)r;
    }
    const long long* T = b->ts.data();
    const double* S = b->s.data();
    for (size_t p = 0; p < np; ++p) {
      int32_t* g0 = ev.data() + start[p];
      int32_t* g1 = ev.data() + start[p + 1];
      if (g1 - g0 == 1) {
        emit(*g0, S[*g0]);
        continue;
      }
      bool sorted = true;
      for (int32_t* e = g0 + 1; e < g1; ++e) sorted &= T[e[-1]] <= T[*e];
      if (!sorted)
        std::stable_sort(g0, g1, [&](int32_t x, int32_t y) { return T[x] < T[y]; });
      double v;
      if (implicit) {
        int32_t* from = g0;
        for (int32_t* e = g0; e < g1; ++e)
          if (std::isnan(S[*e])) from = e + 1;
        if (from == g1) {
          v = std::numeric_limits<double>::quiet_NaN();
        } else {
          v = 0.0;
          for (int32_t* e = from; e < g1; ++e) v += S[*e];
        }
      } else {
        v = S[g1[-1]];
      }
      emit(*g0, v);
    }
  }
  rep.resize(m);
  return (long long)m;
}

long long oryx_log_append_fill(void* h, int partition, const char* key, int key_len,
                               const long long* lens, int n,
                               void (*fill)(void* ctx, long long j, char* dst), void* ctx,
                               long long ts_ms, int do_fsync);

}  // extern "C"

namespace {

// What oryx_speed_append's fill callback needs: message m is side sides[m] (0 X, 1 Y) of
// aggregated pair pair[m] (indexed from lo).
struct SpeedFill {
  const SpeedBatch* b;
  long long lo;
  const char* xtext;
  const long long* xends;
  const char* ytext;
  const long long* yends;
  int with_known;
  std::vector<int32_t> pair;
  std::vector<uint8_t> side;
};

void speed_fill(void* ctx, long long m, char* o) {
  const SpeedFill& F = *static_cast<const SpeedFill*>(ctx);
  const long long e = F.pair[(size_t)m];
  const int64_t r = F.b->rep[(size_t)(F.lo + e)];
  const std::string_view uk = F.b->uk[(size_t)r], ik = F.b->ik[(size_t)r];
  const bool y = F.side[(size_t)m] != 0;
  const long long* ends = y ? F.yends : F.xends;
  const long long s0 = e ? ends[e - 1] : 0;
  memcpy(o, y ? "[\"Y\"," : "[\"X\",", 5);
  const size_t uq = F.b->uql[(size_t)r], iq = F.b->iql[(size_t)r];
  o = put_quoted(y ? ik : uk, y ? iq : uq, o + 5);
  *o++ = ',';
  memcpy(o, (y ? F.ytext : F.xtext) + s0, (size_t)(ends[e] - s0));
  o += ends[e] - s0;
  if (F.with_known) {
    *o++ = ',';
    *o++ = '[';
    o = put_quoted(y ? uk : ik, y ? uq : iq, o);
    *o++ = ']';
  }
  *o = ']';
}

}  // namespace

extern "C" {

// The aggregated pairs [lo, hi)'s UP messages (the layout of oryx_speed_assemble, without the
// separators) appended to the log `topic` as records with key "UP", formatted by the log's
// writer threads straight into the segment (oryx_log_append_fill): the row text crosses
// memory once between the GPU's copy and the page cache.  Valid until the batch's next
// parse.  Returns the last offset written, -1 on error, -2 when a message exceeds the topic's
// maximum size (nothing written); *n_msgs receives the number of messages.
long long oryx_speed_append(void* h, void* topic, int partition, long long lo, long long hi,
                            const char* xtext, const long long* xends, const char* ytext,
                            const long long* yends, const unsigned char* vx,
                            const unsigned char* vy, int with_known, long long ts_ms,
                            int do_fsync, long long* n_msgs) {
  const auto T0 = std::chrono::steady_clock::now();
  const SpeedBatch* b = static_cast<const SpeedBatch*>(h);
  const long long n = hi - lo;
  SpeedFill F{b, lo, xtext, xends, ytext, yends, with_known, {}, {}};
  std::vector<long long> cnt((size_t)n + 1, 0);
  for (long long e = 0; e < n; ++e) cnt[(size_t)e + 1] = cnt[(size_t)e] + (vx[e] ? 1 : 0) + (vy[e] ? 1 : 0);
  const long long m = cnt[(size_t)n];
  *n_msgs = m;
  if (m == 0) return -1;
  F.pair.resize((size_t)m);
  F.side.resize((size_t)m);
  std::vector<long long> lens((size_t)m);
  const auto T1 = std::chrono::steady_clock::now();
  oryx_ff::parallel_ranges(n, 32768, [&](long long a, long long z, int) {
    for (long long e = a; e < z; ++e) {
      const int64_t r = b->rep[(size_t)(lo + e)];
      const long long lu = b->uql[(size_t)r], li = b->iql[(size_t)r];
      long long j = cnt[(size_t)e];
      if (vx[e]) {
        const long long xs = e ? xends[e - 1] : 0;
        F.pair[(size_t)j] = (int32_t)e;
        F.side[(size_t)j] = 0;
        lens[(size_t)j++] = 5 + lu + 1 + (xends[e] - xs) + (with_known ? 3 + li : 0) + 1;
      }
      if (vy[e]) {
        const long long ys = e ? yends[e - 1] : 0;
        F.pair[(size_t)j] = (int32_t)e;
        F.side[(size_t)j] = 1;
        lens[(size_t)j++] = 5 + li + 1 + (yends[e] - ys) + (with_known ? 3 + lu : 0) + 1;
      }
    }
  });
  if (std::getenv("ORYX_LOG_DEBUG"))
    fprintf(stderr, "speed_append sizes %.3f ms (setup %.3f)\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count(),
            std::chrono::duration<double, std::milli>(T1 - T0).count());
  const long long res = oryx_log_append_fill(topic, partition, "UP", 2, lens.data(), (int)m,
                                             speed_fill, &F, ts_ms, do_fsync);
  if (std::getenv("ORYX_LOG_DEBUG"))
    fprintf(stderr, "speed_append total %.3f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count());
  return res;
}

// The aggregated pairs [lo, hi)'s UP messages (same layout as oryx_assemble_als_updates:
// ["X",user,row(,[item])] and ["Y",item,row(,[user])], one per valid side, '\n' after each),
// keys taken from the events' own bytes.  xtext / ytext rows are indexed from lo.  Returns
// bytes, or -(bytes needed).
long long oryx_speed_assemble(void* h, long long lo, long long hi, const char* xtext,
                              const long long* xends, const char* ytext, const long long* yends,
                              const unsigned char* vx, const unsigned char* vy, int with_known,
                              char* out, long long cap, long long* msg_ends, long long* n_msgs) {
  SpeedBatch* b = static_cast<SpeedBatch*>(h);
  const long long n = hi - lo;
  std::vector<long long> bytes((size_t)n + 1, 0), msgs((size_t)n + 1, 0);
  std::vector<std::string> qu((size_t)n), qi((size_t)n);
  oryx_ff::parallel_ranges(n, 256, [&](long long a, long long z, int) {
    for (long long e = a; e < z; ++e) {
      const int64_t r = b->rep[(size_t)(lo + e)];
      json_quote(b->uk[(size_t)r].data(), b->uk[(size_t)r].size(), qu[(size_t)e]);
      json_quote(b->ik[(size_t)r].data(), b->ik[(size_t)r].size(), qi[(size_t)e]);
      const long long lu = (long long)qu[(size_t)e].size(), li = (long long)qi[(size_t)e].size();
      const long long xs = e ? xends[e - 1] : 0, ys = e ? yends[e - 1] : 0;
      long long bb = 0;
      if (vx[e]) bb += 5 + lu + 1 + (xends[e] - xs) + (with_known ? 3 + li : 0) + 2;
      if (vy[e]) bb += 5 + li + 1 + (yends[e] - ys) + (with_known ? 3 + lu : 0) + 2;
      bytes[(size_t)e + 1] = bb;
      msgs[(size_t)e + 1] = (vx[e] ? 1 : 0) + (vy[e] ? 1 : 0);
    }
  });
  for (long long e = 0; e < n; ++e) {
    bytes[(size_t)e + 1] += bytes[(size_t)e];
    msgs[(size_t)e + 1] += msgs[(size_t)e];
  }
  if (bytes[(size_t)n] > cap) return -bytes[(size_t)n];
  oryx_ff::parallel_ranges(n, 256, [&](long long a, long long z, int) {
    for (long long e = a; e < z; ++e) {
      const std::string& su = qu[(size_t)e];
      const std::string& si = qi[(size_t)e];
      char* o = out + bytes[(size_t)e];
      long long m = msgs[(size_t)e];
      auto put = [&](const char* p, size_t len) { std::memcpy(o, p, len); o += len; };
      auto one = [&](const char* kind, const std::string& self, const char* row, size_t rl,
                     const std::string& other) {
        put(kind, 5);
        put(self.data(), self.size());
        *o++ = ',';
        put(row, rl);
        if (with_known) {
          put(",[", 2);
          put(other.data(), other.size());
          *o++ = ']';
        }
        *o++ = ']';
        if (msg_ends) msg_ends[m++] = o - out;
        *o++ = '\n';
      };
      const long long xs = e ? xends[e - 1] : 0, ys = e ? yends[e - 1] : 0;
      if (vx[e]) one("[\"X\",", su, xtext + xs, (size_t)(xends[e] - xs), si);
      if (vy[e]) one("[\"Y\",", si, ytext + ys, (size_t)(yends[e] - ys), su);
    }
  });
  if (n_msgs) *n_msgs = msgs[(size_t)n];
  return bytes[(size_t)n];
}

}  // extern "C"

// ---- k-means speed-layer updates: [clusterID,[center...],count] lines with every double
// written as Python's repr (json.dumps) writes it -- the shortest digits that round-trip,
// fixed notation for decimal exponents -4..15, else d.ddde+XX -- so the native messages are
// byte-identical to text.join_json's ([speed-app]/kmeans/KMeansSpeedModelManager.java:
// 110-124 builds them per touched cluster).

namespace {

// Python repr of a finite double (json.dumps: NaN / Infinity for the others) at o; returns
// the end.
char* write_double_repr(double v, char* o) {
  if (std::isnan(v)) { memcpy(o, "NaN", 3); return o + 3; }
  if (std::isinf(v)) {
    if (v < 0) *o++ = '-';
    memcpy(o, "Infinity", 8);
    return o + 8;
  }
  if (v == 0.0) {
    if (std::signbit(v)) *o++ = '-';
    memcpy(o, "0.0", 3);
    return o + 3;
  }
  char buf[40];
  // shortest round-trip digits in scientific form: [-]d[.ddd]e(+|-)XX
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  const char* p = buf;
  if (*p == '-') { *o++ = '-'; ++p; }
  const char* e = static_cast<const char*>(memchr(p, 'e', (size_t)(r.ptr - p)));
  char digits[24];
  int nd = 0;
  for (const char* q = p; q < e; ++q)
    if (*q != '.') digits[nd++] = *q;
  int exp10 = 0;
  {
    const char* q = e + 1;
    const bool neg = *q == '-';
    if (*q == '+' || *q == '-') ++q;
    std::from_chars(q, r.ptr, exp10);
    if (neg) exp10 = -exp10;
  }
  if (exp10 >= -4 && exp10 < 16) {
    if (exp10 >= 0) {
      for (int j = 0; j <= exp10; ++j) *o++ = j < nd ? digits[j] : '0';
      *o++ = '.';
      if (nd > exp10 + 1) {
        for (int j = exp10 + 1; j < nd; ++j) *o++ = digits[j];
      } else {
        *o++ = '0';
      }
    } else {
      *o++ = '0';
      *o++ = '.';
      for (int j = 0; j < -exp10 - 1; ++j) *o++ = '0';
      for (int j = 0; j < nd; ++j) *o++ = digits[j];
    }
    return o;
  }
  *o++ = digits[0];
  if (nd > 1) {
    *o++ = '.';
    for (int j = 1; j < nd; ++j) *o++ = digits[j];
  }
  *o++ = 'e';
  *o++ = exp10 < 0 ? '-' : '+';
  const int ax = exp10 < 0 ? -exp10 : exp10;
  if (ax < 10) *o++ = '0';
  char eb[8];
  const int el = snprintf(eb, sizeof(eb), "%d", ax);
  memcpy(o, eb, (size_t)el);
  return o + el;
}

}  // namespace

extern "C" {

// The lines of oryx_format_cluster_updates from the centers' texts already formatted into
// 24-byte slots (slots[(j d + f) 24], lens[j d + f]: csrc/kernels/fmt64.hip on the device).
// Returns bytes, or -(bytes needed).
long long oryx_format_cluster_updates_slots(const long long* ids, const char* slots,
                                            const unsigned char* lens, const long long* counts,
                                            long long n, int d, char* out, long long cap,
                                            long long* ends) {
  std::vector<long long> off((size_t)n + 1, 0);
  oryx_ff::parallel_ranges(n, 64, [&](long long lo, long long hi, int) {
    char b[24];
    for (long long j = lo; j < hi; ++j) {
      long long L = 1 + snprintf(b, sizeof(b), "%lld", ids[j]) + 2 + (d > 0 ? d - 1 : 0) + 2 +
                    snprintf(b, sizeof(b), "%lld", counts[j]) + 1;
      const unsigned char* lj = lens + j * d;
      for (int f = 0; f < d; ++f) L += lj[f];
      off[(size_t)j + 1] = L + 1;   // and its '\n'
    }
  });
  for (long long j = 0; j < n; ++j) off[(size_t)j + 1] += off[(size_t)j];
  if (off[(size_t)n] > cap) return -off[(size_t)n];
  oryx_ff::parallel_ranges(n, 64, [&](long long lo, long long hi, int) {
    for (long long j = lo; j < hi; ++j) {
      char* o = out + off[(size_t)j];
      *o++ = '[';
      o += snprintf(o, 24, "%lld", ids[j]);
      *o++ = ',';
      *o++ = '[';
      for (int f = 0; f < d; ++f) {
        if (f) *o++ = ',';
        const long long k = j * d + f;
        memcpy(o, slots + k * 24, lens[k]);
        o += lens[k];
      }
      *o++ = ']';
      *o++ = ',';
      o += snprintf(o, 24, "%lld", counts[j]);
      *o++ = ']';
      ends[j] = (long long)(o - out);
      *o = '\n';
    }
  });
  return off[(size_t)n];
}

// Python repr of v[0..n) into 24-byte slots, lens[j] = the text's length (the reference for
// the device formatter, csrc/kernels/fmt64.hip, and its checks).
void oryx_format_f64_repr_host(const double* v, long long n, char* slots, unsigned char* lens) {
  oryx_ff::parallel_ranges(n, 4096, [&](long long lo, long long hi, int) {
    for (long long j = lo; j < hi; ++j) {
      char* o = slots + j * 24;
      lens[j] = (unsigned char)(write_double_repr(v[j], o) - o);
    }
  });
}

// n lines "[id,[c_0,...,c_{d-1}],count]" ('\n' after each) for the rows of centers [n][d];
// ends[j] = end of line j (before its '\n').  Returns bytes, or -(bytes needed).
long long oryx_format_cluster_updates(const long long* ids, const double* centers,
                                      const long long* counts, long long n, int d, char* out,
                                      long long cap, long long* ends) {
  // a double takes at most 24 characters, an int64 20
  const long long per = 2 + 21 + 2 + (long long)d * 25 + 2 + 21 + 2;
  if (n * per > cap) return -(n * per);
  std::vector<long long> len((size_t)n + 1, 0);
  std::vector<std::string> lines((size_t)n);
  oryx_ff::parallel_ranges(n, 64, [&](long long lo, long long hi, int) {
    for (long long j = lo; j < hi; ++j) {
      std::string& s = lines[(size_t)j];
      s.resize((size_t)per);
      char* o = &s[0];
      *o++ = '[';
      o += snprintf(o, 24, "%lld", ids[j]);
      *o++ = ',';
      *o++ = '[';
      for (int f = 0; f < d; ++f) {
        if (f) *o++ = ',';
        o = write_double_repr(centers[j * d + f], o);
      }
      *o++ = ']';
      *o++ = ',';
      o += snprintf(o, 24, "%lld", counts[j]);
      *o++ = ']';
      s.resize((size_t)(o - &s[0]));
    }
  });
  long long pos = 0;
  for (long long j = 0; j < n; ++j) {
    memcpy(out + pos, lines[(size_t)j].data(), lines[(size_t)j].size());
    pos += (long long)lines[(size_t)j].size();
    ends[j] = pos;
    out[pos++] = '\n';
  }
  return pos;
}

}  // extern "C"

extern "C" {

// RDF speed-layer updates for n touched leaves ([speed-app]/rdf/RDFSpeedModelManager.java:
// 112-151): classification (nc > 0) '[tree,ID,{"c":count,...}]' over the classes with a
// nonzero count (counts [n][nc]), regression (nc == 0) '[tree,ID,mean,count]' (means [n],
// counts [n]); ID = leaf_ids' pre-quoted JSON text of leaf j (idx[j] into the blob).  Lines
// '\n'-separated, ends[j] before the '\n'.  Returns bytes, or -(bytes needed).
long long oryx_format_leaf_updates(long long n, const long long* trees, const char* id_blob,
                                   const long long* id_ends, const long long* idx,
                                   const long long* counts, int nc, const double* means,
                                   char* out, long long cap, long long* ends) {
  long long need = 0;
  for (long long j = 0; j < n; ++j) {
    const long long k = idx[j];
    const long long il = id_ends[k] - (k ? id_ends[k - 1] : 0);
    need += 2 * 21 + il + 8 + (nc > 0 ? (long long)nc * 46 : 24 + 21) + 1;
  }
  if (need > cap) return -need;
  char* o = out;
  for (long long j = 0; j < n; ++j) {
    const long long k = idx[j];
    const long long ib = k ? id_ends[k - 1] : 0;
    *o++ = '[';
    o += snprintf(o, 24, "%lld", trees[j]);
    *o++ = ',';
    memcpy(o, id_blob + ib, (size_t)(id_ends[k] - ib));
    o += id_ends[k] - ib;
    *o++ = ',';
    if (nc > 0) {
      *o++ = '{';
      bool first = true;
      for (int c = 0; c < nc; ++c) {
        const long long v = counts[j * nc + c];
        if (!v) continue;
        if (!first) *o++ = ',';
        first = false;
        o += snprintf(o, 48, "\"%d\":%lld", c, v);
      }
      *o++ = '}';
    } else {
      o = write_double_repr(means[j], o);
      *o++ = ',';
      o += snprintf(o, 24, "%lld", counts[j]);
    }
    *o++ = ']';
    ends[j] = o - out;
    *o++ = '\n';
  }
  return o - out;
}

// Top-N launch inputs of one batch (ops/topn.py ItemIndex._prep) packed into `out` (the
// pinned staging buffer of the single host-to-device copy), sections 16-byte aligned in this
// order: Q [max_batch][kp] fp32 (targets, zero padded), ranges [nr][2] i64 (the union of the
// queries' LSH buckets as merged store-position ranges; the whole store without LSH), tile0
// [nr + 1] i64 (16-row tile prefix), then with LSH per-query bucket bitmaps [nq][words] u32
// (bit b of word b / 32), then with exclusions ptr [nq + 1] i32 and the sorted excluded
// positions ex [max(1, total)] i32.  cand_ptr == nullptr: no LSH; cand_all[j] = 1: query j
// scans every bucket.  ex_ptr == nullptr: no exclusions.  [delta_lo, delta_hi): the index's
// unsorted delta segment of positions (rows added or moved since its last sort), scanned by
// every query after the bucket ranges (the kernel's bucket mask still filters its rows).
// info: n_ranges, n_tiles, and the byte offsets of ranges, tile0, bits, ptr, ex (-1 when
// absent), then the bytes used.  Returns 0, 1 when no range is left to scan, -1 when `out` is
// too small.
long long oryx_topn_prep(int nq, int k, int kp, int max_batch, const float* targets,
                         const long long* cand_ptr, const long long* cand,
                         const unsigned char* cand_all, int num_buckets, int words,
                         const long long* bucket_start, long long n_rows, const long long* ex_ptr,
                         const long long* ex_rows, const long long* pos_of_row, long long n_pos,
                         long long delta_lo, long long delta_hi,
                         unsigned char* out, long long out_cap, long long* info) {
  auto al = [](long long v) { return (v + 15) & ~15LL; };
  std::vector<std::pair<long long, long long>> rs;
  std::vector<uint32_t> bits;
  if (cand_ptr) {
    bits.assign((size_t)nq * (size_t)words, 0u);
    std::vector<unsigned char> any((size_t)num_buckets, 0);
    for (int j = 0; j < nq; ++j) {
      uint32_t* bj = bits.data() + (size_t)j * words;
      if (cand_all && cand_all[j]) {
        for (int b = 0; b < num_buckets; ++b) bj[b >> 5] |= 1u << (b & 31);
        std::fill(any.begin(), any.end(), (unsigned char)1);
        continue;
      }
      for (long long q = cand_ptr[j]; q < cand_ptr[j + 1]; ++q) {
        const long long b = cand[q];
        if (b < 0 || b >= num_buckets) continue;
        bj[b >> 5] |= 1u << (b & 31);
        any[(size_t)b] = 1;
      }
    }
    for (int b = 0; b < num_buckets; ++b) {
      if (!any[(size_t)b]) continue;
      const long long s0 = bucket_start[b], e0 = bucket_start[b + 1];
      if (e0 <= s0) continue;
      if (!rs.empty() && rs.back().second == s0) rs.back().second = e0;
      else rs.emplace_back(s0, e0);
    }
  } else if (n_rows > 0) {
    rs.emplace_back(0, n_rows);
  }
  if (delta_hi > delta_lo) {
    if (!rs.empty() && rs.back().second == delta_lo) rs.back().second = delta_hi;
    else rs.emplace_back(delta_lo, delta_hi);
  }
  if (rs.empty()) return 1;
  const long long nr = (long long)rs.size();
  // excluded rows -> sorted positions per query
  std::vector<int32_t> ptr, ex;
  if (ex_ptr) {
    ptr.assign((size_t)nq + 1, 0);
    std::vector<int32_t> pj;
    for (int j = 0; j < nq; ++j) {
      pj.clear();
      for (long long q = ex_ptr[j]; q < ex_ptr[j + 1]; ++q) {
        const long long r = ex_rows[q];
        if (r < 0 || r >= n_pos) continue;
        const long long p = pos_of_row[r];
        if (p >= 0) pj.push_back((int32_t)p);
      }
      std::sort(pj.begin(), pj.end());
      ex.insert(ex.end(), pj.begin(), pj.end());
      ptr[(size_t)j + 1] = (int32_t)ex.size();
    }
    if (ex.empty()) ex.push_back(0);
  }
  const long long o_q = 0;
  const long long o_rs = al(o_q + (long long)max_batch * kp * 4);
  const long long o_t0 = al(o_rs + nr * 16);
  long long o = al(o_t0 + (nr + 1) * 8);
  const long long o_bits = cand_ptr ? o : -1;
  if (cand_ptr) o = al(o + (long long)bits.size() * 4);
  const long long o_ptr = ex_ptr ? o : -1;
  if (ex_ptr) o = al(o + (long long)ptr.size() * 4);
  const long long o_ex = ex_ptr ? o : -1;
  if (ex_ptr) o = al(o + (long long)ex.size() * 4);
  if (o > out_cap) return -1;
  float* Q = reinterpret_cast<float*>(out + o_q);
  std::memset(Q, 0, (size_t)max_batch * kp * 4);
  for (int j = 0; j < nq; ++j)
    std::memcpy(Q + (size_t)j * kp, targets + (size_t)j * k, (size_t)k * 4);
  long long* R = reinterpret_cast<long long*>(out + o_rs);
  long long* T0 = reinterpret_cast<long long*>(out + o_t0);
  T0[0] = 0;
  for (long long r = 0; r < nr; ++r) {
    R[2 * r] = rs[(size_t)r].first;
    R[2 * r + 1] = rs[(size_t)r].second;
    T0[r + 1] = T0[r] + (rs[(size_t)r].second - rs[(size_t)r].first + 15) / 16;
  }
  if (cand_ptr) std::memcpy(out + o_bits, bits.data(), bits.size() * 4);
  if (ex_ptr) {
    std::memcpy(out + o_ptr, ptr.data(), ptr.size() * 4);
    std::memcpy(out + o_ex, ex.data(), ex.size() * 4);
  }
  info[0] = nr;
  info[1] = T0[nr];
  info[2] = o_rs;
  info[3] = o_t0;
  info[4] = o_bits;
  info[5] = o_ptr;
  info[6] = o_ex;
  info[7] = o;
  info[8] = (long long)ex.size();
  return 0;
}

// 128-bit content digest of a byte range (the identity under which parsed text is cached:
// ALS / feature histories adopt a parse when the same bytes come back as a part file; not
// cryptographic).  4 MB chunks over the native threads, each with a hardware CRC-32C and a
// position-weighted 64-bit sum of its 8-byte words; the per-chunk values are then mixed in
// chunk order with the length.  ~20 GB/s per thread, where a single-threaded xxh3 pass over a
// 29 GB interval took seconds.
__attribute__((target("sse4.2"))) static void digest_chunk(const unsigned char* p, size_t n,
                                                           uint32_t* crc_out,
                                                           uint64_t* sum_out) {
  uint64_t c = 0xFFFFFFFFu, sum = 0, i = 1;
  size_t k = 0;
  for (; k + 8 <= n; k += 8, i += 2) {
    uint64_t v;
    std::memcpy(&v, p + k, 8);
    c = __builtin_ia32_crc32di(c, v);
    sum += v * i;
  }
  uint32_t c32 = (uint32_t)c;
  uint64_t tail = 0;
  for (size_t j = 0; k + j < n; ++j) {
    c32 = __builtin_ia32_crc32qi(c32, p[k + j]);
    tail |= (uint64_t)p[k + j] << (8 * j);
  }
  sum += tail * i;
  *crc_out = ~c32;
  *sum_out = sum;
}

static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oryx_digest128(const unsigned char* p, long long n, unsigned long long* out) {
  constexpr long long kChunk = 4LL << 20;
  const long long nch = n > 0 ? (n + kChunk - 1) / kChunk : 0;
  std::vector<uint32_t> crc((size_t)nch);
  std::vector<uint64_t> sum((size_t)nch);
  oryx_ff::parallel_ranges(nch, 1, [&](long long lo, long long hi, int) {
    for (long long c = lo; c < hi; ++c) {
      const long long o = c * kChunk;
      digest_chunk(p + o, (size_t)std::min(kChunk, n - o), &crc[(size_t)c], &sum[(size_t)c]);
    }
  });
  uint64_t h1 = mix64((uint64_t)n), h2 = mix64((uint64_t)n ^ 0x5851F42D4C957F2Dull);
  for (long long c = 0; c < nch; ++c) {
    h1 = mix64(h1 ^ ((uint64_t)crc[(size_t)c] << 32 | (uint64_t)c));
    h2 = mix64(h2 + sum[(size_t)c]);
  }
  out[0] = h1;
  out[1] = h2;
}

// A 64-bit hash of every key of a blob (key i = bytes [ends[i-1], ends[i])), mixed with
// `seed`: FNV-1a over the bytes, then the splitmix64 finalizer.  The ALS trainer keys its
// random factor initialisation by it, so a row starts from the same vector at any world size.
void oryx_blob_hash64(const unsigned char* blob, const long long* ends, long long n,
                      unsigned long long seed, unsigned long long* out) {
  oryx_ff::parallel_ranges(n, 1 << 14, [&](long long lo, long long hi, int) {
    for (long long i = lo; i < hi; ++i) {
      const long long b = i ? ends[i - 1] : 0;
      uint64_t h = 0xCBF29CE484222325ull ^ seed;
      for (long long j = b; j < ends[i]; ++j) h = (h ^ blob[j]) * 0x100000001B3ull;
      out[i] = mix64(h ^ (uint64_t)(ends[i] - b));
    }
  });
}

}  // extern "C"

extern "C" {

// Categorical codes of n byte spans (span j = base[off[j * stride], + len[j * stride])), in
// order of first appearance, an empty span -1 (missing): the feature apps' encoding of a
// categorical column (RDFUpdate.getDistinctValues, [mllib]/rdf/RDFUpdate.java:207-225, then
// the value -> index maps).  Each thread encodes a contiguous range of rows with a local
// table; the tables are merged in range order, so the numbering is the sequential one.
// first_row[k] = the row where distinct value k first appears.  Returns the number of
// distinct values.
long long oryx_encode_spans(const char* base, const long long* off, const int* len, long long n,
                            long long stride, long long* codes, long long* first_row) {
  if (n <= 0) return 0;
  const int T = oryx_ff::native_threads();
  std::vector<std::unordered_map<std::string_view, long long>> local((size_t)T);
  std::vector<std::vector<long long>> lfirst((size_t)T);
  const int P = oryx_ff::parallel_ranges(n, 1 << 15, [&](long long lo, long long hi, int t) {
    auto& m = local[(size_t)t];
    auto& fr = lfirst[(size_t)t];
    for (long long j = lo; j < hi; ++j) {
      const int l = len[j * stride];
      if (l <= 0) {
        codes[j] = -1;
        continue;
      }
      const std::string_view k(base + off[j * stride], (size_t)l);
      auto it = m.try_emplace(k, (long long)fr.size());
      if (it.second) fr.push_back(j);
      codes[j] = it.first->second;
    }
  });
  // merge in range order: global ids in order of first appearance
  std::unordered_map<std::string_view, long long> global;
  std::vector<std::vector<long long>> remap((size_t)P);
  long long G = 0;
  for (int t = 0; t < P; ++t) {
    remap[(size_t)t].resize(lfirst[(size_t)t].size());
    for (size_t k = 0; k < lfirst[(size_t)t].size(); ++k) {
      const long long j = lfirst[(size_t)t][k];
      const std::string_view key(base + off[j * stride], (size_t)len[j * stride]);
      auto it = global.try_emplace(key, G);
      if (it.second) first_row[G++] = j;
      remap[(size_t)t][k] = it.first->second;
    }
  }
  if (P > 1 || G != (long long)lfirst[0].size()) {
    // (the same n and piece size: the same P ranges as the encoding pass)
    oryx_ff::parallel_ranges(n, 1 << 15, [&](long long lo, long long hi, int t) {
      const auto& rm = remap[(size_t)t];
      for (long long j = lo; j < hi; ++j)
        if (codes[j] >= 0) codes[j] = rm[(size_t)codes[j]];
    });
  }
  return G;
}

}  // extern "C"
