// oryx_ingest.cpp -- native data loading for the batch/speed layers.
//
// The reference parses input lines inside Spark tasks ([app-common]/common/fn/MLFunctions.java:39-65,
// [mllib]/als/ALSUpdate.java:260-290) and maps string IDs to ints by parse-or-MD5-hash with a
// reverse lookup collected to the driver (C4 in SURVEY.md section 2.5).  Here one C++ pass turns a
// buffer of "user,item[,strength[,timestamp]]" lines (or JSON arrays) into dense dictionary
// codes, strengths (NaN = delete) and timestamps, ready to upload as device tensors; the
// dictionaries are collision-free (no hashing of IDs) and persist across intervals.
// Also: shortest-round-trip float formatting of factor rows for JSON update messages.

#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace {

struct Dict {
  std::unordered_map<std::string, int64_t> map;
  std::vector<std::string> keys;
  std::mutex mu;
  int64_t encode(std::string_view s) {
    auto it = map.find(std::string(s));
    if (it != map.end()) return it->second;
    int64_t code = (int64_t)keys.size();
    keys.emplace_back(s);
    map.emplace(keys.back(), code);
    return code;
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

long long oryx_dict_get(void* dh, const char* s, long long len) {
  Dict* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  auto it = d->map.find(std::string(s, (size_t)len));
  return it == d->map.end() ? -1 : it->second;
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

// Parses newline-separated rating lines.  users/items: dictionaries; outputs per parsed row:
// user code, item code, strength (NaN when the field is empty = delete; 1 when missing),
// timestamp (default_ts when missing).  Returns rows parsed, or -(line number + 1) of the
// first malformed line when strict.
long long oryx_parse_ratings(const char* buf, long long len, void* users, void* items,
                             long long* out_u, long long* out_i, double* out_s,
                             long long* out_ts, long long max_rows, long long default_ts,
                             int strict) {
  Dict* du = static_cast<Dict*>(users);
  Dict* di = static_cast<Dict*>(items);
  std::lock_guard<std::mutex> gu(du->mu);
  std::unique_lock<std::mutex> gi(di->mu, std::defer_lock);
  if (di != du) gi.lock();
  const char* p = buf;
  const char* end = buf + len;
  long long rows = 0, line_no = 0;
  std::vector<std::string> toks;
  std::string field;
  while (p < end && rows < max_rows) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', end - p));
    const char* le = nl ? nl : end;
    const char* lend = le;
    if (lend > p && lend[-1] == '\r') --lend;
    if (lend > p) {
      toks.clear();
      if (*p == '[' && lend[-1] == ']') {
        if (!json_fields(p, lend, toks)) toks.clear();
      } else {
        const char* q = p;
        while (true) {
          q = csv_field(q, lend, field);
          toks.push_back(field);
          if (q >= lend) break;
          ++q;  // comma
          if (q >= lend) { toks.emplace_back(); break; }
        }
      }
      bool ok = toks.size() >= 2;
      double s = 1.0;
      long long ts = default_ts;
      if (ok && toks.size() >= 3) {
        if (toks[2].empty()) s = std::numeric_limits<double>::quiet_NaN();
        else ok = parse_double(toks[2], &s);
      }
      if (ok && toks.size() >= 4 && !toks[3].empty()) {
        double t;
        ok = parse_double(toks[3], &t);
        ts = (long long)t;
      }
      if (ok) {
        out_u[rows] = du->encode(toks[0]);
        out_i[rows] = di->encode(toks[1]);
        out_s[rows] = s;
        out_ts[rows] = ts;
        ++rows;
      } else if (strict) {
        return -(line_no + 1);
      }
    }
    ++line_no;
    p = nl ? nl + 1 : end;
  }
  return rows;
}

// Formats rows of a float matrix as JSON arrays "[v0,v1,...]" with shortest round-trip
// float32 text, back to back in out; row_ends[r] = end offset of row r.  Returns bytes used
// or -1 when out is too small.
long long oryx_format_float_rows(const float* mat, long long n, int k, long long stride,
                                 char* out, long long cap, long long* row_ends) {
  long long pos = 0;
  char tmp[32];
  for (long long r = 0; r < n; ++r) {
    const float* row = mat + r * stride;
    if (pos + 2 + (long long)k * 16 > cap) return -1;
    out[pos++] = '[';
    for (int j = 0; j < k; ++j) {
      if (j) out[pos++] = ',';
      float v = row[j];
      if (std::isnan(v)) { memcpy(out + pos, "NaN", 3); pos += 3; continue; }
      if (std::isinf(v)) {
        const char* s = v > 0 ? "Infinity" : "-Infinity";
        size_t l = strlen(s);
        memcpy(out + pos, s, l);
        pos += l;
        continue;
      }
      auto res = std::to_chars(tmp, tmp + sizeof(tmp), v);
      size_t l = res.ptr - tmp;
      // Java-style: always show a decimal point for integral values ("1.0")
      bool has_dot = false;
      for (size_t q = 0; q < l; ++q) if (tmp[q] == '.' || tmp[q] == 'e') { has_dot = true; break; }
      memcpy(out + pos, tmp, l);
      pos += l;
      if (!has_dot) { out[pos++] = '.'; out[pos++] = '0'; }
    }
    out[pos++] = ']';
    row_ends[r] = pos;
  }
  return pos;
}

// All keys from `from` on, back to back in out; ends[j] = end offset of key from + j.
// Returns bytes used, or -(bytes needed) when out is too small.
long long oryx_dict_keys_blob(void* dh, long long from, char* out, long long cap,
                              long long* ends) {
  auto* d = static_cast<Dict*>(dh);
  std::lock_guard<std::mutex> g(d->mu);
  long long need = 0;
  for (size_t c = (size_t)from; c < d->keys.size(); ++c) need += (long long)d->keys[c].size();
  if (need > cap) return -need;
  long long pos = 0;
  for (size_t c = (size_t)from; c < d->keys.size(); ++c) {
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
void json_quote(const std::string& s, std::string& o) {
  static const char* hex = "0123456789abcdef";
  auto u4 = [&](unsigned v) {
    o += "\\u";
    o += hex[(v >> 12) & 15]; o += hex[(v >> 8) & 15]; o += hex[(v >> 4) & 15]; o += hex[v & 15];
  };
  o += '"';
  for (size_t p = 0; p < s.size();) {
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
    for (int q = 1; q <= extra && p + q < s.size(); ++q) cp = (cp << 6) | (s[p + q] & 0x3F);
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

void float_row(const float* row, int k, std::string& o) {
  char tmp[32];
  o += '[';
  for (int j = 0; j < k; ++j) {
    if (j) o += ',';
    float v = row[j];
    if (std::isnan(v)) { o += "NaN"; continue; }
    if (std::isinf(v)) { o += v > 0 ? "Infinity" : "-Infinity"; continue; }
    auto res = std::to_chars(tmp, tmp + sizeof(tmp), v);
    size_t l = res.ptr - tmp;
    bool has_dot = false;
    for (size_t q = 0; q < l; ++q) if (tmp[q] == '.' || tmp[q] == 'e') { has_dot = true; break; }
    o.append(tmp, l);
    if (!has_dot) o += ".0";
  }
  o += ']';
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
}

extern "C" {

// Parses n messages ["X"|"Y", id, [k floats], optional [ids...]] (back to back in buf, ends
// = message end offsets).  kinds[j] = 0 (X) / 1 (Y) / 2 (unparseable: the caller falls back);
// vecs [n][k]; id_ends[j] / known_cnt[j] index the id and known-item texts, fetched with
// oryx_up_texts (ids, then known items, each back to back; known_ends per item).  Returns the
// total number of known items.
long long oryx_parse_up_batch(const char* buf, const long long* ends, long long n, int k,
                              unsigned char* kinds, float* vecs, long long* id_ends,
                              long long* known_cnt) {
  g_up_ids.clear();
  g_up_known.clear();
  std::string tok;
  long long start = 0, total_known = 0;
  for (long long j = 0; j < n; ++j) {
    JsonCursor c{buf + start, buf + ends[j]};
    start = ends[j];
    kinds[j] = 2;
    known_cnt[j] = 0;
    const size_t id_mark = g_up_ids.size(), known_mark = g_up_known.size();
    bool ok = c.eat('[') && c.token(tok) && (tok == "X" || tok == "Y");
    unsigned char kind = ok && tok == "Y" ? 1 : 0;
    ok = ok && c.eat(',') && c.token(tok);
    if (ok) g_up_ids += tok;
    ok = ok && c.eat(',') && c.eat('[');
    float* v = vecs + j * k;
    for (int f = 0; ok && f < k; ++f) {
      if (f && !c.eat(',')) { ok = false; break; }
      c.ws();
      const char* b = c.p;
      while (c.p < c.end && *c.p != ',' && *c.p != ']' && *c.p != ' ') ++c.p;
      auto r = std::from_chars(b, c.p, v[f]);
      if (r.ec != std::errc() || r.ptr != c.p) {
        std::string t(b, c.p - b);   // NaN / Infinity spellings
        if (t == "NaN") v[f] = std::numeric_limits<float>::quiet_NaN();
        else if (t == "Infinity") v[f] = std::numeric_limits<float>::infinity();
        else if (t == "-Infinity") v[f] = -std::numeric_limits<float>::infinity();
        else ok = false;
      }
    }
    ok = ok && c.eat(']');
    long long cnt = 0;
    if (ok && c.eat(',')) {
      ok = c.eat('[');
      if (ok && !c.eat(']')) {
        do {
          if (!c.token(tok)) { ok = false; break; }
          g_up_known += tok;
          g_up_known += '\0';
          ++cnt;
        } while (c.eat(','));
        ok = ok && c.eat(']');
      }
    }
    ok = ok && c.eat(']');
    if (!ok) {
      g_up_ids.resize(id_mark);
      g_up_known.resize(known_mark);
      id_ends[j] = (long long)g_up_ids.size();
      continue;
    }
    kinds[j] = kind;
    id_ends[j] = (long long)g_up_ids.size();
    known_cnt[j] = cnt;
    total_known += cnt;
  }
  return total_known;
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
  std::string o;
  o.reserve((size_t)n * (size_t)(k * 12 + 48));
  std::string qu, qi;
  for (long long e = 0; e < n; ++e) {
    qu.clear();
    qi.clear();
    json_quote(du->keys[(size_t)u[e]], qu);
    json_quote(di->keys[(size_t)i[e]], qi);
    if (vx[e]) {
      o += "[\"X\",";
      o += qu;
      o += ',';
      float_row(nx + e * k, k, o);
      if (with_known) { o += ",["; o += qi; o += ']'; }
      o += "]\n";
    }
    if (vy[e]) {
      o += "[\"Y\",";
      o += qi;
      o += ',';
      float_row(ny + e * k, k, o);
      if (with_known) { o += ",["; o += qu; o += ']'; }
      o += "]\n";
    }
  }
  if ((long long)o.size() > cap) return -(long long)o.size();
  memcpy(out, o.data(), o.size());
  return (long long)o.size();
}

}  // extern "C"
