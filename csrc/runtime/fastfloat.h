// fastfloat.h -- float32 <-> shortest decimal text for the model-update messages, plus a
// small thread fan-out helper for the bulk text loops of the runtime.
//
// Every factor row the batch / speed layers publish ("UP" messages, [lambda]/... ALSUpdate's
// publishAdditionalModelData and ALSSpeedModelManager.java:182-215) is k floats of JSON text,
// and every serving / speed replica parses all of them back on load.  At 20M x 250 that is
// 5e9 floats each way, so both directions are hand-written here:
//
// * write_float: the shortest decimal that rounds back to the float (Schubfach, R. Giulietti:
//   one 64x32-bit multiply per bound with a 77-entry table of 64-bit powers of ten built at
//   load time from exact big-integer arithmetic), printed exactly like std::to_chars' plain
//   mode (fixed or scientific, whichever is shorter, fixed on a tie).  libstdc++ 11's
//   to_chars takes ~70 ns per float; this ~15.
// * parse_float: Clinger's fast path in double (<= 19 significant digits, |exp10| <= 22: one
//   correctly rounded multiply or divide), then double -> float, which is exact unless the
//   double lands exactly on a float midpoint (then, and for anything else, std::from_chars).

#pragma once

#include <unistd.h>

#include <atomic>
#include <charconv>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace oryx_ff {

constexpr int kPowMin = -31, kPowMax = 45;

inline int floor_log2_pow10(int e) { return (e * 1741647) >> 19; }
inline int floor_log10_pow2(int e) { return (e * 1262611) >> 22; }
inline int floor_log10_three_quarters_pow2(int e) { return (e * 1262611 - 524031) >> 22; }

// g(e) = floor(10^e * 2^(63 - floor(log2 10^e))) + 1, in [2^63, 2^64)
struct Pow10Table {
  uint64_t g[kPowMax - kPowMin + 1];
  Pow10Table() {
    for (int e = kPowMin; e <= kPowMax; ++e) {
      std::vector<uint32_t> x;   // little-endian base 2^32
      if (e >= 0) {
        x.push_back(1);
        for (int i = 0; i < e; ++i) mul_small(x, 10);
        g[e - kPowMin] = top64(x, 64 - bitlen(x)) + 1;
      } else {
        const int n = 63 - floor_log2_pow10(e);
        x.assign((size_t)n / 32 + 1, 0);
        x[(size_t)n / 32] = 1u << (n % 32);
        for (int i = 0; i < -e; ++i) div_small(x, 10);
        g[e - kPowMin] = top64(x, 0) + 1;
      }
    }
  }
  static void mul_small(std::vector<uint32_t>& x, uint32_t m) {
    uint64_t carry = 0;
    for (auto& w : x) {
      const uint64_t t = (uint64_t)w * m + carry;
      w = (uint32_t)t;
      carry = t >> 32;
    }
    if (carry) x.push_back((uint32_t)carry);
  }
  static void div_small(std::vector<uint32_t>& x, uint32_t d) {
    uint64_t rem = 0;
    for (size_t i = x.size(); i-- > 0;) {
      const uint64_t cur = (rem << 32) | x[i];
      x[i] = (uint32_t)(cur / d);
      rem = cur % d;
    }
    while (x.size() > 1 && x.back() == 0) x.pop_back();
  }
  static int bitlen(const std::vector<uint32_t>& x) {
    return (int)(x.size() - 1) * 32 + (32 - __builtin_clz(x.back()));
  }
  // floor(x * 2^shift) as 64 bits (shift may be negative); the caller knows it fits
  static uint64_t top64(const std::vector<uint32_t>& x, int shift) {
    uint64_t r = 0;
    const int len = bitlen(x);
    for (int b = len - 1; b >= 0; --b) {
      const int dst = b + shift;
      if (dst < 0) break;
      if ((x[(size_t)b / 32] >> (b % 32)) & 1u) r |= 1ull << dst;
    }
    return r;
  }
};

inline const Pow10Table& pow10_table() {
  static const Pow10Table t;
  return t;
}

inline uint32_t round_to_odd(uint64_t g, uint32_t cp) {
  const unsigned __int128 p = (unsigned __int128)g * cp;
  const uint32_t y1 = (uint32_t)(p >> 64);
  const uint32_t y0 = (uint32_t)(p >> 32);
  return y1 | (y0 > 1);
}

struct Decimal {
  uint32_t digits;
  int exponent;
};

// Shortest (then closest) decimal in the rounding interval of a finite, non-zero float.
inline Decimal to_decimal(uint32_t ieee_significand, uint32_t ieee_exponent) {
  uint32_t c;
  int q;
  if (ieee_exponent != 0) {
    c = (1u << 23) | ieee_significand;
    q = (int)ieee_exponent - 150;
    if (0 <= -q && -q < 24 && (c & ((1u << -q) - 1)) == 0) return {c >> -q, 0};
  } else {
    c = ieee_significand;
    q = 1 - 150;
  }
  const bool is_even = (c % 2) == 0;
  const bool lower_closer = ieee_significand == 0 && ieee_exponent > 1;
  const uint32_t cbl = 4 * c - 2 + (lower_closer ? 1 : 0);
  const uint32_t cb = 4 * c;
  const uint32_t cbr = 4 * c + 2;
  const int k = lower_closer ? floor_log10_three_quarters_pow2(q) : floor_log10_pow2(q);
  const int h = q + floor_log2_pow10(-k) + 1;
  const uint64_t pow10 = pow10_table().g[-k - kPowMin];
  const uint32_t vbl = round_to_odd(pow10, cbl << h);
  const uint32_t vb = round_to_odd(pow10, cb << h);
  const uint32_t vbr = round_to_odd(pow10, cbr << h);
  const uint32_t lower = vbl + (is_even ? 0 : 1);
  const uint32_t upper = vbr - (is_even ? 0 : 1);
  const uint32_t s = vb / 4;
  if (s >= 10) {
    const uint32_t sp = s / 10;
    const bool up_inside = lower <= 40 * sp;
    const bool wp_inside = 40 * sp + 40 <= upper;
    if (up_inside != wp_inside) return {wp_inside ? sp + 1 : sp, k + 1};
  }
  const bool u_inside = lower <= 4 * s;
  const bool w_inside = 4 * s + 4 <= upper;
  if (u_inside != w_inside) return {w_inside ? s + 1 : s, k};
  const uint32_t mid = 4 * s + 2;
  const bool round_up = vb > mid || (vb == mid && (s & 1) != 0);
  return {round_up ? s + 1 : s, k};
}

inline int decimal_length(uint32_t v) {
  return v >= 100000000u ? 9 : v >= 10000000u ? 8 : v >= 1000000u ? 7 : v >= 100000u ? 6
       : v >= 10000u ? 5 : v >= 1000u ? 4 : v >= 100u ? 3 : v >= 10u ? 2 : 1;
}

// writes the n decimal digits of D ending at o + n
inline void put_digits(char* o, uint32_t D, int n) {
  static const char kPairs[201] =
      "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
      "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
      "8081828384858687888990919293949596979899";
  char* p = o + n;
  while (D >= 100) {
    const uint32_t r = D % 100;
    D /= 100;
    p -= 2;
    std::memcpy(p, kPairs + 2 * r, 2);
  }
  if (D >= 10) {
    p -= 2;
    std::memcpy(p, kPairs + 2 * D, 2);
  } else {
    *--p = (char)('0' + D);
  }
}

// std::to_chars(first, last, v) text for a finite float (at most 15 bytes); returns the end.
// *plain (optional) is set when the text has neither '.' nor an exponent.
inline char* write_float(float v, char* o, bool* plain = nullptr) {
  uint32_t bits;
  std::memcpy(&bits, &v, 4);
  const uint32_t sig = bits & 0x7FFFFFu, exp = (bits >> 23) & 0xFFu;
  if (bits >> 31) *o++ = '-';
  if (exp == 0 && sig == 0) {
    *o++ = '0';
    if (plain) *plain = true;
    return o;
  }
  Decimal d = to_decimal(sig, exp);
  uint32_t D = d.digits;
  int k = d.exponent;
  while (D % 10 == 0) {
    D /= 10;
    ++k;
  }
  const int n = decimal_length(D);
  const int E = n + k - 1;   // scientific exponent
  const int aE = E < 0 ? -E : E;
  const int sci_len = n + (n > 1 ? 1 : 0) + 2 + (aE >= 100 ? 3 : 2);
  const int fix_len = E >= 0 ? (k >= 0 ? n + k : n + 1) : n + 1 - E;
  if (plain) *plain = fix_len <= sci_len && k >= 0;
  if (fix_len <= sci_len) {
    if (E < 0) {            // 0.000ddd
      *o++ = '0';
      *o++ = '.';
      for (int z = 0; z < -E - 1; ++z) *o++ = '0';
      put_digits(o, D, n);
      return o + n;
    }
    if (k > 0) {
      // fixed notation of an integral float prints its exact value (as printf's %.0f
      // would), not the shortest digits padded with zeros; fixed wins only below ~1e13 here
      uint64_t iv = (uint64_t)(v < 0 ? -v : v);
      char t[24];
      int m = 0;
      for (; iv; iv /= 10) t[m++] = (char)('0' + iv % 10);
      while (m) *o++ = t[--m];
      return o;
    }
    if (k == 0) {
      put_digits(o, D, n);
      return o + n;
    }
    // ddd.ddd: write the digits one slot right, then move the integer part left over the
    // point's slot
    put_digits(o + 1, D, n);
    for (int j = 0; j <= E; ++j) o[j] = o[j + 1];
    o[E + 1] = '.';
    return o + n + 1;
  }
  put_digits(o + 1, D, n);
  o[0] = o[1];
  if (n > 1) {
    o[1] = '.';
    o += n + 1;
  } else {
    o += 1;
  }
  *o++ = 'e';
  *o++ = E < 0 ? '-' : '+';
  if (aE >= 100) *o++ = (char)('0' + aE / 100);
  *o++ = (char)('0' + (aE / 10) % 10);
  *o++ = (char)('0' + aE % 10);
  return o;
}

// The JSON spelling of a factor value (Java-like: integral values keep ".0"; NaN / Infinity
// spelled out); at most 17 bytes.
inline char* write_float_json(float v, char* o) {
  uint32_t bits;
  std::memcpy(&bits, &v, 4);
  if (((bits >> 23) & 0xFFu) == 0xFFu) {
    const char* s = (bits & 0x7FFFFFu) ? "NaN" : (bits >> 31) ? "-Infinity" : "Infinity";
    const size_t l = std::strlen(s);
    std::memcpy(o, s, l);
    return o + l;
  }
  bool plain;
  o = write_float(v, o, &plain);
  if (plain) {
    *o++ = '.';
    *o++ = '0';
  }
  return o;
}

inline bool is_8digits(uint64_t x) {
  return (((x & 0xF0F0F0F0F0F0F0F0ull) |
           (((x + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) >> 4)) ==
          0x3333333333333333ull);
}

inline uint32_t parse_8digits(uint64_t x) {   // little-endian load of 8 ASCII digits
  const uint64_t mask = 0x000000FF000000FFull;
  const uint64_t mul1 = 0x000F424000000064ull;   // 100 + (1000000 << 32)
  const uint64_t mul2 = 0x0000271000000001ull;   // 1 + (10000 << 32)
  x -= 0x3030303030303030ull;
  x = (x * 10) + (x >> 8);
  x = (((x & mask) * mul1) + (((x >> 16) & mask) * mul2)) >> 32;
  return (uint32_t)x;
}

// Parses the number starting at b (not past e) as a float; *stop receives the first byte
// after it.  PREFIX = false: the number must span all of [b, e).  False when there is no
// number (NaN / Infinity spellings are the caller's).
template <bool PREFIX>
inline bool parse_float_impl(const char* b, const char* e, float& out, const char** stop) {
  static const double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  const char* p = b;
  bool neg = false;
  if (p < e && *p == '-') {
    neg = true;
    ++p;
  }
  uint64_t D = 0;
  int nd = 0, exp10 = 0;
  bool any = false, fallback = false;
  for (; p < e && (unsigned)(*p - '0') < 10u; ++p) {
    any = true;
    const unsigned dgt = (unsigned)(*p - '0');
    if (D == 0 && dgt == 0) continue;
    if (nd < 19) {
      D = D * 10 + dgt;
      ++nd;
    } else {
      ++exp10;
      if (dgt) fallback = true;
    }
  }
  if (p < e && *p == '.') {
    ++p;
    if (D != 0 && nd + 8 <= 19) {
      // the common case: the digits after the point in blocks of 8
      while (e - p >= 8 && nd + 8 <= 19) {
        uint64_t blk;
        std::memcpy(&blk, p, 8);
        if (!is_8digits(blk)) break;
        D = D * 100000000ull + parse_8digits(blk);
        nd += 8;
        exp10 -= 8;
        p += 8;
      }
    }
    for (; p < e && (unsigned)(*p - '0') < 10u; ++p) {
      any = true;
      const unsigned dgt = (unsigned)(*p - '0');
      if (D == 0 && dgt == 0) {
        --exp10;
        continue;
      }
      if (nd < 19) {
        D = D * 10 + dgt;
        ++nd;
        --exp10;
      } else if (dgt) {
        fallback = true;
      }
    }
  }
  if (!any) return false;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '-' || *p == '+')) eneg = *p++ == '-';
    if (p >= e || (unsigned)(*p - '0') >= 10u) return false;
    int x = 0;
    for (; p < e && (unsigned)(*p - '0') < 10u; ++p)
      if (x < 100000) x = x * 10 + (*p - '0');
    exp10 += eneg ? -x : x;
  }
  if (!PREFIX && p != e) return false;
  *stop = p;
  if (D == 0) {
    out = neg ? -0.0f : 0.0f;
    return true;
  }
  if (!fallback && D <= (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
    double x = (double)D;
    x = exp10 < 0 ? x / kP10[-exp10] : x * kP10[exp10];
    uint64_t xb;
    std::memcpy(&xb, &x, 8);
    // x is a normal float magnitude here; a double exactly on a float midpoint could round
    // differently than the decimal itself would
    if ((xb & ((1ull << 29) - 1)) != (1ull << 28)) {
      out = (float)(neg ? -x : x);
      return true;
    }
  }
  auto r = std::from_chars(b, p, out);
  return r.ec == std::errc() && r.ptr == p;
}

inline bool parse_float(const char* b, const char* e, float& out) {
  const char* stop;
  return parse_float_impl<false>(b, e, out, &stop);
}

// The number at the start of [b, e) (JSON array elements: the caller checks the delimiter
// at *stop) -- one pass instead of a delimiter scan followed by parse_float.
inline bool parse_float_prefix(const char* b, const char* e, float& out, const char** stop) {
  return parse_float_impl<true>(b, e, out, stop);
}

// Parses [b, e) as a double: exact fast path for <= 19 significant digits, a mantissa that
// fits 53 bits and |exp10| <= 22 (one correctly rounded operation), else std::from_chars.
// Leading '+' and spaces are accepted (CSV strengths / timestamps).
inline bool parse_double(const char* b, const char* e, double& out) {
  static const double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  while (b < e && (*b == ' ' || *b == '+')) ++b;
  const char* p = b;
  bool neg = false;
  if (p < e && *p == '-') {
    neg = true;
    ++p;
  }
  uint64_t D = 0;
  int nd = 0, exp10 = 0;
  bool any = false, slow = false;
  for (; p < e && (unsigned)(*p - '0') < 10u; ++p) {
    any = true;
    const unsigned dgt = (unsigned)(*p - '0');
    if (D == 0 && dgt == 0) continue;
    if (nd < 19) { D = D * 10 + dgt; ++nd; } else { ++exp10; if (dgt) slow = true; }
  }
  if (p < e && *p == '.') {
    ++p;
    for (; p < e && (unsigned)(*p - '0') < 10u; ++p) {
      any = true;
      const unsigned dgt = (unsigned)(*p - '0');
      if (D == 0 && dgt == 0) { --exp10; continue; }
      if (nd < 19) { D = D * 10 + dgt; ++nd; --exp10; } else if (dgt) slow = true;
    }
  }
  if (!any) slow = true;
  if (!slow && p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '-' || *p == '+')) eneg = *p++ == '-';
    if (p >= e || (unsigned)(*p - '0') >= 10u) {
      slow = true;
    } else {
      int x = 0;
      for (; p < e && (unsigned)(*p - '0') < 10u; ++p)
        if (x < 100000) x = x * 10 + (*p - '0');
      exp10 += eneg ? -x : x;
    }
  }
  if (!slow && p == e && D <= (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
    double x = (double)D;
    x = exp10 < 0 ? x / kP10[-exp10] : x * kP10[exp10];
    out = neg ? -x : x;
    return true;
  }
  auto r = std::from_chars(b, e, out);
  return r.ec == std::errc() && r.ptr == e;
}

// Threads for the bulk text loops: ORYX_NATIVE_THREADS, else the hardware threads, at most 16.
inline int native_threads() {
  static const int n = [] {
    const char* s = std::getenv("ORYX_NATIVE_THREADS");
    int v = s ? std::atoi(s) : (int)std::thread::hardware_concurrency();
    if (v < 1) v = 1;
    return v > 16 ? 16 : v;
  }();
  return n;
}

// Persistent worker threads for parallel_ranges (native_threads() - 1 of them, started on
// first use): a speed-layer micro-batch runs several parallel loops of ~0.1 ms each, where
// creating and joining fresh threads per loop cost about as much as the work.  Tasks are
// queued; a caller waiting for its own tasks runs queued ones meanwhile, so nested and
// concurrent calls (the speed layer's writer thread beside the main thread) cannot deadlock.
// A forked child (pid differs) starts a pool of its own.
struct ThreadPool {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  std::atomic<int> queued{0};

  explicit ThreadPool(int workers) {
    for (int w = 0; w < workers; ++w)
      std::thread([this] {
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> l(mu);
            cv.wait(l, [&] { return !q.empty(); });
            f = std::move(q.front());
            q.pop_front();
            queued.fetch_sub(1, std::memory_order_relaxed);
          }
          f();
        }
      }).detach();
  }

  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(std::move(f));
      queued.fetch_add(1, std::memory_order_relaxed);
    }
    cv.notify_one();
  }

  bool run_one() {
    if (queued.load(std::memory_order_relaxed) == 0) return false;
    std::function<void()> f;
    {
      std::lock_guard<std::mutex> g(mu);
      if (q.empty()) return false;
      f = std::move(q.front());
      q.pop_front();
      queued.fetch_sub(1, std::memory_order_relaxed);
    }
    f();
    return true;
  }
};

inline ThreadPool& thread_pool() {
  static std::mutex mu;
  static ThreadPool* pool = nullptr;   // never destroyed: its workers are detached
  static long pid = 0;
  std::lock_guard<std::mutex> g(mu);
  if (!pool || pid != (long)getpid()) {
    pool = new ThreadPool(native_threads() - 1);
    pid = (long)getpid();
  }
  return *pool;
}

// Runs fn(lo, hi, part) over `parts` contiguous ranges of [0, n) (part 0 on the caller's
// thread, the rest on the pool); parts = min(threads, n / min_per_part), at least 1.
// Returns parts.
template <class Fn>
int parallel_ranges(long long n, long long min_per_part, Fn&& fn) {
  long long parts = min_per_part > 0 ? n / min_per_part : n;
  if (parts > native_threads()) parts = native_threads();
  if (parts < 1) parts = 1;
  const int P = (int)parts;
  if (P == 1) {
    fn(0LL, n, 0);
    return 1;
  }
  ThreadPool& pool = thread_pool();
  std::atomic<int> left(P - 1);
  for (int t = 1; t < P; ++t)
    pool.push([&, t] {
      fn(n * t / P, n * (t + 1) / P, t);
      left.fetch_sub(1, std::memory_order_acq_rel);
    });
  fn(0LL, n / P, 0);
  while (left.load(std::memory_order_acquire) > 0)
    if (!pool.run_one()) std::this_thread::yield();
  return P;
}

}  // namespace oryx_ff
