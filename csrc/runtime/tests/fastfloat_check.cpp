// Checks oryx_ff::write_float against std::to_chars (plain mode) and oryx_ff::parse_float
// against std::from_chars: every float of a strided sweep over all 2^32 bit patterns, random
// patterns, the boundaries of every binade, and random decimal strings.  Prints "ok N" or the
// first mismatch.
#include <charconv>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "../fastfloat.h"

static bool check_bits(uint32_t bits, long long& n) {
  float v;
  std::memcpy(&v, &bits, 4);
  if (((bits >> 23) & 0xFF) == 0xFF) return true;
  char a[64], b[64];
  auto r = std::to_chars(a, a + 64, v);
  *r.ptr = 0;
  char* e = oryx_ff::write_float(v, b);
  *e = 0;
  if (std::strcmp(a, b) != 0) {
    std::printf("format mismatch bits=%08x to_chars=%s ours=%s\n", bits, a, b);
    return false;
  }
  float p = 0;
  if (!oryx_ff::parse_float(b, e, p) || std::memcmp(&p, &v, 4) != 0) {
    std::printf("parse mismatch %s\n", b);
    return false;
  }
  ++n;
  return true;
}

int main(int argc, char** argv) {
  const long long stride = argc > 1 ? std::atoll(argv[1]) : 997;
  long long n = 0;
  for (unsigned long long x = 0; x < (1ull << 32); x += stride)
    if (!check_bits((uint32_t)x, n)) return 1;
  std::mt19937_64 g(7);
  for (int t = 0; t < 2000000; ++t)
    if (!check_bits((uint32_t)g(), n)) return 1;
  for (uint32_t ex = 0; ex < 255; ++ex)
    for (uint32_t s : {0u, 1u, 2u, 0x7FFFFEu, 0x7FFFFFu, 0x400000u})
      for (uint32_t sign : {0u, 1u})
        if (!check_bits((sign << 31) | (ex << 23) | s, n)) return 1;
  // decimal strings of up to 20 digits with exponents: parse vs from_chars
  std::uniform_int_distribution<int> nd(1, 20), ex(-50, 40), dg(0, 9);
  for (int t = 0; t < 3000000; ++t) {
    std::string s;
    if (t & 1) s += '-';
    const int len = nd(g), dot = std::uniform_int_distribution<int>(0, len)(g);
    for (int i = 0; i < len; ++i) {
      if (i == dot && i) s += '.';
      s += (char)('0' + dg(g));
    }
    if (t % 3) s += "e" + std::to_string(ex(g));
    float a = 0, b = 0;
    auto r = std::from_chars(s.data(), s.data() + s.size(), a);
    const bool ok = oryx_ff::parse_float(s.data(), s.data() + s.size(), b);
    if (r.ec == std::errc::result_out_of_range) continue;
    if (!ok || r.ec != std::errc() || std::memcmp(&a, &b, 4) != 0) {
      std::printf("string parse mismatch %s from_chars=%.9g ours=%.9g ok=%d\n", s.c_str(), a, b,
                  (int)ok);
      return 1;
    }
    ++n;
  }
  std::printf("ok %lld\n", n);
  return 0;
}
