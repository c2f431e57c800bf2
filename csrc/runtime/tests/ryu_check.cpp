// ryu_check.cpp -- the device double formatter's algorithm (csrc/kernels/ryu_d2s.h, compiled
// here for the host) against the runtime's formatter (oryx_format_f64_repr_host:
// std::to_chars digits in Python repr layout), byte for byte, over classes of doubles that
// reach every branch: random bit patterns (all exponents, subnormals), integers below and
// above 2^53, short decimals, powers of two and ten, values next to them, halfway cases, and
// running means like the k-means speed layer's.
//
//   g++ -O2 -std=c++17 -I csrc/kernels csrc/runtime/tests/ryu_check.cpp \
//       -L oryx_amd/_native -loryx_runtime -Wl,-rpath,$PWD/oryx_amd/_native -o /tmp/ryu_check
//   /tmp/ryu_check [millions of random values, default 20]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ryu_d2s.h"

extern "C" void oryx_format_f64_repr_host(const double* v, long long n, char* slots,
                                          unsigned char* lens);

static long long g_bad = 0;

static void check(const std::vector<double>& v, const char* what) {
  const long long n = (long long)v.size();
  std::vector<char> slots((size_t)n * 24);
  std::vector<unsigned char> lens((size_t)n);
  oryx_format_f64_repr_host(v.data(), n, slots.data(), lens.data());
  long long bad = 0;
  for (long long j = 0; j < n; ++j) {
    char o[32];
    const int l = oryx_ryu::repr(v[(size_t)j], o);
    if (l != lens[(size_t)j] || memcmp(o, slots.data() + j * 24, (size_t)l) != 0) {
      if (bad < 5)
        fprintf(stderr, "%s: %.17g: ryu '%.*s' host '%.*s'\n", what, v[(size_t)j], l, o,
                (int)lens[(size_t)j], slots.data() + j * 24);
      ++bad;
    }
  }
  printf("%-28s %10lld values, %lld mismatches\n", what, n, bad);
  g_bad += bad;
}

int main(int argc, char** argv) {
  const long long millions = argc > 1 ? atoll(argv[1]) : 20;
  std::mt19937_64 g(12345);
  std::vector<double> v;
  // random bit patterns: every exponent, subnormals, NaN / Inf
  for (long long r = 0; r < millions; ++r) {
    v.clear();
    for (int j = 0; j < 1000000; ++j) {
      const uint64_t b = g();
      double d;
      memcpy(&d, &b, 8);
      v.push_back(d);
    }
    check(v, "random bits");
  }
  // integers, small and large, and their neighbours
  v.clear();
  for (long long j = 0; j < 2000000; ++j) {
    const double d = (double)(int64_t)(g() >> (g() % 64));
    v.push_back(d);
    v.push_back(-d);
    v.push_back(std::nextafter(d, INFINITY));
    v.push_back(std::nextafter(d, -INFINITY));
  }
  check(v, "integers and neighbours");
  // short decimals: k / 10^p, and powers of two / ten with their neighbours
  v.clear();
  for (int p = 0; p < 20; ++p)
    for (int k = 0; k < 100000; ++k) v.push_back((double)k / std::pow(10.0, p));
  for (int e = -1074; e <= 1023; ++e) {
    const double d = std::ldexp(1.0, e);
    v.push_back(d);
    v.push_back(std::nextafter(d, INFINITY));
    v.push_back(std::nextafter(d, 0.0));
  }
  for (int e = -323; e <= 308; ++e) {
    const double d = std::pow(10.0, e);
    v.push_back(d);
    v.push_back(std::nextafter(d, INFINITY));
    v.push_back(std::nextafter(d, 0.0));
    v.push_back(5.0 * d);
    v.push_back(2.5 * d);
  }
  check(v, "decimals, powers");
  // halfway-ish values: k + 0.5 ulp patterns, small mantissas at every exponent
  v.clear();
  for (int e = -1074; e <= 971; e += 1)
    for (int k = 1; k < 200; ++k) v.push_back(std::ldexp((double)k, e));
  check(v, "small mantissas");
  // running means (the k-means speed layer's centers)
  v.clear();
  std::normal_distribution<double> nd(0.0, 3.0);
  for (int j = 0; j < 2000000; ++j) {
    const double c = nd(g), mean = nd(g);
    const double n1 = 1 + (double)(g() % 1000), n0 = 1 + (double)(g() % 100000);
    v.push_back(c + n1 / (n0 + n1) * (mean - c));
  }
  check(v, "running means");
  printf("%s\n", g_bad ? "MISMATCHES" : "all equal");
  return g_bad ? 1 : 0;
}
