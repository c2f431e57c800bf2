// csv.hip -- numeric CSV lines to a feature matrix on the GPU (the k-means / RDF batch layers'
// parse of millions of feature rows; SURVEY.md section 2: KMeansUpdate / RDFUpdate parse every
// record into vectors, [mllib]/kmeans/KMeansUpdate.java:223-232).
//
// The host parser (csrc/runtime/oryx_ingest.cpp csv_to_matrix) writes a [rows][F] float64
// matrix to host memory that is then copied to the device and freed: at 12.5M x 256 that is a
// 25.6 GB host array (page faults, then a 25.6 GB copy, then a 25.6 GB free).  Here the text
// itself goes to the device (smaller than its parse) and one thread per line parses it there,
// with the host parser's exact fast path: up to 19 significant digits, a decimal exponent
// within +-22, mantissa <= 2^53 -> one correctly rounded double operation (Clinger's fast
// path), then cast to the output type like the host's (T)v.  An empty field is NaN.  A line in
// any other form (17-digit mantissas past 2^53, other exponents, quotes, escapes, JSON arrays,
// a field count other than F, an empty line) is flagged in bad[line] and counted in *n_bad;
// the caller parses just those lines on the host and writes their rows in, so the matrix is
// bitwise the host parser's.
//
// Non-numeric (categorical) fields are not parsed here: their byte spans go to span_off /
// span_len ([rows][S], offsets into the buffer, in field order) and the host encodes them
// (np.unique over the spans' bytes, as for its own parse), writing the codes into the matrix.
//
// Bytes are read as aligned 16-byte words (the device buffer is padded by 16 bytes), one word
// per 16 characters of the thread's line.
#include "common.h"

namespace {

__constant__ double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

struct ByteReader {
  const uint4* base;
  long long word = -1;
  uint4 w;
  __device__ __forceinline__ int at(long long pos) {
    const long long wi = pos >> 4;
    if (wi != word) {
      w = base[wi];
      word = wi;
    }
    const int k = (int)(pos & 15);
    const unsigned u = k < 4 ? w.x : k < 8 ? w.y : k < 12 ? w.z : w.w;
    return (int)((u >> (8 * (k & 3))) & 0xFFu);
  }
};

template <typename T>
__global__ __launch_bounds__(256) void csv_lines_kernel(const uint4* __restrict__ buf,
                                                        const long long* __restrict__ starts,
                                                        const long long* __restrict__ ends,
                                                        long long n, int F,
                                                        const unsigned char* __restrict__ is_num,
                                                        const int* __restrict__ out_col, int P,
                                                        T* __restrict__ out,
                                                        long long* __restrict__ span_off,
                                                        int* __restrict__ span_len, int S,
                                                        unsigned char* __restrict__ bad,
                                                        int* n_bad) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    ByteReader rd{buf};
    long long p = starts[i];
    long long le = ends[i];
    if (le > p && rd.at(le - 1) == '\r') --le;
    // (a JSON array line starts with '[': the host parser takes it, so it is flagged here)
    bool ok = le > p && rd.at(p) != '[';
    T* o = out + i * P;
    int f = 0, si = 0;
    while (ok) {
      // one field starting at p
      int c = p < le ? rd.at(p) : ',';
      if (f < F && !is_num[f]) {   // categorical: its span, NaN in the matrix for now
        const long long q0 = p;
        while (p < le && c != ',' && c != '"' && c != '\\') {
          ++p;
          c = p < le ? rd.at(p) : ',';
        }
        if (c == '"' || c == '\\' || si >= S) { ok = false; break; }
        span_off[i * S + si] = q0;
        span_len[i * S + si] = (int)(p - q0);
        ++si;
        if (out_col[f] >= 0) o[out_col[f]] = (T)__builtin_nan("");
      } else if (c == ',') {   // empty field: NaN
        if (f >= F) { ok = false; break; }
        if (out_col[f] >= 0) o[out_col[f]] = (T)__builtin_nan("");
      } else {
        bool neg = false;
        if (c == '-' || c == '+') {
          neg = c == '-';
          ++p;
          c = p < le ? rd.at(p) : ',';
        }
        unsigned long long D = 0;
        int nd = 0, frac = 0;
        while ((unsigned)(c - '0') < 10u) {
          D = D * 10 + (unsigned long long)(c - '0');
          ++nd;
          ++p;
          c = p < le ? rd.at(p) : ',';
        }
        if (c == '.') {
          ++p;
          c = p < le ? rd.at(p) : ',';
          while ((unsigned)(c - '0') < 10u) {
            D = D * 10 + (unsigned long long)(c - '0');
            ++nd;
            ++frac;
            ++p;
            c = p < le ? rd.at(p) : ',';
          }
        }
        if (nd == 0 || nd > 19) { ok = false; break; }
        int e10 = -frac;
        if (c == 'e' || c == 'E') {
          ++p;
          c = p < le ? rd.at(p) : ',';
          bool eneg = false;
          if (c == '-' || c == '+') {
            eneg = c == '-';
            ++p;
            c = p < le ? rd.at(p) : ',';
          }
          int x = 0, ne = 0;
          while ((unsigned)(c - '0') < 10u && ne < 4) {
            x = x * 10 + (c - '0');
            ++ne;
            ++p;
            c = p < le ? rd.at(p) : ',';
          }
          if (!ne) { ok = false; break; }
          e10 += eneg ? -x : x;
        }
        if (c != ',' || f >= F || D > (1ull << 53) || e10 < -22 || e10 > 22) {
          ok = false;
          break;
        }
        const double v = e10 < 0 ? (double)D / kP10[-e10] : (double)D * kP10[e10];
        if (out_col[f] >= 0) o[out_col[f]] = (T)(neg ? -v : v);
      }
      ++f;
      if (p >= le) break;   // the line ended with this field
      ++p;                  // past the comma
      if (p >= le) {        // a trailing comma: one more (empty) field
        if (f >= F) { ok = false; break; }
        if (!is_num[f]) {
          if (si >= S) { ok = false; break; }
          span_off[i * S + si] = p;
          span_len[i * S + si] = 0;
          ++si;
        }
        if (out_col[f] >= 0) o[out_col[f]] = (T)__builtin_nan("");
        ++f;
        break;
      }
    }
    const bool b = !ok || f != F;
    bad[i] = b ? 1 : 0;
    if (b) atomicAdd(n_bad, 1);
  }
}

// Wide numeric lines (k-means / RDF rows of hundreds of features, ~2.6 KB at 256 dims): one
// WAVE per line instead of one thread.  A thread walking a 2.6 KB line issues ~160 dependent
// 16-byte loads, and a 10k-line speed-layer micro-batch fills 157 waves of a 1024-SIMD chip:
// 1.4 ms for 26 MB (profiles/r6_km_speed_prof_v1.json).  Here the wave copies its line into LDS
// with coalesced 16-byte loads, each lane counts the commas of a 1/64 slice, a wave prefix sum
// numbers the fields, and every lane parses the fields that start in its slice -- with the
// thread kernel's exact number rules (same fast path, same flags), so the matrix is bitwise
// the host parser's; a categorical field's span goes to span_off / span_len (slot
// span_slot[f]) and NaN to the matrix, as above.  A line longer than kWideLineCap, or with
// quotes, escapes, a leading '[' or a field count other than F is flagged for the host.
constexpr int kWideLineCap = 12288;

// the wave's LDS writes visible to its other lanes (LDS operations of one wave stay in order;
// this keeps the compiler from moving them across)
__device__ __forceinline__ void csv_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// the staged line is read through an LDS-address-space pointer (ds_read_u8): through a
// generic pointer every byte was a flat load waiting on both counters
typedef __attribute__((address_space(3))) const unsigned char lds_u8;

// one numeric field of the staged line s[0, L) starting at q (the thread kernel's rules); the
// value in *v, false when the field is not in the fast-path form
__device__ __forceinline__ bool wide_field(const lds_u8* s, int q, int L, double* v) {
  auto at = [&](int k) -> int { return k < L ? (int)s[k] : ','; };
  int c = at(q);
  if (c == ',') {   // empty field: NaN
    *v = __builtin_nan("");
    return true;
  }
  bool neg = false;
  if (c == '-' || c == '+') {
    neg = c == '-';
    c = at(++q);
  }
  unsigned long long D = 0;
  int nd = 0, frac = 0;
  while ((unsigned)(c - '0') < 10u) {
    D = D * 10 + (unsigned long long)(c - '0');
    ++nd;
    c = at(++q);
  }
  if (c == '.') {
    c = at(++q);
    while ((unsigned)(c - '0') < 10u) {
      D = D * 10 + (unsigned long long)(c - '0');
      ++nd;
      ++frac;
      c = at(++q);
    }
  }
  if (nd == 0 || nd > 19) return false;
  int e10 = -frac;
  if (c == 'e' || c == 'E') {
    c = at(++q);
    bool eneg = false;
    if (c == '-' || c == '+') {
      eneg = c == '-';
      c = at(++q);
    }
    int x = 0, ne = 0;
    while ((unsigned)(c - '0') < 10u && ne < 4) {
      x = x * 10 + (c - '0');
      ++ne;
      c = at(++q);
    }
    if (!ne) return false;
    e10 += eneg ? -x : x;
  }
  if (c != ',' || D > (1ull << 53) || e10 < -22 || e10 > 22) return false;
  const double r = e10 < 0 ? (double)D / kP10[-e10] : (double)D * kP10[e10];
  *v = neg ? -r : r;
  return true;
}

template <typename T>
__global__ __launch_bounds__(256) void csv_wide_kernel(const uint4* __restrict__ buf,
                                                       const long long* __restrict__ starts,
                                                       const long long* __restrict__ ends,
                                                       long long n, int F,
                                                       const int* __restrict__ out_col, int P,
                                                       T* __restrict__ out,
                                                       const int* __restrict__ span_slot,
                                                       long long* __restrict__ span_off,
                                                       int* __restrict__ span_len, int S,
                                                       unsigned char* __restrict__ bad,
                                                       int* n_bad) {
  __shared__ uint4 sm[4][kWideLineCap / 16 + 1];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const lds_u8* lb = (const lds_u8*)sm[w];
  for (long long i = (long long)blockIdx.x * 4 + w; i < n; i += (long long)gridDim.x * 4) {
    const long long p0 = starts[i];
    const int skew = (int)(p0 & 15);
    const long long len = ends[i] - p0;
    bool ok = len > 0 && len + skew <= kWideLineCap;
    int L = ok ? (int)len : 0;
    csv_wave_sync();   // the previous line's reads of this wave's LDS are done
    if (ok) {
      const long long w0 = p0 >> 4;
      const int nw = (skew + L + 15) >> 4;
      for (int j = lane; j < nw; j += 64) sm[w][j] = buf[w0 + j];
    }
    csv_wave_sync();
    const lds_u8* s = lb + skew;
    if (ok && s[L - 1] == '\r') --L;
    ok = ok && L > 0 && s[0] != '[';
    bool lane_ok = true;
    int fields = 0;
    if (ok) {
      const int slice = (L + 63) >> 6;
      const int a = min(lane * slice, L), b = min(a + slice, L);
      int commas = 0;
      for (int q = a; q < b; ++q) {
        const int c = s[q];
        commas += c == ',';
        lane_ok &= c != '"' && c != '\\';
      }
      const int incl = wave_incl_scan(commas, lane);
      fields = __shfl(incl, 63, 64) + 1;
      if (fields == F) {
        T* o = out + i * P;
        // field f starting at q: a number, or a categorical span (NaN in the matrix)
        auto field = [&](int f, int q) {
          double v;
          const int slot = span_slot[f];
          if (slot >= 0) {
            int e = q;
            while (e < L && s[e] != ',') ++e;
            span_off[i * S + slot] = p0 + q;
            span_len[i * S + slot] = e - q;
            v = __builtin_nan("");
          } else {
            lane_ok &= wide_field(s, q, L, &v);
          }
          if (out_col[f] >= 0) o[out_col[f]] = (T)v;
        };
        // the lanes take their fields in lockstep -- each round every lane finds its next
        // field start (field 0 at the line's start for lane 0, else the byte after its next
        // comma) and then they all parse at once: parsing inside the comma scan ran the
        // parser once per byte position at which ANY lane met a comma (~40 passes per line
        // instead of ~5)
        int f = incl - commas;        // commas before this slice
        int q = a;
        bool at0 = lane == 0;
        for (;;) {
          int start = -1;
          if (at0) {
            start = 0;
            at0 = false;
          } else {
            while (q < b && s[q] != ',') ++q;
            if (q < b) {
              start = ++q;            // field f + 1 starts after this comma
              ++f;
            }
          }
          if (__ballot(start >= 0) == 0) break;
          if (start >= 0) field(f, start);   // (lane 0's first round: f = 0, the line start)
        }
      }
    }
    const bool b = !ok || fields != F || __ballot(!lane_ok) != 0;
    if (lane == 0) {
      bad[i] = b ? 1 : 0;
      if (b) atomicAdd(n_bad, 1);
    }
  }
}

// ALS rating lines "user,item[,strength[,timestamp]]" (ALSUpdate.parsedToRatingRDD,
// [mllib]/als/ALSUpdate.java:260-290) on the GPU: one thread per line, the host parser's plain
// CSV fast path (csrc/runtime/oryx_ingest.cpp parse_rating_fields) for lines whose user and
// item IDs are canonical decimal keys below 2^24 (the dense-array keys of the host
// dictionaries, numeric_key) -- out_u / out_i get the key VALUES (the caller numbers them in
// first-appearance order, as the host dictionaries do).  Strength: 1 without the field, NaN
// when it is empty, else the fast-path double (bitwise the host's); timestamp: default_ts
// without the field or when it is empty, else up to 18 plain digits.  Fields past the fourth
// are ignored, as on the host.  Any other line (an empty one, quotes, escapes, a JSON array,
// a non-canonical key, another number form) is flagged in bad[] / *n_bad: the caller then
// parses the whole range on the host.
__device__ __forceinline__ bool rating_key(ByteReader& rd, long long& p, long long le, int& c,
                                           int* v) {
  // canonical decimal: 1..8 digits, no leading zero unless the key is "0", below 2^24
  const long long q0 = p;
  unsigned x = 0;
  while ((unsigned)(c - '0') < 10u) {
    x = x * 10 + (unsigned)(c - '0');
    ++p;
    c = p < le ? rd.at(p) : ',';
    if (p - q0 > 8) return false;
  }
  const long long nd = p - q0;
  if (nd == 0 || c != ',' || x >= (1u << 24)) return false;
  if (nd > 1 && rd.at(q0) == '0') return false;
  *v = (int)x;
  return true;
}

__global__ __launch_bounds__(256) void rating_lines_kernel(
    const uint4* __restrict__ buf, const long long* __restrict__ starts,
    const long long* __restrict__ ends, long long n, long long default_ts,
    int* __restrict__ out_u, int* __restrict__ out_i, double* __restrict__ out_s,
    long long* __restrict__ out_ts, unsigned char* __restrict__ bad, int* n_bad) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    ByteReader rd{buf};
    long long p = starts[i];
    long long le = ends[i];
    if (le > p && rd.at(le - 1) == '\r') --le;
    bool ok = le > p && rd.at(p) != '[';
    // the host's fast path needs a line without quotes or backslashes anywhere
    for (long long q = p; ok && q < le; ++q) {
      const int ch = rd.at(q);
      ok = ch != '"' && ch != '\\';
    }
    int uv = 0, iv = 0;
    double sv = 1.0;
    long long tv = default_ts;
    int c = ok ? rd.at(p) : 0;
    ok = ok && rating_key(rd, p, le, c, &uv);
    if (ok) {
      if (p >= le) {
        ok = false;                          // no item field
      } else {
        ++p;
        c = p < le ? rd.at(p) : ',';
        ok = rating_key(rd, p, le, c, &iv);
      }
    }
    if (ok && p < le) {
      // strength: the third field
      ++p;
      c = p < le ? rd.at(p) : ',';
      if (c == ',') {
        sv = __builtin_nan("");
      } else {
        bool neg = false;
        if (c == '-' || c == '+') {
          neg = c == '-';
          ++p;
          c = p < le ? rd.at(p) : ',';
        }
        unsigned long long D = 0;
        int nd = 0, frac = 0;
        while ((unsigned)(c - '0') < 10u) {
          D = D * 10 + (unsigned long long)(c - '0');
          ++nd;
          ++p;
          c = p < le ? rd.at(p) : ',';
        }
        if (c == '.') {
          ++p;
          c = p < le ? rd.at(p) : ',';
          while ((unsigned)(c - '0') < 10u) {
            D = D * 10 + (unsigned long long)(c - '0');
            ++nd;
            ++frac;
            ++p;
            c = p < le ? rd.at(p) : ',';
          }
        }
        int e10 = -frac;
        if (nd > 0 && (c == 'e' || c == 'E')) {
          ++p;
          c = p < le ? rd.at(p) : ',';
          bool eneg = false;
          if (c == '-' || c == '+') {
            eneg = c == '-';
            ++p;
            c = p < le ? rd.at(p) : ',';
          }
          int x = 0, ne = 0;
          while ((unsigned)(c - '0') < 10u && ne < 4) {
            x = x * 10 + (c - '0');
            ++ne;
            ++p;
            c = p < le ? rd.at(p) : ',';
          }
          if (!ne) nd = 0;
          e10 += eneg ? -x : x;
        }
        ok = nd > 0 && nd <= 19 && c == ',' && D <= (1ull << 53) && e10 >= -22 && e10 <= 22;
        if (ok) {
          const double v = e10 < 0 ? (double)D / kP10[-e10] : (double)D * kP10[e10];
          sv = neg ? -v : v;
        }
      }
      if (ok && p < le) {
        // timestamp: the fourth field (up to the next comma; later fields are ignored)
        ++p;
        c = p < le ? rd.at(p) : ',';
        long long t = 0;
        int nd = 0;
        while ((unsigned)(c - '0') < 10u && nd < 18) {
          t = t * 10 + (c - '0');
          ++nd;
          ++p;
          c = p < le ? rd.at(p) : ',';
        }
        if (c != ',') ok = false;            // another number form: the host parses it
        else if (nd > 0) tv = t;
      }
    }
    out_u[i] = uv;
    out_i[i] = iv;
    out_s[i] = sv;
    out_ts[i] = tv;
    bad[i] = ok ? 0 : 1;
    if (!ok) atomicAdd(n_bad, 1);
  }
}

}  // namespace

extern "C" {

// buf: the lines' bytes on the device, padded to a multiple of 16 plus 16; starts / ends: each
// line's first byte and its '\n' (device int64, n lines); is_num[F]: numeric fields (the others
// are categorical: spans in span_off / span_len [n][S], S of them); out: [n][P] (f64 when
// is_f64, else f32); bad[n]: 1 for each line not in the fast-path form, *n_bad (zeroed by the
// caller) their count.
int oryx_csv_lines_to_matrix(const void* buf, const long long* starts, const long long* ends,
                             long long n, int F, const unsigned char* is_num,
                             const int* out_col, int P, void* out, int is_f64,
                             long long* span_off, int* span_len, int S, unsigned char* bad,
                             int* n_bad, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (F <= 0 || P <= 0 || (reinterpret_cast<uintptr_t>(buf) & 15)) return ORYX_EINVAL;
  long long blocks = (n + 255) / 256;
  if (blocks > 256LL * 64) blocks = 256LL * 64;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (is_f64)
    hipLaunchKernelGGL(csv_lines_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const uint4*>(buf), starts, ends, n, F, is_num, out_col, P,
                       static_cast<double*>(out), span_off, span_len, S, bad, n_bad);
  else
    hipLaunchKernelGGL(csv_lines_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const uint4*>(buf), starts, ends, n, F, is_num, out_col, P,
                       static_cast<float*>(out), span_off, span_len, S, bad, n_bad);
  return oryx_check_launch();
}

// Wide lines (see csv_wide_kernel): arguments as oryx_csv_lines_to_matrix, with span_slot[F]
// (the span column of each categorical field, -1 for numeric ones) in place of is_num.
int oryx_csv_wide_lines_to_matrix(const void* buf, const long long* starts,
                                  const long long* ends, long long n, int F, const int* out_col,
                                  int P, void* out, int is_f64, const int* span_slot,
                                  long long* span_off, int* span_len, int S, unsigned char* bad,
                                  int* n_bad, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (F <= 0 || P <= 0 || (reinterpret_cast<uintptr_t>(buf) & 15)) return ORYX_EINVAL;
  long long blocks = (n + 3) / 4;
  if (blocks > 256LL * 64) blocks = 256LL * 64;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (is_f64)
    hipLaunchKernelGGL(csv_wide_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const uint4*>(buf), starts, ends, n, F, out_col, P,
                       static_cast<double*>(out), span_slot, span_off, span_len, S, bad, n_bad);
  else
    hipLaunchKernelGGL(csv_wide_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const uint4*>(buf), starts, ends, n, F, out_col, P,
                       static_cast<float*>(out), span_slot, span_off, span_len, S, bad, n_bad);
  return oryx_check_launch();
}

// Rating lines (see rating_lines_kernel): buf padded as for oryx_csv_lines_to_matrix; per line
// the user / item key values, strength, timestamp; bad[n] / *n_bad (zeroed by the caller).
int oryx_rating_lines(const void* buf, const long long* starts, const long long* ends,
                      long long n, long long default_ts, int* out_u, int* out_i, double* out_s,
                      long long* out_ts, unsigned char* bad, int* n_bad, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (reinterpret_cast<uintptr_t>(buf) & 15) return ORYX_EINVAL;
  long long blocks = (n + 255) / 256;
  if (blocks > 256LL * 64) blocks = 256LL * 64;
  hipLaunchKernelGGL(rating_lines_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const uint4*>(buf),
                     starts, ends, n, default_ts, out_u, out_i, out_s, out_ts, bad, n_bad);
  return oryx_check_launch();
}

}  // extern "C"
