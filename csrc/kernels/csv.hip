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

}  // extern "C"
