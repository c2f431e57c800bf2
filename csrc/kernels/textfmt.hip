// textfmt.hip -- factor rows -> JSON text on the GPU.
//
// Every model update the batch and speed layers publish carries factor rows as JSON arrays
// of shortest round-trip floats (ALSUpdate publishAdditionalModelData / ALSSpeedModelManager
// .java:182-215 via TextUtils.joinJSON).  The rows already live in HBM (trainer factors,
// fold-in outputs), and shortest-decimal conversion is ~60 ns per float on a host core, so
// the conversion runs here instead: two launches over one 64-lane wave per row
//   1. fmt_row_len  -- every lane converts its features (lane + 64 j) and the wave sums the
//                      text lengths into row_len[r] ("[" + values + commas + "]");
//   2. fmt_row_text -- after an exclusive scan of row_len (row offsets), the lanes convert
//                      again, place their values with a wave prefix sum and write the bytes.
// Output text is byte-identical to the host formatter (csrc/runtime/fastfloat.h
// write_float_json: std::to_chars plain-mode digits, ".0" on integral values, NaN /
// Infinity spelled out): the same Schubfach conversion with the same 77-entry table of
// 64-bit powers of ten.

#include "common.h"

namespace {

__constant__ unsigned long long kPow10G[77] = {
    0x81CEB32C4B43FCF5ull, 0xA2425FF75E14FC32ull, 0xCAD2F7F5359A3B3Full, 0xFD87B5F28300CA0Eull,
    0x9E74D1B791E07E49ull, 0xC612062576589DDBull, 0xF79687AED3EEC552ull, 0x9ABE14CD44753B53ull,
    0xC16D9A0095928A28ull, 0xF1C90080BAF72CB2ull, 0x971DA05074DA7BEFull, 0xBCE5086492111AEBull,
    0xEC1E4A7DB69561A6ull, 0x9392EE8E921D5D08ull, 0xB877AA3236A4B44Aull, 0xE69594BEC44DE15Cull,
    0x901D7CF73AB0ACDAull, 0xB424DC35095CD810ull, 0xE12E13424BB40E14ull, 0x8CBCCC096F5088CCull,
    0xAFEBFF0BCB24AAFFull, 0xDBE6FECEBDEDD5BFull, 0x89705F4136B4A598ull, 0xABCC77118461CEFDull,
    0xD6BF94D5E57A42BDull, 0x8637BD05AF6C69B6ull, 0xA7C5AC471B478424ull, 0xD1B71758E219652Cull,
    0x83126E978D4FDF3Cull, 0xA3D70A3D70A3D70Bull, 0xCCCCCCCCCCCCCCCDull, 0x8000000000000001ull,
    0xA000000000000001ull, 0xC800000000000001ull, 0xFA00000000000001ull, 0x9C40000000000001ull,
    0xC350000000000001ull, 0xF424000000000001ull, 0x9896800000000001ull, 0xBEBC200000000001ull,
    0xEE6B280000000001ull, 0x9502F90000000001ull, 0xBA43B74000000001ull, 0xE8D4A51000000001ull,
    0x9184E72A00000001ull, 0xB5E620F480000001ull, 0xE35FA931A0000001ull, 0x8E1BC9BF04000001ull,
    0xB1A2BC2EC5000001ull, 0xDE0B6B3A76400001ull, 0x8AC7230489E80001ull, 0xAD78EBC5AC620001ull,
    0xD8D726B7177A8001ull, 0x878678326EAC9001ull, 0xA968163F0A57B401ull, 0xD3C21BCECCEDA101ull,
    0x84595161401484A1ull, 0xA56FA5B99019A5C9ull, 0xCECB8F27F4200F3Bull, 0x813F3978F8940985ull,
    0xA18F07D736B90BE6ull, 0xC9F2C9CD04674EDFull, 0xFC6F7C4045812297ull, 0x9DC5ADA82B70B59Eull,
    0xC5371912364CE306ull, 0xF684DF56C3E01BC7ull, 0x9A130B963A6C115Dull, 0xC097CE7BC90715B4ull,
    0xF0BDC21ABB48DB21ull, 0x96769950B50D88F5ull, 0xBC143FA4E250EB32ull, 0xEB194F8E1AE525FEull,
    0x92EFD1B8D0CF37BFull, 0xB7ABC627050305AEull, 0xE596B7B0C643C71Aull, 0x8F7E32CE7BEA5C70ull,
    0xB35DBF821AE4F38Cull};
constexpr int kPowMin = -31;

__device__ __forceinline__ int floor_log2_pow10(int e) { return (e * 1741647) >> 19; }
__device__ __forceinline__ int floor_log10_pow2(int e) { return (e * 1262611) >> 22; }
__device__ __forceinline__ int floor_log10_tq_pow2(int e) { return (e * 1262611 - 524031) >> 22; }

__device__ __forceinline__ unsigned round_to_odd(unsigned long long g, unsigned cp) {
  const unsigned long long lo = g * (unsigned long long)cp;
  const unsigned long long hi = __umul64hi(g, (unsigned long long)cp);
  return (unsigned)hi | ((unsigned)(lo >> 32) > 1u ? 1u : 0u);
}

// Shortest-then-closest decimal digits * 10^exp of a finite non-zero float (Schubfach).
__device__ void to_decimal(unsigned sig, unsigned ex, unsigned& digits, int& exp10) {
  unsigned c;
  int q;
  if (ex != 0) {
    c = (1u << 23) | sig;
    q = (int)ex - 150;
    if (0 <= -q && -q < 24 && (c & ((1u << -q) - 1u)) == 0) {
      digits = c >> -q;
      exp10 = 0;
      return;
    }
  } else {
    c = sig;
    q = 1 - 150;
  }
  const bool is_even = (c & 1u) == 0;
  const bool lower_closer = sig == 0 && ex > 1;
  const unsigned cbl = 4 * c - 2 + (lower_closer ? 1u : 0u);
  const unsigned cb = 4 * c, cbr = 4 * c + 2;
  const int k = lower_closer ? floor_log10_tq_pow2(q) : floor_log10_pow2(q);
  const int h = q + floor_log2_pow10(-k) + 1;
  const unsigned long long g = kPow10G[-k - kPowMin];
  const unsigned vbl = round_to_odd(g, cbl << h);
  const unsigned vb = round_to_odd(g, cb << h);
  const unsigned vbr = round_to_odd(g, cbr << h);
  const unsigned lower = vbl + (is_even ? 0u : 1u);
  const unsigned upper = vbr - (is_even ? 0u : 1u);
  const unsigned s = vb / 4;
  if (s >= 10) {
    const unsigned sp = s / 10;
    const bool up_in = lower <= 40 * sp, wp_in = 40 * sp + 40 <= upper;
    if (up_in != wp_in) {
      digits = wp_in ? sp + 1 : sp;
      exp10 = k + 1;
      return;
    }
  }
  const bool u_in = lower <= 4 * s, w_in = 4 * s + 4 <= upper;
  if (u_in != w_in) {
    digits = w_in ? s + 1 : s;
    exp10 = k;
    return;
  }
  const unsigned mid = 4 * s + 2;
  const bool up = vb > mid || (vb == mid && (s & 1u) != 0);
  digits = up ? s + 1 : s;
  exp10 = k;
}

__device__ __forceinline__ int dec_len32(unsigned v) {
  int n = 1;
  while (v >= 10u) {
    v /= 10u;
    ++n;
  }
  return n;
}

// The JSON text of v into buf (<= 18 bytes); returns the length.
__device__ int float_json(float v, char* buf) {
  const unsigned bits = __float_as_uint(v);
  const unsigned sig = bits & 0x7FFFFFu, ex = (bits >> 23) & 0xFFu;
  int o = 0;
  if (ex == 0xFFu) {
    const char* s = sig ? "NaN" : (bits >> 31) ? "-Infinity" : "Infinity";
    while (*s) buf[o++] = *s++;
    return o;
  }
  if (bits >> 31) buf[o++] = '-';
  if (ex == 0 && sig == 0) {
    buf[o++] = '0';
    buf[o++] = '.';
    buf[o++] = '0';
    return o;
  }
  unsigned D;
  int k;
  to_decimal(sig, ex, D, k);
  while (D % 10u == 0) {
    D /= 10u;
    ++k;
  }
  const int n = dec_len32(D);
  const int E = n + k - 1;
  const int aE = E < 0 ? -E : E;
  const int sci_len = n + (n > 1 ? 1 : 0) + 2 + (aE >= 100 ? 3 : 2);
  const int fix_len = E >= 0 ? (k >= 0 ? n + k : n + 1) : n + 1 - E;
  if (fix_len <= sci_len) {
    if (E < 0) {
      buf[o++] = '0';
      buf[o++] = '.';
      for (int z = 0; z < -E - 1; ++z) buf[o++] = '0';
      for (int j = n - 1; j >= 0; --j, D /= 10u) buf[o + j] = (char)('0' + D % 10u);
      return o + n;
    }
    if (k >= 0) {
      // integral: the exact value (fixed notation prints it, not padded shortest digits)
      unsigned long long iv = k == 0 ? (unsigned long long)D
                                     : (unsigned long long)(v < 0 ? -v : v);
      int m = 1;
      for (unsigned long long t = iv; t >= 10ull; t /= 10ull) ++m;
      for (int j = m - 1; j >= 0; --j, iv /= 10ull) buf[o + j] = (char)('0' + iv % 10ull);
      o += m;
      buf[o++] = '.';
      buf[o++] = '0';
      return o;
    }
    // dd.ddd
    for (int j = n; j >= 0; --j) {
      if (j == E + 1) {
        buf[o + j] = '.';
        continue;
      }
      buf[o + j] = (char)('0' + D % 10u);
      D /= 10u;
    }
    return o + n + 1;
  }
  // d.ddde+XX
  for (int j = n; j >= 1; --j) {
    if (j == 1) {
      buf[o + 1] = '.';
      continue;
    }
    buf[o + j] = (char)('0' + D % 10u);
    D /= 10u;
  }
  buf[o] = (char)('0' + D);
  o += n > 1 ? n + 1 : 1;
  buf[o++] = 'e';
  buf[o++] = E < 0 ? '-' : '+';
  if (aE >= 100) buf[o++] = (char)('0' + aE / 100);
  buf[o++] = (char)('0' + (aE / 10) % 10);
  buf[o++] = (char)('0' + aE % 10);
  return o;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(v, off, 64);
    if (lane >= off) v += t;
  }
  return v;
}

constexpr int WPB = 4;   // waves (rows) per block

// CSV: the row as "v0,v1,...\n" (the batch layers' input lines) instead of "[v0,v1,...]"
template <bool CSV = false>
__global__ __launch_bounds__(WPB * 64) void fmt_row_len(const float* __restrict__ M,
                                                        long long n, int k, long long ld,
                                                        int* __restrict__ row_len) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (r >= n) return;
  char buf[20];
  int len = 0;
  for (int f = lane; f < k; f += 64) len += float_json(M[r * ld + f], buf);
  len = wave_sum_i(len);
  if (lane == 0) row_len[r] = len + (k > 0 ? k - 1 : 0) + (CSV ? 1 : 2);
}

template <bool CSV = false>
__global__ __launch_bounds__(WPB * 64) void fmt_row_text(const float* __restrict__ M,
                                                         long long n, int k, long long ld,
                                                         const long long* __restrict__ row_end,
                                                         const int* __restrict__ row_len,
                                                         char* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (r >= n) return;
  const long long start = row_end[r] - row_len[r];
  char* o = out + start;
  if (!CSV && lane == 0) o[0] = '[';
  long long base = CSV ? 0 : 1;   // bytes of the row before this chunk of 64 features
  char buf[20];
  for (int f0 = 0; f0 < k; f0 += 64) {
    const int f = f0 + lane;
    int len = 0;
    if (f < k) len = float_json(M[r * ld + f], buf);
    const int with_comma = len + (f < k - 1 ? 1 : 0);
    const int incl = wave_incl_scan(f < k ? with_comma : 0, lane);
    if (f < k) {
      char* p = o + base + (incl - with_comma);
      for (int c = 0; c < len; ++c) p[c] = buf[c];
      if (f < k - 1) p[len] = ',';
    }
    base += __shfl(incl, 63, 64);
  }
  if (lane == 0) o[row_len[r] - 1] = CSV ? '\n' : ']';
}

}  // namespace

extern "C" {

// row_len[r] = bytes of the JSON array text of row r of M [n, k] (leading dimension ld).
int oryx_format_rows_len(const float* M, long long n, int k, long long ld, int* row_len,
                         void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k < 0 || ld < k) return ORYX_EINVAL;
  const unsigned blocks = (unsigned)((n + WPB - 1) / WPB);
  hipLaunchKernelGGL(fmt_row_len<false>, dim3(blocks), dim3(WPB * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), M, n, k, ld, row_len);
  return oryx_check_launch();
}

// Writes the rows' text back to back into out: row r occupies
// [row_end[r] - row_len[r], row_end[r]) (row_end = inclusive scan of row_len).
int oryx_format_rows_text(const float* M, long long n, int k, long long ld,
                          const long long* row_end, const int* row_len, char* out,
                          void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k < 0 || ld < k) return ORYX_EINVAL;
  const unsigned blocks = (unsigned)((n + WPB - 1) / WPB);
  hipLaunchKernelGGL(fmt_row_text<false>, dim3(blocks), dim3(WPB * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), M, n, k, ld, row_end, row_len, out);
  return oryx_check_launch();
}

// As the two calls above with each row as a CSV line "v0,v1,...\n" (row_len includes the
// newline).
int oryx_format_csv_len(const float* M, long long n, int k, long long ld, int* row_len,
                        void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k < 0 || ld < k) return ORYX_EINVAL;
  const unsigned blocks = (unsigned)((n + WPB - 1) / WPB);
  hipLaunchKernelGGL(fmt_row_len<true>, dim3(blocks), dim3(WPB * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), M, n, k, ld, row_len);
  return oryx_check_launch();
}

int oryx_format_csv_text(const float* M, long long n, int k, long long ld,
                         const long long* row_end, const int* row_len, char* out,
                         void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k < 0 || ld < k) return ORYX_EINVAL;
  const unsigned blocks = (unsigned)((n + WPB - 1) / WPB);
  hipLaunchKernelGGL(fmt_row_text<true>, dim3(blocks), dim3(WPB * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), M, n, k, ld, row_end, row_len, out);
  return oryx_check_launch();
}

}  // extern "C"
