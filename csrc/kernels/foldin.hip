// foldin.hip -- the ALS speed layer's fold-in of new interactions, fused.
//
// For every aggregated event (user u, item i, strength v) both factor rows are updated as
// ALSUtils.computeUpdatedXu does it ([app-common]/als/ALSUtils.java:37-106, driven per event
// at [speed-app]/als/ALSSpeedModelManager.java:182-204):
//   Qui   = Xu . Yi            (float products, double sum; 0 when Xu is absent)
//   t     = targetQui(implicit, v, Xu ? Qui : 0.5)        (NaN: no update)
//   dXu   = (YtY)^-1 float(Yi * (t - Qui))                (double solve, float result)
//   Xu'   = Xu + dXu   (or dXu when Xu is absent); no update when Yi is absent
// and symmetrically Yi' from Xu with (XtX)^-1.  One 64-lane wave per (event, side): lanes own
// features (lane + 64 j), the dot product is a wave reduction in double, the target is
// computed once and broadcast, the right-hand side goes through LDS and each lane forms its
// rows of inv * rhs in double.  One launch replaces the dozen tensor ops of the unfused path
// and reads the factor rows straight from the device mirrors by row index.

#include "common.h"

namespace {

constexpr int FW = 4;   // waves per block

__device__ __forceinline__ double target_qui(int implicit, double value, double current) {
  if (!implicit) return value;
  if (value > 0.0 && current < 1.0) {
    const double diff = 1.0 - (current > 0.0 ? current : 0.0);
    return current + (value / (1.0 + value)) * diff;
  }
  if (value < 0.0 && current > 0.0) {
    const double diff = -(current < 1.0 ? current : 1.0);
    return current + (value / (value - 1.0)) * diff;
  }
  return __builtin_nan("");
}

template <int KW>   // features per lane (k <= 64 * KW)
__global__ __launch_bounds__(FW * 64) void als_foldin(
    const float* __restrict__ X, const float* __restrict__ Y, int k,
    const long long* __restrict__ xrow, const long long* __restrict__ yrow,
    const float* __restrict__ vals, const double* __restrict__ xinv,
    const double* __restrict__ yinv, int implicit, long long n, float* __restrict__ new_x,
    float* __restrict__ new_y, unsigned char* __restrict__ vx, unsigned char* __restrict__ vy) {
  __shared__ double s_rhs[FW][64 * KW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long w = (long long)blockIdx.x * FW + wave;
  if (w >= 2 * n) return;
  const long long e = w >> 1;
  const bool side_x = (w & 1) == 0;          // side X: update Xu from Yi with (YtY)^-1
  const long long r_self = side_x ? xrow[e] : yrow[e];
  const long long r_other = side_x ? yrow[e] : xrow[e];
  const float* M_self = side_x ? X : Y;
  const float* M_other = side_x ? Y : X;
  const double* inv = side_x ? yinv : xinv;
  float* out = (side_x ? new_x : new_y) + e * k;
  unsigned char* valid = side_x ? vx : vy;
  if (r_other < 0) {                         // Yi absent: computeUpdatedXu returns null
    if (lane == 0) valid[e] = 0;
    return;
  }
  float xs[KW], yo[KW];
  double part = 0.0;
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int f = lane + 64 * j;
    xs[j] = (f < k && r_self >= 0) ? M_self[r_self * k + f] : 0.f;
    yo[j] = f < k ? M_other[r_other * k + f] : 0.f;
    part += (double)(xs[j] * yo[j]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
  const double qui = r_self >= 0 ? part : 0.0;
  const double tgt = target_qui(implicit, (double)vals[e], r_self >= 0 ? qui : 0.5);
  if (tgt != tgt) {
    if (lane == 0) valid[e] = 0;
    return;
  }
  const double dq = tgt - qui;
  double* rhs = s_rhs[wave];
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int f = lane + 64 * j;
    // Java: dQuiYi[i] *= dQui -- float times double, stored as float
    rhs[f] = f < k ? (double)(float)((double)yo[j] * dq) : 0.0;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int f = lane + 64 * j;
    if (f < k) {
      const double* row = inv + (long long)f * k;
      double acc = 0.0;
      for (int g = 0; g < k; ++g) acc += row[g] * rhs[g];
      const float dx = (float)acc;
      out[f] = r_self >= 0 ? xs[j] + dx : dx;
    }
  }
  if (lane == 0) valid[e] = 1;
}

}  // namespace

extern "C" {

// X [*, k], Y [*, k] fp32 (the speed model's device mirrors); xrow / yrow [n] (-1 = absent);
// vals [n]; xinv / yinv [k][k] fp64 inverses of XtX / YtY; outputs new_x / new_y [n][k],
// vx / vy [n] (1 = an update row was produced).  k <= 256.
int oryx_als_foldin(const float* X, const float* Y, int k, const long long* xrow,
                    const long long* yrow, const float* vals, const double* xinv,
                    const double* yinv, int implicit, long long n, float* new_x, float* new_y,
                    unsigned char* vx, unsigned char* vy, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k <= 0 || k > 256) return ORYX_EINVAL;
  const unsigned blocks = (unsigned)((2 * n + FW - 1) / FW);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define FOLD(KWV)                                                                         \
  hipLaunchKernelGGL(als_foldin<KWV>, dim3(blocks), dim3(FW * 64), 0, s, X, Y, k, xrow, yrow, \
                     vals, xinv, yinv, implicit, n, new_x, new_y, vx, vy)
  if (k <= 64) FOLD(1);
  else if (k <= 128) FOLD(2);
  else FOLD(4);
#undef FOLD
  return oryx_check_launch();
}

}  // extern "C"
