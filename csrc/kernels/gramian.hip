// gramian.hip -- X^T X of a tall-skinny fp32 factor matrix on fp32 MFMA (split-K).
//
// The ALS half-step needs the Gramian of the opposite factor matrix (YtY for implicit
// feedback; the reference's MLlib computes it per iteration) and the speed layer
// needs X^T X / Y^T Y (K3).  The shape is n x KP with n ~ 1e5..1e7 and KP <= 128: a pure
// K-reduction.  Library GEMMs tile the 64 x 64 output and leave most CUs idle; here every
// wave owns a contiguous slab of rows, the KP x KP product accumulates on
// v_mfma_f32_16x16x4_f32 (A = B = 4 rows x 16 features: a 16-lane group reads 64 contiguous
// bytes of a row, so each load instruction covers 4 full rows), the 4 waves of a workgroup
// combine in LDS in a fixed order, and a second pass sums the per-workgroup partials in a
// fixed order (deterministic, exactly symmetric result).  HBM traffic is one read of X.

#include "common.h"

namespace {

constexpr int GRAM_BLOCKS = 512;

template <int M>  // KP = 16 * M
__global__ __launch_bounds__(256) void gramian_partial(const float* __restrict__ X, long long n,
                                                       int ld, float* __restrict__ part) {
  constexpr int KP = 16 * M;
  constexpr int NT = M * (M + 1) / 2;
  __shared__ float red[KP * KP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < KP * KP; i += 256) red[i] = 0.f;
  __syncthreads();

  const long long waves = (long long)gridDim.x * 4;
  const long long wid = (long long)blockIdx.x * 4 + wave;
  const long long per = ((n + waves - 1) / waves + 3) / 4 * 4;   // rows per wave, mult. of 4
  const long long r0 = wid * per;
  const long long r1 = r0 + per < n ? r0 + per : n;
  const int rsub = lane >> 4, f = lane & 15;

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (long long r = r0; r < r1; r += 4) {
    const long long rr = r + rsub;
    float frag[M];
#pragma unroll
    for (int b = 0; b < M; ++b) frag[b] = rr < r1 ? X[rr * ld + b * 16 + f] : 0.f;
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < M; ++bi)
#pragma unroll
      for (int bj = 0; bj <= bi; ++bj, ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(frag[bi], frag[bj], acc[t], 0, 0, 0);
  }
  // C/D layout of 16x16 f32 MFMA: col = lane & 15, row = 4 * (lane >> 4) + v.  The 4 waves
  // add their lower tiles into LDS one after another (fixed order: deterministic); the upper
  // triangle is mirrored in the final pass (exactly symmetric result).
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < M; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int i = bi * 16 + 4 * rsub + v, j = bj * 16 + f;
            red[i * KP + j] += acc[t][v];
          }
    }
    __syncthreads();
  }
  float* dst = part + (long long)blockIdx.x * KP * KP;
  for (int i = tid; i < KP * KP; i += 256) dst[i] = red[i];
}

// Second pass: 64 output entries per workgroup, 16 waves.  Wave w sums partials w, w+16, ...
// (eight loads in flight per lane, each a coalesced 256-byte run), then wave 0 adds the 16
// wave sums in a fixed order: deterministic, and ~kp*kp/64 workgroups x 16 waves instead of
// kp*kp/256 threads each walking all partials serially (122 us -> a few us at kp=64).
// Only entries with i >= j are reduced (the 16x16 diagonal tiles hold both halves, the
// strictly-upper off-diagonal tiles are zero); each is written to (i, j) and (j, i).
__global__ __launch_bounds__(1024) void gramian_reduce(const float* __restrict__ part, int nblk,
                                                       int kp, float* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int idx = blockIdx.x * 64 + lane;
  const int kk = kp * kp;
  const int src = idx < kk ? idx : 0;
  float s = 0.f;
  int b = wave;
  for (; b + 7 * 16 < nblk; b += 8 * 16) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(long long)(b + u * 16) * kk + src];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; b < nblk; b += 16) s += part[(long long)b * kk + src];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && idx < kk) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    const int i = idx / kp, j = idx % kp;
    if (i >= j) {
      out[idx] = t;
      if (i != j) out[j * kp + i] = t;
    }
  }
}

}  // namespace

extern "C" {

// X fp32 [n][ld] (first kp columns used, kp % 16 == 0, kp <= 128); out fp32 [kp][kp];
// ws: oryx_gramian_ws_floats(kp) floats of scratch.
int oryx_gramian_ws_floats(int kp) { return GRAM_BLOCKS * kp * kp; }

int oryx_gramian_f32(const float* X, long long n, int ld, int kp, float* out, float* ws,
                     void* stream) {
  if (kp % 16 || kp <= 0 || kp > 128 || ld < kp) return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  long long blocks = (n + 4 * 64 - 1) / (4 * 64);   // >= 64 rows per wave
  if (blocks > GRAM_BLOCKS) blocks = GRAM_BLOCKS;
  if (blocks < 1) blocks = 1;
  switch (kp / 16) {
#define GRAM_CASE(MV)                                                                    \
  case MV:                                                                               \
    hipLaunchKernelGGL(gramian_partial<MV>, dim3((unsigned)blocks), dim3(256), 0, s, X, n, \
                       ld, ws);                                                          \
    break;
    GRAM_CASE(1)
    GRAM_CASE(2)
    GRAM_CASE(3)
    GRAM_CASE(4)
    GRAM_CASE(5)
    GRAM_CASE(6)
    GRAM_CASE(7)
    GRAM_CASE(8)
#undef GRAM_CASE
    default:
      return ORYX_EINVAL;
  }
  hipLaunchKernelGGL(gramian_reduce, dim3((kp * kp + 63) / 64), dim3(1024), 0, s, ws,
                     (int)blocks, kp, out);
  return oryx_check_launch();
}

}  // extern "C"
