// kmeans_speed.hip -- the k-means speed layer's nearest-center search, exact fp64.
//
// KMeansSpeedModelManager.buildUpdates ([speed-app]/kmeans/KMeansSpeedModelManager.java:
// 88-125) assigns every point of a micro-batch to its closest cluster by Euclidean distance
// (KMeansUtils.closestCluster: squared differences summed in double, first strictly smaller
// distance wins).  Here one launch does a whole micro-batch: a 256-thread block holds PT
// points in LDS and each thread runs through the clusters c = tid, tid + 256, ... reading the
// centers from a feature-major copy (C^T [d][k]: consecutive threads read consecutive
// centers, one coalesced line per feature); the per-point minimum is then reduced over the
// block with the lowest index winning ties, as the sequential scan picks it.

#include "common.h"

namespace {

constexpr int KS_THREADS = 256;
constexpr int PT = 16;            // points per block
constexpr int FU = 16;            // features whose center values load together

__global__ __launch_bounds__(KS_THREADS) void km_nearest_f64(
    const double* __restrict__ X, long long n, int d, const double* __restrict__ CT, int k,
    long long* __restrict__ out_idx, double* __restrict__ out_dist) {
  extern __shared__ __attribute__((aligned(16))) double xs[];      // [PT][d]
  __shared__ double rbest[KS_THREADS / 64][PT];
  __shared__ int ridx[KS_THREADS / 64][PT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long p0 = (long long)blockIdx.x * PT;
  for (int i = tid; i < PT * d; i += KS_THREADS) {
    const int r = i / d, f = i - r * d;
    xs[i] = p0 + r < n ? X[(p0 + r) * d + f] : 0.0;
  }
  __syncthreads();
  double best[PT];
  int bi[PT];
#pragma unroll
  for (int r = 0; r < PT; ++r) {
    best[r] = INFINITY;
    bi[r] = 0x7fffffff;
  }
  for (int c = tid; c < k; c += KS_THREADS) {
    double acc[PT];
#pragma unroll
    for (int r = 0; r < PT; ++r) acc[r] = 0.0;
    // FU features' center values are loaded before they are used: one load in flight per
    // thread left the kernel waiting on L2 latency (586 us for 10k points x 1000 centers x
    // 256 dims, profiles/r6_km_speed_kernel_stats_v1.txt).  The sums still run over the
    // features in order (the host scan's rounding).
    const double* cp = CT + c;
    int f0 = 0;
    for (; f0 + FU <= d; f0 += FU) {
      double cv[FU];
#pragma unroll
      for (int u = 0; u < FU; ++u) cv[u] = cp[(long long)(f0 + u) * k];
#pragma unroll
      for (int u = 0; u < FU; ++u)
#pragma unroll
        for (int r = 0; r < PT; ++r) {
          const double df = xs[r * d + f0 + u] - cv[u];
          acc[r] += df * df;
        }
    }
    for (int f = f0; f < d; ++f) {
      const double cv = cp[(long long)f * k];
#pragma unroll
      for (int r = 0; r < PT; ++r) {
        const double df = xs[r * d + f] - cv;
        acc[r] += df * df;
      }
    }
#pragma unroll
    for (int r = 0; r < PT; ++r)
      if (acc[r] < best[r]) {      // c grows: the first strictly smaller one wins
        best[r] = acc[r];
        bi[r] = c;
      }
  }
  // block argmin per point, ties to the lower cluster index
#pragma unroll
  for (int r = 0; r < PT; ++r) {
    double b = best[r];
    int i = bi[r];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ob = __shfl_xor(b, off, 64);
      const int oi = __shfl_xor(i, off, 64);
      if (ob < b || (ob == b && oi < i)) {
        b = ob;
        i = oi;
      }
    }
    if (lane == 0) {
      rbest[wave][r] = b;
      ridx[wave][r] = i;
    }
  }
  __syncthreads();
  if (tid < PT && p0 + tid < n) {
    double b = rbest[0][tid];
    int i = ridx[0][tid];
    for (int w = 1; w < KS_THREADS / 64; ++w) {
      const double ob = rbest[w][tid];
      const int oi = ridx[w][tid];
      if (ob < b || (ob == b && oi < i)) {
        b = ob;
        i = oi;
      }
    }
    out_idx[p0 + tid] = i;
    out_dist[p0 + tid] = sqrt(b);
  }
}

}  // namespace

extern "C" {

// X [n][d] fp64 points, CT [d][k] fp64 centers feature-major; out_idx [n] (cluster position),
// out_dist [n] (Euclidean distance).  d <= 1024 (PT points of d doubles in LDS).
int oryx_kmeans_nearest_f64(const double* X, long long n, int d, const double* CT, int k,
                            long long* out_idx, double* out_dist, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (d <= 0 || d > 1024 || k <= 0) return ORYX_EINVAL;
  const int lds = PT * d * (int)sizeof(double);
  if (lds > 64 * 1024 && !oryx_set_max_lds(&km_nearest_f64, lds)) return ORYX_ELAUNCH;
  const unsigned blocks = (unsigned)((n + PT - 1) / PT);
  hipLaunchKernelGGL(km_nearest_f64, dim3(blocks), dim3(KS_THREADS), lds,
                     reinterpret_cast<hipStream_t>(stream), X, n, d, CT, k, out_idx, out_dist);
  return oryx_check_launch();
}

}  // extern "C"
