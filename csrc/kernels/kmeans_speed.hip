// kmeans_speed.hip -- the k-means speed layer's nearest-center search, exact fp64.
//
// KMeansSpeedModelManager.buildUpdates ([speed-app]/kmeans/KMeansSpeedModelManager.java:
// 88-125) assigns every point of a micro-batch to its closest cluster by Euclidean distance
// (KMeansUtils.closestCluster: squared differences summed in double, first strictly smaller
// distance wins).  A 256-thread block takes PT points, read by the scalar unit (SGPR operands
// of the VALU ops: the same values for every lane), and each thread runs through the clusters
// c = c0 + tid, c0 + tid + 256, ... of the block's cluster chunk [c0, c1), reading the centers
// from a feature-major copy (C^T [d][k]: consecutive threads read consecutive centers, one
// coalesced line per feature) FA features ahead; the per-point minimum is reduced over the
// block with the lowest index winning ties, and km_nearest_merge takes the chunks in cluster
// order with the same rule -- the sequential scan's pick.  (The squared differences are
// accumulated with fused multiply-adds.)  At 10k points x 1000 centers x 256 dims: 264 us;
// the first version (points broadcast from LDS, one center load in flight, one chunk) took
// 586 us (profiles/r6_km_speed_kernel_stats_v1.txt, _v2.txt).

#include "common.h"

namespace {

constexpr int KS_THREADS = 256;
constexpr int PT = 8;             // points per block (16: 326 us, 8: 264 us at 10k x 1000 x 256)
constexpr int FA = 4;             // features whose center values load ahead (even)

// D > 0: the feature count at compile time (the point rows' offsets become immediates of the
// scalar loads, sparing the SGPRs 16 row pointers); D = 0: d at run time.  n >= PT: the
// last block starts at n - PT (it overlaps the one before it; both write the same values).
template <int D>
__global__ __launch_bounds__(KS_THREADS) void km_nearest_f64(
    const double* __restrict__ X, long long n, int d_rt, const double* __restrict__ CT, int k,
    int kc, double* __restrict__ part_best, int* __restrict__ part_idx) {
  const int d = D > 0 ? D : d_rt;
  __shared__ double rbest[KS_THREADS / 64][PT];
  __shared__ int ridx[KS_THREADS / 64][PT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long p0 = min((long long)blockIdx.x * PT, n - PT);
  double best[PT];
  int bi[PT];
#pragma unroll
  for (int r = 0; r < PT; ++r) {
    best[r] = INFINITY;
    bi[r] = 0x7fffffff;
  }
  const double* xb = X + p0 * d;   // the block's PT rows, d apart
  const int chunk = blockIdx.y, nch = gridDim.y;
  const int c1 = min(k, (chunk + 1) * kc);
  for (int c = chunk * kc + tid; c < c1; c += KS_THREADS) {
    double acc[PT];
#pragma unroll
    for (int r = 0; r < PT; ++r) acc[r] = 0.0;
    // the block's points are the same for every lane: read through the scalar unit (s_load
    // into SGPRs, an operand of each VALU op) instead of 16 broadcast LDS reads per feature,
    // each waited on; the next FA features' center values load under this FA's work
    // (profiles/r6_km_speed_kernel_stats_v*.txt).  The sums run over the features in order.
    const double* cp = CT + c;
    // center values FA features ahead (an L2 read takes longer than one feature pair's work)
    double cur[FA], nxt[FA];
#pragma unroll
    for (int u = 0; u < FA; ++u) cur[u] = cp[(long long)min(u, d - 1) * k];
    int f = 0;
    for (; f + FA <= d; f += FA) {
#pragma unroll
      for (int u = 0; u < FA; ++u) nxt[u] = cp[(long long)min(f + FA + u, d - 1) * k];
#pragma unroll
      for (int u = 0; u < FA; u += 2) {
        double x0[PT], x1[PT];
#pragma unroll
        for (int r = 0; r < PT; ++r) {
          x0[r] = xb[r * d + f + u];
          x1[r] = xb[r * d + f + u + 1];
        }
#pragma unroll
        for (int r = 0; r < PT; ++r) {
          const double df0 = x0[r] - cur[u];
          acc[r] += df0 * df0;
          const double df1 = x1[r] - cur[u + 1];
          acc[r] += df1 * df1;
        }
      }
#pragma unroll
      for (int u = 0; u < FA; ++u) cur[u] = nxt[u];
    }
    // the last d % FA features (their center values are in cur)
#pragma unroll
    for (int u = 0; u < FA - 1; ++u) {
      if (f + u < d) {
#pragma unroll
        for (int r = 0; r < PT; ++r) {
          const double df = xb[r * d + f + u] - cur[u];
          acc[r] += df * df;
        }
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
  if (tid < PT) {
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
    part_best[(p0 + tid) * nch + chunk] = b;
    part_idx[(p0 + tid) * nch + chunk] = i;
  }
}

// per point: the chunks' minima in cluster order, strictly smaller wins (ties stay with the
// lower cluster index); a chunk with no clusters reports +inf
__global__ __launch_bounds__(256) void km_nearest_merge(const double* __restrict__ part_best,
                                                        const int* __restrict__ part_idx,
                                                        long long n, int nch,
                                                        long long* __restrict__ out_idx,
                                                        double* __restrict__ out_dist) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  double b = part_best[p * nch];
  int i = part_idx[p * nch];
  for (int j = 1; j < nch; ++j) {
    const double ob = part_best[p * nch + j];
    if (ob < b) {
      b = ob;
      i = part_idx[p * nch + j];
    }
  }
  out_idx[p] = i;
  out_dist[p] = sqrt(b);
}

}  // namespace

extern "C" {

// X [n][d] fp64 points (n >= PT), CT [d][k] fp64 centers feature-major; out_idx [n] (cluster
// position),
// out_dist [n] (Euclidean distance).  part_best /
// part_idx: scratch of n * oryx_kmeans_nearest_chunks(n, k) entries.
int oryx_kmeans_nearest_chunks(long long n, int k) {
  // about 2048 blocks, chunks of at least one cluster per thread
  const long long pb = (n + PT - 1) / PT;
  long long ch = (2048 + pb - 1) / pb;
  const long long most = (k + KS_THREADS - 1) / KS_THREADS;
  if (ch > most) ch = most;
  return (int)(ch < 1 ? 1 : ch);
}

int oryx_kmeans_nearest_f64(const double* X, long long n, int d, const double* CT, int k,
                            long long* out_idx, double* out_dist, double* part_best,
                            int* part_idx, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (d <= 0 || k <= 0 || n < PT) return ORYX_EINVAL;   // (the caller pads to PT points)
  const int nch = oryx_kmeans_nearest_chunks(n, k);
  const int kc = (k + nch - 1) / nch;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned blocks = (unsigned)((n + PT - 1) / PT);
  if (d == 256)
    hipLaunchKernelGGL(km_nearest_f64<256>, dim3(blocks, (unsigned)nch), dim3(KS_THREADS), 0, s,
                       X, n, d, CT, k, kc, part_best, part_idx);
  else
    hipLaunchKernelGGL(km_nearest_f64<0>, dim3(blocks, (unsigned)nch), dim3(KS_THREADS), 0, s,
                       X, n, d, CT, k, kc, part_best, part_idx);
  const int rc = oryx_check_launch();
  if (rc != ORYX_OK) return rc;
  hipLaunchKernelGGL(km_nearest_merge, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     part_best, part_idx, n, nch, out_idx, out_dist);
  return oryx_check_launch();
}

}  // extern "C"
