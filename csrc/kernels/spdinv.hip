// spdinv.hip -- the speed layer's two Gramian inverses, certified, in one launch.
//
// ALSSpeedModel keeps a solver for XtX and YtY (LinearSystemSolver.getSolver over an RRQR,
// [app-common]/math/LinearSystemSolver.java:38-56, refreshed per micro-batch by
// [speed-app]/als/ALSSpeedModel.java getXTXSolver / getYTYSolver).  The fold-in only needs the
// inverses, so each is formed directly: one workgroup per matrix holds it in LDS as fp64 and
// runs an in-place Gauss-Jordan elimination without pivoting (which, for a symmetric matrix,
// meets exactly the pivots of its LDL^T factorisation: all positive iff it is positive
// definite).  The same workgroup certifies the result against the reference's acceptance
// test: for SPD A every |R_ii| of a pivoted QR is >= lambda_min(A) >= 1 / ||A^-1||_F, so
//   all pivots > 0,  A^-1 finite,  ||A^-1||_F * ||A||_inf * ratio < 1
// implies the RRQR check passes (ok[m] = 1); anything else sends the caller to the host RRQR
// path.  This replaces ~15 tensor ops per matrix (fp64 cast, cholesky_ex, cholesky_inverse,
// norms) with one launch.

#include "common.h"

namespace {

constexpr int SI_THREADS = 512;

__device__ double block_reduce(double v, double* red, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double o = __shfl_xor(v, off, 64);
    v = is_max ? fmax(v, o) : v + o;
  }
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double r = red[0];
  for (int w = 1; w < SI_THREADS / 64; ++w) r = is_max ? fmax(r, red[w]) : r + red[w];
  return r;
}

__global__ __launch_bounds__(SI_THREADS) void spd_inverse_pair(
    const float* __restrict__ G0, const float* __restrict__ G1, int k, double* __restrict__ I0,
    double* __restrict__ I1, double ratio, int* __restrict__ ok) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* A = lds;                 // [k][k]
  double* rowp = A + k * k;        // scaled pivot row
  double* col = rowp + k;          // pivot column before the step
  __shared__ double red[SI_THREADS / 64];
  const float* G = blockIdx.x ? G1 : G0;
  double* out = blockIdx.x ? I1 : I0;
  const int tid = threadIdx.x;
  const int kk = k * k;
  for (int x = tid; x < kk; x += SI_THREADS) A[x] = (double)G[x];
  __syncthreads();
  // ||A||_inf: the largest absolute row sum
  double rs = 0.0;
  for (int r = tid; r < k; r += SI_THREADS) {
    double s = 0.0;
    for (int c = 0; c < k; ++c) s += fabs(A[r * k + c]);
    rs = fmax(rs, s);
  }
  const double norm_inf = block_reduce(rs, red, true);
  bool bad = false;
  for (int p = 0; p < k; ++p) {
    __syncthreads();
    const double piv = A[p * k + p];
    if (!(piv > 0.0)) {            // uniform: every thread read the same pivot
      bad = true;
      break;
    }
    const double rp = 1.0 / piv;
    for (int j = tid; j < k; j += SI_THREADS) {
      rowp[j] = (j == p ? 1.0 : A[p * k + j]) * rp;
      col[j] = A[j * k + p];
    }
    __syncthreads();
    for (int x = tid; x < kk; x += SI_THREADS) {
      const int i = x / k, j = x - i * k;
      A[x] = i == p ? rowp[j] : (j == p ? 0.0 : A[x]) - col[i] * rowp[j];
    }
  }
  __syncthreads();
  double ss = 0.0;
  bool finite = true;
  for (int x = tid; x < kk; x += SI_THREADS) {
    const double v = A[x];
    finite = finite && (v - v == 0.0);
    ss += v * v;
    out[x] = v;
  }
  const double fro2 = block_reduce(ss, red, false);
  const double all_finite = block_reduce(finite ? 1.0 : 0.0, red, false);
  if (tid == 0)
    ok[blockIdx.x] = (!bad && all_finite == (double)SI_THREADS &&
                      sqrt(fro2) * norm_inf * ratio < 1.0) ? 1 : 0;
}

}  // namespace

extern "C" {

// G0 / G1 [k][k] fp32 Gramians -> I0 / I1 [k][k] fp64 inverses and ok[2] (1: certified, see
// above; 0: not SPD to working precision or too ill-conditioned -- use the host path).
// k <= 128 (the LDS holds the fp64 matrix).
int oryx_spd_inverse_pair(const float* G0, const float* G1, int k, double* I0, double* I1,
                          double ratio, int* ok, void* stream) {
  if (k <= 0 || k > 128) return ORYX_EINVAL;
  const int lds = (k * k + 2 * k) * (int)sizeof(double);
  if (lds > 64 * 1024 && !oryx_set_max_lds(&spd_inverse_pair, lds)) return ORYX_ELAUNCH;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(spd_inverse_pair, dim3(2), dim3(SI_THREADS), lds, s, G0, G1, k, I0, I1,
                     ratio, ok);
  return oryx_check_launch();
}

}  // extern "C"
