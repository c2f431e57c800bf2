// als.hip -- fused ALS half-step: gather + segmented Gramian on MFMA + Cholesky solve.
//
// For every row u of a CSR ratings matrix this solves the ALS normal equations
// (Hu-Koren-Volinsky implicit form / plain explicit form, as Spark MLlib's ALS does when the
// reference calls it at [mllib]/als/ALSUpdate.java:116-124):
//
//   implicit:  (YtY + sum_i c1_ui y_i y_i^T + lambda*n+_u I) x_u = sum_{r_ui>0} (1+c1_ui) y_i
//              c1_ui = alpha*|r_ui|, n+_u = #positive ratings
//   explicit:  (sum_i y_i y_i^T + lambda*n_u I) x_u = sum_i r_ui y_i
//
// MI355X design:
//   * the factor matrix Y is bf16, zero-padded to KP = k rounded up to 16 columns, row-major;
//     rows are gathered 32 ratings at a time (16-byte loads) and written transposed into LDS
//     so that each lane's MFMA fragment is one ds_read_b128;
//   * the per-row Gramian sum_i c_i y_i y_i^T accumulates in fp32 on
//     v_mfma_f32_16x16x32_bf16 (only the (M(M+1)/2) lower 16x16 tiles; M = KP/16), with the
//     c_i scaling applied to the A fragment in registers;
//   * KP <= 64 ("wave" kernel): one 64-lane wave owns one row end-to-end; after the Gramian
//     is redistributed through LDS each lane owns one column of A in registers and the
//     Cholesky factorization / forward solve run entirely in registers with v_readlane
//     broadcasts (no barriers, no LDS traffic in the O(k^3) part); only the back-substitution
//     reads the factor back through LDS;
//   * 64 < KP <= 128 ("block" kernel): a 256-thread workgroup owns one row and factors in LDS.
//   * rows are processed in the order given by row_ids (longest first from the host), with a
//     grid-stride loop so long rows start early and short rows fill the tail.
// Output is the fp32 solution plus an optional bf16 copy (the operand of the next half-step).

#include "common.h"

namespace {

struct AlsParams {
  const int64_t* row_ptr;  // [n_rows + 1]
  const int32_t* row_ids;  // [n_work] (nullable: rows 0..n_work-1)
  const int32_t* col_idx;  // [nnz]
  const float* vals;       // [nnz]
  const __bf16* Y;         // [n_cols][KP]
  const float* YtY;        // [KP][KP] (zeros for explicit feedback)
  float* X;                // [n_rows][KP]
  __bf16* Xb;              // [n_rows][KP] (nullable)
  int n_work;
  int k;
  float lambda;
  float alpha;
  int implicit;
  int* fail_count;         // nullable: incremented when a pivot is not positive
};

__device__ __forceinline__ void als_weights(float r, float alpha, int implicit, float& wa,
                                            float& wb, float& cnt) {
  if (implicit) {
    const float c1 = alpha * fabsf(r);
    wa = c1;
    wb = r > 0.f ? 1.f + c1 : 0.f;
    cnt = r > 0.f ? 1.f : 0.f;
  } else {
    wa = 1.f;
    wb = r;
    cnt = 1.f;
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

constexpr int TS = 40;  // LDS row stride (bf16 elements) of the transposed chunk: 32 + 8 pad

// ------------------------------------------------------------------ wave-per-row kernel

template <int KP>
struct WaveSmem {
  static constexpr int AS = KP + 1;
  static constexpr int T_BYTES = KP * TS * 2;
  static constexpr int A_BYTES = KP * AS * 4;
  static constexpr int RAW = T_BYTES > A_BYTES ? T_BYTES : A_BYTES;
  // + 32 floats of b weights + 64 floats of the broadcast L column
  static constexpr int BYTES = (RAW + 15) / 16 * 16 + 128 + 256;
};

template <int KP>
__global__ __launch_bounds__(256) void als_solve_wave(AlsParams p) {
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int AS = WaveSmem<KP>::AS;
  constexpr int PPR = KP / 8;         // 16-byte pieces per factor row
  constexpr int PIECES = 32 * PPR;    // pieces per 32-rating chunk
  static_assert(PIECES % 64 == 0, "KP must be a multiple of 16");
  __shared__ __attribute__((aligned(16))) char smem[4 * WaveSmem<KP>::BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  char* my = smem + wave * WaveSmem<KP>::BYTES;
  __bf16* T = reinterpret_cast<__bf16*>(my);
  float* A = reinterpret_cast<float*>(my);
  float* Wb = reinterpret_cast<float*>(my + WaveSmem<KP>::BYTES - 384);
  float* Lb = reinterpret_cast<float*>(my + WaveSmem<KP>::BYTES - 256);
  const int g = lane >> 4, fl = lane & 15;
  const int total_waves = gridDim.x * 4;

  for (int w = blockIdx.x * 4 + wave; w < p.n_work; w += total_waves) {
    const int row = p.row_ids ? p.row_ids[w] : w;
    const int64_t beg = p.row_ptr[row], end = p.row_ptr[row + 1];
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bacc = 0.f, cnt_acc = 0.f;

    for (int64_t c0 = beg; c0 < end; c0 += 32) {
      const int n = (int)min((int64_t)32, end - c0);
      int col = 0;
      float wa = 0.f, wb = 0.f, cn = 0.f;
      if (lane < n) {
        col = p.col_idx[c0 + lane];
        als_weights(p.vals[c0 + lane], p.alpha, p.implicit, wa, wb, cn);
      }
      cnt_acc += cn;
      if (lane < 32) Wb[lane] = wb;
      // gather 32 factor rows, transposed into T[feature][rating]
#pragma unroll
      for (int it = 0; it < PIECES / 64; ++it) {
        const int pid = it * 64 + lane;
        const int r = pid / PPR, pc = pid % PPR;
        const int cr = oryx_shfl_i(col, r);
        bf16x8 v;
        if (r < n) {
          v = *reinterpret_cast<const bf16x8*>(p.Y + (int64_t)cr * KP + pc * 8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) T[(pc * 8 + j) * TS + r] = v[j];
      }
      wave_sync();
      // per-lane Gramian weights of this lane's 8 ratings
      float wsc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) wsc[j] = oryx_shfl(wa, 8 * g + j);
      bf16x8 fa[M], fb[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
        const bf16x8 raw = *reinterpret_cast<const bf16x8*>(T + (pi * 16 + fl) * TS + 8 * g);
        fb[pi] = raw;
#pragma unroll
        for (int j = 0; j < 8; ++j) fa[pi][j] = (__bf16)((float)raw[j] * wsc[j]);
      }
      {
        int t = 0;
#pragma unroll
        for (int pi = 0; pi < M; ++pi)
#pragma unroll
          for (int qi = 0; qi <= pi; ++qi, ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[pi], fb[qi], acc[t], 0, 0, 0);
      }
      // b += sum_r wb_r * y_r  (lane f owns feature f; wb broadcast from LDS)
      {
        const int f = lane < KP ? lane : KP - 1;
        const bf16x8* trow = reinterpret_cast<const bf16x8*>(T + f * TS);
        const f32x4* wbv = reinterpret_cast<const f32x4*>(Wb);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bf16x8 v = trow[q];
          const f32x4 w0 = wbv[2 * q], w1 = wbv[2 * q + 1];
#pragma unroll
          for (int j = 0; j < 4; ++j) bacc += w0[j] * (float)v[j];
#pragma unroll
          for (int j = 0; j < 4; ++j) bacc += w1[j] * (float)v[4 + j];
        }
      }
      wave_sync();
    }

    const float cnt = wave_sum(cnt_acc);
    // scatter the lower tiles (and their mirror) into A[KP][AS]
    {
      int t = 0;
#pragma unroll
      for (int pi = 0; pi < M; ++pi)
#pragma unroll
        for (int qi = 0; qi <= pi; ++qi, ++t)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int i = pi * 16 + g * 4 + v, j = qi * 16 + fl;
            A[i * AS + j] = acc[t][v];
            if (pi != qi) A[j * AS + i] = acc[t][v];
          }
    }
    wave_sync();
    // lane c owns column c
    const int c = lane < KP ? lane : 0;
    const float diag = c < p.k ? p.lambda * cnt : 1.f;
    float a[KP];
    int cc = c;
    asm volatile("" : "+v"(cc));
    // YtY is always present (zeros for explicit feedback); the opaque per-row pointer keeps
    // the compiler from hoisting KP 64-bit addresses out of the row loop
    const float* ycol = p.YtY + cc;
    asm volatile("" : "+v"(ycol));
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      a[i] = A[i * AS + c] + ycol[i * KP] + (i == cc ? diag : 0.f);
      if ((i & 15) == 15) __builtin_amdgcn_sched_barrier(0);
    }
    // Cholesky A = L L^T in registers: after step j lane c holds L[c][j] in a[j]
    // (lane j keeps the pivot d_j in a[j])
    bool bad = false;
    // opaque copy of the lane id: stops the compiler hoisting 2*KP lane masks out of the row
    // loop (which would exhaust SGPRs)
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      float s = oryx_readlane(a[j], j);
      bad |= !(s > 0.f);
      s = s > 1e-30f ? s : 1e-30f;
      const float d = __builtin_sqrtf(s);
      const float inv = __builtin_amdgcn_rcpf(d);
      float l = a[j] * inv;
      l = ln < j ? 0.f : (ln == j ? d : l);
      a[j] = l;
      // broadcast column j of L through LDS (same-address reads are conflict-free)
      Lb[lane] = l;
      wave_sync();
#pragma unroll
      for (int i4 = ((j + 1) / 4) * 4; i4 < KP; i4 += 4) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(Lb + i4);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (i4 + q > j) a[i4 + q] -= lv[q] * l;
      }
      // pin the updated trailing column values here: without this LLVM sinks the rank-1
      // updates into a left-looking form that keeps every broadcast L column live (spills)
#pragma unroll
      for (int i = j + 1; i < KP; ++i) asm volatile("" : "+v"(a[i]));
      wave_sync();
    }
    if (bad && lane == 0 && p.fail_count) atomicAdd(p.fail_count, 1);
    // forward: L z = b
    float zv = lane < KP ? bacc : 0.f, z_own = 0.f;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      const float zj = oryx_readlane(zv, j) / oryx_readlane(a[j], j);
      z_own = ln == j ? zj : z_own;
      zv -= a[j] * zj;
      __builtin_amdgcn_sched_barrier(0);
    }
    // back: L^T x = z, reading row j of L (and its pivot) from LDS
    wave_sync();
    if (lane < KP) {
#pragma unroll
      for (int i = 0; i < KP; ++i) A[lane * AS + i] = a[i];
    }
    wave_sync();
    float xv = z_own, x_own = 0.f;
#pragma unroll
    for (int j = KP - 1; j >= 0; --j) {
      const float xj = oryx_readlane(xv, j) / A[j * AS + j];
      x_own = ln == j ? xj : x_own;
      xv -= A[j * AS + c] * xj;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < KP) {
      p.X[(int64_t)row * KP + lane] = x_own;
      if (p.Xb) p.Xb[(int64_t)row * KP + lane] = (__bf16)x_own;
    }
    wave_sync();
  }
}

// ------------------------------------------------------------------ block-per-row kernel

template <int KP>
struct BlockSmem {
  static constexpr int AS = KP + 1;
  static constexpr int T_BYTES = KP * TS * 2;
  static constexpr int A_BYTES = KP * AS * 4;
  static constexpr int RAW = T_BYTES > A_BYTES ? T_BYTES : A_BYTES;
  static constexpr int BYTES = (RAW + 15) / 16 * 16;
};

template <int KP>
__global__ __launch_bounds__(256) void als_solve_block(AlsParams p) {
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int TPW = (NT + 3) / 4;
  constexpr int AS = BlockSmem<KP>::AS;
  constexpr int PPR = KP / 8;
  constexpr int PIECES = 32 * PPR;
  __shared__ __attribute__((aligned(16))) char smem[BlockSmem<KP>::BYTES];
  __shared__ int s_col[32];
  __shared__ float s_wa[32], s_wb[32], s_b[KP], s_diag[KP], s_cnt;
  __bf16* T = reinterpret_cast<__bf16*>(smem);
  float* A = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, fl = lane & 15;

  // tile coordinates of this wave's tiles
  int tpi[TPW], tqi[TPW];
#pragma unroll
  for (int s = 0; s < TPW; ++s) {
    int t = wave + 4 * s, pi = 0;
    while ((pi + 1) * (pi + 2) / 2 <= t) ++pi;
    tpi[s] = pi;
    tqi[s] = t - pi * (pi + 1) / 2;
    if (t >= NT) tpi[s] = -1;
  }

  for (int w = blockIdx.x; w < p.n_work; w += gridDim.x) {
    const int row = p.row_ids ? p.row_ids[w] : w;
    const int64_t beg = p.row_ptr[row], end = p.row_ptr[row + 1];
    f32x4 acc[TPW];
#pragma unroll
    for (int s = 0; s < TPW; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bacc = 0.f, cnt_acc = 0.f;

    for (int64_t c0 = beg; c0 < end; c0 += 32) {
      const int n = (int)min((int64_t)32, end - c0);
      __syncthreads();
      if (tid < 32) {
        float wa = 0.f, wb = 0.f, cn = 0.f;
        int col = 0;
        if (tid < n) {
          col = p.col_idx[c0 + tid];
          als_weights(p.vals[c0 + tid], p.alpha, p.implicit, wa, wb, cn);
        }
        s_col[tid] = col;
        s_wa[tid] = wa;
        s_wb[tid] = wb;
        cnt_acc += cn;
      }
      __syncthreads();
      for (int pid = tid; pid < PIECES; pid += 256) {
        const int r = pid / PPR, pc = pid % PPR;
        bf16x8 v;
        if (r < n) {
          v = *reinterpret_cast<const bf16x8*>(p.Y + (int64_t)s_col[r] * KP + pc * 8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) T[(pc * 8 + j) * TS + r] = v[j];
      }
      __syncthreads();
      float wsc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) wsc[j] = s_wa[8 * g + j];
#pragma unroll
      for (int s = 0; s < TPW; ++s) {
        if (tpi[s] < 0) continue;
        const bf16x8 ra = *reinterpret_cast<const bf16x8*>(T + (tpi[s] * 16 + fl) * TS + 8 * g);
        const bf16x8 rb = *reinterpret_cast<const bf16x8*>(T + (tqi[s] * 16 + fl) * TS + 8 * g);
        bf16x8 fa;
#pragma unroll
        for (int j = 0; j < 8; ++j) fa[j] = (__bf16)((float)ra[j] * wsc[j]);
        acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, rb, acc[s], 0, 0, 0);
      }
      if (tid < KP) {
        const bf16x8* trow = reinterpret_cast<const bf16x8*>(T + tid * TS);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bf16x8 v = trow[q];
#pragma unroll
          for (int j = 0; j < 8; ++j) bacc += s_wb[q * 8 + j] * (float)v[j];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
      if (tpi[s] < 0) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = tpi[s] * 16 + g * 4 + v, j = tqi[s] * 16 + fl;
        A[i * AS + j] = acc[s][v];
        if (tpi[s] != tqi[s]) A[j * AS + i] = acc[s][v];
      }
    }
    if (wave == 0) {
      const float c = wave_sum(cnt_acc);
      if (lane == 0) s_cnt = c;
    }
    if (tid < KP) s_b[tid] = bacc;
    __syncthreads();
    const float reg = p.lambda * s_cnt;
    for (int idx = tid; idx < KP * KP; idx += 256) {
      const int i = idx / KP, j = idx % KP;
      float v = A[i * AS + j];
      v += p.YtY[idx];
      if (i == j) v += i < p.k ? reg : 1.f;
      A[i * AS + j] = v;
    }
    __syncthreads();
    // right-looking Cholesky in LDS (lower triangle)
    for (int j = 0; j < KP; ++j) {
      __syncthreads();
      float s = A[j * AS + j];
      if (tid == 0 && !(s > 0.f) && p.fail_count) atomicAdd(p.fail_count, 1);
      s = s > 1e-30f ? s : 1e-30f;
      const float d = sqrtf(s);
      if (tid == 0) s_diag[j] = d;
      for (int i = j + 1 + tid; i < KP; i += 256) A[i * AS + j] /= d;
      __syncthreads();
      const int rem = KP - j - 1;
      for (int idx = tid; idx < rem * rem; idx += 256) {
        const int ii = j + 1 + idx / rem, cc = j + 1 + idx % rem;
        if (cc <= ii) A[ii * AS + cc] -= A[ii * AS + j] * A[cc * AS + j];
      }
    }
    __syncthreads();
    if (wave == 0) {
      // forward: L z = b
      for (int j = 0; j < KP; ++j) {
        const float z = s_b[j] / s_diag[j];
        wave_sync();
        for (int i = j + 1 + lane; i < KP; i += 64) s_b[i] -= A[i * AS + j] * z;
        if (lane == 0) s_b[j] = z;
        wave_sync();
      }
      // back: L^T x = z
      for (int j = KP - 1; j >= 0; --j) {
        const float x = s_b[j] / s_diag[j];
        wave_sync();
        for (int i = lane; i < j; i += 64) s_b[i] -= A[j * AS + i] * x;
        if (lane == 0) s_b[j] = x;
        wave_sync();
      }
      for (int i = lane; i < KP; i += 64) {
        p.X[(int64_t)row * KP + i] = s_b[i];
        if (p.Xb) p.Xb[(int64_t)row * KP + i] = (__bf16)s_b[i];
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ helpers

// sum over a row of dot(X[u], Y[i]) for (u, i) pairs: predictions for evaluation (K7)
__global__ __launch_bounds__(256) void pair_dots(const float* __restrict__ X,
                                                 const float* __restrict__ Y,
                                                 const int32_t* __restrict__ us,
                                                 const int32_t* __restrict__ is, int64_t n,
                                                 int kp, float* __restrict__ out) {
  // one 16-lane group per pair, kp a multiple of 16
  const int64_t gid = ((int64_t)blockIdx.x * 256 + threadIdx.x);
  const int64_t pair = gid >> 4;
  const int sub = threadIdx.x & 15;
  float s = 0.f;
  if (pair < n) {
    const float* x = X + (int64_t)us[pair] * kp;
    const float* y = Y + (int64_t)is[pair] * kp;
    for (int f = sub; f < kp; f += 16) s += x[f] * y[f];
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) s += __shfl_xor(s, off, 16);
  if (pair < n && sub == 0) out[pair] = s;
}

}  // namespace

extern "C" {

int oryx_als_solve(const int64_t* row_ptr, const int32_t* row_ids, const int32_t* col_idx,
                   const float* vals, const void* Y, const float* YtY, float* X, void* Xb,
                   int n_work, int k, int kp, float lambda, float alpha, int implicit,
                   int* fail_count, void* stream) {
  if (n_work <= 0) return ORYX_OK;
  AlsParams p{row_ptr, row_ids, col_idx, vals, reinterpret_cast<const __bf16*>(Y), YtY, X,
              reinterpret_cast<__bf16*>(Xb), n_work, k, lambda, alpha, implicit, fail_count};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int max_blocks = 256 * 16;
  switch (kp) {
#define WAVE_CASE(KPV)                                                                \
  case KPV: {                                                                         \
    int blocks = (n_work + 3) / 4;                                                    \
    if (blocks > max_blocks) blocks = max_blocks;                                     \
    hipLaunchKernelGGL(als_solve_wave<KPV>, dim3(blocks), dim3(256), 0, s, p);       \
    break;                                                                            \
  }
    WAVE_CASE(16)
    WAVE_CASE(32)
    WAVE_CASE(48)
    WAVE_CASE(64)
#undef WAVE_CASE
#define BLOCK_CASE(KPV)                                                               \
  case KPV: {                                                                         \
    int blocks = n_work < max_blocks ? n_work : max_blocks;                           \
    hipLaunchKernelGGL(als_solve_block<KPV>, dim3(blocks), dim3(256), 0, s, p);      \
    break;                                                                            \
  }
    BLOCK_CASE(80)
    BLOCK_CASE(96)
    BLOCK_CASE(112)
    BLOCK_CASE(128)
#undef BLOCK_CASE
    default:
      return ORYX_EINVAL;
  }
  return oryx_check_launch();
}

int oryx_pair_dots(const float* X, const float* Y, const int32_t* us, const int32_t* is,
                   long long n, int kp, float* out, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (kp % 16) return ORYX_EINVAL;
  const long long threads = n * 16;
  const int blocks = (int)((threads + 255) / 256);
  hipLaunchKernelGGL(pair_dots, dim3(blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), X, Y, us, is, (int64_t)n, kp, out);
  return oryx_check_launch();
}

int oryx_kernels_version() { return 1; }

}  // extern "C"
