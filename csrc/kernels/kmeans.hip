// kmeans.hip -- k-means assignment (MFMA distance GEMM + fused argmin) and accumulation.
//
// SURVEY.md K8/K9 (the Lloyd step MLlib runs for the reference at
// [mllib]/kmeans/KMeansUpdate.java:116-117, the evaluation assignment of
// [mllib]/kmeans/AbstractKMeansEvaluation.java:59-74 and the speed/serving nearest-cluster
// scans [speed-app]/kmeans/KMeansSpeedModelManager.java:93-101, [app-common]/kmeans/KMeansUtils.java:40-56).
//
// kmeans_assign: squared distance |x|^2 - 2 x.c + |c|^2 for a tile of points against every
// center, keeping the running (min, argmin) per point, without materialising the N x K
// distance matrix:
//   * workgroup = 4 waves = BM points (ROW_TILES x 16 per wave); each lane keeps its points'
//     bf16 MFMA A-fragments in registers for the whole kernel (X is read from HBM once);
//   * centers stream through LDS 64 at a time (register-staged double buffer, rows padded by
//     16 B so the B-fragment ds_read_b128 is bank-conflict free), shared by the 4 waves;
//   * v_mfma_f32_16x16x32_bf16 accumulates the dot products in fp32; the epilogue folds the
//     norms and updates the per-point best in registers; a 16-lane shuffle reduction at the end.
// kmeans_accumulate: per point, adds its fp32 row into sums[assign] plus counts and distance
// statistics (count, sum d, sum d^2 for the DB / Dunn / SSE metrics): LDS-privatised column
// slices when K x (slice) fits (kmeans_accumulate_lds_kernel), else one wave per row of L2
// atomics (every atomic instruction covers 256 contiguous bytes).

#include "common.h"

#include <cstdlib>

namespace {

constexpr int BN = 64;  // centers per LDS tile

template <int DK, int ROW_TILES>
__global__ __launch_bounds__(256) void kmeans_assign_kernel(
    const __bf16* __restrict__ X, const float* __restrict__ xnorm, const __bf16* __restrict__ C,
    const float* __restrict__ cnorm, long long n, int k_pad, int* __restrict__ assign,
    float* __restrict__ mind) {
  constexpr int DPAD = DK * 32;               // feature dim (bf16 elements)
  constexpr int ROWB = DPAD * 2 + 16;         // padded LDS row (bytes)
  constexpr int TILE_BYTES = BN * ROWB;
  constexpr int PIECES = BN * DPAD / 8;       // 16-byte pieces per center tile
  constexpr int PPT = (PIECES + 255) / 256;   // pieces per thread
  constexpr int BM = 4 * ROW_TILES * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, fl = lane & 15;
  const int nblocks = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nblocks);
  const long long row0 = (long long)bid * BM + wave * ROW_TILES * 16;

  // A fragments: row (row0 + rt*16 + fl), k = s*32 + 8g .. +7
  bf16x8 a[ROW_TILES][DK];
#pragma unroll
  for (int rt = 0; rt < ROW_TILES; ++rt) {
    const long long r = row0 + rt * 16 + fl;
#pragma unroll
    for (int s = 0; s < DK; ++s) {
      if (r < n) {
        a[rt][s] = *reinterpret_cast<const bf16x8*>(X + r * DPAD + s * 32 + 8 * g);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[rt][s][j] = (__bf16)0.f;
      }
    }
  }
  // per-lane best for rows (rt, g*4 + v)
  float best[ROW_TILES][4];
  int besti[ROW_TILES][4];
  float xn[ROW_TILES][4];
#pragma unroll
  for (int rt = 0; rt < ROW_TILES; ++rt)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      best[rt][v] = INFINITY;
      besti[rt][v] = 0;
      const long long r = row0 + rt * 16 + g * 4 + v;
      xn[rt][v] = r < n ? xnorm[r] : 0.f;
    }

  const int ntiles = k_pad / BN;
  i32x4 stage[PPT];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int pid = q * 256 + tid;
      if (pid < PIECES) {
        const int row = pid / (DPAD / 8), pc = pid % (DPAD / 8);
        stage[q] = *reinterpret_cast<const i32x4*>(C + ((long long)t * BN + row) * DPAD + pc * 8);
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* base = smem + buf * TILE_BYTES;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int pid = q * 256 + tid;
      if (pid < PIECES) {
        const int row = pid / (DPAD / 8), pc = pid % (DPAD / 8);
        *reinterpret_cast<i32x4*>(base + row * ROWB + pc * 16) = stage[q];
      }
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);  // global loads in flight during the MFMAs
    const char* base = smem + buf * TILE_BYTES;
    // B fragments double-buffered in registers: the reads for center group ct+1 are in flight
    // while group ct's MFMAs run (reading right before use exposed the LDS latency on every
    // pair of MFMAs)
    bf16x8 bfr[2][DK];
    auto read_b = [&](int ct, bf16x8* dst) {
#pragma unroll
      for (int s = 0; s < DK; ++s)
        dst[s] = *reinterpret_cast<const bf16x8*>(base + (ct * 16 + fl) * ROWB +
                                                  (s * 32 + 8 * g) * 2);
    };
    read_b(0, bfr[0]);
#pragma unroll
    for (int ct = 0; ct < BN / 16; ++ct) {
      if (ct + 1 < BN / 16) read_b(ct + 1, bfr[(ct + 1) & 1]);
      const float cn = cnorm[t * BN + ct * 16 + fl];
      f32x4 acc[ROW_TILES];
#pragma unroll
      for (int rt = 0; rt < ROW_TILES; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DK; ++s) {
#pragma unroll
        for (int rt = 0; rt < ROW_TILES; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][s], bfr[ct & 1][s], acc[rt],
                                                            0, 0, 0);
      }
      // C/D layout: col = fl (center), row = g*4 + v (point)
      const int c = t * BN + ct * 16 + fl;
#pragma unroll
      for (int rt = 0; rt < ROW_TILES; ++rt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float d = xn[rt][v] + cn - 2.f * acc[rt][v];
          if (d < best[rt][v]) {
            best[rt][v] = d;
            besti[rt][v] = c;
          }
        }
    }
    if (t + 1 < ntiles) {
      __syncthreads();  // everyone done reading buf^1's previous contents (tile t-1)
      store_tile(buf ^ 1);
      __syncthreads();
    }
  }
  // reduce over the 16 lanes (centers) sharing each row; ties -> lowest center index
#pragma unroll
  for (int rt = 0; rt < ROW_TILES; ++rt)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float bv = best[rt][v];
      int bi = besti[rt][v];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov < bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      const long long r = row0 + rt * 16 + g * 4 + v;
      if (fl == 0 && r < n) {
        assign[r] = bi;
        mind[r] = bv > 0.f ? bv : 0.f;
      }
    }
}

// one wave per row: sums[assign[r]] += x[r] (fp32 atomics, 256 contiguous bytes per instr)
__global__ __launch_bounds__(256) void kmeans_accumulate_kernel(
    const float* __restrict__ X, const int* __restrict__ assign, const float* __restrict__ mind,
    long long n, int d, int ld, float* __restrict__ sums,
    unsigned long long* __restrict__ counts, double* __restrict__ dstats) {
  const int lane = threadIdx.x & 63;
  const long long wave_id = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const long long nwaves = ((long long)gridDim.x * 256) >> 6;
  for (long long r = wave_id; r < n; r += nwaves) {
    const int c = assign[r];
    const float* xr = X + r * ld;
    float* sr = sums + (long long)c * d;
    for (int j = lane; j < d; j += 64) atomicAdd(sr + j, xr[j]);
    if (lane == 0) {
      atomicAdd(counts + c, 1ull);
      if (dstats) {
        const double dist = sqrt((double)mind[r]);
        atomicAdd(dstats + 2 * c, dist);
        atomicAdd(dstats + 2 * c + 1, dist * dist);
      }
    }
  }
}

// LDS-privatised accumulation: block (x, y) owns rows [x*rpb, ...) and the column slice
// [y*CW, y*CW + CW) of every center.  Its K x CW partial sums (row stride CW+1 when it fits,
// so that two rows of one wave hitting different clusters fall on different banks), plus the
// K counts and distance statistics for the y == 0 column, live in LDS; ds_add_f32 replaces the
// per-(row, column) L2 atomic of kmeans_accumulate_kernel -- with 1000 clusters and millions
// of rows the L2 atomics serialise on hot lines -- and each block flushes K x CW values once.
// 1024 threads per block: the LDS image allows one block per CU, so the block itself carries
// the 16 waves of memory-level parallelism the row stream needs.
template <bool VEC>
__global__ __launch_bounds__(1024) void kmeans_accumulate_lds_kernel(
    const float* __restrict__ X, const int* __restrict__ assign, const float* __restrict__ mind,
    long long n, int d, int ld, int k, int cw, int stride, long long rpb,
    float* __restrict__ sums, unsigned long long* __restrict__ counts,
    double* __restrict__ dstats) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  double* lstat = reinterpret_cast<double*>(smem_raw);                  // [k][2]
  unsigned int* lcnt = reinterpret_cast<unsigned int*>(lstat + 2 * k);  // [k]
  float* lsum = reinterpret_cast<float*>(lcnt + k);                     // [k][stride]
  const int tid = threadIdx.x;
  const int c0 = blockIdx.y * cw;
  const int cwe = min(cw, d - c0);                 // columns of this slice that exist
  const bool lead = blockIdx.y == 0;
  for (int i = tid; i < k * stride; i += 1024) lsum[i] = 0.f;
  if (lead) {
    for (int i = tid; i < k; i += 1024) lcnt[i] = 0u;
    if (dstats)
      for (int i = tid; i < 2 * k; i += 1024) lstat[i] = 0.0;
  }
  __syncthreads();
  // VEC: a thread owns 4 consecutive columns (one 16-byte load per row); else 1 column
  constexpr int W = VEC ? 4 : 1;
  const int lanes = (cw + W - 1) / W;
  const int tpr = lanes < 64 ? lanes : 64;         // threads per row
  const int rpp = 1024 / tpr;                      // rows per pass
  const int sub = tid / tpr, col = (tid % tpr) * W;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < n ? r0 + rpb : n;
  // U rows per thread per step: all U assignment loads, then all U row loads, are in flight
  // together (a row costs two dependent HBM round trips; one row per step left the loop
  // latency-bound at 16 waves per CU)
  constexpr int U = 8;
  for (long long base = r0 + sub; base < r1; base += (long long)U * rpp) {
    int c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = base + (long long)u * rpp;
      c[u] = r < r1 ? assign[r] : -1;
    }
    for (int j = col; j < cwe; j += tpr * W) {
      if (VEC) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = base + (long long)u * rpp;
          if (c[u] >= 0) v[u] = *reinterpret_cast<const f32x4*>(X + r * ld + c0 + j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (c[u] >= 0) {
            float* sr = lsum + c[u] * stride + j;
            atomicAdd(sr, v[u][0]);
            atomicAdd(sr + 1, v[u][1]);
            atomicAdd(sr + 2, v[u][2]);
            atomicAdd(sr + 3, v[u][3]);
          }
        }
      } else {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = base + (long long)u * rpp;
          if (c[u] >= 0) v[u] = X[r * ld + c0 + j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (c[u] >= 0) atomicAdd(lsum + c[u] * stride + j, v[u]);
      }
    }
    if (lead && col == 0) {
      float md[U];
      if (dstats) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = base + (long long)u * rpp;
          md[u] = c[u] >= 0 ? mind[r] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (c[u] < 0) continue;
        atomicAdd(lcnt + c[u], 1u);
        if (dstats) {
          const double dist = sqrt((double)md[u]);
          atomicAdd(lstat + 2 * c[u], dist);
          atomicAdd(lstat + 2 * c[u] + 1, dist * dist);
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < k * cwe; i += 1024) {
    const int cc = i / cwe, j = i - cc * cwe;
    const float v = lsum[cc * stride + j];
    if (v != 0.f) atomicAdd(sums + (long long)cc * d + c0 + j, v);
  }
  if (lead) {
    for (int i = tid; i < k; i += 1024) {
      const unsigned int v = lcnt[i];
      if (v) atomicAdd(counts + i, (unsigned long long)v);
    }
    if (dstats)
      for (int i = tid; i < 2 * k; i += 1024) {
        const double v = lstat[i];
        if (v != 0.0) atomicAdd(dstats + i, v);
      }
  }
}

}  // namespace

extern "C" {

// X: bf16 [n][d_pad] (d_pad = 32 * dk), xnorm fp32 [n]; C: bf16 [k_pad][d_pad],
// cnorm fp32 [k_pad] (+inf for padding rows); k_pad multiple of 64.
int oryx_kmeans_assign(const void* X, const float* xnorm, const void* C, long long n,
                       int d_pad, int k_pad, const float* cnorm, int* assign, float* mind,
                       void* stream) {
  if (n <= 0) return ORYX_OK;
  if (d_pad % 32 || k_pad % BN || d_pad > 512) return ORYX_EINVAL;
  const int dk = d_pad / 32;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* x = reinterpret_cast<const __bf16*>(X);
  const __bf16* c = reinterpret_cast<const __bf16*>(C);
#define ASSIGN_CASE(DKV, RT)                                                                  \
  case DKV: {                                                                                 \
    constexpr int BM = 4 * RT * 16;                                                           \
    const int smem = 2 * BN * (DKV * 64 + 16);                                                \
    const long long blocks = (n + BM - 1) / BM;                                               \
    static bool attr_set = false;                                                             \
    if (!attr_set && smem > 65536) {                                                          \
      hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_assign_kernel<DKV, RT>),     \
                          hipFuncAttributeMaxDynamicSharedMemorySize, smem);                  \
      attr_set = true;                                                                        \
    }                                                                                         \
    hipLaunchKernelGGL((kmeans_assign_kernel<DKV, RT>), dim3((unsigned)blocks), dim3(256),   \
                       smem, s, x, xnorm, c, cnorm, n, k_pad, assign, mind);                  \
    break;                                                                                    \
  }
  // rows per wave = 16 * RT: RT = 4 halves the LDS B-fragment reads and the L2 -> LDS center
  // traffic per MFMA relative to RT = 2 but drops to one wave per SIMD; measured at d = 256,
  // K = 1000 it ran 7% slower (10.2 vs 9.5 ms per 12.5M points), so RT = 2 is the default and
  // ORYX_KMEANS_RT=4 selects the wide tiles
  static const int rt_pref = getenv("ORYX_KMEANS_RT") ? atoi(getenv("ORYX_KMEANS_RT")) : 2;
  if (rt_pref != 4 && dk <= 8) {
    switch (dk) {
      ASSIGN_CASE(1, 2)
      ASSIGN_CASE(2, 2)
      ASSIGN_CASE(3, 2)
      ASSIGN_CASE(4, 2)
      ASSIGN_CASE(5, 2)
      ASSIGN_CASE(6, 2)
      ASSIGN_CASE(7, 2)
      ASSIGN_CASE(8, 2)
      default:
        return ORYX_EINVAL;
    }
    return oryx_check_launch();
  }
  switch (dk) {
    ASSIGN_CASE(1, 4)
    ASSIGN_CASE(2, 4)
    ASSIGN_CASE(3, 4)
    ASSIGN_CASE(4, 4)
    ASSIGN_CASE(5, 4)
    ASSIGN_CASE(6, 4)
    ASSIGN_CASE(7, 4)
    ASSIGN_CASE(8, 4)
    ASSIGN_CASE(10, 2)
    ASSIGN_CASE(12, 2)
    ASSIGN_CASE(16, 1)
    default:
      return ORYX_EINVAL;
  }
#undef ASSIGN_CASE
  return oryx_check_launch();
}

// k: number of clusters (rows of sums/counts/dstats).
int oryx_kmeans_accumulate(const float* X, const int* assign, const float* mind, long long n,
                           int d, int ld, int k, float* sums, unsigned long long* counts,
                           double* dstats, void* stream) {
  if (n <= 0) return ORYX_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // LDS budget: 160 KB minus the counts / stats arrays; slice width = the largest power of two
  // whose K x (CW + 1) fp32 partials fit
  constexpr long long LDS = 160 * 1024;
  const long long fixed = (long long)k * (4 + 16);
  int cw = 256;
  while (cw >= 4 && fixed + (long long)k * (cw + 1) * 4 > LDS) cw >>= 1;
  if (cw >= 4 && k > 0) {
    if (cw > d) {
      cw = 4;
      while (cw < d) cw <<= 1;
    }
    const int stride = fixed + (long long)k * (cw + 1) * 4 <= LDS ? cw + 1 : cw;
    const int slices = (d + cw - 1) / cw;
    long long target = 1024 / slices;
    if (target < 1) target = 1;
    long long rpb = (n + target - 1) / target;
    const long long min_rows = 16ll * k > 8192 ? 16ll * k : 8192;   // amortise the flush
    if (rpb < min_rows) rpb = min_rows;
    const long long blocks = (n + rpb - 1) / rpb;
    const size_t smem = (size_t)fixed + (size_t)k * stride * 4;
    // 16-byte row loads need 16-byte aligned rows and slice starts
    const bool vec = (ld % 4 == 0) && (cw % 4 == 0) &&
                     (reinterpret_cast<unsigned long long>(X) % 16 == 0);
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_accumulate_lds_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
      hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_accumulate_lds_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
      attr_set = true;
    }
    const dim3 grid((unsigned)blocks, (unsigned)slices);
    if (vec)
      hipLaunchKernelGGL(kmeans_accumulate_lds_kernel<true>, grid, dim3(1024), smem, s, X,
                         assign, mind, n, d, ld, k, cw, stride, rpb, sums, counts, dstats);
    else
      hipLaunchKernelGGL(kmeans_accumulate_lds_kernel<false>, grid, dim3(1024), smem, s, X,
                         assign, mind, n, d, ld, k, cw, stride, rpb, sums, counts, dstats);
    return oryx_check_launch();
  }
  long long waves = n < (1ll << 20) ? n : (1ll << 20);
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL(kmeans_accumulate_kernel, dim3(blocks), dim3(256), 0, s, X, assign, mind,
                     n, d, ld, sums, counts, dstats);
  return oryx_check_launch();
}

}  // extern "C"
