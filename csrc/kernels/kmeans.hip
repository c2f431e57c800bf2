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
// kmeans_accumulate: per point, atomically adds its fp32 row into sums[assign] (a wave owns a
// row so every atomic instruction covers 256 contiguous bytes -- the full-rate shape), plus
// counts and distance statistics (count, sum d, sum d^2 for the DB / Dunn / SSE metrics).

#include "common.h"

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
#pragma unroll
    for (int ct = 0; ct < BN / 16; ++ct) {
      f32x4 acc[ROW_TILES];
#pragma unroll
      for (int rt = 0; rt < ROW_TILES; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DK; ++s) {
        const bf16x8 b =
            *reinterpret_cast<const bf16x8*>(base + (ct * 16 + fl) * ROWB + (s * 32 + 8 * g) * 2);
#pragma unroll
        for (int rt = 0; rt < ROW_TILES; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][s], b, acc[rt], 0, 0, 0);
      }
      // C/D layout: col = fl (center), row = g*4 + v (point)
      const int c = t * BN + ct * 16 + fl;
      const float cn = cnorm[c];
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
  switch (dk) {
    ASSIGN_CASE(1, 2)
    ASSIGN_CASE(2, 2)
    ASSIGN_CASE(3, 2)
    ASSIGN_CASE(4, 2)
    ASSIGN_CASE(5, 2)
    ASSIGN_CASE(6, 2)
    ASSIGN_CASE(7, 2)
    ASSIGN_CASE(8, 2)
    ASSIGN_CASE(10, 1)
    ASSIGN_CASE(12, 1)
    ASSIGN_CASE(16, 1)
    default:
      return ORYX_EINVAL;
  }
#undef ASSIGN_CASE
  return oryx_check_launch();
}

int oryx_kmeans_accumulate(const float* X, const int* assign, const float* mind, long long n,
                           int d, int ld, float* sums, unsigned long long* counts, double* dstats,
                           void* stream) {
  if (n <= 0) return ORYX_OK;
  long long waves = n < (1ll << 20) ? n : (1ll << 20);
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL(kmeans_accumulate_kernel, dim3(blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), X, assign, mind, n, d, ld, sums,
                     counts, dstats);
  return oryx_check_launch();
}

}  // extern "C"
