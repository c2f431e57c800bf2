// als.hip -- fused ALS half-step: gather + segmented Gramian on MFMA + Cholesky solve
// (dispatch, long-row partial sums, pair dots; the default solve kernels are in
// als_batch.hip, the superseded ones in tuning/als_variants.hip).
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


#include "als_wave.h"

namespace {


// ------------------------------------------------------------------ split long rows

// One wave per segment (row, slot, beg, end) of a long row: accumulate the segment's partial
// Gramian / b / count and add them into the row's workspace record with fp32 atomics (one
// 256-byte run per atomic instruction).  Runs before the solve kernel, which then takes long
// rows' normal equations from the workspace: a row with 1e5 ratings is spread over ~100
// waves instead of serialising on one (the tail of the popular-item half-step).
// STORE: each segment's record goes to its own slot of seg_ws with plain stores instead (no
// atomics; als_partial_reduce then sums each row's segments), which lets the segments be
// short -- more waves in flight for the latency-bound gather -- without the atomic traffic
// growing with their number.
template <int KP, bool SPLIT = false, bool STORE = false>
__global__ __launch_bounds__(256) void als_partial(AlsParams p, const int64_t* __restrict__ segs,
                                                  int n_seg, float* __restrict__ ws,
                                                  float* __restrict__ seg_ws) {
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int GB = ChunkImage<KP>::BYTES * (SPLIT ? 2 : 1);
  constexpr int BYTES = GB + 256;
  __shared__ __attribute__((aligned(16))) char smem[4 * BYTES];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  char* G = smem + wave * BYTES;
  float* Wab = reinterpret_cast<float*>(G + GB);
  const int g = lane >> 4, fl = lane & 15;
  for (int sgi = blockIdx.x * 4 + wave; sgi < n_seg; sgi += gridDim.x * 4) {
    const int64_t slot = segs[4 * sgi + 1], beg = segs[4 * sgi + 2], end = segs[4 * sgi + 3];
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bpart[M];
#pragma unroll
    for (int pi = 0; pi < M; ++pi) bpart[pi] = 0.f;
    float cnt_acc = 0.f;
    wave_accumulate<KP, false, SPLIT>(p, beg, end, G, Wab, acc, bpart, cnt_acc);
    reduce_bpart<M>(bpart);
    const float cnt = wave_sum(cnt_acc);
    float* dst = STORE ? seg_ws + (int64_t)sgi * ws_stride(KP) : ws + slot * ws_stride(KP);
    int t = 0;
#pragma unroll
    for (int pi = 0; pi < M; ++pi) {
      // per-tile addresses formed here from opaque lane coordinates: hoisted out of the
      // unrolled loops, the 2 x NT x 4 atomic addresses did not fit the register file at KP=128
      int gg = g, ff = fl;
      asm volatile("" : "+v"(gg), "+v"(ff));
#pragma unroll
      for (int qi = 0; qi <= pi; ++qi, ++t)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int i = pi * 16 + gg * 4 + v, j = qi * 16 + ff;
          if constexpr (STORE) {
            dst[i * KP + j] = acc[t][v];
            if (pi != qi) dst[j * KP + i] = acc[t][v];
          } else {
            atomicAdd(dst + i * KP + j, acc[t][v]);
            if (pi != qi) atomicAdd(dst + j * KP + i, acc[t][v]);
          }
        }
    }
    // after the reduction lane (g, fl) holds b[pi*16 + fl] for every pi: lane l adds
    // features l and l + 64
    if constexpr (STORE) {
      if (lane < KP) dst[KP * KP + lane] = pick_bpart<M>(bpart, g);
      if (lane + 64 < KP) dst[KP * KP + 64 + lane] = pick_bpart<M>(bpart, g + 4);
      if (lane == 0) dst[KP * KP + KP] = cnt;
    } else {
      if (lane < KP) atomicAdd(dst + KP * KP + lane, pick_bpart<M>(bpart, g));
      if (lane + 64 < KP) atomicAdd(dst + KP * KP + 64 + lane, pick_bpart<M>(bpart, g + 4));
      if (lane == 0) atomicAdd(dst + KP * KP + KP, cnt);
    }
  }
}


// Sum of each long row's segment records (STORE mode of als_partial): block (slot, chunk)
// adds up floats [256 chunk, 256 chunk + 256) of the slot's records, in segment order (the
// segments of a slot are contiguous in segs, slot-major).
// flags (nullable): flags[slot] += 1 once a block's part of the record is written (the
// batched solve, running concurrently, waits for all of a record's blocks).
__global__ __launch_bounds__(256) void als_partial_reduce(const int64_t* __restrict__ segs,
                                                         int n_seg, const float* __restrict__ seg_ws,
                                                         float* __restrict__ ws, int stride,
                                                         unsigned* __restrict__ flags) {
  __shared__ int s_lo, s_hi;
  const int slot = blockIdx.x;
  if (threadIdx.x == 0) {
    int lo = 0, hi = n_seg;                     // first segment with slot >= this one
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (segs[4 * (int64_t)mid + 1] < slot) lo = mid + 1; else hi = mid;
    }
    int e = lo;
    while (e < n_seg && segs[4 * (int64_t)e + 1] == slot) ++e;
    s_lo = lo;
    s_hi = e;
  }
  __syncthreads();
  const int f = blockIdx.y * 256 + threadIdx.x;
  if (f < stride) {
    float acc = 0.f;
    for (int sg = s_lo; sg < s_hi; ++sg) acc += seg_ws[(int64_t)sg * stride + f];
    ws[(int64_t)slot * stride + f] = acc;
  }
  if (flags) {
    __threadfence();   // this block's writes, agent scope, before the count goes up
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(flags + slot, 1u);
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

// The superseded solve kernels' dispatch (tuning/als_variants.hip), linked only into the
// tuning build; null here otherwise.
extern "C" __attribute__((weak)) int oryx_als_solve_variant(
    const oryx_als::AlsParams& p, int kp, int split, int variant, int wide, int max_blocks,
    int panel_blocks, hipStream_t s);

// KP <= 64 solve kernel: 5 = als_solve_batch (als_batch.hip: four rows per wave, batched
// block-LDL^T), 2 = als_solve_panel with three chunks of gathers in flight at 2 waves
// per SIMD, 0 = als_solve_panel with one chunk in flight at 3 waves per SIMD, 1 =
// als_solve_wave (register column Cholesky), 3 (default) / 4 = variant 2 with the
// factorisation at raised issue priority (s_setprio 2 / 3: 2-6% faster half-steps than 2)
static int g_als_variant = 5;
// 64 < KP <= 128 and the fp32 factor mode: 2 (default, with variant 5) = als_solve_batch_gl
// (als_batch.hip: LDS-DMA gather, batched block LDL^T; rank-128 fp32 12.3 ms per iteration vs
// 13.9 for als_solve_wide); 0 = als_solve_wide (fp32 mode at KP <= 64: als_solve_wave),
// 1 = als_solve_block (LDS Cholesky, bf16 only)
static int g_als_wide_variant = 2;

extern "C" {

int oryx_als_set_variant(int v) {
  if (v < 0 || v > 5 || (v != 5 && !oryx_als_solve_variant)) return ORYX_EINVAL;
  g_als_variant = v;
  return ORYX_OK;
}

int oryx_als_get_variant() { return g_als_variant; }

int oryx_als_get_wide_variant() { return g_als_wide_variant; }

int oryx_als_set_wide_variant(int v) {
  if (v < 0 || v > 2 || (v != 2 && !oryx_als_solve_variant)) return ORYX_EINVAL;
  g_als_wide_variant = v;
  return ORYX_OK;
}

// long_slot [n_work] (nullable) marks split rows; segs [n_seg][4] = (row, slot, beg, end);
// ws: workspace of n_long * ws_stride(kp) floats (zeroed here).
// epoch (1, 2, ... per workspace; 0: no overlap): the long rows' partial sums run on a side
// stream concurrently with the batched solve, which waits per long row on the flags after
// the workspace's records (zeroed when the workspace was allocated).
int oryx_als_solve(const int64_t* row_ptr, const int32_t* row_ids, const int32_t* col_idx,
                   const float* vals, const void* Y, const float* YtY, float* X, void* Xb,
                   int n_work, int k, int kp, float lambda, float alpha, int implicit,
                   int* fail_count, const int32_t* long_slot, const int64_t* segs, int n_seg,
                   int n_long, float* ws, int split, long long nnz, unsigned epoch,
                   void* stream) {
  if (n_work <= 0) return ORYX_OK;
  if (n_seg > 0 && (!long_slot || !segs || !ws || n_long <= 0)) return ORYX_EINVAL;
  AlsParams p{row_ptr, row_ids, col_idx, vals, reinterpret_cast<const __bf16*>(Y), YtY, X,
              reinterpret_cast<__bf16*>(Xb), n_work, k, lambda, alpha, implicit, fail_count,
              n_seg > 0 ? long_slot : nullptr, ws};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // grid caps (the waves loop over rows with a stride of 4 x grid).  The 2-wave-per-SIMD panel
  // kernels run best as one resident generation, 2 blocks per CU: 512 blocks on MI355X
  // measured 2.14-2.16 ms per rank-64 iteration against 2.18-2.19 ms at 4096
  // (profiles/r2_als_grid_sweep.txt); the one-wave wide kernels and als_partial keep 4096
  // (rank 128 fp32: 13.86 ms at 4096, 14.0 at 512).  ORYX_ALS_MAX_BLOCKS overrides both.
  static const int env_blocks = [] {
    const char* e = getenv("ORYX_ALS_MAX_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v >= 64 && v <= 65536 ? v : 0;
  }();
  static const int resident_panel_blocks = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    return 2 * cus;
  }();
  const int max_blocks = env_blocks ? env_blocks : 256 * 16;
  const bool deep = g_als_variant >= 2 && g_als_variant <= 4;
  const int panel_blocks = env_blocks ? env_blocks : (deep ? resident_panel_blocks : 256 * 16);
  // long rows: segment records stored, then reduced per row (ws: n_long reduced records
  // followed by n_seg segment records); ORYX_ALS_PARTIAL_ATOMIC=1: the older atomic adds
  static const bool atomic_partial = [] {
    const char* e = getenv("ORYX_ALS_PARTIAL_ATOMIC");
    return e && atoi(e) == 1;
  }();
  // the overlap needs the batched kernels (they wait per long row) and the stored records
  const bool batched = g_als_variant == 5 && (g_als_wide_variant == 2 || (!split && kp <= 64));
  const bool overlap = n_seg > 0 && epoch > 0 && batched && !atomic_partial;
  hipStream_t ps = s;   // the stream of the long rows' partial sums
  hipEvent_t done = nullptr;
  if (overlap) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return ORYX_ELAUNCH;
    static hipStream_t side[16] = {};
    static hipEvent_t ev_in[16] = {}, ev_done[16] = {};
    if (!side[dev]) {
      if (hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&ev_in[dev], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&ev_done[dev], hipEventDisableTiming) != hipSuccess)
        return ORYX_ELAUNCH;
    }
    // the side stream starts after everything already queued on s (the factors it reads)
    if (hipEventRecord(ev_in[dev], s) != hipSuccess ||
        hipStreamWaitEvent(side[dev], ev_in[dev], 0) != hipSuccess)
      return ORYX_ELAUNCH;
    ps = side[dev];
    done = ev_done[dev];
  }
  if (n_seg > 0) {
    // ws: n_long reduced records | n_seg segment records | n_long uint32 flags
    const int stride = ws_stride(kp);
    float* seg_ws = ws + (size_t)n_long * stride;
    // (counted at every epoch, overlapped or not, so that they keep pace with the epochs)
    unsigned* flags = epoch > 0 && !atomic_partial
                          ? reinterpret_cast<unsigned*>(ws + (size_t)(n_long + n_seg) * stride)
                          : nullptr;
    if (atomic_partial &&
        hipMemsetAsync(ws, 0, sizeof(float) * (size_t)n_long * stride, s) != hipSuccess)
      return ORYX_ELAUNCH;
    int blocks = (n_seg + 3) / 4;
    if (blocks > max_blocks) blocks = max_blocks;
    switch (kp) {
#define PART_CASE(KPV)                                                                    \
  case KPV:                                                                               \
    if (atomic_partial) {                                                                 \
      if (split)                                                                          \
        hipLaunchKernelGGL((als_partial<KPV, true>), dim3(blocks), dim3(256), 0, s, p,     \
                           segs, n_seg, ws, nullptr);                                     \
      else                                                                                \
        hipLaunchKernelGGL((als_partial<KPV, false>), dim3(blocks), dim3(256), 0, s, p,    \
                           segs, n_seg, ws, nullptr);                                     \
    } else {                                                                              \
      if (split)                                                                          \
        hipLaunchKernelGGL((als_partial<KPV, true, true>), dim3(blocks), dim3(256), 0, ps, \
                           p, segs, n_seg, ws, seg_ws);                                   \
      else                                                                                \
        hipLaunchKernelGGL((als_partial<KPV, false, true>), dim3(blocks), dim3(256), 0,    \
                           ps, p, segs, n_seg, ws, seg_ws);                               \
    }                                                                                     \
    break;
      PART_CASE(16)
      PART_CASE(32)
      PART_CASE(48)
      PART_CASE(64)
      PART_CASE(80)
      PART_CASE(96)
      PART_CASE(112)
      PART_CASE(128)
#undef PART_CASE
      default:
        return ORYX_EINVAL;
    }
    if (!atomic_partial) {
      const unsigned chunks = (unsigned)((stride + 255) / 256);
      hipLaunchKernelGGL(als_partial_reduce, dim3((unsigned)n_long, chunks), dim3(256), 0, ps,
                         segs, n_seg, seg_ws, ws, stride, flags);
      if (overlap) {
        // the batched solve takes the long rows (first in row_ids) last and waits for each
        // row's record: every one of its `chunks` reduce blocks of this epoch counted
        p.rot = n_long < n_work ? n_long : 0;
        p.part_flags = flags;
        p.part_want = epoch * chunks;
        if (hipEventRecord(done, ps) != hipSuccess) return ORYX_ELAUNCH;
      }
    }
  }
  if (oryx_check_launch() != ORYX_OK) return ORYX_ELAUNCH;
  int rc = -1;
  if (g_als_variant == 5 && g_als_wide_variant == 2 && (split || kp > 64)) {
    // two rows per wave, LDS-DMA gather (als_batch.hip): 64 < KP <= 128 and the fp32 mode
    const int cus = resident_panel_blocks / 2;
    const long long mean_len = n_work > 0 ? nnz / n_work : 0;
    rc = oryx_als::batch_gl_launch(p, kp, split != 0, env_blocks ? env_blocks : cus, mean_len,
                                   s);
  } else if (g_als_variant == 5 && !split && kp <= 64) {
    // two rows per wave, two waves per SIMD (als_batch.hip)
    const int cus = resident_panel_blocks / 2;
    rc = oryx_als::batch_solve_launch(p, kp, env_blocks ? env_blocks : cus, s);
  }
  if (rc >= 0) {
    // later work on s (the next half-step rewrites the workspace) follows the side stream
    if (done && hipStreamWaitEvent(s, done, 0) != hipSuccess) return ORYX_ELAUNCH;
    return rc;
  }
  // a superseded kernel selected for an A/B run: only in the tuning build
  if (!oryx_als_solve_variant) return ORYX_EINVAL;
  return oryx_als_solve_variant(p, kp, split, g_als_variant, g_als_wide_variant, max_blocks,
                                panel_blocks, s);
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

// analysis: subsequent KP=64 variant-5 solves count per-phase cycles into prof[0..6]
// (7 u64, zeroed by the caller; nullptr switches it off)
int oryx_als_batch_profile(unsigned long long* prof) {
  oryx_als::batch_set_profile(prof);
  return ORYX_OK;
}

// 1 when the superseded kernels (tuning/als_variants.hip) are linked into this library
int oryx_als_tuning_available() { return oryx_als_solve_variant ? 1 : 0; }

int oryx_kernels_version() { return 29; }

int oryx_als_ws_stride(int kp) { return ws_stride(kp); }

}  // extern "C"
