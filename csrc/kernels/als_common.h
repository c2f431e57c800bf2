// als_common.h -- pieces shared by the ALS solve kernels (als.hip, als_batch.hip).
#pragma once
#include "common.h"

#include <type_traits>

namespace oryx_als {

// Parameters of one ALS half-step solve (see csrc/kernels/als.hip for the math).
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
  // split long rows: work item w with long_slot[w] >= 0 takes its Gramian, b and count from
  // ws[slot] (summed beforehand by als_partial over fixed-size segments of the row)
  const int32_t* long_slot;  // [n_work] (nullable)
  const float* ws;           // [n_long][ws_stride(KP)]
  // the long rows' records are reduced on a concurrent stream while the batched solve runs:
  // it takes its work items rotated by rot (the long rows, first in row_ids, come last) and
  // waits until part_flags[slot] reaches part_want before reading ws[slot] (nullable: the
  // records were complete before the launch)
  int rot = 0;
  const unsigned* part_flags = nullptr;
  unsigned part_want = 0;
};

// Wait (lane 0 of the wave, bounded) until a long row's reduced record is complete, then
// acquire at agent scope: the record was written on other CUs / XCDs.  A timeout (2 s) marks
// the solve failed (fail_count += 2^20) instead of hanging the GPU.
#ifndef ORYX_ALS_NO_PART_WAIT
#define ORYX_ALS_NO_PART_WAIT 0
#endif
__device__ __forceinline__ void wait_long_row(const AlsParams& p, int slot) {
  if (ORYX_ALS_NO_PART_WAIT || !p.part_flags) return;
  if ((threadIdx.x & 63) == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(p.part_flags + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           p.part_want) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
        if (p.fail_count) atomicAdd(p.fail_count, 1 << 20);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __builtin_amdgcn_wave_barrier();
}

// als_batch.hip: four rows per wave, block-LDL^T solve (KP <= 64, bf16 factors)
int batch_solve_launch(const AlsParams& p, int kp, int max_blocks, hipStream_t s);
// als_batch.hip: two rows per wave, LDS-DMA gather (64 < KP <= 128, and the fp32 factor mode)
int batch_gl_launch(const AlsParams& p, int kp, bool split, int cus, long long mean_len,
                    hipStream_t s);
// analysis: route KP=64 batch launches to the per-phase cycle counting build (nullptr: off)
void batch_set_profile(unsigned long long* prof);

}  // namespace oryx_als

namespace {

using oryx_als::AlsParams;

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>) (or descending); the body
// sees its index as a constant, so register arrays indexed by it never fall back to scratch
// (#pragma unroll gives up on very large bodies)
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (N > 0) {
    static_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}
template <int N, typename F>
__device__ __forceinline__ void static_for_desc(F&& f) {
  if constexpr (N > 0) {
    f(std::integral_constant<int, N - 1>{});
    static_for_desc<N - 1>(f);
  }
}

// fp32 factor mode (SPLIT kernels): every factor row is stored as 2*KP bf16, the hi part
// bf16(y) followed by the lo part bf16(y - hi), so hi + lo = y to ~2^-17 relative; the Gramian
// takes s_hi*y_hi + s_lo*y_hi + s_hi*y_lo (s = c*y in fp32, split the same way).  Y, Xb and the
// gathered operands then have a row stride of 2*KP.
template <bool SPLIT, int KP>
__device__ __forceinline__ void store_xb(__bf16* Xb, int64_t row, int c, float x) {
  const __bf16 h = (__bf16)x;
  if constexpr (SPLIT) {
    Xb[row * 2 * KP + c] = h;
    Xb[row * 2 * KP + KP + c] = (__bf16)(x - (float)h);
  } else {
    Xb[row * KP + c] = h;
  }
}

// workspace record of one split row: full symmetric A [KP*KP], b [KP], count, padded to 16 B
__host__ __device__ constexpr int ws_stride(int kp) { return (kp * kp + kp + 1 + 3) / 4 * 4; }

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

// Gathered chunk image in LDS: 32 rating rows x KP bf16, row-major (KP*2 bytes per row),
// written lane-linearly (lane l of staging instruction `it` owns 16-byte slot it*64 + l).  The
// 16-byte chunks of row r are rotated by rot(r) so that the ds_read_b64_tr_b16 operand reads
// (4 ratings x 16 features per 16-lane group) are bank-conflict free (KP 32/64/96/128) or
// 2-way (others); the rotation is applied on the GLOBAL side: slot (r, sc) holds feature
// chunk (sc + rot(r)) % PPR.  Constants found by exhaustive search over the bank model.
template <int KP>
struct ChunkImage {
  static constexpr int PPR = KP / 8;              // 16-byte chunks per row
  static constexpr int NPL = KP / 16;             // staging slots per lane (32*PPR/64)
  static constexpr int BYTES = 32 * KP * 2;
  static constexpr int SM = KP == 64 ? 1 : KP == 128 ? 2 : 0;
  static constexpr int ST = KP == 64 ? 2 : KP == 128 ? 4 : (KP == 32 || KP == 96) ? 1 : 0;
  __device__ static constexpr int rot(int r) { return (r * SM + (r >> 2) * ST) % PPR; }
};

// sum the per-lane b partials over the 4 lane groups; lane f then takes feature f (+64h)
template <int M>
__device__ __forceinline__ void reduce_bpart(float (&bpart)[M]) {
#pragma unroll
  for (int pi = 0; pi < M; ++pi) {
    bpart[pi] += __shfl_xor(bpart[pi], 16, 64);
    bpart[pi] += __shfl_xor(bpart[pi], 32, 64);
  }
}

template <int M>
__device__ __forceinline__ float pick_bpart(const float (&bpart)[M], int sel) {
  float r = bpart[0];
#pragma unroll
  for (int pi = 1; pi < M; ++pi) r = sel == pi ? bpart[pi] : r;
  return r;
}

}  // namespace
