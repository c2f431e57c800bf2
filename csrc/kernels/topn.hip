// topn.hip -- fused batched top-N scan of the ALS serving model.
//
// Replaces the reference's per-request thread-pool scan of LSH partitions with bounded heaps
// ([serving-app]/als/model/ALSServingModel.java:289-335, TopNConsumer.java:55-74,
// LocalitySensitiveHash.java:156-177).  One launch scores up to 16 queries against the item
// matrix and leaves each (wave, query) pair's 64 best candidates; a small device top-k merges
// them.  MI355X design:
//   * Y is fp32 [n][kp] (kp a multiple of 16), rows sorted by LSH bucket, so a query's
//     candidate buckets are contiguous row ranges: only the union of the batch's candidate
//     ranges is read (sample-rate 0.3 reads ~30% of Y for one query);
//   * scores on v_mfma_f32_16x16x4_f32: A = 16 item rows (one 16-byte load per lane per 16
//     features, four MFMAs per load), B = the 16 queries held in registers for the whole
//     kernel, C = 16 items x 16 queries (lane: 4 items of query lane & 15);
//   * epilogue: cosine scale (1/|y|), per-query candidate-bucket bit, then a per-(wave,
//     query) threshold test -- only scores above the query's current 64th best enter an LDS
//     buffer (128 slots); known / excluded items are binary-searched only for those; a full
//     buffer is cut back to its best 64 by a wave bitonic sort, raising the threshold, so after
//     the first few tiles almost nothing is appended;
//   * waves take equal contiguous shares of the union's 16-row tiles (grid sized to the tile
//     count), so the scan is one streaming pass over HBM.

#include "common.h"

namespace {

constexpr int QB = 16;     // queries per launch (MFMA N)
constexpr int KL = 64;     // candidates kept per (wave, query)
constexpr int CAP = 128;   // LDS slots per (wave, query)
constexpr int WPB = 2;     // waves per block (2 x 32 KB of candidate buffers)

struct TopnParams {
  const float* Y;             // [n][kp] bucket-sorted
  const float* inv_norm;      // [n] (cosine) or null
  const float* Q;             // [QB][kp] (rows >= nq zero)
  int kp;
  int nq;
  const int* bucket_of;       // [n] bucket id per row (null: no LSH mask)
  const unsigned* cand_bits;  // [nq][words] candidate-bucket bitmap
  int words;
  const long long* ranges;    // [n_ranges][2] rows to scan, ascending, disjoint
  const long long* tile0;     // [n_ranges + 1] prefix count of 16-row tiles
  int n_ranges;
  long long n_tiles;
  const int* excl_ptr;        // [nq + 1] (null: none)
  const int* excl_rows;       // sorted row positions per query
  float* out_score;           // [n_waves][QB][KL]
  int* out_row;               // [n_waves][QB][KL]
};

__device__ __forceinline__ bool excluded(const TopnParams& p, int q, int row) {
  if (!p.excl_ptr) return false;
  int lo = p.excl_ptr[q], hi = p.excl_ptr[q + 1];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const int v = p.excl_rows[mid];
    if (v == row) return true;
    if (v < row) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

// descending bitonic sort of CAP (score, row) pairs in LDS by one wave (2 pairs per lane per
// step); -inf pads
__device__ __forceinline__ void wave_sort_desc(float* sc, int* rw, int lane) {
#pragma unroll
  for (int k = 2; k <= CAP; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      // pair p = lane: i = 2j(p / j) + p % j, partner i + j
      const int i = 2 * j * (lane / j) + (lane % j);
      const int l = i + j;
      const float a = sc[i], b = sc[l];
      const int ra = rw[i], rb = rw[l];
      const bool desc = (i & k) == 0;
      // descending blocks keep the larger first
      const bool swap = desc ? (a < b) : (a > b);
      if (swap) {
        sc[i] = b;
        sc[l] = a;
        rw[i] = rb;
        rw[l] = ra;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// Cut query q's buffer back to its best KL entries; returns the new threshold (the KL-th).
__device__ __forceinline__ float compact(float* sc, int* rw, int* cnt, int q, int lane) {
  float* s = sc + q * CAP;
  int* r = rw + q * CAP;
  const int c = cnt[q];
  for (int i = lane; i < CAP; i += 64)
    if (i >= c) {
      s[i] = -INFINITY;
      r[i] = -1;
    }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  wave_sort_desc(s, r, lane);
  if (lane == 0) cnt[q] = c < KL ? c : KL;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return c >= KL ? s[KL - 1] : -INFINITY;
}

template <int KP>
__global__ __launch_bounds__(WPB * 64) void topn_scan(TopnParams p) {
  constexpr int S = KP / 16;
  __shared__ float s_sc[WPB][QB * CAP];
  __shared__ int s_rw[WPB][QB * CAP];
  __shared__ int s_cnt[WPB][QB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* sc = s_sc[wave];
  int* rw = s_rw[wave];
  int* cnt = s_cnt[wave];
  if (lane < QB) cnt[lane] = 0;
  const int q = lane & 15, kg = lane >> 4;
  // B operand (queries) for every 16-feature step, resident: component j of step s is
  // Q[q][16 s + 4 kg + j]
  f32x4 qb[S];
#pragma unroll
  for (int s = 0; s < S; ++s)
    qb[s] = *reinterpret_cast<const f32x4*>(p.Q + q * KP + 16 * s + 4 * kg);
  float theta = -INFINITY;   // this lane's query's admission threshold
  const unsigned* cbits = p.cand_bits ? p.cand_bits + (long long)(q < p.nq ? q : 0) * p.words
                                      : nullptr;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();

  const long long nw = (long long)gridDim.x * WPB;
  const long long w = (long long)blockIdx.x * WPB + wave;
  const long long t_beg = p.n_tiles * w / nw, t_end = p.n_tiles * (w + 1) / nw;
  // locate the range of the first tile
  int r = 0;
  {
    int lo = 0, hi = p.n_ranges - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (p.tile0[mid] <= t_beg) lo = mid;
      else hi = mid - 1;
    }
    r = lo;
  }
  for (long long t = t_beg; t < t_end; ++t) {
    while (t >= p.tile0[r + 1]) ++r;
    const long long rbeg = p.ranges[2 * r], rend = p.ranges[2 * r + 1];
    const long long i0 = rbeg + 16 * (t - p.tile0[r]);
    // A: item row i0 + (lane & 15), features 16 s + 4 kg .. + 3
    const long long ia = i0 + (lane & 15) < rend ? i0 + (lane & 15) : rend - 1;
    const float* yrow = p.Y + ia * KP + 4 * kg;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(yrow + 16 * s);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], qb[s][j], acc, 0, 0, 0);
    }
    // C: lane holds items i0 + 4 kg + v of query q
    bool any = false;
    float v4[4];
    int r4[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const long long it = i0 + 4 * kg + v;
      float sv = acc[v];
      bool ok = it < rend && q < p.nq;
      if (ok && p.inv_norm) sv *= p.inv_norm[it];
      if (ok && cbits) {
        const int b = p.bucket_of[it];
        ok = (cbits[b >> 5] >> (b & 31)) & 1u;
      }
      ok = ok && sv > theta && !(sv != sv);
      if (ok && excluded(p, q, (int)it)) ok = false;
      v4[v] = ok ? sv : -INFINITY;
      r4[v] = (int)it;
      any |= ok;
    }
    if (__any(any)) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (v4[v] > -INFINITY) {
          const int pos = atomicAdd(&cnt[q], 1);
          sc[q * CAP + pos] = v4[v];
          rw[q * CAP + pos] = r4[v];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // queries whose buffer cannot take another tile (16 entries) are cut back to KL
      const int my = lane < QB ? cnt[lane] : 0;
      unsigned long long full = __ballot(lane < QB && my > CAP - 16);
      while (full) {
        const int fq = __builtin_ctzll(full);
        full &= full - 1;
        const float th = compact(sc, rw, cnt, fq, lane);
        if (q == fq) theta = th;
      }
    }
  }
  // final: every query's best KL (sorted) to global
  const long long ob = w * QB * KL;
  for (int fq = 0; fq < QB; ++fq) {
    compact(sc, rw, cnt, fq, lane);
    p.out_score[ob + fq * KL + lane] = sc[fq * CAP + lane];
    p.out_row[ob + fq * KL + lane] = rw[fq * CAP + lane];
  }
}

}  // namespace

extern "C" {

// Number of waves the scan uses for n_tiles 16-row tiles (the caller sizes out_* to
// waves * 16 * 64).
long long oryx_topn_waves(long long n_tiles) {
  // ~8 tiles per wave at least, at most 8 waves per SIMD of 256 CUs
  long long w = (n_tiles + 7) / 8;
  const long long cap = 256 * 4 * 8;
  if (w > cap) w = cap;
  if (w < 1) w = 1;
  return (w + WPB - 1) / WPB * WPB;
}

int oryx_topn_scan(const float* Y, const float* inv_norm, const float* Q, int kp, int nq,
                   const int* bucket_of, const unsigned* cand_bits, int words,
                   const long long* ranges, const long long* tile0, int n_ranges,
                   long long n_tiles, const int* excl_ptr, const int* excl_rows,
                   float* out_score, int* out_row, void* stream) {
  if (nq <= 0 || nq > QB || n_ranges <= 0 || n_tiles <= 0) return ORYX_EINVAL;
  if (cand_bits && !bucket_of) return ORYX_EINVAL;
  TopnParams p{Y, inv_norm, Q, kp, nq, bucket_of, cand_bits, words, ranges, tile0, n_ranges,
               n_tiles, excl_ptr, excl_rows, out_score, out_row};
  const long long waves = oryx_topn_waves(n_tiles);
  const unsigned blocks = (unsigned)(waves / WPB);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (kp) {
#define TOPN_CASE(KPV)                                                                \
  case KPV:                                                                           \
    hipLaunchKernelGGL(topn_scan<KPV>, dim3(blocks), dim3(WPB * 64), 0, s, p);        \
    break;
    TOPN_CASE(16)
    TOPN_CASE(32)
    TOPN_CASE(48)
    TOPN_CASE(64)
    TOPN_CASE(80)
    TOPN_CASE(96)
    TOPN_CASE(112)
    TOPN_CASE(128)
    TOPN_CASE(160)
    TOPN_CASE(192)
    TOPN_CASE(256)
#undef TOPN_CASE
    default:
      return ORYX_EINVAL;
  }
  return oryx_check_launch();
}

}  // extern "C"
