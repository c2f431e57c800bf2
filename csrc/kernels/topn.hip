// topn.hip -- fused batched top-N scan of the ALS serving model.
//
// Replaces the reference's per-request thread-pool scan of LSH partitions with bounded heaps
// ([serving-app]/als/model/ALSServingModel.java:289-335, TopNConsumer.java:55-74,
// LocalitySensitiveHash.java:156-177).  One launch scores up to 16 queries against the item
// matrix and leaves each (wave, query) pair's KL best candidates; a small device top-k merges
// them.  MI355X design:
//   * the item matrix is read IN PLACE from the feature store's device mirror (fp32 rows of
//     stride ld, a multiple of 16, zero padded): the index only holds a bucket-sorted
//     permutation (position -> store row), so a query's candidate buckets are contiguous
//     position ranges and only the union of the batch's candidate ranges is read, and there is
//     one device copy of Y (a 20M x 250 model fits in ~21 GiB);
//   * scores on v_mfma_f32_16x16x4_f32: A = 16 item rows (one 16-byte load per lane per 16
//     features, four MFMAs per load), B = the 16 queries held in registers for the whole
//     kernel, C = 16 items x 16 queries (lane: 4 items of query lane & 15);
//   * software pipelined: the next tile's rows are loaded before this tile's epilogue runs;
//   * cosine: each row's norm is summed from the A operand already in registers (no norm
//     array), then moved to the C layout with four lane shuffles;
//   * epilogue: per-query candidate-bucket bit, then a per-(wave, query) threshold test --
//     only scores above the query's current KL-th best enter an LDS buffer (2 KL slots);
//     excluded items are binary-searched only for those; a full buffer is cut back to its
//     best KL by a wave bitonic sort, raising the threshold;
//   * KL = 64 (the common howMany + offset), 256 or 1024 candidates per (wave, query): deep
//     requests run in the same single pass (LDS is sized for the launch's queries only);
//   * waves take equal contiguous shares of the union's 16-row tiles, so the scan is one
//     streaming pass over HBM.

#include "common.h"

namespace {

constexpr int QB = 16;     // queries per launch (MFMA N)
constexpr int WPB = 2;     // waves per block

struct TopnParams {
  const float* Y;             // store rows, stride ld floats (ld >= kp, pad columns zero)
  const __bf16* Yb;           // bf16 scan: the rows' bf16 mirror, stride ldb (>= kp, pad 0)
  long long ldb;
  const int* perm;            // [n] position -> store row (null: identity)
  long long ld;
  const float* Q;             // [QB][kp] (rows >= nq zero)
  int nq;
  int cosine;
  const int* bucket_of;       // [n] bucket id per position (null: no LSH mask)
  const unsigned* cand_bits;  // [nq][words] candidate-bucket bitmap
  int words;
  const long long* ranges;    // [n_ranges][2] positions to scan, ascending, disjoint
  const long long* tile0;     // [n_ranges + 1] prefix count of 16-row tiles
  int n_ranges;
  long long n_tiles;
  const int* excl_ptr;        // [nq + 1] (null: none)
  const int* excl_rows;       // sorted excluded positions per query
  float* out_score;           // [n_waves][nq][KL]
  int* out_row;               // [n_waves][nq][KL] positions
};

__device__ __forceinline__ bool excluded(const TopnParams& p, int q, int pos) {
  if (!p.excl_ptr) return false;
  int lo = p.excl_ptr[q], hi = p.excl_ptr[q + 1];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const int v = p.excl_rows[mid];
    if (v == pos) return true;
    if (v < pos) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// descending bitonic sort of CAP (score, row) pairs in LDS by one wave; -inf pads
template <int CAP>
__device__ __forceinline__ void wave_sort_desc(float* sc, int* rw, int lane) {
  for (int k = 2; k <= CAP; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int p = lane; p < CAP / 2; p += 64) {
        // pair p: i = 2j (p / j) + p % j, partner i + j
        const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1));
        const int l = i + j;
        const float a = sc[i], b = sc[l];
        const int ra = rw[i], rb = rw[l];
        const bool desc = (i & k) == 0;
        const bool swap = desc ? (a < b) : (a > b);
        if (swap) {
          sc[i] = b;
          sc[l] = a;
          rw[i] = rb;
          rw[l] = ra;
        }
      }
      wave_sync();
    }
  }
}

// Cut query q's buffer back to its best KL entries; returns the new threshold (the KL-th).
template <int KL>
__device__ __forceinline__ float compact(float* sc, int* rw, int* cnt, int q, int lane) {
  constexpr int CAP = 2 * KL;
  float* s = sc + q * CAP;
  int* r = rw + q * CAP;
  const int c = cnt[q];
  for (int i = lane; i < CAP; i += 64)
    if (i >= c) {
      s[i] = -INFINITY;
      r[i] = -1;
    }
  wave_sync();
  wave_sort_desc<CAP>(s, r, lane);
  if (lane == 0) cnt[q] = c < KL ? c : KL;
  wave_sync();
  return c >= KL ? s[KL - 1] : -INFINITY;
}

// BF: scores from the bf16 mirror (queries rounded to bf16 too) on
// v_mfma_f32_16x16x32_bf16 -- half the bytes of the fp32 scan; the caller re-ranks the
// candidates exactly in fp32 and certifies the cut (ops/topn.py ItemIndex._launch_bf16).
// KP % 32 == 0 there, no cosine.
template <int KP, int KL, bool BF>
__global__ __launch_bounds__(WPB * 64) void topn_scan(TopnParams p) {
  constexpr int S = KP / 16;
  constexpr int SB = BF ? KP / 32 : 1;
  constexpr int CAP = 2 * KL;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nq = p.nq;
  // per wave: scores [nq][CAP], rows [nq][CAP], counts [QB]
  unsigned char* base = smem + (size_t)wave * ((size_t)nq * CAP * 8 + QB * 4);
  float* sc = reinterpret_cast<float*>(base);
  int* rw = reinterpret_cast<int*>(base + (size_t)nq * CAP * 4);
  int* cnt = reinterpret_cast<int*>(base + (size_t)nq * CAP * 8);
  if (lane < QB) cnt[lane] = 0;
  const int q = lane & 15, kg = lane >> 4;
  // B operand (queries) for every 16-feature step, resident: component j of step s is
  // Q[q][16 s + 4 kg + j]
  f32x4 qb[BF ? 1 : S];
  bf16x8 qb8[SB];
  if constexpr (BF) {
    // lane (q, kg) holds Q[q][32 s + 8 kg .. + 7] for every 32-feature step
#pragma unroll
    for (int s = 0; s < SB; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) qb8[s][j] = (__bf16)p.Q[q * KP + 32 * s + 8 * kg + j];
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s)
      qb[s] = *reinterpret_cast<const f32x4*>(p.Q + q * KP + 16 * s + 4 * kg);
  }
  float theta = -INFINITY;   // this lane's query's admission threshold
  const unsigned* cbits = p.cand_bits ? p.cand_bits + (long long)(q < nq ? q : 0) * p.words
                                      : nullptr;
  wave_sync();

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
  // A: item position i0 + (lane & 15), features 16 s + 4 kg .. + 3
  f32x4 a[BF ? 1 : S];
  bf16x8 a8[SB];
  long long i0 = 0, rend = 0;
  auto load_tile = [&](long long t) {
    while (t >= p.tile0[r + 1]) ++r;
    const long long rbeg = p.ranges[2 * r];
    rend = p.ranges[2 * r + 1];
    i0 = rbeg + 16 * (t - p.tile0[r]);
    const long long ia = i0 + (lane & 15) < rend ? i0 + (lane & 15) : rend - 1;
    const long long row = p.perm ? (long long)p.perm[ia] : ia;
    if constexpr (BF) {
      const __bf16* yrow = p.Yb + row * p.ldb + 8 * kg;
#pragma unroll
      for (int s = 0; s < SB; ++s) a8[s] = *reinterpret_cast<const bf16x8*>(yrow + 32 * s);
    } else {
      const float* yrow = p.Y + row * p.ld + 4 * kg;
#pragma unroll
      for (int s = 0; s < S; ++s) a[s] = *reinterpret_cast<const f32x4*>(yrow + 16 * s);
    }
  };
  if (t_beg < t_end) load_tile(t_beg);
  for (long long t = t_beg; t < t_end; ++t) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float ss = 0.f;
    if constexpr (BF) {
#pragma unroll
      for (int s = 0; s < SB; ++s)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8[s], qb8[s], acc, 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][j], qb[s][j], acc, 0, 0, 0);
          ss += a[s][j] * a[s][j];
        }
      }
    }
    const long long c_i0 = i0, c_rend = rend;
    // the next tile's rows are in flight while this tile's epilogue runs
    if (t + 1 < t_end) load_tile(t + 1);
    float inv4[4] = {1.f, 1.f, 1.f, 1.f};
    if (!BF && p.cosine) {
      // row (lane & 15)'s squared norm: sum over the four feature groups (lanes +16, +32, +48)
      ss += __shfl_xor(ss, 16);
      ss += __shfl_xor(ss, 32);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float n2 = __shfl(ss, 4 * kg + v);
        inv4[v] = n2 > 0.f ? 1.f / sqrtf(n2) : 0.f;
      }
    }
    // C: lane holds items c_i0 + 4 kg + v of query q
    bool any = false;
    float v4[4];
    int r4[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const long long it = c_i0 + 4 * kg + v;
      const float sv = acc[v] * inv4[v];
      bool ok = it < c_rend && q < nq;
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
      wave_sync();
      // queries whose buffer cannot take another tile (16 entries) are cut back to KL
      const int my = lane < nq ? cnt[lane] : 0;
      unsigned long long full = __ballot(lane < nq && my > CAP - 16);
      while (full) {
        const int fq = __builtin_ctzll(full);
        full &= full - 1;
        const float th = compact<KL>(sc, rw, cnt, fq, lane);
        if (q == fq) theta = th;
      }
    }
  }
  // final: every query's best KL (sorted) to global
  const long long ob = w * nq * KL;
  for (int fq = 0; fq < nq; ++fq) {
    compact<KL>(sc, rw, cnt, fq, lane);
    for (int i = lane; i < KL; i += 64) {
      p.out_score[ob + fq * KL + i] = sc[fq * CAP + i];
      p.out_row[ob + fq * KL + i] = rw[fq * CAP + i];
    }
  }
}

constexpr size_t kLdsBudget = 160u * 1024u;

size_t lds_bytes(int kl, int nq) { return (size_t)WPB * ((size_t)nq * 2 * kl * 8 + QB * 4); }

}  // namespace

extern "C" {

// Most queries one launch can hold for a per-(wave, query) list of `kl` candidates (LDS).
int oryx_topn_max_queries(int kl) {
  int nq = QB;
  while (nq > 1 && lds_bytes(kl, nq) > kLdsBudget) --nq;
  return lds_bytes(kl, nq) <= kLdsBudget ? nq : 0;
}

// Number of waves the scan uses for n_tiles 16-row tiles with `kl` candidates per (wave,
// query) (the caller sizes out_* to waves * nq * kl).
long long oryx_topn_waves_kl(long long n_tiles, int kl) {
  // ~8 tiles per wave at least; at most 8 waves per SIMD of 256 CUs for kl = 64, and at
  // least 2 per SIMD for the deep lists (their candidate output and final sorts grow with
  // kl; with 2 waves per CU the 1024-deep scan of 20M x 250 ran at half the bandwidth)
  // 32 tiles (512 rows) per wave, but at least 512 waves while a wave still gets 8 tiles:
  // fewer, longer per-wave lists make the host-side merge (a top-k over waves x kl
  // candidates) cheaper -- 16 queries top-10 over 1M x 50 at LSH 0.3: 1.11 -> 0.86 ms --
  // with the same scan time at 20M x 250 (r4_topn_*_tpw*).  ORYX_TOPN_TILES_PER_WAVE
  // overrides the 32 (sweeps).
  static const long long tpw = [] {
    const char* e = getenv("ORYX_TOPN_TILES_PER_WAVE");
    const long long v = e ? atoll(e) : 32;
    return v > 0 ? v : 32;
  }();
  long long w = (n_tiles + tpw - 1) / tpw;
  const long long floor_w = std::min<long long>(512, (n_tiles + 7) / 8);
  if (w < floor_w) w = floor_w;
  long long cap = 256 * 4 * 8 / (kl / 64 > 0 ? kl / 64 : 1);
  if (cap < 2048) cap = 2048;
  if (w > cap) w = cap;
  if (w < 1) w = 1;
  return (w + WPB - 1) / WPB * WPB;
}

long long oryx_topn_waves(long long n_tiles) { return oryx_topn_waves_kl(n_tiles, 64); }

// Y fp32 rows (stride ld) or, with Yb non-null, the bf16 mirror (stride ldb; kp % 32 == 0,
// cosine 0, kl 64): the bf16 scan.
int oryx_topn_scan3(const float* Y, const __bf16* Yb, long long ldb, const int* perm,
                    long long ld, const float* Q, int kp, int nq, int cosine, int kl,
                    const int* bucket_of, const unsigned* cand_bits, int words,
                    const long long* ranges, const long long* tile0, int n_ranges,
                    long long n_tiles, const int* excl_ptr, const int* excl_rows,
                    float* out_score, int* out_row, void* stream) {
  if (nq <= 0 || nq > QB || n_ranges <= 0 || n_tiles <= 0) return ORYX_EINVAL;
  if (cand_bits && !bucket_of) return ORYX_EINVAL;
  const bool bf = Yb != nullptr;
  if (bf ? (ldb < kp || ldb % 8 != 0 || kp % 32 != 0 || cosine || kl != 64)
         : (ld < kp || ld % 4 != 0))
    return ORYX_EINVAL;
  if (nq > oryx_topn_max_queries(kl)) return ORYX_EINVAL;
  TopnParams p{Y, Yb, ldb, perm, ld, Q, nq, cosine, bucket_of, cand_bits, words, ranges,
               tile0, n_ranges, n_tiles, excl_ptr, excl_rows, out_score, out_row};
  const long long waves = oryx_topn_waves_kl(n_tiles, kl);
  const unsigned blocks = (unsigned)(waves / WPB);
  const size_t lds = lds_bytes(kl, nq);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define TOPN_CASE3(KPV, KLV, BFV)                                                        \
  if (kp == KPV && kl == KLV && bf == BFV) {                                             \
    static bool attr_set = false;                                                        \
    if (!attr_set && lds > 65536) {                                                      \
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topn_scan<KPV, KLV, BFV>),  \
                              hipFuncAttributeMaxDynamicSharedMemorySize,                \
                              (int)kLdsBudget) != hipSuccess)                            \
        return ORYX_ELAUNCH;                                                             \
      attr_set = true;                                                                   \
    }                                                                                    \
    hipLaunchKernelGGL((topn_scan<KPV, KLV, BFV>), dim3(blocks), dim3(WPB * 64), lds, s, \
                       p);                                                               \
    return oryx_check_launch();                                                          \
  }
#define TOPN_CASE(KPV, KLV) TOPN_CASE3(KPV, KLV, false)
#define TOPN_KP(KPV) TOPN_CASE(KPV, 64) TOPN_CASE(KPV, 256) TOPN_CASE(KPV, 1024)
#define TOPN_BF(KPV) TOPN_CASE3(KPV, 64, true)
  TOPN_BF(32)
  TOPN_BF(64)
  TOPN_BF(96)
  TOPN_BF(128)
  TOPN_BF(160)
  TOPN_BF(192)
  TOPN_BF(256)
  TOPN_KP(16)
  TOPN_KP(32)
  TOPN_KP(48)
  TOPN_KP(64)
  TOPN_KP(80)
  TOPN_KP(96)
  TOPN_KP(112)
  TOPN_KP(128)
  TOPN_KP(160)
  TOPN_KP(192)
  TOPN_KP(256)
#undef TOPN_BF
#undef TOPN_KP
#undef TOPN_CASE
#undef TOPN_CASE3
  return ORYX_EINVAL;
}

int oryx_topn_scan2(const float* Y, const int* perm, long long ld, const float* Q, int kp,
                    int nq, int cosine, int kl, const int* bucket_of,
                    const unsigned* cand_bits, int words, const long long* ranges,
                    const long long* tile0, int n_ranges, long long n_tiles,
                    const int* excl_ptr, const int* excl_rows, float* out_score, int* out_row,
                    void* stream) {
  return oryx_topn_scan3(Y, nullptr, 0, perm, ld, Q, kp, nq, cosine, kl, bucket_of, cand_bits,
                         words, ranges, tile0, n_ranges, n_tiles, excl_ptr, excl_rows,
                         out_score, out_row, stream);
}

}  // extern "C"
