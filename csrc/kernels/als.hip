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

#include "als_common.h"

// 1: the next row's first chunk gathers are issued during this row's factorization
#ifndef ORYX_ALS_XROW_PREFETCH
#define ORYX_ALS_XROW_PREFETCH 0
#endif

#ifndef ORYX_ALS_PANEL_WAVES
#define ORYX_ALS_PANEL_WAVES 3
#endif

#ifndef ORYX_ALS_CHOL_LDS
#define ORYX_ALS_CHOL_LDS 1
#endif

namespace {

// bf16 factor mode: the MFMA A operand is bf16(c_i * y_i) (bf16 operands, fp32 accumulation;
// modelled exactly by solve_rows_reference(..., bf16_operands=True)).  ORYX_ALS_EXACT_C=1
// builds split c_i * y_i into bf16 hi + lo there too (one extra MFMA per tile, ~18% slower
// half-steps at rank 64); the fp32 factor mode (SPLIT kernels) always splits it.
#ifndef ORYX_ALS_EXACT_C
#define ORYX_ALS_EXACT_C 0
#endif
constexpr bool kExactC = ORYX_ALS_EXACT_C != 0;

constexpr int TS = 40;  // LDS row stride (bf16 elements) of the transposed chunk: 32 + 8 pad

// ------------------------------------------------------------------ wave-per-row kernel


template <int KP, bool SPLIT = false>
struct WaveSmem {
  static constexpr int AS = KP + 1;
  static constexpr int G_BYTES = ChunkImage<KP>::BYTES * (SPLIT ? 2 : 1);
  static constexpr int A_BYTES = KP * AS * 4;
  static constexpr int RAW = G_BYTES > A_BYTES ? G_BYTES : A_BYTES;
  // + 64 floats of per-rating weights (wa | wb) + 64 floats of the broadcast L column
  static constexpr int BYTES = (RAW + 15) / 16 * 16 + 256 + 256;
};

// Accumulate ratings [beg, end) of one row, one wave:
//   acc   += lower 16x16 tiles of sum_r wa_r y_r y_r^T   (v_mfma_f32_16x16x32_bf16)
//   bpart[pi] += sum over this lane's 8 ratings of wb_r * y_r[pi*16 + (lane&15)]
//   cnt_acc   += #positive ratings (lanes < 32)
// Software-pipelined one chunk deep: while the MFMAs of chunk c run, the 16-byte gathers of
// chunk c+1 and the (col, value) metadata of chunk c+2 are in flight in registers.  All
// gathers of a chunk are issued back to back (lanes past the row end re-read a valid row and
// get zero weights), then written lane-linearly into the chunk image and read back
// transposed with ds_read_b64_tr_b16 as the MFMA fragments.
template <int KP, bool INIT_YTY, bool SPLIT = false>
__device__ __forceinline__ void wave_accumulate(const AlsParams& p, int64_t beg, int64_t end,
                                                char* G, float* Wab,
                                                f32x4 (&acc)[(KP / 16) * (KP / 16 + 1) / 2],
                                                float (&bpart)[KP / 16], float& cnt_acc) {
  using CI = ChunkImage<KP>;
  constexpr int M = KP / 16;
  constexpr int PPR = CI::PPR;
  constexpr int NPL = CI::NPL;
  // INIT_YTY: the accumulators start at this lane's fragment of YtY (zeros for explicit
  // feedback), so A = YtY + sum c1 y yT comes out of the MFMA chain; the YtY loads are issued
  // after the first chunk's gathers so both latencies overlap
  auto init_yty = [&](int ln) {
    const int gg = ln >> 4, ff = ln & 15;
    int t = 0;
#pragma unroll
    for (int pi = 0; pi < M; ++pi)
#pragma unroll
      for (int qi = 0; qi <= pi; ++qi, ++t)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          acc[t][v] = p.YtY[(pi * 16 + gg * 4 + v) * KP + qi * 16 + ff];
  };
  if (beg >= end) {
    if (INIT_YTY) init_yty(threadIdx.x & 63);
    return;
  }
  // opaque lane id: keeps the per-lane geometry below from being hoisted out of the caller's
  // row loop (it would stay live through the register-heavy Cholesky phase)
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int g = lane >> 4, fl = lane & 15;
  // per-lane staging geometry (constant over chunks).  SPLIT and KP > 64 (the fp32 wide
  // kernels at 512 registers): recomputed at each use from an opaque lane id -- a handful of
  // integer ops -- instead of 2 x NPL registers held across the chunk loop (the fp32 rank-128
  // kernel spilled them to scratch and reloaded them every chunk)
  constexpr bool RECOMP = SPLIT && KP > 64;
  int srow_[RECOMP ? 1 : NPL], soff_[RECOMP ? 1 : NPL];
  if constexpr (!RECOMP) {
#pragma unroll
    for (int it = 0; it < NPL; ++it) {
      const int sl = it * 64 + lane, r = sl / PPR, sc = sl % PPR;
      srow_[it] = r;
      soff_[it] = ((sc + CI::rot(r)) % PPR) * 8;
    }
  }
  auto srow = [&](int it) -> int {
    if constexpr (RECOMP) {
      int ln = lane;
      asm volatile("" : "+v"(ln));
      return (it * 64 + ln) / PPR;
    } else {
      return srow_[it];
    }
  };
  auto soff = [&](int it) -> int {
    if constexpr (RECOMP) {
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int sl = it * 64 + ln, r = sl / PPR, sc = sl % PPR;
      return ((sc + CI::rot(r)) % PPR) * 8;
    } else {
      return soff_[it];
    }
  };
  // transposed-read byte offsets: operand pi, half h; lane 4q+p of group g reads row
  // 8g+4h+q, features pi*16 + 4p .. +3
  const int q = fl >> 2, pp = fl & 3;
  auto tr_addr = [&](int pi, int h) -> int {
    const int row = 8 * g + 4 * h + q;
    const int pc = 2 * pi + (pp >> 1);
    const int sc = (pc - CI::rot(row) + PPR) % PPR;
    return row * KP * 2 + sc * 16 + (pp & 1) * 8;
  };
  auto load_meta = [&](int64_t c, int (&cols)[NPL], float& val) {
#pragma unroll
    for (int it = 0; it < NPL; ++it) {
      const int64_t ri = c + srow(it) < end ? c + srow(it) : end - 1;
      cols[it] = p.col_idx[ri];
    }
    const int64_t vi = c + (lane & 31) < end ? c + (lane & 31) : end - 1;
    val = p.vals[vi];
  };
  i32x4 stg[NPL];
  i32x4 stgl[SPLIT ? NPL : 1];
  constexpr int YS = SPLIT ? 2 * KP : KP;
  auto gather = [&](const int (&cols)[NPL]) {
#pragma unroll
    for (int it = 0; it < NPL; ++it) {
      const __bf16* yr = p.Y + (int64_t)cols[it] * YS + soff(it);
      stg[it] = *reinterpret_cast<const i32x4*>(yr);
      if constexpr (SPLIT) stgl[it] = *reinterpret_cast<const i32x4*>(yr + KP);
    }
  };

  // two metadata sets used ping-pong (chunk parity) so that no register copies force an
  // early wait on the in-flight prefetch loads
  int cols0[NPL], cols1[NPL];
  float val0, val1 = 0.f;
  auto chunk = [&](int64_t c0, int (&cur_cols)[NPL], float& cur_val, int (&nxt_cols)[NPL]) {
    const int n = (int)min((int64_t)32, end - c0);
    float wa = 0.f, wb = 0.f, cn = 0.f;
    if (lane < n) als_weights(cur_val, p.alpha, p.implicit, wa, wb, cn);
    cnt_acc += cn;
    if (lane < 32) {
      Wab[lane] = wa;
      Wab[32 + lane] = wb;
    }
#pragma unroll
    for (int it = 0; it < NPL; ++it) {
      *reinterpret_cast<i32x4*>(G + (it * 64 + lane) * 16) = stg[it];
      if constexpr (SPLIT)
        *reinterpret_cast<i32x4*>(G + CI::BYTES + (it * 64 + lane) * 16) = stgl[it];
    }
    wave_sync();
    if (c0 + 32 < end) {              // wave-uniform: prefetch chunk c+1, metadata of c+2
      gather(nxt_cols);
      if (c0 + 64 < end) load_meta(c0 + 64, cur_cols, cur_val);
    }
    const f32x4* wv = reinterpret_cast<const f32x4*>(Wab);
    const f32x4 wa0 = wv[2 * g], wa1 = wv[2 * g + 1];
    const f32x4 wb0 = wv[8 + 2 * g], wb1 = wv[8 + 2 * g + 1];
    constexpr bool LO = SPLIT || kExactC;
    if constexpr (!LO) {
      // bf16 factor mode: A fragments bf16(c * y) for all row blocks, then the MFMAs
      bf16x8 fa[M], fb[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 0)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 1)));
        const bf16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        fb[pi] = v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          fa[pi][j] = (__bf16)((float)v[j] * wa0[j]);
          fa[pi][4 + j] = (__bf16)((float)v[4 + j] * wa1[j]);
        }
      }
      int t = 0;
#pragma unroll
      for (int pi = 0; pi < M; ++pi)
#pragma unroll
        for (int qi = 0; qi <= pi; ++qi, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[pi], fb[qi], acc[t], 0, 0, 0);
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bpart[pi] += wb0[j] * (float)fb[pi][j];
#pragma unroll
        for (int j = 0; j < 4; ++j) bpart[pi] += wb1[j] * (float)fb[pi][4 + j];
      }
      wave_sync();
      return;
    }
    bf16x8 fb[M], fbl[SPLIT ? M : 1];
#pragma unroll
    for (int pi = 0; pi < M; ++pi) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 0)));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 1)));
      fb[pi] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      if constexpr (SPLIT) {
        const bf16x4 lo2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + CI::BYTES + tr_addr(pi, 0)));
        const bf16x4 hi2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + CI::BYTES + tr_addr(pi, 1)));
        fbl[pi] = __builtin_shufflevector(lo2, hi2, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    {
      // A operand of row block pi made just before its MFMAs (two fragments live, not 2M)
      int t = 0;
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
        bf16x8 fa, fal;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float yv = (float)fb[pi][j];
          if constexpr (SPLIT) yv += (float)fbl[pi][j];
          const float sv = yv * (j < 4 ? wa0[j] : wa1[j - 4]);
          fa[j] = (__bf16)sv;
          if constexpr (LO) fal[j] = (__bf16)(sv - (float)fa[j]);
        }
#pragma unroll
        for (int qi = 0; qi <= pi; ++qi, ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[qi], acc[t], 0, 0, 0);
          if constexpr (LO)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fal, fb[qi], acc[t], 0, 0, 0);
          if constexpr (SPLIT)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fbl[qi], acc[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int pi = 0; pi < M; ++pi) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float y0 = (float)fb[pi][j], y1 = (float)fb[pi][4 + j];
        if constexpr (SPLIT) {
          y0 += (float)fbl[pi][j];
          y1 += (float)fbl[pi][4 + j];
        }
        bpart[pi] += wb0[j] * y0;
        bpart[pi] += wb1[j] * y1;
      }
    }
    wave_sync();
  };

  load_meta(beg, cols0, val0);
  gather(cols0);
  if (beg + 32 < end) load_meta(beg + 32, cols1, val1);
  if (INIT_YTY) init_yty(lane);
  for (int64_t c0 = beg; c0 < end; c0 += 64) {
    chunk(c0, cols0, val0, cols1);
    if (c0 + 32 < end) chunk(c0 + 32, cols1, val1, cols0);
  }
}

// Same accumulation with THREE chunks of gathers in flight (register rings of 3 by chunk
// index mod 3), kept as state across rows so that the next row's first three chunks are
// issued (prefetch) before the current row is factored: the factorization's VALU work hides
// the next row's gather latency.  Issue order inside chunk c, after its image is in LDS:
// [cols(c+5), val(c+3), gathers(c+3)].  vmcnt retires in issue order, so every load a later
// wait needs is issued before the gather groups that should stay in flight past that wait:
// when chunk c+1 starts, gathers(c+1), val(c+1) and cols(c+4) are all older than
// gathers(c+2) and gathers(c+3), which stay in flight.  (The factorization therefore takes
// YtY from LDS, not global memory: a global load there would drain the prefetch.)
template <int KP>
struct GatherRing {
  using CI = ChunkImage<KP>;
  static constexpr int M = KP / 16;
  static constexpr int PPR = CI::PPR;
  static constexpr int NPL = CI::NPL;
  int lane, g, fl, q4, p4;
  int srow[NPL], soff[NPL];
  int64_t beg = 0, end = 0, nch = 0;
  i32x4 stg0[NPL], stg1[NPL], stg2[NPL];
  int cols0[NPL], cols1[NPL], cols2[NPL];
  float val0 = 0.f, val1 = 0.f, val2 = 0.f;

  __device__ __forceinline__ void init() {
    lane = threadIdx.x & 63;
    g = lane >> 4;
    fl = lane & 15;
    q4 = fl >> 2;
    p4 = fl & 3;
#pragma unroll
    for (int it = 0; it < NPL; ++it) {
      const int sl = it * 64 + lane, r = sl / PPR, sc = sl % PPR;
      srow[it] = r;
      soff[it] = ((sc + CI::rot(r)) % PPR) * 8;
    }
  }
  // transposed-read byte offsets: operand pi, half h; lane 4q+p of group g reads row
  // 8g+4h+q, features pi*16 + 4p .. +3
  __device__ __forceinline__ int tr_addr(int pi, int h) const {
    const int row = 8 * g + 4 * h + q4;
    const int pc = 2 * pi + (p4 >> 1);
    const int sc = (pc - CI::rot(row) + PPR) % PPR;
    return row * KP * 2 + sc * 16 + (p4 & 1) * 8;
  }
  __device__ __forceinline__ void load_cols(const AlsParams& p, int64_t ch, int (&cols)[NPL]) {
    const int64_t c = beg + ch * 32;
#pragma unroll
    for (int it = 0; it < NPL; ++it) {
      const int64_t ri = c + srow[it] < end ? c + srow[it] : end - 1;
      cols[it] = p.col_idx[ri];
    }
  }
  __device__ __forceinline__ void load_val(const AlsParams& p, int64_t ch, float& val) {
    const int64_t c = beg + ch * 32;
    const int64_t vi = c + (lane & 31) < end ? c + (lane & 31) : end - 1;
    val = p.vals[vi];
  }
  __device__ __forceinline__ void gather(const AlsParams& p, const int (&cols)[NPL],
                                         i32x4 (&stg)[NPL]) {
#pragma unroll
    for (int it = 0; it < NPL; ++it)
      stg[it] = *reinterpret_cast<const i32x4*>(p.Y + (int64_t)cols[it] * KP + soff[it]);
  }
  // issue the first three chunks of ratings [b, e) in two stages, so the second stage (the
  // gathers, which need the column indices) can come once the indices have arrived:
  // stage 1 [cols(0..2), val(0..2)], stage 2 G(0) [cols(3)] G(1) [cols(4)] G(2)
  __device__ __forceinline__ void prefetch_meta(const AlsParams& p, int64_t b, int64_t e) {
    beg = b;
    end = e;
    nch = e > b ? (e - b + 31) / 32 : 0;
    if (nch == 0) return;
    load_cols(p, 0, cols0);
    if (nch > 1) load_cols(p, 1, cols1);
    if (nch > 2) load_cols(p, 2, cols2);
    load_val(p, 0, val0);
    if (nch > 1) load_val(p, 1, val1);
    if (nch > 2) load_val(p, 2, val2);
  }
  __device__ __forceinline__ void prefetch_gather(const AlsParams& p) {
    if (nch == 0) return;
    gather(p, cols0, stg0);
    if (nch > 3) load_cols(p, 3, cols0);
    if (nch > 1) gather(p, cols1, stg1);
    if (nch > 4) load_cols(p, 4, cols1);
    if (nch > 2) gather(p, cols2, stg2);
  }
  // chunk ch: stg / val hold its data, cols_g the metadata of chunk ch+3 (gathered into stg
  // once its image is in LDS), cols_l the free slot that receives cols(ch+5)
  __device__ __forceinline__ void chunk(const AlsParams& p, int64_t ch, i32x4 (&stg)[NPL],
                                        float& val, int (&cols_g)[NPL], int (&cols_l)[NPL],
                                        char* G, float* Wab, f32x4 (&acc)[M * (M + 1) / 2],
                                        float (&bpart)[M], float& cnt_acc) {
    const int64_t c0 = beg + ch * 32;
    const int n = (int)min((int64_t)32, end - c0);
    float wa = 0.f, wb = 0.f, cn = 0.f;
    if (lane < n) als_weights(val, p.alpha, p.implicit, wa, wb, cn);
    cnt_acc += cn;
    if (lane < 32) {
      Wab[lane] = wa;
      Wab[32 + lane] = wb;
    }
#pragma unroll
    for (int it = 0; it < NPL; ++it)
      *reinterpret_cast<i32x4*>(G + (it * 64 + lane) * 16) = stg[it];
    wave_sync();
    if (ch + 5 < nch) load_cols(p, ch + 5, cols_l);
    if (ch + 3 < nch) {
      load_val(p, ch + 3, val);
      gather(p, cols_g, stg);
    }
    const f32x4* wv = reinterpret_cast<const f32x4*>(Wab);
    const f32x4 wa0 = wv[2 * g], wa1 = wv[2 * g + 1];
    const f32x4 wb0 = wv[8 + 2 * g], wb1 = wv[8 + 2 * g + 1];
    if constexpr (kExactC) {
      bf16x8 fb[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 0)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 1)));
        fb[pi] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      // A operand of row block pi made just before its MFMAs (two fragments live, not 2M)
      int t = 0;
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
        bf16x8 fa, fal;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float sv = (float)fb[pi][j] * (j < 4 ? wa0[j] : wa1[j - 4]);
          fa[j] = (__bf16)sv;
          fal[j] = (__bf16)(sv - (float)fa[j]);
        }
#pragma unroll
        for (int qi = 0; qi <= pi; ++qi, ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[qi], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fal, fb[qi], acc[t], 0, 0, 0);
        }
      }
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bpart[pi] += wb0[j] * (float)fb[pi][j];
#pragma unroll
        for (int j = 0; j < 4; ++j) bpart[pi] += wb1[j] * (float)fb[pi][4 + j];
      }
      wave_sync();
      return;
    }
    bf16x8 fa[M], fb[M];
#pragma unroll
    for (int pi = 0; pi < M; ++pi) {
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 0)));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 1)));
      const bf16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      fb[pi] = v;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fa[pi][j] = (__bf16)((float)v[j] * wa0[j]);
        fa[pi][4 + j] = (__bf16)((float)v[4 + j] * wa1[j]);
      }
    }
    {
      int t = 0;
#pragma unroll
      for (int pi = 0; pi < M; ++pi)
#pragma unroll
        for (int qi = 0; qi <= pi; ++qi, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[pi], fb[qi], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int pi = 0; pi < M; ++pi) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bpart[pi] += wb0[j] * (float)fb[pi][j];
#pragma unroll
      for (int j = 0; j < 4; ++j) bpart[pi] += wb1[j] * (float)fb[pi][4 + j];
    }
    wave_sync();
  }
  // consume every chunk of the prefetched ratings
  __device__ __forceinline__ void run(const AlsParams& p, char* G, float* Wab,
                                      f32x4 (&acc)[M * (M + 1) / 2], float (&bpart)[M],
                                      float& cnt_acc) {
    for (int64_t ch = 0; ch < nch; ch += 3) {
      chunk(p, ch, stg0, val0, cols0, cols2, G, Wab, acc, bpart, cnt_acc);
      if (ch + 1 < nch) chunk(p, ch + 1, stg1, val1, cols1, cols0, G, Wab, acc, bpart, cnt_acc);
      if (ch + 2 < nch) chunk(p, ch + 2, stg2, val2, cols2, cols1, G, Wab, acc, bpart, cnt_acc);
    }
  }
};


// PROF: accumulate per-phase shader-clock cycles of every row into prof[0..6] (analysis
// builds only; see scripts/als_phase_profile.py)
template <int KP, bool PROF = false, bool SPLIT = false>
__global__ __launch_bounds__(256) void als_solve_wave(AlsParams p, unsigned long long* prof) {
  using WSM = WaveSmem<KP, SPLIT>;
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int AS = WSM::AS;
  __shared__ __attribute__((aligned(16))) char smem[4 * WSM::BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  char* my = smem + wave * WSM::BYTES;
  char* G = my;
  float* A = reinterpret_cast<float*>(my);
  float* Wab = reinterpret_cast<float*>(my + WSM::BYTES - 512);
  float* Lb = reinterpret_cast<float*>(my + WSM::BYTES - 256);
  const int g = lane >> 4, fl = lane & 15;
  const int total_waves = gridDim.x * 4;
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};

  for (int w = blockIdx.x * 4 + wave; w < p.n_work; w += total_waves) {
    const int row = p.row_ids ? p.row_ids[w] : w;
    const int64_t beg = p.row_ptr[row], end = p.row_ptr[row + 1];
    const int slot = p.long_slot ? p.long_slot[w] : -1;
    unsigned long long tp = PROF ? __builtin_amdgcn_s_memtime() : 0;
#define ORYX_PHASE(ix)                                                   \
  if (PROF) {                                                            \
    const unsigned long long tn = __builtin_amdgcn_s_memtime();          \
    ph[ix] += tn - tp;                                                   \
    tp = tn;                                                             \
  }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bacc, cnt_acc = 0.f;
    {
      // split rows were accumulated by als_partial: skip their ratings here
      float bpart[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[pi] = 0.f;
      wave_accumulate<KP, false, SPLIT>(p, beg, slot < 0 ? end : beg, G, Wab, acc, bpart,
                                        cnt_acc);
      reduce_bpart<M>(bpart);
      bacc = pick_bpart<M>(bpart, g);
    }
    ORYX_PHASE(0)
    float cnt = wave_sum(cnt_acc);
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
    if (slot >= 0) {
      // add the split row's partial sums; lane-private opaque pointers so no per-i
      // addresses get hoisted into SGPRs
      const float* src = p.ws + (int64_t)slot * ws_stride(KP) + (lane < KP ? lane : 0);
      asm volatile("" : "+v"(src));
      float* dstc = A + (lane < KP ? lane : 0);
      asm volatile("" : "+v"(dstc));
      wave_sync();
#pragma unroll 8
      for (int i = 0; i < KP; ++i) dstc[i * AS] += src[i * KP];
      bacc = src[KP * KP];
      cnt = oryx_readlane(src[KP * KP + KP - (lane < KP ? lane : 0)], 0);
    }
    wave_sync();
    ORYX_PHASE(1)
    // lane c owns column c
    const int c = lane < KP ? lane : 0;
    const float diag = c < p.k ? p.lambda * cnt : 1.f;
    float a[KP];
    int cc = c;
    asm volatile("" : "+v"(cc));
    // + YtY column c = row c (symmetric): 16-byte loads off one opaque per-row base (YtY is
    // always present: zeros for explicit feedback)
    const f32x4* yrow = reinterpret_cast<const f32x4*>(p.YtY + cc * KP);
    asm volatile("" : "+v"(yrow));
#pragma unroll
    for (int i4 = 0; i4 < KP / 4; ++i4) {
      const f32x4 yv = yrow[i4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 4 * i4 + q;
        a[i] = A[i * AS + c] + yv[q] + (i == cc ? diag : 0.f);
      }
      if ((i4 & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    ORYX_PHASE(2)
    // Cholesky A = L L^T in registers: after step j lane c holds L[c][j] in a[j]
    // (lane j keeps the pivot d_j in a[j] and 1/d_j in dinv).  The column of L that the
    // rank-1 update needs is broadcast with v_readlane (one SGPR per row i, consumed by one
    // FMA) -- no LDS round trip on the step's critical path.
    bool bad = false;
    // opaque copy of the lane id: stops the compiler hoisting 2*KP lane masks out of the row
    // loop (which would exhaust SGPRs)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    float dinv = 0.f;
#if ORYX_ALS_CHOL_LDS
    // the column of L goes through LDS: one ds_write_b32 per step, then broadcast
    // ds_read_b128 (all lanes read the same 16 bytes) of the trailing entries -- the rank-1
    // update's FMAs take VGPR operands instead of one v_readlane (+ SGPR hazard) each.  A's
    // LDS image is dead during the factorization, so its first row is the broadcast buffer.
    typedef __attribute__((address_space(3))) float lds_float;
    lds_float* bc = (lds_float*)(A);
#endif
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      float s = oryx_readlane(a[j], j);
      bad |= !(s > 0.f);
      s = s > 1e-30f ? s : 1e-30f;
      // one v_rsq_f32 (~1 ulp) instead of the IEEE sqrt expansion + reciprocal
      const float inv = __builtin_amdgcn_rsqf(s);
      const float d = s * inv;
      float l = a[j] * inv;
      l = ln < j ? 0.f : (ln == j ? d : l);
      dinv = ln == j ? inv : dinv;
      a[j] = l;
#if ORYX_ALS_CHOL_LDS
      if (j + 1 < KP) {
        bc[c] = l;      // lanes >= KP (KP < 64) rewrite slot 0, which is never read back
        // each updated entry passes through an empty asm: otherwise the SLP vectoriser fuses
        // the straight-line updates into vector ops on a[] and the array lands in scratch
        // all broadcast reads first (16-byte, in flight together), then the FMAs
        f32x4 bv[KP / 4];
#pragma unroll
        for (int i4 = (j + 1) / 4; i4 < KP / 4; ++i4)
          bv[i4] = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(bc + 4 * i4);
        // (v_pk_fma_f32 on pairs was measured slower here: 26.5K vs 23.3K cycles per row)
#pragma unroll
        for (int i = j + 1; i < KP; ++i) {
          a[i] -= bv[i / 4][i % 4] * l;
          asm volatile("" : "+v"(a[i]));
        }
      }
#else
#pragma unroll
      for (int i = j + 1; i < KP; ++i) {
        a[i] -= oryx_readlane(l, i) * l;
        if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
      }
#endif
      // pin the updated trailing column values here: without this LLVM sinks the rank-1
      // updates into a left-looking form that keeps every broadcast L column live (spills)
#pragma unroll
      for (int i = j + 1; i < KP; ++i) asm volatile("" : "+v"(a[i]));
    }
    ORYX_PHASE(3)
    if (bad && lane == 0 && p.fail_count) atomicAdd(p.fail_count, 1);
    // forward: L z = b
    float zv = lane < KP ? bacc : 0.f, z_own = 0.f;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      const float zj = oryx_readlane(zv * dinv, j);   // lane j scales by its own 1/d_j
      z_own = ln == j ? zj : z_own;
      zv -= a[j] * zj;
    }
    ORYX_PHASE(4)
    // back: L^T x = z.  Step j needs row j of L in every lane (lane c: L[j][c]); the rows go
    // through LDS once and are read back independently of the solve chain.
    if (lane < KP) {
#pragma unroll
      for (int i = 0; i < KP; ++i) A[lane * AS + i] = a[i];
    }
    wave_sync();
    float xv = z_own, x_own = 0.f;
#pragma unroll
    for (int j = KP - 1; j >= 0; --j) {
      const float xj = oryx_readlane(xv * dinv, j);
      x_own = ln == j ? xj : x_own;
      xv -= A[j * AS + c] * xj;
      if ((j & 7) == 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < KP) {
      p.X[(int64_t)row * KP + lane] = x_own;
      if (p.Xb) store_xb<SPLIT, KP>(p.Xb, row, lane, x_own);
    }
    wave_sync();
    ORYX_PHASE(5)
#undef ORYX_PHASE
  }
  if (PROF && lane == 0)
    for (int i = 0; i < 6; ++i) atomicAdd(prof + i, ph[i]);
}

// ------------------------------------------------------------------ panel-Cholesky kernel

// LDS of one wave in als_solve_panel: the lower block-column panels of L (panel p = rows
// 16p..KP-1 x columns 16p..16p+15, LS floats per row), aliased with the gather's chunk image,
// plus the per-rating weights.  LS = 20: lane-per-row ds_read_b128, the accumulator-layout
// scatter and the MFMA-fragment reads are all bank-conflict free.  KP=64: 12.8 KB per wave
// (the register-Cholesky kernel keeps a 64x65 fp32 image, 17 KB).
template <int KP>
struct PanelSmem {
  static constexpr int M = KP / 16;
  static constexpr int LS = 20;
  static constexpr int ROWS = 16 * M * (M + 1) / 2;
  static constexpr int L_BYTES = ROWS * LS * 4;
  static constexpr int G_BYTES = ChunkImage<KP>::BYTES;
  static constexpr int RAW = L_BYTES > G_BYTES ? L_BYTES : G_BYTES;
  static constexpr int BYTES = (RAW + 15) / 16 * 16 + 256;
  // first LDS row of panel p: sum_{q<p} (KP - 16 q)
  __host__ __device__ static constexpr int base(int p) { return 16 * (p * M - p * (p - 1) / 2); }
};

// One wave per row, KP <= 64.  The normal-equation matrix never leaves the MFMA accumulators
// until it is factored:
//   * A = YtY + sum_i c_i y_i y_i^T accumulates on v_mfma_f32_16x16x32_bf16 starting from YtY
//     (wave_accumulate<KP, true>); lambda*n_u goes onto the diagonal in accumulator layout;
//   * right-looking blocked Cholesky over 16-column panels.  Panel p's tiles go to LDS once
//     and come back lane-per-row (lane r holds A[r][16p..16p+15]); its 16 columns are
//     eliminated in registers (the in-panel broadcasts are v_readlane of the panel's own
//     diagonal-block rows: <= 15 per step instead of one per trailing row), the forward solve
//     L z = b rides along as an augmented column (lane r holds b_r), and the trailing tiles
//     (i, j > p) are updated on v_mfma_f32_16x16x4_f32 straight in the accumulators;
//   * back substitution L^T x = z reads the LDS panels (off the dependency chain).
// Per row (KP=64): 480 in-panel FMAs per lane + 40 small MFMAs, versus 2016 FMAs per lane for
// the all-register column Cholesky of als_solve_wave.
template <int KP, bool PROF = false, bool DEEP = false, int PRIO = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEEP ? 2 : ORYX_ALS_PANEL_WAVES, DEEP ? 2 : ORYX_ALS_PANEL_WAVES))) void als_solve_panel(AlsParams p, unsigned long long* prof) {
  using PS = PanelSmem<KP>;
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int LS = PS::LS;
  __shared__ __attribute__((aligned(16))) char smem[4 * PS::BYTES];
  // DEEP: the block's copy of YtY, row stride KP + 4 floats (lane-per-row 16-byte reads are
  // bank-conflict free); global loads during the factorization would drain the prefetch
  constexpr int YS = KP + 4;
  __shared__ __attribute__((aligned(16))) float ytys[DEEP ? KP * YS : 4];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  char* my = smem + wave * PS::BYTES;
  float* Lp = reinterpret_cast<float*>(my);
  float* Wab = reinterpret_cast<float*>(my + PS::BYTES - 256);
  const int g = lane >> 4, fl = lane & 15;
  const int total_waves = gridDim.x * 4;
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
  GatherRing<KP> ring;
  if (DEEP) {
    for (int i = threadIdx.x; i < KP * KP / 4; i += 256) {
      const int r = (4 * i) / KP, c = (4 * i) % KP;
      *reinterpret_cast<f32x4*>(ytys + r * YS + c) =
          reinterpret_cast<const f32x4*>(p.YtY)[i];
    }
    __syncthreads();
    ring.init();
    const int w0 = blockIdx.x * 4 + wave;
    if (ORYX_ALS_XROW_PREFETCH && w0 < p.n_work) {
      const int row0 = p.row_ids ? p.row_ids[w0] : w0;
      const int slot0 = p.long_slot ? p.long_slot[w0] : -1;
      const int64_t b0 = p.row_ptr[row0];
      ring.prefetch_meta(p, b0, slot0 < 0 ? p.row_ptr[row0 + 1] : b0);
      ring.prefetch_gather(p);
    }
  }

  for (int w = blockIdx.x * 4 + wave; w < p.n_work; w += total_waves) {
    const int row = p.row_ids ? p.row_ids[w] : w;
    const int64_t beg = p.row_ptr[row], end = p.row_ptr[row + 1];
    const int slot = p.long_slot ? p.long_slot[w] : -1;
    unsigned long long tp = PROF ? __builtin_amdgcn_s_memtime() : 0;
#define ORYX_PHASE(ix)                                                   \
  if (PROF) {                                                            \
    const unsigned long long tn = __builtin_amdgcn_s_memtime();          \
    ph[ix] += tn - tp;                                                   \
    tp = tn;                                                             \
  }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bz, cnt_acc = 0.f;
    {
      float bpart[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[pi] = 0.f;
      // acc = sum over the row's ratings (split rows: nothing here, partials from ws below)
      if (DEEP) {
        if (!ORYX_ALS_XROW_PREFETCH) {
          ring.prefetch_meta(p, beg, slot < 0 ? end : beg);
          ring.prefetch_gather(p);
        }
        ring.run(p, my, Wab, acc, bpart, cnt_acc);
        // the next row's metadata now, its first three chunk gathers after this row's first
        // panel: they are in flight while this row is factored
        const int wn = w + total_waves;
        if (ORYX_ALS_XROW_PREFETCH && wn < p.n_work) {
          const int rown = p.row_ids ? p.row_ids[wn] : wn;
          const int slotn = p.long_slot ? p.long_slot[wn] : -1;
          const int64_t bn = p.row_ptr[rown];
          ring.prefetch_meta(p, bn, slotn < 0 ? p.row_ptr[rown + 1] : bn);
        } else {
          ring.nch = 0;
        }
      } else
        wave_accumulate<KP, false>(p, beg, slot < 0 ? end : beg, my, Wab, acc, bpart, cnt_acc);
      reduce_bpart<M>(bpart);
      bz = pick_bpart<M>(bpart, g);   // lane l (< KP): b[l]
    }
    float cnt = wave_sum(cnt_acc);
    const float* wsrow = nullptr;
    if (slot >= 0) {
      const float* src = p.ws + (int64_t)slot * ws_stride(KP);
      bz = src[KP * KP + (lane < KP ? lane : 0)];
      cnt = src[KP * KP + KP];
      wsrow = src;
    }
    ORYX_PHASE(0)
    // PRIO > 0: the serial factorisation runs at raised issue priority, so when the SIMD's
    // other wave is gathering, this wave's dependent chain is not left waiting behind it
    if (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
    float dinv = 0.f, z_own = 0.f;
    // opaque lane id (keeps per-step lane masks from being hoisted into SGPR pairs)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    typedef __attribute__((address_space(3))) float lds_float;
    typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
    lds_float* bcl = (lds_float*)Wab;   // 64 floats: the weights' slot, free after the gather
#pragma unroll
    for (int pp = 0; pp < M; ++pp) {
      float* P = Lp + PS::base(pp) * LS;
      // panel tiles (i, pp), i >= pp: accumulator layout -> LDS rows 16pp.. of the panel
#pragma unroll
      for (int i = pp; i < M; ++i) {
        const int t = i * (i + 1) / 2 + pp;
#pragma unroll
        for (int v = 0; v < 4; ++v) P[(16 * (i - pp) + 4 * g + v) * LS + fl] = acc[t][v];
      }
      wave_sync();
      const bool inp = ln >= 16 * pp && ln < KP;
      const int prow = inp ? ln - 16 * pp : 0;
      // + YtY (and a split row's partial sums) and lambda * n_u, added to each panel as it is
      // loaded: all are plain additions to A, and tile (i, j)'s share is only needed once
      // panel j is factored (the trailing updates before that just subtract from it)
      const int rr = ln < KP ? ln : 0;
      f32x4 yv[4];
      if (DEEP) {
        const lds_f32x4* yr = reinterpret_cast<const lds_f32x4*>(
            (const lds_float*)ytys + rr * YS + 16 * pp);
#pragma unroll
        for (int q = 0; q < 4; ++q) yv[q] = yr[q];
      } else {
        const f32x4* yr = reinterpret_cast<const f32x4*>(p.YtY + rr * KP + 16 * pp);
#pragma unroll
        for (int q = 0; q < 4; ++q) yv[q] = yr[q];
      }
      if (wsrow) {
        const f32x4* wr = reinterpret_cast<const f32x4*>(wsrow + rr * KP + 16 * pp);
#pragma unroll
        for (int q = 0; q < 4; ++q) yv[q] += wr[q];
      }
      float pr[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(P + prow * LS + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) pr[4 * q + e] = v[e] + yv[q][e];
      }
      {
        int rel = ln - 16 * pp;
        asm volatile("" : "+v"(rel));
        const float dg = ln < p.k ? p.lambda * cnt : 1.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) pr[j] += rel == j ? dg : 0.f;
      }
      ORYX_PHASE(2)
      // eliminate the panel's 16 columns; lane r > J ends with L[r][J] in pr[J - 16pp], lane J
      // with d_J (lanes below J hold values that are never read: the trailing update uses rows
      // below the diagonal block, and back substitution only lanes c < J of row J).
      // Critical path per step: pivot -> rsq -> l -> readlane L[J+1][J] -> update column j+1
      // -> next pivot, all in registers; the other columns (j+2..15) take column J through an
      // LDS broadcast whose round trip overlaps the next step's pivot work.  A wave's LDS
      // accesses complete in order and the slot array aliases, so no fence is needed between
      // a step's broadcast write, its reads, and the next step's write.
      float sp = oryx_readlane(pr[0], 16 * pp);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int J = 16 * pp + j;
        // not positive (or NaN) -> clamped to 1e-30; detected from 1/d below (per-step
        // boolean flags get sunk to the end of the row and pin all 64 pivots in SGPRs)
        const float s = sp > 1e-30f ? sp : 1e-30f;
        const float inv = __builtin_amdgcn_rsqf(s);
        const float l = pr[j] * inv;   // lane J: s / sqrt(s) = d_J
        pr[j] = l;
        // forward solve on the augmented column: z_J = b_J / d_J; lanes <= J keep junk in bz
        // from here on (z_J is captured in z_own)
        const float zJ = oryx_readlane(bz, J) * inv;
        bz -= l * zJ;
        // lane-relative index made opaque per step so the mask is formed here, not hoisted
        int rel = ln - J;
        asm volatile("" : "+v"(rel));
        dinv = rel == 0 ? inv : dinv;
        z_own = rel == 0 ? zJ : z_own;
        // materialise both selects now: otherwise LLVM sinks the 64-deep select chains to their
        // use in the back substitution and keeps every step's 1/d and z live (spills)
        asm volatile("" : "+v"(dinv), "+v"(z_own), "+v"(bz));
        if (j < 15) {
          if (j < 14) bcl[ln] = l;
          const float a1 = oryx_readlane(l, J + 1);   // L[J+1][J]
          pr[j + 1] -= l * a1;
          asm volatile("" : "+v"(pr[j + 1]));
          sp = oryx_readlane(pr[j + 1], J + 1);
          if (j < 14) {
            f32x4 bq[4];
#pragma unroll
            for (int q = (j + 2) / 4; q < 4; ++q)
              bq[q] = *reinterpret_cast<const lds_f32x4*>(bcl + 16 * pp + 4 * q);
#pragma unroll
            for (int jj = j + 2; jj < 16; ++jj) {
              pr[jj] -= l * bq[jj / 4][jj % 4];
              asm volatile("" : "+v"(pr[jj]));
            }
          }
        }
      }
      if (inp) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(P + prow * LS + 4 * q) =
              f32x4{pr[4 * q], pr[4 * q + 1], pr[4 * q + 2], pr[4 * q + 3]};
      }
      wave_sync();
      ORYX_PHASE(3)
      // trailing update: A(i, jt) -= L(i, pp) L(jt, pp)^T for i >= jt > pp, on fp32 MFMA
      if (pp + 1 < M) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          float fr[M];
#pragma unroll
          for (int i = pp + 1; i < M; ++i) fr[i] = P[(16 * (i - pp) + fl) * LS + 4 * kk + g];
#pragma unroll
          for (int i = pp + 1; i < M; ++i)
#pragma unroll
            for (int jt = pp + 1; jt <= i; ++jt) {
              const int t = i * (i + 1) / 2 + jt;
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(-fr[i], fr[jt], acc[t], 0, 0, 0);
            }
        }
      }
      if (DEEP && ORYX_ALS_XROW_PREFETCH && pp == 0) ring.prefetch_gather(p);
      ORYX_PHASE(4)
    }
    // a clamped pivot gives 1/d = 1e15
    const bool bad = __any(lane < KP && !(dinv < 9.9e14f));
    if (bad && lane == 0 && p.fail_count) atomicAdd(p.fail_count, 1);
    // back substitution L^T x = z: step J takes L[J][c] (lane c) from panel c/16
    const int c = lane < KP ? lane : 0;
    const int pc = c >> 4;
    const lds_float* lcol = (const lds_float*)(Lp + (PS::base(pc) - 16 * pc) * LS + (c & 15));
    float xv = z_own, x_own = 0.f;
#pragma unroll
    for (int J = KP - 1; J >= 0; --J) {
      int rel = ln - J;
      asm volatile("" : "+v"(rel));
      const float lv = lcol[J * LS];
      const float xj = oryx_readlane(xv * dinv, J);
      x_own = rel == 0 ? xj : x_own;
      // lanes c > J are finished (x_own captured); for c in a later panel than row J the read
      // lands on another panel's rows (in bounds, value irrelevant), so no mask is needed
      xv -= lv * xj;
      if ((J & 7) == 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < KP) {
      p.X[(int64_t)row * KP + lane] = x_own;
      if (p.Xb) p.Xb[(int64_t)row * KP + lane] = (__bf16)x_own;
    }
    wave_sync();
    if (PRIO > 0) __builtin_amdgcn_s_setprio(0);
    ORYX_PHASE(5)
#undef ORYX_PHASE
  }
  if (PROF && lane == 0)
    for (int i = 0; i < 6; ++i) atomicAdd(prof + i, ph[i]);
}

// Debug/verification: the raw normal equations (Gramian without YtY/lambda, b, count) of the
// single row [beg, end), as accumulated by wave_accumulate.  One wave.
template <int KP, bool SPLIT = false>
__global__ __launch_bounds__(64) void als_debug_gram(AlsParams p, int64_t beg, int64_t end,
                                                     float* __restrict__ out) {
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int GB = ChunkImage<KP>::BYTES * (SPLIT ? 2 : 1);
  __shared__ __attribute__((aligned(16))) char smem[GB + 256];
  const int lane = threadIdx.x, g = lane >> 4, fl = lane & 15;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bpart[M];
#pragma unroll
  for (int pi = 0; pi < M; ++pi) bpart[pi] = 0.f;
  float cnt_acc = 0.f;
  wave_accumulate<KP, false, SPLIT>(p, beg, end, smem, reinterpret_cast<float*>(smem + GB), acc,
                                    bpart, cnt_acc);
  reduce_bpart<M>(bpart);
  const float cnt = wave_sum(cnt_acc);
  int t = 0;
#pragma unroll
  for (int pi = 0; pi < M; ++pi)
#pragma unroll
    for (int qi = 0; qi <= pi; ++qi, ++t)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = pi * 16 + g * 4 + v, j = qi * 16 + fl;
        out[i * KP + j] = acc[t][v];
        out[j * KP + i] = acc[t][v];
      }
  if (lane < KP) out[KP * KP + lane] = pick_bpart<M>(bpart, g);
  if (lane + 64 < KP) out[KP * KP + 64 + lane] = pick_bpart<M>(bpart, g + 4);
  if (lane == 0) out[KP * KP + KP] = cnt;
}

// ------------------------------------------------------------------ split long rows

// One wave per segment (row, slot, beg, end) of a long row: accumulate the segment's partial
// Gramian / b / count and add them into the row's workspace record with fp32 atomics (one
// 256-byte run per atomic instruction).  Runs before the solve kernel, which then takes long
// rows' normal equations from the workspace: a row with 1e5 ratings is spread over ~100
// waves instead of serialising on one (the tail of the popular-item half-step).
template <int KP, bool SPLIT = false>
__global__ __launch_bounds__(256) void als_partial(AlsParams p, const int64_t* __restrict__ segs,
                                                  int n_seg, float* __restrict__ ws) {
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
    float* dst = ws + slot * ws_stride(KP);
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
          atomicAdd(dst + i * KP + j, acc[t][v]);
          if (pi != qi) atomicAdd(dst + j * KP + i, acc[t][v]);
        }
    }
    // after the reduction lane (g, fl) holds b[pi*16 + fl] for every pi: lane l adds
    // features l and l + 64
    if (lane < KP) atomicAdd(dst + KP * KP + lane, pick_bpart<M>(bpart, g));
    if (lane + 64 < KP) atomicAdd(dst + KP * KP + 64 + lane, pick_bpart<M>(bpart, g + 4));
    if (lane == 0) atomicAdd(dst + KP * KP + KP, cnt);
  }
}

// ------------------------------------------------------------------ wide panel kernel (KP 80..128)

// One wave per row for 64 < KP <= 128: lane r owns rows r and r + 64 in the panel phases.
//   * A = YtY + sum c_i y_i y_i^T accumulates in 36 (KP=128) 16x16 MFMA tiles that start at YtY
//     (wave_accumulate<KP, true>); lambda * n_u goes onto the diagonal in accumulator layout;
//   * right-looking blocked Cholesky over 16-column panels, as in als_solve_panel, with the
//     trailing tiles updated on v_mfma_f32_16x16x4_f32; each factored panel's L tiles are
//     written back into the accumulators it came from, so the whole factor stays in registers
//     and LDS only ever holds one panel (10 KB at KP=128 instead of 46 KB for all of them);
//   * the forward solve rides along as an augmented column; pivots' 1/d and z go to LDS;
//   * blocked back substitution from the last panel: panel p comes back to LDS once, 64
//     lanes form sum_{J in later blocks} L[J][c] x_J for its 16 columns (4 row groups, two
//     cross-lane adds), then a 16-step triangular solve finishes the block.
template <int KP, bool SPLIT = false>
struct WideSmem {
  static constexpr int LS = 20;
  static constexpr int PB = KP * LS * 4;
  static constexpr int GB = ChunkImage<KP>::BYTES * (SPLIT ? 2 : 1);
  static constexpr int RAW = PB > GB ? PB : GB;
  // + broadcast slots (128), 1/d (128), z (128), x (128), weights (64)
  static constexpr int BYTES = (RAW + 15) / 16 * 16 + (4 * 128 + 64) * 4;
};

template <int KP, bool SPLIT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void als_solve_wide(
    AlsParams p) {
  using WS = WideSmem<KP, SPLIT>;
  constexpr int M = KP / 16;
  constexpr int NT = M * (M + 1) / 2;
  constexpr int LS = WS::LS;
  typedef __attribute__((address_space(3))) float lds_float;
  typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
  __shared__ __attribute__((aligned(16))) char smem[4 * WS::BYTES];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  char* my = smem + wave * WS::BYTES;
  float* P = reinterpret_cast<float*>(my);
  lds_float* bcl = (lds_float*)(my + (WS::RAW + 15) / 16 * 16);
  lds_float* invs = bcl + 128;
  lds_float* zs = bcl + 256;
  lds_float* xs = bcl + 384;
  float* Wab = reinterpret_cast<float*>(my + (WS::RAW + 15) / 16 * 16 + 512 * 4);
  const int g = lane >> 4, fl = lane & 15;
  const int total_waves = gridDim.x * 4;

  for (int w = blockIdx.x * 4 + wave; w < p.n_work; w += total_waves) {
    const int row = p.row_ids ? p.row_ids[w] : w;
    const int64_t beg = p.row_ptr[row], end = p.row_ptr[row + 1];
    const int slot = p.long_slot ? p.long_slot[w] : -1;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bz0, bz1, cnt_acc = 0.f;
    {
      float bpart[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[pi] = 0.f;
      wave_accumulate<KP, false, SPLIT>(p, beg, slot < 0 ? end : beg, my, Wab, acc, bpart,
                                        cnt_acc);
      reduce_bpart<M>(bpart);
      // lane (g, fl) holds b[pi*16 + fl] for every pi: rows lane and lane + 64
      bz0 = pick_bpart<M>(bpart, g);
      bz1 = pick_bpart<M>(bpart, g + 4);
    }
    float cnt = wave_sum(cnt_acc);
    const float* wsrow = nullptr;
    if (slot >= 0) {
      const float* src = p.ws + (int64_t)slot * ws_stride(KP);
      bz0 = src[KP * KP + lane];
      bz1 = src[KP * KP + (lane + 64 < KP ? lane + 64 : 0)];
      cnt = src[KP * KP + KP];
      wsrow = src;
    }
    int ln = lane;
    asm volatile("" : "+v"(ln));

    static_for<M>([&](auto PPc) {
      constexpr int pp = decltype(PPc)::value;
      // panel tiles (i, pp), i >= pp -> LDS rows (r - 16pp)
#pragma unroll
      for (int i = pp; i < M; ++i) {
        const int t = i * (i + 1) / 2 + pp;
#pragma unroll
        for (int v = 0; v < 4; ++v) P[(16 * (i - pp) + 4 * g + v) * LS + fl] = acc[t][v];
      }
      wave_sync();
      // lane rows ln (set 0) and ln + 64 (set 1); rows outside [16pp, KP) read row 16pp (junk)
      const int r0 = ln >= 16 * pp ? ln - 16 * pp : 0;
      const int r1 = ln + 64 >= 16 * pp && ln + 64 < KP ? ln + 64 - 16 * pp : 0;
      // + YtY (and a split row's partial sums) and lambda * n_u, added as each panel is loaded
      // (plain additions to A; tile (i, j)'s share is only needed once panel j is factored)
      const int ra = ln, rb = ln + 64 < KP ? ln + 64 : 0;
      f32x4 ya[4], yb[4];
      {
        const f32x4* y0 = reinterpret_cast<const f32x4*>(p.YtY + ra * KP + 16 * pp);
        const f32x4* y1 = reinterpret_cast<const f32x4*>(p.YtY + rb * KP + 16 * pp);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ya[q] = y0[q];
          yb[q] = y1[q];
        }
        if (wsrow) {
          const f32x4* w0 = reinterpret_cast<const f32x4*>(wsrow + ra * KP + 16 * pp);
          const f32x4* w1 = reinterpret_cast<const f32x4*>(wsrow + rb * KP + 16 * pp);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            ya[q] += w0[q];
            yb[q] += w1[q];
          }
        }
      }
      float pa[16], pb[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 va = *reinterpret_cast<const f32x4*>(P + r0 * LS + 4 * q);
        const f32x4 vb = *reinterpret_cast<const f32x4*>(P + r1 * LS + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pa[4 * q + e] = va[e] + ya[q][e];
          pb[4 * q + e] = vb[e] + yb[q][e];
        }
      }
      {
        int rel = ln - 16 * pp;
        asm volatile("" : "+v"(rel));
        const float dga = ln < p.k ? p.lambda * cnt : 1.f;
        const float dgb = ln + 64 < p.k ? p.lambda * cnt : 1.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          pa[j] += rel == j ? dga : 0.f;
          pb[j] += rel + 64 == j ? dgb : 0.f;
        }
      }
      // the panel's diagonal block lives in set 0 (pp < 4) or set 1 (pp >= 4)
      const bool hi = pp >= 4;
      float sp = hi ? oryx_readlane(pb[0], 16 * pp - 64) : oryx_readlane(pa[0], 16 * pp);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int J = 16 * pp + j;
        const float s = sp > 1e-30f ? sp : 1e-30f;
        const float inv = __builtin_amdgcn_rsqf(s);
        const float la = pa[j] * inv, lb = pb[j] * inv;   // row J's lane: d_J
        pa[j] = la;
        pb[j] = lb;
        const float zJ = (hi ? oryx_readlane(bz1, J - 64) : oryx_readlane(bz0, J)) * inv;
        bz0 -= la * zJ;
        bz1 -= lb * zJ;
        if (lane == 0) {
          invs[J] = inv;
          zs[J] = zJ;
        }
        asm volatile("" : "+v"(bz0), "+v"(bz1));
        if (j < 15) {
          const float lJ = hi ? lb : la;     // column J of the diagonal-block rows
          if (j < 14) bcl[ln] = lJ;
          const float a1 = oryx_readlane(lJ, (J + 1) & 63);   // L[J+1][J]
          pa[j + 1] -= la * a1;
          pb[j + 1] -= lb * a1;
          asm volatile("" : "+v"(pa[j + 1]), "+v"(pb[j + 1]));
          sp = hi ? oryx_readlane(pb[j + 1], J + 1 - 64) : oryx_readlane(pa[j + 1], J + 1);
          if (j < 14) {
            const int base = (16 * pp) & 63;
            f32x4 bq[4];
#pragma unroll
            for (int q = (j + 2) / 4; q < 4; ++q)
              bq[q] = *reinterpret_cast<const lds_f32x4*>(bcl + base + 4 * q);
#pragma unroll
            for (int jj = j + 2; jj < 16; ++jj) {
              pa[jj] -= la * bq[jj / 4][jj % 4];
              pb[jj] -= lb * bq[jj / 4][jj % 4];
              asm volatile("" : "+v"(pa[jj]), "+v"(pb[jj]));
            }
          }
        }
      }
      // factored panel back to LDS (rows >= 16pp of each set)
      if (ln >= 16 * pp) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(P + r0 * LS + 4 * q) =
              f32x4{pa[4 * q], pa[4 * q + 1], pa[4 * q + 2], pa[4 * q + 3]};
      }
      if (ln + 64 >= 16 * pp && ln + 64 < KP) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(P + r1 * LS + 4 * q) =
              f32x4{pb[4 * q], pb[4 * q + 1], pb[4 * q + 2], pb[4 * q + 3]};
      }
      wave_sync();
      // trailing update A(i, jt) -= L(i, pp) L(jt, pp)^T on fp32 MFMA
      if (pp + 1 < M) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          float fr[M];
#pragma unroll
          for (int i = pp + 1; i < M; ++i) fr[i] = P[(16 * (i - pp) + fl) * LS + 4 * kk + g];
#pragma unroll
          for (int i = pp + 1; i < M; ++i)
#pragma unroll
            for (int jt = pp + 1; jt <= i; ++jt) {
              const int t = i * (i + 1) / 2 + jt;
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(-fr[i], fr[jt], acc[t], 0, 0, 0);
            }
        }
      }
      // L(i, pp) tiles back into the accumulators they came from (kept for the solve)
#pragma unroll
      for (int i = pp; i < M; ++i) {
        const int t = i * (i + 1) / 2 + pp;
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[t][v] = P[(16 * (i - pp) + 4 * g + v) * LS + fl];
      }
      wave_sync();
    });
    {
      // a clamped pivot gives 1/d = 1e15
      const float d0 = invs[lane], d1 = lane + 64 < KP ? invs[lane + 64] : 0.f;
      if (__any(!(d0 < 9.9e14f) || !(d1 < 9.9e14f)) && lane == 0 && p.fail_count)
        atomicAdd(p.fail_count, 1);
    }
    // blocked back substitution L^T x = z, last panel first
    static_for_desc<M>([&](auto PPc) {
      constexpr int pp = decltype(PPc)::value;
#pragma unroll
      for (int i = pp; i < M; ++i) {
        const int t = i * (i + 1) / 2 + pp;
#pragma unroll
        for (int v = 0; v < 4; ++v) P[(16 * (i - pp) + 4 * g + v) * LS + fl] = acc[t][v];
      }
      wave_sync();
      // rhs_c = z_c - sum_{J >= 16(pp+1)} L[J][c] x_J; lane (g, fl): column 16pp + fl, rows
      // J = 16(pp+1) + 4m + g
      float part = 0.f;
#pragma unroll
      for (int m = 0; m < 4 * (M - 1 - pp); ++m) {
        const int jr = 16 + 4 * m;   // panel-local row of J - g
        part += P[(jr + g) * LS + fl] * xs[16 * (pp + 1) + 4 * m + g];
      }
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      float rhs = zs[16 * pp + fl] - part;   // every g-group holds the same 16 values
#pragma unroll
      for (int cc = 15; cc >= 0; --cc) {
        const int c = 16 * pp + cc;
        const float x = oryx_readlane(rhs, cc) * invs[c];
        if (lane == 0) xs[c] = x;
        rhs -= P[cc * LS + fl] * x;     // row c of the panel, column 16pp + fl (fl < cc used)
      }
      wave_sync();
    });
    if (lane < KP) {
      const float x0 = xs[lane];
      p.X[(int64_t)row * KP + lane] = x0;
      if (p.Xb) store_xb<SPLIT, KP>(p.Xb, row, lane, x0);
    }
    if (lane + 64 < KP) {
      const float x1 = xs[lane + 64];
      p.X[(int64_t)row * KP + lane + 64] = x1;
      if (p.Xb) store_xb<SPLIT, KP>(p.Xb, row, lane + 64, x1);
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

    const int slot = p.long_slot ? p.long_slot[w] : -1;
    const int64_t stop = slot < 0 ? end : beg;  // split rows come from the workspace
    for (int64_t c0 = beg; c0 < stop; c0 += 32) {
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
        bf16x8 fa, fal;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float sv = (float)ra[j] * wsc[j];
          fa[j] = (__bf16)sv;
          fal[j] = (__bf16)(sv - (float)fa[j]);
        }
        acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, rb, acc[s], 0, 0, 0);
        if constexpr (kExactC)
          acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fal, rb, acc[s], 0, 0, 0);
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
    if (slot >= 0) {
      const float* src = p.ws + (int64_t)slot * ws_stride(KP);
      for (int idx = tid; idx < KP * KP; idx += 256) A[(idx / KP) * AS + idx % KP] = src[idx];
      if (tid < KP) s_b[tid] = src[KP * KP + tid];
      if (tid == 0) s_cnt = src[KP * KP + KP];
    }
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
  if (v < 0 || v > 5) return ORYX_EINVAL;
  g_als_variant = v;
  return ORYX_OK;
}

int oryx_als_get_variant() { return g_als_variant; }

int oryx_als_get_wide_variant() { return g_als_wide_variant; }

int oryx_als_set_wide_variant(int v) {
  if (v < 0 || v > 2) return ORYX_EINVAL;
  g_als_wide_variant = v;
  return ORYX_OK;
}

// long_slot [n_work] (nullable) marks split rows; segs [n_seg][4] = (row, slot, beg, end);
// ws: workspace of n_long * ws_stride(kp) floats (zeroed here).
int oryx_als_solve(const int64_t* row_ptr, const int32_t* row_ids, const int32_t* col_idx,
                   const float* vals, const void* Y, const float* YtY, float* X, void* Xb,
                   int n_work, int k, int kp, float lambda, float alpha, int implicit,
                   int* fail_count, const int32_t* long_slot, const int64_t* segs, int n_seg,
                   int n_long, float* ws, int split, long long nnz, void* stream) {
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
  if (n_seg > 0) {
    if (hipMemsetAsync(ws, 0, sizeof(float) * (size_t)n_long * ws_stride(kp), s) != hipSuccess)
      return ORYX_ELAUNCH;
    int blocks = (n_seg + 3) / 4;
    if (blocks > max_blocks) blocks = max_blocks;
    switch (kp) {
#define PART_CASE(KPV)                                                                    \
  case KPV:                                                                               \
    if (split)                                                                            \
      hipLaunchKernelGGL((als_partial<KPV, true>), dim3(blocks), dim3(256), 0, s, p, segs,  \
                         n_seg, ws);                                                      \
    else                                                                                  \
      hipLaunchKernelGGL((als_partial<KPV, false>), dim3(blocks), dim3(256), 0, s, p, segs, \
                         n_seg, ws);                                                      \
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
  }
  if (g_als_variant == 5 && g_als_wide_variant == 2 && (split || kp > 64)) {
    // two rows per wave, LDS-DMA gather (als_batch.hip): 64 < KP <= 128 and the fp32 mode
    const int cus = resident_panel_blocks / 2;
    const long long mean_len = n_work > 0 ? nnz / n_work : 0;
    if (const int rc = oryx_als::batch_gl_launch(p, kp, split != 0, env_blocks ? env_blocks : cus,
                                                 mean_len, s))
      return rc;
    return ORYX_OK;
  }
  if (g_als_variant == 5 && !split && kp <= 64) {
    // four rows per wave, one wave per SIMD: one resident block per CU
    const int cus = resident_panel_blocks / 2;
    if (const int rc = oryx_als::batch_solve_launch(p, kp, env_blocks ? env_blocks : cus, s))
      return rc;
    return ORYX_OK;
  }
  switch (kp) {
#define WAVE_CASE(KPV)                                                                \
  case KPV: {                                                                         \
    int blocks = (n_work + 3) / 4;                                                    \
    if (blocks > (split ? max_blocks : panel_blocks))                                 \
      blocks = split ? max_blocks : panel_blocks;                                     \
    if (split)                                                                        \
      hipLaunchKernelGGL((als_solve_wave<KPV, false, true>), dim3(blocks), dim3(256), 0, \
                         s, p, nullptr);                                              \
    else if (g_als_variant == 0)                                                      \
      hipLaunchKernelGGL((als_solve_panel<KPV, false>), dim3(blocks), dim3(256), 0, s, p, \
                         nullptr);                                                    \
    else if (g_als_variant == 2)                                                      \
      hipLaunchKernelGGL((als_solve_panel<KPV, false, true>), dim3(blocks), dim3(256), 0, \
                         s, p, nullptr);                                              \
    else if (g_als_variant == 3)                                                      \
      hipLaunchKernelGGL((als_solve_panel<KPV, false, true, 2>), dim3(blocks), dim3(256), \
                         0, s, p, nullptr);                                           \
    else if (g_als_variant == 4)                                                      \
      hipLaunchKernelGGL((als_solve_panel<KPV, false, true, 3>), dim3(blocks), dim3(256), \
                         0, s, p, nullptr);                                           \
    else                                                                              \
      hipLaunchKernelGGL((als_solve_wave<KPV, false>), dim3(blocks), dim3(256), 0, s, p, \
                         nullptr);                                                    \
    break;                                                                            \
  }
    WAVE_CASE(16)
    WAVE_CASE(32)
    WAVE_CASE(48)
    WAVE_CASE(64)
#undef WAVE_CASE
#define BLOCK_CASE(KPV)                                                               \
  case KPV: {                                                                         \
    if (split || g_als_wide_variant == 0) {                                           \
      int blocks = (n_work + 3) / 4;                                                  \
      if (blocks > max_blocks) blocks = max_blocks;                                   \
      if (split)                                                                      \
        hipLaunchKernelGGL((als_solve_wide<KPV, true>), dim3(blocks), dim3(256), 0, s, p); \
      else                                                                            \
        hipLaunchKernelGGL((als_solve_wide<KPV, false>), dim3(blocks), dim3(256), 0, s, p); \
    } else {                                                                          \
      int blocks = n_work < max_blocks ? n_work : max_blocks;                         \
      hipLaunchKernelGGL(als_solve_block<KPV>, dim3(blocks), dim3(256), 0, s, p);    \
    }                                                                                 \
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

// analysis: als_solve_wave<64> with per-phase cycle counters (prof: 6 u64, zeroed by caller)
int oryx_als_solve_profile64(const int64_t* row_ptr, const int32_t* row_ids,
                             const int32_t* col_idx, const float* vals, const void* Y,
                             const float* YtY, float* X, int n_work, int k, float lambda,
                             float alpha, int implicit, unsigned long long* prof, void* stream) {
  if (n_work <= 0) return ORYX_OK;
  AlsParams p{row_ptr, row_ids, col_idx, vals, reinterpret_cast<const __bf16*>(Y), YtY, X,
              nullptr, n_work, k, lambda, alpha, implicit, nullptr, nullptr, nullptr};
  int blocks = (n_work + 3) / 4;
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (g_als_variant == 0)
    hipLaunchKernelGGL((als_solve_panel<64, true>), dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), p, prof);
  else if (g_als_variant == 2)
    hipLaunchKernelGGL((als_solve_panel<64, true, true>), dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), p, prof);
  else if (g_als_variant == 3)
    hipLaunchKernelGGL((als_solve_panel<64, true, true, 2>), dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), p, prof);
  else if (g_als_variant == 4)
    hipLaunchKernelGGL((als_solve_panel<64, true, true, 3>), dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), p, prof);
  else
    hipLaunchKernelGGL((als_solve_wave<64, true>), dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), p, prof);
  return oryx_check_launch();
}

// analysis: subsequent KP=64 variant-5 solves count per-phase cycles into prof[0..6]
// (7 u64, zeroed by the caller; nullptr switches it off)
int oryx_als_batch_profile(unsigned long long* prof) {
  oryx_als::batch_set_profile(prof);
  return ORYX_OK;
}

int oryx_als_debug_gram(const int64_t* row_ptr, const int32_t* col_idx, const float* vals,
                        const void* Y, int kp, float alpha, int implicit, long long beg,
                        long long end, float* out, int split, void* stream) {
  AlsParams p{row_ptr, nullptr, col_idx, vals, reinterpret_cast<const __bf16*>(Y), nullptr,
              nullptr, nullptr, 1, kp, 0.f, alpha, implicit, nullptr, nullptr, nullptr};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (kp) {
#define DBG_CASE(KPV)                                                                       \
  case KPV:                                                                                 \
    if (split)                                                                              \
      hipLaunchKernelGGL((als_debug_gram<KPV, true>), dim3(1), dim3(64), 0, s, p,           \
                         (int64_t)beg, (int64_t)end, out);                                  \
    else                                                                                    \
      hipLaunchKernelGGL((als_debug_gram<KPV, false>), dim3(1), dim3(64), 0, s, p,          \
                         (int64_t)beg, (int64_t)end, out);                                  \
    break;
    DBG_CASE(16)
    DBG_CASE(32)
    DBG_CASE(48)
    DBG_CASE(64)
    DBG_CASE(80)
    DBG_CASE(96)
    DBG_CASE(112)
    DBG_CASE(128)
#undef DBG_CASE
    default:
      return ORYX_EINVAL;
  }
  return oryx_check_launch();
}

int oryx_kernels_version() { return 18; }

int oryx_als_ws_stride(int kp) { return ws_stride(kp); }

}  // extern "C"
