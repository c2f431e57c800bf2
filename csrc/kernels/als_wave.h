// als_wave.h -- the wave-per-row accumulation machinery of the ALS solve kernels:
// chunked bf16 gathers, the transposed LDS chunk image, the segmented MFMA Gramian
// (wave_accumulate) and its LDS / register layouts.  Shared by als.hip (the long-row
// partial sums of the default path) and tuning/als_variants.hip (the superseded solve
// kernels kept for A/B runs).  See als.hip for the math.
#pragma once

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

}  // namespace
