// als_batch.hip -- ALS half-step, FOUR rows per wave: gather + MFMA Gramian, then a batched
// block-LDL^T solve whose serial part runs on the 4 lane groups at once.
//
// Same math as als.hip (MLlib's ALS normal equations, [mllib]/als/ALSUpdate.java:116-124):
//   implicit: (YtY + sum_i c1_ui y_i y_i^T + lambda n+_u I) x_u = sum_{r_ui>0} (1 + c1_ui) y_i
//   explicit: (sum_i y_i y_i^T + lambda n_u I) x_u = sum_i r_ui y_i
//
// Why a second design (profiles/README.md, r1 v4/v5 phase tables): the one-row-per-wave panel
// kernel spends ~60% of a user row in a 64-step serial Cholesky (pivot -> rsq -> LDS/readlane
// broadcast -> update, ~200 cycles a step) and only 2 waves per SIMD cover it.  Here one wave
// owns four rows (KP <= 64):
//
//   * gather: the four rows' chunks of 32 ratings are consumed round-robin (chunk k of rows
//     0..3, then chunk k+1 ...) so every register ring slot and accumulator set is a
//     compile-time index; two chunks per row are in flight (register staged, 16-byte gathers
//     into a lane-linear swizzled LDS image, ds_read_b64_tr_b16 fragments, v_mfma_f32_16x16x32
//     _bf16 on the UPPER 16x16 tiles of each row's Gramian, which starts at YtY);
//   * solve, per 16-column panel p (block LDL^T):
//       - the 4 diagonal tiles go to the lane groups (group m = row m, lane r = tile row r);
//         LDL^T of all four 16x16 blocks runs at once, pivot rows broadcast inside each
//         16-lane row with DPP row_newbcast; the same row operations on [A | I] give
//         Li = L^{-1} (unit lower) alongside D;
//       - K_j = D^-1/2 Li U_pj for the blocks right of the diagonal: v_mfma_f32_16x16x4_f32
//         straight on the accumulator tiles (an accumulator-layout tile Y used as the A operand
//         is Y^T: D = Y^T X needs no data movement);
//       - trailing update U_ij -= K_i^T K_j on the same MFMA (exact fp32);
//       - forward solve z_p = D^-1/2 Li r_p, r_i -= K_i^T z_p (DPP broadcasts, group layout);
//   * back substitution x_p = Li^T D^-1/2 (z_p - sum_{i>p} K_i x_i), all four rows per
//     instruction.
// One wave per SIMD (512 registers: four 10-tile accumulator sets + the gather ring).

#include "als_common.h"
#include "dpp_fmac.h"

namespace {

// DPP row_newbcast:N -- every 16-lane row receives lane N of that row
template <int N>
__device__ __forceinline__ float rbc(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + N, 0xF, 0xF, true));
}

// wave-uniform copies in SGPRs (the metadata loads are vector loads: the kernel's stores keep
// the compiler from proving the arrays read-only)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// scalar (s_load) read of a read-only array through the constant address space: the value
// lands in SGPRs and is waited on lgkmcnt, never on the vmcnt of the gather ring
template <typename T>
__device__ __forceinline__ T sload(const T* base, int64_t i) {
  return ((const __attribute__((address_space(4))) T*)base)[i];
}

// index of upper tile (pi, qi), pi <= qi, row-major over the upper triangle
template <int M>
__host__ __device__ constexpr int tix(int pi, int qi) {
  return pi * M - pi * (pi - 1) / 2 + (qi - pi);
}

// scratch row stride in floats (20: ds_read_b128 rows conflict free; ORYX_ALS_BATCH_DS=16 packs
// the rows, A/B only)
#ifndef ORYX_ALS_BATCH_DS
#define ORYX_ALS_BATCH_DS 20
#endif
constexpr int BATCH_DS = ORYX_ALS_BATCH_DS;

template <int KP, int NM, int D, bool YG = false>
struct BatchCfg {
  static constexpr int M = KP / 16;
  static constexpr int NT = M * (M + 1) / 2;
  static constexpr int IMG = ChunkImage<KP>::BYTES;
  static constexpr int DS = BATCH_DS;
  static constexpr int SCR = NM * 16 * DS * 4;
  static constexpr int VEC = NM * 16 * 4;
  static constexpr int WAVE_BYTES = NM * IMG + NM * 256 + SCR + VEC;
  // YG: YtY read from global memory into the accumulators instead of staged in LDS (frees
  // the block's LDS for a third block per CU)
  static constexpr int YTY_BYTES = YG ? 0 : NT * 64 * 16;
  static constexpr int BYTES = YTY_BYTES + 4 * WAVE_BYTES;
};

typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(3))) f32x4 lds_f32x4;

// ---- replica layout of the solve (NM < 4 rows per wave): lane group g works on batch row
// g % NM as replica q = g / NM of R = 4 / NM.  The group-layout work (LDL^T of the diagonal
// tiles, forward / rhs / back substitution) splits a 16-column panel over the replicas --
// replica q owns columns R k + q, k < 16 / R -- instead of repeating it R times.
// v_permlane32_swap / v_permlane16_swap of a value with itself: (lo, hi) = the lower / upper
// half's value (32) or the even / odd row's value of each row pair (16), on every lane.  Inline
// asm: hipcc treats the two results of the swap builtins as interchangeable when both operands
// hold the same value, and picks the wrong one.  The nops cover a VALU write of the operands
// before the swap and a DPP read of its results right after it (neither is visible to the
// compiler's hazard recognizer through the asm).
__device__ __forceinline__ void swap32(float v, float& lo, float& hi) {
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  lo = a;
  hi = b;
}
__device__ __forceinline__ void swap16(float v, float& ev, float& od) {
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  ev = a;
  od = b;
}
// The value replica QJ holds for the same (row, tile row r), on every lane:
template <int R, int QJ>
__device__ __forceinline__ float from_rep(float v) {
  if constexpr (R == 1) {
    return v;
  } else if constexpr (R == 2) {   // replicas = wave halves
    float lo, hi;
    swap32(v, lo, hi);
    return QJ == 0 ? lo : hi;
  } else {                         // replicas = 16-lane rows: pair rows, then halves
    float ev, od, lo, hi;
    swap16(v, ev, od);
    swap32((QJ & 1) ? od : ev, lo, hi);
    return (QJ >> 1) ? hi : lo;
  }
}
// sum over the replicas (every replica gets it)
template <int R>
__device__ __forceinline__ float rep_sum(float v) {
  if constexpr (R == 1) {
    return v;
  } else if constexpr (R == 2) {
    float lo, hi;
    swap32(v, lo, hi);
    return lo + hi;
  } else {
    float ev, od, lo, hi;
    swap16(v, ev, od);
    swap32(ev + od, lo, hi);
    return lo + hi;
  }
}
// DPP row_ror:N (lane i of each 16-lane row reads lane (i - N) mod 16)
template <int N>
__device__ __forceinline__ float ror(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x120 + N, 0xF, 0xF, false));
}
// a copy in which lane i of replica q holds lane (i + q) mod 16's value, so that a DPP
// broadcast of lane R k reads column R k + q of the replica
template <int R>
__device__ __forceinline__ float rep_rot(float v, int q) {
  if constexpr (R == 1) {
    return v;
  } else if constexpr (R == 2) {
    const float t = ror<15>(v);
    return q ? t : v;
  } else {
    const float t1 = ror<15>(v), t2 = ror<14>(v), t3 = ror<13>(v);
    float r = q == 1 ? t1 : v;
    r = q == 2 ? t2 : r;
    return q == 3 ? t3 : r;
  }
}

#ifndef ORYX_ALS_SOLVE_LEGACY
#define ORYX_ALS_SOLVE_LEGACY 0
#endif
#if !ORYX_ALS_SOLVE_LEGACY
// Normal equations, batched block LDL^T + forward solve, back substitution of the NM rows one
// wave holds (lane group g works on row g % NM as replica g / NM, see from_rep).  acc: the
// upper 16x16 tiles of each row's Gramian (YtY included), bpart / cnt: the gather's per-lane
// partials.  scr / vdis: the wave's LDS scratch (NM*16 rows of DS floats, NM*16 floats).  Out:
// lane (m, r) holds x_m[16 pp + r] in xs[pp] (every replica).  hook(integral_constant<0>) runs
// after the first panel's LDL^T, hook(<1>) after the first (M == 1) or second panel -- the
// next batch's metadata is fetched there, under the solve.  phase(i) marks the per-phase cycle
// counters (analysis builds).
//
// Per panel p, the diagonal tile's LDL^T runs as row operations on [A | I] in row form: lane
// (row r, replica q) holds A[r][R k + q] and Li[r][R k + q]; step j subtracts m_r = A[r][j] /
// A[j][j] times pivot row j (a DPP broadcast of lane j inside each 16-lane row) from the rows
// below it.  The A half only needs the columns right of j and the Li half the ones up to j,
// so a step costs about 16 / R + 1 fused DPP FMAs; m_r comes from replica j % R by one or two
// lane-swap instructions.  Row form reads the pivot row's entries right of the diagonal, so
// the tile is made symmetric in LDS first (the upper entries of a Gramian tile built from
// bf16(c y) operands are not exactly the lower ones: the lower triangle is the matrix).
template <int KP, int NM, typename Hook, typename Phase>
__device__ __forceinline__ void batch_solve(const AlsParams& p, int lane,
                                            f32x4 (&acc)[NM][(KP / 16) * (KP / 16 + 1) / 2],
                                            float (&bpart)[NM][KP / 16], const float (&cnt)[NM],
                                            const int (&slot)[NM], const bool (&valid)[NM],
                                            lds_float* scr, lds_float* vdis, float (&xs)[KP / 16],
                                            Hook&& hook, Phase&& phase) {
  constexpr int M = KP / 16;
  constexpr int DS = BATCH_DS;
  constexpr int R = 4 / NM;
  constexpr int NC = 16 / R;
  const int g = lane >> 4, f = lane & 15;
  const int mg = g & (NM - 1);
  int q = g / NM;
  asm volatile("" : "+v"(q));
  // this lane's scratch row and its first column (R k + q: immediate offsets R k)
  lds_float* srow = scr + (mg * 16 + f) * DS + q;
  // ------------------------------------------------------------ normal equations
  float cntw[NM];
  static_for<NM>([&](auto Mc) {
    constexpr int m = decltype(Mc)::value;
    cntw[m] = wave_sum(cnt[m]);
    reduce_bpart<M>(bpart[m]);   // lane (g, f): bpart[m][pi] = b_m[16 pi + f]
    if (slot[m] >= 0) {
      // split row: Gramian, b and count were summed by als_partial into ws[slot]
      wait_long_row(p, slot[m]);
      const float* src = p.ws + (int64_t)slot[m] * ws_stride(KP);
#pragma unroll
      for (int pi = 0; pi < M; ++pi)
#pragma unroll
        for (int qi = pi; qi < M; ++qi)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            acc[m][tix<M>(pi, qi)][v] += src[(16 * pi + 4 * g + v) * KP + 16 * qi + f];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[m][pi] = src[KP * KP + 16 * pi + f];
      cntw[m] = src[KP * KP + KP];
    }
    // lambda n_u on the diagonal (1 on the zero-padded features, so they solve to 0)
    int rel = f - 4 * g;
    asm volatile("" : "+v"(rel));
#pragma unroll
    for (int pp = 0; pp < M; ++pp) {
      const float dg = 16 * pp + f < p.k ? p.lambda * cntw[m] : 1.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[m][tix<M>(pp, pp)][v] += rel == v ? dg : 0.f;
    }
  });
  // right-hand sides in group layout: lane (m, r) holds b_m[16 pi + r]
  float rhs[M];
#pragma unroll
  for (int pi = 0; pi < M; ++pi) {
    float r = bpart[0][pi];
    static_for<NM - 1>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value + 1;
      r = mg == m ? bpart[m][pi] : r;
    });
    rhs[pi] = r;
  }

  phase(2);
  // ------------------------------------------------------------ block LDL^T + forward
  float zp[M], disv[M];
  int bad = 0;
  static_for<M>([&](auto Pc) {
    constexpr int pp = decltype(Pc)::value;
    constexpr int td = tix<M>(pp, pp);
    // diagonal tiles -> symmetric rows in LDS: scratch row (m, b) position a = T(a, b) for
    // a <= b (the accumulator column), then T(a, b) also to row a position b for a < b
#pragma unroll
    for (int m = 0; m < NM; ++m)
      *reinterpret_cast<lds_f32x4*>(scr + (m * 16 + f) * DS + 4 * g) = acc[m][td];
    {
      int rel = f - 4 * g;
      asm volatile("" : "+v"(rel));
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (rel > v) scr[(m * 16 + 4 * g + v) * DS + f] = acc[m][td][v];
    }
    wave_sync();
    float a[NC], e[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) a[k] = srow[R * k];
    wave_sync();
    {
      int fq = f - q;
      asm volatile("" : "+v"(fq));
#pragma unroll
      for (int k = 0; k < NC; ++k) e[k] = R * k == fq ? 1.f : 0.f;
    }
    static_for<16>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      const float val = from_rep<R, j % R>(a[j / R]);   // A[r][j], every replica
      float piv = rbc<j>(val);
      piv = piv > 1e-30f ? piv : 1e-30f;
      int rl = f - j;
      asm volatile("" : "+v"(rl));
      const float nml = rl > 0 ? -(val * __builtin_amdgcn_rcpf(piv)) : 0.f;
      // A half: columns right of j; Li half: columns up to j (Li[r][j] = -m_r comes out of
      // the pivot row's Li[j][j] = 1)
      dfb_n<j, (j + 1) / R, NC - (j + 1) / R>(nml, a);
      dfb_n<j, 0, j / R + 1>(nml, e);
    });
    phase(3);
    if constexpr (pp == 0) hook(std::integral_constant<int, 0>{});
    // the pivots: A[r][r] is left in place (rows are not touched from their own step on)
#pragma unroll
    for (int k = 0; k < NC; ++k) srow[R * k] = a[k];
    wave_sync();
    float dself = scr[(mg * 16 + f) * DS + f];
    wave_sync();
    bad |= !(dself > 0.f);
    dself = dself > 1e-30f ? dself : 1e-30f;
    const float dis = __builtin_amdgcn_rsqf(dself);
    disv[pp] = dis;
    // forward: z_p = D^-1/2 Li r_p
    float z0 = 0.f, z1 = 0.f;
    dfc_s<R, 0, NC>(z0, z1, rep_rot<R>(rhs[pp], q), e);
    const float z = rep_sum<R>(z0 + z1) * dis;
    zp[pp] = z;
    const float zq = rep_rot<R>(z, q);
    // Li rows and D^-1/2 to LDS; back as Li^T in accumulator layout (lane (g, f): Li[f][4g+v])
#pragma unroll
    for (int k = 0; k < NC; ++k) srow[R * k] = e[k];
    vdis[mg * 16 + f] = dis;
    wave_sync();
    f32x4 Y[NM], d4[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      Y[m] = *reinterpret_cast<const lds_f32x4*>(scr + (m * 16 + f) * DS + 4 * g);
      d4[m] = *reinterpret_cast<const lds_f32x4*>(vdis + m * 16 + 4 * g);
    }
    wave_sync();
    // K_j = D^-1/2 Li U_pj in place of U_pj
    static_for<M - 1 - pp>([&](auto Jc) {
      constexpr int j = pp + 1 + decltype(Jc)::value;
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        f32x4 K = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int v = 0; v < 4; ++v)
          K = __builtin_amdgcn_mfma_f32_16x16x4f32(Y[m][v], acc[m][tix<M>(pp, j)][v], K, 0, 0,
                                                    0);
#pragma unroll
        for (int v = 0; v < 4; ++v) K[v] *= d4[m][v];
        acc[m][tix<M>(pp, j)] = K;
      }
    });
    // trailing update U_ij -= K_i^T K_j (i <= j), before the rhs work so it overlaps it
    static_for<M - 1 - pp>([&](auto Ic) {
      constexpr int i = pp + 1 + decltype(Ic)::value;
      static_for<M - i>([&](auto Jc) {
        constexpr int j = i + decltype(Jc)::value;
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            acc[m][tix<M>(i, j)] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                -acc[m][tix<M>(pp, i)][v], acc[m][tix<M>(pp, j)][v], acc[m][tix<M>(i, j)], 0,
                0, 0);
      });
    });
    // r_i -= K_i^T z_p: column r of K_i to lane (m, r) through LDS (the replica's columns),
    // z broadcast by DPP
    static_for<M - 1 - pp>([&](auto Ic) {
      constexpr int i = pp + 1 + decltype(Ic)::value;
#pragma unroll
      for (int m = 0; m < NM; ++m)
        *reinterpret_cast<lds_f32x4*>(scr + (m * 16 + f) * DS + 4 * g) = acc[m][tix<M>(pp, i)];
      wave_sync();
      float col[NC];
#pragma unroll
      for (int k = 0; k < NC; ++k) col[k] = srow[R * k];
      wave_sync();
      float o0 = 0.f, o1 = 0.f;
      dfc_s<R, 0, NC>(o0, o1, zq, col);
      rhs[i] -= rep_sum<R>(o0 + o1);
    });
    // keep Li^T (accumulator layout) for the back substitution in the dead diagonal tile
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m][td] = Y[m];
    if constexpr (pp == (M > 1 ? 1 : 0)) hook(std::integral_constant<int, 1>{});
    phase(4);
  });
  {
    const unsigned long long bm = __ballot(bad != 0);
    if (lane == 0 && p.fail_count) {
      int nbad = 0;
#pragma unroll
      for (int m = 0; m < NM; ++m) nbad += (valid[m] && ((bm >> (16 * m)) & 0xFFFFull)) ? 1 : 0;
      if (nbad) atomicAdd(p.fail_count, nbad);
    }
  }

  // ------------------------------------------------------------ back substitution
  // row form of an accumulator-layout tile T of every row: lane (m, r, q) gets T_m[r][R k + q]
  auto rows_of = [&](const f32x4* T, float (&out)[NC]) {
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int v = 0; v < 4; ++v) scr[(m * 16 + 4 * g + v) * DS + f] = T[m][v];
    wave_sync();
#pragma unroll
    for (int k = 0; k < NC; ++k) out[k] = srow[R * k];
    wave_sync();
  };
  static_for_desc<M>([&](auto Pc) {
    constexpr int pp = decltype(Pc)::value;
    float w0 = 0.f, w1 = 0.f;
    static_for<M - 1 - pp>([&](auto Ic) {
      constexpr int i = pp + 1 + decltype(Ic)::value;
      f32x4 T[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) T[m] = acc[m][tix<M>(pp, i)];
      float row[NC];
      rows_of(T, row);   // K_i[r][R k + q]
      dfc_s<R, 0, NC>(w0, w1, rep_rot<R>(xs[i], q), row);
    });
    const float yv = (zp[pp] - rep_sum<R>(w0 + w1)) * disv[pp];
    f32x4 T[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) T[m] = acc[m][tix<M>(pp, pp)];
    float col[NC];
    rows_of(T, col);   // Li^T[a][c] = Li[c][a], c = R k + q
    float x0 = 0.f, x1 = 0.f;
    dfc_s<R, 0, NC>(x0, x1, rep_rot<R>(yv, q), col);
    xs[pp] = rep_sum<R>(x0 + x1);
  });
}

#else   // the pre-r5 solve (each replica repeats the group-layout work), for A/B builds
// Normal equations, batched block LDL^T + forward solve, back substitution of the NM rows one
// wave holds (lane group g works on row g % NM).  acc: the upper 16x16 tiles of each row's
// Gramian (YtY included), bpart / cnt: the gather's per-lane partials.  scr / vdis: the wave's
// LDS scratch (NM*16 rows of DS floats, NM*16 floats).  Out: lane (m, r) holds x_m[16 pp + r]
// in xs[pp].  hook(integral_constant<0>) runs after the first panel's LDL^T, hook(<1>) after the
// first (M == 1) or second panel -- the next batch's metadata is fetched there, under the
// solve.  phase(i) marks the per-phase cycle counters (analysis builds).
template <int KP, int NM, typename Hook, typename Phase>
__device__ __forceinline__ void batch_solve(const AlsParams& p, int lane,
                                            f32x4 (&acc)[NM][(KP / 16) * (KP / 16 + 1) / 2],
                                            float (&bpart)[NM][KP / 16], const float (&cnt)[NM],
                                            const int (&slot)[NM], const bool (&valid)[NM],
                                            lds_float* scr, lds_float* vdis, float (&xs)[KP / 16],
                                            Hook&& hook, Phase&& phase) {
  constexpr int M = KP / 16;
  constexpr int DS = BATCH_DS;
  const int g = lane >> 4, f = lane & 15;
  const int mg = g & (NM - 1);
  // ------------------------------------------------------------ normal equations
  float cntw[NM];
  static_for<NM>([&](auto Mc) {
    constexpr int m = decltype(Mc)::value;
    cntw[m] = wave_sum(cnt[m]);
    reduce_bpart<M>(bpart[m]);   // lane (g, f): bpart[m][pi] = b_m[16 pi + f]
    if (slot[m] >= 0) {
      // split row: Gramian, b and count were summed by als_partial into ws[slot]
      wait_long_row(p, slot[m]);
      const float* src = p.ws + (int64_t)slot[m] * ws_stride(KP);
#pragma unroll
      for (int pi = 0; pi < M; ++pi)
#pragma unroll
        for (int qi = pi; qi < M; ++qi)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            acc[m][tix<M>(pi, qi)][v] += src[(16 * pi + 4 * g + v) * KP + 16 * qi + f];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[m][pi] = src[KP * KP + 16 * pi + f];
      cntw[m] = src[KP * KP + KP];
    }
    // lambda n_u on the diagonal (1 on the zero-padded features, so they solve to 0)
    int rel = f - 4 * g;
    asm volatile("" : "+v"(rel));
#pragma unroll
    for (int pp = 0; pp < M; ++pp) {
      const float dg = 16 * pp + f < p.k ? p.lambda * cntw[m] : 1.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[m][tix<M>(pp, pp)][v] += rel == v ? dg : 0.f;
    }
  });
  // right-hand sides in group layout: lane (m, r) holds b_m[16 pi + r]
  float rhs[M];
#pragma unroll
  for (int pi = 0; pi < M; ++pi) {
    float r = bpart[0][pi];
    static_for<NM - 1>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value + 1;
      r = mg == m ? bpart[m][pi] : r;
    });
    rhs[pi] = r;
  }

  phase(2);
  // ------------------------------------------------------------ block LDL^T + forward
  float zp[M], disv[M];
  int bad = 0;
  static_for<M>([&](auto Pc) {
    constexpr int pp = decltype(Pc)::value;
    constexpr int td = tix<M>(pp, pp);
    // diagonal tiles -> group layout: lane (m, r) gets column r of the tile, whose entries
    // c <= r are the lower-triangle row r (the elimination below reads nothing else)
#pragma unroll
    for (int m = 0; m < NM; ++m)
      *reinterpret_cast<lds_f32x4*>(scr + (m * 16 + f) * DS + 4 * g) = acc[m][td];
    wave_sync();
    float a[16], e[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = *reinterpret_cast<const lds_f32x4*>(scr + (mg * 16 + f) * DS + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) a[4 * q + u] = v[u];
    }
    wave_sync();
    int fr = f;
    asm volatile("" : "+v"(fr));
#pragma unroll
    for (int c = 0; c < 16; ++c) e[c] = c == fr ? 1.f : 0.f;
    float dself = 1.f;
    // [A | I] row operations on the lower triangle only: row r -= m_r row j uses the pivot
    // row's entries a_j[c] (c > j), which by symmetry are a_c[j] -- column j of lane c,
    // broadcast inside each 16-lane row; the identity half takes lane j's row as it is
    static_for<16>([&](auto Jc) {
      constexpr int j = decltype(Jc)::value;
      float piv = rbc<j>(a[j]);
      bad |= !(piv > 0.f);
      piv = piv > 1e-30f ? piv : 1e-30f;
      const float mr = a[j] * __builtin_amdgcn_rcpf(piv);
      int rl = f - j;
      asm volatile("" : "+v"(rl));
      const float nml = rl > 0 ? -mr : 0.f;   // -L[r][j] (rows r <= j untouched)
      dself = rl == 0 ? piv : dself;
      // fused DPP FMAs (dpp_fmac.h); the next pivot column a[j+1] is the first of the group
      dfa_range<j + 1, 15 - j>(a, a[j], nml);
      dfb_range<j, 0, j>(nml, e);
      e[j] = rl > 0 ? -mr : e[j];
    });
    phase(3);
    if constexpr (pp == 0) hook(std::integral_constant<int, 0>{});
    const float dis = __builtin_amdgcn_rsqf(dself);
    disv[pp] = dis;
    // forward: z_p = D^-1/2 Li r_p
    float z0 = 0.f, z1 = 0.f;
    dfc_range<0, 16>(z0, z1, rhs[pp], e);
    const float z = (z0 + z1) * dis;
    zp[pp] = z;
    // Li rows and D^-1/2 to LDS; back as Li^T in accumulator layout (lane (g, f): Li[f][4g+v])
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<lds_f32x4*>(scr + (mg * 16 + f) * DS + 4 * q) =
          f32x4{e[4 * q], e[4 * q + 1], e[4 * q + 2], e[4 * q + 3]};
    vdis[mg * 16 + f] = dis;
    wave_sync();
    f32x4 Y[NM], d4[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      Y[m] = *reinterpret_cast<const lds_f32x4*>(scr + (m * 16 + f) * DS + 4 * g);
      d4[m] = *reinterpret_cast<const lds_f32x4*>(vdis + m * 16 + 4 * g);
    }
    wave_sync();
    // K_j = D^-1/2 Li U_pj in place of U_pj
    static_for<M - 1 - pp>([&](auto Jc) {
      constexpr int j = pp + 1 + decltype(Jc)::value;
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        f32x4 K = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int v = 0; v < 4; ++v)
          K = __builtin_amdgcn_mfma_f32_16x16x4f32(Y[m][v], acc[m][tix<M>(pp, j)][v], K, 0, 0,
                                                    0);
#pragma unroll
        for (int v = 0; v < 4; ++v) K[v] *= d4[m][v];
        acc[m][tix<M>(pp, j)] = K;
      }
    });
    // trailing update U_ij -= K_i^T K_j (i <= j), before the rhs work so it overlaps it
    static_for<M - 1 - pp>([&](auto Ic) {
      constexpr int i = pp + 1 + decltype(Ic)::value;
      static_for<M - i>([&](auto Jc) {
        constexpr int j = i + decltype(Jc)::value;
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            acc[m][tix<M>(i, j)] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                -acc[m][tix<M>(pp, i)][v], acc[m][tix<M>(pp, j)][v], acc[m][tix<M>(i, j)], 0,
                0, 0);
      });
    });
    // r_i -= K_i^T z_p: column f of K_i to lane (m, f) through LDS, z broadcast by DPP
    static_for<M - 1 - pp>([&](auto Ic) {
      constexpr int i = pp + 1 + decltype(Ic)::value;
#pragma unroll
      for (int m = 0; m < NM; ++m)
        *reinterpret_cast<lds_f32x4*>(scr + (m * 16 + f) * DS + 4 * g) = acc[m][tix<M>(pp, i)];
      wave_sync();
      float col[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *reinterpret_cast<const lds_f32x4*>(scr + (mg * 16 + f) * DS + 4 * q);
#pragma unroll
        for (int u = 0; u < 4; ++u) col[4 * q + u] = v[u];
      }
      wave_sync();
      float o0 = 0.f, o1 = 0.f;
      dfc_range<0, 16>(o0, o1, z, col);
      rhs[i] -= o0 + o1;
    });
    // keep Li^T (accumulator layout) for the back substitution in the dead diagonal tile
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m][td] = Y[m];
    if constexpr (pp == (M > 1 ? 1 : 0)) hook(std::integral_constant<int, 1>{});
    phase(4);
  });
  {
    const unsigned long long bm = __ballot(bad != 0);
    if (lane == 0 && p.fail_count) {
      int nbad = 0;
#pragma unroll
      for (int m = 0; m < NM; ++m) nbad += (valid[m] && ((bm >> (16 * m)) & 0xFFFFull)) ? 1 : 0;
      if (nbad) atomicAdd(p.fail_count, nbad);
    }
  }

  // ------------------------------------------------------------ back substitution
  // row form of an accumulator-layout tile T of every row: lane (m, r) gets T_m[r][0..15]
  auto rows_of = [&](const f32x4* T, float (&out)[16]) {
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int v = 0; v < 4; ++v) scr[(m * 16 + 4 * g + v) * DS + f] = T[m][v];
    wave_sync();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = *reinterpret_cast<const lds_f32x4*>(scr + (mg * 16 + f) * DS + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) out[4 * q + u] = v[u];
    }
    wave_sync();
  };
  static_for_desc<M>([&](auto Pc) {
    constexpr int pp = decltype(Pc)::value;
    float w = zp[pp];
    static_for<M - 1 - pp>([&](auto Ic) {
      constexpr int i = pp + 1 + decltype(Ic)::value;
      f32x4 T[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) T[m] = acc[m][tix<M>(pp, i)];
      float row[16];
      rows_of(T, row);   // lane (m, r): K_i[r][0..15]
      float o0 = 0.f, o1 = 0.f;
      dfc_range<0, 16>(o0, o1, xs[i], row);
      w -= o0 + o1;
    });
    const float yv = w * disv[pp];
    f32x4 T[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) T[m] = acc[m][tix<M>(pp, pp)];
    float col[16];
    rows_of(T, col);   // lane (m, a): Li^T[a][c] = Li[c][a]
    float x0 = 0.f, x1 = 0.f;
    dfc_range<0, 16>(x0, x1, yv, col);
    xs[pp] = x0 + x1;
  });
}

#endif  // ORYX_ALS_SOLVE_LEGACY

// D: chunks in flight per row (register ring depth); the wave keeps NM * D gathers in flight.
// PROF: per-phase shader-clock cycles summed into prof[0..7] (analysis build,
// scripts/als_phase_profile.py)
// NM = 4: one wave per SIMD (512 registers), lane group g owns row g.  NM = 2: two waves per
// SIMD (256 registers each), lane groups g and g + 2 both hold row g & 1 (the group-layout
// work is duplicated, but the SIMD interleaves the two waves' VALU streams -- one wave alone
// issues a VALU instruction every 4 cycles, two fill the SIMD-32's 2-cycle slots -- and one
// wave's gather overlaps the other's MFMA-heavy solve).
// BPC: resident blocks of 4 waves per CU (waves per SIMD).  Past 4 / NM the YtY tiles come
// from global memory (YG) so that BPC blocks' LDS fits the CU's 160 KB: at NM = 2, rank 64,
// three blocks of 45.5 KB instead of two of 55.8 KB -- a third wave per SIMD to hide the
// solve's latency-bound LDL^T chain behind the other waves' work.
template <int KP, int NM, int D, bool PROF = false, int BPC = 4 / NM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BPC, BPC))) void
als_solve_batch(AlsParams p, unsigned long long* prof) {
  // YtY from global memory only when BPC blocks with it staged in LDS do not fit
  constexpr bool YG = BPC > 4 / NM && BatchCfg<KP, NM, D, false>::BYTES * BPC > 160 * 1024;
  using C = BatchCfg<KP, NM, D, YG>;
  static_assert(C::BYTES * BPC <= 160 * 1024, "BPC blocks do not fit the CU's LDS");
  using CI = ChunkImage<KP>;
  constexpr int M = C::M;
  constexpr int NT = C::NT;
  constexpr int NPL = CI::NPL;
  constexpr int PPR = CI::PPR;
  constexpr int DS = C::DS;
  static_assert(NM == 4 || NM == 2, "lane group g owns row g % NM of the batch");
  __shared__ __attribute__((aligned(16))) char smem[C::BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, f = lane & 15;
  const int mg = g & (NM - 1);   // the row of the batch this lane's group works on
  char* my = smem + C::YTY_BYTES + wave * C::WAVE_BYTES;
  char* img = my;
  float* wab = reinterpret_cast<float*>(my + NM * C::IMG);
  lds_float* scr = (lds_float*)(my + NM * C::IMG + NM * 256);
  lds_float* vdis = scr + NM * 16 * DS;

  // YtY in accumulator order: tile t, lane l -> rows 16pi + 4(l>>4) + v, column 16qi + (l&15)
  if constexpr (!YG) {
    float* ya = reinterpret_cast<float*>(smem);
    for (int i = threadIdx.x; i < NT * 64; i += 256) {
      const int t = i >> 6, ln = i & 63;
      int pi = 0, rem = t;
      while (rem >= M - pi) {
        rem -= M - pi;
        ++pi;
      }
      const int qi = pi + rem;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        ya[i * 4 + v] = p.YtY[(16 * pi + 4 * (ln >> 4) + v) * KP + 16 * qi + (ln & 15)];
    }
    __syncthreads();
  }
  const lds_f32x4* ytya = (const lds_f32x4*)smem;

  // per-lane staging geometry: slot it of a chunk = rating srow[it], feature chunk soff[it]
  int srow[NPL], soff[NPL];
#pragma unroll
  for (int it = 0; it < NPL; ++it) {
    const int sl = it * 64 + lane, r = sl / PPR, sc = sl % PPR;
    srow[it] = r;
    soff[it] = ((sc + CI::rot(r)) % PPR) * 8;
  }
  const int q4 = f >> 2, p4 = f & 3;
  auto tr_addr = [&](int pi, int h) -> int {
    const int row = 8 * g + 4 * h + q4;
    const int pc = 2 * pi + (p4 >> 1);
    const int sc = (pc - CI::rot(row) + PPR) % PPR;
    return row * KP * 2 + sc * 16 + (p4 & 1) * 8;
  };

  const int nb = (p.n_work + NM - 1) / NM;
  const int total_waves = gridDim.x * 4;
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = PROF ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int ix) {
    if constexpr (PROF) {
      const unsigned long long tn = __builtin_amdgcn_s_memtime();
      ph[ix] += tn - tp;
      tp = tn;
    }
  };
  // Row metadata of a batch arrives in three dependent round trips (work list -> row_ptr ->
  // column ids of the first chunks).  For the next batch they are issued in stages under this
  // batch's solve (stage1 after the gather loop, stage2 after the first LDL^T, stage3 after the
  // first panel), so a batch starts with its first gathers' column ids already in registers.
  int rows_n[NM], slot_n[NM], len_n[NM];
  int64_t b_n[NM], e_n[NM], beg_n[NM];
  bool valid_n[NM];
  int cols_n[NM][D][NPL];
  float val_n[NM][D];
  auto stage1 = [&](int b) {
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      const int w = b * NM + m;
      valid_n[m] = w < p.n_work;
      int ww = valid_n[m] ? w : p.n_work - 1;   // tail: a real row, solved, not stored
      if (!ORYX_ALS_NO_PART_WAIT) {
        ww += p.rot;                                // (rotated: the long rows come last)
        ww -= ww >= p.n_work ? p.n_work : 0;
      }
      rows_n[m] = p.row_ids ? sload(p.row_ids, ww) : ww;
      slot_n[m] = (valid_n[m] && p.long_slot) ? sload(p.long_slot, ww) : -1;
    });
  };
  auto stage2 = [&]() {
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      b_n[m] = sload(p.row_ptr, rows_n[m]);
      e_n[m] = sload(p.row_ptr, rows_n[m] + 1);
    });
  };
  // byte offset of rating o of a row of length n, clamped into the row (a uniform base plus a
  // 32-bit offset is one global_load with an SGPR base)
  auto clampo = [&](int n, int o) -> unsigned {
    o = o < n ? o : n - 1;
    return (unsigned)(o < 0 ? 0 : o) * 4u;
  };
  auto ld_cols_at = [&](const int32_t* cb, int n, int ch, int (&c)[NPL]) {
    const char* b = reinterpret_cast<const char*>(cb);
#pragma unroll
    for (int it = 0; it < NPL; ++it)
      c[it] = *reinterpret_cast<const int*>(b + clampo(n, 32 * ch + srow[it]));
  };
  auto ld_val_at = [&](const float* vb, int n, int ch, float& v) {
    v = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(vb) +
                                        clampo(n, 32 * ch + (lane & 31)));
  };
  auto stage3 = [&]() {
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      beg_n[m] = b_n[m];
      const int64_t en = (slot_n[m] >= 0 || !valid_n[m]) ? beg_n[m] : e_n[m];
      len_n[m] = (int)(en - beg_n[m]);
      const int64_t b0 = len_n[m] > 0 ? beg_n[m] : 0;
      static_for<D>([&](auto Sc) {
        constexpr int s = decltype(Sc)::value;
        ld_cols_at(p.col_idx + b0, len_n[m], s, cols_n[m][s]);
        ld_val_at(p.vals + b0, len_n[m], s, val_n[m][s]);
      });
    });
  };
  if (blockIdx.x * 4 + wave < nb) {
    stage1(blockIdx.x * 4 + wave);
    stage2();
    stage3();
  }

  for (int bi = blockIdx.x * 4 + wave; bi < nb; bi += total_waves) {
    // the next batch of this wave (the last one re-loads itself: the stages run
    // unconditionally, so their results are dead during the gather loop -- a conditional stage
    // would keep the previous values live through it and spill)
    const int bnext = bi + total_waves < nb ? bi + total_waves : bi;
    int rows[NM], slot[NM];
    bool valid[NM];
    int nr = 0;
    // per-row uniform bases, per-lane 32-bit offsets
    const int32_t* cbase[NM];
    const float* vbase[NM];
    int len[NM];
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      rows[m] = rows_n[m];
      slot[m] = slot_n[m];
      valid[m] = valid_n[m];
      len[m] = len_n[m];
      const int64_t b0 = len[m] > 0 ? beg_n[m] : 0;
      cbase[m] = p.col_idx + b0;
      vbase[m] = p.vals + b0;
      const int nch = (len[m] + 31) / 32;
      nr = nch > nr ? nch : nr;
    });

    phase(0);
    // ------------------------------------------------------------ gather + MFMA Gramian
    f32x4 acc[NM][NT];
    float bpart[NM][M], cnt[NM];
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      if constexpr (YG) {
        if constexpr (m == 0) {
          // (rows 16 pi + 4 g + v, columns 16 qi + f of YtY; L2-resident, 4 KB per row)
          static_for<M>([&](auto Pc) {
            constexpr int pi = decltype(Pc)::value;
            static_for<M - pi>([&](auto Qc) {
              constexpr int qi = pi + decltype(Qc)::value;
#pragma unroll
              for (int v = 0; v < 4; ++v)
                acc[0][tix<M>(pi, qi)][v] = p.YtY[(16 * pi + 4 * g + v) * KP + 16 * qi + f];
            });
          });
        } else {
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[m][t] = acc[0][t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[m][t] = ytya[t * 64 + lane];
      }
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[m][pi] = 0.f;
      cnt[m] = 0.f;
    });

    auto ld_cols = [&](int m, int ch, int (&c)[NPL]) { ld_cols_at(cbase[m], len[m], ch, c); };
    auto ld_val = [&](int m, int ch, float& v) { ld_val_at(vbase[m], len[m], ch, v); };
    const char* ybase = reinterpret_cast<const char*>(p.Y);
    auto gather = [&](const int (&c)[NPL], i32x4 (&st)[NPL]) {
#pragma unroll
      for (int it = 0; it < NPL; ++it)
        st[it] = *reinterpret_cast<const i32x4*>(
            ybase + ((unsigned)c[it] * (unsigned)(KP * 2) + (unsigned)(soff[it] * 2)));
    };

    // ring: chunk s of every row; its column ids and values were prefetched (stage3)
    i32x4 stg[NM][D][NPL];
    int cols[NM][D][NPL];
    float val[NM][D];
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      static_for<D>([&](auto Sc) {
        constexpr int s = decltype(Sc)::value;
#pragma unroll
        for (int it = 0; it < NPL; ++it) cols[m][s][it] = cols_n[m][s][it];
        val[m][s] = val_n[m][s];
      });
    });
    if (nr > 0) {
      static_for<NM>([&](auto Mc) {
        constexpr int m = decltype(Mc)::value;
        static_for<D>([&](auto Sc) {
          constexpr int s = decltype(Sc)::value;
          gather(cols[m][s], stg[m][s]);
          ld_cols(m, D + s, cols[m][s]);
        });
      });
    }
    // consume chunk kk of row m from ring slot s (= kk % D); refill the slot with chunk kk + D
    // (its columns were loaded a round earlier) and load the columns of chunk kk + 2D.
    // Branch-free on purpose: a conditional prefetch or a divergent block splits the round
    // into basic blocks, and the waitcnt insertion then waits for nearly every load in flight
    // (vmcnt(4)) before each prefetch -- the ring drained every chunk.  Past the row's end
    // the loads are clamped to its last rating (one cached Y row) and the weights are zero.
    const float alpha = p.alpha;
    const bool implicit = p.implicit != 0;
    auto consume = [&](auto Mc, auto Sc, int kk) {
      constexpr int m = decltype(Mc)::value;
      constexpr int s = decltype(Sc)::value;
      const int left = len[m] - 32 * kk;
      const bool live = (lane & 31) < left;
      const float r = val[m][s];
      const float c1 = alpha * fabsf(r);
      const bool pos = r > 0.f;
      const float wa = live ? (implicit ? c1 : 1.f) : 0.f;
      const float wb = live ? (implicit ? (pos ? 1.f + c1 : 0.f) : r) : 0.f;
      cnt[m] += (live && (!implicit || pos) && lane < 32) ? 1.f : 0.f;
      float* W = wab + m * 64;
      char* G = img + m * C::IMG;
      // lanes l and l + 32 hold the same rating: both write the same value
      W[lane & 31] = wa;
      W[32 + (lane & 31)] = wb;
#pragma unroll
      for (int it = 0; it < NPL; ++it)
        *reinterpret_cast<i32x4*>(G + (it * 64 + lane) * 16) = stg[m][s][it];
      wave_sync();
      ld_val(m, kk + D, val[m][s]);
      gather(cols[m][s], stg[m][s]);
      ld_cols(m, kk + 2 * D, cols[m][s]);
      const f32x4* wv = reinterpret_cast<const f32x4*>(W);
      const f32x4 wa0 = wv[2 * g], wa1 = wv[2 * g + 1];
      const f32x4 wb0 = wv[8 + 2 * g], wb1 = wv[8 + 2 * g + 1];
      bf16x8 fb[M];
#pragma unroll
      for (int pi = 0; pi < M; ++pi) {
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 0)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf16x4*)(G + tr_addr(pi, 1)));
        fb[pi] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      // upper tile (pi, qi) = y_(16pi+a) bf16(c y_(16qi+b)): the weighted operand is always
      // the one of the larger feature index, so every entry equals the LOWER-triangle entry
      // bf16(c y_r) y_c (r >= c) of the reference model (the bf16 rounding of c*y makes the
      // accumulated Gramian slightly asymmetric; only its lower triangle is the matrix)
      // weights as register pairs matching the fragment's bf16 pairs (ratings 8g+2i, +1)
      const f32x2 wap[4] = {f32x2{wa0[0], wa0[1]}, f32x2{wa0[2], wa0[3]},
                            f32x2{wa1[0], wa1[1]}, f32x2{wa1[2], wa1[3]}};
      const f32x2 wbp[4] = {f32x2{wb0[0], wb0[1]}, f32x2{wb0[2], wb0[3]},
                            f32x2{wb1[0], wb1[1]}, f32x2{wb1[2], wb1[3]}};
#pragma unroll
      for (int qi = 0; qi < M; ++qi) {
        // bf16(c y) per pair: unpack (shift / mask), v_pk_mul_f32, v_cvt_pk_bf16_f32; the same
        // unpacked pair feeds b's v_pk_fma_f32
        const i32x4 raw = __builtin_bit_cast(i32x4, fb[qi]);
        i32x4 wraw;
        f32x2 bacc = f32x2{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned u = (unsigned)raw[i];
          const f32x2 y = f32x2{__builtin_bit_cast(float, u << 16),
                                __builtin_bit_cast(float, u & 0xffff0000u)};
          const f32x2 cy = y * wap[i];
          bacc = y * wbp[i] + bacc;
          typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
          wraw[i] = __builtin_bit_cast(int, __builtin_convertvector(cy, bf16x2));
        }
        const bf16x8 fa = __builtin_bit_cast(bf16x8, wraw);
        bpart[m][qi] += bacc[0] + bacc[1];
#pragma unroll
        for (int pi = 0; pi <= qi; ++pi)
          acc[m][tix<M>(pi, qi)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              fb[pi], fa, acc[m][tix<M>(pi, qi)], 0, 0, 0);
      }
      wave_sync();
    };
    for (int k = 0; k < nr; k += D) {
      static_for<D>([&](auto Sc) {
        const int kk = k + decltype(Sc)::value;
        if (kk < nr) static_for<NM>([&](auto Mc) { consume(Mc, Sc, kk); });
      });
    }

    phase(1);
    stage1(bnext);
    float xs[M];
    batch_solve<KP, NM>(p, lane, acc, bpart, cnt, slot, valid, scr, vdis, xs,
                        [&](auto Hc) {
                          if constexpr (decltype(Hc)::value == 0) stage2();
                          else stage3();
                        },
                        phase);

    // lane (m, r) holds x_m[16 pp + r]
    int orow = rows[0];
    bool ok = valid[0];
    static_for<NM - 1>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value + 1;
      orow = mg == m ? rows[m] : orow;
      ok = mg == m ? valid[m] : ok;
    });
    if (ok && g < NM) {
#pragma unroll
      for (int pp = 0; pp < M; ++pp) {
        p.X[(int64_t)orow * KP + 16 * pp + f] = xs[pp];
        if (p.Xb) p.Xb[(int64_t)orow * KP + 16 * pp + f] = (__bf16)xs[pp];
      }
    }
    phase(5);
    if constexpr (PROF) ph[6] += 1;
  }
  if constexpr (PROF) {
    if (lane == 0)
      for (int i = 0; i < 7; ++i) atomicAdd(prof + i, ph[i]);
  }
}

// ------------------------------------------------------------------ LDS-DMA batched kernel
//
// als_solve_batch_gl: the same two-rows-per-wave batched block-LDL^T solve for the kernels whose
// Gramians do not leave room for a register gather ring: 64 < KP <= 128 (36 accumulator tiles
// per row at KP = 128, 288 registers for the pair) and the fp32 factor mode (SPLIT: every
// factor row is bf16 hi + lo, so a chunk is twice the bytes).  Y rows go straight from global
// memory into the wave's LDS chunk image with global_load_lds_dwordx4 (no VGPR staging, no
// ds_write pass); the chunk's 32 column ids and 32 values arrive the same way (one
// global_load_lds_dword: lanes 0-31 ids, 32-63 values) one chunk ahead, so the column ids that
// address the next gather are read from LDS, and the chunk loop holds no ordinary global load.
//
// Per wave: one image slot per row (SLOT bytes) and two metadata slots per row.  Round kk
// consumes chunk kk of row 0 then of row 1; consuming (m, kk) ends by issuing the gather of
// (m, kk + 1) into m's slot and the metadata of (m, kk + 2), so each row's gather lands while
// the other row's chunk is on the MFMAs.  The DMA loads are issued from inline asm, outside the
// compiler's waitcnt bookkeeping; the kernel waits for them itself: when (m, kk) starts, the
// only VMEM operations issued after its gather are the other row's G, so vmcnt(G) retires it.
// The next batch's metadata and first chunks are fetched under the current batch's solve
// (hooks of batch_solve); the scratch of the solve does not alias the image slots.
//
// One wave per SIMD at KP > 64 (the pair's accumulators), two at KP <= 64 (fp32 factor mode).
template <int KP, bool SPLIT, int NM_, int WPE_>
struct GlCfg {
  static constexpr int NM = NM_;
  static constexpr int M = KP / 16;
  static constexpr int NT = M * (M + 1) / 2;
  static constexpr int IMG = ChunkImage<KP>::BYTES;
  static constexpr int SLOT = IMG * (SPLIT ? 2 : 1);
  static constexpr int NPL = ChunkImage<KP>::NPL;
  static constexpr int G = NPL * (SPLIT ? 2 : 1) + 1;   // VMEM operations of one chunk issue
  static constexpr int META = 256;                      // 32 column ids + 32 values
  static constexpr int SCR = NM * 16 * BATCH_DS * 4;
  // four rows per wave: the solve's scratch lives in image slots 2-3 (their next chunks are
  // issued after the solve), so two such waves per SIMD fit the CU's LDS
  // (when it fits there: KP >= 64)
  static constexpr bool ALIAS = NM == 4 && 2 * SLOT >= SCR + NM * 16 * 4;
  static constexpr int WAVE_BYTES =
      NM * SLOT + NM * 2 * META + (ALIAS ? 0 : SCR + NM * 16 * 4);
  // image slots whose next chunks are prefetched under the solve
  static constexpr int PRE = ALIAS ? 2 : NM;
  // waves per SIMD (1: 512 registers per wave)
  static constexpr int WPE = WPE_;
  static constexpr int BYTES = 4 * WAVE_BYTES;
};

// one LDS-DMA load: lane l's 16 (4) bytes from src land at LDS byte address lds + 16 l (4 l).
// M0 carries the wave-uniform LDS base and is restored afterwards (the compiler reserves it).
__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void glds4(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
// N LDS-DMA loads of 16 bytes per lane into consecutive 1 KB pieces from lds on: one asm
// statement, M0 stepped by s_add (instead of saving / setting / restoring it per load)
#ifndef ORYX_GL_ISSUE_BATCH
#define ORYX_GL_ISSUE_BATCH 1
#endif
#ifndef ORYX_GL_COMPACT
#define ORYX_GL_COMPACT 0
#endif
#define GL_L(i) "s_nop 0\n\tglobal_load_lds_dwordx4 %" #i ", off\n\t"
#define GL_A "s_add_u32 m0, m0, 0x400\n\t"
template <int N>
__device__ __forceinline__ void glds16_run(const char* const (&src)[N], uint32_t lds) {
  unsigned keep;
  if constexpr (N == 8) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %9\n\t"
                 GL_L(1) GL_A GL_L(2) GL_A GL_L(3) GL_A GL_L(4) GL_A GL_L(5) GL_A GL_L(6) GL_A
                 GL_L(7) GL_A GL_L(8) "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src[0]), "v"(src[1]), "v"(src[2]), "v"(src[3]), "v"(src[4]), "v"(src[5]),
                   "v"(src[6]), "v"(src[7]), "s"(lds)
                 : "memory", "scc");
  } else if constexpr (N == 16) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %17\n\t"
                 GL_L(1) GL_A GL_L(2) GL_A GL_L(3) GL_A GL_L(4) GL_A GL_L(5) GL_A GL_L(6) GL_A
                 GL_L(7) GL_A GL_L(8) GL_A GL_L(9) GL_A GL_L(10) GL_A GL_L(11) GL_A GL_L(12) GL_A
                 GL_L(13) GL_A GL_L(14) GL_A GL_L(15) GL_A GL_L(16) "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src[0]), "v"(src[1]), "v"(src[2]), "v"(src[3]), "v"(src[4]), "v"(src[5]),
                   "v"(src[6]), "v"(src[7]), "v"(src[8]), "v"(src[9]), "v"(src[10]),
                   "v"(src[11]), "v"(src[12]), "v"(src[13]), "v"(src[14]), "v"(src[15]),
                   "s"(lds)
                 : "memory", "scc");
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) glds16(src[i], lds + i * 1024);
  }
}
#undef GL_L
#undef GL_A

// wait until at most N vector-memory operations of this wave are outstanding
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// every LDS read issued so far has returned (before a DMA overwrites what they read)
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// HOLD_HI: the hi fragments of a chunk stay in registers (the lo ones are re-read from the image
// where they are used); otherwise both are re-read (KP > 64: registers)
// WPE_: waves per SIMD -- one for a pair of rows at KP > 64 (the pair's accumulators), and for
// single rows of long average length (no spills at 512 registers); two otherwise
template <int KP, bool SPLIT, int NM_ = 2, bool PROF = false, bool HOLD_HI = (KP <= 64),
          int WPE_ = ((NM_ == 2 && KP > 64) ? 1 : 2)>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE_, WPE_))) void
als_solve_batch_gl(AlsParams p, unsigned long long* prof) {
  using C = GlCfg<KP, SPLIT, NM_, WPE_>;
  using CI = ChunkImage<KP>;
  constexpr int NM = C::NM;
  constexpr int M = C::M;
  constexpr int NT = C::NT;
  constexpr int NPL = C::NPL;
  constexpr int PPR = CI::PPR;
  constexpr int G = C::G;
  constexpr int YS = SPLIT ? 2 * KP : KP;   // factor row stride in bf16 elements
  __shared__ __attribute__((aligned(16))) char smem[C::BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, f = lane & 15;
  char* my = smem + wave * C::WAVE_BYTES;
  const uint32_t my_lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)my);
  auto slot_ptr = [&](int m) -> char* { return my + m * C::SLOT; };
  auto slot_lds = [&](int m) -> uint32_t { return my_lds + m * C::SLOT; };
  auto meta_ptr = [&](int m, int q) -> char* {
    return my + NM * C::SLOT + (m * 2 + q) * C::META;
  };
  auto meta_lds = [&](int m, int q) -> uint32_t {
    return my_lds + NM * C::SLOT + (m * 2 + q) * C::META;
  };
  lds_float* scr =
      (lds_float*)(C::ALIAS ? my + 2 * C::SLOT : my + NM * C::SLOT + NM * 2 * C::META);
  lds_float* vdis = scr + NM * 16 * BATCH_DS;

  // Lane-derived values are recomputed from an opaque lane id at each use in the chunk loop:
  // hoisted out of it, they were spilled, and every scratch reload is a VMEM wait that the
  // compiler counts as vmcnt(0) -- draining the LDS-DMA prefetch of the other row.
  auto olane = [&]() -> int {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    return ln;
  };
  // per-lane image geometry: slot it*64 + lane of a chunk = rating srow(it), piece soff(it)
  auto srow = [&](int it) -> int {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    return (it * 64 + ln) / PPR;
  };
  auto soff = [&](int it) -> int {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int sl = it * 64 + ln, r = sl / PPR, sc = sl % PPR;
    return ((sc + CI::rot(r)) % PPR) * 8;
  };
  const int nb = (p.n_work + NM - 1) / NM;
  const int total_waves = gridDim.x * 4;
  // ph[7]: cycles waiting for LDS-DMA gathers, ph[8]: issuing them (both inside phase 1)
  unsigned long long ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = PROF ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int ix) {
    if constexpr (PROF) {
      const unsigned long long tn = __builtin_amdgcn_s_memtime();
      ph[ix] += tn - tp;
      tp = tn;
    }
  };

  // ---- next-batch metadata (wave-uniform; scalar loads) and its first chunks (LDS-DMA)
  int rows_n[NM], slot_n[NM], len_n[NM];
  int64_t b_n[NM], e_n[NM], beg_n[NM];
  bool valid_n[NM];
  auto stage1 = [&](int b) {
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      const int w = b * NM + m;
      valid_n[m] = w < p.n_work;
      int ww = valid_n[m] ? w : p.n_work - 1;   // tail: a real row, solved, not stored
      if (!ORYX_ALS_NO_PART_WAIT) {
        ww += p.rot;                                // (rotated: the long rows come last)
        ww -= ww >= p.n_work ? p.n_work : 0;
      }
      rows_n[m] = p.row_ids ? sload(p.row_ids, ww) : ww;
      slot_n[m] = (valid_n[m] && p.long_slot) ? sload(p.long_slot, ww) : -1;
    });
  };
  // chunk ch's column ids (lanes 0-31) and values (lanes 32-63) of row m into meta slot q;
  // offsets clamped into the row (a row without ratings reads element 0)
  auto issue_meta = [&](int m, int64_t beg, int len, int ch, int q) {
    const int64_t b0 = len > 0 ? beg : 0;
    const int ln = olane();
    int o = 32 * ch + (ln & 31);
    o = o < len ? o : len - 1;
    o = o < 0 ? 0 : o;
    // ids and values are both 4-byte arrays: one uniform base each, the lane picks
    const char* cb = reinterpret_cast<const char*>(p.col_idx + b0);
    const char* vb = reinterpret_cast<const char*>(p.vals + b0);
    const uint64_t d = (uint64_t)(vb - cb);
    glds4(cb + ((uint64_t)((unsigned)o * 4u) + (ln < 32 ? 0ull : d)), meta_lds(m, q));
  };
  // chunk gather of row m into its image slot, column ids from meta slot q
  const char* ybase = reinterpret_cast<const char*>(p.Y);
  auto issue_y = [&](int m, int q) {
    const __attribute__((address_space(3))) int* cid =
        (const __attribute__((address_space(3))) int*)meta_ptr(m, q);
    int c[NPL];
#pragma unroll
    for (int it = 0; it < NPL; ++it) c[it] = cid[srow(it)];
    if constexpr (ORYX_GL_ISSUE_BATCH && C::IMG == NPL * 1024) {
      // the hi pieces, then (fp32 mode) the lo pieces right behind them: one asm run
      constexpr int NS = NPL * (SPLIT ? 2 : 1);
      const char* src[NS];
#pragma unroll
      for (int it = 0; it < NPL; ++it) {
        src[it] = ybase + ((size_t)(unsigned)c[it] * (YS * 2) + (unsigned)(soff(it) * 2));
        if constexpr (SPLIT) src[NPL + it] = src[it] + KP * 2;
      }
      glds16_run<NS>(src, slot_lds(m));
    } else {
#pragma unroll
      for (int it = 0; it < NPL; ++it) {
        const char* src =
            ybase + ((size_t)(unsigned)c[it] * (YS * 2) + (unsigned)(soff(it) * 2));
        glds16(src, slot_lds(m) + it * 1024);
        if constexpr (SPLIT) glds16(src + KP * 2, slot_lds(m) + C::IMG + it * 1024);
      }
    }
  };
  auto stage2 = [&]() {
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      b_n[m] = sload(p.row_ptr, rows_n[m]);
      e_n[m] = sload(p.row_ptr, rows_n[m] + 1);
      beg_n[m] = b_n[m];
      const int64_t en = (slot_n[m] >= 0 || !valid_n[m]) ? beg_n[m] : e_n[m];
      len_n[m] = (int)(en - beg_n[m]);
    });
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      issue_meta(m, beg_n[m], len_n[m], 0, 0);
      issue_meta(m, beg_n[m], len_n[m], 1, 1);
    });
  };
  // the first chunks of rows 0 .. N-1 (under the solve: the slots its scratch does not use)
  auto stage3 = [&](auto Nc) {
    vm_wait<0>();   // the metadata above (and anything older) has landed
    static_for<decltype(Nc)::value>([&](auto Mc) { issue_y(decltype(Mc)::value, 0); });
  };
  if (blockIdx.x * 4 + wave < nb) {
    stage1(blockIdx.x * 4 + wave);
    stage2();
    stage3(std::integral_constant<int, NM>{});
  }

  const float alpha = p.alpha;
  const bool implicit = p.implicit != 0;
  for (int bi = blockIdx.x * 4 + wave; bi < nb; bi += total_waves) {
    const int bnext = bi + total_waves < nb ? bi + total_waves : bi;
    int rows[NM], slot[NM], len[NM];
    bool valid[NM];
    int nr = 0;
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      rows[m] = rows_n[m];
      slot[m] = slot_n[m];
      valid[m] = valid_n[m];
      len[m] = len_n[m];
      const int nch = (len[m] + 31) / 32;
      nr = nch > nr ? nch : nr;
    });
    int64_t beg[NM];
    static_for<NM>([&](auto Mc) { beg[decltype(Mc)::value] = beg_n[decltype(Mc)::value]; });

    phase(0);
    // ------------------------------------------------------------ gather + MFMA Gramian
    f32x4 acc[NM][NT];
    float bpart[NM][M], cnt[NM];
    // YtY in accumulator order: tile (pi, qi), lane (g, f) -> rows 16pi + 4g + v, column 16qi + f
    // (one uniform base + a 32-bit lane offset per load: 64-bit per-load addresses hoisted out of
    // the batch loop were spilled)
    {
      int lo = (4 * g * KP + f) * 4;
      asm volatile("" : "+v"(lo));
      const char* yb = reinterpret_cast<const char*>(p.YtY);
#pragma unroll
      for (int pi = 0; pi < M; ++pi)
#pragma unroll
        for (int qi = pi; qi < M; ++qi)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            acc[0][tix<M>(pi, qi)][v] = *reinterpret_cast<const float*>(
                yb + (unsigned)(lo + ((16 * pi + v) * KP + 16 * qi) * 4));
    }
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      if constexpr (m > 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[m][t] = acc[0][t];
      }
#pragma unroll
      for (int pi = 0; pi < M; ++pi) bpart[m][pi] = 0.f;
      cnt[m] = 0.f;
    });

    auto consume = [&](auto Mc, int kk) {
      constexpr int m = decltype(Mc)::value;
      const char* S = slot_ptr(m);
      const int q = kk & 1;
      // this lane's 8 ratings (8g .. 8g+7 of the chunk) -> Gramian / rhs weights
      const int gl = olane() >> 4;
      const f32x4 r0 = *(const lds_f32x4*)(meta_ptr(m, q) + 128 + 32 * gl);
      const f32x4 r1 = *(const lds_f32x4*)(meta_ptr(m, q) + 128 + 32 * gl + 16);
      // transposed-read byte offsets of this lane (operand pi, half h), made once per chunk from
      // an opaque lane id: slot row 8g + 4h + q4, piece (2 pi + p4/2 - rot(row)) mod PPR
      // COMPACT (power-of-two pieces per row): two row bases and the rotation instead of the
      // 2M-entry table, the piece offset recomputed per read (two VALU ops).  On by default
      // at two waves per SIMD, where the 16 registers it frees cut the chunk loop's spills
      // (rank-128 fp32 users half-step 6.38 vs 6.57 ms; profiles/r3_als128_gl_ab.txt); at
      // 512 registers it only adds VALU work.
      constexpr bool COMPACT = (ORYX_GL_COMPACT || C::WPE == 2) && (PPR & (PPR - 1)) == 0 &&
                               !(KP <= 64);
      int tra[COMPACT ? 1 : M][2];
      int tb[2], tc[2];
      {
        const int ln = olane();
        const int sb = (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)S;
        const int q4 = (ln >> 2) & 3, p4 = ln & 3, gg = ln >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = 8 * gg + 4 * h + q4;
          const int base = sb + row * KP * 2 + (p4 & 1) * 8;
          const int c = (p4 >> 1) - CI::rot(row) + PPR;
          tb[h] = base;
          tc[h] = c;
          if constexpr (!COMPACT) {
#pragma unroll
            for (int pi = 0; pi < M; ++pi) tra[pi][h] = base + ((2 * pi + c) % PPR) * 16;
          }
        }
      }
      auto addr = [&](int pi, int h) -> int {
        if constexpr (COMPACT) return tb[h] + (((2 * pi + tc[h]) & (PPR - 1)) << 4);
        else return tra[pi][h];
      };
      auto rd = [&](int off, int pi) -> bf16x8 {
        typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4*)(uintptr_t)(uint32_t)(addr(pi, 0) + off));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4*)(uintptr_t)(uint32_t)(addr(pi, 1) + off));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      // each tile row re-reads its fragments at opaque (in-place redefined) addresses: merged
      // with the previous row's reads of the same bytes, they would all be held in registers
      auto fresh_addresses = [&]() {
        if constexpr (COMPACT) {
          asm volatile("" : "+v"(tb[0]), "+v"(tb[1]), "+v"(tc[0]), "+v"(tc[1]));
        } else {
#pragma unroll
          for (int pi = 0; pi < M; ++pi) asm volatile("" : "+v"(tra[pi][0]), "+v"(tra[pi][1]));
        }
      };
      // Fragments are re-read from the image where they are used (KP > 64: holding them would
      // spill the pair's accumulators; KP <= 64 holds the hi fragments).  LDS has the room: at
      // KP = 128 fp32, 144 ds_read_b64_tr_b16 per chunk and row cost 288 LDS-array cycles per
      // wave against 1728 cycles of MFMAs.
      constexpr bool HOLD = HOLD_HI;
      // a single row at 512 registers also holds the fp32 mode's lo fragments (all reads up
      // front, no re-reads, no per-tile-row LDS waits)
      constexpr bool HOLD_LO = HOLD && SPLIT && NM == 1 && C::WPE == 1;
      bf16x8 fbh[HOLD ? M : 1], fbl[HOLD_LO ? M : 1];
      if constexpr (HOLD) {
#pragma unroll
        for (int pi = 0; pi < M; ++pi) fbh[pi] = rd(0, pi);
      }
      if constexpr (HOLD_LO) {
#pragma unroll
        for (int pi = 0; pi < M; ++pi) fbl[pi] = rd(C::IMG, pi);
      }
      auto fbr = [&](int pi) -> bf16x8 {
        if constexpr (HOLD) return fbh[pi];
        else return rd(0, pi);
      };
      auto flr = [&](int pi) -> bf16x8 {
        if constexpr (HOLD_LO) return fbl[pi];
        else return rd(C::IMG, pi);
      };
      const int left = len[m] - 32 * kk - 8 * gl;
      float wa[8], wb[8], cn = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // straight-line selects (a conditional expression here became a divergent branch)
        const float r = j < 4 ? r0[j] : r1[j - 4];
        const float lv = __builtin_amdgcn_fmed3f((float)(left - j), 0.f, 1.f);   // 1 iff j < left
        const float c1 = alpha * fabsf(r);
        const float pos = r > 0.f ? 1.f : 0.f;
        const float a_ = implicit ? c1 : 1.f;
        const float b_ = implicit ? pos * (1.f + c1) : r;
        wa[j] = a_ * lv;
        wb[j] = b_ * lv;
        cn += (implicit ? pos : 1.f) * lv;
      }
      cnt[m] += (olane() & 15) == 0 ? cn : 0.f;
      const f32x2 wap[4] = {f32x2{wa[0], wa[1]}, f32x2{wa[2], wa[3]}, f32x2{wa[4], wa[5]},
                            f32x2{wa[6], wa[7]}};
      const f32x2 wbp[4] = {f32x2{wb[0], wb[1]}, f32x2{wb[2], wb[3]}, f32x2{wb[4], wb[5]},
                            f32x2{wb[6], wb[7]}};
      typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
#pragma unroll
      for (int qi = 0; qi < M; ++qi) {
        // weighted operand of the larger feature index (see als_solve_batch): bf16(c y), and in
        // the fp32 factor mode y = hi + lo and c y split into bf16 hi + lo
        if constexpr (!(KP <= 64)) fresh_addresses();
        const bf16x8 fq = fbr(qi);
        const i32x4 raw = __builtin_bit_cast(i32x4, fq);
        i32x4 rawl;
        if constexpr (SPLIT) rawl = __builtin_bit_cast(i32x4, flr(qi));
        i32x4 whi, wlo;
        f32x2 bacc = f32x2{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned u = (unsigned)raw[i];
          f32x2 y = f32x2{__builtin_bit_cast(float, u << 16),
                          __builtin_bit_cast(float, u & 0xffff0000u)};
          if constexpr (SPLIT) {
            const unsigned ul = (unsigned)rawl[i];
            y += f32x2{__builtin_bit_cast(float, ul << 16),
                       __builtin_bit_cast(float, ul & 0xffff0000u)};
          }
          const f32x2 cy = y * wap[i];
          bacc = y * wbp[i] + bacc;
          const bf16x2 h = __builtin_convertvector(cy, bf16x2);
          whi[i] = __builtin_bit_cast(int, h);
          if constexpr (SPLIT) {
            const f32x2 hb = __builtin_convertvector(h, f32x2);
            wlo[i] = __builtin_bit_cast(int, __builtin_convertvector(cy - hb, bf16x2));
          }
        }
        const bf16x8 fa = __builtin_bit_cast(bf16x8, whi);
        bpart[m][qi] += bacc[0] + bacc[1];
#pragma unroll
        for (int pi = 0; pi <= qi; ++pi) {
          const bf16x8 fp = pi == qi ? fq : fbr(pi);
          acc[m][tix<M>(pi, qi)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              fp, fa, acc[m][tix<M>(pi, qi)], 0, 0, 0);
          if constexpr (SPLIT) {
            const bf16x8 fal = __builtin_bit_cast(bf16x8, wlo);
            acc[m][tix<M>(pi, qi)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                pi == qi ? __builtin_bit_cast(bf16x8, rawl) : flr(pi), fa,
                acc[m][tix<M>(pi, qi)], 0, 0, 0);
            acc[m][tix<M>(pi, qi)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fp, fal, acc[m][tix<M>(pi, qi)], 0, 0, 0);
          }
        }
      }
      if (kk + 1 < nr) {
        // the slot's fragments and meta slot q's values have been read: overwrite them with
        // chunk kk + 1 (ids from meta slot q ^ 1) and the metadata of chunk kk + 2
        phase(1);
        lds_drain();
        issue_y(m, q ^ 1);
        issue_meta(m, beg[m], len[m], kk + 2, q);
        phase(8);
      }
    };
    // Round kk consumes chunk kk of rows 0 .. NM-1.  Waiting for (m, kk)'s gather: the VMEM
    // operations issued after it are (m+1 .. NM-1, kk) from the previous round and, unless
    // this is the last round, (0 .. m-1, kk+1) from this one -- G each (round 0: everything of
    // the first chunks has been waited for at m = 0).
    for (int kk = 0; kk < nr; ++kk) {
      static_for<NM>([&](auto Mc) {
        constexpr int m = decltype(Mc)::value;
        phase(1);
        if (kk == 0) {
          if (m == 0 || nr == 1) vm_wait<0>();
          else vm_wait<m * G>();
        } else if (kk + 1 < nr) {
          vm_wait<(NM - 1) * G>();
        } else {
          vm_wait<(NM - 1 - m) * G>();
        }
        phase(7);
        consume(Mc, kk);
      });
    }

    phase(1);
    stage1(bnext);
    float xs[M];
    batch_solve<KP, NM>(p, lane, acc, bpart, cnt, slot, valid, scr, vdis, xs,
                        [&](auto Hc) {
                          if constexpr (decltype(Hc)::value == 0) stage2();
                          else stage3(std::integral_constant<int, C::PRE>{});
                        },
                        phase);
    if constexpr (C::ALIAS) {
      // the scratch slots are free again: the next batch's first chunks of rows PRE ..
      lds_drain();
      static_for<NM - C::PRE>([&](auto Mc) { issue_y(C::PRE + decltype(Mc)::value, 0); });
    }

    // lane (m, r) holds x_m[16 pp + r] (NM < 4: the other groups duplicate rows 0 .. NM-1)
    int orow = rows[0];
    bool ok = valid[0];
    static_for<NM - 1>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value + 1;
      orow = (g & (NM - 1)) == m ? rows[m] : orow;
      ok = (g & (NM - 1)) == m ? valid[m] : ok;
    });
    if (ok && g < NM) {
#pragma unroll
      for (int pp = 0; pp < M; ++pp) {
        p.X[(int64_t)orow * KP + 16 * pp + f] = xs[pp];
        if (p.Xb) store_xb<SPLIT, KP>(p.Xb, orow, 16 * pp + f, xs[pp]);
      }
    }
    phase(5);
    if constexpr (PROF) ph[6] += 1;
  }
  // no DMA into this workgroup's LDS may be in flight when the wave retires
  vm_wait<0>();
  if constexpr (PROF) {
    if (lane == 0)
      for (int i = 0; i < 9; ++i) atomicAdd(prof + i, ph[i]);
  }
}

}  // namespace

namespace oryx_als {

#ifndef ORYX_ALS_BATCH_DEPTH
#define ORYX_ALS_BATCH_DEPTH 1
#endif
// rows per wave: 2 (two waves per SIMD, default) or 4 (one wave per SIMD)
#ifndef ORYX_ALS_BATCH_BPC_DEFAULT
#define ORYX_ALS_BATCH_BPC_DEFAULT 2
#endif
#ifndef ORYX_ALS_BATCH_NM
#define ORYX_ALS_BATCH_NM 2
#endif

static unsigned long long* g_batch_prof = nullptr;

void batch_set_profile(unsigned long long* prof) { g_batch_prof = prof; }

// blocks of 4 waves per CU for the rank <= 64 solve: ORYX_ALS_BATCH_BPC (NM = 2: 2 or 3)
static int batch_bpc() {
  static const int v = [] {
    const char* e = getenv("ORYX_ALS_BATCH_BPC");
    return e ? atoi(e) : ORYX_ALS_BATCH_BPC_DEFAULT;
  }();
  return v;
}

int batch_solve_launch(const AlsParams& p, int kp, int max_blocks, hipStream_t s) {
  constexpr int NM = ORYX_ALS_BATCH_NM;
  constexpr int D = ORYX_ALS_BATCH_DEPTH;
  constexpr int BPC0 = 4 / NM;
  const bool three = NM == 2 && batch_bpc() == 3;
  // one resident generation: BPC blocks of 4 waves per CU (max_blocks = CUs unless
  // overridden by ORYX_ALS_MAX_BLOCKS)
  const int nb = (p.n_work + NM - 1) / NM;
  int blocks = (nb + 3) / 4;
  const int cap = max_blocks * (three ? 3 : BPC0);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  constexpr int BPC3 = NM == 2 ? 3 : BPC0;   // (the third block exists only for NM = 2)
  if (g_batch_prof && kp == 64) {
    if (three)
      hipLaunchKernelGGL((als_solve_batch<64, NM, D, true, BPC3>), dim3(blocks), dim3(256), 0,
                         s, p, g_batch_prof);
    else
      hipLaunchKernelGGL((als_solve_batch<64, NM, D, true>), dim3(blocks), dim3(256), 0, s, p,
                         g_batch_prof);
    return oryx_check_launch();
  }
  switch (kp) {
#define BATCH_CASE(KPV)                                                                       \
  case KPV:                                                                                   \
    if (three)                                                                                \
      hipLaunchKernelGGL((als_solve_batch<KPV, NM, D, false, BPC3>), dim3(blocks), dim3(256), \
                         0, s, p, nullptr);                                                  \
    else                                                                                      \
      hipLaunchKernelGGL((als_solve_batch<KPV, NM, D>), dim3(blocks), dim3(256), 0, s, p,    \
                         nullptr);                                                           \
    break;
    BATCH_CASE(16)
    BATCH_CASE(32)
    BATCH_CASE(48)
    BATCH_CASE(64)
#undef BATCH_CASE
    default:
      return ORYX_EINVAL;
  }
  return oryx_check_launch();
}

// Rank-128 configuration (rows per wave NM, waves per SIMD WPE).  Measured per half-step
// before the replica-split solve (rank-128 fp32, 25M ratings; profiles/r3_als128_gl_*):
//   items (423 ratings per row): NM 1 / WPE 1 4.63 ms, NM 2 / WPE 1 5.17, NM 1 / WPE 2 5.54;
//   users (154 per row):         NM 1 / WPE 2 6.46 ms, NM 1 / WPE 1 7.02, NM 2 / WPE 1 7.08.
// Long rows want the spill-free 512-register wave (the gather dominates and a spill reload
// waits for the whole DMA in flight); short rows want two waves per SIMD to overlap one row's
// serial LDL^T with the other's gather.  ORYX_ALS_GL_NM / ORYX_ALS_GL_WPE force either.
static void gl_config(long long mean_len, int& nm, int& wpe) {
  static const int fnm = [] {
    const char* e = getenv("ORYX_ALS_GL_NM");
    return e ? atoi(e) : 0;
  }();
  static const int fwpe = [] {
    const char* e = getenv("ORYX_ALS_GL_WPE");
    return e ? atoi(e) : 0;
  }();
  nm = fnm == 2 ? 2 : 1;
  // r5: with the replica-split solve (a panel's group-layout work on four lane groups instead
  // of repeated by each) the one-wave configuration wins at every row length: users 6.11 ms
  // (two waves: 8.0, where the 256-register wave spills), items 4.18 ms
  (void)mean_len;
  wpe = 1;
  if (nm == 1 && (fwpe == 1 || fwpe == 2)) wpe = fwpe;
}

static bool gl_hold() {
  static const bool v = [] {
    const char* e = getenv("ORYX_ALS_GL_HOLD");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

int batch_gl_launch(const AlsParams& p, int kp, bool split, int cus, long long mean_len,
                    hipStream_t s) {
  // one resident generation: WPE blocks of 4 waves per CU, NM rows per wave
  int nm = 2, wpe = kp > 64 ? 1 : 2;
  if (kp == 128) gl_config(mean_len, nm, wpe);
  const int nb = (p.n_work + nm - 1) / nm;
  int blocks = (nb + 3) / 4;
  if (blocks > cus * wpe) blocks = cus * wpe;
  if (blocks < 1) blocks = 1;
  if (kp == 128) {
#define GL128(SP, NMV, WV, HV)                                                                \
  do {                                                                                        \
    if (g_batch_prof)                                                                         \
      hipLaunchKernelGGL((als_solve_batch_gl<128, SP, NMV, true, HV, WV>), dim3(blocks),      \
                         dim3(256), 0, s, p, g_batch_prof);                                   \
    else                                                                                      \
      hipLaunchKernelGGL((als_solve_batch_gl<128, SP, NMV, false, HV, WV>), dim3(blocks),     \
                         dim3(256), 0, s, p, nullptr);                                        \
  } while (0)
    if (nm == 2) {
      if (split) GL128(true, 2, 1, false); else GL128(false, 2, 1, false);
    } else if (wpe == 1) {
      // one row per 512-register wave: fragments held in registers (ORYX_ALS_GL_HOLD=0: re-read)
      if (gl_hold()) {
        if (split) GL128(true, 1, 1, true); else GL128(false, 1, 1, true);
      } else {
        if (split) GL128(true, 1, 1, false); else GL128(false, 1, 1, false);
      }
    } else {
      if (split) GL128(true, 1, 2, false); else GL128(false, 1, 2, false);
    }
#undef GL128
    return oryx_check_launch();
  }
  switch (kp) {
#define GL_CASE(KPV)                                                                          \
  case KPV:                                                                                   \
    if (split)                                                                                \
      hipLaunchKernelGGL((als_solve_batch_gl<KPV, true>), dim3(blocks), dim3(256), 0, s, p,   \
                         nullptr);                                                           \
    else                                                                                      \
      hipLaunchKernelGGL((als_solve_batch_gl<KPV, false>), dim3(blocks), dim3(256), 0, s, p,  \
                         nullptr);                                                           \
    break;
    GL_CASE(16)
    GL_CASE(32)
    GL_CASE(48)
    GL_CASE(64)
    GL_CASE(80)
    GL_CASE(96)
    GL_CASE(112)
#undef GL_CASE
    default:
      return ORYX_EINVAL;
  }
  return oryx_check_launch();
}

}  // namespace oryx_als
