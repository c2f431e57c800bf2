// tuning/als_variants.hip -- superseded ALS solve kernels, kept OUT of the default build
// (python -m oryx_amd._build --tuning builds liboryx_kernels_tuning.so with them; point
// ORYX_KERNELS_SO at it and select with ORYX_ALS_VARIANT / ORYX_ALS_WIDE_VARIANT):
//   * als_solve_wave   (variant 1, and the fp32 mode at KP <= 64 with wide variant 0):
//     one wave per row, register column Cholesky with v_readlane broadcasts;
//   * als_solve_panel  (variants 0, 2, 3, 4): 16-column panel Cholesky, gathers 1 or 3
//     chunks deep, optional raised issue priority;
//   * als_solve_wide   (wide variant 0): one wave per row for 64 < KP <= 128;
//   * als_solve_block  (wide variant 1): one workgroup per row, LDS Cholesky (bf16 only);
//   * als_debug_gram   (analysis: one row's accumulated Gramian).
// The default path (als_batch.hip: als_solve_batch / als_solve_batch_gl) replaced them;
// rocprof comparisons are in profiles/ (r1_*, r2_*).

#include "../als_wave.h"

namespace {



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

}  // namespace

extern "C" {

// Non-default solve kernels (called by oryx_als_solve in als.hip when a tuning variant is
// selected).  Returns ORYX_EINVAL for a combination this build does not have.
int oryx_als_solve_variant(const oryx_als::AlsParams& p, int kp, int split, int variant,
                           int wide, int max_blocks, int panel_blocks, hipStream_t s) {
  switch (kp) {
#define WAVE_CASE(KPV)                                                                \
  case KPV: {                                                                         \
    int blocks = (p.n_work + 3) / 4;                                                  \
    if (blocks > (split ? max_blocks : panel_blocks))                                 \
      blocks = split ? max_blocks : panel_blocks;                                     \
    if (split)                                                                        \
      hipLaunchKernelGGL((als_solve_wave<KPV, false, true>), dim3(blocks), dim3(256), 0, \
                         s, p, nullptr);                                              \
    else if (variant == 0)                                                            \
      hipLaunchKernelGGL((als_solve_panel<KPV, false>), dim3(blocks), dim3(256), 0, s, p, \
                         nullptr);                                                    \
    else if (variant == 2)                                                            \
      hipLaunchKernelGGL((als_solve_panel<KPV, false, true>), dim3(blocks), dim3(256), 0, \
                         s, p, nullptr);                                              \
    else if (variant == 3)                                                            \
      hipLaunchKernelGGL((als_solve_panel<KPV, false, true, 2>), dim3(blocks), dim3(256), \
                         0, s, p, nullptr);                                           \
    else if (variant == 4)                                                            \
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
    if (split || wide == 0) {                                                         \
      int blocks = (p.n_work + 3) / 4;                                                \
      if (blocks > max_blocks) blocks = max_blocks;                                   \
      if (split)                                                                      \
        hipLaunchKernelGGL((als_solve_wide<KPV, true>), dim3(blocks), dim3(256), 0, s, p); \
      else                                                                            \
        hipLaunchKernelGGL((als_solve_wide<KPV, false>), dim3(blocks), dim3(256), 0, s, p); \
    } else {                                                                          \
      int blocks = p.n_work < max_blocks ? p.n_work : max_blocks;                     \
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

// analysis: KP = 64 solve with per-phase cycle counters (prof: 6 u64, zeroed by caller)
int oryx_als_solve_profile64(const int64_t* row_ptr, const int32_t* row_ids,
                             const int32_t* col_idx, const float* vals, const void* Y,
                             const float* YtY, float* X, int n_work, int k, float lambda,
                             float alpha, int implicit, int variant, unsigned long long* prof,
                             void* stream) {
  if (n_work <= 0) return ORYX_OK;
  oryx_als::AlsParams p{row_ptr, row_ids, col_idx, vals, reinterpret_cast<const __bf16*>(Y),
                        YtY, X, nullptr, n_work, k, lambda, alpha, implicit, nullptr, nullptr,
                        nullptr};
  int blocks = (n_work + 3) / 4;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (variant == 0)
    hipLaunchKernelGGL((als_solve_panel<64, true>), dim3(blocks), dim3(256), 0, s, p, prof);
  else if (variant == 2)
    hipLaunchKernelGGL((als_solve_panel<64, true, true>), dim3(blocks), dim3(256), 0, s, p,
                       prof);
  else if (variant == 3)
    hipLaunchKernelGGL((als_solve_panel<64, true, true, 2>), dim3(blocks), dim3(256), 0, s, p,
                       prof);
  else if (variant == 4)
    hipLaunchKernelGGL((als_solve_panel<64, true, true, 3>), dim3(blocks), dim3(256), 0, s, p,
                       prof);
  else
    hipLaunchKernelGGL((als_solve_wave<64, true>), dim3(blocks), dim3(256), 0, s, p, prof);
  return oryx_check_launch();
}

int oryx_als_debug_gram(const int64_t* row_ptr, const int32_t* col_idx, const float* vals,
                        const void* Y, int kp, float alpha, int implicit, long long beg,
                        long long end, float* out, int split, void* stream) {
  oryx_als::AlsParams p{row_ptr, nullptr, col_idx, vals, reinterpret_cast<const __bf16*>(Y),
                        nullptr, nullptr, nullptr, 1, kp, 0.f, alpha, implicit, nullptr,
                        nullptr, nullptr};
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

}  // extern "C"
