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

template <int KP, int NM, int D>
struct BatchCfg {
  static constexpr int M = KP / 16;
  static constexpr int NT = M * (M + 1) / 2;
  static constexpr int IMG = ChunkImage<KP>::BYTES;
  static constexpr int DS = 20;   // scratch row stride in floats (ds_read_b128 rows conflict free)
  static constexpr int SCR = NM * 16 * DS * 4;
  static constexpr int VEC = NM * 16 * 4;
  static constexpr int WAVE_BYTES = NM * IMG + NM * 256 + SCR + VEC;
  static constexpr int YTY_BYTES = NT * 64 * 16;
  static constexpr int BYTES = YTY_BYTES + 4 * WAVE_BYTES;
};

// D: chunks in flight per row (register ring depth); the wave keeps NM * D gathers in flight.
// PROF: per-phase shader-clock cycles summed into prof[0..7] (analysis build,
// scripts/als_phase_profile.py)
// NM = 4: one wave per SIMD (512 registers), lane group g owns row g.  NM = 2: two waves per
// SIMD (256 registers each), lane groups g and g + 2 both hold row g & 1 (the group-layout
// work is duplicated, but the SIMD interleaves the two waves' VALU streams -- one wave alone
// issues a VALU instruction every 4 cycles, two fill the SIMD-32's 2-cycle slots -- and one
// wave's gather overlaps the other's MFMA-heavy solve).
template <int KP, int NM, int D, bool PROF = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4 / NM, 4 / NM))) void
als_solve_batch(AlsParams p, unsigned long long* prof) {
  using C = BatchCfg<KP, NM, D>;
  using CI = ChunkImage<KP>;
  constexpr int M = C::M;
  constexpr int NT = C::NT;
  constexpr int NPL = CI::NPL;
  constexpr int PPR = CI::PPR;
  constexpr int DS = C::DS;
  static_assert(NM == 4 || NM == 2, "lane group g owns row g % NM of the batch");
  typedef __attribute__((address_space(3))) float lds_float;
  typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
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
  {
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
      const int ww = valid_n[m] ? w : p.n_work - 1;   // tail: a real row, solved, not stored
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
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[m][t] = ytya[t * 64 + lane];
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
    // ------------------------------------------------------------ normal equations
    float cntw[NM];
    static_for<NM>([&](auto Mc) {
      constexpr int m = decltype(Mc)::value;
      cntw[m] = wave_sum(cnt[m]);
      reduce_bpart<M>(bpart[m]);   // lane (g, f): bpart[m][pi] = b_m[16 pi + f]
      if (slot[m] >= 0) {
        // split row: Gramian, b and count were summed by als_partial into ws[slot]
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
      if constexpr (pp == 0) stage2();
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
      if constexpr (pp == (M > 1 ? 1 : 0)) stage3();
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
    float xs[M];
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

}  // namespace

namespace oryx_als {

#ifndef ORYX_ALS_BATCH_DEPTH
#define ORYX_ALS_BATCH_DEPTH 1
#endif
// rows per wave: 2 (two waves per SIMD, default) or 4 (one wave per SIMD)
#ifndef ORYX_ALS_BATCH_NM
#define ORYX_ALS_BATCH_NM 2
#endif

static unsigned long long* g_batch_prof = nullptr;

void batch_set_profile(unsigned long long* prof) { g_batch_prof = prof; }

int batch_solve_launch(const AlsParams& p, int kp, int max_blocks, hipStream_t s) {
  constexpr int NM = ORYX_ALS_BATCH_NM;
  constexpr int D = ORYX_ALS_BATCH_DEPTH;
  // one resident generation: 4 / NM blocks of 4 waves per CU (max_blocks = CUs unless
  // overridden by ORYX_ALS_MAX_BLOCKS)
  const int nb = (p.n_work + NM - 1) / NM;
  int blocks = (nb + 3) / 4;
  const int cap = max_blocks * (4 / NM);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (g_batch_prof && kp == 64) {
    hipLaunchKernelGGL((als_solve_batch<64, NM, D, true>), dim3(blocks), dim3(256), 0, s, p,
                       g_batch_prof);
    return oryx_check_launch();
  }
  switch (kp) {
#define BATCH_CASE(KPV)                                                                       \
  case KPV:                                                                                   \
    hipLaunchKernelGGL((als_solve_batch<KPV, NM, D>), dim3(blocks), dim3(256), 0, s, p,      \
                       nullptr);                                                             \
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

}  // namespace oryx_als
