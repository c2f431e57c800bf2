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
// kmeans_accumulate: per point, adds its fp32 row into sums[assign] plus counts and distance
// statistics (count, sum d, sum d^2 for the DB / Dunn / SSE metrics): LDS-privatised column
// slices when K x (slice) fits (kmeans_accumulate_lds_kernel), else one wave per row of L2
// atomics (every atomic instruction covers 256 contiguous bytes).

#include "common.h"

#include <cstdlib>

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
  // per-lane best for rows (rt, g*4 + v).  argmin_c |x|^2 + |c|^2 - 2 x.c = argmax_c
  // (x.c - |c|^2 / 2): the accumulator starts at -|c|^2 / 2 (the lane's center), so the
  // epilogue is one compare and two selects per value; |x|^2 only enters the final distance.
  float best[ROW_TILES][4];
  int besti[ROW_TILES][4];
#pragma unroll
  for (int rt = 0; rt < ROW_TILES; ++rt)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      best[rt][v] = -INFINITY;
      besti[rt][v] = 0;
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
    // B fragments double-buffered in registers: the reads for center group ct+1 are in flight
    // while group ct's MFMAs run (reading right before use exposed the LDS latency on every
    // pair of MFMAs)
    bf16x8 bfr[2][DK];
    auto read_b = [&](int ct, bf16x8* dst) {
#pragma unroll
      for (int s = 0; s < DK; ++s)
        dst[s] = *reinterpret_cast<const bf16x8*>(base + (ct * 16 + fl) * ROWB +
                                                  (s * 32 + 8 * g) * 2);
    };
    read_b(0, bfr[0]);
#pragma unroll
    for (int ct = 0; ct < BN / 16; ++ct) {
      if (ct + 1 < BN / 16) read_b(ct + 1, bfr[(ct + 1) & 1]);
      const int c = t * BN + ct * 16 + fl;
      const float h = -0.5f * cnorm[c];       // +inf padding rows -> -inf, never chosen
      f32x4 acc[ROW_TILES];
#pragma unroll
      for (int rt = 0; rt < ROW_TILES; ++rt) acc[rt] = f32x4{h, h, h, h};
#pragma unroll
      for (int s = 0; s < DK; ++s) {
#pragma unroll
        for (int rt = 0; rt < ROW_TILES; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][s], bfr[ct & 1][s], acc[rt],
                                                            0, 0, 0);
      }
      // C/D layout: col = fl (center), row = g*4 + v (point)
#pragma unroll
      for (int rt = 0; rt < ROW_TILES; ++rt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          if (acc[rt][v] > best[rt][v]) {
            best[rt][v] = acc[rt][v];
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
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      const long long r = row0 + rt * 16 + g * 4 + v;
      if (fl == 0 && r < n) {
        const float d = xnorm[r] - 2.f * bv;
        assign[r] = bi;
        mind[r] = d > 0.f ? d : 0.f;
      }
    }
}

// kmeans_assign_wide: the same argmin with the roles of the MFMA operands swapped, so that
// each wave covers 64 points with one (best, argbest) pair per lane and point tile:
//   * points are the B operand (column = lane & 15) of v_mfma_f32_16x16x32_bf16, held in
//     registers for the whole kernel (4 tiles x DK k-steps); centers are the A operand
//     (row = 4 (lane >> 4) + v), so each lane scans 4 centers of one point per 16x16 tile;
//   * 64 points per wave halves the LDS operand reads per MFMA against 32-point waves, and the
//     per-point state is 8 registers instead of 32, which keeps two waves per SIMD;
//   * center tiles (64 rows) are copied global -> LDS by global_load_lds_dwordx4 (no staging
//     registers), double-buffered; the LDS image is written linearly and the 16-byte units of
//     each row are XOR-swizzled through the per-lane SOURCE address so that each lane group
//     of the fragment ds_read_b128 is bank-conflict free (see swz below);
//   * |c|^2 of the tile rides along in LDS (a 4-byte glds by wave 0), the accumulator starts
//     at -|c|^2 / 2 and the argmax of x.c - |c|^2 / 2 is the nearest center.
template <int RU>
__host__ __device__ constexpr int km_swz(int r) {
  return RU >= 16 ? (r & 15) : ((r >> 1) & 7);
}

__device__ __forceinline__ float km_pack(float x, unsigned v) {
  return __uint_as_float((__float_as_uint(x) & ~3u) | v);
}

__device__ __forceinline__ float km_max3(float a, float b, float c) {
  float m;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(a), "v"(b), "v"(c));
  return m;
}

// Packed epilogue of one 16-center group and point tile: each value gets its row-in-group v (0..3) in the
// two low mantissa bits (a 2^-21 relative perturbation), so the running best is two v_max3
// per 4 values and only the group index needs a compare + select.
__device__ __forceinline__ void km_epilogue_one(const f32x4& ac, int ctg, float& bestp,
                                                int& bestct) {
  float m = km_max3(bestp, km_pack(ac[0], 0), km_pack(ac[1], 1));
  m = km_max3(m, km_pack(ac[2], 2), km_pack(ac[3], 3));
  bestct = __float_as_uint(m) != __float_as_uint(bestp) ? ctg : bestct;
  bestp = m;
}

// Certified assignment (fp32 parity; see kmeans_assign_wide_kernel<..., TOP3 = true>): the
// full center index rides in the low `bits` mantissa bits of each packed value and every lane
// keeps its three best packed values in order; inserting p into (b1 >= b2 >= b3) is three
// ops: b3 = med3(b2, b3, p), b2 = med3(b1, b2, p), b1 = max(b1, p).
struct CertParams {
  int* idx2;               // [n] second-best center
  unsigned char* flags;    // [n] 0 = top-1 certified, 1 = rescore top-2, 2 = full rescan
  unsigned mask;           // (1 << bits) - 1
  float u;                 // bf16 rounding bound (relative, per operand)
  float eta_scale;         // packing + accumulation slack, times (|x| + cmax)^2
  float cmax;              // max |c| over the real centers
};

__device__ __forceinline__ float km_packi(float x, unsigned idx, unsigned mask) {
  return __uint_as_float((__float_as_uint(x) & ~mask) | idx);
}

// v_max_f32 without the operand canonicalisation fmaxf gets (the packed values are finite
// numbers, never signalling NaNs): one instruction instead of three
__device__ __forceinline__ float km_max2(float a, float b) {
  float m;
  asm("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(a), "v"(b));
  return m;
}

__device__ __forceinline__ void km_insert3(float p, float& b1, float& b2, float& b3) {
  b3 = __builtin_amdgcn_fmed3f(b2, b3, p);
  b2 = __builtin_amdgcn_fmed3f(b1, b2, p);
  b1 = km_max2(b1, p);
}

// Most groups hold nothing above the lane's third best once the scan is under way: a group
// max (two ops) and a wave vote skip the three-op insertions unless some lane needs them.
__device__ __forceinline__ void km_epilogue_top3(const f32x4& ac, int ctg, int g, unsigned mask,
                                                 float& b1, float& b2, float& b3) {
  const unsigned base = (unsigned)(ctg * 16 + 4 * g);
  float p[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) p[v] = km_packi(ac[v], base + v, mask);
  const float m = km_max3(km_max3(p[0], p[1], p[2]), p[3], p[3]);
  if (__builtin_expect(__any(m > b3), 0)) {
#pragma unroll
    for (int v = 0; v < 4; ++v) km_insert3(p[v], b1, b2, b3);
  }
}

// Requires d_pad = 32 DK with 2 <= DK <= 8 (each LDS row has at least 8 units).
// PK selects the packed, software-pipelined epilogue (the group-ct epilogue runs while the
// MFMAs of group ct+1 are in flight, on a second accumulator set; the A fragments are
// refilled in place, one k-step at a time).
template <int DK, int NW, bool PK, bool TOP3 = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void
kmeans_assign_wide_kernel(const __bf16* __restrict__ X, const float* __restrict__ xnorm,
                          const __bf16* __restrict__ C, const float* __restrict__ cnorm,
                          long long n, int k_pad, int* __restrict__ assign,
                          float* __restrict__ mind, CertParams cert) {
  constexpr int DPAD = DK * 32;
  constexpr int RU = DPAD / 8;             // 16-byte units per center row
  constexpr int CT = 64;                   // centers per LDS stage
  constexpr int STAGE = CT * DPAD * 2;     // bytes of one center tile
  constexpr int BUF = STAGE + CT * 4;      // + |c|^2 of the tile
  constexpr int PT = 4;                    // 16-point tiles per wave
  constexpr int GPW = RU / NW;             // 1 KB glds chunks per wave per stage
  static_assert(GPW * NW == RU && RU % 8 == 0 && RU <= 32, "glds chunking");
  typedef __attribute__((address_space(3))) void lds_void;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, fl = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const long long p0 = (long long)bid * (NW * PT * 16) + wave * PT * 16;
  const int ntiles = k_pad / CT;

  // LDS image of a tile: linear, row r's 16-byte unit q stored at unit q ^ swz(r).  The
  // ds_read_b128 lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32) read
  // rows fl of unit 4 ks + g; with swz = row & 15 (rows of >= 16 units) or (row >> 1) & 7
  // (8-unit rows, two rows per 256 B) every group covers the 16 bank quads of a 256-byte LDS
  // cycle exactly once.  glds writes lane-linearly, so the permutation goes on the source:
  // chunk (i * NW + wave) = units u = chunk * 64 + lane, row u / RU, source unit
  // (u % RU) ^ swz(row).
  const int u0 = wave * 64 + lane;
  const int srow = u0 / RU, sus = u0 % RU;
  constexpr int RSTEP = NW * 64 / RU;      // rows between a wave's consecutive chunks
  auto issue_tile = [&](int t, int buf) {
    char* dst = smem + buf * BUF;
    const __bf16* src = C + (long long)t * CT * DPAD;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      // swz(r) spelled out: a call out of this lambda drops the kernel's host stub (hipcc 7.2)
      const int r = srow + i * RSTEP;
      __builtin_amdgcn_global_load_lds(src + r * DPAD + (sus ^ (RU >= 16 ? (r & 15) : ((r >> 1) & 7))) * 8,
                                       (lds_void*)(dst + (i * NW + wave) * 1024), 16, 0, 0);
    }
    if (wave == 0)
      __builtin_amdgcn_global_load_lds(cnorm + (long long)t * CT + lane,
                                       (lds_void*)(dst + STAGE), 4, 0, 0);
  };
  issue_tile(0, 0);

  // points: B fragment (k = ks*32 + 8g + j, column = point fl of tile pt); rows past n are
  // clamped to row n-1 (their results are never stored)
  bf16x8 b[PT][DK];
  const __bf16* xrow[PT];
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    const long long r = p0 + pt * 16 + fl;
    xrow[pt] = X + (r < n ? r : n - 1) * DPAD + 8 * g;
  }
#pragma unroll
  for (int s = 0; s < DK; ++s)
#pragma unroll
    for (int pt = 0; pt < PT; ++pt)
      b[pt][s] = *reinterpret_cast<const bf16x8*>(xrow[pt] + s * 32);
  float best[PT];
  int besti[PT];
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    best[pt] = -INFINITY;
    besti[pt] = 0;
  }
  // A fragment of center group ct, k-step ks: row ct*16 + fl (swz(row) = swz(fl)), unit
  // 4 ks + g.  The swizzle only touches the low 4 unit bits, so ks >> 2 is an immediate
  // offset and ks & 3 selects one of (at most) 4 lane bases.
  int aoff[DK < 4 ? DK : 4];
#pragma unroll
  for (int m = 0; m < (DK < 4 ? DK : 4); ++m)
    aoff[m] = fl * RU * 16 + 16 * ((4 * m + g) ^ km_swz<RU>(fl));

  __syncthreads();
  if constexpr (PK) {
    float bestp[PT];
    int bestct[PT];
    float t2[TOP3 ? PT : 1], t3[TOP3 ? PT : 1];
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) {
      bestp[pt] = -3.0e38f;
      bestct[pt] = 0;
      if constexpr (TOP3) {
        t2[pt] = -3.0e38f;
        t3[pt] = -3.0e38f;
      }
    }
    auto epi = [&](const f32x4& ac, int ctg, int pt) {
      if constexpr (TOP3)
        km_epilogue_top3(ac, ctg, g, cert.mask, bestp[pt], t2[pt], t3[pt]);
      else
        km_epilogue_one(ac, ctg, bestp[pt], bestct[pt]);
    };
    f32x4 acc[2][PT];
    bf16x8 a[DK];
    for (int t = 0; t < ntiles; ++t) {
      const int buf = t & 1;
      if (t + 1 < ntiles) issue_tile(t + 1, buf ^ 1);
      const char* base = smem + buf * BUF;
      const float* cn = reinterpret_cast<const float*>(base + STAGE);
      auto a_addr = [&](int ct, int s) {
        return reinterpret_cast<const bf16x8*>(base + aoff[s & 3] + ct * 16 * RU * 16 +
                                               256 * (s >> 2));
      };
#pragma unroll
      for (int s = 0; s < DK; ++s) a[s] = *a_addr(0, s);
      // |c|^2 of group ct + 1 is read during group ct (an LDS read right before the first
      // MFMA of each group would expose its latency once per group)
      f32x4 c4n = *reinterpret_cast<const f32x4*>(cn + 4 * g);
#pragma unroll
      for (int ct = 0; ct < CT / 16; ++ct) {
        const f32x4 c4 = c4n;
        if (ct + 1 < CT / 16) c4n = *reinterpret_cast<const f32x4*>(cn + (ct + 1) * 16 + 4 * g);
        // padding rows (|c|^2 = +inf) start at -5e29: finite, so the packed bits stay a number
        f32x4 h;
#pragma unroll
        for (int v = 0; v < 4; ++v) h[v] = -0.5f * fminf(c4[v], 1.0e30f);
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) acc[ct & 1][pt] = h;
        // the previous group's epilogue (other accumulator set) is spread over the k-steps,
        // point tile pt at step pt % DK, and a scheduling barrier closes each step so the
        // refill reads and the epilogue stay where they are put
        const bool prev = ct > 0 || t > 0;
        const int pset = (ct + 1) & 1;
        const int pctg = t * (CT / 16) + ct - 1;
#pragma unroll
        for (int s = 0; s < DK; ++s) {
#pragma unroll
          for (int pt = 0; pt < PT; ++pt)
            acc[ct & 1][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], b[pt][s],
                                                                      acc[ct & 1][pt], 0, 0, 0);
          if (ct + 1 < CT / 16) a[s] = *a_addr(ct + 1, s);
          if (prev) {
#pragma unroll
            for (int pt = 0; pt < PT; ++pt)
              if (pt % DK == s) epi(acc[pset][pt], pctg, pt);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (t + 1 < ntiles) __syncthreads();
    }
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) epi(acc[1][pt], ntiles * (CT / 16) - 1, pt);
    if constexpr (TOP3) {
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) {
        float b1 = bestp[pt], b2 = t2[pt], b3 = t3[pt];
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) {
          const float o1 = __shfl_xor(b1, off, 64);
          const float o2 = __shfl_xor(b2, off, 64);
          const float o3 = __shfl_xor(b3, off, 64);
          km_insert3(o1, b1, b2, b3);
          km_insert3(o2, b1, b2, b3);
          km_insert3(o3, b1, b2, b3);
        }
        const long long r = p0 + pt * 16 + fl;
        if (g == 0 && r < n) {
          const float xn = xnorm[r];
          const float d1 = xn - 2.f * b1, d2 = xn - 2.f * b2, d3 = xn - 2.f * b3;
          // true distances lie in [lower(d~), upper(d~)] (bf16 operand rounding delta,
          // packing / accumulation slack eta); both bounds are monotone in d~
          const float xr = sqrtf(fmaxf(xn, 0.f)) + cert.cmax;
          const float delta = cert.u * xr, eta = cert.eta_scale * xr * xr;
          auto lower = [&](float t) {
            const float q = fmaxf(sqrtf(fmaxf(t, 0.f)) - delta, 0.f);
            return q * q - eta;
          };
          const float up1 = sqrtf(fmaxf(d1, 0.f)) + delta;
          const float upper1 = up1 * up1 + eta;
          assign[r] = (int)(__float_as_uint(b1) & cert.mask);
          cert.idx2[r] = (int)(__float_as_uint(b2) & cert.mask);
          cert.flags[r] = lower(d2) > upper1 ? 0 : (lower(d3) > upper1 ? 1 : 2);
          mind[r] = d1 > 0.f ? d1 : 0.f;
        }
      }
      return;
    }
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) {
      float bv = bestp[pt];
      int bi = bestct[pt] * 16 + 4 * g + (int)(__float_as_uint(bv) & 3u);
#pragma unroll
      for (int off = 16; off < 64; off <<= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      const long long r = p0 + pt * 16 + fl;
      if (g == 0 && r < n) {
        const float d = xnorm[r] - 2.f * bv;
        assign[r] = bi;
        mind[r] = d > 0.f ? d : 0.f;
      }
    }
    return;
  }
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) issue_tile(t + 1, buf ^ 1);
    const char* base = smem + buf * BUF;
    const float* cn = reinterpret_cast<const float*>(base + STAGE);
    bf16x8 a[2][DK];
    auto read_a = [&](int ct, bf16x8* dst) {
#pragma unroll
      for (int s = 0; s < DK; ++s)
        dst[s] = *reinterpret_cast<const bf16x8*>(base + aoff[s & 3] + ct * 16 * RU * 16 +
                                                  256 * (s >> 2));
    };
    read_a(0, a[0]);
#pragma unroll
    for (int ct = 0; ct < CT / 16; ++ct) {
      if (ct + 1 < CT / 16) read_a(ct + 1, a[(ct + 1) & 1]);
      const f32x4 c4 = *reinterpret_cast<const f32x4*>(cn + ct * 16 + 4 * g);
      const f32x4 h = c4 * -0.5f;            // +inf padding rows -> -inf, never chosen
      f32x4 acc[PT];
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) acc[pt] = h;
#pragma unroll
      for (int s = 0; s < DK; ++s)
#pragma unroll
        for (int pt = 0; pt < PT; ++pt)
          acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct & 1][s], b[pt][s], acc[pt], 0, 0,
                                                            0);
      const int c0 = t * CT + ct * 16 + 4 * g;
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int pt = 0; pt < PT; ++pt)
          if (acc[pt][v] > best[pt]) {
            best[pt] = acc[pt][v];
            besti[pt] = c0 + v;
          }
    }
    if (t + 1 < ntiles) __syncthreads();  // tile t+1 landed (each wave drained its glds) and
                                          // every wave is done reading tile t's buffer
  }
  // reduce over the 4 lane groups holding the same point; ties -> lowest center index
#pragma unroll
  for (int pt = 0; pt < PT; ++pt) {
    float bv = best[pt];
    int bi = besti[pt];
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) {
      const float ov = __shfl_xor(bv, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    const long long r = p0 + pt * 16 + fl;
    if (g == 0 && r < n) {
      const float d = xnorm[r] - 2.f * bv;
      assign[r] = bi;
      mind[r] = d > 0.f ? d : 0.f;
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

// LDS-privatised accumulation: block (x, y) owns rows [x*rpb, ...) and the column slice
// [y*CW, y*CW + CW) of every center.  Its K x CW partial sums (row stride CW+1 when it fits,
// so that two rows of one wave hitting different clusters fall on different banks), plus the
// K counts and distance statistics for the y == 0 column, live in LDS; ds_add_f32 replaces the
// per-(row, column) L2 atomic of kmeans_accumulate_kernel -- with 1000 clusters and millions
// of rows the L2 atomics serialise on hot lines -- and each block flushes K x CW values once.
// 1024 threads per block: the LDS image allows one block per CU, so the block itself carries
// the 16 waves of memory-level parallelism the row stream needs.
template <bool VEC>
__global__ __launch_bounds__(1024) void kmeans_accumulate_lds_kernel(
    const float* __restrict__ X, const int* __restrict__ assign, const float* __restrict__ mind,
    long long n, int d, int ld, int k, int cw, int stride, long long rpb,
    float* __restrict__ sums, unsigned long long* __restrict__ counts,
    double* __restrict__ dstats) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  double* lstat = reinterpret_cast<double*>(smem_raw);                  // [k][2]
  unsigned int* lcnt = reinterpret_cast<unsigned int*>(lstat + 2 * k);  // [k]
  float* lsum = reinterpret_cast<float*>(lcnt + k);                     // [k][stride]
  const int tid = threadIdx.x;
  const int c0 = blockIdx.y * cw;
  const int cwe = min(cw, d - c0);                 // columns of this slice that exist
  const bool lead = blockIdx.y == 0;
  for (int i = tid; i < k * stride; i += 1024) lsum[i] = 0.f;
  if (lead) {
    for (int i = tid; i < k; i += 1024) lcnt[i] = 0u;
    if (dstats)
      for (int i = tid; i < 2 * k; i += 1024) lstat[i] = 0.0;
  }
  __syncthreads();
  // VEC: a thread owns 4 consecutive columns (one 16-byte load per row); else 1 column
  constexpr int W = VEC ? 4 : 1;
  const int lanes = (cw + W - 1) / W;
  const int tpr = lanes < 64 ? lanes : 64;         // threads per row
  const int rpp = 1024 / tpr;                      // rows per pass
  const int sub = tid / tpr, col = (tid % tpr) * W;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < n ? r0 + rpb : n;
  // U rows per thread per step: all U assignment loads, then all U row loads, are in flight
  // together (a row costs two dependent HBM round trips; one row per step left the loop
  // latency-bound at 16 waves per CU)
  constexpr int U = 8;
  for (long long base = r0 + sub; base < r1; base += (long long)U * rpp) {
    int c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = base + (long long)u * rpp;
      c[u] = r < r1 ? assign[r] : -1;
    }
    for (int j = col; j < cwe; j += tpr * W) {
      if (VEC) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = base + (long long)u * rpp;
          if (c[u] >= 0) v[u] = *reinterpret_cast<const f32x4*>(X + r * ld + c0 + j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (c[u] >= 0) {
            float* sr = lsum + c[u] * stride + j;
            atomicAdd(sr, v[u][0]);
            atomicAdd(sr + 1, v[u][1]);
            atomicAdd(sr + 2, v[u][2]);
            atomicAdd(sr + 3, v[u][3]);
          }
        }
      } else {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = base + (long long)u * rpp;
          if (c[u] >= 0) v[u] = X[r * ld + c0 + j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (c[u] >= 0) atomicAdd(lsum + c[u] * stride + j, v[u]);
      }
    }
    if (lead && col == 0) {
      float md[U];
      if (dstats) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = base + (long long)u * rpp;
          md[u] = c[u] >= 0 ? mind[r] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (c[u] < 0) continue;
        atomicAdd(lcnt + c[u], 1u);
        if (dstats) {
          const double dist = sqrt((double)md[u]);
          atomicAdd(lstat + 2 * c[u], dist);
          atomicAdd(lstat + 2 * c[u] + 1, dist * dist);
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < k * cwe; i += 1024) {
    const int cc = i / cwe, j = i - cc * cwe;
    const float v = lsum[cc * stride + j];
    if (v != 0.f) atomicAdd(sums + (long long)cc * d + c0 + j, v);
  }
  if (lead) {
    for (int i = tid; i < k; i += 1024) {
      const unsigned int v = lcnt[i];
      if (v) atomicAdd(counts + i, (unsigned long long)v);
    }
    if (dstats)
      for (int i = tid; i < 2 * k; i += 1024) {
        const double v = lstat[i];
        if (v != 0.0) atomicAdd(dstats + i, v);
      }
  }
}

// ---- sort-based accumulation (counting sort by cluster + segmented row sums) ----
// LDS float atomics run at a fraction of a lane per cycle, so with K = 1000 and d = 256 the
// 3.2G (row, column) adds of one Lloyd step dominate.  Instead: (1) per-block cluster
// histograms, (2) per-cluster prefix offsets over blocks, (3) scatter of row ids into cluster
// order (integer LDS cursors, one per row), (4) one workgroup per (cluster, piece of
// PIECE rows) summing its rows -- a 1 KB coalesced row read per step, fp32 register
// accumulation, one global atomic per column per piece.  X is read once, in row order per
// cluster; counts come out of the scan exactly (no atomics).
constexpr int SORT_BLOCKS = 512;
constexpr int PIECE = 2048;
constexpr int SORT_U = 8;

__global__ __launch_bounds__(256) void km_block_hist(const int* __restrict__ assign, long long n,
                                                     int k, long long rpb,
                                                     unsigned int* __restrict__ bh) {
  extern __shared__ unsigned int h[];
  for (int i = threadIdx.x; i < k; i += 256) h[i] = 0u;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < n ? r0 + rpb : n;
  // SORT_U coalesced key loads issued before their LDS atomics, so a wave keeps SORT_U loads in
  // flight instead of one HBM round trip per key
  for (long long rb = r0 + threadIdx.x; rb < r1; rb += 256ll * SORT_U) {
    int c[SORT_U];
#pragma unroll
    for (int u = 0; u < SORT_U; ++u) {
      const long long r = rb + 256ll * u;
      c[u] = r < r1 ? assign[r] : -1;
    }
#pragma unroll
    for (int u = 0; u < SORT_U; ++u)
      if (c[u] >= 0) atomicAdd(h + c[u], 1u);
  }
  __syncthreads();
  unsigned int* out = bh + (long long)blockIdx.x * k;
  for (int i = threadIdx.x; i < k; i += 256) out[i] = h[i];
}

// per cluster: running sum over blocks (bh becomes the block's start within the cluster);
// 16 block rows are loaded per step so the loop is not one HBM round trip per block
__global__ __launch_bounds__(256) void km_cluster_scan(unsigned int* __restrict__ bh, int nb,
                                                       int k,
                                                       unsigned long long* __restrict__ counts) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= k) return;
  unsigned int run = 0;
  constexpr int V = 16;
  for (int b0 = 0; b0 < nb; b0 += V) {
    unsigned int v[V];
#pragma unroll
    for (int u = 0; u < V; ++u) v[u] = b0 + u < nb ? bh[(long long)(b0 + u) * k + c] : 0u;
#pragma unroll
    for (int u = 0; u < V; ++u) {
      if (b0 + u < nb) bh[(long long)(b0 + u) * k + c] = run;
      run += v[u];
    }
  }
  counts[c] = run;
}

// one block: exclusive scan of counts -> off[c]; pieces_prefix[c] = pieces before cluster c
__global__ __launch_bounds__(1024) void km_offsets(const unsigned long long* __restrict__ counts,
                                                   int k, long long* __restrict__ off,
                                                   int* __restrict__ pieces) {
  __shared__ long long s_off[1024];
  __shared__ int s_pc[1024];
  __shared__ long long carry_off;
  __shared__ int carry_pc;
  if (threadIdx.x == 0) {
    carry_off = 0;
    carry_pc = 0;
  }
  __syncthreads();
  for (int base = 0; base < k; base += 1024) {
    const int c = base + threadIdx.x;
    const long long cnt = c < k ? (long long)counts[c] : 0;
    s_off[threadIdx.x] = cnt;
    s_pc[threadIdx.x] = (int)((cnt + PIECE - 1) / PIECE);
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {      // Hillis-Steele inclusive scan
      long long a = 0;
      int b = 0;
      if (threadIdx.x >= d) {
        a = s_off[threadIdx.x - d];
        b = s_pc[threadIdx.x - d];
      }
      __syncthreads();
      s_off[threadIdx.x] += a;
      s_pc[threadIdx.x] += b;
      __syncthreads();
    }
    if (c < k) {
      off[c] = carry_off + s_off[threadIdx.x] - cnt;
      pieces[c] = carry_pc + s_pc[threadIdx.x] - (int)((cnt + PIECE - 1) / PIECE);
    }
    __syncthreads();
    if (threadIdx.x == 1023) {
      carry_off += s_off[1023];
      carry_pc += s_pc[1023];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) pieces[k] = carry_pc;
}

__global__ __launch_bounds__(256) void km_scatter(const int* __restrict__ assign, long long n,
                                                  int k, long long rpb,
                                                  const unsigned int* __restrict__ bh,
                                                  const long long* __restrict__ off,
                                                  int* __restrict__ perm) {
  // cursors hold absolute output positions (off[c] + this block's start; n < 2^31), so the
  // store needs no dependent global load of off[c]
  extern __shared__ unsigned int cur[];
  const unsigned int* start = bh + (long long)blockIdx.x * k;
  for (int i = threadIdx.x; i < k; i += 256) cur[i] = (unsigned int)off[i] + start[i];
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < n ? r0 + rpb : n;
  for (long long rb = r0 + threadIdx.x; rb < r1; rb += 256ll * SORT_U) {
    int c[SORT_U];
#pragma unroll
    for (int u = 0; u < SORT_U; ++u) {
      const long long r = rb + 256ll * u;
      c[u] = r < r1 ? assign[r] : -1;
    }
#pragma unroll
    for (int u = 0; u < SORT_U; ++u)
      if (c[u] >= 0) perm[atomicAdd(cur + c[u], 1u)] = (int)(rb + 256ll * u);
  }
}

// block = one piece of one cluster; T threads per row (power of two >= d, <= 256), 256 / T
// rows in flight, U rows unrolled per thread so the row loads overlap
template <bool STATS>
__global__ __launch_bounds__(256) void km_segment_sum(
    const float* __restrict__ X, const float* __restrict__ mind, int d, int ld, int k,
    const int* __restrict__ perm, const unsigned long long* __restrict__ counts,
    const long long* __restrict__ off, const int* __restrict__ pieces, int tpr,
    float* __restrict__ sums, double* __restrict__ dstats) {
  __shared__ float red[256];
  __shared__ double dred[256];
  const int total = pieces[k];
  const int p = blockIdx.x;
  if (p >= total) return;
  // cluster of this piece: last c with pieces[c] <= p
  int lo = 0, hi = k - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pieces[mid] <= p) lo = mid; else hi = mid - 1;
  }
  const int c = lo;
  const long long cnt = (long long)counts[c];
  const long long i0 = (long long)(p - pieces[c]) * PIECE;
  const long long i1 = i0 + PIECE < cnt ? i0 + PIECE : cnt;
  const int* rows = perm + off[c];
  const int rpp = 256 / tpr;
  const int sub = threadIdx.x / tpr, col = threadIdx.x % tpr;
  constexpr int U = 8;
  for (int cb = 0; cb < d; cb += tpr) {
    const int j = cb + col;
    float acc = 0.f;
    double dacc = 0.0;
    for (long long i = i0 + sub; i < i1; i += (long long)U * rpp) {
      int r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long ii = i + (long long)u * rpp;
        r[u] = ii < i1 ? rows[ii] : -1;
      }
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = (r[u] >= 0 && j < d) ? X[(long long)r[u] * ld + j] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u];
      if (STATS && cb == 0 && col == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (r[u] >= 0) dacc += sqrt((double)mind[r[u]]);
      }
    }
    red[threadIdx.x] = acc;
    if (STATS && cb == 0) dred[threadIdx.x] = dacc;
    __syncthreads();
    if (sub == 0) {
      float s = 0.f;
      for (int q = 0; q < rpp; ++q) s += red[q * tpr + col];
      if (j < d && s != 0.f) atomicAdd(sums + (long long)c * d + j, s);
    }
    if (STATS && cb == 0 && threadIdx.x == 0) {
      double s = 0.0;
      for (int q = 0; q < rpp; ++q) s += dred[q * tpr];
      atomicAdd(dstats + 2 * c, s);
    }
    __syncthreads();
  }
  // sum of squared distances (= sum of mind) in a second light pass over the piece's rows
  if (STATS) {
    double s2 = 0.0;
    for (long long i = i0 + threadIdx.x; i < i1; i += 256) s2 += (double)mind[rows[i]];
    dred[threadIdx.x] = s2;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) dred[threadIdx.x] += dred[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(dstats + 2 * c + 1, dred[0]);
  }
}

// km_segment_sum with 16-byte loads (d % 4 == 0, rows 16-byte aligned): a row is read as
// float4s by tpr4 = (power of two >= d / 4) threads, 256 / tpr4 rows per pass and U rows in
// flight per thread -- a quarter of the load instructions of the scalar kernel, which at
// d = 256 read 256 bytes per wave instruction and fell short of the HBM rate.
template <bool STATS>
__global__ __launch_bounds__(256) void km_segment_sum4(
    const float* __restrict__ X, const float* __restrict__ mind, int d, int ld, int k,
    const int* __restrict__ perm, const unsigned long long* __restrict__ counts,
    const long long* __restrict__ off, const int* __restrict__ pieces, int tpr4,
    float* __restrict__ sums, double* __restrict__ dstats) {
  __shared__ f32x4 red4[256];
  __shared__ double dred[256];
  const int total = pieces[k];
  const int p = blockIdx.x;
  if (p >= total) return;
  int lo = 0, hi = k - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pieces[mid] <= p) lo = mid; else hi = mid - 1;
  }
  const int c = lo;
  const long long cnt = (long long)counts[c];
  const long long i0 = (long long)(p - pieces[c]) * PIECE;
  const long long i1 = i0 + PIECE < cnt ? i0 + PIECE : cnt;
  const int* rows = perm + off[c];
  const int rpp = 256 / tpr4;
  const int sub = threadIdx.x / tpr4, col = threadIdx.x % tpr4;
  const int d4 = d >> 2;
  constexpr int U = 8;
  for (int cb = 0; cb < d4; cb += tpr4) {
    const int j = cb + col;                         // float4 column
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    double dacc = 0.0;
    for (long long i = i0 + sub; i < i1; i += (long long)U * rpp) {
      int r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long ii = i + (long long)u * rpp;
        r[u] = ii < i1 ? rows[ii] : -1;
      }
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = (r[u] >= 0 && j < d4)
                   ? *reinterpret_cast<const f32x4*>(X + (long long)r[u] * ld + 4 * j)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u];
      if (STATS && cb == 0 && col == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (r[u] >= 0) dacc += sqrt((double)mind[r[u]]);
      }
    }
    red4[threadIdx.x] = acc;
    if (STATS && cb == 0) dred[threadIdx.x] = dacc;
    __syncthreads();
    if (sub == 0 && j < d4) {
      f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
      for (int q = 0; q < rpp; ++q) s4 += red4[q * tpr4 + col];
      float* dst = sums + (long long)c * d + 4 * j;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (s4[e] != 0.f) atomicAdd(dst + e, s4[e]);
    }
    if (STATS && cb == 0 && threadIdx.x == 0) {
      double s = 0.0;
      for (int q = 0; q < rpp; ++q) s += dred[q * tpr4];
      atomicAdd(dstats + 2 * c, s);
    }
    __syncthreads();
  }
  if (STATS) {
    double s2 = 0.0;
    for (long long i = i0 + threadIdx.x; i < i1; i += 256) s2 += (double)mind[rows[i]];
    dred[threadIdx.x] = s2;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) dred[threadIdx.x] += dred[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(dstats + 2 * c + 1, dred[0]);
  }
}

// Exact fp32 re-check of the points the certified assignment could not decide: one wave per
// 64 points.  flag 1 (two candidates): the point is handled by the whole wave, lanes over the
// dimensions (the row stays in registers, center rows are read coalesced), squared distances
// sum (x - c)^2 to the two bf16 candidates, ties to the lower center index.  flag 2 (the bf16
// ranking certifies no short list): the point is appended to list2 ([0] = count, then rows)
// for km_rescore_full.  stats[0] / stats[1] count flag-1 / flag-2 points (nullable).  d <= 512.
__global__ __launch_bounds__(256) void km_rescore(const float* __restrict__ X, int ldx, int d,
                                                  const float* __restrict__ C, int k, long long n,
                                                  int* __restrict__ assign,
                                                  const int* __restrict__ idx2,
                                                  const unsigned char* __restrict__ flags,
                                                  float* __restrict__ mind,
                                                  unsigned long long* __restrict__ stats,
                                                  int* __restrict__ list2) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  // float4 loads of rows and centers when every row starts on 16 bytes
  const bool vec = (d & 3) == 0 && (ldx & 3) == 0 &&
                   ((reinterpret_cast<unsigned long long>(X) |
                     reinterpret_cast<unsigned long long>(C)) & 15) == 0;
  // per-wave tallies, one atomic per wave at the end (a per-point atomic on one address
  // serialised ~10^6 updates in L2)
  unsigned long long n1 = 0, n2 = 0;
  for (long long w = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); w * 64 < n; w += nw) {
    const long long r0 = w * 64;
    const int f = r0 + lane < n ? flags[r0 + lane] : 0;
    // flag-2 points go to the list of km_rescore_full (one list atomic per wave)
    const unsigned long long m2 = __ballot(f == 2);
    if (m2) {
      int base = 0;
      if (lane == 0) base = atomicAdd(list2, (int)__popcll(m2));
      base = __shfl(base, 0, 64);
      if (f == 2) list2[1 + base + (int)__popcll(m2 & ((1ull << lane) - 1ull))] = (int)(r0 + lane);
      n2 += __popcll(m2);
    }
    // flag-1 points four at a time, one per 16-lane quarter of the wave (each lane sums a
    // quarter of the dimensions in 4-wide runs, then four xor-shuffles within the quarter):
    // a window's few flag-1 points no longer run one after another through the whole wave
    unsigned long long m = __ballot(f == 1);
    const int qr = lane >> 4, ql = lane & 15;
    while (m) {
      int js[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        js[t] = m ? __builtin_ctzll(m) : -1;
        if (m) m &= m - 1;
      }
      const int j = js[qr];
      float s1 = 0.f, s2 = 0.f;
      int i1 = 0, i2 = 0;
      const long long r = r0 + (j >= 0 ? j : 0);
      if (j >= 0) {
        i1 = assign[r];
        i2 = idx2[r];
        const float* xr = X + r * ldx;
        const float* c1 = C + (long long)i1 * d;
        const float* c2 = C + (long long)i2 * d;
        if (vec) {
          // same per-lane order as the scalar loop below, with the row and both center slices
          // of a 256-dimension chunk loaded as float4s before any arithmetic (12 loads in
          // flight instead of one round trip per 4-dimension run)
          for (int e0 = 4 * ql; e0 < d; e0 += 256) {
            f32x4 xv[4], av[4], bv[4];
#pragma unroll
            for (int it = 0; it < 4; ++it) {
              const int e = e0 + 64 * it;
              if (e < d) {
                xv[it] = *reinterpret_cast<const f32x4*>(xr + e);
                av[it] = *reinterpret_cast<const f32x4*>(c1 + e);
                bv[it] = *reinterpret_cast<const f32x4*>(c2 + e);
              }
            }
#pragma unroll
            for (int it = 0; it < 4; ++it) {
              if (e0 + 64 * it < d) {
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                  const float a = xv[it][v] - av[it][v], b = xv[it][v] - bv[it][v];
                  s1 += a * a;
                  s2 += b * b;
                }
              }
            }
          }
        } else {
          for (int e = 4 * ql; e < d; e += 64) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              if (e + v < d) {
                const float xv = xr[e + v];
                const float a = xv - c1[e + v], b = xv - c2[e + v];
                s1 += a * a;
                s2 += b * b;
              }
            }
          }
        }
      }
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) {
        s1 += __shfl_xor(s1, off, 64);
        s2 += __shfl_xor(s2, off, 64);
      }
      if (j >= 0 && ql == 0) {
        const bool first = s1 < s2 || (s1 == s2 && i1 < i2);
        assign[r] = first ? i1 : i2;
        mind[r] = first ? s1 : s2;
      }
      n1 += (js[0] >= 0) + (js[1] >= 0) + (js[2] >= 0) + (js[3] >= 0);
    }
  }
  if (stats && lane == 0) {
    if (n1) atomicAdd(stats, n1);
    if (n2) atomicAdd(stats + 1, n2);
  }
}

// Exact fp32 argmin over every center for the flag-2 points of km_rescore (list2: [0] =
// count, then rows).  A workgroup takes RP points at a time with their rows staged in LDS
// (read as broadcasts); each lane owns CPL centers (c0 + lane + 64 j: coalesced loads) and
// walks the dimensions in SL-wide slices held in registers, so one LDS read of 4 dimensions
// of a point feeds 4 CPL packed-fp32 ops -- register blocking over points x centers keeps the
// LDS data path (one 8-cycle broadcast per read) under the VALU rate, and consecutive FMAs go
// to independent accumulators.  Each (point, center) sum runs over the dimensions in
// increasing order in two halves (even / odd dimensions, the halves of the packed pairs)
// that are added at the end.  (min, lowest index) per point is reduced over lanes, then over
// the 4 waves through LDS.  Persistent grid: every workgroup walks tiles of the list until
// the device-side count is exhausted.
template <int RP, int CPL, int SL>
__global__ __launch_bounds__(256, 2) void km_rescore_full(const float* __restrict__ X, int ldx,
                                                       int d, const float* __restrict__ CT2,
                                                       int k, const int* __restrict__ list2,
                                                       int* __restrict__ assign,
                                                       float* __restrict__ mind) {
  extern __shared__ __attribute__((aligned(16))) float xs[];     // [RP][dq] + reduction
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // LDS rows padded to whole SL-dimension slices with zeros, as are the centers (CT2): the
  // padding adds (0 - 0)^2 = +0 to the sums, and the slice loop has no bounds test
  const int dq = (d + SL - 1) / SL * SL;
  float* red_d = xs + RP * dq;                                   // [4][RP]
  int* red_i = reinterpret_cast<int*>(red_d + 4 * RP);          // [4][RP]
  const int cnt = list2[0];
  const f32x2* ct2 = reinterpret_cast<const f32x2*>(CT2);
  for (int t0 = blockIdx.x * RP; t0 < cnt; t0 += gridDim.x * RP) {
    const int np = cnt - t0 < RP ? cnt - t0 : RP;
    __syncthreads();                                             // previous tile done
    for (int i = tid; i < RP * dq; i += 256) {
      const int p = i / dq, e = i - p * dq;
      xs[i] = (p < np && e < d) ? X[(long long)list2[1 + t0 + p] * ldx + e] : 0.f;
    }
    __syncthreads();
    float best[RP];
    int bidx[RP];
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      best[p] = INFINITY;
      bidx[p] = 0x7fffffff;
    }
    for (int c0 = wave * 64 * CPL; c0 < k; c0 += 256 * CPL) {
      // CT2 [k / 64][dq / 2][64] (64-center tiles of dimension pairs, zero padded): lane
      // `lane` of tile c0 / 64 + j reads its pairs 512 bytes apart
      const f32x2* cb[CPL];
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const int tile = c0 / 64 + j;
        cb[j] = ct2 + ((long long)(tile * 64 < k ? tile : 0) * (dq / 2)) * 64 + lane;
      }
      f32x2 acc[RP][CPL];
#pragma unroll
      for (int p = 0; p < RP; ++p)
#pragma unroll
        for (int j = 0; j < CPL; ++j) acc[p][j] = f32x2{0.f, 0.f};
      for (int e0 = 0; e0 < dq; e0 += SL) {
        f32x2 cv[CPL][SL / 2];
#pragma unroll
        for (int q = 0; q < SL / 2; ++q)
#pragma unroll
          for (int j = 0; j < CPL; ++j) cv[j][q] = cb[j][((e0 >> 1) + q) * 64];
#pragma unroll
        for (int q4 = 0; q4 < SL / 4; ++q4) {
#pragma unroll
          for (int p = 0; p < RP; ++p) {
            const f32x4 xv = *reinterpret_cast<const f32x4*>(xs + p * dq + e0 + 4 * q4);
            const f32x2 xa = f32x2{xv[0], xv[1]}, xb = f32x2{xv[2], xv[3]};
#pragma unroll
            for (int j = 0; j < CPL; ++j) {
              f32x2 t = xa - cv[j][2 * q4];
              acc[p][j] = __builtin_elementwise_fma(t, t, acc[p][j]);
              t = xb - cv[j][2 * q4 + 1];
              acc[p][j] = __builtin_elementwise_fma(t, t, acc[p][j]);
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const int c = c0 + 64 * j + lane;
        if (c < k) {
#pragma unroll
          for (int p = 0; p < RP; ++p) {
            const float v = acc[p][j][0] + acc[p][j][1];
            if (v < best[p]) {                       // a lane's centers grow with j: ties keep
              best[p] = v;                           // the lower index
              bidx[p] = c;
            }
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      float bd = best[p];
      int bi = bidx[p];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const float od = __shfl_xor(bd, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (od < bd || (od == bd && oi < bi)) {
          bd = od;
          bi = oi;
        }
      }
      if (lane == 0) {
        red_d[wave * RP + p] = bd;
        red_i[wave * RP + p] = bi;
      }
    }
    __syncthreads();
    if (tid < np) {
      float bd = red_d[tid];
      int bi = red_i[tid];
      for (int w = 1; w < 4; ++w) {
        const float od = red_d[w * RP + tid];
        const int oi = red_i[w * RP + tid];
        if (od < bd || (od == bd && oi < bi)) {
          bd = od;
          bi = oi;
        }
      }
      if (bi < 0 || bi >= k) bi = 0;                             // NaN row: no ordering
      const int r = list2[1 + t0 + tid];
      assign[r] = bi;
      mind[r] = bd;
    }
  }
}

// Silhouette coefficient of a sample (K10; SilhouetteCoefficient.java:39-147): for every
// point i, a_i = mean distance to the other points of its cluster, b_i = smallest mean
// distance to another cluster, s_i = (b - a) / max(a, b) (0 for singleton clusters).  The
// sample is sorted by cluster, so the columns of one cluster are contiguous: a thread owns row
// i and streams the columns of its block's column range once, accumulating Euclidean
// distances (fp32 differences squared, sqrt, fp64 sums) into a running per-cluster sum that is
// finalised whenever the column's cluster changes -- no [s, s] distance matrix and no [s, k]
// per-cluster GEMM.  The columns are split into ranges at cluster boundaries (blockIdx.y), so
// a 100k sample runs as thousands of blocks instead of 391, each range giving per row the sum
// over its own cluster (when the range holds it) and the smallest mean over the others;
// km_silhouette_fin combines the ranges.  Column tiles (32 columns x 64 dimensions) come
// through LDS as broadcast reads; the row's own coordinates come from the transposed copy
// xT [d][s] (coalesced across the block's rows); differences and squares are packed pairs
// (v_pk_add_f32 / v_pk_fma_f32).
constexpr int SIL_TC = 32, SIL_DC = 64;
__global__ __launch_bounds__(256) void km_silhouette_part(
    const float* __restrict__ x, const float* __restrict__ xT, const int* __restrict__ cl,
    const int* __restrict__ csize, int s, int d, const int* __restrict__ bounds,
    double* __restrict__ a_part, double* __restrict__ b_part) {
  __shared__ float tile[SIL_DC][SIL_TC];
  __shared__ int tcl[SIL_TC];
  const int tid = threadIdx.x;
  const int i = blockIdx.x * 256 + tid;
  const bool live = i < s;
  const int own = live ? cl[i] : -1;
  const int c0 = bounds[blockIdx.y], c1 = bounds[blockIdx.y + 1];
  double a = 0.0, b = INFINITY;
  int cur = -1;
  double cur_sum = 0.0;
  auto finish = [&](int c, double sum) {
    if (c < 0) return;
    if (c == own) {
      a = sum;
    } else {
      const double m = sum / (double)csize[c];
      b = m < b ? m : b;
    }
  };
  for (int j0 = c0; j0 < c1; j0 += SIL_TC) {
    f32x2 acc[SIL_TC / 2];
#pragma unroll
    for (int c = 0; c < SIL_TC / 2; ++c) acc[c] = f32x2{0.f, 0.f};
    __syncthreads();
    if (tid < SIL_TC) tcl[tid] = j0 + tid < c1 ? cl[j0 + tid] : -1;
    for (int d0 = 0; d0 < d; d0 += SIL_DC) {
      __syncthreads();
      for (int e = tid; e < SIL_TC * SIL_DC; e += 256) {
        const int c = e / SIL_DC, dd = e % SIL_DC;
        const int j = j0 + c, dim = d0 + dd;
        tile[dd][c] = (j < c1 && dim < d) ? x[(long long)j * d + dim] : 0.f;
      }
      __syncthreads();
      const int dn = d - d0 < SIL_DC ? d - d0 : SIL_DC;
      for (int dd = 0; dd < dn; ++dd) {
        const float xi = live ? xT[(long long)(d0 + dd) * s + i] : 0.f;
        const f32x2 xi2 = f32x2{xi, xi};
        const f32x4* tr = reinterpret_cast<const f32x4*>(&tile[dd][0]);
#pragma unroll
        for (int q = 0; q < SIL_TC / 4; ++q) {
          const f32x4 v = tr[q];
          const f32x2 d01 = xi2 - f32x2{v[0], v[1]};
          const f32x2 d23 = xi2 - f32x2{v[2], v[3]};
          acc[2 * q] = d01 * d01 + acc[2 * q];
          acc[2 * q + 1] = d23 * d23 + acc[2 * q + 1];
        }
      }
    }
    if (live) {
#pragma unroll
      for (int c = 0; c < SIL_TC; ++c) {
        const int cc = tcl[c];
        if (cc < 0) continue;
        if (cc != cur) {
          finish(cur, cur_sum);
          cur = cc;
          cur_sum = 0.0;
        }
        cur_sum += (double)sqrtf(acc[c >> 1][c & 1]);
      }
    }
  }
  if (live) {
    finish(cur, cur_sum);
    a_part[(long long)blockIdx.y * s + i] = a;
    b_part[(long long)blockIdx.y * s + i] = b;
  }
}

// The column ranges' per-row results -> s_i, per-block partial sums (fp64).
__global__ __launch_bounds__(256) void km_silhouette_fin(
    const int* __restrict__ cl, const int* __restrict__ csize, int s, int nsplit,
    const double* __restrict__ a_part, const double* __restrict__ b_part,
    double* __restrict__ partial) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const int i = blockIdx.x * 256 + tid;
  double sil = 0.0;
  if (i < s) {
    double a = 0.0, b = INFINITY;
    for (int r = 0; r < nsplit; ++r) {
      a += a_part[(long long)r * s + i];
      const double br = b_part[(long long)r * s + i];
      b = br < b ? br : b;
    }
    const int n_own = csize[cl[i]];
    if (n_own > 1) {
      a /= (double)(n_own - 1);
      sil = a < b ? 1.0 - a / b : (a > b ? b / a - 1.0 : 0.0);
    }
  }
  red[tid] = sil;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) partial[blockIdx.x] = red[0];
}

// MFMA silhouette (K10 on the matrix cores; SilhouetteCoefficient.java:52-77, :107-137): the
// same per-point quantities as km_silhouette_part (the sum of distances to the point's own
// cluster, the smallest mean distance to another one, per column range), with the pairwise
// distances from d^2(i, j) = |x_i|^2 + |x_j|^2 - 2 x_i.x_j and the dot products on
// v_mfma_f32_16x16x4_f32 (exact fp32 products and sums: the fmaf chain, bitwise) -- half the
// arithmetic of the difference-square form, at the matrix-core rate.  The caller centres the
// sample (distances unchanged, norms small: less cancellation) and pads rows to 4 KS floats.
//
// Workgroup: 4 waves x RS subtiles of 16 rows; a wave keeps its rows' whole coordinates in
// registers (rf[r][kk], KS VGPRs per subtile: KS <= 64, d <= 256; at KS = 64, RS = 2 fits two
// waves per SIMD, 214 VGPRs, so one wave's epilogue hides under the other's MFMAs) and streams
// 16-column tiles
// of its column range through LDS (double-buffered, one barrier per tile).  The k index of the
// 16x16x4 MFMA is the lane group g: step kk uses dimension g KS + kk, so each lane reads its
// column's (and row's) dimensions contiguously (ds_read_b128).  Tile output, lane l: row i =
// l % 16 of the subtile, columns 4 g .. 4 g + 3 of the tile (D' = columns x rows).  Epilogue per
// tile: sqrt of the clamped d^2 (the point itself: 0), a lane-group reduction per distinct
// column cluster of the tile (usually one: the sample is sorted by cluster), and a running fp64
// per-cluster sum finalised when the column cluster changes.
template <int KS, int RS, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void
km_silhouette_mfma(const float* __restrict__ x, const float* __restrict__ xn,
                   const int* __restrict__ cl, const int* __restrict__ csize, int s,
                   const int* __restrict__ bounds, double* __restrict__ a_part,
                   double* __restrict__ b_part) {
  constexpr int DP = 4 * KS;        // padded row length (floats)
  constexpr int LS = DP + 4;        // LDS row stride: column rows 4 banks apart
  constexpr int PF = KS / 16;       // float4 staging loads per thread per tile
  __shared__ __attribute__((aligned(16))) float ct[2][16 * LS];
  __shared__ float cn[2][16];
  __shared__ int ccl[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int row0 = blockIdx.x * (64 * RS) + wave * (16 * RS);
  float rf[RS][KS];
  float ni[RS];
  int own[RS];
  double a[RS], b[RS], cur_sum[RS];
#pragma unroll
  for (int r = 0; r < RS; ++r) {
    const int i = row0 + 16 * r + li;
    const f32x4* src = reinterpret_cast<const f32x4*>(x + (long long)i * DP + g * KS);
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const f32x4 v = src[q];
      rf[r][4 * q] = v[0];
      rf[r][4 * q + 1] = v[1];
      rf[r][4 * q + 2] = v[2];
      rf[r][4 * q + 3] = v[3];
    }
    ni[r] = xn[i];
    own[r] = i < s ? cl[i] : -1;
    a[r] = 0.0;
    b[r] = INFINITY;
    cur_sum[r] = 0.0;
  }
  int cur = -1;
  auto finish = [&](int c) {
    if (c < 0) return;
    const double inv = 1.0 / (double)csize[c];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      if (c == own[r]) {
        a[r] = cur_sum[r];
      } else {
        const double m = cur_sum[r] * inv;
        b[r] = m < b[r] ? m : b[r];
      }
      cur_sum[r] = 0.0;
    }
  };
  const int c0 = bounds[blockIdx.y], c1 = bounds[blockIdx.y + 1];
  const int nt = (c1 - c0 + 15) / 16;
  // staging: thread (column sc = tid / 16, part sp = tid % 16) moves PF float4s of the column
  const int sc = tid >> 4, sp = tid & 15;
  f32x4 pf[PF];
  auto fetch = [&](int t) {
    const int j = c0 + 16 * t + sc;
    const int jj = j < s ? j : s - 1;     // columns past the range: loaded, never counted
    const f32x4* src = reinterpret_cast<const f32x4*>(x + (long long)jj * DP + sp * (DP / 16));
#pragma unroll
    for (int q = 0; q < PF; ++q) pf[q] = src[q];
  };
  auto stage = [&](int t, int buf) {
    f32x4* dst = reinterpret_cast<f32x4*>(&ct[buf][sc * LS + sp * (DP / 16)]);
#pragma unroll
    for (int q = 0; q < PF; ++q) dst[q] = pf[q];
    if (tid < 16) {
      const int j = c0 + 16 * t + tid;
      const bool in = j < c1;
      cn[buf][tid] = in ? xn[j] : 0.f;
      ccl[buf][tid] = in ? cl[j] : -1;
    }
  };
  if (nt > 0) {
    fetch(0);
    stage(0, 0);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) fetch(t + 1);
    f32x4 acc[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4* cb = reinterpret_cast<const f32x4*>(&ct[buf][li * LS + g * KS]);
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const f32x4 cv = cb[q];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int r = 0; r < RS; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(cv[e], rf[r][4 * q + e], acc[r], 0, 0,
                                                        0);
    }
    // distances of this lane's (row, column) pairs
    const int jt = c0 + 16 * t;
    float v[RS][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float nj = cn[buf][4 * g + e];
      const int j = jt + 4 * g + e;
#pragma unroll
      for (int r = 0; r < RS; ++r) {
        const float d2 = fmaf(-2.f, acc[r][e], ni[r] + nj);
        const float dv = sqrtf(d2 > 0.f ? d2 : 0.f);
        v[r][e] = j == row0 + 16 * r + li ? 0.f : dv;
      }
    }
    const int cfirst = ccl[buf][0], clast = ccl[buf][15];
    if (cfirst == clast && cfirst >= 0) {
      // the whole tile in one cluster (the common case)
      if (cfirst != cur) {
        finish(cur);
        cur = cfirst;
      }
#pragma unroll
      for (int r = 0; r < RS; ++r) {
        float p = (v[r][0] + v[r][1]) + (v[r][2] + v[r][3]);
        p += __shfl_xor(p, 16, 64);
        p += __shfl_xor(p, 32, 64);
        cur_sum[r] += (double)p;
      }
    } else {
      // a cluster boundary inside the tile: each run of equal column clusters in order
      int pos = 0;
      while (pos < 16) {
        const int cc = ccl[buf][pos];
        if (cc < 0) break;                 // past the range's end
        int end = pos + 1;
        while (end < 16 && ccl[buf][end] == cc) ++end;
        if (cc != cur) {
          finish(cur);
          cur = cc;
        }
#pragma unroll
        for (int r = 0; r < RS; ++r) {
          float p = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = 4 * g + e;
            p += (m >= pos && m < end) ? v[r][e] : 0.f;
          }
          p += __shfl_xor(p, 16, 64);
          p += __shfl_xor(p, 32, 64);
          cur_sum[r] += (double)p;
        }
        pos = end;
      }
    }
    if (t + 1 < nt) stage(t + 1, buf ^ 1);
    __syncthreads();
  }
  finish(cur);
  if (g == 0) {
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const int i = row0 + 16 * r + li;
      if (i < s) {
        a_part[(long long)blockIdx.y * s + i] = a[r];
        b_part[(long long)blockIdx.y * s + i] = b[r];
      }
    }
  }
}

}  // namespace


// ---- weighted k-means++ over the k-means|| candidates (one draw + one D^2 update per center)
//
// km_pp_draw: ONE workgroup: p_i = w_i * d2_i (w alone for the first draw), an fp64 block
// scan in a fixed order (deterministic, unlike a decoupled look-back scan), and the inverse
// CDF lookup of uniform u[s]: the first i with cdf_i >= u[s] * total (torch.searchsorted's
// left side), clamped to n - 1; a zero total takes fallback[s].  Writes chosen[s].
// km_pp_update: d2_i = min(d2_i, max(|c_i|^2 - 2 c_i . c_j + |c_j|^2, 0)) for j = chosen[s]
// (d2 initialised when `first`).  Two launches per center instead of a dozen torch ops.
__global__ __launch_bounds__(1024) void km_pp_draw(const double* __restrict__ w,
                                                   const double* __restrict__ d2, long long n,
                                                   const double* __restrict__ u,
                                                   const long long* __restrict__ fallback,
                                                   int s, long long* __restrict__ chosen) {
  __shared__ double part[1024];
  __shared__ long long found;
  const int tid = threadIdx.x;
  const long long per = (n + 1023) / 1024;
  const long long lo = tid * per, hi = lo + per < n ? lo + per : n;
  double sum = 0.0;
  for (long long i = lo; i < hi; ++i) sum += d2 ? w[i] * d2[i] : w[i];
  part[tid] = sum;
  if (tid == 0) found = -1;
  __syncthreads();
  // inclusive scan of the 1024 partial sums (Hillis-Steele, fixed order)
  for (int off = 1; off < 1024; off <<= 1) {
    const double v = tid >= off ? part[tid - off] : 0.0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  const double total = part[1023];
  if (!(total > 0.0)) {
    if (tid == 0) chosen[s] = fallback[s];
    return;
  }
  const double target = u[s] * total;
  const double before = tid ? part[tid - 1] : 0.0;
  if (lo < hi && part[tid] >= target && (tid == 0 || before < target)) {
    double c = before;
    long long j = hi - 1;
    for (long long i = lo; i < hi; ++i) {
      c += d2 ? w[i] * d2[i] : w[i];
      if (c >= target) { j = i; break; }
    }
    found = j;
  }
  __syncthreads();
  if (tid == 0) {
    long long j = found >= 0 ? found : n - 1;
    chosen[s] = j < n - 1 ? j : n - 1;
  }
}

// ct: the candidates dimension-major ([d][n]), so a wave's 64 candidates read one coalesced
// 512-byte run per dimension (row-major reads put 64 rows' lines behind every load)
__global__ __launch_bounds__(256) void km_pp_update(const double* __restrict__ ct,
                                                    const double* __restrict__ cn, long long n,
                                                    int d, const long long* __restrict__ chosen,
                                                    int s, int first, double* __restrict__ d2) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long j = chosen[s];
  double dot = 0.0;
  for (int e = 0; e < d; ++e) dot += ct[(long long)e * n + i] * ct[(long long)e * n + j];
  double v = cn[i] - 2.0 * dot + cn[j];
  v = v > 0.0 ? v : 0.0;
  d2[i] = first ? v : (v < d2[i] ? v : d2[i]);
}

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
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_assign_kernel<DKV, RT>), \
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem) != hipSuccess) \
        return ORYX_ELAUNCH;                                                                  \
      attr_set = true;                                                                        \
    }                                                                                         \
    hipLaunchKernelGGL((kmeans_assign_kernel<DKV, RT>), dim3((unsigned)blocks), dim3(256),   \
                       smem, s, x, xnorm, c, cnorm, n, k_pad, assign, mind);                  \
    break;                                                                                    \
  }
  // rows per wave = 16 * RT: RT = 4 halves the LDS B-fragment reads and the L2 -> LDS center
  // traffic per MFMA relative to RT = 2 but drops to one wave per SIMD; measured at d = 256,
  // K = 1000 it ran 7% slower (10.2 vs 9.5 ms per 12.5M points), so RT = 2 is the default and
  // ORYX_KMEANS_RT=4 selects the wide tiles
  static const int rt_pref = getenv("ORYX_KMEANS_RT") ? atoi(getenv("ORYX_KMEANS_RT")) : 0;
#define WIDE_CASE(DKV, NWV, PKV)                                                              \
  case DKV: {                                                                                 \
    const int smem = 2 * (64 * DKV * 64 + 256);                                               \
    const long long blocks = (n + NWV * 64 - 1) / (NWV * 64);                                 \
    static bool attr_set = false;                                                             \
    if (!attr_set && smem > 65536) {                                                          \
      if (hipFuncSetAttribute(                                                                \
              reinterpret_cast<const void*>(&kmeans_assign_wide_kernel<DKV, NWV, PKV>),       \
              hipFuncAttributeMaxDynamicSharedMemorySize, smem) != hipSuccess)                \
        return ORYX_ELAUNCH;                                                                  \
      attr_set = true;                                                                        \
    }                                                                                         \
    hipLaunchKernelGGL((kmeans_assign_wide_kernel<DKV, NWV, PKV>), dim3((unsigned)blocks),    \
                       dim3(NWV * 64), smem, s, x, xnorm, c, cnorm, n, k_pad, assign, mind,   \
                       CertParams{});                                                         \
    return oryx_check_launch();                                                               \
  }
  // default: the 64-point-per-wave kernel where its LDS swizzle applies (d_pad 64/128/256);
  // ORYX_KMEANS_RT=2 or 4 selects the 32- or 64-point A-operand kernel.  ORYX_KMEANS_WAVES=8
  // runs 8-wave blocks (512 points share each center tile: half the L2 -> LDS traffic, one
  // block per CU)
  static const int nw_pref = getenv("ORYX_KMEANS_WAVES") ? atoi(getenv("ORYX_KMEANS_WAVES")) : 4;
  // ORYX_KMEANS_EPI=0 selects the unpacked compare/select epilogue
  static const bool pk = !(getenv("ORYX_KMEANS_EPI") && atoi(getenv("ORYX_KMEANS_EPI")) == 0);
#define WIDE_SWITCH(NWV, PKV)                                                                 \
  switch (dk) {                                                                               \
    WIDE_CASE(2, NWV, PKV)                                                                    \
    WIDE_CASE(4, NWV, PKV)                                                                    \
    WIDE_CASE(8, NWV, PKV)                                                                    \
    default:                                                                                  \
      break;                                                                                  \
  }
  if (rt_pref == 0) {
    if (nw_pref == 8) {
      if (pk) {
        WIDE_SWITCH(8, true)
      } else {
        WIDE_SWITCH(8, false)
      }
    } else if (pk) {
      WIDE_SWITCH(4, true)
    } else {
      WIDE_SWITCH(4, false)
    }
  }
#undef WIDE_SWITCH
#undef WIDE_CASE
  if (rt_pref != 4 && dk <= 8) {
    switch (dk) {
      ASSIGN_CASE(1, 2)
      ASSIGN_CASE(2, 2)
      ASSIGN_CASE(3, 2)
      ASSIGN_CASE(4, 2)
      ASSIGN_CASE(5, 2)
      ASSIGN_CASE(6, 2)
      ASSIGN_CASE(7, 2)
      ASSIGN_CASE(8, 2)
      default:
        return ORYX_EINVAL;
    }
    return oryx_check_launch();
  }
  switch (dk) {
    ASSIGN_CASE(1, 4)
    ASSIGN_CASE(2, 4)
    ASSIGN_CASE(3, 4)
    ASSIGN_CASE(4, 4)
    ASSIGN_CASE(5, 4)
    ASSIGN_CASE(6, 4)
    ASSIGN_CASE(7, 4)
    ASSIGN_CASE(8, 4)
    ASSIGN_CASE(10, 2)
    ASSIGN_CASE(12, 2)
    ASSIGN_CASE(16, 1)
    default:
      return ORYX_EINVAL;
  }
#undef ASSIGN_CASE
  return oryx_check_launch();
}

// Certified fp32-parity assignment: the bf16 MFMA kernel keeps each point's three best
// centers and flags the points whose bf16 ranking is not provably the fp32 one; km_rescore
// then decides those exactly from the fp32 rows (Xf [n][ldx], Cf [k][d]), the flag-2 points
// through km_rescore_full.  Only d_pad 64 / 128 / 256 (the 64-point-per-wave kernel) and
// k_pad <= 65536.  idx2 / flags: [n] scratch; list2: [n + 1] int32 scratch.
int oryx_kmeans_rescore_list(const float* Xf, int ldx, int d, const float* CT2, int k,
                             const int* list2, long long max_rows, int* assign, float* mind,
                             void* stream);

int oryx_kmeans_assign_cert(const void* X, const float* xnorm, const void* C, long long n,
                            int d_pad, int k_pad, const float* cnorm, const float* Xf, int ldx,
                            int d, const float* Cf, const float* CT2, int k, float cmax,
                            int* assign, float* mind, int* idx2, unsigned char* flags,
                            unsigned long long* stats, int* list2, int defer_full,
                            void* stream) {
  if (n <= 0) return ORYX_OK;
  if (n >= 0x7fffffffLL) return ORYX_EINVAL;                   // list2 holds int32 rows
  const int dk = d_pad / 32;
  if (d_pad % 32 || k_pad % 64 || k_pad > 65536 || (dk != 2 && dk != 4 && dk != 8) || k <= 0 ||
      k > k_pad || d > d_pad || d > 512)
    return ORYX_EINVAL;
  int bits = 2;
  while ((1 << bits) < k_pad) ++bits;
  CertParams cp;
  cp.idx2 = idx2;
  cp.flags = flags;
  cp.mask = (1u << bits) - 1u;
  // bf16 round-to-nearest unit roundoff 2^-8 (8-bit significand), 1% slack for |x| being
  // taken from the bf16 row
  cp.u = 1.01f / 256.0f;
  cp.eta_scale = ldexpf(1.0f, bits - 22) + (float)d_pad * ldexpf(1.0f, -22) + 1e-6f;
  cp.cmax = cmax;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* x = reinterpret_cast<const __bf16*>(X);
  const __bf16* c = reinterpret_cast<const __bf16*>(C);
#define CERT_CASE(DKV)                                                                        \
  case DKV: {                                                                                 \
    const int smem = 2 * (64 * DKV * 64 + 256);                                               \
    constexpr int PPB = 4 * 16 * 4;                                                           \
    const long long blocks = (n + PPB - 1) / PPB;                                             \
    static bool attr_set = false;                                                             \
    if (!attr_set && smem > 65536) {                                                          \
      if (!oryx_set_max_lds(&kmeans_assign_wide_kernel<DKV, 4, true, true>, smem))            \
        return ORYX_ELAUNCH;                                                                  \
      attr_set = true;                                                                        \
    }                                                                                         \
    hipLaunchKernelGGL((kmeans_assign_wide_kernel<DKV, 4, true, true>), dim3((unsigned)blocks), \
                       dim3(256), smem, s, x, xnorm, c, cnorm, n, k_pad, assign, mind, cp);   \
    break;                                                                                    \
  }
  switch (dk) {
    CERT_CASE(2)
    CERT_CASE(4)
    CERT_CASE(8)
    default:
      return ORYX_EINVAL;
  }
#undef CERT_CASE
  long long waves = (n + 63) / 64;
  long long blocks = (waves + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (hipMemsetAsync(list2, 0, sizeof(int), s) != hipSuccess) return ORYX_ELAUNCH;
  hipLaunchKernelGGL(km_rescore, dim3((unsigned)blocks), dim3(256), 0, s, Xf, ldx, d, Cf, k, n,
                     assign, idx2, flags, mind, stats, list2);
  // defer_full: the caller takes the flag-2 list (list2) itself (a GEMM over the listed points
  // with a certified top-1, the rest through oryx_kmeans_rescore_list)
  if (defer_full) return oryx_check_launch();
  return oryx_kmeans_rescore_list(Xf, ldx, d, CT2, k, list2, n, assign, mind, stream);
}

// Exact fp32 full rescan (km_rescore_full) of the rows in list2 ([0] = count, then rows);
// max_rows bounds the count (sizes the grid).
int oryx_kmeans_rescore_list(const float* Xf, int ldx, int d, const float* CT2, int k,
                             const int* list2, long long max_rows, int* assign, float* mind,
                             void* stream) {
  if (max_rows <= 0) return ORYX_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // (points per tile, centers per lane, dimension slice): ORYX_KM_FULL_VARIANT picks one of
  // the instantiations for A/B runs; CT2 is padded to 16 dimensions, so SL <= 16
  static const int variant =
      getenv("ORYX_KM_FULL_VARIANT") ? atoi(getenv("ORYX_KM_FULL_VARIANT")) : 0;
  constexpr int SL = 16;
  const int dq = (d + SL - 1) / SL * SL;              // CT2 holds dq / 2 pair rows
#define FULL_LAUNCH(RP, CPL)                                                                  \
  {                                                                                           \
    const size_t smem = (size_t)RP * dq * 4 + 8 * RP * 4;                                     \
    long long fblocks = (max_rows + RP - 1) / RP;                                             \
    if (fblocks > 4096) fblocks = 4096;                                                       \
    static bool full_attr = false;                                                            \
    if (!full_attr && smem > 65536) {                                                         \
      if (!oryx_set_max_lds(&km_rescore_full<RP, CPL, SL>, (int)smem)) return ORYX_ELAUNCH;   \
      full_attr = true;                                                                       \
    }                                                                                         \
    hipLaunchKernelGGL((km_rescore_full<RP, CPL, SL>), dim3((unsigned)fblocks), dim3(256),    \
                       smem, s, Xf, ldx, d, CT2, k, list2, assign, mind);                     \
  }
  switch (variant) {
    case 1: FULL_LAUNCH(16, 2) break;
    case 2: FULL_LAUNCH(4, 4) break;
    case 3: FULL_LAUNCH(8, 4) break;
    case 4: FULL_LAUNCH(4, 2) break;
    default: FULL_LAUNCH(8, 2) break;   // K = 1000, d = 256: 0.55 ms per 37k points
                                        // (8, 4): 0.68, (4, 4): 0.69, (16, 2): 1.24

  }
#undef FULL_LAUNCH
  return oryx_check_launch();
}

// k: number of clusters (rows of sums/counts/dstats).
int oryx_kmeans_accumulate(const float* X, const int* assign, const float* mind, long long n,
                           int d, int ld, int k, float* sums, unsigned long long* counts,
                           double* dstats, void* stream) {
  if (n <= 0) return ORYX_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // LDS budget: 160 KB minus the counts / stats arrays; slice width = the largest power of two
  // whose K x (CW + 1) fp32 partials fit
  constexpr long long LDS = 160 * 1024;
  const long long fixed = (long long)k * (4 + 16);
  int cw = 256;
  while (cw >= 4 && fixed + (long long)k * (cw + 1) * 4 > LDS) cw >>= 1;
  if (cw >= 4 && k > 0) {
    if (cw > d) {
      cw = 4;
      while (cw < d) cw <<= 1;
    }
    const int stride = fixed + (long long)k * (cw + 1) * 4 <= LDS ? cw + 1 : cw;
    const int slices = (d + cw - 1) / cw;
    long long target = 1024 / slices;
    if (target < 1) target = 1;
    long long rpb = (n + target - 1) / target;
    const long long min_rows = 16ll * k > 8192 ? 16ll * k : 8192;   // amortise the flush
    if (rpb < min_rows) rpb = min_rows;
    const long long blocks = (n + rpb - 1) / rpb;
    const size_t smem = (size_t)fixed + (size_t)k * stride * 4;
    // 16-byte row loads need 16-byte aligned rows and slice starts
    const bool vec = (ld % 4 == 0) && (cw % 4 == 0) &&
                     (reinterpret_cast<unsigned long long>(X) % 16 == 0);
    static bool attr_set = false;
    if (!attr_set) {
      if (!oryx_set_max_lds(&kmeans_accumulate_lds_kernel<true>, (int)LDS)) return ORYX_ELAUNCH;
      if (!oryx_set_max_lds(&kmeans_accumulate_lds_kernel<false>, (int)LDS)) return ORYX_ELAUNCH;
      attr_set = true;
    }
    const dim3 grid((unsigned)blocks, (unsigned)slices);
    if (vec)
      hipLaunchKernelGGL(kmeans_accumulate_lds_kernel<true>, grid, dim3(1024), smem, s, X,
                         assign, mind, n, d, ld, k, cw, stride, rpb, sums, counts, dstats);
    else
      hipLaunchKernelGGL(kmeans_accumulate_lds_kernel<false>, grid, dim3(1024), smem, s, X,
                         assign, mind, n, d, ld, k, cw, stride, rpb, sums, counts, dstats);
    return oryx_check_launch();
  }
  long long waves = n < (1ll << 20) ? n : (1ll << 20);
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL(kmeans_accumulate_kernel, dim3(blocks), dim3(256), 0, s, X, assign, mind,
                     n, d, ld, sums, counts, dstats);
  return oryx_check_launch();
}

// Generic counting sort: perm lists 0..n-1 grouped by key (keys in [0, k), k * 4 bytes of
// LDS, so k <= 16384); counts[k] = group sizes; group c occupies [off[c], off[c] + counts[c])
// with off returned in ws (first k * 8 bytes after the block histograms; see
// oryx_counting_sort_offsets).  Order within a group is unspecified.  ws:
// oryx_kmeans_sorted_ws_bytes(n, k) bytes.
int oryx_counting_sort(const int* keys, long long n, int k, int* perm, unsigned long long* counts,
                       void* ws, void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k <= 0 || k > 16384 || n >= (1ll << 31)) return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* w = reinterpret_cast<char*>(ws);
  unsigned int* bh = reinterpret_cast<unsigned int*>(w);
  w += (long long)SORT_BLOCKS * k * 4;
  long long* off = reinterpret_cast<long long*>(w);
  w += (long long)k * 8;
  int* pieces = reinterpret_cast<int*>(w);
  const long long rpb = (n + SORT_BLOCKS - 1) / SORT_BLOCKS;
  const size_t hsm = (size_t)k * 4;
  hipLaunchKernelGGL(km_block_hist, dim3(SORT_BLOCKS), dim3(256), hsm, s, keys, n, k, rpb, bh);
  hipLaunchKernelGGL(km_cluster_scan, dim3((k + 255) / 256), dim3(256), 0, s, bh, SORT_BLOCKS, k,
                     counts);
  hipLaunchKernelGGL(km_offsets, dim3(1), dim3(1024), 0, s, counts, k, off, pieces);
  hipLaunchKernelGGL(km_scatter, dim3(SORT_BLOCKS), dim3(256), hsm, s, keys, n, k, rpb, bh, off,
                     perm);
  return oryx_check_launch();
}

// Workspace bytes for oryx_kmeans_accumulate_sorted.
long long oryx_kmeans_sorted_ws_bytes(long long n, int k) {
  return (long long)SORT_BLOCKS * k * 4 + (long long)k * 8 + (long long)(k + 1) * 4 + n * 4 + 64;
}

// Sort-based accumulation (see km_segment_sum): sums fp32 [k][d] and dstats f64 [k][2] must be
// zeroed; counts u64 [k] is written (not accumulated).  ws: oryx_kmeans_sorted_ws_bytes.
int oryx_kmeans_accumulate_sorted(const float* X, const int* assign, const float* mind,
                                  long long n, int d, int ld, int k, float* sums,
                                  unsigned long long* counts, double* dstats, void* ws,
                                  void* stream) {
  if (n <= 0) return ORYX_OK;
  if (k <= 0 || (long long)k * 4 > 64 * 1024 || n >= (1ll << 31)) return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* w = reinterpret_cast<char*>(ws);
  unsigned int* bh = reinterpret_cast<unsigned int*>(w);
  w += (long long)SORT_BLOCKS * k * 4;
  long long* off = reinterpret_cast<long long*>(w);
  w += (long long)k * 8;
  int* pieces = reinterpret_cast<int*>(w);
  w += (long long)(k + 1) * 4;
  int* perm = reinterpret_cast<int*>(w);
  const long long rpb = (n + SORT_BLOCKS - 1) / SORT_BLOCKS;
  const size_t hsm = (size_t)k * 4;
  hipLaunchKernelGGL(km_block_hist, dim3(SORT_BLOCKS), dim3(256), hsm, s, assign, n, k, rpb, bh);
  hipLaunchKernelGGL(km_cluster_scan, dim3((k + 255) / 256), dim3(256), 0, s, bh, SORT_BLOCKS, k,
                     counts);
  hipLaunchKernelGGL(km_offsets, dim3(1), dim3(1024), 0, s, counts, k, off, pieces);
  hipLaunchKernelGGL(km_scatter, dim3(SORT_BLOCKS), dim3(256), hsm, s, assign, n, k, rpb, bh, off,
                     perm);
  int tpr = 1;
  while (tpr < d && tpr < 256) tpr <<= 1;
  if (tpr < 1) tpr = 1;
  const long long max_pieces = (n + PIECE - 1) / PIECE + k;
  static const bool vec_off =
      getenv("ORYX_KM_SEGSUM_VEC") && atoi(getenv("ORYX_KM_SEGSUM_VEC")) == 0;
  if (!vec_off && d % 4 == 0 && ld % 4 == 0 &&
      (reinterpret_cast<unsigned long long>(X) & 15) == 0) {
    int tpr4 = 1;
    while (tpr4 < d / 4 && tpr4 < 256) tpr4 <<= 1;
    if (dstats)
      hipLaunchKernelGGL(km_segment_sum4<true>, dim3((unsigned)max_pieces), dim3(256), 0, s, X,
                         mind, d, ld, k, perm, counts, off, pieces, tpr4, sums, dstats);
    else
      hipLaunchKernelGGL(km_segment_sum4<false>, dim3((unsigned)max_pieces), dim3(256), 0, s, X,
                         mind, d, ld, k, perm, counts, off, pieces, tpr4, sums, dstats);
    return oryx_check_launch();
  }
  if (dstats)
    hipLaunchKernelGGL(km_segment_sum<true>, dim3((unsigned)max_pieces), dim3(256), 0, s, X,
                       mind, d, ld, k, perm, counts, off, pieces, tpr, sums, dstats);
  else
    hipLaunchKernelGGL(km_segment_sum<false>, dim3((unsigned)max_pieces), dim3(256), 0, s, X,
                       mind, d, ld, k, perm, counts, off, pieces, tpr, sums, dstats);
  return oryx_check_launch();
}

// x [s][d] and xT [d][s] fp32 of the sample sorted by cluster id cl [s] (every id in
// [0, k), csize[k] = points per cluster); bounds [nsplit + 1]: column ranges (increasing, 0
// to s, each boundary the first column of a cluster); work: 2 * nsplit * s doubles; partial
// [ceil(s / 256)] receives per-block sums of the points' silhouettes.
int oryx_kmeans_silhouette(const float* x, const float* xT, const int* cl, const int* csize,
                           int s, int d, const int* bounds, int nsplit, double* work,
                           double* partial, void* stream) {
  if (s <= 0) return ORYX_OK;
  if (d <= 0 || nsplit <= 0 || nsplit > 65535) return ORYX_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned rb = (unsigned)((s + 255) / 256);
  double* a_part = work;
  double* b_part = work + (long long)nsplit * s;
  hipLaunchKernelGGL(km_silhouette_part, dim3(rb, (unsigned)nsplit), dim3(256), 0, st, x, xT,
                     cl, csize, s, d, bounds, a_part, b_part);
  hipLaunchKernelGGL(km_silhouette_fin, dim3(rb), dim3(256), 0, st, cl, csize, s, nsplit,
                     a_part, b_part, partial);
  return oryx_check_launch();
}


// Rows per workgroup of the MFMA form (the padding unit of its input).
static int sil_rs64() {
  // 16-row subtiles per wave at ks = 64: 22 (the default: two subtiles, two waves per SIMD --
  // one wave's epilogue and tile staging run under the other's MFMAs; 51.4 ms at 100k x 256,
  // profiles/r6_silhouette_mfma_rs22_v1.json), 3 (ORYX_KM_SIL_RS=3: 192 VGPRs of coordinates,
  // one wave per SIMD, 59.7 ms) or 2 (one wave per SIMD, 61.6 ms)
  static const int rs = getenv("ORYX_KM_SIL_RS") ? atoi(getenv("ORYX_KM_SIL_RS")) : 22;
  return rs == 2 || rs == 3 ? rs : 22;
}

int oryx_kmeans_silhouette_mfma_rows(int ks) {
  return ks == 64 ? 64 * (sil_rs64() == 22 ? 2 : sil_rs64()) : 256;
}

// The MFMA form (km_silhouette_mfma): xp [rows padded to oryx_kmeans_silhouette_mfma_rows][4 ks]
// fp32 of the CENTRED sample sorted by cluster (padding rows and dimensions past d zero), xn
// [same rows] squared norms; ks in {16, 32, 64} (d <= 4 ks); the rest as
// oryx_kmeans_silhouette.
int oryx_kmeans_silhouette_mfma(const float* xp, const float* xn, const int* cl,
                                const int* csize, int s, int ks, const int* bounds, int nsplit,
                                double* work, double* partial, void* stream) {
  if (s <= 0) return ORYX_OK;
  if (nsplit <= 0 || nsplit > 65535 || (ks != 16 && ks != 32 && ks != 64) ||
      (reinterpret_cast<unsigned long long>(xp) & 15))
    return ORYX_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* a_part = work;
  double* b_part = work + (long long)nsplit * s;
  const unsigned rows = (unsigned)oryx_kmeans_silhouette_mfma_rows(ks);
  const dim3 grid((unsigned)((s + rows - 1) / rows), (unsigned)nsplit);
  if (ks == 16)
    hipLaunchKernelGGL((km_silhouette_mfma<16, 4>), grid, dim3(256), 0, st, xp, xn, cl, csize,
                       s, bounds, a_part, b_part);
  else if (ks == 32)
    hipLaunchKernelGGL((km_silhouette_mfma<32, 4>), grid, dim3(256), 0, st, xp, xn, cl, csize,
                       s, bounds, a_part, b_part);
  else if (sil_rs64() == 2)
    hipLaunchKernelGGL((km_silhouette_mfma<64, 2>), grid, dim3(256), 0, st, xp, xn, cl, csize,
                       s, bounds, a_part, b_part);
  else if (sil_rs64() == 22)
    hipLaunchKernelGGL((km_silhouette_mfma<64, 2, 2>), grid, dim3(256), 0, st, xp, xn, cl,
                       csize, s, bounds, a_part, b_part);
  else
    hipLaunchKernelGGL((km_silhouette_mfma<64, 3>), grid, dim3(256), 0, st, xp, xn, cl, csize,
                       s, bounds, a_part, b_part);
  const unsigned rb = (unsigned)((s + 255) / 256);
  hipLaunchKernelGGL(km_silhouette_fin, dim3(rb), dim3(256), 0, st, cl, csize, s, nsplit,
                     a_part, b_part, partial);
  return oryx_check_launch();
}


// Weighted k-means++ over n candidates ct [d][n] (fp64, dimension-major; norms cn): k draws
// with uniforms u[k]
// (fallback[k] for zero-mass draws) into chosen[k]; d2 [n] is workspace.
int oryx_kmeans_pp(const double* ct, const double* cn, const double* w, long long n, int d,
                   int k, const double* u, const long long* fallback, long long* chosen,
                   double* d2, void* stream) {
  if (n <= 0 || k <= 0 || d <= 0) return ORYX_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned ub = (unsigned)((n + 255) / 256);
  for (int s = 0; s < k; ++s) {
    hipLaunchKernelGGL(km_pp_draw, dim3(1), dim3(1024), 0, st, w, s ? d2 : nullptr, n, u,
                       fallback, s, chosen);
    if (s + 1 < k)
      hipLaunchKernelGGL(km_pp_update, dim3(ub), dim3(256), 0, st, ct, cn, n, d, chosen, s,
                         s == 0 ? 1 : 0, d2);
  }
  return oryx_check_launch();
}
}  // extern "C"
