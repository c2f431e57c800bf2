// rdf.hip -- random-decision-forest training and scoring kernels.
//
// the reference trains with Spark MLlib RandomForest
// ([mllib]/rdf/RDFUpdate.java:115-177), whose inner loop is the per-level aggregation of label
// statistics into (node, feature, bin) histograms followed by a best-split search; the
// examples are then pushed through every tree to count node visits (RDFUpdate.java:269-333).
//
// rdf_histogram: one level of all trees at once.  Rows are binned predictors (uint8 or int16,
// row-major [n][P]); every (tree, row) pair whose node is still open adds its bootstrap weight
// times the label statistics (class one-hot for classification; w, w*y, w*y^2 for regression)
// into hist[t][node][j][bin][s] for the node's sampled features j.  When one tree's level
// histogram of a chunk of nodes fits in LDS (<= 128 KB) the workgroup accumulates privately
// (ds_add_f32) and flushes non-zero bins with one global atomic each -- the root levels, where
// every row of a tree hits the same few thousand bins, would otherwise serialise on L2 atomics,
// and deep levels would issue one L2 atomic per (row, feature).  Levels wider than one chunk
// run one block column per node chunk.  Only a node whose own histogram exceeds the budget
// goes straight to global fp32 atomics.
//
// rdf_route: moves every row of every tree one level down after the splits are chosen
// (numeric: bin > split bin goes right; categorical: bit of the bin in the node's left-set mask)
// and counts unweighted node visits (the PMML recordCount and feature-importance inputs).
//
// rdf_forest_leaf: scoring -- walks flattened trees (K14) for a batch of examples.

#include <cmath>

#include "common.h"

namespace {

template <typename BinT, bool CLS, bool USE_LDS>
__global__ __launch_bounds__(256) void rdf_histogram(
    const BinT* __restrict__ Xb, long long n, int P, const int* __restrict__ label,
    const float* __restrict__ y, int S, const unsigned char* __restrict__ weight,
    const int* __restrict__ node_of, int node_lo, int nodes, const int* __restrict__ feats,
    int Fs, int B, float* __restrict__ hist, long long rows_per_block, int node_chunk) {
  extern __shared__ float lh[];
  const int t = blockIdx.y;
  const long long per_node = (long long)Fs * B * S;
  const long long per_tree = (long long)nodes * per_node;
  float* gh = hist + (long long)t * per_tree;
  // LDS path: this block owns the node slots [c_lo, c_hi) of the pass (blockIdx.z chunk)
  const int c_lo = USE_LDS ? (int)blockIdx.z * node_chunk : 0;
  const int c_hi = USE_LDS ? min(nodes, c_lo + node_chunk) : nodes;
  const long long lds_len = (long long)(c_hi - c_lo) * per_node;
  if (USE_LDS) {
    for (long long i = threadIdx.x; i < lds_len; i += 256) lh[i] = 0.f;
    __syncthreads();
  }
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  const int* nodes_t = node_of + (long long)t * n;
  const unsigned char* w_t = weight ? weight + (long long)t * n : nullptr;
  const int* feats_t = feats + (long long)t * nodes * Fs;
  for (long long i = r0 + threadIdx.x; i < r1; i += 256) {
    // node slots [node_lo, node_lo + nodes) of this level are histogrammed in this pass
    const int node = nodes_t[i] - node_lo;
    if (node < c_lo || node >= c_hi) continue;
    const float w = w_t ? (float)w_t[i] : 1.f;
    if (w == 0.f) continue;
    const BinT* xr = Xb + i * P;
    const int* fj = feats_t + node * Fs;
    int s0;
    float v0 = w, v1 = 0.f, v2 = 0.f;
    if (CLS) {
      s0 = label[i];
    } else {
      s0 = 0;
      const float yi = y[i];
      v1 = w * yi;
      v2 = w * yi * yi;
    }
    float* base = USE_LDS ? lh + (long long)(node - c_lo) * per_node : gh + node * per_node;
    for (int j = 0; j < Fs; ++j) {
      const int b = (int)xr[fj[j]];
      float* h = base + ((long long)j * B + b) * S;
      if (CLS) {
        atomicAdd(h + s0, v0);
      } else {
        atomicAdd(h, v0);
        atomicAdd(h + 1, v1);
        atomicAdd(h + 2, v2);
      }
    }
  }
  if (USE_LDS) {
    __syncthreads();
    float* out = gh + (long long)c_lo * per_node;
    for (long long k = threadIdx.x; k < lds_len; k += 256) {
      const float v = lh[k];
      if (v != 0.f) atomicAdd(out + k, v);
    }
  }
}

// node_of[t][i] (open node at this level or -1) -> child at the next level, for every row.
// split_feat[t][node] (-1: node became a leaf), split_bin (numeric: go right if bin > split_bin),
// cat_left[t][node][B] (categorical: 1 if the bin goes left; nullptr when no categorical split),
// child_base[t][node]: index of the node's left child in the next level (right = +1).
// visits[t][node] counts rows reaching each open node (unweighted, all rows).  Grid: x = row
// blocks, y = tree.  Visit counts are privatised in LDS per block (a level's rows all hit a few
// counters -- the root level hits ONE per tree -- so direct global atomics serialise) and
// flushed with one atomic per touched node.
template <typename BinT, bool LDS_VISITS>
__global__ __launch_bounds__(256) void rdf_route(const BinT* __restrict__ Xb, long long n, int P,
                                                 int* __restrict__ node_of, int nodes,
                                                 const int* __restrict__ split_feat,
                                                 const int* __restrict__ split_bin,
                                                 const unsigned char* __restrict__ cat_left,
                                                 int B, const int* __restrict__ child_base,
                                                 unsigned long long* __restrict__ visits,
                                                 long long rows_per_block) {
  extern __shared__ unsigned int vis[];
  const int t = blockIdx.y;
  if (LDS_VISITS) {
    for (int j = threadIdx.x; j < nodes; j += 256) vis[j] = 0u;
    __syncthreads();
  }
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  int* nodes_t = node_of + (long long)t * n;
  const long long tb = (long long)t * nodes;
  for (long long i = r0 + threadIdx.x; i < r1; i += 256) {
    const int node = nodes_t[i];
    if (node < 0) continue;
    const long long tn = tb + node;
    if (visits) {
      if (LDS_VISITS) atomicAdd(vis + node, 1u);
      else atomicAdd(visits + tn, 1ull);
    }
    const int f = split_feat[tn];
    if (f < 0) {
      nodes_t[i] = -1;
      continue;
    }
    const int b = (int)Xb[i * P + f];
    bool right;
    if (cat_left && split_bin[tn] < 0) {
      right = cat_left[tn * B + b] == 0;
    } else {
      right = b > split_bin[tn];
    }
    nodes_t[i] = child_base[tn] + (right ? 1 : 0);
  }
  if (LDS_VISITS) {
    __syncthreads();
    for (int j = threadIdx.x; j < nodes; j += 256) {
      const unsigned int v = vis[j];
      if (v) atomicAdd(visits + tb + j, (unsigned long long)v);
    }
  }
}

// Route without visit counting (the grouped path takes node visits from the per-level
// counting sort): one thread per row walks ALL trees, so the row's bytes come from HBM once
// per level and the other trees' reads of it hit L1/L2, instead of every tree streaming the
// whole bin matrix (grid y = tree in rdf_route).  KEYS: also writes the next level's
// counting-sort keys (see rdf_sort_keys: width = the next level's node slots; bootstrap
// weight 0 -> the visits-only key range; rows in leaves -> 2 T width), which saves the
// separate pass that re-reads node_of and the weights.
template <typename BinT, bool KEYS>
__global__ __launch_bounds__(256) void rdf_route_rows(const BinT* __restrict__ Xb, long long n,
                                                      int P, int T, int* __restrict__ node_of,
                                                      int nodes,
                                                      const int* __restrict__ split_feat,
                                                      const int* __restrict__ split_bin,
                                                      const unsigned char* __restrict__ cat_left,
                                                      int B, const int* __restrict__ child_base,
                                                      const unsigned char* __restrict__ weight,
                                                      int width, int* __restrict__ keys) {
  const int dead = 2 * T * width;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const BinT* xr = Xb + i * P;
    // trees in groups of 8 with each dependent load step issued for the whole group: three
    // memory round trips per 8 trees instead of three per tree
    for (int t0 = 0; t0 < T; t0 += 8) {
      int node[8], f[8], sb[8], cb[8], b[8];
      unsigned int w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        node[u] = t0 + u < T ? node_of[(long long)(t0 + u) * n + i] : -1;
      if (KEYS) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
          w[u] = (weight && node[u] >= 0) ? weight[(long long)(t0 + u) * n + i] : 1u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long long tn = (long long)(t0 + u) * nodes + node[u];
        f[u] = node[u] >= 0 ? split_feat[tn] : -1;
        sb[u] = node[u] >= 0 ? split_bin[tn] : 0;
        cb[u] = node[u] >= 0 ? child_base[tn] : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) b[u] = f[u] >= 0 ? (int)xr[f[u]] : 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (t0 + u >= T) break;
        const long long k = (long long)(t0 + u) * n + i;
        if (node[u] < 0) {
          if (KEYS) keys[k] = dead;
          continue;
        }
        if (f[u] < 0) {
          node_of[k] = -1;
          if (KEYS) keys[k] = dead;
          continue;
        }
        const long long tn = (long long)(t0 + u) * nodes + node[u];
        const bool right =
            (cat_left && sb[u] < 0) ? cat_left[tn * B + b[u]] == 0 : b[u] > sb[u];
        const int nn = cb[u] + (right ? 1 : 0);
        node_of[k] = nn;
        if (KEYS) keys[k] = (t0 + u) * width + nn + (w[u] == 0 ? T * width : 0);
      }
    }
  }
}

// LDS variant of rdf_route_rows for byte bins without categorical splits.  Per (row, tree) the
// global kernel gathers three split-table entries and one bin byte, each a scattered access
// (a wave touches up to 64 lines per load), so the texture-address path bounds it.  Here a
// workgroup first packs the level's split tables into LDS (one word per node: feature in
// bits 0-7, 255 = leaf; split bin in bits 8-15; child base in bits 16-31), then walks tiles
// of 256 consecutive rows: the tile's row bytes are copied into LDS with coalesced dword
// loads (pitch `pitch` dwords, odd, so the 64 lanes' byte reads hit distinct banks) and each
// thread routes its row through all trees with LDS lookups only.  node_of / weight / keys
// stay coalesced global accesses.  Requires P % 4 == 0 (every row starts on a dword),
// features < 255, B <= 256 and child bases < 65536 (the launcher checks).
template <bool KEYS>
__global__ __launch_bounds__(256) void rdf_route_lds(const unsigned char* __restrict__ Xb,
                                                     long long n, int P, int ndw, int pitch,
                                                     int T, int* __restrict__ node_of, int nodes,
                                                     const int* __restrict__ split_feat,
                                                     const int* __restrict__ split_bin,
                                                     const int* __restrict__ child_base,
                                                     const unsigned char* __restrict__ weight,
                                                     int width, int* __restrict__ keys) {
  extern __shared__ unsigned int rsm[];
  const int tid = threadIdx.x;
  const int tn_all = T * nodes;
  unsigned int* tab = rsm;                                  // [T * nodes]
  unsigned int* rows = rsm + tn_all;                        // [256][pitch]
  const unsigned char* rowb = reinterpret_cast<const unsigned char*>(rows);
  for (int j = tid; j < tn_all; j += 256) {
    const int f = split_feat[j];
    tab[j] = f < 0 ? 0xFFu
                   : ((unsigned)f | (((unsigned)split_bin[j] & 0xFFu) << 8) |
                      ((unsigned)child_base[j] << 16));
  }
  const int dead = 2 * T * width;
  const unsigned int* Xw = reinterpret_cast<const unsigned int*>(Xb);
  const int rw = P >> 2;                                    // row pitch in dwords
  constexpr int TG = 32;                                    // trees whose loads go out together
  for (long long r0 = (long long)blockIdx.x * 256; r0 < n; r0 += (long long)gridDim.x * 256) {
    const int nr = n - r0 < 256 ? (int)(n - r0) : 256;
    const long long i = r0 + tid;
    const bool mine = tid < nr;
    // this tile's node ids and bootstrap weights for the first TG trees are loaded before the
    // row staging, so their round trip overlaps it (one memory wait per tile, not one per tree
    // group and operand)
    int node[TG];
    unsigned int w[TG];
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      node[u] = (mine && u < T) ? node_of[(long long)u * n + i] : -1;
      if (KEYS) w[u] = (mine && u < T && weight) ? weight[(long long)u * n + i] : 1u;
    }
    __syncthreads();                                        // table ready / previous tile done
    // 32 lanes per row, 8 rows per pass: consecutive rows are consecutive in memory
    for (int r = tid >> 5; r < nr; r += 8) {
      const int c = tid & 31;
      const unsigned int* src = Xw + (r0 + r) * rw;
      for (int cc = c; cc < ndw; cc += 32) rows[r * pitch + cc] = src[cc];
    }
    __syncthreads();
    if (!mine) continue;
    const unsigned char* xr = rowb + tid * pitch * 4;
    for (int t0 = 0; t0 < T; t0 += TG) {
      if (t0 > 0) {
#pragma unroll
        for (int u = 0; u < TG; ++u) {
          node[u] = t0 + u < T ? node_of[(long long)(t0 + u) * n + i] : -1;
          if (KEYS) w[u] = (t0 + u < T && weight) ? weight[(long long)(t0 + u) * n + i] : 1u;
        }
      }
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        if (t0 + u >= T) break;
        const long long k = (long long)(t0 + u) * n + i;
        if (node[u] < 0) {
          if (KEYS) keys[k] = dead;
          continue;
        }
        const unsigned int e = tab[(t0 + u) * nodes + node[u]];
        const unsigned int f = e & 0xFFu;
        if (f == 0xFFu) {
          node_of[k] = -1;
          if (KEYS) keys[k] = dead;
          continue;
        }
        const unsigned int b = xr[f];
        const int nn = (int)(e >> 16) + (b > ((e >> 8) & 0xFFu) ? 1 : 0);
        node_of[k] = nn;
        if (KEYS) keys[k] = (t0 + u) * width + nn + (w[u] == 0 ? T * width : 0);
      }
    }
  }
}

// Poisson(1) bootstrap counts of every (tree, row), [T][n] uint8, in one pass: a counter-
// based hash (splitmix64 of seed and the flat index) gives one 24-bit uniform per entry and
// the inverse CDF (P(X <= k), k < 23, in constant memory) turns it into a count -- the
// distribution torch.poisson / rand + bucketize give, without the 4-byte uniforms and 8-byte
// bucket indices they write and re-read.  Four entries per thread, one dword store.
__constant__ float kPoissonCdf[23];

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ unsigned int poisson1(unsigned long long seed, unsigned long long k) {
  const float u = (float)(splitmix64(seed ^ (k * 0xD1B54A32D192ED03ull)) >> 40) *
                  (1.0f / 16777216.0f);
  unsigned int c = 0;
  while (c < 23 && kPoissonCdf[c] <= u) ++c;
  return c;
}

__global__ __launch_bounds__(256) void rdf_poisson_weights(unsigned long long seed,
                                                           long long total,
                                                           unsigned char* __restrict__ out) {
  const long long nq = (total + 3) / 4;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < nq;
       q += (long long)gridDim.x * 256) {
    const long long k0 = q * 4;
    if (k0 + 4 <= total) {
      unsigned int v = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) v |= poisson1(seed, (unsigned long long)(k0 + j)) << (8 * j);
      reinterpret_cast<unsigned int*>(out)[q] = v;
    } else {
      for (long long k = k0; k < total; ++k) out[k] = (unsigned char)poisson1(seed, k);
    }
  }
}

// Counting-sort keys of one level (RowGroups.from_nodes): open rows with bootstrap weight
// > 0 -> t * width + node, weight-0 open rows -> T * width + t * width + node (visits only),
// rows in leaves -> 2 T width.  One pass instead of four elementwise tensor ops.
__global__ __launch_bounds__(256) void rdf_sort_keys(const int* __restrict__ node_of,
                                                     const unsigned char* __restrict__ weight,
                                                     int T, long long n, int width,
                                                     int* __restrict__ keys) {
  const int t = blockIdx.y;                                   // grid y = tree: no division
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const long long k = (long long)t * n + i;
    const int node = node_of[k];
    int key = 2 * T * width;
    if (node >= 0) {
      key = t * width + node;
      if (weight && weight[k] == 0) key += T * width;
    }
    keys[k] = key;
  }
}

// Segmented level histogram: rows are kept grouped by (tree, node) -- a counting sort of the
// routed rows after every level (oryx_counting_sort) -- so a workgroup owns one PIECE of one
// node's rows: it reads only those rows (row ids through the permutation), accumulates the
// node's Fs x B x S histogram in LDS (8 KB for 10 features x 100 bins x 2 classes, so many
// workgroups share a CU), and flushes it once.  Versus scanning every row once per node chunk
// (rdf_histogram) the deep levels do no skipped-row work and the LDS image stays small.
// perm: indices into the flattened [T][n] row space (nullptr: identity), pieces: per piece
// (tree, node slot relative to node_lo, begin, end) positions into perm.
template <typename BinT, bool CLS, bool USE_LDS>
__global__ __launch_bounds__(256) void rdf_histogram_pieces(
    const BinT* __restrict__ Xb, long long n, int P, const int* __restrict__ label,
    const float* __restrict__ y, int S, const unsigned char* __restrict__ weight,
    const int* __restrict__ perm, const int* __restrict__ piece_tree,
    const int* __restrict__ piece_node, const long long* __restrict__ piece_lo,
    const long long* __restrict__ piece_hi, int nodes, const int* __restrict__ feats, int Fs,
    int B, float* __restrict__ hist, const int* __restrict__ n_live) {
  extern __shared__ float lh[];
  // device pieces (n_live set) come sorted by their first row: the XCD-aware order puts the
  // pieces of different trees over the same rows on one XCD, so those rows come from its L2
  // grid sized by an upper bound (device pieces): the surplus workgroups retire, and the
  // XCD-aware order is taken over the LIVE pieces only -- remapping over the whole grid would
  // leave the live pieces on the first XCDs and the last ones idle
  const int nl = n_live ? *n_live : (int)gridDim.x;
  if ((int)blockIdx.x >= nl) return;
  const int pc = n_live ? xcd_remap(blockIdx.x, nl) : (int)blockIdx.x;
  const int t = piece_tree[pc];
  const int node = piece_node[pc];
  const long long per_node = (long long)Fs * B * S;
  float* gh = hist + ((long long)t * nodes + node) * per_node;
  float* base = USE_LDS ? lh : gh;
  if (USE_LDS) {
    for (long long i = threadIdx.x; i < per_node; i += 256) lh[i] = 0.f;
    __syncthreads();
  }
  const int* fj = feats + ((long long)t * nodes + node) * Fs;
  const long long p0 = piece_lo[pc], p1 = piece_hi[pc];
  const long long toff = (long long)t * n;
  constexpr int U = 4;
  for (long long q = p0 + threadIdx.x; q < p1; q += 256 * U) {
    long long row[U];
    float w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long qq = q + (long long)u * 256;
      row[u] = qq < p1 ? (perm ? (long long)perm[qq] - toff : qq - toff) : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      w[u] = row[u] >= 0 ? (weight ? (float)weight[toff + row[u]] : 1.f) : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (w[u] == 0.f) continue;
      const long long i = row[u];
      int s0;
      float v0 = w[u], v1 = 0.f, v2 = 0.f;
      if (CLS) {
        s0 = label[i];
      } else {
        s0 = 0;
        const float yi = y[i];
        v1 = v0 * yi;
        v2 = v0 * yi * yi;
      }
      const BinT* xr = Xb + i * P;
      for (int j = 0; j < Fs; ++j) {
        const int b = (int)xr[fj[j]];
        float* h = base + ((long long)j * B + b) * S;
        if (CLS) {
          atomicAdd(h + s0, v0);
        } else {
          atomicAdd(h, v0);
          atomicAdd(h + 1, v1);
          atomicAdd(h + 2, v2);
        }
      }
    }
  }
  if (USE_LDS) {
    __syncthreads();
    for (long long k = threadIdx.x; k < per_node; k += 256) {
      const float v = lh[k];
      if (v != 0.f) atomicAdd(gh + k, v);
    }
  }
}

// Row-staged variant (byte bins): the Fs single-byte loads per row of rdf_histogram_pieces
// each touch 64 different cache lines per wave instruction (the rows come through the
// permutation), so the texture-address path, not HBM, bounds it.  Here every wave copies its
// 64 rows whole into its own LDS slice first -- one dword load instruction covers two rows
// (lanes 0-31 and 32-63, lane & 31 = dword of the row), i.e. a handful of cache lines -- and
// each lane then reads its row's Fs feature bytes from LDS.  Waves stage and consume only
// their own rows, so no workgroup barrier is needed until the histogram flush.  A row takes
// RSW dwords of LDS (odd, so the 64 lanes' byte reads fall on distinct banks); a row that
// starts off a dword boundary (P % 4 != 0) is copied from the aligned dword below it and read
// at byte offset (i * P) & 3.
template <bool CLS, bool SPARSE, int HS>
__global__ __launch_bounds__(256) void rdf_histogram_staged(
    const unsigned char* __restrict__ Xb, long long n, int P, const int* __restrict__ label,
    const float* __restrict__ y, int S, const unsigned char* __restrict__ weight,
    const int* __restrict__ perm, const int* __restrict__ piece_tree,
    const int* __restrict__ piece_node, const long long* __restrict__ piece_lo,
    const long long* __restrict__ piece_hi, int nodes, const int* __restrict__ feats, int Fs,
    int B, float* __restrict__ hist, int NDW, int RSW, const int* __restrict__ n_live) {
  extern __shared__ __attribute__((aligned(16))) float lsm[];
  // see rdf_histogram_pieces: sorted device pieces in XCD-aware order
  const int nl = n_live ? *n_live : (int)gridDim.x;   // see rdf_histogram_pieces
  if ((int)blockIdx.x >= nl) return;
  const int pc = n_live ? xcd_remap(blockIdx.x, nl) : (int)blockIdx.x;
  const int per_node = Fs * B * S;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* lh = lsm;                                                        // [per_node]
  int* fjs = reinterpret_cast<int*>(lsm + per_node);                      // [Fs]
  unsigned int* rows = reinterpret_cast<unsigned int*>(lsm + per_node + ((Fs + 3) & ~3)) +
                       wave * 64 * RSW;
  const unsigned char* rowb = reinterpret_cast<const unsigned char*>(rows);
  // (pc: see above)
  const int t = piece_tree[pc];
  const int node = piece_node[pc];
  float* gh = hist + ((long long)t * nodes + node) * per_node;
  for (int i = tid; i < per_node; i += 256) lh[i] = 0.f;   // 0.f and 0u share the bits
  const int* fj = feats + ((long long)t * nodes + node) * Fs;
  for (int j = tid; j < Fs; j += 256) fjs[j] = fj[j];
  // SPARSE (dword-aligned rows, Fs <= 32): only the distinct dwords holding the node's
  // features are staged -- at most Fs of the row's P / 4 -- so the staging slices are that
  // much smaller (more workgroups per CU) and each feature byte is read at s_fo[j]
  __shared__ int s_dw[32], s_fo[32], s_nd;
  __syncthreads();
  if (SPARSE) {
    if (tid == 0) {
      int nd = 0;
      for (int j = 0; j < Fs; ++j) {
        const int d = fjs[j] >> 2;
        int q = 0;
        while (q < nd && s_dw[q] != d) ++q;
        if (q == nd) s_dw[nd++] = d;
        s_fo[j] = q * 4 + (fjs[j] & 3);
      }
      s_nd = nd;
    }
    __syncthreads();
  }
  const int ndw = SPARSE ? s_nd : NDW;
  const long long p0 = piece_lo[pc], p1 = piece_hi[pc];
  const long long toff = (long long)t * n;
  const unsigned int* Xw = reinterpret_cast<const unsigned int*>(Xb);
  // word indices fit 32 bits (the launcher checks n * P < 2^34); the partial last word, if
  // any, is assembled once from its bytes
  const long long nbytes = n * P;
  const unsigned int nfull = (unsigned int)(nbytes >> 2);
  unsigned int tailw = 0;
  for (int b = 0; b < (int)(nbytes & 3); ++b)
    tailw |= (unsigned int)Xb[(long long)nfull * 4 + b] << (8 * b);
  const int half = lane >> 5, wl = lane & 31;
  // software pipeline over the wave's 64-row batches: the next batch's row ids are loaded
  // with this batch's row bytes, and its weights / labels while this batch's bytes go
  // through LDS, so each batch waits on one memory round trip instead of three
  long long i = -1;
  {
    const long long q = p0 + wave * 64 + lane;
    if (q < p1) i = perm ? (long long)perm[q] - toff : q - toff;
  }
  unsigned int wgt = 0;
  float ylab = 0.f;
  int lab = 0;
  if (i >= 0) {
    wgt = weight ? weight[toff + i] : 1u;
    if (CLS) lab = label[i]; else ylab = y[i];
  }
  for (long long q0 = p0 + wave * 64; q0 < p1; q0 += 256) {
    long long inext = -1;
    {
      const long long q = q0 + 256 + lane;
      if (q < p1) inext = perm ? (long long)perm[q] - toff : q - toff;
    }
    const float v0 = (float)wgt;
    const int s0 = lab;
    const float v1 = v0 * ylab, v2 = v0 * ylab * ylab;
    const int nr = (int)((p1 - q0) < 64 ? (p1 - q0) : 64);
    // stage: step it copies rows 2 it (lanes 0-31) and 2 it + 1 (lanes 32-63), dword
    // wp * 32 + (lane & 31) of each; all 32 steps' loads are issued before the first LDS
    // store, so the wave has up to 32 row loads in flight instead of one round trip per step
    const unsigned int wb = i >= 0 ? (unsigned int)((i * P) >> 2) : 0u;   // first word of row
    // row word bases of the 64 rows, shuffled with every lane active (a bpermute reads 0
    // from a lane that is switched off)
    // in two halves of HS steps: HS loads in flight per lane instead of 32 keeps the kernel
    // under the VGPR count of 3 waves per SIMD (ORYX_RDF_STAGE_STEPS=32: one pass)
    for (int h0 = 0; h0 < 32; h0 += HS) {
      unsigned int wbr[HS];
#pragma unroll
      for (int it = 0; it < HS; ++it)
        wbr[it] = (unsigned int)__shfl((int)wb, 2 * (h0 + it) + half, 64);
      for (int wp = 0; wp * 32 < ndw; ++wp) {
        const int w = wp * 32 + wl;
        if (w < ndw) {
          // rows past the batch end load row 0 into their (unused) slots: no per-step
          // predicate.  Only words wi <= nfull can hold bytes of a row, so the index is
          // clamped to the last full word and the partial one comes from tailw.
          unsigned int v[HS];
#pragma unroll
          for (int it = 0; it < HS; ++it) {
            const unsigned int wi = wbr[it] + (unsigned int)(SPARSE ? s_dw[w] : w);
            v[it] = Xw[wi < nfull ? wi : nfull - 1];
            if (wi == nfull) v[it] = tailw;
          }
#pragma unroll
          for (int it = 0; it < HS; ++it) rows[(2 * (h0 + it) + half) * RSW + w] = v[it];
        }
      }
    }
    // this wave's LDS writes before its reads (LDS executes one wave's accesses in order;
    // the fence only stops the compiler from reordering them)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // next batch's weights / labels, in flight during this batch's LDS work
    const long long icur = i;
    i = inext;
    wgt = 0;
    if (i >= 0) {
      wgt = weight ? weight[toff + i] : 1u;
      if (CLS) lab = label[i]; else ylab = y[i];
    }
    const unsigned int wcnt = (unsigned int)v0;
    if (v0 != 0.f) {
      const unsigned char* xr = rowb + lane * RSW * 4 + (SPARSE ? 0 : (int)((icur * P) & 3));
      // features in groups of 8: the 8 byte reads are issued before the 8 atomics (the
      // feature indices come from LDS, copied there once per workgroup)
      for (int j0 = 0; j0 < Fs; j0 += 8) {
        int b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          b[u] = j0 + u < Fs ? xr[SPARSE ? s_fo[j0 + u] : fjs[j0 + u]] : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (j0 + u >= Fs) break;
          float* h = lh + ((j0 + u) * B + b[u]) * S;
          if (CLS) {
            // integer counts (bootstrap weights are small integers): ds_add_u32, exact
            atomicAdd(reinterpret_cast<unsigned int*>(h) + s0, wcnt);
          } else {
            atomicAdd(h, v0);
            atomicAdd(h + 1, v1);
            atomicAdd(h + 2, v2);
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __syncthreads();
  for (int k = tid; k < per_node; k += 256) {
    const float v = CLS ? (float)reinterpret_cast<const unsigned int*>(lh)[k] : lh[k];
    if (v != 0.f) atomicAdd(gh + k, v);
  }
}

// Node label totals only (the last level: every node there becomes a leaf, so the split search
// needs its weighted label statistics and nothing per feature).  Rows in their natural order
// (node_of, the bootstrap weights and the labels are all read coalesced -- through the
// counting-sort permutation they would be one scattered cache line per row): grid x = row
// blocks, y = tree; the tree's width x S totals are privatised in LDS (integer counts for
// classification: bootstrap weights are small integers) and flushed with one global atomic
// per non-zero entry into hist [T][width][S].  visits [T][width] (+=) counts every row at
// the node, bootstrap weight 0 included (the PMML recordCount input the counting sort gives
// the other levels).
template <bool CLS>
__global__ __launch_bounds__(256) void rdf_node_totals(const int* __restrict__ node_of,
                                                       const unsigned char* __restrict__ weight,
                                                       const int* __restrict__ label,
                                                       const float* __restrict__ y, int S,
                                                       long long n, int width,
                                                       long long rows_per_block,
                                                       float* __restrict__ hist,
                                                       unsigned long long* __restrict__ visits) {
  extern __shared__ float lh[];                      // [width][S], then [width] visit counts
  const int t = blockIdx.y;
  const int len = width * S;
  unsigned int* lv = reinterpret_cast<unsigned int*>(lh + len);
  for (int i = threadIdx.x; i < len + width; i += 256) lh[i] = 0.f;   // 0.f, 0u: same bits
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  const int* nd = node_of + (long long)t * n;
  const unsigned char* wt = weight ? weight + (long long)t * n : nullptr;
  for (long long i = r0 + threadIdx.x; i < r1; i += 256) {
    const int node = nd[i];
    if (node < 0) continue;
    atomicAdd(lv + node, 1u);
    const unsigned int w = wt ? wt[i] : 1u;
    if (w == 0) continue;
    if (CLS) {
      atomicAdd(reinterpret_cast<unsigned int*>(lh) + node * S + label[i], w);
    } else {
      const float yi = y[i], wf = (float)w;
      atomicAdd(lh + node * S, wf);
      atomicAdd(lh + node * S + 1, wf * yi);
      atomicAdd(lh + node * S + 2, wf * yi * yi);
    }
  }
  __syncthreads();
  float* gh = hist + (long long)t * len;
  for (int i = threadIdx.x; i < len; i += 256) {
    const float v = CLS ? (float)reinterpret_cast<const unsigned int*>(lh)[i] : lh[i];
    if (v != 0.f) atomicAdd(gh + i, v);
  }
  for (int i = threadIdx.x; i < width; i += 256)
    if (lv[i]) atomicAdd(visits + (long long)t * width + i, (unsigned long long)lv[i]);
}

// Flattened forest scoring: per (example, tree) walk from the tree's root to a leaf.
// feat[node] (-1 leaf), thr[node] (numeric: x >= thr goes right, i.e. the positive child),
// cat_off[node] (>= 0: categorical, bit table at cat_bits[cat_off + encoding]),
// defaults unused (no missing values in dense input), right[node], left[node].
// X: double [n][F] (categorical encodings as values; double so that thresholds compare exactly
// as on the host path).  Output leaf[example][tree].
__global__ __launch_bounds__(256) void rdf_forest_leaf(
    const double* __restrict__ X, long long n, int F, int T, const int* __restrict__ roots,
    const int* __restrict__ feat, const double* __restrict__ thr, const int* __restrict__ cat_off,
    const unsigned char* __restrict__ cat_bits, const int* __restrict__ cat_len,
    const int* __restrict__ left, const int* __restrict__ right, int* __restrict__ leaf) {
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)T * n;
  for (long long k = gid; k < total; k += (long long)gridDim.x * 256) {
    const long long e = k / T;
    const int t = (int)(k - e * T);
    const double* x = X + e * F;
    int node = roots[t];
    for (int guard = 0; guard < 4096; ++guard) {
      const int f = feat[node];
      if (f < 0) break;
      bool pos;
      const int co = cat_off[node];
      if (co >= 0) {
        const int enc = (int)x[f];
        pos = enc >= 0 && enc < cat_len[node] && cat_bits[co + enc] != 0;
      } else {
        pos = x[f] >= thr[node];
      }
      node = pos ? right[node] : left[node];
    }
    leaf[k] = node;
  }
}

// Device-side piece list of one level (no host round trip): slot c = t * W + node of the
// level's counting sort has counts[c] live rows at offset sum(counts[< c]); the slots with
// node in [lo, hi) are cut into ceil(counts / piece) pieces, written in slot order.  One
// 1024-thread block scans the (<= 16384) slots; *n_live receives the piece count, which the
// histogram kernels (grid = an upper bound) read to retire their surplus workgroups.
__global__ __launch_bounds__(1024) void rdf_expand_pieces(
    const long long* __restrict__ counts, int T, int W, int lo, int hi, long long piece,
    int max_pieces, int* __restrict__ ptree, int* __restrict__ pnode,
    long long* __restrict__ pbeg, long long* __restrict__ pend, int* __restrict__ n_live) {
  __shared__ long long s_cnt[1024], s_np[1024];
  const int tid = threadIdx.x;
  const int nslot = T * W;
  const int per = (nslot + 1023) / 1024;
  const int c0 = tid * per;
  long long my_cnt = 0, my_np = 0;
  for (int c = c0; c < c0 + per && c < nslot; ++c) {
    my_cnt += counts[c];
    const int node = c % W;
    if (node >= lo && node < hi) my_np += (counts[c] + piece - 1) / piece;
  }
  s_cnt[tid] = my_cnt;
  s_np[tid] = my_np;
  __syncthreads();
  // inclusive Hillis-Steele scans of both arrays
  for (int off = 1; off < 1024; off <<= 1) {
    const long long a = tid >= off ? s_cnt[tid - off] : 0;
    const long long b = tid >= off ? s_np[tid - off] : 0;
    __syncthreads();
    s_cnt[tid] += a;
    s_np[tid] += b;
    __syncthreads();
  }
  long long off_rows = s_cnt[tid] - my_cnt, off_p = s_np[tid] - my_np;
  for (int c = c0; c < c0 + per && c < nslot; ++c) {
    const long long cnt = counts[c];
    const int node = c % W;
    if (node >= lo && node < hi) {
      const long long np = (cnt + piece - 1) / piece;
      for (long long k = 0; k < np && off_p + k < max_pieces; ++k) {
        const long long b = off_rows + k * piece;
        ptree[off_p + k] = c / W;
        pnode[off_p + k] = node - lo;
        pbeg[off_p + k] = b;
        pend[off_p + k] = b + piece < off_rows + cnt ? b + piece : off_rows + cnt;
      }
      off_p += np;
    }
    off_rows += cnt;
  }
  if (tid == 1023) *n_live = (int)(s_np[1023] < max_pieces ? s_np[1023] : max_pieces);
}

// Fused forest scoring + weighted vote (K14 + K15): one thread per example walks every tree
// (the same traversal as rdf_forest_leaf) and accumulates w_t * leaf_value[leaf] into its own
// output row, then divides by the weight sum -- the [n, T, C] gather of per-tree leaf values
// never exists.  vote [n][C] (regression: C = 1, the weighted mean).
__global__ __launch_bounds__(256) void rdf_forest_vote(
    const double* __restrict__ X, long long n, int F, int T, const int* __restrict__ roots,
    const int* __restrict__ feat, const double* __restrict__ thr, const int* __restrict__ cat_off,
    const unsigned char* __restrict__ cat_bits, const int* __restrict__ cat_len,
    const int* __restrict__ left, const int* __restrict__ right,
    const double* __restrict__ leaf_value, int C, const double* __restrict__ weights,
    double* __restrict__ vote) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (long long)gridDim.x * 256) {
    const double* x = X + e * F;
    double* out = vote + e * C;
    for (int c = 0; c < C; ++c) out[c] = 0.0;
    double wsum = 0.0;
    for (int t = 0; t < T; ++t) {
      int node = roots[t];
      for (int guard = 0; guard < 4096; ++guard) {
        const int f = feat[node];
        if (f < 0) break;
        bool pos;
        const int co = cat_off[node];
        if (co >= 0) {
          const int enc = (int)x[f];
          pos = enc >= 0 && enc < cat_len[node] && cat_bits[co + enc] != 0;
        } else {
          pos = x[f] >= thr[node];
        }
        node = pos ? right[node] : left[node];
      }
      const double w = weights[t];
      wsum += w;
      const double* lv = leaf_value + (long long)node * C;
      for (int c = 0; c < C; ++c) out[c] += w * lv[c];
    }
    const double inv = wsum != 0.0 ? 1.0 / wsum : 0.0;
    for (int c = 0; c < C; ++c) out[c] *= inv;
  }
}

// impurity of label statistics st[0..S) (classification counts; regression w, sum wy,
// sum wy^2), weight in *w.  kind: 0 gini, 1 entropy (log2), 2 variance.
__device__ double rdf_impurity(const double* st, int S, int kind, double* w) {
  if (kind == 2) {
    *w = st[0];
    const double safe = st[0] > 1e-30 ? st[0] : 1e-30;
    const double mean = st[1] / safe;
    const double v = st[2] / safe - mean * mean;
    return v > 0.0 ? v : 0.0;
  }
  double tot = 0.0;
  for (int s = 0; s < S; ++s) tot += st[s];
  *w = tot;
  const double inv = 1.0 / (tot > 1e-30 ? tot : 1e-30);
  double acc = 0.0;
  for (int s = 0; s < S; ++s) {
    const double pr = st[s] * inv;
    if (kind == 0) acc += pr * pr;
    else acc -= pr * log2(pr > 1e-30 ? pr : 1e-30);
  }
  return kind == 0 ? 1.0 - acc : acc;
}

constexpr int RDF_MAX_S = 32;   // label statistics per bin the split kernel keeps in registers

// label centroid of bin b (regression: mean; classification: share of class maj); +inf when
// the bin is empty
// (a NaN centroid -- from a NaN in the histogram -- ranks as an empty bin: rdf_cat_order's
// counting ranks must stay a permutation of [0, B), or ord[] keeps stale entries that later
// index the histogram and cat_left out of bounds)
__device__ __forceinline__ double rdf_centroid(const float* hf, int b, int S, int kind, int maj) {
  double v;
  if (kind == 2) {
    const double cnt = (double)hf[(long long)b * S];
    v = cnt > 0.0 ? (double)hf[(long long)b * S + 1] / cnt : INFINITY;
  } else {
    double c2 = 0.0;
    for (int s = 0; s < S; ++s) c2 += (double)hf[(long long)b * S + s];
    v = c2 > 0.0 ? (double)hf[(long long)b * S + maj] / c2 : INFINITY;
  }
  return v == v ? v : INFINITY;
}

// ord[r] = the bin of rank r in centroid order (ties by bin index, empty bins last)
__device__ void rdf_cat_order(const float* hf, int B, int S, int kind, int maj,
                              unsigned short* ord) {
  for (int b = 0; b < B; ++b) {
    const double cb = rdf_centroid(hf, b, S, kind, maj);
    int r = 0;
    for (int o = 0; o < B; ++o) {
      const double co = rdf_centroid(hf, o, S, kind, maj);
      r += (co < cb || (co == cb && o < b)) ? 1 : 0;
    }
    ord[r] = (unsigned short)b;
  }
}

// Best split of every (tree, node) of a level -- the per-level search MLlib runs over its
// aggregated bins (RandomForest.findBestSplits via RDFUpdate.java:143-165), as one kernel:
// one wave per node, one lane per candidate feature (lane, lane + 64, ...).  A lane walks its
// feature's bins in order (categorical features: bins ordered by label centroid -- regression
// mean, classification share of the node's majority class -- empty bins last, ranks computed
// in the lane and kept in LDS), carries the left statistics as a prefix sum in fp64, and
// scores every split position by the impurity decrease (w_l imp_l + w_r imp_r over the node
// weight; both sides need weight >= 1).  The wave keeps the best (gain, then the lowest
// feature-slot x position index); the node becomes a leaf at max depth, when pure, with < 2
// weighted examples, or without a positive gain.  hist [T][W][Fs][B][S] fp32, feats
// [T][W][Fs]; outputs feat / bin [T][W] (-1: leaf; bin -1 for a categorical split),
// totals [T][W][S] fp64, gain [T][W], cat_left [T][W][B] (nullable when no predictor is
// categorical).
__global__ __launch_bounds__(64) void rdf_best_split(
    const float* __restrict__ hist, const int* __restrict__ feats,
    const unsigned char* __restrict__ is_cat, int T, int W, int Fs, int B, int S, int kind,
    int force_leaf, int* __restrict__ out_feat, int* __restrict__ out_bin,
    double* __restrict__ out_tot, float* __restrict__ out_gain,
    unsigned char* __restrict__ cat_left, int* __restrict__ err) {
  extern __shared__ unsigned short s_ord[];   // [64][B] categorical orders (when used)
  const int lane = threadIdx.x;
  const long long node = blockIdx.x;          // t * W + slot
  const float* h = hist + node * (long long)Fs * B * S;
  const int* fj = feats + node * Fs;
  // node totals = sum over the bins of feature slot 0
  double tot[RDF_MAX_S];
  for (int s = 0; s < S; ++s) tot[s] = 0.0;
  for (int b = lane; b < B; b += 64)
    for (int s = 0; s < S; ++s) tot[s] += (double)h[(long long)b * S + s];
  for (int s = 0; s < S; ++s) {
    double v = tot[s];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    tot[s] = v;
  }
  // every statistic of the node must be finite (label counts, weights and label sums: an
  // all-reduced histogram holding NaN / inf means corrupted input -- a peer's stale or
  // poisoned slot -- and must fail the forest, not quietly drop bins from the search)
  bool finite = true;
  for (long long i = lane; i < (long long)Fs * B * S; i += 64) finite = finite && isfinite(h[i]);
  const bool bad = __any(!finite);
  if (bad && lane == 0 && err) atomicOr(err, 1);
  double wn;
  const double parent = rdf_impurity(tot, S, kind, &wn);
  int maj = 0;
  if (kind != 2)
    for (int s = 1; s < S; ++s) if (tot[s] > tot[maj]) maj = s;
  double best = -INFINITY;
  long long best_idx = 0x7FFFFFFFFFFFFFFFLL;
  const bool leaf_node = bad || force_leaf || wn < 2.0 || parent <= 1e-12 || B < 2;
  unsigned short* ord = s_ord + lane * B;
  // without categorical predictors a feature's split positions are spread over LPF lanes
  // (Fs = 10: 6 lanes each instead of 10 busy lanes of 64); a lane first sums the bins
  // before its chunk in bin order, so every left-hand total -- and so every gain -- is the
  // same fp64 number the one-lane walk computes
  const int LPF = (!is_cat && Fs <= 32) ? 64 / Fs : 1;
  const int CH = (B - 1 + LPF - 1) / LPF;
  if (!leaf_node) {
    for (int u = lane; u < Fs * LPF; u += 64) {
      // the chunk start is clamped to the last split position: the trailing lanes of a
      // feature can start past it ((LPF - 1) * CH > B - 1, e.g. B = 32, Fs = 6: LPF = 10,
      // CH = 4, k0 up to 36), and their prefix walk over bins [0, k0) then read the next
      // feature's bins -- for the last feature of the last node, past the end of hist.  That
      // read ran off the histogram's allocation whenever the caching allocator had placed it
      // at the end of a segment: the intermittent illegal access of the world-2 RDF test.
      const int jj = u / LPF;
      const int k0 = min((u - jj * LPF) * CH, B - 1);
      const int k1 = LPF == 1 ? B - 1 : (k0 + CH < B - 1 ? k0 + CH : B - 1);
      const int f = fj[jj];
      const float* hf = h + (long long)jj * B * S;
      const bool cat = is_cat && is_cat[f];
      if (cat) rdf_cat_order(hf, B, S, kind, maj, ord);
      double left[RDF_MAX_S], right[RDF_MAX_S];
      for (int s = 0; s < S; ++s) left[s] = 0.0;
      for (int b = 0; b < k0; ++b)
        for (int s = 0; s < S; ++s) left[s] += (double)hf[(long long)b * S + s];
      for (int k = k0; k < k1; ++k) {
        const int b = cat ? ord[k] : k;
        for (int s = 0; s < S; ++s) {
          left[s] += (double)hf[(long long)b * S + s];
          right[s] = tot[s] - left[s];
        }
        double wl, wr;
        const double il = rdf_impurity(left, S, kind, &wl);
        const double ir = rdf_impurity(right, S, kind, &wr);
        if (wl >= 1.0 && wr >= 1.0) {
          const double wt = wn > 1e-30 ? wn : 1e-30;
          const double gain = parent - (wl * il + wr * ir) / wt;
          const long long idx = (long long)jj * (B - 1) + k;
          if (gain > best || (gain == best && idx < best_idx)) {
            best = gain;
            best_idx = idx;
          }
        }
      }
    }
  }
  // wave arg-max (gain, then lowest index)
  for (int off = 32; off > 0; off >>= 1) {
    const double og = __shfl_xor(best, off, 64);
    const long long oi = __shfl_xor(best_idx, off, 64);
    if (og > best || (og == best && oi < best_idx)) {
      best = og;
      best_idx = oi;
    }
  }
  const bool leaf = leaf_node || !(best > 1e-12) || isinf(best);
  const int jbest = leaf ? 0 : (int)(best_idx / (B - 1));
  const int kbest = leaf ? 0 : (int)(best_idx % (B - 1));
  const int fbest = leaf ? -1 : fj[jbest];
  const bool cbest = !leaf && is_cat && is_cat[fbest];
  if (lane == 0) {
    out_feat[node] = fbest;
    out_bin[node] = (leaf || cbest) ? -1 : kbest;
    out_gain[node] = leaf ? 0.f : (float)best;
  }
  for (int s = lane; s < S; s += 64) out_tot[node * S + s] = tot[s];
  if (cat_left) {
    unsigned char* cl = cat_left + node * (long long)B;
    if (!cbest) {
      for (int b = lane; b < B; b += 64) cl[b] = 0;
    } else {
      // the winning feature's order (recomputed: a lane's slot holds its last feature's):
      // the first kbest + 1 bins in centroid order go left
      if (lane == 0) rdf_cat_order(h + (long long)jbest * B * S, B, S, kind, maj, s_ord);
      for (int b = lane; b < B; b += 64) cl[b] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int r = lane; r <= kbest; r += 64) cl[s_ord[r]] = 1;
    }
  }
}

}  // namespace

extern "C" {

int oryx_rdf_forest_vote(const double* X, long long n, int F, int T, const int* roots,
                         const int* feat, const double* thr, const int* cat_off,
                         const unsigned char* cat_bits, const int* cat_len, const int* left,
                         const int* right, const double* leaf_value, int C,
                         const double* weights, double* vote, void* stream) {
  if (n <= 0 || T <= 0) return ORYX_OK;
  if (C < 1) return ORYX_EINVAL;
  long long blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(rdf_forest_vote, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), X, n, F, T, roots, feat, thr,
                     cat_off, cat_bits, cat_len, left, right, leaf_value, C, weights, vote);
  return oryx_check_launch();
}

int oryx_rdf_expand_pieces(const long long* counts, int T, int W, int lo, int hi,
                           long long piece, int max_pieces, int* ptree, int* pnode,
                           long long* pbeg, long long* pend, int* n_live, void* stream) {
  if (T <= 0 || W <= 0 || T * W > 16384 || piece <= 0) return ORYX_EINVAL;
  hipLaunchKernelGGL(rdf_expand_pieces, dim3(1), dim3(1024), 0,
                     reinterpret_cast<hipStream_t>(stream), counts, T, W, lo, hi, piece,
                     max_pieces, ptree, pnode, pbeg, pend, n_live);
  return oryx_check_launch();
}

// hist [T][W][Fs][B][S] fp32 -> best split per (tree, node); see rdf_best_split.  err
// (nullable): set to 1 when some node's histogram holds a non-finite value.
int oryx_rdf_best_split(const float* hist, const int* feats, const unsigned char* is_cat, int T,
                        int W, int Fs, int B, int S, int kind, int force_leaf, int* out_feat,
                        int* out_bin, double* out_tot, float* out_gain,
                        unsigned char* cat_left, int* err, void* stream) {
  if (T <= 0 || W <= 0) return ORYX_OK;
  if (S < 1 || S > RDF_MAX_S || B < 1 || kind < 0 || kind > 2) return ORYX_EINVAL;
  const size_t smem = is_cat ? (size_t)64 * B * sizeof(unsigned short) : 0;
  if (smem > 64 * 1024) return ORYX_EINVAL;
  hipLaunchKernelGGL(rdf_best_split, dim3((unsigned)(T * W)), dim3(64), smem,
                     reinterpret_cast<hipStream_t>(stream), hist, feats, is_cat, T, W, Fs, B, S,
                     kind, force_leaf, out_feat, out_bin, out_tot, out_gain, cat_left, err);
  return oryx_check_launch();
}


// bin_bytes: 1 (uint8 bins) or 2 (int16 bins); cls: 1 classification (label, S classes),
// 0 regression (y, S == 3).  hist must be zeroed: [T][nodes][Fs][B][S] fp32.
// node_of holds level-wide slot ids; this pass covers slots [node_lo, node_lo + nodes) and
// feats/hist are indexed by slot - node_lo.
int oryx_rdf_histogram(const void* Xb, int bin_bytes, long long n, int P, const int* label,
                       const float* y, int S, int cls, const unsigned char* weight, int T,
                       const int* node_of, int node_lo, int nodes, const int* feats, int Fs,
                       int B, float* hist, void* stream) {
  if (n <= 0 || T <= 0 || nodes <= 0) return ORYX_OK;
  if ((bin_bytes != 1 && bin_bytes != 2) || (cls && !label) || (!cls && (!y || S != 3)))
    return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // LDS privatisation: a block histograms `chunk` node slots of one tree into LDS (up to
  // 128 KB of the 160 KB); the level is covered by ceil(nodes / chunk) block columns that all
  // scan the rows (rows outside the column's slots are skipped after a 5-byte read).  Rows per
  // block are sized so each block's LDS flush stays small next to its accumulation work.
  const long long per_node_bytes = (long long)Fs * B * S * 4;
  constexpr long long LDS_BUDGET = 128 * 1024;
  const bool lds = per_node_bytes <= LDS_BUDGET;
  int chunk = lds ? (int)(LDS_BUDGET / per_node_bytes) : nodes;
  if (chunk > nodes) chunk = nodes;
  const int nchunks = lds ? (nodes + chunk - 1) / chunk : 1;
  long long target = 2048 / ((long long)T * nchunks);
  if (target < 1) target = 1;
  long long rpb = (n + target - 1) / target;
  const long long min_rows = lds ? 4096 : 1024;
  if (rpb < min_rows) rpb = min_rows;
  const long long blocks = (n + rpb - 1) / rpb;
  dim3 grid((unsigned)blocks, (unsigned)T, (unsigned)nchunks);
  const size_t smem = lds ? (size_t)chunk * per_node_bytes : 0;
#define HIST_LAUNCH(BT, C, L)                                                                 \
  do {                                                                                        \
    if (L && smem > 65536) {                                                                  \
      if (!oryx_set_max_lds(&rdf_histogram<BT, C, L>, (int)smem)) return ORYX_ELAUNCH;     \
    }                                                                                         \
    hipLaunchKernelGGL((rdf_histogram<BT, C, L>), grid, dim3(256), smem, s,                  \
                       reinterpret_cast<const BT*>(Xb), n, P, label, y, S, weight, node_of,   \
                       node_lo, nodes, feats, Fs, B, hist, rpb, chunk);                       \
  } while (0)
  if (bin_bytes == 1) {
    if (cls) {
      if (lds) HIST_LAUNCH(unsigned char, true, true); else HIST_LAUNCH(unsigned char, true, false);
    } else {
      if (lds) HIST_LAUNCH(unsigned char, false, true); else HIST_LAUNCH(unsigned char, false, false);
    }
  } else {
    if (cls) {
      if (lds) HIST_LAUNCH(short, true, true); else HIST_LAUNCH(short, true, false);
    } else {
      if (lds) HIST_LAUNCH(short, false, true); else HIST_LAUNCH(short, false, false);
    }
  }
#undef HIST_LAUNCH
  return oryx_check_launch();
}

// rdf_route_lds when it applies (byte bins, no categorical split tables, dword-aligned rows,
// the packed table fields fit, LDS fits); returns false to fall back to rdf_route_rows.
static bool route_lds_launch(const void* Xb, int bin_bytes, long long n, int P, int p_used,
                             int T, int* node_of, int nodes, const int* split_feat,
                             const int* split_bin, const unsigned char* cat_left,
                             const int* child_base, const unsigned char* weight, int width,
                             int* keys, hipStream_t s) {
  static const bool off = getenv("ORYX_RDF_ROUTE_LDS") && atoi(getenv("ORYX_RDF_ROUTE_LDS")) == 0;
  if (off || bin_bytes != 1 || cat_left || P % 4 != 0 || p_used <= 0 || p_used > 255 ||
      p_used > P || 2LL * nodes >= 65536)
    return false;
  const int ndw = (p_used + 3) / 4;
  const int pitch = ndw | 1;
  const size_t smem = ((size_t)T * nodes + 256 * (size_t)pitch) * 4;
  if (smem > 64 * 1024) return false;
  long long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (keys)
    hipLaunchKernelGGL(rdf_route_lds<true>, dim3((unsigned)blocks), dim3(256), smem, s,
                       reinterpret_cast<const unsigned char*>(Xb), n, P, ndw, pitch, T, node_of,
                       nodes, split_feat, split_bin, child_base, weight, width, keys);
  else
    hipLaunchKernelGGL(rdf_route_lds<false>, dim3((unsigned)blocks), dim3(256), smem, s,
                       reinterpret_cast<const unsigned char*>(Xb), n, P, ndw, pitch, T, node_of,
                       nodes, split_feat, split_bin, child_base, nullptr, 0, nullptr);
  return true;
}

int oryx_rdf_route(const void* Xb, int bin_bytes, long long n, int P, int p_used, int T,
                   int* node_of, int nodes, const int* split_feat, const int* split_bin,
                   const unsigned char* cat_left, int B, const int* child_base,
                   unsigned long long* visits, void* stream) {
  if (n <= 0 || T <= 0) return ORYX_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!visits && route_lds_launch(Xb, bin_bytes, n, P, p_used, T, node_of, nodes, split_feat,
                                  split_bin, cat_left, child_base, nullptr, 1, nullptr, s))
    return oryx_check_launch();
  if (!visits) {
    long long blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (bin_bytes == 1)
      hipLaunchKernelGGL((rdf_route_rows<unsigned char, false>), dim3((unsigned)blocks),
                         dim3(256), 0, s, reinterpret_cast<const unsigned char*>(Xb), n, P, T,
                         node_of, nodes, split_feat, split_bin, cat_left, B, child_base,
                         nullptr, 0, nullptr);
    else if (bin_bytes == 2)
      hipLaunchKernelGGL((rdf_route_rows<short, false>), dim3((unsigned)blocks), dim3(256), 0, s,
                         reinterpret_cast<const short*>(Xb), n, P, T, node_of, nodes, split_feat,
                         split_bin, cat_left, B, child_base, nullptr, 0, nullptr);
    else
      return ORYX_EINVAL;
    return oryx_check_launch();
  }
  long long target = 4096 / T;
  if (target < 1) target = 1;
  long long rpb = (n + target - 1) / target;
  if (rpb < 2048) rpb = 2048;
  const long long blocks = (n + rpb - 1) / rpb;
  dim3 grid((unsigned)blocks, (unsigned)T);
  const bool lds = nodes <= 16384;
  const size_t smem = lds ? (size_t)nodes * 4 : 0;
#define ROUTE_LAUNCH(BT, L)                                                                   \
  hipLaunchKernelGGL((rdf_route<BT, L>), grid, dim3(256), smem, s,                           \
                     reinterpret_cast<const BT*>(Xb), n, P, node_of, nodes, split_feat,       \
                     split_bin, cat_left, B, child_base, visits, rpb)
  if (bin_bytes == 1) {
    if (lds) ROUTE_LAUNCH(unsigned char, true); else ROUTE_LAUNCH(unsigned char, false);
  } else if (bin_bytes == 2) {
    if (lds) ROUTE_LAUNCH(short, true); else ROUTE_LAUNCH(short, false);
  } else {
    return ORYX_EINVAL;
  }
#undef ROUTE_LAUNCH
  return oryx_check_launch();
}

// Route every open row one level down AND write the next level's counting-sort keys
// (keys [T][n] int32, next-level width `width`; weight [T][n] nullable) in one pass.
int oryx_rdf_route_keys(const void* Xb, int bin_bytes, long long n, int P, int p_used, int T,
                        int* node_of, int nodes, const int* split_feat, const int* split_bin,
                        const unsigned char* cat_left, int B, const int* child_base,
                        const unsigned char* weight, int width, int* keys, void* stream) {
  if (n <= 0 || T <= 0) return ORYX_OK;
  if (!keys || width <= 0 || 2LL * T * width >= (1LL << 31)) return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (route_lds_launch(Xb, bin_bytes, n, P, p_used, T, node_of, nodes, split_feat, split_bin,
                       cat_left, child_base, weight, width, keys, s))
    return oryx_check_launch();
  long long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (bin_bytes == 1)
    hipLaunchKernelGGL((rdf_route_rows<unsigned char, true>), dim3((unsigned)blocks), dim3(256),
                       0, s, reinterpret_cast<const unsigned char*>(Xb), n, P, T, node_of, nodes,
                       split_feat, split_bin, cat_left, B, child_base, weight, width, keys);
  else if (bin_bytes == 2)
    hipLaunchKernelGGL((rdf_route_rows<short, true>), dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const short*>(Xb), n, P, T, node_of, nodes, split_feat,
                       split_bin, cat_left, B, child_base, weight, width, keys);
  else
    return ORYX_EINVAL;
  return oryx_check_launch();
}

int oryx_rdf_histogram_pieces(const void* Xb, int bin_bytes, long long n, int P, int p_used,
                              const int* label, const float* y, int S, int cls,
                              const unsigned char* weight, const int* perm,
                              const int* piece_tree, const int* piece_node,
                              const long long* piece_lo, const long long* piece_hi,
                              int n_pieces, int nodes, const int* feats, int Fs, int B,
                              float* hist, const int* n_live, void* stream) {
  if (n_pieces <= 0) return ORYX_OK;
  if ((bin_bytes != 1 && bin_bytes != 2) || (cls && !label) || (!cls && (!y || S != 3)))
    return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const long long per_node_bytes = (long long)Fs * B * S * 4;
  // row-staged kernel for byte bins when histogram + 256 staged rows fit in 64 KB of LDS
  // (ORYX_RDF_HIST=0 selects the direct-gather kernel)
  static const bool staged_ok =
      !(getenv("ORYX_RDF_HIST") && atoi(getenv("ORYX_RDF_HIST")) == 0);
  if (staged_ok && bin_bytes == 1 && n * (long long)P < (1LL << 34) && n * (long long)P >= 4) {
    // dwords covering the row's used bytes (p_used <= P: the padding of a padded pitch is
    // never read) at any row alignment; a row pitch that is a multiple of 4 bytes (the padded
    // pitch of ops/rdf.py) starts every row on a dword
    const int pu = p_used > 0 && p_used < P ? p_used : P;
    const int ndw = P % 4 == 0 ? (pu + 3) / 4 : (pu + 3) / 4 + 1;
    // sparse staging (only the node's feature dwords) when rows are dword-aligned and the
    // subset is small: ORYX_RDF_STAGE_SPARSE=0 stages whole rows
    static const bool sparse_ok =
        !(getenv("ORYX_RDF_STAGE_SPARSE") && atoi(getenv("ORYX_RDF_STAGE_SPARSE")) == 0);
    const bool sparse = sparse_ok && P % 4 == 0 && Fs <= 32 && Fs < ndw;
    static const int steps =
        getenv("ORYX_RDF_STAGE_STEPS") ? atoi(getenv("ORYX_RDF_STAGE_STEPS")) : 16;
    const int rsw = (sparse ? Fs : ndw) | 1;
    const long long smem_st = per_node_bytes + ((Fs + 3) & ~3) * 4LL + 256LL * rsw * 4;
    if (smem_st <= 64 * 1024) {
#define STAGED_LAUNCH(C, SP)                                                                  \
  if (steps == 32)                                                                            \
    hipLaunchKernelGGL((rdf_histogram_staged<C, SP, 32>), dim3((unsigned)n_pieces), dim3(256), \
                       smem_st, s, reinterpret_cast<const unsigned char*>(Xb), n, P, label, y, \
                       S, weight, perm, piece_tree, piece_node, piece_lo, piece_hi, nodes,    \
                       feats, Fs, B, hist, ndw, rsw, n_live);                                 \
  else if (steps == 8)                                                                        \
    hipLaunchKernelGGL((rdf_histogram_staged<C, SP, 8>), dim3((unsigned)n_pieces), dim3(256),  \
                       smem_st, s, reinterpret_cast<const unsigned char*>(Xb), n, P, label, y, \
                       S, weight, perm, piece_tree, piece_node, piece_lo, piece_hi, nodes,    \
                       feats, Fs, B, hist, ndw, rsw, n_live);                                 \
  else                                                                                        \
  hipLaunchKernelGGL((rdf_histogram_staged<C, SP, 16>), dim3((unsigned)n_pieces), dim3(256),   \
                     smem_st, s, reinterpret_cast<const unsigned char*>(Xb), n, P, label, y,  \
                     S, weight, perm, piece_tree, piece_node, piece_lo, piece_hi, nodes,      \
                     feats, Fs, B, hist, ndw, rsw, n_live)
      if (cls) {
        if (sparse) STAGED_LAUNCH(true, true); else STAGED_LAUNCH(true, false);
      } else {
        if (sparse) STAGED_LAUNCH(false, true); else STAGED_LAUNCH(false, false);
      }
#undef STAGED_LAUNCH
      return oryx_check_launch();
    }
  }
  const bool lds = per_node_bytes <= 64 * 1024;
  const size_t smem = lds ? (size_t)per_node_bytes : 0;
#define PIECE_LAUNCH(BT, C, L)                                                                \
  hipLaunchKernelGGL((rdf_histogram_pieces<BT, C, L>), dim3((unsigned)n_pieces), dim3(256),  \
                     smem, s, reinterpret_cast<const BT*>(Xb), n, P, label, y, S, weight,     \
                     perm, piece_tree, piece_node, piece_lo, piece_hi, nodes, feats, Fs, B,   \
                     hist, n_live)
  if (bin_bytes == 1) {
    if (cls) {
      if (lds) PIECE_LAUNCH(unsigned char, true, true); else PIECE_LAUNCH(unsigned char, true, false);
    } else {
      if (lds) PIECE_LAUNCH(unsigned char, false, true); else PIECE_LAUNCH(unsigned char, false, false);
    }
  } else {
    if (cls) {
      if (lds) PIECE_LAUNCH(short, true, true); else PIECE_LAUNCH(short, true, false);
    } else {
      if (lds) PIECE_LAUNCH(short, false, true); else PIECE_LAUNCH(short, false, false);
    }
  }
#undef PIECE_LAUNCH
  return oryx_check_launch();
}

// Last-level node totals: hist [T][width][S] and visits [T][width] (+=) from node_of [T][n]
// (-1: in a leaf).
int oryx_rdf_node_totals(const int* node_of, const unsigned char* weight, const int* label,
                         const float* y, int S, int cls, int T, long long n, int width,
                         float* hist, unsigned long long* visits, void* stream) {
  if (n <= 0 || T <= 0 || width <= 0) return ORYX_OK;
  if (S <= 0 || !visits || (cls && !label) || (!cls && (!y || S != 3))) return ORYX_EINVAL;
  const size_t smem = (size_t)width * (S + 1) * 4;
  if (smem > 64 * 1024) return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // ~2048 workgroups in all: enough to fill the chip, few flushes
  long long per_tree = 2048 / T;
  if (per_tree < 1) per_tree = 1;
  long long rpb = (n + per_tree - 1) / per_tree;
  if (rpb < 4096) rpb = 4096;
  const dim3 grid((unsigned)((n + rpb - 1) / rpb), (unsigned)T);
  if (cls)
    hipLaunchKernelGGL(rdf_node_totals<true>, grid, dim3(256), smem, s, node_of, weight, label,
                       y, S, n, width, rpb, hist, visits);
  else
    hipLaunchKernelGGL(rdf_node_totals<false>, grid, dim3(256), smem, s, node_of, weight, label,
                       y, S, n, width, rpb, hist, visits);
  return oryx_check_launch();
}

// Poisson(1) bootstrap weights [total] uint8 (total = T * n; out 4-byte aligned).
int oryx_rdf_poisson_weights(unsigned long long seed, long long total, unsigned char* out,
                             void* stream) {
  if (total <= 0) return ORYX_OK;
  if (reinterpret_cast<unsigned long long>(out) & 3) return ORYX_EINVAL;
  static bool table = false;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!table) {
    float cdf[23];
    double p = std::exp(-1.0), acc = 0.0;
    for (int k = 0; k < 23; ++k) {
      acc += p;
      cdf[k] = (float)acc;
      p /= (double)(k + 1);
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(kPoissonCdf), cdf, sizeof(cdf)) != hipSuccess)
      return ORYX_ELAUNCH;
    table = true;
  }
  long long blocks = ((total + 3) / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(rdf_poisson_weights, dim3((unsigned)blocks), dim3(256), 0, s, seed, total,
                     out);
  return oryx_check_launch();
}

int oryx_rdf_sort_keys(const int* node_of, const unsigned char* weight, int T, long long n,
                       int width, int* keys, void* stream) {
  if (T <= 0 || n <= 0) return ORYX_OK;
  long long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(rdf_sort_keys, dim3((unsigned)blocks, (unsigned)T), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), node_of, weight, T, n, width, keys);
  return oryx_check_launch();
}

int oryx_rdf_forest_leaf(const double* X, long long n, int F, int T, const int* roots,
                         const int* feat, const double* thr, const int* cat_off,
                         const unsigned char* cat_bits, const int* cat_len, const int* left,
                         const int* right, int* leaf, void* stream) {
  if (n <= 0 || T <= 0) return ORYX_OK;
  long long blocks = ((long long)T * n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(rdf_forest_leaf, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), X, n, F, T, roots, feat, thr,
                     cat_off, cat_bits, cat_len, left, right, leaf);
  return oryx_check_launch();
}

}  // extern "C"
