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
    int B, float* __restrict__ hist) {
  extern __shared__ float lh[];
  const int pc = blockIdx.x;
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

}  // namespace

extern "C" {

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
      hipFuncSetAttribute(reinterpret_cast<const void*>(&rdf_histogram<BT, C, L>),           \
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);             \
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

int oryx_rdf_route(const void* Xb, int bin_bytes, long long n, int P, int T, int* node_of,
                   int nodes, const int* split_feat, const int* split_bin,
                   const unsigned char* cat_left, int B, const int* child_base,
                   unsigned long long* visits, void* stream) {
  if (n <= 0 || T <= 0) return ORYX_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
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

int oryx_rdf_histogram_pieces(const void* Xb, int bin_bytes, long long n, int P,
                              const int* label, const float* y, int S, int cls,
                              const unsigned char* weight, const int* perm,
                              const int* piece_tree, const int* piece_node,
                              const long long* piece_lo, const long long* piece_hi,
                              int n_pieces, int nodes, const int* feats, int Fs, int B,
                              float* hist, void* stream) {
  if (n_pieces <= 0) return ORYX_OK;
  if ((bin_bytes != 1 && bin_bytes != 2) || (cls && !label) || (!cls && (!y || S != 3)))
    return ORYX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const long long per_node_bytes = (long long)Fs * B * S * 4;
  const bool lds = per_node_bytes <= 64 * 1024;
  const size_t smem = lds ? (size_t)per_node_bytes : 0;
#define PIECE_LAUNCH(BT, C, L)                                                                \
  hipLaunchKernelGGL((rdf_histogram_pieces<BT, C, L>), dim3((unsigned)n_pieces), dim3(256),  \
                     smem, s, reinterpret_cast<const BT*>(Xb), n, P, label, y, S, weight,     \
                     perm, piece_tree, piece_node, piece_lo, piece_hi, nodes, feats, Fs, B,   \
                     hist)
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
