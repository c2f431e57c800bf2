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
// histogram fits in LDS the workgroup accumulates privately (ds_add_f32) and flushes non-zero
// bins with one global atomic each -- the root levels, where every row of a tree hits the same
// few thousand bins, would otherwise serialise on L2 atomics.  Deeper levels (many nodes, low
// contention) go straight to global fp32 atomics.
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
    int Fs, int B, float* __restrict__ hist, long long rows_per_block) {
  extern __shared__ float lh[];
  const int t = blockIdx.y;
  const long long per_tree = (long long)nodes * Fs * B * S;
  float* gh = hist + (long long)t * per_tree;
  if (USE_LDS) {
    for (long long i = threadIdx.x; i < per_tree; i += 256) lh[i] = 0.f;
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
    if (node < 0 || node >= nodes) continue;
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
    float* base = (USE_LDS ? lh : gh) + (long long)node * Fs * B * S;
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
    for (long long k = threadIdx.x; k < per_tree; k += 256) {
      const float v = lh[k];
      if (v != 0.f) atomicAdd(gh + k, v);
    }
  }
}

// node_of[t][i] (open node at this level or -1) -> child at the next level, for every row.
// split_feat[t][node] (-1: node became a leaf), split_bin (numeric: go right if bin > split_bin),
// cat_left[t][node][B] (categorical: 1 if the bin goes left; nullptr when no categorical split),
// child_base[t][node]: index of the node's left child in the next level (right = +1).
// visits[t][node] counts rows reaching each open node (unweighted, all rows).
template <typename BinT>
__global__ __launch_bounds__(256) void rdf_route(const BinT* __restrict__ Xb, long long n, int P,
                                                 int T, int* __restrict__ node_of, int nodes,
                                                 const int* __restrict__ split_feat,
                                                 const int* __restrict__ split_bin,
                                                 const unsigned char* __restrict__ cat_left,
                                                 int B, const int* __restrict__ child_base,
                                                 unsigned long long* __restrict__ visits) {
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)T * n;
  for (long long k = gid; k < total; k += (long long)gridDim.x * 256) {
    const int t = (int)(k / n);
    const long long i = k - (long long)t * n;
    const int node = node_of[k];
    if (node < 0) continue;
    const long long tn = (long long)t * nodes + node;
    if (visits) atomicAdd(visits + tn, 1ull);
    const int f = split_feat[tn];
    if (f < 0) {
      node_of[k] = -1;
      continue;
    }
    const int b = (int)Xb[i * P + f];
    bool right;
    if (cat_left && split_bin[tn] < 0) {
      right = cat_left[tn * B + b] == 0;
    } else {
      right = b > split_bin[tn];
    }
    node_of[k] = child_base[tn] + (right ? 1 : 0);
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
  const long long per_tree = (long long)nodes * Fs * B * S;
  const bool lds = per_tree * 4 <= 64 * 1024;
  // enough workgroups to fill the chip several times over across the T trees
  long long blocks = (2048 + T - 1) / T;
  long long rpb = (n + blocks - 1) / blocks;
  if (rpb < 1024) rpb = 1024;
  blocks = (n + rpb - 1) / rpb;
  dim3 grid((unsigned)blocks, (unsigned)T);
  const size_t smem = lds ? (size_t)per_tree * 4 : 0;
#define HIST_LAUNCH(BT, C, L)                                                                 \
  hipLaunchKernelGGL((rdf_histogram<BT, C, L>), grid, dim3(256), smem, s,                    \
                     reinterpret_cast<const BT*>(Xb), n, P, label, y, S, weight, node_of,     \
                     node_lo, nodes, feats, Fs, B, hist, rpb)
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
  long long blocks = ((long long)T * n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(rdf_route<unsigned char>, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const unsigned char*>(Xb), n, P, T, node_of, nodes,
                       split_feat, split_bin, cat_left, B, child_base, visits);
  } else if (bin_bytes == 2) {
    hipLaunchKernelGGL(rdf_route<short>, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const short*>(Xb), n, P, T, node_of, nodes, split_feat,
                       split_bin, cat_left, B, child_base, visits);
  } else {
    return ORYX_EINVAL;
  }
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
