// ipc_allreduce.hip -- one-shot all-reduce of small fp32 payloads through peer mappings of the
// ranks' exchange buffers (latency-optimal collectives for the k x k
// Gramian and the K x (d + 1) centroid sums that replace MLlib's shuffles,
// [mllib]/als/ALSUpdate.java:116-124, [mllib]/kmeans/KMeansUpdate.java:116-117).
//
// A ring all-reduce of a 64 KB Gramian over 8 GPUs is 14 dependent steps of ~8 KB each: it is
// bound by per-step latency, not by xGMI bandwidth.  Here every rank stages its payload in its
// own exchange buffer (uncached device memory, mapped into every other rank of the node with
// hipIpcOpenMemHandle), raises a flag, waits for every peer's flag, and then each workgroup
// sums its slice of all W payloads straight out of the peers' HBM over the point-to-point
// xGMI links -- one dependent step.  Every rank sums in rank order 0..W-1, so all ranks get
// bitwise the same result.
//
// Exchange buffer of one rank: [flags: 2 x 128 B][slot meta: 2 x 136 words][pad][slot 0: cap
// floats][slot 1: cap floats].  Call `epoch` (1, 2, ...) uses slot epoch & 1 and sets
// flag[epoch & 1] = epoch.  A rank rewrites a slot only two calls later, after it has seen
// every peer arrive at the call in between -- which each peer does only after finishing its
// reads of the call before -- so two slots suffice.  The flag wait is bounded (timeout_s, 120 s
// by default): a peer that never arrives sets *err instead of hanging the GPU, and the call's
// output (and that of every later call until the host clears *err) is NaN rather than a sum
// over a stale slot; the host checks and clears it (parallel/ipc.py).
//
// Every staged payload carries a header in its slot's meta: the epoch and the element count of
// the call that wrote it, and one checksum per staging workgroup (an xor of hashed (bits,
// index) pairs over the elements that workgroup copied).  The reducer runs the same grid with
// the same grid-stride loop, so its workgroup b reads exactly the elements staging workgroup b
// wrote: it checks every peer's epoch and count before summing and recomputes each peer's
// checksum over what it read.  A mismatch -- ranks that disagree on the sequence or size of
// their collectives, a slot overwritten early, a stale read -- sets *err (1000 + 1 + peer:
// header, 2000 + 1 + peer: checksum) instead of passing silently into the sum.
#include <cstring>

#include "common.h"

namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxBlocks = 128;
constexpr int kMetaWords = 8 + kMaxBlocks;      // epoch, n (lo, hi), pad, checksums
constexpr long long kHeaderFloats = 384;        // flags (64) + 2 metas (272), 256 B aligned
struct Peers {
  float* p[kMaxRanks];
};

__device__ __forceinline__ unsigned* flag_of(float* buf, int slot) {
  return reinterpret_cast<unsigned*>(buf) + slot * 32;
}

__device__ __forceinline__ unsigned* meta_of(float* buf, int slot) {
  return reinterpret_cast<unsigned*>(buf) + 64 + slot * kMetaWords;
}

__device__ __forceinline__ unsigned elem_hash(float v, long long i) {
  unsigned h = __float_as_uint(v) ^ ((unsigned)i * 0x9E3779B1u);
  h *= 0x85EBCA6Bu;
  return h ^ (h >> 13);
}

// xor over the 256 threads of the workgroup (lds: 4 words); the result is valid in every thread
__device__ __forceinline__ unsigned block_xor(unsigned v, unsigned* lds) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v ^= (unsigned)__shfl_xor((int)v, off, 64);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  const unsigned r = lds[0] ^ lds[1] ^ lds[2] ^ lds[3];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void ipc_stage(const float* __restrict__ src,
                                                 float* __restrict__ buf, long long slot_off,
                                                 int slot, unsigned epoch, long long n) {
  __shared__ unsigned s_x[4];
  float* dst = buf + slot_off;
  unsigned cs = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float v = src[i];
    dst[i] = v;
    cs ^= elem_hash(v, i);
  }
  cs = block_xor(cs, s_x);
  unsigned* meta = meta_of(buf, slot);
  if (threadIdx.x == 0) {
    meta[8 + blockIdx.x] = cs;
    if (blockIdx.x == 0) {
      meta[0] = epoch;
      meta[1] = (unsigned)(n & 0xFFFFFFFFll);
      meta[2] = (unsigned)(n >> 32);
    }
  }
}

__global__ __launch_bounds__(256) void ipc_signal_reduce(float* __restrict__ out, long long n,
                                                         Peers peers, int W, int rank, int slot,
                                                         unsigned epoch, long long slot_off,
                                                         unsigned long long timeout_ticks,
                                                         int* err) {
  __shared__ unsigned s_cs[kMaxRanks][4];
  __shared__ int s_err;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the staged payload and its header (previous launch on this stream) are written back
    // before the flag
    __threadfence_system();
    __hip_atomic_store(flag_of(peers.p[rank], slot), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < W) {
    // ranks may legitimately arrive seconds apart (host work before a collective); give up
    // after timeout_ticks of the 100 MHz real-time clock
    const unsigned* f = flag_of(peers.p[threadIdx.x], slot);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool arrived = true;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        atomicExch(err, 1 + (int)threadIdx.x);
        arrived = false;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (arrived) {
      // the peer's slot must hold THIS call's payload: same epoch, same element count
      const unsigned* m = meta_of(peers.p[threadIdx.x], slot);
      const unsigned e = __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned lo = __hip_atomic_load(m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned hi = __hip_atomic_load(m + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (e != epoch || (((long long)hi << 32) | lo) != n)
        atomicExch(err, 1001 + (int)threadIdx.x);
    }
  }
  __syncthreads();
  // a peer that never arrived (this block's wait or any other block's) poisons the result
  // with NaN instead of summing its stale slot: the caller's tensor is visibly wrong even
  // before the host reads *err.  One read per workgroup, so its threads agree on the branch.
  if (threadIdx.x == 0) s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_err != 0) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (long long)gridDim.x * 256)
      out[i] = __builtin_nanf("");
    return;
  }
  unsigned cs[kMaxRanks];
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r) cs[r] = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) {
      if (r < W) {
        const float v = __hip_atomic_load(peers.p[r] + slot_off + i, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
        acc += v;
        cs[r] ^= elem_hash(v, i);
      }
    }
    out[i] = acc;
  }
  // per-peer checksums of what this workgroup read vs what the peer's workgroup staged
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r) {
    if (r < W) {
      unsigned v = cs[r];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v ^= (unsigned)__shfl_xor((int)v, off, 64);
      if ((threadIdx.x & 63) == 0) s_cs[r][threadIdx.x >> 6] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < W) {
    const int r = threadIdx.x;
    const unsigned mine = s_cs[r][0] ^ s_cs[r][1] ^ s_cs[r][2] ^ s_cs[r][3];
    const unsigned theirs = __hip_atomic_load(meta_of(peers.p[r], slot) + 8 + blockIdx.x,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (mine != theirs) atomicExch(err, 2001 + r);
  }
}

}  // namespace

extern "C" {

int oryx_ipc_alloc(long long bytes, void** out) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess)
    return ORYX_ELAUNCH;
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess) return ORYX_ELAUNCH;
  *out = p;
  return ORYX_OK;
}

int oryx_ipc_free(void* p) { return hipFree(p) == hipSuccess ? ORYX_OK : ORYX_ELAUNCH; }

int oryx_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

int oryx_ipc_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) return ORYX_ELAUNCH;
  std::memcpy(out, &h, sizeof(h));
  return ORYX_OK;
}

int oryx_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
    return ORYX_ELAUNCH;
  *out = p;
  return ORYX_OK;
}

int oryx_ipc_close(void* p) {
  return hipIpcCloseMemHandle(p) == hipSuccess ? ORYX_OK : ORYX_ELAUNCH;
}

// data: this rank's payload, reduced in place; peers: W exchange-buffer pointers (this rank's
// own at [rank]); cap: slot capacity in floats.
int oryx_ipc_allreduce_f32(float* data, long long n, void* const* peers, int W, int rank,
                           unsigned epoch, long long cap, double timeout_s, int* err,
                           void* stream) {
  if (n <= 0) return ORYX_OK;
  if (W < 1 || W > kMaxRanks || rank < 0 || rank >= W || n > cap || epoch == 0)
    return ORYX_EINVAL;
  Peers ps{};
  for (int r = 0; r < W; ++r) ps.p[r] = static_cast<float*>(peers[r]);
  const int slot = (int)(epoch & 1u);
  const long long slot_off = kHeaderFloats + (long long)slot * cap;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  long long blocks = (n + 255) / 256;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  // both kernels run this grid: reducer workgroup b checks what staging workgroup b wrote
  hipLaunchKernelGGL(ipc_stage, dim3((unsigned)blocks), dim3(256), 0, s, data, ps.p[rank],
                     slot_off, slot, epoch, n);
  const unsigned long long ticks =
      (unsigned long long)((timeout_s > 0 ? timeout_s : 120.0) * 1e8);   // 100 MHz clock
  hipLaunchKernelGGL(ipc_signal_reduce, dim3((unsigned)blocks), dim3(256), 0, s, data, n, ps, W,
                     rank, slot, epoch, slot_off, ticks, err);
  return oryx_check_launch();
}

long long oryx_ipc_header_floats() { return kHeaderFloats; }

}  // extern "C"
