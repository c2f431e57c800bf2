// ipc_allgather.hip -- peer-push all-gather of a replicated factor matrix over the node's
// point-to-point xGMI links (the ALS half-step's exchange of
// the freshly solved rows, the stand-in for MLlib's factor shuffle,
// [mllib]/als/ALSUpdate.java:116-124).
//
// A ring all-gather moves every byte over one link per step: (W - 1) dependent steps, two of
// a GPU's seven links busy.  Here every rank owns a peer mapping (hipIpcOpenMemHandle) of every
// other rank's replicated matrix and, as soon as a row range is solved, writes it straight
// into all W copies: the W - 1 remote copies go out over W - 1 different links at once, and the
// push of range c runs on a side stream while range c + 1 is being solved.
//
// Ordering, per matrix m (X or Y) and exchange epoch e (1, 2, ...; every rank counts the same):
//   * READY: a rank stores ready[m] = e in its own flag buffer (stream-ordered after the last
//     kernel that read the matrix's previous contents).  A pusher waits for ready[m] >= e of
//     every peer before writing into that peer's copy, so it never overwrites rows the peer is
//     still reading.
//   * DONE: after a workgroup's rows are written, every thread fences at system scope and
//     thread 0 stores done[m][src][c][g] = e into each destination's flag buffer.
//   * WAIT: before the matrix is read, a kernel of 32 workgroups waits for every done flag of
//     the epoch and then fences at system scope.
//
// Why the readers cannot see stale rows (the receive copy is ordinary coarse-grained device
// memory, which the solve kernels read through L2): in the gfx942 / gfx950 memory model (LLVM
// AMDGPUUsage, "Memory Model GFX942"), device-local memory is mapped MTYPE RW with the PTE C-bit
// set when the agent has several L2s, and the C-bit makes a write to a local line that does not
// come through this XCD's L2 probe and invalidate the line there (the document names writes
// from CUs of other L2s and from the CPU; a peer GPU's xGMI write enters this HBM through the
// same data fabric as the CPU's -- that it is probed the same way is our reading, which the
// self-test below checks).  So the L2s cannot hold a line older than a completed peer write;
// what can be stale is a CU's vector L1, which every kernel start
// invalidates (the dispatch's acquire), and the solve kernels start after the wait kernel has
// seen the DONE flags (which each pusher raises after a system-scope release of its writes).
// The system-scope fence at the end of the wait covers what the model leaves to software for
// memory that is not local (peer-mapped flag words, uncached).  This is the hardware's
// contract as documented, not something a one-GPU test can show, so the start-up self-test
// (IpcAllGather.self_test) checks it where it matters: every XCD reads the whole destination
// before each push round (ipc_xcd_probe: its L2 and L1 then hold the old lines) and compares it
// with the reference after; any stale line fails the self-test and the exchange falls back to
// RCCL.
// Every wait is bounded (timeout_s, the 100 MHz real-time clock): a peer that never arrives
// sets *err (1 + its rank) and the waiter gives up instead of hanging the GPU; the host checks
// *err after the exchange (parallel/ipc.py) and falls back to RCCL.
//
// Flag buffer of one rank (uncached device memory, zeroed): ready[m] at word 32 m (m < 4),
// then done words from word kDoneBase, index ((m * W + src) * C + c) * G + g.
#include "common.h"

namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxMats = 4;
constexpr int kMaxChunks = 64;
constexpr int kMaxGroups = 64;
constexpr long long kDoneBase = 32LL * kMaxMats;
constexpr long long kFlagWords = kDoneBase + (long long)kMaxMats * kMaxRanks * kMaxChunks *
                                                 kMaxGroups;

struct Ptrs {
  void* p[kMaxRanks];
};

__device__ __forceinline__ bool wait_at_least(const unsigned* f, unsigned epoch,
                                              unsigned long long t0,
                                              unsigned long long ticks, int* err, int who) {
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      atomicCAS(err, 0, 1 + who);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  return true;
}

__global__ __launch_bounds__(64) void ipc_ready(unsigned* own_flags, int m, unsigned epoch) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(own_flags + 32 * m, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// src: n16 16-byte units (this rank's solved range c); dst.p[r] + dst_off16: where the range
// goes in rank r's copy; flags.p[r]: rank r's flag buffer.
__global__ __launch_bounds__(256) void ipc_push(const uint4* __restrict__ src, long long n16,
                                                Ptrs dst, long long dst_off16, Ptrs flags,
                                                int W, int rank, int m, int C, int c,
                                                unsigned epoch, unsigned long long ticks,
                                                int* err) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  if (threadIdx.x < (unsigned)W && (int)threadIdx.x != rank) {
    const unsigned* rdy = static_cast<const unsigned*>(flags.p[threadIdx.x]) + 32 * m;
    if (!wait_at_least(rdy, epoch, __builtin_amdgcn_s_memrealtime(), ticks, err,
                       (int)threadIdx.x))
      ok = 0;
  }
  __syncthreads();
  if (!ok) return;
  const int G = gridDim.x;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16;
       i += (long long)G * 256) {
    const uint4 v = src[i];
    for (int r = 0; r < W; ++r) static_cast<uint4*>(dst.p[r])[dst_off16 + i] = v;
  }
  // every thread's stores are out of its wave before the flags go up
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < (unsigned)W) {
    unsigned* d = static_cast<unsigned*>(flags.p[threadIdx.x]) + kDoneBase +
                  (((long long)m * W + rank) * C + c) * G + blockIdx.x;
    __hip_atomic_store(d, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(256) void ipc_wait_gathered(const unsigned* own_flags, int W,
                                                         int m, int C, int G, unsigned epoch,
                                                         unsigned long long ticks, int* err) {
  const long long total = (long long)W * C * G;
  const unsigned* base = own_flags + kDoneBase + (long long)m * W * C * G;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long long i = threadIdx.x; i < total; i += 256) {
    const int src = (int)(i / ((long long)C * G));
    if (!wait_at_least(base + i, epoch, t0, ticks, err, src)) break;
  }
  __syncthreads();
  // acquire side: drop this XCD's L2 copies of lines the peers rewrote
  __threadfence_system();
}

// Coherence probe of the self-test: every workgroup reads the WHOLE buffer (16-byte units) and
// counts units that differ from ref (out[0] +=), and records the XCD it ran on (out[1] |= 1 <<
// XCC_ID): with enough workgroups every XCD's L2 (and its CUs' L1s) reads every line.  The
// loads are plain loads on purpose -- the ones the solve kernels use.
__global__ __launch_bounds__(256) void ipc_xcd_probe(const uint4* __restrict__ buf,
                                                     const uint4* __restrict__ ref, long long n16,
                                                     int* out) {
  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  int bad = 0;
  for (long long i = threadIdx.x; i < n16; i += 256) {
    const uint4 a = buf[i], b = ref[i];
    bad += (a.x != b.x) | (a.y != b.y) | (a.z != b.z) | (a.w != b.w);
  }
  if (bad) atomicAdd(&s_bad, bad);
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (s_bad) atomicAdd(out, s_bad);
    atomicOr(out + 1, 1 << (xcc & 15));
  }
}

}  // namespace

extern "C" {

// out[0] += units of buf (n16 16-byte units) that differ from ref; out[1] |= the XCDs that read
int oryx_ipc_xcd_probe(const void* buf, const void* ref, long long n16, int* out,
                       void* stream) {
  if (n16 <= 0) return ORYX_OK;
  if ((reinterpret_cast<uintptr_t>(buf) & 15) || (reinterpret_cast<uintptr_t>(ref) & 15))
    return ORYX_EINVAL;
  hipLaunchKernelGGL(ipc_xcd_probe, dim3(64), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const uint4*>(buf),
                     static_cast<const uint4*>(ref), n16, out);
  return oryx_check_launch();
}

long long oryx_ipc_gather_flag_bytes() { return kFlagWords * 4; }

int oryx_ipc_gather_limits(int* out) {
  out[0] = kMaxRanks;
  out[1] = kMaxMats;
  out[2] = kMaxChunks;
  out[3] = kMaxGroups;
  return ORYX_OK;
}

// A pointer inside a device allocation -> (IPC handle of the allocation, byte offset of the
// pointer in it): a peer opens the handle and adds the offset.
int oryx_ipc_handle_range(void* p, void* out_handle, long long* out_offset) {
  void* base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, p) != hipSuccess || base == nullptr)
    return ORYX_ELAUNCH;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, base) != hipSuccess) return ORYX_ELAUNCH;
  __builtin_memcpy(out_handle, &h, sizeof(h));
  *out_offset = (long long)((char*)p - (char*)base);
  return ORYX_OK;
}

int oryx_ipc_gather_ready(void* own_flags, int m, unsigned epoch, void* stream) {
  if (m < 0 || m >= kMaxMats || epoch == 0) return ORYX_EINVAL;
  hipLaunchKernelGGL(ipc_ready, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<unsigned*>(own_flags), m, epoch);
  return oryx_check_launch();
}

// Push this rank's range c (bytes, a multiple of 16) from src into every rank's copy at byte
// offset dst_off; G workgroups (the same G for every range of the exchange).
int oryx_ipc_gather_push(const void* src, long long bytes, void* const* dst, long long dst_off,
                         void* const* flags, int W, int rank, int m, int C, int c, int G,
                         unsigned epoch, double timeout_s, int* err, void* stream) {
  if (W < 1 || W > kMaxRanks || rank < 0 || rank >= W || m < 0 || m >= kMaxMats || C < 1 ||
      C > kMaxChunks || c < 0 || c >= C || G < 1 || G > kMaxGroups || epoch == 0 ||
      bytes < 0 || (bytes & 15) || (dst_off & 15) ||
      (reinterpret_cast<uintptr_t>(src) & 15))
    return ORYX_EINVAL;
  Ptrs d{}, f{};
  for (int r = 0; r < W; ++r) {
    if ((reinterpret_cast<uintptr_t>(dst[r]) & 15) != 0) return ORYX_EINVAL;
    d.p[r] = dst[r];
    f.p[r] = flags[r];
  }
  const unsigned long long ticks = (unsigned long long)((timeout_s > 0 ? timeout_s : 120.0) * 1e8);
  hipLaunchKernelGGL(ipc_push, dim3(G), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(src), bytes / 16, d, dst_off / 16, f, W, rank, m,
                     C, c, epoch, ticks, err);
  return oryx_check_launch();
}

int oryx_ipc_gather_wait(void* own_flags, int W, int m, int C, int G, unsigned epoch,
                         double timeout_s, int* err, void* stream) {
  if (W < 1 || W > kMaxRanks || m < 0 || m >= kMaxMats || C < 1 || C > kMaxChunks || G < 1 ||
      G > kMaxGroups || epoch == 0)
    return ORYX_EINVAL;
  const unsigned long long ticks = (unsigned long long)((timeout_s > 0 ? timeout_s : 120.0) * 1e8);
  hipLaunchKernelGGL(ipc_wait_gathered, dim3(32), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream),
                     static_cast<const unsigned*>(own_flags), W, m, C, G, epoch, ticks, err);
  return oryx_check_launch();
}

}  // extern "C"
