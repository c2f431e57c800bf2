// Shared helpers for the oryx_amd CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) int i32x4;

#define ORYX_WAVE 64

// Error codes returned through the C ABI.
#define ORYX_OK 0
#define ORYX_EINVAL 1
#define ORYX_ELAUNCH 2

__device__ __forceinline__ float oryx_readlane(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ float oryx_shfl(float v, int src_lane) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}

__device__ __forceinline__ int oryx_shfl_i(int v, int src_lane) {
  return __builtin_amdgcn_ds_bpermute(src_lane << 2, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D block id (8 XCDs, round-robin dispatch): blocks that
// the remapped order places next to each other land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nxcd = 8;
  if (nblocks < nxcd) return bid;
  int q = nblocks / nxcd, r = nblocks % nxcd;
  int xcd = bid % nxcd, idx = bid / nxcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

static inline int oryx_check_launch() {
  return hipGetLastError() == hipSuccess ? ORYX_OK : ORYX_ELAUNCH;
}

// Raises a kernel's dynamic-LDS limit (needed past 64 KB); false when the runtime refuses.
template <class K>
inline bool oryx_set_max_lds(K* kernel, int bytes) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                             hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
}

