// fmt64.hip -- doubles -> Python repr text on the GPU (ryu_d2s.h: Ryu shortest digits in the
// host formatter's layout, byte-identical to it; csrc/runtime/tests/ryu_check.cpp holds the
// two to each other over 2e8 values).  One thread per value writes its text into a 24-byte
// slot and the length beside it; the host assembles the messages from the slots
// (oryx_format_cluster_updates_slots).  Used by the k-means speed layer, whose touched
// centers are already on the device: 256k values of a 10k-point micro-batch took ~1.2 ms on
// 16 host threads.
#include "common.h"

#define ORYX_HD __device__
#define ORYX_RYU_TABLE __constant__
#include "ryu_d2s.h"

namespace {

__global__ __launch_bounds__(256) void fmt_f64_slots(const double* __restrict__ v, long long n,
                                                     uint2* __restrict__ slots,
                                                     unsigned char* __restrict__ lens) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    union {
      char c[24];
      uint2 w[3];
    } o;
    const int l = oryx_ryu::repr(v[i], o.c);
    uint2* s = slots + i * 3;
    s[0] = o.w[0];
    s[1] = o.w[1];
    s[2] = o.w[2];
    lens[i] = (unsigned char)l;
  }
}

}  // namespace

extern "C" {

// v[n] (device doubles) -> slots[n][24] (device bytes, 8-byte aligned), lens[n].
int oryx_format_f64_slots(const double* v, long long n, void* slots, unsigned char* lens,
                          void* stream) {
  if (n <= 0) return ORYX_OK;
  if (reinterpret_cast<uintptr_t>(slots) & 7) return ORYX_EINVAL;
  long long blocks = (n + 255) / 256;
  if (blocks > 256LL * 64) blocks = 256LL * 64;
  hipLaunchKernelGGL(fmt_f64_slots, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), v, n, static_cast<uint2*>(slots),
                     lens);
  return oryx_check_launch();
}

}  // extern "C"
