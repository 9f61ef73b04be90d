// Internal helpers shared by the gfx950 kernels of libsdk_amd.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <string>

#include "../../include/sdk_amd.h"

namespace sdk {

typedef _Float16 half_t;
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

// Raise a kernel's dynamic-LDS cap on the CURRENT device.  hipFuncSetAttribute is per device, so
// the "already done" state is one bit per device id (a process that drives a second GPU sets it
// there too); `done` is a per-kernel-instantiation static.
inline int ensure_dyn_lds(const void* fn, int bytes, std::atomic<unsigned long long>& done, const char* what) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(SDK_EHIP, std::string(what) + ": hipGetDevice failed");
  const unsigned long long bit = 1ull << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return SDK_OK;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    return fail(SDK_EHIP, std::string(what) + ": cannot raise the dynamic LDS limit");
  done.fetch_or(bit, std::memory_order_acq_rel);
  return SDK_OK;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
// erf by Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7, far below the fp16 output's ulp):
// one rcp + one exp + 5 FMAs instead of the libm erff branches
__device__ __forceinline__ float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float r = 1.0f - y * __expf(-a * a);
  return copysignf(r, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// Bijective XCD-aware remap (MI355X: 8 XCDs, workgroups dealt round-robin):
// consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk >> 3, r = nblk & 7, x = bid & 7, i = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

}  // namespace sdk
