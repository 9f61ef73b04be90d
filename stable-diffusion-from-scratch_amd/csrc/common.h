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

// Cross-lane moves inside groups of 4 / 16 lanes.  SDK_XLANE_DPP (diagnostics only) selects the DPP
// form (v_mov_b32_dpp quad_perm / row_ror); the default is ds_swizzle_b32 (quad-perm and xor bit
// modes: a lane crossbar op of the LDS pipe, no LDS memory, counted by lgkmcnt like any LDS access).
// Round 3 traced a rare corruption of the fused norm3 output (one 16-lane group's LayerNorm variance
// <= 0) to the DPP reductions of ln_quad_stats in an SLP-vectorised build; DESIGN.md §4 has the record.
#ifndef SDK_XLANE_DPP
#define SDK_XLANE_DPP 0
#endif
// CTRL: a DPP quad_perm code (0x00-0xFF: four 2-bit source lanes) or 0x124 / 0x128 (row_ror:4 / 8 in
// the DPP form, xor 4 / xor 8 inside 32-lane halves in the swizzle form: the same set of summands)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  static_assert(CTRL <= 0xFF || CTRL == 0x124 || CTRL == 0x128, "dpp_f: quad_perm, row_ror:4 or row_ror:8");
#if SDK_XLANE_DPP
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
#else
  constexpr int pat = CTRL <= 0xFF ? 0x8000 | CTRL : (0x1F | ((CTRL == 0x124 ? 4 : 8) << 10));
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x), pat));
#endif
}
__device__ __forceinline__ float readlane_f(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
// Sum over the 64 lanes, the same bits in every lane: quad butterfly, then the 16-lane group by two
// more steps, the four group sums read out of lanes 0 / 16 / 32 / 48 and added in a fixed order (a
// wave-uniform value).
__device__ __forceinline__ float wave_sum_f(float x) {
  x += dpp_f<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_f<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_f<0x124>(x);
  x += dpp_f<0x128>(x);
  return (readlane_f(x, 0) + readlane_f(x, 16)) + (readlane_f(x, 32) + readlane_f(x, 48));
}

// LayerNorm row math, shared by layer_norm_kernel (norm.hip) and the cross-attention block's
// fused norm2 / norm3 (xattn.hip) so both produce the same bits.  One wave per row; lane holds
// the 8-channel chunks k = lane + 64 i (i < MAXV, zeros where k >= cols / 8).  Mean and variance
// come out of ONE pair of wave sums: of (x - x0) and (x - x0)^2 around a pivot x0 taken from the
// row itself (its first element), so the E[d^2] - E[d]^2 form does not cancel.  Branch-free, so
// independent rows interleave.
// The row math below fixes every rounding point (contraction off, the fused steps written as fmaf):
// the same source then compiles to the same bits whether or not the translation unit is built with SLP
// vectorisation (packed v_pk_*_f32 code) — the separate LayerNorm launch (norm.hip) and the norms fused
// into the cross-attention block (xattn.hip) and the token linear (token.hip) agree bit for bit.
template <int MAXV>
__device__ __forceinline__ void ln_row_stats(const h8 (&v)[MAXV], int cols, float eps, float& mean, float& rstd) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int c8 = cols / 8;
  const float x0 = readlane_f((float)v[0][0], 0);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const bool ok = lane + 64 * i < c8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = ok ? (float)v[i][j] - x0 : 0.f;
      s1 += d;
      s2 = __builtin_fmaf(d, d, s2);
    }
  }
  s1 = wave_sum_f(s1);
  s2 = wave_sum_f(s2);
  const float inv_n = 1.f / cols;
  const float dm = s1 * inv_n;
  const float var = fmaxf(__builtin_fmaf(-dm, dm, s2 * inv_n), 0.f);
  mean = x0 + dm;
  rstd = rsqrtf(var + eps);
}

// LayerNorm of rows of C = 32 * CPL channels (C <= 640 on the SD path), FOUR lanes per row (16 rows
// per wave): lane q = lane & 3 of a row holds its 8-channel chunks k = q + 4 i (i < CPL), so a row's
// sums are in-lane except for one quad butterfly (the same bits in all four lanes), and a wave
// normalises 16 rows with the instructions a wave-per-row layout spends on ~3.  Shared by
// layer_norm_quad_kernel (norm.hip), the cross-attention block's fused norm2 / norm3 (xattn.hip) and
// token_linear_ln (token.hip), so all produce the same bits.  Pivot x0 = the row's first element.
template <int CPL>
__device__ __forceinline__ void ln_quad_stats(const h8 (&v)[CPL], float eps, float& mean, float& rstd) {
#pragma clang fp contract(off)
  const float x0 = dpp_f<0x00>((float)v[0][0]);    // quad_perm [0,0,0,0]
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = (float)v[i][j] - x0;
      s1 += d;
      s2 = __builtin_fmaf(d, d, s2);
    }
  s1 += dpp_f<0xB1>(s1);
  s2 += dpp_f<0xB1>(s2);
  s1 += dpp_f<0x4E>(s1);
  s2 += dpp_f<0x4E>(s2);
  const float inv_n = 1.f / (32 * CPL);
  const float dm = s1 * inv_n;
  const float var = fmaxf(__builtin_fmaf(-dm, dm, s2 * inv_n), 0.f);
  mean = x0 + dm;
  rstd = rsqrtf(var + eps);
}

// normalised chunk k of a row: gamma / beta (fp32) from LDS (`gb`: gamma[C] then beta[C])
__device__ __forceinline__ h8 ln_quad_apply(const h8& v, float mean, float rstd, const float* gb, int C, int k) {
#pragma clang fp contract(off)
  const f4 g0 = *reinterpret_cast<const f4*>(gb + 8 * k), g1 = *reinterpret_cast<const f4*>(gb + 8 * k + 4);
  const f4 b0 = *reinterpret_cast<const f4*>(gb + C + 8 * k), b1 = *reinterpret_cast<const f4*>(gb + C + 8 * k + 4);
  h8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (half_t)__builtin_fmaf(((float)v[j] - mean) * rstd, g0[j], b0[j]);
    o[4 + j] = (half_t)__builtin_fmaf(((float)v[4 + j] - mean) * rstd, g1[j], b1[j]);
  }
  return o;
}

__device__ __forceinline__ h8 ln_apply8(const h8& v, float mean, float rstd, const float (&g)[8], const float (&b)[8]) {
#pragma clang fp contract(off)
  h8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (half_t)__builtin_fmaf(((float)v[j] - mean) * rstd, g[j], b[j]);
  return o;
}

}  // namespace sdk
