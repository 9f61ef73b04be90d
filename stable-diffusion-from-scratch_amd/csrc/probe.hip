// Device calibration probes (not on the sampling path): the dense fp16 MFMA rate this MI355X holds
// under load and the HBM streaming rate, measured on the box the bench runs on, next to the spec
// figures the roofline is quoted against (MI355X_MICROARCH.md: ~2.5 PFLOP/s dense fp16, 8 TB/s).
//
// MFMA: every wave keeps independent accumulators (8 of 16x16x32, 4 of 32x32x16) and issues
// back-to-back MFMAs on random operands held in registers (the clock under load depends on operand
// entropy, MICROARCH 'DVFS give-back'); 4-wave workgroups, the caller launches 2 per CU (2 waves per
// SIMD).  The result is folded into `sink` so the work cannot be elided.
// HBM: a grid-stride 16-B copy (read + write counted).
#include <algorithm>

#include "common.h"

namespace sdk {
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
namespace {

// (__launch_bounds__(256, 2): with the default bounds hipcc kept the 16x16x32 accumulators in AGPRs and copied all
// 32 of them through VGPRs every iteration — 48 accvgpr moves per 8 MFMAs — and the probe read 1.19 PF/s; with the
// occupancy stated the loop is 8 bare MFMAs, as the conv kernels' are)
template <bool M16>
__global__ void __launch_bounds__(256, 2) mfma_probe_kernel(const half_t* seed, int iters, float* sink) {
  const int lane = threadIdx.x & 63;
  h8 a = *reinterpret_cast<const h8*>(seed + (size_t)((blockIdx.x * 256 + threadIdx.x) & 4095) * 8);
  h8 b = *reinterpret_cast<const h8*>(seed + (size_t)((blockIdx.x * 256 + threadIdx.x + 1777) & 4095) * 8);
  float r = 0.f;
  if constexpr (M16) {
    f4 acc[8];
    h8 bs[8];   // a distinct B operand per accumulator: eight independent chains, nothing to fold
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = f4{};
      bs[i] = b;
      bs[i][i] = (half_t)((float)b[i] + 0.25f * (float)(i + 1));
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bs[i], acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) r += (acc[i][0] + acc[i][1]) + (acc[i][2] + acc[i][3]);   // every element live
  } else {
    f16v acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f16v{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) r += acc[i][j];
  }
  if (lane == 0) sink[blockIdx.x * 4 + (threadIdx.x >> 6)] = r;
}

// U independent 16-B loads in flight per thread, then their stores; NT: non-temporal loads and stores
// (streamed once: no cache allocation on the way through)
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_probe_kernel(const h8* src, h8* dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    h8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// The flat form: one pass, no loop — workgroup b copies its own contiguous 256*U-vector chunk (each
// wave-instruction 1 KiB contiguous), the grid covers the buffer
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_flat_kernel(const h8* src, h8* dst, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  h8 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) {
      if constexpr (NT) __builtin_nontemporal_store(v[u], dst + i);
      else dst[i] = v[u];
    }
  }
}

// LDS-DMA fill rate (diagnostic, tools/probe_dma.py): every wave of a workgroup streams 1-KiB pieces
// (64 lanes x 16 B, one buffer_load ... lds) from `src` into its own LDS ring, keeping INF pieces in
// flight (counted vmcnt), `pieces` per wave; consecutive waves / workgroups read consecutive pieces,
// wrapped at `bytes` (2 MiB: L2-resident and shared by every CU; 1 GiB: HBM).  MODE 1: the same bytes
// through registers (buffer_load_dwordx4 + ds_write_b128).  The caller divides bytes moved by time.
template <int NW, int INF, int MODE>
__global__ void __launch_bounds__(NW * 64) dma_probe_kernel(const half_t* src, long long bytes, int pieces,
                                                            float* sink) {
  extern __shared__ __attribute__((aligned(16))) half_t lds[];
  constexpr int RING = 128 / NW;                       // pieces per wave (128 KiB per workgroup)
  static_assert(RING > INF, "ring");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<half_t*>(src), 0,
                                                                   (int)std::min(bytes, 0x7fffffffLL), 0x00020000);
  const long long np = bytes / 1024;
  long long g = ((long long)blockIdx.x * NW + wave) * pieces;
  half_t* ring = lds + wave * RING * 512;
  u4 held[INF];
  if constexpr (MODE == 0) {
    for (int i = 0; i < pieces; ++i, ++g) {
      const unsigned off = (unsigned)((g % np) * 1024) + lane * 16u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ring + (i % RING) * 512), 16,
                                               off, 0, 0, 0);
      if (i >= INF) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF) : "memory");
    }
  } else {
    // rounds of INF loads in flight; each round's data is written to LDS as the next round issues
    for (int i = 0; i < pieces; i += INF, g += INF) {
#pragma unroll
      for (int u = 0; u < INF; ++u) {
        if (i > 0) *reinterpret_cast<u4*>(ring + ((i - INF + u) % RING) * 512 + lane * 8) = held[u];
        held[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(((g + u) % np) * 1024) + lane * 16u, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = (float)lds[lane * 8] + (MODE ? (float)held[0][0] : 0.f);
}

}  // namespace
}  // namespace sdk

using namespace sdk;

// diagnostics only (not in sdk_amd.h): one launch of the LDS-DMA fill probe, nw in {4, 8, 16} waves per
// workgroup, inflight in {1, 2, 4, 6} pieces per wave, mode 0 LDS-DMA / 1 register staging
extern "C" int sdk_probe_dma(int32_t nw, int32_t inflight, int32_t mode, const void* src, int64_t bytes, int32_t pieces,
                             int32_t blocks, float* sink, sdk_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
#define SDK_DP(NW_, INF_, MODE_)                                                                                   \
  if (nw == NW_ && inflight == INF_ && mode == MODE_) {                                                            \
    static bool attr = false;                                                                                       \
    if (!attr) {                                                                                                    \
      hipFuncSetAttribute((const void*)dma_probe_kernel<NW_, INF_, MODE_>,                                          \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);                                 \
      attr = true;                                                                                                  \
    }                                                                                                               \
    hipLaunchKernelGGL((dma_probe_kernel<NW_, INF_, MODE_>), dim3(blocks), dim3(NW_ * 64), 128 * 1024, s,            \
                       (const half_t*)src, (long long)bytes, pieces, sink);                                         \
    return check_launch("probe_dma");                                                                               \
  }
  SDK_DP(4, 1, 0) SDK_DP(4, 2, 0) SDK_DP(4, 4, 0) SDK_DP(4, 6, 0)
  SDK_DP(8, 1, 0) SDK_DP(8, 2, 0) SDK_DP(8, 4, 0) SDK_DP(8, 6, 0)
  SDK_DP(16, 1, 0) SDK_DP(16, 2, 0) SDK_DP(16, 4, 0) SDK_DP(16, 6, 0)
  SDK_DP(8, 2, 1) SDK_DP(8, 4, 1) SDK_DP(16, 2, 1) SDK_DP(16, 4, 1)
#undef SDK_DP
  return fail(SDK_EINVAL, "probe_dma: unsupported (nw, inflight, mode)");
}

// FLOPs of one launch of the MFMA probe (2*M*N*K per MFMA x MFMAs per wave x waves)
extern "C" double sdk_probe_mfma_flops(int32_t m16, int32_t blocks, int32_t iters) {
  const double per = m16 ? 2.0 * 16 * 16 * 32 * 8 : 2.0 * 32 * 32 * 16 * 4;
  return per * (double)iters * (double)blocks * 4.0;
}

// seed: >= 4096*8 random fp16 values; sink: >= blocks*4 floats
extern "C" int sdk_probe_mfma(int32_t m16, int32_t blocks, int32_t iters, const void* seed, float* sink,
                              sdk_stream_t stream) {
  if (!seed || !sink || blocks <= 0 || iters <= 0) return fail(SDK_EINVAL, "probe_mfma: bad arguments");
  if (m16)
    hipLaunchKernelGGL(mfma_probe_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const half_t*)seed, iters, sink);
  else
    hipLaunchKernelGGL(mfma_probe_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const half_t*)seed, iters, sink);
  return check_launch("probe_mfma");
}

// mode: bit 0 = 8 loads in flight per thread (else 4), bit 1 = non-temporal, bits 2-7 = workgroups per CU (0: 16);
// bit 8: the flat one-pass form (bits 2-7 ignored: the grid covers the buffer)
extern "C" int sdk_probe_copy_ex(const void* src, void* dst, int64_t bytes, int32_t mode, sdk_stream_t stream) {
  if (!src || !dst || bytes <= 0 || bytes % 16 || mode < 0) return fail(SDK_EINVAL, "probe_copy: bad arguments");
  const int64_t n = bytes / 16;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int per_cu = (mode >> 2) & 63 ? (mode >> 2) & 63 : 16;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, (int64_t)cus * per_cu);
  const hipStream_t s = (hipStream_t)stream;
  if (mode & 256) {
    const int u = (mode & 1) ? 8 : 4;
    const int64_t fb = (n + 256 * u - 1) / (256 * u);
    if (fb > 0x7fffffffLL) return fail(SDK_EINVAL, "probe_copy: buffer too large for the flat form");
    switch (mode & 3) {
      case 0: hipLaunchKernelGGL((copy_flat_kernel<4, false>), dim3((unsigned)fb), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
      case 1: hipLaunchKernelGGL((copy_flat_kernel<8, false>), dim3((unsigned)fb), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
      case 2: hipLaunchKernelGGL((copy_flat_kernel<4, true>), dim3((unsigned)fb), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
      default: hipLaunchKernelGGL((copy_flat_kernel<8, true>), dim3((unsigned)fb), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
    }
    return check_launch("probe_copy");
  }
  switch (mode & 3) {
    case 0: hipLaunchKernelGGL((copy_probe_kernel<4, false>), dim3(blocks), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
    case 1: hipLaunchKernelGGL((copy_probe_kernel<8, false>), dim3(blocks), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
    case 2: hipLaunchKernelGGL((copy_probe_kernel<4, true>), dim3(blocks), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
    default: hipLaunchKernelGGL((copy_probe_kernel<8, true>), dim3(blocks), dim3(256), 0, s, (const h8*)src, (h8*)dst, n); break;
  }
  return check_launch("probe_copy");
}

extern "C" int sdk_probe_copy(const void* src, void* dst, int64_t bytes, sdk_stream_t stream) {
  return sdk_probe_copy_ex(src, dst, bytes, 0, stream);
}
