// Fused GEGLU feed-forward of the 320-channel transformer blocks (SD-1's 64x64 level, 65,536 tokens
// at B = 16):
//   out = res + W2 (a * gelu(g)) + b2,   [a | g] = t W1^T + b1
// (reference openai_model/attention.py:129-172, GEGLU -> Dropout -> Linear, called as
// x = self.ff(self.norm3(x)) + x at :253).  Two GEMMs and the GEGLU in ONE kernel: the 4C-wide
// intermediate (168 MB per launch at the bench shape) never leaves the chip.
//
// Workgroup = 128 tokens, 8 waves = 4 pairs; waves w and w + 4 (one SIMD) own the same 32 tokens.
//  * Each wave holds its 32 t rows for the whole kernel as the B operand of v_mfma_f32_32x32x16_f16
//    (20 K-steps x 8 halfs = 80 VGPRs) and HALF of the transposed output tile: wave w + 4h owns
//    channels [160 h, 160 h + 160) of OUT^T (5 accumulators, 80 registers) — 2 waves per SIMD, so
//    one wave's GEGLU / LDS work issues under the other's MFMAs.
//  * The GEGLU features are walked in blocks of 16, two blocks per iteration: wave w + 4h computes
//    block 2i + h.  A block's 32 W1 rows (the 16 'a' rows of the features, then the same features'
//    16 'g' rows) give S^T = W1_blk t^T (20 MFMAs); in the 32x32 accumulator lane l holds token l%32
//    and rows 8(i/4) + 4(l/32) + i%4, so a[f] (register i) and g[f] (register i + 8) of one feature
//    sit in the same lane and h = a gelu(g) is formed in place (b1 seeds the accumulator).
//  * The 8 fp16 h values of a lane are directly the B operand (K = 16 features) of
//    OUT^T += W2_blk h^T: W2's columns are packed in the accumulator's feature order (slot
//    8(l/32) + j <-> feature 8(j/4) + 4(l/32) + j%4).  The pair swaps its h through LDS (1 KiB per
//    wave, same lane layout), then each wave applies both blocks to its channel half (10 MFMAs).
//  * b2 and the residual are added in the epilogue, which stages the tile through LDS for 16-B row
//    stores (the same fp16 rounding points as the two-GEMM path: h, acc + b2, then + res).
//  * W1 | W2 | b1 of a block are pre-packed (sdk_ff_pack) as the exact LDS image of its half of a
//    ring stage (W1 as 5 swizzled [32][64] sub-tiles, W2 as [2][320][8], b1 [32]) and streamed by
//    buffer_load ... lds (LDS-DMA, 1-KiB wave pieces, 8 per wave) one iteration ahead.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace sdk {
namespace {

constexpr int FFC = 320;                         // model channels
constexpr int FF_KS = FFC / 16;                  // 20 K-steps of the first GEMM
constexpr int FF_OB = FFC / 32;                  // 10 output blocks of 32 channels
constexpr int FF_OBH = FF_OB / 2;                // 5 per wave (channel half)
constexpr int FF_W1 = 32 * FFC * 2;              // 20480 B: 32 W1 rows
constexpr int FF_W2 = 2 * FFC * 16;              // 10240 B: 320 W2 rows x 16 (permuted) features
constexpr int FF_B1 = 32 * 4;                    // 128 B: the 32 rows' b1
constexpr int FF_BLK = FF_W1 + FF_W2 + FF_B1;    // 30848 B packed per feature block
constexpr int FF_BSL = FF_W1 + FF_W2 + 1024;     // LDS bytes per block (the b1 piece lands a full KiB)
constexpr int FF_BPC = (FF_W1 + FF_W2) / 1024 + 1;      // 31 one-KiB DMA pieces per block
constexpr int FF_SLOT = 2 * FF_BSL;              // a stage = two blocks
constexpr int FF_PIECES = 2 * FF_BPC;            // 62
constexpr int FF_NW = 8, FF_NT = FF_NW * 64, FF_ROWS = 128;
constexpr int FF_GPW = (FF_PIECES + FF_NW - 1) / FF_NW; // 8 per wave (two dummies): exact vmcnt immediates
constexpr int FF_NS = 2;                         // ring stages
constexpr int FF_XB = FF_NS * FF_SLOT;           // h exchange: 1 KiB per wave
constexpr int FF_LDS = FF_XB + FF_NW * 1024 + 1024;     // + the dummy pieces' slot = 136,192 B
constexpr int FF_ORS = FFC + 8;                  // epilogue staging row stride (halfs)
constexpr unsigned FF_OOB = 0x80000000u;         // past the buffer range: the DMA loads zeros
static_assert(FF_ROWS * FF_ORS * 2 <= FF_NS * FF_SLOT, "epilogue staging fits the ring");
static_assert(FF_LDS <= 160 * 1024, "LDS");

struct FfParams {
  const half_t* t;
  const half_t* res;
  half_t* out;
  const char* w;
  const float* b2;
  int t_ld, res_ld, out_ld;
  int M, nfb;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ff_rsrc(const void* base, long long bytes) {
  const int n = (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

__device__ __forceinline__ void ff_dma(__amdgpu_buffer_rsrc_t r, char* dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0, 0);
}

// DBG (diagnostics build only, SDK_FF_DBG): bit 0 = no weight DMAs, bit 1 = no MFMAs, bit 2 = no GEGLU
// math (h = a) — wrong results by design, for locating the bound
template <int DBG>
__global__ void __launch_bounds__(FF_NT, 1) ff_geglu_kernel(FfParams p) {
  extern __shared__ __attribute__((aligned(16))) char ffl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pr = wave & 3, half = wave >> 2;
  const int fr = lane & 31, hh = lane >> 5;
  const int m0 = blockIdx.x * FF_ROWS;
  const __amdgpu_buffer_rsrc_t rw = ff_rsrc(p.w, (long long)p.nfb * FF_BLK);

  // this wave's pieces of a stage: piece j*8 + wave of the pair's 62 (block = piece / 31); wave-uniform
  // source / LDS offsets (SGPRs) + the lane's 16 B, selected branch-free (2 VGPRs of addressing)
  const unsigned lane16 = (unsigned)lane * 16u;
  const unsigned lane16_b1 = lane < 8 ? lane16 : FF_OOB;   // b1 piece: 128 B, lanes 8.. load zeros
  unsigned soff[FF_GPW];
  int doff[FF_GPW];
  unsigned b1mask = 0;
#pragma unroll
  for (int j = 0; j < FF_GPW; ++j) {
    const int piece = j * FF_NW + wave;
    const int blk = piece / FF_BPC, q = piece - blk * FF_BPC;
    const bool dummy = piece >= FF_PIECES, b1p = !dummy && q == FF_BPC - 1;
    soff[j] = dummy ? FF_OOB : (unsigned)(blk * FF_BLK + (b1p ? FF_W1 + FF_W2 : q * 1024));
    doff[j] = dummy ? FF_LDS - 1024 : blk * FF_BSL + (b1p ? FF_W1 + FF_W2 : q * 1024);
    b1mask |= (b1p ? 1u : 0u) << j;
  }
  auto issue = [&](int it, int slot) __attribute__((always_inline)) {
    if constexpr ((DBG & 1) != 0) return;
    const unsigned base = 2 * it < p.nfb ? (unsigned)(2 * it) * FF_BLK : FF_OOB;
#pragma unroll
    for (int j = 0; j < FF_GPW; ++j) {
      const bool dummy = doff[j] == FF_LDS - 1024;
      char* d = ffl + (dummy ? 0 : slot * FF_SLOT) + doff[j];
      ff_dma(rw, d, base + soff[j] + (((b1mask >> j) & 1u) ? lane16_b1 : lane16));
    }
  };

  // t rows of this pair (B operand: lane = token fr, channels 16 ks + 8 hh .. + 7); issued before the
  // first stage's DMAs, so its vmcnt wait covers them
  h8 tq[FF_KS];
  {
    const int tok = min(m0 + pr * 32 + fr, p.M - 1);
    const half_t* tp = p.t + (size_t)tok * p.t_ld + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < FF_KS; ++ks) tq[ks] = *reinterpret_cast<const h8*>(tp + 16 * ks);
  }
  issue(0, 0);

  const int sw = (fr >> 1) & 7;              // W1 sub-tile swizzle of row fr
  f16v o[FF_OBH];
#pragma unroll
  for (int ob = 0; ob < FF_OBH; ++ob) o[ob] = f16v{};
  const int niter = p.nfb / 2;
  h8* xb_own = reinterpret_cast<h8*>(ffl + FF_XB + wave * 1024) + lane;
  const h8* xb_par = reinterpret_cast<const h8*>(ffl + FF_XB + (wave ^ 4) * 1024) + lane;
  for (int it = 0; it < niter; ++it) {
    const int slot = it & 1;
    // stage `it` landed in this wave; after the barrier in every wave, and every wave is done with
    // iteration it - 1 (stage it - 1's slot is free, and the exchange slots were read)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(it + 1, slot ^ 1);
    // first GEMM of this wave's block (2 it + half)
    const char* st = ffl + slot * FF_SLOT + half * FF_BSL;
    const float* b1 = reinterpret_cast<const float*>(st + FF_W1 + FF_W2);
    f16v s;
    {
      const f4 q0 = *reinterpret_cast<const f4*>(b1 + 4 * hh), q1 = *reinterpret_cast<const f4*>(b1 + 8 + 4 * hh);
      const f4 q2 = *reinterpret_cast<const f4*>(b1 + 16 + 4 * hh), q3 = *reinterpret_cast<const f4*>(b1 + 24 + 4 * hh);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s[q] = q0[q];
        s[4 + q] = q1[q];
        s[8 + q] = q2[q];
        s[12 + q] = q3[q];
      }
    }
    auto w1frag = [&](int ks) __attribute__((always_inline)) {
      const int c = 2 * (ks & 3) + hh;
      return *reinterpret_cast<const h8*>(st + (ks >> 2) * 4096 + fr * 128 + ((c ^ sw) << 4));
    };
    constexpr int LA = 4;                    // fragment reads run LA K-steps ahead of their MFMA
    h8 wa[FF_KS];
#pragma unroll
    for (int j = 0; j < LA; ++j) wa[j] = w1frag(j);
#pragma unroll
    for (int ks = 0; ks < FF_KS; ++ks) {
      if (ks + LA < FF_KS) wa[ks + LA] = w1frag(ks + LA);
      if constexpr ((DBG & 2) == 0) s = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[ks], tq[ks], s, 0, 0, 0);
      else s[ks & 15] += (float)wa[ks][0];
    }
    __builtin_amdgcn_sched_group_barrier(0x100, LA + 4, 0);
#pragma unroll
    for (int i = 0; i < FF_KS; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    h8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr ((DBG & 4) != 0) h[j] = (half_t)s[j];
      else h[j] = (half_t)(s[j] * gelu_erf(s[j + 8]));
    }
    *xb_own = h;
    __syncthreads();                         // the pair's h visible
    const h8 hp = *xb_par;
    const h8 he = half ? hp : h, ho = half ? h : hp;   // blocks 2 it, 2 it + 1
    const char* w2e = ffl + slot * FF_SLOT + FF_W1 + (hh * FFC + half * 160 + fr) * 16;
    const char* w2o = w2e + FF_BSL;
#pragma unroll
    for (int ob = 0; ob < FF_OBH; ++ob) {
      const h8 ae = *reinterpret_cast<const h8*>(w2e + ob * 32 * 16);
      const h8 ao = *reinterpret_cast<const h8*>(w2o + ob * 32 * 16);
      if constexpr ((DBG & 2) == 0) {
        o[ob] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ae, he, o[ob], 0, 0, 0);
        o[ob] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ao, ho, o[ob], 0, 0, 0);
      } else {
        o[ob][ob] += (float)ae[0] + (float)ao[0] + (float)he[ob & 7] + (float)ho[ob & 7];
      }
    }
  }

  // epilogue: (acc + b2) as fp16 rows in LDS (the ring is idle once the trailing pieces land), then
  // 16-B row stores with the residual
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  half_t* os = reinterpret_cast<half_t*>(ffl);
  const int trow = pr * 32 + fr;
#pragma unroll
  for (int ob = 0; ob < FF_OBH; ++ob)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = half * 160 + ob * 32 + 8 * g + 4 * hh;
      const f4 bb = p.b2 ? *reinterpret_cast<const f4*>(p.b2 + ch) : f4{0.f, 0.f, 0.f, 0.f};
      h4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = (half_t)(o[ob][4 * g + q] + bb[q]);
      *reinterpret_cast<h4*>(os + trow * FF_ORS + ch) = v;
    }
  __syncthreads();
  constexpr int CPR = FFC / 8;               // 16-B chunks per row
  for (int e = tid; e < FF_ROWS * CPR; e += FF_NT) {
    const int r = e / CPR, c8 = e - r * CPR;
    const int m = m0 + r;
    if (m >= p.M) break;                     // rows ascend with e
    h8 v = *reinterpret_cast<const h8*>(os + r * FF_ORS + c8 * 8);
    if (p.res) {
      const h8 rr = *reinterpret_cast<const h8*>(p.res + (size_t)m * p.res_ld + c8 * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = (half_t)((float)v[q] + (float)rr[q]);
    }
    *reinterpret_cast<h8*>(p.out + (size_t)m * p.out_ld + c8 * 8) = v;
  }
}

// One thread per 16-B chunk of the packed blob (layout: see ff_geglu_kernel and sdk_amd.h).
__global__ void __launch_bounds__(256) ff_pack_kernel(const half_t* __restrict__ w1, const float* __restrict__ b1,
                                                      const half_t* __restrict__ w2, char* __restrict__ out, int F,
                                                      int nfb) {
  constexpr int CPB = FF_BLK / 16;   // 1928 chunks per block
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long long)nfb * CPB) return;
  const int fb = (int)(q / CPB), e = (int)(q - (long long)fb * CPB);
  char* dst = out + (size_t)fb * FF_BLK + (size_t)e * 16;
  auto w1row = [&](int r) { return r < 16 ? 16 * fb + r : F + 16 * fb + (r - 16); };
  if (e < FF_W1 / 16) {
    const int u = e / 256, rem = e - u * 256, r = rem / 8, cpos = rem - r * 8;
    const int c = cpos ^ ((r >> 1) & 7);
    *reinterpret_cast<h8*>(dst) = *reinterpret_cast<const h8*>(w1 + (size_t)w1row(r) * FFC + 64 * u + 8 * c);
  } else if (e < (FF_W1 + FF_W2) / 16) {
    const int x = e - FF_W1 / 16, hv = x / FFC, o = x - hv * FFC;
    h8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = w2[(size_t)o * F + 16 * fb + 8 * (j >> 2) + 4 * hv + (j & 3)];
    *reinterpret_cast<h8*>(dst) = v;
  } else {
    const int r0 = (e - (FF_W1 + FF_W2) / 16) * 4;
    f4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = b1 ? b1[w1row(r0 + i)] : 0.f;
    *reinterpret_cast<f4*>(dst) = v;
  }
}

template <int DBG>
int ff_launch(const FfParams& p, unsigned blocks, hipStream_t s) {
  static std::atomic<unsigned long long> lds_done{0};
  const int rc = ensure_dyn_lds((const void*)ff_geglu_kernel<DBG>, FF_LDS, lds_done, "feed_forward");
  if (rc != SDK_OK) return rc;
  hipLaunchKernelGGL(ff_geglu_kernel<DBG>, dim3(blocks), dim3(FF_NT), FF_LDS, s, p);
  return check_launch("feed_forward");
}

int ff_launch_dbg(const FfParams& p, unsigned blocks, int dbg, hipStream_t s) {
#if defined(SDK_CONV_DIAGNOSTICS)
  switch (dbg) {
    case 1: return ff_launch<1>(p, blocks, s);
    case 2: return ff_launch<2>(p, blocks, s);
    case 3: return ff_launch<3>(p, blocks, s);
    case 4: return ff_launch<4>(p, blocks, s);
    case 5: return ff_launch<5>(p, blocks, s);
    default: break;
  }
#endif
  (void)dbg;
  return ff_launch<0>(p, blocks, s);
}

bool ff_shape_ok(int channels, int features) { return channels == FFC && features > 0 && features % 32 == 0; }

}  // namespace
}  // namespace sdk

using namespace sdk;

extern "C" int sdk_ff_supported(int32_t channels, int32_t features) { return ff_shape_ok(channels, features) ? 1 : 0; }

extern "C" int64_t sdk_ff_packed_bytes(int32_t channels, int32_t features) {
  return ff_shape_ok(channels, features) ? (int64_t)(features / 16) * FF_BLK : -1;
}

extern "C" int sdk_ff_pack(const void* w1, const float* b1, const void* w2, void* packed, int32_t channels,
                           int32_t features, sdk_stream_t stream) {
  if (!w1 || !w2 || !packed) return fail(SDK_EINVAL, "ff_pack: null pointer");
  if (!ff_shape_ok(channels, features)) return fail(SDK_EINVAL, "ff_pack: channels must be 320, features a multiple of 32");
  if (((uintptr_t)w1 | (uintptr_t)packed) & 15) return fail(SDK_EINVAL, "ff_pack: w1 / packed must be 16-B aligned");
  const int nfb = features / 16;
  const long long chunks = (long long)nfb * (FF_BLK / 16);
  hipLaunchKernelGGL(ff_pack_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const half_t*)w1, b1, (const half_t*)w2, (char*)packed, (int)features, nfb);
  return check_launch("ff_pack");
}

extern "C" int sdk_feed_forward(const sdk_ff_args* a, sdk_stream_t stream) {
  if (!a || !a->t || !a->out || !a->packed) return fail(SDK_EINVAL, "feed_forward: null pointer");
  if (!ff_shape_ok(a->channels, a->features))
    return fail(SDK_EINVAL, "feed_forward: channels must be 320, features a multiple of 32");
  if (a->rows <= 0) return fail(SDK_EINVAL, "feed_forward: empty");
  if (a->t_ld % 8 || a->out_ld % 8 || (a->res && a->res_ld % 8) || a->t_ld < a->channels || a->out_ld < a->channels)
    return fail(SDK_EINVAL, "feed_forward: row strides must be multiples of 8 and >= channels");
  if (((uintptr_t)a->t | (uintptr_t)a->out | (uintptr_t)a->res | (uintptr_t)a->packed | (uintptr_t)a->b2) & 15)
    return fail(SDK_EINVAL, "feed_forward: pointers must be 16-B aligned");
  if ((long long)(a->features / 16) * FF_BLK >= 0x7fffffffLL) return fail(SDK_EINVAL, "feed_forward: too many features");
  FfParams p{(const half_t*)a->t, (const half_t*)a->res, (half_t*)a->out, (const char*)a->packed, a->b2,
             a->t_ld, a->res_ld, a->out_ld, a->rows, a->features / 16};
  const unsigned blocks = (unsigned)((a->rows + FF_ROWS - 1) / FF_ROWS);
#if defined(SDK_CONV_DIAGNOSTICS)
  static const int dbg = getenv("SDK_FF_DBG") ? atoi(getenv("SDK_FF_DBG")) & 7 : 0;
#else
  constexpr int dbg = 0;
#endif
  return ff_launch_dbg(p, blocks, dbg, (hipStream_t)stream);
}
