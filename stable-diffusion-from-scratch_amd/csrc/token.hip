// Token linear of the 320-channel transformer blocks (SD-1's 64x64 level, 65,536 tokens at B = 16):
//   out = [res +] (x W^T + b),   x [rows, 320] fp16, W [320][320] (nn.Linear layout)
// — the SpatialTransformer's proj_in (reference openai_model/attention.py:293-300, a 1x1 conv over the
// GroupNorm output) and the self-attention's to_out + residual (:203-206, x = attn1(norm1(x)) + x at :251).
//
// Why a kernel of its own: K = 320 gives the tiled conv kernels five K-steps per tile, so every tile is a
// serial fill -> 5 K-steps -> store tail and each one re-streams the whole 200 KB weight into LDS
// (profiles/r2_gemm_cost_model.txt: 30.6 us without / 46 us with the residual, about 2x the HBM time).
// At 32 tokens x 320 channels a block is 6.6 MFLOP against 61 KB of HBM traffic (x, residual, out):
// the kernel is HBM-bound, and what it needs is enough bytes in flight per CU.  So:
//  * W lives in REGISTERS for the whole kernel, the grid is persistent (one workgroup per CU): 4 waves
//    (one per SIMD, 512-register budget); wave w owns output channels [80 w, 80 w + 80) and holds their
//    W rows as the A operand of v_mfma_f32_16x16x32_f16 (5 channel blocks x 10 K-steps x 8 halfs = 200
//    registers), loaded once per workgroup (51 MB of L2 reads chip-wide, no HBM re-reads);
//  * a workgroup walks 32-token blocks grid-stride; each block's x rows (and residual rows) go HBM -> LDS
//    by buffer_load ... lds (LDS-DMA: no register staging) into a 3-stage ring, TWO blocks ahead of the
//    one being computed (~80 KB in flight per CU), with counted vmcnt waits and raw barriers (the stores
//    of earlier blocks stay in flight across them);
//  * an LDS tile row is the 640-B token row with its 16-B chunks XOR-swizzled inside groups of 8
//    (chunk c of row r at c ^ (r & 7)): the DMA writes 1-KiB linear pieces, the b128 fragment reads of
//    16 rows hit 8 distinct bank quads per phase;
//  * D^T = W X^T: lane l of a 16x16 accumulator holds token l % 16 and 4 consecutive channels; the fp32
//    accumulators + bias are rounded to fp16 into an output tile, then every thread stores whole 16-B
//    row chunks (+ the residual chunk from the ring) — the conv epilogue's rounding points (acc + b ->
//    fp16, then + res -> fp16).
//  * LN = true (sdk_token_linear_ln): the finished rows go back into that tile and two waves apply a
//    LayerNorm to them with the row math of layer_norm_quad_kernel (common.h ln_quad_stats /
//    ln_quad_apply: the same bits), written as a second output — the SpatialTransformer's proj_in
//    emits the first block's norm1 input AND output, so the 64x64 level has no LayerNorm launch
//    (attention.py:251: x = attn1(norm1(x)) + x right after proj_in at :330).
#include "common.h"

namespace sdk {
namespace {

constexpr int TLC = 320;                 // channels (in = out)
constexpr int TL_KS = TLC / 32;          // 10 K-steps of v_mfma_f32_16x16x32_f16
constexpr int TL_NB = 5;                 // 16-channel blocks per wave (80 channels)
constexpr int TL_ROWS = 32;              // tokens per block
constexpr int TL_RB = TLC * 2;           // bytes per token row in a ring tile (640, swizzled, no pad)
constexpr int TL_TILE = TL_ROWS * TL_RB; // 20480 B = 20 one-KiB DMA pieces
constexpr int TL_PPW = TL_TILE / 1024 / 4;   // pieces per wave per tile (5)
constexpr int TL_NS = 3;                 // ring stages (compute block b while b+1, b+2 land)
constexpr int TL_OLD = TLC + 8;          // output tile row stride (halfs) = 656 B
constexpr int TL_CPR = TLC / 8;          // 16-B chunks per row (40)
constexpr int TL_CPT = TL_ROWS * TL_CPR / 256;   // chunks per thread per block (5)
constexpr int TL_TG = TL_ROWS / 16;      // 16-token groups per block
static_assert(TL_ROWS * TL_CPR % 256 == 0 && TL_TILE % 4096 == 0, "whole chunks / pieces per thread / wave");

struct TokenLn {
  const float* gamma; const float* beta; float eps;
  half_t* out; int out_ld;
};

// position of 16-B chunk c of ring-tile row r (XOR inside groups of 8 chunks; an involution)
__device__ __forceinline__ int tl_swz(int r, int c) { return (c & ~7) | ((c & 7) ^ (r & 7)); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tl_rsrc(const void* base, long long bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

template <bool LN, bool RES>
__global__ void __launch_bounds__(256, 1) token_linear320_kernel(const half_t* __restrict__ x, int x_ld,
                                                                 const half_t* __restrict__ w,
                                                                 const float* __restrict__ bias, const half_t* res,
                                                                 int res_ld, half_t* out, int out_ld, int rows,
                                                                 TokenLn ln) {
  extern __shared__ __attribute__((aligned(16))) char tl_lds[];
  constexpr int STAGE = (RES ? 2 : 1) * TL_TILE;
  char* ring = tl_lds;                                                       // TL_NS x {x tile, res tile}
  half_t* os = reinterpret_cast<half_t*>(tl_lds + TL_NS * STAGE);           // [32][656 B]
  float* gb = reinterpret_cast<float*>(tl_lds + TL_NS * STAGE + TL_ROWS * TL_OLD * 2);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int nblk = (rows + TL_ROWS - 1) / TL_ROWS;
  const int G = (int)gridDim.x;
  if constexpr (LN) {   // gamma | beta for ln_quad_apply; the first block's barrier orders these writes
    if (t < TLC / 4) {
      *reinterpret_cast<f4*>(gb + 4 * t) = *reinterpret_cast<const f4*>(ln.gamma + 4 * t);
      *reinterpret_cast<f4*>(gb + TLC + 4 * t) = *reinterpret_cast<const f4*>(ln.beta + 4 * t);
    }
  }

  // this lane's DMA sources: piece j*4 + wave of a tile covers linear bytes [1 KiB piece, + lane*16):
  // ring row rr, chunk position c, holding global chunk tl_swz(rr, c) of token row rr
  unsigned xoff[TL_PPW], roff[TL_PPW];
#pragma unroll
  for (int j = 0; j < TL_PPW; ++j) {
    const int o = (j * 4 + wave) * 1024 + lane * 16;
    const int rr = o / TL_RB, c = (o - rr * TL_RB) / 16;
    const int gch = tl_swz(rr, c);
    xoff[j] = (unsigned)((rr * x_ld + gch * 8) * 2);
    roff[j] = RES ? (unsigned)((rr * res_ld + gch * 8) * 2) : 0u;
  }
  // DMA of block `blk` into ring stage `st`; a block past the end loads zeros (range check of a
  // zero-size resource), so every wave issues the same count every time (exact vmcnt immediates)
  auto dma = [&](int blk, int st) __attribute__((always_inline)) {
    const long long r0 = (long long)blk * TL_ROWS;
    const long long left = blk < nblk ? rows - r0 : 0;
    const __amdgpu_buffer_rsrc_t rx = tl_rsrc(x + (blk < nblk ? r0 * x_ld : 0), left * x_ld * 2);
    char* dst = ring + st * STAGE;
#pragma unroll
    for (int j = 0; j < TL_PPW; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(dst + (j * 4 + wave) * 1024),
                                               16, xoff[j], 0, 0, 0);
    if constexpr (RES) {
      const __amdgpu_buffer_rsrc_t rs = tl_rsrc(res + (blk < nblk ? r0 * res_ld : 0), left * res_ld * 2);
#pragma unroll
      for (int j = 0; j < TL_PPW; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(dst + TL_TILE + (j * 4 + wave) * 1024), 16, roff[j], 0, 0, 0);
    }
  };
  int b = blockIdx.x;
  dma(b, 0);
  dma(b + G, 1);

  // W rows of this wave's channels: A operand rows = channel 80 w + 16 nb + r16, k = 32 ks + 8 kq + [0, 8)
  h8 wf[TL_NB][TL_KS];
#pragma unroll
  for (int nb = 0; nb < TL_NB; ++nb)
#pragma unroll
    for (int ks = 0; ks < TL_KS; ++ks)
      wf[nb][ks] = *reinterpret_cast<const h8*>(w + (size_t)(80 * wave + 16 * nb + r16) * TLC + 32 * ks + 8 * kq);
  f4 bv[TL_NB];
#pragma unroll
  for (int nb = 0; nb < TL_NB; ++nb)
    bv[nb] = bias ? *reinterpret_cast<const f4*>(bias + 80 * wave + 16 * nb + 4 * kq) : f4{};
  // this thread's output chunks of a block: row crow, channels ccol .. ccol + 7
  int crow[TL_CPT], ccol[TL_CPT];
#pragma unroll
  for (int i = 0; i < TL_CPT; ++i) {
    const int idx = t + 256 * i;
    crow[i] = idx / TL_CPR;
    ccol[i] = (idx - crow[i] * TL_CPR) * 8;
  }
  // vm ops a wave issues per block after its DMA: D pieces, then S stores (+ the LN rows of waves 0 / 1)
  constexpr int D = (RES ? 2 : 1) * TL_PPW;
  const bool ln_wave = LN && wave < TL_ROWS / 16;

  for (int it = 0; b < nblk; b += G, ++it) {
    const int st = it % TL_NS;
    // block b's pieces have landed in this wave (the ops issued after them may stay in flight), then in all
    if (it == 0) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
    } else if (it == 1) {
      if (ln_wave) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D + TL_CPT + (LN ? TLC / 32 : 0)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D + TL_CPT) : "memory");
    } else {
      if (ln_wave) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D + 2 * (TL_CPT + (LN ? TLC / 32 : 0))) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D + 2 * TL_CPT) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    // every wave is past block b - 1 (its stage and the output tile are free): block b + 2 -> that stage
    dma(b + 2 * G, (it + 2) % TL_NS);

    const char* xs = ring + st * STAGE;
    f4 acc[TL_TG][TL_NB];
#pragma unroll
    for (int tg = 0; tg < TL_TG; ++tg)
#pragma unroll
      for (int nb = 0; nb < TL_NB; ++nb) acc[tg][nb] = f4{};
    // all 20 B fragments of the block issued at once (80 registers): one LDS latency per block
    h8 xf[TL_KS][TL_TG];
#pragma unroll
    for (int ks = 0; ks < TL_KS; ++ks)
#pragma unroll
      for (int tg = 0; tg < TL_TG; ++tg) {
        const int rr = tg * 16 + r16;
        xf[ks][tg] = *reinterpret_cast<const h8*>(xs + rr * TL_RB + tl_swz(rr, 4 * ks + kq) * 16);
      }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead (the scheduler would sink each next to its MFMA)
#pragma unroll
    for (int ks = 0; ks < TL_KS; ++ks)
#pragma unroll
      for (int tg = 0; tg < TL_TG; ++tg)
#pragma unroll
        for (int nb = 0; nb < TL_NB; ++nb)
          acc[tg][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nb][ks], xf[ks][tg], acc[tg][nb], 0, 0, 0);
    // acc[tg][nb] lane l: token tg*16 + r16, channels 80 w + 16 nb + 4 kq + q
#pragma unroll
    for (int tg = 0; tg < TL_TG; ++tg)
#pragma unroll
      for (int nb = 0; nb < TL_NB; ++nb) {
        h4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (half_t)(acc[tg][nb][q] + bv[nb][q]);
        *reinterpret_cast<h4*>(os + (tg * 16 + r16) * TL_OLD + 80 * wave + 16 * nb + 4 * kq) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int r0 = b * TL_ROWS;
#pragma unroll
    for (int i = 0; i < TL_CPT; ++i) {
      const int row = r0 + crow[i];
      h8 v = *reinterpret_cast<const h8*>(os + crow[i] * TL_OLD + ccol[i]);
      if constexpr (RES) {
        const h8 rr = *reinterpret_cast<const h8*>(xs + TL_TILE + crow[i] * TL_RB + tl_swz(crow[i], ccol[i] / 8) * 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] + (float)rr[j]);
      }
      if (row < rows) *reinterpret_cast<h8*>(out + (size_t)row * out_ld + ccol[i]) = v;
      if constexpr (LN) *reinterpret_cast<h8*>(os + crow[i] * TL_OLD + ccol[i]) = v;
    }
    if constexpr (LN) {
      // waves 0 / 1: rows [16 wave, 16 wave + 16) of the block, four lanes per row (lane q holds chunks
      // q + 4 i); the next block's output-tile writes come after its first barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (ln_wave) {
        constexpr int CPL = TLC / 32;
        const int q = lane & 3, r = 16 * wave + (lane >> 2), row = r0 + r;
        h8 v[CPL];
#pragma unroll
        for (int i = 0; i < CPL; ++i) v[i] = *reinterpret_cast<const h8*>(os + r * TL_OLD + 8 * (q + 4 * i));
        float mean, rstd;
        ln_quad_stats<CPL>(v, ln.eps, mean, rstd);
        if (row < rows) {
          half_t* yr = ln.out + (size_t)row * ln.out_ld + 8 * q;
#pragma unroll
          for (int i = 0; i < CPL; ++i)
            *reinterpret_cast<h8*>(yr + 32 * i) = ln_quad_apply(v[i], mean, rstd, gb, TLC, q + 4 * i);
        }
      }
    }
  }
  // the trailing DMAs (zeros or blocks of no one) must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool LN, bool RES>
int token_linear_launch2(const sdk_token_linear_args* a, const TokenLn& ln, hipStream_t s) {
  constexpr int LDS = TL_NS * (RES ? 2 : 1) * TL_TILE + TL_ROWS * TL_OLD * 2 + (LN ? 2 * TLC * 4 : 0);
  static_assert(LDS <= 160 * 1024, "LDS");
  static std::atomic<unsigned long long> attr{0};
  if (int e = ensure_dyn_lds((const void*)token_linear320_kernel<LN, RES>, LDS, attr, "token_linear")) return e;
  const int nblk = (a->rows + TL_ROWS - 1) / TL_ROWS;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const unsigned grid = (unsigned)(nblk < cus ? nblk : cus);
  hipLaunchKernelGGL((token_linear320_kernel<LN, RES>), dim3(grid), dim3(256), LDS, s, (const half_t*)a->x, a->x_ld,
                     (const half_t*)a->w, a->bias, (const half_t*)a->res, a->res_ld, (half_t*)a->out, a->out_ld,
                     a->rows, ln);
  return check_launch(LN ? "token_linear_ln" : "token_linear");
}

template <bool LN>
int token_linear_launch(const sdk_token_linear_args* a, const TokenLn& ln, hipStream_t s) {
  return a->res ? token_linear_launch2<LN, true>(a, ln, s) : token_linear_launch2<LN, false>(a, ln, s);
}

int token_linear_check(const sdk_token_linear_args* a) {
  if (!a || !a->x || !a->w || !a->out) return fail(SDK_EINVAL, "token_linear: null pointer");
  if (a->in_features != TLC || a->out_features != TLC)
    return fail(SDK_EINVAL, "token_linear: in_features and out_features must be 320");
  if (a->rows <= 0) return fail(SDK_EINVAL, "token_linear: empty");
  if (a->x_ld % 8 || a->out_ld % 8 || (a->res && a->res_ld % 8) || a->x_ld < TLC || a->out_ld < TLC ||
      (a->res && a->res_ld < TLC))
    return fail(SDK_EINVAL, "token_linear: row strides must be multiples of 8 and >= 320");
  if (((uintptr_t)a->x | (uintptr_t)a->w | (uintptr_t)a->out | (uintptr_t)a->res | (uintptr_t)a->bias) & 15)
    return fail(SDK_EINVAL, "token_linear: pointers must be 16-B aligned");
  // the x tile of a block is read by other threads than the ones storing its output: x must not alias out
  const char *x0 = (const char*)a->x, *o0 = (const char*)a->out;
  const long long xb = ((long long)(a->rows - 1) * a->x_ld + TLC) * 2, ob = ((long long)(a->rows - 1) * a->out_ld + TLC) * 2;
  if (x0 < o0 + ob && o0 < x0 + xb) return fail(SDK_EINVAL, "token_linear: x and out overlap");
  return SDK_OK;
}

}  // namespace
}  // namespace sdk

using namespace sdk;

extern "C" int sdk_token_linear_supported(int32_t in_features, int32_t out_features) {
  return in_features == TLC && out_features == TLC ? 1 : 0;
}

extern "C" int sdk_token_linear(const sdk_token_linear_args* a, sdk_stream_t stream) {
  if (int e = token_linear_check(a)) return e;
  return token_linear_launch<false>(a, TokenLn{}, (hipStream_t)stream);
}

extern "C" int sdk_token_linear_ln(const sdk_token_linear_args* a, const float* gamma, const float* beta, float eps,
                                   void* out_ln, int32_t out_ln_ld, sdk_stream_t stream) {
  if (int e = token_linear_check(a)) return e;
  if (!gamma || !beta || !out_ln) return fail(SDK_EINVAL, "token_linear_ln: null gamma / beta / out_ln");
  if (((uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)out_ln) & 15 || out_ln_ld % 8 || out_ln_ld < TLC)
    return fail(SDK_EINVAL, "token_linear_ln: gamma / beta / out_ln must be 16-B aligned, out_ln_ld % 8 == 0 and >= 320");
  // out_ln is written by the LN waves while other workgroups still read x / res / write out
  const char *x0 = (const char*)a->x, *l0 = (const char*)out_ln, *o0 = (const char*)a->out;
  const long long lb = ((long long)(a->rows - 1) * out_ln_ld + TLC) * 2;
  const long long xb = ((long long)(a->rows - 1) * a->x_ld + TLC) * 2, ob = ((long long)(a->rows - 1) * a->out_ld + TLC) * 2;
  if ((x0 < l0 + lb && l0 < x0 + xb) || (o0 < l0 + lb && l0 < o0 + ob) ||
      (a->res && (const char*)a->res < l0 + lb && l0 < (const char*)a->res + ((long long)(a->rows - 1) * a->res_ld + TLC) * 2))
    return fail(SDK_EINVAL, "token_linear_ln: out_ln overlaps x, res or out");
  return token_linear_launch<true>(a, TokenLn{gamma, beta, eps, (half_t*)out_ln, out_ln_ld}, (hipStream_t)stream);
}
