// Token linear of the 320-channel transformer blocks (SD-1's 64x64 level, 65,536 tokens at B = 16):
//   out = [res +] (x W^T + b),   x [rows, 320] fp16, W [320][320] (nn.Linear layout)
// — the SpatialTransformer's proj_in (reference openai_model/attention.py:293-300, a 1x1 conv over the
// GroupNorm output) and the self-attention's to_out + residual (:203-206, x = attn1(norm1(x)) + x at :251).
//
// Why a kernel of its own: K = 320 gives the tiled conv kernels five K-steps per tile, so every tile is a
// serial fill -> 5 K-steps -> store tail and each one re-streams the whole 200 KB weight into LDS
// (profiles/r2_gemm_cost_model.txt: 30.6 us without / 46 us with the residual, about 2x the HBM time).
// Here W lives in REGISTERS for the whole kernel and the grid is persistent:
//  * 4 waves (one per SIMD, 512-register budget); wave w owns output channels [80 w, 80 w + 80) and holds
//    their W rows as the A operand of v_mfma_f32_16x16x32_f16 (5 channel blocks x 10 K-steps x 8 halfs
//    = 200 registers), loaded once per workgroup (51 MB of L2 reads chip-wide, no HBM re-reads).
//  * A workgroup walks 32-token blocks grid-stride.  A block's x rows arrive by 16-B coalesced loads
//    one block AHEAD (in registers across the previous block's MFMAs / stores), are written to a padded
//    LDS tile (row stride 656 B: the 16 rows of one b128 read phase hit 16 distinct bank quads), and all
//    four waves read their B fragments from it (D^T = W X^T: lane l holds token l % 16, 4 channels).
//  * The fp32 accumulators + bias are rounded to fp16 into a second LDS tile, then every thread stores
//    whole 16-B row chunks (+ the residual, loaded before the MFMAs) — the conv epilogue's rounding
//    points (acc + b -> fp16, then + res -> fp16).
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
constexpr int TL_LD = TLC + 8;           // LDS row stride (halfs) = 656 B
constexpr int TL_CPR = TLC / 8;          // 16-B chunks per row (40)
constexpr int TL_CPT = TL_ROWS * TL_CPR / 256;   // chunks per thread per block (5)
constexpr int TL_TG = TL_ROWS / 16;     // 16-token groups per block
static_assert(TL_ROWS * TL_CPR % 256 == 0, "whole chunks per thread");

struct TokenLn {
  const float* gamma; const float* beta; float eps;
  half_t* out; int out_ld;
};

template <bool LN>
__global__ void __launch_bounds__(256, 1) token_linear320_kernel(const half_t* __restrict__ x, int x_ld,
                                                                 const half_t* __restrict__ w,
                                                                 const float* __restrict__ bias, const half_t* res,
                                                                 int res_ld, half_t* out, int out_ld, int rows,
                                                                 TokenLn ln) {
  __shared__ __attribute__((aligned(16))) half_t xs[TL_ROWS * TL_LD];
  __shared__ __attribute__((aligned(16))) half_t os[TL_ROWS * TL_LD];
  __shared__ __attribute__((aligned(16))) float gb[LN ? 2 * TLC : 4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if constexpr (LN) {   // gamma | beta for ln_quad_apply; the first block's barrier orders these writes
    if (t < TLC / 4) {
      *reinterpret_cast<f4*>(gb + 4 * t) = *reinterpret_cast<const f4*>(ln.gamma + 4 * t);
      *reinterpret_cast<f4*>(gb + TLC + 4 * t) = *reinterpret_cast<const f4*>(ln.beta + 4 * t);
    }
  }
  const int r16 = lane & 15, kq = lane >> 4;
  const int nblk = (rows + TL_ROWS - 1) / TL_ROWS;
  int b = blockIdx.x;

  // this thread's chunks of a block: row i * 256 / 40 + ..., fixed offsets
  int crow[TL_CPT], ccol[TL_CPT];
#pragma unroll
  for (int i = 0; i < TL_CPT; ++i) {
    const int idx = t + 256 * i;
    crow[i] = idx / TL_CPR;
    ccol[i] = (idx - crow[i] * TL_CPR) * 8;
  }
  h8 pre[TL_CPT];
  auto load_x = [&](int blk) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TL_CPT; ++i) {
      const int row = blk * TL_ROWS + crow[i];
      pre[i] = row < rows ? *reinterpret_cast<const h8*>(x + (size_t)row * x_ld + ccol[i]) : h8{};
    }
  };
  if (b < nblk) load_x(b);

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

  for (; b < nblk; b += gridDim.x) {
#pragma unroll
    for (int i = 0; i < TL_CPT; ++i) *reinterpret_cast<h8*>(xs + crow[i] * TL_LD + ccol[i]) = pre[i];
    // residual of this block first, then the next block's x: the store phase's wait for the residual
    // leaves the prefetch in flight (vmcnt counts in issue order)
    h8 rr[TL_CPT];
    if (res) {
#pragma unroll
      for (int i = 0; i < TL_CPT; ++i) {
        const int row = b * TL_ROWS + crow[i];
        rr[i] = row < rows ? *reinterpret_cast<const h8*>(res + (size_t)row * res_ld + ccol[i]) : h8{};
      }
    }
    if (b + (int)gridDim.x < nblk) load_x(b + gridDim.x);
    __syncthreads();

    f4 acc[TL_TG][TL_NB];
#pragma unroll
    for (int tg = 0; tg < TL_TG; ++tg)
#pragma unroll
      for (int nb = 0; nb < TL_NB; ++nb) acc[tg][nb] = f4{};
#pragma unroll
    for (int ks = 0; ks < TL_KS; ++ks)
#pragma unroll
      for (int tg = 0; tg < TL_TG; ++tg) {
        const h8 xf = *reinterpret_cast<const h8*>(xs + (tg * 16 + r16) * TL_LD + 32 * ks + 8 * kq);
#pragma unroll
        for (int nb = 0; nb < TL_NB; ++nb)
          acc[tg][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nb][ks], xf, acc[tg][nb], 0, 0, 0);
      }
    // acc[tg][nb] lane l: token tg*16 + r16, channels 80 w + 16 nb + 4 kq + q
#pragma unroll
    for (int tg = 0; tg < TL_TG; ++tg)
#pragma unroll
      for (int nb = 0; nb < TL_NB; ++nb) {
        h4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (half_t)(acc[tg][nb][q] + bv[nb][q]);
        *reinterpret_cast<h4*>(os + (tg * 16 + r16) * TL_LD + 80 * wave + 16 * nb + 4 * kq) = o;
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TL_CPT; ++i) {
      const int row = b * TL_ROWS + crow[i];
      if (row >= rows) continue;
      h8 v = *reinterpret_cast<const h8*>(os + crow[i] * TL_LD + ccol[i]);
      if (res) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] + (float)rr[i][j]);
      }
      *reinterpret_cast<h8*>(out + (size_t)row * out_ld + ccol[i]) = v;
      if constexpr (LN) *reinterpret_cast<h8*>(os + crow[i] * TL_LD + ccol[i]) = v;
    }
    if constexpr (LN) {
      // waves 0 / 1: rows [16 wave, 16 wave + 16) of the block, four lanes per row (lane q holds chunks
      // q + 4 i); the next block's os writes come after its first barrier, so this tile stays intact
      __syncthreads();
      if (wave < TL_ROWS / 16) {
        constexpr int CPL = TLC / 32;
        const int q = lane & 3, r = 16 * wave + (lane >> 2), row = b * TL_ROWS + r;
        h8 v[CPL];
#pragma unroll
        for (int i = 0; i < CPL; ++i) v[i] = *reinterpret_cast<const h8*>(os + r * TL_LD + 8 * (q + 4 * i));
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
}

template <bool LN>
int token_linear_launch(const sdk_token_linear_args* a, const TokenLn& ln, hipStream_t s) {
  const int nblk = (a->rows + TL_ROWS - 1) / TL_ROWS;
  const unsigned grid = (unsigned)(nblk < 256 ? nblk : 256);
  hipLaunchKernelGGL(token_linear320_kernel<LN>, dim3(grid), dim3(256), 0, s, (const half_t*)a->x, a->x_ld,
                     (const half_t*)a->w, a->bias, (const half_t*)a->res, a->res_ld, (half_t*)a->out, a->out_ld,
                     a->rows, ln);
  return check_launch(LN ? "token_linear_ln" : "token_linear");
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
