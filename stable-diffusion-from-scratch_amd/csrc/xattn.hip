// Fused cross-attention block for gfx950: the per-step work of CrossAttention.forward with a
// cached context K|V (reference openai_model/attention.py:63-117: to_q -> flash_attn_func ->
// to_out Linear + bias; BasicTransformerBlock adds the residual, attention.py:249):
//
//   q   = t Wq^T                      t: LayerNorm output [M, C], Wq [C, C] (no bias)
//   o_h = softmax(scale q_h K_h^T) V_h   per head h, K|V of the image's context [nk, 2C]
//   out = o Wo^T + bo + residual
//
// One workgroup (4 waves) owns 64 query rows of one image and keeps q / o in LDS, so of the
// three separate launches' HBM traffic (t, q twice, o twice, residual, out) only t, the
// residual and out remain.  Every product runs on MFMA:
//  * projections: D^T = W X^T on v_mfma_f32_16x16x32_f16 (lane = pixel, 4 consecutive
//    channels), wave w owns channels [w*C/4, (w+1)*C/4) of all 64 pixels; W fragments come
//    straight from global memory (the C x C weight is L2-resident, shared by every workgroup);
//  * attention on v_mfma_f32_16x16x16_f16, transposed as in attention.hip: S^T = K q^T puts
//    one query per lane column, so the S^T accumulator is already the B operand of
//    O^T = V^T P^T and a query row's max / sum is a register chain plus two lane swaps;
//    all nk <= 80 keys fit one tile, so the softmax is exact (no running rescale).
#include "common.h"

namespace sdk {
namespace {

struct XAttnParams {
  const half_t* t;      // [M, t_ld] LayerNorm output (query tokens)
  const half_t* kv;     // [batch * nk, kv_ld]: K at columns [0, C), V at [C, 2C)
  const half_t* wq;     // [>= C rows][C] (PackedConv 1x1 layout: row n, K contiguous)
  const half_t* wo;     // [>= C rows][C]
  const float* bo;      // [C] or null
  const half_t* res;    // [M, res_ld] or null
  half_t* out;          // [M, out_ld]
  int t_ld, kv_ld, res_ld, out_ld;
  int n_img;            // query tokens per image (multiple of 64)
  int nk;               // context tokens (<= 80)
  float c;              // softmax scale * log2(e)
};

typedef _Float16 h4v __attribute__((ext_vector_type(4)));

constexpr int XQ = 64;     // query rows per workgroup
constexpr int XKP = 80;    // key slots (5 blocks of 16)

template <int C, int D>
struct XCfg {
  static constexpr int NT = 256;                    // 4 waves, one channel quarter each
  static constexpr int H = C / D;
  static constexpr int DP = (D + 15) / 16 * 16;     // head dim padded to the 16-wide MFMA K / N
  static constexpr int CW = C / 4;                  // channels per wave in the projections
  static constexpr int NB = CW / 16;
  static constexpr int QLD = C + 8;                 // q / o row stride (halfs); 8 zero pad columns
  static constexpr int KLD = DP + 8;                // K rows [key][d]
  static constexpr int VLD = XKP + 8;               // V^T rows [d][key]
  static constexpr int LDS_HALFS = XQ * QLD + XKP * KLD + DP * VLD;
  static constexpr int LDS_BYTES = LDS_HALFS * 2;
  static_assert(C % 64 == 0 && CW % 16 == 0 && D % 8 == 0 && C % D == 0, "shape");
  static_assert(DP - D <= 8, "q padding columns cover the last head's d padding");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// D^T[n, m] = sum_k W[n, k] X[m, k] for the wave's NB 16-channel blocks x 4 16-pixel blocks.
// X rows come from global (phase A: t) or LDS (phase C: o), W rows from global (L2-resident).
// K-steps of 32, fully unrolled, fragments loaded two steps ahead (three register sets): the
// W / t fragments come from L2 / HBM, and one step of prefetch leaves the MFMAs waiting.
template <int C, int NB>
__device__ __forceinline__ void proj_wave(const half_t* __restrict__ x, int x_ld, const half_t* __restrict__ w,
                                          int n_w, f4 (&acc)[NB][4]) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, c16 = lane >> 4;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f4{};
  const half_t* wp = w + (size_t)(n_w + r16) * C + 8 * c16;
  const half_t* xp = x + (size_t)r16 * x_ld + 8 * c16;
  constexpr int KS = C / 32;
  h8 fw[3][NB], fx[3][4];
  auto load = [&](int ks, int slot) {
#pragma unroll
    for (int j = 0; j < NB; ++j) fw[slot][j] = *reinterpret_cast<const h8*>(wp + (size_t)j * 16 * C + 32 * ks);
#pragma unroll
    for (int i = 0; i < 4; ++i) fx[slot][i] = *reinterpret_cast<const h8*>(xp + (size_t)i * 16 * x_ld + 32 * ks);
  };
  load(0, 0);
  if (KS > 1) load(1, 1);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 2 < KS) load(ks + 2, (ks + 2) % 3);
    const int sl = ks % 3;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[sl][j], fx[sl][i], acc[j][i], 0, 0, 0);
  }
}

template <int C, int D>
__global__ void __launch_bounds__(256, 1) xattn_block_kernel(XAttnParams p) {
  using X = XCfg<C, D>;
  extern __shared__ __attribute__((aligned(16))) half_t xl[];
  half_t* qo = xl;                              // [64][QLD]
  half_t* kl = qo + XQ * X::QLD;                // [80][KLD]
  half_t* vt = kl + XKP * X::KLD;               // [DP][VLD]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, c16 = lane >> 4;
  const int m0 = blockIdx.x * XQ;
  const int b = m0 / p.n_img;
  const int n_w = wave * X::CW;

  // zero: K / V^T padding (keys >= nk, d >= D) and the q pad columns
  for (int e = tid; e < XKP * X::KLD + X::DP * X::VLD; e += 256) kl[e] = (half_t)0.f;
  for (int e = tid; e < XQ * 8; e += 256) qo[(e >> 3) * X::QLD + C + (e & 7)] = (half_t)0.f;

  // ---- phase A: q = t Wq^T -> LDS (fp16, as the separate to_q GEMM stores it).  The t tile is
  // staged into the q buffer first with every 16-B load in flight at once (one HBM latency
  // instead of one per K-step); q overwrites it after all waves are past their MFMAs.
  {
    constexpr int C8 = C / 8;
    constexpr int TL = XQ * C8 / 256;           // 16-B chunks per thread
    static_assert(XQ * C8 % 256 == 0, "t tile chunks");
    h8 tv[TL];
#pragma unroll
    for (int u = 0; u < TL; ++u) {
      const int e = tid + 256 * u, row = e / C8, c8 = e - row * C8;
      tv[u] = *reinterpret_cast<const h8*>(p.t + (size_t)(m0 + row) * p.t_ld + 8 * c8);
    }
#pragma unroll
    for (int u = 0; u < TL; ++u) {
      const int e = tid + 256 * u, row = e / C8, c8 = e - row * C8;
      *reinterpret_cast<h8*>(qo + row * X::QLD + 8 * c8) = tv[u];
    }
  }
  __syncthreads();
  {
    f4 acc[X::NB][4];
    proj_wave<C, X::NB>(qo, X::QLD, p.wq, n_w, acc);
    __syncthreads();   // every wave is done reading t
#pragma unroll
    for (int j = 0; j < X::NB; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        h4v v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (half_t)acc[j][i][r];
        *reinterpret_cast<h4v*>(qo + (16 * i + r16) * X::QLD + n_w + 16 * j + 4 * c16) = v;
      }
  }
  __syncthreads();

  // ---- phase B: per head, exact softmax over <= 80 keys; o_h overwrites q_h in LDS.  The
  // next head's K / V chunks (16 B) are loaded into registers while the current head
  // computes, and written to LDS after its closing barrier.
  const half_t* kvb = p.kv + (size_t)b * p.nk * p.kv_ld;
  const int qrow = 16 * wave + r16;             // this lane's query (S^T column)
  constexpr int CH = D / 8;                     // 16-B chunks per key row
  constexpr int NCH = (XKP * CH + 255) / 256;   // chunks per thread
  h8 rk[NCH], rv[NCH];
  auto kv_load = [&](int h) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int e = tid + 256 * u;
      const int key = e / CH, ch = e - key * CH;
      if (key < p.nk) {
        const half_t* src = kvb + (size_t)key * p.kv_ld + h * D + 8 * ch;
        rk[u] = *reinterpret_cast<const h8*>(src);
        rv[u] = *reinterpret_cast<const h8*>(src + C);
      }
    }
  };
  kv_load(0);
  for (int h = 0; h < X::H; ++h) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int e = tid + 256 * u;
      const int key = e / CH, ch = e - key * CH;
      if (key < p.nk) {
        *reinterpret_cast<h8*>(kl + key * X::KLD + 8 * ch) = rk[u];
#pragma unroll
        for (int q = 0; q < 8; ++q) vt[(8 * ch + q) * X::VLD + key] = rv[u][q];
      }
    }
    __syncthreads();
    if (h + 1 < X::H) kv_load(h + 1);
    // S^T[key, q] for the 5 key blocks
    f4 s[XKP / 16];
#pragma unroll
    for (int kb = 0; kb < XKP / 16; ++kb) s[kb] = f4{};
#pragma unroll
    for (int dd = 0; dd < X::DP; dd += 16) {
      const h4v fq = *reinterpret_cast<const h4v*>(qo + qrow * X::QLD + h * D + dd + 4 * c16);
#pragma unroll
      for (int kb = 0; kb < XKP / 16; ++kb) {
        const h4v fk = *reinterpret_cast<const h4v*>(kl + (16 * kb + r16) * X::KLD + dd + 4 * c16);
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x16f16(fk, fq, s[kb], 0, 0, 0);
      }
    }
    // lane holds keys 16kb + 4*c16 + r of query qrow
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < XKP / 16; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * kb + 4 * c16 + r;
        const float v = key < p.nk ? s[kb][r] * p.c : -INFINITY;
        s[kb][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
    h4v pf[XKP / 16];
#pragma unroll
    for (int kb = 0; kb < XKP / 16; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[kb][r] - mx);
        sum += e;
        pf[kb][r] = (half_t)e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    // O^T[d, q] = sum_key V^T[d, key] P^T[key, q]
#pragma unroll
    for (int dd = 0; dd < X::DP; dd += 16) {
      f4 o = f4{};
#pragma unroll
      for (int kb = 0; kb < XKP / 16; ++kb) {
        const h4v fv = *reinterpret_cast<const h4v*>(vt + (dd + r16) * X::VLD + 16 * kb + 4 * c16);
        o = __builtin_amdgcn_mfma_f32_16x16x16f16(fv, pf[kb], o, 0, 0, 0);
      }
      const int d0 = dd + 4 * c16;              // lane holds d0..d0+3 of query qrow
      if (d0 < D) {
        h4v w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = (half_t)(o[r] * inv);
        *reinterpret_cast<h4v*>(qo + qrow * X::QLD + h * D + d0) = w;
      }
    }
    __syncthreads();   // o_h visible; K / V^T free for the next head
  }

  // ---- phase C: out = o Wo^T + bo (fp16) + residual, staged through LDS for row stores
  {
    f4 acc[X::NB][4];
    proj_wave<C, X::NB>(qo, X::QLD, p.wo, n_w, acc);
    __syncthreads();   // every wave is done reading o
#pragma unroll
    for (int j = 0; j < X::NB; ++j) {
      const int n = n_w + 16 * j + 4 * c16;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = p.bo ? p.bo[n + r] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        h4v v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (half_t)(acc[j][i][r] + bv[r]);
        *reinterpret_cast<h4v*>(qo + (16 * i + r16) * X::QLD + n) = v;
      }
    }
    __syncthreads();
    constexpr int C8 = C / 8;
    for (int e = tid; e < XQ * C8; e += 256) {
      const int row = e / C8, c8 = e - row * C8;
      h8 v = *reinterpret_cast<const h8*>(qo + row * X::QLD + 8 * c8);
      const size_t m = (size_t)m0 + row;
      if (p.res) {
        const h8 rr = *reinterpret_cast<const h8*>(p.res + m * p.res_ld + 8 * c8);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (half_t)((float)v[q] + (float)rr[q]);
      }
      *reinterpret_cast<h8*>(p.out + m * p.out_ld + 8 * c8) = v;
    }
  }
}

template <int C, int D>
int launch_xattn(const XAttnParams& p, int m, hipStream_t s) {
  using X = XCfg<C, D>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)xattn_block_kernel<C, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            X::LDS_BYTES) != hipSuccess)
      return fail(SDK_EHIP, "cross_attention_block: cannot raise the dynamic LDS limit");
    attr = true;
  }
  hipLaunchKernelGGL((xattn_block_kernel<C, D>), dim3(m / XQ), dim3(X::NT), X::LDS_BYTES, s, p);
  return check_launch("xattn_block");
}

}  // namespace
}  // namespace sdk

using namespace sdk;

extern "C" int sdk_cross_attention_block_supported(int32_t channels, int32_t head_dim, int32_t nk, int32_t n_img) {
  const bool cd = (channels == 320 && (head_dim == 40 || head_dim == 64)) ||
                  (channels == 640 && (head_dim == 80 || head_dim == 64));
  return cd && nk >= 1 && nk <= XKP && n_img > 0 && n_img % XQ == 0;
}

extern "C" int sdk_cross_attention_block(const sdk_xattn_args* a, sdk_stream_t stream) {
  if (!a || !a->t || !a->kv || !a->wq || !a->wo || !a->out) return fail(SDK_EINVAL, "cross_attention_block: null");
  if (!sdk_cross_attention_block_supported(a->channels, a->head_dim, a->nk, a->n_img))
    return fail(SDK_EINVAL, "cross_attention_block: unsupported shape (channels 320/640, head_dim 40/64/80, "
                            "nk <= 80, tokens per image a multiple of 64)");
  if (a->batch <= 0) return fail(SDK_EINVAL, "cross_attention_block: empty batch");
  if (a->t_ld % 8 || a->kv_ld % 8 || a->out_ld % 8 || (a->res && a->res_ld % 8) || a->kv_ld < 2 * a->channels)
    return fail(SDK_EINVAL, "cross_attention_block: row strides must be multiples of 8 (kv >= 2*channels)");
  if (a->w_ld != a->channels) return fail(SDK_EINVAL, "cross_attention_block: weight rows must be channels long");
  XAttnParams p{(const half_t*)a->t, (const half_t*)a->kv, (const half_t*)a->wq, (const half_t*)a->wo, a->bias,
                (const half_t*)a->res, (half_t*)a->out, a->t_ld, a->kv_ld, a->res_ld, a->out_ld, a->n_img, a->nk,
                a->scale * 1.4426950408889634f};
  const int m = a->batch * a->n_img;
  hipStream_t s = (hipStream_t)stream;
  if (a->channels == 320) return a->head_dim == 40 ? launch_xattn<320, 40>(p, m, s) : launch_xattn<320, 64>(p, m, s);
  return a->head_dim == 80 ? launch_xattn<640, 80>(p, m, s) : launch_xattn<640, 64>(p, m, s);
}
