// Fused cross-attention block for gfx950: the per-step work of CrossAttention.forward with a
// cached context K|V (reference openai_model/attention.py:63-117: to_q -> flash_attn_func ->
// to_out Linear + bias; BasicTransformerBlock adds the residual, attention.py:249):
//
//   q   = t Wq^T                      t: LayerNorm output [M, C], Wq [C, C] (no bias)
//   o_h = softmax(scale q_h K_h^T) V_h   per head h, K|V of the image's context [nk, 2C]
//   out = o Wo^T + bo + residual
//
// One workgroup owns 64 or 128 query rows of one image and keeps q / o in LDS, so of the
// three separate launches' HBM traffic (t, q twice, o twice, residual, out) only t, the
// residual and out remain (forms by channel count: XCfg).  Every product runs on MFMA:
//  * projections: D^T = W X^T on v_mfma_f32_16x16x32_f16 (lane = pixel, 4 consecutive
//    channels), a wave owns 80 (160 in the A/B-only 4-wave 640 form) channels of 64 pixels; W
//    fragments come straight from global memory (the C x C weight is L2-resident, shared by every
//    workgroup);
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
  // fused LayerNorms (BasicTransformerBlock norm2 / norm3, reference attention.py:249-250), or null
  // gamma: t is norm2's INPUT and is normalised in LDS; out_ln = norm3(out)
  const float* ln_in_g; const float* ln_in_b; float ln_in_eps;
  const float* ln_out_g; const float* ln_out_b; float ln_out_eps;
  half_t* out_ln; int out_ln_ld;
  unsigned long long* stamps;   // diagnostics (tools/bench_xattn.py --phases): 6 clock stamps per group, or null
};

__device__ __forceinline__ void stamp(const XAttnParams& p, int i) {
  if (p.stamps && threadIdx.x == 0) p.stamps[blockIdx.x * 8 + i] = wall_clock64();
}

unsigned long long* g_xattn_stamps = nullptr;
int g_xattn_waves640 = 8;

typedef _Float16 h4v __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_t __attribute__((ext_vector_type(4)));

constexpr int XQ = 64;     // query rows per workgroup
constexpr int XKP = 80;    // key slots (5 blocks of 16)

// NWV waves over the 64 query rows.  Projections: wave w owns channels [w*CW, (w+1)*CW) of all 64 rows.
// Head phase: 4 groups of 16 query rows, WPR = NWV / 4 waves per group, each taking HPI / WPR of an
// iteration's heads.  Forms:
//  * 4 waves: one channel quarter per wave (320 channels; at 640 the A/B-only form, sdk_xattn_debug_waves640);
//  * 8 waves at 640 channels: one channel eighth per wave, i.e. the 320-channel form's 80 channels x 64 rows,
//    whose registers allow 2 waves per SIMD where the 4-wave 640 form holds 512 registers per lane (one wave
//    per SIMD); the two waves of a 16-row group take one head each.
//  (a 128-row / 8-wave form at 320 channels — two row halves sharing W fragment fetches and one K / V
//  staging — measured 5-25 % slower than two 4-wave groups per CU: profiles/r6_xattn_waves640_ab.txt)
template <int C, int D, int NWV = 4>
struct XCfg {
  static constexpr int NT = 64 * NWV;
  static constexpr int H = C / D;
  static constexpr int DP = (D + 15) / 16 * 16;     // head dim padded to the 16-wide MFMA K / N
  static constexpr int RG = XQ / 16, WPR = NWV / RG;
  static constexpr int CW = C / NWV;                // channels per wave in the projections
  static constexpr int NB = CW / 16;
  static constexpr int WP = NB <= 5 ? 3 : 4;        // W prefetch depth (K-steps): 80-channel waves keep 2 waves / SIMD
  static constexpr int QLD = C + 8;                 // q / o row stride (halfs); 8 zero pad columns
  static constexpr int KLD = DP + 8;                // K rows [key][d]
  // V rows [key][d] (row-major, 16-B copies like K; the PV operand V^T is read with ds_read_b64_tr_b16):
  // VLD / 2 = 8 * odd (mod 64) dwords puts the 8 rows of a transposed read's 32-lane half on 8 disjoint
  // 8-bank spans (conflict-free): DP = 48 and 80 qualify, DP = 64 takes 80
  static constexpr int VLD = (DP / 2) % 16 == 8 ? DP : DP + 16;
  static_assert((VLD / 2) % 16 == 8, "V row stride: conflict-free transposed reads");
  static constexpr int KVH = XKP * KLD + XKP * VLD; // one head's K + V (halfs)
  // heads per iteration: 2 where the second K / V^T buffer keeps the resident group count
  static constexpr int ONE = (XQ * QLD + KVH) * 2, TWO = (XQ * QLD + 2 * KVH) * 2;
  static constexpr int HPI = (TWO <= 80 * 1024 || ONE > 80 * 1024) && H > 1 ? 2 : 1;
  static constexpr int LDS_HALFS = XQ * QLD + HPI * KVH;
  static constexpr int LDS_BYTES = LDS_HALFS * 2;
  static_assert(C % 64 == 0 && CW % 16 == 0 && D % 8 == 0 && C % D == 0, "shape");
  static_assert((NWV == 4 || NWV == 8) && HPI % WPR == 0, "waves");
  static constexpr int GPW = HPI / WPR;             // heads per wave and iteration
  static_assert(DP - D <= 8, "q padding columns cover the last head's d padding");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// D^T[n, m] = sum_k W[n, k] X[m, k] for the wave's NB 16-channel blocks x 4 16-pixel blocks.
// X rows come from LDS (t in phase A, o in phase C), W rows from global (L2-resident, shared by
// every workgroup).  K-steps of 32, fully unrolled.  The W fragments are the long-latency operand:
// they run WP K-steps ahead through a ring of WP + 1 register sets (the phase was L2-latency-bound
// at two steps ahead: 13 us for 1.3 us of MFMAs); the LDS fragments run one step ahead.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xattn_rsrc(const void* base, long long bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// PK: W in the fragment-packed layout of sdk_xattn_pack_weight — the 64 lanes' 16-B pieces of one (16-channel
// block, K-step) are 1 KiB contiguous, so a wave-instruction fetches 8 whole 128-B lines instead of 64 B of 16 rows
template <int C, int NB, int WP, bool PK>
__device__ __forceinline__ void proj_wave(const half_t* __restrict__ x, int x_ld, const half_t* __restrict__ w,
                                          int n_w, f4 (&acc)[NB][4]) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, c16 = lane >> 4;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f4{};
  constexpr int KS = C / 32;
  const half_t* wp = w + (size_t)(n_w + r16) * C + 8 * c16;
  // packed: one buffer descriptor over the wave's NB x KS KiB pieces, the lane's 16 B as the only VGPR offset and
  // the piece as the scalar offset (no per-block 64-bit pointers)
  const __amdgpu_buffer_rsrc_t wr = xattn_rsrc(w + (size_t)(n_w / 16) * KS * 512, (long long)NB * KS * 1024);
  const half_t* xp = x + (size_t)r16 * x_ld + 8 * c16;
  constexpr int WR = WP + 1;
  h8 fw[WR][NB], fx[2][4];
  auto load_w = [&](int ks) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if constexpr (PK)
        fw[ks % WR][j] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 16, (j * KS + ks) * 1024, 0));
      else
        fw[ks % WR][j] = *reinterpret_cast<const h8*>(wp + (size_t)j * 16 * C + 32 * ks);
    }
  };
  auto load_x = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fx[ks & 1][i] = *reinterpret_cast<const h8*>(xp + (size_t)i * 16 * x_ld + 32 * ks);
  };
#pragma unroll
  for (int ks = 0; ks < WP && ks < KS; ++ks) load_w(ks);
  load_x(0);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + WP < KS) load_w(ks + WP);
    if (ks + 1 < KS) load_x(ks + 1);
    // keep the prefetch where it is: left alone, the scheduler sinks each load next to its
    // MFMA (one step ahead, vmcnt(1) waits) to save registers
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[ks % WR][j], fx[ks & 1][i], acc[j][i], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// norm2 / norm3 of the workgroup's 64 rows with the row math of layer_norm_quad_kernel (common.h:
// the same bits as the separate launch): wave w normalises rows [16w, 16w + 16) of the LDS tile
// `src`, four lanes per row, gamma / beta read from LDS (`gb`, staged in the K / V^T area, which is
// free before phase B and after it), and hands every normalised 8-channel chunk to
// store(row, channel, value).
template <int C, class Store>
__device__ __forceinline__ void ln_quad_rows(const half_t* src, int ld, const float* gb, float eps, Store store) {
  constexpr int CPL = C / 32;
  const int lane = threadIdx.x & 63, q = lane & 3, row = 16 * (threadIdx.x >> 6) + (lane >> 2);
  h8 v[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) v[i] = *reinterpret_cast<const h8*>(src + row * ld + 8 * (q + 4 * i));
  float mean, rstd;
  ln_quad_stats<CPL>(v, eps, mean, rstd);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    store(row, 8 * (q + 4 * i), ln_quad_apply(v[i], mean, rstd, gb, C, q + 4 * i));
    // two chunks' gamma / beta reads in flight at a time: hoisting all of them costs the 2nd
    // resident workgroup (registers)
    if (i & 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// gamma | beta (fp32, C each) of a fused norm: GBT 16-B pieces per thread, loaded into registers
// well ahead of use (under the kernel's own HBM stream an L2 miss costs microseconds), then
// written to the LDS staging area
template <int C, int NT>
struct LnStage {
  static constexpr int GBT = (C / 2 + NT - 1) / NT;
  f4 r[GBT];
  __device__ __forceinline__ void load(const float* gamma, const float* beta) {
#pragma unroll
    for (int u = 0; u < GBT; ++u) {
      const int e = threadIdx.x + NT * u;
      if (e < C / 2) r[u] = *reinterpret_cast<const f4*>(e < C / 4 ? gamma + 4 * e : beta + 4 * (e - C / 4));
    }
  }
  __device__ __forceinline__ void store(float* gb) const {
#pragma unroll
    for (int u = 0; u < GBT; ++u) {
      const int e = threadIdx.x + NT * u;
      if (e < C / 2) *reinterpret_cast<f4*>(gb + 4 * e) = r[u];
    }
  }
};

// the packed 320-channel form is held to 2 waves per SIMD (two groups per CU) explicitly: left alone hipcc spends
// 262 registers on it
template <int C, int D, int NWV, bool PK>
__global__ void __launch_bounds__(64 * NWV, PK && C <= 320 ? 2 : 1) xattn_block_kernel(XAttnParams p) {
  using X = XCfg<C, D, NWV>;
  constexpr int NT = X::NT;
  extern __shared__ __attribute__((aligned(16))) half_t xl[];
  half_t* qo = xl;                              // [64][QLD]
  half_t* kvl = qo + XQ * X::QLD;               // HPI x { K [80][KLD], V [80][VLD] }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, c16 = lane >> 4;
  const int m0 = blockIdx.x * XQ;
  const int b = m0 / p.n_img;
  const int n_w = wave * X::CW;

  static_assert(2 * C * 4 <= X::HPI * X::KVH * 2, "norm gamma / beta staging fits the K / V^T area");
  float* gbl = reinterpret_cast<float*>(kvl);
  LnStage<C, NT> ln2;
  if (p.ln_in_g) ln2.load(p.ln_in_g, p.ln_in_b);
  // zero the q pad columns (the K / V^T padding is zeroed after norm2 has used that area)
  for (int e = tid; e < XQ * 8; e += NT) qo[(e >> 3) * X::QLD + C + (e & 7)] = (half_t)0.f;
  stamp(p, 0);
  // ---- phase A: q = t Wq^T -> LDS (fp16, as the separate to_q GEMM stores it).  The t tile is
  // staged into the q buffer first with every 16-B load in flight at once (one HBM latency
  // instead of one per K-step); q overwrites it after all waves are past their MFMAs.
  {
    constexpr int C8 = C / 8;
    constexpr int TL = XQ * C8 / NT;            // 16-B chunks per thread
    static_assert(XQ * C8 % NT == 0, "t tile chunks");
    h8 tv[TL];
#pragma unroll
    for (int u = 0; u < TL; ++u) {
      const int e = tid + NT * u, row = e / C8, c8 = e - row * C8;
      tv[u] = *reinterpret_cast<const h8*>(p.t + (size_t)(m0 + row) * p.t_ld + 8 * c8);
    }
#pragma unroll
    for (int u = 0; u < TL; ++u) {
      const int e = tid + NT * u, row = e / C8, c8 = e - row * C8;
      *reinterpret_cast<h8*>(qo + row * X::QLD + 8 * c8) = tv[u];
    }
    if (p.ln_in_g) ln2.store(gbl);
  }
  __syncthreads();
  if (p.ln_in_g) {   // norm2 in place: t = LN(tokens); rows 16w .. 16w + 15 on waves 0-3
    if (wave < 4)
      ln_quad_rows<C>(qo, X::QLD, gbl, p.ln_in_eps,
                    [&](int row, int c, const h8& v) { *reinterpret_cast<h8*>(qo + row * X::QLD + c) = v; });
    __syncthreads();
  }
  // K / V^T padding (keys >= nk, d >= D) stays zero through phase B; phase A's barriers order this
  // before the first K / V^T writes
  static_assert(X::HPI * X::KVH % 8 == 0, "K / V^T area in 16-B pieces");
  for (int e = tid; e < X::HPI * X::KVH / 8; e += NT) reinterpret_cast<h8*>(kvl)[e] = h8{};
  stamp(p, 1);
  {
    f4 acc[X::NB][4];
    proj_wave<C, X::NB, X::WP, PK>(qo, X::QLD, p.wq, n_w, acc);
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

  stamp(p, 2);
  // ---- phase B: HPI heads per barrier pair (independent chains the scheduler interleaves),
  // exact softmax over <= 80 keys; o_h overwrites q_h in LDS.  The K / V chunks (16 B) of later
  // iterations' heads are loaded into registers KVA iterations ahead and written to LDS after
  // the current iteration's closing barrier.
  const half_t* kvb = p.kv + (size_t)b * p.nk * p.kv_ld;
  const int qrow = 16 * (NWV == 4 ? wave : wave & 3) + r16;   // this lane's query (S^T column)
  constexpr int HPI = X::HPI, GPW = X::GPW;
  const int g0 = NWV == 4 ? 0 : (wave >> 2) * GPW;            // the wave's first head slot of an iteration
  constexpr int CH = D / 8;                     // 16-B chunks per key row
  constexpr int NCH = (XKP * CH + NT - 1) / NT; // chunks per thread per head
  constexpr int NIT = (X::H + HPI - 1) / HPI;
  constexpr int KVA = HPI == 2 ? 1 : 2;          // iterations of K / V prefetch (register budget)
  h8 rk[KVA][HPI][NCH], rv[KVA][HPI][NCH];
  auto kv_load = [&](int it, int sl) {
#pragma unroll
    for (int g = 0; g < HPI; ++g) {
      const int h = it * HPI + g;
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int e = tid + NT * u;
        const int key = e / CH, ch = e - key * CH;
        if (key < p.nk && h < X::H) {
          const half_t* src = kvb + (size_t)key * p.kv_ld + h * D + 8 * ch;
          rk[sl][g][u] = *reinterpret_cast<const h8*>(src);
          rv[sl][g][u] = *reinterpret_cast<const h8*>(src + C);
        }
      }
    }
  };
  kv_load(0, 0);
  if (KVA == 2 && NIT > 1) kv_load(1, 1 % KVA);
#pragma unroll 2
  for (int it = 0; it < NIT; ++it) {
    const int sl = it % KVA;
#pragma unroll
    for (int g = 0; g < HPI; ++g) {
      half_t* kl = kvl + g * X::KVH;
      half_t* vr = kl + XKP * X::KLD;
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const int e = tid + NT * u;
        const int key = e / CH, ch = e - key * CH;
        if (key < p.nk && it * HPI + g < X::H) {
          *reinterpret_cast<h8*>(kl + key * X::KLD + 8 * ch) = rk[sl][g][u];
          *reinterpret_cast<h8*>(vr + key * X::VLD + 8 * ch) = rv[sl][g][u];
        }
      }
    }
    __syncthreads();
    if (it + KVA < NIT) kv_load(it + KVA, sl);
    __builtin_amdgcn_sched_barrier(0);
    const int ng = X::H - it * HPI < HPI ? X::H - it * HPI : HPI;   // heads this iteration
    // S^T[key, q] for the 5 key blocks of each head
    f4 s[GPW][XKP / 16];
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi)
#pragma unroll
      for (int kb = 0; kb < XKP / 16; ++kb) s[gi][kb] = f4{};
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
      const int g = g0 + gi;
      if (g < ng) {
        const int h = it * HPI + g;
        const half_t* kl = kvl + g * X::KVH;
#pragma unroll
        for (int dd = 0; dd < X::DP; dd += 16) {
          const h4v fq = *reinterpret_cast<const h4v*>(qo + qrow * X::QLD + h * D + dd + 4 * c16);
#pragma unroll
          for (int kb = 0; kb < XKP / 16; ++kb) {
            const h4v fk = *reinterpret_cast<const h4v*>(kl + (16 * kb + r16) * X::KLD + dd + 4 * c16);
            s[gi][kb] = __builtin_amdgcn_mfma_f32_16x16x16f16(fk, fq, s[gi][kb], 0, 0, 0);
          }
        }
      }
    }
    // lane holds keys 16kb + 4*c16 + r of query qrow
    float mx[GPW], sum[GPW], inv[GPW];
    h4v pf[GPW][XKP / 16];
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      mx[g] = -__builtin_inff();
#pragma unroll
      for (int kb = 0; kb < XKP / 16; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = 16 * kb + 4 * c16 + r;
          const float v = key < p.nk ? s[g][kb][r] * p.c : -__builtin_inff();
          s[g][kb][r] = v;
          mx[g] = fmaxf(mx[g], v);
        }
    }
#pragma unroll
    for (int g = 0; g < GPW; ++g) mx[g] = fmaxf(mx[g], __shfl_xor(mx[g], 16, 64));
#pragma unroll
    for (int g = 0; g < GPW; ++g) mx[g] = fmaxf(mx[g], __shfl_xor(mx[g], 32, 64));
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      sum[g] = 0.f;
#pragma unroll
      for (int kb = 0; kb < XKP / 16; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[g][kb][r] - mx[g]);
          sum[g] += e;
          pf[g][kb][r] = (half_t)e;
        }
    }
#pragma unroll
    for (int g = 0; g < GPW; ++g) sum[g] += __shfl_xor(sum[g], 16, 64);
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      sum[g] += __shfl_xor(sum[g], 32, 64);
      inv[g] = 1.f / sum[g];
    }
    // O^T[d, q] = sum_key V^T[d, key] P^T[key, q]; the A operand V^T[dd + i][16 kb + 4 g' + q] comes from the
    // row-major V by the hardware transposed read: lane 4 q + pp of 16-lane group g' supplies the address of
    // V[16 kb + 4 g' + q][dd + 4 pp .. + 3] and receives column dd + (lane & 15) of the group's 4 rows
    // (EXEC is all ones here: g < ng is wave-uniform)
    const int tr_off = (4 * c16 + ((lane & 15) >> 2)) * X::VLD + 4 * (lane & 3);
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
      const int g = g0 + gi;
      if (g < ng) {
        const int h = it * HPI + g;
        const half_t* vr = kvl + g * X::KVH + XKP * X::KLD;
#pragma unroll
        for (int dd = 0; dd < X::DP; dd += 16) {
          f4 o = f4{};
#pragma unroll
          for (int kb = 0; kb < XKP / 16; ++kb) {
            const auto t4 = __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                (__attribute__((address_space(3))) fp16x4_t*)(vr + 16 * kb * X::VLD + dd + tr_off));
            const h4v fv = __builtin_bit_cast(h4v, t4);
            o = __builtin_amdgcn_mfma_f32_16x16x16f16(fv, pf[gi][kb], o, 0, 0, 0);
          }
          const int d0 = dd + 4 * c16;          // lane holds d0..d0+3 of query qrow
          if (d0 < D) {
            h4v w;
#pragma unroll
            for (int r = 0; r < 4; ++r) w[r] = (half_t)(o[r] * inv[gi]);
            *reinterpret_cast<h4v*>(qo + qrow * X::QLD + h * D + d0) = w;
          }
        }
      }
    }
    __syncthreads();   // o of these heads visible; K / V^T buffers free for the next iteration
  }

  stamp(p, 3);
  // ---- phase C: out = o Wo^T + bo (fp16) + residual, staged through LDS for row stores
  {
    LnStage<C, NT> ln3;
    if (p.out_ln) ln3.load(p.ln_out_g, p.ln_out_b);
    f4 acc[X::NB][4];
    proj_wave<C, X::NB, X::WP, PK>(qo, X::QLD, p.wo, n_w, acc);
    __syncthreads();   // every wave is done reading o
    stamp(p, 4);
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
    if (p.out_ln) ln3.store(gbl);   // phase B is over: the K / V^T area is free
    __syncthreads();
    constexpr int C8 = C / 8;
    for (int e = tid; e < XQ * C8; e += NT) {
      const int row = e / C8, c8 = e - row * C8;
      h8 v = *reinterpret_cast<const h8*>(qo + row * X::QLD + 8 * c8);
      const size_t m = (size_t)m0 + row;
      if (p.res) {
        const h8 rr = *reinterpret_cast<const h8*>(p.res + m * p.res_ld + 8 * c8);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (half_t)((float)v[q] + (float)rr[q]);
      }
      *reinterpret_cast<h8*>(p.out + m * p.out_ld + 8 * c8) = v;
      if (p.out_ln) *reinterpret_cast<h8*>(qo + row * X::QLD + 8 * c8) = v;
    }
    if (p.out_ln) {   // norm3 of the finished rows
      __syncthreads();
      half_t* dst = p.out_ln + (size_t)m0 * p.out_ln_ld;
      const int ld = p.out_ln_ld;
      if (wave < 4)
        ln_quad_rows<C>(qo, X::QLD, gbl, p.ln_out_eps,
                      [&](int row, int c, const h8& v) { *reinterpret_cast<h8*>(dst + (size_t)row * ld + c) = v; });
    }
  }
  stamp(p, 5);
}

template <int C, int D, int NWV, bool PK>
int launch_xattn2(const XAttnParams& p, int m, hipStream_t s) {
  using X = XCfg<C, D, NWV>;
  static std::atomic<unsigned long long> attr{0};
  if (int e = ensure_dyn_lds((const void*)xattn_block_kernel<C, D, NWV, PK>, X::LDS_BYTES, attr, "cross_attention_block"))
    return e;
  hipLaunchKernelGGL((xattn_block_kernel<C, D, NWV, PK>), dim3(m / XQ), dim3(X::NT), X::LDS_BYTES, s, p);
  return check_launch("xattn_block");
}

template <int C, int D, int NWV = 4>
int launch_xattn(const XAttnParams& p, int m, bool packed, hipStream_t s) {
  return packed ? launch_xattn2<C, D, NWV, true>(p, m, s) : launch_xattn2<C, D, NWV, false>(p, m, s);
}

// fragment-packed copy of a [C][w_ld] fp16 projection weight: piece ((nb * KS + ks) * 64 + lane) holds row
// 16 nb + (lane & 15), columns 32 ks + 8 (lane >> 4) .. + 7 (the A-fragment of v_mfma_f32_16x16x32_f16)
__global__ void __launch_bounds__(256) xattn_pack_kernel(const half_t* __restrict__ w, int w_ld, half_t* __restrict__ pk,
                                                         int C) {
  const int e = blockIdx.x * 256 + threadIdx.x;     // 16-B piece
  if (e >= C * C / 8) return;
  const int lane = e & 63, f = e >> 6, ks_n = C / 32;
  const int nb = f / ks_n, ks = f - nb * ks_n;
  *reinterpret_cast<h8*>(pk + (size_t)e * 8) =
      *reinterpret_cast<const h8*>(w + (size_t)(16 * nb + (lane & 15)) * w_ld + 32 * ks + 8 * (lane >> 4));
}

// Segment softmax of the reassociated cross-attention (1280-channel levels, attention.py:106-112
// rearranged): row m of s holds, for every head h, the 77 scores of its query against the context
// keys in columns [h*seglen, (h+1)*seglen); p = softmax over each segment of scale*s, fp16, with the
// columns from nseg*seglen up to the row's K padding written as zeros.  One wave per row, one
// segment at a time: 64 + 64 columns per lane pair, a DPP max and sum per segment.
__device__ __forceinline__ float wave_max_f(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x124>(x));
  x = fmaxf(x, dpp_f<0x128>(x));
  return fmaxf(fmaxf(readlane_f(x, 0), readlane_f(x, 16)), fmaxf(readlane_f(x, 32), readlane_f(x, 48)));
}

__global__ void __launch_bounds__(256) segment_softmax_kernel(const float* __restrict__ s, int ld_s,
                                                               half_t* __restrict__ p, int ld_p, int rows, int nseg,
                                                               int seglen, float c) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* sr = s + (size_t)row * ld_s;
  half_t* pr = p + (size_t)row * ld_p;
  for (int h = 0; h < nseg; ++h) {
    const int c0 = h * seglen + lane, c1 = c0 + 64;
    const bool ok0 = lane < seglen, ok1 = lane + 64 < seglen;
    const float x0 = ok0 ? sr[c0] : -__builtin_inff(), x1 = ok1 ? sr[c1] : -__builtin_inff();
    const float m = wave_max_f(fmaxf(x0, x1));
    const float e0 = ok0 ? __builtin_amdgcn_exp2f((x0 - m) * c) : 0.f;
    const float e1 = ok1 ? __builtin_amdgcn_exp2f((x1 - m) * c) : 0.f;
    const float inv = 1.f / wave_sum_f(e0 + e1);
    if (ok0) pr[c0] = (half_t)(e0 * inv);
    if (ok1) pr[c1] = (half_t)(e1 * inv);
  }
  for (int col = nseg * seglen + lane; col < ld_p; col += 64) pr[col] = (half_t)0.f;
}

}  // namespace
}  // namespace sdk

using namespace sdk;

// diagnostics only (not in sdk_amd.h): per-workgroup phase clock stamps into a device buffer of
// 8 * groups uint64 (wall_clock64, 100 MHz), for tools/bench_xattn.py --phases; null turns it off
extern "C" void sdk_xattn_debug_stamps(unsigned long long* dev) { g_xattn_stamps = dev; }
// A/B only (not in sdk_amd.h): waves of the 640-channel form, 8 (default) or 4
extern "C" int sdk_xattn_debug_waves640(int waves) {
  if (waves != 4 && waves != 8) return fail(SDK_EINVAL, "xattn waves: 4 or 8");
  g_xattn_waves640 = waves;
  return SDK_OK;
}

extern "C" int sdk_cross_attention_block_supported(int32_t channels, int32_t head_dim, int32_t nk, int32_t n_img) {
  const bool cd = (channels == 320 && (head_dim == 40 || head_dim == 64)) ||
                  (channels == 640 && (head_dim == 80 || head_dim == 64));
  return cd && nk >= 1 && nk <= XKP && n_img > 0 && n_img % XQ == 0;
}

namespace {
int xattn_run(const sdk_xattn_args* a, const sdk_xattn_ln_args* ln, sdk_stream_t stream) {
  if (!a || !a->t || !a->kv || !a->wq || !a->wo || !a->out) return fail(SDK_EINVAL, "cross_attention_block: null");
  if (!sdk_cross_attention_block_supported(a->channels, a->head_dim, a->nk, a->n_img))
    return fail(SDK_EINVAL, "cross_attention_block: unsupported shape (channels 320/640, head_dim 40/64/80, "
                            "nk <= 80, tokens per image a multiple of 64)");
  if (a->batch <= 0) return fail(SDK_EINVAL, "cross_attention_block: empty batch");
  if (a->t_ld % 8 || a->kv_ld % 8 || a->out_ld % 8 || (a->res && a->res_ld % 8) || a->kv_ld < 2 * a->channels)
    return fail(SDK_EINVAL, "cross_attention_block: row strides must be multiples of 8 (kv >= 2*channels)");
  if (a->w_ld != a->channels && a->w_ld != 0)
    return fail(SDK_EINVAL, "cross_attention_block: w_ld must be channels (row layout) or 0 (sdk_xattn_pack_weight layout)");
  const bool packed = a->w_ld == 0;
  XAttnParams p{};
  p.t = (const half_t*)a->t; p.kv = (const half_t*)a->kv; p.wq = (const half_t*)a->wq; p.wo = (const half_t*)a->wo;
  p.bo = a->bias; p.res = (const half_t*)a->res; p.out = (half_t*)a->out;
  p.t_ld = a->t_ld; p.kv_ld = a->kv_ld; p.res_ld = a->res_ld; p.out_ld = a->out_ld;
  p.n_img = a->n_img; p.nk = a->nk; p.c = a->scale * 1.4426950408889634f;
  p.stamps = g_xattn_stamps;
  if (ln) {
    if (ln->in_gamma) {
      if (!ln->in_beta || (((uintptr_t)ln->in_gamma | (uintptr_t)ln->in_beta) & 15))
        return fail(SDK_EINVAL, "cross_attention_block_ln: norm2 gamma / beta null or not 16-B aligned");
      p.ln_in_g = ln->in_gamma; p.ln_in_b = ln->in_beta; p.ln_in_eps = ln->in_eps;
    }
    if (ln->out_gamma) {
      if (!ln->out_beta || !ln->out_ln || (((uintptr_t)ln->out_gamma | (uintptr_t)ln->out_beta) & 15))
        return fail(SDK_EINVAL, "cross_attention_block_ln: norm3 gamma / beta / output null or not 16-B aligned");
      if (ln->out_ln_ld % 8 || ln->out_ln_ld < a->channels)
        return fail(SDK_EINVAL, "cross_attention_block_ln: norm3 output row stride");
      p.ln_out_g = ln->out_gamma; p.ln_out_b = ln->out_beta; p.ln_out_eps = ln->out_eps;
      p.out_ln = (half_t*)ln->out_ln; p.out_ln_ld = ln->out_ln_ld;
    }
  }
  const int m = a->batch * a->n_img;
  hipStream_t s = (hipStream_t)stream;
  if (a->channels == 320)
    return a->head_dim == 40 ? launch_xattn<320, 40>(p, m, packed, s) : launch_xattn<320, 64>(p, m, packed, s);
  if (g_xattn_waves640 == 4)
    return a->head_dim == 80 ? launch_xattn<640, 80, 4>(p, m, packed, s) : launch_xattn<640, 64, 4>(p, m, packed, s);
  return a->head_dim == 80 ? launch_xattn<640, 80, 8>(p, m, packed, s) : launch_xattn<640, 64, 8>(p, m, packed, s);
}
}  // namespace

extern "C" int sdk_xattn_pack_weight(const void* w, int32_t w_ld, void* packed, int32_t channels, sdk_stream_t stream) {
  if (!w || !packed) return fail(SDK_EINVAL, "xattn_pack_weight: null pointer");
  if (channels != 320 && channels != 640) return fail(SDK_EINVAL, "xattn_pack_weight: channels must be 320 or 640");
  if (w_ld < channels || w_ld % 8 || (((uintptr_t)w | (uintptr_t)packed) & 15))
    return fail(SDK_EINVAL, "xattn_pack_weight: w_ld >= channels, w_ld % 8 == 0, 16-B aligned pointers");
  const int pieces = channels * channels / 8;
  hipLaunchKernelGGL(xattn_pack_kernel, dim3((pieces + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const half_t*)w, w_ld, (half_t*)packed, channels);
  return check_launch("xattn_pack_weight");
}

extern "C" int sdk_cross_attention_block(const sdk_xattn_args* a, sdk_stream_t stream) {
  return xattn_run(a, nullptr, stream);
}

extern "C" int sdk_cross_attention_block_ln(const sdk_xattn_args* a, const sdk_xattn_ln_args* ln,
                                            sdk_stream_t stream) {
  if (!ln) return fail(SDK_EINVAL, "cross_attention_block_ln: null norm arguments");
  return xattn_run(a, ln, stream);
}

extern "C" int sdk_segment_softmax(const float* s, int32_t ld_s, void* p, int32_t ld_p, int32_t rows, int32_t nseg,
                                   int32_t seglen, float scale, sdk_stream_t stream) {
  if (!s || !p) return fail(SDK_EINVAL, "segment_softmax: null pointer");
  if (rows <= 0 || nseg <= 0 || seglen <= 0 || seglen > 128)
    return fail(SDK_EINVAL, "segment_softmax: rows / nseg must be positive, 1 <= seglen <= 128");
  if (ld_s < nseg * seglen || ld_p < nseg * seglen) return fail(SDK_EINVAL, "segment_softmax: row stride too small");
  const int blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(segment_softmax_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, s, ld_s, (half_t*)p,
                     ld_p, rows, nseg, seglen, scale * 1.4426950408889634f);
  return check_launch("segment_softmax");
}
