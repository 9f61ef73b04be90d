// Flash-style attention forward for gfx950: O = softmax(scale*Q K^T) V, fp16 I/O,
// fp32 scores/softmax, v_mfma_f32_32x32x16_f16.
//
// Workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32
// rows.  Keys stream through LDS in tiles of 64.  The score tile is computed
// transposed, S^T = K Q^T (A = K rows from LDS, B = Q^T fragments held in
// registers for the whole loop), so each lane owns ONE query row: the softmax
// row max / row sum are in-register reductions plus one exchange with lane^32.
// The S^T accumulator, converted to fp16, is directly the B operand of
// O^T += V^T P^T (its row index = the key = the contraction index).  V stays
// row-major in LDS and the V^T operand is read with ds_read_b64_tr_b16 (the
// hardware transpose read), rows padded so a 32-lane half touches 64 distinct
// banks.
//
// Per-tile VALU is the budget at small head dims (d = 40: 14 MFMAs per 64-key
// tile), so: the softmax scale is one FMA feeding v_exp_f32 (scores stay raw),
// key masking runs only in a ragged last tile, the O rescale is skipped when
// no lane's running max grew, and when d is below the padded V width the row
// sum comes out of the PV MFMA itself (a ones column in V's zero padding).
// Head dims that are not multiples of 16/32 (40, 80, 160 in SD-1) are padded
// inside LDS/registers only; HBM traffic is the unpadded tensors.
#include "common.h"

namespace sdk {
namespace {

struct AttnParams {
  const half_t* q;
  const half_t* k;
  const half_t* v;
  half_t* o;
  int q_ld, k_ld, v_ld, o_ld;
  int batch, heads, nq, nk, d;
  float c;              // scale * log2(e)
};

typedef __fp16 fp16x4_t __attribute__((ext_vector_type(4)));

constexpr int KT = 64;          // keys per tile

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int DQK, int DV>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnParams p) {
  constexpr int KLD = DQK + 8;                                       // K row stride (halfs)
  constexpr int VLD = ((DV * 2 / 64) % 2 == 0) ? DV + 32 : DV;       // V row stride: 64 or 192 B mod 256
  __shared__ __attribute__((aligned(16))) half_t smem[KT * KLD + KT * VLD];
  half_t* Ks = smem;
  half_t* Vs = smem + KT * KLD;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  const int head = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int qrow = q0 + fr;
  const bool qvalid = qrow < p.nq;
  const bool ones_row = p.d < DV;          // row sum from the PV MFMA (ones column at d)

  // Q^T fragments (B operand): lane holds Q[qrow][ks*16 + 8*fh + j]
  h8 qf[DQK / 16];
  {
    const half_t* qp = p.q + ((size_t)b * p.nq + (qvalid ? qrow : 0)) * p.q_ld + head * p.d;
#pragma unroll
    for (int ks = 0; ks < DQK / 16; ++ks) {
      const int dd = ks * 16 + 8 * fh;
      h8 v = {};
      if (qvalid && dd < p.d) v = *reinterpret_cast<const h8*>(qp + dd);
      qf[ks] = v;
    }
  }

  f16v o[DV / 32];
#pragma unroll
  for (int i = 0; i < DV / 32; ++i) o[i] = f16v{};
  float m_run = -1e30f, l_run = 0.f;

  const half_t* kbase = p.k + (size_t)b * p.nk * p.k_ld + head * p.d;
  const half_t* vbase = p.v + (size_t)b * p.nk * p.v_ld + head * p.d;
  const int ntiles = (p.nk + KT - 1) / KT;

  // transposed-read addressing for the V^T operand (32x32x16, A side):
  // group g = lane>>4 reads keys 16ks + 4*(g>>1) + 8*hi .. +3, columns 32*db + 16*(g&1) .. +15;
  // lane 4q+pp of the group supplies row q, columns 4pp..4pp+3
  const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
  const int vrow_off = 4 * (g >> 1) + q4;
  const int vcol_off = 16 * (g & 1) + 4 * pp;

  // K/V tiles are prefetched into registers one tile ahead (issue-early / write-late):
  // the global loads of tile t+1 are in flight while tile t is multiplied
  constexpr int KV_K = (KT * (DQK / 8) + 255) / 256, KV_V = (KT * (DV / 8) + 255) / 256;
  h8 pk_k[KV_K], pk_v[KV_V];
  auto fetch = [&](int key0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KV_K; ++i) {
      const int e = tid + 256 * i;
      const int kr = e / (DQK / 8), dd = (e - kr * (DQK / 8)) * 8;
      const int key = key0 + kr;
      h8 v = {};
      if (e < KT * (DQK / 8) && key < p.nk && dd < p.d) v = *reinterpret_cast<const h8*>(kbase + (size_t)key * p.k_ld + dd);
      pk_k[i] = v;
    }
#pragma unroll
    for (int i = 0; i < KV_V; ++i) {
      const int e = tid + 256 * i;
      const int kr = e / (DV / 8), dd = (e - kr * (DV / 8)) * 8;
      const int key = key0 + kr;
      h8 v = {};
      if (e < KT * (DV / 8) && key < p.nk) {
        if (dd + 8 <= p.d) {
          v = *reinterpret_cast<const h8*>(vbase + (size_t)key * p.v_ld + dd);
        } else if (ones_row && dd <= p.d && p.d < dd + 8) {
          v[p.d - dd] = (half_t)1.0f;       // ones column -> row sum of P in O^T row d
        }
      }
      pk_v[i] = v;
    }
  };
  constexpr bool PREFETCH = DV <= 128;   // d = 160 has no registers to spare
  if (PREFETCH) fetch(0);
  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * KT;
    __syncthreads();   // previous tile fully consumed
    if (!PREFETCH) {
      for (int e = tid; e < KT * (DQK / 8); e += 256) {
        const int kr = e / (DQK / 8), dd = (e - kr * (DQK / 8)) * 8;
        const int key = key0 + kr;
        h8 v = {};
        if (key < p.nk && dd < p.d) v = *reinterpret_cast<const h8*>(kbase + (size_t)key * p.k_ld + dd);
        *reinterpret_cast<h8*>(Ks + kr * KLD + dd) = v;
      }
      for (int e = tid; e < KT * (DV / 8); e += 256) {
        const int kr = e / (DV / 8), dd = (e - kr * (DV / 8)) * 8;
        const int key = key0 + kr;
        h8 v = {};
        if (key < p.nk) {
          if (dd + 8 <= p.d) v = *reinterpret_cast<const h8*>(vbase + (size_t)key * p.v_ld + dd);
          else if (ones_row && dd <= p.d && p.d < dd + 8) v[p.d - dd] = (half_t)1.0f;
        }
        *reinterpret_cast<h8*>(Vs + kr * VLD + dd) = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < KV_K; ++i) {
        const int e = tid + 256 * i;
        const int kr = e / (DQK / 8), dd = (e - kr * (DQK / 8)) * 8;
        if (e < KT * (DQK / 8)) *reinterpret_cast<h8*>(Ks + kr * KLD + dd) = pk_k[i];
      }
#pragma unroll
      for (int i = 0; i < KV_V; ++i) {
        const int e = tid + 256 * i;
        const int kr = e / (DV / 8), dd = (e - kr * (DV / 8)) * 8;
        if (e < KT * (DV / 8)) *reinterpret_cast<h8*>(Vs + kr * VLD + dd) = pk_v[i];
      }
    }
    __syncthreads();
    if (PREFETCH && t + 1 < ntiles) fetch(key0 + KT);

    // S^T = K Q^T for two 32-key sub-blocks (raw, unscaled scores)
    f16v s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = f16v{};
#pragma unroll
      for (int ks = 0; ks < DQK / 16; ++ks) {
        const h8 a = *reinterpret_cast<const h8*>(Ks + (kb * 32 + fr) * KLD + ks * 16 + 8 * fh);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[ks], s[kb], 0, 0, 0);
      }
    }
    if (key0 + KT > p.nk) {           // ragged last tile only
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (key >= p.nk) s[kb][r] = -1e30f;
        }
    }
    float mt = s[0][0];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kb][r]);
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    if (__any(m_new > m_run)) {       // rescale only when some row's max grew
      const float alpha = fast_exp2((m_run - m_new) * p.c);
      l_run *= alpha;
#pragma unroll
      for (int db = 0; db < DV / 32; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
      m_run = m_new;
    }
    const float nmc = -m_run * p.c;
    h8 pf[4];
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        h8 pk;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = fast_exp2(fmaf(s[kb][hlf * 8 + j], p.c, nmc));
          if (!ones_row) ls += e;
          pk[j] = (half_t)e;
        }
        pf[kb * 2 + hlf] = pk;
      }
    if (!ones_row) l_run += ls + __shfl_xor(ls, 32, 64);

    // O^T += V^T P^T ; element j of lane half fh in k-step ks is key 16ks + 8(j>>2) + 4fh + (j&3)
#pragma unroll
    for (int db = 0; db < DV / 32; ++db) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const half_t* base = Vs + (16 * ks + vrow_off) * VLD + 32 * db + vcol_off;
        const fp16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4f16(
            (__attribute__((address_space(3))) fp16x4_t*)(base));
        const fp16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4f16(
            (__attribute__((address_space(3))) fp16x4_t*)(base + 8 * VLD));
        const h4 lo4 = __builtin_bit_cast(h4, lo), hi4 = __builtin_bit_cast(h4, hi);
        const h8 a = __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, pf[ks], o[db], 0, 0, 0);
      }
    }
  }

  // row sum: explicit, or O^T row d (block d/32, row rho = d%32 held by lanes with h = (rho>>2)&1)
  float l = l_run;
  if (ones_row) {
    const int rho = p.d & 31, hsrc = (rho >> 2) & 1, rsel = (rho & 3) + 4 * (rho >> 3);
    float v = 0.f;
#pragma unroll
    for (int db = 0; db < DV / 32; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (db == (p.d >> 5) && r == rsel) v = o[db][r];
    l = __shfl(v, fr + 32 * hsrc, 64);
  }
  if (!qvalid) return;
  const float inv = 1.f / l;
  half_t* op = p.o + ((size_t)b * p.nq + qrow) * p.o_ld + head * p.d;
#pragma unroll
  for (int db = 0; db < DV / 32; ++db)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int dd = db * 32 + 8 * gg + 4 * fh;
      if (dd < p.d) {
        h4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (half_t)(o[db][4 * gg + j] * inv);
        *reinterpret_cast<h4*>(op + dd) = w;
      }
    }
}

template <int DQK, int DV>
int launch(const AttnParams& p, hipStream_t s) {
  dim3 grid((p.nq + 127) / 128, p.heads, p.batch);
  hipLaunchKernelGGL((attn_fwd_kernel<DQK, DV>), grid, dim3(256), 0, s, p);
  return check_launch("attn_fwd");
}

}  // namespace
}  // namespace sdk

using namespace sdk;

extern "C" int sdk_attention(const sdk_attention_args* a, sdk_stream_t stream) {
  if (!a || !a->q || !a->k || !a->v || !a->o) return fail(SDK_EINVAL, "attention: null pointer");
  if (a->head_dim <= 0 || a->head_dim % 8 || a->head_dim > 160)
    return fail(SDK_EINVAL, "attention: head_dim must be a multiple of 8 in [8, 160]");
  if (a->q_ld % 8 || a->k_ld % 8 || a->v_ld % 8 || a->o_ld % 4)
    return fail(SDK_EINVAL, "attention: row strides must be multiples of 8 (o: 4)");
  if (a->nk <= 0 || a->nq <= 0 || a->batch <= 0 || a->heads <= 0) return fail(SDK_EINVAL, "attention: empty");
  AttnParams p{(const half_t*)a->q, (const half_t*)a->k, (const half_t*)a->v, (half_t*)a->o,
               a->q_ld, a->k_ld, a->v_ld, a->o_ld, a->batch, a->heads, a->nq, a->nk, a->head_dim,
               a->scale * 1.4426950408889634f};
  hipStream_t s = (hipStream_t)stream;
  const int d = a->head_dim;
  if (d <= 16) return launch<16, 32>(p, s);
  if (d <= 32) return launch<32, 32>(p, s);
  if (d <= 48) return launch<48, 64>(p, s);
  if (d <= 64) return launch<64, 64>(p, s);
  if (d <= 80) return launch<80, 96>(p, s);
  if (d <= 96) return launch<96, 96>(p, s);
  if (d <= 128) return launch<128, 128>(p, s);
  return launch<160, 160>(p, s);
}
