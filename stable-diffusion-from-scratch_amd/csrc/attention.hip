// Flash-style attention forward for gfx950: O = softmax(scale*Q K^T) V, fp16 I/O,
// fp32 scores/softmax, v_mfma_f32_32x32x16_f16.
//
// Workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32
// rows.  Keys stream through LDS in tiles of 64.  The score tile is computed
// transposed, S^T = K Q^T (A = K rows from LDS, B = Q^T fragments held in
// registers for the whole loop), so each lane owns ONE query row: the softmax
// row max / row sum are in-register reductions plus one exchange with lane^32.
// The S^T accumulator is then, converted to fp16, directly the B operand of
// O^T += V^T P^T (the accumulator's row index = the key = the contraction
// index), with the V^T operand read from a transposed LDS image whose rows are
// padded to 136 B so the ds_read_b64 fragment reads are bank-conflict-free.
// Head dims that are not multiples of 16/32 (40, 80, 160 in SD-1) are
// zero-padded inside LDS/registers only; HBM traffic is the unpadded tensors.
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
  float scale_log2;
};

constexpr int KT = 64;          // keys per tile
constexpr int VLD = KT + 4;     // V^T row stride (halfs): 136 B

template <int DQK, int DV>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnParams p) {
  constexpr int KLD = DQK + 8;
  __shared__ __attribute__((aligned(16))) half_t Ks[KT * KLD];
  __shared__ __attribute__((aligned(16))) half_t Vt[DV * VLD];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  const int head = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int qrow = q0 + fr;
  const bool qvalid = qrow < p.nq;

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

  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * KT;
    __syncthreads();   // previous tile fully consumed
    // K tile: [64 keys][DQK] (coalesced 16-B chunks along d)
    for (int e = tid; e < KT * (DQK / 8); e += 256) {
      const int kr = e / (DQK / 8), c = e - kr * (DQK / 8);
      const int key = key0 + kr, dd = c * 8;
      h8 v = {};
      if (key < p.nk && dd < p.d) v = *reinterpret_cast<const h8*>(kbase + (size_t)key * p.k_ld + dd);
      *reinterpret_cast<h8*>(Ks + kr * KLD + dd) = v;
    }
    // V^T tile: [DV][64 keys]
    for (int e = tid; e < KT * (DV / 8); e += 256) {
      const int kr = e / (DV / 8), c = e - kr * (DV / 8);
      const int key = key0 + kr, dd = c * 8;
      h8 v = {};
      if (key < p.nk && dd < p.d) v = *reinterpret_cast<const h8*>(vbase + (size_t)key * p.v_ld + dd);
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(dd + j) * VLD + kr] = v[j];
    }
    __syncthreads();

    // S^T = K Q^T for two 32-key sub-blocks
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
    // scale, mask, row max (keys are rows: regs + lane^32)
    float mt = -1e30f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        float x = s[kb][r] * p.scale_log2;
        if (key >= p.nk) x = -1e30f;
        s[kb][r] = x;
        mt = fmaxf(mt, x);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float ls = 0.f;
    h8 pf[4];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        h8 pk;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = exp2f(s[kb][hlf * 8 + j] - m_new);
          ls += e;
          pk[j] = (half_t)e;
        }
        pf[kb * 2 + hlf] = pk;
      }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int db = 0; db < DV / 32; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[db][r] *= alpha;

    // O^T += V^T P^T ; k-step ks covers keys 16ks..16ks+15, element j of lane half fh is
    // key 16ks + 8(j>>2) + 4fh + (j&3) (accumulator row order)
#pragma unroll
    for (int db = 0; db < DV / 32; ++db) {
      const half_t* vr = Vt + (db * 32 + fr) * VLD + 4 * fh;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const h4 lo = *reinterpret_cast<const h4*>(vr + ks * 16);
        const h4 hi = *reinterpret_cast<const h4*>(vr + ks * 16 + 8);
        h8 a;
        a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
        a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, pf[ks], o[db], 0, 0, 0);
      }
    }
  }

  if (!qvalid) return;
  const float inv = 1.f / l_run;
  half_t* op = p.o + ((size_t)b * p.nq + qrow) * p.o_ld + head * p.d;
#pragma unroll
  for (int db = 0; db < DV / 32; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = db * 32 + 8 * g + 4 * fh;
      if (dd < p.d) {
        h4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (half_t)(o[db][4 * g + j] * inv);
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
