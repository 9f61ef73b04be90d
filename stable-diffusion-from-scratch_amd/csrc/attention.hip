// Flash-style attention forward for gfx950: O = softmax(scale*Q K^T) V, fp16 I/O,
// fp32 scores/softmax, v_mfma_f32_32x32x16_f16.
//
// Workgroup = NW waves = 32*NW query rows of one (batch, head); each wave owns 32
// rows.  Keys stream through a double-buffered LDS ring in tiles of 64 (one
// barrier per tile).  The score tile is computed transposed, S^T = K Q^T (A = K
// rows from LDS, B = Q^T fragments held in registers for the whole loop), so each
// lane owns ONE query row: the row max is an in-register v_max3 chain plus one
// v_permlane32_swap with the other half-wave.  The S^T accumulator, converted to
// fp16, is directly the B operand of O^T += V^T P^T (its row index = the key = the
// contraction index).  V stays row-major in LDS and the V^T operand is read with
// ds_read_b64_tr_b16 (the hardware transpose read).
//
// At SD's small head dims (d = 40: 14 MFMAs per 64-key tile against 32 exp per
// lane) the loop is VALU-bound, so everything that is not softmax arithmetic is
// taken off the vector pipe:
//  * K/V tiles are register-staged through buffer loads whose hardware range check
//    supplies the zero rows past nk (no per-element predicates); the per-thread
//    chunk offsets are computed once, a tile costs one v_add per load; the loads of
//    tile t+2 are issued after the LDS write of tile t+1 (issue-early / write-late);
//  * only the ceil(d/8) real 16-B chunks of each row are moved; the LDS padding up
//    to the MFMA widths is zeroed once, and when d < DV the padding holds a column
//    of ones so the row sum of P comes out of the PV MFMA (O^T row d);
//  * Q is pre-scaled by scale*log2(e) and the score MFMA chain is seeded with C = -m
//    (the running row max), so the accumulator is already the exp2 argument and the
//    common path is one v_exp_f32 per score; the max is only raised when a row's
//    tile max exceeds it by more than 8 (defer-max: P <= 256, exact in fp16), so the
//    rescale of O (and of the scores) is rare;
//  * key masking runs only in a ragged last tile.
#include <cstdlib>

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
  int causal;           // mask key > query
};

typedef __fp16 fp16x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

constexpr int KT = 64;                 // keys per tile
constexpr float DEFER = 8.0f;          // exp2-domain headroom before the running max is raised

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Buffer descriptor from provably wave-uniform words (readfirstlane of the pointer halves and
// the size), so hipcc keeps it in SGPRs instead of wrapping every load in a waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// CAUSAL is a template flag: the SD UNet's non-causal instantiations carry no masking code
template <int DQK, int DV, int NW, int QB, bool CAUSAL = false, bool STAG = false, int QSD = 0>
__global__ void __launch_bounds__(NW * 64, (STAG && DQK <= 64) ? 4 : QB == 2 ? 1 : 2) attn_fwd_kernel(AttnParams p) {
  static_assert(!STAG || (QB == 1 && NW % 2 == 0), "stagger: one query block per wave, paired waves");
  static_assert(QSD == 0 || (!CAUSAL && QSD % 8 == 0 && QSD < DQK), "score seed column: a padding column of Q/K");
  constexpr int NB = STAG ? 3 : 2;   // LDS stages
  constexpr int NT = NW * 64;
  constexpr int KLD = DQK + 8;                                       // K row stride (halfs)
  constexpr int VLD = ((DV * 2 / 64) % 2 == 0) ? DV + 32 : DV;       // V row stride: 64 or 192 B mod 256
  constexpr int KS = KT * KLD, STAGE = KS + KT * VLD;
  constexpr int SL = (KT * (DQK / 8) + NT - 1) / NT;                 // staging slots per thread (K and V each)
  __shared__ __attribute__((aligned(16))) half_t smem[NB * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  // 1-D grid, XCD-aware: the q-blocks of one (batch, head) are consecutive logical blocks and
  // xcd_remap puts consecutive logical blocks on one XCD, so that head's K/V is fetched into one
  // L2 instead of into all eight (blocks are dealt round-robin over the XCDs)
  constexpr int ROWS = 32 * QB * NW;
  const int nqb = (p.nq + ROWS - 1) / ROWS;
  const int lin = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int qblk = lin % nqb, bh = lin / nqb;
  const int head = bh % p.heads, b = bh / p.heads;
  const int q0 = qblk * ROWS + wave * 32 * QB;      // this wave's first query row
  const int d = p.d, nch = (d + 7) >> 3;   // real 16-B chunks per row
  const bool ones_row = d < DV;            // row sum from the PV MFMA (ones column at d)

  // zero the LDS padding of every stage once (K columns >= 8*nch, V columns >= 8*nch),
  // with the ones column at d; the staged chunks never touch it
  for (int e = tid; e < NB * KT; e += NT) {
    half_t* kr = smem + (e / KT) * STAGE + (e % KT) * KLD;
    for (int c = nch * 8; c < KLD; ++c) kr[c] = (half_t)((QSD > 0 && c == QSD) ? 1.0f : 0.0f);
    half_t* vr = smem + (e / KT) * STAGE + KS + (e % KT) * VLD;
    for (int c = nch * 8; c < VLD; ++c) vr[c] = (half_t)((ones_row && c == d) ? 1.0f : 0.0f);
  }

  // staging slots: chunk e = tid + NT*i of the tile = (key e/nch, chunk e%nch) of K and of V
  const __amdgpu_buffer_rsrc_t rk = rsrc(p.k + (size_t)b * p.nk * p.k_ld, (long long)p.nk * p.k_ld * 2);
  const __amdgpu_buffer_rsrc_t rv = rsrc(p.v + (size_t)b * p.nk * p.v_ld, (long long)p.nk * p.v_ld * 2);
  unsigned gk[SL], gv[SL];
  int lk[SL], lv[SL];
#pragma unroll
  for (int i = 0; i < SL; ++i) {
    const int e = tid + NT * i;
    const int key = e / nch, c = e - key * nch;
    const bool ok = e < KT * nch;
    gk[i] = (unsigned)((key * p.k_ld + head * d + c * 8) * 2);
    gv[i] = (unsigned)((key * p.v_ld + head * d + c * 8) * 2);
    lk[i] = ok ? key * KLD + c * 8 : -1;
    lv[i] = KS + key * VLD + c * 8;
  }
  const unsigned kstep = (unsigned)(KT * p.k_ld * 2), vstep = (unsigned)(KT * p.v_ld * 2);
  u4 rk_[SL], rv_[SL];
  auto fetch = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < SL; ++i)
      if (lk[i] >= 0) {
        rk_[i] = __builtin_amdgcn_raw_buffer_load_b128(rk, gk[i] + t * kstep, 0, 0);
        rv_[i] = __builtin_amdgcn_raw_buffer_load_b128(rv, gv[i] + t * vstep, 0, 0);
      }
  };
  auto stage = [&](int buf) __attribute__((always_inline)) {
    half_t* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < SL; ++i)
      if (lk[i] >= 0) {
        *reinterpret_cast<u4*>(st + lk[i]) = rk_[i];
        *reinterpret_cast<u4*>(st + lv[i]) = rv_[i];
      }
  };

  // Q^T fragments (B operand) of each 32-row block: lane holds c*Q[row][ks*16 + 8*fh + j]
  h8 qf[QB][DQK / 16];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int row = q0 + qb * 32 + fr;
    const half_t* qp = p.q + ((size_t)b * p.nq + (row < p.nq ? row : 0)) * p.q_ld + head * d;
#pragma unroll
    for (int ks = 0; ks < DQK / 16; ++ks) {
      const int dd = ks * 16 + 8 * fh;
      h8 v = {};
      if (row < p.nq && dd < d) v = *reinterpret_cast<const h8*>(qp + dd);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] * p.c);   // scores land in the exp2 domain
      qf[qb][ks] = v;
    }
  }

  f16v o[QB][DV / 32];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb)
#pragma unroll
    for (int i = 0; i < DV / 32; ++i) o[qb][i] = f16v{};
  // running max m (exp2 domain, per query row = per lane); the score chain is seeded with
  // C = -m, so the MFMA emits s' = c*s - m and the common path is a bare v_exp per score.
  // QSD > 0 (d < DQK, d = QSD): -m rides in Q's padding column QSD against a column of ones in K
  // instead (no 16-register seed, no seed moves per tile); m is then the fp16 value in Q, and
  // every rescale uses the difference of those fp16 values, which softmax's shift invariance makes
  // exact
  float m_run[QB], l_run[QB];
  f16v negm[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) { m_run[qb] = 0.f; l_run[qb] = 0.f; negm[qb] = f16v{}; }
  int ntiles = (p.nk + KT - 1) / KT;
  if constexpr (CAUSAL) {   // tiles past the workgroup's last query row hold only masked keys
    const int qlast = min(p.nq, (qblk + 1) * ROWS) - 1;
    ntiles = min(ntiles, qlast / KT + 1);
  }

  // transposed-read addressing for the V^T operand (32x32x16, A side):
  // group g = lane>>4 reads keys 16ks + 4*(g>>1) + 8*hi .. +3, columns 32*db + 16*(g&1) .. +15;
  // lane 4q+pp of the group supplies row q, columns 4pp..4pp+3
  const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
  const int vrow_off = 4 * (g >> 1) + q4;
  const int vcol_off = 16 * (g & 1) + 4 * pp;

  fetch(0);
  stage(0);
  if (ntiles > 1) fetch(1);
  __syncthreads();
#if !defined(SDK_NO_PRIO)
  // static priority for the second-dispatched half of an 8-wave group (it otherwise loses VALU
  // arbitration to its SIMD partner every tile, MI355X_MICROARCH.md two-waves item 4; UNet step
  // -0.2 %, profiles/r2_static_priority_ab.txt)
  if (NW == 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif

  // the loop's four parts; s / pf are loop-carried so that the lagging half (STAG) can hold a
  // tile's second score block and first P block across the barrier
  f16v s[QB][2];
  h8 pf[QB][4];
  auto qk = [&](const half_t* Ks) __attribute__((always_inline)) {
    // S'^T = K (cQ)^T - m for two 32-key sub-blocks of every query block; each K fragment
    // is read once for all QB blocks
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ks = 0; ks < DQK / 16; ++ks) {
        const h8 a = *reinterpret_cast<const h8*>(Ks + (kb * 32 + fr) * KLD + ks * 16 + 8 * fh);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          s[qb][kb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[qb][ks], ks > 0 ? s[qb][kb] : QSD > 0 ? f16v{} : negm[qb], 0, 0, 0);
      }
  };
  auto exp_block = [&](int kb) __attribute__((always_inline)) {
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      float ls = 0.f;
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        h8 pk;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = fast_exp2(s[qb][kb][hlf * 8 + j]);
          if (!ones_row) ls += e;
          pk[j] = (half_t)e;
        }
        pf[qb][kb * 2 + hlf] = pk;
      }
      if (!ones_row) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(ls), __float_as_uint(ls), false, false);
        l_run[qb] += __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
      }
    }
  };
  // mask, tile max, (rare) rescale, then P of the first 32-key block
  auto softmax_a = [&](int t) __attribute__((always_inline)) {
    const int key0 = t * KT;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      if constexpr (CAUSAL) {
        const int qrow = q0 + qb * 32 + fr;
        if (key0 + KT > p.nk || key0 + KT - 1 > q0 + qb * 32) {   // ragged / diagonal tiles only
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
              if (key >= p.nk || key > qrow) s[qb][kb][r] = -1e30f;
            }
        }
      } else if (key0 + KT > p.nk) {           // ragged last tile only
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            if (key >= p.nk) s[qb][kb][r] = -1e30f;
          }
      }
      float mt = fmaxf(s[qb][0][0], s[qb][0][1]);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = (kb == 0 ? 2 : 0); r < 16; r += 2) mt = fmaxf(fmaxf(mt, s[qb][kb][r]), s[qb][kb][r + 1]);
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mt), __float_as_uint(mt), false, false);
        mt = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      // raise the running max only on the first tile or past the headroom (P <= 2^DEFER)
      if (t == 0 || __any(mt > DEFER)) {
        float dm = t == 0 ? mt : fmaxf(mt, 0.f);
        if constexpr (QSD > 0) {
          const half_t mh = (half_t)(-(m_run[qb] + dm));
          dm = -(float)mh - m_run[qb];
          if (fh == ((QSD & 15) >> 3)) qf[qb][QSD >> 4][QSD & 7] = mh;
        }
        const float alpha = fast_exp2(-dm);
        l_run[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < DV / 32; ++db)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[qb][db][r] *= alpha;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) s[qb][kb][r] -= dm;
        m_run[qb] += dm;
        if constexpr (QSD == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) negm[qb][r] = -m_run[qb];
        }
      }
    }
    exp_block(0);
  };
  // O^T += V^T P^T ; element j of lane half fh in k-step ks is key 16ks + 8(j>>2) + 4fh + (j&3);
  // each V^T fragment (ds_read_b64_tr_b16 pair) is read once for all QB blocks
  auto pv = [&](const half_t* Vs) __attribute__((always_inline)) {
#pragma unroll
    for (int db = 0; db < DV / 32; ++db) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const half_t* base = Vs + (16 * ks + vrow_off) * VLD + 32 * db + vcol_off;
        const fp16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4_t*)(base));
        const fp16x4_t hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4_t*)(base + 8 * VLD));
        const h4 lo4 = __builtin_bit_cast(h4, lo), hi4 = __builtin_bit_cast(h4, hi);
        const h8 a = __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) o[qb][db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, pf[qb][ks], o[qb][db], 0, 0, 0);
      }
    }
  };

  // STAG: waves NW/2.. run half a tile behind their SIMD partners (waves w and w + NW/2 share a
  // SIMD): the lead half computes [QK_t | softmax_t | PV_t], the lag half [exp2_{t-1} | PV_{t-1}
  // QK_t | max/exp1_t], so one wave's matrix phase meets the other's v_exp phase
  // (MI355X_MICROARCH.md two-waves item 9).  Tile t-1's V stays in its stage for the lag half's
  // PV during iteration t: three stages instead of two.
  const bool lag = STAG && wave >= NW / 2;
  int bcur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const int bnext = bcur + 1 == NB ? 0 : bcur + 1;
    const int bprev = bcur == 0 ? NB - 1 : bcur - 1;
    const half_t* Ks = smem + bcur * STAGE;
    if (lag && t > 0) {
      exp_block(1);
      pv(smem + bprev * STAGE + KS);
    }
    qk(Ks);
    // tile t+1 (in registers since last iteration) -> its stage; then issue t+2
    if (t + 1 < ntiles) {
      stage(bnext);
      if (t + 2 < ntiles) fetch(t + 2);
    }
    softmax_a(t);
    if (!lag) {
      exp_block(1);
      pv(Ks + KS);
    }
    __syncthreads();   // stage t+1 visible; with two stages, stage t fully read before it is restaged
    bcur = bnext;
  }
  if (lag && ntiles > 0) {
    exp_block(1);
    pv(smem + (bcur == 0 ? NB - 1 : bcur - 1) * STAGE + KS);
  }

#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    // row sum: explicit, or O^T row d (block d/32, row rho = d%32 held by lanes with h = (rho>>2)&1)
    float l = l_run[qb];
    if (ones_row) {
      const int rho = d & 31, hsrc = (rho >> 2) & 1, rsel = (rho & 3) + 4 * (rho >> 3);
      float v = 0.f;
#pragma unroll
      for (int db = 0; db < DV / 32; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (db == (d >> 5) && r == rsel) v = o[qb][db][r];
      l = __shfl(v, fr + 32 * hsrc, 64);
    }
    const int row = q0 + qb * 32 + fr;
    if (row < p.nq) {
      const float inv = 1.f / l;
      half_t* op = p.o + ((size_t)b * p.nq + row) * p.o_ld + head * d;
#pragma unroll
      for (int db = 0; db < DV / 32; ++db)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int dd = db * 32 + 8 * gg + 4 * fh;
          if (dd < d) {
            h4 w;
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = (half_t)(o[qb][db][4 * gg + j] * inv);
            *reinterpret_cast<h4*>(op + dd) = w;
          }
        }
    }
  }
}

template <int DQK, int DV, int NW, int QB, bool STAG = false, int QSD = 0>
int launch(const AttnParams& p, hipStream_t s) {
  constexpr int ROWS = 32 * QB * NW;
  const long long blocks = (long long)((p.nq + ROWS - 1) / ROWS) * p.heads * p.batch;
  if (blocks > 0x7fffffffLL) return fail(SDK_EINVAL, "attention: grid too large");
  dim3 grid((unsigned)blocks);
  if (p.causal) {
    if constexpr (QB == 1) {   // the CLIP text tower's head sizes; other forms are not instantiated
      hipLaunchKernelGGL((attn_fwd_kernel<DQK, DV, NW, QB, true>), grid, dim3(NW * 64), 0, s, p);
      return check_launch("attn_fwd_causal");
    }
    return fail(SDK_EINVAL, "attention: causal needs the one-block-per-wave form");
  }
  hipLaunchKernelGGL((attn_fwd_kernel<DQK, DV, NW, QB, false, STAG, QSD>), grid, dim3(NW * 64), 0, s, p);
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
  if (a->heads * a->head_dim > a->k_ld || a->heads * a->head_dim > a->v_ld || a->heads * a->head_dim > a->q_ld)
    return fail(SDK_EINVAL, "attention: row stride smaller than heads*head_dim");
  if ((double)a->nk * std::max(a->k_ld, a->v_ld) * 2 >= 2147483647.0)
    return fail(SDK_EINVAL, "attention: one image's K/V exceeds the 2 GiB buffer range");
  AttnParams p{(const half_t*)a->q, (const half_t*)a->k, (const half_t*)a->v, (half_t*)a->o,
               a->q_ld, a->k_ld, a->v_ld, a->o_ld, a->batch, a->heads, a->nq, a->nk, a->head_dim,
               a->scale * 1.4426950408889634f, a->causal ? 1 : 0};
  hipStream_t s = (hipStream_t)stream;
  const int d = a->head_dim;
  // one 32-row query block per wave at 3-4 waves per SIMD; SDK_ATTN_QB=2 selects two blocks per
  // wave at one wave per SIMD (shared K/V fragments; measured 1.6x slower at d = 40 under hipcc's
  // scheduling, kept as a tuning knob)
  static const int qb2 = getenv("SDK_ATTN_QB") && atoi(getenv("SDK_ATTN_QB")) == 2;
  if (d <= 16) return launch<16, 32, 4, 1>(p, s);
  if (d <= 32) return launch<32, 32, 4, 1>(p, s);
  // d <= 80: 8-wave workgroups (half the staging registers: d = 40 127 VGPRs = 4 waves per SIMD,
  // 547 vs 623 us for the 4-wave form at SD-1's 64x64 level); SDK_ATTN_NW=4 selects the latter.
  // d = 160 keeps 4 waves: at 256 query rows one 8-wave group per head would idle half the CUs
  static const int nw4 = getenv("SDK_ATTN_NW") && atoi(getenv("SDK_ATTN_NW")) == 4;
  // SDK_ATTN_STAG=1: the 8-wave forms with the lag half staggered by half a tile (three stages).  Default on
  // for 48 < d <= 80 (same-box A/Bs: d = 64 975 vs 1060 us at SD-2's 96x96 level, d = 40 582 vs 521 us,
  // profiles/r3_attn_stag_ab.txt; d = 80 at SD-1's 32x32 level 67.1-67.5 vs 69.3 us, profiles/r5_attn80_ab.txt);
  // SDK_ATTN_STAG=0 / 1 forces it off / on everywhere
  static const int stag_env = getenv("SDK_ATTN_STAG") ? atoi(getenv("SDK_ATTN_STAG")) : -1;
  const int stag = stag_env == 1 || (stag_env < 0 && d > 48 && d <= 80);
  if (d <= 48)
    return qb2 ? launch<48, 64, 4, 2>(p, s)
           : nw4  ? launch<48, 64, 4, 1>(p, s)
           : d == 40 ? (stag ? launch<48, 64, 8, 1, true, 40>(p, s) : launch<48, 64, 8, 1, false, 40>(p, s))
           : stag ? launch<48, 64, 8, 1, true>(p, s) : launch<48, 64, 8, 1>(p, s);
  if (d <= 64)
    return nw4 ? launch<64, 64, 4, 1>(p, s) : stag ? launch<64, 64, 8, 1, true>(p, s) : launch<64, 64, 8, 1>(p, s);
  if (d <= 80)   // 165 vs 189 VGPRs
    return nw4 ? launch<80, 96, 4, 1>(p, s) : stag ? launch<80, 96, 8, 1, true>(p, s) : launch<80, 96, 8, 1>(p, s);
  if (d <= 96) return launch<96, 96, 4, 1>(p, s);
  if (d <= 128) return launch<128, 128, 4, 1>(p, s);
  return launch<160, 160, 4, 1>(p, s);
}
