// GroupNorm statistics and LayerNorm for gfx950 (HBM-bound, NHWC fp16 in).
//
// GroupNorm is split: this file produces per-(batch, channel) scale/shift
// (gamma*rstd, beta - mean*gamma*rstd) and the conv kernel applies them (plus
// SiLU) while staging its A tile, so the normalised tensor never round-trips
// through HBM.  Statistics: pass 1 streams the tensor once with 16-B loads,
// one thread per 8 channels, accumulating pivot-shifted sums (pivot = the
// channel's value at pixel 0 of the image, so E[x^2]-E[x]^2 does not cancel
// for offset activations); pass 2 merges chunks in double per channel and
// channels into groups with Chan's parallel-variance formula.
#include <algorithm>
#include <cstdlib>

#include <map>
#include <mutex>

#include "common.h"

namespace sdk {
namespace {

constexpr int GN_U = 8;   // independent 16-B row loads in flight per thread

// Row chunking: a block covers `chunk_rows` pixels of one image; a thread owns 8 channels
// of every ry-th row in it and keeps GN_U loads in flight; ~1500 blocks per launch so
// the whole tensor streams at HBM rate instead of a latency-bound 32-row walk.
struct GnGeom {
  int c8, nv, ry, chunk_rows, nchunks;
};

GnGeom gn_geom(int batch, int hw, int channels) {
  GnGeom g;
  g.c8 = channels / 8;
  g.nv = (g.c8 + 255) / 256;
  g.ry = g.nv > 1 ? 1 : std::max(1, 256 / g.c8);
  const int step = g.ry * GN_U;
  const int want = std::max(1, (1536 + batch - 1) / std::max(batch, 1));
  const int per = std::max(1, (hw + want - 1) / want);
  g.chunk_rows = (per + step - 1) / step * step;
  g.nchunks = (hw + g.chunk_rows - 1) / g.chunk_rows;
  return g;
}

__device__ __forceinline__ h8 load_px(const half_t* s0, const half_t* s1, int c_split, int ld0, int ld1,
                                      size_t pix, int c) {
  if (c < c_split) return *reinterpret_cast<const h8*>(s0 + pix * ld0 + c);
  return *reinterpret_cast<const h8*>(s1 + pix * ld1 + (c - c_split));
}

// grid (nchunks, batch); writes partial[b][chunk][c] = (S1, S2) of (x - pivot_c)
__global__ void __launch_bounds__(256) gn_partial_kernel(const half_t* s0, const half_t* s1, int c_split, int ld0,
                                                         int ld1, int hw, int channels, GnGeom g, float2* partial) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [ry][c8*8] x 2
  const int tid = threadIdx.x, chunk = blockIdx.x, b = blockIdx.y;
  const int r0 = chunk * g.chunk_rows, r1 = min(hw, r0 + g.chunk_rows);
  const size_t img = (size_t)b * hw;
  const int ysub = tid / g.c8;
  for (int vi = 0; vi < g.nv; ++vi) {
    const int vec = g.nv > 1 ? tid + vi * 256 : tid % g.c8;
    const bool active = vec < g.c8 && ysub < g.ry;
    float sum[8], sq[8], piv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sum[j] = 0.f; sq[j] = 0.f; piv[j] = 0.f; }
    if (active) {
      const int c = vec * 8;
      const h8 pv = load_px(s0, s1, c_split, ld0, ld1, img, c);
#pragma unroll
      for (int j = 0; j < 8; ++j) piv[j] = (float)pv[j];
      const int rstart = r0 + (g.nv > 1 ? 0 : ysub);
      const int rstep = g.nv > 1 ? 1 : g.ry;
      for (int r = rstart; r < r1; r += GN_U * rstep) {
        h8 v[GN_U];
#pragma unroll
        for (int u = 0; u < GN_U; ++u) {
          const int rr = r + u * rstep;
          v[u] = rr < r1 ? load_px(s0, s1, c_split, ld0, ld1, img + rr, c) : pv;   // pivot adds 0
        }
#pragma unroll
        for (int u = 0; u < GN_U; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = (float)v[u][j] - piv[j];
            sum[j] += d;
            sq[j] += d * d;
          }
      }
    }
    if (g.ry == 1) {
      if (active) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          partial[((size_t)b * g.nchunks + chunk) * channels + vec * 8 + j] = make_float2(sum[j], sq[j]);
      }
      continue;
    }
    // reduce over ysub through LDS
    const int C = g.c8 * 8;
    if (active) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[ysub * C + vec * 8 + j] = sum[j];
        red[(g.ry + ysub) * C + vec * 8 + j] = sq[j];
      }
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      float a = 0.f, q = 0.f;
      for (int y = 0; y < g.ry; ++y) { a += red[y * C + c]; q += red[(g.ry + y) * C + c]; }
      partial[((size_t)b * g.nchunks + chunk) * channels + c] = make_float2(a, q);
    }
  }
}

// grid (groups, batch), 256 threads: the cg channels of the group get tpc = 256/cg (power of
// two, <= 64) consecutive lanes each; a channel's lanes sum disjoint chunk subsets (all loads
// independent, so they stream instead of one dependent round trip per channel), reduce with
// xor shuffles in double, then wave 0 Chan-merges the group's channels.
__device__ __forceinline__ double wave_sum_d(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ void __launch_bounds__(256) gn_finalize_kernel(const half_t* s0, const half_t* s1, int c_split, int ld0,
                                                          int ld1, int hw, int channels, int groups, GnGeom g,
                                                          const float2* partial, float eps, const float* gamma,
                                                          const float* beta, float* scale, float* shift) {
  __shared__ double cm[256], cq[256];   // per-channel mean, M2 (cg <= 256)
  const int grp = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = channels / groups, c0 = grp * cg;
  const size_t img = (size_t)b * hw;
  const double n = (double)hw;
  int tpc = 64;
  while (tpc > 1 && tpc * cg > 256) tpc >>= 1;
  const int ci = tid / tpc, sub = tid - ci * tpc;
  for (int cbase = 0; cbase < cg; cbase += 256 / tpc) {
    const int cc = cbase + ci;
    const bool act = ci < 256 / tpc && cc < cg;
    double a1 = 0.0, a2 = 0.0;
    if (act) {
      const float2* pp = partial + (size_t)b * g.nchunks * channels + c0 + cc;
      for (int k = sub; k < g.nchunks; k += tpc) {
        const float2 v = pp[(size_t)k * channels];
        a1 += v.x;
        a2 += v.y;
      }
    }
    for (int off = tpc >> 1; off > 0; off >>= 1) {   // lanes of one channel are contiguous and aligned
      a1 += __shfl_xor(a1, off, 64);
      a2 += __shfl_xor(a2, off, 64);
    }
    if (act && sub == 0) {
      const int c = c0 + cc;
      // the pivot pass 1 subtracted: this channel's value at pixel 0 of the image
      const float piv = c < c_split ? (float)s0[img * ld0 + c] : (float)s1[img * ld1 + (c - c_split)];
      cm[cc] = (double)piv + a1 / n;
      cq[cc] = a2 - a1 * a1 / n;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  double mean_sum = 0.0, m2_sum = 0.0, msq_sum = 0.0;
  for (int ci = lane; ci < cg; ci += 64) {
    mean_sum += cm[ci];
    msq_sum += cm[ci] * cm[ci];
    m2_sum += cq[ci];
  }
  mean_sum = wave_sum_d(mean_sum);
  msq_sum = wave_sum_d(msq_sum);
  m2_sum = wave_sum_d(m2_sum);
  const double mg = mean_sum / cg;
  // sum over channels of n*(mc - mg)^2 = n*(sum mc^2 - cg*mg^2)
  double m2g = m2_sum + n * (msq_sum - cg * mg * mg);
  if (m2g < 0) m2g = 0;
  const double var = m2g / (n * cg);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float meanf = (float)mg;
  for (int ci = lane; ci < cg; ci += 64) {
    const int c = c0 + ci;
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    const float sc = gm * rstd;
    scale[(size_t)b * channels + c] = sc;
    shift[(size_t)b * channels + c] = bt - meanf * sc;
  }
}

// Single-launch GroupNorm statistics for the UNet's small levels (hw <= 4096 pixels per image),
// where the two-kernel form is latency-bound (partial + finalize ~17 us of kernel time at 8x8
// for 2.6 MB).  grid (slices, batch): one workgroup owns ONE image and a slice of `gps` whole
// groups (gps*cg channels, a multiple of 8), streams all its pixels (thread = 8 channels of every
// rp-th pixel, pivot-shifted fp32 sums, 8 loads in flight), reduces the rp partial rows through
// LDS, merges channels into groups with Chan's formula in double and writes scale/shift — no
// workspace, no second launch.
constexpr int GNF_T = 512;
// APPLY: the same workgroup then normalises its slice (+ SiLU) straight into y — the image's slice
// is L2-hot from the statistics sweep — optionally into a zero-bordered [h+2pad][w+2pad] image
// for a pad-0 3x3 conv; GroupNorm at the small levels is then ONE launch instead of stats + apply.
template <bool APPLY>
__global__ void __launch_bounds__(GNF_T) gn_stats_fused_kernel(const half_t* s0, const half_t* s1, int c_split,
                                                               int ld0, int ld1, int hw, int channels, int cg,
                                                               int gps, float eps, const float* gamma,
                                                               const float* beta, float* scale, float* shift,
                                                               int silu, half_t* y, int ldy, int h, int w, int pad) {
  __shared__ float2 red[GNF_T * 8];                 // [row-set][slice channel] partial (S1, S2)
  __shared__ double cmean[512], cm2[512];           // per slice channel (slice <= 512 channels)
  const int tid = threadIdx.x, b = blockIdx.y;
  const int sc = gps * cg, c0 = blockIdx.x * sc;     // slice channels, first channel
  const int cv = sc / 8, rp = GNF_T / cv;            // vectors per pixel, pixels in parallel
  const int v = tid % cv, r0 = tid / cv;
  const bool active = r0 < rp;
  const size_t img = (size_t)b * hw;
  const int c = c0 + 8 * v;
  float sum[8], sq[8], piv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sum[j] = 0.f; sq[j] = 0.f; piv[j] = 0.f; }
  if (active) {
    const h8 pv = load_px(s0, s1, c_split, ld0, ld1, img, c);
#pragma unroll
    for (int j = 0; j < 8; ++j) piv[j] = (float)pv[j];
    constexpr int U = 8;
    for (int r = r0; r < hw; r += U * rp) {
      h8 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * rp;
        x[u] = rr < hw ? load_px(s0, s1, c_split, ld0, ld1, img + rr, c) : pv;   // the pivot adds 0
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)x[u][j] - piv[j];
          sum[j] += d;
          sq[j] += d * d;
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[r0 * sc + 8 * v + j] = make_float2(sum[j], sq[j]);
  }
  __syncthreads();
  const double n = (double)hw;
  for (int k = tid; k < sc; k += GNF_T) {           // per slice channel: merge the rp row sets
    double a1 = 0.0, a2 = 0.0;
    for (int r = 0; r < rp; ++r) {
      const float2 q = red[r * sc + k];
      a1 += q.x;
      a2 += q.y;
    }
    const int cc = c0 + k;
    const float p0 = cc < c_split ? (float)s0[img * ld0 + cc] : (float)s1[img * ld1 + (cc - c_split)];
    cmean[k] = (double)p0 + a1 / n;
    cm2[k] = a2 - a1 * a1 / n;
  }
  __syncthreads();
  for (int g = tid; g < gps; g += GNF_T) {          // per group: Chan merge of its cg channels
    double ms = 0.0, m2 = 0.0;
    for (int k = 0; k < cg; ++k) ms += cmean[g * cg + k];
    const double mg = ms / cg;
    for (int k = 0; k < cg; ++k) {
      const double dm = cmean[g * cg + k] - mg;
      m2 += cm2[g * cg + k] + n * dm * dm;
    }
    const double var = (m2 > 0 ? m2 : 0.0) / (n * cg);
    cmean[g * cg] = mg;                              // reuse: group mean / rstd at the group's first slot
    cm2[g * cg] = 1.0 / sqrt(var + (double)eps);
  }
  __syncthreads();
  for (int k = tid; k < sc; k += GNF_T) {
    const int g = k / cg, cc = c0 + k;
    const float rstd = (float)cm2[g * cg], meanf = (float)cmean[g * cg];
    const float gm = gamma ? gamma[cc] : 1.f, bt = beta ? beta[cc] : 0.f;
    const float s = gm * rstd;
    if constexpr (APPLY) {
      red[k] = make_float2(s, bt - meanf * s);       // the row sets were merged above: reuse as (scale, shift)
    } else {
      scale[(size_t)b * channels + cc] = s;
      shift[(size_t)b * channels + cc] = bt - meanf * s;
    }
  }
  if constexpr (APPLY) {
    __syncthreads();
    if (!active) return;
    float sa[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 t = red[8 * v + j];
      sa[j] = t.x;
      sh[j] = t.y;
    }
    const int wp = w + 2 * pad, npix = (h + 2 * pad) * wp;
    half_t* yb = y + (size_t)b * npix * ldy + c;
    constexpr int U = 4;
    for (int r = r0; r < npix; r += U * rp) {
      h8 x[U];
      bool in[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * rp;
        const int py = rr / wp - pad, px = rr - (rr / wp) * wp - pad;
        in[u] = rr < npix && (unsigned)py < (unsigned)h && (unsigned)px < (unsigned)w;
        x[u] = in[u] ? load_px(s0, s1, c_split, ld0, ld1, img + (size_t)py * w + px, c) : h8{};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * rp;
        if (rr >= npix) continue;
        h8 o = {};
        if (in[u]) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = (float)x[u][j] * sa[j] + sh[j];
            if (silu) t = t * __builtin_amdgcn_rcpf(1.0f + __expf(-t));
            o[j] = (half_t)t;
          }
        }
        *reinterpret_cast<h8*>(yb + (size_t)rr * ldy) = o;
      }
    }
  }
}

// GroupNorm statistics merged from the producing convs' per-chunk channel statistics
// (sdk_conv_args.gn_partial: [batch][nch][C] (mean, M2) over hw/nch pixels each; one array per
// concat source) — no pass over the tensor.  grid (groups, batch): per channel a Chan merge of its
// chunks in double, then wave 0 merges the group's channels as gn_finalize_kernel does.
__global__ void __launch_bounds__(256) gn_finalize_part_kernel(const float2* part0, int nch0, const float2* part1,
                                                               int nch1, int c_split, int hw, int channels,
                                                               int groups, float eps, const float* gamma,
                                                               const float* beta, float* scale, float* shift) {
  __shared__ double cm[256], cq[256];   // per-channel mean, M2 over the image (cg <= 256)
  const int grp = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = channels / groups, c0 = grp * cg;
  // tpc consecutive lanes per channel (power of two, <= 64) take disjoint chunk subsets — all loads
  // independent — then merge with xor shuffles (Chan, counts carried along)
  int tpc = 64;
  while (tpc > 1 && tpc * cg > 256) tpc >>= 1;
  const int ci = tid / tpc, sub = tid - ci * tpc;
  for (int cbase = 0; cbase < cg; cbase += 256 / tpc) {
    const int cc = cbase + ci;
    const bool act = ci < 256 / tpc && cc < cg;
    double mean = 0.0, m2 = 0.0, n = 0.0;
    if (act) {
      const int c = c0 + cc;
      const bool second = c >= c_split;
      const float2* pp = second ? part1 : part0;
      const int nch = second ? nch1 : nch0, cs = second ? channels - c_split : c_split, cl = second ? c - c_split : c;
      const double rows = (double)hw / nch;
      for (int k = sub; k < nch; k += tpc) {
        const float2 q = pp[((size_t)b * nch + k) * cs + cl];
        const double dl = (double)q.x - mean, nn = n + rows, f = rows / nn;
        mean += dl * f;
        m2 += (double)q.y + dl * dl * n * f;
        n = nn;
      }
    }
    for (int off = tpc >> 1; off > 0; off >>= 1) {   // lanes of one channel are contiguous and aligned
      const double mb = __shfl_xor(mean, off, 64), qb = __shfl_xor(m2, off, 64), nb = __shfl_xor(n, off, 64);
      const double nn = n + nb;
      if (nn > 0) {
        const double dl = mb - mean, f = nb / nn;
        mean += dl * f;
        m2 += qb + dl * dl * n * f;
      }
      n = nn;
    }
    if (act && sub == 0) {
      cm[cc] = mean;
      cq[cc] = m2;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  const double n = (double)hw;
  double mean_sum = 0.0;
  for (int ci = lane; ci < cg; ci += 64) mean_sum += cm[ci];
  mean_sum = wave_sum_d(mean_sum);
  const double mg = mean_sum / cg;
  double m2g = 0.0;
  for (int ci = lane; ci < cg; ci += 64) {
    const double dm = cm[ci] - mg;
    m2g += cq[ci] + n * dm * dm;
  }
  m2g = wave_sum_d(m2g);
  const double var = (m2g > 0 ? m2g : 0.0) / (n * cg);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float meanf = (float)mg;
  for (int ci = lane; ci < cg; ci += 64) {
    const int c = c0 + ci;
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    const float sc = gm * rstd;
    scale[(size_t)b * channels + c] = sc;
    shift[(size_t)b * channels + c] = bt - meanf * sc;
  }
}

// GroupNorm apply whose prologue merges the producers' partials itself (one launch instead of
// gn_finalize_part + apply: at the 32x32 / 16x16 / 8x8 levels both are latency-floor launches).
// grid (groups / gps channel slices, batch, row splits of the output image): a workgroup Chan-merges
// its slice's channels over the partial chunks (double, chunk order), merges the slice's groups from
// the channels exactly as gn_finalize_part_kernel does, keeps scale / shift in LDS and normalises
// (+ SiLU) its rows of the (optionally zero-bordered) image for the slice's channels.  The partials
// are read once per workgroup from L2 (nch x slice x 8 B), so the path is taken only for hw up to
// SDK_GN_PART_FUSED_MAX_HW (default 256: the 16x16 / 8x8 levels, 7.6 vs 9.8 us per GroupNorm at 8x8;
// at 32x32 the per-workgroup prologue repeats over too many row splits: 16-17 vs 15.4 us, measured
// same-box, UNet step 21.07 -> 21.01 ms at 256 and 21.10 at 1024).
constexpr int GNP_MAXCS = 256, GNP_MAXCH = 16;   // slice channels, partial chunks per source

__global__ void __launch_bounds__(256) gn_apply_part_kernel(const float2* part0, int nch0, const float2* part1,
                                                            int nch1, const half_t* s0, const half_t* s1, int c_split,
                                                            int ld0, int ld1, int h, int w, int pad, int channels,
                                                            int cg, int gps, float eps, const float* gamma,
                                                            const float* beta, float* scale, float* shift, int silu,
                                                            half_t* y, int ldy, int rows_per) {
  __shared__ double cm[GNP_MAXCS], cq[GNP_MAXCS];
  __shared__ float sc_s[GNP_MAXCS], sh_s[GNP_MAXCS];
  __shared__ float2 stage[GNP_MAXCH * GNP_MAXCS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cs = gps * cg, c0 = blockIdx.x * cs, b = blockIdx.y;
  const int hw = h * w;
  // all of the slice's partials into LDS at once (independent, coalesced loads), then the merges
  const int nchm = max(nch0, part1 ? nch1 : 0);
  for (int e = tid; e < nchm * cs; e += 256) {
    const int k = e / cs, cc = e - k * cs, c = c0 + cc;
    const bool second = c >= c_split;
    const int nch = second ? nch1 : nch0, csz = second ? channels - c_split : c_split, cl = second ? c - c_split : c;
    if (k < nch) stage[k * cs + cc] = (second ? part1 : part0)[((size_t)b * nch + k) * csz + cl];
  }
  __syncthreads();
  // equal-count chunks: mean = mean of the chunk means, M2 = sum M2_k + rows * sum (mean_k - mean)^2
  for (int cc = tid; cc < cs; cc += 256) {
    const int c = c0 + cc;
    const int nch = c >= c_split ? nch1 : nch0;
    double ms = 0.0;
    for (int k = 0; k < nch; ++k) ms += (double)stage[k * cs + cc].x;
    const double mean = ms / nch, rows = (double)hw / nch;
    double m2 = 0.0, dd = 0.0;
    for (int k = 0; k < nch; ++k) {
      const float2 q = stage[k * cs + cc];
      const double dl = (double)q.x - mean;
      m2 += (double)q.y;
      dd += dl * dl;
    }
    cm[cc] = mean;
    cq[cc] = m2 + rows * dd;
  }
  __syncthreads();
  for (int gi = wave; gi < gps; gi += 4) {
    double ms = 0.0;
    for (int ci = lane; ci < cg; ci += 64) ms += cm[gi * cg + ci];
    ms = wave_sum_d(ms);
    const double mg = ms / cg;
    double m2g = 0.0;
    for (int ci = lane; ci < cg; ci += 64) {
      const double dm = cm[gi * cg + ci] - mg;
      m2g += cq[gi * cg + ci] + (double)hw * dm * dm;
    }
    m2g = wave_sum_d(m2g);
    const double var = (m2g > 0 ? m2g : 0.0) / ((double)hw * cg);
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float meanf = (float)mg;
    for (int ci = lane; ci < cg; ci += 64) {
      const int c = c0 + gi * cg + ci;
      const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
      const float sc = gm * rstd, sh = bt - meanf * sc;
      sc_s[gi * cg + ci] = sc;
      sh_s[gi * cg + ci] = sh;
      if (scale && blockIdx.z == 0) {
        scale[(size_t)b * channels + c] = sc;
        shift[(size_t)b * channels + c] = sh;
      }
    }
  }
  __syncthreads();
  const int hp = h + 2 * pad, wp = w + 2 * pad, npix = hp * wp, v8 = cs / 8;
  const int r0 = blockIdx.z * rows_per, r1 = min(npix, r0 + rows_per);
  half_t* yb = y + (size_t)b * npix * ldy + c0;
  constexpr int U = 8;   // vectors per thread in flight (the loads of one round are independent)
  const int total = (r1 - r0) * v8;
  for (int base = tid; base < total; base += 256 * U) {
    h8 v[U];
    bool in[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * 256, rr = r0 + e / v8, cv = (e % v8) * 8;
      const int iy = rr / wp - pad, ix = rr % wp - pad;
      in[u] = e < total && (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      v[u] = in[u] ? load_px(s0, s1, c_split, ld0, ld1, ((size_t)b * h + iy) * w + ix, c0 + cv) : h8{};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * 256, rr = r0 + e / v8, cv = (e % v8) * 8;
      if (e >= total) break;
      h8 o = {};
      if (in[u]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = (float)v[u][j] * sc_s[cv + j] + sh_s[cv + j];
          if (silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
          o[j] = (half_t)x;
        }
      }
      *reinterpret_cast<h8*>(yb + (size_t)rr * ldy + cv) = o;
    }
  }
}

// channel slice of gn_apply_part_kernel: the most whole groups with a multiple of 8 channels, at most
// GNP_MAXCS (wider per-pixel runs coalesce better); 0 = not applicable
int gn_part_gps(int channels, int groups) {
  const int cg = channels / groups;
  int best = 0;
  for (int g = 1; g <= groups; ++g)
    if (groups % g == 0 && (g * cg) % 8 == 0 && g * cg <= GNP_MAXCS) best = g;
  return best;
}

// slice size of the single-launch statistics: the fewest whole groups whose channels are a
// multiple of 8 (16-B loads), at most 512 channels; 0 = not applicable
int gn_fused_gps(int channels, int groups) {
  const int cg = channels / groups;
  for (int g = 1; g <= groups; ++g)
    if (groups % g == 0 && (g * cg) % 8 == 0) return g * cg <= 512 ? g : 0;
  return 0;
}

// GroupNorm apply (+ SiLU): y = silu?(x*scale[b,c] + shift[b,c]), 8 channels per thread,
// 16-B loads/stores, reads the (optional) 2-source concat and writes it contiguous.
// Applying the per-tap prologue inside a 3x3 implicit GEMM would repeat this
// VALU work 9x per element; one streaming pass is HBM-bound instead.
__global__ void __launch_bounds__(256) gn_apply_kernel(const half_t* s0, const half_t* s1, int c_split, int ld0,
                                                       int ld1, int hw, int channels, const float* scale,
                                                       const float* shift, int silu, half_t* y, int ldy,
                                                       int64_t nvec) {
  const int c8 = channels / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nvec; e += stride) {
    const int64_t pix = e / c8;
    const int c = (int)(e - pix * c8) * 8;
    const int b = (int)(pix / hw);
    h8 v = load_px(s0, s1, c_split, ld0, ld1, (size_t)pix, c);
    const f4* ps = reinterpret_cast<const f4*>(scale + (size_t)b * channels + c);
    const f4* pt = reinterpret_cast<const f4*>(shift + (size_t)b * channels + c);
    const f4 sa = ps[0], sb = ps[1], ta = pt[0], tb = pt[1];
    const float sc[8] = {sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]};
    const float sh[8] = {ta[0], ta[1], ta[2], ta[3], tb[0], tb[1], tb[2], tb[3]};
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = (float)v[j] * sc[j] + sh[j];
      if (silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      o[j] = (half_t)x;
    }
    *reinterpret_cast<h8*>(y + (size_t)pix * ldy + c) = o;
  }
}

// The same transform written into a zero-bordered image [B][h+2p][w+2p][ldy]: the 3x3 conv that
// consumes it runs with pad 0, every tap in range — no per-tap masks in its A gather.
__global__ void __launch_bounds__(256) gn_apply_pad_kernel(const half_t* s0, const half_t* s1, int c_split, int ld0,
                                                           int ld1, int h, int w, int pad, int channels,
                                                           const float* scale, const float* shift, int silu,
                                                           half_t* y, int ldy, int64_t nvec) {
  const int c8 = channels / 8;
  const int hp = h + 2 * pad, wp = w + 2 * pad;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nvec; e += stride) {
    const int64_t ppix = e / c8;
    const int c = (int)(e - ppix * c8) * 8;
    const int b = (int)(ppix / ((int64_t)hp * wp));
    const int r = (int)(ppix - (int64_t)b * hp * wp);
    const int iy = r / wp - pad, ix = r % wp - pad;
    h8 o = {};
    if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) {
      const size_t pix = ((size_t)b * h + iy) * w + ix;
      const h8 v = load_px(s0, s1, c_split, ld0, ld1, pix, c);
      const f4* ps = reinterpret_cast<const f4*>(scale + (size_t)b * channels + c);
      const f4* pt = reinterpret_cast<const f4*>(shift + (size_t)b * channels + c);
      const f4 sa = ps[0], sb = ps[1], ta = pt[0], tb = pt[1];
      const float sc[8] = {sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]};
      const float sh[8] = {ta[0], ta[1], ta[2], ta[3], tb[0], tb[1], tb[2], tb[3]};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = (float)v[j] * sc[j] + sh[j];
        if (silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
        o[j] = (half_t)x;
      }
    }
    *reinterpret_cast<h8*>(y + (size_t)ppix * ldy + c) = o;
  }
}

// The same transform (padded or not), one pass: each thread owns GNA_U vectors of the output spaced 256 apart (every
// load of the thread issued before the first store), 32-bit element indices split by host-verified multiply-shift
// reciprocals (pad_row_divm) instead of the 64-bit divisions of the grid-stride forms — those cost more VALU than
// the byte moving at the 64x64 / 32x32 levels.  e -> (padded pixel, 8-channel chunk) -> (image, padded row, column).
constexpr int GNA_U = 4;
__global__ void __launch_bounds__(256) gn_apply_flat_kernel(const half_t* s0, const half_t* s1, int c_split, int ld0,
                                                            int ld1, int h, int w, int pad, int channels,
                                                            const float* scale, const float* shift, int silu,
                                                            half_t* y, int ldy, unsigned nvec, unsigned m_c8,
                                                            unsigned m_img, unsigned m_wp) {
  const unsigned c8 = (unsigned)channels / 8, hp = h + 2 * pad, wp = w + 2 * pad, npix = hp * wp;
  const unsigned e0 = blockIdx.x * (256u * GNA_U) + threadIdx.x;
  h8 v[GNA_U];
  unsigned ppix[GNA_U], cc[GNA_U], bb[GNA_U];
  bool in[GNA_U];
#pragma unroll
  for (int u = 0; u < GNA_U; ++u) {
    const unsigned e = e0 + 256u * u;
    const unsigned p = (unsigned)(((unsigned long long)e * m_c8) >> 32);           // e / c8
    const unsigned b = (unsigned)(((unsigned long long)p * m_img) >> 32);          // p / npix
    const unsigned r = p - b * npix;
    const unsigned ry = (unsigned)(((unsigned long long)r * m_wp) >> 32);          // r / wp
    const int iy = (int)ry - pad, ix = (int)(r - ry * wp) - pad;
    ppix[u] = p;
    cc[u] = (e - p * c8) * 8;
    bb[u] = b;
    in[u] = e < nvec && (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
    v[u] = in[u] ? load_px(s0, s1, c_split, ld0, ld1, ((size_t)b * h + iy) * w + ix, (int)cc[u]) : h8{};
  }
#pragma unroll
  for (int u = 0; u < GNA_U; ++u) {
    if (e0 + 256u * u >= nvec) break;
    h8 o = {};
    if (in[u]) {
      const f4* ps = reinterpret_cast<const f4*>(scale + (size_t)bb[u] * channels + cc[u]);
      const f4* pt = reinterpret_cast<const f4*>(shift + (size_t)bb[u] * channels + cc[u]);
      const f4 sa = ps[0], sb = ps[1], ta = pt[0], tb = pt[1];
      const float sc[8] = {sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]};
      const float sh[8] = {ta[0], ta[1], ta[2], ta[3], tb[0], tb[1], tb[2], tb[3]};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = (float)v[u][j] * sc[j] + sh[j];
        if (silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
        o[j] = (half_t)x;
      }
    }
    *reinterpret_cast<h8*>(y + (size_t)ppix[u] * ldy + cc[u]) = o;
  }
}

// The same per padded row: grid (padded row, image); the image's scale / shift staged in LDS once, the row's
// (pixel, 8-channel chunk) elements split by a host-verified multiply-shift (no 64-bit index division per
// element), GNP_U loads in flight per thread.  Same arithmetic per element (profiles/r4_gn_apply_pad_ab.txt).
constexpr int GNP_U = 4;
__global__ void __launch_bounds__(256) gn_apply_pad_row_kernel(const half_t* s0, const half_t* s1, int c_split,
                                                               int ld0, int ld1, int h, int w, int pad, int channels,
                                                               const float* scale, const float* shift, int silu,
                                                               half_t* y, int ldy, unsigned divm) {
  extern __shared__ __attribute__((aligned(16))) float gst[];   // [channels] scale | [channels] shift
  const int tid = threadIdx.x, py = blockIdx.x, b = blockIdx.y;
  const int c8 = channels / 8, hp = h + 2 * pad, wp = w + 2 * pad;
  for (int e = tid; e < channels / 4; e += 256) {
    reinterpret_cast<f4*>(gst)[e] = reinterpret_cast<const f4*>(scale + (size_t)b * channels)[e];
    reinterpret_cast<f4*>(gst + channels)[e] = reinterpret_cast<const f4*>(shift + (size_t)b * channels)[e];
  }
  __syncthreads();
  const int iy = py - pad;
  const bool row_in = (unsigned)iy < (unsigned)h;
  const int n = wp * c8;
  half_t* yrow = y + ((size_t)b * hp + py) * wp * (size_t)ldy;
  const size_t pix0 = ((size_t)b * h + (row_in ? iy : 0)) * w;
  for (int i0 = tid; i0 < n; i0 += 256 * GNP_U) {
    h8 v[GNP_U];
    int px[GNP_U], cc[GNP_U];
    bool in[GNP_U];
#pragma unroll
    for (int u = 0; u < GNP_U; ++u) {
      const int i = i0 + 256 * u;
      px[u] = (int)(((unsigned long long)(unsigned)i * divm) >> 32);
      cc[u] = (i - px[u] * c8) * 8;
      const int ix = px[u] - pad;
      in[u] = i < n && row_in && (unsigned)ix < (unsigned)w;
      v[u] = in[u] ? load_px(s0, s1, c_split, ld0, ld1, pix0 + ix, cc[u]) : h8{};
    }
#pragma unroll
    for (int u = 0; u < GNP_U; ++u) {
      if (i0 + 256 * u >= n) break;
      h8 o = {};
      if (in[u]) {
        const f4* ps = reinterpret_cast<const f4*>(gst + cc[u]);
        const f4* pt = reinterpret_cast<const f4*>(gst + channels + cc[u]);
        const f4 sa = ps[0], sb = ps[1], ta = pt[0], tb = pt[1];
        const float sc[8] = {sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]};
        const float sh[8] = {ta[0], ta[1], ta[2], ta[3], tb[0], tb[1], tb[2], tb[3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = (float)v[u][j] * sc[j] + sh[j];
          if (silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
          o[j] = (half_t)x;
        }
      }
      *reinterpret_cast<h8*>(yrow + (size_t)px[u] * ldy + cc[u]) = o;
    }
  }
}

// Nearest-x2 upsample into a zero-bordered image (UNet Upsample, reference openai_model/model.py:120-131:
// F.interpolate(scale_factor=2, mode="nearest") then the 3x3 conv with padding 1): y[b][py][px] =
// x[b][(py - pad) >> 1][(px - pad) >> 1] inside, 0 on the border — the conv then runs unmasked (pad 0) on the
// linear A issue instead of folding the upsample into every DMA address.  Grid (padded row, image).
__global__ void __launch_bounds__(256) upsample_nearest2x_pad_kernel(const half_t* x, int ldx, int h, int w, int pad,
                                                                     int channels, half_t* y, unsigned divm) {
  const int tid = threadIdx.x, py = blockIdx.x, b = blockIdx.y;
  const int c8 = channels / 8, hp = 2 * h + 2 * pad, wp = 2 * w + 2 * pad;
  const int uy = py - pad;
  const bool row_in = (unsigned)uy < (unsigned)(2 * h);
  const int n = wp * c8;
  half_t* yrow = y + ((size_t)b * hp + py) * wp * (size_t)channels;
  const size_t src0 = ((size_t)b * h + (row_in ? uy >> 1 : 0)) * w;
  for (int i0 = tid; i0 < n; i0 += 256 * GNP_U) {
    h8 v[GNP_U];
    int px[GNP_U], cc[GNP_U];
#pragma unroll
    for (int u = 0; u < GNP_U; ++u) {
      const int i = i0 + 256 * u;
      px[u] = (int)(((unsigned long long)(unsigned)i * divm) >> 32);
      cc[u] = (i - px[u] * c8) * 8;
      const int ux = px[u] - pad;
      const bool in = i < n && row_in && (unsigned)ux < (unsigned)(2 * w);
      v[u] = in ? *reinterpret_cast<const h8*>(x + (src0 + (ux >> 1)) * ldx + cc[u]) : h8{};
    }
#pragma unroll
    for (int u = 0; u < GNP_U; ++u)
      if (i0 + 256 * u < n) *reinterpret_cast<h8*>(yrow + (size_t)px[u] * channels + cc[u]) = v[u];
  }
}

// ceil(2^32 / d) when i * that >> 32 == i / d for every i < n (a closed-form bound), else 0
unsigned pad_row_divm(int n, int d) {
  // m = ceil(2^32 / d) = (2^32 + e) / d with 0 <= e < d, so i * m / 2^32 = i / d + i * e / (d * 2^32): the
  // floor is exact whenever i * e < 2^32 (frac(i / d) <= (d - 1) / d leaves 1 / d of room)
  const unsigned long long m = ((1ull << 32) + (unsigned long long)d - 1) / (unsigned long long)d;
  const unsigned long long e = m * (unsigned long long)d - (1ull << 32);
  if (m > 0xffffffffull) return 0;
  return (n <= 1 || (unsigned long long)(n - 1) * e < (1ull << 32)) ? (unsigned)m : 0u;
}

// Post-activation GroupNorm of the DDPM (C1) UNet's ConvBlock / attention block:
// y = [silu](x*scale + shift) + post_bias[b][c] + residual[pix][c] (either optional).
__global__ void __launch_bounds__(256) gn_apply_ex_kernel(const half_t* s0, const half_t* s1, int c_split, int ld0,
                                                          int ld1, int hw, int channels, const float* scale,
                                                          const float* shift, int silu, const float* pb, int pb_ld,
                                                          const half_t* res, int res_ld, half_t* y, int ldy,
                                                          int64_t nvec) {
  const int c8 = channels / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nvec; e += stride) {
    const int64_t pix = e / c8;
    const int c = (int)(e - pix * c8) * 8;
    const int b = (int)(pix / hw);
    const h8 v = load_px(s0, s1, c_split, ld0, ld1, (size_t)pix, c);
    h8 r = {};
    if (res) r = *reinterpret_cast<const h8*>(res + (size_t)pix * res_ld + c);
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = (float)v[j] * scale[(size_t)b * channels + c + j] + shift[(size_t)b * channels + c + j];
      if (silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      if (pb) x += pb[(size_t)b * pb_ld + c + j];
      if (res) x += (float)r[j];
      o[j] = (half_t)x;
    }
    *reinterpret_cast<h8*>(y + (size_t)pix * ldy + c) = o;
  }
}

// LayerNorm: one wave per row at a time, row cached in registers (cols <= 64*8*LN_MAXV).  Waves
// walk rows grid-stride with the next row's loads in flight while the current one reduces, gamma /
// beta live in registers for the whole walk; the row math (one pivot-shifted pair of shuffle
// chains) is ln_row_stats / ln_apply8 of common.h, shared with the cross-attention block's fused
// norm2 / norm3.
constexpr int LN_MAXV = 4;
template <int MAXV>
__global__ void __launch_bounds__(256) layer_norm_kernel(const half_t* x, half_t* y, int rows, int cols, int ldx,
                                                         int ldy, const float* gamma, const float* beta, float eps) {
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * 4;
  const int c8 = cols / 8;
  float g[MAXV][8], bt[MAXV][8];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int k = lane + 64 * i;
    if (k < c8) {
      const f4* gp = reinterpret_cast<const f4*>(gamma + k * 8);
      const f4* bp = reinterpret_cast<const f4*>(beta + k * 8);
      const f4 g0 = gp[0], g1 = gp[1], b0 = bp[0], b1 = bp[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g[i][j] = g0[j]; g[i][4 + j] = g1[j];
        bt[i][j] = b0[j]; bt[i][4 + j] = b1[j];
      }
    }
  }
  auto load = [&](int r, h8 (&v)[MAXV]) {
    const half_t* xr = x + (size_t)r * ldx;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int k = lane + 64 * i;
      v[i] = (r < rows && k < c8) ? *reinterpret_cast<const h8*>(xr + k * 8) : h8{};
    }
  };
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  h8 v[MAXV];
  load(row, v);
  for (; row < rows; row += nwaves) {
    h8 nv[MAXV];
    load(row + nwaves, nv);
    float mean, rstd;
    ln_row_stats<MAXV>(v, cols, eps, mean, rstd);
    half_t* yr = y + (size_t)row * ldy;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int k = lane + 64 * i;
      if (k < c8) *reinterpret_cast<h8*>(yr + k * 8) = ln_apply8(v[i], mean, rstd, g[i], bt[i]);
    }
#pragma unroll
    for (int i = 0; i < MAXV; ++i) v[i] = nv[i];
  }
}

// LayerNorm for C = 32 * CPL (320 / 640: the transformer widths the fused cross-attention block
// also normalises): 16 rows per wave, four lanes per row (ln_quad_stats, common.h), gamma / beta
// staged once per block in LDS; waves walk 16-row groups grid-stride with the next group's loads
// in flight.
template <int CPL>
__global__ void __launch_bounds__(256) layer_norm_quad_kernel(const half_t* x, half_t* y, int rows, int ldx, int ldy,
                                                              const float* gamma, const float* beta, float eps) {
  constexpr int C = 32 * CPL;
  __shared__ __attribute__((aligned(16))) float gb[2 * C];
  for (int e = threadIdx.x; e < C / 4; e += 256) {
    *reinterpret_cast<f4*>(gb + 4 * e) = *reinterpret_cast<const f4*>(gamma + 4 * e);
    *reinterpret_cast<f4*>(gb + C + 4 * e) = *reinterpret_cast<const f4*>(beta + 4 * e);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, q = lane & 3, rl = lane >> 2;
  const int nwaves = gridDim.x * 4;
  auto load = [&](int r, h8 (&v)[CPL]) {
    const half_t* xr = x + (size_t)r * ldx + 8 * q;
#pragma unroll
    for (int i = 0; i < CPL; ++i) v[i] = r < rows ? *reinterpret_cast<const h8*>(xr + 32 * i) : h8{};
  };
  int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  h8 v[CPL];
  load(r0 + rl, v);
  for (; r0 < rows; r0 += nwaves * 16) {
    h8 nv[CPL];
    load(r0 + nwaves * 16 + rl, nv);
    float mean, rstd;
    ln_quad_stats<CPL>(v, eps, mean, rstd);
    const int row = r0 + rl;
    if (row < rows) {
      half_t* yr = y + (size_t)row * ldy + 8 * q;
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        *reinterpret_cast<h8*>(yr + 32 * i) = ln_quad_apply(v[i], mean, rstd, gb, C, q + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i) v[i] = nv[i];
  }
}

}  // namespace
}  // namespace sdk

using namespace sdk;

// largest pixels-per-image for the single-launch statistics (SDK_GN_FUSED_MAX_HW, read at load;
// measured crossover on MI355X: tools/bench_norm.py)
static const int g_gn_fused_max_hw = [] {
  const char* e = getenv("SDK_GN_FUSED_MAX_HW");
  return e ? atoi(e) : 1024;
}();

extern "C" int64_t sdk_group_norm_workspace(int32_t batch, int32_t hw, int32_t channels) {
  if (batch <= 0 || hw <= 0 || channels <= 0) return 0;
  GnGeom g = gn_geom(batch, hw, channels);
  return (int64_t)batch * g.nchunks * channels * (int64_t)sizeof(float2);
}

extern "C" int sdk_group_norm_affine(const sdk_group_norm_args* a, sdk_stream_t stream) {
  if (!a || !a->src0 || !a->scale || !a->shift) return fail(SDK_EINVAL, "group_norm: null pointer");
  if (a->channels % 8 || a->channels % a->groups || a->c_split % 8 || a->c_split <= 0 || a->c_split > a->channels)
    return fail(SDK_EINVAL, "group_norm: channels/c_split must be multiples of 8, channels % groups == 0");
  if (a->channels / a->groups > 256) return fail(SDK_EINVAL, "group_norm: > 256 channels per group");
  if (a->c_split < a->channels && !a->src1) return fail(SDK_EINVAL, "group_norm: concat without src1");
  if (a->ld0 % 8 || (a->c_split < a->channels && a->ld1 % 8)) return fail(SDK_EINVAL, "group_norm: ld % 8");
  if (a->channels / 8 > 512) return fail(SDK_EINVAL, "group_norm: channels > 4096");
  hipStream_t s = (hipStream_t)stream;
  const int gps = gn_fused_gps(a->channels, a->groups);
  if (gps > 0 && a->hw <= g_gn_fused_max_hw) {
    hipLaunchKernelGGL(gn_stats_fused_kernel<false>, dim3(a->groups / gps, a->batch), dim3(GNF_T), 0, s,
                       (const half_t*)a->src0, (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, a->hw, a->channels,
                       a->channels / a->groups, gps, a->eps, a->gamma, a->beta, a->scale, a->shift, 0, nullptr, 0,
                       0, 0, 0);
    return check_launch("gn_stats_fused");
  }
  const int64_t need = sdk_group_norm_workspace(a->batch, a->hw, a->channels);
  if (!a->workspace || a->workspace_bytes < need) return fail(SDK_EWORKSPACE, "group_norm: workspace too small");
  GnGeom g = gn_geom(a->batch, a->hw, a->channels);
  const size_t lds = g.ry > 1 ? (size_t)2 * g.ry * g.c8 * 8 * sizeof(float) : 0;
  hipLaunchKernelGGL(gn_partial_kernel, dim3(g.nchunks, a->batch), dim3(256), lds, s, (const half_t*)a->src0,
                     (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, a->hw, a->channels, g,
                     (float2*)a->workspace);
  if (int e = check_launch("gn_partial")) return e;
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(a->groups, a->batch), dim3(256), 0, s, (const half_t*)a->src0,
                     (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, a->hw, a->channels, a->groups, g,
                     (const float2*)a->workspace, a->eps, a->gamma, a->beta, a->scale, a->shift);
  return check_launch("gn_finalize");
}

// SDK_GN_APPLY_FLAT: 1 (default) = gn_apply_flat_kernel below 128x128 pixels, 2 = everywhere, 0 = the grid-stride /
// row forms only (A/B)
static const int g_gn_apply_flat = [] {
  const char* e = getenv("SDK_GN_APPLY_FLAT");
  return e ? atoi(e) : 1;
}();

// the one-pass apply when its reciprocals are exact over every index it forms (tail lanes included); 1 = launched
static int gn_apply_flat(const sdk_group_norm_args* a, int silu, void* y, int ld_y, int h, int w, int pad,
                         hipStream_t s) {
  if (g_gn_apply_flat == 0 || (g_gn_apply_flat == 1 && (int64_t)h * w >= 128 * 128)) return 0;
  const int64_t npix = (int64_t)(h + 2 * pad) * (w + 2 * pad), c8 = a->channels / 8;
  const int64_t nvec = (int64_t)a->batch * npix * c8, span = nvec + 256 * GNA_U;
  if (span >= (1LL << 31) || npix >= (1 << 30)) return 0;
  const unsigned m_c8 = c8 > 1 ? pad_row_divm((int)span, (int)c8) : 0u;
  const unsigned m_img = npix > 1 ? pad_row_divm((int)(span / c8 + 1), (int)npix) : 0u;
  const unsigned m_wp = (w + 2 * pad) > 1 ? pad_row_divm((int)npix, w + 2 * pad) : 0u;
  if (!m_c8 || !m_img || !m_wp) return 0;
  const unsigned blocks = (unsigned)((nvec + 256 * GNA_U - 1) / (256 * GNA_U));
  hipLaunchKernelGGL(gn_apply_flat_kernel, dim3(blocks), dim3(256), 0, s, (const half_t*)a->src0,
                     (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, h, w, pad, a->channels, a->scale, a->shift,
                     silu, (half_t*)y, ld_y, (unsigned)nvec, m_c8, m_img, m_wp);
  return 1;
}

extern "C" int sdk_group_norm_apply(const sdk_group_norm_args* a, int32_t silu, void* y, int32_t ld_y,
                                    sdk_stream_t stream) {
  if (!a || !a->src0 || !a->scale || !a->shift || !y) return fail(SDK_EINVAL, "group_norm_apply: null pointer");
  if (a->channels % 8 || a->c_split % 8 || a->c_split <= 0 || a->c_split > a->channels || ld_y % 8 ||
      ld_y < a->channels)
    return fail(SDK_EINVAL, "group_norm_apply: channels/c_split/ld_y must be multiples of 8");
  if (a->c_split < a->channels && !a->src1) return fail(SDK_EINVAL, "group_norm_apply: concat without src1");
  const int64_t nvec = (int64_t)a->batch * a->hw * (a->channels / 8);
  if (nvec <= 0) return SDK_OK;
  if (a->hw < (1 << 30) && gn_apply_flat(a, silu, y, ld_y, 1, (int)a->hw, 0, (hipStream_t)stream))
    return check_launch("gn_apply_flat");
  const int blocks = (int)std::min<int64_t>((nvec + 255) / 256, 8192);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const half_t*)a->src0,
                     (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, a->hw, a->channels, a->scale, a->shift,
                     silu, (half_t*)y, ld_y, nvec);
  return check_launch("gn_apply");
}

extern "C" int sdk_group_norm_apply_padded(const sdk_group_norm_args* a, int32_t silu, void* y, int32_t ld_y,
                                           int32_t h, int32_t w, int32_t pad, sdk_stream_t stream) {
  if (!a || !a->src0 || !a->scale || !a->shift || !y) return fail(SDK_EINVAL, "group_norm_apply: null pointer");
  if (a->channels % 8 || a->c_split % 8 || a->c_split <= 0 || a->c_split > a->channels || ld_y % 8 ||
      ld_y < a->channels)
    return fail(SDK_EINVAL, "group_norm_apply: channels/c_split/ld_y must be multiples of 8");
  if (a->c_split < a->channels && !a->src1) return fail(SDK_EINVAL, "group_norm_apply: concat without src1");
  if (h <= 0 || w <= 0 || (int64_t)h * w != a->hw || pad < 0 || pad > 4)
    return fail(SDK_EINVAL, "group_norm_apply_padded: h*w must equal hw, pad in [0, 4]");
  const int64_t nvec = (int64_t)a->batch * (h + 2 * pad) * (w + 2 * pad) * (a->channels / 8);
  if (nvec <= 0) return SDK_OK;
  const int hp = h + 2 * pad, wp = w + 2 * pad;
  if (gn_apply_flat(a, silu, y, ld_y, h, w, pad, (hipStream_t)stream)) return check_launch("gn_apply_flat");
  const unsigned divm = (int64_t)wp * (a->channels / 8) < (1 << 24) ? pad_row_divm(wp * (a->channels / 8), a->channels / 8) : 0;
  // the row form where it measured faster (the VAE decoder's >= 128x128 images: 206.6 -> 182.5 us at 128x128x512,
  // 696.6 -> 677.8 at 512x512x128); the grid-stride form elsewhere (64x64x640 56.6 vs 58.9 us, 16x16 17.4 vs 19.4)
  if (divm && (int64_t)h * w >= 128 * 128 && a->channels <= 4096 && hp <= 65535 && a->batch <= 65535) {
    hipLaunchKernelGGL(gn_apply_pad_row_kernel, dim3(hp, a->batch), dim3(256), (size_t)a->channels * 8,
                       (hipStream_t)stream, (const half_t*)a->src0, (const half_t*)a->src1, a->c_split, a->ld0, a->ld1,
                       h, w, pad, a->channels, a->scale, a->shift, silu, (half_t*)y, ld_y, divm);
    return check_launch("gn_apply_pad");
  }
  const int blocks = (int)std::min<int64_t>((nvec + 255) / 256, 8192);
  hipLaunchKernelGGL(gn_apply_pad_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const half_t*)a->src0,
                     (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, h, w, pad, a->channels, a->scale, a->shift,
                     silu, (half_t*)y, ld_y, nvec);
  return check_launch("gn_apply_pad");
}

extern "C" int sdk_group_norm_apply_ex(const sdk_group_norm_args* a, int32_t silu, const float* post_bias,
                                       int32_t pb_ld, const void* residual, int32_t res_ld, void* y, int32_t ld_y,
                                       sdk_stream_t stream) {
  if (!a || !a->src0 || !a->scale || !a->shift || !y) return fail(SDK_EINVAL, "group_norm_apply_ex: null pointer");
  if (a->channels % 8 || a->c_split % 8 || a->c_split <= 0 || a->c_split > a->channels || ld_y % 8 ||
      ld_y < a->channels || (residual && res_ld % 8))
    return fail(SDK_EINVAL, "group_norm_apply_ex: channels/c_split/ld_y/res_ld must be multiples of 8");
  if (a->c_split < a->channels && !a->src1) return fail(SDK_EINVAL, "group_norm_apply_ex: concat without src1");
  const int64_t nvec = (int64_t)a->batch * a->hw * (a->channels / 8);
  if (nvec <= 0) return SDK_OK;
  const int blocks = (int)std::min<int64_t>((nvec + 255) / 256, 8192);
  hipLaunchKernelGGL(gn_apply_ex_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const half_t*)a->src0,
                     (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, a->hw, a->channels, a->scale, a->shift,
                     silu, post_bias, pb_ld, (const half_t*)residual, res_ld, (half_t*)y, ld_y, nvec);
  return check_launch("gn_apply_ex");
}

extern "C" int sdk_layer_norm(const void* x, void* y, int32_t rows, int32_t cols, int32_t ld_x, int32_t ld_y,
                              const float* gamma, const float* beta, float eps, sdk_stream_t stream) {
  if (!x || !y || !gamma || !beta) return fail(SDK_EINVAL, "layer_norm: null pointer");
  if (cols % 8 || ld_x % 8 || ld_y % 8 || cols > 64 * 8 * LN_MAXV) return fail(SDK_EINVAL, "layer_norm: cols");
  if (((uintptr_t)gamma | (uintptr_t)beta) & 15) return fail(SDK_EINVAL, "layer_norm: gamma/beta 16-B alignment");
  if (rows <= 0) return SDK_OK;
  // 4 rows (waves) per block; up to 8 resident blocks per CU on 256 CUs, each wave then walks rows
  const int blocks = std::min((rows + 3) / 4, 2048);
  hipStream_t s = (hipStream_t)stream;
  const int c8 = cols / 8;
  if (cols == 320 || cols == 640) {
    const int qblocks = std::min((rows + 63) / 64, 2048);
    if (cols == 320)
      hipLaunchKernelGGL(layer_norm_quad_kernel<10>, dim3(qblocks), dim3(256), 0, s, (const half_t*)x, (half_t*)y, rows,
                         ld_x, ld_y, gamma, beta, eps);
    else
      hipLaunchKernelGGL(layer_norm_quad_kernel<20>, dim3(qblocks), dim3(256), 0, s, (const half_t*)x, (half_t*)y, rows,
                         ld_x, ld_y, gamma, beta, eps);
  } else if (c8 <= 64)
    hipLaunchKernelGGL(layer_norm_kernel<1>, dim3(blocks), dim3(256), 0, s, (const half_t*)x, (half_t*)y, rows, cols,
                       ld_x, ld_y, gamma, beta, eps);
  else if (c8 <= 128)
    hipLaunchKernelGGL(layer_norm_kernel<2>, dim3(blocks), dim3(256), 0, s, (const half_t*)x, (half_t*)y, rows, cols,
                       ld_x, ld_y, gamma, beta, eps);
  else
    hipLaunchKernelGGL(layer_norm_kernel<LN_MAXV>, dim3(blocks), dim3(256), 0, s, (const half_t*)x, (half_t*)y, rows,
                       cols, ld_x, ld_y, gamma, beta, eps);
  return check_launch("layer_norm");
}

// GroupNorm (+ SiLU) end to end: statistics and apply, written contiguous (pad = 0) or into a
// zero-bordered [B][h+2pad][w+2pad][ld_y] image.  Statistics: merged from the producing convs'
// per-chunk partials when given (part0, and part1 for a concat), else one fused statistics+apply
// launch at the smallest levels (hw <= SDK_GN_APPLY_FUSED_MAX_HW), else the statistics pass; then
// the apply pass.  a->scale / a->shift (and a->workspace for the statistics pass) as for
// sdk_group_norm_affine.
static const int g_gn_apply_fused_max_hw = [] {
  const char* e = getenv("SDK_GN_APPLY_FUSED_MAX_HW");
  return e ? atoi(e) : 64;
}();
// largest image (h*w) whose GroupNorm-from-partials runs as one gn_apply_part_kernel launch
static const int g_gn_part_fused_max_hw = [] {
  const char* e = getenv("SDK_GN_PART_FUSED_MAX_HW");
  return e ? atoi(e) : 256;
}();

extern "C" int sdk_group_norm_finalize(const sdk_group_norm_args* a, const float* part0, int32_t nch0,
                                       const float* part1, int32_t nch1, sdk_stream_t stream) {
  if (!a || !a->src0 || !a->scale || !a->shift) return fail(SDK_EINVAL, "group_norm_finalize: null pointer");
  if (a->channels % 8 || a->groups <= 0 || a->channels % a->groups || a->c_split % 8 || a->c_split <= 0 ||
      a->c_split > a->channels)
    return fail(SDK_EINVAL, "group_norm_finalize: channels/c_split must be multiples of 8, channels % groups == 0");
  const bool concat = a->c_split < a->channels;
  const bool parts = part0 && (!concat || part1);
  if (!parts) return sdk_group_norm_affine(a, stream);
  if (nch0 <= 0 || a->hw % nch0 || (concat && (nch1 <= 0 || a->hw % nch1)))
    return fail(SDK_EINVAL, "group_norm_finalize: partial chunks must divide hw");
  if (a->batch <= 0) return SDK_OK;
  hipLaunchKernelGGL(gn_finalize_part_kernel, dim3(a->groups, a->batch), dim3(256), 0, (hipStream_t)stream,
                     (const float2*)part0, nch0, (const float2*)part1, nch1, a->c_split, a->hw, a->channels, a->groups,
                     a->eps, a->gamma, a->beta, a->scale, a->shift);
  return check_launch("gn_finalize_part");
}

extern "C" int sdk_group_norm(const sdk_group_norm_args* a, int32_t silu, void* y, int32_t ld_y, int32_t h, int32_t w,
                              int32_t pad, const float* part0, int32_t nch0, const float* part1, int32_t nch1,
                              sdk_stream_t stream) {
  if (!a || !a->src0 || !y) return fail(SDK_EINVAL, "group_norm: null pointer");
  if (a->channels % 8 || a->groups <= 0 || a->channels % a->groups || a->c_split % 8 || a->c_split <= 0 ||
      a->c_split > a->channels || ld_y % 8 || ld_y < a->channels)
    return fail(SDK_EINVAL, "group_norm: channels/c_split/ld_y must be multiples of 8, channels % groups == 0");
  if (a->channels / a->groups > 256) return fail(SDK_EINVAL, "group_norm: > 256 channels per group");
  if (a->c_split < a->channels && !a->src1) return fail(SDK_EINVAL, "group_norm: concat without src1");
  if (a->ld0 % 8 || (a->c_split < a->channels && a->ld1 % 8)) return fail(SDK_EINVAL, "group_norm: ld % 8");
  if (h <= 0 || w <= 0 || (int64_t)h * w != a->hw || pad < 0 || pad > 4)
    return fail(SDK_EINVAL, "group_norm: h*w must equal hw, pad in [0, 4]");
  const bool concat = a->c_split < a->channels;
  const bool parts = part0 && (!concat || part1);
  if (parts && (nch0 <= 0 || a->hw % nch0 || (concat && (nch1 <= 0 || a->hw % nch1))))
    return fail(SDK_EINVAL, "group_norm: partial chunks must divide hw");
  hipStream_t s = (hipStream_t)stream;
  const int gps = gn_fused_gps(a->channels, a->groups);
  if (!parts && gps > 0 && a->hw <= g_gn_apply_fused_max_hw && a->batch > 0) {
    hipLaunchKernelGGL(gn_stats_fused_kernel<true>, dim3(a->groups / gps, a->batch), dim3(GNF_T), 0, s,
                       (const half_t*)a->src0, (const half_t*)a->src1, a->c_split, a->ld0, a->ld1, a->hw, a->channels,
                       a->channels / a->groups, gps, a->eps, a->gamma, a->beta, nullptr, nullptr, silu, (half_t*)y,
                       ld_y, h, w, pad);
    return check_launch("gn_fused_apply");
  }
  const int pgps = gn_part_gps(a->channels, a->groups);
  if (parts && pgps > 0 && a->hw <= g_gn_part_fused_max_hw && a->batch > 0 && nch0 <= GNP_MAXCH &&
      (!concat || nch1 <= GNP_MAXCH)) {
    const int cs = pgps * (a->channels / a->groups), slices = a->groups / pgps;
    const int npix = (h + 2 * pad) * (w + 2 * pad);
    // ~8 vectors per thread (one round of loads in flight), at least ~512 workgroups when the image allows
    int splits = std::max(1, (npix * (cs / 8) + 2047) / 2048);
    const int want = (512 + slices * a->batch - 1) / (slices * a->batch);
    splits = std::min(std::max(splits, want), std::max(1, npix / 16));
    const int rows_per = (npix + splits - 1) / splits;
    splits = (npix + rows_per - 1) / rows_per;
    hipLaunchKernelGGL(gn_apply_part_kernel, dim3(slices, a->batch, splits), dim3(256), 0, s, (const float2*)part0,
                       nch0, (const float2*)part1, nch1, (const half_t*)a->src0, (const half_t*)a->src1, a->c_split,
                       a->ld0, a->ld1, h, w, pad, a->channels, a->channels / a->groups, pgps, a->eps, a->gamma,
                       a->beta, a->scale, a->shift, silu, (half_t*)y, ld_y, rows_per);
    return check_launch("gn_apply_part");
  }
  if (!a->scale || !a->shift) return fail(SDK_EINVAL, "group_norm: scale/shift buffers needed");
  if (parts) {
    if (a->batch > 0) {
      hipLaunchKernelGGL(gn_finalize_part_kernel, dim3(a->groups, a->batch), dim3(256), 0, s, (const float2*)part0,
                         nch0, (const float2*)part1, nch1, a->c_split, a->hw, a->channels, a->groups, a->eps, a->gamma,
                         a->beta, a->scale, a->shift);
      if (int e = check_launch("gn_finalize_part")) return e;
    }
  } else if (int e = sdk_group_norm_affine(a, stream)) {
    return e;
  }
  return pad ? sdk_group_norm_apply_padded(a, silu, y, ld_y, h, w, pad, stream)
             : sdk_group_norm_apply(a, silu, y, ld_y, stream);
}

extern "C" int sdk_upsample_nearest2x_padded(const void* x, int32_t ld_x, void* y, int32_t batch, int32_t h, int32_t w,
                                             int32_t channels, int32_t pad, sdk_stream_t stream) {
  if (!x || !y || batch <= 0 || h <= 0 || w <= 0 || channels <= 0 || channels % 8 || ld_x % 8 || ld_x < channels ||
      pad < 0 || pad > 4)
    return fail(SDK_EINVAL, "upsample_nearest2x_padded: bad args (channels / ld_x multiples of 8, pad in [0, 4])");
  const int hp = 2 * h + 2 * pad, wp = 2 * w + 2 * pad;
  if (hp > 65535 || batch > 65535 || (int64_t)wp * (channels / 8) >= (1 << 24))
    return fail(SDK_EINVAL, "upsample_nearest2x_padded: image too large");
  const unsigned divm = pad_row_divm(wp * (channels / 8), channels / 8);
  if (!divm) return fail(SDK_EINVAL, "upsample_nearest2x_padded: no exact row split");
  hipLaunchKernelGGL(upsample_nearest2x_pad_kernel, dim3(hp, batch), dim3(256), 0, (hipStream_t)stream,
                     (const half_t*)x, ld_x, h, w, pad, channels, (half_t*)y, divm);
  return check_launch("upsample_nearest2x_padded");
}
