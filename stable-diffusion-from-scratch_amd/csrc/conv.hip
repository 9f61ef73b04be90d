// Implicit-GEMM convolution / GEMM for gfx950 (MI355X), fp16 in, fp32 accumulate on MFMA.
//
// One kernel covers every conv and Linear of the UNet and the VAE decoder:
//   out[m, n] = sum_k A[m, k] * W[n, k] + epilogue
// m = output pixel (b, oy, ox) of an NHWC tensor, k = (segment, tap, channel).
//
// Tile: 128(M) x 128(N) x 64(K), 256 threads = 4 waves in 2x2, each wave a
// 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_f16.  A and W tiles are staged
// global -> registers -> LDS (double buffer, one barrier per K step); the
// register stage is where the A prologue runs: channel-concat source select,
// nearest-x2 upsample indexing, GroupNorm affine + SiLU and zero padding.  The
// next tile's global loads are issued before the current tile's MFMAs and
// written to LDS after them (issue-early / write-late).  LDS rows are 128 B,
// XOR-swizzled on the 16-B chunk index with (row>>1)&7 so the MFMA fragment
// reads (ds_read_b128, 16 distinct rows per lane group) are conflict-free.
// The epilogue adds bias and the per-(batch, channel) timestep-embedding
// broadcast in registers, optionally pairs (x, gate) columns for GEGLU,
// stages the fp16 tile through LDS and writes it with 16-B coalesced stores
// fused with the residual add.  Low-parallelism shapes (the 16x16 / 8x8 UNet
// levels) split K across workgroups into fp32 slabs reduced by a second kernel.
#include "common.h"

namespace sdk {
namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_H = BM * BK;          // halfs per A (or B) tile
constexpr int CT_LD = BN + 8;            // epilogue LDS row stride (halfs)

struct Seg {
  const half_t* src0;
  const half_t* src1;
  const float* gscale;
  const float* gshift;
  int c_split, cin, cin_pad, ld0, ld1;
  int h, w, ksize, stride, pad, upsample, silu;
  int k_off;            // first packed-K column of this segment
  int tiles_per_tap;    // cin_pad / BK
  int kt_begin;         // first global K tile of this segment
};

struct Params {
  Seg seg[2];
  int nseg, kt_total;
  int M, N, Npad, batch, ho, wo, hw_out;
  const half_t* W;
  int ldw;
  const float* bias;
  const float* row_bias;
  int rb_ld;
  const half_t* res;
  int res_ld;
  void* out;
  int out_ld, out_mode;
  float* partial;       // split-K slabs [split][M][Npad]
  int split, kt_per_split;
  int tiles_m, tiles_n;
};

__device__ __forceinline__ int swz(int row, int chunk) {   // element offset inside a [128][64] tile
  return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3);
}

__device__ __forceinline__ h8 ldg16(const half_t* p) { return *reinterpret_cast<const h8*>(p); }

// A-row context: per thread 4 rows (r = (tid>>3) + 32*i), fixed over the K loop.
struct RowCtx {
  int b[4], oy[4], ox[4];
  bool valid[4];
};

__device__ __forceinline__ void load_a(const Params& p, const RowCtx& rc, int kt, int chunk, h8 (&va)[4],
                                       bool (&ok)[4], int& cglob, int& segi) {
  segi = (p.nseg > 1 && kt >= p.seg[1].kt_begin) ? 1 : 0;
  const Seg& s = p.seg[segi];
  const int local = kt - s.kt_begin;
  const int tap = local / s.tiles_per_tap;
  const int c = (local - tap * s.tiles_per_tap) * BK + chunk * 8;
  const int ky = tap / s.ksize, kx = tap - ky * s.ksize;
  cglob = c;
  const bool cok = c < s.cin;
  const half_t* base;
  int ld, cc;
  if (c < s.c_split) { base = s.src0; ld = s.ld0; cc = c; }
  else { base = s.src1; ld = s.ld1; cc = c - s.c_split; }
  const int lh = s.upsample ? 2 * s.h : s.h, lw = s.upsample ? 2 * s.w : s.w;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int iy = rc.oy[i] * s.stride - s.pad + ky;
    int ix = rc.ox[i] * s.stride - s.pad + kx;
    bool in = rc.valid[i] && cok && iy >= 0 && iy < lh && ix >= 0 && ix < lw;
    ok[i] = in;
    if (s.upsample) { iy >>= 1; ix >>= 1; }
    h8 v = {};
    if (in) v = ldg16(base + ((size_t)((size_t)rc.b[i] * s.h + iy) * s.w + ix) * ld + cc);
    va[i] = v;
  }
}

// GroupNorm affine + SiLU on the staged registers; zero after the transform
// (the conv pads the *normalised* activation).
__device__ __forceinline__ void transform_a(const Params& p, const RowCtx& rc, int segi, int c, h8 (&va)[4],
                                            const bool (&ok)[4]) {
  const Seg& s = p.seg[segi];
  if (s.gscale == nullptr && !s.silu) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (!ok[i]) va[i] = h8{};
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h8 v = va[i];
    if (ok[i]) {
      float sc[8], sh[8];
      if (s.gscale) {
        const f4* ps = reinterpret_cast<const f4*>(s.gscale + (size_t)rc.b[i] * s.cin + c);
        const f4* pt = reinterpret_cast<const f4*>(s.gshift + (size_t)rc.b[i] * s.cin + c);
        f4 s0 = ps[0], s1 = ps[1], t0 = pt[0], t1 = pt[1];
        sc[0] = s0[0]; sc[1] = s0[1]; sc[2] = s0[2]; sc[3] = s0[3];
        sc[4] = s1[0]; sc[5] = s1[1]; sc[6] = s1[2]; sc[7] = s1[3];
        sh[0] = t0[0]; sh[1] = t0[1]; sh[2] = t0[2]; sh[3] = t0[3];
        sh[4] = t1[0]; sh[5] = t1[1]; sh[6] = t1[2]; sh[7] = t1[3];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { sc[j] = 1.f; sh[j] = 0.f; }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = (float)v[j] * sc[j] + sh[j];
        if (s.silu) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
        v[j] = (half_t)x;
      }
    } else {
      v = h8{};
    }
    va[i] = v;
  }
}

__global__ void __launch_bounds__(NT, 2) conv_igemm_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) half_t smem[4 * TILE_H];   // A0 A1 B0 B1 = 64 KiB
  half_t* As = smem;
  half_t* Bs = smem + 2 * TILE_H;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int kt1 = min(p.kt_total, kt0 + p.kt_per_split);

  const int lrow = tid >> 3, chunk = tid & 7;
  RowCtx rc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = m0 + lrow + 32 * i;
    rc.valid[i] = m < p.M;
    int mm = rc.valid[i] ? m : 0;
    int b = mm / p.hw_out, rem = mm - b * p.hw_out;
    int oy = rem / p.wo;
    rc.b[i] = b; rc.oy[i] = oy; rc.ox[i] = rem - oy * p.wo;
  }
  const half_t* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wrow[i] = p.W + (size_t)(n0 + lrow + 32 * i) * p.ldw + chunk * 8;

  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f16v{};

  h8 va[4], vb[4];
  bool ok[4];
  int cglob = 0, segi = 0;

  auto load_b = [&](int kt) {
    const int si = (p.nseg > 1 && kt >= p.seg[1].kt_begin) ? 1 : 0;
    const int kcol = p.seg[si].k_off + (kt - p.seg[si].kt_begin) * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) vb[i] = ldg16(wrow[i] + kcol);
  };
  auto store_tiles = [&](int buf) {
    half_t* a = As + buf * TILE_H;
    half_t* bsh = Bs + buf * TILE_H;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = lrow + 32 * i;
      *reinterpret_cast<h8*>(a + swz(r, chunk)) = va[i];
      *reinterpret_cast<h8*>(bsh + swz(r, chunk)) = vb[i];
    }
  };

  if (kt0 < kt1) {
    load_a(p, rc, kt0, chunk, va, ok, cglob, segi);
    load_b(kt0);
    transform_a(p, rc, segi, cglob, va, ok);
    store_tiles(0);
  }
  __syncthreads();

  const int fr = lane & 31, fh = lane >> 5;
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      load_a(p, rc, kt + 1, chunk, va, ok, cglob, segi);
      load_b(kt + 1);
    }
    const half_t* a = As + cur * TILE_H;
    const half_t* bsh = Bs + cur * TILE_H;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      h8 fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[t] = *reinterpret_cast<const h8*>(a + swz(wm * 64 + t * 32 + fr, kk * 2 + fh));
        fb[t] = *reinterpret_cast<const h8*>(bsh + swz(wn * 64 + t * 32 + fr, kk * 2 + fh));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      transform_a(p, rc, segi, cglob, va, ok);
      store_tiles(cur ^ 1);
    }
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // acc[i][j] element r: row = wm*64 + i*32 + (r&3) + 8*(r>>2) + 4*fh, col = wn*64 + j*32 + fr
  if (p.split > 1) {
    float* slab = p.partial + (size_t)blockIdx.y * p.M * p.Npad;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          const int n = n0 + wn * 64 + j * 32 + fr;
          if (m < p.M) slab[(size_t)m * p.Npad + n] = acc[i][j][r];
        }
    return;
  }

  const int mode = p.out_mode;
  if (mode == SDK_OUT_GEGLU_F16) {
    // weight rows of this wave: [x (32) | gate (32)] -> output col = n0/2 + wn*32 + fr
    half_t* ct = smem;   // [128][CT_LD], only 64 columns used
    const int nx = n0 + wn * 64 + fr, ng = nx + 32;
    const float bx = (p.bias && nx < p.N) ? p.bias[nx] : 0.f, bg = (p.bias && ng < p.N) ? p.bias[ng] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        const float x = acc[i][0][r] + bx, g = acc[i][1][r] + bg;
        ct[rl * CT_LD + wn * 32 + fr] = (half_t)(x * gelu_erf(g));
      }
    __syncthreads();
    const int outw = BN / 2, ncol0 = n0 / 2;
    half_t* out = reinterpret_cast<half_t*>(p.out);
    for (int e = tid; e < BM * (outw / 8); e += NT) {
      const int rl = e / (outw / 8), c8 = (e - rl * (outw / 8)) * 8;
      const int m = m0 + rl, n = ncol0 + c8;
      if (m >= p.M || n >= p.N / 2) continue;
      h8 v = *reinterpret_cast<const h8*>(ct + rl * CT_LD + c8);
      if (p.res) {
        h8 rr = ldg16(p.res + (size_t)m * p.res_ld + n);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] + (float)rr[j]);
      }
      *reinterpret_cast<h8*>(out + (size_t)m * p.out_ld + n) = v;
    }
    return;
  }

  float bn[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + fr;
    bn[j] = (p.bias && n < p.N) ? p.bias[n] : 0.f;
  }

  if (mode == SDK_OUT_NHWC_F16) {
    half_t* ct = smem;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // a 32-row MFMA block straddles two images only when ho*wo % 32 != 0 (4x4 levels)
      const int mblk = m0 + wm * 64 + i * 32;
      const int bidx = min(mblk, p.M - 1) / p.hw_out;
      const bool uniform_b = (p.hw_out % 32) == 0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + j * 32 + fr;
        float add = bn[j];
        if (p.row_bias && n < p.N && uniform_b) add += p.row_bias[(size_t)bidx * p.rb_ld + n];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          float v = acc[i][j][r] + add;
          if (p.row_bias && n < p.N && !uniform_b) {
            const int m = min(m0 + rl, p.M - 1);
            v += p.row_bias[(size_t)(m / p.hw_out) * p.rb_ld + n];
          }
          ct[rl * CT_LD + wn * 64 + j * 32 + fr] = (half_t)v;
        }
      }
    }
    __syncthreads();
    half_t* out = reinterpret_cast<half_t*>(p.out);
    for (int e = tid; e < BM * (BN / 8); e += NT) {
      const int rl = e >> 4, c8 = (e & 15) * 8;
      const int m = m0 + rl, n = n0 + c8;
      if (m >= p.M || n >= p.N) continue;
      h8 v = *reinterpret_cast<const h8*>(ct + rl * CT_LD + c8);
      if (p.res) {
        h8 rr = ldg16(p.res + (size_t)m * p.res_ld + n);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] + (float)rr[j]);
      }
      *reinterpret_cast<h8*>(out + (size_t)m * p.out_ld + n) = v;
    }
    return;
  }

  // fp32 outputs (small: time-embedding projections, final 4/3-channel convs)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + fr;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        if (m >= p.M) continue;
        const int b = m / p.hw_out;
        float v = acc[i][j][r] + bn[j];
        if (p.row_bias) v += p.row_bias[(size_t)b * p.rb_ld + n];
        if (p.res) v += (float)p.res[(size_t)m * p.res_ld + n];
        float* out = reinterpret_cast<float*>(p.out);
        if (mode == SDK_OUT_NCHW_F32)
          out[((size_t)b * p.N + n) * p.hw_out + (m - b * p.hw_out)] = v;
        else
          out[(size_t)m * p.out_ld + n] = v;
      }
    }
}

// Split-K reduction + epilogue: 8 columns per thread.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(Params p) {
  const int groups = p.N / 8;
  const size_t total = (size_t)p.M * groups;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(e / groups), n = (int)(e - (size_t)m * groups) * 8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    for (int s = 0; s < p.split; ++s) {
      const f4* src = reinterpret_cast<const f4*>(p.partial + ((size_t)s * p.M + m) * p.Npad + n);
      f4 a = src[0], b = src[1];
      v[0] += a[0]; v[1] += a[1]; v[2] += a[2]; v[3] += a[3];
      v[4] += b[0]; v[5] += b[1]; v[6] += b[2]; v[7] += b[3];
    }
    const int b = m / p.hw_out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (p.bias) v[j] += p.bias[n + j];
      if (p.row_bias) v[j] += p.row_bias[(size_t)b * p.rb_ld + n + j];
    }
    if (p.out_mode == SDK_OUT_NHWC_F16) {
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)v[j];
      if (p.res) {
        h8 rr = ldg16(p.res + (size_t)m * p.res_ld + n);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (half_t)((float)o[j] + (float)rr[j]);
      }
      *reinterpret_cast<h8*>(reinterpret_cast<half_t*>(p.out) + (size_t)m * p.out_ld + n) = o;
    } else {
      float* out = reinterpret_cast<float*>(p.out);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = v[j];
        if (p.res) x += (float)p.res[(size_t)m * p.res_ld + n + j];
        if (p.out_mode == SDK_OUT_NCHW_F32)
          out[((size_t)b * p.N + n + j) * p.hw_out + (m - b * p.hw_out)] = x;
        else
          out[(size_t)m * p.out_ld + n + j] = x;
      }
    }
  }
}

int build_params(const sdk_conv_args* a, Params& p, sdk_conv_plan_info* info) {
  if (!a) return fail(SDK_EINVAL, "conv2d: null args");
  if (a->nseg < 1 || a->nseg > 2) return fail(SDK_EINVAL, "conv2d: nseg must be 1 or 2");
  if (a->batch <= 0 || a->ho <= 0 || a->wo <= 0 || a->cout <= 0)
    return fail(SDK_EINVAL, "conv2d: empty output shape");
  if (!a->weight || !a->out) return fail(SDK_EINVAL, "conv2d: null weight/out");
  p = Params{};
  p.batch = a->batch; p.ho = a->ho; p.wo = a->wo; p.hw_out = a->ho * a->wo;
  p.M = a->batch * p.hw_out;
  p.N = a->cout;
  p.Npad = (a->cout + BN - 1) / BN * BN;
  p.nseg = a->nseg;
  double kreal = 0;
  int kt = 0, koff = 0;
  for (int s = 0; s < a->nseg; ++s) {
    const sdk_conv_src& g = a->seg[s];
    Seg& d = p.seg[s];
    if (!g.src0) return fail(SDK_EINVAL, "conv2d: null src0");
    if (g.cin <= 0 || g.cin % 8 || g.c_split % 8 || g.c_split <= 0 || g.c_split > g.cin)
      return fail(SDK_EINVAL, "conv2d: cin/c_split must be positive multiples of 8 (c_split <= cin)");
    if (g.c_split < g.cin && !g.src1) return fail(SDK_EINVAL, "conv2d: concat without src1");
    if (g.ld0 % 8 || (g.c_split < g.cin && g.ld1 % 8)) return fail(SDK_EINVAL, "conv2d: ld must be a multiple of 8");
    if (g.ksize != 1 && g.ksize != 3) return fail(SDK_EINVAL, "conv2d: ksize must be 1 or 3");
    if ((g.gn_scale == nullptr) != (g.gn_shift == nullptr)) return fail(SDK_EINVAL, "conv2d: gn scale/shift pair");
    const int lh = g.upsample ? 2 * g.h : g.h, lw = g.upsample ? 2 * g.w : g.w;
    const int eh = (lh + 2 * g.pad - g.ksize) / g.stride + 1, ew = (lw + 2 * g.pad - g.ksize) / g.stride + 1;
    if (eh != a->ho || ew != a->wo) return fail(SDK_EINVAL, "conv2d: output size does not match source geometry");
    d.src0 = (const half_t*)g.src0; d.src1 = (const half_t*)g.src1;
    d.gscale = g.gn_scale; d.gshift = g.gn_shift;
    d.c_split = g.c_split; d.cin = g.cin; d.cin_pad = (g.cin + BK - 1) / BK * BK;
    d.ld0 = g.ld0; d.ld1 = g.ld1; d.h = g.h; d.w = g.w; d.ksize = g.ksize; d.stride = g.stride; d.pad = g.pad;
    d.upsample = g.upsample; d.silu = g.silu;
    d.k_off = koff; d.tiles_per_tap = d.cin_pad / BK; d.kt_begin = kt;
    const int taps = g.ksize * g.ksize;
    kt += taps * d.tiles_per_tap;
    koff += taps * d.cin_pad;
    kreal += (double)taps * g.cin;
  }
  if (koff != a->k_total) return fail(SDK_EINVAL, "conv2d: k_total does not match the packed segment layout");
  if (a->out_mode == SDK_OUT_NHWC_F16 || a->out_mode == SDK_OUT_GEGLU_F16) {
    if (a->cout % 8 || a->out_ld % 8 || (a->residual && a->res_ld % 8))
      return fail(SDK_EINVAL, "conv2d: fp16 NHWC output needs cout/out_ld/res_ld multiples of 8");
  }
  if (a->out_mode == SDK_OUT_GEGLU_F16 && (a->cout % 64)) return fail(SDK_EINVAL, "conv2d: GEGLU cout % 64");
  p.kt_total = kt;
  p.W = (const half_t*)a->weight; p.ldw = a->k_total;
  p.bias = a->bias; p.row_bias = a->row_bias; p.rb_ld = a->row_bias_ld;
  p.res = (const half_t*)a->residual; p.res_ld = a->res_ld;
  p.out = a->out; p.out_ld = a->out_ld; p.out_mode = a->out_mode;
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = p.Npad / BN;
  const int tiles = p.tiles_m * p.tiles_n;
  int split = a->split_k;
  if (split <= 0) {
    split = 1;
    // fill the 256 CUs x 2 resident workgroups; keep >= 8 K tiles per split
    while (tiles * split < 384 && kt / (split * 2) >= 8 && split < 16) split *= 2;
  }
  if (a->out_mode == SDK_OUT_GEGLU_F16 || a->cout % 8) split = 1;
  if (split > kt) split = kt;
  p.kt_per_split = (kt + split - 1) / split;
  split = (kt + p.kt_per_split - 1) / p.kt_per_split;
  p.split = split;
  const int64_t ws = split > 1 ? (int64_t)split * p.M * p.Npad * 4 : 0;
  if (info) {
    info->split_k = split;
    info->grid_tiles = tiles;
    info->workspace_bytes = ws;
    info->variant = split > 1 ? 1 : 0;
    info->flops = 2.0 * p.M * (double)p.N * kreal;
  }
  if (split > 1) {
    if (a->cout % 8) return fail(SDK_EINVAL, "conv2d: split-K needs cout % 8 == 0 (pass split_k = 1)");
    p.partial = a->workspace;
  }
  return SDK_OK;
}

}  // namespace
}  // namespace sdk

using namespace sdk;

extern "C" int sdk_conv2d_plan(const sdk_conv_args* a, sdk_conv_plan_info* info) {
  Params p;
  return build_params(a, p, info);
}

extern "C" int sdk_conv2d(const sdk_conv_args* a, sdk_stream_t stream) {
  Params p;
  sdk_conv_plan_info info;
  int rc = build_params(a, p, &info);
  if (rc) return rc;
  if (p.split > 1 && (!a->workspace || a->workspace_bytes < info.workspace_bytes))
    return fail(SDK_EWORKSPACE, "conv2d: split-K workspace too small");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(p.tiles_m * p.tiles_n, p.split);
  hipLaunchKernelGGL(conv_igemm_kernel, grid, dim3(NT), 0, s, p);
  if (int e = check_launch("conv_igemm")) return e;
  if (p.split > 1) {
    const size_t total = (size_t)p.M * (p.N / 8);
    int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, p);
    if (int e = check_launch("splitk_reduce")) return e;
  }
  return SDK_OK;
}
