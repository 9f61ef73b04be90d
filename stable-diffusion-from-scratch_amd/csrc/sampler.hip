// Sampler-side elementwise kernels (HBM-bound, fp32) and layout glue, plus the
// library's error/introspection entry points.
//
// The DDIM / DDPM updates are compiled with floating-point contraction OFF
// (see the pragma) so each a*b+c is two correctly-rounded operations, exactly
// as torch's CPU kernels evaluate the reference expression; fed the same
// inputs the result is bit-identical to the oracle.
#include <cmath>
#include <cstdio>

#include "common.h"

#pragma clang fp contract(off)

namespace sdk {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SDK_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  return SDK_OK;
}

namespace {

__global__ void __launch_bounds__(256) ddim_step_kernel(sdk_ddim_args a) {
  const int64_t n4 = a.n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f4 x = reinterpret_cast<const f4*>(a.x)[i];
    f4 e = reinterpret_cast<const f4*>(a.e)[i];
    if (a.e_uncond) {
      const f4 u = reinterpret_cast<const f4*>(a.e_uncond)[i];
      f4 d;
      for (int j = 0; j < 4; ++j) d[j] = e[j] - u[j];
      for (int j = 0; j < 4; ++j) e[j] = u[j] + a.guidance * d[j];
    }
    if (a.v_param) {
      for (int j = 0; j < 4; ++j) {
        const float t0 = a.v_sqrt_a * e[j];
        const float t1 = a.v_sqrt_1ma * x[j];
        e[j] = t0 + t1;
      }
    }
    f4 nz = {0.f, 0.f, 0.f, 0.f};
    if (a.noise) nz = reinterpret_cast<const f4*>(a.noise)[i];
    f4 xp, p0;
    for (int j = 0; j < 4; ++j) {
      const float t1 = a.sqrt_one_minus_at * e[j];
      const float t2 = x[j] - t1;
      const float pred = t2 / a.sqrt_at;
      const float dir = a.dir_coef * e[j];
      const float t3 = a.sqrt_a_prev * pred;
      const float t4 = t3 + dir;
      const float nn = (a.sigma * nz[j]) * a.temperature;
      xp[j] = t4 + nn;
      p0[j] = pred;
    }
    reinterpret_cast<f4*>(a.x_prev)[i] = xp;
    if (a.pred_x0) reinterpret_cast<f4*>(a.pred_x0)[i] = p0;
  }
}

__global__ void __launch_bounds__(256) ddpm_step_kernel(const float* x, const float* eps, const float* noise,
                                                        float* out, int64_t n, float inv_sqrt_alpha, float coef,
                                                        float sigma) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float t = coef * eps[i];
    float v = inv_sqrt_alpha * (x[i] - t);
    if (noise) v = v + sigma * noise[i];
    out[i] = v;
  }
}

__global__ void temb_kernel(const int64_t* t, const float* freqs, half_t* out, int batch, int dim) {
  const int half = dim / 2;
  const int b = blockIdx.x;
  const float tf = (float)t[b];
  for (int k = threadIdx.x; k < dim; k += blockDim.x) {
    float v = 0.f;
    if (k < half) v = cosf(tf * freqs[k]);
    else if (k < 2 * half) v = sinf(tf * freqs[k - half]);
    out[(size_t)b * dim + k] = (half_t)v;
  }
}

__global__ void __launch_bounds__(256) nchw_to_nhwc_kernel(const float* x, half_t* y, int C, int HW, int Cp,
                                                           float scale) {
  // grid (ceil(HW/64), B); tile 64 pixels x C through LDS so both sides are coalesced
  __shared__ float tile[64][33];
  const int b = blockIdx.y, p0 = blockIdx.x * 64;
  for (int c0 = 0; c0 < Cp; c0 += 32) {
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int cc = e / 64, pp = e % 64;
      const int c = c0 + cc, pix = p0 + pp;
      float v = 0.f;
      if (c < C && pix < HW) v = x[((size_t)b * C + c) * HW + pix] * scale;
      tile[pp][cc] = v;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int pp = e / 32, cc = e % 32;
      const int c = c0 + cc, pix = p0 + pp;
      if (c < Cp && pix < HW) y[((size_t)b * HW + pix) * Cp + c] = (half_t)tile[pp][cc];
    }
    __syncthreads();
  }
}

// grid-stride over the latent elements; moments = [mean | logvar] along channels (NCHW)
__global__ void __launch_bounds__(256) diag_gauss_kernel(const float* moments, const float* noise, float* z,
                                                         int channels, int hw, int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t per_img = (int64_t)channels * hw;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t b = i / per_img, r = i - b * per_img;
    const float mean = moments[b * 2 * per_img + r];
    float v = mean;
    if (noise) {
      const float lv = fminf(fmaxf(moments[b * 2 * per_img + per_img + r], -30.f), 20.f);
      const float sd = expf(0.5f * lv);
      v = mean + sd * noise[i];
    }
    z[i] = scale * v;
  }
}

__global__ void __launch_bounds__(256) stochastic_encode_kernel(const float* x0, const float* noise, float* out,
                                                                int64_t n, float sa, float s1ma) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float t0 = sa * x0[i];
    const float t1 = s1ma * noise[i];
    out[i] = t0 + t1;
  }
}

// one block per token row: 8 channels per thread, fp32 sum rounded once to fp16
__global__ void __launch_bounds__(128) token_embedding_kernel(const int64_t* ids, const float* tok, const float* pos,
                                                              half_t* out, int seq, int dim) {
  const int row = blockIdx.x, t = row % seq;
  const int64_t id = ids[row];
  for (int c = threadIdx.x * 4; c < dim; c += blockDim.x * 4) {
    const f4 a = *reinterpret_cast<const f4*>(tok + id * dim + c);
    const f4 b = *reinterpret_cast<const f4*>(pos + (int64_t)t * dim + c);
    h4 o;
    for (int j = 0; j < 4; ++j) o[j] = (half_t)(a[j] + b[j]);
    *reinterpret_cast<h4*>(out + (int64_t)row * dim + c) = o;
  }
}

// F.interpolate(scale_factor=2, mode="bilinear", align_corners=True) on NHWC fp16, 8 channels per
// thread: source coordinate = dst * (in - 1) / (out - 1), fp32 weights as torch computes them
__global__ void __launch_bounds__(256) upsample_bilinear2x_kernel(const half_t* x, half_t* y, int h, int w, int c,
                                                                  int64_t nvec) {
  const int c8 = c / 8, ho = 2 * h, wo = 2 * w;
  const float ry = ho > 1 ? (float)(h - 1) / (float)(ho - 1) : 0.f;
  const float rx = wo > 1 ? (float)(w - 1) / (float)(wo - 1) : 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nvec; e += stride) {
    const int cc = (int)(e % c8) * 8;
    int64_t r = e / c8;
    const int ox = (int)(r % wo); r /= wo;
    const int oy = (int)(r % ho);
    const int b = (int)(r / ho);
    const float sy = ry * oy, sx = rx * ox;
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = min(y0 + 1, h - 1), x1 = min(x0 + 1, w - 1);
    const float ly = sy - y0, lx = sx - x0, hy = 1.f - ly, hx = 1.f - lx;
    const half_t* base = x + (size_t)b * h * w * c + cc;
    const h8 a = *reinterpret_cast<const h8*>(base + ((size_t)y0 * w + x0) * c);
    const h8 bb = *reinterpret_cast<const h8*>(base + ((size_t)y0 * w + x1) * c);
    const h8 cq = *reinterpret_cast<const h8*>(base + ((size_t)y1 * w + x0) * c);
    const h8 d = *reinterpret_cast<const h8*>(base + ((size_t)y1 * w + x1) * c);
    h8 o;
    for (int j = 0; j < 8; ++j)
      o[j] = (half_t)(hy * (hx * (float)a[j] + lx * (float)bb[j]) + ly * (hx * (float)cq[j] + lx * (float)d[j]));
    *reinterpret_cast<h8*>(y + ((size_t)(b * ho + oy) * wo + ox) * c + cc) = o;
  }
}

// exact (erf) GELU, nn.GELU(): fp16 in / out, fp32 math
__global__ void __launch_bounds__(256) gelu_kernel(const half_t* x, half_t* y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = (float)x[i];
    y[i] = (half_t)(0.5f * v * (1.0f + erff(v * 0.70710678118654752f)));
  }
}

// patch p = ((ly*Lx + lx)*B + b): out[p][c][i][j] = z[b][c][ly*sy + i][lx*sx + j] (torch.nn.Unfold order)
__global__ void __launch_bounds__(256) extract_patches_kernel(const float* z, float* out, int B, int C, int H, int W,
                                                              int kh, int kw, int sy, int sx, int Lx, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += stride) {
    const int j = (int)(e % kw);
    int64_t r = e / kw;
    const int i = (int)(r % kh); r /= kh;
    const int c = (int)(r % C); r /= C;
    const int b = (int)(r % B);
    const int l = (int)(r / B);
    const int ly = l / Lx, lx = l - ly * Lx;
    out[e] = z[(((int64_t)b * C + c) * H + ly * sy + i) * W + lx * sx + j];
  }
}

// overlap-add of weighted decoded patches, normalised per pixel:
// out = sum_l w(l, y, x) * patch_l / sum_l w(l, y, x), w = pix_w[i][j] * (l_w ? l_w[l] : 1)
// (torch.nn.Fold of o*weighting divided by Fold(weighting)); one thread per output element
// gathers the <= ceil(ph/sy) x ceil(pw/sx) covering patches — no atomics, deterministic
__global__ void __launch_bounds__(256) fold_patches_kernel(const float* patches, const float* pix_w, const float* l_w,
                                                           float* out, int B, int C, int H, int W, int ph, int pw,
                                                           int sy, int sx, int Ly, int Lx, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += stride) {
    const int x = (int)(e % W);
    int64_t r = e / W;
    const int y = (int)(r % H); r /= H;
    const int c = (int)(r % C);
    const int b = (int)(r / C);
    const int ly0 = y >= ph ? (y - ph) / sy + 1 : 0, ly1 = min(Ly - 1, y / sy);
    const int lx0 = x >= pw ? (x - pw) / sx + 1 : 0, lx1 = min(Lx - 1, x / sx);
    float num = 0.f, den = 0.f;
    for (int ly = ly0; ly <= ly1; ++ly)
      for (int lx = lx0; lx <= lx1; ++lx) {
        const int l = ly * Lx + lx, i = y - ly * sy, j = x - lx * sx;
        float w = pix_w[i * pw + j];
        if (l_w) w = w * l_w[l];
        const float v = patches[((((int64_t)l * B + b) * C + c) * ph + i) * pw + j];
        num = num + v * w;
        den = den + w;
      }
    out[e] = num / den;   // 0/0 = NaN where no patch covers the pixel, as Fold / normalization
  }
}

}  // namespace
}  // namespace sdk

using namespace sdk;

extern "C" int sdk_upsample_bilinear2x(const void* x, void* y, int32_t batch, int32_t h, int32_t w,
                                       int32_t channels, sdk_stream_t stream) {
  if (!x || !y || batch <= 0 || h <= 0 || w <= 0 || channels <= 0 || channels % 8)
    return fail(SDK_EINVAL, "upsample_bilinear2x: bad args (channels % 8)");
  const int64_t nvec = (int64_t)batch * 4 * h * w * (channels / 8);
  const int blocks = (int)std::min<int64_t>((nvec + 255) / 256, 8192);
  hipLaunchKernelGGL(upsample_bilinear2x_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const half_t*)x,
                     (half_t*)y, h, w, channels, nvec);
  return check_launch("upsample_bilinear2x");
}

extern "C" int sdk_gelu(const void* x, void* y, int64_t n, sdk_stream_t stream) {
  if (!x || !y || n <= 0) return fail(SDK_EINVAL, "gelu: bad args");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(gelu_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const half_t*)x, (half_t*)y, n);
  return check_launch("gelu");
}

extern "C" int sdk_extract_patches(const float* z, float* out, int32_t batch, int32_t channels, int32_t h, int32_t w,
                                   int32_t kh, int32_t kw, int32_t sy, int32_t sx, sdk_stream_t stream) {
  if (!z || !out || batch <= 0 || channels <= 0 || kh <= 0 || kw <= 0 || sy <= 0 || sx <= 0 || kh > h || kw > w)
    return fail(SDK_EINVAL, "extract_patches: bad geometry");
  const int Ly = (h - kh) / sy + 1, Lx = (w - kw) / sx + 1;
  const int64_t n = (int64_t)Ly * Lx * batch * channels * kh * kw;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(extract_patches_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, z, out, batch, channels,
                     h, w, kh, kw, sy, sx, Lx, n);
  return check_launch("extract_patches");
}

extern "C" int sdk_fold_patches(const float* patches, const float* pix_w, const float* l_w, float* out, int32_t batch,
                                int32_t channels, int32_t h, int32_t w, int32_t ph, int32_t pw, int32_t sy, int32_t sx,
                                int32_t ly, int32_t lx, sdk_stream_t stream) {
  if (!patches || !pix_w || !out || batch <= 0 || channels <= 0 || ph <= 0 || pw <= 0 || sy <= 0 || sx <= 0 ||
      ly <= 0 || lx <= 0 || (ly - 1) * sy + ph > h || (lx - 1) * sx + pw > w)
    return fail(SDK_EINVAL, "fold_patches: bad geometry");
  const int64_t n = (int64_t)batch * channels * h * w;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(fold_patches_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, patches, pix_w, l_w, out,
                     batch, channels, h, w, ph, pw, sy, sx, ly, lx, n);
  return check_launch("fold_patches");
}

extern "C" int sdk_token_embedding(const int64_t* ids, const float* tok, const float* pos, void* out, int32_t batch,
                                   int32_t seq, int32_t dim, sdk_stream_t stream) {
  if (!ids || !tok || !pos || !out || batch <= 0 || seq <= 0 || dim <= 0 || dim % 4)
    return fail(SDK_EINVAL, "token_embedding: bad args (dim must be a multiple of 4)");
  hipLaunchKernelGGL(token_embedding_kernel, dim3(batch * seq), dim3(128), 0, (hipStream_t)stream, ids, tok, pos,
                     (half_t*)out, seq, dim);
  return check_launch("token_embedding");
}

extern "C" int sdk_diag_gaussian_sample(const float* moments, const float* noise, float* z, int32_t batch,
                                        int32_t channels, int32_t hw, float scale, sdk_stream_t stream) {
  if (!moments || !z || batch <= 0 || channels <= 0 || hw <= 0) return fail(SDK_EINVAL, "diag_gaussian_sample: bad args");
  const int64_t n = (int64_t)batch * channels * hw;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(diag_gauss_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, moments, noise, z, channels,
                     hw, n, scale);
  return check_launch("diag_gaussian_sample");
}

extern "C" int sdk_stochastic_encode(const float* x0, const float* noise, float* out, int64_t n, float sqrt_a,
                                     float sqrt_1ma, sdk_stream_t stream) {
  if (!x0 || !noise || !out || n <= 0) return fail(SDK_EINVAL, "stochastic_encode: bad args");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(stochastic_encode_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x0, noise, out, n,
                     sqrt_a, sqrt_1ma);
  return check_launch("stochastic_encode");
}

extern "C" int sdk_ddim_step(const sdk_ddim_args* a, sdk_stream_t stream) {
  if (!a || !a->x || !a->e || !a->x_prev) return fail(SDK_EINVAL, "ddim_step: null pointer");
  if (a->n <= 0 || a->n % 4) return fail(SDK_EINVAL, "ddim_step: n must be a positive multiple of 4");
  const int64_t n4 = a->n / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(ddim_step_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *a);
  return check_launch("ddim_step");
}

extern "C" int sdk_ddpm_step(const float* x, const float* eps, const float* noise, float* out, int64_t n,
                             float inv_sqrt_alpha, float coef, float sigma, sdk_stream_t stream) {
  if (!x || !eps || !out || n <= 0) return fail(SDK_EINVAL, "ddpm_step: bad args");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(ddpm_step_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, eps, noise, out, n,
                     inv_sqrt_alpha, coef, sigma);
  return check_launch("ddpm_step");
}

extern "C" int sdk_timestep_embedding(const int64_t* t, const float* freqs, void* out, int32_t batch, int32_t dim,
                                      sdk_stream_t stream) {
  if (!t || !freqs || !out || batch <= 0 || dim <= 0) return fail(SDK_EINVAL, "timestep_embedding: bad args");
  hipLaunchKernelGGL(temb_kernel, dim3(batch), dim3(256), 0, (hipStream_t)stream, t, freqs, (half_t*)out, batch,
                     dim);
  return check_launch("timestep_embedding");
}

extern "C" int sdk_nchw_to_nhwc(const float* x, void* y, int32_t batch, int32_t channels, int32_t hw, int32_t c_pad,
                                float scale, sdk_stream_t stream) {
  if (!x || !y || batch <= 0 || channels <= 0 || hw <= 0 || c_pad < channels)
    return fail(SDK_EINVAL, "nchw_to_nhwc: bad args");
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3((hw + 63) / 64, batch), dim3(256), 0, (hipStream_t)stream, x,
                     (half_t*)y, channels, hw, c_pad, scale);
  return check_launch("nchw_to_nhwc");
}

extern "C" const char* sdk_last_error(void) { return g_last_error.c_str(); }

extern "C" int sdk_version(void) { return 1; }

extern "C" const char* sdk_kernel_name(int32_t variant) {
  switch (variant) {
    case 0: return "conv_igemm_kernel";
    case 2: return "conv_glds_kernel<Cfg<256,256,2,4>>";
    case 3: return "conv_glds_kernel<Cfg<256,128,4,2>>";
    case 4: return "conv_glds_kernel<Cfg<128,128,2,2>>";
    case 5: return "conv_glds_kernel<Cfg<256,320,8,2>>";
    case 6: return "conv_glds_kernel<Cfg<256,160,8,1>>";
    case 7: return "conv_glds_kernel<Cfg<128,320,4,2>>";
    case 8: return "conv_ph_kernel<256x256,ring8>";
    case 9: return "conv_ph_kernel<256x256,ring10>";
    case 16: return "conv_glds_kernel<Cfg<128,128,2,2,4>>";
    case 17: return "conv_glds_kernel<Cfg<256,128,4,2,3>>";
    case 18: return "conv_glds_kernel<Cfg<128,128,2,2,3>>";
    case 19: return "conv_glds_kernel<Cfg<128,256,2,4,3>>";
    case 20: return "conv_ph_kernel<256x256,ring8,m16>";
    case 21: return "conv_ph_kernel<256x256,ring10,m16>";
    case 22: return "conv_glds_kernel<Cfg<256,320,8,2,2,m16>>";
    case 23: return "conv_glds_kernel<Cfg<128,320,4,2,2,m16>>";
    case 24: return "conv_glds_kernel<Cfg<256,160,8,1,2,m16>>";
    case 25: return "conv_glds_kernel<Cfg<128,256,2,4,3,m16>>";
    case 26: return "conv_glds_kernel<Cfg<128,128,2,2,3,m16>>";
    case 31: return "conv_glds_kernel<Cfg<128,160,4,1,2,m16,occ2>>";
    case 32: return "conv_glds_kernel<Cfg<128,128,2,2,2,m16,occ2>>";
    case 33: return "conv_glds_kernel<Cfg<128,160,4,1,4,m16>>";
    case 34: return "conv_direct_kernel";
    case 35: return "conv_skinny_kernel";
    case 38: return "conv_glds_kernel<Cfg<256,320,4,2,2,m16>>";
    case 40: return "conv_glds_kernel<Cfg<256,256,2,4,2,m16>>";
    default: return "unknown";
  }
}
