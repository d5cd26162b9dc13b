// MS-SSIM of the YUV420 distortion path (calc_msssim, DCVC-DC/src/utils/
// metrics.py:15-62, as test_video.py:182-184 calls it per plane with
// data_range=1), in fp64 as the reference computes it.
//
//   * dcvc_yuv_planes_f64: the float64 planes calc_msssim receives: the
//     uint8/255 source planes and the clamped recon's ycbcr444_to_420 planes
//     (functional.py:75-95), cropped.
//   * dcvc_ssim_level: calc_ssim's 'valid' 11x11 Gaussian filtering of img1,
//     img2, img1^2, img2^2, img1*img2 (fftconvolve there, a direct fp64 sum
//     here: the same linear map, rounded differently at the 1e-16 level),
//     the ssim / cs maps and their means (fixed-order reduction).
//   * dcvc_down2_f64: ndimage.convolve(im, ones((2,2))/4, mode='reflect')
//     followed by [::2, ::2]: a 2x2 mean whose row/column beyond an odd edge
//     reflects to the edge itself.
#include "common.h"

namespace {

constexpr int SB = 256;
constexpr int SMAXB = 1024;

__device__ __forceinline__ double wsum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

struct Planes {
  double *src;  // [Y h*w | U hh*hw | V hh*hw]
  double *rec;
};

// one thread per 2x2 block of the crop: Y (4 pixels) and one U, V sample
__global__ void planes_kernel(const float *xh, int xW, int xcs, int xco, const uint8_t *ysrc,
                              const uint8_t *uvsrc, int h, int w, Planes pl) {
  const int hh = h / 2, hw = w / 2;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (int64_t)hh * hw) return;
  const int by = (int)(b / hw), bx = (int)(b - (int64_t)by * hw);
  float v[2][2][3];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const float *p = xh + ((int64_t)(2 * by + dy) * xW + 2 * bx + dx) * xcs + xco;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[dy][dx][c] = fminf(fmaxf(p[c], 0.f), 1.f);
    }
  const int64_t plane = (int64_t)h * w, cplane = (int64_t)hh * hw;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int64_t o = (int64_t)(2 * by + dy) * w + 2 * bx + dx;
      pl.src[o] = (double)((float)ysrc[o] / 255.f);
      pl.rec[o] = (double)v[dy][dx][0];
    }
#pragma unroll
  for (int c = 1; c < 3; ++c) {
    const float s = (v[0][0][c] + v[0][1][c]) + (v[1][0][c] + v[1][1][c]);
    const int64_t o = plane + (int64_t)(c - 1) * cplane + b;
    pl.src[o] = (double)((float)uvsrc[(int64_t)(c - 1) * cplane + b] / 255.f);
    pl.rec[o] = (double)fminf(fmaxf(s / 4.f, 0.f), 1.f);
  }
}

// calc_ssim for one level: one thread per 'valid' output pixel, 11x11 window
__global__ void __launch_bounds__(SB) ssim_kernel(const double *a, const double *b, int h, int w,
                                                  const double *win, double C1, double C2, double *part) {
  __shared__ double wl[121];
  __shared__ double red[SB / 64][2];
  for (int i = threadIdx.x; i < 121; i += SB) wl[i] = win[i];
  __syncthreads();
  const int oh = h - 10, ow = w - 10;
  const int64_t n = (int64_t)oh * ow;
  double s_ssim = 0.0, s_cs = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * SB + threadIdx.x; i < n; i += (int64_t)gridDim.x * SB) {
    const int oy = (int)(i / ow), ox = (int)(i - (int64_t)oy * ow);
    double m1 = 0.0, m2 = 0.0, s11 = 0.0, s22 = 0.0, s12 = 0.0;
    for (int ky = 0; ky < 11; ++ky) {
      const double *ra = a + (int64_t)(oy + ky) * w + ox;
      const double *rb = b + (int64_t)(oy + ky) * w + ox;
#pragma unroll
      for (int kx = 0; kx < 11; ++kx) {
        // fftconvolve(window, img): a convolution, i.e. the window flipped;
        // fspecial_gauss is symmetric, so the flip is the identity
        const double g = wl[(10 - ky) * 11 + (10 - kx)];
        const double x = ra[kx], y = rb[kx];
        m1 += g * x;
        m2 += g * y;
        s11 += g * (x * x);
        s22 += g * (y * y);
        s12 += g * (x * y);
      }
    }
    const double m1s = m1 * m1, m2s = m2 * m2, m12 = m1 * m2;
    const double v1 = s11 - m1s, v2 = s22 - m2s, v12 = s12 - m12;
    s_ssim += ((2 * m12 + C1) * (2 * v12 + C2)) / ((m1s + m2s + C1) * (v1 + v2 + C2));
    s_cs += (2.0 * v12 + C2) / (v1 + v2 + C2);
  }
  s_ssim = wsum(s_ssim);
  s_cs = wsum(s_cs);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[wv][0] = s_ssim;
    red[wv][1] = s_cs;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < SB / 64; ++k) s += red[k][threadIdx.x];
    part[2 * blockIdx.x + threadIdx.x] = s;
  }
}

// fixed-order sum of the block partials, divided by the map size: the means
__global__ void __launch_bounds__(256) ssim_final_kernel(const double *part, int nb, double inv_n, double *out) {
  __shared__ double red[4][2];
  double a0 = 0.0, a1 = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) {
    a0 += part[2 * b];
    a1 += part[2 * b + 1];
  }
  a0 = wsum(a0);
  a1 = wsum(a1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[wv][0] = a0;
    red[wv][1] = a1;
  }
  __syncthreads();
  if (threadIdx.x < 2)
    out[threadIdx.x] = (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x]) *
                       inv_n;
}

__global__ void down2_kernel(const double *in, int h, int w, double *out) {
  const int oh = (h + 1) / 2, ow = (w + 1) / 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)oh * ow) return;
  const int oy = (int)(i / ow), ox = (int)(i - (int64_t)oy * ow);
  const int y0 = 2 * oy, x0 = 2 * ox;
  const int y1 = min(y0 + 1, h - 1), x1 = min(x0 + 1, w - 1);  // 'reflect' past the last row / column
  const double s = ((in[(int64_t)y0 * w + x0] + in[(int64_t)y0 * w + x1]) + in[(int64_t)y1 * w + x0]) +
                   in[(int64_t)y1 * w + x1];
  out[i] = s * 0.25;
}

unsigned nblocks(int64_t n) {
  const int64_t g = (n + SB - 1) / SB;
  return (unsigned)(g < SMAXB ? (g > 0 ? g : 1) : SMAXB);
}

}  // namespace

extern "C" int dcvc_yuv_planes_f64(dcvc_tensor x_hat, const uint8_t *y, const uint8_t *uv, int h, int w,
                                   double *src_planes, double *rec_planes, void *stream) {
  if (!x_hat.ptr || x_hat.dtype != DCVC_F32 || x_hat.C != 3 || x_hat.H < h || x_hat.W < w || !y || !uv ||
      !src_planes || !rec_planes || h < 2 || w < 2 || (h & 1) || (w & 1))
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)(h / 2) * (w / 2);
  hipLaunchKernelGGL(planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const float *>(x_hat.ptr), x_hat.W, x_hat.cstride, x_hat.coff, y, uv, h, w,
                     Planes{src_planes, rec_planes});
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int64_t dcvc_ssim_workspace(void) { return (int64_t)2 * SMAXB * sizeof(double); }

extern "C" int dcvc_ssim_level(const double *a, const double *b, int h, int w, const double *window121, double C1,
                               double C2, double *workspace, double *out2, void *stream) {
  if (!a || !b || !window121 || !workspace || !out2 || h < 11 || w < 11) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)(h - 10) * (w - 10);
  const unsigned g = nblocks(n);
  hipLaunchKernelGGL(ssim_kernel, dim3(g), dim3(SB), 0, st, a, b, h, w, window121, C1, C2, workspace);
  DCVC_LAUNCH_CHECK();
  hipLaunchKernelGGL(ssim_final_kernel, dim3(1), dim3(256), 0, st, workspace, (int)g, 1.0 / (double)n, out2);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_down2_f64(const double *in, int h, int w, double *out, void *stream) {
  if (!in || !out || h < 1 || w < 1) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)((h + 1) / 2) * ((w + 1) / 2);
  hipLaunchKernelGGL(down2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, h, w, out);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// ---- RGB MS-SSIM (pytorch_msssim.ms_ssim as DCVC-DC/test_video.py:188 and
// DCVC-HEM/test_video.py:153 call it; the package is not installed here, so
// this follows its published algorithm: same Gaussian statistics per level,
// downsampling by F.avg_pool2d(kernel 2, padding = size % 2,
// count_include_pad=True), relu on cs / ssim).
namespace {

__global__ void rgb_planes_kernel(const float *xh, int xW, int xcs, int xco, const uint8_t *src, int h, int w,
                                  double *sp, double *rp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)h * w;
  if (i >= n) return;
  const int y = (int)(i / w), x = (int)(i - (int64_t)y * w);
  const float *p = xh + ((int64_t)y * xW + x) * xcs + xco;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    sp[c * n + i] = (double)((float)src[c * n + i] / 255.f);
    rp[c * n + i] = (double)fminf(fmaxf(p[c], 0.f), 1.f);
  }
}

// F.avg_pool2d(kernel_size=2, stride=2, padding=(h % 2, w % 2)),
// count_include_pad=True: output (h + 2 ph - 2) / 2 + 1 rows; window i covers
// input rows 2i - ph, 2i - ph + 1 (zeros outside), always divided by 4
__global__ void avgpool2_kernel(const double *in, int h, int w, double *out) {
  const int ph = h & 1, pw = w & 1;
  const int oh = (h + 2 * ph - 2) / 2 + 1, ow = (w + 2 * pw - 2) / 2 + 1;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)oh * ow) return;
  const int oy = (int)(i / ow), ox = (int)(i - (int64_t)oy * ow);
  double s = 0.0;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int y = 2 * oy - ph + dy, x = 2 * ox - pw + dx;
      if (y >= 0 && y < h && x >= 0 && x < w) s += in[(int64_t)y * w + x];
    }
  out[i] = s / 4.0;
}

}  // namespace

extern "C" int dcvc_rgb_planes_f64(dcvc_tensor x_hat, const uint8_t *src, int h, int w, double *src_planes,
                                   double *rec_planes, void *stream) {
  if (!x_hat.ptr || x_hat.dtype != DCVC_F32 || x_hat.C != 3 || x_hat.H < h || x_hat.W < w || !src ||
      !src_planes || !rec_planes || h < 1 || w < 1)
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)h * w;
  hipLaunchKernelGGL(rgb_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const float *>(x_hat.ptr), x_hat.W, x_hat.cstride, x_hat.coff, src, h, w,
                     src_planes, rec_planes);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_avgpool2_f64(const double *in, int h, int w, double *out, void *stream) {
  if (!in || !out || h < 2 || w < 2) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int oh = (h + 2 * (h & 1) - 2) / 2 + 1, ow = (w + 2 * (w & 1) - 2) / 2 + 1;
  const int64_t n = (int64_t)oh * ow;
  hipLaunchKernelGGL(avgpool2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, h, w, out);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}
