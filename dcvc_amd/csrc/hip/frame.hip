// Harness-side frame kernels: YUV420 source frames into the codec's NHWC
// input, and the per-frame distortion of run_test (DCVC-DC/test_video.py:
// 108-195) with the in-place clamp of the reconstruction.
#include "common.h"

namespace {

struct FView {
  float *p;
  int H, W, cs, co;
};

__device__ __forceinline__ float u8f(uint8_t v) { return (float)v / 255.f; }

// scipy.ndimage.zoom(uv, (1, 2, 2), order=0) as ycbcr420_to_444(order=0)
// calls it (DCVC-DC/src/transforms/functional.py:61-72): output index i of an
// axis of length 2n samples input index round(i * (n - 1) / (2n - 1)).  The
// product i(n-1)/(2n-1) is never a half-integer (2i(n-1) is even, (2n-1)
// odd) and lies at least 1/(2(2n-1)) from one, so the double evaluation
// rounds exactly as scipy's does.
__device__ __forceinline__ int zoom_src(int i, int n) {
  if (n <= 1) return 0;
  const double z = (double)(n - 1) / (double)(2 * n - 1);
  return (int)floor((double)i * z + 0.5);
}

// ycbcr420_to_444(order=0) + np_image_to_tensor + F.pad(replicate) in one
// pass (test_video.py:111-132): uint8 Y (h x w) and UV (2 x h/2 x w/2) to
// fp32 NHWC [0, 1] of the padded size.
__global__ void yuv420_kernel(const uint8_t *__restrict__ ysrc, const uint8_t *__restrict__ uvsrc, int h, int w,
                              FView out) {
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (int64_t)out.H * out.W) return;
  const int py = (int)(pix / out.W), px = (int)(pix - (int64_t)py * out.W);
  const int sy = min(py, h - 1), sx = min(px, w - 1);
  const int hh = h / 2, hw = w / 2;
  const int uy = zoom_src(sy, hh), ux = zoom_src(sx, hw);
  float *o = out.p + pix * out.cs + out.co;
  o[0] = u8f(ysrc[(int64_t)sy * w + sx]);
  o[1] = u8f(uvsrc[(int64_t)uy * hw + ux]);
  o[2] = u8f(uvsrc[(int64_t)hh * hw + (int64_t)uy * hw + ux]);
}

constexpr int SSE_BLOCK = 256;
constexpr int SSE_MAX_BLOCKS = 1024;

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// Block sum of three doubles in a fixed order: wave shuffles, then the four
// wave results in index order.  Thread 0 writes part[3 * blockIdx.x + c].
__device__ void block_sum3(double a0, double a1, double a2, double *part) {
  __shared__ double red[SSE_BLOCK / 64][3];
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[wv][0] = a0;
    red[wv][1] = a1;
    red[wv][2] = a2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double s = 0.0;
    for (int i = 0; i < SSE_BLOCK / 64; ++i) s += red[i][threadIdx.x];
    part[3 * blockIdx.x + threadIdx.x] = s;
  }
}

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }

// RGB: recon_frame.clamp_(0, 1) over the padded frame (test_video.py:169),
// then per channel sum((x_hat - x)^2) over the crop, the difference and its
// square in fp32 as PSNR() forms them (:65-68), summed in fp64.
__global__ void __launch_bounds__(SSE_BLOCK) sse_rgb_kernel(FView xh, const uint8_t *__restrict__ src, int h,
                                                            int w, double *part) {
  double a[3] = {0.0, 0.0, 0.0};
  const int64_t n = (int64_t)xh.H * xh.W;
  for (int64_t pix = (int64_t)blockIdx.x * SSE_BLOCK + threadIdx.x; pix < n; pix += (int64_t)gridDim.x * SSE_BLOCK) {
    const int py = (int)(pix / xh.W), px = (int)(pix - (int64_t)py * xh.W);
    float *p = xh.p + pix * xh.cs + xh.co;
    const float v0 = clamp01(p[0]), v1 = clamp01(p[1]), v2 = clamp01(p[2]);
    p[0] = v0;
    p[1] = v1;
    p[2] = v2;
    if (py < h && px < w) {
      const int64_t o = (int64_t)py * w + px, plane = (int64_t)h * w;
      const float d0 = v0 - u8f(src[o]), d1 = v1 - u8f(src[plane + o]), d2 = v2 - u8f(src[2 * plane + o]);
      a[0] += (double)(d0 * d0);
      a[1] += (double)(d1 * d1);
      a[2] += (double)(d2 * d2);
    }
  }
  block_sum3(a[0], a[1], a[2], part);
}

// YUV420 (dist_in_yuv420, test_video.py:171-181): clamp_ in place, then
// ycbcr444_to_420 of the crop (U/V = float32 mean of each 2x2 block, summed
// (x00 + x01) + (x10 + x11) as numpy's mean over axes (-1, -3) does, then
// clip) and calc_psnr's fp64 squared error against the uint8/255 source
// planes (metrics.py:81-92).  One thread per 2x2 block of the padded frame.
__global__ void __launch_bounds__(SSE_BLOCK) sse_yuv420_kernel(FView xh, const uint8_t *__restrict__ ysrc,
                                                               const uint8_t *__restrict__ uvsrc, int h, int w,
                                                               double *part) {
  double a[3] = {0.0, 0.0, 0.0};
  const int bh = xh.H / 2, bw = xh.W / 2, hw = w / 2, hh = h / 2;
  const int64_t n = (int64_t)bh * bw;
  for (int64_t b = (int64_t)blockIdx.x * SSE_BLOCK + threadIdx.x; b < n; b += (int64_t)gridDim.x * SSE_BLOCK) {
    const int by = (int)(b / bw), bx = (int)(b - (int64_t)by * bw);
    float v[2][2][3];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float *p = xh.p + ((int64_t)(2 * by + dy) * xh.W + 2 * bx + dx) * xh.cs + xh.co;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          v[dy][dx][c] = clamp01(p[c]);
          p[c] = v[dy][dx][c];
        }
      }
    if (by < hh && bx < hw) {
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          const double d = (double)v[dy][dx][0] - (double)u8f(ysrc[(int64_t)(2 * by + dy) * w + 2 * bx + dx]);
          a[0] += d * d;
        }
#pragma unroll
      for (int c = 1; c < 3; ++c) {
        const float s = (v[0][0][c] + v[0][1][c]) + (v[1][0][c] + v[1][1][c]);
        const float m = clamp01(s / 4.f);
        const double d = (double)m - (double)u8f(uvsrc[(int64_t)(c - 1) * hh * hw + (int64_t)by * hw + bx]);
        a[c] += d * d;
      }
    }
  }
  block_sum3(a[0], a[1], a[2], part);
}

__device__ __forceinline__ uint8_t q255(float v) {
  return (uint8_t)fminf(fmaxf(rintf(v * 255.f), 0.f), 255.f);  // np.clip(np.rint(v * 255), 0, 255)
}

// dcvc_recon_to_u8, RGB: one thread per crop pixel, HWC uint8
__global__ void recon_rgb_u8_kernel(FView xh, int h, int w, uint8_t *out) {
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (int64_t)h * w) return;
  const int py = (int)(pix / w), px = (int)(pix - (int64_t)py * w);
  const float *p = xh.p + ((int64_t)py * xh.W + px) * xh.cs + xh.co;
#pragma unroll
  for (int c = 0; c < 3; ++c) out[pix * 3 + c] = q255(p[c]);
}

// dcvc_recon_to_u8, YUV420: one thread per 2x2 block of the crop; Y of the
// four pixels and the block's U, V means, ycbcr444_to_420 of the values as
// given (clip after the mean; run_test hands over the frame already clamped)
// with sse_yuv420_kernel's summation order
__global__ void recon_yuv_u8_kernel(FView xh, int h, int w, uint8_t *out) {
  const int hh = h / 2, hw = w / 2;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (int64_t)hh * hw) return;
  const int by = (int)(b / hw), bx = (int)(b - (int64_t)by * hw);
  float s[3] = {0.f, 0.f, 0.f};
  float v[2][2][3];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const float *p = xh.p + ((int64_t)(2 * by + dy) * xh.W + 2 * bx + dx) * xh.cs + xh.co;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[dy][dx][c] = p[c];
      out[(int64_t)(2 * by + dy) * w + 2 * bx + dx] = q255(clamp01(v[dy][dx][0]));
    }
#pragma unroll
  for (int c = 1; c < 3; ++c) {
    s[c] = (v[0][0][c] + v[0][1][c]) + (v[1][0][c] + v[1][1][c]);
    out[(int64_t)h * w + (int64_t)(c - 1) * hh * hw + b] = q255(clamp01(s[c] / 4.f));
  }
}

// Fixed-order final reduction of the per-block partials: out[c] = sum_b part[3b + c].
__global__ void __launch_bounds__(256) sse_final_kernel(const double *part, int nb, double *out) {
  __shared__ double red[4][3];
  double a[3] = {0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nb; b += 256)
#pragma unroll
    for (int c = 0; c < 3; ++c) a[c] += part[3 * b + c];
#pragma unroll
  for (int c = 0; c < 3; ++c) a[c] = wave_sum(a[c]);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < 3; ++c) red[wv][c] = a[c];
  __syncthreads();
  if (threadIdx.x < 3) out[threadIdx.x] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                          red[3][threadIdx.x];
}

bool frame_ok(const dcvc_tensor &t) {
  return t.ptr && t.dtype == DCVC_F32 && t.C == 3 && t.H > 0 && t.W > 0 && t.coff >= 0 && t.coff + 3 <= t.cstride;
}

FView fv(const dcvc_tensor &t) { return FView{reinterpret_cast<float *>(t.ptr), t.H, t.W, t.cstride, t.coff}; }

unsigned sse_blocks(int64_t n) {
  const int64_t g = (n + SSE_BLOCK - 1) / SSE_BLOCK;
  return (unsigned)(g < SSE_MAX_BLOCKS ? (g > 0 ? g : 1) : SSE_MAX_BLOCKS);
}

}  // namespace

extern "C" int dcvc_yuv420_to_nhwc(const uint8_t *y, const uint8_t *uv, int h, int w, dcvc_tensor out,
                                   void *stream) {
  if (!y || !uv || !frame_ok(out) || h < 2 || w < 2 || (h & 1) || (w & 1) || out.H < h || out.W < w)
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)out.H * out.W;
  hipLaunchKernelGGL(yuv420_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, uv, h, w, fv(out));
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int64_t dcvc_frame_sse_workspace(void) { return (int64_t)3 * SSE_MAX_BLOCKS * sizeof(double); }

extern "C" int dcvc_frame_sse(dcvc_tensor x_hat, const uint8_t *src, const uint8_t *uv, int h, int w, int yuv420,
                              double *workspace, double *out3, void *stream) {
  if (!frame_ok(x_hat) || !src || !workspace || !out3 || h <= 0 || w <= 0 || x_hat.H < h || x_hat.W < w)
    return DCVC_HIP_EINVAL;
  if (yuv420 && (!uv || (h & 1) || (w & 1) || (x_hat.H & 1) || (x_hat.W & 1))) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  unsigned g;
  if (yuv420) {
    g = sse_blocks((int64_t)(x_hat.H / 2) * (x_hat.W / 2));
    hipLaunchKernelGGL(sse_yuv420_kernel, dim3(g), dim3(SSE_BLOCK), 0, st, fv(x_hat), src, uv, h, w, workspace);
  } else {
    g = sse_blocks((int64_t)x_hat.H * x_hat.W);
    hipLaunchKernelGGL(sse_rgb_kernel, dim3(g), dim3(SSE_BLOCK), 0, st, fv(x_hat), src, h, w, workspace);
  }
  DCVC_LAUNCH_CHECK();
  hipLaunchKernelGGL(sse_final_kernel, dim3(1), dim3(256), 0, st, workspace, (int)g, out3);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_recon_to_u8(dcvc_tensor x_hat, int h, int w, int yuv420, uint8_t *out, void *stream) {
  if (!frame_ok(x_hat) || !out || h <= 0 || w <= 0 || x_hat.H < h || x_hat.W < w) return DCVC_HIP_EINVAL;
  if (yuv420 && ((h & 1) || (w & 1))) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = yuv420 ? (int64_t)(h / 2) * (w / 2) : (int64_t)h * w;
  if (yuv420)
    hipLaunchKernelGGL(recon_yuv_u8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, fv(x_hat), h, w, out);
  else
    hipLaunchKernelGGL(recon_rgb_u8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, fv(x_hat), h, w, out);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}
