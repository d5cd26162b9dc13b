// DCVC-HEM specific kernels: the dual (checkerboard) prior steps, int32
// factorized symbols, and the squeeze-excitation layer of the HEM UNet.
//
// Dual prior (DCVC-HEM/src/models/common_model.py:84-188).  Latent y has C
// channels; the spatial prior's input is one fp32 NHWC buffer
//   buf = [y_hat_0_0 | y_hat_1_1 (C) | means (C) | scales (C) | quant_step (C)]
// in the reference's torch.cat order (:124).  Step k = 0 codes channel half 0
// at mask_0 sites ((y + x) even) and half 1 at mask_1 sites, step k = 1 the
// complement, with scales/means from the spatial prior output
// sm = [scales_0 | means_0 | scales_1 | means_1] (C/2 each, :125).  One
// thread per (channel-in-half c, pixel), i = c * H * W + pixel: the NCHW
// order of y_q_w_k (:151-152), so symbols/indexes land in coder order.
#include "common.h"

namespace {

struct View {
  void *p;
  int H, W, C, cs, co;
};
View mk(const dcvc_tensor &t) { return View{t.ptr, t.H, t.W, t.C, t.cstride, t.coff}; }

bool ok(const dcvc_tensor &t) {
  return t.ptr && t.H > 0 && t.W > 0 && t.C > 0 && t.coff >= 0 && t.coff + t.C <= t.cstride &&
         (t.dtype == DCVC_F32 || t.dtype == DCVC_BF16);
}

inline unsigned blocks_for(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

struct DP {
  View y, buf, sm, yhat;
  int C;
  const float *post;  // optional per-channel factor applied after quant_step (curr_q)
};

__device__ __forceinline__ float bufv(const DP &t, int64_t pix, int ch) {
  return ld<float>(t.buf.p, pix * t.buf.cs + t.buf.co + ch);
}

// channel, scale, mean and quant step of site (c, pixel) at step k
__device__ __forceinline__ void dp_site(const DP &t, int k, int64_t pix, int py, int px, int c, int &ch, float &sc,
                                        float &me, float &qs, int &other) {
  const int C = t.C, C2 = C / 2;
  const bool m0 = ((py ^ px) & 1) == 0;
  const int half = (k == 0) ? (m0 ? 0 : 1) : (m0 ? 1 : 0);
  ch = half * C2 + c;
  other = (1 - half) * C2 + c;
  if (k == 0) {
    me = bufv(t, pix, C + ch);
    sc = bufv(t, pix, 2 * C + ch);
  } else {
    sc = ld<float>(t.sm.p, pix * t.sm.cs + t.sm.co + half * C + c);
    me = ld<float>(t.sm.p, pix * t.sm.cs + t.sm.co + half * C + C2 + c);
  }
  qs = fmaxf(bufv(t, pix, 3 * C + ch), 0.5f);  // LowerBound(quant_step, 0.5)
}

__device__ __forceinline__ int16_t scale_index(float s, float log_min, float log_step) {
  // GaussianEncoder.build_indexes (entropy_models/entropy_models.py:264-268)
  s = fmaxf(s, 1e-5f);
  float v = (logf(s) - log_min) / log_step;
  v = fminf(fmaxf(v, 0.f), 255.f);
  return (int16_t)(int)v;
}

// the y_hat outputs shared by encode / decode / estimate
__device__ __forceinline__ void dp_store(const DP &t, int k, int64_t pix, int ch, int other, float yh, float qs) {
  if (k == 0) {
    // y_hat_0_0 / y_hat_1_1 for the spatial prior: this site's channel, and
    // zero for the other half's channel (it is masked out at this site);
    // the spatial prior sees quant_step after LowerBound(., 0.5) (:118, :124)
    float *b = reinterpret_cast<float *>(t.buf.p) + pix * t.buf.cs + t.buf.co;
    b[ch] = yh;
    b[other] = 0.f;
    b[3 * t.C + ch] = qs;
    b[3 * t.C + other] = fmaxf(b[3 * t.C + other], 0.5f);
  }
  // y_hat * quant_step, then (video_model.py:278-279) * curr_q
  const float v = yh * qs;
  st<float>(t.yhat.p, pix * t.yhat.cs + t.yhat.co + ch, t.post ? v * t.post[ch] : v);
}

__global__ void dp_encode_kernel(DP t, int k, int32_t *sym, int16_t *idx, float log_min, float log_step) {
  const int C2 = t.C / 2;
  const int64_t HW = (int64_t)t.y.H * t.y.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C2) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  const int py = (int)(pix / t.y.W), px = (int)(pix - (int64_t)py * t.y.W);
  int ch, other;
  float sc, me, qs;
  dp_site(t, k, pix, py, px, c, ch, sc, me, qs, other);
  const float yv = ld<float>(t.y.p, pix * t.y.cs + t.y.co + ch) / qs;  // y / quant_step
  const float yq = rintf(yv - me);                                     // round((y - means) * mask)
  sym[i] = (int32_t)yq;
  idx[i] = scale_index(sc, log_min, log_step);
  dp_store(t, k, pix, ch, other, yq + me, qs);
}

__global__ void dp_index_kernel(DP t, int k, int16_t *idx, float log_min, float log_step) {
  const int C2 = t.C / 2;
  const int64_t HW = (int64_t)t.buf.H * t.buf.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C2) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  const int py = (int)(pix / t.buf.W), px = (int)(pix - (int64_t)py * t.buf.W);
  int ch, other;
  float sc, me, qs;
  dp_site(t, k, pix, py, px, c, ch, sc, me, qs, other);
  idx[i] = scale_index(sc, log_min, log_step);
}

__global__ void dp_decode_kernel(DP t, int k, const int32_t *sym) {
  const int C2 = t.C / 2;
  const int64_t HW = (int64_t)t.buf.H * t.buf.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C2) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  const int py = (int)(pix / t.buf.W), px = (int)(pix - (int64_t)py * t.buf.W);
  int ch, other;
  float sc, me, qs;
  dp_site(t, k, pix, py, px, c, ch, sc, me, qs, other);
  dp_store(t, k, pix, ch, other, (float)sym[i] + me, qs);  // (y_q_r + means) * mask
}

__device__ __forceinline__ float probs_to_bits(float p) {
  const float b = -1.f * logf(p + 1e-5f) / 0.6931471805599453f;  // LowerBound(bits, 0)
  return b > 0.f ? b : 0.f;
}
__device__ __forceinline__ float dist_cdf(int gaussian, float v, float s) {
  if (gaussian) return 0.5f * (1.f + erff(v * (1.f / s) / 1.4142135623730951f));
  const float sg = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
  return 0.5f - 0.5f * sg * expm1f(-fabsf(v) / s);
}

// estimate mode: y_hat outputs + per-site bits (get_y_laplace_bits with
// sigma >= 1e-5, get_y_gaussian_bits with sigma >= 0.11, common_model.py:58-70)
__global__ void dp_estimate_kernel(DP t, int k, float *bits, int gaussian, float smin) {
  const int C2 = t.C / 2;
  const int64_t HW = (int64_t)t.y.H * t.y.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C2) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  const int py = (int)(pix / t.y.W), px = (int)(pix - (int64_t)py * t.y.W);
  int ch, other;
  float sc, me, qs;
  dp_site(t, k, pix, py, px, c, ch, sc, me, qs, other);
  const float yv = ld<float>(t.y.p, pix * t.y.cs + t.y.co + ch) / qs;
  const float yq = rintf(yv - me);
  const float s = fminf(fmaxf(sc, smin), 1e10f);
  bits[i] = probs_to_bits(dist_cdf(gaussian, yq + 0.5f, s) - dist_cdf(gaussian, yq - 0.5f, s));
  dp_store(t, k, pix, ch, other, yq + me, qs);
}

// ---- int32 factorized symbols (BitEstimator.encode/decode_stream,
// entropy_models/entropy_models.py:182-195: x.reshape(-1).int(), no clamp)
template <typename TX>
__global__ void to_sym32_kernel(View x, int32_t *sym) {
  const int64_t HW = (int64_t)x.H * x.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * x.C) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  sym[i] = (int32_t)ld<TX>(x.p, pix * x.cs + x.co + c);
}

template <typename TY>
__global__ void from_sym32_kernel(const int32_t *sym, View y) {
  const int64_t HW = (int64_t)y.H * y.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * y.C) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  st<TY>(y.p, pix * y.cs + y.co + c, (float)sym[i]);
}

// ---- SELayer (models/video_net.py:157-170): y = mean_hw(x); s = sigmoid(W2
// relu(W1 y)); out = a + x * s[c] (ConvBlockResidual's up_dim(x) + SE(x1),
// :185-188).  The mean is a fixed-order two-stage sum (partial sums over
// pixel ranges, then one block), so it is reproducible.
constexpr int kSePart = 256;  // pixel ranges of the first stage (work = kSePart * C floats)

// V consecutive channels of one pixel as floats (16-byte loads when V > 1).
template <typename T, int V> struct VecLd;
template <> struct VecLd<uint16_t, 8> {
  __device__ __forceinline__ static void load(const void *p, int64_t i, float *v) {
    const uint4 q = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint16_t *>(p) + i);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(void *p, int64_t i, const float *v) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (uint32_t)f2bf(v[2 * j]) | ((uint32_t)f2bf(v[2 * j + 1]) << 16);
    *reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(p) + i) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct VecLd<float, 4> {
  __device__ __forceinline__ static void load(const void *p, int64_t i, float *v) {
    const float4 q = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + i);
    v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
  }
  __device__ __forceinline__ static void store(void *p, int64_t i, const float *v) {
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <typename T> struct VecLd<T, 1> {
  __device__ __forceinline__ static void load(const void *p, int64_t i, float *v) { v[0] = ld<T>(p, i); }
  __device__ __forceinline__ static void store(void *p, int64_t i, const float *v) { st<T>(p, i, v[0]); }
};

// Stage 1: block b sums pixels [b * n / kSePart, (b + 1) * n / kSePart).
// Thread t owns channel vector t % CV of pixel lane t / CV (CV = C / V
// vectors per pixel, lanes = 256 / CV pixels per iteration), so a wave reads
// whole contiguous pixels; lanes are then folded in LDS in lane order.  The
// summation order is fixed by (n, C), so the mean is reproducible.
template <typename TX, int V>
__global__ __launch_bounds__(256) void se_partial_kernel(View x, float *part) {
  __shared__ float red[256 * V];
  const int C = x.C, CV = C / V, lanes = 256 / CV;
  const int t = threadIdx.x, lane = t / CV, cv = t - lane * CV;
  const int64_t n = (int64_t)x.H * x.W;
  const int64_t p0 = blockIdx.x * n / kSePart, p1 = (blockIdx.x + 1) * n / kSePart;
  float a[V];
#pragma unroll
  for (int j = 0; j < V; ++j) a[j] = 0.f;
  if (lane < lanes) {
    int64_t p = p0 + lane;
    for (; p + lanes < p1; p += 2 * lanes) {  // two pixels in flight per thread
      float u[V], w[V];
      VecLd<TX, V>::load(x.p, p * x.cs + x.co + cv * V, u);
      VecLd<TX, V>::load(x.p, (p + lanes) * x.cs + x.co + cv * V, w);
#pragma unroll
      for (int j = 0; j < V; ++j) a[j] += u[j] + w[j];
    }
    if (p < p1) {
      float u[V];
      VecLd<TX, V>::load(x.p, p * x.cs + x.co + cv * V, u);
#pragma unroll
      for (int j = 0; j < V; ++j) a[j] += u[j];
    }
#pragma unroll
    for (int j = 0; j < V; ++j) red[lane * C + cv * V + j] = a[j];
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float s = 0.f;
    for (int l = 0; l < lanes; ++l) s += red[l * C + c];
    part[(int64_t)blockIdx.x * C + c] = s;
  }
}

// Scalar fallback (channel views that are not 16-byte aligned, or C / V > 256).
template <typename TX>
__global__ void se_partial_scalar_kernel(View x, float *part) {
  const int64_t n = (int64_t)x.H * x.W;
  const int64_t p0 = blockIdx.x * n / kSePart, p1 = (blockIdx.x + 1) * n / kSePart;
  for (int c = threadIdx.x; c < x.C; c += blockDim.x) {
    float a = 0.f;
    for (int64_t p = p0; p < p1; ++p) a += ld<TX>(x.p, p * x.cs + x.co + c);
    part[(int64_t)blockIdx.x * x.C + c] = a;
  }
}

__global__ void se_fc_kernel(const float *part, int C, int R, float inv_n, const float *w1, const float *w2,
                             float *s) {
  __shared__ float mean[1024], hid[64], red[1024];
  // stage 2: 1024 threads = G groups of C' = min(C, 1024) channels; group g
  // sums ranges g, g + G, ...; groups are folded in order.
  for (int c0 = 0; c0 < C; c0 += 1024) {
    const int cc = min(C - c0, 1024), G = 1024 / cc;
    const int g = threadIdx.x / cc, c = threadIdx.x - g * cc;
    if (g < G) {
      float a = 0.f;
      for (int b = g; b < kSePart; b += G) a += part[b * C + c0 + c];
      red[g * cc + c] = a;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < cc; k += blockDim.x) {
      float a = 0.f;
      for (int q = 0; q < G; ++q) a += red[q * cc + k];
      mean[c0 + k] = a * inv_n;
    }
    __syncthreads();
  }
  for (int r = threadIdx.x; r < R; r += blockDim.x) {  // fc.0: Linear(C, C/16, bias=False) + ReLU
    float a = 0.f;
    for (int c = 0; c < C; ++c) a += w1[r * C + c] * mean[c];
    hid[r] = a > 0.f ? a : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {  // fc.2: Linear(C/16, C, bias=False) + Sigmoid
    float a = 0.f;
    for (int r = 0; r < R; ++r) a += w2[c * R + r] * hid[r];
    s[c] = 1.f / (1.f + expf(-a));
  }
}

template <typename T>
__global__ void fill_kernel(View y, float v) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * y.C) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  st<T>(y.p, pix * y.cs + y.co + c, v);
}

// y = x / q[c] (video_model.py:270, 289: y / curr_q, a true division)
__global__ void channel_div_kernel(View x, const float *q, View y) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * y.C) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  st<float>(y.p, pix * y.cs + y.co + c, ld<float>(x.p, pix * x.cs + x.co + c) / q[c]);
}

// y = a + x * s[c], V channels per thread (V = 1: scalar views)
template <typename T, int V>
__global__ void se_apply_kernel(View a, View x, const float *s, View y) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int CV = y.C / V;
  if (idx >= (int64_t)y.H * y.W * CV) return;
  const int c = (int)(idx % CV) * V;
  const int64_t pix = idx / CV;
  float u[V], w[V];
  VecLd<T, V>::load(x.p, pix * x.cs + x.co + c, u);
  VecLd<T, V>::load(a.p, pix * a.cs + a.co + c, w);
#pragma unroll
  for (int j = 0; j < V; ++j) w[j] += u[j] * s[c + j];
  VecLd<T, V>::store(y.p, pix * y.cs + y.co + c, w);
}

// 16-byte vector access to V consecutive channels is legal for this view
bool vec_ok(const dcvc_tensor &t, int V) {
  const int es = t.dtype == DCVC_F32 ? 4 : 2;
  return t.C % V == 0 && t.cstride % V == 0 && t.coff % V == 0 && (reinterpret_cast<uintptr_t>(t.ptr) % 16) == 0 &&
         V * es == 16;
}

bool dp_ok(const dcvc_tensor &buf, const dcvc_tensor &sm, int k, int C) {
  if (!ok(buf) || buf.dtype != DCVC_F32 || buf.C != 4 * C || C % 2 || k < 0 || k > 1) return false;
  if (k == 0) return sm.ptr == nullptr;
  return ok(sm) && sm.dtype == DCVC_F32 && sm.C == 2 * C && sm.H == buf.H && sm.W == buf.W;
}

}  // namespace

extern "C" int dcvc_dual_prior_encode_step(dcvc_tensor y, dcvc_tensor buf, dcvc_tensor sm, int k, dcvc_tensor yhat,
                                           const float *post_scale, int32_t *symbols, int16_t *indexes,
                                           float log_min, float log_step, void *stream) {
  const int C = y.C;
  if (!ok(y) || y.dtype != DCVC_F32 || !dp_ok(buf, sm, k, C) || !ok(yhat) || yhat.dtype != DCVC_F32 ||
      yhat.C != C || !symbols || !indexes || buf.H != y.H || buf.W != y.W || yhat.H != y.H || yhat.W != y.W)
    return DCVC_HIP_EINVAL;
  DP t{mk(y), mk(buf), mk(sm), mk(yhat), C, post_scale};
  hipLaunchKernelGGL(dp_encode_kernel, dim3(blocks_for((int64_t)y.H * y.W * (C / 2))), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), t, k, symbols, indexes, log_min, log_step);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_dual_prior_indexes_step(dcvc_tensor buf, dcvc_tensor sm, int k, int16_t *indexes,
                                            float log_min, float log_step, void *stream) {
  const int C = buf.C / 4;
  if (!dp_ok(buf, sm, k, C) || !indexes) return DCVC_HIP_EINVAL;
  DP t{};
  t.buf = mk(buf);
  t.sm = mk(sm);
  t.C = C;
  hipLaunchKernelGGL(dp_index_kernel, dim3(blocks_for((int64_t)buf.H * buf.W * (C / 2))), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), t, k, indexes, log_min, log_step);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_dual_prior_decode_step(dcvc_tensor buf, dcvc_tensor sm, int k, const int32_t *symbols,
                                           dcvc_tensor yhat, const float *post_scale, void *stream) {
  const int C = buf.C / 4;
  if (!dp_ok(buf, sm, k, C) || !symbols || !ok(yhat) || yhat.dtype != DCVC_F32 || yhat.C != C ||
      yhat.H != buf.H || yhat.W != buf.W)
    return DCVC_HIP_EINVAL;
  DP t{};
  t.buf = mk(buf);
  t.sm = mk(sm);
  t.yhat = mk(yhat);
  t.C = C;
  t.post = post_scale;
  hipLaunchKernelGGL(dp_decode_kernel, dim3(blocks_for((int64_t)buf.H * buf.W * (C / 2))), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), t, k, symbols);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_dual_prior_estimate_step(dcvc_tensor y, dcvc_tensor buf, dcvc_tensor sm, int k,
                                             dcvc_tensor yhat, const float *post_scale, float *bits, int gaussian,
                                             float scale_min, void *stream) {
  const int C = y.C;
  if (!ok(y) || y.dtype != DCVC_F32 || !dp_ok(buf, sm, k, C) || !ok(yhat) || yhat.dtype != DCVC_F32 ||
      yhat.C != C || !bits || buf.H != y.H || buf.W != y.W || yhat.H != y.H || yhat.W != y.W)
    return DCVC_HIP_EINVAL;
  DP t{mk(y), mk(buf), mk(sm), mk(yhat), C, post_scale};
  hipLaunchKernelGGL(dp_estimate_kernel, dim3(blocks_for((int64_t)y.H * y.W * (C / 2))), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), t, k, bits, gaussian ? 1 : 0, scale_min);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_nhwc_to_symbols_i32(dcvc_tensor x, int32_t *symbols, void *stream) {
  if (!ok(x) || !symbols) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)x.H * x.W * x.C);
  if (x.dtype == DCVC_F32)
    hipLaunchKernelGGL((to_sym32_kernel<float>), dim3(g), dim3(256), 0, st, mk(x), symbols);
  else
    hipLaunchKernelGGL((to_sym32_kernel<uint16_t>), dim3(g), dim3(256), 0, st, mk(x), symbols);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_symbols_i32_to_nhwc(const int32_t *symbols, dcvc_tensor y, void *stream) {
  if (!ok(y) || !symbols) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * y.C);
  if (y.dtype == DCVC_F32)
    hipLaunchKernelGGL((from_sym32_kernel<float>), dim3(g), dim3(256), 0, st, symbols, mk(y));
  else
    hipLaunchKernelGGL((from_sym32_kernel<uint16_t>), dim3(g), dim3(256), 0, st, symbols, mk(y));
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_se_scale(dcvc_tensor x, const float *w1, const float *w2, int reduced, float *work,
                             float *scale_out, void *stream) {
  if (!ok(x) || !w1 || !w2 || !work || !scale_out || reduced < 1 || reduced > 64 || x.C > 1024)
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int V = x.dtype == DCVC_F32 ? 4 : 8;
  if (vec_ok(x, V) && x.C / V <= 256) {
    if (x.dtype == DCVC_F32)
      hipLaunchKernelGGL((se_partial_kernel<float, 4>), dim3(kSePart), dim3(256), 0, st, mk(x), work);
    else
      hipLaunchKernelGGL((se_partial_kernel<uint16_t, 8>), dim3(kSePart), dim3(256), 0, st, mk(x), work);
  } else if (x.dtype == DCVC_F32) {
    hipLaunchKernelGGL((se_partial_scalar_kernel<float>), dim3(kSePart), dim3(128), 0, st, mk(x), work);
  } else {
    hipLaunchKernelGGL((se_partial_scalar_kernel<uint16_t>), dim3(kSePart), dim3(128), 0, st, mk(x), work);
  }
  DCVC_LAUNCH_CHECK();
  hipLaunchKernelGGL(se_fc_kernel, dim3(1), dim3(1024), 0, st, work, x.C, reduced,
                     1.f / (float)((int64_t)x.H * x.W), w1, w2, scale_out);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_se_apply(dcvc_tensor a, dcvc_tensor x, const float *scale, dcvc_tensor y, void *stream) {
  if (!ok(a) || !ok(x) || !ok(y) || !scale || a.dtype != x.dtype || y.dtype != x.dtype || a.C != y.C ||
      x.C != y.C || a.H != y.H || x.H != y.H || a.W != y.W || x.W != y.W)
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int V = y.dtype == DCVC_F32 ? 4 : 8;
  const bool vec = vec_ok(a, V) && vec_ok(x, V) && vec_ok(y, V);
  const unsigned g = blocks_for((int64_t)y.H * y.W * y.C / (vec ? V : 1));
#define LAUNCH(T, VV) \
  hipLaunchKernelGGL((se_apply_kernel<T, VV>), dim3(g), dim3(256), 0, st, mk(a), mk(x), scale, mk(y))
  if (y.dtype == DCVC_F32) {
    if (vec) LAUNCH(float, 4); else LAUNCH(float, 1);
  } else {
    if (vec) LAUNCH(uint16_t, 8); else LAUNCH(uint16_t, 1);
  }
#undef LAUNCH
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_channel_div(dcvc_tensor x, const float *q, dcvc_tensor y, void *stream) {
  if (!ok(x) || !ok(y) || !q || x.dtype != DCVC_F32 || y.dtype != DCVC_F32 || x.C != y.C || x.H != y.H ||
      x.W != y.W)
    return DCVC_HIP_EINVAL;
  hipLaunchKernelGGL(channel_div_kernel, dim3(blocks_for((int64_t)y.H * y.W * y.C)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), mk(x), q, mk(y));
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_fill(dcvc_tensor y, float value, void *stream) {
  if (!ok(y)) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * y.C);
  if (y.dtype == DCVC_F32)
    hipLaunchKernelGGL((fill_kernel<float>), dim3(g), dim3(256), 0, st, mk(y), value);
  else
    hipLaunchKernelGGL((fill_kernel<uint16_t>), dim3(g), dim3(256), 0, st, mk(y), value);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}
