// Depthwise conv, elementwise/copy/pad kernels and the quadtree-prior
// quantise / index / dequantise kernels.
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

#define DISPATCH2(tx, ty, KERNEL)                                        \
  do {                                                                   \
    if ((tx) == DCVC_F32 && (ty) == DCVC_F32) { KERNEL(float, float); }  \
    else if ((tx) == DCVC_F32) { KERNEL(float, uint16_t); }              \
    else if ((ty) == DCVC_F32) { KERNEL(uint16_t, float); }              \
    else { KERNEL(uint16_t, uint16_t); }                                 \
  } while (0)

inline unsigned blocks_for(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

// ------------------------------------------------------------ depthwise 3x3
template <typename TX, typename TY>
__global__ void dw_kernel(View x, View y, const float *w, const float *b) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * y.C) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  float acc = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = py + dy;
    if (yy < 0 || yy >= x.H) continue;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = px + dx;
      if (xx < 0 || xx >= x.W) continue;
      acc += w[((dy + 1) * 3 + dx + 1) * y.C + c] * ld<TX>(x.p, ((int64_t)yy * x.W + xx) * x.cs + x.co + c);
    }
  }
  st<TY>(y.p, pix * y.cs + y.co + c, acc + b[c]);
}

// 8 channels per thread, 16-byte loads/stores (C % 8 == 0, aligned views)
template <typename T> struct V8;
template <> struct V8<uint16_t> {
  __device__ __forceinline__ static void load(const void *b, int64_t e, float v[8]) {
    const u16x8 a = *reinterpret_cast<const u16x8 *>(reinterpret_cast<const uint16_t *>(b) + e);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
  }
  __device__ __forceinline__ static void store(void *b, int64_t e, const float v[8]) {
    u16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = f2bf(v[j]);
    *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(b) + e) = a;
  }
};
template <> struct V8<float> {
  __device__ __forceinline__ static void load(const void *b, int64_t e, float v[8]) {
    const float4 x = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(b) + e);
    const float4 y = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(b) + e + 4);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  }
  __device__ __forceinline__ static void store(void *b, int64_t e, const float v[8]) {
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(b) + e) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(b) + e + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <typename TX, typename TY>
__global__ void dw8_kernel(View x, View y, const float *w, const float *b) {
  // workgroup (x, y): 256 (pixel, 8-channel group) items of row y (32-bit
  // index math: no 64-bit divisions per thread)
  const unsigned cg = (unsigned)y.C >> 3;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (unsigned)y.W * cg) return;
  const int py = blockIdx.y, px = (int)(t / cg);
  const int c = (int)(t - (unsigned)px * cg) * 8;
  const int64_t pix = (int64_t)py * y.W + px;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = py + dy;
    if (yy < 0 || yy >= x.H) continue;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = px + dx;
      if (xx < 0 || xx >= x.W) continue;
      float v[8];
      V8<TX>::load(x.p, ((int64_t)yy * x.W + xx) * x.cs + x.co + c, v);
      const float *wt = w + ((dy + 1) * 3 + dx + 1) * y.C + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += wt[j] * v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] += b[c + j];
  V8<TY>::store(y.p, pix * y.cs + y.co + c, acc);
}

// fp32 maps with 4-channel-aligned views (Precision.split()): one thread per
// (4 channels, pixel column, 4 rows): the 6 x 3 input pieces of 4 outputs
// are loaded once (18 16-byte loads instead of 36) and the taps' weights once.
// Per output the same taps in the same order as dw8_kernel (out-of-image taps
// skipped), so identical bits.
constexpr int kDwRows = 4;
__global__ void __launch_bounds__(256) dw4r_kernel(View x, View y, const float *w, const float *b) {
  const unsigned cg = (unsigned)y.C >> 2;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (unsigned)y.W * cg) return;
  const int px = (int)(t / cg), c = (int)(t - (unsigned)px * cg) * 4;
  const int py0 = blockIdx.y * kDwRows;
  float4 wt[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wt[k] = *reinterpret_cast<const float4 *>(w + k * y.C + c);
  const float4 bb = *reinterpret_cast<const float4 *>(b + c);
  const float *xp = reinterpret_cast<const float *>(x.p) + x.co + c;
  float4 v[kDwRows + 2][3];
#pragma unroll
  for (int i = 0; i < kDwRows + 2; ++i) {
    const int yy = py0 - 1 + i;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int xx = px - 1 + dx;
      const bool in = yy >= 0 && yy < x.H && xx >= 0 && xx < x.W;
      v[i][dx] = in ? *reinterpret_cast<const float4 *>(xp + ((int64_t)yy * x.W + xx) * x.cs)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int r = 0; r < kDwRows; ++r) {
    const int py = py0 + r;
    if (py >= y.H) break;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = py + dy;
      if (yy < 0 || yy >= x.H) continue;
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int xx = px + dx;
        if (xx < 0 || xx >= x.W) continue;
        const float4 q = v[r + dy + 1][dx + 1], ww = wt[(dy + 1) * 3 + dx + 1];
        acc.x += ww.x * q.x;
        acc.y += ww.y * q.y;
        acc.z += ww.z * q.z;
        acc.w += ww.w * q.w;
      }
    }
    acc.x += bb.x;
    acc.y += bb.y;
    acc.z += bb.z;
    acc.w += bb.w;
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(y.p) + ((int64_t)py * y.W + px) * y.cs + y.co + c) = acc;
  }
}

// ------------------------------------------------------------ elementwise
template <typename TA, typename TY>
__global__ void add_kernel(View a, View b, int b32, View y) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * y.C) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  const float va = ld<TA>(a.p, pix * a.cs + a.co + c);
  const float vb = b32 ? ld<float>(b.p, pix * b.cs + b.co + c) : ld<uint16_t>(b.p, pix * b.cs + b.co + c);
  st<TY>(y.p, pix * y.cs + y.co + c, va + vb);
}

template <typename TX, typename TY>
__global__ void copy_kernel(View x, View y) {
  // replicate-pad / crop / dtype convert: y(py, px) = x(min(py, H-1), min(px, W-1))
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * y.C) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  const int sy = min(py, x.H - 1), sx = min(px, x.W - 1);
  st<TY>(y.p, pix * y.cs + y.co + c, ld<TX>(x.p, ((int64_t)sy * x.W + sx) * x.cs + x.co + c));
}

// copy_kernel with 8 channels per thread (16/32-byte loads and stores) when
// every channel count, stride and offset is a multiple of 8: the concat
// copies of the contexts into the contextual encoder / recon inputs.
template <typename TX, typename TY>
__global__ void copy8_kernel(View x, View y) {
  const int cg = y.C >> 3;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * cg) return;
  const int c = (int)(idx % cg) * 8;
  const int64_t pix = idx / cg;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  const int sy = min(py, x.H - 1), sx = min(px, x.W - 1);
  float v[8];
  V8<TX>::load(x.p, ((int64_t)sy * x.W + sx) * x.cs + x.co + c, v);
  V8<TY>::store(y.p, pix * y.cs + y.co + c, v);
}

template <typename TY>
__global__ void frame_kernel(const uint8_t *src, int h, int w, int zero_pad, View y) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.H * y.W * 3) return;
  const int c = (int)(idx % 3);
  const int64_t pix = idx / 3;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  const int sy = min(py, h - 1), sx = min(px, w - 1);
  float v = (float)src[((int64_t)c * h + sy) * w + sx] / 255.f;
  if (zero_pad && (py >= h || px >= w)) v = 0.f;
  st<TY>(y.p, pix * y.cs + y.co + c, v);
}

// ------------------------------------------------------------ quadtree prior
// Step k processes, for each pixel with parity m = 2*(y&1) + (x&1), the
// channel quarter q with STEP_MASK[k][q] == m (common_model.py:168-220).
// STEP_MASK = {{0,1,2,3},{3,2,1,0},{2,3,0,1},{1,0,3,2}} is q -> q ^ {0,3,2,1}[k],
// an involution, so the quarter of mask m at step k is m ^ {0,3,2,1}[k].
__device__ __forceinline__ int quarter_of(int k, int m) {
  return m ^ ((0x1230 >> (k << 2)) & 3);
}

__device__ __forceinline__ int16_t scale_index(float s, float log_min, float log_step) {
  // GaussianEncoder.build_indexes (entropy_models.py:269-273)
  s = fmaxf(s, 1e-5f);
  float v = (logf(s) - log_min) / log_step;
  v = fminf(fmaxf(v, 0.f), 255.f);
  return (int16_t)(int)v;
}

struct QT {
  View y, params, sm, yhs, yhat;
  int has_sm;
  int C;  // latent channels
};

__device__ __forceinline__ void step_scales_means(const QT &t, int64_t pix, int q, int cc, float &sc,
                                                  float &me) {
  const int C4 = t.C / 4;
  if (t.has_sm) {
    sc = ld<float>(t.sm.p, pix * t.sm.cs + t.sm.co + q * C4 + cc);
    me = ld<float>(t.sm.p, pix * t.sm.cs + t.sm.co + t.C + q * C4 + cc);
  } else {
    sc = ld<float>(t.params.p, pix * t.params.cs + t.params.co + t.C + q * C4 + cc);
    me = ld<float>(t.params.p, pix * t.params.cs + t.params.co + 2 * t.C + q * C4 + cc);
  }
}

// one thread per (channel-in-quarter cc, pixel): NCHW order of y_q_w_k
__global__ void qt_encode_kernel(QT t, int k, int16_t *sym, int16_t *idx, float log_min,
                                 float log_step) {
  const int C4 = t.C / 4;
  const int64_t HW = (int64_t)t.y.H * t.y.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C4) return;
  const int cc = (int)(i / HW);
  const int64_t pix = i - (int64_t)cc * HW;
  const int py = (int)(pix / t.y.W), px = (int)(pix - (int64_t)py * t.y.W);
  const int m = ((py & 1) << 1) | (px & 1);
  const int q = quarter_of(k, m);
  const int ch = q * C4 + cc;
  float qs = ld<float>(t.params.p, pix * t.params.cs + t.params.co + ch);
  qs = fmaxf(qs, 0.5f);                                  // clamp_min(quant_step, 0.5)
  const float yv = ld<float>(t.y.p, pix * t.y.cs + t.y.co + ch) / qs;
  float sc, me;
  step_scales_means(t, pix, q, cc, sc, me);
  const float yres = yv - me;                            // (y - means*1) * 1
  const float yq = rintf(yres);
  const float yh = yq + me;
  const float cl = fminf(fmaxf(yq, -30000.f), 30000.f);
  sym[i] = (int16_t)(int)cl;
  idx[i] = scale_index(sc, log_min, log_step);
  st<float>(t.yhs.p, pix * t.yhs.cs + t.yhs.co + ch, yh);
  st<float>(t.yhat.p, pix * t.yhat.cs + t.yhat.co + ch, yh * qs);
}

// ---- estimate mode (forward_four_part_prior + get_y_*_bits,
// common_model.py:39-58): y_q and its step's scale give the element's bits;
// the same quantise / y_hat outputs as qt_encode_kernel.
__device__ __forceinline__ float probs_to_bits(float p) {
  // -1.0 * log(p + 1e-5) / log(2.0), clamp_min 0 (common_model.py:39-43)
  const float b = -1.f * logf(p + 1e-5f) / 0.6931471805599453f;
  return b > 0.f ? b : 0.f;
}
__device__ __forceinline__ float dist_cdf(int gaussian, float v, float s) {
  if (gaussian) return 0.5f * (1.f + erff(v * (1.f / s) / 1.4142135623730951f));  // Normal(0, s).cdf
  const float sg = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
  return 0.5f - 0.5f * sg * expm1f(-fabsf(v) / s);                                  // Laplace(0, s).cdf
}

__global__ void qt_estimate_kernel(QT t, int k, float *bits, int gaussian) {
  const int C4 = t.C / 4;
  const int64_t HW = (int64_t)t.y.H * t.y.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C4) return;
  const int cc = (int)(i / HW);
  const int64_t pix = i - (int64_t)cc * HW;
  const int py = (int)(pix / t.y.W), px = (int)(pix - (int64_t)py * t.y.W);
  const int q = quarter_of(k, ((py & 1) << 1) | (px & 1));
  const int ch = q * C4 + cc;
  float qs = ld<float>(t.params.p, pix * t.params.cs + t.params.co + ch);
  qs = fmaxf(qs, 0.5f);
  const float yv = ld<float>(t.y.p, pix * t.y.cs + t.y.co + ch) / qs;
  float sc, me;
  step_scales_means(t, pix, q, cc, sc, me);
  const float yq = rintf(yv - me);
  const float yh = yq + me;
  const float s = fminf(fmaxf(sc, 1e-5f), 1e10f);       // sigma.clamp(1e-5, 1e10)
  bits[i] = probs_to_bits(dist_cdf(gaussian, yq + 0.5f, s) - dist_cdf(gaussian, yq - 0.5f, s));
  st<float>(t.yhs.p, pix * t.yhs.cs + t.yhs.co + ch, yh);
  st<float>(t.yhat.p, pix * t.yhat.cs + t.yhat.co + ch, yh * qs);
}

// BitEstimator.get_cdf (entropy_models.py:56-122) at z +- 0.5 -> bits;
// tab[c][11] = softplus(h1), b1, tanh(a1), ..., softplus(h4), b4
__device__ __forceinline__ float factorized_cdf(const float *t, float x) {
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    x = x * t[3 * l] + t[3 * l + 1];
    x = x + tanhf(x) * t[3 * l + 2];
  }
  x = x * t[9] + t[10];
  return 1.f / (1.f + expf(-x));
}

__global__ void factorized_bits_kernel(View z, const float *tab, float *bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)z.H * z.W * z.C) return;
  const int c = (int)(i % z.C);
  const int64_t pix = i / z.C;
  const float v = ld<float>(z.p, pix * z.cs + z.co + c);
  const float *t = tab + c * 11;
  bits[i] = probs_to_bits(factorized_cdf(t, v + 0.5f) - factorized_cdf(t, v - 0.5f));
}

// deterministic sum of n floats: one 1024-thread block, fixed strides and
// a fixed tree, so the total is reproducible run to run
__global__ void __launch_bounds__(1024) sum_kernel(const float *x, int64_t n, float *out) {
  __shared__ float part[1024];
  float a = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) a += x[i];
  part[threadIdx.x] = a;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = part[0];
}

__global__ void qt_index_kernel(QT t, int k, int16_t *idx, float log_min, float log_step) {
  const int C4 = t.C / 4;
  const int64_t HW = (int64_t)t.params.H * t.params.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C4) return;
  const int cc = (int)(i / HW);
  const int64_t pix = i - (int64_t)cc * HW;
  const int py = (int)(pix / t.params.W), px = (int)(pix - (int64_t)py * t.params.W);
  const int q = quarter_of(k, ((py & 1) << 1) | (px & 1));
  float sc, me;
  step_scales_means(t, pix, q, cc, sc, me);
  idx[i] = scale_index(sc, log_min, log_step);
}

__global__ void qt_decode_kernel(QT t, int k, const int16_t *sym) {
  const int C4 = t.C / 4;
  const int64_t HW = (int64_t)t.params.H * t.params.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * C4) return;
  const int cc = (int)(i / HW);
  const int64_t pix = i - (int64_t)cc * HW;
  const int py = (int)(pix / t.params.W), px = (int)(pix - (int64_t)py * t.params.W);
  const int q = quarter_of(k, ((py & 1) << 1) | (px & 1));
  const int ch = q * C4 + cc;
  float sc, me;
  step_scales_means(t, pix, q, cc, sc, me);
  float qs = ld<float>(t.params.p, pix * t.params.cs + t.params.co + ch);
  qs = fmaxf(qs, 0.5f);
  const float yh = ((float)sym[i] + me);                 // (y_q_r + means) * 1
  st<float>(t.yhs.p, pix * t.yhs.cs + t.yhs.co + ch, yh);
  st<float>(t.yhat.p, pix * t.yhat.cs + t.yhat.co + ch, yh * qs);
}

template <typename TX>
__global__ void to_sym_kernel(View x, int16_t *sym) {
  const int64_t HW = (int64_t)x.H * x.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * x.C) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  const float v = fminf(fmaxf(ld<TX>(x.p, pix * x.cs + x.co + c), -30000.f), 30000.f);
  sym[i] = (int16_t)(int)v;
}

template <typename TY>
__global__ void from_sym_kernel(const int16_t *sym, View y) {
  const int64_t HW = (int64_t)y.H * y.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW * y.C) return;
  const int c = (int)(i / HW);
  const int64_t pix = i - (int64_t)c * HW;
  st<TY>(y.p, pix * y.cs + y.co + c, (float)sym[i]);
}

bool qt_ok(const dcvc_tensor &params, const dcvc_tensor &sm, int C) {
  if (!ok(params) || params.dtype != DCVC_F32 || params.C != 3 * C || (C % 4)) return false;
  if (sm.ptr && (!ok(sm) || sm.dtype != DCVC_F32 || sm.C != 2 * C || sm.H != params.H || sm.W != params.W))
    return false;
  return true;
}

}  // namespace

extern "C" int dcvc_dwconv3x3(dcvc_tensor x, dcvc_tensor y, const float *w, const float *bias,
                              void *stream) {
  if (!ok(x) || !ok(y) || !w || !bias || x.C != y.C || x.H != y.H || x.W != y.W) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec = (x.C % 8 == 0) && (x.cstride % 8 == 0) && (x.coff % 8 == 0) && (y.cstride % 8 == 0) &&
                   (y.coff % 8 == 0);
  if (x.dtype == DCVC_F32 && y.dtype == DCVC_F32 && x.C % 4 == 0 && x.cstride % 4 == 0 && x.coff % 4 == 0 &&
      y.cstride % 4 == 0 && y.coff % 4 == 0 && ((uintptr_t)x.ptr & 15) == 0 && ((uintptr_t)y.ptr & 15) == 0 &&
      ((uintptr_t)w & 15) == 0 && ((uintptr_t)bias & 15) == 0) {
    const dim3 g(blocks_for((int64_t)y.W * (y.C / 4)), (unsigned)((y.H + kDwRows - 1) / kDwRows));
    hipLaunchKernelGGL(dw4r_kernel, g, dim3(256), 0, st, mk(x), mk(y), w, bias);
    DCVC_LAUNCH_CHECK();
    return DCVC_HIP_OK;
  }
  if (vec) {
    const dim3 g(blocks_for((int64_t)y.W * (y.C / 8)), (unsigned)y.H);
#define K(TX, TY) hipLaunchKernelGGL((dw8_kernel<TX, TY>), g, dim3(256), 0, st, mk(x), mk(y), w, bias)
    DISPATCH2(x.dtype, y.dtype, K);
#undef K
  } else {
    const unsigned g = blocks_for((int64_t)y.H * y.W * y.C);
#define K(TX, TY) hipLaunchKernelGGL((dw_kernel<TX, TY>), dim3(g), dim3(256), 0, st, mk(x), mk(y), w, bias)
    DISPATCH2(x.dtype, y.dtype, K);
#undef K
  }
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_add(dcvc_tensor a, dcvc_tensor b, dcvc_tensor y, void *stream) {
  if (!ok(a) || !ok(b) || !ok(y) || a.C != y.C || b.C != y.C || a.H != y.H || b.H != y.H ||
      a.W != y.W || b.W != y.W)
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * y.C);
  const int b32 = b.dtype == DCVC_F32;
#define K(TX, TY) hipLaunchKernelGGL((add_kernel<TX, TY>), dim3(g), dim3(256), 0, st, mk(a), mk(b), b32, mk(y))
  DISPATCH2(a.dtype, y.dtype, K);
#undef K
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

static int copy_impl(dcvc_tensor x, dcvc_tensor y, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (x.C % 8 == 0 && x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 8 == 0 && y.coff % 8 == 0 &&
      ((uintptr_t)x.ptr & 15) == 0 && ((uintptr_t)y.ptr & 15) == 0) {
    const unsigned g8 = blocks_for((int64_t)y.H * y.W * (y.C / 8));
#define K(TX, TY) hipLaunchKernelGGL((copy8_kernel<TX, TY>), dim3(g8), dim3(256), 0, st, mk(x), mk(y))
    DISPATCH2(x.dtype, y.dtype, K);
#undef K
    DCVC_LAUNCH_CHECK();
    return DCVC_HIP_OK;
  }
  const unsigned g = blocks_for((int64_t)y.H * y.W * y.C);
#define K(TX, TY) hipLaunchKernelGGL((copy_kernel<TX, TY>), dim3(g), dim3(256), 0, st, mk(x), mk(y))
  DISPATCH2(x.dtype, y.dtype, K);
#undef K
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_copy(dcvc_tensor x, dcvc_tensor y, void *stream) {
  if (!ok(x) || !ok(y) || x.C != y.C || x.H != y.H || x.W != y.W) return DCVC_HIP_EINVAL;
  return copy_impl(x, y, stream);
}

extern "C" int dcvc_pad_replicate(dcvc_tensor x, dcvc_tensor y, void *stream) {
  if (!ok(x) || !ok(y) || x.C != y.C) return DCVC_HIP_EINVAL;
  return copy_impl(x, y, stream);
}

static int frame_impl(const uint8_t *src, int h, int w, int zero_pad, dcvc_tensor y, void *stream) {
  if (!src || !ok(y) || y.C != 3 || h <= 0 || w <= 0 || y.H < h || y.W < w) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * 3);
  if (y.dtype == DCVC_F32)
    hipLaunchKernelGGL((frame_kernel<float>), dim3(g), dim3(256), 0, st, src, h, w, zero_pad, mk(y));
  else
    hipLaunchKernelGGL((frame_kernel<uint16_t>), dim3(g), dim3(256), 0, st, src, h, w, zero_pad, mk(y));
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_frame_to_nhwc(const uint8_t *src, int h, int w, dcvc_tensor y, void *stream) {
  return frame_impl(src, h, w, 0, y, stream);
}

extern "C" int dcvc_frame_to_nhwc_zero_pad(const uint8_t *src, int h, int w, dcvc_tensor y, void *stream) {
  return frame_impl(src, h, w, 1, y, stream);
}

extern "C" int dcvc_quadtree_encode_step(dcvc_tensor y, dcvc_tensor params, dcvc_tensor sm, int k,
                                         dcvc_tensor yhs, dcvc_tensor yhat, int16_t *symbols,
                                         int16_t *indexes, float log_min, float log_step,
                                         void *stream) {
  const int C = y.C;
  if (!ok(y) || y.dtype != DCVC_F32 || !qt_ok(params, sm, C) || k < 0 || k > 3) return DCVC_HIP_EINVAL;
  if ((k == 0) != (sm.ptr == nullptr)) return DCVC_HIP_EINVAL;
  if (!ok(yhs) || !ok(yhat) || yhs.dtype != DCVC_F32 || yhat.dtype != DCVC_F32 || yhs.C != C ||
      yhat.C != C || !symbols || !indexes)
    return DCVC_HIP_EINVAL;
  if (params.H != y.H || params.W != y.W || yhs.H != y.H || yhat.H != y.H || yhs.W != y.W || yhat.W != y.W)
    return DCVC_HIP_EINVAL;
  QT t{mk(y), mk(params), mk(sm), mk(yhs), mk(yhat), sm.ptr != nullptr, C};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * (C / 4));
  hipLaunchKernelGGL(qt_encode_kernel, dim3(g), dim3(256), 0, st, t, k, symbols, indexes, log_min, log_step);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_quadtree_indexes_step(dcvc_tensor params, dcvc_tensor sm, int k, int16_t *indexes,
                                          float log_min, float log_step, void *stream) {
  const int C = params.C / 3;
  if (!qt_ok(params, sm, C) || k < 0 || k > 3 || !indexes) return DCVC_HIP_EINVAL;
  if ((k == 0) != (sm.ptr == nullptr)) return DCVC_HIP_EINVAL;
  QT t{};
  t.params = mk(params);
  t.sm = mk(sm);
  t.has_sm = sm.ptr != nullptr;
  t.C = C;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)params.H * params.W * (C / 4));
  hipLaunchKernelGGL(qt_index_kernel, dim3(g), dim3(256), 0, st, t, k, indexes, log_min, log_step);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_quadtree_decode_step(dcvc_tensor params, dcvc_tensor sm, int k, const int16_t *symbols,
                                         dcvc_tensor yhs, dcvc_tensor yhat, void *stream) {
  const int C = params.C / 3;
  if (!qt_ok(params, sm, C) || k < 0 || k > 3 || !symbols) return DCVC_HIP_EINVAL;
  if ((k == 0) != (sm.ptr == nullptr)) return DCVC_HIP_EINVAL;
  if (!ok(yhs) || !ok(yhat) || yhs.dtype != DCVC_F32 || yhat.dtype != DCVC_F32 || yhs.C != C || yhat.C != C)
    return DCVC_HIP_EINVAL;
  QT t{};
  t.params = mk(params);
  t.sm = mk(sm);
  t.yhs = mk(yhs);
  t.yhat = mk(yhat);
  t.has_sm = sm.ptr != nullptr;
  t.C = C;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)params.H * params.W * (C / 4));
  hipLaunchKernelGGL(qt_decode_kernel, dim3(g), dim3(256), 0, st, t, k, symbols);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_nhwc_to_symbols(dcvc_tensor x, int16_t *symbols, void *stream) {
  if (!ok(x) || !symbols) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)x.H * x.W * x.C);
  if (x.dtype == DCVC_F32)
    hipLaunchKernelGGL((to_sym_kernel<float>), dim3(g), dim3(256), 0, st, mk(x), symbols);
  else
    hipLaunchKernelGGL((to_sym_kernel<uint16_t>), dim3(g), dim3(256), 0, st, mk(x), symbols);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_symbols_to_nhwc(const int16_t *symbols, dcvc_tensor y, void *stream) {
  if (!ok(y) || !symbols) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * y.C);
  if (y.dtype == DCVC_F32)
    hipLaunchKernelGGL((from_sym_kernel<float>), dim3(g), dim3(256), 0, st, symbols, mk(y));
  else
    hipLaunchKernelGGL((from_sym_kernel<uint16_t>), dim3(g), dim3(256), 0, st, symbols, mk(y));
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_quadtree_estimate_step(dcvc_tensor y, dcvc_tensor params, dcvc_tensor sm, int k,
                                           dcvc_tensor yhs, dcvc_tensor yhat, float *bits, int gaussian,
                                           void *stream) {
  const int C = y.C;
  if (!ok(y) || y.dtype != DCVC_F32 || !qt_ok(params, sm, C) || k < 0 || k > 3) return DCVC_HIP_EINVAL;
  if ((k == 0) != (sm.ptr == nullptr)) return DCVC_HIP_EINVAL;
  if (!ok(yhs) || !ok(yhat) || yhs.dtype != DCVC_F32 || yhat.dtype != DCVC_F32 || yhs.C != C ||
      yhat.C != C || !bits)
    return DCVC_HIP_EINVAL;
  if (params.H != y.H || params.W != y.W || yhs.H != y.H || yhat.H != y.H || yhs.W != y.W || yhat.W != y.W)
    return DCVC_HIP_EINVAL;
  QT t{mk(y), mk(params), mk(sm), mk(yhs), mk(yhat), sm.ptr != nullptr, C};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = blocks_for((int64_t)y.H * y.W * (C / 4));
  hipLaunchKernelGGL(qt_estimate_kernel, dim3(g), dim3(256), 0, st, t, k, bits, gaussian ? 1 : 0);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_factorized_bits(dcvc_tensor z, const float *table, float *bits, void *stream) {
  if (!ok(z) || z.dtype != DCVC_F32 || !table || !bits) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(factorized_bits_kernel, dim3(blocks_for((int64_t)z.H * z.W * z.C)), dim3(256), 0, st, mk(z),
                     table, bits);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_sum_f32(const float *x, int64_t n, float *out, void *stream) {
  if (!x || !out || n < 0) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, st, x, n, out);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// ------------------------------------------------------------ debug aid
// Fill the LDS of as many workgroups as fit on the chip with all-ones bytes
// (bf16 / fp32 NaN).  LDS is not cleared between dispatches, so a kernel
// launched next that reads LDS it never wrote sees NaN instead of whatever an
// earlier kernel left there (scripts/lds_poison_check.py).
__global__ void __launch_bounds__(256) lds_poison_kernel(int words) {
  extern __shared__ uint32_t lds_words[];
  for (int i = threadIdx.x; i < words; i += 256) lds_words[i] = 0xFFFFFFFFu;
  __syncthreads();
}

extern "C" int dcvc_debug_poison_lds(int bytes, int blocks, void *stream) {
  if (bytes <= 0 || bytes > 160 * 1024 || blocks <= 0) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dcvc_ensure_lds(reinterpret_cast<const void *>(lds_poison_kernel), bytes);
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(256), bytes, st, bytes / 4);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// Fill the VGPRs of as many waves as fit (8 per SIMD at 128 VGPRs each) with
// all-ones bits: a kernel launched next that reads a register it never wrote
// sees NaN (scripts/lds_poison_check.py --vgpr).
__global__ void __launch_bounds__(256) vgpr_poison_kernel(int *sink) {
#define P4(a) "v_mov_b32 v" #a "0, -1\n v_mov_b32 v" #a "1, -1\n v_mov_b32 v" #a "2, -1\n v_mov_b32 v" #a "3, -1\n" \
              "v_mov_b32 v" #a "4, -1\n v_mov_b32 v" #a "5, -1\n v_mov_b32 v" #a "6, -1\n v_mov_b32 v" #a "7, -1\n" \
              "v_mov_b32 v" #a "8, -1\n v_mov_b32 v" #a "9, -1\n"
  asm volatile(P4(1) P4(2) P4(3) P4(4) P4(5) P4(6) P4(7) P4(8) P4(9) P4(10) P4(11) ::
                   : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22",
                     "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35",
                     "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",
                     "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61",
                     "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74",
                     "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87",
                     "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100",
                     "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111",
                     "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119");
#undef P4
  if (threadIdx.x == 1024) *sink = 0;  // never true: keeps the kernel from being empty
}

extern "C" int dcvc_debug_poison_vgpr(int blocks, void *stream) {
  if (blocks <= 0) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(vgpr_poison_kernel, dim3(blocks), dim3(256), 0, st, nullptr);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}
