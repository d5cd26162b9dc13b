// Gather / resampling kernels: bilinear flow warp (grid_sample border,
// align_corners=True), the fused OffsetDiversity warp+fusion, bilinear x2
// resize (align_corners=False) and 2x2 pooling.
//
// The float arithmetic follows the PyTorch CPU kernels the reference runs on
// (unnormalize as (g + 1) * ((size - 1) / 2), clip, floor-based bilinear
// weights, corner sum nw + ne + sw + se; separable resize as
// (x00*w0 + x01*w1)*h0 + (x10*w0 + x11*w1)*h1; avg pool as a running sum / 4)
// with FMA contraction disabled, so the f32 path can match the CPU oracle
// element for element.
#include "common.h"

#pragma clang fp contract(off)

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

struct Bilin {
  int x0, x1, y0, y1;
  float nw, ne, sw, se;
};

// grid_sample(bilinear, border, align_corners=True) sample position for
// pixel (x, y) displaced by (fx, fy) pixels (video_net.py:22-33).
__device__ __forceinline__ Bilin warp_coords(float gxv, float gyv, float fx, float fy, int W, int H) {
  const float fxn = fx / (float)((W - 1.0) / 2.0);
  const float fyn = fy / (float)((H - 1.0) / 2.0);
  const float grid_x = gxv + fxn;
  const float grid_y = gyv + fyn;
  float ix = (grid_x + 1.f) * ((float)(W - 1) / 2.f);
  float iy = (grid_y + 1.f) * ((float)(H - 1) / 2.f);
  ix = fminf((float)(W - 1), fmaxf(ix, 0.f));
  iy = fminf((float)(H - 1), fmaxf(iy, 0.f));
  const float xw = floorf(ix), yn = floorf(iy);
  const float w = ix - xw, e = 1.f - w, n = iy - yn, s = 1.f - n;
  Bilin b;
  b.x0 = (int)xw;
  b.y0 = (int)yn;
  b.x1 = min(b.x0 + 1, W - 1);
  b.y1 = min(b.y0 + 1, H - 1);
  b.nw = s * e;
  b.ne = s * w;
  b.sw = n * e;
  b.se = n * w;
  return b;
}

template <typename T>
__device__ __forceinline__ float sample(const View &x, const Bilin &b, int c) {
  const int64_t r0 = (int64_t)b.y0 * x.W, r1 = (int64_t)b.y1 * x.W;
  const float vnw = ld<T>(x.p, (r0 + b.x0) * x.cs + x.co + c);
  const float vne = ld<T>(x.p, (r0 + b.x1) * x.cs + x.co + c);
  const float vsw = ld<T>(x.p, (r1 + b.x0) * x.cs + x.co + c);
  const float vse = ld<T>(x.p, (r1 + b.x1) * x.cs + x.co + c);
  return vnw * b.nw + vne * b.ne + vsw * b.sw + vse * b.se;
}

template <typename TX, typename TY>
__global__ void warp_kernel(View x, View f, View y, const float *gx, const float *gy) {
  const int64_t pix = (int64_t)blockIdx.x * blockDim.y + threadIdx.y;
  if (pix >= (int64_t)y.H * y.W) return;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  const float fx = ld<float>(f.p, pix * f.cs + f.co);
  const float fy = ld<float>(f.p, pix * f.cs + f.co + 1);
  const Bilin b = warp_coords(gx[px], gy[py], fx, fy, x.W, x.H);
  for (int c = threadIdx.x; c < y.C; c += blockDim.x)
    st<TY>(y.p, pix * y.cs + y.co + c, sample<TX>(x, b, c));
}

// Workgroups are dealt to the 8 XCDs round robin; with a grid padded to a
// multiple of 8, this bijection gives each XCD one contiguous band of the
// frame, so the bilinear gathers of neighbouring pixels share that XCD's L2.
__device__ __forceinline__ int64_t xcd_band(unsigned b, unsigned nb) {
  return (int64_t)(b & 7u) * (nb >> 3) + (b >> 3);
}

// Vector form for bf16 maps with 8-channel-aligned views: one thread per
// (pixel, 8 channels), 16-byte corner loads and one 16-byte store instead of
// 32 two-byte loads (the scalar kernel is load-instruction bound).  Same
// per-channel arithmetic, so results are identical.
__global__ void warp8_kernel(View x, View f, View y, const float *gx, const float *gy) {
  const int q8 = y.C >> 3;
  const int64_t t = xcd_band(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int64_t pix = t / q8;
  if (pix >= (int64_t)y.H * y.W) return;
  const int c = (int)(t - pix * q8) * 8;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  const float2 fv = *reinterpret_cast<const float2 *>(reinterpret_cast<const float *>(f.p) + pix * f.cs + f.co);
  const Bilin b = warp_coords(gx[px], gy[py], fv.x, fv.y, x.W, x.H);
  const uint16_t *xp = reinterpret_cast<const uint16_t *>(x.p) + x.co + c;
  const int64_t r0 = (int64_t)b.y0 * x.W, r1 = (int64_t)b.y1 * x.W;
  const u16x8 a = *reinterpret_cast<const u16x8 *>(xp + (r0 + b.x0) * x.cs);
  const u16x8 bb = *reinterpret_cast<const u16x8 *>(xp + (r0 + b.x1) * x.cs);
  const u16x8 cc = *reinterpret_cast<const u16x8 *>(xp + (r1 + b.x0) * x.cs);
  const u16x8 d = *reinterpret_cast<const u16x8 *>(xp + (r1 + b.x1) * x.cs);
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    o[j] = f2bf(bf2f(a[j]) * b.nw + bf2f(bb[j]) * b.ne + bf2f(cc[j]) * b.sw + bf2f(d[j]) * b.se);
  *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(y.p) + pix * y.cs + y.co + c) = o;
}

// The same for fp32 maps with 4-channel-aligned views: one thread per
// (pixel, 4 channels), 16-byte corner loads and one 16-byte store (Precision.
// split() keeps every feature map in fp32).  Same per-channel arithmetic.
__global__ void __launch_bounds__(256) warp4_kernel(View x, View f, View y, const float *gx, const float *gy) {
  const int q4 = y.C >> 2;
  const int64_t t = xcd_band(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int64_t pix = t / q4;
  if (pix >= (int64_t)y.H * y.W) return;
  const int c = (int)(t - pix * q4) * 4;
  const int py = (int)(pix / y.W), px = (int)(pix - (int64_t)py * y.W);
  const float2 fv = *reinterpret_cast<const float2 *>(reinterpret_cast<const float *>(f.p) + pix * f.cs + f.co);
  const Bilin b = warp_coords(gx[px], gy[py], fv.x, fv.y, x.W, x.H);
  const float *xp = reinterpret_cast<const float *>(x.p) + x.co + c;
  const int64_t r0 = (int64_t)b.y0 * x.W, r1 = (int64_t)b.y1 * x.W;
  const float4 a = *reinterpret_cast<const float4 *>(xp + (r0 + b.x0) * x.cs);
  const float4 bb = *reinterpret_cast<const float4 *>(xp + (r0 + b.x1) * x.cs);
  const float4 cc = *reinterpret_cast<const float4 *>(xp + (r1 + b.x0) * x.cs);
  const float4 d = *reinterpret_cast<const float4 *>(xp + (r1 + b.x1) * x.cs);
  float4 o;
  o.x = a.x * b.nw + bb.x * b.ne + cc.x * b.sw + d.x * b.se;
  o.y = a.y * b.nw + bb.y * b.ne + cc.y * b.sw + d.y * b.se;
  o.z = a.z * b.nw + bb.z * b.ne + cc.z * b.sw + d.z * b.se;
  o.w = a.w * b.nw + bb.w * b.ne + cc.w * b.sw + d.w * b.se;
  *reinterpret_cast<float4 *>(reinterpret_cast<float *>(y.p) + pix * y.cs + y.co + c) = o;
}

// bilinear x2 upsample value of channel c at full-res pixel (oy, ox) from a
// half-res map (align_corners=False, UpSampleKernel.cpp cpu_upsample_linear)
template <typename T>
__device__ __forceinline__ float up2_at(const View &m, int oy, int ox, int c) {
  float sy = 0.5f * ((float)oy + 0.5f) - 0.5f;
  float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
  sy = sy < 0.f ? 0.f : sy;
  sx = sx < 0.f ? 0.f : sx;
  const int h0 = (int)sy, w0 = (int)sx;
  const int h1 = h0 + (h0 < m.H - 1 ? 1 : 0), w1 = w0 + (w0 < m.W - 1 ? 1 : 0);
  const float hl1 = sy - (float)h0, hl0 = 1.f - hl1;
  const float wl1 = sx - (float)w0, wl0 = 1.f - wl1;
  const float a = ld<T>(m.p, ((int64_t)h0 * m.W + w0) * m.cs + m.co + c);
  const float b = ld<T>(m.p, ((int64_t)h0 * m.W + w1) * m.cs + m.co + c);
  const float cc = ld<T>(m.p, ((int64_t)h1 * m.W + w0) * m.cs + m.co + c);
  const float d = ld<T>(m.p, ((int64_t)h1 * m.W + w1) * m.cs + m.co + c);
  return (a * wl0 + b * wl1) * hl0 + (cc * wl0 + d * wl1) * hl1;
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + expf(-v)); }

// OffsetDiversity (video_model.py:43-63), one thread per (pixel, group g):
// warps i = 2g, 2g+1 feed fusion group g (output channels 3g..3g+2).
// Three consecutive bf16 channels c0..c0+2 at the four corners with ONE
// 8-byte load per corner: the dword-aligned 4-channel window starting at c0
// (ODD == 0) or c0 - 1 (ODD == 1) holds all three.  The kernel is bound by
// vector-memory instruction issue on these gathers (SQ_WAIT_INST_ANY 0.75 of
// wave cycles, profiles/r01_*), not by bytes.  ODD = parity of the element
// index of c0 (uniform per call site); the interpolation order is sample()'s.
struct __attribute__((aligned(4))) u32x2a4 { uint32_t lo, hi; };

template <int ODD>
__device__ __forceinline__ void sample3_bf16(const View &x, const Bilin &b, int c0, float v[3]) {
  const uint16_t *base = reinterpret_cast<const uint16_t *>(x.p) + x.co + c0 - ODD;
  const int64_t r0 = (int64_t)b.y0 * x.W, r1 = (int64_t)b.y1 * x.W;
  const int64_t e[4] = {(r0 + b.x0) * x.cs, (r0 + b.x1) * x.cs, (r1 + b.x0) * x.cs, (r1 + b.x1) * x.cs};
  float q[4][3];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32x2a4 w = *reinterpret_cast<const u32x2a4 *>(base + e[k]);
    if constexpr (ODD == 0) {
      q[k][0] = bf2f((uint16_t)(w.lo & 0xffffu));
      q[k][1] = bf2f((uint16_t)(w.lo >> 16));
      q[k][2] = bf2f((uint16_t)(w.hi & 0xffffu));
    } else {
      q[k][0] = bf2f((uint16_t)(w.lo >> 16));
      q[k][1] = bf2f((uint16_t)(w.hi & 0xffffu));
      q[k][2] = bf2f((uint16_t)(w.hi >> 16));
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = q[0][c] * b.nw + q[1][c] * b.ne + q[2][c] * b.sw + q[3][c] * b.se;
}

// fp32 features: three consecutive channels per corner in one 12-byte load
struct __attribute__((aligned(4))) f32x3a4 { float a, b, c; };
// (element offsets in 32 bits: the host checks H * W * cstride < 2^31)
__device__ __forceinline__ void sample3_f32(const View &x, const Bilin &b, int c0, float v[3]) {
  const float *base = reinterpret_cast<const float *>(x.p) + x.co + c0;
  const int r0 = b.y0 * x.W, r1 = b.y1 * x.W;
  const int e[4] = {(r0 + b.x0) * x.cs, (r0 + b.x1) * x.cs, (r1 + b.x0) * x.cs, (r1 + b.x1) * x.cs};
  float q[4][3];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x3a4 w = *reinterpret_cast<const f32x3a4 *>(base + e[k]);
    q[k][0] = w.a;
    q[k][1] = w.b;
    q[k][2] = w.c;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = q[0][c] * b.nw + q[1][c] * b.ne + q[2][c] * b.sw + q[3][c] * b.se;
}

// PAIRED: bf16 features whose element offsets keep the parity of the channel
// (even channel stride and offset, 4-byte aligned base): sample3_bf16.
template <typename TF, typename TO, typename TY, bool PAIRED>
__global__ void __launch_bounds__(256) offset_div_kernel(View feat, View offs, View flow, View y, const float *fw,
                                                         const float *fb, const float *gx, const float *gy,
                                                         float mag) {
  // the grouped 1x1 fusion weights, read by every thread: LDS, not 21 more
  // vector loads per thread
  __shared__ float sfw[48 * 6], sfb[48];
  for (int i = threadIdx.x; i < 48 * 6; i += 256) sfw[i] = fw[i];
  if (threadIdx.x < 48) sfb[threadIdx.x] = fb[threadIdx.x];
  __syncthreads();
  // workgroup (x, y): pixels 16 x .. 16 x + 15 of row y, thread = 16 pixel + group
  const int g = threadIdx.x & 15;
  const int py = blockIdx.y, px = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (px >= y.W) return;
  const int64_t pix = (int64_t)py * y.W + px;
  const float fx = ld<float>(flow.p, pix * flow.cs + flow.co);
  const float fy = ld<float>(flow.p, pix * flow.cs + flow.co + 1);
  // bilinear x2 upsample of the half-resolution offset map (up2_at), the
  // corner geometry shared by this group's 4 offset and 2 mask channels
  float sy = 0.5f * ((float)py + 0.5f) - 0.5f;
  float sx = 0.5f * ((float)px + 0.5f) - 0.5f;
  sy = sy < 0.f ? 0.f : sy;
  sx = sx < 0.f ? 0.f : sx;
  const int h0 = (int)sy, w0 = (int)sx;
  const int h1 = h0 + (h0 < offs.H - 1 ? 1 : 0), w1 = w0 + (w0 < offs.W - 1 ? 1 : 0);
  const float hl1 = sy - (float)h0, hl0 = 1.f - hl1;
  const float wl1 = sx - (float)w0, wl0 = 1.f - wl1;
  float ov[6];  // offset channels 4g..4g+3 (dx, dy of warps 2g, 2g+1), mask channels 64+2g, 65+2g
  {
    const int64_t e[4] = {((int64_t)h0 * offs.W + w0) * offs.cs + offs.co, ((int64_t)h0 * offs.W + w1) * offs.cs + offs.co,
                          ((int64_t)h1 * offs.W + w0) * offs.cs + offs.co, ((int64_t)h1 * offs.W + w1) * offs.cs + offs.co};
    float cv[4][6];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (sizeof(TO) == 4) {
        const float *op = reinterpret_cast<const float *>(offs.p) + e[k];
        const float4 o4 = *reinterpret_cast<const float4 *>(op + 4 * g);
        const float2 m2 = *reinterpret_cast<const float2 *>(op + 64 + 2 * g);
        cv[k][0] = o4.x; cv[k][1] = o4.y; cv[k][2] = o4.z; cv[k][3] = o4.w;
        cv[k][4] = m2.x; cv[k][5] = m2.y;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) cv[k][j] = ld<TO>(offs.p, e[k] + 4 * g + j);
        cv[k][4] = ld<TO>(offs.p, e[k] + 64 + 2 * g);
        cv[k][5] = ld<TO>(offs.p, e[k] + 65 + 2 * g);
      }
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) ov[j] = (cv[0][j] * wl0 + cv[1][j] * wl1) * hl0 + (cv[2][j] * wl0 + cv[3][j] * wl1) * hl1;
  }
  float xm[6];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = 2 * g + k;                       // warp index 0..31
    // offset channels 2i, 2i+1 of cat(o1, o2) = channels 2i, 2i+1 of the map
    float dx = mag * tanhf(ov[2 * k]);
    float dy = mag * tanhf(ov[2 * k + 1]);
    dx = dx + fx;                                  // flow.repeat: even ch -> dx
    dy = dy + fy;
    const float msk = sigmoidf_(ov[4 + k]);
    const Bilin b = warp_coords(gx[px], gy[py], dx, dy, feat.W, feat.H);
    const int src_group = i & 15;                  // x.repeat(2,1,1,1)
    if constexpr (sizeof(TF) == 4) {
      float v3[3];
      sample3_f32(feat, b, 3 * src_group, v3);
#pragma unroll
      for (int c = 0; c < 3; ++c) xm[3 * k + c] = v3[c] * msk;
    } else if constexpr (PAIRED) {
      float v3[3];
      if (k == 0)
        sample3_bf16<0>(feat, b, 3 * src_group, v3);  // src_group = 2g mod 16: even
      else
        sample3_bf16<1>(feat, b, 3 * src_group, v3);  // odd
#pragma unroll
      for (int c = 0; c < 3; ++c) xm[3 * k + c] = v3[c] * msk;
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) xm[3 * k + c] = sample<TF>(feat, b, 3 * src_group + c) * msk;
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int o = 3 * g + c;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) acc = acc + sfw[o * 6 + k] * xm[k];
    st<TY>(y.p, pix * y.cs + y.co + o, acc + sfb[o]);
  }
}

// ---- OffsetDiversity on fp32 maps (Precision.split / parity), group-planar.
//
// The kernel above runs one thread per (pixel, group) with a wave holding 4
// pixels x 16 groups: every group samples at its own offset, so each of its
// eight 12-byte corner gathers touches 64 different cache lines, and the L1
// tag lookups, not bytes, bound it.  Here the 48-channel
// feature is first copied group-planar, P[16][H][W][3] (planar3_kernel), and a
// wave holds 64 neighbouring pixels of ONE group: their corners lie in a few
// consecutive 12-byte cells of one plane (6-7 lines per gather instead of 64).
// The half-resolution offset rows a block needs are staged in LDS with
// coalesced 16-byte loads, and the 48 output channels of the block's pixels
// are staged in LDS and stored as whole pixels.  Per element the arithmetic
// is offset_div_kernel's, in the same order: identical results.
constexpr int OD_PX = 64;    // pixels of one row per workgroup
constexpr int OD_OCOLS = 34; // half-resolution offset columns such a run reads
constexpr int OD_OST = 100;  // LDS floats per staged offset pixel (96 + pad)

// NHWC 48-channel fp32 -> P[16][H][W][3], one workgroup per 64 pixels (flat
// pixel order), through LDS: coalesced 16-byte loads and stores
__global__ void __launch_bounds__(256) planar3_kernel(View x, float *P, int64_t npix) {
  __shared__ float s[OD_PX * 49];
  const int64_t pix0 = (int64_t)blockIdx.x * OD_PX;
  const int n = (int)(npix - pix0 < OD_PX ? npix - pix0 : OD_PX);
  const float *xp = reinterpret_cast<const float *>(x.p) + x.co;
  for (int i = threadIdx.x; i < n * 12; i += 256) {
    const int p = i / 12, q = i - p * 12;
    const float4 v = *reinterpret_cast<const float4 *>(xp + (pix0 + p) * x.cs + 4 * q);
    float *d = s + p * 49 + 4 * q;
    d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
  }
  __syncthreads();
  if (n == OD_PX) {
    // group sg: 192 contiguous floats = 48 float4 (pix0 * 3 floats is 16-byte aligned)
    for (int i = threadIdx.x; i < 16 * 48; i += 256) {
      const int sg = i / 48, q = i - sg * 48;
      float4 v;
      float *e = &v.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = 4 * q + k, p = f / 3, c = f - p * 3;
        e[k] = s[p * 49 + 3 * sg + c];
      }
      *reinterpret_cast<float4 *>(P + (int64_t)sg * npix * 3 + pix0 * 3 + 4 * q) = v;
    }
  } else {
    for (int i = threadIdx.x; i < 16 * n * 3; i += 256) {
      const int sg = i / (n * 3), f = i - sg * n * 3, p = f / 3, c = f - p * 3;
      P[(int64_t)sg * npix * 3 + pix0 * 3 + f] = s[p * 49 + 3 * sg + c];
    }
  }
}

__global__ void __launch_bounds__(256) offset_div_pl_kernel(const float *P, View offs, View flow, View y,
                                                            const float *fw, const float *fb, const float *gx,
                                                            const float *gy, float mag) {
  __shared__ float sfw[48 * 6], sfb[48];
  __shared__ __align__(16) float so[2 * OD_OCOLS * OD_OST];   // offset rows h0, h1
  __shared__ float sy[OD_PX * 49];                            // output pixels
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int py = blockIdx.y, px0 = blockIdx.x * OD_PX;
  const int W = y.W, H = y.H;
  for (int i = tid; i < 48 * 6; i += 256) sfw[i] = fw[i];
  if (tid < 48) sfb[tid] = fb[tid];
  // the two half-resolution rows and the columns [c0, c0 + OD_OCOLS) of the
  // offset map this row of pixels interpolates from (up2_at's geometry)
  float syf = 0.5f * ((float)py + 0.5f) - 0.5f;
  syf = syf < 0.f ? 0.f : syf;
  const int h0 = (int)syf, h1 = h0 + (h0 < offs.H - 1 ? 1 : 0);
  const float hl1 = syf - (float)h0, hl0 = 1.f - hl1;
  const int c0 = px0 / 2 > 0 ? px0 / 2 - 1 : 0;
  const int nc = offs.W - c0 < OD_OCOLS ? offs.W - c0 : OD_OCOLS;
  const float *op = reinterpret_cast<const float *>(offs.p) + offs.co;
  for (int i = tid; i < 2 * nc * 24; i += 256) {
    const int r = i / (nc * 24), f = i - r * nc * 24, c = f / 24, q = f - c * 24;
    const float4 v = *reinterpret_cast<const float4 *>(op + ((int64_t)(r ? h1 : h0) * offs.W + c0 + c) * offs.cs + 4 * q);
    *reinterpret_cast<float4 *>(so + (r * OD_OCOLS + c) * OD_OST + 4 * q) = v;
  }
  __syncthreads();
  const int px = px0 + lane;
  const bool live = px < W;
  const int pxc = live ? px : W - 1;
  const int64_t pix = (int64_t)py * W + pxc;
  const float2 fv = *reinterpret_cast<const float2 *>(reinterpret_cast<const float *>(flow.p) + pix * flow.cs + flow.co);
  float sxf = 0.5f * ((float)pxc + 0.5f) - 0.5f;
  sxf = sxf < 0.f ? 0.f : sxf;
  const int w0 = (int)sxf, w1 = w0 + (w0 < offs.W - 1 ? 1 : 0);
  const float wl1 = sxf - (float)w0, wl0 = 1.f - wl1;
  const float *o00 = so + (w0 - c0) * OD_OST, *o01 = so + (w1 - c0) * OD_OST;
  const float *o10 = so + (OD_OCOLS + w0 - c0) * OD_OST, *o11 = so + (OD_OCOLS + w1 - c0) * OD_OST;
  const float gxv = gx[pxc], gyv = gy[py];
  const int64_t plane = (int64_t)H * W * 3;
  // wave w: groups w, w + 4, w + 8, w + 12
#pragma unroll 1
  for (int gi = 0; gi < 4; ++gi) {
    const int g = wave + 4 * gi;
    float ov[6];
    {
      float cv[4][6];
      const float *cs4[4] = {o00, o01, o10, o11};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 a = *reinterpret_cast<const float4 *>(cs4[k] + 4 * g);
        const float2 m = *reinterpret_cast<const float2 *>(cs4[k] + 64 + 2 * g);
        cv[k][0] = a.x, cv[k][1] = a.y, cv[k][2] = a.z, cv[k][3] = a.w, cv[k][4] = m.x, cv[k][5] = m.y;
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) ov[j] = (cv[0][j] * wl0 + cv[1][j] * wl1) * hl0 + (cv[2][j] * wl0 + cv[3][j] * wl1) * hl1;
    }
    float xm[6];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = 2 * g + k;
      float dx = mag * tanhf(ov[2 * k]);
      float dy = mag * tanhf(ov[2 * k + 1]);
      dx = dx + fv.x;
      dy = dy + fv.y;
      const float msk = sigmoidf_(ov[4 + k]);
      const Bilin b = warp_coords(gxv, gyv, dx, dy, W, H);
      const float *base = P + (i & 15) * plane;
      const int r0 = b.y0 * W, r1 = b.y1 * W;
      const int e[4] = {(r0 + b.x0) * 3, (r0 + b.x1) * 3, (r1 + b.x0) * 3, (r1 + b.x1) * 3};
      float q[4][3];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const f32x3a4 wv = *reinterpret_cast<const f32x3a4 *>(base + e[kk]);
        q[kk][0] = wv.a;
        q[kk][1] = wv.b;
        q[kk][2] = wv.c;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c)
        xm[3 * k + c] = (q[0][c] * b.nw + q[1][c] * b.ne + q[2][c] * b.sw + q[3][c] * b.se) * msk;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int o = 3 * g + c;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 6; ++k) acc = acc + sfw[o * 6 + k] * xm[k];
      sy[lane * 49 + o] = acc + sfb[o];
    }
  }
  __syncthreads();
  // whole output pixels: 12 float4 each
  const int n = W - px0 < OD_PX ? W - px0 : OD_PX;
  float *yp = reinterpret_cast<float *>(y.p) + y.co;
  for (int i = tid; i < n * 12; i += 256) {
    const int p = i / 12, q = i - p * 12;
    const float *s = sy + p * 49 + 4 * q;
    *reinterpret_cast<float4 *>(yp + ((int64_t)py * W + px0 + p) * y.cs + 4 * q) = make_float4(s[0], s[1], s[2], s[3]);
  }
}

template <typename TX, typename TY>
__global__ void resize_kernel(View x, View y, int up, float mul) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)y.H * y.W * y.C;
  if (idx >= total) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  const int oy = (int)(pix / y.W), ox = (int)(pix - (int64_t)oy * y.W);
  float v;
  if (up) {
    v = up2_at<TX>(x, oy, ox, c);
  } else {
    const float scy = (float)x.H / (float)y.H, scx = (float)x.W / (float)y.W;
    float sy = scy * ((float)oy + 0.5f) - 0.5f;
    float sx = scx * ((float)ox + 0.5f) - 0.5f;
    sy = sy < 0.f ? 0.f : sy;
    sx = sx < 0.f ? 0.f : sx;
    const int h0 = (int)sy, w0 = (int)sx;
    const int h1 = h0 + (h0 < x.H - 1 ? 1 : 0), w1 = w0 + (w0 < x.W - 1 ? 1 : 0);
    const float hl1 = sy - (float)h0, hl0 = 1.f - hl1;
    const float wl1 = sx - (float)w0, wl0 = 1.f - wl1;
    const float a = ld<TX>(x.p, ((int64_t)h0 * x.W + w0) * x.cs + x.co + c);
    const float b = ld<TX>(x.p, ((int64_t)h0 * x.W + w1) * x.cs + x.co + c);
    const float cc = ld<TX>(x.p, ((int64_t)h1 * x.W + w0) * x.cs + x.co + c);
    const float d = ld<TX>(x.p, ((int64_t)h1 * x.W + w1) * x.cs + x.co + c);
    v = (a * wl0 + b * wl1) * hl0 + (cc * wl0 + d * wl1) * hl1;
  }
  st<TY>(y.p, pix * y.cs + y.co + c, v * mul);
}

template <typename TX, typename TY>
__global__ void pool_kernel(View x, View y, int is_max) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)y.H * y.W * y.C;
  if (idx >= total) return;
  const int c = (int)(idx % y.C);
  const int64_t pix = idx / y.C;
  const int oy = (int)(pix / y.W), ox = (int)(pix - (int64_t)oy * y.W);
  const int64_t r0 = (int64_t)(2 * oy) * x.W, r1 = r0 + x.W;
  const float a = ld<TX>(x.p, (r0 + 2 * ox) * x.cs + x.co + c);
  const float b = ld<TX>(x.p, (r0 + 2 * ox + 1) * x.cs + x.co + c);
  const float cc = ld<TX>(x.p, (r1 + 2 * ox) * x.cs + x.co + c);
  const float d = ld<TX>(x.p, (r1 + 2 * ox + 1) * x.cs + x.co + c);
  float v;
  if (is_max) {
    v = a;
    v = (b > v || isnan(b)) ? b : v;
    v = (cc > v || isnan(cc)) ? cc : v;
    v = (d > v || isnan(d)) ? d : v;
  } else {
    float s = 0.f;
    s = s + a;
    s = s + b;
    s = s + cc;
    s = s + d;
    v = s / 4.f;
  }
  st<TY>(y.p, pix * y.cs + y.co + c, v);
}

#define DISPATCH2(tx, ty, KERNEL, ...)                                         \
  do {                                                                         \
    if ((tx) == DCVC_F32 && (ty) == DCVC_F32) { KERNEL(float, float, __VA_ARGS__); }            \
    else if ((tx) == DCVC_F32) { KERNEL(float, uint16_t, __VA_ARGS__); }                        \
    else if ((ty) == DCVC_F32) { KERNEL(uint16_t, float, __VA_ARGS__); }                        \
    else { KERNEL(uint16_t, uint16_t, __VA_ARGS__); }                                           \
  } while (0)

}  // namespace

extern "C" int dcvc_flow_warp(dcvc_tensor x, dcvc_tensor flow, dcvc_tensor y, const float *gx,
                              const float *gy, void *stream) {
  if (!ok(x) || !ok(flow) || !ok(y) || !gx || !gy) return DCVC_HIP_EINVAL;
  if (flow.dtype != DCVC_F32 || flow.C != 2 || flow.H != y.H || flow.W != y.W || x.H != y.H ||
      x.W != y.W || x.C != y.C)
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (x.dtype == DCVC_BF16 && y.dtype == DCVC_BF16 && y.C % 8 == 0 && x.cstride % 8 == 0 && x.coff % 8 == 0 &&
      y.cstride % 8 == 0 && y.coff % 8 == 0 && flow.cstride % 2 == 0 && flow.coff % 2 == 0 &&
      ((uintptr_t)x.ptr & 15) == 0 && ((uintptr_t)y.ptr & 15) == 0 && ((uintptr_t)flow.ptr & 7) == 0) {
    const int64_t total = (int64_t)y.H * y.W * (y.C / 8);
    hipLaunchKernelGGL(warp8_kernel, dim3((unsigned)((total + 255) / 256 + 7) & ~7u), dim3(256), 0, st, mk(x), mk(flow),
                       mk(y), gx, gy);
    DCVC_LAUNCH_CHECK();
    return DCVC_HIP_OK;
  }
  if (x.dtype == DCVC_F32 && y.dtype == DCVC_F32 && y.C % 4 == 0 && x.cstride % 4 == 0 && x.coff % 4 == 0 &&
      y.cstride % 4 == 0 && y.coff % 4 == 0 && flow.cstride % 2 == 0 && flow.coff % 2 == 0 &&
      ((uintptr_t)x.ptr & 15) == 0 && ((uintptr_t)y.ptr & 15) == 0 && ((uintptr_t)flow.ptr & 7) == 0) {
    const int64_t total = (int64_t)y.H * y.W * (y.C / 4);
    hipLaunchKernelGGL(warp4_kernel, dim3((unsigned)((total + 255) / 256 + 7) & ~7u), dim3(256), 0, st, mk(x), mk(flow),
                       mk(y), gx, gy);
    DCVC_LAUNCH_CHECK();
    return DCVC_HIP_OK;
  }
  const int tpc = y.C >= 32 ? 32 : (y.C >= 8 ? 8 : 4);  // threads per pixel
  const int ppb = 256 / tpc;
  const int64_t npix = (int64_t)y.H * y.W;
  dim3 blk(tpc, ppb);
  dim3 grd((unsigned)((npix + ppb - 1) / ppb));
#define K(TX, TY, ...) hipLaunchKernelGGL((warp_kernel<TX, TY>), grd, blk, 0, st, mk(x), mk(flow), mk(y), gx, gy)
  DISPATCH2(x.dtype, y.dtype, K, 0);
#undef K
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_offset_diversity(dcvc_tensor feat, dcvc_tensor offs, dcvc_tensor flow,
                                     dcvc_tensor y, const float *fw, const float *fb,
                                     const float *gx, const float *gy, float max_mag,
                                     void *stream) {
  if (!ok(feat) || !ok(offs) || !ok(flow) || !ok(y) || !fw || !fb || !gx || !gy)
    return DCVC_HIP_EINVAL;
  if (feat.C != 48 || y.C != 48 || offs.C != 96 || flow.C != 2 || flow.dtype != DCVC_F32 ||
      feat.H != y.H || feat.W != y.W || flow.H != y.H || flow.W != y.W ||
      offs.H * 2 != y.H || offs.W * 2 != y.W)
    return DCVC_HIP_EINVAL;
  if (offs.dtype == DCVC_F32 && (offs.cstride % 4 || offs.coff % 4 || ((uintptr_t)offs.ptr & 15)))
    return DCVC_HIP_EUNSUPPORTED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grd((unsigned)((y.W + 15) / 16), (unsigned)y.H);
  if ((int64_t)feat.H * feat.W * feat.cstride >= ((int64_t)1 << 31)) return DCVC_HIP_EUNSUPPORTED;
#define LAUNCH(TF, TO, TY, PR)                                                                  \
  hipLaunchKernelGGL((offset_div_kernel<TF, TO, TY, PR>), grd, dim3(256), 0, st, mk(feat),       \
                     mk(offs), mk(flow), mk(y), fw, fb, gx, gy, max_mag)
  const bool f32 = feat.dtype == DCVC_F32, o32 = offs.dtype == DCVC_F32, y32 = y.dtype == DCVC_F32;
  const bool paired = !f32 && feat.cstride % 2 == 0 && feat.coff % 2 == 0 && ((uintptr_t)feat.ptr & 3) == 0;
  if (f32 && o32 && y32) LAUNCH(float, float, float, false);
  else if (!f32 && !o32 && !y32) {
    if (paired) LAUNCH(uint16_t, uint16_t, uint16_t, true);
    else LAUNCH(uint16_t, uint16_t, uint16_t, false);
  } else if (!f32 && o32 && !y32) {
    if (paired) LAUNCH(uint16_t, float, uint16_t, true);
    else LAUNCH(uint16_t, float, uint16_t, false);
  } else return DCVC_HIP_EUNSUPPORTED;
#undef LAUNCH
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int64_t dcvc_offset_diversity_workspace(int H, int W) {
  return H > 0 && W > 0 ? (int64_t)16 * H * W * 3 * 4 : 0;
}

extern "C" int dcvc_offset_diversity_ws(dcvc_tensor feat, dcvc_tensor offs, dcvc_tensor flow, dcvc_tensor y,
                                        const float *fw, const float *fb, const float *gx, const float *gy,
                                        float max_mag, void *workspace, int64_t ws_bytes, void *stream) {
  if (!ok(feat) || !ok(offs) || !ok(flow) || !ok(y) || !fw || !fb || !gx || !gy) return DCVC_HIP_EINVAL;
  if (feat.C != 48 || y.C != 48 || offs.C != 96 || flow.C != 2 || flow.dtype != DCVC_F32 || feat.H != y.H ||
      feat.W != y.W || flow.H != y.H || flow.W != y.W || offs.H * 2 != y.H || offs.W * 2 != y.W)
    return DCVC_HIP_EINVAL;
  const bool vec = feat.dtype == DCVC_F32 && offs.dtype == DCVC_F32 && y.dtype == DCVC_F32 &&
                   feat.cstride % 4 == 0 && feat.coff % 4 == 0 && ((uintptr_t)feat.ptr & 15) == 0 &&
                   offs.cstride % 4 == 0 && offs.coff % 4 == 0 && ((uintptr_t)offs.ptr & 15) == 0 &&
                   y.cstride % 4 == 0 && y.coff % 4 == 0 && ((uintptr_t)y.ptr & 15) == 0 &&
                   flow.cstride % 2 == 0 && flow.coff % 2 == 0 && ((uintptr_t)flow.ptr & 7) == 0 &&
                   (int64_t)y.H * y.W * 3 < ((int64_t)1 << 31);
  // (no workspace or another layout: the pixel-major kernel)
  if (!vec || !workspace || ((uintptr_t)workspace & 15) || ws_bytes < dcvc_offset_diversity_workspace(y.H, y.W))
    return dcvc_offset_diversity(feat, offs, flow, y, fw, fb, gx, gy, max_mag, stream);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t npix = (int64_t)y.H * y.W;
  float *P = reinterpret_cast<float *>(workspace);
  hipLaunchKernelGGL(planar3_kernel, dim3((unsigned)((npix + OD_PX - 1) / OD_PX)), dim3(256), 0, st, mk(feat), P, npix);
  DCVC_LAUNCH_CHECK();
  hipLaunchKernelGGL(offset_div_pl_kernel, dim3((unsigned)((y.W + OD_PX - 1) / OD_PX), (unsigned)y.H), dim3(256), 0,
                     st, P, mk(offs), mk(flow), mk(y), fw, fb, gx, gy, max_mag);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_resize2x(dcvc_tensor x, dcvc_tensor y, int up, float mul, void *stream) {
  if (!ok(x) || !ok(y) || x.C != y.C) return DCVC_HIP_EINVAL;
  if (up ? (y.H != 2 * x.H || y.W != 2 * x.W) : (y.H != x.H / 2 || y.W != x.W / 2))
    return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = (int64_t)y.H * y.W * y.C;
  const unsigned grd = (unsigned)((total + 255) / 256);
#define K(TX, TY, ...) hipLaunchKernelGGL((resize_kernel<TX, TY>), dim3(grd), dim3(256), 0, st, mk(x), mk(y), up, mul)
  DISPATCH2(x.dtype, y.dtype, K, 0);
#undef K
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

extern "C" int dcvc_pool2x2(dcvc_tensor x, dcvc_tensor y, int is_max, void *stream) {
  if (!ok(x) || !ok(y) || x.C != y.C || y.H != x.H / 2 || y.W != x.W / 2) return DCVC_HIP_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = (int64_t)y.H * y.W * y.C;
  const unsigned grd = (unsigned)((total + 255) / 256);
#define K(TX, TY, ...) hipLaunchKernelGGL((pool_kernel<TX, TY>), dim3(grd), dim3(256), 0, st, mk(x), mk(y), is_max)
  DISPATCH2(x.dtype, y.dtype, K, 0);
#undef K
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}
