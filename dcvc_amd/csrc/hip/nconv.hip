// Split-fp16 convolution for stride-1 7x7 layers with very few output
// channels: SpyNet's last 7x7 of every basic module, 16 -> 2
// (DCVC-DC/src/models/video_net.py:79-100): 378 -> 142 us at 1088 x 1920, 94
// -> 38 us at 544 x 960 (profiles/r05w_nconv_micro.jsonl).
//
// sconv.hip puts the output channels on the MFMA's 16 M rows, so 2 of 16 rows
// carry results and every product is computed 8 times over.  Here the GEMM is
// turned around: pixels on M, and on N the COUT x KS pairs (output channel c,
// tap column dx), n = c KS + dx <= 16 (14 for 16 -> 2 7x7, 9 for 48 -> 3 3x3);
// K runs over (tap row dy, input channel), KS x CIN, in 32-deep steps:
//   P[pixel p][c, dx] = sum_{dy, ci} x[y + dy - pad][p][ci] * w[c][ci][dy][dx]
// and an output is the sum of KS shifted partials:
//   out[y][x][c] = bias[c] + sum_dx P[x + dx - pad][c, dx].
// A wave owns one output row of TW = 80 - (KS - 1) pixels: five 16-pixel
// groups of partials (80 pixels, the halo included), written to its own LDS
// strip and summed there.  Products are sconv.hip's split (xh*wh + 2^-11
// (xh*wl + xl*wh), fp32 accumulation); the weights' hi / lo halves come
// straight from the layer's F16X3 packed buffer and stay in registers (one B
// fragment per K step) for the wave's tasks.  The K order and the dx sum
// differ from sconv.hip, so the outputs agree with it to the split bound, not
// bit for bit (tests/test_gpu_nconv.py).
#include "common.h"
#include "split.h"

#include <cstring>

namespace {

struct NP {
  const float *x;
  int H, W, xcs, xco, xbytes;
  const uint16_t *w;   // F16X3 packed weights (dcvc_conv_pack_weights)
  const float *bias, *scale;
  float *y;
  int Wo, ycs, yco;
  const float *res, *res2;
  int rcs, rco, r2cs, r2co;
  int cout, pad, ntx, ntasks;
  int in_lrelu;
  float in_slope;
  int act;
  float slope;
  int *ovf;
};

constexpr int kGroups = 5, kPW = 16 * kGroups;   // partial pixels per task
constexpr int kPS = 17;                            // LDS floats per partial pixel (16 + pad)

// raw (hi, lo) halves of w(n, tap, ci) in dcvc_conv_pack_weights' F16X3 layout
__device__ __forceinline__ void packed_hl(const uint16_t *w, int n, int tap, int ci, int cin, int cout, int kt,
                                          uint16_t &h, uint16_t &l) {
  const int nch = (cin + 31) >> 5, c = ci >> 5, lc = ci & 31;
  const int64_t wchunk = (int64_t)2 * kt * cout * 32;
  int rows, r, within;
  if (c < nch - 1) {
    rows = kt;
    r = tap;
    within = lc;
  } else {
    const int vcl = cin - 32 * (nch - 1);
    const int tpkl = vcl <= 8 ? 4 : vcl <= 16 ? 2 : 1, spl = 4 / tpkl;
    rows = (kt + tpkl - 1) / tpkl;
    r = tap / tpkl;
    within = ((tap % tpkl) * spl + (lc >> 3)) * 8 + (lc & 7);
  }
  const int64_t o = c * wchunk + ((int64_t)r * cout + n) * 32 + within;
  h = w[o];
  l = w[o + (int64_t)rows * cout * 32];
}

template <int KS, int CIN, int COUT, bool INL>
__global__ void __launch_bounds__(256) nconv_kernel(NP p) {
  static_assert(COUT * KS <= 16 && CIN % 8 == 0, "shape");
  constexpr int NS = (KS * CIN + 31) / 32;   // K steps
  constexpr int TW = kPW - (KS - 1);          // output pixels per task
  SplitRange rg(p.ovf);
  __shared__ float Lp[4][kPW * kPS];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int col = lane & 15, q = lane >> 4;
  float *P = Lp[wave];

  // B fragments: lane (col = n, q) holds w[c][ci][dy][dx] for k = 32 s + 8 q + j
  f16x8 bh[NS], bl[NS];
  {
    const int c = col / KS, dx = col - c * KS;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint16_t hh[8], ll[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * q + j, dy = k / CIN, ci = k - dy * CIN;
        hh[j] = ll[j] = 0;
        if (c < COUT && dy < KS) packed_hl(p.w, c, dy * KS + dx, ci, CIN, p.cout, KS * KS, hh[j], ll[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bh[s][j] = __builtin_bit_cast(_Float16, hh[j]);
        bl[s][j] = __builtin_bit_cast(_Float16, ll[j]);
      }
    }
  }
  float bias[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) bias[c] = p.bias[c];
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.x), (short)0, p.xbytes, 0x00020000);

  for (int t = blockIdx.x * 4 + wave; t < p.ntasks; t += gridDim.x * 4) {
    const int oy = t / p.ntx, x0 = (t - oy * p.ntx) * TW, px0 = x0 - p.pad;
    f32x4 am[kGroups], ac[kGroups];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
      am[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      ac[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // A fragments: lane (col = pixel, q) holds 8 channels of tap row dy
      const int k0 = 32 * s + 8 * q, dy = k0 / CIN, ci0 = k0 - dy * CIN;
      const int iy = oy + dy - p.pad;
      const bool rok = dy < KS && (unsigned)iy < (unsigned)p.H;
      float v[kGroups][8];
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        const int ix = px0 + 16 * g + col;
        const int o = rok && (unsigned)ix < (unsigned)p.W ? ((iy * p.W + ix) * p.xcs + p.xco + ci0) * 4 : 0x7fffffe0;
        const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
        const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[g][e] = a[e];
          v[g][4 + e] = b[e];
        }
      }
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        if constexpr (INL) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[g][e] = lrelu_in(v[g][e], p.in_slope);
        }
        rg.add8(v[g]);
        u32x4_t h, l;
        split8(v[g], h, l);
        const f16x8 ah = __builtin_bit_cast(f16x8, h), al = __builtin_bit_cast(f16x8, l);
        am[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[s], am[g], 0, 0, 0);
        ac[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[s], ac[g], 0, 0, 0);
        ac[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[s], ac[g], 0, 0, 0);
      }
    }
    // partials to the wave's strip: D[m = 4 q + e][n = col] of group g
    wave_lds_sync();   // the previous task's reads of the strip are done
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) P[(16 * g + 4 * q + e) * kPS + col] = am[g][e] + ac[g][e] * kLoInv;
    wave_lds_sync();
    // outputs: out[x0 + x][c] = act(sum_dx P[x + dx][c KS + dx] + bias) ...
    for (int i = lane; i < TW * COUT; i += 64) {
      const int x = i / COUT, c = i - x * COUT, ox = x0 + x;
      if (ox >= p.Wo) continue;
      float a = 0.f;
#pragma unroll
      for (int dx = 0; dx < KS; ++dx) a += P[(x + dx) * kPS + c * KS + dx];
      float r = 0.f;
#pragma unroll
      for (int cc = 0; cc < COUT; ++cc) r = cc == c ? bias[cc] : r;
      float o = apply_act(p.act, a + r, p.slope);
      const int64_t pix = (int64_t)oy * p.Wo + ox;
      if (p.res) o = p.res[pix * p.rcs + p.rco + c] + o;
      if (p.res2) o = p.res2[pix * p.r2cs + p.r2co + c] + o;
      if (p.scale) o *= p.scale[c];
      p.y[pix * p.ycs + p.yco + c] = o;
    }
  }
}

int g_enable = 1;   // dcvc_set_option("nconv", 0): these layers to sconv.hip
int g_cus = 0;

template <int KS, int CIN, int COUT>
int launch(NP p, int in_lrelu, hipStream_t st) {
  constexpr int TW = kPW - (KS - 1);
  p.ntx = (p.Wo + TW - 1) / TW;
  const int64_t tasks = (int64_t)p.ntx * p.H;   // (row, column tile); stride 1: Ho = H
  if (tasks <= 0) return DCVC_HIP_OK;
  if (tasks > 0x7fffffff) return DCVC_HIP_EINVAL;
  p.ntasks = (int)tasks;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  // a few tasks per wave, so each wave gathers its weight fragments once
  int64_t grid = (tasks + 4 * 4 - 1) / (4 * 4);
  if (grid > (int64_t)g_cus * 8) grid = (int64_t)g_cus * 8;
  if (grid < 1) grid = 1;
  auto kern = in_lrelu ? nconv_kernel<KS, CIN, COUT, true> : nconv_kernel<KS, CIN, COUT, false>;
  dcvc_note_kernel("nconv_kernel<%d, %d, %d, %s>", KS, CIN, COUT, in_lrelu ? "true" : "false");
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), 0, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

extern "C" void dcvc_internal_nconv_enable(int v) { g_enable = v; }

// Stride-1 7x7 split convolutions with COUT * KS <= 16 output (channel, tap
// column) pairs: SpyNet's 16 -> 2 (dcvc_conv2d tries it before the other
// split kernels).  DCVC_HIP_EUNSUPPORTED otherwise.
extern "C" int dcvc_internal_nconv(const dcvc_conv_args *a, void *stream) {
  if (!g_enable) return DCVC_HIP_EUNSUPPORTED;
  if (a->stride != 1 || a->kh != a->kw || a->pad != a->kh / 2 || a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32 || !a->bias) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && !(a->in_op == DCVC_IN_LRELU && a->in_slope >= 0.f && a->in_slope <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->res2.ptr && !a->res.ptr) return DCVC_HIP_EUNSUPPORTED;
  if ((a->res.ptr && a->res.dtype != DCVC_F32) || (a->res2.ptr && a->res2.dtype != DCVC_F32)) return DCVC_HIP_EUNSUPPORTED;
  if ((uintptr_t)a->x.ptr % 16 || a->x.cstride % 4 || a->x.coff % 4) return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)a->x.H * a->x.W * a->x.cstride * 4 >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  if (a->y.H != a->x.H || a->y.W != a->x.W) return DCVC_HIP_EUNSUPPORTED;
  NP p{};
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.xbytes = (int)((int64_t)a->x.H * a->x.W * a->x.cstride * 4);
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.bias = a->bias;
  p.scale = a->scale;
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.Wo = a->x.W;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  if (a->res.ptr) {
    p.res = reinterpret_cast<const float *>(a->res.ptr);
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
  }
  if (a->res2.ptr) {
    p.res2 = reinterpret_cast<const float *>(a->res2.ptr);
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
  }
  p.cout = a->cout;
  p.pad = a->pad;
  p.in_lrelu = a->in_op == DCVC_IN_LRELU;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.ovf = dcvc_internal_split_flag();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int il = p.in_lrelu;
  if (a->kh == 7 && a->cin == 16 && a->cout == 2) return launch<7, 16, 2>(p, il, st);
  if (a->kh == 7 && a->cin == 16 && a->cout == 1) return launch<7, 16, 1>(p, il, st);
  if (a->kh == 7 && a->cin == 32 && a->cout == 2) return launch<7, 32, 2>(p, il, st);
  // (3x3 heads, 48 -> 3: 212 us here against 205 on sconv.hip, whose halo
  // image loads each input pixel once where this kernel loads it per tap row,
  // profiles/r05w_nconv_micro.jsonl: left to sconv)
  return DCVC_HIP_EUNSUPPORTED;
}
