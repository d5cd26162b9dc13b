// Thin convolutions in fp32 VALU arithmetic: the layers with 2 input
// channels, where a 32-deep MFMA K step would be 94 % padding: the motion
// encoder's first ResidualBlockWithStride on the 2-channel flow, 3x3 / 1x1
// stride 2, 2 -> 64 (DCVC-DC/src/models/video_model.py:121-140, layers.py
// ResidualBlockWithStride): 125 -> 58 us and 143 -> 29 us at 1080p against
// sconv.hip (profiles/r05r_tconv_ci_micro.jsonl).  (The few-output-channel
// layers have an MFMA kernel of their own, nconv.hip; an fp32-VALU one lost
// to sconv there)
// The weights are read from the split-packed buffer the layer already has
// (dcvc_conv_pack_weights' F16X3 layout) and rebuilt in LDS as hi + 2^-11 lo,
// a 22-bit fp32 value (the split kernels' products drop the lo x lo term
// instead); every product is an fp32 FMA.  The arithmetic is therefore not
// sconv.hip's bit for bit: tests/test_gpu_tconv.py holds it to fp64 and to
// sconv within the split precision's bound.
#include "common.h"

#include <cstring>

namespace {

struct TP {
  const float *x;
  int H, W, xcs, xco;
  const uint16_t *w;   // F16X3 packed weights
  const float *bias, *scale;
  float *y;
  int Ho, Wo, ycs, yco;
  const float *res, *res2;
  int rcs, rco, r2cs, r2co;
  int cin, cout, kt, S, pad;
  int in_lrelu;
  float in_slope;
  int act;
  float slope;
  int vec_out;
  int nq;               // pixel quads per output row
};

// w(n, tap, ci) of dcvc_conv_pack_weights' F16X3 layout: 32-channel chunks,
// per chunk a hi then a lo block of [row][cout][32]; the last chunk packs
// tpkl taps per row when it holds <= 8 / <= 16 channels
__device__ __forceinline__ float packed_w(const uint16_t *w, int n, int tap, int ci, int cin, int cout, int kt) {
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
  const float hi = (float)__builtin_bit_cast(_Float16, w[o]);
  const float lo = (float)__builtin_bit_cast(_Float16, w[o + (int64_t)rows * cout * 32]);
  return hi + lo * (1.f / 2048.f);
}

// out = scale * (res2 + (res + act(acc + bias))) for output channel n of pixel pix
__device__ __forceinline__ float epi(const TP &p, float acc, int n, int64_t pix) {
  float v = apply_act(p.act, acc + p.bias[n], p.slope);
  if (p.res) v = p.res[pix * p.rcs + p.rco + n] + v;
  if (p.res2) v = p.res2[pix * p.r2cs + p.r2co + n] + v;
  if (p.scale) v *= p.scale[n];
  return v;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xrsrc(const TP &p) {
  // the host keeps H * W * cstride * 4 below 2^31 - 64: 32-bit offsets, and
  // an out-of-range offset (kOob) reads zeros (the zero padding)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.x), (short)0,
                                           (int)((int64_t)p.H * p.W * p.xcs * 4), 0x00020000);
}
constexpr int kOob = 0x7ffffff0;

// ---- few input channels: thread = (16 output channels, 4 consecutive output
// pixels of a row); lane g of a pixel quad's 4 lanes owns the channels
// 16 j + 4 g + e (j, e < 4), so each of its 16-byte stores lands beside the
// other three lanes' (64 contiguous bytes of the pixel).  Input pixels by
// buffer loads (zeros outside the image), one tap row at a time.  LDS: the
// weights as [tap][ci][cout].
template <int KS, int S, int CIN, bool INL>
__global__ void __launch_bounds__(256) tconv_ci_kernel(TP p) {
  extern __shared__ __align__(16) unsigned char smem[];
  float *Lw = reinterpret_cast<float *>(smem);
#pragma clang loop vectorize(disable) interleave(disable)
  for (int i = threadIdx.x; i < KS * KS * CIN * p.cout; i += 256) {
    const int n = i % p.cout, r = i / p.cout, ci = r % CIN, tap = r / CIN;
    Lw[i] = packed_w(p.w, n, tap, ci, CIN, p.cout, KS * KS);
  }
  __syncthreads();
  // threads: (row, quad, 64-channel block, lane g)
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int g = (int)(gid & 3);
  const int64_t t = gid >> 2;
  const int nb = p.cout >> 6;
  const int b = (int)(t % nb);
  const int64_t q = t / nb;
  if (q >= (int64_t)p.Ho * p.nq) return;
  const int oy = (int)(q / p.nq), ox0 = (int)(q - (int64_t)oy * p.nq) * 4;
  const int n0 = b * 64 + 4 * g;   // channels n0 + 16 j + e
  const __amdgpu_buffer_rsrc_t xr = xrsrc(p);
  float acc[4][16];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[k][i] = 0.f;
  // one tap row at a time: its KS x 4 input pixels, then their products
#pragma unroll 1
  for (int dy = 0; dy < KS; ++dy) {
    const int iy = oy * S + dy - p.pad;
    const bool rok = (unsigned)iy < (unsigned)p.H;
    float xv[KS][4][CIN];
#pragma unroll
    for (int dx = 0; dx < KS; ++dx)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ix = (ox0 + k) * S + dx - p.pad;
        const int o = rok && (unsigned)ix < (unsigned)p.W ? ((iy * p.W + ix) * p.xcs + p.xco) * 4 : kOob;
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o + 4 * ci, 0, 0));
          if constexpr (INL) v = fmaxf(v, v * p.in_slope);
          xv[dx][k][ci] = v;
        }
      }
#pragma unroll
    for (int dx = 0; dx < KS; ++dx)
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) {
        const float *wr = Lw + ((dy * KS + dx) * CIN + ci) * p.cout + n0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 wv = *reinterpret_cast<const f32x4 *>(wr + 16 * j);
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[k][4 * j + e] = __builtin_fmaf(wv[e], xv[dx][k][ci], acc[k][4 * j + e]);
        }
      }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ox = ox0 + k;
    if (ox >= p.Wo) break;
    const int64_t pix = (int64_t)oy * p.Wo + ox;
    float *yp = p.y + pix * p.ycs + p.yco;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = epi(p, acc[k][4 * j + e], n0 + 16 * j + e, pix);
      if (p.vec_out) {
        *reinterpret_cast<f32x4 *>(yp + n0 + 16 * j) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) yp[n0 + 16 * j + e] = v[e];
      }
    }
  }
}

int g_enable = 1;   // dcvc_set_option("tconv", 0): these layers to the split kernels

template <typename K>
int launch(K kern, const char *name, int64_t threads, size_t lds, const TP &p, hipStream_t st) {
  const int64_t blocks = (threads + 255) / 256;
  if (blocks <= 0) return DCVC_HIP_OK;
  if (blocks > 0x7fffffff) return DCVC_HIP_EINVAL;
  dcvc_note_kernel("%s", name);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

extern "C" void dcvc_internal_tconv_enable(int v) { g_enable = v; }

// Thin split-precision convolutions (dcvc_conv2d tries it first for
// DCVC_F16X3 weights): 2-channel-input 3x3 / 1x1 layers of a multiple of 64
// output channels.  DCVC_HIP_EUNSUPPORTED otherwise.
extern "C" int dcvc_internal_tconv(const dcvc_conv_args *a, void *stream) {
  if (!g_enable) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != a->kw || a->pad != a->kh / 2 || a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && !(a->in_op == DCVC_IN_LRELU)) return DCVC_HIP_EUNSUPPORTED;
  if (a->res2.ptr && !a->res.ptr) return DCVC_HIP_EUNSUPPORTED;
  if ((a->res.ptr && a->res.dtype != DCVC_F32) || (a->res2.ptr && a->res2.dtype != DCVC_F32)) return DCVC_HIP_EUNSUPPORTED;
  const bool ci = a->cin == 2 && (a->kh == 3 || a->kh == 1) && a->cout % 64 == 0 && a->cout <= 256 &&
                  (a->stride == 1 || a->stride == 2);
  if (!ci) return DCVC_HIP_EUNSUPPORTED;
  TP p{};
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.bias = a->bias;
  p.scale = a->scale;
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.S = a->stride;
  p.pad = a->pad;
  p.Ho = (a->x.H + 2 * a->pad - a->kh) / a->stride + 1;
  p.Wo = (a->x.W + 2 * a->pad - a->kw) / a->stride + 1;
  if (a->y.H != p.Ho || a->y.W != p.Wo) return DCVC_HIP_EUNSUPPORTED;
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
  p.cin = a->cin;
  p.cout = a->cout;
  p.kt = a->kh * a->kw;
  p.in_lrelu = a->in_op == DCVC_IN_LRELU;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.vec_out = (uintptr_t)a->y.ptr % 16 == 0 && a->y.cstride % 4 == 0 && a->y.coff % 4 == 0;
  p.nq = (p.Wo + 3) / 4;
  if (!p.bias) return DCVC_HIP_EUNSUPPORTED;
  // 32-bit buffer offsets of the input map
  if ((int64_t)p.H * p.W * p.xcs * 4 >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t quads = (int64_t)p.Ho * p.nq;
  const size_t lds = (size_t)a->kh * a->kw * 2 * a->cout * 4;
  const int64_t threads = quads * (a->cout / 64) * 4;
#define TCI(KS, S)                                                                                     \
  if (a->kh == KS && a->stride == S)                                                                   \
    return p.in_lrelu ? launch(tconv_ci_kernel<KS, S, 2, true>, "tconv_ci_kernel<" #KS ", " #S ", 2, true>", \
                               threads, lds, p, st)                                                    \
                      : launch(tconv_ci_kernel<KS, S, 2, false>, "tconv_ci_kernel<" #KS ", " #S ", 2, false>", \
                               threads, lds, p, st);
  TCI(3, 2) TCI(3, 1) TCI(1, 2) TCI(1, 1)
#undef TCI
  return DCVC_HIP_EUNSUPPORTED;
}
