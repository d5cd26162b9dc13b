// NHWC implicit-GEMM convolution on gfx950 MFMA.
//
// One workgroup = 4 waves (256 threads) computes an output tile of TH rows x
// 16 columns x BN channels.  The GEMM is D[n][pixel] = W[n][k] * X[k][pixel]
// with k = (tap, input channel); the output channel is the MFMA row so each
// lane ends with 4 consecutive channels of one pixel (NHWC-friendly stores).
//
// K is walked in chunks of 32 input channels.  Per chunk the input tile
// (rows (TH-1)*S+KH, cols 15*S+KW, 32 channels) is staged once into LDS with
// the input transform applied (lrelu / ConvFFN2 gate) and converted to the
// compute type; weights are staged per kernel row (KW taps x BN x 32).  Every
// (dy, dx) tap then reuses the same LDS image: the LDS-staged im2col of the
// design.  bf16 mode issues v_mfma_f32_16x16x32_bf16 with an XOR-swizzled LDS
// image (16-byte slots, conflict-free ds_read_b128 lane groups for aligned
// rows); f32 mode issues v_mfma_f32_16x16x4_f32 (exact f32 fma chain) from a
// padded image.  The epilogue fuses bias, activation, up to two residual adds,
// a per-channel scale and pixel-shuffle, in the order the reference applies
// them (see dcvc_conv_args in include/dcvc_hip.h).
#include "common.h"

#include <cstring>

namespace {

constexpr int kChunk = 32;  // input channels per K chunk
__constant__ int kSwz[4] = {0, 2, 3, 1};

struct ConvP {
  const void *x;
  int H, W, xcs, xco;
  const void *w;
  const float *bias;
  void *y;
  int Ho, Wo, ycs, yco;  // conv output size (before shuffle)
  int cin, cout, cinp;
  int kh, kw, s, pad;
  int in_op;
  float in_slope;
  int act;
  float slope;
  int shuffle;
  const float *scale;
  const void *res;
  int rcs, rco;
  const void *res2;
  int r2cs, r2co;
  int Wout;  // width of y buffer (after shuffle)
  int tiles_x, tiles_y;
};

// LDS image helpers ---------------------------------------------------------
// bf16: a "row" is 32 channels = 64 B = 4 slots of 16 B; slot is swizzled.
__device__ __forceinline__ int swz_off_bf16(int row, int slot) {
  return row * 32 + ((slot ^ kSwz[(row >> 2) & 3]) << 3);  // in bf16 elements
}
// f32: a row is 32 floats padded to 33.
__device__ __forceinline__ int off_f32(int row, int k) { return row * 33 + k; }

template <typename TIN>
__device__ __forceinline__ float load_in(const ConvP &p, int gy, int gx, int c) {
  const int64_t base = ((int64_t)gy * p.W + gx) * p.xcs + p.xco;
  float v = ld<TIN>(p.x, base + c);
  if (p.in_op == DCVC_IN_LRELU) {
    v = v >= 0.f ? v : v * p.in_slope;
  } else if (p.in_op == DCVC_IN_GATE) {
    float g = ld<TIN>(p.x, base + c + p.cin);
    g = g >= 0.f ? g : g * p.in_slope;
    v = v * g;
  }
  return v;
}

template <typename TIN, bool F32, int TH>
__device__ __forceinline__ void stage_input(const ConvP &p, void *lds_in, int ch0,
                                            int iy0, int ix0, int IH, int IW,
                                            int IWp) {
  // 8 channels per work item
  const int items = IH * IW * 4;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int slot = it & 3;
    const int pix = it >> 2;
    const int iy = pix / IW, ix = pix - iy * IW;
    const int gy = iy0 + iy, gx = ix0 + ix;
    float v[8];
    const bool inb = gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = ch0 + slot * 8 + j;
      v[j] = (inb && c < p.cin) ? load_in<TIN>(p, gy, gx, c) : 0.f;
    }
    const int row = iy * IWp + ix;
    if constexpr (F32) {
      float *L = reinterpret_cast<float *>(lds_in);
#pragma unroll
      for (int j = 0; j < 8; ++j) L[off_f32(row, slot * 8 + j)] = v[j];
    } else {
      u16x8 pk;
#pragma unroll
      for (int j = 0; j < 8; ++j) pk[j] = f2bf(v[j]);
      *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(lds_in) + swz_off_bf16(row, slot)) = pk;
    }
  }
}

template <bool F32, int BN>
__device__ __forceinline__ void stage_weights(const ConvP &p, void *lds_w, int n0,
                                              int chunk, int dy) {
  const int items = p.kw * BN * 4;  // 8-channel pieces
  for (int it = threadIdx.x; it < items; it += 256) {
    const int slot = it & 3;
    const int rr = it >> 2;  // rr = dx * BN + nn
    const int dx = rr / BN, nn = rr - dx * BN;
    const int n = n0 + nn;
    const int64_t src = (((int64_t)n * p.kh + dy) * p.kw + dx) * p.cinp + chunk * kChunk + slot * 8;
    if constexpr (F32) {
      float *L = reinterpret_cast<float *>(lds_w);
      const float *W = reinterpret_cast<const float *>(p.w);
      if (n < p.cout) {
        const float4 a = *reinterpret_cast<const float4 *>(W + src);
        const float4 b = *reinterpret_cast<const float4 *>(W + src + 4);
        float *d = L + off_f32(rr, slot * 8);
        d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
        d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
      } else {
        float *d = L + off_f32(rr, slot * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = 0.f;
      }
    } else {
      u16x8 v;
      if (n < p.cout) {
        v = *reinterpret_cast<const u16x8 *>(reinterpret_cast<const uint16_t *>(p.w) + src);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0;
      }
      *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(lds_w) + swz_off_bf16(rr, slot)) = v;
    }
  }
}

template <typename TIN, typename TOUT, bool F32, int BN, int TH>
__global__ void __launch_bounds__(256) conv_kernel(ConvP p) {
  constexpr int RW = TH / 4;   // output rows per wave
  constexpr int NT = BN / 16;  // n tiles per wave
  extern __shared__ __align__(16) unsigned char smem[];

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  int b = blockIdx.x;
  const int tx = b % p.tiles_x;
  b /= p.tiles_x;
  const int ty = b % p.tiles_y;
  const int tn = b / p.tiles_y;
  const int ox0 = tx * 16, oy0 = ty * TH, n0 = tn * BN;

  const int S = p.s;
  const int IH = (TH - 1) * S + p.kh;
  const int IW = 15 * S + p.kw;
  const int IWp = (IW + 3) & ~3;
  const int in_elems = IH * IWp * (F32 ? 33 : 32);
  void *lds_in = smem;
  void *lds_w = smem + ((in_elems * (F32 ? 4 : 2) + 15) & ~15);

  f32x4 acc[RW][NT];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = p.cinp / kChunk;
  const int iy0 = oy0 * S - p.pad, ix0 = ox0 * S - p.pad;
  const int col = lane & 15, hi = lane >> 4;

  for (int ch = 0; ch < nchunks; ++ch) {
    __syncthreads();
    stage_input<TIN, F32, TH>(p, lds_in, ch * kChunk, iy0, ix0, IH, IW, IWp);
    for (int dy = 0; dy < p.kh; ++dy) {
      __syncthreads();
      stage_weights<F32, BN>(p, lds_w, n0, ch, dy);
      __syncthreads();
      for (int dx = 0; dx < p.kw; ++dx) {
        if constexpr (F32) {
          const float *Li = reinterpret_cast<const float *>(lds_in);
          const float *Lw = reinterpret_cast<const float *>(lds_w);
#pragma unroll
          for (int s4 = 0; s4 < 8; ++s4) {
            const int k = s4 * 4 + hi;
            float a[NT], bb[RW];
#pragma unroll
            for (int j = 0; j < NT; ++j) a[j] = Lw[off_f32(dx * BN + j * 16 + col, k)];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
              const int row = ((wave * RW + r) * S + dy) * IWp + col * S + dx;
              bb[r] = Li[off_f32(row, k)];
            }
#pragma unroll
            for (int r = 0; r < RW; ++r)
#pragma unroll
              for (int j = 0; j < NT; ++j)
                acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], bb[r], acc[r][j], 0, 0, 0);
          }
        } else {
          const uint16_t *Li = reinterpret_cast<const uint16_t *>(lds_in);
          const uint16_t *Lw = reinterpret_cast<const uint16_t *>(lds_w);
          bf16x8 a[NT], bb[RW];
#pragma unroll
          for (int j = 0; j < NT; ++j)
            a[j] = *reinterpret_cast<const bf16x8 *>(Lw + swz_off_bf16(dx * BN + j * 16 + col, hi));
#pragma unroll
          for (int r = 0; r < RW; ++r) {
            const int row = ((wave * RW + r) * S + dy) * IWp + col * S + dx;
            bb[r] = *reinterpret_cast<const bf16x8 *>(Li + swz_off_bf16(row, hi));
          }
#pragma unroll
          for (int r = 0; r < RW; ++r)
#pragma unroll
            for (int j = 0; j < NT; ++j)
              acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], bb[r], acc[r][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: lane owns pixel (oy, ox) and channels n..n+3 per tile
  const int ox = ox0 + col;
  if (ox >= p.Wo) return;
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int oy = oy0 + wave * RW + r;
    if (oy >= p.Ho) continue;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + j * 16 + hi * 4 + i;
        if (n >= p.cout) continue;
        float v = acc[r][j][i];
        if (p.bias) v += p.bias[n];
        v = apply_act(p.act, v, p.slope);
        int c = n, yy = oy, xx = ox;
        if (p.shuffle) {
          c = n >> 2;
          yy = oy * 2 + ((n >> 1) & 1);
          xx = ox * 2 + (n & 1);
        }
        const int64_t pix = (int64_t)yy * p.Wout + xx;
        if (p.res) v = ld<TOUT>(p.res, pix * p.rcs + p.rco + c) + v;
        if (p.res2) v = ld<TOUT>(p.res2, pix * p.r2cs + p.r2co + c) + v;
        if (p.scale) v = v * p.scale[c];
        st<TOUT>(p.y, pix * p.ycs + p.yco + c, v);
      }
    }
  }
}

template <typename TIN, typename TOUT, bool F32, int BN, int TH>
int launch(const ConvP &p0, hipStream_t st) {
  ConvP p = p0;
  p.tiles_x = (p.Wo + 15) / 16;
  p.tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles_n = (p.cout + BN - 1) / BN;
  const int IH = (TH - 1) * p.s + p.kh;
  const int IW = 15 * p.s + p.kw;
  const int IWp = (IW + 3) & ~3;
  const size_t in_bytes = (size_t)IH * IWp * (F32 ? 33 * 4 : 32 * 2);
  const size_t w_bytes = (size_t)p.kw * BN * (F32 ? 33 * 4 : 32 * 2);
  const size_t lds = ((in_bytes + 15) & ~(size_t)15) + w_bytes;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  const int64_t blocks = (int64_t)p.tiles_x * p.tiles_y * tiles_n;
  if (blocks <= 0) return DCVC_HIP_OK;
  if (blocks > 0x7fffffff) return DCVC_HIP_EINVAL;
  auto kern = conv_kernel<TIN, TOUT, F32, BN, TH>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

template <typename TIN, typename TOUT, bool F32>
int pick_bn(const ConvP &p, hipStream_t st) {
  const bool strided = p.s > 1;
  if (p.cout <= 16)
    return strided ? launch<TIN, TOUT, F32, 16, 8>(p, st) : launch<TIN, TOUT, F32, 16, 16>(p, st);
  if (p.cout <= 32)
    return strided ? launch<TIN, TOUT, F32, 32, 8>(p, st) : launch<TIN, TOUT, F32, 32, 16>(p, st);
  return strided ? launch<TIN, TOUT, F32, 64, 8>(p, st) : launch<TIN, TOUT, F32, 64, 16>(p, st);
}

bool valid_view(const dcvc_tensor &t) {
  return t.ptr && t.H > 0 && t.W > 0 && t.C > 0 && t.coff >= 0 && t.coff + t.C <= t.cstride &&
         (t.dtype == DCVC_F32 || t.dtype == DCVC_BF16);
}

}  // namespace

extern "C" int64_t dcvc_conv_pack_weights(const float *w, int cout, int cin, int kh, int kw,
                                          int compute, void *out) {
  if (!w || !out || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return DCVC_HIP_EINVAL;
  const int cinp = (cin + kChunk - 1) / kChunk * kChunk;
  const int64_t total = (int64_t)cout * kh * kw * cinp;
  for (int n = 0; n < cout; ++n)
    for (int y = 0; y < kh; ++y)
      for (int x = 0; x < kw; ++x)
        for (int c = 0; c < cinp; ++c) {
          const float v = c < cin ? w[(((int64_t)n * cin + c) * kh + y) * kw + x] : 0.f;
          const int64_t o = (((int64_t)n * kh + y) * kw + x) * cinp + c;
          if (compute == DCVC_F32) {
            reinterpret_cast<float *>(out)[o] = v;
          } else {
            // host round-to-nearest-even f32 -> bf16
            uint32_t u;
            std::memcpy(&u, &v, 4);
            uint32_t r = ((u >> 16) & 1u) + 0x7fffu;
            uint16_t h = (uint16_t)((u + r) >> 16);
            if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) h = (uint16_t)((u >> 16) | 0x40);
            reinterpret_cast<uint16_t *>(out)[o] = h;
          }
        }
  return total;
}

extern "C" int dcvc_conv2d(const dcvc_conv_args *a, void *stream) {
  if (!a || !a->w || !valid_view(a->x) || !valid_view(a->y)) return DCVC_HIP_EINVAL;
  if (a->x.C != (a->in_op == DCVC_IN_GATE ? 2 * a->cin : a->cin)) return DCVC_HIP_EINVAL;
  if (a->stride < 1 || a->kh < 1 || a->kw < 1 || a->kh > 7 || a->kw > 7) return DCVC_HIP_EINVAL;
  ConvP p{};
  p.x = a->x.ptr;
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = a->w;
  p.bias = a->bias;
  p.y = a->y.ptr;
  p.Ho = (a->x.H + 2 * a->pad - a->kh) / a->stride + 1;
  p.Wo = (a->x.W + 2 * a->pad - a->kw) / a->stride + 1;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.cinp = (a->cin + kChunk - 1) / kChunk * kChunk;
  p.kh = a->kh;
  p.kw = a->kw;
  p.s = a->stride;
  p.pad = a->pad;
  p.in_op = a->in_op;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.shuffle = a->shuffle;
  p.scale = a->scale;
  const int f = a->shuffle ? 2 : 1;
  const int cy = a->shuffle ? a->cout / 4 : a->cout;
  if (a->shuffle && (a->cout % 4)) return DCVC_HIP_EINVAL;
  if (a->y.H != p.Ho * f || a->y.W != p.Wo * f || a->y.C != cy) return DCVC_HIP_EINVAL;
  p.Wout = a->y.W;
  if (a->res.ptr) {
    if (!valid_view(a->res) || a->res.dtype != a->y.dtype || a->res.H != a->y.H ||
        a->res.W != a->y.W || a->res.C != cy)
      return DCVC_HIP_EINVAL;
    p.res = a->res.ptr;
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
  }
  if (a->res2.ptr) {
    if (!valid_view(a->res2) || a->res2.dtype != a->y.dtype || a->res2.H != a->y.H ||
        a->res2.W != a->y.W || a->res2.C != cy)
      return DCVC_HIP_EINVAL;
    p.res2 = a->res2.ptr;
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool xin32 = a->x.dtype == DCVC_F32, yout32 = a->y.dtype == DCVC_F32;
  if (a->compute == DCVC_F32) {
    if (!xin32 || !yout32) return DCVC_HIP_EUNSUPPORTED;
    return pick_bn<float, float, true>(p, st);
  }
  if (xin32 && yout32) return pick_bn<float, float, false>(p, st);
  if (xin32 && !yout32) return pick_bn<float, uint16_t, false>(p, st);
  if (!xin32 && yout32) return pick_bn<uint16_t, float, false>(p, st);
  return pick_bn<uint16_t, uint16_t, false>(p, st);
}
