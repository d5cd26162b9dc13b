// Fused ConvFFN in split-fp16 arithmetic (Precision.split()):
//   out = scale * (x + lrelu(ffn2(lrelu(ffn1(x) + b1)) + b2))
// DCVC-DC/src/models/layers.py:166-179 (ConvFFN: conv 1x1 C -> 4C, LeakyReLU,
// conv 1x1 4C -> C, LeakyReLU, + x), as the DepthConvBlocks of the UNets,
// context refinement and reconstruction use it.  Unfused, the 4C-wide hidden
// map makes a round trip through HBM in fp32 (32 C bytes per pixel against
// the 8 C of input and output): a 48-channel block at 1080p read and wrote
// 1.6 GB for it.  Here it never leaves LDS.
//
// One 512-thread workgroup per CU walks tiles of 128 consecutive pixels of
// the (flattened) map, persistent:
//   * the tile's input (C fp32 channels) is loaded into registers one tile
//     ahead, split into (hi, lo) fp16 images in LDS when the tile starts;
//   * the hidden layer is computed in slices of HS channels: wave w owns
//     pixels [16 w, 16 w + 16) and computes its hidden slice with three f16
//     MFMAs per product (sconv.hip's split), applies bias and LeakyReLU in
//     fp32, splits the result into its own rows of the hidden image (no
//     barrier: a wave's LDS operations complete in order, wave_lds_sync keeps
//     the compiler from reordering them) and accumulates ffn2 over the slice;
//   * the weight slices are the packed LDS images (dcvc_ffn_pack_weights,
//     swizzle included) moved by LDS-DMA: all of them resident for the launch
//     when NBUF buffers hold them (C = 32, 48), else streamed through two
//     buffers one slice ahead (C = 64, 128);
//   * the epilogue adds the residual (the fp32 input, re-read from L2), the
//     bias, the activation and the scale in the reference's order and stores
//     fp32 from the accumulators.
#include "common.h"
#include "split.h"

namespace {

constexpr int kNW = 8, kNT = kNW * 64;
constexpr int TP = kNW * 16;   // pixels per tile

struct FP {
  const float *x;
  int npix, xcs, xco;          // flattened H x W map, channel view
  float *y;
  int ycs, yco;
  int c, hidden, nslices;
  const uint16_t *w;           // packed slices
  int wbytes;
  const float *b1, *b2, *scale;
  float slope;
  int ntiles;
  int *ovf;               // fp16 range guard (split.h SplitRange)
};

template <int C, int HS, int NBUF>
struct FG {
  static constexpr int KC1 = (C + 31) / 32;          // K chunks of ffn1 (C padded to 32)
  static constexpr int C16 = (C + 15) / 16 * 16;     // ffn2 rows
  static constexpr int NT = C16 / 16;                // ffn2 n-tiles
  static constexpr int NH = HS / 16;                 // ffn1 n-tiles per slice
  static constexpr int KC2 = HS / 32;                // ffn2 K chunks per slice
  // LDS images in halves; each row 32 halves (4 swizzled 16-byte slots)
  static constexpr int W1 = KC1 * HS * 32;           // ffn1 slice, hi or lo: [kc][h][32]
  static constexpr int W2 = KC2 * C16 * 32;          // ffn2 slice, hi or lo: [kc2][n][32]
  static constexpr int SLICE = 2 * W1 + 2 * W2;      // halves per packed slice
  static constexpr int XI = KC1 * TP * 32;           // input image, hi or lo: [kc][px][32]
  static constexpr int HI = KC2 * TP * 32;           // hidden image, hi or lo: [kc2][px][32]
  static constexpr size_t OX = 0, OH = OX + (size_t)2 * XI * 2, OW = OH + (size_t)2 * HI * 2;
  static constexpr size_t OC = OW + (size_t)NBUF * SLICE * 2;   // b1 [hidden] | b2 [C] | scale [C]
  static constexpr size_t LDS_BASE = OC;                          // + (hidden + 2 C) floats
  static constexpr int PP = (TP * C / 8 + kNT - 1) / kNT;   // 8-channel input pieces per thread
  static constexpr int NDMA = SLICE * 2 / 1024;              // 1-KiB LDS-DMA pieces per slice
};

__device__ __forceinline__ float lrelu(float v, float s) { return fmaxf(v, v * s); }

template <int C, int HS, int NBUF>
__global__ void __launch_bounds__(kNT) sffn_kernel(FP p) {
  SplitRange rg(p.ovf);
  typedef FG<C, HS, NBUF> G_;
  constexpr int KC1 = G_::KC1, NT = G_::NT, NH = G_::NH, KC2 = G_::KC2, PP = G_::PP;
  constexpr int W1 = G_::W1, W2 = G_::W2, SLICE = G_::SLICE, XI = G_::XI, HI = G_::HI, NDMA = G_::NDMA;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Xh = reinterpret_cast<uint16_t *>(smem + G_::OX), *Xl = Xh + XI;
  uint16_t *Hh = reinterpret_cast<uint16_t *>(smem + G_::OH), *Hl = Hh + HI;
  uint16_t *Wb = reinterpret_cast<uint16_t *>(smem + G_::OW);
  float *Lb1 = reinterpret_cast<float *>(smem + G_::OC), *Lb2 = Lb1 + p.hidden, *Lsc = Lb2 + C;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);   // consecutive tiles per XCD
  if (g >= p.ntiles) return;
  const int ns = p.nslices;
  const bool resident = ns <= NBUF;

  // ---- input pieces: piece u = (pixel, 8-channel group), 16 B x 2
  constexpr int QP = C / 8;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(p.x), (short)0, (int)((int64_t)p.npix * p.xcs * 4 < 0x7fff0000 ? (int64_t)p.npix * p.xcs * 4
                                                                                          : 0x7fff0000), 0x00020000);
  float pf[PP][8];
  auto prefetch = [&](int t) {
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * kNT;
      const int px = it / QP, q = it - px * QP;
      const int gp = t * TP + px;
      const int o = (it < TP * QP && gp < p.npix) ? (gp * p.xcs + p.xco + q * 8) * 4 : 0x7fffffe0;
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[u][j] = a[j];
        pf[u][4 + j] = b[j];
      }
    }
  };
  auto publish = [&]() {
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * kNT;
      if (it < TP * QP) {
        const int px = it / QP, q = it - px * QP;
        const int kc = q >> 2, slot = q & 3;
        u32x4_t h, l;
        rg.add8(pf[u]);
        split8(pf[u], h, l);
        const int o = swz(kc * TP + px, slot);
        *reinterpret_cast<u32x4_t *>(Xh + o) = h;
        *reinterpret_cast<u32x4_t *>(Xl + o) = l;
      }
    }
  };
  // channels [C, 32 KC1) of the input image stay zero for the launch
  if constexpr (C % 32 != 0) {
    for (int it = tid; it < TP * (KC1 * 4 - QP); it += kNT) {
      const int px = it / (KC1 * 4 - QP), slot = QP + it % (KC1 * 4 - QP);
      const int o = swz((slot >> 2) * TP + px, slot & 3);
      *reinterpret_cast<u32x4_t *>(Xh + o) = u32x4_t{0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4_t *>(Xl + o) = u32x4_t{0u, 0u, 0u, 0u};
    }
  }
  // ---- weight slice s -> buffer b (a linear copy of the packed image)
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
  auto issue_w = [&](int s, int b) {
    for (int i = wave; i < NDMA; i += kNW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (__attribute__((address_space(3))) void *)(Wb + (size_t)b * SLICE + i * 512), 16,
          (int)(((int64_t)s * SLICE + i * 512) * 2 + lane * 16), 0, 0, 0);
  };

  if (resident) {
    for (int s = 0; s < ns; ++s) issue_w(s, s);
  } else {
    issue_w(0, 0);
  }
  prefetch(g);
  for (int i = tid; i < p.hidden + 2 * C; i += kNT)
    Lb1[i] = i < p.hidden ? p.b1[i] : i < p.hidden + C ? p.b2[i - p.hidden] : (p.scale ? p.scale[i - p.hidden - C] : 1.f);
  int k = 0;   // slice stages over the launch (streamed buffers alternate)
  for (int t = g; t < p.ntiles; t += G) {
    const bool more = t + G < p.ntiles;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < ns; ++s, ++k) {
      // this slice's weights have landed (issued one slice ago, before any
      // input prefetch, so the younger prefetch loads may stay in flight; at
      // s = 0 the input pieces are needed too)
      if (s == 0) wait_vm_lgkm();
      else wait_vm_n_lgkm<2 * PP>();
      raw_barrier();    // ... for every wave; every wave is done with the previous slice's buffer
      if (s == 0) {
        publish();
        wait_lgkm();
        raw_barrier();
      }
      int b;
      if (resident) {
        b = s;
      } else {
        b = k & 1;
        if (s + 1 < ns) issue_w(s + 1, (k + 1) & 1);
        else if (more) issue_w(0, (k + 1) & 1);
      }
      if (s == 0 && more) prefetch(t + G);
      const uint16_t *W1h = Wb + (size_t)b * SLICE, *W1l = W1h + W1, *W2h = W1l + W1, *W2l = W2h + W2;
      // ffn1 slice: hidden channels [s HS, s HS + HS) of pixels 16 wave + col
      f32x4 hm[NH], hc[NH];
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        hm[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        hc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int kc = 0; kc < KC1; ++kc) {
        const int ob = swz(kc * TP + wave * 16 + col, hi);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Xh + ob);
        const f16x8 bl = *reinterpret_cast<const f16x8 *>(Xl + ob);
#pragma unroll
        for (int j = 0; j < NH; ++j) {
          const int oa = swz(kc * HS + j * 16 + col, hi);
          const f16x8 ah = *reinterpret_cast<const f16x8 *>(W1h + oa);
          const f16x8 al = *reinterpret_cast<const f16x8 *>(W1l + oa);
          hm[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, hm[j], 0, 0, 0);
          hc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, hc[j], 0, 0, 0);
          hc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, hc[j], 0, 0, 0);
        }
      }
      // h = lrelu(ffn1 + b1), split into this wave's rows of the hidden image:
      // lane (col, hi) holds hidden channels 16 j + 4 hi .. + 3 of its pixel
      wave_lds_sync();   // the previous slice's hidden-image reads (other lanes) come first
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const int hc0 = j * 16 + hi * 4;                    // channel within the slice
        const float4 bb = *reinterpret_cast<const float4 *>(Lb1 + s * HS + hc0);
        float v[4];
        v[0] = lrelu((hm[j][0] + hc[j][0] * kLoInv) + bb.x, p.slope);
        v[1] = lrelu((hm[j][1] + hc[j][1] * kLoInv) + bb.y, p.slope);
        v[2] = lrelu((hm[j][2] + hc[j][2] * kLoInv) + bb.z, p.slope);
        v[3] = lrelu((hm[j][3] + hc[j][3] * kLoInv) + bb.w, p.slope);
        rg.add4(v);
        const auto h01 = __builtin_amdgcn_cvt_pkrtz(v[0], v[1]);
        const auto h23 = __builtin_amdgcn_cvt_pkrtz(v[2], v[3]);
        const uint32_t l01 = pk(split_lo(v[0], (float)h01[0]), split_lo(v[1], (float)h01[1]));
        const uint32_t l23 = pk(split_lo(v[2], (float)h23[0]), split_lo(v[3], (float)h23[1]));
        const int kc2 = hc0 >> 5, kk = hc0 & 31;             // chunk, channel within it
        const int o = swz(kc2 * TP + wave * 16 + col, kk >> 3) + (kk & 7);
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2_t *>(Hh + o) = u32x2_t{__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23)};
        *reinterpret_cast<u32x2_t *>(Hl + o) = u32x2_t{l01, l23};
      }
      wave_lds_sync();   // the hidden image rows are written before other lanes read them
      // ffn2 partial sums over this slice
      f32x4 cm[NT], cc[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        cm[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        cc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int kc = 0; kc < KC2; ++kc) {
        const int ob = swz(kc * TP + wave * 16 + col, hi);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Hh + ob);
        const f16x8 bl = *reinterpret_cast<const f16x8 *>(Hl + ob);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int oa = swz(kc * G_::C16 + j * 16 + col, hi);
          const f16x8 ah = *reinterpret_cast<const f16x8 *>(W2h + oa);
          const f16x8 al = *reinterpret_cast<const f16x8 *>(W2l + oa);
          cm[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, cm[j], 0, 0, 0);
          cc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, cc[j], 0, 0, 0);
          cc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, cc[j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[j][e] += cm[j][e] + cc[j][e] * kLoInv;
    }
    // ---- epilogue: out = scale * (x + lrelu(acc + b2)), 4 channels per lane
    const int gp = t * TP + wave * 16 + col;
    if (gp < p.npix) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = j * 16 + hi * 4;
        if (n >= C) continue;
        const f32x4 xv = *reinterpret_cast<const f32x4 *>(p.x + (int64_t)gp * p.xcs + p.xco + n);
        const float4 bb = *reinterpret_cast<const float4 *>(Lb2 + n);
        f32x4 v;
        v[0] = xv[0] + lrelu(acc[j][0] + bb.x, p.slope);
        v[1] = xv[1] + lrelu(acc[j][1] + bb.y, p.slope);
        v[2] = xv[2] + lrelu(acc[j][2] + bb.z, p.slope);
        v[3] = xv[3] + lrelu(acc[j][3] + bb.w, p.slope);
        if (p.scale) {
          const float4 sc = *reinterpret_cast<const float4 *>(Lsc + n);
          v[0] *= sc.x;
          v[1] *= sc.y;
          v[2] *= sc.z;
          v[3] *= sc.w;
        }
        *reinterpret_cast<f32x4 *>(p.y + (int64_t)gp * p.ycs + p.yco + n) = v;
      }
    }
  }
  wait_vm_lgkm();   // no LDS-DMA in flight at exit
}

int g_cus = 0;

template <int C, int HS, int NBUF>
int run(FP p, hipStream_t st) {
  typedef FG<C, HS, NBUF> G_;
  if (p.hidden % HS) return DCVC_HIP_EUNSUPPORTED;
  const size_t lds = G_::LDS_BASE + (size_t)(p.hidden + 2 * C) * 4;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  p.nslices = p.hidden / HS;
  p.ntiles = (p.npix + TP - 1) / TP;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  int G = g_cus;
  if (G > p.ntiles) G = p.ntiles;
  auto kern = sffn_kernel<C, HS, NBUF>;
  dcvc_note_kernel("sffn_kernel<%d, %d, %d>@%lld", C, HS, NBUF, (long long)G * kNT);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(kNT), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

int hs_of(int c) { return c >= 128 ? 32 : 64; }

}  // namespace

extern "C" int dcvc_internal_lffn_supported(int c, int hidden);
extern "C" int64_t dcvc_internal_lffn_pack(const float *w1, const float *w2, int c, int hidden, void *out);
extern "C" int dcvc_internal_lffn(const dcvc_ffn_args *a, void *stream);

// Packed slices of one ConvFFN: w1 [hidden][c] (conv.0, fp32 host), w2
// [c][hidden] (conv.2); each slice of HS hidden channels is the LDS image
// sffn_kernel reads (hi and lo of ffn1 as [kc][h][32], then of ffn2 as
// [kc2][n][32], 16-byte slots swizzled by swz()).  out NULL: size query.
extern "C" int64_t dcvc_ffn_pack_weights(const float *w1, const float *w2, int c, int hidden, void *out) {
  if (!w1 || !w2 || c <= 0 || hidden <= 0) return DCVC_HIP_EINVAL;
  if (out && (!host_split_range_ok(w1, (int64_t)hidden * c) || !host_split_range_ok(w2, (int64_t)c * hidden)))
    return DCVC_HIP_EINVAL;
  // the latent widths: MFMA fragments for slffn.hip
  if (dcvc_internal_lffn_supported(c, hidden)) return dcvc_internal_lffn_pack(w1, w2, c, hidden, out);
  const int HS = hs_of(c);
  if (hidden % HS) return DCVC_HIP_EINVAL;
  const int kc1 = (c + 31) / 32, c16 = (c + 15) / 16 * 16, kc2 = HS / 32;
  const int64_t w1n = (int64_t)kc1 * HS * 32, w2n = (int64_t)kc2 * c16 * 32, slice = 2 * w1n + 2 * w2n;
  const int ns = hidden / HS;
  if (!out) return slice * ns;
  uint16_t *o = reinterpret_cast<uint16_t *>(out);
  // physical position of logical (row, k) in a swizzled image of 32-half rows
  auto at = [](int row, int k) {
    const int x = (0x1320 >> (((row >> 2) & 3) << 2)) & 3;
    return (int64_t)row * 32 + ((((k >> 3) ^ x) & 3) << 3) + (k & 7);
  };
  for (int s = 0; s < ns; ++s) {
    uint16_t *sl = o + s * slice;
    for (int kc = 0; kc < kc1; ++kc)
      for (int h = 0; h < HS; ++h)
        for (int k = 0; k < 32; ++k) {
          const int ch = kc * 32 + k;
          const float v = ch < c ? w1[(int64_t)(s * HS + h) * c + ch] : 0.f;
          const int64_t q = at(kc * HS + h, k);
          host_split(v, sl[q], sl[w1n + q]);
        }
    uint16_t *s2 = sl + 2 * w1n;
    for (int kc = 0; kc < kc2; ++kc)
      for (int n = 0; n < c16; ++n)
        for (int k = 0; k < 32; ++k) {
          const float v = n < c ? w2[(int64_t)n * hidden + s * HS + kc * 32 + k] : 0.f;
          const int64_t q = at(kc * c16 + n, k);
          host_split(v, s2[q], s2[w2n + q]);
        }
  }
  return slice * ns;
}

extern "C" int dcvc_conv_ffn(const dcvc_ffn_args *a, void *stream) {
  if (!a || !a->x.ptr || !a->y.ptr || !a->w || !a->b1 || !a->b2) return DCVC_HIP_EINVAL;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32 || a->x.C != a->c || a->y.C != a->c ||
      a->x.H != a->y.H || a->x.W != a->y.W)
    return DCVC_HIP_EINVAL;
  if (!(a->slope >= 0.f && a->slope <= 1.f)) return DCVC_HIP_EUNSUPPORTED;   // lrelu as max(v, s v)
  if (a->x.cstride % 4 || a->x.coff % 4 || a->y.cstride % 4 || a->y.coff % 4 || a->c % 8 ||
      ((uintptr_t)a->x.ptr & 15) || ((uintptr_t)a->y.ptr & 15))
    return DCVC_HIP_EUNSUPPORTED;
  if (dcvc_internal_lffn_supported(a->c, a->hidden)) return dcvc_internal_lffn(a, stream);   // slffn.hip
  FP p{};
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.npix = a->x.H * a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.c = a->c;
  p.hidden = a->hidden;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  const int64_t wb = dcvc_ffn_pack_weights(reinterpret_cast<const float *>(1), reinterpret_cast<const float *>(1),
                                           a->c, a->hidden, nullptr) * 2;
  if (wb <= 0 || wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EINVAL;
  p.wbytes = (int)wb;
  p.b1 = a->b1;
  p.b2 = a->b2;
  p.scale = a->scale;
  p.slope = a->slope;
  if ((int64_t)p.npix * p.xcs * 4 >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (a->c) {
    case 32: return run<32, 64, 2>(p, st);
    case 48: return run<48, 64, 3>(p, st);
    case 64: return run<64, 64, 2>(p, st);
    case 128: return run<128, 32, 2>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}
