// Fused ConvFFN in split-fp16 arithmetic (Precision.split()):
//   out = scale * (x + lrelu(ffn2(lrelu(ffn1(x) + b1)) + b2))
// DCVC-DC/src/models/layers.py:166-179 (ConvFFN: conv 1x1 C -> 4C, LeakyReLU,
// conv 1x1 4C -> C, LeakyReLU, + x), as the DepthConvBlocks of the UNets,
// context refinement and reconstruction use it.  Unfused, the 4C-wide hidden
// map makes a round trip through HBM in fp32 (32 C bytes per pixel against
// the 8 C of input and output).  Here it never leaves the registers.
//
// Register-resident design (round 5).  Every product is three f16 MFMAs
// (x * w ~ xh*wh + 2^-11 (xh*wl + xl*wh), sconv.hip's split).  A wave owns
// NP tiles of 16 pixels:
//   * its input, 32 channels a K chunk, is loaded straight into the lanes
//     that hold it as the MFMA B operand (lane (col, q): pixel col, channels
//     32 kc + 8 q .. + 7) and split there, one tile ahead;
//   * the hidden layer is computed 32 channels (one "slice") at a time: two
//     16-row MFMA tiles of ffn1, whose accumulator lanes (col, q) hold hidden
//     channels 4 q .. + 3 and 16 + 4 q .. + 3 of pixel col.  Bias, LeakyReLU
//     and the split turn those eight values into the lane's B operand of
//     ffn2 directly: ffn2's weights are packed with their K order permuted to
//     match (dcvc_ffn_pack_weights: position 8 q + m of a slice is hidden
//     channel 4 q + m, m < 4, or 16 + 4 q + m - 4), so no hidden value goes
//     through LDS and no barrier separates the layers;
//   * ffn2 accumulates over all slices in two fp32 accumulators (hi*hi and
//     the cross terms), combined once in the epilogue;
//   * the weights are the only LDS traffic: all slices resident for the
//     launch (C <= 64: 32 to 128 KB), or streamed slice by slice by LDS-DMA
//     through NBUF buffers (C = 128: 32 KB a slice), shared by the waves.
// The epilogue adds b2, the activation, the residual (the fp32 input,
// re-read from L2) and the scale in the reference's order.
#include "common.h"
#include "split.h"

#include <type_traits>
#include <utility>

namespace {

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

template <int C, int NW, int NP, int NBUF>
struct FG {
  static constexpr int NT_ = NW * 64;
  static constexpr int KC1 = (C + 31) / 32;          // K chunks of ffn1 (C padded to 32)
  static constexpr int C16 = (C + 15) / 16 * 16;     // ffn2 rows
  static constexpr int NT = C16 / 16;                // ffn2 n-tiles
  static constexpr int NS = 4 * C / 32;              // hidden slices of 32
  static constexpr int TP = NW * NP * 16;            // pixels per tile
  // LDS images in halves; each row 32 halves (4 swizzled 16-byte slots)
  static constexpr int W1 = KC1 * 32 * 32;           // ffn1 slice, hi or lo: [kc][h][32]
  static constexpr int W2 = C16 * 32;                // ffn2 slice, hi or lo: [n][32] (K permuted)
  static constexpr int SLICE = 2 * W1 + 2 * W2;      // halves per packed slice
  static constexpr bool RES = NBUF == 0;             // every slice resident
  static constexpr int NB = RES ? NS : NBUF;
  static constexpr size_t OC = (size_t)NB * SLICE * 2;   // b1 [4C] | b2 [C] | scale [C]
  static constexpr size_t LDS = OC + (size_t)6 * C * 4;
  static constexpr int NDMA = SLICE * 2 / 1024;      // 1-KiB LDS-DMA pieces per slice
  static constexpr int NDW = NDMA / NW;              // ... per wave (streamed: exact)
  static_assert(RES || NDMA % NW == 0, "streamed DMA pieces per slice must divide over the waves");
  static constexpr int PFN = 2 * NP * KC1;           // input loads per lane per tile
};

__device__ __forceinline__ float lrelu(float v, float s) { return fmaxf(v, v * s); }

template <typename F, int... I>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}

template <int C, int NW, int NP, int NBUF>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4)))
sffn_kernel(FP p) {
  SplitRange rg(p.ovf);
  typedef FG<C, NW, NP, NBUF> G_;
  constexpr int KC1 = G_::KC1, NT = G_::NT, NS = G_::NS, TP = G_::TP, W1 = G_::W1, W2 = G_::W2;
  constexpr int SLICE = G_::SLICE, NB = G_::NB, NDW = G_::NDW, NTH = G_::NT_;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *const Wb = reinterpret_cast<uint16_t *>(smem);
  float *const Lb1 = reinterpret_cast<float *>(smem + G_::OC), *const Lb2 = Lb1 + 4 * C, *const Lsc = Lb2 + C;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int col = lane & 15, q = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);   // consecutive tiles per XCD
  if (g >= p.ntiles) return;

  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
  // slice s -> buffer b: NDW 1-KiB pieces per wave (a linear copy of the packed image)
  auto issue_w = [&](int s, int b) {
#pragma unroll
    for (int d = 0; d < NDW; ++d) {
      const int i = wave + NW * d;
#ifdef __HIP_DEVICE_COMPILE__
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)(Wb + (size_t)b * SLICE + i * 512),
                                               16, lane * 16, (int)(((int64_t)s * SLICE + i * 512) * 2), 0, 0);
#endif
    }
  };
  // ---- input: lane (col, q) of pixel tile j holds channels 32 kc + 8 q .. + 7
  // of pixel 16 (NP wave + j) + col (zeros past C and past the map)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(p.x), (short)0, (int)((int64_t)p.npix * p.xcs * 4 < 0x7fff0000 ? (int64_t)p.npix * p.xcs * 4
                                                                                          : 0x7fff0000), 0x00020000);
  float pf[NP][KC1][8];
  auto prefetch = [&](int t) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int gp = t * TP + (wave * NP + j) * 16 + col;
#pragma unroll
      for (int kc = 0; kc < KC1; ++kc) {
        const int ch = kc * 32 + q * 8;
        const int o = (gp < p.npix && ch < C) ? (gp * p.xcs + p.xco + ch) * 4 : 0x7fffffe0;
        const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
        const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pf[j][kc][e] = a[e];
          pf[j][kc][4 + e] = b[e];
        }
      }
    }
  };

  for (int i = tid; i < 6 * C; i += NTH)
    Lb1[i] = i < 4 * C ? p.b1[i] : i < 5 * C ? p.b2[i - 4 * C] : (p.scale ? p.scale[i - 5 * C] : 1.f);
  if constexpr (G_::RES) {
    const __amdgpu_buffer_rsrc_t wr0 = wr;
    for (int i = wave; i < NS * G_::NDMA; i += NW) {
#ifdef __HIP_DEVICE_COMPILE__
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr0, (__attribute__((address_space(3))) void *)(Wb + (size_t)i * 512), 16,
                                               lane * 16, i * 1024, 0, 0);
#endif
    }
  } else {
    issue_w(0, 0);
    issue_w(1, 1);
  }
  prefetch(g);
  if constexpr (G_::RES) {
    wait_vm_lgkm();
    __syncthreads();
  }
  const int aw = swz(col, q);   // lane offset of the A fragments (row col of a 16-row tile, slot q)
  // ffn1 of slice s into hh[j][h][0: hi*hi, 1: cross terms]
  auto ffn1 = [&](auto &hh, const uint16_t *W1h, const f16x8 (&xh)[NP][KC1], const f16x8 (&xl)[NP][KC1]) {
    const uint16_t *W1l = W1h + W1;
#pragma unroll
    for (int j = 0; j < NP; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        hh[j][h][0] = f32x4{0.f, 0.f, 0.f, 0.f};
        hh[j][h][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int kc = 0; kc < KC1; ++kc)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int oa = aw + (kc * 32 + h * 16) * 32;
        const f16x8 ah = *reinterpret_cast<const f16x8 *>(W1h + oa);
        const f16x8 al = *reinterpret_cast<const f16x8 *>(W1l + oa);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          hh[j][h][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, xh[j][kc], hh[j][h][0], 0, 0, 0);
          hh[j][h][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, xl[j][kc], hh[j][h][1], 0, 0, 0);
          hh[j][h][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, xh[j][kc], hh[j][h][1], 0, 0, 0);
        }
      }
  };
  // h = lrelu(ffn1 + b1) of hidden channels 32 s + {4 q + e, 16 + 4 q + e},
  // split into the lane's ffn2 B operand (K order 8 q + m)
  auto act = [&](const auto &hh, int s, f16x8 (&hb)[NP], f16x8 (&hl)[NP]) {
    const float4 ba = *reinterpret_cast<const float4 *>(Lb1 + s * 32 + 4 * q);
    const float4 bb = *reinterpret_cast<const float4 *>(Lb1 + s * 32 + 16 + 4 * q);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      float v[8];
      v[0] = lrelu((hh[j][0][0][0] + hh[j][0][1][0] * kLoInv) + ba.x, p.slope);
      v[1] = lrelu((hh[j][0][0][1] + hh[j][0][1][1] * kLoInv) + ba.y, p.slope);
      v[2] = lrelu((hh[j][0][0][2] + hh[j][0][1][2] * kLoInv) + ba.z, p.slope);
      v[3] = lrelu((hh[j][0][0][3] + hh[j][0][1][3] * kLoInv) + ba.w, p.slope);
      v[4] = lrelu((hh[j][1][0][0] + hh[j][1][1][0] * kLoInv) + bb.x, p.slope);
      v[5] = lrelu((hh[j][1][0][1] + hh[j][1][1][1] * kLoInv) + bb.y, p.slope);
      v[6] = lrelu((hh[j][1][0][2] + hh[j][1][1][2] * kLoInv) + bb.z, p.slope);
      v[7] = lrelu((hh[j][1][0][3] + hh[j][1][1][3] * kLoInv) + bb.w, p.slope);
      u32x4_t h, l;
      rg.add8(v);
      split8(v, h, l);
      hb[j] = __builtin_bit_cast(f16x8, h);
      hl[j] = __builtin_bit_cast(f16x8, l);
    }
  };
  // streamed weights: barrier B_s before ffn1 of tile slice s reads buffer
  // s % NB.  Program order per wave: B_s, ffn1(s), act(s - 1), ffn2(s - 1),
  // B_(s+1), ...: at B_s every wave is done with slice s - 2's buffer, so
  // the DMA of slice s + 2 (into that buffer) is issued right after it, and
  // B_s waits for slice s's DMA (issued at B_(s-2)): younger than it are
  // slice s + 1's DMA and, at B_1 and B_2, the next tile's input prefetch
  // (issued after B_0's DMA; on the last tile too, all of it out of range,
  // so that the counts are fixed).  pf: std::true_type at B_1 and B_2
  static_assert(G_::RES || (NS % NB == 0 && NB == 4), "streamed: four buffers, slices a multiple of them");
  auto barrier_w = [&](int s, auto pf) {
    if constexpr (!G_::RES) {
      if constexpr (decltype(pf)::value) wait_vm_n_lgkm<NDW + G_::PFN>();
      else wait_vm_n_lgkm<NDW>();
      raw_barrier();
      issue_w((s + 2) % NS, (s + 2) % NB);
    }
  };
  auto wslice = [&](int s) -> const uint16_t * { return Wb + (size_t)(G_::RES ? s : s % NB) * SLICE; };
  for (int t = g; t < p.ntiles; t += G) {
    // this tile's input: split into the B operands (waits for the prefetch)
    f16x8 xh[NP][KC1], xl[NP][KC1];
#pragma unroll
    for (int j = 0; j < NP; ++j)
#pragma unroll
      for (int kc = 0; kc < KC1; ++kc) {
        u32x4_t h, l;
        rg.add8(pf[j][kc]);
        split8(pf[j][kc], h, l);
        xh[j][kc] = __builtin_bit_cast(f16x8, h);
        xl[j][kc] = __builtin_bit_cast(f16x8, l);
      }
    f32x4 am[NP][NT], ac[NP][NT];
#pragma unroll
    for (int j = 0; j < NP; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        am[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        ac[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    const bool more = t + G < p.ntiles;
    // software pipeline over the slices: ffn1 of slice s + 1 (MFMAs) is
    // issued before the activation of slice s (VALU), whose results ffn2 of
    // slice s then consumes, so the VALU runs under the matrix pipe's work
    f32x4 hA[NP][2][2], hB[NP][2][2];
    // the next tile's input: loaded under this tile's work, right after B_0;
    // where the registers are short (C = 64, resident weights: no DMA count
    // to keep) after the tile's last ffn1 instead, into the registers of the
    // input operands, dead by then
    constexpr bool LATE_PF = G_::RES && C == 64;
    barrier_w(0, std::false_type{});
    if constexpr (!G_::RES) prefetch(t + G);
    else if (!LATE_PF && more) prefetch(t + G);
    ffn1(hA, wslice(0), xh, xl);
    // ffn2 of slice s from the activation of hh
    auto ffn2 = [&](const auto &hh, int s) {
      f16x8 hb[NP], hl[NP];
      act(hh, s, hb, hl);
      const uint16_t *W2h = wslice(s) + 2 * W1, *W2l = W2h + W2;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int oa = aw + n * 16 * 32;
        const f16x8 ah = *reinterpret_cast<const f16x8 *>(W2h + oa);
        const f16x8 al = *reinterpret_cast<const f16x8 *>(W2l + oa);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          am[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, hb[j], am[j][n], 0, 0, 0);
          ac[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, hl[j], ac[j][n], 0, 0, 0);
          ac[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, hb[j], ac[j][n], 0, 0, 0);
        }
      }
    };
    static_assert(NS % 2 == 0 && NS >= 4, "slices come in pairs, at least two");
    // two slices an iteration (hA, hB alternate), not unrolled further: the
    // registers stay those of one pair.  The first pair is peeled (its
    // barriers count the prefetch), so no barrier's vmcnt depends on a
    // runtime condition: the build-time check (scripts/check_xconv_vmcnt.py)
    // walks every path to each barrier
    barrier_w(1, std::true_type{});
    ffn1(hB, wslice(1), xh, xl);
    ffn2(hA, 0);
    barrier_w(2, std::true_type{});
    ffn1(hA, wslice(2), xh, xl);
    ffn2(hB, 1);
#pragma unroll 1
    for (int s = 2; s < NS; s += 2) {
      barrier_w(s + 1, std::false_type{});
      ffn1(hB, wslice(s + 1), xh, xl);
      if (LATE_PF && s + 2 >= NS && more) prefetch(t + G);
      ffn2(hA, s);
      if (s + 2 < NS) {
        barrier_w(s + 2, std::false_type{});
        ffn1(hA, wslice(s + 2), xh, xl);
      }
      ffn2(hB, s + 1);
    }
    // ---- epilogue: out = scale * (x + lrelu(acc + b2)), 4 channels per lane
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int gp = t * TP + (wave * NP + j) * 16 + col;
      if (gp < p.npix) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int c = n * 16 + q * 4;
          if (c >= C) continue;
          const f32x4 xv = *reinterpret_cast<const f32x4 *>(p.x + (int64_t)gp * p.xcs + p.xco + c);
          const float4 b2 = *reinterpret_cast<const float4 *>(Lb2 + c);
          f32x4 v;
          v[0] = xv[0] + lrelu((am[j][n][0] + ac[j][n][0] * kLoInv) + b2.x, p.slope);
          v[1] = xv[1] + lrelu((am[j][n][1] + ac[j][n][1] * kLoInv) + b2.y, p.slope);
          v[2] = xv[2] + lrelu((am[j][n][2] + ac[j][n][2] * kLoInv) + b2.z, p.slope);
          v[3] = xv[3] + lrelu((am[j][n][3] + ac[j][n][3] * kLoInv) + b2.w, p.slope);
          if (p.scale) {
            const float4 sc = *reinterpret_cast<const float4 *>(Lsc + c);
            v[0] *= sc.x;
            v[1] *= sc.y;
            v[2] *= sc.z;
            v[3] *= sc.w;
          }
          *reinterpret_cast<f32x4 *>(p.y + (int64_t)gp * p.ycs + p.yco + c) = v;
        }
      }
    }
  }
  wait_vm_lgkm();   // no LDS-DMA in flight at exit
}

int g_cus = 0;
int g_c128 = 1;   // dcvc_set_option("sffn128", 0): C = 128 feature maps on 4 waves of two pixel tiles (A/B)

template <int C, int NW, int NP, int NBUF>
int run(FP p, hipStream_t st) {
  typedef FG<C, NW, NP, NBUF> G_;
  if (p.hidden != 4 * C) return DCVC_HIP_EUNSUPPORTED;
  const size_t lds = G_::LDS;
  static_assert(G_::LDS <= 160 * 1024, "LDS");
  p.nslices = G_::NS;
  p.ntiles = (p.npix + G_::TP - 1) / G_::TP;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  int G = g_cus;
  if (G > p.ntiles) G = p.ntiles;
  auto kern = sffn_kernel<C, NW, NP, NBUF>;
  dcvc_note_kernel("sffn_kernel<%d, %d, %d, %d>@%lld", C, NW, NP, NBUF, (long long)G * NW * 64);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(NW * 64), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

extern "C" int dcvc_internal_lffn_supported(int c, int hidden);
extern "C" int64_t dcvc_internal_lffn_pack(const float *w1, const float *w2, int c, int hidden, void *out);
extern "C" int dcvc_internal_lffn(const dcvc_ffn_args *a, void *stream);

// Packed slices of one ConvFFN: w1 [hidden][c] (conv.0, fp32 host), w2
// [c][hidden] (conv.2); each slice of 32 hidden channels is the LDS image
// sffn_kernel reads (hi and lo of ffn1 as [kc][h][32], then of ffn2 as
// [n][32] with the slice's K order permuted, 16-byte slots swizzled by
// swz()).  out NULL: size query.
extern "C" int64_t dcvc_ffn_pack_weights(const float *w1, const float *w2, int c, int hidden, void *out) {
  if (!w1 || !w2 || c <= 0 || hidden <= 0) return DCVC_HIP_EINVAL;
  if (out && (!host_split_range_ok(w1, (int64_t)hidden * c) || !host_split_range_ok(w2, (int64_t)c * hidden)))
    return DCVC_HIP_EINVAL;
  // the latent widths: MFMA fragments for slffn.hip
  if (dcvc_internal_lffn_supported(c, hidden)) return dcvc_internal_lffn_pack(w1, w2, c, hidden, out);
  constexpr int HS = 32;
  if (hidden % HS) return DCVC_HIP_EINVAL;
  const int kc1 = (c + 31) / 32, c16 = (c + 15) / 16 * 16;
  const int64_t w1n = (int64_t)kc1 * HS * 32, w2n = (int64_t)c16 * 32, slice = 2 * w1n + 2 * w2n;
  const int ns = hidden / HS;
  if (!out) return slice * ns;
  uint16_t *o = reinterpret_cast<uint16_t *>(out);
  // physical position of logical (row, k) in a swizzled image of 32-half rows
  auto at = [](int row, int k) {
    const int x = (0x1320 >> (((row >> 2) & 3) << 2)) & 3;
    return (int64_t)row * 32 + ((((k >> 3) ^ x) & 3) << 3) + (k & 7);
  };
  // ffn2's K position 8 q + m of a slice holds hidden channel 4 q + m (m < 4)
  // or 16 + 4 q + m - 4: the order ffn1's accumulators leave them in
  auto perm = [](int k) { const int q = k >> 3, m = k & 7; return m < 4 ? 4 * q + m : 16 + 4 * q + m - 4; };
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
    for (int n = 0; n < c16; ++n)
      for (int k = 0; k < 32; ++k) {
        const float v = n < c ? w2[(int64_t)n * hidden + s * HS + perm(k)] : 0.f;
        const int64_t q = at(n, k);
        host_split(v, s2[q], s2[w2n + q]);
      }
  }
  return slice * ns;
}

extern "C" void dcvc_internal_sffn128(int v) { g_c128 = v; }

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
  // (the kernel clamps the input's buffer record to 0x7fff0000 bytes)
  if ((int64_t)p.npix * p.xcs * 4 >= 0x7fff0000) return DCVC_HIP_EUNSUPPORTED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // 8 waves (two per SIMD) of two 16-pixel tiles with every slice resident
  // (C <= 64); C = 128 streams its 16 slices through four 32 KiB buffers, to
  // 8 waves of one pixel tile on feature maps, and to 4 waves of 512
  // registers (one per SIMD) of one tile where more waves would leave CUs
  // idle (the 68 x 120 latent-rate blocks)
  const int ntiles2 = (p.npix + 4 * 2 * 16 - 1) / (4 * 2 * 16);
  switch (a->c) {
    case 32: return run<32, 8, 2, 0>(p, st);
    case 48: return run<48, 8, 2, 0>(p, st);
    case 64: return run<64, 8, 2, 0>(p, st);
    case 128:
      // feature maps: 8 waves (two per SIMD, 232 VGPRs, no AGPR copies) of one
      // pixel tile: 128 -> 512 -> 128 at 272 x 480 154 -> 126 us against 4
      // waves of two tiles (256 VGPRs + 231 AGPRs, accumulators copied
      // between the files), profiles/r05t_ffn128_ab.jsonl
      if (ntiles2 < 2 * 256) return run<128, 4, 1, 4>(p, st);
      return g_c128 ? run<128, 8, 1, 4>(p, st) : run<128, 4, 2, 4>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}
