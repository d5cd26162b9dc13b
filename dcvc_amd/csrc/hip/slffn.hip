// Fused latent DepthConvBlock stages in split-fp16 arithmetic (slffn_kernel:
// the ConvFFN; sldc_kernel below: the DepthConv tail).
//
// Fused ConvFFN of the latent DepthConvBlocks in split-fp16 arithmetic:
//   out = scale * (x + lrelu(ffn2(lrelu(ffn1(x) + b1)) + b2))
// DCVC-DC/src/models/layers.py:166-179 (ConvFFN, hidden = max(min(4C, 1024),
// 2C)) as the entropy model's prior fusion and spatial prior stacks run it on
// the 1/16 latent (video_model.py:288-305: C = 384, hidden 1024; the motion
// branch :250-267: C = 192, hidden 768).
//
// Why a kernel of its own: at 1080p the latent is 68 x 120 = 8160 pixels, so
// each of the two unfused 1x1 GEMMs (sgemm.hip) has only ~250 pixel x channel
// tiles, walks K = 384..1024 serially and pays a launch, a grid ramp and an
// epilogue, while the 4C-wide hidden map makes an fp32 round trip through
// memory: ~95 us per 384-channel FFN for ~13 GFLOP of f16x3 work.  Here one
// workgroup owns 32 pixels and ALL channels of the block:
//   * the tile's input (C fp32 channels) is split once into (hi, lo) fp16
//     LDS images (sconv.hip's split and swizzle);
//   * the hidden layer goes in slices of 64 channels: wave w computes hidden
//     rows [16 w, 16 w + 16) of the slice for the 32 pixels (K = C), adds
//     b1, applies the LeakyReLU in fp32, splits the result into a hidden LDS
//     image (two buffers: one barrier per slice), and every wave then
//     accumulates its C / 4 output rows over the slice (ffn2, K = 64);
//   * no LDS staging of weights: they are packed as MFMA A fragments (1 KiB
//     per 16 rows x 32 K, lane-ordered, hi and lo planes) and loaded straight
//     into registers, ffn1's of slice s + 1 during ffn2 of slice s and
//     ffn2's of slice s during ffn1 of slice s; every weight byte crosses
//     the L2 once per workgroup;
//   * the epilogue runs from the accumulators: + b2, LeakyReLU, + x (fp32,
//     re-read from L2), * scale, 16-byte stores.
// The products and the K order of both GEMMs are those of sgemm.hip (chunks
// of 32 ascending, main and correction accumulators), so the block's output
// is bit-identical to the two unfused launches.
#include "common.h"
#include "split.h"

#include <cstring>

namespace {

constexpr int kNW = 4, kNT = kNW * 64;

constexpr int HS = 64;    // hidden channels per slice (4 row blocks: one per wave)
// pixel blocks (16 pixels each) per workgroup of slffn_kernel<384>.  Every
// workgroup streams the block's whole packed weight set (3.1 MB of hi / lo
// fragments at C = 384) from L2 into registers; 4 blocks halve those L2
// bytes per pixel and the grid, but measured 100 vs 60 us (sldc 59 vs 34 us,
// profiles/r06c_latent_pb_ab.jsonl): the time follows the MFMAs of its one
// wave per SIMD, not the L2 bytes, so 2 stays.
#ifndef SLFFN_PB384
#define SLFFN_PB384 2
#endif
// the same for sldc_kernel<384> (the conv2 weights: 0.6 MB per workgroup)
#ifndef SLDC_PB384
#define SLDC_PB384 2
#endif
constexpr int kOob = 0x7fffffe0;

struct LP {
  const float *x;
  int npix, xcs, xco, xbytes;
  float *y;
  int ycs, yco, ybytes;
  const uint16_t *w1, *w2;   // packed fragments (dcvc_internal_lffn_pack)
  int w1bytes, w2bytes;
  const float *b1, *b2, *scale;
  int hidden;
  float slope;
  int *ovf;               // fp16 range guard (split.h SplitRange)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}

template <int C, int PB>
__global__ void __launch_bounds__(kNT) slffn_kernel(LP p) {
  SplitRange rg(p.ovf);
  constexpr int P = 16 * PB;        // pixels per workgroup
  constexpr int KC = C / 32;        // ffn1 K chunks
  constexpr int NTW = C / 64;       // ffn2 output row blocks per wave
  constexpr int XI = KC * P * 32;   // halves of the input image (hi or lo)
  constexpr int HI = 2 * P * 32;    // halves of one hidden image (hi or lo): 2 chunks of 32
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Xh = reinterpret_cast<uint16_t *>(smem), *Xl = Xh + XI;
  uint16_t *Hb = Xl + XI;           // [buf][hi, lo][HI]
  float *Lb1 = reinterpret_cast<float *>(Hb + 4 * HI);
  float *Lb2 = Lb1 + p.hidden, *Lsc = Lb2 + C;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int pix0 = blockIdx.x * P;
  const int KH = p.hidden / 32;     // ffn2 K chunks over the whole hidden layer
  const int nsl = p.hidden / HS;

  const __amdgpu_buffer_rsrc_t xr = rsrc(p.x + p.xco, p.xbytes);
  const __amdgpu_buffer_rsrc_t w1r = rsrc(p.w1, p.w1bytes);
  const __amdgpu_buffer_rsrc_t w2r = rsrc(p.w2, p.w2bytes);

  // fragment f of a packed matrix: lane's 8 halves of the hi plane at f *
  // 1024 + lane * 8, of the lo plane 512 halves further
  auto ldfrag = [&](const __amdgpu_buffer_rsrc_t &r, int f, f16x8 &h, f16x8 &l) {
    const int o = (f * 1024 + lane * 8) * 2;
    h = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
    l = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, o + 1024, 0, 0));
  };

  // ffn1 fragments of slice 0 first: their latency hides behind the image
  f16x8 a1h[KC], a1l[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) ldfrag(w1r, wave * KC + kc, a1h[kc], a1l[kc]);

  // input image: piece u = (pixel, 8-channel group), split once
  {
    constexpr int NPC = P * C / 8;
#pragma unroll
    for (int u = tid; u < NPC; u += kNT) {
      const int px = u / (C / 8), c8 = u - px * (C / 8);
      const bool ok = pix0 + px < p.npix;
      const int o = ok ? ((pix0 + px) * p.xcs + c8 * 8) * 4 : kOob;
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
      const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
      u32x4_t h, l;
      rg.add8(v);
      split8(v, h, l);
      const int off = swz((c8 >> 2) * P + px, c8 & 3);
      *reinterpret_cast<u32x4_t *>(Xh + off) = h;
      *reinterpret_cast<u32x4_t *>(Xl + off) = l;
    }
    for (int i = tid; i < p.hidden; i += kNT) Lb1[i] = p.b1[i];
    for (int i = tid; i < C; i += kNT) {
      Lb2[i] = p.b2[i];
      Lsc[i] = p.scale ? p.scale[i] : 1.f;
    }
  }
  __syncthreads();

  f32x4 om[NTW][PB], oc[NTW][PB];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      om[j][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
      oc[j][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  const float slope = p.slope;

  for (int s = 0; s < nsl; ++s) {
    // ffn2 fragments of this slice: rows (wave * NTW + j) * 16, K chunks 2 s, 2 s + 1
    f16x8 a2h[NTW][2], a2l[NTW][2];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ldfrag(w2r, (wave * NTW + j) * KH + 2 * s + kk, a2h[j][kk], a2l[j][kk]);

    // ffn1: hidden rows s * 64 + 16 wave .. + 15 for both pixel blocks
    f32x4 hm[PB], hc[PB];
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      hm[pb] = f32x4{0.f, 0.f, 0.f, 0.f};
      hc[pb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) {
        const int o = swz(kc * P + pb * 16 + col, g);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Xh + o);
        const f16x8 bl = *reinterpret_cast<const f16x8 *>(Xl + o);
        hm[pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1h[kc], bh, hm[pb], 0, 0, 0);
        hc[pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1h[kc], bl, hc[pb], 0, 0, 0);
        hc[pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1l[kc], bh, hc[pb], 0, 0, 0);
      }
    // the next slice's ffn1 fragments (the registers are free now)
    if (s + 1 < nsl) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) ldfrag(w1r, ((s + 1) * 4 + wave) * KC + kc, a1h[kc], a1l[kc]);
    }
    // hidden = lrelu(acc + b1) in fp32, split into this slice's hidden image:
    // lane (col, g) holds hidden channels 16 wave + 4 g .. + 3 of pixel
    // pb * 16 + col: chunk wave >> 1, slot (wave & 1) * 2 + (g >> 1), halves
    // (g & 1) * 4 .. + 3 of the slot
    uint16_t *Hh = Hb + (s & 1) * 2 * HI, *Hl = Hh + HI;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = (hm[pb][e] + hc[pb][e] * kLoInv) + Lb1[s * HS + wave * 16 + g * 4 + e];
        v[e] = t >= 0.f ? t : t * slope;
      }
      rg.add4(v);
      const auto h0 = __builtin_amdgcn_cvt_pkrtz(v[0], v[1]);
      const auto h1 = __builtin_amdgcn_cvt_pkrtz(v[2], v[3]);
      const uint32_t l0 = pk(split_lo(v[0], (float)h0[0]), split_lo(v[1], (float)h0[1]));
      const uint32_t l1 = pk(split_lo(v[2], (float)h1[0]), split_lo(v[3], (float)h1[1]));
      const int off = swz((wave >> 1) * P + pb * 16 + col, (wave & 1) * 2 + (g >> 1)) + (g & 1) * 4;
      typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2_t *>(Hh + off) =
          u32x2_t{__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1)};
      *reinterpret_cast<u32x2_t *>(Hl + off) = u32x2_t{l0, l1};
    }
    // every wave's hidden rows of slice s are in; (every wave finished ffn2
    // of slice s - 1 before it got here, so buffer (s + 1) & 1 is free next)
    __syncthreads();
    // ffn2 over the slice: K chunks 2 s, 2 s + 1 of the hidden layer (the
    // image operands read at their use: a register ring here and in ffn1
    // measured 26.8 vs 24.8 us at C = 192, profiles/r06f_lat_ab.jsonl)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) {
        const int o = swz(kk * P + pb * 16 + col, g);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Hh + o);
        const f16x8 bl = *reinterpret_cast<const f16x8 *>(Hl + o);
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          om[j][pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2h[j][kk], bh, om[j][pb], 0, 0, 0);
          oc[j][pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2h[j][kk], bl, oc[j][pb], 0, 0, 0);
          oc[j][pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2l[j][kk], bh, oc[j][pb], 0, 0, 0);
        }
      }
  }

  // epilogue: lane (col, g) of fragment (j, pb) holds output channels
  // (wave * NTW + j) * 16 + 4 g .. + 3 of pixel pix0 + pb * 16 + col
  const __amdgpu_buffer_rsrc_t yr = rsrc(p.y + p.yco, p.ybytes);
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int px = pix0 + pb * 16 + col;
    const bool ok = px < p.npix;
    f32x4 xv[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (wave * NTW + j) * 16 + 4 * g;
      xv[j] = __builtin_bit_cast(f32x4,
                                 __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (px * p.xcs + n) * 4 : kOob, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (wave * NTW + j) * 16 + 4 * g;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = (om[j][pb][e] + oc[j][pb][e] * kLoInv) + Lb2[n + e];
        t = t >= 0.f ? t : t * slope;
        t = xv[j][e] + t;
        v[e] = t * Lsc[n + e];
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), yr, ok ? (px * p.ycs + n) * 4 : kOob, 0,
                                             0);
    }
  }
}

// The tail of a latent DepthConv (DCVC-DC/src/models/layers.py:135-163,
// adaptor-free blocks C -> C of the entropy model, video_model.py:250-305):
//   out = conv2(dw3x3(t) + bdw) + b2 + x
// with t = lrelu(conv1(x) + b1) from the previous launch.  Unfused this is a
// depthwise launch (an fp32 round trip of the C-channel map) and a 1x1 GEMM
// launch on 8160 pixels.  One workgroup owns 32 pixels: every thread runs
// the depthwise taps of its (pixel, 8-channel group) items in the order and
// with the fp32 fma chain of misc.hip's dw8_kernel (taps (dy, dx) ascending,
// then the bias), splits the result into an LDS image, and the waves run
// conv2 on it with packed weight fragments streamed from L2 two K chunks
// ahead (sgemm.hip's products and K order); the epilogue adds b2 and the
// identity from the accumulators.  Bit-identical to the two unfused launches.
struct DP {
  const float *t;
  int npix, H, W, tcs, tco, tbytes;
  const float *r;
  int rcs, rco, rbytes;
  float *y;
  int ycs, yco, ybytes;
  const float *w9, *bdw;   // depthwise taps [9][C], bias [C]
  const uint16_t *w2;      // conv2 [C][C] as packed fragments
  int w2bytes;
  const float *b2;
  int *ovf;               // fp16 range guard (split.h SplitRange)
};

template <int C, int PB>
__global__ void __launch_bounds__(kNT) sldc_kernel(DP p) {
  SplitRange rg(p.ovf);
  constexpr int P = 16 * PB;        // pixels per workgroup
  constexpr int KC = C / 32, NTW = C / 64, PF = 2;
  constexpr int XI = KC * P * 32;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Dh = reinterpret_cast<uint16_t *>(smem), *Dl = Dh + XI;
  float *Lw9 = reinterpret_cast<float *>(Dl + XI);   // [9][C]
  float *Lbd = Lw9 + 9 * C, *Lb2 = Lbd + C;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int pix0 = blockIdx.x * P;
  const __amdgpu_buffer_rsrc_t tr = rsrc(p.t + p.tco, p.tbytes);
  const __amdgpu_buffer_rsrc_t w2r = rsrc(p.w2, p.w2bytes);

  f16x8 ah[PF + 1][NTW], al[PF + 1][NTW];
  auto ldw = [&](int kc, int q) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int o = (((wave * NTW + j) * KC + kc) * 1024 + lane * 8) * 2;
      ah[q][j] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(w2r, o, 0, 0));
      al[q][j] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(w2r, o + 1024, 0, 0));
    }
  };
#pragma unroll
  for (int kc = 0; kc < PF; ++kc) ldw(kc, kc);

  for (int i = tid; i < 9 * C; i += kNT) Lw9[i] = p.w9[i];
  for (int i = tid; i < C; i += kNT) {
    Lbd[i] = p.bdw[i];
    Lb2[i] = p.b2[i];
  }
  __syncthreads();

  // depthwise: items (pixel, 8-channel group)
  for (int u = tid; u < P * C / 8; u += kNT) {
    const int px = u / (C / 8), c8 = u - px * (C / 8);
    const int P0 = pix0 + px;
    const bool okp = P0 < p.npix;
    const int py = P0 / p.W, pxx = P0 - py * p.W;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = py + dy, xx = pxx + dx;
        const bool ok = okp && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
        if (!ok) continue;   // (uniform for most items; dw8_kernel skips the out-of-map taps too)
        const int o = ((yy * p.W + xx) * p.tcs + c8 * 8) * 4;
        const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(tr, o, 0, 0));
        const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(tr, o + 16, 0, 0));
        const float *wt = Lw9 + ((dy + 1) * 3 + dx + 1) * C + c8 * 8;
        const float4 w0 = *reinterpret_cast<const float4 *>(wt), w1 = *reinterpret_cast<const float4 *>(wt + 4);
        acc[0] = __builtin_fmaf(w0.x, a[0], acc[0]);
        acc[1] = __builtin_fmaf(w0.y, a[1], acc[1]);
        acc[2] = __builtin_fmaf(w0.z, a[2], acc[2]);
        acc[3] = __builtin_fmaf(w0.w, a[3], acc[3]);
        acc[4] = __builtin_fmaf(w1.x, b[0], acc[4]);
        acc[5] = __builtin_fmaf(w1.y, b[1], acc[5]);
        acc[6] = __builtin_fmaf(w1.z, b[2], acc[6]);
        acc[7] = __builtin_fmaf(w1.w, b[3], acc[7]);
      }
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = okp ? acc[e] + Lbd[c8 * 8 + e] : 0.f;
    u32x4_t h, l;
    rg.add8(v);
    split8(v, h, l);
    const int off = swz((c8 >> 2) * P + px, c8 & 3);
    *reinterpret_cast<u32x4_t *>(Dh + off) = h;
    *reinterpret_cast<u32x4_t *>(Dl + off) = l;
  }
  __syncthreads();

  f32x4 am[NTW][PB], ac[NTW][PB];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      am[j][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
      ac[j][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // (the image operands one K chunk ahead in a second register set: 12.4 vs
  // 13.5 us at C = 192, 34.2 vs 34.5 at 384, profiles/r06f_lat_ab.jsonl)
  f16x8 rbh[2][PB], rbl[2][PB];
  auto rd2 = [&](int kc, int q) {
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      const int o = swz(kc * P + pb * 16 + col, g);
      rbh[q][pb] = *reinterpret_cast<const f16x8 *>(Dh + o);
      rbl[q][pb] = *reinterpret_cast<const f16x8 *>(Dl + o);
    }
  };
  rd2(0, 0);
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    if (kc + PF < KC) ldw(kc + PF, (kc + PF) % (PF + 1));
    if (kc + 1 < KC) rd2(kc + 1, (kc + 1) & 1);
    sched_fence();
    const int q = kc % (PF + 1), qb = kc & 1;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        am[j][pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[q][j], rbh[qb][pb], am[j][pb], 0, 0, 0);
        ac[j][pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[q][j], rbl[qb][pb], ac[j][pb], 0, 0, 0);
        ac[j][pb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[q][j], rbh[qb][pb], ac[j][pb], 0, 0, 0);
      }
    }
  }

  // epilogue: out = (acc + b2) + identity
  const __amdgpu_buffer_rsrc_t rr = rsrc(p.r + p.rco, p.rbytes);
  const __amdgpu_buffer_rsrc_t yr = rsrc(p.y + p.yco, p.ybytes);
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int px = pix0 + pb * 16 + col;
    const bool ok = px < p.npix;
    f32x4 rv[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (wave * NTW + j) * 16 + 4 * g;
      rv[j] = __builtin_bit_cast(f32x4,
                                 __builtin_amdgcn_raw_buffer_load_b128(rr, ok ? (px * p.rcs + n) * 4 : kOob, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (wave * NTW + j) * 16 + 4 * g;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = rv[j][e] + ((am[j][pb][e] + ac[j][pb][e] * kLoInv) + Lb2[n + e]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), yr, ok ? (px * p.ycs + n) * 4 : kOob, 0,
                                             0);
    }
  }
}

template <int C, int PB>
int run_dc(DP p, hipStream_t st) {
  constexpr int PX = 16 * PB;
  const size_t lds = (size_t)2 * (C / 32) * PX * 32 * 2 + (size_t)11 * C * 4;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  const int G = (p.npix + PX - 1) / PX;
  auto kern = sldc_kernel<C, PB>;
  dcvc_note_kernel("sldc_kernel<%d, %d>@%lld", C, PB, (long long)G * kNT);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(kNT), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

template <int C, int PB>
int run(LP p, hipStream_t st) {
  constexpr int KC = C / 32, PX = 16 * PB;
  const size_t lds = (size_t)2 * KC * PX * 32 * 2 + (size_t)4 * 2 * PX * 32 * 2 + (size_t)(p.hidden + 2 * C) * 4;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  const int G = (p.npix + PX - 1) / PX;
  auto kern = slffn_kernel<C, PB>;
  dcvc_note_kernel("slffn_kernel<%d, %d>@%lld", C, PB, (long long)G * kNT);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(kNT), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// packed fragments of an R x K matrix (R multiple of 16, K of 32): fragment
// (rb, kc) = rows [16 rb, 16 rb + 16) x K [32 kc, 32 kc + 32), index rb *
// (K / 32) + kc, 1024 halves: hi plane then lo plane, each lane-ordered --
// lane (i, kg) = kg * 16 + i holds row 16 rb + i, K 32 kc + 8 kg .. + 7
void pack_frags(const float *m, int R, int K, uint16_t *o) {
  const int kcs = K / 32;
  for (int rb = 0; rb < R / 16; ++rb)
    for (int kc = 0; kc < kcs; ++kc) {
      uint16_t *f = o + ((int64_t)rb * kcs + kc) * 1024;
      for (int lane = 0; lane < 64; ++lane) {
        const int i = lane & 15, kg = lane >> 4;
        for (int e = 0; e < 8; ++e) {
          const float v = m[(int64_t)(rb * 16 + i) * K + kc * 32 + kg * 8 + e];
          host_split(v, f[lane * 8 + e], f[512 + lane * 8 + e]);
        }
      }
    }
}

}  // namespace

// the latent widths this kernel takes (C = 192, 384; hidden a multiple of 64)
extern "C" int dcvc_internal_lffn_supported(int c, int hidden) {
  return (c == 192 || c == 384) && hidden > 0 && hidden % HS == 0;
}

// w1 [hidden][c] (conv.0), w2 [c][hidden] (conv.2) as packed fragments: ffn1's
// (hidden / 16 x c / 32 fragments) then ffn2's (c / 16 x hidden / 32).
extern "C" int64_t dcvc_internal_lffn_pack(const float *w1, const float *w2, int c, int hidden, void *out) {
  if (!dcvc_internal_lffn_supported(c, hidden)) return DCVC_HIP_EINVAL;
  const int64_t n1 = (int64_t)hidden * c * 2, n2 = (int64_t)c * hidden * 2;
  if (!out) return n1 + n2;
  uint16_t *o = reinterpret_cast<uint16_t *>(out);
  pack_frags(w1, hidden, c, o);
  pack_frags(w2, c, hidden, o + n1);
  return n1 + n2;
}

extern "C" int dcvc_internal_lffn(const dcvc_ffn_args *a, void *stream) {
  if (!dcvc_internal_lffn_supported(a->c, a->hidden)) return DCVC_HIP_EUNSUPPORTED;
  const int64_t npix = (int64_t)a->x.H * a->x.W;
  if (npix <= 0) return DCVC_HIP_OK;
  auto bytes = [&](int cs, int co) { return (npix * cs - co) * 4; };
  if (bytes(a->x.cstride, a->x.coff) > 0x7fff0000 || bytes(a->y.cstride, a->y.coff) > 0x7fff0000)
    return DCVC_HIP_EUNSUPPORTED;
  LP p{};
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.npix = (int)npix;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.xbytes = (int)bytes(a->x.cstride, a->x.coff);
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.ybytes = (int)bytes(a->y.cstride, a->y.coff);
  const int64_t n1 = (int64_t)a->hidden * a->c * 2;
  p.w1 = reinterpret_cast<const uint16_t *>(a->w);
  p.w2 = p.w1 + n1;
  p.w1bytes = (int)(n1 * 2);
  p.w2bytes = (int)(n1 * 2);
  p.b1 = a->b1;
  p.b2 = a->b2;
  p.scale = a->scale;
  p.hidden = a->hidden;
  p.slope = a->slope;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return a->c == 384 ? run<384, SLFFN_PB384>(p, st) : run<192, 2>(p, st);
}

// MFMA A-fragment packing of an R x K fp32 matrix (R % 16 == 0, K % 32 ==
// 0): R / 16 x K / 32 fragments of 1024 halves (pack_frags); out NULL: size.
extern "C" int64_t dcvc_frag_pack_weights(const float *w, int rows, int k, void *out) {
  if (!w || rows <= 0 || k <= 0 || rows % 16 || k % 32) return DCVC_HIP_EINVAL;
  if (out && !host_split_range_ok(w, (int64_t)rows * k)) return DCVC_HIP_EINVAL;
  const int64_t n = (int64_t)rows * k * 2;
  if (out) pack_frags(w, rows, k, reinterpret_cast<uint16_t *>(out));
  return n;
}

extern "C" int dcvc_dw_conv2_split(const dcvc_dwc_args *a, void *stream) {
  if (!a || !a->t.ptr || !a->r.ptr || !a->y.ptr || !a->w9 || !a->bdw || !a->w2 || !a->b2) return DCVC_HIP_EINVAL;
  const int c = a->c;
  if (a->t.dtype != DCVC_F32 || a->r.dtype != DCVC_F32 || a->y.dtype != DCVC_F32 || a->t.C != c || a->r.C != c ||
      a->y.C != c || a->t.H != a->y.H || a->t.W != a->y.W || a->r.H != a->y.H || a->r.W != a->y.W)
    return DCVC_HIP_EINVAL;
  // (128: the feature-rate blocks at 1/4 resolution, dcvc_amd/layers.py DW128)
  if (c != 192 && c != 384 && c != 128) return DCVC_HIP_EUNSUPPORTED;
  auto al = [](const dcvc_tensor &v) { return (uintptr_t)v.ptr % 16 == 0 && v.cstride % 4 == 0 && v.coff % 4 == 0; };
  if (!al(a->t) || !al(a->r) || !al(a->y) || a->t.cstride % 8 || a->t.coff % 8) return DCVC_HIP_EUNSUPPORTED;
  const int64_t npix = (int64_t)a->t.H * a->t.W;
  if (npix <= 0) return DCVC_HIP_OK;
  auto bytes = [&](const dcvc_tensor &v) { return (npix * v.cstride - v.coff) * 4; };
  if (bytes(a->t) > 0x7fff0000 || bytes(a->r) > 0x7fff0000 || bytes(a->y) > 0x7fff0000) return DCVC_HIP_EUNSUPPORTED;
  DP p{};
  p.ovf = dcvc_internal_split_flag();
  p.t = reinterpret_cast<const float *>(a->t.ptr);
  p.npix = (int)npix;
  p.H = a->t.H;
  p.W = a->t.W;
  p.tcs = a->t.cstride;
  p.tco = a->t.coff;
  p.tbytes = (int)bytes(a->t);
  p.r = reinterpret_cast<const float *>(a->r.ptr);
  p.rcs = a->r.cstride;
  p.rco = a->r.coff;
  p.rbytes = (int)bytes(a->r);
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.ybytes = (int)bytes(a->y);
  p.w9 = a->w9;
  p.bdw = a->bdw;
  p.w2 = reinterpret_cast<const uint16_t *>(a->w2);
  p.w2bytes = (int)((int64_t)c * c * 2 * 2);
  p.b2 = a->b2;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return c == 384 ? run_dc<384, SLDC_PB384>(p, st) : c == 192 ? run_dc<192, 2>(p, st) : run_dc<128, 2>(p, st);
}
