// Split-fp16 ("f16x3", sconv.hip's header) 1x1 convolution as a pixel GEMM:
// y[p][n] = sum_c x[p][c] w[n][c] over the pixels of an fp32 NHWC view.
//
// The 1x1 layers of DCVC-DC's entropy model run on the 68 x 120 latent
// (8160 pixels, 192..1024 channels, ~200 launches per P-frame): too few
// pixels to fill 256 CUs with sconv.hip's 2-D halo tiles, and a long K walk
// (up to 32 chunks of 32 channels) that sconv.hip covers one chunk at a time
// with two barriers, an LDS image write and a register prefetch only one chunk
// ahead, i.e. latency bound at ~5-10% of the MFMA rate.  Here:
//   * a workgroup owns BM = 64 * PXW consecutive pixels x BN output channels
//     (4 waves; wave w: pixels [w * 16 PXW, (w + 1) * 16 PXW), all BN
//     channels, PXW x BN/16 x 2 f32x4 accumulators);
//   * the pixel operand goes global -> registers -> split -> MFMA B operand
//     with no LDS round trip (a wave is the only reader of its pixels): lane
//     (col, hi) loads channels [8 hi, 8 hi + 8) of pixel col of each of its
//     16-pixel groups, 2 x 16-byte buffer loads, PD stages ahead;
//   * the weight operand (pre-split by dcvc_conv_pack_weights, BN rows x 32
//     halves, hi and lo, swizzled as split.h's swz) arrives by LDS-DMA into
//     a ring of PD + 1 stage buffers, PD stages ahead;
//   * one barrier per 32-channel stage (every wave's own loads of the stage
//     waited with a counted vmcnt first), no LDS writes by the waves at all;
//   * the epilogue runs straight from the accumulators (lane: 4 consecutive
//     output channels of one pixel), out = scale * (res2 + (res + act(acc +
//     bias))) in the reference's order, 16-byte loads and stores.
// Every load is unconditional: pixels past the view, channels past cin and
// stages past the last chunk read zeros through out-of-range buffer offsets,
// so the per-stage vector-memory count is constant and vmcnt can be counted.
#include "common.h"
#include "split.h"

#include <utility>

namespace {

struct GP {
  const float *x;
  int xcs, xco;
  int npix;
  const uint16_t *w;
  int wbytes;
  int64_t wchunk;   // halves of one 32-channel chunk's packed weights (hi + lo)
  const float *bias;
  float *y;
  int ycs, yco;
  int cin, cout, nchunks, nblk, ntiles;
  int in_op;
  float in_slope;
  int act;
  float slope;
  const float *scale;
  const float *res;
  int rcs, rco;
  const float *res2;
  int r2cs, r2co;
  int shuffle, W;   // pixel shuffle (x2) on store: the input map's width W
  int *ovf;               // fp16 range guard (split.h SplitRange)
};

template <int BN, int PXW, int PD, bool GATE = false>
struct GG {
  static constexpr int NT = BN / 16;
  static constexpr int BM = 4 * PXW * 16;
  static constexpr int NB = PD + 1;                 // LDS stage buffers
  static constexpr int NX = GATE ? 2 : 1;           // pixel operands per stage: the values (and the gates)
  static constexpr int WH = BN * 64;                // halves of a stage's weights (hi rows, then lo rows)
  static constexpr int XH = NX * BM * 64;           // halves of a stage's pixels (fp32, 2 rows of 64 B per pixel each)
  static constexpr int SH = WH + XH;                // halves of one stage buffer
  static constexpr int DPW = BN / 32;               // weight LDS-DMA pieces (1 KiB) per stage per wave
  static constexpr int L = 2 * NX * PXW + DPW;      // LDS-DMA instructions per stage per wave
  static constexpr size_t LDS = (size_t)NB * SH * 2 + 2 * BN * 4;
  static_assert(BN % 32 == 0, "BN must be a multiple of 32");
  static_assert((PD - 1) * L < 64, "vmcnt is 6 bits");
};

constexpr int kOob = 0x7fffffe0;

// f(integral_constant<int, I>) for I = 0 .. N - 1, in order
template <typename F, int... I>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}   // a buffer offset past any num_records: the load returns zeros

template <int BN, int PXW, int PD, bool GATE>
__global__ void __launch_bounds__(256) sgemm_kernel(GP p) {
  SplitRange rg(p.ovf);
  typedef GG<BN, PXW, PD, GATE> G_;
  constexpr int NT = G_::NT, BM = G_::BM, NB = G_::NB, WH = G_::WH, SH = G_::SH, DPW = G_::DPW, L = G_::L;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Ls = reinterpret_cast<uint16_t *>(smem);
  float *Lc = reinterpret_cast<float *>(smem + (size_t)NB * SH * 2);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  // the n-blocks of one pixel block (consecutive g) on one XCD: its L2 serves
  // the pixel block's reloads (workgroups are dealt to XCDs round robin)
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);
  const int nb = g % p.nblk, pb = g / p.nblk;
  const int n0 = nb * BN, pix0 = pb * BM;

  // bias | scale of the n-block (read before the first barrier)
  for (int i = tid; i < BN; i += 256) {
    const int n = n0 + i;
    Lc[i] = (p.bias && n < p.cout) ? p.bias[n] : 0.f;
    Lc[BN + i] = (p.scale && n < p.cout) ? p.scale[p.shuffle ? n / 4 : n] : 1.f;
  }

  // Both operands arrive by LDS-DMA (16 bytes per lane, lane-linear LDS
  // destination), so the waves' only waits on them are the counted ones below.
  // A 1-KiB piece is 16 rows of 64 bytes, rows swizzled as split.h's swz
  // (conflict-free reads of 16 consecutive rows at one slot): lane i writes
  // (row i / 4, physical slot i % 4) and fetches the logical slot there.
  //   weights: row nn (output channel n0 + nn) of the hi then the lo block,
  //            32 halves of the chunk's 32 input channels;
  //   pixels:  per 16-pixel group r and channel half h, row h * 16 + px holds
  //            fp32 channels 16 h .. 16 h + 15 of the chunk (4 per slot).
  const int64_t eb = (int64_t)pix0 * p.xcs + p.xco;
  // (gated input, ConvFFN2's second 1x1: 2 cin channels, the gates past the values)
  int64_t nrec = ((int64_t)(p.npix - pix0 - 1) * p.xcs + (GATE ? 2 : 1) * p.cin) * 4;
  if (nrec > 0x7fff0000) nrec = 0x7fff0000;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.x + eb), (short)0, (int)nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
  const int dpx = lane >> 2;
  const int dls = (lane & 3) ^ ((0x1320 >> (((dpx >> 2) & 3) << 2)) & 3);   // (rows h * 16 + px: same swizzle)
  int xoff[PXW];
#pragma unroll
  for (int r = 0; r < PXW; ++r) {
    const int lp = (wave * PXW + r) * 16 + dpx;
    xoff[r] = pix0 + lp < p.npix ? (lp * p.xcs + dls * 4) * 4 : -1;
  }
  // per-lane parts of every LDS-DMA offset, computed once: a stage adds its
  // chunk's uniform offset (s * wchunk halves of weights, 32 channels of
  // pixels) and compares the chunk against per-lane limits (weights: the
  // chunk count and cout; pixels: cin), so a stage's address work is an add
  // and a select per DMA instead of its 64-bit index arithmetic
  int wbase[DPW];
  bool wok[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) {
    const int i = wave + 4 * d;
    const int hl = i >= BN / 16, k = hl ? i - BN / 16 : i;
    const int R = k * 16 + dpx;
    const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
    const int n = n0 + R;
    wok[d] = n < p.cout;
    wbase[d] = ((hl ? p.cout * 32 : 0) + n * 32 + ls * 8) * 2;
  }
  const int wcb = (int)(p.wchunk * 2);
  int xbase[G_::NX][PXW][2], xlim[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) xlim[h] = p.cin - h * 16 - dls * 4;   // chunk s reads channel s * 32 + (cin - xlim)
#pragma unroll
  for (int gx = 0; gx < G_::NX; ++gx)
#pragma unroll
    for (int r = 0; r < PXW; ++r)
#pragma unroll
      for (int h = 0; h < 2; ++h) xbase[gx][r][h] = xoff[r] >= 0 ? xoff[r] + (h * 16 + gx * p.cin) * 4 : -1;
  auto issue = [&](int s, int b) {
    uint16_t *Lb = Ls + (size_t)b * SH;
    const bool live = s < p.nchunks;
    const int wso = live ? s * wcb : 0, xso = s * 128, c0 = s * 32;
#pragma unroll
    for (int d = 0; d < DPW; ++d) {
      const int i = wave + 4 * d;
      const int hl = i >= BN / 16, k = hl ? i - BN / 16 : i;
      const int voff = live && wok[d] ? wbase[d] + wso : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (__attribute__((address_space(3))) void *)(Lb + hl * (WH / 2) + k * 512), 16, voff, 0, 0, 0);
    }
#pragma unroll
    for (int gx = 0; gx < G_::NX; ++gx)
#pragma unroll
      for (int r = 0; r < PXW; ++r)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int o = (xbase[gx][r][h] >= 0 && c0 < xlim[h]) ? xbase[gx][r][h] + xso : kOob;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              xr, (__attribute__((address_space(3))) void *)(Lb + WH + gx * (BM * 64) + ((wave * PXW + r) * 2 + h) * 512),
              16, o, 0, 0, 0);
        }
  };

  f32x4 am[PXW][NT], ac[PXW][NT];
#pragma unroll
  for (int r = 0; r < PXW; ++r)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      am[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ac[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

#pragma unroll
  for (int j = 0; j < PD; ++j) issue(j, j);
  const int nst = p.nchunks;
  const bool lrelu = p.in_op == DCVC_IN_LRELU;
  // one 32-channel stage on stage buffer B (compile-time: the loop below runs
  // the NB buffers in turn, so every LDS address is an immediate offset)
  auto stage = [&](int s, auto B_) {
    constexpr int B = decltype(B_)::value;
    // stage s's pieces (issued PD stages ago) have landed for this wave; the
    // barrier makes every wave's pieces visible and retires stage s - 1's
    // reads of the buffer the next issue refills
    wait_vm_n_lgkm<(PD - 1) * L>();
    raw_barrier();
    issue(s + PD, (B + PD) % NB);
    const uint16_t *Lb = Ls + (size_t)B * SH;
    f16x8 bh[PXW], bl[PXW];
#pragma unroll
    for (int r = 0; r < PXW; ++r) {
      // lane (col, hi): channels 8 hi .. 8 hi + 7 = half hi / 2, slots 2 (hi & 1), + 1
      const uint16_t *xrow = Lb + WH + ((wave * PXW + r) * 2 + (hi >> 1)) * 512;
      const f32x4 a = *reinterpret_cast<const f32x4 *>(xrow + swz(col, (hi & 1) * 2));
      const f32x4 c = *reinterpret_cast<const f32x4 *>(xrow + swz(col, (hi & 1) * 2 + 1));
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = a[e];
        v[4 + e] = c[e];
      }
      if constexpr (GATE) {
        // x1 * lrelu(x2) (sconv.hip's gate, same order)
        const uint16_t *grow = xrow + BM * 64;
        const f32x4 ga = *reinterpret_cast<const f32x4 *>(grow + swz(col, (hi & 1) * 2));
        const f32x4 gc = *reinterpret_cast<const f32x4 *>(grow + swz(col, (hi & 1) * 2 + 1));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float g0 = ga[e] >= 0.f ? ga[e] : ga[e] * p.in_slope;
          const float g1 = gc[e] >= 0.f ? gc[e] : gc[e] * p.in_slope;
          v[e] = v[e] * g0;
          v[4 + e] = v[4 + e] * g1;
        }
      } else if (lrelu) {
        // (max(v, s v): the host admits 0 <= s <= 1 only, where it is the
        // leaky ReLU, signed zeros included)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = lrelu_in(v[e], p.in_slope);
      }
      u32x4_t h, l;
      rg.add8(v);
      split8(v, h, l);
      bh[r] = __builtin_bit_cast(f16x8, h);
      bl[r] = __builtin_bit_cast(f16x8, l);
    }
    // (the second ac product of every (r, jn) after all the first ones: no
    // MFMA waits on its predecessor's result; the same accumulation order)
    f16x8 al[NT];
#pragma unroll
    for (int jn = 0; jn < NT; ++jn) {
      const int o = swz(jn * 16 + col, hi);
      const f16x8 ah = *reinterpret_cast<const f16x8 *>(Lb + o);
      al[jn] = *reinterpret_cast<const f16x8 *>(Lb + WH / 2 + o);
#pragma unroll
      for (int r = 0; r < PXW; ++r) {
        am[r][jn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[r], am[r][jn], 0, 0, 0);
        ac[r][jn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[r], ac[r][jn], 0, 0, 0);
      }
    }
#pragma unroll
    for (int jn = 0; jn < NT; ++jn)
#pragma unroll
      for (int r = 0; r < PXW; ++r)
        ac[r][jn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[jn], bh[r], ac[r][jn], 0, 0, 0);
  };
  for (int s = 0; s < nst; s += NB)
    sfor<NB>([&](auto B_) {
      if (s + decltype(B_)::value < nst) stage(s + decltype(B_)::value, B_);
    });
  wait_vm_lgkm();   // the zero-fill pieces past the last stage: no LDS-DMA in flight at exit

  if (p.shuffle) {
    // pixel shuffle (subpel_conv1x1, r = 2): conv channels n .. n + 3 (n % 4
    // == 0) of pixel (oy, ox) go to output channel n / 4 of the 2x2 block
    // (2 oy + (e >> 1), 2 ox + (e & 1)); residuals and the scale are indexed in
    // the output map, bias and activation per conv channel (epilogue.h order)
#pragma unroll
    for (int r = 0; r < PXW; ++r) {
      const int P = pix0 + (wave * PXW + r) * 16 + col;
      const bool okp = P < p.npix;
      const int oy = P / p.W, ox = P - (P / p.W) * p.W;
#pragma unroll
      for (int jn = 0; jn < NT; ++jn) {
        const int nl = jn * 16 + hi * 4, n = n0 + nl;
        if (!okp || n >= p.cout) continue;
        const float4 bb = *reinterpret_cast<const float4 *>(Lc + nl);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
        const float sc = Lc[BN + nl];   // scale[n / 4] staged at the n-block's channel nl (below)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t q = (int64_t)(2 * oy + (e >> 1)) * (2 * p.W) + 2 * ox + (e & 1);
          float v = apply_act(p.act, (am[r][jn][e] + ac[r][jn][e] * kLoInv) + bv[e], p.slope);
          if (p.res) v = p.res[q * p.rcs + p.rco + n / 4] + v;
          if (p.res2) v = p.res2[q * p.r2cs + p.r2co + n / 4] + v;
          if (p.scale) v *= sc;
          p.y[q * p.ycs + p.yco + n / 4] = v;
        }
      }
    }
    return;
  }
  // epilogue: lane (col, hi) of fragment (r, jn) holds output channels
  // n0 + 16 jn + 4 hi .. + 3 of pixel (wave * PXW + r) * 16 + col
#pragma unroll
  for (int r = 0; r < PXW; ++r) {
    const int P = pix0 + (wave * PXW + r) * 16 + col;
    const bool okp = P < p.npix;
    f32x4 r1[NT], r2[NT];
#pragma unroll
    for (int jn = 0; jn < NT; ++jn) {
      const int n = n0 + jn * 16 + hi * 4;
      const bool ok = okp && n < p.cout;
      r1[jn] = (p.res && ok) ? *reinterpret_cast<const f32x4 *>(p.res + (int64_t)P * p.rcs + p.rco + n)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
      r2[jn] = (p.res2 && ok) ? *reinterpret_cast<const f32x4 *>(p.res2 + (int64_t)P * p.r2cs + p.r2co + n)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int jn = 0; jn < NT; ++jn) {
      const int nl = jn * 16 + hi * 4, n = n0 + nl;
      const float4 bb = *reinterpret_cast<const float4 *>(Lc + nl);
      const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + nl);
      f32x4 v;
      v[0] = (am[r][jn][0] + ac[r][jn][0] * kLoInv) + bb.x;
      v[1] = (am[r][jn][1] + ac[r][jn][1] * kLoInv) + bb.y;
      v[2] = (am[r][jn][2] + ac[r][jn][2] * kLoInv) + bb.z;
      v[3] = (am[r][jn][3] + ac[r][jn][3] * kLoInv) + bb.w;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = apply_act(p.act, v[e], p.slope);
      if (p.res) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = r1[jn][e] + v[e];
      }
      if (p.res2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = r2[jn][e] + v[e];
      }
      if (p.scale) {
        v[0] *= sc.x;
        v[1] *= sc.y;
        v[2] *= sc.z;
        v[3] *= sc.w;
      }
      if (okp && n < p.cout) *reinterpret_cast<f32x4 *>(p.y + (int64_t)P * p.ycs + p.yco + n) = v;
    }
  }
}

template <int BN, int PXW>
int64_t tiles_of(const GP &p) {
  return (int64_t)((p.npix + 64 * PXW - 1) / (64 * PXW)) * ((p.cout + BN - 1) / BN);
}

template <int BN, int PXW, int PD, bool GATE = false>
int launch(GP p, hipStream_t st) {
  typedef GG<BN, PXW, PD, GATE> G_;
  p.nblk = (p.cout + BN - 1) / BN;
  const int64_t nt = tiles_of<BN, PXW>(p);
  if (nt <= 0) return DCVC_HIP_OK;
  if (nt > 0x7fffffff) return DCVC_HIP_EINVAL;
  p.ntiles = (int)nt;
  auto kern = sgemm_kernel<BN, PXW, PD, GATE>;
  if (G_::LDS > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  if (GATE) dcvc_note_kernel("sgemm_kernel<%d, %d, %d, true>", BN, PXW, PD);
  else dcvc_note_kernel("sgemm_kernel<%d, %d, %d>", BN, PXW, PD);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
  hipLaunchKernelGGL(kern, dim3((unsigned)nt), dim3(256), G_::LDS, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// dcvc_set_option("sgemm", v): 0 = auto, -1 = off (sconv.hip's 1x1 path),
// 1..6 = force (BN, PXW) = (128, 2), (64, 2), (32, 2), (128, 1), (64, 1), (32, 1)
int g_cfg = 0;
int g_cus = 0;
int g_pd = 0;   // dcvc_set_option("sgemm_pd", 1 | 2 | 3 | 5): stages in flight (A/B); 0 = auto
// dcvc_set_option("sgemm_gate", 0): ConvFFN2's gated 1x1 below dconv.hip's
// pixel count back to sconv.hip (A/B)
int g_gate = 1;

template <int PD>
int run_pd(int cfg, const GP &p, hipStream_t st) {
  switch (cfg) {
    case 1: return launch<128, 2, PD>(p, st);
    case 2: return launch<64, 2, PD>(p, st);
    case 3: return launch<32, 2, PD>(p, st);
    case 4: return launch<128, 1, PD>(p, st);
    case 5: return launch<64, 1, PD>(p, st);
    case 6: return launch<32, 1, PD>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}
// auto: 2 stages in flight.  Three buffers instead of four let two
// workgroups share a CU, and a second workgroup hides a tile's DMA latency
// and epilogue better than a deeper ring: measured on the codec's 1x1 layers
// (scripts/gpu_r03za.sh), 384 -> 384 at 68x120 25.5 -> 17.7 us, 96 -> 48 at
// 1080p 394 -> 272 us, 128 -> 64 at 544x960 148 -> 120 us
// gated input: the auto depth only
int run_gate(int cfg, const GP &p, hipStream_t st) {
  switch (cfg) {
    case 1: return launch<128, 2, 2, true>(p, st);
    case 2: return launch<64, 2, 2, true>(p, st);
    case 3: return launch<32, 2, 2, true>(p, st);
    case 4: return launch<128, 1, 2, true>(p, st);
    case 5: return launch<64, 1, 2, true>(p, st);
    case 6: return launch<32, 1, 2, true>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}
int run_cfg(int cfg, const GP &p, hipStream_t st) {
  if (p.in_op == DCVC_IN_GATE) return run_gate(cfg, p, st);
  const int pd = g_pd ? g_pd : 2;
  if (pd == 1) return run_pd<1>(cfg, p, st);
  if (pd == 2) return run_pd<2>(cfg, p, st);
  if (pd == 5) return run_pd<5>(cfg, p, st);
  return run_pd<3>(cfg, p, st);
}

}  // namespace

extern "C" void dcvc_internal_sgemm_cfg(int v) { g_cfg = v; }
extern "C" void dcvc_internal_sgemm_pd(int v) { g_pd = v; }
extern "C" void dcvc_internal_sgemm_gate(int v) { g_gate = v; }

// The f16x3 1x1 stride-1 convolutions sconv.hip hands over (no pad, no pixel
// shuffle with a gate, 8-channel aligned input, 4-channel aligned output pieces);
// DCVC_HIP_EUNSUPPORTED sends the call back to sconv.hip.
extern "C" int dcvc_internal_sgemm(const dcvc_conv_args *a, void *stream) {
  if (g_cfg < 0) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != 1 || a->kw != 1 || a->stride != 1 || a->pad != 0) return DCVC_HIP_EUNSUPPORTED;
  const bool gate = a->in_op == DCVC_IN_GATE;
  if (a->in_op != DCVC_IN_NONE && a->in_op != DCVC_IN_LRELU && !(gate && g_gate)) return DCVC_HIP_EUNSUPPORTED;
  // (the kernel's input leaky ReLU is max(v, s v): 0 <= s <= 1)
  if (a->in_op == DCVC_IN_LRELU && !(a->in_slope >= 0.f && a->in_slope <= 1.f)) return DCVC_HIP_EUNSUPPORTED;
  if (gate && a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  const int f = a->shuffle ? 2 : 1;
  if (a->x.H * f != a->y.H || a->x.W * f != a->y.W) return DCVC_HIP_EUNSUPPORTED;
  if (a->shuffle && (a->cout % 4 || a->y.C * 4 != a->cout)) return DCVC_HIP_EUNSUPPORTED;
  auto al = [](const void *ptr, int cs, int co) {
    return ptr == nullptr || ((uintptr_t)ptr % 16 == 0 && cs % 4 == 0 && co % 4 == 0);
  };
  if (a->cin % 8 || a->cout % 4 || !al(a->x.ptr, a->x.cstride, a->x.coff) || !al(a->y.ptr, a->y.cstride, a->y.coff) ||
      !al(a->res.ptr, a->res.cstride, a->res.coff) || !al(a->res2.ptr, a->res2.cstride, a->res2.coff))
    return DCVC_HIP_EUNSUPPORTED;
  if ((a->res.ptr && a->res.dtype != DCVC_F32) || (a->res2.ptr && a->res2.dtype != DCVC_F32))
    return DCVC_HIP_EUNSUPPORTED;
  GP p{};
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  const int64_t np = (int64_t)a->x.H * a->x.W;
  if (np <= 0) return DCVC_HIP_OK;
  if (np > 0x7fffffff - 256) return DCVC_HIP_EUNSUPPORTED;
  p.npix = (int)np;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.cin = a->cin;
  p.cout = a->cout;
  p.nchunks = (a->cin + 31) / 32;
  p.wchunk = (int64_t)2 * a->cout * 32;
  {
    const int64_t wb = (int64_t)p.nchunks * p.wchunk * 2;
    if (wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
    p.wbytes = (int)wb;
  }
  p.shuffle = a->shuffle ? 1 : 0;
  p.W = a->x.W;
  p.bias = a->bias;
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.in_op = a->in_op;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.scale = a->scale;
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
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (g_cfg > 0) return run_cfg(g_cfg, p, st);
  // auto: n-blocks by padded output channels (fewest first; 64 before 128 on
  // a tie); 2 pixel groups per wave while that still gives 8 workgroups per
  // CU, else 1.  scripts/gpu_r04q.sh (profiles/r04q_sgemm_ab.jsonl): 128 ->
  // 128 at 272x480 49.1 -> 37.0 us, 384 -> 384 at 68x120 18.4 -> 16.3 us, the
  // 1080p 1x1 layers unchanged (BN 128 never ahead)
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  int order[3] = {64, 128, 32};
  auto padded = [&](int bn) { return (p.cout + bn - 1) / bn * bn - p.cout; };
  for (int i = 0; i < 3; ++i)
    for (int j = i + 1; j < 3; ++j)
      if (padded(order[j]) < padded(order[i])) std::swap(order[i], order[j]);
  auto cfg_of = [](int bn, int pxw) { return (pxw == 2 ? 1 : 4) + (bn == 128 ? 0 : bn == 64 ? 1 : 2); };
  for (int pxw = 2; pxw >= 1; --pxw)
    for (int i = 0; i < 3; ++i) {
      const int bn = order[i];
      if (padded(bn) > padded(order[0])) break;
      const int64_t nt = (np + 64 * pxw - 1) / (64 * pxw) * ((p.cout + bn - 1) / bn);
      if (nt >= (pxw == 2 ? 8 : 1) * g_cus) return run_cfg(cfg_of(bn, pxw), p, st);
    }
  return run_cfg(cfg_of(order[0], 1), p, st);
}
