// Fused DepthConv in split-fp16 arithmetic (Precision.split()):
//   dc = conv2(dw3x3(lrelu(conv1(x) + b1)) + bdw) + b2 + (adaptor(x) + ba | x)
// DCVC-DC/src/models/layers.py:135-163 (DepthConv: 1x1 conv, LeakyReLU(0.01),
// depthwise 3x3 with zero padding, 1x1 conv, + identity).  Unfused this is
// two 1x1 convs, a depthwise pass and their fp32 intermediates through HBM;
// here one persistent 512-thread workgroup per CU walks 8 x 16 output tiles:
//   P1a (adaptor blocks) the adaptor on the tile's interior, kept in
//       registers (wave w owns interior row w);
//   P1b t1 = lrelu(conv1(x) + b1) on the 10 x 18 halo, 0 outside the image
//       (the depthwise conv's zero padding of t1), written in fp32 IN PLACE
//       over the split input image: conv1 is pointwise, and a 32-channel
//       chunk of a halo row keeps the bytes of that row's (hi, lo) input
//       pieces, so a wave only overwrites rows it has finished reading;
//   P2  the depthwise 3x3 in fp32 VALU, split into the image conv2 reads;
//   P3  conv2 + b2 + identity, stored fp32 straight from the accumulators
//       (the identity without an adaptor is x itself, re-read exactly).
// Every 1x1 product is three f16 MFMAs (sconv.hip's split).  All weights are
// resident in LDS for the launch (packed LDS images, dcvc_dc_pack_weights);
// the next tile's halo is loaded into registers while the current one runs.
#include "common.h"
#include "split.h"

namespace {

constexpr int kNW = 8, kNT = kNW * 64;
constexpr int TH = 8, TW = 16;
constexpr int HW_ = TW + 2, NPH = (TH + 2) * HW_;   // 180 halo pixels
constexpr int HR = 192;                              // halo rows in the images (12 pixel tiles)

struct DP {
  const float *x;
  int H, W, xcs, xco;
  float *y;
  int ycs, yco;
  const uint16_t *w;   // packed images: conv1 | conv2 | adaptor (hi, lo each)
  int wbytes;
  const float *b1, *wdw, *bdw, *b2, *ba;
  float slope;
  int tiles_x, ntiles;
  int *ovf;               // fp16 range guard (split.h SplitRange)
};

template <int CIN, int COUT, bool ADAPT>
struct DG {
  static constexpr int KCI = (CIN + 31) / 32;
  static constexpr int NTI = (CIN + 15) / 16, NTO = (COUT + 15) / 16;
  static constexpr int CI16 = NTI * 16, CO16 = NTO * 16;
  // weight images (halves): [kc][n][32], hi then lo
  static constexpr int W1 = KCI * CI16 * 32, W2 = KCI * CO16 * 32, WA = ADAPT ? KCI * CO16 * 32 : 0;
  static constexpr int NWH = 2 * (W1 + W2 + WA);             // halves of all weight images
  static constexpr int XI = KCI * HR * 32;                   // input image, hi or lo: [kc][row][32]
  static constexpr int DI = KCI * TH * TW * 32;              // depthwise output image, hi or lo
  static constexpr size_t OX = 0, OD = OX + (size_t)2 * XI * 2, OW = OD + (size_t)2 * DI * 2;
  static constexpr size_t OC = OW + (size_t)NWH * 2;         // b1 | bdw | wdw[9][CIN] | b2 | ba
  static constexpr int NC = CIN * 11 + 2 * COUT;
  static constexpr size_t LDS = OC + (size_t)NC * 4;
  static constexpr int QP = CIN / 8;
  static constexpr int PP = (NPH * QP + kNT - 1) / kNT;      // input pieces per thread
};

__device__ __forceinline__ float lrelu(float v, float s) { return fmaxf(v, v * s); }

template <int CIN, int COUT, bool ADAPT>
__global__ void __launch_bounds__(kNT) sdc_kernel(DP p) {
  SplitRange rg(p.ovf);
  typedef DG<CIN, COUT, ADAPT> G_;
  constexpr int KCI = G_::KCI, NTI = G_::NTI, NTO = G_::NTO, CO16 = G_::CO16, CI16 = G_::CI16;
  constexpr int XI = G_::XI, DI = G_::DI, QP = G_::QP, PP = G_::PP;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Xh = reinterpret_cast<uint16_t *>(smem + G_::OX), *Xl = Xh + XI;
  uint16_t *Dh = reinterpret_cast<uint16_t *>(smem + G_::OD), *Dl = Dh + DI;
  uint16_t *W1h = reinterpret_cast<uint16_t *>(smem + G_::OW), *W1l = W1h + G_::W1;
  uint16_t *W2h = W1l + G_::W1, *W2l = W2h + G_::W2;
  uint16_t *WAh = W2l + G_::W2, *WAl = WAh + G_::WA;
  float *Lb1 = reinterpret_cast<float *>(smem + G_::OC), *Lbdw = Lb1 + CIN, *Lwdw = Lbdw + CIN;
  float *Lb2 = Lwdw + 9 * CIN, *Lba = Lb2 + COUT;
  // t1 (fp32) in place over the input image: channel c of halo row r lives in
  // the bytes of chunk c / 32 of row r, the first 16 channels in the hi
  // piece's 64 bytes, the last 16 in the lo piece's
  auto t1p = [&](int r, int c) -> float * {
    return reinterpret_cast<float *>((c & 16) ? Xl : Xh) + (((c >> 5) * HR + r) * 16 + (c & 15));
  };

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);   // consecutive tiles per XCD
  if (g >= p.ntiles) return;

  // ---- resident weights (LDS-DMA of the packed images) and constants
  {
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
    constexpr int ND = G_::NWH * 2 / 1024;
    for (int i = wave; i < ND; i += kNW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)(W1h + i * 512), 16,
                                               i * 1024 + lane * 16, 0, 0, 0);
    for (int i = tid; i < G_::NC; i += kNT) {
      float v;
      if (i < CIN) v = p.b1[i];
      else if (i < 2 * CIN) v = p.bdw[i - CIN];
      else if (i < 11 * CIN) v = p.wdw[i - 2 * CIN];
      else if (i < 11 * CIN + COUT) v = p.b2[i - 11 * CIN];
      else v = ADAPT ? p.ba[i - 11 * CIN - COUT] : 0.f;
      Lb1[i] = v;
    }
  }

  // ---- halo prefetch plan: piece u = (halo pixel, 8-channel group)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(p.x), (short)0,
      (int)((int64_t)p.H * p.W * p.xcs * 4 < 0x7fff0000 ? (int64_t)p.H * p.W * p.xcs * 4 : 0x7fff0000), 0x00020000);
  int pyx[PP], prel[PP], pofs[PP];
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    const int it = tid + u * kNT;
    pyx[u] = -1;
    prel[u] = 0;
    pofs[u] = 0;
    if (it < NPH * QP) {
      const int pix = it / QP, q = it - pix * QP;
      const int hy = pix / HW_, hx = pix - hy * HW_;
      pyx[u] = (hy << 8) | hx;
      prel[u] = ((hy - 1) * p.W + (hx - 1)) * p.xcs + p.xco + q * 8;
      pofs[u] = swz((q >> 2) * HR + pix, q & 3);
    }
  }
  float pf[PP][8];
  auto prefetch = [&](int t) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
    const int base = oy0 * p.W + ox0;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int gy = oy0 - 1 + (pyx[u] >> 8), gx = ox0 - 1 + (pyx[u] & 255);
      const bool in = pyx[u] >= 0 && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
      const int o = in ? (base * p.xcs + prel[u]) * 4 : 0x7fffffe0;
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[u][j] = a[j];
        pf[u][4 + j] = b[j];
      }
    }
  };
  prefetch(g);

  // C % 32 != 0: the input image's padding channels of every halo row are zero
  // for every tile (P1b rewrites only the t1 bytes of channels < CIN)
  auto zero_pad = [&]() {
    if constexpr (CIN % 32 != 0) {
      constexpr int PADQ = KCI * 4 - QP;
      for (int it = tid; it < HR * PADQ; it += kNT) {
        const int row = it / PADQ, q = QP + it % PADQ;
        const int o = swz((q >> 2) * HR + row, q & 3);
        *reinterpret_cast<u32x4_t *>(Xh + o) = u32x4_t{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4_t *>(Xl + o) = u32x4_t{0u, 0u, 0u, 0u};
      }
    }
  };

  wait_vm_lgkm();   // resident weights, first halo
  for (int t = g; t < p.ntiles; t += G) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
    raw_barrier();    // the previous tile's P3 reads of D / P2 reads of t1 are done
    // ---- publish the halo (split) and prefetch the next one
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      u32x4_t h, l;
      rg.add8(pf[u]);
      split8(pf[u], h, l);
      if (pyx[u] >= 0) {
        *reinterpret_cast<u32x4_t *>(Xh + pofs[u]) = h;
        *reinterpret_cast<u32x4_t *>(Xl + pofs[u]) = l;
      }
    }
    zero_pad();
    wait_lgkm();
    raw_barrier();
    if (t + G < p.ntiles) prefetch(t + G);

    // ---- P1a: adaptor on the interior row of this wave (registers)
    f32x4 idn[NTO];
    if constexpr (ADAPT) {
      f32x4 am[NTO], ac[NTO];
#pragma unroll
      for (int j = 0; j < NTO; ++j) {
        am[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ac[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const int hr = (wave + 1) * HW_ + 1 + col;
#pragma unroll
      for (int kc = 0; kc < KCI; ++kc) {
        const int ob = swz(kc * HR + hr, hi);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Xh + ob), bl = *reinterpret_cast<const f16x8 *>(Xl + ob);
#pragma unroll
        for (int j = 0; j < NTO; ++j) {
          const int oa = swz(kc * CO16 + j * 16 + col, hi);
          const f16x8 ah = *reinterpret_cast<const f16x8 *>(WAh + oa), al = *reinterpret_cast<const f16x8 *>(WAl + oa);
          am[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, am[j], 0, 0, 0);
          ac[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, ac[j], 0, 0, 0);
          ac[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, ac[j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < NTO; ++j) {
        const int n = j * 16 + hi * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) idn[j][e] = (am[j][e] + ac[j][e] * kLoInv) + Lba[n + e < COUT ? n + e : 0];
      }
      wait_lgkm();
      raw_barrier();   // P1b overwrites the input image
    }

    // ---- P1b: t1 = lrelu(conv1(x) + b1) on the halo, in place
    for (int ht = wave; ht < HR / 16; ht += kNW) {
      f32x4 tm[NTI], tc[NTI];
#pragma unroll
      for (int j = 0; j < NTI; ++j) {
        tm[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        tc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const int r = ht * 16 + col;
#pragma unroll
      for (int kc = 0; kc < KCI; ++kc) {
        const int ob = swz(kc * HR + r, hi);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Xh + ob), bl = *reinterpret_cast<const f16x8 *>(Xl + ob);
#pragma unroll
        for (int j = 0; j < NTI; ++j) {
          const int oa = swz(kc * CI16 + j * 16 + col, hi);
          const f16x8 ah = *reinterpret_cast<const f16x8 *>(W1h + oa), al = *reinterpret_cast<const f16x8 *>(W1l + oa);
          tm[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, tm[j], 0, 0, 0);
          tc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, tc[j], 0, 0, 0);
          tc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, tc[j], 0, 0, 0);
        }
      }
      const int hy = r / HW_, hx = r - hy * HW_;
      const int gy = oy0 - 1 + hy, gx = ox0 - 1 + hx;
      const bool inside = r < NPH && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
      wave_lds_sync();   // every lane of the wave has read its rows before any is overwritten
#pragma unroll
      for (int j = 0; j < NTI; ++j) {
        const int n = j * 16 + hi * 4;
        if (n >= CIN) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = inside ? lrelu((tm[j][e] + tc[j][e] * kLoInv) + Lb1[n + e], p.slope) : 0.f;
        *reinterpret_cast<f32x4 *>(t1p(r, n)) = v;
      }
    }
    wait_lgkm();
    raw_barrier();

    // ---- P2: d = dw3x3(t1) + bdw, split into D.  Thread task = (4-channel
    // group, column, run of RR output rows): a 3 x 3 window of t1 pieces
    // slides down the run (3 LDS reads per output row, not 9) and the group's
    // 9 tap weights stay in registers for the run; per output the taps in
    // (dy, dx) order, then the bias
    {
      constexpr int CG = CIN / 4;
      constexpr int R = kNT / (CG * TW) >= 4 ? 4 : kNT / (CG * TW) >= 2 ? 2 : 1;   // runs per column
      constexpr int RR = TH / R;
      static_assert(CG * TW * R <= kNT && TH % R == 0, "P2 tasks");
      if (tid < CG * TW * R) {
        const int cg = tid % CG, rest = tid / CG;
        const int ix = rest % TW, y0 = (rest / TW) * RR;
        const int c = cg * 4;
        f32x4 wv[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) wv[k] = *reinterpret_cast<const f32x4 *>(Lwdw + k * CIN + c);
        const float4 bd = *reinterpret_cast<const float4 *>(Lbdw + c);
        f32x4 win[3][3];   // [halo row mod 3][dx]
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            win[r][dx] = *reinterpret_cast<const f32x4 *>(t1p((y0 + r) * HW_ + ix + dx, c));
#pragma unroll
        for (int i = 0; i < RR; ++i) {
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            win[(i + 2) % 3][dx] = *reinterpret_cast<const f32x4 *>(t1p((y0 + i + 2) * HW_ + ix + dx, c));
          f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
              for (int e = 0; e < 4; ++e) a[e] = __builtin_fmaf(wv[dy * 3 + dx][e], win[(i + dy) % 3][dx][e], a[e]);
          float v[4];
          v[0] = a[0] + bd.x;
          v[1] = a[1] + bd.y;
          v[2] = a[2] + bd.z;
          v[3] = a[3] + bd.w;
          rg.add4(v);
          const auto h01 = __builtin_amdgcn_cvt_pkrtz(v[0], v[1]);
          const auto h23 = __builtin_amdgcn_cvt_pkrtz(v[2], v[3]);
          const uint32_t l01 = pk(split_lo(v[0], (float)h01[0]), split_lo(v[1], (float)h01[1]));
          const uint32_t l23 = pk(split_lo(v[2], (float)h23[0]), split_lo(v[3], (float)h23[1]));
          const int px = (y0 + i) * TW + ix;
          const int o = swz((c >> 5) * (TH * TW) + px, (c & 31) >> 3) + (c & 7);
          typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u32x2_t *>(Dh + o) = u32x2_t{__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23)};
          *reinterpret_cast<u32x2_t *>(Dl + o) = u32x2_t{l01, l23};
        }
      }
      if constexpr (CIN % 32 != 0) {   // D's padding channels: zero
        constexpr int PADQ = KCI * 4 - CIN / 8;
        for (int it = tid; it < TH * TW * PADQ; it += kNT) {
          const int px = it / PADQ, q = CIN / 8 + it % PADQ;
          const int o = swz((q >> 2) * (TH * TW) + px, q & 3);
          *reinterpret_cast<u32x4_t *>(Dh + o) = u32x4_t{0u, 0u, 0u, 0u};
          *reinterpret_cast<u32x4_t *>(Dl + o) = u32x4_t{0u, 0u, 0u, 0u};
        }
      }
    }
    wait_lgkm();
    raw_barrier();

    // ---- P3: dc = conv2(d) + b2 + identity on interior row `wave`
    {
      f32x4 cm[NTO], cc[NTO];
#pragma unroll
      for (int j = 0; j < NTO; ++j) {
        cm[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        cc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int kc = 0; kc < KCI; ++kc) {
        const int ob = swz(kc * (TH * TW) + wave * TW + col, hi);
        const f16x8 bh = *reinterpret_cast<const f16x8 *>(Dh + ob), bl = *reinterpret_cast<const f16x8 *>(Dl + ob);
#pragma unroll
        for (int j = 0; j < NTO; ++j) {
          const int oa = swz(kc * CO16 + j * 16 + col, hi);
          const f16x8 ah = *reinterpret_cast<const f16x8 *>(W2h + oa), al = *reinterpret_cast<const f16x8 *>(W2l + oa);
          cm[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, cm[j], 0, 0, 0);
          cc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, cc[j], 0, 0, 0);
          cc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, cc[j], 0, 0, 0);
        }
      }
      const int gy = oy0 + wave, gx = ox0 + col;
      if (gy < p.H && gx < p.W) {
        const int64_t pix = (int64_t)gy * p.W + gx;
#pragma unroll
        for (int j = 0; j < NTO; ++j) {
          const int n = j * 16 + hi * 4;
          if (n >= COUT) continue;
          f32x4 id;
          if constexpr (ADAPT) id = idn[j];
          else id = *reinterpret_cast<const f32x4 *>(p.x + pix * p.xcs + p.xco + n);
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ((cm[j][e] + cc[j][e] * kLoInv) + Lb2[n + e]) + id[e];
          *reinterpret_cast<f32x4 *>(p.y + pix * p.ycs + p.yco + n) = v;
        }
      }
    }
  }
  wait_vm_lgkm();
}

int g_cus = 0;

template <int CIN, int COUT, bool ADAPT>
int run(DP p, hipStream_t st) {
  typedef DG<CIN, COUT, ADAPT> G_;
  static_assert(G_::LDS <= 160 * 1024, "LDS");
  static_assert(G_::NWH * 2 % 1024 == 0, "weight images in whole 1-KiB pieces");
  p.tiles_x = (p.W + TW - 1) / TW;
  const int64_t nt = (int64_t)p.tiles_x * ((p.H + TH - 1) / TH);
  if (nt <= 0) return DCVC_HIP_OK;
  p.ntiles = (int)nt;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  int G = g_cus;
  if (G > p.ntiles) G = p.ntiles;
  auto kern = sdc_kernel<CIN, COUT, ADAPT>;
  dcvc_note_kernel("sdc_kernel<%d, %d, %s>@%lld", CIN, COUT, bname(ADAPT), (long long)G * kNT);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(kNT), G_::LDS, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

bool supported(int cin, int cout, bool adapt) {
  return (cin == 64 && cout == 48 && adapt) || (cin == 48 && cout == 32 && adapt) ||
         (cin == 64 && cout == 64 && !adapt) || (cin == 32 && cout == 64 && adapt) ||
         (cin == 48 && cout == 48 && !adapt) || (cin == 32 && cout == 32 && !adapt);
}

}  // namespace

// Packed DepthConv weights: the LDS images sdc_kernel reads, conv1 (w1
// [cin][cin]), conv2 (w2 [cout][cin]) and, if wa, the adaptor ([cout][cin]),
// each as hi then lo [kc][n padded to 16][32] with swizzled 16-byte slots.
// out NULL: size query (halves).
extern "C" int64_t dcvc_dc_pack_weights(const float *w1, const float *w2, const float *wa, int cin, int cout,
                                        void *out) {
  if (!w1 || !w2 || cin <= 0 || cout <= 0) return DCVC_HIP_EINVAL;
  if (out && (!host_split_range_ok(w1, (int64_t)cin * cin) || !host_split_range_ok(w2, (int64_t)cout * cin) ||
              (wa && !host_split_range_ok(wa, (int64_t)cout * cin))))
    return DCVC_HIP_EINVAL;
  const int kci = (cin + 31) / 32, ci16 = (cin + 15) / 16 * 16, co16 = (cout + 15) / 16 * 16;
  const int64_t n1 = (int64_t)kci * ci16 * 32, n2 = (int64_t)kci * co16 * 32, na = wa ? n2 : 0;
  const int64_t total = 2 * (n1 + n2 + na);
  if (!out) return total;
  uint16_t *o = reinterpret_cast<uint16_t *>(out);
  auto at = [](int row, int k) {
    const int x = (0x1320 >> (((row >> 2) & 3) << 2)) & 3;
    return (int64_t)row * 32 + ((((k >> 3) ^ x) & 3) << 3) + (k & 7);
  };
  auto put = [&](uint16_t *img, int64_t n, const float *w, int rows, int rows16) {
    for (int kc = 0; kc < kci; ++kc)
      for (int r = 0; r < rows16; ++r)
        for (int k = 0; k < 32; ++k) {
          const int ch = kc * 32 + k;
          const float v = (r < rows && ch < cin) ? w[(int64_t)r * cin + ch] : 0.f;
          const int64_t q = at(kc * rows16 + r, k);
          host_split(v, img[q], img[n + q]);
        }
  };
  put(o, n1, w1, cin, ci16);
  put(o + 2 * n1, n2, w2, cout, co16);
  if (wa) put(o + 2 * n1 + 2 * n2, na, wa, cout, co16);
  return total;
}

extern "C" int dcvc_depth_conv_split(const dcvc_dc_args *a, void *stream) {
  if (!a || !a->x.ptr || !a->y.ptr || !a->w || !a->b1 || !a->wdw || !a->bdw || !a->b2) return DCVC_HIP_EINVAL;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32 || a->x.C != a->cin || a->y.C != a->cout ||
      a->x.H != a->y.H || a->x.W != a->y.W)
    return DCVC_HIP_EINVAL;
  const bool adapt = a->adaptor != 0;
  if (!supported(a->cin, a->cout, adapt) || (adapt && !a->ba)) return DCVC_HIP_EUNSUPPORTED;
  if (!(a->slope >= 0.f && a->slope <= 1.f)) return DCVC_HIP_EUNSUPPORTED;   // lrelu as max(v, s v)
  if (a->x.cstride % 4 || a->x.coff % 4 || a->y.cstride % 4 || a->y.coff % 4 || ((uintptr_t)a->x.ptr & 15) ||
      ((uintptr_t)a->y.ptr & 15))
    return DCVC_HIP_EUNSUPPORTED;
  // (the kernel clamps the input's buffer record to 0x7fff0000 bytes)
  if ((int64_t)a->x.H * a->x.W * a->x.cstride * 4 >= 0x7fff0000) return DCVC_HIP_EUNSUPPORTED;
  DP p{};
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.wbytes = (int)(dcvc_dc_pack_weights(reinterpret_cast<const float *>(1), reinterpret_cast<const float *>(1),
                                        adapt ? reinterpret_cast<const float *>(1) : nullptr, a->cin, a->cout,
                                        nullptr) * 2);
  p.b1 = a->b1;
  p.wdw = a->wdw;
  p.bdw = a->bdw;
  p.b2 = a->b2;
  p.ba = a->ba;
  p.slope = a->slope;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->cin == 64 && a->cout == 48) return run<64, 48, true>(p, st);
  if (a->cin == 48 && a->cout == 32) return run<48, 32, true>(p, st);
  if (a->cin == 32 && a->cout == 64) return run<32, 64, true>(p, st);
  if (a->cin == 64 && a->cout == 64) return run<64, 64, false>(p, st);
  if (a->cin == 48 && a->cout == 48) return run<48, 48, false>(p, st);
  return run<32, 32, false>(p, st);
}
