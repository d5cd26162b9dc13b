// Persistent fused DepthConvBlock (DCVC-DC/src/models/layers.py:135-222,
// non-gated ConvFFN) for the blocks whose whole weight set fits in LDS next
// to one tile's activations: the full-resolution recon UNet blocks (64->48,
// 48->32) and the half-resolution ones (64->64, 32->64).
//
// Same arithmetic as dcb.hip (one 8x16 output tile, t1 on the 10x18 halo,
// depthwise in fp32 from bf16 t1, dc rounded to bf16, FFN hidden layer in
// 64-channel slices), reorganised for the latency profile that kernel showed
// (1.2 ms for a 1080p 64->48 block at 0.39 TB/s: every phase restaged its
// weights from L2 between barriers, and every tile paid its own HBM round
// trip):
//   * one workgroup per CU walks tiles; every weight matrix, bias and
//     depthwise tap is staged into LDS once per launch;
//   * the next tile's halo input is loaded into registers (buffer loads,
//     zero outside the image) while the current tile runs its five phases;
//   * the adaptor reads the interior rows of the halo image in place.
// The MFMA K order and every rounding point are those of dcb.hip, so outputs
// are bit-identical to it (tests/test_gpu_kernels.py).
#include "common.h"

namespace {

constexpr int TH = 8, TW = 16;
constexpr int HW_ = TW + 2;
constexpr int NPH = (TH + 2) * HW_;          // 180 halo pixels
constexpr int NPH_T = (NPH + 15) / 16;       // 12 pixel tiles (192 rows)
constexpr int NPI = TH * TW;                 // 128 interior pixels
constexpr int NPI_T = NPI / 16;              // 8 pixel tiles
constexpr int NWV = 8;                       // waves: 2 per SIMD, so one wave's VALU phases
                                             // overlap the other's MFMA / LDS waits
constexpr int NTHR = NWV * 64;

struct DcbP {
  const uint16_t *x;
  int H, W, xcs, xco;
  uint16_t *y;
  int ycs, yco;
  const uint16_t *w1; int ld1; const float *b1;
  const float *wdw; const float *bdw;
  const uint16_t *w2; int ld2; const float *b2;
  const uint16_t *wa; int lda; const float *ba;
  const uint16_t *wf1; int ldf1; const float *bf1;
  const uint16_t *wf2; int ldf2; const float *bf2;
  const float *scale;
  float slope_dc, slope_ffn;
  int tiles_x, tiles_y, xbytes;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int RL>
__device__ __forceinline__ int img(int row, int ch) {
  constexpr int NS = RL / 8;
  constexpr int SH = RL == 32 ? 2 : (RL == 64 ? 1 : 0);
  constexpr int MSK = NS < 16 ? NS - 1 : 15;
  const int slot = ch >> 3;
  return row * RL + (((slot ^ ((row >> SH) & MSK)) & (NS - 1)) << 3) + (ch & 7);
}

template <int C>
constexpr int rl() { return C <= 32 ? 32 : (C <= 64 ? 64 : 128); }

// leaky ReLU as max(v, s * v): the same value as (v >= 0 ? v : s * v) for
// 0 <= s <= 1 (the host checks), in two VALU instructions instead of three
__device__ __forceinline__ float lrelu(float v, float s) { return fmaxf(v, v * s); }

template <int CIN, int COUT, bool ADAPT>
struct DG {
  static constexpr int RLI = rl<CIN>(), RLO = rl<COUT>();
  static constexpr int NTI = (CIN + 15) / 16, NTO = (COUT + 15) / 16;
  static constexpr int HID = 4 * COUT < 1024 ? (4 * COUT > 2 * COUT ? 4 * COUT : 2 * COUT) : 1024;
  static constexpr int NHS = HID / 64;       // hidden slices
  // weight images (elements)
  static constexpr int OW1 = 0;
  static constexpr int OW2 = OW1 + NTI * 16 * RLI;
  static constexpr int OWA = OW2 + NTO * 16 * RLI;
  static constexpr int OF1 = OWA + (ADAPT ? NTO * 16 * RLI : 0);
  static constexpr int OF2 = OF1 + HID * RLO;
  static constexpr int NW = OF2 + NHS * NTO * 16 * 64;
  // fp32 constants (floats)
  static constexpr int CB1 = 0, CB2 = CB1 + CIN, CBA = CB2 + COUT, CF1 = CBA + COUT, CF2 = CF1 + HID,
                       CSC = CF2 + COUT, CDW = CSC + COUT, NC = CDW + 10 * CIN;
  // activations (elements)
  static constexpr int XS = NPH_T * 16 * RLI, TS = NPH_T * 16 * RLI, DS = NPI * RLI;
  static constexpr bool CS_IN_TS = NPI * RLO <= TS;
  static constexpr bool HS_IN_DS = RLI >= 64;
  static constexpr int NA = XS + TS + DS + (CS_IN_TS ? 0 : NPI * RLO) + (HS_IN_DS ? 0 : NPI * 64);
  static constexpr size_t LDS = (size_t)NW * 2 + (size_t)NA * 2 + (size_t)NC * 4;
  static constexpr int QP = CIN / 8;
  static constexpr int PP = (NPH * QP + NTHR - 1) / NTHR;   // prefetch pieces per thread
  static_assert((NW + NA) % 8 == 0 && CDW % 4 == 0 && CIN % 4 == 0, "16-byte aligned depthwise taps");
};

// acc[i][j] += A[16j + ..][k] * B[row_i + col][k], k in [0, K)
template <int RLA, int RLB, int NPT, int NT>
__device__ __forceinline__ void mma(f32x4 (&acc)[NPT][NT], const uint16_t *imgb, const int (&rowb)[NPT],
                                    const uint16_t *Al, int K, int lane, int kb = 0) {
  const int col = lane & 15, hi = lane >> 4;
  for (int k0 = 0; k0 < K; k0 += 32) {
    bf16x8 a[NT], b[NPT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
      a[j] = *reinterpret_cast<const bf16x8 *>(Al + img<RLA>(j * 16 + col, k0 + hi * 8));
#pragma unroll
    for (int i = 0; i < NPT; ++i)
      b[i] = *reinterpret_cast<const bf16x8 *>(imgb + img<RLB>(rowb[i] + col, kb + k0 + hi * 8));
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[i], acc[i][j], 0, 0, 0);
  }
}

template <int RL>
__device__ __forceinline__ void put4(uint16_t *imgb, int row, int ch, const float v[4]) {
  u16x4 o;
  o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
  *reinterpret_cast<u16x4 *>(imgb + img<RL>(row, ch)) = o;
}

// rows [0, nrows) x channels [0, RL) of a packed [N][ld] matrix (columns
// [koff, koff + RL)) -> LDS image; zeros beyond nmax rows / ld columns
template <int RL>
__device__ __forceinline__ void stage_w(uint16_t *Wl, const uint16_t *W, int ld, int nrows, int nmax, int koff) {
  constexpr int NS = RL / 8;
  for (int it = threadIdx.x; it < nrows * NS; it += NTHR) {
    const int r = it / NS, s = it % NS;
    const int c = koff + s * 8;
    u16x8 v{};
    if (r < nmax && c < ld) v = *reinterpret_cast<const u16x8 *>(W + (int64_t)r * ld + c);
    *reinterpret_cast<u16x8 *>(Wl + img<RL>(r, s * 8)) = v;
  }
}

template <int CIN, int COUT, bool ADAPT>
__global__ void __launch_bounds__(NTHR) dcbp_kernel(DcbP p) {
  typedef DG<CIN, COUT, ADAPT> G_;
  constexpr int RLI = G_::RLI, RLO = G_::RLO, NTI = G_::NTI, NTO = G_::NTO, HID = G_::HID;
  constexpr int NTH = 4;  // 64 hidden channels per slice
  constexpr int QP = G_::QP, PP = G_::PP;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Wl = reinterpret_cast<uint16_t *>(smem);
  uint16_t *Xs = Wl + G_::NW;
  uint16_t *Ts = Xs + G_::XS;
  uint16_t *Ds = Ts + G_::TS;
  uint16_t *Cs = G_::CS_IN_TS ? Ts : Ds + G_::DS;
  uint16_t *Hs = G_::HS_IN_DS ? Ds : Ds + G_::DS + (G_::CS_IN_TS ? 0 : NPI * RLO);
  float *Lc = reinterpret_cast<float *>(Xs + G_::NA);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);  // consecutive tiles per XCD
  const int ntiles = p.tiles_x * p.tiles_y;
  if (g >= ntiles) return;

  // ---- prefetch plan: piece u = (halo pixel, 16-byte channel piece)
  int lofs[PP], pyx[PP], rel[PP];
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    const int it = tid + u * NTHR;
    lofs[u] = -1;
    pyx[u] = 0;
    rel[u] = 0;
    if (it < NPH * QP) {
      const int pix = it / QP, q = it - pix * QP;
      const int hy = pix / HW_, hx = pix - hy * HW_;
      lofs[u] = img<RLI>(pix, q * 8);
      pyx[u] = (hy << 8) | hx;
      rel[u] = ((hy - 1) * p.W + (hx - 1)) * p.xcs + p.xco + q * 8;
    }
  }
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.x), (short)0, p.xbytes, 0x00020000);
  u16x8 pf[PP];
  auto issue = [&](int t) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
    const int base = (oy0 * p.W + ox0) * p.xcs;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int gy = oy0 - 1 + (pyx[u] >> 8), gx = ox0 - 1 + (pyx[u] & 255);
      const bool in = lofs[u] >= 0 && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
      const int off = in ? (base + rel[u]) * 2 : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  issue(g);

  // ---- resident weights and constants (once per launch)
  stage_w<RLI>(Wl + G_::OW1, p.w1, p.ld1, NTI * 16, CIN, 0);
  stage_w<RLI>(Wl + G_::OW2, p.w2, p.ld2, NTO * 16, COUT, 0);
  if constexpr (ADAPT) stage_w<RLI>(Wl + G_::OWA, p.wa, p.lda, NTO * 16, COUT, 0);
  stage_w<RLO>(Wl + G_::OF1, p.wf1, p.ldf1, HID, HID, 0);
#pragma unroll 1
  for (int s = 0; s < G_::NHS; ++s) stage_w<64>(Wl + G_::OF2 + s * NTO * 16 * 64, p.wf2, p.ldf2, NTO * 16, COUT, s * 64);
  for (int i = tid; i < G_::NC; i += NTHR) {
    float v;
    if (i < G_::CB2) v = p.b1[i];
    else if (i < G_::CBA) v = p.b2[i - G_::CB2];
    else if (i < G_::CF1) v = ADAPT ? p.ba[i - G_::CBA] : 0.f;
    else if (i < G_::CF2) v = p.bf1[i - G_::CF1];
    else if (i < G_::CSC) v = p.bf2[i - G_::CF2];
    else if (i < G_::CDW) v = p.scale ? p.scale[i - G_::CSC] : 1.f;
    else v = i < G_::CDW + 9 * CIN ? p.wdw[i - G_::CDW] : p.bdw[i - G_::CDW - 9 * CIN];
    Lc[i] = v;
  }
  // channel padding of the input image stays zero for the whole launch
  if constexpr (RLI > CIN) {
    for (int it = tid; it < NPH_T * 16 * (RLI - CIN) / 8; it += NTHR) {
      const int row = it / ((RLI - CIN) / 8), s = it % ((RLI - CIN) / 8);
      *reinterpret_cast<u16x8 *>(Xs + img<RLI>(row, CIN + s * 8)) = u16x8{};
    }
  }
  const float *b1 = Lc + G_::CB1, *b2 = Lc + G_::CB2, *ba = Lc + G_::CBA, *bf1 = Lc + G_::CF1;
  const float *bf2 = Lc + G_::CF2, *sc = Lc + G_::CSC, *Dw = Lc + G_::CDW;

  constexpr int NPT = NPI_T / NWV;  // interior pixel tiles per wave
  int pt[NPT], rowi[NPT], rowh[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    pt[i] = wave + NWV * i;
    rowi[i] = pt[i] * 16;
    rowh[i] = (pt[i] + 1) * HW_ + 1;  // interior pixel tile -> its halo-image rows
  }

  for (int t = g;;) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
#pragma unroll
    for (int u = 0; u < PP; ++u)
      if (lofs[u] >= 0) *reinterpret_cast<u16x8 *>(Xs + lofs[u]) = pf[u];
    __syncthreads();
    const int tn = t + G;
    const bool more = tn < ntiles;
    if (more) issue(tn);

    // ---- P1: t1 = lrelu(conv1(x) + b1) on the halo (0 outside the image);
    // halo pixel tiles wave, wave + NWV, ... (wave-uniform bound)
#pragma unroll
    for (int ht = wave; ht < NPH_T; ht += NWV) {
      int rb[1] = {ht * 16};
      f32x4 acc[1][NTI];
#pragma unroll
      for (int j = 0; j < NTI; ++j) acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma<RLI, RLI, 1, NTI>(acc, Xs, rb, Wl + G_::OW1, CIN, lane);
      const int row = rb[0] + col;
      const int hy = row / HW_, hx = row % HW_;
      const int gy = oy0 - 1 + hy, gx = ox0 - 1 + hx;
      const bool inside = row < NPH && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
#pragma unroll
      for (int j = 0; j < RLI / 16; ++j) {
        const int c = j * 16 + hi * 4;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = (j < NTI && inside && c + q < CIN) ? lrelu(acc[0][j < NTI ? j : 0][q] + b1[c + q], p.slope_dc)
                                                      : 0.f;
        put4<RLI>(Ts, row, c, v);
      }
    }
    __syncthreads();

    // ---- P2: d = dw3x3(t1) + bdw on interior pixels: each thread a column
    // of RPT output pixels x 4 channels, every t1 value converted once
    {
      constexpr int NQ = RLI / 4, NRG = NTHR / (NQ * TW), RPT = TH / NRG;
      static_assert(NQ * TW * NRG == NTHR && RPT * NRG == TH, "depthwise tasks");
      const int dq = tid % NQ, dcol = (tid / NQ) % TW, drg = tid / (NQ * TW);
      if (dq * 4 < CIN) {
        float w[9][4], bias[4];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const float4 v = *reinterpret_cast<const float4 *>(Dw + k * CIN + dq * 4);
          w[k][0] = v.x; w[k][1] = v.y; w[k][2] = v.z; w[k][3] = v.w;
        }
        {
          const float4 v = *reinterpret_cast<const float4 *>(Dw + 9 * CIN + dq * 4);
          bias[0] = v.x; bias[1] = v.y; bias[2] = v.z; bias[3] = v.w;
        }
        float tv[3][3][4];   // rolling window: t1 row r in tv[r % 3]
        auto load_row = [&](int r) {
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) {
            const u16x4 v = *reinterpret_cast<const u16x4 *>(Ts + img<RLI>((drg * RPT + r) * HW_ + dcol + dx, dq * 4));
#pragma unroll
            for (int q = 0; q < 4; ++q) tv[r % 3][dx][q] = bf2f(v[q]);
          }
        };
        load_row(0);
        load_row(1);
#pragma unroll
        for (int o = 0; o < RPT; ++o) {
          load_row(o + 2);
          float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[q] = __builtin_fmaf(w[dy * 3 + dx][q], tv[(o + dy) % 3][dx][q], acc[q]);
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[q] + bias[q];
          u16x4 o4;
#pragma unroll
          for (int q = 0; q < 4; ++q) o4[q] = f2bf(v[q]);
          *reinterpret_cast<u16x4 *>(Ds + img<RLI>((drg * RPT + o) * TW + dcol, dq * 4)) = o4;
        }
      } else {
#pragma unroll
        for (int o = 0; o < RPT; ++o)
          *reinterpret_cast<u16x4 *>(Ds + img<RLI>((drg * RPT + o) * TW + dcol, dq * 4)) = u16x4{0, 0, 0, 0};
      }
    }
    __syncthreads();

    // ---- P3: dc = conv2(d) + b2 + (adaptor(x) + ba | x)
    f32x4 dc[NPT][NTO];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NTO; ++j) dc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma<RLI, RLI, NPT, NTO>(dc, Ds, rowi, Wl + G_::OW2, CIN, lane);
    if constexpr (ADAPT) {
      f32x4 ad[NPT][NTO];
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTO; ++j) ad[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma<RLI, RLI, NPT, NTO>(ad, Xs, rowh, Wl + G_::OWA, CIN, lane);
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTO; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = j * 16 + hi * 4 + q;
            if (c < COUT) dc[i][j][q] = bf2f(f2bf(ad[i][j][q] + ba[c])) + (dc[i][j][q] + b2[c]);
          }
    } else {
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTO; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = j * 16 + hi * 4 + q;
            if (c < COUT) dc[i][j][q] = (dc[i][j][q] + b2[c]) + bf2f(Xs[img<RLI>(rowh[i] + col, c)]);
          }
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int pix = rowi[i] + col;
#pragma unroll
      for (int j = 0; j < RLO / 16; ++j) {
        const int c = j * 16 + hi * 4;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = (j < NTO && c + q < COUT) ? dc[i][j < NTO ? j : 0][q] : 0.f;
          if (j < NTO) dc[i][j < NTO ? j : 0][q] = bf2f(f2bf(v[q]));
        }
        put4<RLO>(Cs, pix, c, v);
      }
    }
    // From here to P5 every wave touches only its own pixel tile's rows of
    // Cs, Ds / Hs and (read-only) Xs: a wave's LDS operations complete in
    // order, so P3 -> P4 -> P5 need no barriers, only wave-scope ordering.
    wave_lds_sync();

    // ---- P4: FFN over 64-channel hidden slices
    f32x4 acc[NPT][NTO];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NTO; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int s = 0; s < G_::NHS; ++s) {
      f32x4 hacc[NPT][NTH];
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTH; ++j) hacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma<RLO, RLO, NPT, NTH>(hacc, Cs, rowi, Wl + G_::OF1 + s * 64 * RLO, COUT, lane);
      wave_lds_sync();   // the previous slice's Hs reads before these writes
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTH; ++j) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = lrelu(hacc[i][j][q] + bf1[s * 64 + j * 16 + hi * 4 + q], p.slope_ffn);
          put4<64>(Hs, rowi[i] + col, j * 16 + hi * 4, v);
        }
      wave_lds_sync();   // Hs written before other lanes read it
      mma<64, 64, NPT, NTO>(acc, Hs, rowi, Wl + G_::OF2 + s * NTO * 16 * 64, 64, lane);
    }
    wave_lds_sync();   // P4's Cs reads before P5 overwrites the rows

    // ---- P5: out = dc + lrelu(acc + bf2) [* scale] -> Cs (bf16), whole-line stores
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int pix = rowi[i] + col;
#pragma unroll
      for (int j = 0; j < NTO; ++j) {
        const int c = j * 16 + hi * 4;
        if (c >= COUT) continue;
        u16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = lrelu(acc[i][j][q] + bf2[c + q], p.slope_ffn);
          v = dc[i][j][q] + v;
          if (p.scale) v = v * sc[c + q];
          o[q] = f2bf(v);
        }
        *reinterpret_cast<u16x4 *>(Cs + img<RLO>(pix, c)) = o;
      }
    }
    __syncthreads();   // every wave's output rows in Cs
    constexpr int NSO = COUT / 8;
    for (int it = tid; it < NPI * NSO; it += NTHR) {
      const int pix = it / NSO, s8 = (it % NSO) * 8;
      const int gy = oy0 + pix / TW, gx = ox0 + pix % TW;
      if (gy >= p.H || gx >= p.W) continue;
      *reinterpret_cast<u16x8 *>(p.y + ((int64_t)gy * p.W + gx) * p.ycs + p.yco + s8) =
          *reinterpret_cast<const u16x8 *>(Cs + img<RLO>(pix, s8));
    }
    if (!more) break;
    __syncthreads();  // Cs (aliasing Ts) read before the next tile's P1 writes Ts
    t = tn;
  }
}

int g_cus = 0;
int g_enabled = 1;

template <int CIN, int COUT, bool ADAPT>
int run(DcbP p, hipStream_t st) {
  typedef DG<CIN, COUT, ADAPT> G_;
  if constexpr (G_::LDS > 160 * 1024) {
    return DCVC_HIP_EUNSUPPORTED;
  } else {
    p.tiles_x = (p.W + TW - 1) / TW;
    p.tiles_y = (p.H + TH - 1) / TH;
    const int64_t ntiles = (int64_t)p.tiles_x * p.tiles_y;
    if (g_cus <= 0) {
      int dev = 0;
      hipDeviceProp_t prop;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return DCVC_HIP_ELAUNCH;
      g_cus = prop.multiProcessorCount;
    }
    if (ntiles < 2LL * g_cus) return DCVC_HIP_EUNSUPPORTED;  // small maps: per-tile kernel
    const int G = g_cus;
    auto kern = dcbp_kernel<CIN, COUT, ADAPT>;
    dcvc_note_kernel("dcbp_kernel<%d, %d, %s>@%lld", CIN, COUT, bname(ADAPT), (long long)G * NTHR);
    dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
    hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(NTHR), G_::LDS, st, p);
    DCVC_LAUNCH_CHECK();
    return DCVC_HIP_OK;
  }
}

}  // namespace

// Called by dcvc_depthconv_block (dcb.hip) after its argument checks, for
// non-gated blocks; DCVC_HIP_EUNSUPPORTED hands the call to dcb_kernel.
extern "C" int dcvc_internal_dcbp(const dcvc_dcb_args *a, void *stream) {
  if (!g_enabled || a->gated) return DCVC_HIP_EUNSUPPORTED;
  if (!(a->slope_dc >= 0.f && a->slope_dc <= 1.f && a->slope_ffn >= 0.f && a->slope_ffn <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;   // lrelu as max(v, s v)
  if ((int64_t)a->x.H * a->x.W * a->x.cstride >= ((int64_t)1 << 30) - 16) return DCVC_HIP_EUNSUPPORTED;
  const bool adapt = a->w_adaptor != nullptr;
  DcbP p{};
  p.x = reinterpret_cast<const uint16_t *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.xbytes = a->x.H * a->x.W * a->x.cstride * 2;
  p.y = reinterpret_cast<uint16_t *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.w1 = reinterpret_cast<const uint16_t *>(a->w_conv1); p.ld1 = a->ld_conv1; p.b1 = a->b_conv1;
  p.wdw = a->w_dw; p.bdw = a->b_dw;
  p.w2 = reinterpret_cast<const uint16_t *>(a->w_conv2); p.ld2 = a->ld_conv2; p.b2 = a->b_conv2;
  p.wa = reinterpret_cast<const uint16_t *>(a->w_adaptor); p.lda = a->ld_adaptor; p.ba = a->b_adaptor;
  p.wf1 = reinterpret_cast<const uint16_t *>(a->w_ffn1); p.ldf1 = a->ld_ffn1; p.bf1 = a->b_ffn1;
  p.wf2 = reinterpret_cast<const uint16_t *>(a->w_ffn2); p.ldf2 = a->ld_ffn2; p.bf2 = a->b_ffn2;
  p.scale = a->scale;
  p.slope_dc = a->slope_dc;
  p.slope_ffn = a->slope_ffn;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->cin == 64 && a->cout == 48 && adapt) return run<64, 48, true>(p, st);
  if (a->cin == 48 && a->cout == 32 && adapt) return run<48, 32, true>(p, st);
  if (a->cin == 32 && a->cout == 64 && adapt) return run<32, 64, true>(p, st);
  if (a->cin == 64 && a->cout == 64 && !adapt) return run<64, 64, false>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

// dcvc_set_option("dcb_persistent", 0/1) (A/B switch, via conv.hip)
extern "C" void dcvc_internal_dcbp_enable(int v) { g_enabled = v; }
