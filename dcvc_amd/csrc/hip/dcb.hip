// Fused DepthConvBlock / DepthConvBlock2 (DCVC-DC/src/models/layers.py:135-222)
// for feature-domain channel counts (<= 128), one kernel per block:
//
//   t1  = lrelu(conv1x1(x) + b1)                 on an 10x18 halo tile
//   d   = dwconv3x3(t1) + bdw                    (zero padding at image edges)
//   dc  = conv1x1(d) + b2 + [adaptor(x) | x]     (DepthConv)
//   out = dc + lrelu(W2 lrelu(W1 dc + bf1) + bf2)            (ConvFFN)
//   out = dc + W2 (x1 * lrelu(x2)) + bf2, [x1|x2] = W1 dc    (ConvFFN2, gated)
//   out *= scale[c]                              (optional quant_step)
//
// One workgroup = 4 waves owns an 8x16-pixel output tile.  The input tile,
// t1, d, dc and one 64-wide slice of the FFN hidden layer live in LDS as
// bf16 [pixel][channel] images (16-byte slots XOR-swizzled per row); each
// phase's weights are staged through an LDS image 64 input channels at a
// time (L2-hot: every workgroup reads the same few KB), the output tile is
// assembled in LDS and written with whole-line 16-byte stores.
// HBM traffic is one read of x (with halo) and one write of out: the 4x-wide
// FFN intermediate and the three other intermediates never leave the CU.
// Every GEMM is D[n][pixel] = W[n][k] X[pixel][k] on v_mfma_f32_16x16x32_bf16;
// wave w owns pixel tiles {w, w+4, ...} and all n tiles of its phase.
#include "common.h"

namespace {

constexpr int TH = 8, TW = 16;               // output tile
constexpr int HH = TH + 2, HW_ = TW + 2;     // halo tile
constexpr int NPH = HH * HW_;                // 180 halo pixels
constexpr int NPH_T = (NPH + 15) / 16;       // 12 pixel tiles (192 rows)
constexpr int NPI = TH * TW;                 // 128 interior pixels
constexpr int NPI_T = NPI / 16;              // 8 pixel tiles

struct DcbP {
  const uint16_t *x;
  int H, W, xcs, xco;
  uint16_t *y;
  int ycs, yco;
  const uint16_t *w1; int ld1; const float *b1;      // conv1   [CIN][ld1]
  const float *wdw; const float *bdw;                // dw      [9][CIN]
  const uint16_t *w2; int ld2; const float *b2;      // conv2   [COUT][ld2]
  const uint16_t *wa; int lda; const float *ba;      // adaptor [COUT][lda] or null
  const uint16_t *wf1; int ldf1; const float *bf1;   // ffn in  [HID|4C][ldf1]
  const uint16_t *wf2; int ldf2; const float *bf2;   // ffn out [COUT][ldf2]
  const float *scale;
  float slope_dc, slope_ffn;
  int tiles_x;
};

// LDS image with rows of RL bf16 channels (RL in {32, 64, 128}); the 16-byte
// slot index is XORed with a row-dependent value so that the 16 rows read by
// one MFMA operand land in distinct bank groups.
template <int RL>
__device__ __forceinline__ int img(int row, int ch) {
  constexpr int NS = RL / 8;                         // slots per row
  constexpr int SH = RL == 32 ? 2 : (RL == 64 ? 1 : 0);
  constexpr int MSK = NS < 16 ? NS - 1 : 15;
  const int slot = ch >> 3;
  return row * RL + (((slot ^ ((row >> SH) & MSK)) & (NS - 1)) << 3) + (ch & 7);
}

template <int C>
constexpr int rl() { return C <= 32 ? 32 : (C <= 64 ? 64 : 128); }

template <int CIN, int COUT>
constexpr bool kAlias() { return NPI * rl<COUT>() + NPI * 64 <= NPH_T * 16 * rl<CIN>(); }

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// elements of the weight image: up to 128 rows x 64 input channels
template <int CIN, int COUT, bool GATED>
constexpr int kWl() {
  return cmax(cmax((CIN + 15) / 16 * 16, (COUT + 15) / 16 * 16), (GATED ? 2 : 1) * 64) * 64;
}

__device__ __forceinline__ float lrelu(float v, float s) { return v >= 0.f ? v : v * s; }

// Cooperatively copy weight rows [n0, n0 + nrows) x channels [0, RL) of a
// packed [N][ldw] bf16 matrix into an LDS image (zeros for rows >= nmax and
// channels >= ldw); kB loads are kept in flight per thread.
template <int RL>
__device__ __forceinline__ void load_w(uint16_t *Wl, const uint16_t *W, int ldw, int n0, int nrows, int nmax,
                                       int koff = 0) {
  constexpr int NS = RL / 8;
  constexpr int kB = 8;
  const int items = nrows * NS;
  for (int base = threadIdx.x; base < items; base += 256 * kB) {
    u16x8 v[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int it = base + u * 256;
      const int r = it / NS, s = it % NS;
      const int n = n0 + r, c = koff + s * 8;
      v[u] = u16x8{};
      if (it < items && n < nmax && c < ldw) v[u] = *reinterpret_cast<const u16x8 *>(W + (int64_t)n * ldw + c);
    }
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int it = base + u * 256;
      if (it < items) *reinterpret_cast<u16x8 *>(Wl + img<RL>(it / NS, (it % NS) * 8)) = v[u];
    }
  }
}

// acc[i][j] += A[16j + ..][k] * B[pixel tile pt_i][k], k in [0, K): both
// operands are LDS images (A rows = output channels, B rows = pixels)
template <int RLA, int RLB, int NPT, int NT>
__device__ __forceinline__ void mma(f32x4 (&acc)[NPT][NT], const uint16_t *imgb, const int (&pt)[NPT],
                                    const uint16_t *Al, int K, int lane, int kb = 0) {
  const int col = lane & 15, hi = lane >> 4;
  for (int k0 = 0; k0 < K; k0 += 32) {
    bf16x8 a[NT], b[NPT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
      a[j] = *reinterpret_cast<const bf16x8 *>(Al + img<RLA>(j * 16 + col, k0 + hi * 8));
#pragma unroll
    for (int i = 0; i < NPT; ++i)
      b[i] = *reinterpret_cast<const bf16x8 *>(imgb + img<RLB>(pt[i] * 16 + col, kb + k0 + hi * 8));
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[i], acc[i][j], 0, 0, 0);
  }
}

// GEMM against a weight matrix streamed through LDS 64 input channels at a
// time: rows [n0, n0 + nrows) of the packed [N][ldw] matrix, K channels.
// Starts and ends with a workgroup barrier (Wl is reused between phases).
template <int RLB, int NPT, int NT>
__device__ __forceinline__ void mma_w(f32x4 (&acc)[NPT][NT], const uint16_t *imgb, const int (&pt)[NPT],
                                      uint16_t *Wl, const uint16_t *W, int ldw, int n0, int nrows, int nmax,
                                      int K, int lane) {
  for (int kc = 0; kc < K; kc += 64) {
    __syncthreads();
    load_w<64>(Wl, W, ldw, n0, nrows, nmax, kc);
    __syncthreads();
    mma<64, RLB, NPT, NT>(acc, imgb, pt, Wl, K - kc < 64 ? K - kc : 64, lane, kc);
  }
  __syncthreads();
}

// write 4 consecutive channels (lane's D fragment) of pixel row `row` into an image
template <int RL>
__device__ __forceinline__ void put4(uint16_t *imgb, int row, int ch, const float v[4]) {
  u16x4 o;
  o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
  *reinterpret_cast<u16x4 *>(imgb + img<RL>(row, ch)) = o;
}

template <int CIN, int COUT, bool GATED, bool ADAPT>
__global__ void __launch_bounds__(256) dcb_kernel(DcbP p) {
  constexpr int RLI = rl<CIN>(), RLO = rl<COUT>();
  constexpr int NTI = (CIN + 15) / 16, NTO = (COUT + 15) / 16;
  constexpr int HID = GATED ? 2 * COUT : (4 * COUT < 1024 ? (4 * COUT > 2 * COUT ? 4 * COUT : 2 * COUT) : 1024);
  constexpr int HC = HID < 64 ? HID : 64;            // hidden channels per slice
  constexpr int NTH = HC / 16;
  static_assert(HID % HC == 0, "hidden slicing");
  extern __shared__ __align__(16) unsigned char smem[];
  // Xs [192][RLI] input (halo) | Ts [192][RLI] t1 (halo) | Ds [128][RLI] dw out;
  // dc (Cs [128][RLO]) and the hidden slice (Hs [128][64]) reuse Ts once the
  // depthwise pass is done, when they fit there.
  uint16_t *Xs = reinterpret_cast<uint16_t *>(smem);
  uint16_t *Ts = Xs + NPH_T * 16 * RLI;
  uint16_t *Ds = Ts + NPH_T * 16 * RLI;
  uint16_t *Cs = kAlias<CIN, COUT>() ? Ts : Ds + NPI * RLI;
  uint16_t *Hs = Cs + NPI * RLO;
  uint16_t *Wl = kAlias<CIN, COUT>() ? Ds + NPI * RLI : Hs + NPI * 64;   // phase weights
  float *Dw = reinterpret_cast<float *>(Wl + kWl<CIN, COUT, GATED>());  // [9][CIN] taps, [CIN] bias

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int tx = blockIdx.x % p.tiles_x, ty = blockIdx.x / p.tiles_x;
  const int ox0 = tx * TW, oy0 = ty * TH;

  // ---- P0: halo input tile -> Xs (zeros outside the image / beyond CIN)
  for (int it = threadIdx.x; it < NPH_T * 16 * (RLI / 8); it += 256) {
    const int row = it / (RLI / 8), s = it % (RLI / 8);
    const int hy = row / HW_, hx = row % HW_;
    const int gy = oy0 - 1 + hy, gx = ox0 - 1 + hx;
    u16x8 v{};
    if (row < NPH && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W && s * 8 < CIN)
      v = *reinterpret_cast<const u16x8 *>(p.x + ((int64_t)gy * p.W + gx) * p.xcs + p.xco + s * 8);
    *reinterpret_cast<u16x8 *>(Xs + img<RLI>(row, s * 8)) = v;
  }
  for (int it = threadIdx.x; it < 10 * CIN; it += 256) Dw[it] = it < 9 * CIN ? p.wdw[it] : p.bdw[it - 9 * CIN];
  __syncthreads();

  // ---- P1: t1 = lrelu(conv1(x) + b1) on all halo pixels (0 outside the image)
  {
    constexpr int NPT = NPH_T / 4;  // 3 pixel tiles per wave
    int pt[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) pt[i] = wave + 4 * i;
    f32x4 acc[NPT][NTI];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NTI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma_w<RLI, NPT, NTI>(acc, Xs, pt, Wl, p.w1, p.ld1, 0, NTI * 16, CIN, CIN, lane);
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int row = pt[i] * 16 + col;
      const int hy = row / HW_, hx = row % HW_;
      const int gy = oy0 - 1 + hy, gx = ox0 - 1 + hx;
      const bool inside = row < NPH && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
#pragma unroll
      for (int j = 0; j < RLI / 16; ++j) {
        const int c = j * 16 + hi * 4;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = (j < NTI && inside && c + q < CIN) ? lrelu(acc[i][j < NTI ? j : 0][q] + p.b1[c + q], p.slope_dc)
                                                      : 0.f;
        put4<RLI>(Ts, row, c, v);
      }
    }
  }
  __syncthreads();

  // ---- P2: d = dw3x3(t1) + bdw on interior pixels (8 channels per item)
  for (int it = threadIdx.x; it < NPI * (RLI / 8); it += 256) {
    const int pix = it / (RLI / 8), s = it % (RLI / 8);
    const int r = pix / TW, c = pix % TW;
    float acc[8];
    u16x8 o{};
    if (s * 8 < CIN) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const u16x8 t = *reinterpret_cast<const u16x8 *>(Ts + img<RLI>((r + dy) * HW_ + c + dx, s * 8));
          const float *w = Dw + (dy * 3 + dx) * CIN + s * 8;
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] += w[q] * bf2f(t[q]);
        }
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q] + Dw[9 * CIN + s * 8 + q]);
    }
    *reinterpret_cast<u16x8 *>(Ds + img<RLI>(pix, s * 8)) = o;
  }
  __syncthreads();

  // ---- P3: dc = conv2(d) + b2 + identity
  constexpr int NPT = NPI_T / 4;  // 2 pixel tiles per wave
  int pt[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) pt[i] = wave + 4 * i;
  f32x4 dc[NPT][NTO];
#pragma unroll
  for (int i = 0; i < NPT; ++i)
#pragma unroll
    for (int j = 0; j < NTO; ++j) dc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mma_w<RLI, NPT, NTO>(dc, Ds, pt, Wl, p.w2, p.ld2, 0, NTO * 16, COUT, CIN, lane);
  if constexpr (ADAPT) {
    // adaptor(x) on interior pixels: gather the interior rows of Xs into Ds
    for (int it = threadIdx.x; it < NPI * (RLI / 8); it += 256) {
      const int pix = it / (RLI / 8), s = it % (RLI / 8);
      const int r = pix / TW, c = pix % TW;
      *reinterpret_cast<u16x8 *>(Ds + img<RLI>(pix, s * 8)) =
          *reinterpret_cast<const u16x8 *>(Xs + img<RLI>((r + 1) * HW_ + c + 1, s * 8));
    }
    __syncthreads();
    f32x4 ad[NPT][NTO];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NTO; ++j) ad[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma_w<RLI, NPT, NTO>(ad, Ds, pt, Wl, p.wa, p.lda, 0, NTO * 16, COUT, CIN, lane);
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NTO; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = j * 16 + hi * 4 + q;
          if (c < COUT) dc[i][j][q] = bf2f(f2bf(ad[i][j][q] + p.ba[c])) + (dc[i][j][q] + p.b2[c]);
        }
  } else {
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int pix = pt[i] * 16 + col;
      const int r = pix / TW, cc = pix % TW;
#pragma unroll
      for (int j = 0; j < NTO; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = j * 16 + hi * 4 + q;
          if (c < COUT)
            dc[i][j][q] = (dc[i][j][q] + p.b2[c]) + bf2f(Xs[img<RLI>((r + 1) * HW_ + cc + 1, c)]);
        }
    }
  }
  // dc as bf16 (the precision the unfused path stores it in) -> Cs, and
  // keep that rounded value as the FFN residual
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int pix = pt[i] * 16 + col;
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
  __syncthreads();

  // ---- P4: FFN over hidden slices of HC channels
  f32x4 acc[NPT][NTO];
#pragma unroll
  for (int i = 0; i < NPT; ++i)
#pragma unroll
    for (int j = 0; j < NTO; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int h0 = 0; h0 < HID; h0 += HC) {
    f32x4 hacc[NPT][NTH];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NTH; ++j) hacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma_w<RLO, NPT, NTH>(hacc, Cs, pt, Wl, p.wf1, p.ldf1, h0, HC, h0 + HC, COUT, lane);
    if constexpr (GATED) {
      f32x4 gacc[NPT][NTH];
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTH; ++j) gacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma_w<RLO, NPT, NTH>(gacc, Cs, pt, Wl, p.wf1, p.ldf1, HID + h0, HC, HID + h0 + HC, COUT, lane);
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTH; ++j) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int h = h0 + j * 16 + hi * 4 + q;
            // the unfused path stores conv(dc) in bf16 before gating it
            v[q] = bf2f(f2bf(hacc[i][j][q] + p.bf1[h])) *
                   lrelu(bf2f(f2bf(gacc[i][j][q] + p.bf1[HID + h])), p.slope_ffn);
          }
          put4<64>(Hs, pt[i] * 16 + col, j * 16 + hi * 4, v);
        }
    } else {
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NTH; ++j) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = lrelu(hacc[i][j][q] + p.bf1[h0 + j * 16 + hi * 4 + q], p.slope_ffn);
          put4<64>(Hs, pt[i] * 16 + col, j * 16 + hi * 4, v);
        }
    }
    // acc += W2[:, h0:h0+HC] . hidden slice (mma_w's leading barrier publishes Hs)
    f32x4 (&accr)[NPT][NTO] = acc;
    {
      __syncthreads();
      load_w<64>(Wl, p.wf2, p.ldf2, 0, NTO * 16, COUT, h0);
      __syncthreads();
      mma<64, 64, NPT, NTO>(accr, Hs, pt, Wl, HC, lane);
      __syncthreads();
    }
  }

  // ---- P5: out = dc + act(acc + bf2) [* scale] as bf16 -> Cs (free since
  // the last FFN slice's trailing barrier), then whole-line stores to y
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int pix = pt[i] * 16 + col;
#pragma unroll
    for (int j = 0; j < NTO; ++j) {
      const int c = j * 16 + hi * 4;
      if (c >= COUT) continue;
      u16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float t = acc[i][j][q] + p.bf2[c + q];
        if (!GATED) t = lrelu(t, p.slope_ffn);
        t = dc[i][j][q] + t;
        if (p.scale) t = t * p.scale[c + q];
        o[q] = f2bf(t);
      }
      *reinterpret_cast<u16x4 *>(Cs + img<RLO>(pix, c)) = o;
    }
  }
  __syncthreads();
  constexpr int NSO = COUT / 8;
  for (int it = threadIdx.x; it < NPI * NSO; it += 256) {
    const int pix = it / NSO, s8 = (it % NSO) * 8;
    const int gy = oy0 + pix / TW, gx = ox0 + pix % TW;
    if (gy >= p.H || gx >= p.W) continue;
    *reinterpret_cast<u16x8 *>(p.y + ((int64_t)gy * p.W + gx) * p.ycs + p.yco + s8) =
        *reinterpret_cast<const u16x8 *>(Cs + img<RLO>(pix, s8));
  }
}

template <int CIN, int COUT, bool GATED, bool ADAPT>
size_t lds_bytes() {
  constexpr int RLI = rl<CIN>(), RLO = rl<COUT>();
  const size_t base = (size_t)2 * NPH_T * 16 * RLI + (size_t)NPI * RLI;
  const size_t act = kAlias<CIN, COUT>() ? base : base + (size_t)NPI * RLO + (size_t)NPI * 64;
  return act * 2 + (size_t)kWl<CIN, COUT, GATED>() * 2 + (size_t)10 * CIN * 4;
}

template <int CIN, int COUT, bool GATED, bool ADAPT>
int run(DcbP p, hipStream_t st) {
  p.tiles_x = (p.W + TW - 1) / TW;
  const int tiles_y = (p.H + TH - 1) / TH;
  const size_t lds = lds_bytes<CIN, COUT, GATED, ADAPT>();
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  auto kern = dcb_kernel<CIN, COUT, GATED, ADAPT>;
  dcvc_note_kernel("dcb_kernel<%d, %d, %s, %s>@%lld", CIN, COUT, bname(GATED), bname(ADAPT),
                   (long long)p.tiles_x * tiles_y * 256);
  if (lds > 64 * 1024)
    dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_x * tiles_y)), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

#define DCB_CASE(CI, CO, G, A) \
  if (cin == CI && cout == CO && gated == G && adapt == A) return run<CI, CO, G, A>(p, st)

int dispatch(int cin, int cout, bool gated, bool adapt, const DcbP &p, hipStream_t st) {
  // DCVC-DC feature-domain blocks: UNet (48-32-64-128-128-64-48), MvEnc/MvDec (64),
  // MvEnc adaptor_1 (128->64); IntraNoAR UNet2 (16-32-64-128-128-64-16) and dec (128)
  DCB_CASE(48, 32, false, true);
  DCB_CASE(32, 64, false, true);
  DCB_CASE(64, 128, false, true);
  DCB_CASE(128, 128, false, false);
  DCB_CASE(128, 64, false, true);
  DCB_CASE(64, 48, false, true);
  DCB_CASE(64, 64, false, false);
  DCB_CASE(16, 32, true, true);
  DCB_CASE(32, 64, true, true);
  DCB_CASE(64, 128, true, true);
  DCB_CASE(128, 128, true, false);
  DCB_CASE(128, 64, true, true);
  DCB_CASE(64, 16, true, true);
  return DCVC_HIP_EUNSUPPORTED;
}

}  // namespace

extern "C" int dcvc_internal_dcbp(const dcvc_dcb_args *a, void *stream);
extern "C" int dcvc_internal_dcbs(const dcvc_dcb_args *a, void *stream);

extern "C" int dcvc_depthconv_block(const dcvc_dcb_args *a, void *stream) {
  if (!a || !a->x.ptr || !a->y.ptr) return DCVC_HIP_EINVAL;
  if (a->x.dtype != DCVC_BF16 || a->y.dtype != DCVC_BF16) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.H != a->y.H || a->x.W != a->y.W || a->x.C != a->cin || a->y.C != a->cout) return DCVC_HIP_EINVAL;
  if (a->x.cstride % 8 || a->x.coff % 8 || a->y.cstride % 8 || a->y.coff % 8 ||
      ((uintptr_t)a->x.ptr & 15) || ((uintptr_t)a->y.ptr & 15))
    return DCVC_HIP_EUNSUPPORTED;
  const bool adapt = a->w_adaptor != nullptr;
  if (!adapt && a->cin != a->cout) return DCVC_HIP_EINVAL;
  {
    const int r = dcvc_internal_dcbp(a, stream);  // persistent resident-weight kernel (dcbp.hip) first
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  {
    const int r = dcvc_internal_dcbs(a, stream);  // then persistent streamed-weight kernel (dcbs.hip)
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  DcbP p{};
  p.x = reinterpret_cast<const uint16_t *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
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
  return dispatch(a->cin, a->cout, a->gated != 0, adapt, p, reinterpret_cast<hipStream_t>(stream));
}
