// Persistent fused DepthConvBlock with streamed weights (DCVC-DC/src/models/
// layers.py:135-222, DepthConv + ConvFFN) for the 128-channel blocks of the
// DC UNets whose weights do not fit in LDS next to a tile's activations:
// 128->128 at 1/4 resolution, 128->64 at 1/2, 64->128 at 1/4.
//
// Same arithmetic as dcb.hip (8x16 output tile, t1 on the 10x18 halo,
// depthwise in fp32 from bf16 t1 with the taps in (dy, dx) order, dc rounded
// to bf16, FFN hidden layer in 64-channel slices, every MFMA K order
// ascending in 32-wide steps), so outputs are bit-identical to it
// (tests/test_gpu_kernels.py).  The organisation is built for one workgroup
// per CU (the activations take ~100 KB of LDS) running at two waves per SIMD:
//   * 8 waves; in conv1 / adaptor / conv2 wave w works on pixel tiles
//     {w % 4, w % 4 + 4, ...} and output-channel half w / 4 (0.6-0.75 LDS
//     reads per MFMA); in the FFN on pixel tile w and all channels, so its
//     hidden slices stay wave-private (no barrier between the two FFN
//     GEMMs); one wave's VALU work (depthwise, epilogues) overlaps its SIMD
//     partner's MFMAs;
//   * weights stream through two 32 KB LDS buffers in 256-row x 64-channel
//     chunks: conv1 (+ adaptor), conv2, then one chunk per FFN slice (both of
//     its 1x1 layers) or per two slices; chunk c + 1 is loaded into registers
//     while chunk c is in use, the stream runs on across tiles (the weights
//     do not depend on the tile), one barrier per chunk;
//   * the adaptor runs in phase 1 and the identity residual is read from
//     global memory, so the input image is dead after phase 1: the depthwise
//     output and the FFN hidden slices live in its place, and the next tile's
//     halo input (loaded into registers during the FFN) is written there at
//     the end of the tile;
//   * the depthwise pass gives each thread a column of output pixels for 4
//     channels, so every t1 value is converted from bf16 once per column,
//     not once per tap.
#include "common.h"

namespace {

constexpr int TH = 8, TW = 16;
constexpr int HW_ = TW + 2;
constexpr int NPH = (TH + 2) * HW_;          // 180 halo pixels (MFMA rows up to 191 read the next image)
constexpr int NPI = TH * TW;                 // 128 interior pixels
constexpr int NWV = 8;
constexpr int NTHR = NWV * 64;
constexpr int CROWS = 256;                   // rows of a weight chunk (x 64 channels)
constexpr int WCH = CROWS * 64;              // elements per LDS weight buffer (32 KB)
constexpr int WPT = CROWS * 8 / NTHR;        // 16-byte pieces per thread per chunk (4)

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

template <int RL>
__device__ __forceinline__ int img(int row, int ch) {
  constexpr int NS = RL / 8;
  constexpr int SH = RL == 32 ? 2 : (RL == 64 ? 1 : 0);
  constexpr int MSK = NS < 16 ? NS - 1 : 15;
  const int slot = ch >> 3;
  return row * RL + (((slot ^ ((row >> SH) & MSK)) & (NS - 1)) << 3) + (ch & 7);
}

// leaky ReLU as max(v, s * v): the same value as (v >= 0 ? v : s * v) for
// 0 <= s <= 1 (the host checks), in two VALU instructions instead of three
__device__ __forceinline__ float lrelu(float v, float s) { return fmaxf(v, v * s); }

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float el(const float4 &v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

template <int CIN, int COUT, bool ADAPT>
struct SG {
  static_assert((CIN == 64 || CIN == 128) && (COUT == 64 || COUT == 128), "dcbs shapes");
  static constexpr int NTI2 = CIN / 32, NTO2 = COUT / 32;   // n tiles per channel half
  static constexpr int HID = 4 * COUT, NSL = HID / 64;      // ConvFFN hidden width, 64-channel slices
  static constexpr int KCI = CIN / 64, KCO = COUT / 64;     // 64-channel K pieces
  // chunk plan (rows of 64 channels; pieces start on 64-row boundaries)
  static constexpr int R1 = KCI * CIN, RA = ADAPT ? KCI * COUT : 0;
  static constexpr bool A_IN_C1 = ADAPT && R1 + RA <= CROWS;
  static constexpr int C_ADAPT = A_IN_C1 ? 0 : 1, OA = A_IN_C1 ? R1 : 0;
  static constexpr int C_CONV2 = (ADAPT && !A_IN_C1) ? 2 : 1, C_FFN = C_CONV2 + 1;
  static constexpr int RS = KCO * 64 + COUT;                // rows of one FFN slice: ffn1 K pieces, ffn2
  static constexpr int SPC = CROWS / RS;                    // FFN slices per chunk
  static_assert(SPC >= 1 && NSL % SPC == 0 && CROWS % RS == 0, "chunk plan");
  static constexpr int NFC = NSL / SPC;
  static constexpr int NCH = C_FFN + NFC, NCHP = NCH + (NCH & 1);
  // LDS images (elements): Xs (halo input; then Ds = depthwise out, then the
  // hidden slices Hs), Ts (halo t1; then Cs = dc in bf16 when it fits), weights
  static constexpr int XS = NPH * CIN, TS = NPH * CIN;
  static constexpr bool CS_IN_TS = NPI * COUT <= TS;
  static constexpr int OT = XS, OC = CS_IN_TS ? OT : OT + TS;
  static constexpr int OW = OT + TS + (CS_IN_TS ? 0 : NPI * COUT);
  static_assert(NPI * CIN <= XS && NPI * 64 <= XS, "Ds / Hs in the input image");
  static constexpr int NA = OW + 2 * WCH;
  static constexpr size_t LDS = (size_t)NA * 2 + (size_t)10 * CIN * 4 + (size_t)2 * COUT * 4;
  static constexpr int QP = CIN / 8;                         // 16-byte input pieces per pixel
  static constexpr int PP = (NPH * QP + NTHR - 1) / NTHR;    // halo pieces per thread
  // depthwise tasks: (4-channel quad, column, row group) = one thread each
  static constexpr int NQ = CIN / 4, NRG = NTHR / (NQ * TW), RPT = TH / NRG;
  static_assert(NQ * TW * NRG == NTHR && RPT * NRG == TH, "depthwise tasks");
};

__device__ __forceinline__ u16x8 ldw(const uint16_t *W, int ld, int n, int k) {
  return *reinterpret_cast<const u16x8 *>(W + (int64_t)n * ld + k);
}

// rows [64u, 64u + 64) of head chunk C (conv1 [+ adaptor], adaptor, conv2)
template <int CIN, int COUT, bool ADAPT, int C>
__device__ __forceinline__ void fetch_head(u16x8 (&r)[WPT], const DcbP &p, int tid) {
  typedef SG<CIN, COUT, ADAPT> G_;
  const int rr = tid >> 3, k8 = (tid & 7) * 8;
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int row = 64 * u;   // first row of this thread's block u
    r[u] = u16x8{};
    if constexpr (C == 0) {
      if (row < G_::R1) {
        r[u] = ldw(p.w1, p.ld1, row % CIN + rr, (row / CIN) * 64 + k8);
        continue;
      }
    }
    if constexpr (ADAPT && C == G_::C_ADAPT) {
      if (row >= G_::OA && row < G_::OA + G_::RA) {
        const int o = row - G_::OA;
        r[u] = ldw(p.wa, p.lda, o % COUT + rr, (o / COUT) * 64 + k8);
        continue;
      }
    }
    if constexpr (C == G_::C_CONV2) {
      if (row < G_::KCI * COUT) r[u] = ldw(p.w2, p.ld2, row % COUT + rr, (row / COUT) * 64 + k8);
    }
  }
}

// rows of FFN chunk f (run-time): per slice s = f * SPC + ss, KCO ffn1 pieces
// (hidden channels s*64.., input channels kc*64..) then the ffn2 piece
// (output channels, hidden channels s*64..)
template <int CIN, int COUT, bool ADAPT>
__device__ __forceinline__ void fetch_ffn(u16x8 (&r)[WPT], const DcbP &p, int f, int tid) {
  typedef SG<CIN, COUT, ADAPT> G_;
  const int rr = tid >> 3, k8 = (tid & 7) * 8;
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int ss = (64 * u) / G_::RS, o = 64 * u - ss * G_::RS;
    const int s = f * G_::SPC + ss;
    if (o < G_::KCO * 64) r[u] = ldw(p.wf1, p.ldf1, s * 64 + rr, (o / 64) * 64 + k8);
    else r[u] = ldw(p.wf2, p.ldf2, o - G_::KCO * 64 + rr, s * 64 + k8);
  }
}

template <int CIN, int COUT, bool ADAPT>
__device__ __forceinline__ void fetch_chunk(u16x8 (&r)[WPT], const DcbP &p, int c, int tid) {
  typedef SG<CIN, COUT, ADAPT> G_;
  if (c >= G_::C_FFN) {
    if (c < G_::NCH) fetch_ffn<CIN, COUT, ADAPT>(r, p, c - G_::C_FFN, tid);
  } else if (c == 0) {
    fetch_head<CIN, COUT, ADAPT, 0>(r, p, tid);
  } else if (c == 1) {
    fetch_head<CIN, COUT, ADAPT, 1>(r, p, tid);
  } else {
    fetch_head<CIN, COUT, ADAPT, 2>(r, p, tid);
  }
}

__device__ __forceinline__ void put(uint16_t *Wl, const u16x8 (&r)[WPT], int tid) {
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int it = tid + u * NTHR;
    *reinterpret_cast<u16x8 *>(Wl + img<64>(it >> 3, (it & 7) * 8)) = r[u];
  }
}

// acc[i][j] += W[(n0 + j) * 16 + ..][k] * B[rowb_i + ..][kb + k], k in [0, 64):
// W one 64-channel piece of a chunk image, B an activation image
template <int RLB, int NPT, int NT>
__device__ __forceinline__ void mma(f32x4 (&acc)[NPT][NT], const uint16_t *imgb, const int (&rowb)[NPT],
                                    const uint16_t *Wp, int n0, int lane, int kb) {
  const int col = lane & 15, hi = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < 64; k0 += 32) {
    bf16x8 a[NT], b[NPT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
      a[j] = *reinterpret_cast<const bf16x8 *>(Wp + img<64>((n0 + j) * 16 + col, k0 + hi * 8));
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

template <int A, int B>
__device__ __forceinline__ void zero(f32x4 (&a)[A][B]) {
#pragma unroll
  for (int i = 0; i < A; ++i)
#pragma unroll
    for (int j = 0; j < B; ++j) a[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int CIN, int COUT, bool ADAPT>
__global__ void __launch_bounds__(NTHR) dcbs_kernel(DcbP p) {
  typedef SG<CIN, COUT, ADAPT> G_;
  constexpr int NTI2 = G_::NTI2, NTO2 = G_::NTO2, KCI = G_::KCI, KCO = G_::KCO;
  constexpr int NCH = G_::NCH, NCHP = G_::NCHP, SPC = G_::SPC, RS = G_::RS;
  constexpr int QP = G_::QP, PP = G_::PP;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *const Xs = reinterpret_cast<uint16_t *>(smem);
  uint16_t *const Ds = Xs;
  uint16_t *const Ts = Xs + G_::OT;
  uint16_t *const Cs = Xs + G_::OC;
  uint16_t *const Wl = Xs + G_::OW;
  float *const Dw = reinterpret_cast<float *>(Xs + G_::NA);   // [9][CIN] taps, [CIN] bias
  float *const Lo = Dw + 10 * CIN;                              // [COUT] ffn2 bias, [COUT] scale

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int pr = wave & 3, hf = wave >> 2;   // pixel-tile set, output-channel half
  const int G = gridDim.x;
  int g = blockIdx.x;
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);  // consecutive tiles per XCD
  const int ntiles = p.tiles_x * p.tiles_y;
  if (g >= ntiles) return;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.x), (short)0, p.xbytes, 0x00020000);
  int atid = tid;   // thread id for the loaders' addresses (made opaque per tile, see the tile loop)
  // ---- halo input: piece u of thread tid = (halo pixel, 16-byte channel piece)
  u16x8 pf[PP];
  auto issue = [&](int t) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
    const int base = (oy0 * p.W + ox0) * p.xcs + p.xco;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = atid + u * NTHR;
      const int pix = it / QP, q = it - pix * QP;
      const int hy = pix / HW_, hx = pix - hy * HW_;
      const int gy = oy0 - 1 + hy, gx = ox0 - 1 + hx;
      const bool in = it < NPH * QP && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
      const int off = in ? (base + ((hy - 1) * p.W + (hx - 1)) * p.xcs + q * 8) * 2 : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto publish = [&]() {
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = atid + u * NTHR;
      const int pix = it / QP, q = it - pix * QP;
      if (it < NPH * QP) *reinterpret_cast<u16x8 *>(Xs + img<CIN>(pix, q * 8)) = pf[u];
    }
  };

  // ---- weight stream: chunk c goes global -> registers while chunk c - 1
  // is in use, then -> LDS buffer c & 1
  u16x8 R[WPT];
  fetch_head<CIN, COUT, ADAPT, 0>(R, p, atid);
  issue(g);
  bool more = g + G < ntiles;
  // acquire(c, c & 1): chunk c -> LDS buffer c & 1, one barrier, then the
  // loads of chunk c + 1 (this tile's or the next one's) into R.  Buffer
  // c & 1 was last read by chunk c - 2's MFMAs, which every wave finished
  // before chunk c - 1's barrier.  `par` folds to a constant at every call
  // site; c may be a run-time value (the FFN loop).
  auto acquire = [&](int c, int par) -> const uint16_t * {
    uint16_t *B = Wl + par * WCH;
    put(B, R, atid);
    __syncthreads();
    const int cn = c + 1 < NCHP ? c + 1 : c + 1 - NCHP;
    if (c + 1 < NCHP || more) fetch_chunk<CIN, COUT, ADAPT>(R, p, cn, atid);
    return B;
  };

  for (int i = tid; i < 10 * CIN; i += NTHR) Dw[i] = i < 9 * CIN ? p.wdw[i] : p.bdw[i - 9 * CIN];
  for (int i = tid; i < 2 * COUT; i += NTHR) Lo[i] = i < COUT ? p.bf2[i] : (p.scale ? p.scale[i - COUT] : 1.f);
  publish();   // the first tile's halo (chunk 0's barrier publishes it)

  constexpr int NQ = G_::NQ, RPT = G_::RPT;
#pragma unroll 1
  for (int t = g;;) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
    const int tn = t + G;
    // Lane-dependent LDS addresses are recomputed per tile from an opaque
    // copy of the lane id: hoisted out of the tile loop they would be ~100
    // live registers (one per swizzled operand address) and spill.
    int lane_ = lane;
    asm volatile("" : "+v"(lane_));
    const int col = lane_ & 15, hi = lane_ >> 4;
    const int ltid = wave * 64 + lane_;
    atid = ltid;
    int rb1[3], rowi[2], rowh[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) rb1[i] = (pr + 4 * i) * 16;   // halo pixel tiles (12)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pt = pr + 4 * i;   // interior pixel tile = output row pt of the tile
      rowi[i] = pt * 16;
      rowh[i] = (pt + 1) * HW_ + 1;
    }
    // depthwise task of this thread
    const int dq = ltid % NQ, dcol = (ltid / NQ) % TW, drg = ltid / (NQ * TW);

    // ---- P1: t1 = lrelu(conv1(x) + b1) on the halo (0 outside the image);
    // the adaptor on the interior rows of the same image
    float4 b1v[NTI2];   // loaded before the MFMAs that hide their latency
#pragma unroll
    for (int j = 0; j < NTI2; ++j) b1v[j] = ld4(p.b1 + (hf * NTI2 + j) * 16 + hi * 4);
    const uint16_t *B0 = acquire(0, 0);
    f32x4 ad[2][ADAPT ? NTO2 : 1];
    {
      f32x4 acc[3][NTI2];
      zero(acc);
#pragma unroll
      for (int kc = 0; kc < KCI; ++kc) mma<CIN, 3, NTI2>(acc, Xs, rb1, B0 + kc * CIN * 64, hf * NTI2, lane_, kc * 64);
      if constexpr (ADAPT) {
        const uint16_t *BA = G_::A_IN_C1 ? B0 : acquire(1, 1);
        zero(ad);
#pragma unroll
        for (int kc = 0; kc < KCI; ++kc)
          mma<CIN, 2, NTO2>(ad, Xs, rowh, BA + (G_::OA + kc * COUT) * 64, hf * NTO2, lane_, kc * 64);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int row = rb1[i] + col;
        const int hy = row / HW_, hx = row % HW_;
        const int gy = oy0 - 1 + hy, gx = ox0 - 1 + hx;
        const bool inside = gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
        if (row < NPH) {
#pragma unroll
          for (int j = 0; j < NTI2; ++j) {
            const int c = (hf * NTI2 + j) * 16 + hi * 4;
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = inside ? lrelu(acc[i][j][q] + el(b1v[j], q), p.slope_dc) : 0.f;
            put4<CIN>(Ts, row, c, v);
          }
        }
      }
    }
    // identity residual x (interior pixels, this wave's channels) from global memory
    u16x4 res[2][ADAPT ? 1 : NTO2];
    if constexpr (!ADAPT) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int gy = oy0 + (pr + 4 * i), gx = ox0 + col;
        const bool in = gy < p.H && gx < p.W;
#pragma unroll
        for (int j = 0; j < NTO2; ++j) {
          const int c = (hf * NTO2 + j) * 16 + hi * 4;
          const int off = in ? (((gy * p.W + gx) * p.xcs + p.xco + c) * 2) : 0x7ffffff0;
          res[i][j] = __builtin_bit_cast(u16x4, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
        }
      }
    }
    float4 b2v[NTO2], bav[ADAPT ? NTO2 : 1];
#pragma unroll
    for (int j = 0; j < NTO2; ++j) {
      b2v[j] = ld4(p.b2 + (hf * NTO2 + j) * 16 + hi * 4);
      if constexpr (ADAPT) bav[j] = ld4(p.ba + (hf * NTO2 + j) * 16 + hi * 4);
    }
    // conv2's chunk; its barrier also publishes t1 (and ends every read of x)
    const uint16_t *B2 = acquire(G_::C_CONV2, G_::C_CONV2 & 1);

    // ---- P2: d = dw3x3(t1) + bdw: a column of RPT output pixels x 4 channels per thread
    {
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
      // rolling window of three converted t1 rows (row r in tv[r % 3])
      float tv[3][3][4];
      auto load_row = [&](int r) {
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const u16x4 v = *reinterpret_cast<const u16x4 *>(Ts + img<CIN>((drg * RPT + r) * HW_ + dcol + dx, dq * 4));
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
        put4<CIN>(Ds, (drg * RPT + o) * TW + dcol, dq * 4, v);
      }
    }
    __syncthreads();

    // ---- P3: dc = conv2(d) + b2 + (adaptor(x) + ba | x), rounded to bf16 -> Cs
    {
      f32x4 dc[2][NTO2];
      zero(dc);
#pragma unroll
      for (int kc = 0; kc < KCI; ++kc) mma<CIN, 2, NTO2>(dc, Ds, rowi, B2 + kc * COUT * 64, hf * NTO2, lane_, kc * 64);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NTO2; ++j) {
          const int c = (hf * NTO2 + j) * 16 + hi * 4;
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if constexpr (ADAPT)
              v[q] = bf2f(f2bf(ad[i][j][q] + el(bav[j], q))) + (dc[i][j][q] + el(b2v[j], q));
            else
              v[q] = (dc[i][j][q] + el(b2v[j], q)) + bf2f(res[i][j][q]);
          }
          put4<COUT>(Cs, rowi[i] + col, c, v);   // Ts (t1) was last read before P2's barrier
        }
    }
    // the next tile's halo: in flight during the FFN, written to Xs in P5
    if (more) issue(tn);

    // ---- P4: FFN, one or two 64-channel hidden slices per weight chunk.
    // Wave w owns pixel tile w here (all channels): its hidden slice rows in
    // Hs are written and read by itself only, and a wave's LDS operations
    // complete in order, so no barrier separates ffn1 from ffn2.
    constexpr int NTO = COUT / 16;
    const int rowf[1] = {wave * 16};
    f32x4 acc[1][NTO];
    zero(acc);
    uint16_t *const Hs = Xs;
#pragma unroll 1
    for (int fp = 0; fp < G_::NFC; fp += 2)
#pragma unroll
      for (int fu = 0; fu < 2; ++fu) {
        if ((G_::NFC & 1) && fp + fu >= G_::NFC) break;
        const int f = fp + fu;
        // publishes chunk f (and, the first time, Cs)
        const uint16_t *B = acquire(G_::C_FFN + f, (G_::C_FFN + fu) & 1);
#pragma unroll
        for (int ss = 0; ss < SPC; ++ss) {
          const int s = f * SPC + ss;
          const uint16_t *Bs = B + ss * RS * 64;
          float4 f1v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) f1v[j] = ld4(p.bf1 + s * 64 + j * 16 + hi * 4);
          f32x4 hacc[1][4];
          zero(hacc);
#pragma unroll
          for (int kc = 0; kc < KCO; ++kc) mma<COUT, 1, 4>(hacc, Cs, rowf, Bs + kc * 64 * 64, 0, lane_, kc * 64);
          wave_lds_sync();   // the previous slice's Hs reads (other lanes) before these writes
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = lrelu(hacc[0][j][q] + el(f1v[j], q), p.slope_ffn);
            put4<64>(Hs, rowf[0] + col, j * 16 + hi * 4, v);
          }
          wave_lds_sync();   // Hs written before other lanes read it
          mma<64, 1, NTO>(acc, Hs, rowf, Bs + KCO * 64 * 64, 0, lane_, 0);
        }
      }

    // ---- P5: out = dc + lrelu(acc + bf2) [* scale] -> Cs (each wave over
    // its own pixel tile's rows), whole-line stores
#pragma unroll
    for (int j = 0; j < NTO; ++j) {
      const int c = j * 16 + hi * 4;
      u16x4 *cp = reinterpret_cast<u16x4 *>(Cs + img<COUT>(rowf[0] + col, c));
      const u16x4 dcv = *cp;
      const float4 f2v = ld4(Lo + c), scv = ld4(Lo + COUT + c);
      u16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = bf2f(dcv[q]) + lrelu(acc[0][j][q] + el(f2v, q), p.slope_ffn);
        if (p.scale) v = v * el(scv, q);
        o[q] = f2bf(v);
      }
      *cp = o;
    }
    if constexpr (NCHP != NCH) acquire(NCH, NCH & 1);   // padding chunk: keeps the parity, gives the barrier
    else __syncthreads();
    if (more) publish();   // Xs (Ds / Hs) is dead: the last hidden slice was read before this barrier
    constexpr int NSO = COUT / 8;
    for (int it = tid; it < NPI * NSO; it += NTHR) {
      const int pix = it / NSO, s8 = (it % NSO) * 8;
      const int gy = oy0 + pix / TW, gx = ox0 + pix % TW;
      if (gy >= p.H || gx >= p.W) continue;
      *reinterpret_cast<u16x8 *>(p.y + ((int64_t)gy * p.W + gx) * p.ycs + p.yco + s8) =
          *reinterpret_cast<const u16x8 *>(Cs + img<COUT>(pix, s8));
    }
    // the next tile's chunk-0 barrier orders these Cs reads before P1 writes Ts
    if (!more) break;
    t = tn;
    more = t + G < ntiles;
  }
}

int g_cus = 0;
int g_enabled = 1;

template <int CIN, int COUT, bool ADAPT>
int run(DcbP p, hipStream_t st) {
  typedef SG<CIN, COUT, ADAPT> G_;
  static_assert(G_::LDS <= 160 * 1024, "LDS");
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
  const int G = ntiles < g_cus ? (int)ntiles : g_cus;
  auto kern = dcbs_kernel<CIN, COUT, ADAPT>;
  dcvc_note_kernel("dcbs_kernel<%d, %d, %s>@%lld", CIN, COUT, bname(ADAPT), (long long)G * NTHR);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(NTHR), G_::LDS, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

// Called by dcvc_depthconv_block (dcb.hip) after its argument checks and after
// dcbp.hip declined; DCVC_HIP_EUNSUPPORTED hands the call to dcb_kernel.
extern "C" int dcvc_internal_dcbs(const dcvc_dcb_args *a, void *stream) {
  if (!g_enabled || a->gated) return DCVC_HIP_EUNSUPPORTED;
  if (!(a->slope_dc >= 0.f && a->slope_dc <= 1.f && a->slope_ffn >= 0.f && a->slope_ffn <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;   // lrelu as max(v, s v)
  if ((int64_t)a->x.H * a->x.W * a->x.cstride >= ((int64_t)1 << 30) - 16) return DCVC_HIP_EUNSUPPORTED;
  const bool adapt = a->w_adaptor != nullptr;
  // the streamed chunks are whole 64-channel pieces of the packed weights
  if (a->ld_conv1 != a->cin || a->ld_conv2 != a->cin || a->ld_ffn1 != a->cout || a->ld_ffn2 != 4 * a->cout ||
      (adapt && a->ld_adaptor != a->cin))
    return DCVC_HIP_EUNSUPPORTED;
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
  if (a->cin == 128 && a->cout == 128 && !adapt) return run<128, 128, false>(p, st);
  if (a->cin == 128 && a->cout == 64 && adapt) return run<128, 64, true>(p, st);
  if (a->cin == 64 && a->cout == 128 && adapt) return run<64, 128, true>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

// dcvc_set_option("dcb_stream", 0/1) (A/B switch, via conv.hip)
extern "C" void dcvc_internal_dcbs_enable(int v) { g_enabled = v; }
