// Wave-specialised split-fp16 3x3 stride-1 convolution (round 6): the
// feature-rate 3x3 layers of Precision.split() with 48- .. 192-channel inputs
// (ResBlocks, context fusion, UNet / recon convs of
// DCVC-DC/src/models/video_net.py:58-76, 129-170 and video_model.py:89-118,
// 173-232).  The products, their K order and the epilogue are xconv.hip's
// (and sconv.hip's), so the outputs are bit-identical to both.
//
// Why another schedule.  xconv's eight waves all run the same program: a
// stage's image loads, split VALU, LDS publish and weight DMA and its MFMAs
// are issued by the same waves, and the two waves of a SIMD meet every
// barrier together, so their memory / VALU phases coincide and leave the
// matrix pipe idle: timing ablations of the 48 -> 48 layer at 1080p
// (profiles/r06c_xconv_ablation.jsonl) add up -- MFMAs 142 us, global memory
// 133 us, publish and image-operand reads 47 us, the rest 70 us -- with no
// overlap.  Here the roles are split by wave:
//
//   consumer waves 0-3 (one per SIMD): rows RW c .. RW c + RW - 1 of the
//       4 RW-row tile (RW = 4, or 3 at 48-channel n-blocks with a residual);
//       per stage they read the next stage's operands from LDS and issue
//       their 36 (or 24) MFMAs back to back; at a tile's last stage they run
//       the epilogue from the accumulators (bias, activation, residual,
//       scale, 16-byte stores);
//   weight-DMA wave 4: the weight ring (LDS-DMA, issued a ring's depth
//       ahead) and its exact vmcnt waits, which count nothing else;
//   image waves 5-7: the image pipeline (global loads two chunks ahead into
//       two register sets, the leaky ReLU / range fold / hi-lo split and the
//       swizzled LDS publish spread over the stages of the chunk before).
//
// A SIMD then holds one MFMA wave and one memory / VALU wave, which the
// hardware runs side by side.  One barrier per stage.  Instantiated for even
// chunk counts (48, 64, 128, 192 input channels), n-blocks of 32 or 48
// channels and at most one residual; the rest stays on xconv.hip.
#include "common.h"
#include "split.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>

// consumer (MFMA) waves: 4 (one per SIMD, 4 rows each) or 8 (two per SIMD,
// 2 rows each; 12 waves in all, 3 per SIMD)
#ifndef WCONV_NC
#define WCONV_NC 4
#endif

namespace {

struct WP {
  const float *x;
  int H, W, xcs, xco;
  const uint16_t *w;       // DCVC_F16X3 packed weights (dcvc_conv_pack_weights)
  float *y;
  int Ho, Wo, ycs, yco;
  int cout;
  int in_lrelu;
  float in_slope;
  int act;
  float slope;
  const float *res;
  int rcs, rco;
  int has_res;
  int tiles_x, nblk, ntiles;
  int wbytes;
  int64_t wchunk;          // halves of one full chunk's packed weights (hi + lo)
  const float *bias;
  const float *scale;
  int *ovf;               // fp16 range guard (split.h SplitRange)
  int dbg;                // timing ablations (dcvc_set_option("wconv_dbg"), WCONV_DBG builds), 0 in production
};

// WCONV_DBG builds (diagnostics, wrong results): dcvc_set_option("wconv_dbg",
// bits) skips 1 the consumer MFMAs, 2 the consumer LDS operand reads, 4 the
// producer publish, 8 the producer image loads, 16 the weight DMA and its
// waits, 32 the stage barriers, 64 the epilogue's residual loads and stores,
// 128 the consumer waves' raised issue priority
#ifdef WCONV_DBG
#define WDBG(bit) (p.dbg & (bit))
#else
#define WDBG(bit) false
#endif

template <typename F, int... I>
__device__ __forceinline__ void wfor_(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void wfor(F &&f) {
  wfor_(f, std::make_integer_sequence<int, N>{});
}

template <int CIN, int BN, int NRES>
struct WG {
  // waves: NC consumers (0-3), NDW weight-DMA producer (4), NIW image
  // producers (5-7).  The DMA wave issues nothing but LDS-DMAs, so its
  // exact vmcnt waits count only those: vmcnt completes in issue order, and
  // with the image loads in the same waves (the first version of this kernel,
  // and xconv.hip) every weight wait also waited for the image loads issued
  // before it -- a 50 us share of 397 us at 48 -> 48 1080p in the timing
  // ablation (profiles/r06g_wconv_ablation.jsonl)
  static constexpr int KS = 3, KT = 9, NC = WCONV_NC, NIW = 3, NDW = 1, NT = BN / 16;
  static constexpr int NTH = (NC + NDW + NIW) * 64;         // threads (the kernel's launch bound: (WCONV_NC + 4) * 64)
  static_assert(NDW + NIW == 4, "launch bound");
  // rows per consumer wave: 4, or 3 for 48-channel n-blocks with a residual
  // (the residual's 12 fragments on top of 24 accumulator pairs and two
  // operand sets would not fit the 256 registers of 2 waves / SIMD)
  static constexpr int RW = NC == 8 ? 2 : (NRES >= 1 && NT == 3 ? 3 : 4), TH = NC * RW;
  static constexpr int PT = NIW * 64;                      // image-producer threads
  static constexpr int IH = TH + 2, IW = 18, IWP = 20;
  static constexpr int CH = (CIN + 31) / 32;
  static constexpr int VCL = CIN - 32 * (CH - 1);
  static constexpr int TPKL = VCL <= 8 ? 4 : (VCL <= 16 ? 2 : 1);
  static constexpr int ROWSL = (KT + TPKL - 1) / TPKL;
  static constexpr int NST = (CH - 1) * KT + ROWSL;
  static constexpr int NSLF = 4, NSLL = TPKL == 1 ? 4 : 4 / TPKL;
  static constexpr int PPF = (IH * IW * NSLF + PT - 1) / PT;   // image pieces per producer thread, full chunk
  static constexpr int PPL = (IH * IW * NSLL + PT - 1) / PT;   // ... last chunk
  static constexpr int PPM = PPF > PPL ? PPF : PPL;
  static constexpr int IMG = IH * IWP * 32;
  static constexpr int WST = BN * 32;
  static constexpr int NDMA = 2 * BN / 16;
  static constexpr int DPW = (NDMA + NDW - 1) / NDW;      // LDS-DMAs per DMA wave and stage
  static_assert(CH % 2 == 0, "two image register sets by chunk parity need an even chunk count");
  static_assert(NT == 2 || NT == 3, "n-blocks of 32 or 48 channels");
  static_assert(NRES <= 1, "at most one residual");
  static_assert(NST * RW % 2 == 0, "a tile's row count must be even (the image-operand ring restarts at slot 0)");

  static constexpr int chunk(int s) { return s < (CH - 1) * KT ? s / KT : CH - 1; }
  static constexpr int row(int s) { return s - chunk(s) * KT; }
  static constexpr int rows(int c) { return c == CH - 1 ? ROWSL : KT; }
  static constexpr int pp(int c) { return c == CH - 1 ? PPL : PPF; }
  // the weight ring: NSW slots; stage s's DMA is issued AH = NSW stages
  // ahead, into the slot of stage s - NSW... = the slot of the current stage,
  // whose fragments the consumers read during the stage before.  At the end
  // of stage s the weights of stage s + 2 must have landed (read during
  // stage s + 1): their DMA closed stage s + 2 - AH, the DPW DMAs of each
  // later stage may stay in flight
  static constexpr int LDS_WG = 160 * 1024;
  static constexpr int NSW_FIT = (LDS_WG - 2048 - 4 * IMG * 2 - 1024) / (2 * WST * 2);
  static constexpr int pick_nsw() {
    int n = NSW_FIT < 12 ? NSW_FIT : 12;
    if (n > NST) n = NST;
    for (int d = n; d >= 5; --d)   // a depth dividing the stage count: compile-time slots
      if (NST % d == 0) return d;
    return n;
  }
  static constexpr int NSW = pick_nsw(), AH = NSW;
  static constexpr bool RING_STATIC = NST % NSW == 0;
  static_assert(NSW >= 3, "weight ring too shallow");
  static constexpr int WAIT_N = (AH - 2) * DPW;
  static_assert(WAIT_N < 64, "vmcnt is 6 bits");
  static constexpr int L_W = 4 * IMG;
  static constexpr int L_SINK = L_W + 2 * NSW * WST;
  static constexpr int L_C = L_SINK + 512;
  static constexpr size_t lds(int cout) { return (size_t)L_C * 2 + (size_t)2 * cout * 4; }
  static constexpr int wait_n(int) { return WAIT_N; }
  // the publish of chunk c + 1 during chunk c: pieces [pub0(rr), pub0(rr + 1))
  // at chunk row rr, spread over rows 0 .. rows(c) - 2
  static constexpr int pub0(int c, int rr) {
    const int n = pp((c + 1) % CH), st = rows(c) - 1;
    return rr >= st ? n : rr * n / st;
  }
};

template <int CIN, int BN, int NRES>
__global__ void __launch_bounds__((WCONV_NC + 4) * 64)
    __attribute__((amdgpu_waves_per_eu(WCONV_NC == 8 ? 3 : 2, WCONV_NC == 8 ? 3 : 2)))
wconv3_kernel(WP p) {
  typedef WG<CIN, BN, NRES> G;
  constexpr int NT = G::NT, RW = G::RW, IH = G::IH, IW = G::IW, IWP = G::IWP, IMG = G::IMG, WST = G::WST;
  constexpr int CH = G::CH, KT = G::KT, TPKL = G::TPKL, NST = G::NST;
  constexpr int NDMA = G::NDMA, DPW = G::DPW, PPF = G::PPF, PPL = G::PPL, PPM = G::PPM, PT = G::PT;
  constexpr int NSW = G::NSW, AH = G::AH;
  SplitRange rg(p.ovf);
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *const L = reinterpret_cast<uint16_t *>(smem);
  float *const Lc = reinterpret_cast<float *>(smem + (size_t)G::L_C * 2);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const bool producer = wave >= G::NC, dma_wave = producer && wave < G::NC + G::NDW;
  const int col = lane & 15, hi = lane >> 4;
  const int GR = gridDim.x;
  int g = blockIdx.x;
  if ((GR & 7) == 0) g = (g & 7) * (GR >> 3) + (g >> 3);   // consecutive tiles on one XCD
  if (g >= p.ntiles) return;

  for (int i = tid; i < p.cout; i += G::NTH) {
    Lc[i] = p.bias ? p.bias[i] : 0.f;
    Lc[p.cout + i] = p.scale ? p.scale[i] : 1.f;
  }

  struct TI {
    int oy0, ox0, n0;
    int nb, tx, ty;
  };
  auto tile_of = [&](int t) {
    const int nb = t % p.nblk, sp = t / p.nblk;
    const int ty = sp / p.tiles_x;
    TI r;
    r.nb = nb;
    r.ty = ty;
    r.tx = sp - ty * p.tiles_x;
    r.n0 = nb * BN;
    r.oy0 = ty * G::TH;
    r.ox0 = r.tx * 16;
    return r;
  };
  const int dsp = GR / p.nblk, dnb = GR - dsp * p.nblk;
  const int dty = dsp / p.tiles_x, dtx = dsp - dty * p.tiles_x;
  auto tile_next = [&](const TI &a) {
    TI r;
    r.nb = a.nb + dnb;
    const int c1 = r.nb >= p.nblk;
    if (c1) r.nb -= p.nblk;
    r.tx = a.tx + dtx + c1;
    const int c2 = r.tx >= p.tiles_x;
    if (c2) r.tx -= p.tiles_x;
    r.ty = a.ty + dty + c2;
    r.n0 = r.nb * BN;
    r.oy0 = r.ty * G::TH;
    r.ox0 = r.tx * 16;
    return r;
  };

  // ---------------------------------------------------------------- producer
  // image piece u of producer thread pt: (halo row, halo column, 8-channel slot)
  const int pt = tid - (G::NC + G::NDW) * 64;
  constexpr int NTOTF = IH * IW * 4, NTOTL = IH * IW * G::NSLL;
  struct Piece {
    int iy, ix, slot, valid;
  };
  auto piece = [&](int u, auto NS_) {
    constexpr int NS = decltype(NS_)::value;
    const int it = pt + u * PT;
    const int pix = it / NS;
    Piece q;
    q.slot = it - pix * NS;
    q.iy = pix / IW;
    q.ix = pix - q.iy * IW;
    q.valid = it < IH * IW * NS;
    return q;
  };
  float pf[2][PPM][8];   // image pieces in flight: set c & 1 holds chunk c
  auto load_img = [&](const TI &ti, auto C_, auto SET_) {
    constexpr int c = decltype(C_)::value, set = decltype(SET_)::value;
    constexpr bool last = c == CH - 1;
    constexpr int PP = last ? PPL : PPF, NTOT = last ? NTOTL : NTOTF;
    const int iy0 = ti.oy0 - 1, ix0 = ti.ox0 - 1;
    const int rb = iy0 > 0 ? iy0 : 0;
    const int64_t eb = (int64_t)rb * p.W * p.xcs + p.xco + c * 32;
    int64_t nrec = ((int64_t)p.H * p.W * p.xcs - eb) * 4;
    if (nrec > 0x7fff0000) nrec = 0x7fff0000;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.x + eb), (short)0, (int)nrec, 0x00020000);
    const int toff = ((iy0 - rb) * p.W + ix0) * p.xcs;
    const bool inner = iy0 >= 0 && ix0 >= 0 && iy0 + IH <= p.H && ix0 + IW <= p.W;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const Piece q = piece(u, std::integral_constant<int, last ? G::NSLL : 4>{});
      int o = (toff + (q.iy * p.W + q.ix) * p.xcs + q.slot * 8) * 4;
      if (!inner) {
        const int gy = iy0 + q.iy, gx = ix0 + q.ix;
        if (!((unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W)) o = 0x7fffffe0;
      }
      if ((u + 1) * PT > NTOT && !q.valid) o = 0x7fffffe0;
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[set][u][j] = a[j];
        pf[set][u][4 + j] = b[j];
      }
    }
  };
  // LDS image buffer ib <- pieces [U0, U1) of register set SET (chunk c)
  auto publish = [&](int ib, auto C_, auto SET_, auto U0_, auto U1_) {
    constexpr int c = decltype(C_)::value, set = decltype(SET_)::value;
    constexpr bool last = c == CH - 1;
    constexpr int PP = last ? PPL : PPF, NTOT = last ? NTOTL : NTOTF;
    constexpr int U0 = decltype(U0_)::value, U1 = decltype(U1_)::value < PP ? decltype(U1_)::value : PP;
    uint16_t *const Lh = L + ib * 2 * IMG;
    if (p.in_lrelu) {
#pragma unroll
      for (int u = U0; u < U1; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[set][u][j] = lrelu_in(pf[set][u][j], p.in_slope);
    }
#pragma unroll
    for (int u = U0; u < U1; ++u) {
      u32x4_t h, l;
      rg.add8(pf[set][u]);
      split8(pf[set][u], h, l);
      const Piece q = piece(u, std::integral_constant<int, last ? G::NSLL : 4>{});
      const int o = swzx(q.iy * IWP + q.ix, q.ix, q.slot);
      const bool ok = (u + 1) * PT <= NTOT || q.valid;
      if (ok) {
        *reinterpret_cast<u32x4_t *>(Lh + o) = h;
        *reinterpret_cast<u32x4_t *>(Lh + IMG + o) = l;
      }
    }
  };
  // weight DMA pieces: DMA wave pw issues pieces pw, pw + NDW, .. (DPW of
  // them; the surplus into the sink).  xconv.hip's source / slot layout
  const int pw = wave - G::NC;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
  int dlane[DPW], drow[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) {
    const int i = pw + G::NDW * d;
    const int hl = i >= NDMA / 2, k = hl ? i - NDMA / 2 : i;
    const int R = k * 16 + (lane >> 2);
    const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
    dlane[d] = (R * 32 + ls * 8) * 2;
    drow[d] = i < NDMA ? R : 0x7fff;
  }
  auto dma_lanes = [&](int n0, int (&dv)[DPW]) {
#pragma unroll
    for (int d = 0; d < DPW; ++d) dv[d] = drow[d] < p.cout - n0 ? dlane[d] : 0x7ffffff0;
  };
  int wcb = (int)(p.wchunk * 2), wrb = p.cout * 64;
  auto dma_w = [&](int n0, const int (&dv)[DPW], auto s_, int ws) {
#pragma unroll
    for (int d = 0; d < DPW; ++d) {
#ifdef __HIP_DEVICE_COMPILE__
      constexpr int s = decltype(s_)::value;
      constexpr int c = G::chunk(s), rr = G::row(s);
      constexpr int rows = G::rows(c);
      const int i = pw + G::NDW * d;
      const int hl = i >= NDMA / 2, k = hl ? i - NDMA / 2 : i;
      const int ub = c * wcb + (hl ? rows * wrb : 0) + rr * wrb + n0 * 64;
      uint16_t *dst = i < NDMA ? L + G::L_W + ws * 2 * WST + hl * WST + k * 512 : L + G::L_SINK;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)dst, 16, dv[d], ub, 0,
                                               0);
#else
      (void)n0, (void)dv, (void)ws, (void)wr, (void)wcb, (void)wrb;
#endif
    }
  };

  // ---------------------------------------------------------------- consumer
  const int cw = wave;   // consumer wave: rows RW cw .. RW cw + RW - 1
  int aoff = swz(col, hi);
  int bo1[3], bo2[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int x = col + dx;
    bo1[dx] = swzx(cw * RW * IWP + x, x, hi);
    constexpr int spt = 4 / TPKL;
    bo2[dx] = swzx(cw * RW * IWP + x, x, hi % spt);
  }
  const int sub = hi / (4 / TPKL);
  // operands: the weight fragments of a stage (two sets: the next stage's
  // are read during this one), the image fragments by row through a
  // two-deep ring (row r + 1's read while row r's MFMAs run)
  f16x8 oa[2][NT][2], ob[2][2];
  auto read_a = [&](auto S_, int ws) {
    constexpr int S = decltype(S_)::value;
    const uint16_t *Lw = L + G::L_W + ws * 2 * WST + aoff;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      oa[S][j][0] = *reinterpret_cast<const f16x8 *>(Lw + j * 512);
      oa[S][j][1] = *reinterpret_cast<const f16x8 *>(Lw + j * 512 + WST);
    }
  };
  // image fragment of row r of stage s (buffer ib) into ring slot q
  auto read_b = [&](auto s_, auto R_, int ib, auto Q_) {
    constexpr int s = decltype(s_)::value, r = decltype(R_)::value, Q = decltype(Q_)::value;
    constexpr int c = G::chunk(s), rr = G::row(s);
    constexpr int tpk = c == CH - 1 ? TPKL : 1;
    const uint16_t *Li = L + ib * 2 * IMG;
    int o;
    if constexpr (tpk == 1) {
      constexpr int dy = rr / 3, dx = rr % 3;
      o = bo1[dx] + (r + dy) * IWP * 32;
    } else {
      constexpr int ta = tpk * rr, tb = tpk * rr + 1;
      constexpr int ta_ = ta < KT ? ta : 0, tb_ = tb < KT ? tb : 0;
      const int oA = bo2[ta_ % 3] + (ta_ / 3) * IWP * 32;
      const int oB = bo2[tb_ % 3] + (tb_ / 3) * IWP * 32;
      int o0 = sub ? oB : oA;
      if constexpr (tpk == 4) {
        constexpr int tc = tpk * rr + 2, td = tpk * rr + 3;
        constexpr int tc_ = tc < KT ? tc : 0, td_ = td < KT ? td : 0;
        const int oC = bo2[tc_ % 3] + (tc_ / 3) * IWP * 32;
        const int oD = bo2[td_ % 3] + (td_ / 3) * IWP * 32;
        o0 = sub == 0 ? oA : sub == 1 ? oB : sub == 2 ? oC : oD;
      }
      o = o0 + r * IWP * 32;
    }
    ob[Q][0] = *reinterpret_cast<const f16x8 *>(Li + o);
    ob[Q][1] = *reinterpret_cast<const f16x8 *>(Li + IMG + o);
  };
  f32x4 am[RW][NT], ac[RW][NT];
  f32x4 rv1[NRES >= 1 ? RW : 1][NT];
  auto full_tile = [&](const TI &ti) {
    return ti.oy0 + G::TH <= p.Ho && ti.ox0 + 16 <= p.Wo && ti.n0 + BN <= p.cout;
  };
  auto load_res = [&](const TI &ti) {
    if constexpr (NRES == 0) return;
    const int64_t rowb = (int64_t)ti.oy0 * p.Wo;
    const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(p.res + rowb * p.rcs + p.rco), (short)0, 0x7fff0000, 0x00020000);
    const bool full = full_tile(ti);
    const int px = cw * RW * p.Wo + ti.ox0 + col, n = ti.n0 + hi * 4;
    const int rows_ok = p.Ho - ti.oy0 - cw * RW;
    const bool lane_ok = ti.ox0 + col < p.Wo;
    const int o1b = (px * p.rcs + n) * 4, r1row = p.Wo * p.rcs * 4;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bool ok = full | ((r < rows_ok) & lane_ok & (n + j * 16 < p.cout));
        const int o1 = ok ? o1b + r * r1row + j * 64 : 0x7ffffff0;
        if constexpr (NRES >= 1)
          rv1[r][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r1, o1, 0, 0));
      }
  };
  // out = scale * (res + act((am + 2^-11 ac) + bias)), sconv's order
  auto epilogue = [&](const TI &ti) {
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        p.y + (int64_t)ti.oy0 * p.Wo * p.ycs + p.yco, (short)0, 0x7fff0000, 0x00020000);
    const bool full = full_tile(ti);
    const int px = cw * RW * p.Wo + ti.ox0 + col, n = ti.n0 + hi * 4;
    f32x4 bb[NT], sc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int nc = n + j * 16 < p.cout ? n + j * 16 : 0;
      bb[j] = lds_read16(Lc + nc);
      sc[j] = lds_read16(Lc + p.cout + nc);
    }
    lds_wait4(bb);
    lds_wait4(sc);
    const int rows_ok = p.Ho - ti.oy0 - cw * RW;
    const bool lane_ok = ti.ox0 + col < p.Wo;
    const int o0 = (px * p.ycs + n) * 4, orow = p.Wo * p.ycs * 4;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (am[r][j][e] + ac[r][j][e] * kLoInv) + bb[j][e];
        if (p.act == DCVC_ACT_LRELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = lrelu_in(v[e], p.slope);
        }
        if constexpr (NRES >= 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = rv1[r][j][e] + v[e];
        }
        if (p.scale) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= sc[j][e];
        }
        const bool ok = full | ((r < rows_ok) & lane_ok & (n + j * 16 < p.cout));
        const int o = ok ? o0 + r * orow + j * 64 : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), yr, o, 0, 0);
      }
  };

  // ---------------------------------------------------------------- prologue
  // (each role's prologue and tile loop sit in one branch: the register
  // allocator then never sees the producer's image registers and the
  // consumer's operands live at once)
  TI tcur = tile_of(g);
  if (dma_wave) {
    {
      int dv0[DPW];
      dma_lanes(tcur.n0, dv0);
      wfor<AH>([&](auto k_) {
        constexpr int k = decltype(k_)::value;
        if constexpr (k < NST) dma_w(tcur.n0, dv0, std::integral_constant<int, k>{}, k);
      });
    }
    wait_vm_lgkm();
    raw_barrier();
    // (a second prologue barrier: the consumers read stage 0's fragments
    // from slot 0 between the two, and stage 0 DMAs into slot 0)
    raw_barrier();
    int kw = 0;   // ring slot of the current stage (stage counter mod NSW)
    for (int t = g; t < p.ntiles; t += GR) {
      TI tc = tcur, tx = t + GR < p.ntiles ? tile_next(tcur) : tcur;
      opaque_s(tc.n0);
      opaque_s(tx.n0);
      opaque_s(wcb);
      opaque_s(wrb);
      int dvc[DPW], dvx[DPW];
      dma_lanes(tc.n0, dvc);
      dma_lanes(tx.n0, dvx);
      wfor<NST>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        const int kw_ = G::RING_STATIC ? s % NSW : kw;
        // the weights of stage s + AH (this tile or the next) into the
        // current stage's slot (its fragments were read during stage s - 1)
        if (WDBG(16)) {
        } else if constexpr (s + AH < NST) dma_w(tc.n0, dvc, std::integral_constant<int, (s + AH) % NST>{}, kw_);
        else dma_w(tx.n0, dvx, std::integral_constant<int, (s + AH) % NST>{}, kw_);
        // stage s + 2's weights landed: the DMAs of the AH - 2 later stages
        // may stay in flight
        constexpr int N = G::wait_n(s);
        sched_fence();
        if (WDBG(16)) wait_lgkm();
        else wait_vm_n_lgkm<N>();
        sched_fence();
        if (!WDBG(32)) raw_barrier();
        sched_fence();
        kw = kw + 1 >= NSW ? 0 : kw + 1;
      });
      tcur = tx;
    }
    wait_vm_lgkm();   // no LDS-DMA left in flight when the workgroup exits
  } else if (producer) {
    load_img(tcur, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    load_img(tcur, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    publish(0, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},
            std::integral_constant<int, PPM>{});
    wait_lgkm();
    raw_barrier();
    raw_barrier();
    for (int t = g; t < p.ntiles; t += GR) {
      TI tc = tcur, tx = t + GR < p.ntiles ? tile_next(tcur) : tcur;
      opaque_s(tc.n0), opaque_s(tc.oy0), opaque_s(tc.ox0);
      opaque_s(tx.n0), opaque_s(tx.oy0), opaque_s(tx.ox0);
      wfor<NST>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        constexpr int c = G::chunk(s), rr = G::row(s);
        // image loads of chunk c + 2 (this tile's, or the next tile's) into
        // set c & 1, whose chunk c went to LDS during chunk c - 1
        if constexpr (rr == 0) {
          constexpr int c2 = (c + 2) % CH;
          if (WDBG(8)) {
          } else if constexpr (c + 2 < CH) load_img(tc, std::integral_constant<int, c2>{}, std::integral_constant<int, c & 1>{});
          else load_img(tx, std::integral_constant<int, c2>{}, std::integral_constant<int, c & 1>{});
        }
        // this stage's share of chunk c + 1's publish into image buffer
        // (c + 1) & 1, whose previous chunk (c - 1) the consumers last read
        // during chunk c - 1's last stage
        {
          constexpr int c1 = (c + 1) % CH;
          constexpr int u0 = G::pub0(c, rr), u1 = G::pub0(c, rr + 1);
          if constexpr (u1 > u0)
            if (!WDBG(4)) publish((c + 1) & 1, std::integral_constant<int, c1>{}, std::integral_constant<int, (c + 1) & 1>{},
                    std::integral_constant<int, u0>{}, std::integral_constant<int, u1>{});
        }
        sched_fence();
        wait_lgkm();
        sched_fence();
        if (!WDBG(32)) raw_barrier();
        sched_fence();
      });
      tcur = tx;
    }
  } else {
    // the MFMA waves win the issue arbitration against their SIMD's producer
    // wave (which has VALU / memory work to spread into their MFMA shadows)
    if (!WDBG(128)) __builtin_amdgcn_s_setprio(2);
    wait_lgkm();
    raw_barrier();
    read_a(std::integral_constant<int, 0>{}, 0);
    read_b(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, 0, std::integral_constant<int, 0>{});
    wait_lgkm();
    raw_barrier();
    int kw = 0;
    for (int t = g; t < p.ntiles; t += GR) {
      TI tc = tcur, tx = t + GR < p.ntiles ? tile_next(tcur) : tcur;
      opaque_s(tc.n0), opaque_s(tc.oy0), opaque_s(tc.ox0);
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          am[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          ac[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      if (!WDBG(64)) load_res(tc);
      opaque_v(aoff);
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) opaque_v(bo1[dx]), opaque_v(bo2[dx]);
      wfor<NST>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        constexpr int c = G::chunk(s);
        constexpr int S = s & 1;                       // operand set of stage s
        const int kw_ = G::RING_STATIC ? s % NSW : kw;
        // operands of stage s + 1 (the next tile's stage 0 at the last
        // stage): the weight fragments now, the image rows through the ring
        constexpr int s1 = s + 1 < NST ? s + 1 : 0;
        constexpr int c1 = G::chunk(s1);
        const int ib = c & 1;                                        // this stage's image buffer
        const int ib1 = s + 1 < NST ? (c1 & 1) : 0;                  // the next stage's
        const int ws1 = kw_ + 1 >= NSW ? 0 : kw_ + 1;
        if (!WDBG(2)) read_a(std::integral_constant<int, S ^ 1>{}, ws1);
        // rows: row r + 1 (after row 3: row 0 of stage s + 1) read while row
        // r's MFMAs run; row 0 of this stage came in at the previous stage
        // (ring slot of row r: the parity of the wave's row count s RW + r,
        // so that with RW = 3 the next stage's row 0 does not land on row 2)
        wfor<RW>([&](auto r_) {
          constexpr int r = decltype(r_)::value;
          constexpr int q = (s * RW + r) & 1;
          if (WDBG(2)) {
          } else if constexpr (r + 1 < RW)
            read_b(s_, std::integral_constant<int, r + 1>{}, ib, std::integral_constant<int, q ^ 1>{});
          else
            read_b(std::integral_constant<int, s1>{}, std::integral_constant<int, 0>{}, ib1,
                   std::integral_constant<int, q ^ 1>{});
          if (WDBG(1)) return;
          // (two passes, so the two products accumulated into ac[r][j] sit
          // 2 NT - 1 MFMAs apart: none waits on its predecessor's result;
          // the accumulation order, and so the bits, are unchanged)
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            am[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[S][j][0], ob[q][0], am[r][j], 0, 0, 0);
            ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[S][j][0], ob[q][1], ac[r][j], 0, 0, 0);
          }
#pragma unroll
          for (int j = 0; j < NT; ++j)
            ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[S][j][1], ob[q][0], ac[r][j], 0, 0, 0);
        });
        if constexpr (s == NST - 1) {
          if (!WDBG(64)) epilogue(tc);
        }
        sched_fence();
        wait_lgkm();
        sched_fence();
        if (!WDBG(32)) raw_barrier();
        sched_fence();
        kw = kw + 1 >= NSW ? 0 : kw + 1;
      });
      tcur = tx;
    }
  }
}

// The DMA waves' vector-memory schedule the exact vmcnt waits assume, per
// stage (every stage ends at a barrier): DPW weight LDS-DMAs (D) and the
// wait's count.
// scripts/check_xconv_vmcnt.py compares it with the emitted producer loop, as
// for xconv.hip (make runs it).  Line per stage: "<ops> <wait>".
template <int CIN, int BN, int NRES>
int sched_dump(char *buf, int cap) {
  typedef WG<CIN, BN, NRES> G;
  std::string out = "nst " + std::to_string(G::NST) + " nsw " + std::to_string(G::NSW) + "\n";
  for (int x = 0; x < G::NST; ++x) {
    std::string ops(G::DPW, 'D');
    out += ops + " " + std::to_string(G::wait_n(x)) + "\n";
  }
  if ((int)out.size() + 1 > cap) return DCVC_HIP_EINVAL;
  std::memcpy(buf, out.c_str(), out.size() + 1);
  return DCVC_HIP_OK;
}
struct SchedEntry {
  int cin, bn, nres;
  int (*dump)(char *, int);
};
#define WCONV_SCHED(C) {C, 32, 0, &sched_dump<C, 32, 0>}, {C, 32, 1, &sched_dump<C, 32, 1>}, \
                       {C, 48, 0, &sched_dump<C, 48, 0>}, {C, 48, 1, &sched_dump<C, 48, 1>}
const SchedEntry g_sched[] = {WCONV_SCHED(48), WCONV_SCHED(64), WCONV_SCHED(128), WCONV_SCHED(192)};
#undef WCONV_SCHED

int g_cus = 0;
int g_dbg = 0;
int g_enable = 0;   // dcvc_set_option("wconv", 1) routes these layers here (else xconv.hip)

template <int CIN, int BN, int NRES>
int launch(WP p, hipStream_t st) {
  typedef WG<CIN, BN, NRES> G;
  const size_t lds = G::lds(p.cout);
  if (lds > (size_t)G::LDS_WG) return DCVC_HIP_EUNSUPPORTED;
  p.tiles_x = (p.Wo + 15) / 16;
  const int tiles_y = (p.Ho + G::TH - 1) / G::TH;
  p.nblk = (p.cout + BN - 1) / BN;
  const int64_t nt = (int64_t)p.tiles_x * tiles_y * p.nblk;
  if (nt <= 0) return DCVC_HIP_OK;
  if (nt > 0x7fffffff) return DCVC_HIP_EINVAL;
  p.ntiles = (int)nt;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  int64_t grid = g_cus;
  if (grid > nt) grid = nt;
  auto kern = wconv3_kernel<CIN, BN, NRES>;
  dcvc_note_kernel("wconv3_kernel<%d, %d, %d>@%lld", CIN, BN, NRES, (long long)grid * G::NTH);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(G::NTH), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

template <int CIN>
int pick(WP p, hipStream_t st) {
  // n-block: the whole cout at 32 / 48 channels, else 48- or 32-channel blocks
  if (p.cout == 32 || (p.cout % 48 && p.cout % 32 == 0))
    return p.has_res ? launch<CIN, 32, 1>(p, st) : launch<CIN, 32, 0>(p, st);
  if (p.cout % 48 == 0) return p.has_res ? launch<CIN, 48, 1>(p, st) : launch<CIN, 48, 0>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

}  // namespace

// 3x3 stride-1 f16x3 convolutions the wave-specialised kernel takes (conv.hip
// tries it before xconv.hip); DCVC_HIP_EUNSUPPORTED leaves the call to xconv.
extern "C" int dcvc_internal_wconv(const dcvc_conv_args *a, void *stream) {
  if (!g_enable) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1 || a->shuffle || a->res2.ptr)
    return DCVC_HIP_EUNSUPPORTED;
  if (a->cin != 48 && a->cin != 64 && a->cin != 128 && a->cin != 192) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && a->in_op != DCVC_IN_LRELU) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  if (a->act != DCVC_ACT_NONE && !(a->act == DCVC_ACT_LRELU && a->slope >= 0.f && a->slope <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op == DCVC_IN_LRELU && !(a->in_slope >= 0.f && a->in_slope <= 1.f)) return DCVC_HIP_EUNSUPPORTED;
  if (a->cout % 32 && a->cout % 48) return DCVC_HIP_EUNSUPPORTED;
  WP p{};
  p.dbg = g_dbg;
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.Ho = a->x.H;
  p.Wo = a->x.W;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cout = a->cout;
  p.in_lrelu = a->in_op == DCVC_IN_LRELU;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.bias = a->bias;
  p.scale = a->scale;
  if (a->y.W != p.Wo || a->y.H != p.Ho) return DCVC_HIP_EUNSUPPORTED;
  bool ok = p.xcs % 4 == 0 && p.xco % 4 == 0 && (uintptr_t)p.x % 16 == 0;
  ok = ok && p.ycs % 4 == 0 && p.yco % 4 == 0 && (uintptr_t)p.y % 16 == 0;
  if (a->res.ptr) {
    p.res = reinterpret_cast<const float *>(a->res.ptr);
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
    p.has_res = 1;
    ok = ok && a->res.dtype == DCVC_F32 && p.rcs % 4 == 0 && p.rco % 4 == 0 && (uintptr_t)p.res % 16 == 0;
  }
  if (!ok) return DCVC_HIP_EUNSUPPORTED;
  // per-tile buffer offsets below 2^31 bytes (xconv.hip's bounds)
  if ((int64_t)16 * p.Wo * std::max(p.ycs, p.rcs) * 4 >= ((int64_t)1 << 30)) return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)19 * p.W * p.xcs * 4 >= 0x7fff0000) return DCVC_HIP_EUNSUPPORTED;
  const int nch = (a->cin + 31) / 32;
  const int vc = a->cin - 32 * (nch - 1);
  const int tpkl = vc <= 8 ? 4 : vc <= 16 ? 2 : 1;
  p.wchunk = (int64_t)2 * 9 * a->cout * 32;
  {
    const int rl = (9 + tpkl - 1) / tpkl;
    const int64_t wb = ((int64_t)(nch - 1) * p.wchunk + (int64_t)2 * rl * a->cout * 32) * 2;
    if (wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
    p.wbytes = (int)wb;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (a->cin) {
    case 48: return pick<48>(p, st);
    case 64: return pick<64>(p, st);
    case 128: return pick<128>(p, st);
    case 192: return pick<192>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}

extern "C" void dcvc_internal_wconv_enable(int v) { g_enable = v; }
extern "C" void dcvc_internal_wconv_dbg(int v) { g_dbg = v; }

// scripts/check_xconv_vmcnt.py: the producer schedule of instantiation i
// (cin, bn, nres into prm[3]); DCVC_HIP_EINVAL past the last
extern "C" int dcvc_internal_wconv_schedule(int i, int *prm, char *buf, int cap) {
  if (i < 0 || i >= (int)(sizeof g_sched / sizeof g_sched[0])) return DCVC_HIP_EINVAL;
  const SchedEntry &e = g_sched[i];
  prm[0] = e.cin, prm[1] = e.bn, prm[2] = e.nres;
  return e.dump(buf, cap);
}
