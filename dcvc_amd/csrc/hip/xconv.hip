// Static-shape split-fp16 3x3 stride-1 convolution: the feature-rate 3x3
// layers of Precision.split() (ResBlocks, context fusion, UNet / recon convs
// of DCVC-DC/src/models/video_net.py:58-76, 129-170 and video_model.py:89-118,
// 173-232).  Same arithmetic as sconv.hip (x * w ~ xh*wh + 2^-11 (xh*wl +
// xl*wh) on v_mfma_f32_16x16x32_f16, fp32 accumulation, the same K order and
// the same epilogue), so the outputs are bit-identical to sconv_kernel's.
//
// What differs is the schedule.  sconv.hip carries the channel count, chunk
// count and tap packing at run time; hipcc then keeps the stage loop as a
// chain of run-time branches with the accumulators copied at every merge and
// spills SGPRs into VGPR lanes (~5 VALU per MFMA, MFMA busy ~30 %).  Here CIN,
// the n-block BN and the tile are template parameters, the K walk of a tile is
// unrolled at compile time, and every stage has the same shape:
//
//   stage = one K step of 32 (one tap of a 32-channel chunk, or 2 / 4 packed
//           taps of a 16- / 8-channel last chunk), one workgroup barrier;
//   weights: streamed through a ring of LDS slots by LDS-DMA, issued as many
//           stages ahead as the ring is deep (6 to 12 slots, a depth that
//           divides the tile's stage count where one fits, so every slot
//           address is compile-time; L2-resident: every tile reads the same
//           weights);
//   operands: the next stage's A (weights) and B (image) fragments are read
//           from LDS while the current stage's MFMAs run (two register sets),
//           so no wave waits on LDS latency at a stage start;
//   image:  two LDS buffers (hi / lo f16 images, XOR-swizzled); the next
//           chunk's input pieces are loaded into registers at a chunk's first
//           stage and split into the other buffer at its second-to-last, so
//           the publish VALU runs between MFMAs and never behind a barrier;
//   residual / second residual: loaded into registers at the tile's first
//           stage, consumed by the epilogue straight from the accumulators.
//
// Every vector-memory instruction of a stage is issued unconditionally (buffer
// loads / stores with out-of-range offsets where there is nothing to move), so
// the count of vector-memory operations younger than a stage's weight DMA is a
// compile-time constant and the DMA is waited for with an exact vmcnt(N) that
// never drains the younger image / residual loads.  Exact means issued AND
// used: hipcc deletes a load whose value is dead, so a padding load counted
// but never read (round 5 loaded a 16-channel chunk's image with the 32-channel
// chunk's piece count) makes N too large and the wait pass early.
#include "common.h"
#include "split.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace {

struct XP {
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
  const float *res2;
  int r2cs, r2co;
  int has_res, has_res2;
  int tiles_x, nblk, ntiles;
  int wbytes;
  int64_t wchunk;          // halves of one full chunk's packed weights (hi + lo)
  const float *bias;
  const float *scale;
  int *ovf;               // fp16 range guard (split.h SplitRange)
  int shuffle;            // pixel-shuffled output (r = 2)
  int dbg;                // timing ablations (dcvc_set_option("xconv_dbg")), 0 in production
};

template <typename F, int... I>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}

#ifdef XCONV_DBG
// per-stage clock stamps of workgroup 0's second tile (ablation builds):
// [wave][2 * stage + {0: MFMAs issued, 1: past the barrier}], low 32 bits of s_memtime
__device__ unsigned g_xstamps[8 * 64];
#endif

template <int CIN, int BN, int RW, int NW, int NRES, int KS = 3>
struct XG {
  // KS x KS kernel (3 or 7), pad KS / 2: a 16-column tile reads a halo image
  // of IH x IW pixels, rows padded to IWP (a multiple of 4 pixels, swzx)
  static constexpr int KT = KS * KS, NTH = NW * 64, TH = NW * RW, NT = BN / 16;
  static constexpr int IH = TH + KS - 1, IW = 15 + KS, IWP = (IW + 3) & ~3;
  static constexpr int CH = (CIN + 31) / 32;
  static constexpr int VCL = CIN - 32 * (CH - 1);
  static constexpr int TPKL = VCL <= 8 ? 4 : (VCL <= 16 ? 2 : 1);
  static constexpr int ROWSL = (KT + TPKL - 1) / TPKL;
  static constexpr int NST = (CH - 1) * KT + ROWSL;         // K steps (stages) per tile
  static constexpr int NSLF = 4, NSLL = TPKL == 1 ? 4 : 4 / TPKL;   // 8-channel slots staged per chunk
  static constexpr int PPF = (IH * IW * NSLF + NTH - 1) / NTH;      // image pieces per thread, full chunk
  static constexpr int PPL = (IH * IW * NSLL + NTH - 1) / NTH;      // ... last chunk
  static constexpr int PPM = PPF > PPL ? PPF : PPL;
  static constexpr int IMG = IH * IWP * 32;                 // halves per image (hi or lo)
  static constexpr int WST = BN * 32;                       // halves per weight stage (hi or lo)
  static constexpr int NDMA = 2 * BN / 16;                  // 1-KiB LDS-DMA pieces per stage
  static constexpr int DPW = (NDMA + NW - 1) / NW;          // ... per wave (every wave issues DPW)
  // vector-memory instructions per thread: image chunk loads (two per piece of
  // the chunk loaded: a last chunk of 8 or 16 channels has fewer pieces), tile
  // loads (res, res2), epilogue stores
  static constexpr int NTILE = NRES * RW * NT;
  // stages that publish an image piece, and the tile's last stage, issue
  // their weight DMA after that work (its epilogue stores then precede the
  // DMA).  hipcc's own vmcnt waits do not count LDS-DMAs, so its wait for a
  // published piece's loads, and its wait before the epilogue's LDS reads,
  // also waited for a DMA issued a few instructions earlier: a memory round
  // trip per tile in each case
  static constexpr bool DMA_LATE = true;
  static constexpr int NSTORE = RW * NT;
  // image loads of stage x: a chunk's first stage loads the next chunk (of
  // this tile, or the next tile's first).  Exact, not an upper bound: a count
  // above the loads really issued lets a vmcnt wait pass with the DMA it
  // waits for still in flight (the round-5 ring race)
  static constexpr int img_ops(int x) {
    if (st_row_(x) != 0) return 0;
    const int c = x < (CH - 1) * KT ? x / KT : CH - 1;
    const int cl = c + 1 < CH ? c + 1 : 0;
#ifdef XCONV_DEAD_LOAD_PROBE
    // (tests/test_xconv_vmcnt_check.py: round 5's count, every chunk's load
    // counted at the larger piece count, which the emitted code contradicts)
    return 2 * PPM;
#endif
    return 2 * (cl == CH - 1 ? PPL : PPF);
  }
  // vector-memory instructions per thread issued by stage x of a tile after
  // its weight DMA, and in all
  static constexpr int after_dma(int x) {
    return img_ops(x) + (x == 0 ? NTILE : 0) + (x == NST - 1 && !DMA_LATE ? NSTORE : 0);
  }
  static constexpr int all_ops(int x) { return DPW + after_dma(x); }
  // does stage x publish (a piece of) the next chunk's image (the kernel's step 6)
  static constexpr bool publishes(int x) {
    const int c = x < (CH - 1) * KT ? x / KT : CH - 1, rr = st_row_(x);
    const int rows = c == CH - 1 ? ROWSL : KT;
    const int cn = c + 1 < CH ? c + 1 : 0;
    const int ppn = cn == CH - 1 ? PPL : PPF;
    const int pend = bar(x - rr + rows - 2) ? rows - 2 : rows - 3;
    const int w0 = pend + 1 - ppn;
    return w0 >= 1 ? (rr >= w0 && rr <= pend) : rr == pend;
  }
  static constexpr int st_row_(int x) { return x < (CH - 1) * KT ? x % KT : x - (CH - 1) * KT; }
  // stage s + 1 reads the weight fragments of stage s + 2 (after its MFMAs),
  // so at the end of stage s the weights of stage s + 2 must have landed:
  // their DMA was issued by stage s + 2 - AH (of this tile or the previous
  // one, the schedule repeats per tile); the operations issued after it may
  // stay in flight (vmcnt counts them in issue order)
  static constexpr int wait_for_old(int s, int ah) {
    int n = after_dma((s + 2 - ah + 2 * NST) % NST);
    for (int k = 1; k < ah - 1; ++k) n += all_ops((s + 2 - ah + k + 2 * NST) % NST);
    return n;
  }
  // Barriers at every other stage (PB): at the end of odd stages and of the
  // tile's last stage.  A barrier stage s then waits for the weights read
  // before the next barrier: the reads of stages s + 1 .. nb (the next
  // barrier stage) take stages s + 2 .. nb + 1, so DMA(nb + 1) must have
  // landed; non-barrier stages wait for nothing
  static constexpr bool PB = true;
  static constexpr bool bar(int s) { return !PB || (s % 2 == 1) || s == NST - 1; }
  static constexpr int next_bar(int s) {   // extended stage index (past NST: the next tile)
    for (int x = s + 1; x < s + 2 * NST + 2; ++x)
      if (bar(x % NST)) return x;
    return s + 1;
  }
  static constexpr int wait_for(int s, int ah) {
    if (!bar(s)) return 63;   // (unused)
    const int x0 = next_bar(s) + 1 - ah;   // the stage that issued DMA(nb + 1), <= s
    int n = after_dma((x0 + 2 * NST) % NST);
    for (int x = x0 + 1; x <= s; ++x) n += all_ops((x + 2 * NST) % NST);
    return n;
  }
  // weight ring: NSW slots, the DMA of a stage issued AH = NSW - 1 stages
  // ahead; as many slots as the LDS holds beside the image buffers (at most a
  // tile's stages + 1).  vmcnt completes in issue order, so every image /
  // residual load and output store issued before a weight DMA has to land
  // before that DMA is waited for: a deep ring gives them AH - 1 stages (the
  // HBM latency under load), not the one or two a shallow ring would.
  // One workgroup per CU: 8 waves of 2 rows (two waves per SIMD, 256
  // registers each) or 4 waves of 4 rows (one wave per SIMD, 512 registers)
  static constexpr int WPC = 1;                              // workgroups per CU
  static constexpr int WPE = NW == 4 ? 1 : 2;                // waves per SIMD
  static constexpr int LDS_WG = 160 * 1024 / WPC;
  static constexpr int NSW_FIT = (LDS_WG - 2048 - 4 * IMG * 2 - 1024) / (2 * WST * 2);
  // the deepest ring that fits, has at most a tile's stages + 1 slots and
  // keeps every stage's count of younger vector-memory operations below 64
  // (vmcnt is 6 bits); preferably (6 slots or more) one whose depth divides
  // the tile's stage count: every stage of every tile then uses the same slot,
  // so the slot arithmetic and the LDS / DMA addresses built from it are
  // compile-time (2-3 % faster on 48 -> 48)
  static constexpr bool vm_ok(int n) {
    for (int x = 0; x < NST; ++x)
      if (bar(x) && wait_for(x, n - 1) >= 64) return false;
    return true;
  }
  static constexpr int pick_nsw() {
    int n = NSW_FIT < 12 ? NSW_FIT : 12;
    if (n > NST + 1) n = NST + 1;
#ifndef XCONV_RING_DYN
    for (int d = n; d >= 6; --d)
      if (NST % d == 0 && vm_ok(d)) return d;
#endif
    for (; n > 4; --n)
      if (vm_ok(n)) break;
    return n;
  }
  static constexpr int NSW = pick_nsw(), AH = NSW - 1;
  static constexpr bool RING_STATIC = NST % NSW == 0;
  static_assert(NSW >= 4, "weight ring too shallow");
  // LDS (halves): [2 image buffers][hi, lo][IMG] | [NSW weight slots][hi, lo][WST] | DMA sink 512 | consts
  static constexpr int L_W = 4 * IMG;
  static constexpr int L_SINK = L_W + 2 * NSW * WST;
  static constexpr int L_C = L_SINK + 512;
  static constexpr size_t lds(int cout) { return (size_t)L_C * 2 + (size_t)2 * cout * 4; }
  static constexpr int wait_n(int s) { return wait_for(s, AH); }
};

// stage s of a tile -> (chunk, row of the chunk)
template <int KT, int CH>
__host__ __device__ constexpr int st_chunk(int s) { return s < (CH - 1) * KT ? s / KT : CH - 1; }
template <int KT, int CH>
__host__ __device__ constexpr int st_row(int s) { return s - st_chunk<KT, CH>(s) * KT; }

template <int CIN, int BN, int RW, int NW, int NRES, bool SHUF, int KS>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 4 ? 1 : 2, NW == 4 ? 1 : 2)))
xconv3_kernel(XP p) {
  typedef XG<CIN, BN, RW, NW, NRES, KS> G;
  static_assert(!SHUF || NRES == 0, "pixel-shuffle outputs take no residuals");
  constexpr int PAD = KS / 2;
  SplitRange rg(p.ovf);
#ifdef XCONV_DBG
  const int XDBG = p.dbg;   // timing ablations (ablation builds only)
#else
  constexpr int XDBG = 0;
#endif
  constexpr int NTH = G::NTH, NT = G::NT, IH = G::IH, IW = G::IW, IWP = G::IWP, IMG = G::IMG;
  constexpr int WST = G::WST, CH = G::CH, KT = G::KT, TPKL = G::TPKL, ROWSL = G::ROWSL, NST = G::NST;
  constexpr int NDMA = G::NDMA, DPW = G::DPW, PPF = G::PPF, PPL = G::PPL, PPM = G::PPM;
  static_assert(NST >= 3, "a tile needs at least three stages");
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *const L = reinterpret_cast<uint16_t *>(smem);
  float *const Lc = reinterpret_cast<float *>(smem + (size_t)G::L_C * 2);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;   // wave-uniform
  const int col = lane & 15, hi = lane >> 4;
  const int GR = gridDim.x;
  int g = blockIdx.x;
  if ((GR & 7) == 0) g = (g & 7) * (GR >> 3) + (g >> 3);   // consecutive tiles on one XCD
  if (g >= p.ntiles) return;

  // bias / scale of every output channel, once
  for (int i = tid; i < p.cout; i += NTH) {
    Lc[i] = p.bias ? p.bias[i] : 0.f;
    // (with pixel shuffle the scale is per output channel, cout / 4 of them)
    Lc[p.cout + i] = p.scale && i < (SHUF ? p.cout >> 2 : p.cout) ? p.scale[i] : 1.f;
  }

  // ---- image piece plan.  Piece u of a chunk with NS staged 8-channel slots
  // = (halo row iy, halo column ix, slot), recomputed where it is used (a few
  // VALU with constant divisors) rather than kept live through the kernel
  constexpr int NTOTF = IH * IW * 4, NTOTL = IH * IW * G::NSLL;
  struct Piece {
    int iy, ix, slot, valid;
  };
  auto piece = [&](int u, auto NS_) {
    constexpr int NS = decltype(NS_)::value;
    const int it = tid + u * NTH;
    const int pix = it / NS;
    Piece q;
    q.slot = it - pix * NS;
    q.iy = pix / IW;
    q.ix = pix - q.iy * IW;
    q.valid = it < IH * IW * NS;
    return q;
  };
  float pf[PPM][8];   // image pieces in flight (one chunk)

  struct TI {
    int oy0, ox0, n0;
    int nb, tx, ty;   // n-block, tile column, tile row
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
  // tile t + GR from tile t: the grid stride split once into n-block, column
  // and row steps, so a tile's coordinates cost a few adds instead of
  // tile_of's four divisions (~100 scalar instructions at every tile start,
  // issued by every wave of the CU ahead of the tile's first MFMAs)
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

  // registers <- global: the input pieces of chunk c of a tile.  Every load is
  // issued (halo outside the image and pieces past the plan read zeros
  // through out-of-range offsets); tiles whose halo lies inside the image
  // skip the per-piece bounds tests
  auto load_img = [&](const TI &ti, auto C_) {
    constexpr int c = decltype(C_)::value;
    constexpr bool last = c == CH - 1;
    constexpr int PP = last ? PPL : PPF, NTOT = last ? NTOTL : NTOTF;
    if (XDBG & 64) return;
    const int iy0 = ti.oy0 - PAD, ix0 = ti.ox0 - PAD;
    const int rb = iy0 > 0 ? iy0 : 0;
    const int64_t eb = (int64_t)rb * p.W * p.xcs + p.xco + c * 32;
    int64_t nrec = ((int64_t)p.H * p.W * p.xcs - eb) * 4;
    if (nrec > 0x7fff0000) nrec = 0x7fff0000;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.x + eb), (short)0, (int)nrec, 0x00020000);
    const int toff = ((iy0 - rb) * p.W + ix0) * p.xcs;
    const bool inner = iy0 >= 0 && ix0 >= 0 && iy0 + IH <= p.H && ix0 + IW <= p.W;
    // (PP pieces, every one published: G::img_ops counts exactly these loads)
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const Piece q = piece(u, std::integral_constant<int, last ? G::NSLL : 4>{});
      int o = (toff + (q.iy * p.W + q.ix) * p.xcs + q.slot * 8) * 4;
      if (!inner) {
        const int gy = iy0 + q.iy, gx = ix0 + q.ix;
        if (!((unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W)) o = 0x7fffffe0;
      }
      if ((u + 1) * NTH > NTOT && !q.valid) o = 0x7fffffe0;
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[u][j] = a[j];
        pf[u][4 + j] = b[j];
      }
    }
  };
  // LDS image buffer ib <- registers, split (ResBlock's leaky ReLU first:
  // lrelu(v) = max(v, slope v) for 0 <= slope <= 1)
  // (pieces [U0, U1) of the chunk: a chunk's publish is spread over several
  // stages, so no stage carries all of its VALU work beside its 18 MFMAs)
  auto publish = [&](int ib, auto C_, auto U0_, auto U1_) {
    constexpr int c = decltype(C_)::value;
    constexpr bool last = c == CH - 1;
    constexpr int PP = last ? PPL : PPF, NTOT = last ? NTOTL : NTOTF;
    constexpr int U0 = decltype(U0_)::value, U1 = decltype(U1_)::value < PP ? decltype(U1_)::value : PP;
    uint16_t *const Lh = L + ib * 2 * IMG;
    if (p.in_lrelu) {
#pragma unroll
      for (int u = U0; u < U1; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[u][j] = lrelu_in(pf[u][j], p.in_slope);
    }
#pragma unroll
    for (int u = U0; u < U1; ++u) {
      u32x4_t h, l;
      rg.add8(pf[u]);
      split8(pf[u], h, l);
      const Piece q = piece(u, std::integral_constant<int, last ? G::NSLL : 4>{});
      const int o = swzx(q.iy * IWP + q.ix, q.ix, q.slot);
      const bool ok = (u + 1) * NTH <= NTOT || q.valid;
      if (ok) {
        *reinterpret_cast<u32x4_t *>(Lh + o) = h;
        *reinterpret_cast<u32x4_t *>(Lh + IMG + o) = l;
      }
    }
  };

  // LDS-DMA of the weights of stage s into slot ws: 16 rows of 64 bytes per
  // instruction; lane i writes physical slot i % 4 of row i / 4, so it reads
  // the logical slot the swizzle puts there.  Every wave issues DPW
  // instructions (the surplus into a sink).  The source offset is split into a
  // per-lane part (dv: the lane's row and slot, or out of range for rows past
  // cout and sink pieces; fixed per tile) and a uniform part (soffset: chunk,
  // hi / lo block, kernel row, n-block)
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
  int dlane[DPW], drow[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) {
    const int i = wave + NW * d;
    const int hl = i >= NDMA / 2, k = hl ? i - NDMA / 2 : i;
    const int R = k * 16 + (lane >> 2);
    const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
    dlane[d] = (R * 32 + ls * 8) * 2;
    drow[d] = i < NDMA ? R : 0x7fff;
  }
  // per-lane DMA offsets of an n-block starting at n0
  auto dma_lanes = [&](int n0, int (&dv)[DPW]) {
#pragma unroll
    for (int d = 0; d < DPW; ++d) dv[d] = drow[d] < p.cout - n0 ? dlane[d] : 0x7ffffff0;
  };
  int wcb = (int)(p.wchunk * 2), wrb = p.cout * 64;   // bytes per full chunk, per kernel row (hi or lo block)
  auto dma_w = [&](int n0, const int (&dv)[DPW], auto s_, int ws) {
    constexpr int s = decltype(s_)::value;
    // one piece per wave: the waves past the stage's pieces issue nothing
    // (their vmcnt waits then only cover their own register loads, which the
    // compiler waits for at their use); with several pieces per wave every
    // wave issues DPW (the surplus into the sink) to keep its count exact
    if (DPW == 1 && wave >= NDMA) return;
    constexpr int c = st_chunk<KT, CH>(s), rr = st_row<KT, CH>(s);
    constexpr int rows = c == CH - 1 ? ROWSL : KT;
#pragma unroll
    for (int d = 0; d < DPW; ++d) {
      const int i = wave + NW * d;   // wave-uniform
      const int hl = i >= NDMA / 2, k = hl ? i - NDMA / 2 : i;
      const int ub = c * wcb + (hl ? rows * wrb : 0) + rr * wrb + n0 * 64;
      uint16_t *dst = i < NDMA ? L + G::L_W + ws * 2 * WST + hl * WST + k * 512 : L + G::L_SINK;
      // device pass only: with a non-constant soffset the host pass drops the
      // kernel's launch stubs without a diagnostic
#ifdef __HIP_DEVICE_COMPILE__
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)dst, 16, dv[d], ub, 0,
                                               0);
#endif
    }
  };

  // per-lane operand offsets (halves): weights (row j * 16 + col, slot hi)
  int aoff = swz(col, hi);
  // image, one tap per K step: pixel (wave rows + dy, col + dx), slot hi
  int bo1[KS], bo2[KS];
#pragma unroll
  for (int dx = 0; dx < KS; ++dx) {
    const int x = col + dx;
    bo1[dx] = swzx(wave * RW * IWP + x, x, hi);
    // packed taps: slot hi % (4 / TPKL)
    constexpr int spt = 4 / TPKL;
    bo2[dx] = swzx(wave * RW * IWP + x, x, hi % spt);
  }
  const int sub = hi / (4 / TPKL);

  // operand registers: two sets of image fragments and, where the registers
  // allow it (at most one residual, and no 64-channel block with two waves
  // per SIMD: scripts/isa_probe.sh), two sets of weight fragments; the next
  // stage's are read at the start of a stage, so no LDS latency is left to
  // wait for at its end.  With one weight set, each fragment is refilled with
  // the next stage's right after its last MFMA of the stage
  constexpr bool DBA = NRES < 2 && (RW == 4 || BN < 64);
  f16x8 oa[DBA ? 2 : 1][NT][2], ob[2][RW][2];   // [set][frag][hi, lo]
  // LDS -> registers: the weight fragments of a stage (weight slot ws) into set S
  auto read_a = [&](auto S_, int ws) {
    constexpr int S = DBA ? decltype(S_)::value : 0;
    const uint16_t *Lw = L + G::L_W + ws * 2 * WST + aoff;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      oa[S][j][0] = *reinterpret_cast<const f16x8 *>(Lw + j * 512);
      oa[S][j][1] = *reinterpret_cast<const f16x8 *>(Lw + j * 512 + WST);
    }
  };
  // LDS -> registers: the image fragments of stage s (image buffer ib) into set S
  auto read_b = [&](auto S_, auto s_, int ib) {
    constexpr int S = decltype(S_)::value;
    constexpr int s = decltype(s_)::value;
    constexpr int c = st_chunk<KT, CH>(s), rr = st_row<KT, CH>(s);
    constexpr int tpk = c == CH - 1 ? TPKL : 1;
    const uint16_t *Li = L + ib * 2 * IMG;
    if constexpr (tpk == 1) {
      constexpr int dy = rr / KS, dx = rr % KS;
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int o = bo1[dx] + (r + dy) * IWP * 32;
        ob[S][r][0] = *reinterpret_cast<const f16x8 *>(Li + o);
        ob[S][r][1] = *reinterpret_cast<const f16x8 *>(Li + IMG + o);
      }
    } else {
      // lane group hi reads tap tpk * rr + sub (a tap past the kernel has
      // zero weights: any finite data, tap 0)
      constexpr int ta = tpk * rr, tb = tpk * rr + 1;
      constexpr int ta_ = ta < KT ? ta : 0, tb_ = tb < KT ? tb : 0;
      const int oA = bo2[ta_ % KS] + (ta_ / KS) * IWP * 32;
      const int oB = bo2[tb_ % KS] + (tb_ / KS) * IWP * 32;
      int o0 = sub ? oB : oA;
      if constexpr (tpk == 4) {
        // (8-channel last chunk: four taps per K step, one per lane group)
        constexpr int tc = tpk * rr + 2, td = tpk * rr + 3;
        constexpr int tc_ = tc < KT ? tc : 0, td_ = td < KT ? td : 0;
        const int oC = bo2[tc_ % KS] + (tc_ / KS) * IWP * 32;
        const int oD = bo2[td_ % KS] + (td_ / KS) * IWP * 32;
        o0 = sub == 0 ? oA : sub == 1 ? oB : sub == 2 ? oC : oD;
      }
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int o = o0 + r * IWP * 32;
        ob[S][r][0] = *reinterpret_cast<const f16x8 *>(Li + o);
        ob[S][r][1] = *reinterpret_cast<const f16x8 *>(Li + IMG + o);
      }
    }
  };

  f32x4 am[RW][NT], ac[RW][NT];
  // the MFMAs of a stage (operand set S); with one weight set, fragment j is
  // refilled from weight slot wsn after its last MFMA
  // (PASS with two operand sets: 0 all, 1 the am pass, 2 the two ac passes)
  auto mfmas = [&](auto S_, int wsn, auto PASS_) {
    constexpr int S = decltype(S_)::value, SA = DBA ? S : 0, PASS = decltype(PASS_)::value;
    if constexpr (DBA) {
      // in three passes, so the two products accumulated into ac[r][j] are
      // RW * NT MFMAs apart (no MFMA waits on its predecessor's result); the
      // same accumulation order, so the same bits
      if constexpr (PASS != 2) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < RW; ++r)
            am[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[SA][j][0], ob[S][r][0], am[r][j], 0, 0, 0);
      }
      if constexpr (PASS != 1) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < RW; ++r)
            ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[SA][j][0], ob[S][r][1], ac[r][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < RW; ++r)
            ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[SA][j][1], ob[S][r][0], ac[r][j], 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        am[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[SA][j][0], ob[S][r][0], am[r][j], 0, 0, 0);
        ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[SA][j][0], ob[S][r][1], ac[r][j], 0, 0, 0);
        ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oa[SA][j][1], ob[S][r][0], ac[r][j], 0, 0, 0);
      }
      if constexpr (!DBA) {
        const uint16_t *Lw = L + G::L_W + wsn * 2 * WST + aoff + j * 512;
        oa[0][j][0] = *reinterpret_cast<const f16x8 *>(Lw);
        oa[0][j][1] = *reinterpret_cast<const f16x8 *>(Lw + WST);
      }
    }
  };

  // the lane's output pieces: pixel (row wave * RW + r, column col), channels
  // n0 + 16 j + 4 hi .. + 3; offsets in elements from the tile's first output
  // pixel.  Full tiles (every piece inside the output) skip the tests
  auto full_tile = [&](const TI &ti) {
    return ti.oy0 + G::TH <= p.Ho && ti.ox0 + 16 <= p.Wo && ti.n0 + BN <= p.cout;
  };
  // tile-level register loads: the NRES residuals of the lane's output
  // pieces (always issued; zeros outside the output)
  f32x4 rv1[NRES >= 1 ? RW : 1][NT], rv2[NRES >= 2 ? RW : 1][NT];
  auto load_res = [&](const TI &ti) {
    if constexpr (NRES == 0) return;
    if (XDBG & 128) return;
    const int64_t rowb = (int64_t)ti.oy0 * p.Wo;
    const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(p.res + rowb * p.rcs + p.rco), (short)0, 0x7fff0000, 0x00020000);
    __amdgpu_buffer_rsrc_t r2 = r1;
    if constexpr (NRES >= 2)
      r2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.res2 + rowb * p.r2cs + p.r2co), (short)0,
                                             0x7fff0000, 0x00020000);
    const bool full = full_tile(ti);
    const int px = wave * RW * p.Wo + ti.ox0 + col, n = ti.n0 + hi * 4;
    // offsets computed unconditionally, then selected: a select whose
    // offset needs a multiply became a branch with a load on each side,
    // issuing two counted loads on a wave whose lanes diverge
    // (scripts/check_xconv_vmcnt.py)
    const int rows_ok = p.Ho - ti.oy0 - wave * RW;   // wave-uniform
    const bool lane_ok = ti.ox0 + col < p.Wo;
    const int o1b = (px * p.rcs + n) * 4, r1row = p.Wo * p.rcs * 4;
    const int o2b = (px * p.r2cs + n) * 4, r2row = p.Wo * p.r2cs * 4;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bool ok = full | ((r < rows_ok) & lane_ok & (n + j * 16 < p.cout));
        const int o1 = ok ? o1b + r * r1row + j * 64 : 0x7ffffff0;
        if constexpr (NRES >= 1)
          rv1[r][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r1, o1, 0, 0));
        if constexpr (NRES >= 2) {
          const int o2 = ok ? o2b + r * r2row + j * 64 : 0x7ffffff0;
          rv2[r][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r2, o2, 0, 0));
        }
      }
  };
  // out = scale * (res2 + (res + act((am + 2^-11 ac) + bias))), sconv's order
  // (act: none, or leaky ReLU as max(v, slope v) for 0 <= slope <= 1)
  auto epilogue = [&](const TI &ti) {
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        p.y + (int64_t)ti.oy0 * p.Wo * p.ycs + p.yco, (short)0, 0x7fff0000, 0x00020000);
    const bool full = full_tile(ti);
    const int px = wave * RW * p.Wo + ti.ox0 + col, n = ti.n0 + hi * 4;
    // bias (and scale) of the lane's channels, read past the compiler's wait
    // insertion (lds_read16: a plain read here waited for the stage's newest
    // weight DMA)
    f32x4 bb[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bb[j] = lds_read16(Lc + (n + j * 16 < p.cout ? n + j * 16 : 0));
    constexpr int NSC = SHUF ? (NT % 4 == 0 ? NT / 4 : NT) : NT;
    f32x4 sc[NSC];
#pragma unroll
    for (int k = 0; k < NSC; ++k) {
      int cb;
      if constexpr (!SHUF) cb = n + k * 16 < p.cout ? n + k * 16 : 0;
      else if constexpr (NT % 4 == 0) cb = (ti.n0 >> 2) + 16 * k + 4 * hi;
      else cb = (ti.n0 >> 2) + 4 * k;
      sc[k] = lds_read16(Lc + p.cout + cb);
    }
    lds_wait4(bb);
    lds_wait4(sc);
    f32x4 v[RW][NT];
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        v[r][j][0] = (am[r][j][0] + ac[r][j][0] * kLoInv) + bb[j][0];
        v[r][j][1] = (am[r][j][1] + ac[r][j][1] * kLoInv) + bb[j][1];
        v[r][j][2] = (am[r][j][2] + ac[r][j][2] * kLoInv) + bb[j][2];
        v[r][j][3] = (am[r][j][3] + ac[r][j][3] * kLoInv) + bb[j][3];
      }
    if (p.act == DCVC_ACT_LRELU) {
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[r][j][e] = lrelu_in(v[r][j][e], p.slope);
    }
    if constexpr (SHUF) {
      // pixel shuffle (r = 2): conv channel 4 c + 2 dy + dx of pixel (oy, ox)
      // is output channel c of pixel (2 oy + dy, 2 ox + dx).  Lane row hi
      // holds conv channels n0 + 16 j + 4 hi + e (e = 2 dy + dx): a 4 x 4
      // transpose across the rows (v_permlane32_swap, then v_permlane16_swap)
      // gives row hi the 4 consecutive output channels (n0 + 16 j) / 4 + e of
      // sub-pixel hi; then the output-channel scale
      const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
          p.y + (int64_t)(2 * ti.oy0) * (2 * p.Wo) * p.ycs + p.yco, (short)0, 0x7fff0000, 0x00020000);
      // store offsets from per-lane bases and uniform steps, selected (no
      // branch, see load_res): output row 2 (wave RW + r) + dy, column
      // 2 (ox0 + col) + dx
      const int srow = 2 * p.Wo * p.ycs * 4, scol = p.ycs * 4;
      const int sbase = ((2 * wave * RW * 2 * p.Wo + 2 * (ti.ox0 + col)) * p.ycs + (ti.n0 >> 2)) * 4;
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        uint32_t sh[4][4];   // a group of four j (NT % 4 == 0)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          // (__float_as_uint: hipcc's __builtin_bit_cast of a vector element
          // reads element 0 whatever the index)
          uint32_t x0 = __float_as_uint(v[r][j][0]), x1 = __float_as_uint(v[r][j][1]);
          uint32_t x2 = __float_as_uint(v[r][j][2]), x3 = __float_as_uint(v[r][j][3]);
          xpose4(x0, x1, x2, x3);
          const bool okp = (ti.oy0 + wave * RW + r < p.Ho) & (ti.ox0 + col < p.Wo);
          if constexpr (NT % 4 == 0) {
            // groups of four j: a second transpose, across (row, j), gives
            // row hi the output channels (n0 + 64 g) / 4 + 4 hi .. + 3 of
            // every sub-pixel, so the 4 rows store 64 contiguous bytes of one
            // output pixel per instruction (not 16 bytes of 4 pixels)
            const int g = j >> 2, k = j & 3;
            sh[k][0] = x0;
            sh[k][1] = x1;
            sh[k][2] = x2;
            sh[k][3] = x3;
            if (k == 3) {
#pragma unroll
              for (int e = 0; e < 4; ++e) xpose4(sh[0][e], sh[1][e], sh[2][e], sh[3][e]);
              const bool ok = okp & (ti.n0 + 64 * g + 16 * hi < p.cout);   // (row hi: conv block j = 4 g + hi)
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                f32x4 o;
                o[0] = __uint_as_float(sh[s][0]) * sc[g][0];
                o[1] = __uint_as_float(sh[s][1]) * sc[g][1];
                o[2] = __uint_as_float(sh[s][2]) * sc[g][2];
                o[3] = __uint_as_float(sh[s][3]) * sc[g][3];
                // pixel (ry0 + (s >> 1), cx0 + (s & 1)), channels (n0 >> 2) + 16 g + 4 hi ..
                int off = ok ? sbase + (2 * r + (s >> 1)) * srow + (s & 1) * scol + (16 * g + 4 * hi) * 4
                             : 0x7ffffff0;
                opaque_v(off);   // (one store: hipcc otherwise duplicated it into both sides of a branch)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), ys, off, 0, 0);
              }
            }
          } else {
            f32x4 o;
            o[0] = __uint_as_float(x0) * sc[j][0];
            o[1] = __uint_as_float(x1) * sc[j][1];
            o[2] = __uint_as_float(x2) * sc[j][2];
            o[3] = __uint_as_float(x3) * sc[j][3];
            // pixel (ry0 + (hi >> 1), cx0 + (hi & 1)), channels (n0 >> 2) + 4 j ..
            const bool ok = okp & (ti.n0 + 16 * j < p.cout);
            int off = ok ? sbase + (2 * r + (hi >> 1)) * srow + (hi & 1) * scol + 16 * j : 0x7ffffff0;
            opaque_v(off);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), ys, off, 0, 0);
          }
        }
      }
      return;
    }
    if constexpr (NRES >= 1) {
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[r][j][e] = rv1[r][j][e] + v[r][j][e];
    }
    if constexpr (NRES >= 2) {
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[r][j][e] = rv2[r][j][e] + v[r][j][e];
    }
    if (p.scale) {
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          v[r][j][0] *= sc[j][0];
          v[r][j][1] *= sc[j][1];
          v[r][j][2] *= sc[j][2];
          v[r][j][3] *= sc[j][3];
        }
    }
    // store offsets computed unconditionally, then selected (an offset past
    // the buffer for pieces outside the output): no per-piece branches
    const int rows_ok = p.Ho - ti.oy0 - wave * RW;                 // wave-uniform
    const bool lane_ok = ti.ox0 + col < p.Wo;
    const int o0 = (px * p.ycs + n) * 4, orow = p.Wo * p.ycs * 4;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bool ok = full | ((r < rows_ok) & lane_ok & (n + j * 16 < p.cout));
        const int o = ok ? o0 + r * orow + j * 64 : 0x7ffffff0;
        if (!(XDBG & 128)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v[r][j]), yr, o, 0, 0);
      }
  };

  // ---- prologue: weights of stages 0 .. AH - 1, the first chunk's image
  const int G0 = GR;
  {
    const TI t0 = tile_of(g);
    int dv0[DPW];
    dma_lanes(t0.n0, dv0);
    sfor<G::AH>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      dma_w(t0.n0, dv0, std::integral_constant<int, k>{}, k);
    });
    load_img(t0, std::integral_constant<int, 0>{});
  }
  publish(0, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},
          std::integral_constant<int, PPF>{});   // (waits for its own loads, so for every DMA before them)
  wait_vm_lgkm();
  __syncthreads();
  read_a(std::integral_constant<int, 0>{}, 0);
  read_b(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, 0);

#ifdef XCONV_DBG
  unsigned stampv = 0;   // lane 2 s (+1) of one VGPR per stage stamp
#endif
  int kw = 0;   // weight slot of the current stage (stage counter mod NSW)
  int q = 0;    // image buffer of the current chunk (chunk counter mod 2)
  TI tcur = tile_of(g);
  for (int t = g; t < p.ntiles; t += G0) {
    // this tile and the next (prefetch target; itself when last)
    TI tc = tcur, tx = t + G0 < p.ntiles ? tile_next(tcur) : tcur;
    // computed once per tile: opaque, so the compiler keeps (or spills) them
    // instead of redoing tile_of's divisions in every stage that reads them
    opaque_s(tc.n0), opaque_s(tc.oy0), opaque_s(tc.ox0);
    opaque_s(tx.n0), opaque_s(tx.oy0), opaque_s(tx.ox0);
    // the per-lane LDS / DMA offsets are opaque to the compiler here, so it
    // computes each stage's addresses inside the stage (an add or two) instead
    // of hoisting dozens of them out of the tile loop into live registers
    opaque_v(aoff);
#pragma unroll
    for (int dx = 0; dx < KS; ++dx) opaque_v(bo1[dx]), opaque_v(bo2[dx]);
#pragma unroll
    for (int d = 0; d < DPW; ++d) opaque_v(dlane[d]), opaque_v(drow[d]);
    opaque_s(wcb);
    opaque_s(wrb);
    int dvc[DPW], dvx[DPW];
    dma_lanes(tc.n0, dvc);
    dma_lanes(tx.n0, dvx);
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        am[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ac[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    sfor<NST>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      // register set of stage s; with an odd stage count the last stage
      // reads the next tile's stage-0 operands into set 0 after its MFMAs
      constexpr int S = s & 1;
      constexpr bool late = (NST & 1) && s == NST - 1;
      constexpr int c = st_chunk<KT, CH>(s), rr = st_row<KT, CH>(s);
      constexpr int rows = c == CH - 1 ? ROWSL : KT;
      // stage s: its weights (slot kw) and image (buffer q) are visible, its
      // operands are in register set S (read during the previous stage)
      constexpr int AH = G::AH, NSW = G::NSW;
      // the ring slot and the image buffer of this stage: compile-time when
      // the ring depth divides the stage count and a tile has an even number
      // of chunks (the tile loop then returns both counters to 0)
      const int kw_ = G::RING_STATIC ? s % NSW : kw;
      const int q_ = CH % 2 == 0 ? (c & 1) : q;
      // per-stage opacity of the lane offsets: an address of this stage is
      // computed in it, never shared (CSE) with an equal one of a later stage
      // of the tile (the same tap of another chunk in the same image buffer,
      // the same ring slot), which would keep it live in between
      opaque_v(aoff);
#pragma unroll
      for (int dx = 0; dx < KS; ++dx) opaque_v(bo1[dx]), opaque_v(bo2[dx]);
      const int wsa = kw_ + AH >= NSW ? kw_ + AH - NSW : kw_ + AH;
      // 1-3: the stage's vector-memory work, in this order (vmcnt counts it):
      // 1. weights of stage s + AH (this tile or the next) into slot kw + AH;
      // 2. the next chunk's image pieces (first stage of a chunk);
      // 3. the tile's residuals.  With two operand sets it is issued after the
      // stage's first MFMA pass, so its scalar work and DMA issue overlap the
      // other wave's MFMAs instead of holding both waves of a SIMD at the
      // stage's start
      auto issue_mem = [&]() {
        if (!(XDBG & 8)) {
          if constexpr (s + AH < NST) dma_w(tc.n0, dvc, std::integral_constant<int, (s + AH) % NST>{}, wsa);
          else dma_w(tx.n0, dvx, std::integral_constant<int, (s + AH) % NST>{}, wsa);
        }
        if constexpr (rr == 0) {
          if constexpr (c + 1 < CH) load_img(tc, std::integral_constant<int, (c + 1 < CH ? c + 1 : 0)>{});
          else load_img(tx, std::integral_constant<int, 0>{});
        }
        if constexpr (s == 0) load_res(tc);
      };
      // stages that publish an image piece or run the epilogue issue their
      // weight DMA after that work (G::DMA_LATE)
      constexpr bool dlate = G::DMA_LATE && (s == NST - 1 || G::publishes(s));
      constexpr bool SPLITMF = DBA && !late;
      if constexpr (!SPLITMF && !dlate) issue_mem();
      // 4. operands of stage s + 1 into the other register set (the next
      // stage's weights landed and were published one barrier ago)
      const int ws1 = kw_ + 1 >= NSW ? 0 : kw_ + 1;
      constexpr int s1 = s + 1 < NST ? s + 1 : 0;
      constexpr int c1 = st_chunk<KT, CH>(s1);
      const int ib1 = (s + 1 < NST ? (c1 == c ? q_ : q_ ^ 1) : q_ ^ 1);
      if constexpr (!late) {
        if constexpr (DBA)
          if (!(XDBG & 1)) read_a(std::integral_constant<int, S ^ 1>{}, ws1);
        if (!(XDBG & 32)) read_b(std::integral_constant<int, S ^ 1>{}, std::integral_constant<int, s1>{}, ib1);
      }
      // 5. MFMAs of stage s.  With two operand sets, the next stage's reads
      // above are interleaved one per MFMA from the stage's first MFMA on
      // (the MFMAs read the other set): no MFMA waits behind the stage's
      // scalar work and reads, and no read is left to the stage's end (where
      // the scheduler would sink them to reuse this stage's registers, and
      // expose their latency).  With one set the reads stay ahead of them
      if constexpr (!SPLITMF) {
        sched_fence();
        if (!(XDBG & 1)) mfmas(std::integral_constant<int, S>{}, ws1, std::integral_constant<int, 0>{});
      } else {
        // the am pass with the reads interleaved (one or two per MFMA), then
        // the memory work, then the two ac passes
        if (!(XDBG & 1)) mfmas(std::integral_constant<int, S>{}, ws1, std::integral_constant<int, 1>{});
#ifdef __HIP_DEVICE_COMPILE__
        constexpr int NMA = RW * NT, NRD = 2 * NT + 2 * RW;
        sfor<NMA>([&](auto k_) {
          constexpr int k = decltype(k_)::value;
          constexpr int nr = (k + 1) * NRD / NMA - k * NRD / NMA;
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          // one MFMA
          if constexpr (nr > 0) __builtin_amdgcn_sched_group_barrier(0x100, nr, 0);   // LDS reads
        });
#endif
        sched_fence();
        if constexpr (!dlate) issue_mem();
        sched_fence();
        if (!(XDBG & 1)) mfmas(std::integral_constant<int, S>{}, ws1, std::integral_constant<int, 2>{});
      }
      if constexpr (late) {
        if constexpr (DBA) read_a(std::integral_constant<int, 0>{}, ws1);
        read_b(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, ib1);
      }
      // 6. the next chunk's image into the other buffer, visible at the
      // chunk's last stage, whose operand reads need it: one piece per stage
      // up to the second-to-last stage where the chunk has room for that
      // (the pieces loaded at its first stage), else all at the second-to-last
      {
        constexpr int cn = c + 1 < CH ? c + 1 : 0;
        constexpr int PPn = cn == CH - 1 ? PPL : PPF;
        // (the last piece at a stage that ends with a barrier before the
        // chunk's last stage)
        constexpr int s0c = s - rr;   // the chunk's first stage
        constexpr int pend = G::bar(s0c + rows - 2) ? rows - 2 : rows - 3;
        constexpr int w0 = pend + 1 - PPn;   // the first publishing stage
        using CN = std::integral_constant<int, cn>;
        if constexpr (w0 >= 1) {
          if constexpr (rr >= w0 && rr <= pend)
            if (!(XDBG & 16))
              publish(q_ ^ 1, CN{}, std::integral_constant<int, rr - w0>{}, std::integral_constant<int, rr - w0 + 1>{});
        } else if constexpr (rr == pend) {
          if (!(XDBG & 16)) publish(q_ ^ 1, CN{}, std::integral_constant<int, 0>{}, std::integral_constant<int, PPn>{});
        }
      }
      // 7. epilogue
      if constexpr (s == NST - 1) epilogue(tc);
      if constexpr (dlate) {
        sched_fence();
        issue_mem();
      }
      // end of stage: stage s + 2's weights must have landed, every
      // vector-memory operation issued after their DMA may stay in flight
      // (fenced: the scheduler would hoist the wait above the MFMAs, right
      // behind the operand reads it would then wait for)
      sched_fence();
#ifdef XCONV_DBG
      if (2 * s + 1 < 64 && t == g + G0)
        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(stampv) : "s"((unsigned)__builtin_amdgcn_s_memtime()), "i"(2 * s));
#endif
      if constexpr (G::bar(s)) {
        constexpr int N = G::wait_n(s);
        static_assert(N < 64, "too many vector-memory operations in flight for vmcnt");
        if (XDBG & 4) wait_lgkm();
        else wait_vm_n_lgkm<N>();
      }
      // nothing of one stage is scheduled into another: the MFMAs of a stage
      // stay between its operand reads and its barrier, so operand and
      // accumulator registers live one stage long
      sched_fence();
      if constexpr (G::bar(s))
        if (!(XDBG & 2)) raw_barrier();
      sched_fence();
#ifdef XCONV_DBG
      if (2 * s + 1 < 64 && t == g + G0)
        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(stampv) : "s"((unsigned)__builtin_amdgcn_s_memtime()), "i"(2 * s + 1));
#endif
      if constexpr (rr == rows - 1) q ^= 1;
      kw = kw + 1 >= NSW ? 0 : kw + 1;
    });
    tcur = tx;
  }
  wait_vm_lgkm();   // no LDS-DMA left in flight when the workgroup exits
#ifdef XCONV_DBG
  if (blockIdx.x == 0 && wave < 8) g_xstamps[wave * 64 + lane] = stampv;
#endif
}

// The vector-memory schedule the kernel's exact vmcnt waits assume, per
// stage: its vector-memory instructions in issue order (D weight LDS-DMA,
// I image load, R residual load, S output store) and, at a barrier stage,
// the wait's count.  scripts/check_xconv_vmcnt.py compares it with the
// instructions hipcc emitted for every instantiation (make runs it): a load
// the compiler deleted, merged or moved ahead of a DMA, or a spill's scratch
// access, would make a wait pass with its DMA in flight (the round-5 ring
// race).  Line per stage: "<ops> <wait or -1>".
template <int CIN, int BN, int RW, int NW, int NRES, int KS>
int sched_dump(char *buf, int cap) {
  typedef XG<CIN, BN, RW, NW, NRES, KS> G;
  std::string out = "nst " + std::to_string(G::NST) + " nsw " + std::to_string(G::NSW) + "\n";
  for (int x = 0; x < G::NST; ++x) {
    const bool dlate = G::DMA_LATE && (x == G::NST - 1 || G::publishes(x));
    std::string ops;
    if (!dlate) ops.append(G::DPW, 'D');
    ops.append(G::img_ops(x), 'I');
    if (x == 0) ops.append(G::NTILE, 'R');
    if (x == G::NST - 1) ops.append(G::NSTORE, 'S');
    if (dlate) ops.append(G::DPW, 'D');
    out += (ops.empty() ? "-" : ops) + " " + std::to_string(G::bar(x) ? G::wait_n(x) : -1) + "\n";
  }
  if ((int)out.size() + 1 > cap) return DCVC_HIP_EINVAL;
  std::memcpy(buf, out.c_str(), out.size() + 1);
  return DCVC_HIP_OK;
}

// every instantiation launch<> uses registers its sched_dump at load time
struct SchedEntry {
  int cin, bn, rw, nw, nres, ks;
  int (*dump)(char *, int);
};
std::vector<SchedEntry> &sched_registry() {
  static std::vector<SchedEntry> r;
  return r;
}
template <int CIN, int BN, int RW, int NW, int NRES, int KS>
struct SchedReg {
  SchedReg() { sched_registry().push_back({CIN, BN, RW, NW, NRES, KS, &sched_dump<CIN, BN, RW, NW, NRES, KS>}); }
  static SchedReg inst;
};
template <int CIN, int BN, int RW, int NW, int NRES, int KS>
SchedReg<CIN, BN, RW, NW, NRES, KS> SchedReg<CIN, BN, RW, NW, NRES, KS>::inst;

int g_cus = 0;
int g_enable = 1;   // dcvc_set_option("xconv", 0): route every split conv to sconv.hip
// dcvc_set_option("xconv_dbg", bits) in builds with -DXCONV_DBG (make
// XCONV_DBG=1): timing ablations, wrong results: 1 no MFMAs,
// 2 no stage barrier, 4 no weight-DMA wait, 8 no weight DMA, 16 no image
// publish, 32 no image-operand reads, 64 no image loads, 128 no residual loads
// and output stores
int g_dbg = 0;
int g_rw1 = 1;

template <int CIN, int BN, int RW, int NW, int NRES, bool SHUF = false, int KS = 3>
int launch(XP p, hipStream_t st) {
  typedef XG<CIN, BN, RW, NW, NRES, KS> G;
  (void)&SchedReg<CIN, BN, RW, NW, NRES, KS>::inst;   // (scripts/check_xconv_vmcnt.py)
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
  int64_t grid = (int64_t)g_cus * G::WPC;
  if (grid > nt) grid = nt;
  auto kern = xconv3_kernel<CIN, BN, RW, NW, NRES, SHUF, KS>;
  // (the name as rocprofv3 prints the instantiation: scripts/pmc_summary.py keys on it)
  dcvc_note_kernel("xconv3_kernel<%d, %d, %d, %d, %d, %s, %d>@%lld", CIN, BN, RW, NW, NRES, SHUF ? "true" : "false", KS,
                   (long long)grid * NW * 64);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NW * 64), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// the residual count picks the instantiation
template <int CIN, int BN, int RW, int NW, bool RES_OK = true>
int pick_res(XP p, hipStream_t st) {
  if constexpr (RES_OK) {
    if (p.has_res2) return launch<CIN, BN, RW, NW, 2>(p, st);
    if (p.has_res) return launch<CIN, BN, RW, NW, 1>(p, st);
  } else if (p.has_res) {
    return DCVC_HIP_EUNSUPPORTED;
  }
  return launch<CIN, BN, RW, NW, 0>(p, st);
}

// n-block: the whole cout when it is 32 or 48 channels, else 64-, 48- or
// 32-channel blocks.  64-channel blocks with residuals would spill
// (scripts/isa_probe.sh; a spill's scratch traffic would break the per-stage
// vmcnt accounting), so those layers take 48- or 32-channel blocks.  8 waves
// of 2 rows each (two waves per SIMD): 4 waves of 4 rows (one wave per SIMD,
// 512 registers) measured 3-8 % slower (profiles/r04_xconv_ab.jsonl)
// RES_OK false: no residual instantiations (80 input channels: they spill,
// and no 80-channel layer of the codecs takes a residual)
template <int CIN, bool RES_OK = true>
int pick_bn(XP p, hipStream_t st) {
  if (p.shuffle) {   // no residuals, cout % 16 == 0 (dcvc_internal_xconv)
    if (p.cout % 64 == 0) return launch<CIN, 64, 2, 8, 0, true>(p, st);
    if (p.cout % 48 == 0) return launch<CIN, 48, 2, 8, 0, true>(p, st);
    return launch<CIN, 32, 2, 8, 0, true>(p, st);
  }
  if constexpr (CIN == 64) {
    // residual layers of 64-channel multiples: 8-row tiles (one row per wave)
    // of 64-channel blocks instead of 16-row tiles of 32-channel blocks, which
    // load and split the input once per block: 64 -> 64 + residual at 544 x
    // 960 4-6 %, 64 -> 128 3 % faster; 128 -> 128 at 272 x 480 1 % slower, so
    // 64 input channels only (profiles/r05u_xconv_rw1_ab.jsonl; "xconv_rw1" 0: off)
    if (g_rw1 && p.has_res && p.cout % 64 == 0) return pick_res<CIN, 64, 1, 8, RES_OK>(p, st);
  }
  if (p.cout == 32 || p.cout == 48) return p.cout == 32 ? pick_res<CIN, 32, 2, 8, RES_OK>(p, st) : pick_res<CIN, 48, 2, 8, RES_OK>(p, st);
  if (p.cout % 64 == 0 && !p.has_res) return launch<CIN, 64, 2, 8, 0>(p, st);
  if (p.cout % 48 == 0) return pick_res<CIN, 48, 2, 8, RES_OK>(p, st);
  if (p.cout % 32 == 0) return pick_res<CIN, 32, 2, 8, RES_OK>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

}  // namespace

// scripts/check_xconv_vmcnt.py: the schedule of xconv3_kernel<cin, bn, rw, nw,
// nres, *, ks> (above), host-side, no GPU needed
// (index i of the registered instantiations: its parameters into p[6] and its
// schedule into buf; DCVC_HIP_EINVAL past the last)
extern "C" int dcvc_internal_xconv_schedule(int i, int *prm, char *buf, int cap) {
  const auto &r = sched_registry();
  if (i < 0 || i >= (int)r.size()) return DCVC_HIP_EINVAL;
  const SchedEntry &e = r[i];
  const int v[6] = {e.cin, e.bn, e.rw, e.nw, e.nres, e.ks};
  std::memcpy(prm, v, sizeof v);
  return e.dump(buf, cap);
}

extern "C" void dcvc_internal_xconv_enable(int v) { g_enable = v; }

// the stamps of the last launch (ablation builds; DCVC_HIP_EUNSUPPORTED otherwise)
extern "C" int dcvc_internal_xconv_stamps(unsigned *host) {
#ifdef XCONV_DBG
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xstamps), sizeof(unsigned) * 8 * 64) == hipSuccess
             ? DCVC_HIP_OK : DCVC_HIP_ELAUNCH;
#else
  (void)host;
  return DCVC_HIP_EUNSUPPORTED;
#endif
}
extern "C" void dcvc_internal_sconv_dbg(int v);
extern "C" void dcvc_internal_wconv_dbg(int v);
extern "C" void dcvc_internal_sconv_rw(int v);

// the split-precision kernels' A/B and timing-ablation options (dcvc_set_option)
extern "C" int dcvc_internal_set_option_split(const char *name, int value) {
  if (std::strcmp(name, "sconv_dbg") == 0) dcvc_internal_sconv_dbg(value);
  else if (std::strcmp(name, "sconv_rw") == 0) dcvc_internal_sconv_rw(value);
  else if (std::strcmp(name, "xconv_dbg") == 0) g_dbg = value;
  else if (std::strcmp(name, "xconv_rw1") == 0) g_rw1 = value;
  else if (std::strcmp(name, "wconv_dbg") == 0) dcvc_internal_wconv_dbg(value);
  else return DCVC_HIP_EINVAL;
  return DCVC_HIP_OK;
}

// 3x3 stride-1 f16x3 convolutions with fp32 views (dcvc_internal_sconv calls
// this first).  DCVC_HIP_EUNSUPPORTED: a shape / view without an
// instantiation, left to sconv.hip.
extern "C" int dcvc_internal_xconv(const dcvc_conv_args *a, void *stream) {
  if (!g_enable) return DCVC_HIP_EUNSUPPORTED;
  // 3x3 (pad 1) and SpyNet's 7x7 (pad 3), stride 1
  if (a->kh != a->kw || a->stride != 1 || !((a->kh == 3 && a->pad == 1) || (a->kh == 7 && a->pad == 3)))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->kh == 7 && (a->shuffle || a->res.ptr)) return DCVC_HIP_EUNSUPPORTED;
  // pixel shuffle: whole 16-channel groups (4 output channels per lane after
  // the epilogue's transpose), no residuals
  if (a->shuffle && (a->cout % 16 || a->res.ptr || a->res2.ptr)) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && a->in_op != DCVC_IN_LRELU) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  // leaky ReLUs are computed as max(v, slope v): exact for 0 <= slope <= 1
  if (a->act != DCVC_ACT_NONE && !(a->act == DCVC_ACT_LRELU && a->slope >= 0.f && a->slope <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op == DCVC_IN_LRELU && !(a->in_slope >= 0.f && a->in_slope <= 1.f)) return DCVC_HIP_EUNSUPPORTED;
  XP p{};
  p.ovf = dcvc_internal_split_flag();
  p.dbg = g_dbg;
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
  p.shuffle = a->shuffle ? 1 : 0;
  if (a->y.W != (a->shuffle ? 2 : 1) * p.Wo || a->y.H != (a->shuffle ? 2 : 1) * p.Ho) return DCVC_HIP_EUNSUPPORTED;
  // 16-byte pieces everywhere: input slots of 8 channels, output / residual pieces of 4
  bool ok = a->cin % 8 == 0 && p.xcs % 4 == 0 && p.xco % 4 == 0 && (uintptr_t)p.x % 16 == 0;
  ok = ok && a->cout % 4 == 0 && p.ycs % 4 == 0 && p.yco % 4 == 0 && (uintptr_t)p.y % 16 == 0;
  if (a->res.ptr) {
    p.res = reinterpret_cast<const float *>(a->res.ptr);
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
    p.has_res = 1;
    ok = ok && a->res.dtype == DCVC_F32 && p.rcs % 4 == 0 && p.rco % 4 == 0 && (uintptr_t)p.res % 16 == 0;
  }
  if (a->res2.ptr) {
    p.res2 = reinterpret_cast<const float *>(a->res2.ptr);
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
    p.has_res2 = 1;
    ok = ok && a->res2.dtype == DCVC_F32 && p.r2cs % 4 == 0 && p.r2co % 4 == 0 && (uintptr_t)p.res2 % 16 == 0;
  }
  if (p.has_res2 && !p.has_res) return DCVC_HIP_EUNSUPPORTED;
  if (!ok) return DCVC_HIP_EUNSUPPORTED;
  // per-tile buffer offsets stay below 2^31 bytes: output / residual rows of
  // a tile (16 rows; with the pixel shuffle 32 rows of 2 Wo pixels) and the
  // input halo rows (16 + 6 at most)
  if ((int64_t)16 * p.Wo * std::max(p.ycs, std::max(p.rcs, p.r2cs)) * 4 >= ((int64_t)1 << 30))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->shuffle && (int64_t)32 * 2 * p.Wo * p.ycs * 4 >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  // (the halo rows a tile reads fit the input record, clamped to 0x7fff0000 bytes)
  if ((int64_t)(16 + a->kh) * p.W * p.xcs * 4 >= 0x7fff0000) return DCVC_HIP_EUNSUPPORTED;
  const int nch = (a->cin + 31) / 32;
  const int vc = a->cin - 32 * (nch - 1);
  const int tpkl = vc <= 8 ? 4 : vc <= 16 ? 2 : 1;
  const int kt = a->kh * a->kw;
  p.wchunk = (int64_t)2 * kt * a->cout * 32;
  {
    const int rl = (kt + tpkl - 1) / tpkl;
    const int64_t wb = ((int64_t)(nch - 1) * p.wchunk + (int64_t)2 * rl * a->cout * 32) * 2;
    if (wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
    p.wbytes = (int)wb;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#ifdef XCONV_ISA_PROBE
  // (ISA inspection builds, scripts/isa_probe.sh: one channel count, n-block and residual count)
  return launch<XCONV_ISA_PROBE, XCONV_PROBE_BN, XCONV_PROBE_RW, 8 / (XCONV_PROBE_RW / 2), XCONV_PROBE_NRES, false,
                XCONV_PROBE_KS>(p, st);
#else
  if (a->kh == 7) {
    // SpyNet's 7x7 layers (video_net.py:79-100): the halo image of a 22 x 22
    // pixel tile leaves LDS for a weight ring of 16- or 32-channel blocks
    switch (a->cin) {
      case 8: return a->cout % 32 == 0 ? launch<8, 32, 2, 8, 0, false, 7>(p, st) : DCVC_HIP_EUNSUPPORTED;
      case 16: return a->cout == 16 ? launch<16, 16, 2, 8, 0, false, 7>(p, st)
                                    : a->cout % 32 == 0 ? launch<16, 32, 2, 8, 0, false, 7>(p, st) : DCVC_HIP_EUNSUPPORTED;
      case 32: return a->cout == 16 ? launch<32, 16, 2, 8, 0, false, 7>(p, st)
                                    : a->cout % 32 == 0 ? launch<32, 32, 2, 8, 0, false, 7>(p, st) : DCVC_HIP_EUNSUPPORTED;
      case 64: return a->cout == 16 ? launch<64, 16, 2, 8, 0, false, 7>(p, st)
                                    : a->cout % 32 == 0 ? launch<64, 32, 2, 8, 0, false, 7>(p, st) : DCVC_HIP_EUNSUPPORTED;
      default: return DCVC_HIP_EUNSUPPORTED;
    }
  }
  switch (a->cin) {
    case 32: return pick_bn<32>(p, st);
    case 48: return pick_bn<48>(p, st);
    case 64: return pick_bn<64>(p, st);
    case 80: return pick_bn<80, false>(p, st);
    case 96: return pick_bn<96>(p, st);
    case 128: return pick_bn<128>(p, st);
    case 192: return pick_bn<192>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
#endif
}
