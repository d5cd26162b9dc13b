// Split-fp16 ("f16x3") implicit-GEMM convolution for fp32 NHWC feature maps:
// the arithmetic of Precision.split(), the precision the bench runs in.
//
// Why: the reference computes every conv in fp32, and its symbols / CDF
// indexes are discontinuous functions of those fp32 values, so a bf16 conv
// (8-bit operands) moves far more symbols than rounding ties explain, while
// fp32 MFMA tops out at 157 TF on gfx950.  Here each fp32 operand a is split
// into two fp16 values, a = hi + lo * 2^-11 (hi = a rounded toward zero to
// fp16; lo = the remainder scaled by 2^11, so lo lies in the same range as a
// and stays a normal fp16 number wherever a does), and
// every product is taken as
//     x * w  ~  xh * wh  +  2^-11 * (xh * wl + xl * wh)
// on v_mfma_f32_16x16x32_f16 with fp32 accumulation: three MFMAs per product
// (the xl * wl term is 2^-22 of it and is dropped), two accumulators (main and
// correction) combined in the epilogue.  Operand error is ~2^-21 relative,
// within a small factor of fp32 rounding, at 2.5 PF / 3 = 833 TF of effective
// fp32 rate.  scripts/split_precision_sim.py measured the choice on the CPU
// against the strict parity bar before this kernel existed:
// bf16 x 3 misses ties by up to 2.5e-3, fp16 x 3 stays at fp32 reordering
// level.
//
// Kernel structure (one 256-thread workgroup per CU, one wave per SIMD, so a
// wave has the whole 512-register file: accumulators live in AGPRs;
// persistent over tiles):
//   * output tile = TH = 4 * RW rows x 16 columns x BN channels; wave w owns
//     rows [w * RW, (w + 1) * RW) and all BN channels (NT = BN / 16 MFMA
//     n-tiles), i.e. RW x NT x 2 f32x4 accumulators.  Per tap a wave reads
//     2 (NT + RW) operand pieces from LDS for 3 NT RW MFMAs: the large RW = 4,
//     NT = 4 tile keeps the LDS below its 128 B/clk;
//   * the K dimension is walked in STAGES: one stage = one kernel row (KS
//     taps) of one 32-channel input chunk.  A chunk's input halo image is
//     split once when it is written to LDS (hi and lo images, 16-byte
//     XOR-swizzled slots), so all KS x KS taps reuse it; the weights of a
//     stage arrive by LDS-DMA (pre-swizzled source addresses) into one of two
//     buffers while the other stage's MFMAs run;
//   * chunks with 16 or 8 valid channels (Cin = 48, 80, 8, 16, 2, ...) pack 2
//     or 4 taps into one 32-deep MFMA K step (the weights are packed the same
//     way by dcvc_conv_pack_weights), so a 48-channel conv wastes no MFMA work;
//   * the next chunk's input pieces (also the next tile's first chunk) are
//     loaded into registers right after the current chunk's image is
//     published, so their latency hides behind a whole chunk of MFMAs;
//   * the epilogue (epilogue.h) combines the accumulators, adds bias, applies
//     the activation, residuals, scale and pixel shuffle in the reference's
//     order and stores fp32 whole lines per wave instruction.
#include "common.h"
#include "epilogue.h"
#include "split.h"

#include <utility>

namespace {

struct SP {
  const float *x;
  int H, W, xcs, xco;
  const uint16_t *w;     // split weights (dcvc_conv_pack_weights, DCVC_F16X3)
  const float *bias;
  void *y;
  int Ho, Wo, ycs, yco;  // conv output size (before shuffle)
  int cin, cout;
  int pad;
  int in_op;
  float in_slope;
  int act;
  float slope;
  int shuffle;
  const float *scale;
  const void *res;
  int rcs, rco;
  const void *res2;
  int r2cs, r2co;
  int Wout;
  int vec, vec_out;
  int direct;              // epilogue straight from the accumulators (no shuffle, 16-byte aligned pieces)
  int tiles_x, tiles_y, nblk, ntiles;
  int nchunks, tpk_last;   // taps per K step of the last chunk (1, 2 or 4)
  int64_t wchunk;          // halves of one full chunk's packed weights (hi + lo)
  int wbytes;              // bytes of the packed weights
  int dbg;                 // dcvc_set_option("sconv_dbg", mask): timing ablations, wrong results
                           // (1 no MFMA, 2 no image publish, 4 no image loads, 8 no epilogue)
  int *ovf;               // fp16 range guard (split.h SplitRange)
};

// RES = false: weights streamed one kernel row (KS taps) of one chunk per
// stage by LDS-DMA into two buffers; RES = true: every weight row of the
// workgroup's n-block resident in LDS for the whole launch (loaded once), one
// stage = one input chunk with all its taps (the LDS size then depends on cin
// and is passed at launch)
template <int KS, int S, int BN, int RW, int NW, bool RES = false>
struct SG {
  static constexpr int kNW = NW, kNT = NW * 64;
  static constexpr int TH = kNW * RW;
  static constexpr int NT = BN / 16;
  static constexpr int KT = KS * KS;
  static constexpr int RG = RES ? KT : KS;         // kernel rows (taps) per stage
  static constexpr int IH = (TH - 1) * S + KS;
  static constexpr int IW = 15 * S + KS;
  static constexpr int IWP = (IW + 3) & ~3;
  static constexpr int IMG = IH * IWP * 32;        // halves per image (hi or lo)
  static constexpr int WIMG = RG * BN * 32;        // halves per weight image (hi or lo)
  static constexpr int PPI = (IH * IW * 4 + kNT - 1) / kNT;   // image pieces per thread
  static constexpr int NDMA = 2 * RG * BN / 16;               // 1-KiB LDS-DMA pieces per stage
  static constexpr int DPW = (NDMA + kNW - 1) / kNW;          // ... per wave
  static constexpr int LD = BN + 4;
  static constexpr size_t TB = (size_t)TH * 16 * LD * 4;      // fp32 epilogue tile
  static constexpr size_t IB = (size_t)2 * IMG * 2;           // hi + lo image
  static constexpr size_t R0 = IB > TB ? IB : TB;             // image / epilogue region
  static constexpr size_t LC = R0;                            // bias | scale
  static constexpr size_t DUMMY = LC + (size_t)epi::consts_floats(BN) * 4;   // 16-byte sink
  static constexpr size_t WOFF = DUMMY + 16;                  // weights
  static constexpr size_t WB = RES ? 0 : (size_t)4 * WIMG * 2;  // streamed: two stage buffers x (hi, lo)
  static constexpr size_t LDS = WOFF + WB;                    // (+ the resident weights when RES)
  static constexpr size_t WROW = (size_t)BN * 32 * 2 * 2;     // resident bytes per weight row (hi + lo)
  static constexpr int NLV = PPI * 2 * (1 + 0);   // vector-memory instructions of one vec image prefetch
};

// rows of the packed weights of a chunk with tpk taps per K step
__device__ __forceinline__ int chunk_rows(int kt, int tpk) { return (kt + tpk - 1) / tpk; }

template <int KS, int S, int BN, int RW, int NW, bool GATE, bool RES>
__global__ void __launch_bounds__(NW * 64) sconv_kernel(SP p) {
  SplitRange rg(p.ovf);
  typedef SG<KS, S, BN, RW, NW, RES> G_;
  constexpr int kNW = NW, kNT = NW * 64;
  constexpr int TH = G_::TH, NT = G_::NT, KT = G_::KT, RG = G_::RG;
  constexpr int IH = G_::IH, IW = G_::IW, IWP = G_::IWP, IMG = G_::IMG, WIMG = G_::WIMG;
  constexpr int PPI = G_::PPI, NDMA = G_::NDMA, DPW = G_::DPW;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Lih = reinterpret_cast<uint16_t *>(smem);
  uint16_t *Lil = Lih + IMG;
  uint16_t *Lw = reinterpret_cast<uint16_t *>(smem + G_::WOFF);   // [buf][hi, lo][WIMG] | [hi, lo][wrows][BN][32]
  float *T = reinterpret_cast<float *>(smem);
  float *Lc = reinterpret_cast<float *>(smem + G_::LC);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  // consecutive tiles on one XCD (workgroups are dealt to XCDs round robin)
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);
  if (g >= p.ntiles) return;

  // stages of one tile: chunk c has chunk_rows(KT, tpk_c) rows, RG per stage
  const int spc_full = (KT + RG - 1) / RG;                  // stages per full chunk (KS; 1 when RES)
  const int spc_last = (chunk_rows(KT, p.tpk_last) + RG - 1) / RG;
  const int nstages = (p.nchunks - 1) * spc_full + spc_last;

  // image piece plan (constant): piece u = (halo pixel, 8-channel slot);
  // prel = its element offset from the tile's first halo pixel
  int ipix[PPI], iofs[PPI], prel[PPI];
#pragma unroll
  for (int u = 0; u < PPI; ++u) {
    const int it = tid + u * kNT;
    ipix[u] = -1;
    iofs[u] = 0;
    prel[u] = 0;
    if (it < IH * IW * 4) {
      const int slot = it & 3, pix = it >> 2;
      const int iy = pix / IW, ix = pix - iy * IW;
      ipix[u] = (iy << 16) | (ix << 2) | slot;
      iofs[u] = swzx(iy * IWP + ix, ix, slot);
      prel[u] = (iy * p.W + ix) * p.xcs + slot * 8;
    }
  }
  float pfi[PPI][8];
  float pfg[GATE ? PPI : 1][8];

  auto tile_of = [&](int t, int &oy0, int &ox0, int &n0) {
    const int nb = t % p.nblk;
    const int sp = t / p.nblk;
    n0 = nb * BN;
    oy0 = (sp / p.tiles_x) * TH;
    ox0 = (sp % p.tiles_x) * 16;
  };
  auto stage_of = [&](int s, int &c, int &r0, int &tpk) {
    if constexpr (RES) {
      c = s;
      r0 = 0;
    } else {
      c = s / spc_full;
      if (c > p.nchunks - 1) c = p.nchunks - 1;
      r0 = (s - c * spc_full) * RG;
    }
    tpk = c == p.nchunks - 1 ? p.tpk_last : 1;
  };
  // registers <- global: the input pieces of chunk c of tile t.  Buffer
  // loads through a descriptor based at the tile's first input row, every
  // load unconditional (an out-of-range offset reads zeros: halo outside the
  // image, channels past cin, pieces past the plan), so hipcc keeps them all
  // in flight instead of waiting per conditional load
  auto prefetch_img = [&](int t, int c) {
    int oy0, ox0, n0;
    tile_of(t, oy0, ox0, n0);
    const int iy0 = oy0 * S - p.pad, ix0 = ox0 * S - p.pad;
    const int rb = iy0 > 0 ? iy0 : 0;
    const int64_t eb = (int64_t)rb * p.W * p.xcs + p.xco + c * 32;     // element offset of the base
    int64_t nrec = ((int64_t)p.H * p.W * p.xcs - eb) * 4;
    if (nrec > 0x7fff0000) nrec = 0x7fff0000;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(p.x + eb), (short)0, (int)nrec, 0x00020000);
    const int cl = p.cin - c * 32;   // channels of this chunk left in the input
    const int toff = ((iy0 - rb) * p.W + ix0) * p.xcs;   // the tile's first halo pixel, from the base
#pragma unroll
    for (int u = 0; u < PPI; ++u) {
      const int q = ipix[u];
      const int gy = iy0 + (q >> 16), gx = ix0 + ((q >> 2) & 0x3fff);
      const int c0 = (q & 3) * 8;
      const bool in = q >= 0 && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
      const int off = toff + prel[u];   // elements from the base
      if (p.vec) {
        const int o = in && c0 < cl ? off * 4 : 0x7fffffe0;
        const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
        const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pfi[u][j] = a[j];
          pfi[u][4 + j] = b[j];
        }
        if constexpr (GATE) {
          const int og = in && c0 < cl ? (off + p.cin) * 4 : 0x7fffffe0;
          const f32x4 ga = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, og, 0, 0));
          const f32x4 gb = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, og + 16, 0, 0));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pfg[u][j] = ga[j];
            pfg[u][4 + j] = gb[j];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int o = in && c0 + j < cl ? (off + j) * 4 : 0x7ffffff0;
          pfi[u][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o, 0, 0));
          if constexpr (GATE) {
            const int og = in && c0 + j < cl ? (off + j + p.cin) * 4 : 0x7ffffff0;
            pfg[u][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, og, 0, 0));
          }
        }
      }
    }
  };
  // LDS image <- registers, split on the way (input transform first); pieces
  // past the plan write a dummy slot, so the stores need no branch
  uint16_t *const Ldummy = reinterpret_cast<uint16_t *>(smem + G_::DUMMY);
  // (ResBlock's leaky ReLU on the input, lrelu(x) = max(x, slope x) for
  // 0 <= slope <= 1, and the ConvFFN2 gate are applied before the split)
  auto publish_one = [&](int u, const float (&v)[8]) {
    u32x4_t h, l;
    rg.add8(v);
    split8(v, h, l);
    const bool ok = ipix[u] >= 0;
    *reinterpret_cast<u32x4_t *>(ok ? Lih + iofs[u] : Ldummy) = h;
    *reinterpret_cast<u32x4_t *>(ok ? Lil + iofs[u] : Ldummy) = l;
  };
  auto publish_img = [&]() {
    if constexpr (GATE) {
#pragma unroll
      for (int u = 0; u < PPI; ++u) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gv = pfg[u][j];
          v[j] = pfi[u][j] * (gv >= 0.f ? gv : gv * p.in_slope);
        }
        publish_one(u, v);
      }
    } else if (p.in_op == DCVC_IN_LRELU) {
#pragma unroll
      for (int u = 0; u < PPI; ++u) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = pfi[u][j] >= 0.f ? pfi[u][j] : pfi[u][j] * p.in_slope;
        publish_one(u, v);
      }
    } else {
#pragma unroll
      for (int u = 0; u < PPI; ++u) publish_one(u, pfi[u]);
    }
  };
  // LDS-DMA of weight rows [r0, r0 + RG) of the stage into buffer b: each
  // instruction moves 16 rows of 64 bytes; lane i writes the LDS bytes of
  // (row i / 4, physical slot i % 4), so it reads the logical slot that the
  // swizzle puts there (rows past the chunk or channels past cout: zeros)
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
  auto issue_w = [&](int t, int s, int b) {
    int oy0, ox0, n0, c, r0, tpk;
    tile_of(t, oy0, ox0, n0);
    stage_of(s, c, r0, tpk);
    const int rows = chunk_rows(KT, tpk);
    const int64_t cbase = (int64_t)c * p.wchunk;
    const int64_t lo_off = (int64_t)rows * p.cout * 32;
#pragma unroll
    for (int d = 0; d < DPW; ++d) {
      const int i = wave + kNW * d;
      if (i < NDMA) {
        const int hl = i >= NDMA / 2, k = hl ? i - NDMA / 2 : i;
        const int R = k * 16 + (lane >> 2);          // row of the weight image: r * BN + nn
        const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
        const int r = R / BN, n = n0 + R - r * BN;
        int voff = 0x7ffffff0;                       // out of range: zeros
        if (r0 + r < rows && n < p.cout)
          voff = (int)((cbase + (hl ? lo_off : 0) + ((int64_t)(r0 + r) * p.cout + n) * 32 + ls * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wr, (__attribute__((address_space(3))) void *)(Lw + (2 * b + hl) * WIMG + k * 512), 16, voff, 0, 0, 0);
      }
    }
  };

  // RES: every weight row of n-block n0 into LDS (once per launch): flattened
  // row R = (chunk row) * BN + nn, the chunk rows of all chunks in order
  const int wrows = (p.nchunks - 1) * KT + chunk_rows(KT, p.tpk_last);
  auto load_resident = [&](int n0) {
    const int nd = 2 * wrows * BN / 16;   // 1-KiB pieces (16 rows of 64 bytes)
    for (int i = wave; i < nd; i += kNW) {
      const int hl = i >= nd / 2, k = hl ? i - nd / 2 : i;
      const int R = k * 16 + (lane >> 2);
      const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
      const int cr = R / BN, nn = R - cr * BN;
      int c = cr / KT;
      if (c > p.nchunks - 1) c = p.nchunks - 1;
      const int r = cr - c * KT;
      const int rows = c == p.nchunks - 1 ? chunk_rows(KT, p.tpk_last) : KT;
      const int n = n0 + nn;
      int voff = 0x7ffffff0;
      if (n < p.cout)
        voff = (int)(((int64_t)c * p.wchunk + (hl ? (int64_t)rows * p.cout * 32 : 0) + ((int64_t)r * p.cout + n) * 32 +
                      ls * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (__attribute__((address_space(3))) void *)(Lw + (size_t)hl * wrows * BN * 32 + k * 512), 16, voff, 0, 0, 0);
    }
  };

  f32x4 am[RW][NT], ac[RW][NT];
  auto mfmas = [&](const f16x8 (&ah)[NT], const f16x8 (&al)[NT], const f16x8 (&bh)[RW], const f16x8 (&bl)[RW]) {
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        am[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j], bh[r], am[r][j], 0, 0, 0);
        ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[j], bl[r], ac[r][j], 0, 0, 0);
        ac[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[j], bh[r], ac[r][j], 0, 0, 0);
      }
  };
  // the K steps of stage s from weight buffer b: rows [r0, r0 + RG)
  auto compute = [&](int s, int b) {
    int c, r0, tpk;
    stage_of(s, c, r0, tpk);
    const uint16_t *Lwh = RES ? Lw + (size_t)c * KT * BN * 32 : Lw + 2 * b * WIMG;
    const uint16_t *Lwl = RES ? Lwh + (size_t)wrows * BN * 32 : Lwh + WIMG;
    if (tpk == 1) {
      // one tap per K step, uniform over the wave: the RG taps from r0
#pragma unroll
      for (int tt = 0; tt < RG; ++tt) {
        const int dy = (r0 + tt) / KS, dx = (r0 + tt) - dy * KS;
        f16x8 ah[NT], al[NT], bh[RW], bl[RW];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int o = swz(tt * BN + j * 16 + col, hi);
          ah[j] = *reinterpret_cast<const f16x8 *>(Lwh + o);
          al[j] = *reinterpret_cast<const f16x8 *>(Lwl + o);
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const int o = swzx(((wave * RW + r) * S + dy) * IWP + col * S + dx, col * S + dx, hi);
          bh[r] = *reinterpret_cast<const f16x8 *>(Lih + o);
          bl[r] = *reinterpret_cast<const f16x8 *>(Lil + o);
        }
        mfmas(ah, al, bh, bl);
      }
    } else {
      // tpk taps per K step: lane group hi reads tap tpk * row + hi / spt,
      // channel slot hi % spt (the packed weights follow the same order)
      const int rows = chunk_rows(KT, tpk);
      const int nr = rows - r0 < RG ? rows - r0 : RG;
      const int spt = 4 / tpk;
      const int sub = hi / spt, slot = hi - sub * spt;
      constexpr int RMAX = RG < (KT + 1) / 2 ? RG : (KT + 1) / 2;   // rows of a stage with >= 2 taps per row
#pragma unroll
      for (int rr = 0; rr < RMAX; ++rr) {
        if (rr >= nr) break;
        int tap = tpk * (r0 + rr) + sub;
        if (tap >= KT) tap = 0;  // zero weights, any finite data
        const int dy = tap / KS, dx = tap - dy * KS;
        f16x8 ah[NT], al[NT], bh[RW], bl[RW];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int o = swz(rr * BN + j * 16 + col, hi);
          ah[j] = *reinterpret_cast<const f16x8 *>(Lwh + o);
          al[j] = *reinterpret_cast<const f16x8 *>(Lwl + o);
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const int o = swzx(((wave * RW + r) * S + dy) * IWP + col * S + dx, col * S + dx, slot);
          bh[r] = *reinterpret_cast<const f16x8 *>(Lih + o);
          bl[r] = *reinterpret_cast<const f16x8 *>(Lil + o);
        }
        mfmas(ah, al, bh, bl);
      }
    }
  };

  // Pipeline (k counts stages over all of this workgroup's tiles; stage k's
  // weights are in buffer k & 1):
  //   top barrier: stage k's LDS-DMA has landed (each wave waited for its own
  //   loads before it) and every wave is done with stage k - 1;
  //   chunk start: publish the image from registers, barrier, then refill the
  //   registers with the next chunk's pieces (a whole chunk of MFMAs ahead);
  //   issue stage k + 1's weights into the other buffer; MFMAs of stage k.
  if constexpr (RES) {
    int oy0, ox0, n0;
    tile_of(g, oy0, ox0, n0);
    load_resident(n0);   // the n-block is fixed per workgroup (grid stride is a multiple of nblk)
  } else {
    issue_w(g, 0, 0);
  }
  prefetch_img(g, 0);
  bool img_inflight = false;   // the image loads are consumed at the first publish
  int k = 0;
  for (int t = g; t < p.ntiles; t += G) {
    int oy0, ox0, n0;
    tile_of(t, oy0, ox0, n0);
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        am[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ac[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    const bool more = t + G < p.ntiles;
    for (int s = 0; s < nstages; ++s, ++k) {
      // stage s's weights (the LDS-DMA issued one stage ago, before that
      // stage's image loads) have landed; image loads issued then may still
      // be in flight (vector path: their count is known)
      if (RES) wait_lgkm();   // (the resident weights: vmcnt(0) before the first barrier below)
      else if (img_inflight && p.vec) wait_vm_n_lgkm<G_::NLV * (GATE ? 2 : 1)>();
      else wait_vm_lgkm();
      if (RES && k == 0) wait_vm_lgkm();
      raw_barrier();
      img_inflight = false;
      int c, r0, tpk;
      stage_of(s, c, r0, tpk);
      if (r0 == 0) {
        if (!(p.dbg & 2)) publish_img();   // waits for its own image loads
        if (s == 0) epi::stage_consts(p, Lc, n0, BN);
        wait_lgkm();
        raw_barrier();
      }
      if constexpr (!RES) {
        if (s + 1 < nstages) issue_w(t, s + 1, (k + 1) & 1);
        else if (more) issue_w(t + G, 0, (k + 1) & 1);
      }
      if (r0 == 0) {
        if (p.dbg & 4) {
        } else if (c + 1 < p.nchunks) prefetch_img(t, c + 1), img_inflight = true;
        else if (more) prefetch_img(t + G, 0), img_inflight = true;
      }
      if (!(p.dbg & 1)) compute(s, k & 1);
    }
    if (p.dbg & 8) continue;
    if (p.direct) {
      // epilogue straight from the accumulators: lane (col, hi) of fragment
      // (r, j) holds output channels n0 + 16 j + 4 hi .. + 3 of pixel (row
      // wave * RW + r, column col); out = scale * (res2 + (res + act(acc +
      // bias))) in the reference's order, 16-byte loads and stores
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int oy = oy0 + wave * RW + r, ox = ox0 + col;
        const bool okp = oy < p.Ho && ox < p.Wo;
        const int64_t pix = (int64_t)oy * p.Wout + ox;
        f32x4 r1[NT], r2[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int n = n0 + j * 16 + hi * 4;
          const bool ok = okp && n < p.cout;
          r1[j] = (p.res && ok) ? *reinterpret_cast<const f32x4 *>(reinterpret_cast<const float *>(p.res) +
                                                                  pix * p.rcs + p.rco + n)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
          r2[j] = (p.res2 && ok) ? *reinterpret_cast<const f32x4 *>(reinterpret_cast<const float *>(p.res2) +
                                                                   pix * p.r2cs + p.r2co + n)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int nl = j * 16 + hi * 4, n = n0 + nl;
          const float4 bb = *reinterpret_cast<const float4 *>(Lc + nl);
          const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + nl);
          f32x4 v;
          v[0] = (am[r][j][0] + ac[r][j][0] * kLoInv) + bb.x;
          v[1] = (am[r][j][1] + ac[r][j][1] * kLoInv) + bb.y;
          v[2] = (am[r][j][2] + ac[r][j][2] * kLoInv) + bb.z;
          v[3] = (am[r][j][3] + ac[r][j][3] * kLoInv) + bb.w;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(p.act, v[e], p.slope);
          if (p.res) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = r1[j][e] + v[e];
          }
          if (p.res2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = r2[j][e] + v[e];
          }
          if (p.scale) {
            v[0] *= sc.x;
            v[1] *= sc.y;
            v[2] *= sc.z;
            v[3] *= sc.w;
          }
          if (okp && n < p.cout)
            *reinterpret_cast<f32x4 *>(reinterpret_cast<float *>(p.y) + pix * p.ycs + p.yco + n) = v;
        }
      }
      continue;
    }
    wait_lgkm();
    raw_barrier();     // every wave is done reading the image: T may overwrite it
    constexpr int LD = G_::LD;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = am[r][j][e] + ac[r][j][e] * kLoInv;
        epi::put4(p, T, LD, (wave * RW + r) * 16 + col, j * 16 + hi * 4, Lc, v);
      }
    wait_lgkm();
    raw_barrier();
    epi::store_tile<float, epi::ipt(TH * 16, BN, kNT)>(p, T, LD, TH * 16, n0, min(BN, p.cout - n0), Lc, BN,
                                                       [&](int l, int &oy, int &ox) {
      oy = oy0 + (l >> 4);
      ox = ox0 + (l & 15);
      return oy < p.Ho && ox < p.Wo;
    });
  }
  wait_vm_lgkm();   // no LDS-DMA left in flight when the workgroup exits
}

int g_cus = 0;
int g_dbg = 0;
int g_occ = 0;   // dcvc_set_option("sconv_occupancy", n): workgroups per CU (0 = as many as the LDS holds)

template <int KS, int S, int BN, int RW, int NW, bool GATE, bool RES>
int launch(SP p, hipStream_t st) {
  typedef SG<KS, S, BN, RW, NW, RES> G_;
  constexpr int kNT = NW * 64;
  const int wrows = (p.nchunks - 1) * G_::KT + (G_::KT + p.tpk_last - 1) / p.tpk_last;
  const size_t lds = G_::LDS + (RES ? (size_t)wrows * G_::WROW : 0);
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  p.tiles_x = (p.Wo + 15) / 16;
  p.tiles_y = (p.Ho + G_::TH - 1) / G_::TH;
  p.nblk = (p.cout + BN - 1) / BN;
  const int64_t nt = (int64_t)p.tiles_x * p.tiles_y * p.nblk;
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
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu > 8 / NW * 2) per_cu = 8 / NW * 2;
  if (g_occ > 0 && g_occ < per_cu) per_cu = g_occ;
  int64_t G = (int64_t)g_cus * per_cu;
  if (G > nt) G = nt;
  // a workgroup keeps one n-block (resident weights, loaded once): the grid
  // stride must be a multiple of the n-block count.  A grid smaller than the
  // n-block count (few CUs, or the sconv_occupancy option) cannot keep that:
  // the caller then takes the streamed-weight kernel, or for a 1x1 layer
  // (no streamed variant) the grid grows to one workgroup per n-block
  if (RES && G < p.nblk) {
    if (KS != 1) return DCVC_HIP_EUNSUPPORTED;
    G = p.nblk;
  }
  if (RES && G % p.nblk) G = G / p.nblk * p.nblk;
  if (G < 1) G = 1;
  auto kern = sconv_kernel<KS, S, BN, RW, NW, GATE, RES>;
  dcvc_note_kernel("sconv_kernel<%d, %d, %d, %d, %d, %s, %s>@%lld", KS, S, BN, RW, NW, bname(GATE), bname(RES),
                   (long long)G * kNT);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  p.dbg = g_dbg;
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(kNT), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

int g_waves = 8;   // dcvc_set_option("sconv_waves", 4 | 8): waves per workgroup of the streamed-weight kernels
int g_resident = 1;   // dcvc_set_option("sconv_resident", 0): streamed weights only (A/B)

// tile rows per wave: the tallest tile that still gives >= 1.5 tiles per CU
// and whose image prefetch fits the registers, else the smallest
int g_rw = 0;   // dcvc_set_option("sconv_rw", 1 | 2 | 4): force the tile rows per wave (A/B; 0 = auto)

template <int KS, int S, int BN, int NW, bool GATE, bool RES>
int pick_rw_nw(SP p, hipStream_t st) {
  const int64_t tx = (p.Wo + 15) / 16, nb = (p.cout + BN - 1) / BN;
  auto tiles = [&](int th) { return g_rw ? 384 : tx * ((p.Ho + th - 1) / th) * nb; };
  constexpr int PMAX = NW == 8 ? 5 : 8;   // image pieces per thread the registers allow
  if (g_rw == 1) return launch<KS, S, BN, 1, NW, GATE, RES>(p, st);
  if constexpr (SG<KS, S, BN, 4, NW, RES>::LDS <= 160 * 1024 && SG<KS, S, BN, 4, NW, RES>::PPI <= PMAX &&
                !(NW == 4 && KS == 3 && BN == 64)) {
    if (tiles(4 * NW) >= 384 && g_rw != 2) {
      const int r = launch<KS, S, BN, 4, NW, GATE, RES>(p, st);
      if (r != DCVC_HIP_EUNSUPPORTED) return r;
    }
  }
  if constexpr (SG<KS, S, BN, 2, NW, RES>::LDS <= 160 * 1024 && SG<KS, S, BN, 2, NW, RES>::PPI <= PMAX) {
    if (tiles(2 * NW) >= 384) {
      const int r = launch<KS, S, BN, 2, NW, GATE, RES>(p, st);
      if (r != DCVC_HIP_EUNSUPPORTED) return r;
    }
  }
  return launch<KS, S, BN, 1, NW, GATE, RES>(p, st);
}

// n-blocks in preference order: fewest padded output channels, wider first
inline void bn_order(int cout, int maxbn, int out[4]) {
  int c[4] = {64, 48, 32, 16}, n = 0;
  for (int i = 0; i < 4; ++i)
    if (c[i] <= maxbn) out[n++] = c[i];
  for (int i = n; i < 4; ++i) out[i] = 0;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const int pi = (cout + out[i] - 1) / out[i] * out[i] - cout, pj = (cout + out[j] - 1) / out[j] * out[j] - cout;
      if (pj < pi) std::swap(out[i], out[j]);
    }
}

template <int KS, int S, bool GATE, bool RES, int NW>
int try_bn(SP p, int bn, hipStream_t st) {
  switch (bn) {
    case 16: return pick_rw_nw<KS, S, 16, NW, GATE, RES>(p, st);
    case 32: return pick_rw_nw<KS, S, 32, NW, GATE, RES>(p, st);
    case 48: return pick_rw_nw<KS, S, 48, NW, GATE, RES>(p, st);
    case 64: return pick_rw_nw<KS, S, 64, NW, GATE, RES>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}

// dcvc_set_option("sconv_res_waves", 4 | 8 | 0 = auto): waves per workgroup of
// the resident kernels; auto = 8 for 3x3 (two waves per SIMD hide each
// other's LDS and VALU phases: 48->48 at 1080p 548 -> 465 us), 4 for 1x1
// (a wave per SIMD with the whole register file: 48->192 at 1080p 2300 ->
// 1056 us)
int g_res_waves = 0;

template <int KS, int S, bool GATE>
int pick_bn(SP p, hipStream_t st) {
  int order[4];
  // stride-2 3x3 layers stream their weights: a 32- or 16-channel resident
  // n-block re-reads the 4x larger input once per n-block, and the streamed
  // 48/64-channel blocks win at every DC shape (128->96 at 544x960 436 -> 267
  // us, 64->64 at 1088x1920 367 -> 320, 48->64 303 -> 280, 56->64 346 vs 348;
  // scripts/gpu_r04o.sh, profiles/r04o_sconv_s2_ab.jsonl)
  if constexpr (KS != 7 && !(KS == 3 && S == 2)) {
    // resident weights where they fit
    if (g_resident) {
      bn_order(p.cout, 64, order);
      for (int i = 0; i < 4 && order[i]; ++i) {
        // a 16-channel resident n-block of a wide layer re-reads and re-splits
        // the input once per n-block (8+ times): streamed 64-channel blocks win
        // there (128 -> 192 at 544x960: 1063 -> 969 us, 192 -> 256 at 272x480:
        // 742 -> 462 us), not at 3-6 n-blocks (96 -> 48 at 1080p: 868 vs 1164
        // us, 192 -> 96 at 272x480: 258 vs 370 us; scripts/gpu_r03zd.sh, r03zf)
        if (KS == 3 && order[i] == 16 && (p.cout + 15) / 16 >= 8) continue;
        const int nw = g_res_waves ? g_res_waves : (KS == 1 ? 4 : 8);
        const int r = nw == 4 ? try_bn<KS, S, GATE, true, 4>(p, order[i], st)
                              : try_bn<KS, S, GATE, true, 8>(p, order[i], st);
        if (r != DCVC_HIP_EUNSUPPORTED) return r;
      }
    }
  }
  if constexpr (KS == 1) {
    return DCVC_HIP_EUNSUPPORTED;   // (a 1x1 n-block of 16 channels always fits resident, at any grid)
  } else {
    // streamed weights; 7x7 layers stay <= 32 channels per n-block
    bn_order(p.cout, KS == 7 ? 32 : 64, order);
    if (g_waves == 4) return try_bn<KS, S, GATE, false, 4>(p, order[0], st);
    return try_bn<KS, S, GATE, false, 8>(p, order[0], st);
  }
}

}  // namespace

extern "C" void dcvc_internal_sconv_occupancy(int v) { g_occ = v; }
extern "C" void dcvc_internal_sconv_dbg(int v) { g_dbg = v; }
extern "C" void dcvc_internal_sconv_rw(int v) { g_rw = v; }
extern "C" int dcvc_internal_sgemm(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_sconv_waves(int v) { g_waves = v; }
extern "C" void dcvc_internal_sconv_resident(int v) { g_resident = v; }
extern "C" void dcvc_internal_sconv_res_waves(int v) { g_res_waves = v; }

// f16x3 convolutions (a->compute == DCVC_F16X3): fp32 input and output views.
// Kernel sizes 1, 3 (stride 1 or 2) and 7 (stride 1); the ConvFFN2 gate input
// op for 1x1.  Called by dcvc_conv2d after its shape validation.
extern "C" int dcvc_internal_sconv(const dcvc_conv_args *a, void *stream) {
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EINVAL;
  if (a->kh != a->kw || (a->kh != 1 && a->kh != 3 && a->kh != 7)) return DCVC_HIP_EUNSUPPORTED;
  if (a->stride != 1 && !(a->stride == 2 && a->kh != 7)) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op == DCVC_IN_GATE && a->kh != 1) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh == 1) {   // the pixel-GEMM kernel (sgemm.hip) where it applies
    const int r = dcvc_internal_sgemm(a, stream);
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  SP p{};
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.bias = a->bias;
  p.y = a->y.ptr;
  p.Ho = (a->x.H + 2 * a->pad - a->kh) / a->stride + 1;
  p.Wo = (a->x.W + 2 * a->pad - a->kw) / a->stride + 1;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.pad = a->pad;
  p.in_op = a->in_op;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.shuffle = a->shuffle;
  p.scale = a->scale;
  p.Wout = a->y.W;
  if (a->res.ptr) {
    p.res = a->res.ptr;
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
  }
  if (a->res2.ptr) {
    p.res2 = a->res2.ptr;
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
  }
  p.vec = (a->cin % 8 == 0) && (p.xcs % 4 == 0) && (p.xco % 4 == 0) && ((uintptr_t)p.x % 16 == 0);
  {
    bool vo = (p.ycs % 8 == 0) && (p.yco % 8 == 0) && ((uintptr_t)p.y % 16 == 0);
    if (a->res.ptr) vo = vo && (p.rcs % 8 == 0) && (p.rco % 8 == 0) && ((uintptr_t)p.res % 16 == 0);
    if (a->res2.ptr) vo = vo && (p.r2cs % 8 == 0) && (p.r2co % 8 == 0) && ((uintptr_t)p.res2 % 16 == 0);
    p.vec_out = vo ? 1 : 0;
    // the direct epilogue stores 4 channels per lane: needs cout % 4 == 0 and
    // 16-byte aligned output / residual pieces
    p.direct = !a->shuffle && a->cout % 4 == 0 && (p.ycs % 4 == 0) && (p.yco % 4 == 0) && ((uintptr_t)p.y % 16 == 0);
    if (a->res.ptr) p.direct = p.direct && (p.rcs % 4 == 0) && (p.rco % 4 == 0) && ((uintptr_t)p.res % 16 == 0);
    if (a->res2.ptr) p.direct = p.direct && (p.r2cs % 4 == 0) && (p.r2co % 4 == 0) && ((uintptr_t)p.res2 % 16 == 0);
  }
  p.nchunks = (a->cin + 31) / 32;
  const int vc = a->cin - 32 * (p.nchunks - 1);
  p.tpk_last = vc <= 8 ? 4 : vc <= 16 ? 2 : 1;
  const int kt = a->kh * a->kw;
  p.wchunk = (int64_t)2 * kt * a->cout * 32;
  {
    const int rl = (kt + p.tpk_last - 1) / p.tpk_last;
    const int64_t wb = ((int64_t)(p.nchunks - 1) * p.wchunk + (int64_t)2 * rl * a->cout * 32) * 2;
    if (wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
    p.wbytes = (int)wb;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool gate = a->in_op == DCVC_IN_GATE;
  switch (a->kh) {
    case 1:
      if (a->stride == 1) return gate ? pick_bn<1, 1, true>(p, st) : pick_bn<1, 1, false>(p, st);
      return pick_bn<1, 2, false>(p, st);
    case 3:
      if (a->stride == 1) return pick_bn<3, 1, false>(p, st);
      return pick_bn<3, 2, false>(p, st);
    default:
      return pick_bn<7, 1, false>(p, st);
  }
}
