// Persistent 3x3 stride-1 convolution for bf16 NHWC feature maps with
// 32..128 input channels and <= 64 output channels per workgroup: the
// full-resolution ResBlock / context-fusion / recon convs of DCVC-DC
// (SURVEY §8 a13-a15).
//
// Why a second 3x3 kernel: the per-workgroup kernel (conv3x3.hip) restages
// the whole weight slice for every 16x16 tile and waits out one HBM round
// trip per 32-channel chunk; rocprofv3 counted 49 % of its wave cycles in
// s_waitcnt/barrier waits and ~13 VALU instructions per MFMA (epilogue and
// staging generality), with the MFMA pipe 14 % busy (profiles/r01_*).
// This kernel is organised around hiding that latency instead:
//   * one 512-thread workgroup per CU (grid = #CUs x n-blocks) keeps its
//     BN-channel weight slice resident in LDS for the whole launch and walks
//     output tiles 16 pixels wide and 32, 16 or 8 rows high (8 waves x 4, 2
//     or 1 pixel rows: the tallest whose weights, halo images and fp32
//     epilogue tile fit the LDS; 32-row tiles read 7 LDS operands per 12
//     MFMAs instead of 5 per 6 and 34 / 32 halo rows instead of 18 / 16);
//   * the next tile's input is loaded into registers right after the current
//     tile's image is published, so its HBM latency hides behind the current
//     tile's MFMAs and epilogue (software pipeline, prefetch distance 1; 2
//     for 16-row tiles, where the registers allow a second set);
//   * a thread's staging pieces run along the channel axis first, so the
//     threads of a wave read whole contiguous pixel rows (CIN * 2 bytes per
//     pixel) instead of 64-byte pieces one pixel stride apart;
//   * the tiles of one XCD's workgroups are consecutive in raster order, so
//     halo rows and columns shared by neighbouring tiles are L2 hits;
//   * the epilogue is specialised to what these layers need (bias, leaky
//     ReLU, up to two bf16 residuals, per-channel scale, bf16 store); for
//     16-row tiles it runs straight from the accumulators (each lane stores
//     4 channels of one pixel, residual pieces prefetched a tile ahead in the
//     same shape), so waves leave a tile without a barrier and, where two
//     input images fit, tile t + 1 is published while slower waves still
//     read tile t's: one barrier per tile.  Pixel shuffle and 8-row tiles go
//     through an fp32 LDS tile that reuses the input image's space.
// The MFMA sequence (per 32-channel chunk, taps 0..8; then a 16-channel tail
// as five tap pairs) and the fp32 epilogue order are those of conv3x3.hip, so
// results are bit-identical to it (tests/test_gpu_kernels.py).
#include "common.h"

namespace {

constexpr int kPitch = 20;  // LDS pixels per halo row (18 used)

struct P3 {
  const uint16_t *x;
  int H, W, xcs, xco;
  const uint16_t *w;  // packed [cout][3][3][cinp] bf16
  int cinp;
  const float *bias;
  const float *scale;
  void *y;
  int ycs, yco, Wout;
  const void *res;
  int rcs, rco;
  const void *res2;
  int r2cs, r2co;
  int cout;
  int in_lrelu;
  float in_slope;
  int act;
  float slope;
  int tiles_x, tiles_y, nblk_n;
  int xbytes, rbytes, r2bytes, ybytes;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// 8-element pieces of the output / residual type; an element index < 0
// reads zeros (out-of-range buffer offset)
template <typename T> struct Vec8;
template <> struct Vec8<uint16_t> {
  typedef u16x8 raw;
  __device__ __forceinline__ static raw load(__amdgpu_buffer_rsrc_t r, int e) {
    return __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(r, e < 0 ? 0x7ffffff0 : e * 2, 0, 0));
  }
  __device__ __forceinline__ static float get(const raw &v, int j) { return bf2f(v[j]); }
  __device__ __forceinline__ static void bstore(__amdgpu_buffer_rsrc_t r, int e, const float v[8]) {
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), r, e < 0 ? 0x7ffffff0 : e * 2, 0, 0);
  }
};
typedef float f32x8 __attribute__((ext_vector_type(8)));
template <> struct Vec8<float> {
  typedef f32x8 raw;
  __device__ __forceinline__ static raw load(__amdgpu_buffer_rsrc_t r, int e) {
    const int o = e < 0 ? 0x7fffffe0 : e * 4;
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, o + 16, 0, 0);
    const f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
    return f32x8{fa[0], fa[1], fa[2], fa[3], fb[0], fb[1], fb[2], fb[3]};
  }
  __device__ __forceinline__ static float get(const raw &v, int j) { return v[j]; }
  __device__ __forceinline__ static void bstore(__amdgpu_buffer_rsrc_t r, int e, const float v[8]) {
    const int o = e < 0 ? 0x7fffffe0 : e * 4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v[0], v[1], v[2], v[3]}), r, o, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v[4], v[5], v[6], v[7]}), r, o + 16, 0, 0);
  }
};

__device__ __forceinline__ int swz(int row, int x, int slot) {
  return row * 32 + ((slot ^ (((x >> 2) & 1) << 1)) << 3);
}

// MODE 0: epilogue through an fp32 LDS tile (pixel shuffle), one input
// image; 1: epilogue straight from the accumulators, one image; 2: direct
// epilogue, two images (tile t + 1 is published while slower waves still
// read tile t's, so one barrier per tile)
template <int CIN, int BN, int NW, int RW, int MODE = 0>
struct Geo {
  static constexpr int NCH = CIN / 32;
  static constexpr bool TAIL = (CIN % 32) == 16;
  static constexpr int NIMG = NCH + (TAIL ? 1 : 0);
  static constexpr int KS = 9 * NCH + (TAIL ? 5 : 0);
  static constexpr int TH = NW * RW;
  static constexpr int IH = TH + 2;
  static constexpr int NT = BN / 16;
  static constexpr int NTHR = NW * 64;
  static constexpr int IMG = IH * kPitch * 32;            // elements per chunk image
  static constexpr size_t WB = (size_t)KS * BN * 64;      // resident weights
  static constexpr int LD = BN + 4;                       // fp32 epilogue tile row
  static constexpr size_t TB = (size_t)TH * 16 * LD * 4;
  static constexpr size_t IB = (size_t)NIMG * IMG * 2;
  static constexpr size_t BUF = MODE == 2 ? 2 * IB : MODE == 1 ? IB : (IB > TB ? IB : TB);
  static constexpr size_t LC = WB + BUF;                  // bias | scale
  static constexpr size_t DUMMY = LC + 2 * BN * 4;        // 16-byte sink for idle staging lanes
  static constexpr size_t LDS = DUMMY + 16;
  static constexpr int QP = CIN / 8;                      // 16-byte pieces per pixel
  static constexpr int PIX = IH * 18;
  static constexpr int PP = (PIX * QP + NTHR - 1) / NTHR; // input pieces per thread
  static constexpr int OQ = BN / 8;
  static constexpr int PO = (TH * 16 * OQ + NTHR - 1) / NTHR;  // output pieces per thread (either layout)
};

template <int CIN, int BN, int NW, int RW, typename TOUT, bool SHUF, int MODE>
__global__ void __launch_bounds__(NW * 64) conv3p_kernel(P3 p) {
  static_assert(!SHUF || MODE == 0, "pixel shuffle goes through the LDS tile");
  typedef Geo<CIN, BN, NW, RW, MODE> G_;
  constexpr bool kDirect = MODE != 0;
  constexpr int NCH = G_::NCH, KS = G_::KS, NT = G_::NT, TH = G_::TH, IMG = G_::IMG;
  constexpr int NTHR = G_::NTHR, QP = G_::QP, PP = G_::PP, LD = G_::LD, OQ = G_::OQ, PO = G_::PO;
  constexpr int ROWB = kPitch * 32;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Lw = reinterpret_cast<uint16_t *>(smem);
  uint16_t *Li = reinterpret_cast<uint16_t *>(smem + G_::WB);
  float *T = reinterpret_cast<float *>(smem + G_::WB);
  float *Lc = reinterpret_cast<float *>(smem + G_::LC);
  uint16_t *const Ldummy = reinterpret_cast<uint16_t *>(smem + G_::DUMMY);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int nb = blockIdx.x % p.nblk_n;
  const int n0 = nb * BN;
  const int G = gridDim.x / p.nblk_n;
  int g = blockIdx.x / p.nblk_n;
  // consecutive tiles on one XCD (workgroups are dealt to XCDs round robin)
  if (p.nblk_n == 1 && (G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);
  const int ntiles = p.tiles_x * p.tiles_y;
  if (g >= ntiles) return;

  // ---- per-thread staging plan: piece u = (halo pixel, 16-byte channel piece)
  int lofs[PP], rel[PP], pyx[PP];
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    const int it = tid + u * NTHR;
    lofs[u] = -1;
    rel[u] = 0;
    pyx[u] = 0;
    if (it < G_::PIX * QP) {
      const int pix = it / QP, q = it - pix * QP;
      const int iy = pix / 18, ix = pix - iy * 18;
      const int c = q >> 2, slot = q & 3;
      lofs[u] = c * IMG + swz(iy * kPitch + ix, ix, slot);
      rel[u] = ((iy - 1) * p.W + (ix - 1)) * p.xcs + p.xco + q * 8;
      pyx[u] = (iy << 8) | ix;
    }
  }
  // buffer loads: an out-of-range offset returns zeros, so halo pixels outside
  // the image (and tiles past the last) need no branch.  Every global load and
  // store in the tile loop is unconditional and every loaded value is
  // consumed unconditionally: hipcc's s_waitcnt placement counts outstanding
  // memory operations per path, and one conditional load or store makes it
  // fall back to vmcnt(0), which waits for the prefetch two tiles ahead too.
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.x), (short)0, p.xbytes, 0x00020000);
  auto issue = [&](int t, u16x8 (&pf)[PP]) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * 16;
    const int base = (oy0 * p.W + ox0) * p.xcs;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int gy = oy0 - 1 + (pyx[u] >> 8), gx = ox0 - 1 + (pyx[u] & 255);
      const bool in = lofs[u] >= 0 && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
      const int off = in ? (base + rel[u]) * 2 : 0x7ffffff0;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      pf[u] = __builtin_bit_cast(u16x8, v);
    }
  };
  auto publish = [&](const u16x8 (&pf)[PP], uint16_t *Li) {
    if (p.in_lrelu) {
#pragma unroll
      for (int u = 0; u < PP; ++u) {
        u16x8 v = pf[u];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(v[j]);
          v[j] = f2bf(f >= 0.f ? f : f * p.in_slope);
        }
        *reinterpret_cast<u16x8 *>(lofs[u] >= 0 ? Li + lofs[u] : Ldummy) = v;
      }
    } else {
#pragma unroll
      for (int u = 0; u < PP; ++u) *reinterpret_cast<u16x8 *>(lofs[u] >= 0 ? Li + lofs[u] : Ldummy) = pf[u];
    }
  };

  // input tiles two ahead: tile t's halo is loaded while tiles t - 2G and
  // t - G run (two register sets, alternating between consecutive tiles)
  // (16-row tiles only: for 8-row tiles, 128->64 at 1/2 resolution, one
  // tile ahead measured faster)
  constexpr bool kDeep = RW == 2;
  u16x8 pfa[PP], pfb[PP];
  issue(g, pfa);
  if constexpr (kDeep) issue(g + G, pfb);
  // ---- resident weights [KS][BN][32] (swizzled by row) + epilogue constants
  for (int it = tid; it < KS * BN * 4; it += NTHR) {
    const int row = it >> 2, sl = it & 3;
    const int ks = row / BN, n = n0 + row - ks * BN;
    int tap, c;
    if (ks < 9 * NCH) {
      tap = ks % 9;
      c = (ks / 9) * 32 + sl * 8;
    } else {
      tap = 2 * (ks - 9 * NCH) + (sl >> 1);
      c = NCH * 32 + (sl & 1) * 8;
    }
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0;
    if (tap < 9 && n < p.cout) v = *reinterpret_cast<const u16x8 *>(p.w + ((int64_t)n * 9 + tap) * p.cinp + c);
    *reinterpret_cast<u16x8 *>(Lw + swz(row, row, sl)) = v;
  }
  for (int i = tid; i < BN; i += NTHR) {
    const int n = n0 + i;
    const int cy = (SHUF ? n0 / 4 : n0) + i;  // scale is per output channel (after shuffle)
    Lc[i] = (p.bias && n < p.cout) ? p.bias[n] : 0.f;
    Lc[BN + i] = (p.scale && cy < (SHUF ? p.cout / 4 : p.cout)) ? p.scale[cy] : 1.f;
  }

  // per-lane MFMA operand bases (elements)
  int offB[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) offB[dx] = swz(wave * RW * kPitch + col + dx, col + dx, hi);
  int offT[5];
#pragma unroll
  for (int pr = 0; pr < 5; ++pr) {
    int t = 2 * pr + (hi >> 1);
    if (t > 8) t = 0;  // tap 9: zero weights, any finite data
    const int dy = t / 3, dx = t - dy * 3;
    offT[pr] = NCH * IMG + swz((wave * RW + dy) * kPitch + col + dx, col + dx, hi & 1);
  }
  const uint16_t *LwA = Lw + swz(col, col, hi);
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p.res), (short)0, p.rbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr2 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p.res2), (short)0, p.r2bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.ybytes, 0x00020000);

  // epilogue-B piece u of tile t: 8 consecutive output channels of one
  // output pixel, in output-row order (SHUF: conv channel n of pixel (y, x)
  // is output channel n >> 2 of pixel (2y + (n >> 1 & 1), 2x + (n & 1)),
  // pixel_shuffle(2)); ob = output pixel index, src = its fp32 tile offset
  auto piece = [&](int t, int u, int64_t &ob, int &src, int &cq, bool &ok) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * 16;
    constexpr int NQ = SHUF ? BN / 32 : BN / 8;  // pieces per (pixel, sub-position)
    const int it = tid + u * NTHR;
    const int q = it % NQ, r = it / NQ;
    int l, oy, ox;
    if constexpr (SHUF) {
      const int dx = r & 1, cx = (r >> 1) & 15, dy = (r >> 5) & 1, cyl = r >> 6;
      l = cyl * 16 + cx;
      oy = 2 * (oy0 + cyl) + dy;
      ox = 2 * (ox0 + cx) + dx;
      ok = it < TH * 16 * 4 * NQ && oy0 + cyl < p.H && ox0 + cx < p.W;
      src = l * LD + 4 * q * 8 + dy * 2 + dx;
    } else {
      l = r;
      oy = oy0 + (l >> 4);
      ox = ox0 + (l & 15);
      ok = it < TH * 16 * NQ && oy < p.H && ox < p.W;
      src = l * LD + q * 8;
    }
    cq = q * 8;
    ob = (int64_t)oy * p.Wout + ox;
  };
  // residual pieces of tile t, loaded right after tile t - G's epilogue has
  // consumed its own, so their HBM latency hides behind tile t's publish and
  // MFMAs
  typedef typename Vec8<TOUT>::raw RV;
  // 32-row tiles (RW = 4) take no second residual (the host routes such
  // layers to 16-row tiles): its pieces would not fit the register budget
  constexpr bool kR2 = RW != 4;
  constexpr int PO2 = kR2 ? PO : 1;
  auto load_res = [&](int t, RV (&r1)[PO], RV (&r2)[PO2]) {
#pragma unroll
    for (int u = 0; u < PO; ++u) {
      int64_t ob;
      int src, cq;
      bool ok;
      piece(t, u, ob, src, cq, ok);
      const int cb = (SHUF ? n0 / 4 : n0) + cq;
      r1[u] = Vec8<TOUT>::load(rr, ok ? (int)(ob * p.rcs + p.rco + cb) : -1);  // no residual: 0-byte buffer
      if constexpr (kR2) r2[u] = Vec8<TOUT>::load(rr2, ok ? (int)(ob * p.r2cs + p.r2co + cb) : -1);
    }
  };
  // MODE != 0: residual pieces are the accumulators' own (4 channels of one
  // pixel per lane and (row, n-tile)), 8 (bf16) or 16 (f32) bytes each
  typedef typename std::conditional<sizeof(TOUT) == 2, u16x4, f32x4>::type DV;
  auto dload = [&](__amdgpu_buffer_rsrc_t r, int e) -> DV {
    if constexpr (sizeof(TOUT) == 2) {
      return __builtin_bit_cast(u16x4, __builtin_amdgcn_raw_buffer_load_b64(r, e < 0 ? 0x7ffffff0 : e * 2, 0, 0));
    } else {
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, e < 0 ? 0x7ffffff0 : e * 4, 0, 0));
    }
  };
  auto dget = [](const DV &v, int e) -> float {
    if constexpr (sizeof(TOUT) == 2) return bf2f(v[e]);
    else return v[e];
  };
  auto load_dres = [&](int t, DV (&d1)[RW][NT], DV (&d2)[RW][NT]) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * 16;
    const int ox = ox0 + col;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int oy = oy0 + wave * RW + r;
      const bool ok = oy < p.H && ox < p.W;
      const int ob = oy * p.Wout + ox;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + j * 16 + hi * 4;
        d1[r][j] = dload(rr, ok ? ob * p.rcs + p.rco + n : -1);     // no residual: 0-byte buffer
        d2[r][j] = dload(rr2, ok ? ob * p.r2cs + p.r2co + n : -1);
      }
    }
  };
  RV ra1[kDirect ? 1 : PO], ra2[kDirect ? 1 : PO2];
  DV da1[kDirect ? RW : 1][NT], da2[kDirect ? RW : 1][NT];
  if constexpr (kDirect) load_dres(g, da1, da2);
  else load_res(g, ra1, ra2);
  int ib = 0;  // MODE 2: image buffer of the current tile

  // one tile; returns whether this workgroup has a next one
  auto tile = [&](int t, u16x8 (&pf)[PP], RV (&r1)[kDirect ? 1 : PO], RV (&r2)[kDirect ? 1 : PO2],
                  DV (&d1)[kDirect ? RW : 1][NT], DV (&d2)[kDirect ? RW : 1][NT]) -> bool {
    uint16_t *const Lt = Li + (MODE == 2 ? ib * (G_::NIMG * IMG) : 0);
    publish(pf, Lt);
    __syncthreads();
    const int tn = t + G;
    const bool more = tn < ntiles;
    issue(kDeep ? tn + G : tn, pf);  // kDeep: in flight across the next two tiles

    f32x4 acc[RW][NT];
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int dy = k / 3, dx = k % 3;
        bf16x8 a[NT], b[RW];
#pragma unroll
        for (int j = 0; j < NT; ++j)
          a[j] = *reinterpret_cast<const bf16x8 *>(LwA + ((c * 9 + k) * BN + j * 16) * 32);
#pragma unroll
        for (int r = 0; r < RW; ++r)
          b[r] = *reinterpret_cast<const bf16x8 *>(Lt + c * IMG + offB[dx] + (r + dy) * ROWB);
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[r], acc[r][j], 0, 0, 0);
      }
    }
    if constexpr (G_::TAIL) {
#pragma unroll
      for (int pr = 0; pr < 5; ++pr) {
        bf16x8 a[NT], b[RW];
#pragma unroll
        for (int j = 0; j < NT; ++j)
          a[j] = *reinterpret_cast<const bf16x8 *>(LwA + ((9 * NCH + pr) * BN + j * 16) * 32);
#pragma unroll
        for (int r = 0; r < RW; ++r) b[r] = *reinterpret_cast<const bf16x8 *>(Lt + offT[pr] + r * ROWB);
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[r], acc[r][j], 0, 0, 0);
      }
    }
    if constexpr (kDirect) {
      // ---- epilogue straight from the accumulators: out = scale * (res2 +
      // (res + act(acc + bias))), the fp32 operations and order of the LDS
      // tile path (bit-identical); lane stores 4 channels of one pixel
      const int oy0 = (t / p.tiles_x) * TH, ox = (t % p.tiles_x) * 16 + col;
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int oy = oy0 + wave * RW + r;
        const bool ok = oy < p.H && ox < p.W;
        const int yb = (oy * p.Wout + ox) * p.ycs + p.yco + n0;  // element offset (< 2^31 / 4, checked on the host)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int nl = j * 16 + hi * 4;
          const float4 bb = *reinterpret_cast<const float4 *>(Lc + nl);
          float v[4] = {acc[r][j][0] + bb.x, acc[r][j][1] + bb.y, acc[r][j][2] + bb.z, acc[r][j][3] + bb.w};
          if (p.act == DCVC_ACT_LRELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * p.slope;
          }
          if (p.res) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = dget(d1[r][j], e) + v[e];
          }
          if (p.res2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = dget(d2[r][j], e) + v[e];
          }
          if (p.scale) {
            const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + nl);
            v[0] *= sc.x;
            v[1] *= sc.y;
            v[2] *= sc.z;
            v[3] *= sc.w;
          }
          // out-of-range pixels: an out-of-range offset drops the store
          const int so = ok ? (yb + nl) * (int)sizeof(TOUT) : 0x7ffffff0;
          if constexpr (sizeof(TOUT) == 2) {
            u16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), yr, so, 0, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v[0], v[1], v[2], v[3]}), yr, so, 0, 0);
          }
        }
      }
      if (!more) return false;
      load_dres(tn, d1, d2);  // the next tile's residual pieces
      if constexpr (MODE == 1) __syncthreads();  // image read by every wave before the next publish
      if constexpr (MODE == 2) ib ^= 1;
      return true;
    } else {
    __syncthreads();  // every wave is done reading the image: T may overwrite it

    // ---- epilogue A: v = act(acc + bias) -> fp32 tile T[pixel][LD]
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int nl = j * 16 + hi * 4;
        const float4 b = *reinterpret_cast<const float4 *>(Lc + nl);
        float4 o;
        o.x = acc[r][j][0] + b.x;
        o.y = acc[r][j][1] + b.y;
        o.z = acc[r][j][2] + b.z;
        o.w = acc[r][j][3] + b.w;
        if (p.act == DCVC_ACT_LRELU) {
          o.x = o.x >= 0.f ? o.x : o.x * p.slope;
          o.y = o.y >= 0.f ? o.y : o.y * p.slope;
          o.z = o.z >= 0.f ? o.z : o.z * p.slope;
          o.w = o.w >= 0.f ? o.w : o.w * p.slope;
        }
        *reinterpret_cast<float4 *>(T + ((wave * RW + r) * 16 + col) * LD + nl) = o;
      }
    __syncthreads();

    // ---- epilogue B: out = scale * (res2 + (res + v)) in pieces of 8
    // consecutive output channels (plan and residual loads issued above)
    {
#pragma unroll
      for (int u = 0; u < PO; ++u) {
        int64_t ob;
        int src, cq;
        bool ok;
        piece(t, u, ob, src, cq, ok);
        src = ok ? src : 0;  // keep idle lanes' tile reads in range
        float v[8];
        if constexpr (SHUF) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = T[src + 4 * j];
        } else {
          const float4 a = *reinterpret_cast<const float4 *>(T + src);
          const float4 b = *reinterpret_cast<const float4 *>(T + src + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
          v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
        if (p.res) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = Vec8<TOUT>::get(r1[u], j) + v[j];
        }
        if constexpr (kR2) {
          if (p.res2) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = Vec8<TOUT>::get(r2[u], j) + v[j];
          }
        }
        if (p.scale) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] * Lc[BN + cq + j];
        }
        // pieces outside the map or past the tile plan: an out-of-range offset drops the store
        Vec8<TOUT>::bstore(yr, ok ? (int)(ob * p.ycs + p.yco + (SHUF ? n0 / 4 : n0) + cq) : -1, v);
      }
    }
    if (!more) return false;
    load_res(tn, r1, r2);   // the next tile's residual pieces, in flight during its publish and MFMAs
    __syncthreads();  // T read by every thread before the next image overwrites it
    return true;
    }
  };
  for (int t = g;;) {
    if (!tile(t, pfa, ra1, ra2, da1, da2)) break;
    t += G;
    if (!tile(t, kDeep ? pfb : pfa, ra1, ra2, da1, da2)) break;
    t += G;
  }
}

int g_cus = 0;
int g_enabled = 1;
int g_occ = 1;  // dcvc_set_option("conv3x3_occupancy", 2): two 8-row workgroups per CU where they fit
int g_rows4 = 1;  // dcvc_set_option("conv3x3_rows4", 0/1): 32-row tiles where they fit (A/B; 48->48 at 1080p 176 -> 172 us, 32->32 81 -> 69)
int g_mode = 0;  // dcvc_set_option("conv3x3_epilogue", 0/1/2, 3 = also 8-row tiles): highest epilogue mode (launch_mode)

template <int CIN, int BN, int NW, int RW, typename TOUT, bool SHUF, int MODE>
int launch(P3 p, hipStream_t st, int per_cu = 1) {
  typedef Geo<CIN, BN, NW, RW, MODE> G_;
  if constexpr (G_::LDS > 160 * 1024) {
    return DCVC_HIP_EUNSUPPORTED;
  } else {
    p.tiles_x = (p.W + 15) / 16;
    p.tiles_y = (p.H + G_::TH - 1) / G_::TH;
    p.nblk_n = (p.cout + BN - 1) / BN;
    const int64_t ntiles = (int64_t)p.tiles_x * p.tiles_y;
    if (g_cus <= 0) {
      int dev = 0;
      hipDeviceProp_t prop;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return DCVC_HIP_ELAUNCH;
      g_cus = prop.multiProcessorCount;
    }
    // a grid of fewer tiles than CUs is better served per tile
    if (ntiles * p.nblk_n < g_cus) return DCVC_HIP_EUNSUPPORTED;
    int64_t G = (int64_t)g_cus * per_cu / p.nblk_n;
    if (G > ntiles) G = ntiles;
    if (G < 1) G = 1;
    auto kern = conv3p_kernel<CIN, BN, NW, RW, TOUT, SHUF, MODE>;
    dcvc_note_kernel("conv3p_kernel<%d, %d, %d, %d, %s, %s, %d>@%lld", CIN, BN, NW, RW, tname<TOUT>(), bname(SHUF),
                     MODE, (long long)G * p.nblk_n * NW * 64);
    dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
    hipLaunchKernelGGL(kern, dim3((unsigned)(G * p.nblk_n)), dim3(NW * 64), G_::LDS, st, p);
    DCVC_LAUNCH_CHECK();
    return DCVC_HIP_OK;
  }
}

// Epilogue / image mode for layers without pixel shuffle, at most g_mode
// (dcvc_set_option("conv3x3_epilogue", m), A/B): 2 when two input images fit
// in the LDS beside the weights, else 1 (0: the fp32 LDS tile).  8-row tiles
// at one workgroup per CU keep the LDS tile (128->64 at 544x960: 128.5 us vs
// 133.4 direct); 16-row tiles gain (48->48 at 1080p: 206.5 -> 173.7 us,
// 96->48 261.7 -> 238.0, 64->64 241.9 -> 232.3; conv3_bench, same box).
template <int CIN, int BN, int NW, int RW, typename TOUT, bool SHUF>
int launch_mode(const P3 &p, hipStream_t st, int per_cu) {
  constexpr size_t cap = 160 * 1024;
  if constexpr (!SHUF) {
    if (RW == 1 && per_cu == 1 && g_mode < 3) return launch<CIN, BN, NW, RW, TOUT, SHUF, 0>(p, st, per_cu);
    if constexpr (Geo<CIN, BN, NW, RW, 2>::LDS * 1 <= cap) {
      if (g_mode >= 2 && Geo<CIN, BN, NW, RW, 2>::LDS * per_cu <= cap) return launch<CIN, BN, NW, RW, TOUT, SHUF, 2>(p, st, per_cu);
    }
    if constexpr (Geo<CIN, BN, NW, RW, 1>::LDS <= cap) {
      if (g_mode >= 1 && Geo<CIN, BN, NW, RW, 1>::LDS * per_cu <= cap) return launch<CIN, BN, NW, RW, TOUT, SHUF, 1>(p, st, per_cu);
    }
  }
  return launch<CIN, BN, NW, RW, TOUT, SHUF, 0>(p, st, per_cu);
}

// 16 output rows per tile (8 waves x 2) when the LDS holds it, else 8.
template <int CIN, int BN, typename TOUT, bool SHUF>
int pick_th(const P3 &p, hipStream_t st) {
  // 32-row tiles (4 rows per wave) where the LDS holds them (A/B: option
  // "conv3x3_rows4"): 7 LDS operand reads per 12 MFMAs instead of 5 per 6,
  // 34 / 32 halo rows instead of 18 / 16, half the tiles' fixed work
  if constexpr (!SHUF && Geo<CIN, BN, 8, 4, 0>::LDS <= 160 * 1024) {
    if (g_rows4 && !p.res2) return launch<CIN, BN, 8, 4, TOUT, SHUF, 0>(p, st, 1);
  }
  if constexpr (2 * Geo<CIN, BN, 8, 1, SHUF ? 0 : 1>::LDS <= 160 * 1024) {
    if (g_occ >= 2) return launch_mode<CIN, BN, 8, 1, TOUT, SHUF>(p, st, 2);
  }
  if constexpr (Geo<CIN, BN, 8, 2, SHUF ? 0 : 1>::LDS <= 160 * 1024) return launch_mode<CIN, BN, 8, 2, TOUT, SHUF>(p, st, 1);
  return launch_mode<CIN, BN, 8, 1, TOUT, SHUF>(p, st, 1);
}

// BN: 64 / 48 / 32 output channels per workgroup (a multiple of 32 with
// shuffle, so every sub-position gets whole 8-channel pieces)
template <int CIN>
int pick_bn(const P3 &p, bool f32out, bool shuf, hipStream_t st) {
  if (shuf) {
    if (f32out) return DCVC_HIP_EUNSUPPORTED;
    if (p.cout % 64 == 0 && Geo<CIN, 64, 8, 1>::LDS <= 160 * 1024) return pick_th<CIN, 64, uint16_t, true>(p, st);
    if (p.cout % 32 == 0) return pick_th<CIN, 32, uint16_t, true>(p, st);
    return DCVC_HIP_EUNSUPPORTED;
  }
  if (f32out) {
    if (p.cout % 64 == 0 && Geo<CIN, 64, 8, 1>::LDS <= 160 * 1024) return pick_th<CIN, 64, float, false>(p, st);
    if (p.cout % 48 == 0) return pick_th<CIN, 48, float, false>(p, st);
    if (p.cout % 32 == 0) return pick_th<CIN, 32, float, false>(p, st);
    return DCVC_HIP_EUNSUPPORTED;
  }
  if (p.cout % 64 == 0 && Geo<CIN, 64, 8, 1>::LDS <= 160 * 1024) return pick_th<CIN, 64, uint16_t, false>(p, st);
  if (p.cout % 48 == 0) return pick_th<CIN, 48, uint16_t, false>(p, st);
  if (p.cout % 32 == 0) return pick_th<CIN, 32, uint16_t, false>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

}  // namespace

// Called by dcvc_internal_conv3x3 for bf16 -> bf16 3x3 stride-1 convs without
// pixel shuffle; DCVC_HIP_EUNSUPPORTED hands the call on to conv3x3.hip.
extern "C" int dcvc_internal_conv3p(const dcvc_conv_args *a, void *stream) {
  if (!g_enabled) return DCVC_HIP_EUNSUPPORTED;
  const bool f32out = a->y.dtype == DCVC_F32;
  const int ye = f32out ? 4 : 2;
  if (a->x.dtype != DCVC_BF16 || (a->y.dtype != DCVC_BF16 && !f32out)) return DCVC_HIP_EUNSUPPORTED;
  if (a->act != DCVC_ACT_NONE && a->act != DCVC_ACT_LRELU) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && a->in_op != DCVC_IN_LRELU) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.cstride % 8 || a->x.coff % 8 || ((uintptr_t)a->x.ptr & 15)) return DCVC_HIP_EUNSUPPORTED;
  if (a->y.cstride % 8 || a->y.coff % 8 || ((uintptr_t)a->y.ptr & 15) || a->cout % 8) return DCVC_HIP_EUNSUPPORTED;
  for (const dcvc_tensor *r : {&a->res, &a->res2})
    if (r->ptr && (r->dtype != a->y.dtype || r->cstride % 8 || r->coff % 8 || ((uintptr_t)r->ptr & 15) ||
                   (int64_t)r->H * r->W * r->cstride * ye >= ((int64_t)1 << 31) - 64))
      return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)a->x.H * a->x.W * a->x.cstride * 2 >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)a->y.H * a->y.W * a->y.cstride * ye >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  P3 p{};
  p.x = reinterpret_cast<const uint16_t *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.cinp = (a->cin + 31) / 32 * 32;
  p.bias = a->bias;
  p.scale = a->scale;
  p.y = a->y.ptr;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.Wout = a->y.W;
  if (a->res.ptr) {
    p.res = a->res.ptr;
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
    p.rbytes = a->res.H * a->res.W * a->res.cstride * ye;
  }
  if (a->res2.ptr) {
    p.res2 = a->res2.ptr;
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
    p.r2bytes = a->res2.H * a->res2.W * a->res2.cstride * ye;
  }
  p.xbytes = a->x.H * a->x.W * a->x.cstride * 2;
  p.ybytes = a->y.H * a->y.W * a->y.cstride * ye;
  p.cout = a->cout;
  p.in_lrelu = a->in_op == DCVC_IN_LRELU;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  const bool shuf = a->shuffle != 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (a->cin) {
    case 32: return pick_bn<32>(p, f32out, shuf, st);
    case 48: return pick_bn<48>(p, f32out, shuf, st);
    case 64: return pick_bn<64>(p, f32out, shuf, st);
    case 80: return pick_bn<80>(p, f32out, shuf, st);
    case 96: return pick_bn<96>(p, f32out, shuf, st);
    case 128: return pick_bn<128>(p, f32out, shuf, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}

// dcvc_set_option("conv3x3_persistent", 0/1) (A/B switch, via conv.hip)
extern "C" void dcvc_internal_conv3p_enable(int v) { g_enabled = v; }
extern "C" void dcvc_internal_conv3p_occupancy(int v) { g_occ = v; }
extern "C" void dcvc_internal_conv3p_mode(int v) { g_mode = v; }
extern "C" void dcvc_internal_conv3p_rows4(int v) { g_rows4 = v; }
