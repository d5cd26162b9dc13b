// Split-fp16 ("f16x3", sconv.hip's header) 3x3 stride-1 convolution with the
// image operand taken straight from global memory into registers.
//
// Why: sconv.hip stages each 32-channel chunk of a halo tile through a
// shared LDS image (split on the way in), so every chunk costs the
// workgroup two barriers, a publish phase in which no MFMA runs, and a
// global prefetch only one chunk ahead; measured on the 48->48 1080p layer
// (PMC, r03o): MFMA busy ~30 %, 42 % of wave cycles waiting, ~38k VALU per
// wave.  Here the waves of a workgroup share nothing but the resident
// weights, so after the one-time weight load there is no barrier at all:
//   * a workgroup (8 waves, two per SIMD) keeps the packed split weights of
//     one n-block of BN = 16 NT output channels resident in LDS (every chunk
//     and tap, sconv.hip's resident layout and swizzle) plus bias | scale;
//   * a wave owns output tiles of RW rows x 16 columns x BN channels
//     (RW x NT x 2 f32x4 accumulators) and walks them persistently;
//   * the K walk of a tile goes chunk by chunk (32 input channels); inside a
//     full chunk the order is (dx, input row i, dy): lane (col, hi) loads
//     the fp32 channels [8 hi, 8 hi + 8) of input pixel (oy0 + i - 1,
//     ox0 + col + dx - 1) -- one "piece", two 16-byte buffer loads (out-of-
//     range offsets read zeros: the zero padding, channels past cin) --
//     splits it once into the (hi, lo) f16x8 B operands and uses it for
//     every output row r = i - dy: 3 (RW + 2) pieces per chunk instead of
//     9 RW, and the weights of one dx (3 dy x NT x hi/lo) sit in registers
//     for the whole column of input rows;
//   * a chunk with 16 or 8 valid channels (cin = 48, 80, ...) packs 2 or 4
//     taps into one 32-deep K step (dcvc_conv_pack_weights packs the weights
//     the same way): lane group hi loads its own tap's pixel;
//   * pieces are loaded two items ahead of their use, across chunk and tile
//     boundaries, into a 2-slot register ring (item counts are even, so the
//     slot of every item is a compile-time constant);
//   * the epilogue runs straight from the accumulators: out = scale * (res2 +
//     (res + act(acc + bias))) in the reference's order (sconv.hip's direct
//     epilogue), 16-byte buffer loads / stores.
// The products and their fp32 accumulation are the split of sconv.hip; only
// the order in which the taps reach an accumulator differs.
#include "common.h"
#include "split.h"

#include <cstring>
#include <type_traits>
#include <utility>

namespace {

struct RP {
  const float *x;
  int H, W, xcs, xco;
  int xbytes;              // bytes of the input buffer from x (buffer descriptor range)
  const uint16_t *w;       // split weights (dcvc_conv_pack_weights, DCVC_F16X3)
  int wbytes;
  int64_t wchunk;          // halves of one full chunk's packed weights (hi + lo)
  const float *bias;
  const float *scale;
  float *y;
  int ycs, yco, ybytes;
  const float *res;
  int rcs, rco, rbytes;
  const float *res2;
  int r2cs, r2co, r2bytes;
  int cin, cout, nchunks, nfull, tpk_last, wrows;
  int in_lrelu;
  float in_slope;
  int act;
  float slope;
  int tiles_x, nsp, nblk;  // spatial tiles, n-blocks
};

constexpr int kOob = 0x7fffffe0;   // a buffer offset past any range: loads read zeros, stores are dropped

template <int NT>
struct RL {
  static constexpr int BN = NT * 16;
  static constexpr size_t WROW = (size_t)BN * 32 * 2 * 2;   // bytes of one weight row of the n-block (hi + lo)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}

template <int NT, int RW, int NRES, int kNW>
__global__ void __launch_bounds__(kNW * 64) sconvr_kernel(RP p) {
  constexpr int BN = NT * 16;
  constexpr int NI = RW + 2;       // input rows of a tile
  static_assert(RW % 2 == 0, "item counts must be even (2-slot ring)");
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Lw = reinterpret_cast<uint16_t *>(smem);
  float *Lc = reinterpret_cast<float *>(smem + (size_t)p.wrows * RL<NT>::WROW);   // bias | scale

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  int g = blockIdx.x;
  // consecutive workgroups on one XCD (dealt round robin): the n-blocks of a
  // spatial group, and neighbouring spatial groups, share that XCD's L2
  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);
  const int nb = g % p.nblk;
  const int n0 = nb * BN;
  const int sgroups = G / p.nblk;
  const int s0 = (g / p.nblk) * kNW + wave;
  const int sstride = sgroups * kNW;

  // resident weights of n-block n0 by LDS-DMA: flattened row R = (chunk row)
  // * BN + nn, 1-KiB pieces of 16 rows (sconv.hip's load_resident)
  {
    const __amdgpu_buffer_rsrc_t wr = rsrc(p.w, p.wbytes);
    const int nd = 2 * p.wrows * BN / 16;
    for (int i = wave; i < nd; i += kNW) {
      const int hl = i >= nd / 2, k = hl ? i - nd / 2 : i;
      const int R = k * 16 + (lane >> 2);
      const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
      const int cr = R / BN, nn = R - cr * BN;
      int c = cr / 9;
      if (c > p.nchunks - 1) c = p.nchunks - 1;
      const int r = cr - c * 9;
      const int rows = c == p.nchunks - 1 ? (9 + p.tpk_last - 1) / p.tpk_last : 9;
      const int n = n0 + nn;
      int voff = kOob;
      if (n < p.cout)
        voff = (int)(((int64_t)c * p.wchunk + (hl ? (int64_t)rows * p.cout * 32 : 0) + ((int64_t)r * p.cout + n) * 32 +
                      ls * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (__attribute__((address_space(3))) void *)(Lw + (size_t)hl * p.wrows * BN * 32 + k * 512), 16, voff, 0, 0,
          0);
    }
    for (int i = threadIdx.x; i < BN; i += kNW * 64) {
      const int n = n0 + i;
      Lc[i] = (p.bias && n < p.cout) ? p.bias[n] : 0.f;
      Lc[BN + i] = (p.scale && n < p.cout) ? p.scale[n] : 1.f;
    }
    wait_vm_lgkm();
    __syncthreads();
  }
  const uint16_t *Lwl = Lw + (size_t)p.wrows * BN * 32;

  const __amdgpu_buffer_rsrc_t xr = rsrc(p.x + p.xco, p.xbytes);
  const int H = p.H, W = p.W, xcs = p.xcs, cin = p.cin;

  // piece loads: lane's fp32 channels [ch, ch + 8) of input pixel (iy, ix)
  auto ld = [&](float (&d)[8], int iy, int ix, int ch) {
    const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W && ch < cin;
    const int o = ok ? ((iy * W + ix) * xcs + ch) * 4 : kOob;
    const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
    const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d[j] = a[j];
      d[4 + j] = b[j];
    }
  };
  auto origin = [&](int s, int &oy0, int &ox0) {
    const int ty = s / p.tiles_x;
    oy0 = ty * RW;
    ox0 = (s - ty * p.tiles_x) * 16;
  };
  // item m of a full chunk c: (dx, i) = (m / NI, m % NI)
  auto ld_full = [&](float (&d)[8], int oy0, int ox0, int c, int m) {
    const int dx = m / NI, i = m - dx * NI;
    ld(d, oy0 + i - 1, ox0 + col + dx - 1, c * 32 + 8 * hi);
  };
  // item m = s * RW + r of the tail chunk c (TPK taps per K step)
  auto ld_tail = [&](float (&d)[8], int oy0, int ox0, int c, int m, int tpk) {
    const int s = m / RW, r = m - s * RW;
    const int spt = 4 / tpk;
    const int tap = s * tpk + hi / spt, slot = hi - (hi / spt) * spt;
    const int dy = tap / 3, dx = tap - dy * 3;
    if (tap < 9) ld(d, oy0 + r + dy - 1, ox0 + col + dx - 1, c * 32 + 8 * slot);
    else ld(d, -1, 0, 0);
  };
  // item m' (0 or 1) of the chunk after chunk c of tile s
  auto ld_next = [&](float (&d)[8], int s, int c, int mp) {
    int cn = c + 1;
    if (cn == p.nchunks) {
      cn = 0;
      s += sstride;
    }
    if (s >= p.nsp) {
      ld(d, -1, 0, 0);
      return;
    }
    int oy0, ox0;
    origin(s, oy0, ox0);
    if (cn < p.nfull) ld_full(d, oy0, ox0, cn, mp);
    else ld_tail(d, oy0, ox0, cn, mp, p.tpk_last);
  };

  float raw[2][8];
  f32x4 am[RW][NT], ac[RW][NT];
  const float slope_in = p.in_slope;
  const bool lrelu = p.in_lrelu != 0;
  auto split_piece = [&](const float (&v0)[8], f16x8 &bh, f16x8 &bl) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lrelu ? (v0[e] >= 0.f ? v0[e] : v0[e] * slope_in) : v0[e];
    u32x4_t h, l;
    split8(v, h, l);
    bh = __builtin_bit_cast(f16x8, h);
    bl = __builtin_bit_cast(f16x8, l);
  };
  auto mma = [&](f32x4 &m, f32x4 &cc, const f16x8 &wh, const f16x8 &wl, const f16x8 &bh, const f16x8 &bl) {
    m = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, m, 0, 0, 0);
    cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, cc, 0, 0, 0);
    cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, cc, 0, 0, 0);
  };

  // a full chunk: (dx, i, dy) order, weights of one dx in registers
  auto full_chunk = [&](int s, int oy0, int ox0, int c) {
#pragma unroll 1
    for (int dx = 0; dx < 3; ++dx) {
      f16x8 wh[3][NT], wl[3][NT];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int o = swz((c * 9 + dy * 3 + dx) * BN + j * 16 + col, hi);
          wh[dy][j] = *reinterpret_cast<const f16x8 *>(Lw + o);
          wl[dy][j] = *reinterpret_cast<const f16x8 *>(Lwl + o);
        }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        // (NI is even: item dx * NI + i uses slot i & 1)
        f16x8 bh, bl;
        split_piece(raw[i & 1], bh, bl);
        if (i + 2 < NI) ld_full(raw[i & 1], oy0, ox0, c, dx * NI + i + 2);
        else if (dx < 2) ld_full(raw[i & 1], oy0, ox0, c, (dx + 1) * NI + i + 2 - NI);
        else ld_next(raw[i & 1], s, c, i + 2 - NI);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const int r = i - dy;
          if (r < 0 || r >= RW) continue;
#pragma unroll
          for (int j = 0; j < NT; ++j) mma(am[r][j], ac[r][j], wh[dy][j], wl[dy][j], bh, bl);
        }
      }
    }
  };
  // the tail chunk: NK = ceil(9 / TPK) K steps, (s, r) order
  auto tail_chunk = [&](auto tpkc, int s, int oy0, int ox0, int c) {
    constexpr int TPK = decltype(tpkc)::value;
    constexpr int NK = (9 + TPK - 1) / TPK;
    constexpr int NTI = NK * RW;
#pragma unroll 1
    for (int k = 0; k < NK; ++k) {
      f16x8 wh[NT], wl[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int o = swz((c * 9 + k) * BN + j * 16 + col, hi);
        wh[j] = *reinterpret_cast<const f16x8 *>(Lw + o);
        wl[j] = *reinterpret_cast<const f16x8 *>(Lwl + o);
      }
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        // (RW is even: item k * RW + r uses slot r & 1)
        const int m = k * RW + r;
        f16x8 bh, bl;
        split_piece(raw[r & 1], bh, bl);
        if (m + 2 < NTI) ld_tail(raw[r & 1], oy0, ox0, c, m + 2, TPK);
        else ld_next(raw[r & 1], s, c, m + 2 - NTI);
#pragma unroll
        for (int j = 0; j < NT; ++j) mma(am[r][j], ac[r][j], wh[j], wl[j], bh, bl);
      }
    }
  };

  const __amdgpu_buffer_rsrc_t yr = rsrc(p.y + p.yco, p.ybytes);
  const __amdgpu_buffer_rsrc_t rr = rsrc(NRES >= 1 ? p.res + p.rco : p.y, NRES >= 1 ? p.rbytes : 0);
  const __amdgpu_buffer_rsrc_t r2r = rsrc(NRES >= 2 ? p.res2 + p.r2co : p.y, NRES >= 2 ? p.r2bytes : 0);

  // prologue: the first two items of the wave's first tile
  if (s0 < p.nsp) {
    int oy0, ox0;
    origin(s0, oy0, ox0);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (p.nfull > 0) ld_full(raw[m], oy0, ox0, 0, m);
      else ld_tail(raw[m], oy0, ox0, 0, m, p.tpk_last);
    }
  }
  for (int s = s0; s < p.nsp; s += sstride) {
    int oy0, ox0;
    origin(s, oy0, ox0);
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        am[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ac[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    for (int c = 0; c < p.nfull; ++c) full_chunk(s, oy0, ox0, c);
    if (p.nfull < p.nchunks) {
      if (p.tpk_last == 2) tail_chunk(std::integral_constant<int, 2>{}, s, oy0, ox0, p.nfull);
      else tail_chunk(std::integral_constant<int, 4>{}, s, oy0, ox0, p.nfull);
    }

    // epilogue: lane (col, hi) of fragment (r, j) holds output channels
    // n0 + 16 j + 4 hi .. + 3 of pixel (oy0 + r, ox0 + col)
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int oy = oy0 + r, ox = ox0 + col;
      const bool okp = oy < H && ox < W;
      const int pix = oy * W + ox;
      f32x4 r1[NT], r2[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + j * 16 + hi * 4;
        const bool ok = okp && n < p.cout;
        if constexpr (NRES >= 1)
          r1[j] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, ok ? (pix * p.rcs + n) * 4 : kOob, 0, 0));
        if constexpr (NRES >= 2)
          r2[j] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(r2r, ok ? (pix * p.r2cs + n) * 4 : kOob, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int nl = j * 16 + hi * 4, n = n0 + nl;
        const float4 bb = *reinterpret_cast<const float4 *>(Lc + nl);
        f32x4 v;
        v[0] = (am[r][j][0] + ac[r][j][0] * kLoInv) + bb.x;
        v[1] = (am[r][j][1] + ac[r][j][1] * kLoInv) + bb.y;
        v[2] = (am[r][j][2] + ac[r][j][2] * kLoInv) + bb.z;
        v[3] = (am[r][j][3] + ac[r][j][3] * kLoInv) + bb.w;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_act(p.act, v[e], p.slope);
        if constexpr (NRES >= 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = r1[j][e] + v[e];
        }
        if constexpr (NRES >= 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = r2[j][e] + v[e];
        }
        if (p.scale) {
          const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + nl);
          v[0] *= sc.x;
          v[1] *= sc.y;
          v[2] *= sc.z;
          v[3] *= sc.w;
        }
        const bool ok = okp && n < p.cout;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), yr, ok ? (pix * p.ycs + n) * 4 : kOob,
                                               0, 0);
      }
    }
  }
}

int g_enable = 0;   // dcvc_set_option("sconvr", 1): route the 3x3 stride-1 layers here (A/B; off: sconv.hip)
int g_cus = 0;
int g_force_nt = 0; // dcvc_set_option("sconvr_nt", 1..4): force the n-block width (tests / A/B)

int g_waves = 4;   // dcvc_set_option("sconvr_waves", 4 | 8): waves per workgroup (one or two per SIMD)

template <int NT, int RW, int NRES, int kNW>
int launch(RP p, hipStream_t st) {
  constexpr int BN = NT * 16;
  p.nblk = (p.cout + BN - 1) / BN;
  const size_t lds = (size_t)p.wrows * RL<NT>::WROW + 2 * BN * 4;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  p.tiles_x = (p.W + 15) / 16;
  const int64_t nsp = (int64_t)p.tiles_x * ((p.H + RW - 1) / RW);
  if (nsp <= 0) return DCVC_HIP_OK;
  if (nsp * p.nblk > 0x7fffffff) return DCVC_HIP_EINVAL;
  p.nsp = (int)nsp;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  // one workgroup per CU; the grid is a multiple of the n-block count (a
  // workgroup keeps one n-block) and needs no more spatial groups than tiles
  int64_t groups = g_cus / p.nblk;
  if (groups < 1) groups = 1;
  const int64_t need = (nsp + kNW - 1) / kNW;
  if (groups > need) groups = need;
  const int64_t G = groups * p.nblk;
  auto kern = sconvr_kernel<NT, RW, NRES, kNW>;
  dcvc_note_kernel("sconvr_kernel<%d, %d, %d, %d>@%lld", NT, RW, NRES, kNW, (long long)G * kNW * 64);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(kNW * 64), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

template <int NT, int RW, int NW>
int launch_res(RP p, int nres, hipStream_t st) {
  switch (nres) {
    case 0: return launch<NT, RW, 0, NW>(p, st);
    case 1: return launch<NT, RW, 1, NW>(p, st);
    default: return launch<NT, RW, 2, NW>(p, st);
  }
}

// tile rows per wave by n-block width and waves per workgroup: the
// accumulators (RW x NT x 8 registers), the weights of one dx (24 NT) and the
// piece ring within 512 (one wave per SIMD) or 256 (two) registers
int launch_nt(RP p, int nt, int nres, hipStream_t st) {
  if (g_waves == 8) {
    switch (nt) {
      case 1: return launch_res<1, 8, 8>(p, nres, st);
      case 2: return launch_res<2, 6, 8>(p, nres, st);
      case 3: return launch_res<3, 4, 8>(p, nres, st);
      case 4: return launch_res<4, 2, 8>(p, nres, st);
      default: return DCVC_HIP_EUNSUPPORTED;
    }
  }
  switch (nt) {
    case 1: return launch_res<1, 8, 4>(p, nres, st);
    case 2: return launch_res<2, 8, 4>(p, nres, st);
    case 3: return launch_res<3, 6, 4>(p, nres, st);
    case 4: return launch_res<4, 4, 4>(p, nres, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}

}  // namespace

extern "C" void dcvc_internal_sconv_dbg(int v);
extern "C" void dcvc_internal_sconv_rw(int v);

// options of the split-precision kernels (dcvc_set_option falls through to
// here, so adding one does not rebuild conv.hip)
extern "C" int dcvc_internal_set_option_split(const char *name, int value) {
  if (std::strcmp(name, "sconvr") == 0) g_enable = value;
  else if (std::strcmp(name, "sconvr_nt") == 0) g_force_nt = value;
  else if (std::strcmp(name, "sconvr_waves") == 0) g_waves = value;
  else if (std::strcmp(name, "sconv_dbg") == 0) dcvc_internal_sconv_dbg(value);
  else if (std::strcmp(name, "sconv_rw") == 0) dcvc_internal_sconv_rw(value);
  else return DCVC_HIP_EINVAL;
  return DCVC_HIP_OK;
}

// f16x3 3x3 stride-1 pad-1 convolutions that sconv.hip hands over: fp32
// 8-channel aligned input, no pixel shuffle, no gate, 16-byte output pieces,
// the packed weights of one n-block resident in LDS.  DCVC_HIP_EUNSUPPORTED
// sends the call back to sconv.hip.
extern "C" int dcvc_internal_sconvr(const dcvc_conv_args *a, void *stream) {
  if (!g_enable) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1 || a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && a->in_op != DCVC_IN_LRELU) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.H != a->y.H || a->x.W != a->y.W) return DCVC_HIP_EUNSUPPORTED;
  if ((a->res.ptr && a->res.dtype != DCVC_F32) || (a->res2.ptr && a->res2.dtype != DCVC_F32))
    return DCVC_HIP_EUNSUPPORTED;
  auto al = [](const void *ptr, int cs, int co) {
    return ptr == nullptr || ((uintptr_t)ptr % 16 == 0 && cs % 4 == 0 && co % 4 == 0);
  };
  if (a->cin % 8 || a->cout % 4 || !al(a->x.ptr, a->x.cstride, a->x.coff) || !al(a->y.ptr, a->y.cstride, a->y.coff) ||
      !al(a->res.ptr, a->res.cstride, a->res.coff) || !al(a->res2.ptr, a->res2.cstride, a->res2.coff))
    return DCVC_HIP_EUNSUPPORTED;
  // one buffer descriptor per tensor: 32-bit byte offsets
  const int64_t npix = (int64_t)a->x.H * a->x.W;
  auto bytes = [&](int cs, int co) { return (npix * cs - co) * 4; };
  const int64_t lim = 0x7fff0000;
  if (bytes(a->x.cstride, a->x.coff) > lim || bytes(a->y.cstride, a->y.coff) > lim ||
      (a->res.ptr && bytes(a->res.cstride, a->res.coff) > lim) ||
      (a->res2.ptr && bytes(a->res2.cstride, a->res2.coff) > lim))
    return DCVC_HIP_EUNSUPPORTED;
  if (npix <= 0) return DCVC_HIP_OK;
  RP p{};
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.xbytes = (int)bytes(a->x.cstride, a->x.coff);
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.bias = a->bias;
  p.scale = a->scale;
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.ybytes = (int)bytes(a->y.cstride, a->y.coff);
  int nres = 0;
  if (a->res.ptr) {
    p.res = reinterpret_cast<const float *>(a->res.ptr);
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
    p.rbytes = (int)bytes(a->res.cstride, a->res.coff);
    nres = 1;
  }
  if (a->res2.ptr) {
    if (!a->res.ptr) return DCVC_HIP_EUNSUPPORTED;
    p.res2 = reinterpret_cast<const float *>(a->res2.ptr);
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
    p.r2bytes = (int)bytes(a->res2.cstride, a->res2.coff);
    nres = 2;
  }
  p.cin = a->cin;
  p.cout = a->cout;
  p.nchunks = (a->cin + 31) / 32;
  const int vc = a->cin - 32 * (p.nchunks - 1);
  p.tpk_last = vc <= 8 ? 4 : vc <= 16 ? 2 : 1;
  p.nfull = p.tpk_last == 1 ? p.nchunks : p.nchunks - 1;
  p.wrows = (p.nchunks - 1) * 9 + (9 + p.tpk_last - 1) / p.tpk_last;
  p.wchunk = (int64_t)2 * 9 * a->cout * 32;
  {
    const int64_t wb = ((int64_t)(p.nchunks - 1) * p.wchunk + (int64_t)2 * ((9 + p.tpk_last - 1) / p.tpk_last) *
                                                                 a->cout * 32) * 2;
    if (wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
    p.wbytes = (int)wb;
  }
  p.in_lrelu = a->in_op == DCVC_IN_LRELU;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (g_force_nt) return launch_nt(p, g_force_nt, nres, st);
  // n-block width: fewest padded output channels, then the widest whose
  // resident weights fit the LDS
  int order[4] = {4, 3, 2, 1};
  auto padded = [&](int nt) { return (a->cout + 16 * nt - 1) / (16 * nt) * (16 * nt) - a->cout; };
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 4; ++j)
      if (padded(order[j]) < padded(order[i])) std::swap(order[i], order[j]);
  for (int i = 0; i < 4; ++i) {
    const int r = launch_nt(p, order[i], nres, st);
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  return DCVC_HIP_EUNSUPPORTED;
}
