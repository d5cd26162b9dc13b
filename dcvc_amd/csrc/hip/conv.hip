// NHWC implicit-GEMM convolution on gfx950 MFMA.
//
// One workgroup = 4 waves (256 threads) computes an output tile of TH rows x
// 16 columns x BN channels.  The GEMM is D[n][pixel] = W[n][k] * X[k][pixel]
// with k = (tap, input channel); the output channel is the MFMA row so each
// lane ends with 4 consecutive channels of one pixel (NHWC-friendly stores).
//
// K is walked in chunks of 32 input channels.  Per chunk the input tile
// (rows (TH-1)*S+KH, cols 15*S+KW, 32 channels) is staged once into LDS with
// the input transform applied (lrelu / ConvFFN2 gate) and converted to the
// compute type; weights are staged per kernel row (KW taps x BN x 32).  Every
// (dy, dx) tap then reuses the same LDS image: the LDS-staged im2col of the
// design.  bf16 mode issues v_mfma_f32_16x16x32_bf16 with an XOR-swizzled LDS
// image (16-byte slots, conflict-free ds_read_b128 lane groups for aligned
// rows); f32 mode issues v_mfma_f32_16x16x4_f32 (exact f32 fma chain) from a
// padded image.  The epilogue fuses bias, activation, up to two residual adds,
// a per-channel scale and pixel-shuffle, in the order the reference applies
// them (see dcvc_conv_args in include/dcvc_hip.h).
#include "common.h"
#include "epilogue.h"
#include "split.h"

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unordered_map>

static thread_local char g_last_kernel[192];

void dcvc_ensure_lds(const void *kern, int bytes) {
  static std::mutex mu;
  static std::unordered_map<const void *, int> done;
  std::lock_guard<std::mutex> lk(mu);
  int &have = done[kern];
  if (have >= bytes) return;
  (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  have = bytes;
}

void dcvc_note_kernel(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_kernel, sizeof(g_last_kernel), fmt, ap);
  va_end(ap);
}

extern "C" const char *dcvc_last_kernel(void) { return g_last_kernel; }

namespace {

constexpr int kChunk = 32;  // input channels per K chunk

struct ConvP {
  const void *x;
  int H, W, xcs, xco;
  const void *w;
  const float *bias;
  void *y;
  int Ho, Wo, ycs, yco;  // conv output size (before shuffle)
  int cin, cout, cinp;
  int kh, kw, s, pad;
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
  int Wout;  // width of y buffer (after shuffle)
  int tiles_x, tiles_y;
  int vec;      // 16-byte input staging allowed (channel alignment)
  int vec_out;  // 8-channel vector epilogue allowed (alignment)
  int lc_off;   // LDS byte offset of the epilogue constants (bias, scale)
  int wall;     // stage all kernel rows' weights per chunk
};

// LDS image helpers ---------------------------------------------------------
// bf16: a "row" is 32 channels = 64 B = 4 slots of 16 B; slot is swizzled.
// slot XOR {0, 2, 3, 1}[(row >> 2) & 3], as a nibble table in a register
__device__ __forceinline__ int swz_off_bf16(int row, int slot) {
  const int x = (0x1320 >> (((row >> 2) & 3) << 2)) & 3;
  return row * 32 + ((slot ^ x) << 3);  // in bf16 elements
}
// f32: a row is 32 floats padded to 34, so an operand read (ds_read_b32 of 16
// consecutive rows at k..k+3, 32-lane halves) lands on banks (2 row + hi) % 32:
// conflict-free (a pad to 33 put rows r and r + 1 of different k on one bank)
constexpr int kF32Row = 34;
__device__ __forceinline__ int off_f32(int row, int k) { return row * kF32Row + k; }

template <typename TIN>
__device__ __forceinline__ float load_in(const ConvP &p, int gy, int gx, int c) {
  const int64_t base = ((int64_t)gy * p.W + gx) * p.xcs + p.xco;
  float v = ld<TIN>(p.x, base + c);
  if (p.in_op == DCVC_IN_LRELU) {
    v = v >= 0.f ? v : v * p.in_slope;
  } else if (p.in_op == DCVC_IN_GATE) {
    float g = ld<TIN>(p.x, base + c + p.cin);
    g = g >= 0.f ? g : g * p.in_slope;
    v = v * g;
  }
  return v;
}

// 8 consecutive input channels starting at element offset e (16-byte aligned)
__device__ __forceinline__ void load8(const float *x, int64_t e, float v[8]) {
  const float4 a = *reinterpret_cast<const float4 *>(x + e);
  const float4 b = *reinterpret_cast<const float4 *>(x + e + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const uint16_t *x, int64_t e, float v[8]) {
  const u16x8 a = *reinterpret_cast<const u16x8 *>(x + e);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
}

// Input tile staging.  One work item = one pixel x 8 channels (a 16-byte LDS
// slot).  Items are processed in groups of kU per thread: all kU global loads
// are issued before any LDS store, so kU loads are in flight per thread.
constexpr int kU = 4;

template <typename TIN, bool F32>
__device__ __forceinline__ void stage_input(const ConvP &p, void *lds_in, int ch0,
                                            int iy0, int ix0, int IH, int IW,
                                            int IWp) {
  const int items = IH * IW * 4;
  const TIN *X = reinterpret_cast<const TIN *>(p.x);
  // bf16 -> bf16 with no input transform: move the raw 16-byte pieces
  constexpr bool kRawOk = !F32 && sizeof(TIN) == 2;
  const bool raw = kRawOk && p.vec && p.in_op == DCVC_IN_NONE;
  for (int base = threadIdx.x; base < items; base += 256 * kU) {
    float v[kU][8];
    u16x8 rv[kU];
    int rows[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int it = base + u * 256;
      rows[u] = -1;
      if (it >= items) continue;
      const int slot = it & 3;
      const int pix = it >> 2;
      const int iy = pix / IW, ix = pix - iy * IW;
      const int gy = iy0 + iy, gx = ix0 + ix;
      const int c0 = ch0 + slot * 8;
      rows[u] = (iy * IWp + ix) * 4 + slot;
      const bool inb = gy >= 0 && gy < p.H && gx >= 0 && gx < p.W && c0 < p.cin;
      if constexpr (kRawOk) {
        if (raw) {
          const int64_t e = ((int64_t)gy * p.W + gx) * p.xcs + p.xco + c0;
          if (inb) {
            rv[u] = *reinterpret_cast<const u16x8 *>(reinterpret_cast<const uint16_t *>(X) + e);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) rv[u][j] = 0;
          }
          continue;
        }
      }
      if (p.vec) {
        if (inb) {
          const int64_t e = ((int64_t)gy * p.W + gx) * p.xcs + p.xco + c0;
          load8(X, e, v[u]);
          if (p.in_op == DCVC_IN_GATE) {
            float g[8];
            load8(X, e + p.cin, g);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[u][j] = v[u][j] * (g[j] >= 0.f ? g[j] : g[j] * p.in_slope);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] = 0.f;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = c0 + j;
          v[u][j] = (inb && c < p.cin) ? load_in<TIN>(p, gy, gx, c) : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (rows[u] < 0) continue;
      const int row = rows[u] >> 2, slot = rows[u] & 3;
      if constexpr (kRawOk) {
        if (raw) {
          *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(lds_in) + swz_off_bf16(row, slot)) = rv[u];
          continue;
        }
      }
      if (p.vec && p.in_op == DCVC_IN_LRELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] = v[u][j] >= 0.f ? v[u][j] : v[u][j] * p.in_slope;
      }
      if constexpr (F32) {
        float *L = reinterpret_cast<float *>(lds_in);
#pragma unroll
        for (int j = 0; j < 8; ++j) L[off_f32(row, slot * 8 + j)] = v[u][j];
      } else {
        u16x8 pk;
#pragma unroll
        for (int j = 0; j < 8; ++j) pk[j] = f2bf(v[u][j]);
        *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(lds_in) + swz_off_bf16(row, slot)) = pk;
      }
    }
  }
}

// Stage weights of kernel rows [dy0, dy0 + ndy) of one channel chunk; LDS
// row index = ((dy - dy0) * kw + dx) * BN + n.  Batched like stage_input.
template <bool F32, int BN>
__device__ __forceinline__ void stage_weights(const ConvP &p, void *lds_w, int n0,
                                              int chunk, int dy0, int ndy) {
  const int items = ndy * p.kw * BN * 4;  // 8-channel pieces
  for (int base = threadIdx.x; base < items; base += 256 * kU) {
    int rrs[kU];
    if constexpr (F32) {
      float4 va[kU], vb[kU];
      const float *W = reinterpret_cast<const float *>(p.w);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int it = base + u * 256;
        rrs[u] = -1;
        if (it >= items) continue;
        const int slot = it & 3, rr = it >> 2;
        const int tap = rr / BN, nn = rr - tap * BN;
        const int n = n0 + nn;
        rrs[u] = it;
        if (n < p.cout) {
          const int64_t src = (((int64_t)n * p.kh + dy0 + tap / p.kw) * p.kw + tap % p.kw) * p.cinp +
                              chunk * kChunk + slot * 8;
          va[u] = *reinterpret_cast<const float4 *>(W + src);
          vb[u] = *reinterpret_cast<const float4 *>(W + src + 4);
        } else {
          va[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          vb[u] = va[u];
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (rrs[u] < 0) continue;
        float *d = reinterpret_cast<float *>(lds_w) + off_f32(rrs[u] >> 2, (rrs[u] & 3) * 8);
        d[0] = va[u].x; d[1] = va[u].y; d[2] = va[u].z; d[3] = va[u].w;
        d[4] = vb[u].x; d[5] = vb[u].y; d[6] = vb[u].z; d[7] = vb[u].w;
      }
    } else {
      u16x8 v[kU];
      const uint16_t *W = reinterpret_cast<const uint16_t *>(p.w);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int it = base + u * 256;
        rrs[u] = -1;
        if (it >= items) continue;
        const int slot = it & 3, rr = it >> 2;
        const int tap = rr / BN, nn = rr - tap * BN;
        const int n = n0 + nn;
        rrs[u] = it;
        if (n < p.cout) {
          const int64_t src = (((int64_t)n * p.kh + dy0 + tap / p.kw) * p.kw + tap % p.kw) * p.cinp +
                              chunk * kChunk + slot * 8;
          v[u] = *reinterpret_cast<const u16x8 *>(W + src);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] = 0;
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (rrs[u] < 0) continue;
        *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(lds_w) + swz_off_bf16(rrs[u] >> 2, rrs[u] & 3)) =
            v[u];
      }
    }
  }
}

template <typename TIN, typename TOUT, bool F32, int BN, int TH>
__global__ void __launch_bounds__(256) conv_kernel(ConvP p) {
  constexpr int RW = TH / 4;   // output rows per wave
  constexpr int NT = BN / 16;  // n tiles per wave
  extern __shared__ __align__(16) unsigned char smem[];

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  int b = blockIdx.x;
  const int tx = b % p.tiles_x;
  b /= p.tiles_x;
  const int ty = b % p.tiles_y;
  const int tn = b / p.tiles_y;
  const int ox0 = tx * 16, oy0 = ty * TH, n0 = tn * BN;

  const int S = p.s;
  const int IH = (TH - 1) * S + p.kh;
  const int IW = 15 * S + p.kw;
  const int IWp = (IW + 3) & ~3;
  const int in_elems = IH * IWp * (F32 ? kF32Row : 32);
  void *lds_in = smem;
  void *lds_w = smem + ((in_elems * (F32 ? 4 : 2) + 15) & ~15);
  float *Lc = reinterpret_cast<float *>(smem + p.lc_off);
  epi::stage_consts(p, Lc, n0, BN);  // published by the chunk loop's first barrier

  f32x4 acc[RW][NT];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = p.cinp / kChunk;
  const int iy0 = oy0 * S - p.pad, ix0 = ox0 * S - p.pad;
  const int col = lane & 15, hi = lane >> 4;
  const int ndy = p.wall ? p.kh : 1;  // kernel rows staged at once

  for (int ch = 0; ch < nchunks; ++ch) {
    __syncthreads();
    stage_input<TIN, F32>(p, lds_in, ch * kChunk, iy0, ix0, IH, IW, IWp);
    for (int dy0 = 0; dy0 < p.kh; dy0 += ndy) {
      if (dy0 > 0) __syncthreads();
      stage_weights<F32, BN>(p, lds_w, n0, ch, dy0, ndy);
      __syncthreads();
      for (int t = 0; t < ndy * p.kw; ++t) {
        const int dy = dy0 + t / p.kw, dx = t % p.kw;
        const int wrow = t * BN;
        if constexpr (F32) {
          const float *Li = reinterpret_cast<const float *>(lds_in);
          const float *Lw = reinterpret_cast<const float *>(lds_w);
#pragma unroll
          for (int s4 = 0; s4 < 8; ++s4) {
            const int k = s4 * 4 + hi;
            float a[NT], bb[RW];
#pragma unroll
            for (int j = 0; j < NT; ++j) a[j] = Lw[off_f32(wrow + j * 16 + col, k)];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
              const int row = ((wave * RW + r) * S + dy) * IWp + col * S + dx;
              bb[r] = Li[off_f32(row, k)];
            }
#pragma unroll
            for (int r = 0; r < RW; ++r)
#pragma unroll
              for (int j = 0; j < NT; ++j)
                acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], bb[r], acc[r][j], 0, 0, 0);
          }
        } else {
          const uint16_t *Li = reinterpret_cast<const uint16_t *>(lds_in);
          const uint16_t *Lw = reinterpret_cast<const uint16_t *>(lds_w);
          bf16x8 a[NT], bb[RW];
#pragma unroll
          for (int j = 0; j < NT; ++j)
            a[j] = *reinterpret_cast<const bf16x8 *>(Lw + swz_off_bf16(wrow + j * 16 + col, hi));
#pragma unroll
          for (int r = 0; r < RW; ++r) {
            const int row = ((wave * RW + r) * S + dy) * IWp + col * S + dx;
            bb[r] = *reinterpret_cast<const bf16x8 *>(Li + swz_off_bf16(row, hi));
          }
#pragma unroll
          for (int r = 0; r < RW; ++r)
#pragma unroll
            for (int j = 0; j < NT; ++j)
              acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], bb[r], acc[r][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue (epilogue.h): fp32 tile in LDS, then coalesced stores
  __syncthreads();
  float *T = reinterpret_cast<float *>(smem);
  constexpr int LD = BN + 4;
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int j = 0; j < NT; ++j)
      epi::put4(p, T, LD, (wave * RW + r) * 16 + col, j * 16 + hi * 4, Lc, acc[r][j]);
  __syncthreads();
  epi::store_tile<TOUT, epi::ipt(TH * 16, BN, 256)>(p, T, LD, TH * 16, n0, min(BN, p.cout - n0), Lc, BN,
                                                     [&](int l, int &oy, int &ox) {
    oy = oy0 + (l >> 4);
    ox = ox0 + (l & 15);
    return oy < p.Ho && ox < p.Wo;
  });
}

template <bool F32, int BN, int TH>
size_t lds_bytes(const ConvP &p, bool wall) {
  const int IH = (TH - 1) * p.s + p.kh;
  const int IW = 15 * p.s + p.kw;
  const int IWp = (IW + 3) & ~3;
  const size_t row = F32 ? kF32Row * 4 : 32 * 2;
  const size_t in_bytes = (size_t)IH * IWp * row;
  const size_t w_bytes = (size_t)(wall ? p.kh : 1) * p.kw * BN * row;
  const size_t stage = ((in_bytes + 15) & ~(size_t)15) + w_bytes;
  const size_t epi = (size_t)TH * 16 * (BN + 4) * 4;  // fp32 output tile
  return stage > epi ? stage : epi;
}

template <typename TIN, typename TOUT, bool F32, int BN, int TH>
int launch(const ConvP &p0, hipStream_t st) {
  ConvP p = p0;
  p.tiles_x = (p.Wo + 15) / 16;
  p.tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles_n = (p.cout + BN - 1) / BN;
  // stage every kernel row's weights at once when that keeps LDS modest
  p.wall = lds_bytes<F32, BN, TH>(p, true) <= 64 * 1024 ? 1 : 0;
  p.lc_off = (int)((lds_bytes<F32, BN, TH>(p, p.wall) + 15) & ~(size_t)15);
  const size_t lds = p.lc_off + epi::consts_floats(BN) * 4;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  const int64_t blocks = (int64_t)p.tiles_x * p.tiles_y * tiles_n;
  if (blocks <= 0) return DCVC_HIP_OK;
  if (blocks > 0x7fffffff) return DCVC_HIP_EINVAL;
  auto kern = conv_kernel<TIN, TOUT, F32, BN, TH>;
  dcvc_note_kernel("conv_kernel<%s, %s, %s, %d, %d>@%lld", tname<TIN>(), tname<TOUT>(), bname(F32), BN, TH,
                   (long long)blocks * 256);
  if (lds > 64 * 1024)
    dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// Tile choice: BN covers Cout in the fewest n-tiles (max 128); TH shrinks
// from 16 (8 when strided) to 4 until the grid has >= 1024 workgroups, so
// the small latent-resolution GEMMs still fill the 256 CUs.
int g_force_th = 0;  // dcvc_set_option("conv_th", 4 | 8 | 16): A/B of the tile height (7x7 convs)
int g_force_bn = 0;  // dcvc_set_option("conv_bn", 16..128): A/B of the n-tile width (7x7 convs)

template <typename TIN, typename TOUT, bool F32, int BN>
int pick_th(const ConvP &p, hipStream_t st) {
  const int64_t tx = (p.Wo + 15) / 16, tn = (p.cout + BN - 1) / BN;
  auto blocks = [&](int th) { return tx * ((p.Ho + th - 1) / th) * tn; };
  int th = (p.s > 1 || BN > 64) ? 8 : 16;
  while (th > 4 && blocks(th) < 1024) th /= 2;
  if (g_force_th && p.kh == 7) th = g_force_th;
  if (th == 16 && BN <= 64 && lds_bytes<F32, BN, 16>(p, false) <= 160 * 1024)
    return launch<TIN, TOUT, F32, BN, 16>(p, st);
  if (th >= 8) return launch<TIN, TOUT, F32, BN, 8>(p, st);
  return launch<TIN, TOUT, F32, BN, 4>(p, st);
}

// BN: the n-tile width (multiple of 16) that wastes the fewest MFMA columns,
// preferring wider tiles on ties; 7x7 kernels stay <= 64 for LDS.
template <typename TIN, typename TOUT, bool F32>
int pick_bn(const ConvP &p, hipStream_t st) {
  static const int cand[6] = {16, 32, 48, 64, 96, 128};
  int best = 16;
  long best_pad = -1;
  for (int i = 0; i < 6; ++i) {
    const int bn = cand[i];
    if (p.kh * p.kw > 9 && bn > 64) continue;
    const long tiles = (p.cout + bn - 1) / bn;
    const long pad = tiles * bn - p.cout;
    if (best_pad < 0 || pad < best_pad || (pad == best_pad && bn > best)) {
      best = bn;
      best_pad = pad;
    }
  }
  // latent-resolution maps (68x120 at 1080p) give few spatial tiles even at
  // TH = 4: split Cout into narrower n-tiles until the grid has >= 2 x 256
  // workgroups (each output channel's sum is unchanged, so results are too)
  {
    const long tiles4 = (long)((p.Wo + 15) / 16) * ((p.Ho + 3) / 4);
    while (best > 32 && tiles4 * ((p.cout + best - 1) / best) < 512) {
      const int nb = best == 96 ? 48 : best / 2;
      if ((p.cout + nb - 1) / nb * nb - p.cout > best_pad) break;  // no extra padding
      best = nb;
    }
  }
  if (g_force_bn && p.kh == 7) best = g_force_bn;
  switch (best) {
    case 16: return pick_th<TIN, TOUT, F32, 16>(p, st);
    case 32: return pick_th<TIN, TOUT, F32, 32>(p, st);
    case 48: return pick_th<TIN, TOUT, F32, 48>(p, st);
    case 64: return pick_th<TIN, TOUT, F32, 64>(p, st);
    case 96: return pick_th<TIN, TOUT, F32, 96>(p, st);
    default: return pick_th<TIN, TOUT, F32, 128>(p, st);
  }
}

int g_use_gemm = 1;   // dcvc_set_option("gemm1x1", 0) routes 1x1 convs to the generic kernel
int g_use_conv3 = 1;  // dcvc_set_option("conv3x3", 0) routes 3x3 s1 convs to the generic kernel

bool valid_view(const dcvc_tensor &t) {
  return t.ptr && t.H > 0 && t.W > 0 && t.C > 0 && t.coff >= 0 && t.coff + t.C <= t.cstride &&
         (t.dtype == DCVC_F32 || t.dtype == DCVC_BF16);
}

}  // namespace

// DCVC_F16X3 layout (sconv.hip): per 32-channel input chunk c, a hi block
// [rows][cout][32] then a lo block of the same shape, chunk c at c * 2 * kt *
// cout * 32 halves.  A chunk with vc <= 16 (<= 8) valid channels packs tpk =
// 2 (4) taps per 32-deep row: k = s * 8 + e holds tap tpk * row + s / (4 /
// tpk), channel 32 c + (s % (4 / tpk)) * 8 + e.  hi = f16(w), lo = f16((w -
// hi) * 2^11): w = hi + 2^-11 lo to ~2^-22.
static int64_t pack_f16x3(const float *w, int cout, int cin, int kh, int kw, uint16_t *out) {
  const int kt = kh * kw;
  const int nch = (cin + 31) / 32;
  const int vcl = cin - 32 * (nch - 1);
  const int tpkl = vcl <= 8 ? 4 : vcl <= 16 ? 2 : 1;
  const int64_t full = (int64_t)2 * kt * cout * 32;
  const int64_t total = (int64_t)(nch - 1) * full + (int64_t)2 * ((kt + tpkl - 1) / tpkl) * cout * 32;
  if (!out) return total;
  for (int c = 0; c < nch; ++c) {
    const int tpk = c == nch - 1 ? tpkl : 1;
    const int spt = 4 / tpk;
    const int rows = (kt + tpk - 1) / tpk;
    uint16_t *hi = out + (int64_t)c * full;
    uint16_t *lo = hi + (int64_t)rows * cout * 32;
    for (int r = 0; r < rows; ++r)
      for (int n = 0; n < cout; ++n)
        for (int k = 0; k < 32; ++k) {
          const int s = k >> 3, e = k & 7;
          const int tap = tpk * r + s / spt;
          const int ch = c * 32 + (s % spt) * 8 + e;
          float v = 0.f;
          if (tap < kt && ch < cin) v = w[(((int64_t)n * cin + ch) * kh + tap / kw) * kw + tap % kw];
          const int64_t o = ((int64_t)r * cout + n) * 32 + k;
          host_split(v, hi[o], lo[o]);
        }
  }
  return total;
}

extern "C" int64_t dcvc_conv_pack_weights(const float *w, int cout, int cin, int kh, int kw,
                                          int compute, void *out) {
  if (!w || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return DCVC_HIP_EINVAL;
  if (compute == DCVC_F16X3) {
    if (out && !host_split_range_ok(w, (int64_t)cout * cin * kh * kw)) return DCVC_HIP_EINVAL;
    return pack_f16x3(w, cout, cin, kh, kw, reinterpret_cast<uint16_t *>(out));
  }
  if (!out) return DCVC_HIP_EINVAL;
  const int cinp = (cin + kChunk - 1) / kChunk * kChunk;
  const int64_t total = (int64_t)cout * kh * kw * cinp;
  for (int n = 0; n < cout; ++n)
    for (int y = 0; y < kh; ++y)
      for (int x = 0; x < kw; ++x)
        for (int c = 0; c < cinp; ++c) {
          const float v = c < cin ? w[(((int64_t)n * cin + c) * kh + y) * kw + x] : 0.f;
          const int64_t o = (((int64_t)n * kh + y) * kw + x) * cinp + c;
          if (compute == DCVC_F32) {
            reinterpret_cast<float *>(out)[o] = v;
          } else {
            // host round-to-nearest-even f32 -> bf16
            uint32_t u;
            std::memcpy(&u, &v, 4);
            uint32_t r = ((u >> 16) & 1u) + 0x7fffu;
            uint16_t h = (uint16_t)((u + r) >> 16);
            if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) h = (uint16_t)((u >> 16) | 0x40);
            reinterpret_cast<uint16_t *>(out)[o] = h;
          }
        }
  return total;
}

extern "C" int dcvc_internal_gemm1x1(const dcvc_conv_args *a, void *stream);
extern "C" int dcvc_internal_gemm1x1_f32(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_gemm1x1_f32_enable(int v);
extern "C" void dcvc_internal_gemm3x3_f32_enable(int v);
extern "C" void dcvc_internal_gemm1x1_f32_cfg(int v);
extern "C" void dcvc_internal_gemm1x1_f32_upfront(int v);
extern "C" void dcvc_internal_gemm1x1_f32_direct(int v);
extern "C" int dcvc_internal_conv3x3(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_conv3x3_resident(int v);
extern "C" void dcvc_internal_conv3p_enable(int v);
extern "C" void dcvc_internal_dcbp_enable(int v);
extern "C" void dcvc_internal_dcbs_enable(int v);
extern "C" int dcvc_internal_conv7s(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_conv7s_enable(int v);
extern "C" int dcvc_internal_conv7w(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_conv7w_enable(int v);
extern "C" int dcvc_internal_conv3s2(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_conv3s2_enable(int v);
extern "C" void dcvc_internal_conv3p_occupancy(int v);
extern "C" void dcvc_internal_conv3p_mode(int v);
extern "C" void dcvc_internal_conv3p_rows4(int v);
extern "C" void dcvc_internal_gemm1x1_bm(int v);
extern "C" int dcvc_internal_sconv(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_sconv_occupancy(int v);
extern "C" void dcvc_internal_sconv_waves(int v);
extern "C" void dcvc_internal_sconv_resident(int v);
extern "C" void dcvc_internal_sconv_res_waves(int v);
extern "C" void dcvc_internal_sgemm_cfg(int v);
extern "C" void dcvc_internal_sgemm_pd(int v);
extern "C" void dcvc_internal_sgemm_gate(int v);
extern "C" int dcvc_internal_set_option_split(const char *name, int value);
extern "C" int dcvc_internal_xconv(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_xconv_enable(int v);
extern "C" int dcvc_internal_wconv(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_wconv_enable(int v);
extern "C" int dcvc_internal_dconv(const dcvc_conv_args *a, void *stream);
extern "C" int dcvc_internal_tconv(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_tconv_enable(int v);
extern "C" int dcvc_internal_nconv(const dcvc_conv_args *a, void *stream);
extern "C" void dcvc_internal_nconv_enable(int v);
extern "C" void dcvc_internal_sffn128(int v);
extern "C" void dcvc_internal_dconv_enable(int v);
extern "C" void dcvc_internal_dconv_1x1(int v);
extern "C" void dcvc_internal_dconv_xcd(int v);
extern "C" void dcvc_internal_dconv_gate(int v);
extern "C" void dcvc_internal_dconv_s2blocks(int v);
extern "C" void dcvc_internal_dconv_bn128(int v);

// fp16 range guard of the split kernels (split.h SplitRange): one flag per
// calling host thread (concurrent GOP lanes each launch from their own thread
// on their own stream)
namespace {
thread_local int *t_split_flag = nullptr;
}
int *dcvc_internal_split_flag() { return t_split_flag; }
extern "C" int dcvc_split_range_flag(int *flag) {
  t_split_flag = flag;
  return DCVC_HIP_OK;
}

extern "C" int dcvc_conv2d(const dcvc_conv_args *a, void *stream) {
  if (!a || !a->w || !valid_view(a->x) || !valid_view(a->y)) return DCVC_HIP_EINVAL;
  if (a->x.C != (a->in_op == DCVC_IN_GATE ? 2 * a->cin : a->cin)) return DCVC_HIP_EINVAL;
  if (a->stride < 1 || a->kh < 1 || a->kw < 1 || a->kh > 7 || a->kw > 7) return DCVC_HIP_EINVAL;
  ConvP p{};
  p.x = a->x.ptr;
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = a->w;
  p.bias = a->bias;
  p.y = a->y.ptr;
  p.Ho = (a->x.H + 2 * a->pad - a->kh) / a->stride + 1;
  p.Wo = (a->x.W + 2 * a->pad - a->kw) / a->stride + 1;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.cinp = (a->cin + kChunk - 1) / kChunk * kChunk;
  p.kh = a->kh;
  p.kw = a->kw;
  p.s = a->stride;
  p.pad = a->pad;
  p.in_op = a->in_op;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.shuffle = a->shuffle;
  p.scale = a->scale;
  const int f = a->shuffle ? 2 : 1;
  const int cy = a->shuffle ? a->cout / 4 : a->cout;
  if (a->shuffle && (a->cout % 4)) return DCVC_HIP_EINVAL;
  if (a->y.H != p.Ho * f || a->y.W != p.Wo * f || a->y.C != cy) return DCVC_HIP_EINVAL;
  p.Wout = a->y.W;
  if (a->res.ptr) {
    if (!valid_view(a->res) || a->res.dtype != a->y.dtype || a->res.H != a->y.H ||
        a->res.W != a->y.W || a->res.C != cy)
      return DCVC_HIP_EINVAL;
    p.res = a->res.ptr;
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
  }
  if (a->res2.ptr) {
    if (!valid_view(a->res2) || a->res2.dtype != a->y.dtype || a->res2.H != a->y.H ||
        a->res2.W != a->y.W || a->res2.C != cy)
      return DCVC_HIP_EINVAL;
    p.res2 = a->res2.ptr;
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
  }
  if (a->compute == DCVC_F16X3) {   // the split-fp16 kernels only
    int r = dcvc_internal_tconv(a, stream);   // 2-channel inputs: fp32 VALU (tconv.hip)
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
    r = dcvc_internal_nconv(a, stream);       // 2- / 3-channel outputs: pixels on M (nconv.hip)
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
    r = dcvc_internal_wconv(a, stream);       // wave-specialised 3x3 stride-1 kernel (wconv.hip)
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
    r = dcvc_internal_xconv(a, stream);       // static-shape 3x3 stride-1 kernel (xconv.hip)
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
    r = dcvc_internal_dconv(a, stream);       // stride 2, feature-rate 1x1: direct operand loads (dconv.hip)
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
    return dcvc_internal_sconv(a, stream);
  }
  if (a->compute != DCVC_F32 && a->compute != DCVC_BF16) return DCVC_HIP_EINVAL;
  if (a->kh == 3 && a->kw == 3 && a->stride == 1 && a->compute == DCVC_BF16 && g_use_conv3) {
    const int r = dcvc_internal_conv3x3(a, stream);
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  if (a->kh == 1 && a->kw == 1 && a->stride == 1 && a->compute == DCVC_BF16 && g_use_gemm) {
    const int r = dcvc_internal_gemm1x1(a, stream);
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  if (((a->kh == 1 && a->kw == 1) || (a->kh == 3 && a->kw == 3)) && a->stride == 1 && a->compute == DCVC_F32) {
    const int r = dcvc_internal_gemm1x1_f32(a, stream);   // 1x1 and 3x3 (shifted GEMMs) fp32
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  if (a->kh == 3 && a->kw == 3 && a->stride == 2 && a->compute == DCVC_BF16) {
    const int r = dcvc_internal_conv3s2(a, stream);   // downsampling convs, persistent
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  if (a->kh == 7 && a->kw == 7 && a->compute == DCVC_BF16) {
    int r = dcvc_internal_conv7s(a, stream);   // SpyNet's 8- / 16-channel layers
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
    r = dcvc_internal_conv7w(a, stream);       // and its 32- / 64-channel ones
    if (r != DCVC_HIP_EUNSUPPORTED) return r;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool xin32 = a->x.dtype == DCVC_F32, yout32 = a->y.dtype == DCVC_F32;
  {
    const int xa = xin32 ? 4 : 8;   // elements per 16 bytes
    p.vec = (a->cin % 8 == 0) && (p.xcs % xa == 0) && (p.xco % xa == 0) &&
            ((uintptr_t)p.x % 16 == 0);
    // 8-channel (16/32-byte) pieces in the epilogue
    bool vo = (p.ycs % 8 == 0) && (p.yco % 8 == 0) && ((uintptr_t)p.y % 16 == 0);
    if (a->res.ptr) vo = vo && (p.rcs % 8 == 0) && (p.rco % 8 == 0) && ((uintptr_t)p.res % 16 == 0);
    if (a->res2.ptr) vo = vo && (p.r2cs % 8 == 0) && (p.r2co % 8 == 0) && ((uintptr_t)p.res2 % 16 == 0);
    p.vec_out = vo ? 1 : 0;
  }
  if (a->compute == DCVC_F32) {
    if (!xin32 || !yout32) return DCVC_HIP_EUNSUPPORTED;
    return pick_bn<float, float, true>(p, st);
  }
  if (xin32 && yout32) return pick_bn<float, float, false>(p, st);
  if (xin32 && !yout32) return pick_bn<float, uint16_t, false>(p, st);
  if (!xin32 && yout32) return pick_bn<uint16_t, float, false>(p, st);
  return pick_bn<uint16_t, uint16_t, false>(p, st);
}

extern "C" int dcvc_set_option(const char *name, int value) {
  if (!name) return DCVC_HIP_EINVAL;
  if (std::strcmp(name, "gemm1x1") == 0) {
    g_use_gemm = value;
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "gemm1x1_f32") == 0) {
    dcvc_internal_gemm1x1_f32_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "gemm3x3_f32") == 0) {
    dcvc_internal_gemm3x3_f32_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "gemm1x1_f32_cfg") == 0) {
    dcvc_internal_gemm1x1_f32_cfg(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "gemm1x1_f32_upfront") == 0) {
    dcvc_internal_gemm1x1_f32_upfront(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "gemm1x1_f32_direct") == 0) {
    dcvc_internal_gemm1x1_f32_direct(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3") == 0) {
    g_use_conv3 = value;
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dcb_persistent") == 0) {
    dcvc_internal_dcbp_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3_s2") == 0) {
    dcvc_internal_conv3s2_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv7_wide_cin") == 0) {
    dcvc_internal_conv7w_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv7_small_cin") == 0) {
    dcvc_internal_conv7s_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dcb_stream") == 0) {
    dcvc_internal_dcbs_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3_persistent") == 0) {
    dcvc_internal_conv3p_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3_resident") == 0) {
    dcvc_internal_conv3x3_resident(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv_th") == 0) {
    g_force_th = value;
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv_bn") == 0) {
    g_force_bn = value;
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "gemm1x1_bm") == 0) {
    dcvc_internal_gemm1x1_bm(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3_occupancy") == 0) {
    dcvc_internal_conv3p_occupancy(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3_epilogue") == 0) {
    dcvc_internal_conv3p_mode(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sconv_res_waves") == 0) {
    dcvc_internal_sconv_res_waves(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sgemm_pd") == 0) {
    dcvc_internal_sgemm_pd(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sgemm_gate") == 0) {
    dcvc_internal_sgemm_gate(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sgemm") == 0) {
    dcvc_internal_sgemm_cfg(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sconv_resident") == 0) {
    dcvc_internal_sconv_resident(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sconv_waves") == 0) {
    dcvc_internal_sconv_waves(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sconv_occupancy") == 0) {
    dcvc_internal_sconv_occupancy(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "xconv") == 0) {
    dcvc_internal_xconv_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "wconv") == 0) {
    dcvc_internal_wconv_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dconv") == 0) {
    dcvc_internal_dconv_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dconv_1x1") == 0) {
    dcvc_internal_dconv_1x1(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "sffn128") == 0) {
    dcvc_internal_sffn128(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "nconv") == 0) {
    dcvc_internal_nconv_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "tconv") == 0) {
    dcvc_internal_tconv_enable(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dconv_xcd") == 0) {
    dcvc_internal_dconv_xcd(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dconv_gate") == 0) {
    dcvc_internal_dconv_gate(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dconv_s2blocks") == 0) {
    dcvc_internal_dconv_s2blocks(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "dconv_bn128") == 0) {
    dcvc_internal_dconv_bn128(value);
    return DCVC_HIP_OK;
  }
  if (std::strcmp(name, "conv3x3_rows4") == 0) {
    dcvc_internal_conv3p_rows4(value);
    return DCVC_HIP_OK;
  }
  return dcvc_internal_set_option_split(name, value);   // the split-precision kernels' options (xconv.hip)
}
