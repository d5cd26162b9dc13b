// Coalesced conv epilogue shared by the MFMA kernels (conv.hip, conv3x3.hip,
// gemm1x1.hip).
//
// The MFMA D layout leaves each lane with 4 consecutive channels of one
// pixel: storing from there writes 8-16 B pieces 16 pixels apart, i.e.
// partial cache lines, which measured at ~1.5 TB/s on 48-channel bf16 maps.
// Instead the epilogue runs in two phases:
//   A (put4)        every lane writes v = act(acc + bias) in fp32 for its
//                   4 channels into an LDS tile T[pixel][LD] (LD = BN + 4,
//                   conflict-free ds_write_b128 for BN = 16k);
//   B (store_tile)  the workgroup walks the output tile in pieces of 8
//                   consecutive output channels of one output pixel, in
//                   output-row order, adds res then res2, applies the
//                   per-channel scale, converts and stores 16 B (bf16) / 32 B
//                   (fp32) per lane — whole lines per wave-instruction.
// Bias and scale are staged once per workgroup in LDS (stage_consts): a
// global load inside the epilogue would make the wave wait (vmcnt is in
// order) for every load and store issued before it, including the next
// tile's prefetch.  For the same reason phase B issues all residual loads of
// a thread before its first store.
// The arithmetic and its order are unchanged (fp32 until the single final
// conversion), so results are bit-identical to a per-lane epilogue:
//   out = scale[c] * (res2 + (res + act(conv + bias)))
// Pixel shuffle (r = 2) is applied in phase B: conv channel n of pixel
// (oy, ox) goes to output channel n >> 2 of pixel (2oy + (n>>1 & 1),
// 2ox + (n & 1)).
#pragma once
#include "common.h"

namespace epi {

template <typename T> struct V8;
template <> struct V8<uint16_t> {
  typedef u16x8 raw;
  __device__ __forceinline__ static raw load(const void *b, int64_t e) {
    return *reinterpret_cast<const u16x8 *>(reinterpret_cast<const uint16_t *>(b) + e);
  }
  __device__ __forceinline__ static float get(const raw &r, int j) { return bf2f(r[j]); }
  __device__ __forceinline__ static void store(void *b, int64_t e, const float v[8]) {
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
    *reinterpret_cast<u16x8 *>(reinterpret_cast<uint16_t *>(b) + e) = o;
  }
};
typedef float f32x8 __attribute__((ext_vector_type(8)));
template <> struct V8<float> {
  typedef f32x8 raw;
  __device__ __forceinline__ static raw load(const void *b, int64_t e) {
    const float *p = reinterpret_cast<const float *>(b) + e;
    const float4 a = *reinterpret_cast<const float4 *>(p);
    const float4 c = *reinterpret_cast<const float4 *>(p + 4);
    return f32x8{a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  }
  __device__ __forceinline__ static float get(const raw &r, int j) { return r[j]; }
  __device__ __forceinline__ static void store(void *b, int64_t e, const float v[8]) {
    float *p = reinterpret_cast<float *>(b) + e;
    *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4 *>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// LDS floats needed by stage_consts for a BN-wide tile
__host__ __device__ constexpr int consts_floats(int BN) { return 2 * BN; }

// Stage bias[n0 .. n0+BN) (0 beyond cout) and the output-channel scales of
// the tile (1 when absent) into Lc[0..BN) and Lc[BN..2BN).  Call before a
// barrier that precedes the first put4.
template <typename P>
__device__ __forceinline__ void stage_consts(const P &p, float *Lc, int n0, int BN) {
  const int cy0 = p.shuffle ? n0 >> 2 : n0;
  const int ncy = p.shuffle ? p.cout >> 2 : p.cout;
  for (int i = threadIdx.x; i < BN; i += blockDim.x) {
    const int n = n0 + i, c = cy0 + i;
    Lc[i] = (p.bias && n < p.cout) ? p.bias[n] : 0.f;
    Lc[BN + i] = (p.scale && c < ncy) ? p.scale[c] : 1.f;
  }
}

// Phase A: v = act(acc + bias) for local channels nl..nl+3 of tile pixel l.
template <typename P>
__device__ __forceinline__ void put4(const P &p, float *T, int LD, int l, int nl, const float *Lc,
                                     const f32x4 &acc) {
  const float4 b = *reinterpret_cast<const float4 *>(Lc + nl);
  float4 o;
  o.x = apply_act(p.act, acc[0] + b.x, p.slope);
  o.y = apply_act(p.act, acc[1] + b.y, p.slope);
  o.z = apply_act(p.act, acc[2] + b.z, p.slope);
  o.w = apply_act(p.act, acc[3] + b.w, p.slope);
  *reinterpret_cast<float4 *>(T + l * LD + nl) = o;
}

// Phase B.  npix tile pixels; conv channels n0 .. n0 + nvalid - 1 are valid;
// Lc as staged by stage_consts (scales at Lc + BN).  pix_of(l, oy, ox) maps
// tile pixel l to conv-output coordinates and returns false outside the
// image.  IPT >= ceil(items / blockDim.x) bounds the pieces per thread so the
// residual loads can all be issued before the first store.  RES = false
// compiles the residual adds out (p.res / p.res2 must then be null): a kernel
// that keeps LDS-DMA loads in flight across its epilogue needs no register
// loads there, or the compiler's vmcnt waits for them would drain the DMA.
// With RES the residual loads are retired before returning.  Every thread
// of the workgroup calls it after a barrier that follows phase A.
template <typename TOUT, int IPT, bool RES = true, typename P, typename PixFn>
__device__ __forceinline__ void store_tile(const P &p, const float *T, int LD, int npix, int n0,
                                           int nvalid, const float *Lc, int BN, PixFn pix_of) {
  typedef typename V8<TOUT>::raw raw;
  const bool shuf = p.shuffle != 0;
  const int ncy = shuf ? nvalid >> 2 : nvalid;
  const int cy0 = shuf ? n0 >> 2 : n0;
  const int pieces = (ncy + 7) >> 3;
  const int items = npix * (shuf ? 4 : 1) * pieces;
  int64_t pix[IPT];
  int cl[IPT], src[IPT], nc[IPT];
  raw r1[IPT], r2[IPT];
  // pass 1: addresses, and every residual load in flight
#pragma unroll
  for (int u = 0; u < IPT; ++u) {
    const int it = threadIdx.x + u * blockDim.x;
    nc[u] = 0;
    if (it >= items) continue;
    int t = it / pieces;
    const int q = it - t * pieces;
    int l = t, s = 0, oy, ox;
    if (shuf) {
      const int dx = t & 1;
      t >>= 1;
      const int dy = t / npix;
      l = t - dy * npix;
      s = dy * 2 + dx;
    }
    if (!pix_of(l, oy, ox)) continue;
    pix[u] = shuf ? (int64_t)(2 * oy + (s >> 1)) * p.Wout + 2 * ox + (s & 1) : (int64_t)oy * p.Wout + ox;
    cl[u] = q * 8;
    src[u] = l * LD + (shuf ? 4 * q * 8 + s : q * 8);
    nc[u] = min(8, ncy - q * 8);
    if (RES && p.vec_out && nc[u] == 8 && ((cy0 + cl[u]) & 7) == 0) {
      if (p.res) r1[u] = V8<TOUT>::load(p.res, pix[u] * p.rcs + p.rco + cy0 + cl[u]);
      if (p.res2) r2[u] = V8<TOUT>::load(p.res2, pix[u] * p.r2cs + p.r2co + cy0 + cl[u]);
    }
  }
  // pass 2: finish and store
#pragma unroll
  for (int u = 0; u < IPT; ++u) {
    if (nc[u] == 0) continue;
    const int c = cy0 + cl[u];
    float v[8];
    if (shuf) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = j < nc[u] ? T[src[u] + 4 * j] : 0.f;
    } else {
      const float4 a = *reinterpret_cast<const float4 *>(T + src[u]);
      const float4 b = *reinterpret_cast<const float4 *>(T + src[u] + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    const float *sc = Lc + BN + cl[u];
    if (p.vec_out && nc[u] == 8 && (c & 7) == 0) {
      if (RES && p.res) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = V8<TOUT>::get(r1[u], j) + v[j];
      }
      if (RES && p.res2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = V8<TOUT>::get(r2[u], j) + v[j];
      }
      if (p.scale) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[j];
      }
      V8<TOUT>::store(p.y, pix[u] * p.ycs + p.yco + c, v);
      continue;
    }
    for (int j = 0; j < nc[u]; ++j) {
      float t = v[j];
      if (RES && p.res) t = ld<TOUT>(p.res, pix[u] * p.rcs + p.rco + c + j) + t;
      if (RES && p.res2) t = ld<TOUT>(p.res2, pix[u] * p.r2cs + p.r2co + c + j) + t;
      if (p.scale) t = t * sc[j];
      st<TOUT>(p.y, pix[u] * p.ycs + p.yco + c + j, t);
    }
  }
  if (RES) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no register load left in flight
}

// pieces per thread bound for a tile of npix pixels x BN conv channels
__host__ __device__ constexpr int ipt(int npix, int BN, int threads) {
  return (npix * ((BN / 8 > 4 * ((BN + 31) / 32)) ? BN / 8 : 4 * ((BN + 31) / 32)) + threads - 1) / threads;
}

}  // namespace epi
