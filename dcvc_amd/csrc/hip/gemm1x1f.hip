// Pointwise (1x1, stride 1) convolution in fp32 (f32 in, f32 MFMA, f32 out):
// the entropy-parameter tail of the codecs (hyperprior decoders, prior
// fusion, the quadtree / dual spatial priors: DepthConvBlocks on the
// 68x120 latent grid at 1080p) that the reference computes in fp32.
//
// D[n][p] = sum_k W[n][k] * X[p][k] on v_mfma_f32_16x16x4_f32 (exact f32,
// the same accumulation order as conv.hip's f32 path: k ascending, 4 per
// MFMA, so the two kernels are bit-identical).  Workgroup = 4 waves = BM
// pixels x BN channels; K advances 32 channels per step.  Each step's global
// loads (32 B per lane) are issued into registers before the MFMAs of the
// previous step and written to the other LDS buffer after them (one barrier
// per step), so the load latency hides behind the matrix work; conv.hip's
// generic path waited on it twice per 32 channels (47 TF/s at 384->384,
// 68x120).  LDS row stride: ldk() below.  Epilogue: epilogue.h.
#include "common.h"
#include "epilogue.h"

namespace {

constexpr int kK = 32;   // weight rows are padded to 32 channels (conv.hip's chunk)

struct GF {
  const float *x;
  int M, W;
  int xcs, xco;
  const float *w;  // [cout][wstride] f32 (dcvc_conv_pack_weights, compute f32)
  const float *bias;
  void *y;
  int ycs, yco;
  int cin, cout, wstride;
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
  int vec_out;
  int tiles_m;
};

// LDS row stride: KK + 2 floats.  An operand read is a ds_read_b32 of rows
// r..r+15 at k..k+3 (lane = 16 hi + col); its 32-lane halves see banks
// (a / 4) % 32 = (2 col + hi + const) % 32: all distinct, conflict-free (a
// stride of KK + 4 put col and col + 8 on one bank: 2-way).  Rows are then
// 8-byte aligned, so staging writes are ds_write_b64.
template <int KK> __host__ __device__ constexpr int ldk() { return KK + 2; }

template <int BM, int BN, int KK>
__host__ __device__ constexpr size_t lds_main() {
  return (size_t)2 * (BM + BN) * ldk<KK>() * 4 > (size_t)BM * (BN + 4) * 4 ? (size_t)2 * (BM + BN) * ldk<KK>() * 4
                                                                            : (size_t)BM * (BN + 4) * 4;
}

// Direct epilogue of a wave's TM x TN 16x16 accumulator tiles: tile (i, j)
// holds, per lane, local channels nl + 16 j .. + 3 of pixel m + 16 i.
// out = scale * (res2 + (res + act(acc + bias))), epilogue.h's order.  Every
// residual load is issued before the first store (vmcnt is in order).  The
// host takes this path only when cout is a multiple of 16, every view is
// 16-byte aligned (vec_out) and there is no shuffle.
template <int TM, int TN, int BN>
__device__ __forceinline__ void direct_epilogue(const GF &p, const f32x4 (&acc)[TM][TN], const float *Lc, int m,
                                                int n0, int nl) {
  f32x4 r1[TM][TN], r2[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int mm = m + 16 * i, n = n0 + nl + 16 * j;
      const bool ok = mm < p.M && n < p.cout;
      if (p.res && ok) r1[i][j] = *reinterpret_cast<const f32x4 *>(reinterpret_cast<const float *>(p.res) +
                                                                      (int64_t)mm * p.rcs + p.rco + n);
      if (p.res2 && ok) r2[i][j] = *reinterpret_cast<const f32x4 *>(reinterpret_cast<const float *>(p.res2) +
                                                                       (int64_t)mm * p.r2cs + p.r2co + n);
    }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int mm = m + 16 * i, n = n0 + nl + 16 * j, c = nl + 16 * j;
      if (!(mm < p.M && n < p.cout)) continue;
      const float4 b = *reinterpret_cast<const float4 *>(Lc + c);
      f32x4 v;
      v[0] = apply_act(p.act, acc[i][j][0] + b.x, p.slope);
      v[1] = apply_act(p.act, acc[i][j][1] + b.y, p.slope);
      v[2] = apply_act(p.act, acc[i][j][2] + b.z, p.slope);
      v[3] = apply_act(p.act, acc[i][j][3] + b.w, p.slope);
      if (p.res) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = r1[i][j][e] + v[e];
      }
      if (p.res2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = r2[i][j][e] + v[e];
      }
      if (p.scale) {
        const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + c);  // stage_consts: scales at Lc + BN
        v[0] = v[0] * sc.x;
        v[1] = v[1] * sc.y;
        v[2] = v[2] * sc.z;
        v[3] = v[3] * sc.w;
      }
      *reinterpret_cast<f32x4 *>(reinterpret_cast<float *>(p.y) + (int64_t)mm * p.ycs + p.yco + n) = v;
    }
}

// K3: 3x3 stride-1 pad-1 conv as nine shifted 1x1 GEMMs over the same
// pixel tile: step s = (32-channel chunk s / 9, tap s % 9), the order of
// conv.hip's f32 path (chunk-major, taps inside), so again bit-identical;
// the shifted rows of a tap are contiguous in memory (zero outside the map).
int g_upfront = 1;  // dcvc_set_option("gemm1x1_f32_upfront", 0/1): step operands read up front (A/B)
int g_direct = 1;   // dcvc_set_option("gemm1x1_f32_direct", 0/1): epilogue straight from the accumulators (A/B)

template <int BM, int BN, int WMW, int KK, bool LIN, bool K3 = false, bool kUpfront = true, bool kDirect = false>
__global__ void __launch_bounds__(256) gemm1x1f_kernel(GF p) {
  constexpr int kLD = ldk<KK>();
  constexpr int Q = KK / 8;                 // 8-float pieces per row per step
  constexpr int WNW = 4 / WMW;
  constexpr int TM = BM / WMW / 16;
  constexpr int TN = BN / WNW / 16;
  constexpr int PX = (BM * Q + 255) / 256;  // 8-float pieces per thread per step
  constexpr int PW = (BN * Q + 255) / 256;
  static_assert(TM >= 1 && TN >= 1, "tile");
  extern __shared__ __align__(16) unsigned char smem[];
  float *Xs = reinterpret_cast<float *>(smem);  // [2][BM][kLD]
  float *Ws = Xs + 2 * BM * kLD;                 // [2][BN][kLD]
  float *Lc = reinterpret_cast<float *>(smem + lds_main<BM, BN, KK>());

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WMW, wn = wave / WMW;
  const int tm = blockIdx.x % p.tiles_m, tn = blockIdx.x / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nsteps = (p.wstride + KK - 1) / KK;
  epi::stage_consts(p, Lc, n0, BN);
  static_assert(!K3 || KK == 32, "3x3: 32-channel steps");
  const int cinp = K3 ? p.wstride / 9 : 0;
  int py[PX], px_[PX];   // K3: map coordinates of this thread's staged pixels
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int m = m0 + (threadIdx.x + i * 256) / Q;
    py[i] = m / p.W;
    px_[i] = m - py[i] * p.W;
  }

  float4 pxa[PX], pxb[PX], pwa[PW], pwb[PW];
  auto load_step = [&](int s) {
    int k0 = s * KK, kw = k0, dy = 0, dx = 0;
    if constexpr (K3) {
      const int chunk = s / 9, tap = s - chunk * 9;
      dy = tap / 3 - 1;
      dx = tap % 3 - 1;
      k0 = chunk * 32;
      kw = tap * cinp + k0;
    }
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int it = threadIdx.x + i * 256;
      const int r = it / Q, q = it % Q;
      int m = m0 + r;
      const int c = k0 + q * 8;
      bool ok = it < BM * Q && m < p.M && c < p.cin;
      if constexpr (K3) {
        const int sy = py[i] + dy, sx = px_[i] + dx;
        ok = ok && sy >= 0 && sy < p.M / p.W && sx >= 0 && sx < p.W;
        m = sy * p.W + sx;
      }
      if (ok) {
        const float *src = p.x + (int64_t)m * p.xcs + p.xco + c;
        pxa[i] = *reinterpret_cast<const float4 *>(src);
        pxb[i] = *reinterpret_cast<const float4 *>(src + 4);
      } else {
        pxa[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        pxb[i] = pxa[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int it = threadIdx.x + i * 256;
      const int r = it / Q, q = it % Q;
      const int n = n0 + r, c = kw + q * 8;
      if (it < BN * Q && n < p.cout && c < p.wstride) {
        const float *src = p.w + (int64_t)n * p.wstride + c;
        pwa[i] = *reinterpret_cast<const float4 *>(src);
        pwb[i] = *reinterpret_cast<const float4 *>(src + 4);
      } else {
        pwa[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        pwb[i] = pwa[i];
      }
    }
  };
  auto lrelu4 = [&](float4 v) {
    const float s = p.in_slope;
    v.x = v.x >= 0.f ? v.x : v.x * s;
    v.y = v.y >= 0.f ? v.y : v.y * s;
    v.z = v.z >= 0.f ? v.z : v.z * s;
    v.w = v.w >= 0.f ? v.w : v.w * s;
    return v;
  };
  auto store_step = [&](int buf) {
    float *xs = Xs + buf * BM * kLD;
    float *ws = Ws + buf * BN * kLD;
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int it = threadIdx.x + i * 256;
      if (BM * Q % 256 == 0 || it < BM * Q) {
        const int r = it / Q, q = it % Q;
        float4 a = pxa[i], b = pxb[i];
        if constexpr (LIN) {  // input op leaky ReLU (a template flag: no run-time branch)
          a = lrelu4(a);
          b = lrelu4(b);
        }
        float2 *d = reinterpret_cast<float2 *>(xs + r * kLD + q * 8);
        d[0] = make_float2(a.x, a.y);
        d[1] = make_float2(a.z, a.w);
        d[2] = make_float2(b.x, b.y);
        d[3] = make_float2(b.z, b.w);
      }
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int it = threadIdx.x + i * 256;
      if (BN * Q % 256 == 0 || it < BN * Q) {
        const int r = it / Q, q = it % Q;
        float2 *d = reinterpret_cast<float2 *>(ws + r * kLD + q * 8);
        d[0] = make_float2(pwa[i].x, pwa[i].y);
        d[1] = make_float2(pwa[i].z, pwa[i].w);
        d[2] = make_float2(pwb[i].x, pwb[i].y);
        d[3] = make_float2(pwb[i].z, pwb[i].w);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int col = lane & 15, hi = lane >> 4;
  load_step(0);
  store_step(0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load_step(s + 1);
    const float *xs = Xs + buf * BM * kLD;
    const float *ws = Ws + buf * BN * kLD;
    if constexpr (kUpfront) {
      // every operand of the step read up front (KK / 4 * (TN + TM) VGPRs):
      // the LDS reads stream back to back and the MFMAs issue without
      // waiting on a read issued one MFMA earlier
      float a[KK / 4][TN], b[KK / 4][TM];
#pragma unroll
      for (int g = 0; g < KK / 4; ++g) {
#pragma unroll
        for (int j = 0; j < TN; ++j) a[g][j] = ws[((wn * TN + j) * 16 + col) * kLD + g * 4 + hi];
#pragma unroll
        for (int i = 0; i < TM; ++i) b[g][i] = xs[((wm * TM + i) * 16 + col) * kLD + g * 4 + hi];
      }
#pragma unroll
      for (int g = 0; g < KK / 4; ++g)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][j], b[g][i], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
    for (int g = 0; g < KK / 4; ++g) {
      float a[TN], b[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) a[j] = ws[((wn * TN + j) * 16 + col) * kLD + g * 4 + hi];
#pragma unroll
      for (int i = 0; i < TM; ++i) b[i] = xs[((wm * TM + i) * 16 + col) * kLD + g * 4 + hi];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[i], acc[i][j], 0, 0, 0);
    }
    }
    if (s + 1 < nsteps) store_step(buf ^ 1);
    __syncthreads();
  }

  if constexpr (kDirect) {
    // straight from the accumulators (no shuffle, 16-byte aligned fp32 views,
    // output pixel = input pixel): a lane holds channels n..n+3 of pixel m
    // (16x16x4 D layout), one 16-byte residual load and store each; the
    // operations and their order are epilogue.h's, so results are identical
    direct_epilogue<TM, TN, BN>(p, acc, Lc, m0 + wm * TM * 16 + col, n0, (wn * TN) * 16 + hi * 4);
    return;
  }
  float *T = reinterpret_cast<float *>(smem);
  constexpr int LD = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      epi::put4(p, T, LD, (wm * TM + i) * 16 + col, (wn * TN + j) * 16 + hi * 4, Lc, acc[i][j]);
  __syncthreads();
  epi::store_tile<float, epi::ipt(BM, BN, 256)>(p, T, LD, BM, n0, min(BN, p.cout - n0), Lc, BN,
                                                [&](int l, int &oy, int &ox) {
    const int m = m0 + l;
    oy = m / p.W;
    ox = m - oy * p.W;
    return m < p.M;
  });
}

// Variant on v_mfma_f32_32x32x2_f32 (64-cycle issue, 16 accumulators per
// lane): half the MFMA instructions of the 16x16x4 form for the same work and
// one f32 operand per lane per MFMA.  Both forms are a k-ascending f32 fma
// chain, so the results are bit-identical.  4 waves in a 2 x 2 grid, each
// (BM / 2) x (BN / 2) in 32 x 32 MFMA tiles; LDS rows of KK + 1 floats (odd:
// a 32-lane half reading rows r..r+31 at one k touches 32 banks).
template <int KK> __host__ __device__ constexpr int ldk32() { return KK + 1; }

template <int BM, int BN, int KK>
__host__ __device__ constexpr size_t lds_main32() {
  return (size_t)2 * (BM + BN) * ldk32<KK>() * 4 > (size_t)BM * (BN + 4) * 4 ? (size_t)2 * (BM + BN) * ldk32<KK>() * 4
                                                                              : (size_t)BM * (BN + 4) * 4;
}

template <int BM, int BN, int KK, bool kUpfront = true>
__global__ void __launch_bounds__(256) gemm1x1f32_kernel(GF p) {
  constexpr int kLD = ldk32<KK>();
  constexpr int Q = KK / 8;
  constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 tiles per wave
  constexpr int PX = (BM * Q + 255) / 256;
  constexpr int PW = (BN * Q + 255) / 256;
  static_assert(TM >= 1 && TN >= 1, "tile");
  extern __shared__ __align__(16) unsigned char smem[];
  float *Xs = reinterpret_cast<float *>(smem);  // [2][BM][kLD]
  float *Ws = Xs + 2 * BM * kLD;                 // [2][BN][kLD]
  float *Lc = reinterpret_cast<float *>(smem + lds_main32<BM, BN, KK>());

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave & 1, wn = wave >> 1;
  const int tm = blockIdx.x % p.tiles_m, tn = blockIdx.x / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nsteps = (p.wstride + KK - 1) / KK;
  epi::stage_consts(p, Lc, n0, BN);

  float4 pxa[PX], pxb[PX], pwa[PW], pwb[PW];
  auto load_step = [&](int s) {
    const int k0 = s * KK;
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int it = threadIdx.x + i * 256;
      const int r = it / Q, q = it % Q;
      const int m = m0 + r, c = k0 + q * 8;
      if (it < BM * Q && m < p.M && c < p.cin) {
        const float *src = p.x + (int64_t)m * p.xcs + p.xco + c;
        pxa[i] = *reinterpret_cast<const float4 *>(src);
        pxb[i] = *reinterpret_cast<const float4 *>(src + 4);
      } else {
        pxa[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        pxb[i] = pxa[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int it = threadIdx.x + i * 256;
      const int r = it / Q, q = it % Q;
      const int n = n0 + r, c = k0 + q * 8;
      if (it < BN * Q && n < p.cout && c < p.wstride) {
        const float *src = p.w + (int64_t)n * p.wstride + c;
        pwa[i] = *reinterpret_cast<const float4 *>(src);
        pwb[i] = *reinterpret_cast<const float4 *>(src + 4);
      } else {
        pwa[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        pwb[i] = pwa[i];
      }
    }
  };
  auto lrelu4 = [&](float4 v) {
    const float s = p.in_slope;
    v.x = v.x >= 0.f ? v.x : v.x * s;
    v.y = v.y >= 0.f ? v.y : v.y * s;
    v.z = v.z >= 0.f ? v.z : v.z * s;
    v.w = v.w >= 0.f ? v.w : v.w * s;
    return v;
  };
  auto put8 = [&](float *d, float4 a, float4 b) {
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
    d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
  };
  auto store_step = [&](int buf) {
    float *xs = Xs + buf * BM * kLD;
    float *ws = Ws + buf * BN * kLD;
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int it = threadIdx.x + i * 256;
      if (BM * Q % 256 == 0 || it < BM * Q) {
        const int r = it / Q, q = it % Q;
        float4 a = pxa[i], b = pxb[i];
        if (p.in_op == DCVC_IN_LRELU) {
          a = lrelu4(a);
          b = lrelu4(b);
        }
        put8(xs + r * kLD + q * 8, a, b);
      }
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int it = threadIdx.x + i * 256;
      if (BN * Q % 256 == 0 || it < BN * Q) {
        const int r = it / Q, q = it % Q;
        put8(ws + r * kLD + q * 8, pwa[i], pwb[i]);
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  load_step(0);
  store_step(0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load_step(s + 1);
    const float *xs = Xs + buf * BM * kLD;
    const float *ws = Ws + buf * BN * kLD;
    if constexpr (kUpfront) {
      float a[KK / 2][TN], b[KK / 2][TM];  // the step's operands up front (gemm1x1f_kernel)
#pragma unroll
      for (int kk = 0; kk < KK / 2; ++kk) {
#pragma unroll
        for (int j = 0; j < TN; ++j) a[kk][j] = ws[((wn * TN + j) * 32 + r32) * kLD + 2 * kk + h];
#pragma unroll
        for (int i = 0; i < TM; ++i) b[kk][i] = xs[((wm * TM + i) * 32 + r32) * kLD + 2 * kk + h];
      }
#pragma unroll
      for (int kk = 0; kk < KK / 2; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][j], b[kk][i], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
    for (int kk = 0; kk < KK / 2; ++kk) {
      float a[TN], b[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) a[j] = ws[((wn * TN + j) * 32 + r32) * kLD + 2 * kk + h];
#pragma unroll
      for (int i = 0; i < TM; ++i) b[i] = xs[((wm * TM + i) * 32 + r32) * kLD + 2 * kk + h];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[i], acc[i][j], 0, 0, 0);
    }
    }
    if (s + 1 < nsteps) store_step(buf ^ 1);
    __syncthreads();
  }

  float *T = reinterpret_cast<float *>(smem);
  constexpr int LD = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        epi::put4(p, T, LD, (wm * TM + i) * 32 + r32, (wn * TN + j) * 32 + 8 * g + 4 * h, Lc,
                  f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]});
  __syncthreads();
  epi::store_tile<float, epi::ipt(BM, BN, 256)>(p, T, LD, BM, n0, min(BN, p.cout - n0), Lc, BN,
                                                [&](int l, int &oy, int &ox) {
    const int m = m0 + l;
    oy = m / p.W;
    ox = m - oy * p.W;
    return m < p.M;
  });
}

template <int BM, int BN, int KK>
int launch32(GF p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.cout + BN - 1) / BN;
  const size_t lds = lds_main32<BM, BN, KK>() + epi::consts_floats(BN) * 4;
  auto kern = g_upfront ? gemm1x1f32_kernel<BM, BN, KK, true> : gemm1x1f32_kernel<BM, BN, KK, false>;
  dcvc_note_kernel("gemm1x1f32_kernel<%d, %d, %d, %s>@%lld", BM, BN, KK, bname(g_upfront), (long long)p.tiles_m * tiles_n * 256);
  if (lds > 64 * 1024) dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * tiles_n)), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

template <int BM, int BN, int WMW, int KK, bool K3 = false>
int launch(GF p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.cout + BN - 1) / BN;
  const size_t lds = lds_main<BM, BN, KK>() + epi::consts_floats(BN) * 4;
  const bool lin = p.in_op == DCVC_IN_LRELU;
  // direct epilogue (A/B: dcvc_set_option("gemm1x1_f32_direct", 0/1)): no
  // shuffle, whole 16-channel blocks, 16-byte aligned views
  const bool direct = g_direct && !p.shuffle && p.vec_out && p.cout % 16 == 0;
  typedef void (*KF)(GF);
  KF kern;
  if (direct) kern = lin ? gemm1x1f_kernel<BM, BN, WMW, KK, true, K3, true, true> : gemm1x1f_kernel<BM, BN, WMW, KK, false, K3, true, true>;
  else if (g_upfront) kern = lin ? gemm1x1f_kernel<BM, BN, WMW, KK, true, K3, true> : gemm1x1f_kernel<BM, BN, WMW, KK, false, K3, true>;
  else kern = lin ? gemm1x1f_kernel<BM, BN, WMW, KK, true, K3, false> : gemm1x1f_kernel<BM, BN, WMW, KK, false, K3, false>;
  dcvc_note_kernel("gemm1x1f_kernel<%d, %d, %d, %d, %s, %s, %s, %s>@%lld", BM, BN, WMW, KK, bname(lin), bname(K3),
                   bname(direct || g_upfront), bname(direct), (long long)p.tiles_m * tiles_n * 256);
  if (lds > 64 * 1024) dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * tiles_n)), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

int g_use_gemm_f32 = 1;
int g_use_k3 = 1;   // dcvc_set_option("gemm3x3_f32", 0/1): fp32 3x3 s1 convs as shifted GEMMs (A/B)
int g_cfg = 0;  // dcvc_set_option("gemm1x1_f32_cfg", i): force tile config i (A/B), 0 = automatic

// Tile choice, from A/B timings of every configuration on the 68x120 latent
// shapes (scripts/gemm_f32_bench.py, profiles/r02_gemm_f32.jsonl): 128 x 64
// tiles on the 32x32x2 form for narrow-in / wide-out layers, 64 x 64
// tiles with 32-channel steps for Cout >= 256, 64 x 32 tiles with 64-channel
// steps below (1.2-1.8x over the widest-tile rule at 384->1024, 768->192,
// 512->128); maps too small to give 512 such workgroups use 32-pixel tiles.
int dispatch(const GF &p, hipStream_t st) {
  switch (g_cfg) {
    case 1: return launch<64, 64, 2, 32>(p, st);
    case 2: return launch<64, 64, 2, 64>(p, st);
    case 3: return launch<64, 128, 2, 32>(p, st);
    case 4: return launch<128, 64, 2, 32>(p, st);
    case 5: return launch<128, 128, 2, 32>(p, st);
    case 6: return launch<64, 128, 2, 64>(p, st);
    case 7: return launch<32, 64, 2, 32>(p, st);
    case 8: return launch<64, 32, 4, 32>(p, st);
    case 9: return launch<32, 128, 1, 32>(p, st);
    case 10: return launch<128, 32, 4, 32>(p, st);
    case 11: return launch<64, 32, 4, 64>(p, st);
    case 12: return launch32<64, 64, 32>(p, st);
    case 13: return launch32<128, 64, 32>(p, st);
    case 14: return launch32<64, 128, 32>(p, st);
    case 15: return launch32<64, 64, 64>(p, st);
    default: break;
  }
  auto blocks = [&](int bm, int bn) { return (long)((p.M + bm - 1) / bm) * ((p.cout + bn - 1) / bn); };
  // 32x32x2 MFMA, 128-pixel tiles: 192->768 at 68x120 33 -> 30.5 us
  if (p.cin <= 256 && p.cout >= 512 && blocks(128, 64) >= 512) return launch32<128, 64, 32>(p, st);
  if (p.cout >= 256 && blocks(64, 64) >= 512) return launch<64, 64, 2, 32>(p, st);
  if (blocks(64, 32) >= 512) return launch<64, 32, 4, 64>(p, st);
  if (p.cout > 32) return launch<32, 64, 2, 32>(p, st);
  return launch<32, 32, 2, 32>(p, st);
}

// 3x3: 32-channel steps only (the chunk-major K order of conv.hip)
int dispatch3(const GF &p, hipStream_t st) {
  auto blocks = [&](int bm, int bn) { return (long)((p.M + bm - 1) / bm) * ((p.cout + bn - 1) / bn); };
  if (p.cout >= 256 && p.cout % 64 == 0 && blocks(64, 64) >= 512) return launch<64, 64, 2, 32, true>(p, st);
  if (blocks(64, 32) >= 512) return launch<64, 32, 4, 32, true>(p, st);
  if (p.cout > 32) return launch<32, 64, 2, 32, true>(p, st);
  return launch<32, 32, 2, 32, true>(p, st);
}

}  // namespace

// Called by dcvc_conv2d for 1x1 stride-1 convs with f32 compute, f32 in/out
// and 32-byte-aligned channel views; returns DCVC_HIP_EUNSUPPORTED otherwise.
extern "C" int dcvc_internal_gemm1x1_f32(const dcvc_conv_args *a, void *stream) {
  const bool k3 = a->kh == 3 && a->kw == 3 && a->stride == 1 && a->pad == 1;
  if (!(k3 ? g_use_k3 : g_use_gemm_f32) || a->compute != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  if (!k3 && (a->kh != 1 || a->kw != 1 || a->stride != 1)) return DCVC_HIP_EUNSUPPORTED;
  if (k3 && a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && a->in_op != DCVC_IN_LRELU) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  if (a->cin % 8 || a->x.cstride % 4 || a->x.coff % 4 || ((uintptr_t)a->x.ptr & 15) || ((uintptr_t)a->w & 15))
    return DCVC_HIP_EUNSUPPORTED;
  GF p{};
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.M = a->x.H * a->x.W;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const float *>(a->w);
  p.bias = a->bias;
  p.y = a->y.ptr;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.wstride = (a->cin + kK - 1) / kK * kK * (k3 ? 9 : 1);  // packed row length; steps of KK = 64 read zeros past it
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
  bool vo = (p.ycs % 8 == 0) && (p.yco % 8 == 0) && (((uintptr_t)p.y & 15) == 0);
  if (a->res.ptr) vo = vo && (p.rcs % 8 == 0) && (p.rco % 8 == 0) && (((uintptr_t)p.res & 15) == 0);
  if (a->res2.ptr) vo = vo && (p.r2cs % 8 == 0) && (p.r2co % 8 == 0) && (((uintptr_t)p.res2 & 15) == 0);
  p.vec_out = vo ? 1 : 0;
  if (k3) return dispatch3(p, reinterpret_cast<hipStream_t>(stream));
  return dispatch(p, reinterpret_cast<hipStream_t>(stream));
}

extern "C" void dcvc_internal_gemm1x1_f32_enable(int v) { g_use_gemm_f32 = v; }
extern "C" void dcvc_internal_gemm3x3_f32_enable(int v) { g_use_k3 = v; }
extern "C" void dcvc_internal_gemm1x1_f32_cfg(int v) { g_cfg = v; }
extern "C" void dcvc_internal_gemm1x1_f32_upfront(int v) { g_upfront = v; }
extern "C" void dcvc_internal_gemm1x1_f32_direct(int v) { g_direct = v; }
