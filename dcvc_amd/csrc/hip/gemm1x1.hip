// Pointwise (1x1, stride 1) convolution as a double-buffered MFMA GEMM.
//
// D[n][p] = sum_k W[n][k] * X[p][k] over flattened pixels p (no halo, so the
// 2-D tiling of conv.hip is unnecessary).  Workgroup = 4 waves = BM pixels x
// BN output channels; K advances 64 channels per step.  Each step's global
// loads (16 B per lane, K-contiguous rows of weights and pixels) are issued
// into registers before the MFMAs of the previous step and written to the
// other LDS buffer after them, so one barrier separates steps and the HBM/L2
// latency hides behind the matrix work.  LDS rows are 128 B (64 bf16) with
// the 16-byte slot XOR-swizzled by (row >> 1) & 7 so the 16 lanes of an MFMA
// operand read (16 consecutive rows, same slot) hit 16 distinct bank groups.
// The epilogue is conv.hip's: bias, act, residual(s), scale, pixel shuffle.
#include "common.h"

namespace {

constexpr int kK = 64;  // K per pipeline step

struct G1 {
  const void *x;
  int M, W;  // pixels, image width (for shuffle / 2-D addressing)
  int xcs, xco;
  const uint16_t *w;  // [cout][cinp] bf16
  const float *bias;
  void *y;
  int ycs, yco;
  int cin, cout, cinp;  // cinp: cin rounded up to the 64-channel step
  int wstride;          // packed weight row length (cin rounded up to 32)
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

__device__ __forceinline__ int swz(int row, int slot) {  // element offset in a [rows][64] bf16 image
  return row * kK + ((slot ^ ((row >> 1) & 7)) << 3);
}

template <typename TIN> struct Piece;
template <> struct Piece<uint16_t> {
  u16x8 v;
  __device__ __forceinline__ void load(const uint16_t *p) { v = *reinterpret_cast<const u16x8 *>(p); }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0;
  }
  __device__ __forceinline__ float get(int j) const { return bf2f(v[j]); }
};
template <> struct Piece<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float *p) {
    a = *reinterpret_cast<const float4 *>(p);
    b = *reinterpret_cast<const float4 *>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ float get(int j) const {
    switch (j) {
      case 0: return a.x; case 1: return a.y; case 2: return a.z; case 3: return a.w;
      case 4: return b.x; case 5: return b.y; case 6: return b.z; default: return b.w;
    }
  }
};

template <typename TOUT>
__device__ __forceinline__ void store4(void *y, int64_t e, const float v[4]);
template <>
__device__ __forceinline__ void store4<float>(void *y, int64_t e, const float v[4]) {
  *reinterpret_cast<float4 *>(reinterpret_cast<float *>(y) + e) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void store4<uint16_t>(void *y, int64_t e, const float v[4]) {
  u16x4 o;
  o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
  *reinterpret_cast<u16x4 *>(reinterpret_cast<uint16_t *>(y) + e) = o;
}
template <typename T>
__device__ __forceinline__ void load4(const void *base, int64_t e, float v[4]);
template <>
__device__ __forceinline__ void load4<float>(const void *base, int64_t e, float v[4]) {
  const float4 a = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(base) + e);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <>
__device__ __forceinline__ void load4<uint16_t>(const void *base, int64_t e, float v[4]) {
  const u16x4 a = *reinterpret_cast<const u16x4 *>(reinterpret_cast<const uint16_t *>(base) + e);
  v[0] = bf2f(a[0]); v[1] = bf2f(a[1]); v[2] = bf2f(a[2]); v[3] = bf2f(a[3]);
}

template <typename TIN, typename TOUT, int BM, int BN, int WMW>
__global__ void __launch_bounds__(256) gemm1x1_kernel(G1 p) {
  constexpr int WNW = 4 / WMW;        // waves along N
  constexpr int TM = BM / WMW / 16;   // pixel tiles per wave
  constexpr int TN = BN / WNW / 16;   // channel tiles per wave
  constexpr int PX = BM * 8 / 256;    // pixel pieces per thread per step
  constexpr int PW = (BN * 8 + 255) / 256;  // weight pieces per thread per step
  static_assert(BM * 8 % 256 == 0, "BM");
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Xs = reinterpret_cast<uint16_t *>(smem);             // [2][BM][64]
  uint16_t *Ws = Xs + 2 * BM * kK;                                // [2][BN][64]

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WMW, wn = wave / WMW;
  const int tm = blockIdx.x % p.tiles_m, tn = blockIdx.x / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const TIN *X = reinterpret_cast<const TIN *>(p.x);
  const int nsteps = p.cinp / kK;

  Piece<TIN> px[PX];
  u16x8 pw[PW];

  auto load_step = [&](int s) {
    const int k0 = s * kK;
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int it = threadIdx.x + i * 256;
      const int r = it >> 3, slot = it & 7;
      const int m = m0 + r, c = k0 + slot * 8;
      if (m < p.M && c < p.cin) {
        const int64_t e = (int64_t)m * p.xcs + p.xco + c;
        px[i].load(X + e);
      } else {
        px[i].zero();
      }
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int it = threadIdx.x + i * 256;
      if (it >= BN * 8) break;
      const int r = it >> 3, slot = it & 7;
      const int n = n0 + r, c = k0 + slot * 8;
      if (n < p.cout && c < p.wstride) {
        pw[i] = *reinterpret_cast<const u16x8 *>(p.w + (int64_t)n * p.wstride + c);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) pw[i][j] = 0;
      }
    }
  };
  auto store_step = [&](int buf) {
    uint16_t *xs = Xs + buf * BM * kK;
    uint16_t *ws = Ws + buf * BN * kK;
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int it = threadIdx.x + i * 256;
      const int r = it >> 3, slot = it & 7;
      u16x8 o;
      if (p.in_op == DCVC_IN_LRELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = px[i].get(j);
          o[j] = f2bf(v >= 0.f ? v : v * p.in_slope);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(px[i].get(j));
      }
      *reinterpret_cast<u16x8 *>(xs + swz(r, slot)) = o;
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int it = threadIdx.x + i * 256;
      if (it >= BN * 8) break;
      const int r = it >> 3, slot = it & 7;
      *reinterpret_cast<u16x8 *>(ws + swz(r, slot)) = pw[i];
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
    const uint16_t *xs = Xs + buf * BM * kK;
    const uint16_t *ws = Ws + buf * BN * kK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[TN], b[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        a[j] = *reinterpret_cast<const bf16x8 *>(ws + swz((wn * TN + j) * 16 + col, kk * 4 + hi));
#pragma unroll
      for (int i = 0; i < TM; ++i)
        b[i] = *reinterpret_cast<const bf16x8 *>(xs + swz((wm * TM + i) * 16 + col, kk * 4 + hi));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[i], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) store_step(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane owns pixel m and channels nb..nb+3 of each (i, j) tile
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + (wm * TM + i) * 16 + col;
    if (m >= p.M) continue;
    const int oy = m / p.W, ox = m - oy * p.W;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nb = n0 + (wn * TN + j) * 16 + hi * 4;
      if (nb >= p.cout) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float t = acc[i][j][q];
        if (p.bias && nb + q < p.cout) t += p.bias[nb + q];
        v[q] = apply_act(p.act, t, p.slope);
      }
      if (p.vec_out && nb + 3 < p.cout) {
        const int64_t pix = m;
        if (p.res) {
          float rv[4];
          load4<TOUT>(p.res, pix * p.rcs + p.rco + nb, rv);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = rv[q] + v[q];
        }
        if (p.res2) {
          float rv[4];
          load4<TOUT>(p.res2, pix * p.r2cs + p.r2co + nb, rv);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = rv[q] + v[q];
        }
        if (p.scale) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = v[q] * p.scale[nb + q];
        }
        store4<TOUT>(p.y, pix * p.ycs + p.yco + nb, v);
        continue;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nb + q;
        if (n >= p.cout) continue;
        float t = v[q];
        int c = n, yy = oy, xx = ox;
        if (p.shuffle) {
          c = n >> 2;
          yy = oy * 2 + ((n >> 1) & 1);
          xx = ox * 2 + (n & 1);
        }
        const int64_t pix = (int64_t)yy * p.Wout + xx;
        if (p.res) t = ld<TOUT>(p.res, pix * p.rcs + p.rco + c) + t;
        if (p.res2) t = ld<TOUT>(p.res2, pix * p.r2cs + p.r2co + c) + t;
        if (p.scale) t = t * p.scale[c];
        st<TOUT>(p.y, pix * p.ycs + p.yco + c, t);
      }
    }
  }
}

template <typename TIN, typename TOUT, int BM, int BN, int WMW>
int launch(G1 p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.cout + BN - 1) / BN;
  const size_t lds = (size_t)2 * (BM + BN) * kK * 2;
  auto kern = gemm1x1_kernel<TIN, TOUT, BM, BN, WMW>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * tiles_n)), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// Tile selection: BN is the 16-multiple tile (<= 128) that wastes the fewest
// MFMA columns; BM is as large as the grid allows while keeping >= 512
// workgroups (the 68x120 latent GEMMs need the small tiles to fill 256 CUs).
template <typename TIN, typename TOUT>
int dispatch(const G1 &p, hipStream_t st) {
  static const int cand[6] = {16, 32, 48, 64, 96, 128};
  int bn = 16;
  long best = -1;
  for (int c : cand) {
    const long pad = ((p.cout + c - 1) / c) * (long)c - p.cout;
    if (best < 0 || pad < best || (pad == best && c > bn)) {
      bn = c;
      best = pad;
    }
  }
  const long tn = (p.cout + bn - 1) / bn;
  auto blocks = [&](int bm) { return ((p.M + bm - 1) / bm) * tn; };
  const bool big = blocks(bn <= 64 ? 256 : 128) >= 512;
  const bool mid = blocks(128) >= 512;
  switch (bn) {
    case 16: return big ? launch<TIN, TOUT, 256, 16, 4>(p, st) : launch<TIN, TOUT, 64, 16, 4>(p, st);
    case 32: return big ? launch<TIN, TOUT, 256, 32, 4>(p, st) : launch<TIN, TOUT, 64, 32, 4>(p, st);
    case 48: return big ? launch<TIN, TOUT, 256, 48, 4>(p, st) : launch<TIN, TOUT, 64, 48, 4>(p, st);
    case 64:
      if (big) return launch<TIN, TOUT, 256, 64, 4>(p, st);
      return mid ? launch<TIN, TOUT, 128, 64, 4>(p, st) : launch<TIN, TOUT, 64, 64, 4>(p, st);
    case 96: return big ? launch<TIN, TOUT, 128, 96, 2>(p, st) : launch<TIN, TOUT, 64, 96, 2>(p, st);
    default: return big ? launch<TIN, TOUT, 128, 128, 2>(p, st) : launch<TIN, TOUT, 64, 128, 2>(p, st);
  }
}

}  // namespace

// Called by dcvc_conv2d for 1x1 stride-1 convs with bf16 compute and
// 16-byte-aligned channel views; returns DCVC_HIP_EUNSUPPORTED otherwise.
extern "C" int dcvc_internal_gemm1x1(const dcvc_conv_args *a, void *stream) {
  if (a->kh != 1 || a->kw != 1 || a->stride != 1 || a->compute != DCVC_BF16) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op == DCVC_IN_GATE) return DCVC_HIP_EUNSUPPORTED;
  const bool xin32 = a->x.dtype == DCVC_F32, yout32 = a->y.dtype == DCVC_F32;
  const int xa = xin32 ? 4 : 8;
  if (a->cin % 8 || a->x.cstride % xa || a->x.coff % xa || ((uintptr_t)a->x.ptr & 15))
    return DCVC_HIP_EUNSUPPORTED;
  G1 p{};
  p.x = a->x.ptr;
  p.M = a->x.H * a->x.W;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.bias = a->bias;
  p.y = a->y.ptr;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.cinp = (a->cin + kK - 1) / kK * kK;
  p.wstride = (a->cin + 31) / 32 * 32;
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
  bool vo = !a->shuffle && (p.ycs % 4 == 0) && (p.yco % 4 == 0) && (((uintptr_t)p.y & 15) == 0);
  if (a->res.ptr) vo = vo && (p.rcs % 4 == 0) && (p.rco % 4 == 0);
  if (a->res2.ptr) vo = vo && (p.r2cs % 4 == 0) && (p.r2co % 4 == 0);
  p.vec_out = vo ? 1 : 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (xin32 && yout32) return dispatch<float, float>(p, st);
  if (xin32) return dispatch<float, uint16_t>(p, st);
  if (yout32) return dispatch<uint16_t, float>(p, st);
  return dispatch<uint16_t, uint16_t>(p, st);
}
