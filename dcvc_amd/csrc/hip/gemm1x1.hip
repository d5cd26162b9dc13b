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
// The epilogue is epilogue.h's: bias, act, residual(s), scale, pixel shuffle.
#include "common.h"
#include "epilogue.h"

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

// staging double buffer, or the fp32 epilogue tile, whichever is larger
template <int BM, int BN>
__host__ __device__ constexpr size_t lds_main() {
  return ((size_t)2 * (BM + BN) * kK * 2 > (size_t)BM * (BN + 4) * 4 ? (size_t)2 * (BM + BN) * kK * 2
                                                                      : (size_t)BM * (BN + 4) * 4);
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
  float *Lc = reinterpret_cast<float *>(smem + lds_main<BM, BN>());  // bias | scale

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WMW, wn = wave / WMW;
  const int tm = blockIdx.x % p.tiles_m, tn = blockIdx.x / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const TIN *X = reinterpret_cast<const TIN *>(p.x);
  const int nsteps = p.cinp / kK;
  epi::stage_consts(p, Lc, n0, BN);  // published by the first barrier below

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

  // epilogue (epilogue.h): fp32 tile in LDS (the loop ended on a barrier),
  // then coalesced stores
  float *T = reinterpret_cast<float *>(smem);
  constexpr int LD = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      epi::put4(p, T, LD, (wm * TM + i) * 16 + col, (wn * TN + j) * 16 + hi * 4, Lc, acc[i][j]);
  __syncthreads();
  epi::store_tile<TOUT, epi::ipt(BM, BN, 256)>(p, T, LD, BM, n0, min(BN, p.cout - n0), Lc, BN,
                                               [&](int l, int &oy, int &ox) {
    const int m = m0 + l;
    oy = m / p.W;
    ox = m - oy * p.W;
    return m < p.M;
  });
}

template <typename TIN, typename TOUT, int BM, int BN, int WMW>
int launch(G1 p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.cout + BN - 1) / BN;
  const size_t lds = lds_main<BM, BN>() + epi::consts_floats(BN) * 4;
  auto kern = gemm1x1_kernel<TIN, TOUT, BM, BN, WMW>;
  dcvc_note_kernel("gemm1x1_kernel<%s, %s, %d, %d, %d>@%lld", tname<TIN>(), tname<TOUT>(), BM, BN, WMW,
                   (long long)p.tiles_m * tiles_n * 256);
  if (lds > 64 * 1024)
    dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * tiles_n)), dim3(256), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// Tile selection: BN is the 16-multiple tile (<= 128) that wastes the fewest
// MFMA columns; BM is as large as the grid allows while keeping >= 512
// workgroups.  The 68x120 latent GEMMs (8160 pixels) are latency-bound at
// one workgroup per CU: below 768 workgroups at BM = 64 they take BM = 32
// (where a 2x2 wave layout exists), so each CU holds ~3 workgroups' loads in
// flight.
int g_big_bm = 0;  // 0: automatic

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
  // Full-resolution 1x1 convs (2 M pixels): 256-pixel tiles hold 2 x 80 KB of
  // LDS per CU and leave too few loads in flight; 128-pixel tiles (BN >= 48)
  // and 64-pixel tiles (BN <= 32) measured 1.1-2.1x faster (64->64 at
  // 1088x1920: 325 -> 153 us).  dcvc_set_option("gemm1x1_bm", 64 | 128 | 256)
  // forces one size (A/B).
  if (big && bn <= 64 && g_big_bm != 256) {
    const bool b128 = g_big_bm == 128 || (g_big_bm == 0 && bn >= 48);
    switch (bn) {
      case 16: return b128 ? launch<TIN, TOUT, 128, 16, 4>(p, st) : launch<TIN, TOUT, 64, 16, 4>(p, st);
      case 32: return b128 ? launch<TIN, TOUT, 128, 32, 4>(p, st) : launch<TIN, TOUT, 64, 32, 4>(p, st);
      case 48: return b128 ? launch<TIN, TOUT, 128, 48, 4>(p, st) : launch<TIN, TOUT, 64, 48, 4>(p, st);
      default: return b128 ? launch<TIN, TOUT, 128, 64, 4>(p, st) : launch<TIN, TOUT, 64, 64, 4>(p, st);
    }
  }
  const bool mid = blocks(128) >= 512;
  const bool small = blocks(64) < 768;
  switch (bn) {
    case 16: return big ? launch<TIN, TOUT, 256, 16, 4>(p, st) : launch<TIN, TOUT, 64, 16, 4>(p, st);
    case 32:
      if (big) return launch<TIN, TOUT, 256, 32, 4>(p, st);
      return small ? launch<TIN, TOUT, 32, 32, 2>(p, st) : launch<TIN, TOUT, 64, 32, 4>(p, st);
    case 48: return big ? launch<TIN, TOUT, 256, 48, 4>(p, st) : launch<TIN, TOUT, 64, 48, 4>(p, st);
    case 64:
      if (big) return launch<TIN, TOUT, 256, 64, 4>(p, st);
      if (mid) return launch<TIN, TOUT, 128, 64, 4>(p, st);
      return small ? launch<TIN, TOUT, 32, 64, 2>(p, st) : launch<TIN, TOUT, 64, 64, 4>(p, st);
    case 96:
      if (big) return launch<TIN, TOUT, 128, 96, 2>(p, st);
      return small ? launch<TIN, TOUT, 32, 96, 2>(p, st) : launch<TIN, TOUT, 64, 96, 2>(p, st);
    default:
      if (big) return launch<TIN, TOUT, 128, 128, 2>(p, st);
      return small ? launch<TIN, TOUT, 32, 128, 2>(p, st) : launch<TIN, TOUT, 64, 128, 2>(p, st);
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
  bool vo = (p.ycs % 8 == 0) && (p.yco % 8 == 0) && (((uintptr_t)p.y & 15) == 0);
  if (a->res.ptr) vo = vo && (p.rcs % 8 == 0) && (p.rco % 8 == 0) && (((uintptr_t)p.res & 15) == 0);
  if (a->res2.ptr) vo = vo && (p.r2cs % 8 == 0) && (p.r2co % 8 == 0) && (((uintptr_t)p.res2 & 15) == 0);
  p.vec_out = vo ? 1 : 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (xin32 && yout32) return dispatch<float, float>(p, st);
  if (xin32) return dispatch<float, uint16_t>(p, st);
  if (yout32) return dispatch<uint16_t, float>(p, st);
  return dispatch<uint16_t, uint16_t>(p, st);
}

extern "C" void dcvc_internal_gemm1x1_bm(int v) { g_big_bm = (v == 64 || v == 128 || v == 256) ? v : 0; }
