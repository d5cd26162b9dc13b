// 3x3 stride-2 convolutions (padding 1) on bf16 NHWC maps with <= 64 input
// channels: the downsampling convs of DCVC-DC's feature extractor, contextual
// encoder and MV encoder (video_model.py:66-118, 173-200; ResidualBlockWithStride,
// layers.py:42-73) at full and half resolution.
//
// The generic implicit GEMM (conv.hip) stages its weight slice (up to 74 KB)
// and a 17x33-pixel input tile per 8x16 output tile: about as many L2 bytes
// of weights as of activations.  Here, as in conv3x3p.hip:
//   * one 8-wave workgroup per CU, persistent over 8x16 output tiles, keeps
//     its BN-channel weight slice resident in LDS ([BN][9 * CINP] bf16 rows,
//     32-byte skew per row);
//   * the next tile's 17x33 input window is prefetched into registers and
//     written into a column-de-interleaved image (even and odd input columns
//     in two planes), so the stride-2 B reads of 16 output columns are 16
//     consecutive pixels; 16-byte slots rotate with the pixel index so those
//     reads spread over all LDS banks;
//   * wave w computes output row w for all BN channels, K tap by tap, 32
//     channels per MFMA; input channels past CIN read as zeros (CINP = 64);
//   * the conv epilogue of epilogue.h (bias, activation, residuals, scale,
//     whole-line stores) through an fp32 tile that reuses the image.
#include "common.h"
#include "epilogue.h"

namespace {

constexpr int TH = 8, TW = 16;             // output tile
constexpr int IH = 2 * TH + 1;             // 17 input rows
constexpr int IWE = TW + 1;                // 17 even input columns (16 odd + 1 spare)
constexpr int NPX = 2 * IH * IWE;          // image pixels (two column planes)
constexpr int NWV = 8, NTHR = NWV * 64;

struct S2 {
  const uint16_t *x;
  int H, W, xcs, xco, xbytes;
  const uint16_t *w;  // [cout][3][3][cinp32] bf16 (dcvc_conv_pack_weights)
  int cinp;           // packed row channel count (cin rounded up to 32)
  const float *bias;
  const float *scale;
  void *y;
  int ycs, yco, Wout;
  const void *res;
  int rcs, rco;
  const void *res2;
  int r2cs, r2co;
  int cin, cout, act;
  float slope;
  int shuffle, vec_out;
  int Ho, Wo, tiles_x, tiles_y, nblk_n;
};

template <int BN>
struct GS {
  static constexpr int CINP = 64;                    // image channels (zero past cin)
  static constexpr int NS = CINP / 8;
  static constexpr int KPT = CINP / 32;
  static constexpr int KP = 9 * CINP;
  static constexpr int WP = KP + 16;
  static constexpr int NT = BN / 16;
  static constexpr int LD = BN + 4;
  static constexpr size_t WB = (size_t)BN * WP * 2;
  static constexpr size_t IB = (size_t)NPX * CINP * 2;
  static constexpr size_t TB = (size_t)TH * TW * LD * 4;
  static constexpr size_t BUF = IB > TB ? IB : TB;
  static constexpr size_t LDS = WB + BUF + (size_t)epi::consts_floats(BN) * 4;
  static constexpr int QP = 8;                       // 16-byte input pieces per pixel (64 channels)
  static constexpr int NIN = IH * (2 * TW + 1);      // 17 x 33 input pixels
  static constexpr int PP = (NIN * QP + NTHR - 1) / NTHR;
};

// image element offset of input pixel (iy, ix) of the window, channel slot s
__device__ __forceinline__ int img_off(int iy, int ix, int s) {
  const int p = ((ix & 1) * IH + iy) * IWE + (ix >> 1);
  return p * 64 + (((s + p) & 7) << 3);
}

template <int BN, typename TOUT>
__global__ void __launch_bounds__(NTHR) conv3s2_kernel(S2 p) {
  typedef GS<BN> G_;
  constexpr int KPT = G_::KPT, KP = G_::KP, WP = G_::WP, NT = G_::NT, LD = G_::LD, QP = G_::QP, PP = G_::PP;
  constexpr int NIN = G_::NIN;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Lw = reinterpret_cast<uint16_t *>(smem);
  uint16_t *Li = reinterpret_cast<uint16_t *>(smem + G_::WB);
  float *T = reinterpret_cast<float *>(smem + G_::WB);
  float *Lc = reinterpret_cast<float *>(smem + G_::WB + G_::BUF);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int nb = blockIdx.x % p.nblk_n, n0 = nb * BN;
  const int G = gridDim.x / p.nblk_n;
  int g = blockIdx.x / p.nblk_n;
  if (p.nblk_n == 1 && (G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);  // consecutive tiles per XCD
  const int ntiles = p.tiles_x * p.tiles_y;
  if (g >= ntiles) return;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.x), (short)0, p.xbytes, 0x00020000);
  // input piece u of thread tid = (window pixel, 16-byte channel piece); outside
  // the image or past cin the buffer load returns zeros
  u16x8 pf[PP];
  auto issue = [&](int t) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * NTHR;
      const int pix = it / QP, q = it - pix * QP;
      const int iy = pix / (2 * TW + 1), ix = pix - iy * (2 * TW + 1);
      const int gy = 2 * oy0 - 1 + iy, gx = 2 * ox0 - 1 + ix;
      const bool in = it < NIN * QP && q * 8 < p.cin && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
      const int off = in ? ((gy * p.W + gx) * p.xcs + p.xco + q * 8) * 2 : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto publish = [&]() {
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * NTHR;
      const int pix = it / QP, q = it - pix * QP;
      const int iy = pix / (2 * TW + 1), ix = pix - iy * (2 * TW + 1);
      if (it < NIN * QP) *reinterpret_cast<u16x8 *>(Li + img_off(iy, ix, q)) = pf[u];
    }
  };
  issue(g);

  // ---- resident weights: row n, k = tap * 64 + c (zero past cin / cout)
  for (int it = tid; it < BN * (KP / 8); it += NTHR) {
    const int n = it / (KP / 8), k8 = (it % (KP / 8)) * 8;
    const int tap = k8 / 64, c = k8 % 64;
    u16x8 v = u16x8{};
    if (n0 + n < p.cout && c < p.cinp) v = *reinterpret_cast<const u16x8 *>(p.w + ((int64_t)(n0 + n) * 9 + tap) * p.cinp + c);
    *reinterpret_cast<u16x8 *>(Lw + n * WP + k8) = v;
  }
  epi::stage_consts(p, Lc, n0, BN);
  // the odd plane's spare column (x = 33) is never loaded: keep it finite
  for (int iy = tid; iy < IH; iy += NTHR)
#pragma unroll
    for (int s = 0; s < 8; ++s) *reinterpret_cast<u16x8 *>(Li + img_off(iy, 33, s)) = u16x8{};
  const uint16_t *LwA = Lw + col * WP + hi * 8;

  for (int t = g;;) {
    const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
    int lane_ = lane;   // opaque per tile: the swizzled B addresses are not hoisted into registers
    asm volatile("" : "+v"(lane_));
    const int colq = lane_ & 15, hiq = lane_ >> 4;
    publish();
    __syncthreads();
    const int tn = t + G;
    const bool more = tn < ntiles;
    if (more) issue(tn);

    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap % 3;
#pragma unroll
      for (int c = 0; c < KPT; ++c) {
        const int ks = tap * KPT + c;
        bf16x8 a[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) a[j] = *reinterpret_cast<const bf16x8 *>(LwA + j * 16 * WP + ks * 32);
        const bf16x8 b = *reinterpret_cast<const bf16x8 *>(Li + img_off(2 * wave + dy, 2 * colq + dx, c * 4 + hiq));
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();  // the image is read: the fp32 tile may overwrite it

#pragma unroll
    for (int j = 0; j < NT; ++j) epi::put4(p, T, LD, wave * TW + col, j * 16 + hi * 4, Lc, acc[j]);
    __syncthreads();
    epi::store_tile<TOUT, epi::ipt(TH * TW, BN, NTHR)>(p, T, LD, TH * TW, n0, min(BN, p.cout - n0), Lc, BN,
                                                        [&](int l, int &oy, int &ox) {
      oy = oy0 + l / TW;
      ox = ox0 + l % TW;
      return oy < p.Ho && ox < p.Wo;
    });
    if (!more) break;
    __syncthreads();  // T read before the next image overwrites it
    t = tn;
  }
}

int g_cus = 0;
int g_enabled = 1;

template <int BN, typename TOUT>
int launch(S2 p, hipStream_t st) {
  typedef GS<BN> G_;
  static_assert(G_::LDS <= 160 * 1024, "LDS");
  p.tiles_x = (p.Wo + TW - 1) / TW;
  p.tiles_y = (p.Ho + TH - 1) / TH;
  p.nblk_n = (p.cout + BN - 1) / BN;
  const int64_t ntiles = (int64_t)p.tiles_x * p.tiles_y;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  if (ntiles < 2LL * g_cus) return DCVC_HIP_EUNSUPPORTED;  // small maps: the per-tile kernel
  const int per_n = g_cus / p.nblk_n;
  const int G = per_n * p.nblk_n;
  auto kern = conv3s2_kernel<BN, TOUT>;
  dcvc_note_kernel("conv3s2_kernel<%d, %s>@%lld", BN, tname<TOUT>(), (long long)G * NTHR);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(NTHR), G_::LDS, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

// Called by dcvc_conv2d (conv.hip) for 3x3 stride-2 pad-1 bf16 convs with
// <= 64 input channels on maps of >= 2 output tiles per CU;
// DCVC_HIP_EUNSUPPORTED hands the call back to the generic kernel.
extern "C" int dcvc_internal_conv3s2(const dcvc_conv_args *a, void *stream) {
  if (!g_enabled) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != 3 || a->kw != 3 || a->stride != 2 || a->pad != 1 || a->compute != DCVC_BF16) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_BF16 || a->y.dtype != DCVC_BF16 || a->in_op != DCVC_IN_NONE || a->shuffle)
    return DCVC_HIP_EUNSUPPORTED;
  if (a->cin > 64 || a->cin % 8) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.cstride % 8 || a->x.coff % 8 || ((uintptr_t)a->x.ptr & 15)) return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)a->x.H * a->x.W * a->x.cstride >= ((int64_t)1 << 30) - 16) return DCVC_HIP_EUNSUPPORTED;
  S2 p{};
  p.x = reinterpret_cast<const uint16_t *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.xbytes = a->x.H * a->x.W * a->x.cstride * 2;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.cinp = (a->cin + 31) / 32 * 32;
  p.bias = a->bias;
  p.scale = a->scale;
  p.y = a->y.ptr;
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.Wout = a->y.W;
  p.res = a->res.ptr;
  p.rcs = a->res.cstride;
  p.rco = a->res.coff;
  p.res2 = a->res2.ptr;
  p.r2cs = a->res2.cstride;
  p.r2co = a->res2.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.act = a->act;
  p.slope = a->slope;
  p.shuffle = 0;
  p.Ho = (a->x.H + 2 - 3) / 2 + 1;
  p.Wo = (a->x.W + 2 - 3) / 2 + 1;
  {
    bool vo = (p.ycs % 8 == 0) && (p.yco % 8 == 0) && ((uintptr_t)a->y.ptr % 16 == 0);
    if (p.res) vo = vo && (p.rcs % 8 == 0) && (p.rco % 8 == 0) && ((uintptr_t)p.res % 16 == 0);
    if (p.res2) vo = vo && (p.r2cs % 8 == 0) && (p.r2co % 8 == 0) && ((uintptr_t)p.res2 % 16 == 0);
    p.vec_out = vo ? 1 : 0;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->cout <= 64 && a->cout % 16 == 0) return launch<64, uint16_t>(p, st);
  if (a->cout % 48 == 0) return launch<48, uint16_t>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

// dcvc_set_option("conv3x3_s2", 0/1) (A/B switch, via conv.hip)
extern "C" void dcvc_internal_conv3s2_enable(int v) { g_enabled = v; }
