// 7x7 stride-1 convolutions with 8 or 16 input channels: the first and last
// layers of SpyNet's basic module (DCVC-DC/src/models/video_net.py:79-100,
// Conv2d(8, 32, 7) on [im1 | warp(im2) | flow] and Conv2d(16, 2, 7) to the
// flow residual), run at every pyramid level of the motion estimation.
//
// The generic implicit GEMM (conv.hip) walks K in 32-channel chunks per tap,
// so with 8 input channels 3/4 of every MFMA multiplies zero padding, and with
// 2 output channels 7/8 of its rows are padding as well; it also restages
// weights per kernel row.  Here K is packed across taps: one 32-wide K step
// covers 4 taps x 8 channels (or 2 taps x 16), i.e. 13 (25) MFMA K steps per
// 7x7 window instead of 49, and the B operand of a lane is one 16-byte pixel
// (8 channels) of the halo image at that lane's tap offset, read straight
// from LDS.  Workgroups are persistent (two per CU) with the packed weights
// resident in LDS, the next 16x16 tile's 22x22 halo prefetched into
// registers, and the conv epilogue of epilogue.h (bias, activation,
// residual, whole-line stores) through an fp32 tile that reuses the image.
// Accumulation order differs from conv.hip (taps summed inside one MFMA), so
// the results match a torch fp32 reference to bf16-operand tolerance, not
// conv.hip bit for bit (tests/test_gpu_kernels.py).
#include "common.h"
#include "epilogue.h"

namespace {

constexpr int TT = 16;          // 16x16 output tile
constexpr int HP = TT + 6;      // 22x22 halo
constexpr int NPX = HP * HP;    // 484 halo pixels
constexpr int NTHR = 256;       // 4 waves x 4 output rows

struct C7 {
  const uint16_t *x;
  int H, W, xcs, xco, xbytes;
  const uint16_t *w;  // [cout][7][7][32] bf16 (dcvc_conv_pack_weights)
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
  int tiles_x, tiles_y;
};

template <int CIN, int BN>
struct G7 {
  static constexpr int TPK = 32 / CIN;               // taps per 32-wide K step
  static constexpr int KS = (49 + TPK - 1) / TPK;    // K steps per window (13 | 25)
  static constexpr int KP = KS * 32;                 // packed K
  static constexpr int WP = KP + 16;                 // LDS weight row pitch (32-byte skew per row: conflict-free A reads)
  static constexpr int NT = BN / 16;
  static constexpr int LD = BN + 4;                  // fp32 epilogue tile row
  static constexpr size_t WB = (size_t)BN * WP * 2;
  static constexpr size_t IB = (size_t)NPX * CIN * 2;
  static constexpr size_t TB = (size_t)TT * TT * LD * 4;
  static constexpr size_t BUF = IB > TB ? IB : TB;
  static constexpr size_t LDS = WB + BUF + (size_t)epi::consts_floats(BN) * 4;
  static constexpr int QP = CIN / 8;                 // 16-byte pieces per pixel
  static constexpr int PP = (NPX * QP + NTHR - 1) / NTHR;
};

template <int CIN, int BN, typename TOUT>
__global__ void __launch_bounds__(NTHR) conv7s_kernel(C7 p) {
  typedef G7<CIN, BN> G_;
  constexpr int TPK = G_::TPK, KS = G_::KS, KP = G_::KP, WP = G_::WP, NT = G_::NT, LD = G_::LD;
  constexpr int QP = G_::QP, PP = G_::PP;
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *Lw = reinterpret_cast<uint16_t *>(smem);
  uint16_t *Li = reinterpret_cast<uint16_t *>(smem + G_::WB);
  float *T = reinterpret_cast<float *>(smem + G_::WB);
  float *Lc = reinterpret_cast<float *>(smem + G_::WB + G_::BUF);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, hi = lane >> 4;
  const int G = gridDim.x;
  const int g = blockIdx.x;
  const int ntiles = p.tiles_x * p.tiles_y;
  if (g >= ntiles) return;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.x), (short)0, p.xbytes, 0x00020000);
  // halo piece u of thread tid = (halo pixel, 16-byte channel piece); outside
  // the image the buffer load returns zeros (the conv's zero padding)
  u16x8 pf[PP];
  auto issue = [&](int t) {
    const int oy0 = (t / p.tiles_x) * TT, ox0 = (t % p.tiles_x) * TT;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * NTHR;
      const int pix = it / QP, q = it - pix * QP;
      const int hy = pix / HP, hx = pix - hy * HP;
      const int gy = oy0 - 3 + hy, gx = ox0 - 3 + hx;
      const bool in = it < NPX * QP && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
      const int off = in ? ((gy * p.W + gx) * p.xcs + p.xco + q * 8) * 2 : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto publish = [&]() {
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * NTHR;
      if (it < NPX * QP) *reinterpret_cast<u16x8 *>(Li + it * 8) = pf[u];
    }
  };
  issue(g);

  // ---- resident packed weights: row n, k = tap * CIN + c (zero past 49 taps / cout)
  for (int it = tid; it < BN * (KP / 8); it += NTHR) {
    const int n = it / (KP / 8), k8 = (it % (KP / 8)) * 8;
    const int tap = k8 / CIN, c = k8 % CIN;
    u16x8 v = u16x8{};
    if (n < p.cout && tap < 49) v = *reinterpret_cast<const u16x8 *>(p.w + ((int64_t)n * 49 + tap) * 32 + c);
    *reinterpret_cast<u16x8 *>(Lw + n * WP + k8) = v;
  }
  epi::stage_consts(p, Lc, 0, BN);

  // per-lane B offsets (elements) of each K step: this lane's tap of the step
  // (taps past 48 multiply zero weights; they read tap 48's finite data)
  int offb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    int tap = ks * TPK + hi / QP;
    if (tap > 48) tap = 48;
    const int dy = tap / 7, dx = tap - dy * 7;
    offb[ks] = ((wave * 4 + dy) * HP + col + dx) * CIN + (hi % QP) * 8;
  }
  const uint16_t *LwA = Lw + col * WP + hi * 8;

  for (int t = g;;) {
    const int oy0 = (t / p.tiles_x) * TT, ox0 = (t % p.tiles_x) * TT;
    publish();
    __syncthreads();
    const int tn = t + G;
    const bool more = tn < ntiles;
    if (more) issue(tn);

    f32x4 acc[4][NT];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 a[NT], b[4];
#pragma unroll
      for (int j = 0; j < NT; ++j) a[j] = *reinterpret_cast<const bf16x8 *>(LwA + j * 16 * WP + ks * 32);
#pragma unroll
      for (int r = 0; r < 4; ++r) b[r] = *reinterpret_cast<const bf16x8 *>(Li + offb[ks] + r * HP * CIN);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[r], acc[r][j], 0, 0, 0);
    }
    __syncthreads();  // the image is read: the fp32 tile may overwrite it

#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) epi::put4(p, T, LD, (wave * 4 + r) * TT + col, j * 16 + hi * 4, Lc, acc[r][j]);
    __syncthreads();
    epi::store_tile<TOUT, epi::ipt(TT * TT, BN, NTHR)>(p, T, LD, TT * TT, 0, p.cout, Lc, BN,
                                                        [&](int l, int &oy, int &ox) {
      oy = oy0 + l / TT;
      ox = ox0 + l % TT;
      return oy < p.H && ox < p.W;
    });
    if (!more) break;
    __syncthreads();  // T read before the next image overwrites it
    t = tn;
  }
}

int g_cus = 0;
int g_enabled = 1;

template <int CIN, int BN, typename TOUT>
int launch(C7 p, hipStream_t st) {
  typedef G7<CIN, BN> G_;
  static_assert(G_::LDS <= 80 * 1024, "two workgroups per CU");
  p.tiles_x = (p.W + TT - 1) / TT;
  p.tiles_y = (p.H + TT - 1) / TT;
  const int64_t ntiles = (int64_t)p.tiles_x * p.tiles_y;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  const int G = ntiles < 2 * g_cus ? (int)ntiles : 2 * g_cus;
  auto kern = conv7s_kernel<CIN, BN, TOUT>;
  dcvc_note_kernel("conv7s_kernel<%d, %d, %s>@%lld", CIN, BN, tname<TOUT>(), (long long)G * NTHR);
  if (G_::LDS > 64 * 1024) dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(NTHR), G_::LDS, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

// Called by dcvc_conv2d (conv.hip) for 7x7 stride-1 pad-3 bf16 convs with 8 or
// 16 input channels and <= 32 output channels; DCVC_HIP_EUNSUPPORTED hands the
// call back to the generic kernel.
extern "C" int dcvc_internal_conv7s(const dcvc_conv_args *a, void *stream) {
  if (!g_enabled) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != 7 || a->kw != 7 || a->stride != 1 || a->pad != 3 || a->compute != DCVC_BF16) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_BF16 || a->in_op != DCVC_IN_NONE || a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (!((a->cin == 8 && a->cout <= 32) || (a->cin == 16 && a->cout <= 16))) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.cstride % 8 || a->x.coff % 8 || ((uintptr_t)a->x.ptr & 15)) return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)a->x.H * a->x.W * a->x.cstride >= ((int64_t)1 << 30) - 16) return DCVC_HIP_EUNSUPPORTED;
  C7 p{};
  p.x = reinterpret_cast<const uint16_t *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.xbytes = a->x.H * a->x.W * a->x.cstride * 2;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
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
  {
    bool vo = (p.ycs % 8 == 0) && (p.yco % 8 == 0) && ((uintptr_t)a->y.ptr % 16 == 0);
    if (p.res) vo = vo && (p.rcs % 8 == 0) && (p.rco % 8 == 0) && ((uintptr_t)p.res % 16 == 0);
    if (p.res2) vo = vo && (p.r2cs % 8 == 0) && (p.r2co % 8 == 0) && ((uintptr_t)p.res2 % 16 == 0);
    p.vec_out = vo ? 1 : 0;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool y32 = a->y.dtype == DCVC_F32;
  if (a->cin == 8 && a->cout > 16)
    return y32 ? launch<8, 32, float>(p, st) : launch<8, 32, uint16_t>(p, st);
  if (a->cin == 8) return y32 ? launch<8, 16, float>(p, st) : launch<8, 16, uint16_t>(p, st);
  return y32 ? launch<16, 16, float>(p, st) : launch<16, 16, uint16_t>(p, st);
}

// dcvc_set_option("conv7_small_cin", 0/1) (A/B switch, via conv.hip)
extern "C" void dcvc_internal_conv7s_enable(int v) { g_enabled = v; }
