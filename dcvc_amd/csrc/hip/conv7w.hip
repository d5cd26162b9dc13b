// 7x7 stride-1 convolutions with 32 or 64 input channels: the three middle
// layers of SpyNet's basic module (DCVC-DC/src/models/video_net.py:79-100:
// Conv2d(32, 64, 7), Conv2d(64, 32, 7), Conv2d(32, 16, 7)), at every pyramid
// level of the motion estimation (the full-resolution level dominates).
//
// The generic implicit GEMM (conv.hip) restages the weights of each kernel
// row per tile and runs one 4-wave workgroup per tile (about 0.23 of MFMA
// peak on these layers).  This kernel is organised like conv3x3p.hip:
//   * one 8-wave workgroup per CU, persistent over 16x16 output tiles, with
//     its BN-channel slice of the weights resident in LDS for the launch
//     ([BN][49 * CIN] bf16 rows, 32-byte skew per row: conflict-free A reads);
//   * the next tile's 22x22 halo prefetched into registers during the
//     current tile, and written into a [pixel][CIN] image whose 16-byte slots
//     are rotated by the pixel index, so the B reads (16 consecutive pixels x
//     32 channels per MFMA) touch all 64 LDS banks once;
//   * wave w computes output rows 2w, 2w + 1 for all BN channels; K runs tap
//     by tap, 32 channels per MFMA (the same K order as conv.hip, which walks
//     taps inside each 32-channel chunk: for CIN = 64 the order differs);
//   * the conv epilogue of epilogue.h through an fp32 tile over the image.
#include "common.h"
#include "epilogue.h"

namespace {

constexpr int TT = 16, HP = TT + 6, NPX = HP * HP;
constexpr int NWV = 8, NTHR = NWV * 64, RW = 2;

struct C7W {
  const uint16_t *x;
  int H, W, xcs, xco, xbytes;
  const uint16_t *w;  // [cout][7][7][CIN] bf16 (dcvc_conv_pack_weights, CIN a multiple of 32)
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
  int tiles_x, tiles_y, nblk_n;
};

template <int CIN, int BN>
struct GW {
  static constexpr int NS = CIN / 8;                  // 16-byte slots per pixel
  static constexpr int SH = CIN == 32 ? 1 : 0;        // slot rotation: + (pixel >> SH)
  static constexpr int KPT = CIN / 32;                // MFMA K steps per tap
  static constexpr int KP = 49 * CIN;
  static constexpr int WP = KP + 16;                  // weight row pitch (elements)
  static constexpr int NT = BN / 16;
  static constexpr int LD = BN + 4;
  static constexpr size_t WB = (size_t)BN * WP * 2;
  static constexpr size_t IB = (size_t)NPX * CIN * 2;
  static constexpr size_t TB = (size_t)TT * TT * LD * 4;
  static constexpr size_t BUF = IB > TB ? IB : TB;
  static constexpr size_t LDS = WB + BUF + (size_t)epi::consts_floats(BN) * 4;
  static constexpr int PP = (NPX * NS + NTHR - 1) / NTHR;
};

template <int CIN>
__device__ __forceinline__ int pix_slot(int p, int s) {
  typedef GW<CIN, 16> G_;
  return p * CIN + (((s + (p >> G_::SH)) & (G_::NS - 1)) << 3);
}

template <int CIN, int BN, typename TOUT>
__global__ void __launch_bounds__(NTHR) conv7w_kernel(C7W p) {
  typedef GW<CIN, BN> G_;
  constexpr int NS = G_::NS, KPT = G_::KPT, KP = G_::KP, WP = G_::WP, NT = G_::NT, LD = G_::LD, PP = G_::PP;
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
  u16x8 pf[PP];
  auto issue = [&](int t) {
    const int oy0 = (t / p.tiles_x) * TT, ox0 = (t % p.tiles_x) * TT;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * NTHR;
      const int pix = it / NS, s = it - pix * NS;
      const int hy = pix / HP, hx = pix - hy * HP;
      const int gy = oy0 - 3 + hy, gx = ox0 - 3 + hx;
      const bool in = it < NPX * NS && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
      const int off = in ? ((gy * p.W + gx) * p.xcs + p.xco + s * 8) * 2 : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto publish = [&]() {
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int it = tid + u * NTHR;
      const int pix = it / NS, s = it - pix * NS;
      if (it < NPX * NS) *reinterpret_cast<u16x8 *>(Li + pix_slot<CIN>(pix, s)) = pf[u];
    }
  };
  issue(g);

  // ---- resident weights: rows n0 .. n0 + BN of the packed [cout][49 * CIN] matrix
  for (int it = tid; it < BN * (KP / 8); it += NTHR) {
    const int n = it / (KP / 8), k8 = (it % (KP / 8)) * 8;
    u16x8 v = u16x8{};
    if (n0 + n < p.cout) v = *reinterpret_cast<const u16x8 *>(p.w + (int64_t)(n0 + n) * KP + k8);
    *reinterpret_cast<u16x8 *>(Lw + n * WP + k8) = v;
  }
  epi::stage_consts(p, Lc, n0, BN);
  const uint16_t *LwA = Lw + col * WP + hi * 8;

  for (int t = g;;) {
    const int oy0 = (t / p.tiles_x) * TT, ox0 = (t % p.tiles_x) * TT;
    // the lane's swizzled B addresses (49 taps x K steps x rows) are
    // recomputed per tile from an opaque copy of the lane id: hoisted out of
    // the tile loop they would be ~100-200 live registers
    int lane_ = lane;
    asm volatile("" : "+v"(lane_));
    const int colq = lane_ & 15, hiq = lane_ >> 4;
    publish();
    __syncthreads();
    const int tn = t + G;
    const bool more = tn < ntiles;
    if (more) issue(tn);

    f32x4 acc[RW][NT];
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 49; ++tap) {
      const int dy = tap / 7, dx = tap % 7;
#pragma unroll
      for (int c = 0; c < KPT; ++c) {
        const int ks = tap * KPT + c;
        bf16x8 a[NT], b[RW];
#pragma unroll
        for (int j = 0; j < NT; ++j) a[j] = *reinterpret_cast<const bf16x8 *>(LwA + j * 16 * WP + ks * 32);
#pragma unroll
        for (int r = 0; r < RW; ++r)
          b[r] = *reinterpret_cast<const bf16x8 *>(Li + pix_slot<CIN>((wave * RW + r + dy) * HP + colq + dx, c * 4 + hiq));
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[r], acc[r][j], 0, 0, 0);
      }
    }
    __syncthreads();  // the image is read: the fp32 tile may overwrite it

#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < NT; ++j) epi::put4(p, T, LD, (wave * RW + r) * TT + col, j * 16 + hi * 4, Lc, acc[r][j]);
    __syncthreads();
    epi::store_tile<TOUT, epi::ipt(TT * TT, BN, NTHR)>(p, T, LD, TT * TT, n0, min(BN, p.cout - n0), Lc, BN,
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
int launch(C7W p, hipStream_t st) {
  typedef GW<CIN, BN> G_;
  static_assert(G_::LDS <= 160 * 1024, "LDS");
  p.tiles_x = (p.W + TT - 1) / TT;
  p.tiles_y = (p.H + TT - 1) / TT;
  p.nblk_n = (p.cout + BN - 1) / BN;
  const int64_t ntiles = (int64_t)p.tiles_x * p.tiles_y;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  // one workgroup per CU over the n-blocks; small maps: one per tile
  int per_n = g_cus / p.nblk_n;
  if (per_n > ntiles) per_n = (int)ntiles;
  const int G = per_n * p.nblk_n;
  auto kern = conv7w_kernel<CIN, BN, TOUT>;
  dcvc_note_kernel("conv7w_kernel<%d, %d, %s>@%lld", CIN, BN, tname<TOUT>(), (long long)G * NTHR);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), (int)G_::LDS);
  hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(NTHR), G_::LDS, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

}  // namespace

// Called by dcvc_conv2d (conv.hip) for 7x7 stride-1 pad-3 bf16 convs with 32
// or 64 input channels; DCVC_HIP_EUNSUPPORTED hands the call back to the
// generic kernel.
extern "C" int dcvc_internal_conv7w(const dcvc_conv_args *a, void *stream) {
  if (!g_enabled) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != 7 || a->kw != 7 || a->stride != 1 || a->pad != 3 || a->compute != DCVC_BF16) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_BF16 || a->in_op != DCVC_IN_NONE || a->shuffle) return DCVC_HIP_EUNSUPPORTED;
  if (a->cin != 32 && a->cin != 64) return DCVC_HIP_EUNSUPPORTED;
  if (a->x.cstride % 8 || a->x.coff % 8 || ((uintptr_t)a->x.ptr & 15)) return DCVC_HIP_EUNSUPPORTED;
  if ((int64_t)a->x.H * a->x.W * a->x.cstride >= ((int64_t)1 << 30) - 16) return DCVC_HIP_EUNSUPPORTED;
  C7W p{};
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
  if (a->y.dtype != DCVC_BF16) return DCVC_HIP_EUNSUPPORTED;
  if (a->cin == 32) return a->cout > 16 ? launch<32, 32, uint16_t>(p, st) : launch<32, 16, uint16_t>(p, st);
  return launch<64, 16, uint16_t>(p, st);
}

// dcvc_set_option("conv7_wide_cin", 0/1) (A/B switch, via conv.hip)
extern "C" void dcvc_internal_conv7w_enable(int v) { g_enabled = v; }
