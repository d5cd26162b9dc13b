// Direct split-fp16 convolution for the layers whose input pixels are reused
// by few outputs: stride-2 3x3 / 1x1 convolutions (the strided encoders,
// DCVC-DC/src/models/video_model.py:66-86, 173-195; ResidualBlockWithStride,
// layers.py) and the feature-rate 1x1 convolutions (DepthConv conv1 / conv2
// / adaptor, subpel_conv1x1 upsamplers, layers.py:23-34, 135-163).  Same arithmetic as sconv.hip: x * w ~
// xh*wh + 2^-11 (xh*wl + xl*wh) on v_mfma_f32_16x16x32_f16 with fp32
// accumulation, the same K order (32-channel chunks, taps inside a chunk,
// dcvc_conv_pack_weights' F16X3 layout) and the same epilogue, so the
// outputs are sconv_kernel's bit for bit.
//
// What differs is the data flow.  sconv / xconv stage a halo image of the
// input in LDS, split once, because a stride-1 3x3 tap reuses every input
// pixel nine times; at stride 2 a pixel feeds 2.25 outputs on average (a
// 1x1 layer not at all), and the stride-2 halo image (2 TH + 1 rows of 2 x 16 + 1 columns) no longer fits beside the
// weights.  Here:
//   * the weights of the workgroup's output-channel block are resident in
//     LDS for the launch (one LDS-DMA pass, swizzled for conflict-free
//     16-byte fragment reads);
//   * each wave owns runs of NP x 16 output pixels of one row and loads its
//     B operands (lane (col, q): pixel col, the 8 channels of K slot q) from
//     global memory (L2 / L1) straight into registers, splits them there,
//     DEPTH K steps ahead of their MFMAs;
//   * waves never wait for each other: no barrier after the weight load.
#include "common.h"
#include "split.h"

#include <cstring>
#include <utility>

namespace {

struct DP {
  const float *x;
  int H, W, xcs, xco;
  const uint16_t *w;
  int wbytes;
  float *y;
  int Ho, Wo, ycs, yco;
  int cin, cout, kt, S, pad;
  int nch, tpkl, nst;      // 32-channel chunks, taps packed in the last one, K steps
  int64_t wchunk;          // halves of one full chunk's block (hi + lo)
  int in_lrelu;
  float in_slope;
  int act;
  float slope;
  const float *bias, *scale;
  int nblk, nseg, ntiles;  // output-channel blocks, row segments, tiles (rows x segments)
  int vec_out;             // 16-byte output pieces (4-aligned channel view)
  const float *res, *res2; // residuals (output views) or NULL
  int rcs, rco, r2cs, r2co;
  int shuffle;             // pixel_shuffle(2) on store (output H, W doubled, channels / 4)
  int xcd;                 // XCD-aware n-block mapping (grid a multiple of 8 nblk)
  int *ovf;
};

template <int KS, int BN, int NP>
struct DG {
  static constexpr int NW = 8, NTH = NW * 64, NT = BN / 16;
};
constexpr int DEPTH = 4;

template <typename F, int... I>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}

template <int KS, int BN, int NP, bool GATE>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) dconv_kernel(DP p) {
  typedef DG<KS, BN, NP> G;
  constexpr int NT = G::NT, NW = G::NW;
  SplitRange rg(p.ovf);
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t *const L = reinterpret_cast<uint16_t *>(smem);
  const int nst = p.nst;
  float *const Lc = reinterpret_cast<float *>(smem + (size_t)nst * 2 * BN * 32 * 2);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int col = lane & 15, q = lane >> 4;
  const int GR = gridDim.x;
  // workgroup -> (output-channel block, first tile): the block is fixed per
  // workgroup, so its weights are loaded once
  int nb = blockIdx.x % p.nblk, gs = blockIdx.x / p.nblk;
  if (p.xcd) {
    // workgroups are dealt to the 8 XCDs round robin: the nblk workgroups
    // that walk the same tiles (one per n-block) on one XCD, so all but the
    // first read each input pixel from that XCD's L2
    const int b = blockIdx.x >> 3;
    nb = b % p.nblk;
    gs = (blockIdx.x & 7) + 8 * (b / p.nblk);
  }
  const int GS = GR / p.nblk;
  if (gs >= GS) return;
  const int n0 = nb * BN;

  // ---- resident weights: step st (chunk c, row r), hi then lo, 16-row blocks
  {
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(p.w), (short)0, p.wbytes, 0x00020000);
    const int npieces = nst * 2 * NT;
    const int R = lane >> 2;
    const int ls = (lane & 3) ^ ((0x1320 >> (((R >> 2) & 3) << 2)) & 3);
    for (int i = wave; i < npieces; i += NW) {
      const int j = i % NT, hl = (i / NT) & 1, st = i / (2 * NT);
      const int c = st < (p.nch - 1) * p.kt ? st / p.kt : p.nch - 1;
      const int r = st - c * p.kt;
      const int rows = c == p.nch - 1 ? (p.kt + p.tpkl - 1) / p.tpkl : p.kt;
      const int n = n0 + j * 16 + R;
      const int64_t src = c * p.wchunk + (int64_t)hl * rows * p.cout * 32 + ((int64_t)r * p.cout + n) * 32 + ls * 8;
      const int off = n < p.cout ? (int)(src * 2) : 0x7ffffff0;
#ifdef __HIP_DEVICE_COMPILE__
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void *)(L + (size_t)i * 512), 16,
                                               off, 0, 0, 0);
#endif
    }
    for (int i = tid; i < BN; i += G::NTH) {
      const int n = n0 + i;
      Lc[i] = p.bias && n < p.cout ? p.bias[n] : 0.f;
      // (pixel shuffle: the scale of output channel n0 / 4 + i, i < BN / 4)
      const int ns = p.shuffle ? (n0 >> 2) + i : n;
      const bool sv = p.shuffle ? i < BN / 4 && ns < p.cout / 4 : n < p.cout;
      Lc[BN + i] = p.scale && sv ? p.scale[ns] : 1.f;
    }
    wait_vm_lgkm();
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(p.x), (short)0,
      (int)((int64_t)p.H * p.W * p.xcs * 4 < 0x7fff0000 ? (int64_t)p.H * p.W * p.xcs * 4 : 0x7fff0000), 0x00020000);
  const int aoff = swz(col, q);
  const int spl = 4 / p.tpkl;             // 8-channel slots per tap in the last chunk

  // wave-level tiles: tile = (output row, segment of NP x 16 pixels)
  const int gw = gs * NW + wave, GW = GS * NW;
  int t = gw;
  if (t >= p.ntiles) return;
  // the (tile, K step) whose operands load next, wave-uniform: tile ta at
  // output row ly, first column lx; step = chunk lc, row lr of the chunk
  int ta = t, ly = t / p.nseg, lx = (t - ly * p.nseg) * (16 * NP), lc = 0, lr = 0;
  // 1x1 layers: the one tap's input pixel of each lane's output pixels, as a
  // byte offset (-1 outside the tile / image), set once per tile, so a K
  // step's address is that plus its channel offset (the generic path below
  // recomputes the pixel index, a per-lane multiply by the channel stride,
  // every step)
  int obase[NP];
  auto setup = [&]() __attribute__((always_inline)) {
    if constexpr (KS == 1) {
      const int iy = ly * p.S - p.pad;
      const bool rowok = ta < p.ntiles && (unsigned)iy < (unsigned)p.H;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int ox = lx + j * 16 + col;
        const int ix = ox * p.S - p.pad;
        const bool ok = rowok && (unsigned)ix < (unsigned)p.W && ox < p.Wo;
        obase[j] = ok ? ((iy * p.W + ix) * p.xcs + p.xco) * 4 : -1;
      }
    }
  };
  setup();
  auto next = [&]() __attribute__((always_inline)) {
    ++lr;
    if (lc < p.nch - 1 && lr == p.kt) {
      ++lc;
      lr = 0;
    } else if (lc == p.nch - 1 && lr == (p.kt + p.tpkl - 1) / p.tpkl) {
      lc = 0;
      lr = 0;
      ta += GW;
      ly = ta / p.nseg;
      lx = (ta - ly * p.nseg) * (16 * NP);
      setup();
    }
  };
  // B-operand raw loads of the next (tile, step) into pr (GATE: the gate
  // half of the input, channels cin + ch .., in pr[j][8 ..])
  constexpr int PW = GATE ? 16 : 8;
  auto load = [&](float (&pr)[NP][PW]) __attribute__((always_inline)) {
    int tap, ch;
    if (lc < p.nch - 1) {
      tap = lr;
      ch = lc * 32 + q * 8;
    } else {
      tap = p.tpkl * lr + q / spl;
      ch = lc * 32 + (q % spl) * 8;
    }
    const int dy = tap / KS, dx = tap - dy * KS;
    const int iy = ly * p.S + dy - p.pad;
    const bool rowok = ta < p.ntiles && tap < p.kt && ch < p.cin && (unsigned)iy < (unsigned)p.H;
    const bool chok = tap < p.kt && ch < p.cin;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      int o;
      bool ok;
      if constexpr (KS == 1) {
        ok = chok && obase[j] >= 0;
        o = ok ? obase[j] + ch * 4 : 0x7fffffe0;
      } else {
        const int ox = lx + j * 16 + col;
        const int ix = ox * p.S + dx - p.pad;
        ok = rowok && (unsigned)ix < (unsigned)p.W && ox < p.Wo;
        o = ok ? ((iy * p.W + ix) * p.xcs + p.xco + ch) * 4 : 0x7fffffe0;
      }
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o + 16, 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pr[j][e] = a[e];
        pr[j][4 + e] = b[e];
      }
      if constexpr (GATE) {
        const int og = ok ? o + p.cin * 4 : 0x7fffffe0;
        const f32x4 ga = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, og, 0, 0));
        const f32x4 gb = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, og + 16, 0, 0));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pr[j][8 + e] = ga[e];
          pr[j][12 + e] = gb[e];
        }
      }
    }
  };
  // DEPTH steps of operand loads in flight (the L2 / HBM latency of a
  // step's loads is covered by the MFMAs of the DEPTH - 1 steps before it)
  float pr[DEPTH][NP][PW];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    load(pr[d]);
    next();
  }
  f32x4 am[NP][NT], ac[NP][NT];
  auto zero = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NP; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        am[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        ac[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
  };
  zero();
  // one K step from the raw operands pr (then refilled with the step two ahead)
  auto step = [&](int st, float (&pr)[NP][PW]) __attribute__((always_inline)) {
    f16x8 bh[NP], bl[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if constexpr (GATE) {
        // ConvFFN2's gate (sconv.hip's order): x1 * lrelu(x2)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gv = pr[j][8 + e];
          pr[j][e] = pr[j][e] * (gv >= 0.f ? gv : gv * p.in_slope);
        }
      } else if (p.in_lrelu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) pr[j][e] = lrelu_in(pr[j][e], p.in_slope);
      }
      u32x4_t h, l;
      rg.add8(pr[j]);
      split8(pr[j], h, l);
      bh[j] = __builtin_bit_cast(f16x8, h);
      bl[j] = __builtin_bit_cast(f16x8, l);
    }
    load(pr);
    next();
    const uint16_t *Lw = L + (size_t)st * 2 * NT * 512 + aoff;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const f16x8 ah = *reinterpret_cast<const f16x8 *>(Lw + n * 512);
      const f16x8 al = *reinterpret_cast<const f16x8 *>(Lw + (NT + n) * 512);
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        am[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], am[j][n], 0, 0, 0);
        ac[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], ac[j][n], 0, 0, 0);
        ac[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], ac[j][n], 0, 0, 0);
      }
    }
  };
  // out = scale * (res2 + (res + act((am + 2^-11 ac) + bias))), sconv's
  // order; with pixel shuffle (r = 2) conv channel 4 c + 2 dy + dx of pixel
  // (oy, ox) is output channel c of pixel (2 oy + dy, 2 ox + dx), scaled by
  // the output channel's scale
  auto epilogue = [&](int tt) __attribute__((always_inline)) {
    const int oy = tt / p.nseg, ox0 = (tt - oy * p.nseg) * (16 * NP);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int ox = ox0 + j * 16 + col;
      const bool live = ox < p.Wo;
      uint32_t sh[4][4];   // (pixel shuffle, NT % 4 == 0) a group of four n
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int c = n * 16 + q * 4;
        const float4 bb = *reinterpret_cast<const float4 *>(Lc + c);
        f32x4 v;
        v[0] = (am[j][n][0] + ac[j][n][0] * kLoInv) + bb.x;
        v[1] = (am[j][n][1] + ac[j][n][1] * kLoInv) + bb.y;
        v[2] = (am[j][n][2] + ac[j][n][2] * kLoInv) + bb.z;
        v[3] = (am[j][n][3] + ac[j][n][3] * kLoInv) + bb.w;
        if (p.act == DCVC_ACT_LRELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], v[e] * p.slope);
        }
        if (p.shuffle && p.cout % 16) {
          // (narrow upsampler, subpel_conv1x1 to 4 x 2 channels: element
          // stores) conv channel n0 + c + e -> output channel (n0 + c) / 4 of
          // sub-pixel e
          const int cc = n0 + c;
          if (live && cc < p.cout) {
            const float s = Lc[BN + c / 4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int ry = 2 * oy + (e >> 1), cx = 2 * ox + (e & 1);
              p.y[((int64_t)ry * 2 * p.Wo + cx) * p.ycs + p.yco + cc / 4] = v[e] * s;
            }
          }
          continue;
        }
        if (p.shuffle) {
          // lane row q holds conv channels n0 + 16 n + 4 q + e: a 4 x 4
          // transpose across the rows gives row q the 4 consecutive output
          // channels (n0 + 16 n) / 4 + e of sub-pixel q (xconv.hip's epilogue)
          uint32_t x0 = __float_as_uint(v[0]), x1 = __float_as_uint(v[1]);
          uint32_t x2 = __float_as_uint(v[2]), x3 = __float_as_uint(v[3]);
          xpose4(x0, x1, x2, x3);
          if constexpr (NT % 4 == 0) {
            // groups of four n: a second transpose, across (row, n), gives row
            // q the output channels (n0 + 64 g) / 4 + 4 q .. + 3 of every
            // sub-pixel, so the 4 rows store 64 contiguous bytes of one
            // output pixel per instruction (not 16 bytes of 4 pixels)
            const int g = n >> 2, k = n & 3;
            sh[k][0] = x0;
            sh[k][1] = x1;
            sh[k][2] = x2;
            sh[k][3] = x3;
            if (k == 3) {
#pragma unroll
              for (int e = 0; e < 4; ++e) xpose4(sh[0][e], sh[1][e], sh[2][e], sh[3][e]);
              const int cl = 16 * g + 4 * q;   // the lane's 4 channels, relative to n0 / 4
              const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + cl);
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                f32x4 o;
                o[0] = __uint_as_float(sh[s][0]) * sc.x;
                o[1] = __uint_as_float(sh[s][1]) * sc.y;
                o[2] = __uint_as_float(sh[s][2]) * sc.z;
                o[3] = __uint_as_float(sh[s][3]) * sc.w;
                const int ry = 2 * oy + (s >> 1), cx = 2 * ox + (s & 1);
                if (live && n0 + 64 * g + 16 * q < p.cout)   // (row q: n = 4 g + q)
                  *reinterpret_cast<f32x4 *>(p.y + ((int64_t)ry * 2 * p.Wo + cx) * p.ycs + p.yco + (n0 >> 2) + cl) = o;
              }
            }
            continue;
          }
          const int cb = (n0 >> 2) + 4 * n;   // first output channel of the 16-channel group
          const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + 4 * n);
          f32x4 o;
          o[0] = __uint_as_float(x0) * sc.x;
          o[1] = __uint_as_float(x1) * sc.y;
          o[2] = __uint_as_float(x2) * sc.z;
          o[3] = __uint_as_float(x3) * sc.w;
          const int ry = 2 * oy + (q >> 1), cx = 2 * ox + (q & 1);
          if (live && n0 + 16 * n < p.cout)
            *reinterpret_cast<f32x4 *>(p.y + ((int64_t)ry * 2 * p.Wo + cx) * p.ycs + p.yco + cb) = o;
          continue;
        }
        if (!live || n0 + c >= p.cout) continue;
        const int64_t pix = (int64_t)oy * p.Wo + ox;
        if (p.res) {
          const f32x4 r = *reinterpret_cast<const f32x4 *>(p.res + pix * p.rcs + p.rco + n0 + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = r[e] + v[e];
        }
        if (p.res2) {
          const f32x4 r = *reinterpret_cast<const f32x4 *>(p.res2 + pix * p.r2cs + p.r2co + n0 + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = r[e] + v[e];
        }
        if (p.scale) {
          const float4 sc = *reinterpret_cast<const float4 *>(Lc + BN + c);
          v[0] *= sc.x;
          v[1] *= sc.y;
          v[2] *= sc.z;
          v[3] *= sc.w;
        }
        float *yp = p.y + pix * p.ycs + p.yco;
        if (p.vec_out) {
          *reinterpret_cast<f32x4 *>(yp + n0 + c) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n0 + c + e < p.cout) yp[n0 + c + e] = v[e];
        }
      }
    }
  };
  // the steps of consecutive tiles form one stream: step (tile, st) uses the
  // ring slot of its position in the stream
  int cs = 0;
  while (t < p.ntiles) {
    sfor<DEPTH>([&](auto D_) {
      constexpr int d = decltype(D_)::value;
      if (t < p.ntiles) {
        step(cs, pr[d]);
        if (++cs == nst) {
          epilogue(t);
          zero();
          cs = 0;
          t += GW;
        }
      }
    });
  }
  wait_vm_lgkm();
}

int g_cus = 0;
int g_enable = 1;   // dcvc_set_option("dconv", 0): route these layers to sconv.hip
int g_k1 = 1;       // dcvc_set_option("dconv_1x1", 0): stride-1 1x1 layers to sgemm.hip
int g_bn128 = 1;   // dcvc_set_option("dconv_bn128", 0): 64-channel n-blocks for 1x1 layers (A/B)
int g_s2blk = 2;   // dcvc_set_option("dconv_s2blocks", n): most n-blocks of a 3x3 layer (A/B)
int g_gate = 1;     // dcvc_set_option("dconv_gate", 0): ConvFFN2's gated 1x1 to sconv.hip
int g_xcd = 1;      // dcvc_set_option("dconv_xcd", 0): n-blocks of a tile on different XCDs (A/B)

template <int KS, int BN, int NP, bool GATE = false>
int launch(DP p, hipStream_t st) {
  const size_t lds = (size_t)p.nst * 2 * BN * 32 * 2 + (size_t)2 * BN * 4;
  if (lds > 160 * 1024) return DCVC_HIP_EUNSUPPORTED;
  p.nblk = (p.cout + BN - 1) / BN;
  p.nseg = (p.Wo + 16 * NP - 1) / (16 * NP);
  const int64_t nt = (int64_t)p.Ho * p.nseg;
  if (nt <= 0) return DCVC_HIP_OK;
  if (nt > 0x7fffffff) return DCVC_HIP_EINVAL;
  p.ntiles = (int)nt;
  if (g_cus <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      return DCVC_HIP_ELAUNCH;
    g_cus = prop.multiProcessorCount;
  }
  // one workgroup per CU, a whole number of output-channel blocks; no more
  // workgroups per block than its tiles need (8 waves each)
  int64_t per = (g_cus + p.nblk - 1) / p.nblk;
  const int64_t need = (nt + 7) / 8;
  if (per > need) per = need;
  if (per < 1) per = 1;
  const int64_t grid = per * p.nblk;
  p.xcd = p.nblk > 1 && g_xcd && grid % (8 * p.nblk) == 0;
  auto kern = dconv_kernel<KS, BN, NP, GATE>;
  dcvc_note_kernel("dconv_kernel<%d, %d, %d, %s>@%lld", KS, BN, NP, GATE ? "true" : "false", (long long)grid * 512);
  dcvc_ensure_lds(reinterpret_cast<const void *>(kern), 160 * 1024);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, st, p);
  DCVC_LAUNCH_CHECK();
  return DCVC_HIP_OK;
}

// n-block: all of cout when its weights fit LDS, else the widest of 64 / 48 /
// 32 / 16 that does (each block then re-reads the input: more than two
// blocks of a 3x3 layer lose to sconv.hip's halo image)
// ConvFFN2's gated second 1x1 (in_op DCVC_IN_GATE: x1 * lrelu(x2) of the
// two halves of a 2 cin-channel input): one 16-pixel group per wave, the
// gate half's loads beside the value half's
int pick_gate(DP p, hipStream_t st) {
  auto fits = [&](int bn) { return (size_t)p.nst * 2 * bn * 32 * 2 + (size_t)2 * bn * 4 <= 160 * 1024; };
  if (p.cout % 64 == 0 && fits(64)) return launch<1, 64, 1, true>(p, st);
  if (p.cout % 48 == 0 && fits(48)) return launch<1, 48, 1, true>(p, st);
  if (p.cout % 32 == 0 && fits(32)) return launch<1, 32, 1, true>(p, st);
  if (fits(16)) return launch<1, 16, 1, true>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

template <int KS, int NP>
int pick(DP p, hipStream_t st) {
  auto fits = [&](int bn) {
    return (size_t)p.nst * 2 * bn * 32 * 2 + (size_t)2 * bn * 4 <= 160 * 1024 && (KS == 1 || g_s2blk * bn >= p.cout);
  };
  if (p.cout % 16) return fits(16) ? launch<KS, 16, NP>(p, st) : DCVC_HIP_EUNSUPPORTED;
  // (1x1 with 128-channel multiples: one 128-row block of one 16-pixel group
  // per wave reads the input once instead of once per 64-channel block;
  // 64 -> 128 + shuffle at 544 x 960 110 -> 103 us, 64 -> 256 + shuffle at
  // 272 x 480 50 -> 47 us, profiles/r05m_dconv_shuffle_bn128_ab.jsonl)
  if (KS == 1 && g_bn128 && p.cout % 128 == 0 && fits(128)) return launch<KS, 128, 1>(p, st);
  if (p.cout % 64 == 0 && fits(64)) return launch<KS, 64, NP>(p, st);
  if (p.cout % 48 == 0 && fits(48)) return launch<KS, 48, NP>(p, st);
  if (p.cout % 32 == 0 && fits(32)) return launch<KS, 32, NP>(p, st);
  if (fits(16)) return launch<KS, 16, NP>(p, st);
  return DCVC_HIP_EUNSUPPORTED;
}

}  // namespace

extern "C" void dcvc_internal_dconv_enable(int v) { g_enable = v; }
extern "C" void dcvc_internal_dconv_1x1(int v) { g_k1 = v; }
extern "C" void dcvc_internal_dconv_xcd(int v) { g_xcd = v; }
extern "C" void dcvc_internal_dconv_gate(int v) { g_gate = v; }
extern "C" void dcvc_internal_dconv_s2blocks(int v) { g_s2blk = v; }
extern "C" void dcvc_internal_dconv_bn128(int v) { g_bn128 = v; }

// Stride-2 3x3 / 1x1 and feature-rate 1x1 f16x3 convolutions with fp32
// views (dcvc_conv2d tries it before sconv.hip).  DCVC_HIP_EUNSUPPORTED:
// shapes / views / options it does not take.
extern "C" int dcvc_internal_dconv(const dcvc_conv_args *a, void *stream) {
  if (!g_enable) return DCVC_HIP_EUNSUPPORTED;
  if (a->kh != a->kw || a->pad != a->kh / 2) return DCVC_HIP_EUNSUPPORTED;
  // taken where it beats sconv / sgemm (scripts/sconv_bench.py A/B,
  // profiles/r05*_micro.jsonl): stride 2; stride-1 1x1 on feature-rate maps
  // (>= 64 Ki pixels: at the 68 x 120 latent rate a wave gets one tile and
  // its K loop's load latency shows; sgemm.hip keeps those)
  const bool s2 = a->stride == 2 && (a->kh == 3 || a->kh == 1);
  const bool k1 = a->stride == 1 && a->kh == 1 && g_k1 && (int64_t)a->x.H * a->x.W >= 65536;
  // (stride-1 3x3 / 7x7 layers with fewer than 16 output channels stay on
  // sconv.hip: 48 -> 3 3x3 at 1080p 204 us there vs 337 us here, 16 -> 2 7x7
  // 375 vs 525 us, profiles/r05k_micro.jsonl)
  // (SpyNet's first 7x7, 8 -> 32, stays on sconv.hip: 383 vs 366 us here,
  // profiles/r05w_nconv_micro.jsonl)
  if (!s2 && !k1) return DCVC_HIP_EUNSUPPORTED;
  if (a->shuffle && (!k1 || a->cout % 4 || a->res.ptr || a->res2.ptr)) return DCVC_HIP_EUNSUPPORTED;
  if (a->res2.ptr && !a->res.ptr) return DCVC_HIP_EUNSUPPORTED;
  const bool gate = a->in_op == DCVC_IN_GATE;
  if (gate && (!k1 || !g_gate || a->shuffle)) return DCVC_HIP_EUNSUPPORTED;
  if (a->in_op != DCVC_IN_NONE && !gate && !(a->in_op == DCVC_IN_LRELU && a->in_slope >= 0.f && a->in_slope <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->act != DCVC_ACT_NONE && !(a->act == DCVC_ACT_LRELU && a->slope >= 0.f && a->slope <= 1.f))
    return DCVC_HIP_EUNSUPPORTED;
  if (a->x.dtype != DCVC_F32 || a->y.dtype != DCVC_F32) return DCVC_HIP_EUNSUPPORTED;
  if (a->cin % 8 || (uintptr_t)a->x.ptr % 16 || a->x.cstride % 4 || a->x.coff % 4) return DCVC_HIP_EUNSUPPORTED;
  auto vec_ok = [&](const dcvc_tensor &t) {
    return (uintptr_t)t.ptr % 16 == 0 && t.cstride % 4 == 0 && t.coff % 4 == 0 && t.dtype == DCVC_F32;
  };
  if (a->res.ptr && (!vec_ok(a->res) || a->cout % 4)) return DCVC_HIP_EUNSUPPORTED;
  if (a->res2.ptr && !vec_ok(a->res2)) return DCVC_HIP_EUNSUPPORTED;
  if (a->shuffle && a->cout % 16 == 0 && !vec_ok(a->y)) return DCVC_HIP_EUNSUPPORTED;
  DP p{};
  // outputs: 16-byte pieces of 4 channels where the view allows, else
  // element stores (SpyNet's 2-channel flow)
  p.vec_out = (uintptr_t)a->y.ptr % 16 == 0 && a->y.cstride % 4 == 0 && a->y.coff % 4 == 0 && a->cout % 4 == 0;
  p.ovf = dcvc_internal_split_flag();
  p.x = reinterpret_cast<const float *>(a->x.ptr);
  p.H = a->x.H;
  p.W = a->x.W;
  p.xcs = a->x.cstride;
  p.xco = a->x.coff;
  p.w = reinterpret_cast<const uint16_t *>(a->w);
  p.y = reinterpret_cast<float *>(a->y.ptr);
  p.S = a->stride;
  p.pad = a->pad;
  p.Ho = (a->x.H + 2 * a->pad - a->kh) / a->stride + 1;
  p.Wo = (a->x.W + 2 * a->pad - a->kw) / a->stride + 1;
  const int f = a->shuffle ? 2 : 1;
  if (a->y.H != p.Ho * f || a->y.W != p.Wo * f) return DCVC_HIP_EUNSUPPORTED;
  p.shuffle = a->shuffle ? 1 : 0;
  if (a->res.ptr) {
    p.res = reinterpret_cast<const float *>(a->res.ptr);
    p.rcs = a->res.cstride;
    p.rco = a->res.coff;
  }
  if (a->res2.ptr) {
    p.res2 = reinterpret_cast<const float *>(a->res2.ptr);
    p.r2cs = a->res2.cstride;
    p.r2co = a->res2.coff;
  }
  p.ycs = a->y.cstride;
  p.yco = a->y.coff;
  p.cin = a->cin;
  p.cout = a->cout;
  p.kt = a->kh * a->kw;
  p.nch = (a->cin + 31) / 32;
  const int vcl = a->cin - 32 * (p.nch - 1);
  p.tpkl = vcl <= 8 ? 4 : vcl <= 16 ? 2 : 1;
  p.nst = (p.nch - 1) * p.kt + (p.kt + p.tpkl - 1) / p.tpkl;
  p.wchunk = (int64_t)2 * p.kt * a->cout * 32;
  const int64_t wb = ((int64_t)(p.nch - 1) * p.wchunk + (int64_t)2 * ((p.kt + p.tpkl - 1) / p.tpkl) * a->cout * 32) * 2;
  if (wb >= ((int64_t)1 << 31) - 64) return DCVC_HIP_EUNSUPPORTED;
  p.wbytes = (int)wb;
  p.in_lrelu = a->in_op == DCVC_IN_LRELU;
  p.in_slope = a->in_slope;
  p.act = a->act;
  p.slope = a->slope;
  p.bias = a->bias;
  p.scale = a->scale;
  // 32-bit element offsets of the input and output maps; the input's buffer
  // record is clamped to 0x7fff0000 bytes (kernel), so a larger input map
  // would read zeros in its last 64 KiB: refused here instead
  if ((int64_t)p.H * p.W * p.xcs * 4 >= 0x7fff0000 || (int64_t)p.Ho * p.Wo * 4 * p.ycs >= ((int64_t)1 << 29))
    return DCVC_HIP_EUNSUPPORTED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // cout < 16: one 16-row block, rows past cout are zero weights, their
  // outputs not stored
  if (gate) return pick_gate(p, st);
  switch (a->kh) {
    case 1: return pick<1, 2>(p, st);
    case 3: return pick<3, 2>(p, st);
    default: return DCVC_HIP_EUNSUPPORTED;
  }
}
