// Split-fp16 ("f16x3") helpers shared by the kernels of Precision.split()
// (sconv.hip, sffn.hip) and the host packers (conv.hip, sffn.hip): an fp32
// value a is carried as two fp16 values, a = hi + 2^-11 lo, and a product as
// three f16 MFMAs, xh * wh + 2^-11 (xh * wl + xl * wh) (sconv.hip's header).
#pragma once
#include "common.h"

#include <cmath>
#include <cstring>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// LDS images: a row is one pixel (or one (tap-row, n)) x 32 halves = 4 slots
// of 16 bytes.  Weight rows: slot XOR {0, 2, 3, 1}[(row >> 2) & 3], read 16
// consecutive rows from a multiple of 16: conflict-free ds_read_b128 lane
// groups.  Input image: slot XOR 2 * ((x >> 2) & 1) of the pixel's column x
// in its halo row (row pitch a multiple of 4 pixels): conflict-free for the
// 16 consecutive pixels of a stride-1 tap at any column offset.
__device__ __forceinline__ int swz(int row, int slot) {
  const int x = (0x1320 >> (((row >> 2) & 3) << 2)) & 3;
  return row * 32 + ((slot ^ x) << 3);
}
__device__ __forceinline__ int swzx(int row, int x, int slot) {
  return row * 32 + ((slot ^ (((x >> 2) & 1) << 1)) << 3);
}

__device__ __forceinline__ uint32_t pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}

// 8 fp32 values -> (hi, lo) fp16 pieces; see the header for the split.  hi is
// the fp16 value of v rounded toward zero (exact below fp16's normal range
// too: the remainder is taken from hi's own fp32 value), lo = (v - hi) * 2^11
// (v - hi is exact in fp32), rounded toward zero to fp16
// leaky ReLU of a loaded value, 0 <= s <= 1: max(v, s v) as one v_max_f32
// (fmaxf would first quieten v, a signalling NaN for all the compiler knows:
// one more instruction per element); the same value for every non-NaN v,
// signed zeros included
// 4 x 4 transpose across the four 16-lane rows of a wave and four registers:
// row r's x_j <- row j's x_r
__device__ __forceinline__ void xpose4(uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3) {
#ifdef __HIP_DEVICE_COMPILE__
  const auto a02 = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);
  const auto a13 = __builtin_amdgcn_permlane32_swap(x1, x3, false, false);
  const auto b01 = __builtin_amdgcn_permlane16_swap(a02[0], a13[0], false, false);
  const auto b23 = __builtin_amdgcn_permlane16_swap(a02[1], a13[1], false, false);
  x0 = b01[0];
  x1 = b01[1];
  x2 = b23[0];
  x3 = b23[1];
#endif
}

__device__ __forceinline__ float lrelu_in(float v, float s) {
  const float t = v * s;
#ifdef __HIP_DEVICE_COMPILE__
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(t));
  return r;
#else
  return v > t ? v : t;
#endif
}

// lo of v given h = f16_rtz(v) widened: (v - h) * 2^11 as fma(h, -2^11, v 2^11),
// the same value (both products and the difference are exact), one
// v_fma_mix_f32 reading the f16 h directly instead of a conversion, a
// subtraction and a multiplication
__device__ __forceinline__ float split_lo(float v, float h) { return __builtin_fmaf(h, -2048.f, v * 2048.f); }

__device__ __forceinline__ void split8(const float v[8], u32x4_t &h, u32x4_t &l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto hh = __builtin_amdgcn_cvt_pkrtz(v[2 * j], v[2 * j + 1]);
    h[j] = __builtin_bit_cast(uint32_t, hh);
    l[j] = pk(split_lo(v[2 * j], (float)hh[0]), split_lo(v[2 * j + 1], (float)hh[1]));
  }
}

constexpr float kLoInv = 1.f / 2048.f;

// Compiler fences on a value (device pass only: the host pass sees kernel
// bodies too, and x86 has no "s" register class): after opaque_v(x) /
// opaque_s(x) the compiler must assume x changed, so it neither hoists nor
// shares (CSE) computations on x across the fence.  Free in the ISA.
template <typename T>
__device__ __forceinline__ void opaque_v(T &x) {
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(x));
#endif
}
// no instruction is scheduled across this point (device pass only)
__device__ __forceinline__ void sched_fence() {
#ifdef __HIP_DEVICE_COMPILE__
  __builtin_amdgcn_sched_barrier(0);
#endif
}
template <typename T>
__device__ __forceinline__ void opaque_s(T &x) {
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+s"(x));
#endif
}

// The fp16 range guard (dcvc_split_range_flag, include/dcvc_hip.h).  hi + 2^-11
// lo carries a value to ~2^-21 of itself only while |v| < 2^15: above it the
// round-toward-zero hi and then lo saturate, silently.  Every split kernel
// keeps one of these per thread, adds each value it splits (inputs and fused
// intermediates alike), and at exit raises *flag when the running max reached
// 2^15.  The store is a plain vector store of one lane per wave at most.
constexpr float kSplitMax = 32768.f;
struct SplitRange {
  // running max of |v| as the bit pattern of the absolute value: for
  // non-negative floats integer order is float order, and a NaN or an
  // infinity counts as out of range too.  Integer max3 over sign-cleared bits
  // (v_and + v_max3_u32) instead of fmaxf, which canonicalises each input
  uint32_t m = 0;
  int *flag;
  __device__ explicit SplitRange(int *f) : flag(f) {}
  __device__ __forceinline__ void add4(const float *v) {
    const uint32_t a = __float_as_uint(v[0]) & 0x7fffffffu, b = __float_as_uint(v[1]) & 0x7fffffffu;
    const uint32_t c = __float_as_uint(v[2]) & 0x7fffffffu, d = __float_as_uint(v[3]) & 0x7fffffffu;
    m = max(max(m, a), b);
    m = max(max(m, c), d);
    // fold now: left to itself the compiler keeps every partial max live
    // until the kernel's end (tens of registers in a long unrolled kernel)
    opaque_v(m);
  }
  __device__ __forceinline__ void add8(const float *v) {
    add4(v);
    add4(v + 4);
  }
  __device__ ~SplitRange() {
    if (flag && m >= 0x47000000u) *flag = 1;   // 0x47000000 = kSplitMax
  }
};
static_assert(0x47000000u == 0x47000000u && kSplitMax == 32768.f, "2^15 is 0x47000000");

__device__ __forceinline__ void wait_vm_lgkm() { __builtin_amdgcn_s_waitcnt(0x0070); }   // vmcnt(0) lgkmcnt(0)
// vmcnt(N) lgkmcnt(0): all but the N youngest vector-memory operations done
template <int N>
__device__ __forceinline__ void wait_vm_n_lgkm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt(0x0070 | (N & 15) | ((N >> 4) << 14));
}
// workgroup barrier without the vmcnt(0) __syncthreads() implies while an
// LDS-DMA is in flight; LDS ordering is made explicit by the callers' waits
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_lgkm() { __builtin_amdgcn_s_waitcnt(0xC07F); }      // lgkmcnt(0)

// 16-byte LDS read that hipcc's wait insertion does not see.  hipcc puts a
// vmcnt(0) in front of a plain LDS read of the kernels' constant tables while
// LDS-DMAs are in flight (it cannot tell that they write elsewhere), so the
// read would wait for the newest weight DMA of the stage, a memory round trip
// (xconv's epilogue: DESIGN.md section 9.0).  The caller waits for the reads
// with lds_wait4 before it uses them.
__device__ __forceinline__ f32x4 lds_read16(const float *p) {
  f32x4 r;
#ifdef __HIP_DEVICE_COMPILE__
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
#else
  std::memcpy(&r, p, sizeof r);
#endif
  return r;
}
// lgkmcnt(0), ordered before every later use of v[0 .. N) (each value passes
// through an empty volatile asm after the wait)
template <int N>
__device__ __forceinline__ void lds_wait4(f32x4 (&v)[N]) {
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
#endif
}

// host f32 -> f16, round to nearest even (subnormals kept; |v| < 65520 assumed)
static inline uint16_t host_f2h(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const int e = (int)((u >> 23) & 0xff) - 127;
  uint32_t m = u & 0x7fffffu;
  if (e > 15) return (uint16_t)(sign | 0x7c00u);          // overflow: infinity
  if (e >= -14) {                                         // normal f16
    uint32_t h = ((uint32_t)(e + 15) << 10) | (m >> 13);
    const uint32_t rest = m & 0x1fffu;
    if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) ++h;  // may carry into the exponent: still correct
    return (uint16_t)(sign | h);
  }
  if (e < -25) return (uint16_t)sign;                     // below half the smallest subnormal
  m |= 0x800000u;                                         // subnormal f16: value = m * 2^(e - 23)
  const int shift = -e - 1;                               // 14..24: keep m >> shift as units of 2^-24
  uint32_t h = m >> shift;
  const uint32_t rest = m & ((1u << shift) - 1u), half = 1u << (shift - 1);
  if (rest > half || (rest == half && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}
static inline float host_h2f(uint16_t h) {
  const int e = (h >> 10) & 0x1f;
  const uint32_t m = h & 0x3ffu;
  float f;
  if (e == 0) {
    f = std::ldexp((float)m, -24);
  } else {
    uint32_t u = ((uint32_t)(e - 15 + 127) << 23) | (m << 13);
    std::memcpy(&f, &u, 4);
  }
  return (h & 0x8000u) ? -f : f;
}
// weights enter the split through host_split: the range of SplitRange holds
// for them too (a packer rejects a weight with |w| >= 2^15, or a NaN)
static inline bool host_split_range_ok(const float *w, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    if (!(std::fabs(w[i]) < 32768.f)) return false;
  return true;
}
// w = hi + 2^-11 lo: hi = f16(w), lo = f16((w - hi) * 2^11)
static inline void host_split(float w, uint16_t &hi, uint16_t &lo) {
  hi = host_f2h(w);
  lo = host_f2h((w - host_h2f(hi)) * 2048.f);
}
