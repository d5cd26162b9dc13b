// Shared device helpers for the gfx950 kernels of libdcvc_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../../include/dcvc_hip.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

// bf16 is carried as raw uint16 in memory; conversion is round-to-nearest-even
// (v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t *>(&b);
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  __device__ __forceinline__ static float load(const float *p) { return *p; }
  __device__ __forceinline__ static void store(float *p, float v) { *p = v; }
};
template <> struct Elem<uint16_t> {
  __device__ __forceinline__ static float load(const uint16_t *p) { return bf2f(*p); }
  __device__ __forceinline__ static void store(uint16_t *p, float v) { *p = f2bf(v); }
};

template <typename T>
__device__ __forceinline__ float ld(const void *base, int64_t i) {
  return Elem<T>::load(reinterpret_cast<const T *>(base) + i);
}
template <typename T>
__device__ __forceinline__ void st(void *base, int64_t i, float v) {
  Elem<T>::store(reinterpret_cast<T *>(base) + i, v);
}

// Orders a wave's LDS writes before its later LDS reads of the same region by
// other lanes of that wave (and reads before later overwrites) in the
// wave-private phases of the fused kernels.  LDS operations of one wave
// complete in order, so no wait or barrier instruction is needed; the fences
// keep the compiler from moving a read above a write (or a write above a read)
// whose same-lane addresses it can prove disjoint.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Epilogue / prologue activations (see dcvc_act in dcvc_hip.h).
__device__ __forceinline__ float apply_act(int act, float v, float slope) {
  switch (act) {
    case DCVC_ACT_LRELU: return v >= 0.f ? v : v * slope;
    case DCVC_ACT_CLAMP01: return fminf(fmaxf(v, 0.f), 1.f);
    case DCVC_ACT_ROUND: return rintf(v);
    default: return v;
  }
}

// Name of the last kernel instantiation launched by a dcvc_conv2d /
// dcvc_depthconv_block call on this host thread, spelled as rocprofv3 prints
// it ("conv3x3_kernel<48, 16, false, unsigned short>"), so per-launch HIP-event
// timings can be matched to a rocprof kernel summary (dcvc_last_kernel).
void dcvc_note_kernel(const char *fmt, ...);
// Raise kern's dynamic-LDS limit to at least `bytes`, once per process and
// under a lock: setting the attribute while another host thread launches the
// same kernel on another stream (concurrent GOP lanes) is not safe.
void dcvc_ensure_lds(const void *kern, int bytes);
// the calling host thread's fp16 range-guard flag of the split kernels
// (dcvc_split_range_flag; nullptr: guard off), read by their launchers
int *dcvc_internal_split_flag();
template <typename T> constexpr const char *tname();
template <> constexpr const char *tname<float>() { return "float"; }
template <> constexpr const char *tname<uint16_t>() { return "unsigned short"; }
inline const char *bname(bool b) { return b ? "true" : "false"; }

#define DCVC_LAUNCH_CHECK()                          \
  do {                                               \
    hipError_t e__ = hipGetLastError();              \
    if (e__ != hipSuccess) return DCVC_HIP_ELAUNCH;  \
  } while (0)
