// Sustained v_mfma_f32_16x16x32_f16 rate of this GPU (a calibration of the
// f16x3 roofline's peak): every SIMD of every CU runs
// waves that issue back-to-back MFMAs on NACC independent accumulators, with
// random or zero fp16 operands, timed with HIP events.  Prints one JSON line per
// configuration: MFMAs per SIMD per second and the implied cycles per MFMA at the
// measured kernel time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rate tools/mfma_rate.hip && tools/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) mfma_loop(const f16x8 *a, const f16x8 *b, float *out, int iters) {
  const int lane = threadIdx.x & 63;
  f16x8 va = a[(blockIdx.x * 256 + threadIdx.x) & 4095];
  f16x8 vb = b[(blockIdx.x * 256 + threadIdx.x) & 4095];
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, vb, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5f) out[lane] = s;   // (keeps the loop; never true in practice)
}

template <int NACC>
void run(const char *data, const f16x8 *a, const f16x8 *b, float *o, int cus, int waves_per_simd) {
  const int iters = 40000;   // (tens of ms per launch: clocks settle)
  const int blocks = cus * waves_per_simd;   // 256 threads = 4 waves = one per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, a, b, o, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, a, b, o, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double per_simd = (double)iters * NACC * waves_per_simd;   // MFMAs per SIMD
  const double rate = per_simd / (ms * 1e-3);
  const double tflops = rate * cus * 4 * 16.0 * 16 * 32 * 2 / 1e12;
  printf("{\"data\": \"%s\", \"nacc\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"mfma_per_simd_per_s\": %.4g, "
         "\"cycles_per_mfma_at_2.4GHz\": %.2f, \"f16_tflops\": %.1f}\n",
         data, NACC, waves_per_simd, ms, rate, 2.4e9 / rate, tflops);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 1;
  const int cus = prop.multiProcessorCount;
  std::vector<_Float16> h(4096 * 8);
  f16x8 *a, *b;
  float *o;
  if (hipMalloc(&a, 4096 * 16) != hipSuccess || hipMalloc(&b, 4096 * 16) != hipSuccess || hipMalloc(&o, 256) != hipSuccess)
    return 1;
  for (int pass = 0; pass < 2; ++pass) {
    srand(1);
    for (auto &v : h) v = pass ? (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f) : (_Float16)0.f;
    hipMemcpy(a, h.data(), 4096 * 16, hipMemcpyHostToDevice);
    hipMemcpy(b, h.data(), 4096 * 16, hipMemcpyHostToDevice);
    const char *data = pass ? "random" : "zero";
    run<4>(data, a, b, o, cus, 1);
    run<12>(data, a, b, o, cus, 1);
    run<24>(data, a, b, o, cus, 1);
    run<12>(data, a, b, o, cus, 2);
  }
  hipFree(a);
  hipFree(b);
  hipFree(o);
  return 0;
}
