// Issue-rate probe of the MFMA shapes the kernels use (gfx950): one wave per
// SIMD, 8 independent accumulators, cycles per MFMA from s_memtime (core clock).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, long long* cyc, int iters) {
  f4 acc[8];
  for (int t = 0; t < 8; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  b8 ab;
  for (int j = 0; j < 8; ++j) ab[j] = (__bf16)(a + j);
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (KIND == 0) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
      else acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, acc[t], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int t = 0; t < 8; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out; long long* cyc;
  hipMalloc(&out, 256 * 1024 * 4); hipMalloc(&cyc, 256 * 8);
  const int iters = 4096;
  for (int kind = 0; kind < 2; ++kind) {
    for (int th = 256; th <= 1024; th *= 2) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(th), 0, 0, out, cyc, iters);
      else hipLaunchKernelGGL(k<1>, dim3(256), dim3(th), 0, 0, out, cyc, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const double n = (double)iters * 8;
      printf("{\"shape\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_mfma_per_wave\": %.2f, \"us\": %.1f, \"tflops_chip\": %.1f}\n",
             kind == 0 ? "f32_16x16x4" : "bf16_16x16x32", th / 256, (double)c / n, ms * 1e3,
             (kind == 0 ? 2048.0 : 16384.0) * n * 256 * (th / 64) / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
