// Shared device-side helpers for the hipdsml CDNA4 (gfx950) kernels.
//
// Everything here is written for a 64-lane wavefront and the gfx950 MFMA
// operand/accumulator lane maps (see cdna_hip_programming.md §3):
//   v_mfma_f32_16x16x4_f32 : lane l supplies A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]
//                            and holds D[row=(l>>4)*4+r][col=l&15], r=0..3.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace dsml {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ f32x4 mfma_f32_16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 sel4(bool p, float4 v) {
  return p ? v : zero4();
}

// bf16 <-> f32 (round-to-nearest-even on the way down; NaN kept quiet).
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Full-wave (64-lane) reductions.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace dsml
