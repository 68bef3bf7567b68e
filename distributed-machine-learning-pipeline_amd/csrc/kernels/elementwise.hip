// Memory-bound elementwise kernels: fused SGD over the flat parameter buffer,
// dtype-aware reductions for the in-house ring / naive all-reduce paths, and
// the MNIST data-prep conversion.
//
// Reference hot spots replaced:
//   updateWeights     client.go:254-267                (SGD, 4 tensors -> 1 flat launch)
//   ring byte-reduce  gpu_coordinator_server.go:539-546 (uint8 += on fp32 bytes, Q2)
//   naive byte-sum    gpu_coordinator_server.go:681-686
//   idx u8 -> f32/255 client.go:307-310
// All kernels are grid-stride, 16 B per lane per access where the dtype allows.
#include "common.h"
#include "../dsml.h"

namespace dsml {

static inline int grid_for(int64_t nvec, int block = 256) {
  int64_t g = (nvec + block - 1) / block;
  if (g > 2048) g = 2048;  // 256 CUs x 8 blocks, grid-stride the rest
  if (g < 1) g = 1;
  return (int)g;
}

__global__ __launch_bounds__(256) void sgd_update_f32_k(float* __restrict__ P,
                                                        const float* __restrict__ G,
                                                        int64_t n, float scale) {
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* P4 = reinterpret_cast<float4*>(P);
  const float4* G4 = reinterpret_cast<const float4*>(G);
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    float4 p = P4[v];
    const float4 g = G4[v];
    p.x -= scale * g.x; p.y -= scale * g.y; p.z -= scale * g.z; p.w -= scale * g.w;
    P4[v] = p;
  }
  for (int64_t e = (nv << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    P[e] -= scale * G[e];
}

hipError_t sgd_update_f32(float* P, const float* G, int64_t n, float scale, hipStream_t s) {
  hipLaunchKernelGGL(sgd_update_f32_k, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, P, G, n,
                     scale);
  return hipGetLastError();
}

// v = momentum*v + (g*gscale + wd*p);  p -= lr*v
__global__ __launch_bounds__(256) void sgd_momentum_f32_k(float* __restrict__ P,
                                                          const float* __restrict__ G,
                                                          float* __restrict__ V, int64_t n,
                                                          float lr, float mom, float wd,
                                                          float gscale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const float p = P[e];
    const float g = G[e] * gscale + wd * p;
    const float v = mom * V[e] + g;
    V[e] = v;
    P[e] = p - lr * v;
  }
}

hipError_t sgd_momentum_f32(float* P, const float* G, float* V, int64_t n, float lr,
                            float momentum, float weight_decay, float gscale, hipStream_t s) {
  hipLaunchKernelGGL(sgd_momentum_f32_k, dim3(grid_for(n)), dim3(256), 0, s, P, G, V, n, lr,
                     momentum, weight_decay, gscale);
  return hipGetLastError();
}

// ---- reductions --------------------------------------------------------------
template <int OP>
__device__ __forceinline__ float rop(float a, float b) {
  if constexpr (OP == kSum) return a + b;
  else if constexpr (OP == kProd) return a * b;
  else if constexpr (OP == kMin) return fminf(a, b);
  else return fmaxf(a, b);
}
template <int OP>
__device__ __forceinline__ int32_t ropi(int32_t a, int32_t b) {
  if constexpr (OP == kSum) return a + b;
  else if constexpr (OP == kProd) return a * b;
  else if constexpr (OP == kMin) return a < b ? a : b;
  else return a > b ? a : b;
}

// f32: 4 elements per lane-step.
template <int OP>
__global__ __launch_bounds__(256) void reduce_f32_k(float* __restrict__ dst,
                                                    const float* __restrict__ a,
                                                    const float* __restrict__ b, int64_t n,
                                                    int vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nv = vec ? n >> 2 : 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const float4 x = reinterpret_cast<const float4*>(a)[v];
    const float4 y = reinterpret_cast<const float4*>(b)[v];
    float4 z;
    z.x = rop<OP>(x.x, y.x); z.y = rop<OP>(x.y, y.y);
    z.z = rop<OP>(x.z, y.z); z.w = rop<OP>(x.w, y.w);
    reinterpret_cast<float4*>(dst)[v] = z;
  }
  for (int64_t e = (nv << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = rop<OP>(a[e], b[e]);
}

// bf16 / f16 (computed in f32): 8 elements per lane-step.
template <int OP, bool BF>
__device__ __forceinline__ float h2f(uint16_t h) {
  if constexpr (BF) return bf16_to_f32(h);
  else return __half2float(__ushort_as_half(h));
}
template <int OP, bool BF>
__device__ __forceinline__ uint16_t f2h(float f) {
  if constexpr (BF) return f32_to_bf16(f);
  else return __half_as_ushort(__float2half(f));
}
template <int OP, bool BF>
__global__ __launch_bounds__(256) void reduce_h16_k(uint16_t* __restrict__ dst,
                                                    const uint16_t* __restrict__ a,
                                                    const uint16_t* __restrict__ b, int64_t n,
                                                    int vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nv = vec ? n >> 3 : 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const uint4 x = reinterpret_cast<const uint4*>(a)[v];
    const uint4 y = reinterpret_cast<const uint4*>(b)[v];
    const uint16_t* xs = reinterpret_cast<const uint16_t*>(&x);
    const uint16_t* ys = reinterpret_cast<const uint16_t*>(&y);
    uint4 z;
    uint16_t* zs = reinterpret_cast<uint16_t*>(&z);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      zs[j] = f2h<OP, BF>(rop<OP>(h2f<OP, BF>(xs[j]), h2f<OP, BF>(ys[j])));
    reinterpret_cast<uint4*>(dst)[v] = z;
  }
  for (int64_t e = (nv << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = f2h<OP, BF>(rop<OP>(h2f<OP, BF>(a[e]), h2f<OP, BF>(b[e])));
}

// u8 (wrapping, like the reference's byte-wise reduction) : 16 per lane-step.
template <int OP>
__device__ __forceinline__ uint8_t ropu8(uint8_t a, uint8_t b) {
  if constexpr (OP == kSum) return (uint8_t)(a + b);
  else if constexpr (OP == kProd) return (uint8_t)(a * b);
  else if constexpr (OP == kMin) return a < b ? a : b;
  else return a > b ? a : b;
}
template <int OP>
__global__ __launch_bounds__(256) void reduce_u8_k(uint8_t* __restrict__ dst,
                                                   const uint8_t* __restrict__ a,
                                                   const uint8_t* __restrict__ b, int64_t n,
                                                   int vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nv = vec ? n >> 4 : 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const uint4 x = reinterpret_cast<const uint4*>(a)[v];
    const uint4 y = reinterpret_cast<const uint4*>(b)[v];
    const uint8_t* xs = reinterpret_cast<const uint8_t*>(&x);
    const uint8_t* ys = reinterpret_cast<const uint8_t*>(&y);
    uint4 z;
    uint8_t* zs = reinterpret_cast<uint8_t*>(&z);
#pragma unroll
    for (int j = 0; j < 16; ++j) zs[j] = ropu8<OP>(xs[j], ys[j]);
    reinterpret_cast<uint4*>(dst)[v] = z;
  }
  for (int64_t e = (nv << 4) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = ropu8<OP>(a[e], b[e]);
}

template <int OP>
__global__ __launch_bounds__(256) void reduce_i32_k(int32_t* __restrict__ dst,
                                                    const int32_t* __restrict__ a,
                                                    const int32_t* __restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = ropi<OP>(a[e], b[e]);
}

template <int OP>
static hipError_t launch_reduce(void* dst, const void* a, const void* b, int64_t n,
                                int32_t dtype, hipStream_t s) {
  // 16 B vector body when all three pointers are 16 B aligned, else the
  // element-wise path (ring segments of odd sizes land on any byte offset).
  const uintptr_t al = (uintptr_t)dst | (uintptr_t)a | (uintptr_t)b;
  const int vec = (al & 15) == 0;
  switch (dtype) {
    case kF32:
      hipLaunchKernelGGL(reduce_f32_k<OP>, dim3(grid_for(vec ? (n + 3) / 4 : n)), dim3(256), 0, s,
                         (float*)dst, (const float*)a, (const float*)b, n, vec);
      break;
    case kBF16:
      hipLaunchKernelGGL((reduce_h16_k<OP, true>), dim3(grid_for(vec ? (n + 7) / 8 : n)), dim3(256),
                         0, s, (uint16_t*)dst, (const uint16_t*)a, (const uint16_t*)b, n, vec);
      break;
    case kF16:
      hipLaunchKernelGGL((reduce_h16_k<OP, false>), dim3(grid_for(vec ? (n + 7) / 8 : n)),
                         dim3(256), 0, s, (uint16_t*)dst, (const uint16_t*)a, (const uint16_t*)b, n,
                         vec);
      break;
    case kU8:
      hipLaunchKernelGGL(reduce_u8_k<OP>, dim3(grid_for(vec ? (n + 15) / 16 : n)), dim3(256), 0, s,
                         (uint8_t*)dst, (const uint8_t*)a, (const uint8_t*)b, n, vec);
      break;
    case kI32:
      hipLaunchKernelGGL(reduce_i32_k<OP>, dim3(grid_for(n)), dim3(256), 0, s, (int32_t*)dst,
                         (const int32_t*)a, (const int32_t*)b, n);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t reduce_into(void* dst, const void* a, const void* b, int64_t n, int32_t dtype,
                       int32_t op, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  switch (op) {
    case kSum: return launch_reduce<kSum>(dst, a, b, n, dtype, s);
    case kProd: return launch_reduce<kProd>(dst, a, b, n, dtype, s);
    case kMin: return launch_reduce<kMin>(dst, a, b, n, dtype, s);
    case kMax: return launch_reduce<kMax>(dst, a, b, n, dtype, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t reduce_inplace(void* dst, const void* src, int64_t n, int32_t dtype, int32_t op,
                          hipStream_t s) {
  return reduce_into(dst, dst, src, n, dtype, op, s);
}

// ---- several in-place reductions in ONE launch (the in-house ring's step:
// one receive segment per directed ring, all reduced by a single kernel
// instead of one launch per ring).  blockIdx.y picks the segment; 16-B vector
// body when both of its pointers are 16-B aligned, element tail otherwise.
template <int OP, int DT>
__device__ __forceinline__ void red_elem(void* dst, const void* src, int64_t e) {
  if constexpr (DT == kF32) {
    float* d = static_cast<float*>(dst);
    d[e] = rop<OP>(d[e], static_cast<const float*>(src)[e]);
  } else if constexpr (DT == kBF16 || DT == kF16) {
    uint16_t* d = static_cast<uint16_t*>(dst);
    d[e] = f2h<OP, DT == kBF16>(rop<OP>(h2f<OP, DT == kBF16>(d[e]),
                                        h2f<OP, DT == kBF16>(static_cast<const uint16_t*>(src)[e])));
  } else if constexpr (DT == kU8) {
    uint8_t* d = static_cast<uint8_t*>(dst);
    d[e] = ropu8<OP>(d[e], static_cast<const uint8_t*>(src)[e]);
  } else {
    int32_t* d = static_cast<int32_t*>(dst);
    d[e] = ropi<OP>(d[e], static_cast<const int32_t*>(src)[e]);
  }
}
template <int DT>
constexpr int dt_size() { return DT == kU8 ? 1 : (DT == kBF16 || DT == kF16) ? 2 : 4; }

template <int OP, int DT>
__global__ __launch_bounds__(256) void reduce_multi_k(ReduceSegs m) {
  const ReduceSeg sg = m.seg[blockIdx.y];
  constexpr int per = 16 / dt_size<DT>();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool vec = ((((uintptr_t)sg.dst) | ((uintptr_t)sg.src)) & 15) == 0;
  const int64_t nv = vec ? sg.n / per : 0;
  uint4* d4 = static_cast<uint4*>(sg.dst);
  const uint4* s4 = static_cast<const uint4*>(sg.src);
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    uint4 x = d4[v];
    const uint4 y = s4[v];
#pragma unroll
    for (int j = 0; j < per; ++j) red_elem<OP, DT>(&x, &y, j);
    d4[v] = x;
  }
  for (int64_t e = nv * per + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < sg.n; e += stride)
    red_elem<OP, DT>(sg.dst, sg.src, e);
}

template <int OP>
static hipError_t launch_reduce_multi(const ReduceSegs& m, int32_t dtype, int64_t nmax, hipStream_t s) {
  const int esz = dtype == kU8 ? 1 : (dtype == kBF16 || dtype == kF16) ? 2 : 4;
  int gx = grid_for((nmax * esz + 15) / 16);
  gx = (gx + m.count - 1) / m.count;  // ~ the same total blocks as one launch of the largest
  const dim3 grid(gx, m.count);
  switch (dtype) {
    case kF32: hipLaunchKernelGGL((reduce_multi_k<OP, kF32>), grid, dim3(256), 0, s, m); break;
    case kBF16: hipLaunchKernelGGL((reduce_multi_k<OP, kBF16>), grid, dim3(256), 0, s, m); break;
    case kF16: hipLaunchKernelGGL((reduce_multi_k<OP, kF16>), grid, dim3(256), 0, s, m); break;
    case kU8: hipLaunchKernelGGL((reduce_multi_k<OP, kU8>), grid, dim3(256), 0, s, m); break;
    case kI32: hipLaunchKernelGGL((reduce_multi_k<OP, kI32>), grid, dim3(256), 0, s, m); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t reduce_multi_inplace(const ReduceSegs& m, int32_t dtype, int32_t op, hipStream_t s) {
  if (m.count < 1 || m.count > kMaxReduceSegs) return hipErrorInvalidValue;
  int64_t nmax = 0;
  for (int k = 0; k < m.count; ++k) nmax = m.seg[k].n > nmax ? m.seg[k].n : nmax;
  if (nmax <= 0) return hipSuccess;
  switch (op) {
    case kSum: return launch_reduce_multi<kSum>(m, dtype, nmax, s);
    case kProd: return launch_reduce_multi<kProd>(m, dtype, nmax, s);
    case kMin: return launch_reduce_multi<kMin>(m, dtype, nmax, s);
    case kMax: return launch_reduce_multi<kMax>(m, dtype, nmax, s);
    default: return hipErrorInvalidValue;
  }
}

// ---- scale / conversions -----------------------------------------------------
__global__ __launch_bounds__(256) void scale_f32_k(float* x, int64_t n, float alpha) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    x[e] *= alpha;
}
template <bool BF>
__global__ __launch_bounds__(256) void scale_h16_k(uint16_t* x, int64_t n, float alpha) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    x[e] = f2h<0, BF>(h2f<0, BF>(x[e]) * alpha);
}

hipError_t scale_inplace(void* x, int64_t n, int32_t dtype, float alpha, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  switch (dtype) {
    case kF32:
      hipLaunchKernelGGL(scale_f32_k, dim3(grid_for(n)), dim3(256), 0, s, (float*)x, n, alpha);
      break;
    case kBF16:
      hipLaunchKernelGGL(scale_h16_k<true>, dim3(grid_for(n)), dim3(256), 0, s, (uint16_t*)x, n,
                         alpha);
      break;
    case kF16:
      hipLaunchKernelGGL(scale_h16_k<false>, dim3(grid_for(n)), dim3(256), 0, s, (uint16_t*)x,
                         n, alpha);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void u8_to_f32_k(float* __restrict__ dst,
                                                   const uint8_t* __restrict__ src, int64_t n,
                                                   float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = (float)src[e] * scale;
}

hipError_t u8_to_f32_scaled(float* dst, const uint8_t* src, int64_t n, float scale,
                            hipStream_t s) {
  hipLaunchKernelGGL(u8_to_f32_k, dim3(grid_for(n)), dim3(256), 0, s, dst, src, n, scale);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void f32_to_bf16_k(uint16_t* __restrict__ dst,
                                                     const float* __restrict__ src, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = f32_to_bf16(src[e]);
}
__global__ __launch_bounds__(256) void bf16_to_f32_k(float* __restrict__ dst,
                                                     const uint16_t* __restrict__ src,
                                                     int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    dst[e] = bf16_to_f32(src[e]);
}

hipError_t f32_to_bf16(uint16_t* dst, const float* src, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(f32_to_bf16_k, dim3(grid_for(n)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}
hipError_t bf16_to_f32(float* dst, const uint16_t* src, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(bf16_to_f32_k, dim3(grid_for(n)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

}  // namespace dsml
