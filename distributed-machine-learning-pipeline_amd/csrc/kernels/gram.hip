// Gram tables of the persistent step's Gram form (kernels/mlp_persist.hip):
//
//   T[b][r'][m'][m] = X_r'(b-1)[m'] . X_cur(b)[m] + 1        (b - 1 wraps)
//
// for every batch b of a shard, every source replica r' (1 for the single
// replica), 64 x 64 rows (rows past a short batch repeat its last row, as the
// kernel's X tiles do).  It replaces the host-orchestrated float64 torch.bmm
// loop of engine/gram.py (250 ms for one 60 k-row shard, most of a real
// 10-epoch job's wall time) with one launch.
//
// Accumulation is fp64 on v_mfma_f64_16x16x4_f64, rounded once to fp32 after
// the + 1, exactly like the torch reference (`_bmm64`): the table must not move
// the correction off the fp32 reference, and the 784-term dot products of
// [0, 1] pixels reach a few hundred, where an fp32 accumulator would lose
// ~1e-4.  One workgroup per (batch, source): wave w owns rows m' = 16 w .. +15
// of the 64 x 64 block, the four 16-column tiles of m share each A fragment.
// Operands stream straight from the (L2-resident) shard as 16-B loads: lane
// (i, q) takes k = k0 + 4 q .. +3 of its row, and MFMA j of a 16-k group
// contracts k = k0 + 4 q + j -- the same permutation on both operands, so the
// products pair up as in the plain order (fp64 makes the order immaterial at
// fp32 output precision).
//
// Reference: the data of the per-step update this reorders, client.go:112-202.
#include "common.h"
#include "../dsml.h"

namespace dsml {

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gram_table_k(const float* __restrict__ Xs, int64_t src_stride,
                                                    int64_t ld_src, const float* __restrict__ Xc, int64_t ldc,
                                                    int nb, int B, int K, int nsrc, float* __restrict__ T) {
  const int b = blockIdx.x, r2 = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int bp = (b + nb - 1) % nb;
  const int64_t rowa = (int64_t)bp * B + min(16 * w + i, B - 1);
  const float* A = Xs + (int64_t)r2 * src_stride + rowa * ld_src;
  const float* Bt[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) Bt[t] = Xc + ((int64_t)b * B + min(16 * t + i, B - 1)) * ldc;
  f64x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int kfull = K & ~15;
  for (int k0 = 0; k0 < kfull; k0 += 16) {
    const float4 av = *reinterpret_cast<const float4*>(A + k0 + 4 * q);
    float4 bv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) bv[t] = *reinterpret_cast<const float4*>(Bt[t] + k0 + 4 * q);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)av.x, (double)bv[t].x, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)av.y, (double)bv[t].y, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)av.z, (double)bv[t].z, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)av.w, (double)bv[t].w, acc[t], 0, 0, 0);
    }
  }
  // K tail (K % 16): scalar k per lane q, zeros past K
  for (int k0 = kfull; k0 < K; k0 += 4) {
    const int k = k0 + q;
    const double a = k < K ? (double)A[k] : 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const double bb = k < K ? (double)Bt[t][k] : 0.0;
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc[t], 0, 0, 0);
    }
  }
  // f64 C/D layout: column = lane & 15 (m within tile t), row = q + 4 reg (m')
  float* out = T + ((int64_t)b * nsrc + r2) * 4096;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
      out[(16 * w + q + 4 * reg) * 64 + 16 * t + i] = (float)(acc[t][reg] + 1.0);
}

}  // namespace

hipError_t gram_table(const float* Xs, int64_t src_stride, int64_t ld_src, const float* Xc, int64_t ldc, int nb,
                      int B, int K, int nsrc, float* T, hipStream_t s) {
  if (nb < 1 || B < 1 || B > 64 || K < 1 || nsrc < 1 || nsrc > 65535 || (ld_src & 3) || (ldc & 3) ||
      (src_stride & 3) || (((uintptr_t)Xs | (uintptr_t)Xc) & 15))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(gram_table_k, dim3(nb, nsrc), dim3(256), 0, s, Xs, src_stride, ld_src, Xc, ldc, nb, B, K,
                     nsrc, T);
  return hipGetLastError();
}

}  // namespace dsml
