// bf16 MFMA GEMM + fused epilogues for the wide-MLP path (BASELINE config 4:
// MLP 784-4096-4096-10 in bf16).  Every GEMM of the step is expressed in "NT"
// form, C[M x N] = A[M x K] . B[N x K]^T, with both operands K-contiguous, by
// keeping transposed bf16 copies where a product needs them (W^T for the
// activation gradients, H^T / dZ^T for the weight gradients).  With K
// contiguous each lane's MFMA fragment is one 16-byte load straight from
// global/L2 (v_mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4)..+7]).
//
//   gemm_bf16_nt_k   : 64x64 tile per workgroup (4 waves x 32x32, 2x2 MFMA tiles),
//                      K split across blockIdx.z into fp32 partial slabs,
//                      4 K-steps (128) of loads in flight before their MFMAs.
//   gemm_epilogue_k  : sum slabs, *alpha, +bias, ReLU, ReLU'-mask, write fp32
//                      and/or bf16 and/or the transposed bf16 copy (LDS tile).
//   cast_transpose_k : f32 [M x K] -> bf16 [M x Kp] + bf16^T [Kp x M]  (input batch)
//   softmax_xent_k   : fp32 logits -> CE stats, dZ = (p - y)/B in bf16 (+ ^T)
//   rowsum_bf16_k    : bias gradients  db[n] = sum_m dZ^T[n][m]
//   sgd_cast_k       : fp32 master W -= lr*g, refresh bf16 W and bf16 W^T
#include "common.h"
#include "../dsml.h"

namespace dsml {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint4 zero_u4() { return make_uint4(0u, 0u, 0u, 0u); }

// ---------------------------------------------------------------------------
constexpr int kGemmU = 4;  // K-steps (x32) whose loads are in flight together

__global__ __launch_bounds__(256) void gemm_bf16_nt_k(
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
    float* __restrict__ Cp, int M, int N, int K, int kchunk, GemmEpi epi, int fused) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int mb = blockIdx.y * 64 + (w >> 1) * 32;
  const int nb = blockIdx.x * 64 + (w & 1) * 32;
  const int kb = blockIdx.z * kchunk;
  const int ke = min(K, kb + kchunk);
  int ra[2], rb[2];
  bool va[2], vb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    ra[t] = mb + 16 * t + i;
    rb[t] = nb + 16 * t + i;
    va[t] = ra[t] < M;
    vb[t] = rb[t] < N;
    ra[t] = va[t] ? ra[t] : M - 1;
    rb[t] = vb[t] ? rb[t] : N - 1;
  }
  const uint16_t* pa[2] = {A + (int64_t)ra[0] * lda + 8 * g, A + (int64_t)ra[1] * lda + 8 * g};
  const uint16_t* pb[2] = {B + (int64_t)rb[0] * ldb + 8 * g, B + (int64_t)rb[1] * ldb + 8 * g};
  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};

  for (int k0 = kb; k0 < ke; k0 += 32 * kGemmU) {
    uint4 fa[kGemmU][2], fb[kGemmU][2];
#pragma unroll
    for (int u = 0; u < kGemmU; ++u) {
      const int kk = k0 + 32 * u + 8 * g;
      const int kc = kk < ke ? k0 + 32 * u : kb;  // clamp to a valid address
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[u][t] = *reinterpret_cast<const uint4*>(pa[t] + kc);
        fb[u][t] = *reinterpret_cast<const uint4*>(pb[t] + kc);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kGemmU; ++u) {
      const bool kv = k0 + 32 * u + 8 * g < ke;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[u][t] = (kv && va[t]) ? fa[u][t] : zero_u4();
        fb[u][t] = (kv && vb[t]) ? fb[u][t] : zero_u4();
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = mfma_bf16(fa[u][x], fb[u][y], acc[x][y]);
    }
  }
  if (fused) {
    // Single K split: apply the whole epilogue from the accumulators (no slab
    // round trip).  Optional fused SGD: W[m][n] -= lr * acc, and the bf16 /
    // transposed-bf16 outputs then receive the UPDATED weight.
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int n = nb + 16 * y + i;
        const int m4 = mb + 16 * x + 4 * g;
        if (n >= N) continue;
        uint16_t hb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m4 + r;
          float v = acc[x][y][r] * epi.alpha;
          if (m < M) {
            if (epi.bias) v += epi.bias[n];
            if (epi.relu) v = fmaxf(v, 0.f);
            if (epi.mask) v = bf16_to_f32(epi.mask[(int64_t)m * epi.ldm + n]) > 0.f ? v : 0.f;
            if (epi.sgdW) {
              float* wp = epi.sgdW + (int64_t)m * epi.ldw + n;
              v = *wp - epi.lr * v;
              *wp = v;
            }
            if (epi.of32) epi.of32[(int64_t)m * epi.ldo + n] = v;
            if (epi.obf) epi.obf[(int64_t)m * epi.ldb + n] = f32_to_bf16(v);
          }
          hb[r] = m < M ? f32_to_bf16(v) : (uint16_t)0;
        }
        if (epi.obfT) {
          uint16_t* tp = epi.obfT + (int64_t)n * epi.ldt + m4;
          if (m4 + 3 < M) {
            *reinterpret_cast<uint2*>(tp) = make_uint2(hb[0] | ((uint32_t)hb[1] << 16),
                                                       hb[2] | ((uint32_t)hb[3] << 16));
          } else {
            for (int r = 0; r < 4 && m4 + r < M; ++r) tp[r] = hb[r];
          }
        }
      }
    return;
  }
  float* out = Cp + (int64_t)blockIdx.z * M * N;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int n = nb + 16 * y + i;
      if (n < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mb + 16 * x + 4 * g + r;
          if (m < M) out[(int64_t)m * N + n] = acc[x][y][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------
// Epilogue over 32x32 tiles (256 threads, 4 elements each).
__global__ __launch_bounds__(256) void gemm_epilogue_k(
    const float* __restrict__ Cp, int S, int M, int N, float alpha, const float* __restrict__ bias,
    int relu, const uint16_t* __restrict__ mask, int64_t ldm, float* __restrict__ of32,
    int64_t ldo, uint16_t* __restrict__ obf, int64_t ldb, uint16_t* __restrict__ obfT,
    int64_t ldt) {
  __shared__ uint16_t tile[32][34];
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // ty in 0..7
  const int n = n0 + tx;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int mr = ty + 8 * j;
    const int m = m0 + mr;
    float v = 0.f;
    if (m < M && n < N) {
      for (int s = 0; s < S; ++s) v += Cp[((int64_t)s * M + m) * N + n];
      v *= alpha;
      if (bias) v += bias[n];
      if (relu) v = fmaxf(v, 0.f);
      if (mask) v = bf16_to_f32(mask[(int64_t)m * ldm + n]) > 0.f ? v : 0.f;
      if (of32) of32[(int64_t)m * ldo + n] = v;
      if (obf) obf[(int64_t)m * ldb + n] = f32_to_bf16(v);
    }
    tile[mr][tx] = f32_to_bf16(v);
  }
  if (!obfT) return;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nr = ty + 8 * j;
    const int nn = n0 + nr, mm = m0 + tx;
    if (nn < N && mm < M) obfT[(int64_t)nn * ldt + mm] = tile[tx][nr];
  }
}

// f32 [M x K] (ld ldi) -> bf16 [M x Kp] (ld ldo, zero cols K..Kp) and bf16^T [Kp x M] (ld ldt)
__global__ __launch_bounds__(256) void cast_transpose_k(const float* __restrict__ X, int64_t ldi,
                                                        int M, int K, int Kp,
                                                        uint16_t* __restrict__ Y, int64_t ldo,
                                                        uint16_t* __restrict__ YT, int64_t ldt) {
  __shared__ uint16_t tile[32][34];
  const int k0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + ty + 8 * j, k = k0 + tx;
    uint16_t h = 0;
    if (m < M && k < K) h = f32_to_bf16(X[(int64_t)m * ldi + k]);
    if (m < M && k < Kp && Y) Y[(int64_t)m * ldo + k] = h;
    tile[ty + 8 * j][tx] = h;
  }
  if (!YT) return;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + ty + 8 * j, m = m0 + tx;
    if (k < Kp && m < M) YT[(int64_t)k * ldt + m] = tile[tx][ty + 8 * j];
  }
}

// One wave per row; C <= 64 classes (one lane each).
__global__ __launch_bounds__(64) void softmax_xent_k(const float* __restrict__ logits, int64_t ldl,
                                                     const int32_t* __restrict__ labels, int B,
                                                     int C, int Cp, float inv_batch,
                                                     uint16_t* __restrict__ dz, int64_t ldz,
                                                     uint16_t* __restrict__ dzT, int64_t ldt,
                                                     float* __restrict__ stats) {
  const int m = blockIdx.x, c = threadIdx.x;
  const bool cv = c < C;
  const float z = cv ? logits[(int64_t)m * ldl + c] : -3.402823466e38f;
  const int y = labels[m];
  // wave max / argmax / sum via shuffles (64 lanes, tiny kernel)
  float mx = z;
  int am = cv ? c : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    argmax_combine(mx, am, om, oa);
  }
  const float e = cv ? expf(z - mx) : 0.f;
  float se = e;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
  const float p = e / se;
  const float g = cv ? (p - (c == y ? 1.f : 0.f)) * inv_batch : 0.f;
  if (c < Cp) {
    const uint16_t h = f32_to_bf16(g);
    dz[(int64_t)m * ldz + c] = h;
    if (dzT) dzT[(int64_t)c * ldt + m] = h;
  }
  if (c == y && stats) {
    atomicAdd(stats + 0, -logf(p + 1e-10f));
    atomicAdd(stats + 1, am == y ? 1.f : 0.f);
    atomicAdd(stats + 2, 1.f);
  }
}

// db[n] = sum_m X[n][m]  (X bf16 [N x ld], m < cols); 16 B loads when the row
// is 16 B aligned.  With `bias` != nullptr the sum is applied as an SGD step to
// the bias instead (b -= lr * db).
__global__ __launch_bounds__(256) void rowsum_bf16_k(const uint16_t* __restrict__ X, int64_t ld,
                                                     int N, int cols, float* __restrict__ out,
                                                     float* __restrict__ bias, float lr) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const uint16_t* row = X + (int64_t)n * ld;
  float s = 0.f;
  int m = 0;
  if ((((uintptr_t)row) & 15) == 0) {
    for (; m + 8 <= cols; m += 8) {
      const uint4 v = *reinterpret_cast<const uint4*>(row + m);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
    }
  }
  for (; m < cols; ++m) s += bf16_to_f32(row[m]);
  if (bias) bias[n] -= lr * s;
  else out[n] = s;
}

// W (fp32 [N x K] contiguous) -= lr * G ; refresh Wb bf16 [N x ldw] and WbT bf16 [K.. x ldt]
__global__ __launch_bounds__(256) void sgd_cast_k(float* __restrict__ W, const float* __restrict__ G,
                                                  int N, int K, float lr,
                                                  uint16_t* __restrict__ Wb, int64_t ldw,
                                                  uint16_t* __restrict__ WbT, int64_t ldt) {
  __shared__ uint16_t tile[32][34];
  const int k0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + ty + 8 * j, k = k0 + tx;
    uint16_t h = 0;
    if (n < N && k < K) {
      const int64_t idx = (int64_t)n * K + k;
      float w = W[idx];
      if (G) {
        w -= lr * G[idx];
        W[idx] = w;
      }
      h = f32_to_bf16(w);
      Wb[(int64_t)n * ldw + k] = h;
    }
    tile[ty + 8 * j][tx] = h;
  }
  if (!WbT) return;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + ty + 8 * j, n = n0 + tx;
    if (k < K && n < N) WbT[(int64_t)k * ldt + n] = tile[tx][ty + 8 * j];
  }
}

// ---------------------------------------------------------------------------
hipError_t gemm_bf16_nt(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, float* Cp,
                        int M, int N, int K, int splits, hipStream_t s, const GemmEpi* epi) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return hipErrorInvalidValue;
  if ((K & 7) || (lda & 7) || (ldb & 7)) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return hipErrorInvalidValue;
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 31) / 32 * 32;
  const int S = (K + kchunk - 1) / kchunk;
  if (epi != nullptr && S != 1) return hipErrorInvalidValue;  // fused epilogue needs one split
  if (epi != nullptr && epi->obfT && (epi->ldt & 3)) return hipErrorInvalidValue;
  GemmEpi e{};
  e.alpha = 1.f;
  if (epi) e = *epi;
  dim3 grid((N + 63) / 64, (M + 63) / 64, S);
  hipLaunchKernelGGL(gemm_bf16_nt_k, grid, dim3(256), 0, s, A, lda, B, ldb, Cp, M, N, K, kchunk, e,
                     epi != nullptr ? 1 : 0);
  return hipGetLastError();
}

int gemm_bf16_num_splits(int K, int splits) {
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 31) / 32 * 32;
  return (K + kchunk - 1) / kchunk;
}

hipError_t gemm_epilogue(const float* Cp, int S, int M, int N, float alpha, const float* bias,
                         int relu, const uint16_t* mask, int64_t ldm, float* of32, int64_t ldo,
                         uint16_t* obf, int64_t ldb, uint16_t* obfT, int64_t ldt, hipStream_t s) {
  dim3 grid((N + 31) / 32, (M + 31) / 32);
  hipLaunchKernelGGL(gemm_epilogue_k, grid, dim3(256), 0, s, Cp, S, M, N, alpha, bias, relu, mask,
                     ldm, of32, ldo, obf, ldb, obfT, ldt);
  return hipGetLastError();
}

hipError_t cast_transpose(const float* X, int64_t ldi, int M, int K, int Kp, uint16_t* Y,
                          int64_t ldo, uint16_t* YT, int64_t ldt, hipStream_t s) {
  dim3 grid((Kp + 31) / 32, (M + 31) / 32);
  hipLaunchKernelGGL(cast_transpose_k, grid, dim3(256), 0, s, X, ldi, M, K, Kp, Y, ldo, YT, ldt);
  return hipGetLastError();
}

hipError_t softmax_xent(const float* logits, int64_t ldl, const int32_t* labels, int B, int C,
                        int Cp, float inv_batch, uint16_t* dz, int64_t ldz, uint16_t* dzT,
                        int64_t ldt, float* stats, hipStream_t s) {
  if (C > 64 || Cp > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_xent_k, dim3(B), dim3(64), 0, s, logits, ldl, labels, B, C, Cp,
                     inv_batch, dz, ldz, dzT, ldt, stats);
  return hipGetLastError();
}

hipError_t rowsum_bf16(const uint16_t* X, int64_t ld, int N, int cols, float* out, float* bias,
                       float lr, hipStream_t s) {
  hipLaunchKernelGGL(rowsum_bf16_k, dim3((N + 255) / 256), dim3(256), 0, s, X, ld, N, cols, out,
                     bias, lr);
  return hipGetLastError();
}

hipError_t sgd_cast(float* W, const float* G, int N, int K, float lr, uint16_t* Wb, int64_t ldw,
                    uint16_t* WbT, int64_t ldt, hipStream_t s) {
  dim3 grid((K + 31) / 32, (N + 31) / 32);
  hipLaunchKernelGGL(sgd_cast_k, grid, dim3(256), 0, s, W, G, N, K, lr, Wb, ldw, WbT, ldt);
  return hipGetLastError();
}

}  // namespace dsml
