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
#include <cstdlib>

#include "common.h"
#include "head_row.h"
#include "../dsml.h"

namespace dsml {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint4 zero_u4() { return make_uint4(0u, 0u, 0u, 0u); }

// ---------------------------------------------------------------------------
// Main kernel.  Workgroup = 64x64 output tile, 4 waves of 32x32 (2x2 MFMA
// 16x16x32 tiles); U K-steps (x32) of operand loads in flight per batch.
//   mode 0: write the fp32 partial of this K split to its slab (Cp[z]);
//           a separate gemm_epilogue_k sums the slabs.
//   mode 1: single K split, epilogue applied from the accumulators.
//   mode 2: split-K with the epilogue fused: every split writes its slab,
//           the LAST split to finish a tile (per-tile arrival counter, no
//           spinning) sums all slabs in split order (deterministic) and
//           applies the epilogue, then re-arms the counter.
// Optional (mode 1): row sums of A over K (bias gradient of the dW GEMM,
// A = dZ^T) written to epi.bgrad or applied as SGD to epi.bsgd.
// ---------------------------------------------------------------------------
constexpr int kTileLdsStride = 68;  // fp32 words per LDS row of the SGD epilogue

typedef __attribute__((address_space(1))) uint32_t gu32a;
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef uint32_t nu2 __attribute__((ext_vector_type(2)));
typedef uint32_t nu4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store((gu32a*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __uint_as_float(__hip_atomic_load((const gu32a*)p, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ float bf16lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Epilogue from accumulators in MFMA layout: acc[x][y][r] = C[mb+16x+4g+r][nb+16y+i].
__device__ __forceinline__ void epilogue_regs(f32x4 (&acc)[2][2], int mb, int nb, int i, int g,
                                              int M, int N, const GemmEpi& epi) {
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
}

// Fused SGD epilogue staged through LDS so every global access is a full
// 16 B vector along a row: W (fp32) read-modify-write as float4, the bf16 copy
// as 8 B runs, the transposed bf16 copy as 16 B runs of 8 rows.  Requires
// N % 4 == 0, M % 8 == 0 and 16 B-aligned rows (checked on the host).
__device__ __forceinline__ void epilogue_sgd_lds(f32x4 (&acc)[2][2], float* tile, int m0, int n0,
                                                 int M, int N, const GemmEpi& epi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        tile[(wm + 16 * x + 4 * g + r) * kTileLdsStride + wn + 16 * y + i] = acc[x][y][r] * epi.alpha;
  __syncthreads();
  // row pass: 64 rows x 16 float4 -> 4 per thread
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int idx = threadIdx.x + 256 * j;
    const int r = idx >> 4, c = (idx & 15) * 4;
    const int m = m0 + r, n = n0 + c;
    float* tp = tile + r * kTileLdsStride + c;
    if (m < M && n < N) {
      float4* wp = reinterpret_cast<float4*>(epi.sgdW + (int64_t)m * epi.ldw + n);
      float4 wv = *wp;
      wv.x -= epi.lr * tp[0];
      wv.y -= epi.lr * tp[1];
      wv.z -= epi.lr * tp[2];
      wv.w -= epi.lr * tp[3];
      __builtin_nontemporal_store(nf4{wv.x, wv.y, wv.z, wv.w}, reinterpret_cast<nf4*>(wp));
      tp[0] = wv.x; tp[1] = wv.y; tp[2] = wv.z; tp[3] = wv.w;
      if (epi.obf) {
        const uint32_t lo = f32_to_bf16(wv.x) | ((uint32_t)f32_to_bf16(wv.y) << 16);
        const uint32_t hi = f32_to_bf16(wv.z) | ((uint32_t)f32_to_bf16(wv.w) << 16);
        __builtin_nontemporal_store(nu2{lo, hi},
                                    reinterpret_cast<nu2*>(epi.obf + (int64_t)m * epi.ldb + n));
      }
    }
  }
  if (!epi.obfT) return;
  __syncthreads();
  // column pass: W^T rows n (64) x 8 runs of 8 m -> 2 per thread
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j;
    const int c = idx >> 3, r8 = (idx & 7) * 8;
    const int n = n0 + c, m = m0 + r8;
    if (n < N && m < M) {
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        q[k] = f32_to_bf16(tile[(r8 + 2 * k) * kTileLdsStride + c]) |
               ((uint32_t)f32_to_bf16(tile[(r8 + 2 * k + 1) * kTileLdsStride + c]) << 16);
      __builtin_nontemporal_store(nu4{q[0], q[1], q[2], q[3]},
                                  reinterpret_cast<nu4*>(epi.obfT + (int64_t)n * epi.ldt + m));
    }
  }
}

// SPLIT = false compiles the split-K paths (modes 0 and 2) out: the
// weight-gradient GEMMs (K = batch, mode 1) then need few enough registers to
// keep 6 waves per SIMD, and their fused SGD epilogue is a streaming RMW of W.
template <int U, bool SPLIT = true>
__global__ __launch_bounds__(256, SPLIT ? 1 : 6) void gemm_bf16_nt_k(
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
    float* __restrict__ Cp, int M, int N, int K, int kchunk, GemmEpi epi, int mode,
    int* __restrict__ tile_ctr, int sgd_lds) {
  __shared__ float tile[64 * kTileLdsStride];  // the ONE LDS array (also the last-arriver flag)
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
  // Row bases; each lane's K offset is clamped on its own (k + 8g may run past
  // a short row's end when K % 32 != 0: never read past the buffer).
  const uint16_t* pa[2] = {A + (int64_t)ra[0] * lda, A + (int64_t)ra[1] * lda};
  const uint16_t* pb[2] = {B + (int64_t)rb[0] * ldb, B + (int64_t)rb[1] * ldb};
  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};
  const bool want_rowsum = mode == 1 && (epi.bgrad || epi.bsgd);
  float rs[2] = {0.f, 0.f};

  for (int k0 = kb; k0 < ke; k0 += 32 * U) {
    uint4 fa[U][2], fb[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k0 + 32 * u + 8 * g;
      const int kc = kk < ke ? kk : kb;  // clamp to a valid 16 B run of the row
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[u][t] = *reinterpret_cast<const uint4*>(pa[t] + kc);
        fb[u][t] = *reinterpret_cast<const uint4*>(pb[t] + kc);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool kv = k0 + 32 * u + 8 * g < ke;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[u][t] = (kv && va[t]) ? fa[u][t] : zero_u4();
        fb[u][t] = (kv && vb[t]) ? fb[u][t] : zero_u4();
      }
      if (want_rowsum) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint4 v = fa[u][t];
          rs[t] += bf16lo(v.x) + bf16hi(v.x) + bf16lo(v.y) + bf16hi(v.y) + bf16lo(v.z) +
                   bf16hi(v.z) + bf16lo(v.w) + bf16hi(v.w);
        }
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = mfma_bf16(fa[u][x], fb[u][y], acc[x][y]);
    }
  }

  if (SPLIT && mode == 0) {
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
    return;
  }
  if (SPLIT && mode == 2) {
    // ---- split-K, last arriver finishes the tile -------------------------
    // Slabs in the MFMA-native layout (16 floats per thread per split, 16 B
    // runs): written WRITE-THROUGH (sc1, raw_buffer_store_b128 aux 16) so no
    // release fence is needed, and read back by the last arriver with sc1
    // loads (placement-independent; cdna_hip_programming.md split-K recipe).
    const int T = gridDim.x * gridDim.y;
    const int tid = blockIdx.y * gridDim.x + blockIdx.x;
    const int S = gridDim.z;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(Cp, (short)0, 0x7fffffff, 0x00020000);
    const int base = ((blockIdx.z * T + tid) * 256 + threadIdx.x) * 64;  // bytes
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nu4, acc[x][y]), rs,
                                               base + (x * 2 + y) * 16, 0, 16);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      tile[0] = __hip_atomic_fetch_add(tile_ctr + tid, 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) == S - 1 ? 1.f : 0.f;
    __syncthreads();
    if (tile[0] == 0.f) return;
    __syncthreads();  // tile[] is reused by the SGD epilogue below
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < S; z += 4) {  // split order: deterministic
      nu4 v[4][4];
#pragma unroll
      for (int zz = 0; zz < 4; ++zz) {
        const int zc = min(z + zz, S - 1);
        const int b = ((zc * T + tid) * 256 + threadIdx.x) * 64;
#pragma unroll
        for (int p = 0; p < 4; ++p)
          v[zz][p] = __builtin_amdgcn_raw_buffer_load_b128(rs, b + p * 16, 0, 16);
      }
#pragma unroll
      for (int zz = 0; zz < 4; ++zz)
        if (z + zz < S) {
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
              const f32x4 f = __builtin_bit_cast(f32x4, v[zz][x * 2 + y]);
              acc[x][y][0] += f[0];
              acc[x][y][1] += f[1];
              acc[x][y][2] += f[2];
              acc[x][y][3] += f[3];
            }
        }
    }
    if (threadIdx.x == 0)  // re-arm for the next GEMM using the counters
      __hip_atomic_store(tile_ctr + tid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  if (want_rowsum) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      rs[t] += __shfl_xor(rs[t], 16, 64);
      rs[t] += __shfl_xor(rs[t], 32, 64);
    }
    if (blockIdx.x == 0 && (w & 1) == 0 && g == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int m = mb + 16 * t + i;
        if (m < M) {
          if (epi.bsgd) epi.bsgd[m] -= epi.lr * epi.alpha * rs[t];
          else epi.bgrad[m] = epi.alpha * rs[t];
        }
      }
    }
  }
  if (sgd_lds) {
    epilogue_sgd_lds(acc, tile, blockIdx.y * 64, blockIdx.x * 64, M, N, epi);
  } else {
    epilogue_regs(acc, mb, nb, i, g, M, N, epi);
  }
}

// ---------------------------------------------------------------------------
// Skinny GEMM for the batch-row products (M <= 64 rows per block: the batch):
// C[64 x 16] per workgroup over the FULL K, the 4 waves splitting K four ways
// and combining through LDS — no cross-workgroup split-K, so no slabs, no
// counters and the whole epilogue in the same launch.  N / 16 workgroups
// (256 for N = 4096 = one per CU); each streams its 16 weight rows once and
// the 64-row activation block through L2.
// ---------------------------------------------------------------------------
constexpr int kR64Pad = 17;  // LDS row stride (floats) of a 16-wide partial tile

template <int U, int WAVES, bool ABLK = false>
__global__ __launch_bounds__(64 * WAVES) void gemm_rows64_k(const uint16_t* __restrict__ A, int64_t lda,
                                                     const uint16_t* __restrict__ B, int64_t ldb,
                                                     int M, int N, int K, GemmEpi epi, int vec) {
  constexpr int NT = 64 * WAVES;
  __shared__ float red[WAVES * 64 * kR64Pad];
  // ABLK: the block's 16 weight rows (K <= 1024), whole, + a tail instruction's overrun
  __shared__ __attribute__((aligned(16))) char bimg[ABLK ? 16 * 1024 * 2 + 1024 : 16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 64;
  const int kq = ((K + WAVES - 1) / WAVES + 31) / 32 * 32;
  const int kb = w * kq, ke = min(K, kb + kq);
  int ra[4];
  bool va[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    ra[t] = m0 + 16 * t + i;
    va[t] = ra[t] < M;
    ra[t] = va[t] ? ra[t] : M - 1;
  }
  const bool vb = n0 + i < N;
  const uint16_t* pb = B + (int64_t)(vb ? n0 + i : N - 1) * ldb;
  // the epilogue's bias and mask operands fetched up front: their round trip
  // hides under the K loop instead of following it
  constexpr int PER = 1024 / NT;  // outputs of the 64x16 tile per thread
  float bias_v[PER];
  uint16_t mask_v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + NT * j;
    const int m = m0 + (e >> 4), n = n0 + (e & 15);
    const bool ok = m < M && n < N;
    bias_v[j] = (epi.bias && ok) ? epi.bias[n] : 0.f;
    mask_v[j] = (epi.mask && ok) ? epi.mask[(int64_t)m * epi.ldm + n] : (uint16_t)0x3f80;  // 1.0
  }
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (ABLK) {
    // The input layer (K <= 1024: one U-round per wave).  A (the batch rows) is
    // k-blocked, so each fragment load is 1 KiB contiguous; B (this block's 16
    // weight rows, one contiguous run when ldb == K) is copied whole into LDS
    // by LDS-DMA, 1 KiB whole lines per instruction, instead of 16 half lines
    // per fragment load.  Same operands, same MFMA order: bit-exact.
    const int K8 = K / 8, chunks = 16 * K8;
    uint4 fa[U][4];
    if (kb < ke) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = kb + 32 * u + 8 * g;
        const int kc = kk < ke ? kk : kb;
#pragma unroll
        for (int t = 0; t < 4; ++t)
          fa[u][t] = *reinterpret_cast<const uint4*>(A + (int64_t)(kc >> 5) * lda + 32 * ra[t] + (kc & 31));
      }
    }
    for (int j = w; 64 * j < chunks; j += WAVES) {
      const int c = min(64 * j + lane, chunks - 1);  // the tail instruction re-reads the last chunk
      const int r = c / K8, col = c - r * K8;
      const int n = min(n0 + r, N - 1);
      __builtin_amdgcn_global_load_lds(
          (__attribute__((address_space(1))) void*)(B + (int64_t)n * ldb + 8 * col),
          (__attribute__((address_space(3))) void*)(bimg + 1024 * j), 16, 0, 0);
    }
    __syncthreads();  // every wave's DMA landed (the barrier's vmcnt(0) covers it)
    if (kb < ke) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = kb + 32 * u + 8 * g;
        const bool kv = kk < ke;
        const int kc = kv ? kk : kb;
        const uint4 bl = *reinterpret_cast<const uint4*>(bimg + 16 * (i * K8 + (kc >> 3)));
        const uint4 b = (kv && vb) ? bl : zero_u4();
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = mfma_bf16((kv && va[t]) ? fa[u][t] : zero_u4(), b, acc[t]);
      }
    }
  } else {
    for (int k0 = kb; k0 < ke; k0 += 32 * U) {
      uint4 fa[U][4], fb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k0 + 32 * u + 8 * g;
        const int kc = kk < ke ? kk : kb;  // per-lane clamp: never past the row
        fb[u] = *reinterpret_cast<const uint4*>(pb + kc);
#pragma unroll
        for (int t = 0; t < 4; ++t) fa[u][t] = *reinterpret_cast<const uint4*>(A + (int64_t)ra[t] * lda + kc);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool kv = k0 + 32 * u + 8 * g < ke;
        const uint4 b = (kv && vb) ? fb[u] : zero_u4();
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[t] = mfma_bf16((kv && va[t]) ? fa[u][t] : zero_u4(), b, acc[t]);
      }
    }
  }
  // partials -> LDS, then the fixed-order 4-way sum (deterministic)
  float* mine = red + w * 64 * kR64Pad;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) mine[(16 * t + 4 * g + r) * kR64Pad + i] = acc[t][r];
  __syncthreads();
  float v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + NT * j;
    const int mr = e >> 4, nc = e & 15;
    const int o = mr * kR64Pad + nc;
    float x = red[o];
#pragma unroll
    for (int q = 1; q < WAVES; ++q) x += red[q * 64 * kR64Pad + o];
    const int m = m0 + mr, n = n0 + nc;
    x *= epi.alpha;
    if (m < M && n < N) {
      x += bias_v[j];
      if (epi.relu) x = fmaxf(x, 0.f);
      if (epi.mask) x = bf16_to_f32(mask_v[j]) > 0.f ? x : 0.f;
    } else {
      x = 0.f;
    }
    v[j] = x;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + NT * j;
    red[(e >> 4) * kR64Pad + (e & 15)] = v[j];
  }
  __syncthreads();
  if (threadIdx.x >= 256) return;  // stores below use 256 threads
  if (vec) {
    // rows: thread -> (m = t / 4, 4 consecutive n)
    const int mr = threadIdx.x >> 2, nc = (threadIdx.x & 3) * 4;
    const int m = m0 + mr, n = n0 + nc;
    if (m < M && n < N) {
      const float* s4 = red + mr * kR64Pad + nc;
      if (epi.of32)
        *reinterpret_cast<float4*>(epi.of32 + (int64_t)m * epi.ldo + n) =
            make_float4(s4[0], s4[1], s4[2], s4[3]);
      if (epi.obf)
        *reinterpret_cast<uint2*>(epi.obf + (int64_t)m * epi.ldb + n) =
            make_uint2(f32_to_bf16(s4[0]) | ((uint32_t)f32_to_bf16(s4[1]) << 16),
                       f32_to_bf16(s4[2]) | ((uint32_t)f32_to_bf16(s4[3]) << 16));
    }
    // transposed: thread -> (n = t / 16, 4 consecutive m)
    if (epi.obfT) {
      const int nr = threadIdx.x >> 4, mc = (threadIdx.x & 15) * 4;
      const int nn = n0 + nr, mm = m0 + mc;
      if (nn < N && mm < M) {
        uint16_t h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = f32_to_bf16(red[(mc + r) * kR64Pad + nr]);
        *reinterpret_cast<uint2*>(epi.obfT + (int64_t)nn * epi.ldt + mm) =
            make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = threadIdx.x + 256 * j;
      const int mr = e >> 4, nc = e & 15;
      const int m = m0 + mr, n = n0 + nc;
      if (m < M && n < N) {
        const float x = red[mr * kR64Pad + nc];
        if (epi.of32) epi.of32[(int64_t)m * epi.ldo + n] = x;
        if (epi.obf) epi.obf[(int64_t)m * epi.ldb + n] = f32_to_bf16(x);
        if (epi.obfT) epi.obfT[(int64_t)n * epi.ldt + m] = f32_to_bf16(x);
      }
    }
  }
}

hipError_t gemm_bf16_rows64(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int M,
                            int N, int K, const GemmEpi& epi, hipStream_t s, bool a_blk) {
  if (M <= 0 || N <= 0 || K <= 0 || (K & 7) || (lda & 7) || (ldb & 7)) return hipErrorInvalidValue;
  if (a_blk && (lda < 32 * (int64_t)M)) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return hipErrorInvalidValue;
  if (epi.sgdW || epi.bgrad || epi.bsgd) return hipErrorInvalidValue;
  // vector stores when every written row run is aligned and whole
  const int vec = ((N % 4) == 0 && (M % 4) == 0 && (!epi.of32 || ((epi.ldo % 4) == 0 && ((uintptr_t)epi.of32 & 15) == 0)) &&
                   (!epi.obf || ((epi.ldb % 4) == 0 && ((uintptr_t)epi.obf & 7) == 0)) &&
                   (!epi.obfT || ((epi.ldt % 4) == 0 && ((uintptr_t)epi.obfT & 7) == 0))) ? 1 : 0;
  dim3 grid((N + 15) / 16, (M + 63) / 64);
  // Long K: 8 waves (512 threads) each streaming K/8 with 8 K-steps of loads
  // in flight: twice the bytes in flight per CU of the 4-wave form.
  // Mid K (the 784-wide input layer): 8 waves of 4 K-steps, so every wave's
  // whole K range (<= 128) is ONE load batch instead of two dependent rounds.
  if (K >= 8 * 32 * 8)
    hipLaunchKernelGGL((gemm_rows64_k<8, 8>), grid, dim3(512), 0, s, A, lda, B, ldb, M, N, K, epi, vec);
  else if (K >= 4 * 32 * 4 && K <= 8 * 128 && a_blk)
    hipLaunchKernelGGL((gemm_rows64_k<4, 8, true>), grid, dim3(512), 0, s, A, lda, B, ldb, M, N, K, epi, vec);
  else if (a_blk)
    return hipErrorInvalidValue;  // k-blocked A: the input-layer shape only
  else if (K >= 4 * 32 * 4 && K <= 8 * 128)
    hipLaunchKernelGGL((gemm_rows64_k<4, 8>), grid, dim3(512), 0, s, A, lda, B, ldb, M, N, K, epi, vec);
  else if (K >= 4 * 32 * 4)
    hipLaunchKernelGGL((gemm_rows64_k<4, 4>), grid, dim3(256), 0, s, A, lda, B, ldb, M, N, K, epi, vec);
  else
    hipLaunchKernelGGL((gemm_rows64_k<2, 4>), grid, dim3(256), 0, s, A, lda, B, ldb, M, N, K, epi, vec);
  return hipGetLastError();
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
      int s = 0;
      for (; s + 4 <= S; s += 4) {
        const float a0 = Cp[((int64_t)s * M + m) * N + n], a1 = Cp[((int64_t)(s + 1) * M + m) * N + n];
        const float a2 = Cp[((int64_t)(s + 2) * M + m) * N + n], a3 = Cp[((int64_t)(s + 3) * M + m) * N + n];
        v += a0; v += a1; v += a2; v += a3;
      }
      for (; s < S; ++s) v += Cp[((int64_t)s * M + m) * N + n];
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
                        int M, int N, int K, int splits, hipStream_t s, const GemmEpi* epi,
                        int* tile_ctr) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return hipErrorInvalidValue;
  if ((K & 7) || (lda & 7) || (ldb & 7)) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return hipErrorInvalidValue;
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 31) / 32 * 32;
  const int S = (K + kchunk - 1) / kchunk;
  int mode = 0;
  if (epi != nullptr) {
    mode = S == 1 ? 1 : 2;
    if (mode == 2 && (tile_ctr == nullptr || Cp == nullptr)) return hipErrorInvalidValue;
    if (mode == 2 && (epi->bgrad || epi->bsgd)) return hipErrorInvalidValue;
    if (epi->obfT && (epi->ldt & 3)) return hipErrorInvalidValue;
  }
  GemmEpi e{};
  e.alpha = 1.f;
  if (epi) e = *epi;
  // Vectorised SGD epilogue when every row access is 16 B aligned.
  const int sgd_lds = (epi && e.sgdW && !e.mask && !e.of32 && !e.bias && !e.relu && (N % 4) == 0 &&
                       (M % 8) == 0 && (e.ldw % 4) == 0 && (!e.obf || (e.ldb % 4) == 0) &&
                       (!e.obfT || (e.ldt % 8) == 0) && ((uintptr_t)e.sgdW & 15) == 0 &&
                       (!e.obf || ((uintptr_t)e.obf & 7) == 0) &&
                       (!e.obfT || ((uintptr_t)e.obfT & 15) == 0)) ? 1 : 0;
  dim3 grid((N + 63) / 64, (M + 63) / 64, S);
  if (kchunk >= 256)
    hipLaunchKernelGGL(gemm_bf16_nt_k<8>, grid, dim3(256), 0, s, A, lda, B, ldb, Cp, M, N, K,
                       kchunk, e, mode, tile_ctr, sgd_lds);
  else if (kchunk <= 64 && mode == 1)  // weight-gradient GEMMs (K = batch): more blocks per CU
    hipLaunchKernelGGL((gemm_bf16_nt_k<2, false>), grid, dim3(256), 0, s, A, lda, B, ldb, Cp, M, N,
                       K, kchunk, e, mode, tile_ctr, sgd_lds);
  else
    hipLaunchKernelGGL(gemm_bf16_nt_k<4>, grid, dim3(256), 0, s, A, lda, B, ldb, Cp, M, N, K,
                       kchunk, e, mode, tile_ctr, sgd_lds);
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

// Fused classifier head (kernels/head_row.h): one 256-thread block per row;
// replaces a K-long, N = C GEMM (one tile: no parallelism) + the softmax launch.
__device__ uint64_t g_head_stamps[64][6];
__constant__ int g_head_stamp_on;  // __constant__: scalar loads, no vector wait ahead of the batch
#ifdef HIPDSML_MEASURE
__constant__ int g_head_dbg;  // measurement builds: bit 0 skips the stats atomics, bit 1 the dzp phase
#endif
// MAXC: the class count rounded up to an instantiated size (even: class pairs);
// SL: 0 = bf16 H, else H from SL raw split-K slices (head_row.h)
template <int MAXC, int SL = 0>
__global__ __launch_bounds__(256) void head_softmax_xent_k(HeadRow h) {
  __shared__ float part[MAXC][17];     // [class][wave * 4 + 16-lane row] partial sums (+1: pad)
  __shared__ uint32_t gz2[MAXC / 2];   // bf16-rounded dLogits of this row, class pairs
  const int m = blockIdx.x;
#ifdef HIPDSML_MEASURE
  h.dbg = g_head_dbg;
#else
  h.dbg = 0;
#endif
  head_row<MAXC, SL>(h, m, part, gz2, (g_head_stamp_on && m < 64) ? g_head_stamps[m] : nullptr);
}

hipError_t head_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_head_stamps), sizeof(uint64_t) * 64 * 6, 0,
                             hipMemcpyDeviceToHost);
}
#ifdef HIPDSML_MEASURE
void head_set_debug(int v) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_head_dbg), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
#endif
void head_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_head_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}


hipError_t head_softmax_xent(const uint16_t* H, int64_t ldh, const uint16_t* W, int64_t ldw,
                             const float* bias, int B, int K, int C, const int32_t* labels,
                             float inv_batch, float* logits, int64_t ldl, uint16_t* dz, int64_t ldz,
                             uint16_t* dzT, int64_t ldt, int Cp, float* stats, hipStream_t s,
                             uint16_t* dzp, int64_t ldzp, uint16_t* dzpT, int64_t ldpt,
                             int row_stats, const HeadSlabs* hs) {
  if (dzp && ((ldzp & 7) || ((uintptr_t)dzp & 15))) return hipErrorInvalidValue;
  if (row_stats && stats && ((uintptr_t)stats & 15)) return hipErrorInvalidValue;  // float4 per row
  if (C < 1 || C > kHeadMaxC || Cp > 64 || (K & 7) || K > 256 * 8 * kHeadMaxK8 || (ldh & 7) ||
      (ldw & 7) ||
      (((uintptr_t)H | (uintptr_t)W) & 15))
    return hipErrorInvalidValue;
  HeadRow h{H, ldh, W, ldw, bias, K, C, Cp, labels, inv_batch, logits, ldl, dz, ldz, dzT, ldt, stats,
            dzp, ldzp, dzpT, ldpt, row_stats, 0,
            nullptr, 0, 1.f, nullptr, 0, nullptr, 0};
  int sl = 0;
  if (hs != nullptr) {
    // raw split-K slices of ONE 64-row tile block: rows <= 64, K in whole tiles
    if (B > 64 || (K & 63) || !(hs->S == 2 || hs->S == 4 || hs->S == 8) || hs->slabs == nullptr ||
        hs->stride < (int64_t)(K / 64) * 4096 || (hs->stride & 3) || ((uintptr_t)hs->slabs & 15) ||
        (hs->bias && ((uintptr_t)hs->bias & 15)) || hs->Hout == nullptr || (hs->ldo & 7) ||
        ((uintptr_t)hs->Hout & 15))
      return hipErrorInvalidValue;
    sl = hs->S;
    h.hs = hs->slabs;
    h.hs_stride = hs->stride;
    h.hs_alpha = hs->alpha;
    h.hs_bias = hs->bias;
    h.hs_relu = hs->relu;
    h.hout = hs->Hout;
    h.ldho = hs->ldo;
  }
#define DSML_HEAD_LAUNCH(MC)                                                                         \
  switch (sl) {                                                                                      \
    case 0: hipLaunchKernelGGL((head_softmax_xent_k<MC, 0>), dim3(B), dim3(256), 0, s, h); break;  \
    case 2: hipLaunchKernelGGL((head_softmax_xent_k<MC, 2>), dim3(B), dim3(256), 0, s, h); break;  \
    case 4: hipLaunchKernelGGL((head_softmax_xent_k<MC, 4>), dim3(B), dim3(256), 0, s, h); break;  \
    default: hipLaunchKernelGGL((head_softmax_xent_k<MC, 8>), dim3(B), dim3(256), 0, s, h); break; \
  }
  if (C <= 10) {
    DSML_HEAD_LAUNCH(10)
  } else {
    DSML_HEAD_LAUNCH(kHeadMaxC)
  }
#undef DSML_HEAD_LAUNCH
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
