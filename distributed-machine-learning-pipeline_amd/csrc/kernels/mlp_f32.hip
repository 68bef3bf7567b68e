// Fused fp32 MLP training step for CDNA4 (gfx950), exact-f32 MFMA.
//
// Replaces the reference's scalar Go loops (forwardPass client.go:112-141,
// backwardPass client.go:143-202, updateWeights client.go:254-267) with three
// launches per step that the engine captures into one hipGraph:
//
//   K_A  mlp_f32_first_layer_k : Z_1 partials = X . W_1^T     split-K MFMA GEMM,
//                                (ceil(d1/32) x ceil(B/32) x nsplit) workgroups
//   K_B  mlp_f32_rowchain_k    : per 16-row tile, entirely in LDS:
//                                H_1 = relu(sum slabs + b_1), layers 2..L forward,
//                                softmax + cross-entropy (+ eps 1e-10, client.go:151),
//                                dLogits = (p - y)/B, activation gradients down to dZ_1
//                                (ReLU' fused as the H>0 mask, client.go:104-110)
//   K_C  mlp_f32_wgrad_k       : dW_l = dZ_l^T . H_{l-1}, db_l = colsum(dZ_l) for all l
//                                in one flattened tile grid; optionally fused SGD.
//
// Batch rows are independent through the forward and the activation-gradient
// chain, so K_B needs no cross-workgroup communication; only the weight
// gradients reduce over the batch (K_C).  All MFMAs are v_mfma_f32_16x16x4_f32
// (exact f32 fma chain, the numerics class of the reference's fp32 loops).
//
// Latency structure: at B=64 every kernel is latency-bound, so each kernel
// issues ALL of its global loads for a phase before the first dependent use
// (explicit load batches + sched_barrier), giving one memory round trip per
// phase instead of one per K-step.
#include <cstdlib>

#include "common.h"
#include "../dsml.h"

namespace dsml {

__device__ __forceinline__ uint64_t ld_ctr(const int64_t* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ctr(int64_t* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t row_of_step(uint64_t s, int nbatches, int batch) {
  return (int64_t)(s % (uint64_t)nbatches) * (int64_t)batch;
}

// Phase stamps for profiling (block 0, thread 0; s_memrealtime = 100 MHz).
__device__ uint64_t g_dsml_stamps[kMaxStamps];
__device__ int g_dsml_stamp_on;
#define DSML_STAMP(i)                                                        \
  do {                                                                       \
    if (stamp_on && blockIdx.x == 0 && threadIdx.x == 0)                     \
      g_dsml_stamps[(i)] = __builtin_amdgcn_s_memrealtime();                 \
  } while (0)

// ---------------------------------------------------------------------------
// K_A: first layer, split-K.  Workgroup = 4 waves = 32x32 output tile; wave w
// owns the 16x16 sub-tile (w>>1, w&1).  Each lane loads float4 runs along K for
// both operands (X rows and W rows are K-contiguous), so one 16-deep K step is
// 2 x 16 B loads + 4 MFMAs per lane.  All (<=8) K steps of a split are loaded
// before the MFMA chain.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mlp_f32_first_layer_k(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ P,
    float* __restrict__ slab, int64_t* __restrict__ ctr, int64_t row0, MlpDesc d,
    int kchunk, const int32_t* __restrict__ labels, float* __restrict__ ws) {
  const int B = d.batch, K = d.dims[0], N = d.dims[1];
  const float* __restrict__ W = P + d.w_off[0];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int mt = blockIdx.y * 32 + (w >> 1) * 16;
  const int nt = blockIdx.x * 32 + (w & 1) * 16;
  const int m = mt + i, n = nt + i;
  const bool mv = m < B, nv = n < N;
  const int kb = blockIdx.z * kchunk;
  const int ke = min(K, kb + kchunk);

  // Step counter first, then the weight loads (independent of it) so the
  // counter's wait does not also drain the weight loads (vmcnt is in order).
  const uint64_t step = ctr ? ld_ctr(ctr + 1) : 0;
  const float* wb = W + (int64_t)(nv ? n : N - 1) * K;
  float4 a[8], b[8];
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int kk = kb + it * 16 + 4 * q;
    b[it] = *reinterpret_cast<const float4*>(wb + (kk < ke ? kk : ke - 4));
  }
  const int64_t r0 = ctr ? row_of_step(step, d.nbatches, B) : row0;
  if (ctr != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
    // Stage this batch's labels for K_B and hand the counter on: A = s + 1.
    int32_t* lab = reinterpret_cast<int32_t*>(ws + d.lab_off);
    for (int t = threadIdx.x; t < B; t += 256) lab[t] = labels[r0 + t];
    if (threadIdx.x == 0) st_ctr(ctr, step + 1);
  }
  const float* xa = X + (r0 + (mv ? m : B - 1)) * ldx;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int kk = kb + it * 16 + 4 * q;
    a[it] = *reinterpret_cast<const float4*>(xa + (kk < ke ? kk : ke - 4));
  }
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int kk = kb + it * 16 + 4 * q;
    const bool kv = kk < ke;
    const float4 av = sel4(kv && mv, a[it]);
    const float4 bv = sel4(kv && nv, b[it]);
    acc0 = mfma_f32_16x16x4(av.x, bv.x, acc0);
    acc1 = mfma_f32_16x16x4(av.y, bv.y, acc1);
    acc0 = mfma_f32_16x16x4(av.z, bv.z, acc0);
    acc1 = mfma_f32_16x16x4(av.w, bv.w, acc1);
  }
  float* out = slab + (int64_t)blockIdx.z * B * N;
  if (nv) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt + 4 * q + r;
      if (row < B) out[(int64_t)row * N + n] = acc0[r] + acc1[r];
    }
  }
}

// Copy `rows` x `cols` floats (cols % 4 == 0, 16 B aligned, contiguous rows)
// from global into LDS with row stride `lstride`, 8 float4 loads in flight per
// thread before the first LDS store.
__device__ __forceinline__ void stage_rows(float* __restrict__ dst, int lstride,
                                           const float* __restrict__ src, int rows, int cols,
                                           int tid) {
  const int c4 = cols >> 2;
  const int n4 = rows * c4;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  for (int base = tid; base < n4; base += 256 * 8) {
    float4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int idx = base + j * 256;
      v[j] = s4[idx < n4 ? idx : n4 - 1];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int idx = base + j * 256;
      if (idx < n4) {
        const int r = idx / c4, c = idx - r * c4;
        *reinterpret_cast<float4*>(dst + r * lstride + 4 * c) = v[j];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K_B: row chain.  One workgroup (4 waves) per 16 batch rows.  Phase 1 stages
// W_l, b_l (l >= 2) into LDS and reduces the split-K slabs of layer 1; phase 2
// runs every remaining GEMM from LDS.
// ---------------------------------------------------------------------------
template <bool WLDS>
__global__ __launch_bounds__(256) void mlp_f32_rowchain_k(
    const float* __restrict__ P, const float* __restrict__ slab, int nsplit,
    float* __restrict__ ws, const int32_t* __restrict__ labels, int64_t* __restrict__ ctr,
    int64_t row0, MlpDesc d, float* __restrict__ stats, int train, float inv_batch) {
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int L = d.nlayers, B = d.batch;
  const int m0 = blockIdx.x * kRowTile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int stamp_on = g_dsml_stamp_on;
  DSML_STAMP(0);

  // Labels: staged by K_A for training steps (ctr != nullptr), direct for eval.
  const int32_t* lab = ctr ? reinterpret_cast<const int32_t*>(ws + d.lab_off) : labels + row0;
  // ---- phase 1a: stage weights of layers 2..L into LDS ----------------------
  if constexpr (WLDS) {
    for (int l = 2; l <= L; ++l) {
      const int K = d.dims[l - 1], N = d.dims[l];
      stage_rows(lds + d.lds_w[l], K + 4, P + d.w_off[l - 1], N, K, tid);
      for (int c = tid; c < N; c += 256) lds[d.lds_b[l] + c] = P[d.b_off[l - 1] + c];
    }
  }

  // ---- phase 1b: layer-1 epilogue  H_1 = relu(sum_s slab_s + b_1) -----------
  {
    const int N1 = d.dims[1];
    const int s1 = d.lds_stride[1];
    const int N1p = (N1 + 15) & ~15;
    float* a1 = lds + d.lds_act[1];
    const float* b1 = P + d.b_off[0];
    const bool relu = L > 1;
    float* H1 = ws + d.act_off[1];
    if ((N1 & 3) == 0) {
      const int c4n = N1 >> 2;
      for (int idx = tid; idx < kRowTile * c4n; idx += 256) {
        const int r = idx / c4n, c = (idx - r * c4n) * 4;
        const int m = m0 + r;
        const int mc = m < B ? m : B - 1;
        float4 part[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int sc = s < nsplit ? s : nsplit - 1;
          part[s] = *reinterpret_cast<const float4*>(slab + ((int64_t)sc * B + mc) * N1 + c);
        }
        float4 v = *reinterpret_cast<const float4*>(b1 + c);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          if (s < nsplit) { v.x += part[s].x; v.y += part[s].y; v.z += part[s].z; v.w += part[s].w; }
        }
        if (m >= B) v = zero4();
        if (relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        *reinterpret_cast<float4*>(a1 + r * s1 + c) = v;
        if (train && relu && m < B) *reinterpret_cast<float4*>(H1 + (int64_t)m * N1 + c) = v;
      }
      for (int idx = tid; idx < kRowTile * (N1p - N1); idx += 256) {
        const int r = idx / (N1p - N1), c = N1 + idx - r * (N1p - N1);
        a1[r * s1 + c] = 0.f;
      }
    } else {
      for (int idx = tid; idx < kRowTile * N1p; idx += 256) {
        const int r = idx / N1p, c = idx - r * N1p;
        const int m = m0 + r;
        float v = 0.f;
        if (c < N1 && m < B) {
          v = b1[c];
          for (int s = 0; s < nsplit; ++s) v += slab[((int64_t)s * B + m) * N1 + c];
          if (relu) v = fmaxf(v, 0.f);
          if (train && relu) H1[(int64_t)m * N1 + c] = v;
        }
        a1[r * s1 + c] = v;
      }
    }
  }
  __syncthreads();
  DSML_STAMP(1);

  // ---- phase 2: forward through layers 2..L (all operands in LDS) ----------
  for (int l = 2; l <= L; ++l) {
    const int K = d.dims[l - 1], N = d.dims[l];
    const int sA = d.lds_stride[l - 1], sO = d.lds_stride[l];
    const float* A = lds + d.lds_act[l - 1];
    float* O = lds + d.lds_act[l];
    const float* W = WLDS ? lds + d.lds_w[l] : P + d.w_off[l - 1];
    const int sW = WLDS ? K + 4 : K;
    const float* bias = WLDS ? lds + d.lds_b[l] : P + d.b_off[l - 1];
    const bool relu = l < L;
    float* Hg = ws + d.act_off[l];
    const int nblk = (N + 15) >> 4;
    for (int cb = wave; cb < nblk; cb += 4) {
      const int n = cb * 16 + i;
      const bool nv = n < N;
      const float* wr = W + (nv ? n : N - 1) * sW;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < K; k += 16) {
        const int kk = k + 4 * q;
        const bool kv = kk < K;
        const float4 av = sel4(kv, *reinterpret_cast<const float4*>(A + i * sA + kk));
        const float4 bv = sel4(kv && nv, *reinterpret_cast<const float4*>(wr + (kv ? kk : 0)));
        acc0 = mfma_f32_16x16x4(av.x, bv.x, acc0);
        acc1 = mfma_f32_16x16x4(av.y, bv.y, acc1);
        acc0 = mfma_f32_16x16x4(av.z, bv.z, acc0);
        acc1 = mfma_f32_16x16x4(av.w, bv.w, acc1);
      }
      const float bn = nv ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        float v = nv ? acc0[r] + acc1[r] + bn : 0.f;
        if (relu) v = fmaxf(v, 0.f);
        if (m0 + row >= B) v = 0.f;
        O[row * sO + n] = v;
        if (train && relu && nv && m0 + row < B) Hg[(int64_t)(m0 + row) * N + n] = v;
      }
    }
    __syncthreads();
  }
  DSML_STAMP(2);

  // ---- softmax + cross-entropy + dLogits (wave 0: 4 lanes per row) --------
  {
    const int C = d.dims[L];
    const int sL = d.lds_stride[L];
    const int Cp = (C + 15) & ~15;
    const float* Z = lds + d.lds_act[L];
    float* G = lds + d.lds_dz[L];
    float* Gg = ws + d.dz_off[L];
    if (wave == 0) {
      const int r = lane >> 2, sub = lane & 3;
      const int m = m0 + r;
      const bool valid = m < B;
      const int y = valid ? lab[m] : -1;
      float mx = -3.402823466e38f;
      int amax = 0x7fffffff;
      for (int c = sub; c < C; c += 4) {
        const float z = Z[r * sL + c];
        if (z > mx) { mx = z; amax = c; }
      }
      quad_argmax(mx, amax);
      float se = 0.f;
      for (int c = sub; c < C; c += 4) se += expf(Z[r * sL + c] - mx);
      se = quad_sum(se);
      const float inv = 1.f / se;
      float loss = 0.f;
      for (int c = sub; c < Cp; c += 4) {
        float g = 0.f;
        if (c < C && valid) {
          const float p = expf(Z[r * sL + c] - mx) * inv;
          if (c == y) loss = -logf(p + 1e-10f);
          g = (p - (c == y ? 1.f : 0.f)) * inv_batch;
          if (train == 1) Gg[(int64_t)m * C + c] = g;
          else if (train == 2) Gg[(int64_t)m * C + c] = Z[r * sL + c];  // logits out
        }
        G[r * sL + c] = g;
      }
      float correct = (sub == 0 && valid && amax == y) ? 1.f : 0.f;
      float cnt = (sub == 0 && valid) ? 1.f : 0.f;
      loss = wave_sum(loss);
      correct = wave_sum(correct);
      cnt = wave_sum(cnt);
      if (lane == 0 && stats != nullptr) {
        atomicAdd(stats + 0, loss);
        atomicAdd(stats + 1, correct);
        atomicAdd(stats + 2, cnt);
      }
    }
  }
  if (train != 1) return;
  __syncthreads();
  DSML_STAMP(3);

  // ---- backward activation chain: dZ_{l-1} = (dZ_l . W_l) * (H_{l-1} > 0) --
  for (int l = L; l >= 2; --l) {
    const int N = d.dims[l];       // reduction dim
    const int K = d.dims[l - 1];   // output columns
    const int sG = d.lds_stride[l], sH = d.lds_stride[l - 1];
    const float* Gz = lds + d.lds_dz[l];
    const float* H = lds + d.lds_act[l - 1];
    float* Go = lds + d.lds_dz[l - 1];
    float* Gg = ws + d.dz_off[l - 1];
    const float* W = WLDS ? lds + d.lds_w[l] : P + d.w_off[l - 1];
    const int sW = WLDS ? K + 4 : K;
    const int kblk = (K + 15) >> 4;
    for (int cb = wave; cb < kblk; cb += 4) {
      const int kc = cb * 16 + i;
      const bool kcv = kc < K;
      const int kcc = kcv ? kc : K - 1;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int n = 0; n < N; n += 16) {
        const int nn = n + 4 * q;
        const float4 av = *reinterpret_cast<const float4*>(Gz + i * sG + nn);
        float bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = nn + s;
          const float t = W[(row < N ? row : N - 1) * sW + kcc];
          bv[s] = (row < N && kcv) ? t : 0.f;
        }
        acc0 = mfma_f32_16x16x4(av.x, bv[0], acc0);
        acc1 = mfma_f32_16x16x4(av.y, bv[1], acc1);
        acc0 = mfma_f32_16x16x4(av.z, bv[2], acc0);
        acc1 = mfma_f32_16x16x4(av.w, bv[3], acc1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        float v = 0.f;
        if (kcv) v = (H[row * sH + kc] > 0.f) ? acc0[r] + acc1[r] : 0.f;
        Go[row * sH + kc] = v;
        if (kcv && m0 + row < B) Gg[(int64_t)(m0 + row) * K + kc] = v;
      }
    }
    __syncthreads();
  }
  DSML_STAMP(4);
}

// ---------------------------------------------------------------------------
// K_C: weight gradients.  One wave per 16(n) x 32(k) tile of dW_l; reduction
// over the batch rows in MFMA k-steps of 4, 64 rows (16 k-steps, 48 loads per
// lane) per load batch.  Tiles of all layers are flattened into one grid.
// db_l comes from the A-operand values of the k-tile-0 waves.  Fused SGD
// (single replica) updates P in place; the kernel never reads W, so the
// in-place update inside the launch is race-free.
// ---------------------------------------------------------------------------
// System-coherent accesses for the peer exchange (bypass the non-coherent
// caches: sc0 sc1), so no L2 writeback / invalidate fences are needed.
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ float ld_sys(const float* p) {
  return __builtin_bit_cast(float, __hip_atomic_load((const gu32*)(p), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ void st_sys(float* p, float v) {
  __hip_atomic_store((gu32*)(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys64(uint64_t* p, uint64_t v) {
  __hip_atomic_store((gu64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a[k] for a runtime k from a kernel-argument array, by selects (a dynamic
// index would copy the array to scratch memory first)
template <typename T>
__device__ __forceinline__ T pick_peer(const T (&a)[kMaxPeers], int k) {
  T r = a[0];
#pragma unroll
  for (int j = 1; j < kMaxPeers; ++j) r = k == j ? a[j] : r;
  return r;
}

template <bool XCHG>
__global__ __launch_bounds__(64) void mlp_f32_wgrad_k(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ P, float* __restrict__ Gout,
    const float* __restrict__ ws, int64_t* __restrict__ ctr, int64_t row0, MlpDesc d, float lr,
    int fused_sgd, XchgArgs xa, XchgTab tab) {
  const int B = d.batch;
  int bid = blockIdx.x;
  int l = 0;
  for (; l < d.nlayers - 1; ++l) {
    const int nt = ((d.dims[l + 1] + 15) >> 4) * ((d.dims[l] + 31) >> 5);
    if (bid < nt) break;
    bid -= nt;
  }
  const int N = d.dims[l + 1], K = d.dims[l];
  const int ntk = (K + 31) >> 5;
  const int tn = bid / ntk, tk = bid - tn * ntk;
  const int lane = threadIdx.x, i = lane & 15, q = lane >> 4;
  const int n = tn * 16 + i;
  const int k0 = tk * 32 + i, k1 = k0 + 16;
  const bool nv = n < N, k0v = k0 < K, k1v = k1 < K;
  const int nc = nv ? n : N - 1, k0c = k0v ? k0 : K - 1, k1c = k1v ? k1 : K - 1;
  const float* dZ = ws + d.dz_off[l + 1];
  const float* Ain;
  int64_t lda;
  if (l == 0) {
    const int64_t r0 = ctr ? row_of_step(ld_ctr(ctr) - 1, d.nbatches, B) : row0;
    Ain = X + r0 * ldx;
    lda = ldx;
  } else {
    Ain = ws + d.act_off[l];
    lda = K;
  }

  // Fused SGD reads the old weights: issue those loads with the operand batch.
  float wold[4][2] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  float bold = 0.f;
  const int64_t woff = d.w_off[l];
  if (fused_sgd) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = tn * 16 + 4 * q + r;
      const float* wr = P + woff + (int64_t)(row < N ? row : N - 1) * K;
      wold[r][0] = wr[k0c];
      wold[r][1] = wr[k1c];
    }
    bold = P[d.b_off[l] + nc];
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  for (int mb = 0; mb < B; mb += 64) {
    float av[16], b0[16], b1[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int mm = mb + 4 * s + q;
      const int mc = mm < B ? mm : B - 1;
      av[s] = dZ[(int64_t)mc * N + nc];
      b0[s] = Ain[(int64_t)mc * lda + k0c];
      b1[s] = Ain[(int64_t)mc * lda + k1c];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool mv = (mb + 4 * s + q) < B;
      const float a = (mv && nv) ? av[s] : 0.f;
      const float x0 = (mv && k0v) ? b0[s] : 0.f;
      const float x1 = (mv && k1v) ? b1[s] : 0.f;
      dbacc += a;
      acc0 = mfma_f32_16x16x4(a, x0, acc0);
      acc1 = mfma_f32_16x16x4(a, x1, acc1);
    }
  }
  dbacc += __shfl_xor(dbacc, 16, 64);
  dbacc += __shfl_xor(dbacc, 32, 64);

  if constexpr (XCHG) {
    // ---- publish this tile, wait for the peers' copies, sum in rank order ----
    const uint64_t step = ld_ctr(ctr) - 1;
    const uint64_t want = step + 1;
    const int64_t poff = (int64_t)(step & 1) * xa.half;
    // the peer pointer table is a kernel argument (no dependent load of the
    // device copy before the first publish / poll address is known)
    const bool bl = tk == 0 && q == 0;
    float* mine = pick_peer(tab.buf, xa.rank) + poff;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = tn * 16 + 4 * q + r;
      if (row < N) {
        if (k0v) st_sys(mine + woff + (int64_t)row * K + k0, acc0[r]);
        if (k1v) st_sys(mine + woff + (int64_t)row * K + k1, acc1[r]);
      }
    }
    if (bl && nv) st_sys(mine + d.b_off[l] + n, dbacc);
    // every lane's payload stores are complete before the flag is raised
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      st_sys64(pick_peer(tab.flags, xa.rank) + blockIdx.x, want);
    if (lane < xa.nranks && lane != xa.rank)
      (void)poll_flag_ge<2>(pick_peer(tab.flags, lane) + blockIdx.x, want, xa.err,
                            xa.timeout_ticks);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __asm__ volatile("" ::: "memory");
    // All peers' tiles in one load batch, then the ordered sum.
    const int rc[4] = {min(tn * 16 + 4 * q + 0, N - 1), min(tn * 16 + 4 * q + 1, N - 1),
                       min(tn * 16 + 4 * q + 2, N - 1), min(tn * 16 + 4 * q + 3, N - 1)};
    float pv[kMaxPeers][9];
#pragma unroll
    for (int p = 0; p < kMaxPeers; ++p) {
      if (p < xa.nranks && p != xa.rank) {
        const float* pb = tab.buf[p] + poff;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pv[p][2 * r] = ld_sys(pb + woff + (int64_t)rc[r] * K + k0c);
          pv[p][2 * r + 1] = ld_sys(pb + woff + (int64_t)rc[r] * K + k1c);
        }
        pv[p][8] = bl ? ld_sys(pb + d.b_off[l] + nc) : 0.f;
      }
    }
    float sum[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) sum[j] = 0.f;
#pragma unroll
    for (int p = 0; p < kMaxPeers; ++p) {
      if (p < xa.nranks) {
        const bool me = p == xa.rank;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sum[2 * r] += me ? acc0[r] : pv[p][2 * r];
          sum[2 * r + 1] += me ? acc1[r] : pv[p][2 * r + 1];
        }
        sum[8] += me ? dbacc : pv[p][8];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc0[r] = sum[2 * r];
      acc1[r] = sum[2 * r + 1];
    }
    dbacc = sum[8];
  }

  float* Wt = fused_sgd ? P : Gout;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = tn * 16 + 4 * q + r;
    if (row < N) {
      float* wr = Wt + woff + (int64_t)row * K;
      if (fused_sgd) {
        if (k0v) wr[k0] = wold[r][0] - lr * acc0[r];
        if (k1v) wr[k1] = wold[r][1] - lr * acc1[r];
      } else {
        if (k0v) wr[k0] = acc0[r];
        if (k1v) wr[k1] = acc1[r];
      }
    }
  }
  if (tk == 0 && q == 0 && nv) {
    float* bp = Wt + d.b_off[l] + n;
    if (fused_sgd) *bp = bold - lr * dbacc;
    else *bp = dbacc;
  }
  // Step-counter hand-off: B = A (K_C never reads B; A is not written here).
  if (ctr != nullptr && blockIdx.x == 0 && lane == 0) st_ctr(ctr + 1, ld_ctr(ctr));
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
MlpLaunchCfg mlp_plan_first_layer(const MlpDesc& d) {
  const int K = d.dims[0];
  const int kblocks = (K + 15) / 16;
  const int tiles = ((d.dims[1] + 31) / 32) * ((d.batch + 31) / 32);
  // Aim for >= ~64 workgroups; each split covers at most 8 K-steps (128).
  const int want = (64 + tiles - 1) / tiles;
  const int minsplit = (kblocks + 7) / 8;
  int nsplit = want > minsplit ? want : minsplit;
  if (nsplit > 8 && minsplit <= 8) nsplit = 8;  // the row chain sums <= 8 slabs
  if (nsplit > kblocks) nsplit = kblocks;
  const int per = (kblocks + nsplit - 1) / nsplit;
  MlpLaunchCfg c;
  c.kchunk = per * 16;
  c.nsplit = (kblocks + per - 1) / per;
  return c;
}

int mlp_wgrad_tiles(const MlpDesc& d) {
  int t = 0;
  for (int l = 0; l < d.nlayers; ++l) t += ((d.dims[l + 1] + 15) / 16) * ((d.dims[l] + 31) / 32);
  return t;
}

bool mlp_rowchain_fits(const MlpDesc& d) { return d.lds_floats * 4 <= 160 * 1024; }

hipError_t mlp_f32_first_layer(const float* X, int64_t ldx, const float* P, float* slab,
                               int64_t* ctr, int64_t row0, const MlpDesc& d,
                               const MlpLaunchCfg& c, const int32_t* labels, float* ws,
                               hipStream_t s) {
  dim3 grid((d.dims[1] + 31) / 32, (d.batch + 31) / 32, c.nsplit);
  hipLaunchKernelGGL(mlp_f32_first_layer_k, grid, dim3(256), 0, s, X, ldx, P, slab, ctr, row0,
                     d, c.kchunk, labels, ws);
  return hipGetLastError();
}

hipError_t mlp_f32_rowchain(const float* P, const float* slab, int nsplit, float* ws,
                            const int32_t* labels, int64_t* ctr, int64_t row0,
                            const MlpDesc& d, float* stats, int train, float inv_batch,
                            hipStream_t s) {
  if (nsplit < 1 || nsplit > 8) return hipErrorInvalidValue;
  {
    const hipError_t e = mlp_f32_rowchain_fast(P, slab, nsplit, ws, labels, ctr, row0, d, stats,
                                               train, inv_batch, s);
    if (e != hipErrorNotSupported) return e;
  }
  dim3 grid((d.batch + kRowTile - 1) / kRowTile);
  const size_t lds = (size_t)d.lds_floats * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (d.w_in_lds) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(mlp_f32_rowchain_k<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(mlp_f32_rowchain_k<true>, grid, dim3(256), lds, s, P, slab, nsplit, ws,
                       labels, ctr, row0, d, stats, train, inv_batch);
  } else {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(mlp_f32_rowchain_k<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(mlp_f32_rowchain_k<false>, grid, dim3(256), lds, s, P, slab, nsplit, ws,
                       labels, ctr, row0, d, stats, train, inv_batch);
  }
  return hipGetLastError();
}

hipError_t mlp_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_dsml_stamps), sizeof(uint64_t) * kMaxStamps,
                             0, hipMemcpyDeviceToHost);
}

void mlp_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dsml_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

hipError_t mlp_f32_wgrad(const float* X, int64_t ldx, float* P, float* G, const float* ws,
                         int64_t* ctr, int64_t row0, const MlpDesc& d, float lr, int fused_sgd,
                         hipStream_t s) {
  dim3 grid(mlp_wgrad_tiles(d));
  hipLaunchKernelGGL(mlp_f32_wgrad_k<false>, grid, dim3(64), 0, s, X, ldx, P, G, ws, ctr, row0, d,
                     lr, fused_sgd, XchgArgs{}, XchgTab{});
  return hipGetLastError();
}

hipError_t mlp_f32_wgrad_xchg(const float* X, int64_t ldx, float* P, const float* ws, int64_t* ctr,
                              const MlpDesc& d, float lr_over_n, const XchgArgs& x,
                              const XchgTab& tab, hipStream_t s) {
  if (ctr == nullptr || x.tab == nullptr || x.err == nullptr || x.nranks < 1 ||
      x.nranks > kMaxPeers || x.rank < 0 || x.rank >= x.nranks)
    return hipErrorInvalidValue;
  dim3 grid(mlp_wgrad_tiles(d));
  hipLaunchKernelGGL(mlp_f32_wgrad_k<true>, grid, dim3(64), 0, s, X, ldx, P, nullptr, ws, ctr, 0,
                     d, lr_over_n, 1, x, tab);
  return hipGetLastError();
}

}  // namespace dsml
