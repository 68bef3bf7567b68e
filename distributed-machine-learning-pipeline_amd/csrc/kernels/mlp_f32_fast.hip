// Shape-specialised row-chain kernel (K_B) for 3-layer MLPs D0-D1-D2-D3 with
// compile-time hidden/output dims (instantiated for the BASELINE model
// 784-128-64-10 and a few neighbours).  Same math and outputs as the generic
// mlp_f32_rowchain_k (mlp_f32.hip), restructured for latency at B = 64:
//
//  * every global load of the kernel (split-K slabs of layer 1, b1, W2, W3,
//    b2, b3) is issued in ONE straight-line batch (~27 x 16 B per lane), so the
//    whole prologue costs one memory round trip; the step counter and the
//    labels ride in the same batch;
//  * all trip counts are compile-time, so every MFMA chain is fully unrolled
//    with its LDS operand reads hoisted ahead of the MFMAs;
//  * layer 3 (N = D3 <= 16) splits its K = D2 reduction across the 4 waves
//    and reduces the 4 partial 16x16 tiles through LDS inside the softmax.
//
// Reference math: client.go:112-202 (forward, softmax-CE eps 1e-10, (p-y)/B,
// ReLU' mask).
#include "common.h"
#include "../dsml.h"

namespace dsml {

// Phase stamps of block 0 (s_memrealtime, 100 MHz), profiling only.
__device__ uint64_t g_fast_stamps[kMaxStamps];
__device__ int g_fast_stamp_on;
#define FAST_STAMP(i)                                                        \
  do {                                                                       \
    if (stamp_on && blockIdx.x == 0 && threadIdx.x == 0) {                   \
      g_fast_stamps[(i)] = __builtin_amdgcn_s_memrealtime();                 \
      g_fast_stamps[16 + (i)] = __builtin_amdgcn_s_memtime();                \
    }                                                                        \
  } while (0)

typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

template <int D1, int D2, int D3>
struct Mlp3Lds {
  static constexpr int S1 = D1 + 4;   // H1 row stride (floats)
  static constexpr int S2 = D2 + 4;   // H2 / dZ2 row stride
  static constexpr int S3 = 16 + 4;   // logits / dZ3 row stride (padded to 16 cols)
  static constexpr int W2S = D1 + 4;  // W2 [D2][D1] staged row stride
  static constexpr int W3S = D2 + 4;  // W3 [D3][D2]
  static constexpr int H1 = 0;
  static constexpr int H2 = H1 + kRowTile * S1;
  static constexpr int DZ2 = H2 + kRowTile * S2;
  static constexpr int DZ3 = DZ2 + kRowTile * S2;
  static constexpr int RED = DZ3 + kRowTile * S3;         // 4 x 16 x 16 partial logits
  static constexpr int W2 = RED + 4 * 16 * 16;
  static constexpr int W3 = W2 + D2 * W2S;
  static constexpr int B2 = W3 + 16 * W3S;                // W3 rows padded to 16 (zeros)
  static constexpr int B3 = B2 + D2;
  static constexpr int TOTAL = B3 + 16;
};

template <int D1, int D2, int D3>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void mlp3_rowchain_k(
    const float* __restrict__ P, const float* __restrict__ slab, int nsplit,
    float* __restrict__ ws, const int32_t* __restrict__ labels, int64_t* __restrict__ ctr,
    int64_t row0, MlpDesc d, float* __restrict__ stats, int train, float inv_batch) {
  static_assert(D1 % 16 == 0 && D2 % 16 == 0 && D3 >= 1 && D3 <= 16, "unsupported dims");
  using Lay = Mlp3Lds<D1, D2, D3>;
  constexpr int NS = 8;  // max split-K slabs
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int B = d.batch;
  const int m0 = blockIdx.x * kRowTile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int stamp_on = g_fast_stamp_on;
  FAST_STAMP(0);

  // ------------------------------------------------------------------ loads
  // W2 [D2][D1] and W3 [D3][D2] go global -> LDS by LDS-DMA (no VGPRs, no
  // waits): one dword per lane, 256 B per wave instruction, so the +4 padded
  // LDS rows stay legal (no instruction crosses a row).
  {
    constexpr int P2 = (D1 + 63) / 64;  // dword-DMA instructions per W2 row
    const float* W2g = P + d.w_off[1];
    for (int idx = wave; idx < D2 * P2; idx += 4) {
      const int row = idx / P2, part = idx - row * P2;
      const int col = part * 64 + lane;
      if (col < D1)
        __builtin_amdgcn_global_load_lds((gptr_t)(W2g + row * D1 + col),
                                         (lptr_t)(lds + Lay::W2 + row * Lay::W2S + part * 64), 4, 0, 0);
    }
    constexpr int P3 = (D2 + 63) / 64;
    const float* W3g = P + d.w_off[2];
    for (int idx = wave; idx < D3 * P3; idx += 4) {
      const int row = idx / P3, part = idx - row * P3;
      const int col = part * 64 + lane;
      if (col < D2)
        __builtin_amdgcn_global_load_lds((gptr_t)(W3g + row * D2 + col),
                                         (lptr_t)(lds + Lay::W3 + row * Lay::W3S + part * 64), 4, 0, 0);
    }
  }
  constexpr int C4 = D1 / 4;                     // float4 per H1 row
  constexpr int E = kRowTile * C4;               // float4 elements of the H1 tile
  constexpr int EPT = (E + 255) / 256;
  float4 part[EPT][NS];
  float4 bias1[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = tid + 256 * j;
    const int ec = e < E ? e : E - 1;
    const int r = ec / C4, c = (ec - r * C4) * 4;
    const int m = (m0 + r) < B ? (m0 + r) : B - 1;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int sc = s < nsplit ? s : nsplit - 1;
      part[j][s] = *reinterpret_cast<const float4*>(slab + ((int64_t)sc * B + m) * D1 + c);
    }
    bias1[j] = *reinterpret_cast<const float4*>(P + d.b_off[0] + c);
  }
  float b2v = 0.f, b3v = 0.f;
  if (tid < D2) b2v = P[d.b_off[1] + tid];
  if (tid < 16) b3v = tid < D3 ? P[d.b_off[2] + tid] : 0.f;
  // Labels: staged by K_A for training steps (ctr != nullptr), direct for eval.
  const int32_t* lab = ctr ? reinterpret_cast<const int32_t*>(ws + d.lab_off) : labels + row0;
  // softmax: wave w owns rows 4w..4w+3, 16 lanes (one class each) per row
  const int srow = wave * 4 + (lane >> 4);
  int y = -1;
  if (m0 + srow < B) y = lab[m0 + srow];
  __builtin_amdgcn_sched_barrier(0);

  // ------------------------------------------------- stage + layer-1 epilogue
  // zero the padding rows D3..15 of W3 (read by the layer-3 backward)
  for (int e = tid; e < (16 - D3) * D2; e += 256)
    lds[Lay::W3 + (D3 + e / D2) * Lay::W3S + (e % D2)] = 0.f;
  if (tid < D2) lds[Lay::B2 + tid] = b2v;
  if (tid < 16) lds[Lay::B3 + tid] = b3v;
  float* H1g = ws + d.act_off[1];
  float4 h1v[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = tid + 256 * j;
    if (e < E) {
      const int r = e / C4, c = (e - r * C4) * 4;
      const int m = m0 + r;
      float4 v = bias1[j];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        // select (not branch): keeps the unrolled adds, no runtime-indexed array
        const float4 p = sel4(s < nsplit, part[j][s]);
        v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
      }
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
      if (m >= B) v = zero4();
      *reinterpret_cast<float4*>(lds + Lay::H1 + r * Lay::S1 + c) = v;
      h1v[j] = v;
    }
  }
  full_barrier();  // W2/W3 LDS-DMA + H1 tile complete
  FAST_STAMP(1);
  // H1 -> HBM for the weight-gradient kernel, issued after the barrier so no
  // barrier waits on these stores.
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = tid + 256 * j;
    const int r = e / C4, c = (e - r * C4) * 4;
    if (train && e < E && m0 + r < B) *reinterpret_cast<float4*>(H1g + (int64_t)(m0 + r) * D1 + c) = h1v[j];
  }

  // --------------------------------------------- layer 2: H2 = relu(H1 W2^T + b2)
  float* H2g = ws + d.act_off[2];
#pragma unroll
  for (int cb = wave; cb < D2 / 16; cb += 4) {
    const int n = cb * 16 + i;
    float4 av[D1 / 16], bv[D1 / 16];
#pragma unroll
    for (int ks = 0; ks < D1 / 16; ++ks) {
      av[ks] = *reinterpret_cast<const float4*>(lds + Lay::H1 + i * Lay::S1 + ks * 16 + 4 * q);
      bv[ks] = *reinterpret_cast<const float4*>(lds + Lay::W2 + n * Lay::W2S + ks * 16 + 4 * q);
    }
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < D1 / 16; ++ks) {
      a0 = mfma_f32_16x16x4(av[ks].x, bv[ks].x, a0);
      a1 = mfma_f32_16x16x4(av[ks].y, bv[ks].y, a1);
      a0 = mfma_f32_16x16x4(av[ks].z, bv[ks].z, a0);
      a1 = mfma_f32_16x16x4(av[ks].w, bv[ks].w, a1);
    }
    const float bn = lds[Lay::B2 + n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * q + r;
      float v = fmaxf(a0[r] + a1[r] + bn, 0.f);
      if (m0 + row >= B) v = 0.f;
      lds[Lay::H2 + row * Lay::S2 + n] = v;
      if (train && m0 + row < B) H2g[(int64_t)(m0 + row) * D2 + n] = v;
    }
  }
  lds_barrier();
  FAST_STAMP(2);

  // ------------------------------ layer 3 partial logits: K = D2 split over waves
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = wave; ks < D2 / 16; ks += 4) {
      const float4 av = *reinterpret_cast<const float4*>(lds + Lay::H2 + i * Lay::S2 + ks * 16 + 4 * q);
      const float4 bv = *reinterpret_cast<const float4*>(lds + Lay::W3 + i * Lay::W3S + ks * 16 + 4 * q);
      acc = mfma_f32_16x16x4(av.x, bv.x, acc);
      acc = mfma_f32_16x16x4(av.y, bv.y, acc);
      acc = mfma_f32_16x16x4(av.z, bv.z, acc);
      acc = mfma_f32_16x16x4(av.w, bv.w, acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) lds[Lay::RED + wave * 256 + (4 * q + r) * 16 + i] = acc[r];
  }
  lds_barrier();
  FAST_STAMP(3);

  // ---------------------- softmax + CE + dLogits: 16 lanes per row, 4 rows per wave
  float* G3g = ws + d.dz_off[3];
  {
    const int r = srow, c = lane & 15;
    const int m = m0 + r;
    const bool valid = m < B;
    const bool cv = c < D3;
    float z = -3.402823466e38f;
    if (cv) {
      z = lds[Lay::B3 + c];
#pragma unroll
      for (int w = 0; w < 4; ++w) z += lds[Lay::RED + w * 256 + r * 16 + c];
    }
    float mx = z;
    int amax = cv ? c : 0x7fffffff;
    row16_argmax(mx, amax);
    const float e = cv ? expf(z - mx) : 0.f;
    const float se = row16_sum(e);
    const float p = e / se;
    float g = 0.f, loss = 0.f;
    if (cv && valid) {
      g = (p - (c == y ? 1.f : 0.f)) * inv_batch;
      if (c == y) loss = -logf(p + 1e-10f);
      if (train == 1) G3g[(int64_t)m * D3 + c] = g;
      else if (train == 2) G3g[(int64_t)m * D3 + c] = z;  // logits out (RunForward)
    }
    lds[Lay::DZ3 + r * Lay::S3 + c] = g;
    float correct = (c == 0 && valid && amax == y) ? 1.f : 0.f;
    float cnt = (c == 0 && valid) ? 1.f : 0.f;
    loss = wave_sum(loss);
    correct = wave_sum(correct);
    cnt = wave_sum(cnt);
    if (lane == 0 && stats != nullptr && cnt > 0.f) {
      atomicAdd(stats + 0, loss);
      atomicAdd(stats + 1, correct);
      atomicAdd(stats + 2, cnt);
    }
  }
  if (train != 1) return;
  lds_barrier();
  FAST_STAMP(4);

  // ------------------------- layer 3 backward: dZ2 = (dZ3 W3) * (H2 > 0)
  float* G2g = ws + d.dz_off[2];
#pragma unroll
  for (int cb = wave; cb < D2 / 16; cb += 4) {
    const int kc = cb * 16 + i;
    const float4 av = *reinterpret_cast<const float4*>(lds + Lay::DZ3 + i * Lay::S3 + 4 * q);
    float bv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) bv[s] = lds[Lay::W3 + (4 * q + s) * Lay::W3S + kc];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mfma_f32_16x16x4(av.x, bv[0], acc);
    acc = mfma_f32_16x16x4(av.y, bv[1], acc);
    acc = mfma_f32_16x16x4(av.z, bv[2], acc);
    acc = mfma_f32_16x16x4(av.w, bv[3], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * q + r;
      const float v = lds[Lay::H2 + row * Lay::S2 + kc] > 0.f ? acc[r] : 0.f;
      lds[Lay::DZ2 + row * Lay::S2 + kc] = v;
      if (m0 + row < B) G2g[(int64_t)(m0 + row) * D2 + kc] = v;
    }
  }
  lds_barrier();
  FAST_STAMP(5);

  // ------------------------- layer 2 backward: dZ1 = (dZ2 W2) * (H1 > 0)
  float* G1g = ws + d.dz_off[1];
#pragma unroll
  for (int cb = wave; cb < D1 / 16; cb += 4) {
    const int kc = cb * 16 + i;
    float4 av[D2 / 16];
    float bv[D2 / 16][4];
#pragma unroll
    for (int ks = 0; ks < D2 / 16; ++ks) {
      av[ks] = *reinterpret_cast<const float4*>(lds + Lay::DZ2 + i * Lay::S2 + ks * 16 + 4 * q);
#pragma unroll
      for (int s = 0; s < 4; ++s) bv[ks][s] = lds[Lay::W2 + (ks * 16 + 4 * q + s) * Lay::W2S + kc];
    }
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < D2 / 16; ++ks) {
      a0 = mfma_f32_16x16x4(av[ks].x, bv[ks][0], a0);
      a1 = mfma_f32_16x16x4(av[ks].y, bv[ks][1], a1);
      a0 = mfma_f32_16x16x4(av[ks].z, bv[ks][2], a0);
      a1 = mfma_f32_16x16x4(av[ks].w, bv[ks][3], a1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * q + r;
      const float v = lds[Lay::H1 + row * Lay::S1 + kc] > 0.f ? a0[r] + a1[r] : 0.f;
      if (m0 + row < B) G1g[(int64_t)(m0 + row) * D1 + kc] = v;
    }
  }
  FAST_STAMP(7);
}

template <int D1, int D2, int D3>
static hipError_t launch_mlp3(const float* P, const float* slab, int nsplit, float* ws,
                              const int32_t* labels, int64_t* ctr, int64_t row0, const MlpDesc& d,
                              float* stats, int train, float inv_batch, hipStream_t s) {
  const size_t lds = Mlp3Lds<D1, D2, D3>::TOTAL * sizeof(float);
  if (lds > 160 * 1024) return hipErrorNotSupported;  // generic kernel streams W from L2
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(mlp3_rowchain_k<D1, D2, D3>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((d.batch + kRowTile - 1) / kRowTile);
  hipLaunchKernelGGL((mlp3_rowchain_k<D1, D2, D3>), grid, dim3(256), lds, s, P, slab, nsplit, ws,
                     labels, ctr, row0, d, stats, train, inv_batch);
  return hipGetLastError();
}

hipError_t mlp_read_stamps_fast(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_fast_stamps), sizeof(uint64_t) * kMaxStamps,
                             0, hipMemcpyDeviceToHost);
}
void mlp_set_stamping_fast(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fast_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

// Returns hipErrorNotSupported when no specialisation matches (caller falls
// back to the generic kernel).
hipError_t mlp_f32_rowchain_fast(const float* P, const float* slab, int nsplit, float* ws,
                                 const int32_t* labels, int64_t* ctr, int64_t row0,
                                 const MlpDesc& d, float* stats, int train, float inv_batch,
                                 hipStream_t s) {
  if (d.nlayers != 3 || nsplit < 1 || nsplit > 8) return hipErrorNotSupported;
  const int a = d.dims[1], b = d.dims[2], c = d.dims[3];
#define DSML_MLP3(A, Bd, Cd)                                                               \
  if (a == A && b == Bd && c == Cd)                                                        \
    return launch_mlp3<A, Bd, Cd>(P, slab, nsplit, ws, labels, ctr, row0, d, stats, train, \
                                  inv_batch, s);
  DSML_MLP3(128, 64, 10)
  DSML_MLP3(128, 128, 10)
  DSML_MLP3(64, 32, 10)
#undef DSML_MLP3
  return hipErrorNotSupported;
}

}  // namespace dsml
