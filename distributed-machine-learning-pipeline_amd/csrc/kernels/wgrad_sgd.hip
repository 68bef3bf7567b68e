// Weight gradient + SGD of the wide-MLP step, straight from the row-major
// activations (BASELINE config 4):
//
//   G[n][k] = alpha * sum_m Z[m][n] X[m][k]        (Z = dZ_{l+1}, X = H_l; m = batch)
//   W[n][k] -= lr * G   (fp32 master, float4 RMW)  ;  Wb[n][k] = bf16(W)   (next GEMMs' copy)
//   b[n]    -= lr * alpha * sum_m Z[m][n]          (or G / db written out for an all-reduce)
//
// The reduction runs over the batch rows, which are the STRIDED dimension of
// both stored activations: the 64 x 64 tiles of Z and X are staged row-major
// by LDS-DMA and turned into MFMA operands by ds_read_b64_tr_b16 (gfx950's
// transposing LDS read; cdna_hip_programming.md T10) — so no producer has to
// write transposed activation copies (dZ^T, H^T) any more.
//
// The kernel is bound by the fp32 master read-modify-write (+ the bf16 copy):
// every workgroup issues its W-tile loads FIRST, so that HBM round trip
// overlaps the operand staging and the MFMAs instead of following them.
// Reference hot loop replaced: the per-sample weight update of client.go:112-202.
#include "common.h"
#include "../dsml.h"

namespace dsml {
namespace {

typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));
typedef short wg_i16x4 __attribute__((ext_vector_type(4)));
typedef float wg_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t wg_u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) void* wg_gptr;
typedef __attribute__((address_space(3))) void* wg_lptr;
typedef __attribute__((address_space(3))) wg_i16x4* wg_lv4;

constexpr int kWgImg = 64 * 128;  // one 64-row x 64-column bf16 image, 128-B rows
constexpr int kWgPitch = 68;      // floats per row of the fp32 epilogue tile

__device__ __forceinline__ int wg_swz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

typedef WgLayer WgArgs;  // dsml.h: one layer's operands, targets and step

// Several layers' weight gradients in ONE launch (flattened tile grid): the
// step's last kernel updates every layer, one launch ramp and tail instead of
// one per layer.
constexpr int kWgMaxLayers = 4;
struct WgMulti {
  WgArgs l[kWgMaxLayers];
  int start[kWgMaxLayers + 1];  // first tile of each layer (prefix sums)
  int ktiles[kWgMaxLayers];
  int n;
};

// Operand fragment of the 16 x 16 x 32 MFMA: lane (i, g) gets image column
// c0 + i at rows m0 + 8g .. +7 (two transposing reads of 4 rows each).
__device__ __forceinline__ uint4 wg_frag(const char* img, int m0, int c0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = (c0 >> 3) + (p >> 1);
  const int r0 = m0 + 8 * g + q, r1 = r0 + 4;
  const wg_i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (wg_lv4)(img + r0 * 128 + 16 * (chunk ^ wg_swz(r0)) + 8 * (p & 1)));
  const wg_i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (wg_lv4)(img + r1 * 128 + 16 * (chunk ^ wg_swz(r1)) + 8 * (p & 1)));
  const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
  return make_uint4(l2.x, l2.y, h2.x, h2.y);
}

constexpr int kWgLds = 64 * kWgPitch * 4;  // two operand images (16 KiB), later the fp32 tile (17 KiB)
static_assert(kWgLds >= 2 * kWgImg, "LDS carve");
// + the bias gradient's 4 row-group partials per column ([4][64] floats)
constexpr int kWgLdsTot = kWgLds + 4 * 64 * 4;

// 1. a tile's W loads (rows rl + 16j, columns cl..cl+3), issued before anything else
__device__ __forceinline__ void wg_load_w(const WgArgs& a, int kt, int nt, float4 (&wold)[4]) {
  const int tid = threadIdx.x, rl = tid >> 4, kc = kt * 64 + 4 * (tid & 15);
  const bool kv = kc < a.K;  // K % 4 == 0: a 4-column group is whole or absent
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nr = min(nt * 64 + rl + 16 * j, a.N - 1);
    wold[j] = (kv && a.W) ? *reinterpret_cast<const float4*>(a.W + (int64_t)nr * a.ldw + kc)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// 2. Z[mb.., n0..] and X[mb.., k0..] as row-major images: 2 LDS-DMA pieces per wave each
__device__ __forceinline__ void wg_stage(const WgArgs& a, int k0, int n0, int mb, char* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* imz = lds;
  char* imx = lds + kWgImg;
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) {
    const int piece = 2 * w + pc;  // 8 rows x 128 B
    const int r = 8 * piece + (lane >> 3), p = lane & 7;
    const int m = min(mb + r, a.M - 1);
    const int zc = min(n0 + 8 * (p ^ wg_swz(r)), (int)((a.N + 7) & ~7) - 8);
    const int xc = min(k0 + 8 * (p ^ wg_swz(r)), (int)((a.K + 7) & ~7) - 8);
    __builtin_amdgcn_global_load_lds((wg_gptr)(a.Z + (int64_t)m * a.ldz + zc),
                                     (wg_lptr)(imz + piece * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((wg_gptr)(a.X + (int64_t)m * a.ldx + xc),
                                     (wg_lptr)(imx + piece * 1024), 16, 0, 0);
  }
}

// 2-4. One 64 (n) x 64 (k) tile of layer `a` (k tile kt, n tile nt) whose W
// loads are already in flight in `wold`.
__device__ __forceinline__ void wgrad_tile_body(const WgArgs& a, int kt, int nt, char* lds,
                                                const float4 (&wold)[4]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k0 = kt * 64, n0 = nt * 64;
  char* imz = lds;
  char* imx = lds + kWgImg;
  const int rl = tid >> 4, cl = 4 * (tid & 15);
  const int kc = k0 + cl;
  const bool kv = kc < a.K;

  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};
  float dbias = 0.f;
  const int wn = (w >> 1) * 32, wk = (w & 1) * 32;

  for (int mb = 0; mb < a.M; mb += 64) {
    // ---- 2. Z[mb.., n0..] and X[mb.., k0..] row-major images ----
    wg_stage(a, k0, n0, mb, lds);
    full_barrier();  // every piece landed (vmcnt(0) also retires the W loads: issued earlier)

    // ---- 3. MFMAs: wave tile 32 n x 32 k, reduction over the batch rows ----
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint4 fz[2], fx[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) fz[x] = wg_frag(imz, 32 * h, wn + 16 * x, lane);
#pragma unroll
      for (int y = 0; y < 2; ++y) fx[y] = wg_frag(imx, 32 * h, wk + 16 * y, lane);
      if (mb + 32 * h + 32 > a.M) {  // batch tail: rows >= M (clamped copies) contribute 0
        const int g = lane >> 4;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          uint32_t* e = reinterpret_cast<uint32_t*>(&fz[x]);
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (mb + 32 * h + 8 * g + t >= a.M) e[t >> 1] &= (t & 1) ? 0x0000ffffu : 0xffff0000u;
        }
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wg_bf16x8, fz[x]),
                                                              __builtin_bit_cast(wg_bf16x8, fx[y]),
                                                              acc[x][y], 0, 0, 0);
    }
    // bias gradient (k-tile 0 only): column sums of the Z image, all 256
    // threads (column tid & 63, rows 16 (tid >> 6) .. +15): a quarter of the
    // serial LDS reads of one 64-thread loop, which made these tiles the grid's
    // stragglers
    if (kt == 0) {
      const int c = tid & 63, ch = c >> 3, e = c & 7, r0 = 16 * (tid >> 6);
#pragma unroll 1  // (unrolled, the loads raise VGPRs past occupancy 5)
      for (int r = r0; r < r0 + 16 && mb + r < a.M; ++r) {
        const uint16_t v = *reinterpret_cast<const uint16_t*>(imz + r * 128 + 16 * (ch ^ wg_swz(r)) + 2 * e);
        dbias += bf16_to_f32(v);
      }
    }
    lds_barrier();  // images free for the next batch block / the epilogue tile (no DMA in flight here)
  }

  // ---- 4. epilogue: acc -> LDS tile [64 n][64 k] -> float4 RMW of W + bf16 copy ----
  float* tile = reinterpret_cast<float*>(lds);
  {
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(wn + 16 * x + 4 * g + r) * kWgPitch + wk + 16 * y + i] = acc[x][y][r] * a.alpha;
  }
  float* bsum = reinterpret_cast<float*>(lds + kWgLds);
  if (kt == 0) bsum[tid] = dbias;  // [row group][column]
  __syncthreads();
  if (kv) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nr = n0 + rl + 16 * j;
      if (nr >= a.N) continue;
      const float4 gv = *reinterpret_cast<const float4*>(tile + (rl + 16 * j) * kWgPitch + cl);
      if (a.W) {
        float4 v = wold[j];
        v.x -= a.lr * gv.x; v.y -= a.lr * gv.y; v.z -= a.lr * gv.z; v.w -= a.lr * gv.w;
        __builtin_nontemporal_store(wg_f4{v.x, v.y, v.z, v.w},
                                    reinterpret_cast<wg_f4*>(a.W + (int64_t)nr * a.ldw + kc));
        if (a.Wb) {
          const uint32_t lo = f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16);
          const uint32_t hi = f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16);
          __builtin_nontemporal_store(wg_u2{lo, hi},
                                      reinterpret_cast<wg_u2*>(a.Wb + (int64_t)nr * a.ldwb + kc));
        }
      } else if (a.G) {
        *reinterpret_cast<float4*>(a.G + (int64_t)nr * a.ldg + kc) = gv;
      }
    }
  }
  if (kt == 0 && tid < 64 && n0 + tid < a.N) {
    const float db = a.alpha * (((bsum[tid] + bsum[64 + tid]) + bsum[128 + tid]) + bsum[192 + tid]);
    if (a.bias) a.bias[n0 + tid] -= a.lr * db;
    if (a.bgrad) a.bgrad[n0 + tid] = db;
  }
}

__device__ __forceinline__ void wgrad_tile(const WgArgs& a, int kt, int nt, char* lds) {
  float4 wold[4];
  wg_load_w(a, kt, nt, wold);
  wgrad_tile_body(a, kt, nt, lds, wold);
}

__global__ __launch_bounds__(256) void wgrad_sgd_k(WgArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[kWgLdsTot];
  wgrad_tile(a, blockIdx.x, blockIdx.y, lds);
}

__global__ __launch_bounds__(256) void wgrad_multi_k(WgMulti m) {
  __shared__ __attribute__((aligned(16))) char lds[kWgLdsTot];
  const int b = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (q < m.n && b >= m.start[q]) j = q;
  const int t = b - m.start[j];
  // layers are few: select the operands with uniform branches, no dynamic
  // indexing of the kernel-argument array
  WgArgs a = m.l[0];
  int kts = m.ktiles[0];
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (j == q) { a = m.l[q]; kts = m.ktiles[q]; }
  wgrad_tile(a, t % kts, t / kts, lds);
}

// Tile selection of the flattened multi-layer grid (probe kernels below).
__device__ __forceinline__ void wg_pick(const WgMulti& m, int b, WgArgs& a, int& kt, int& nt) {
  int j = 0;
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (q < m.n && b >= m.start[q]) j = q;
  const int t = b - m.start[j];
  a = m.l[0];
  int kts = m.ktiles[0];
#pragma unroll
  for (int q = 1; q < kWgMaxLayers; ++q)
    if (j == q) { a = m.l[q]; kts = m.ktiles[q]; }
  kt = t % kts;
  nt = t / kts;
}

bool wg_valid(const WgArgs& a) {
  if (a.M < 1 || a.N < 1 || a.K < 8 || (a.K & 3) || (a.ldz & 7) || (a.ldx & 7) ||
      a.ldz < ((a.N + 7) & ~7) || a.ldx < ((a.K + 7) & ~7) || (((uintptr_t)a.Z | (uintptr_t)a.X) & 15))
    return false;
  if (a.W == nullptr && a.G == nullptr && a.bias == nullptr && a.bgrad == nullptr) return false;
  if ((a.W && (((uintptr_t)a.W & 15) || (a.ldw & 3))) || (a.Wb && (((uintptr_t)a.Wb & 7) || (a.ldwb & 3))) ||
      (a.G && (((uintptr_t)a.G & 15) || (a.ldg & 3))))
    return false;
  return true;
}

}  // namespace

hipError_t wgrad_sgd(const uint16_t* Z, int64_t ldz, const uint16_t* X, int64_t ldx, int M, int N,
                     int K, float alpha, float lr, float* W, int64_t ldw, uint16_t* Wb, int64_t ldwb,
                     float* G, int64_t ldg, float* bias, float* bgrad, hipStream_t s) {
  WgArgs a{Z, ldz, X, ldx, M, N, K, alpha, lr, W, ldw, Wb, ldwb, G, ldg, bias, bgrad};
  if (!wg_valid(a)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wgrad_sgd_k, dim3((K + 63) / 64, (N + 63) / 64), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t wgrad_sgd_multi(const WgLayer* layers, int n, hipStream_t s) {
  if (n < 1 || n > kWgMaxLayers) return hipErrorInvalidValue;
  WgMulti m{};
  m.n = n;
  int t = 0;
  for (int j = 0; j < n; ++j) {
    if (!wg_valid(layers[j])) return hipErrorInvalidValue;
    m.l[j] = layers[j];
    m.start[j] = t;
    m.ktiles[j] = (layers[j].K + 63) / 64;
    t += m.ktiles[j] * ((layers[j].N + 63) / 64);
  }
  for (int j = n; j <= kWgMaxLayers; ++j) m.start[j] = t;
  for (int j = n; j < kWgMaxLayers; ++j) { m.l[j] = layers[0]; m.ktiles[j] = m.ktiles[0]; }
  hipLaunchKernelGGL(wgrad_multi_k, dim3(t), dim3(256), 0, s, m);
  return hipGetLastError();
}

}  // namespace dsml
