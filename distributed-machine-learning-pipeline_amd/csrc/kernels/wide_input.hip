// The wide step's input layer in ONE launch (BASELINE config 4, one replica,
// batch 64, 784-4096-...): everything the step does to W_0 plus the NEXT
// step's input-layer forward.
//
//   dZ_1  = (sum_z slab_z) * (H_1 > 0)          the last dgrad's raw split-K
//           slices (gemm_skinny raw), summed in slice order and masked here
//   W_0  -= lr * alpha * dZ_1^T X_t             split fp32 master (hi + lo words)
//   b_0  -= lr * alpha * colsum(dZ_1)
//   H_1' = relu(X_{t+1} . W_0'^T + b_0')        the next step's first layer
//
// A workgroup owns 16 rows of W_0 (16 hidden units) across the whole input
// width: the gradient, the update and the forward of those units need nothing
// from any other workgroup, so the update's output feeds the forward from
// registers -- the updated hi words ARE the forward's B fragments -- and the
// separate input-layer forward launch (gemm_rows64, 6.4 MB of W_0 re-read)
// disappears from the step, as does the dgrad's split-K combine tail (its
// consumer sums the slices).  The next step's input rows are static data, so
// computing its first layer inside this step is exactly the same work in the
// same order; the engine runs a standalone forward whenever no carried H_1 is
// valid (first step, after evaluation or a checkpoint load).
//
// Bit-exact with the separate kernels it replaces (tests/test_gpu_wide.py):
//  * dZ_1: the split-K combine's order (((0 + s_0) + s_1) + ...), alpha, mask,
//    bf16 rounding (gemm_skinny.hip);
//  * dW_0 / W_0 / b_0: the same 16x16x32 MFMA fragments (batch rows 32h + 8g ..
//    of column i) and the same update arithmetic as wgrad_sgd.hip's 64 x 64
//    tiles, the bias from the same four 16-row partial sums;
//  * H_1': gemm_rows64_k<4, 8, ABLK>'s order: wave c sums its 128-column chunk
//    in 32-column steps, the 8 chunk partials are added in chunk order.
//
// 8 waves (wave c = input chunk c = columns 128c ..), one workgroup per CU:
// N / 16 = 256 workgroups for the 4096-unit layer.
// Reference hot loop replaced: client.go:112-202 (per-sample update + forward).
#include "common.h"
#include "../dsml.h"

namespace dsml {
namespace {

typedef __bf16 wi_bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t wi_u4 __attribute__((ext_vector_type(4)));

constexpr int kWiThreads = 512;
constexpr int kWiZp = 72;    // bf16 per row of the dZ_1^T image [16 n][64 m] (+8: conflict-free b128 reads)
constexpr int kWiScP = 68;   // floats per row of a wave's gradient tile [16 n][64 k]
constexpr int kWiRedP = 17;  // floats per row of a chunk's forward partial [64 m][16 n]

#ifdef HIPDSML_MEASURE
// measurement builds: per-workgroup phase stamps (s_memrealtime, wave 0)
__device__ uint64_t g_wi_stamps[1024][8];
__device__ int g_wi_stamp_on;
__device__ int g_wi_dbg;  // drop loads: 1 the gradient's X, 2 the forward's X, 4 W, 8 the slices
#define WI_STAMP(k)                                                                       \
  do {                                                                                    \
    if (g_wi_stamp_on && threadIdx.x == 0 && blockIdx.x < 1024)                            \
      g_wi_stamps[blockIdx.x][(k)] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
#else
#define WI_STAMP(k) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ f32x4 wi_mfma(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wi_bf16x8, a),
                                                  __builtin_bit_cast(wi_bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ uint4 wi_zero() { return make_uint4(0u, 0u, 0u, 0u); }

// split fp32 master words (wgrad_sgd.hip hl_*: bits = (hi << 16) + int16 lo)
__device__ __forceinline__ float wi_join(uint32_t h, uint32_t l) {
  return __uint_as_float((h << 16) + (uint32_t)(int32_t)(int16_t)l);
}
__device__ __forceinline__ uint32_t wi_hi(float v) { return (__float_as_uint(v) + 0x8000u) >> 16; }
__device__ __forceinline__ uint32_t wi_lo(float v, uint32_t h) { return (__float_as_uint(v) - (h << 16)) & 0xffffu; }

// S: the dgrad's split-K slices (compile time: a runtime count let the compiler
// sink a slice load under a branch that waited for every earlier load)
template <int S>
__global__ __launch_bounds__(kWiThreads, 1) void wide_input_k(WideInArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t zt[16 * kWiZp];
  // the waves' gradient tiles [8][16 x 68], later (behind the bias barrier) the
  // chunks' forward partials [8][64 x 17]: the same 34 KiB
  __shared__ __attribute__((aligned(16))) float scr[8 * 16 * kWiScP];
  static_assert(16 * kWiScP == 64 * kWiRedP, "LDS alias");
  __shared__ float bs[4][16];
  __shared__ float bn[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int K = a.K;
  const int kb = a.kq * w, ke = min(K, kb + a.kq);  // this wave's input chunk (gemm_rows64's split)
  WI_STAMP(0);

  // ---- 1. every load of the workgroup up front (W from HBM first) ----
  // W_0 words of row n0 + i, columns kb + 32u + 8g .. +7 (hi, lo)
  uint4 wh[4], wl[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = kb + 32 * u + 8 * g;
    const bool v = k < ke;
    const int kc = v ? k : 0;
    if (DSML_MEASURE_KNOB(g_wi_dbg & 4)) {
      wh[u] = wl[u] = wi_zero();
      continue;
    }
    wh[u] = *reinterpret_cast<const uint4*>(a.Wh + (int64_t)(n0 + i) * a.ldwh + kc);
    wl[u] = *reinterpret_cast<const uint4*>(a.Wl + (int64_t)(n0 + i) * a.ldwl + kc);
  }
  const float bold = a.bias[n0 + (tid & 15)];
  // dZ_1 slices: thread -> (m = tid >> 3, columns n0 + 2 (tid & 7) .. +1)
  const int zm = tid >> 3, zn = 2 * (tid & 7);
  const int tile = n0 >> 6, nl = (n0 & 63) + zn;
  float2 sl[S];
#pragma unroll
  for (int z = 0; z < S; ++z)
    sl[z] = DSML_MEASURE_KNOB(g_wi_dbg & 8)
                ? make_float2(1.f, 1.f)
                : *reinterpret_cast<const float2*>(a.slabs + ((int64_t)z * a.tiles + tile) * 4096 + zm * 64 + nl);
  const uint32_t mk = *reinterpret_cast<const uint32_t*>(a.H1 + (int64_t)zm * a.ldh1 + n0 + zn);
  // every wave's W / slice / mask loads enter the CU's memory pipeline before
  // any wave's activation fragments (a plain s_barrier: no wait on the loads),
  // so dZ_1 -- the first thing every wave needs -- is not queued behind them
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  // X_t fragments of the gradient: [u][y][h] = X_t rows 32h + 8g .. +7 at column
  // kb + 32u + 16y + i.  XG is the batch's rows in fragment order ([K/16][2][16][32]:
  // column group, row half, column, row), so each load instruction reads 1 KiB
  // contiguous (8 whole lines) instead of 16 half lines.
  uint4 xf[4][2][2];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int k = kb + 32 * u + 16 * y;
      const int kg = k < ke ? k >> 4 : 0;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        xf[u][y][h] = DSML_MEASURE_KNOB(g_wi_dbg & 1)
                          ? wi_zero()
                          : *reinterpret_cast<const uint4*>(a.XG + (int64_t)kg * 1024 + 512 * h + 32 * i + 8 * g);
    }
  // X_{t+1} fragments of the forward: [u][t] = row 16t + i, columns kb + 32u + 8g .. +7;
  // XF k-blocked ([K/32][64][32]): again 1 KiB contiguous a load
  uint4 fa[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = kb + 32 * u;
    const int kc = k < ke ? k : 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      fa[u][t] = DSML_MEASURE_KNOB(g_wi_dbg & 2)
                     ? wi_zero()
                     : *reinterpret_cast<const uint4*>(a.XF + (int64_t)(kc >> 5) * 2048 + 32 * (16 * t + i) + 8 * g);
  }
  // every load above is issued before the first wait: vmcnt retires in order,
  // so any use scheduled in between would hold the rest behind W's HBM trip
  __builtin_amdgcn_sched_barrier(0);

  // ---- 2. dZ_1 = mask(sum of the slices in slice order) as bf16, transposed into LDS ----
  {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int z = 0; z < S; ++z) {
      s0 += sl[z].x;
      s1 += sl[z].y;
    }
    float x0 = s0 * a.zalpha + a.zbias, x1 = s1 * a.zalpha + a.zbias;
    if (!(__uint_as_float(mk << 16) > 0.f)) x0 = 0.f;
    if (!(__uint_as_float(mk & 0xffff0000u) > 0.f)) x1 = 0.f;
    const uint16_t b0 = f32_to_bf16(x0), b1 = f32_to_bf16(x1);
    zt[zn * kWiZp + zm] = b0;
    zt[(zn + 1) * kWiZp + zm] = b1;
    if (a.dzo) *reinterpret_cast<uint32_t*>(a.dzo + (int64_t)zm * a.lddz + n0 + zn) = b0 | ((uint32_t)b1 << 16);
  }
  WI_STAMP(1);
  __syncthreads();
  WI_STAMP(2);
  // A fragments of the gradient: dZ_1 column n0 + i at batch rows 32h + 8g .. +7
  uint4 zf[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) zf[h] = *reinterpret_cast<const uint4*>(zt + i * kWiZp + 32 * h + 8 * g);
  // bias gradient: the four 16-row partial column sums (wave 0), combined below
  if (w == 0) {
    const int c = lane & 15, q = lane >> 4;
    float d = 0.f;
#pragma unroll
    for (int r = 16 * q; r < 16 * q + 16; ++r) d += bf16_to_f32(zt[c * kWiZp + r]);
    bs[q][c] = d;
  }

  // ---- 3. two 32-column steps at a time: gradient MFMAs, ONE trip through the
  // wave's LDS tile, update, keep the new hi words (the forward's B fragments) ----
  uint4 bw[4];
  float* mysc = scr + w * 16 * kWiScP;
#pragma unroll
  for (int u2 = 0; u2 < 4; u2 += 2) {
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) {
      const int u = u2 + uu;
      if (kb + 32 * u >= ke) continue;  // wave-uniform
      f32x4 acc[2];
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        acc[y] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[y] = wi_mfma(zf[h], xf[u][y][h], acc[y]);
      }
      // [16 n][64 k] tile: lane (i, g) holds rows 4g + r, column 32 uu + 16y + i
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) mysc[(4 * g + r) * kWiScP + 32 * uu + 16 * y + i] = acc[y][r] * a.alpha;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) {
      const int u = u2 + uu;
      bw[u] = wi_zero();
      const int k = kb + 32 * u + 8 * g;
      if (kb + 32 * u >= ke || k >= ke) continue;
      const float4 g0 = *reinterpret_cast<const float4*>(mysc + i * kWiScP + 32 * uu + 8 * g);
      const float4 g1 = *reinterpret_cast<const float4*>(mysc + i * kWiScP + 32 * uu + 8 * g + 4);
      const uint32_t hw[4] = {wh[u].x, wh[u].y, wh[u].z, wh[u].w}, lw[4] = {wl[u].x, wl[u].y, wl[u].z, wl[u].w};
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = wi_join(hw[e] & 0xffffu, lw[e] & 0xffffu);
        v[2 * e + 1] = wi_join(hw[e] >> 16, lw[e] >> 16);
      }
      v[0] -= a.lr * g0.x; v[1] -= a.lr * g0.y; v[2] -= a.lr * g0.z; v[3] -= a.lr * g0.w;
      v[4] -= a.lr * g1.x; v[5] -= a.lr * g1.y; v[6] -= a.lr * g1.z; v[7] -= a.lr * g1.w;
      uint32_t nh[4], nlw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t h0 = wi_hi(v[2 * e]), h1 = wi_hi(v[2 * e + 1]);
        nh[e] = h0 | (h1 << 16);
        nlw[e] = wi_lo(v[2 * e], h0) | (wi_lo(v[2 * e + 1], h1) << 16);
      }
      __builtin_nontemporal_store(wi_u4{nh[0], nh[1], nh[2], nh[3]},
                                  reinterpret_cast<wi_u4*>(a.Wb + (int64_t)(n0 + i) * a.ldwb + k));
      __builtin_nontemporal_store(wi_u4{nlw[0], nlw[1], nlw[2], nlw[3]},
                                  reinterpret_cast<wi_u4*>(a.Wl + (int64_t)(n0 + i) * a.ldwl + k));
      bw[u] = make_uint4(nh[0], nh[1], nh[2], nh[3]);
    }
    __builtin_amdgcn_wave_barrier();  // the tile's reads are done before the next pair rewrites it
  }
  WI_STAMP(3);
  __syncthreads();  // bs complete
  WI_STAMP(4);
  if (tid < 16) {
    const float db = a.alpha * (((bs[0][tid] + bs[1][tid]) + bs[2][tid]) + bs[3][tid]);
    float b = bold;
    b -= a.lr * db;
    a.bias[n0 + tid] = b;
    bn[tid] = b;
  }

  // ---- 4. the next step's forward with the updated rows: chunk w, 32-column steps ----
  f32x4 af[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) af[t] = {0.f, 0.f, 0.f, 0.f};
  if (kb < ke) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool kv = kb + 32 * u + 8 * g < ke;
      const uint4 b = kv ? bw[u] : wi_zero();
#pragma unroll
      for (int t = 0; t < 4; ++t) af[t] = wi_mfma(kv ? fa[u][t] : wi_zero(), b, af[t]);
    }
  }
  WI_STAMP(5);
  float* mine = scr + w * 64 * kWiRedP;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) mine[(16 * t + 4 * g + r) * kWiRedP + i] = af[t][r];
  __syncthreads();
  WI_STAMP(6);
  // chunk partials in chunk order, alpha, the updated bias, ReLU -> bf16
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = tid + kWiThreads * j;
    const int m = e >> 4, n = e & 15;
    const int o = m * kWiRedP + n;
    float x = scr[o];
#pragma unroll
    for (int q = 1; q < 8; ++q) x += scr[q * 64 * kWiRedP + o];
    x *= a.falpha;
    x += bn[n];
    x = fmaxf(x, 0.f);
    a.Hn[(int64_t)m * a.ldhn + n0 + n] = f32_to_bf16(x);
  }
  WI_STAMP(7);
}

}  // namespace

#ifdef HIPDSML_MEASURE
hipError_t wide_input_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wi_stamps), sizeof(uint64_t) * 1024 * 8, 0,
                             hipMemcpyDeviceToHost);
}
void wide_input_set_dbg(int bits) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wi_dbg), &bits, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
void wide_input_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wi_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
#endif

hipError_t wide_input_check(const WideInArgs& a) {
  // shapes the kernels' maps assume (checked here, before any launch)
  if (a.M != 64 || a.N <= 0 || (a.N & 15) || a.K <= 0 || (a.K & 15) || a.K > 8 * 128) return hipErrorInvalidValue;
  if (a.kq != (((a.K + 7) / 8 + 31) / 32) * 32) return hipErrorInvalidValue;  // gemm_rows64_k's 8-wave split
  if ((a.S != 1 && a.S != 2 && a.S != 4 && a.S != 8) || a.tiles != (a.N + 63) / 64) return hipErrorInvalidValue;
  if (!a.slabs || !a.H1 || !a.XG || !a.XF || !a.Wh || !a.Wl || !a.Wb || !a.bias || !a.Hn)
    return hipErrorInvalidValue;
  if ((a.ldwh & 7) || (a.ldwl & 7) || (a.ldwb & 7) || (a.ldh1 & 3) || (a.dzo && (a.lddz & 3)))
    return hipErrorInvalidValue;
  const uintptr_t al = (uintptr_t)a.Wh | (uintptr_t)a.Wl | (uintptr_t)a.Wb | (uintptr_t)a.XG | (uintptr_t)a.XF;
  if ((al & 15) || ((uintptr_t)a.slabs & 15) || ((uintptr_t)a.H1 & 7) || ((uintptr_t)a.dzo & 7))
    return hipErrorInvalidValue;
  return hipSuccess;
}

hipError_t wide_input_step(const WideInArgs& a, hipStream_t s) {
  if (wide_input_check(a) != hipSuccess) return hipErrorInvalidValue;
  // shapes the kernel's maps assume (checked here, before any launch)
  if (a.M != 64 || a.N <= 0 || (a.N & 15) || a.K <= 0 || (a.K & 15) || a.K > 8 * 128) return hipErrorInvalidValue;
  if (a.kq != (((a.K + 7) / 8 + 31) / 32) * 32) return hipErrorInvalidValue;  // gemm_rows64_k's 8-wave split
  if (a.S < 1 || a.S > 8 || a.tiles != (a.N + 63) / 64) return hipErrorInvalidValue;
  if (!a.slabs || !a.H1 || !a.XG || !a.XF || !a.Wh || !a.Wl || !a.Wb || !a.bias || !a.Hn)
    return hipErrorInvalidValue;
  if ((a.ldwh & 7) || (a.ldwl & 7) || (a.ldwb & 7) || (a.ldh1 & 1) || (a.dzo && (a.lddz & 1)))
    return hipErrorInvalidValue;
  const uintptr_t al = (uintptr_t)a.Wh | (uintptr_t)a.Wl | (uintptr_t)a.Wb | (uintptr_t)a.XG | (uintptr_t)a.XF;
  if ((al & 15) || ((uintptr_t)a.slabs & 7) || ((uintptr_t)a.H1 & 3) || ((uintptr_t)a.dzo & 3))
    return hipErrorInvalidValue;
  switch (a.S) {
    case 1: hipLaunchKernelGGL(wide_input_k<1>, dim3(a.N / 16), dim3(kWiThreads), 0, s, a); break;
    case 2: hipLaunchKernelGGL(wide_input_k<2>, dim3(a.N / 16), dim3(kWiThreads), 0, s, a); break;
    case 4: hipLaunchKernelGGL(wide_input_k<4>, dim3(a.N / 16), dim3(kWiThreads), 0, s, a); break;
    case 8: hipLaunchKernelGGL(wide_input_k<8>, dim3(a.N / 16), dim3(kWiThreads), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dsml
