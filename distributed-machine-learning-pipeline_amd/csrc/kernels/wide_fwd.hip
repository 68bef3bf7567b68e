// Fused forward of the wide MLP's two hidden layers (BASELINE config 4,
// 784-4096-4096-10 bf16, batch M <= 64) in ONE launch of 256 workgroups:
//
//   H1 = relu(X . W1^T + b1)     layer 1: a 64 x 16 tile per workgroup, full K
//   H2 = relu(H1 . W2^T + b2)    layer 2: a 64 x 64 tile x one of 4 K slices
//
// Why one launch (profiles/r4_wide_kernels.csv): the separate layer-1 kernel
// (gemm_rows64_k, 7.7 us) and layer-2 kernel (gemm_skinny_k, 14.5 us) each pay
// a launch ramp, a load latency before the first MFMA and a reduce tail, and
// the layer-2 kernel cannot fetch a byte of W2 before layer 1 has finished.
// W2 does not depend on layer 1: here every workgroup streams its whole
// 128 KiB W2 slice (64 rows x 1024 k) into LDS by DMA while the slice's 64
// layer-1 tiles are published, then waits for them.
//
// STATUS: correct (bit-exact, tests/test_gpu_wide.py) but NOT faster, so
// opt-in (engine/wide.py fused_fwd, HIPDSML_WIDE_FUSED_FWD=1): 25.0 us against
// 22.2 us for the two launches (profiles/r4_wide_fused_fwd_ab.json).  Layer 1
// needs ~5.5 us to land its operands and publishes at ~7.4 us; the 32 MB W2
// stream then takes ~9.5 us.  Started at entry instead (testing switch
// wide_fwd2_set_early_dma), the stream delays the layer-1 publish to ~11.5 us:
// the tile's write-through stores and LDS writes queue behind the DMA.
//
// Workgroup b: layer-1 columns 16b..16b+15; layer-2 tile t = b % 64, slice
// z = b / 64 (H1 columns 1024z..1024z+1023 = the layer-1 tiles of workgroups
// 64z..64z+63, so a slice depends on its own 64 workgroups only).  All 256
// workgroups must be co-resident (one per CU, 156 KiB of LDS each): the host
// checks the CU count, and every wait is bounded (error word, no hang).
//
// Hand-off (MI355X_MICROARCH.md "Valid forms", first row): ONE wave stores the
// tile with 16-B sc1 (write-through) stores, drains them (s_waitcnt vmcnt(0))
// and one lane stores the flag sc1; consumers poll the flags with sc1 loads and
// read the tiles with sc1 buffer loads.  Flags carry a launch epoch kept on the
// device (graph-replay safe): every workgroup reads it at entry, the last
// workgroup to finish advances it.  Wave 0 issues no LDS-DMA, so its drain
// waits for its own stores only (vmcnt retires in issue order: a wave with the
// W2 DMA in flight could not drain before the DMA landed).
//
// Bit-exact with the two-kernel path: layer 1 repeats gemm_rows64_k<4, 8>'s
// arithmetic (each wave plays two of its eight K-waves, partials summed in the
// same order), layer 2 repeats gemm_skinny_k<false>'s (stage order per wave,
// wave-order and slice-order sums, same epilogue).  Reference hot loop:
// client.go:112-202 (per-sample matrix-vector forward).
#include "common.h"
#include "../dsml.h"

namespace dsml {
namespace {

typedef __bf16 wf_bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t wf_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void* wf_gptr;
typedef __attribute__((address_space(3))) void* wf_lptr;
typedef __attribute__((address_space(1))) int wf_gi32;

constexpr int kWfThreads = 256;
constexpr int kWfN = 4096;                  // N1 = N2 = K2
constexpr int kWfBlocks = kWfN / 16;        // 256: one layer-1 tile each
constexpr int kWfS = 4;                     // layer-2 K slices (gemm_skinny_splits(64, 4096, 4096))
constexpr int kWfTiles = kWfN / 64;         // 64 layer-2 tiles
constexpr int kWfStages = kWfN / kWfS / 64; // 16 stages of 64 k per slice
constexpr int kWfImg = 64 * 128;            // one 64 x 64 bf16 image
constexpr int kWfB2 = kWfStages * kWfImg;   // 128 KiB: the W2 slice
constexpr int kWfP1 = 7 * 64 * 16 * 4;      // 28 KiB: layer-1 partial tiles
constexpr int kWfLds = kWfB2 + kWfP1 + 16;
constexpr int kWfRedPitch = 68;
// sync words: [0, 256) tile flags, then epoch, done ticket, error
constexpr int kWfEpoch = kWfBlocks, kWfDone = kWfBlocks + 1, kWfErr = kWfBlocks + 2;

struct WfArgs {
  const uint16_t* X;
  int64_t ldx;
  const uint16_t* W1;
  int64_t ldw1;
  const float* b1;
  uint16_t* H1;
  int64_t ldh1;
  const uint16_t* W2;
  int64_t ldw2;
  const float* b2;
  uint16_t* H2;
  int64_t ldh2;
  int M, K1;
  float* slabs;
  int* ctr;
  int* sync;
  uint32_t timeout;  // s_memrealtime ticks (100 MHz) per wait
};

__device__ __forceinline__ f32x4 wf_mfma(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wf_bf16x8, a),
                                                  __builtin_bit_cast(wf_bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ uint4 wf_zero() { return make_uint4(0u, 0u, 0u, 0u); }
__device__ __forceinline__ uint32_t wf_la(const void* p) { return (uint32_t)(uintptr_t)(wf_lptr)p; }
__device__ __forceinline__ int wf_swz(int r) { return (r >> 1) & 7; }  // = gemm_skinny's row swizzle
// LDS accesses while LDS-DMA is in flight are inline asm: the compiler would
// put s_waitcnt vmcnt(0) (every outstanding DMA) in front of any it emits.
__device__ __forceinline__ void wf_dsw(uint32_t addr, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ wf_u4 wf_ds128(uint32_t addr) {
  wf_u4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ void wf_lgkm0(wf_u4 (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])::"memory");
}
// layer-1 partial slot s, row m, column c (16 floats a row, 16-B chunks XOR-swizzled by row)
__device__ __forceinline__ int wf_p1(int s, int m, int c) {
  return kWfB2 + 4 * ((s * 64 + m) * 16 + 4 * ((c >> 2) ^ ((m >> 2) & 3)) + (c & 3));
}

// Profiling only: per workgroup s_memrealtime (wave 0) at entry, layer-1
// tile published, slice ready, A loaded + W2 landed, MFMAs done, exit, layer-1
// operands landed, layer-1 partials in LDS.
__device__ uint64_t g_wf_stamps[kWfBlocks][8];
__device__ int g_wf_stamp_on;
#define WF_STAMP(k)                                                                          \
  do {                                                                                       \
    if (stamp && threadIdx.x == 0) g_wf_stamps[bid][(k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

__device__ int g_wf_early_dma;  // testing: 1 = stream W2 from the start

// The W2 slice of layer-2 tile t, K slice z, by LDS-DMA: waves 1..3, stage s by
// wave 1 + s % 3 (wave 0 stays free of DMA: its drains and polls then wait
// for its own traffic only).
__device__ __forceinline__ void wf_issue_w2(const WfArgs& a, char* wf_lds, int t, int z, int w, int lane) {
  if (w > 0) {
    const int rr = lane >> 3, p = lane & 7;
    for (int s = w - 1; s < kWfStages; s += 3) {
      const int k0 = 1024 * z + 64 * s;
      char* img = wf_lds + s * kWfImg;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = 8 * j + rr;
        const uint16_t* src = a.W2 + (int64_t)(64 * t + r) * a.ldw2 + k0 + 8 * (p ^ wf_swz(r));
        __builtin_amdgcn_global_load_lds((wf_gptr)src, (wf_lptr)(img + j * 1024), 16, 0, 0);
      }
    }
  }
}

__global__ __launch_bounds__(kWfThreads, 1) void wide_fwd2_k(WfArgs a) {
  extern __shared__ __attribute__((aligned(16))) char wf_lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int bid = blockIdx.x;
  const int t = bid % kWfTiles, z = bid / kWfTiles;
  const int n1 = 16 * bid;
  const int M = a.M, K = a.K1;
  int* sync = a.sync;
  const bool stamp = g_wf_stamp_on != 0;
  WF_STAMP(0);
  const int ep = __hip_atomic_load((wf_gi32*)(sync + kWfEpoch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;

  // ---- layer 1: operands of the two rows64 K-waves this wave plays ----
  const int kq = ((K + 7) / 8 + 31) / 32 * 32;  // <= 128 (K <= 1024): one U = 4 round each
  int ra[4];
  bool va[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    ra[x] = 16 * x + i;
    va[x] = ra[x] < M;
    ra[x] = va[x] ? ra[x] : M - 1;
  }
  const uint16_t* pb = a.W1 + (int64_t)(n1 + i) * a.ldw1;
  int kb[2], ke[2];
  uint4 fa[2][4][4], fb[2][4];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    kb[v] = (2 * w + v) * kq;
    ke[v] = min(K, kb[v] + kq);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kk = kb[v] + 32 * u + 8 * g;
      const int kc = kk < ke[v] ? kk : (kb[v] < K ? kb[v] : 0);  // never past the row
      fb[v][u] = *reinterpret_cast<const uint4*>(pb + kc);
#pragma unroll
      for (int x = 0; x < 4; ++x) fa[v][u][x] = *reinterpret_cast<const uint4*>(a.X + (int64_t)ra[x] * a.ldx + kc);
    }
  }
  // epilogue operands: layer-1 bias (wave 0's 16 columns), layer-2 bias
  const int rl = tid >> 4, cl = 4 * (tid & 15);
  const float4 bias2 = *reinterpret_cast<const float4*>(a.b2 + 64 * t + cl);
  float bias1[16];
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const float4 q = *reinterpret_cast<const float4*>(a.b1 + n1 + c);
    bias1[c] = q.x; bias1[c + 1] = q.y; bias1[c + 2] = q.z; bias1[c + 3] = q.w;
  }
  f32x4 acc1[2][4];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
#pragma unroll
    for (int x = 0; x < 4; ++x) acc1[v][x] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool kv = kb[v] + 32 * u + 8 * g < ke[v];
      const uint4 b = kv ? fb[v][u] : wf_zero();
#pragma unroll
      for (int x = 0; x < 4; ++x) acc1[v][x] = wf_mfma((kv && va[x]) ? fa[v][u][x] : wf_zero(), b, acc1[v][x]);
    }
  }
  WF_STAMP(6);
  const bool early = g_wf_early_dma != 0;
  if (early) wf_issue_w2(a, wf_lds, t, z, w, lane);
  // partials -> LDS: slot 0 = K-waves 0 + 1 (wave 0 folds them: the same
  // left-to-right sum), slot 2w - 1 + v = K-wave 2w + v for w >= 1
  const uint32_t base = wf_la(wf_lds);
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    if (w == 0 && v == 1) break;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float val = w == 0 ? acc1[0][x][r] + acc1[1][x][r] : acc1[v][x][r];
        wf_dsw(base + wf_p1(w == 0 ? 0 : 2 * w - 1 + v, 16 * x + 4 * g + r, i), val);
      }
  }
  lds_barrier();  // the partial tiles are in LDS
  WF_STAMP(7);

  // ---- wave 0: sum, bias, ReLU, publish the H1 tile, raise the flag ----
  if (w == 0) {
    const int m = lane;
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = 0.f;
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const float4 q = *reinterpret_cast<const float4*>(wf_lds + wf_p1(s, m, 4 * cc) - 0);
        if (s == 0) {
          x[4 * cc] = q.x; x[4 * cc + 1] = q.y; x[4 * cc + 2] = q.z; x[4 * cc + 3] = q.w;
        } else {
          x[4 * cc] += q.x; x[4 * cc + 1] += q.y; x[4 * cc + 2] += q.z; x[4 * cc + 3] += q.w;
        }
      }
    if (m < M) {
      uint32_t h[8];
#pragma unroll
      for (int c = 0; c < 16; c += 2) {
        const float lo = fmaxf(x[c] + bias1[c], 0.f), hi = fmaxf(x[c + 1] + bias1[c + 1], 0.f);
        h[c / 2] = f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
      }
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.H1, (short)0, 0x7fffffff, 0x00020000);
      const int off = (int)(((int64_t)m * a.ldh1 + n1) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(wf_u4{h[0], h[1], h[2], h[3]}, rs, off, 0, 16);       // sc1
      __builtin_amdgcn_raw_buffer_store_b128(wf_u4{h[4], h[5], h[6], h[7]}, rs, off + 16, 0, 16);  // sc1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile acknowledged before its flag
    if (lane == 0) __hip_atomic_store((wf_gi32*)(sync + bid), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    WF_STAMP(1);
  }

  lds_barrier();  // wave 0's tile is acknowledged: the W2 stream may start
  // ---- waves 1..3: the W2 slice by LDS-DMA (stage s by wave 1 + s % 3) ----
  // Issued once the layer-1 tile is published: streamed any earlier, the
  // 32 MB of W2 (all workgroups) queue ahead of the tile's write-through
  // stores and their acknowledgement, and the publish slips from ~4 to ~11 us
  // (measured, tools/wide_fwd_stamps.py).
  if (!early) wf_issue_w2(a, wf_lds, t, z, w, lane);
  // ---- wave 0 waits for the 64 layer-1 tiles of slice z; the others join
  // it at the barrier (a poll in a wave with DMA in flight would retire only
  // behind that DMA: vmcnt counts in issue order) ----
  if (w == 0) {
    const wf_gi32* f = (const wf_gi32*)(sync + 64 * z + lane);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_ballot_w64(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ep)) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
        if (lane == 0) __hip_atomic_fetch_or((wf_gi32*)(sync + kWfErr), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    WF_STAMP(2);
  }
  asm volatile("s_barrier" ::: "memory");  // no waits: waves 1..3 keep their DMA in flight

  // ---- layer 2: this wave's A operand (stages w + 4j of the slice), sc1 loads ----
  uint4 fa2[4][2][4];
  {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.H1, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const int m = min(16 * x + i, M - 1);
          const int k = 1024 * z + 64 * (w + 4 * j) + 32 * h + 8 * g;
          fa2[j][h][x] = __builtin_bit_cast(
              uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((int64_t)m * a.ldh1 + k) * 2), 0, 16));
        }
  }
  full_barrier();  // every wave's DMA and A loads landed: the W2 images are readable
  WF_STAMP(3);
  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lb = base + (w + 4 * j) * kWfImg;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      wf_u4 fb2[4];
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int r = 16 * y + i;
        fb2[y] = wf_ds128(lb + r * 128 + 16 * ((4 * h + g) ^ wf_swz(r)));
      }
      wf_lgkm0(fb2);
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = wf_mfma(fa2[j][h][x], __builtin_bit_cast(uint4, fb2[y]), acc[x][y]);
    }
  }
  __syncthreads();  // every wave is out of the W2 images: the LDS is reused below
  WF_STAMP(4);

  // ---- the 4 waves' partial tiles, summed in wave order (gemm_skinny_k) ----
  float* red = reinterpret_cast<float*>(wf_lds);
  {
    float* mine = red + w * 64 * kWfRedPitch;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) mine[(16 * x + 4 * g + r) * kWfRedPitch + 16 * y + i] = acc[x][y][r];
  }
  __syncthreads();
  float4 v4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = (rl + 16 * j) * kWfRedPitch + cl;
    float4 s = *reinterpret_cast<const float4*>(red + o);
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float4 u = *reinterpret_cast<const float4*>(red + q * 64 * kWfRedPitch + o);
      s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
    }
    v4[j] = s;
  }
  // ---- split-K: the last slice of the tile to arrive finishes it ----
  const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(a.slabs, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(wf_u4, v4[j]), rsl,
                                           ((z * kWfTiles + t) * 4096 + (j * 256 + tid) * 4) * 4, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* last = reinterpret_cast<int*>(wf_lds + kWfLds - 16);
  if (tid == 0) {
    *last = __hip_atomic_fetch_add(a.ctr + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kWfS - 1;
    // the launch's done ticket: the last workgroup advances the flag epoch
    if (__hip_atomic_fetch_add(sync + kWfDone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kWfBlocks - 1) {
      __hip_atomic_store(sync + kWfDone, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sync + kWfEpoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!*last) {
    WF_STAMP(5);
    return;
  }
  {
    float4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int zz = 0; zz < kWfS; ++zz) {  // slice order: deterministic
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float4 u = v4[j];
        if (zz != z)
          u = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsl, ((zz * kWfTiles + t) * 4096 + (j * 256 + tid) * 4) * 4, 0, 16));
        s[j].x += u.x; s[j].y += u.y; s[j].z += u.z; s[j].w += u.w;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v4[j] = s[j];
    if (tid == 0) __hip_atomic_store(a.ctr + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ---- epilogue: bias, ReLU, bf16 H2 ----
  const int n = 64 * t + cl;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = rl + 16 * j;
    float4 x = v4[j];
    x.x = fmaxf(x.x * 1.0f + bias2.x, 0.f); x.y = fmaxf(x.y * 1.0f + bias2.y, 0.f);
    x.z = fmaxf(x.z * 1.0f + bias2.z, 0.f); x.w = fmaxf(x.w * 1.0f + bias2.w, 0.f);
    if (m < M)
      *reinterpret_cast<uint2*>(a.H2 + (int64_t)m * a.ldh2 + n) =
          make_uint2(f32_to_bf16(x.x) | ((uint32_t)f32_to_bf16(x.y) << 16),
                     f32_to_bf16(x.z) | ((uint32_t)f32_to_bf16(x.w) << 16));
  }
  WF_STAMP(5);
}

}  // namespace

int wide_fwd2_lds_bytes() { return kWfLds; }

hipError_t wide_fwd2_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wf_stamps), sizeof(uint64_t) * kWfBlocks * 8, 0,
                             hipMemcpyDeviceToHost);
}
void wide_fwd2_set_early_dma(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wf_early_dma), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}
void wide_fwd2_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wf_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

// Can this device hold the whole grid at once (one workgroup per CU)?
bool wide_fwd2_supported(int device) {
  int cus = 0, lds = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess)
    return false;
  return cus >= kWfBlocks && lds >= kWfLds;
}

hipError_t wide_fwd2(const uint16_t* X, int64_t ldx, const uint16_t* W1, int64_t ldw1, const float* b1,
                     uint16_t* H1, int64_t ldh1, const uint16_t* W2, int64_t ldw2, const float* b2,
                     uint16_t* H2, int64_t ldh2, int M, int K1, float* slabs, int* tile_ctr, int* sync,
                     hipStream_t s) {
  if (M < 1 || M > 64 || K1 < 512 || K1 > 1024 || (K1 & 7)) return hipErrorInvalidValue;
  if ((ldx & 7) || (ldw1 & 7) || (ldh1 & 7) || (ldw2 & 7) || (ldh2 & 3) || ldw1 < K1 || ldx < K1 ||
      ldh1 < kWfN || ldw2 < kWfN || ldh2 < kWfN)
    return hipErrorInvalidValue;
  if (((uintptr_t)X | (uintptr_t)W1 | (uintptr_t)H1 | (uintptr_t)W2 | (uintptr_t)b1 | (uintptr_t)b2) & 15)
    return hipErrorInvalidValue;
  if (((uintptr_t)H2 & 7) || !slabs || !tile_ctr || !sync) return hipErrorInvalidValue;
  // buffer-resource offsets are 32-bit
  if ((int64_t)M * ldh1 * 2 > 0x7fffffffLL) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(wide_fwd2_k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kWfLds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  WfArgs a{X, ldx, W1, ldw1, b1, H1, ldh1, W2, ldw2, b2, H2, ldh2, M, K1, slabs, tile_ctr, sync,
           10000000u /* 100 ms */};
  hipLaunchKernelGGL(wide_fwd2_k, dim3(kWfBlocks), dim3(kWfThreads), kWfLds, s, a);
  return hipGetLastError();
}

}  // namespace dsml
