// Skinny bf16 GEMMs of the wide-MLP step (BASELINE config 4, batch M = 64):
//
//   NT:  C[M x N] = A[M x K] . B[N x K]^T   forward   H_{l+1} = H_l . W_l^T
//   NN:  C[M x N] = A[M x K] . B[K x N]     dgrad     dZ_l   = dZ_{l+1} . W_l
//
// Both read the weight matrix in its ONE stored layout ([out][in], the fp32
// master's bf16 copy): the dgrad reduces over W's rows, so its B operand is
// k-strided — the LDS image of the W tile is read with ds_read_b64_tr_b16
// (gfx950's transposing LDS read, cdna_hip_programming.md T10) instead of
// keeping (and rewriting every step) a second, transposed bf16 copy of W.
//
// Decomposition (per-CU bytes, not FLOPs, bound these products): a workgroup
// owns a 64 x 64 output tile and one of S contiguous K slices; S is chosen so
// the launch has >= 256 workgroups (one per CU).  Against the 64 x 16 tiles of
// gemm_rows64_k this reads the activation block A once per 64 output columns
// instead of once per 16 (4x less L2 traffic) and streams every weight byte
// exactly once.
//
// Inside a workgroup each of the 4 waves takes every 4th 64-deep K stage and
// stages it by LDS-DMA (global_load_lds_dwordx4: full 128-B lines, no
// registers) into its own double-buffered ring: A 64 x 64 and B 64 x 64 bf16
// per stage, 16 KiB, both images XOR-swizzled on the SOURCE address so the
// fragment reads are conflict-free (ds_read_b128 rows: chunk ^ (row>>1)&7;
// tr_b16 columns: chunk ^ 2*((row>>1)&1 | ((row>>3)&1)<<1)).  No workgroup
// barrier inside the K loop: a wave waits only for its own DMA (vmcnt).
//
// The 4 waves' partial tiles are summed through LDS in fixed order; with S > 1
// every slice writes its tile write-through (sc1) and the LAST slice to arrive
// (per-tile ticket, no spinning) sums all S in slice order — deterministic —
// and applies the fused epilogue: alpha, bias, ReLU, ReLU'-mask, fp32 / bf16 /
// transposed-bf16 outputs.  Reference hot loop this replaces: the per-sample
// matrix-vector loops of client.go:112-202.
#include "common.h"
#include "../dsml.h"

namespace dsml {
namespace {

typedef __bf16 sk_bf16x8 __attribute__((ext_vector_type(8)));
typedef short sk_i16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t sk_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void* sk_gptr;
typedef __attribute__((address_space(3))) void* sk_lptr;
typedef __attribute__((address_space(3))) sk_i16x4* sk_lv4;

constexpr int kSkThreads = 256;
constexpr int kSkStage = 64;               // K depth of one staged step
constexpr int kSkImg = 64 * 128;           // bytes of one 64 x 64 bf16 image
constexpr int kSkWaveRing = 2 * 2 * kSkImg;  // 2 buffers x (A + B) = 32 KiB
constexpr int kSkLds = 4 * kSkWaveRing;    // 128 KiB
constexpr int kSkRedPitch = 68;            // floats per row of the reduction tiles

__device__ __forceinline__ f32x4 sk_mfma(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, a),
                                                  __builtin_bit_cast(sk_bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ float sk_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float sk_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
// LDS fragment reads as inline asm: the compiler cannot tell which LDS-DMA
// wrote which ring buffer, so before any ds_read it emits itself it waits for
// ALL outstanding DMA (vmcnt(0)) — including the next stage's, which collapses
// the double buffer.  Ordering is explicit instead: the per-stage vmcnt wait
// before the reads, and sk_lgkm0 after them (it also carries the read
// results, so no use can be scheduled above it).
typedef uint32_t sk_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t sk_la(const void* p) { return (uint32_t)(uintptr_t)(sk_lptr)p; }
__device__ __forceinline__ sk_u4 sk_ds128(uint32_t addr) {
  sk_u4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ sk_u2 sk_dstr(uint32_t addr) {
  sk_u2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ void sk_lgkm0(sk_u4 (&a)[4], sk_u4 (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])
               :: "memory");
}

// 16-B chunk swizzles of the two image kinds (row pitch 128 B, 8 chunks).
__device__ __forceinline__ int sk_swz_row(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int sk_swz_tr(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

struct SkArgs {
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;
  int64_t ldb;
  int M, N, K;
  int stages;  // ceil(K / 64)
  float* slabs;
  int* ctr;
  GemmEpi epi;
  int raw;  // every slice stores its partial tile to slabs[z] and exits: the CONSUMER sums
            // the S slices in slice order and applies the epilogue on load (the wide head)
};

// Profiling only (tools/skinny_stamps.py): per workgroup s_memrealtime at
// entry, K loop done, wave partials summed, split-K combine done, exit.
__device__ uint64_t g_sk_stamps[1024][5];
__device__ int g_sk_stamp_on;
#define SK_STAMP(k)                                                                        \
  do {                                                                                     \
    if (stamp && threadIdx.x == 0) g_sk_stamps[bid][(k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// One 64-deep stage of this wave's ring: A rows m0.. and the B tile (NT: rows
// n0.., NN: k-rows k0..), 8 LDS-DMA instructions each (8 rows x 128 B).
template <bool NN>
__device__ __forceinline__ void sk_issue(const SkArgs& a, char* ring, int buf, int stage, int m0,
                                         int n0, int lane) {
  const int k0 = stage * kSkStage;
  char* img_a = ring + buf * (2 * kSkImg);
  char* img_b = img_a + kSkImg;
  const int rr = lane >> 3, p = lane & 7;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 8 * j + rr;
    const int m = min(m0 + r, a.M - 1);
    const int ka = min(k0 + 8 * (p ^ sk_swz_row(r)), a.K - 8);  // tail: clamped, zeroed at use
    __builtin_amdgcn_global_load_lds((sk_gptr)(a.A + (int64_t)m * a.lda + ka),
                                     (sk_lptr)(img_a + j * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 8 * j + rr;
    const uint16_t* src;
    if (NN) {
      const int k = min(k0 + r, a.K - 1);
      const int n = min(n0 + 8 * (p ^ sk_swz_tr(r)), a.N - 8);
      src = a.B + (int64_t)k * a.ldb + n;
    } else {
      const int n = min(n0 + r, a.N - 1);
      const int k = min(k0 + 8 * (p ^ sk_swz_row(r)), a.K - 8);
      src = a.B + (int64_t)n * a.ldb + k;
    }
    __builtin_amdgcn_global_load_lds((sk_gptr)src, (sk_lptr)(img_b + j * 1024), 16, 0, 0);
  }
}

template <bool NN>
__device__ __forceinline__ void sk_compute(const SkArgs& a, const char* ring, int buf, int stage,
                                           int lane, f32x4 (&acc)[4][4]) {
  const char* img_a = ring + buf * (2 * kSkImg);
  const char* img_b = img_a + kSkImg;
  const int i = lane & 15, g = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const bool kv = stage * kSkStage + 32 * h + 8 * g < a.K;
    const uint32_t la = sk_la(img_a), lb = sk_la(img_b);
    sk_u4 fa[4], fb[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int r = 16 * x + i;
      fa[x] = sk_ds128(la + r * 128 + 16 * ((4 * h + g) ^ sk_swz_row(r)));
    }
    if (NN) {
      const int q = (lane & 15) >> 2, p = lane & 3;
      sk_u2 lo[4], hi[4];
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int c = 2 * y + (p >> 1);
        const int r0 = 32 * h + 8 * g + q, r1 = r0 + 4;
        lo[y] = sk_dstr(lb + r0 * 128 + 16 * (c ^ sk_swz_tr(r0)) + 8 * (p & 1));
        hi[y] = sk_dstr(lb + r1 * 128 + 16 * (c ^ sk_swz_tr(r1)) + 8 * (p & 1));
      }
#pragma unroll
      for (int y = 0; y < 4; ++y) fb[y] = sk_u4{lo[y].x, lo[y].y, hi[y].x, hi[y].y};
    } else {
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int r = 16 * y + i;
        fb[y] = sk_ds128(lb + r * 128 + 16 * ((4 * h + g) ^ sk_swz_row(r)));
      }
    }
    sk_lgkm0(fa, fb);
    if (!kv) {  // K tail (clamped loads): zero contribution
#pragma unroll
      for (int x = 0; x < 4; ++x) fa[x] = sk_u4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
        acc[x][y] = sk_mfma(__builtin_bit_cast(uint4, fa[x]), __builtin_bit_cast(uint4, fb[y]), acc[x][y]);
  }
}

template <bool NN>
__global__ __launch_bounds__(kSkThreads, 1) void gemm_skinny_k(SkArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sk_lds[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int n0 = blockIdx.x * 64, m0 = blockIdx.z * 64;
  const int S = gridDim.y, z = blockIdx.y;
  const int st0 = (int)(((int64_t)z * a.stages) / S), st1 = (int)(((int64_t)(z + 1) * a.stages) / S);
  const int ns = st1 - st0 > w ? (st1 - st0 - w + 3) / 4 : 0;  // stages st0 + w + 4j
  char* ring = sk_lds + w * kSkWaveRing;
  const int bid = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  const bool stamp = g_sk_stamp_on && bid < 1024;
  SK_STAMP(0);

  // epilogue operands fetched up front: their latency hides under the K loop
  const GemmEpi& e = a.epi;
  const int rl = tid >> 4, cl = 4 * (tid & 15);  // epilogue map: rows rl + 16j, columns cl..cl+3
  const int n = n0 + cl;
  const bool nv = n < a.N;  // N % 8 == 0: a 4-column group is whole or absent
  // Unpredicated: absent operands read A's first bytes instead and are dropped
  // at their use, columns past N read column 0 and are never stored.  A load
  // under a condition (even a uniform one) compiled to a branch whose copy out
  // waited vmcnt(0): one memory round trip before the first DMA (rounds 2-4,
  // ~0.5 us a launch).
  const int nc = nv ? n : 0;
  const float* bp = e.bias ? e.bias + nc : reinterpret_cast<const float*>(a.A);
  float4 bias = *reinterpret_cast<const float4*>(bp);
  const uint16_t* mp = e.mask ? e.mask + nc : a.A;
  const int64_t ldm = e.mask ? e.ldm : 0;
  uint2 mk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) mk[j] = *reinterpret_cast<const uint2*>(mp + (int64_t)min(m0 + rl + 16 * j, a.M - 1) * ldm);

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = {0.f, 0.f, 0.f, 0.f};

  if (ns > 0) sk_issue<NN>(a, ring, 0, st0 + w, m0, n0, lane);
  if (ns > 1) sk_issue<NN>(a, ring, 1, st0 + w + 4, m0, n0, lane);
  for (int j = 0; j < ns; ++j) {
    if (j + 1 < ns)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // this stage landed, the next in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sk_compute<NN>(a, ring, j & 1, st0 + w + 4 * j, lane, acc);
    if (j + 2 < ns) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of this buffer retired
      sk_issue<NN>(a, ring, j & 1, st0 + w + 4 * (j + 2), m0, n0, lane);
    }
  }
  __syncthreads();  // every wave is out of its ring: the LDS is reused below
  SK_STAMP(1);

  // ---- the 4 waves' partial tiles, summed in wave order ----
  float* red = reinterpret_cast<float*>(sk_lds);
  {
    float* mine = red + w * 64 * kSkRedPitch;
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) mine[(16 * x + 4 * g + r) * kSkRedPitch + 16 * y + i] = acc[x][y][r];
  }
  __syncthreads();
  float4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = (rl + 16 * j) * kSkRedPitch + cl;
    float4 s = *reinterpret_cast<const float4*>(red + o);
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float4 t = *reinterpret_cast<const float4*>(red + q * 64 * kSkRedPitch + o);
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    v[j] = s;
  }

  SK_STAMP(2);
  if (a.raw) {
    // consumer-combined split-K: this slice's tile into its slab, nothing else
    // (no ticket, no write-acknowledge wait, no combine: kernels/head_row.h
    // sums the slices in slice order as it loads them).  Plain stores: the
    // kernel boundary publishes them.
    const int tiles = gridDim.x * gridDim.z;
    const int tile = blockIdx.z * gridDim.x + blockIdx.x;
    float* dst = a.slabs + ((int64_t)z * tiles + tile) * 4096 + tid * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<float4*>(dst + j * 1024) = v[j];
    SK_STAMP(3);
    SK_STAMP(4);
    return;
  }
  // ---- split-K: the last slice of the tile to arrive finishes it ----
  if (S > 1) {
    const int tiles = gridDim.x * gridDim.z;
    const int tile = blockIdx.z * gridDim.x + blockIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.slabs, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sk_u4, v[j]), rs,
                                             ((z * tiles + tile) * 4096 + (j * 256 + tid) * 4) * 4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the ticket goes through the dynamic LDS (a static __shared__ would shift
    // the dynamic base off its 16-B alignment: wrong tr_b16 reads)
    int* last = reinterpret_cast<int*>(sk_lds + kSkLds - 16);
    if (tid == 0)
      *last = __hip_atomic_fetch_add(a.ctr + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
    __syncthreads();
    if (!*last) { SK_STAMP(3); SK_STAMP(4); return; }
    float4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int zz = 0; zz < S; ++zz) {  // slice order: deterministic
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float4 t = v[j];
        if (zz != z)
          t = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, ((zz * tiles + tile) * 4096 + (j * 256 + tid) * 4) * 4, 0, 16));
        s[j].x += t.x; s[j].y += t.y; s[j].z += t.z; s[j].w += t.w;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = s[j];
    if (tid == 0) __hip_atomic_store(a.ctr + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  SK_STAMP(3);
  if (!e.bias) bias = make_float4(0.f, 0.f, 0.f, 0.f);
  // ---- epilogue ----
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + rl + 16 * j;
    float4 x = v[j];
    x.x = x.x * e.alpha + bias.x; x.y = x.y * e.alpha + bias.y;
    x.z = x.z * e.alpha + bias.z; x.w = x.w * e.alpha + bias.w;
    if (e.relu) { x.x = fmaxf(x.x, 0.f); x.y = fmaxf(x.y, 0.f); x.z = fmaxf(x.z, 0.f); x.w = fmaxf(x.w, 0.f); }
    if (m < a.M && nv) {
      if (e.mask) {
        if (!(sk_lo(mk[j].x) > 0.f)) x.x = 0.f;
        if (!(sk_hi(mk[j].x) > 0.f)) x.y = 0.f;
        if (!(sk_lo(mk[j].y) > 0.f)) x.z = 0.f;
        if (!(sk_hi(mk[j].y) > 0.f)) x.w = 0.f;
      }
      if (e.of32) *reinterpret_cast<float4*>(e.of32 + (int64_t)m * e.ldo + n) = x;
      if (e.obf)
        *reinterpret_cast<uint2*>(e.obf + (int64_t)m * e.ldb + n) =
            make_uint2(f32_to_bf16(x.x) | ((uint32_t)f32_to_bf16(x.y) << 16),
                       f32_to_bf16(x.z) | ((uint32_t)f32_to_bf16(x.w) << 16));
    }
    v[j] = x;
  }
  if (!e.obfT) { SK_STAMP(4); return; }
  // transposed copy through LDS: [64 n][64 m], then 32-B runs of 16 m per thread
  // (LDS-only barriers: the row stores above need not land first)
  lds_barrier();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ml = rl + 16 * j;
    red[(cl + 0) * kSkRedPitch + ml] = v[j].x;
    red[(cl + 1) * kSkRedPitch + ml] = v[j].y;
    red[(cl + 2) * kSkRedPitch + ml] = v[j].z;
    red[(cl + 3) * kSkRedPitch + ml] = v[j].w;
  }
  lds_barrier();
  const int nl = tid >> 2, ms = 16 * (tid & 3);
  const int nn = n0 + nl, mm = m0 + ms;
  SK_STAMP(4);
  if (nn >= a.N || mm >= a.M) return;
  uint32_t q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    q[k] = f32_to_bf16(red[nl * kSkRedPitch + ms + 2 * k]) |
           ((uint32_t)f32_to_bf16(red[nl * kSkRedPitch + ms + 2 * k + 1]) << 16);
  uint16_t* dst = e.obfT + (int64_t)nn * e.ldt + mm;
  if (mm + 16 <= a.M) {
    *reinterpret_cast<uint4*>(dst) = make_uint4(q[0], q[1], q[2], q[3]);
    *reinterpret_cast<uint4*>(dst + 8) = make_uint4(q[4], q[5], q[6], q[7]);
  } else {
    for (int k = 0; k < 16 && mm + k < a.M; ++k)
      dst[k] = (uint16_t)(k & 1 ? q[k >> 1] >> 16 : q[k >> 1] & 0xffffu);
  }
}

}  // namespace

hipError_t gemm_skinny_read_stamps(uint64_t* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_sk_stamps), sizeof(uint64_t) * 1024 * 5, 0,
                             hipMemcpyDeviceToHost);
}
void gemm_skinny_set_stamping(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sk_stamp_on), &v, sizeof(int), 0, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
}

void gemm_skinny_ws(int M, int N, int K, int splits, int64_t* ws_words, int64_t* ctr_words) {
  const int S = gemm_skinny_splits(M, N, K, splits);
  const int64_t tiles = ((N + 63) / 64) * ((M + 63) / 64);
  *ws_words = S > 1 ? (int64_t)S * tiles * 4096 : 0;  // every slice's fp32 partial tile
  *ctr_words = S > 1 ? tiles : 0;                     // an arrival ticket per tile
}

int gemm_skinny_splits(int M, int N, int K, int splits) {
  const int stages = (K + kSkStage - 1) / kSkStage;
  const int tiles = ((N + 63) / 64) * ((M + 63) / 64);
  int S = splits > 0 ? splits : (256 + tiles - 1) / tiles;
  return std::max(1, std::min({S, stages, 64}));
}

hipError_t gemm_skinny(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int M, int N,
                       int K, bool nn, int splits, float* slabs, int* tile_ctr, const GemmEpi& epi,
                       hipStream_t s, bool raw_slabs) {
  if (M <= 0 || N <= 0 || K < 8 || (K & 7) || (N & 7) || (lda & 7) || (ldb & 7))
    return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return hipErrorInvalidValue;
  if (epi.sgdW || epi.bgrad || epi.bsgd) return hipErrorInvalidValue;
  if ((epi.of32 && (((uintptr_t)epi.of32 & 15) || (epi.ldo & 3))) ||
      (epi.obf && (((uintptr_t)epi.obf & 7) || (epi.ldb & 3))) ||
      (epi.obfT && (((uintptr_t)epi.obfT & 15) || (epi.ldt & 7))) ||
      (epi.mask && (((uintptr_t)epi.mask & 7) || (epi.ldm & 3))) ||
      (epi.bias && ((uintptr_t)epi.bias & 15)))
    return hipErrorInvalidValue;
  const int S = gemm_skinny_splits(M, N, K, splits);
  if (raw_slabs && (slabs == nullptr || epi.of32 || epi.obf || epi.obfT || epi.mask))
    return hipErrorInvalidValue;  // raw: slabs only, the consumer applies the epilogue
  if (!raw_slabs && S > 1 && (slabs == nullptr || tile_ctr == nullptr)) return hipErrorInvalidValue;
  SkArgs a{A, lda, B, ldb, M, N, K, (K + kSkStage - 1) / kSkStage, slabs, tile_ctr, epi, raw_slabs ? 1 : 0};
  static bool attr[2] = {false, false};
  if (!attr[nn]) {
    const void* f = nn ? reinterpret_cast<const void*>(gemm_skinny_k<true>)
                       : reinterpret_cast<const void*>(gemm_skinny_k<false>);
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kSkLds);
    if (e != hipSuccess) return e;
    attr[nn] = true;
  }
  dim3 grid((N + 63) / 64, S, (M + 63) / 64);
  if (nn)
    hipLaunchKernelGGL(gemm_skinny_k<true>, grid, dim3(kSkThreads), kSkLds, s, a);
  else
    hipLaunchKernelGGL(gemm_skinny_k<false>, grid, dim3(kSkThreads), kSkLds, s, a);
  return hipGetLastError();
}

}  // namespace dsml
