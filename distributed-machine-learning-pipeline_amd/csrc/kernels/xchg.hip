// One-shot all-reduce over xGMI peer memory (standalone buffers).
//
// The same protocol as the exchange fused into the MLP weight-gradient kernel
// (mlp_f32.hip, XCHG path), for arbitrary fp32 buffers: every rank copies its
// input into its own IPC-shared, uncached exchange buffer (parity = call & 1),
// raises one flag per workgroup chunk, waits for the same chunk's flag of every
// peer, reads the peers' chunks directly over xGMI and writes the rank-ordered
// sum.  One kernel, one synchronisation round, N-1 concurrent links: the
// latency-optimal shape for the small (<= a few MiB) messages of MLP training,
// where a ring pays 2(N-1) dependent hops (reference ring: 2(n-1) gRPC rounds,
// gpu_coordinator_server.go:338-356).
#include "common.h"
#include "../dsml.h"

namespace dsml {

namespace {

typedef __attribute__((address_space(1))) uint64_t gu64x;
// System-coherent 16 B accesses as two 8 B relaxed atomics (global_*_dwordx2
// sc0 sc1): compiler-visible, so the usual waitcnt tracking applies.
__device__ __forceinline__ float4 ld_sys4(const float* p) {
  const gu64x* q = (const gu64x*)p;
  const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)),
                     __uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32)));
}
__device__ __forceinline__ void st_sys4(float* p, float4 v) {
  gu64x* q = (gu64x*)p;
  const uint64_t a = (uint64_t)__float_as_uint(v.x) | ((uint64_t)__float_as_uint(v.y) << 32);
  const uint64_t b = (uint64_t)__float_as_uint(v.z) | ((uint64_t)__float_as_uint(v.w) << 32);
  __hip_atomic_store(q, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(q + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_flag(uint64_t* p, uint64_t v) {
  __hip_atomic_store((__attribute__((address_space(1))) uint64_t*)p, v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kXThreads = 256;

// Each thread owns U float4s of the workgroup's chunk (strided by the block).
template <int U>
__global__ __launch_bounds__(kXThreads) void xchg_allreduce_k(const float* __restrict__ in,
                                                              float* __restrict__ out, int64_t n,
                                                              XchgArgs xa, uint64_t seq) {
  const int64_t chunk = (int64_t)kXThreads * 4 * U;
  const int64_t base = (int64_t)blockIdx.x * chunk;
  const int64_t poff = (int64_t)(seq & 1) * xa.half;
  const XchgTab* __restrict__ tab = xa.tab;
  float* mine = tab->buf[xa.rank] + poff;
  float4 own[U];
  // n is a multiple of 4 (checked on the host): whole float4s only.
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + ((int64_t)u * kXThreads + threadIdx.x) * 4;
    own[u] = i < n ? *reinterpret_cast<const float4*>(in + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + ((int64_t)u * kXThreads + threadIdx.x) * 4;
    if (i < n) st_sys4(mine + i, own[u]);
  }
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) st_flag(tab->flags[xa.rank] + blockIdx.x, seq);
  if (threadIdx.x < xa.nranks && threadIdx.x != xa.rank)
    (void)poll_flag_ge<1>(tab->flags[threadIdx.x] + blockIdx.x, seq, xa.err, xa.timeout_ticks);
  __syncthreads();
  float4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  // Rank-ordered sum (identical on every rank).
  for (int p = 0; p < xa.nranks; ++p) {
    float4 v[U];
    if (p == xa.rank) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = own[u];
    } else {
      const float* pb = tab->buf[p] + poff;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + ((int64_t)u * kXThreads + threadIdx.x) * 4;
        v[u] = ld_sys4(pb + (i < n ? i : 0));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[u].x += v[u].x;
      acc[u].y += v[u].y;
      acc[u].z += v[u].z;
      acc[u].w += v[u].w;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + ((int64_t)u * kXThreads + threadIdx.x) * 4;
    if (i < n) *reinterpret_cast<float4*>(out + i) = acc[u];
  }
}


// Two-shot variant: reduce-scatter then all-gather over the same peer memory.
// Rank r owns chunk r (ceil(n / N) floats, float4-aligned).  Phase 1: every
// rank publishes its whole input (local stores) and raises flag1; the owner of
// each chunk reads that chunk from every peer, sums in rank order, publishes
// the reduced chunk and raises flag2.  Phase 2: every rank reads each peer's
// reduced chunk.  Per link 2 n / N bytes instead of the one-shot's n — the
// form for larger messages and wider groups (1 MiB at N = 8: 256 KB per link
// instead of 1 MiB).  Blocks own the same float4 slice of every chunk, so all
// hand-offs stay inside a block (no cross-block dependency on a GPU).
// Exchange buffer (per parity half): [0, n) input copy, [n, n + cs) reduced chunk;
// flags: [0, fo) phase 1, [fo, 2 fo) phase 2.
template <int U>
__global__ __launch_bounds__(kXThreads) void xchg_allreduce2_k(const float* __restrict__ in,
                                                               float* __restrict__ out, int64_t n,
                                                               int64_t cs, XchgArgs xa, uint64_t seq,
                                                               int fo) {
  const int N = xa.nranks, me = xa.rank;
  const int64_t poff = (int64_t)(seq & 1) * xa.half;
  const XchgTab* __restrict__ tab = xa.tab;
  float* mine = tab->buf[me] + poff;
  const int64_t slice = (int64_t)blockIdx.x * kXThreads * 4 * U;  // float offset within a chunk
  auto chunk_len = [&](int c) -> int64_t {
    const int64_t b = (int64_t)c * cs;
    return b >= n ? 0 : (n - b < cs ? n - b : cs);
  };
  auto wait_flags = [&](int base) {
    if (threadIdx.x < N && threadIdx.x != me)
      (void)poll_flag_ge<1>(tab->flags[threadIdx.x] + base + blockIdx.x, seq, xa.err,
                            xa.timeout_ticks);
    __syncthreads();
  };
  // ---- phase 1a: publish this block's slice of every chunk ----
  float4 own[U];
  for (int c = 0; c < N; ++c) {
    const int64_t len = chunk_len(c), cb = (int64_t)c * cs;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = slice + ((int64_t)u * kXThreads + threadIdx.x) * 4;
      if (i < len) {
        const float4 v = *reinterpret_cast<const float4*>(in + cb + i);
        st_sys4(mine + cb + i, v);
        if (c == me) own[u] = v;
      }
    }
  }
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) st_flag(tab->flags[me] + blockIdx.x, seq);
  wait_flags(0);
  // ---- phase 1b: reduce my chunk's slice in rank order, publish it ----
  const int64_t mlen = chunk_len(me), mcb = (int64_t)me * cs;
  float4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int p = 0; p < N; ++p) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = slice + ((int64_t)u * kXThreads + threadIdx.x) * 4;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < mlen) v[u] = p == me ? own[u] : ld_sys4(tab->buf[p] + poff + mcb + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = slice + ((int64_t)u * kXThreads + threadIdx.x) * 4;
    if (i < mlen) {
      st_sys4(mine + n + i, acc[u]);
      *reinterpret_cast<float4*>(out + mcb + i) = acc[u];
    }
  }
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) st_flag(tab->flags[me] + fo + blockIdx.x, seq);
  wait_flags(fo);
  // ---- phase 2: gather every peer's reduced slice ----
  for (int p = 0; p < N; ++p) {
    if (p == me) continue;
    const int64_t len = chunk_len(p), cb = (int64_t)p * cs;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = slice + ((int64_t)u * kXThreads + threadIdx.x) * 4;
      if (i < len) v[u] = ld_sys4(tab->buf[p] + poff + n + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = slice + ((int64_t)u * kXThreads + threadIdx.x) * 4;
      if (i < len) *reinterpret_cast<float4*>(out + cb + i) = v[u];
    }
  }
}

}  // namespace

int xchg_allreduce_blocks(int64_t n, int max_blocks, int* unroll) {
  // Prefer >= 256 workgroups (one per CU) for latency; grow U when the flag
  // table would be exceeded.
  for (int u : {1, 2, 4, 8}) {
    const int64_t chunk = (int64_t)kXThreads * 4 * u;
    const int64_t g = (n + chunk - 1) / chunk;
    if (g <= max_blocks) {
      *unroll = u;
      return (int)(g < 1 ? 1 : g);
    }
  }
  return -1;
}

hipError_t xchg_allreduce_f32(const float* in, float* out, int64_t n, const XchgArgs& x,
                              int max_blocks, uint64_t seq, hipStream_t s) {
  if (n % 4 || x.tab == nullptr || n > x.half || seq == 0) return hipErrorInvalidValue;
  int u = 0;
  const int g = xchg_allreduce_blocks(n, max_blocks, &u);
  if (g < 0) return hipErrorInvalidValue;
  switch (u) {
    case 1: hipLaunchKernelGGL(xchg_allreduce_k<1>, dim3(g), dim3(kXThreads), 0, s, in, out, n, x, seq); break;
    case 2: hipLaunchKernelGGL(xchg_allreduce_k<2>, dim3(g), dim3(kXThreads), 0, s, in, out, n, x, seq); break;
    case 4: hipLaunchKernelGGL(xchg_allreduce_k<4>, dim3(g), dim3(kXThreads), 0, s, in, out, n, x, seq); break;
    default: hipLaunchKernelGGL(xchg_allreduce_k<8>, dim3(g), dim3(kXThreads), 0, s, in, out, n, x, seq); break;
  }
  return hipGetLastError();
}

hipError_t xchg_allreduce2_f32(const float* in, float* out, int64_t n, const XchgArgs& x,
                               int max_blocks, uint64_t seq, hipStream_t s) {
  // flags: max_blocks / 2 per phase (the exchange holds max_blocks flags)
  const int fo = max_blocks / 2;
  if (n % 4 || x.tab == nullptr || seq == 0 || x.nranks < 1 || fo < 1) return hipErrorInvalidValue;
  const int64_t cs = ((n + x.nranks - 1) / x.nranks + 3) / 4 * 4;
  if (n + cs > x.half) return hipErrorInvalidValue;
  int u = 0;
  const int g = xchg_allreduce_blocks(cs, fo, &u);
  if (g < 0) return hipErrorInvalidValue;
  switch (u) {
    case 1: hipLaunchKernelGGL(xchg_allreduce2_k<1>, dim3(g), dim3(kXThreads), 0, s, in, out, n, cs, x, seq, fo); break;
    case 2: hipLaunchKernelGGL(xchg_allreduce2_k<2>, dim3(g), dim3(kXThreads), 0, s, in, out, n, cs, x, seq, fo); break;
    case 4: hipLaunchKernelGGL(xchg_allreduce2_k<4>, dim3(g), dim3(kXThreads), 0, s, in, out, n, cs, x, seq, fo); break;
    default: hipLaunchKernelGGL(xchg_allreduce2_k<8>, dim3(g), dim3(kXThreads), 0, s, in, out, n, cs, x, seq, fo); break;
  }
  return hipGetLastError();
}

}  // namespace dsml
