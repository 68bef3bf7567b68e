// Microbenchmark: latency of polling loads from uncached (MTYPE UC) device
// memory -- the receive buffers of the persistent step's xGMI exchanges
// (runtime/peer_exchange.cpp, hipDeviceMallocUncached) -- against the same
// loads from ordinary (coarse-grained) memory, as a function of the number of
// 16-B-per-lane load instructions a wave has in flight and of how many waves
// (and blocks) share them.  The mlp_persist.hip exchange waits are rounds of
// such loads (px_tagged_gather: 2 per source; the DZR poll: 2 per source).
//
// Build:  hipcc -O3 --offload-arch=gfx950 tools/uc_bench.hip -o tools/bin/uc_bench
// Output: one JSON line per (memory, blocks, waves, loads/wave): median ns of
// one round (issue -> all data back), from s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void poll_k(const float* buf, int loads, int waves, int rounds,
                                              uint64_t* out, int aux_mode, int stride_kib = 1) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(buf), (short)0, 0x7fffffff, 0x00020000);
  const int base = (blockIdx.x * 4 + w) * 16 * 1024 * stride_kib;  // 16 strides per wave
  uint32_t acc = 0;
  for (int it = 0; it < rounds; ++it) {
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (w < waves) {
      u4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < loads) {
          if (aux_mode == 0)
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, base + j * stride_kib * 1024 + lane * 16, 0, 17);  // sc0 sc1
          else
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, base + j * stride_kib * 1024 + lane * 16, 0, 16);  // sc1
        }
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < loads) acc += v[j].x ^ v[j].w;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[blockIdx.x * rounds + it] = t1 - t0;
  }
  if (acc == 0x12345678u) out[0] = 0;  // keep the loads
}

// Push side: `stores` 16-B-per-lane (or 8-B with narrow) system-scope stores
// per wave; t_issue = the last store issued, t_done = all acknowledged.
__global__ __launch_bounds__(256) void push_k(float* buf, int stores, int waves, int rounds, uint64_t* out,
                                              int narrow, int aux = 17) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 0x7fffffff, 0x00020000);
  const int base = (blockIdx.x * 4 + w) * 64 * 1024;
  for (int it = 0; it < rounds; ++it) {
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (w < waves) {
      const u4 v = {(uint32_t)it, (uint32_t)lane, 1u, 2u};
      typedef uint32_t u2 __attribute__((ext_vector_type(2)));
      const u2 v2 = {(uint32_t)it, (uint32_t)lane};
      for (int j = 0; j < stores; ++j) {
        if (aux == 0) {
          if (narrow) __builtin_amdgcn_raw_buffer_store_b64(v2, r, base + (j * 64 + lane) * 8, 0, 0);
          else __builtin_amdgcn_raw_buffer_store_b128(v, r, base + (j * 64 + lane) * 16, 0, 0);
        } else if (aux == 16) {
          if (narrow) __builtin_amdgcn_raw_buffer_store_b64(v2, r, base + (j * 64 + lane) * 8, 0, 16);
          else __builtin_amdgcn_raw_buffer_store_b128(v, r, base + (j * 64 + lane) * 16, 0, 16);
        } else if (aux == 2) {
          if (narrow) __builtin_amdgcn_raw_buffer_store_b64(v2, r, base + (j * 64 + lane) * 8, 0, 2);
          else __builtin_amdgcn_raw_buffer_store_b128(v, r, base + (j * 64 + lane) * 16, 0, 2);
        } else {
          if (narrow) __builtin_amdgcn_raw_buffer_store_b64(v2, r, base + (j * 64 + lane) * 8, 0, 17);
          else __builtin_amdgcn_raw_buffer_store_b128(v, r, base + (j * 64 + lane) * 16, 0, 17);
        }
      }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      out[(blockIdx.x * rounds + it) * 2] = t1 - t0;
      out[(blockIdx.x * rounds + it) * 2 + 1] = t2 - t0;
    }
  }
}

// Mixed: wave 3 issues `stores` system-scope 16-B stores (region A) while waves
// 0-2 issue `loads` loads each (region B): does a pushing wave on the same CU
// slow the polling waves' loads?  out = waves 0-2's round time (wave 0).
__global__ __launch_bounds__(256) void mixed_k(float* bufA, const float* bufB, int stores, int loads, int rounds,
                                               uint64_t* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(bufA, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bufB), (short)0, 0x7fffffff, 0x00020000);
  uint32_t acc = 0;
  for (int it = 0; it < rounds; ++it) {
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (w == 3) {
      const u4 v = {(uint32_t)it, (uint32_t)lane, 1u, 2u};
      for (int j = 0; j < stores; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(v, ra, (blockIdx.x * 64 + j) * 1024 + lane * 16, 0, 17);
    } else {
      u4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < loads)
          v[j] = __builtin_amdgcn_raw_buffer_load_b128(rbb, ((blockIdx.x * 4 + w) * 16 + j) * 1024 + lane * 16, 0, 17);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < loads) acc += v[j].x ^ v[j].w;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[blockIdx.x * rounds + it] = t1 - t0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) out[0] = 0;
}

// The pkx step's exchange traffic at 8 replicas, on one GPU: 16 "tile" blocks
// (wave 3 pushes 42 stores, waves 0-2 time 14 loads), 4 "chain" blocks (32
// stores a wave), `l1` "layer-1" blocks (14 loads a wave, or none).
__global__ __launch_bounds__(256) void contend_k(float* bufA, const float* bufB, int l1, int rounds,
                                                 uint64_t* out, int chain_stores) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, b = blockIdx.x;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(bufA, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bufB), (short)0, 0x7fffffff, 0x00020000);
  uint32_t acc = 0;
  if (b >= 20 + l1) return;
  for (int it = 0; it < rounds; ++it) {
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const bool tile = b < 16, chain = b >= 16 && b < 20;
    if ((tile && w == 3) || chain) {
      const u4 v = {(uint32_t)it, (uint32_t)lane, 1u, 2u};
      const int ns = tile ? 42 : chain_stores;
      for (int j = 0; j < ns; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(v, ra, ((b * 4 + w) * 64 + j) * 1024 + lane * 16, 0, 17);
    } else {
      u4 v[14];
#pragma unroll
      for (int j = 0; j < 14; ++j)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(rbb, ((b * 4 + w) * 16 + j) * 1024 + lane * 16, 0, 17);
#pragma unroll
      for (int j = 0; j < 14; ++j) acc += v[j].x ^ v[j].w;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && tile) out[b * rounds + it] = t1 - t0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) out[0] = 0;
}

int main() {
  const size_t bytes = 1024ull << 20;
  float *uc = nullptr, *cg = nullptr;
  if (hipExtMallocWithFlags((void**)&uc, bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  if (hipMalloc((void**)&cg, bytes) != hipSuccess) return 1;
  hipMemset(uc, 0, bytes);
  hipMemset(cg, 0, bytes);
  const int rounds = 64;
  uint64_t* out = nullptr;
  hipMalloc((void**)&out, 256 * rounds * sizeof(uint64_t));
  std::vector<uint64_t> h(256 * rounds);
  for (int mem = 0; mem < 0; ++mem)
    for (int stride : {1, 4, 64, 1024})
      for (int blocks : {1, 16})
        for (int loads : {1, 2, 6, 14}) {
          const int waves = 1, aux = 0;
          if ((size_t)(blocks * 4) * 16 * stride * 1024 > bytes) continue;
          hipLaunchKernelGGL(poll_k, dim3(blocks), dim3(256), 0, 0, mem ? cg : uc, loads, waves, rounds, out, aux,
                             stride);
          hipDeviceSynchronize();
          hipMemcpy(h.data(), out, blocks * rounds * sizeof(uint64_t), hipMemcpyDeviceToHost);
          std::vector<uint64_t> v;
          for (int b = 0; b < blocks; ++b)
            for (int it = 8; it < rounds; ++it) v.push_back(h[b * rounds + it]);
          std::sort(v.begin(), v.end());
          printf("{\"mem\": \"%s\", \"stride_kib\": %d, \"blocks\": %d, \"loads_per_wave\": %d, "
                 "\"median_ns\": %llu, \"p90_ns\": %llu}\n",
                 mem ? "coarse" : "uncached", stride, blocks, loads, (unsigned long long)(v[v.size() / 2] * 10),
                 (unsigned long long)(v[v.size() * 9 / 10] * 10));
        }
  for (int blocks : {1, 16})
    for (int stores : {0, 14, 28, 42})
      for (int loads : {2, 14}) {
        hipLaunchKernelGGL(mixed_k, dim3(blocks), dim3(256), 0, 0, uc, uc + (256 << 20) / 4, stores, loads, rounds,
                           out);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), out, blocks * rounds * sizeof(uint64_t), hipMemcpyDeviceToHost);
        std::vector<uint64_t> v;
        for (int b = 0; b < blocks; ++b)
          for (int it = 8; it < rounds; ++it) v.push_back(h[b * rounds + it]);
        std::sort(v.begin(), v.end());
        printf("{\"mixed\": 1, \"blocks\": %d, \"stores_wave3\": %d, \"loads_per_wave\": %d, \"median_ns\": %llu}\n",
               blocks, stores, loads, (unsigned long long)(v[v.size() / 2] * 10));
      }
  for (int l1 : {0, 56, 224})
    for (int cs : {0, 32}) {
      hipLaunchKernelGGL(contend_k, dim3(20 + l1), dim3(256), 0, 0, uc, uc + (256 << 20) / 4, l1, rounds, out, cs);
      hipDeviceSynchronize();
      hipMemcpy(h.data(), out, 16 * rounds * sizeof(uint64_t), hipMemcpyDeviceToHost);
      std::vector<uint64_t> v;
      for (int b = 0; b < 16; ++b)
        for (int it = 8; it < rounds; ++it) v.push_back(h[b * rounds + it]);
      std::sort(v.begin(), v.end());
      printf("{\"contend\": 1, \"l1_blocks\": %d, \"chain_stores\": %d, \"tile_gather_median_ns\": %llu, \"p90\": %llu}\n",
             l1, cs, (unsigned long long)(v[v.size() / 2] * 10), (unsigned long long)(v[v.size() * 9 / 10] * 10));
    }
  std::vector<uint64_t> h2(256 * rounds * 2);
  uint64_t* out2 = nullptr;
  hipMalloc((void**)&out2, 256 * rounds * 2 * sizeof(uint64_t));
  for (int mem = 0; mem < 2; ++mem)
    for (int aux : {0, 2, 16, 17})
      for (int stores : {14, 42}) {
        const int blocks = 1, waves = 1, narrow = 0;
        hipLaunchKernelGGL(push_k, dim3(blocks), dim3(256), 0, 0, mem ? cg : uc, stores, waves, rounds, out2, narrow,
                           aux);
        hipDeviceSynchronize();
        hipMemcpy(h2.data(), out2, blocks * rounds * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost);
        std::vector<uint64_t> vi, vd;
        for (int it = 8; it < rounds; ++it) {
          vi.push_back(h2[it * 2]);
          vd.push_back(h2[it * 2 + 1]);
        }
        std::sort(vi.begin(), vi.end());
        std::sort(vd.begin(), vd.end());
        printf("{\"push_aux\": %d, \"mem\": \"%s\", \"stores\": %d, \"issue_ns\": %llu, \"done_ns\": %llu}\n", aux,
               mem ? "coarse" : "uncached", stores, (unsigned long long)(vi[vi.size() / 2] * 10),
               (unsigned long long)(vd[vd.size() / 2] * 10));
      }
  return 0;
}
