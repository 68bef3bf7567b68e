// Microbenchmark: throughput of 16-B-a-lane stores into uncached (MTYPE UC)
// device memory -- the receive buffers every pkx push lands in
// (runtime/peer_exchange.cpp, hipDeviceMallocUncached) -- against the same
// stores into ordinary device memory.  B blocks x 4 waves, each wave storing
// S contiguous 1-KiB rows (buffer_store_dwordx4, system-scope sc0|sc1 as the
// pushes, or plain); per wave: time to ISSUE the S stores and time until the
// last is acknowledged (s_waitcnt vmcnt(0)), from s_memrealtime (100 MHz).
//
// Build:  hipcc -O3 --offload-arch=gfx950 tools/uc_store_bench.hip -o tools/bin/uc_store_bench
// Output: one JSON line per (memory, policy, blocks, stores a wave).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(256) void store_k(float* buf, int stores, uint64_t* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 0x7fffffff, 0x00020000);
  const int base = (blockIdx.x * 4 + w) * stores * 256;  // floats: S rows of 1 KiB a wave
  const u4 v = {(uint32_t)lane, 1u, (uint32_t)w, 1u};
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < stores; ++k)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (base + k * 256 + lane * 4) * 4, 0, AUX);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    out[(blockIdx.x * 4 + w) * 2 + 0] = t1 - t0;
    out[(blockIdx.x * 4 + w) * 2 + 1] = t2 - t0;
  }
}

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                       \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main() {
  const size_t bytes = 256ull << 20;
  float *uc = nullptr, *cg = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&uc), bytes, hipDeviceMallocUncached));
  CK(hipMalloc(&cg, bytes));
  uint64_t* d_out = nullptr;
  CK(hipMalloc(&d_out, 256 * 4 * 2 * sizeof(uint64_t)));
  std::vector<uint64_t> h(256 * 4 * 2);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mem = 0; mem < 2; ++mem) {
    for (int pol = 0; pol < 2; ++pol) {
      for (int blocks : {1, 8, 32, 128, 256}) {
        for (int stores : {24, 96}) {
          if ((size_t)blocks * 4 * stores * 1024 > bytes) continue;
          float* buf = mem ? cg : uc;
          auto launch = [&]() {
            if (pol == 0)
              hipLaunchKernelGGL(store_k<17>, dim3(blocks), dim3(256), 0, 0, buf, stores, d_out);
            else
              hipLaunchKernelGGL(store_k<0>, dim3(blocks), dim3(256), 0, 0, buf, stores, d_out);
          };
          for (int k = 0; k < 3; ++k) launch();
          CK(hipDeviceSynchronize());
          std::vector<double> issue, done, kern;
          for (int rep = 0; rep < 20; ++rep) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            kern.push_back(ms * 1e3);
            CK(hipMemcpy(h.data(), d_out, blocks * 4 * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
            double mi = 0, md = 0;
            for (int i = 0; i < blocks * 4; ++i) {
              mi = std::max(mi, h[i * 2] / 100.0);
              md = std::max(md, h[i * 2 + 1] / 100.0);
            }
            issue.push_back(mi);
            done.push_back(md);
          }
          auto med = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
          };
          const double mb = (double)blocks * 4 * stores * 1024 / 1e6;
          printf("{\"memory\": \"%s\", \"policy\": \"%s\", \"blocks\": %d, \"stores_per_wave\": %d, "
                 "\"MB\": %.3f, \"issue_us_max_wave\": %.2f, \"acked_us_max_wave\": %.2f, "
                 "\"GBps_acked\": %.1f, \"kernel_us_event\": %.1f}\n",
                 mem ? "coarse" : "uncached", pol ? "plain" : "sc0|sc1", blocks, stores, mb, med(issue),
                 med(done), mb * 1e3 / med(done), med(kern));
          fflush(stdout);
        }
      }
    }
  }
  return 0;
}
