// Host implementations of the hip_runtime.h stand-in (sanitizer build only).
// Every call validates its arguments the way the runtime relies on (null
// handles, double frees) so misuse fails loudly under the sanitizers.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

struct ihipStream_t { unsigned flags; };
struct ihipEvent_t { std::atomic<int> recorded{0}; };

const char* hipGetErrorString(hipError_t e) {
  switch (e) {
    case hipSuccess: return "hipSuccess";
    case hipErrorInvalidValue: return "hipErrorInvalidValue";
    case hipErrorOutOfMemory: return "hipErrorOutOfMemory";
    default: return "hipError";
  }
}
hipError_t hipSetDevice(int device) { return device >= 0 ? hipSuccess : hipErrorInvalidValue; }
hipError_t hipMalloc(void** p, size_t n) {
  if (!p) return hipErrorInvalidValue;
  *p = std::malloc(n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipMemset(void* p, int v, size_t n) {
  if (!p && n) return hipErrorInvalidValue;
  std::memset(p, v, n);
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned) { return hipMalloc(p, n); }
hipError_t hipHostFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind, hipStream_t s) {
  if (!s || (n && (!dst || !src))) return hipErrorInvalidValue;
  std::memmove(dst, src, n);
  return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned flags) {
  if (!s) return hipErrorInvalidValue;
  *s = new ihipStream_t{flags};
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) { delete s; return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t s) { return s ? hipSuccess : hipErrorInvalidValue; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  if (!e) return hipErrorInvalidValue;
  *e = new ihipEvent_t();
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) { delete e; return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  if (!e || !s) return hipErrorInvalidValue;
  e->recorded.store(1);
  return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
  if (!e || !e->recorded.load()) return hipErrorInvalidValue;  // sync on a never-recorded event
  return hipSuccess;
}
