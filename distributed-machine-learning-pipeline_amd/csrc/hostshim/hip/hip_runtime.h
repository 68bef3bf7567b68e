// Host-only stand-in for <hip/hip_runtime.h>, used ONLY by the sanitizer build
// of the host runtime (tests/test_host_sanitizers.py): "device" memory is host
// memory, copies are synchronous memcpy, streams and events are tokens.  It
// lets g++ -fsanitize=address,undefined / thread compile the runtime's host
// logic (DeviceArena bounds, CopyEngine chunking, StreamTable state machine,
// ring_plan.h schedules) — GPU sanitizers are not available on this pool.
// Never on the include path of the real build (_build.py).
#pragma once
#include <cstddef>
#include <cstdint>

typedef enum hipError_t {
  hipSuccess = 0,
  hipErrorInvalidValue = 1,
  hipErrorOutOfMemory = 2,
  hipErrorNotSupported = 801,
} hipError_t;
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;
typedef struct ihipGraph* hipGraph_t;
typedef struct hipGraphExec* hipGraphExec_t;
typedef enum hipMemcpyKind {
  hipMemcpyHostToHost = 0,
  hipMemcpyHostToDevice = 1,
  hipMemcpyDeviceToHost = 2,
  hipMemcpyDeviceToDevice = 3,
} hipMemcpyKind;
#define hipStreamNonBlocking 0x1
#define hipEventDisableTiming 0x2
#define hipHostMallocDefault 0x0

const char* hipGetErrorString(hipError_t e);
hipError_t hipSetDevice(int device);
hipError_t hipMalloc(void** p, size_t n);
hipError_t hipFree(void* p);
hipError_t hipMemset(void* p, int v, size_t n);
hipError_t hipHostMalloc(void** p, size_t n, unsigned flags);
hipError_t hipHostFree(void* p);
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t s);
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned flags);
hipError_t hipStreamDestroy(hipStream_t s);
hipError_t hipStreamSynchronize(hipStream_t s);
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned flags);
hipError_t hipEventDestroy(hipEvent_t e);
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s);
hipError_t hipEventSynchronize(hipEvent_t e);
