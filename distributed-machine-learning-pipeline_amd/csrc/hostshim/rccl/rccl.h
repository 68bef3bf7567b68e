// Host-only stand-in for <rccl/rccl.h> (sanitizer build only; see
// ../hip/hip_runtime.h).  Declares the types runtime.h names; the sanitizer
// build compiles no RCCL-calling code.
#pragma once
typedef struct ncclComm* ncclComm_t;
typedef enum { ncclSuccess = 0, ncclInProgress = 7 } ncclResult_t;
