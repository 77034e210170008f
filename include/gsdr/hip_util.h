/*
 * gsdr-mi355x: error-handling helpers for host code that calls HIP directly.
 *
 * Replaces reference include/gsdr/cuda_util.h:
 *   CHECK_CUDA_RET  (cuda_util.h:32-57) -> GSDR_CHECK_HIP_RET  (device sync + error check, only with GSDR_DEBUG_SYNC)
 *   SAFE_CUDA_RET   (cuda_util.h:59-82) -> GSDR_SAFE_HIP_RET   (run a HIP call, print "file:line - Error n - name - cmd"
 *                                                                to stderr and return its error on failure)
 *   getCurrentCudaDevice (cuda_util.h:88-97) -> gsdrGetCurrentHipDevice (current device, or -error on failure)
 *
 * The macros return from the enclosing function, so they are only usable in functions that return
 * hipError_t -- exactly as in the reference.
 */
#ifndef GSDR_HIP_UTIL_H_
#define GSDR_HIP_UTIL_H_

#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>

#ifdef GSDR_DEBUG_SYNC
#define GSDR_CHECK_HIP_RET(descriptionCStr)                                                        \
  do {                                                                                             \
    const hipError_t gsdrCheckStatus_ = hipDeviceSynchronize();                                    \
    if (gsdrCheckStatus_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d - Error %d - %s - %s\n", __FILE__, __LINE__, (int)gsdrCheckStatus_,   \
              hipGetErrorName(gsdrCheckStatus_), (descriptionCStr));                               \
      return gsdrCheckStatus_;                                                                     \
    }                                                                                              \
  } while (0)
#else
#define GSDR_CHECK_HIP_RET(descriptionCStr) ((void)0)
#endif

#define GSDR_SAFE_HIP_RET(cmd)                                                                     \
  do {                                                                                             \
    GSDR_CHECK_HIP_RET("Before: " #cmd);                                                           \
    const hipError_t gsdrSafeStatus_ = (cmd);                                                      \
    if (gsdrSafeStatus_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d - Error %d - %s - %s\n", __FILE__, __LINE__, (int)gsdrSafeStatus_,    \
              hipGetErrorName(gsdrSafeStatus_), #cmd);                                             \
      return gsdrSafeStatus_;                                                                      \
    }                                                                                              \
    GSDR_CHECK_HIP_RET("After: " #cmd);                                                            \
  } while (0)

/** Current HIP device of the calling host thread, or the negated hipError_t on failure. */
static inline int32_t gsdrGetCurrentHipDevice(void) {
  int device = -1;
  const hipError_t status = hipGetDevice(&device);
  if (status != hipSuccess) {
    return -(int32_t)status;
  }
  return (int32_t)device;
}

#endif /* GSDR_HIP_UTIL_H_ */
