/*
 * gsdr-mi355x: the reference's caller-facing error helpers under their reference names
 * (reference include/gsdr/cuda_util.h:32-97), so host code written against the reference's
 * `#include <gsdr/gsdr.h>` keeps compiling. They operate on HIP: the commands they wrap return
 * hipError_t and the functions using them return hipError_t, as every gsdr entry point does.
 *
 *   CHECK_CUDA_RET(descriptionCStr)  cuda_util.h:32-57. Only when DEBUG is defined (as in the
 *                                    reference): hipDeviceSynchronize(), and on failure print
 *                                    "file:line - Error n - name - description" to stderr and return
 *                                    the error. Otherwise a no-op.
 *   SAFE_CUDA_RET(cmd)               cuda_util.h:59-82. Run `cmd` (a hipError_t expression); on failure
 *                                    print "file:line - Error n - name - cmd" and return the error.
 *                                    Bracketed by CHECK_CUDA_RET("Before: cmd") / ("After: cmd").
 *   getCurrentCudaDevice()           cuda_util.h:88-97. The calling thread's current device, or the
 *                                    negated hipError_t on failure.
 *
 * The GSDR_*_HIP_RET / gsdrGetCurrentHipDevice spellings of hip_util.h are the same helpers.
 */
#ifndef GSDR_CUDA_UTIL_H_
#define GSDR_CUDA_UTIL_H_

#include <gsdr/hip_util.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>

#ifdef DEBUG
#define CHECK_CUDA_RET(descriptionCStr)                                                            \
  do {                                                                                             \
    const hipError_t gsdrCheckCudaRetStatus_ = hipDeviceSynchronize();                             \
    if (gsdrCheckCudaRetStatus_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d - Error %d - %s - %s\n", __FILE__, __LINE__,                         \
              (int)gsdrCheckCudaRetStatus_, hipGetErrorName(gsdrCheckCudaRetStatus_),              \
              (descriptionCStr));                                                                  \
      return gsdrCheckCudaRetStatus_;                                                              \
    }                                                                                              \
  } while (0)
#else
#define CHECK_CUDA_RET(descriptionCStr) (void)0
#endif

#define SAFE_CUDA_RET(cmd)                                                                         \
  do {                                                                                             \
    CHECK_CUDA_RET("Before: " #cmd);                                                               \
    const hipError_t gsdrSafeCudaRetStatus_ = (cmd);                                               \
    if (gsdrSafeCudaRetStatus_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d - Error %d - %s - %s\n", __FILE__, __LINE__,                         \
              (int)gsdrSafeCudaRetStatus_, hipGetErrorName(gsdrSafeCudaRetStatus_), #cmd);        \
      return gsdrSafeCudaRetStatus_;                                                               \
    }                                                                                              \
    CHECK_CUDA_RET("After: " #cmd);                                                                \
  } while (0)

/** Current device of the calling host thread, or the negated hipError_t (cuda_util.h:88-97). */
static inline int32_t getCurrentCudaDevice(void) { return gsdrGetCurrentHipDevice(); }

#endif /* GSDR_CUDA_UTIL_H_ */
