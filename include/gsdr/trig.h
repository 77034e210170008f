/*
 * gsdr-mi355x: phase-ramp tone generators (drop-in for reference include/gsdr/trig.h:26-40,
 * kernels src/trig.cu:20-75).
 *
 *   m = (float)((double)(phiEnd - phiBegin) / (double)numElements)   (host, as trig.cu:55, 70)
 *   theta[x] = fmaf((float)(uint32_t)x, m, phiBegin)                 (trig.cu:26 as nvcc contracts it)
 *   gsdrCosineC: output[x] = (cosf(theta), sinf(theta))
 *   gsdrCosineF: output[x] = cosf(theta)
 * The index is 32-bit as in the reference (x wraps past 2^32 elements). Exactly numElements
 * outputs are written; numElements == 0 returns hipSuccess without a launch.
 */
#ifndef GSDR_TRIG_H_
#define GSDR_TRIG_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/trig.h:26-32 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrCosineC(
    float phiBegin,
    float phiEnd,
    hipFloatComplex* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/trig.h:34-40 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrCosineF(
    float phiBegin,
    float phiEnd,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_TRIG_H_ */
