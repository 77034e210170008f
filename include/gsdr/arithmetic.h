/*
 * gsdr-mi355x: element-wise magnitude (drop-in for reference include/gsdr/arithmetic.h:90-92,
 * kernel src/magnitude.cu:20-45). The rest of the reference's arithmetic.h (add-constant, multiply,
 * abs) is outside the hot-path scope of this build.
 *
 *   gsdrMagnitude: out[k] = hypot(in[k].x, in[k].y), k < numElements
 *   (the reference's `x > n` bound check also writes out[numElements]; this build does not).
 */
#ifndef GSDR_ARITHMETIC_H_
#define GSDR_ARITHMETIC_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/arithmetic.h:90-92 (gsdrMagnitude) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrMagnitude(
    const hipFloatComplex* in,
    float* out,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_ARITHMETIC_H_ */
