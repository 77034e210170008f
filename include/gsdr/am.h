/*
 * gsdr-mi355x: fused NCO frequency shift + low-pass FIR + decimation + AM envelope
 * (drop-in for reference include/gsdr/am.h:25-37, kernel src/am.cu:21-81).
 *
 * Semantics: z and y exactly as in gsdr/fm.h, for m in [0, numElements);
 *   output[m] = 2 * clamp(|y[m]|, 0, 1) - 1          (reference src/am.cu:49)
 * `input` must hold (numElements - 1) * decimation + numLowPassTaps samples.
 */
#ifndef GSDR_AM_H_
#define GSDR_AM_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/am.h:25-37 (gsdrAmDemod) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAmDemod(
    float rfSampleRate,
    float tuningFrequency,
    float channelFrequency,
    uint32_t decimation,
    size_t firstSampleIndex,
    const float* lowPassTaps,
    size_t numLowPassTaps,
    const hipFloatComplex* input,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_AM_H_ */
