/*
 * gsdr-mi355x: fused NCO frequency shift + low-pass FIR + decimation + FM quadrature discriminator
 * (drop-in for reference include/gsdr/fm.h:42-55, kernel src/fm.cu:21-69, 181-218).
 *
 * Semantics (the reference's NCO helper src/adjustFrequency.cu:25-56 never
 * returns its value, so its behaviour is re-specified here):
 *
 *   NCO:  inc  = (uint32) round((tuningFrequency - channelFrequency) / rfSampleRate * 2^32)
 *         P(n) = (uint32)((firstSampleIndex + n) * inc)            (exact integer phase)
 *         z[n] = input[n] * exp(+j * 2*pi * P(n) / 2^32)           (mixer sign as adjustFrequency.cu:50-51)
 *   FIR:  y[m] = sum_{i<numLowPassTaps} z[m*decimation + i] * lowPassTaps[i],   m in [0, numOutputs]
 *   FM:   output[m] = g * atan2(Im, Re)(y[m+1] * conj(y[m])),                   m in [0, numOutputs)
 *         g = rfSampleRate / (2*pi*frequencyDeviation)                         (as src/fm.cu:203)
 *
 * `input` must hold numOutputs * decimation + numLowPassTaps samples (the reference header's
 * "(numOutputs + 1) * decimation" under-states what its kernel reads). Streaming (as fm.h:26 asks:
 * an overlap of numLowPassTaps inputs): start the next call at input + numOutputs * decimation with
 * firstSampleIndex + numOutputs * decimation; the NCO phase is a function of the absolute sample
 * index, so chunked runs reproduce one monolithic run. The mixer frequency is quantised to
 * rfSampleRate / 2^32.
 */
#ifndef GSDR_FM_H_
#define GSDR_FM_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/fm.h:42-55 (gsdrFmDemod) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrFmDemod(
    float rfSampleRate,
    float tuningFrequency,
    float channelFrequency,
    float frequencyDeviation,
    uint32_t decimation,
    size_t firstSampleIndex,
    const float* lowPassTaps,
    size_t numLowPassTaps,
    const hipFloatComplex* input,
    float* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_FM_H_ */
