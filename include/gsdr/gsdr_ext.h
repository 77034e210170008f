/*
 * gsdr-mi355x extensions: entry points that the reference does not have. Nothing on the drop-in path
 * needs them; they expose the exact NCO definition to callers that want to reproduce it, and a
 * tile-shape override used by the benchmark's tuning sweep.
 */
#ifndef GSDR_EXT_H_
#define GSDR_EXT_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/** Library version string, e.g. "gsdr-mi355x 0.1.0 (gfx950)". */
GSDR_C_LINKAGE GSDR_PUBLIC const char* gsdrVersion(void) GSDR_NO_EXCEPT;

/**
 * NCO phase increment used by gsdrFmDemod / gsdrAmDemod:
 * (uint32) llround((tuningFrequency - channelFrequency) / rfSampleRate * 2^32), two's complement for
 * negative shifts. Sample n (absolute index) is mixed with exp(+j*2*pi*((uint32)(n * inc)) / 2^32).
 */
GSDR_C_LINKAGE GSDR_PUBLIC uint32_t gsdrNcoPhaseIncrement(
    float rfSampleRate,
    float tuningFrequency,
    float channelFrequency) GSDR_NO_EXCEPT;

/**
 * gsdrFirFC with an explicit tile shape for decimation 4 (variant 0 = the default shape used by
 * gsdrFirFC; 1..6 alternative workgroup / outputs-per-thread / chunk shapes; 7 = the generic
 * one-output-per-thread kernel). Other decimations ignore `variant`.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxFirFCVariant(
    int variant,
    size_t decimation,
    const float* taps,
    size_t tapCount,
    const hipFloatComplex* input,
    hipFloatComplex* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_EXT_H_ */
