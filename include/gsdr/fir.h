/*
 * gsdr-mi355x: decimating FIR filters (drop-in for reference include/gsdr/fir.h:30-68).
 *
 * Semantics (reference src/fir.cu:26-71, restated in SURVEY.md App. A.1):
 *
 *     output[k] = sum_{i=0}^{tapCount-1} input[k * decimation + i] * taps[i],   k in [0, numOutputs)
 *
 * i.e. a correlation with `taps` exactly as passed (the reference names them "tapsReversed").
 * The accumulator starts at zero; tapCount == 0 yields all-zero output.
 * `input` must hold at least (numOutputs - 1) * decimation + tapCount samples.
 * Letters: first = tap type, second = input type (F = float, C = hipFloatComplex).
 *   FC: real taps, complex input -> complex output     FF: real taps, real input -> real output
 *   CC: complex taps, complex input -> complex output   CF: complex taps, real input -> complex output
 *
 * All pointers are caller-owned device memory on `cudaDevice`; input and output must not overlap.
 * The call switches the calling thread to `cudaDevice`, enqueues one kernel on `cudaStream`, restores
 * the previous device and returns without synchronising. Unlike the reference, launch errors are
 * reported (hipGetLastError), decimation == 0 returns hipErrorInvalidValue and numOutputs == 0
 * returns hipSuccess without launching.
 */
#ifndef GSDR_FIR_H_
#define GSDR_FIR_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/fir.h:30-38 (gsdrFirFC) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrFirFC(
    size_t decimation,
    const float* taps,
    size_t tapCount,
    const hipFloatComplex* input,
    hipFloatComplex* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/fir.h:40-48 (gsdrFirFF) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrFirFF(
    size_t decimation,
    const float* taps,
    size_t tapCount,
    const float* input,
    float* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/fir.h:50-58 (gsdrFirCC) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrFirCC(
    size_t decimation,
    const hipFloatComplex* taps,
    size_t tapCount,
    const hipFloatComplex* input,
    hipFloatComplex* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/fir.h:60-68 (gsdrFirCF) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrFirCF(
    size_t decimation,
    const hipFloatComplex* taps,
    size_t tapCount,
    const float* input,
    hipFloatComplex* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_FIR_H_ */
