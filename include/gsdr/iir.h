/*
 * gsdr-mi355x: IIR filter as a true recursive filter (drop-in for
 * reference include/gsdr/iir.h, kernels src/iir.cu).
 *
 *   y[n] = sum_{i=0}^{K-1} b[i] x[n-i] - sum_{i=1}^{K-1} a[i] y[n-i]        (K = coeffCount)
 *
 * a[0] is not used (taken as 1, as the reference's loop from i = 1, iir.cu:170-174). bCoeffs and
 * aCoeffs are device arrays of K floats; 2 <= K <= 32 (the reference's limits, iir.cu:229-235).
 *
 * History (the parameters the reference accepts but ignores, iir.cu:213-214): when non-null,
 * inputHistory[i] = x[-1-i] and outputHistory[i] = y[-1-i] for i < K-1 are read as the state before
 * input[0], and on completion they hold the last K-1 inputs / outputs of the signal seen so far
 * (including older history when numElements < K-1), so consecutive calls continue one recursion.
 * Null history means zero state and is not written. The reference instead restarts from zero state
 * every 8 samples (iir.cu:121-127), which is not an IIR; its complex variant does not compile
 * (operator- on cuComplex, iir.cu:178).
 *
 * The recursion runs as a parallel scan (chunks of the signal filtered from zero state, the (K-1)-
 * dimensional state carried across chunks with transition-matrix powers, then each chunk re-run from
 * its true start state), so float32 results differ from a sequential float32 loop by rounding only;
 * tests bound the difference against a float64 evaluation. Scratch memory comes from the stream-
 * ordered allocator on `cudaStream` (hipMallocAsync / hipFreeAsync); the call stays asynchronous.
 * gsdrIir*Custom accept samplesPerThread in [1, 32] as the reference does; the results do not depend
 * on it (the chunking is chosen internally).
 */
#ifndef GSDR_IIR_H_
#define GSDR_IIR_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/iir.h gsdrIirFF */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrIirFF(
    const float* bCoeffs,
    const float* aCoeffs,
    size_t coeffCount,
    float* inputHistory,
    float* outputHistory,
    const float* input,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/iir.h gsdrIirCC (real coefficients, complex samples) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrIirCC(
    const float* bCoeffs,
    const float* aCoeffs,
    size_t coeffCount,
    hipFloatComplex* inputHistory,
    hipFloatComplex* outputHistory,
    const hipFloatComplex* input,
    hipFloatComplex* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/iir.h gsdrIirFFCustom */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrIirFFCustom(
    const float* bCoeffs,
    const float* aCoeffs,
    size_t coeffCount,
    float* inputHistory,
    float* outputHistory,
    const float* input,
    float* output,
    size_t numElements,
    size_t samplesPerThread,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/iir.h gsdrIirCCCustom */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrIirCCCustom(
    const float* bCoeffs,
    const float* aCoeffs,
    size_t coeffCount,
    hipFloatComplex* inputHistory,
    hipFloatComplex* outputHistory,
    const hipFloatComplex* input,
    hipFloatComplex* output,
    size_t numElements,
    size_t samplesPerThread,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_IIR_H_ */
