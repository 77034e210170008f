/*
 * gsdr-mi355x: stand-alone quadrature FM discriminator and AM envelope detector
 * (drop-in for reference include/gsdr/quad_demod.h:30-43, kernels src/quad_demod.cu:23-74).
 *
 *   gsdrQuadFmDemod: output[k] = gain * atan2(Im, Re)(input[k+1] * conj(input[k])), k < numOutputElements;
 *                    input holds numOutputElements + 1 samples; atan2(+-0, +0) = +-0.
 *   gsdrQuadAmDemod: output[k] = 2 * clamp(|input[k]|, 0, 1) - 1 (NaN magnitude -> -1, as __saturatef).
 */
#ifndef GSDR_QUAD_DEMOD_H_
#define GSDR_QUAD_DEMOD_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/quad_demod.h:30-36 (gsdrQuadFmDemod) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQuadFmDemod(
    const hipFloatComplex* input,
    float* output,
    float gain,
    size_t numOutputElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/quad_demod.h:38-43 (gsdrQuadAmDemod) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQuadAmDemod(
    const hipFloatComplex* input,
    float* output,
    size_t numOutputElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_QUAD_DEMOD_H_ */
