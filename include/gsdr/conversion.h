/*
 * gsdr-mi355x: int8 sample conversion (drop-in for reference include/gsdr/conversion.h:24-26,
 * kernel src/conversion.cu:20-35).
 *
 *   gsdrInt8ToNormFloat: output[k] = max(-1.0f, (float)input[k] / 127.0f)   (IEEE division)
 * Exactly numElements outputs (the reference also wrote output[numElements]).
 * Interleaved int8 I/Q feeds the fused FIR directly: gsdrxFirFCInt8 (gsdr_ext.h) applies this
 * conversion to each component while staging, so the float samples never touch HBM.
 */
#ifndef GSDR_CONVERSION_H_
#define GSDR_CONVERSION_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/conversion.h:24-26 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrInt8ToNormFloat(
    const int8_t* input,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_CONVERSION_H_ */
