/*
 * gsdr-mi355x: 256-point constellation modulation / demodulation (drop-in for reference
 * include/gsdr/qpsk256.h:125-230, src/qpsk256.cu). One byte per symbol.
 *
 * Constellations (built on the host in float exactly as qpsk256.cu:29-71, uploaded per device):
 *   type 0, rectangular: point[16*i + q] = ((i - 7.5f) / 7.5f * a, (q - 7.5f) / 7.5f * a)
 *   type != 0, circular: rings of {1,8,16,24,32,40,48,56} points at radii {0,.3,.6,.85,1.1,1.35,1.6,1.85}*a,
 *                        angle 2*pi*p/P + 0.5*ring; points 225..255 at radius 0.95*a, angle 2*pi*idx/256.
 *
 * gsdrQpsk256InitConstellation must run on a device before modulate/demodulate use that type there.
 * It is stream-ordered on `cudaStream` (the reference's symbol copy ran on the legacy stream,
 * qpsk256.cu:285-289) and synchronises that stream before returning.
 *
 *   Modulate   (qpsk256.cu:74-101):  output[k] = point_type[input[k]]; `amplitude` is ignored, the scale is
 *                                     fixed by InitConstellation (as in the reference).
 *   Demodulate (qpsk256.cu:154-195): output[k] = the first index i attaining the minimum of
 *                                     cuCabsf(input[k] - point_i) (qpsk256.cu:171-181; CUDA's cuCabsf with IEEE
 *                                     division and square root), bit for bit; a non-finite received symbol
 *                                     yields 0 as in the reference.
 */
#ifndef GSDR_QPSK256_H_
#define GSDR_QPSK256_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/qpsk256.h:125-132 (gsdrQpsk256Modulate) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpsk256Modulate(
    const uint8_t* inputBytes,
    hipFloatComplex* output,
    uint32_t numSymbols,
    float amplitude,
    uint32_t constellationType,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk256.h:145-151 (gsdrQpsk256Demodulate) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpsk256Demodulate(
    const hipFloatComplex* input,
    uint8_t* outputBytes,
    uint32_t numSymbols,
    uint32_t constellationType,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk256.h:171-184 (gsdrQpsk256Modulate4x) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpsk256Modulate4x(
    const uint8_t* inputBytes0,
    const uint8_t* inputBytes1,
    const uint8_t* inputBytes2,
    const uint8_t* inputBytes3,
    hipFloatComplex* output0,
    hipFloatComplex* output1,
    hipFloatComplex* output2,
    hipFloatComplex* output3,
    uint32_t numSymbols,
    float amplitude,
    uint32_t constellationType,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk256.h:203-215 (gsdrQpsk256Demodulate4x) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpsk256Demodulate4x(
    const hipFloatComplex* input0,
    const hipFloatComplex* input1,
    const hipFloatComplex* input2,
    const hipFloatComplex* input3,
    uint8_t* outputBytes0,
    uint8_t* outputBytes1,
    uint8_t* outputBytes2,
    uint8_t* outputBytes3,
    uint32_t numSymbols,
    uint32_t constellationType,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk256.h:226-230 (gsdrQpsk256InitConstellation) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpsk256InitConstellation(
    uint32_t constellationType,
    float amplitude,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_QPSK256_H_ */
