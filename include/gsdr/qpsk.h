/*
 * gsdr-mi355x: QPSK modulation / demodulation (drop-in for reference include/gsdr/qpsk.h:116-239,
 * kernels src/qpsk.cu). Symbols are 2 bits, packed four per byte, least-significant pair first.
 *
 *   Modulate   (qpsk.cu:108-146): s = (bits[k >> 2] >> 2*(k & 3)) & 3
 *                                 re = (s & 1) ? -amplitude : +amplitude, im = (s & 2) ? -amplitude : +amplitude
 *                                 (00 -> +a+aj, 01 -> -a+aj, 11 -> -a-aj, 10 -> +a-aj)
 *   Demodulate (qpsk.cu:221-268): s = (re >= 0 ? 0 : 1) | (im >= 0 ? 0 : 2)   (-0.0 -> 0, NaN -> bit set)
 *                                 packed into outputBits[k >> 2]; every byte that holds one of the
 *                                 numSymbols symbols is written, and in a final partial byte the unused
 *                                 high bit pairs are preserved (the reference's read-modify-write intent;
 *                                 this build writes whole bytes, no atomics).
 *   4x:        the same on four independent pointer sets, one launch.
 *   Templated: numStreams in {1, 2, 4, 8} streams in one consolidated buffer: stream s reads/writes its
 *              packed bits at byte offset s * (numSymbols / 4 + 1) and its symbols at element offset
 *              s * numSymbols (qpsk.cu:42, 56, 75, 87); any other numStreams processes stream 0 only,
 *              as the reference's fallback (qpsk.cu:619-622, 658-661).
 *
 * The reference also declares its __global__ kernels in this header (qpsk.h:34-103); they are
 * C++-mangled device symbols, not part of the C ABI, and are not exported here.
 */
#ifndef GSDR_QPSK_H_
#define GSDR_QPSK_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/qpsk.h:116-122 (gsdrQpskModulate) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpskModulate(
    const uint8_t* inputBits,
    hipFloatComplex* output,
    uint32_t numSymbols,
    float amplitude,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk.h:141-153 (gsdrQpskModulate4x) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpskModulate4x(
    const uint8_t* inputBits0,
    const uint8_t* inputBits1,
    const uint8_t* inputBits2,
    const uint8_t* inputBits3,
    hipFloatComplex* output0,
    hipFloatComplex* output1,
    hipFloatComplex* output2,
    hipFloatComplex* output3,
    uint32_t numSymbols,
    float amplitude,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk.h:171-182 (gsdrQpskDemodulate4x) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpskDemodulate4x(
    const hipFloatComplex* input0,
    const hipFloatComplex* input1,
    const hipFloatComplex* input2,
    const hipFloatComplex* input3,
    uint8_t* outputBits0,
    uint8_t* outputBits1,
    uint8_t* outputBits2,
    uint8_t* outputBits3,
    uint32_t numSymbols,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk.h:194-199 (gsdrQpskDemodulate) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpskDemodulate(
    const hipFloatComplex* input,
    uint8_t* outputBits,
    uint32_t numSymbols,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk.h:213-220 (gsdrQpskModulateTemplated) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpskModulateTemplated(
    const uint8_t* inputBits,
    hipFloatComplex* output,
    uint32_t numSymbols,
    float amplitude,
    int numStreams,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/qpsk.h:233-239 (gsdrQpskDemodulateTemplated) */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrQpskDemodulateTemplated(
    const hipFloatComplex* input,
    uint8_t* outputBits,
    uint32_t numSymbols,
    int numStreams,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_QPSK_H_ */
