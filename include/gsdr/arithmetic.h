/*
 * gsdr-mi355x: element-wise arithmetic (drop-in for reference include/gsdr/arithmetic.h:26-95;
 * kernels src/add_const.cu:20-42, src/multiply.cu:20-27, src/magnitude.cu:20-36).
 *
 * Results are the reference's operator semantics (src/cuComplexOperatorOverloads.cuh:25-56):
 *   gsdrAddConstFF:     out = c + x
 *   gsdrAddConstCC:     out = (c.x + x.x, c.y + x.y)
 *   gsdrAddConstCF:     out = (x.x + c, x.y)       complex input + real constant: real part only
 *   gsdrAddConstFC:     out = (c.x + x, c.y)       real input + complex constant
 *     (the reference's tests/test_arithmetic.cpp:100, 116 expect the constant on both parts; the
 *      reference's operator+ adds it to the real part only, and this build returns what the reference
 *      computes — DESIGN.md section 7)
 *   gsdrMultiplyCC:     out = (a.x b.x - a.y b.y, a.x b.y + a.y b.x)   (cuCmulf, each product rounded)
 *   gsdrMultiplyFF:     out = a * b
 *   gsdrMultiplyCF:     out = (a.x b, a.y b)
 *   gsdrAddToMagnitude: m = hypot(x); out = (x.x / m * (c + m), x.y / m * (c + m))  (NaN for x = 0)
 *   gsdrMagnitude:      out = hypot(x.x, x.y)
 *   gsdrAbs:            out = |x|
 * Each writes exactly numElements outputs (the reference's `x > n` bound check also wrote
 * out[numElements]). numElements == 0 returns hipSuccess without a launch.
 */
#ifndef GSDR_ARITHMETIC_H_
#define GSDR_ARITHMETIC_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/util.h>
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

/* replaces reference include/gsdr/arithmetic.h:26-32 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAddConstFF(
    const float* input,
    float addConst,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:34-40 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAddConstCC(
    const hipFloatComplex* input,
    hipFloatComplex addConst,
    hipFloatComplex* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:42-48 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAddConstCF(
    const hipFloatComplex* input,
    float addConst,
    hipFloatComplex* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:50-56 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAddConstFC(
    const float* input,
    hipFloatComplex addConst,
    hipFloatComplex* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:58-64 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrMultiplyCC(
    const hipFloatComplex* in1,
    const hipFloatComplex* in2,
    hipFloatComplex* out,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:66-72 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrMultiplyFF(
    const float* in1,
    const float* in2,
    float* out,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:74-80 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrMultiplyCF(
    const hipFloatComplex* in1,
    const float* in2,
    hipFloatComplex* out,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:82-88 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAddToMagnitude(
    const hipFloatComplex* input,
    float addToMagnitude,
    hipFloatComplex* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:90-92 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrMagnitude(
    const hipFloatComplex* in,
    float* out,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/* replaces reference include/gsdr/arithmetic.h:94-95 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrAbs(
    const float* in,
    float* out,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_ARITHMETIC_H_ */
