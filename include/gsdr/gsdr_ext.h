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

/* input sample formats taken by the multi-channel chains and the streaming object (stream.h) */
#define GSDRX_SAMPLES_CF32 0 /* hipFloatComplex */
#define GSDRX_SAMPLES_CS8 1  /* interleaved int8 I/Q, converted as gsdrInt8ToNormFloat */

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
 * gsdrFirFC with an explicit kernel for decimation 4 (variant 0 = the default shape used by
 * gsdrFirFC; 1, 3, 4, 5, 24, 25, 26, 28 alternative workgroup / outputs-per-thread / chunk shapes; 7 = the
 * generic one-output-per-thread kernel; 8 = plain loads/stores; 9 = XCD-aware tile order; 10, 11 =
 * tile stored through LDS; 13 = exact-f32 matrix-core core, bit-identical to an ascending-tap fmaf
 * loop, tapCount <= 132; 14 = tile staged by LDS-DMA; >= 100 = ablation probes, not filters).
 * Unknown variants return hipErrorInvalidValue. Other decimations ignore `variant`.
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

/*
 * int8 I/Q front end fused into the filters. `input` holds interleaved
 * int8 I/Q pairs (2 bytes per complex sample; sample counts as in the float entry points). Each
 * component is converted exactly as gsdrInt8ToNormFloat does (max(-1, v / 127.0f), reference
 * src/conversion.cu:26) while the tile is staged, so the results are bit-identical to running
 * gsdrInt8ToNormFloat over the 2*L components and then the float entry point with the same
 * arguments -- without the float intermediate in HBM (2 instead of 8 input bytes per sample).
 */

/**
 * gsdrFirFC (fir.h) on int8 I/Q input.
 * Exception to the bit-identity above: decimation 4 with tapCount <= 196 runs on the matrix cores. The
 * samples are exact in bf16; the taps are scaled by a power of two and split EXACTLY into three bf16
 * parts (t = b1 + b2 + b3, 8 significant bits each, fp32's exponent range), so every product is exact and
 * the only roundings are the fp32 accumulation, in the matrix core's order, and the final scale. For every
 * input -- dense, sparse or impulsive, with taps spanning any range a float holds -- the result meets the
 * floating-point parity bar of the float path, max_k |y_k - y_float,k| / sum_i |t_i||x_(4k+i)| <= 1e-5
 * (an output whose window is all zero is exactly zero), rather than matching it bit for bit. Taps that are
 * not all finite, or whose nonzero magnitudes span more than ~2^200 (no exact split), take the exact
 * ascending loop. The summation order of output k depends only on the taps, its own window and
 * k mod 16 (k counted from the first output of the call; the streaming object, stream.h, passes the
 * stream's absolute output index instead), so the bits do not depend on the input or output pointers'
 * alignment. Variant 0 of gsdrxFirFCInt8Variant is the bit-identical packed-VALU path.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxFirFCInt8(
    size_t decimation,
    const float* taps,
    size_t tapCount,
    const int8_t* input,
    hipFloatComplex* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/** gsdrxFirFCInt8 with an explicit decimation-4 tile shape (tuning sweep; -1 = default; 40 / 41 = the
 *  matrix-core kernel at 2 / 3 workgroups per CU; 42 / 43 = at 3 workgroups per CU with 1,024- / 512-output
 *  tiles at every size; 44 = 512-output tiles at 4 workgroups per CU; 45 / 46 = 512-output tiles at 3 / 4
 *  workgroups per CU with two tiles in flight a workgroup; 42-46: tapCount <= 132, the default's outputs bit
 *  for bit). */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxFirFCInt8Variant(
    int variant,
    size_t decimation,
    const float* taps,
    size_t tapCount,
    const int8_t* input,
    hipFloatComplex* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/**
 * gsdrFmDemod (fm.h) on int8 I/Q input. Exception to the bit-identity above: decimation 4 with
 * numLowPassTaps <= 132 runs on the matrix cores with the NCO folded into complex taps
 * t_i e^{j 2 pi (i inc mod 2^32) / 2^32} (the discriminator adds the 4-sample phase step back, the
 * envelope needs no rotation), samples exact in bf16 and the complex taps split exactly into three bf16
 * parts as in gsdrxFirFCInt8. Parity with the float chain, not its bits:
 *   - the FIR outputs y meet the normwise bar above, so the envelope is within 1e-5 of the float chain's
 *     wherever |x| <= 1 (the int8 range);
 *   - the discriminator angle follows y: on a constant-envelope (FM) signal it is within 1e-5 pi g of the
 *     float chain's; an output whose window cancels to a small |y| (noise only, an out-of-band channel) or
 *     whose product y[k+1] conj y[k] falls below fp32's normal range is as uncertain as any fp32 evaluation
 *     of it (tests/helpers.py fm_conditioned_err states the bar);
 *   - where the product is exactly zero (a zero window beside another, silence, zero taps) the output is
 *     the reference's atan2f(+-0, +-0) value of the rotated outputs (fm.cu:66-68), bit for bit.
 * Non-finite or unsplittable taps take the exact per-output chain. The summation blocks follow the
 * absolute output index firstSampleIndex / 4 + k (mod 16), so a stream cut into calls by hand (each call
 * given its own firstSampleIndex) reproduces one call bit for bit; so do gsdrxStream (stream.h) and
 * gsdrxFmDemodMulti. A caller that needs gsdrFmDemod's own bits converts with gsdrInt8ToNormFloat first.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxFmDemodInt8(
    float rfSampleRate,
    float tuningFrequency,
    float channelFrequency,
    float frequencyDeviation,
    uint32_t decimation,
    size_t firstSampleIndex,
    const float* lowPassTaps,
    size_t numLowPassTaps,
    const int8_t* input,
    float* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/** gsdrAmDemod (am.h) on int8 I/Q input (decimation 4, <= 132 taps: the matrix cores, as gsdrxFmDemodInt8;
 * envelope within 1e-5 of the float chain's). */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxAmDemodInt8(
    float rfSampleRate,
    float tuningFrequency,
    float channelFrequency,
    uint32_t decimation,
    size_t firstSampleIndex,
    const float* lowPassTaps,
    size_t numLowPassTaps,
    const int8_t* input,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/*
 * Multi-channel chains (the intent of the reference's unused k_Fm4x,
 * src/fm.cu:71-179): numChannels channels of one RF input, each with its own channel frequency (and
 * FM deviation), sharing the tuning frequency, decimation, taps and firstSampleIndex. Channel c writes
 * output[c * numOutputs + m]; its outputs are bit-identical to gsdrFmDemod / gsdrAmDemod (int8 I/Q input:
 * gsdrxFmDemodInt8 / gsdrxAmDemodInt8) called with channelFrequencies[c] (and frequencyDeviations[c]).
 * For decimation 2, 4 and 8 one kernel reads each input tile from HBM once for up to 16 channels; int8
 * I/Q at decimation 4 with <= 132 taps runs each channel through the single-channel matrix-core chain;
 * other shapes run the channels one after another. channelFrequencies / frequencyDeviations are host
 * arrays.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxFmDemodMulti(
    float rfSampleRate,
    float tuningFrequency,
    const float* channelFrequencies,
    const float* frequencyDeviations,
    uint32_t numChannels,
    uint32_t decimation,
    size_t firstSampleIndex,
    const float* lowPassTaps,
    size_t numLowPassTaps,
    int sampleFormat,
    const void* input,
    float* output,
    size_t numOutputs,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxAmDemodMulti(
    float rfSampleRate,
    float tuningFrequency,
    const float* channelFrequencies,
    uint32_t numChannels,
    uint32_t decimation,
    size_t firstSampleIndex,
    const float* lowPassTaps,
    size_t numLowPassTaps,
    int sampleFormat,
    const void* input,
    float* output,
    size_t numElements,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/*
 * Config 5's channel model (BASELINE configs[4]: QPSK256 modulate -> AWGN -> demod): the output of
 * gsdrQpsk256Modulate (the table set by gsdrQpsk256InitConstellation for constellationType) plus
 * additive white Gaussian noise of standard deviation `sigma` per axis, in one pass:
 *     output[k] = table[inputBytes[k]] + (fl(sigma * g0), fl(sigma * g1)),  per component the product
 *     rounded, then the sum rounded (two roundings, no fused multiply-add),
 * where (g0, g1) are the standard normals of absolute symbol index firstSymbolIndex + k: 21 bits of
 * Philox4x32-10 keyed by `seed` per normal, mapped by inverse-CDF interpolation in a 672-entry
 * half-normal quantile table (within 2.5e-5 of the exact quantile); a component in the deep tail
 * (|g| > 4.17, ~3e-5 of them) draws 18 more bits from a second Philox block and a 768-entry tail table,
 * so the tails follow the Gaussian to within 1 % of its tail mass out to 6.5 and reach 7.0 (P(|g| > 7) =
 * 2.6e-12 per axis is the only mass missing: SER / BER sweeps are unbiased above ~1e-10). The exact
 * construction is in gsdr_amd/csrc/awgn.hpp and its host restatement in oracle/gsdr_oracle.h, built
 * from exact integer operations and one correctly rounded fmaf. The noise
 * is therefore a pure function of (seed, absolute index): a host can regenerate the noisy buffer bit
 * for bit, and splitting a buffer over several calls (advancing firstSymbolIndex) yields the same
 * samples. Returns hipErrorInvalidValue for null pointers or a negative / non-finite sigma.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxQpsk256ModulateAwgn(
    const uint8_t* inputBytes,
    hipFloatComplex* output,
    uint32_t numSymbols,
    uint32_t constellationType,
    float sigma,
    uint64_t seed,
    uint64_t firstSymbolIndex,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/*
 * Config 5's whole round trip in one pass: exactly what gsdrxQpsk256ModulateAwgn(inputBytes, noisySymbols, ...)
 * followed by gsdrQpsk256Demodulate(noisySymbols, outputBytes, numSymbols, constellationType, ...) write --
 * the same noisy symbols and the same decisions, bit for bit -- but for the rectangular table
 * (constellationType 0) one kernel demodulates each noisy symbol from the registers it was formed in, so the
 * noisy buffer is written once and never read back. Other tables run the two calls. Same errors as
 * gsdrxQpsk256ModulateAwgn, plus hipErrorInvalidValue for a null outputBytes.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxQpsk256ModulateAwgnDemodulate(
    const uint8_t* inputBytes,
    hipFloatComplex* noisySymbols,
    uint8_t* outputBytes,
    uint32_t numSymbols,
    uint32_t constellationType,
    float sigma,
    uint64_t seed,
    uint64_t firstSymbolIndex,
    int32_t cudaDevice,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

#endif /* GSDR_EXT_H_ */
