/*
 * gsdr-mi355x extension: streaming continuity.
 *
 * The reference leaves the overlap between consecutive calls to the caller (include/gsdr/fm.h:26,
 * `firstSampleIndex` fm.h:48, am.h:30, fm.cu:202): to filter a stream in chunks, the caller must
 * re-supply the last taps-1 samples of the previous chunk and advance the NCO index itself. A
 * gsdrxStream object does that bookkeeping on the device: it keeps the samples the next output still
 * needs (fewer than one filter window) in a small device buffer, and each call is ONE kernel launch that
 * reads the outputs whose window straddles the seam partly from that history (by offset) and every other
 * output straight from the caller's chunk, while one workgroup of the same launch copies the next history;
 * it advances the absolute sample index that the NCO phase is derived from. (Decimations served by the
 * runtime-decimation or generic kernels take three launches: history + chunk head gathered into a seam
 * buffer, then the seam outputs and the remaining outputs.)
 *
 * Contract: feeding a signal x[0..S) in chunks of any sizes (including 0 and chunks shorter than the
 * filter) produces, concatenated over the calls, exactly the outputs of ONE call of the underlying
 * entry point over x[0..S) with firstSampleIndex = the value given at creation -- bit for bit
 * (the launch runs the kernel the single call runs, whose per-output summation order does not depend on
 * where a call or tile starts, and the NCO phase is a function of the absolute sample index). Output m is produced by the first call after which its
 * whole window has arrived: FIR/AM windows are taps samples, FM windows taps + decimation samples.
 *
 * Kinds: GSDRX_STREAM_FIR (gsdrFirFC), GSDRX_STREAM_FM (gsdrFmDemod), GSDRX_STREAM_AM (gsdrAmDemod).
 * Sample formats: GSDRX_SAMPLES_CF32 (hipFloatComplex) or GSDRX_SAMPLES_CS8 (interleaved int8 I/Q,
 * the gsdrx*Int8 entry points of gsdr_ext.h). int8 streams reproduce those entry points' defaults, the
 * decimation-4 matrix-core kernels included: their summation blocks follow the absolute output index
 * (the stream passes it to every launch), not where a call starts.
 *
 * Threading and streams: one object is one signal stream, and every gsdrxStreamProcess call on it must
 * be given the SAME hipStream_t. The object keeps its history in two device buffers used alternately
 * (each call reads the previous call's history buffer and writes the other one, with no event or
 * synchronisation between calls), so the calls are ordered only by the HIP stream they share: feeding
 * one object from two HIP streams lets call k+1 read the history before call k has written it. To move
 * an object to another HIP stream, synchronise the old one first. Do not call one object from two host
 * threads concurrently. The taps buffer is the caller's and must stay valid while the object is used.
 */
#ifndef GSDR_STREAM_H_
#define GSDR_STREAM_H_

#include <gsdr/gsdr_export.h>
#include <gsdr/gsdr_ext.h>
#include <gsdr/util.h>
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#define GSDRX_STREAM_FIR 0
#define GSDRX_STREAM_FM 1
#define GSDRX_STREAM_AM 2

typedef struct gsdrxStream_t* gsdrxStream;

/**
 * Create a stream on `cudaDevice` (allocates two history buffers and a seam buffer of at most
 * 2 * (tapCount + decimation) samples each; nothing is allocated later). For GSDRX_STREAM_FIR the
 * frequency arguments are ignored; for GSDRX_STREAM_AM frequencyDeviation is ignored.
 * Returns hipErrorInvalidValue for a null handle pointer, decimation == 0, tapCount == 0, null taps
 * or an unknown kind / sample format.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxStreamCreate(
    gsdrxStream* stream,
    int kind,
    int sampleFormat,
    uint32_t decimation,
    const float* taps,
    size_t tapCount,
    float rfSampleRate,
    float tuningFrequency,
    float channelFrequency,
    float frequencyDeviation,
    size_t firstSampleIndex,
    int32_t cudaDevice) GSDR_NO_EXCEPT;

/**
 * Create a MULTI-CHANNEL stream: `numChannels` FM or AM channels of one RF input (the streaming form of
 * gsdrxFmDemodMulti / gsdrxAmDemodMulti; the intent of the reference's dead k_Fm4x, src/fm.cu:71-179).
 * Channel c mixes by tuningFrequency - channelFrequencies[c] and, for FM, uses frequencyDeviations[c]
 * (ignored, and may be null, for AM). The input history is kept once for all channels. Each
 * gsdrxStreamProcess call is one launch per 16 channels for complex float input at decimation 2, 4 or 8
 * (the grouped kernel: each input tile read from HBM about once for all its channels), one launch per channel
 * otherwise (int8 I/Q at decimation 4: the matrix-core chain of each channel). Channel c's outputs are
 * bit-identical to a single-channel gsdrxStream with that channel's frequency (and so to one monolithic
 * gsdrFmDemod / gsdrAmDemod / gsdrx*Int8 call). In gsdrxStreamProcess, channel c's outputs go to
 * output + c * outputCapacity (outputCapacity = the per-channel capacity, in outputs), and
 * *numOutputsWritten / gsdrxStreamOutputsFor count the outputs of ONE channel.
 * Returns hipErrorInvalidValue for kind GSDRX_STREAM_FIR, numChannels == 0, null channelFrequencies, null
 * frequencyDeviations for FM, and as gsdrxStreamCreate.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxStreamCreateMulti(
    gsdrxStream* stream,
    int kind,
    int sampleFormat,
    uint32_t decimation,
    const float* taps,
    size_t tapCount,
    float rfSampleRate,
    float tuningFrequency,
    const float* channelFrequencies,
    const float* frequencyDeviations,
    uint32_t numChannels,
    size_t firstSampleIndex,
    int32_t cudaDevice) GSDR_NO_EXCEPT;

/** Number of outputs (per channel) the next gsdrxStreamProcess call with `numInputSamples` samples will write. */
GSDR_C_LINKAGE GSDR_PUBLIC size_t gsdrxStreamOutputsFor(gsdrxStream stream, size_t numInputSamples) GSDR_NO_EXCEPT;

/**
 * Append `numInputSamples` samples (device memory, in the stream's sample format) and write every
 * output that became computable to `output` (hipFloatComplex for FIR, float for FM/AM), in order
 * (a multi-channel stream: channel c's at output + c * outputCapacity).
 * `*numOutputsWritten` receives the count (host-known, no synchronisation). Asynchronous on
 * `cudaStream`; the input chunk may be reused once the stream's work has completed. Returns
 * hipErrorInvalidValue, leaving the stream unchanged, when outputCapacity is too small.
 * On any other error (a launch failing) the stream's state is also left unchanged -- the same chunk can
 * be passed again -- but the contents of `output` are unspecified: a multi-channel stream launches its
 * channels (or groups of 16) in turn, and the launches before the failing one have written their
 * channels' outputs.
 */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxStreamProcess(
    gsdrxStream stream,
    const void* input,
    size_t numInputSamples,
    void* output,
    size_t outputCapacity,
    size_t* numOutputsWritten,
    hipStream_t cudaStream) GSDR_NO_EXCEPT;

/** Free the stream's device buffers (synchronises the device, as hipFree does). Null is a no-op. */
GSDR_C_LINKAGE GSDR_PUBLIC hipError_t gsdrxStreamDestroy(gsdrxStream stream) GSDR_NO_EXCEPT;

/**
 * The host-side plan of one Process call, exposed so the planning logic can be tested without a GPU.
 * Inputs: decimation D, window W (samples one output needs), samples consumed so far, index of the
 * next output, chunk length. plan[0] = seam outputs (computed from history + chunk head),
 * plan[1] = samples of the chunk head copied behind the history for them, plan[2] = outputs computed
 * directly from the chunk, plan[3] = chunk offset of the first direct output's window,
 * plan[4] = history length after the call.
 */
GSDR_C_LINKAGE GSDR_PUBLIC void gsdrxStreamPlan(
    uint32_t decimation,
    size_t window,
    uint64_t consumed,
    uint64_t nextOutput,
    size_t chunk,
    uint64_t plan[5]) GSDR_NO_EXCEPT;

#endif /* GSDR_STREAM_H_ */
