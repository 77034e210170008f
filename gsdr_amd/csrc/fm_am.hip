// gsdr-mi355x: fused NCO + low-pass FIR + decimation + FM discriminator / AM envelope.
//   gsdrFmDemod  replaces reference src/fm.cu:181-218 (kernel k_Fm, fm.cu:21-69)
//   gsdrAmDemod  replaces reference src/am.cu:52-81  (kernel k_Am, am.cu:21-50)
// Both run the FIR engine of fir_engine.hpp with the NCO applied once per staged input sample
// (the reference recomputes it per tap, adjustFrequency.cu:36-55) and the demodulator fused into the
// epilogue, so the mixed and filtered intermediates never touch HBM.
#include <hip/hip_runtime.h>
#include <math.h>

#include "fir_dispatch.hpp"
#include "gsdr/am.h"
#include "gsdr/fm.h"
#include "gsdr/gsdr_ext.h"
#include "launch.hpp"

namespace gsdr {

static constexpr float kPiF = 3.14159265358979323846f;

// inc = llround(df / fs * 2^32) mod 2^32, df = tuning - channel (fm.cu:204, am.cu:68).
static bool nco_increment(float fs, float tune, float chan, uint32_t* inc) {
  if (!(fs > 0.0f) || !isfinite(fs)) return false;
  const float df = tune - chan;
  if (!isfinite(df)) return false;
  const double turns = (double)df / (double)fs;
  const double scaled = turns * 4294967296.0;
  // reduce to [-2^32, 2^32] before rounding so llround never overflows
  const double reduced = fmod(scaled, 4294967296.0);
  *inc = (uint32_t)(int64_t)llround(reduced);
  return true;
}

template <class InT>
static hipError_t chain_entry(int mode, float fs, float tune, float chan, float dev, uint32_t decimation,
                              size_t firstSampleIndex, const float* taps, size_t tapCount, const InT* input,
                              float* output, size_t numOutputs, int32_t device, hipStream_t stream,
                              int variant = -1) {
  if (numOutputs == 0) return hipSuccess;
  if (decimation == 0 || output == nullptr || input == nullptr) return hipErrorInvalidValue;
  if (tapCount > 0 && taps == nullptr) return hipErrorInvalidValue;
  FirJob job;
  if (!nco_increment(fs, tune, chan, &job.nco_inc)) return hipErrorInvalidValue;
  job.in = input;
  job.taps = taps;
  job.out = output;
  job.D = decimation;
  job.T = tapCount;
  job.N = numOutputs;
  job.mode = mode;
  job.variant = variant;
  job.nco_n0 = (uint32_t)firstSampleIndex;
  // the int8 matrix-core chains align their 16-output blocks to the absolute output index
  // firstSampleIndex / D + k, so chunked calls reproduce one call bit for bit (fir_i8_mfma.hpp)
  job.out_phase = (uint32_t)((firstSampleIndex / decimation) & 15u);
  job.q0 = (uint32_t)(firstSampleIndex / decimation);  // the anchored tiles' NCO cell grid
  if (mode == kModeFm) {
    job.L = numOutputs * (size_t)decimation + tapCount;  // N + 1 FIR outputs
    job.fm_gain = fs / (2.0f * kPiF * dev);              // as reference src/fm.cu:203
  } else {
    job.L = (numOutputs - 1) * (size_t)decimation + tapCount;
  }
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  if (tapCount == 0) {
    // y == 0 everywhere: the generic kernel evaluates the epilogue on zero without touching taps
    return mode == kModeFm ? launch_generic<float, InT, kModeFm>(job, stream)
                           : launch_generic<float, InT, kModeAm>(job, stream);
  }
  return mode == kModeFm ? launch_fir<float, InT, kModeFm>(job, stream)
                         : launch_fir<float, InT, kModeAm>(job, stream);
}

template <class InT>
static hipError_t chain_multi_entry(int mode, float fs, float tune, const float* chans, const float* devs,
                                    uint32_t count, uint32_t decimation, size_t firstSampleIndex, const float* taps,
                                    size_t tapCount, const InT* input, float* output, size_t numOutputs,
                                    int32_t device, hipStream_t stream) {
  if (numOutputs == 0 || count == 0) return hipSuccess;
  if (chans == nullptr || (mode == kModeFm && devs == nullptr)) return hipErrorInvalidValue;
  if (decimation == 0 || output == nullptr || input == nullptr) return hipErrorInvalidValue;
  if (tapCount > 0 && taps == nullptr) return hipErrorInvalidValue;
  for (uint32_t c0 = 0; c0 < count; c0 += kMaxMultiChannels) {
    const uint32_t n = count - c0 < (uint32_t)kMaxMultiChannels ? count - c0 : (uint32_t)kMaxMultiChannels;
    MultiParams mp{};
    mp.count = n;
    mp.out_stride = numOutputs;
    for (uint32_t c = 0; c < n; ++c) {
      if (!nco_increment(fs, tune, chans[c0 + c], &mp.inc[c])) return hipErrorInvalidValue;
      mp.gain[c] = mode == kModeFm ? fs / (2.0f * kPiF * devs[c0 + c]) : 0.0f;
    }
    float* out = output + (size_t)c0 * numOutputs;
    hipError_t e = hipErrorNotSupported;
    // int8 I/Q at decimation 4: the single-channel default is the matrix-core chain, so each channel runs
    // it (bit-identical to gsdrxFmDemodInt8 / gsdrxAmDemodInt8 with that channel's frequency)
    bool grouped = tapCount > 0;
    if constexpr (std::is_same<InT, Iq8>::value) {
      if (decimation == 4 && tapCount <= (size_t)I8ChainMfma<kModeFm>::MAXT) grouped = false;
    }
    if (grouped) {
      FirJob job;
      job.in = input;
      job.taps = taps;
      job.out = out;
      job.D = decimation;
      job.T = tapCount;
      job.N = numOutputs;
      job.mode = mode;
      job.nco_n0 = (uint32_t)firstSampleIndex;
      job.q0 = (uint32_t)(firstSampleIndex / decimation);
      job.L = mode == kModeFm ? numOutputs * (size_t)decimation + tapCount
                              : (numOutputs - 1) * (size_t)decimation + tapCount;
      DeviceScope scope(device);
      if (scope.status() != hipSuccess) return scope.status();
      e = mode == kModeFm ? launch_multi_chain<InT, kModeFm>(job, mp, stream)
                          : launch_multi_chain<InT, kModeAm>(job, mp, stream);
    }
    // launch_multi_chain returns hipErrorNotSupported before launching anything (so there is no
    // sticky launch error of ours to clear): one channel at a time through the single-channel path
    if (e == hipErrorNotSupported) {
      e = hipSuccess;
      for (uint32_t c = 0; c < n && e == hipSuccess; ++c) {
        e = chain_entry(mode, fs, tune, chans[c0 + c], mode == kModeFm ? devs[c0 + c] : 1.0f, decimation,
                        firstSampleIndex, taps, tapCount, input, out + (size_t)c * numOutputs, numOutputs, device,
                        stream);
      }
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The streaming object's one-launch int8 chain step at decimation 4 (stream.hip; see fir_int8_stream_step):
// firstSampleIndex is the absolute index of output 0's first sample. hipErrorNotSupported: not this path.
hipError_t chain_int8_stream_step(int mode, float fs, float tune, float chan, float dev, size_t firstSampleIndex,
                                  const float* taps, size_t tapCount, const int8_t* chunk, uint64_t chunkLen,
                                  int64_t inOff, const int8_t* hist, uint64_t histLen, int8_t* histOut,
                                  int64_t histFrom, uint64_t histN, float* output, size_t numOutputs, int32_t device,
                                  hipStream_t stream) {
  if (numOutputs == 0 || tapCount == 0 || taps == nullptr || tapCount > (size_t)I8ChainMfma<kModeFm>::MAXT) {
    return hipErrorNotSupported;
  }
  FirJob job;
  if (!nco_increment(fs, tune, chan, &job.nco_inc)) return hipErrorInvalidValue;
  job.in = chunk;
  job.taps = taps;
  job.out = output;
  job.D = 4;
  job.T = tapCount;
  job.N = numOutputs;
  job.L = chunkLen;
  job.mode = mode;
  job.nco_n0 = (uint32_t)firstSampleIndex;
  job.out_phase = (uint32_t)((firstSampleIndex / 4) & 15u);
  job.q0 = (uint32_t)(firstSampleIndex / 4);
  if (mode == kModeFm) job.fm_gain = fs / (2.0f * kPiF * dev);
  job.in_off = inOff;
  job.hist = hist;
  job.hist_len = histLen;
  job.hist_out = histOut;
  job.hist_from = histFrom;
  job.hist_n = histN;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  return mode == kModeFm ? launch_chain_i8_mfma<kModeFm>(job, stream) : launch_chain_i8_mfma<kModeAm>(job, stream);
}

// The streaming object's one-launch chain step on the tiled kernels (stream_step_tiled), complex float or
// int8 I/Q chunks: firstSampleIndex is the absolute index of output 0's first sample.
hipError_t chain_stream_step_tiled(int mode, bool int8, float fs, float tune, float chan, float dev, uint32_t decimation,
                                   size_t firstSampleIndex, const float* taps, size_t tapCount, const void* chunk,
                                   uint64_t chunkLen, int64_t inOff, const void* hist, uint64_t histLen, void* histOut,
                                   int64_t histFrom, uint64_t histN, float* output, size_t numOutputs, int32_t device,
                                   hipStream_t stream) {
  FirJob job;
  if (!nco_increment(fs, tune, chan, &job.nco_inc)) return hipErrorInvalidValue;
  job.in = chunk;
  job.taps = taps;
  job.out = output;
  job.D = decimation;
  job.T = tapCount;
  job.N = numOutputs;
  job.L = chunkLen;
  job.mode = mode;
  job.nco_n0 = (uint32_t)firstSampleIndex;
  job.q0 = (uint32_t)(firstSampleIndex / decimation);
  if (mode == kModeFm) job.fm_gain = fs / (2.0f * kPiF * dev);
  job.in_off = inOff;
  job.hist = hist;
  job.hist_len = histLen;
  job.hist_out = histOut;
  job.hist_from = histFrom;
  job.hist_n = histN;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  if (int8) {
    return mode == kModeFm ? stream_step_tiled<Iq8, kModeFm>(job, stream) : stream_step_tiled<Iq8, kModeAm>(job, stream);
  }
  return mode == kModeFm ? stream_step_tiled<float2, kModeFm>(job, stream)
                         : stream_step_tiled<float2, kModeAm>(job, stream);
}

// The multi-channel streaming object's one-launch step (stream.hip, gsdrxStreamCreateMulti) on complex float
// chunks: the grouped kernel of gsdrxFmDemodMulti / gsdrxAmDemodMulti (up to kMaxMultiChannels channels a
// launch) with the single-channel stream step's operands -- output 0's window at chunk offset inOff, seam
// samples read from the shared input history, the next history copied by workgroup 0 of the first launch.
// Channel c's outputs go to output + c * outStride. Each workgroup runs the single-channel tile, so channel c
// is bit-identical to its own gsdrxStream (and to one monolithic call). hipErrorNotSupported (nothing
// launched): the shape has no grouped kernel; the stream then runs the channels one by one.
hipError_t chain_multi_stream_step(int mode, float fs, float tune, const float* chans, const float* devs, uint32_t count,
                                   uint32_t decimation, size_t firstSampleIndex, const float* taps, size_t tapCount,
                                   const hipFloatComplex* chunk, uint64_t chunkLen, int64_t inOff,
                                   const hipFloatComplex* hist, uint64_t histLen, hipFloatComplex* histOut,
                                   int64_t histFrom, uint64_t histN, float* output, size_t outStride, size_t numOutputs,
                                   int32_t device, hipStream_t stream) {
  if (numOutputs == 0 || count == 0 || tapCount == 0 || taps == nullptr || tapCount > (1u << 26)) {
    return hipErrorNotSupported;
  }
  if (decimation != 2 && decimation != 4 && decimation != 8) return hipErrorNotSupported;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  for (uint32_t c0 = 0; c0 < count; c0 += kMaxMultiChannels) {
    const uint32_t n = count - c0 < (uint32_t)kMaxMultiChannels ? count - c0 : (uint32_t)kMaxMultiChannels;
    MultiParams mp{};
    mp.count = n;
    mp.out_stride = outStride;
    for (uint32_t c = 0; c < n; ++c) {
      if (!nco_increment(fs, tune, chans[c0 + c], &mp.inc[c])) return hipErrorInvalidValue;
      mp.gain[c] = mode == kModeFm ? fs / (2.0f * kPiF * devs[c0 + c]) : 0.0f;
    }
    FirJob job;
    job.in = reinterpret_cast<const float2*>(chunk) + inOff;  // output 0's window (may precede the chunk)
    job.L = (uint64_t)((int64_t)chunkLen - inOff);
    job.taps = taps;
    job.out = output + (size_t)c0 * outStride;
    job.D = decimation;
    job.T = tapCount;
    job.N = numOutputs;
    job.mode = mode;
    job.nco_n0 = (uint32_t)firstSampleIndex;
    job.q0 = (uint32_t)(firstSampleIndex / decimation);
    job.in_off = inOff;
    job.hist = hist;
    job.hist_len = histLen;
    job.hist_out = c0 == 0 ? histOut : nullptr;  // every group reads the old history; the first writes the next
    job.hist_from = histFrom;
    job.hist_n = histN;
    job.stream_tiled = true;
    const hipError_t e = mode == kModeFm ? launch_multi_chain<float2, kModeFm>(job, mp, stream)
                                         : launch_multi_chain<float2, kModeAm>(job, mp, stream);
    if (e != hipSuccess) return e;  // hipErrorNotSupported only from the first group (same shape for all)
  }
  return hipSuccess;
}

}  // namespace gsdr

GSDR_C_LINKAGE hipError_t gsdrFmDemod(float rfSampleRate, float tuningFrequency, float channelFrequency,
                                      float frequencyDeviation, uint32_t decimation, size_t firstSampleIndex,
                                      const float* lowPassTaps, size_t numLowPassTaps, const hipFloatComplex* input,
                                      float* output, size_t numOutputs, int32_t cudaDevice,
                                      hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::chain_entry(gsdr::kModeFm, rfSampleRate, tuningFrequency, channelFrequency, frequencyDeviation,
                           decimation, firstSampleIndex, lowPassTaps, numLowPassTaps,
                           reinterpret_cast<const float2*>(input), output, numOutputs, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrAmDemod(float rfSampleRate, float tuningFrequency, float channelFrequency,
                                      uint32_t decimation, size_t firstSampleIndex, const float* lowPassTaps,
                                      size_t numLowPassTaps, const hipFloatComplex* input, float* output,
                                      size_t numElements, int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::chain_entry(gsdr::kModeAm, rfSampleRate, tuningFrequency, channelFrequency, 1.0f, decimation,
                           firstSampleIndex, lowPassTaps, numLowPassTaps, reinterpret_cast<const float2*>(input),
                           output, numElements, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrxFmDemodInt8(float rfSampleRate, float tuningFrequency, float channelFrequency,
                                           float frequencyDeviation, uint32_t decimation, size_t firstSampleIndex,
                                           const float* lowPassTaps, size_t numLowPassTaps, const int8_t* input,
                                           float* output, size_t numOutputs, int32_t cudaDevice,
                                           hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::chain_entry(gsdr::kModeFm, rfSampleRate, tuningFrequency, channelFrequency, frequencyDeviation,
                           decimation, firstSampleIndex, lowPassTaps, numLowPassTaps,
                           reinterpret_cast<const gsdr::Iq8*>(input), output, numOutputs, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrxAmDemodInt8(float rfSampleRate, float tuningFrequency, float channelFrequency,
                                           uint32_t decimation, size_t firstSampleIndex, const float* lowPassTaps,
                                           size_t numLowPassTaps, const int8_t* input, float* output,
                                           size_t numElements, int32_t cudaDevice,
                                           hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::chain_entry(gsdr::kModeAm, rfSampleRate, tuningFrequency, channelFrequency, 1.0f, decimation,
                           firstSampleIndex, lowPassTaps, numLowPassTaps, reinterpret_cast<const gsdr::Iq8*>(input),
                           output, numElements, cudaDevice, cudaStream);
}


GSDR_C_LINKAGE uint32_t gsdrNcoPhaseIncrement(float rfSampleRate, float tuningFrequency,
                                              float channelFrequency) GSDR_NO_EXCEPT {
  uint32_t inc = 0;
  (void)gsdr::nco_increment(rfSampleRate, tuningFrequency, channelFrequency, &inc);
  return inc;
}

GSDR_C_LINKAGE const char* gsdrVersion(void) GSDR_NO_EXCEPT { return "gsdr-mi355x 0.1.0 (gfx950)"; }

GSDR_C_LINKAGE hipError_t gsdrxFmDemodMulti(float rfSampleRate, float tuningFrequency, const float* channelFrequencies,
                                            const float* frequencyDeviations, uint32_t numChannels,
                                            uint32_t decimation, size_t firstSampleIndex, const float* lowPassTaps,
                                            size_t numLowPassTaps, int sampleFormat, const void* input, float* output,
                                            size_t numOutputs, int32_t cudaDevice,
                                            hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (sampleFormat == GSDRX_SAMPLES_CS8) {
    return gsdr::chain_multi_entry(gsdr::kModeFm, rfSampleRate, tuningFrequency, channelFrequencies,
                                   frequencyDeviations, numChannels, decimation, firstSampleIndex, lowPassTaps,
                                   numLowPassTaps, static_cast<const gsdr::Iq8*>(input), output, numOutputs,
                                   cudaDevice, cudaStream);
  }
  if (sampleFormat != GSDRX_SAMPLES_CF32) return hipErrorInvalidValue;
  return gsdr::chain_multi_entry(gsdr::kModeFm, rfSampleRate, tuningFrequency, channelFrequencies,
                                 frequencyDeviations, numChannels, decimation, firstSampleIndex, lowPassTaps,
                                 numLowPassTaps, static_cast<const float2*>(input), output, numOutputs, cudaDevice,
                                 cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrxAmDemodMulti(float rfSampleRate, float tuningFrequency, const float* channelFrequencies,
                                            uint32_t numChannels, uint32_t decimation, size_t firstSampleIndex,
                                            const float* lowPassTaps, size_t numLowPassTaps, int sampleFormat,
                                            const void* input, float* output, size_t numElements, int32_t cudaDevice,
                                            hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (sampleFormat == GSDRX_SAMPLES_CS8) {
    return gsdr::chain_multi_entry(gsdr::kModeAm, rfSampleRate, tuningFrequency, channelFrequencies, nullptr,
                                   numChannels, decimation, firstSampleIndex, lowPassTaps, numLowPassTaps,
                                   static_cast<const gsdr::Iq8*>(input), output, numElements, cudaDevice, cudaStream);
  }
  if (sampleFormat != GSDRX_SAMPLES_CF32) return hipErrorInvalidValue;
  return gsdr::chain_multi_entry(gsdr::kModeAm, rfSampleRate, tuningFrequency, channelFrequencies, nullptr,
                                 numChannels, decimation, firstSampleIndex, lowPassTaps, numLowPassTaps,
                                 static_cast<const float2*>(input), output, numElements, cudaDevice, cudaStream);
}
