// gsdr-mi355x: streaming continuity object (include/gsdr/stream.h).
//
// Host-side bookkeeping around the filter kernels. The reference has no equivalent: its callers
// re-supply the overlap themselves (include/gsdr/fm.h:26, fm.cu:202), one launch per chunk. Per Process
// call, ONE launch (round 4; the int8 matrix-core kernels since round 3):
//   * seam outputs (window starts in the history, ends in the new chunk) read their first samples from
//     the history buffer by offset, every other output straight from the caller's chunk;
//   * workgroup 0 of the same launch copies the samples the next output still needs (< one window) into
//     the spare history buffer (ping-pong).
// The launch runs the kernel one monolithic call would run, with the absolute index of output 0's first
// sample as firstSampleIndex, so the NCO phase and the per-output MAC order are those of that call: the
// outputs are bit-identical. Shapes without a one-launch kernel (runtime-decimation and generic kernels)
// keep the older plan: a gather launch (seam = history + chunk head, next history), then the seam and the
// main outputs as two filter calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>
#include <vector>

#include "gsdr/am.h"
#include "gsdr/fir.h"
#include "gsdr/fm.h"
#include "gsdr/gsdr_ext.h"
#include "gsdr/stream.h"
#include "launch.hpp"

struct gsdrxStream_t {
  int kind = GSDRX_STREAM_FIR;
  int format = GSDRX_SAMPLES_CF32;
  uint32_t D = 1;
  const float* taps = nullptr;
  size_t T = 0;
  size_t W = 0;  // samples one output needs
  float fs = 0.0f, tune = 0.0f;
  uint64_t n0 = 0;  // absolute index of stream sample 0
  int32_t device = 0;
  size_t sb = 8;  // bytes per input sample
  size_t ob = 8;  // bytes per output
  uint64_t consumed = 0;
  uint64_t next_out = 0;
  char* hist = nullptr;   // samples [next_out * D, consumed) (empty if next_out * D >= consumed)
  char* spare = nullptr;  // the other history buffer (ping-pong)
  char* seam = nullptr;   // history + chunk head for the seam outputs
  // channels of one RF input (gsdrxStreamCreateMulti; one channel for gsdrxStreamCreate): frequency and
  // deviation per channel, channel c's outputs at output + c * outputCapacity
  std::vector<float> chans, devs;
};

namespace gsdr {
// fir_int8.hip: gsdrxFirFCInt8 for outputs starting at absolute output index outputIndex
hipError_t fir_int8_at(uint64_t outputIndex, size_t decimation, const float* taps, size_t tapCount,
                       const int8_t* input, hipFloatComplex* output, size_t numOutputs, int32_t device,
                       hipStream_t stream);
hipError_t fir_int8_stream_step(uint64_t outputIndex, const float* taps, size_t tapCount, const int8_t* chunk,
                                uint64_t chunkLen, int64_t inOff, const int8_t* hist, uint64_t histLen, int8_t* histOut,
                                int64_t histFrom, uint64_t histN, hipFloatComplex* output, size_t numOutputs,
                                int32_t device, hipStream_t stream);
// the one-launch steps on the tiled kernels (fir_dispatch.hpp stream_step_tiled): fir.hip, fir_int8.hip, fm_am.hip
hipError_t fir_fc_stream_step(size_t decimation, const float* taps, size_t tapCount, const hipFloatComplex* chunk,
                              uint64_t chunkLen, int64_t inOff, const hipFloatComplex* hist, uint64_t histLen,
                              hipFloatComplex* histOut, int64_t histFrom, uint64_t histN, hipFloatComplex* output,
                              size_t numOutputs, int32_t device, hipStream_t stream);
hipError_t fir_int8_stream_step_tiled(size_t decimation, const float* taps, size_t tapCount, const int8_t* chunk,
                                      uint64_t chunkLen, int64_t inOff, const int8_t* hist, uint64_t histLen,
                                      int8_t* histOut, int64_t histFrom, uint64_t histN, hipFloatComplex* output,
                                      size_t numOutputs, int32_t device, hipStream_t stream);
hipError_t chain_stream_step_tiled(int mode, bool int8, float fs, float tune, float chan, float dev, uint32_t decimation,
                                   size_t firstSampleIndex, const float* taps, size_t tapCount, const void* chunk,
                                   uint64_t chunkLen, int64_t inOff, const void* hist, uint64_t histLen, void* histOut,
                                   int64_t histFrom, uint64_t histN, float* output, size_t numOutputs, int32_t device,
                                   hipStream_t stream);
hipError_t chain_multi_stream_step(int mode, float fs, float tune, const float* chans, const float* devs, uint32_t count,
                                   uint32_t decimation, size_t firstSampleIndex, const float* taps, size_t tapCount,
                                   const hipFloatComplex* chunk, uint64_t chunkLen, int64_t inOff,
                                   const hipFloatComplex* hist, uint64_t histLen, hipFloatComplex* histOut,
                                   int64_t histFrom, uint64_t histN, float* output, size_t outStride, size_t numOutputs,
                                   int32_t device, hipStream_t stream);
// fm_am.hip (mode 1 = FM, 2 = AM as in fir_engine.hpp)
hipError_t chain_int8_stream_step(int mode, float fs, float tune, float chan, float dev, size_t firstSampleIndex,
                                  const float* taps, size_t tapCount, const int8_t* chunk, uint64_t chunkLen,
                                  int64_t inOff, const int8_t* hist, uint64_t histLen, int8_t* histOut,
                                  int64_t histFrom, uint64_t histN, float* output, size_t numOutputs, int32_t device,
                                  hipStream_t stream);

namespace {

struct Plan {
  uint64_t n_seam, head, n_main, main_off, hist_after, m_mid, m_end;
};

Plan make_plan(uint32_t D, uint64_t W, uint64_t S, uint64_t m_next, uint64_t M) {
  Plan p{};
  const uint64_t S_new = S + M;
  uint64_t m_end = S_new >= W ? (S_new - W) / D + 1 : 0;  // first output whose window is incomplete
  m_end = std::max(m_end, m_next);
  const uint64_t m_mid = std::min(std::max(ceil_div<uint64_t>(S, D), m_next), m_end);
  p.m_mid = m_mid;
  p.m_end = m_end;
  p.n_seam = m_mid - m_next;
  p.head = p.n_seam ? (m_mid - 1) * D + W - S : 0;  // chunk samples the last seam output reads
  p.n_main = m_end - m_mid;
  p.main_off = p.n_main ? m_mid * D - S : 0;
  const uint64_t from = m_end * D;
  p.hist_after = S_new > from ? S_new - from : 0;
  return p;
}

hipError_t filter(const gsdrxStream_t& s, size_t c, const void* in, uint64_t first, void* out, size_t n,
                  hipStream_t st) {
  const bool i8 = s.format == GSDRX_SAMPLES_CS8;
  const float chan = s.chans[c], dev = s.devs[c];
  switch (s.kind) {
    case GSDRX_STREAM_FIR:
      // the default path of gsdrxFirFCInt8 told the output's absolute index: the decimation-4 matrix-core
      // kernel aligns its summation blocks to it, so chunks reproduce one call (fir_i8_mfma.hpp)
      return i8 ? fir_int8_at((first - s.n0) / s.D, s.D, s.taps, s.T, static_cast<const int8_t*>(in),
                              static_cast<hipFloatComplex*>(out), n, s.device, st)
                : gsdrFirFC(s.D, s.taps, s.T, static_cast<const hipFloatComplex*>(in),
                            static_cast<hipFloatComplex*>(out), n, s.device, st);
    case GSDRX_STREAM_FM:
      return i8 ? gsdrxFmDemodInt8(s.fs, s.tune, chan, dev, s.D, first, s.taps, s.T,
                                   static_cast<const int8_t*>(in), static_cast<float*>(out), n, s.device, st)
                : gsdrFmDemod(s.fs, s.tune, chan, dev, s.D, first, s.taps, s.T,
                              static_cast<const hipFloatComplex*>(in), static_cast<float*>(out), n, s.device, st);
    default:
      return i8 ? gsdrxAmDemodInt8(s.fs, s.tune, chan, s.D, first, s.taps, s.T,
                                   static_cast<const int8_t*>(in), static_cast<float*>(out), n, s.device, st)
                : gsdrAmDemod(s.fs, s.tune, chan, s.D, first, s.taps, s.T, static_cast<const hipFloatComplex*>(in),
                              static_cast<float*>(out), n, s.device, st);
  }
}

// The small device-to-device moves of one call (seam = history + chunk head, next history = the tail of
// old history + chunk), gathered into ONE launch: as separate hipMemcpyAsync calls each was a runtime blit
// launch of ~4-5 us, four of them per call, which is what a short float call paid (tools/float_stream_time.py).
// Segments never overlap (they write seam / spare and read hist / the chunk).
struct Gather {
  static constexpr int kMax = 4;
  struct Seg {
    char* dst;
    const char* src;
    uint64_t bytes;
  } seg[kMax];
  int n = 0;
  void add(void* dst, const void* src, size_t bytes) {
    if (bytes) seg[n++] = Seg{static_cast<char*>(dst), static_cast<const char*>(src), bytes};
  }
};

__global__ __launch_bounds__(256) void k_stream_gather(Gather g) {
  for (int i = 0; i < g.n; ++i) {
    const Gather::Seg sg = g.seg[i];
    // 4-byte moves when both ends and the length allow (every sample format is 2 or 8 bytes)
    if (((reinterpret_cast<uintptr_t>(sg.dst) | reinterpret_cast<uintptr_t>(sg.src) | sg.bytes) & 3u) == 0) {
      uint32_t* d = reinterpret_cast<uint32_t*>(sg.dst);
      const uint32_t* s = reinterpret_cast<const uint32_t*>(sg.src);
      for (uint64_t k = threadIdx.x + (uint64_t)blockIdx.x * blockDim.x; k < sg.bytes / 4; k += (uint64_t)gridDim.x * blockDim.x)
        d[k] = s[k];
    } else {
      for (uint64_t k = threadIdx.x + (uint64_t)blockIdx.x * blockDim.x; k < sg.bytes; k += (uint64_t)gridDim.x * blockDim.x)
        sg.dst[k] = sg.src[k];
    }
  }
}

hipError_t gather(const Gather& g, hipStream_t st) {
  if (g.n == 0) return hipSuccess;
  uint64_t most = 0;
  for (int i = 0; i < g.n; ++i) most = std::max<uint64_t>(most, g.seg[i].bytes);
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(64, ceil_div<uint64_t>(most, 256u * 4u));
  k_stream_gather<<<blocks, 256, 0, st>>>(g);
  return launch_status();
}

}  // namespace
}  // namespace gsdr

using gsdr::Plan;

GSDR_C_LINKAGE void gsdrxStreamPlan(uint32_t decimation, size_t window, uint64_t consumed, uint64_t nextOutput,
                                    size_t chunk, uint64_t plan[5]) GSDR_NO_EXCEPT {
  if (plan == nullptr) return;
  if (decimation == 0 || window == 0) {
    for (int i = 0; i < 5; ++i) plan[i] = 0;
    return;
  }
  const Plan p = gsdr::make_plan(decimation, window, consumed, nextOutput, chunk);
  plan[0] = p.n_seam;
  plan[1] = p.head;
  plan[2] = p.n_main;
  plan[3] = p.main_off;
  plan[4] = p.hist_after;
}

namespace gsdr {
namespace {
hipError_t create_stream(gsdrxStream* stream, int kind, int sampleFormat, uint32_t decimation, const float* taps,
                         size_t tapCount, float rfSampleRate, float tuningFrequency, const float* chans,
                         const float* devs, uint32_t count, size_t firstSampleIndex, int32_t cudaDevice) {
  if (stream == nullptr) return hipErrorInvalidValue;
  *stream = nullptr;
  if (decimation == 0 || tapCount == 0 || taps == nullptr || count == 0) return hipErrorInvalidValue;
  if (kind != GSDRX_STREAM_FIR && kind != GSDRX_STREAM_FM && kind != GSDRX_STREAM_AM) return hipErrorInvalidValue;
  if (sampleFormat != GSDRX_SAMPLES_CF32 && sampleFormat != GSDRX_SAMPLES_CS8) return hipErrorInvalidValue;
  gsdrxStream s = new (std::nothrow) gsdrxStream_t;
  if (s == nullptr) return hipErrorOutOfMemory;
  s->kind = kind;
  s->format = sampleFormat;
  s->D = decimation;
  s->taps = taps;
  s->T = tapCount;
  s->W = kind == GSDRX_STREAM_FM ? tapCount + decimation : tapCount;
  s->fs = rfSampleRate;
  s->tune = tuningFrequency;
  try {
    s->chans.assign(chans, chans + count);
    s->devs.assign(devs, devs + count);
  } catch (...) {
    delete s;
    return hipErrorOutOfMemory;
  }
  s->n0 = firstSampleIndex;
  s->device = cudaDevice;
  s->sb = sampleFormat == GSDRX_SAMPLES_CS8 ? 2 : 8;
  s->ob = kind == GSDRX_STREAM_FIR ? 8 : 4;
  DeviceScope scope(cudaDevice);
  hipError_t e = scope.status();
  const size_t hist_bytes = s->W * s->sb;  // history < W samples
  const size_t seam_bytes = 2 * s->W * s->sb;
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->hist), hist_bytes);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->spare), hist_bytes);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->seam), seam_bytes);
  if (e != hipSuccess) {
    (void)gsdrxStreamDestroy(s);
    return e;
  }
  *stream = s;
  return hipSuccess;
}
}  // namespace
}  // namespace gsdr

GSDR_C_LINKAGE hipError_t gsdrxStreamCreate(gsdrxStream* stream, int kind, int sampleFormat, uint32_t decimation,
                                            const float* taps, size_t tapCount, float rfSampleRate,
                                            float tuningFrequency, float channelFrequency, float frequencyDeviation,
                                            size_t firstSampleIndex, int32_t cudaDevice) GSDR_NO_EXCEPT {
  return gsdr::create_stream(stream, kind, sampleFormat, decimation, taps, tapCount, rfSampleRate, tuningFrequency,
                             &channelFrequency, &frequencyDeviation, 1, firstSampleIndex, cudaDevice);
}

GSDR_C_LINKAGE hipError_t gsdrxStreamCreateMulti(gsdrxStream* stream, int kind, int sampleFormat, uint32_t decimation,
                                                 const float* taps, size_t tapCount, float rfSampleRate,
                                                 float tuningFrequency, const float* channelFrequencies,
                                                 const float* frequencyDeviations, uint32_t numChannels,
                                                 size_t firstSampleIndex, int32_t cudaDevice) GSDR_NO_EXCEPT {
  if (stream != nullptr) *stream = nullptr;
  if (kind != GSDRX_STREAM_FM && kind != GSDRX_STREAM_AM) return hipErrorInvalidValue;
  if (numChannels == 0 || channelFrequencies == nullptr) return hipErrorInvalidValue;
  if (kind == GSDRX_STREAM_FM && frequencyDeviations == nullptr) return hipErrorInvalidValue;
  std::vector<float> ones;
  if (frequencyDeviations == nullptr) {  // AM: deviations unused
    try {
      ones.assign(numChannels, 1.0f);
    } catch (...) {
      return hipErrorOutOfMemory;
    }
    frequencyDeviations = ones.data();
  }
  return gsdr::create_stream(stream, kind, sampleFormat, decimation, taps, tapCount, rfSampleRate, tuningFrequency,
                             channelFrequencies, frequencyDeviations, numChannels, firstSampleIndex, cudaDevice);
}

GSDR_C_LINKAGE size_t gsdrxStreamOutputsFor(gsdrxStream s, size_t numInputSamples) GSDR_NO_EXCEPT {
  if (s == nullptr) return 0;
  const Plan p = gsdr::make_plan(s->D, s->W, s->consumed, s->next_out, numInputSamples);
  return p.n_seam + p.n_main;
}

GSDR_C_LINKAGE hipError_t gsdrxStreamProcess(gsdrxStream s, const void* input, size_t numInputSamples, void* output,
                                             size_t outputCapacity, size_t* numOutputsWritten,
                                             hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (numOutputsWritten) *numOutputsWritten = 0;
  if (s == nullptr) return hipErrorInvalidValue;
  if (numInputSamples == 0) return hipSuccess;
  if (input == nullptr) return hipErrorInvalidValue;
  const Plan p = gsdr::make_plan(s->D, s->W, s->consumed, s->next_out, numInputSamples);
  const size_t n_out = p.n_seam + p.n_main;
  if (n_out > outputCapacity || (n_out && output == nullptr)) return hipErrorInvalidValue;
  gsdr::DeviceScope scope(s->device);
  if (scope.status() != hipSuccess) return scope.status();
  const char* chunk = static_cast<const char*>(input);
  char* out = static_cast<char*>(output);
  const size_t C = s->chans.size();
  const size_t ostride = outputCapacity * s->ob;  // bytes between channels' output blocks
  const uint64_t S = s->consumed, h0 = s->next_out * s->D;
  const uint64_t h = S > h0 ? S - h0 : 0;
  hipError_t e = hipSuccess;
  if (n_out > 0) {
    // ONE launch (per channel, or per 16 channels on the grouped kernel) does the seam outputs (their samples
    // before the chunk read from the history buffer), the direct outputs and the next history copy: the int8
    // matrix-core kernels at decimation 4, the tiled kernels otherwise (the same kernels as one monolithic
    // call, tile for tile). Every channel reads the old history; only channel 0's launch writes the next one.
    const int64_t in_off = (int64_t)(s->next_out * s->D) - (int64_t)S;
    const int64_t from = (int64_t)(p.m_end * s->D) - (int64_t)S;
    const bool i8 = s->format == GSDRX_SAMPLES_CS8;
    const int mode = s->kind == GSDRX_STREAM_FM ? 1 : 2;
    e = hipErrorNotSupported;
    if (C > 1 && !i8) {
      e = gsdr::chain_multi_stream_step(mode, s->fs, s->tune, s->chans.data(), s->devs.data(), (uint32_t)C, s->D,
                                        s->n0 + h0, s->taps, s->T, reinterpret_cast<const hipFloatComplex*>(chunk),
                                        numInputSamples, in_off, reinterpret_cast<const hipFloatComplex*>(s->hist), h,
                                        reinterpret_cast<hipFloatComplex*>(s->spare), from, p.hist_after,
                                        reinterpret_cast<float*>(out), outputCapacity, n_out, s->device, cudaStream);
    }
    // otherwise one launch per channel; a shape without a one-launch step returns hipErrorNotSupported from
    // channel 0, before anything was launched, and the call takes the seam path below
    for (size_t c = 0; c < C && e == hipErrorNotSupported; ++c) {
      void* hout = c == 0 ? s->spare : nullptr;
      char* oc = out + c * ostride;
      hipError_t ec = hipErrorNotSupported;
      if (i8 && s->D == 4) {
        const int8_t* c8 = reinterpret_cast<const int8_t*>(chunk);
        const int8_t* h8 = reinterpret_cast<const int8_t*>(s->hist);
        int8_t* n8 = static_cast<int8_t*>(hout);
        if (s->kind == GSDRX_STREAM_FIR) {
          ec = gsdr::fir_int8_stream_step(s->next_out, s->taps, s->T, c8, numInputSamples, in_off, h8, h, n8, from,
                                          p.hist_after, reinterpret_cast<hipFloatComplex*>(oc), n_out, s->device,
                                          cudaStream);
        } else {
          ec = gsdr::chain_int8_stream_step(mode, s->fs, s->tune, s->chans[c], s->devs[c], s->n0 + h0, s->taps, s->T,
                                            c8, numInputSamples, in_off, h8, h, n8, from, p.hist_after,
                                            reinterpret_cast<float*>(oc), n_out, s->device, cudaStream);
        }
      }
      if (ec == hipErrorNotSupported) {
        if (s->kind == GSDRX_STREAM_FIR) {
          ec = i8 ? gsdr::fir_int8_stream_step_tiled(s->D, s->taps, s->T, reinterpret_cast<const int8_t*>(chunk),
                                                     numInputSamples, in_off, reinterpret_cast<const int8_t*>(s->hist), h,
                                                     static_cast<int8_t*>(hout), from, p.hist_after,
                                                     reinterpret_cast<hipFloatComplex*>(oc), n_out, s->device, cudaStream)
                  : gsdr::fir_fc_stream_step(s->D, s->taps, s->T, reinterpret_cast<const hipFloatComplex*>(chunk),
                                             numInputSamples, in_off, reinterpret_cast<const hipFloatComplex*>(s->hist), h,
                                             static_cast<hipFloatComplex*>(hout), from, p.hist_after,
                                             reinterpret_cast<hipFloatComplex*>(oc), n_out, s->device, cudaStream);
        } else {
          ec = gsdr::chain_stream_step_tiled(mode, i8, s->fs, s->tune, s->chans[c], s->devs[c], s->D, s->n0 + h0,
                                             s->taps, s->T, chunk, numInputSamples, in_off, s->hist, h, hout, from,
                                             p.hist_after, reinterpret_cast<float*>(oc), n_out, s->device, cudaStream);
        }
      }
      if (ec == hipErrorNotSupported && c == 0) break;
      // a failure after channel 0 leaves channels 0..c-1 written and the stream unchanged (stream.h: the
      // outputs of a failed call are unspecified)
      if (ec != hipSuccess) {
        e = ec == hipErrorNotSupported ? hipErrorUnknown : ec;  // (one shape for every channel: cannot happen)
        break;
      }
      if (c + 1 == C) e = hipSuccess;
    }
    if (e == hipSuccess) {
      std::swap(s->hist, s->spare);
      s->consumed += numInputSamples;
      s->next_out = p.m_end;
      if (numOutputsWritten) *numOutputsWritten = n_out;
      return hipSuccess;
    }
    if (e != hipErrorNotSupported) return e;
    e = hipSuccess;  // not this shape: the seam path below
  }
  // every small move of the call (seam assembly, next history) in one launch ahead of the filters
  gsdr::Gather g;
  if (p.n_seam) {
    g.add(s->seam, s->hist, h * s->sb);
    g.add(s->seam + h * s->sb, chunk, p.head * s->sb);
  }
  if (p.hist_after) {
    const uint64_t from = p.m_end * s->D, S_new = S + numInputSamples;
    uint64_t done = 0;
    if (from < S) {  // part of the new history is still in the old one
      done = S - from;
      g.add(s->spare, s->hist + (from - h0) * s->sb, done * s->sb);
    }
    const uint64_t c0 = from > S ? from - S : 0;
    g.add(s->spare + done * s->sb, chunk + c0 * s->sb, (S_new - S - c0) * s->sb);
  }
  e = gsdr::gather(g, cudaStream);
  for (size_t c = 0; c < C && e == hipSuccess; ++c) {
    char* oc = out + c * ostride;
    if (p.n_seam) e = gsdr::filter(*s, c, s->seam, s->n0 + h0, oc, p.n_seam, cudaStream);
    if (e == hipSuccess && p.n_main) {
      e = gsdr::filter(*s, c, chunk + p.main_off * s->sb, s->n0 + p.m_mid * s->D, oc + p.n_seam * s->ob, p.n_main,
                       cudaStream);
    }
  }
  if (e == hipSuccess && p.hist_after) std::swap(s->hist, s->spare);
  if (e != hipSuccess) return e;
  s->consumed += numInputSamples;
  s->next_out = p.m_end;
  if (numOutputsWritten) *numOutputsWritten = n_out;
  return hipSuccess;
}

GSDR_C_LINKAGE hipError_t gsdrxStreamDestroy(gsdrxStream s) GSDR_NO_EXCEPT {
  if (s == nullptr) return hipSuccess;
  hipError_t e = hipSuccess;
  {
    gsdr::DeviceScope scope(s->device);
    if (scope.status() == hipSuccess) {
      for (char* b : {s->hist, s->spare, s->seam}) {
        if (b) {
          const hipError_t f = hipFree(b);
          if (e == hipSuccess) e = f;
        }
      }
    } else {
      e = scope.status();
    }
  }
  delete s;
  return e;
}
