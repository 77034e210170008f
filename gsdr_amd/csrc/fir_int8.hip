// gsdr-mi355x: gsdrxFirFCInt8 / gsdrxFirFCInt8Variant: gsdrFirFC from interleaved int8 I/Q (gsdr_ext.h).
#include <hip/hip_runtime.h>

#include "fir_entry.hpp"
#include "gsdr/fir.h"
#include "gsdr/gsdr_ext.h"

using gsdr::fir_entry;

GSDR_C_LINKAGE hipError_t gsdrxFirFCInt8(size_t decimation, const float* taps, size_t tapCount, const int8_t* input,
                                         hipFloatComplex* output, size_t numOutputs, int32_t cudaDevice,
                                         hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, gsdr::Iq8>(decimation, taps, tapCount, reinterpret_cast<const gsdr::Iq8*>(input), output,
                                     numOutputs, cudaDevice, cudaStream, -1);
}

GSDR_C_LINKAGE hipError_t gsdrxFirFCInt8Variant(int variant, size_t decimation, const float* taps, size_t tapCount,
                                                const int8_t* input, hipFloatComplex* output, size_t numOutputs,
                                                int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, gsdr::Iq8>(decimation, taps, tapCount, reinterpret_cast<const gsdr::Iq8*>(input), output,
                                     numOutputs, cudaDevice, cudaStream, variant < 0 ? -1 : variant);
}

namespace gsdr {
// The streaming object's int8 FIR (stream.hip): gsdrxFirFCInt8 for outputs whose absolute index (counted
// from the stream's first output) starts at outputIndex. The decimation-4 matrix-core kernel aligns its
// 16-output blocks to that index, so chunked calls reproduce one call bit for bit (fir_i8_mfma.hpp).
hipError_t fir_int8_at(uint64_t outputIndex, size_t decimation, const float* taps, size_t tapCount,
                       const int8_t* input, hipFloatComplex* output, size_t numOutputs, int32_t device,
                       hipStream_t stream) {
  return fir_entry<float, Iq8>(decimation, taps, tapCount, reinterpret_cast<const Iq8*>(input), output, numOutputs,
                               device, stream, -1, (uint32_t)(outputIndex & 15u));
}

// The streaming object's one-launch step at decimation 4 (stream.hip): outputs [outputIndex, + N) of the
// stream, output 0's window at chunk offset inOff (negative: it starts in the history buffer), the next
// history copied by the same launch. Returns hipErrorNotSupported (nothing launched) for shapes that do
// not take the matrix-core kernel; the stream then takes its seam path.
hipError_t fir_int8_stream_step(uint64_t outputIndex, const float* taps, size_t tapCount, const int8_t* chunk,
                                uint64_t chunkLen, int64_t inOff, const int8_t* hist, uint64_t histLen, int8_t* histOut,
                                int64_t histFrom, uint64_t histN, hipFloatComplex* output, size_t numOutputs,
                                int32_t device, hipStream_t stream) {
  if (numOutputs == 0 || tapCount == 0 || taps == nullptr || tapCount > (size_t)I8Mfma<4, 8>::MAXT ||
      (reinterpret_cast<uintptr_t>(output) % 8) != 0) {
    return hipErrorNotSupported;
  }
  FirJob job;
  job.in = chunk;
  job.taps = taps;
  job.out = output;
  job.D = 4;
  job.T = tapCount;
  job.N = numOutputs;
  job.L = chunkLen;
  job.mode = kModeFir;
  job.out_phase = (uint32_t)(outputIndex & 15u);
  job.in_off = inOff;
  job.hist = hist;
  job.hist_len = histLen;
  job.hist_out = histOut;
  job.hist_from = histFrom;
  job.hist_n = histN;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  return launch_i8_mfma<4, 3>(job, stream);
}

// The same on the tiled kernels (decimations other than 4, or tap counts the matrix-core kernel does not
// take): the exact path, as the monolithic call runs for those shapes (stream_step_tiled).
hipError_t fir_int8_stream_step_tiled(size_t decimation, const float* taps, size_t tapCount, const int8_t* chunk,
                                      uint64_t chunkLen, int64_t inOff, const int8_t* hist, uint64_t histLen,
                                      int8_t* histOut, int64_t histFrom, uint64_t histN, hipFloatComplex* output,
                                      size_t numOutputs, int32_t device, hipStream_t stream) {
  FirJob job;
  job.in = chunk;
  job.taps = taps;
  job.out = output;
  job.D = decimation;
  job.T = tapCount;
  job.N = numOutputs;
  job.L = chunkLen;
  job.mode = kModeFir;
  job.in_off = inOff;
  job.hist = hist;
  job.hist_len = histLen;
  job.hist_out = histOut;
  job.hist_from = histFrom;
  job.hist_n = histN;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  return stream_step_tiled<Iq8, kModeFir>(job, stream);
}
}  // namespace gsdr
