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
}  // namespace gsdr
