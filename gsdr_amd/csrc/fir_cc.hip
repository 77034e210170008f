// gsdr-mi355x: gsdrFirCC (reference src/fir.cu:73-171, include/gsdr/fir.h:30-68).
#include <hip/hip_runtime.h>

#include "fir_entry.hpp"
#include "gsdr/fir.h"
#include "gsdr/gsdr_ext.h"

using gsdr::fir_entry;

GSDR_C_LINKAGE hipError_t gsdrFirCC(size_t decimation, const hipFloatComplex* taps, size_t tapCount,
                                    const hipFloatComplex* input, hipFloatComplex* output, size_t numOutputs,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float2, float2>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream,
                                   -1);
}
