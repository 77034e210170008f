// gsdr-mi355x: gsdrFirFC / gsdrFirFF / gsdrFirCC / gsdrFirCF (reference src/fir.cu:73-171,
// include/gsdr/fir.h:30-68) and the kernel dispatch shared with the FM / AM chains.
#include <hip/hip_runtime.h>

#include "fir_dispatch.hpp"
#include "gsdr/fir.h"
#include "gsdr/gsdr_ext.h"
#include "launch.hpp"

namespace gsdr {

template <class TapT, class InT>
static hipError_t fir_entry(size_t decimation, const TapT* taps, size_t tapCount, const InT* input,
                            typename Product<TapT, InT>::type* output, size_t numOutputs, int32_t device,
                            hipStream_t stream, int variant) {
  using OutT = typename Product<TapT, InT>::type;
  if (numOutputs == 0) return hipSuccess;
  if (decimation == 0 || output == nullptr) return hipErrorInvalidValue;
  GSDR_ON_DEVICE(device, ([&]() -> hipError_t {
                   if (tapCount == 0) {
                     // reference: the tap loop never runs, every output is zero<OUT_T>() (fir.cu:43-46)
                     const hipError_t st = hipMemsetAsync(output, 0, numOutputs * sizeof(OutT), stream);
                     return st != hipSuccess ? st : launch_status();
                   }
                   if (taps == nullptr || input == nullptr) return hipErrorInvalidValue;
                   FirJob job;
                   job.in = input;
                   job.taps = taps;
                   job.out = output;
                   job.D = decimation;
                   job.T = tapCount;
                   job.N = numOutputs;
                   job.L = (numOutputs - 1) * decimation + tapCount;
                   job.mode = kModeFir;
                   job.variant = variant;
                   return launch_fir<TapT, InT, kModeFir>(job, stream);
                 })());
}

}  // namespace gsdr

using gsdr::fir_entry;

GSDR_C_LINKAGE hipError_t gsdrFirFC(size_t decimation, const float* taps, size_t tapCount,
                                    const hipFloatComplex* input, hipFloatComplex* output, size_t numOutputs,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, float2>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream, -1);
}

GSDR_C_LINKAGE hipError_t gsdrFirFF(size_t decimation, const float* taps, size_t tapCount, const float* input,
                                    float* output, size_t numOutputs, int32_t cudaDevice,
                                    hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, float>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream, -1);
}

GSDR_C_LINKAGE hipError_t gsdrFirCC(size_t decimation, const hipFloatComplex* taps, size_t tapCount,
                                    const hipFloatComplex* input, hipFloatComplex* output, size_t numOutputs,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float2, float2>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream,
                                   -1);
}

GSDR_C_LINKAGE hipError_t gsdrFirCF(size_t decimation, const hipFloatComplex* taps, size_t tapCount,
                                    const float* input, hipFloatComplex* output, size_t numOutputs,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float2, float>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream, -1);
}

GSDR_C_LINKAGE hipError_t gsdrxFirFCVariant(int variant, size_t decimation, const float* taps, size_t tapCount,
                                            const hipFloatComplex* input, hipFloatComplex* output,
                                            size_t numOutputs, int32_t cudaDevice,
                                            hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, float2>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream,
                                  variant);
}
