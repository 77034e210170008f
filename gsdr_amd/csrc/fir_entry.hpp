// gsdr-mi355x: the common body of the gsdrFir* entry points (reference src/fir.cu:73-171): argument
// checks, the T = 0 case and the kernel dispatch. Each sample-type pair is instantiated in its own
// translation unit (fir.hip: FC, fir_ff.hip, fir_cc.hip, fir_cf.hip, fir_int8.hip) so they build in
// parallel.
#pragma once

#include <hip/hip_runtime.h>

#include "fir_dispatch.hpp"
#include "launch.hpp"

namespace gsdr {

template <class TapT, class InT>
inline hipError_t fir_entry(size_t decimation, const TapT* taps, size_t tapCount, const InT* input,
                            typename Product<TapT, InT>::type* output, size_t numOutputs, int32_t device,
                            hipStream_t stream, int variant, uint32_t out_phase = 0) {
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
                   job.out_phase = out_phase;
                   return launch_fir<TapT, InT, kModeFir>(job, stream);
                 })());
}

}  // namespace gsdr
