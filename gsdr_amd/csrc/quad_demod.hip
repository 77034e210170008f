// gsdr-mi355x: stand-alone discriminators and magnitude.
//   gsdrQuadFmDemod  replaces reference src/quad_demod.cu:23-37, 56-66
//   gsdrQuadAmDemod  replaces reference src/quad_demod.cu:39-54, 68-74
//   gsdrMagnitude    replaces reference src/magnitude.cu:20-28, 39-45
// HBM-bound maps: each thread owns 4 consecutive outputs, reads its samples with 16-byte loads and
// writes one 16-byte store (the reference uses 32-thread blocks, one output per thread).
#include <hip/hip_runtime.h>

#include "fir_engine.hpp"
#include "gsdr/arithmetic.h"
#include "gsdr/quad_demod.h"
#include "launch.hpp"

namespace gsdr {

constexpr int kMapBlock = 256;
constexpr int kPerThread = 4;

enum MapOp : int { kOpQuadFm = 0, kOpQuadAm = 1, kOpMagnitude = 2 };

template <int OP>
__device__ __forceinline__ float map_one(const float2* __restrict__ in, uint64_t k, float gain) {
  if constexpr (OP == kOpQuadFm) {
    return fm_disc(in[k], in[k + 1], gain);
  } else if constexpr (OP == kOpQuadAm) {
    return am_env(in[k]);
  } else {
    const float2 v = in[k];
    return hypotf(v.x, v.y);
  }
}

// VEC: input and output 16-byte aligned. Threads whose 4 outputs are not all in range fall back to
// one output at a time.
template <int OP, bool VEC>
__global__ __launch_bounds__(kMapBlock) void k_map(const float2* __restrict__ in, float* __restrict__ out,
                                                   uint64_t n, float gain) {
  const uint64_t k0 = ((uint64_t)blockIdx.x * kMapBlock + threadIdx.x) * kPerThread;
  if (k0 >= n) return;
  if (VEC && k0 + kPerThread <= n) {
    const float4* src = reinterpret_cast<const float4*>(in + k0);
    const float4 a = src[0];
    const float4 b = src[1];
    float4 r;
    if constexpr (OP == kOpQuadFm) {
      const float2 x4 = in[k0 + 4];  // one sample past this thread's group (an L1/L2 hit)
      r.x = fm_disc(make_float2(a.x, a.y), make_float2(a.z, a.w), gain);
      r.y = fm_disc(make_float2(a.z, a.w), make_float2(b.x, b.y), gain);
      r.z = fm_disc(make_float2(b.x, b.y), make_float2(b.z, b.w), gain);
      r.w = fm_disc(make_float2(b.z, b.w), x4, gain);
    } else if constexpr (OP == kOpQuadAm) {
      r.x = am_env(make_float2(a.x, a.y));
      r.y = am_env(make_float2(a.z, a.w));
      r.z = am_env(make_float2(b.x, b.y));
      r.w = am_env(make_float2(b.z, b.w));
    } else {
      r.x = hypotf(a.x, a.y);
      r.y = hypotf(a.z, a.w);
      r.z = hypotf(b.x, b.y);
      r.w = hypotf(b.z, b.w);
    }
    *reinterpret_cast<float4*>(out + k0) = r;
  } else {
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
      if (k0 + e < n) out[k0 + e] = map_one<OP>(in, k0 + e, gain);
    }
  }
}

template <int OP>
static hipError_t map_entry(const hipFloatComplex* input, float* output, float gain, size_t n, int32_t device,
                            hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (input == nullptr || output == nullptr) return hipErrorInvalidValue;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  const uint64_t blocks = ceil_div<uint64_t>(n, (uint64_t)kMapBlock * kPerThread);
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  if (aligned16(input) && aligned16(output)) {
    k_map<OP, true><<<dim3((uint32_t)blocks), dim3(kMapBlock), 0, stream>>>(input, output, n, gain);
  } else {
    k_map<OP, false><<<dim3((uint32_t)blocks), dim3(kMapBlock), 0, stream>>>(input, output, n, gain);
  }
  return launch_status();
}

}  // namespace gsdr

GSDR_C_LINKAGE hipError_t gsdrQuadFmDemod(const hipFloatComplex* input, float* output, float gain,
                                          size_t numOutputElements, int32_t cudaDevice,
                                          hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::map_entry<gsdr::kOpQuadFm>(input, output, gain, numOutputElements, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQuadAmDemod(const hipFloatComplex* input, float* output, size_t numOutputElements,
                                          int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::map_entry<gsdr::kOpQuadAm>(input, output, 0.0f, numOutputElements, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrMagnitude(const hipFloatComplex* in, float* out, size_t numElements,
                                        int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::map_entry<gsdr::kOpMagnitude>(in, out, 0.0f, numElements, cudaDevice, cudaStream);
}
