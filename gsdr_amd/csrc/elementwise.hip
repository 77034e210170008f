// gsdr-mi355x: element-wise arithmetic, tone generators and int8 conversion.
//   gsdrAddConst{FF,CC,CF,FC}  replace reference src/add_const.cu:20-28, 44-95
//   gsdrAddToMagnitude         replaces reference src/add_const.cu:30-42, 97-107
//   gsdrMultiply{CC,FF,CF}     replace reference src/multiply.cu:20-27, 29-70
//   gsdrAbs                    replaces reference src/magnitude.cu:30-36, 47-51
//   gsdrCosine{C,F}            replace reference src/trig.cu:20-75
//   gsdrInt8ToNormFloat        replaces reference src/conversion.cu:20-35
// All are HBM-bound maps. One templated kernel: each thread owns kPerThread consecutive elements,
// moves them with the widest aligned loads/stores (16 B where the element block allows), and a
// thread whose block runs past n (or any misaligned pointer) falls back to one element at a time.
#include <hip/hip_runtime.h>

#include "gsdr/arithmetic.h"
#include "gsdr/conversion.h"
#include "gsdr/trig.h"
#include "launch.hpp"

namespace gsdr {

constexpr int kEwBlock = 256;
constexpr int kPerThread = 8;

struct NoInput {};

// Result semantics follow the reference's operators (src/cuComplexOperatorOverloads.cuh:25-56);
// the library builds with -ffp-contract=off, so every product below is rounded as written.
struct OpAddFF {
  float c;
  __device__ float operator()(uint64_t, float x, NoInput) const { return c + x; }
};
struct OpAddCC {
  float2 c;
  __device__ float2 operator()(uint64_t, float2 x, NoInput) const { return make_float2(c.x + x.x, c.y + x.y); }
};
struct OpAddCF {  // complex input + real constant: operator+(float, cuComplex) = c + r, real part only
  float c;
  __device__ float2 operator()(uint64_t, float2 x, NoInput) const { return make_float2(x.x + c, x.y); }
};
struct OpAddFC {  // real input + complex constant: operator+(cuComplex, float)
  float2 c;
  __device__ float2 operator()(uint64_t, float x, NoInput) const { return make_float2(c.x + x, c.y); }
};
struct OpAddToMagnitude {
  float c;
  __device__ float2 operator()(uint64_t, float2 x, NoInput) const {
    const float m = hypotf(x.x, x.y);
    const float nx = x.x / m, ny = x.y / m;  // operator/(cuComplex, float)
    const float len = c + m;
    return make_float2(nx * len, ny * len);  // operator*(float, cuComplex)
  }
};
struct OpMulCC {  // cuCmulf
  __device__ float2 operator()(uint64_t, float2 a, float2 b) const {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
  }
};
struct OpMulFF {
  __device__ float operator()(uint64_t, float a, float b) const { return a * b; }
};
struct OpMulCF {
  __device__ float2 operator()(uint64_t, float2 a, float b) const { return make_float2(a.x * b, a.y * b); }
};
struct OpAbs {
  __device__ float operator()(uint64_t, float x, NoInput) const { return fabsf(x); }
};
struct OpInt8 {
  __device__ float operator()(uint64_t, int8_t x, NoInput) const { return fmaxf(-1.0f, (float)x / 127.0f); }
};
struct OpCosineC {
  float m, phi;
  __device__ float2 operator()(uint64_t k, NoInput, NoInput) const {
    const float th = fmaf((float)(uint32_t)k, m, phi);
    float s, c;
    sincosf(th, &s, &c);
    return make_float2(c, s);
  }
};
struct OpCosineF {
  float m, phi;
  __device__ float operator()(uint64_t k, NoInput, NoInput) const { return cosf(fmaf((float)(uint32_t)k, m, phi)); }
};

// kPerThread elements from p (aligned to min(16, block bytes) when VEC) into registers
template <class T>
__device__ __forceinline__ void load_block(const T* __restrict__ p, T (&v)[kPerThread]) {
  constexpr size_t B = sizeof(T) * kPerThread;
  constexpr size_t A = B >= 16 ? 16 : B;
  __builtin_memcpy(v, __builtin_assume_aligned(p, A), B);
}
__device__ __forceinline__ void load_block(const NoInput*, NoInput (&)[kPerThread]) {}

template <class T>
__device__ __forceinline__ void store_block(T* __restrict__ p, const T (&v)[kPerThread]) {
  constexpr size_t B = sizeof(T) * kPerThread;
  constexpr size_t A = B >= 16 ? 16 : B;
  __builtin_memcpy(__builtin_assume_aligned(p, A), v, B);
}

template <class T>
__device__ __forceinline__ T load_one(const T* p, uint64_t k) {
  return p[k];
}
__device__ __forceinline__ NoInput load_one(const NoInput*, uint64_t) { return {}; }

template <class In1, class In2, class Out, class Op, bool VEC>
__global__ __launch_bounds__(kEwBlock) void k_elementwise(const In1* __restrict__ a, const In2* __restrict__ b,
                                                          Out* __restrict__ out, uint64_t n, Op op) {
  const uint64_t k0 = ((uint64_t)blockIdx.x * kEwBlock + threadIdx.x) * kPerThread;
  if (k0 >= n) return;
  if (VEC && k0 + kPerThread <= n) {
    In1 va[kPerThread];
    In2 vb[kPerThread];
    Out r[kPerThread];
    load_block(a + k0, va);
    load_block(b + k0, vb);
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) r[e] = op(k0 + e, va[e], vb[e]);
    store_block(out + k0, r);
  } else {
    for (int e = 0; e < kPerThread && k0 + e < n; ++e) out[k0 + e] = op(k0 + e, load_one(a, k0 + e), load_one(b, k0 + e));
  }
}

template <class T>
static bool block_aligned(const T* p) {
  if constexpr (std::is_same<T, NoInput>::value) {
    return true;
  } else {
    constexpr size_t B = sizeof(T) * kPerThread;
    constexpr size_t A = B >= 16 ? 16 : B;
    return (reinterpret_cast<uintptr_t>(p) % A) == 0;
  }
}

template <class In1, class In2, class Out, class Op>
static hipError_t ew_entry(const In1* a, const In2* b, Out* out, size_t n, Op op, int32_t device, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (out == nullptr) return hipErrorInvalidValue;
  if (!std::is_same<In1, NoInput>::value && a == nullptr) return hipErrorInvalidValue;
  if (!std::is_same<In2, NoInput>::value && b == nullptr) return hipErrorInvalidValue;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  const uint64_t blocks = ceil_div<uint64_t>(n, (uint64_t)kEwBlock * kPerThread);
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  if (block_aligned(a) && block_aligned(b) && block_aligned(out)) {
    k_elementwise<In1, In2, Out, Op, true><<<dim3((uint32_t)blocks), dim3(kEwBlock), 0, stream>>>(a, b, out, n, op);
  } else {
    k_elementwise<In1, In2, Out, Op, false><<<dim3((uint32_t)blocks), dim3(kEwBlock), 0, stream>>>(a, b, out, n, op);
  }
  return launch_status();
}

inline float2 f2(hipFloatComplex c) { return make_float2(c.x, c.y); }
inline const float2* f2p(const hipFloatComplex* p) { return reinterpret_cast<const float2*>(p); }
inline float2* f2p(hipFloatComplex* p) { return reinterpret_cast<float2*>(p); }
constexpr const NoInput* kNone = nullptr;

// phase step per element, as the reference computes it on the host (src/trig.cu:55, 70)
inline float ramp_step(float phiBegin, float phiEnd, size_t n) {
  return static_cast<float>((phiEnd - phiBegin) / static_cast<double>(n));
}

}  // namespace gsdr

using namespace gsdr;

GSDR_C_LINKAGE hipError_t gsdrAddConstFF(const float* input, float addConst, float* output, size_t numElements,
                                         int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(input, kNone, output, numElements, OpAddFF{addConst}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrAddConstCC(const hipFloatComplex* input, hipFloatComplex addConst,
                                         hipFloatComplex* output, size_t numElements, int32_t cudaDevice,
                                         hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(f2p(input), kNone, f2p(output), numElements, OpAddCC{f2(addConst)}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrAddConstCF(const hipFloatComplex* input, float addConst, hipFloatComplex* output,
                                         size_t numElements, int32_t cudaDevice,
                                         hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(f2p(input), kNone, f2p(output), numElements, OpAddCF{addConst}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrAddConstFC(const float* input, hipFloatComplex addConst, hipFloatComplex* output,
                                         size_t numElements, int32_t cudaDevice,
                                         hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(input, kNone, f2p(output), numElements, OpAddFC{f2(addConst)}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrMultiplyCC(const hipFloatComplex* in1, const hipFloatComplex* in2,
                                         hipFloatComplex* out, size_t numElements, int32_t cudaDevice,
                                         hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(f2p(in1), f2p(in2), f2p(out), numElements, OpMulCC{}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrMultiplyFF(const float* in1, const float* in2, float* out, size_t numElements,
                                         int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(in1, in2, out, numElements, OpMulFF{}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrMultiplyCF(const hipFloatComplex* in1, const float* in2, hipFloatComplex* out,
                                         size_t numElements, int32_t cudaDevice,
                                         hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(f2p(in1), in2, f2p(out), numElements, OpMulCF{}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrAddToMagnitude(const hipFloatComplex* input, float addToMagnitude,
                                             hipFloatComplex* output, size_t numElements, int32_t cudaDevice,
                                             hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(f2p(input), kNone, f2p(output), numElements, OpAddToMagnitude{addToMagnitude}, cudaDevice,
                  cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrAbs(const float* in, float* out, size_t numElements, int32_t cudaDevice,
                                  hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(in, kNone, out, numElements, OpAbs{}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrInt8ToNormFloat(const int8_t* input, float* output, size_t numElements,
                                              int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return ew_entry(input, kNone, output, numElements, OpInt8{}, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrCosineC(float phiBegin, float phiEnd, hipFloatComplex* output, size_t numElements,
                                      int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (numElements == 0) return hipSuccess;
  return ew_entry(kNone, kNone, f2p(output), numElements, OpCosineC{ramp_step(phiBegin, phiEnd, numElements), phiBegin},
                  cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrCosineF(float phiBegin, float phiEnd, float* output, size_t numElements,
                                      int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (numElements == 0) return hipSuccess;
  return ew_entry(kNone, kNone, output, numElements, OpCosineF{ramp_step(phiBegin, phiEnd, numElements), phiBegin},
                  cudaDevice, cudaStream);
}
