// gsdr-mi355x: element-wise arithmetic, tone generators and int8 conversion.
//   gsdrAddConst{FF,CC,CF,FC}  replace reference src/add_const.cu:20-28, 44-95
//   gsdrAddToMagnitude         replaces reference src/add_const.cu:30-42, 97-107
//   gsdrMultiply{CC,FF,CF}     replace reference src/multiply.cu:20-27, 29-70
//   gsdrAbs                    replaces reference src/magnitude.cu:30-36, 47-51
//   gsdrCosine{C,F}            replace reference src/trig.cu:20-75
//   gsdrInt8ToNormFloat        replaces reference src/conversion.cu:20-35
// All are HBM-bound maps. One templated kernel: a block owns kEwBlock * kPerThread consecutive
// elements, moved as 16-byte groups of the widest stream with lanes on consecutive groups (coalesced
// 1 KB per wave instruction); the last, partial block (or any misaligned pointer) goes one element at
// a time with the same element-to-thread mapping.
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

template <class T>
constexpr size_t size_of() {
  if constexpr (std::is_same<T, NoInput>::value) {
    return 1;
  } else {
    return sizeof(T);
  }
}

// Elements per group: one 16-byte vector of the widest type the map touches. Each thread owns
// kPerThread / kGroup(...) groups, and group slot s of lane t is group s * kEwBlock + t of the block,
// so every load/store instruction of a wave covers one contiguous 1 KB run of the widest stream (a
// thread owning consecutive elements would put its lanes 64-128 B apart and touch 8x the cache lines
// per instruction; measured 42 -> 24 us for a 128 MB write-only map).
template <class In1, class In2, class Out>
constexpr int kGroup() {
  constexpr size_t w = size_of<In1>() > size_of<In2>() ? (size_of<In1>() > size_of<Out>() ? size_of<In1>() : size_of<Out>())
                                                       : (size_of<In2>() > size_of<Out>() ? size_of<In2>() : size_of<Out>());
  return (int)(16 / w);
}

template <class T, int G>
__device__ __forceinline__ void load_group(const T* __restrict__ p, uint64_t k, T (&v)[G]) {
  if constexpr (!std::is_same<T, NoInput>::value) {
    __builtin_memcpy(v, __builtin_assume_aligned(p + k, sizeof(T) * G), sizeof(T) * G);
  }
}

template <class T, int G>
__device__ __forceinline__ void store_group(T* __restrict__ p, const T (&v)[G]) {
  __builtin_memcpy(__builtin_assume_aligned(p, sizeof(T) * G), v, sizeof(T) * G);
}

template <class T>
__device__ __forceinline__ T load_one(const T* p, uint64_t k) {
  return p[k];
}
__device__ __forceinline__ NoInput load_one(const NoInput*, uint64_t) { return {}; }

template <class In1, class In2, class Out, class Op, bool VEC>
__global__ __launch_bounds__(kEwBlock) void k_elementwise(const In1* __restrict__ a, const In2* __restrict__ b,
                                                          Out* __restrict__ out, uint64_t n, Op op) {
  constexpr int G = kGroup<In1, In2, Out>();
  constexpr int S = kPerThread / G;
  static_assert(S * G == kPerThread, "group must divide the per-thread element count");
  const uint64_t base = (uint64_t)blockIdx.x * kEwBlock * kPerThread;
  if (VEC && base + (uint64_t)kEwBlock * kPerThread <= n) {
    In1 va[S][G];
    In2 vb[S][G];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint64_t k = base + (uint64_t)(s * kEwBlock + threadIdx.x) * G;
      load_group<In1, G>(a, k, va[s]);
      load_group<In2, G>(b, k, vb[s]);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint64_t k = base + (uint64_t)(s * kEwBlock + threadIdx.x) * G;
      Out r[G];
#pragma unroll
      for (int e = 0; e < G; ++e) r[e] = op(k + e, va[s][e], vb[s][e]);
      store_group<Out, G>(out + k, r);
    }
  } else {
    for (int s = 0; s < S; ++s) {
      const uint64_t k = base + (uint64_t)(s * kEwBlock + threadIdx.x) * G;
      for (int e = 0; e < G && k + e < n; ++e) out[k + e] = op(k + e, load_one(a, k + e), load_one(b, k + e));
    }
  }
}

template <class T, int G>
static bool group_aligned(const T* p) {
  if constexpr (std::is_same<T, NoInput>::value) {
    return true;
  } else {
    return (reinterpret_cast<uintptr_t>(p) % (sizeof(T) * G)) == 0;
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
  constexpr int G = kGroup<In1, In2, Out>();
  if (group_aligned<In1, G>(a) && group_aligned<In2, G>(b) && group_aligned<Out, G>(out)) {
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
