// gsdr-mi355x: QPSK modulate / demodulate, single, 4x and consolidated ("templated") layouts.
// Replaces reference src/qpsk.cu (kernels :26-364, wrappers :366-484, :588-665; header qpsk.h:116-239).
//
// Mapping (qpsk.cu:121-145, 239-254): 2-bit symbol s, LSB pair first in each byte;
//   s -> ((s & 1) ? -a : a, (s & 2) ? -a : a);  demod: s = (re >= 0 ? 0 : 1) | (im >= 0 ? 0 : 2).
//
// Layout on MI355X: one thread owns 16 symbols = 4 packed bytes = 128 bytes of IQ, so demodulation
// assembles whole bytes in registers and writes them once -- no byte atomics (the reference's
// atomicCAS(uint8_t*) loop does not compile, qpsk.cu:92-98). The last, partially used byte keeps its
// unused high bit pairs (read-modify-write by the single thread that owns it).
#include <hip/hip_runtime.h>

#include "gsdr/qpsk.h"
#include "launch.hpp"

namespace gsdr {

constexpr int kQBlock = 256;
constexpr int kQSym = 16;  // symbols per thread

struct QpskStreams {
  const void* in[8];
  void* out[8];
};

__device__ __forceinline__ float2 qpsk_point(uint32_t s, float a) {
  return make_float2((s & 1u) ? -a : a, (s & 2u) ? -a : a);
}

__device__ __forceinline__ uint32_t qpsk_bits(float2 v) {
  return (v.x >= 0.0f ? 0u : 1u) | (v.y >= 0.0f ? 0u : 2u);
}

// grid.y = stream index. A block owns kQBlock * kQSym consecutive symbols. A full, aligned block is
// moved with lanes on consecutive 16-byte symbol pairs (each wave instruction covers 1 KB of IQ);
// the last block keeps the thread-owns-16-symbols path below.
__global__ __launch_bounds__(kQBlock) void k_qpsk_mod(QpskStreams st, uint32_t n, float a) {
  const uint8_t* __restrict__ in = reinterpret_cast<const uint8_t*>(st.in[blockIdx.y]);
  float2* __restrict__ out = reinterpret_cast<float2*>(st.out[blockIdx.y]);
  const uint64_t base = (uint64_t)blockIdx.x * kQBlock * kQSym;
  if (base + kQBlock * kQSym <= n && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    const uint8_t* bin = in + (base >> 2);
    float4* o = reinterpret_cast<float4*>(out + base);
    uint32_t byte[kQSym / 2];
#pragma unroll
    for (int q = 0; q < kQSym / 2; ++q) byte[q] = bin[(q * kQBlock + threadIdx.x) >> 1];
#pragma unroll
    for (int q = 0; q < kQSym / 2; ++q) {
      const uint32_t nib = byte[q] >> (4 * (threadIdx.x & 1u));  // pair (q * kQBlock + t): symbols 2p, 2p + 1
      const float2 p0 = qpsk_point(nib & 3u, a);
      const float2 p1 = qpsk_point((nib >> 2) & 3u, a);
      o[q * kQBlock + threadIdx.x] = make_float4(p0.x, p0.y, p1.x, p1.y);
    }
    return;
  }
  const uint64_t s0 = base + (uint64_t)threadIdx.x * kQSym;
  if (s0 >= n) return;
  const uint64_t b0 = s0 >> 2;
  const uint32_t nbytes = (uint32_t)(((uint64_t)n + 3u) >> 2);
  uint32_t word = 0;
  if ((reinterpret_cast<uintptr_t>(in + b0) & 3u) == 0 && b0 + 4 <= nbytes) {
    word = *reinterpret_cast<const uint32_t*>(in + b0);
  } else {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b0 + b < nbytes) word |= (uint32_t)in[b0 + b] << (8 * b);
    }
  }
  if (s0 + kQSym <= n && (reinterpret_cast<uintptr_t>(out + s0) & 15u) == 0) {
    float4* o = reinterpret_cast<float4*>(out + s0);
#pragma unroll
    for (int q = 0; q < kQSym / 2; ++q) {
      const float2 p0 = qpsk_point((word >> (4 * q)) & 3u, a);
      const float2 p1 = qpsk_point((word >> (4 * q + 2)) & 3u, a);
      o[q] = make_float4(p0.x, p0.y, p1.x, p1.y);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kQSym; ++k) {
      if (s0 + k < n) out[s0 + k] = qpsk_point((word >> (2 * k)) & 3u, a);
    }
  }
}

__global__ __launch_bounds__(kQBlock) void k_qpsk_demod(QpskStreams st, uint32_t n) {
  const float2* __restrict__ in = reinterpret_cast<const float2*>(st.in[blockIdx.y]);
  uint8_t* __restrict__ out = reinterpret_cast<uint8_t*>(st.out[blockIdx.y]);
  const uint64_t base = (uint64_t)blockIdx.x * kQBlock * kQSym;
  if (base + kQBlock * kQSym <= n && (reinterpret_cast<uintptr_t>(in) & 15u) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 3u) == 0) {
    // lane t of slot q reads symbol pair p = q * kQBlock + t; 8 lanes assemble one 32-bit word
    const float4* src = reinterpret_cast<const float4*>(in + base);
    float4 v[kQSym / 2];
#pragma unroll
    for (int q = 0; q < kQSym / 2; ++q) v[q] = src[q * kQBlock + threadIdx.x];
    uint32_t* dst = reinterpret_cast<uint32_t*>(out + (base >> 2));
#pragma unroll
    for (int q = 0; q < kQSym / 2; ++q) {
      uint32_t w = (qpsk_bits(make_float2(v[q].x, v[q].y)) | (qpsk_bits(make_float2(v[q].z, v[q].w)) << 2))
                   << (4 * (threadIdx.x & 7u));
      w |= __shfl_xor(w, 1);
      w |= __shfl_xor(w, 2);
      w |= __shfl_xor(w, 4);
      if ((threadIdx.x & 7u) == 0) dst[(q * kQBlock + threadIdx.x) >> 3] = w;
    }
    return;
  }
  const uint64_t s0 = base + (uint64_t)threadIdx.x * kQSym;
  if (s0 >= n) return;
  const uint64_t b0 = s0 >> 2;
  uint32_t word = 0;
  if (s0 + kQSym <= n) {
    if ((reinterpret_cast<uintptr_t>(in + s0) & 15u) == 0) {
      const float4* src = reinterpret_cast<const float4*>(in + s0);
#pragma unroll
      for (int q = 0; q < kQSym / 2; ++q) {
        const float4 v = src[q];
        word |= qpsk_bits(make_float2(v.x, v.y)) << (4 * q);
        word |= qpsk_bits(make_float2(v.z, v.w)) << (4 * q + 2);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kQSym; ++k) word |= qpsk_bits(in[s0 + k]) << (2 * k);
    }
    if ((reinterpret_cast<uintptr_t>(out + b0) & 3u) == 0) {
      *reinterpret_cast<uint32_t*>(out + b0) = word;
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) out[b0 + b] = (uint8_t)(word >> (8 * b));
    }
    return;
  }
  // tail: fewer than 16 symbols left; keep the unused bit pairs of the final byte
  const uint32_t left = (uint32_t)(n - s0);
  for (uint32_t k = 0; k < left; ++k) word |= qpsk_bits(in[s0 + k]) << (2 * k);
  const uint32_t nb = (left + 3u) >> 2;
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t byte = (word >> (8 * b)) & 0xffu;
    const uint32_t used = left - 4 * b;  // symbols of this byte that are in range
    if (used < 4) {
      const uint32_t keep = 0xffu & ~((1u << (2 * used)) - 1u);
      byte = (byte & ~keep) | (out[b0 + b] & keep);
    }
    out[b0 + b] = (uint8_t)byte;
  }
}

static hipError_t qpsk_launch(bool modulate, const QpskStreams& st, int nstreams, uint32_t n, float a,
                              int32_t device, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  for (int s = 0; s < nstreams; ++s) {
    if (st.in[s] == nullptr || st.out[s] == nullptr) return hipErrorInvalidValue;
  }
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  // in 64 bits: n + kQSym - 1 wraps a uint32_t for n near 2^32 (numSymbols is uint32_t)
  const uint32_t blocks = (uint32_t)ceil_div<uint64_t>(ceil_div<uint64_t>(n, kQSym), kQBlock);
  const dim3 grid(blocks, (uint32_t)nstreams);
  if (modulate) {
    k_qpsk_mod<<<grid, dim3(kQBlock), 0, stream>>>(st, n, a);
  } else {
    k_qpsk_demod<<<grid, dim3(kQBlock), 0, stream>>>(st, n);
  }
  return launch_status();
}

// Consolidated layout (qpsk.cu:42, 56, 75, 87): bits of stream s at byte s * (n / 4 + 1),
// symbols of stream s at element s * n. Unsupported stream counts process stream 0 only.
static int consolidated_streams(int numStreams) {
  return (numStreams == 1 || numStreams == 2 || numStreams == 4 || numStreams == 8) ? numStreams : 1;
}

}  // namespace gsdr

using gsdr::QpskStreams;

GSDR_C_LINKAGE hipError_t gsdrQpskModulate(const uint8_t* inputBits, hipFloatComplex* output, uint32_t numSymbols,
                                           float amplitude, int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  QpskStreams st{};
  st.in[0] = inputBits;
  st.out[0] = output;
  return gsdr::qpsk_launch(true, st, 1, numSymbols, amplitude, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpskModulate4x(const uint8_t* inputBits0, const uint8_t* inputBits1,
                                             const uint8_t* inputBits2, const uint8_t* inputBits3,
                                             hipFloatComplex* output0, hipFloatComplex* output1,
                                             hipFloatComplex* output2, hipFloatComplex* output3, uint32_t numSymbols,
                                             float amplitude, int32_t cudaDevice,
                                             hipStream_t cudaStream) GSDR_NO_EXCEPT {
  QpskStreams st{};
  st.in[0] = inputBits0;
  st.in[1] = inputBits1;
  st.in[2] = inputBits2;
  st.in[3] = inputBits3;
  st.out[0] = output0;
  st.out[1] = output1;
  st.out[2] = output2;
  st.out[3] = output3;
  return gsdr::qpsk_launch(true, st, 4, numSymbols, amplitude, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpskDemodulate(const hipFloatComplex* input, uint8_t* outputBits, uint32_t numSymbols,
                                             int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  QpskStreams st{};
  st.in[0] = input;
  st.out[0] = outputBits;
  return gsdr::qpsk_launch(false, st, 1, numSymbols, 0.0f, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpskDemodulate4x(const hipFloatComplex* input0, const hipFloatComplex* input1,
                                               const hipFloatComplex* input2, const hipFloatComplex* input3,
                                               uint8_t* outputBits0, uint8_t* outputBits1, uint8_t* outputBits2,
                                               uint8_t* outputBits3, uint32_t numSymbols, int32_t cudaDevice,
                                               hipStream_t cudaStream) GSDR_NO_EXCEPT {
  QpskStreams st{};
  st.in[0] = input0;
  st.in[1] = input1;
  st.in[2] = input2;
  st.in[3] = input3;
  st.out[0] = outputBits0;
  st.out[1] = outputBits1;
  st.out[2] = outputBits2;
  st.out[3] = outputBits3;
  return gsdr::qpsk_launch(false, st, 4, numSymbols, 0.0f, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpskModulateTemplated(const uint8_t* inputBits, hipFloatComplex* output,
                                                    uint32_t numSymbols, float amplitude, int numStreams,
                                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  const int ns = gsdr::consolidated_streams(numStreams);
  QpskStreams st{};
  for (int s = 0; s < ns; ++s) {
    st.in[s] = inputBits == nullptr ? nullptr : inputBits + (size_t)s * (numSymbols / 4 + 1);
    st.out[s] = output == nullptr ? nullptr : output + (size_t)s * numSymbols;
  }
  return gsdr::qpsk_launch(true, st, ns, numSymbols, amplitude, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpskDemodulateTemplated(const hipFloatComplex* input, uint8_t* outputBits,
                                                      uint32_t numSymbols, int numStreams, int32_t cudaDevice,
                                                      hipStream_t cudaStream) GSDR_NO_EXCEPT {
  const int ns = gsdr::consolidated_streams(numStreams);
  QpskStreams st{};
  for (int s = 0; s < ns; ++s) {
    st.in[s] = input == nullptr ? nullptr : input + (size_t)s * numSymbols;
    st.out[s] = outputBits == nullptr ? nullptr : outputBits + (size_t)s * (numSymbols / 4 + 1);
  }
  return gsdr::qpsk_launch(false, st, ns, numSymbols, 0.0f, cudaDevice, cudaStream);
}
