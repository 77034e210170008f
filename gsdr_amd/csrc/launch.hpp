// gsdr-mi355x: host-side launch plumbing shared by every C-ABI entry point.
//
// Mirrors the reference's SIMPLE_CUDA_FNC_START / SIMPLE_CUDA_FNC_END pair
// (reference src/cuComplexOperatorOverloads.cuh:74-93): remember the calling thread's device, switch
// to the requested one, launch, restore. Differences, all stricter: the previous device is restored
// on every exit path (RAII), and the launch status is returned (the reference returns cudaSuccess
// even when a launch failed, cuh:90-93).
#pragma once

#include <atomic>

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gsdr/hip_util.h"

namespace gsdr {

class DeviceScope {
 public:
  explicit DeviceScope(int32_t device) noexcept {
    const int32_t prev = gsdrGetCurrentHipDevice();
    if (prev < 0) {
      status_ = (hipError_t)(-prev);
      return;
    }
    prev_ = prev;
    if (prev != device) {
      status_ = hipSetDevice(device);
      if (status_ == hipSuccess) switched_ = true;
    }
  }
  ~DeviceScope() {
    if (switched_) (void)hipSetDevice(prev_);
  }
  hipError_t status() const noexcept { return status_; }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;

 private:
  int32_t prev_ = 0;
  bool switched_ = false;
  hipError_t status_ = hipSuccess;
};

// Compute units of the current device, cached per device index (the persistent kernels size their grid
// by it on every launch; the attribute query is a host round trip worth avoiding on small calls).
inline hipError_t current_device_cus(int* cus) noexcept {
  static std::atomic<int> cache[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev >= 0 && dev < 64) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) {
      *cus = c;
      return hipSuccess;
    }
  }
  e = hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess && dev >= 0 && dev < 64) cache[dev].store(*cus, std::memory_order_relaxed);
  return e;
}

// Status of the most recent launch on this thread. hipGetLastError also clears the sticky
// per-thread error so a later call does not report a stale failure.
inline hipError_t launch_status() noexcept { return hipGetLastError(); }

inline bool aligned16(const void* p) noexcept { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <class T>
constexpr T ceil_div(T a, T b) {
  return (a + b - 1) / b;
}

}  // namespace gsdr

// Body wrapper for C-ABI functions: switch device, run `body` (which returns hipError_t), restore.
#define GSDR_ON_DEVICE(device, body)                          \
  do {                                                        \
    ::gsdr::DeviceScope gsdrScope_(device);                   \
    if (gsdrScope_.status() != hipSuccess) {                  \
      return gsdrScope_.status();                             \
    }                                                         \
    return (body);                                            \
  } while (0)
