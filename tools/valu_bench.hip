// Microbenchmark (development tool): issue rate of v_pk_fma_f32 and v_fmac_f32 with an SGPR
// operand on gfx950, at 1/2/4/8 waves per SIMD (occupancy forced with dynamic LDS).
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_bench.hip -o /tmp/valu_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PACKED>
__global__ __launch_bounds__(256) void k(float* out, const float* __restrict__ taps, int iters) {
  extern __shared__ float lds[];
  f2 acc[16];
  f2 x[4];
  for (int i = 0; i < 16; ++i) acc[i] = f2{0.f, 0.f};
  for (int i = 0; i < 4; ++i) x[i] = f2{(float)threadIdx.x * 0.001f + i, 1.0f - i};
  for (int it = 0; it < iters; ++it) {
    const float t = taps[it & 63];  // uniform -> SGPR
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (PACKED) {
        acc[i] = __builtin_elementwise_fma(x[i & 3], f2{t, t}, acc[i]);
      } else {
        acc[i].x = __builtin_fmaf(x[i & 3].x, t, acc[i].x);
        acc[i].y = __builtin_fmaf(x[i & 3].y, t, acc[i].y);
      }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
  if (s == 12345.f) lds[threadIdx.x] = s;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float *out, *taps;
  (void)hipMalloc(&out, 256 * 256 * 64 * sizeof(float));
  (void)hipMalloc(&taps, 64 * sizeof(float));
  float host[64];
  for (int i = 0; i < 64; ++i) host[i] = 0.999f - 0.001f * i;
  (void)hipMemcpy(taps, host, sizeof(host), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096;
  for (int packed = 0; packed < 2; ++packed) {
    for (int wps : {1, 2, 4, 8}) {
      // 256-thread WG = 1 wave per SIMD; wps WGs per CU by LDS: 160 KiB / wps
      const size_t lds = (160 * 1024) / wps - 1024;
      const int blocks = 256 * wps * 4;  // 4 rounds
      auto fn = packed ? k<true> : k<false>;
      hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      fn<<<blocks, 256, lds>>>(out, taps, iters);
      hipEventRecord(a);
      fn<<<blocks, 256, lds>>>(out, taps, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double fma = (double)blocks * 256 * iters * 16 * 2;  // scalar FMAs
      printf("%s waves/SIMD=%d: %.3f ms, %.1f TFLOP/s (fp32 FMA=2 flop)\n", packed ? "pk_fma" : "fmac  ", wps, ms,
             2 * fma / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
