// Microbenchmark (development tool): sustained FP32 throughput of v_pk_fma_f32 vs
// v_mfma_f32_16x16x4_f32 on every CU for ~2 s each, to compare their power (sample rocm-smi beside it).
// Build: hipcc -O3 --offload-arch=gfx950 tools/power_bench.hip -o tools/power_bench.bin
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_pk(float* out, const float* __restrict__ taps, int iters) {
  f2 acc[16];
  f2 x[4];
  for (int i = 0; i < 16; ++i) acc[i] = f2{0.f, 0.f};
  for (int i = 0; i < 4; ++i) x[i] = f2{(float)threadIdx.x * 0.001f + i, 1.0f - i};
  for (int it = 0; it < iters; ++it) {
    const float t = taps[it & 63];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma(x[i & 3], f2{t, t}, acc[i]);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mfma(float* out, const float* __restrict__ taps, int iters) {
  f4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  float a = (float)threadIdx.x * 0.001f, b = taps[threadIdx.x & 63];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    a += 1e-7f;
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  float *out, *taps;
  (void)hipMalloc(&out, 256 * 256 * 64 * sizeof(float));
  (void)hipMalloc(&taps, 64 * sizeof(float));
  float host[64];
  for (int i = 0; i < 64; ++i) host[i] = 0.999f - 0.001f * i;
  (void)hipMemcpy(taps, host, sizeof(host), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
  for (int which = 0; which < 2; ++which) {
    const int blocks = 256 * 8;  // 8 waves per SIMD
    const int iters = which ? 2048 : 4096;
    auto t0 = std::chrono::steady_clock::now();
    double flop = 0, ms_total = 0;
    int launches = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
      (void)hipEventRecord(a);
      for (int r = 0; r < 20; ++r) {
        if (which) k_mfma<<<blocks, 256>>>(out, taps, iters);
        else k_pk<<<blocks, 256>>>(out, taps, iters);
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      ms_total += ms;
      launches += 20;
    }
    // per launch: pk: blocks*256 lanes*iters*16 pk_fma*4 flop; mfma: blocks*4 waves*iters*4 mfma*16*16*4*2
    flop = which ? (double)blocks * 4 * iters * 4 * 2048.0 : (double)blocks * 256 * iters * 16 * 4.0;
    printf("%s: %d launches, %.1f TFLOP/s sustained\n", which ? "mfma_f32_16x16x4" : "v_pk_fma_f32   ", launches,
           flop * launches / (ms_total * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
