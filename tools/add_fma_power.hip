// Microbenchmark (development tool): sustained packed-FP32 instruction rate of an all-v_pk_fma_f32 loop
// vs a half v_pk_add_f32 / half v_pk_fma_f32 loop on varying (random-like) operands, every CU, ~2 s
// each; run beside rocm-smi sampling (tools/power_watch.sh) to compare power at equal issue rate.
// Question it answers: would folding symmetric taps (x[a] + x[b]) * t, which trades FMAs for adds
// one for one, lower the energy per instruction of the FIR core under the 1400 W cap?
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool ADD>
__global__ __launch_bounds__(256) void k_loop(float* out, const float* __restrict__ seed, int iters) {
  f2 acc[8], x[8];
  const float s0 = seed[threadIdx.x & 255];
  for (int i = 0; i < 8; ++i) {
    acc[i] = f2{0.f, 0.f};
    x[i] = f2{s0 * (i + 1) * 0.37f, s0 * (i + 3) * -0.71f};
  }
  f2 t = f2{0.61f * s0, 0.61f * s0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (ADD && (i & 1)) {
        x[i] = x[i] + x[i - 1];  // v_pk_add_f32: data keeps changing
      } else {
        acc[i] = __builtin_elementwise_fma(x[i], t, acc[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (ADD && !(i & 1)) {
        acc[i] = acc[i] + x[i];
      } else {
        acc[i] = __builtin_elementwise_fma(x[i], t, acc[i]);
      }
    }
    t = t * f2{0.999f, 0.999f} + f2{1e-3f, 1e-3f};
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y + x[i].x;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  float *out, *seed;
  (void)hipMalloc(&out, 256 * 256 * 64 * sizeof(float));
  (void)hipMalloc(&seed, 256 * sizeof(float));
  float host[256];
  for (int i = 0; i < 256; ++i) host[i] = (float)((i * 2654435761u) % 1000) / 997.0f - 0.5f;
  (void)hipMemcpy(seed, host, sizeof(host), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
  for (int which = 0; which < 2; ++which) {
    const int blocks = 256 * 8;
    const int iters = 2048;
    auto t0 = std::chrono::steady_clock::now();
    double ms_total = 0;
    int launches = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
      (void)hipEventRecord(a);
      for (int r = 0; r < 10; ++r) {
        if (which) k_loop<true><<<blocks, 256>>>(out, seed, iters);
        else k_loop<false><<<blocks, 256>>>(out, seed, iters);
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      ms_total += ms;
      launches += 10;
    }
    // 17 packed instructions per iteration per lane (16 + the tap update's mul/add pair counts ~2)
    const double inst = (double)blocks * 256 / 64 * iters * 16.0 * launches;
    printf("%s: %d launches, %.1f G wave-instr/s (packed), %.3f ms/launch\n", which ? "pk_add+pk_fma" : "pk_fma only ",
           launches, inst / (ms_total * 1e-3) / 1e9, ms_total / launches);
    fflush(stdout);
  }
  return 0;
}
