// gsdr-mi355x: receiver-sized calls timed from a plain C++ caller (no Python, no ctypes in the loop).
// Issues back-to-back gsdrFmDemod calls and gsdrxStreamProcess calls (CF32 FM stream, D = 4, 127 taps) of
// 2^16, 2^18 and 2^20 input samples over one 64 M-sample channel, plus the library's smallest launch (a
// 256-element gsdrMagnitude), and prints per call: the GPU time per call (HIP events around the whole loop
// of back-to-back calls) and the host issue time per call. Run it under
//     rocprofv3 --kernel-trace --stats -d <dir> -- ./build/short_call_timer
// and tools/trace_gaps.py splits every call into its kernel's duration and the gap to the next kernel.
//   make examples && ./build/short_call_timer [calls_per_size]
#include <gsdr/gsdr.h>
#include <gsdr/gsdr_ext.h>
#include <gsdr/stream.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    const hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorName(e_)); \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
  const float fs = 1.0e6f, tune = 0.0f, chan = 1.0e5f, dev = 2.0e4f;
  const uint32_t D = 4;
  const size_t T = 127, L = (size_t)1 << 26;
  std::vector<float> taps(T);
  double sum = 0.0;
  for (size_t i = 0; i < T; ++i) {
    const double n = (double)i - (T - 1) / 2.0;
    const double s = n == 0.0 ? 0.2 : std::sin(2 * M_PI * 0.1 * n) / (M_PI * n);
    taps[i] = (float)(s * (0.54 - 0.46 * std::cos(2 * M_PI * i / (T - 1))));
    sum += taps[i];
  }
  for (auto& t : taps) t = (float)(t / sum);
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *dTaps, *y;
  hipFloatComplex* x;
  CHECK(hipMalloc(&dTaps, T * sizeof(float)));
  CHECK(hipMalloc(&x, L * sizeof(hipFloatComplex)));
  CHECK(hipMalloc(&y, (L / D + 4096) * sizeof(float)));
  CHECK(hipMemcpy(dTaps, taps.data(), T * sizeof(float), hipMemcpyHostToDevice));
  {
    // a constant-envelope FM signal around the channel (config 3's kind of input; an all-zero input would send
    // every discriminator output down its atan2f(0, 0) path)
    std::vector<hipFloatComplex> h(L);
    double ph = 0.0;
    for (size_t i = 0; i < L; ++i) {
      ph += 2 * M_PI * (chan + dev * std::sin(2 * M_PI * 1e3 * (double)i / fs)) / fs;
      h[i] = make_hipFloatComplex((float)std::cos(ph), (float)std::sin(ph));
    }
    CHECK(hipMemcpy(x, h.data(), L * sizeof(hipFloatComplex), hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // warm the clock: a few hundred launches of a whole channel
  for (int i = 0; i < 300; ++i) {
    CHECK(gsdrFmDemod(fs, tune, chan, dev, D, 0, dTaps, T, x, y, L / D - 64, 0, st));
  }
  CHECK(hipStreamSynchronize(st));
  std::printf("{\"tool\": \"short_call_timer\", \"calls_per_size\": %d, \"rows\": [\n", calls);
  bool first = true;
  auto row = [&](const char* what, size_t samples, double gpu_us, double host_us) {
    std::printf("%s  {\"what\": \"%s\", \"samples_per_call\": %zu, \"gpu_us_per_call\": %.3f, \"host_us_per_call\": %.3f}",
                first ? "" : ",\n", what, samples, gpu_us, host_us);
    first = false;
  };
  // the smallest launch of the library
  {
    float* m;
    CHECK(hipMalloc(&m, 256 * sizeof(float)));
    CHECK(hipEventRecord(e0, st));
    const auto h0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) CHECK(gsdrMagnitude(x, m, 256, 0, st));
    const auto h1 = std::chrono::steady_clock::now();
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    row("gsdrMagnitude_256", 256, ms * 1e3 / calls, std::chrono::duration<double, std::micro>(h1 - h0).count() / calls);
    CHECK(hipFree(m));
  }
  for (size_t chunk : {(size_t)1 << 16, (size_t)1 << 18, (size_t)1 << 20}) {
    // direct calls: consecutive windows of the channel (each call's outputs and NCO index continue the last)
    {
      const size_t n_out = (chunk - T) / D;
      CHECK(hipEventRecord(e0, st));
      const auto h0 = std::chrono::steady_clock::now();
      size_t pos = 0;
      for (int i = 0; i < calls; ++i) {
        if (pos + chunk > L) pos = 0;
        CHECK(gsdrFmDemod(fs, tune, chan, dev, D, pos, dTaps, T, x + pos, y + pos / D, n_out, 0, st));
        pos += n_out * D;
      }
      const auto h1 = std::chrono::steady_clock::now();
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.0f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      row("gsdrFmDemod", chunk, ms * 1e3 / calls, std::chrono::duration<double, std::micro>(h1 - h0).count() / calls);
    }
    // the streaming object: one launch a call
    {
      gsdrxStream s = nullptr;
      CHECK(gsdrxStreamCreate(&s, GSDRX_STREAM_FM, GSDRX_SAMPLES_CF32, D, dTaps, T, fs, tune, chan, dev, 0, 0));
      const size_t cap = chunk / D + 64;
      size_t written = 0, pos = 0;
      CHECK(hipEventRecord(e0, st));
      const auto h0 = std::chrono::steady_clock::now();
      for (int i = 0; i < calls; ++i) {
        if (pos + chunk > L) pos = 0;
        CHECK(gsdrxStreamProcess(s, x + pos, chunk, y, cap, &written, st));
        pos += chunk;
      }
      const auto h1 = std::chrono::steady_clock::now();
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.0f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      row("gsdrxStreamProcess_fm", chunk, ms * 1e3 / calls,
          std::chrono::duration<double, std::micro>(h1 - h0).count() / calls);
      CHECK(gsdrxStreamDestroy(s));
    }
  }
  std::printf("\n]}\n");
  CHECK(hipStreamSynchronize(st));
  CHECK(hipFree(dTaps));
  CHECK(hipFree(x));
  CHECK(hipFree(y));
  return 0;
}
