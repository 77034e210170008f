// gsdr-mi355x example: a reference-style C++ host caller of the C ABI (no Python, no torch).
// Builds an FM test signal on the host, filters/decimates it with gsdrFirFC, demodulates it with the
// fused gsdrFmDemod in two streaming chunks, and checks the chunks match a single call.
//   make examples && ./build/fm_receiver [dump_dir]
// With dump_dir, the taps, the input and the gsdrFirFC / gsdrFmDemod outputs are written there as raw
// little-endian float32 files (taps.f32, x.c64, fir.c64, fm.f32) for tests/test_gpu_example.py, which
// checks them against the CPU oracle.
#include <gsdr/gsdr.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    const hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorName(e_)); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

static bool dump(const char* dir, const char* name, const void* data, size_t bytes) {
  char path[4096];
  std::snprintf(path, sizeof(path), "%s/%s", dir, name);
  FILE* f = std::fopen(path, "wb");
  if (f == nullptr) return false;
  const bool ok = std::fwrite(data, 1, bytes, f) == bytes;
  return std::fclose(f) == 0 && ok;
}

int main(int argc, char** argv) {
  const float fs = 1.0e6f, chan = 1.0e5f, dev = 2.0e4f;
  const uint32_t D = 4;
  const size_t T = 127, N = 1 << 20, L = N * D + T;

  // Hamming-windowed sinc low-pass, fc = 0.1 fs, unit DC gain
  std::vector<float> taps(T);
  double sum = 0.0;
  for (size_t i = 0; i < T; ++i) {
    const double n = (double)i - (T - 1) / 2.0;
    const double s = n == 0.0 ? 0.2 : std::sin(2 * M_PI * 0.1 * n) / (M_PI * n);
    taps[i] = (float)(s * (0.54 - 0.46 * std::cos(2 * M_PI * i / (T - 1))));
    sum += taps[i];
  }
  for (auto& t : taps) t = (float)(t / sum);

  // FM carrier at +0.1 fs, 1 kHz tone, 20 kHz deviation
  std::vector<hipFloatComplex> x(L);
  for (size_t n = 0; n < L; ++n) {
    const double ph = 2 * M_PI * 0.1 * n + 20.0 * std::sin(2 * M_PI * 0.001 * n);
    x[n] = make_hipFloatComplex((float)std::cos(ph), (float)std::sin(ph));
  }

  hipStream_t stream;
  CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  float* dTaps;
  hipFloatComplex *dX, *dY;
  float *dFm, *dFm2;
  CHECK(hipMalloc(&dTaps, T * sizeof(float)));
  CHECK(hipMalloc(&dX, L * sizeof(hipFloatComplex)));
  CHECK(hipMalloc(&dY, N * sizeof(hipFloatComplex)));
  CHECK(hipMalloc(&dFm, N * sizeof(float)));
  CHECK(hipMalloc(&dFm2, N * sizeof(float)));
  CHECK(hipMemcpyAsync(dTaps, taps.data(), T * sizeof(float), hipMemcpyHostToDevice, stream));
  CHECK(hipMemcpyAsync(dX, x.data(), L * sizeof(hipFloatComplex), hipMemcpyHostToDevice, stream));

  // drop-in calls, same argument order as the reference headers
  CHECK(gsdrFirFC(D, dTaps, T, dX, dY, N, 0, stream));
  CHECK(gsdrFmDemod(fs, 0.0f, chan, dev, D, 0, dTaps, T, dX, dFm, N, 0, stream));
  // the same stream in two chunks: overlap numLowPassTaps inputs, advance firstSampleIndex (fm.h:26)
  const size_t n1 = N / 3;
  CHECK(gsdrFmDemod(fs, 0.0f, chan, dev, D, 0, dTaps, T, dX, dFm2, n1, 0, stream));
  CHECK(gsdrFmDemod(fs, 0.0f, chan, dev, D, n1 * D, dTaps, T, dX + n1 * D, dFm2 + n1, N - n1, 0, stream));

  // extensions: an int8 I/Q front end fed through the streaming object in uneven buffers, which must
  // reproduce one gsdrxFmDemodInt8 call over the whole signal bit for bit (decimation 4: the matrix-core
  // chain, whose summation blocks follow the absolute output index); that call meets the float chain's
  // parity bar against the exact path (gsdrInt8ToNormFloat + gsdrFmDemod)
  std::vector<int8_t> x8(2 * L);
  for (size_t n = 0; n < L; ++n) {
    x8[2 * n] = (int8_t)std::lrint(100.0f * x[n].x);
    x8[2 * n + 1] = (int8_t)std::lrint(100.0f * x[n].y);
  }
  int8_t* dX8;
  float *dFm8, *dFm8s, *dFm8m, *dX8f;
  CHECK(hipMalloc(&dX8, 2 * L));
  CHECK(hipMalloc(&dX8f, 2 * L * sizeof(float)));
  CHECK(hipMalloc(&dFm8, N * sizeof(float)));
  CHECK(hipMalloc(&dFm8s, N * sizeof(float)));
  CHECK(hipMalloc(&dFm8m, N * sizeof(float)));
  CHECK(hipMemcpyAsync(dX8, x8.data(), 2 * L, hipMemcpyHostToDevice, stream));
  CHECK(gsdrInt8ToNormFloat(dX8, dX8f, 2 * L, 0, stream));
  CHECK(gsdrFmDemod(fs, 0.0f, chan, dev, D, 0, dTaps, T, reinterpret_cast<const hipFloatComplex*>(dX8f), dFm8, N, 0,
                    stream));
  CHECK(gsdrxFmDemodInt8(fs, 0.0f, chan, dev, D, 0, dTaps, T, dX8, dFm8m, N, 0, stream));
  gsdrxStream rx;
  CHECK(gsdrxStreamCreate(&rx, GSDRX_STREAM_FM, GSDRX_SAMPLES_CS8, D, dTaps, T, fs, 0.0f, chan, dev, 0, 0));
  size_t consumed = 0, produced = 0;
  const size_t buffers[] = {1000, 7, 123457, 50000};
  for (size_t b = 0; consumed < L; ++b) {
    const size_t m = std::min(buffers[b % 4], L - consumed);
    size_t n_out = 0;
    CHECK(gsdrxStreamProcess(rx, dX8 + 2 * consumed, m, dFm8s + produced, N - produced, &n_out, stream));
    consumed += m;
    produced += n_out;
  }
  CHECK(gsdrxStreamDestroy(rx));

  std::vector<float> fm(N), fm2(N), fm8(N), fm8s(N), fm8m(N);
  std::vector<hipFloatComplex> y(N);
  CHECK(hipMemcpyAsync(y.data(), dY, N * sizeof(hipFloatComplex), hipMemcpyDeviceToHost, stream));
  CHECK(hipMemcpyAsync(fm.data(), dFm, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  CHECK(hipMemcpyAsync(fm2.data(), dFm2, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  CHECK(hipMemcpyAsync(fm8.data(), dFm8, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  CHECK(hipMemcpyAsync(fm8s.data(), dFm8s, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  CHECK(hipMemcpyAsync(fm8m.data(), dFm8m, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  CHECK(hipStreamSynchronize(stream));
  if (argc > 1 && !(dump(argv[1], "taps.f32", taps.data(), T * sizeof(float)) &&
                    dump(argv[1], "x.c64", x.data(), L * sizeof(hipFloatComplex)) &&
                    dump(argv[1], "fir.c64", y.data(), N * sizeof(hipFloatComplex)) &&
                    dump(argv[1], "fm.f32", fm.data(), N * sizeof(float)))) {
    std::fprintf(stderr, "cannot write to %s\n", argv[1]);
    return 1;
  }
  // the stream emits every output whose window has arrived: all N (the input holds N*D + T samples)
  const bool stream_same = produced == N && std::memcmp(fm8m.data(), fm8s.data(), N * sizeof(float)) == 0;
  // matrix-core int8 chain vs the exact path: wrapped angle within 1e-5 pi g (g = fs / (2 pi dev))
  const double g = fs / (2.0 * 3.141592653589793 * dev);
  double worst = 0.0;
  for (size_t i = 0; i < N; ++i) {
    double d = std::fmod((double)fm8m[i] - (double)fm8[i] + 3.0 * 3.141592653589793 * g, 2.0 * 3.141592653589793 * g);
    worst = std::fmax(worst, std::fabs(d - 3.141592653589793 * g));
  }
  const bool mfma_ok = worst <= 1e-5 * 3.141592653589793 * g;

  double lo = 1e30, hi = -1e30;
  for (size_t i = 1000; i < N; ++i) {
    lo = std::fmin(lo, fm[i]);
    hi = std::fmax(hi, fm[i]);
  }
  const bool same = std::memcmp(fm.data(), fm2.data(), N * sizeof(float)) == 0;
  // gsdrFmDemod's gain is fs / (2 pi dev) at the RF rate (reference fm.cu:203), so a full-deviation
  // tone reads +-D after decimation by D
  std::printf("%s: FM output range [%.3f, %.3f] (expect about +-%u), chunked == monolithic: %s, "
              "int8 stream == monolithic: %s, int8 matrix-core chain within the parity bar: %s\n",
              gsdrVersion(), lo, hi, D, same ? "yes" : "NO", stream_same ? "yes" : "NO", mfma_ok ? "yes" : "NO");
  (void)hipFree(dTaps);
  (void)hipFree(dX);
  (void)hipFree(dY);
  (void)hipFree(dFm);
  (void)hipFree(dFm2);
  (void)hipFree(dX8);
  (void)hipFree(dFm8);
  (void)hipFree(dFm8s);
  (void)hipFree(dFm8m);
  (void)hipFree(dX8f);
  (void)hipStreamDestroy(stream);
  return same && stream_same && mfma_ok && hi > 0.8 * D && hi < 1.2 * D && lo < -0.8 * D && lo > -1.2 * D ? 0 : 1;
}
