// gsdr-mi355x: gsdrFirFC (reference src/fir.cu:73-171, include/gsdr/fir.h:30-68), its tuning variants
// and probes. FF / CC / CF and the int8 front end live in fir_ff.hip, fir_cc.hip, fir_cf.hip and
// fir_int8.hip (one sample-type pair per translation unit, built in parallel).
#include <hip/hip_runtime.h>

#include "fir_dispatch.hpp"
#include "fir_entry.hpp"
#include "gsdr/fir.h"
#include "gsdr/gsdr_ext.h"
#include "launch.hpp"

namespace gsdr {

#ifdef GSDR_TUNING_PROBES
// Tuning probes are not part of the product library: they are compiled only into
// build/probes/libgsdr_probes.so (`make probes`), which the tools/ scripts load through GSDR_LIB.

// Streaming ceiling probe for this traffic mix: reads the 8*N_in input bytes with fully coalesced
// 16-byte loads and writes 8*N_out bytes (outputs are a sum of loaded samples, not a FIR).
template <bool NT>
__global__ __launch_bounds__(256) void k_stream_probe(const float4* __restrict__ in, float4* __restrict__ out,
                                                      uint64_t n_in16, uint64_t n_out16) {
  // each thread: 4 input granules (one per 1 KiB wave-slab) -> 1 output granule
  const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t o = wave * 64u + lane;
  if (o >= n_out16) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t i = (wave * 4u + k) * 64u + lane;
    if (i < n_in16) {
      const float4 v = NT ? load16_nt(in + i) : in[i];
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
  }
  out[o] = a;
}

hipError_t launch_stream_probe(const FirJob& j, hipStream_t s, bool nt) {
  const uint64_t n_in16 = j.L * 8 / 16, n_out16 = j.N * 8 / 16;
  const uint32_t blocks = (uint32_t)ceil_div<uint64_t>(n_out16, 256);
  if (nt) {
    k_stream_probe<true><<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(j.in),
                                                reinterpret_cast<float4*>(j.out), n_in16, n_out16);
  } else {
    k_stream_probe<false><<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(j.in),
                                                 reinterpret_cast<float4*>(j.out), n_in16, n_out16);
  }
  return launch_status();
}

// Ablation probes (gsdrxFirFCVariant >= 100) used for the energy split in DESIGN.md section 3.1:
// the default shape with only one half of its work.
hipError_t launch_fc_probe(const FirJob& j, hipStream_t s) {
  switch (j.variant) {
    case 104:  // compute only (no staging; the tile holds whatever LDS held)
      return launch_poly<float, float2, 4, 4, 16, 256, kModeFir, 2, true>(j, s);
    case 105:  // staging only, plain loads
      return launch_poly<float, float2, 4, 4, 16, 256, kModeFir, 1>(j, s);
    case 107:  // staging only, non-temporal loads
      return launch_poly<float, float2, 4, 4, 16, 256, kModeFir, 1, true>(j, s);
    case 113:  // matrix-core kernel with register taps, compute only
      return launch_mfma_bc<256, 9, 2>(j, s);
    case 117:  // staging only by LDS-DMA, non-temporal
      return launch_poly<float, float2, 4, 4, 16, 256, kModeFir, 1, true, false, 0, true>(j, s);
    // FM chain (config 3 shape) split: 120 full FM kernel, 121 no NCO mix, 122 no discriminator (plain
    // float store), 123 neither, 124 staging + NCO + discriminator without the FIR, 125 staging only
    case 120:
    case 121:
    case 122:
    case 123:
    case 124:
    case 125: {
      FirJob c = j;
      c.mode = kModeFm;
      c.N = j.N - 1;  // an FM output needs one more FIR output than the input holds for N FIR outputs
      c.nco_inc = 429496730u;  // 0.1 fs
      c.fm_gain = 7.957747f;   // fs / (2 pi 0.02 fs)
      switch (j.variant) {
        case 120: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 0, true>(c, s);
        case 121: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 8, true>(c, s);
        case 122: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 16, true>(c, s);
        case 123: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 24, true>(c, s);
        case 124: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 1, true>(c, s);
        default: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 25, true>(c, s);
      }
    }
    // FM chain (config 3 shape) tile-shape sweep: 130 default (R 4, JC 16, WG 256), 131 R 8 WG 128,
    // 132 JC 8, 133 R 2, 134 WG 128, 135 R 8 JC 8 WG 128, 136 default with the XCD-aware tile order
    case 130:
    case 131:
    case 132:
    case 133:
    case 134:
    case 135:
    case 136: {
      FirJob c = j;
      c.mode = kModeFm;
      c.N = j.N - 1;
      c.nco_inc = 429496730u;  // 0.1 fs
      c.fm_gain = 7.957747f;   // fs / (2 pi 0.02 fs)
      switch (j.variant) {
        case 130: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 0, true>(c, s);
        case 131: return launch_poly<float, float2, 4, 8, 16, 128, kModeFm, 0, true>(c, s);
        case 132: return launch_poly<float, float2, 4, 4, 8, 256, kModeFm, 0, true>(c, s);
        case 133: return launch_poly<float, float2, 4, 2, 16, 256, kModeFm, 0, true>(c, s);
        case 134: return launch_poly<float, float2, 4, 4, 16, 128, kModeFm, 0, true>(c, s);
        case 135: return launch_poly<float, float2, 4, 8, 8, 128, kModeFm, 0, true>(c, s);
        default: return launch_poly<float, float2, 4, 4, 16, 256, kModeFm, 0, true, true>(c, s);
      }
    }
    // LDS-read probe: the default kernel with the register window served from the
    // thread's own R rows only (4 of 19 ds_read_b128 per column and chunk; wrong results, same FMAs):
    // 140 full kernel, 141 compute only
    case 140:
      return launch_poly<float, float2, 4, 4, 16, 256, kModeFir, 64, true>(j, s);
    case 141:
      return launch_poly<float, float2, 4, 4, 16, 256, kModeFir, 66, true>(j, s);
    case 110:
    case 111:
      return launch_stream_probe(j, s, j.variant == 111);
    default:
      return hipErrorInvalidValue;
  }
}
#else
hipError_t launch_fc_probe(const FirJob&, hipStream_t) { return hipErrorInvalidValue; }
#endif  // GSDR_TUNING_PROBES

// The streaming object's one-launch FIR step on complex float samples (stream.hip; stream_step_tiled).
hipError_t fir_fc_stream_step(size_t decimation, const float* taps, size_t tapCount, const hipFloatComplex* chunk,
                              uint64_t chunkLen, int64_t inOff, const hipFloatComplex* hist, uint64_t histLen,
                              hipFloatComplex* histOut, int64_t histFrom, uint64_t histN, hipFloatComplex* output,
                              size_t numOutputs, int32_t device, hipStream_t stream) {
  FirJob job;
  job.in = chunk;
  job.taps = taps;
  job.out = output;
  job.D = decimation;
  job.T = tapCount;
  job.N = numOutputs;
  job.L = chunkLen;
  job.mode = kModeFir;
  job.in_off = inOff;
  job.hist = hist;
  job.hist_len = histLen;
  job.hist_out = histOut;
  job.hist_from = histFrom;
  job.hist_n = histN;
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  return stream_step_tiled<float2, kModeFir>(job, stream);
}

}  // namespace gsdr

using gsdr::fir_entry;

GSDR_C_LINKAGE hipError_t gsdrFirFC(size_t decimation, const float* taps, size_t tapCount,
                                    const hipFloatComplex* input, hipFloatComplex* output, size_t numOutputs,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, float2>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream, -1);
}

GSDR_C_LINKAGE hipError_t gsdrxFirFCVariant(int variant, size_t decimation, const float* taps, size_t tapCount,
                                            const hipFloatComplex* input, hipFloatComplex* output,
                                            size_t numOutputs, int32_t cudaDevice,
                                            hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return fir_entry<float, float2>(decimation, taps, tapCount, input, output, numOutputs, cudaDevice, cudaStream,
                                  variant);
}
