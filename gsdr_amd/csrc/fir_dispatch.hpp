// gsdr-mi355x: host-side choice of FIR kernel instantiation for a job (FIR, FM chain or AM chain).
//
// Fast paths (tiled, LDS-staged, register-windowed; see fir_engine.hpp):
//   complex input: D in {2, 4, 8} polyphase kernel, D == 1 contiguous-window kernel
//   real input:    D in {4, 8}    polyphase kernel, D in {1, 2} contiguous-window kernel
// Everything else (other decimations, tap spans that would not fit the LDS budget) runs the generic
// one-output-per-thread kernel, which is correct for any shape.
#pragma once

#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "fir_engine.hpp"
#include "launch.hpp"

namespace gsdr {

struct FirJob {
  const void* in = nullptr;
  const void* taps = nullptr;
  void* out = nullptr;
  size_t D = 1;
  size_t T = 0;
  size_t N = 0;  // outputs written
  size_t L = 0;  // input samples readable
  int mode = kModeFir;
  int variant = -1;  // FC / D=4 tile-shape override for tuning (-1 = default)
  uint32_t nco_inc = 0;
  uint32_t nco_n0 = 0;
  float fm_gain = 0.0f;
};

// LDS budget per workgroup for the tiled kernels (keeps >= 2 workgroups per CU on 160 KiB).
constexpr size_t kMaxTileLds = 64 * 1024;

inline FirParams make_params(const FirJob& j) {
  FirParams p{};
  p.in = j.in;
  p.taps = j.taps;
  p.out = j.out;
  p.L = j.L;
  p.N = j.N;
  p.T = (uint32_t)j.T;
  p.D = (uint32_t)j.D;
  p.nco_inc = j.nco_inc;
  p.nco_n0 = j.nco_n0;
  p.fm_gain = j.fm_gain;
  return p;
}

template <class TapT, class InT, int MODE>
hipError_t launch_generic(const FirJob& j, hipStream_t s) {
  FirParams p = make_params(j);
  const uint64_t blocks = ceil_div<uint64_t>(j.N, 256);
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  k_fir_generic<TapT, InT, MODE><<<dim3((uint32_t)blocks), dim3(256), 0, s>>>(p);
  return launch_status();
}

template <class TapT, class InT, int D, int R, int JC, int WG, int MODE, int ABL = 0, bool NT = false,
          bool TL = false>
hipError_t launch_poly(const FirJob& j, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG>;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  const uint64_t span = nch * JC * D;
  if (span > 0x40000000ull) return launch_generic<TapT, InT, MODE>(j, s);
  const size_t lds = poly_lds_bytes<InT, D, R, WG>((uint32_t)span, MODE, TL ? span * sizeof(TapT) : 0);
  if (lds > kMaxTileLds) return launch_generic<TapT, InT, MODE>(j, s);
  p.nch = (uint32_t)nch;
  const uint32_t stride = (MODE == kModeFm) ? Geo::KT - 1 : Geo::KT;
  p.tile_stride = stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  const bool vec = (reinterpret_cast<uintptr_t>(j.in) % A) == 0 && ((uint64_t)stride * D * sizeof(InT)) % A == 0;
  if (vec) {
    k_fir_poly<TapT, InT, D, R, JC, WG, true, MODE, ABL, NT, TL><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  } else {
    k_fir_poly<TapT, InT, D, R, JC, WG, false, MODE, ABL, NT, TL><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  }
  return launch_status();
}

template <class TapT, class InT, int D, int R, int IC, int WG, int MODE>
hipError_t launch_contig(const FirJob& j, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG>;
  FirParams p = make_params(j);
  const uint64_t nch = ceil_div<uint64_t>(j.T, (uint64_t)IC);
  const uint64_t span = nch * IC;
  if (span > 0x40000000ull) return launch_generic<TapT, InT, MODE>(j, s);
  const size_t lds = poly_lds_bytes<InT, D, R, WG>((uint32_t)span, MODE);
  if (lds > kMaxTileLds) return launch_generic<TapT, InT, MODE>(j, s);
  p.nch = (uint32_t)nch;
  const uint32_t stride = (MODE == kModeFm) ? Geo::KT - 1 : Geo::KT;
  p.tile_stride = stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  const bool vec = aligned16(j.in) && ((uint64_t)stride * D * sizeof(InT)) % 16 == 0;
  if (vec) {
    k_fir_contig<TapT, InT, D, R, IC, WG, true, MODE><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  } else {
    k_fir_contig<TapT, InT, D, R, IC, WG, false, MODE><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  }
  return launch_status();
}

// Workgroups per CU that the hardware keeps resident for `kernel` at `lds` bytes (occupancy query,
// capped by the LDS budget), times the CU count: the persistent grid.
inline uint32_t persistent_grid(const void* kernel, int wg, size_t lds, int oversubscribe) {
  int dev = 0, cus = 0, per_cu = 0, lds_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess) {
    lds_cu = 160 * 1024;
  }
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, wg, lds) != hipSuccess) return 0;
  const int by_lds = lds > 0 ? (int)((size_t)lds_cu / lds) : per_cu;
  if (by_lds < per_cu) per_cu = by_lds;
  if (per_cu < 1) per_cu = 1;
  const uint32_t grid = (uint32_t)(cus * per_cu * (oversubscribe < 1 ? 1 : oversubscribe));
  static bool debug = getenv("GSDR_DEBUG") != nullptr;
  if (debug) {
    fprintf(stderr, "gsdr: persistent grid %u = %d CUs x %d WG/CU x %d (wg %d, lds %zu B, lds/CU %d)\n", grid, cus,
            per_cu, oversubscribe, wg, lds, lds_cu);
  }
  return grid;
}

// Persistent, register-prefetching polyphase kernel (k_fir_poly_pipe). Falls back to the one-tile
// kernel when the halo does not fit the HALO registers per thread.
template <class TapT, class InT, int D, int R, int JC, int WG, int HALO, int MODE>
hipError_t launch_poly_pipe(const FirJob& j, hipStream_t s, int oversubscribe = 1) {
  using Geo = TileGeo<InT, D, R, WG>;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  const uint64_t span = nch * JC * D;
  const uint64_t NG = ((uint64_t)(Geo::KT - 1) * D + span + Geo::G - 1) / Geo::G;
  if (NG > (uint64_t)(Geo::SG + HALO) * WG) return launch_poly<TapT, InT, D, R, JC, WG, MODE>(j, s);
  const size_t lds = poly_lds_bytes<InT, D, R, WG>((uint32_t)span, MODE);
  if (lds > kMaxTileLds) return launch_generic<TapT, InT, MODE>(j, s);
  p.nch = (uint32_t)nch;
  const uint32_t stride = (MODE == kModeFm) ? Geo::KT - 1 : Geo::KT;
  p.tile_stride = stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  const bool vec = aligned16(j.in) && ((uint64_t)stride * D * sizeof(InT)) % 16 == 0;
  if (!vec) return launch_poly<TapT, InT, D, R, JC, WG, MODE>(j, s);
  const void* kern = reinterpret_cast<const void*>(&k_fir_poly_pipe<TapT, InT, D, R, JC, WG, HALO, MODE>);
  uint32_t grid = persistent_grid(kern, WG, lds, oversubscribe);
  if (grid == 0) return hipErrorInvalidDevice;
  if (grid > tiles) grid = (uint32_t)tiles;
  k_fir_poly_pipe<TapT, InT, D, R, JC, WG, HALO, MODE><<<dim3(grid), dim3(WG), lds, s>>>(p, (uint32_t)tiles);
  return launch_status();
}

// Persistent LDS-DMA pipeline (k_fir_poly_dma), FIR mode, 16-byte aligned input only; otherwise the
// one-tile kernel.
template <class TapT, class InT, int D, int R, int JC, int WG, bool TL = false>
hipError_t launch_poly_dma(const FirJob& j, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG>;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  const uint64_t span = nch * JC * D;
  const uint64_t stride = Geo::KT;
  const bool vec = aligned16(j.in) && (stride * D * sizeof(InT)) % 16 == 0;
  if (!vec || span > (1u << 20)) return launch_poly<TapT, InT, D, R, JC, WG, kModeFir>(j, s);
  const uint64_t NG = ((uint64_t)(Geo::KT - 1) * D + span + Geo::G - 1) / Geo::G;
  const uint64_t NGP = Geo::padded((uint32_t)(NG - 1)) + 1;
  const uint32_t slots = (uint32_t)ceil_div<uint64_t>(NGP, WG) * WG;
  const size_t lds = 2ull * slots * 16u + (TL ? span * sizeof(TapT) : 0);
  if (lds > 160 * 1024) return launch_poly<TapT, InT, D, R, JC, WG, kModeFir>(j, s);
  p.nch = (uint32_t)nch;
  p.tile_stride = (uint32_t)stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  const void* kern = reinterpret_cast<const void*>(&k_fir_poly_dma<TapT, InT, D, R, JC, WG, TL>);
  if (lds > 64 * 1024) {
    const hipError_t st = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (st != hipSuccess) return st;
  }
  uint32_t grid = persistent_grid(kern, WG, lds, 1);
  if (grid == 0) return hipErrorInvalidDevice;
  if (grid > tiles) grid = (uint32_t)tiles;
  k_fir_poly_dma<TapT, InT, D, R, JC, WG, TL><<<dim3(grid), dim3(WG), lds, s>>>(p, (uint32_t)tiles, slots);
  return launch_status();
}

// Column-split polyphase kernel (k_fir_poly_cs): D = 2 granules per row, FIR mode, NCH compile-time
// chunk count (taps held in SGPRs for the whole kernel).
template <class TapT, class InT, int D, int R, int JC, int WG, int NCH, bool NT = false>
hipError_t launch_poly_cs(const FirJob& j, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG / 2>;
  using OutT = typename Product<TapT, InT>::type;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  if (nch > (uint64_t)NCH) return launch_poly<TapT, InT, D, R, JC, WG, kModeFir>(j, s);
  p.nch = NCH;  // fewer real chunks read zero taps (range-checked) -- same result
  const uint32_t span = NCH * JC * D;
  const uint32_t NG = ((Geo::KT - 1) * D + span + Geo::G - 1) / Geo::G;
  const size_t lds = (size_t)(Geo::padded(NG - 1) + 1) * 16u + (size_t)(WG / 2) * R * sizeof(OutT);
  if (lds > kMaxTileLds) return launch_generic<TapT, InT, kModeFir>(j, s);
  p.tile_stride = Geo::KT;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, (uint64_t)Geo::KT);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  const bool vec = aligned16(j.in) && ((uint64_t)Geo::KT * D * sizeof(InT)) % 16 == 0;
  if (vec) {
    k_fir_poly_cs<TapT, InT, D, R, JC, WG, NCH, true, NT><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  } else {
    k_fir_poly_cs<TapT, InT, D, R, JC, WG, NCH, false, NT><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  }
  return launch_status();
}

// Tile-shape variants of the headline case (real taps, complex input, D = 4), selectable through
// gsdrxFirFCVariant for tuning sweeps. Variant 0 is the default (WG = 256, R = 4, JC = 16);
// variant 1 is the round-1 starting shape (WG = 128, R = 8).
// Tuning probes (variant >= 100): 100-102 live in fir_probe.hip (compiled with -fno-slp-vectorize),
// 103+ in fir.hip (packed-FMA build).
hipError_t launch_fc_probe(const FirJob& j, hipStream_t s);
hipError_t launch_fc_probe_packed(const FirJob& j, hipStream_t s);

template <class TapT, class InT, int MODE>
hipError_t launch_d4_complex(const FirJob& j, hipStream_t s) {
  if (j.variant >= 103) return launch_fc_probe_packed(j, s);
  if (j.variant >= 100) return launch_fc_probe(j, s);
  switch (j.variant) {
    case 1:
      return launch_poly<TapT, InT, 4, 8, 16, 128, MODE>(j, s);
    case 2:
      return launch_poly<TapT, InT, 4, 8, 16, 256, MODE>(j, s);
    case 3:
      return launch_poly<TapT, InT, 4, 8, 16, 64, MODE>(j, s);
    case 4:
      return launch_poly<TapT, InT, 4, 8, 32, 128, MODE>(j, s);
    case 5:
      return launch_poly<TapT, InT, 4, 4, 8, 256, MODE>(j, s);
    case 6:
      return launch_poly<TapT, InT, 4, 16, 16, 128, MODE>(j, s);
    case 7:
      return launch_generic<TapT, InT, MODE>(j, s);
    case 20:
      return launch_poly_pipe<TapT, InT, 4, 4, 16, 256, 1, MODE>(j, s);
    case 21:
      return launch_poly_pipe<TapT, InT, 4, 4, 8, 256, 1, MODE>(j, s);
    case 22:
      return launch_poly_pipe<TapT, InT, 4, 4, 16, 128, 1, MODE>(j, s);
    case 23:
      return launch_poly_pipe<TapT, InT, 4, 4, 16, 256, 1, MODE>(j, s, 2);
    case 24:  // single-wave workgroups: wave-local barriers, waves drift apart freely
      return launch_poly<TapT, InT, 4, 4, 16, 64, MODE>(j, s);
    case 25:
      return launch_poly_pipe<TapT, InT, 4, 4, 16, 64, 1, MODE>(j, s);
    case 26:
      return launch_poly_pipe<TapT, InT, 4, 4, 8, 64, 1, MODE>(j, s);
    case 27:
      return launch_poly<TapT, InT, 4, 8, 16, 64, MODE>(j, s);
    case 30:  // LDS-DMA double-buffered pipeline: 2 x 38 KB per WG -> 2 WGs (8 waves) per CU
      return launch_poly_dma<TapT, InT, 4, 4, 16, 256>(j, s);
    case 31:  // R = 2: 2 x 25 KB -> 3 WGs (12 waves) per CU
      return launch_poly_dma<TapT, InT, 4, 2, 16, 256>(j, s);
    case 32:  // WG = 512, R = 2: 8 waves in one WG per CU
      return launch_poly_dma<TapT, InT, 4, 2, 16, 512>(j, s);
    case 33:  // WG = 128, R = 4: 2 x 20 KB -> 3 WGs per CU
      return launch_poly_dma<TapT, InT, 4, 4, 16, 128>(j, s);
    case 40:  // default shape, taps staged in LDS
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, false, true>(j, s);
    case 41:  // R = 8, WG = 128, taps in LDS
      return launch_poly<TapT, InT, 4, 8, 16, 128, MODE, 0, false, true>(j, s);
    case 42:  // DMA pipeline, taps in LDS
      return launch_poly_dma<TapT, InT, 4, 4, 16, 256, true>(j, s);
    case 43:
      return launch_poly_dma<TapT, InT, 4, 4, 16, 128, true>(j, s);
    case 44:  // R = 4, WG = 256, JC = 32, taps in LDS
      return launch_poly<TapT, InT, 4, 4, 32, 256, MODE, 0, false, true>(j, s);
    case 45:
      return launch_poly<TapT, InT, 4, 4, 8, 256, MODE, 0, false, true>(j, s);
    case 46:
      return launch_poly<TapT, InT, 4, 8, 8, 128, MODE, 0, false, true>(j, s);
    case 47:
      return launch_poly<TapT, InT, 4, 8, 8, 64, MODE, 0, false, true>(j, s);
    case 50:  // column split, R = 8, 2 pairs of waves, taps in SGPRs once
      return launch_poly_cs<TapT, InT, 4, 8, 16, 256, 2>(j, s);
    case 51:
      return launch_poly_cs<TapT, InT, 4, 4, 16, 256, 2>(j, s);
    case 52:
      return launch_poly_cs<TapT, InT, 4, 8, 16, 128, 2>(j, s);
    case 53:
      return launch_poly_cs<TapT, InT, 4, 4, 16, 512, 2>(j, s);
    case 54:  // column split R = 8 with non-temporal loads and stores
      return launch_poly_cs<TapT, InT, 4, 8, 16, 256, 2, true>(j, s);
    case 55:  // default shape with non-temporal loads and stores
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, true>(j, s);
    case 56:
      return launch_poly_cs<TapT, InT, 4, 4, 16, 256, 2, true>(j, s);
    case 48:
      return launch_poly_dma<TapT, InT, 4, 4, 8, 256, true>(j, s);
    case 49:
      return launch_poly_dma<TapT, InT, 4, 8, 8, 128, true>(j, s);
    default:
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE>(j, s);
  }
}

// Multi-channel chain (k_fir_multi): one launch per group of <= kMaxMultiChannels channels. Returns
// hipErrorNotSupported when the shape does not apply (the caller then runs the channels one by one).
template <class TapT, class InT, int D, int R, int JC, int WG, int MODE>
hipError_t launch_multi(const FirJob& j, const MultiParams& mp, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG>;
  constexpr int HMAX = 1;
  constexpr int BPT = Geo::SG * (Geo::KT / Geo::ROUT) / WG;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  const uint64_t span = nch * JC * D;
  if (span > 0x40000000ull) return hipErrorNotSupported;
  const uint64_t NG = ((uint64_t)(Geo::KT - 1) * D + span + Geo::G - 1) / Geo::G;
  if (NG > (uint64_t)(BPT + HMAX) * WG) return hipErrorNotSupported;  // halo does not fit the registers
  const size_t lds = poly_lds_bytes<InT, D, R, WG>((uint32_t)span, MODE);
  if (lds > kMaxTileLds) return hipErrorNotSupported;
  p.nch = (uint32_t)nch;
  const uint32_t stride = (MODE == kModeFm) ? Geo::KT - 1 : Geo::KT;
  p.tile_stride = stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  const bool vec = (reinterpret_cast<uintptr_t>(j.in) % A) == 0 && ((uint64_t)stride * D * sizeof(InT)) % A == 0;
  if (vec) {
    k_fir_multi<TapT, InT, D, R, JC, WG, HMAX, true, MODE, true><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p, mp);
  } else {
    k_fir_multi<TapT, InT, D, R, JC, WG, HMAX, false, MODE, true><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p, mp);
  }
  return launch_status();
}

// same D and JC as launch_fir's single-channel kernels -> identical per-output MAC order
template <class InT, int MODE>
hipError_t launch_multi_chain(const FirJob& j, const MultiParams& mp, hipStream_t s) {
  if (j.T > (1u << 26)) return hipErrorNotSupported;
  switch (j.D) {
    case 2:
      return launch_multi<float, InT, 2, 8, 16, 128, MODE>(j, mp, s);
    case 4:
      return launch_multi<float, InT, 4, 4, 16, 256, MODE>(j, mp, s);
    case 8:
      return launch_multi<float, InT, 8, 2, 8, 256, MODE>(j, mp, s);
    default:
      return hipErrorNotSupported;
  }
}

// tile-shape sweep for the int8 front end (gsdrxFirFCInt8Variant): the shapes of launch_d4_complex
// whose staging is generic over the input type
inline hipError_t launch_d4_int8(const FirJob& j, hipStream_t s) {
  switch (j.variant) {
    case 0:
      return launch_poly<float, Iq8, 4, 4, 16, 256, kModeFir, 0, true>(j, s);
    case 1:
      return launch_poly<float, Iq8, 4, 8, 16, 128, kModeFir, 0, true>(j, s);
    case 3:
      return launch_poly<float, Iq8, 4, 8, 16, 64, kModeFir, 0, true>(j, s);
    case 4:
      return launch_poly<float, Iq8, 4, 8, 32, 128, kModeFir, 0, true>(j, s);
    case 5:
      return launch_poly<float, Iq8, 4, 4, 8, 256, kModeFir, 0, true>(j, s);
    case 24:
      return launch_poly<float, Iq8, 4, 4, 16, 64, kModeFir, 0, true>(j, s);
    case 27:
      return launch_poly<float, Iq8, 4, 8, 16, 64, kModeFir, 0, true>(j, s);
    case 28:
      return launch_poly<float, Iq8, 4, 4, 16, 128, kModeFir, 0, true>(j, s);
    case 50:
      return launch_poly_cs<float, Iq8, 4, 8, 16, 256, 2, true>(j, s);
    case 56:
      return launch_poly_cs<float, Iq8, 4, 4, 16, 256, 2, true>(j, s);
    case 57:
      return launch_poly_cs<float, Iq8, 4, 8, 16, 128, 2, true>(j, s);
    default:
      return launch_generic<float, Iq8, kModeFir>(j, s);
  }
}

// A default shape whose tile does not fit kMaxTileLds at the headline tap count would silently run
// the generic kernel: reject that at compile time (FM layout = the largest).
template <class InT, int D, int R, int JC, int WG>
constexpr bool fits_lds_at_t127() {
  constexpr uint32_t rows = (127 + D - 1) / D;
  constexpr uint32_t span = (rows + JC - 1) / JC * JC * D;
  return poly_lds_bytes<InT, D, R, WG>(span, kModeFm) <= kMaxTileLds;
}

template <class TapT, class InT, int D, int R, int JC, int WG, int MODE>
hipError_t launch_poly_default(const FirJob& j, hipStream_t s) {
  static_assert(fits_lds_at_t127<InT, D, R, JC, WG>(), "default polyphase shape exceeds the LDS budget");
  return launch_poly<TapT, InT, D, R, JC, WG, MODE, 0, true>(j, s);
}

template <class TapT, class InT, int MODE>
hipError_t launch_fir(const FirJob& j, hipStream_t s) {
  constexpr bool kComplexIn = SampleT<InT>::kPerGranule == 2;
  // the tiled kernels address taps through a 32-bit buffer descriptor
  if (j.T > (1u << 26)) return launch_generic<TapT, InT, MODE>(j, s);
  if constexpr (std::is_same<InT, Iq8>::value) {
    // int8 I/Q: the polyphase kernel (even D keeps every staged dword 4-byte aligned), else generic
    if constexpr (MODE == kModeFir) {
      if (j.D == 4 && j.variant >= 0) return launch_d4_int8(j, s);
    }
    switch (j.D) {
      case 2:
        return launch_poly_default<TapT, InT, 2, 8, 16, 128, MODE>(j, s);
      case 4:
        return launch_poly_default<TapT, InT, 4, 4, 16, 256, MODE>(j, s);
      case 8:
        return launch_poly_default<TapT, InT, 8, 2, 8, 256, MODE>(j, s);
      default:
        return launch_generic<TapT, InT, MODE>(j, s);
    }
  } else if constexpr (kComplexIn) {
    switch (j.D) {
      case 1:
        return launch_contig<TapT, InT, 1, 8, 16, 256, MODE>(j, s);
      case 2:
        return launch_poly_default<TapT, InT, 2, 8, 16, 128, MODE>(j, s);
      case 4:
        if constexpr (MODE == kModeFir && std::is_same<TapT, float>::value) {
          if (j.variant >= 0) return launch_d4_complex<TapT, InT, MODE>(j, s);
        }
        // 4 waves/SIMD (16 per CU): the shape that measured fastest at T = 127
        return launch_poly_default<TapT, InT, 4, 4, 16, 256, MODE>(j, s);
      case 8:
        return launch_poly_default<TapT, InT, 8, 2, 8, 256, MODE>(j, s);
      default:
        return launch_generic<TapT, InT, MODE>(j, s);
    }
  } else {
    switch (j.D) {
      case 1:
        return launch_contig<TapT, InT, 1, 16, 32, 256, MODE>(j, s);
      case 2:
        return launch_contig<TapT, InT, 2, 8, 16, 256, MODE>(j, s);
      case 4:
        return launch_poly_default<TapT, InT, 4, 8, 8, 128, MODE>(j, s);
      case 8:
        return launch_poly_default<TapT, InT, 8, 8, 8, 128, MODE>(j, s);
      default:
        return launch_generic<TapT, InT, MODE>(j, s);
    }
  }
}

}  // namespace gsdr
