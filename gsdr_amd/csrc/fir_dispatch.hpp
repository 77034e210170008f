// gsdr-mi355x: host-side choice of FIR kernel instantiation for a job (FIR, FM chain or AM chain).
//
// Fast paths (tiled, LDS-staged, register-windowed; see fir_engine.hpp):
//   complex input: D in {2, 4, 6, 8, 10, 12, 16, 20, 24, 32, 40, 48, 64} polyphase kernel,
//                  D in {1, 3, 5, 7} contiguous-window kernel
//   real input:    D in {4, 8, 12, 16, 20, 24, 32, 40, 48, 64} polyphase kernel,
//                  D in {1, 2, 3, 5, 6, 7, 10} contiguous-window kernel
//   int8 I/Q:      as complex input
// Other decimations with T > D: runtime-decimation LDS tile kernel (k_fir_rt) with 256, 128 or 64
// outputs a tile, while the tile fits the LDS budget. Everything else (D >= T, tap spans that would
// not fit) runs the generic one-output-per-thread kernel, which is correct for any shape.
#pragma once

#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "fir_engine.hpp"
#include "fir_i8_mfma.hpp"
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
  uint32_t out_phase = 0;  // absolute index of output 0 mod 16 (fir_i8_mfma.hpp)
  uint64_t q0 = 0;         // chains: absolute index of output 0 (firstSampleIndex / D) -- the anchored
                           // polyphase tiles' NCO cell grid (fir_engine.hpp, stage_tile_rel)
  // the int8 matrix-core kernels' streaming inputs (FirParams)
  int64_t in_off = 0;
  const void* hist = nullptr;
  uint64_t hist_len = 0;
  void* hist_out = nullptr;
  int64_t hist_from = 0;
  uint64_t hist_n = 0;
  // the streaming object's one-launch path on the tiled kernels (stream_step_tiled): only the polyphase and
  // contiguous-window kernels take it; the others return hipErrorNotSupported before launching anything
  bool stream_tiled = false;
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
  p.out_phase = j.out_phase & 15u;
  p.in_off = j.in_off;
  p.hist = j.hist;
  p.hist_len = j.hist_len;
  p.hist_out = j.hist_out;
  p.hist_from = j.hist_from;
  p.hist_n = j.hist_n;
  return p;
}

// FM tiles overlap by one FIR output (the discriminator pairs y[m] with y[m + 1]). With odd D that
// stride would put every other tile off the staging alignment (and all of them on the per-sample load
// path), so those tiles overlap by two outputs instead.
template <class InT>
inline uint32_t fm_tile_stride(uint32_t kt, size_t D) {
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  return ((uint64_t)(kt - 1) * D * sizeof(InT)) % A == 0 ? kt - 1 : kt - 2;
}

// Complex input 8 bytes off 16-byte alignment, or int8 I/Q 2 bytes off 4-byte alignment, with every tile
// start equally off (even samples per tile stride): the tiled kernels stage it with shifted aligned
// loads (stage_tile's SH mode).
template <class InT>
inline bool shifted_staging(const void* in, uint64_t samples_per_tile) {
  if constexpr (std::is_same<InT, float2>::value) {
    return (reinterpret_cast<uintptr_t>(in) % 16) == 8 && samples_per_tile % 2 == 0;
  } else if constexpr (std::is_same<InT, Iq8>::value) {
    // int8 I/Q one sample (2 bytes) off 4-byte alignment: shifted 4-byte word loads
    return (reinterpret_cast<uintptr_t>(in) % 4) == 2 && samples_per_tile % 2 == 0;
  } else {
    // real samples 1..3 floats off 16-byte alignment (stage_tile's real SH mode, SH = the offset)
    return (reinterpret_cast<uintptr_t>(in) % 4) == 0 && (reinterpret_cast<uintptr_t>(in) % 16) != 0 &&
           samples_per_tile % 4 == 0;
  }
}

// Launch kernel template K<SH> with the shift the input pointer needs (shifted_staging is true): 1 for
// complex / int8 I/Q input, the float offset 1..3 for real input.
template <class InT, class F>
inline void launch_shifted(const void* in, F&& f) {
  if constexpr (std::is_same<InT, float>::value) {
    switch ((reinterpret_cast<uintptr_t>(in) % 16) / 4) {
      case 1: f(std::integral_constant<int, 1>{}); break;
      case 2: f(std::integral_constant<int, 2>{}); break;
      default: f(std::integral_constant<int, 3>{}); break;
    }
  } else {
    f(std::integral_constant<int, 1>{});
  }
}

template <class TapT, class InT, int MODE>
hipError_t launch_generic(const FirJob& j, hipStream_t s) {
  if (j.stream_tiled) return hipErrorNotSupported;
  FirParams p = make_params(j);
  const uint64_t blocks = ceil_div<uint64_t>(j.N, 256);
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  k_fir_generic<TapT, InT, MODE><<<dim3((uint32_t)blocks), dim3(256), 0, s>>>(p);
  return launch_status();
}

// Tile grid of the polyphase kernels. FIR: tile t = outputs [t KT, (t + 1) KT). FM / AM chains (anchored NCO,
// fir_engine.hpp stage_tile_rel): tiles on an absolute output grid of stride S -- KT for AM; KT - R for FM, whose
// tiles overlap by one thread's outputs so that every discriminator pairs two outputs of one tile -- output 0
// (absolute index q0) sits at tile_shift = q0 mod S in tile 0, which is sub-tile cell_sub0 of its NCO cell of
// SUBS tiles (CELL = SUBS S outputs; the short-call shapes of a decimation are sub-tiles of its largest tile, whose
// stride is SUBS times theirs). Returns the tile count.
template <int MODE>
inline uint64_t poly_grid(const FirJob& j, FirParams& p, uint32_t kt, uint32_t r, uint32_t subs) {
  const uint32_t stride = MODE == kModeFm ? kt - r : kt;
  p.tile_stride = stride;
  if constexpr (MODE == kModeFir) {
    p.tile_shift = 0;
    p.cell_sub0 = 0;
  } else {
    p.tile_shift = (uint32_t)(j.q0 % stride);
    p.cell_sub0 = (uint32_t)((j.q0 % ((uint64_t)stride * subs)) / stride);
  }
  return ceil_div<uint64_t>(j.N + p.tile_shift, stride);
}

template <class TapT, class InT, int D, int R, int JC, int WG, int MODE, int ABL = 0, bool NT = false, bool XM = false,
          int CST = 0, bool DMA = false, int SUBS = 1>
hipError_t launch_poly(const FirJob& j, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG>;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  const uint64_t span = nch * JC * D;
  if (span > 0x40000000ull) return launch_generic<TapT, InT, MODE>(j, s);
  const size_t lds = poly_lds_bytes<InT, D, R, WG>((uint32_t)span, MODE);
  if (lds > kMaxTileLds) return launch_generic<TapT, InT, MODE>(j, s);
  p.nch = (uint32_t)nch;
  const uint64_t tiles = poly_grid<MODE>(j, p, Geo::KT, R, SUBS);
  const uint32_t stride = p.tile_stride;
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  // (the anchored grid moves every tile start by tile_shift * D samples: a whole number of aligned units, D even)
  const bool vec = (reinterpret_cast<uintptr_t>(j.in) % A) == 0 && ((uint64_t)stride * D * sizeof(InT)) % A == 0;
  if (vec) {
    k_fir_poly<TapT, InT, D, R, JC, WG, true, MODE, ABL, NT, XM, CST, DMA, 0, SUBS>
        <<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  } else if (shifted_staging<InT>(j.in, (uint64_t)stride * D)) {
    launch_shifted<InT>(j.in, [&](auto sh) {
      k_fir_poly<TapT, InT, D, R, JC, WG, false, MODE, ABL, NT, XM, CST, false, decltype(sh)::value, SUBS>
          <<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
    });
  } else {
    k_fir_poly<TapT, InT, D, R, JC, WG, false, MODE, ABL, NT, XM, CST, DMA, 0, SUBS>
        <<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  }
  return launch_status();
}

// Matrix-core FIR with register-resident taps (k_fir_mfma_bc): FC, D = 4, 3D + T <= 16 * MAXSEG.
template <int WG, int MAXSEG, int ABL = 0>
hipError_t launch_mfma_bc(const FirJob& j, hipStream_t s) {
  using Geo = TileGeo<float2, 4, 4, WG>;
  if (j.D != 4 || 12 + j.T > 16u * MAXSEG) return hipErrorInvalidValue;
  const size_t lds = mfma_bc_lds_bytes<WG>((uint32_t)j.T);
  FirParams p = make_params(j);
  p.tile_stride = Geo::KT;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, Geo::KT);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  if (aligned16(j.in)) {
    k_fir_mfma_bc<WG, MAXSEG, true, true, ABL><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  } else {
    k_fir_mfma_bc<WG, MAXSEG, false, true, ABL><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
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
  const uint32_t stride = (MODE == kModeFm) ? fm_tile_stride<InT>(Geo::KT, j.D) : Geo::KT;
  p.tile_stride = stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  const bool vec = (reinterpret_cast<uintptr_t>(j.in) % A) == 0 && ((uint64_t)stride * D * sizeof(InT)) % A == 0;
  if (vec) {
    k_fir_contig<TapT, InT, D, R, IC, WG, true, MODE><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  } else if (shifted_staging<InT>(j.in, (uint64_t)stride * D)) {
    launch_shifted<InT>(j.in, [&](auto sh) {
      k_fir_contig<TapT, InT, D, R, IC, WG, false, MODE, decltype(sh)::value>
          <<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
    });
  } else {
    k_fir_contig<TapT, InT, D, R, IC, WG, false, MODE><<<dim3((uint32_t)tiles), dim3(WG), lds, s>>>(p);
  }
  return launch_status();
}

// Tile-shape variants of the headline case (real taps, complex input, D = 4), selectable through
// gsdrxFirFCVariant for tuning sweeps (all with non-temporal streaming unless noted):
//   0 default WG=256 R=4 JC=16 | 1 WG=128 R=8 | 3 WG=64 R=8 | 4 WG=128 R=8 JC=32 | 5 WG=256 R=4 JC=8
//   7 generic kernel | 8 default shape with plain (temporal) loads/stores | 9 default, XCD-aware tile order
//   10/11 default, tile stored through LDS | 13 matrix-core core (k_fir_mfma_bc, T <= 132)
//   14 default, tile body staged by LDS-DMA (global_load_lds)
//   24 WG=64 R=4 | 25 WG=256 R=2 | 26 WG=256 R=1 | 28 WG=128 R=4
// Ablation probes (fir.hip, compiled only into the probes library, `make probes`; the product library
// returns hipErrorInvalidValue for them): 104 compute only, 105 staging only, 107 staging only
// (non-temporal), 113 matrix-core compute only, 117 staging only by LDS-DMA, 110/111 streaming ceiling
// of this traffic mix (plain / non-temporal).
hipError_t launch_fc_probe(const FirJob& j, hipStream_t s);

template <class TapT, class InT, int MODE>
hipError_t launch_d4_complex(const FirJob& j, hipStream_t s) {
  if (j.variant >= 100) return launch_fc_probe(j, s);
  switch (j.variant) {
    case 0:
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, true>(j, s);
    case 1:
      return launch_poly<TapT, InT, 4, 8, 16, 128, MODE, 0, true>(j, s);
    case 3:
      return launch_poly<TapT, InT, 4, 8, 16, 64, MODE, 0, true>(j, s);
    case 4:
      return launch_poly<TapT, InT, 4, 8, 32, 128, MODE, 0, true>(j, s);
    case 5:
      return launch_poly<TapT, InT, 4, 4, 8, 256, MODE, 0, true>(j, s);
    case 7:
      return launch_generic<TapT, InT, MODE>(j, s);
    case 8:
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE>(j, s);
    case 9:  // default shape, XCD-aware tile order
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, true, true>(j, s);
    case 10:  // default shape, tile stored through LDS (coalesced), plain stores
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, true, false, 1>(j, s);
    case 11:  // default shape, tile stored through LDS (coalesced), streaming stores
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, true, false, 2>(j, s);
    case 13:  // matrix-core core, taps broadcast from registers (k_fir_mfma_bc), FIR mode, T <= 132
      if constexpr (MODE == kModeFir && std::is_same<TapT, float>::value && std::is_same<InT, float2>::value) {
        return launch_mfma_bc<256, 9>(j, s);
      }
      return hipErrorInvalidValue;
    case 14:  // default shape, tile body staged by LDS-DMA (global_load_lds), non-temporal
      return launch_poly<TapT, InT, 4, 4, 16, 256, MODE, 0, true, false, 0, true>(j, s);
    case 24:
      return launch_poly<TapT, InT, 4, 4, 16, 64, MODE, 0, true>(j, s);
    case 25:  // WG 256, R 2 (512-output tiles; a short-call shape)
      return launch_poly<TapT, InT, 4, 2, 16, 256, MODE, 0, true>(j, s);
    case 26:  // WG 256, R 1 (256-output tiles)
      return launch_poly<TapT, InT, 4, 1, 16, 256, MODE, 0, true>(j, s);
    case 28:
      return launch_poly<TapT, InT, 4, 4, 16, 128, MODE, 0, true>(j, s);
    default:
      return hipErrorInvalidValue;
  }
}

// Multi-channel chain (k_fir_poly_grouped): one launch per group of <= kMaxMultiChannels channels, the
// single-channel polyphase tile with the C channels of an input tile grouped on one XCD (same staging
// choice as launch_poly, so each channel is that kernel's call bit for bit). Returns
// hipErrorNotSupported, before launching anything, when the shape does not apply (the caller then runs
// the channels one by one).
template <class TapT, class InT, int D, int R, int JC, int WG, int MODE>
hipError_t launch_multi_grouped(const FirJob& j, const MultiParams& mp, hipStream_t s) {
  using Geo = TileGeo<InT, D, R, WG>;
  FirParams p = make_params(j);
  const uint64_t rows = ceil_div<uint64_t>(j.T, (uint64_t)D);
  const uint64_t nch = ceil_div<uint64_t>(rows, (uint64_t)JC);
  const uint64_t span = nch * JC * D;
  if (span > 0x40000000ull) return hipErrorNotSupported;
  const size_t lds = poly_lds_bytes<InT, D, R, WG>((uint32_t)span, MODE);
  if (lds > kMaxTileLds) return hipErrorNotSupported;
  p.nch = (uint32_t)nch;
  const uint64_t tiles = poly_grid<MODE>(j, p, Geo::KT, R, 1);
  const uint32_t stride = p.tile_stride;
  const uint64_t blocks = ceil_div<uint64_t>(tiles, 8) * 8 * mp.count;
  if (blocks > 0x7fffffffull) return hipErrorNotSupported;
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  const bool vec = (reinterpret_cast<uintptr_t>(j.in) % A) == 0 && ((uint64_t)stride * D * sizeof(InT)) % A == 0;
  if (vec) {
    k_fir_poly_grouped<TapT, InT, D, R, JC, WG, true, MODE, 0><<<dim3((uint32_t)blocks), dim3(WG), lds, s>>>(
        p, mp, (uint32_t)tiles);
  } else if (shifted_staging<InT>(j.in, (uint64_t)stride * D)) {
    k_fir_poly_grouped<TapT, InT, D, R, JC, WG, false, MODE, 1><<<dim3((uint32_t)blocks), dim3(WG), lds, s>>>(
        p, mp, (uint32_t)tiles);
  } else {
    k_fir_poly_grouped<TapT, InT, D, R, JC, WG, false, MODE, 0><<<dim3((uint32_t)blocks), dim3(WG), lds, s>>>(
        p, mp, (uint32_t)tiles);
  }
  return launch_status();
}

// same D, JC and NCO cell as launch_fir's single-channel kernels -> identical per-output MAC order and phasors
template <class InT, int MODE>
hipError_t launch_multi_chain(const FirJob& j, const MultiParams& mp, hipStream_t s) {
  if (j.T > (1u << 26)) return hipErrorNotSupported;
  switch (j.D) {
    case 2:
      return launch_multi_grouped<float, InT, 2, 8, 16, 128, MODE>(j, mp, s);
    case 4:
      return launch_multi_grouped<float, InT, 4, 4, 16, 256, MODE>(j, mp, s);
    case 8:
      return launch_multi_grouped<float, InT, 8, 2, 8, 256, MODE>(j, mp, s);
    default:
      return hipErrorNotSupported;
  }
}

// int8 I/Q FIR on the matrix cores (k_fir_i8_mfma, fir_i8_mfma.hpp): D = 4, T <= 196; persistent
// workgroups (their tap fragments are built once). The tile grid starts at output -out_phase, so the
// staging granule and the output pairs are aligned per call from the pointers and the phase.
template <int D, int NS, int BPC, int NCT, int PF = 1>
hipError_t launch_i8_mfma_nct(const FirJob& j, const FirParams& p, uint32_t ns, uint64_t tiles, uint32_t grid,
                              hipStream_t s) {
  using C = I8Mfma<D, NS, NCT>;
  // tile starts are at sample (j KT - phase) D + in_off: byte offset 2 D (j KT - phase) + 2 in_off
  const uintptr_t in0 = reinterpret_cast<uintptr_t>(j.in) + (uintptr_t)(2 * j.in_off) - 2u * D * p.out_phase;
  const bool oa = ((reinterpret_cast<uintptr_t>(j.out) - 8u * p.out_phase) % 16) == 0;
#define GSDR_I8_LAUNCH(G, LM)                                                                                     \
  (oa ? (k_fir_i8_mfma<D, NS, G, LM, true, BPC, NCT, PF><<<dim3(grid), dim3(C::WG), 0, s>>>(p, ns, (uint32_t)tiles), 0) \
      : (k_fir_i8_mfma<D, NS, G, LM, false, BPC, NCT, PF><<<dim3(grid), dim3(C::WG), 0, s>>>(p, ns, (uint32_t)tiles), 0))
  if (in0 % 16 == 0) {
    (void)GSDR_I8_LAUNCH(8, 1);
  } else if (in0 % 8 == 0) {
    (void)GSDR_I8_LAUNCH(4, 1);
  } else if (in0 % 2 == 0) {
    (void)GSDR_I8_LAUNCH(4, 2);  // 2-byte aligned: shifted 8-byte loads
  } else {
    (void)GSDR_I8_LAUNCH(8, 0);
  }
#undef GSDR_I8_LAUNCH
  return launch_status();
}

template <int D, int NS, int BPC>
hipError_t launch_i8_mfma_ns(const FirJob& j, hipStream_t s) {
  FirParams p = make_params(j);
  const uint32_t ns = (uint32_t)ceil_div<uint64_t>(15u * D + j.T, 32u);
  int cus = 0;
  const hipError_t e = current_device_cus(&cus);
  if (e != hipSuccess) return e;
  const uint64_t slots = (uint64_t)cus * BPC;
  const uint64_t tiles = ceil_div<uint64_t>(j.N + p.out_phase, (uint64_t)I8Mfma<D, NS>::KT);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  if constexpr (BPC == 3) {
    // A short call (fewer 2,048-output tiles than two rounds of workgroup slots) takes 512-output tiles:
    // one large tile alone is ~10 us (load, 24 MFMAs a wave, stores), so a call of a few hundred tiles
    // was one tile's latency on a third of the slots. Same outputs bit for bit (the summation order is
    // per 16-output block, aligned to the absolute output index).
    if (tiles < 2 * slots) {
      const uint64_t t1 = ceil_div<uint64_t>(j.N + p.out_phase, (uint64_t)I8Mfma<D, NS, 1>::KT);
      return launch_i8_mfma_nct<D, NS, BPC, 1>(j, p, ns, t1, (uint32_t)std::min<uint64_t>(t1, slots), s);
    }
  }
  return launch_i8_mfma_nct<D, NS, BPC, 4>(j, p, ns, tiles, (uint32_t)std::min<uint64_t>(tiles, slots), s);
}

template <int D, int BPC = 3>
hipError_t launch_i8_mfma(const FirJob& j, hipStream_t s) {
  if (j.D != (size_t)D || j.T < 1 || j.T > (size_t)I8Mfma<D, 8>::MAXT ||
      (reinterpret_cast<uintptr_t>(j.out) % 8) != 0) {
    return hipErrorInvalidValue;
  }
  // 6 K steps (15 D + T <= 192) cover T <= 132 with fewer fragment registers than 8
  if (j.T <= (size_t)I8Mfma<D, 6>::MAXT) return launch_i8_mfma_ns<D, 6, BPC>(j, s);
  return launch_i8_mfma_ns<D, 8, BPC>(j, s);
}

// int8 I/Q FM / AM chain on the matrix cores (k_chain_i8_mfma): D = 4, T <= 132
#ifndef GSDR_CHAIN_NCT
#define GSDR_CHAIN_NCT 4
#endif
#ifndef GSDR_CHAIN_BPC
#define GSDR_CHAIN_BPC 3
#endif
template <int MODE, int NCT, int BPC>
hipError_t launch_chain_i8_mfma_nct(const FirJob& j, const FirParams& p, uint32_t ns, uint64_t tiles, uint32_t grid,
                                    hipStream_t s) {
  using C = I8ChainMfma<MODE, NCT>;
  // tile starts are at sample 4 (j STRIDE - phase) + in_off: 8 (j STRIDE - phase) + 2 in_off bytes
  const uintptr_t in0 = reinterpret_cast<uintptr_t>(j.in) + (uintptr_t)(2 * j.in_off);
  if (in0 % 8 == 0) {
    k_chain_i8_mfma<MODE, 1, BPC, NCT><<<dim3(grid), dim3(C::WG), 0, s>>>(p, ns, (uint32_t)tiles);
  } else if (in0 % 2 == 0) {  // 2-byte aligned: shifted 8-byte loads
    k_chain_i8_mfma<MODE, 2, BPC, NCT><<<dim3(grid), dim3(C::WG), 0, s>>>(p, ns, (uint32_t)tiles);
  } else {
    k_chain_i8_mfma<MODE, 0, BPC, NCT><<<dim3(grid), dim3(C::WG), 0, s>>>(p, ns, (uint32_t)tiles);
  }
  return launch_status();
}

template <int MODE>
hipError_t launch_chain_i8_mfma(const FirJob& j, hipStream_t s) {
  constexpr int NCT = GSDR_CHAIN_NCT, BPC = GSDR_CHAIN_BPC;
  FirParams p = make_params(j);
  const uint32_t ns = (uint32_t)ceil_div<uint64_t>(7u * 4u + j.T, 32u);
  const uint64_t tiles = ceil_div<uint64_t>(j.N + p.out_phase, (uint64_t)I8ChainMfma<MODE, NCT>::STRIDE);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  int cus = 0;
  const hipError_t e = current_device_cus(&cus);
  if (e != hipSuccess) return e;
  const uint64_t slots = (uint64_t)cus * BPC;
  if constexpr (NCT > 1) {
    // short calls take one C tile a wave (as launch_i8_mfma_ns); the outputs are the same bit for bit
    if (tiles < 2 * slots) {
      const uint64_t t1 = ceil_div<uint64_t>(j.N + p.out_phase, (uint64_t)I8ChainMfma<MODE, 1>::STRIDE);
      return launch_chain_i8_mfma_nct<MODE, 1, BPC>(j, p, ns, t1, (uint32_t)std::min<uint64_t>(t1, slots), s);
    }
  }
  return launch_chain_i8_mfma_nct<MODE, NCT, BPC>(j, p, ns, tiles, (uint32_t)std::min<uint64_t>(tiles, slots), s);
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
    case 7:
      return launch_generic<float, Iq8, kModeFir>(j, s);
    case 24:
      return launch_poly<float, Iq8, 4, 4, 16, 64, kModeFir, 0, true>(j, s);
    case 28:
      return launch_poly<float, Iq8, 4, 4, 16, 128, kModeFir, 0, true>(j, s);
    case 40:  // matrix cores (exact bf16 tap parts, normwise parity), 2 workgroups per CU (round 2: 4, which the
              // round-4 conflict-free LDS layout, 41 KB a workgroup, no longer fits)
      return launch_i8_mfma<4, 2>(j, s);
    case 41:  // matrix cores, 3 workgroups per CU: the default for D = 4
      return launch_i8_mfma<4, 3>(j, s);
    case 42:  // matrix cores, 3 workgroups per CU, 1,024-output tiles at every size (tile-shape sweep)
    case 43:    // the same with 512-output tiles
    case 44:    // 512-output tiles, 4 workgroups per CU
    case 45:    // 512-output tiles, two tiles in flight a workgroup
    case 46: {  // 512-output tiles, 4 workgroups per CU, two tiles in flight
      if (j.D != 4 || j.T < 1 || j.T > (size_t)I8Mfma<4, 6>::MAXT || (reinterpret_cast<uintptr_t>(j.out) % 8) != 0) {
        return hipErrorInvalidValue;
      }
      const FirParams p = make_params(j);
      const uint32_t ns = (uint32_t)ceil_div<uint64_t>(15u * 4u + j.T, 32u);
      int cus = 0;
      const hipError_t e = current_device_cus(&cus);
      if (e != hipSuccess) return e;
      const uint64_t kt = j.variant == 42 ? (uint64_t)I8Mfma<4, 6, 2>::KT : (uint64_t)I8Mfma<4, 6, 1>::KT;
      const uint64_t t = ceil_div<uint64_t>(j.N + p.out_phase, kt);
      const uint64_t bpc = (j.variant == 44 || j.variant == 46) ? 4 : 3;
      const uint32_t grid = (uint32_t)std::min<uint64_t>(t, (uint64_t)cus * bpc);
      switch (j.variant) {
        case 42:
          return launch_i8_mfma_nct<4, 6, 3, 2>(j, p, ns, t, grid, s);
        case 44:
          return launch_i8_mfma_nct<4, 6, 4, 1>(j, p, ns, t, grid, s);
        case 45:
          return launch_i8_mfma_nct<4, 6, 3, 1, 2>(j, p, ns, t, grid, s);
        case 46:
          return launch_i8_mfma_nct<4, 6, 4, 1, 2>(j, p, ns, t, grid, s);
        default:
          return launch_i8_mfma_nct<4, 6, 3, 1>(j, p, ns, t, grid, s);
      }
    }
    default:
      return hipErrorInvalidValue;
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

// Decimation 4 (the headline shape, complex or int8 I/Q samples) with the tile sized to the call: the
// 1,024-output tiles (WG 256, R 4) measured fastest for a whole channel, but a call of a few rounds of
// workgroup slots (a stream chunk) pays each round's latency on part of the chip. Kernel trace of the shapes
// (tools/short_call_shapes.py, profiles/r04_short_call_shapes.txt): at 2.1 M / 524 K / 131 K outputs
// WG 256 R 4 took 24.5 / 9.0 / 6.3 us, WG 256 R 2 (512-output tiles) 22.0 / 8.5 / 5.4, WG 64 R 4
// 23.5 / 8.9 / 5.7, WG 256 R 1 29.2 / 9.9 / 5.1 -- so calls of fewer than three rounds of 1,024-output
// tiles take R 2. The per-output MAC order depends only on (D, JC): every shape gives the same outputs bit
// for bit.
#ifndef GSDR_SHORT_R1
#define GSDR_SHORT_R1 1
#endif
template <class TapT, class InT, int MODE>
hipError_t launch_poly_d4(const FirJob& j, hipStream_t s) {
  int cus = 0;
  if (current_device_cus(&cus) == hipSuccess && cus > 0) {
    const uint64_t slots = (uint64_t)cus * 4;  // 38 KB tiles: 4 workgroups a CU
#if GSDR_SHORT_R1
    // calls of at most one 256-output tile for every second slot (2^19 input samples at D = 4 on 256 CUs):
    // 256-output tiles (same JC: the same outputs bit for bit). Measured per FM call (tools/short_call_floor.py):
    // 2^16 / 2^18 samples 5.41 / 5.51 -> 4.74 / 4.89 us direct, 7.98 / 7.71 -> 5.95 / 5.96 us as a stream call;
    // at 2^20 samples (one such tile a slot) 6.93 -> 8.39 us, so larger calls keep the 512-output tiles
    if (2 * ceil_div<uint64_t>(j.N, 256) <= slots) {
      return launch_poly<TapT, InT, 4, 1, 16, 256, MODE, 0, true, false, 0, false, 4>(j, s);
    }
#endif
    if (ceil_div<uint64_t>(j.N, 1024) < 3 * slots) {
      return launch_poly<TapT, InT, 4, 2, 16, 256, MODE, 0, true, false, 0, false, 2>(j, s);
    }
  }
  // (one NCO cell grid for every D = 4 shape -- 1,024 outputs for AM, 1,020 for FM -- so the three give the same
  // outputs bit for bit)
  return launch_poly_default<TapT, InT, 4, 4, 16, 256, MODE>(j, s);
}

// Runtime-decimation tile kernel (k_fir_rt) for decimations without a compile-time shape, when taps
// overlap between outputs (T > D): the widest workgroup (256, 128 or 64 outputs a tile) whose tile fits
// the LDS budget; otherwise the generic kernel.
template <class TapT, class InT, int MODE, int WG>
hipError_t launch_rt_wg(const FirJob& j, uint32_t nch, size_t lds, hipStream_t s) {
  constexpr int IC = 16;
  FirParams p = make_params(j);
  p.nch = nch;
  const uint32_t stride = (MODE == kModeFm) ? fm_tile_stride<InT>(WG, j.D) : WG;
  p.tile_stride = stride;
  const uint64_t tiles = ceil_div<uint64_t>(j.N, stride);
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  constexpr uint64_t A = SampleT<InT>::kSrcAlign;
  const bool vec = (reinterpret_cast<uintptr_t>(j.in) % A) == 0 && ((uint64_t)stride * j.D * sizeof(InT)) % A == 0;
  const dim3 grid((uint32_t)tiles), block(WG);
  if (j.D % 2 == 0) {  // paired LDS reads (k_fir_rt): same products, same order
    if (vec) {
      k_fir_rt<TapT, InT, IC, WG, true, MODE, true><<<grid, block, lds, s>>>(p);
    } else {
      k_fir_rt<TapT, InT, IC, WG, false, MODE, true><<<grid, block, lds, s>>>(p);
    }
  } else if (vec) {
    k_fir_rt<TapT, InT, IC, WG, true, MODE><<<grid, block, lds, s>>>(p);
  } else {
    k_fir_rt<TapT, InT, IC, WG, false, MODE><<<grid, block, lds, s>>>(p);
  }
  return launch_status();
}

template <class TapT, class InT, int MODE>
hipError_t launch_rt(const FirJob& j, hipStream_t s) {
  constexpr int IC = 16;
  if (j.stream_tiled) return hipErrorNotSupported;
  if (j.T <= j.D || j.D > 4096) return launch_generic<TapT, InT, MODE>(j, s);
  const uint32_t nch = (uint32_t)ceil_div<uint64_t>(j.T, (uint64_t)IC);
  const uint32_t D = (uint32_t)j.D, span = nch * IC;
  size_t lds = rt_lds_bytes<InT>(D, span, 256, MODE);
  if (lds <= kMaxTileLds) return launch_rt_wg<TapT, InT, MODE, 256>(j, nch, lds, s);
  lds = rt_lds_bytes<InT>(D, span, 128, MODE);
  if (lds <= kMaxTileLds) return launch_rt_wg<TapT, InT, MODE, 128>(j, nch, lds, s);
  lds = rt_lds_bytes<InT>(D, span, 64, MODE);
  if (lds <= kMaxTileLds) return launch_rt_wg<TapT, InT, MODE, 64>(j, nch, lds, s);
  return launch_generic<TapT, InT, MODE>(j, s);
}

template <class InT, int D, int R, int IC, int WG>
constexpr bool contig_fits_lds_at_t127() {
  constexpr uint32_t span = (127 + IC - 1) / IC * IC;
  return poly_lds_bytes<InT, D, R, WG>(span, kModeFm) <= kMaxTileLds;
}

template <class TapT, class InT, int D, int R, int IC, int WG, int MODE>
hipError_t launch_contig_default(const FirJob& j, hipStream_t s) {
  static_assert(contig_fits_lds_at_t127<InT, D, R, IC, WG>(), "default contiguous shape exceeds the LDS budget");
  return launch_contig<TapT, InT, D, R, IC, WG, MODE>(j, s);
}

// Decimations without a polyphase column layout (odd D, or real D not a multiple of 4) and the large
// even ones: the contiguous-window kernel with R outputs a thread (R * D whole granules) or a one-row
// polyphase tile. The one-output-per-thread generic kernel ran these 10-20x slower.
template <class TapT, class InT, int MODE>
hipError_t launch_other_d(const FirJob& j, hipStream_t s) {
  constexpr bool kComplexIn = SampleT<InT>::kPerGranule == 2;
  switch (j.D) {
    // (tap chunks of 24-40: every chunk costs one scalar tap-load wait)
    case 3:
      return launch_contig_default<TapT, InT, 3, 4, (kComplexIn ? 24 : 36), 256, MODE>(j, s);
    case 5:
      return launch_contig_default<TapT, InT, 5, 4, (kComplexIn ? 20 : 40), 128, MODE>(j, s);
    case 6:
      if constexpr (kComplexIn) {
        return launch_poly_default<TapT, InT, 6, 2, 8, 256, MODE>(j, s);
      } else {
        return launch_contig_default<TapT, InT, 6, 2, 36, 256, MODE>(j, s);
      }
    case 7:
      return launch_contig_default<TapT, InT, 7, 4, 28, 128, MODE>(j, s);
    case 10:
      if constexpr (kComplexIn) {
        return launch_poly_default<TapT, InT, 10, 2, 8, 256, MODE>(j, s);
      } else {
        return launch_contig_default<TapT, InT, 10, 2, 40, 256, MODE>(j, s);
      }
    case 12:
      if constexpr (kComplexIn) {
        return launch_poly_default<TapT, InT, 12, 2, 8, 256, MODE>(j, s);
      } else {
        return launch_poly_default<TapT, InT, 12, 4, 8, 128, MODE>(j, s);
      }
    case 16:
      return launch_poly_default<TapT, InT, 16, (kComplexIn ? 2 : 4), 8, 128, MODE>(j, s);
    // large even D: one output a thread on a polyphase tile (odd padded lane stride, conflict-free
    // reads), where the runtime-D kernel's lane stride of D samples hits one LDS bank over and over
    case 20:
      return launch_poly_default<TapT, InT, 20, 1, 8, 256, MODE>(j, s);
    case 24:
      return launch_poly_default<TapT, InT, 24, 1, 8, 256, MODE>(j, s);
    case 32:
      return launch_poly_default<TapT, InT, 32, 1, 8, (kComplexIn ? 128 : 256), MODE>(j, s);
    case 40:
      return launch_poly_default<TapT, InT, 40, 1, 8, (kComplexIn ? 128 : 256), MODE>(j, s);
    case 48:
      return launch_poly_default<TapT, InT, 48, 1, 8, 128, MODE>(j, s);
    case 64:
      return launch_poly_default<TapT, InT, 64, 1, 8, (kComplexIn ? 64 : 128), MODE>(j, s);
    default:
      return launch_rt<TapT, InT, MODE>(j, s);
  }
}

template <class TapT, class InT, int MODE>
hipError_t launch_fir(const FirJob& j, hipStream_t s) {
  constexpr bool kComplexIn = SampleT<InT>::kPerGranule == 2;
  // the tiled kernels address taps through a 32-bit buffer descriptor
  if (j.T > (1u << 26)) return launch_generic<TapT, InT, MODE>(j, s);
  if constexpr (std::is_same<InT, Iq8>::value) {
    // int8 I/Q
    if constexpr (MODE == kModeFir) {
      if (j.D == 4 && j.variant >= 0) return launch_d4_int8(j, s);
    }
    // D = 4 FM / AM chains: the matrix-core kernel with the NCO folded into complex taps (normwise
    // parity with the float chains: DESIGN.md section 3.3); variant 0 keeps the exact path (streams)
    if constexpr (MODE != kModeFir && std::is_same<TapT, float>::value) {
      if (j.D == 4 && j.variant < 0 && !j.stream_tiled && j.T <= (size_t)I8ChainMfma<MODE>::MAXT) {
        return launch_chain_i8_mfma<MODE>(j, s);
      }
    }
    // D = 4 FIR: the matrix-core kernel (bf16-exact samples, exact three-part taps; normwise parity with
    // the float path, twice its speed: DESIGN.md section 3.3)
    if constexpr (MODE == kModeFir && std::is_same<TapT, float>::value) {
      if (j.D == 4 && !j.stream_tiled && j.T <= (size_t)I8Mfma<4, 8>::MAXT &&
          (reinterpret_cast<uintptr_t>(j.out) % 8) == 0) {
        return launch_i8_mfma<4, 3>(j, s);
      }
    }
    // otherwise the float-input shapes, so int8 and float inputs of one decimation give bit-identical
    // outputs
    switch (j.D) {
      case 1:
        return launch_contig<TapT, InT, 1, 8, 16, 256, MODE>(j, s);
      case 2:
        return launch_poly_default<TapT, InT, 2, 8, 16, 128, MODE>(j, s);
      case 4:
        return launch_poly_d4<TapT, InT, MODE>(j, s);
      case 8:
        return launch_poly_default<TapT, InT, 8, 2, 8, 256, MODE>(j, s);
      default:
        return launch_other_d<TapT, InT, MODE>(j, s);
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
        // 4 waves/SIMD (16 per CU): the shape that measured fastest at T = 127; smaller tiles
        // for short calls
        return launch_poly_d4<TapT, InT, MODE>(j, s);
      case 8:
        return launch_poly_default<TapT, InT, 8, 2, 8, 256, MODE>(j, s);
      default:
        return launch_other_d<TapT, InT, MODE>(j, s);
    }
  } else {
    switch (j.D) {
      case 1:
        // complex taps on real samples: R = 16 with 32 two-float taps in flight spilled to scratch
        if constexpr (!std::is_same<TapT, float>::value) {
          return launch_contig<TapT, InT, 1, 8, 16, 256, MODE>(j, s);
        } else {
          return launch_contig<TapT, InT, 1, 16, 32, 256, MODE>(j, s);
        }
      case 2:
        return launch_contig<TapT, InT, 2, 8, 16, 256, MODE>(j, s);
      case 4:
        return launch_poly_default<TapT, InT, 4, 8, 8, 128, MODE>(j, s);
      case 8:
        return launch_poly_default<TapT, InT, 8, 8, 8, 128, MODE>(j, s);
      default:
        return launch_other_d<TapT, InT, MODE>(j, s);
    }
  }
}

// The streaming object's one-launch step on the tiled kernels (stream.hip): outputs [0, N) of the call,
// output 0's window at chunk offset j.in_off (negative: it starts in the history j.hist of j.hist_len
// samples), the next history (chunk offsets [hist_from, + hist_n)) copied by workgroup 0 of the same
// launch. j.in is the chunk and j.L its length here. The kernels are the monolithic call's, tile for tile,
// so the outputs are bit-identical to it. hipErrorNotSupported (nothing launched) when the shape runs
// another kernel; the stream then takes its seam path.
template <class InT, int MODE>
hipError_t stream_step_tiled(FirJob j, hipStream_t s) {
  if (j.N == 0 || j.T == 0 || j.taps == nullptr || j.T > (1u << 26)) return hipErrorNotSupported;
  j.stream_tiled = true;
  j.variant = -1;
  j.in = static_cast<const InT*>(j.in) + j.in_off;  // output 0's window (may precede the chunk)
  j.L = (uint64_t)((int64_t)j.L - j.in_off);         // samples readable from there
  return launch_fir<float, InT, MODE>(j, s);
}

}  // namespace gsdr
