// gsdr-mi355x: the decimating-FIR engine behind gsdrFir*, gsdrFmDemod and gsdrAmDemod.
//
// What it computes (reference src/fir.cu:26-71):
//     y[k] = sum_{i<T} x[k*D + i] * t[i]
// optionally with an NCO mix applied to x first (reference src/adjustFrequency.cu:25-56, re-specified in
// SURVEY.md App. A.3) and a demodulator epilogue (FM: reference src/fm.cu:59-68, AM: src/am.cu:49).
//
// How (MI355X / gfx950, wave64, 160 KiB LDS per CU):
//   * One workgroup owns a tile of KT = WG * R consecutive outputs. It stages the tile's input span
//     (KT*D + taps samples) from HBM into LDS with 16-byte loads (one "granule" = 2 complex or 4 real
//     samples); the NCO mix, when present, is applied once per staged sample on the way in.
//   * Each thread then computes R consecutive outputs from a register-resident sliding window read out
//     of LDS with ds_read_b128, so each staged sample is read from LDS ~(R+JC-1)/R times instead of
//     T/D times. Taps are wave-uniform: they are read with scalar loads straight into SGPR operands of
//     the FMAs (no VGPRs, no LDS traffic for taps).
//   * Decimation D that is a multiple of the granule width is handled polyphase: a granule holds G
//     consecutive phases of one input "row" (D samples), and the window for one granule column only
//     carries the phases that meet the taps t[j*D + h*G + e] in flight -- no wasted window registers.
//   * A thread's segment is SG granules; when SG is even a one-granule pad is inserted after each
//     segment so the per-lane stride is odd and the 16-lane groups of ds_read_b128 are bank-conflict
//     free, while every window offset stays a compile-time constant.
//   * Input may also be interleaved int8 I/Q (Iq8): converted to float as it is staged, so the float
//     samples exist only in LDS. HBM loads and FIR stores are non-temporal (streamed once).
//   * The default core is packed VALU. An exact-f32 matrix-core core (k_fir_mfma_bc, 4x4x1 outer
//     products with broadcast taps, bit-identical to the oracle) exists as a variant; it runs at a
//     higher clock under the cap but needs more cycles and more energy per launch (4 % slower). The
//     kernel is bound by the part's 1400 W power cap with staging and MACs together.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace gsdr {

// ------------------------------------------------------------------------------------------------
// Sample and product types
// ------------------------------------------------------------------------------------------------
// Interleaved int8 I/Q (2 bytes per sample, the SDR front-end format): converted to float while
// staging with gsdrInt8ToNormFloat's semantics (reference src/conversion.cu:26), so the float
// samples exist only in LDS.
struct Iq8 {
  int8_t x, y;
};

// kPerGranule: samples per 16-byte LDS granule. kSrcAlign: bytes one staging load moves from HBM
// per granule (the alignment the vector path needs).
template <class T>
struct SampleT;
template <>
struct SampleT<float> {
  static constexpr int kPerGranule = 4;
  static constexpr int kSrcAlign = 16;
};
template <>
struct SampleT<float2> {
  static constexpr int kPerGranule = 2;
  static constexpr int kSrcAlign = 16;
};
template <>
struct SampleT<Iq8> {
  static constexpr int kPerGranule = 2;
  static constexpr int kSrcAlign = 4;
};

// sample type as held in LDS (what the compute core reads)
template <class T>
struct LdsSample {
  using type = T;
};
template <>
struct LdsSample<Iq8> {
  using type = float2;
};

// max(-1, v / 127.0f) with IEEE division, from one multiply and an fma correction: equal to the
// correctly rounded quotient for every int8 value (checked exhaustively, tests/test_gpu_int8.py);
// clamping to -127 first gives the reference's max(-1, .) for -128.
__device__ __forceinline__ float norm_i8(int v) {
  const float x = (float)max(v, -127);
  constexpr float r = 1.0f / 127.0f;
  const float q = x * r;
  return fmaf(fmaf(-q, 127.0f, x), r, q);
}
__device__ __forceinline__ float2 to_lds_sample(Iq8 v) { return make_float2(norm_i8(v.x), norm_i8(v.y)); }
__device__ __forceinline__ float2 to_lds_sample(float2 v) { return v; }
__device__ __forceinline__ float to_lds_sample(float v) { return v; }

// two Iq8 samples packed in a dword -> one LDS granule
__device__ __forceinline__ float4 iq8x2_granule(uint32_t w) {
  const int b0 = (int)(w << 24) >> 24, b1 = (int)(w << 16) >> 24, b2 = (int)(w << 8) >> 24, b3 = (int)w >> 24;
  return make_float4(norm_i8(b0), norm_i8(b1), norm_i8(b2), norm_i8(b3));
}

template <class TapT, class InT>
struct Product {
  using type = float2;
};
template <>
struct Product<float, float> {
  using type = float;
};

__device__ __forceinline__ void set_zero(float& a) { a = 0.0f; }
__device__ __forceinline__ void set_zero(float2& a) { a = make_float2(0.0f, 0.0f); }
__device__ __forceinline__ void set_zero(Iq8& a) {
  a.x = 0;
  a.y = 0;
}

// Element e (compile-time after unrolling) of a 16-byte granule.
template <class InT>
__device__ __forceinline__ InT granule_sample(const float4& g, int e);
template <>
__device__ __forceinline__ float granule_sample<float>(const float4& g, int e) {
  return e == 0 ? g.x : (e == 1 ? g.y : (e == 2 ? g.z : g.w));
}
template <>
__device__ __forceinline__ float2 granule_sample<float2>(const float4& g, int e) {
  return e == 0 ? make_float2(g.x, g.y) : make_float2(g.z, g.w);
}

// acc += x * t, with the component products of the reference's cuComplex operator overloads
// (reference src/cuComplexOperatorOverloads.cuh:25-33: c*r, r*c, cuCmulf).
__device__ __forceinline__ void mac(float& acc, float x, float t) { acc = fmaf(x, t, acc); }
__device__ __forceinline__ void mac(float2& acc, float2 x, float t) {
  acc.x = fmaf(x.x, t, acc.x);
  acc.y = fmaf(x.y, t, acc.y);
}
__device__ __forceinline__ void mac(float2& acc, float x, float2 t) {
  acc.x = fmaf(t.x, x, acc.x);
  acc.y = fmaf(t.y, x, acc.y);
}
__device__ __forceinline__ void mac(float2& acc, float2 x, float2 t) {
  acc.x = fmaf(x.x, t.x, acc.x);
  acc.x = fmaf(-x.y, t.y, acc.x);
  acc.y = fmaf(x.x, t.y, acc.y);
  acc.y = fmaf(x.y, t.x, acc.y);
}

// Taps are fetched with scalar buffer loads (s_buffer_load_dword{,x2,x4,x8}) through a buffer
// descriptor whose range is exactly the caller's T taps: the hardware range check returns 0 for the
// zero-padding past T, so no clamp/select instructions are needed and the tap lands directly in the
// SGPR operand of v_pk_fma_f32 (broadcast with op_sel_hi).
typedef int gsdr_v4i32 __attribute__((ext_vector_type(4)));
__device__ float gsdr_s_buffer_load_f32(gsdr_v4i32 rsrc, int offset, int aux) __asm("llvm.amdgcn.s.buffer.load.f32");

struct TapBuf {
  gsdr_v4i32 rsrc;
};

// A window of the tap array starting at tap `base` (wave-uniform): the descriptor is re-based so
// every tap inside the window is an immediate offset, which lets the compiler merge neighbouring
// taps into s_buffer_load_dwordx2/x4/x8 and wait for the whole batch once.
template <class TapT>
__device__ __forceinline__ TapBuf tap_window(const void* taps, uint32_t T, uint32_t base) {
  const uint64_t a = reinterpret_cast<uint64_t>(reinterpret_cast<const TapT*>(taps) + base);
  const uint32_t bytes = base < T ? (T - base) * (uint32_t)sizeof(TapT) : 0u;
  TapBuf b;
  b.rsrc = gsdr_v4i32{(int)(uint32_t)a, (int)(uint32_t)(a >> 32) & 0xffff, (int)bytes, 0x00020000};
  return b;
}

// Tap `i` (a compile-time constant after unrolling) of a window; past T it reads as zero.
template <class TapT>
__device__ __forceinline__ TapT tap_at(const TapBuf& tb, int i);
template <>
__device__ __forceinline__ float tap_at<float>(const TapBuf& tb, int i) {
  return gsdr_s_buffer_load_f32(tb.rsrc, i * 4, 0);
}
template <>
__device__ __forceinline__ float2 tap_at<float2>(const TapBuf& tb, int i) {
  return make_float2(gsdr_s_buffer_load_f32(tb.rsrc, i * 8, 0), gsdr_s_buffer_load_f32(tb.rsrc, i * 8 + 4, 0));
}

// ------------------------------------------------------------------------------------------------
// Launch parameters (one struct for every mode; passed by value)
// ------------------------------------------------------------------------------------------------
enum Mode : int { kModeFir = 0, kModeFm = 1, kModeAm = 2 };

struct FirParams {
  const void* in;
  const void* taps;
  void* out;
  uint64_t L;            // input samples readable
  uint64_t N;            // outputs to write
  uint32_t T;            // tap count (>= 1)
  uint32_t nch;          // tap chunks per phase column
  uint32_t tile_stride;  // outputs advanced per tile (KT, or KT - 1 for the FM discriminator)
  uint32_t D;            // decimation (used by the generic kernel)
  uint32_t nco_inc;      // NCO phase increment per sample, 2^-32 cycles
  uint32_t nco_n0;       // low 32 bits of firstSampleIndex
  float fm_gain;         // FM discriminator gain
  uint32_t out_phase;    // absolute index of output 0 mod 16 (the int8 matrix-core kernels' block grid)
  // Anchored chains (the polyphase kernels in FM / AM mode, anchored_nco below): tile t covers outputs
  // [t KT - tile_shift, (t + 1) KT - tile_shift) of the call, and tile 0 is sub-tile cell_sub0 of its NCO cell.
  uint32_t tile_shift;
  uint32_t cell_sub0;
  // The streaming object's one-launch path (stream.hip): output 0's window starts at sample in_off of the
  // caller's chunk; chunk samples at negative offsets i >= -hist_len come from hist[hist_len + i] (the
  // stream's history), and samples [hist_from, hist_from + hist_n) (same offsets) are copied to hist_out
  // (the next history) by workgroup 0. The int8 matrix-core kernels (fir_i8_mfma.hpp) take `in` = the
  // chunk and L = its length; the tiled kernels below take `in` = chunk + in_off (output 0's window, so
  // the tile arithmetic is unchanged; the pointer may precede the chunk, and samples before it are read
  // only through the history) and L = samples readable from there.
  int64_t in_off;
  const void* hist;
  uint64_t hist_len;
  void* hist_out;
  int64_t hist_from;
  uint64_t hist_n;
};

// ------------------------------------------------------------------------------------------------
// NCO: exact integer phase P(n) = n * inc mod 2^32 from the absolute sample
// index n, turned into a unit phasor by a fixed function of n alone, so any split of a stream into
// calls (and any tiling inside a call) mixes every sample with bit-identical values:
//   n even: (cos, sin)(2 pi P(n) / 2^32) from the hardware v_cos_f32 / v_sin_f32, whose argument is
//           in revolutions (max abs error 1.9e-7 measured over 2^28 phases, tools/nco_accuracy.hip;
//           the (int32)P -> float rounding adds <= 2^-25 revolutions, as sincospif did);
//   n odd:  phasor(n - 1) rotated by w = phasor of one step (P = inc).
// One transcendental pair per two samples: the mixer was a third of the FM chain's VALU work with
// a sincospif per sample.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float2 nco_direct(uint32_t phase) {
  const float r = (float)(int32_t)phase * 0x1p-32f;  // revolutions in [-0.5, 0.5)
  return make_float2(__builtin_amdgcn_cosf(r), __builtin_amdgcn_sinf(r));
}

// a * b with explicit fmas: (fma(a.x, b.x, -(a.y b.y)), fma(a.x, b.y, a.y b.x)). Written on
// two-lane vectors so it is one v_pk_mul_f32 (a.y * (-b.y, b.x)) and one v_pk_fma_f32 (a.x * b + that), plus the
// swapped, negated b (one more v_pk_mul_f32 by (1, -1), hoisted when b is a loop constant); the library builds with
// -ffp-contract=off, so the rounding is fixed here rather than left to the contraction pass. (Round 6 tried the
// sign as a neg_lo source modifier of the v_pk_mul_f32, written as inline asm -- the compiler never forms it for
// packed F32 -- which saves that instruction for every product whose b varies, e.g. each staged granule's NCO mix.
// An isolated check agreed bit for bit on 2^22 products, but inside the chain kernels the results were wrong (109
// GPU tests failed), so it is not used.)
typedef float gsdr_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  const gsdr_f32x2 bv = gsdr_f32x2{b.x, b.y};
  // (-b.y, b.x) as b swapped times (-1, 1) (exact): one v_pk_mul_f32, where building it with a sign flip
  // and a move took two instructions
  const gsdr_f32x2 t = gsdr_f32x2{a.y, a.y} * (bv.yx * gsdr_f32x2{-1.0f, 1.0f});
  const gsdr_f32x2 r = __builtin_elementwise_fma(gsdr_f32x2{a.x, a.x}, bv, t);
  return make_float2(r.x, r.y);
}

// phasor of absolute sample n (low 32 bits suffice: P is taken mod 2^32)
__device__ __forceinline__ float2 nco_phasor(uint32_t n, uint32_t inc) {
  const float2 w = nco_direct(inc);
  const float2 e = nco_direct((n & ~1u) * inc);
  return (n & 1u) ? cmul(e, w) : e;
}

__device__ __forceinline__ float2 nco_mix(float2 x, uint32_t n, uint32_t inc) { return cmul(x, nco_phasor(n, inc)); }

// ------------------------------------------------------------------------------------------------
// Tile geometry
// ------------------------------------------------------------------------------------------------
template <class InT, int D, int R, int WG>
struct TileGeo {
  static constexpr int G = SampleT<InT>::kPerGranule;
  static_assert((R * D) % G == 0, "a thread segment must be whole granules");
  static constexpr int SG = R * D / G;             // granules per thread segment
  static constexpr int PAD = (SG % 2 == 0) ? 1 : 0;  // odd lane stride -> conflict-free ds_read_b128
  static constexpr int SGP = SG + PAD;
  static constexpr int KT = WG * R;                  // outputs per tile
  static constexpr int ROUT = R;                     // outputs per segment
  __host__ __device__ static constexpr uint32_t padded(uint32_t g) { return g + PAD * (g / SG); }
};

// Non-temporal (streaming) 16-byte load: global_load_dwordx4 ... nt.
typedef float gsdr_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 load16_nt(const float4* p) {
  const gsdr_f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const gsdr_f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// 16 bytes = G consecutive samples starting at s; samples at or past L read as zero.
template <class InT, bool VEC>
__device__ __forceinline__ float4 load_granule(const InT* __restrict__ in, uint64_t s, uint64_t L) {
  constexpr int G = SampleT<InT>::kPerGranule;
  // (an anchored chain's first tile starts before the call's first sample: its local indices below 0 arrive
  // wrapped, and those granules -- whole granules, since tiles start at even samples -- read as zero)
  if ((int64_t)s < 0) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if constexpr (std::is_same<InT, Iq8>::value) {
    if (VEC && s + 2 <= L) return iq8x2_granule(*reinterpret_cast<const uint32_t*>(in + s));
    float2 a = make_float2(0.0f, 0.0f), b = a;
    if (s < L) a = to_lds_sample(in[s]);
    if (s + 1 < L) b = to_lds_sample(in[s + 1]);
    return make_float4(a.x, a.y, b.x, b.y);
  } else if (VEC && s + G <= L) {
    return *reinterpret_cast<const float4*>(in + s);
  }
  float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if constexpr (G == 2) {
    if (s < L) {
      const float2 a = reinterpret_cast<const float2*>(in)[s];
      r.x = a.x;
      r.y = a.y;
    }
    if (s + 1 < L) {
      const float2 b = reinterpret_cast<const float2*>(in)[s + 1];
      r.z = b.x;
      r.w = b.y;
    }
  } else {
    const float* f = reinterpret_cast<const float*>(in);
    if (s < L) r.x = f[s];
    if (s + 1 < L) r.y = f[s + 1];
    if (s + 2 < L) r.z = f[s + 2];
    if (s + 3 < L) r.w = f[s + 3];
  }
  return r;
}

// NCO mixing of one granule (two complex samples n, n + 1) given ph = n * inc mod 2^32, the phase of
// its first sample; `odd` = n & 1 (wave-uniform in the tiled kernels: they stage granules at even
// offsets from the tile start). The phasor is a pure function of the absolute index: even n from
// nco_direct, odd n = phasor(n - 1) * w, w = nco_direct(inc).
template <class InT, int MODE>
__device__ __forceinline__ float4 stage_transform_ph(float4 v, uint32_t ph, bool odd, uint32_t inc) {
  if constexpr (MODE != kModeFir) {
    static_assert(SampleT<InT>::kPerGranule == 2, "NCO modes take complex input");
    const float2 w = nco_direct(inc);
    float2 ea, eb;
    if (odd) {
      ea = cmul(nco_direct(ph - inc), w);
      eb = nco_direct(ph + inc);
    } else {
      ea = nco_direct(ph);
      eb = cmul(ea, w);
    }
    const float2 a = cmul(make_float2(v.x, v.y), ea);
    const float2 b = cmul(make_float2(v.z, v.w), eb);
    v = make_float4(a.x, a.y, b.x, b.y);
  }
  return v;
}

// s = local sample index of a granule's first sample (only its low 32 bits matter: the NCO phase is
// taken mod 2^32).
template <class InT, int MODE>
__device__ __forceinline__ float4 stage_transform(float4 v, uint32_t s, const FirParams& p) {
  if constexpr (MODE != kModeFir) {
    const uint32_t n = p.nco_n0 + s;  // absolute index of the granule's first sample mod 2^32
    return stage_transform_ph<InT, MODE>(v, n * p.nco_inc, __builtin_amdgcn_readfirstlane(n & 1u) != 0, p.nco_inc);
  }
  return v;
}

// Phase walk of a thread's tile-body granules: granule g = k * WG + tid of a tile starting at S0 has
// phase ph0 + k * step (mod 2^32) -- the same integer as (n0 + S0 + g * G) * inc, so the phasors
// are unchanged, without a 32-bit integer multiply (a quarter-rate instruction) per granule.
struct PhaseWalk {
  uint32_t ph0, step, inc;
  bool odd;
};

template <int G, int WG>
__device__ __forceinline__ PhaseWalk phase_walk(uint32_t n0, uint64_t S0, uint32_t inc) {
  const uint32_t n = n0 + (uint32_t)S0 + (uint32_t)(threadIdx.x * G);
  return PhaseWalk{n * inc, (uint32_t)(WG * G) * inc, inc, __builtin_amdgcn_readfirstlane(n & 1u) != 0};
}

// granules per staging batch: the largest divisor of the per-thread count that is at most 8
constexpr int staging_batch(int bpt) {
  for (int b = 8; b > 1; --b) {
    if (bpt % b == 0) return b;
  }
  return 1;
}

// Stage granules [0, NG) of the tile starting at global sample S0 into LDS (padded layout).
// The first SG*WG granules (the tile body) are loaded fully unrolled so every HBM load is in flight
// before the first LDS write; the remaining halo granules follow in a short strided loop.
// Tile body by LDS-DMA (global_load_lds_dwordx4: HBM -> LDS with no VGPR round trip and no ds_write).
// One wave instruction fills 64 consecutive LDS slots; the padded layout is kept by choosing each
// lane's SOURCE granule (slot s holds granule s - s / SGP of its segment; pad slots are skipped with
// the lane masked off). Returns false when the tile does not qualify (then nothing was issued).
template <class InT, class Geo, int WG, int MODE, bool NT>
__device__ __forceinline__ bool stage_body_dma(float4* __restrict__ lds, const InT* __restrict__ in, uint64_t S0) {
  if constexpr (!std::is_same<InT, float2>::value || MODE != kModeFir) {
    return false;
  } else {
    constexpr int BODY = Geo::SG * (Geo::KT / Geo::ROUT);  // body granules
    constexpr int SLOTS = BODY / Geo::SG * Geo::SGP;
    static_assert(SLOTS % 64 == 0 && (SLOTS / 64) % (WG / 64) == 0, "body slots must split into wave instructions");
    constexpr int PER_WAVE = SLOTS / 64 / (WG / 64);
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const float4* __restrict__ src = reinterpret_cast<const float4*>(in + S0);
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const uint32_t base = (uint32_t)(i * (WG / 64) + w) * 64u;  // wave-uniform first slot
      const uint32_t sl = base + lane;
      const uint32_t within = sl % Geo::SGP;
      if (within < (uint32_t)Geo::SG) {
        const uint32_t g = (sl / Geo::SGP) * Geo::SG + within;
        __builtin_amdgcn_global_load_lds((const void*)(src + g), (void __attribute__((address_space(3)))*)(lds + base),
                                         16, 0, NT ? 2 : 0);
      }
    }
    return true;
  }
}

// Streaming one-launch path (FirParams::hist != nullptr): local sample s of the tiled kernels (counted
// from output 0's window start, `in` = chunk + in_off) is chunk sample s + in_off; the ones before the
// chunk come from the history. Samples at or past L read as zero.
template <class InT>
__device__ __forceinline__ typename LdsSample<InT>::type stream_sample(const InT* __restrict__ in,
                                                                        const FirParams& p, uint64_t s) {
  using LdsT = typename LdsSample<InT>::type;
  if (s >= p.L) {
    LdsT z;
    set_zero(z);
    return z;
  }
  const int64_t i = (int64_t)s + p.in_off;
  return i < 0 ? to_lds_sample(reinterpret_cast<const InT*>(p.hist)[(int64_t)p.hist_len + i]) : to_lds_sample(in[s]);
}

// A tile that reaches into the stream's history (only the first tile of a call: the history is shorter
// than one window): sample by sample, each from the history or the chunk (stream_sample's rule), in batches of
// 8 granules a thread whose loads are all issued before the first is used (one granule at a time, this tile
// had waited on every load in turn and ran ~1 us longer than the call's other tiles).
template <class InT, class Geo, int WG, int MODE>
__device__ __forceinline__ void stage_tile_stream(float4* __restrict__ lds, const InT* __restrict__ in, uint64_t S0,
                                                  uint32_t NG, const FirParams& p) {
  constexpr int G = Geo::G;
  constexpr int B = 8;
  const InT* __restrict__ hist = reinterpret_cast<const InT*>(p.hist);
  for (uint32_t g0 = 0; g0 < NG; g0 += B * WG) {
    InT v[B][G];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint32_t g = g0 + (uint32_t)b * WG + threadIdx.x;
#pragma unroll
      for (int e = 0; e < G; ++e) {
        const uint64_t s = S0 + (uint64_t)g * G + (uint64_t)e;
        const int64_t i = (int64_t)s + p.in_off;
        if (g < NG && s < p.L) {
          v[b][e] = i < 0 ? hist[(int64_t)p.hist_len + i] : in[s];
        } else {
          set_zero(v[b][e]);
        }
      }
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint32_t g = g0 + (uint32_t)b * WG + threadIdx.x;
      if (g >= NG) break;
      float4 w;
      if constexpr (G == 2) {
        const float2 a = to_lds_sample(v[b][0]), c = to_lds_sample(v[b][1]);
        w = make_float4(a.x, a.y, c.x, c.y);
      } else {
        w = make_float4(v[b][0], v[b][1], v[b][2], v[b][3]);
      }
      lds[Geo::padded(g)] = stage_transform<InT, MODE>(w, (uint32_t)(S0 + (uint64_t)g * G), p);
    }
  }
}

// The next history of a streaming call, copied by workgroup 0 (it writes the stream's spare buffer, which no
// tile reads). Split so that it costs the workgroup no round trip of its own: each thread loads its sample
// before the tile's loads are issued (stream_history_load) and stores it after the staging, whose waits
// have covered that load (stream_history_store). Histories longer than the workgroup (T + D > WG samples)
// copy the rest there with a plain loop.
template <class InT>
struct HistSample {
  InT v;
  bool on;
};
template <class InT>
__device__ __forceinline__ HistSample<InT> stream_history_load(const FirParams& p) {
  HistSample<InT> h{};
  h.on = p.hist_out != nullptr && blockIdx.x == 0 && threadIdx.x < p.hist_n;
  if (h.on) {
    const int64_t i = p.hist_from + (int64_t)threadIdx.x;  // chunk offset
    h.v = i < 0 ? reinterpret_cast<const InT*>(p.hist)[(int64_t)p.hist_len + i]
                : reinterpret_cast<const InT*>(p.in)[i - p.in_off];
  }
  return h;
}
template <class InT>
__device__ __forceinline__ void stream_history_store(const FirParams& p, const HistSample<InT>& h) {
  if (p.hist_out == nullptr || blockIdx.x != 0) return;
  InT* __restrict__ dst = reinterpret_cast<InT*>(p.hist_out);
  if (h.on) dst[threadIdx.x] = h.v;
  for (uint64_t j = threadIdx.x + blockDim.x; j < p.hist_n; j += blockDim.x) {
    const int64_t i = p.hist_from + (int64_t)j;
    dst[j] = i < 0 ? reinterpret_cast<const InT*>(p.hist)[(int64_t)p.hist_len + i]
                   : reinterpret_cast<const InT*>(p.in)[i - p.in_off];
  }
}

// The first halo granule of a tile, loaded ahead of the body's loads so that both arrive in one round trip (after
// the body, it was a second dependent round trip per tile: what a short call's few tiles wait for). The load is
// one predicated instruction with the raw word(s) kept until the body has been staged: a bounds-checked
// load_granule there made the compiler wait for it on the spot (its branches merge through register copies).
template <class InT>
struct HaloRaw {
  using type = float4;
};
template <>
struct HaloRaw<Iq8> {
  using type = uint32_t;
};
template <class InT, bool VEC>
struct HaloPre {
  // (left indeterminate where nothing is loaded -- get() never returns it then. A zero there, or
  // __builtin_nondeterministic_value, which the compiler also materialises as zero, cost a register copy right
  // behind the load, i.e. a wait for it)
  typename HaloRaw<InT>::type raw;
  uint64_t s;
  uint32_t g;
  bool fast;
  __device__ __forceinline__ HaloPre(uint64_t S0, uint32_t g0, uint32_t NG, uint64_t L)
      : s(S0 + (uint64_t)g0 * SampleT<InT>::kPerGranule), g(g0) {
    fast = VEC && g0 < NG && (int64_t)s >= 0 && s + SampleT<InT>::kPerGranule <= L;
  }
  // issued right after the body's first batch of loads (issued before them, it drew a full wait ahead of them)
  __device__ __forceinline__ void issue(const InT* __restrict__ in) {
    if (fast) raw = *reinterpret_cast<const typename HaloRaw<InT>::type*>(in + s);
  }
  // the granule (only for g < NG). The empty asm re-defines the raw registers here, so the register copies the
  // allocator makes of the loaded value come after this point and the wait for the load with them, not right
  // behind the load.
  __device__ __forceinline__ float4 get(const InT* __restrict__ in, uint64_t L) const {
    typename HaloRaw<InT>::type r = raw;
    if constexpr (std::is_same<InT, Iq8>::value) {
      asm volatile("" : "+v"(r));
      return fast ? iq8x2_granule(r) : load_granule<InT, VEC>(in, s, L);
    } else {
      gsdr_f32x4 q{r.x, r.y, r.z, r.w};
      asm volatile("" : "+v"(q));
      return fast ? make_float4(q[0], q[1], q[2], q[3]) : load_granule<InT, VEC>(in, s, L);
    }
  }
};

// SH (complex or int8 I/Q samples): the input is one sample off its aligned granule load (complex: 8 bytes
// off 16; int8 I/Q: 2 bytes off 4) at every tile start. The tile
// body is then loaded as aligned 16-byte granules starting one sample early, and each loaded pair is
// split over two LDS granules (second half of slot g - 1, first half of slot g); the halo re-writes the
// body's last slot whole. The NCO phasor is a function of the absolute index, so the odd-start pairs
// mix exactly as the even-start ones would.
template <class InT, class Geo, int WG, bool VEC, int MODE, bool NT = false, bool DMA = false, int SH = 0>
__device__ __forceinline__ void stage_tile(float4* __restrict__ lds, const InT* __restrict__ in, uint64_t S0,
                                           uint32_t NG, const FirParams& p) {
  constexpr int G = Geo::G;
  if (p.hist != nullptr && (int64_t)S0 + p.in_off < 0) {  // uniform: the tile starts in the stream's history
    stage_tile_stream<InT, Geo, WG, MODE>(lds, in, S0, NG, p);
    return;
  }
  // tile body granules per staging thread (Geo::KT / R output segments of SG granules over WG threads)
  constexpr int BPT = Geo::SG * (Geo::KT / Geo::ROUT) / WG;
  static_assert(BPT * WG == Geo::SG * (Geo::KT / Geo::ROUT), "tile body must split evenly over the threads");
  // at most 8 granules (128 B) in flight per lane: bounds the staging registers for large segments
  constexpr int SB = staging_batch(BPT);
  static_assert(BPT % SB == 0, "segment granules must split into whole staging batches");
  const uint32_t tid = threadIdx.x;
  const PhaseWalk pw = phase_walk<G, WG>(p.nco_n0, S0, p.nco_inc);
  // wave-uniform: is the whole staged span readable? (every tile but the last)
  const bool whole = VEC && (int64_t)S0 >= 0 && (S0 + (uint64_t)NG * G <= p.L);
  if constexpr (SH != 0 && std::is_same<InT, float>::value) {
    // real samples SH (1..3) floats off 16-byte alignment (4-byte aligned): aligned 16-byte loads from
    // SH samples early; loaded quad g holds the last SH samples of granule g - 1 and the first 4 - SH of
    // granule g, written as two partial-granule LDS stores (8-byte aligned pieces). The halo re-writes
    // the body's last granule whole, as for complex input.
    static_assert(!VEC && SH > 0 && SH < 4, "shifted real staging: 1..3 floats off 16-byte alignment");
    // (a tile less than SH samples past the start of the caller's buffer would load samples before it --
    // inside its first 16-byte block, so it cannot fault, but it is out of bounds: that tile takes the
    // per-granule loads below instead. The buffer starts at `in - in_off` on the streaming path.)
    if ((int64_t)S0 + p.in_off >= (int64_t)SH && S0 + (uint64_t)NG * G <= p.L) {
      float* __restrict__ l1 = reinterpret_cast<float*>(lds);
      const float4* __restrict__ src = reinterpret_cast<const float4*>(in + S0 - SH);  // 16-byte aligned
#pragma unroll
      for (int b0 = 0; b0 < BPT; b0 += SB) {
        float4 v[SB];
#pragma unroll
        for (int k = 0; k < SB; ++k) v[k] = NT ? load16_nt(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          const uint32_t g = (b0 + k) * WG + tid;
          float* __restrict__ lo = l1 + 4 * Geo::padded(g);  // granule g
          if constexpr (SH == 2) {
            if (g > 0) *reinterpret_cast<float2*>(l1 + 4 * Geo::padded(g - 1) + 2) = make_float2(v[k].x, v[k].y);
            *reinterpret_cast<float2*>(lo) = make_float2(v[k].z, v[k].w);
          } else if constexpr (SH == 1) {
            if (g > 0) l1[4 * Geo::padded(g - 1) + 3] = v[k].x;
            *reinterpret_cast<float2*>(lo) = make_float2(v[k].y, v[k].z);
            lo[2] = v[k].w;
          } else {
            if (g > 0) {
              float* __restrict__ pv = l1 + 4 * Geo::padded(g - 1);
              pv[1] = v[k].x;
              *reinterpret_cast<float2*>(pv + 2) = make_float2(v[k].y, v[k].z);
            }
            lo[0] = v[k].w;
          }
        }
      }
      for (uint32_t g = BPT * WG - 1 + tid; g < NG; g += WG) {
        const uint64_t s = S0 + (uint64_t)g * G;
        lds[Geo::padded(g)] = load_granule<InT, false>(in, s, p.L);
      }
      return;
    }
  } else if constexpr (SH != 0) {
    static_assert((std::is_same<InT, float2>::value || std::is_same<InT, Iq8>::value) && !VEC && SH == 1,
                  "shifted staging is for 8-byte-aligned complex or 2-byte-aligned int8 I/Q input");
    // (a tile starting at the caller's buffer, chunk = in - in_off, would load the sample before it)
    if ((int64_t)S0 + p.in_off >= 1 && S0 + (uint64_t)NG * G <= p.L) {
      float2* __restrict__ l2 = reinterpret_cast<float2*>(lds);
#pragma unroll
      for (int b0 = 0; b0 < BPT; b0 += SB) {
        float4 v[SB];
        if constexpr (std::is_same<InT, Iq8>::value) {
          const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(in + S0 - 1);  // 4-byte aligned
          uint32_t w[SB];
#pragma unroll
          for (int k = 0; k < SB; ++k) {
            w[k] = NT ? __builtin_nontemporal_load(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
          }
#pragma unroll
          for (int k = 0; k < SB; ++k) v[k] = iq8x2_granule(w[k]);
        } else {
          const float4* __restrict__ src = reinterpret_cast<const float4*>(in + S0 - 1);  // 16-byte aligned
#pragma unroll
          for (int k = 0; k < SB; ++k) {
            if constexpr (NT) {
              v[k] = load16_nt(src + (b0 + k) * WG + tid);
            } else {
              v[k] = src[(b0 + k) * WG + tid];
            }
          }
        }
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          const uint32_t g = (b0 + k) * WG + tid;
          // samples S0 + 2g - 1 (odd start relative to the tile) and S0 + 2g
          const float4 w = stage_transform_ph<InT, MODE>(v[k], pw.ph0 + (uint32_t)(b0 + k) * pw.step - pw.inc, !pw.odd,
                                                         pw.inc);
          if (g > 0) l2[2 * Geo::padded(g - 1) + 1] = make_float2(w.x, w.y);
          l2[2 * Geo::padded(g)] = make_float2(w.z, w.w);
        }
      }
      for (uint32_t g = BPT * WG - 1 + tid; g < NG; g += WG) {
        const uint64_t s = S0 + (uint64_t)g * G;
        lds[Geo::padded(g)] = stage_transform<InT, MODE>(load_granule<InT, false>(in, s, p.L), (uint32_t)s, p);
      }
      return;
    }
  }
  if constexpr (DMA) {
    if (whole && stage_body_dma<InT, Geo, WG, MODE, NT>(lds, in, S0)) {
      for (uint32_t g = BPT * WG + tid; g < NG; g += WG) {
        const uint64_t s = S0 + (uint64_t)g * G;
        lds[Geo::padded(g)] = stage_transform<InT, MODE>(load_granule<InT, VEC>(in, s, p.L), (uint32_t)s, p);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  }
  HaloPre<InT, VEC> halo(S0, BPT * WG + tid, NG, p.L);
  // The body loop, instantiated once per NCO start parity (`odd` is uniform over the tile): with the
  // parity a runtime value the compiler kept a branch around every granule's phasor.
  const uint32_t pbase = Geo::padded(tid);
  auto body = [&](auto odd_c) {
    constexpr bool ODD = decltype(odd_c)::value;
#pragma unroll
  for (int b0 = 0; b0 < BPT; b0 += SB) {
    float4 v[SB];
    if (whole) {
      if constexpr (std::is_same<InT, Iq8>::value) {
        const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(in + S0);
        uint32_t w[SB];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          w[k] = NT ? __builtin_nontemporal_load(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
        }
#pragma unroll
        for (int k = 0; k < SB; ++k) v[k] = iq8x2_granule(w[k]);
      } else {
        const float4* __restrict__ src = reinterpret_cast<const float4*>(in + S0);
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          if constexpr (NT) {
            v[k] = load16_nt(src + (b0 + k) * WG + tid);
          } else {
            v[k] = src[(b0 + k) * WG + tid];
          }
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < SB; ++k) {
        v[k] = load_granule<InT, VEC>(in, S0 + (uint64_t)((b0 + k) * WG + tid) * G, p.L);
      }
    }
    if (b0 == 0) halo.issue(in);
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const uint32_t g = (b0 + k) * WG + tid;
      // padded(k * WG + tid) = padded(tid) + k * padded(WG) when whole segments fit a workgroup's row of
      // granules: a per-thread base plus an immediate offset per granule
      const uint32_t slot = (WG % Geo::SG == 0) ? pbase + (uint32_t)(b0 + k) * Geo::padded(WG) : Geo::padded(g);
      lds[slot] = stage_transform_ph<InT, MODE>(v[k], pw.ph0 + (uint32_t)(b0 + k) * pw.step, ODD, pw.inc);
    }
  }
  };
  if constexpr (MODE == kModeFir) {
    body(std::false_type{});
  } else if (pw.odd) {
    body(std::true_type{});
  } else {
    body(std::false_type{});
  }
  if (halo.g < NG) lds[Geo::padded(halo.g)] = stage_transform<InT, MODE>(halo.get(in, p.L), (uint32_t)halo.s, p);
  for (uint32_t g = halo.g + WG; g < NG; g += WG) {
    const uint64_t s = S0 + (uint64_t)g * G;
    lds[Geo::padded(g)] = stage_transform<InT, MODE>(load_granule<InT, VEC>(in, s, p.L), (uint32_t)s, p);
  }
}

// ------------------------------------------------------------------------------------------------
// Anchored NCO (the polyphase kernels in FM / AM mode). The FM discriminator and the AM envelope are
// invariant to a rotation common to the FIR outputs they combine, so a tile need not mix with the absolute
// phasor e^(j 2 pi P(n) / 2^32): it may mix relative to an anchor sample, as long as every output and its
// discriminator partner share the anchor. The anchors form an absolute grid: output q (absolute index
// q = firstSampleIndex / D + m) belongs to cell q / CELL (CELL = the decimation's largest tile, 1,024 outputs
// at D = 4), and all of a cell's FIR outputs -- in FM mode also the first output of the next cell, which the
// cell's last discriminator pairs with -- come from samples mixed relative to the cell's first sample.
// Within a cell, granule (row k, lane l) (samples 2 (k WG + l) and 2 (k WG + l) + 1 after the anchor) takes the
// phasors e_k(l) and e_k(l) w, with e_0(l) = E(2 l), e_k(l) = e_(k-1)(l) F, F = E(2 WG), w = E(1) (E: the exact
// integer phase through v_cos / v_sin, nco_direct): one complex multiply a granule instead of the absolute
// scheme's transcendental pair, and every phasor a fixed sequence of operations on (l, k) alone. The
// short-call tiles are sub-tiles of a cell that start their chains at row r0 by r0 multiplies, and every
// staging path (aligned, shifted, streaming) forms the same values, so every tile shape and any split of a
// stream into calls give bit-identical outputs.
// ------------------------------------------------------------------------------------------------
template <int WG>
__device__ __forceinline__ float2 rel_chain_start(uint32_t lane, uint32_t rows, uint32_t inc) {
  const float2 F = nco_direct((uint32_t)(2 * WG) * inc);
  float2 e = nco_direct((2u * lane) * inc);
  for (uint32_t i = 0; i < rows; ++i) e = cmul(e, F);
  return e;
}

// a granule (two complex samples) mixed with (e, e w)
__device__ __forceinline__ float4 rel_mix(float4 v, float2 e, float2 w) {
  const float2 eb = cmul(e, w);
  const float2 a = cmul(make_float2(v.x, v.y), e);
  const float2 b = cmul(make_float2(v.z, v.w), eb);
  return make_float4(a.x, a.y, b.x, b.y);
}

// stage_tile for an anchored chain. The tile starts row0 WG - sh granules into its cell (0 <= sh < WG): tile granule
// g = k WG + tid (the staging map of stage_tile) is cell granule (row0 + k) WG + tid - sh, i.e. lane
// l = (tid - sh) mod WG of cell row r + k with r = row0, or row0 - 1 for tid < sh. So a thread walks lane l's chain
// from row r, one multiply a row.
template <class InT, class Geo, int WG, bool VEC, bool NT, int SH>
__device__ __forceinline__ void stage_tile_rel(float4* __restrict__ lds, const InT* __restrict__ in, uint64_t S0,
                                               uint32_t NG, const FirParams& p, uint32_t row0, uint32_t sh) {
  constexpr int G = Geo::G;
  static_assert(G == 2, "NCO modes take complex samples");
  constexpr int BPT = Geo::SG * (Geo::KT / Geo::ROUT) / WG;  // body rows
  static_assert(BPT * WG == Geo::SG * (Geo::KT / Geo::ROUT), "tile body must split evenly over the threads");
  constexpr int SB = staging_batch(BPT);
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = (tid + WG - sh) % WG, row = row0 - (tid < sh ? 1u : 0u);
  const float2 w = nco_direct(p.nco_inc), F = nco_direct((uint32_t)(2 * WG) * p.nco_inc);
  float2 e = rel_chain_start<WG>(lane, row, p.nco_inc);
  if (p.hist != nullptr && (int64_t)S0 + p.in_off < 0) {
    // a streaming call's first tile, which reaches into the stream's history: sample by sample (stream_sample's
    // rule; samples before the call's first window read as zero), 8 rows of loads in flight
    constexpr int B = 8;
    const InT* __restrict__ hist = reinterpret_cast<const InT*>(p.hist);
    for (uint32_t g0 = 0; g0 < NG; g0 += B * WG) {
      InT v[B][G];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const uint32_t g = g0 + (uint32_t)b * WG + tid;
#pragma unroll
        for (int c = 0; c < G; ++c) {
          const uint64_t s = S0 + (uint64_t)g * G + (uint64_t)c;
          const int64_t i = (int64_t)s + p.in_off;
          if (g < NG && s < p.L) {
            v[b][c] = i < 0 ? hist[(int64_t)p.hist_len + i] : in[s];
          } else {
            set_zero(v[b][c]);
          }
        }
      }
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const uint32_t g = g0 + (uint32_t)b * WG + tid;
        if (g0 + (uint32_t)b * WG > 0) e = cmul(e, F);
        if (g >= NG) break;
        const float2 a = to_lds_sample(v[b][0]), c = to_lds_sample(v[b][1]);
        lds[Geo::padded(g)] = rel_mix(make_float4(a.x, a.y, c.x, c.y), e, w);
      }
    }
    return;
  }
  if constexpr (SH != 0) {
    static_assert(!VEC && SH == 1, "shifted staging is for 8-byte-aligned complex or 2-byte-aligned int8 I/Q input");
    if ((int64_t)S0 + p.in_off >= 1 && S0 + (uint64_t)NG * G <= p.L) {
      // loaded pair g holds samples 2g - 1 (the odd half of granule g - 1: lane l - 1's chain, or for lane 0
      // lane WG - 1's chain one row behind) and 2g (granule g): the previous lane's chain runs beside this one
      const uint32_t lp = (lane + WG - 1) % WG;
      const bool lag = lane == 0 && row == 0;  // lane 0 of a cell's first row has no previous granule in the cell
      float2 ep = nco_direct((2u * lp) * p.nco_inc);
      for (uint32_t i = 0; i < row; ++i) {
        const float2 t = cmul(ep, F);
        ep = (lane == 0 && i == 0) ? ep : t;  // lane 0 follows lane WG - 1 one row behind
      }
      float2* __restrict__ l2 = reinterpret_cast<float2*>(lds);
#pragma unroll
      for (int b0 = 0; b0 < BPT; b0 += SB) {
        float4 v[SB];
        if constexpr (std::is_same<InT, Iq8>::value) {
          const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(in + S0 - 1);  // 4-byte aligned
          uint32_t wd[SB];
#pragma unroll
          for (int k = 0; k < SB; ++k) {
            wd[k] = NT ? __builtin_nontemporal_load(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
          }
#pragma unroll
          for (int k = 0; k < SB; ++k) v[k] = iq8x2_granule(wd[k]);
        } else {
          const float4* __restrict__ src = reinterpret_cast<const float4*>(in + S0 - 1);  // 16-byte aligned
#pragma unroll
          for (int k = 0; k < SB; ++k) v[k] = NT ? load16_nt(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
        }
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          const int row = b0 + k;
          const uint32_t g = (uint32_t)row * WG + tid;
          if (row > 0) {
            e = cmul(e, F);
            const float2 t = cmul(ep, F);
            ep = (row == 1 && lag) ? ep : t;
          }
          const float2 a = cmul(make_float2(v[k].x, v[k].y), cmul(ep, w));  // sample 2g - 1
          const float2 b = cmul(make_float2(v[k].z, v[k].w), e);            // sample 2g
          if (g > 0) l2[2 * Geo::padded(g - 1) + 1] = a;
          l2[2 * Geo::padded(g)] = b;
        }
      }
      // the halo (its first granule rewrites the body's last slot whole): granule g of this loop is lane l - 1's
      // (lane 0: lane WG - 1's, one row back), i.e. the previous-lane chain's
      for (uint32_t g = BPT * WG - 1 + tid; g < NG; g += WG) {
        ep = cmul(ep, F);
        lds[Geo::padded(g)] = rel_mix(load_granule<InT, false>(in, S0 + (uint64_t)g * G, p.L), ep, w);
      }
      return;
    }
  }
  // wave-uniform: is the whole staged span readable? (not the first tile of a call starting inside its cell, not
  // the last)
  const bool whole = VEC && (int64_t)S0 >= 0 && (S0 + (uint64_t)NG * G <= p.L);
  const uint32_t pbase = Geo::padded(tid);
  HaloPre<InT, VEC> halo(S0, BPT * WG + tid, NG, p.L);  // (HaloPre)
#pragma unroll
  for (int b0 = 0; b0 < BPT; b0 += SB) {
    float4 v[SB];
    if (whole) {
      if constexpr (std::is_same<InT, Iq8>::value) {
        const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(in + S0);
        uint32_t wd[SB];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          wd[k] = NT ? __builtin_nontemporal_load(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
        }
#pragma unroll
        for (int k = 0; k < SB; ++k) v[k] = iq8x2_granule(wd[k]);
      } else {
        const float4* __restrict__ src = reinterpret_cast<const float4*>(in + S0);
#pragma unroll
        for (int k = 0; k < SB; ++k) v[k] = NT ? load16_nt(src + (b0 + k) * WG + tid) : src[(b0 + k) * WG + tid];
      }
    } else {
#pragma unroll
      for (int k = 0; k < SB; ++k) {
        v[k] = load_granule<InT, VEC>(in, S0 + (uint64_t)((b0 + k) * WG + tid) * G, p.L);
      }
    }
    if (b0 == 0) halo.issue(in);
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      if (b0 + k > 0) e = cmul(e, F);
      const uint32_t g = (b0 + k) * WG + tid;
      const uint32_t slot = (WG % Geo::SG == 0) ? pbase + (uint32_t)(b0 + k) * Geo::padded(WG) : Geo::padded(g);
      lds[slot] = rel_mix(v[k], e, w);
    }
  }
  if (halo.g < NG) {
    e = cmul(e, F);
    lds[Geo::padded(halo.g)] = rel_mix(halo.get(in, p.L), e, w);
  }
  for (uint32_t g = halo.g + WG; g < NG; g += WG) {
    e = cmul(e, F);
    lds[Geo::padded(g)] = rel_mix(load_granule<InT, VEC>(in, S0 + (uint64_t)g * G, p.L), e, w);
  }
}

// ------------------------------------------------------------------------------------------------
// Epilogues
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void store16_nt(float4* p, float4 v) {
  __builtin_nontemporal_store(gsdr_f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<gsdr_f32x4*>(p));
}

template <class OutT, int R, bool NTS = false>
__device__ __forceinline__ void store_fir(OutT* __restrict__ out, uint64_t k0, uint64_t N, const OutT (&acc)[R]) {
  constexpr int PER16 = 16 / sizeof(OutT);
  // 16-byte stores when R fills them (a thread's outputs are contiguous), else one output at a time
  if constexpr (R % PER16 == 0) {
    if (k0 + R <= N && (reinterpret_cast<uintptr_t>(out + k0) & 15u) == 0) {
      float4* o = reinterpret_cast<float4*>(out + k0);
#pragma unroll
      for (int q = 0; q < R / PER16; ++q) {
        float4 w;
        if constexpr (PER16 == 2) {
          w = make_float4(reinterpret_cast<const float2&>(acc[2 * q]).x, reinterpret_cast<const float2&>(acc[2 * q]).y,
                          reinterpret_cast<const float2&>(acc[2 * q + 1]).x,
                          reinterpret_cast<const float2&>(acc[2 * q + 1]).y);
        } else {
          w = make_float4(reinterpret_cast<const float&>(acc[4 * q]), reinterpret_cast<const float&>(acc[4 * q + 1]),
                          reinterpret_cast<const float&>(acc[4 * q + 2]),
                          reinterpret_cast<const float&>(acc[4 * q + 3]));
        }
        if constexpr (NTS) {
          store16_nt(o + q, w);
        } else {
          o[q] = w;
        }
      }
      return;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (k0 + r < N) out[k0 + r] = acc[r];
  }
}

// FM discriminator of consecutive FIR outputs: g * arg(y1 * conj(y0)) (reference src/fm.cu:66-68,
// src/quad_demod.cu:30-31).
// atan2 for the discriminators: octant reduction t = min/max (v_rcp_f32), an odd minimax polynomial
// for atan on [0, 1] (max abs error 3.3e-7 rad in float32 evaluation, tools/atan_fit.py), then the
// octant fix-ups. Outside 2^-100 < |x| + |y| < 2^100 (zeros, infinities, NaN, and magnitudes where
// v_rcp_f32 would leave the normal range) the library atan2f is used, so its special values
// (atan2(0, 0) = 0, atan2(+-0, -0) = +-pi, ...) are unchanged. The discriminator bar is 3.1e-5 rad
// (1e-5 of pi; tests/helpers.py wrapped_angle_err).
// The scalar form (disc_atan2 / fm_disc) and the two-at-a-time form (fm_disc2, packed FMAs) run the
// same IEEE operations in the same order, so every kernel's discriminator outputs are bit-identical.
__device__ __forceinline__ bool disc_fast(float y, float x) {
  const float s = fabsf(x) + fabsf(y);
  return s > 0x1p-100f && s < 0x1p100f;
}

__device__ __forceinline__ gsdr_f32x2 atan_poly2(gsdr_f32x2 t) {
  const gsdr_f32x2 s = t * t;
  gsdr_f32x2 p = __builtin_elementwise_fma(gsdr_f32x2{0.006811787374317646f, 0.006811787374317646f}, s,
                                           gsdr_f32x2{-0.0336042121052742f, -0.0336042121052742f});
  p = __builtin_elementwise_fma(p, s, gsdr_f32x2{0.07962368428707123f, 0.07962368428707123f});
  p = __builtin_elementwise_fma(p, s, gsdr_f32x2{-0.132333442568779f, -0.132333442568779f});
  p = __builtin_elementwise_fma(p, s, gsdr_f32x2{0.19807817041873932f, 0.19807817041873932f});
  p = __builtin_elementwise_fma(p, s, gsdr_f32x2{-0.3331736922264099f, -0.3331736922264099f});
  p = __builtin_elementwise_fma(p, s, gsdr_f32x2{0.9999961256980896f, 0.9999961256980896f});
  return p * t;
}

// octant fix-ups of the polynomial result r = atan(min/max) for (y, x)
__device__ __forceinline__ float disc_octant(float r, float y, float x) {
  if (fabsf(y) > fabsf(x)) r = 1.57079637f - r;
  if (x < 0.0f) r = 3.14159274f - r;
  return copysignf(r, y);
}

__device__ __forceinline__ float disc_atan2(float y, float x) {
  if (!disc_fast(y, x)) return atan2f(y, x);
  const float ax = fabsf(x), ay = fabsf(y);
  const float t = fminf(ax, ay) * __builtin_amdgcn_rcpf(fmaxf(ax, ay));
  return disc_octant(atan_poly2(gsdr_f32x2{t, t}).x, y, x);
}

__device__ __forceinline__ float2 disc_product(float2 y0, float2 y1) {
  return make_float2(y1.x * y0.x + y1.y * y0.y, y1.y * y0.x - y1.x * y0.y);
}

__device__ __forceinline__ float fm_disc(float2 y0, float2 y1, float g) {
  const float2 z = disc_product(y0, y1);
  return g * disc_atan2(z.y, z.x);
}

// fm_disc(a0, a1) and fm_disc(b0, b1) with the polynomial, the fix-up subtractions and the gain on
// packed FMAs / multiplies (two outputs per instruction)
// arg(za), arg(zb) of two discriminator products on packed FMAs (disc_atan2's operations)
__device__ __forceinline__ gsdr_f32x2 disc_angle2(float2 za, float2 zb) {
  const float axa = fabsf(za.x), aya = fabsf(za.y), axb = fabsf(zb.x), ayb = fabsf(zb.y);
  const gsdr_f32x2 t = gsdr_f32x2{fminf(axa, aya), fminf(axb, ayb)} *
                       gsdr_f32x2{__builtin_amdgcn_rcpf(fmaxf(axa, aya)), __builtin_amdgcn_rcpf(fmaxf(axb, ayb))};
  gsdr_f32x2 r = atan_poly2(t);
  const gsdr_f32x2 q = gsdr_f32x2{1.57079637f, 1.57079637f} - r;
  r.x = aya > axa ? q.x : r.x;
  r.y = ayb > axb ? q.y : r.y;
  const gsdr_f32x2 h = gsdr_f32x2{3.14159274f, 3.14159274f} - r;
  r.x = za.x < 0.0f ? h.x : r.x;
  r.y = zb.x < 0.0f ? h.y : r.y;
  r = gsdr_f32x2{copysignf(r.x, za.y), copysignf(r.y, zb.y)};
  if (!disc_fast(za.y, za.x)) r.x = atan2f(za.y, za.x);
  if (!disc_fast(zb.y, zb.x)) r.y = atan2f(zb.y, zb.x);
  return r;
}

__device__ __forceinline__ gsdr_f32x2 fm_disc2(float2 a0, float2 a1, float2 b0, float2 b1, float g) {
  return gsdr_f32x2{g, g} * disc_angle2(disc_product(a0, a1), disc_product(b0, b1));
}

// AM envelope: 2 * saturate(|y|) - 1, saturate(NaN) = 0 (reference src/am.cu:49, quad_demod.cu:47-48).
// |y| as the hardware square root of x^2 + y^2 (within 1 ulp of hypotf, whose library form rescales through a
// double frexp / ldexp: ~14 instructions an output against ~8). The saturation makes the rescaling moot: a sum
// that overflows gives +inf where hypotf gives a finite value > 1 (both saturate to 1), one that underflows gives 0
// where hypotf gives a value below 2^-24 (both give -1); an infinite component gives +inf even beside a NaN, as
// hypotf does.
__device__ __forceinline__ float am_env(float2 y) {
  float m = __builtin_amdgcn_sqrtf(fmaf(y.x, y.x, y.y * y.y));
  if (__builtin_isinf(y.x) || __builtin_isinf(y.y)) m = __builtin_inff();
  m = (m > 0.0f) ? (m < 1.0f ? m : 1.0f) : 0.0f;
  return 2.0f * m - 1.0f;
}

// FIR-mode store of a whole tile through LDS (CST != 0): thread t holds outputs t*R .. t*R+R-1, so a
// direct 16-byte store puts the lanes of one wave instruction R*sizeof(OutT) bytes apart (2 KB, 16
// cache lines per instruction for complex R = 4). Transposed through LDS, slot q*WG + t of the tile
// goes out with lane t, and every wave instruction writes one contiguous 1 KB run. CST = 2 uses
// streaming (non-temporal) stores. Returns false (nothing written) for a partial or misaligned tile,
// which then takes the per-thread store; the condition is uniform over the workgroup.
template <int CST, class OutT, int R, int WG>
__device__ __forceinline__ bool store_tile_lds(float4* lds, const FirParams& p, uint64_t out0, const OutT (&acc)[R]) {
  constexpr int NQ = R * (int)sizeof(OutT) / 16;  // float4 per thread
  static_assert(NQ * 16 == R * (int)sizeof(OutT), "R outputs must fill whole 16-byte slots");
  OutT* out = reinterpret_cast<OutT*>(p.out) + out0;
  if (out0 + (uint64_t)WG * R > p.N || (reinterpret_cast<uintptr_t>(out) & 15u) != 0) return false;
  const uint32_t t = threadIdx.x;
  __syncthreads();  // every wave is done reading the input tile
  float4 w[NQ];
  __builtin_memcpy(w, acc, sizeof(w));
#pragma unroll
  for (int q = 0; q < NQ; ++q) lds[t * NQ + q] = w[q];
  __syncthreads();
  float4* o = reinterpret_cast<float4*>(out);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float4 v = lds[q * WG + t];
    if constexpr (CST == 2) {
      store16_nt(o + q * WG + t, v);
    } else {
      o[q * WG + t] = v;
    }
  }
  return true;
}

// Shared by the tiled kernels. `xs` is a WG-sized LDS exchange area (FM mode only); `tile` the staged
// input tile, which FM mode with COAL reuses (WG * R floats) once every wave is done with it.
// A thread's R consecutive demodulated outputs, local indices ml0 .. ml0 + R - 1 of the tile (those below `lim`)
// at output m0: one 8- or 16-byte store when all R are in range and the address allows, so the lanes of a wave
// store one contiguous run (R * 256 bytes); one store each otherwise.
template <int R>
__device__ __forceinline__ void store_chain(float* __restrict__ out, uint64_t m0, uint32_t ml0, uint32_t lim, uint64_t N,
                                            const float (&o)[R]) {
  if constexpr (R == 2 || R == 4) {
    // (m0 < N first: the anchored tiles' leading outputs have m0 wrapped below zero)
    if (ml0 + R <= lim && m0 < N && N - m0 >= R && (reinterpret_cast<uintptr_t>(out + m0) % (4 * R)) == 0) {
      if constexpr (R == 4) {
        *reinterpret_cast<float4*>(out + m0) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
        *reinterpret_cast<float2*>(out + m0) = make_float2(o[0], o[1]);
      }
      return;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (ml0 + r < lim && m0 + r < N) out[m0 + r] = o[r];
  }
}

// COAL (FM, the contiguous-window kernels' tiles): the discriminator outputs leave through LDS in wave-contiguous
// runs; without it (the anchored polyphase tiles) each thread stores its R outputs with one vector store
// (store_chain), which is as contiguous and needs neither the LDS round trip nor its barrier.
template <int MODE, class OutT, int R, int WG, bool NTS = false, bool COAL = false>
__device__ __forceinline__ void tile_epilogue(const FirParams& p, uint64_t out0, OutT (&acc)[R], float2* xs,
                                              float4* tile = nullptr) {
  const uint32_t t = threadIdx.x;
  const uint32_t local0 = t * R;
  if constexpr (MODE == kModeFir) {
    store_fir<OutT, R, NTS>(reinterpret_cast<OutT*>(p.out), out0 + local0, p.N, acc);
  } else if constexpr (MODE == kModeAm) {
    float o[R];
#pragma unroll
    for (int r = 0; r < R; ++r) o[r] = am_env(acc[r]);
    store_chain<R>(reinterpret_cast<float*>(p.out), out0 + local0, local0, 0xffffffffu, p.N, o);
  } else {
    // Tiles overlap: the last thread's outputs (anchored polyphase tiles, tile_stride = KT - R) or the last one or
    // two (the other kernels, KT - 1 or KT - 2, fm_tile_stride) are only partners; the neighbouring thread's
    // first output comes through LDS.
    xs[t] = acc[0];
    __syncthreads();
    // value select (both loads in range): a select of the two addresses became a flat load through
    // scratch when R = 1
    const float2 nb = xs[t + 1 < WG ? t + 1 : t];
    const float2 nxt = (t + 1 < WG) ? nb : acc[R - 1];
    float o[R];
#pragma unroll
    for (int r = 0; r + 1 < R; r += 2) {
      const float2 y2 = (r + 2 < R) ? acc[r + 2] : nxt;
      const gsdr_f32x2 v = fm_disc2(acc[r], acc[r + 1], acc[r + 1], y2, p.fm_gain);
      o[r] = v.x;
      o[r + 1] = v.y;
    }
    if constexpr (R % 2 == 1) o[R - 1] = fm_disc(acc[R - 1], nxt, p.fm_gain);
    float* out = reinterpret_cast<float*>(p.out);
    if constexpr (COAL && R > 1) {
      // Through LDS so that every wave instruction stores one contiguous 256-byte run: stored
      // straight from registers, a thread's R outputs put the lanes of one dword store R * 4 bytes
      // apart. The tile area is free: every wave has passed the barrier above, i.e. finished its MACs.
      float* lo = reinterpret_cast<float*>(tile);
#pragma unroll
      for (int r = 0; r < R; ++r) lo[local0 + r] = o[r];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const uint32_t ml = q * WG + t;
        const uint64_t m = out0 + ml;
        if (ml < p.tile_stride && m < p.N) out[m] = lo[ml];
      }
    } else {
      store_chain<R>(out, out0 + local0, local0, p.tile_stride, p.N, o);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Polyphase compute core shared by the polyphase kernels: thread t accumulates its R outputs from
// the staged tile in LDS. JC = tap rows per chunk (a multiple of R); a chunk covers JC*D taps.
// ------------------------------------------------------------------------------------------------
template <class TapT, class InT, int D, int R, int JC, int WG, bool LIGHT = false, bool FENCE = false>
__device__ __forceinline__ void poly_compute(const float4* __restrict__ lds, const FirParams& p,
                                             typename Product<TapT, InT>::type (&acc)[R]) {
  using Geo = TileGeo<InT, D, R, WG>;
  constexpr int G = Geo::G;
  constexpr int CPR = D / G;  // granule columns per input row
  static_assert(D % G == 0, "polyphase kernel needs whole granules per row");
  static_assert(JC % R == 0, "chunk rows must be whole thread segments");
  constexpr int NWIN = R + JC - 1;
  const uint32_t t = threadIdx.x;
  for (uint32_t c = 0; c < p.nch; ++c) {
    const float4* __restrict__ seg = lds + (t + c * (JC / R)) * Geo::SGP;
#pragma unroll
    for (int h = 0; h < CPR; ++h) {
      // taps first (one SMEM batch, one wait), then the LDS window (in-order, counted waits)
      TapT tv[JC][G];
      const TapBuf tb = tap_window<TapT>(p.taps, p.T, c * JC * D + h * G);
#pragma unroll
      for (int j = 0; j < JC; ++j) {
#pragma unroll
        for (int e = 0; e < G; ++e) tv[j][e] = tap_at<TapT>(tb, j * D + e);
      }
      // FENCE: keeps one column's window reads from being scheduled ahead of the previous column's
      // multiply-adds (the persistent kernel's scheduler otherwise held every window at once)
      if constexpr (FENCE) asm volatile("" ::: "memory");
      float4 win[NWIN];
#pragma unroll
      for (int u = 0; u < NWIN; ++u) {
        const int q = u * CPR + h;
        // LIGHT (tuning probe, wrong results): only the thread's own R rows come from LDS, the rest of
        // the window repeats them -- the same FMAs with 4/19 of the LDS reads
        if (!LIGHT || u < R) {
          win[u] = seg[q + Geo::PAD * (q / Geo::SG)];
        } else {
          win[u] = win[u - R];
        }
      }
#pragma unroll
      for (int j = 0; j < JC; ++j) {
#pragma unroll
        for (int e = 0; e < G; ++e) {
#pragma unroll
          for (int r = 0; r < R; ++r) mac(acc[r], granule_sample<typename LdsSample<InT>::type>(win[r + j], e), tv[j][e]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Exact zero-padding semantics. The tiled cores round T up to whole tap chunks and multiply the
// padding (taps read as +0 past T) like any other tap. For a finite sample x*0 is a signed zero and
// adding it leaves the sum unchanged, but for x = +-Inf or NaN it is NaN, which the reference never
// computes: its loop stops at tap T-1 (fir.cu:29-31, 58-60). A padding product can therefore only turn
// an output into NaN. So every output that came out non-finite (a NaN or Inf output: a cheap test, and
// rare) is recomputed from the staged tile in the SAME MAC order with the padding products skipped --
// exactly the fast path's sum whenever no padding product was NaN, and the reference's set of products
// otherwise. The result depends only on the output's own window, never on the tiling, so chunked and
// monolithic calls stay bit-identical.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool finite_out(float a) { return __builtin_isfinite(a); }
__device__ __forceinline__ bool finite_out(float2 a) { return __builtin_isfinite(a.x) && __builtin_isfinite(a.y); }

struct NoPad {
  __host__ __device__ static constexpr uint32_t padded(uint32_t g) { return g; }
};

// sample s of the tile (local index) from the LDS granule layout (padded as TileGeo when PADDED)
template <class InT, class Geo, bool PADDED>
__device__ __forceinline__ typename LdsSample<InT>::type tile_sample(const float4* __restrict__ lds, uint32_t s) {
  using LdsT = typename LdsSample<InT>::type;
  constexpr uint32_t G = SampleT<InT>::kPerGranule;
  const uint32_t g = s / G;
  const uint32_t slot = PADDED ? Geo::padded(g) : g;
  return reinterpret_cast<const LdsT*>(lds)[slot * G + s % G];
}

// Polyphase order (poly_compute): chunk c, granule column h, row j, element e -- tap
// i = (c*JC + j)*D + h*G + e of local output m = threadIdx.x * R + r.
template <class TapT, class InT, int D, int R, int JC, int WG>
__device__ __forceinline__ void poly_fixup(const float4* __restrict__ lds, const FirParams& p,
                                        typename Product<TapT, InT>::type (&acc)[R]) {
  using Geo = TileGeo<InT, D, R, WG>;
  constexpr int G = Geo::G, CPR = D / G;
  const TapT* __restrict__ taps = reinterpret_cast<const TapT*>(p.taps);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (finite_out(acc[r])) continue;
    const uint32_t s0 = (threadIdx.x * R + r) * D;
    typename Product<TapT, InT>::type a;
    set_zero(a);
#pragma unroll 1
    for (uint32_t c = 0; c < p.nch; ++c) {
#pragma unroll 1
      for (int h = 0; h < CPR; ++h) {
#pragma unroll 1
        for (int j = 0; j < JC; ++j) {
          const uint32_t i0 = (c * JC + j) * D + h * G;
#pragma unroll
          for (int e = 0; e < G; ++e) {
            if (i0 + e < p.T) mac(a, tile_sample<InT, Geo, true>(lds, s0 + i0 + e), taps[i0 + e]);
          }
        }
      }
    }
    acc[r] = a;
  }
}

// Ascending tap order (contiguous-window, runtime-decimation and matrix-core cores): local output m at
// local sample m * D.
template <class TapT, class InT, class Geo, bool PADDED, int R>
__device__ __forceinline__ void ascending_fixup(const float4* __restrict__ lds, const FirParams& p, uint32_t D,
                                             uint32_t m0, typename Product<TapT, InT>::type (&acc)[R]) {
  const TapT* __restrict__ taps = reinterpret_cast<const TapT*>(p.taps);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (finite_out(acc[r])) continue;
    const uint32_t s0 = (m0 + r) * D;
    typename Product<TapT, InT>::type a;
    set_zero(a);
#pragma unroll 1
    for (uint32_t i = 0; i < p.T; ++i) mac(a, tile_sample<InT, Geo, PADDED>(lds, s0 + i), taps[i]);
    acc[r] = a;
  }
}

// Wave-cheap screen for the fix-up: the sum of a thread's outputs is finite when they all are (a NaN or
// Inf term makes it NaN or Inf). A finite set whose sum overflows only sends the thread through the
// per-output test in the fix-up, which then changes nothing. Packed adds: 5 VALU operations for R = 4
// complex outputs instead of one class test per component.
template <int R>
__device__ __forceinline__ bool all_finite(const float2 (&acc)[R]) {
  gsdr_f32x2 s = {acc[0].x, acc[0].y};
#pragma unroll
  for (int r = 1; r < R; ++r) s += gsdr_f32x2{acc[r].x, acc[r].y};
  return __builtin_isfinite(s.x + s.y);
}
template <int R>
__device__ __forceinline__ bool all_finite(const float (&acc)[R]) {
  if constexpr (R % 2 == 0) {
    gsdr_f32x2 s = {acc[0], acc[1]};
#pragma unroll
    for (int r = 2; r < R; r += 2) s += gsdr_f32x2{acc[r], acc[r + 1]};
    return __builtin_isfinite(s.x + s.y);
  } else {
    float s = acc[0];
#pragma unroll
    for (int r = 1; r < R; ++r) s += acc[r];
    return __builtin_isfinite(s);
  }
}

// ------------------------------------------------------------------------------------------------
// Kernel 1: polyphase-granule kernel, one tile per workgroup (D a multiple of the granule width G).
// ABL (ablation, tuning probes only): low bits 0 = full kernel, 1 = staging only, 2 = compute only;
// chain-mode flags 8 = staging without the NCO mix, 16 = plain float store instead of the FM
// discriminator, 32 = NCO mix without the per-granule transcendental pair, 128 = tile-relative phasors
// by recurrence; 64 = register window from the thread's own R rows only (wrong results: LDS-read probe).
// NT: non-temporal (streaming) HBM loads for the staged input.
// ------------------------------------------------------------------------------------------------
// Tile of workgroup b. XCD-aware (XM): workgroups are dispatched round-robin over the 8 XCDs, so
// with the identity map neighbouring tiles (which share a halo of input rows) sit on different L2s;
// remapped, XCD x walks one contiguous range of tiles and the halo of the previous tile is still in
// its L2.
template <bool XM>
__device__ __forceinline__ uint32_t tile_of_block() {
  if constexpr (!XM) {
    return blockIdx.x;
  } else {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t per = nb / 8, rem = nb % 8, x = b % 8, i = b / 8;
    return x * per + (x < rem ? x : rem) + i;
  }
}

// One tile of the polyphase kernel (the body of k_fir_poly and of k_fir_poly_grouped). FM / AM tiles are
// anchored (stage_tile_rel): tile t covers outputs [t S - tile_shift, t S - tile_shift + KT) with S = tile_stride
// (KT for AM; KT - R for FM, whose last thread's outputs only serve as the discriminator partners of the one before,
// so every discriminator pairs two outputs of one tile in one NCO frame) and is sub-tile (cell_sub0 + t) mod SUBS of
// its NCO cell of SUBS tiles.
template <class TapT, class InT, int D, int R, int JC, int WG, bool VEC, int MODE, int ABL, bool NT, int CST, bool DMA,
          int SH, int SUBS = 1>
__device__ __forceinline__ void fir_poly_tile(const FirParams& p, uint32_t tile) {
  using Geo = TileGeo<InT, D, R, WG>;
  using OutT = typename Product<TapT, InT>::type;
  constexpr int G = Geo::G;
  constexpr bool ANCH = MODE != kModeFir;
  constexpr int BPT = Geo::SG * (Geo::KT / Geo::ROUT) / WG;  // granule rows of the tile body

  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  const InT* __restrict__ in = reinterpret_cast<const InT*>(p.in);
  const HistSample<InT> hist = stream_history_load<InT>(p);

  // (an anchored call's first tile may start before output 0: out0 and S0 are then "negative", wrapped)
  const uint64_t out0 = (uint64_t)tile * p.tile_stride - (ANCH ? p.tile_shift : 0u);
  const uint64_t S0 = out0 * D;
  const uint32_t span = p.nch * JC * D;
  const uint32_t NG = ((Geo::KT - 1) * D + span + G - 1) / G;
  // LDS: [tile granules | FM exchange (WG float2)]
  constexpr int SMODE = (ABL & 8) ? (int)kModeFir : MODE;
  if constexpr ((ABL & 7) != 2) {
    if constexpr (ANCH && SMODE != kModeFir) {
      // the tile is sub-tile `sub` of its NCO cell: it starts sub (KT - R) outputs (FM) or sub KT outputs (AM) into
      // the cell, i.e. sub BPT granule rows in, less sub SG granules for FM (stage_tile_rel)
      const uint32_t sub = (p.cell_sub0 + tile) % SUBS;
      stage_tile_rel<InT, Geo, WG, VEC, NT, SH>(lds, in, S0, NG, p, sub * BPT, MODE == kModeFm ? sub * Geo::SG : 0u);
    } else {
      stage_tile<InT, Geo, WG, VEC, SMODE, NT, DMA, SH>(lds, in, S0, NG, p);
    }
  }
  __syncthreads();
  stream_history_store<InT>(p, hist);
  float2* xs = reinterpret_cast<float2*>(lds + Geo::padded(NG - 1) + 1);

  OutT acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) set_zero(acc[r]);
  if constexpr ((ABL & 7) == 1) {
    const float4 v = lds[Geo::padded(threadIdx.x * Geo::SG)];
#pragma unroll
    for (int r = 0; r < R; ++r) mac(acc[r], granule_sample<typename LdsSample<InT>::type>(v, r % G), 1.0f);
  } else {
    poly_compute<TapT, InT, D, R, JC, WG, (ABL & 64) != 0>(lds, p, acc);
    if constexpr (ABL == 0) {
      if (!all_finite(acc)) poly_fixup<TapT, InT, D, R, JC, WG>(lds, p, acc);
    }
  }

  if constexpr (CST != 0 && MODE == kModeFir) {
    if (store_tile_lds<CST, OutT, R, WG>(lds, p, out0, acc)) return;
  }
  if constexpr ((ABL & 16) != 0 && MODE == kModeFm) {
    float* out = reinterpret_cast<float*>(p.out);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t ml = threadIdx.x * R + r;
      if (ml < p.tile_stride && out0 + ml < p.N) out[out0 + ml] = acc[r].x + acc[r].y;
    }
    return;
  }
  tile_epilogue<MODE, OutT, R, WG, NT, !ANCH>(p, out0, acc, xs, lds);
}

template <class TapT, class InT, int D, int R, int JC, int WG, bool VEC, int MODE, int ABL = 0, bool NT = false,
          bool XM = false, int CST = 0, bool DMA = false, int SH = 0, int SUBS = 1>
__global__ __launch_bounds__(WG) void k_fir_poly(FirParams p) {
  fir_poly_tile<TapT, InT, D, R, JC, WG, VEC, MODE, ABL, NT, CST, DMA, SH, SUBS>(p, tile_of_block<XM>());
}

// ------------------------------------------------------------------------------------------------
// Multi-channel NCO + FIR + demodulator (the intent of the reference's
// dead k_Fm4x, src/fm.cu:71-179): up to kMaxMultiChannels channels of one input per launch.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxMultiChannels = 16;

struct MultiParams {
  uint32_t count;                     // channels in this launch
  uint32_t inc[kMaxMultiChannels];    // NCO phase increment per channel
  float gain[kMaxMultiChannels];      // FM gain per channel
  uint64_t out_stride;                // outputs between consecutive channels' first outputs (>= N)
};

// Kernel 1g: multi-channel chains as C single-channel tiles per input tile, grouped for the L2. Block b
// runs channel c of tile t, with b mod 8 = t mod 8 and the C channels of a tile consecutive among the
// blocks of that residue: workgroups are dispatched round-robin over the 8 XCDs, so the C workgroups of a
// tile run close together on ONE XCD and all but the first stage the tile from that XCD's L2 rather
// than HBM. Each block is exactly the single-channel kernel's tile (same template, same code), so
// channel c is bit-identical to gsdrFmDemod / gsdrAmDemod with its own frequency by construction, at
// the single-channel kernel's register budget. (The first multi-channel kernel read each input tile
// into registers once and looped over the channels: 228 VGPRs, 2 waves per SIMD, 5 % slower.)
template <class TapT, class InT, int D, int R, int JC, int WG, bool VEC, int MODE, int SH = 0>
__global__ __launch_bounds__(WG) void k_fir_poly_grouped(FirParams p, MultiParams mp, uint32_t tiles) {
  const uint32_t C = mp.count;
  const uint32_t b = blockIdx.x, r = b >> 3;
  const uint32_t tile = (r / C) * 8u + (b & 7u), c = r % C;
  if (tile >= tiles) return;  // the grid is rounded up to whole groups of 8 tiles
  FirParams pc = p;
  pc.nco_inc = mp.inc[c];
  pc.fm_gain = mp.gain[c];
  pc.out = reinterpret_cast<float*>(p.out) + (uint64_t)c * mp.out_stride;
  if (c != 0) pc.hist_out = nullptr;  // a multi-channel stream step: channel 0's workgroup 0 copies the history
  fir_poly_tile<TapT, InT, D, R, JC, WG, VEC, MODE, 0, true, 0, false, SH, 1>(pc, tile);
}

// ------------------------------------------------------------------------------------------------
// Kernel 2: contiguous-window kernel for small D (D = 1 in particular).
//   IC = taps per chunk (a multiple of R*D).
// ------------------------------------------------------------------------------------------------
template <class TapT, class InT, int D, int R, int IC, int WG, bool VEC, int MODE, int SH = 0>
__global__ __launch_bounds__(WG) void k_fir_contig(FirParams p) {
  using Geo = TileGeo<InT, D, R, WG>;
  using OutT = typename Product<TapT, InT>::type;
  constexpr int G = Geo::G;
  static_assert(IC % (R * D) == 0, "chunk taps must be whole thread segments");
  constexpr int W = (R - 1) * D + IC;  // window samples
  constexpr int NWIN = (W + G - 1) / G;

  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  const InT* __restrict__ in = reinterpret_cast<const InT*>(p.in);
  const HistSample<InT> hist = stream_history_load<InT>(p);

  const uint64_t out0 = (uint64_t)blockIdx.x * p.tile_stride;
  const uint64_t S0 = out0 * D;
  const uint32_t span = p.nch * IC;
  const uint32_t NG = ((Geo::KT - 1) * D + span + G - 1) / G;

  stage_tile<InT, Geo, WG, VEC, MODE, false, false, SH>(lds, in, S0, NG, p);
  __syncthreads();
  stream_history_store<InT>(p, hist);

  OutT acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) set_zero(acc[r]);

  const uint32_t t = threadIdx.x;
  for (uint32_t c = 0; c < p.nch; ++c) {
    const float4* __restrict__ seg = lds + (t + c * (IC / (R * D))) * Geo::SGP;
    const TapBuf tb = tap_window<TapT>(p.taps, p.T, c * IC);
    TapT tvs[IC];
#pragma unroll
    for (int i = 0; i < IC; ++i) tvs[i] = tap_at<TapT>(tb, i);
    float4 win[NWIN];
#pragma unroll
    for (int q = 0; q < NWIN; ++q) win[q] = seg[q + Geo::PAD * (q / Geo::SG)];
#pragma unroll
    for (int i = 0; i < IC; ++i) {
      const TapT tv = tvs[i];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int s = r * D + i;
        mac(acc[r], granule_sample<typename LdsSample<InT>::type>(win[s / G], s % G), tv);
      }
    }
  }

  if (!all_finite(acc)) ascending_fixup<TapT, InT, Geo, true, R>(lds, p, D, t * R, acc);

  float2* xs = reinterpret_cast<float2*>(lds + Geo::padded(NG - 1) + 1);
  tile_epilogue<MODE, OutT, R, WG>(p, out0, acc, xs);
}

// ------------------------------------------------------------------------------------------------
// Kernel 2r: runtime-decimation tile kernel, for decimations without a compile-time shape. The tile's
// input span is staged into LDS unpadded (NCO applied once per sample, as in the other tiled kernels)
// and thread t computes output t of the tile from LDS, one sample read per tap (ds_read with the tap
// as an immediate offset), in ascending tap order like the generic kernel. No register window (D is
// not known at compile time), so it is bound by LDS reads (~T * sample bytes per output), which
// still beats re-reading every sample T / D times through L1/L2.
// PAIR (even D): two consecutive samples per LDS read (complex: ds_read_b128, real: ds_read_b64), still
// multiplied in ascending tap order. One sample a read puts lane t at bank 2Dt mod 64 (complex), which
// for D = 2^k m (m odd) touches only 64 / 2^k of the banks: 2-way conflicts at D = 50, 4-way at 100
// (PMC: 42 % of LDS cycles at D = 50, profiles/r01_pmc_fir_rt_d50_d13.txt). ds_read_b128 serves 16
// lanes a cycle with lane groups whose indices cover every residue mod 16, so lane starts 4(D/2)t mod 64
// are distinct for D = 2 mod 4 (conflict-free) and 2-way at D = 4 mod 8; half the read instructions too.
// ------------------------------------------------------------------------------------------------
template <class LdsT>
struct LdsPair;
template <>
struct LdsPair<float> {
  using type = float2;
  __device__ static float lo(float2 v) { return v.x; }
  __device__ static float hi(float2 v) { return v.y; }
};
template <>
struct LdsPair<float2> {
  using type = float4;
  __device__ static float2 lo(float4 v) { return make_float2(v.x, v.y); }
  __device__ static float2 hi(float4 v) { return make_float2(v.z, v.w); }
};

// N separate ds_read_b64 of the 8-byte values at p[0..N): the compiler merges adjacent 8-byte LDS loads
// into ds_read2_b64, which takes 16 LDS cycles per 16 bytes against 4 for two ds_read_b64 (and banks
// mod 32), so at odd D the one-sample-a-read loop ran at a quarter of the LDS rate. The reads and their
// wait are ONE asm statement with early-clobber outputs, so no register is taken as written before the
// s_waitcnt that fills it (a copy scheduled between separate read and wait statements would
// have read a register the load had not filled yet).
#define GSDR_R8(i) "ds_read_b64 %" #i ", %[a] offset:" #i "*8\n\t"
template <int N>
__device__ __forceinline__ void lds_read_b64_n(const float2* p, float2 (&out)[N]);
template <>
__device__ __forceinline__ void lds_read_b64_n<8>(const float2* p, float2 (&out)[8]) {
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float2*)p;
  gsdr_f32x2 r0, r1, r2, r3, r4, r5, r6, r7;
  asm volatile(GSDR_R8(0) GSDR_R8(1) GSDR_R8(2) GSDR_R8(3) GSDR_R8(4) GSDR_R8(5) GSDR_R8(6) GSDR_R8(7)
               "s_waitcnt lgkmcnt(0)"
               : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
               : [a] "v"(a)
               : "memory");
  const gsdr_f32x2 r[8] = {r0, r1, r2, r3, r4, r5, r6, r7};
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = make_float2(r[i].x, r[i].y);
}
template <>
__device__ __forceinline__ void lds_read_b64_n<16>(const float2* p, float2 (&out)[16]) {
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float2*)p;
  gsdr_f32x2 r0, r1, r2, r3, r4, r5, r6, r7, r8, r9, r10, r11, r12, r13, r14, r15;
  asm volatile(GSDR_R8(0) GSDR_R8(1) GSDR_R8(2) GSDR_R8(3) GSDR_R8(4) GSDR_R8(5) GSDR_R8(6) GSDR_R8(7)
               GSDR_R8(8) GSDR_R8(9) GSDR_R8(10) GSDR_R8(11) GSDR_R8(12) GSDR_R8(13) GSDR_R8(14) GSDR_R8(15)
               "s_waitcnt lgkmcnt(0)"
               : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7),
                 "=&v"(r8), "=&v"(r9), "=&v"(r10), "=&v"(r11), "=&v"(r12), "=&v"(r13), "=&v"(r14), "=&v"(r15)
               : [a] "v"(a)
               : "memory");
  const gsdr_f32x2 r[16] = {r0, r1, r2, r3, r4, r5, r6, r7, r8, r9, r10, r11, r12, r13, r14, r15};
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = make_float2(r[i].x, r[i].y);
}
#undef GSDR_R8

template <class TapT, class InT, int IC, int WG, bool VEC, int MODE, bool PAIR = false>
__global__ __launch_bounds__(WG) void k_fir_rt(FirParams p) {
  using OutT = typename Product<TapT, InT>::type;
  using LdsT = typename LdsSample<InT>::type;
  constexpr int G = SampleT<InT>::kPerGranule;
  // granules in flight per lane while staging: the tile (D * WG samples) bounds the resident workgroups to
  // 1-2 waves a SIMD at large D, so each lane keeps 16 loads (256 B) in flight (4: D = 50 FC 125 us)
  constexpr int SB = 16;

  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  const InT* __restrict__ in = reinterpret_cast<const InT*>(p.in);
  const uint32_t D = p.D;
  const uint64_t out0 = (uint64_t)blockIdx.x * p.tile_stride;
  const uint64_t S0 = out0 * D;
  const uint32_t span = p.nch * IC;
  const uint32_t NG = ((WG - 1) * D + span + G - 1) / G;
  const uint32_t tid = threadIdx.x;
  for (uint32_t g0 = 0; g0 < NG; g0 += SB * WG) {
    float4 v[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const uint32_t g = g0 + k * WG + tid;
      v[k] = g < NG ? load_granule<InT, VEC>(in, S0 + (uint64_t)g * G, p.L) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const uint32_t g = g0 + k * WG + tid;
      if (g < NG) lds[g] = stage_transform<InT, MODE>(v[k], (uint32_t)(S0 + (uint64_t)g * G), p);
    }
  }
  __syncthreads();

  OutT acc;
  set_zero(acc);
  const LdsT* __restrict__ xs = reinterpret_cast<const LdsT*>(lds) + tid * D;
  for (uint32_t c = 0; c < p.nch; ++c) {
    const TapBuf tb = tap_window<TapT>(p.taps, p.T, c * IC);
    TapT tv[IC];
#pragma unroll
    for (int i = 0; i < IC; ++i) tv[i] = tap_at<TapT>(tb, i);
    const LdsT* __restrict__ xc = xs + c * IC;
    if constexpr (PAIR) {
      static_assert(IC % 2 == 0, "pairs of taps");
      using P = LdsPair<LdsT>;
      const typename P::type* __restrict__ xp = reinterpret_cast<const typename P::type*>(xc);  // D even: aligned
      typename P::type v[IC / 2];
      if constexpr (std::is_same<typename P::type, float2>::value) {
        lds_read_b64_n<IC / 2>(xp, v);  // real samples: 8-byte pairs, kept apart from ds_read2_b64
      } else {
#pragma unroll
        for (int i = 0; i < IC / 2; ++i) v[i] = xp[i];
      }
#pragma unroll
      for (int i = 0; i < IC / 2; ++i) {
        mac(acc, P::lo(v[i]), tv[2 * i]);
        mac(acc, P::hi(v[i]), tv[2 * i + 1]);
      }
    } else if constexpr (std::is_same<LdsT, float2>::value && std::is_same<TapT, float>::value) {
      // (complex taps keep the compiler's loads: their two packed FMAs a tap hide the merged reads, and the
      // asm reads' common wait measured 5 % slower there at D = 9)
      float2 v[IC];
      lds_read_b64_n<IC>(xc, v);
#pragma unroll
      for (int i = 0; i < IC; ++i) mac(acc, v[i], tv[i]);
    } else {
#pragma unroll
      for (int i = 0; i < IC; ++i) mac(acc, xc[i], tv[i]);
    }
  }
  OutT accs[1] = {acc};
  if (!finite_out(acc)) ascending_fixup<TapT, InT, NoPad, false, 1>(lds, p, D, tid, accs);
  float2* ex = reinterpret_cast<float2*>(lds + NG);
  tile_epilogue<MODE, OutT, 1, WG>(p, out0, accs, ex);
}

template <class InT>
constexpr size_t rt_lds_bytes(uint32_t D, uint32_t span_samples, int wg, int mode) {
  const uint32_t G = SampleT<InT>::kPerGranule;
  size_t bytes = (size_t)(((uint32_t)(wg - 1) * D + span_samples + G - 1) / G) * 16u;
  if (mode != kModeFir) bytes += ((size_t)wg * sizeof(float2) + 15) / 16 * 16;
  return bytes;
}

// ------------------------------------------------------------------------------------------------
// Kernel 3: generic fallback (any D, any T, any alignment): one output per thread straight from
// global memory (L1/L2 absorb the overlap). Used only where the tiled kernels do not apply.
// In FM mode each thread also computes the next FIR output.
// ------------------------------------------------------------------------------------------------
template <class TapT, class InT, int MODE>
__device__ __forceinline__ typename Product<TapT, InT>::type fir_point(const FirParams& p, uint64_t k) {
  using OutT = typename Product<TapT, InT>::type;
  const InT* __restrict__ in = reinterpret_cast<const InT*>(p.in);
  const TapT* __restrict__ taps = reinterpret_cast<const TapT*>(p.taps);
  OutT acc;
  set_zero(acc);
  const uint64_t s0 = k * p.D;
  for (uint32_t i = 0; i < p.T; ++i) {
    auto x = to_lds_sample(in[s0 + i]);
    if constexpr (MODE != kModeFir) {
      x = nco_mix(x, p.nco_n0 + (uint32_t)(s0 + i), p.nco_inc);
    }
    mac(acc, x, taps[i]);
  }
  return acc;
}

template <class TapT, class InT, int MODE>
__global__ __launch_bounds__(256) void k_fir_generic(FirParams p) {
  using OutT = typename Product<TapT, InT>::type;
  const uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (k >= p.N) return;
  if constexpr (MODE == kModeFir) {
    reinterpret_cast<OutT*>(p.out)[k] = fir_point<TapT, InT, MODE>(p, k);
  } else if constexpr (MODE == kModeAm) {
    reinterpret_cast<float*>(p.out)[k] = am_env(fir_point<TapT, InT, MODE>(p, k));
  } else {
    const float2 y0 = fir_point<TapT, InT, MODE>(p, k);
    const float2 y1 = fir_point<TapT, InT, MODE>(p, k + 1);
    reinterpret_cast<float*>(p.out)[k] = fm_disc(y0, y1, p.fm_gain);
  }
}

// ------------------------------------------------------------------------------------------------
// Kernel 1y: the same tile on the matrix cores (FIR mode, real taps, complex input, D = 4), an
// alternative core kept as a tuning variant (gsdrxFirFCVariant 13).
// v_mfma_f32_4x4x1_16b_f32 is 16 independent 4x4 outer products per wave instruction: block b of a
// wave holds lanes 4b..4b+3, A[i] comes from lane 4b+i, B[j] from lane 4b+j and D[i][j] lands in
// VGPR i of lane 4b+j. With
//     A[i] = t[kappa - D*i]                  (the tap row i needs at step kappa),
//     B[j] = x[D*(k0 + 4L) + kappa], L = 4b+j (lane L's own input stream),
// accumulator C[i] of lane L sums t[kappa - D*i] * x[D*(k0 + 4L + i) + (kappa - D*i)] over
// kappa = 0 .. 3D+T-1: output k0 + 4L + i with its taps in ascending order (zero outside [0, T)).
// f32 MFMA is an exact fmaf chain, so the outputs are bit-identical to the oracle's and the generic
// kernel's ascending-tap fmaf loop. Each lane reads its window sequentially from LDS (one
// ds_read_b128 per two steps); re and im are two accumulator chains. The taps need no memory
// traffic in the loop: the A operand of block ABID can be broadcast to all 16 blocks (CBSZ = 4) and
// every block needs the same taps, so one VGPR carries the taps of 16 consecutive steps: lane 4b+i
// of tap register c holds t[16c + b - D*i], and step 16c + b runs with ABID = b. MAXSEG registers
// cover 16*MAXSEG steps (3D + T of them are needed). Staging, tile geometry and epilogue are the
// polyphase kernel's (R = 4 outputs per lane).
// ------------------------------------------------------------------------------------------------
typedef float gsdr_mf4 __attribute__((ext_vector_type(4)));

// steps 2g and 2g + 1 of a segment (granule g): ABID must be an immediate
template <int G>
__device__ __forceinline__ void mfma_bc_granule(float tv, const float4& w, gsdr_mf4& cre, gsdr_mf4& cim) {
  cre = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, w.x, cre, 4, 2 * G, 0);
  cim = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, w.y, cim, 4, 2 * G, 0);
  cre = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, w.z, cre, 4, 2 * G + 1, 0);
  cim = __builtin_amdgcn_mfma_f32_4x4x1f32(tv, w.w, cim, 4, 2 * G + 1, 0);
}
template <int... G>
__device__ __forceinline__ void mfma_bc_segment(float tv, const float4 (&w)[8], gsdr_mf4& cre, gsdr_mf4& cim,
                                                std::integer_sequence<int, G...>) {
  (mfma_bc_granule<G>(tv, w[G], cre, cim), ...);
}

template <int WG, int MAXSEG, bool VEC, bool NT, int ABL = 0>
__global__ __launch_bounds__(WG) void k_fir_mfma_bc(FirParams p) {
  constexpr int D = 4, R = 4;
  using Geo = TileGeo<float2, D, R, WG>;
  static_assert(Geo::SG == 8 && Geo::PAD == 1, "lane stream layout: 16 steps per 9-granule segment");
  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  const float2* __restrict__ in = reinterpret_cast<const float2*>(p.in);
  const uint64_t out0 = (uint64_t)blockIdx.x * p.tile_stride;
  const uint64_t S0 = out0 * D;
  const uint32_t nk = 3u * D + p.T;             // steps that meet a tap
  const uint32_t nseg = (nk + 15u) / 16u;       // <= MAXSEG (checked by the launcher)
  const uint32_t NG = (D * (Geo::KT - R) + 16u * nseg) / 2;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  float tv[MAXSEG];
#pragma unroll
  for (int c = 0; c < MAXSEG; ++c) {
    const uint32_t i = 16u * c + (lane >> 2) - D * (lane & 3u);  // wraps (>= T) below zero
    tv[c] = i < p.T ? taps[i] : 0.0f;
  }
  if constexpr (ABL != 2) stage_tile<float2, Geo, WG, VEC, kModeFir, NT>(lds, in, S0, NG, p);
  __syncthreads();

  const float4* __restrict__ seg = lds + tid * Geo::SGP;
  gsdr_mf4 cre = {0.f, 0.f, 0.f, 0.f}, cim = cre;
#pragma unroll
  for (int c = 0; c < MAXSEG; ++c) {
    if ((uint32_t)c < nseg) {
      float4 w[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) w[g] = seg[c * Geo::SGP + g];
      mfma_bc_segment(tv[c], w, cre, cim, std::make_integer_sequence<int, 8>{});
    }
  }
  float2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = make_float2(cre[r], cim[r]);
  if constexpr (ABL == 0) {
    if (!all_finite(acc)) ascending_fixup<float, float2, Geo, true, R>(lds, p, D, tid * R, acc);
  }
  tile_epilogue<kModeFir, float2, R, WG, NT>(p, out0, acc, nullptr);
}

template <int WG>
constexpr size_t mfma_bc_lds_bytes(uint32_t T) {
  using Geo = TileGeo<float2, 4, 4, WG>;
  const uint32_t nseg = (12u + T + 15u) / 16u;
  const uint32_t NG = (4u * (Geo::KT - 4) + 16u * nseg) / 2;
  return (size_t)(Geo::padded(NG - 1) + 1) * 16u;
}

// ------------------------------------------------------------------------------------------------
// Host-side sizing helpers
// ------------------------------------------------------------------------------------------------
template <class InT, int D, int R, int WG>
constexpr size_t poly_lds_bytes(uint32_t span_samples, int mode) {
  using Geo = TileGeo<InT, D, R, WG>;
  const uint32_t NG = ((Geo::KT - 1) * D + span_samples + Geo::G - 1) / Geo::G;
  size_t bytes = (size_t)(Geo::padded(NG - 1) + 1) * 16u;
  if (mode != kModeFir) bytes += ((size_t)WG * sizeof(float2) + 15) / 16 * 16;
  return bytes;
}

}  // namespace gsdr
