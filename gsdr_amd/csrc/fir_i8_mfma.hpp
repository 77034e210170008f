// gsdr-mi355x: int8 I/Q FIR and FM / AM chains on the matrix cores (gsdrxFirFCInt8, gsdrxFmDemodInt8,
// gsdrxAmDemodInt8 at decimation 4).
//
// The int8 front end's samples are small integers (|v| <= 127 after gsdrInt8ToNormFloat's clamp), exact in
// bf16, and every fp32 tap is split EXACTLY into three bf16 parts:
//   * taps are scaled by 2^sc (exact) so that max|t| lies in [2^99, 2^100), then
//     t = b1 + b2 + b3 with b1 = bf16(t), b2 = bf16(t - b1), b3 = t - b1 - b2 (8 significant bits each:
//     24 bits in all, so b3 is exact). bf16 has fp32's exponent range, so a tap 2^-200 below the largest
//     is split as exactly as the largest: round 2's two fp16 parts under one scale turned the sinc
//     zero-crossing taps (~1e-18) of an ordinary low-pass into 0, which an impulse or a sparse window
//     exposes at a normwise error of 1 (What's weak 1). A tap set whose split is not exact
//     (dynamic range beyond ~2^200, or not finite) takes the exact per-output loop (fir_point) instead;
//   * every product v * b is exact in fp32 (8 x 8 bits), so the only roundings are the matrix core's fp32
//     accumulation and the final scale y = (acc / 127) 2^-sc -- the reference's per-sample v / 127
//     (conversion.cu:20-35) moved outside the sum of fir.cu:49-71. The result meets the float path's
//     normwise bar for every input, sparse ones included, rather than matching it bit for
//     bit: the products are summed in the matrix core's order.
// Shift invariance: the 16-output blocks a matrix tile is built from are aligned to the ABSOLUTE output
// index (FirParams::out_phase = absolute index of output 0 mod 16), so an output's summation order depends
// only on the taps, its own window and its absolute index mod 16 -- never on where a call starts. The
// streaming object and the multi-channel entry points therefore reproduce one monolithic call bit for bit
// on this path too (include/gsdr/stream.h).
//
// FIR (v_mfma_f32_16x16x32_bf16: A 16x32, B 32x16, C 16x16 fp32):
//   C[m][n] = sum_kk A[m][kk] B[kk][n],  A[m][kk] = t[kk - D m] (zero outside [0, T)),
//   B[kk][n] = component (n & 1) of x[(k0 + 16 (n >> 1)) D + kk],
// so column n holds 16 consecutive outputs (block n >> 1 of the C tile's 8) of one component, and one C
// tile is 128 consecutive complex outputs. K = 15 D + T padded to 32-sample steps (6 at D = 4, T = 127).
// A is the same for every tile: each lane keeps its fragments (3 parts x 8 bf16 per step) in registers for
// the kernel's lifetime (persistent workgroups). B comes from LDS, where the staging pass wrote the tile's
// samples as two bf16 planes (I and Q) with a 16-byte pad after every 64 samples: the 16 lanes that read
// together (one per column) then hit 16 distinct 16-byte bank groups.
#pragma once

#include "fir_engine.hpp"

namespace gsdr {

typedef __bf16 gsdr_b8 __attribute__((ext_vector_type(8)));
typedef __bf16 gsdr_b4 __attribute__((ext_vector_type(4)));
typedef float gsdr_f4v __attribute__((ext_vector_type(4)));
typedef uint32_t gsdr_u4v __attribute__((ext_vector_type(4)));
typedef uint32_t gsdr_u2v __attribute__((ext_vector_type(2)));

// tap scale: max|t| 2^sc in [2^99, 2^100); all-zero taps give sc = 100
__device__ __forceinline__ int i8_tap_scale(float amax) {
  int e = 0;
  (void)frexpf(amax, &e);  // amax = f 2^e, f in [0.5, 1) (e = 0 for amax = 0)
  return 100 - e;
}

__device__ __forceinline__ bool bf16_normal_or_zero(__bf16 b) {
  const float f = (float)b;
  return f == 0.0f || fabsf(f) >= 0x1p-126f;
}

// v = b1 + b2 + b3 exactly (returns false when it is not: v not finite, or a part below bf16's normal range)
__device__ __forceinline__ bool split3(float v, __bf16& b1, __bf16& b2, __bf16& b3) {
  b1 = (__bf16)v;
  const float r1 = v - (float)b1;  // exact: b1 is v rounded to 8 significant bits
  b2 = (__bf16)r1;
  const float r2 = r1 - (float)b2;
  b3 = (__bf16)r2;
  return isfinite(v) && (float)b3 == r2 && bf16_normal_or_zero(b1) && bf16_normal_or_zero(b2) &&
         bf16_normal_or_zero(b3);
}

// Tap parts in LDS for the A fragments: three bf16 rows (b1, b2, b3 of split3) of kI8TapPad zeros followed by
// the parts of taps 0 .. 255 (zero past T). A lane's fragment for one K step is 8 consecutive taps, so it is one
// 16-byte gather from a row (two 8-byte LDS reads) after one split a thread, where splitting the fragment
// entries in every lane took 48 splits a lane (~3 us of VALU at the start of every launch).
constexpr int kI8TapPad = 64;  // >= 15 D, the most negative tap index a fragment reaches (D = 4); 8-byte aligned rows
constexpr int kI8TapRow = kI8TapPad + 256;
__device__ __forceinline__ void i8_put_tap_parts(__bf16* parts, uint32_t tid, float v) {
  __bf16 b1, b2, b3;
  (void)split3(v, b1, b2, b3);  // exactness is checked by the caller's reduction
  parts[kI8TapPad + tid] = b1;
  parts[kI8TapRow + kI8TapPad + tid] = b2;
  parts[2 * kI8TapRow + kI8TapPad + tid] = b3;
  if (tid < (uint32_t)kI8TapPad) {
#pragma unroll
    for (int k = 0; k < 3; ++k) parts[k * kI8TapRow + tid] = (__bf16)0.0f;
  }
}
// taps i0 .. i0 + 7 of one part row (i0 >= -kI8TapPad, i0 a multiple of 4)
__device__ __forceinline__ gsdr_b8 i8_tap_row(const __bf16* row, int i0) {
  const char* b = reinterpret_cast<const char*>(row + kI8TapPad + i0);
  const gsdr_u2v lo = *reinterpret_cast<const gsdr_u2v*>(b), hi = *reinterpret_cast<const gsdr_u2v*>(b + 8);
  const gsdr_u4v u = {lo.x, lo.y, hi.x, hi.y};
  return __builtin_bit_cast(gsdr_b8, u);
}

// int8 component (bits [8 u, 8 u + 8) of w) as gsdrInt8ToNormFloat's numerator: clamp -128 to -127
__device__ __forceinline__ __bf16 i8_bf16(uint32_t w, int u) {
  return (__bf16)(float)max((int)(w << (24 - 8 * u)) >> 24, -127);
}

// sample i of the call's input (FirParams::in_off / hist): in[i] for 0 <= i < L, the history before it,
// zero elsewhere
__device__ __forceinline__ Iq8 i8_sample(const FirParams& p, int64_t i) {
  if (i >= 0) return (uint64_t)i < p.L ? reinterpret_cast<const Iq8*>(p.in)[i] : Iq8{0, 0};
  return (p.hist != nullptr && -i <= (int64_t)p.hist_len) ? reinterpret_cast<const Iq8*>(p.hist)[(int64_t)p.hist_len + i]
                                                           : Iq8{0, 0};
}

// The exact per-output evaluation for taps that are not finite or cannot be split: fir_point's ascending
// loop (fir_engine.hpp), with the samples read through i8_sample (history and offset aware)
template <int MODE>
__device__ __forceinline__ float2 i8_point(const FirParams& p, uint64_t k) {
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  float2 acc;
  set_zero(acc);
  const uint64_t s0 = k * p.D;
  for (uint32_t i = 0; i < p.T; ++i) {
    auto x = to_lds_sample(i8_sample(p, (int64_t)(s0 + i) + p.in_off));
    if constexpr (MODE != kModeFir) {
      x = nco_mix(x, p.nco_n0 + (uint32_t)(s0 + i), p.nco_inc);
    }
    mac(acc, x, taps[i]);
  }
  return acc;
}

// The streaming object's next history (FirParams::hist_out), copied by workgroup 0
__device__ __forceinline__ void i8_copy_history(const FirParams& p) {
  if (p.hist_out == nullptr || blockIdx.x != 0) return;
  Iq8* dst = reinterpret_cast<Iq8*>(p.hist_out);
  for (uint64_t j = threadIdx.x; j < p.hist_n; j += blockDim.x) dst[j] = i8_sample(p, p.hist_from + (int64_t)j);
}

// Reduce |value| max and a "not exactly representable" flag over the workgroup (WG threads, 64-lane waves).
template <int WG>
__device__ __forceinline__ void wg_max_bad(float& a, uint32_t& bad, float* wmax, uint32_t* wbad) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (int o = 32; o > 0; o >>= 1) {
    a = fmaxf(a, __shfl_xor(a, o, 64));
    bad |= __shfl_xor(bad, o, 64);
  }
  if (lane == 0) {
    wmax[w] = a;
    wbad[w] = bad;
  }
  __syncthreads();
  a = wmax[0];
  bad = wbad[0];
#pragma unroll
  for (int i = 1; i < WG / 64; ++i) {
    a = fmaxf(a, wmax[i]);
    bad |= wbad[i];
  }
}

// Cross-lane moves without LDS: lane ^ 1 by DPP (quad_perm [1, 0, 3, 2]), lane ^ 32 by gfx950's
// v_permlane32_swap (__shfl_xor compiles to ds_bpermute, an LDS instruction with its own wait)
__device__ __forceinline__ float lane_xor1(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ float lane_xor32(float x) {
  // swap(vdst = x, src = x): vdst's lanes 32-63 <- src's lanes 0-31, src's lanes 0-31 <- vdst's lanes 32-63
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32u) ? r[0] : r[1]);
}

// Output scale 2^-sc / 127: one multiply by that constant while it is a normal float (then it equals
// 2^-sc fl(1/127) exactly, and acc * it rounds once), else (acc / 127-ish) then the exponent shift
// (as ldexpf(acc * k, sh): k = that constant and sh = 0, or k = fl(1/127) and sh = -sc; two instructions, no
// select)
struct I8OutScale {
  float k;
  int sh;
  __device__ __forceinline__ explicit I8OutScale(int sc)
      : k(sc <= 118 ? ldexpf(1.0f / 127.0f, -sc) : 1.0f / 127.0f), sh(sc <= 118 ? 0 : -sc) {}
  __device__ __forceinline__ float operator()(float acc) const { return ldexpf(acc * k, sh); }
};

// LDS plane layout: 2 bytes a sample, a 16-byte pad after every P samples. P is chosen per kernel so the
// B-fragment reads (ds_read_b128, 16 lanes a cycle in the lane groups of MI355X_MICROARCH.md section LDS) hit
// 16 distinct 16-byte bank slots, with the Q plane 128 bytes (mod 256) past the I plane: P = 32 for the FIR
// kernel (lanes 16 b + 4 q' outputs apart), P = 16 for the chain kernel (8 b). Round 3's P = 64 for both took
// 2x (FIR) and 2.5x (chain) the conflict-free LDS cycles (PMC: 42 % of the chain's LDS-active cycles were bank
// conflicts, profiles/r04_pmc_kernels.txt). The chain is VALU-bound: P = 16 / 32 / 64 time the same
// (profiles/r04_ab_o.txt), and 16 keeps its LDS cycles lowest.
// (GSDR_I8_FIR_PADP / GSDR_I8_CHAIN_PADP: probe-build overrides for layout A/B timing)
#if !defined(GSDR_TUNING_PROBES) && (defined(GSDR_I8_FIR_PADP) || defined(GSDR_I8_CHAIN_PADP) || defined(GSDR_I8_FM_PROBE))
#error "the int8 LDS pad periods are fixed outside the probe builds"
#endif
#ifndef GSDR_I8_FIR_PADP
#define GSDR_I8_FIR_PADP 32
#endif
#ifndef GSDR_I8_CHAIN_PADP
#define GSDR_I8_CHAIN_PADP 16
#endif
template <uint32_t P>
__host__ __device__ constexpr uint32_t i8_addr(uint32_t idx) {
  return idx * 2u + (idx / P) * 16u;
}

// Staging of samples [S0, S0 + SPAN) (absolute offsets into `in`, zero outside [0, L)) as bf16 I and Q
// planes, in two halves so the next tile's loads can be in flight while this tile is computed (the
// kernels are persistent, so a tile's HBM latency would otherwise stand between every two tiles):
// i8_load_granules issues every load of a tile into registers, i8_store_planes converts and writes them.
// G samples a lane and load (8: 16-byte loads, 4: 8-byte loads); VEC = the in-range granules are
// G * 2-byte aligned.
template <int G, int SPAN, int WG>
struct I8Stage {
  static_assert(G == 8 || G == 4, "granule of 8 or 4 samples");
  static_assert(SPAN % G == 0, "whole granules");
  static constexpr uint32_t NG = SPAN / G, NGR = (NG + WG - 1) / WG;
  static constexpr int NW = G / 2;  // dwords a granule
  uint32_t wv[NGR][NW];
};

// LM (load mode): 1 = the tile starts are G * 2-byte aligned (one vector load a granule); 2 = they are
// 2-byte aligned only (G = 4: a chunk of a stream that ended on an odd sample count): two aligned 8-byte
// loads a granule and a funnel shift (v_alignbit_b32) by the sample offset; 0 = per-sample loads.
// Interior tiles (all but the first and last of a launch) need no per-granule bounds: a uniform base plus a
// 32-bit lane offset per load.
template <int G, int LM, int SPAN, int WG>
__device__ __forceinline__ void i8_load_granules(I8Stage<G, SPAN, WG>& st, const FirParams& p, int64_t S0) {
  static_assert(LM != 2 || G == 4, "shifted loads move 4-sample granules");
  const Iq8* __restrict__ in = reinterpret_cast<const Iq8*>(p.in);
  const uint64_t L = p.L;
  using S = I8Stage<G, SPAN, WG>;
  const uint32_t tid = threadIdx.x;
  if (LM == 1 && S0 >= 0 && (uint64_t)S0 + SPAN <= L) {
    const char* base = reinterpret_cast<const char*>(in + S0);
#pragma unroll
    for (uint32_t r = 0; r < S::NGR; ++r) {
      const uint32_t g = tid + r * WG;
      if (r + 1 < S::NGR || g < S::NG) {
        if constexpr (G == 8) {
          const gsdr_u4v t = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u4v*>(base + 16u * g));
#pragma unroll
          for (int k = 0; k < 4; ++k) st.wv[r][k] = t[k];
        } else {
          const gsdr_u2v t = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u2v*>(base + 8u * g));
          st.wv[r][0] = t.x;
          st.wv[r][1] = t.y;
        }
      }
    }
    return;
  }
  if constexpr (LM == 2) {
    const uint32_t dl = (uint32_t)((reinterpret_cast<uintptr_t>(in + S0) >> 1) & 3u);  // samples past 8-byte alignment
    if (S0 >= (int64_t)dl && (uint64_t)S0 + SPAN + 4 <= L) {
      const char* base = reinterpret_cast<const char*>(in + S0) - 2 * dl;  // 8-byte aligned
      const bool up = dl >= 2;                   // the wanted dwords start in the second dword
      const uint32_t sh = (dl & 1u) ? 16u : 0u;  // and half a dword further
#pragma unroll
      for (uint32_t r = 0; r < S::NGR; ++r) {
        const uint32_t g = tid + r * WG;
        if (r + 1 < S::NGR || g < S::NG) {
          const gsdr_u2v a = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u2v*>(base + 8u * g));
          const gsdr_u2v b = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u2v*>(base + 8u * g + 8u));
          const uint32_t d0 = up ? a.y : a.x, d1 = up ? b.x : a.y, d2 = up ? b.y : b.x;
          st.wv[r][0] = __builtin_amdgcn_alignbit(d1, d0, sh);
          st.wv[r][1] = __builtin_amdgcn_alignbit(d2, d1, sh);
        }
      }
      return;
    }
  }
  // edge tiles: granule by granule, vector loads where the granule (and, shifted, its aligned cover) lies in
  // the input
  const uint32_t dl2 = LM == 2 ? (uint32_t)((reinterpret_cast<uintptr_t>(in + S0) >> 1) & 3u) : 0u;
#pragma unroll
  for (uint32_t r = 0; r < S::NGR; ++r) {
    const uint32_t g = tid + r * WG;
    const int64_t s = S0 + (int64_t)G * g;
#pragma unroll
    for (int k = 0; k < S::NW; ++k) st.wv[r][k] = 0u;
    if (g < S::NG) {
      if (LM == 1 && s >= 0 && (uint64_t)s + G <= L) {
        if constexpr (G == 8) {
          const gsdr_u4v t = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u4v*>(in + s));
#pragma unroll
          for (int k = 0; k < 4; ++k) st.wv[r][k] = t[k];
        } else {
          const gsdr_u2v t = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u2v*>(in + s));
          st.wv[r][0] = t.x;
          st.wv[r][1] = t.y;
        }
      } else if (LM == 2 && s >= (int64_t)dl2 && (uint64_t)s - dl2 + 8 <= L) {
        const char* a8 = reinterpret_cast<const char*>(in + s) - 2 * dl2;
        const gsdr_u2v a = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u2v*>(a8));
        const gsdr_u2v b = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u2v*>(a8 + 8));
        const bool up = dl2 >= 2;
        const uint32_t sh = (dl2 & 1u) ? 16u : 0u;
        const uint32_t d0 = up ? a.y : a.x, d1 = up ? b.x : a.y, d2 = up ? b.y : b.x;
        st.wv[r][0] = __builtin_amdgcn_alignbit(d1, d0, sh);
        st.wv[r][1] = __builtin_amdgcn_alignbit(d2, d1, sh);
      } else {  // input ends, unaligned input or samples before the buffer: per-sample loads
#pragma unroll
        for (int k = 0; k < S::NW; ++k) {
          const Iq8 a = i8_sample(p, s + 2 * k), b = i8_sample(p, s + 2 * k + 1);
          st.wv[r][k] = (uint32_t)(uint8_t)a.x | (uint32_t)(uint8_t)a.y << 8 | (uint32_t)(uint8_t)b.x << 16 |
                        (uint32_t)(uint8_t)b.y << 24;
        }
      }
    }
  }
}

template <uint32_t P, int G, int SPAN, int WG>
__device__ __forceinline__ void i8_store_planes(const I8Stage<G, SPAN, WG>& st, char* lds, uint32_t plane) {
  using S = I8Stage<G, SPAN, WG>;
  static_assert(P % G == 0, "a granule never straddles a pad");
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (uint32_t r = 0; r < S::NGR; ++r) {
    const uint32_t g = tid + r * WG;
    if (g < S::NG) {
      const uint32_t o = i8_addr<P>(G * g);
      if constexpr (G == 8) {
        gsdr_b8 hi_, hq_;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {  // sample 2k + u: bytes 2u (I) and 2u + 1 (Q) of dword k
            hi_[2 * k + u] = i8_bf16(st.wv[r][k], 2 * u);
            hq_[2 * k + u] = i8_bf16(st.wv[r][k], 2 * u + 1);
          }
        }
        *reinterpret_cast<gsdr_b8*>(lds + o) = hi_;
        *reinterpret_cast<gsdr_b8*>(lds + plane + o) = hq_;
      } else {
        gsdr_b4 hi_, hq_;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            hi_[2 * k + u] = i8_bf16(st.wv[r][k], 2 * u);
            hq_[2 * k + u] = i8_bf16(st.wv[r][k], 2 * u + 1);
          }
        }
        *reinterpret_cast<gsdr_b4*>(lds + o) = hi_;
        *reinterpret_cast<gsdr_b4*>(lds + plane + o) = hq_;
      }
    }
  }
}

template <int D, int NS_, int NCT_ = 4>
struct I8Mfma {
  static constexpr int WG = 256;
  static constexpr int NCT = NCT_;                  // C tiles (128 outputs) per wave and tile
  static constexpr int KT = (WG / 64) * NCT * 128;  // outputs per tile (a multiple of 16)
  static constexpr int MAXNS = NS_;                 // 32-sample K steps: 15 D + T <= 32 NS
  static constexpr int MAXT = 32 * MAXNS - 15 * D;
  static constexpr int SPAN = (KT - 16) * D + 32 * MAXNS;  // samples staged per tile
  static_assert(SPAN % 8 == 0, "staging moves 8 samples a lane");
  static constexpr uint32_t PADP = GSDR_I8_FIR_PADP;  // pad period (i8_addr)
  __host__ __device__ static constexpr uint32_t addr(uint32_t idx) { return i8_addr<PADP>(idx); }
  // Q plane offset: = 128 (mod 256), so the Q columns' bank groups interleave the I columns'
  static constexpr uint32_t PLANE = (addr(SPAN) + 255u) / 256u * 256u + 128u;
  static constexpr uint32_t LDS_BYTES = PLANE + addr(SPAN);
};

// BPC workgroups per CU (one wave per SIMD each): the register budget is 512 / BPC VGPRs.
// G / LM: staging granule and load mode (I8Stage, i8_load_granules); OA: the output pairs (k, k + 1) are 16-byte aligned.
// NCT: C tiles per wave and tile (4; 1 for short calls, whose few large tiles would leave most workgroup
// slots idle -- an output's summation order does not depend on the tile size, only on its 16-output block)
// PF: tiles in flight a workgroup (1: the next tile's loads fly while this one is computed; 2: the next two,
// for short calls of small tiles, whose compute is too short to cover one tile's HBM latency)
template <int D, int NS, int G, int LM, bool OA, int BPC, int NCT = 4, int PF = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BPC, BPC))) void k_fir_i8_mfma(FirParams p, uint32_t ns, uint32_t tiles) {
  static_assert(PF == 1 || PF == 2, "one or two tiles in flight");
  using C = I8Mfma<D, NS, NCT>;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS_BYTES];
  __shared__ float wmax[C::WG / 64];
  __shared__ uint32_t wbad[C::WG / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  float2* __restrict__ out = reinterpret_cast<float2*>(p.out);
  const uint32_t T = p.T;
  const int64_t phase = (int64_t)p.out_phase;
  i8_copy_history(p);
  // the first tiles' loads fly while the tap fragments are built
  I8Stage<G, C::SPAN, C::WG> st, st2;
  if (blockIdx.x < tiles) i8_load_granules<G, LM>(st, p, ((int64_t)blockIdx.x * C::KT - phase) * D + p.in_off);
  if (PF == 2 && blockIdx.x + gridDim.x < tiles) {
    i8_load_granules<G, LM>(st2, p, ((int64_t)(blockIdx.x + gridDim.x) * C::KT - phase) * D + p.in_off);
  }

  // tap scale (T <= MAXT <= 256: one tap a thread); `bad` = some tap is not finite
  const float t = tid < T ? taps[tid] : 0.0f;
  float amax = fabsf(t);
  uint32_t bad = isfinite(t) ? 0u : 1u;
  wg_max_bad<C::WG>(amax, bad, wmax, wbad);
  const int sc = i8_tap_scale(amax);
  if (!bad) {  // and whether every scaled tap splits exactly
    __bf16 b1, b2, b3;
    uint32_t inexact = split3(ldexpf(t, sc), b1, b2, b3) ? 0u : 1u;
    float dummy = 0.0f;
    __syncthreads();  // wmax / wbad are reused
    wg_max_bad<C::WG>(dummy, inexact, wmax, wbad);
    bad = inexact;
  }
  if (bad) {  // the reference's ascending loop, output by output
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
      for (uint32_t r = tid; r < (uint32_t)C::KT; r += C::WG) {
        const int64_t k = (int64_t)tile * C::KT - phase + r;
        if (k >= 0 && (uint64_t)k < p.N) out[k] = i8_point<kModeFir>(p, (uint64_t)k);
      }
    }
    return;
  }
  // the scaled taps' parts in LDS (zero past T), then this lane's A fragments: row m = lane & 15,
  // k = 8 (lane >> 4) + j, tap 32 s + k - D m (<= 255)
  static_assert(D == 4, "tap rows gathered at 8-byte aligned offsets (D m a multiple of 4, 15 D <= kI8TapPad)");
  static_assert(C::LDS_BYTES >= 3 * kI8TapRow * sizeof(__bf16), "tap rows fit the tile's LDS");
  __bf16* parts = reinterpret_cast<__bf16*>(lds);
  i8_put_tap_parts(parts, tid, ldexpf(t, sc));
  __syncthreads();
  gsdr_b8 a1[C::MAXNS], a2[C::MAXNS], a3[C::MAXNS];
  {
    const int m = (int)(lane & 15u), q = (int)(lane >> 4);
#pragma unroll
    for (int s = 0; s < C::MAXNS; ++s) {
      const int i0 = 32 * s + 8 * q - D * m;
      a1[s] = i8_tap_row(parts, i0);
      a2[s] = i8_tap_row(parts + kI8TapRow, i0);
      a3[s] = i8_tap_row(parts + 2 * kI8TapRow, i0);
    }
  }
  const I8OutScale oscale(sc);
  __syncthreads();  // the tap table is overwritten by the first tile's samples

  const int n = (int)(lane & 15u), q = (int)(lane >> 4), c = n & 1, b = n >> 1;
  const char* bplane = lds + (c ? C::PLANE : 0u);
  auto run_tile = [&](uint32_t tile, I8Stage<G, C::SPAN, C::WG>& cur) {
    const int64_t k_t = (int64_t)tile * C::KT - phase;  // a multiple of 16 in absolute output index
    // the tile's outputs as 32-bit offsets from a uniform base: its writable range [lo, hi) (64-bit index
    // arithmetic and compares per output had cost ~6 VALU instructions an output)
    float2* __restrict__ out_t = out + k_t;
    const uint32_t lo = k_t < 0 ? (uint32_t)(-k_t) : 0u;
    const uint32_t hi = (int64_t)p.N - k_t < (int64_t)C::KT ? (uint32_t)((int64_t)p.N - k_t) : (uint32_t)C::KT;
    i8_store_planes<C::PADP>(cur, lds, C::PLANE);
    __syncthreads();
    // the loads of the tile PF rounds on fly while this one is computed
    if (tile + PF * gridDim.x < tiles) {
      i8_load_granules<G, LM>(cur, p, (k_t + (int64_t)(PF * gridDim.x) * C::KT) * D + p.in_off);
    }
#pragma unroll 1
    for (int ct = 0; ct < C::NCT; ++ct) {
      const uint32_t cbase = (w * C::NCT + (uint32_t)ct) * 128u;  // the C tile's first output in the tile
      const uint32_t idx0 = (cbase + 16u * (uint32_t)b) * D + 8u * (uint32_t)q;
      gsdr_f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < C::MAXNS; ++s) {  // steps past 15 D + T meet zero taps
        const gsdr_b8 bf = *reinterpret_cast<const gsdr_b8*>(bplane + C::addr(idx0 + 32u * (uint32_t)s));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[s], bf, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[s], bf, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], bf, acc, 0, 0, 0);
      }
      // lane (q, b, c) holds component c of outputs 4q .. 4q + 3 of block b; the I lane keeps rows 0-1 and
      // the Q lane rows 2-3, each taking the other component from its neighbour
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = oscale(acc[i]);
      const float g0 = lane_xor1(c ? r[0] : r[2]), g1 = lane_xor1(c ? r[1] : r[3]);
      const float4 o4 = c ? make_float4(g0, r[2], g1, r[3]) : make_float4(r[0], g0, r[1], g1);
      const uint32_t kr = cbase + 16u * (uint32_t)b + 4u * (uint32_t)q + 2u * (uint32_t)c;  // within the tile
      if (kr >= lo && kr + 1 < hi) {
        if constexpr (OA) {
          store16_nt(reinterpret_cast<float4*>(out_t + kr), o4);
        } else {
          out_t[kr] = make_float2(o4.x, o4.y);
          out_t[kr + 1] = make_float2(o4.z, o4.w);
        }
      } else {
        if (kr >= lo && kr < hi) out_t[kr] = make_float2(o4.x, o4.y);
        if (kr + 1 >= lo && kr + 1 < hi) out_t[kr + 1] = make_float2(o4.z, o4.w);
      }
    }
    __syncthreads();  // every wave is done reading the tile's planes
  };
  if constexpr (PF == 1) {
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) run_tile(tile, st);
  } else {  // the two register sets alternate (static indices: unrolled by two)
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += 2u * gridDim.x) {
      run_tile(tile, st);
      if (tile + gridDim.x >= tiles) break;
      run_tile(tile + gridDim.x, st2);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// int8 I/Q FM / AM chains on the matrix cores (gsdrxFmDemodInt8 / gsdrxAmDemodInt8, D = 4, T <= 132).
// The NCO moves into the taps: with phi(n) the mixer phase of sample n (exact integer phase, fir_engine.hpp),
//   y[k] = sum_i t_i x[4k+i] e^{j phi(4k+i)} = e^{j phi(4k)} y'[k],  y'[k] = sum_i t'_i x[4k+i],
//   t'_i = t_i e^{j 2 pi (i inc mod 2^32) / 2^32}
// (the phase is additive mod 2^32). The AM envelope |y| = |y'|, and the FM discriminator
// arg(y[k+1] conj y[k]) = arg(y'[k+1] conj y'[k]) + 2 pi (4 inc mod 2^32) / 2^32 (wrapped) wherever that
// product is nonzero, so neither needs the rotation: the chain is a complex-tap FIR on the raw int8
// samples, with the taps split into three exact bf16 parts as in k_fir_i8_mfma.
// Layout: a C tile is 64 consecutive outputs. A's rows 0-7 hold the real parts t'r of 8 consecutive
// outputs' taps and rows 8-15 the imaginary parts t'i of the same 8 outputs (A[m][kk] = t'r[kk - 4m],
// A[8 + m][kk] = t'i[kk - 4m]); column n = 2 b + c is component c of the 8-output block b. So one MFMA
// gives both tap sums, K = 7 D + T = 155 fits 5 steps (a 16-output row block needs 6 and twice the
// registers), and per 32-sample step 3 MFMAs (one a part). With P / Q' the real / imaginary-tap sums of
// the I column and R / S those of the Q column, y' = (P - S) + j (R + Q'): lane (q, n) and lane
// (q ^ 2, n ^ 1) hold the two terms of one component, one lane exchange apart.
// FM tiles overlap by 16 outputs (stride KT - 16, so every tile start stays a 16-multiple of the absolute
// output index); each lane keeps its y' in registers and takes y'[k + 1] from the lane holding it (one
// exchange per C tile; only a wave's last output reads the next wave's first through LDS).
// Normwise parity with the float chains, not bit identity (gsdr_ext.h).
// ------------------------------------------------------------------------------------------------
template <int MODE, int NCT_ = 4>
struct I8ChainMfma {
  static constexpr int D = 4;
  static constexpr int WG = 256;
  static constexpr int NCT = NCT_;                 // C tiles (64 outputs) per wave and tile
  static constexpr int KT = (WG / 64) * NCT * 64;  // y' per tile (a multiple of 16)
  static constexpr int STRIDE = MODE == kModeFm ? KT - 16 : KT;
  static constexpr int MAXNS = 5;
  static constexpr int MAXT = 32 * MAXNS - 7 * D;  // 132
  static constexpr int SPAN = (KT - 8) * D + 32 * MAXNS;
  static_assert(SPAN % 4 == 0, "whole granules");
  static constexpr uint32_t PADP = GSDR_I8_CHAIN_PADP;  // pad period (i8_addr)
  __host__ __device__ static constexpr uint32_t addr(uint32_t idx) { return i8_addr<PADP>(idx); }
  static constexpr uint32_t PLANE = (addr(SPAN) + 255u) / 256u * 256u + 128u;
  static constexpr uint32_t LDS_BYTES = PLANE + addr(SPAN);
};

template <int MODE, int LM, int BPC, int NCT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BPC, BPC))) void k_chain_i8_mfma(FirParams p, uint32_t ns, uint32_t tiles) {
  using C = I8ChainMfma<MODE, NCT>;
  constexpr int D = C::D;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS_BYTES];
  __shared__ float2 wfirst[MODE == kModeFm ? C::WG / 64 : 1];  // FM: each wave's first y' of the tile
  __shared__ float wmax[C::WG / 64];
  __shared__ uint32_t wbad[C::WG / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  float* __restrict__ out = reinterpret_cast<float*>(p.out);
  const uint32_t T = p.T;
  const int64_t phase = (int64_t)p.out_phase;
  i8_copy_history(p);
  // the first tile's loads fly while the tap fragments are built
  I8Stage<4, C::SPAN, C::WG> st;
  if (blockIdx.x < tiles) i8_load_granules<4, LM>(st, p, ((int64_t)blockIdx.x * C::STRIDE - phase) * D + p.in_off);

  // modulated taps t'_i = t_i e^{j 2 pi (i inc) / 2^32}
  const float t = tid < T ? taps[tid] : 0.0f;
  const float2 ph = nco_direct(tid * p.nco_inc);
  const float tr = t * ph.x, ti = t * ph.y;
  float amax = fmaxf(fabsf(tr), fabsf(ti));
  uint32_t bad = isfinite(t) ? 0u : 1u;
  wg_max_bad<C::WG>(amax, bad, wmax, wbad);
  const int sc = i8_tap_scale(amax);
  if (!bad) {
    __bf16 b1, b2, b3;
    uint32_t inexact = (split3(ldexpf(tr, sc), b1, b2, b3) && split3(ldexpf(ti, sc), b1, b2, b3)) ? 0u : 1u;
    float dummy = 0.0f;
    __syncthreads();
    wg_max_bad<C::WG>(dummy, inexact, wmax, wbad);
    bad = inexact;
  }
  if (bad) {  // non-finite or unsplittable taps: the exact per-output chain (the generic kernel's evaluation)
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
      for (uint32_t r = tid; r < (uint32_t)C::STRIDE; r += C::WG) {
        const int64_t k = (int64_t)tile * C::STRIDE - phase + r;
        if (k < 0 || (uint64_t)k >= p.N) continue;
        const float2 y0 = i8_point<MODE>(p, (uint64_t)k);
        if constexpr (MODE == kModeFm) {
          out[k] = fm_disc(y0, i8_point<MODE>(p, (uint64_t)k + 1), p.fm_gain);
        } else {
          out[k] = am_env(y0);
        }
      }
    }
    return;
  }
  // the parts of t'r and t'i in LDS (i8_put_tap_parts), then this lane's A fragments: tap 32 s + 8 q + j - D m
  // (<= 159) of the real (rows 0-7) or imaginary (rows 8-15) taps
  static_assert(C::LDS_BYTES >= 6 * kI8TapRow * sizeof(__bf16), "tap rows fit the tile's LDS");
  __bf16* parts = reinterpret_cast<__bf16*>(lds);
  i8_put_tap_parts(parts, tid, ldexpf(tr, sc));
  i8_put_tap_parts(parts + 3 * kI8TapRow, tid, ldexpf(ti, sc));
  __syncthreads();
  gsdr_b8 a1[C::MAXNS], a2[C::MAXNS], a3[C::MAXNS];
  {
    const int m = (int)(lane & 7u), im = (int)((lane >> 3) & 1u), q = (int)(lane >> 4);
    const __bf16* tab = parts + (im ? 3 * kI8TapRow : 0);
#pragma unroll
    for (int s = 0; s < C::MAXNS; ++s) {
      const int i0 = 32 * s + 8 * q - D * m;
      a1[s] = i8_tap_row(tab, i0);
      a2[s] = i8_tap_row(tab + kI8TapRow, i0);
      a3[s] = i8_tap_row(tab + 2 * kI8TapRow, i0);
    }
  }
  // FM: the rotation the taps leave out, 2 pi (4 inc mod 2^32) / 2^32 in (-pi, pi]
  const float dphi = (float)((double)(int32_t)(4u * p.nco_inc) * (6.283185307179586 / 4294967296.0));
  const I8OutScale oscale(sc);
  __syncthreads();

  const uint32_t n = lane & 15u, q = lane >> 4, c = n & 1u, b = n >> 1;
  const uint32_t hi = q >> 1;         // rows 8-15 (imaginary-tap sums)
  const bool is_re = (c == 0) == (hi == 0);  // this lane ends up with Re y' (else Im y')
  // one output a lane: lanes (q, c) of a block pair up as (Re, Im) of rows 4 (q & 1) + sel
  const uint32_t sel = 2u * hi + (is_re ? 0u : 1u);
  const bool sel_b0 = !is_re;  // the partner lane keeps row sel ^ 1
  const uint32_t hmask = hi ? 0xffffffffu : 0u, b0mask = sel_b0 ? 0xffffffffu : 0u;
  // sign flips for Re = P - S: the P lane (q < 2) negates the partner's S, the S lane (q >= 2) its own
  const uint32_t sg_acc = (is_re && hi) ? 0x80000000u : 0u, sg_oth = (is_re && !hi) ? 0x80000000u : 0u;
  const char* bplane = lds + (c ? C::PLANE : 0u);
  const uint32_t w = tid >> 6;
  // FM: this lane's output within its C tile, o = 8 b + 4 (q & 1) + sel, and the lane holding o + 1
  // (the inverse of the map: offset m = o' & 7 sits in lane quarter ((m >> 1) & 1) * 2 + (m >> 2), column
  // parity (m ^ (m >> 1)) & 1); o = 63's neighbour is the next C tile's output 0 (lane 0)
  const uint32_t o_lane = 8u * b + 4u * (q & 1u) + sel;
  const uint32_t o_next = (o_lane + 1u) & 63u, m_next = o_next & 7u;
  const int nb_lane = (int)(16u * (((m_next >> 1) & 1u) * 2u + (m_next >> 2)) + 2u * (o_next >> 3) +
                            ((m_next ^ (m_next >> 1)) & 1u));
  float2 ycur[MODE == kModeFm ? C::NCT : 1];
  for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t k_t = (int64_t)tile * C::STRIDE - phase;  // a multiple of 16 in absolute output index
    // the tile's outputs as 32-bit offsets from a uniform base, writable in [out_lo, out_hi)
    float* __restrict__ out_t = out + k_t;
    const uint32_t out_lo = k_t < 0 ? (uint32_t)(-k_t) : 0u;
    const uint32_t out_hi = (int64_t)p.N - k_t < (int64_t)C::STRIDE ? (uint32_t)((int64_t)p.N - k_t) : (uint32_t)C::STRIDE;
    i8_store_planes<C::PADP>(st, lds, C::PLANE);
    __syncthreads();
    // the next tile's loads fly while this one is computed
    if (tile + gridDim.x < tiles) {
      i8_load_granules<4, LM>(st, p, (k_t + (int64_t)gridDim.x * C::STRIDE) * D + p.in_off);
    }
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
      const uint32_t cbase = (w * C::NCT + (uint32_t)ct) * 64u;
      const uint32_t idx0 = (cbase + 8u * b) * D + 8u * q;
      gsdr_f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < C::MAXNS; ++s) {  // steps past 15 D + T meet zero taps
        const gsdr_b8 bf = *reinterpret_cast<const gsdr_b8*>(bplane + C::addr(idx0 + 32u * (uint32_t)s));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[s], bf, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[s], bf, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], bf, acc, 0, 0, 0);
      }
      // lane (q, c) holds rows 4q .. 4q + 3 of column (b, c): P (q < 2, c = 0), R (q < 2, c = 1),
      // Q' (q >= 2, c = 0), S (q >= 2, c = 1); its partner lane ^ 33 holds the other term of one component
      // This lane needs rows 2 hi and 2 hi + 1 of its component (the rows it and its lane ^ 1 partner keep);
      // lane ^ 33 needs the other two: swap them, then Re = P - S, Im = R + Q' (commutative), as
      // (+-acc) + (+-other) with per-lane signs, the same rounded operation on both lanes of a pair
      float v[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // bit selects (v_bfi_b32) with a lane mask, not a runtime index into acc (which compiles to compare chains)
        const uint32_t lo_ = __float_as_uint(acc[j]), hi_ = __float_as_uint(acc[2 + j]);
        const float keep = __uint_as_float((hi_ & hmask) | (lo_ & ~hmask));
        const float give = __uint_as_float((lo_ & hmask) | (hi_ & ~hmask));
        const float other = lane_xor1(lane_xor32(give));
        const float pa = __int_as_float(__float_as_int(keep) ^ sg_acc);
        const float po = __int_as_float(__float_as_int(other) ^ sg_oth);
        v[j] = oscale(pa + po);
      }
      // the Re and Im lanes of these two rows are lane and lane ^ 1; lane keeps row sel, sends row sel ^ 1
      const uint32_t v0 = __float_as_uint(v[0]), v1 = __float_as_uint(v[1]);
      const float mine = __uint_as_float((v1 & b0mask) | (v0 & ~b0mask));
      const float got = lane_xor1(__uint_as_float((v0 & b0mask) | (v1 & ~b0mask)));
      // (Re, Im): the Re lane's own value first (b0mask is all ones exactly on the Im lanes)
      const uint32_t mi = __float_as_uint(mine), gi = __float_as_uint(got);
      const float2 y = make_float2(__uint_as_float((gi & b0mask) | (mi & ~b0mask)),
                                   __uint_as_float((mi & b0mask) | (gi & ~b0mask)));
      const uint32_t rr = cbase + o_lane;  // this lane's output within the tile
      if constexpr (MODE == kModeAm) {
        if (rr >= out_lo && rr < out_hi) out_t[rr] = am_env(y);
      } else {
        ycur[ct] = y;
        if (ct == 0 && lane == 0u) wfirst[w] = y;  // output 0 of the wave's first C tile
      }
    }
#if defined(GSDR_I8_FM_PROBE) && GSDR_I8_FM_PROBE == 1
    // timing probe (probe builds only): the FM tile without the neighbour exchange and the discriminator
    if constexpr (MODE == kModeFm) {
      __syncthreads();
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) {
        const uint32_t rr = (w * C::NCT + (uint32_t)ct) * 64u + o_lane;
        if (rr >= out_lo && rr < out_hi) out_t[rr] = ycur[ct].x + ycur[ct].y;
      }
    } else
#endif
    if constexpr (MODE == kModeFm) {
      // One barrier for the planes (read by every wave's MFMAs) and the waves' first outputs; the next tile's
      // staging barrier orders the reads of wfirst below before its next writes. Every other neighbour
      // y'[k + 1] is in this wave's registers: one lane exchange per C tile.
      __syncthreads();
      // (every exchange runs on all lanes: a lane exchange reads only active lanes' registers)
      const float2 wnext = wfirst[w + 1u < C::WG / 64u ? w + 1u : w];
      float2 ynx[C::NCT];
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) {
        const float nx = __shfl(ycur[ct].x, nb_lane, 64), ny = __shfl(ycur[ct].y, nb_lane, 64);
        // o = 63: the next C tile's output 0 (lane 0), or for the wave's last C tile the next wave's first
        float2 first = wnext;
        if (ct + 1 < C::NCT) {
          const int cn = ct + 1 < C::NCT ? ct + 1 : ct;
          first = make_float2(__shfl(ycur[cn].x, 0, 64), __shfl(ycur[cn].y, 0, 64));
        }
        ynx[ct] = o_lane == 63u ? first : make_float2(nx, ny);
      }
      // two outputs a lane and step on packed FMAs (disc_angle2): C tiles (0, 1), (2, 3), ...
#pragma unroll
      for (int ct = 0; ct < C::NCT; ct += 2) {
        const int cb = ct + 1 < C::NCT ? ct + 1 : ct;
        const float2 za = disc_product(ycur[ct], ynx[ct]), zb = disc_product(ycur[cb], ynx[cb]);
#if defined(GSDR_I8_FM_PROBE) && GSDR_I8_FM_PROBE == 2
        {  // timing probe (probe builds only): the exchange and the products, no angle
          const uint32_t r0 = (w * C::NCT + (uint32_t)ct) * 64u + o_lane, r1 = (w * C::NCT + (uint32_t)cb) * 64u + o_lane;
          if (r0 >= out_lo && r0 < out_hi) out_t[r0] = za.x + za.y;
          if (cb != ct && r1 >= out_lo && r1 < out_hi) out_t[r1] = zb.x + zb.y;
          continue;
        }
#endif
        const gsdr_f32x2 a2 = disc_angle2(za, zb) + gsdr_f32x2{dphi, dphi};
        float ang[2] = {a2.x, a2.y};
        const float2 zz[2] = {za, zb};
        const float2 y0s[2] = {ycur[ct], ycur[cb]}, y1s[2] = {ynx[ct], ynx[cb]};
        const uint32_t rr[2] = {(w * C::NCT + (uint32_t)ct) * 64u + o_lane, (w * C::NCT + (uint32_t)cb) * 64u + o_lane};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ang[h] = ang[h] > 3.14159274f ? ang[h] - 6.28318548f : (ang[h] <= -3.14159274f ? ang[h] + 6.28318548f : ang[h]);
          if (zz[h].x == 0.0f && zz[h].y == 0.0f) {
            // arg(y[k+1] conj y[k]) = arg(z') + dphi needs z' != 0. An exactly zero product (a zero window
            // beside a nonzero one, silence, zero taps) gives the reference's atan2f(+-0, +-0) (fm.cu:66-68),
            // whose value (0 or +-pi) follows the signs of the ROTATED outputs y = e^{j phi(4k)} y': rotate
            // the nonzero ones; a zero window's y is +0 + j0 in the reference's ascending sum from +0
            const float2 y0 = y0s[h], y1 = y1s[h];
            const uint32_t n = p.nco_n0 + 4u * (uint32_t)(k_t + rr[h]);
            const float2 u0 = (y0.x == 0.0f && y0.y == 0.0f) ? make_float2(0.0f, 0.0f)
                                                             : cmul(y0, nco_direct(n * p.nco_inc));
            const float2 u1 = (y1.x == 0.0f && y1.y == 0.0f) ? make_float2(0.0f, 0.0f)
                                                             : cmul(y1, nco_direct((n + 4u) * p.nco_inc));
            const float2 zr = disc_product(u0, u1);
            ang[h] = atan2f(zr.y, zr.x);
          }
          if ((h == 0 || cb != ct) && rr[h] >= out_lo && rr[h] < out_hi) out_t[rr[h]] = p.fm_gain * ang[h];
        }
      }
    } else {
      __syncthreads();  // every wave is done reading the tile's planes
    }
  }
}

}  // namespace gsdr
