// gsdr-mi355x: counter-based additive white Gaussian noise for the config-5 channel
// (gsdrxQpsk256ModulateAwgn, include/gsdr/gsdr_ext.h).
//
// The noise of absolute symbol k is a pure function of (seed, k), so the host can regenerate the exact
// noisy buffer a launch produced (tests compare the full 2^24-symbol round trip against the CPU
// oracle) and any split of a buffer into launches yields the same samples:
//   * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11): key = seed, counter = (k / 3 lo, hi, 0, 0);
//     one 128-bit block serves three symbols (slot k % 3), 39 bits each (awgn_slot_bits):
//     slot 0: a = w0 >> 9, b = w3 & 0xffff; slot 1: a = w1 >> 9, b = w3 >> 16;
//     slot 2: a = w2 >> 9, b = (w0 & 0x1ff) << 7 | (w1 & 0x7f).
//   * u1 = (a + 0.5) 2^-23 in (0, 1), u2 = b 2^-16 in [0, 1), both exact in float (u2 quantises the
//     angle to 2^-16 turn; drawing 47 bits a symbol instead cost 50 % more Philox blocks, which bound
//     the kernel).
//   * Box-Muller: (g0, g1) = sqrt(-2 ln u1) (cos, sin)(2 pi u2), with ln, cos and sin evaluated by
//     fixed sequences of correctly rounded IEEE operations (+, -, *, sqrt, fmaf) -- no hardware
//     transcendental, no libm -- so the host restatement (oracle/gsdr_oracle.c) rounds
//     identically. ln: u = m 2^e, m in [sqrt(1/2), sqrt(2)), ln m = t q(t), t = m - 1 (degree-8 q);
//     sin/cos: quadrant q = floor(4 u2), f = 4 u2 - q, odd/even Taylor polynomials of f pi / 2 (errors
//     below 2e-7). Tails are cut at sqrt(-2 ln 2^-24) = 5.8 sigma.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsdr {

__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t (&w)[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32 x 32 -> 64-bit product per multiplier (v_mad_u64_u32) instead of separate mul_lo / mul_hi:
    // both are quarter-rate, and these 40 products per pair of symbols bound the kernel
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    c1 = (uint32_t)p1;
    c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  w[0] = c0;
  w[1] = c1;
  w[2] = c2;
  w[3] = c3;
}

__device__ __forceinline__ float awgn_log(float u) {
  const uint32_t b = __float_as_uint(u);
  int e = (int)((b >> 23) & 0xffu) - 127;
  float m = __uint_as_float((b & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421354f) {
    m = m * 0.5f;
    e += 1;
  }
  /* ln m = t q(t), t = m - 1 in [sqrt(1/2) - 1, sqrt(2) - 1]: degree-8 q fitted on Chebyshev nodes,
     max abs error 4.8e-8 in float32 Horner evaluation (no division) */
  const float t = m - 1.0f;
  float p = 0.08743945509195328f;
  p = fmaf(p, t, -0.14377330243587494f);
  p = fmaf(p, t, 0.14949095249176025f);
  p = fmaf(p, t, -0.16560696065425873f);
  p = fmaf(p, t, 0.19956977665424347f);
  p = fmaf(p, t, -0.2500215470790863f);
  p = fmaf(p, t, 0.3333418369293213f);
  p = fmaf(p, t, -0.49999988079071045f);
  p = fmaf(p, t, 1.0f);
  const float lnm = p * t;
  const float fe = (float)e;
  return fmaf(fe, 0.693145751953125f, fmaf(fe, 1.428606765330187e-06f, lnm));
}

__device__ __forceinline__ float2 awgn_cos_sin_turns(float u) {
  const float u4 = u * 4.0f;
  const int q = (int)u4;
  const float f = u4 - (float)q;
  const float z = f * f;
  float sp = 5.6921727775716136e-08f;
  sp = fmaf(sp, z, -3.598843250074424e-06f);
  sp = fmaf(sp, z, 0.00016044118092395365f);
  sp = fmaf(sp, z, -0.004681753925979137f);
  sp = fmaf(sp, z, 0.07969262450933456f);
  sp = fmaf(sp, z, -0.6459640860557556f);
  sp = fmaf(sp, z, 1.5707963705062866f);
  const float sn = sp * f;
  float cp = -6.386603246255618e-09f;
  cp = fmaf(cp, z, 4.710874748070637e-07f);
  cp = fmaf(cp, z, -2.520204179745633e-05f);
  cp = fmaf(cp, z, 0.0009192602592520416f);
  cp = fmaf(cp, z, -0.020863480865955353f);
  cp = fmaf(cp, z, 0.25366950035095215f);
  cp = fmaf(cp, z, -1.2337005138397217f);
  const float cs = fmaf(cp, z, 1.0f);
  switch (q & 3) {
    case 0: return make_float2(cs, sn);
    case 1: return make_float2(-sn, cs);
    case 2: return make_float2(-cs, -sn);
    default: return make_float2(sn, -cs);
  }
}

// a: 23 bits for u1, b: 16 bits for u2
__device__ __forceinline__ float2 awgn_box_muller(uint32_t a, uint32_t b) {
  const float u1 = ((float)a + 0.5f) * 1.1920928955078125e-07f;  // 2^-23
  const float u2 = (float)b * 1.52587890625e-05f;                 // 2^-16
  // __builtin_sqrtf is the correctly rounded IEEE square root (HIP's default); __fsqrt_rn is NOT: in
  // this toolchain it maps to __ocml_native_sqrt_f32 (the ~1-ulp hardware v_sqrt_f32).
  const float r = __builtin_sqrtf(-2.0f * awgn_log(u1));
  const float2 cs = awgn_cos_sin_turns(u2);
  return make_float2(r * cs.x, r * cs.y);
}

// The Philox block holding absolute symbols 3 blk .. 3 blk + 2.
__device__ __forceinline__ void awgn_block_words(uint64_t seed, uint64_t blk, uint32_t (&w)[4]) {
  philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32), w);
}

// The normal pair of slot `slot` (0..2, compile-time after unrolling) of a block.
__device__ __forceinline__ float2 awgn_slot(const uint32_t (&w)[4], int slot) {
  if (slot == 0) return awgn_box_muller(w[0] >> 9, w[3] & 0xffffu);
  if (slot == 1) return awgn_box_muller(w[1] >> 9, w[3] >> 16);
  return awgn_box_muller(w[2] >> 9, ((w[0] & 0x1ffu) << 7) | (w[1] & 0x7fu));
}

}  // namespace gsdr
