// gsdr-mi355x: counter-based additive white Gaussian noise for the config-5 channel
// (gsdrxQpsk256ModulateAwgn, include/gsdr/gsdr_ext.h).
//
// The noise of absolute symbol k is a pure function of (seed, k), so the host can regenerate the exact
// noisy buffer a launch produced (tests compare the full 2^24-symbol round trip against the CPU
// oracle) and any split of a buffer into launches yields the same samples:
//   * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11): key = seed, counter = (k >> 1 lo, hi, 0, 0);
//     words (0, 1) belong to the even symbol of the pair, (2, 3) to the odd one.
//   * u1 = ((w0 >> 9) + 0.5) 2^-23 in (0, 1), u2 = (w1 >> 8) 2^-24 in [0, 1), both exact in float.
//   * Box-Muller: (g0, g1) = sqrt(-2 ln u1) (cos, sin)(2 pi u2), with ln, cos and sin evaluated by
//     fixed sequences of correctly rounded IEEE operations (+, -, *, /, sqrt, fmaf) --
//     no hardware transcendental, no libm -- so the host restatement (oracle/gsdr_oracle.c) rounds
//     identically. ln: u = m 2^e, m in [sqrt(1/2), sqrt(2)), ln m = 2 s P(s^2), s = (m - 1)/(m + 1);
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
  const float s = (m - 1.0f) / (m + 1.0f);  // correctly rounded: HIP's default f32 division
  const float z = s * s;
  float p = 0.09090909361839294f;
  p = fmaf(p, z, 0.1111111119389534f);
  p = fmaf(p, z, 0.1428571492433548f);
  p = fmaf(p, z, 0.20000000298023224f);
  p = fmaf(p, z, 0.3333333432674408f);
  p = fmaf(p, z, 1.0f);
  const float lnm = (2.0f * s) * p;
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

__device__ __forceinline__ float2 awgn_box_muller(uint32_t w0, uint32_t w1) {
  const float u1 = ((float)(w0 >> 9) + 0.5f) * 1.1920928955078125e-07f;  // 2^-23
  const float u2 = (float)(w1 >> 8) * 5.9604644775390625e-08f;           // 2^-24
  // __builtin_sqrtf is the correctly rounded IEEE square root (HIP's default); __fsqrt_rn is NOT: in
  // this toolchain it maps to __ocml_native_sqrt_f32 (the ~1-ulp hardware v_sqrt_f32).
  const float r = __builtin_sqrtf(-2.0f * awgn_log(u1));
  const float2 cs = awgn_cos_sin_turns(u2);
  return make_float2(r * cs.x, r * cs.y);
}

// The Philox words of the pair holding absolute symbol k.
__device__ __forceinline__ void awgn_pair_words(uint64_t seed, uint64_t pair, uint32_t (&w)[4]) {
  philox4x32_10((uint32_t)pair, (uint32_t)(pair >> 32), 0u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32), w);
}

}  // namespace gsdr
