// gsdr-mi355x: counter-based additive white Gaussian noise for the config-5 channel
// (gsdrxQpsk256ModulateAwgn, include/gsdr/gsdr_ext.h).
//
// The noise of absolute symbol k is a pure function of (seed, k), so the host can regenerate the exact
// noisy buffer a launch produced (tests compare the full 2^24-symbol round trip against the CPU
// oracle) and any split of a buffer into launches yields the same samples:
//   * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11): key = seed, counter = (k / 3 lo, hi, 0, 0);
//     one 128-bit block (w0..w3) serves three symbols (slot k % 3), 21 bits per component:
//     slot 0: (w0 >> 11, w1 >> 11); slot 1: (w2 >> 11, w3 >> 11);
//     slot 2: ((w0 & 0x7ff) << 10 | (w1 & 0x7ff) >> 1, (w2 & 0x7ff) << 10 | (w3 & 0x7ff) >> 1).
//   * A component's 21 bits r: sign = bit 20, a = the low 20 bits. The tail probability is
//     v = (2a + 1) 2^-21 in (0, 1) and |g| = h(v) = -Phi^-1(v / 2), the half-normal quantile, read from
//     a 21 x 32 table (awgn_table.inc, tools/make_awgn_table.py) by inverse-CDF interpolation: the float
//     (float)(2a + 1) (exact) gives index = (bits >> 18) - 127 * 32 (its exponent and top 5 mantissa bits)
//     and f = (bits & 0x3ffff) 2^-18 (exact), |g| = fmaf(S, f, R) -- within 2.5e-5 of h, unbiased (the
//     table holds S 2^-18, so the product is S' times the integer: the same bits, one multiply fewer).
//   * Tail extension (round 4): a component whose a < 32 (v < 2^-15, |g| > 4.17) takes 18 more bits e
//     from a second Philox block of the same key (counter (k / 3 lo, hi, 1, 0)): component c of the
//     block (slot s: c = 2s for the first normal, 2s + 1 for the second) uses x0 >> 14, x1 >> 14,
//     x2 >> 14, x3 >> 14, (x0 & 0x3fff) << 4 | (x2 & 0xf), (x1 & 0x3fff) << 4 | (x3 & 0xf) for c = 0..5.
//     Then x' = 2 (a 2^18 + e) + 1 < 2^24 (exact in float), v' = x' 2^-39, and |g| is read the same way
//     from a 24 x 32 tail table (awgn_tail_table.inc): the tails reach h(2^-39) = 7.0 sigma, where a
//     single 21-bit draw cut them at h(2^-21) = 5.035 (P(|g| > 5.035) = 4.8e-7 per axis had been lost).
//     ~3e-5 of the components take it; the second Philox block is evaluated only then.
// Every operation is exact or one correctly rounded IEEE fmaf, so the host restatement
// (oracle/gsdr_oracle.c, which reads the same table) reproduces every bit. Round 2's Box-Muller with
// correctly rounded sqrt and polynomial ln / sin / cos cost ~320 of the ~450 cycles per symbol and wave.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsdr {

constexpr int kAwgnTableSize = 21 * 32;

// (R, S) pairs; copied into LDS by the kernel that uses them (awgn_fetch_table, awgn_store_table).
__constant__ float2 c_awgn_table[kAwgnTableSize] = {
#define GSDR_AWGN_ENTRY(r, s) {r, s},
#include "awgn_table.inc"
#undef GSDR_AWGN_ENTRY
};

constexpr int kAwgnTailSize = 24 * 32;

// (R, S) pairs of the tail extension: read straight from this array (rarely: ~3e-5 of the components).
__constant__ float2 c_awgn_tail[kAwgnTailSize] = {
#define GSDR_AWGN_ENTRY(r, s) {r, s},
#include "awgn_tail_table.inc"
#undef GSDR_AWGN_ENTRY
};

// a ^ b ^ k in one v_bitop3_b32 (gfx950; the compiler emits two v_xor_b32), k wave-uniform (the key)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}

// GSDR_PHILOX_ROUNDS: a timing probe (tools/awgn_time.py builds): any other round count changes every
// noise sample, so it is refused outside the probe builds (-DGSDR_TUNING_PROBES).
#ifndef GSDR_PHILOX_ROUNDS
#define GSDR_PHILOX_ROUNDS 10
#endif
#if GSDR_PHILOX_ROUNDS != 10 && !defined(GSDR_TUNING_PROBES)
#error "GSDR_PHILOX_ROUNDS != 10 breaks the channel's bit parity with the oracle: probe builds only"
#endif

__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t (&w)[4]) {
#pragma unroll
  for (int r = 0; r < GSDR_PHILOX_ROUNDS; ++r) {
    // one 32 x 32 -> 64-bit product per multiplier (v_mad_u64_u32) instead of separate mul_lo / mul_hi:
    // both are quarter-rate, and these 40 products per three symbols bound the kernel
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    c0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    c1 = (uint32_t)p1;
    c2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  w[0] = c0;
  w[1] = c1;
  w[2] = c2;
  w[3] = c3;
}

// The table in LDS as two float planes R and S (all threads of the workgroup; the caller's barrier
// publishes it): a normal's two loads then land in any registers, where (R, S) pairs had to be shuffled
// apart for the packed fma of a symbol's two normals (three moves a symbol).
// (GSDR_AWGN_PAIRS, a probe-build switch: the round-3 (R, S) pairs, one ds_read_b64 a normal.)
#if defined(GSDR_AWGN_PAIRS) && !defined(GSDR_TUNING_PROBES)
#error "GSDR_AWGN_PAIRS is a timing probe: probe builds only"
#endif
constexpr int kAwgnLdsSize = 3 * 256;  // the table padded to three entries a thread (awgn_store_table)
struct AwgnLds {
#ifdef GSDR_AWGN_PAIRS
  float2 rs[kAwgnLdsSize];
#else
  float r[kAwgnLdsSize], s[kAwgnLdsSize];
#endif
};
// Entries below kAwgnTailIndex serve only tail components (a < 32 <=> x = 2 a + 1 < 64 <=> index < 6 * 32),
// whose values the tail extension replaces: their R is NaN in LDS, so a tail component turns its symbol's
// noisy output into NaN and one NaN test over a lane's outputs finds it (awgn_has_tail).
constexpr uint32_t kAwgnTailIndex = 6 * 32;
// The table's copy into LDS in two halves, so the caller can issue other loads between them: awgn_fetch_table
// loads a 256-thread workgroup's entries (thread t: t, t + 256, t + 512) into registers, awgn_store_table writes
// them (entries below kAwgnTailIndex with R = NaN). The caller's barrier publishes the table.
struct AwgnRegs {
  float2 e[3];
};
__device__ __forceinline__ AwgnRegs awgn_fetch_table() {
  static_assert(kAwgnTableSize <= 3 * 256 && kAwgnTableSize > 2 * 256, "three entries a thread of 256");
  AwgnRegs r;
  const uint32_t t = threadIdx.x;
  r.e[0] = c_awgn_table[t];
  r.e[1] = c_awgn_table[t + 256];
  r.e[2] = c_awgn_table[t + 512 < (uint32_t)kAwgnTableSize ? t + 512 : t];
  return r;
}
__device__ __forceinline__ void awgn_store_table(AwgnLds& tab, const AwgnRegs& r) {
  static_assert(kAwgnLdsSize == 3 * 256, "three entries a thread");
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {  // (entries past the table land in the padding: no branch around the loads)
    const uint32_t i = threadIdx.x + 256u * k;
    float2 e = r.e[k];
    if (i < kAwgnTailIndex) e.x = __builtin_nanf("");
#ifdef GSDR_AWGN_PAIRS
    tab.rs[i] = e;
#else
    tab.r[i] = e.x;
    tab.s[i] = e.y;
#endif
  }
}
__device__ __forceinline__ float awgn_fma(const AwgnLds& t, uint32_t i, float f) {
#if defined(GSDR_TUNING_PROBES) && defined(GSDR_AWGN_PROBE_NOGATHER)
  i = 256u + (threadIdx.x & 63u) + (i & 0x100u);  // timing probe only: conflict-free, no tail entries, wrong noise
#endif
#ifdef GSDR_AWGN_PAIRS
  const float2 e = t.rs[i];
  return fmaf(e.y, f, e.x);
#else
  return fmaf(t.s[i], f, t.r[i]);
#endif
}

// m with its sign flipped where bit 31 of `sgn` is set: one v_bitop3_b32 (m ^ (sgn & 0x80000000))
__device__ __forceinline__ float awgn_sign(float m, uint32_t sgn) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(r) : "v"(__float_as_uint(m)), "v"(sgn), "s"(0x80000000u));
  return __uint_as_float(r);
}

// One standard normal from a 20-bit a and a sign (bit 31 of sgn): x = 2 a + 1.
__device__ __forceinline__ float awgn_normal_a(const AwgnLds& t, uint32_t a, uint32_t sgn) {
  const uint32_t x = (a << 1) | 1u;
  const uint32_t b = __float_as_uint((float)x);
  const uint32_t i = __builtin_amdgcn_ubfe(b, 18, 14) - 127u * 32u;
  const float m = awgn_fma(t, i, (float)(b & 0x3ffffu));
  return awgn_sign(m, sgn);
}

// One standard normal from 21 random bits (the low 21 of r).
__device__ __forceinline__ float awgn_normal(const AwgnLds& t, uint32_t r) {
  const uint32_t x = ((r << 1) & 0x1ffffeu) | 1u;
  const uint32_t b = __float_as_uint((float)x);
  // index (b >> 18) - 127 * 32: the exponent and the top 5 mantissa bits
  const uint32_t i = __builtin_amdgcn_ubfe(b, 18, 14) - 127u * 32u;
  // S is stored pre-scaled by 2^-18 (exact), so S f = S' (b & 0x3ffff) with the integer converted exactly
  const float m = awgn_fma(t, i, (float)(b & 0x3ffffu));
  return awgn_sign(m, r << 11);
}

// The tail normal of a component with a = r & 0xfffff < 32 and its 18 extension bits e.
__device__ __forceinline__ float awgn_tail_normal(uint32_t r, uint32_t e) {
  const uint32_t x = ((((r & 0x1fu) << 18) | e) << 1) | 1u;  // < 2^24: exact in float
  const uint32_t b = __float_as_uint((float)x);
  const float2 rs = c_awgn_tail[(b >> 18) - 127u * 32u];
  const float m = fmaf(rs.y, (float)(b & 0x3ffffu), rs.x);
  return awgn_sign(m, r << 11);
}

__device__ __forceinline__ bool awgn_in_tail(uint32_t r) { return (r & 0xfffe0u) == 0u; }

// The Philox block holding absolute symbols 3 blk .. 3 blk + 2.
__device__ __forceinline__ void awgn_block_words(uint64_t seed, uint64_t blk, uint32_t (&w)[4]) {
  philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32), w);
}

// Both normals of slot `slot` when at least one of them is in the tail: the extension block, then the
// tail-table value for each tail component (out of line: ~2e-4 of the lanes' blocks take it).
__device__ __forceinline__ float2 awgn_slot_tail(uint64_t seed, uint64_t blk, int slot, uint32_t r0, uint32_t r1,
                                             float2 g) {
  uint32_t x[4];
  philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), 1u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32), x);
  uint32_t e0, e1;
  if (slot == 0) {
    e0 = x[0] >> 14;
    e1 = x[1] >> 14;
  } else if (slot == 1) {
    e0 = x[2] >> 14;
    e1 = x[3] >> 14;
  } else {
    e0 = ((x[0] & 0x3fffu) << 4) | (x[2] & 0xfu);
    e1 = ((x[1] & 0x3fffu) << 4) | (x[3] & 0xfu);
  }
  if (awgn_in_tail(r0)) g.x = awgn_tail_normal(r0, e0);
  if (awgn_in_tail(r1)) g.y = awgn_tail_normal(r1, e1);
  return g;
}

// The 21-bit components of slot `slot`.
__device__ __forceinline__ void awgn_slot_bits(const uint32_t (&w)[4], int slot, uint32_t& r0, uint32_t& r1) {
  if (slot == 0) {
    r0 = w[0] >> 11;
    r1 = w[1] >> 11;
  } else if (slot == 1) {
    r0 = w[2] >> 11;
    r1 = w[3] >> 11;
  } else {
    r0 = ((w[0] & 0x7ffu) << 10) | ((w[1] & 0x7ffu) >> 1);
    r1 = ((w[2] & 0x7ffu) << 10) | ((w[3] & 0x7ffu) >> 1);
  }
}

// The normal pair of slot `slot` from the main table only: exact unless a component is in the tail, where it
// is NaN (awgn_has_tail tests a lane's outputs once, so the common path has no branch a slot).
__device__ __forceinline__ float2 awgn_slot_main(const AwgnLds& tab, const uint32_t (&w)[4], int slot) {
  if (slot < 2) {  // a = bits 11..30 of the word, the sign its bit 31
    const uint32_t wa = w[2 * slot], wb = w[2 * slot + 1];
    return make_float2(awgn_normal_a(tab, __builtin_amdgcn_ubfe(wa, 11, 20), wa),
                       awgn_normal_a(tab, __builtin_amdgcn_ubfe(wb, 11, 20), wb));
  }
  uint32_t r0, r1;
  awgn_slot_bits(w, 2, r0, r1);
  return make_float2(awgn_normal(tab, r0), awgn_normal(tab, r1));
}

// Whether outputs y[0 .. K) computed from awgn_slot_main normals may hold a tail component: a NaN in their
// sum (the tail entries' NaN R, kAwgnTailIndex). Also true for outputs that are NaN or overflow for other
// reasons (a non-finite sigma); the caller's exact pass (awgn_slot_fix) then just reproduces them.
template <int K>
__device__ __forceinline__ bool awgn_has_tail(const float2 (&y)[K]) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  f2v c = {y[0].x, y[0].y};
#pragma unroll
  for (int j = 1; j < K; ++j) c += f2v{y[j].x, y[j].y};
  return __builtin_isnan(c.x + c.y);
}

// The normal pair of slot `slot` (0..2, compile-time after unrolling) of block `blk` (words w).
__device__ __forceinline__ float2 awgn_slot(const AwgnLds& tab, const uint32_t (&w)[4], int slot, uint64_t seed,
                                            uint64_t blk) {
  uint32_t r0, r1;
  if (slot == 0) {
    r0 = w[0] >> 11;
    r1 = w[1] >> 11;
  } else if (slot == 1) {
    r0 = w[2] >> 11;
    r1 = w[3] >> 11;
  } else {
    r0 = ((w[0] & 0x7ffu) << 10) | ((w[1] & 0x7ffu) >> 1);
    r1 = ((w[2] & 0x7ffu) << 10) | ((w[3] & 0x7ffu) >> 1);
  }
  float2 g;
  if (slot < 2) {  // a = bits 11..30 of the word, the sign its bit 31
    const uint32_t wa = w[2 * slot], wb = w[2 * slot + 1];
    g = make_float2(awgn_normal_a(tab, __builtin_amdgcn_ubfe(wa, 11, 20), wa),
                    awgn_normal_a(tab, __builtin_amdgcn_ubfe(wb, 11, 20), wb));
  } else {
    g = make_float2(awgn_normal(tab, r0), awgn_normal(tab, r1));
  }
  if (__builtin_expect(awgn_in_tail(r0) || awgn_in_tail(r1), 0)) return awgn_slot_tail(seed, blk, slot, r0, r1, g);
  return g;
}

}  // namespace gsdr
