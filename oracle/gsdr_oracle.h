/*
 * gsdr CPU oracle -- TEST INFRASTRUCTURE ONLY.
 *
 * A scalar C restatement of the reference's hot-path semantics (kernrj/gsdr, read as text; the
 * reference itself cannot be built here: it needs nvcc/CUDA and a CMake-generated gsdr_export.h).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker or the timed CPU baseline -- never as a product path.
 *
 * Parity pinning: see oracle/README.md and DESIGN.md section "Oracle". The oracle is checked against
 * (a) the known-answer tests of the reference's gtest suite, re-encoded with the kernel's actual
 * semantics, and (b) an independent float64 numpy restatement (tests/golden/). No executable output
 * of the reference exists, so transcendental results (atan2f, hypotf, sincos) are pinned by tolerance.
 *
 * Complex arrays are interleaved float pairs (re, im), the layout of cuComplex / hipFloatComplex.
 * Range arguments [k0, k1) select which outputs to compute, so full-size inputs can be spot-checked.
 */
#ifndef GSDR_ORACLE_H_
#define GSDR_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A.1 FIR, reference src/fir.cu:26-71: y[k] = sum_{i<T} x[k*D + i] * t[i], i ascending, fmaf per
 * component, accumulator from zero (cuComplexOperatorOverloads.cuh:25-72). */
void oracle_fir_ff(size_t D, const float* t, size_t T, const float* x, float* y, size_t k0, size_t k1);
void oracle_fir_fc(size_t D, const float* t, size_t T, const float* x, float* y, size_t k0, size_t k1);
void oracle_fir_cc(size_t D, const float* t, size_t T, const float* x, float* y, size_t k0, size_t k1);
void oracle_fir_cf(size_t D, const float* t, size_t T, const float* x, float* y, size_t k0, size_t k1);

/* Multi-threaded FC FIR over [0, N) (static split by output range) -- the CPU baseline. */
void oracle_fir_fc_mt(size_t D, const float* t, size_t T, const float* x, float* y, size_t N, int nthreads);

/* Condition bound S_k = sum_i |t_i| * |x_{kD+i}| (complex |.|), for the normwise parity metric. */
void oracle_fir_bound_fc(size_t D, const float* t, size_t T, const float* x, float* s, size_t k0, size_t k1);

/* A.3 NCO: inc = llround(fmod((tune - chan) / fs * 2^32, 2^32)) mod 2^32 (fm.cu:204, am.cu:68). */
uint32_t oracle_nco_inc(float fs, float tune, float chan);
/* z[n] = x[n] * exp(+j 2 pi P / 2^32), P = (uint32)((n0 + n) * inc), for n in [i0, i1). */
void oracle_nco_mix(const float* x, float* z, uint64_t n0, uint32_t inc, size_t i0, size_t i1);

/* A.4 FM chain (fm.cu:21-69, 181-218, re-specified): outputs m in [m0, m1), input N*D + T samples. */
void oracle_fm_demod(float fs, float tune, float chan, float dev, uint32_t D, uint64_t n0, const float* taps,
                     size_t T, const float* x, float* out, size_t m0, size_t m1);
/* A.4 AM chain (am.cu:21-81): outputs m in [m0, m1). */
void oracle_am_demod(float fs, float tune, float chan, uint32_t D, uint64_t n0, const float* taps, size_t T,
                     const float* x, float* out, size_t m0, size_t m1);
/* FIR stage of the chains (NCO-mixed, filtered), y[m] for m in [m0, m1): exposes the pre-discriminator
 * signal for the normwise FIR check. */
void oracle_chain_fir(float fs, float tune, float chan, uint32_t D, uint64_t n0, const float* taps, size_t T,
                      const float* x, float* y, size_t m0, size_t m1);

/* A.2 quad demods (quad_demod.cu:23-54) and magnitude (magnitude.cu:20-28). */
void oracle_quad_fm(const float* x, float* out, float gain, size_t n);
void oracle_quad_am(const float* x, float* out, size_t n);
void oracle_magnitude(const float* x, float* out, size_t n);

/* A.5 QPSK (qpsk.cu:108-146, 221-268). demod rewrites every byte holding one of the n symbols and
 * preserves the unused high bit pairs of a final partial byte. */
void oracle_qpsk_mod(const uint8_t* bits, float* out, uint32_t n, float a);
void oracle_qpsk_demod(const float* in, uint8_t* bits, uint32_t n);

/* A.6 QPSK256 (qpsk256.cu:29-71, 74-101, 154-195). table: 256 interleaved points. */
void oracle_qpsk256_table(uint32_t type, float amplitude, float* table);
void oracle_qpsk256_mod(const float* table, const uint8_t* in, float* out, uint32_t n);
/* bit-exact contract: first index of min fl(fl(dx*dx) + fl(dy*dy)), strict <, init +inf */
void oracle_qpsk256_demod(const float* table, const float* in, uint8_t* out, uint32_t n);
/* the reference's literal rule with hypotf in place of cuCabsf (non-gating cross-check) */
void oracle_qpsk256_demod_hypot(const float* table, const float* in, uint8_t* out, uint32_t n);

#ifdef __cplusplus
}
#endif


/* Element-wise maps: reference src/add_const.cu:20-42, multiply.cu:20-27,
 * magnitude.cu:30-36, trig.cu:20-75, conversion.cu:20-35, with the operator semantics of
 * src/cuComplexOperatorOverloads.cuh:25-56. Complex arrays are interleaved float pairs.
 * add_const variant: 0 FF, 1 CC, 2 CF (complex + real: real part only), 3 FC (real + complex).
 * multiply variant: 0 CC (cuCmulf), 1 FF, 2 CF. */
void oracle_add_const(int variant, const float* x, float cr, float ci, float* out, size_t n);
void oracle_multiply(int variant, const float* a, const float* b, float* out, size_t n);
void oracle_add_to_magnitude(const float* x, float c, float* out, size_t n);
void oracle_abs(const float* x, float* out, size_t n);
void oracle_int8_to_float(const int8_t* x, float* out, size_t n);
void oracle_cosine(int complex_out, float phi_begin, float phi_end, float* out, size_t n);


/* IIR (re-specified, include/gsdr/iir.h): y[n] = sum_{i<K} b[i] x[n-i] -
 * sum_{1<=i<K} a[i] y[n-i], evaluated sequentially in double. xh / yh (K-1 entries, may be NULL) hold
 * x[-1-i] / y[-1-i] on entry and the last K-1 inputs / outputs on return. cplx: samples are
 * interleaved complex floats (two independent recursions). */
void oracle_iir(int cplx, const float* b, const float* a, size_t K, float* xh, float* yh, const float* x, float* y,
                size_t n);
/* The same recursion as a plain sequential float32 loop (acc = b0 x; fmaf(b_i, x_{n-i}, acc);
 * fmaf(-a_i, y_{n-i}, acc)): the error any sequential fp32 implementation makes, used to scale the
 * GPU test bar to the filter's conditioning. */
void oracle_iir_f32(int cplx, const float* b, const float* a, size_t K, const float* xh, const float* yh,
                    const float* x, float* y, size_t n);

/* QPSK256 demodulation with the reference's literal rule (qpsk256.cu:171-181): first index of the
 * minimum cuCabsf(received - point), strict <. cuCabsf restated from CUDA's public cuComplex.h
 * (v = max(|a|, |b|), w = min, t = w / v, |z| = v * sqrtf(1 + t*t), v + w when v == 0 or either is
 * beyond FLT_MAX), with `1 + t*t` contracted to fmaf(t, t, 1) as nvcc does by default (-fmad=true). */
float oracle_cuCabsf(float re, float im);
void oracle_qpsk256_demod_cuabs(const float* table, const float* in, uint8_t* out, uint32_t n);

/* Config 5's channel (gsdrxQpsk256ModulateAwgn, include/gsdr/gsdr_ext.h): counter-based AWGN that the
 * host reproduces bit for bit. Philox4x32-10 (Salmon et al., SC'11) keyed by the 64-bit seed, counter
 * = (block lo, hi, 0, 0) with block = absolute symbol index / 3; slot k % 3 takes 21 bits a component
 * from the block's words w0..w3 (slot 0: w0 >> 11, w1 >> 11; slot 1: w2 >> 11, w3 >> 11; slot 2:
 * (w0 & 0x7ff) << 10 | (w1 & 0x7ff) >> 1, (w2 & 0x7ff) << 10 | (w3 & 0x7ff) >> 1). A component's bits
 * give a sign and the tail probability v = (2a + 1) 2^-21; |g| is the half-normal quantile -Phi^-1(v/2)
 * by linear interpolation in a 21 x 32 table (gsdr_amd/csrc/awgn_table.inc; one fmaf), so the device
 * and the host round identically. A component with a < 32 (|g| > 4.17) takes 18 more bits from the
 * extension block (counter (block lo, hi, 1, 0)) and the 24 x 32 tail table (awgn_tail_table.inc), so the
 * tails reach 7.0 instead of 5.035. Output = fl(table[s] + fl(sigma g)) per component (no FMA). */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float oracle_awgn_normal21(uint32_t r);
/* tail extension: a = r & 0xfffff < 32 with 18 more bits e (gsdr_amd/csrc/awgn.hpp) */
float oracle_awgn_tail_normal(uint32_t r, uint32_t e);
void oracle_awgn_normals(uint64_t seed, uint64_t symbol_index, float* g0, float* g1);
void oracle_qpsk256_mod_awgn(const float* table, const uint8_t* in, float* out, uint32_t n, float sigma,
                             uint64_t seed, uint64_t first_symbol);

/* Multi-threaded forms for the timed CPU baseline (static split of the output range over nthreads
 * pthreads); each thread runs the scalar restatement above on its range. rule: 0 squared distance,
 * 1 cuCabsf. */
void oracle_fir_ff_mt(size_t D, const float* t, size_t T, const float* x, float* y, size_t N, int nthreads);
void oracle_fm_demod_mt(float fs, float tune, float chan, float dev, uint32_t D, uint64_t n0, const float* taps,
                        size_t T, const float* x, float* out, size_t m0, size_t m1, int nthreads);
void oracle_qpsk256_demod_mt(int rule, const float* table, const float* in, uint8_t* out, uint32_t n, int nthreads);
void oracle_qpsk256_mod_awgn_mt(const float* table, const uint8_t* in, float* out, uint32_t n, float sigma,
                                uint64_t seed, uint64_t first_symbol, int nthreads);

#endif /* GSDR_ORACLE_H_ */
