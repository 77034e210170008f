// gsdr-mi355x: int8 I/Q FIR on the matrix cores (gsdrxFirFCInt8).
//
// The int8 front end's samples are small integers (|v| <= 127 after gsdrInt8ToNormFloat's clamp), so
// they are EXACT in fp16, and the FIR becomes an f16 matrix product with fp32 accumulation whose only
// rounding is the accumulation itself:
//   * taps: scaled by 2^sc (exact) so that max|t| lies in [2^13, 2^14), then split t = hi + lo into two
//     fp16 parts (|t - hi - lo| <= 2^-22 |t|; tiny taps lose only absolute precision far below the
//     normwise bar); each product v * hi and v * lo is exact in fp32;
//   * y[k] = (sum_i t[i] v[kD + i]) * (2^-sc / 127), the reference's per-sample v / 127 moved outside
//     the sum (fir.cu:49-71 with conversion.cu:20-35's normalisation).
// The result matches the float path within the floating-point parity bar (normwise)
// rather than bit for bit: the products are summed in the matrix core's order. Taps that are not all
// finite take an exact per-output loop instead (fir_point), so non-finite semantics stay the reference's.
//
// Matrix formulation (v_mfma_f32_16x16x32_f16: A 16x32, B 32x16, C 16x16 fp32):
//   C[m][n] = sum_kk A[m][kk] B[kk][n],  A[m][kk] = t[kk - D m] (zero outside [0, T)),
//   B[kk][n] = component (n & 1) of x[(k0 + 16 (n >> 1)) D + kk],
// so column n holds 16 consecutive outputs (block n >> 1 of the C tile's 8) of one component, and one C
// tile is 128 consecutive complex outputs. K = 15 D + T padded to 32-sample steps (6 at D = 4, T = 127).
// A is the same for every tile: each lane keeps its fragments (hi and lo, 8 fp16 per step) in registers
// for the kernel's lifetime (persistent workgroups). B comes from LDS, where the staging pass wrote the
// tile's samples as two fp16 planes (I and Q) with a 16-byte pad after every 64 samples: the 16 lanes
// that read together (one per column) then hit 16 distinct 16-byte bank groups.
#pragma once

#include "fir_engine.hpp"

namespace gsdr {

typedef _Float16 gsdr_h8 __attribute__((ext_vector_type(8)));
typedef float gsdr_f4v __attribute__((ext_vector_type(4)));
typedef uint32_t gsdr_u4v __attribute__((ext_vector_type(4)));

template <int D>
struct I8Mfma {
  static constexpr int WG = 256;
  static constexpr int NCT = 4;                     // C tiles (128 outputs) per wave and tile
  static constexpr int KT = (WG / 64) * NCT * 128;  // outputs per tile
  static constexpr int MAXNS = 8;                   // 32-sample K steps: 15 D + T <= 256
  static constexpr int MAXT = 32 * MAXNS - 15 * D;
  static constexpr int SPAN = (KT - 16) * D + 32 * MAXNS;  // samples staged per tile
  static_assert(SPAN % 8 == 0, "staging moves 8 samples a lane");
  __host__ __device__ static constexpr uint32_t addr(uint32_t idx) { return idx * 2u + (idx / 64u) * 16u; }
  // Q plane offset: = 128 (mod 256), so the Q columns' bank groups interleave the I columns'
  static constexpr uint32_t PLANE = (addr(SPAN) + 255u) / 256u * 256u + 128u;
  static constexpr uint32_t LDS_BYTES = PLANE + addr(SPAN);
};

// BPC workgroups per CU (one wave per SIMD each): the register budget is 512 / BPC VGPRs
template <int D, bool VEC, int BPC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BPC, BPC))) void k_fir_i8_mfma(FirParams p, uint32_t ns, uint32_t tiles) {
  using C = I8Mfma<D>;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS_BYTES];
  __shared__ float wmax[C::WG / 64];
  __shared__ uint32_t wbad[C::WG / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  const Iq8* __restrict__ in = reinterpret_cast<const Iq8*>(p.in);
  float2* __restrict__ out = reinterpret_cast<float2*>(p.out);
  const uint32_t T = p.T;

  // tap scale (T <= MAXT <= 256: one tap a thread), and whether every tap is finite
  const float t = tid < T ? taps[tid] : 0.0f;
  float a = fabsf(t);
  uint32_t bad = isfinite(t) ? 0u : 1u;
  for (int o = 32; o > 0; o >>= 1) {
    a = fmaxf(a, __shfl_xor(a, o, 64));
    bad |= __shfl_xor(bad, o, 64);
  }
  if (lane == 0) {
    wmax[w] = a;
    wbad[w] = bad;
  }
  __syncthreads();
  float amax = wmax[0];
  bad = wbad[0];
#pragma unroll
  for (int i = 1; i < C::WG / 64; ++i) {
    amax = fmaxf(amax, wmax[i]);
    bad |= wbad[i];
  }
  if (bad) {  // non-finite taps: the reference's ascending loop, output by output
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
      for (uint32_t r = tid; r < (uint32_t)C::KT; r += C::WG) {
        const uint64_t k = (uint64_t)tile * C::KT + r;
        if (k < p.N) out[k] = fir_point<float, Iq8, kModeFir>(p, k);
      }
    }
    return;
  }
  int e = 0;
  (void)frexpf(amax, &e);  // amax = f 2^e, f in [0.5, 1) (e = 0 for all-zero taps)
  const int sc = 14 - e;
  // scaled taps in LDS (zero past T), then this lane's A fragments: row m = lane & 15, k = 8 (lane >> 4) + j
  float* ldsT = reinterpret_cast<float*>(lds);
  ldsT[tid] = ldexpf(t, sc);
  __syncthreads();
  gsdr_h8 ahi[C::MAXNS], alo[C::MAXNS];
  {
    const int m = (int)(lane & 15u), q = (int)(lane >> 4);
#pragma unroll
    for (int s = 0; s < C::MAXNS; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 32 * s + 8 * q + j - D * m;
        const float v = i >= 0 ? ldsT[i] : 0.0f;  // i <= 255
        const _Float16 h = (_Float16)v;
        ahi[s][j] = h;
        alo[s][j] = (_Float16)(v - (float)h);  // v - h is exact in fp32
      }
    }
  }
  const float oscale = ldexpf(1.0f / 127.0f, -sc);
  __syncthreads();  // the tap table is overwritten by the first tile's samples

  const int n = (int)(lane & 15u), q = (int)(lane >> 4), c = n & 1, b = n >> 1;
  const char* bplane = lds + (c ? C::PLANE : 0u);
  for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const uint64_t k_t = (uint64_t)tile * C::KT;
    const uint64_t S0 = k_t * D;
    // stage SPAN samples as fp16 I and Q planes (16 bytes = 8 samples a lane and step), every load in
    // flight before the first conversion
    constexpr uint32_t NG = C::SPAN / 8, NGR = (NG + C::WG - 1) / C::WG;
    gsdr_u4v wv[NGR];
#pragma unroll
    for (uint32_t r = 0; r < NGR; ++r) {
      const uint32_t g = tid + r * C::WG;
      const uint64_t s = S0 + 8ull * g;
      if (g < NG) {
        if (VEC && s + 8 <= p.L) {
          wv[r] = __builtin_nontemporal_load(reinterpret_cast<const gsdr_u4v*>(in + s));
        } else {  // input end or unaligned input: per-sample loads, zero past L
          uint32_t d[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const Iq8 a = s + 2 * k < p.L ? in[s + 2 * k] : Iq8{0, 0};
            const Iq8 b2 = s + 2 * k + 1 < p.L ? in[s + 2 * k + 1] : Iq8{0, 0};
            d[k] = (uint32_t)(uint8_t)a.x | (uint32_t)(uint8_t)a.y << 8 | (uint32_t)(uint8_t)b2.x << 16 |
                   (uint32_t)(uint8_t)b2.y << 24;
          }
          wv[r] = gsdr_u4v{d[0], d[1], d[2], d[3]};
        }
      }
    }
#pragma unroll
    for (uint32_t r = 0; r < NGR; ++r) {
      const uint32_t g = tid + r * C::WG;
      if (g < NG) {
        gsdr_h8 hi_, hq_;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {  // sample 2k + u: bytes 2u (I) and 2u + 1 (Q) of dword k
            // gsdrInt8ToNormFloat clamps -128 to -1.0 = -127 / 127
            hi_[2 * k + u] = (_Float16)max((int)(wv[r][k] << (24 - 16 * u)) >> 24, -127);
            hq_[2 * k + u] = (_Float16)max((int)(wv[r][k] << (16 - 16 * u)) >> 24, -127);
          }
        }
        const uint32_t o = C::addr(8u * g);
        *reinterpret_cast<gsdr_h8*>(lds + o) = hi_;
        *reinterpret_cast<gsdr_h8*>(lds + C::PLANE + o) = hq_;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int ct = 0; ct < C::NCT; ++ct) {
      const uint32_t cbase = (w * C::NCT + (uint32_t)ct) * 128u;  // the C tile's first output in the tile
      const uint32_t idx0 = (cbase + 16u * (uint32_t)b) * D + 8u * (uint32_t)q;
      gsdr_f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < C::MAXNS; ++s) {
        if ((uint32_t)s < ns) {
          const gsdr_h8 bf = *reinterpret_cast<const gsdr_h8*>(bplane + C::addr(idx0 + 32u * (uint32_t)s));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[s], bf, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[s], bf, acc, 0, 0, 0);
        }
      }
      // lane (q, b, c) holds component c of outputs 4q .. 4q + 3 of block b; the I lane keeps rows 0-1 and
      // the Q lane rows 2-3, each taking the other component from its neighbour
      const float r0 = acc[0] * oscale, r1 = acc[1] * oscale, r2 = acc[2] * oscale, r3 = acc[3] * oscale;
      const float g0 = __shfl_xor(c ? r0 : r2, 1, 64), g1 = __shfl_xor(c ? r1 : r3, 1, 64);
      const float4 o4 = c ? make_float4(g0, r2, g1, r3) : make_float4(r0, g0, r1, g1);
      const uint64_t k = k_t + cbase + 16u * (uint32_t)b + 4u * (uint32_t)q + 2u * (uint32_t)c;
      if (k + 1 < p.N) {
        store16_nt(reinterpret_cast<float4*>(out + k), o4);
      } else if (k < p.N) {
        out[k] = make_float2(o4.x, o4.y);
      }
    }
    __syncthreads();  // every wave is done reading the tile's planes
  }
}



// ------------------------------------------------------------------------------------------------
// int8 I/Q FM / AM chains on the matrix cores (gsdrxFmDemodInt8 / gsdrxAmDemodInt8, D = 4, T <= 132).
// The NCO moves into the taps: with phi(n) the mixer phase of sample n (exact integer phase, fir_engine.hpp),
//   y[k] = sum_i t_i x[4k+i] e^{j phi(4k+i)} = e^{j phi(4k)} y'[k],  y'[k] = sum_i t'_i x[4k+i],
//   t'_i = t_i e^{j 2 pi (i inc mod 2^32) / 2^32}
// (the phase is additive mod 2^32). The AM envelope |y| = |y'|, and the FM discriminator
// arg(y[k+1] conj y[k]) = arg(y'[k+1] conj y'[k]) + 2 pi (4 inc mod 2^32) / 2^32 (wrapped), so neither
// needs the rotation: the chain is a complex-tap FIR on the raw int8 samples, exact in fp16 as in
// k_fir_i8_mfma. Complex taps on real planes: with P/Q' the real/imaginary-tap sums of the I column and
// R/S those of the Q column, y' = (P - S) + j (R + Q'); two fp16 parts per tap component -> 4 MFMAs per
// 32-sample step. FM tiles overlap by one output (stride KT - 1) and stage 8-byte granules, so every
// tile start stays aligned. Normwise parity with the float chains, not bit identity (gsdr_ext.h).
// ------------------------------------------------------------------------------------------------
template <int MODE, int NCT_ = 4>
struct I8ChainMfma {
  static constexpr int D = 4;
  static constexpr int WG = 256;
  static constexpr int NCT = NCT_;
  static constexpr int KT = (WG / 64) * NCT * 128;
  static constexpr int STRIDE = MODE == kModeFm ? KT - 1 : KT;
  static constexpr int MAXNS = 6;
  static constexpr int MAXT = 32 * MAXNS - 15 * D;  // 132
  static constexpr int SPAN = (KT - 16) * D + 32 * MAXNS;
  static constexpr int NG = SPAN / 4;  // 8-byte granules (4 samples)
  static constexpr int NGR = (NG + WG - 1) / WG;
  static_assert(SPAN % 4 == 0, "whole granules");
  __host__ __device__ static constexpr uint32_t addr(uint32_t idx) { return idx * 2u + (idx / 64u) * 16u; }
  static constexpr uint32_t PLANE = (addr(SPAN) + 255u) / 256u * 256u + 128u;
  static constexpr uint32_t LDS_BYTES = PLANE + addr(SPAN);
};

template <int MODE, bool VEC, int BPC, int NCT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BPC, BPC))) void k_chain_i8_mfma(FirParams p, uint32_t ns, uint32_t tiles) {
  using C = I8ChainMfma<MODE, NCT>;
  constexpr int D = C::D;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS_BYTES];
  __shared__ float4 ybuf[MODE == kModeFm ? C::KT / 2 : 1];  // FM: the tile's FIR outputs y'
  __shared__ float wmax[C::WG / 64];
  __shared__ uint32_t wbad[C::WG / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  const Iq8* __restrict__ in = reinterpret_cast<const Iq8*>(p.in);
  float* __restrict__ out = reinterpret_cast<float*>(p.out);
  const uint32_t T = p.T;

  // modulated taps t'_i = t_i e^{j 2 pi (i inc) / 2^32}
  const float t = tid < T ? taps[tid] : 0.0f;
  const float2 ph = nco_direct(tid * p.nco_inc);
  const float tr = t * ph.x, ti = t * ph.y;
  float a = fmaxf(fabsf(tr), fabsf(ti));
  uint32_t bad = isfinite(t) ? 0u : 1u;
  for (int o = 32; o > 0; o >>= 1) {
    a = fmaxf(a, __shfl_xor(a, o, 64));
    bad |= __shfl_xor(bad, o, 64);
  }
  if (lane == 0) {
    wmax[w] = a;
    wbad[w] = bad;
  }
  __syncthreads();
  float amax = wmax[0];
  bad = wbad[0];
#pragma unroll
  for (int i = 1; i < C::WG / 64; ++i) {
    amax = fmaxf(amax, wmax[i]);
    bad |= wbad[i];
  }
  if (bad) {  // non-finite taps: the exact per-output chain (the generic kernel's evaluation)
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
      for (uint32_t r = tid; r < (uint32_t)C::STRIDE; r += C::WG) {
        const uint64_t k = (uint64_t)tile * C::STRIDE + r;
        if (k >= p.N) continue;
        const float2 y0 = fir_point<float, Iq8, MODE>(p, k);
        if constexpr (MODE == kModeFm) {
          out[k] = fm_disc(y0, fir_point<float, Iq8, MODE>(p, k + 1), p.fm_gain);
        } else {
          out[k] = am_env(y0);
        }
      }
    }
    return;
  }
  int e = 0;
  (void)frexpf(amax, &e);
  const int sc = 14 - e;
  float* ldsT = reinterpret_cast<float*>(lds);
  ldsT[tid] = ldexpf(tr, sc);
  ldsT[C::WG + tid] = ldexpf(ti, sc);
  __syncthreads();
  gsdr_h8 arh[C::MAXNS], arl[C::MAXNS], aih[C::MAXNS], ail[C::MAXNS];
  {
    const int m = (int)(lane & 15u), q = (int)(lane >> 4);
#pragma unroll
    for (int s = 0; s < C::MAXNS; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 32 * s + 8 * q + j - D * m;  // <= 191 < WG
        const float vr = i >= 0 ? ldsT[i] : 0.0f, vi = i >= 0 ? ldsT[C::WG + i] : 0.0f;
        const _Float16 hr = (_Float16)vr, hi = (_Float16)vi;
        arh[s][j] = hr;
        arl[s][j] = (_Float16)(vr - (float)hr);
        aih[s][j] = hi;
        ail[s][j] = (_Float16)(vi - (float)hi);
      }
    }
  }
  const float oscale = ldexpf(1.0f / 127.0f, -sc);
  // FM: the rotation the taps leave out, 2 pi (4 inc mod 2^32) / 2^32 in (-pi, pi]
  const float dphi = (float)((double)(int32_t)(4u * p.nco_inc) * (6.283185307179586 / 4294967296.0));
  __syncthreads();

  const int n = (int)(lane & 15u), q = (int)(lane >> 4), c = n & 1, b = n >> 1;
  const char* bplane = lds + (c ? C::PLANE : 0u);
  for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const uint64_t k_t = (uint64_t)tile * C::STRIDE;
    const uint64_t S0 = k_t * D;
    uint2 wv[C::NGR];
#pragma unroll
    for (int r = 0; r < C::NGR; ++r) {
      const uint32_t g = tid + (uint32_t)r * C::WG;
      const uint64_t s = S0 + 4ull * g;
      wv[r] = make_uint2(0u, 0u);
      if (g < (uint32_t)C::NG) {
        if (VEC && s + 4 <= p.L) {
          typedef uint32_t u2v __attribute__((ext_vector_type(2)));
          const u2v t2 = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(in + s));
          wv[r] = make_uint2(t2.x, t2.y);
        } else {
          uint32_t d[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const Iq8 a0 = s + 2 * k < p.L ? in[s + 2 * k] : Iq8{0, 0};
            const Iq8 a1 = s + 2 * k + 1 < p.L ? in[s + 2 * k + 1] : Iq8{0, 0};
            d[k] = (uint32_t)(uint8_t)a0.x | (uint32_t)(uint8_t)a0.y << 8 | (uint32_t)(uint8_t)a1.x << 16 |
                   (uint32_t)(uint8_t)a1.y << 24;
          }
          wv[r] = make_uint2(d[0], d[1]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < C::NGR; ++r) {
      const uint32_t g = tid + (uint32_t)r * C::WG;
      if (g < (uint32_t)C::NG) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 hi_, hq_;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const uint32_t wd = k ? wv[r].y : wv[r].x;
#pragma unroll
          for (int u = 0; u < 2; ++u) {  // gsdrInt8ToNormFloat clamps -128 to -1.0 = -127 / 127
            hi_[2 * k + u] = (_Float16)max((int)(wd << (24 - 16 * u)) >> 24, -127);
            hq_[2 * k + u] = (_Float16)max((int)(wd << (16 - 16 * u)) >> 24, -127);
          }
        }
        const uint32_t o = C::addr(4u * g);
        *reinterpret_cast<h4*>(lds + o) = hi_;
        *reinterpret_cast<h4*>(lds + C::PLANE + o) = hq_;
      }
    }
    __syncthreads();
    float4 res[C::NCT];
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
      const uint32_t cbase = (w * C::NCT + (uint32_t)ct) * 128u;
      const uint32_t idx0 = (cbase + 16u * (uint32_t)b) * D + 8u * (uint32_t)q;
      gsdr_f4v ar = {0.0f, 0.0f, 0.0f, 0.0f}, ai = ar;
#pragma unroll
      for (int s = 0; s < C::MAXNS; ++s) {
        if ((uint32_t)s < ns) {
          const gsdr_h8 bf = *reinterpret_cast<const gsdr_h8*>(bplane + C::addr(idx0 + 32u * (uint32_t)s));
          ar = __builtin_amdgcn_mfma_f32_16x16x32_f16(arl[s], bf, ar, 0, 0, 0);
          ai = __builtin_amdgcn_mfma_f32_16x16x32_f16(ail[s], bf, ai, 0, 0, 0);
          ar = __builtin_amdgcn_mfma_f32_16x16x32_f16(arh[s], bf, ar, 0, 0, 0);
          ai = __builtin_amdgcn_mfma_f32_16x16x32_f16(aih[s], bf, ai, 0, 0, 0);
        }
      }
      // I lane (c = 0): ar = P, ai = Q'; Q lane: ar = R, ai = S.  y' = (P - S) + j (R + Q')
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float other = __shfl_xor(ai[i], 1, 64);
        v[i] = (c ? ar[i] + other : ar[i] - other) * oscale;
      }
      // lane (q, b, c) keeps rows 2c, 2c + 1 of its 4q group, both components
      const float g0 = __shfl_xor(c ? v[0] : v[2], 1, 64), g1 = __shfl_xor(c ? v[1] : v[3], 1, 64);
      res[ct] = c ? make_float4(g0, v[2], g1, v[3]) : make_float4(v[0], g0, v[1], g1);
      if constexpr (MODE == kModeAm) {
        const uint32_t rr = cbase + 16u * (uint32_t)b + 4u * (uint32_t)q + 2u * (uint32_t)c;
        const uint64_t k = k_t + rr;
        const float e0 = am_env(make_float2(res[ct].x, res[ct].y)), e1 = am_env(make_float2(res[ct].z, res[ct].w));
        if (k + 1 < p.N) {
          *reinterpret_cast<float2*>(out + k) = make_float2(e0, e1);
        } else if (k < p.N) {
          out[k] = e0;
        }
      }
    }
    if constexpr (MODE == kModeFm) {
      // the tile's y' in their own LDS slots (y'[rr], y'[rr + 1] at float4 slot rr / 2), then one barrier
      // for both the planes (read by every wave's MFMAs) and y' (read across waves below); the next
      // tile's staging barrier orders this pass's reads before the next writes of ybuf
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) {
        const uint32_t rr = (w * C::NCT + (uint32_t)ct) * 128u + 16u * (uint32_t)b + 4u * (uint32_t)q + 2u * (uint32_t)c;
        ybuf[rr >> 1] = res[ct];
      }
      __syncthreads();
      const float2* y2 = reinterpret_cast<const float2*>(ybuf);
      for (uint32_t r = tid; r < (uint32_t)C::STRIDE; r += C::WG) {
        const uint64_t k = k_t + r;
        if (k < p.N) {
          const float2 z = disc_product(y2[r], y2[r + 1]);
          float ang = disc_atan2(z.y, z.x) + dphi;
          ang = ang > 3.14159274f ? ang - 6.28318548f : (ang <= -3.14159274f ? ang + 6.28318548f : ang);
          out[k] = p.fm_gain * ang;
        }
      }
    } else {
      __syncthreads();  // every wave is done reading the tile's planes
    }
  }
}

}  // namespace gsdr
