// gsdr-mi355x: complex<float> FIR, decimation 4, on the matrix cores (gsdrxFirFCVariant 42/43;
// DESIGN.md section 3.1).
//
// The int8 kernel (fir_i8_mfma.hpp) showed that the matrix cores do the 127-tap sums for a fraction of
// the packed-VALU energy. Float samples are not exact in fp16, so each one is split:
//   * per 32-sample chunk (both components) a power of two 2^k puts the chunk's largest magnitude M in
//     [2^14, 2^15); every sample y = x 2^k is split y = hi + lo into two fp16 parts (|y - hi - lo| <=
//     2^-22 |y| whenever |x| >= 2^-17 M, which is checked, see below);
//   * taps as in the int8 kernel: scaled by 2^sc (max |t| in [2^13, 2^14)) and split into two fp16 parts;
//   * y[k] = 2^-sc sum_chunks 2^-k (sum over the chunk's products hi*thi + hi*tlo + lo*thi), each product
//     exact in fp32, the dropped lo*tlo below 2^-22 of its term: normwise error ~3 2^-22 plus the fp32
//     accumulation, against the float parity bar max_k |y - y_ref| / sum_i |t_i||x_4k+i| <= 1e-5.
// One 32-sample chunk is exactly one K step of one MFMA column (column windows start at multiples of
// 64 samples, steps are 32 samples), so each step has its own accumulator, rescaled by 2^-k into the
// column's total with one FMA per value.
// Chunks that a two-part split cannot carry to 2^-22 -- a non-finite sample, a nonzero sample below
// 2^-17 M, or M below 2^-109 -- are staged as zeros and every output whose window touches them is
// recomputed by the reference's ascending loop (fir_point): the reference's values and non-finite
// semantics for those outputs. Taps that are not all finite take that loop for every output.
// Summation order depends on an output's position within its 16-output block, i.e. on where a call
// starts: this kernel is not used where chunked calls must reproduce a monolithic call bit for bit.
#pragma once

#include "fir_i8_mfma.hpp"

namespace gsdr {

template <int NCT_>
struct F32Mfma {
  static constexpr int D = 4;
  static constexpr int WG = 256;
  static constexpr int NCT = NCT_;                  // C tiles (128 outputs) per wave and tile
  static constexpr int KT = (WG / 64) * NCT * 128;  // outputs per tile
  static constexpr int MAXNS = 6;                   // 32-sample K steps: 15 D + T <= 192
  static constexpr int MAXT = 32 * MAXNS - 15 * D;  // 132
  static constexpr int SPAN = (KT - 16) * D + 32 * MAXNS;
  static constexpr int NCH = SPAN / 32;  // scale chunks per tile
  static constexpr int NG = SPAN / 2;    // 16-byte granules (2 complex samples)
  static constexpr int NGR = (NG + WG - 1) / WG;
  static_assert(SPAN % 32 == 0, "whole chunks");
  static constexpr int MW = KT / 32;  // output-flag words
  __host__ __device__ static constexpr uint32_t addr(uint32_t idx) { return idx * 2u + (idx / 64u) * 16u; }
  // plane stride = 128 (mod 256): I and Q columns interleave their bank groups (as fir_i8_mfma.hpp)
  static constexpr uint32_t PLANE = (addr(SPAN) + 255u) / 256u * 256u + 128u;
  static constexpr uint32_t LDS_PLANES = 4 * PLANE;  // I hi, Q hi, I lo, Q lo
};

__device__ __forceinline__ uint32_t dpp_max16(uint32_t m) {
  // max over each 16-lane row: xor 1, xor 2 (quad_perm), half-row mirror, row mirror
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false));
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xF, 0xF, false));
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x141, 0xF, 0xF, false));
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x140, 0xF, 0xF, false));
  return m;
}

__device__ __forceinline__ uint32_t split_pair(float a, float b, float sc, uint32_t& lo) {
  const float ya = a * sc, yb = b * sc;  // exact: power-of-two scale, no overflow (|y| < 2^15)
  const _Float16 ha = (_Float16)ya, hb = (_Float16)yb;
  const _Float16 la = (_Float16)(ya - (float)ha), lb = (_Float16)(yb - (float)hb);  // y - h exact
  lo = (uint32_t)__builtin_bit_cast(uint16_t, la) | (uint32_t)__builtin_bit_cast(uint16_t, lb) << 16;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | (uint32_t)__builtin_bit_cast(uint16_t, hb) << 16;
}

template <int NCT, bool VEC, int BPC, bool NOFIX = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BPC, BPC))) void k_fir_f32_mfma(FirParams p, uint32_t ns, uint32_t tiles) {
  using C = F32Mfma<NCT>;
  constexpr int D = C::D;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS_PLANES];
  __shared__ float invk[C::NCH];
  __shared__ uint32_t oflag[2][C::MW];
  __shared__ float wmax[C::WG / 64];
  __shared__ uint32_t wbad[C::WG / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const float* __restrict__ taps = reinterpret_cast<const float*>(p.taps);
  const float2* __restrict__ in = reinterpret_cast<const float2*>(p.in);
  float2* __restrict__ out = reinterpret_cast<float2*>(p.out);
  const uint32_t T = p.T;

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
  if (tid < (uint32_t)C::MW) {
    oflag[0][tid] = 0u;
    oflag[1][tid] = 0u;
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
        if (k < p.N) out[k] = fir_point<float, float2, kModeFir>(p, k);
      }
    }
    return;
  }
  int e = 0;
  (void)frexpf(amax, &e);
  const int sc = 14 - e;
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
        const float v = i >= 0 ? ldsT[i] : 0.0f;  // i <= 191 < WG
        const _Float16 h = (_Float16)v;
        ahi[s][j] = h;
        alo[s][j] = (_Float16)(v - (float)h);
      }
    }
  }
  const float oscale = ldexpf(1.0f, -sc);
  __syncthreads();

  const int n = (int)(lane & 15u), q = (int)(lane >> 4), c = n & 1, b = n >> 1;
  const char* bhi = lds + (c ? C::PLANE : 0u);
  const char* blo = bhi + 2u * C::PLANE;
  uint32_t par = 0;
  for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x, par ^= 1u) {
    const uint64_t k_t = (uint64_t)tile * C::KT;
    const uint64_t S0 = k_t * D;
    float4 v[C::NGR];
#pragma unroll
    for (int r = 0; r < C::NGR; ++r) {
      const uint32_t g = tid + (uint32_t)r * C::WG;
      const uint64_t s = S0 + 2ull * g;
      v[r] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (g < (uint32_t)C::NG) {
        if (VEC && s + 2 <= p.L) {
          v[r] = load16_nt(reinterpret_cast<const float4*>(in + s));
        } else {
          if (s < p.L) {
            const float2 x0 = in[s];
            v[r].x = x0.x;
            v[r].y = x0.y;
          }
          if (s + 1 < p.L) {
            const float2 x1 = in[s + 1];
            v[r].z = x1.x;
            v[r].w = x1.y;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < C::NGR; ++r) {
      const uint32_t g = tid + (uint32_t)r * C::WG;  // chunk g / 16: one 16-lane row of the wave
      const uint32_t ax = __float_as_uint(v[r].x) & 0x7fffffffu, ay = __float_as_uint(v[r].y) & 0x7fffffffu;
      const uint32_t az = __float_as_uint(v[r].z) & 0x7fffffffu, aw = __float_as_uint(v[r].w) & 0x7fffffffu;
      const uint32_t M = dpp_max16(max(max(ax, ay), max(az, aw)));  // NaN bits above Inf above finite
      const uint32_t E = M >> 23;
      const uint32_t thr = M - (17u << 23);  // bits of M 2^-17 (E >= 18)
      const bool tiny = (ax - 1u < thr - 1u) | (ay - 1u < thr - 1u) | (az - 1u < thr - 1u) | (aw - 1u < thr - 1u);
      const bool lane_bad = !NOFIX && M != 0u && (E >= 255u || E < 18u || tiny);
      const uint64_t bal = __ballot(lane_bad);
      const bool chunk_bad = ((bal >> (lane & 48u)) & 0xffffull) != 0ull;
      const float scl = (M == 0u || chunk_bad) ? 0.0f : __uint_as_float((268u - E) << 23);
      uint32_t loI, loQ;
      uint32_t hiI = split_pair(v[r].x, v[r].z, scl, loI);
      uint32_t hiQ = split_pair(v[r].y, v[r].w, scl, loQ);
      if (chunk_bad) {  // staged as zeros (Inf * 0 would be NaN); its outputs are recomputed below
        hiI = hiQ = loI = loQ = 0u;
      }
      if (g < (uint32_t)C::NG) {
        const uint32_t o = C::addr(2u * g);
        *reinterpret_cast<uint32_t*>(lds + o) = hiI;
        *reinterpret_cast<uint32_t*>(lds + C::PLANE + o) = hiQ;
        *reinterpret_cast<uint32_t*>(lds + 2u * C::PLANE + o) = loI;
        *reinterpret_cast<uint32_t*>(lds + 3u * C::PLANE + o) = loQ;
        if ((lane & 15u) == 0u) {
          const uint32_t ch = g >> 4;
          invk[ch] = (M == 0u || chunk_bad) ? 0.0f : __uint_as_float((E - 14u) << 23);
          if (chunk_bad) {  // outputs whose window [4r, 4r + T) meets samples [32 ch, 32 ch + 32)
            const int num = (int)(32u * ch) - (int)T + 1;
            const int r_lo = num <= 0 ? 0 : (num + 3) >> 2;
            const int r_hi = min(C::KT - 1, (int)((32u * ch + 31u) >> 2));
            for (int r2 = r_lo; r2 <= r_hi; ++r2) atomicOr(&oflag[par][r2 >> 5], 1u << (r2 & 31));
          }
        }
      }
    }
    __syncthreads();
    if (tid < (uint32_t)C::MW) oflag[par ^ 1u][tid] = 0u;  // next tile's flags (last read a tile ago)
#pragma unroll 1
    for (int ct = 0; ct < C::NCT; ++ct) {
      const uint32_t cbase = (w * C::NCT + (uint32_t)ct) * 128u;
      const uint32_t blk = cbase + 16u * (uint32_t)b;
      const uint32_t idx0 = blk * D + 8u * (uint32_t)q;
      gsdr_f4v tot = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < C::MAXNS; ++s) {
        if ((uint32_t)s < ns) {
          const uint32_t o = C::addr(idx0 + 32u * (uint32_t)s);
          const gsdr_h8 bh = *reinterpret_cast<const gsdr_h8*>(bhi + o);
          const gsdr_h8 bl = *reinterpret_cast<const gsdr_h8*>(blo + o);
          gsdr_f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[s], bh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[s], bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[s], bh, acc, 0, 0, 0);
          const float ik = invk[(blk >> 3) + (uint32_t)s];
#pragma unroll
          for (int i = 0; i < 4; ++i) tot[i] = fmaf(acc[i], ik, tot[i]);
        }
      }
      const float r0 = tot[0] * oscale, r1 = tot[1] * oscale, r2 = tot[2] * oscale, r3 = tot[3] * oscale;
      const float g0 = __shfl_xor(c ? r0 : r2, 1, 64), g1 = __shfl_xor(c ? r1 : r3, 1, 64);
      float4 o4 = c ? make_float4(g0, r2, g1, r3) : make_float4(r0, g0, r1, g1);
      const uint32_t rr = blk + 4u * (uint32_t)q + 2u * (uint32_t)c;
      const uint64_t k = k_t + rr;
      const uint32_t fl = (oflag[par][rr >> 5] >> (rr & 31u)) & 3u;
      if (fl != 0u) {  // rare: outputs next to a chunk the split cannot carry
        if ((fl & 1u) && k < p.N) {
          const float2 y = fir_point<float, float2, kModeFir>(p, k);
          o4.x = y.x;
          o4.y = y.y;
        }
        if ((fl & 2u) && k + 1 < p.N) {
          const float2 y = fir_point<float, float2, kModeFir>(p, k + 1);
          o4.z = y.x;
          o4.w = y.y;
        }
      }
      if (k + 1 < p.N) {
        store16_nt(reinterpret_cast<float4*>(out + k), o4);
      } else if (k < p.N) {
        out[k] = make_float2(o4.x, o4.y);
      }
    }
    __syncthreads();
  }
}

}  // namespace gsdr
