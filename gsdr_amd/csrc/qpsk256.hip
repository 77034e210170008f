// gsdr-mi355x: 256-point constellation modulate / demodulate.
// Replaces reference src/qpsk256.cu (tables :25-71, modulate :74-151, demodulate :154-259,
// wrappers :262-431; header qpsk256.h:125-230).
//
// Tables are built on the host, in float, with exactly the reference's expressions
// (qpsk256.cu:33-34, 54-56, 64-67), and uploaded per device on the caller's stream. Each workgroup
// copies the 2 KiB table it needs into LDS, so lookups are LDS reads rather than divergent
// constant-cache accesses.
//
// Demodulation decision: the reference's own rule (qpsk256.cu:171-181), bit for bit -- the first index
// attaining the minimum of cuCabsf(received - point) over all 256 points, strict '<', initialised to
// +inf (so a NaN/inf symbol maps to 0). cuCabsf is CUDA cuComplex.h's scaled hypot (ref_cabsf below),
// with `1 + t*t` contracted to one fma as nvcc does by default. The fast paths rank candidates by the
// cheaper squared distance s_i = fl(fl(dx*dx) + fl(dy*dy)) of the same rounded differences: when the
// smallest s beats every other candidate by a relative margin of 2^-18, which is far wider than the
// combined rounding of s (2^-23) and of cuCabsf (about 4 ulp), the cuCabsf order agrees and that
// candidate is the reference's answer. Otherwise (a near-tie) the candidates are re-ranked with
// cuCabsf itself in ascending index order. For the rectangular grid a received point inside
// |re|,|im| <= 4|a| can only be won by one of the 3 x 3 grid points around its per-axis nearest level
// (every other point is farther by >= 0.035 a^2); circular tables use per-cell candidate lists;
// anything else takes the exhaustive cuCabsf search.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <type_traits>
#include <vector>

#include "awgn.hpp"
#include "gsdr/gsdr_ext.h"
#include "gsdr/qpsk256.h"
#include "launch.hpp"

namespace gsdr {

constexpr int kCBlock = 256;
constexpr int kCSym = 16;  // symbols per thread

// [0] rectangular, [1] circular; per device (module globals are per-device copies).
__constant__ float2 c_qpsk256_tables[2][256];

// Circular table: per-cell candidate lists over a kCellGrid^2 grid covering [-R, R)^2, built on the
// host by gsdrQpsk256InitConstellation. A point is listed for a cell when its distance to the cell is
// at most the smallest worst-case distance of any table point over the cell (plus a margin for float
// rounding), so every point that can win the argmin anywhere in the cell -- ties included -- is on the
// list, and the argmin over the list in index order is the exhaustive one -- for the squared distance
// and, with the near-tie re-ranking of the demodulation kernel, for the reference's cuCabsf rule.
// R == 0 disables the lookup.
// One 16-bit word per cell: length (bits 12-15) and, for a one-point list, the point itself (bits
// 0-11), else the offset of the list in `lists` (ascending indices). Neighbouring cells mostly share
// their lists, which are stored once: the circular table at any amplitude has 2,863 one-point cells
// and 6,353 longer lists of which 1,078 are distinct (3,293 bytes), so one cell lookup decides 87 % of
// noisy symbols with a single LDS load and the whole structure is 22.5 KB of LDS.
constexpr int kCellGrid = 96;
constexpr int kCellListBytes = 4096;  // 12-bit offsets
constexpr double kCellSpan = 1.3;  // grid half-width R = 1.3 * max |c|: noisy symbols stay on the grid
struct alignas(16) CircCells {
  float R;
  float inv_cs;  // kCellGrid / (2 R)
  uint16_t cell[kCellGrid * kCellGrid];
  uint8_t lists[kCellListBytes];
};
__device__ CircCells g_circ_cells;

struct C256Streams {
  const void* in[4];
  void* out[4];
};

__device__ __forceinline__ float sqdist(float2 r, float2 c) {
  const float dx = __fsub_rn(r.x, c.x);
  const float dy = __fsub_rn(r.y, c.y);
  return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
}

// cuCabsf (CUDA cuComplex.h, called at qpsk256.cu:173, 182): v = max(|a|, |b|), w = min, t = w / v,
// |z| = v * sqrt(fma(t, t, 1)), v + w when v == 0 or either exceeds FLT_MAX. IEEE division and square
// root, as nvcc's defaults (-prec-div, -prec-sqrt) give: '/' and __builtin_sqrtf are correctly rounded
// under HIP's defaults (__fsqrt_rn is not: this toolchain maps it to the ~1-ulp v_sqrt_f32).
__device__ __forceinline__ float ref_cabsf(float re, float im) {
  const float a = fabsf(re), b = fabsf(im);
  const float v = a > b ? a : b;
  const float w = a > b ? b : a;
  float t = __fdiv_rn(w, v);
  t = fmaf(t, t, 1.0f);
  t = __fmul_rn(v, __builtin_sqrtf(t));
  if (v == 0.0f || v > 3.402823466e38f || w > 3.402823466e38f) t = __fadd_rn(v, w);
  return t;
}

// the reference's distance of received point r to table point c (cuCsubf, then cuCabsf)
__device__ __forceinline__ float ref_dist(float2 r, float2 c) { return ref_cabsf(__fsub_rn(r.x, c.x), __fsub_rn(r.y, c.y)); }

// fast-path acceptance: every other candidate's squared distance exceeds s_min by 2^-18 relative
__device__ __forceinline__ float tie_threshold(float smin) { return fmaf(smin, 0x1p-18f, smin); }

__device__ __noinline__ uint32_t demod_exhaustive(const float2* __restrict__ tab, float2 r) {
  float best = INFINITY;
  uint32_t idx = 0;
  for (uint32_t i = 0; i < 256; ++i) {
    const float d = ref_dist(r, tab[i]);
    if (d < best) {
      best = d;
      idx = i;
    }
  }
  return idx;
}

__device__ __forceinline__ int nearest_level(float v, float scale) {
  // level i sits at (i - 7.5) / 7.5 * a  =>  i ~= v * (7.5 / a) + 7.5
  const float u = fmaf(v, scale, 7.5f);
  int i = (int)rintf(u);
  return i < 0 ? 0 : (i > 15 ? 15 : i);
}

// Rectangular fast path. Table entry 16 i + q is (lx[i], ly[q]) -- the I coordinate depends on i only
// and the Q coordinate on q only (qpsk256.cu:33-34) -- so every candidate distance is a rounded sum
// fl(ex[i] + ey[q]) of per-axis squares read from level arrays, bit-identical to sqdist() on the
// table entries. lxp / lyp are the level arrays padded with +inf at both ends (entry k + 1 = level k),
// so neighbours outside [0, 15] have infinite distance and never win.
//
// The 3 x 3 neighbourhood of the per-axis nearest levels contains the exhaustive argmin for
// |re|,|im| <= 4|a|. Rounded addition is monotone in each operand, so with a = first argmin of ex and
// b = first argmin of ey the minimum is dmin = fl(ex[a] + ey[b]), and every other candidate is >= the
// second-smallest ex plus ey[b], or >= ex[a] plus the second-smallest ey. When both of those exceed
// dmin by the 2^-18 margin, (a, b) is the reference's answer; otherwise (a near-tie at a decision
// boundary) the 9 candidates are ranked by cuCabsf in ascending index order with strict '<', as the
// reference's exhaustive loop does (no point outside the 3 x 3 can be that close). Returns 256 when the
// symbol needs the exhaustive search (outside |re|,|im| <= 4|a|, or NaN).
// The near-tie ranking of demod_rect_fast's 3 x 3 candidates by cuCabsf, in ascending index order with
// strict '<' as the reference's loop. Out of line: it runs for a few symbols in a million, and inlined
// into each of a thread's 16 unrolled symbols (nine divisions and square roots each) it made the
// kernel ~60 KB of code.
__device__ __noinline__ uint32_t demod_rect_tie(float dx0, float dx1, float dx2, float dy0, float dy1, float dy2,
                                                int i0, int q0) {
  const float dx[3] = {dx0, dx1, dx2}, dy[3] = {dy0, dy1, dy2};
  float best = INFINITY;
  uint32_t idx = 0;
#pragma unroll
  for (int di = 0; di < 3; ++di) {
#pragma unroll
    for (int dq = 0; dq < 3; ++dq) {
      // out-of-grid neighbours (padded +inf levels) give an infinite difference and never win
      const float d = ref_cabsf(dx[di], dy[dq]);
      if (d < best) {
        best = d;
        idx = (uint32_t)((i0 - 1 + di) * 16 + (q0 - 1 + dq));
      }
    }
  }
  return idx;
}

typedef float gsdr_f32x2 __attribute__((ext_vector_type(2)));

// floor(v + 0.5) as an integer in one instruction (v_cvt_rpi_i32_f32); the centre of the 3 x 3 neighbourhood.
// (It differs from rintf only at exact halves, where both nearest levels are in either neighbourhood.)
__device__ __forceinline__ int cvt_rpi(float v) {
  int r;
  asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// The three per-axis candidates (levels c - 1, c, c + 1 of the padded array lp): squared differences e0..e2
// (the first two on packed instructions, straight from the two loaded levels), their minimum, median and
// the first index reaching the minimum.
struct AxisCand {
  float d[3], e[3], emin, emed;
  int arg;
};
__device__ __forceinline__ AxisCand axis_cand(const float* __restrict__ lp, float v) {
  AxisCand c;
  const gsdr_f32x2 l01 = gsdr_f32x2{lp[0], lp[1]};
  const gsdr_f32x2 d01 = gsdr_f32x2{v, v} - l01;  // __fsub_rn each: -ffp-contract=off, no fusing
  const float d2 = v - lp[2];
  const gsdr_f32x2 e01 = d01 * d01;
  c.d[0] = d01.x;
  c.d[1] = d01.y;
  c.d[2] = d2;
  c.e[0] = e01.x;
  c.e[1] = e01.y;
  c.e[2] = d2 * d2;
  c.emin = fminf(fminf(c.e[0], c.e[1]), c.e[2]);
  c.emed = __builtin_amdgcn_fmed3f(c.e[0], c.e[1], c.e[2]);
  c.arg = c.e[0] == c.emin ? 0 : (c.e[1] == c.emin ? 1 : 2);
  return c;
}

__device__ __forceinline__ uint32_t demod_rect_fast(const float* __restrict__ lxp, const float* __restrict__ lyp, float2 r,
                                                    float lim, float scale) {
  if (!(fabsf(r.x) <= lim && fabsf(r.y) <= lim)) return 256u;
  // level i sits at (i - 7.5) / 7.5 * a  =>  i ~= v * (7.5 / a) + 7.5 (both axes in one packed fma)
  const gsdr_f32x2 u = __builtin_elementwise_fma(gsdr_f32x2{r.x, r.y}, gsdr_f32x2{scale, scale}, gsdr_f32x2{7.5f, 7.5f});
  const int i0 = min(max(cvt_rpi(u.x), 0), 15);
  const int q0 = min(max(cvt_rpi(u.y), 0), 15);
  const AxisCand cx = axis_cand(lxp + i0, r.x), cy = axis_cand(lyp + q0, r.y);
  const float thr = tie_threshold(__fadd_rn(cx.emin, cy.emin));
  if (__fadd_rn(cx.emed, cy.emin) > thr && __fadd_rn(cx.emin, cy.emed) > thr) {
    return (uint32_t)((i0 - 1 + cx.arg) * 16 + (q0 - 1 + cy.arg));
  }
  return demod_rect_tie(cx.d[0], cx.d[1], cx.d[2], cy.d[0], cy.d[1], cy.d[2], i0, q0);
}

// Rectangular decision in ~15 VALU operations, taken when it is provably the reference's answer. u is the symbol's
// position in level units per axis (level k at u = k up to rounding: < 2^-17 of a level spacing, from scale, the
// fma and the host-built levels). When the clamped u of both axes is more than kRectMargin from every midpoint
// between two levels, the nearest level is unambiguous by a margin (in squared distance the runner-up is farther by
// >= 2^-11 of dmin) that no rounding of the reference's cuCabsf ranking can reverse, so (i, q) is its first argmin.
// Symbols within the margin of a midpoint (~1e-4 of noisy symbols) or beyond |re|,|im| <= 4|a| (or NaN) return
// false and take demod_rect_fast's careful path.
constexpr float kRectMargin = 0x1p-10f;
__device__ __forceinline__ bool demod_rect_quick(float2 r, float lim, float scale, uint32_t& k) {
  const gsdr_f32x2 u = __builtin_elementwise_fma(gsdr_f32x2{r.x, r.y}, gsdr_f32x2{scale, scale}, gsdr_f32x2{7.5f, 7.5f});
  const float tx = __builtin_amdgcn_fmed3f(u.x, 0.0f, 15.0f), ty = __builtin_amdgcn_fmed3f(u.y, 0.0f, 15.0f);
  const float ix = __builtin_rintf(tx), iy = __builtin_rintf(ty);
  const gsdr_f32x2 d = gsdr_f32x2{tx, ty} - gsdr_f32x2{ix, iy};
  k = (uint32_t)ix * 16u + (uint32_t)iy;
  return fabsf(r.x) <= lim && fabsf(r.y) <= lim && fmaxf(fabsf(d.x), fabsf(d.y)) <= 0.5f - kRectMargin;
}

__device__ __forceinline__ void load_table(float2* lds_tab, uint32_t type) {
  const float2* src = c_qpsk256_tables[type == 0 ? 0 : 1];
  for (uint32_t i = threadIdx.x; i < 256; i += kCBlock) lds_tab[i] = src[i];
  __syncthreads();
}

__global__ __launch_bounds__(kCBlock) void k_c256_mod(C256Streams st, uint32_t n, uint32_t type) {
  __shared__ float2 tab[256];
  load_table(tab, type);
  const uint8_t* __restrict__ in = reinterpret_cast<const uint8_t*>(st.in[blockIdx.y]);
  float2* __restrict__ out = reinterpret_cast<float2*>(st.out[blockIdx.y]);
  // a full, aligned block: lane t of slot q handles symbol pair q * kCBlock + t (coalesced 1 KB stores)
  const uint64_t base = (uint64_t)blockIdx.x * kCBlock * kCSym;
  if (base + kCBlock * kCSym <= n && (reinterpret_cast<uintptr_t>(in) & 1u) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    const uint16_t* pin = reinterpret_cast<const uint16_t*>(in + base);
    float4* o = reinterpret_cast<float4*>(out + base);
    uint32_t pr[kCSym / 2];
#pragma unroll
    for (int q = 0; q < kCSym / 2; ++q) pr[q] = pin[q * kCBlock + threadIdx.x];
#pragma unroll
    for (int q = 0; q < kCSym / 2; ++q) {
      const float2 p0 = tab[pr[q] & 0xffu];
      const float2 p1 = tab[pr[q] >> 8];
      o[q * kCBlock + threadIdx.x] = make_float4(p0.x, p0.y, p1.x, p1.y);
    }
    return;
  }
  const uint64_t s0 = base + (uint64_t)threadIdx.x * kCSym;
  if (s0 >= n) return;
  if (s0 + kCSym <= n && (reinterpret_cast<uintptr_t>(in + s0) & 15u) == 0 &&
      (reinterpret_cast<uintptr_t>(out + s0) & 15u) == 0) {
    const uint4 w = *reinterpret_cast<const uint4*>(in + s0);
    const uint32_t words[4] = {w.x, w.y, w.z, w.w};
    float4* o = reinterpret_cast<float4*>(out + s0);
#pragma unroll
    for (int q = 0; q < kCSym / 2; ++q) {
      const uint32_t word = words[q / 2];
      const float2 p0 = tab[(word >> (16 * (q & 1))) & 0xffu];
      const float2 p1 = tab[(word >> (16 * (q & 1) + 8)) & 0xffu];
      o[q] = make_float4(p0.x, p0.y, p1.x, p1.y);
    }
  } else {
    for (int k = 0; k < kCSym; ++k) {
      if (s0 + k < n) out[s0 + k] = tab[in[s0 + k]];
    }
  }
}

// Modulate + counter-based AWGN (gsdrxQpsk256ModulateAwgn; awgn.hpp). One Philox block serves three
// symbols, so a lane takes six consecutive symbols a step: two blocks when the first absolute index is a
// multiple of 3 (R3 = firstSymbolIndex % 3, uniform, a template parameter so every slot and block index
// is a compile-time constant), three otherwise. A wave's 384 noisy symbols (3 KB) go through LDS so that
// each of its three 16-byte store instructions writes 1 KB contiguous: stored straight from the lanes
// (48-byte lane stride) they ran at about half the copy rate, which bound the kernel once the normals
// were cheap (the write-heavy maps of section 3.6 showed the same).
constexpr int kAwgnSym = 6;    // symbols per lane per step
#ifndef GSDR_AWGN_STEPS
#define GSDR_AWGN_STEPS 3
#endif
constexpr int kAwgnSteps = GSDR_AWGN_STEPS;  // steps per workgroup
constexpr uint32_t kAwgnWaveSyms = 64u * kAwgnSym;
constexpr uint32_t kAwgnBlockSyms = kCBlock * kAwgnSym * kAwgnSteps;

// LDS hand-off between the lanes of one wave: without it the compiler, reasoning per thread, may
// forward a lane's own earlier LDS store to its later load past another lane's store.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// RECT (GSDR_C256_RECT_LEVELS = 1, a timing switch, off by default): the rectangular table's entry 16 i + q is
// (lx[i], ly[q]) (qpsk256.cu:33-34), so a symbol's point can be two 4-byte reads from 16-entry level arrays --
// conflict-free (distinct levels sit in distinct banks, equal ones broadcast) where the gather from the 256-entry
// table puts up to ~4 lanes of a group on one bank. Measured side by side (profiles/r05_ab_config5.txt): 29.8 us
// against 28.8 us for the gather. The kernel is VALU-bound (Philox), and the level reads cost ~17 more VALU
// instructions per lane step (index splits, two address computations) than the bank conflicts cost in LDS time.
// firstBlk = firstSymbolIndex / 3: with every lane's first symbol a multiple of 6 from the launch's first, its
// first Philox block is firstBlk + s / 3 (no 64-bit division per lane).
#ifndef GSDR_C256_RECT_LEVELS
#define GSDR_C256_RECT_LEVELS 0
#endif
// This lane's six symbols of a step as loaded (a 4-byte and a 2-byte load), kept so until the step needs them:
// nothing waits for the loads before then.
struct SymRaw {
  uint32_t lo;     // symbols 0..3
  uint32_t hi;     // symbols 4, 5 (low 16 bits)
  uint32_t shift;  // bytes to drop (the last symbols of the input, loaded from an address moved back)
};

// The symbols are loaded one step AHEAD: step 0's with the tables, step it + 1's before step it's stores. Vector
// loads and stores share one in-order counter, so a load issued after a step's stores could only be waited for
// together with them (an HBM write's whole latency, each step); and issued before the Philox blocks, a step's
// loads are in flight while they are computed. To keep the compiler's wait counts exact the loads have no branch
// around them: every lane loads 6 bytes from min(s, n - 6) (so no load leaves the input; unaligned loads are
// fine on this part) and drops the bytes before s. SMALL (n < 6, chosen by the launcher): byte loads.
// DEMOD (gsdrxQpsk256ModulateAwgnDemodulate, rectangular table): the same kernel also demodulates every noisy symbol
// it writes, from the registers that hold it -- the decision of gsdrQpsk256Demodulate's rectangular kernel on the
// same float values, bit for bit -- and writes the decisions to `dec`: the round trip in one pass, without reading
// the 134 MB of noisy symbols back.
template <int R3, bool RECT, bool SMALL, bool DEMOD = false>
__global__ __launch_bounds__(kCBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_c256_mod_awgn(const uint8_t* __restrict__ in, float2* __restrict__ out,
                                                            uint32_t n, uint32_t type, float sigma, uint64_t seed,
                                                            uint64_t firstBlk, uint8_t* __restrict__ dec = nullptr) {
  __shared__ float2 tab[256];
  __shared__ float lev[32];  // RECT: lx[0..15], ly[0..15]
  __shared__ AwgnLds ntab;
  __shared__ float4 stage[kCBlock / 64][kAwgnWaveSyms / 2];  // per wave: 384 symbols as 192 float4
  __shared__ float levp[DEMOD ? 40 : 1];  // DEMOD: the demodulator's padded level arrays (lxp, lyp; k_c256_demod)
  float* const lxp = levp;
  float* const lyp = levp + 20;
  constexpr int NB = R3 == 0 ? 2 : 3;  // Philox blocks touched by six symbols starting at slot R3
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  float4* __restrict__ st = stage[wv];
  // 16-byte aligned output: the wave's stores can be whole float4s (every wave step starts at a multiple
  // of 384 symbols from `out`)
  const bool aligned = (reinterpret_cast<uintptr_t>(out) & 15u) == 0;
  const uint64_t base = (uint64_t)blockIdx.x * kAwgnBlockSyms;
  auto wave_first = [&](int it) { return base + (uint64_t)kAwgnWaveSyms * ((uint32_t)it * (kCBlock / 64) + wv); };
  auto load_syms = [&](int it) {
    SymRaw r;
    const uint64_t s = wave_first(it) + (uint64_t)kAwgnSym * lane;
    if constexpr (SMALL) {
      uint32_t b[kAwgnSym];
#pragma unroll
      for (int j = 0; j < kAwgnSym; ++j) b[j] = s + j < n ? in[s + j] : 0u;
      r.lo = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
      r.hi = b[4] | (b[5] << 8);
      r.shift = 0;
    } else {
      const uint64_t sl = s < (uint64_t)n - kAwgnSym ? s : (uint64_t)n - kAwgnSym;
      __builtin_memcpy(&r.lo, in + sl, 4);
      uint16_t h;
      __builtin_memcpy(&h, in + sl + 4, 2);
      r.hi = h;
      r.shift = (uint32_t)min<uint64_t>(s - sl, kAwgnSym);
    }
    return r;
  };
  const AwgnRegs treg = awgn_fetch_table();
  const float2 trow = c_qpsk256_tables[type == 0 ? 0 : 1][threadIdx.x];
  SymRaw raw = load_syms(0);
  awgn_store_table(ntab, treg);
  tab[threadIdx.x] = trow;
  if constexpr (RECT) {
    const float2* src = c_qpsk256_tables[0];
    if (threadIdx.x < 32) lev[threadIdx.x] = threadIdx.x < 16 ? src[threadIdx.x * 16].x : src[threadIdx.x - 16].y;
  }
  float lim = -1.0f, scale = 0.0f;
  if constexpr (DEMOD) {
    const float2* tsrc = c_qpsk256_tables[0];
    if (threadIdx.x < 18) {
      const int k = (int)threadIdx.x - 1;
      lxp[threadIdx.x] = (k < 0 || k > 15) ? INFINITY : tsrc[k * 16].x;
      lyp[threadIdx.x] = (k < 0 || k > 15) ? INFINITY : tsrc[k].y;
    }
    const float a = tsrc[255].x;  // as k_c256_demod<0>: (15 - 7.5) / 7.5 * a == a exactly
    scale = 7.5f / a;
    lim = isfinite(scale) ? 4.0f * fabsf(a) : -1.0f;
  }
  __syncthreads();  // publishes the tables
  // DEMOD: k_c256_demod<0>'s decisions of a lane's six noisy symbols (the reference's cuCabsf argmin, bit for
  // bit): the quick per-axis decision inline for all six, then -- for the ~1e-4 of symbols within its margin of a
  // decision boundary, beyond 4|a| or NaN -- the careful path one symbol at a time (unrolled six times over, its
  // 3 x 3 search had held the kernel at 5 waves a SIMD)
  auto decide6 = [&](const float2 (&y)[kAwgnSym], uint32_t (&d)[kAwgnSym]) {
    uint32_t slow = 0;
#pragma unroll
    for (int j = 0; j < kAwgnSym; ++j) slow |= demod_rect_quick(y[j], lim, scale, d[j]) ? 0u : 1u << j;
    if (__builtin_expect(slow != 0, 0)) {
#pragma unroll 1
      for (int j = 0; j < kAwgnSym; ++j) {
        if (!((slow >> j) & 1u)) continue;
        float2 r = y[0];
#pragma unroll
        for (int i = 1; i < kAwgnSym; ++i) r = j == i ? y[i] : r;  // (a select chain: y stays in registers)
        uint32_t k = demod_rect_fast(lxp, lyp, r, lim, scale);
        if (k >= 256u) {  // demod_exhaustive's loop, inline: its call (the ABI's saved registers) cost 17 VGPRs
          float best = INFINITY;
          k = 0;
#pragma unroll 1
          for (uint32_t i = 0; i < 256; ++i) {
            const float dd = ref_dist(r, tab[i]);
            if (dd < best) {
              best = dd;
              k = i;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < kAwgnSym; ++i) d[i] = j == i ? k : d[i];
      }
    }
  };
  // the noisy symbols of step it (the lane's six, from `raw`)
  auto step_outputs = [&](int it, float2 (&y)[kAwgnSym]) {
    // (first + s) / 3 with s = base + 384 (it * waves + wv) + 6 lane, every term a multiple of 3
    const uint32_t s3 = (uint32_t)blockIdx.x * (kAwgnBlockSyms / 3u) + (kAwgnWaveSyms / 3u) * ((uint32_t)it * (kCBlock / 64) + wv) +
                        2u * lane;
    const uint64_t b0 = firstBlk + s3;
    uint8_t sym[kAwgnSym];
    {
      uint32_t w[NB][4];
#pragma unroll
      for (int b = 0; b < NB; ++b) awgn_block_words(seed, b0 + b, w[b]);
      const uint64_t v6 = ((uint64_t)raw.hi << 32 | raw.lo) >> (8u * raw.shift);
#pragma unroll
      for (int j = 0; j < kAwgnSym; ++j) sym[j] = (uint8_t)(v6 >> (8 * j));
#pragma unroll
      for (int j = 0; j < kAwgnSym; ++j) {
        const float2 g = awgn_slot_main(ntab, w[(R3 + j) / 3], (R3 + j) % 3);
#if defined(GSDR_TUNING_PROBES) && defined(GSDR_C256_PROBE_NOSYMGATHER)
        const float2 p = tab[(lane + (sym[j] & 0x80u)) & 255u];  // timing probe only: conflict-free, wrong symbols
#else
        const float2 p = RECT ? make_float2(lev[sym[j] >> 4], lev[16 + (sym[j] & 15)]) : tab[sym[j]];
#endif
        y[j] = make_float2(p.x + sigma * g.x, p.y + sigma * g.y);
      }
    }
    // a lane whose blocks hold a tail component (~4e-4 of the lanes: its outputs hold a NaN, awgn.hpp) redoes
    // them exactly, regenerating its blocks (so they do not stay live in the common path)
    if (__builtin_expect(awgn_has_tail(y), 0)) {
      uint32_t w[NB][4];
#pragma unroll
      for (int b = 0; b < NB; ++b) awgn_block_words(seed, b0 + b, w[b]);
#pragma unroll
      for (int j = 0; j < kAwgnSym; ++j) {
        const float2 g = awgn_slot(ntab, w[(R3 + j) / 3], (R3 + j) % 3, seed, b0 + (R3 + j) / 3);
        const float2 p = RECT ? make_float2(lev[sym[j] >> 4], lev[16 + (sym[j] & 15)]) : tab[sym[j]];
        y[j] = make_float2(p.x + sigma * g.x, p.y + sigma * g.y);
      }
    }
    // the next step's symbols, before this step's stores
    if (it + 1 < kAwgnSteps) raw = load_syms(it + 1);
  };
  // Whole wave steps to an aligned output: a wave's 384 noisy symbols go through LDS so each of its three store
  // instructions writes 1 KB. (Their own loop: with the per-symbol stores of the other steps in the same loop,
  // the compiler's wait for the next step's symbols had to cover this step's stores as well.)
  // Step 0 is peeled off the loop, so that the loop is entered as its back edge enters it -- the next symbols' two
  // loads, then the three stores -- and the wait for the symbols leaves the stores in flight.
  auto fast_step = [&](int it) {
    const uint64_t ws = wave_first(it);  // wave's first
    float2 y[kAwgnSym];
    step_outputs(it, y);
#pragma unroll
    for (int q = 0; q < kAwgnSym / 2; ++q) {
      st[lane * 3 + q] = make_float4(y[2 * q].x, y[2 * q].y, y[2 * q + 1].x, y[2 * q + 1].y);
    }
    wave_sync();
    float4* __restrict__ o = reinterpret_cast<float4*>(out + ws);
#pragma unroll
    for (int q = 0; q < kAwgnSym / 2; ++q) o[q * 64 + lane] = st[q * 64 + lane];
    wave_sync();  // the next step's LDS writes come after every lane's reads
    if constexpr (DEMOD) {  // the lane's six decisions: three 2-byte stores (s even, dec 2-byte aligned)
      uint32_t d[kAwgnSym];
      decide6(y, d);
      uint16_t* __restrict__ d2 = reinterpret_cast<uint16_t*>(dec + ws + (uint64_t)kAwgnSym * lane);
#pragma unroll
      for (int q = 0; q < kAwgnSym / 2; ++q) d2[q] = (uint16_t)(d[2 * q] | (d[2 * q + 1] << 8));
    }
  };
  const bool dec_even = !DEMOD || (reinterpret_cast<uintptr_t>(dec) & 1u) == 0;
  auto fast = [&](int it) { return aligned && dec_even && wave_first(it) + kAwgnWaveSyms <= n; };  // wave-uniform
  int it = 0;
  if (fast(0)) {
    fast_step(0);
#pragma unroll 1
    for (it = 1; it < kAwgnSteps && fast(it); ++it) fast_step(it);
  }
  // the rest (the input's last, partial wave step; an output only 8-byte aligned): one store a symbol
#pragma unroll 1
  for (; it < kAwgnSteps; ++it) {
    const uint64_t ws = wave_first(it);
    if (ws >= n) break;
    const uint64_t s = ws + (uint64_t)kAwgnSym * lane;  // this lane's first symbol (a multiple of 6)
    float2 y[kAwgnSym];
    step_outputs(it, y);
    uint32_t d[kAwgnSym] = {};
    if constexpr (DEMOD) decide6(y, d);
#pragma unroll
    for (int j = 0; j < kAwgnSym; ++j) {
      if (s + j < n) {
        out[s + j] = y[j];
        if constexpr (DEMOD) dec[s + j] = (uint8_t)d[j];
      }
    }
  }
}


// TYPE 0: rectangular table (per-axis fast path); TYPE 1: circular table (per-cell candidate lists).
// Both fall back to the exhaustive search for inputs their fast path does not cover.
template <int TYPE>
__global__ __launch_bounds__(kCBlock) void k_c256_demod(C256Streams st, uint32_t n) {
  // the rectangular levels, padded with +inf (demod_rect_fast), at the start of the table's LDS block: their
  // reads then need no base add (ds_read2_b32 offsets reach 1 KB)
  __shared__ float2 tab_lev[20 + 256];
  float* const lxp = reinterpret_cast<float*>(tab_lev);
  float* const lyp = lxp + 20;
  float2* const tab = tab_lev + 20;
  // the circular cell lists: an LDS image of g_circ_cells (cell words and the distinct lists)
  __shared__ uint4 ccells[TYPE == 0 ? 1 : sizeof(CircCells) / 16];
  const uint16_t* cword = reinterpret_cast<const CircCells*>(ccells)->cell;
  const uint8_t* clists = reinterpret_cast<const CircCells*>(ccells)->lists;
  // circular full tiles: the tile's decisions, and per wave the symbols whose search is not finished
  // after the first four candidates (see below)
  __shared__ uint16_t otile[TYPE == 0 ? 1 : kCBlock * kCSym / 2];
  __shared__ uint16_t cq[TYPE == 0 ? 1 : kCBlock / 64][TYPE == 0 ? 1 : 64 * kCSym];
  const float2* tsrc = c_qpsk256_tables[TYPE];
  for (uint32_t i = threadIdx.x; i < 256; i += kCBlock) tab[i] = tsrc[i];
  if (TYPE == 0 && threadIdx.x < 18) {
    const int k = (int)threadIdx.x - 1;
    lxp[threadIdx.x] = (k < 0 || k > 15) ? INFINITY : tsrc[k * 16].x;
    lyp[threadIdx.x] = (k < 0 || k > 15) ? INFINITY : tsrc[k].y;
  }
  if (TYPE != 0 && g_circ_cells.R > 0.0f) {  // the circular candidate lists, into LDS
    // 16-byte copies, all issued before the first LDS store (22.5 KB: six loads a lane; a per-entry
    // 2-byte copy loop waited on each load in turn and cost ~5 % of the kernel)
    constexpr uint32_t kWords = sizeof(CircCells) / 16, kFull = kWords / kCBlock;
    const uint4* src = reinterpret_cast<const uint4*>(&g_circ_cells);
    uint4 w[kFull], wt = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t it = kFull * kCBlock + threadIdx.x;
#pragma unroll
    for (uint32_t k = 0; k < kFull; ++k) w[k] = src[k * kCBlock + threadIdx.x];
    if (it < kWords) wt = src[it];
#pragma unroll
    for (uint32_t k = 0; k < kFull; ++k) ccells[k * kCBlock + threadIdx.x] = w[k];
    if (it < kWords) ccells[it] = wt;
  }
  __syncthreads();
  const float2* __restrict__ in = reinterpret_cast<const float2*>(st.in[blockIdx.y]);
  uint8_t* __restrict__ out = reinterpret_cast<uint8_t*>(st.out[blockIdx.y]);
  float lim = -1.0f, scale = 0.0f, cR = 0.0f, inv_cs = 0.0f;
  if constexpr (TYPE == 0) {
    const float a = tab[255].x;  // rectangular: (15 - 7.5) / 7.5 * a == a exactly
    scale = 7.5f / a;
    // the fast path needs a finite, non-zero amplitude (else every symbol takes the exhaustive search)
    lim = isfinite(scale) ? 4.0f * fabsf(a) : -1.0f;
  } else {
    cR = g_circ_cells.R;
    inv_cs = g_circ_cells.inv_cs;
  }
  auto demod = [&](float2 r) -> uint32_t {
    if constexpr (TYPE == 0) {
      uint32_t k;
      if (demod_rect_quick(r, lim, scale, k)) return k;
      k = demod_rect_fast(lxp, lyp, r, lim, scale);
      return k < 256u ? k : demod_exhaustive(tab, r);
    } else {
      const float fx = (r.x + cR) * inv_cs, fy = (r.y + cR) * inv_cs;
      if (cR > 0.0f && fx >= 0.0f && fy >= 0.0f && fx < (float)kCellGrid && fy < (float)kCellGrid) {
        const uint32_t wc = cword[(int)fy * kCellGrid + (int)fx], len = wc >> 12;
        if (len == 1u) return wc & 0xfffu;  // a one-point cell: no distance needed
        const uint32_t b = wc & 0xfffu, e = b + len;
        float best = INFINITY, second = INFINITY;
        uint32_t idx = 0;
        // four candidates per step with independent LDS loads; slots past the list end repeat its
        // last entry (a duplicate of an entry already ranked: skipped for the runner-up)
        for (uint32_t m = b; m < e; m += 4) {
          uint32_t k[4];
          float2 pt[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) k[j] = clists[m + j < e ? m + j : e - 1];
#pragma unroll
          for (int j = 0; j < 4; ++j) pt[j] = tab[k[j]];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = (j == 0 || m + j < e) ? sqdist(r, pt[j]) : INFINITY;
            if (d < best) {
              second = best;
              best = d;
              idx = k[j];
            } else if (d < second) {
              second = d;
            }
          }
        }
        if (second > tie_threshold(best)) return idx;
        // near-tie: the list (ascending indices, every point that can win in the cell) ranked by
        // cuCabsf with strict '<', as the reference's loop
        best = INFINITY;
        idx = 0;
        for (uint32_t m = b; m < e; ++m) {
          const uint32_t k = clists[m];
          const float d = ref_dist(r, tab[k]);
          if (d < best) {
            best = d;
            idx = k;
          }
        }
        return idx;
      }
      return demod_exhaustive(tab, r);
    }
  };
  // circular, first step: a cell whose candidate list holds a single point decides the symbol without
  // any distance; false for longer lists and outside the grid
  auto circ_first = [&](float2 r, uint32_t& idx) -> bool {
    const float fx = (r.x + cR) * inv_cs, fy = (r.y + cR) * inv_cs;
    if (!(cR > 0.0f && fx >= 0.0f && fy >= 0.0f && fx < (float)kCellGrid && fy < (float)kCellGrid)) return false;
    const uint32_t wc = cword[(int)fy * kCellGrid + (int)fx];
    idx = wc & 0xffu;  // the point of a one-point cell; the low byte of an offset otherwise (overwritten)
    return (wc >> 12) == 1u;
  };
  // grid-stride over 4096-symbol tiles, so the LDS tables are staged once per workgroup
  const uint32_t tiles = (uint32_t)((n + (uint64_t)kCBlock * kCSym - 1) / ((uint64_t)kCBlock * kCSym));
  const bool aligned = (reinterpret_cast<uintptr_t>(in) & 15u) == 0 && (reinterpret_cast<uintptr_t>(out) & 1u) == 0;
  // rectangular: one tile per workgroup (the launcher starts `tiles` workgroups), so the loop ends after
  // its first pass and nothing stays live around it (91 -> 79 VGPRs); circular: grid-stride, so the cell
  // lists are staged into LDS once per workgroup
  for (uint32_t tile = blockIdx.x; tile < tiles; tile += (TYPE == 0 ? tiles : gridDim.x)) {
    const uint64_t base = (uint64_t)tile * kCBlock * kCSym;
    if (TYPE == 1 && aligned && base + kCBlock * kCSym <= n) {
      // Circular full tile. The candidate lists average 1.6 entries but the longest list in a wave is
      // 8-9, so walking each symbol's list in lockstep leaves most lanes idle. Here every symbol first
      // looks up its cell (single-point cells are decided there); the wave's other symbols go to a
      // wave queue in LDS, which its 64 lanes then drain one symbol each (whole list or exhaustive).
      const float4* src = reinterpret_cast<const float4*>(in + base);
      float4 v[kCSym / 2];
#pragma unroll
      for (int q = 0; q < kCSym / 2; ++q) v[q] = src[q * kCBlock + threadIdx.x];
      const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
      uint16_t* qw = cq[TYPE == 0 ? 0 : w];
      uint32_t qn = 0;  // wave-uniform
#pragma unroll
      for (int q = 0; q < kCSym / 2; ++q) {
        const uint32_t pair = q * kCBlock + threadIdx.x;
        uint32_t i0 = 0, i1 = 0;
        const bool d0 = circ_first(make_float2(v[q].x, v[q].y), i0);
        const bool d1 = circ_first(make_float2(v[q].z, v[q].w), i1);
        otile[pair] = (uint16_t)(i0 | (i1 << 8));
        const uint64_t m0 = __ballot(!d0), m1 = __ballot(!d1);
        const uint64_t below = (1ull << lane) - 1ull;
        if (!d0) qw[qn + __popcll(m0 & below)] = (uint16_t)(2u * pair);
        qn += (uint32_t)__popcll(m0);
        if (!d1) qw[qn + __popcll(m1 & below)] = (uint16_t)(2u * pair + 1u);
        qn += (uint32_t)__popcll(m1);
      }
      wave_sync();  // the queue and the first-step decisions come from other lanes of the wave
      uint8_t* ob = reinterpret_cast<uint8_t*>(otile);
      for (uint32_t i = lane; i < qn; i += 64) {
        const uint32_t pos = qw[i];
        ob[pos] = (uint8_t)demod(in[base + pos]);
      }
      wave_sync();
      uint16_t* dst = reinterpret_cast<uint16_t*>(out + base);
#pragma unroll
      for (int q = 0; q < kCSym / 2; ++q) dst[q * kCBlock + threadIdx.x] = otile[q * kCBlock + threadIdx.x];
    } else if (aligned && base + kCBlock * kCSym <= n) {
      // full, aligned tile: lane t of slot q reads symbol pair q * kCBlock + t (coalesced 1 KB loads)
      const float4* src = reinterpret_cast<const float4*>(in + base);
      uint16_t* dst = reinterpret_cast<uint16_t*>(out + base);
      float4 v[kCSym / 2];
#pragma unroll
      for (int q = 0; q < kCSym / 2; ++q) v[q] = src[q * kCBlock + threadIdx.x];
#pragma unroll
      for (int q = 0; q < kCSym / 2; ++q) {
        const uint32_t i0 = demod(make_float2(v[q].x, v[q].y));
        const uint32_t i1 = demod(make_float2(v[q].z, v[q].w));
        dst[q * kCBlock + threadIdx.x] = (uint16_t)(i0 | (i1 << 8));
      }
    } else {
      // last tile or misaligned pointers: one symbol at a time, thread t owning symbols s0 .. s0 + 15
      const uint64_t s0 = base + (uint64_t)threadIdx.x * kCSym;
      for (int k = 0; k < kCSym; ++k) {
        if (s0 + k < n) out[s0 + k] = (uint8_t)demod(in[s0 + k]);
      }
    }
  }
}

// circular demodulation workgroups per stream (grid-stride): 4 resident per CU x 256 CUs (37 KB LDS)
constexpr uint32_t kCircBlocks = 1024;

static hipError_t c256_launch(bool modulate, const C256Streams& st, int nstreams, uint32_t n, uint32_t type,
                              int32_t device, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  for (int s = 0; s < nstreams; ++s) {
    if (st.in[s] == nullptr || st.out[s] == nullptr) return hipErrorInvalidValue;
  }
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  // in 64 bits: n + kCSym - 1 wraps a uint32_t for n near 2^32 (numSymbols is uint32_t)
  const uint32_t blocks = (uint32_t)ceil_div<uint64_t>(ceil_div<uint64_t>(n, kCSym), kCBlock);
  const dim3 grid(blocks, (uint32_t)nstreams);
  if (modulate) {
    k_c256_mod<<<grid, dim3(kCBlock), 0, stream>>>(st, n, type);
  } else {
    // rectangular: one workgroup per tile; circular: one resident round of workgroups (cell lists,
    // decision tile and wave queues take 37 KB of LDS, 4 workgroups per CU) striding over the tiles
    const dim3 dgrid(type == 0 ? blocks : std::min<uint32_t>(blocks, kCircBlocks), (uint32_t)nstreams);
    if (type == 0) {
      k_c256_demod<0><<<dgrid, dim3(kCBlock), 0, stream>>>(st, n);
    } else {
      k_c256_demod<1><<<dgrid, dim3(kCBlock), 0, stream>>>(st, n);
    }
  }
  return launch_status();
}

static constexpr float kPiF = 3.14159265358979323846f;

// Host construction, float arithmetic in the reference's evaluation order.
static void build_table(uint32_t type, float amplitude, float2* t) {
  if (type == 0) {
    for (int i = 0; i < 16; ++i) {
      for (int q = 0; q < 16; ++q) {
        const float I = ((float)i - 7.5f) / 7.5f * amplitude;
        const float Q = ((float)q - 7.5f) / 7.5f * amplitude;
        t[i * 16 + q] = make_float2(I, Q);
      }
    }
    return;
  }
  static const int kPoints[8] = {1, 8, 16, 24, 32, 40, 48, 56};
  static const float kRadii[8] = {0.0f, 0.3f, 0.6f, 0.85f, 1.1f, 1.35f, 1.6f, 1.85f};
  int idx = 0;
  for (int c = 0; c < 8 && idx < 256; ++c) {
    const int points = kPoints[c] < 256 - idx ? kPoints[c] : 256 - idx;
    const float radius = kRadii[c] * amplitude;
    for (int p = 0; p < points && idx < 256; ++p) {
      const float angle = 2.0f * kPiF * (float)p / (float)points + ((float)c * 0.5f);
      t[idx++] = make_float2(radius * cosf(angle), radius * sinf(angle));
    }
  }
  while (idx < 256) {
    const float angle = 2.0f * kPiF * (float)idx / 256.0f;
    const float radius = amplitude * 0.95f;
    t[idx] = make_float2(radius * cosf(angle), radius * sinf(angle));
    ++idx;
  }
}

// Candidate lists for the circular table (see CircCells). Distances in double on the float table.
static bool build_cells(const float2* t, CircCells* cc) {
  double rmax = 0.0;
  for (int i = 0; i < 256; ++i) rmax = std::max(rmax, std::hypot((double)t[i].x, (double)t[i].y));
  cc->R = 0.0f;
  if (!(rmax > 0.0) || !std::isfinite(rmax)) return true;  // degenerate table: exhaustive search
  const float R = (float)(rmax * kCellSpan);
  const float inv_cs = (float)kCellGrid / (2.0f * R);
  const double cs = 1.0 / (double)inv_cs;
  const double margin = 1e-4 * rmax;  // >> float rounding of positions and distances
  int n = 0;
  std::map<std::vector<uint8_t>, int> seen;  // distinct lists -> offset
  std::vector<uint8_t> list;
  for (int iy = 0; iy < kCellGrid; ++iy) {
    for (int ix = 0; ix < kCellGrid; ++ix) {
      const double x0 = -(double)R + ix * cs, x1 = x0 + cs, y0 = -(double)R + iy * cs, y1 = y0 + cs;
      double bound2 = INFINITY;  // smallest worst-case squared distance of a point over the cell
      for (int q = 0; q < 256; ++q) {
        const double dx = std::max(std::fabs(t[q].x - x0), std::fabs(t[q].x - x1));
        const double dy = std::max(std::fabs(t[q].y - y0), std::fabs(t[q].y - y1));
        bound2 = std::min(bound2, dx * dx + dy * dy);
      }
      const double bound = std::sqrt(bound2) + margin;
      const double lim2 = bound * bound;
      list.clear();
      for (int p = 0; p < 256; ++p) {
        const double dx = std::max({x0 - t[p].x, 0.0, t[p].x - x1});
        const double dy = std::max({y0 - t[p].y, 0.0, t[p].y - y1});
        if (dx * dx + dy * dy <= lim2) list.push_back((uint8_t)p);
      }
      const int len = (int)list.size();  // >= 1: the point defining the bound is always listed
      if (len < 1 || len > 15) return true;  // does not fit the cell word: keep the exhaustive search
      int field = list[0];
      if (len > 1) {
        auto it = seen.find(list);
        if (it == seen.end()) {
          if (n + len > kCellListBytes) return true;  // does not fit: keep the exhaustive search
          std::copy(list.begin(), list.end(), cc->lists + n);
          it = seen.emplace(list, n).first;
          n += len;
        }
        field = it->second;
      }
      cc->cell[iy * kCellGrid + ix] = (uint16_t)((len << 12) | field);
    }
  }
  cc->R = R;
  cc->inv_cs = inv_cs;
  return true;
}

}  // namespace gsdr

using gsdr::C256Streams;

GSDR_C_LINKAGE hipError_t gsdrQpsk256InitConstellation(uint32_t constellationType, float amplitude,
                                                       int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  gsdr::DeviceScope scope(cudaDevice);
  if (scope.status() != hipSuccess) return scope.status();
  float2 table[256];
  gsdr::build_table(constellationType, amplitude, table);
  const size_t offset = (constellationType == 0 ? 0 : 1) * sizeof(table);
  hipError_t st = hipMemcpyToSymbolAsync(HIP_SYMBOL(gsdr::c_qpsk256_tables), table, sizeof(table), offset,
                                         hipMemcpyHostToDevice, cudaStream);
  if (st != hipSuccess) return st;
  static thread_local gsdr::CircCells cells;  // host staging (~38 KiB): waited for below
  if (constellationType != 0) {
    try {
      gsdr::build_cells(table, &cells);
    } catch (...) {  // allocation failure: no lookup, the exhaustive search stays exact
      cells.R = 0.0f;
    }
    st = hipMemcpyToSymbolAsync(HIP_SYMBOL(gsdr::g_circ_cells), &cells, sizeof(cells), 0, hipMemcpyHostToDevice,
                                cudaStream);
  }
  // the host table lives on this stack frame: wait for the copies before returning -- on every path
  // once the first copy was issued, so a failed second copy cannot leave the first reading a dead frame
  const hipError_t sync = hipStreamSynchronize(cudaStream);
  return st != hipSuccess ? st : sync;
}

GSDR_C_LINKAGE hipError_t gsdrQpsk256Modulate(const uint8_t* inputBytes, hipFloatComplex* output, uint32_t numSymbols,
                                              float amplitude, uint32_t constellationType, int32_t cudaDevice,
                                              hipStream_t cudaStream) GSDR_NO_EXCEPT {
  (void)amplitude;  // scale is fixed by InitConstellation, as in the reference (qpsk256.cu:74-101)
  C256Streams st{};
  st.in[0] = inputBytes;
  st.out[0] = output;
  return gsdr::c256_launch(true, st, 1, numSymbols, constellationType, cudaDevice, cudaStream);
}

namespace gsdr {
// gsdrxQpsk256ModulateAwgn, and with dec != nullptr the fused round trip of gsdrxQpsk256ModulateAwgnDemodulate
// (rectangular table only; the caller checks)
static hipError_t mod_awgn_launch(const uint8_t* inputBytes, hipFloatComplex* output, uint8_t* dec, uint32_t numSymbols,
                                  uint32_t constellationType, float sigma, uint64_t seed, uint64_t firstSymbolIndex,
                                  hipStream_t cudaStream) {
  const uint32_t blocks = (uint32_t)ceil_div<uint64_t>(numSymbols, kAwgnBlockSyms);
  float2* out = reinterpret_cast<float2*>(output);
  const uint64_t blk = firstSymbolIndex / 3u;
  auto launch = [&](auto r3, auto rect, auto demod) {
    constexpr int R3 = decltype(r3)::value;
    constexpr bool RECT = decltype(rect)::value, DEMOD = decltype(demod)::value;
    if (numSymbols < (uint32_t)kAwgnSym) {
      k_c256_mod_awgn<R3, RECT, true, DEMOD><<<dim3(blocks), dim3(kCBlock), 0, cudaStream>>>(
          inputBytes, out, numSymbols, constellationType, sigma, seed, blk, dec);
    } else {
      k_c256_mod_awgn<R3, RECT, false, DEMOD><<<dim3(blocks), dim3(kCBlock), 0, cudaStream>>>(
          inputBytes, out, numSymbols, constellationType, sigma, seed, blk, dec);
    }
  };
  auto by_type = [&](auto r3) {
    if (dec != nullptr) {
      launch(r3, std::false_type{}, std::true_type{});
    } else if constexpr (GSDR_C256_RECT_LEVELS != 0) {
      if (constellationType == 0) {
        launch(r3, std::true_type{}, std::false_type{});
      } else {
        launch(r3, std::false_type{}, std::false_type{});
      }
    } else {
      launch(r3, std::false_type{}, std::false_type{});
    }
  };
  switch (firstSymbolIndex % 3u) {
    case 0:
      by_type(std::integral_constant<int, 0>{});
      break;
    case 1:
      by_type(std::integral_constant<int, 1>{});
      break;
    default:
      by_type(std::integral_constant<int, 2>{});
      break;
  }
  return launch_status();
}
}  // namespace gsdr

GSDR_C_LINKAGE hipError_t gsdrxQpsk256ModulateAwgn(const uint8_t* inputBytes, hipFloatComplex* output,
                                                    uint32_t numSymbols, uint32_t constellationType, float sigma,
                                                    uint64_t seed, uint64_t firstSymbolIndex, int32_t cudaDevice,
                                                    hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (numSymbols == 0) return hipSuccess;
  if (inputBytes == nullptr || output == nullptr || !(sigma >= 0.0f) || !(sigma < INFINITY)) {
    return hipErrorInvalidValue;
  }
  gsdr::DeviceScope scope(cudaDevice);
  if (scope.status() != hipSuccess) return scope.status();
  return gsdr::mod_awgn_launch(inputBytes, output, nullptr, numSymbols, constellationType, sigma, seed, firstSymbolIndex,
                               cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrxQpsk256ModulateAwgnDemodulate(const uint8_t* inputBytes, hipFloatComplex* noisySymbols,
                                                              uint8_t* outputBytes, uint32_t numSymbols,
                                                              uint32_t constellationType, float sigma, uint64_t seed,
                                                              uint64_t firstSymbolIndex, int32_t cudaDevice,
                                                              hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (numSymbols == 0) return hipSuccess;
  if (inputBytes == nullptr || noisySymbols == nullptr || outputBytes == nullptr || !(sigma >= 0.0f) ||
      !(sigma < INFINITY)) {
    return hipErrorInvalidValue;
  }
  if (constellationType != 0) {  // circular table: the two calls (the cell lists do not fit beside the AWGN tables)
    const hipError_t e = gsdrxQpsk256ModulateAwgn(inputBytes, noisySymbols, numSymbols, constellationType, sigma, seed,
                                                  firstSymbolIndex, cudaDevice, cudaStream);
    if (e != hipSuccess) return e;
    return gsdrQpsk256Demodulate(noisySymbols, outputBytes, numSymbols, constellationType, cudaDevice, cudaStream);
  }
  gsdr::DeviceScope scope(cudaDevice);
  if (scope.status() != hipSuccess) return scope.status();
  return gsdr::mod_awgn_launch(inputBytes, noisySymbols, outputBytes, numSymbols, 0, sigma, seed, firstSymbolIndex,
                               cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpsk256Demodulate(const hipFloatComplex* input, uint8_t* outputBytes,
                                                uint32_t numSymbols, uint32_t constellationType, int32_t cudaDevice,
                                                hipStream_t cudaStream) GSDR_NO_EXCEPT {
  C256Streams st{};
  st.in[0] = input;
  st.out[0] = outputBytes;
  return gsdr::c256_launch(false, st, 1, numSymbols, constellationType, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpsk256Modulate4x(const uint8_t* inputBytes0, const uint8_t* inputBytes1,
                                                const uint8_t* inputBytes2, const uint8_t* inputBytes3,
                                                hipFloatComplex* output0, hipFloatComplex* output1,
                                                hipFloatComplex* output2, hipFloatComplex* output3,
                                                uint32_t numSymbols, float amplitude, uint32_t constellationType,
                                                int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  (void)amplitude;
  C256Streams st{};
  st.in[0] = inputBytes0;
  st.in[1] = inputBytes1;
  st.in[2] = inputBytes2;
  st.in[3] = inputBytes3;
  st.out[0] = output0;
  st.out[1] = output1;
  st.out[2] = output2;
  st.out[3] = output3;
  return gsdr::c256_launch(true, st, 4, numSymbols, constellationType, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrQpsk256Demodulate4x(const hipFloatComplex* input0, const hipFloatComplex* input1,
                                                  const hipFloatComplex* input2, const hipFloatComplex* input3,
                                                  uint8_t* outputBytes0, uint8_t* outputBytes1, uint8_t* outputBytes2,
                                                  uint8_t* outputBytes3, uint32_t numSymbols,
                                                  uint32_t constellationType, int32_t cudaDevice,
                                                  hipStream_t cudaStream) GSDR_NO_EXCEPT {
  C256Streams st{};
  st.in[0] = input0;
  st.in[1] = input1;
  st.in[2] = input2;
  st.in[3] = input3;
  st.out[0] = outputBytes0;
  st.out[1] = outputBytes1;
  st.out[2] = outputBytes2;
  st.out[3] = outputBytes3;
  return gsdr::c256_launch(false, st, 4, numSymbols, constellationType, cudaDevice, cudaStream);
}
