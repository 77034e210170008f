// gsdr-mi355x: IIR filter as a true recursive filter (include/gsdr/iir.h; SURVEY.md section 8(f)
// row 4). Replaces reference src/iir.cu, whose kernel restarts every thread's 8-sample chunk from
// zero state (iir.cu:121-127) and ignores the history arguments (iir.cu:213-214).
//
//   y[n] = sum_{i<=P} b[i] x[n-i] - sum_{1<=i<=P} a[i] y[n-i],   P = K - 1
//
// Parallel scan over the linear recursion (state s = (y[n-1], ..., y[n-P])):
//   1. k_iir_chunks<kTails>: the signal is cut into 32-sample chunks (a workgroup stages WG chunks
//      through LDS for coalesced HBM access); each thread filters its chunk from zero output state
//      (the FIR part sees the true previous inputs) and stores the chunk's zero-state tail T_c.
//   2. The true state entering chunk c obeys S_{c+1} = M S_c + T_c, M = the P x P transition over a
//      chunk of the homogeneous recursion (k_iir_setup, with its powers M^(G^k)). That affine
//      recurrence is scanned hierarchically in groups of 64 elements, one wave per group and one
//      element per lane: up-sweep = Hillis-Steele scan within the wave (6 steps with M^(2^s)),
//      whose last lane is the group aggregate for the next level; down-sweep = every element's start
//      state M^r S_group + prefix_(r-1) at once (table of M^r, r < 64, per level).
//   3. k_iir_chunks<kFinal>: each chunk re-runs from its true start state and writes y.
//   4. k_iir_history: the caller's history buffers receive the last P inputs / outputs.
// For P <= 8 level 0's up-sweep runs inside the tails pass and its down-sweep in the final pass; up to
// 2^25 samples the levels above 1 and level 1's down-sweep take one launch (k_iir_scan_upper), so 2^24
// samples run as tails, level-1 up-sweep, upper scan, final: 4 launches.
// State, scan and matrices are double (see Acc below); complex samples with real coefficients are
// two independent recursions sharing M. State dimensions are padded to a compiled P (zero
// coefficients beyond K-1 leave the recursion unchanged).
#include <hip/hip_runtime.h>


#include <algorithm>

#include "gsdr/iir.h"
#include "launch.hpp"

namespace gsdr {
namespace iir {

constexpr int kChunk = 32;  // samples per level-0 chunk (>= the largest P)
constexpr int kGroup = 64;  // scan elements per group = one wave, one element per lane
constexpr int kMaxLevels = 8;

// The recursion state, the scan and the transition matrices are kept in double: the direct form
// amplifies an inconsistent perturbation of its P-sample state by 10^2..10^3 (tests/test_gpu_iir.py),
// and rounding a scanned state to float32 at every chunk boundary is exactly such a perturbation.
// Samples stay float32 in HBM and LDS; only the outputs are rounded.
template <class S>
struct Acc;
template <>
struct Acc<float> {
  using type = double;
};
template <>
struct Acc<float2> {
  using type = double2;
};

__device__ __forceinline__ float zero_s(float) { return 0.0f; }
__device__ __forceinline__ float2 zero_s(float2) { return make_float2(0.0f, 0.0f); }
__device__ __forceinline__ double zero_s(double) { return 0.0; }
__device__ __forceinline__ double2 zero_s(double2) { return make_double2(0.0, 0.0); }
__device__ __forceinline__ double fma_s(double c, double x, double acc) { return fma(c, x, acc); }
__device__ __forceinline__ double2 fma_s(double c, double2 x, double2 acc) {
  return make_double2(fma(c, x.x, acc.x), fma(c, x.y, acc.y));
}
__device__ __forceinline__ double fma_s(double c, float x, double acc) { return fma(c, (double)x, acc); }
__device__ __forceinline__ double2 fma_s(double c, float2 x, double2 acc) {
  return make_double2(fma(c, (double)x.x, acc.x), fma(c, (double)x.y, acc.y));
}
__device__ __forceinline__ double to_acc(float v) { return (double)v; }
__device__ __forceinline__ double2 to_acc(float2 v) { return make_double2(v.x, v.y); }
__device__ __forceinline__ float to_sample(double v) { return (float)v; }
__device__ __forceinline__ float2 to_sample(double2 v) { return make_float2((float)v.x, (float)v.y); }
__device__ __forceinline__ double add_s(double a, double b) { return a + b; }
__device__ __forceinline__ double shfl_up_s(double v, int d) { return __shfl_up(v, d, 64); }
__device__ __forceinline__ double2 shfl_up_s(double2 v, int d) {
  return make_double2(__shfl_up(v.x, d, 64), __shfl_up(v.y, d, 64));
}
__device__ __forceinline__ double2 add_s(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double shfl_xor_s(double v, int d) { return __shfl_xor(v, d, 64); }
__device__ __forceinline__ double2 shfl_xor_s(double2 v, int d) {
  return make_double2(__shfl_xor(v.x, d, 64), __shfl_xor(v.y, d, 64));
}

struct Coeffs {
  const float* b;
  const float* a;
  int K;
};

// coefficient i of a zero-padded array (uniform: the compiler turns these into scalar loads)
// every load unconditional (clamped index, K >= 1), so the coefficient loads issue together instead of one
// round trip each behind a branch
__device__ __forceinline__ double coeff(const float* c, int K, int i) {
  const float v = c[i < K ? i : K - 1];
  return i < K ? (double)v : 0.0;
}

enum ChunkPass : int { kTails = 0, kFinal = 1 };

// x[n] for n >= -P: the input, or the caller's input history (K-1 entries) for n < 0, else zero
template <class S>
__device__ __forceinline__ S x_at(const S* __restrict__ x, const S* __restrict__ xh, int K, int64_t n) {
  if (n >= 0) return x[n];
  return (xh && -1 - n < K - 1) ? xh[-1 - n] : zero_s(S{});
}

// workgroup barrier for LDS-only phases: waits for this wave's LDS accesses, not its global loads
// (__syncthreads would also drain the tile loads in flight)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// matrix product C = A * B (P x P, row-major) by a workgroup: each thread computes entries
template <int P>
__device__ __forceinline__ void mat_mul(const double* __restrict__ A, const double* __restrict__ B,
                                        double* __restrict__ C, int t, int nt) {
  for (int e = t; e < P * P; e += nt) {
    const int i = e / P, j = e % P;
    double acc = 0.0;
#pragma unroll
    for (int l = 0; l < P; ++l) acc = fma(A[i * P + l], B[l * P + j], acc);
    C[e] = acc;
  }
}

// One workgroup prepares the scan's constants:
//   s0        = entry state (double) from the caller's output history, zero-padded to P;
//   T[k][r]   = M_k^r for r in [0, 64), with M_0 the transition over one chunk (column j = state after
//               kChunk steps of y[n] = -sum a[i] y[n-i] from e_j) and M_{k+1} = M_k^64,
// for every level k = 0..levels. Each level's table is built by doubling in `work` (LDS when it fits,
// else the global table itself): T[h] = T[h/2]^2, then T[h + q] = T[h] T[q].
// barrier for the setup workgroup; the device-scope fence is needed only when the table lives in
// global memory (it costs ~1 us, and the doubling rounds need ~50 barriers)
template <bool INLDS>
__device__ __forceinline__ void sync_table() {
  if constexpr (!INLDS) __threadfence();
  __syncthreads();
}

// INLDS (compile time): `work` is the caller's LDS table. Inlined with a compile-time choice, the table
// accesses compile to ds_read / ds_write; a runtime select between LDS and global made every one of
// them a flat access.
template <class S, int P, int NT, bool INLDS>
__device__ __forceinline__ void iir_setup(const Coeffs& cf, const S* __restrict__ yh,
                                          typename Acc<S>::type* __restrict__ s0, double* __restrict__ T, int levels,
                                          double* __restrict__ work) {
  const int t = threadIdx.x;
  const int Pk = cf.K - 1;
  constexpr int PP = P * P;
  if (t < P) s0[t] = (yh && t < Pk) ? to_acc(yh[t]) : zero_s(typename Acc<S>::type{});
  for (int lv = 0; lv <= levels; ++lv) {
    double* __restrict__ W = INLDS ? work : T + (size_t)lv * kGroup * PP;
    if (lv == 0) {
      if (t < P) {  // M_0, column t
        double am[P + 1];
#pragma unroll
        for (int i = 0; i <= P; ++i) am[i] = -coeff(cf.a, cf.K, i);
        double ys[P];
#pragma unroll
        for (int i = 0; i < P; ++i) ys[i] = i == t ? 1.0 : 0.0;
        for (int k = 0; k < kChunk; ++k) {
          double acc = 0.0;
#pragma unroll
          for (int i = 1; i <= P; ++i) acc = fma(am[i], ys[i - 1], acc);
#pragma unroll
          for (int i = P - 1; i > 0; --i) ys[i] = ys[i - 1];
          ys[0] = acc;
        }
#pragma unroll
        for (int i = 0; i < P; ++i) W[PP + i * P + t] = ys[i];
      }
    } else {  // M_lv = M_{lv-1}^64 = (M_{lv-1}^32)^2, from the previous level's table
      const double* Tp = INLDS ? work : T + (size_t)(lv - 1) * kGroup * PP;
      double m2[(PP + NT - 1) / NT];
      int c = 0;
      for (int e = t; e < PP; e += NT, ++c) {
        const int i = e / P, j = e % P;
        double acc = 0.0;
#pragma unroll
        for (int l = 0; l < P; ++l) acc = fma(Tp[32 * PP + i * P + l], Tp[32 * PP + l * P + j], acc);
        m2[c] = acc;
      }
      sync_table<INLDS>();
      c = 0;
      for (int e = t; e < PP; e += NT, ++c) W[PP + e] = m2[c];
    }
    for (int e = t; e < PP; e += NT) W[e] = (e / P == e % P) ? 1.0 : 0.0;
    sync_table<INLDS>();
    for (int h = 2; h < kGroup; h *= 2) {
      mat_mul<P>(W + (h / 2) * PP, W + (h / 2) * PP, W + h * PP, t, NT);
      sync_table<INLDS>();
      for (int w = t; w < (h - 1) * PP; w += NT) {
        const int q = 1 + w / PP, e = w % PP;
        if (h + q < kGroup) {
          const int i = e / P, j = e % P;
          double acc = 0.0;
#pragma unroll
          for (int l = 0; l < P; ++l) acc = fma(W[h * PP + i * P + l], W[q * PP + l * P + j], acc);
          W[(h + q) * PP + e] = acc;
        }
      }
      sync_table<INLDS>();
    }
    if constexpr (INLDS) {  // publish the level's table
      double* Tl = T + (size_t)lv * kGroup * PP;
      for (int e = t; e < kGroup * PP; e += NT) Tl[e] = W[e];
      __syncthreads();
    }
  }
}

// Workgroup of WG threads = WG consecutive chunks = one tile of WG * kChunk samples, staged through
// LDS so HBM sees coalesced loads/stores; thread t runs the recursion over its chunk from the tile
// (chunk stride kChunk + 1 elements: consecutive lanes land on different banks).
template <class S>
struct TileShape {
  static constexpr int WG = 128;
  static constexpr int NC = sizeof(S) / sizeof(float);  // components per sample: one lane each
  static constexpr int CPW = WG / NC;                     // chunks per workgroup
  static constexpr int TS = CPW * kChunk;                 // samples per tile: 33 KB of LDS either way
  static constexpr int STRIDE = kChunk + 1;
  __device__ static int at(int idx) { return idx + idx / kChunk; }
};

struct SetupArgs {
  const void* yh;
  void* s0;
  double* T;
  int levels;
  const void* xh;  // the caller's input history, copied to xh_copy for the final pass
  void* xh_copy;
};

template <int P>
constexpr bool kTableInLds = kGroup * P * P * sizeof(double) <= 32 * 1024;

// Level-0 scan fused into the chunk passes (P <= kFusedMaxP): the tails pass runs the up-sweep of its
// own groups from LDS (no tails round trip through HBM, no separate launch) and the final pass
// derives each chunk's start state itself (the level-0 down-sweep). IIR_FUSED_MAXP=0 at build time
// gives the unfused form (two more launches), kept for side-by-side measurement.
#ifndef IIR_FUSED_MAXP
#define IIR_FUSED_MAXP 8
#endif
constexpr int kFusedMaxP = IIR_FUSED_MAXP;
// Ablation probes for timing only (wrong results; never set in the product build): IIR_PROBE_TAILS bits
// 1 = no transition powers, 2 = no level-0 up-sweep, 4 = no recursion in the tails pass; IIR_PROBE_FINAL
// bits 1 = no start-state prologue, 2 = no recursion in the final pass.
#ifndef IIR_PROBE_TAILS
#define IIR_PROBE_TAILS 0
#endif
#ifndef IIR_PROBE_FINAL
#define IIR_PROBE_FINAL 0
#endif
#if (IIR_PROBE_TAILS || IIR_PROBE_FINAL) && !defined(GSDR_TUNING_PROBES)
#error "IIR_PROBE_TAILS / IIR_PROBE_FINAL produce wrong results (timing ablations): probe builds only"
#endif

struct ScanArgs {
  double* incl;          // level-0 inclusive zero-state prefixes (A[P] per chunk); tails pass writes
  double* aggs;          // level-1 elements (group aggregates), or null when level 0 is the top
  const double* T0;      // M_0^r, r < 64 (final pass)
  const double* gstart;  // level-1 start states (final pass), or null: s0 is the group start
  const double* s0;
  // final pass: the caller's history buffers, written by the last chunk (the pass reads the input history
  // from the tails pass's copy, so no tile reads what the last one overwrites); Pk = K - 1 entries
  float* xh_out;
  float* yh_out;
  int Pk;
};

// Up-sweep of one level-0 group from the workgroup's tails in LDS (loc = the group's 64 elements),
// with the powers M_0^(2^s) in pw[s]: as up_group, same operations.
template <class A, int P>
__device__ __forceinline__ void up_group_fused(const A* __restrict__ loc, uint64_t E, const double* __restrict__ pw,
                                               A* __restrict__ incl, A* __restrict__ aggs, uint64_t g, int r) {
  constexpr int PP = P * P;
  const uint64_t j = g * kGroup + r;
  const uint64_t last = (E - 1 < g * kGroup + kGroup - 1) ? E - 1 - g * kGroup : kGroup - 1;
  A v[P];
#pragma unroll
  for (int i = 0; i < P; ++i) v[i] = j < E ? loc[r * P + i] : zero_s(A{});
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int d = 1 << s;
    const double* __restrict__ Md = pw + s * PP;
    A w[P];
#pragma unroll
    for (int i = 0; i < P; ++i) w[i] = shfl_up_s(v[i], d);
    if (r >= d) {
#pragma unroll
      for (int i = 0; i < P; ++i) {
        A acc = v[i];
#pragma unroll
        for (int l = 0; l < P; ++l) acc = fma_s(Md[i * P + l], w[l], acc);
        v[i] = acc;
      }
    }
  }
  if (j < E) {
#pragma unroll
    for (int i = 0; i < P; ++i) incl[j * P + i] = v[i];
  }
  if (aggs && (uint64_t)r == last) {
#pragma unroll
    for (int i = 0; i < P; ++i) aggs[g * P + i] = v[i];
  }
}

template <class S, int P, int PASS, bool VEC, bool FUSED = false>
__global__ __launch_bounds__(TileShape<S>::WG) void k_iir_chunks(Coeffs cf, const S* __restrict__ x,
                                                                 const S* __restrict__ xh, uint64_t n,
                                                                 const typename Acc<S>::type* __restrict__ starts,
                                                                 typename Acc<S>::type* __restrict__ tails,
                                                                 S* __restrict__ y, SetupArgs setup, ScanArgs sc) {
  using TSh = TileShape<S>;
  using A = typename Acc<S>::type;
  constexpr size_t kTileBytes = sizeof(S) * TSh::CPW * TSh::STRIDE;
  constexpr size_t kTableBytes = kTableInLds<P> ? kGroup * P * P * sizeof(double) : 0;
  __shared__ __attribute__((aligned(16))) char smem[kTileBytes > kTableBytes ? kTileBytes : kTableBytes];
  // fused tails pass: M_0^(2^s), s < 6, and the workgroup's chunk tails
  constexpr int kPow = (FUSED && PASS == kTails) ? 6 * P * P : 1;
  static_assert(!FUSED || TSh::CPW * P * sizeof(A) <= kTileBytes, "tails alias the tile");
  __shared__ double mpow[kPow];
  __shared__ S pre[P];  // x[base - 1 - i], i < P
  S* tile = reinterpret_cast<S*>(smem);
  A* tl = reinterpret_cast<A*>(smem);  // fused tails pass: the chunk tails, once the tile is consumed
  const int t = threadIdx.x;
  if constexpr (PASS == kTails) {
    // the extra FIRST workgroup builds the scan constants while the others compute the tails (as the
    // last one it was dispatched after most tiles and finished after them: ~7 us at the kernel's end)
    if (blockIdx.x == 0) {
      if (setup.xh != nullptr && t < cf.K - 1) static_cast<S*>(setup.xh_copy)[t] = static_cast<const S*>(setup.xh)[t];
      iir_setup<S, P, TSh::WG, kTableInLds<P>>(cf, static_cast<const S*>(setup.yh), static_cast<A*>(setup.s0), setup.T,
                                               setup.levels, reinterpret_cast<double*>(smem));
      return;
    }
  }
  // Workgroup b filters tile b (a register prefetch of the next tile in a persistent grid measured no
  // faster). Barriers wait for LDS only (lds_barrier), so global loads issued before them stay in flight.
  const uint64_t ntiles = (n + TSh::TS - 1) / TSh::TS;
  constexpr int SPV = 16 / sizeof(S);          // samples per 16-byte load
  constexpr int NV = TSh::TS / SPV / TSh::WG;   // 16-byte loads per thread for a whole tile
  constexpr int NC = TSh::NC;
  const int comp = t % NC;
  auto is_whole = [&](uint64_t i) { return VEC && (i + 1) * (uint64_t)TSh::TS <= n; };
  auto load_tile = [&](uint64_t i, float4 (&r)[NV]) {
    const float4* __restrict__ src = reinterpret_cast<const float4*>(x + i * TSh::TS);
#pragma unroll
    for (int k = 0; k < NV; ++k) r[k] = src[k * TSh::WG + t];
  };
  uint64_t ti = PASS == kTails ? blockIdx.x - 1 : blockIdx.x;
  const uint64_t first_ti = ti;
  auto build_pow = [&]() {
    // M_0 (column j = state after kChunk steps of the homogeneous recursion from e_j), then squared:
    // the same operations as iir_setup's T[1], T[2], ..., T[32], so the same doubles
    if (t < P) {
      double am[P + 1];
#pragma unroll
      for (int i = 0; i <= P; ++i) am[i] = -coeff(cf.a, cf.K, i);
      double m[P];
#pragma unroll
      for (int i = 0; i < P; ++i) m[i] = i == t ? 1.0 : 0.0;
      for (int k = 0; k < kChunk; ++k) {
        double acc = 0.0;
#pragma unroll
        for (int i = 1; i <= P; ++i) acc = fma(am[i], m[i - 1], acc);
#pragma unroll
        for (int i = P - 1; i > 0; --i) m[i] = m[i - 1];
        m[0] = acc;
      }
#pragma unroll
      for (int i = 0; i < P; ++i) mpow[i * P + t] = m[i];
    }
    lds_barrier();
    for (int q = 1; q < 6; ++q) {
      mat_mul<P>(mpow + (q - 1) * P * P, mpow + (q - 1) * P * P, mpow + q * P * P, t, TSh::WG);
      lds_barrier();
    }
  };
  double b[P + 1], am[P + 1];
#pragma unroll
  for (int i = 0; i <= P; ++i) {
    b[i] = coeff(cf.b, cf.K, i);
    am[i] = -coeff(cf.a, cf.K, i);
  }
  double* __restrict__ tails_d = reinterpret_cast<double*>(tails);
  // One tile per workgroup (the launcher starts ntiles workgroups): written as a loop that ends after its
  // first pass, so nothing is live across iterations. With `ti += nwg` the compiler kept the coefficients
  // and the fused scan's state live around the loop: 148 VGPRs, 3 waves per SIMD, instead of 66 / 112.
  for (; ti < ntiles; ti = ntiles) {
    const uint64_t base = ti * TSh::TS;
    const uint32_t tlen = n - base < (uint64_t)TSh::TS ? (uint32_t)(n - base) : (uint32_t)TSh::TS;
    const bool whole = is_whole(ti);
    const uint64_t c = ti * TSh::CPW + t / NC;
    const uint64_t n0 = c * kChunk;
    double ys[P];  // component of y[n-1-i]: the chunk's start state
#pragma unroll
    for (int i = 0; i < P; ++i) ys[i] = 0.0;
    // Final pass: the operands of the chunk's start state are loaded BEFORE the tile. Vector loads retire
    // in order, so operands loaded after the tile could only be used once the whole tile had arrived: the
    // start state's FMAs would then sit on the critical path instead of under the tile's load latency.
    constexpr bool kPro = FUSED && PASS == kFinal && !(IIR_PROBE_FINAL & 1);
    constexpr int PP = P * P;
    double mr[kPro ? PP : 1], inc[kPro ? P : 1], sgc[kPro ? P : 1];
    const uint64_t g = c / kGroup;
    const int r = (int)(c % kGroup);
    if constexpr (kPro) {
      // level-0 down-sweep for this chunk: start = M_0^r S_g + prefix_(r-1) (as down_group)
      if (n0 < n) {
        const double* __restrict__ Mr = sc.T0 + (size_t)r * PP;
#pragma unroll
        for (int e = 0; e < PP; ++e) mr[e] = Mr[e];
#pragma unroll
        for (int i = 0; i < P; ++i) inc[i] = r > 0 ? sc.incl[((c - 1) * P + i) * NC + comp] : 0.0;
        const double* __restrict__ sg = sc.gstart ? sc.gstart + g * P * NC : sc.s0;
#pragma unroll
        for (int l = 0; l < P; ++l) sgc[l] = sg[l * NC + comp];
      }
    }
    float4 v[NV];
    if (whole) load_tile(ti, v);  // in flight while the final pass computes the chunk start state

    // the P samples before the tile (the input history for the first tile), loaded beside it
    S pv = zero_s(S{});
    if (t < P) pv = x_at(x, xh, cf.K, (int64_t)base - 1 - t);
    if constexpr (kPro) {
      if (n0 < n) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
          double acc = inc[i];
#pragma unroll
          for (int l = 0; l < P; ++l) acc = fma(mr[i * P + l], sgc[l], acc);
          ys[i] = acc;
        }
      }
    } else if constexpr (PASS == kFinal && !FUSED) {
      if (n0 < n) {
        const double* __restrict__ starts_d = reinterpret_cast<const double*>(starts);
#pragma unroll
        for (int i = 0; i < P; ++i) ys[i] = starts_d[(c * P + i) * NC + comp];
      }
    }
    if (whole) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int idx = (k * TSh::WG + t) * SPV;  // SPV consecutive samples, all in one chunk row
        float* d = reinterpret_cast<float*>(tile + TSh::at(idx));
        d[0] = v[k].x;
        d[1] = v[k].y;
        d[2] = v[k].z;
        d[3] = v[k].w;
      }
    } else {
      for (int idx = t; idx < (int)tlen; idx += TSh::WG) tile[TSh::at(idx)] = x[base + idx];
    }
    if (t < P) pre[t] = pv;
    lds_barrier();
    // component of x[n-1-i] for every chunk, read before any row is overwritten with y
    double xd[P];
    {
      const int lc = t / NC;  // chunk within the tile
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int m = lc * kChunk - 1 - i;  // tile index of x[n0-1-i]; < 0: before the tile
        xd[i] = (double)reinterpret_cast<const float*>(m >= 0 ? tile + TSh::at(m) : pre + (-1 - m))[comp];
      }
    }
    if constexpr (PASS == kFinal) lds_barrier();
    // lane t runs the recursion of component t % NC of chunk t / NC (complex samples with real
    // coefficients are two independent real recursions): scalar double state, twice the lanes
    if (n0 < n) {
      const uint32_t len = n - n0 < (uint64_t)kChunk ? (uint32_t)(n - n0) : (uint32_t)kChunk;
      float* __restrict__ row = reinterpret_cast<float*>(tile + (t / NC) * TSh::STRIDE) + comp;
      // inputs held as doubles (converted once per sample, exact); a whole chunk is fully unrolled
      // so the state shifts are register renames
      // The feedback terms are added oldest first, so only the last FMA (a[1] y[n-1]) waits for the
      // previous step's output: one FMA latency per sample on the recursion's critical path instead of
      // P (the chunk passes are latency-bound).
      auto step = [&](uint32_t k) {
        const double xv = (double)row[k * NC];
        double acc = b[0] * xv;
#pragma unroll
        for (int i = 1; i <= P; ++i) acc = fma(b[i], xd[i - 1], acc);
#pragma unroll
        for (int i = P; i >= 1; --i) acc = fma(am[i], ys[i - 1], acc);
#pragma unroll
        for (int i = P - 1; i > 0; --i) {
          xd[i] = xd[i - 1];
          ys[i] = ys[i - 1];
        }
        xd[0] = xv;
        ys[0] = acc;
        if constexpr (PASS == kFinal) row[k * NC] = (float)acc;  // y replaces x in this chunk's row
      };
      if ((PASS == kTails && (IIR_PROBE_TAILS & 4)) || (PASS == kFinal && (IIR_PROBE_FINAL & 2))) {
      } else if (len == (uint32_t)kChunk) {
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)kChunk; ++k) step(k);
      } else {
        for (uint32_t k = 0; k < len; ++k) step(k);
      }
      if constexpr (PASS == kTails && !FUSED) {
#pragma unroll
        for (int i = 0; i < P; ++i) tails_d[(c * P + i) * NC + comp] = ys[i];
      } else if constexpr (PASS == kFinal) {
        if (n0 + len == n) {
          // the last chunk's state after the call (outputs, then inputs, newest first) into the caller's
          // history buffers (component comp of entry i)
#pragma unroll
          for (int i = 0; i < P; ++i) {
            if (i < sc.Pk) {
              if (sc.yh_out) sc.yh_out[i * NC + comp] = (float)ys[i];
              if (sc.xh_out) sc.xh_out[i * NC + comp] = (float)xd[i];
            }
          }
        }
      }
    }
    if constexpr (PASS == kTails && FUSED) {
      if (!(IIR_PROBE_TAILS & 1) && ti == first_ti) build_pow();
      lds_barrier();  // every lane is done reading the tile
      if (n0 < n) {
#pragma unroll
        for (int i = 0; i < P; ++i) reinterpret_cast<double*>(&tl[(t / NC) * P + i])[comp] = ys[i];
      }
      lds_barrier();
      const int w = t / kGroup;
      if (!(IIR_PROBE_TAILS & 2) && w < TSh::CPW / kGroup) {
        const uint64_t C = (n + kChunk - 1) / kChunk;
        const uint64_t g = ti * (TSh::CPW / kGroup) + w;
        up_group_fused<A, P>(tl + w * kGroup * P, C, mpow, reinterpret_cast<A*>(sc.incl),
                             reinterpret_cast<A*>(sc.aggs), g, t % kGroup);
      }
    }
    if constexpr (PASS == kFinal) {
      lds_barrier();
      if (whole) {
        float4* __restrict__ dst = reinterpret_cast<float4*>(y + base);
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const int idx = (k * TSh::WG + t) * SPV;
          const float* d = reinterpret_cast<const float*>(tile + TSh::at(idx));
          dst[k * TSh::WG + t] = make_float4(d[0], d[1], d[2], d[3]);
        }
      } else {
        for (int idx = t; idx < (int)tlen; idx += TSh::WG) y[base + idx] = tile[TSh::at(idx)];
      }
    }
    lds_barrier();  // the tile's LDS is free for the next one
  }
}

// Up-sweep of group g of one level (one wave, lane r = element g*64 + r): Hillis-Steele over the
// affine composition from zero state, v_r <- v_r + M^(2^s) v_(r-2^s). Lane r's result is the
// zero-state prefix through element r (kept in `incl` for the down-sweep); the group's last lane holds
// the group aggregate for the next level.
template <class A, int P>
__device__ __forceinline__ void up_group(const A* __restrict__ elems, uint64_t E, const double* __restrict__ T,
                                         A* __restrict__ incl, A* __restrict__ aggs, uint64_t g, int r) {
  constexpr int PP = P * P;
  const uint64_t j = g * kGroup + r;
  const uint64_t last = (E - 1 < g * kGroup + kGroup - 1) ? E - 1 - g * kGroup : kGroup - 1;
  A v[P];
#pragma unroll
  for (int i = 0; i < P; ++i) v[i] = j < E ? elems[j * P + i] : zero_s(A{});
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int d = 1 << s;
    const double* __restrict__ Md = T + (size_t)d * PP;
    A w[P];
#pragma unroll
    for (int i = 0; i < P; ++i) w[i] = shfl_up_s(v[i], d);
    if (r >= d) {
#pragma unroll
      for (int i = 0; i < P; ++i) {
        A acc = v[i];
#pragma unroll
        for (int l = 0; l < P; ++l) acc = fma_s(Md[i * P + l], w[l], acc);
        v[i] = acc;
      }
    }
  }
  if (j < E) {
#pragma unroll
    for (int i = 0; i < P; ++i) incl[j * P + i] = v[i];
  }
  if (aggs && (uint64_t)r == last) {
#pragma unroll
    for (int i = 0; i < P; ++i) aggs[g * P + i] = v[i];
  }
}

// Down-sweep of group g: element j = g*64 + r starts in state M^r S_g + prefix_(r-1), with S_g the
// group's start state (group_starts[g], or s0 at the top level) and prefix the up-sweep's inclusive
// zero-state prefix of the previous lane. Overwrites incl with the start states.
template <class A, int P>
__device__ __forceinline__ void down_group(uint64_t E, const double* __restrict__ T, const A* __restrict__ group_starts,
                                           const A* __restrict__ s0, A* __restrict__ incl_starts, uint64_t g, int r) {
  constexpr int PP = P * P;
  const uint64_t j = g * kGroup + r;
  A pre[P], sg[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const A mine = j < E ? incl_starts[j * P + i] : zero_s(A{});
    pre[i] = shfl_up_s(mine, 1);
    sg[i] = group_starts ? group_starts[g * P + i] : s0[i];
  }
  if (j < E) {
    const double* __restrict__ Mr = T + (size_t)r * PP;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      A acc = r > 0 ? pre[i] : zero_s(A{});
#pragma unroll
      for (int l = 0; l < P; ++l) acc = fma_s(Mr[i * P + l], sg[l], acc);
      incl_starts[j * P + i] = acc;
    }
  }
}

// level 0 (many groups): one wave per group
template <class A, int P>
__global__ __launch_bounds__(64) void k_iir_up(const A* __restrict__ elems, uint64_t E, const double* __restrict__ T,
                                               A* __restrict__ incl, A* __restrict__ aggs) {
  up_group<A, P>(elems, E, T, incl, aggs, blockIdx.x, threadIdx.x);
}

template <class A, int P>
__global__ __launch_bounds__(64) void k_iir_down(uint64_t E, const double* __restrict__ T,
                                                 const A* __restrict__ group_starts, A* __restrict__ incl_starts) {
  down_group<A, P>(E, T, group_starts, nullptr, incl_starts, blockIdx.x, threadIdx.x);
}

// The upper levels with at most kRestGroups groups run in ONE single-workgroup launch, up-sweeps then
// down-sweeps (one wave per group, a barrier between levels, workgroup-scope visibility); larger levels
// get one launch each. A single workgroup is latency-bound walking many groups: 128 groups per level
// took 5x longer than a launch per level, and even with each wave scanning 4-8 groups at once (their
// loads issued together) the whole of levels 1..3 for 2^24 samples took 72 us on one CU against ~19 us
// for the per-level launches. Up and down in one launch: 8.9 us instead of 6.2 + 4.9 us.
constexpr int kRestWaves = 16;
constexpr int kRestGroups = 16;
template <class A>
struct Levels {
  A* elems[kMaxLevels + 1];
  A* starts[kMaxLevels + 1];
  const double* T[kMaxLevels + 1];
  uint64_t E[kMaxLevels + 1];
  int levels;
};

template <class A, int P>
__global__ __launch_bounds__(64 * kRestWaves) void k_iir_scan_rest(Levels<A> L, const A* __restrict__ s0, int first) {
  const int w = threadIdx.x / 64, r = threadIdx.x % 64;
  for (int k = first; k <= L.levels; ++k) {
    const uint64_t groups = ceil_div<uint64_t>(L.E[k], kGroup);
    for (uint64_t g = w; g < groups; g += kRestWaves) {
      up_group<A, P>(L.elems[k], L.E[k], L.T[k], L.starts[k], k < L.levels ? L.elems[k + 1] : nullptr, g, r);
    }
    __syncthreads();
  }
  for (int k = L.levels; k >= first; --k) {
    const uint64_t groups = ceil_div<uint64_t>(L.E[k], kGroup);
    for (uint64_t g = w; g < groups; g += kRestWaves) {
      down_group<A, P>(L.E[k], L.T[k], k < L.levels ? L.starts[k + 1] : nullptr, s0, L.starts[k], g, r);
    }
    __syncthreads();
  }
}

// Levels >= 2 up and down plus level 1's down-sweep in ONE launch (E2 <= kUpperE2 level-2 elements:
// 2^25 samples), after level 1's up-sweep (k_iir_up). Every workgroup scans all of level 2 itself (at most 4
// groups of 64, one wave each, in registers and LDS: a few KB from L2) and derives the level-2 start states
// its own level-1 groups need; then wave j down-sweeps level-1 group 4 b + j of its workgroup b. The
// redundant upper scan costs nothing next to what it replaces: the single-workgroup upper-level kernel
// walked levels 2..3 through global memory (one dependent round trip per phase, 8.3 us at 2^24 samples) and
// a separate level-1 down-sweep (or its fold into the final pass's prologue).
constexpr int kUpperWaves = 4;
constexpr uint64_t kUpperE2 = kUpperWaves * kGroup;

template <int P>
__device__ __forceinline__ void mat_vec_acc(const double* __restrict__ M, const double (&x)[P], double (&acc)[P]) {
#pragma unroll
  for (int i = 0; i < P; ++i) {
    double a = acc[i];
#pragma unroll
    for (int l = 0; l < P; ++l) a = fma(M[i * P + l], x[l], a);
    acc[i] = a;
  }
}

// T[k] = M_k^r, r < 64 (setup tables); elems1 = level-1 elements (their inclusive prefixes in starts1 from
// k_iir_up, overwritten with start states), elems2 = level-2 elements (group aggregates of level 1)
template <int P>
__global__ __launch_bounds__(64 * kUpperWaves) void k_iir_scan_upper(uint64_t E1, uint64_t E2, int NC,
                                                                     const double* __restrict__ T1,
                                                                     const double* __restrict__ T2,
                                                                     const double* __restrict__ T3,
                                                                     const double* __restrict__ elems2,
                                                                     const double* __restrict__ s0,
                                                                     double* __restrict__ starts1) {
  constexpr int PP = P * P;
  __shared__ double incl2[kUpperE2][P];      // level-2 zero-state inclusive prefixes within their group
  __shared__ double gstart[kUpperWaves][P];  // level-2 group start states
  const int comp = blockIdx.y;
  const int t = threadIdx.x, r = t % 64, w = t / 64;
  // this wave's level-1 group (= level-2 element) and its own operands, loaded first
  const uint64_t e2 = (uint64_t)blockIdx.x * kUpperWaves + w;
  const uint64_t e1 = e2 * kGroup + r;
  const bool live = e2 < E2 && e1 < E1;
  double mine[P], m1r[PP];
#pragma unroll
  for (int i = 0; i < P; ++i) mine[i] = live ? starts1[(e1 * P + i) * NC + comp] : 0.0;
#pragma unroll
  for (int q = 0; q < PP; ++q) m1r[q] = T1[(size_t)r * PP + q];
  // 1. level 2: every workgroup scans all E2 elements, wave j the group j (one element a lane)
  double v[P];
  const uint64_t j2 = (uint64_t)t;
#pragma unroll
  for (int i = 0; i < P; ++i) v[i] = j2 < E2 ? elems2[(j2 * P + i) * NC + comp] : 0.0;
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int d = 1 << s;
    double u[P];
#pragma unroll
    for (int i = 0; i < P; ++i) u[i] = __shfl_up(v[i], d, 64);
    if (r >= d) mat_vec_acc<P>(T2 + (size_t)d * PP, u, v);
  }
#pragma unroll
  for (int i = 0; i < P; ++i) incl2[t][i] = v[i];
  __syncthreads();
  // 2. the level-2 groups' start states: at most 4, composed in order from s0 (M_3 = M_2^64)
  if (t < P) {
    double sg[P];
#pragma unroll
    for (int i = 0; i < P; ++i) sg[i] = s0[i * NC + comp];
    const int ng = (int)((E2 + kGroup - 1) / kGroup);
    for (int q = 0; q < kUpperWaves; ++q) {
      gstart[q][t] = sg[t];
      if (q + 1 < ng) {
        double nv[P];
#pragma unroll
        for (int i = 0; i < P; ++i) nv[i] = incl2[q * kGroup + kGroup - 1][i];
        mat_vec_acc<P>(T3 + PP, sg, nv);
#pragma unroll
        for (int i = 0; i < P; ++i) sg[i] = nv[i];
      }
    }
  }
  __syncthreads();
  if (!(e2 < E2)) return;
  // 3. this wave's level-2 element start: M_2^r2 S_group + incl2[e2 - 1] (uniform across the wave)
  const int r2 = (int)(e2 % kGroup);
  const int q2 = (int)(e2 / kGroup);
  double s2[P], sg[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    s2[i] = r2 > 0 ? incl2[e2 - 1][i] : 0.0;
    sg[i] = gstart[q2][i];
  }
  mat_vec_acc<P>(T2 + (size_t)r2 * PP, sg, s2);
  // 4. level-1 down-sweep of group e2: element e1 starts in M_1^r S2 + incl1[e1 - 1]
  double st[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const double prev = __shfl_up(mine[i], 1, 64);
    st[i] = r > 0 ? prev : 0.0;
  }
  mat_vec_acc<P>(m1r, s2, st);
  if (live) {
#pragma unroll
    for (int i = 0; i < P; ++i) starts1[(e1 * P + i) * NC + comp] = st[i];
  }
}

// Which formulation a call runs: the multi-pass scan below (the product's only path), or -- in the tuning-probe
// build only -- the single-pass kernel of iir_resident.hpp, chosen per call (gsdrxIirFFSinglePass / CC).
struct PathSel {
  bool single_pass = false;
  uint32_t max_polls = 0;  // the single-pass kernel's bound on every wait
};

#ifdef GSDR_TUNING_PROBES
#include "iir_resident.hpp"

// bit 0: a single-pass tile gave up waiting since the last gsdrxIirSinglePassStatus (per device)
__device__ uint32_t g_res_status;

template <class S, int P>
static hipError_t run_resident(const Coeffs& cf, S* xh, S* yh, const S* x, S* y, uint64_t n, hipStream_t st,
                               uint32_t max_polls) {
  using Sh = res::Shape<S>;
  constexpr int NC = Sh::NC;
  const uint64_t ntiles = ceil_div<uint64_t>(n, Sh::TS);
  const uint64_t nsb = ceil_div<uint64_t>(ntiles, res::kResSB);
  // one block: the tile aggregates, the superblock aggregates (both filled with kResEmpty by the setup
  // kernel), the tables and coefficients
  const uint64_t nagg = (ntiles + nsb) * P * NC;
  const size_t off_tabs = nagg * sizeof(double);
  const size_t off_ticket = off_tabs + (res::res_tab_doubles<P>() + res::res_coef_doubles<P>()) * sizeof(double);
  const size_t bytes = off_ticket + 16;
  void* status = nullptr;
  hipError_t se = hipGetSymbolAddress(&status, HIP_SYMBOL(g_res_status));
  if (se != hipSuccess) return se;
  char* ws = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&ws), bytes, st);
  if (e != hipSuccess) return e;
  res::ResArgs ra{};
  ra.loc = reinterpret_cast<double*>(ws);
  ra.sbagg = ra.loc + ntiles * P * NC;
  double* tabs = reinterpret_cast<double*>(ws + off_tabs);
  ra.tabs = tabs;
  ra.xh_out = reinterpret_cast<float*>(xh);
  ra.yh_out = reinterpret_cast<float*>(yh);
  ra.Pk = cf.K - 1;
  ra.ticket = reinterpret_cast<uint32_t*>(ws + off_ticket);
  ra.status = static_cast<uint32_t*>(status);
  ra.max_polls = max_polls;
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15u) == 0;
  const uint32_t nclear = (uint32_t)std::min<uint64_t>(512, ceil_div<uint64_t>(nagg, 8 * res::kResWG));
  res::k_res_setup<S, P><<<1 + nclear, res::kResWG, 0, st>>>(cf, tabs, reinterpret_cast<uint64_t*>(ws), nagg, ra.ticket);
  if (vec) {
    res::k_iir_resident<S, P, true><<<(uint32_t)ntiles, res::kResWG, 0, st>>>(cf, x, xh, yh, n, y, ra);
  } else {
    res::k_iir_resident<S, P, false><<<(uint32_t)ntiles, res::kResWG, 0, st>>>(cf, x, xh, yh, n, y, ra);
  }
  e = launch_status();
  const hipError_t f = hipFreeAsync(ws, st);
  return e != hipSuccess ? e : f;
}

#endif  // GSDR_TUNING_PROBES

template <class S, int P>
static hipError_t run(const Coeffs& cf, S* xh, S* yh, const S* x, S* y, uint64_t n, hipStream_t st, PathSel ps) {
  if (ps.single_pass) {
#ifdef GSDR_TUNING_PROBES
    // K <= 9 and up to 2^16 tiles (2^29 real / 2^28 complex samples); anything else is refused, not rerouted
    if constexpr (P <= kFusedMaxP) {
      if (ceil_div<uint64_t>(n, res::Shape<S>::TS) <= res::kResMaxTiles)
        return run_resident<S, P>(cf, xh, yh, x, y, n, st, ps.max_polls);
    }
#endif
    return hipErrorNotSupported;
  }
  using A = typename Acc<S>::type;
  const uint64_t C = ceil_div<uint64_t>(n, kChunk);
  // level sizes: E[0] = C chunks, E[k+1] = ceil(E[k] / G) until one group remains
  constexpr uint64_t G = kGroup;
  uint64_t E[kMaxLevels + 1];
  int levels = 0;
  E[0] = C;
  while (E[levels] > G) {
    if (levels == kMaxLevels) return hipErrorInvalidValue;
    E[levels + 1] = ceil_div<uint64_t>(E[levels], G);
    ++levels;
  }
  // workspace: per level the elements (tails / aggregates) and their start states, the matrices,
  // and a copy of the entry state (the history buffers are rewritten at the end)
  size_t off[kMaxLevels + 1][2];
  size_t bytes = 0;
  for (int k = 0; k <= levels; ++k) {
    off[k][0] = bytes;
    bytes += E[k] * P * sizeof(A);
    off[k][1] = bytes;
    bytes += E[k] * P * sizeof(A);
  }
  constexpr bool F = P <= kFusedMaxP;
  // levels >= 2 and level 1's down-sweep in one launch when level 2 fits (k_iir_scan_upper, which reads
  // the powers of M_1, M_2, M_3 from the tables)
  const bool upper = F && levels >= 2 && E[2] <= kUpperE2;
  const size_t off_m = bytes;
  bytes += (size_t)(levels + 1) * kGroup * P * P * sizeof(double);  // T[level][r] = M_level^r
  const size_t off_s0 = bytes;
  bytes += P * sizeof(A);
  const size_t off_xh = bytes;  // the caller's input history, copied by the tails pass for the final pass
  bytes += (P * sizeof(S) + 15) / 16 * 16;
  char* ws = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&ws), bytes, st);
  if (e != hipSuccess) return e;
  auto elems = [&](int k) { return reinterpret_cast<A*>(ws + off[k][0]); };
  auto starts = [&](int k) { return reinterpret_cast<A*>(ws + off[k][1]); };
  auto table = [&](int k) { return reinterpret_cast<double*>(ws + off_m) + (size_t)k * kGroup * P * P; };
  A* s0 = reinterpret_cast<A*>(ws + off_s0);
  S* xh_copy = reinterpret_cast<S*>(ws + off_xh);
  const int K = cf.K;
  const int Pk = K - 1;  // live state components (<= P); the rest stay zero

  constexpr int WG = TileShape<S>::WG;
  const uint64_t ntiles = ceil_div<uint64_t>(n, TileShape<S>::TS);
  if (ntiles >= 0x7fffffffull) return hipErrorInvalidValue;  // one workgroup per tile (k_iir_chunks)
  const uint32_t blocks = (uint32_t)ntiles;
  const SetupArgs sa{yh, s0, table(0), levels, xh, xh_copy};
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15u) == 0;
  // fused: the tails pass leaves level-0 inclusive prefixes in starts(0) and the group aggregates in
  // elems(1); the final pass finishes level 0 itself
  const ScanArgs up_args{reinterpret_cast<double*>(starts(0)), levels > 0 ? reinterpret_cast<double*>(elems(1)) : nullptr,
                         nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  if (vec) {
    k_iir_chunks<S, P, kTails, true, F><<<blocks + 1, WG, 0, st>>>(cf, x, xh, n, nullptr, elems(0), nullptr, sa, up_args);
  } else {
    k_iir_chunks<S, P, kTails, false, F><<<blocks + 1, WG, 0, st>>>(cf, x, xh, n, nullptr, elems(0), nullptr, sa,
                                                                    up_args);
  }
  // levels with more than kRestGroups groups: one launch each; the rest: one single-workgroup launch
  Levels<A> L{};
  for (int k = 0; k <= levels; ++k) {
    L.elems[k] = elems(k);
    L.starts[k] = starts(k);
    L.T[k] = table(k);
    L.E[k] = E[k];
  }
  L.levels = levels;
  const int lowest = F ? 1 : 0;  // levels scanned outside the chunk passes
  int rest = lowest;             // first level handled by the single-workgroup kernels
  while (rest <= levels && ceil_div<uint64_t>(E[rest], kGroup) > (uint64_t)kRestGroups) ++rest;
  const int stop = upper ? 2 : rest;  // with k_iir_scan_upper: level 1's up-sweep, then that kernel
  for (int k = lowest; k < stop; ++k) {
    k_iir_up<A, P><<<(uint32_t)ceil_div<uint64_t>(E[k], kGroup), 64, 0, st>>>(elems(k), E[k], table(k), starts(k),
                                                                             elems(k + 1));
  }
  if constexpr (F) {
    if (upper) {
      const dim3 grid((uint32_t)ceil_div<uint64_t>(E[2], kUpperWaves), TileShape<S>::NC);
      k_iir_scan_upper<P><<<grid, 64 * kUpperWaves, 0, st>>>(
          E[1], E[2], TileShape<S>::NC, table(1), table(2), levels >= 3 ? table(3) : nullptr,
          reinterpret_cast<const double*>(elems(2)), reinterpret_cast<const double*>(s0),
          reinterpret_cast<double*>(starts(1)));
    }
  }
  if (!upper && rest <= levels) k_iir_scan_rest<A, P><<<1, 64 * kRestWaves, 0, st>>>(L, s0, rest);
  for (int k = upper ? 0 : stop - 1; k >= lowest; --k) {
    k_iir_down<A, P><<<(uint32_t)ceil_div<uint64_t>(E[k], kGroup), 64, 0, st>>>(E[k], table(k), starts(k + 1),
                                                                               starts(k));
  }
  // the last chunk writes the caller's history itself (round 4: one launch fewer than a separate history
  // kernel); the input history it reads comes from the tails pass's copy
  const ScanArgs down_args{reinterpret_cast<double*>(starts(0)), nullptr, table(0),
                           levels > 0 ? reinterpret_cast<const double*>(starts(1)) : nullptr,
                           reinterpret_cast<const double*>(s0), reinterpret_cast<float*>(xh),
                           reinterpret_cast<float*>(yh), Pk};
  const S* xh_in = xh ? xh_copy : nullptr;
  if (vec) {
    k_iir_chunks<S, P, kFinal, true, F><<<blocks, WG, 0, st>>>(cf, x, xh_in, n, starts(0), nullptr, y, SetupArgs{},
                                                               down_args);
  } else {
    k_iir_chunks<S, P, kFinal, false, F><<<blocks, WG, 0, st>>>(cf, x, xh_in, n, starts(0), nullptr, y, SetupArgs{},
                                                                down_args);
  }
  e = launch_status();
  const hipError_t f = hipFreeAsync(ws, st);
  return e != hipSuccess ? e : f;
}

template <class S>
static hipError_t entry(const float* b, const float* a, size_t K, S* xh, S* yh, const S* x, S* y, size_t n,
                        int32_t device, hipStream_t st, PathSel ps = {}) {
  if (K < 2 || K > 32) return hipErrorInvalidValue;  // reference limits (iir.cu:229-235)
  if (n == 0) return hipSuccess;
  if (b == nullptr || a == nullptr || x == nullptr || y == nullptr) return hipErrorInvalidValue;
  static_assert(kChunk >= 31, "a chunk must hold the largest state");
  DeviceScope scope(device);
  if (scope.status() != hipSuccess) return scope.status();
  const Coeffs cf{b, a, (int)K};
  const size_t P = K - 1;
  if (P <= 1) return run<S, 1>(cf, xh, yh, x, y, n, st, ps);
  if (P <= 2) return run<S, 2>(cf, xh, yh, x, y, n, st, ps);
  if (P <= 4) return run<S, 4>(cf, xh, yh, x, y, n, st, ps);
  if (P <= 8) return run<S, 8>(cf, xh, yh, x, y, n, st, ps);
  if (P <= 16) return run<S, 16>(cf, xh, yh, x, y, n, st, ps);
  return run<S, 31>(cf, xh, yh, x, y, n, st, ps);
}

}  // namespace iir
}  // namespace gsdr

GSDR_C_LINKAGE hipError_t gsdrIirFF(const float* bCoeffs, const float* aCoeffs, size_t coeffCount, float* inputHistory,
                                    float* outputHistory, const float* input, float* output, size_t numElements,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::iir::entry<float>(bCoeffs, aCoeffs, coeffCount, inputHistory, outputHistory, input, output,
                                 numElements, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrIirCC(const float* bCoeffs, const float* aCoeffs, size_t coeffCount,
                                    hipFloatComplex* inputHistory, hipFloatComplex* outputHistory,
                                    const hipFloatComplex* input, hipFloatComplex* output, size_t numElements,
                                    int32_t cudaDevice, hipStream_t cudaStream) GSDR_NO_EXCEPT {
  return gsdr::iir::entry<float2>(bCoeffs, aCoeffs, coeffCount, reinterpret_cast<float2*>(inputHistory),
                                  reinterpret_cast<float2*>(outputHistory), reinterpret_cast<const float2*>(input),
                                  reinterpret_cast<float2*>(output), numElements, cudaDevice, cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrIirFFCustom(const float* bCoeffs, const float* aCoeffs, size_t coeffCount,
                                          float* inputHistory, float* outputHistory, const float* input, float* output,
                                          size_t numElements, size_t samplesPerThread, int32_t cudaDevice,
                                          hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (samplesPerThread == 0 || samplesPerThread > 32) return hipErrorInvalidValue;  // iir.cu (Custom) limits
  return gsdrIirFF(bCoeffs, aCoeffs, coeffCount, inputHistory, outputHistory, input, output, numElements, cudaDevice,
                   cudaStream);
}

GSDR_C_LINKAGE hipError_t gsdrIirCCCustom(const float* bCoeffs, const float* aCoeffs, size_t coeffCount,
                                          hipFloatComplex* inputHistory, hipFloatComplex* outputHistory,
                                          const hipFloatComplex* input, hipFloatComplex* output, size_t numElements,
                                          size_t samplesPerThread, int32_t cudaDevice,
                                          hipStream_t cudaStream) GSDR_NO_EXCEPT {
  if (samplesPerThread == 0 || samplesPerThread > 32) return hipErrorInvalidValue;
  return gsdrIirCC(bCoeffs, aCoeffs, coeffCount, inputHistory, outputHistory, input, output, numElements, cudaDevice,
                   cudaStream);
}

#ifdef GSDR_TUNING_PROBES
// Tuning-probe build only (libgsdr_probes.so; tools/ and tests/test_gpu_iir_single_pass.py bind them by name):
// gsdrIirFF / gsdrIirCC on the single-pass kernel, chosen per call. maxPolls bounds every wait in polling rounds
// (2^22 is the measured setting; 0 makes every tile that has to wait give up at once, which is how the status
// path is tested); hipErrorNotSupported for K > 9 or more than 2^16 tiles. A give-up is reported by
// gsdrxIirSinglePassStatus, which synchronises the stream and returns hipErrorLaunchFailure (clearing the word)
// when any tile gave up since the last query.
#define GSDR_PROBE_API extern "C" __attribute__((visibility("default")))
GSDR_PROBE_API hipError_t gsdrxIirFFSinglePass(const float* bCoeffs, const float* aCoeffs, size_t coeffCount,
                                               float* inputHistory, float* outputHistory, const float* input,
                                               float* output, size_t numElements, uint32_t maxPolls,
                                               int32_t cudaDevice, hipStream_t cudaStream) noexcept {
  return gsdr::iir::entry<float>(bCoeffs, aCoeffs, coeffCount, inputHistory, outputHistory, input, output,
                                 numElements, cudaDevice, cudaStream,
                                 gsdr::iir::PathSel{true, maxPolls});
}

GSDR_PROBE_API hipError_t gsdrxIirCCSinglePass(const float* bCoeffs, const float* aCoeffs, size_t coeffCount,
                                               hipFloatComplex* inputHistory, hipFloatComplex* outputHistory,
                                               const hipFloatComplex* input, hipFloatComplex* output,
                                               size_t numElements, uint32_t maxPolls, int32_t cudaDevice,
                                               hipStream_t cudaStream) noexcept {
  return gsdr::iir::entry<float2>(bCoeffs, aCoeffs, coeffCount, reinterpret_cast<float2*>(inputHistory),
                                  reinterpret_cast<float2*>(outputHistory), reinterpret_cast<const float2*>(input),
                                  reinterpret_cast<float2*>(output), numElements, cudaDevice, cudaStream,
                                  gsdr::iir::PathSel{true, maxPolls});
}

// hipSuccess when no single-pass tile gave up since the last query, else hipErrorLaunchFailure
GSDR_PROBE_API hipError_t gsdrxIirSinglePassStatus(int32_t cudaDevice, hipStream_t cudaStream) noexcept {
  gsdr::DeviceScope scope(cudaDevice);
  if (scope.status() != hipSuccess) return scope.status();
  uint32_t v = 0;
  hipError_t e = hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(gsdr::iir::g_res_status), sizeof(v), 0,
                                          hipMemcpyDeviceToHost, cudaStream);
  if (e == hipSuccess) e = hipStreamSynchronize(cudaStream);
  if (e != hipSuccess) return e;
  if (v == 0) return hipSuccess;
  const uint32_t z = 0;
  e = hipMemcpyToSymbolAsync(HIP_SYMBOL(gsdr::iir::g_res_status), &z, sizeof(z), 0, hipMemcpyHostToDevice,
                             cudaStream);
  if (e == hipSuccess) e = hipStreamSynchronize(cudaStream);
  return e != hipSuccess ? e : hipErrorLaunchFailure;
}
#endif
