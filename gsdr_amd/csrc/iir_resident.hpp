// gsdr-mi355x: single-pass IIR (K <= 9, up to 2^16 tiles), included by iir.hip in the tuning-probe build only
// (GSDR_TUNING_PROBES: gsdrxIirFFSinglePass / gsdrxIirCCSinglePass of libgsdr_probes.so). It measured slower than
// the multi-pass scan that gsdrIirFF / gsdrIirCC run, so the product library does not
// carry it.
//
// The multi-pass scan of iir.hip reads the input twice (tails pass, final pass) with scan launches between,
// and both chunk passes are latency-bound. Here one launch reads x once and writes y
// once: every workgroup keeps its tile's samples in LDS from the zero-state pass to the final pass and gets
// its entry state from its predecessors' published aggregates (decoupled look-back, Merrill & Garland):
//   1. the tile (kResWG chunks of 32 samples per component, one lane a chunk) is staged into LDS (rows of 33
//      floats, as iir.hip's chunk passes); each lane filters its chunk from zero output state -> its tail;
//   2. an inclusive affine scan of the chunk tails across the workgroup (Hillis-Steele with M0^(2^s), M0 =
//      the transition over one chunk) gives every chunk's zero-entry prefix and the tile's aggregate, which
//      the workgroup publishes (into aggregate arrays the setup kernel fills with a sentinel on every call);
//   3. the tile's entry state: tiles are grouped in superblocks of 256; the last tile of a superblock also
//      publishes the superblock's aggregate. A workgroup waits for the aggregates of the tiles before it in
//      its superblock and of the superblocks before its own, scans each list across its threads (fixed
//      Hillis-Steele trees, so the result does not depend on timing) and composes
//        S_tile = M_T^k S_sb + U_(k-1),  S_sb = M_SB^sb s0 + Q_(sb-1)
//      (k = its index in the superblock, U / Q the inclusive scans, M_T = M0^(chunks a tile), M_SB = M_T^256);
//   4. every chunk starts from M0^e S_tile + prefix_(e-1), the recursion re-runs over the staged tile and y leaves
//      through LDS in coalesced rows.
// Tile numbers come from an atomic ticket taken when a workgroup starts, so a workgroup waits only on tiles
// whose workgroups are already running: the waits cannot deadlock whatever order the hardware dispatches the
// grid in. Every wait is bounded (ResArgs::max_polls rounds): a tile that gives up records it in the device
// status word (gsdrxIirSinglePassStatus turns it into hipErrorLaunchFailure), writes NaN outputs and leaves
// the caller's history buffers alone. The transition matrices and their powers are built once per call by a
// one-workgroup kernel ahead of the tiles (k_res_setup); every tile loads them beside its samples.
#pragma once

namespace res {

constexpr int kResWG = 256;
constexpr uint32_t kResSB = 256;        // tiles per superblock
constexpr uint32_t kResMaxTiles = 256 * kResSB;

template <class S>
struct Shape {
  static constexpr int NC = sizeof(S) / sizeof(float);   // components (one lane each)
  static constexpr int CPT = kResWG / NC;                 // chunks a tile
  static constexpr int TS = CPT * kChunk;                 // samples a tile
  static constexpr int LOGCPT = NC == 1 ? 8 : 7;
  static constexpr int STRIDE = kChunk + 1;               // LDS row stride (floats of one component)
  static constexpr size_t kTileFloats = (size_t)kResWG * STRIDE;  // 256 rows of 33 floats
  __device__ static int at(int idx) { return idx + idx / kChunk; }  // sample idx -> padded slot (in S units)
};

struct ResArgs {
  double* loc;       // [tile][P][NC]: tile aggregates (zero entry), kResEmpty until written
  double* sbagg;     // [superblock][P][NC]: superblock aggregates, likewise
  const double* tabs;  // k_res_setup's tables: gk [kChunk][P], M0^(2^s) (s <= 8), M_T^(2^s), M_SB^(2^s) (s < 8),
                       // then the coefficients as doubles
  float* xh_out;
  float* yh_out;
  int Pk;
  uint32_t* ticket;     // tile ticket counter (zeroed by k_res_setup)
  uint32_t* status;     // device status word: bit 0 set by a tile that gave up waiting
  uint32_t max_polls;   // bound on every wait's polling rounds
};

// Cross-workgroup values (the aggregates). Every XCD has its own L2, not coherent with the others, and
// acquire / release write back and invalidate the whole L2 of the XCD; with hundreds of polls a tile that cost
// more than the filter. So there are no flags: the setup kernel fills the aggregate arrays with kResEmpty (a
// signalling NaN whose low payload bits no float input or arithmetic result can carry), a workgroup writes its
// aggregate with relaxed atomic stores at GSDR_RES_SCOPE (system scope by default -- the setting every
// measurement used; they bypass the non-coherent caching) and a reader polls the values themselves with relaxed
// atomic loads of the same scope until none is kResEmpty: each 8-byte value is written and read whole, so no
// value can be seen half-written, and a write needs no fence or completion wait before the writer moves on.
constexpr uint64_t kResEmpty = 0x7FF4DEAD5EED1234ull;
#ifndef GSDR_RES_SCOPE
#define GSDR_RES_SCOPE __HIP_MEMORY_SCOPE_SYSTEM
#endif

__device__ __forceinline__ void st_co(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, GSDR_RES_SCOPE);
}

// load one value (GSDR_RES_SCOPE, bypassing the non-coherent caching)
__device__ __forceinline__ uint64_t ld_bits(const double* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, GSDR_RES_SCOPE);
}

// oa / ob <- the N values at a / b once none is kResEmpty (either source may be null: nothing to wait for). Each
// round polls only the last value of each source (one load per source while waiting), then reads them whole;
// false after `lim` rounds (never expected: the writers are workgroups that took earlier tickets)
template <int N>
__device__ __forceinline__ bool poll_vals2(const double* a, double (&oa)[N], const double* b, double (&ob)[N],
                                           uint32_t lim) {
  if (!a && !b) {  // nothing to wait for (whatever the bound)
#pragma unroll
    for (int i = 0; i < N; ++i) oa[i] = ob[i] = 0.0;
    return true;
  }
  for (uint32_t it = 0; it < lim; ++it) {
    const bool ra = !a || ld_bits(a + N - 1) != kResEmpty;
    const bool rb = !b || ld_bits(b + N - 1) != kResEmpty;
    if (ra && rb) {
      bool all = true;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const uint64_t va = a ? ld_bits(a + i) : 0, vb = b ? ld_bits(b + i) : 0;
        oa[i] = __builtin_bit_cast(double, va);
        ob[i] = __builtin_bit_cast(double, vb);
        all = all && va != kResEmpty && vb != kResEmpty;
      }
      if (all) return true;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  return false;
}

// wave 0 waits until the last value of each of na vectors at a (and nb at b, stride N doubles, na, nb <= 256)
// is written, then the workgroup barrier: one polling wave, so the co-resident workgroups still computing keep
// their issue slots; false (for every thread) after `lim` rounds
template <int N>
__device__ __forceinline__ bool wave0_wait(const double* a, uint32_t na, const double* b, uint32_t nb, uint32_t lim) {
  bool ok = true;
  if (threadIdx.x < 64 && (na | nb) != 0) {
    const uint32_t lane = threadIdx.x;
    ok = false;
    for (uint32_t it = 0; it < lim; ++it) {
      bool all = true;
#pragma unroll
      for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t j = lane + 64 * r;
        if (j < na) all = all && ld_bits(a + (size_t)j * N + N - 1) != kResEmpty;
        if (j < nb) all = all && ld_bits(b + (size_t)j * N + N - 1) != kResEmpty;
      }
      if (__all(all)) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  return __syncthreads_and(ok);
}

template <int N>
__device__ __forceinline__ bool poll_vals(const double* src, double (&out)[N], uint32_t lim) {
  double dummy[N];
  return poll_vals2<N>(src, out, nullptr, dummy, lim);
}

// v <- M v (P x P row-major M in LDS or global)
template <class V, int P>
__device__ __forceinline__ void mat_vec(const double* __restrict__ M, V (&v)[P]) {
  V r[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    V acc = zero_s(V{});
#pragma unroll
    for (int l = 0; l < P; ++l) acc = fma_s(M[i * P + l], v[l], acc);
    r[i] = acc;
  }
#pragma unroll
  for (int i = 0; i < P; ++i) v[i] = r[i];
}

// v <- M^k v with pw[s] = M^(2^s), k < 2^8 (binary powering: the set bits of k, ascending)
template <class V, int P>
__device__ __forceinline__ void mat_pow_vec(const double* __restrict__ pw, uint32_t k, V (&v)[P]) {
#pragma unroll 1  // unrolled, the compiler loads every power ahead (registers for 8 P x P matrices)
  for (int s = 0; s < 8; ++s) {
    if (k & (1u << s)) mat_vec<V, P>(pw + s * P * P, v);
  }
}

// Inclusive affine scan across the workgroup: element e = threadIdx.x / LS (each lane scans its own vector),
// v_e <- sum_{e' <= e} Mp^(e - e') v_e', pw[s] = Mp^(2^s). Each wave scans its EW = 64 / LS elements by
// Hillis-Steele over lane shuffles; the waves' aggregates go through sc (4 * LS * P values of double), every wave
// folds the aggregates of the waves before it into a carry c (Horner, oldest first) and element j of the wave
// adds Mp^(j + 1) c. The order of operations is fixed, so the result is a pure function of the inputs. Every
// thread must call it. (sc must not be __restrict__: threads write their slots and read others', and restrict
// lets the compiler drop such a store as dead.)
template <class V, int P, int LS>
__device__ __forceinline__ void wg_scan(V (&v)[P], const double* __restrict__ pw, V* sc) {
  constexpr int EW = 64 / LS, LOGEW = LS == 1 ? 6 : 5, PP = P * P;
  static_assert(LS == 1 || LS == 2, "one or two components");
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, comp = lane % LS;
#pragma unroll 1
  for (int s = 0; (1 << s) < EW; ++s) {
    const int dl = (1 << s) * LS;  // lanes between partners
    V u[P];
#pragma unroll
    for (int i = 0; i < P; ++i) u[i] = shfl_up_s(v[i], dl);
    if (lane >= dl) {
      const double* __restrict__ M = pw + s * PP;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        V acc = v[i];
#pragma unroll
        for (int l = 0; l < P; ++l) acc = fma_s(M[i * P + l], u[l], acc);
        v[i] = acc;
      }
    }
  }
  lds_barrier();  // earlier readers of sc are done
  if (lane >= 64 - LS) {
#pragma unroll
    for (int i = 0; i < P; ++i) sc[(w * LS + comp) * P + i] = v[i];
  }
  lds_barrier();
  if (w > 0) {
    V c[P];
#pragma unroll
    for (int i = 0; i < P; ++i) c[i] = sc[comp * P + i];
    for (int wp = 1; wp < w; ++wp) {
      mat_vec<V, P>(pw + LOGEW * PP, c);
#pragma unroll
      for (int i = 0; i < P; ++i) c[i] = add_s(c[i], sc[(wp * LS + comp) * P + i]);
    }
    mat_pow_vec<V, P>(pw, (uint32_t)(lane / LS + 1), c);
#pragma unroll
    for (int i = 0; i < P; ++i) v[i] = add_s(v[i], c[i]);
  }
}

// tot <- sum of v over the workgroup, the same bits on every thread (butterfly within each wave, then the
// four wave sums in a fixed order through sc, 4 * P values of V); every thread must call it
template <class V, int P>
__device__ __forceinline__ void wg_sum(const V (&v)[P], V (&tot)[P], V* sc) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  V r[P];
#pragma unroll
  for (int i = 0; i < P; ++i) r[i] = v[i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int i = 0; i < P; ++i) r[i] = add_s(r[i], shfl_xor_s(r[i], off));
  }
  lds_barrier();  // earlier readers of sc are done
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < P; ++i) sc[w * P + i] = r[i];
  }
  lds_barrier();
#pragma unroll
  for (int i = 0; i < P; ++i) tot[i] = add_s(add_s(add_s(sc[i], sc[P + i]), sc[2 * P + i]), sc[3 * P + i]);
}

// C = A * B (P x P) by the workgroup, then a barrier
template <int P>
__device__ __forceinline__ void sq_step(const double* __restrict__ A, const double* __restrict__ B,
                                        double* __restrict__ C) {
  mat_mul<P>(A, B, C, threadIdx.x, kResWG);
  lds_barrier();
}

// the per-call tables, one workgroup ahead of the tiles (stream order publishes them): gk[k][i] = output k of the
// homogeneous recursion from state e_i (k < kChunk), M0 = the transition over a chunk (column j: the state after
// kChunk steps from e_j) and M0^(2^s) for s <= 8, M_T = M0^(chunks a tile) and M_SB = M_T^256 with their
// powers M^(2^s), s < 8
template <int P>
constexpr int res_coef_doubles() { return 2 * (P + 1); }  // b[0..P], -a[0..P], zero past K
template <int P>
constexpr int res_tab_doubles() { return kChunk * P + 25 * P * P; }

template <class S, int P>
__global__ __launch_bounds__(kResWG) void k_res_setup(Coeffs cf, double* __restrict__ tabs, uint64_t* __restrict__ agg,
                                                     uint64_t nagg, uint32_t* __restrict__ ticket) {
  constexpr int PP = P * P;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;
  if (blockIdx.x > 0) {  // the aggregate arrays to kResEmpty
    for (uint64_t e = (uint64_t)(blockIdx.x - 1) * kResWG + threadIdx.x; e < nagg; e += (uint64_t)(gridDim.x - 1) * kResWG)
      agg[e] = kResEmpty;
    return;
  }
  __shared__ double tl[res_tab_doubles<P>()];
  double* gk = tl;
  double* pw0 = tl + kChunk * P;
  double* pwg = pw0 + 9 * PP;
  const int t = threadIdx.x;
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
      gk[k * P + t] = acc;
    }
#pragma unroll
    for (int i = 0; i < P; ++i) pw0[i * P + t] = m[i];
  }
  lds_barrier();
  for (int s = 1; s <= 8; ++s) sq_step<P>(pw0 + (s - 1) * PP, pw0 + (s - 1) * PP, pw0 + s * PP);
  for (int e = t; e < PP; e += kResWG) pwg[e] = pw0[Shape<S>::LOGCPT * PP + e];
  lds_barrier();
  for (int s = 1; s < 8; ++s) sq_step<P>(pwg + (s - 1) * PP, pwg + (s - 1) * PP, pwg + s * PP);
  sq_step<P>(pwg + 7 * PP, pwg + 7 * PP, pwg + 8 * PP);  // M_SB = M_T^256
  for (int s = 9; s < 16; ++s) sq_step<P>(pwg + (s - 1) * PP, pwg + (s - 1) * PP, pwg + s * PP);
  for (int e = t; e < res_tab_doubles<P>(); e += kResWG) tabs[e] = tl[e];
  if (t <= P) {
    tabs[res_tab_doubles<P>() + t] = coeff(cf.b, cf.K, t);
    tabs[res_tab_doubles<P>() + P + 1 + t] = -coeff(cf.a, cf.K, t);
  }
}

#ifdef GSDR_IIR_RES_TIMING
#define GSDR_RES_TS0() uint64_t ts_[12] = {}; ts_[0] = wall_clock64();
#define GSDR_RES_TS(i) ts_[i] = wall_clock64();
#else
#define GSDR_RES_TS0()
#define GSDR_RES_TS(i)
#endif
// waves a SIMD for the register budget: 4 fit P <= 4 without spills (LDS holds 4 tiles a CU); P = 8 needs
// ~230-250 VGPRs, 2 waves
template <class S, int P>
constexpr int res_waves() {
  return sizeof(S) == 4 ? (P <= 4 ? 4 : 2) : (P <= 4 ? 4 : 2);
}

template <class S, int P, bool VEC>
__global__ __launch_bounds__(kResWG) __attribute__((amdgpu_waves_per_eu(res_waves<S, P>()))) void k_iir_resident(Coeffs cf, const S* __restrict__ x, const S* __restrict__ xh,
                                                        const S* __restrict__ yh, uint64_t n, S* __restrict__ y,
                                                        ResArgs ra) {
  using Sh = Shape<S>;
  using A = typename Acc<S>::type;
  constexpr int NC = Sh::NC, PP = P * P;
  constexpr int SPV = 16 / sizeof(S);               // samples per 16-byte load
  constexpr int NV = Sh::TS / SPV / kResWG;         // 16-byte loads a thread
  // LDS: the tile (x, then y, for the whole kernel), the scans' scratch, M0^(2^s) (s <= 8), the
  // superblock-level tables, small vectors. (Holding the chunk in registers instead let the compiler convert
  // and scale all 32 samples ahead of the recursion: 210-256 VGPRs.)
  __shared__ __attribute__((aligned(16))) float tile[Sh::kTileFloats];
  __shared__ __attribute__((aligned(16))) double scd[4 * NC * P];  // the scans' wave aggregates
  __shared__ __attribute__((aligned(16))) double bnd[4 * NC * P];  // each wave's last chunk prefixes
  __shared__ double tab[res_tab_doubles<P>()];  // k_res_setup's tables
  const double* gk = tab;                        // gk[k][i]: output k of the homogeneous recursion from e_i
  const double* pw0 = tab + kChunk * P;          // M0^(2^s), s = 0..8
  const double* pwg = pw0 + 9 * PP;              // M_T^(2^s), M_SB^(2^s), s < 8
  __shared__ A sv[2][P];           // the tile's entry state, s0
  __shared__ S pre[P];             // x[base - 1 - i], i < P
  const int t = threadIdx.x;
  GSDR_RES_TS0();
  const int comp = t % NC;
  const int lc = t / NC;  // chunk within the tile
  // the tile this workgroup filters: the next ticket (not blockIdx.x), so every tile it waits for belongs to a
  // workgroup that is already running, whatever order the grid is dispatched in
  __shared__ uint32_t tile_sh;
  if (t == 0) tile_sh = atomicAdd(ra.ticket, 1u);
  __syncthreads();
  const uint32_t tile_id = tile_sh;
  const uint64_t base = (uint64_t)tile_id * Sh::TS;
  const uint64_t ntiles = (n + Sh::TS - 1) / Sh::TS;
  const uint32_t tlen = n - base < (uint64_t)Sh::TS ? (uint32_t)(n - base) : (uint32_t)Sh::TS;
  const bool whole = VEC && tlen == (uint32_t)Sh::TS;

  // 1. loads first (in flight while the M0 powers are built), then the entry state s0 and the P samples
  //    before the tile: every workgroup reads the caller's histories before publishing anything, so the last
  //    tile (which waits for every aggregate) rewrites them only after all reads
  // the tile's loads first, then the tables and the P samples before the tile and the entry state (raw until
  // the tile has arrived); the coefficients come as doubles from the setup kernel (scalar loads)
  float4 v4[NV];
  if (whole) {
    const float4* __restrict__ src = reinterpret_cast<const float4*>(x + base);
#pragma unroll
    for (int k = 0; k < NV; ++k) v4[k] = src[k * kResWG + t];
  }
  constexpr int NTAB = res_tab_doubles<P>(), NTR = (NTAB + kResWG - 1) / kResWG;
  double tv[NTR];
#pragma unroll
  for (int r = 0; r < NTR; ++r) {
    const int e = r * kResWG + t;
    tv[r] = e < NTAB ? ra.tabs[e] : 0.0;
  }
  double b[P + 1], am[P + 1];
#pragma unroll
  for (int i = 0; i <= P; ++i) {
    b[i] = ra.tabs[NTAB + i];
    am[i] = ra.tabs[NTAB + P + 1 + i];
  }
  S pre_v = zero_s(S{}), s0_v = zero_s(S{});
  if (t < P) {
    pre_v = x_at(x, xh, cf.K, (int64_t)base - 1 - t);
    if (yh && t < cf.K - 1) s0_v = yh[t];
  }
  GSDR_RES_TS(1);

  // the tile into LDS (rows of 33 floats per component), then each lane's chunk row into registers
  if (whole) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int idx = (k * kResWG + t) * SPV;  // SPV consecutive samples, one chunk row
      float* d = reinterpret_cast<float*>(reinterpret_cast<S*>(tile) + Sh::at(idx));
      d[0] = v4[k].x;
      d[1] = v4[k].y;
      d[2] = v4[k].z;
      d[3] = v4[k].w;
    }
  } else {
    for (int idx = t; idx < (int)Sh::TS; idx += kResWG) {
      reinterpret_cast<S*>(tile)[Sh::at(idx)] = idx < (int)tlen ? x[base + idx] : zero_s(S{});
    }
  }
#pragma unroll
  for (int r = 0; r < NTR; ++r) {
    const int e = r * kResWG + t;
    if (e < NTAB) tab[e] = tv[r];
  }
  if (t < P) {
    pre[t] = pre_v;
    sv[1][t] = to_acc(s0_v);
  }
  lds_barrier();
  GSDR_RES_TS(2);
  // this lane's chunk (component comp); not __restrict__: the rows are read through `tile` by other lanes and by
  // the coalesced output loop, and restrict would let the compiler move those accesses across this lane's stores
  float* row = tile + (size_t)lc * Sh::STRIDE * NC + comp;
  double xd[P];  // component of x[n0 - 1 - i], read before any row is overwritten
  {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int m = lc * kChunk - 1 - i;  // tile index of x[n0 - 1 - i]; < 0: before the tile
      xd[i] = (double)reinterpret_cast<const float*>(m >= 0 ? reinterpret_cast<S*>(tile) + Sh::at(m) : pre + (-1 - m))[comp];
    }
  }
  lds_barrier();
  const uint64_t n0 = base + (uint64_t)lc * kChunk;
  const uint32_t len = n0 >= n ? 0u : (n - n0 < (uint64_t)kChunk ? (uint32_t)(n - n0) : (uint32_t)kChunk);
  // one chunk of the recursion from state ys (the feedback terms oldest first: one FMA on the critical path)
  auto run_chunk = [&](double (&ys)[P], double (&xs)[P], bool write) {
    auto step = [&](int k) {
      const double xv = (double)row[k * NC];
      double acc = b[0] * xv;
#pragma unroll
      for (int i = 1; i <= P; ++i) acc = fma(b[i], xs[i - 1], acc);
#pragma unroll
      for (int i = P; i >= 1; --i) acc = fma(am[i], ys[i - 1], acc);
#pragma unroll
      for (int i = P - 1; i > 0; --i) {
        xs[i] = xs[i - 1];
        ys[i] = ys[i - 1];
      }
      xs[0] = xv;
      ys[0] = acc;
      if (write) row[k * NC] = (float)acc;  // y replaces x in this chunk's row
    };
    if (len == (uint32_t)kChunk) {
#pragma unroll
      for (int k = 0; k < kChunk; ++k) step(k);
    } else {
      for (int k = 0; k < (int)len; ++k) step(k);
    }
  };
  // 1b. zero-state pass: the chunk's zero-state outputs replace its inputs in the row; the tail in registers
  double tl[P], xe[P];
  {
    double ys[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      ys[i] = 0.0;
      xe[i] = xd[i];
    }
    run_chunk(ys, xe, true);
#pragma unroll
    for (int i = 0; i < P; ++i) tl[i] = ys[i];
  }
  GSDR_RES_TS(3);
  // 2. chunk prefixes across the workgroup (lanes of one component, NC apart); the last chunk's is the tile's
  //    aggregate
  double pfx[P];
#pragma unroll
  for (int i = 0; i < P; ++i) pfx[i] = tl[i];
  wg_scan<double, P, NC>(pfx, pw0, scd);
  A* scA = reinterpret_cast<A*>(scd);
  const uint32_t sb = tile_id / kResSB, k_in = tile_id % kResSB;
  if (lc == Sh::CPT - 1) {
#pragma unroll
    for (int i = 0; i < P; ++i) st_co(ra.loc + ((size_t)tile_id * P + i) * NC + comp, pfx[i]);
  }
#ifdef GSDR_IIR_RES_TIMING
  GSDR_RES_TS(3);  // stores issued (the pass-1 mark moves here)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  GSDR_RES_TS(4);

  // 3. entry state of the tile: with L_j tile j's zero-entry aggregate, G_t superblock t's and k = k_in,
  //      S_tile = M_T^k S_sb + sum_{j<k} M_T^(k-1-j) L_j,   S_sb = M_SB^sb s0 + sum_{t<sb} M_SB^(sb-1-t) G_t.
  //    Thread j forms the j-th term of each sum (binary powering with its own exponent; the s0 term on the last
  //    thread, which no sum uses), then one fixed-order sum over the workgroup: no matrix-weighted scan and
  //    no serial composition. Thread t polls tile sb * 256 + t's aggregate for t < k and superblock t's for
  //    t < sb, together (one round trip when they are written already); the last tile of a superblock polls
  //    the superblocks only after writing its own (else each superblock's aggregate would wait for the one
  //    before).
  const bool last_in_sb = k_in == kResSB - 1;
  const uint32_t h = sb * kResSB + (uint32_t)t;
  constexpr int NV2 = P * NC;
  A ut[P], qt[P];  // this thread's term of each sum
#pragma unroll
  for (int i = 0; i < P; ++i) ut[i] = qt[i] = zero_s(A{});
  const bool u_mine = (uint32_t)t < k_in, q_mine = (uint32_t)t < sb, s0_mine = t == kResWG - 1;
  bool ok = true;
  auto poll_into = [&](const double* src, A (&v)[P]) {
    double tmp[NV2];
    ok = poll_vals<NV2>(src, tmp, ra.max_polls) && ok;
#pragma unroll
    for (int i = 0; i < P; ++i) {
#pragma unroll
      for (int c = 0; c < NC; ++c) reinterpret_cast<double*>(&v[i])[c] = tmp[i * NC + c];
    }
  };
  auto q_term = [&]() {
    if (s0_mine) {
#pragma unroll
      for (int i = 0; i < P; ++i) qt[i] = sv[1][i];
    }
    if (q_mine || s0_mine) {
      mat_pow_vec<A, P>(pwg + 8 * PP, q_mine ? sb - 1 - (uint32_t)t : sb, qt);
      mat_pow_vec<A, P>(pwg, k_in, qt);
    }
  };
  GSDR_RES_TS(5);
  A tot[P];
  if (!last_in_sb) {
    {
      ok = wave0_wait<NV2>(ra.loc + (size_t)sb * kResSB * P * NC, k_in, ra.sbagg, sb, ra.max_polls);
      double tu[NV2], tq[NV2];
      ok = poll_vals2<NV2>(u_mine ? ra.loc + (size_t)h * P * NC : nullptr, tu,
                           q_mine ? ra.sbagg + (size_t)t * P * NC : nullptr, tq, ra.max_polls) && ok;
      GSDR_RES_TS(9);
#pragma unroll
      for (int i = 0; i < P; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (u_mine) reinterpret_cast<double*>(&ut[i])[c] = tu[i * NC + c];
          if (q_mine) reinterpret_cast<double*>(&qt[i])[c] = tq[i * NC + c];
        }
      }
    }
    q_term();
    if (u_mine) mat_pow_vec<A, P>(pwg, k_in - 1 - (uint32_t)t, ut);
    GSDR_RES_TS(10);
#pragma unroll
    for (int i = 0; i < P; ++i) ut[i] = add_s(ut[i], qt[i]);
    wg_sum<A, P>(ut, tot, scA);
    GSDR_RES_TS(11);
  } else {
    // the superblock's aggregate first: G_sb = M_T (sum_{j<255} M_T^(254-j) L_j) + L_255 (the last thread
    // holds this tile's own L, the last chunk's prefix, for NC == 1; both components' lanes for NC == 2)
    ok = wave0_wait<NV2>(ra.loc + (size_t)sb * kResSB * P * NC, k_in, nullptr, 0, ra.max_polls);
    if (u_mine) poll_into(ra.loc + (size_t)h * P * NC, ut);
    if (u_mine) mat_pow_vec<A, P>(pwg, k_in - 1 - (uint32_t)t, ut);
    A us[P];
    wg_sum<A, P>(ut, us, scA);
    if (lc == Sh::CPT - 1 && sb + 1 < (ntiles + kResSB - 1) / kResSB) {
      double g[P];
#pragma unroll
      for (int i = 0; i < P; ++i) g[i] = reinterpret_cast<const double*>(&us[i])[comp];
      mat_vec<double, P>(pwg, g);
#pragma unroll
      for (int i = 0; i < P; ++i) st_co(ra.sbagg + ((size_t)sb * P + i) * NC + comp, g[i] + pfx[i]);
    }
    ok = wave0_wait<NV2>(nullptr, 0, ra.sbagg, sb, ra.max_polls) && ok;
    if (q_mine) poll_into(ra.sbagg + (size_t)t * P * NC, qt);
    q_term();
    wg_sum<A, P>(qt, tot, scA);
#pragma unroll
    for (int i = 0; i < P; ++i) tot[i] = add_s(tot[i], us[i]);
  }
  ok = __syncthreads_and(ok);
  if (t == 0) {
#pragma unroll
    for (int i = 0; i < P; ++i) sv[0][i] = tot[i];  // the tile's entry state (also for the history out)
  }
  // the previous chunk's prefix: a lane shuffle, or the previous wave's last chunk through LDS
  double pv[P];
  const int lane = t & 63, w = t >> 6;
#pragma unroll
  for (int i = 0; i < P; ++i) pv[i] = shfl_up_s(pfx[i], NC);
  if (lane >= 64 - NC) {
#pragma unroll
    for (int i = 0; i < P; ++i) bnd[(w * NC + comp) * P + i] = pfx[i];
  }
  lds_barrier();
  if (lane < NC && w > 0) {
#pragma unroll
    for (int i = 0; i < P; ++i) pv[i] = bnd[((w - 1) * NC + comp) * P + i];
  }
  GSDR_RES_TS(6);
  // 4. this chunk's start state M0^lc S_tile + prefix_(lc-1), the recursion again, y through LDS
  double st[P];
#pragma unroll
  for (int i = 0; i < P; ++i) st[i] = reinterpret_cast<const double*>(&tot[i])[comp];
  mat_pow_vec<double, P>(pw0, (uint32_t)lc, st);
  if (lc > 0) {
#pragma unroll
    for (int i = 0; i < P; ++i) st[i] += pv[i];
  }
  if (!ok) {  // gave up waiting: NaN outputs, and the status word tells the host (gsdrxIirSinglePassStatus)
#pragma unroll
    for (int i = 0; i < P; ++i) st[i] = __builtin_nan("");
    if (t == 0) atomicOr(ra.status, 1u);
  }
  // y = y_zs + sum_i gk[k][i] st_i: the free response from the chunk's start state, added without a recursion
  {
    auto fix = [&](int k) {
      double acc = (double)row[k * NC];
#pragma unroll
      for (int i = 0; i < P; ++i) acc = fma(gk[k * P + i], st[i], acc);
      row[k * NC] = (float)acc;
    };
    if (len == (uint32_t)kChunk) {
#pragma unroll
      for (int k = 0; k < kChunk; ++k) fix(k);
    } else {
      for (int k = 0; k < (int)len; ++k) fix(k);
    }
  }
  lds_barrier();
  GSDR_RES_TS(7);
  if (len > 0 && n0 + len == n && ok) {  // (a tile that gave up may not have waited for the readers)
    // the state after the call (outputs, then inputs, newest first) into the caller's history buffers: the
    // outputs as written (from the tile; before it, the tile's entry state)
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i < ra.Pk) {
        const int m = (int)tlen - 1 - i;
        if (ra.yh_out) {
          ra.yh_out[i * NC + comp] = m >= 0 ? reinterpret_cast<const float*>(reinterpret_cast<const S*>(tile) + Sh::at(m))[comp]
                                            : (float)reinterpret_cast<const double*>(&sv[0][-1 - m])[comp];
        }
        if (ra.xh_out) ra.xh_out[i * NC + comp] = (float)xe[i];
      }
    }
  }
  if (whole) {
    float4* __restrict__ dst = reinterpret_cast<float4*>(y + base);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int idx = (k * kResWG + t) * SPV;
      const float* d = reinterpret_cast<const float*>(reinterpret_cast<const S*>(tile) + Sh::at(idx));
      dst[k * kResWG + t] = make_float4(d[0], d[1], d[2], d[3]);
    }
  } else {
    for (int idx = t; idx < (int)tlen; idx += kResWG) y[base + idx] = reinterpret_cast<const S*>(tile)[Sh::at(idx)];
  }
#ifdef GSDR_IIR_RES_TIMING
  __syncthreads();
  ts_[8] = wall_clock64();
  if (t == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(y + base);
    for (int i = 0; i < 12; ++i) o[i] = ts_[i];
    o[12] = __smid();
  }
#endif
}

}  // namespace res
