// perc_resident.h -- the resident cooperative solve.
//
// Device code of libperc, included by perc_solve.hip (every definition sits in an
// anonymous namespace: each translation unit keeps its own copy of what it
// launches).
#pragma once
#include "perc_cg.h"

// (each TU launches a subset of these internal-linkage helpers)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
namespace perc {
namespace {

// ---------------------------------------------------------------------------
// Resident persistent solve for small lattices (every band's state fits on
// chip).  One cooperative launch runs the whole linbcg loop: workgroup w
// (NT threads, one per CU) owns lattice rows [w H, w H + H) at full width;
// p of its rows lives in LDS, r, q and the row codes in registers (thread t
// holds columns t + j NT, j < MT, of every own row).  Per iteration (the
// order of linbcg, bondc.f:780-835, every per-row operation as in the other
// kernels):
//   1. p = bk p + r/d (z = r/d at k = 1) into LDS, and p(k) of the
//      neighbours' rows next to the band from their exchanged r(k-1) and
//      p(k-1) with the same arithmetic (no barrier);
//   2. q = A p, q.p;  grid-wide reduction -> ak (the same everywhere);
//   3. r -= ak q, z = r/d, z.r, r.r, x += ak p on the rows x is kept on; the
//      band's first and last rows of r(k) and p(k) to the exchange
//      (write-through, parity-buffered);  grid-wide reduction -> bk, err,
//      stop test (identical in every workgroup, so all leave together)
// Two grid-wide reductions and no launches per iteration (an iteration of
// the launched kernels at L = 1024 is ~28 us, almost all fixed costs).  The
// reductions: res_allreduce_x (XCD-grouped, the default) or res_gather (flat
// all-gather).  One grid barrier before the loop (res_barrier) publishes the
// first exchange rows; data crossing workgroups is written and read with
// sc1 (agent-scope) accesses, as in publish_and_reduce.  A wait that
// exceeds ~1 s sets an error flag and leaves the kernel instead of hanging
// the device.
constexpr int kResThreads = 1024;
constexpr int kResLdsRows = 16384;  // own-row p elements per workgroup (128 KB)
constexpr unsigned kResSquareMask = 0x5Au;  // raster positions (-1,0) (0,-1) (0,1) (1,0)

struct ResArgs {
  StencilView St;
  int m, nrows, pbc, G, H;
  int xrows;
  const double* r0;  // r after k_cg_init
  double* x;
  CGScalars* S;
  double* err_hist;
  int err_hist_cap;
  double* xch;       // [2 parity][G][top, bottom][r, p][m]
  unsigned* bar;     // 9 counters, 128 B apart (zeroed before the launch)
  double* gran;      // [3][G] 16-B granules {partial, tag}, then kResLitGran result
                     // granules of the literal folds (zeroed before the launch)
  // literal dot order (PERC_DOT_LITERAL): the elements' q.p, z.r and r.r terms
  // at their row-major index in lit[0..N), [N..2N), [2N..3N), folded in
  // ascending j by workgroup 0 (res_fold); nullptr in the fast order (the
  // term stores then go to a zero-size buffer view and are dropped)
  double* lit;
  // XCD-grouped reductions (res_allreduce_x): registration counters (8 per-XCD
  // + 1 arrival, kTicketStride apart) and the granules: level 1
  // [kind][j][xcd][kResXcdMax], level 2 [kind][parity][j][xcd] (zeroed
  // before the launch)
  unsigned* reg;
  double* xg;
};
constexpr int kResLitGran = 4;
constexpr int kResXcdMax = 64;  // workgroups per XCD the grouped reductions take
constexpr size_t kResXgDoubles = 2 * (2 * 2 * 8 * kResXcdMax + 2 * 2 * 2 * 8);


// single-level (m = 1024: 0.0166 vs 0.0178 ms per iteration)
__device__ __forceinline__ bool res_barrier1(const ResArgs& a, unsigned& epoch, int* s_flag) {
  __syncthreads();  // (a release fence: every wave's stores are complete)
  ++epoch;
  if (threadIdx.x < 64) {
    // one arrival on the workgroup's XCD-group counter, then wave 0 polls
    // the (up to) 8 group counters together, one per lane, until they sum
    // to epoch * G: no second-level counter hop on the critical path
    const int lane = threadIdx.x, G = a.G, ngrp = G < 8 ? G : 8;
    if (lane == 0)
      __hip_atomic_fetch_add(&a.bar[(blockIdx.x & 7) * kTicketStride], 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    const unsigned want = epoch * (unsigned)G;
    int ok = 1;
    for (unsigned spin = 0;; ++spin) {
      unsigned v = lane < ngrp ? __hip_atomic_load(&a.bar[lane * kTicketStride], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                               : 0u;
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) v += __shfl_xor(v, o);  // lanes 0..7
      if (__builtin_amdgcn_readfirstlane(v) >= want) break;
      if (spin > (1u << 25)) {  // ~1 s: give up, report, leave
        if (lane == 0) a.S->pad[0] = 1;
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) s_flag[0] = ok;
  }
  __syncthreads();
  return s_flag[0] != 0;
}

// two-level: the last arriver of an XCD group bumps one top counter, which
// thread 0 of every workgroup polls (m = 2048: arrivals are spread out over
// the longer phases, and polling all 8 group counters slows them: 0.0373
// vs 0.0352 ms per iteration)
__device__ __forceinline__ bool res_barrier2(const ResArgs& a, unsigned& epoch, int* s_flag) {
  __syncthreads();
  ++epoch;  // in every thread: res_gather's tags are per lane
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int G = a.G, grp = blockIdx.x & 7, ngrp = G < 8 ? G : 8;
    const unsigned ng = (unsigned)((G - grp + 7) / 8);
    const unsigned old = __hip_atomic_fetch_add(&a.bar[grp * kTicketStride], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == epoch * ng - 1)
      __hip_atomic_fetch_add(&a.bar[8 * kTicketStride], 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    for (unsigned spin = 0;; ++spin) {
      if (__hip_atomic_load(&a.bar[8 * kTicketStride], __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT) >= epoch * (unsigned)ngrp)
        break;
      if (spin > (1u << 25)) {  // ~1 s: give up, report, leave
        a.S->pad[0] = 1;
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    s_flag[0] = ok;
  }
  __syncthreads();
  return s_flag[0] != 0;
}

template <bool POLL8>
__device__ __forceinline__ bool res_barrier(const ResArgs& a, unsigned& epoch, int* s_flag) {
  return POLL8 ? res_barrier1(a, epoch, s_flag) : res_barrier2(a, epoch, s_flag);
}

// Reduction by all-gather of tagged granules (no counter): thread 0 of every
// workgroup publishes each of its NV partials as one 16-B {value, tag}
// write-through store after the workgroup barrier that drained every wave's
// stores (its exchange rows included: payload sc1 -> vmcnt(0) -> granule,
// MI355X_MICROARCH.md hand-off table, granule row); wave 0 of every
// workgroup sweeps the G granules of each slot (16-B sc1 loads, lane l takes
// workgroups l, l+64, ...) until every tag equals this reduction's epoch,
// then sums the values lane-strided + butterfly (the association of
// res_total, the same on every workgroup).  One slot per reduction kind
// suffices: no workgroup can publish the next epoch of a kind before every
// workgroup has left the other kind's reduction, i.e. finished polling this
// one.  Returns false after a ~1 s timeout (a.S->pad[0] set).
template <int NV>
__device__ __forceinline__ bool res_gather(const ResArgs& a, unsigned& epoch, double* gran,
                                           const double (&v)[NV], double (&tot)[NV],
                                           double* s_red) {
  __syncthreads();  // every wave's stores complete (release)
  ++epoch;
  const double tag = (double)epoch;
  const int G = a.G;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * G * 16));
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j)  // one 16-B write-through (sc1) store per granule: untorn
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, make_double2(v[j], tag)), rg,
          (int)(((size_t)j * G + blockIdx.x) * 16), 0, 16);
  }
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int ok = 1;
    double acc[NV];
    for (unsigned spin = 0;; ++spin) {
      bool all = true;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        acc[j] = 0.0;
        for (int i = lane; i < G; i += 64) {
          // one 16-B sc1 load: value and tag of one granule, untorn
          const double2 g2 = __builtin_bit_cast(
              double2, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(((size_t)j * G + i) * 16), 0, 16));
          all = all && g2.y == tag;
          acc[j] = acc[j] + g2.x;
        }
      }
      if (__builtin_amdgcn_readfirstlane(__all(all))) break;
      if (spin > (1u << 24)) {  // ~1 s: give up, report, leave
        if (lane == 0) a.S->pad[0] = 1;
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const double t = wave_sum(acc[j]);
      if (lane == 0) s_red[24 + j] = t;
    }
    if (lane == 0) s_red[30] = ok ? 1.0 : 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[24 + j];
  const bool ok = s_red[30] != 0.0;
  __syncthreads();  // s_red reuse by the next block_sum
  return ok;
}

// XCD-grouped all-reduction (the fast order's two reductions per iteration).
// At the start of the launch every workgroup reads the XCD it runs on
// (HW_REG_XCC_ID) and takes a rank there; when the G workgroups sit G/8 on
// each XCD, a workgroup's LOGICAL id -- the band of rows it owns -- is xcd
// * G/8 + rank (res_register).  The association of a reduction is then
// fixed in logical ids whatever the placement: level 1 sums the XCD's G/8
// partials in rank order, level 2 the 8 XCD totals in XCD order.  Level 1
// crosses no XCD: the workgroups store their 16-B {value, tag} granules
// plainly (kept in the XCD's L2) and the XCD's rank-0 workgroup reads them
// with sc1 loads (past its L1, served by the same L2); it then publishes
// the XCD total write-through, and wave 0 of every workgroup polls the 8
// XCD granules (parity-buffered: a fast XCD's next total must not replace
// one a slow workgroup has yet to read).  The two reductions (1 + 2 values) of an
// iteration cost 7.9 vs 12.2 us for the flat all-gather at G = 256, 1024
// threads (tools/sync_bench.hip, profiles/r5_18_sync_bench.log).  Any
// other placement (G not a multiple of 8, or an XCD holding more or fewer
// than G/8 workgroups) ends the grouped launch at once and the host runs
// the flat instantiation (kResPadUneven).
#if defined(PERC_RES_FLAT)  // (A/B probe builds only: the flat all-gather everywhere)
constexpr bool kResXcdGather = false;
#else
constexpr bool kResXcdGather = true;
#endif
// S->pad[1] of a grouped launch (k_cg_res<..., XG = true>) that found the
// placement uneven: every workgroup left before touching any state, and
// the host runs the flat instantiation instead
constexpr int kResPadUneven = 1;
struct ResXcd {
  int w;     // logical workgroup id (the band)
  int xcd, rank, nx;
  bool ok;   // grouped reductions (else res_gather, w = blockIdx.x)
};
__device__ __forceinline__ ResXcd res_register(const ResArgs& a, int* s_flag) {
  __shared__ int s_x[4];
  if (threadIdx.x == 0) {
    const int G = a.G;
    const int x = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u);  // HW_REG_XCC_ID
    const unsigned r = __hip_atomic_fetch_add(&a.reg[x * kTicketStride], 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    // release / acquire on the arrival counter: a workgroup's per-XCD add is
    // ordered before its arrival, and the poll that sees all G arrivals
    // synchronises with every one of them (the RMWs form one release
    // sequence), so every workgroup reads the same, final per-XCD counts
    // below and takes the same grouped / flat decision
    __hip_atomic_fetch_add(&a.reg[8 * kTicketStride], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    for (unsigned spin = 0; __hip_atomic_load(&a.reg[8 * kTicketStride], __ATOMIC_ACQUIRE,
                                               __HIP_MEMORY_SCOPE_AGENT) < (unsigned)G;
         ++spin) {
      if (spin > (1u << 25)) {  // ~1 s: the grid is not co-resident
        a.S->pad[0] = 1;
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    bool even = G % 8 == 0 && G / 8 <= kResXcdMax;
    for (int y = 0; y < 8 && even; ++y)
      even = __hip_atomic_load(&a.reg[y * kTicketStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned)(G / 8);
    s_x[0] = even ? x * (G / 8) + (int)r : (int)blockIdx.x;
    s_x[1] = x;
    s_x[2] = (int)r;
    s_x[3] = even ? 1 : 0;
    s_flag[1] = ok;
  }
  __syncthreads();
  ResXcd X;  // (workgroup-uniform: scalar registers, not VGPRs, across the loop)
  X.w = __builtin_amdgcn_readfirstlane(s_x[0]);
  X.xcd = __builtin_amdgcn_readfirstlane(s_x[1]);
  X.rank = __builtin_amdgcn_readfirstlane(s_x[2]);
  X.nx = a.G / 8;
  X.ok = __builtin_amdgcn_readfirstlane(s_x[3]) != 0;
  return X;
}

// The block sum is part of it: every wave's lane 0 leaves its wave's sums
// in s_red, and behind the one workgroup barrier wave 0 adds the waves'
// values (lane-parallel + butterfly) and publishes; a second barrier hands
// the totals (s_res) to the workgroup.  The waves' stores are drained by the
// first barrier, before the granule that releases them is issued.
template <int NV>
__device__ __forceinline__ bool res_allreduce_x(const ResArgs& a, unsigned& epoch, int kind, const ResXcd& X,
                                                const double (&v)[NV], double (&tot)[NV], double* s_red,
                                                double* s_res) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const double t = wave_sum(v[j]);
    if (lane == 0) s_red[wid * NV + j] = t;
  }
  __syncthreads();  // every wave's sums in LDS and its stores complete (release)
  ++epoch;
  if (threadIdx.x < 64) {
    const double tag = (double)epoch;
    const int par = (epoch >> 1) & 1;  // the kinds alternate: a kind's epochs step by 2
    const __amdgpu_buffer_rsrc_t r1 = rsrc(a.xg, (unsigned)(2 * 2 * 8 * kResXcdMax * 16));
    const __amdgpu_buffer_rsrc_t r2 = rsrc(a.xg + 2 * 2 * 2 * 8 * kResXcdMax, (unsigned)(2 * 2 * 2 * 8 * 16));
    auto o1 = [&](int j, int r) { return (((kind * 2 + j) * 8 + X.xcd) * kResXcdMax + r) * 16; };
    auto o2 = [&](int j, int x) { return (((kind * 2 + par) * 2 + j) * 8 + x) * 16; };
    double wv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) wv[j] = wave_sum(lane < nw ? s_red[lane * NV + j] : 0.0);
    if (lane == 0)
#pragma unroll
      for (int j = 0; j < NV; ++j)  // plain 16-B stores: the line stays in this XCD's L2
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(wv[j], tag)), r1,
                                               o1(j, X.rank), 0, 0);
    int ok = 1;
    if (X.rank == 0) {  // the XCD's partials in rank order, then its total write-through
      double acc[NV];
      for (unsigned spin = 0;; ++spin) {
        bool all = true;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          acc[j] = 0.0;
          if (lane < X.nx) {
            const double2 g2 = __builtin_bit_cast(
                double2, __builtin_amdgcn_raw_buffer_load_b128(r1, o1(j, lane), 0, 16));
            all = all && g2.y == tag;
            acc[j] = g2.x;
          }
        }
        if (__builtin_amdgcn_readfirstlane(__all(all))) break;
        if (spin > (1u << 24)) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const double t = wave_sum(acc[j]);
        if (lane == 0)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(t, tag)), r2,
                                                 o2(j, X.xcd), 0, 16);
      }
    }
    double acc[NV];
    for (unsigned spin = 0; ok; ++spin) {  // the 8 XCD totals, lanes 0..7
      bool all = true;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        acc[j] = 0.0;
        if (lane < 8) {
          const double2 g2 =
              __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r2, o2(j, lane), 0, 16));
          all = all && g2.y == tag;
          acc[j] = g2.x;
        }
      }
      if (__builtin_amdgcn_readfirstlane(__all(all))) break;
      if (spin > (1u << 24)) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const double t = wave_sum(acc[j]);
      if (lane == 0) s_res[j] = t;
    }
    if (lane == 0) {
      s_res[7] = ok ? 1.0 : 0.0;
      if (!ok) a.S->pad[0] = 1;
    }
  }
  // (wave 0 has read s_red before this barrier, and every wave reads s_res
  // before the next reduction's first barrier: neither needs another one)
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_res[j];
  return s_res[7] != 0.0;
}

// The literal dot order inside the resident solve (bondc.f:785-787, 803-805,
// 872-875).  Every workgroup has stored its elements' terms of sums c0 ..
// c0+NC-1 write-through (sc1) at lit[c N + i]; behind the workgroup barrier
// that drains those stores thread 0 publishes an arrival granule {0, tag} in
// `arr` (the kind's res_gather slot).  Wave 0 of workgroup 0 waits for all
// G arrivals, folds the N terms of each sum in ascending j (fold_wave, sc1
// loads: the terms come from every XCD's workgroups within this launch) and
// publishes the totals as result granules {sum, tag}; wave 0 of every
// workgroup polls them (s_sleep-paced: a fold takes milliseconds).  The
// reduction's association is the reference's, so iter, err and every
// iterate are its linbcg's bitwise.  A verification mode: one serial fold of
// N terms per reduction.  Returns false after a timeout (a.S->pad[0] set).
// workgroup 0's part (wave 0): wait for the G arrivals, fold, publish
template <int NC>
__device__ __forceinline__ int res_fold_wg0(const ResArgs& a, const double* arr, int c0, double tag) {
  const int lane = threadIdx.x & 63, G = a.G, N = a.St.N;
  const __amdgpu_buffer_rsrc_t ra = rsrc(arr, (unsigned)(G * 16));
  const __amdgpu_buffer_rsrc_t rr = rsrc(a.gran + 6 * (size_t)G, (unsigned)(kResLitGran * 16));
  int ok = 1;
  for (unsigned spin = 0;; ++spin) {
    bool all = true;
    for (int i = lane; i < G; i += 64) {
      const double2 g2 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(ra, i * 16, 0, 16));
      all = all && g2.y == tag;
    }
    if (__builtin_amdgcn_readfirstlane(__all(all))) break;
    if (spin > (1u << 24)) {
      ok = 0;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  const __amdgpu_buffer_rsrc_t rl = rsrc(a.lit, (unsigned)N * 24u);
  double acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.0;
  struct RawN {
    double v[NC];
  };
  fold_wave<NC, 4, RawN, 8>(
      N,
      [&](int j) {
        RawN r;
#pragma unroll
        for (int c = 0; c < NC; ++c) r.v[c] = bld1s(rl, (unsigned)((c0 + c) * (size_t)N + j) * 8u);
        return r;
      },
      [&](const RawN& r, double (&t)[NC]) {
#pragma unroll
        for (int c = 0; c < NC; ++c) t[c] = r.v[c];
      },
      acc);
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < NC; ++c)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(acc[c], tag)), rr,
                                             (c0 + c) * 16, 0, 16);
  return ok;
}

template <int NC>
__device__ __forceinline__ bool res_fold(const ResArgs& a, unsigned& epoch, double* arr, int c0,
                                         double (&tot)[NC], double* s_red) {
  __syncthreads();  // every wave's term stores complete (release)
  ++epoch;
  const double tag = (double)epoch;
  const int G = a.G;
  const __amdgpu_buffer_rsrc_t ra = rsrc(arr, (unsigned)(G * 16));
  const __amdgpu_buffer_rsrc_t rr = rsrc(a.gran + 6 * (size_t)G, (unsigned)(kResLitGran * 16));
  if (threadIdx.x == 0)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(0.0, tag)), ra,
                                           (int)(blockIdx.x * 16), 0, 16);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int ok = 1;
    if (blockIdx.x == 0) ok = res_fold_wg0<NC>(a, arr, c0, tag);
    double v = 0.0;
    for (unsigned spin = 0; ok; ++spin) {
      const double2 g2 = lane < NC ? __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                                                                     rr, (c0 + lane) * 16, 0, 16))
                                   : make_double2(0.0, tag);
      v = g2.x;
      if (__builtin_amdgcn_readfirstlane(__all(g2.y == tag))) break;
      if (spin > (1u << 22)) {  // ~4 s at s_sleep 64 (64 x 64 cycles per poll)
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(64);
    }
    if (lane < NC) s_red[24 + lane] = v;
    if (lane == 0) {
      s_red[30] = ok ? 1.0 : 0.0;
      if (!ok) a.S->pad[0] = 1;
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c) tot[c] = s_red[24 + c];
  const bool ok = s_red[30] != 0.0;
  __syncthreads();  // s_red reuse
  return ok;
}

// one raster position KP of an element's q (compile-time row / column
// offsets: the neighbours' rows next to the band come from named registers,
// never from an indexed register array, which hipcc puts in scratch)
struct ResHalo {
  double l, c, r;  // columns c-1, c, c+1
};
template <int DC>
__device__ __forceinline__ double halo_at(const ResHalo& h) {
  return DC < 0 ? h.l : (DC == 0 ? h.c : h.r);
}
template <int KP, unsigned UMC>
__device__ __forceinline__ void res_pos(double& acc, unsigned um, unsigned map, unsigned cc, int lr,
                                        int Hw, int m, int c, const double* s_p, const ResHalo& hu,
                                        const ResHalo& hd, double ng0, double nleak) {
  constexpr int DR = KP < 3 ? -1 : (KP < 5 ? 0 : 1);
  constexpr int DC = KP < 3 ? KP - 1 : (KP == 3 ? -1 : (KP == 4 ? 1 : KP - 6));
  if (!(UMC & (1u << KP))) return;  // position no form of the lattice uses
  if (!(um & (1u << KP))) return;   // wave-uniform
  const int col = c + DC;  // in range for every position a regular form uses
  double v;
  if (DR < 0) {
    v = lr > 0 ? s_p[(lr > 0 ? lr - 1 : 0) * m + col] : halo_at<DC>(hu);
  } else if (DR > 0) {
    v = lr + 1 < Hw ? s_p[(lr + 1 < Hw ? lr + 1 : lr) * m + col] : halo_at<DC>(hd);
  } else {
    v = s_p[lr * m + col];
  }
  const unsigned sj = (map >> (4 * KP)) & 15u;
  const double gv = ((cc >> sj) & 1u) ? ng0 : nleak;
  const double pr = gv * v;
  acc = sj != 15u ? acc + pr : acc;
}

// the same term for a wave whose elements all share one regular form (slot
// order = raster order, used positions `mask`, wave-uniform): the slot of
// position KP is the count js of used positions before it, a scalar, so
// the term needs no lane-private raster -> slot map and no unused-slot
// select; the arithmetic (acc + gv v in slot order) is res_pos's
template <int KP, unsigned UMC>
__device__ __forceinline__ void res_pos_u(double& acc, unsigned mask, unsigned& js, unsigned cc,
                                          int lr, int Hw, int m, int c, const double* s_p,
                                          const ResHalo& hu, const ResHalo& hd, double ng0,
                                          double nleak) {
  constexpr int DR = KP < 3 ? -1 : (KP < 5 ? 0 : 1);
  constexpr int DC = KP < 3 ? KP - 1 : (KP == 3 ? -1 : (KP == 4 ? 1 : KP - 6));
  if (!(UMC & (1u << KP))) return;
  if (!(mask & (1u << KP))) return;  // wave-uniform
  const int col = c + DC;
  double v;
  if (DR < 0) {
    v = lr > 0 ? s_p[(lr > 0 ? lr - 1 : 0) * m + col] : halo_at<DC>(hu);
  } else if (DR > 0) {
    v = lr + 1 < Hw ? s_p[(lr + 1 < Hw ? lr + 1 : lr) * m + col] : halo_at<DC>(hd);
  } else {
    v = s_p[lr * m + col];
  }
  const double gv = ((cc >> js) & 1u) ? ng0 : nleak;
  acc = acc + gv * v;
  ++js;
}

// QREG: q of the own rows kept in registers between the q.p reduction and
// the r update; else (wider / taller bands: L = 2048 has 16 elements per
// thread) q is formed again from p(k) in LDS and the halo registers with
// the same arithmetic (bitwise the same q), so the thread holds only r and
// the codes
// UMC: compile-time superset of the raster positions the forms use (0x5A:
// the square lattice's four neighbours), so unused positions and their
// halo columns take no registers
// LIT: the literal dot order (a.lit): the elements' terms are stored and the
// two all-gathers become res_fold's serial folds; every other line of the
// loop is the fast instantiation's (a separate instantiation because the
// fold's registers would otherwise join the fast loop's allocation: 122 ->
// 256 VGPRs with spills at m = 1024)
// XG: the XCD-grouped reductions (res_register / res_allreduce_x); without
// it the flat all-gather (res_gather), the literal folds, w = blockIdx.x
template <int MT, int HMAX, bool QREG = true, unsigned UMC = 0xFFu, int NT = kResThreads, bool LIT = false,
          bool XG = false>
__global__ __launch_bounds__(NT) void k_cg_res(ResArgs a) {
  __shared__ double s_p[kResLdsRows];
  __shared__ double2 s_dt[kDiagTab];
  __shared__ unsigned s_rmap[kMaxForms], s_umask[kMaxForms];
  __shared__ double s_red[32];
  __shared__ double s_res[8];
  __shared__ int s_flag[2];
  int t = threadIdx.x;  // re-made opaque each iteration when !QREG (below)
  // the band this workgroup owns: its logical id (res_register) with the
  // grouped reductions, else its block index
  ResXcd X{(int)blockIdx.x, 0, 0, 0, false};
  if constexpr (XG) {
    X = res_register(a, s_flag);
    if (!X.ok || !s_flag[1]) {  // (uniform: every workgroup read the same final counters)
      if (blockIdx.x == 0 && threadIdx.x == 0 && s_flag[1]) a.S->pad[kResPadUneven] = 1;
      return;
    }
  }
  const int w = X.w;
  const int m = a.m, nrows = a.nrows, N = a.St.N, G = a.G;
  const int R0 = w * a.H, Hw = min(a.H, nrows - R0);  // >= 1 (host sizes G)
  // one column per thread below m = 1024, the workgroup rounded up to whole
  // waves: threads past the last column own no element (they join the
  // barriers and reductions with zeros)
  const bool tin = MT > 1 || t < m;
  const bool has_up = R0 > 0, has_dn = R0 + Hw < nrows;
  const double ng0 = a.St.ng0, nleak = a.St.nleak;
  CGScalars* S = a.S;
  if (t < kMaxForms) {
    s_rmap[t] = a.St.F.rmap[t];
    s_umask[t] = a.St.F.regular[t] ? a.St.F.rmask[t] : 0u;  // (a regular form uses >= 1 position)
  }
  load_dtab(a.St, s_dt);
  // own state: r and the codes of (row lr, column t + j NT)
  double rv[HMAX][MT], qv[QREG ? HMAX : 1][QREG ? MT : 1];
  // the row codes (u16), two per register when MT = 2
  unsigned cv[HMAX][(MT + 1) / 2];
  auto code_at = [&](int lr, int j) { return (cv[lr][j / 2] >> (16 * (j & 1))) & 0xffffu; };
#pragma unroll
  for (int lr = 0; lr < HMAX; ++lr)
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int i = (R0 + lr) * m + t + j * NT;
      const bool own = lr < Hw && tin;
      rv[lr][j] = own ? a.r0[i] : 0.0;
      const unsigned cj = own ? a.St.code[i] : 0u;
      if (j & 1) cv[lr][j / 2] |= cj << 16;
      else cv[lr][j / 2] = cj;
      if constexpr (QREG) qv[lr][j] = 0.0;
    }
  // the neighbours' rows next to the band, columns c-1 .. c+1: their codes
  // (static) and whether the position exists
  // (column c + d - 1 exists unless c + d - 1 is -1 or m; regular forms
  // use no wrapped column)
  auto hin = [&](int j, int d) { const int cc = t + j * NT + d - 1; return cc >= 0 && cc < m; };
  auto hcol = [&](int j, int d) { const int cc = t + j * NT + d - 1; return cc < 0 ? 0 : (cc >= m ? m - 1 : cc); };
  unsigned hcu[MT][3], hcd[MT][3];
#pragma unroll
  for (int j = 0; j < MT; ++j)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      if (!(UMC & (1u << d)) && !(UMC & (1u << (5 + d)))) {
        hcu[j][d] = hcd[j][d] = 0u;
        continue;
      }
      hcu[j][d] = has_up && hin(j, d) ? a.St.code[(R0 - 1) * m + hcol(j, d)] : 0u;
      hcd[j][d] = has_dn && hin(j, d) ? a.St.code[(R0 + Hw) * m + hcol(j, d)] : 0u;
    }
  const __amdgpu_buffer_rsrc_t rx = rsrc(a.xch, (unsigned)((size_t)2 * G * 4 * m * 8));
  // literal dot terms, write-through (sc1): workgroup 0 folds them in this
  // launch (size 0 in the fast order: the stores are dropped)
  const __amdgpu_buffer_rsrc_t rl = rsrc(a.lit, LIT ? (unsigned)N * 24u : 0u);
  // exchange rows: [parity][w][top, bottom][r, p][m]
  auto xrow = [&](int par, int ww, int tb, int rp) {
    return a.xch + ((((size_t)par * G + ww) * 2 + tb) * 2 + rp) * m;
  };
  // r(1) of the band's first and last rows, for the neighbours' p(1)
#pragma unroll
  for (int lr = 0; lr < HMAX; ++lr)
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int c = t + j * NT;
      if (tin && lr == 0) store_sc1(&xrow(1, w, 0, 0)[c], rv[lr][j]);
      if (tin && lr == Hw - 1) store_sc1(&xrow(1, w, 1, 0)[c], rv[lr][j]);
    }
  // x kept on the lattice's first and last interior rows only (xrows = m,
  // the default): those rows' x live in registers of the two workgroups
  // that own them for the whole solve (a global load + store per iteration
  // put ~1-1.5 us of latency on those workgroups, which every other one
  // then waited for at the next reduction)
  const bool xreg = QREG && a.xrows == m;  // (not with 16 elements per thread: spills)
  const bool x0w = xreg && tin && R0 == 0, x1w = xreg && tin && R0 + Hw == nrows && nrows > 1;
  double xa[MT], xb[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int c = t + j * NT;
    xa[j] = x0w ? a.x[c] : 0.0;
    xb[j] = x1w ? a.x[(size_t)(nrows - 1) * m + c] : 0.0;
  }
  unsigned epoch = 0;
  bool ok = res_barrier<MT == 1>(a, epoch, s_flag);
  double bknum = S->bknum, bk = 0.0, ak = 0.0;
  const double bnrm = S->bnrm, tol = S->tol;
  const int itmax = S->itmax;
  int k = 0;
  double err = 0.0;
  bool done = !ok;
  while (!done) {
    // 16 elements per thread: keep the compiler from hoisting every
    // element's addresses out of the loop (they would stay live across it
    // and spill); recomputing them is a few integer ops
    if constexpr (!QREG) asm volatile("" : "+v"(t));
    ++k;
    const int par = k & 1;
    // 1. halo loads first (their latency overlaps the own rows' p(k))
    // (buffer loads with sc1, out-of-range offsets for absent positions: one
    // per-lane offset register for all of them, no branches)
    double hur[MT][3], hup[MT][3], hdr[MT][3], hdp[MT][3];
    {
      const unsigned um = a.St.F.umask;
      const unsigned bu = (unsigned)((xrow(par, w - 1, 1, 0) - a.xch) * 8);
      const unsigned bd = (unsigned)((xrow(par, w + 1, 0, 0) - a.xch) * 8);
      const unsigned rs = (unsigned)m * 8u;  // r -> p row of one exchange slot
#pragma unroll
      for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          if (!(UMC & (1u << d)) && !(UMC & (1u << (5 + d)))) {
            hur[j][d] = hup[j][d] = hdr[j][d] = hdp[j][d] = 0.0;
            continue;
          }
          const bool u = has_up && hin(j, d) && (um & (1u << d));
          const bool dn = has_dn && hin(j, d) && (um & (1u << (5 + d)));
          const unsigned co = (unsigned)hcol(j, d) * 8u;
          hur[j][d] = bld1s(rx, u ? bu + co : kOOB);
          hup[j][d] = bld1s(rx, u && k > 1 ? bu + rs + co : kOOB);
          hdr[j][d] = bld1s(rx, dn ? bd + co : kOOB);
          hdp[j][d] = bld1s(rx, dn && k > 1 ? bd + rs + co : kOOB);
        }
    }
    // p(k) of the own rows into LDS
#pragma unroll
    for (int lr = 0; lr < HMAX; ++lr)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if (lr < Hw && tin) {
          const int e = lr * m + t + j * NT;
          const double z = div_tab(rv[lr][j], s_dt[diag_idx(code_at(lr, j))]);
          s_p[e] = k == 1 ? z : bk * s_p[e] + z;
        }
        if constexpr (!QREG) __builtin_amdgcn_sched_barrier(0);
      }
    // p(k) of the neighbours' rows, with the same arithmetic
    ResHalo hu[MT], hd[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      double u3[3], d3[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        if (!(UMC & (1u << d)) && !(UMC & (1u << (5 + d)))) {
          u3[d] = d3[d] = 0.0;
          continue;
        }
        const double zu = div_tab(hur[j][d], s_dt[diag_idx(hcu[j][d])]);
        const double zd = div_tab(hdr[j][d], s_dt[diag_idx(hcd[j][d])]);
        u3[d] = has_up && hin(j, d) ? (k == 1 ? zu : bk * hup[j][d] + zu) : 0.0;
        d3[d] = has_dn && hin(j, d) ? (k == 1 ? zd : bk * hdp[j][d] + zd) : 0.0;
      }
      hu[j] = ResHalo{u3[0], u3[1], u3[2]};
      hd[j] = ResHalo{d3[0], d3[1], d3[2]};
    }
    __syncthreads();
    // q of own element (lr, j) from p(k) in LDS and the halo rows
    auto qcalc = [&](int lr, int j, double xi) {
      const int c = t + j * NT;
      const unsigned cc = code_at(lr, j);
      double acc = s_dt[diag_idx(cc)].x * xi;
      // raster positions in order (compile-time row / column offsets):
      // for the regular forms the resident path is limited to, raster
      // order is slot order
      const unsigned f = cc >> 11, ff = __builtin_amdgcn_readfirstlane(f);
      const unsigned mask = s_umask[ff];  // 0: not a regular form
      // (the square lattice's 4-element variant only: with 16 elements per
      // thread, or all eight positions, the second path's registers spill)
      if (QREG && UMC == kResSquareMask && !__any(f != ff) && mask != 0u) {
        unsigned js = 0;
        res_pos_u<0, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<1, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<2, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<3, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<4, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<5, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<6, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        res_pos_u<7, UMC>(acc, mask, js, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
        return acc;
      }
      // mixed forms (edge columns): the slot of position kp comes from rmap
      const unsigned map = s_rmap[f];
      const unsigned um = a.St.F.umask;
      res_pos<0, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<1, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<2, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<3, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<4, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<5, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<6, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      res_pos<7, UMC>(acc, um, map, cc, lr, Hw, m, c, s_p, hu[j], hd[j], ng0, nleak);
      return acc;
    };
    // 2. q = A p, q.p
    double dot = 0.0;
#pragma unroll
    for (int lr = 0; lr < HMAX; ++lr)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if (lr < Hw && tin) {
          const double xi = s_p[lr * m + t + j * NT];
          const double acc = qcalc(lr, j, xi);
          if constexpr (QREG) qv[lr][j] = acc;
          const double tq = acc * xi;  // akden's term (bondc.f:803-805)
          dot = dot + tq;
          if constexpr (LIT)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, tq), rl,
                                                  (int)((unsigned)((R0 + lr) * m + t + j * NT) * 8u), 0, 16);
        }
        // one element at a time (hoisting every element's LDS reads spills)
        __builtin_amdgcn_sched_barrier(0);
      }
    {
      double tot[1];
      if constexpr (LIT) {
        if (!(ok = res_fold<1>(a, epoch, a.gran, 0, tot, s_red))) break;
      } else {
        double v1[1] = {dot};
        if constexpr (XG) {
          ok = res_allreduce_x<1>(a, epoch, 0, X, v1, tot, s_red, s_res);
        } else {
          block_sum<1>(v1, s_red);
          ok = res_gather<1>(a, epoch, a.gran, v1, tot, s_red);
        }
        if (!ok) break;
      }
      ak = bknum / tot[0];
    }
    // 3. r, z, dots, x; the band's first / last rows of r(k+1) and p(k)
    //    to the exchange for the neighbours' p(k+1)
    const int npar = (k + 1) & 1;
    double acc2[2] = {0.0, 0.0};
#pragma unroll
    for (int lr = 0; lr < HMAX; ++lr)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if (lr < Hw && tin) {
          const int c = t + j * NT;
          double qq;
          if constexpr (QREG) qq = qv[lr][j];
          else qq = qcalc(lr, j, s_p[lr * m + c]);
          const double rn = rv[lr][j] - ak * qq;
          rv[lr][j] = rn;
          const double z = div_tab(rn, s_dt[diag_idx(code_at(lr, j))]);
          const double tz = z * rn, tr = rn * rn;  // bknum's, snrm's terms
          acc2[0] = acc2[0] + tz;
          acc2[1] = acc2[1] + tr;
          const double pk = s_p[lr * m + c];
          const int i = (R0 + lr) * m + c;
          if constexpr (LIT) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, tz), rl,
                                                  (int)((unsigned)(N + i) * 8u), 0, 16);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, tr), rl,
                                                  (int)((unsigned)(2 * N + i) * 8u), 0, 16);
          }
          if (xreg) {
            if (x0w && lr == 0) xa[j] = xa[j] + ak * pk;
            if (x1w && lr == Hw - 1) xb[j] = xb[j] + ak * pk;
          } else if (a.xrows == 0 || i < a.xrows || i >= N - a.xrows) {
            a.x[i] = a.x[i] + ak * pk;
          }
          if (lr == 0) {
            store_sc1(&xrow(npar, w, 0, 0)[c], rn);
            store_sc1(&xrow(npar, w, 0, 1)[c], pk);
          }
          if (lr == Hw - 1) {
            store_sc1(&xrow(npar, w, 1, 0)[c], rn);
            store_sc1(&xrow(npar, w, 1, 1)[c], pk);
          }
        }
        if constexpr (!QREG) __builtin_amdgcn_sched_barrier(0);
      }
    {
      double tot[2];
      if constexpr (LIT) {
        if (!(ok = res_fold<2>(a, epoch, a.gran + 2 * (size_t)G, 1, tot, s_red))) break;
      } else {
        if constexpr (XG) {
          ok = res_allreduce_x<2>(a, epoch, 1, X, acc2, tot, s_red, s_res);
        } else {
          block_sum<2>(acc2, s_red);
          ok = res_gather<2>(a, epoch, a.gran + 2 * (size_t)G, acc2, tot, s_red);
        }
        if (!ok) break;
      }
      err = sqrt(tot[1]) / bnrm;
      bk = tot[0] / bknum;
      bknum = tot[0];
      if (w == 0 && t == 0 && k - 1 < a.err_hist_cap) a.err_hist[k - 1] = err;
      done = !(err > tol) || k >= itmax + 1;
    }
  }
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int c = t + j * NT;
    if (x0w) a.x[c] = xa[j];
    if (x1w) a.x[(size_t)(nrows - 1) * m + c] = xb[j];
  }
  if (w == 0 && t == 0) {
    S->iter = k;
    S->err = err;
    S->ak = ak;
    S->bk = bk;
    S->bknum = bknum;
    S->done = ok ? 1 : 0;
  }
}


}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
